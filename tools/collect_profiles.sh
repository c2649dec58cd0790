#!/bin/bash
# Round measurement on the GPU box, all of the driver's EXACT bench command
# (python3 bench.py --gpus 1 --steps 20 --warmup 5), in this order:
#   1. FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel trace only,
#      restricted to the pass kernel) -> HBM bytes per launch;
#   2. rocprofv3 --kernel-trace --stats -> per-dispatch durations;
#   3. the bench line itself (unprofiled);
#   4. the HBM ceiling probes (tools/bw_probe) and rocPRIM (tools/calib_copy).
# Usage: tools/collect_profiles.sh TAG   (outputs under gpurun_out/prof_TAG;
# then tools/make_profile_summary.py TAG here writes profiles/TAG_*)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --gpus 1 --steps 20 --warmup 5"
echo "$BENCH" > "$OUT/cmd.txt"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv \
    --kernel-include-regex "tile_pass|bucket_sort|bucket_count|bucket_pairs|tile_counts" -- $BENCH > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; tail -5 "$OUT/pmc_$c.log"; exit 1; }
  echo "pmc $c done"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- $BENCH \
  > "$OUT/stats.log" 2>&1 || { echo "stats failed"; tail -5 "$OUT/stats.log"; exit 1; }
echo "stats done"
timeout -k 10 300 $BENCH > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -x tools/bw_probe ]; then timeout -k 10 120 ./tools/bw_probe 28 > "$OUT/bw_probe.txt" 2>&1; fi
if [ -x tools/calib_copy ]; then timeout -k 10 120 ./tools/calib_copy 28 > "$OUT/calib.txt" 2>&1; fi
echo collected
