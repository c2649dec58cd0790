#!/bin/bash
# Round measurement on the GPU box, in this order:
#   1. FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel trace only) of
#      the bench command -> profiles/pmc_<kernel>.json (HBM bytes per launch),
#      so the bench line below reports the traffic of the same build;
#   2. the bench line (default arguments);
#   3. rocprofv3 --kernel-trace --stats of the bench command;
#   4. the HBM ceiling probes (tools/bw_probe) and rocPRIM's sort (tools/calib_copy).
# Usage: tools/collect_profiles.sh TAG   (outputs under gpurun_out/prof_TAG;
# run tools/make_profile_summary.py TAG locally afterwards to commit them)
set -e
cd "$(dirname "$0")/.."
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --no-host-abi"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv \
    --kernel-include-regex "tile_pass|onesweep|downsweep|tile_counts" -- $BENCH > "$OUT/pmc_$c.log" 2>&1
done
python3 tools/make_profile_summary.py "$TAG" > "$OUT/pmc_summary.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- $BENCH > "$OUT/stats.log" 2>&1
if [ -x tools/bw_probe ]; then timeout -k 10 120 ./tools/bw_probe 28 > "$OUT/bw_probe.txt" 2>&1; fi
if [ -x tools/calib_copy ]; then timeout -k 10 120 ./tools/calib_copy 28 > "$OUT/calib.txt" 2>&1; fi
echo collected
