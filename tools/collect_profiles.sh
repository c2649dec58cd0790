#!/bin/bash
# Round measurement on the GPU box: bench line, rocprofv3 kernel stats of the
# same bench command, FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel
# trace only) for the pass kernels, copy-kernel ceiling + rocPRIM reference.
# Usage: tools/collect_profiles.sh TAG   (outputs under gpurun_out/prof_TAG)
set -e
cd "$(dirname "$0")/.."
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
BENCH="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- $BENCH > "$OUT/stats.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv \
    --kernel-include-regex "tile_pass|onesweep|downsweep|tile_counts" -- $BENCH > "$OUT/pmc_$c.log" 2>&1
done
if [ -x tools/calib_copy ]; then timeout -k 10 120 ./tools/calib_copy 28 > "$OUT/calib.txt" 2>&1; fi
echo collected
