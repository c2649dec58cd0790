#!/bin/bash
# One GPU-box check of the tree: distributed/bench tests, the default bench
# line, and the N>1 self-launch rehearsal at configs[3]'s per-GPU share.
# Usage: tools/gpu_check.sh TAG [pytest selection...]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-chk}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SEL=${@:-tests/test_gpu_distrib.py}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $SEL > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench1.json" 2> "$OUT/bench1.err" || { echo "bench failed"; tail -20 "$OUT/bench1.err"; exit 1; }
cat "$OUT/bench1.json"
BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 3 --warmup 1 > "$OUT/bench2r.json" 2> "$OUT/bench2r.err" || { echo "rehearsal failed"; tail -20 "$OUT/bench2r.err"; exit 1; }
cat "$OUT/bench2r.json"
echo done
