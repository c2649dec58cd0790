#!/bin/bash
# Full GPU suite + smoke + the default bench line on one box.
# Usage: tools/gpu_full.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-full}; shift
SEL=${@:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $SEL > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench1.json" 2> "$OUT/bench1.err" || { echo "bench failed"; tail -20 "$OUT/bench1.err"; exit 1; }
cat "$OUT/bench1.json"
echo done
