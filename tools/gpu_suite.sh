#!/bin/bash
# The round-end GPU tiers as the driver runs them (pytest -m gpu, smoke), with
# per-test durations for the suite budget.  tools/gpu_suite.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/suite}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --durations=120 --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
