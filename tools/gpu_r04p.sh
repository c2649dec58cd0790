#!/bin/bash
# 2-bit cells with a 3-bit retry list: full GPU suite, A/B vs 3-bit cells, the bench line
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 bash tools/ab_env.sh LIBSORT_BUCKET2 "0 1" 2 c2 > $O/ab_bucket2.txt 2>&1 || { echo ab failed; tail -5 $O/ab_bucket2.txt; exit 1; }
cat $O/ab_bucket2.txt
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
