#!/bin/bash
# ext-launch timing events + 2-bit vs 3-bit cells on the headline: quick tests, A/B, trace
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hybrid.py tests/test_gpu_pieces.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_env.sh LIBSORT_BUCKET2 "0 1" 3 c2 > $O/ab_bucket2.txt 2>&1 || { echo ab failed; tail -5 $O/ab_bucket2.txt; exit 1; }
cat $O/ab_bucket2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --no-host-abi --no-legs > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-400
