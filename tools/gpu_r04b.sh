#!/bin/bash
# lab3 (persistent prefetch bucket sort) + tests of the round-4 changes
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 tools/bucket_lab3 > $O/lab3.txt 2>&1 || { echo lab3 failed; tail -5 $O/lab3.txt; exit 1; }
cat $O/lab3.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hybrid.py tests/test_gpu_distrib_abi.py tests/test_gpu_pieces.py tests/test_gpu_faas.py -k "nomem or duplicates or forced_distributions or reserved_depth0 or auto_large or range_digit or pairs_engine or sharing or one_rank or round_pieces or skewed_rounds or other_widths or distrib_worker or 2pow29 or shape8" > $O/pytest.log 2>&1
echo rc=$?
tail -5 $O/pytest.log
