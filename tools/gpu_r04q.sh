#!/bin/bash
# packed-rank kCntSmall (7 blocks per CU): piece/distrib/hybrid tests, then the 8-GPU-shape schedule
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pieces.py tests/test_gpu_distrib_abi.py tests/test_gpu_hybrid.py > $O/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
MSD_LG=29 MSD_SHAPE8=1 MSD_DIGIT8=0 timeout -k 10 200 python3 tools/msd_rccl1.py 4 > $O/shape8_1.txt 2>&1 || { echo shape8 failed; tail -5 $O/shape8_1.txt; exit 1; }
grep "{" $O/shape8_1.txt
MSD_LG=29 MSD_SHAPE8=1 MSD_PROFILE=15 MSD_ENGINE=cabi timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/msd_rccl1.py > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/kstats.py "$f" 17 30 > $O/kernels.txt
cat $O/kernels.txt
