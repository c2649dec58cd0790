#!/bin/bash
# fused planning (children + tile prefix + host stats), sized second bucket launch: full GPU suite, then the 8-GPU-shape schedule
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for shape in 1 arith; do
  MSD_LG=29 MSD_SHAPE8=$shape MSD_DIGIT8=0 timeout -k 10 200 python3 tools/msd_rccl1.py 4 > $O/shape8_$shape.txt 2>&1 || { echo shape8 failed; tail -5 $O/shape8_$shape.txt; exit 1; }
  grep "{" $O/shape8_$shape.txt
done
MSD_LG=29 MSD_SHAPE8=1 MSD_PROFILE=15 MSD_ENGINE=cabi timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/msd_rccl1.py > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/kstats.py "$f" 17 30 > $O/kernels.txt
cat $O/kernels.txt
