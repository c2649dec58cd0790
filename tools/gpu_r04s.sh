#!/bin/bash
# final tree: the whole GPU suite, smoke(), the 8-GPU-shape schedule
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
MSD_LG=29 MSD_SHAPE8=1 MSD_DIGIT8=0 timeout -k 10 200 python3 tools/msd_rccl1.py 4 > $O/shape8_1.txt 2>&1 || { echo shape8 failed; tail -5 $O/shape8_1.txt; exit 1; }
grep "{" $O/shape8_1.txt
