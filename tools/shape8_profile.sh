#!/bin/bash
# The 8-GPU per-rank shape on one MI355X (tools/msd_rccl1.py, 2^29 keys in
# 32 top digits, one RCCL rank): the schedule timings at both wire formats,
# then a kernel trace of 8 steps of the C engine per format.
#   tools/shape8_profile.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/shape8}
mkdir -p "$OUT"
export TMPDIR=/tmp MSD_LG=29 MSD_SHAPE8=1 MSD_DIGIT8=0
timeout -k 10 300 python3 tools/msd_rccl1.py 4 > "$OUT/schedule.txt" 2>&1 || { tail -5 "$OUT/schedule.txt"; exit 1; }
for w in 24 32; do
  if [ $w = 32 ]; then export MSD_WIRE32=1; else unset MSD_WIRE32; fi
  MSD_PROFILE=8 MSD_ENGINE=cabi timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace$w" -o run \
    --output-format csv -- python3 tools/msd_rccl1.py > "$OUT/trace$w.log" 2>&1 || { tail -5 "$OUT/trace$w.log"; exit 1; }
done
echo done
