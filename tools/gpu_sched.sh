#!/bin/bash
# 2^29-per-rank top-digit schedule on one GPU (tools/msd_rccl1.py), uniform and
# the 8-GPU per-rank shape, plus a rocprofv3 kernel-stats pass of the C-ABI
# engine's step.  tools/gpu_sched.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/sched}
mkdir -p "$OUT"
export TMPDIR=/tmp
MSD_LG=29 MSD_SHAPE8=1 MSD_DIGIT8=0 timeout -k 10 300 python3 tools/msd_rccl1.py 4 > "$OUT/shape8.txt" 2>&1 || { echo shape8 failed; tail -5 "$OUT/shape8.txt"; exit 1; }
MSD_LG=29 MSD_DIGIT8=0 timeout -k 10 300 python3 tools/msd_rccl1.py 4 > "$OUT/uniform.txt" 2>&1 || { echo uniform failed; tail -5 "$OUT/uniform.txt"; exit 1; }
MSD_LG=29 MSD_SHAPE8=1 MSD_PROFILE=5 MSD_ENGINE=cabi timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 tools/msd_rccl1.py > "$OUT/prof.log" 2>&1 || { echo prof failed; tail -5 "$OUT/prof.log"; exit 1; }
f=$(ls "$OUT"/prof/*/run_kernel_stats.csv "$OUT"/prof/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/kstats.py "$f" 7 25 > "$OUT/kernels.txt"
grep -h "{" "$OUT/shape8.txt" "$OUT/uniform.txt"; grep -h trace "$OUT/shape8.txt"; tail -3 "$OUT/kernels.txt"
