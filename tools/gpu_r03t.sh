set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
export TMPDIR=/tmp
MSD_LG=29 MSD_SHAPE8=1 MSD_PROFILE=5 MSD_ENGINE=cabi timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 tools/msd_rccl1.py > "$OUT/prof.log" 2>&1 || { echo prof failed; tail -5 "$OUT/prof.log"; exit 1; }
f=$(ls "$OUT"/prof/*/run_kernel_stats.csv "$OUT"/prof/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/kstats.py "$f" 7 25 > "$OUT/kernels.txt"
tail -25 "$OUT/kernels.txt"
g=$(ls "$OUT"/prof/*/run_hip_api_stats.csv "$OUT"/prof/run_hip_api_stats.csv 2>/dev/null | head -1)
head -25 "$g" | cut -c1-120
