#!/bin/bash
# Round-4 baseline on a fresh box: the driver's bench command, the 8-GPU-shape
# schedule's kernel stats at two step counts (per-step vs one-off launches),
# and PMC of the configs[2] bucket sort (1024-thread class).
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
export LIBSORT_PATH=$PWD/ablibs/head_r03.so
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
for S in 5 15; do
  MSD_LG=29 MSD_SHAPE8=1 MSD_PROFILE=$S MSD_ENGINE=cabi timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sched$S -o run --output-format csv -- python3 tools/msd_rccl1.py > $O/sched$S.log 2>&1 || { echo sched$S failed; tail -5 $O/sched$S.log; exit 1; }
  f=$(ls $O/sched$S/*/run_kernel_stats.csv $O/sched$S/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 tools/kstats.py "$f" $((S + 2)) 30 > $O/sched${S}_kernels.txt
done
B="python3 bench.py --workload c3 --steps 3 --warmup 1 --no-variants --no-cpu-baseline --no-host-abi --no-legs"
bash tools/pmc_cmd.sh $O/c3pmc "bucket_sort" $B && python3 tools/pmc_summary.py $O/c3pmc > $O/c3pmc/summary.txt || { echo pmc failed; exit 1; }
echo done
