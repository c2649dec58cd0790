#!/bin/bash
# PMC "after" for the bucket kernels: configs[2]'s 1024 x 17 counting kernel and the headline's
# 2-bit kernel + 3-bit retry (same counter groups as profiles/r04a_c3_bucketsort_pmc.txt)
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-variants --no-cpu-baseline --no-host-abi --no-legs"
bash tools/pmc_cmd.sh $O/c3 "bucket_count|bucket_sort" $B --workload c3 && python3 tools/pmc_summary.py $O/c3 > $O/c3/summary.txt || exit 1
bash tools/pmc_cmd.sh $O/c2 "bucket_count|bucket_sort" $B && python3 tools/pmc_summary.py $O/c2 > $O/c2/summary.txt || exit 1
head -60 $O/c3/summary.txt
