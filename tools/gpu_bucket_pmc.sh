#!/bin/bash
# PMC passes (tools/pmc_cmd.sh) over the bench's bucket sort, the LSD-step
# kernel (LIBSORT_BUCKET_COUNT=0) and the counting kernel (default):
#   tools/gpu_bucket_pmc.sh OUTDIR  -> OUTDIR/{lsd,count}/summary.txt
set -o pipefail
OUT=${1:-gpurun_out/bucket_pmc}
B="python3 bench.py --steps 3 --warmup 1 --no-variants --no-cpu-baseline --no-host-abi --no-legs"
LIBSORT_BUCKET_COUNT=0 bash tools/pmc_cmd.sh "$OUT/lsd" "bucket_sort" $B && python3 tools/pmc_summary.py "$OUT/lsd" > "$OUT/lsd/summary.txt" || exit 1
bash tools/pmc_cmd.sh "$OUT/count" "bucket_sort" $B && python3 tools/pmc_summary.py "$OUT/count" > "$OUT/count/summary.txt" || exit 1
echo done
