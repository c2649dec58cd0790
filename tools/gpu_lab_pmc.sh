#!/bin/bash
# PMC passes over bucket-lab variants (bucket_lab2 FILTER) -> gpurun_out/$1
set -o pipefail
OUT=$1; FILT=$2
bash tools/pmc_cmd.sh "$OUT" "bucket_sort|k_copy|k_cnt" ./tools/bucket_lab2 28 "$FILT" && python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
