#!/bin/bash
# PMC of the configs[4] leg (2^28 (u64, u32) pairs, 8-bit digits, stable):
# the pair pass, the pair bucket sort and the digit-stream count kernel, one
# rocprofv3 pass per counter group (tools/pmc_cmd.sh) plus the vector-L1
# address-translation counters (TLB), then a kernel trace of the same command.
#   tools/pmc_c5.sh OUTDIR     (on the GPU box)
set -o pipefail
OUT=${1:-gpurun_out/pmc_c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
B=(python3 bench.py --workload c5 --steps 4 --warmup 1 --no-variants --no-cpu-baseline --no-host-abi --no-legs)
RE="tile_pass|bucket_sort|bucket_pairs|tile_counts"
bash tools/pmc_cmd.sh "$OUT" "$RE" "${B[@]}" || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
  TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum -d "$OUT/p_tlb" -o run --output-format csv \
  --kernel-include-regex "$RE" -- "${B[@]}" > "$OUT/p_tlb.log" 2>&1 || echo "tlb pass failed (see p_tlb.log)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- "${B[@]}" \
  > "$OUT/trace.log" 2>&1 || exit 1
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
echo done
