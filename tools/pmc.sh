#!/bin/bash
# PMC passes over one sort configuration (run on the GPU box).  Counters are
# collected in separate passes with --kernel-trace only (no other tracing),
# as MI355X_MICROARCH.md "rocprofv3 PMC slots" prescribes.
#   tools/pmc.sh OUTDIR CONFIG [KEYS_LOG2]     e.g. tools/pmc.sh gpurun_out/pmc 8:onesweep:512 28
set -e
OUT=${1:-gpurun_out/pmc}
CFG=${2:-8:onesweep:256}
K=${3:-28}
export TMPDIR=/tmp
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
    --kernel-include-regex "onesweep|downsweep|upsweep|window_hist|copy_kernel|tile_pass|tile_counts|colscan" \
    -- python3 tools/ab_sort.py --keys-log2 "$K" --rounds 1 --reps 2 "$CFG" > "$OUT/$name.log" 2>&1
}
run p_fetch FETCH_SIZE
run p_write WRITE_SIZE
run p_sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run p_sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE
