#!/bin/bash
# PMC passes over an arbitrary command (run on the GPU box), one rocprofv3
# pass per counter group, --kernel-trace only (MI355X_MICROARCH.md "rocprofv3
# PMC slots").  tools/pmc_cmd.sh OUTDIR KERNEL_REGEX CMD...
set -e
OUT=$1; RE=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $1 -d "$OUT/$name" -o run --output-format csv \
    --kernel-include-regex "$RE" -- "${CMD[@]}" > "$OUT/$name.log" 2>&1
}
CMD=("$@")
run p_sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
run p_sq2 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE"
run p_sq3 "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
run p_fetch "FETCH_SIZE"
run p_write "WRITE_SIZE"
