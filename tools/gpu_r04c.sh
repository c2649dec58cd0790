#!/bin/bash
# native callers (plain, host-ASan, torch-free RCCL) + RCCL-only self-send repros
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_native.py > $O/native.log 2>&1
echo native rc=$?
tail -6 $O/native.log
for lg in 30 31; do
  timeout -k 10 120 tools/rccl_selfsend /opt/rocm/lib/librccl.so.1 $lg 1 >> $O/rccl_repro.txt 2>&1; echo "rocm rccl lg=$lg rc=$?" >> $O/rccl_repro.txt
  timeout -k 10 120 python3 tools/rccl_selfsend_torch.py $lg 1 >> $O/rccl_repro.txt 2>&1; echo "torch rccl lg=$lg rc=$?" >> $O/rccl_repro.txt
done
timeout -k 10 120 tools/rccl_selfsend /opt/rocm/lib/librccl.so.1 31 8 >> $O/rccl_repro.txt 2>&1; echo "rocm rccl lg=31 chunks=8 rc=$?" >> $O/rccl_repro.txt
timeout -k 10 120 python3 tools/rccl_selfsend_torch.py 31 8 >> $O/rccl_repro.txt 2>&1; echo "torch rccl lg=31 chunks=8 rc=$?" >> $O/rccl_repro.txt
grep -v "^\[W\|amdgpu.ids\|hostname" $O/rccl_repro.txt
