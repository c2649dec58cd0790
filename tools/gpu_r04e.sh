#!/bin/bash
# bucket labs 3 and 4, then the test/native/RCCL script
set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 300 tools/bucket_lab4 > gpurun_out/r04e/lab4.txt 2>&1; echo "lab4 rc=$?"; cat gpurun_out/r04e/lab4.txt
bash tools/gpu_r04bc.sh
