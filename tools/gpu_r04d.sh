#!/bin/bash
# Interleaved A/B of the configs[4] pair sort: this tree vs round 2's and round 3's libraries (one box)
set -o pipefail
export TMPDIR=/tmp LIBSORT_AB_MISSING_OK=1
AB_REPS=3 AB_WL=c5 timeout -k 10 900 bash tools/ab_c5.sh ablibs/r02.so ablibs/head_r03.so > gpurun_out/r04d_c5_ab.txt 2>&1
echo rc=$?
cat gpurun_out/r04d_c5_ab.txt
