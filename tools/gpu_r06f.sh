#!/bin/bash
# round 6: LSD 8-bit tile A/B on the gpuPartial legs (3 interleaved runs),
# then the whole GPU suite with durations and smoke()
set -o pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 200 python tools/partial_ab.py >> $OUT/partial_ab.txt 2>> $OUT/partial_ab.err || { tail -5 $OUT/partial_ab.err; exit 1; }
  LIBSORT_PATH=$PWD/build_ab/lsd1024.so timeout -k 10 200 python tools/partial_ab.py >> $OUT/partial_ab.txt 2>> $OUT/partial_ab.err || { tail -5 $OUT/partial_ab.err; exit 1; }
done
echo partial ab done
bash tools/gpu_suite.sh $OUT
