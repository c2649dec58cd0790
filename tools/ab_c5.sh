#!/bin/bash
# Interleaved A/B of library builds on the C5 pair line and the c3 line.
#   AB_REPS=3 AB_WL="c5 c3" tools/ab_c5.sh build_ab/a.so ...
set -e
mkdir -p gpurun_out/abc5
rm -f gpurun_out/abc5/*.json
for i in $(seq 1 ${AB_REPS:-2}); do
  for lib in intree "$@"; do
    if [ "$lib" = intree ]; then unset LIBSORT_PATH; name=intree; else export LIBSORT_PATH=$PWD/$lib; name=$(basename $lib .so); fi
    for wl in ${AB_WL:-c5 c3}; do
      timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-host-abi --steps 10 --warmup 3 > gpurun_out/abc5/${wl}_${name}_$i.json 2>/dev/null
    done
  done
done
for f in gpurun_out/abc5/*.json; do
  python -c "
import json,sys
d=json.load(open(sys.argv[1])); k=d['kernels']
print('%-28s %8.3f %8.4f ms  ' % (sys.argv[1].split('/')[-1], d['value'], d['ms_per_step']) + '  '.join('%s %.1f' % (n, v['avg_us']) for n, v in k.items()))" $f
done
