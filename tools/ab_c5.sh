#!/bin/bash
# Interleaved A/B of library builds on the C5 pair line and the c3 line.
#   tools/ab_c5.sh build_ab/a.so ...
set -e
mkdir -p gpurun_out/abc5
for i in 1 2; do
  for lib in intree "$@"; do
    if [ "$lib" = intree ]; then unset LIBSORT_PATH; name=intree; else export LIBSORT_PATH=$PWD/$lib; name=$(basename $lib .so); fi
    timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline --no-host-abi > gpurun_out/abc5/c5_${name}_$i.json 2>/dev/null
    timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/abc5/c3_${name}_$i.json 2>/dev/null
  done
done
for f in gpurun_out/abc5/*.json; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-28s %8.3f %8.4f ms pass %7.1f' % (sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['kernels']['tilepass']['avg_us']))" $f
done
