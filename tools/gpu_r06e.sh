#!/bin/bash
# round 6: configs[2] next-digit byte stream A/B (LIBSORT_DSTREAM_U32), 3
# interleaved runs each, then the 2^30 bit-exact test with the stream on
set -o pipefail
OUT=gpurun_out/r06e
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --workload c3 --steps 10 --warmup 3 --no-variants --no-cpu-baseline --no-host-abi"
for i in 1 2 3; do
  for v in 0 1; do
    LIBSORT_DSTREAM_U32=$v timeout -k 10 200 $B > $OUT/c3_ds${v}_$i.json 2> $OUT/c3_ds${v}_$i.err || { tail -5 $OUT/c3_ds${v}_$i.err; exit 1; }
    echo "ds=$v run $i: $(python3 -c "import json,sys;d=json.load(open('$OUT/c3_ds${v}_$i.json'));print(d['ms_per_step'],{k:v['avg_us'] for k,v in d['kernels'].items()})")"
  done
done
LIBSORT_DSTREAM_U32=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "config3_2pow30" -x -q --timeout 250 --timeout-method thread > $OUT/pt.log 2>&1 || { tail -20 $OUT/pt.log; exit 1; }
tail -2 $OUT/pt.log
echo done
