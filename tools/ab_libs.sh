#!/bin/bash
# Interleaved A/B of library builds on one box: bench.py (c2 line + its 8-bit
# variant) with the in-tree libsort.so and with each build_ab/*.so given.
#   tools/ab_libs.sh build_ab/a.so build_ab/b.so ...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/*.json
for i in $(seq 1 ${AB_REPS:-2}); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs --no-host-abi $AB_ARGS > gpurun_out/ab/intree_$i.json 2>/dev/null || exit 1
  for lib in "$@"; do
    LIBSORT_PATH=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs --no-host-abi $AB_ARGS \
      > gpurun_out/ab/$(basename $lib .so)_$i.json 2>/dev/null || exit 1
  done
done
for f in gpurun_out/ab/*.json; do
  python - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); k = d["kernels"]
print("%-40s %7.3f Gkeys/s %7.4f ms  counts %6.1f  pass %6.1f  bucket %6.1f  8-bit %6.4f ms" % (
    sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"], k.get("tilecounts", {}).get("avg_us", 0.0),
    k["tilepass"]["avg_us"], k.get("bucketsort", {}).get("avg_us", 0.0), (d.get("variants") or {}).get("digit8", {}).get("ms_per_step", 0.0)))
PY
done
