#!/bin/bash
# pass durations after 2-bit vs 3-bit bucket phases (kernel traces of the bench, both modes, interleaved)
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
for m in 1 0 1 0; do
  LIBSORT_BUCKET2=$m timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof_$m -o run_$m --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-variants --no-host-abi --no-legs > $O/b_$m.log 2>&1 || { echo prof $m failed; tail -5 $O/b_$m.log; exit 1; }
  python3 tools/pass_split.py $O/prof_$m >> $O/split.txt || exit 1
done
cat $O/split.txt
