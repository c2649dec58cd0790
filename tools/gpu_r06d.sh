#!/bin/bash
# round 6: partial parity + the coded schedule's one-GPU shape + kernel trace + bench
set -o pipefail
OUT=gpurun_out/r06d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "partial" -x -q --timeout 300 --timeout-method thread > $OUT/pt.log 2>&1 || { tail -20 $OUT/pt.log; exit 1; }
timeout -k 10 300 python -u tools/coded_shape.py 2 4 > $OUT/coded_shape.txt 2>&1 || { tail -20 $OUT/coded_shape.txt; exit 1; }
CODED_PROFILE=2,msdz timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_msdz2 -o run --output-format csv -- python3 tools/coded_shape.py > $OUT/prof_msdz2.log 2>&1 || { tail -5 $OUT/prof_msdz2.log; exit 1; }
CODED_PROFILE=2,msd timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_msd2 -o run --output-format csv -- python3 tools/coded_shape.py > $OUT/prof_msd2.log 2>&1 || { tail -5 $OUT/prof_msd2.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo part d done
bash tools/gpu_r06e.sh || exit 1
for m in torch slab torch slab; do
  timeout -k 10 200 python tools/pair_slab_ab.py $m 10 >> $OUT/pair_slab.txt 2>> $OUT/pair_slab.err || { tail -5 $OUT/pair_slab.err; exit 1; }
done
for m in torch slab; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT -d $OUT/pmc_tlb_$m -o run --output-format csv --kernel-include-regex "tile_pass" -- python3 tools/pair_slab_ab.py $m 3 > $OUT/pmc_tlb_$m.log 2>&1 || { tail -5 $OUT/pmc_tlb_$m.log; exit 1; }
done
echo all done
