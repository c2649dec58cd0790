#!/bin/bash
cd /root/repo
for r in 1 2; do for h in 0 1; do for lg in 27 28; do
LIBSORT_HYBRID=$h timeout -k 10 200 python3 bench.py --keys-log2 $lg --steps 10 --warmup 3 --no-cpu-baseline --no-variants --no-host-abi --no-legs > gpurun_out/ab27_${h}_${lg}_$r.json 2>/dev/null || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], d['ms_per_step'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})" gpurun_out/ab27_${h}_${lg}_$r.json
done; done; done
