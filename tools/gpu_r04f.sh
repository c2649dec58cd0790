#!/bin/bash
# bucket lab 4 (product counting modes), the bench line, the hybrid/parity tests
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 tools/bucket_lab4 "prod,cnt2 256x17 wpe=1,cnt3 1024x17 wpe=8" > $O/lab4.txt 2>&1; echo "lab4 rc=$?"; cat $O/lab4.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d['kernels'].items(): print(k, round(v['avg_us'],1))
for k,v in (d.get('variants') or {}).items(): print('V', k, v.get('ms_per_step'), v.get('value'))"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hybrid.py tests/test_gpu_parity.py tests/test_gpu_pieces.py tests/test_gpu_faas.py > $O/pytest.log 2>&1
echo pytest rc=$?
tail -5 $O/pytest.log
