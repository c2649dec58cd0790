#!/bin/bash
# the bench line, then the whole GPU suite
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d['kernels'].items(): print(k, round(v['avg_us'],1))
for k,v in (d.get('variants') or {}).items(): print('V', k, v.get('ms_per_step'), v.get('value'))"
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
echo pytest rc=$?
tail -8 $O/pytest.log
