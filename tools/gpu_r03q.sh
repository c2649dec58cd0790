set -o pipefail
mkdir -p gpurun_out/r03q
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hybrid.py -k "reserved or (forced and not pairs and not u64) or range" > gpurun_out/r03q/pytest_hyb.log 2>&1 && \
bash tools/ab_env.sh LIBSORT_HYB_RESERVE "0 1" 2 c2 > gpurun_out/r03q/ab.log 2>&1 && \
LIBSORT_HYB_RESERVE=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03q/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --no-host-abi --no-legs > gpurun_out/r03q/prof.log 2>&1
echo rc=$?
tail -3 gpurun_out/r03q/pytest_hyb.log; cat gpurun_out/r03q/ab.log
