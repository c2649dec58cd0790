set -o pipefail
mkdir -p gpurun_out/r03k
timeout -k 10 120 ./tools/bucket_lab2 28 > gpurun_out/r03k/lab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hybrid.py tests/test_gpu_pieces.py > gpurun_out/r03k/pytest.log 2>&1 && \
bash tools/ab_env.sh LIBSORT_BUCKET_COUNT "0 1" 2 c2 > gpurun_out/r03k/ab.log 2>&1
echo rc=$?
cat gpurun_out/r03k/lab.log | grep -E "prod 256x17 lbits=16|cnt12 256x17 lbits=1[26] |cntF|copy"; tail -3 gpurun_out/r03k/pytest.log; cat gpurun_out/r03k/ab.log
