set -o pipefail
mkdir -p gpurun_out/r03s
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hybrid.py tests/test_gpu_pieces.py > gpurun_out/r03s/pytest.log 2>&1 && \
AB_REPS=3 bash tools/ab_libs.sh build_ab/prev.so > gpurun_out/r03s/ab.log 2>&1
echo rc=$?
tail -3 gpurun_out/r03s/pytest.log; cat gpurun_out/r03s/ab.log
