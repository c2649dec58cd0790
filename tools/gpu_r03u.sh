set -o pipefail
mkdir -p gpurun_out/r03u
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hybrid.py -k "reserved or digit8" > gpurun_out/r03u/pytest.log 2>&1 && \
AB_REPS=3 AB_ARGS="--workload c3" bash tools/ab_libs.sh build_ab/prev.so > gpurun_out/r03u/ab2.log 2>&1
echo rc=$?
tail -3 gpurun_out/r03u/pytest.log; cat gpurun_out/r03u/ab2.log
