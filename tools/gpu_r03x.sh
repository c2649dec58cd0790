set -o pipefail
mkdir -p gpurun_out/r03x
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_distrib.py -k "cabi or rehearsal" > gpurun_out/r03x/pytest.log 2>&1
echo rc=$?
tail -12 gpurun_out/r03x/pytest.log
