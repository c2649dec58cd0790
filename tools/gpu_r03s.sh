set -o pipefail
mkdir -p gpurun_out/r03s
export TMPDIR=/tmp
AB_REPS=3 bash tools/ab_libs.sh build_ab/prev.so > gpurun_out/r03s/ab.log 2>&1
echo rc=$?
cat gpurun_out/r03s/ab.log
