set -e
mkdir -p gpurun_out/abp
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export LIBSORT_PATH=$PWD/build_ab/old.so; else unset LIBSORT_PATH; fi
    timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline --no-host-abi > gpurun_out/abp/c5_${lib}_$i.json 2>/dev/null
    timeout -k 10 200 python tools/bench_rows.py 4 > gpurun_out/abp/rows_${lib}_$i.txt 2>/dev/null
  done
done
for f in gpurun_out/abp/c5_*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['kernels']['tilepass']['avg_us'])" $f; done
grep -H "" gpurun_out/abp/rows_*.txt
