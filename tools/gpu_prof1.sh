#!/bin/bash
# One GPU session: copy ceiling + rocPRIM reference, then PMC passes.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 ./tools/calib_copy 28 > gpurun_out/calib.txt 2>&1
export TMPDIR=/tmp
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass -d gpurun_out/pmc_calib/$pass -o run --output-format csv -- ./tools/calib_copy 26 > /dev/null 2>&1
done
tools/pmc.sh gpurun_out/pmc_8os512 8:onesweep:512 28
tools/pmc.sh gpurun_out/pmc_8rts 8:rts:256 28
tools/pmc.sh gpurun_out/pmc_4os256 4:onesweep:256 28
echo done
