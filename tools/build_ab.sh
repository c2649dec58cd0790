#!/bin/bash
# Builds an A/B variant of libsort.so with extra -D flags into build_ab/NAME.so
#   tools/build_ab.sh NAME -DLIBSORT_TP4_BLOCK=512 ...
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
D=build_ab/obj_$NAME
mkdir -p "$D"
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -fvisibility=hidden -Iinclude -I/opt/rocm/include --offload-arch=gfx950"
C=gpu-radix-sort_amd/csrc
$H -munsafe-fp-atomics "$@" -c $C/radix_kernels.hip -o $D/radix_kernels.o &
$H "$@" -x hip -c $C/libsort_abi.cpp -o $D/libsort_abi.o &
$H "$@" -x hip -c $C/distrib.cpp -o $D/distrib.o &
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build_ab/$NAME.so $D/*.o -L/opt/rocm/lib -lrocprofiler-sdk-roctx -ldl -Wl,-rpath,/opt/rocm/lib
echo build_ab/$NAME.so
