#!/bin/bash
# Builds an A/B variant of libsort.so into build_ab/NAME.so: radix_kernels.hip
# (as it is in the tree when this runs, with the extra -D flags given) linked
# with the in-tree host objects (make -C gpu-radix-sort_amd/csrc first).
#   tools/build_ab.sh NAME -DLIBSORT_TP4_BLOCK=512 ...
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
D=build_ab/obj_$NAME
mkdir -p "$D"
C=gpu-radix-sort_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -fvisibility=hidden -Iinclude \
  -I/opt/rocm/include --offload-arch=gfx950 -munsafe-fp-atomics "$@" -c $C/radix_kernels.hip -o $D/radix_kernels.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build_ab/$NAME.so $D/radix_kernels.o $C/libsort_abi.o \
  $C/distrib.o -L/opt/rocm/lib -lrocprofiler-sdk-roctx -ldl -Wl,-rpath,/opt/rocm/lib
echo build_ab/$NAME.so
