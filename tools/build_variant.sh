#!/bin/bash
# Build a variant of the product library with extra compile flags for A/B
# timing (tools/gpu_ab.sh).  The flags go to the kernel AND the host launcher
# (layout constants such as CCSX_RINGA size the launch's LDS on the host).
#   tools/build_variant.sh TAG -DFOO=1 ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
OBJ=$ROOT/build/obj
C=$ROOT/ccsx_amd/csrc
INC="-I$ROOT/include -I$C -I$C/host"
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -mllvm -amdgpu-sched-strategy=max-ilp "$@" \
  -c $C/ccsx_kernel.hip -o $OBJ/ccsx_kernel_$TAG.hip.o
/opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -fPIC $INC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include "$@" \
  -c $C/ccsx_gpu.cpp -o $OBJ/ccsx_gpu_$TAG.cpp.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/ccsx_amd/libccsx_amd_$TAG.so $OBJ/ccsx_kernel_$TAG.hip.o \
  $OBJ/ccsx_gpu_$TAG.cpp.o $OBJ/bspoa_gpu.cpp.o $OBJ/prepare.cpp.o $OBJ/pairwise.cpp.o $OBJ/seqio.cpp.o \
  $OBJ/dispatch.cpp.o $OBJ/ingest.cpp.o -lz -lpthread
echo $ROOT/ccsx_amd/libccsx_amd_$TAG.so
