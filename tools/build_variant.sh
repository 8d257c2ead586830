#!/bin/bash
# Build a variant of the product library with extra compile flags for A/B
# timing (tools/gpu_ab.sh).  The flags go to both kernel configurations (after
# their own defines, so they override them) and to the host launcher.
#   tools/build_variant.sh TAG -DFOO=1 ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
OBJ=$ROOT/build/obj
C=$ROOT/ccsx_amd/csrc
INC="-I$ROOT/include -I$C -I$C/host"
K="/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -mllvm -amdgpu-sched-strategy=max-ilp -Wno-macro-redefined"
$K -DCCSX_KCFG=lat -DCCSX_LAUNCH=ccsx_launch_zmw_lat -DCCSX_RINGA=32 -DCCSX_BLK=8 "$@" -c $C/ccsx_kernel.hip -o $OBJ/ccsx_kernel_lat_$TAG.hip.o &
$K -DCCSX_KCFG=occ -DCCSX_LAUNCH=ccsx_launch_zmw_occ -DCCSX_RINGA=24 -DCCSX_BLK=4 "$@" -c $C/ccsx_kernel.hip -o $OBJ/ccsx_kernel_occ_$TAG.hip.o &
/opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -fPIC $INC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include "$@" \
  -c $C/ccsx_gpu.cpp -o $OBJ/ccsx_gpu_$TAG.cpp.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/ccsx_amd/libccsx_amd_$TAG.so $OBJ/ccsx_kernel_lat_$TAG.hip.o \
  $OBJ/ccsx_kernel_occ_$TAG.hip.o $OBJ/ccsx_gpu_$TAG.cpp.o $OBJ/bspoa_gpu.cpp.o $OBJ/prepare.cpp.o $OBJ/pairwise.cpp.o \
  $OBJ/seqio.cpp.o $OBJ/dispatch.cpp.o $OBJ/ingest.cpp.o -lz -lpthread
echo $ROOT/ccsx_amd/libccsx_amd_$TAG.so
