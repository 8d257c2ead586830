#!/bin/bash
# Build a variant of the product library with extra compile flags for A/B
# timing (tools/gpu_ab.sh).  The flags go to every kernel configuration
# (after its own defines, so they override them) and to the host launcher;
# the configurations' defines come from ccsx_amd/build.py (KCFGS).
#   [CFGS="tput occ"] [KSRC=path/to/kernel.hip] [KSCHED="..."] tools/build_variant.sh TAG -DFOO=1 ...
# CSRC=dir takes ccsx_kernel.hip, ccsx_gpu.cpp and their headers from dir.
# CFGS limits the variant to the named configurations (default: all): the
# others reuse the product's objects (also when KSRC names another source).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
OBJ=$ROOT/build/obj
# CSRC: another source tree (e.g. a git archive of an older commit) for the kernel and ccsx_gpu.cpp
C=${CSRC:-$ROOT/ccsx_amd/csrc}
INC="-I$ROOT/include -I$C -I$C/host"
# KSCHED overrides the machine-scheduler flags (default: the configuration's strategy in
# build.py's KSCHED, else max-ilp; KSCHED=" " for LLVM's default)
K="/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -Wno-macro-redefined"
KOBJS=""
while read -r NAME SCHED DEFS; do
  X=("$@")
  if [ -n "$CFGS" ] && [[ " $CFGS " != *" $NAME "* ]] && [ -f $OBJ/ccsx_kernel_${NAME}.hip.o ]; then
    # a configuration outside CFGS: the product's object (also with KSRC)
    KOBJS="$KOBJS $OBJ/ccsx_kernel_${NAME}.hip.o"
    continue
  fi
  [ -n "$CFGS" ] && [[ " $CFGS " != *" $NAME "* ]] && X=()
  rm -f $OBJ/ccsx_kernel_${NAME}_$TAG.hip.o
  $K ${KSCHED:--mllvm -amdgpu-sched-strategy=$SCHED} $DEFS "${X[@]}" -c ${KSRC:-$C/ccsx_kernel.hip} -o $OBJ/ccsx_kernel_${NAME}_$TAG.hip.o &
  KOBJS="$KOBJS $OBJ/ccsx_kernel_${NAME}_$TAG.hip.o"
done < <(cd "$ROOT" && python3 -c "from ccsx_amd.build import KCFGS, KSCHED; [print(n, KSCHED.get(n, 'max-ilp'), ' '.join(d)) for n, d in KCFGS]")
/opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -fPIC $INC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include "$@" \
  -c $C/ccsx_gpu.cpp -o $OBJ/ccsx_gpu_$TAG.cpp.o
wait
for o in $KOBJS; do [ -f $o ] || { echo "kernel object $o failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/ccsx_amd/libccsx_amd_$TAG.so $KOBJS \
  $OBJ/ccsx_gpu_$TAG.cpp.o $OBJ/bspoa_gpu.cpp.o $OBJ/prepare.cpp.o $OBJ/pairwise.cpp.o \
  $OBJ/seqio.cpp.o $OBJ/dispatch.cpp.o $OBJ/ingest.cpp.o -lz -lpthread
echo $ROOT/ccsx_amd/libccsx_amd_$TAG.so
