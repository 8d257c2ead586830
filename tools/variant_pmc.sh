#!/bin/bash
# LDS counters and interleaved timing of library variants (tools/build_variant.sh).
#   gpurun -- bash tools/variant_pmc.sh <tag> libccsx_amd.so libccsx_amd_X.so ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  export CCSX_LIB=$L
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/pmc_$L -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --e2e-zmws 0 > $OUT/pmc_$L.log 2>&1) || exit 1
done
for i in 1 2; do
  for L in "$@"; do
    export CCSX_LIB=$L
    timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --e2e-zmws 0 "${BENCH_ARGS[@]}" > $OUT/t_${L}_$i.json 2> $OUT/t_${L}_$i.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$OUT/t_${L}_$i.json')); print('$L', d['ms_per_step'])"
  done
done
