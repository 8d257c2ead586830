#!/bin/bash
# Interleaved timing of several builds of the product library on one box.
# Usage: bash tools/abn.sh "LIB_A LIB_B ..." ROUNDS [bench args...]
# Prints one line per run: lib round ms_per_step
mkdir -p gpurun_out
LIBS=$1; N=$2; shift 2
for i in $(seq 1 $N); do
  for L in $LIBS; do
    CCSX_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/abn_${L}_$i.json 2> gpurun_out/abn_${L}_$i.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/abn_${L}_$i.json')); print('$L', $i, d['ms_per_step'])"
  done
done
