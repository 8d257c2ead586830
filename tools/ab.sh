# A/B timing of two builds of the product library on one box, interleaved.
# Usage: bash tools/ab.sh LIB_A LIB_B [bench args...]
set -e
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for i in 1 2; do
  for L in $A $B; do
    CCSX_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_${L}_$i.log 2>&1
  done
done
