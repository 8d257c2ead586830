# A/B of variants on config-E-shaped launches (bench --config E with N ZMWs)
#   gpurun -- bash tools/gpu_abE.sh TAG NZMW lib1 lib2 ...
set -o pipefail
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$TAG
cd $R
for i in 1 2; do
  for L in "$@"; do
    CCSX_LIB=$L timeout -k 10 300 python3 bench.py --config E --nzmw $N --steps 2 --warmup 1 --no-cpu-baseline --e2e-zmws 0 > gpurun_out/$TAG/e_${L}_$i.json 2> gpurun_out/$TAG/e_${L}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/$TAG/e_${L}_$i.json')); print('$L E', $N, d['ms_per_step'], d['value'])"
  done
done
