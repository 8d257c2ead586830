# A/B of two product builds (tools/gpu_ab.sh) plus one LDS-counter PMC pass per
# build (bank conflicts, LDS instructions, over one bench step)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd $R
bash tools/gpu_ab.sh $TAG "$@" || exit 1
export TMPDIR=/tmp
for L in "$@"; do
  (cd /tmp && CCSX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_$L -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --e2e-zmws 0 > $OUT/pmc_$L.log 2>&1) || exit 1
done
echo pmc done
