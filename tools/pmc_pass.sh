# SQ counter passes over one bench step (one pass per rocprofv3 run; the
# counter sets respect gfx950's 8 SQ slots).  Usage: bash tools/pmc_pass.sh TAG
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
P2="SQ_INSTS SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
P3="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_THREAD_CYCLES_VALU"
i=2
for P in "$P2" "$P3"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/$TAG$i -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --e-zmws 0 --roofline-zmws 0 --e2e-zmws 0 > gpurun_out/$TAG$i.log 2>&1
  i=$((i+1))
done
