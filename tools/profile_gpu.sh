#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats + PMC passes (one counter
# group per pass, never combined with tracing domains).  Run on the GPU box:
#   [CFG=B|C|D|E|H|HP|E16384] [NZMW=n] bash tools/profile_gpu.sh <tag> [bench args...]
# Output: gpurun_out/prof_<tag>/...
set -e
TAG=${1:-r01}; shift || true
CFG=${CFG:-B}
SIZE=${NZMW:+--nzmw $NZMW}
# the lines bench.py measures: CFG=E16384 is the headline's roofline line (16,384
# config-E ZMWs per launch, inputs resident), any other CFG its kernel line
if [ "$CFG" = E16384 ]; then
  LINE="--no-kernel-line --roofline-zmws 16384"
else
  LINE="--config $CFG $SIZE --roofline-zmws 0"
fi
ARGS="$LINE ${@:---steps 1 --warmup 0 --no-cpu-baseline --e2e-zmws 0 --e-zmws 0}"
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
# kernel trace over bench's own timed run (default steps / warmup), so the
# rocprof average and bench.py's HIP-event average cover the same launches
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py $LINE --no-cpu-baseline --e2e-zmws 0 --e-zmws 0 > $OUT/kt_bench.json 2> $OUT/kt.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc1 -o pmc1 -- python3 $R/bench.py $ARGS > $OUT/pmc1_bench.json 2> $OUT/pmc1.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d $OUT/pmc2 -o pmc2 -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc2.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/write.err
echo "profile $TAG done"
