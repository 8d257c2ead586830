#!/bin/bash
# One GPU-box pass: the -m gpu tests, a default bench line, the rocprofv3
# kernel-trace summary of the same bench command, and one PMC pass (LDS /
# issue counters).  Every GPU step has its own time limit; the steps are
# chained so the first failure ends the call.
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh <tag> [tests|bench|prof|all]
set -o pipefail
TAG=${1:-r02}
WHAT=${2:-all}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
  local rc=$?; tail -3 $OUT/gputest.log; return $rc
}
run_bench() {
  timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json
}
run_prof() {
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --no-cpu-baseline --e2e-zmws 0 > $OUT/kt_bench.json 2> $OUT/kt.err) &&
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/pmc_lds -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --e2e-zmws 0 > $OUT/pmc_lds.log 2>&1) &&
  echo "prof done"
}
case $WHAT in
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  all) run_tests && run_bench && run_prof ;;
  *) echo "unknown step $WHAT"; exit 2 ;;
esac
