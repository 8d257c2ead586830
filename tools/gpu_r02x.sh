# GPU tests of the product build, then the CLI on 22k config-E ZMWs (timing)
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$1; mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1; rc=$?; tail -2 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
TIMING=1 timeout -k 10 600 python -u tools/cli_e2e.py 22000 0 0 16 1x1 1x1 > $OUT/cli_e22k.log 2>&1 || exit 1
grep -v "^\[" $OUT/cli_e22k.log
