set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r02g
cd $R
TIMING=1 timeout -k 10 600 python -u tools/cli_e2e.py 22000 0 0 16 1x1 1x2 > gpurun_out/r02g/cli_e22k_timing.log 2>&1; rc=$?; tail -5 gpurun_out/r02g/cli_e22k_timing.log; exit $rc
