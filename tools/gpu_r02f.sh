set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r02f
cd $R
bash tools/gpu_check.sh r02f tests || exit 1
timeout -k 10 600 python -u tools/cli_e2e.py 22000 0 0 16 1x1 1x2 2x1 1x3 > gpurun_out/r02f/cli_e22k.log 2>&1; rc=$?; tail -12 gpurun_out/r02f/cli_e22k.log; exit $rc
