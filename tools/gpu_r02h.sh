set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r02h
cd $R
bash tools/gpu_check.sh r02h tests || exit 1
TIMING=1 timeout -k 10 600 python -u tools/cli_e2e.py 22000 0 0 16 1x1 1x2 1x1 1x2 > gpurun_out/r02h/cli_e22k_timing.log 2>&1; rc=$?; grep -E "layout|identical|ingest" gpurun_out/r02h/cli_e22k_timing.log; exit $rc
