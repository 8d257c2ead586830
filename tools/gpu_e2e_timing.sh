# config-E end-to-end line with per-slice timing (CCSX_TIMING=1)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$1
cd $R
CCSX_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$1/bench_e2e.json 2> gpurun_out/$1/bench_e2e.err || exit 1
tail -c 3000 gpurun_out/$1/bench_e2e.json
