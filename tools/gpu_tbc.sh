# traceback step counters (product build + -DCCSX_TB_COUNT) on config B
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$1
cd $R
CCSX_LIB=libccsx_amd_tbc.so timeout -k 10 200 python tools/phase_prof.py > gpurun_out/$1/phase_tbc.json 2>&1 || exit 1
timeout -k 10 200 python tools/phase_prof.py > gpurun_out/$1/phase_product.json 2>&1 || exit 1
echo done
