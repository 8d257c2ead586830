set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r02j
cd $R
timeout -k 10 200 python tools/phase_prof.py > gpurun_out/r02j/phase_product.json 2>&1 || exit 1
CCSX_LIB=libccsx_amd_diag.so timeout -k 10 200 python tools/phase_prof.py > gpurun_out/r02j/phase_diag.json 2>&1 || exit 1
bash tools/profile_gpu.sh r02j > gpurun_out/r02j/prof.log 2>&1 || exit 1
echo done
