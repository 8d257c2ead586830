set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r02k
cd $R
CCSX_LIB=libccsx_amd_diag.so timeout -k 10 200 python tools/phase_prof.py > gpurun_out/r02k/phase_diag.json 2>&1 || exit 1
echo done
