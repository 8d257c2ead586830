# GPU tests of the product build (and a parity subset on every variant), then
# the interleaved A/B timing of the variants.
#   gpurun -- bash tools/gpu_ab.sh TAG lib1 lib2 ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1; rc=$?; tail -2 gpurun_out/$TAG/gputest.log; [ $rc -eq 0 ] || exit $rc
for L in "$@"; do
  [ "$L" = libccsx_amd.so ] && continue
  CCSX_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest_$L.log 2>&1; rc=$?; echo "$L: $(tail -1 gpurun_out/$TAG/gputest_$L.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3; do
  for L in "$@"; do
    CCSX_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --e2e-zmws 0 --e-zmws 0 --roofline-zmws 0 > gpurun_out/$TAG/t_${L}_$i.json 2> gpurun_out/$TAG/t_${L}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/$TAG/t_${L}_$i.json')); print('$L', d['ms_per_step'])"
  done
done
