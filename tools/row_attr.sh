#!/bin/bash
# Device assembly of one kernel configuration with line tables (for
# tools/row_attr.py and tools/spill_attr.py): tools/row_attr.sh solo16 OUT.s [extra hipcc flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CFG=${1:-solo16}; OUTS=${2:-/tmp/${CFG}_g.s}; shift 2 || true
D=$(cd "$ROOT" && python3 -c "from ccsx_amd.build import KCFGS; print(' '.join(dict(KCFGS)['$CFG']))")
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -I$ROOT/include -I$ROOT/ccsx_amd/csrc \
  -I$ROOT/ccsx_amd/csrc/host -mllvm -amdgpu-sched-strategy=max-ilp $D "$@" -Wno-macro-redefined -gline-tables-only \
  --offload-device-only -S $ROOT/ccsx_amd/csrc/ccsx_kernel.hip -o $OUTS 2>&1 | grep -v "hip-link" || true
grep -E "^\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size):" $OUTS | tr -s ' ' | tr '\n' ' '; echo
