#!/bin/bash
# LDS bank-conflict attribution: SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (and the
# LDS issue stalls) over one launch of a bench line, per library variant.
#   bash tools/lds_attr.sh TAG LINE LIB [LIB ...]     (LINE: D | B | E16k)
set -o pipefail
TAG=$1; LINE=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ "$LINE" = E16k ]; then A="--no-kernel-line --roofline-zmws 16384"; else A="--config $LINE --roofline-zmws 0"; fi
for L in "$@"; do
  CCSX_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU \
    -d "$OUT/${LINE}_${L%.so}" -o p --output-format csv -- python3 "$R/bench.py" $A --steps 1 --warmup 0 --no-cpu-baseline \
    --e2e-zmws 0 --e-zmws 0 > "$OUT/${LINE}_${L%.so}.json" 2> "$OUT/${LINE}_${L%.so}.err" || exit 1
  python3 - "$OUT/${LINE}_${L%.so}" "$L" <<'PY'
import csv, glob, sys
c = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ccsx_zmw_kernel" in r["Kernel_Name"]:
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
print(sys.argv[2], {k: f"{v:.4g}" for k, v in sorted(c.items())},
      "conflict/lds", round(c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_INSTS_LDS", 1), 1), 3))
PY
done
