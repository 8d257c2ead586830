# Where a bench line's wave time goes: SQ stall / issue / instruction-fetch
# counters, one rocprofv3 --pmc pass per counter group (gfx950: at most 8 SQ
# counters a pass), each under its own time limit.
#   bash tools/pmc_stall.sh OUTDIR LINE      LINE = B | D | C | E16k (CCSX_LIB picks a library)
set -e
OUT=$1
LINE=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$LINE" = E16k ]; then
  A="--no-kernel-line --roofline-zmws 16384 --steps 1 --warmup 0 --no-cpu-baseline --e2e-zmws 0 --e-zmws 0"
else
  A="--config $LINE --steps 1 --warmup 0 --no-cpu-baseline --e2e-zmws 0 --e-zmws 0 --roofline-zmws 0"
fi
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVES"
P3="SQ_IFETCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_VMEM"
P4="SQC_ICACHE_HITS SQC_ICACHE_MISSES"
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 180 rocprofv3 --pmc $P -d "$OUT/p$i" -o p --output-format csv -- python3 bench.py $A > "$OUT/p$i.log" 2>&1
  i=$((i+1))
done
# (the instruction-cache counters last and allowed to fail: their block's
# availability on gfx950 is unverified)
timeout -s KILL 120 rocprofv3 --pmc $P4 -d "$OUT/p4" -o p --output-format csv -- python3 bench.py $A > "$OUT/p4.log" 2>&1 ||
  echo "icache pass failed: $?"
python3 - "$OUT" <<'EOF'
import csv, glob, sys, collections
tot = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "ccsx_zmw_kernel" in row.get("Kernel_Name", ""):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
for k in sorted(tot):
    print(f"{k} {tot[k]:.4g}")
EOF
