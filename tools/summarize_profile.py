"""Summarise a tools/profile_gpu.sh run into profiles/<tag>_summary.md and
profiles/traffic.json (HBM bytes per launch of ccsx_zmw_kernel, corrected as
MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE x2 for wide streaming reads is
NOT applied because our reads are narrow/uncoalesced -- both raw and x2 given)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
KERNEL = "ccsx_zmw_kernel"


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(src, d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if KERNEL in row["Kernel_Name"]:
                out.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}  # per launch (mean over launches)


stats = list(csv.DictReader(open(glob.glob(os.path.join(src, "kt", "*kernel_stats.csv"))[0])))
bench = json.loads(open(os.path.join(src, "kt_bench.json")).read().strip().splitlines()[-1])
c = {}
for d in ("pmc1", "pmc2", "fetch", "write"):
    c.update(counters(d))
k = [s for s in stats if KERNEL in s["Name"]][0]
avg_ns = float(k["AverageNs"])
fetch_b = c.get("FETCH_SIZE", 0) * 1024
write_b = c.get("WRITE_SIZE", 0) * 1024
lines = [f"# rocprofv3 summary `{tag}` — {bench['config']['workload']}", "",
         "Command: `bash tools/profile_gpu.sh " + tag + "` (bench.py, one launch per PMC pass).", "",
         "## Kernel trace (`--kernel-trace --stats`)", "",
         "| kernel | calls | avg ns | min ns | max ns |", "|---|---|---|---|---|"]
for s in stats:
    lines.append(f"| `{s['Name'][:60]}` | {s['Calls']} | {float(s['AverageNs']):.0f} | {s['MinNs']} | {s['MaxNs']} |")
# per-dispatch durations of the kernel: the last `steps` dispatches are the
# launches bench.py timed (its warmup launches come first)
durs = []
for f in glob.glob(os.path.join(src, "kt", "*kernel_trace.csv")):
    for row in csv.DictReader(open(f)):
        if KERNEL in row["Kernel_Name"]:
            durs.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
durs = [d for _, d in sorted(durs)]
timed = durs[-int(bench["steps"]):] if durs else []
timed_ms = sum(timed) / len(timed) / 1e6 if timed else float("nan")
lines += ["", f"bench.py (same run, {bench['warmup']} warmup + {bench['steps']} timed launches): avg timed launch "
          f"{bench['roofline']['avg_launch_ms']} ms (HIP events), steps {bench.get('step_ms') or bench['roofline'].get('launch_ms')}; rocprof avg over all "
          f"launches {avg_ns / 1e6:.3f} ms (includes the cold first launch); rocprof avg over the "
          f"{len(timed)} timed launches {timed_ms:.3f} ms (kernel trace).", "",
          "## PMC (per launch of ccsx_zmw_kernel, one-launch runs)", "",
          "| counter | value |", "|---|---|"]
for n in sorted(c):
    lines.append(f"| {n} | {c[n]:.4g} |")
waves = c.get("SQ_WAVES", 0) or 1
cyc = c.get("SQ_WAVE_CYCLES", 0)
derived = {
    "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / waves,
    "salu_insts_per_wave": c.get("SQ_INSTS_SALU", 0) / waves,
    "lds_insts_per_wave": c.get("SQ_INSTS_LDS", 0) / waves,
    "wave_cycles_per_wave(quad-cycles)": cyc / waves,
    "frac_wait_any": c.get("SQ_WAIT_ANY", 0) / cyc if cyc else None,
    "frac_wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0) / cyc if cyc else None,
    "frac_active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / cyc if cyc else None,
    "hbm_fetch_bytes": fetch_b, "hbm_write_bytes": write_b,
}
# GRBM_GUI_ACTIVE (summed over the 8 XCDs) against the PMC pass's own launch
# (HIP events of that one-launch run), not the warm timed average
pmc1 = os.path.join(src, "pmc1_bench.json")
if os.path.exists(pmc1):
    pb = json.loads(open(pmc1).read().strip().splitlines()[-1])
    pmc_ms = pb["roofline"]["avg_launch_ms"]
    derived["pmc_pass_launch_ms"] = pmc_ms
    derived["effective_clock_GHz"] = c.get("GRBM_GUI_ACTIVE", 0) / 8 / (pmc_ms * 1e6) if pmc_ms else None
lines += ["", "## Derived", "", "| quantity | value |", "|---|---|"]
for n, v in derived.items():
    lines.append(f"| {n} | {v if v is None else (round(v, 4) if isinstance(v, float) else v)} |")
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
for f in ("kt_kernel_stats.csv",):
    p = glob.glob(os.path.join(src, "kt", "*" + f))
    if p:
        open(os.path.join(ROOT, "profiles", f"{tag}_{f}"), "w").write(open(p[0]).read())
# the bench config profiled (traffic.json key): the second argument, else the
# tag's suffix (r04ze_E16384 -> E16384); never a silent default
cfg = sys.argv[2] if len(sys.argv) > 2 else tag.rsplit("_", 1)[-1]
if cfg not in ("B", "C", "D", "E", "H", "HP") and not cfg.startswith("E") and "_n" not in cfg:
    raise SystemExit(f"traffic.json key: pass the config as the second argument (tag suffix {cfg!r} is not one)")
# the workload the PMC passes launched, so bench.py attaches this entry only
# to a line that launched the same cells (bench.traffic_entry)
pmc_b = json.loads(open(pmc1).read().strip().splitlines()[-1]) if os.path.exists(pmc1) else bench
cells = (pmc_b.get("roofline") or {}).get("cells_per_launch") or pmc_b.get("cells_per_step")
tj = os.path.join(ROOT, "profiles", "traffic.json")
t = json.load(open(tj)) if os.path.exists(tj) else {}
t[cfg] = {"bytes_per_launch": fetch_b + write_b, "fetch_bytes": fetch_b, "write_bytes": write_b,
          "cells_per_launch": cells, "workload": pmc_b["config"]["workload"],
          "source": f"profiles/{tag}_summary.md (FETCH_SIZE+WRITE_SIZE in KB x1024, raw; FETCH_SIZE "
                    f"would be x2 only for wide coalesced streams)"}
json.dump(t, open(tj, "w"), indent=1)
print("\n".join(lines[-14:]))
