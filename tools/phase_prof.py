"""Per-phase cycle breakdown of the consensus kernel (s_memtime counters).

Needs the diagnostic library, whose objects carry the counters:
CCSX_LIB=libccsx_amd_diag.so python tools/phase_prof.py ...  (with the product
library ccsx_gpu_set_profiling fails and this tool stops with its message)."""
import argparse, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccsx_amd as cx
ap = argparse.ArgumentParser()
ap.add_argument("--L", type=int, default=10000)
ap.add_argument("--passes", type=int, default=8)
ap.add_argument("--n", type=int, default=1000)
ap.add_argument("--mode", type=int, default=0)
ap.add_argument("--kcfg", type=int, default=-1, help="force a kernel configuration (ccsx_layout.h KernelCfg)")
a = ap.parse_args()
zs = [cx.prepare(cx.synth_zmw(20201104, h, a.L, a.passes)[0]) for h in range(a.n)]
e = cx.Engine(0)
if a.kcfg >= 0:
    e.set_kernel_cfg(a.kcfg)
e.stage(zs, a.mode)
e.launch(a.mode)
e.set_profiling(True)
ms = e.launch(a.mode)
p = e.profile()
res = e.fetch()
cells = sum(r[2] for r in res)
tot = p["total"]
out = {"config": vars(a), "kernel_ms": ms, "gcups": cells / ms / 1e6,
       "share": {k: round(v / tot, 4) for k, v in p.items() if k not in ("total", "dp_rows")},
       "cycles_per_zmw": tot / a.n, "row_cycles": {k: round(v / max(p["dp_rows"], 1), 1) for k, v in p.items() if k.startswith("row_")}, "tb_share": {k: round(p[k] / tot, 4) for k in ("spare0", "spare1", "flush")}, "dp_cycles_per_row": p["dp"] / max(p["dp_rows"], 1),
       "rows_per_zmw": p["dp_rows"] / a.n,
       "two_wave": {k: round(p[k] / max(p["tw_rows"], 1), 1) for k in ("a_busy", "a_wait", "b_busy", "b_wait")},
       "tw_rows_frac": round(p["tw_rows"] / max(p["dp_rows"], 1), 4),
       "rows": {"a_fast_pred": round(p["row_A_fast"] / max(p["dp_rows"] - p["row_D_nfast"], 1), 1),
                "a_cold_pred": round(p["row_B_general"] / max(p["row_D_nfast"], 1), 1),
                "a_common": round(p["row_C_unused"] / max(p["dp_rows"], 1), 1),
                "a_cold_frac": round(p["row_D_nfast"] / max(p["dp_rows"], 1), 4),
                "b_fast_pred_per_row": round(p["spare2"] / max(p["dp_rows"], 1), 1),
                "b_cold_pred_per_row": round(p["spare3"] / max(p["dp_rows"], 1), 1),
                "b_common": round(p["flush"] / max(p["dp_rows"], 1), 1)}}
nf = max(p["a_fast"], 1)
out["a_fast_row"] = {"rows_frac": round(p["a_fast"] / max(p["dp_rows"], 1), 4),
                     "start_to_decision": round(p["a_tail"] / nf, 1),
                     "start_to_scan": round(p["a_head"] / nf, 1),
                     "scan_to_end": round(p["a_body"] / nf, 1)}
out["a_cold_rows"] = {k: {"frac": round(p["n_" + k] / max(p["dp_rows"], 1), 4),
                          "cycles": round(p["cold_" + k] / max(p["n_" + k], 1), 1)}
                      for k in ("far", "chain", "np1", "np2", "gen", "spill", "near")}
out["per_zmw"] = {k: round(v / a.n, 1) for k, v in p.items()}
print(json.dumps(out))
