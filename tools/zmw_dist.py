"""Distribution of per-ZMW kernel cycles (development tool): the launch ends
with its slowest ZMW, so the tail, not the mean, sets ms per step.
Needs CCSX_LIB=libccsx_amd_diag.so (the product objects carry no counters)."""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccsx_amd as cx
import bench

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="B")
ap.add_argument("--nzmw", type=int, default=0)
a = ap.parse_args()
cfg = dict(bench.CONFIGS[a.config])
if a.nzmw:
    cfg["nzmw"] = a.nzmw
zs = bench.make_batch(cfg, 0)
e = cx.Engine(0)
e.stage(zs, cfg["mode"])
plain = [e.launch(cfg["mode"]) for _ in range(3)]
e.set_profiling(True)
ms = e.launch(cfg["mode"])
pz = e.profile_zmw(len(zs))
e.set_profiling(False)
plain += [e.launch(cfg["mode"]) for _ in range(2)]
tot = sorted(p["total"] for p in pz)
n = len(tot)
q = lambda f: tot[min(n - 1, int(f * n))]
slow = sorted(range(n), key=lambda i: -pz[i]["total"])[:8]
out = {"kernel_ms": ms, "plain_ms": plain, "n": n, "mean": sum(tot) / n, "min": tot[0], "p50": q(0.5), "p90": q(0.9), "p99": q(0.99),
       "max": tot[-1], "max_over_mean": tot[-1] / (sum(tot) / n),
       "slowest": [{"zmw": i, "segs": len(zs[i].lens), "bases": int(sum(zs[i].lens)),
                    **{k: pz[i][k] for k in ("total", "dp", "traceback", "merge", "dp_rows")}} for i in slow],
       "mean_bases": sum(int(sum(z.lens)) for z in zs) / n,
       "mean_phase": {k: round(sum(p[k] for p in pz) / n / 1e6, 2) for k in
                      ("total", "load_read", "dp", "traceback", "merge", "columns", "shred", "dp_rows")}}


def simd(v):  # HW_ID: simd 5:4, cu 11:8, sh 12, se 15:13; XCC_ID in bits 32+
    return ((v >> 32) & 15, (v >> 13) & 7, (v >> 12) & 1, (v >> 8) & 15, (v >> 4) & 3)


from collections import Counter, defaultdict
w0 = Counter(simd(p["hw0"]) for p in pz)
hl = Counter(simd(p[k]) for p in pz for k in ("hw1", "hw2"))
cu = Counter(simd(p["hw0"])[:4] for p in pz)
by = defaultdict(list)
for p in pz:
    k = simd(p["hw0"])
    by[(w0[k] - 1, hl[k])].append(p["total"])
out["simds_with_wave0"] = len(w0)
out["cus_used"] = len(cu)
out["zmws_per_cu_hist"] = sorted(Counter(cu.values()).items())
out["placement"] = {f"{a} other wave0, {b} helpers": [len(v), round(sum(v) / len(v) / 1e6, 1), round(max(v) / 1e6, 1)]
                    for (a, b), v in sorted(by.items())}
st = [p["start_rt"] for p in pz]
en = [p["end_rt"] for p in pz]
out["start_spread_us"] = (max(st) - min(st)) / 100.0
out["late_starts"] = sum(1 for x in st if x - min(st) > 100000)
out["end_max_ms"] = (max(en) - min(st)) / 1e5
print(json.dumps(out))
