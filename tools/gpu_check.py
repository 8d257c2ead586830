"""Quick GPU-vs-oracle parity check on synthetic ZMWs (development tool)."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccsx_amd as cx

ap = argparse.ArgumentParser()
ap.add_argument("--L", type=int, default=2000)
ap.add_argument("--passes", type=int, default=8)
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--mode", type=int, default=0)
ap.add_argument("--seed", type=int, default=20201104)
ap.add_argument("--mixed", action="store_true", help="config E shapes: insert ~U[5,25] kb, 5-12 passes")
ap.add_argument("--h0", type=int, default=0, help="first hole id")
a = ap.parse_args()

import bench
from oracle import oracle as orc
zs = []
for h in range(a.h0, a.h0 + a.n):
    L, passes = bench.zmw_shape(bench.CONFIGS["E"], h) if a.mixed else (a.L, a.passes)
    subs, ins = cx.synth_zmw(a.seed, h, L, passes)
    zs.append(cx.prepare(subs))
ref, ocells, tcpu = orc.batch(zs, a.mode, min(16, os.cpu_count() or 1))
e = cx.Engine(0)
e.stage(zs)
ms = e.launch(a.mode)
res = e.fetch()
bad = 0
for i, (r, (c, st, cells)) in enumerate(zip(ref, res)):
    if st != 0 or c != r:
        bad += 1
        if bad <= 5:
            k = next((j for j in range(min(len(c), len(r))) if c[j] != r[j]), min(len(c), len(r)))
            print(f"MISMATCH zmw {i}: status {st} gpu_len {len(c)} ref_len {len(r)} first diff at {k}")
cells = sum(x[2] for x in res)
print(f"L={a.L} passes={a.passes} n={a.n} mode={a.mode}: {a.n - bad}/{a.n} identical; kernel {ms:.2f} ms "
      f"({a.n / ms * 1e3:.1f} ZMW/s, {cells / ms / 1e6:.2f} GCUPS); oracle {tcpu:.2f} s; oracle cells {sum(ocells)} gpu cells {cells}")
sys.exit(1 if bad else 0)
