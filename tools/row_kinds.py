#!/usr/bin/env python3
"""DP rows by kernel row class (fast band move 0 / 1, chain, np1, np2, 3-4
predecessors, far) on synthetic config-shaped ZMWs, from the oracle's debug
counter (oracle/poa_oracle.c opoa_row_kinds; test infrastructure, CPU only).

    python tools/row_kinds.py --config E --n 24 [--json out.json]

Pairs with the per-class instruction counts of tools/row_attr.py to give the
instructions per average DP row.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KINDS = ["fast0", "fast1", "chain", "np1", "np2", "gen", "far", "spill"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="E")
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--json")
    ap.add_argument("--tb", action="store_true", help="also the traceback's predecessor moves by row distance")
    a = ap.parse_args()
    import bench
    from oracle.oracle import Poa, lib, prepare as oracle_prepare
    import ccsx_amd as cx
    L = lib()
    L.opoa_row_kinds.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    cfg = bench.CONFIGS[a.config]
    holes = list(bench.rank_holes(dict(cfg, nzmw=a.n), 0))[: a.n] if a.config != "E" else \
        [bench.E_LAUNCH_HOLE0 + i for i in range(a.n)]
    out = (C.c_uint64 * len(KINDS))()
    L.opoa_row_kinds(out, 1)
    TB = ["d1", "d2", "d3", "d4_8", "far", "moves_D", "steps", "M_d4", "M_d5_8", "D_d1", "D_far", "D_d2_8"]
    tbo = (C.c_uint64 * len(TB))()
    L.opoa_tb_moves.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    L.opoa_tb_moves(tbo, 1)
    p = Poa()
    for h in holes:
        Ls, passes = bench.zmw_shape(cfg, h)
        z = oracle_prepare(cx.synth_zmw(bench.SEED, h, Ls, passes)[0])
        p.zmw(z.seqs, z.offs, z.lens, cfg["mode"])
    L.opoa_row_kinds(out, 1)
    cnt = dict(zip(KINDS, [int(x) for x in out]))
    rows = sum(cnt[k] for k in KINDS if k != "spill")
    res = {"config": a.config, "zmws": len(holes), "rows": rows,
           "frac": {k: round(cnt[k] / rows, 4) for k in KINDS}}
    if a.tb:
        L.opoa_tb_moves(tbo, 1)
        t = dict(zip(TB, [int(x) for x in tbo]))
        mv = sum(t[k] for k in TB[:5])
        res["tb"] = {"steps": t["steps"], "moves": mv, "moves_D": t["moves_D"],
                     "frac": {k: round(t[k] / max(mv, 1), 5) for k in TB[:5]},
                     "by_kind": {k: t[k] for k in TB[7:]}}
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
