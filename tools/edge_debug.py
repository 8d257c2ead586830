import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccsx_amd as cx
from oracle.oracle import Poa
from tests.zmw_cases import edge_cases
e = cx.Engine(0)
for mode in (1, 0):
    for name, p in edge_cases().items():
        got = e.run([p], mode) if False else None
        e.stage([p]); e.launch(mode)
        try:
            res = e.fetch()
            g, st, cells = res[0]
        except cx.GpuError as ex:
            print(mode, name, "ERROR", ex); continue
        w = Poa().zmw(p.seqs, p.offs, p.lens, mode)
        print(mode, name, "status", st, "ok" if g == w else f"MISMATCH gpu {len(g)} ref {len(w)}")
