"""Generate tests/golden/oracle_ccs.json (regression vectors of the oracle)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.oracle import Poa  # noqa: E402
from tests.zmw_cases import synth  # noqa: E402

cases = []
for hole, L, passes, mode in [(1, 2000, 8, 0), (2, 3000, 6, 0), (3, 2500, 5, 1), (4, 1200, 20, 0), (5, 4500, 7, 0)]:
    p = synth(hole, L, passes)
    out = Poa().zmw(p.seqs, p.offs, p.lens, mode)
    cases.append({"hole": hole, "L": L, "passes": passes, "mode": mode, "len": len(out),
                  "sha256": hashlib.sha256(out).hexdigest(), "prefix": out[:60].decode()})
with open(os.path.join(ROOT, "tests", "golden", "oracle_ccs.json"), "w") as f:
    json.dump({"generator": "tools/make_golden.py", "seed": 20201104, "cases": cases}, f, indent=1)
print("wrote", len(cases), "cases")
