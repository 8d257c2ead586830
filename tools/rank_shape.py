#!/usr/bin/env python3
"""The N = 8 per-rank shape on one GPU: the CLI on one
rank's share of config E (500,000 / 8 = 62,500 ZMWs) at -j 2, 4, 8, 16, bound
to that many CPUs, as bench.py runs each rank at N = 8 (rank_cpus: the job's
CPU share / local ranks).  Per run: process start -> device contexts open ->
first batch -> last batch end -> output done -> exit, the batches' steady
rate, and the whole-run rate against the 500k per-GPU rate.

    python tools/rank_shape.py --n 62500 --jobs 2,4,8,16 --out gpurun_out/TAG

Between runs the device's memory is let back to >= 95 % free (tools/mem_wait.py,
untimed), as bench.py's lines do.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=62500)
    ap.add_argument("--hole0", type=int, default=bench.E_HOLE0)
    ap.add_argument("--jobs", default="2,4,8,16")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--settle", type=float, default=15.0,
                    help="idle seconds before each run: the driver clears the device memory a process freed "
                         "lazily, and the next process's first large allocation waits for it (DESIGN.md §7) -- "
                         "free memory alone (tools/mem_wait.py) does not show it")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="ccsx_shape_", dir=os.environ.get("TMPDIR"))
    fa = os.path.join(tmp, "in.fa")
    allowed = sorted(os.sched_getaffinity(0))
    share = bench.cpu_share()[0]
    t0 = time.perf_counter()
    with open(fa, "wb") as f:
        subprocess.run([bench.SYNTH_FA, str(a.n), str(a.hole0), "0", "0", str(min(16, share))], stdout=f, check=True)
    res = {"n": a.n, "hole0": a.hole0, "input_bytes": os.path.getsize(fa), "gen_s": round(time.perf_counter() - t0, 2),
           "cpu_share": share, "runs": []}
    print(json.dumps({"input_bytes": res["input_bytes"], "gen_s": res["gen_s"]}), flush=True)
    try:
        for rep in range(a.repeat):
            for j in [int(x) for x in a.jobs.split(",")]:
                time.sleep(a.settle)
                mw = bench.wait_device_memory([0])
                cpus = allowed[:j]
                os.sched_setaffinity(0, cpus)
                try:
                    env = dict(os.environ, CCSX_NGPU="1", CCSX_TIMING="1")
                    log = os.path.join(a.out, f"cli_j{j}_{rep}.log")
                    dt, scan = bench.run_cli(fa, a.n, set(), env, j, log)
                finally:
                    os.sched_setaffinity(0, allowed)
                tl = bench.cli_timeline(log)
                r = {"jobs": j, "cpus": bench.cpu_ranges(cpus), "rep": rep, "settle_s": a.settle, "mem_wait_s": mw["mem_wait_s"],
                     "cli_s": round(dt, 3), "zmws_per_s": round(a.n / dt, 1), "records": scan["nrec"],
                     "in_order": scan["in_order"], "timeline": tl}
                if "first_batch_ms" in tl:
                    r["start_to_first_batch_ms"] = tl["first_batch_ms"]
                    r["tail_after_last_batch_ms"] = round(dt * 1e3 - tl["last_batch_end_ms"], 1)
                res["runs"].append(r)
                print(json.dumps(r), flush=True)
    finally:
        os.remove(fa)
        os.rmdir(tmp)
    with open(os.path.join(a.out, "rank_shape.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
