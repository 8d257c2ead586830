"""A/B of the host program's pipeline settings on one config-E input: the
FASTA (tools/synth_fa) is generated once, then ccsx_amd/bin/ccsx -A runs it
from stdin once per variant and round (interleaved), output to /dev/null.

    cli_sweep.py --n 100000 --rounds 2 --out DIR "base" "CCSX_SLOTS=3" "CCSX_CHUNK=32768,CCSX_CHUNK0=16384"

A variant is a comma-separated list of NAME=VALUE environment settings
("base": none).  Writes DIR/cli_sweep.json: seconds per variant and round."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "ccsx_amd", "bin", "ccsx")
GEN = os.path.join(ROOT, "tools", "synth_fa")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--hole0", type=int, default=20_000_000)
    ap.add_argument("--jobs", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--gap", type=float, default=5.0,
                    help="seconds between runs (the driver clears the memory the previous process freed)")
    ap.add_argument("--out", required=True)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="ccsx_sweep_", dir=os.environ.get("TMPDIR"))
    fa = os.path.join(tmp, "in.fa")
    res = {"n": a.n, "jobs": a.jobs, "runs": {}}
    try:
        t0 = time.perf_counter()
        with open(fa, "wb") as f:
            subprocess.run([GEN, str(a.n), str(a.hole0), "0", "0", str(a.jobs)], stdout=f, check=True)
        res["gen_s"] = round(time.perf_counter() - t0, 3)
        for r in range(a.rounds):
            for v in a.variants:
                time.sleep(a.gap)
                env = dict(os.environ, CCSX_TIMING="1")
                if v != "base":
                    for kv in v.split(","):
                        k, _, x = kv.partition("=")
                        env[k] = x
                tag = v.replace(",", "_").replace("=", "")
                with open(fa, "rb") as f, open(os.path.join(a.out, f"{tag}_{r}.log"), "w") as log:
                    e0 = time.time()
                    t0 = time.perf_counter()
                    p = subprocess.run([BIN, "-A", "-j", str(a.jobs), "-", "/dev/null"], stdin=f, stderr=log, env=env)
                    dt = time.perf_counter() - t0
                    e1 = time.time()
                if p.returncode != 0:
                    raise SystemExit(f"variant {v}: ccsx exited {p.returncode}")
                res["runs"].setdefault(v, []).append(round(dt, 3))
                # before main / after the CLI's last line (process start, exit)
                pre = post = None
                for line in open(os.path.join(a.out, f"{tag}_{r}.log")):
                    if "main at epoch" in line:
                        pre = float(line.split("main at epoch ")[1].split()[0]) - e0
                    if "exit at epoch" in line:
                        post = e1 - float(line.split("exit at epoch ")[1].split()[0])
                res.setdefault("pre_main_s", {}).setdefault(v, []).append(pre)
                res.setdefault("exit_s", {}).setdefault(v, []).append(post)
                print(f"{v}: {dt:.2f} s = {a.n / dt:.0f} ZMWs/s (before main {pre}, exit {post})", flush=True)
    finally:
        if os.path.exists(fa):
            os.remove(fa)
        os.rmdir(tmp)
    with open(os.path.join(a.out, "cli_sweep.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
