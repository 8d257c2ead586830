"""End-to-end timing of the host program (ccsx_amd/bin/ccsx) on a synthetic
subread FASTA: each context layout (CCSX_NGPU groups x CCSX_SLOTS contexts) is
timed by wall clock, outputs must be byte-identical, and the ingest +
prepare rate alone is timed with tools/ingest_bench.cpp on the same file.
Usage: cli_e2e.py NZMW L PASSES [JOBS] [NGPUxSLOTS ...]   (L = 0: config E)"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.gen_synth import write  # noqa: E402

BIN = os.path.join(ROOT, "ccsx_amd", "bin", "ccsx")
IB = os.path.join(ROOT, "build", "ingest_bench")


def main():
    nz, L, passes = (int(x) for x in sys.argv[1:4])
    jobs = sys.argv[4] if len(sys.argv) > 4 else "16"
    layouts = sys.argv[5:] or ["1x1", "1x2", "1x1", "1x2"]
    d = tempfile.mkdtemp()
    fa = os.path.join(d, "in.fa")
    t = time.time()
    write(fa, nz, L, passes)
    print(f"input: {nz} ZMWs, {os.path.getsize(fa) / 1e6:.1f} MB, written in {time.time() - t:.1f} s", flush=True)
    if not os.path.exists(IB):
        os.makedirs(os.path.dirname(IB), exist_ok=True)  # (build/ does not travel to the GPU box)
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I",
                        os.path.join(ROOT, "ccsx_amd", "csrc", "host"), os.path.join(ROOT, "tools", "ingest_bench.cpp"),
                        "-L", os.path.join(ROOT, "ccsx_amd"), "-lccsx_amd", "-lz", "-lpthread",
                        "-Wl,-rpath," + os.path.join(ROOT, "ccsx_amd"), "-o", IB], check=True)
    for chunk in ("16384", "65536"):
        r = subprocess.run([IB, fa, "0", jobs, chunk], capture_output=True, text=True, check=True)
        print(f"ingest+prepare (chunk {chunk}, {jobs} threads): {r.stdout.strip()}", flush=True)
    outs = {}
    for lay in layouts:
        g, s = lay.split("x")
        out = os.path.join(d, f"out{lay}.fa")
        t = time.time()
        r = subprocess.run([BIN, "-A", "-j", jobs, fa, out], capture_output=True, timeout=900,
                           env=dict(os.environ, CCSX_NGPU=g, CCSX_SLOTS=s, CCSX_TIMING=os.environ.get("TIMING", "0")))
        dt = time.time() - t
        if r.returncode:
            sys.exit(f"ccsx failed ({lay}): {r.stderr.decode()[-2000:]}")
        o = open(out, "rb").read()
        if os.environ.get("TIMING"):
            sys.stdout.write(r.stderr.decode())
        print(json.dumps({"layout": lay, "wall_s": round(dt, 3), "zmws_per_s": round(nz / dt, 1),
                          "ccs": o.count(b">")}), flush=True)
        if outs and o != next(iter(outs.values())):
            sys.exit(f"output of {lay} differs")
        outs[lay] = o
    print("all layouts byte-identical:", len(outs) > 0)


if __name__ == "__main__":
    main()
