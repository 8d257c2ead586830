"""Time the CLI (ccsx_amd/bin/ccsx) on a synthetic FASTA with one vs two chunk
slots per GPU (CCSX_SLOTS) and check both write identical output.
Usage: cli_slots.py NZMW L PASSES [JOBS]   (L = 0: config E's mixed sizes)"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.gen_synth import write  # noqa: E402

BIN = os.path.join(ROOT, "ccsx_amd", "bin", "ccsx")


def main():
    nz, L, passes = (int(x) for x in sys.argv[1:4])
    jobs = sys.argv[4] if len(sys.argv) > 4 else "16"
    d = tempfile.mkdtemp()
    fa = os.path.join(d, "in.fa")
    t = time.time()
    write(fa, nz, L, passes)
    print(f"input: {nz} ZMWs, {os.path.getsize(fa) / 1e6:.1f} MB, written in {time.time() - t:.1f} s", flush=True)
    outs = {}
    for slots in os.environ.get("SLOTS", "1,2,1,2").split(","):
        out = os.path.join(d, f"out{slots}.fa")
        t = time.time()
        r = subprocess.run([BIN, "-A", "-j", jobs, fa, out], env=dict(os.environ, CCSX_SLOTS=slots, CCSX_TIMING="1"),
                           capture_output=True, timeout=900)
        dt = time.time() - t
        if r.returncode:
            sys.exit(f"ccsx failed (slots {slots}): {r.stderr.decode()[-2000:]}")
        outs[slots] = open(out, "rb").read()
        sys.stdout.write(r.stderr.decode())
        print(f"slots {slots}: {dt:.2f} s wall, {nz / dt:.0f} ZMWs/s, {outs[slots].count(b'>')} CCS", flush=True)
    if len(outs) < 2:
        return
    print("identical output:", outs["1"] == outs["2"])
    if not outs["1"].count(b">"):
        sys.exit("no CCS written")
    if outs["1"] != outs["2"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
