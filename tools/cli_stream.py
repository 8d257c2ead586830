"""The host program (ccsx_amd/bin/ccsx) on config-E-scale input read from
stdin (main.c:804-808: INPUT "-"), timed end to end, with a random sample of
its output checked byte for byte against the oracle on the same ZMWs.

    cli_stream.py --n 100000 [--hole0 H] [--jobs 16] [--sample 1000] [--pipe | --fifo-out] --out DIR

The input is tools/synth_fa's config-E FASTA (insert ~U[5,25] kb x 5-12
passes, 10 % error), written to a file first and fed on stdin (--pipe: the
generator's stdout piped straight into the CLI, so the generator's own rate
bounds the run, and the CLI's output read from a FIFO by a thread that keeps
only the sampled records: nothing touches the disk, so a 500k-ZMW run needs
neither 65 GB of input nor 7.5 GB of output on the box; --fifo-out: the
input from a file as usual, the output through the FIFO).  Writes
DIR/cli_stream.json and DIR/cli_stream_timing.log.
Test infrastructure: the oracle is only the checker of the sample."""
import argparse
import json
import os
import random
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BIN = os.path.join(ROOT, "ccsx_amd", "bin", "ccsx")
GEN = os.path.join(ROOT, "tools", "synth_fa")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--hole0", type=int, default=20_000_000)
    ap.add_argument("--jobs", type=int, default=16)
    ap.add_argument("--sample", type=int, default=1000)
    ap.add_argument("--pipe", action="store_true")
    ap.add_argument("--fifo-out", action="store_true")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="ccsx_stream_")
    fa, ccs = os.path.join(tmp, "in.fa"), os.path.join(tmp, "out.fa")
    res = {"n": a.n, "hole0": a.hole0, "jobs": a.jobs, "pipe": a.pipe, "fifo_out": a.fifo_out or a.pipe,
           "workload": "config E: insert ~U[5,25] kb x passes ~U[5,12] (total <= 450 kb), 10% error, FASTA on stdin, "
                       "shredded mode"}
    gen = [GEN, str(a.n), str(a.hole0), "0", "0", str(a.jobs)]
    env = dict(os.environ, CCSX_TIMING="1")
    log = open(os.path.join(a.out, "cli_stream_timing.log"), "w")
    # the sampled holes, drawn before the run (the FIFO reader keeps only them)
    rnd = random.Random(a.hole0 ^ a.n)
    sample = sorted(rnd.sample(range(a.hole0, a.hole0 + a.n), min(a.sample, a.n)))
    want_holes = set(sample)
    scan = {"got": {}, "nrec": 0, "in_order": True, "bytes": 0}

    def read_output(path):
        got, nrec, in_order, last, cur, nb = {}, 0, True, -1, None, 0
        with open(path, "rb") as f:
            for line in f:
                nb += len(line)
                if line.startswith(b">"):
                    nrec += 1
                    h = int(line.split(b"/")[1])
                    in_order &= h > last
                    last = h
                    cur = h if h in want_holes else None
                elif cur is not None:
                    got[cur] = line.rstrip(b"\n")
        scan.update(got=got, nrec=nrec, in_order=in_order, bytes=nb)

    try:
        if a.pipe:
            os.mkfifo(ccs)
            rd = threading.Thread(target=read_output, args=(ccs,))
            rd.start()
            t0 = time.perf_counter()
            g = subprocess.Popen(gen, stdout=subprocess.PIPE)
            r = subprocess.run([BIN, "-A", "-j", str(a.jobs), "-", ccs], stdin=g.stdout, stderr=log, env=env)
            g.stdout.close()
            g.wait()
            res["cli_s"] = time.perf_counter() - t0
            res["input_bytes"] = None
            if r.returncode != 0:
                # unblock the reader if the CLI never opened its output (no
                # reader left: ENXIO, nothing to unblock)
                try:
                    os.close(os.open(ccs, os.O_WRONLY | os.O_NONBLOCK))
                except OSError:
                    pass
            rd.join()
        else:
            t0 = time.perf_counter()
            with open(fa, "wb") as f:
                subprocess.run(gen, stdout=f, check=True)
            res["gen_s"] = time.perf_counter() - t0
            res["input_bytes"] = os.path.getsize(fa)
            print(f"input: {res['input_bytes'] / 1e9:.2f} GB in {res['gen_s']:.1f} s", flush=True)
            rd = None
            if a.fifo_out:
                os.mkfifo(ccs)
                rd = threading.Thread(target=read_output, args=(ccs,))
                rd.start()
            t0 = time.perf_counter()
            with open(fa, "rb") as f:
                r = subprocess.run([BIN, "-A", "-j", str(a.jobs), "-", ccs], stdin=f, stderr=log, env=env)
            res["cli_s"] = time.perf_counter() - t0
            if rd is not None:
                if r.returncode != 0:
                    try:
                        os.close(os.open(ccs, os.O_WRONLY | os.O_NONBLOCK))
                    except OSError:
                        pass
                rd.join()
        log.close()
        if r.returncode != 0:
            raise SystemExit(f"ccsx exited {r.returncode}")
        res["zmws_per_s"] = a.n / res["cli_s"]
        print(f"cli: {a.n} ZMWs in {res['cli_s']:.2f} s = {res['zmws_per_s']:.0f} ZMWs/s", flush=True)
        # the output: one record per ZMW with a CCS, in input (hole) order
        if not (a.pipe or a.fifo_out):
            read_output(ccs)
        got = scan["got"]
        res["records"] = scan["nrec"]
        res["records_in_input_order"] = scan["in_order"]
        res["output_bytes"] = scan["bytes"]
        # the oracle on the sample's push lists
        import bench
        import ccsx_amd as cx
        from oracle.oracle import batch
        t0 = time.perf_counter()
        zs = []
        for h in sample:
            subs, _ = cx.synth_zmw(bench.SEED, h, *bench.zmw_shape(bench.CONFIGS["E"], h))
            zs.append(cx.prepare(subs))
        want, _, _ = batch(zs, 0, a.jobs)
        res["oracle_s"] = time.perf_counter() - t0
        equal = sum(1 for h, w in zip(sample, want) if got.get(h, b"") == w)
        res["sample"] = len(sample)
        res["sample_equal"] = equal
        print(f"sample: {equal}/{len(sample)} CCS byte-equal to the oracle", flush=True)
    finally:
        for p in (fa, ccs):
            if os.path.exists(p):
                os.remove(p)
        os.rmdir(tmp)
    with open(os.path.join(a.out, "cli_stream.json"), "w") as f:
        json.dump(res, f, indent=1)
    if res.get("sample_equal") != res.get("sample") or res["records"] != a.n or not res["records_in_input_order"]:
        raise SystemExit("cli_stream: output check failed")


if __name__ == "__main__":
    main()
