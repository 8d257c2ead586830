#!/usr/bin/env python3
"""bench.py -- throughput of the ccsx consensus hot path on MI355X.

Headline (BASELINE.json's metric, "CCS ZMWs/sec (whole node)", on config E:
500,000 synthetic ZMWs, inserts ~U[5,25] kb x 5-12 passes, 10 % PacBio-like
error): the C host program ccsx_amd/bin/ccsx -A streams config E's subread
FASTA from stdin (main.c:804-808: INPUT "-") to its ordered CCS output, one
CLI process per GPU, each over its own hole range (the 500,000 ZMWs are split
across the N ranks: strong scaling, no collective on the data path;
torch.distributed (gloo) only for the barrier and the max-over-ranks time).
The timed region is process start to exit of that CLI; a "step" is 1/K of the
rank's ZMWs (the K slices are streamed back to back by the one process), so
ms_per_step x steps is the whole pass.  The FASTA is generated before the
timed region (tools/synth_fa); the CCS are read back through a FIFO, checked
for count and input order, and a sample is compared byte for byte with the
oracle in the cpu_baseline leg (outside the timed region).

Beside it, on the same device:
  * `roofline`: the dominant kernel (the solo object of ccsx_zmw_kernel) on
    16,384 config-E ZMWs per launch, inputs resident in HBM, HIP events on the
    launch stream;
  * `kernel_B`: config B (BASELINE configs[1]: 1,000 ZMWs x 10 kb x 8 passes)
    as K launches with inputs resident, its own roofline;
  * `e2e`: 16,384 config-E ZMWs through ccsx_gpu_run from host buffers;
  * `cpu_baseline` (rank 0, N = 1): oracle/ccsx_cpu -A -j N on a 1,000-ZMW
    sample of the same config-E workload, plus config A (BASELINE configs[0]);
  * `one_process` (rank 0, N > 1): the same 500,000 ZMWs through ONE ccsx
    process driving all N GPUs (CCSX_NGPU=N: host-side dispatch and ordered
    gather), the ranks' inputs concatenated, its sample checked likewise.
Each rank's CLI and generator get the node's CPU share / LOCAL_WORLD_SIZE
threads, bound to a disjoint CPU slice when N > 1 (rank_cpus).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config B|C|D|E|H|HP] [--e-zmws 0]

--e-zmws 0 makes the kernel line of --config the headline (A/B sessions).
Prints ONE JSON line (rank 0).  See DESIGN.md §6 and profiles/.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# SURVEY.md §8d workloads of the kernel line (per GPU).
CONFIGS = {
    "B": dict(workload="B: 1000 ZMWs x 10 kb insert x 8 passes, 10% error, shredded (default) mode",
              nzmw=1000, L=10000, passes=8, mode=0),
    "C": dict(workload="C: 1000 ZMWs x 20 kb insert x 5 passes, 10% error, primitive (-P) mode",
              nzmw=1000, L=20000, passes=5, mode=1),
    "D": dict(workload="D: 10000 ZMWs x 2 kb insert x 30 passes, 10% error, shredded mode",
              nzmw=10000, L=2000, passes=30, mode=0),
    # subreads beyond the LDS read buffer (100 kb; not BASELINE configs, 440 kb
    # per ZMW stays under -M 500000), 1,000 ZMWs like B and C so GCUPS compare
    # at the same chip fill: -P pushes whole segments (the HBM-read kernel
    # instance); shredded mode pushes 2-10 kb windows (the LDS instance)
    "H": dict(workload="H: 1000 ZMWs x 110 kb insert x 4 passes, 10% error, shredded mode (long subreads)",
              nzmw=1000, L=110000, passes=4, mode=0),
    "HP": dict(workload="HP: 1000 ZMWs x 110 kb insert x 4 passes, 10% error, primitive (-P) mode "
                        "(HBM-read kernel instance)", nzmw=1000, L=110000, passes=4, mode=1),
    # a per-GPU slice of config E (500k ZMWs, mixed 5-25 kb inserts, 5-12 passes)
    "E": dict(workload="E-slice: 2000 ZMWs per GPU, insert ~U[5,25] kb x passes ~U[5,12] (total <= 450 kb), "
                       "10% error, shredded mode", nzmw=2000, L=0, passes=0, mode=0),
}
E_WORKLOAD = ("E: 500,000 synthetic ZMWs, insert ~U[5,25] kb x passes ~U[5,12] (total <= 450 kb), 10% error, "
              "subread FASTA on stdin through the ccsx CLI (-A, shredded mode), CCS in input order")
SEED = 20201104
MODE_SHRED = 0
E_HOLE0 = 20_000_000       # config E's holes (the CLI headline)
E_LAUNCH_HOLE0 = 10_000_000  # the roofline / e2e lines' config-E holes
# gfx950 integer VALU: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6e12 int32 lane-ops/s
# (MI355X_MICROARCH.md: SIMD-32, wave64 in 2 cycles); 10 int ops per DP cell
#  -> 7.86e12 cells/s.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
OPS_PER_CELL = 10
CLI = os.path.join(ROOT, "ccsx_amd", "bin", "ccsx")
ORIG_AFFINITY = os.sched_getaffinity(0)  # restored after a rank's CLI ran bound to its slice
SYNTH_FA = os.path.join(ROOT, "tools", "synth_fa")


def rank_holes(cfg: dict, rank: int) -> range:
    """Hole ids of one rank's kernel line: contiguous, disjoint ranges."""
    return range(rank * cfg["nzmw"], (rank + 1) * cfg["nzmw"])


def e_rank_range(total: int, rank: int, world: int) -> range:
    """Config E's holes of one rank: the `total` ZMWs split into contiguous,
    disjoint ranges of near-equal size (strong scaling)."""
    per, extra = divmod(total, world)
    start = rank * per + min(rank, extra)
    return range(E_HOLE0 + start, E_HOLE0 + start + per + (1 if rank < extra else 0))


def aggregate(dist, elapsed: float, cells_per_step: int):
    """(max elapsed over ranks, total cells per step over ranks); dist may be None."""
    if dist is None:
        return elapsed, float(cells_per_step)
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(cells_per_step)], dtype=torch.float64)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), float(c.item())


def zmw_shape(cfg: dict, hole: int):
    """(insert length, passes) of one hole; config E draws them per hole."""
    if cfg["L"]:
        return cfg["L"], cfg["passes"]
    x = (hole * 0x9E3779B97F4A7C15 + SEED) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 31
    x = (x * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 29
    L = 5000 + x % 20001
    passes = 5 + (x >> 20) % 8
    passes = max(5, min(passes, 450000 // (L * 11 // 10)))
    return L, passes


def make_batch(cfg: dict, rank: int):
    import ccsx_amd as cx
    zs = []
    for h in rank_holes(cfg, rank):
        L, passes = zmw_shape(cfg, h)
        subs, _ = cx.synth_zmw(SEED, h, L, passes)
        zs.append(cx.prepare(subs))
    return zs


def e_batch(holes, threads: int):
    """Config-E ZMWs made and prepared on C threads (ccsx_synth_batch_make)."""
    import ccsx_amd.native as nat
    cfg = CONFIGS["E"]
    shapes = [zmw_shape(cfg, h) for h in holes]
    return nat.SynthBatch(SEED, list(holes), [s[0] for s in shapes], [s[1] for s in shapes], threads)


def cgroup_cpu_quota() -> int:
    """CPUs granted by the cgroup (v2 cpu.max, v1 cfs quota), 0 if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, int(q) // int(per))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return 0


def cpu_share():
    """The CPUs this process may use: the affinity mask, bounded by the cgroup
    CPU quota, else by OMP_NUM_THREADS where the environment states the job's
    share that way (a GPU box's affinity mask lists the whole machine while it
    grants the job 16 CPUs).  Returns (threads, affinity, quota)."""
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    share = quota or int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(affinity, share) if share else affinity), affinity, quota


def numa_cpulists():
    """CPU lists of the NUMA nodes (sysfs), [] where unreadable."""
    nodes = []
    base = "/sys/devices/system/node"
    try:
        names = sorted((d for d in os.listdir(base) if d.startswith("node") and d[4:].isdigit()), key=lambda d: int(d[4:]))
    except OSError:
        return []
    for d in names:
        try:
            with open(os.path.join(base, d, "cpulist")) as f:
                spec = f.read().strip()
        except OSError:
            continue
        cpus = []
        for part in filter(None, spec.split(",")):
            lo, _, hi = part.partition("-")
            cpus.extend(range(int(lo), int(hi or lo) + 1))
        nodes.append(cpus)
    return nodes


def rank_cpus(local: int, local_world: int, share: int | None = None, affinity=None, nodes=None):
    """(threads, CPU list) of one local rank's CLI and generator: the job's CPU
    share split over the ranks of the node (each rank's CLI otherwise sizes
    itself to the whole share: local_world-fold oversubscription), and, with
    more than one local rank, a disjoint slice of the allowed CPUs to bind to
    -- ranks dealt over the NUMA nodes in order (GPUs are enumerated in NUMA
    order on the usual nodes), consecutive ranks of a node on consecutive
    slices.  One rank: no binding (None), as in the single-GPU runs."""
    if share is None:
        share = cpu_share()[0]
    per = max(1, share // max(1, local_world))
    if local_world <= 1:
        return per, None
    allowed = sorted(affinity if affinity is not None else os.sched_getaffinity(0))
    aset = set(allowed)
    nodes = [c for c in ([[x for x in n if x in aset] for n in (nodes if nodes is not None else numa_cpulists())]) if c]
    if not nodes:
        nodes = [allowed]
    node = local * len(nodes) // local_world
    peers = [r for r in range(local_world) if r * len(nodes) // local_world == node]
    k, pool = peers.index(local), nodes[node]
    if len(pool) >= per * len(peers):
        cpus = pool[k * per:(k + 1) * per]
    else:
        cpus = pool[k * len(pool) // len(peers):(k + 1) * len(pool) // len(peers)] or pool
    return per, cpus


def read_records(path, want: set, scan: dict):
    """Read a CCS FASTA (a FIFO while the CLI writes it): record count, input
    (hole) order, and the sequences of the holes in `want`."""
    got, nrec, in_order, last, cur, nb = {}, 0, True, -1, None, 0
    with open(path, "rb") as f:
        for line in f:
            nb += len(line)
            if line.startswith(b">"):
                nrec += 1
                h = int(line.split(b"/")[1])
                in_order &= h > last
                last = h
                cur = h if h in want else None
            elif cur is not None:
                got[cur] = line.rstrip(b"\n")
    scan.update(got=got, nrec=nrec, in_order=in_order, bytes=nb)


def run_cli(inp, n_zmw: int, want: set, env: dict, threads: int, log_path: str, gen_cmd=None):
    """ccsx -A -j threads - <FIFO>: the input from file `inp` (or generator
    command gen_cmd piped in), output through a FIFO read by a thread.
    Returns (seconds from process start to exit, scan dict)."""
    d = tempfile.mkdtemp(prefix="ccsx_bench_out_")
    fifo = os.path.join(d, "ccs.fa")
    os.mkfifo(fifo)
    scan = {}
    rd = threading.Thread(target=read_records, args=(fifo, want, scan))
    rd.start()
    try:
        with open(log_path, "w") as log:
            g = None
            if gen_cmd is not None:
                g = subprocess.Popen(gen_cmd, stdout=subprocess.PIPE)
                src = g.stdout
            else:
                src = open(inp, "rb")
            t0 = time.perf_counter()
            r = subprocess.run([CLI, "-A", "-j", str(threads), "-", fifo], stdin=src, stderr=log, env=env)
            dt = time.perf_counter() - t0
            src.close()
            if g is not None:
                g.wait()
        if r.returncode != 0:
            try:  # unblock the reader if the CLI never opened its output
                os.close(os.open(fifo, os.O_WRONLY | os.O_NONBLOCK))
            except OSError:
                pass
        rd.join()
    finally:
        os.remove(fifo)
        os.rmdir(d)
    if r.returncode != 0:
        raise SystemExit(f"ccsx exited {r.returncode} (log {log_path})")
    if scan.get("nrec") != n_zmw or not scan.get("in_order"):
        raise SystemExit(f"ccsx output: {scan.get('nrec')} records for {n_zmw} ZMWs, in order {scan.get('in_order')}")
    return dt, scan


def cli_child_env(local: int, ndev: int, sharing: int) -> dict:
    """The CLI of this rank sees only this rank's GPU (index into what the
    parent sees), shares it with `sharing` ranks, and logs its timing."""
    env = dict(os.environ, CCSX_NGPU="1", CCSX_DEV_SHARE=str(sharing), CCSX_TIMING="1")
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if os.environ.get(var):
            vis = os.environ[var].split(",")
            env["HIP_VISIBLE_DEVICES"] = vis[local % len(vis)]
            break
    else:
        env["HIP_VISIBLE_DEVICES"] = str(local % ndev)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    return env


def cli_cells(log_path: str) -> int:
    with open(log_path) as f:
        for line in f:
            if "device cells " in line:
                return int(line.split("device cells ")[1].split(";")[0].split()[0])
    return 0


def cli_timeline(log_path: str) -> dict:
    """The CLI's CCSX_TIMING log as a timeline (ms from main): device contexts
    open, first batch started, last batch ended, output done, and the batches'
    ZMWs per second between the first start and the last end."""
    t = {}
    first, last, nz = None, None, 0
    try:
        with open(log_path) as f:
            for line in f:
                if "device context(s) open at " in line:
                    t["open_ms"] = float(line.split("open at ")[1].split()[0])
                elif " batch of " in line and " ZMWs on context " in line:
                    a, b = line.rsplit(": ", 1)[1].split(" ms")[0].split("-")
                    a, b = float(a), float(b)
                    first = a if first is None else min(first, a)
                    last = b if last is None else max(last, b)
                    nz += int(line.split(" batch of ")[1].split()[0])
                elif "output done at " in line:
                    t["output_done_ms"] = float(line.split("output done at ")[1].split()[0].rstrip(";"))
    except OSError:
        return t
    if first is not None:
        t["first_batch_ms"], t["last_batch_end_ms"], t["batched_zmws"] = first, last, nz
        if last > first:
            t["batch_rate_zmws_per_s"] = round(nz / ((last - first) / 1e3), 1)
    return t


E_BYTES_PER_ZMW = 132e3 * 1.15  # config-E FASTA bytes per ZMW, with a margin (65.7 GB per 500k)


def input_disk_need(n: int, local_world: int) -> int:
    """Free bytes a rank needs to write its n-ZMW input: every local rank
    writes its input to the same disk at once, plus a 4 GiB margin."""
    return int(n * E_BYTES_PER_ZMW) * max(1, local_world) + (4 << 30)


def cpu_ranges(cpus) -> str:
    """'0-7,16-23' for a CPU list."""
    out, cpus = [], sorted(cpus)
    i = 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(f"{cpus[i]}-{cpus[j]}" if j > i else str(cpus[i]))
        i = j + 1
    return ",".join(out)


def cli_line(args, rank: int, world: int, local: int, local_world: int, ndev: int, sharing: int, dist, out_dir: str):
    """The headline: config E through the CLI, this rank's hole range.  The
    rank's CLI and generator get its share of the node's CPUs (rank_cpus),
    bound to its own CPU slice when several ranks share the node.  Returns
    (result, input path or None, temp dir): the input is kept for the
    one-process line (the caller removes the temp dir)."""
    holes = e_rank_range(args.e_zmws, rank, world)
    n = len(holes)
    threads, cpus = rank_cpus(local, local_world)
    if cpus:
        # children inherit the binding (no preexec_fn: the FIFO reader is a thread)
        os.sched_setaffinity(0, cpus)
    env = cli_child_env(local, ndev, sharing)
    tmp = tempfile.mkdtemp(prefix="ccsx_bench_e_", dir=os.environ.get("TMPDIR"))
    res = {"zmws": n, "hole0": holes.start, "jobs": threads, "cpus": cpu_ranges(cpus) if cpus else "unbound"}
    fa = None
    try:
        # W untimed warmup steps: the same CLI on W x 1,024 other config-E
        # ZMWs (its device memory share quartered, so the driver's clearing
        # of what it frees is done while the main input is generated)
        if args.warmup:
            wn = min(args.warmup * 1024, 16384)
            wf = os.path.join(tmp, "warm.fa")
            with open(wf, "wb") as f:
                subprocess.run([SYNTH_FA, str(wn), str(E_HOLE0 + 5_000_000 + rank * wn), "0", "0", str(threads)],
                               stdout=f, check=True)
            wenv = dict(env, CCSX_DEV_SHARE=str(4 * sharing))
            res["warmup_zmws"] = wn
            res["warmup_s"] = round(run_cli(wf, wn, set(), wenv, threads, os.path.join(out_dir, f"cli_warm_r{rank}.log"))[0], 3)
            os.remove(wf)
        # the input, generated before the timed region (a file; a generator
        # pipe if the disk cannot hold it, whose rate then bounds the run)
        fa = os.path.join(tmp, "e.fa")
        pipe = shutil.disk_usage(tmp).free < input_disk_need(n, local_world)
        gen = [SYNTH_FA, str(n), str(holes.start), "0", "0", str(threads)]
        t0 = time.perf_counter()
        if not pipe:
            with open(fa, "wb") as f:
                subprocess.run(gen, stdout=f, check=True)
            res["input_bytes"] = os.path.getsize(fa)
        res["gen_s"] = round(time.perf_counter() - t0, 3)
        res["input"] = "generator pipe" if pipe else "file on stdin"
        rnd = random.Random(holes.start ^ n)
        sample = sorted(rnd.sample(list(holes), min(args.e_sample, n))) if rank == 0 else []
        if dist is not None:
            dist.barrier()
        log = os.path.join(out_dir, f"cli_r{rank}.log")
        dt, scan = run_cli(fa, n, set(sample), env, threads, log, gen_cmd=gen if pipe else None)
        if dist is not None:
            dist.barrier()
        res["cli_s"] = round(dt, 3)
        res["records"] = scan["nrec"]
        res["records_in_input_order"] = scan["in_order"]
        res["output_bytes"] = scan["bytes"]
        res["cells"] = cli_cells(log)
        res["timeline"] = cli_timeline(log)
        res["sample_holes"] = sample
        res["sample_got"] = scan["got"]
    except BaseException:
        shutil.rmtree(tmp, ignore_errors=True)
        raise
    finally:
        if cpus:
            os.sched_setaffinity(0, ORIG_AFFINITY)
    return res, (None if pipe else fa), tmp


def concat_parts(parts, dst: str) -> None:
    """The per-rank inputs, in rank (= hole) order, into one file; each part
    is removed once appended, so the disk holds the whole input plus one part."""
    with open(dst, "wb") as out:
        for p in parts:
            with open(p, "rb") as src:
                size = os.fstat(src.fileno()).st_size
                off = 0
                try:
                    while off < size:
                        k = os.copy_file_range(src.fileno(), out.fileno(), size - off)
                        if k <= 0:
                            break
                        off += k
                except OSError:
                    pass
                if off < size:  # no in-kernel copy here: the rest by read / write
                    src.seek(off)
                    shutil.copyfileobj(src, out, 16 << 20)
            os.remove(p)


def wait_device_memory(devices, frac: float = 0.95, timeout: float = 120.0) -> dict:
    """Untimed: wait until each device has `frac` of its memory free again
    (the rank CLIs that just exited held most of it, and the driver clears
    it for seconds after: VERDICT r5 weak 7, 6.4 s of a 7.68 s one-process
    line was its device open waiting on that).  Polled in a short-lived
    child process (tools/mem_wait.py), never by re-exec."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "mem_wait.py"), "--devices",
           ",".join(str(d) for d in devices), "--frac", str(frac), "--timeout", str(timeout)]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout + 60)
        out = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else {}
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        out = {}
    out.setdefault("ok", False)
    out["mem_wait_s"] = round(time.perf_counter() - t0, 3)
    return out


def one_process_devices(world: int, ndev: int):
    """The devices the one-process CLI (CCSX_NGPU=world) opens: its context
    groups go to devices g % ndev."""
    return sorted({g % max(1, ndev) for g in range(world)})


def one_process_line(args, world: int, parts, sample, out_dir: str, tmp: str, local_world: int | None = None,
                     ndev: int = 1):
    """N > 1, rank 0: the whole config-E input (the ranks' inputs concatenated
    in hole order) through ONE ccsx process driving all N GPUs (CCSX_NGPU=N:
    the CLI's host-side dispatch of micro-batches to per-GPU contexts and its
    ordered gather, main.c:698-717 / kthread.c:24-46), on the job's whole CPU
    share, timed from process start to exit like the per-rank line, with its
    output checked for count and input order and the same sampled holes kept
    for the oracle comparison."""
    share, _, _ = cpu_share()
    res = {"zmws": args.e_zmws, "jobs": share, "ngpu": world}
    if local_world is not None and local_world != world:
        # the ranks' inputs are files on their own nodes: one process on rank
        # 0's node cannot read them
        res["skipped"] = f"multi-node job ({world} ranks, {local_world} on this node): the one-process line is single-node"
        return res
    if any(p is None for p in parts):
        res["skipped"] = "a rank streamed its input from a generator pipe (no disk room for the inputs)"
        return res
    largest = max(os.path.getsize(p) for p in parts)
    if shutil.disk_usage(tmp).free < largest + (4 << 30):
        res["skipped"] = "no disk room to concatenate the inputs"
        return res
    full = os.path.join(tmp, "e_all.fa")
    t0 = time.perf_counter()
    concat_parts(parts, full)
    res["concat_s"] = round(time.perf_counter() - t0, 3)
    res["input_bytes"] = os.path.getsize(full)
    env = dict(os.environ, CCSX_NGPU=str(world), CCSX_TIMING="1")
    log = os.path.join(out_dir, "cli_one_process.log")
    # untimed, outside cli_s: the memory the rank CLIs just released
    mw = wait_device_memory(one_process_devices(world, ndev))
    res["mem_wait_s"] = mw["mem_wait_s"]
    res["mem_free_frac"] = mw.get("free_frac")
    res["mem_wait_ok"] = mw["ok"]
    try:
        dt, scan = run_cli(full, args.e_zmws, set(sample), env, share, log)
    finally:
        os.remove(full)
    res.update({"cli_s": round(dt, 3), "value": round(args.e_zmws / dt, 3), "unit": "ZMWs/s",
                "records": scan["nrec"], "records_in_input_order": scan["in_order"], "cells": cli_cells(log),
                "timeline": cli_timeline(log), "sample_got": scan["got"]})
    return res


def oracle_check(pairs, threads: int):
    """Checker only (test infrastructure): the oracle's CCS of each prepared
    ZMW against the device's.  pairs = [(Prepared, device CCS bytes)]."""
    from oracle.oracle import batch
    want, _, _ = batch([p for p, _ in pairs], MODE_SHRED, threads)
    return sum(1 for (_, g), w in zip(pairs, want) if g == w)


def cpu_baseline(sample_holes, sample_got, threads: int | None = None, sample_j1: int = 60, timed: bool = True,
                 others=None):
    """The CPU leg: oracle/ccsx_cpu (the product's ingest around the oracle's
    own ccs_prepare and scalar POA, ccsx's chunked pipeline, -j threads with kt_for's
    dynamic sharing) -- a stand-in for `ccsx -A -j N`, unbuildable here
    (bsalign is not vendored): a scalar C restatement, not bsalign's SIMD code.
    On the same workload as the headline: the sampled config-E holes as a
    subread FASTA, timed, and its CCS compared byte for byte with the GPU
    CLI's for those holes (the checker).  Then config A (BASELINE configs[0],
    1,000 ZMWs x 10 kb x 8 passes) and -j 1 on a `sample_j1`-ZMW prefix of it
    for the per-core rate.  -j N = the CPUs the process may use (the
    reference's -j goes straight to kt_for, main.c:794-795).  `others`: more
    {name: {hole: CCS}} outputs of the same holes (the one-process line),
    each compared with the same oracle run."""
    from tools.gen_synth import write
    exe = os.path.join(ROOT, "oracle", "ccsx_cpu")
    if not os.path.exists(exe):
        from ccsx_amd.build import build_oracle
        build_oracle()
    n_thr, affinity, quota = cpu_share()
    if threads is None:
        threads = n_thr
    d = tempfile.mkdtemp(prefix="ccsx_cpu_")

    def ccs_of(out):
        got, cur = {}, None
        with open(out, "rb") as f:
            for line in f:
                if line.startswith(b">"):
                    cur = int(line.split(b"/")[1])
                elif cur is not None:
                    got[cur] = line.rstrip(b"\n")
        return got

    try:
        se = os.path.join(d, "e_sample.fa")
        write(se, 0, 0, 0, seed=SEED, holes=sample_holes)
        t = time.perf_counter()
        subprocess.run([exe, "-A", "-j", str(threads), se, se + ".ccs.fa"], check=True)
        dt = time.perf_counter() - t
        cpu_ccs = ccs_of(se + ".ccs.fa")
        def n_equal(got):
            return sum(1 for h in sample_holes if cpu_ccs.get(h, b"") == got.get(h, b"") and h in cpu_ccs)

        equal = n_equal(sample_got)
        others_equal = {k: n_equal(g) for k, g in (others or {}).items()}
        res = {"value": round(len(sample_holes) / dt, 3), "unit": "ZMWs/s", "cores": threads, "kind": "port",
               "affinity": affinity, "cgroup_cpu_quota": quota, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
               "nproc": os.cpu_count(), "wall_s": round(dt, 3),
               "sample_zmws": len(sample_holes), "sample_equal_to_gpu_cli": equal,
               "sample": f"config E sample: {len(sample_holes)} random holes of the headline's hole range as a subread "
                         f"FASTA, read, ccs_prepare, POA and ordered output by oracle/ccsx_cpu -A -j {threads} "
                         f"(the CPUs the process may use: affinity {affinity}, cgroup quota {quota or 'none'}, "
                         f"OMP_NUM_THREADS {os.environ.get('OMP_NUM_THREADS')}; nproc={os.cpu_count()}) in {dt:.2f} s; "
                         f"{equal}/{len(sample_holes)} CCS byte-equal to the GPU CLI's. A scalar C restatement of "
                         "SPEC.md + main.c, not bsalign's SIMD code (ccsx itself is unbuildable here)"}
        if others_equal:
            res["sample_equal_others"] = others_equal
        if timed:
            fa, fa1 = os.path.join(d, "a.fa"), os.path.join(d, "a1.fa")
            write(fa, 1000, 10000, 8, seed=SEED)
            write(fa1, sample_j1, 10000, 8, seed=SEED)
            t = time.perf_counter()
            subprocess.run([exe, "-A", "-j", str(threads), fa, fa + ".o"], check=True)
            dta = time.perf_counter() - t
            t = time.perf_counter()
            subprocess.run([exe, "-A", "-j", "1", fa1, fa1 + ".o"], check=True)
            dt1 = time.perf_counter() - t
            res["config_A"] = {"value": round(1000 / dta, 3), "unit": "ZMWs/s", "cores": threads, "wall_s": round(dta, 3),
                               "per_core_zmws_per_s": round(sample_j1 / dt1, 3),
                               "sample": f"config A end to end: 1,000 ZMWs (10 kb x 8 passes) -j {threads}; "
                                         f"-j 1 on the first {sample_j1} ZMWs"}
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return res


def kernel_line(eng, cfg: dict, zs, steps: int, warmup: int, dist):
    """K launches of one staged batch (inputs resident in HBM), HIP events on
    the launch stream; returns the line with its roofline."""
    eng.stage(zs, cfg["mode"])  # the capacities ccsx_gpu_run uses for the mode
    for _ in range(warmup):
        eng.launch(cfg["mode"])
    if dist is not None:
        dist.barrier()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        kernel_ms.append(eng.launch(cfg["mode"]))  # synchronises on the stream's end event
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    res = eng.fetch()
    cells_per_step = sum(r[2] for r in res)
    bad = [i for i, r in enumerate(res) if r[1] != 0]
    if bad:
        raise SystemExit(f"device status != 0 for {len(bad)} ZMWs")
    elapsed, cells_total_step = aggregate(dist, t1 - t0, cells_per_step)
    avg_launch_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    # roofline of the dominant kernel (ccsx_zmw_kernel, the only kernel):
    # algorithmic int ops per launch / average launch duration (HIP events)
    achieved = cells_per_step * OPS_PER_CELL / avg_launch_s / 1e12
    return {"value": round(cfg["nzmw"] * (dist.get_world_size() if dist else 1) * steps / elapsed, 3),
            "unit": "ZMWs/s", "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
            "gcups": round(cells_total_step * steps / elapsed / 1e9, 3), "cells_per_step": int(cells_total_step),
            "roofline": {"bound": "valu-int32", "achieved": round(achieved, 4), "peak": round(VALU_PEAK_TOPS, 2),
                         "unit": "TOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 5),
                         "frac_vs_packed_int16": round(achieved / (2 * VALU_PEAK_TOPS), 5),
                         "kernel": "ccsx_zmw_kernel", "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                         "ops_per_cell": OPS_PER_CELL, "kernel_cfg": eng.kernel_cfg()},
            "step_ms": [round(k, 3) for k in kernel_ms]}


def e2e_line(eng, batch, n: int, dist, keep):
    """Config E end to end on the device: n mixed-size ZMWs per GPU from
    prepared host buffers through ccsx_gpu_run (staging, memory-sized slices,
    launches, full-cap re-runs, CCS fetched to host memory).  The first call
    includes growing the workspace; the second (steady state) is the rate."""
    t0 = time.perf_counter()
    eng.run_batch(batch, MODE_SHRED)
    t1 = time.perf_counter()
    reruns0 = eng.rerun_count()
    res, kept = eng.run_batch(batch, MODE_SHRED, keep)
    t2 = time.perf_counter()
    reruns = eng.rerun_count() - reruns0
    bad = sum(1 for r in res if r[0] != 0)
    if bad:
        raise SystemExit(f"e2e: device status != 0 for {bad} ZMWs")
    first, steady = t1 - t0, t2 - t1
    if dist is not None:
        import torch
        t = torch.tensor([first, steady], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        first, steady = float(t[0]), float(t[1])
    world = dist.get_world_size() if dist is not None else 1
    cells = sum(r[1] for r in res)
    return {"metric": "CCS ZMWs/sec end to end (host buffers in, CCS in host memory out)",
            "value": round(n * world / steady, 3), "unit": "ZMWs/s", "zmws_per_gpu": n, "s": round(steady, 3),
            "first_call_s": round(first, 3), "gbases_per_s": round(batch.bases * world / steady / 1e9, 3),
            "gcups": round(cells * world / steady / 1e9, 3), "reruns": reruns,
            "workload": "config E slice: insert ~U[5,25] kb x passes ~U[5,12], 10% error, shredded mode, "
                        "prepared push lists in host memory (ingest timed separately: tools/ingest_bench)"}, kept


def load_traffic(cfg_key: str, path: str | None = None):
    p = path or os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
        return t.get(cfg_key)
    except (OSError, ValueError):
        return None


def traffic_key(config: str | None, nzmw: int = 0, roofline_zmws: int = 0) -> str:
    """profiles/traffic.json key of the workload a line launched: the
    roofline line's config-E launch size (E16384), or the kernel line's
    config, with its ZMW count when --nzmw overrides it (B_n200)."""
    if roofline_zmws:
        return f"E{roofline_zmws}"
    return f"{config}_n{nzmw}" if nzmw else str(config)


def traffic_entry(key: str, cells_per_launch: int, path: str | None = None):
    """The PMC traffic of exactly this workload (None when no profile of it
    exists -- never another workload's), with the algorithmic bytes beside
    it: 2 bits of traceback per DP cell, written by the DP and read back by
    the traceback (north_star's 2-bit traceback matrices), so the ratio says
    how far the HBM traffic is above that."""
    t = load_traffic(key, path)
    if t is None or t.get("cells_per_launch") is None:
        return None  # no profile of this workload (or one too old to say which cells it launched)
    out = dict(t, key=key)
    out["cells_match"] = int(t["cells_per_launch"]) == int(cells_per_launch)
    if not out["cells_match"]:
        return None  # the profile measured a different workload under this key
    alg = cells_per_launch * 2 * 2 / 8
    out["algorithmic_bytes"] = alg
    if alg and t.get("bytes_per_launch"):
        out["traffic_over_algorithmic"] = round(t["bytes_per_launch"] / alg, 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS), help="the kernel line's configuration")
    ap.add_argument("--nzmw", type=int, default=0, help="override the kernel line's ZMWs per GPU (testing only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e-zmws", type=int, default=500_000,
                    help="config E ZMWs of the CLI headline, over all ranks (0: the kernel line is the headline)")
    ap.add_argument("--e-sample", type=int, default=1000, help="sampled config-E holes checked against the oracle")
    ap.add_argument("--roofline-zmws", type=int, default=16384,
                    help="config-E ZMWs per launch of the roofline line (0: skip; the kernel line's roofline)")
    ap.add_argument("--e2e-zmws", type=int, default=16384, help="ZMWs per GPU of the end-to-end line (0: skip)")
    ap.add_argument("--no-kernel-line", action="store_true", help="skip the --config kernel line (profiling runs)")
    ap.add_argument("--kcfg", type=int, default=-1, help="force a kernel configuration (0 latency, 1 occupancy, 3 solo, "
                                                         "2 throughput; -1: by slice size)")
    ap.add_argument("--wg-cap", type=int, default=0, help="measurement: at most this many workgroups per CU (0: off)")
    ap.add_argument("--out-dir", default=os.path.join(ROOT, "gpurun_out", "bench"), help="CLI logs")
    ap.add_argument("--no-one-process", dest="one_process", action="store_false",
                    help="N > 1: skip rank 0's one-process line (one CLI over all N GPUs)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.nzmw:
        cfg["nzmw"] = args.nzmw

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        # gloo's C++ side prints "[Gloo] Rank r is connected ..." to stdout
        # while the group forms: sent to stderr, so rank 0's stdout stays the
        # one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    os.makedirs(args.out_dir, exist_ok=True)

    import ccsx_amd as cx
    import ccsx_amd.native as nat
    zs = make_batch(cfg, rank) if not args.no_kernel_line else None
    # one rank per GPU; with more local ranks than visible GPUs (rehearsing
    # N > 1 on a one-GPU box) ranks share devices round-robin, each with its
    # share of the device memory
    ndev = nat.device_count()
    if ndev <= 0:
        raise SystemExit("bench.py: no HIP device visible")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    sharing = (local_world + ndev - 1) // ndev
    eng = cx.Engine(local % ndev)
    if sharing > 1:
        eng.set_mem_share(sharing)
    if args.kcfg >= 0:
        eng.set_kernel_cfg(args.kcfg)
    if args.wg_cap:
        eng.set_wg_cap(args.wg_cap)
    overrides = {k: os.environ[k] for k in ("CCSX_LIB",) if os.environ.get(k)}
    if args.wg_cap:
        overrides["wg_cap"] = args.wg_cap
    threads = rank_cpus(local, local_world)[0]  # this rank's part of the node's CPU share

    # config B (or --config): K launches, inputs resident
    kline = None
    if zs is not None:
        kline = kernel_line(eng, cfg, zs, args.steps, args.warmup, dist)
        kline["traffic"] = traffic_entry(traffic_key(args.config, args.nzmw), kline["cells_per_step"])
        kline["workload"] = cfg["workload"]
    # the dominant kernel of the headline workload: config-E ZMWs per launch,
    # inputs resident (the solo object at this size)
    rline = None
    ebatch = None
    if args.roofline_zmws:
        ebatch = e_batch(range(E_LAUNCH_HOLE0 + rank * args.roofline_zmws,
                               E_LAUNCH_HOLE0 + (rank + 1) * args.roofline_zmws), min(threads, 16))
        eng.stage_batch(ebatch, MODE_SHRED)
        ecfg = dict(nzmw=args.roofline_zmws, mode=MODE_SHRED)
        rsteps = max(1, min(args.steps, 5))
        for _ in range(min(args.warmup, 1)):
            eng.launch(MODE_SHRED)
        ms = [eng.launch(MODE_SHRED) for _ in range(rsteps)]
        res = eng.fetch()
        if any(r[1] != 0 for r in res):
            raise SystemExit("roofline line: device status != 0")
        cells = sum(r[2] for r in res)
        avg = sum(ms) / len(ms) / 1e3
        achieved = cells * OPS_PER_CELL / avg / 1e12
        rline = {"bound": "valu-int32", "achieved": round(achieved, 4), "peak": round(VALU_PEAK_TOPS, 2),
                 "unit": "TOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 5),
                 "frac_vs_packed_int16": round(achieved / (2 * VALU_PEAK_TOPS), 5),
                 "traffic": traffic_entry(traffic_key(None, roofline_zmws=args.roofline_zmws), cells),
                 "kernel": "ccsx_zmw_kernel", "kernel_cfg": eng.kernel_cfg(),
                 "avg_launch_ms": round(avg * 1e3, 3), "launches": rsteps, "ops_per_cell": OPS_PER_CELL,
                 "cells_per_launch": int(cells), "zmws_per_launch": ecfg["nzmw"],
                 "zmws_per_s_per_launch": round(ecfg["nzmw"] / avg, 3),
                 "launch_ms": [round(x, 3) for x in ms],
                 "workload": f"{ecfg['nzmw']} config-E ZMWs per launch (holes from {E_LAUNCH_HOLE0}), inputs resident"}
    e2e, e2e_kept, e2e_keep = None, {}, []
    if args.e2e_zmws:
        b2 = ebatch if ebatch is not None and ebatch.n == args.e2e_zmws else e_batch(
            range(E_LAUNCH_HOLE0 + rank * args.e2e_zmws, E_LAUNCH_HOLE0 + (rank + 1) * args.e2e_zmws), min(threads, 16))
        e2e_keep = sorted(random.Random(7 + rank).sample(range(args.e2e_zmws), min(64, args.e2e_zmws)))
        e2e, e2e_kept = e2e_line(eng, b2, args.e2e_zmws, dist, e2e_keep)
        e2e_holes = [E_LAUNCH_HOLE0 + rank * args.e2e_zmws + i for i in e2e_keep]
    eng.close()
    del ebatch

    cli = None
    one = None
    if args.e_zmws:
        cli, part, tmp = cli_line(args, rank, world, local, local_world, ndev, sharing, dist, args.out_dir)
        try:
            cli_s, cells_all = aggregate(dist, cli["cli_s"], cli["cells"])
            if dist is not None and args.one_process:
                # the ranks' inputs to rank 0, which runs them through one CLI
                # on all N GPUs while the other ranks wait
                parts = [None] * world
                dist.all_gather_object(parts, part)
                if rank == 0:
                    # (a failure here is reported in the line, never fatal: the
                    # other ranks wait at the barrier and the headline stands)
                    try:
                        one = one_process_line(args, world, parts, cli["sample_holes"], args.out_dir, tmp,
                                               local_world=local_world, ndev=ndev)
                    except Exception as e:  # noqa: BLE001
                        one = {"zmws": args.e_zmws, "ngpu": world, "error": f"{type(e).__name__}: {e}"[:400]}
                dist.barrier()
        finally:
            shutil.rmtree(tmp, ignore_errors=True)

    if rank == 0:
        out = {"metric": "CCS ZMWs/sec (whole node)"}
        if cli is not None:
            value = args.e_zmws / cli_s
            out.update({
                "value": round(value, 3), "unit": "ZMWs/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(cli_s / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "int32",
                "data": "synthetic (SURVEY.md §8d generator, seed 20201104, per-rank hole ranges)",
                "config": {"workload": E_WORKLOAD, "zmws": args.e_zmws, "insert_len": "5000-25000", "passes": "5-12",
                           "mode": "shredded", "parallelism": f"hole-range sharding x{world}, one CLI per GPU, "
                                                              "no collectives",
                           "step": f"1/{args.steps} of each rank's config-E ZMWs; the CLI streams the {args.steps} "
                                   "slices back to back in one process, timed from its start to its exit",
                           "cli_jobs": cli["jobs"], "cli_cpus": cli["cpus"]},
                # steps / ms_per_step are nominal: ONE CLI process per rank is
                # timed from its start to its exit, and ms_per_step x steps is
                # that whole time (no per-step clock); warmup = one separate,
                # smaller CLI run (warmup x 1,024 ZMWs) before the input is made
                "steps_nominal": True,
                "timed_region": "one ccsx process per rank, start to exit (max over ranks); "
                                "ms_per_step = that time / steps",
                "gcups": round(cells_all / cli_s / 1e9, 3),
                "cli": {k: v for k, v in cli.items() if k not in ("sample_holes", "sample_got")},
            })
            out["roofline"] = rline if rline is not None else kline["roofline"] if kline is not None else None
            if kline is not None:
                out["kernel_B" if args.config == "B" else f"kernel_{args.config}"] = kline
        elif kline is None:
            # profiling runs: the config-E launch line alone
            if rline is None:
                raise SystemExit("bench.py: nothing to measure")
            out.update({
                "value": rline["zmws_per_s_per_launch"], "unit": "ZMWs/s", "n_gpus": world,
                "steps": rline["launches"], "warmup": min(args.warmup, 1), "ms_per_step": rline["avg_launch_ms"],
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
                "data": "synthetic (SURVEY.md §8d generator, seed 20201104, per-rank hole ranges)",
                "config": {"workload": rline["workload"], "parallelism": f"hole-batch sharding x{world}"},
                "gcups": round(rline["cells_per_launch"] / rline["avg_launch_ms"] * 1e3 / 1e9, 3),
                "roofline": rline})
        else:
            out.update({
                "value": kline["value"], "unit": "ZMWs/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": kline["ms_per_step"], "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "int32",
                "data": "synthetic (SURVEY.md §8d generator, seed 20201104, per-rank hole ranges)",
                "config": {"workload": cfg["workload"], "zmws_per_gpu": cfg["nzmw"],
                           "insert_len": cfg["L"] or "5000-25000", "passes": cfg["passes"] or "5-12",
                           "mode": "shredded" if cfg["mode"] == 0 else "primitive",
                           "parallelism": f"hole-batch sharding x{world}, no collectives"},
                "gcups": kline["gcups"], "cells_per_step": kline["cells_per_step"],
                "roofline": dict(kline["roofline"], traffic=kline["traffic"]),
                "step_ms": kline["step_ms"],
            })
            if rline is not None:
                out["roofline_E"] = rline
        if sharing > 1:
            # a rehearsal, not a multi-GPU number: ranks share one device
            out["config"]["ranks_per_device"] = sharing
        if overrides:
            out["config"]["overrides"] = overrides
        if e2e is not None:
            out["e2e"] = e2e
        # the checker / CPU leg (outside every timed region)
        if not args.no_cpu_baseline or cli is not None or e2e is not None:
            from ccsx_amd import synth_zmw
            from oracle.oracle import prepare as oracle_prepare  # the checker's own ccs_prepare
            if e2e is not None:
                pairs = [(oracle_prepare(synth_zmw(SEED, h, *zmw_shape(CONFIGS["E"], h))[0]), e2e_kept[i])
                         for h, i in zip(e2e_holes, e2e_keep)]
                e2e["sample"] = len(pairs)
                e2e["sample_equal"] = oracle_check(pairs, threads)
            if cli is not None:
                others = {"one_process": one["sample_got"]} if one is not None and "sample_got" in one else None
                cb = cpu_baseline(cli["sample_holes"], cli["sample_got"],
                                  timed=world == 1 and not args.no_cpu_baseline, others=others)
                out["cli"]["sample"] = cb["sample_zmws"]
                out["cli"]["sample_equal"] = cb["sample_equal_to_gpu_cli"]
                if one is not None:
                    out["one_process"] = {k: v for k, v in one.items() if k != "sample_got"}
                    if others:
                        out["one_process"]["sample"] = cb["sample_zmws"]
                        out["one_process"]["sample_equal"] = cb["sample_equal_others"]["one_process"]
                if world == 1 and not args.no_cpu_baseline:
                    out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
        bad = []
        if cli is not None and out["cli"]["sample_equal"] != out["cli"]["sample"]:
            bad.append("CLI sample")
        op = out.get("one_process", {})
        if "sample" in op and op["sample_equal"] != op["sample"]:
            bad.append("one-process CLI sample")
        if e2e is not None and e2e.get("sample_equal") != e2e.get("sample"):
            bad.append("e2e sample")
        if bad:
            raise SystemExit("bench.py: oracle check failed: " + ", ".join(bad))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
