#!/usr/bin/env python3
"""bench.py -- throughput of the ccsx consensus hot path on MI355X.

Workload (BASELINE.json configs[1], "B"): 1,000 synthetic ZMWs per GPU, 10 kb
insert x 8 passes, 10 % PacBio-like error (6 % ins / 3 % del / 1 % sub),
default shredded mode.  A "step" is one launch of the hot path over the whole
batch, inputs (post-ccs_prepare, strand-normalised segments) already resident
in HBM.  Each rank processes its own 1,000 holes (weak scaling, no collective
on the data path); torch.distributed (gloo) is used only for the barrier and
the max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config B|C|D]

Prints ONE JSON line (rank 0).  See DESIGN.md §6 for the roofline model and
profiles/ for the rocprofv3 summaries these numbers are checked against.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# SURVEY.md §8d workloads (per GPU).  B is the metric's configuration.
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
    # instance); shredded mode pushes 2-10 kb windows (the LDS instance with
    # its 8,192-base tight-cap buffer)
    "H": dict(workload="H: 1000 ZMWs x 110 kb insert x 4 passes, 10% error, shredded mode (long subreads)",
              nzmw=1000, L=110000, passes=4, mode=0),
    "HP": dict(workload="HP: 1000 ZMWs x 110 kb insert x 4 passes, 10% error, primitive (-P) mode "
                        "(HBM-read kernel instance)", nzmw=1000, L=110000, passes=4, mode=1),
    # a per-GPU slice of config E (500k ZMWs, mixed 5-25 kb inserts, 5-12 passes)
    "E": dict(workload="E-slice: 2000 ZMWs per GPU, insert ~U[5,25] kb x passes ~U[5,12] (total <= 450 kb), "
                       "10% error, shredded mode", nzmw=2000, L=0, passes=0, mode=0),
}
SEED = 20201104
MODE_SHRED = 0
# gfx950 integer VALU: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6e12 int32 lane-ops/s
# (MI355X_MICROARCH.md: SIMD-32, wave64 in 2 cycles); 10 int ops per DP cell
#  -> 7.86e12 cells/s.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
OPS_PER_CELL = 10


def rank_holes(cfg: dict, rank: int) -> range:
    """Hole ids of one rank: contiguous, disjoint ranges (weak scaling)."""
    return range(rank * cfg["nzmw"], (rank + 1) * cfg["nzmw"])


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


def cpu_baseline(threads: int | None = None, sample_j1: int = 60):
    """Config A (BASELINE.json configs[0]) end to end on the host's CPU cores:
    1,000 synthetic ZMWs (10 kb x 8 passes) as a subread FASTA through
    oracle/ccsx_cpu -- the product's ingest + ccs_prepare around the oracle's
    scalar POA, with ccsx's chunked pipeline and -j threads (kt_for dynamic
    sharing).  It stands in for `ccsx -A -j N`, unbuildable here (bsalign is
    not vendored): a scalar C restatement, not bsalign's SIMD code.
    -j N = the CPUs this process may use (the reference's -j goes straight
    to kt_for, main.c:794-795, kthread.c:48-65): the affinity mask, bounded by
    the cgroup CPU quota when one is set, else by OMP_NUM_THREADS when the
    environment states the job's share that way (a GPU box's affinity mask
    lists the whole machine while it grants the job 16 CPUs; -j 256 there
    measured 101 ZMWs/s against 182 at -j 16, r03e).  The line records
    affinity, quota, OMP_NUM_THREADS and nproc beside N.
    -j 1 runs on a `sample_j1`-ZMW prefix for the per-core rate."""
    import subprocess
    import tempfile
    from tools.gen_synth import write
    exe = os.path.join(ROOT, "oracle", "ccsx_cpu")
    if not os.path.exists(exe):
        from ccsx_amd.build import build_oracle
        build_oracle()
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    # without a cgroup quota, the job's CPU share as its environment states it
    # (OMP_NUM_THREADS: a GPU box sets it to the CPUs it grants per GPU)
    share = quota or int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if threads is None:
        threads = max(1, min(affinity, share) if share else affinity)
    d = tempfile.mkdtemp(prefix="ccsx_cpu_")
    fa, fa1 = os.path.join(d, "a.fa"), os.path.join(d, "a1.fa")
    write(fa, 1000, 10000, 8, seed=SEED)
    write(fa1, sample_j1, 10000, 8, seed=SEED)

    def run(path, j):
        out = path + ".ccs.fa"
        t = time.perf_counter()
        subprocess.run([exe, "-A", "-j", str(j), path, out], check=True)
        dt = time.perf_counter() - t
        n = open(out, "rb").read().count(b">")
        return dt, n

    dt, n = run(fa, threads)
    dt1, n1 = run(fa1, 1)
    for f in os.listdir(d):
        os.remove(os.path.join(d, f))
    os.rmdir(d)
    return {"value": round(n / dt, 3), "unit": "ZMWs/s", "cores": threads, "affinity": affinity,
            "cgroup_cpu_quota": quota, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "nproc": os.cpu_count(),
            "kind": "port",
            "per_core_zmws_per_s": round(n1 / dt1, 3), "wall_s": round(dt, 3),
            "sample": f"config A end to end: {n} CCS from 1,000 ZMWs (10 kb x 8 passes, 10% error) read from FASTA, "
                      f"ccs_prepare, POA and ordered output by oracle/ccsx_cpu -A -j {threads} (the CPUs the process "
                      f"may use: affinity {affinity}, cgroup quota {quota or 'none'}, OMP_NUM_THREADS "
                      f"{os.environ.get('OMP_NUM_THREADS')}; nproc={os.cpu_count()}) in {dt:.2f} s; -j 1 on the first {sample_j1} ZMWs: {n1 / dt1:.2f} ZMWs/s. "
                      "A scalar C restatement of SPEC.md + main.c, not bsalign's SIMD code (ccsx itself is "
                      "unbuildable here)"}


def e2e_line(eng, rank: int, n: int, dist):
    """Config E end to end on the device: n mixed-size ZMWs per GPU (5-25 kb
    inserts x 5-12 passes) from prepared host buffers through ccsx_gpu_run
    (staging, memory-sized slices, launches, full-cap re-runs, CCS fetched to
    host memory).  The first call includes growing the workspace; the second
    (steady state) is the reported rate."""
    import ccsx_amd.native as nat
    cfg = CONFIGS["E"]
    holes = list(range(10_000_000 + rank * n, 10_000_000 + (rank + 1) * n))
    shapes = [zmw_shape(cfg, h) for h in holes]
    batch = nat.SynthBatch(SEED, holes, [s[0] for s in shapes], [s[1] for s in shapes],
                           max(1, min(len(os.sched_getaffinity(0)), 16)))
    t0 = time.perf_counter()
    res = eng.run_batch(batch, MODE_SHRED)
    t1 = time.perf_counter()
    reruns0 = eng.rerun_count()
    res = eng.run_batch(batch, MODE_SHRED)
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
                        "prepared push lists in host memory (ingest timed separately: tools/ingest_bench)"}


def load_traffic(cfg_key: str):
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
        return t.get(cfg_key)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS))
    ap.add_argument("--nzmw", type=int, default=0, help="override ZMWs per GPU (testing only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-zmws", type=int, default=16384, help="ZMWs per GPU of the end-to-end line (0: skip)")
    ap.add_argument("--kcfg", type=int, default=-1, help="force a kernel configuration (0 latency, 1 occupancy, 3 solo, "
                                                         "2 throughput; -1: by slice size)")
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
        dist.init_process_group("gloo")

    import ccsx_amd as cx
    import ccsx_amd.native as nat
    zs = make_batch(cfg, rank)
    # one rank per GPU; with more local ranks than visible GPUs (rehearsing
    # N > 1 on a one-GPU box) ranks share devices round-robin, each with its
    # share of the device memory
    ndev = nat.device_count()
    if ndev <= 0:
        raise SystemExit("bench.py: no HIP device visible")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    eng = cx.Engine(local % ndev)
    sharing = (local_world + ndev - 1) // ndev
    if sharing > 1:
        eng.set_mem_share(sharing)
    if args.kcfg >= 0:
        eng.set_kernel_cfg(args.kcfg)
    eng.stage(zs, cfg["mode"])  # the capacities ccsx_gpu_run uses for the mode
    for _ in range(args.warmup):
        eng.launch(cfg["mode"])

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        kernel_ms.append(eng.launch(cfg["mode"]))  # synchronises on the stream's end event
    t1 = time.perf_counter()
    barrier()
    # results of the last step: status check and the cell count (read back
    # after the timed region so the warmup and timed launches run back to back)
    res = eng.fetch()
    cells_per_step = sum(r[2] for r in res)
    bad = [i for i, r in enumerate(res) if r[1] != 0]
    if bad:
        raise SystemExit(f"device status != 0 for {len(bad)} ZMWs")
    elapsed = t1 - t0
    elapsed, cells_total_step = aggregate(dist, elapsed, cells_per_step)

    if rank == 0:
        n_total = cfg["nzmw"] * world * args.steps
        value = n_total / elapsed
        avg_launch_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        # roofline for the dominant kernel (ccsx_zmw_kernel, the only kernel):
        # algorithmic int ops per launch / average launch duration (HIP events)
        achieved = cells_per_step * OPS_PER_CELL / avg_launch_s / 1e12
        out = {
            "metric": "CCS ZMWs/sec (whole node)",
            "value": round(value, 3),
            "unit": "ZMWs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (SURVEY.md §8d generator, seed 20201104, per-rank hole ranges)",
            "config": {"workload": cfg["workload"], "zmws_per_gpu": cfg["nzmw"], "insert_len": cfg["L"] or "5000-25000",
                       "passes": cfg["passes"] or "5-12", "mode": "shredded" if cfg["mode"] == 0 else "primitive",
                       "parallelism": f"hole-batch sharding x{world}, no collectives"},
            "gcups": round(cells_total_step * args.steps / elapsed / 1e9, 3),
            "cells_per_step": int(cells_total_step),
            "roofline": {"bound": "valu-int32", "achieved": round(achieved, 4), "peak": round(VALU_PEAK_TOPS, 2),
                         "unit": "TOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 5),
                         "frac_vs_packed_int16": round(achieved / (2 * VALU_PEAK_TOPS), 5),
                         "traffic": load_traffic(args.config),
                         "kernel": "ccsx_zmw_kernel", "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                         "ops_per_cell": OPS_PER_CELL, "kernel_cfg": eng.kernel_cfg()},
            "step_ms": [round(k, 3) for k in kernel_ms],
        }
        if sharing > 1:
            # a rehearsal, not a multi-GPU number: ranks share one device
            out["config"]["ranks_per_device"] = sharing
    if args.e2e_zmws:
        e2e = e2e_line(eng, rank, args.e2e_zmws, dist)
    if rank == 0:
        if args.e2e_zmws:
            out["e2e"] = e2e
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
