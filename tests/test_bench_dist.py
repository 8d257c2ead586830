"""bench.py's multi-rank path on CPU (gloo, world_size 2): disjoint hole
ranges per rank, max-over-ranks time, summed cells."""
import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    el, cells = bench.aggregate(dist, 1.0 + rank, 100 * (rank + 1))
    q.put((rank, el, cells))
    dist.destroy_process_group()


def test_aggregate_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert res == [(0, 2.0, 300.0), (1, 2.0, 300.0)]


def test_rank_holes_disjoint():
    cfg = dict(bench.CONFIGS["B"])
    hs = [set(bench.rank_holes(cfg, r)) for r in range(8)]
    assert all(len(h) == cfg["nzmw"] for h in hs)
    assert len(set().union(*hs)) == 8 * cfg["nzmw"]


def test_single_rank_aggregate():
    assert bench.aggregate(None, 1.5, 7) == (1.5, 7.0)


def _run_bench(nproc: int, extra: list[str]):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(root, "bench.py"),
           "--gpus", str(nproc)] + extra
    r = subprocess.run(cmd, cwd=root, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only prints
    return json.loads(lines[0])


import pytest  # noqa: E402


@pytest.mark.gpu
def test_bench_two_ranks_on_device():
    """The driver's N > 1 launch (torch.distributed.run, one process per rank,
    RANK/LOCAL_RANK/WORLD_SIZE from the env) with both ranks on the box's one
    GPU: per-rank hole ranges, barrier, max-over-ranks time, summed cells, one
    JSON line; the config-E headline split over the ranks' CLIs (each over
    its own hole range, its device share halved) with the sample checked
    against the oracle; the e2e line's gather."""
    small = ["--steps", "2", "--warmup", "1", "--nzmw", "96", "--e2e-zmws", "64", "--no-cpu-baseline",
             "--e-zmws", "600", "--e-sample", "12", "--roofline-zmws", "128"]
    one = _run_bench(1, small)
    two = _run_bench(2, small)
    import ccsx_amd.native as nat
    ndev = nat.device_count()
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert "ranks_per_device" not in one["config"]
    # two ranks on fewer than two visible GPUs share a device: the line must
    # say so (a rehearsal, never a two-GPU number); on two or more, it must not
    if ndev < 2:
        assert two["config"]["ranks_per_device"] == 2
    else:
        assert "ranks_per_device" not in two["config"]
    # rank 1 aligns its own 96 holes: the summed cells are two ranks' worth,
    # and the two ranks' cell counts differ (disjoint synthetic holes)
    k1, k2 = one["kernel_B"], two["kernel_B"]
    assert k2["cells_per_step"] > k1["cells_per_step"]
    assert k2["cells_per_step"] != 2 * k1["cells_per_step"]
    # the headline: 600 config-E ZMWs in both runs, rank 0's 300 in order
    assert one["cli"]["zmws"] == 600 and two["cli"]["zmws"] == 300
    assert one["cli"]["sample_equal"] == one["cli"]["sample"] == 12
    assert two["cli"]["sample_equal"] == two["cli"]["sample"] == 12
    assert two["value"] > 0 and two["e2e"]["value"] > 0
    assert two["e2e"]["sample_equal"] == two["e2e"]["sample"] == 64
    assert one["roofline"]["kernel_cfg"] in (0, 1, 3, 4, 5) and one["scaling"] == "strong"
    # the job's CPU share split over the two local ranks, each bound
    share = bench.cpu_share()[0]
    assert one["config"]["cli_jobs"] == share and one["config"]["cli_cpus"] == "unbound"
    assert two["config"]["cli_jobs"] == max(1, share // 2) and two["config"]["cli_cpus"] != "unbound"
    # N > 1: rank 0's one-process line over the whole input, all ranks' GPUs
    op = two["one_process"]
    assert "skipped" not in op, op
    assert op["records"] == 600 and op["records_in_input_order"] and op["ngpu"] == 2
    assert op["sample_equal"] == op["sample"] == 12
    assert "one_process" not in one


def test_e_rank_ranges_split_the_config():
    for world in (1, 2, 3, 8):
        rs = [bench.e_rank_range(500_000, r, world) for r in range(world)]
        assert sum(len(r) for r in rs) == 500_000
        assert all(a.stop == b.start for a, b in zip(rs, rs[1:]))
        assert rs[0].start == bench.E_HOLE0 and max(map(len, rs)) - min(map(len, rs)) <= 1


def test_rank_cpus_split_the_share_over_local_ranks():
    """LOCAL_WORLD_SIZE = 8 on a node whose job share is 128 CPUs of 256
    (two NUMA nodes): each rank's CLI and generator get 128 / 8 = 16 threads,
    bound to disjoint slices, four ranks per NUMA node in rank order."""
    nodes = [list(range(0, 64)) + list(range(128, 192)), list(range(64, 128)) + list(range(192, 256))]
    seen = set()
    for local in range(8):
        t, cpus = bench.rank_cpus(local, 8, share=128, affinity=range(256), nodes=nodes)
        assert t == 16 and len(cpus) == 16
        assert set(cpus) <= set(nodes[local * 2 // 8])
        assert not seen & set(cpus)
        seen |= set(cpus)
    # one rank: the whole share, no binding (the single-GPU runs as before)
    assert bench.rank_cpus(0, 1, share=16, affinity=range(256), nodes=nodes) == (16, None)
    # the one-GPU box's two-rank rehearsal: 16 CPUs of quota -> 8 per rank
    t0, c0 = bench.rank_cpus(0, 2, share=16, affinity=range(256), nodes=[])
    t1, c1 = bench.rank_cpus(1, 2, share=16, affinity=range(256), nodes=[])
    assert t0 == t1 == 8 and not set(c0) & set(c1)
    # fewer CPUs than ranks x threads: still disjoint, never empty
    for local in range(4):
        t, cpus = bench.rank_cpus(local, 4, share=64, affinity=range(8), nodes=[])
        assert t == 16 and len(cpus) == 2
    assert bench.cpu_ranges([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"


def test_disk_need_counts_every_local_input():
    one = bench.input_disk_need(62_500, 1)
    eight = bench.input_disk_need(62_500, 8)
    margin = 4 << 30
    assert eight - margin == 8 * (one - margin)
    # the whole config E split over 8 ranks needs the whole 65.7 GB at once
    assert eight - margin >= 65.7e9


def test_concat_parts_in_rank_order(tmp_path):
    parts = []
    for r in range(3):
        p = tmp_path / f"p{r}.fa"
        p.write_bytes(b">m/%d/0_10\nACGT\n" % r * (1000 + r))
        parts.append(str(p))
    want = b"".join(open(p, "rb").read() for p in parts)
    dst = str(tmp_path / "all.fa")
    bench.concat_parts(parts, dst)
    assert open(dst, "rb").read() == want
    assert not any(os.path.exists(p) for p in parts)


def test_traffic_keyed_by_the_launched_workload(tmp_path):
    """a line's HBM traffic comes from a profile of the
    same workload (key and cells per launch), never another one's; the
    algorithmic bytes (2 bits per cell written and read back) sit beside it."""
    import json
    assert bench.traffic_key("B") == "B"
    assert bench.traffic_key("B", nzmw=200) == "B_n200"
    assert bench.traffic_key(None, roofline_zmws=16384) == "E16384"
    assert bench.traffic_key(None, roofline_zmws=1024) == "E1024"
    p = tmp_path / "traffic.json"
    p.write_text(json.dumps({
        "E16384": {"bytes_per_launch": 1000.0, "cells_per_launch": 400, "source": "profiles/x_summary.md"},
        "B": {"bytes_per_launch": 50.0, "cells_per_launch": 40, "source": "profiles/b_summary.md"},
        "D": {"bytes_per_launch": 70.0, "source": "profiles/old_summary.md"}}))
    assert bench.traffic_entry("E1024", 400, str(p)) is None  # no profile of a 1,024-ZMW launch
    e = bench.traffic_entry("E16384", 400, str(p))
    assert e["key"] == "E16384" and e["cells_match"] is True
    assert e["algorithmic_bytes"] == 400 * 2 * 2 / 8
    assert e["traffic_over_algorithmic"] == round(1000.0 / 200.0, 2)
    assert bench.traffic_entry("E16384", 401, str(p)) is None  # same key, another workload
    assert bench.traffic_entry("B", 40, str(p))["algorithmic_bytes"] == 20.0
    assert bench.traffic_entry("B_n200", 40, str(p)) is None
    assert bench.traffic_entry("D", 40, str(p)) is None  # an old profile that did not record its cells


def test_cli_timeline_parses_the_timing_log(tmp_path):
    log = tmp_path / "cli.log"
    log.write_text("[ccsx] 2 device context(s) open at 212 ms (main at epoch 1.0 s, 0 ms before)\n"
                   "[ccsx] chunk 0: 100 ZMWs read 0-20 ms, prepared until 30 ms, 2 batches\n"
                   "[ccsx] chunk 0 batch of 60 ZMWs on context 0: 233-1233 ms\n"
                   "[ccsx] chunk 0 batch of 40 ZMWs on context 1: 240-1000 ms\n"
                   "[ccsx] output done at 1300 ms; device cells 5; exit at epoch 2.0 s\n")
    t = bench.cli_timeline(str(log))
    assert t["open_ms"] == 212 and t["first_batch_ms"] == 233 and t["last_batch_end_ms"] == 1233
    assert t["output_done_ms"] == 1300 and t["batched_zmws"] == 100 and t["batch_rate_zmws_per_s"] == 100.0
    assert bench.cli_timeline(str(tmp_path / "missing.log")) == {}


def test_one_process_line_devices_and_multi_node_skip(tmp_path):
    """a multi-node job skips the one-process line with a reason
    (the ranks' inputs live on their own nodes); its device list is the
    CLI's context groups modulo the visible devices."""
    import types
    assert bench.one_process_devices(8, 8) == list(range(8))
    assert bench.one_process_devices(2, 1) == [0]
    args = types.SimpleNamespace(e_zmws=1000)
    res = bench.one_process_line(args, 16, [None] * 16, [], str(tmp_path), str(tmp_path), local_world=8, ndev=8)
    assert "multi-node" in res["skipped"]
