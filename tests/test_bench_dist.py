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
