"""The host program's multi-GPU dispatch (ccsx_amd/csrc/host/dispatch.cpp):
cost model and the round-robin cost-rank partitioner that replaces
kt_for's dynamic dealing of ZMW indices over threads (kthread.c:24-46).
CPU only: the library loads without a GPU."""
import heapq
import random

import pytest

import ccsx_amd as cx


def test_cost_model():
    assert cx.zmw_cost([10000] * 8) == 80000 * 36
    assert cx.zmw_cost([]) == 0


@pytest.mark.parametrize("seed", range(6))
def test_partition_deals_cost_ranks_round_robin(seed):
    rnd = random.Random(seed)
    n = rnd.randint(1, 3000)
    costs = [rnd.randint(0, 10 ** 6) for _ in range(n)]
    nparts, minb = rnd.randint(1, 40), rnd.randint(1, 300)
    order, batches = cx.partition(costs, nparts, minb)
    assert sorted(order) == list(range(n))
    assert [i for b in batches for i in b] == order
    nb = len(batches)
    assert nb == max(1, min(nparts, n // minb))
    # LPT ranks (equal costs in input order), rank r in batch r % nb
    lpt = sorted(range(n), key=lambda i: (-costs[i], i))
    for r, i in enumerate(lpt):
        assert batches[r % nb][r // nb] == i
    # each batch longest first; batch sizes and costs within one ZMW
    for b in batches:
        assert all(costs[x] >= costs[y] for x, y in zip(b, b[1:]))
    assert max(map(len, batches)) - min(map(len, batches)) <= 1
    sums = [sum(costs[i] for i in b) for b in batches]
    assert max(sums) - min(sums) <= max(costs)


def test_partition_edge_cases():
    assert cx.partition([], 4, 10) == ([], [])
    assert cx.partition([5], 4, 10)[1] == [[0]]
    # fewer ZMWs than two minimum batches: one batch
    assert len(cx.partition([1] * 15, 8, 8)[1]) == 1
    # equal costs: ranks in input order, dealt round-robin
    _, bs = cx.partition([1] * 100, 4, 1)
    assert bs == [list(range(k, 100, 4)) for k in range(4)]


def _makespan(costs, batches, workers):
    """Dynamic pulling: each worker takes the next batch when it is free."""
    free = [0.0] * workers
    for b in batches:
        t = heapq.heappop(free)
        heapq.heappush(free, t + sum(costs[i] for i in b))
    return max(free)


def test_partition_balances_a_config_e_chunk():
    """A 16,384-ZMW chunk of config-E-shaped costs (~20x spread) over 16
    contexts, pulled dynamically: the makespan stays within 5 % of perfect
    balance, and no batch is only the chunk's most expensive ZMWs (the
    round-3 contiguous longest-first cut gave its first batch the top 30 %
    of the cost ranks), where an equal-count contiguous split (the round-1
    CLI) is far off when the expensive ZMWs cluster."""
    import bench
    cfg = bench.CONFIGS["E"]
    costs = []
    for h in range(16384):
        L, p = bench.zmw_shape(cfg, h)
        costs.append(int(L * 1.03) * p * (28 + p))
    costs.sort(reverse=True)  # worst case for a count split: the big ones together
    workers = 16
    ideal = sum(costs) / workers
    _, batches = cx.partition(costs, workers, 256)
    assert _makespan(costs, batches, workers) <= 1.05 * ideal
    # every batch spans the cost ranks: its cheapest ZMW is among the chunk's cheapest
    cheap = sorted(costs)[len(costs) // 16]
    assert all(costs[b[-1]] <= cheap for b in batches)
    n = len(costs)
    contiguous = [list(range(n * g // workers, n * (g + 1) // workers)) for g in range(workers)]
    assert _makespan(costs, contiguous, workers) > 1.5 * ideal
