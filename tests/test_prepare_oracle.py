"""The host's ccs_prepare (ccsx_amd/csrc/host/prepare.cpp) against the
oracle's independent restatement of main.c:116-453 (oracle/prep_oracle.c):
push lists (segment offsets, lengths, strands, order) on the reference-pinned
ingest fixtures and on >= 1,000 synthetic ZMWs with truncated, palindromic
(adapter read-through), adapter-carrying, abnormal-length, unrelated and
N-containing subreads -- so the GPU tests' expected outputs, bench.py's
sampled check and oracle/ccsx_cpu compare two independent preparations.
Both sides share only SPEC.md §8 (the un-vendored bsalign aligner's spec),
which each implements on its own; test_pairwise_matches_spec pins them
together.  CPU only."""
import json
import os
import random

import numpy as np
import pytest

import ccsx_amd as cx
from oracle import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "host")
# the PacBio SMRTbell hairpin adapter (45 bases)
ADAPTER = b"ATCTCTCTCAACAACAACAACGGAGGAGGAGGAAAAGAGAGAGAT"
COMP = bytes.maketrans(b"ACGTacgtNn", b"TGCAtgcaNn")


def rc(s: bytes) -> bytes:
    return s.translate(COMP)[::-1]


def same(subs):
    """Product and oracle push lists, and the strand-flipped bases, agree."""
    po, pl, pr = cx.prepare_segments(subs)
    oo, ol, orv = orc.prepare_segments(subs)
    assert list(po) == list(oo) and list(pl) == list(ol) and list(pr) == list(orv), \
        (list(zip(po, pl, pr)), list(zip(oo, ol, orv)))
    assert cx.prepare(subs).seqs == orc.prepare(subs).seqs
    return len(pl), int(np.sum(pr)) if len(pr) else 0


def test_prepare_matches_oracle_on_reference_fixtures():
    with open(os.path.join(GOLD, "expected.json")) as f:
        expected = json.load(f)
    n = 0
    for name, e in sorted(expected.items()):
        for ret, movie, hole, subs in cx.read_calls(os.path.join(GOLD, name), bool(e["is_bam"])):
            if ret > 0:
                same(subs)
                n += 1
    assert n >= 21


def _mutants(rng: random.Random, subs: list[bytes], kind: str) -> list[bytes]:
    subs = list(subs)
    n = len(subs)
    i = rng.randrange(n)
    if kind == "truncated":
        for _ in range(rng.randint(1, 2)):
            j = rng.randrange(n)
            cut = int(len(subs[j]) * rng.uniform(0.2, 0.9))
            subs[j] = subs[j][:cut] if rng.random() < 0.5 else subs[j][-cut:]
    elif kind == "palindromic":
        # adapter read-through: a subread followed by its reverse complement
        subs[i] = subs[i] + (ADAPTER if rng.random() < 0.5 else b"") + rc(subs[i])[: rng.randint(len(subs[i]) // 2,
                                                                                                 len(subs[i]))]
    elif kind == "adapter":
        for _ in range(rng.randint(1, 3)):
            j = rng.randrange(n)
            subs[j] = (ADAPTER + subs[j]) if rng.random() < 0.5 else (subs[j] + ADAPTER)
    elif kind == "long_abnormal":
        # two passes fused (a missed adapter), then the next subreads realigned
        if i + 1 < n:
            subs[i:i + 2] = [subs[i] + subs[i + 1]]
    elif kind == "unrelated":
        subs[i] = bytes(rng.choice(b"ACGT") for _ in range(int(len(subs[i]) * rng.uniform(1.0, 1.5))))
    elif kind == "with_n":
        s = bytearray(subs[i] + subs[(i + 1) % n])
        for _ in range(len(s) // 50):
            s[rng.randrange(len(s))] = ord(rng.choice("NnacgtRY"))
        subs[i] = bytes(s)
    elif kind == "empty":
        subs[i] = b""
    elif kind == "mixed_groups":
        # two length groups of similar size: the template group is chosen by
        # get_template_grp's head / tail checks (main.c:300-342)
        for j in range(0, n, 2):
            subs[j] = subs[j] + subs[j][: len(subs[j]) // 3]
    return subs


KINDS = ["plain", "truncated", "palindromic", "adapter", "long_abnormal", "unrelated", "with_n", "empty",
         "mixed_groups"]


def test_prepare_matches_oracle_on_synthetic_zmws():
    """1,080 synthetic ZMWs (1-3.5 kb inserts, 5-14 passes; 120 per kind),
    compared on a thread pool (ctypes releases the GIL in both preparations)."""
    from concurrent.futures import ThreadPoolExecutor
    rng = random.Random(20201104)
    cases = []
    for k in range(1080):
        kind = KINDS[k % len(KINDS)]
        L = rng.randint(1000, 3500)
        passes = rng.randint(5, 14)
        subs, _ = cx.synth_zmw(20201104, 700_000 + k, L, passes)
        if kind != "plain":
            subs = _mutants(rng, subs, kind)
        cases.append((kind, subs))
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(lambda c: (c[0], len(c[1]), same(c[1])), cases))
    dropped = sum(1 for _, n, (ns, _) in res if ns < n)
    realigned = sum(1 for kind, _, (ns, _) in res if ns and kind in ("palindromic", "long_abnormal", "adapter"))
    flipped = sum(nrev for _, _, (_, nrev) in res)
    # the abnormal-subread paths were exercised, not only the plain walk
    assert dropped > 100 and realigned > 100 and flipped > 1000


@pytest.mark.parametrize("seed", range(6))
def test_pairwise_matches_spec(seed):
    """SPEC.md §8's aligner: the product's (host/pairwise.cpp) and the
    oracle's (prep_oracle.c) agree on every field: related pairs with
    indels, reverse-complement pairs, partial overlaps, unrelated pairs,
    pairs with N (code 4) and short pairs below the k-mer size."""
    rng = np.random.default_rng(seed)
    for _ in range(25):
        t = rng.integers(0, 4, int(rng.integers(5, 4000))).astype(np.uint8)
        kind = rng.integers(0, 5)
        if kind == 0:  # a noisy copy of a window of t
            a = int(rng.integers(0, max(1, len(t) // 3)))
            b = int(rng.integers(a + 1, len(t) + 1))
            q = t[a:b].copy()
            m = rng.random(len(q))
            q[m < 0.05] = rng.integers(0, 4, int((m < 0.05).sum()))
            q = np.delete(q, np.where(rng.random(len(q)) < 0.04)[0])
            q = np.insert(q, np.where(rng.random(len(q)) < 0.06)[0], rng.integers(0, 4, 1)[0])
        elif kind == 1:
            q = (3 - t[::-1]).copy()
        elif kind == 2:
            q = np.concatenate([rng.integers(0, 4, int(rng.integers(0, 400))), t[: len(t) // 2]]).astype(np.uint8)
        elif kind == 3:
            q = rng.integers(0, 4, int(rng.integers(5, 3000))).astype(np.uint8)
        else:
            q = t.copy()
            q[rng.random(len(q)) < 0.03] = 4
        q = q.astype(np.uint8)
        a, b = cx.pairwise(q.tobytes(), t.tobytes()), orc.pairwise(q.tobytes(), t.tobytes())
        assert a == b, (kind, a, b)


def test_prepare_oracle_edge_cases():
    assert orc.prepare_segments([])[1].size == 0
    # one subread: the template alone; two: template + the other reversed
    assert list(orc.prepare_segments([b"ACGT" * 500])[2]) == [0]
    subs, _ = cx.synth_zmw(20201104, 5, 2000, 2)
    assert same(subs)[0] == 2
