"""Synthetic ZMW inputs shared by the CPU and GPU tests (seeded, deterministic)."""
from __future__ import annotations

import random

import numpy as np

import ccsx_amd as cx

SEED = 20201104


def synth(hole: int, L: int, passes: int, seed: int = SEED) -> cx.Prepared:
    subs, _ = cx.synth_zmw(seed, hole, L, passes)
    return cx.prepare(subs)


def raw(segs: list[bytes]) -> cx.Prepared:
    """Segments given directly (already strand-normalised), push order as listed."""
    offs, o = [], 0
    for s in segs:
        offs.append(o)
        o += len(s)
    return cx.Prepared(b"".join(segs), np.array(offs, np.uint32), np.array([len(s) for s in segs], np.uint32))


def mutate(rng: random.Random, s: bytes, p_ins=0.06, p_del=0.03, p_sub=0.01) -> bytes:
    out = bytearray()
    for c in s:
        u = rng.random()
        if u < p_del:
            pass
        elif u < p_del + p_sub:
            out.append(rng.choice([b for b in b"ACGT" if b != c]))
        else:
            out.append(c)
        if rng.random() < p_ins:
            out.append(rng.choice(b"ACGT"))
    return bytes(out)


def edge_cases() -> dict[str, cx.Prepared]:
    rng = random.Random(7)
    ins = bytes(rng.choice(b"ACGT") for _ in range(3500))
    cases = {}
    cases["one_segment"] = raw([mutate(rng, ins)])
    cases["two_segments"] = raw([mutate(rng, ins), mutate(rng, ins)])
    cases["short_reads_60bp"] = raw([mutate(rng, ins[:60]) for _ in range(6)])
    cases["shorter_than_band"] = raw([mutate(rng, ins[:100]) for _ in range(5)])
    cases["with_empty_segment"] = raw([mutate(rng, ins), b"", mutate(rng, ins), mutate(rng, ins), mutate(rng, ins)])
    cases["identical_reads"] = raw([ins] * 5)
    cases["unrelated_reads"] = raw([bytes(rng.choice(b"ACGT") for _ in range(3100)) for _ in range(5)])
    hp = b"".join(bytes([rng.choice(b"ACGT")]) * rng.randint(1, 9) for _ in range(700))
    cases["homopolymers"] = raw([mutate(rng, hp) for _ in range(7)])
    lc = bytes(rng.choice(b"ACGTacgtN") for _ in range(3200))
    cases["lowercase_and_N"] = raw([mutate(rng, lc) for _ in range(5)])
    cases["noisy_no_breakpoint"] = raw([mutate(rng, ins, 0.15, 0.10, 0.05) for _ in range(6)])
    cases["ragged_lengths"] = raw([mutate(rng, ins[rng.randint(0, 300):3500 - rng.randint(0, 300)]) for _ in range(8)])
    cases["many_passes_short"] = raw([mutate(rng, ins[:1200]) for _ in range(40)])
    cases["over_64_reads"] = raw([mutate(rng, ins[:700]) for _ in range(70)])
    return cases


def high_indegree(seed: int = 7):
    """91 reads P + M[:k] + S (k = 100 .. 10): each deletes a different suffix
    of M, so S's first node gets one in-edge per read -- a far row with more
    than 63 predecessors (more than a 6-bit slot tag holds)."""
    import random
    rnd = random.Random(seed)

    def rb(n):
        return bytes(rnd.choice(b"ACGT") for _ in range(n))
    P, M, S = rb(300), rb(100), rb(300)
    return [P + M[:k] + S for k in range(100, 9, -1)]
