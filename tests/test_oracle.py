"""The oracle (CPU restatement of SPEC.md + main.c's shredding loop): internal
invariants, accuracy sanity against the synthetic truth, and the committed
golden vectors (tests/golden/oracle_ccs.json, made by tools/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

import ccsx_amd as cx
from oracle.oracle import Poa, batch
from tests.zmw_cases import edge_cases, synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _reads(p):
    return [p.seqs[o:o + n] for o, n in zip(p.offs, p.lens)]


def _edit_identity(a: bytes, b: bytes) -> float:
    A = np.frombuffer(a, np.uint8)
    B = np.frombuffer(b, np.uint8)
    prev = np.arange(len(B) + 1, dtype=np.int64)
    ar = np.arange(1, len(B) + 1)
    for i in range(1, len(A) + 1):
        x = np.minimum(prev[:-1] + (A[i - 1] != B), prev[1:] + 1)
        t = np.minimum.accumulate(np.concatenate([[i], x - ar]))
        prev = np.concatenate([[i], np.minimum(x, t[1:] + ar)])
    return 1 - prev[-1] / max(len(A), len(B))


def test_msa_rows_reconstruct_reads():
    """Every MSA read row, gaps removed, is exactly the pushed read (2-bit)."""
    enc = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}
    reads = _reads(synth(11, 1500, 7))
    cns, msa = Poa().poa(reads)
    for k, r in enumerate(reads):
        row = msa[:, k + 1]
        assert bytes(row[row < 4]) == bytes(enc[c] for c in r)
    cons = msa[:, len(reads) + 1]
    assert np.array_equal(cons[cons < 4], cns)
    assert np.all(msa[:, 0] == 4) and np.all(msa[:, len(reads) + 2:] == 4)
    assert np.all((msa[:, 1:len(reads) + 1] < 4).any(axis=1))  # no all-gap column


def test_poa_deterministic_and_order_sensitive():
    reads = _reads(synth(12, 1200, 6))
    a = Poa().poa(reads)
    b = Poa().poa(reads)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_single_read_is_its_own_consensus():
    r = b"ACGTTGCAAGGCTTACG" * 20
    cns, msa = Poa().poa([r])
    assert bytes(b"ACGT"[c] for c in cns) == r


def test_empty_poa():
    cns, msa = Poa().poa([])
    assert len(cns) == 0 and msa.shape[0] == 0
    cns, msa = Poa().poa([b"", b""])
    assert len(cns) == 0


@pytest.mark.parametrize("mode", [0, 1])
def test_accuracy_vs_truth(mode):
    """Not parity: a deterministic-but-wrong restatement would fail this."""
    ids = []
    for h in range(4):
        subs, ins = cx.synth_zmw(20201104, 500 + h, 1500, 8)
        p = cx.prepare(subs)
        ccs = Poa().zmw(p.seqs, p.offs, p.lens, mode)
        ids.append(max(_edit_identity(ccs, ins), _edit_identity(ccs, cx.revcomp(ins))))
    assert min(ids) > 0.985 and np.mean(ids) > 0.99


def test_edge_cases_run():
    for name, p in edge_cases().items():
        for mode in (0, 1):
            out = Poa().zmw(p.seqs, p.offs, p.lens, mode)
            assert set(out) <= set(b"ACGT"), name


def test_batch_equals_serial():
    zs = [synth(h, 1500, 6) for h in range(6)]
    par, _, _ = batch(zs, 0, 4)
    ser = [Poa().zmw(z.seqs, z.offs, z.lens, 0) for z in zs]
    assert par == ser


def test_golden_vectors():
    """Regression pin of the restatement (self-generated: the reference has no
    test vectors and bsalign is unavailable -- parity with bsalign unpinned)."""
    with open(os.path.join(GOLDEN, "oracle_ccs.json")) as f:
        gold = json.load(f)
    for case in gold["cases"]:
        p = synth(case["hole"], case["L"], case["passes"])
        out = Poa().zmw(p.seqs, p.offs, p.lens, case["mode"])
        assert len(out) == case["len"]
        assert hashlib.sha256(out).hexdigest() == case["sha256"]


def test_edit_identity_known_answers():
    """The accuracy checks' banded edit identity (oracle/poa_identity.c)
    against the exact numpy distance above."""
    import random
    from oracle.oracle import edit_identity
    rnd = random.Random(5)
    for _ in range(20):
        a = bytes(rnd.choice(b"ACGT") for _ in range(rnd.randint(50, 400)))
        b = bytearray(a)
        for _ in range(rnd.randint(0, 30)):
            k = rnd.randrange(len(b))
            op = rnd.randrange(3)
            if op == 0:
                b[k] = rnd.choice(b"ACGT")
            elif op == 1:
                del b[k]
            else:
                b.insert(k, rnd.choice(b"ACGT"))
        assert abs(edit_identity(a, bytes(b)) - _edit_identity(a, bytes(b))) < 1e-12
    assert edit_identity(b"", b"ACGT") == 0.0


def test_oracle_object_reuse_fewer_reads_more_columns():
    """One POA object (a batch thread's) runs a config-E ZMW, then a 2-pass
    ZMW whose MSA has fewer rows but more columns: the MSA index array has its
    own capacity (it was sized from the byte capacity and the old row count,
    and the second ZMW wrote past it)."""
    import bench
    import ccsx_amd as cx
    from oracle.oracle import batch
    from tests.zmw_cases import synth
    h = 10_500_000
    big = cx.prepare(cx.synth_zmw(bench.SEED, h, *bench.zmw_shape(bench.CONFIGS["E"], h))[0])
    small = synth(7502, 9000, 2)
    both, _, _ = batch([big, small], 0, 1)
    alone, _, _ = batch([small], 0, 1)
    assert both[1] == alone[0] and len(alone[0]) > 9000
