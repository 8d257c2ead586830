"""End to end: the C host program (ccsx_amd/bin/ccsx) on a synthetic subread
FASTA vs the oracle applied to the same records (ingest, filters, prepare,
shredded / -P consensus, ordered FASTA output)."""
import os
import subprocess

import pytest

import ccsx_amd as cx
from oracle.oracle import Poa
from tools.gen_synth import write

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ccsx_amd", "bin", "ccsx")


def _expected(path, mode, min_count=3, mn=5000, mx=500000, exclude=()):
    out = []
    g = Poa()
    for movie, hole, subs in cx.read_zmws(path):
        if len(subs) < min_count + 2 or not (mn <= sum(map(len, subs)) <= mx) or hole in exclude:
            continue
        p = cx.prepare(subs)
        ccs = g.zmw(p.seqs, p.offs, p.lens, mode)
        if ccs:
            out.append(b">%s/%s/ccs\n%s\n" % (movie.encode(), hole.encode(), ccs))
    return b"".join(out)


@pytest.mark.parametrize("mode_flag,mode", [([], 0), (["-P"], 1)])
def test_cli_matches_oracle(tmp_path, mode_flag, mode):
    fa = str(tmp_path / "in.fa")
    write(fa, 12, 1500, 7)
    # a ZMW with too few subreads and one outside -m are filtered out
    with open(fa, "ab") as f:
        f.write(b">synth/900/0_10\nACGTACGTAC\n")
        subs, _ = cx.synth_zmw(20201104, 901, 300, 8)
        for i, s in enumerate(subs):
            f.write(b">synth/901/%d_%d\n%s\n" % (i, i + 1, s))
    out = str(tmp_path / "out.fa")
    r = subprocess.run([BIN, "-A", "-j", "2", "-X", "3,5"] + mode_flag + [fa, out], capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    got = open(out, "rb").read()
    assert got == _expected(fa, mode, exclude={"3", "5"})
    assert got.count(b">") == 10


def test_cli_multi_chunk_order(tmp_path):
    """1,100 ZMWs: more than the first 1,024-ZMW chunk (main.c:686-690), so the
    second chunk is read and prepared while the GPU runs the first; the output
    stays in input order and equal to the oracle's."""
    fa = str(tmp_path / "in.fa")
    write(fa, 1100, 1000, 6)
    out = str(tmp_path / "out.fa")
    r = subprocess.run([BIN, "-A", "-j", "4", fa, out], capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    got = open(out, "rb").read()
    assert got.count(b">") == 1100
    assert got == _expected(fa, 0)


def test_cli_two_slots_match_one(tmp_path):
    """Three chunks (1,024 + 4,096 + 180 ZMWs): with two chunk slots per GPU
    chunk k + 1 runs on the device while chunk k drains; the output must be
    byte-identical to one chunk in flight at a time, in input order."""
    fa = str(tmp_path / "in.fa")
    write(fa, 5300, 1000, 6)
    outs = []
    for slots in ("1", "2"):
        out = str(tmp_path / f"out{slots}.fa")
        r = subprocess.run([BIN, "-A", "-j", "8", fa, out], env=dict(os.environ, CCSX_SLOTS=slots),
                           capture_output=True, timeout=300)
        assert r.returncode == 0, r.stderr.decode()
        outs.append(open(out, "rb").read())
    assert outs[0].count(b">") == 5300
    assert outs[0] == outs[1]
