"""End to end: the C host program (ccsx_amd/bin/ccsx) on a synthetic subread
FASTA vs the oracle applied to the same records (ingest, filters, prepare,
shredded / -P consensus, ordered FASTA output)."""
import os
import subprocess

import pytest

import ccsx_amd as cx
from oracle.oracle import batch
from oracle.oracle import prepare as oracle_prepare
from tools.gen_synth import records, write, write_bam

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ccsx_amd", "bin", "ccsx")


def _expected(path, mode, min_count=3, mn=5000, mx=500000, exclude=(), is_bam=False):
    """The oracle on the same records and filters as the CLI, with its own
    ccs_prepare (oracle/prep_oracle.c, independent of the CLI's host/prepare.cpp)."""
    keep = []
    for movie, hole, subs in cx.read_zmws(path, is_bam):
        if len(subs) < min_count + 2 or not (mn <= sum(map(len, subs)) <= mx) or hole in exclude:
            continue
        keep.append((movie, hole, oracle_prepare(subs)))
    ccs, _, _ = batch([p for _, _, p in keep], mode, 16)
    return b"".join(b">%s/%s/ccs\n%s\n" % (m.encode(), h.encode(), c) for (m, h, _), c in zip(keep, ccs) if c)


def _run(args, env=None, timeout=300):
    r = subprocess.run([BIN] + args, capture_output=True, timeout=timeout, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    return r


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


@pytest.mark.parametrize("async_", ["1", "0"])
def test_cli_multi_chunk_order(tmp_path, async_):
    """1,100 ZMWs in chunks of at most 1,024 (CCSX_CHUNK; the first is half
    of it), so later chunks are read and prepared while the GPU runs the
    first; pipelined submit / collect (CCSX_ASYNC=1, with three batches per
    chunk so batches of the next chunk are submitted before the previous are
    collected) and one ccsx_gpu_run per batch: the output stays in input order
    and equal to the oracle's."""
    fa = str(tmp_path / "in.fa")
    write(fa, 1100, 1000, 6)
    out = str(tmp_path / "out.fa")
    _run(["-A", "-j", "4", fa, out], env=dict(CCSX_CHUNK="1024", CCSX_ASYNC=async_, CCSX_CTX_BATCHES="3"))
    got = open(out, "rb").read()
    assert got.count(b">") == 1100
    assert got == _expected(fa, 0)


def test_cli_logical_contexts_match_one(tmp_path):
    """Chunks of at most 2,048 ZMWs split into cost-balanced micro-batches
    over N >= 2 device contexts (CCSX_NGPU groups beyond the visible GPUs are
    logical contexts on the same device), pipelined or one
    ccsx_gpu_run per batch: byte-identical to one context, in input order
    (main.c:701-704,707-717), and equal to the oracle."""
    fa = str(tmp_path / "in.fa")
    write(fa, 5300, 1000, 6)
    outs = []
    for ngpu, slots, async_ in (("1", "1", "1"), ("3", "2", "1"), ("2", "1", "0"), ("1", "2", "0")):
        out = str(tmp_path / f"out{ngpu}_{slots}_{async_}.fa")
        _run(["-A", "-j", "8", fa, out], env=dict(CCSX_NGPU=ngpu, CCSX_SLOTS=slots, CCSX_ASYNC=async_, CCSX_CHUNK="2048"))
        outs.append(open(out, "rb").read())
    assert outs[0].count(b">") == 5300
    assert all(o == outs[0] for o in outs[1:])
    assert outs[0] == _expected(fa, 0)


def test_cli_bam_input(tmp_path):
    """BAM is the reference's default input (main.c:754): a BGZF subread BAM
    gives the same CCS as the same records as FASTA with -A, and the oracle's."""
    bam, fa = str(tmp_path / "in.bam"), str(tmp_path / "in.fa")
    write_bam(bam, records(40, 1500, 7, hole0=100))
    write(fa, 40, 1500, 7, hole0=100)
    ob, of = str(tmp_path / "b.fa"), str(tmp_path / "f.fa")
    _run(["-j", "4", bam, ob])
    _run(["-A", "-j", "4", fa, of])
    got = open(ob, "rb").read()
    assert got.count(b">") == 40
    assert got == open(of, "rb").read()
    assert got == _expected(bam, 0, is_bam=True)


def test_cli_failed_zmw_is_skipped(tmp_path):
    """A ZMW the device reports as failed is skipped with a message; every
    other ZMW is still written, in input order, and the run exits 0."""
    fa = str(tmp_path / "in.fa")
    write(fa, 30, 1200, 6)
    out = str(tmp_path / "out.fa")
    r = _run(["-A", "-j", "4", fa, out], env=dict(CCSX_FAULT_HOLE="7", CCSX_NGPU="2", CCSX_SLOTS="1"))
    assert b"synth/7: no CCS" in r.stderr
    got = open(out, "rb").read()
    assert got.count(b">") == 29
    assert got == _expected(fa, 0, exclude={"7"})


def test_cli_verbose_segments(tmp_path):
    """-v dumps every oriented segment as main.c:477-479 does (strand= field)."""
    fa = str(tmp_path / "in.fa")
    write(fa, 2, 1200, 6)
    r = _run(["-A", "-v", fa, str(tmp_path / "o.fa")])
    err = r.stderr.decode()
    assert err.count(" strand=") == 12
    assert ">0_0/6 strand=0 len=" in err


@pytest.mark.parametrize("xargs,excluded", [(["-X", "3,5", "-X", "7"], {"3"}), (["-X", "3", "-X", "7"], {"37"}),
                                            (["-X", "1,,2,"], {"1", "2"})])
def test_cli_repeated_exclude(tmp_path, xargs, excluded):
    """-X as main.c:772-782 builds it: each option kputs-appends to one buffer
    that ksplit then splits as a C string in place, and a fresh hole set takes
    the fields, so only the last -X counts and it sees the first field of the
    earlier ones joined with its own text."""
    fa = str(tmp_path / "in.fa")
    write(fa, 40, 1000, 6)
    out = str(tmp_path / "out.fa")
    _run(["-A", "-j", "4"] + xargs + [fa, out])
    got = open(out, "rb").read()
    assert got == _expected(fa, 0, exclude=excluded)
    assert got.count(b">") == 40 - len(excluded)


def test_cli_breakpoint_lines(tmp_path):
    """-v -v -v prints ccs_for2's per-round breakpoint line to stdout
    (main.c:619-620: breakpoint, MSA columns, nseq, hole) for every shredding
    round, the final one included (breakpoint = columns); the values are the
    oracle's rounds for the same push lists, in input order."""
    from oracle.oracle import Poa
    fa = str(tmp_path / "in.fa")
    write(fa, 6, 7000, 6)
    out = str(tmp_path / "out.fa")
    r = _run(["-A", "-v", "-v", "-v", "-j", "2", fa, out])
    got = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("breakpoint=")]
    want = []
    for movie, hole, subs in cx.read_zmws(fa, False):
        p = oracle_prepare(subs)
        _, bps = Poa().zmw_breakpoints(p.seqs, p.offs, p.lens)
        want += [f"breakpoint={i} maplen={c} nseq={len(p.lens)} hole={hole}" for i, c in bps]
    assert len(want) > 12 and got == want
    assert open(out, "rb").read() == _expected(fa, 0)


@pytest.mark.parametrize("fatal", [False, True])
def test_cli_teardown_after_input_release(tmp_path, fatal):
    """A mapped input file larger than a few chunks is unmapped behind the
    reader (ZmwSource::release); the teardown that follows must unmap only
    what is still mapped (the block's destructor unmapped the whole
    original range, over whatever the kernel had placed in the released hole).
    CCSX_EXIT_CLOSE runs the full teardown after a good run; CCSX_FATAL_AFTER
    fails the third batch as a context error, so the fatal path's teardown
    (reader, contexts, written chunks) runs after releases too."""
    fa = str(tmp_path / "in.fa")
    write(fa, 3000, 1000, 6)
    out = str(tmp_path / "out.fa")
    env = dict(CCSX_CHUNK="1024", CCSX_CHUNK0="512", CCSX_SLOTS="1")
    if fatal:
        env["CCSX_FATAL_AFTER"] = "2"
        r = subprocess.run([BIN, "-A", "-j", "4", fa, out], capture_output=True, timeout=300,
                           env=dict(os.environ, **env))
        assert r.returncode == 1, r.stderr.decode()[-2000:]
        assert b"injected fatal error" in r.stderr
        # the fatal path's teardown faulted nowhere: no sanitizer / abort /
        # segfault signature after the injected error (the exit status alone
        # is 1 whether or not a later teardown step misbehaved)
        err = r.stderr.decode(errors="replace")
        for sig in ("Segmentation fault", "Aborted", "core dumped", "AddressSanitizer", "double free",
                    "free(): invalid", "munmap_chunk", "terminate called"):
            assert sig not in err, err[-2000:]
    else:
        env["CCSX_EXIT_CLOSE"] = "1"
        r = _run(["-A", "-j", "4", fa, out], env=env)
        assert b"teardown:" in r.stderr
        got = open(out, "rb").read()
        assert got.count(b">") == 3000
        assert got == _expected(fa, 0)
