"""Host-side code of the C host program (CPU): ccs_prepare, strand flip,
pairwise aligner, subread ingest/grouping, synthetic source."""
import gzip
import os

import numpy as np

import ccsx_amd as cx

# seqio.h:120-137 complement table, restated independently
_COMP = {ord(a): ord(b) for a, b in zip("ABCDGHKMNRSTUVWYabcdghkmnrstuvwy", "TVGHCDMKNYSAABWRtvghcdmknysaabwr")}


def _rc(s: bytes) -> bytes:
    return bytes(_COMP.get(c, c) for c in reversed(s))


def test_revcomp_table():
    s = bytes(range(256))
    assert cx.revcomp(s) == _rc(s)
    assert cx.revcomp(b"ACGTNacgtnRYKM") == _rc(b"ACGTNacgtnRYKM")
    assert cx.revcomp(b"") == b""
    assert cx.revcomp(b"A") == b"T"


def test_synth_shape():
    subs, ins = cx.synth_zmw(20201104, 3, 5000, 7)
    assert len(subs) == 7 and len(ins) == 5000
    for s in subs:
        assert 4700 < len(s) < 5400 and set(s) <= set(b"ACGT")
    assert cx.synth_zmw(20201104, 3, 5000, 7) == (subs, ins)
    assert cx.synth_zmw(20201104, 4, 5000, 7)[1] != ins


def test_prepare_full_passes():
    """All subreads in one length group: template = middle subread, push order
    template, t-1..0, t+1..n-1, strands alternate (main.c:372-446)."""
    subs, _ = cx.synth_zmw(20201104, 9, 4000, 8)
    offs, lens, rev = cx.prepare_segments(subs)
    n = len(subs)
    t = n // 2
    order = [t] + list(range(t - 1, -1, -1)) + list(range(t + 1, n))
    cum = np.cumsum([0] + [len(s) for s in subs])
    assert list(offs) == [cum[i] for i in order]
    assert list(lens) == [len(subs[i]) for i in order]
    assert list(rev) == [abs(i - t) % 2 for i in order]


def test_prepare_apply_flips_reverse_segments():
    subs, _ = cx.synth_zmw(20201104, 10, 3000, 6)
    offs, lens, rev = cx.prepare_segments(subs)
    p = cx.prepare(subs)
    raw = b"".join(subs)
    for o, n, r in zip(offs, lens, rev):
        seg = raw[o:o + n]
        assert p.seqs[o:o + n] == (_rc(seg) if r else seg)


def test_prepare_abnormal_subread_is_realigned():
    """A half-length subread is outside the template group: strand_match decides
    its strand and trims it (main.c:379-406); a too-short one is dropped."""
    subs, ins = cx.synth_zmw(20201104, 11, 4000, 7)
    subs = list(subs)
    subs[5] = subs[5][:1500]
    offs, lens, rev = cx.prepare_segments(subs)
    assert len(lens) == 6  # the short abnormal subread (< template length) is skipped


def test_pairwise_identity_and_trim():
    rng = np.random.default_rng(1)
    t = rng.integers(0, 4, 3000).astype(np.uint8)
    q = np.concatenate([rng.integers(0, 4, 200).astype(np.uint8), t[500:2500]])
    r = cx.pairwise(q.tobytes(), t.tobytes())
    assert r["mat"] >= 1990 and r["qb"] == 200 and r["tb"] == 500
    assert r["qe"] == 2200 and r["te"] == 2500
    none = cx.pairwise(rng.integers(0, 4, 2000).astype(np.uint8).tobytes(), t.tobytes())
    assert none["aln"] * 2 <= 2000 or none["mat"] * 100 < none["aln"] * 75


def _write(path, text, gz=False):
    data = text.encode()
    if gz:
        with gzip.open(path, "wb") as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)


def test_reader_groups_by_hole(tmp_path):
    fa = ">m1/10/0_5 extra\nACGTA\n>m1/10/5_9\nACG\nT\n>m1/11/0_4\nTTTT\n>m2/11/0_3\nGGG\n"
    p = tmp_path / "a.fa"
    _write(p, fa)
    z = list(cx.read_zmws(str(p)))
    assert z == [("m1", "10", [b"ACGTA", b"ACGT"]), ("m1", "11", [b"TTTT"]), ("m2", "11", [b"GGG"])]


def test_reader_fastq_gz_crlf(tmp_path):
    fq = "@m/1/0_4\r\nACGT\r\n+\r\nIIII\r\n@m/1/4_8\r\nTTGG\r\n+\r\nIIII\r\n@m/2/0_2\r\nAA\r\n+\r\nII\r\n"
    p = tmp_path / "a.fq.gz"
    _write(p, fq, gz=True)
    z = list(cx.read_zmws(str(p)))
    assert z == [("m", "1", [b"ACGT", b"TTGG"]), ("m", "2", [b"AA"])]


def test_reader_invalid_name_ends_call(tmp_path):
    """seqio.h:168-172: an invalid name returns -1; main.c's next chunk reads on
    from the pending record (main.c:658-697)."""
    fa = ">m/1/0_2\nAC\n>m/2/0_2\nGG\n>bad_name\nTT\n>m/3/0_2\nCC\n"
    p = tmp_path / "b.fa"
    _write(p, fa)
    calls = [(n, h, s) for n, _, h, s in cx.read_calls(str(p))]
    assert calls == [(1, "1", [b"AC"]), (-1, None, None), (1, "2", [b"GG"]), (1, "3", [b"CC"]), (-1, None, None),
                     (-1, None, None)]


def test_reader_bam(tmp_path):
    import struct
    nt = "=ACMGRSVTWYHKDBN"

    def rec(name, seq):
        qn = name.encode() + b"\0"
        l = len(seq)
        packed = bytearray((l + 1) // 2)
        for i, c in enumerate(seq):
            packed[i // 2] |= nt.index(c) << (4 * (1 - i % 2))
        core = struct.pack("<iiBBHHHiiii", -1, -1, len(qn), 255, 4680, 0, 4, l, -1, -1, 0)
        body = core + qn + bytes(packed) + bytes([255] * l)
        return struct.pack("<i", len(body)) + body

    hdr = b"BAM\1" + struct.pack("<i", 0) + struct.pack("<i", 0)
    data = hdr + rec("mv/7/0_5", "ACGTN") + rec("mv/7/5_8", "GGA") + rec("mv/8/0_2", "TT")
    p = tmp_path / "c.bam"
    with gzip.open(p, "wb") as f:
        f.write(data)
    z = list(cx.read_zmws(str(p), is_bam=True))
    assert z == [("mv", "7", [b"ACGTN", b"GGA"]), ("mv", "8", [b"TT"])]
