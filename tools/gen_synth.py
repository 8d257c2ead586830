"""Write a synthetic subread FASTA: `synth/<hole>/<qs>_<qe>` names,
single-line uppercase records.  Usage: gen_synth.py OUT.fa NZMW L PASSES [HOLE0]
(L = 0: per-hole insert length and passes of bench.py's config E)."""
import os
import struct
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccsx_amd as cx  # noqa: E402


def records(nzmw, L, passes, hole0=0, seed=20201104, movie="synth", holes=None):
    """(name, subread) pairs of the synthetic set, in file order (`holes`: an
    explicit hole list instead of hole0 .. hole0 + nzmw - 1)."""
    for h in (range(hole0, hole0 + nzmw) if holes is None else holes):
        if L:
            subs, _ = cx.synth_zmw(seed, h, L, passes)
        else:
            from bench import CONFIGS, zmw_shape
            subs, _ = cx.synth_zmw(seed, h, *zmw_shape(CONFIGS["E"], h))
        qs = 0
        for s in subs:
            yield b"%s/%d/%d_%d" % (movie.encode(), h, qs, qs + len(s)), s
            qs += len(s)


def write(path, nzmw, L, passes, hole0=0, seed=20201104, movie="synth", holes=None):
    with open(path, "wb") as f:
        for name, s in records(nzmw, L, passes, hole0, seed, movie, holes):
            f.write(b">%s\n%s\n" % (name, s))


_NT16 = {c: i for i, c in enumerate(b"=ACMGRSVTWYHKDBN")}


def _bgzf_block(data: bytes) -> bytes:
    """One BGZF block (RFC 1952 member with the BC extra subfield, SAM spec 4.1)."""
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    cdata = c.compress(data) + c.flush()
    bsize = 18 + len(cdata) + 8 - 1
    head = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    return head + cdata + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def write_bam(path, recs):
    """Unaligned BAM of (name, seq) records: BGZF blocks of <= 64 KiB, the
    layout PacBio subread BAMs have (read by bamlite.c:78-165 via gzread)."""
    text = b"@HD\tVN:1.5\tSO:unknown\n"
    raw = bytearray(b"BAM\x01" + struct.pack("<i", len(text)) + text + struct.pack("<i", 0))
    out = bytearray()

    def flush(final=False):
        nonlocal raw
        while len(raw) >= 0xFF00 or (final and raw):
            out.extend(_bgzf_block(bytes(raw[:0xFF00])))
            del raw[:0xFF00]

    for name, seq in recs:
        rn = name + b"\0"
        n = len(seq)
        codes = [_NT16.get(c, 15) for c in seq.upper()]
        if n & 1:
            codes.append(0)
        packed = bytes((codes[i] << 4) | codes[i + 1] for i in range(0, len(codes), 2))
        qual = bytes([20]) * n
        core = struct.pack("<iiIIiiii", -1, -1, (4680 << 16) | (255 << 8) | len(rn), 4 << 16, n, -1, -1, 0)
        rec = core + rn + packed + qual
        raw += struct.pack("<i", len(rec)) + rec
        flush()
    flush(final=True)
    out.extend(_bgzf_block(b""))  # BGZF end-of-file marker
    with open(path, "wb") as f:
        f.write(out)


if __name__ == "__main__":
    a = sys.argv
    write(a[1], int(a[2]), int(a[3]), int(a[4]), int(a[5]) if len(a) > 5 else 0)
