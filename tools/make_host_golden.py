"""Generate host-ingest golden fixtures (tests/golden/host/).

Writes small FASTA / FASTQ / gzip / BAM inputs covering the grouping rules
and quirks of kseq_zmw_read (seqio.h:152-201) and the BAM decoding of
kseq_extend_read (seqio.h:92-118, bamlite.c:78-165), then runs the
reference's own ingest code, compiled by oracle/ref_build.py into
oracle/_ref/ref_seqio, and stores its output as expected.json.

The driver loop mirrors main.c step 0 (main.c:658-697): after a -1 the next
chunk reads on, and input ends at the first chunk that yields no ZMW.

    python tools/make_host_golden.py      # needs /root/reference (this container)
"""
import gzip
import json
import os
import struct
import subprocess
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "host")

NT16 = "=ACMGRSVTWYHKDBN"


def fasta(recs, width=0):
    s = []
    for name, seq in recs:
        s.append(f">{name}\n")
        if width and len(seq) > width:
            for i in range(0, len(seq), width):
                s.append(seq[i:i + width] + "\n")
        else:
            s.append(seq + "\n")
    return "".join(s).encode()


def fastq(recs):
    return "".join(f"@{n}\n{s}\n+\n{'I' * len(s)}\n" for n, s in recs).encode()


def bgzf(raw, block=20000):
    """BGZF (SAM spec 4.1): deflate members of `block` bytes with the BC extra
    field, then the empty end-of-file member; records span members."""
    out = bytearray()
    for i in range(0, len(raw) + 1, block):
        d = raw[i:i + block]
        if not d and i:
            break
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        cd = co.compress(d) + co.flush()
        out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, 18 + len(cd) + 8 - 1)
        out += cd + struct.pack("<II", zlib.crc32(d) & 0xFFFFFFFF, len(d))
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    cd = co.compress(b"") + co.flush()
    out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, 18 + len(cd) + 8 - 1)
    out += cd + struct.pack("<II", 0, 0)
    return bytes(out)


def bam(recs):
    """Unaligned BAM (gzip-compressed; bamlite reads it through gzread)."""
    return gzip.compress(bam_raw(recs), mtime=0)


def bam_raw(recs):
    """The uncompressed BAM stream of (name, seq) records."""
    text = b"@HD\tVN:1.5\tSO:unknown\n"
    body = b"BAM\x01" + struct.pack("<i", len(text)) + text + struct.pack("<i", 0)
    for name, seq in recs:
        rn = name.encode() + b"\0"
        l = len(seq)
        codes = [NT16.index(c) if c in NT16 else 15 for c in seq.upper()]
        packed = bytes((codes[i] << 4) | (codes[i + 1] if i + 1 < l else 0) for i in range(0, l, 2))
        qual = bytes((i * 7) % 94 for i in range(l))
        core = struct.pack("<iiIIiiii", -1, -1, (4680 << 16) | (255 << 8) | len(rn), (4 << 16) | 0, l, -1, -1, 0)
        rec = core + rn + packed + qual
        body += struct.pack("<i", len(rec)) + rec
    return body


def zmw(movie, hole, n, L, salt=0):
    import random
    rnd = random.Random(zlib.crc32(f"{movie}/{hole}/{salt}".encode()))
    recs, pos = [], 0
    for i in range(n):
        ln = L + rnd.randint(-L // 4, L // 4)
        recs.append((f"{movie}/{hole}/{pos}_{pos + ln}", "".join(rnd.choice("ACGT") for _ in range(ln))))
        pos += ln + 40
    return recs


def cases():
    c = {}
    base = zmw("m64011_190830_220126", 7, 4, 60) + zmw("m64011_190830_220126", 9, 3, 50) + \
        zmw("m64011_190830_220126", 12, 5, 40)
    c["basic.fa"] = (0, fasta(base))
    c["multiline.fa"] = (0, fasta(base, width=17))
    c["basic.fq"] = (0, fastq(base))
    c["basic.fa.gz"] = (0, gzip.compress(fasta(base), mtime=0))
    iupac = [(n, s[:10] + "acgtNnRYKMSWBDHVU" + s[10:]) for n, s in zmw("mv", 3, 3, 30)]
    c["iupac_lower.fa"] = (0, fasta(iupac))
    # an invalid name in the middle of a ZMW (the reference keeps only the
    # ZMW's first record and reads on in the next chunk)
    bad = zmw("mv", 1, 3, 30) + zmw("mv", 2, 2, 30) + [("not_a_zmw_name", "ACGTACGT")] + \
        zmw("mv", 2, 3, 30, salt=1) + zmw("mv", 4, 3, 30)
    c["invalid_name.fa"] = (0, fasta(bad))
    c["invalid_first.fa"] = (0, fasta([("x/y", "ACGT")] + zmw("mv", 5, 3, 20)))
    c["four_fields.fa"] = (0, fasta(zmw("mv", 6, 3, 20) + [("mv/6/1_2/extra", "ACG")] + zmw("mv", 8, 3, 20)))
    # same hole number, different movie; and comments after the name
    mv = zmw("movieA", 5, 3, 25) + zmw("movieB", 5, 3, 25)
    c["movie_change.fa"] = (0, fasta(mv))
    com = [(n + " np=3 rq=0.9", s) for n, s in zmw("mv", 10, 3, 25)]
    c["comments.fa"] = (0, fasta(com))
    # empty records and a missing final newline
    emp = zmw("mv", 11, 2, 20) + [("mv/11/999_999", "")] + zmw("mv", 11, 2, 20, salt=2)
    c["empty_record.fa"] = (0, fasta(emp)[:-1])
    c["empty_fields.fa"] = (0, fasta([("mv//1_2", "ACGT"), ("/mv/1/2", "ACGT")] + zmw("mv", 12, 3, 20)))
    # line-ending and blank-line quirks of kseq.h:178-218: CRLF (one '\r'
    # stripped per appended line), blank lines inside and between records,
    # a tab-terminated name, a lone '\r' line
    crlf = fasta(base[:6], width=13).replace(b"\n", b"\r\n")
    c["crlf.fa"] = (0, crlf)
    c["crlf.fq"] = (0, fastq(base[:6]).replace(b"\n", b"\r\n"))
    blank = b"".join(b">%s\tx=1\n\n%s\n\n%s\n\n" % (n.encode(), s[:7].encode(), s[7:].encode())
                     for n, s in zmw("mv", 13, 4, 30))
    c["blank_lines.fa"] = (0, b"junk before the first header\n" + blank + b">mv/14/0_3\nAC\r\n\r\nGT\n>mv/14/3_6\nACG\n")
    # FASTQ quirks: quality lines starting with '@' / '>' and wrapped over
    # several lines; a record with an empty sequence (kseq still reads one
    # quality line: -2) after which reading goes on
    fq = zmw("mvq", 15, 4, 30)
    body = b"".join(b"@%s\n%s\n+\n%s\n%s\n" % (n.encode(), s.encode(), (b"@" + b">" * (len(s) // 2 - 1)),
                                                  b"I" * (len(s) - len(s) // 2)) for n, s in fq)
    c["fq_quirks.fq"] = (0, body + b"@mvq/16/0_0\n+\nIII\n" + fastq(zmw("mvq", 17, 3, 25)))
    # the input's last byte is a '\r' that starts a line: kseq's ks_getuntil2
    # returns before its '\r' strip, so the '\r' stays a base; a last line of
    # two or more chars without a newline is stripped as usual
    c["cr_last_line.fa"] = (0, fasta(zmw("mv", 18, 3, 20)) + b"\r")
    c["cr_last_line2.fa"] = (0, fasta(zmw("mv", 19, 3, 20))[:-1] + b"\r")
    c["basic.bam"] = (1, bam(base))
    c["bgzf.bam"] = (1, bgzf(bam_raw(base + zmw("mvb", 21, 6, 3000))))
    c["bgzf.fa.gz"] = (0, bgzf(fasta(base + zmw("mvb", 22, 5, 4000), width=61)))
    c["iupac.bam"] = (1, bam([(n, s[:5] + "NRYKM=" + s[5:]) for n, s in zmw("mvb", 3, 3, 31)]))
    c["invalid_name.bam"] = (1, bam(bad))
    return c


def run_ref(exe, isbam, path):
    out = subprocess.run([exe, str(isbam), path], check=True, capture_output=True).stdout.decode()
    return parse(out)


def parse(out):
    res = []
    for line in out.split("\n"):  # (not splitlines: a base may be '\r')
        if not line:
            continue
        f = line.split("\t")
        if len(f) == 1:
            res.append({"ret": int(f[0])})
        else:
            res.append({"ret": int(f[0]), "movie": f[1], "hole": f[2], "lens": [int(x) for x in f[3].split(",")],
                        "seqs": f[4], "rc": f[5]})
    return res


def main():
    from oracle.ref_build import build_ref
    exe = build_ref()
    if exe is None:
        raise SystemExit("needs the reference sources (/root/reference)")
    os.makedirs(OUT, exist_ok=True)
    expected = {}
    for name, (isbam, data) in sorted(cases().items()):
        p = os.path.join(OUT, name)
        with open(p, "wb") as f:
            f.write(data)
        expected[name] = {"is_bam": isbam, "calls": run_ref(exe, isbam, p)}
    with open(os.path.join(OUT, "expected.json"), "w") as f:
        json.dump(expected, f, indent=0, sort_keys=True)
    print(f"{len(expected)} fixtures -> {OUT}")


if __name__ == "__main__":
    main()
