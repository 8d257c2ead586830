"""The host program's step 0 + prepare path as the CLI runs it (span-based
records from host/ingest.cpp, bases assembled and prepared on worker
threads), checked against the C-ABI reader (itself pinned to the reference by
tests/golden/host) on synthetic FASTA, gzip FASTA, bgzip FASTA and BGZF BAM.
CPU only: tools/ingest_bench.cpp links the product library, no GPU."""
import gzip
import os
import subprocess
import zlib

import pytest

import ccsx_amd as cx
from tools.gen_synth import _bgzf_block, records, write, write_bam

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "build", "ingest_bench")


@pytest.fixture(scope="module")
def ingest_bench():
    src = os.path.join(ROOT, "tools", "ingest_bench.cpp")
    lib = os.path.join(ROOT, "ccsx_amd", "libccsx_amd.so")
    if not os.path.exists(BENCH) or os.path.getmtime(BENCH) < max(os.path.getmtime(src), os.path.getmtime(lib)):
        os.makedirs(os.path.dirname(BENCH), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I",
                        os.path.join(ROOT, "ccsx_amd", "csrc", "host"), src, "-L", os.path.join(ROOT, "ccsx_amd"),
                        "-lccsx_amd", "-lz", "-lpthread", "-Wl,-rpath," + os.path.join(ROOT, "ccsx_amd"), "-o",
                        BENCH + f".{os.getpid()}"], check=True)
        os.replace(BENCH + f".{os.getpid()}", BENCH)  # (atomic: pytest -n workers may build it together)
    return BENCH


def _expected(path, is_bam):
    out = []
    for movie, hole, subs in cx.read_zmws(path, is_bam):
        p = cx.prepare(subs)
        c = 0
        for o, n in zip(p.offs, p.lens):
            c = zlib.crc32(p.seqs[o:o + n], c)
        out.append(f"{movie}\t{hole}\t{','.join(str(len(s)) for s in subs)}\t{c:08x}")
    return out


def _bgzip(src, dst):
    raw = open(src, "rb").read()
    with open(dst, "wb") as f:
        for i in range(0, len(raw), 50000):
            f.write(_bgzf_block(raw[i:i + 50000]))
        f.write(_bgzf_block(b""))


@pytest.mark.parametrize("fmt", ["fa", "fa.gz", "bgzf.fa.gz", "bam"])
@pytest.mark.parametrize("threads,chunk", [(1, 1000), (4, 37)])
def test_cli_ingest_path_matches_reader(tmp_path, ingest_bench, fmt, threads, chunk):
    fa = str(tmp_path / "in.fa")
    write(fa, 60, 1500, 7)
    path, is_bam = fa, 0
    if fmt == "fa.gz":
        path = fa + ".gz"
        with open(fa, "rb") as s, gzip.open(path, "wb") as d:
            d.write(s.read())
    elif fmt == "bgzf.fa.gz":
        path = str(tmp_path / "in.bgzf.fa.gz")
        _bgzip(fa, path)
    elif fmt == "bam":
        path, is_bam = str(tmp_path / "in.bam"), 1
        write_bam(path, records(60, 1500, 7))
    got = subprocess.run([ingest_bench, path, str(is_bam), str(threads), str(chunk), "--dump"], check=True,
                         capture_output=True, text=True).stdout.splitlines()
    assert len(got) == 60
    assert got == _expected(path, bool(is_bam))


def test_ingest_bench_reports_throughput(tmp_path, ingest_bench):
    fa = str(tmp_path / "in.fa")
    write(fa, 40, 3000, 6)
    import json
    r = json.loads(subprocess.run([ingest_bench, fa, "0", "2", "16"], check=True, capture_output=True,
                                  text=True).stdout)
    assert r["zmws"] == 40 and r["bases"] > 40 * 6 * 3000


@pytest.mark.parametrize("fmt", ["fa", "fa.gz", "bgzf.fa.gz", "bam"])
@pytest.mark.parametrize("how", ["redirect", "pipe"])
def test_stdin_matches_reader(tmp_path, ingest_bench, fmt, how):
    """INPUT "-" (main.c:804-808): stdin redirected from a regular file takes
    the file's own path (mmap / parallel BGZF / gzread), a pipe the gzread
    stream; both give what the reader gives for the named file."""
    fa = str(tmp_path / "in.fa")
    write(fa, 40, 1200, 6)
    path, is_bam = fa, 0
    if fmt == "fa.gz":
        path = fa + ".gz"
        with open(fa, "rb") as s, gzip.open(path, "wb") as d:
            d.write(s.read())
    elif fmt == "bgzf.fa.gz":
        path = str(tmp_path / "in.bgzf.fa.gz")
        _bgzip(fa, path)
    elif fmt == "bam":
        path, is_bam = str(tmp_path / "in.bam"), 1
        write_bam(path, records(40, 1200, 6))
    cmd = [ingest_bench, "-", str(is_bam), "3", "16", "--dump"]
    if how == "redirect":
        with open(path, "rb") as f:
            got = subprocess.run(cmd, stdin=f, check=True, capture_output=True).stdout
    else:
        got = subprocess.run(cmd, input=open(path, "rb").read(), check=True, capture_output=True).stdout
    assert got.decode().splitlines() == _expected(path, bool(is_bam))
