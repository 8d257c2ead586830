"""The host C++ (ingest, ccs_prepare, pairwise aligner, synthetic source,
dispatch partitioner) under AddressSanitizer + UndefinedBehaviorSanitizer on
the CPU build: tools/host_sanitize.cpp drives the golden ingest fixtures (at
block sizes down to 1 byte) and abnormal synthetic ZMWs; the sanitized
reader must agree with the product library's."""
import glob
import os
import subprocess

import pytest

import ccsx_amd as cx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "host")
EXE = os.path.join(ROOT, "build", "host_sanitize")
SRCS = ["tools/host_sanitize.cpp"] + [f"ccsx_amd/csrc/host/{f}.cpp" for f in
                                       ("ingest", "seqio", "prepare", "pairwise", "dispatch")]


@pytest.fixture(scope="module")
def sanitized():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    srcs = [os.path.join(ROOT, s) for s in SRCS]
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(s) for s in srcs):
        subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", "-I", os.path.join(ROOT, "include"), "-I",
                        os.path.join(ROOT, "ccsx_amd", "csrc", "host"), "-o", EXE] + srcs + ["-lz", "-lpthread"],
                       check=True)
    return EXE


def _corrupt_bgzf(tmp_path):
    """BGZF members whose headers lie: BSIZE below header + trailer, a BC
    subfield running past XLEN, an ISIZE of 4 GB.  The reader must stop with
    its 'truncated or corrupt' message, reading nothing out of bounds."""
    import struct
    import zlib
    sys_path = str(tmp_path)
    out = []

    def member(d, bsize=None, isize=None, sublen=2):
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        cd = co.compress(d) + co.flush()
        bs = 18 + len(cd) + 8 - 1 if bsize is None else bsize
        head = struct.pack("<BBBBIBBHBBH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, sublen) + struct.pack("<H", bs)
        return head + cd + struct.pack("<II", zlib.crc32(d) & 0xFFFFFFFF, len(d) if isize is None else isize)

    good = member(b">mv/1/0_4\nACGT\n")
    for name, bad in (("bsize", member(b">mv/2/0_4\nACGT\n", bsize=10)),
                      ("sublen", member(b">mv/2/0_4\nACGT\n", sublen=40)),
                      ("isize", member(b">mv/2/0_4\nACGT\n", isize=0xFFFFFFF0))):
        p = os.path.join(sys_path, f"corrupt_{name}.fa.gz")
        with open(p, "wb") as f:
            f.write(good + bad + good)
        out.append(f"{p}:0")
    return out


def test_host_code_clean_under_asan_ubsan(sanitized, tmp_path):
    import json
    exp = json.load(open(os.path.join(GOLD, "expected.json")))
    args = [f"{os.path.join(GOLD, n)}:{e['is_bam']}" for n, e in sorted(exp.items())]
    args += _corrupt_bgzf(tmp_path)
    # (verify_asan_link_order=0: the run's environment may preload a library
    # ahead of the ASan runtime)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([sanitized] + args, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.stdout.rstrip().endswith("ok")
    # the sanitized reader reads what the product library reads
    import zlib
    want = []
    for n, e in sorted(exp.items()):
        p = os.path.join(GOLD, n)
        for k, movie, hole, subs in cx.read_calls(p, bool(e["is_bam"])):
            if k < 0:
                want.append(f"{p} -1")
            else:
                s = b"".join(subs)
                want.append(f"{p} {movie}/{hole} {k} {len(s)} {zlib.crc32(s):08x}")
    got = [x for x in r.stdout.splitlines() if x.startswith(GOLD)]
    assert got[:len(want)] == want
