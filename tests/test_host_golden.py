"""Subread ingest vs the reference's own seqio.h / kseq.h / bamlite.c.

tests/golden/host/expected.json holds what the reference code (compiled by
oracle/ref_build.py from /root/reference, driven by
oracle/ref_seqio_driver.c; generator tools/make_host_golden.py) returns on
the fixture inputs next to it.  The product reader (ccsx_amd/csrc/host/
seqio.cpp) and strand flip (ccsx_revcomp) must reproduce every call.
"""
import json
import os
import subprocess

import pytest

import ccsx_amd as cx

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "host")
ROOT = os.path.dirname(HERE)
with open(os.path.join(GOLD, "expected.json")) as f:
    EXPECTED = json.load(f)


def _product_calls(name, is_bam):
    out = []
    for n, movie, hole, subs in cx.read_calls(os.path.join(GOLD, name), bool(is_bam)):
        if n < 0:
            out.append({"ret": n})
        else:
            out.append({"ret": n, "movie": movie, "hole": hole, "lens": [len(s) for s in subs],
                        "seqs": b"".join(subs).decode("latin-1"),
                        "rc": b"".join(cx.revcomp(s) for s in subs).decode("latin-1")})
    return out


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_ingest_matches_reference(name):
    e = EXPECTED[name]
    assert _product_calls(name, e["is_bam"]) == e["calls"]


@pytest.mark.parametrize("block", [1, 7, 64, 4096])
def test_ingest_across_block_boundaries(monkeypatch, block):
    """The block-based parser (host/ingest.cpp) with blocks of a few bytes, so
    every record, name, line ending and BAM record crosses blocks (the tail is
    carried into the next block's headroom or, when larger, copied)."""
    monkeypatch.setenv("CCSX_INGEST_BLOCK", str(block))
    for name, e in sorted(EXPECTED.items()):
        assert _product_calls(name, e["is_bam"]) == e["calls"], name


def test_fixtures_cover_quirks():
    rets = {k: [c["ret"] for c in v["calls"]] for k, v in EXPECTED.items()}
    assert rets["invalid_name.fa"].count(-1) >= 2          # resumed after an invalid name
    assert rets["four_fields.fa"] == [-1]                   # ZMW before an invalid name is lost
    assert any(c.get("lens", [1]).count(0) for c in EXPECTED["empty_record.fa"]["calls"])


def test_reference_build_reproduces_fixtures():
    """When the reference sources are present (this container), rebuild the
    reference ingest and check the committed fixtures are still its output."""
    from oracle.ref_build import build_ref
    exe = build_ref()
    if exe is None:
        pytest.skip("reference sources not present (GPU box)")
    from tools.make_host_golden import parse
    for name, e in EXPECTED.items():
        out = subprocess.run([exe, str(e["is_bam"]), os.path.join(GOLD, name)], check=True,
                             capture_output=True).stdout.decode("latin-1")
        assert parse(out) == e["calls"], name
