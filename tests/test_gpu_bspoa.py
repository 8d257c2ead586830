"""The bspoa-compatible API (include/ccsx_bspoa.h) on the GPU vs the oracle's
bspoa restatement: consensus codes (g->cns) and the tidy MSA
(g->msaidxs / g->msacols, main.c:575-623) must be byte-identical."""
import ctypes as C

import numpy as np
import pytest

import ccsx_amd as cx
from oracle.oracle import Poa
from tests.zmw_cases import edge_cases, synth

pytestmark = pytest.mark.gpu


class BSPOAPar(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("refmode", "shuffle", "realn", "M", "X", "O", "E", "Q", "P", "editbw",
                                       "bandwidth")]


class U1V(C.Structure):
    _fields_ = [("buffer", C.POINTER(C.c_uint8)), ("size", C.c_uint64), ("cap", C.c_uint64)]


class U4V(C.Structure):
    _fields_ = [("buffer", C.POINTER(C.c_uint32)), ("size", C.c_uint64), ("cap", C.c_uint64)]


class BSPOA(C.Structure):
    _fields_ = [("par", BSPOAPar), ("cns", C.POINTER(U1V)), ("msaidxs", C.POINTER(U4V)),
                ("msacols", C.POINTER(U1V)), ("nseq", C.c_uint32), ("impl", C.c_void_p)]


@pytest.fixture(scope="module")
def bspoa():
    L = cx.lib()
    L.init_bspoa.argtypes = [BSPOAPar]
    L.init_bspoa.restype = C.POINTER(BSPOA)
    for f in ("beg_bspoa", "end_bspoa", "tidy_msa_bspoa", "free_bspoa"):
        getattr(L, f).argtypes = [C.POINTER(BSPOA)]
    L.push_bspoa.argtypes = [C.POINTER(BSPOA), C.c_char_p, C.c_uint32]
    par = BSPOAPar(0, 0, 0, 2, -6, -3, -2, 0, 0, 32, 128)  # main.c:841-849
    g = L.init_bspoa(par)
    yield L, g
    L.free_bspoa(g)


def _run(L, g, reads):
    L.beg_bspoa(g)
    for r in reads:
        L.push_bspoa(g, r, len(r))
    L.end_bspoa(g)
    L.tidy_msa_bspoa(g)
    s = g.contents
    cns = np.ctypeslib.as_array(s.cns.contents.buffer, (s.cns.contents.size,)).copy() if s.cns.contents.size else \
        np.zeros(0, np.uint8)
    nc = s.msaidxs.contents.size
    mrow = len(reads) + 4
    idx = np.ctypeslib.as_array(s.msaidxs.contents.buffer, (nc,)).copy() if nc else np.zeros(0, np.uint32)
    cols = np.ctypeslib.as_array(s.msacols.contents.buffer, (nc * mrow,)).copy() if nc else np.zeros(0, np.uint8)
    msa = cols.reshape(-1, mrow)[idx] if nc else np.zeros((0, mrow), np.uint8)
    return cns, msa


def _reads(p):
    return [p.seqs[o:o + n] for o, n in zip(p.offs, p.lens)]


@pytest.mark.parametrize("hole,L,passes", [(1, 2000, 8), (2, 2500, 12), (3, 1800, 5)])
def test_bspoa_synthetic(bspoa, hole, L, passes):
    lib, g = bspoa
    reads = _reads(synth(hole, L, passes))
    cns, msa = _run(lib, g, reads)
    wcns, wmsa = Poa().poa(reads)
    assert np.array_equal(cns, wcns)
    assert np.array_equal(msa, wmsa)


def test_bspoa_edge_cases(bspoa):
    lib, g = bspoa
    for name, p in edge_cases().items():
        reads = _reads(p)
        if sum(len(r) for r in reads) > 40000:
            continue
        cns, msa = _run(lib, g, reads)
        wcns, wmsa = Poa().poa(reads)
        assert np.array_equal(cns, wcns), name
        assert np.array_equal(msa, wmsa), name
