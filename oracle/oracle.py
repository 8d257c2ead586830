"""ctypes bindings of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, as the checker.  The product (ccsx_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import sys
            sys.path.insert(0, os.path.dirname(_HERE))
            from ccsx_amd.build import build_oracle
            build_oracle()
        L = C.CDLL(LIB_PATH)
        L.opoa_init.argtypes = [C.c_int] * 5
        L.opoa_init.restype = C.c_void_p
        L.opoa_free.argtypes = [C.c_void_p]
        L.opoa_beg.argtypes = [C.c_void_p]
        L.opoa_push.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32]
        L.opoa_end.argtypes = [C.c_void_p]
        L.opoa_tidy_msa.argtypes = [C.c_void_p]
        L.opoa_cns.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.opoa_cns.restype = C.c_uint32
        L.opoa_msa.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_uint32)]
        L.opoa_msa.restype = C.c_uint32
        L.opoa_cells.argtypes = [C.c_void_p]
        L.opoa_cells.restype = C.c_uint64
        L.opoa_nrows.argtypes = [C.c_void_p]
        L.opoa_nrows.restype = C.c_uint32
        L.opoa_graph_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.ocsx_zmw.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                               C.c_uint32, C.c_char_p]
        L.ocsx_zmw.restype = C.c_size_t
        if True:
            L.ocsx_batch.argtypes = [C.c_int, C.c_int, C.c_uint32, C.POINTER(C.c_char_p),
                                     C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.POINTER(C.c_uint32)),
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                                     C.POINTER(C.c_uint64)]
        L.ocsx_zmw_log.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                   C.c_uint32, C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32)]
        L.ocsx_zmw_log.restype = C.c_size_t
        L.ocsx_edit_distance.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_uint32]
        L.ocsx_edit_distance.restype = C.c_int64
        L.oprep_prepare.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32),
                                    C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)]
        L.oprep_prepare.restype = C.c_uint32
        L.oprep_prepare_apply.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint32)]
        L.oprep_prepare_apply.restype = C.c_uint32
        L.oprep_pairwise.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32]
        L.oprep_pairwise.restype = OprepAln
        _lib = L
    return _lib


class OprepAln(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("qb", "qe", "tb", "te", "score", "mat", "mis", "ins", "del_", "aln")]


class Prepared:
    """One ZMW after the oracle's ccs_prepare + strand flip (the same fields as
    ccsx_amd.Prepared: segments are slices of seqs)."""

    def __init__(self, seqs: bytes, offs, lens):
        self.seqs, self.offs, self.lens = seqs, offs, lens


def _p32(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def prepare_segments(subreads: list[bytes]):
    """The oracle's ccs_prepare (main.c:344-453): (offs, lens, reverse flags)
    of the push list into the concatenated subreads, template first."""
    seqs = b"".join(subreads)
    lens = np.ascontiguousarray([len(s) for s in subreads], dtype=np.uint32)
    n = len(subreads)
    so = np.zeros(max(n, 1), np.uint32)
    sl = np.zeros(max(n, 1), np.uint32)
    rv = np.zeros(max(n, 1), np.uint8)
    ns = lib().oprep_prepare(seqs, _p32(lens), n, _p32(so), _p32(sl), rv.ctypes.data_as(C.POINTER(C.c_uint8)))
    return so[:ns].copy(), sl[:ns].copy(), rv[:ns].copy()


def prepare(subreads: list[bytes]) -> Prepared:
    """The oracle's ccs_prepare + in-place reverse complement of the reverse
    segments (seqio.h:138-148): what the POA is pushed."""
    seqs = b"".join(subreads)
    buf = C.create_string_buffer(seqs, len(seqs) + 1)
    lens = np.ascontiguousarray([len(s) for s in subreads], dtype=np.uint32)
    n = len(subreads)
    so = np.zeros(max(n, 1), np.uint32)
    sl = np.zeros(max(n, 1), np.uint32)
    ns = lib().oprep_prepare_apply(buf, _p32(lens), n, _p32(so), _p32(sl))
    return Prepared(buf.raw[:len(seqs)], so[:ns].copy(), sl[:ns].copy())


def pairwise(q: bytes, t: bytes) -> dict:
    """SPEC.md §8's aligner as the oracle restates it (2-bit codes in q, t)."""
    r = lib().oprep_pairwise(q, len(q), t, len(t))
    return {n if n != "del_" else "del": getattr(r, n) for n, _ in OprepAln._fields_}


def edit_identity(a: bytes, b: bytes, band: int = 1024) -> float:
    """1 - (banded) edit distance / max length: a lower bound of the identity
    (accuracy sanity check vs synthetic truth; not parity)."""
    if not a or not b:
        return 0.0
    d = lib().ocsx_edit_distance(a, len(a), b, len(b), band)
    return 0.0 if d < 0 else 1.0 - d / max(len(a), len(b))


class Poa:
    """The oracle's bspoa-like object (SPEC.md) with main.c's parameters."""

    def __init__(self, M=2, X=-6, O=-3, E=-2, W=128):
        self._L = lib()
        self._g = self._L.opoa_init(M, X, O, E, W)

    def __del__(self):
        try:
            self._L.opoa_free(self._g)
        except Exception:
            pass

    def poa(self, reads: list[bytes]):
        """beg + push* + end + tidy: returns (cns codes, msa [ncols, nseq+4] uint8)."""
        L = self._L
        L.opoa_beg(self._g)
        for r in reads:
            L.opoa_push(self._g, r, len(r))
        L.opoa_end(self._g)
        L.opoa_tidy_msa(self._g)
        p = C.c_void_p()
        n = L.opoa_cns(self._g, C.byref(p))
        cns = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (n,)).copy() if n else np.zeros(0, np.uint8)
        ip, cp, mrow = C.c_void_p(), C.c_void_p(), C.c_uint32()
        nc = L.opoa_msa(self._g, C.byref(ip), C.byref(cp), C.byref(mrow))
        if nc:
            msa = np.ctypeslib.as_array(C.cast(cp, C.POINTER(C.c_uint8)), (nc * mrow.value,)).copy()
            msa = msa.reshape(nc, mrow.value)
        else:
            msa = np.zeros((0, len(reads) + 4), np.uint8)
        return cns, msa

    def zmw(self, seqs: bytes, offs, lens, mode: int = 0) -> bytes:
        """ccs_for2 (mode 0) / ccs_for (mode 1) on strand-normalised segments."""
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = C.create_string_buffer(int(lens.sum()) + 16)
        n = self._L.ocsx_zmw(self._g, mode, seqs, offs.ctypes.data_as(C.POINTER(C.c_uint32)),
                             lens.ctypes.data_as(C.POINTER(C.c_uint32)), len(lens), out)
        return out.raw[:n]

    def zmw_breakpoints(self, seqs: bytes, offs, lens) -> tuple[bytes, list[tuple[int, int]]]:
        """ccs_for2 plus, per shredding round, (breakpoint, MSA columns): the
        values main.c:619-620 prints at -v >= 3."""
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = C.create_string_buffer(int(lens.sum()) + 16)
        cap = int(lens.sum()) + 2
        log = (C.c_uint32 * (2 * cap))()
        nbp = C.c_uint32(0)
        n = self._L.ocsx_zmw_log(self._g, 0, seqs, offs.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 lens.ctypes.data_as(C.POINTER(C.c_uint32)), len(lens), out, log, cap, C.byref(nbp))
        return out.raw[:n], [(log[2 * i], log[2 * i + 1]) for i in range(nbp.value)]

    def cells(self) -> int:
        return int(self._L.opoa_cells(self._g))

    def nrows(self) -> int:
        return int(self._L.opoa_nrows(self._g))

    def max_indegree(self) -> int:
        """Largest predecessor count of the current graph (after poa())."""
        h = (C.c_uint64 * 8)()
        self._L.opoa_graph_stats(self._g, h)
        return int(h[2])


def batch(zmws, mode: int = 0, nthreads: int = 1):
    """Run ocsx_zmw over prepared ZMWs on nthreads pthreads.

    zmws: objects with .seqs (bytes), .offs, .lens.  Returns (list of CCS bytes,
    list of cells, wall seconds)."""
    import time
    L = lib()
    n = len(zmws)
    keep = []
    seqs = (C.c_char_p * n)()
    offs = (C.POINTER(C.c_uint32) * n)()
    lens = (C.POINTER(C.c_uint32) * n)()
    nseg = (C.c_uint32 * n)()
    outs = (C.c_char_p * n)()
    bufs = []
    for i, z in enumerate(zmws):
        o = np.ascontiguousarray(z.offs, dtype=np.uint32)
        ln = np.ascontiguousarray(z.lens, dtype=np.uint32)
        keep += [o, ln, z.seqs]
        seqs[i] = z.seqs
        offs[i] = o.ctypes.data_as(C.POINTER(C.c_uint32))
        lens[i] = ln.ctypes.data_as(C.POINTER(C.c_uint32))
        nseg[i] = len(ln)
        b = C.create_string_buffer(int(ln.sum()) + 16)
        bufs.append(b)
        outs[i] = C.cast(b, C.c_char_p)
    olen = (C.c_size_t * n)()
    cells = (C.c_uint64 * n)()
    t = time.perf_counter()
    L.ocsx_batch(mode, nthreads, n, seqs, offs, lens, nseg, outs, olen, cells)
    dt = time.perf_counter() - t
    return [bufs[i].raw[:olen[i]] for i in range(n)], [int(cells[i]) for i in range(n)], dt
