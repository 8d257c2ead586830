"""ctypes bindings of libccsx_amd.so (include/ccsx_gpu.h, ccsx_host.h, ccsx_seqio.h).

The GPU engine has no CPU fallback: if the library is missing, or no GPU is
present, every call that needs it raises.  Host-side helpers (ccs_prepare,
reverse complement, the synthetic ZMW source, the subread reader) run on the
CPU and work without a GPU.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, os.environ.get("CCSX_LIB", "libccsx_amd.so"))

MODE_SHRED = 0
MODE_PRIMITIVE = 1

# every symbol the public headers declare (checked by tests/test_abi.py)
EXPORTS = {
    "ccsx_gpu.h": ["ccsx_gpu_device_count", "ccsx_gpu_open", "ccsx_gpu_close", "ccsx_gpu_error", "ccsx_gpu_status_str", "ccsx_gpu_run",
                   "ccsx_gpu_stage", "ccsx_gpu_launch", "ccsx_gpu_fetch", "ccsx_gpu_staged_bytes",
                   "ccsx_gpu_set_profiling", "ccsx_gpu_profile", "ccsx_gpu_profile_zmw", "ccsx_gpu_set_tight_rows", "ccsx_gpu_set_tight_out", "ccsx_gpu_set_tight_far", "ccsx_gpu_set_stage_piece",
                   "ccsx_gpu_set_mem_share", "ccsx_gpu_set_prealloc", "ccsx_gpu_set_fault",
                   "ccsx_gpu_set_kernel_cfg", "ccsx_gpu_kernel_cfg", "ccsx_gpu_rerun_count",
                   "ccsx_gpu_set_bp_log", "ccsx_gpu_bp_log", "ccsx_gpu_stage_for",
                   "ccsx_gpu_run_stats", "ccsx_gpu_zmw_bytes", "ccsx_gpu_set_slot_budget", "ccsx_gpu_set_wg_cap",
                   "ccsx_gpu_set_shred_read_cap", "ccsx_gpu_set_mem_frac", "ccsx_gpu_set_mem_wait",
                   "ccsx_gpu_slot_bytes", "ccsx_gpu_submit", "ccsx_gpu_collect", "ccsx_gpu_reserve_staging"],
    "ccsx_bspoa.h": ["init_bspoa", "beg_bspoa", "push_bspoa", "end_bspoa", "tidy_msa_bspoa", "free_bspoa"],
    "ccsx_host.h": ["ccsx_revcomp", "ccsx_prepare", "ccsx_prepare_apply", "ccsx_pairwise", "ccsx_synth_zmw",
                    "ccsx_zmw_cost", "ccsx_partition",
                    "ccsx_synth_batch_make", "ccsx_synth_batch_zmws", "ccsx_synth_batch_free"],
    "ccsx_seqio.h": ["ccsx_reader_open", "ccsx_reader_next", "ccsx_reader_close"],
}


class ZmwIn(C.Structure):
    _fields_ = [("seqs", C.c_char_p), ("seg_off", C.POINTER(C.c_uint32)), ("seg_len", C.POINTER(C.c_uint32)),
                ("nseg", C.c_uint32)]


class ZmwOut(C.Structure):
    _fields_ = [("ccs", C.c_void_p), ("len", C.c_uint32), ("status", C.c_int32), ("cells", C.c_uint64)]


class PairAln(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("qb", "qe", "tb", "te", "mat", "mis", "ins", "del_", "aln", "score")]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        L.ccsx_gpu_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.ccsx_gpu_close.argtypes = [C.c_void_p]
        L.ccsx_gpu_error.argtypes = [C.c_void_p]
        L.ccsx_gpu_error.restype = C.c_char_p
        L.ccsx_gpu_status_str.argtypes = [C.c_int32]
        L.ccsx_gpu_status_str.restype = C.c_char_p
        L.ccsx_gpu_run.argtypes = [C.c_void_p, C.c_int, C.POINTER(ZmwIn), C.c_size_t, C.POINTER(ZmwOut)]
        L.ccsx_gpu_stage.argtypes = [C.c_void_p, C.POINTER(ZmwIn), C.c_size_t]
        L.ccsx_gpu_stage_for.argtypes = [C.c_void_p, C.c_int, C.POINTER(ZmwIn), C.c_size_t]
        L.ccsx_gpu_launch.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_float)]
        L.ccsx_gpu_fetch.argtypes = [C.c_void_p, C.POINTER(ZmwOut)]
        L.ccsx_gpu_staged_bytes.argtypes = [C.c_void_p]
        L.ccsx_gpu_staged_bytes.restype = C.c_uint64
        L.ccsx_gpu_set_profiling.argtypes = [C.c_void_p, C.c_int]
        L.ccsx_gpu_profile.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]
        if hasattr(L, "ccsx_gpu_profile_zmw"):  # diagnostics; absent from older builds used in A/B runs
            L.ccsx_gpu_profile_zmw.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32, C.c_uint32]
        L.ccsx_gpu_set_tight_rows.argtypes = [C.c_void_p, C.c_uint32]
        L.ccsx_gpu_set_tight_out.argtypes = [C.c_void_p, C.c_uint32]
        if hasattr(L, "ccsx_gpu_set_tight_far"):  # (absent from the older builds used in A/B runs)
            L.ccsx_gpu_set_tight_far.argtypes = [C.c_void_p, C.c_uint32]
        L.ccsx_gpu_set_stage_piece.argtypes = [C.c_void_p, C.c_uint64]
        L.ccsx_gpu_set_prealloc.argtypes = [C.c_void_p, C.c_int]
        L.ccsx_gpu_set_kernel_cfg.argtypes = [C.c_void_p, C.c_int]
        L.ccsx_gpu_kernel_cfg.argtypes = [C.c_void_p]
        L.ccsx_gpu_rerun_count.argtypes = [C.c_void_p]
        L.ccsx_gpu_rerun_count.restype = C.c_int64
        L.ccsx_gpu_run_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]
        L.ccsx_gpu_zmw_bytes.argtypes = [C.c_void_p, C.c_int, C.POINTER(ZmwIn)]
        L.ccsx_gpu_zmw_bytes.restype = C.c_uint64
        L.ccsx_gpu_set_slot_budget.argtypes = [C.c_void_p, C.c_uint64]
        L.ccsx_gpu_set_wg_cap.argtypes = [C.c_void_p, C.c_uint32]
        L.ccsx_gpu_set_shred_read_cap.argtypes = [C.c_void_p, C.c_uint32]
        L.ccsx_gpu_set_mem_share.argtypes = [C.c_void_p, C.c_uint32]
        L.ccsx_gpu_set_mem_frac.argtypes = [C.c_void_p, C.c_float]
        L.ccsx_gpu_set_mem_wait.argtypes = [C.c_void_p, C.c_uint32]
        L.ccsx_gpu_slot_bytes.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.ccsx_gpu_submit.argtypes = [C.c_void_p, C.c_int, C.POINTER(ZmwIn), C.c_size_t, C.POINTER(C.c_int)]
        L.ccsx_gpu_collect.argtypes = [C.c_void_p, C.c_int, C.POINTER(ZmwOut)]
        L.ccsx_gpu_set_bp_log.argtypes = [C.c_void_p, C.c_int]
        L.ccsx_gpu_bp_log.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.POINTER(C.c_uint32)),
                                      C.POINTER(C.c_uint32)]
        L.ccsx_revcomp.argtypes = [C.c_char_p, C.c_uint32]
        L.ccsx_prepare.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)]
        L.ccsx_prepare.restype = C.c_uint32
        L.ccsx_prepare_apply.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32)]
        L.ccsx_prepare_apply.restype = C.c_uint32
        L.ccsx_pairwise.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32]
        L.ccsx_pairwise.restype = PairAln
        L.ccsx_synth_zmw.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_char_p,
                                     C.POINTER(C.c_uint32), C.c_char_p]
        L.ccsx_synth_zmw.restype = C.c_uint64
        L.ccsx_zmw_cost.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
        L.ccsx_zmw_cost.restype = C.c_uint64
        L.ccsx_partition.argtypes = [C.POINTER(C.c_uint64), C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.ccsx_partition.restype = C.c_uint32
        L.ccsx_synth_batch_make.argtypes = [C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                            C.POINTER(C.c_uint32), C.c_uint32, C.c_int]
        L.ccsx_synth_batch_make.restype = C.c_void_p
        L.ccsx_synth_batch_zmws.argtypes = [C.c_void_p]
        L.ccsx_synth_batch_zmws.restype = C.POINTER(ZmwIn)
        L.ccsx_synth_batch_free.argtypes = [C.c_void_p]
        L.ccsx_reader_open.argtypes = [C.c_char_p, C.c_int]
        L.ccsx_reader_open.restype = C.c_void_p
        L.ccsx_reader_next.argtypes = [C.c_void_p] + [C.POINTER(C.c_char_p)] * 2 + [C.POINTER(C.c_void_p),
                                                                                     C.POINTER(C.POINTER(C.c_uint32))]
        L.ccsx_reader_close.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def _p32(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


# ---------------------------------------------------------------- host helpers
def revcomp(seq: bytes) -> bytes:
    b = C.create_string_buffer(bytes(seq), len(seq))
    lib().ccsx_revcomp(b, len(seq))
    return b.raw[:len(seq)]


def synth_zmw(seed: int, hole: int, L: int, passes: int):
    """Synthetic ZMW: returns (list of subread bytes, true insert bytes)."""
    cap = passes * (2 * L + 16) + 16
    out = C.create_string_buffer(cap)
    lens = np.zeros(passes, dtype=np.uint32)
    ins = C.create_string_buffer(L + 1)
    lib().ccsx_synth_zmw(seed, hole, L, passes, out, _p32(lens), ins)
    raw = out.raw
    subs, o = [], 0
    for n in lens:
        subs.append(raw[o:o + int(n)])
        o += int(n)
    return subs, ins.raw[:L]


@dataclass
class Prepared:
    """One ZMW after ccs_prepare + strand flip: segments are slices of seqs."""
    seqs: bytes
    offs: np.ndarray
    lens: np.ndarray


def prepare(subreads: list[bytes]) -> Prepared:
    """ccs_prepare (main.c:344-453) + in-place reverse complement of reverse segments."""
    seqs = b"".join(subreads)
    buf = C.create_string_buffer(seqs, len(seqs) + 1)
    lens = _u32([len(s) for s in subreads])
    n = len(subreads)
    so = np.zeros(max(n, 1), dtype=np.uint32)
    sl = np.zeros(max(n, 1), dtype=np.uint32)
    ns = lib().ccsx_prepare_apply(buf, _p32(lens), n, _p32(so), _p32(sl))
    return Prepared(buf.raw[:len(seqs)], so[:ns].copy(), sl[:ns].copy())


def prepare_segments(subreads: list[bytes]):
    """ccs_prepare only: (offs, lens, reverse flags) into the concatenated subreads."""
    seqs = b"".join(subreads)
    lens = _u32([len(s) for s in subreads])
    n = len(subreads)
    so = np.zeros(max(n, 1), dtype=np.uint32)
    sl = np.zeros(max(n, 1), dtype=np.uint32)
    rv = np.zeros(max(n, 1), dtype=np.uint8)
    ns = lib().ccsx_prepare(seqs, _p32(lens), n, _p32(so), _p32(sl), rv.ctypes.data_as(C.POINTER(C.c_uint8)))
    return so[:ns].copy(), sl[:ns].copy(), rv[:ns].copy()


def zmw_cost(seg_len) -> int:
    """ccsx_zmw_cost: estimated POA work of a prepared ZMW (host/dispatch.cpp)."""
    a = _u32(seg_len)
    return int(lib().ccsx_zmw_cost(_p32(a), len(a)))


def partition(costs, nparts: int, min_batch: int):
    """ccsx_partition: (LPT order, list of batches as index lists into the input)."""
    c = np.ascontiguousarray(np.asarray(costs, dtype=np.uint64))
    n = len(c)
    order = np.zeros(max(n, 1), dtype=np.uint32)
    bounds = np.zeros(n + 1, dtype=np.uint32)
    nb = lib().ccsx_partition(c.ctypes.data_as(C.POINTER(C.c_uint64)), n, nparts, min_batch, _p32(order), _p32(bounds))
    return order[:n].tolist(), [order[bounds[b]:bounds[b + 1]].tolist() for b in range(nb)]


def pairwise(q: bytes, t: bytes) -> dict:
    r = lib().ccsx_pairwise(q, len(q), t, len(t))
    return {n if n != "del_" else "del": getattr(r, n) for n, _ in PairAln._fields_}


def read_calls(path: str, is_bam: bool = False):
    """Yield every ccsx_reader_next result the way main.c step 0 drives
    kseq_zmw_read (main.c:658-697): (n, movie, hole, [subreads]) for a ZMW,
    (-1, None, None, None) for each -1; after a -1 the next chunk reads on,
    and the input ends at the first chunk that yields no ZMW."""
    L = lib()
    r = L.ccsx_reader_open(path.encode(), 1 if is_bam else 0)
    if not r:
        raise OSError(f"cannot open {path}")
    try:
        mv, hl = C.c_char_p(), C.c_char_p()
        sq = C.c_void_p()
        ln = C.POINTER(C.c_uint32)()
        while True:
            got = 0
            while True:
                n = L.ccsx_reader_next(r, C.byref(mv), C.byref(hl), C.byref(sq), C.byref(ln))
                if n < 0:
                    yield n, None, None, None
                    break
                got += 1
                lens = [ln[i] for i in range(n)]
                raw = C.string_at(sq, sum(lens))
                subs, o = [], 0
                for x in lens:
                    subs.append(raw[o:o + x])
                    o += x
                yield n, mv.value.decode(), hl.value.decode(), subs
            if not got:
                break
    finally:
        L.ccsx_reader_close(r)


def read_zmws(path: str, is_bam: bool = False):
    """Yield (movie, hole, [subreads]) per ZMW, as the CLI's step 0 sees them."""
    for n, movie, hole, subs in read_calls(path, is_bam):
        if n >= 0:
            yield movie, hole, subs


class SynthBatch:
    """ccsx_synth_batch_make: n synthetic ZMWs made and prepared on C threads."""

    def __init__(self, seed: int, holes, Ls, passes, nthreads: int = 16):
        n = len(holes)
        h = np.ascontiguousarray(holes, dtype=np.uint64)
        lv, pv = _u32(Ls), _u32(passes)
        self._L = lib()
        self.n = n
        self._b = self._L.ccsx_synth_batch_make(seed, h.ctypes.data_as(C.POINTER(C.c_uint64)), _p32(lv), _p32(pv), n,
                                                nthreads)
        self.zmws = self._L.ccsx_synth_batch_zmws(self._b)
        self.bases = sum(int(self.zmws[i].seg_len[k]) for i in range(n) for k in range(self.zmws[i].nseg))

    def __del__(self):
        try:
            self._L.ccsx_synth_batch_free(self._b)
        except Exception:
            pass


# ---------------------------------------------------------------- GPU engine
def device_count() -> int:
    """Visible HIP devices (0 without a GPU)."""
    return int(lib().ccsx_gpu_device_count())


class GpuError(RuntimeError):
    pass


class Engine:
    """A context on one HIP device: the batched C-ABI of include/ccsx_gpu.h."""

    def __init__(self, device: int = 0):
        self._L = lib()
        self._ctx = C.c_void_p()
        if self._L.ccsx_gpu_open(device, C.byref(self._ctx)) != 0:
            raise GpuError(f"cannot open HIP device {device}")
        self._keep = None
        self._nz = 0

    def close(self):
        if self._ctx:
            self._L.ccsx_gpu_close(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, what: str):
        raise GpuError(f"{what}: {self._L.ccsx_gpu_error(self._ctx).decode()}")

    @staticmethod
    def _build_in(zmws: list[Prepared]):
        arr = (ZmwIn * max(len(zmws), 1))()
        keep = []
        for i, z in enumerate(zmws):
            offs, lens = _u32(z.offs), _u32(z.lens)
            keep += [z.seqs, offs, lens]
            arr[i].seqs = z.seqs
            arr[i].seg_off = _p32(offs)
            arr[i].seg_len = _p32(lens)
            arr[i].nseg = len(lens)
        return arr, keep

    def stage(self, zmws: list[Prepared], mode: int | None = None) -> None:
        """Stage a slice (tight capacities); with `mode`, the capacities
        ccsx_gpu_run uses for that mode (ccsx_gpu_stage_for)."""
        arr, keep = self._build_in(zmws)
        rc = (self._L.ccsx_gpu_stage(self._ctx, arr, len(zmws)) if mode is None
              else self._L.ccsx_gpu_stage_for(self._ctx, mode, arr, len(zmws)))
        if rc != 0:
            self._err("ccsx_gpu_stage")
        self._keep = (arr, keep)
        self._nz = len(zmws)

    def launch(self, mode: int = MODE_SHRED) -> float:
        ms = C.c_float(0)
        if self._L.ccsx_gpu_launch(self._ctx, mode, C.byref(ms)) != 0:
            self._err("ccsx_gpu_launch")
        return ms.value

    def fetch(self):
        out = (ZmwOut * max(self._nz, 1))()
        rc = self._L.ccsx_gpu_fetch(self._ctx, out)
        if rc != 0:
            self._err("ccsx_gpu_fetch")
        res = []
        for i in range(self._nz):
            o = out[i]
            res.append((C.string_at(o.ccs, o.len) if o.len else b"", o.status, o.cells))
        return res

    def run(self, zmws: list[Prepared], mode: int = MODE_SHRED):
        """ccsx_gpu_run (memory-sized slices, full-capacity re-run of ZMWs that
        outgrow the tight workspace): returns [(ccs bytes, status, cells)]."""
        arr, keep = self._build_in(zmws)
        out = (ZmwOut * max(len(zmws), 1))()
        if self._L.ccsx_gpu_run(self._ctx, mode, arr, len(zmws), out) != 0:
            self._err("ccsx_gpu_run")
        return [(C.string_at(out[i].ccs, out[i].len) if out[i].len else b"", out[i].status, out[i].cells)
                for i in range(len(zmws))]

    def run_batch(self, batch: "SynthBatch", mode: int = MODE_SHRED, keep=()):
        """ccsx_gpu_run on a synthetic batch; returns [(status, cells, len)]
        and, when `keep` lists batch indices, also {index: CCS bytes}."""
        out = (ZmwOut * max(batch.n, 1))()
        rc = self._L.ccsx_gpu_run(self._ctx, mode, batch.zmws, batch.n, out)
        if rc != 0:
            self._err("ccsx_gpu_run")
        res = [(out[i].status, out[i].cells, out[i].len) for i in range(batch.n)]
        if keep:
            return res, {i: C.string_at(out[i].ccs, out[i].len) if out[i].len else b"" for i in keep}
        return res

    def stage_batch(self, batch: "SynthBatch", mode: int = MODE_SHRED) -> None:
        """ccsx_gpu_stage_for on a synthetic batch (inputs resident for launch())."""
        if self._L.ccsx_gpu_stage_for(self._ctx, mode, batch.zmws, batch.n) != 0:
            self._err("ccsx_gpu_stage_for")
        self._keep = batch
        self._nz = batch.n

    def set_mem_share(self, share: int) -> None:
        """This context uses at most 1/share of the device's memory (several
        contexts, or processes, on one device)."""
        if self._L.ccsx_gpu_set_mem_share(self._ctx, share) != 0:
            self._err("ccsx_gpu_set_mem_share")

    def set_kernel_cfg(self, cfg: int) -> None:
        """-1 = by slice size, 0 = latency (8-row blocks), 1 = occupancy (4-row blocks)."""
        if self._L.ccsx_gpu_set_kernel_cfg(self._ctx, cfg) != 0:
            self._err("ccsx_gpu_set_kernel_cfg")

    def kernel_cfg(self) -> int:
        return int(self._L.ccsx_gpu_kernel_cfg(self._ctx))

    def rerun_count(self) -> int:
        """ZMWs run() has re-run with full caps so far."""
        return int(self._L.ccsx_gpu_rerun_count(self._ctx))

    def run_stats(self) -> dict:
        """ccsx_gpu_run counters so far: reruns, slices, dealt lists, their
        parts, slices that waited for device memory, slices cut below the plan."""
        st = (C.c_uint64 * 6)()
        if self._L.ccsx_gpu_run_stats(self._ctx, st, 6) != 0:
            self._err("ccsx_gpu_run_stats")
        return dict(zip(("reruns", "slices", "dealt", "parts", "mem_waits", "mem_replans"), (int(x) for x in st)))

    def set_mem_wait(self, ms: int) -> None:
        """How long a slice waits for device memory a neighbour still holds."""
        if self._L.ccsx_gpu_set_mem_wait(self._ctx, ms) != 0:
            self._err("ccsx_gpu_set_mem_wait")

    def zmw_bytes(self, z: Prepared, mode: int = MODE_SHRED) -> int:
        """Device bytes one ZMW occupies in a ccsx_gpu_run slice of `mode`."""
        arr, keep = self._build_in([z])
        return int(self._L.ccsx_gpu_zmw_bytes(self._ctx, mode, arr))

    def slot_bytes(self) -> int:
        """ccsx_gpu_slot_bytes: the bytes one submitted batch may take."""
        v = C.c_uint64(0)
        if self._L.ccsx_gpu_slot_bytes(self._ctx, C.byref(v)) != 0:
            self._err("ccsx_gpu_slot_bytes")
        return int(v.value)

    def submit(self, zmws: list, mode: int = MODE_SHRED) -> int:
        """ccsx_gpu_submit: stage + launch one batch on a free slot (returns
        the slot to collect; raises on -3 / -4 with the code in the message)."""
        arr, keep = self._build_in(zmws)
        slot = C.c_int(-1)
        rc = self._L.ccsx_gpu_submit(self._ctx, mode, arr, len(zmws), C.byref(slot))
        if rc != 0:
            self._err(f"ccsx_gpu_submit ({rc})")
        self._tickets = getattr(self, "_tickets", {})
        self._tickets[slot.value] = (arr, keep, len(zmws))
        return slot.value

    def collect(self, slot: int):
        """ccsx_gpu_collect: [(ccs bytes, status, cells)] of a submitted batch."""
        arr, keep, n = self._tickets.pop(slot)
        out = (ZmwOut * max(n, 1))()
        rc = self._L.ccsx_gpu_collect(self._ctx, slot, out)
        if rc not in (0, -2):
            self._err("ccsx_gpu_collect")
        return [(C.string_at(out[i].ccs, out[i].len) if out[i].len else b"", out[i].status, out[i].cells)
                for i in range(n)]

    def set_bp_log(self, on: bool = True) -> None:
        """Record the -v >= 3 breakpoint log (main.c:619-620) in ccsx_gpu_run."""
        if self._L.ccsx_gpu_set_bp_log(self._ctx, 1 if on else 0) != 0:
            self._err("ccsx_gpu_set_bp_log")

    def bp_log(self, i: int) -> list:
        """(breakpoint, MSA columns) per shredding round of ZMW i of the last run()."""
        pr = C.POINTER(C.c_uint32)()
        n = C.c_uint32(0)
        if self._L.ccsx_gpu_bp_log(self._ctx, i, C.byref(pr), C.byref(n)) != 0:
            self._err("ccsx_gpu_bp_log")
        return [(int(pr[2 * r]), int(pr[2 * r + 1])) for r in range(n.value)]

    def set_slot_budget(self, nbytes: int) -> None:
        """Test hook: bytes per ccsx_gpu_run slot (0 = by device memory)."""
        if self._L.ccsx_gpu_set_slot_budget(self._ctx, nbytes) != 0:
            self._err("ccsx_gpu_set_slot_budget")

    def set_wg_cap(self, wg_per_cu: int) -> None:
        """Measurement hook: at most wg_per_cu resident workgroups per CU (0 = off)."""
        if self._L.ccsx_gpu_set_wg_cap(self._ctx, wg_per_cu) != 0:
            self._err("ccsx_gpu_set_wg_cap")

    def set_shred_read_cap(self, bases: int) -> None:
        """The LDS read buffer of tight-cap shredded slices, in bases."""
        if self._L.ccsx_gpu_set_shred_read_cap(self._ctx, bases) != 0:
            self._err("ccsx_gpu_set_shred_read_cap")

    def set_tight_rows(self, rows: int) -> None:
        """Test hook: override the tight row capacity (0 = default)."""
        self._L.ccsx_gpu_set_tight_rows(self._ctx, rows)

    def set_tight_far(self, rows: int) -> None:
        """Test hook: override the tight far slot record rows (0 = default)."""
        self._L.ccsx_gpu_set_tight_far(self._ctx, rows)

    def set_prealloc(self, on: bool) -> None:
        """Pinned staging floors and one-off slice budget, as the CLI's contexts."""
        self._L.ccsx_gpu_set_prealloc(self._ctx, 1 if on else 0)

    def set_stage_piece(self, nbytes: int) -> None:
        """Test hook: half size of the piecewise subread staging (0 = default)."""
        self._L.ccsx_gpu_set_stage_piece(self._ctx, nbytes)

    def set_tight_out(self, nbytes: int) -> None:
        """Test hook: override the tight output slab in bytes (0 = default)."""
        self._L.ccsx_gpu_set_tight_out(self._ctx, nbytes)

    PROF_SLOTS = ("total", "load_read", "dp", "traceback", "merge", "columns", "shred", "dp_rows",
                  "row_A_fast", "row_B_general", "row_C_unused", "row_D_nfast", "row_E_store_loop", "flush", "spare0", "spare1",
                  "a_busy", "a_wait", "b_busy", "b_wait", "tw_rows", "sw_rows", "spare2", "spare3",
                  "tb_probe", "tb_step", "tb_di", "tb_switch", "tb_nsw", "hw0", "hw1", "hw2", "start_rt", "end_rt", "a_head", "a_body", "a_tail", "a_fast",
                  "cold_far", "cold_chain", "cold_np1", "cold_np2", "cold_gen", "cold_spill", "cold_near",
                  "n_far", "n_chain", "n_np1", "n_np2", "n_gen", "n_spill", "n_near",
                  "tb_isteps", "tb_iruns", "tb_dsteps", "tb_druns")

    def set_profiling(self, on: bool = True) -> None:
        """Per-phase counters on / off; raises with the product library (its
        objects carry none: CCSX_LIB=libccsx_amd_diag.so)."""
        if self._L.ccsx_gpu_set_profiling(self._ctx, 1 if on else 0) != 0:
            self._err("ccsx_gpu_set_profiling")

    def profile(self) -> dict:
        """Per-phase shader-clock cycles summed over the last launch's ZMWs."""
        buf = (C.c_uint64 * len(self.PROF_SLOTS))()
        if self._L.ccsx_gpu_profile(self._ctx, buf, len(self.PROF_SLOTS)) != 0:
            self._err("ccsx_gpu_profile")
        return {k: int(buf[i]) for i, k in enumerate(self.PROF_SLOTS)}

    def profile_zmw(self, nzmw: int) -> list:
        """The same counters per ZMW of the last launch (staging order)."""
        ns = len(self.PROF_SLOTS)
        buf = (C.c_uint64 * (nzmw * ns))()
        if self._L.ccsx_gpu_profile_zmw(self._ctx, buf, nzmw, ns) != 0:
            self._err("ccsx_gpu_profile_zmw")
        return [{k: int(buf[z * ns + i]) for i, k in enumerate(self.PROF_SLOTS)} for z in range(nzmw)]

    def staged_bytes(self) -> int:
        return int(self._L.ccsx_gpu_staged_bytes(self._ctx))
