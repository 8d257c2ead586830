"""GPU (HIP, through the C-ABI) vs oracle (C restatement): bit-exact CCS.

The bar is byte equality of every CCS string (SPEC.md is integer-only, so no
tolerance).  Sizes are chosen so the oracle finishes in seconds; the full
BASELINE sizes are covered by test_gpu_full_size_properties.
"""
import pytest

import ccsx_amd as cx
from oracle.oracle import Poa, batch, edit_identity
from tests.zmw_cases import edge_cases, high_indegree, raw, synth

pytestmark = pytest.mark.gpu


def _check(engine, zs, mode, threads=8):
    want, _, _ = batch(zs, mode, threads)
    got = engine.run(zs, mode)
    for i, (w, (g, status, cells)) in enumerate(zip(want, got)):
        assert status == 0, f"ZMW {i}: device status {status}"
        assert g == w, f"ZMW {i}: GPU CCS ({len(g)} bp) != oracle CCS ({len(w)} bp)"
    return got


@pytest.mark.parametrize("L,passes,n", [(2000, 8, 32), (10000, 8, 8), (2000, 30, 6), (5000, 12, 6)])
def test_shredded_synthetic(engine, L, passes, n):
    zs = [synth(h, L, passes) for h in range(n)]
    _check(engine, zs, cx.MODE_SHRED)


@pytest.mark.parametrize("L,passes,n", [(3000, 5, 16), (20000, 5, 2)])
def test_primitive_synthetic(engine, L, passes, n):
    zs = [synth(1000 + h, L, passes) for h in range(n)]
    _check(engine, zs, cx.MODE_PRIMITIVE)


@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_edge_cases(engine, mode):
    cases = edge_cases()
    names = list(cases)
    zs = [cases[k] for k in names]
    want, _, _ = batch(zs, mode, 8)
    got = engine.run(zs, mode)
    for name, w, (g, status, _) in zip(names, want, got):
        assert status == 0, f"{name}: device status {status}"
        assert g == w, f"{name}: GPU CCS != oracle CCS"


def test_cells_match_oracle(engine):
    zs = [synth(h, 2000, 8) for h in range(4)]
    _, cells, _ = batch(zs, cx.MODE_SHRED, 4)
    got = engine.run(zs, cx.MODE_SHRED)
    assert [c for _, _, c in got] == cells


def test_mixed_batch_order_preserved(engine):
    """Heterogeneous ZMWs in one launch come back in input order (main.c:707-717)."""
    zs = [synth(h, L, p) for h, (L, p) in enumerate([(2000, 8), (6000, 5), (1500, 20), (9000, 6), (2500, 7)])]
    _check(engine, zs, cx.MODE_SHRED)


def test_repeat_launch_deterministic(engine):
    zs = [synth(h, 3000, 8) for h in range(8)]
    engine.stage(zs)
    engine.launch(cx.MODE_SHRED)
    a = engine.fetch()
    engine.launch(cx.MODE_SHRED)
    b = engine.fetch()
    assert a == b


def _identity(ccs, ins):
    """CCS vs the generator's true insert, either strand (the template may be
    a reverse pass): a banded edit identity (not parity)."""
    return max(edit_identity(ccs, ins), edit_identity(ccs, cx.revcomp(ins)))


def test_gpu_full_size_properties(engine):
    """BASELINE config B shape (10 kb x 8) at a 64-ZMW sample: parity on a
    subset plus size-independent properties on all: status, length, cells and
    identity to the synthetic truth (mean >= 0.99, min >= 0.985)."""
    import random
    zs, truth = [], []
    for h in range(64):
        subs, ins = cx.synth_zmw(20201104, h, 10000, 8)
        zs.append(cx.prepare(subs))
        truth.append(ins)
    got = engine.run(zs, cx.MODE_SHRED)
    ids = []
    for (g, status, cells), ins in zip(got, truth):
        assert status == 0
        assert 9700 <= len(g) <= 10300
        assert cells > 8_000_000
        ids.append(_identity(g, ins))
    assert sum(ids) / len(ids) >= 0.99 and min(ids) >= 0.985, (sum(ids) / len(ids), min(ids))
    sample = random.Random(3).sample(range(64), 6)
    want, _, _ = batch([zs[i] for i in sample], cx.MODE_SHRED, 6)
    for i, w in zip(sample, want):
        assert got[i][0] == w


def _config_shapes(name, n):
    import bench
    if name == "E":
        cfg = bench.CONFIGS["E"]
        holes = range(10_000_000, 10_000_000 + 4000)
        shapes = sorted(((h, *bench.zmw_shape(cfg, h)) for h in holes), key=lambda s: s[1] * s[2])
        # the smallest, the median and the largest drawn shapes
        return [shapes[0], shapes[len(shapes) // 2], shapes[-1]] + [shapes[i * 37 % len(shapes)] for i in range(n - 3)]
    L, p = {"C": (20000, 5), "D": (2000, 30)}[name]
    return [(20_000 + h, L, p) for h in range(n)]


@pytest.mark.parametrize("name,mode,n", [("C", cx.MODE_PRIMITIVE, 24), ("D", cx.MODE_SHRED, 48), ("E", cx.MODE_SHRED, 24)])
def test_gpu_accuracy_vs_truth(engine, name, mode, n):
    """Configs C (20 kb x 5, -P, main.c:486-502), D (2 kb x 30) and E (mixed
    5-25 kb inserts x 5-12 passes, shredded, main.c:622-638): the device's
    CCS against the synthetic truth (mean >= 0.99, min >= 0.985), plus oracle
    parity on a 3-ZMW sample.  A restatement that is deterministic but
    degrades at these lengths or pass counts fails here."""
    import bench
    zs, truth = [], []
    for h, L, p in _config_shapes(name, n):
        subs, ins = cx.synth_zmw(bench.SEED, h, L, p)
        zs.append(cx.prepare(subs))
        truth.append(ins)
    got = engine.run(zs, mode)
    ids = []
    for (g, status, _), ins in zip(got, truth):
        assert status == 0
        ids.append(_identity(g, ins))
    assert sum(ids) / len(ids) >= 0.99 and min(ids) >= 0.985, (sum(ids) / len(ids), min(ids))
    want, _, _ = batch(zs[:3], mode, 3)
    assert [g for g, _, _ in got[:3]] == want


@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_capacity_rerun(engine, mode):
    """A ZMW whose graph outgrows the tight workspace is re-run with full caps
    (ccsx_gpu_run) and still matches the oracle; a tiny tight row cap forces
    the re-run for every ZMW of the batch but one tiny one."""
    zs = [synth(h, 3000, 6) for h in range(5)] + [cx.prepare([b"ACGTACGTAC"] * 5)]
    engine.set_tight_rows(600)
    try:
        _check(engine, zs, mode)
    finally:
        engine.set_tight_rows(0)


@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_output_slab_rerun(engine, mode):
    """A consensus longer than the tight output slab (kErrOut) is re-run with
    full caps, by ccsx_gpu_run and inside ccsx_gpu_collect; a 64-byte tight
    slab forces it for every ZMW but the tiny one."""
    zs = [synth(6100 + h, 1500, 6) for h in range(4)] + [cx.prepare([b"ACGTACGTAC"] * 5)]
    want, _, _ = batch(zs, mode, 5)
    engine.set_tight_out(64)
    try:
        before = engine.rerun_count()
        _check(engine, zs, mode)
        assert engine.rerun_count() - before >= 4
        s = engine.submit(zs, mode)
        got = engine.collect(s)
        assert [g for g, _, _ in got] == want and all(st == 0 for _, st, _ in got)
    finally:
        engine.set_tight_out(0)


def test_piecewise_staging():
    """A preallocating context sharing its device (the CLI's) stages subreads
    through two pinned halves; 4 KiB halves here, so pieces split ZMWs and
    every copy waits on the one before last.  ccsx_gpu_run and submit /
    collect both equal the oracle."""
    zs = [synth(6300 + h, 2500, 6) for h in range(6)]
    want, _, _ = batch(zs, cx.MODE_SHRED, 6)
    e = cx.Engine(0)
    try:
        e.set_prealloc(True)
        e.set_mem_share(2)
        e.set_stage_piece(4096)
        got = e.run(zs, cx.MODE_SHRED)
        assert [g for g, _, _ in got] == want and all(st == 0 for _, st, _ in got)
        s = e.submit(zs[:4])
        got = e.collect(s)
        assert [g for g, _, _ in got] == want[:4]
    finally:
        e.close()


@pytest.mark.parametrize("cfg", [0, 5])
def test_far_record_rerun(engine, cfg):
    """Rows with more than four predecessors keep their slots in far slot
    records of a tight capacity (rcap / 16 + 64); a DP that meets more fails
    the ZMW with kErrSpill and ccsx_gpu_run re-runs it with full caps (a
    record per row).  A capacity of one forces it on wide graphs (70 passes):
    byte-equal to the oracle, on the helper and the one-wave objects."""
    zs = [synth(6500 + h, 1500, 70) for h in range(2)]
    engine.set_kernel_cfg(cfg)
    engine.set_tight_far(1)
    try:
        before = engine.rerun_count()
        _check(engine, zs, cx.MODE_SHRED)
        assert engine.rerun_count() - before >= 1
    finally:
        engine.set_tight_far(0)
        engine.set_kernel_cfg(-1)


def test_tight_caps_fail_loudly_without_rerun(engine):
    """stage/launch/fetch (no re-run) reports the capacity status."""
    zs = [synth(h, 3000, 6) for h in range(2)]
    engine.set_tight_rows(600)
    try:
        engine.stage(zs)
        engine.launch(cx.MODE_SHRED)
        with pytest.raises(cx.GpuError):
            engine.fetch()
    finally:
        engine.set_tight_rows(0)


@pytest.mark.parametrize("L,passes,n,mode", [(1500, 70, 2, cx.MODE_SHRED), (2500, 66, 2, cx.MODE_PRIMITIVE)])
def test_wide_graphs(engine, L, passes, n, mode):
    """More than 64 reads (two membership words), in-degrees above 4 and
    predecessors beyond the DP ring: the far-row path with slot tags and the
    HBM spill records of the two-wave DP."""
    zs = [synth(3000 + h, L, passes) for h in range(n)]
    _check(engine, zs, mode)


@pytest.mark.parametrize("L,passes,mode", [(60, 12, cx.MODE_SHRED), (100, 12, cx.MODE_PRIMITIVE), (127, 9, cx.MODE_PRIMITIVE)])
def test_reads_shorter_than_band(engine, L, passes, mode):
    """Reads shorter than W = 128: the partial-band DP (cells past the read
    end invalid, the free end inside the band)."""
    zs = [synth(4000 + h, L, passes) for h in range(16)]
    _check(engine, zs, mode)


def _e_shapes():
    """Config E (bench.py zmw_shape) holes: the largest drawn shapes."""
    import bench
    cfg = bench.CONFIGS["E"]
    shapes = [(h, *bench.zmw_shape(cfg, h)) for h in range(6000)]
    big = [s for s in shapes if s[1] >= 20000 and s[2] >= 10]
    top = max(shapes, key=lambda s: s[1] * s[2])
    return big[:3] + [top]


def test_config_e_largest_shapes(engine):
    """Config E's largest ZMWs (>= 20 kb inserts x >= 10 passes and the
    largest L x passes of 6,000 drawn holes, ~300 kb of subreads) through
    ccsx_gpu_run (tight caps, full-cap re-run) vs the oracle, in one batch
    with small ZMWs so the LPT launch order is exercised."""
    import bench
    zs = []
    for h, L, p in _e_shapes():
        subs, _ = cx.synth_zmw(bench.SEED, h, L, p)
        zs.append(cx.prepare(subs))
    zs += [synth(7000 + h, 2000, 6) for h in range(4)]
    assert max(int(z.lens.sum()) for z in zs) > 250_000
    _check(engine, zs, cx.MODE_SHRED)


def test_zmw_near_max_total_length(engine):
    """A ZMW near ccsx's -M cap (500 kb, main.c:662-665): 25 kb x 17 passes,
    ~440 kb of subreads, shredded mode."""
    zs = [synth(7100, 25000, 17)]
    assert 400_000 < int(zs[0].lens.sum()) < 500_000
    _check(engine, zs, cx.MODE_SHRED)


@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_indegree_above_63(engine, mode):
    """A far row with 74 predecessors: its cell tags do not fit the 6-bit slot
    field, the helpers store the full slots in the wide records and the
    traceback follows them (round 1 failed the ZMW with status 5)."""
    from oracle.oracle import Poa
    reads = high_indegree()
    g = Poa()
    g.poa(reads)
    assert g.max_indegree() > 63
    zs = [raw(reads), raw(high_indegree(8)), synth(7200, 1500, 6)]
    _check(engine, zs, mode)


@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_read_beyond_lds_buffer(engine, mode):
    """Segments of 110 kb (more than the LDS read buffer's 100 kb): the slice
    runs the HBM-read kernel instance, in the same call as ordinary ZMWs."""
    zs = [synth(7300, 110_000, 5), synth(7301, 3000, 6), synth(7302, 40_000, 5)]
    _check(engine, zs, mode)


def test_more_segments_than_lds_cursors(engine):
    """4,200 segments of 60 bases (more than the 4,096 LDS shredding cursors):
    the HBM-read instance keeps the cursors in the workspace."""
    import random
    rnd = random.Random(11)
    ins = bytes(rnd.choice(b"ACGT") for _ in range(60))
    segs = []
    for _ in range(4200):
        s = bytearray(ins)
        s[rnd.randrange(60)] = rnd.choice(b"ACGT")
        segs.append(bytes(s))
    _check(engine, [raw(segs), synth(7400, 2000, 6)], cx.MODE_SHRED)


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_both_kernel_configs(engine, cfg, mode):
    """The latency (8-row DP blocks, 32-row ring), occupancy (4-row blocks,
    24-row ring), throughput (two-wave workgroups, 16-row ring), solo
    (one-wave workgroups, 8-row ring, one traceback buffer) and solo16 (the
    solo one with an int16 ring and 16-row traceback blocks; solo16w: the same
    at 80 VGPRs, 24 per CU) kernel objects,
    each forced, on a mixed batch: short reads, a wide graph, ordinary ZMWs
    (the by-size choice picks only one of them for small test batches)."""
    zs = [synth(7400 + h, L, p) for h, (L, p) in enumerate([(2000, 8), (100, 12), (1500, 70), (4000, 6), (7000, 5)])]
    engine.set_kernel_cfg(cfg)
    try:
        _check(engine, zs, mode)
        assert engine.kernel_cfg() == cfg
    finally:
        engine.set_kernel_cfg(-1)


def test_shred_window_beyond_read_cap(engine):
    """Shredded ZMWs whose pushed windows exceed the 4,096-base read buffer of
    a tight-cap slice (with two passes the whole 12 kb and 9 kb segments are
    pushed, main.c:555-567): kErrReadLen, re-run uncapped, oracle parity."""
    zs = [synth(7500, 12000, 2), synth(7501, 2000, 8), synth(7502, 9000, 2)]
    before = engine.rerun_count()
    _check(engine, zs, cx.MODE_SHRED)
    assert engine.rerun_count() - before >= 2


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_throughput_config_parity(engine, mode, cfg):
    """The throughput (one helper wave), solo (no helper: the wave computes
    its own decision bits) and solo16 (int16 ring) configurations, whose rings
    read back 8 rows (more rows take the far / spill path), forced on the
    parity shapes: config B/C/D-like ZMWs, wide graphs, short reads and the
    edge cases.  (-P pushes the 20 kb segments whole: beyond solo16's 16,256
    bases, so that call runs the solo object.)"""
    cases = edge_cases()
    zs = [synth(7600 + h, L, p) for h, (L, p) in enumerate([(10000, 8), (2000, 30), (20000, 5), (1500, 70), (60, 12)])]
    zs += [cases[k] for k in cases]
    engine.set_kernel_cfg(cfg)
    try:
        _check(engine, zs, mode)
        # (a shredded call's full-cap re-run of the 20 kb ZMW may also run solo)
        assert engine.kernel_cfg() in ((3,) if cfg >= 4 and mode == cx.MODE_PRIMITIVE else (3, cfg) if cfg >= 4 else (cfg,))
    finally:
        engine.set_kernel_cfg(-1)


@pytest.mark.parametrize("mode", [cx.MODE_SHRED, cx.MODE_PRIMITIVE])
def test_solo_config_hbm_read_instance(engine, mode):
    """The solo object (one wave, dp_solo's own read-window slides, one
    traceback buffer) forced on the HBM-read instance's shapes: 110 kb
    segments (-P pushes them whole) and a ZMW of 4,200 segments (its cursors
    live in the workspace), beside an ordinary ZMW."""
    import random
    rnd = random.Random(12)
    ins = bytes(rnd.choice(b"ACGT") for _ in range(60))
    segs = []
    for _ in range(4200):
        s = bytearray(ins)
        s[rnd.randrange(60)] = rnd.choice(b"ACGT")
        segs.append(bytes(s))
    zs = [synth(7700, 110_000, 3), raw(segs), synth(7701, 3000, 6)]
    engine.set_kernel_cfg(3)
    try:
        _check(engine, zs, mode)
        assert engine.kernel_cfg() == 3
    finally:
        engine.set_kernel_cfg(-1)


@pytest.mark.parametrize("cfg", [4, 5])
def test_solo16_int16_bound(engine, cfg):
    """solo16's int16 cells at the object's read-length limit: -P pushes the
    segments whole, 16,256 bases each (kRing16MaxRead), identical or with
    substitutions only, so H' climbs to ~2m and X = H' + 2t to within a few
    units of 2m + 254 = 32,766 -- the bound the int16 recurrence is exact
    under; then 16,257-base segments, which the host sends to
    the int32 solo object instead (stage_slot's max_read)."""
    import random
    from tests.zmw_cases import mutate
    rnd = random.Random(16256)
    ins = bytes(rnd.choice(b"ACGT") for _ in range(16256))
    subs = lambda: mutate(rnd, ins, 0.0, 0.0, 0.003)  # noqa: E731  (length kept)
    zs = [raw([ins] * 3), raw([subs() for _ in range(4)])]
    engine.set_kernel_cfg(cfg)
    try:
        _check(engine, zs, cx.MODE_PRIMITIVE)
        assert engine.kernel_cfg() == cfg
        longer = ins + b"A"
        _check(engine, [raw([longer] * 3)], cx.MODE_PRIMITIVE)
        assert engine.kernel_cfg() == 3
    finally:
        engine.set_kernel_cfg(-1)


def test_large_slice_picks_solo(engine):
    """A slice of several times the occupancy object's resident ZMWs takes
    the solo object by default (ccsx_gpu.cpp stage_slot) and stays byte-equal
    to the oracle: 4,096 short ZMWs (300 bp x 6 passes)."""
    zs = [synth(80000 + h, 300, 6) for h in range(4096)]
    engine.set_kernel_cfg(-1)
    _check(engine, zs, cx.MODE_SHRED, threads=16)
    assert engine.kernel_cfg() == 5  # solo16w: a tight-cap shredded slice of 6-segment ZMWs on the LDS instance
    # ZMWs of 20 segments too (config D's shape: solo16w since the 8-bit records)
    zs = [synth(81000 + h, 300, 20) for h in range(4096)]
    _check(engine, zs, cx.MODE_SHRED, threads=16)
    assert engine.kernel_cfg() == 5
    # ZMWs of 66 segments take solo16 (20 per CU, 96 VGPRs)
    zs = [synth(82000 + h, 150, 66) for h in range(4096)]
    _check(engine, zs, cx.MODE_SHRED, threads=16)
    assert engine.kernel_cfg() == 4


def _e_zmws(hole0, n):
    import bench
    cfg = bench.CONFIGS["E"]
    return [cx.prepare(cx.synth_zmw(bench.SEED, h, *bench.zmw_shape(cfg, h))[0]) for h in range(hole0, hole0 + n)]


def test_multi_slice_run(engine):
    """ccsx_gpu_run's multi-slice paths under a small slot budget
    (ccsx_gpu_set_slot_budget): ~150 config-E ZMWs dealt into >= 4
    interleaved parts on the two slots, two ZMWs whose pushed window outgrows
    the 4,096-base read cap (kErrReadLen, re-run with full caps after the
    pipelined slices), the -v >= 3 breakpoint log gathered across slots; then
    a budget below the largest ZMW, so the list is cut into contiguous
    slices.  CCS, input order and the breakpoint log byte-equal to the
    oracle."""
    from oracle.oracle import Poa
    zs = _e_zmws(10_500_000, 150)
    zs.insert(70, synth(7500, 12000, 2))
    zs.insert(20, synth(7502, 9000, 2))
    tot = sum(engine.zmw_bytes(z) for z in zs)
    st0 = engine.run_stats()
    engine.set_slot_budget(int(tot / 3.5))
    engine.set_bp_log(True)
    try:
        _check(engine, zs, cx.MODE_SHRED, threads=16)
        st = engine.run_stats()
        assert st["dealt"] - st0["dealt"] >= 1
        assert st["parts"] - st0["parts"] >= 4
        assert st["reruns"] - st0["reruns"] >= 2
        assert st["slices"] - st0["slices"] >= 5  # >= 4 parts + the re-run
        ref = Poa()
        for i in (0, 20, 21, 70, 71, len(zs) - 1):
            _, bps = ref.zmw_breakpoints(zs[i].seqs, zs[i].offs, zs[i].lens)
            assert engine.bp_log(i) == [tuple(x) for x in bps], f"ZMW {i}: breakpoint log"
        # contiguous slices: a budget below the largest ZMW of the list
        small = zs[:24]
        sizes = sorted(engine.zmw_bytes(z) for z in small)
        engine.set_slot_budget(sizes[-2])
        st0 = engine.run_stats()
        _check(engine, small, cx.MODE_SHRED, threads=16)
        st = engine.run_stats()
        assert st["dealt"] == st0["dealt"] and st["slices"] - st0["slices"] >= 3
    finally:
        engine.set_slot_budget(0)
        engine.set_bp_log(False)


def test_submit_collect_pipeline(engine):
    """ccsx_gpu_submit / ccsx_gpu_collect: two batches in flight on the two
    slots, a third submit refused (-3) until one is collected, a ZMW whose
    window outgrows the read cap re-run with full caps inside its collect,
    results in input order and equal to the oracle; a batch larger than a
    slot is refused (-4)."""
    zs1 = [synth(8100 + h, 2000, 8) for h in range(12)]
    zs2 = [synth(8200 + h, 3000, 6) for h in range(9)] + [synth(7500, 12000, 2)]
    want1, _, _ = batch(zs1, cx.MODE_SHRED, 8)
    want2, _, _ = batch(zs2, cx.MODE_SHRED, 8)
    before = engine.rerun_count()
    s1 = engine.submit(zs1)
    s2 = engine.submit(zs2)
    assert s1 != s2
    with pytest.raises(cx.GpuError, match=r"\(-3\)"):
        engine.submit(zs1)
    g1 = engine.collect(s1)
    s3 = engine.submit(zs1[:5])
    g2 = engine.collect(s2)
    g3 = engine.collect(s3)
    assert [g for g, st, _ in g1] == want1 and all(st == 0 for _, st, _ in g1)
    assert [g for g, st, _ in g2] == want2 and all(st == 0 for _, st, _ in g2)
    assert [g for g, _, _ in g3] == want1[:5]
    assert engine.rerun_count() - before >= 1
    engine.set_slot_budget(1 << 20)
    try:
        with pytest.raises(cx.GpuError, match=r"\(-4\)"):
            engine.submit(zs1)
    finally:
        engine.set_slot_budget(0)
    # ccsx_gpu_run still works on the same context afterwards
    assert [g for g, _, _ in engine.run(zs1[:3], cx.MODE_SHRED)] == want1[:3]


class _DeviceHold:
    """Device memory held by this process through the HIP runtime the
    library uses (a stand-in for a neighbouring context or a just-exited
    process whose memory the driver has not cleared yet)."""

    def __init__(self):
        import ctypes as C
        self.C = C
        self.hip = C.CDLL("libamdhip64.so.7" if _has_lib("libamdhip64.so.7") else "libamdhip64.so")
        self.hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.hip.hipFree.argtypes = [C.c_void_p]
        self.hip.hipMemGetInfo.argtypes = [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        self.ptrs = []

    def free_bytes(self) -> int:
        f, t = self.C.c_size_t(0), self.C.c_size_t(0)
        assert self.hip.hipMemGetInfo(self.C.byref(f), self.C.byref(t)) == 0
        return int(f.value)

    def hold(self, nbytes: int) -> None:
        p = self.C.c_void_p()
        assert self.hip.hipMalloc(self.C.byref(p), nbytes) == 0, "hipMalloc of the hold failed"
        self.ptrs.append(p)

    def release(self) -> None:
        while self.ptrs:
            self.hip.hipFree(self.ptrs.pop())


def _has_lib(name: str) -> bool:
    import ctypes
    try:
        ctypes.CDLL(name)
        return True
    except OSError:
        return False


def test_run_with_device_memory_held():
    """ccsx_gpu_run planned its slices from its share of
    the device but staged them against what was free at the time, so a
    context whose neighbour still held memory failed the call ("batch needs
    28.2 GB of device memory, 25.7 GB free").  Now (1) a slice is cut to the
    memory free for its slot, and (2) if not even one ZMW fits, the call
    waits for a neighbour to release memory.  Both with results byte-equal
    to the oracle."""
    import threading
    import time
    zs = _e_zmws(10_700_000, 48)
    eng = cx.Engine(0)
    h = _DeviceHold()
    try:
        tot = sum(eng.zmw_bytes(z) for z in zs)
        x0 = max(eng.zmw_bytes(z) for z in zs)
        # (1) the plan says one slice of all of them; the device has room for ~1/3
        eng.set_slot_budget(tot)
        eng.set_mem_wait(2000)
        h.hold(h.free_bytes() - (tot // 3 + (1 << 30) + (64 << 20)))
        st0 = eng.run_stats()
        _check(eng, zs, cx.MODE_SHRED, threads=16)
        st = eng.run_stats()
        assert st["mem_replans"] - st0["mem_replans"] >= 1, st
        assert st["slices"] - st0["slices"] >= 2, st
        h.release()
        # (2) not even the largest ZMW fits; a neighbour frees its memory 1 s later
        eng.close()
        eng = cx.Engine(0)
        eng.set_mem_wait(30000)
        h.hold(h.free_bytes() - ((1 << 30) + x0 // 2))
        t = threading.Timer(1.0, h.release)
        t.start()
        t0 = time.perf_counter()
        st0 = eng.run_stats()
        _check(eng, zs[:12], cx.MODE_SHRED, threads=16)
        st = eng.run_stats()
        t.join()
        assert st["mem_waits"] - st0["mem_waits"] >= 1, st
        assert time.perf_counter() - t0 >= 0.9
    finally:
        h.release()
        eng.close()


def test_profiling_needs_the_diagnostic_library(engine):
    """the product objects compile the phase counters out, so
    turning them on fails loudly instead of reporting zeros."""
    import os
    if "diag" in os.environ.get("CCSX_LIB", ""):
        pytest.skip("the diagnostic library carries the counters")
    with pytest.raises(cx.GpuError, match="phase counters"):
        engine.set_profiling(True)
