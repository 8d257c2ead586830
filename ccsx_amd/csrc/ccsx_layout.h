// ccsx_layout.h -- per-ZMW HBM workspace layout, shared by the host launcher
// (sizing, offsets) and the device code (addressing).  See DESIGN.md §3.
//
// One ZMW owns one contiguous workspace slab.  Every capacity is derived from
// S = sum of the ZMW's segment lengths (an upper bound on the rows and edges of
// any POA the ZMW can build, SPEC.md §5) and n = number of segments.
#pragma once
#include <stdint.h>

#ifndef CCSX_HD
#if defined(__HIPCC__)
#define CCSX_HD __host__ __device__
#else
#define CCSX_HD
#endif
#endif

namespace ccsx {

constexpr int kW = 128;        // DP band (main.c:849 bandwidth = 128)
constexpr uint32_t kRecRow = kW;  // bytes of a DP row's cell records (8 bits per cell)
// DP rows back whose H / D a row reads from the LDS ring (farther
// predecessors: HBM spill records); per kernel configuration
#ifndef CCSX_RING
#define CCSX_RING 16
#endif
constexpr int kRing = CCSX_RING;
constexpr int kRowW = 272;     // LDS words per ring row of the two-wave DP: H and D, each [4 pad | 128 | 4 pad]
#ifndef CCSX_RINGA
#define CCSX_RINGA 32
#endif
// its ring rows: kRing predecessor rows + 2 blocks of the helpers' lag (a
// power of two: slot = row & 31; with 8-row blocks, measured 55.05 ms vs
// 57.0 for 24 rows and 4-row blocks, tools/gpu_ab.sh r02o)
constexpr int kRingA = CCSX_RINGA;
constexpr int kNeg = -(1 << 29);
// the HBM-read kernel instance's LDS window of the read: two chunks of
// kWinChunk bases as 2-bit codes (ccsx_kernel.hip win_load)
constexpr uint32_t kWinChunk = 8192;
constexpr uint32_t kRdWinBytes = kWinChunk / 2;
constexpr uint32_t kNone = 0xFFFFFFFFu;

// The kernel configurations (ccsx_kernel.hip is compiled once per
// configuration, ccsx_gpu.cpp picks one per slice):
//  * latency: three waves, 8-row lockstep blocks and a 32-row ring -- the
//    shortest per-ZMW chain, 4 workgroups per CU (config B: 1,000 ZMWs in one
//    wave of workgroups);
//  * occupancy: three waves, 4-row blocks and a 24-row ring -- 5 workgroups
//    per CU, for slices larger than the latency configuration keeps resident;
//  * throughput: two waves (one helper), 4-row blocks, a 16-row ring of which
//    the last 8 rows are read back -- up to 8 workgroups per CU, for slices of
//    thousands of ZMWs, where resident ZMWs rather than per-ZMW latency bound
//    the launch;
//  * solo: one wave that also computes the decision bits, an 8-row ring and
//    one traceback buffer -- up to 16 workgroups per CU (~10 KB of LDS each);
//  * solo16: the solo one with an int16 ring (exact for reads of at most
//    16,256 bases), 16-row traceback blocks and 96 VGPRs -- up to 20
//    workgroups per CU (~5.5 KB of LDS each); slices whose pushed reads
//    exceed that, or whose reads live in HBM, run the solo one.
// Each configuration's object reports its own LDS words and threads
// (KCfgInfo), so the host never restates the build flags.
enum KernelCfg : int32_t { kCfgLatency = 0, kCfgOccupancy = 1, kCfgThroughput = 2, kCfgSolo = 3, kCfgSolo16 = 4,
                           kCfgSolo16W = 5, kCfgCount = 6 };
struct KCfgInfo {
    uint32_t lds_fixed_words;  // LDS words before the read buffer
    uint32_t threads;          // workgroup size
    uint32_t ring_rows, ring_back;
    uint32_t waves_per_simd;   // the object's register budget (amdgpu_waves_per_eu)
    uint32_t max_read;         // longest pushed read the object takes on the LDS instance (0: any)
    uint32_t profiling;        // 1: the object carries the per-ZMW phase counters (diagnostic builds)
};

// per-ZMW status codes (0 = ok); any non-zero status is fatal for the batch
enum Status : int32_t {
    kOk = 0,
    kErrRows = 1,      // graph rows exceed rcap
    kErrEdges = 2,     // edges exceed ecap
    kErrMulti = 3,     // (unused: kept so status values stay stable)
    kErrSpill = 4,     // spilled DP rows exceed scap
    kErrInDegree = 5,  // (unused since wide slot records: kept so status values stay stable)
    kErrReadLen = 6,   // pushed read longer than the LDS read buffer (re-run with an uncapped buffer)
    kErrOut = 7,       // CCS longer than the output slab
    kErrTrace = 8,     // traceback did not terminate (internal error)
    kErrBpLog = 9,     // more shredding rounds than the breakpoint log holds (re-run with full caps)
};

enum Mode : int32_t { kShred = 0, kPrimitive = 1, kSinglePoa = 2 };

struct ZmwDesc {
    uint64_t seq_off;   // byte offset of the ZMW's sequence bytes in the seq arena
    uint64_t ws_off;    // byte offset of the workspace slab (256-B aligned)
    uint64_t out_off;   // byte offset of the CCS / consensus output slab
    uint64_t msa_off;   // byte offset of the MSA output slab (kSinglePoa only)
    uint32_t seg0;      // index of the first segment in the segment arrays
    uint32_t n;         // number of segments (pushed reads)
    uint32_t rcap, ecap, lcap, scap, nw;
    uint32_t wcap;      // far-row slot records (rows flagged far: u16 M / D slots per cell)
    uint32_t outcap;    // output slab capacity (bytes)
    uint32_t msacap;    // MSA slab capacity (bytes)
    uint64_t bp_off;    // breakpoint log (-v >= 3): word offset of {rounds, (i, ncols) x bpcap}
    uint32_t bpcap;     // rounds the log holds (0: no log)
    uint32_t pad_;
};

struct ZLayout {
    uint64_t nb0, mem0, poff0, pred0, nb1, mem1, poff1, pred1;
    uint64_t rmeta, spf, sslot, codes, dsl, spill, rrec;
    uint64_t ev, tgt, ipt, iinf, ifix, cnt, fixf, addp, cntn;
    uint64_t colof, cons, cmask, colrow, rdoff, rdlen, rfirst, rlast, rfc, rlc;
    uint64_t ext;  // rarely used regions (zext): kept as one offset to spare registers
    uint64_t total;
};

CCSX_HD inline uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// The extension regions, in order (offsets relative to ZLayout::ext):
//  * the far rows' slot records (rows with more than four predecessors or one
//    beyond the DP ring, whose 8-bit cell records carry no tags): per cell the
//    M and D predecessor slots, u16 each, 512 B per far row, taken in the
//    order the DP meets them (the row's index in its tag-plane row, word 0);
//  * the HBM-read kernel instance (reads beyond the LDS read buffer): the read
//    as 2-bit codes and the shredding cursors.
enum ZExt { kExtWtag = 0, kExtRdbuf, kExtPos, kExtEnd };

CCSX_HD inline uint64_t zext_size(const ZmwDesc &d, int which)
{
    switch (which) {
    case kExtWtag: return uint64_t(d.wcap) * kW * 4;
    case kExtRdbuf: return uint64_t((d.lcap + 15) / 16 + 2) * 4;
    default: return uint64_t(d.n) * 4;
    }
}

// offset of extension region `which` from ZLayout::ext (= bytes of the ones before it)
CCSX_HD inline uint64_t zext_bytes(const ZmwDesc &d, int which)
{
    uint64_t o = 0;
    for (int i = 0; i < which; ++i) o = align256(o + zext_size(d, i));
    return o;
}

CCSX_HD inline void zlayout(ZLayout &L, const ZmwDesc &d)
{
    uint64_t o = 0;
    auto take = [&o](uint64_t bytes) {
        uint64_t r = o;
        o = align256(o + bytes);
        return r;
    };
    L.nb0 = take(d.rcap);
    L.mem0 = take(uint64_t(d.rcap) * d.nw * 8);
    L.poff0 = take(uint64_t(d.rcap + 1) * 4);
    L.pred0 = take(uint64_t(d.ecap) * 4);
    L.nb1 = take(d.rcap);
    L.mem1 = take(uint64_t(d.rcap) * d.nw * 8);
    L.poff1 = take(uint64_t(d.rcap + 1) * 4);
    L.pred1 = take(uint64_t(d.ecap) * 4);
    L.rmeta = take(uint64_t(d.rcap) * 4);              // per DP row: band offset | far flag << 31
    L.spf = take(d.rcap);                              // per row: needed beyond the LDS ring
    L.sslot = take(uint64_t(d.rcap) * 4);              // per spilled row: its spill record
    L.codes = take(uint64_t(d.rcap) * kRecRow);        // cell records, 8 bits/cell, 128 B/row
    L.dsl = take(uint64_t(d.rcap) * kRecRow);          // per row: tag plane, escape distances (far rows: word 0 = far record)
    L.spill = take(uint64_t(d.scap) * (kW * 8 + 16));  // spilled rows: H, D, band offset, row-max key
    L.rrec = take(uint64_t(d.rcap) * 8);               // per row: {info, the predecessors' tag bytes} for the DP prefetch
    L.ev = take(uint64_t(d.lcap) * 4);
    L.tgt = take(uint64_t(d.lcap) * 4);
    L.ipt = take(uint64_t(d.lcap) * 4);
    L.iinf = take(d.lcap);
    L.ifix = take(uint64_t(d.lcap) * 4);
    L.cnt = take(uint64_t(d.rcap + 1) * 4);
    L.fixf = take(d.rcap + 1);
    L.addp = take(uint64_t(d.rcap) * 4);
    L.cntn = take(uint64_t(d.rcap + 1) * 4);
    L.colof = take(uint64_t(d.rcap) * 4);
    L.cons = take(d.rcap);
    L.cmask = take(uint64_t(d.rcap) * d.nw * 8);
    L.colrow = take(uint64_t(d.rcap + 1) * 4);
    L.rdoff = take(uint64_t(d.n) * 4);
    L.rdlen = take(uint64_t(d.n) * 4);
    L.rfirst = take(uint64_t(d.n) * 4);
    L.rlast = take(uint64_t(d.n) * 4);
    L.rfc = take(uint64_t(d.n) * 4);
    L.rlc = take(uint64_t(d.n) * 4);
    L.ext = take(zext_bytes(d, kExtEnd));
    L.total = o;
}

// Capacities for a ZMW with segment lengths summing to S, longest segment
// lmax, n segments.  Full caps are exact upper bounds for rows and edges
// (SPEC.md §5: each read base creates at most one node and one in-edge).
// Tight caps (the default launch) size the DP/graph arrays for the graphs a
// ZMW really builds -- rows ~ window length x (1 + error rate x reads) -- at
// a fraction of the memory; every cap is checked on the device (kErrRows,
// kErrEdges, kErrSpill) and ccsx_gpu_run re-runs a ZMW that hits
// one with full caps.  tight_rows overrides the tight row cap (tests).
// shred_win: the ZMW runs the shredded loop (main.c:541-641) with pushed
// windows of at most shred_win bases (the LDS read buffer of a tight-cap
// slice; a longer window fails the ZMW and it is re-run uncapped), whose POAs
// are of 2 kb windows (+2 kb per missed breakpoint) rather than whole
// segments, so the tight row cap follows the window, not the segment (rows ~
// window x (1 + ~0.07 reads): 3 x 4,096 + 4,096 covers 4 kb windows of up to
// ~40 reads).  0: not shredded.  The output slab: S + 16 bytes bound any
// consensus (one base per column, columns <= S); tight caps hold 2 x the
// longest segment + 1,024 (a CCS is about one insert long; kErrOut re-runs
// the ZMW uncapped), tight_out overriding (tests); tight_far overrides the
// far slot records' tight row count (tests).
CCSX_HD inline void zcaps(ZmwDesc &d, uint64_t S, uint32_t lmax, uint32_t n, bool full = true,
                          uint32_t tight_rows = 0, uint32_t shred_win = 0, uint32_t tight_out = 0,
                          uint32_t tight_far = 0)
{
    d.n = n;
    d.rcap = uint32_t(S + 16);
    d.ecap = uint32_t(S + n + 16);
    d.scap = d.rcap / 4 + 64;
    if (!full) {
        const uint64_t lw = shred_win && lmax > shred_win ? shred_win : lmax;
        uint64_t r = tight_rows ? tight_rows : 3ull * lw + 4096;
        if (r < S) {
            d.rcap = uint32_t(r + 16);
            d.ecap = 2 * d.rcap;
        }
        d.scap = d.rcap / 32 + 64;
    }
    d.lcap = lmax + 16;
    d.nw = (n + 63) / 64 ? (n + 63) / 64 : 1;
    // far rows' slot records: every row (full caps), else 1 in 16 (config E
    // 0.02 %, D 0.87 % of DP rows are far); more fail the ZMW with kErrSpill
    // and it is re-run with full caps
    d.wcap = full ? d.rcap : tight_far ? tight_far : d.rcap / 16 + 64;
    d.outcap = uint32_t(S + 16);
    if (!full) {
        const uint64_t oc = tight_out ? tight_out : 2ull * lmax + 1024;
        if (oc < d.outcap) d.outcap = uint32_t(oc);
    }
}

struct KArgs {
    const uint8_t *seq;
    const uint32_t *soff;  // segment offset relative to the ZMW's seq_off
    const uint32_t *slen;
    const ZmwDesc *desc;
    const uint32_t *order;  // workgroup -> ZMW index: most expensive first (host-sorted)
    uint8_t *ws;
    uint8_t *out;
    uint8_t *msa;
    uint32_t *out_len;
    uint32_t *ncols;
    int32_t *status;
    unsigned long long *cells;
    int32_t mode;
    uint32_t nzmw;
    uint32_t lds_read_words;    // 0: the HBM-read kernel instance (read and cursors in the workspace)
    uint32_t lds_nmax;
    unsigned long long *prof;  // optional: kProfSlots shader-clock counters per ZMW (diagnostics)
    uint32_t *bplog;           // optional: per-round breakpoint log (main.c:619-620, ZmwDesc::bp_off)
};

// phase counters written when KArgs::prof != nullptr
enum ProfSlot { kPfTotal = 0, kPfLoad, kPfDp, kPfTrace, kPfMerge, kPfColumns, kPfShred, kPfRows,
                kPfRowA, kPfRowB, kPfRowC, kPfRowD, kPfRowE, kPfFlush, kPfSpare0, kPfSpare1,
                // two-wave DP (diagnostic build): wave 0 / wave 1 busy and barrier-wait
                // cycles, rows through the two-wave and the single-wave DP
                kPfAbusy, kPfAwait, kPfBbusy, kPfBwait, kPfTwRows, kPfSwRows, kPfSpare2, kPfSpare3,
                // traceback (diagnostic build): cycles of probe steps, plain MPRED steps,
                // D / I runs, block switches; number of block switches
                kPfTbProbe, kPfTbStep, kPfTbDI, kPfTbSwitch, kPfTbNsw,
                // placement: HW_ID | XCC_ID << 32 of waves 0, 1, 2; start / end on
                // the constant-rate s_memrealtime clock
                kPfHw0, kPfHw1, kPfHw2, kPfStartRt, kPfEndRt,
                // wave 0 fast rows (diagnostic build): head, body to the scan,
                // scan to end; number of fast rows
                kPfAHead, kPfABody, kPfATail, kPfAFast,
                // wave 0 cold rows by kind (far, chain moved 0..2, one
                // predecessor, two, other; spill rows; rows on the register
                // path for predecessors r-1 / r-2): cycles, then counts
                kPfCold0, kPfCold1, kPfCold2, kPfCold3, kPfCold4, kPfCold5, kPfCold6,
                kPfColdN0, kPfColdN1, kPfColdN2, kPfColdN3, kPfColdN4, kPfColdN5, kPfColdN6,
                // traceback (diagnostic build): insertion steps / runs, deletion steps / runs
                kPfTbIsteps, kPfTbIruns, kPfTbDsteps, kPfTbDruns, kProfSlots };

}  // namespace ccsx
