// ccsx_kernel.hip -- MI355X (gfx950) consensus hot path of ccsx.
//
// One workgroup of three 64-lane waves owns one ZMW for the whole of ccs_for2
// (main.c:510-647, shredded mode) or ccs_for (main.c:455-508, -P): the window
// loop, every bspoa call (beg/push/end/tidy_msa, SPEC.md §2-§6), the
// breakpoint scan and the CCS emission all run on the device.  The host only
// runs ccs_prepare and hands over strand-normalised segments.
//
// DP (SPEC.md §3): wave 0 runs the row recurrence -- per graph row W = 128
// read positions, two adjacent cells per lane, band placement from the
// predecessor's row maximum, the in-row insertion prefix max and the row-max
// key as DPP max-scans -- and writes each row's H and D to an LDS ring of
// kRingA rows, padded by 4 words of -inf per side so any band shift in
// [-3, 4] is three immediate-offset reads.  Rows needed more than kRing rows
// later are spilled to HBM.  Helper waves 1 and 2 follow one lockstep block
// of kBlkAB rows behind, recompute each cell's decision bits from the ring
// and store 8-bit cell records (code | D-ext | I-ext | M tag | D tag) to HBM,
// 128 B per row, rotated per row for the traceback's LDS banks (row_record).
// Traceback (SPEC.md §4) walks those records on wave 0 from 32-row blocks
// LDS-DMA'd double-buffered; merge (§5) and the column counts (§6) run on all
// three waves.  The same source builds four configurations (ccsx_layout.h
// KernelCfg): three-wave latency / occupancy ones, a two-wave throughput one
// (one helper) and a one-wave solo one (dp_solo: the wave computes the
// decision bits itself, an 8-row ring, one traceback buffer; ~15 ZMWs per CU
// for slices of many thousands of ZMWs).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ccsx_layout.h"

// One compilation per kernel configuration (ccsx_layout.h KernelCfg): the
// build passes CCSX_RINGA / CCSX_BLK and names the configuration's namespace
// and launcher, so the two objects link into one library side by side.
#ifndef CCSX_KCFG
#define CCSX_KCFG lat
#endif
#ifndef CCSX_LAUNCH
#define CCSX_LAUNCH ccsx_launch_zmw_lat
#endif
#ifndef CCSX_INFO
#define CCSX_INFO ccsx_kcfg_info_lat
#endif

namespace ccsx {
namespace CCSX_KCFG {

#ifndef CCSX_BLK
#define CCSX_BLK 8
#endif
// helper waves per workgroup: 2 (latency / occupancy configurations), 1
// (throughput configuration: two-wave workgroups, twice the resident ZMWs) or
// 0 (solo configuration: one wave computes the decision bits too, dp_solo)
#ifndef CCSX_HELPERS
#define CCSX_HELPERS 2
#endif
constexpr int kHelpers = CCSX_HELPERS;

constexpr int kO = -3, kE = -2, kMs = 2, kXs = -6;  // main.c:842-847
enum { HC_MPRED = 0, HC_MSRC = 1, HC_DEL = 2, HC_INS = 3 };
enum : uint32_t { EV_ALN = 0u, EV_INS = 1u, EV_LEAD = 2u };
constexpr uint32_t kNewBit = 0x80000000u;



// ----------------------------------------------------------------------------
// wave primitives (gfx9 DPP: row_shr, row_bcast15/31, wave_shr1)
// ----------------------------------------------------------------------------
template <int CTRL, int RM = 0xF, int BM = 0xF>
__device__ __forceinline__ int dpp(int old, int v)
{
    return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, BM, false);
}

// inclusive max-scan over the 64 lanes: six DPP max steps (a lane whose DPP
// source is out of range, or whose row is masked, keeps its own value).  Each
// step is max(v, dpp(INT_MIN, v)): with the max's identity as the DPP mov's
// old value the compiler folds the mov into one v_max_i32_dpp and, unlike an
// asm block, fills the VALU-write -> DPP-read wait states with independent
// work of the row instead of s_nop (a hand-written asm
// scan with s_nop measured slower).
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ int dpp_max(int v)
{
    return max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, CTRL, RM, 0xF, false));
}

__device__ __forceinline__ int wave_incl_max(int v)
{
    v = dpp_max<0x111>(v);
    v = dpp_max<0x112>(v);
    v = dpp_max<0x114>(v);
    v = dpp_max<0x118>(v);
    v = dpp_max<0x142, 0xA>(v);
    return dpp_max<0x143, 0xC>(v);
}

// two independent inclusive max-scans (interleaved by the scheduler)
__device__ __forceinline__ void wave_incl_max2(int &a, int &b)
{
    a = wave_incl_max(a);
    b = wave_incl_max(b);
}

__device__ __forceinline__ int wave_incl_sum(int v)
{
    v += dpp<0x111>(0, v);
    v += dpp<0x112>(0, v);
    v += dpp<0x114>(0, v);
    v += dpp<0x118>(0, v);
    v += dpp<0x142, 0xA>(0, v);
    v += dpp<0x143, 0xC>(0, v);
    return v;
}

// lane within the wave; the workgroup is three waves (wave 0 runs every
// phase, waves 1 and 2 are the DP helpers, see dp_align)
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Visibility point for single-wave phases: LDS and global accesses of the
// wave before it are complete (the workgroup barrier is reserved for the
// DP protocol, which every wave must enter the same number of times)
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); }

// Workgroup barrier for the DP's block handoff: only LDS must be complete
// (__syncthreads would also drain the helpers' in-flight HBM stores)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int wave_shr1(int old, int v) { return dpp<0x138>(old, v); }  // lane l <- l-1

__device__ __forceinline__ int wave_shl1(int old, int v) { return dpp<0x130>(old, v); }  // lane l <- l+1

// K a + C and K a for |a| < 2^23 (v_mad_i32_i24 / v_mul_i32_i24, full rate;
// the compiler cannot see the operand's range across the DP's basic blocks
// and emits the quarter-rate v_mul_lo_u32).  K, C inline constants (-16..64)
template <int K, int C>
__device__ __forceinline__ int32_t mad24(int32_t a)
{
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(K), "i"(C));
    return r;
}
template <int K>
__device__ __forceinline__ int32_t mul24(int32_t a)
{
    int32_t r;
    asm("v_mul_i32_i24 %0, %2, %1" : "=v"(r) : "v"(a), "i"(K));
    return r;
}

// lane l <- l-1, lane 0 <- 0 (the DPP bound control: no old-value register)
__device__ __forceinline__ int wave_shr1_z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

// lane `l` of v <- the uniform value x (v_writelane_b32; l and x in SGPRs)
__device__ __forceinline__ int writelane(int v, int x, int l)
{
    // gfx9 VOP3 reads one SGPR: the lane select goes through m0, given to the
    // compiler as an operand so it keeps m0's other uses (LDS DMA) intact
    asm volatile("v_writelane_b32 %0, %1, %2"
                 : "+v"(v)
                 : "s"(__builtin_amdgcn_readfirstlane(x)), "{m0}"(__builtin_amdgcn_readfirstlane(l)));
    return v;
}


__device__ __forceinline__ int wave_max(int v) { return __builtin_amdgcn_readlane(wave_incl_max(v), 63); }

__device__ __forceinline__ int wave_min(int v) { return -wave_max(-v); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <class T>
__device__ __forceinline__ T uni(T v)
{
    return (T)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ uint32_t enc_base(uint32_t c)
{
    // SPEC.md §1: A/a=0 C/c=1 G/g=2 T/t/U/u=3, anything else 0
    c |= 0x20u;
    return c == 'c' ? 1u : c == 'g' ? 2u : (c == 't' || c == 'u') ? 3u : 0u;
}

// ----------------------------------------------------------------------------
// per-ZMW state
// ----------------------------------------------------------------------------
// Per-ZMW phase counters (KArgs::prof): only the profiling builds carry them
// (-DCCSX_PROF or -DCCSX_TB_COUNT, and the diagnostic library's -DCCSX_DP_STAMPS).  In the
// product they were ~10 live 64-bit counters for the whole kernel -- SGPRs
// the DP and merge spilled for (tools/spill_attr.py); there every counter is
// a sink and KArgs::prof receives zeros.
#if defined(CCSX_PROF) || defined(CCSX_DP_STAMPS) || defined(CCSX_TB_COUNT)
constexpr bool kProfiling = true;
typedef unsigned long long Prof[kProfSlots];
#else
constexpr bool kProfiling = false;
struct PfSink {
    template <class T>
    __device__ PfSink &operator+=(T) { return *this; }
    template <class T>
    __device__ PfSink &operator=(T) { return *this; }
    __device__ operator unsigned long long() const { return 0ull; }
};
struct Prof {
    __device__ PfSink operator[](int) const { return PfSink{}; }
};
#endif

struct Z {
    ZmwDesc d;
    ZLayout L;
    uint8_t *ws;
    const uint8_t *seq;
    int32_t *lds;        // workgroup LDS: DP ring (kRingA rows x kRowW words), offsets, job, read
    uint8_t *rd;         // read as 2-bit codes: byte b = code(4b) | code(4b+1) << 2 | code(4b+2) << 4 | code(4b+3) << 6
    // HBM-read instance: an LDS window of the read (rd_window), two chunks of
    // kWinChunk bases resident, the first one wa (wave 0's view)
    uint8_t *win;
    bool hbm;
    uint32_t wa, rdbytes;
    bool wpend;  // wave 0: chunk wa + 1 is to be loaded at the next block's start
    uint32_t *pos;       // shredding cursors
    uint32_t rdcap;      // bases that fit in rd
    int cur;
    uint32_t R, E;
    int32_t status;
    uint32_t nfar;       // DP: this wave's next far slot record (helper h: h, h + 2, ...)
    unsigned long long cells;
    Prof pf;
};

__device__ __forceinline__ unsigned long long stamp() { return __builtin_amdgcn_s_memtime(); }
// the phase clock of the profiling builds; 0 in the product (no s_memtime)
__device__ __forceinline__ unsigned long long pstamp() { return kProfiling ? stamp() : 0ull; }
__device__ __forceinline__ unsigned long long prealtime() { return kProfiling ? __builtin_amdgcn_s_memrealtime() : 0ull; }

// Raw buffer access: lanes whose byte offset is >= `bytes` are discarded
// (stores) or read 0 (loads) by the hardware, so a masked store is still one
// unconditionally issued instruction -- the compiler's vmcnt bookkeeping stays
// exact and a later wait on a prefetch never waits on these stores.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void *p, uint32_t bytes)
{
    // every field through readfirstlane: a descriptor in VGPRs would make the
    // compiler wrap each access in a waterfall loop
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(u), 0,
                                             __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}

// Diagnostic build only (-DCCSX_DP_STAMPS, libccsx_amd_diag.so): shader-clock
// stamps between the phases of one DP row; never compiled into the product.
#ifdef CCSX_DP_STAMPS
#define DP_STAMP(slot)                                                                      \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        unsigned long long t_;                                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        z.pf[slot] += t_ - t_prev;                                                          \
        t_prev = t_;                                                                        \
    } while (0)
// a shader-clock read whose result is only waited for later (ROW_STAMPS_END)
#define ROW_STAMP(var)                                      \
    do {                                                    \
        __builtin_amdgcn_sched_barrier(0);                  \
        asm volatile("s_memtime %0" : "=s"(var)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                  \
    } while (0)
#else
#define DP_STAMP(slot) \
    do {               \
    } while (0)
#endif
// traceback step counters (and block-switch cycles): the diagnostic build,
// or a product build with -DCCSX_TB_COUNT (tools/phase_prof.py)
#if defined(CCSX_DP_STAMPS) || defined(CCSX_TB_COUNT)
#define CCSX_TB_COUNTING 1
#endif

template <class T>
__device__ __forceinline__ T *P(const Z &z, uint64_t off)
{
    return reinterpret_cast<T *>(z.ws + off);
}

// an extension region (ccsx_layout.h zext), offsets computed where used
template <class T>
__device__ __forceinline__ T *PX(const Z &z, int which)
{
    return reinterpret_cast<T *>(z.ws + z.L.ext + zext_bytes(z.d, which));
}

// graph buffer b (0/1) of the double-buffered rebuild (SPEC.md §5)
__device__ __forceinline__ uint8_t *G_nb(const Z &z, int b) { return P<uint8_t>(z, b ? z.L.nb1 : z.L.nb0); }
__device__ __forceinline__ uint64_t *G_mem(const Z &z, int b) { return P<uint64_t>(z, b ? z.L.mem1 : z.L.mem0); }
__device__ __forceinline__ uint32_t *G_poff(const Z &z, int b) { return P<uint32_t>(z, b ? z.L.poff1 : z.L.poff0); }
__device__ __forceinline__ uint32_t *G_pred(const Z &z, int b) { return P<uint32_t>(z, b ? z.L.pred1 : z.L.pred0); }

__device__ __forceinline__ uint32_t rcode(const Z &z, uint32_t j) { return ((uint32_t)z.rd[j >> 2] >> ((j & 3u) * 2u)) & 3u; }

// ----------------------------------------------------------------------------
// The HBM-read instance's read window.  Reads beyond the LDS read buffer live
// in the workspace; a DP row reads the bytes of its band [off, off + 130)
// once per row (wave 0 a row ahead, each helper for its own rows), which from
// HBM is a global round trip on every row.  So two consecutive chunks of
// kWinChunk bases (chunk c in ring half c & 1) are kept in LDS; when wave 0's
// band enters the upper chunk at the end of a block it publishes the slide
// (job word wa << 1 | 1) and loads the next chunk at the start of its next
// block, over the half that held the chunk below.  During that period the
// helpers (one block behind) trust only the kept chunk; a row outside what
// its wave may trust reads HBM (rare: a band far behind the diagonal).
// ----------------------------------------------------------------------------
constexpr uint32_t kWinBytesMask = kRdWinBytes - 1;

__device__ __forceinline__ void win_load(const Z &z, uint32_t c)
{
    const uint32_t lane = lane_id();
    const auto rs = brsrc(z.rd, z.rdbytes);  // beyond the buffer: zeros
#pragma unroll
    for (uint32_t k = 0; k < kWinChunk / 4 / 1024; ++k) {
        const uint32_t b = c * (kWinChunk / 4) + k * 1024 + lane * 16;
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, b, 0, 0);
        *reinterpret_cast<v4u *>(z.win + (b & kWinBytesMask)) = v;
    }
    wsync();
}

// bases [off, off + 136) within chunks [c0, c0 + nc) (uniform): every byte
// a row's rd_win16 reads
__device__ __forceinline__ bool win_has(uint32_t c0, uint32_t nc, int32_t off)
{
    return (uint32_t)off >= c0 * kWinChunk && (uint32_t)off + 136u <= (c0 + nc) * kWinChunk;
}

// ----------------------------------------------------------------------------
// push: stage read k (ASCII in HBM) into LDS as 2-bit codes, four per byte
// (word w = positions 16 w .. 16 w + 15): 4,096 bases in 1 KiB, so the solo
// object's workgroup fits 16 per CU; a DP row reads two bytes per lane
// (rd_win16)
// ----------------------------------------------------------------------------
__device__ __forceinline__ void stage_read(const Z &z, const uint8_t *src, uint32_t m, uint32_t tid, uint32_t T)
{
    const uint32_t nwd = (m + 15) / 16 + 1;
    uint32_t *dst = reinterpret_cast<uint32_t *>(z.rd);
    for (uint32_t w = tid; w < nwd; w += T) {
        uint32_t x = 0;
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b) {
            const uint32_t j = w * 16 + b;
            x |= (j < m ? enc_base(src[j]) : 0u) << (2 * b);
        }
        dst[w] = x;
    }
}

__device__ __forceinline__ void load_read(Z &z, const uint8_t *src, uint32_t m)
{
    stage_read(z, src, m, lane_id(), 64);
    wsync();
}

// The DP ring's cells: int32, or (CCSX_RING16, the solo16 object) int16 --
// absolute values saturated to int16, exact for reads of at most
// kRing16MaxRead bases: every real H / D value of such a DP lies in
// [-2m - 12, 2m] (the read-prefix source term bounds it below, two points per
// aligned base above), while the -inf class (the kNeg / kNegH sentinels and
// what they propagate) saturates to -32768, below every real value, so every
// max the recurrence takes and every tie it breaks between real values is
// unchanged; a -inf value never wins against the always-real source term of
// M, so its tags and ext bits are never followed
#ifdef CCSX_RING16
typedef int16_t RingT;
#else
typedef int32_t RingT;
#endif
// (16,256 rather than 16,376: round 5's packed-row variant, commit bf58425,
// also held X = H' + 2t, t < 128, as int16 -- at most 2m + 254)
constexpr uint32_t kRing16MaxRead = 16256;

// a value as the ring stores it (-inf class: -32768 in the int16 ring)
__device__ __forceinline__ RingT ring_val(int32_t v) { return sizeof(RingT) == 2 ? (RingT)max(v, -32768) : (RingT)v; }
// the lane's two adjacent cells (row points at cell 2 lane) of H or D
__device__ __forceinline__ void ring_store2(RingT *row, int32_t a, int32_t b)
{
#ifdef CCSX_RING16
    *reinterpret_cast<decltype(__builtin_amdgcn_cvt_pk_i16(a, b)) *>(row) = __builtin_amdgcn_cvt_pk_i16(a, b);
#else
    *reinterpret_cast<int2 *>(row) = make_int2(a, b);
#endif
}

// LDS layout of a workgroup (int32 words)
// (the solo object has no helpers: no diagnostic slots or band-offset ring,
// which keeps a config-D workgroup within 10 KB, 16 per CU)
constexpr int kRingWords = kRingA * kRowW * (int)sizeof(RingT) / 4;  // LDS words of the DP ring area
constexpr int kLdsRing = 0;                              // kRingA DP rows x kRowW cells (traceback: its blocks)
constexpr int kLdsDiag = kLdsRing + kRingWords;          // 32: helpers' diagnostic counters at exit
constexpr int kLdsOffRing = kLdsDiag + (kHelpers ? 32 : 0);  // 64: band offset of DP row q at q & 63
constexpr int kLdsJob = kLdsOffRing + (kHelpers ? 64 : 0);   // 16: DP job / results
constexpr int kLdsFixed = kLdsJob + 16;                  // then: the read (nibble pairs), shredding cursors


// lane's 16-bit window of the read for a row at band offset `off`: the codes
// of positions P .. P + 7, P = (off + 2 lane) & ~3 -- bytes (off + 2 lane) >> 2
// and the next, from the LDS buffer, or the window / HBM on the HBM-read
// instance (`inwin`: the wave may trust the window for this row).  The
// lane's cells t = 2 lane, 2 lane + 1 of a row at offset off + d (0 <= d <= 3)
// are win_codes(window, off, d).  The LDS buffer and the window both start
// at word kLdsFixed of the dynamic LDS, which starts at address 0 (the
// kernel declares no static __shared__): read through an LDS pointer of that
// constant address, the buffer's base folds into the ds_read's offset field
// (through z.rd the compiler kept a per-row `v_add 0` for the base).  The two
// bytes as two ds_read_u8: one unaligned ds_read_u16 measured 0.4 % slower
// (r04zd).
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
__device__ __forceinline__ uint32_t rd_win16(const Z &z, int32_t off, bool inwin)
{
    const uint32_t b = ((uint32_t)off + 2u * lane_id()) >> 2;
    const lds_u8 *lb = (const lds_u8 *)(uintptr_t)(kLdsFixed * 4);
    if (!z.hbm) return (uint32_t)lb[b] | (uint32_t)lb[b + 1] << 8;
    if (inwin) return (uint32_t)lb[b & kWinBytesMask] | (uint32_t)lb[(b + 1) & kWinBytesMask] << 8;
    return (uint32_t)z.rd[b] | (uint32_t)z.rd[b + 1] << 8;
}

// the codes of read positions off + d + 2 lane (bits 0-1) and the next (bits
// 2-3) from the window rd_win16(z, off) loaded
__device__ __forceinline__ uint32_t win_codes(uint32_t win, int32_t off, int32_t d)
{
    return win >> ((((uint32_t)off + 2u * lane_id()) & 3u) * 2u + 2u * (uint32_t)d);
}

// The 8-bit cell record (row_record): code (bits 0-1) | D-ext (2) | I-ext (3)
// | M tag (4-6) | D tag (7).  M tag: -d as 3-bit two's complement for the
// predecessor d = 1..4 rows back, else (0..3) an escape.  Rows of one or two
// predecessors (not far) carry their distances in the row meta (rmeta_word):
// the D tag is the predecessor's slot, an M escape's low bit too.  Rows of 3-4
// predecessors: D tag 1 = row r - 1, else an escape; an escape's distance
// d - 1 sits in the row's tag plane (D: 4 bits per cell; M too where the ring
// is longer than 8 rows -- on the others an M escape is (-d) & 7 = 8 - d for
// d = 5..8).  Rows flagged far carry neither: their slots go to a far slot
// record.  The tag byte of a
// predecessor d rows back (what pred_fold keeps per cell; d <= kRing on rows
// not flagged far): M tag << 4 | D tag << 7 | (d - 1).  merge computes them
// into the DP's row records (RowPre::dpk): in the DP the arithmetic took ~9
// scalar instructions per predecessor, config D +4 % on the scalar unit
// (r06m).  Traceback: 98.8 % of config-E predecessor moves go 1-3 rows back,
// 0.5 % 4-8 (tools/row_kinds.py --tb).
__device__ __forceinline__ uint32_t tagb(uint32_t d)
{
    // d = 8, 1, 2, 3 | 4, 5, 6, 7 by d & 3; beyond 8 rows: M escape 0, D escape
    return d > 8u ? d - 1u : ((d & 4u) ? 0x16253443u : 0x5261F007u) >> ((d & 3u) * 8u);
}
// a row of one or two predecessors: the D tag (and an M escape's low bit) is the slot
__device__ __forceinline__ uint32_t tagb2(uint32_t d, uint32_t s)
{
    const uint32_t t = tagb(d) & 0x7Fu;
    return (t & 0x70u) < 0x40u ? (t & 0x0Fu) | (s << 7) | (s << 4) : t | (s << 7);
}
constexpr uint32_t kTagPrev = 0x70u;  // tagb2(1, 0): the previous row, slot 0
static_assert(kRing <= 16, "tag bytes hold distances up to 16");

// per lane: row r0+lane's info and the tag bytes of its first four
// predecessors (merge writes them: the distance d - 1 in the low nibble, so a
// row without the far flag -- every predecessor within kRing rows, at most
// four -- finds its predecessors too; two VGPRs per 64-row window)
struct RowPre {
    uint32_t info, dpk;
};
// row info bits: base (0-1) | spill (2: a successor lies > kRing rows ahead)
// | chain (3: the only predecessor is the previous row) | far (4: a
// predecessor lies > kRing rows back or there are > 4) | np << 8
constexpr uint32_t kInfoSpill = 4u, kInfoChain = 8u, kInfoFar = 16u;

// tag byte k (< 4) of row r = r0 + li (bits above the byte: the next slots')
__device__ __forceinline__ uint32_t row_tag(const RowPre &W, int li, int k)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)W.dpk, li) >> (8 * k);
}

// predecessor k (< 4) of row r = r0 + li of a non-far row, from the window
__device__ __forceinline__ uint32_t row_pred(const RowPre &W, uint32_t r, int li, int k)
{
    return r - 1u - (row_tag(W, li, k) & 15u);
}

// the row meta word the traceback stages with each record block: band offset
// (< 2^22) | for a row of one or two predecessors (not far) the distances - 1
// of slots 0 / 1 << 22 / 26 and bit 30 | far << 31
__device__ __forceinline__ uint32_t rmeta_word(uint32_t off, uint32_t info, uint32_t dpk)
{
    const bool far = (info & kInfoFar) != 0u;
    const bool two = !far && (info >> 8) <= 2u;
    return off | (far ? 0x80000000u : 0u) | (two ? 0x40000000u | ((dpk & 15u) << 22) | (((dpk >> 8) & 15u) << 26) : 0u);
}
constexpr uint32_t kMetaOff = 0x3FFFFFu;

// the DP's row records {info, tag bytes} (written by merge): coalesced, no
// dependent loads
__device__ __forceinline__ void prefetch_recs(const Z &z, uint32_t r0, RowPre &o)
{
    const uint32_t n = r0 < z.R ? z.R - r0 : 0u;
    const uint32_t sp = __builtin_amdgcn_raw_buffer_load_b8(brsrc(P<const uint8_t>(z, z.L.spf) + r0, n), lane_id(), 0, 0);
    const v2u q = __builtin_amdgcn_raw_buffer_load_b64(brsrc(P<const uint2>(z, z.L.rrec) + r0, n * 8), lane_id() * 8, 0, 0);
    o.info = q.x | (sp ? kInfoSpill : 0u), o.dpk = q.y;
}

// ----------------------------------------------------------------------------
// SPEC.md §3 on three waves.  One wave alone issues about one instruction per
// 6 clocks whatever else runs on its SIMD (tools/ubench/issue.hip), and a
// batch of ~1,000 ZMWs puts ~1 ZMW on each of the 1,024 SIMDs, so the DP of
// one ZMW is split across the three waves of its workgroup:
//  * wave 0 ("A") runs the recurrence: band placement, M / D / H', the
//    insertion prefix-max and row-max scans, H; it writes each row's H and D
//    to an LDS ring of kRingA rows, the exclusive prefix max (Pex) of the
//    row's insertion scan and the row's band offset;
//  * waves 1 and 2 (the helpers) follow one block of kBlkAB = 8 rows behind
//    (wave 1 + h takes the rows of parity h): from the ring they
//    recompute every cell's decision bits (SPEC.md §3.2-§3.4: MPRED / MSRC /
//    DEL / INS, D-ext, I-ext), the predecessor slots of multi-predecessor
//    rows and the free-end candidates, and store the row's records to HBM.
// The waves meet at one workgroup barrier per block.  Everything else in the
// kernel runs on wave 0 alone; the helpers wait in dp_helper for the next DP.
//
// Value-preserving choices (the oracle is followed bit for bit):
//  * ring row = [pad4 | H x 128 | pad4][pad4 | D x 128 | pad4]; pads hold
//    kNegH = kNeg + 5 (H) and kNeg (D), so a predecessor at any band shift in
//    [-3, 4] is three DS reads with immediate offsets, and
//    D = max(H + O + E, D + E) needs no kNeg floor (an out-of-band H then
//    contributes exactly kNeg, which never wins a strict > update);
//  * row max and its first position come from one max-scan of
//    key = H' << 7 | (127 - t) (valid H' lies in (-2^24, 2^24) for m < 2^22),
//    and max H == max H' at the same first position (an insertion value is
//    always below the H' it extends);
//  * free-end candidates are tracked on H' for the same reason.
// ----------------------------------------------------------------------------
// Cell records (8 bits, cell t of row r) sit in the row's 128 B at byte (t +
// tb_rot(r)) & 127: each row is rotated by one word per row of its 32-row
// traceback block, so the traceback's window fill -- 32 lanes reading the
// same column of 32 consecutive rows -- spreads over the LDS banks instead of
// hitting one (a 128 B pitch is a multiple of the bank width).
__device__ __forceinline__ uint32_t tb_rot(uint32_t r) { return (r & 31u) * 4u; }

constexpr int kHc = 4, kDc = 140;  // word of cell 0 of H / D in a ring row
constexpr int32_t kNegH = kNeg - kO - kE;
constexpr int kBlkAB = CCSX_BLK;  // rows per lockstep block: helper h takes rows r0 + h, r0 + h + 2, ...
static_assert(kHelpers >= 0 && kHelpers <= 2, "zero, one or two helper waves");
constexpr int kBlockThreads = 64 * (1 + kHelpers);
constexpr int kHelperStep = kHelpers ? kHelpers : 1;
static_assert(kBlkAB % kHelperStep == 0, "each helper takes the same number of rows per block");
// issue priorities (s_setprio): wave 0 always, helpers during merge; helpers
// run their DP decision bits at the default 0
#ifndef CCSX_PRIO_WAVE0
#define CCSX_PRIO_WAVE0 3
#endif
#ifndef CCSX_PRIO_MERGE
#define CCSX_PRIO_MERGE 2
#endif
constexpr int kPrioWave0 = CCSX_PRIO_WAVE0, kPrioMerge = CCSX_PRIO_MERGE;
// the one-wave objects (no helpers): issue priority of the traceback and the
// merge over the other resident ZMWs' DP rows (s_setprio: VALU issue goes by
// priority, then age).  1 / 1 on solo and solo16 (build.py): E16k -0.9 %, D
// -1.4 % (r05x); 2 / 1, 2 / 2, 3 / 1 measured the same (r05w), everything but
// the DP at 1 or 2 0.1-0.3 % behind
#ifndef CCSX_PRIO_TB
#define CCSX_PRIO_TB 0
#endif
#ifndef CCSX_PRIO_MG
#define CCSX_PRIO_MG 0
#endif
constexpr int kPrioTb = CCSX_PRIO_TB, kPrioMg = CCSX_PRIO_MG;
static_assert(kRingA >= kRing + (kHelpers ? 2 * kBlkAB : 0), "B reads predecessors up to kRing rows behind its row");


enum JobKind : int32_t { kJobExit = 0, kJobDp = 1, kJobMerge = 2, kJobColumns = 3 };
struct DpJob {
    int32_t kind;
    uint32_t m, R, cur;
    uint32_t k;     // merge: read index
    uint32_t K, E;  // merge: new rows (wave 0's M1), edges of the new graph
    uint32_t win;   // DP on the HBM-read instance: first resident window chunk << 1 | slide in progress
    // results of helper wave 1 + h (h = row parity): best free-end value, its
    // row and read position, status
    struct {
        int32_t best;
        uint32_t er, ej;
        int32_t status;
    } res[2];
};
static_assert(sizeof(DpJob) <= 16 * 4, "DP job record exceeds its LDS slot");

__device__ __forceinline__ volatile DpJob *dp_job(const Z &z)
{
    return reinterpret_cast<volatile DpJob *>(z.lds + kLdsJob);
}

// fold predecessor slot s's five cells into the running Mh / D terms
struct PredAcc {
    int32_t Mh0, Mh1, Dv0, Dv1;
    uint32_t ms0, ms1, ds0, ds1, dx0, dx1;
};


// SLOTS: also track, per cell, the tag byte of the predecessor that gave Mh
// and D (first in predecessor order on ties, SPEC.md §3.2) and D's ext bit
// (rows flagged far: the tag is the slot index)
template <bool SLOTS>
__device__ __forceinline__ void pred_fold(PredAcc &A, uint32_t s, uint32_t tag, int32_t hA, int32_t hB, int32_t hC,
                                          int32_t dB, int32_t dC)
{
    const int32_t a0 = hB + (kO + kE), b0 = dB + kE, a1 = hC + (kO + kE), b1 = dC + kE;
    const int32_t c0 = max(a0, b0), c1 = max(a1, b1);
    if (s == 0) {
        A.Mh0 = hA, A.Mh1 = hB, A.Dv0 = c0, A.Dv1 = c1;
        if (SLOTS) {
            A.ms0 = A.ms1 = A.ds0 = A.ds1 = tag;
            A.dx0 = b0 > a0 ? 4u : 0u;
            A.dx1 = b1 > a1 ? 4u : 0u;
        }
    } else if (!SLOTS) {
        A.Mh0 = max(A.Mh0, hA), A.Mh1 = max(A.Mh1, hB), A.Dv0 = max(A.Dv0, c0), A.Dv1 = max(A.Dv1, c1);
    } else {
        if (hA > A.Mh0) A.Mh0 = hA, A.ms0 = tag;
        if (hB > A.Mh1) A.Mh1 = hB, A.ms1 = tag;
        if (c0 > A.Dv0) A.Dv0 = c0, A.ds0 = tag, A.dx0 = b0 > a0 ? 4u : 0u;
        if (c1 > A.Dv1) A.Dv1 = c1, A.ds1 = tag, A.dx1 = b1 > a1 ? 4u : 0u;
    }
}

// the five cells of a predecessor row at band shift sh (lane's cells 2l, 2l+1)
__device__ __forceinline__ void pred_cells(const RingT *row, int32_t sh, int lane, int32_t &hA, int32_t &hB,
                                           int32_t &hC, int32_t &dB, int32_t &dC)
{
    if ((uint32_t)(sh + 3) <= 7u) {
        const RingT *b = row + kHc - 1 + 2 * lane + sh;
        hA = b[0];
        hB = b[1];
        hC = b[2];
        dB = b[kDc - kHc + 1];
        dC = b[kDc - kHc + 2];
    } else {
        const int32_t i = 2 * lane + sh;
        hA = (uint32_t)(i - 1) < (uint32_t)kW ? row[kHc + i - 1] : kNegH;
        hB = (uint32_t)i < (uint32_t)kW ? row[kHc + i] : kNegH;
        hC = (uint32_t)(i + 1) < (uint32_t)kW ? row[kHc + i + 1] : kNegH;
        dB = (uint32_t)i < (uint32_t)kW ? row[kDc + i] : kNeg;
        dC = (uint32_t)(i + 1) < (uint32_t)kW ? row[kDc + i + 1] : kNeg;
    }
}

// the predecessor terms of row r (np <= 4, every predecessor in the ring)
template <bool SLOTS>
__device__ __forceinline__ void pred_terms(const RingT *ring, uint32_t r, int32_t off, uint32_t np, uint32_t p0,
                                           uint32_t p1, uint32_t p2, uint32_t p3, int32_t o0, int32_t o1, int32_t o2,
                                           int32_t o3, uint32_t tg, int lane, PredAcc &A)
{
    const int32_t s0 = off - o0, s1 = off - o1, s2 = off - o2, s3 = off - o3;
    const bool inr = (uint32_t)(s0 + 3) <= 7u && (np < 2 || (uint32_t)(s1 + 3) <= 7u) &&
                     (np < 3 || (uint32_t)(s2 + 3) <= 7u) && (np < 4 || (uint32_t)(s3 + 3) <= 7u);
    if (np == 0) {
        pred_fold<SLOTS>(A, 0, 0, kNegH, kNegH, kNegH, kNeg, kNeg);
    } else if (inr) {
        // every predecessor within the padded band: issue all reads (absent
        // slots re-read slot 0's row), then fold
        const int L2 = 2 * lane;
        const RingT *b0 = ring + (p0 % kRingA) * kRowW + (kHc - 1) + L2 + s0;
        const RingT *b1 = np > 1 ? ring + (p1 % kRingA) * kRowW + (kHc - 1) + L2 + s1 : b0;
        const RingT *b2 = np > 2 ? ring + (p2 % kRingA) * kRowW + (kHc - 1) + L2 + s2 : b0;
        const RingT *b3 = np > 3 ? ring + (p3 % kRingA) * kRowW + (kHc - 1) + L2 + s3 : b0;
        constexpr int dd = kDc - kHc + 1;
        const int32_t a0 = b0[0], a1 = b0[1], a2 = b0[2], a3 = b0[dd], a4 = b0[dd + 1];
        const int32_t c0 = b1[0], c1 = b1[1], c2 = b1[2], c3 = b1[dd], c4 = b1[dd + 1];
        const int32_t e0 = b2[0], e1 = b2[1], e2 = b2[2], e3 = b2[dd], e4 = b2[dd + 1];
        const int32_t g0 = b3[0], g1 = b3[1], g2 = b3[2], g3 = b3[dd], g4 = b3[dd + 1];
        pred_fold<SLOTS>(A, 0, tg, a0, a1, a2, a3, a4);
        if (np > 1) pred_fold<SLOTS>(A, 1, tg >> 8, c0, c1, c2, c3, c4);
        if (np > 2) pred_fold<SLOTS>(A, 2, tg >> 16, e0, e1, e2, e3, e4);
        if (np > 3) pred_fold<SLOTS>(A, 3, tg >> 24, g0, g1, g2, g3, g4);
    } else {
        int32_t hA, hB, hC, dB, dC;
        pred_cells(ring + (p0 % kRingA) * kRowW, s0, lane, hA, hB, hC, dB, dC);
        pred_fold<SLOTS>(A, 0, tg, hA, hB, hC, dB, dC);
        if (np > 1) {
            pred_cells(ring + (p1 % kRingA) * kRowW, s1, lane, hA, hB, hC, dB, dC);
            pred_fold<SLOTS>(A, 1, tg >> 8, hA, hB, hC, dB, dC);
        }
        if (np > 2) {
            pred_cells(ring + (p2 % kRingA) * kRowW, s2, lane, hA, hB, hC, dB, dC);
            pred_fold<SLOTS>(A, 2, tg >> 16, hA, hB, hC, dB, dC);
        }
        if (np > 3) {
            pred_cells(ring + (p3 % kRingA) * kRowW, s3, lane, hA, hB, hC, dB, dC);
            pred_fold<SLOTS>(A, 3, tg >> 24, hA, hB, hC, dB, dC);
        }
    }
}

// the predecessor terms of a row with exactly NP (1 or 2) predecessors, all
// within the ring; reads through the padded band when every shift is in
// [-3, 4], else bounds-checked per cell
template <int NP, bool SLOTS>
__device__ __forceinline__ void pred_terms_n(const RingT *ring, uint32_t r, int32_t off, uint32_t p0, uint32_t p1,
                                             int32_t o0, int32_t o1, uint32_t tg, int lane, PredAcc &A)
{
    const int32_t s0 = off - o0, s1 = off - o1;
    // (one unsigned max: fewer scalar compares and selects than an &&)
    const bool inr = (NP < 2 ? (uint32_t)(s0 + 3) : max((uint32_t)(s0 + 3), (uint32_t)(s1 + 3))) <= 7u;
    constexpr int dd = kDc - kHc + 1;
    if (__builtin_expect(inr, 1)) {
        const int L2 = 2 * lane;
        const RingT *b0 = ring + (p0 % kRingA) * kRowW + (kHc - 1) + L2 + s0;
        const RingT *b1 = ring + (p1 % kRingA) * kRowW + (kHc - 1) + L2 + s1;
        const int32_t a0 = b0[0], a1 = b0[1], a2 = b0[2], a3 = b0[dd], a4 = b0[dd + 1];
        int32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
        if (NP > 1) c0 = b1[0], c1 = b1[1], c2 = b1[2], c3 = b1[dd], c4 = b1[dd + 1];
        pred_fold<SLOTS>(A, 0, tg, a0, a1, a2, a3, a4);
        if (NP > 1) pred_fold<SLOTS>(A, 1, tg >> 8, c0, c1, c2, c3, c4);
    } else {
        int32_t hA, hB, hC, dB, dC;
        pred_cells(ring + (p0 % kRingA) * kRowW, s0, lane, hA, hB, hC, dB, dC);
        pred_fold<SLOTS>(A, 0, tg, hA, hB, hC, dB, dC);
        if (NP > 1) {
            pred_cells(ring + (p1 % kRingA) * kRowW, s1, lane, hA, hB, hC, dB, dC);
            pred_fold<SLOTS>(A, 1, tg >> 8, hA, hB, hC, dB, dC);
        }
    }
}

// Spill records of the two-wave DP (rows with a successor > kRing rows
// ahead): words [0, 128) H, [128, 256) D, 256 band offset, 257 row-max key.
constexpr uint32_t kSpillRec = kW * 8 + 16;

__device__ __forceinline__ void far_meta(const Z &z, uint32_t r, uint32_t p, int32_t vOff, int32_t vKey, int32_t &o,
                                         int32_t &k, const int32_t *&rec)
{
    if (r - p <= (uint32_t)kRing) {
        o = __builtin_amdgcn_readlane(vOff, (int)(p & 63u));
        k = __builtin_amdgcn_readlane(vKey, (int)(p & 63u));
        rec = nullptr;
    } else {
        const uint32_t sl = uni(__builtin_nontemporal_load(P<uint32_t>(z, z.L.sslot) + p));
        rec = reinterpret_cast<const int32_t *>(z.ws + z.L.spill + (size_t)sl * kSpillRec);
        o = uni(__builtin_nontemporal_load(rec + 256));
        k = uni(__builtin_nontemporal_load(rec + 257));
    }
}

__device__ __forceinline__ void far_cells(const Z &z, uint32_t p, const int32_t *rec, int32_t sh, int lane,
                                          int32_t &hA, int32_t &hB, int32_t &hC, int32_t &dB, int32_t &dC)
{
    if (!rec) {
        pred_cells(reinterpret_cast<const RingT *>(z.lds + kLdsRing) + (p % kRingA) * kRowW, sh, lane, hA, hB, hC, dB, dC);
        return;
    }
    const int32_t i = 2 * lane + sh;
    auto h = [&](int32_t t) { return (uint32_t)t < (uint32_t)kW ? __builtin_nontemporal_load(rec + t) : kNegH; };
    auto d = [&](int32_t t) { return (uint32_t)t < (uint32_t)kW ? __builtin_nontemporal_load(rec + kW + t) : kNeg; };
    hA = h(i - 1), hB = h(i), hC = h(i + 1), dB = d(i), dC = d(i + 1);
}

// A row with a predecessor beyond the ring or more than four predecessors:
// the full predecessor list from the graph, far rows from their spill
// records (SPEC.md §3.1-§3.2 with every tie rule)
template <bool SLOTS>
__device__ __forceinline__ void far_terms(const Z &z, uint32_t r, uint32_t np, int32_t vOff, int32_t vKey, int32_t lim,
                                       bool place, int32_t &off, PredAcc &A)
{
    const int lane = lane_id();
    const uint32_t po = uni(G_poff(z, z.cur)[r]);
    const uint32_t *pl = G_pred(z, z.cur) + po;
    if (place) {
        off = 0;
        int32_t bm = INT32_MIN, barg = 0;
        for (uint32_t s = 0; s < np; ++s) {
            const uint32_t p = uni(pl[s]);
            int32_t o, k;
            const int32_t *rec;
            far_meta(z, r, p, vOff, vKey, o, k, rec);
            if ((k >> 7) > bm) bm = k >> 7, barg = o + 127 - (k & 127);
        }
        if (np) off = min(max(barg + 1 - kW / 2, 0), lim);
    }
    if (np == 0) {
        pred_fold<SLOTS>(A, 0, 0, kNegH, kNegH, kNegH, kNeg, kNeg);
        return;
    }
    for (uint32_t s = 0; s < np; ++s) {
        const uint32_t p = uni(pl[s]);
        int32_t o, k, hA, hB, hC, dB, dC;
        const int32_t *rec;
        far_meta(z, r, p, vOff, vKey, o, k, rec);
        far_cells(z, p, rec, off - o, lane, hA, hB, hC, dB, dC);
        pred_fold<SLOTS>(A, s, s, hA, hB, hC, dB, dC);  // far rows: the tag is the slot
    }
}

// the 64-row record window of a wave: superblock s + 1 is loaded during the
// second block of superblock s and becomes current after its last block
// (before any store of that block, so the wait covers only old accesses)
struct RecWin {
    RowPre cur, nxt;
};

__device__ __forceinline__ void recwin_begin(const Z &z, RecWin &W, uint32_t r0)
{
    if (r0 == 0) {
        prefetch_recs(z, 0, W.nxt);
        W.cur = W.nxt;
    } else if ((r0 & 63u) == (uint32_t)kBlkAB) {
        prefetch_recs(z, r0 - kBlkAB + 64, W.nxt);
    }
}

__device__ __forceinline__ void recwin_end(RecWin &W, uint32_t r0)
{
    if ((r0 & 63u) == 64u - kBlkAB) W.cur = W.nxt;
}

struct AState {
    int32_t H0, H1, D0, D1;  // row r-1, this lane's two cells
    int32_t pOff, pArg;      // row r-1: band offset, position of its maximum (solo: + 1 - W / 2, dpS_row)
    int32_t vOff, vKey;      // lane (q & 63): band offset / row-max key of row q
    uint32_t qn;             // rd_win16 at this row's offset pOff: the next row's read codes (loaded a row ahead)
    uint32_t nspill;         // spill records written
    uint64_t fmask;          // bit q & 63: row q is a chain row without far / spill flags
    uint32_t ring;           // LDS word offset of this row's ring slot ((r % kRingA) * kRowW)
    RecWin W;
};

// per-lane constants of a row (t0 = 2 lane, t1 = t0 + 1)
struct LaneK {
    int32_t L2, L4, kc0, kc1, cI0, cI1, src0;  // src0: O + E t0
    // the one-wave DP's tail (dpS_row): X = H' - E t biased by kXBias, so every
    // real X is positive and the scans' out-of-range lanes can read 0 from the
    // DPP bound control (no old-value register per shift, no copy of the
    // scan's input); the insertion term of cell 1 carries -kXBias (cell 0's is
    // cIb1 + 2: at lane 0, where the exclusive prefix max is 0, that is
    // -kXBias - 3, below every real H', i.e. I(0) = NEG)
    int32_t cIb1;
};
// 2^30: the bit pattern of 2.0f, an inline constant (v_add3_u32 takes it
// without a register); every |X| of a read < 2^22 is below 2^24
constexpr int32_t kXBias = 1 << 30;

__device__ __forceinline__ LaneK lane_consts(int lane)
{
    LaneK c;
    c.L2 = 2 * lane, c.L4 = 4 * lane;
    c.kc0 = 127 - c.L2, c.kc1 = 126 - c.L2;
    c.cI0 = kO + kE * c.L2, c.cI1 = kO + kE * (c.L2 + 1);
    c.src0 = kO + kE * c.L2;
    c.cIb1 = c.cI1 - kXBias;
    return c;
}

// wave 0, the rows that are not "chain, band moved by 1": chain rows moved
// by 0 or 2 (DPP) and general rows (predecessors from the ring).  SLOTS
// (the solo configuration, which computes its own decision bits): A also
// carries the predecessor tags and D-ext bits, as the helpers' dpB_cold does.
template <bool SLOTS>
__device__ __forceinline__ void dpA_cold(const Z &z, const AState &S, uint32_t r, uint32_t info, int32_t coff,
                                         int32_t lim, int32_t &off_o, PredAcc &A, int &kind)
{
    const int lane = lane_id();
    const int li = (int)(r & 63u);
    const uint32_t np = info >> 8;
    const int32_t sh = coff - S.pOff;
    const RingT *ring = reinterpret_cast<const RingT *>(z.lds + kLdsRing);
    int32_t off;
    kind = 4;
    if (info & kInfoFar) {
        kind = 0;
        far_terms<SLOTS>(z, r, np, S.vOff, S.vKey, lim, true, off, A);
    } else if ((info & kInfoChain) && (uint32_t)sh <= 2u) {
        kind = 1;
        // chain row, band moved by 0..2 (1: a spill row)
        off = coff;
        int32_t hA, hB, hC, dB, dC;
        if (sh == 0) {
            hA = wave_shr1(kNegH, S.H1), hB = S.H0, hC = S.H1, dB = S.D0, dC = S.D1;
        } else if (sh == 1) {
            hA = S.H0, hB = S.H1, hC = wave_shl1(kNegH, S.H0), dB = S.D1, dC = wave_shl1(kNeg, S.D0);
        } else {
            hA = S.H1, hB = wave_shl1(kNegH, S.H0), hC = wave_shl1(kNegH, S.H1);
            dB = wave_shl1(kNeg, S.D0), dC = wave_shl1(kNeg, S.D1);
        }
        pred_fold<SLOTS>(A, 0, kTagPrev, hA, hB, hC, dB, dC);  // the predecessor is row r - 1
    } else if (np == 1) {
        kind = 2;
        const uint32_t p0 = row_pred(S.W.cur, r, li, 0);
        const int32_t o0 = __builtin_amdgcn_readlane(S.vOff, (int)(p0 & 63u));
        const int32_t k0 = __builtin_amdgcn_readlane(S.vKey, (int)(p0 & 63u));
        off = min(max(o0 + 127 - (k0 & 127) + 1 - kW / 2, 0), lim);
        pred_terms_n<1, SLOTS>(ring, r, off, p0, p0, o0, o0, SLOTS ? row_tag(S.W.cur, li, 0) : 0u, lane, A);
    } else if (np == 2) {
        kind = 3;
        const uint32_t p0 = row_pred(S.W.cur, r, li, 0);
        const uint32_t p1 = row_pred(S.W.cur, r, li, 1);
        const int32_t o0 = __builtin_amdgcn_readlane(S.vOff, (int)(p0 & 63u));
        const int32_t o1 = __builtin_amdgcn_readlane(S.vOff, (int)(p1 & 63u));
        const int32_t k0 = __builtin_amdgcn_readlane(S.vKey, (int)(p0 & 63u));
        const int32_t k1 = __builtin_amdgcn_readlane(S.vKey, (int)(p1 & 63u));
        // band placement (SPEC.md §3.1): first predecessor with the largest row max
        const bool second = (k1 >> 7) > (k0 >> 7);
        const int32_t ko = second ? k1 : k0, oo = second ? o1 : o0;
        off = min(max(oo + 127 - (ko & 127) + 1 - kW / 2, 0), lim);
        pred_terms_n<2, SLOTS>(ring, r, off, p0, p1, o0, o1, SLOTS ? row_tag(S.W.cur, li, 0) : 0u, lane, A);
    } else {
        const uint32_t p0 = row_pred(S.W.cur, r, li, 0);
        const uint32_t p1 = row_pred(S.W.cur, r, li, 1);
        const uint32_t p2 = row_pred(S.W.cur, r, li, 2);
        const uint32_t p3 = row_pred(S.W.cur, r, li, 3);
        const int32_t o0 = __builtin_amdgcn_readlane(S.vOff, (int)(p0 & 63u));
        const int32_t o1 = __builtin_amdgcn_readlane(S.vOff, (int)(p1 & 63u));
        const int32_t o2 = __builtin_amdgcn_readlane(S.vOff, (int)(p2 & 63u));
        const int32_t o3 = __builtin_amdgcn_readlane(S.vOff, (int)(p3 & 63u));
        const int32_t k0 = __builtin_amdgcn_readlane(S.vKey, (int)(p0 & 63u));
        const int32_t k1 = __builtin_amdgcn_readlane(S.vKey, (int)(p1 & 63u));
        const int32_t k2 = __builtin_amdgcn_readlane(S.vKey, (int)(p2 & 63u));
        const int32_t k3 = __builtin_amdgcn_readlane(S.vKey, (int)(p3 & 63u));
        off = 0;
        if (np) {
            int32_t bm = k0 >> 7, barg = o0 + 127 - (k0 & 127);
            if ((k1 >> 7) > bm) bm = k1 >> 7, barg = o1 + 127 - (k1 & 127);
            if ((k2 >> 7) > bm) bm = k2 >> 7, barg = o2 + 127 - (k2 & 127);
            if (np > 3 && (k3 >> 7) > bm) bm = k3 >> 7, barg = o3 + 127 - (k3 & 127);
            off = min(max(barg + 1 - kW / 2, 0), lim);
        }
        pred_terms<SLOTS>(ring, r, off, np, p0, p1, p2, p3, o0, o1, o2, o3, SLOTS ? row_tag(S.W.cur, li, 0) : 0u, lane,
                          A);
    }
    off_o = off;
}

// wave 0: one DP row (SPEC.md §3.1-§3.4 values).  FULL: m >= W, every band
// cell is a read position; else (m < W, off == 0) cells t >= m are invalid:
// H = kNegH, D = kNeg there, and they take no part in the row maximum.
template <bool FULL>
__device__ __forceinline__ void dpA_row(Z &z, AState &S, uint32_t r, int32_t lim, uint32_t m, const LaneK &c,
                                        uint32_t ring, uint32_t chn)
{
    const int lane = lane_id();
#ifdef CCSX_DP_STAMPS
    unsigned long long t_prev = stamp();
#endif
    const int li = (int)(r & 63u);
    const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)S.W.cur.info, li);
    const uint32_t base = info & 3u;
    // (S.pArg: the next band offset before clamping, as dpS_row's; chn: the
    // row is a plain chain row, from the block's chain mask)
    const int32_t coff = min(max(S.pArg, 0), lim);
    const int32_t sh = coff - S.pOff;
    // (an integer test keeps the branch scalar: a bool of && lowers to a lane mask)
    const uint32_t fast = (3u >> min((uint32_t)sh, 2u)) & chn;  // (as dpS_row)
#ifdef CCSX_DP_STAMPS
    unsigned long long ts0, ts1, ts2, ts3;
    int ckind = 0;
    ROW_STAMP(ts0);
#endif
    // everything after the predecessor terms; instantiated on both sides of
    // the fast / cold branch so a fast row meets no further branch
    int32_t row_key = 0;  // the row's key (readlane of the max-scan)
    auto tail = [&](int32_t off, uint32_t qp, int32_t Mh0, int32_t Mh1, int32_t Dv0, int32_t Dv1,
                    bool cold) __attribute__((always_inline)) {
        // the next row's read window, a row ahead of its use (its offset lies
        // in [off, off + 3] on every fast row)
        S.qn = rd_win16(z, off, z.hbm && win_has(z.wa, 2, off));
        const uint32_t q0 = qp & 3u, q1 = (qp >> 2) & 3u;
        const int32_t srcu = c.src0 + kE * off;
        // (the fast rows fold the j = 0 leading term into Mh0, see below)
        const int32_t src0 = (cold && off == 0 && lane == 0) ? 0 : srcu;
        const int32_t M0 = max(Mh0, src0) + (q0 == base ? kMs : kXs);
        const int32_t M1 = max(Mh1, srcu + kE) + (q1 == base ? kMs : kXs);
        const int32_t hp0 = max(M0, Dv0), hp1 = max(M1, Dv1);
        const int32_t X0 = hp0 + c.L4;
        int32_t incl = max(X0, hp1 + c.L4 + 2);
        int32_t rk0 = (hp0 << 7) | c.kc0, rk1 = (hp1 << 7) | c.kc1;
        if (!FULL) {
            if ((uint32_t)c.L2 >= m) rk0 = INT32_MIN, Dv0 = kNeg;
            if ((uint32_t)c.L2 + 1 >= m) rk1 = INT32_MIN, Dv1 = kNeg;
        }
        int32_t rk = max(rk0, rk1);
#ifdef CCSX_DP_STAMPS
        if (!cold && ckind != 6) ROW_STAMP(ts1);
#endif
        wave_incl_max2(incl, rk);
        const int32_t Pex = wave_shr1(kNeg, incl);
        int32_t nH0 = max(Pex + c.cI0, hp0), nH1 = max(max(Pex, X0) + c.cI1, hp1);
        if (!FULL) {
            if ((uint32_t)c.L2 >= m) nH0 = kNegH;
            if ((uint32_t)c.L2 + 1 >= m) nH1 = kNegH;
        }
        const int32_t key = __builtin_amdgcn_readlane(rk, 63);
        // ring row, meta window
        RingT *row = reinterpret_cast<RingT *>(z.lds + kLdsRing) + ring + kHc + c.L2;
        ring_store2(row, nH0, nH1);
        ring_store2(row + (kDc - kHc), Dv0, Dv1);
        // (the offset / key vectors after the fast / cold join, below)
        row_key = key;
        if (cold && (info & kInfoSpill)) {
            // a successor lies beyond the ring: keep this row in HBM
            const uint32_t sl = S.nspill++;
            if (sl < z.d.scap) {
                int32_t *rec = reinterpret_cast<int32_t *>(z.ws + z.L.spill + (size_t)sl * kSpillRec);
                reinterpret_cast<int2 *>(rec)[lane] = make_int2(nH0, nH1);
                reinterpret_cast<int2 *>(rec + kW)[lane] = make_int2(Dv0, Dv1);
                if (lane == 0) rec[256] = off, rec[257] = key, P<uint32_t>(z, z.L.sslot)[r] = sl;
            } else {
                z.status = kErrSpill;
            }
            wsync();  // visible to every wave before any reader (> kRing rows later)
        }
        S.H0 = nH0, S.H1 = nH1, S.D0 = Dv0, S.D1 = Dv1;
        S.pOff = off;
        S.pArg = off + kW / 2 - (key & 127);
#ifdef CCSX_DP_STAMPS
        if (!cold && ckind != 6) {
            ROW_STAMP(ts2);
            ROW_STAMP(ts3);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(ts0), "+s"(ts1), "+s"(ts2), "+s"(ts3)::"memory");
            z.pf[kPfAHead] += ts1 - t_prev;  // row start -> scan, t_prev: last row's end
            z.pf[kPfABody] += ts2 - ts1;      // scan and everything after
            z.pf[kPfATail] += ts0 - t_prev;   // row start -> fast decision
            z.pf[kPfAFast] += 1;
            (void)ts3;
        } else {
            ROW_STAMP(ts2);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(ts2)::"memory");
            // constant indices only: a computed index would move z.pf (and
            // with it much of Z) to scratch
            const unsigned long long dt = ts2 - t_prev;
            switch (ckind) {
            case 0: z.pf[kPfCold0] += dt, z.pf[kPfColdN0] += 1; break;
            case 1: z.pf[kPfCold1] += dt, z.pf[kPfColdN1] += 1; break;
            case 2: z.pf[kPfCold2] += dt, z.pf[kPfColdN2] += 1; break;
            case 3: z.pf[kPfCold3] += dt, z.pf[kPfColdN3] += 1; break;
            case 4: z.pf[kPfCold4] += dt, z.pf[kPfColdN4] += 1; break;
            case 5: z.pf[kPfCold5] += dt, z.pf[kPfColdN5] += 1; break;
            default: z.pf[kPfCold6] += dt, z.pf[kPfColdN6] += 1; break;
            }
        }
#endif
    };
    if (__builtin_expect(fast, 1)) {
        // the only predecessor is row r-1 and the band moved by 0 or 1: its
        // cells are in registers, shifted by DPP.  Lane 0's diagonal term on a
        // row at offset 0 (band unmoved) is the read-prefix source 0 instead
        // of -inf (SPEC.md §3.2 src(0) = 0): it rides in as the DPP's old
        // value, max(0, src) = 0, so the tail needs no lane test.
        const uint32_t qp = win_codes(S.qn, S.pOff, sh);  // sh in [0, 1]
        // band move 0 or 1 as a scalar branch: each side shifts only what it
        // needs (no selects)
        if (sh == 0) {
            const int32_t hL = wave_shr1(coff == 0 ? 0 : kNegH, S.H1);
            const int32_t Dv0 = max(S.H0 + (kO + kE), S.D0 + kE);
            const int32_t Dv1 = max(S.H1 + (kO + kE), S.D1 + kE);
            tail(coff, qp, hL, S.H0, Dv0, Dv1, false);
        } else {
            const int32_t hR = wave_shl1(kNegH, S.H0), dR = wave_shl1(kNeg, S.D0);
            const int32_t Dv0 = max(S.H1 + (kO + kE), S.D1 + kE);
            const int32_t Dv1 = max(hR + (kO + kE), dR + kE);
            tail(coff, qp, S.H0, S.H1, Dv0, Dv1, false);
        }
    } else {
        int32_t off;
        PredAcc A;
        int kind;
        dpA_cold<false>(z, S, r, info, coff, lim, off, A, kind);
        const int32_t Mh0 = A.Mh0, Mh1 = A.Mh1, Dv0 = A.Dv0, Dv1 = A.Dv1;
#ifdef CCSX_DP_STAMPS
        if (info & kInfoSpill) kind = 5;
        ckind = kind;
#endif
        (void)kind;
        const uint32_t d = (uint32_t)(off - S.pOff);
        const uint32_t qp = d <= 3u ? win_codes(S.qn, S.pOff, (int32_t)d)
                                    : win_codes(rd_win16(z, off, z.hbm && win_has(z.wa, 2, off)), off, 0);
        tail(off, qp, Mh0, Mh1, Dv0, Dv1, true);
    }
    // (inline asm measured 0.6 % faster than the compiler's writelane
    // intrinsic: it keeps vOff / vKey out of the scheduler's way; after the
    // join, one pair instead of a pair plus two register copies per branch)
    S.vOff = writelane(S.vOff, S.pOff, li);
    S.vKey = writelane(S.vKey, row_key, li);
}

// wave 0: rows [r0, r0 + kBlkAB)
template <bool FULL>
__device__ __forceinline__ void dpA_block(Z &z, AState &S, uint32_t r0, uint32_t m)
{
    const int lane = lane_id();
    const int32_t lim = FULL ? (int32_t)m - kW : 0;
    const LaneK c = lane_consts(lane);
    recwin_begin(z, S.W, r0);
    if ((r0 & 63u) == 0) {
        const uint32_t inf = S.W.cur.info;
        S.fmask = ballot((inf & (kInfoChain | kInfoFar | kInfoSpill)) == kInfoChain);
    }
    // ring slots of the block's rows: r0 is a multiple of kBlkAB, which
    // divides kRingA, so the block's rows take consecutive slots (constant
    // offsets from the block's first)
    static_assert(kHelpers == 0 || kRingA % kBlkAB == 0, "a block's rows occupy consecutive ring slots");  // (the solo objects run dpS_block)
    const uint32_t rb = (r0 % (uint32_t)kRingA) * (uint32_t)kRowW;
    const uint32_t fm = (uint32_t)(S.fmask >> (r0 & 63u));  // bit i: row r0 + i is a plain chain row
    if (r0 + kBlkAB <= z.R) {
#pragma unroll
        for (uint32_t i = 0; i < (uint32_t)kBlkAB; ++i)
            dpA_row<FULL>(z, S, r0 + i, lim, m, c, rb + i * kRowW, (fm >> i) & 1u);
    } else {
        for (uint32_t i = 0; r0 + i < z.R; ++i) dpA_row<FULL>(z, S, r0 + i, lim, m, c, rb + i * kRowW, (fm >> i) & 1u);
    }
    z.lds[kLdsOffRing + lane] = S.vOff;  // band offsets of the last 64 rows for the helpers
    recwin_end(S.W, r0);
}

struct BState {
    int32_t bE;       // best free-end value of this lane's cells
    uint32_t bKey;    // its row * 2 + cell
    int32_t bOff;     // its row's band offset
    uint32_t wc0, wnc;  // HBM-read instance: the read-window chunks this period may trust
    RecWin W;
    __amdgpu_buffer_rsrc_t rc;  // cell records of this DP (R rows x 256 B)
};

// helper wave: the predecessor terms of a row that does not have exactly one
// in-band predecessor (0 or >= 2 predecessors, or a far band shift)
__device__ __forceinline__ void dpB_cold(Z &z, const BState &S, uint32_t r, uint32_t info, int32_t off,
                                         int32_t vOff, PredAcc &A)
{
    const int lane = lane_id();
    const int li = (int)(r & 63u);
    const uint32_t np = info >> 8;
    const RingT *ring = reinterpret_cast<const RingT *>(z.lds + kLdsRing);
    if (info & kInfoFar) {
        int32_t o = off;
        // band placement is wave 0's; the cell tags are predecessor slots
        // (6 bits in the record; rows above 63 predecessors: dpB_row also
        // stores the full slots)
        far_terms<true>(z, r, np, vOff, 0, 0, false, o, A);
        return;
    }
    const uint32_t tg = row_tag(S.W.cur, li, 0);
    const uint32_t p0 = r - 1u - (tg & 15u), p1 = r - 1u - ((tg >> 8) & 15u);
    const int32_t o0 = __builtin_amdgcn_readlane(vOff, (int)(p0 & 63u));
    const int32_t o1 = __builtin_amdgcn_readlane(vOff, (int)(p1 & 63u));
    if (np == 2) {
        pred_terms_n<2, true>(ring, r, off, p0, p1, o0, o1, tg, lane, A);
    } else if (np == 1) {
        pred_terms_n<1, true>(ring, r, off, p0, p0, o0, o0, tg, lane, A);
    } else {
        const uint32_t p2 = r - 1u - ((tg >> 16) & 15u), p3 = r - 1u - ((tg >> 24) & 15u);
        const int32_t o2 = __builtin_amdgcn_readlane(vOff, (int)(p2 & 63u));
        const int32_t o3 = __builtin_amdgcn_readlane(vOff, (int)(p3 & 63u));
        pred_terms<true>(ring, r, off, np, p0, p1, p2, p3, o0, o1, o2, o3, tg, lane, A);
    }
}

// the DP's cell records and, after them, its tag plane (row_slots)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec_rsrc(const Z &z)
{
    return brsrc(z.ws + z.L.codes, (uint32_t)(z.L.dsl - z.L.codes) + z.R * kRecRow);
}

// The records beside a row's cell bytes: a far row's slot record (u16 M / D
// slot per cell, its index in word 0 of the row's tag-plane row), or, for a
// row of 3-4 predecessors, its tag plane: the D distance - 1 per cell, 4 bits
// (and the M one beside it, a byte per cell, where the ring is longer than 8
// rows).  Rows of one or two predecessors need neither (rmeta_word).
// (Buffer stores: a store through a generic pointer is a flat store, which
// also counts in lgkmcnt, so the next row's wait on its ring reads would wait
// for it to reach memory.)
__device__ __forceinline__ void row_slots(Z &z, const __amdgpu_buffer_rsrc_t &rc, uint32_t r, uint32_t info,
                                          const PredAcc &A)
{
    // the tag plane follows the records: the records' descriptor (rec_rsrc)
    // reaches it at this scalar offset (a descriptor of its own cost the
    // helpers ~10 SGPR spill reloads per row, config B +4 %)
    const uint32_t tpo = (uint32_t)(z.L.dsl - z.L.codes);
    const uint32_t lane = lane_id();
    if (info & kInfoFar) {
        const uint32_t fs = z.nfar;
        z.nfar += (uint32_t)kHelperStep;
        if (fs < z.d.wcap) {
            // (rare: buffer stores, whose descriptors cost scalar work but no VGPRs)
            const auto fr = brsrc(PX<uint8_t>(z, kExtWtag), z.d.wcap * (kW * 4u));
            __builtin_amdgcn_raw_buffer_store_b64(v2u{A.ms0 | (A.ds0 << 16), A.ms1 | (A.ds1 << 16)}, fr,
                                                  fs * (kW * 4u) + lane * 8u, 0, 0);
            if (lane == 0) __builtin_amdgcn_raw_buffer_store_b32(fs, rc, r * kRecRow, tpo, 0);
        } else {
            z.status = kErrSpill;  // (re-run with full caps: a far slot record per row)
        }
    } else {
        if constexpr (kRing <= 8) {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((A.ds0 & 15u) | ((A.ds1 & 15u) << 4)), rc, r * kRecRow + lane, tpo,
                                                 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b16(
                (unsigned short)((A.ms0 & 15u) | ((A.ds0 & 15u) << 4) | ((A.ms1 & 15u) << 8) | ((A.ds1 & 15u) << 12)), rc,
                r * kRecRow + lane * 2u, tpo, 0);
        }
    }
}

// Row r's decision bits from its cell values (SPEC.md §3.4: code, D-ext,
// I-ext, M / D tags), its free-end candidates (§3.5) and the record store:
// the helpers' dpB_tail (values recomputed from the ring) and the solo
// dpS_row (values the wave holds) share it.  mp / d: M came from a
// predecessor / D beat M, per cell; X = H' + 2 t; Pex = the insertion scan's
// exclusive prefix max.  cold: the row may need row_slots (info: its flags).
// a row's position in its DP block, for the solo wave's row bookkeeping
struct RowX {
    uint32_t chn;    // dpS_row: 1 if the row is a plain chain row (one predecessor, r - 1, no far / spill flags)
    uint32_t rot;    // tb_rot(r)
    uint32_t ioff;   // record byte offset of the row from sbase (a constant of the unrolled block)
    uint32_t sbase;  // record byte offset of the block
    int32_t em1;     // -2m - 1 (free-end candidates)
};
__device__ __forceinline__ RowX row_x(uint32_t r, uint32_t m)
{
    return RowX{1u, tb_rot(r), 0u, r * kRecRow, -2 * (int32_t)m - 1};
}

template <bool FULL, bool TRACK_OFF = true>
__device__ __forceinline__ void row_record(Z &z, int32_t &bE, uint32_t &bKey, int32_t &bOff,
                                           const __amdgpu_buffer_rsrc_t &rc, uint32_t r, uint32_t m, int32_t lim,
                                           int32_t off, uint32_t info, bool cold, const PredAcc &A, const LaneK &c,
                                           bool mp0, bool mp1, bool d0, bool d1, int32_t hp0, int32_t hp1, int32_t X0,
                                           int32_t X1, int32_t Pex, const RowX &x)
{
    const int lane = lane_id();
    const int32_t X1L = wave_shr1(INT32_MAX, X1);
    const int32_t ex1 = max(Pex, X0);
    const bool i0 = Pex + c.cI0 > hp0, i1 = ex1 + c.cI1 > hp1;
    const uint32_t iext0 = Pex > X1L ? 8u : 0u, iext1 = Pex > X0 ? 8u : 0u;
    const uint32_t hc0 = i0 ? HC_INS : d0 ? HC_DEL : mp0 ? HC_MPRED : HC_MSRC;
    const uint32_t hc1 = i1 ? HC_INS : d1 ? HC_DEL : mp1 ? HC_MPRED : HC_MSRC;
    uint32_t w0 = hc0 | A.dx0 | iext0 | (A.ms0 & 0x70u) | (A.ds0 & 0x80u);
    uint32_t w1 = hc1 | A.dx1 | iext1 | (A.ms1 & 0x70u) | (A.ds1 & 0x80u);
    if (cold && ((info & kInfoFar) || (info >> 8) >= 3u)) row_slots(z, rc, r, info, A);
    // free-end candidates (SPEC.md §3.5) on H': e = H' + 2j - 2m - 1, and
    // H' at j = m - 1
    const int32_t eb = (off << 1) + x.em1;
    int32_t e0 = X0 + eb;
    int32_t e1 = X1 + eb;
    if (FULL) {
        // (a scalar branch, rarely taken: off == lim only where the band meets
        // the read's end; the lane select cost lane-mask logic on every row:
        // D -0.4 %, r04zn)
        if (__builtin_expect(off == lim, 0)) e1 = writelane(e1, __builtin_amdgcn_readlane(e1, 63) + 3, 63);
    } else {
        if ((uint32_t)c.L2 == m - 1) e0 += 3;
        if ((uint32_t)c.L2 + 1 == m - 1) e1 += 3;
        if ((uint32_t)c.L2 >= m) e0 = INT32_MIN, w0 = 0;
        if ((uint32_t)c.L2 + 1 >= m) e1 = INT32_MIN, w1 = 0;
    }
    // rows come in order: the first maximum is the earliest (min row, min cell)
    // (TRACK_OFF false: the caller looks the winner's band offset up in the
    // row meta afterwards -- two VALU per row fewer)
    if (!TRACK_OFF) {
        // the lane's two cells first (cell 1 only if strictly better), then
        // against the best so far: the same first maximum
        const bool c1 = e1 > e0;
        const int32_t e01 = c1 ? e1 : e0;
        if (e01 > bE) bE = e01, bKey = r * 2 + (c1 ? 1u : 0u);
    } else {
        if (e0 > bE) bE = e0, bKey = r * 2, bOff = TRACK_OFF ? off : bOff;
        if (e1 > bE) bE = e1, bKey = r * 2 + 1, bOff = TRACK_OFF ? off : bOff;
    }
    // rotated by tb_rot(r) words within the row (the traceback's LDS bank skew)
    // (the block's base as the store's scalar offset, the row's in the
    // instruction's offset field)
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(w0 | (w1 << 8)), rc, (((uint32_t)lane * 2u + x.rot) & 127u) + x.ioff,
                                          x.sbase, 0);
}

// row_record for the one-wave DP (dpS_row): the same records and free-end
// candidates from its biased X (LaneK::xb*: X + kXBias, the exclusive prefix
// max 0 at lane 0), and, on FULL rows, the lane's candidate from xm = max(X0,
// X1), the insertion scan's input: one add, a compare for the cell and a
// carry-in add for the key (round 5: two adds, a max, two compares, a select
// and a shift-or per row)
template <bool FULL>
__device__ __forceinline__ void row_record_solo(Z &z, int32_t &bE, uint32_t &bKey, const __amdgpu_buffer_rsrc_t &rc,
                                                uint32_t r, uint32_t m, int32_t lim, int32_t off, uint32_t info,
                                                bool cold, const PredAcc &A, const LaneK &c, bool mp0, bool mp1,
                                                bool d0, bool d1, int32_t hp0, int32_t hp1, int32_t X0, int32_t X1,
                                                int32_t xm, int32_t Pex, int32_t ex1, const RowX &x)
{
    const int lane = lane_id();
    const int32_t X1L = wave_shr1_z(X1);  // lane 0: 0 (t = 0 has no extension)
    const bool i0 = Pex + c.cIb1 + 2 > hp0, i1 = ex1 + c.cIb1 > hp1;
    const uint32_t iext0 = Pex > X1L ? 8u : 0u, iext1 = Pex > X0 ? 8u : 0u;
    const uint32_t hc0 = i0 ? HC_INS : d0 ? HC_DEL : mp0 ? HC_MPRED : HC_MSRC;
    const uint32_t hc1 = i1 ? HC_INS : d1 ? HC_DEL : mp1 ? HC_MPRED : HC_MSRC;
    uint32_t w0 = hc0 | A.dx0 | iext0 | (A.ms0 & 0x70u) | (A.ds0 & 0x80u);
    uint32_t w1 = hc1 | A.dx1 | iext1 | (A.ms1 & 0x70u) | (A.ds1 & 0x80u);
    if (cold && ((info & kInfoFar) || (info >> 8) >= 3u)) row_slots(z, rc, r, info, A);
    // free-end candidates (SPEC.md §3.5) on H': e = H' + 2j - 2m - 1 = X + eb
    // (x.em1 carries -kXBias), and H' at j = m - 1 (+3)
    const int32_t eb = (off << 1) + x.em1;
    if (FULL) {
        int32_t e01;
        uint32_t c1;
        if (__builtin_expect(off == lim, 0)) {
            // the band meets the read's end: cell 127 is j = m - 1
            const int32_t X1e = writelane(X1, __builtin_amdgcn_readlane(X1, 63) + 3, 63);
            c1 = X1e > X0 ? 1u : 0u;
            e01 = max(X0, X1e) + eb;
        } else {
            c1 = X1 > X0 ? 1u : 0u;
            e01 = xm + eb;
        }
        // the lane's cell 1 only if strictly better, then against the best
        // so far (rows come in order: the first maximum is the earliest)
        if (e01 > bE) bE = e01, bKey = r * 2 + c1;
    } else {
        int32_t e0 = X0 + eb, e1 = X1 + eb;
        if ((uint32_t)c.L2 == m - 1) e0 += 3;
        if ((uint32_t)c.L2 + 1 == m - 1) e1 += 3;
        if ((uint32_t)c.L2 >= m) e0 = INT32_MIN, w0 = 0;
        if ((uint32_t)c.L2 + 1 >= m) e1 = INT32_MIN, w1 = 0;
        const bool c1 = e1 > e0;
        const int32_t e01 = c1 ? e1 : e0;
        if (e01 > bE) bE = e01, bKey = r * 2 + (c1 ? 1u : 0u);
    }
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(w0 | (w1 << 8)), rc, (((uint32_t)lane * 2u + x.rot) & 127u) + x.ioff,
                                          x.sbase, 0);
}

// helper wave: everything after the predecessor terms of row r (SPEC.md
// §3.2-§3.5): M, H', the insertion scan, the cell codes and tags, the
// free-end candidates, the record store
template <bool FULL>
__device__ __forceinline__ void dpB_tail(Z &z, BState &S, uint32_t r, uint32_t m, int32_t lim, int32_t off, uint32_t qp,
                                         uint32_t base, uint32_t info, const PredAcc &A, const LaneK &c)
{
    const int lane = lane_id();
    const int32_t srcu = c.src0 + kE * off;
    const int32_t src0 = (off == 0 && lane == 0) ? 0 : srcu;
    const bool mp0 = A.Mh0 >= src0, mp1 = A.Mh1 >= srcu + kE;
    // M as wave 0 computed it (same predecessor terms, same read codes)
    const int32_t M0 = max(A.Mh0, src0) + ((qp & 3u) == base ? kMs : kXs);
    const int32_t M1 = max(A.Mh1, srcu + kE) + (((qp >> 2) & 3u) == base ? kMs : kXs);
    const bool d0 = A.Dv0 > M0, d1 = A.Dv1 > M1;
    const int32_t hp0 = max(M0, A.Dv0), hp1 = max(M1, A.Dv1);
    // insertions (SPEC.md §3.4): the same prefix-max scan as wave 0's
    const int32_t X0 = hp0 + c.L4, X1 = hp1 + c.L4 + 2;
    const int32_t Pex = wave_shr1(kNeg, wave_incl_max(max(X0, X1)));
    row_record<FULL>(z, S.bE, S.bKey, S.bOff, S.rc, r, m, lim, off, info, true, A, c, mp0, mp1, d0, d1, hp0, hp1, X0, X1,
                     Pex, row_x(r, m));
}

// helper wave: the decision bits of one row (wave 0 wrote its ring row and
// {M, Pex}).  Output per cell, 16 bits: code (SPEC.md §3.4) | M tag << 4 |
// D tag << 10; a tag is the distance to the predecessor the cell's M / D
// came from (its slot on rows flagged far).  The row's 64 words go straight
// to HBM (256 B, one store).
template <bool FULL>
__device__ __forceinline__ void dpB_row(Z &z, BState &S, uint32_t r, uint32_t m, int32_t lim, int32_t vOff,
                                        const LaneK &c)
{
    const int lane = lane_id();
#ifdef CCSX_DP_STAMPS
    unsigned long long t_prev = stamp();
#endif
    const int li = (int)(r & 63u);
    const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)S.W.cur.info, li);
    const uint32_t np = info >> 8;
    const int32_t off = __builtin_amdgcn_readlane(vOff, li);
    const uint32_t qp = win_codes(rd_win16(z, off, z.hbm && win_has(S.wc0, S.wnc, off)), off, 0);
    const RingT *dv = reinterpret_cast<const RingT *>(z.lds + kLdsRing) + (r % kRingA) * kRowW + kDc + c.L2;
    PredAcc A;
    A.Dv0 = dv[0], A.Dv1 = dv[1];
    const uint32_t tg = row_tag(S.W.cur, li, 0);
    const uint32_t p0 = r - 1u - (tg & 15u);
    const int32_t sh = off - __builtin_amdgcn_readlane(vOff, (int)(p0 & 63u));
    if (__builtin_expect(np == 1 && (uint32_t)(sh + 3) <= 7u && !(info & kInfoFar), 1)) {
        // one predecessor in the padded band: its H at t-1, t, t+1; D-ext is
        // D > H + O + E (D = max(H + O + E, D' + E))
        const RingT *row = reinterpret_cast<const RingT *>(z.lds + kLdsRing) + (p0 % kRingA) * kRowW;
        const RingT *b = row + (kHc - 1) + c.L2 + sh;  // cell 2l + sh - 1
        // three ds_read_b32 at a 2-word lane stride: a 2-way bank conflict
        // each.  (A variant with one aligned ds_read_b64 per lane and
        // the third cell by DPP cut SQ_LDS_BANK_CONFLICT 1.54e9 -> 1.12e9
        // per launch but ran 1.5 % slower: the parity branch and edge-lane
        // read cost the near-critical helpers more; tools/gpu_lds_ab.sh r02y)
        const int32_t hA = b[0], hB = b[1], hC = b[2];
        A.Mh0 = hA, A.Mh1 = hB;
        A.ms0 = A.ms1 = A.ds0 = A.ds1 = tg;
        A.dx0 = A.Dv0 > hB + (kO + kE) ? 4u : 0u;
        A.dx1 = A.Dv1 > hC + (kO + kE) ? 4u : 0u;
        DP_STAMP(kPfSpare2);
    } else {
        dpB_cold(z, S, r, info, off, vOff, A);
        DP_STAMP(kPfSpare3);
    }
    dpB_tail<FULL>(z, S, r, m, lim, off, qp, info & 3u, info, A, c);
    DP_STAMP(kPfFlush);
}

// helper wave h: rows r0 + h + 2i of the block [r0, r0 + kBlkAB); wave 1 also
// writes the row meta words {band offset | far << 31} of each 16-row group
template <bool FULL>
__device__ __forceinline__ void dpB_block(Z &z, BState &S, uint32_t r0, uint32_t m, uint32_t h, int32_t vOff)
{
    const int lane = lane_id();
    const uint32_t R = z.R;
    const int32_t lim = FULL ? (int32_t)m - kW : 0;
    const LaneK c = lane_consts(lane);
    recwin_begin(z, S.W, r0);
#pragma unroll
    for (uint32_t i = h; i < (uint32_t)kBlkAB; i += kHelperStep)
        if (r0 + i < R) dpB_row<FULL>(z, S, r0 + i, m, lim, vOff, c);
    const uint32_t rend = r0 + kBlkAB < R ? r0 + kBlkAB : R;
    if (h == 0 && ((r0 & 15u) == 16u - kBlkAB || rend == R)) {
        const uint32_t g0 = r0 & ~15u;
        const auto rm = brsrc(reinterpret_cast<uint32_t *>(z.ws + z.L.rmeta) + g0, (rend - g0) * 4);
        __builtin_amdgcn_raw_buffer_store_b32(rmeta_word((uint32_t)vOff, S.W.cur.info, S.W.cur.dpk), rm,
                                              (uint32_t)(lane - (int)(g0 & 63u)) * 4u, 0, 0);
    }
    recwin_end(S.W, r0);
}

__device__ __forceinline__ uint32_t dp_nblk(uint32_t R) { return (R + kBlkAB - 1) / kBlkAB; }

// wave 0's side of a DP (the helpers are in dp_helper)
template <bool FULL>
__device__ __forceinline__ void dp_two_wave(Z &z, uint32_t m, uint32_t &er_out, uint32_t &ej_out)
{
    const int lane = lane_id();
    for (int i = lane; i < kRingA * 16; i += 64) {
        const int k = i & 15;
        const int w = k < 4 ? k : k < 8 ? kHc + kW + (k - 4) : k < 12 ? kDc - 4 + (k - 8) : kDc + kW + (k - 12);
        reinterpret_cast<RingT *>(z.lds + kLdsRing)[(i >> 4) * kRowW + w] = ring_val(k < 8 ? kNegH : kNeg);
    }
    volatile DpJob *job = dp_job(z);
    if (z.hbm) {  // the read's first two window chunks
        z.wa = 0, z.wpend = false;
        win_load(z, 0);
        win_load(z, 1);
    }
    if (lane == 0) job->kind = kJobDp, job->m = m, job->R = z.R, job->cur = (uint32_t)z.cur, job->win = 0;
    __syncthreads();  // J: job posted
    AState S;
    S.H0 = S.H1 = kNegH, S.D0 = S.D1 = kNeg;
    S.pOff = 0, S.pArg = 0, S.vOff = 0, S.vKey = 0, S.ring = 0;
    S.qn = rd_win16(z, 0, true);
    S.nspill = 0;
    S.W.cur = RowPre{0, 0};
    S.W.nxt = S.W.cur;
    const uint32_t nblk = dp_nblk(z.R);
#ifdef CCSX_DP_STAMPS
    unsigned long long t_prev = stamp();
#endif
    for (uint32_t b = 0; b <= nblk; ++b) {
        if (b < nblk) {
            if (z.hbm && z.wpend) {  // the slide published at the last barrier
                win_load(z, z.wa + 1);
                z.wpend = false;
            }
            dpA_block<FULL>(z, S, b * kBlkAB, m);
            if (z.hbm) {
                // the block's last band entered the upper chunk: slide
                z.wpend = (uint32_t)S.pOff >= (z.wa + 1) * kWinChunk;
                z.wa += z.wpend ? 1u : 0u;
                if (lane == 0) job->win = z.wa << 1 | (z.wpend ? 1u : 0u);
            }
        }
        DP_STAMP(kPfAbusy);
        lds_barrier();
        DP_STAMP(kPfAwait);
    }
    // the two helpers' candidates cover disjoint rows: max score, then min row
    int32_t bst;
    if (kHelpers == 1) {
        er_out = uni(job->res[0].er);
        ej_out = uni(job->res[0].ej);
        bst = uni(job->res[0].status);
    } else {
        const int32_t b0 = uni(job->res[0].best), b1 = uni(job->res[1].best);
        const uint32_t r0 = uni(job->res[0].er), r1 = uni(job->res[1].er);
        const bool second = b1 > b0 || (b1 == b0 && r1 < r0);
        er_out = second ? r1 : r0;
        ej_out = second ? uni(job->res[1].ej) : uni(job->res[0].ej);
        const int32_t s0 = uni(job->res[0].status), s1 = uni(job->res[1].status);
        bst = s0 ? s0 : s1;
    }
    if (bst && !z.status) z.status = bst;
    z.cells += (unsigned long long)z.R * (m < (uint32_t)kW ? m : (uint32_t)kW);
}

// helper wave h's side of one DP
template <bool FULL>
__device__ __forceinline__ void dp_wave_b(Z &z, uint32_t m, uint32_t h)
{
    const int lane = lane_id();
    BState S;
    S.bE = INT32_MIN, S.bKey = 0, S.bOff = 0;
    S.wc0 = 0, S.wnc = 2;
    S.W.cur = RowPre{0, 0};
    S.W.nxt = S.W.cur;
    S.rc = rec_rsrc(z);
    z.nfar = h;
    const uint32_t nblk = dp_nblk(z.R);
#ifdef CCSX_DP_STAMPS
    unsigned long long t_prev = stamp();
#endif
    // period b: the decision bits of block b-1
    for (uint32_t b = 0; b <= nblk; ++b) {
        if (z.hbm) {  // the window state wave 0 published at the last barrier
            const uint32_t w = uni(dp_job(z)->win);
            S.wc0 = w >> 1, S.wnc = (w & 1u) ? 1u : 2u;
        }
        if (b >= 1 && !z.status) dpB_block<FULL>(z, S, (b - 1) * kBlkAB, m, h, z.lds[kLdsOffRing + lane]);
        if (b == nblk) {
            // this wave's candidate: lexicographic (max score, min row, min j)
            const int32_t best = wave_max(S.bE);
            const uint32_t rsel = S.bE == best ? S.bKey >> 1 : 0x7FFFFFFFu;
            const int32_t rmin = wave_min((int32_t)rsel);
            const bool mine = S.bE == best && (S.bKey >> 1) == (uint32_t)rmin;
            const int32_t jsel = mine ? S.bOff + 2 * lane + (int32_t)(S.bKey & 1u) : INT32_MAX;
            const int32_t jmin = wave_min(jsel);
            wsync();  // records and row meta in HBM before wave 0 reads them
            volatile DpJob *job = dp_job(z);
            if (lane == 0) {
                job->res[h].best = best;
                job->res[h].er = best == INT32_MIN ? 0xFFFFFFFFu : (uint32_t)rmin;
                job->res[h].ej = (uint32_t)jmin;
                job->res[h].status = z.status;
            }
        }
        DP_STAMP(kPfBbusy);
        lds_barrier();
        DP_STAMP(kPfBwait);
    }
}

// ----------------------------------------------------------------------------
// The solo configuration (kHelpers == 0): one wave per ZMW.  For slices of
// many thousands of ZMWs the launch is bound by how many ZMW chains each SIMD
// holds, not by one chain's latency (config D: 150 / 200 / 222 / 244 GCUPS
// at 4 / 6 / 7 / 8 two-wave workgroups per CU, profiles/r03/r03m_*).  A
// one-wave workgroup needs 16 waves' registers per CU for 16 ZMWs and, with
// no helper lagging behind, a ring of only kRing rows (8: 8.7 KB), so about
// 15 ZMWs are resident per CU instead of 8.  The wave computes each row's
// decision bits itself, from the values it already holds (the helpers
// recompute them from the ring): the cell codes, D-ext / I-ext, predecessor
// tags, the free-end candidates and the record store of dpB_tail, bit for
// bit the same records.
// ----------------------------------------------------------------------------
struct SolB {
    int32_t bE;       // best free-end value of this lane's cells
    uint32_t bKey;    // its row * 2 + cell (the row's band offset: row meta)
    __amdgpu_buffer_rsrc_t rc;  // cell records of this DP (R rows x 256 B)
};

// (the solo wave's S.pArg is the next band offset before clamping, off + 64 -
// (key & 127) = the row max's position + 1 - W / 2: the scalar chain from the
// row key to the next row's fast / cold branch is and, sub, max, min, sub,
// min, lshr, and, cmp)
template <bool FULL>
__device__ __forceinline__ void dpS_row(Z &z, AState &S, SolB &B, uint32_t r, int32_t lim, uint32_t m, const LaneK &c,
                                        uint32_t ring, const RowX &x)
{
    const int lane = lane_id();
    const int li = (int)(r & 63u);
    const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)S.W.cur.info, li);
    const uint32_t base = info & 3u;
    const uint32_t np = info >> 8;
    const int32_t coff = min(max(S.pArg, 0), lim);
    const int32_t sh = coff - S.pOff;
    // fast: a plain chain row whose band moved by 0 or 1 (integer arithmetic
    // only: a bool of the band test lowered to lane-mask selects and a vcc
    // branch, 0.7-0.8 % on D / E16k, r04za; a test of sh | flag < 2 made the
    // compiler merge the two band moves' paths, 176-2,400 VGPR spills)
    const uint32_t fast = (3u >> min((uint32_t)sh, 2u)) & x.chn;
    // everything after the predecessor terms: the recurrence (dpA_row's
    // tail) and the decision bits (dpB_tail's) from the same values;
    // instantiated on both sides of the fast / cold branch, so a fast row's
    // tags are constants and it meets no further branch
    int32_t row_key = 0;  // the row's key (readlane of the max-scan), for the offset / key vectors after the branch
    auto tail = [&](int32_t off, uint32_t qp, const PredAcc &A, bool cold) __attribute__((always_inline)) {
        // the next row's read window, a row ahead of its use
        S.qn = rd_win16(z, off, z.hbm && win_has(z.wa, 2, off));
        const int32_t j0 = off + c.L2;  // < 2^22 + 128 (dp_align): 24-bit multiplies
        // the source terms (SPEC.md §3.2) O + E j, 0 at j = 0: cell 0's is
        // max((O + E) j, O + E j) for every j >= 0 (O < 0), folded into M's
        // max as one max3 (mp: the predecessor term is that max); cell 1's j
        // is never 0 (round 5: a min / select chain of 7 VALU per row)
        const int32_t src1 = mad24<kE, kO + kE>(j0);
        const int32_t Mx0 = max(max(A.Mh0, mul24<kO + kE>(j0)), mad24<kE, kO>(j0));
        const bool mp0 = Mx0 == A.Mh0, mp1 = A.Mh1 >= src1;
        const int32_t M0 = Mx0 + ((qp & 3u) == base ? kMs : kXs);
        const int32_t M1 = max(A.Mh1, src1) + (((qp >> 2) & 3u) == base ? kMs : kXs);
        int32_t Dv0 = A.Dv0, Dv1 = A.Dv1;
        const bool d0 = Dv0 > M0, d1 = Dv1 > M1;
        const int32_t hp0 = max(M0, Dv0), hp1 = max(M1, Dv1);
        // X biased by kXBias (LaneK): positive for every real H'
        const int32_t X0 = hp0 + c.L4 + kXBias, X1 = hp1 + (c.L4 + 2) + kXBias;
        const int32_t xm = max(X0, X1);  // the lane's larger X: the scan's input, its free-end candidate
        int32_t rk0 = (hp0 << 7) | c.kc0, rk1 = (hp1 << 7) | c.kc1;
        if (!FULL) {
            if ((uint32_t)c.L2 >= m) rk0 = INT32_MIN, Dv0 = kNeg;
            if ((uint32_t)c.L2 + 1 >= m) rk1 = INT32_MIN, Dv1 = kNeg;
        }
        int32_t rk = max(rk0, rk1);
        // the insertion scan's first step reads 0 (the bound control) where
        // row_shr has no source: max(0, X) = X, and its result goes to a new
        // register (xm stays); the row-key scan as before
        int32_t incl = max(xm, __builtin_amdgcn_update_dpp(0, xm, 0x111, 0xF, 0xF, true));
        incl = dpp_max<0x112>(incl);
        incl = dpp_max<0x114>(incl);
        incl = dpp_max<0x118>(incl);
        incl = dpp_max<0x142, 0xA>(incl);
        incl = dpp_max<0x143, 0xC>(incl);
        rk = wave_incl_max(rk);
        // exclusive prefix max; lane 0 gets 0, below every biased X: its cell
        // 0 insertion term Pex + cIb1 + 2 is -kXBias - 3, i.e. I(0) = NEG
        const int32_t Pex = wave_shr1_z(incl);
        const int32_t ex1 = max(Pex, X0);
        int32_t nH0 = max(Pex + c.cIb1 + 2, hp0), nH1 = max(ex1 + c.cIb1, hp1);
        if (!FULL) {
            if ((uint32_t)c.L2 >= m) nH0 = kNegH;
            if ((uint32_t)c.L2 + 1 >= m) nH1 = kNegH;
        }
        const int32_t key = __builtin_amdgcn_readlane(rk, 63);
        RingT *row = reinterpret_cast<RingT *>(z.lds + kLdsRing) + ring + kHc + c.L2;
        ring_store2(row, nH0, nH1);
        ring_store2(row + (kDc - kHc), Dv0, Dv1);
        row_key = key;
        if (cold && (info & kInfoSpill)) {
            // a successor lies beyond the ring: keep this row in HBM
            const uint32_t sl = S.nspill++;
            if (sl < z.d.scap) {
                int32_t *rec = reinterpret_cast<int32_t *>(z.ws + z.L.spill + (size_t)sl * kSpillRec);
                reinterpret_cast<int2 *>(rec)[lane] = make_int2(nH0, nH1);
                reinterpret_cast<int2 *>(rec + kW)[lane] = make_int2(Dv0, Dv1);
                if (lane == 0) rec[256] = off, rec[257] = key, P<uint32_t>(z, z.L.sslot)[r] = sl;
            } else {
                z.status = kErrSpill;
            }
        }
        S.H0 = nH0, S.H1 = nH1, S.D0 = Dv0, S.D1 = Dv1;
        S.pOff = off;
        S.pArg = off + kW / 2 - (key & 127);
        // decision bits, free-end candidates, record (only a cold row can
        // have more than 63 predecessors)
        row_record_solo<FULL>(z, B.bE, B.bKey, B.rc, r, m, lim, off, info, cold, A, c, mp0, mp1, d0, d1, hp0, hp1, X0, X1,
                              xm, Pex, ex1, x);
    };
    if (__builtin_expect(fast, 1)) {
        // the only predecessor is row r - 1 (tag 1), band moved by 0 or 1:
        // its cells from registers by DPP; D-ext = the D term won strictly
        PredAcc A;
        A.ms0 = A.ms1 = A.ds0 = A.ds1 = kTagPrev;
        int32_t a0, b0, a1, b1;
        // the tail instantiated per band move: no join of the predecessor
        // terms (whose register copies cost ~5 VALU per row; E16k -0.4 %, r04zd)
        if (sh == 0) {
            A.Mh0 = wave_shr1(kNegH, S.H1), A.Mh1 = S.H0;
            a0 = S.H0 + (kO + kE), b0 = S.D0 + kE, a1 = S.H1 + (kO + kE), b1 = S.D1 + kE;
            A.Dv0 = max(a0, b0), A.Dv1 = max(a1, b1);
            A.dx0 = b0 > a0 ? 4u : 0u, A.dx1 = b1 > a1 ? 4u : 0u;
            tail(coff, win_codes(S.qn, S.pOff, 0), A, false);
        } else {
            A.Mh0 = S.H0, A.Mh1 = S.H1;
            a0 = S.H1 + (kO + kE), b0 = S.D1 + kE;
            a1 = wave_shl1(kNegH, S.H0) + (kO + kE), b1 = wave_shl1(kNeg, S.D0) + kE;
            A.Dv0 = max(a0, b0), A.Dv1 = max(a1, b1);
            A.dx0 = b0 > a0 ? 4u : 0u, A.dx1 = b1 > a1 ? 4u : 0u;
            tail(coff, win_codes(S.qn, S.pOff, 1), A, false);
        }
    } else {
        PredAcc A;
        int32_t off;
        int kind;
        dpA_cold<true>(z, S, r, info, coff, lim, off, A, kind);
        (void)kind;
        const uint32_t d = (uint32_t)(off - S.pOff);
        const uint32_t qp = d <= 3u ? win_codes(S.qn, S.pOff, (int32_t)d)
                                    : win_codes(rd_win16(z, off, z.hbm && win_has(z.wa, 2, off)), off, 0);
        tail(off, qp, A, true);
    }
    // one writelane pair after the fast / cold join (inside each branch the
    // tied operands cost two register copies per row: E16k -0.7 %, r04zb)
    S.vOff = writelane(S.vOff, S.pOff, li);
    S.vKey = writelane(S.vKey, row_key, li);
#ifdef CCSX_PAD_VALU  // (measurement variant: N extra VALU per row -- is the row VALU-issue bound?)
    {
        int32_t v = lane;
#pragma unroll
        for (int k = 0; k < CCSX_PAD_VALU; ++k) asm volatile("v_add_u32 %0, %0, 1" : "+v"(v));
    }
#endif
#ifdef CCSX_PAD_SALU  // (measurement variant: N extra SALU per row)
    {
        uint32_t a = r, b = (uint32_t)li;
#pragma unroll
        for (int k = 0; k < CCSX_PAD_SALU / 2; ++k) asm volatile("s_mov_b32 %0, %1\n\ts_mov_b32 %1, %0" : "+s"(a), "+s"(b));
    }
#endif
}

// rows [r0, r0 + kBlkAB) and, per 16-row group, the row meta words {band
// offset | far << 31} the traceback reads (helper 0's job in dpB_block)
template <bool FULL>
__device__ __forceinline__ void dpS_block(Z &z, AState &S, SolB &B, uint32_t r0, uint32_t m)
{
    const int lane = lane_id();
    const uint32_t R = z.R;
    const int32_t lim = FULL ? (int32_t)m - kW : 0;
    const LaneK c = lane_consts(lane);
    recwin_begin(z, S.W, r0);
    if ((r0 & 63u) == 0) {
        const uint32_t inf = S.W.cur.info;
        S.fmask = ballot((inf & (kInfoChain | kInfoFar | kInfoSpill)) == kInfoChain);
    }
    // the rows' ring slots: consecutive from r0's (kBlkAB divides kRingA), or
    // (a block of several ring lengths, r0 a multiple of kRingA) i mod kRingA
    static_assert(kRingA % kBlkAB == 0 || kBlkAB % kRingA == 0, "a block's rows take constant ring slots");
    const uint32_t rb = (r0 % (uint32_t)kRingA) * (uint32_t)kRowW;
    // per row of the block: bit i of fm = row r0 + i is a plain chain row;
    // tb_rot(r0 + i) = tb_rot(r0) + 4 i (r0 is a multiple of kBlkAB)
    static_assert(kBlkAB <= 16 && 32 % kBlkAB == 0, "a block's rows share tb_rot's 32-row period");
    const uint32_t fm = (uint32_t)(S.fmask >> (r0 & 63u));
    const uint32_t rot0 = tb_rot(r0);
    const int32_t em1 = -2 * (int32_t)m - 1 - kXBias;  // (row_record_solo: X is biased)
    if (r0 + kBlkAB <= R) {
#pragma unroll
        for (uint32_t i = 0; i < (uint32_t)kBlkAB; ++i)
            dpS_row<FULL>(z, S, B, r0 + i, lim, m, c, rb + (i % (uint32_t)kRingA) * kRowW,
                          RowX{(fm >> i) & 1u, rot0 + 4u * i, kRecRow * i, r0 * kRecRow, em1});
    } else {
        for (uint32_t i = 0; r0 + i < R; ++i)
            dpS_row<FULL>(z, S, B, r0 + i, lim, m, c, rb + (i % (uint32_t)kRingA) * kRowW,
                          RowX{(fm >> i) & 1u, rot0 + 4u * i, kRecRow * i, r0 * kRecRow, em1});
    }
    const uint32_t rend = r0 + kBlkAB < R ? r0 + kBlkAB : R;
    if ((r0 & 15u) == 16u - kBlkAB || rend == R) {
        const uint32_t g0 = r0 & ~15u;
        const auto rm = brsrc(reinterpret_cast<uint32_t *>(z.ws + z.L.rmeta) + g0, (rend - g0) * 4);
        __builtin_amdgcn_raw_buffer_store_b32(rmeta_word((uint32_t)S.vOff, S.W.cur.info, S.W.cur.dpk), rm,
                                              (uint32_t)(lane - (int)(g0 & 63u)) * 4u, 0, 0);
    }
    recwin_end(S.W, r0);
}

template <bool FULL>
__device__ __forceinline__ void dp_solo(Z &z, uint32_t m, uint32_t &er_out, uint32_t &ej_out)
{
    const int lane = lane_id();
    for (int i = lane; i < kRingA * 16; i += 64) {
        const int k = i & 15;
        const int w = k < 4 ? k : k < 8 ? kHc + kW + (k - 4) : k < 12 ? kDc - 4 + (k - 8) : kDc + kW + (k - 12);
        reinterpret_cast<RingT *>(z.lds + kLdsRing)[(i >> 4) * kRowW + w] = ring_val(k < 8 ? kNegH : kNeg);
    }
    if (z.hbm) {  // the read's first two window chunks
        z.wa = 0, z.wpend = false;
        win_load(z, 0);
        win_load(z, 1);
    }
    AState S;
    S.H0 = S.H1 = kNegH, S.D0 = S.D1 = kNeg;
    S.pOff = 0, S.pArg = 0, S.vOff = 0, S.vKey = 0, S.ring = 0;
    S.qn = rd_win16(z, 0, true);
    S.nspill = 0;
    S.W.cur = RowPre{0, 0};
    S.W.nxt = S.W.cur;
    SolB B;
    B.bE = INT32_MIN, B.bKey = 0;
    B.rc = rec_rsrc(z);
    z.nfar = 0;
    const uint32_t nblk = dp_nblk(z.R);
    for (uint32_t b = 0; b < nblk && !z.status; ++b) {
        if (z.hbm && z.wpend) {
            win_load(z, z.wa + 1);
            z.wpend = false;
        }
        dpS_block<FULL>(z, S, B, b * kBlkAB, m);
        if (z.hbm) {  // the block's last band entered the upper chunk: slide
            z.wpend = (uint32_t)S.pOff >= (z.wa + 1) * kWinChunk;
            z.wa += z.wpend ? 1u : 0u;
        }
    }
    // the candidate: lexicographic (max score, min row, min j)
    const int32_t best = wave_max(B.bE);
    const uint32_t rsel = B.bE == best ? B.bKey >> 1 : 0x7FFFFFFFu;
    const int32_t rmin = wave_min((int32_t)rsel);
    const bool mine = B.bE == best && (B.bKey >> 1) == (uint32_t)rmin;
    wsync();  // records and row meta in HBM before the traceback's DMA (and the load below) reads them
    // the winning row's band offset from the row meta (L1 bypassed: this
    // wave's stores went to L2)
    int32_t boff = 0;
    if (best != INT32_MIN) {
        const auto rm = brsrc(reinterpret_cast<uint32_t *>(z.ws + z.L.rmeta), z.R * 4u);
        boff = (int32_t)(uni(__builtin_amdgcn_raw_buffer_load_b32(rm, (uint32_t)rmin * 4u, 0, 1)) & kMetaOff);
    }
    const int32_t jsel = mine ? boff + 2 * lane + (int32_t)(B.bKey & 1u) : INT32_MAX;
    er_out = best == INT32_MIN ? 0xFFFFFFFFu : (uint32_t)rmin;
    ej_out = (uint32_t)wave_min(jsel);
    z.cells += (unsigned long long)z.R * (m < (uint32_t)kW ? m : (uint32_t)kW);
}

template <int LM>
__device__ __forceinline__ void merge(Z &z, uint32_t k, uint32_t m, uint32_t tid);
__device__ __forceinline__ void columns_count(const Z &z, uint32_t n, uint32_t ncols, uint32_t tid, uint32_t T);
__device__ __forceinline__ int merge_in_lds(uint32_t R);

// helper wave h (1 + h = wave index): serve DP and merge jobs until wave 0
// posts kJobExit
__device__ __forceinline__ void dp_helper(Z &z, uint32_t h)
{
    for (;;) {
        __syncthreads();  // J: job posted
        volatile DpJob *job = dp_job(z);
        const int32_t kind = uni(job->kind);
        if (kind == kJobExit) break;
        z.R = uni(job->R);
        z.cur = uni((int)job->cur);
        z.status = kOk;
        const uint32_t m = uni(job->m);
        if (kind == kJobColumns) {
            __syncthreads();  // columns numbered by wave 0
            columns_count(z, m, uni(job->K), threadIdx.x, kBlockThreads);
            __syncthreads();
            continue;
        }
        if (kind == kJobMerge) {
            // merge's row-parallel phases are on the critical path: raise the
            // helpers above other workgroups' DP helpers (below any wave 0)
            __builtin_amdgcn_s_setprio(kPrioMerge);
            const int lm = merge_in_lds(z.R);
            if (lm == 2) merge<2>(z, uni(job->k), m, threadIdx.x);
            else if (lm == 1) merge<1>(z, uni(job->k), m, threadIdx.x);
            else merge<0>(z, uni(job->k), m, threadIdx.x);
            __builtin_amdgcn_s_setprio(0);
        }
        else if (m >= (uint32_t)kW) dp_wave_b<true>(z, m, h);
        else dp_wave_b<false>(z, m, h);
    }
}

__device__ __forceinline__ void dp_helper_exit(Z &z)
{
    if (lane_id() == 0) dp_job(z)->kind = kJobExit;
    __syncthreads();
    // the helper waves hand over their diagnostic counters
    __syncthreads();
    const volatile unsigned long long *pf1 = reinterpret_cast<const volatile unsigned long long *>(z.lds + kLdsDiag);
    for (int h = 0; h < kHelpers; ++h) {
        z.pf[kPfBbusy] += pf1[8 * h + 0];
        z.pf[kPfBwait] += pf1[8 * h + 1];
        z.pf[kPfSpare2] += pf1[8 * h + 2];
        z.pf[kPfSpare3] += pf1[8 * h + 3];
        z.pf[kPfFlush] += pf1[8 * h + 4];
        z.pf[kPfHw1 + h] = pf1[8 * h + 5];
    }
}

// placement of the calling wave: HW_ID (wave, SIMD, CU, SE) | XCC_ID << 32
__device__ __forceinline__ unsigned long long wave_hw_id()
{
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    return (unsigned long long)hw | (unsigned long long)xcc << 32;
}

__device__ __forceinline__ void dp_align(Z &z, uint32_t m, uint32_t &er_out, uint32_t &ej_out)
{
    er_out = ej_out = 0;
    // keys of the row-max scan need |H'| < 2^24; the int16 ring, reads of at
    // most kRing16MaxRead bases (the host never sends longer ones to it)
    if (m >= (1u << 22) || (sizeof(RingT) == 2 && m > kRing16MaxRead)) {
        z.status = kErrReadLen;
        return;
    }
    z.pf[kPfTwRows] += z.R;
    if (kHelpers == 0) {
        if (m >= (uint32_t)kW) dp_solo<true>(z, m, er_out, ej_out);
        else dp_solo<false>(z, m, er_out, ej_out);
    } else {
        if (m >= (uint32_t)kW) dp_two_wave<true>(z, m, er_out, ej_out);
        else dp_two_wave<false>(z, m, er_out, ej_out);
    }
}

// ----------------------------------------------------------------------------
// SPEC.md §4: traceback into one event per read base.  The wave walks the
// 8-bit cell records of the DP (row_record: code | D-ext | I-ext | M tag | D
// tag) backwards in blocks of rows staged in LDS by DMA.  The band offsets of
// the staged block sit in one VGPR (readlane); events collect in a VGPR,
// lane j & 63, stored 64 at a time.
// ----------------------------------------------------------------------------
// rows per staged record block: 32, or 16 (the int16-ring objects: two 16-row
// blocks of 2 KiB, the next one loaded while the current one is walked, in
// the 4,352 B ring area)
#ifndef CCSX_TB_ROWS
#define CCSX_TB_ROWS 32
#endif
constexpr uint32_t kTbRows = CCSX_TB_ROWS;
static_assert(kTbRows == 32 || kTbRows == 16, "record blocks of 16 or 32 rows");
constexpr uint32_t kTbBufWords = kTbRows * kRecRow / 4;  // kTbRows rows x 128 B
// record blocks staged at once: two (the next block's DMA overlaps the walk
// of the current one) where the DP ring area holds them, else one (a block
// switch waits for its DMA, which the other ZMWs resident on the SIMD cover);
// after the blocks, 32 row meta words per buffer
#ifdef CCSX_TB_BUFS
constexpr uint32_t kTbBufs = CCSX_TB_BUFS;
#else
constexpr uint32_t kTbBufs = (uint32_t)kRingWords >= 2 * (kTbBufWords + 32) ? 2u : 1u;
#endif
// CCSX_TB_TAGS=1: the blocks' tag-plane rows staged beside them where the area
// holds both (measurement variant: it saved the latency objects' serial walk
// ~2 us of HBM per escape while every row with a predecessor more than one row
// back escaped through the plane; since rows of one or two predecessors carry
// their distances in the row meta, the extra DMA costs config B 0.7 %, r06z)
#ifdef CCSX_TB_TAGS
constexpr bool kTbTags = CCSX_TB_TAGS && (uint32_t)kRingWords >= kTbBufs * (2 * kTbBufWords + 32);
#else
constexpr bool kTbTags = false;
#endif
constexpr uint32_t kTbTag = kTbBufs * kTbBufWords;  // LDS word of the staged tag-plane rows (kTbTags)
constexpr uint32_t kTbMeta = (kTbTags ? 2 : 1) * kTbBufs * kTbBufWords;  // LDS word of the row meta (32 words per buffer)
static_assert(kTbMeta + kTbBufs * 32 <= (uint32_t)kRingWords, "traceback buffers live in the DP ring area");

// Traceback step tables indexed by (state, cell code), state 0 = H, 1 = D,
// 2 = I; code = hcode | D-ext << 2 | I-ext << 3 (SPEC.md §3.4, §4).
// kTbAct[state]: 4 bits per code {emit, move to the predecessor, j -= 1,
// stop (MSRC)}; kTbNext[state]: the next state (4-bit fields).
constexpr uint32_t tb_act(uint32_t st, uint32_t c)
{
    return st == 0 ? ((c & 3u) == 0 ? 0x7u : (c & 3u) == 1 ? 0x9u : 0u)  // MPRED: emit+pred+dj, MSRC: emit+stop
         : st == 1 ? 0x2u                                               // D: move to the D tag's predecessor
                   : 0x5u;                                              // I: emit INS, j -= 1
}
constexpr uint32_t tb_next(uint32_t st, uint32_t c)
{
    return st == 0 ? ((c & 3u) == 2 ? 1u : (c & 3u) == 3 ? 2u : 0u)
         : st == 1 ? ((c >> 2) & 1u)
                   : (((c >> 3) & 1u) ? 2u : 0u);
}
constexpr uint64_t tb_table(uint32_t st, bool act)
{
    uint64_t v = 0;
    for (uint32_t c = 0; c < 16; ++c) v |= (uint64_t)(act ? tb_act(st, c) : tb_next(st, c)) << (c * 4);
    return v;
}
constexpr uint64_t kTbAct[3] = {tb_table(0, true), tb_table(1, true), tb_table(2, true)};
constexpr uint64_t kTbNext[3] = {tb_table(0, false), tb_table(1, false), tb_table(2, false)};

// LDS-DMA of block bi into buffer buf: records (kTbRows x 128 B) and the row
// meta words (band offset | far << 31) of 32 rows; the data bypass VGPRs, so
// nothing in the walk waits on them until the block is entered (explicit
// s_waitcnt)
__device__ __forceinline__ void tb_dma(const Z &z, uint32_t bi, uint32_t buf)
{
    const uint32_t lane = lane_id();
    const uint8_t *src = z.ws + z.L.codes + (size_t)bi * kTbRows * kRecRow + lane * 16u;
    int32_t *dst = z.lds + buf * kTbBufWords;
#pragma unroll
    for (int k = 0; k < (int)(kTbRows * kRecRow / 1024); ++k)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t *>(src + k * 1024), dst + k * 256, 16, 0, 0);
    if constexpr (kTbTags) {
        const uint8_t *tsrc = z.ws + z.L.dsl + (size_t)bi * kTbRows * kRecRow + lane * 16u;
#pragma unroll
        for (int k = 0; k < (int)(kTbRows * kRecRow / 1024); ++k)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t *>(tsrc + k * 1024),
                                             z.lds + kTbTag + buf * kTbBufWords + k * 256, 16, 0, 0);
    }
    const uint32_t *ms = reinterpret_cast<const uint32_t *>(z.ws + z.L.rmeta) + bi * kTbRows + lane;
    if (lane < 32u) __builtin_amdgcn_global_load_lds(ms, z.lds + kTbMeta + buf * 32, 4, 0, 0);
}

// Plain MPRED steps k..7 of an aligned 8-column record window (traceback;
// columns jw - 1 .. jw - 8 of the staged block's rows): wa holds, at lane l <
// 32 = block row l, columns jw - 1 .. jw - 4 as bytes 0-3, wb columns jw - 5
// .. jw - 8 (tb_win's upper 32 lanes moved down by one v_permlane32_swap), so
// every step reads its record at lane r - base.  Per step, emit ALN | r at
// lane j & 63; leave with st = 1, unmoved, when the cell's M tag is not a row
// distance (a slot: the predecessor is 5+ rows back) or the predecessor lies
// below the block, or, on the window's last column (j = 0 mod 8), when j
// completes a 64-base chunk; else j -= 1, r -= the distance and, below the
// last column, read the next record and leave with st = 2 when it is not
// MPRED.  st = 0: moved past the last column (the caller swaps in the next
// window).  The M tag is -d in 3-bit two's complement: s_bfe_i32 gives -d,
// and li + (-d) carries exactly when the predecessor stays in the block (d <=
// li) -- a slot tag (0..3) never carries -- so a step is 9 instructions, its
// dependent chain s_bfe -> s_add -> v_readlane.  rec on entry: the current
// cell's record (low byte); on exit the record of the cell (r, j) in the low
// byte.  Hand-written: compiled, the multi-exit unrolled loop became a
// flag-driven state machine of ~35 scalar instructions per step.
__device__ __forceinline__ void tb_w8_steps(uint32_t k, uint32_t base, uint32_t wa, uint32_t wb, uint32_t &r,
                                            int32_t &j, uint32_t &rec, uint32_t &vev, uint32_t &st)
{
    uint32_t t, li, c, jh, m0v;
    // the asm's scalar operands must live in SGPRs
    r = uni(r), j = uni(j), rec = uni(rec), k = uni(k), base = uni(base);
// m0 = j & 63 is kept by the walk (the window's columns never cross a
// 64-base chunk: jw = 0 mod 8 and the last column leaves on a completed
// chunk), j rebuilt from it at the exits
#define TBW_HEAD(BFE, SLOW)                              \
    "v_writelane_b32 %[vev], %[r], %[m0]\n\t"            \
    "s_bfe_i32 %[t], %[rec], " BFE "\n\t"                \
    "s_add_u32 %[li], %[li], %[t]\n\t"                   \
    "s_cbranch_scc0 .Ltbw_" SLOW "%=\n\t"
#define TBW_MOVE                                         \
    "s_sub_u32 %[m0], %[m0], 1\n\t"                      \
    "s_add_u32 %[r], %[r], %[t]\n\t"
#define TBW_NEXT(W, CODE, OUT)                           \
    "v_readlane_b32 %[rec], %[" W "], %[li]\n\t"         \
    "s_and_b32 %[c], %[rec], " CODE "\n\t"               \
    "s_cbranch_scc1 .Ltbw_" OUT "%=\n\t"
#define TBW_BYTE(LBL, BFE, TO) \
    ".Ltbw_" LBL "%=:\n\t"     \
    "s_bfe_u32 %[rec], %[rec], " BFE "\n\t" \
    "s_branch .Ltbw_" TO "%=\n"
    asm volatile(
        "s_sub_u32 %[li], %[r], %[base]\n\t"
        "s_and_b32 %[m0], %[j], 63\n\t"
        "s_andn2_b32 %[jh], %[j], 63\n\t"
        "s_cmp_eq_u32 %[k], 0\n\t"
        "s_cbranch_scc1 .Ltbw_0%=\n\t"
        "s_cmp_gt_u32 %[k], 3\n\t"
        "s_cbranch_scc1 .Ltbw_e4%=\n\t"
        "s_cmp_eq_u32 %[k], 1\n\t"
        "s_cbranch_scc1 .Ltbw_e1%=\n\t"
        "s_cmp_eq_u32 %[k], 2\n\t"
        "s_cbranch_scc1 .Ltbw_e2%=\n\t"
        "s_lshl_b32 %[rec], %[rec], 24\n\t"
        "s_branch .Ltbw_3%=\n"
        ".Ltbw_e1%=:\n\t"
        "s_lshl_b32 %[rec], %[rec], 8\n\t"
        "s_branch .Ltbw_1%=\n"
        ".Ltbw_e2%=:\n\t"
        "s_lshl_b32 %[rec], %[rec], 16\n\t"
        "s_branch .Ltbw_2%=\n"
        ".Ltbw_e4%=:\n\t"
        "s_cmp_eq_u32 %[k], 4\n\t"
        "s_cbranch_scc1 .Ltbw_4%=\n\t"
        "s_cmp_eq_u32 %[k], 5\n\t"
        "s_cbranch_scc1 .Ltbw_e5%=\n\t"
        "s_cmp_eq_u32 %[k], 6\n\t"
        "s_cbranch_scc1 .Ltbw_e6%=\n\t"
        "s_lshl_b32 %[rec], %[rec], 24\n\t"
        "s_branch .Ltbw_7%=\n"
        ".Ltbw_e5%=:\n\t"
        "s_lshl_b32 %[rec], %[rec], 8\n\t"
        "s_branch .Ltbw_5%=\n"
        ".Ltbw_e6%=:\n\t"
        "s_lshl_b32 %[rec], %[rec], 16\n\t"
        "s_branch .Ltbw_6%=\n"
        ".Ltbw_0%=:\n\t" TBW_HEAD("0x30004", "s0") TBW_MOVE TBW_NEXT("wa", "0x300", "o1")
        ".Ltbw_1%=:\n\t" TBW_HEAD("0x3000c", "s1") TBW_MOVE TBW_NEXT("wa", "0x30000", "o2")
        ".Ltbw_2%=:\n\t" TBW_HEAD("0x30014", "s2") TBW_MOVE TBW_NEXT("wa", "0x3000000", "o3")
        ".Ltbw_3%=:\n\t" TBW_HEAD("0x3001c", "s3") TBW_MOVE TBW_NEXT("wb", "3", "o4")
        ".Ltbw_4%=:\n\t" TBW_HEAD("0x30004", "s0") TBW_MOVE TBW_NEXT("wb", "0x300", "o1")
        ".Ltbw_5%=:\n\t" TBW_HEAD("0x3000c", "s1") TBW_MOVE TBW_NEXT("wb", "0x30000", "o2")
        ".Ltbw_6%=:\n\t" TBW_HEAD("0x30014", "s2") TBW_MOVE TBW_NEXT("wb", "0x3000000", "o3")
        ".Ltbw_7%=:\n\t" TBW_HEAD("0x3001c", "s3")
        "s_cmp_eq_u32 %[m0], 0\n\t"
        "s_cbranch_scc1 .Ltbw_s3%=\n\t" TBW_MOVE
        "s_mov_b32 %[st], 0\n\t"
        "s_branch .Ltbw_clean%=\n"
        // unmoved (st = 1): the current cell's byte
        TBW_BYTE("s0", "0x80000", "slow")
        TBW_BYTE("s1", "0x80008", "slow")
        TBW_BYTE("s2", "0x80010", "slow")
        TBW_BYTE("s3", "0x80018", "slow")
        // a record that is not MPRED (st = 2): the new cell's byte
        TBW_BYTE("o1", "0x80008", "out")
        TBW_BYTE("o2", "0x80010", "out")
        TBW_BYTE("o3", "0x80018", "out")
        TBW_BYTE("o4", "0x80000", "out")
        ".Ltbw_slow%=:\n\t"
        "s_mov_b32 %[st], 1\n\t"
        "s_branch .Ltbw_clean%=\n"
        ".Ltbw_out%=:\n\t"
        "s_mov_b32 %[st], 2\n"
        ".Ltbw_clean%=:\n\t"
        "s_or_b32 %[j], %[jh], %[m0]\n"
        : [r] "+s"(r), [j] "+s"(j), [rec] "+s"(rec), [vev] "+v"(vev), [st] "=s"(st), [t] "=&s"(t), [li] "=&s"(li),
          [c] "=&s"(c), [jh] "=&s"(jh), [m0] "=&{m0}"(m0v)
        : [k] "s"(k), [base] "s"(base), [wa] "v"(wa), [wb] "v"(wb)
        : "scc");
    // (the divergence analysis takes inline-asm results as divergent: without
    // these, everything downstream of r / j would go to VGPRs and exec masks)
    r = uni(r), j = uni(j), rec = uni(rec), st = uni(st);
#undef TBW_HEAD
#undef TBW_MOVE
#undef TBW_NEXT
#undef TBW_BYTE
}

// the lower 32 lanes of wb <- the upper 32 lanes of the 64-lane window
__device__ __forceinline__ uint32_t tb_wb(uint32_t win)
{
    return (uint32_t)__builtin_amdgcn_permlane32_swap(win, win, false, false)[1];
}

// the M tag of a record: -d (d = 1..4 rows back) or a slot (0..3)
__device__ __forceinline__ int32_t rec_mtag(uint32_t rec) { return (int32_t)(rec << 25) >> 29; }

__device__ __forceinline__ void traceback(Z &z, uint32_t m, uint32_t er, uint32_t ej)
{
    const uint32_t lane = lane_id();
    uint32_t *ev = P<uint32_t>(z, z.L.ev);
    for (uint32_t j = ej + 1 + lane; j < m; j += 64) ev[j] = (EV_INS << 30) | er;
    uint32_t r = er, bi = er / kTbRows, buf = 0, base = bi * kTbRows;
    int32_t j = (int32_t)ej;
    // per staged block, lane l (mod 32) = block row l: voff = its band offset,
    // vrot = (tb_rot - off) & 127, so cell (r, j) sits at byte
    // ((buf * kTbRows + l) << 7) | ((vrot + j) & 127) of the LDS; farm = the
    // block's far rows (their tags are in the far slot records)
    uint32_t voff = 0, vrot = 0, farm = 0;
    // record window of the plain MPRED steps: lane l holds the records of
    // block row l & 31 at columns jw - 1 - 4 (l >> 5) .. jw - 4 - 4 (l >> 5),
    // i.e. eight columns of every staged row; valid while j lies in [jw - 8,
    // jw) (entering a block invalidates it)
    uint32_t vrot32 = 0, rowb32 = 0, win = 0;
    int32_t jw = INT32_MIN / 2;
    // the window below it (columns [jw - 16, jw - 8)), valid while jwn == jw
    uint32_t wnx = 0;
    int32_t jwn = INT32_MAX;
    auto enter = [&]() {
        const uint32_t l = lane & 31u;
        const uint32_t mt = (uint32_t)z.lds[kTbMeta + buf * 32 + l];
        voff = mt;  // (the whole meta word: its band offset is voff & kMetaOff)
        vrot = (tb_rot(base + l) - (mt & kMetaOff)) & 127u;  // (base: a multiple of kTbRows)
        farm = (uint32_t)ballot((mt >> 31) != 0u) & (uint32_t)((1ull << kTbRows) - 1u);
        // lanes 32-63 hold the four columns below lanes 0-31's
        vrot32 = vrot - (lane >> 5) * 4u;
        rowb32 = (buf * kTbRows + (lane & (kTbRows - 1u))) << 7;
        jw = INT32_MIN / 2;
        jwn = INT32_MAX;
    };
    tb_dma(z, bi, buf);
    __builtin_amdgcn_s_waitcnt(0);
    enter();
    if (kTbBufs == 2 && bi) tb_dma(z, bi - 1, buf ^ 1u);
    const auto rev = brsrc(ev, m * 4);
    uint32_t vev = 0;                      // events of bases [chunk, chunk + 64), lane = base & 63
    int32_t chunk = j & ~63;
    uint32_t top = (uint32_t)(j - chunk);  // highest lane of the chunk that is ours (the rest are INS events)
    // a completed chunk waits for the next block switch, so that a switch's
    // wait on the prefetch never waits on a freshly issued store
    uint32_t vpend = 0, pend_top = 0;
    int32_t pend = -1;
    uint32_t lead_row = 0, lead_j = 0;
    int32_t err = 0;
    uint32_t guard = 0;
    const uint32_t glim = z.R * 2u + m * 2u + 16u;
    const uint32_t *poff = G_poff(z, z.cur);
    const uint32_t *pred = G_pred(z, z.cur);
    const uint8_t *lds8 = reinterpret_cast<const uint8_t *>(z.lds);
#ifdef CCSX_TB_COUNTING
    unsigned long long t_prev = stamp();
    unsigned long long tq = t_prev;
#define TB_MARK(slot)                     \
    do {                                  \
        const unsigned long long t_ = stamp(); \
        z.pf[slot] += t_ - tq;            \
        tq = t_;                          \
    } while (0)
#endif
    // stage the block holding row r (a switch to the prefetched neighbour
    // waits only for its DMA)
    auto to_block = [&]() {
#ifdef CCSX_TB_COUNTING
        z.pf[kPfTbNsw] += 1;
        const unsigned long long ts0 = stamp();
#endif
        const uint32_t nb = r / kTbRows;
        if (kTbBufs == 1) {
            // one buffer: the walk's LDS reads of the old block complete,
            // then the new block's DMA.  (An L2 prefetch of the block below,
            // one load per 128 B line on entering a block, measured +1.9 %
            // on config D: A/B r03o; the block below held in 17 VGPRs and
            // written to LDS at the switch, +2.7 % on E16k with the
            // traceback's cycles unchanged: r05n / r05o, commit bf58425)
            __builtin_amdgcn_s_waitcnt(0);
            tb_dma(z, nb, 0u);
        } else {
            if (nb + 1 != bi) {
                __builtin_amdgcn_s_waitcnt(0);
                tb_dma(z, nb, buf ^ 1u);  // not the prefetched neighbour
            }
            buf ^= 1u;
        }
        bi = nb;
        base = bi * kTbRows;
        __builtin_amdgcn_s_waitcnt(0);
        enter();
        if (pend >= 0) {
            __builtin_amdgcn_raw_buffer_store_b32(vpend, rev, lane <= pend_top ? (uint32_t)(pend + (int32_t)lane) * 4u : ~0u,
                                                  0, 0);
            pend = -1;
        }
        if (kTbBufs == 2 && bi) tb_dma(z, bi - 1, buf ^ 1u);
#ifdef CCSX_TB_COUNTING
        const unsigned long long ts1 = stamp();
        z.pf[kPfTbSwitch] += ts1 - ts0;
        t_prev += ts1 - ts0;
#endif
    };
    // the record window of columns [jwv - 8, jwv) of the staged block (layout
    // at vrot32 above: four byte reads per lane, a row's 128 B wrap); the
    // compiler's lgkmcnt wait lands at the first use
    auto tb_win = [&](int32_t jwv) -> uint32_t {
        const uint32_t a = vrot32 + (uint32_t)(jwv - 1);
        const uint32_t b0 = lds8[rowb32 | (a & 127u)];
        const uint32_t b1 = lds8[rowb32 | ((a - 1u) & 127u)];
        const uint32_t b2 = lds8[rowb32 | ((a - 2u) & 127u)];
        const uint32_t b3 = lds8[rowb32 | ((a - 3u) & 127u)];
        return b0 | b1 << 8 | b2 << 16 | b3 << 24;
    };
    // the record of column jw - 1 - kk of row r from window w (kk < 8)
    auto win_rec = [&](uint32_t w, uint32_t kk) -> uint32_t {
        return ((uint32_t)__builtin_amdgcn_readlane((int)w, (int)((r - base) + ((kk & 4u) << 3))) >> ((kk & 3u) * 8u)) &
               0xFFu;
    };
    // the record of cell (r, j) from the current 8-column window, or the one
    // below it, by one readlane; else the window holding column j is read
    // (one LDS round trip, which the window steps then reuse); r must lie in
    // the staged block
    auto rec_win = [&]() -> uint32_t {
        uint32_t kk = (uint32_t)(jw - 1 - j);
        if (kk < 8u) return win_rec(win, kk);
        if (kk < 16u && jwn == jw) return win_rec(wnx, kk - 8u);
        jw = (j & ~7) + 8;
        win = tb_win(jw);
        return win_rec(win, (uint32_t)(jw - 1 - j));
    };
    auto cell = [&]() -> uint32_t {
        if (r < base) to_block();
        return rec_win();
    };
    auto emit = [&](uint32_t e) { vev = (uint32_t)writelane((int)vev, (int)e, j & 63); };
    // j -= 1, handing a completed 64-base chunk to the store queue
    auto step_j = [&]() {
        if ((j & 63) == 0) {
            if (pend >= 0)
                __builtin_amdgcn_raw_buffer_store_b32(vpend, rev, lane <= pend_top ? (uint32_t)(pend + (int32_t)lane) * 4u : ~0u,
                                                      0, 0);
            vpend = vev, pend = chunk, pend_top = top;
            chunk -= 64;
            top = 63;
        }
        --j;
    };
    // to the predecessor of cell (r, jc) given by its record rc8: the M tag
    // (isD 0) or the D tag (1); an escape reads the distance from the row's
    // tag plane (M on rings of up to 8 rows: 8 - tag); far rows keep their
    // slots of the graph's predecessor list in a far slot record
    auto to_pred = [&](uint32_t rc8, int32_t jc, uint32_t isD) {
        const uint32_t li = r - base;
        const bool far = (farm >> li) & 1u;
        if (!isD) {
            const int32_t mt = rec_mtag(rc8);
            if (mt < 0 && !far) {
                r = (uint32_t)((int32_t)r + mt);
                return;
            }
        }
        const uint32_t meta = (uint32_t)__builtin_amdgcn_readlane((int)voff, (int)li);
        if (!far && (meta & 0x40000000u)) {
            // one or two predecessors: the tag names the slot, the row meta its distance
            const uint32_t slot = isD ? (rc8 >> 7) & 1u : (rc8 >> 4) & 1u;
            r -= 1u + ((meta >> (22u + 4u * slot)) & 15u);
            return;
        }
        if (!isD) {
            if (kRing <= 8 && !far) {
                r -= 8u - (uint32_t)rec_mtag(rc8);
                return;
            }
        } else if ((rc8 & 0x80u) && !far) {
            r -= 1u;
            return;
        }
        const uint32_t t = (uint32_t)(jc - (int32_t)(meta & kMetaOff));
        // the row's tag-plane row: staged in LDS (kTbTags) or in HBM
        const uint8_t *tp = kTbTags ? lds8 + (kTbTag + buf * kTbBufWords) * 4 + li * kRecRow
                                    : P<const uint8_t>(z, z.L.dsl) + (size_t)r * kRecRow;
        if (far) {
            const uint32_t p0 = uni(poff[r]);
            const uint32_t fs = uni(*reinterpret_cast<const uint32_t *>(tp));
            const uint32_t slot = uni((uint32_t)PX<const uint16_t>(z, kExtWtag)[(size_t)fs * (kW * 2) + t * 2 + isD]);
            r = uni(pred[p0 + slot]);
        } else if (kRing <= 8) {  // (D: 4 bits per cell)
            r -= 1u + ((uni((uint32_t)tp[t >> 1]) >> ((t & 1u) * 4u)) & 15u);
        } else {  // (a byte per cell: M | D << 4)
            r -= 1u + ((uni((uint32_t)tp[t]) >> (isD * 4u)) & 15u);
        }
    };
    uint32_t rec = cell();
    for (;;) {
        if (++guard > glim) {
            err = kErrTrace;
            break;
        }
#ifdef CCSX_TB_COUNTING
        z.pf[kPfSpare0] += 1;
#endif
        const uint32_t hc = rec & 3u;
        bool emitted = false;  // (r, j) MPRED, emitted by the window steps: its move is pending
        if (hc == HC_MPRED && farm == 0u) {
            // A block without far rows: plain steps through 8-column windows
            // aligned to jw = 0 mod 8 (tb_w8_steps), the next window read
            // from LDS while this one is walked.
            uint32_t k = (uint32_t)(jw - 1 - j);
            if (k >= 8u) {
                if (jwn == jw && k < 16u) {
                    win = wnx;  // j moved into the window below (already read)
                    jw -= 8;
                } else {
                    jw = (j & ~7) + 8;
                    win = tb_win(jw);
                }
                k = (uint32_t)(jw - 1 - j);
            }
            if (jwn != jw) {
                wnx = tb_win(jw - 8);
                jwn = jw;
            }
            uint32_t st;
#ifdef CCSX_TB_COUNTING
            const int32_t jin = j;
            TB_MARK(kPfRowE);
            z.pf[kPfRowA] += 1;
#endif
            for (;;) {
                tb_w8_steps(k, base, win, tb_wb(win), r, j, rec, vev, st);
                if (st) break;
                win = wnx;
                jw -= 8;
                wnx = tb_win(jw - 8);
                jwn = jw;
                rec = (uint32_t)__builtin_amdgcn_readlane((int)win, (int)(r - base)) & 0xFFu;
                if (rec & 3u) {
                    st = 2;
                    break;
                }
                k = 0;
            }
#ifdef CCSX_TB_COUNTING
            z.pf[kPfRowB] += (uint32_t)(jin - j);
            z.pf[kPfRowC] += st == 1 ? 1u : 0u;
            TB_MARK(kPfTbStep);
#endif
            if (st == 2) continue;  // a D / I / MSRC record at the new (r, j)
            emitted = true;
        }
        if (hc == HC_MPRED) {  // state H
            if (!emitted) {
                // plain steps while the next cell is in the block, the row not
                // far, no chunk completes and the M tag is a distance
                for (;;) {
                    emit((EV_ALN << 30) | r);
                    const int32_t mt = rec_mtag(rec);
                    const uint32_t li = r - base;
                    // sign-bit arithmetic keeps the test on the scalar unit (a
                    // compare of a bool lowers to VALU selects): far row, a chunk
                    // completes ((j & 63) == 0), a slot tag, or the predecessor
                    // leaves the block (li - d < 0)
                    const uint32_t slow = ((farm >> li) | (((uint32_t)(j & 63) - 1u) >> 31) | (~(uint32_t)mt >> 31) |
                                           ((li + (uint32_t)mt) >> 31)) & 1u;
                    if (slow) break;
                    --j;
                    r = (uint32_t)((int32_t)r + mt);
                    // r stays inside the block: the next record comes from the
                    // window by one readlane; an LDS round trip only every
                    // eighth column
                    uint32_t k = (uint32_t)(jw - 1 - j);
                    if (k >= 8u) {
                        jw = (j & ~7) + 8;  // aligned, as the unrolled walk above assumes
                        win = tb_win(jw);
                        k = (uint32_t)(jw - 1 - j);
                    }
                    rec = win_rec(win, k);
                    if ((rec & 3u) != HC_MPRED) break;
                }
                if ((rec & 3u) != HC_MPRED) continue;
            }
            step_j();
            to_pred(rec, j + 1, 0u);  // the MPRED cell is (r, j + 1)
            if (r < base) to_block();
            rec = rec_win();
            DP_STAMP(kPfTbStep);
#if defined(CCSX_TB_COUNT) && !defined(CCSX_DP_STAMPS)
            TB_MARK(kPfTbProbe);
#endif
            continue;
        }
        if (hc == HC_MSRC) {
            emit((EV_ALN << 30) | r);
            lead_row = r;
            lead_j = (uint32_t)j;
            break;
        }
        if (hc == HC_DEL) {
            // state D: follow D tags while the cell's D extends its predecessor's D
#ifdef CCSX_TB_COUNTING
            z.pf[kPfTbDruns] += 1;
#endif
            for (;;) {
#ifdef CCSX_TB_COUNTING
                z.pf[kPfTbDsteps] += 1;
#endif
                const uint32_t ext = rec & 4u;
                to_pred(rec, j, 1u);
                if (r < base) to_block();
                rec = rec_win();
                if (!ext || ++guard > glim) break;
            }
            DP_STAMP(kPfTbDI);
#if defined(CCSX_TB_COUNT) && !defined(CCSX_DP_STAMPS)
            TB_MARK(kPfTbDI);
#endif
            continue;
        }
        // state I: insertions along the row
#ifdef CCSX_TB_COUNTING
        z.pf[kPfTbIruns] += 1;
#endif
        for (;;) {
#ifdef CCSX_TB_COUNTING
            z.pf[kPfTbIsteps] += 1;
#endif
            emit((EV_INS << 30) | r);
            const uint32_t ext = rec & 8u;
            step_j();
            rec = rec_win();
            if (!ext || ++guard > glim) break;
        }
        DP_STAMP(kPfTbDI);
#if defined(CCSX_TB_COUNT) && !defined(CCSX_DP_STAMPS)
        TB_MARK(kPfSpare2);
#endif
    }
    if (err) {
        z.status = err;
        wsync();
        return;
    }
    // the chunks in flight, then LEAD for every base before the MSRC cell
    if (pend >= 0 && lane <= pend_top) ev[pend + (int32_t)lane] = vpend;
    if ((int32_t)lane + chunk >= (int32_t)lead_j && lane <= top) ev[chunk + (int32_t)lane] = vev;
    for (uint32_t jj = lane; jj < lead_j; jj += 64) ev[jj] = (EV_LEAD << 30) | lead_row;
    wsync();
}

// In-place prefix sums over n + 1 words of an HBM array by one wave, eight
// 64-word chunks loaded ahead of each scan step (the carry makes chunks
// serial; the loads must not be).  EXCL: out[x] = sum of in[0, x) and the
// total is returned; else out[x] = sum of in[0, x].
template <bool EXCL>
__device__ __forceinline__ uint32_t wave_scan_hbm(const uint32_t *in, uint32_t *out, uint32_t n)
{
    const uint32_t lane = lane_id();
    uint32_t carry = 0;
    for (uint32_t x0 = 0; x0 < n; x0 += 512) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t x = x0 + 64u * u + lane;
            v[u] = x < n ? in[x] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t x = x0 + 64u * u + lane;
            const uint32_t inc = (uint32_t)wave_incl_sum((int)v[u]);
            if (x < n) out[x] = carry + (EXCL ? inc - v[u] : inc);
            carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        }
    }
    return uni(carry);
}

// ----------------------------------------------------------------------------
// SPEC.md §5: merge read k into the graph (double-buffered rebuild)
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t col_start(const uint8_t *nb, uint32_t v)
{
    while (!(nb[v] & 4)) --v;
    return v;
}

__device__ __forceinline__ uint32_t col_end(const uint8_t *nb, uint32_t v, uint32_t R)
{
    ++v;
    while (v < R && !(nb[v] & 4)) ++v;
    return v;
}

// All three waves of the workgroup run the merge (thread tid of kBlockThreads):
// the row-parallel loops stride over every thread, the phases meet at
// workgroup barriers (which also make the HBM writes visible); M1's ordered
// compaction and the two prefix scans run on wave 0 between barriers.  Every
// branch that skips a barrier is uniform over the workgroup.
// LM = 2: the graph is small enough (every shredding window of the three-
// wave objects) for the current rows' node bytes and the new-row counts /
// shifts to live in the DP ring's LDS (idle during merge): the column walks,
// the count atomics, the prefix scan and every shift lookup are then LDS
// accesses instead of dependent HBM round trips.  LM = 1 (the solo object's
// 8.7 KB ring, graphs of 1,728-8,700 rows): the node bytes alone, the counts
// in HBM.  LM = 0: larger graphs (-P) take the same steps through HBM.
__device__ __forceinline__ int merge_in_lds(uint32_t R)
{
#ifdef CCSX_MERGE_NO_LDS  // measurement variant (LDS bank-conflict attribution)
    return 0 * R;
#endif
    constexpr uint32_t bytes = (uint32_t)kRingWords * 4u;
    return (R + 1) * 5u + 64u <= bytes ? 2 : R + 64u <= bytes ? 1 : 0;
}

template <int LM>
__device__ __forceinline__ void merge(Z &z, uint32_t k, uint32_t m, uint32_t tid)
{
    constexpr uint32_t T = kBlockThreads;
    const uint32_t lane = lane_id();
    const bool w0 = tid < 64;
    volatile DpJob *job = dp_job(z);
    const uint32_t R = z.R, nw = z.d.nw;
    const int a = z.cur, b = a ^ 1;
    const uint8_t *nbg = G_nb(z, a);
    uint32_t *lcnt = reinterpret_cast<uint32_t *>(z.lds + kLdsRing);  // LM 2: counts / shifts, R + 1 words
    // node bytes, R (+ 3) bytes: after the counts (LM 2) or alone (LM 1)
    uint8_t *lnb = reinterpret_cast<uint8_t *>(LM == 2 ? lcnt + R + 1 : lcnt);
    if (LM) {
        if (LM == 2)
            for (uint32_t x = tid; x <= R; x += T) lcnt[x] = 0;
        for (uint32_t x = 4 * tid; x < R; x += 4 * T)
            *reinterpret_cast<uint32_t *>(lnb + x) = *reinterpret_cast<const uint32_t *>(nbg + x);
        __syncthreads();
    }
    const uint8_t *nb = LM ? lnb : nbg;
    const uint64_t *mem = G_mem(z, a);
    const uint32_t *poff = G_poff(z, a);
    const uint32_t *pred = G_pred(z, a);
    uint8_t *nb2 = G_nb(z, b);
    uint64_t *mem2 = G_mem(z, b);
    uint32_t *poff2 = G_poff(z, b);
    uint32_t *pred2 = G_pred(z, b);
    const uint32_t *ev = P<uint32_t>(z, z.L.ev);
    uint32_t *tgt = P<uint32_t>(z, z.L.tgt);
    uint32_t *ipt = P<uint32_t>(z, z.L.ipt);
    uint8_t *iinf = P<uint8_t>(z, z.L.iinf);
    uint32_t *ifix = P<uint32_t>(z, z.L.ifix);
    uint32_t *cnt = LM == 2 ? lcnt : P<uint32_t>(z, z.L.cnt);
    uint8_t *fixf = P<uint8_t>(z, z.L.fixf);
    uint32_t *addp = P<uint32_t>(z, z.L.addp);
    uint32_t *cntn = P<uint32_t>(z, z.L.cntn);
    uint8_t *spf = P<uint8_t>(z, z.L.spf);  // spill flags of the new graph (SPEC.md §3)

#ifdef CCSX_DP_STAMPS
    unsigned long long t_prev = stamp();
#endif
    // M1 (wave 0): classify every read base, number the new nodes in read order
    uint32_t K = 0;
    // (the next 64 events are loaded while these are classified: the stores
    // below would otherwise keep the next load behind them)
    uint32_t ev_next = w0 && R && lane < m ? ev[lane] : 0u;
    for (uint32_t j0 = 0; w0 && j0 < m; j0 += 64) {
        const uint32_t j = j0 + lane;
        const uint32_t ev_cur = ev_next;
        if (R && j + 64 < m) ev_next = ev[j + 64];
        bool isnew = false;
        uint32_t pt = 0, cs = 1, fix = kNone, t = 0, bq = 0;
        if (j < m) {
            bq = rcode(z, j);
            if (R == 0) {
                isnew = true;
            } else {
                const uint32_t e = ev_cur, v = e & 0x3FFFFFFFu, kind = e >> 30;
                if (kind == EV_ALN) {
                    if ((nb[v] & 3u) == bq) {
                        t = v;
                    } else {
                        const uint32_t s0 = col_start(nb, v), s1 = col_end(nb, v, R);
                        uint32_t u = s0;
                        while (u < s1 && (nb[u] & 3u) < bq) ++u;
                        if (u < s1 && (nb[u] & 3u) == bq) {
                            t = u;
                        } else {
                            isnew = true;
                            pt = u;
                            cs = u == s0;
                            if (cs) fix = s0;
                        }
                    }
                } else if (kind == EV_INS) {
                    isnew = true;
                    pt = col_end(nb, v, R);
                } else {
                    isnew = true;
                    pt = col_start(nb, v);
                }
            }
        }
        const uint64_t bal = ballot(isnew);
        const uint32_t idx = K + lanes_below(bal);
        if (j < m) {
            if (isnew) {
                ipt[idx] = pt;
                iinf[idx] = (uint8_t)(bq | (cs << 2));
                ifix[idx] = fix;
                tgt[j] = kNewBit | idx;
            } else {
                tgt[j] = t;
            }
        }
        K += (uint32_t)__builtin_popcountll(bal);
    }
    if (w0 && lane == 0) job->K = K;
    __syncthreads();
    K = uni(job->K);
    const uint32_t R2 = R + K;
    if (R2 > z.d.rcap) {
        z.status = kErrRows;
        return;
    }
    DP_STAMP(kPfRowA);
    // M2: shift[x] = #new items with point <= x
    for (uint32_t x = tid; x <= R; x += T) {
        if (LM != 2) cnt[x] = 0;
        fixf[x] = 0;
    }
    __syncthreads();
    for (uint32_t i = tid; i < K; i += T) {
        atomicAdd(&cnt[ipt[i]], 1u);
        if (ifix[i] != kNone) fixf[ifix[i]] = 1;
    }
    __syncthreads();
    if (w0) wave_scan_hbm<false>(cnt, cnt, R + 1);
    __syncthreads();
    const uint32_t *shift = cnt;
    auto newidx = [&](uint32_t t) -> uint32_t {
        return (t & kNewBit) ? ipt[t & ~kNewBit] + (t & ~kNewBit) : t + shift[t];
    };
    DP_STAMP(kPfRowB);
    // M3: at most one new in-edge per target of this read (dedup vs existing)
    for (uint32_t x = tid; x < R2; x += T) addp[x] = kNone;
    __syncthreads();
    // (MB read bases per thread per pass: their dependent loads are issued
    // together so the HBM round trips overlap)
    // (8 per thread on the solo object's 64 threads measured -0.25 %: noise, r03u)
#ifndef CCSX_MERGE_MB
#define CCSX_MERGE_MB 4
#endif
    constexpr uint32_t MB = CCSX_MERGE_MB;
    for (uint32_t j0 = 1 + tid; j0 < m; j0 += MB * T) {
        uint32_t sv[MB], dv[MB], e0[MB], e1[MB], p0[MB], p1[MB];
#pragma unroll
        for (uint32_t b = 0; b < MB; ++b) {
            const uint32_t j = j0 + b * T;
            sv[b] = j < m ? tgt[j - 1] : kNewBit;
            dv[b] = j < m ? tgt[j] : kNewBit;
        }
#pragma unroll
        for (uint32_t b = 0; b < MB; ++b) {
            const bool old = !(dv[b] & kNewBit) && !(sv[b] & kNewBit);
            e0[b] = old ? poff[dv[b]] : 0u;
            e1[b] = old ? poff[dv[b] + 1] : 0u;
        }
#pragma unroll
        for (uint32_t b = 0; b < MB; ++b) {
            p0[b] = e0[b] < e1[b] ? pred[e0[b]] : kNone;
            p1[b] = e0[b] + 1 < e1[b] ? pred[e0[b] + 1] : kNone;
        }
#pragma unroll
        for (uint32_t b = 0; b < MB; ++b) {
            const uint32_t j = j0 + b * T;
            if (j >= m) continue;
            const uint32_t s = sv[b], d = dv[b];
            bool dup = p0[b] == s || p1[b] == s;
            for (uint32_t e = e0[b] + 2; !dup && e < e1[b]; ++e) dup = pred[e] == s;
            if (!dup) addp[newidx(d)] = newidx(s);
        }
    }
    __syncthreads();
    DP_STAMP(kPfRowC);
    // M4: rows of the new graph
    if (nw == 1) {
        for (uint32_t x0 = tid; x0 < R; x0 += MB * T) {
            uint32_t n[MB], fx[MB], e0[MB], e1[MB], nbx[MB], ad[MB];
            uint64_t mw[MB];
#pragma unroll
            for (uint32_t b = 0; b < MB; ++b) {
                const uint32_t x = x0 + b * T;
                const bool v = x < R;
                n[b] = v ? x + shift[x] : 0u;
                fx[b] = v ? fixf[x] : 0u;
                nbx[b] = v ? nb[x] : 0u;
                e0[b] = v ? poff[x] : 0u;
                e1[b] = v ? poff[x + 1] : 0u;
                mw[b] = v ? mem[x] : 0ull;
            }
#pragma unroll
            for (uint32_t b = 0; b < MB; ++b) ad[b] = x0 + b * T < R ? addp[n[b]] : kNone;
#pragma unroll
            for (uint32_t b = 0; b < MB; ++b) {
                if (x0 + b * T >= R) continue;
                nb2[n[b]] = fx[b] ? (uint8_t)(nbx[b] & 3u) : (uint8_t)nbx[b];
                spf[n[b]] = 0;
                mem2[n[b]] = mw[b];
                cntn[n[b]] = e1[b] - e0[b] + (ad[b] != kNone ? 1u : 0u);
            }
        }
    } else {
        for (uint32_t x = tid; x < R; x += T) {
            const uint32_t n = x + shift[x];
            nb2[n] = fixf[x] ? (uint8_t)(nb[x] & 3u) : nb[x];
            spf[n] = 0;
            for (uint32_t w = 0; w < nw; ++w) mem2[(size_t)n * nw + w] = mem[(size_t)x * nw + w];
            cntn[n] = poff[x + 1] - poff[x] + (addp[n] != kNone ? 1u : 0u);
        }
    }
    for (uint32_t i = tid; i < K; i += T) {
        const uint32_t n = ipt[i] + i;
        nb2[n] = iinf[i];
        spf[n] = 0;
        for (uint32_t w = 0; w < nw; ++w) mem2[(size_t)n * nw + w] = 0;
        cntn[n] = addp[n] != kNone ? 1u : 0u;
    }
    __syncthreads();
    // (one target row per read base, so the read-modify-writes never collide;
    // MB bases per thread per pass, loads first: each base's three dependent
    // loads -- target, shift, membership word -- overlap the others', where
    // one base per pass serialised them behind the previous pass's store)
    {
        const uint64_t kbit = 1ull << (k & 63u);
        const uint32_t kw = k >> 6;
        for (uint32_t j0 = tid; j0 < m; j0 += MB * T) {
            uint32_t tv[MB], nn[MB];
            uint64_t mv[MB];
#pragma unroll
            for (uint32_t b = 0; b < MB; ++b) tv[b] = j0 + b * T < m ? tgt[j0 + b * T] : 0u;
#pragma unroll
            for (uint32_t b = 0; b < MB; ++b) nn[b] = j0 + b * T < m ? newidx(tv[b]) : 0u;
#pragma unroll
            for (uint32_t b = 0; b < MB; ++b) mv[b] = j0 + b * T < m ? mem2[(size_t)nn[b] * nw + kw] : 0ull;
#pragma unroll
            for (uint32_t b = 0; b < MB; ++b)
                if (j0 + b * T < m) mem2[(size_t)nn[b] * nw + kw] = mv[b] | kbit;
        }
    }
    if (w0) {
        const uint32_t E2 = wave_scan_hbm<true>(cntn, poff2, R2);
        if (lane == 0) poff2[R2] = E2, job->E = E2;
    }
    __syncthreads();
    {
        const uint32_t E2 = uni(job->E);
        if (E2 > z.d.ecap) {
            z.status = kErrEdges;
            return;
        }
        z.E = E2;
    }
    // predecessor lists of the new graph, and each row's DP record
    // {base | chain << 3 | np << 8, p0, p1, p2} + p3 (dp_fast's prefetch)
    uint2 *rrec = P<uint2>(z, z.L.rrec);
    // (PB rows per thread per pass, loads first)
#ifndef CCSX_MERGE_PB
#define CCSX_MERGE_PB 2
#endif
    constexpr uint32_t PB = CCSX_MERGE_PB;
    for (uint32_t x0 = tid; x0 < R; x0 += PB * T) {
      uint32_t bn[PB], be0[PB], be1[PB], bad[PB], bo[PB], bq[PB][4];
#pragma unroll
      for (uint32_t b = 0; b < PB; ++b) {
          const uint32_t x = x0 + b * T;
          const bool v = x < R;
          bn[b] = v ? x + shift[x] : 0u;
          be0[b] = v ? poff[x] : 0u;
          be1[b] = v ? poff[x + 1] : 0u;
      }
#pragma unroll
      for (uint32_t b = 0; b < PB; ++b) {
          const bool v = x0 + b * T < R;
          bad[b] = v ? addp[bn[b]] : kNone;
          bo[b] = v ? poff2[bn[b]] : 0u;
#pragma unroll
          for (int u = 0; u < 4; ++u) bq[b][u] = be0[b] + u < be1[b] ? pred[be0[b] + u] : 0u;
      }
#pragma unroll
      for (uint32_t b = 0; b < PB; ++b) {
        const uint32_t x = x0 + b * T;
        if (x >= R) continue;
        const uint32_t n = bn[b];
        const uint32_t e0 = be0[b], e1 = be1[b];
        const uint32_t ad = bad[b];
        uint32_t o = bo[b];
        const uint32_t ne = e1 - e0;
        const uint32_t np = ne + (ad != kNone ? 1u : 0u);
        // the first four old predecessors (loaded above), then their shifts
        uint32_t q[4], ps[4] = {0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = (uint32_t)u < ne ? bq[b][u] + shift[bq[b][u]] : 0u;
        uint32_t far = np > 4u ? kInfoFar : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if ((uint32_t)u < ne) {
                pred2[o + u] = q[u];
                ps[u] = q[u];
                if (n - q[u] > (uint32_t)kRing) spf[q[u]] = 1, far = kInfoFar;
            }
        }
        for (uint32_t e = e0 + 4; e < e1; ++e) {
            const uint32_t p = pred[e] + shift[pred[e]];
            pred2[o + (e - e0)] = p;
            if (n - p > (uint32_t)kRing) spf[p] = 1;
        }
        o += ne;
        if (ad != kNone) {
            pred2[o] = ad;
            if (ne < 4) ps[ne] = ad;
            if (n - ad > (uint32_t)kRing) spf[ad] = 1, far = kInfoFar;
        }
        const uint32_t chain = (np == 1 && ps[0] + 1 == n) ? kInfoChain : 0u;
        const uint32_t info = (nb[x] & 3u) | chain | far | (np << 8);
        // {info, the predecessors' tag bytes} (RowPre::dpk; only read on rows without the far flag)
        const bool two = np <= 2u && !far;
        uint32_t dpk = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            dpk |= ((uint32_t)u < np ? (two ? tagb2(n - ps[u], (uint32_t)u) : tagb(n - ps[u])) & 255u : 0u) << (8 * u);
        rrec[n] = make_uint2(info, dpk);
      }
    }
    for (uint32_t i = tid; i < K; i += T) {
        const uint32_t n = ipt[i] + i;
        const uint32_t ad = addp[n];
        uint32_t info = (uint32_t)iinf[i] & 3u;
        if (ad != kNone) {
            pred2[poff2[n]] = ad;
            if (n - ad > (uint32_t)kRing) spf[ad] = 1;
            info |= (1u << 8) | (ad + 1 == n ? kInfoChain : 0u) | (n - ad > (uint32_t)kRing ? kInfoFar : 0u);
        }
        rrec[n] = make_uint2(info, ad != kNone ? tagb2(n - ad, 0u) & 255u : 0u);
    }
        DP_STAMP(kPfRowE);
    // M5: first/last rows of the reads
    uint32_t *rfirst = P<uint32_t>(z, z.L.rfirst), *rlast = P<uint32_t>(z, z.L.rlast);
    for (uint32_t kk = tid; kk < k; kk += T)
        if (rfirst[kk] != kNone) {
            rfirst[kk] += shift[rfirst[kk]];
            rlast[kk] += shift[rlast[kk]];
        }
    if (tid == 0) {
        rfirst[k] = newidx(tgt[0]);
        rlast[k] = newidx(tgt[m - 1]);
    }
    z.R = R2;
    z.cur = b;
    __syncthreads();
    // read k + 1 for the next DP, staged by all three waves (the helpers are
    // idle until the DP's job barrier, which also publishes the writes);
    // run_poa skips its own staging under the same condition
    if (k + 1 < z.d.n) {
        const uint32_t m1 = uni(P<uint32_t>(z, z.L.rdlen)[k + 1]);
        if (m1 != 0 && m1 <= z.rdcap && m1 <= z.d.lcap)
            stage_read(z, z.seq + uni(P<uint32_t>(z, z.L.rdoff)[k + 1]), m1, tid, T);
    }
}

// ----------------------------------------------------------------------------
// SPEC.md §6: columns, per-column consensus and the consensus-match masks
// ----------------------------------------------------------------------------
// per-column base counts, consensus base, coverage and the consensus row's
// read mask of columns tid, tid + T, ... (every wave of the workgroup)
__device__ __forceinline__ void columns_count(const Z &z, uint32_t n, uint32_t ncols, uint32_t tid, uint32_t T)
{
    const uint32_t nw = z.d.nw;
    const uint8_t *nb = G_nb(z, z.cur);
    const uint64_t *mem = G_mem(z, z.cur);
    const uint32_t *colrow = P<uint32_t>(z, z.L.colrow);
    uint8_t *cons = P<uint8_t>(z, z.L.cons);
    uint64_t *cmask = P<uint64_t>(z, z.L.cmask);
    const uint32_t *rfc = P<uint32_t>(z, z.L.rfc), *rlc = P<uint32_t>(z, z.L.rlc);
    for (uint32_t c = tid; c < ncols; c += T) {
        const uint32_t a = colrow[c], e = colrow[c + 1];
        uint32_t cnt[4] = {0, 0, 0, 0}, tot = 0, cov = 0;
        for (uint32_t u = a; u < e; ++u) {
            uint32_t pc = 0;
            for (uint32_t w = 0; w < nw; ++w) pc += (uint32_t)__builtin_popcountll(mem[(size_t)u * nw + w]);
            cnt[nb[u] & 3u] += pc;
            tot += pc;
        }
        for (uint32_t k = 0; k < n; ++k) cov += (rfc[k] <= c && c <= rlc[k]) ? 1u : 0u;
        uint32_t best = 0;
        for (uint32_t bb = 1; bb < 4; ++bb)
            if (cnt[bb] > cnt[best]) best = bb;
        const uint32_t gap = cov - tot;
        const uint32_t cb = cnt[best] >= gap ? best : 4u;
        cons[c] = (uint8_t)cb;
        uint32_t crow = kNone;
        for (uint32_t u = a; u < e; ++u)
            if ((nb[u] & 3u) == cb) crow = u;
        for (uint32_t w = 0; w < nw; ++w) cmask[(size_t)c * nw + w] = crow != kNone ? mem[(size_t)crow * nw + w] : 0ull;
    }
}

// Column numbering and the reads' first / last columns on wave 0, then the
// per-column counts on all three waves (job kJobColumns: the helpers join at
// the two barriers after the job barrier)
__device__ __forceinline__ uint32_t call_columns(Z &z, uint32_t n)
{
    const uint32_t lane = lane_id();
    const uint32_t R = z.R;
    const uint8_t *nb = G_nb(z, z.cur);
    uint32_t *colof = P<uint32_t>(z, z.L.colof);
    uint32_t *colrow = P<uint32_t>(z, z.L.colrow);
    const uint32_t *rfirst = P<uint32_t>(z, z.L.rfirst), *rlast = P<uint32_t>(z, z.L.rlast);
    uint32_t *rfc = P<uint32_t>(z, z.L.rfc), *rlc = P<uint32_t>(z, z.L.rlc);
    volatile DpJob *job = dp_job(z);
    if (lane == 0) job->kind = kJobColumns, job->m = n, job->R = R, job->cur = (uint32_t)z.cur;
    __syncthreads();  // J: job posted
    uint32_t carry = 0;
    for (uint32_t r0 = 0; r0 < R; r0 += 64) {
        const uint32_t r = r0 + lane;
        const bool f = r < R && (nb[r] & 4);
        const uint64_t bal = ballot(f);
        const uint32_t c = carry + lanes_below(bal) + (f ? 1u : 0u) - 1u;
        if (r < R) colof[r] = c;
        if (f) colrow[c] = r;
        carry += (uint32_t)__builtin_popcountll(bal);
    }
    const uint32_t ncols = carry;
    if (lane == 0) colrow[ncols] = R;
    wsync();
    for (uint32_t k = lane; k < n; k += 64) {
        rfc[k] = rfirst[k] != kNone ? colof[rfirst[k]] : kNone;
        rlc[k] = rfirst[k] != kNone ? colof[rlast[k]] : 0u;
    }
    if (lane == 0) job->K = ncols;
    __syncthreads();  // columns numbered, ncols posted
    columns_count(z, n, ncols, threadIdx.x, kBlockThreads);
    __syncthreads();  // every column counted
    return ncols;
}

// ----------------------------------------------------------------------------
// end_bspoa over the reads staged in rdoff/rdlen (main.c:492,571)
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t run_poa(Z &z, uint32_t n, const uint8_t *zseq)
{
    const uint32_t *rdoff = P<uint32_t>(z, z.L.rdoff), *rdlen = P<uint32_t>(z, z.L.rdlen);
    uint32_t *rfirst = P<uint32_t>(z, z.L.rfirst), *rlast = P<uint32_t>(z, z.L.rlast);
    z.R = 0;
    z.E = 0;
    z.cur = 0;
    if (lane_id() == 0) G_poff(z, 0)[0] = 0;
    bool staged = false;  // read k was staged by the previous merge (all waves)
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t m = uni(rdlen[k]);
        if (lane_id() == 0) rfirst[k] = rlast[k] = kNone;
        wsync();
        if (m == 0) {
            staged = false;
            continue;
        }
        if (m > z.rdcap || m > z.d.lcap) {
            z.status = kErrReadLen;
            return 0;
        }
        unsigned long long t0 = pstamp();
        if (!staged || zseq != z.seq) load_read(z, zseq + uni(rdoff[k]), m);
        unsigned long long t1 = pstamp();
        z.pf[kPfLoad] += t1 - t0;
        if (z.R) {
            uint32_t er, ej;
            z.pf[kPfRows] += z.R;
            dp_align(z, m, er, ej);
            if (z.status) return 0;
            unsigned long long t2 = pstamp();
            z.pf[kPfDp] += t2 - t1;
            if constexpr (kHelpers == 0 && kPrioTb > 0) __builtin_amdgcn_s_setprio(kPrioTb);
            traceback(z, m, er, ej);
            if constexpr (kHelpers == 0 && kPrioTb > 0) __builtin_amdgcn_s_setprio(0);
            if (z.status) return 0;
            t1 = pstamp();
            z.pf[kPfTrace] += t1 - t2;
        }
        {
            volatile DpJob *job = dp_job(z);
            if (lane_id() == 0) job->kind = kJobMerge, job->m = m, job->R = z.R, job->cur = (uint32_t)z.cur, job->k = k;
            __syncthreads();  // J: job posted
            const int lm = merge_in_lds(z.R);
            if constexpr (kHelpers == 0 && kPrioMg > 0) __builtin_amdgcn_s_setprio(kPrioMg);
            if (lm == 2) merge<2>(z, k, m, threadIdx.x);
            else if (lm == 1) merge<1>(z, k, m, threadIdx.x);
            else merge<0>(z, k, m, threadIdx.x);
            if constexpr (kHelpers == 0 && kPrioMg > 0) __builtin_amdgcn_s_setprio(0);
        }
        if (z.status) return 0;
        staged = k + 1 < z.d.n;  // (the merge staged read k + 1 under run_poa's own checks)
        z.pf[kPfMerge] += pstamp() - t1;
    }
    unsigned long long t3 = pstamp();
    const uint32_t nc = call_columns(z, n);
    z.pf[kPfColumns] += pstamp() - t3;
    return nc;
}

// main.c:580-612: largest i >= 1 whose 10-column window is a clean breakpoint
__device__ __forceinline__ bool bp_ok(const Z &z, uint32_t i, uint32_t nseq, uint32_t colrate)
{
    const uint32_t window = 10, minwin = 5, rowrate = 80, nw = z.d.nw;
    const uint8_t *cons = P<uint8_t>(z, z.L.cons);
    const uint64_t *cmask = P<uint64_t>(z, z.L.cmask);
    uint32_t nogwin = 0, j;
    for (j = i; j < i + window; ++j) {
        if (cons[j] >= 4) {
            if (nogwin) continue;
            else break;
        }
        ++nogwin;
        uint32_t colcnt = 0;
        for (uint32_t w = 0; w < nw; ++w) colcnt += (uint32_t)__builtin_popcountll(cmask[(size_t)j * nw + w]);
        if (colcnt * 100 < colrate * nseq) break;
    }
    if (j < i + window || nogwin < minwin) return false;
    for (uint32_t k = 0; k < nseq; ++k) {
        uint32_t rc = 0;
        for (uint32_t jj = i; jj < i + window; ++jj)
            if (cons[jj] < 4) rc += (uint32_t)(cmask[(size_t)jj * nw + (k >> 6)] >> (k & 63u)) & 1u;
        if (rc * 100 < rowrate * nogwin) return false;
    }
    return true;
}

__device__ __forceinline__ uint32_t find_breakpoint(const Z &z, uint32_t ncols, uint32_t nseq, uint32_t colrate)
{
    const uint32_t window = 10;
    if (ncols <= window) return 0;  // SPEC.md §7 (main.c:580 would underflow)
    for (int32_t top = (int32_t)(ncols - window); top >= 1; top -= 64) {
        const int32_t cand = top - (int32_t)lane_id();
        const bool ok = cand >= 1 && bp_ok(z, (uint32_t)cand, nseq, colrate);
        const uint64_t bal = ballot(ok);
        if (bal) return (uint32_t)(top - (int32_t)__builtin_ctzll(bal));
    }
    return 0;
}

// emit the consensus of columns [0, i) (main.c:622-638); advance pos if flag
__device__ __forceinline__ void emit(Z &z, uint32_t i, uint32_t ncols, uint32_t n, bool flag, uint8_t *out, uint32_t &ol)
{
    const uint32_t lane = lane_id(), nw = z.d.nw;
    const uint8_t *cons = P<uint8_t>(z, z.L.cons);
    if (flag) {
        const uint32_t *colrow = P<uint32_t>(z, z.L.colrow);
        const uint64_t *mem = G_mem(z, z.cur);
        const uint32_t rend = i < ncols ? colrow[i] : z.R;
        for (uint32_t r0 = 0; r0 < rend; r0 += 64) {
            const uint32_t r = r0 + lane;
            for (uint32_t w = 0; w < nw; ++w) {
                const uint64_t x = r < rend ? mem[(size_t)r * nw + w] : 0ull;
                const uint32_t kn = n - w * 64 < 64 ? n - w * 64 : 64;
                for (uint32_t kb = 0; kb < kn; ++kb) {
                    const uint32_t c = (uint32_t)__builtin_popcountll(ballot((x >> kb) & 1ull));
                    if (lane == 0) z.pos[w * 64 + kb] += c;
                }
            }
        }
    }
    for (uint32_t c0 = 0; c0 < i; c0 += 64) {
        const uint32_t c = c0 + lane;
        const uint32_t cb = c < i ? cons[c] : 4u;
        const uint64_t bal = ballot(cb < 4);
        if (cb < 4) {
            const uint32_t o = ol + lanes_below(bal);
            if (o < z.d.outcap) out[o] = (uint8_t)"ACGT"[cb];
        }
        ol += (uint32_t)__builtin_popcountll(bal);
    }
    if (ol > z.d.outcap) z.status = kErrOut;
    wsync();
}

// tidy_msa_bspoa (main.c:572): column-major MSA with mrow = n + 4
__device__ __forceinline__ void write_msa(Z &z, uint32_t ncols, uint32_t n, uint8_t *msa)
{
    const uint32_t lane = lane_id(), nw = z.d.nw, mrow = n + 4;
    const uint8_t *nb = G_nb(z, z.cur);
    const uint64_t *mem = G_mem(z, z.cur);
    const uint32_t *colof = P<uint32_t>(z, z.L.colof);
    const uint8_t *cons = P<uint8_t>(z, z.L.cons);
    const uint64_t tot = (uint64_t)ncols * mrow;
    for (uint64_t x = lane; x < tot; x += 64) msa[x] = 4;
    wsync();
    for (uint32_t r = lane; r < z.R; r += 64) {
        uint8_t *cp = msa + (size_t)colof[r] * mrow;
        for (uint32_t k = 0; k < n; ++k)
            if ((mem[(size_t)r * nw + (k >> 6)] >> (k & 63u)) & 1ull) cp[k + 1] = nb[r] & 3u;
    }
    for (uint32_t c = lane; c < ncols; c += 64) msa[(size_t)c * mrow + n + 1] = cons[c];
    wsync();
}

// Occupancy: ~1,000 ZMWs = 1,000 three-wave workgroups on 256 CUs, 4 per CU.
// At 3 waves per SIMD those fill every wave slot, and the dispatcher then
// strands some workgroups until others finish (bimodal launch times); 4 waves
// per SIMD (<= 128 VGPRs) leaves slack.
#ifndef CCSX_WAVES_PER_EU
#define CCSX_WAVES_PER_EU 4
#endif
// RD_HBM: the instance for ZMWs whose reads do not fit the LDS read buffer
// (or whose cursors do not): the read (nibble pairs) and the shredding cursors
// live in the workspace; every other access is the same code.
template <bool RD_HBM>
__device__ __forceinline__ void zmw_body(const KArgs &a, int32_t *smem)
{
    if (blockIdx.x >= a.nzmw) return;
    // longest-processing-time-first: the host orders the batch by cost so the
    // largest ZMWs start first and the tail of the launch is short ones
    const uint32_t zi = a.order[blockIdx.x];
    const uint32_t lane = lane_id();
    Z z;
    z.d = a.desc[zi];
    zlayout(z.L, z.d);
    z.ws = a.ws + z.d.ws_off;
    z.seq = a.seq + z.d.seq_off;
    z.lds = smem;
    z.hbm = RD_HBM;
    z.wa = 0, z.wpend = false;
    z.win = reinterpret_cast<uint8_t *>(smem + kLdsFixed);
    z.rdbytes = (uint32_t)zext_size(z.d, kExtRdbuf);
    if (RD_HBM) {
        z.rd = PX<uint8_t>(z, kExtRdbuf);
        z.pos = PX<uint32_t>(z, kExtPos);
        z.rdcap = z.d.lcap;
    } else {
        z.rd = reinterpret_cast<uint8_t *>(smem + kLdsFixed);
        z.pos = reinterpret_cast<uint32_t *>(smem + kLdsFixed) + a.lds_read_words;
        z.rdcap = (a.lds_read_words - 2) * 16;
    }
    z.status = kOk;
    z.cells = 0;
#pragma unroll
    for (int i = 0; i < kProfSlots; ++i) z.pf[i] = 0;
    if (kHelpers > 0 && threadIdx.x >= 64) {
        // waves 1 and 2: the decision bits of the even / odd rows of every DP
        const uint32_t h = uni(threadIdx.x >> 6) - 1u;
        dp_helper(z, h);
        volatile unsigned long long *pf1 = reinterpret_cast<volatile unsigned long long *>(z.lds + kLdsDiag) + 8 * h;
        if (lane == 0)
            pf1[0] = z.pf[kPfBbusy], pf1[1] = z.pf[kPfBwait], pf1[2] = z.pf[kPfSpare2], pf1[3] = z.pf[kPfSpare3],
            pf1[4] = z.pf[kPfFlush], pf1[5] = wave_hw_id();
        __syncthreads();
        return;
    }
    // wave 0 carries the ZMW's critical path; its SIMD also runs helper waves
    // of other workgroups, whose DP work has a block of slack: let wave 0 win
    // the issue arbitration (measured: 63.9 -> 58.4 ms per launch, config B)
    __builtin_amdgcn_s_setprio(kPrioWave0);
    const unsigned long long t_start = pstamp();
    z.pf[kPfStartRt] = prealtime();
    if (kProfiling) z.pf[kPfHw0] = wave_hw_id();
    const uint32_t n = z.d.n;
    const uint32_t *soff = a.soff + z.d.seg0, *slen = a.slen + z.d.seg0;
    uint32_t *rdoff = P<uint32_t>(z, z.L.rdoff), *rdlen = P<uint32_t>(z, z.L.rdlen);
    uint8_t *out = a.out + z.d.out_off;
    uint32_t ol = 0;

    if (a.mode != kShred) {
        // ccs_for (main.c:486-502) / single bspoa call: push every segment whole
        for (uint32_t k = lane; k < n; k += 64) rdoff[k] = soff[k], rdlen[k] = slen[k];
        wsync();
        const uint32_t ncols = run_poa(z, n, z.seq);
        if (!z.status) {
            emit(z, ncols, ncols, n, false, out, ol);
            if (a.mode == kSinglePoa && !z.status) {
                if ((uint64_t)ncols * (n + 4) > z.d.msacap) z.status = kErrOut;
                else write_msa(z, ncols, n, a.msa + z.d.msa_off);
                if (lane == 0) a.ncols[zi] = ncols;
            }
        }
    } else if (!RD_HBM && n > a.lds_nmax) {
        z.status = kErrReadLen;
    } else {
        // ccs_for2 (main.c:541-641)
        const uint32_t addlen = 2000, minlen = 1000, initlen = 2000;
        const uint32_t colrate = n < 10 ? 60u : 80u;
        for (uint32_t k = lane; k < n; k += 64) z.pos[k] = 0;
        wsync();
        bool flag = true;
        uint32_t nround = 0;  // shredding rounds (the -v >= 3 breakpoint log)
        while (flag && !z.status) {
            uint32_t i = 0, ncols = 0;
            for (uint32_t ws = initlen;; ws += addlen) {
                bool fin = n < 3;
                for (uint32_t k = 0; k < n && !fin; ++k)
                    if (z.pos[k] + ws + minlen >= slen[k]) fin = true;
                if (fin) flag = false;
                for (uint32_t k = lane; k < n; k += 64) {
                    rdoff[k] = soff[k] + z.pos[k];
                    rdlen[k] = fin ? slen[k] - z.pos[k] : ws;
                }
                wsync();
                ncols = run_poa(z, n, z.seq);
                if (z.status) break;
                if (!flag) {
                    i = ncols;
                    break;
                }
                const unsigned long long tb0 = pstamp();
                i = find_breakpoint(z, ncols, n, colrate);
                z.pf[kPfShred] += pstamp() - tb0;
                if (i >= 1) break;
            }
            if (z.status) break;
            if (a.bplog) {
                // main.c:619-620: "breakpoint=i maplen=ncols" (the host prints it)
                if (lane == 0 && nround < z.d.bpcap) {
                    a.bplog[z.d.bp_off + 1 + 2 * nround] = i;
                    a.bplog[z.d.bp_off + 2 + 2 * nround] = ncols;
                }
                ++nround;
            }
            const unsigned long long te0 = pstamp();
            emit(z, i, ncols, n, flag, out, ol);
            z.pf[kPfShred] += pstamp() - te0;
        }
        if (a.bplog) {
            if (nround > z.d.bpcap && !z.status) z.status = kErrBpLog;
            if (lane == 0) a.bplog[z.d.bp_off] = nround;
        }
    }
    dp_helper_exit(z);
    if (lane == 0) {
        a.out_len[zi] = ol;
        a.status[zi] = z.status;
        a.cells[zi] = z.cells;
        if (a.prof) {
            z.pf[kPfTotal] = pstamp() - t_start;
            z.pf[kPfEndRt] = prealtime();
#pragma unroll
            for (int i = 0; i < kProfSlots; ++i) a.prof[(size_t)zi * kProfSlots + i] = z.pf[i];
        }
    }
}

__global__ void __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(CCSX_WAVES_PER_EU)))
ccsx_zmw_kernel(KArgs a)
{
    extern __shared__ int32_t smem[];
    zmw_body<false>(a, smem);
}

#ifndef CCSX_RING16  // (solo16 takes LDS-instance slices only: ccsx_gpu.cpp stage_slot)
__global__ void __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(CCSX_WAVES_PER_EU)))
ccsx_zmw_kernel_hbm(KArgs a)
{
    extern __shared__ int32_t smem[];
    zmw_body<true>(a, smem);
}
#endif

}  // namespace CCSX_KCFG
}  // namespace ccsx

// lds_read_words == 0 selects the HBM-read instance (ccsx_gpu.cpp decides);
// lds_bytes = this configuration's fixed words (CCSX_INFO) + the read buffer
extern "C" void CCSX_INFO(ccsx::KCfgInfo *o)
{
    namespace K = ccsx::CCSX_KCFG;
    o->lds_fixed_words = (uint32_t)K::kLdsFixed;
    o->threads = (uint32_t)K::kBlockThreads;
    o->ring_rows = (uint32_t)ccsx::kRingA;
    o->ring_back = (uint32_t)ccsx::kRing;
    o->waves_per_simd = CCSX_WAVES_PER_EU;
    o->max_read = sizeof(K::RingT) == 2 ? K::kRing16MaxRead : 0u;
    o->profiling = K::kProfiling ? 1u : 0u;
}

extern "C" hipError_t CCSX_LAUNCH(const ccsx::KArgs *a, uint32_t lds_bytes, hipStream_t s)
{
    namespace K = ccsx::CCSX_KCFG;
    if (lds_bytes < (uint32_t)K::kLdsFixed * 4u) return hipErrorInvalidValue;
#ifdef CCSX_RING16
    if (!a->lds_read_words) return hipErrorInvalidValue;
    const void *f = reinterpret_cast<const void *>(&K::ccsx_zmw_kernel);
#else
    const void *f = a->lds_read_words ? reinterpret_cast<const void *>(&K::ccsx_zmw_kernel)
                                      : reinterpret_cast<const void *>(&K::ccsx_zmw_kernel_hbm);
#endif
    if (lds_bytes > 65536) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        if (e != hipSuccess) return e;
    }
#ifdef CCSX_RING16
    hipLaunchKernelGGL(K::ccsx_zmw_kernel, dim3(a->nzmw), dim3(K::kBlockThreads), lds_bytes, s, *a);
#else
    if (a->lds_read_words)
        hipLaunchKernelGGL(K::ccsx_zmw_kernel, dim3(a->nzmw), dim3(K::kBlockThreads), lds_bytes, s, *a);
    else
        hipLaunchKernelGGL(K::ccsx_zmw_kernel_hbm, dim3(a->nzmw), dim3(K::kBlockThreads), lds_bytes, s, *a);
#endif
    return hipGetLastError();
}
