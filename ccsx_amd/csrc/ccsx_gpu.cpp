// ccsx_gpu.cpp -- host side of the batched C-ABI (include/ccsx_gpu.h).
//
// Stages a chunk of ZMWs into HBM (one sequence arena, segment tables, one
// descriptor and one workspace slab per ZMW, laid out by ccsx_layout.h),
// launches one workgroup per ZMW and copies the CCS strings back; slices of
// a large chunk alternate between two slots (streams) so they overlap.
// This is the device boundary that replaces kt_for(ccs_for2/ccs_for) in step 1
// of ccsx's pipeline (main.c:698-706).
#include "ccsx_gpu.h"
#include "ccsx_host.h"

#include <chrono>
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ccsx_layout.h"

// the kernel configurations (ccsx_layout.h KernelCfg), one object each: the
// launcher and the configuration's own LDS / thread figures
extern "C" hipError_t ccsx_launch_zmw_lat(const ccsx::KArgs *a, uint32_t lds_bytes, hipStream_t s);
extern "C" hipError_t ccsx_launch_zmw_occ(const ccsx::KArgs *a, uint32_t lds_bytes, hipStream_t s);
extern "C" hipError_t ccsx_launch_zmw_tput(const ccsx::KArgs *a, uint32_t lds_bytes, hipStream_t s);
extern "C" hipError_t ccsx_launch_zmw_solo(const ccsx::KArgs *a, uint32_t lds_bytes, hipStream_t s);
extern "C" hipError_t ccsx_launch_zmw_solo16(const ccsx::KArgs *a, uint32_t lds_bytes, hipStream_t s);
extern "C" hipError_t ccsx_launch_zmw_solo16w(const ccsx::KArgs *a, uint32_t lds_bytes, hipStream_t s);
extern "C" void ccsx_kcfg_info_lat(ccsx::KCfgInfo *o);
extern "C" void ccsx_kcfg_info_occ(ccsx::KCfgInfo *o);
extern "C" void ccsx_kcfg_info_tput(ccsx::KCfgInfo *o);
extern "C" void ccsx_kcfg_info_solo(ccsx::KCfgInfo *o);
extern "C" void ccsx_kcfg_info_solo16(ccsx::KCfgInfo *o);
extern "C" void ccsx_kcfg_info_solo16w(ccsx::KCfgInfo *o);

namespace {
typedef hipError_t (*LaunchFn)(const ccsx::KArgs *, uint32_t, hipStream_t);
constexpr LaunchFn kLaunch[ccsx::kCfgCount] = {ccsx_launch_zmw_lat,  ccsx_launch_zmw_occ,    ccsx_launch_zmw_tput,
                                               ccsx_launch_zmw_solo, ccsx_launch_zmw_solo16, ccsx_launch_zmw_solo16w};

ccsx::KCfgInfo kcfg_info(int cfg)
{
    ccsx::KCfgInfo o{};
    if (cfg == ccsx::kCfgLatency) ccsx_kcfg_info_lat(&o);
    else if (cfg == ccsx::kCfgOccupancy) ccsx_kcfg_info_occ(&o);
    else if (cfg == ccsx::kCfgThroughput) ccsx_kcfg_info_tput(&o);
    else if (cfg == ccsx::kCfgSolo) ccsx_kcfg_info_solo(&o);
    else if (cfg == ccsx::kCfgSolo16) ccsx_kcfg_info_solo16(&o);
    else ccsx_kcfg_info_solo16w(&o);
    return o;
}

// LDS bytes of a configuration's workgroup with `extra` words of read
// buffer and cursors
uint32_t kcfg_lds(int cfg, uint32_t extra) { return (kcfg_info(cfg).lds_fixed_words + extra) * 4u; }

// workgroups per CU: 4 SIMDs x the object's waves per SIMD (its register
// budget: 4 at 128 VGPRs, 5 at 96) and 160 KiB of LDS
uint32_t kcfg_wg_per_cu(int cfg, uint32_t extra)
{
    const ccsx::KCfgInfo i = kcfg_info(cfg);
    const uint32_t by_waves = 4u * i.waves_per_simd / (i.threads / 64u);
    const uint32_t by_lds = (160u * 1024u) / kcfg_lds(cfg, extra);
    return std::min(by_waves, by_lds);
}
}  // namespace

namespace {

// pinned host staging (grow-only): DMA straight from / to it,
// no pageable bounce and no per-slice zero-fill of a fresh std::vector.  If
// pinning fails (many contexts x slots each pinning ~1 GB arenas), the buffer
// falls back to pageable memory: the copies then stage through the driver,
// slower but correct.
struct HostBuf {
    uint8_t *p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    bool mapped = false;  // an anonymous mapping with huge pages, registered with HIP
    void release()
    {
        if (p) {
            if (mapped) (void)hipHostUnregister(p), munmap(p, cap);
            else if (pinned) (void)hipHostFree(p);
            else free(p);
        }
        p = nullptr;
        cap = 0;
        pinned = mapped = false;
    }
    // at least `floor` bytes (the CLI's contexts pin their staging once:
    // re-pinning a grown arena costs ~0.25 s per GB)
    hipError_t reserve(size_t n, size_t floor = 0, bool exact = false)
    {
        if (n <= cap) return hipSuccess;
        release();
        size_t c = std::max<size_t>(std::max<size_t>(exact ? n : n + n / 4, floor), 4096);
        {
            // an anonymous mapping with transparent huge pages, touched, then
            // registered with HIP: pinning and (at the process exit)
            // unpinning work per 2 MB page instead of per 4 KB one -- the
            // CLI's exit took 0.55 s less for its ~3 GB of staging buffers
            // (62,500 config-E ZMWs: 4.86 -> 4.40 s, gpurun_out r04h);
            // hipHostMalloc if that fails
            c = (c + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
            void *q = mmap(nullptr, c, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (q != MAP_FAILED) {
                (void)madvise(q, c, MADV_HUGEPAGE);
                memset(q, 0, c);
                if (hipHostRegister(q, c, hipHostRegisterDefault) == hipSuccess) {
                    p = static_cast<uint8_t *>(q);
                    cap = c;
                    pinned = mapped = true;
                    return hipSuccess;
                }
                (void)hipGetLastError();
                munmap(q, c);
            }
        }
        hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&p), c, hipHostMallocDefault);
        if (e == hipSuccess) {
            pinned = true;
        } else {
            (void)hipGetLastError();
            p = static_cast<uint8_t *>(malloc(c));
            if (!p) return hipErrorOutOfMemory;
        }
        cap = c;
        return hipSuccess;
    }
    ~HostBuf() { release(); }
};

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    // exact: allocate exactly n (the CLI's one-off slice-budget reservation)
    hipError_t reserve(size_t n, bool exact = false)
    {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        // grow with 25 % headroom (falling back to the exact size): slices of
        // one chunk differ by a few percent, and re-allocating a workspace a
        // full launch has touched measured 1-5 s per 75-150 GB (DESIGN.md
        // section 7)
        size_t c = std::max<size_t>(exact ? n : n + n / 4, 256);
        hipError_t e = hipMalloc(&p, c);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            c = std::max<size_t>(n, 256);
            e = hipMalloc(&p, c);
        }
        if (e == hipSuccess) cap = c;
        return e;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const
    {
        return static_cast<T *>(p);
    }
};


// One staged slice and everything it owns on the device and the host.  A
// context has two: ccsx_gpu_run stages and launches slice k + 1 on the other
// slot's stream while slice k's kernel runs, so one slice's tail (the launch
// ends with its slowest ZMW) overlaps the next slice's start, and its staging
// overlaps the previous kernel.  stage / launch / fetch (bench.py) use slot 0.
struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t evp[2] = {nullptr, nullptr};  // piecewise staging: the copy out of each half of h_seq
    size_t nz = 0;
    uint32_t lds_read_words = 0, lds_nmax = 0, lds_extra = 0;
    int32_t cfg = ccsx::kCfgLatency;   // kernel configuration of the staged slice
    uint64_t seq_bytes = 0, ws_bytes = 0, out_bytes = 0, msa_bytes = 0, bp_words = 0;
    uint32_t nseg_total = 0;
    bool inflight = false;             // launched, results not fetched yet
    std::vector<ccsx::ZmwDesc> desc;
    std::vector<uint32_t> hoff, hlen, order;  // host copies the async H2D reads from
    DevBuf d_prof, d_bp;
    DevBuf d_seq, d_soff, d_slen, d_desc, d_order, d_ws, d_out, d_msa, d_olen, d_ncols, d_status, d_cells;
    HostBuf h_out, h_seq;
    std::vector<uint32_t> h_olen, h_ncols, h_bp;
    std::vector<int32_t> h_status;
    std::vector<unsigned long long> h_cells, h_prof;
    std::vector<uint8_t> h_msa;
    void release()
    {
        DevBuf *bufs[] = {&d_bp, &d_prof, &d_seq, &d_soff, &d_slen, &d_desc, &d_order, &d_ws, &d_out,
                          &d_msa, &d_olen, &d_ncols, &d_status, &d_cells};
        for (DevBuf *b : bufs) b->release();
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        for (hipEvent_t &e : evp)
            if (e) (void)hipEventDestroy(e), e = nullptr;
        if (stream) (void)hipStreamDestroy(stream);
        ev0 = ev1 = nullptr;
        stream = nullptr;
    }
};

}  // namespace

struct ccsx_ctx {
    int device = 0;
    std::string err;
    Slot slot[2];
    int32_t cfg_force = -1;            // test hook: -1 = by slice size
    uint32_t wg_cap = 0;               // measurement hook (ccsx_gpu_set_wg_cap): LDS request padded to cap workgroups per CU
    uint64_t slot_budget = 0;          // test hook (ccsx_gpu_set_slot_budget): bytes per slot, 0 = by device memory
    // LDS read buffer of tight-cap shredded slices, bases (ccsx_gpu_set_shred_read_cap):
    // pushed windows are 2-3 kb unless a breakpoint is missed (+2 kb each,
    // main.c:552-570); a longer one fails the ZMW with kErrReadLen and
    // ccsx_gpu_run re-runs it uncapped.  4,096 rather than 8,192 bases: 2 KB
    // less LDS per workgroup, 12 -> 14 solo workgroups per CU on config E
    // (16,384-ZMW e2e 14.7k -> 17.1k ZMWs/s, no re-runs; r03o)
    uint32_t shred_read_cap = 4096;
    uint32_t ncu = 256;                // compute units of the device
    uint64_t reruns = 0;               // ZMWs ccsx_gpu_run re-ran with full caps
    uint64_t slices = 0;               // slices ccsx_gpu_run launched
    uint64_t dealt = 0, parts = 0;     // lists ccsx_gpu_run dealt into interleaved parts, and their parts
    bool profiling = false;
    uint32_t tight_rows = 0;           // test hook: override the tight row cap
    uint32_t tight_out = 0;            // test hook: override the tight output slab
    uint32_t tight_far = 0;            // test hook: override the tight far slot record rows
    uint64_t stage_piece = 0;          // test hook: piecewise staging's half size (0: kStagePiece)
    int64_t fault = -1;                // test hook: report this ZMW of the next run as failed
    bool shred_caps = false;           // tight caps sized for shredding windows (ccsx_gpu_run, shredded mode)
    uint32_t mem_share = 1;            // contexts sharing the device concurrently
    float mem_frac = 0.5f;             // of the device memory, the contexts sharing it use at most this fraction
    // a slice staged while another process or context still holds device
    // memory it is about to release waits up to this long for it
    // (ccsx_gpu_set_mem_wait) before the call fails
    uint32_t mem_wait_ms = 60000;
    uint64_t mem_waits = 0, mem_replans = 0;  // slices that waited for memory / were cut below the plan
    bool prealloc = false;             // reserve the slice budget up front
    bool bp_log = false;               // record the -v >= 3 breakpoint log (main.c:619-620)
    std::vector<uint32_t> run_bp;      // ccsx_gpu_run: the gathered logs, (i, ncols) pairs
    std::vector<uint64_t> run_bp_off;  // per ZMW of the call: offset into run_bp (pairs)
    std::vector<uint32_t> run_bp_n;    // per ZMW of the call: rounds
    std::vector<uint8_t> run_arena;    // ccsx_gpu_run's gathered CCS strings
    // ccsx_gpu_submit / ccsx_gpu_collect: one batch per slot
    struct Ticket {
        bool pending = false;          // submitted, not collected
        int mode = 0;
        const ccsx_zmw_in *z = nullptr;  // the caller's batch (valid until collected)
        size_t nz = 0;
        int64_t fault = -1;            // test hook, taken from ccsx_gpu_set_fault at submit
        std::vector<uint8_t> arena;    // the collected batch's CCS strings
    } tk[2];
};

static int fail(ccsx_ctx *c, const char *what, hipError_t e)
{
    if (c) {
        c->err = std::string(what) + ": " + hipGetErrorString(e);
    }
    return -1;
}

#define HIPCHK(c, call)                                   \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return fail((c), #call, e_); \
    } while (0)

extern "C" {

int ccsx_gpu_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ccsx_gpu_open(int device, ccsx_ctx **out)
{
    *out = nullptr;
    auto *c = new ccsx_ctx();
    c->device = device;
    hipError_t e = hipSetDevice(device);
    for (Slot &s : c->slot) {
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreate(&s.ev0);
        if (e == hipSuccess) e = hipEventCreate(&s.ev1);
        for (hipEvent_t &p : s.evp)
            if (e == hipSuccess) e = hipEventCreateWithFlags(&p, hipEventDisableTiming);
    }
    if (e == hipSuccess) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && n > 0)
            c->ncu = (uint32_t)n;
    }
    if (e != hipSuccess) {
        fprintf(stderr, "[ccsx_gpu] cannot open device %d: %s\n", device, hipGetErrorString(e));
        for (Slot &s : c->slot) s.release();
        delete c;
        return -1;
    }
    *out = c;
    return 0;
}

void ccsx_gpu_close(ccsx_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    using ms = std::chrono::duration<double, std::milli>;
    const auto t0 = std::chrono::steady_clock::now();
    for (Slot &s : c->slot) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        s.release();
    }
    const auto t1 = std::chrono::steady_clock::now();
    for (Slot &s : c->slot) s.h_out.release(), s.h_seq.release();
    const auto t2 = std::chrono::steady_clock::now();
    delete c;
    if (getenv("CCSX_TIMING") && atoi(getenv("CCSX_TIMING")))
        fprintf(stderr, "[ccsx_gpu_close] device buffers %.0f ms, pinned host buffers %.0f ms, rest %.0f ms\n",
                ms(t1 - t0).count(), ms(t2 - t1).count(), ms(std::chrono::steady_clock::now() - t2).count());
}

const char *ccsx_gpu_error(const ccsx_ctx *c) { return c ? c->err.c_str() : "no context"; }

const char *ccsx_gpu_status_str(int32_t s)
{
    switch (s) {
    case ccsx::kOk: return "ok";
    case ccsx::kErrRows: return "graph rows exceed capacity";
    case ccsx::kErrEdges: return "graph edges exceed capacity";
    case ccsx::kErrMulti: return "multi-predecessor rows exceed capacity";
    case ccsx::kErrSpill: return "spilled DP rows exceed capacity";
    case ccsx::kErrInDegree: return "far-row in-degree > 63";
    case ccsx::kErrReadLen: return "read longer than the LDS read buffer";
    case ccsx::kErrOut: return "consensus longer than the output slab";
    case ccsx::kErrTrace: return "traceback did not terminate";
    case ccsx::kErrBpLog: return "more shredding rounds than the breakpoint log holds";
    default: return "unknown status";
    }
}

}  // extern "C"

// pinned staging arenas of a preallocating context (per slot): the subreads
// and CCS of a CLI micro-batch (a 16,384-ZMW config-E chunk over one
// context's two batches: ~1 GB of subreads) without re-pinning; grown on
// demand beyond it.  INTEGRATION.md lists the host-memory footprint.
constexpr size_t kPinnedSeqFloor = 512ull << 20, kPinnedOutFloor = 128ull << 20;
// piecewise staging of a CLI context's subreads: two pinned halves of this
constexpr size_t kStagePiece = 64ull << 20;

// LDS read buffer limits of the LDS kernel instance: reads up to 100 kb
// (25 KiB of 2-bit codes) and 4,096 segments; beyond
// them a slice runs the HBM-read instance
constexpr uint32_t kLdsReadMaxBases = 100000, kLdsMaxSegs = 4096;
// slices of at least this many times the occupancy configuration's resident
// workgroups run the solo configuration
constexpr size_t kSoloSliceFactor = 3;
// segments per ZMW (slice mean) below which a solo16 slice runs solo16w (24
// ZMWs per CU, 80 VGPRs); 16 until the 8-bit records, with which solo16w also
// runs config D's 30-segment ZMWs 2.2 % faster (305.9 vs 312.7 ms, r06w)
constexpr uint32_t kSolo16WMaxSegs = 64;

// launch classes of ccsx_gpu_run's slices: LDS read buffer up to 32 kb (4+
// workgroups per CU), up to kLdsReadMaxBases, HBM-read instance; slices never
// mix classes, so one long read does not shrink the occupancy of a slice
// (shred_tight: a tight-cap shredded slice, whose LDS read buffer holds
// shred_read_cap bases whatever the segment lengths -- pushed windows are
// 2-10 kb -- so only the cursor count sends it to the HBM-read instance)
static int zmw_class(const ccsx_zmw_in &zi, bool shred_tight)
{
    uint32_t lmax = 0;
    for (uint32_t k = 0; k < zi.nseg; ++k) lmax = std::max(lmax, zi.seg_len[k]);
    if (zi.nseg > kLdsMaxSegs) return 2;
    if (shred_tight) return 0;
    if (lmax > kLdsReadMaxBases) return 2;
    return lmax > 32768 ? 1 : 0;
}

static void zmw_extent(const ccsx_zmw_in &zi, uint64_t &S, uint64_t &hi, uint32_t &lmax)
{
    S = 0, hi = 0, lmax = 0;
    for (uint32_t k = 0; k < zi.nseg; ++k) {
        S += zi.seg_len[k];
        lmax = std::max(lmax, zi.seg_len[k]);
        hi = std::max<uint64_t>(hi, uint64_t(zi.seg_off[k]) + zi.seg_len[k]);
    }
}

// device bytes one ZMW occupies when staged
static uint64_t zmw_bytes(const ccsx_zmw_in &zi, bool full, const ccsx_ctx *c, uint32_t shred_win)
{
    uint64_t S, hi;
    uint32_t lmax;
    zmw_extent(zi, S, hi, lmax);
    ccsx::ZmwDesc d{};
    ccsx::zcaps(d, S, lmax, zi.nseg, full, c->tight_rows, shred_win, c->tight_out, c->tight_far);
    ccsx::ZLayout L;
    ccsx::zlayout(L, d);
    return ccsx::align256(L.total) + hi + d.outcap + uint64_t(zi.nseg) * 8 + sizeof(ccsx::ZmwDesc) + 32;
}

// The bytes a slice staged into slot s may need now: the device's free memory
// plus what s's arenas already hold, less a 1 GB margin (stage_slot's test).
// A context's slice plan (plan_slots) comes from its share of the device, but
// a neighbour -- another context, or a process that just exited and whose
// memory the driver is still clearing -- may hold part of that share for a
// while (a rank's call failed with 28.2 GB needed, 25.7 GB free).
static int slot_avail(ccsx_ctx *c, const Slot &s, uint64_t &avail)
{
    size_t freeb = 0, totb = 0;
    HIPCHK(c, hipMemGetInfo(&freeb, &totb));
    const uint64_t have = freeb + s.d_ws.cap + s.d_seq.cap + s.d_out.cap + s.d_msa.cap;
    avail = have > (1ull << 30) ? have - (1ull << 30) : 0;
    return 0;
}

// Wait (polling, up to c->mem_wait_ms) until a slice of `need` bytes fits
// slot s; `fits` tells whether it does.
static int wait_slot_mem(ccsx_ctx *c, const Slot &s, uint64_t need, bool &fits)
{
    uint64_t avail = 0;
    int r = slot_avail(c, s, avail);
    if (r) return r;
    fits = need <= avail;
    if (fits) return 0;
    ++c->mem_waits;
    const auto t0 = std::chrono::steady_clock::now();
    while (!fits && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(c->mem_wait_ms)) {
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        if ((r = slot_avail(c, s, avail))) return r;
        fits = need <= avail;
    }
    if (getenv("CCSX_TIMING") && atoi(getenv("CCSX_TIMING")))
        fprintf(stderr, "[ccsx_gpu_run] dev %d: waited %.0f ms for %.1f GB of device memory (%s)\n", c->device,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), need / 1e9,
                fits ? "free" : "timed out");
    return 0;
}

// Stage a slice into slot s: sizes, device buffers, the host packing of the
// sequence arena, and the H2D copies enqueued on the slot's stream (the host
// copies they read stay in the slot until its next stage, which follows the
// slot's fetch, i.e. a stream synchronisation).  with_msa: an MSA slab per
// ZMW (single-POA mode); full_caps: exact upper-bound capacities, else tight
// ones (ccsx_layout.h zcaps).
static int stage_slot(ccsx_ctx *c, Slot &s, const ccsx_zmw_in *z, size_t nz, int with_msa, int full_caps)
{
    HIPCHK(c, hipSetDevice(c->device));
    s.nz = nz;
    s.desc.assign(nz, ccsx::ZmwDesc{});
    uint64_t seq_b = 0, ws_b = 0, out_b = 0, msa_b = 0, bp_w = 0;
    uint32_t nseg = 0, lmax_all = 0, nmax = 0;
    for (size_t i = 0; i < nz; ++i) {
        const ccsx_zmw_in &zi = z[i];
        uint64_t S, hi;
        uint32_t lmax;
        zmw_extent(zi, S, hi, lmax);
        if (S + zi.nseg + 64 > 0x3FFFFFFFull) {
            c->err = "ZMW too large (sum of segment lengths >= 2^30)";
            return -1;
        }
        ccsx::ZmwDesc &d = s.desc[i];
        ccsx::zcaps(d, S, lmax, zi.nseg, full_caps != 0, c->tight_rows, c->shred_caps ? c->shred_read_cap : 0u,
                    c->tight_out, c->tight_far);
        d.seg0 = nseg;
        d.seq_off = seq_b;
        seq_b += hi;
        ccsx::ZLayout L;
        ccsx::zlayout(L, d);
        d.ws_off = ws_b;
        ws_b = ccsx::align256(ws_b + L.total);
        d.out_off = out_b;
        out_b += d.outcap;
        d.msa_off = msa_b;
        d.msacap = with_msa ? uint32_t((S + 16) * (zi.nseg + 4)) : 0u;
        msa_b += d.msacap;
        // breakpoint log: a round emits >= 1 column and advances >= 1 read
        // cursor, so S + 2 rounds bound any ZMW (full caps); tight caps hold
        // far more than the ~L / 1,900 rounds of a real one
        d.bpcap = c->bp_log ? (full_caps ? uint32_t(S + 2) : uint32_t(S / 512 + 64)) : 0u;
        d.bp_off = bp_w;
        bp_w += c->bp_log ? 1 + 2 * uint64_t(d.bpcap) : 0;
        nseg += zi.nseg;
        lmax_all = std::max(lmax_all, lmax);
        nmax = std::max(nmax, zi.nseg);
    }
    s.seq_bytes = seq_b, s.ws_bytes = ws_b, s.out_bytes = out_b, s.msa_bytes = msa_b;
    s.bp_words = bp_w;
    s.nseg_total = nseg;
    // 2-bit read buffer (ccsx_kernel.hip stage_read); at least one band:
    // every lane reads its window bytes even when the read is shorter.  A
    // slice with a read or a cursor array beyond the LDS budget runs the
    // HBM-read kernel instance (lds_read_words = 0)
    const bool shred_tight = c->shred_caps && !full_caps;
    if (nmax > kLdsMaxSegs || (lmax_all > kLdsReadMaxBases && !shred_tight)) {
        s.lds_read_words = 0;
        s.lds_nmax = 0;
    } else {
        // shredded mode pushes windows of ~2-5 kb, not whole segments: with
        // tight caps the buffer is capped at shred_read_cap bases (a longer
        // window fails the ZMW with kErrReadLen and ccsx_gpu_run re-runs it
        // uncapped), which keeps the LDS of config-E slices small enough for
        // one more workgroup per CU
        uint32_t lb = std::max<uint32_t>(lmax_all, ccsx::kW);
        if (shred_tight) lb = std::min(lb, c->shred_read_cap);
        s.lds_read_words = (lb + 15) / 16 + 2;
        s.lds_nmax = std::max<uint32_t>(nmax, 1);
    }
    // LDS words after the configuration's fixed part: the read buffer and
    // the cursors, or the HBM-read instance's read window
    s.lds_extra = s.lds_read_words ? s.lds_read_words + s.lds_nmax : ccsx::kRdWinBytes / 4;
    // kernel configuration (ccsx_layout.h KernelCfg): the latency one if it
    // keeps the whole slice resident; the solo one (one-wave workgroups, ~3x
    // the resident ZMWs) once the slice is several times what the occupancy
    // one keeps resident, so the launch is bound by resident ZMWs rather than
    // by its slowest ZMW's chain (which is ~44 % longer there: config D 316
    // GCUPS solo vs 245 two-wave vs 213 occupancy, config B 74 vs 52 ms;
    // profiles/r03/r03n_*); the occupancy one in between.  (The two-wave
    // throughput configuration is only chosen by ccsx_gpu_set_kernel_cfg.)
    {
        const uint32_t extra = s.lds_extra;
        const size_t res_lat = (size_t)c->ncu * kcfg_wg_per_cu(ccsx::kCfgLatency, extra);
        const size_t res_occ = (size_t)c->ncu * kcfg_wg_per_cu(ccsx::kCfgOccupancy, extra);
        s.cfg = nz <= res_lat ? ccsx::kCfgLatency : nz < kSoloSliceFactor * res_occ ? ccsx::kCfgOccupancy
                                                                                  : ccsx::kCfgSolo16;
        // solo16 at 80 VGPRs, 24 workgroups per CU (solo16w), where the
        // slice's ZMWs have few segments: their DPs' rows are mostly the fast
        // chain rows, which stay in registers at 80 VGPRs (16,384 config-E
        // ZMWs per launch: 582 -> 569 ms); many segments make the multi-
        // predecessor rows, whose predecessor lists then live in scratch,
        // frequent (config D, 30 passes: 314 -> 319 ms), so those keep 96
        // VGPRs and 20 per CU (r06c)
        if (s.cfg == ccsx::kCfgSolo16 && nseg < (uint64_t)kSolo16WMaxSegs * nz) s.cfg = ccsx::kCfgSolo16W;
        if (c->cfg_force >= 0) s.cfg = c->cfg_force;
        // solo16 (int16 ring) takes the LDS instance with pushed reads of at
        // most its max_read bases (a tight-cap shredded slice pushes at most
        // its read cap); other slices run the solo object, forced or not
        if (s.cfg == ccsx::kCfgSolo16 || s.cfg == ccsx::kCfgSolo16W) {
            const uint32_t mr = kcfg_info(s.cfg).max_read;
            const uint32_t pushed = shred_tight ? std::min(lmax_all, c->shred_read_cap) : lmax_all;
            if (!s.lds_read_words || (mr && pushed > mr)) s.cfg = ccsx::kCfgSolo;
        }
    }
    const auto ti = std::chrono::steady_clock::now();
    const uint64_t need = seq_b + ws_b + out_b + msa_b + bp_w * 4 + uint64_t(nseg) * 8 + nz * (sizeof(ccsx::ZmwDesc) + 32);
    {
        // a neighbour still holding memory: wait for it (ccsx_gpu_run has
        // already cut the slice to what is free; a submitted batch cannot be cut)
        bool fits = false;
        const int r = wait_slot_mem(c, s, need, fits);
        if (r) return r;
        if (!fits) {
            size_t freeb = 0, totb = 0;
            HIPCHK(c, hipMemGetInfo(&freeb, &totb));
            char m[200];
            snprintf(m, sizeof m, "batch needs %.1f GB of device memory, %.1f GB free after waiting %u ms: use a smaller chunk",
                     need / 1e9, freeb / 1e9, c->mem_wait_ms);
            c->err = m;
            return -1;
        }
    }
    const bool timing = getenv("CCSX_TIMING") && atoi(getenv("CCSX_TIMING"));
    using tms = std::chrono::duration<double, std::milli>;
    const auto ta = std::chrono::steady_clock::now();
    HIPCHK(c, s.d_seq.reserve(seq_b));
    HIPCHK(c, s.d_soff.reserve(size_t(nseg) * 4));
    HIPCHK(c, s.d_slen.reserve(size_t(nseg) * 4));
    HIPCHK(c, s.d_desc.reserve(nz * sizeof(ccsx::ZmwDesc)));
    HIPCHK(c, s.d_order.reserve(nz * 4));
    HIPCHK(c, s.d_ws.reserve(ws_b));
    HIPCHK(c, s.d_out.reserve(out_b));
    HIPCHK(c, s.d_msa.reserve(msa_b));
    HIPCHK(c, s.d_olen.reserve(nz * 4));
    HIPCHK(c, s.d_ncols.reserve(nz * 4));
    HIPCHK(c, s.d_status.reserve(nz * 4));
    HIPCHK(c, s.d_cells.reserve(nz * 8));
    if (bp_w) HIPCHK(c, s.d_bp.reserve(bp_w * 4));
    const auto tb = std::chrono::steady_clock::now();
    // host staging of the sequence arena and segment tables
    s.hoff.resize(nseg);
    s.hlen.resize(nseg);
    const size_t nthr = c->mem_share > 1 ? 1 : std::min<size_t>(std::min<size_t>(8, nz), std::max<uint64_t>(1, seq_b >> 27));
    const size_t piece = c->stage_piece ? (size_t)c->stage_piece : kStagePiece;
    if (c->prealloc && nthr <= 1 && seq_b > 2 * piece) {
        // a context sharing its device (the CLI's): packed on this thread in
        // pieces through two pinned halves of kStagePiece, each copied while
        // the next is packed -- 128 MiB pinned per slot instead of the whole
        // slice (~1.1 GB for 8,192 config-E ZMWs), which the process exit or
        // ccsx_gpu_close otherwise pays to unpin
        HIPCHK(c, s.h_seq.reserve(2 * piece, 0, true));
        uint8_t *buf[2] = {s.h_seq.p, s.h_seq.p + piece};
        bool used[2] = {false, false};
        int pb = 0;
        size_t ps = 0, fill = 0;  // the piece's slice offset and its bytes
        auto flush = [&]() -> hipError_t {
            hipError_t e = hipMemcpyAsync(s.d_seq.as<uint8_t>() + ps, buf[pb], fill, hipMemcpyHostToDevice, s.stream);
            if (e == hipSuccess) e = hipEventRecord(s.evp[pb], s.stream);
            used[pb] = true;
            ps += fill, fill = 0;
            pb ^= 1;
            // the other half's copy has to be done before it is refilled
            if (e == hipSuccess && used[pb]) e = hipEventSynchronize(s.evp[pb]);
            return e;
        };
        for (size_t i = 0; i < nz; ++i) {
            const ccsx_zmw_in &zi = z[i];
            const ccsx::ZmwDesc &d = s.desc[i];
            uint64_t hi = 0;
            for (uint32_t k = 0; k < zi.nseg; ++k) {
                s.hoff[d.seg0 + k] = zi.seg_off[k];
                s.hlen[d.seg0 + k] = zi.seg_len[k];
                hi = std::max<uint64_t>(hi, uint64_t(zi.seg_off[k]) + zi.seg_len[k]);
            }
            // (d.seq_off == ps + fill: ZMWs are packed back to back)
            for (uint64_t done = 0; done < hi;) {
                const size_t n = (size_t)std::min<uint64_t>(hi - done, piece - fill);
                memcpy(buf[pb] + fill, zi.seqs + done, n);
                fill += n, done += n;
                if (fill == piece) HIPCHK(c, flush());
            }
        }
        if (fill) HIPCHK(c, flush());
    } else {
        HIPCHK(c, s.h_seq.reserve(seq_b, c->prealloc ? kPinnedSeqFloor / c->mem_share : 0));
        uint8_t *hseq = s.h_seq.p;
        // the packing is a memory copy of the whole slice's subreads (1.8 GB for
        // a 10k-ZMW config-E slice, ~100 ms on one thread): split over threads,
        // since the slice's kernel cannot start before it is done (16,384-ZMW
        // e2e line 17.3k -> 19.2k ZMWs/s, r03y).  Contexts sharing a device (the
        // CLI's two per GPU) stage while the other's kernels run and keep to one
        // thread, leaving the CPUs to the host pipeline's preparation.
        auto pack = [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i) {
                const ccsx_zmw_in &zi = z[i];
                const ccsx::ZmwDesc &d = s.desc[i];
                uint64_t hi = 0;
                for (uint32_t k = 0; k < zi.nseg; ++k) {
                    s.hoff[d.seg0 + k] = zi.seg_off[k];
                    s.hlen[d.seg0 + k] = zi.seg_len[k];
                    hi = std::max<uint64_t>(hi, uint64_t(zi.seg_off[k]) + zi.seg_len[k]);
                }
                if (hi) memcpy(hseq + d.seq_off, zi.seqs, hi);
            }
        };
        if (nthr <= 1) {
            pack(0, nz);
        } else {
            std::vector<std::thread> th;
            for (size_t t = 1; t < nthr; ++t) th.emplace_back(pack, nz * t / nthr, nz * (t + 1) / nthr);
            pack(0, nz / nthr);
            for (auto &x : th) x.join();
        }
        HIPCHK(c, hipMemcpyAsync(s.d_seq.p, hseq, seq_b, hipMemcpyHostToDevice, s.stream));
    }
    HIPCHK(c, hipMemcpyAsync(s.d_soff.p, s.hoff.data(), size_t(nseg) * 4, hipMemcpyHostToDevice, s.stream));
    HIPCHK(c, hipMemcpyAsync(s.d_slen.p, s.hlen.data(), size_t(nseg) * 4, hipMemcpyHostToDevice, s.stream));
    HIPCHK(c, hipMemcpyAsync(s.d_desc.p, s.desc.data(), nz * sizeof(ccsx::ZmwDesc), hipMemcpyHostToDevice, s.stream));
    // launch order: decreasing estimated POA work (ccsx_zmw_cost: S x (28 +
    // n)), ties in input order -- longest-processing-time first, so a launch
    // ends on its cheapest ZMWs
    s.order.resize(nz);
    std::vector<uint64_t> cost(nz);
    for (size_t i = 0; i < nz; ++i) s.order[i] = uint32_t(i), cost[i] = ccsx_zmw_cost(z[i].seg_len, z[i].nseg);
    std::stable_sort(s.order.begin(), s.order.end(), [&](uint32_t x, uint32_t y) { return cost[x] > cost[y]; });
    HIPCHK(c, hipMemcpyAsync(s.d_order.p, s.order.data(), nz * 4, hipMemcpyHostToDevice, s.stream));
    if (timing)
        fprintf(stderr, "[ccsx_gpu_stage] %zu ZMWs: meminfo %.0f ms, reserve %.0f ms (ws cap %.1f GB), pack %.1f MB %.0f ms\n",
                nz, tms(ta - ti).count(), tms(tb - ta).count(), s.d_ws.cap / 1e9, seq_b / 1e6,
                tms(std::chrono::steady_clock::now() - tb).count());
    return 0;
}

// Enqueue the slot's kernel between its two events (asynchronous)
static int launch_slot(ccsx_ctx *c, Slot &s, int mode)
{
    HIPCHK(c, hipSetDevice(c->device));
    ccsx::KArgs a{};
    a.seq = s.d_seq.as<uint8_t>();
    a.soff = s.d_soff.as<uint32_t>();
    a.slen = s.d_slen.as<uint32_t>();
    a.desc = s.d_desc.as<ccsx::ZmwDesc>();
    a.order = s.d_order.as<uint32_t>();
    a.ws = s.d_ws.as<uint8_t>();
    a.out = s.d_out.as<uint8_t>();
    a.msa = s.d_msa.as<uint8_t>();
    a.out_len = s.d_olen.as<uint32_t>();
    a.ncols = s.d_ncols.as<uint32_t>();
    a.status = s.d_status.as<int32_t>();
    a.cells = s.d_cells.as<unsigned long long>();
    a.mode = mode;
    a.nzmw = uint32_t(s.nz);
    a.lds_read_words = s.lds_read_words;
    a.lds_nmax = s.lds_nmax;
    a.prof = nullptr;
    a.bplog = s.bp_words ? s.d_bp.as<uint32_t>() : nullptr;
    if (c->profiling) {
        HIPCHK(c, s.d_prof.reserve(s.nz * ccsx::kProfSlots * 8));
        a.prof = s.d_prof.as<unsigned long long>();
    }
    uint32_t lds = kcfg_lds(s.cfg, s.lds_extra);
    if (c->wg_cap) lds = std::max<uint32_t>(lds, 160u * 1024u / (c->wg_cap + 1) + 1024u);
    if (lds > 160 * 1024) {
        c->err = "reads too long for the LDS read buffer";
        return -1;
    }
    HIPCHK(c, hipEventRecord(s.ev0, s.stream));
    HIPCHK(c, kLaunch[s.cfg](&a, lds, s.stream));
    HIPCHK(c, hipEventRecord(s.ev1, s.stream));
    s.inflight = true;
    return 0;
}

// Copy the slot's results back (after its kernel: same stream) and wait for
// them; out[i] for i < s.nz.  Returns 0, -2 (some ZMWs failed) or -1.
static int fetch_slot(ccsx_ctx *c, Slot &s, ccsx_zmw_out *out)
{
    HIPCHK(c, hipSetDevice(c->device));
    const size_t nz = s.nz;
    HIPCHK(c, s.h_out.reserve(s.out_bytes, c->prealloc ? kPinnedOutFloor / c->mem_share : 0));
    s.h_olen.resize(nz);
    s.h_status.resize(nz);
    s.h_cells.resize(nz);
    s.h_bp.resize(s.bp_words);
    if (nz) {
        HIPCHK(c, hipMemcpyAsync(s.h_olen.data(), s.d_olen.p, nz * 4, hipMemcpyDeviceToHost, s.stream));
        HIPCHK(c, hipMemcpyAsync(s.h_status.data(), s.d_status.p, nz * 4, hipMemcpyDeviceToHost, s.stream));
        HIPCHK(c, hipMemcpyAsync(s.h_cells.data(), s.d_cells.p, nz * 8, hipMemcpyDeviceToHost, s.stream));
        HIPCHK(c, hipMemcpyAsync(s.h_out.p, s.d_out.p, s.out_bytes, hipMemcpyDeviceToHost, s.stream));
        if (s.bp_words)
            HIPCHK(c, hipMemcpyAsync(s.h_bp.data(), s.d_bp.p, s.bp_words * 4, hipMemcpyDeviceToHost, s.stream));
    }
    HIPCHK(c, hipStreamSynchronize(s.stream));
    s.inflight = false;
    int bad = 0;
    for (size_t i = 0; i < nz; ++i) {
        out[i].ccs = reinterpret_cast<const char *>(s.h_out.p + s.desc[i].out_off);
        out[i].len = s.h_status[i] ? 0 : s.h_olen[i];
        out[i].status = s.h_status[i];
        out[i].cells = s.h_cells[i];
        if (s.h_status[i] && !bad) {
            bad = 1;
            char m[200];
            snprintf(m, sizeof m, "ZMW %zu of the batch failed on the device: %s", i,
                     ccsx_gpu_status_str(s.h_status[i]));
            c->err = m;
        }
    }
    return bad ? -2 : 0;
}

extern "C" {

// internal: stage with an optional MSA slab per ZMW (single-POA mode) and
// full (exact upper bound) or tight capacities (ccsx_layout.h:zcaps); slot 0
int ccsx_gpu_stage_ex(ccsx_ctx *c, const ccsx_zmw_in *z, size_t nz, int with_msa, int full_caps)
{
    if (!c) return -1;
    Slot &s = c->slot[0];
    if (s.inflight) {  // launched, never fetched: its results are dropped
        HIPCHK(c, hipStreamSynchronize(s.stream));
        s.inflight = false;
    }
    const int r = stage_slot(c, s, z, nz, with_msa, full_caps);
    if (r) return r;
    HIPCHK(c, hipStreamSynchronize(s.stream));
    return 0;
}

int ccsx_gpu_stage(ccsx_ctx *c, const ccsx_zmw_in *z, size_t nz) { return ccsx_gpu_stage_ex(c, z, nz, 0, 0); }

int ccsx_gpu_stage_for(ccsx_ctx *c, int mode, const ccsx_zmw_in *z, size_t nz)
{
    if (!c) return -1;
    if (mode != CCSX_MODE_SHRED && mode != CCSX_MODE_PRIMITIVE) {
        c->err = "mode must be CCSX_MODE_SHRED or CCSX_MODE_PRIMITIVE";
        return -1;
    }
    c->shred_caps = mode == CCSX_MODE_SHRED;
    const int r = ccsx_gpu_stage_ex(c, z, nz, 0, 0);
    c->shred_caps = false;
    return r;
}

int ccsx_gpu_launch_ex(ccsx_ctx *c, int mode, float *kernel_ms)
{
    if (!c) return -1;
    Slot &s = c->slot[0];
    if (s.nz == 0) {
        if (kernel_ms) *kernel_ms = 0.f;
        return 0;
    }
    const int r = launch_slot(c, s, mode);
    if (r) return r;
    HIPCHK(c, hipEventSynchronize(s.ev1));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, s.ev0, s.ev1));
    if (kernel_ms) *kernel_ms = ms;
    return 0;
}

int ccsx_gpu_launch(ccsx_ctx *c, int mode, float *kernel_ms)
{
    if (mode != CCSX_MODE_SHRED && mode != CCSX_MODE_PRIMITIVE) {
        if (c) c->err = "mode must be CCSX_MODE_SHRED or CCSX_MODE_PRIMITIVE";
        return -1;
    }
    return ccsx_gpu_launch_ex(c, mode, kernel_ms);
}

int ccsx_gpu_fetch(ccsx_ctx *c, ccsx_zmw_out *out)
{
    if (!c) return -1;
    return fetch_slot(c, c->slot[0], out);
}

// The bytes one slot's slice may take: what is free plus what the workspaces
// already hold, at most this context's share of the device (mem_frac /
// mem_share), halved for the two slots in flight; a preallocating context
// reserves both slots' workspaces at that size on its first call.
static int plan_slots(ccsx_ctx *c, uint64_t &slot_budget)
{
    size_t freeb = 0, totb = 0;
    HIPCHK(c, hipMemGetInfo(&freeb, &totb));
    // the workspaces may grow into what is free plus what they already hold;
    // the sequence / output arenas they would need beside them stay counted
    // as used (they are re-reserved per slice, not released)
    const uint64_t held = c->slot[0].d_ws.cap + c->slot[1].d_ws.cap;
    uint64_t budget = freeb + held > (3ull << 30) ? freeb + held - (3ull << 30) : (1ull << 30);
    {
        // a fixed share of the device per context (contexts running
        // concurrently cannot all size themselves to the same free memory):
        // allocating up to the last free GB measured 6.3 s of staging for a
        // 305 GB slice vs 0.18 s for 84 GB
        const uint64_t part = (uint64_t)((double)totb * c->mem_frac / c->mem_share);
        budget = std::max<uint64_t>(1ull << 30, std::min<uint64_t>(budget, part > (2ull << 30) ? part - (2ull << 30) : 0));
    }
    // two slots in flight: each holds half
    slot_budget = c->slot_budget ? c->slot_budget : std::max<uint64_t>(1ull << 29, budget / 2);
    if (c->prealloc) {
        const bool timing = getenv("CCSX_TIMING") && atoi(getenv("CCSX_TIMING"));
        // only idle slots: a slot whose batch is still running keeps its
        // workspace (growing it would free the memory under that kernel; the
        // slot is grown by the next plan that finds it idle)
        for (int k = 0; k < 2; ++k) {
            Slot &s = c->slot[k];
            if (c->tk[k].pending || s.inflight) continue;
            if (s.d_ws.cap < slot_budget) {
                const auto t0 = std::chrono::steady_clock::now();
                HIPCHK(c, s.d_ws.reserve(slot_budget, true));
                if (timing)
                    fprintf(stderr, "[ccsx_gpu_run] dev %d: workspace of %.1f GB reserved in %.0f ms\n", c->device,
                            slot_budget / 1e9,
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            }
        }
    }
    return 0;
}

// statuses of a tight-cap slice that the full-cap (uncapped read buffer) re-run clears
static bool is_cap_error(int32_t s)
{
    return s == ccsx::kErrRows || s == ccsx::kErrEdges || s == ccsx::kErrMulti || s == ccsx::kErrSpill ||
           s == ccsx::kErrReadLen || s == ccsx::kErrBpLog || s == ccsx::kErrOut;
}

// One chunk.  The chunk is cut into slices that fit the device's free memory
// (tight caps); a ZMW that outgrows a tight cap is re-run with full caps.
// Slices alternate between the context's two slots: slice k + 1 is staged and
// launched while slice k's kernel runs, and slice k's results are collected
// when its slot is needed again (or at the end).
int ccsx_gpu_run(ccsx_ctx *c, int mode, const ccsx_zmw_in *z, size_t nz, ccsx_zmw_out *out)
{
    if (!c) return -1;
    if (mode != CCSX_MODE_SHRED && mode != CCSX_MODE_PRIMITIVE) {
        c->err = "mode must be CCSX_MODE_SHRED or CCSX_MODE_PRIMITIVE";
        return -1;
    }
    HIPCHK(c, hipSetDevice(c->device));
    for (Slot &s : c->slot)
        if (s.inflight) {  // a stage/launch without fetch: drop its results
            HIPCHK(c, hipStreamSynchronize(s.stream));
            s.inflight = false;
        }
    c->tk[0].pending = c->tk[1].pending = false;  // (uncollected submitted batches are dropped)
    struct ShredCaps {  // the window-sized tight caps for this call only
        ccsx_ctx *c;
        ShredCaps(ccsx_ctx *x, bool on) : c(x) { c->shred_caps = on; }
        ~ShredCaps() { c->shred_caps = false; }
    } shred_caps(c, mode == CCSX_MODE_SHRED);
    uint64_t slot_budget = 0;
    {
        const int r = plan_slots(c, slot_budget);
        if (r) return r;
    }
    const bool timing = getenv("CCSX_TIMING") && atoi(getenv("CCSX_TIMING"));
    using ms = std::chrono::duration<double, std::milli>;
    const auto t_run = std::chrono::steady_clock::now();
    c->run_arena.clear();
    c->run_bp.clear();
    c->run_bp_off.assign(nz, 0);
    c->run_bp_n.assign(nz, 0);
    std::vector<uint64_t> aoff(nz, 0);
    std::vector<int> cls(nz, 0);
    std::string first_err;
    // results of the slice in slot s (input indices idx[b, b + s.nz))
    struct Pending {
        const std::vector<uint32_t> *idx = nullptr;
        size_t b = 0;
        std::vector<uint32_t> *retry = nullptr;
        std::chrono::steady_clock::time_point t0;
    } pend[2];
    std::vector<ccsx_zmw_out> o;
    auto collect = [&](int si) -> int {
        Slot &s = c->slot[si];
        if (!s.inflight) return 0;
        o.assign(s.nz, ccsx_zmw_out{});
        const int r = fetch_slot(c, s, o.data());
        if (r && r != -2) return r;
        if (timing) {
            float kms = 0.f;
            (void)hipEventElapsedTime(&kms, s.ev0, s.ev1);
            fprintf(stderr, "[ccsx_gpu_run] dev %d slot %d: %zu ZMWs (cfg %d), kernel %.0f ms, staged..collected %.0f-%.0f ms\n",
                    c->device, si, s.nz, s.cfg, kms, ms(pend[si].t0 - t_run).count(),
                    ms(std::chrono::steady_clock::now() - t_run).count());
        }
        const Pending &p = pend[si];
        {
            // one growth of the gathered CCS arena per slice, not one per
            // ZMW's append (~150 MB for a 10k-ZMW config-E slice)
            size_t add = 0;
            for (size_t i = 0; i < s.nz; ++i) add += o[i].status ? 0 : o[i].len;
            c->run_arena.reserve(c->run_arena.size() + add);
        }
        for (size_t i = 0; i < s.nz; ++i) {
            const uint32_t g = (*p.idx)[p.b + i];
            out[g].cells = o[i].cells;
            out[g].status = o[i].status;
            out[g].len = 0;
            if (o[i].status) {
                if (p.retry && is_cap_error(o[i].status)) {
                    p.retry->push_back(g);
                } else if (first_err.empty()) {
                    char m[200];
                    snprintf(m, sizeof m, "ZMW %u of the batch failed on the device: %s", g,
                             ccsx_gpu_status_str(o[i].status));
                    first_err = m;
                }
                continue;
            }
            aoff[g] = c->run_arena.size();
            out[g].len = o[i].len;
            c->run_arena.insert(c->run_arena.end(), o[i].ccs, o[i].ccs + o[i].len);
            if (s.bp_words && mode == CCSX_MODE_SHRED) {
                const uint32_t *lg = s.h_bp.data() + s.desc[i].bp_off;
                c->run_bp_off[g] = c->run_bp.size() / 2;
                c->run_bp_n[g] = lg[0];
                c->run_bp.insert(c->run_bp.end(), lg + 1, lg + 1 + 2 * uint64_t(lg[0]));
            }
        }
        return 0;
    };
    int next_slot = 0;
    std::vector<ccsx_zmw_in> sub;
    std::vector<uint32_t> inter;  // run_list's interleaved order (lives until its slots are collected)
    auto run_list = [&](const std::vector<uint32_t> &idx0, bool full, std::vector<uint32_t> *retry) -> int {
        // A list of one launch class that needs k > 1 slots is dealt into k
        // interleaved parts (cost rank i goes to part i % k, each part still
        // most expensive first) instead of being cut into contiguous runs of
        // the cost order: consecutive parts run side by side on the two
        // slots and each ends on cheap ZMWs, so they end together and no
        // slice is a small tail of the cheapest ZMWs (a latency-object
        // launch), nor the most expensive ones running alone with a sparse
        // tail (16,384 config-E ZMWs cut contiguously: the 5,671 cheap ones
        // done after 180 ms, the other 10,713 after 737 ms; one launch of
        // all of them: 698 ms).  k grows until every part fits a slot.
        const std::vector<uint32_t> *lp = &idx0;
        std::vector<size_t> cuts;  // part boundaries in *lp
        bool one_class = !idx0.empty();
        for (uint32_t g : idx0) one_class = one_class && cls[g] == cls[idx0.front()];
        if (one_class) {
            std::vector<uint64_t> xb(idx0.size());
            uint64_t tot = 0, xmax = 0;
            for (size_t i = 0; i < idx0.size(); ++i) {
                xb[i] = zmw_bytes(z[idx0[i]], full, c, c->shred_caps ? c->shred_read_cap : 0u);
                tot += xb[i];
                xmax = std::max(xmax, xb[i]);
            }
            if (tot > slot_budget && xmax <= slot_budget) {
                const size_t k0 = size_t((tot + slot_budget - 1) / slot_budget);
                for (size_t k = k0; k <= std::min<size_t>(idx0.size(), k0 + 8); ++k) {
                    std::vector<uint64_t> part(k, 0);
                    for (size_t i = 0; i < idx0.size(); ++i) part[i % k] += xb[i];
                    if (*std::max_element(part.begin(), part.end()) > slot_budget) continue;
                    inter.clear();
                    for (size_t p = 0; p < k; ++p) {
                        if (p) cuts.push_back(inter.size());
                        for (size_t i = p; i < idx0.size(); i += k) inter.push_back(idx0[i]);
                    }
                    lp = &inter;
                    ++c->dealt;
                    c->parts += k;
                    break;
                }
            }
        }
        const std::vector<uint32_t> &idx = *lp;
        size_t b = 0, ci = 0;
        while (b < idx.size()) {
            while (ci < cuts.size() && cuts[ci] <= b) ++ci;
            const size_t cut = ci < cuts.size() ? cuts[ci] : SIZE_MAX;
            int si = next_slot;
            next_slot ^= 1;
            int r = collect(si);  // the slot's previous slice
            if (r) return r;
            // the slice as planned, cut further to what the device holds free
            // for this slot now (a neighbour may still hold part of this
            // context's share).  If not even its first ZMW fits, the other
            // slot's arenas may hold the room: finish that slot's slice and
            // stage there (the slices then run one after the other); else
            // wait for a neighbour to release memory.
            uint64_t lim = slot_budget;
            {
                uint64_t avail = 0;
                if ((r = slot_avail(c, c->slot[si], avail))) return r;
                const uint64_t x0 = zmw_bytes(z[idx[b]], full, c, c->shred_caps ? c->shred_read_cap : 0u);
                if (avail < x0) {
                    const int so = si ^ 1;
                    if ((r = collect(so))) return r;
                    uint64_t a2 = 0;
                    if ((r = slot_avail(c, c->slot[so], a2))) return r;
                    if (a2 > avail) si = so, avail = a2;  // (next_slot is already so: the next slice waits for this one)
                }
                if (avail < x0) {
                    bool fits = false;
                    if ((r = wait_slot_mem(c, c->slot[si], x0, fits))) return r;
                    if ((r = slot_avail(c, c->slot[si], avail))) return r;
                }
                lim = std::min(lim, avail);
            }
            uint64_t need = 0;
            size_t e = b;
            while (e < idx.size()) {
                const uint64_t x = zmw_bytes(z[idx[e]], full, c, c->shred_caps ? c->shred_read_cap : 0u);
                if (e > b && (need + x > lim || cls[idx[e]] != cls[idx[b]] || e == cut)) break;
                need += x;
                ++e;
            }
            if (lim < slot_budget && (e < idx.size() && e != cut && need + zmw_bytes(z[idx[e]], full, c,
                                                                                c->shred_caps ? c->shred_read_cap : 0u) <= slot_budget &&
                                      cls[idx[e]] == cls[idx[b]]))
                ++c->mem_replans;  // cut below the plan by the free memory
            sub.resize(e - b);
            for (size_t i = b; i < e; ++i) sub[i - b] = z[idx[i]];
            pend[si].idx = &idx;
            pend[si].b = b;
            pend[si].retry = retry;
            pend[si].t0 = std::chrono::steady_clock::now();
            r = stage_slot(c, c->slot[si], sub.data(), sub.size(), 0, full ? 1 : 0);
            if (r) return r;
            r = launch_slot(c, c->slot[si], mode);
            if (r) return r;
            ++c->slices;
            b = e;
        }
        // both slots' results before the list's vectors go away
        for (int k = 0; k < 2; ++k) {
            const int r = collect(next_slot ^ (k == 0 ? 1 : 0));
            if (r) return r;
        }
        return 0;
    };
    // slices: by launch class, then most expensive first -- when a call needs
    // several slices, the last one holds the cheapest ZMWs, whose launch (a
    // few waves of workgroups) ends soonest
    std::vector<uint32_t> all(nz), retry;
    std::vector<uint64_t> cost(nz);
    for (size_t i = 0; i < nz; ++i)
        all[i] = uint32_t(i), cls[i] = zmw_class(z[i], c->shred_caps), cost[i] = ccsx_zmw_cost(z[i].seg_len, z[i].nseg);
    std::stable_sort(all.begin(), all.end(),
                     [&](uint32_t x, uint32_t y) { return cls[x] != cls[y] ? cls[x] < cls[y] : cost[x] > cost[y]; });
    int r = run_list(all, false, &retry);
    if (!r && !retry.empty()) {
        for (uint32_t g : retry) cls[g] = zmw_class(z[g], false);  // full caps: whole segments in the buffer
        // the tight pass had them all in class 0: regroup by the new classes
        // (most expensive first within each), so a slice never ends at every
        // class change of an alternating list
        std::stable_sort(retry.begin(), retry.end(),
                         [&](uint32_t x, uint32_t y) { return cls[x] != cls[y] ? cls[x] < cls[y] : cost[x] > cost[y]; });
        if (timing) fprintf(stderr, "[ccsx_gpu_run] dev %d: %zu ZMWs re-run with full caps\n", c->device, retry.size());
        c->reruns += retry.size();
        r = run_list(retry, true, nullptr);
    }
    if (r) {
        for (Slot &s : c->slot)
            if (s.inflight) (void)hipStreamSynchronize(s.stream), s.inflight = false;
        return r;
    }
    if (c->fault >= 0 && (size_t)c->fault < nz) {
        out[c->fault].status = ccsx::kErrTrace;
        out[c->fault].len = 0;
        if (first_err.empty()) first_err = "ZMW failed on the device: injected fault (test hook)";
    }
    c->fault = -1;
    for (size_t i = 0; i < nz; ++i) out[i].ccs = reinterpret_cast<const char *>(c->run_arena.data() + aoff[i]);
    if (!first_err.empty()) {
        c->err = first_err;
        return -2;
    }
    return 0;
}

// Asynchronous batches: a batch that fits one slot runs as one launch on a
// free slot; the caller submits its next batch before collecting the
// previous one, so the device always holds the next launch (whose workgroups
// fill the CUs the current launch's tail frees) and the host's staging and
// gathering overlap the kernels -- where ccsx_gpu_run's callers wait for
// every slice of a call before staging the next call.
int ccsx_gpu_slot_bytes(ccsx_ctx *c, uint64_t *bytes)
{
    if (!c || !bytes) return -1;
    HIPCHK(c, hipSetDevice(c->device));
    return plan_slots(c, *bytes);
}

int ccsx_gpu_reserve_staging(ccsx_ctx *c, uint64_t seq_bytes, uint64_t out_bytes)
{
    if (!c) return -1;
    HIPCHK(c, hipSetDevice(c->device));
    // the slot the next submit takes; exact sizes (a later batch grows them).
    // A context sharing its device stages subreads piecewise: two halves
    if (c->prealloc && c->mem_share > 1)
        seq_bytes = std::min<uint64_t>(seq_bytes, 2 * (c->stage_piece ? c->stage_piece : kStagePiece));
    for (int k = 0; k < 2; ++k) {
        if (c->tk[k].pending) continue;
        Slot &s = c->slot[k];
        HIPCHK(c, s.h_seq.reserve(seq_bytes, 0, true));
        HIPCHK(c, s.h_out.reserve(out_bytes, 0, true));
        break;
    }
    return 0;
}

int ccsx_gpu_submit(ccsx_ctx *c, int mode, const ccsx_zmw_in *z, size_t nz, int *slot)
{
    if (!c || !slot || (!z && nz)) return -1;
    if (mode != CCSX_MODE_SHRED && mode != CCSX_MODE_PRIMITIVE) {
        c->err = "mode must be CCSX_MODE_SHRED or CCSX_MODE_PRIMITIVE";
        return -1;
    }
    HIPCHK(c, hipSetDevice(c->device));
    int si = -1;
    for (int k = 0; k < 2 && si < 0; ++k)
        if (!c->tk[k].pending) si = k;
    if (si < 0) {
        c->err = "both slots hold batches not collected yet";
        return -3;
    }
    Slot &s = c->slot[si];
    if (s.inflight) {  // a stage/launch without fetch on this slot: drop its results
        HIPCHK(c, hipStreamSynchronize(s.stream));
        s.inflight = false;
    }
    uint64_t slot_budget = 0;
    int r = plan_slots(c, slot_budget);
    if (r) return r;
    c->shred_caps = mode == CCSX_MODE_SHRED;
    uint64_t tot = 0;
    bool one_class = true;
    for (size_t i = 0; i < nz; ++i) {
        tot += zmw_bytes(z[i], false, c, c->shred_caps ? c->shred_read_cap : 0u);
        one_class = one_class && zmw_class(z[i], c->shred_caps) == zmw_class(z[0], c->shred_caps);
    }
    if (tot > slot_budget || !one_class) {
        c->shred_caps = false;
        char m[160];
        snprintf(m, sizeof m, "batch of %.1f GB (%s) does not fit one %.1f GB slot: use ccsx_gpu_run", tot / 1e9,
                 one_class ? "one launch class" : "several launch classes", slot_budget / 1e9);
        c->err = m;
        return -4;
    }
    r = stage_slot(c, s, z, nz, 0, 0);
    if (!r) r = launch_slot(c, s, mode);
    c->shred_caps = false;
    if (r) return r;
    ++c->slices;
    c->tk[si].pending = true;
    c->tk[si].mode = mode;
    c->tk[si].z = z;
    c->tk[si].nz = nz;
    c->tk[si].fault = c->fault;
    c->fault = -1;
    *slot = si;
    return 0;
}

int ccsx_gpu_collect(ccsx_ctx *c, int si, ccsx_zmw_out *out)
{
    if (!c || si < 0 || si > 1 || !c->tk[si].pending) {
        if (c) c->err = "no batch submitted on that slot";
        return -1;
    }
    HIPCHK(c, hipSetDevice(c->device));
    auto &t = c->tk[si];
    Slot &s = c->slot[si];
    const size_t nz = t.nz;
    const ccsx_zmw_in *z = t.z;
    t.pending = false;
    std::vector<ccsx_zmw_out> o(nz);
    int r = fetch_slot(c, s, o.data());
    if (r && r != -2) return r;
    std::vector<uint64_t> aoff(nz, 0);
    std::vector<uint32_t> retry;
    std::string first_err;
    t.arena.clear();
    auto gather = [&](const ccsx_zmw_out *res, const uint32_t *idx, size_t n, bool can_retry) {
        size_t add = 0;
        for (size_t i = 0; i < n; ++i) add += res[i].status ? 0 : res[i].len;
        t.arena.reserve(t.arena.size() + add);
        for (size_t i = 0; i < n; ++i) {
            const uint32_t g = idx ? idx[i] : (uint32_t)i;
            out[g].cells = res[i].cells;
            out[g].status = res[i].status;
            out[g].len = 0;
            if (res[i].status) {
                if (can_retry && is_cap_error(res[i].status)) {
                    retry.push_back(g);
                } else if (first_err.empty()) {
                    char m[200];
                    snprintf(m, sizeof m, "ZMW %u of the batch failed on the device: %s", g,
                             ccsx_gpu_status_str(res[i].status));
                    first_err = m;
                }
                continue;
            }
            aoff[g] = t.arena.size();
            out[g].len = res[i].len;
            t.arena.insert(t.arena.end(), res[i].ccs, res[i].ccs + res[i].len);
        }
    };
    gather(o.data(), nullptr, nz, true);
    if (!retry.empty()) {
        // ZMWs that outgrew a tight cap: full caps, on this slot, slices of
        // at most the slot budget (rare: none of 500,000 config-E ZMWs)
        c->reruns += retry.size();
        uint64_t slot_budget = 0;
        r = plan_slots(c, slot_budget);
        if (r) return r;
        std::vector<uint32_t> todo;
        todo.swap(retry);
        std::vector<ccsx_zmw_in> sub;
        c->shred_caps = t.mode == CCSX_MODE_SHRED;
        for (size_t b = 0; b < todo.size() && !r;) {
            uint64_t need = 0;
            size_t e = b;
            while (e < todo.size()) {
                const uint64_t x = zmw_bytes(z[todo[e]], true, c, c->shred_caps ? c->shred_read_cap : 0u);
                if (e > b && need + x > slot_budget) break;
                need += x;
                ++e;
            }
            sub.resize(e - b);
            for (size_t i = b; i < e; ++i) sub[i - b] = z[todo[i]];
            r = stage_slot(c, s, sub.data(), sub.size(), 0, 1);
            if (!r) r = launch_slot(c, s, t.mode);
            if (!r) {
                o.assign(sub.size(), ccsx_zmw_out{});
                r = fetch_slot(c, s, o.data());
                if (r == -2) r = 0;
                if (!r) gather(o.data(), todo.data() + b, sub.size(), false);
            }
            ++c->slices;
            b = e;
        }
        c->shred_caps = false;
        if (r) return r;
    }
    if (t.fault >= 0 && (size_t)t.fault < nz) {
        out[t.fault].status = ccsx::kErrTrace;
        out[t.fault].len = 0;
        if (first_err.empty()) first_err = "ZMW failed on the device: injected fault (test hook)";
    }
    for (size_t i = 0; i < nz; ++i) out[i].ccs = reinterpret_cast<const char *>(t.arena.data() + aoff[i]);
    if (!first_err.empty()) {
        c->err = first_err;
        return -2;
    }
    return 0;
}

int ccsx_gpu_set_tight_rows(ccsx_ctx *c, uint32_t rows)
{
    if (!c) return -1;
    c->tight_rows = rows;
    return 0;
}

int ccsx_gpu_set_stage_piece(ccsx_ctx *c, uint64_t bytes)
{
    if (!c) return -1;
    c->stage_piece = bytes;
    return 0;
}

int ccsx_gpu_set_tight_out(ccsx_ctx *c, uint32_t bytes)
{
    if (!c) return -1;
    c->tight_out = bytes;
    return 0;
}

int ccsx_gpu_set_tight_far(ccsx_ctx *c, uint32_t rows)
{
    if (!c) return -1;
    c->tight_far = rows;
    return 0;
}

int ccsx_gpu_set_kernel_cfg(ccsx_ctx *c, int cfg)
{
    if (!c || cfg < -1 || cfg >= ccsx::kCfgCount) return -1;
    c->cfg_force = cfg;
    return 0;
}

int ccsx_gpu_kernel_cfg(const ccsx_ctx *c) { return c ? c->slot[0].cfg : -1; }

int64_t ccsx_gpu_rerun_count(const ccsx_ctx *c) { return c ? (int64_t)c->reruns : -1; }

int ccsx_gpu_run_stats(const ccsx_ctx *c, uint64_t *st, uint32_t n)
{
    if (!c || !st) return -1;
    const uint64_t v[6] = {c->reruns, c->slices, c->dealt, c->parts, c->mem_waits, c->mem_replans};
    for (uint32_t i = 0; i < n && i < 6; ++i) st[i] = v[i];
    return 0;
}

int ccsx_gpu_set_mem_wait(ccsx_ctx *c, uint32_t ms)
{
    if (!c) return -1;
    c->mem_wait_ms = ms;
    return 0;
}

uint64_t ccsx_gpu_zmw_bytes(const ccsx_ctx *c, int mode, const ccsx_zmw_in *z)
{
    if (!c || !z) return 0;
    return zmw_bytes(*z, false, c, mode == CCSX_MODE_SHRED ? c->shred_read_cap : 0u);
}

int ccsx_gpu_set_fault(ccsx_ctx *c, int64_t zmw)
{
    if (!c) return -1;
    c->fault = zmw;
    return 0;
}

int ccsx_gpu_set_slot_budget(ccsx_ctx *c, uint64_t bytes)
{
    if (!c) return -1;
    c->slot_budget = bytes;
    return 0;
}

int ccsx_gpu_set_wg_cap(ccsx_ctx *c, uint32_t wg_per_cu)
{
    if (!c || wg_per_cu > 16) return -1;
    c->wg_cap = wg_per_cu;
    return 0;
}

int ccsx_gpu_set_shred_read_cap(ccsx_ctx *c, uint32_t bases)
{
    if (!c || bases < 1024 || bases > 65536) return -1;
    c->shred_read_cap = bases;
    return 0;
}

int ccsx_gpu_set_mem_frac(ccsx_ctx *c, float frac)
{
    if (!c || !(frac > 0.05f && frac <= 0.95f)) return -1;
    c->mem_frac = frac;
    return 0;
}

int ccsx_gpu_set_mem_share(ccsx_ctx *c, uint32_t share)
{
    if (!c || share == 0) return -1;
    c->mem_share = share;
    return 0;
}

int ccsx_gpu_set_bp_log(ccsx_ctx *c, int on)
{
    if (!c) return -1;
    c->bp_log = on != 0;
    return 0;
}

int ccsx_gpu_bp_log(const ccsx_ctx *c, size_t zmw, const uint32_t **pairs, uint32_t *nrounds)
{
    if (!c || zmw >= c->run_bp_n.size()) return -1;
    *nrounds = c->run_bp_n[zmw];
    *pairs = c->run_bp.data() + 2 * c->run_bp_off[zmw];
    return 0;
}

int ccsx_gpu_set_prealloc(ccsx_ctx *c, int on)
{
    if (!c) return -1;
    c->prealloc = on != 0;
    return 0;
}

int ccsx_gpu_set_profiling(ccsx_ctx *c, int on)
{
    if (!c) return -1;
    if (on) {
        // the product objects compile the counters out (KArgs::prof would
        // receive zeros): only the diagnostic library can profile
        for (int k = 0; k < ccsx::kCfgCount; ++k)
            if (!kcfg_info(k).profiling) {
                c->err = "the loaded kernel objects carry no phase counters: load libccsx_amd_diag.so";
                return -1;
            }
    }
    c->profiling = on != 0;
    return 0;
}

int ccsx_gpu_profile(ccsx_ctx *c, uint64_t *sums, uint32_t nslots)
{
    if (!c || !c->profiling || nslots < (uint32_t)ccsx::kProfSlots) return -1;
    HIPCHK(c, hipSetDevice(c->device));
    Slot &s = c->slot[0];
    s.h_prof.assign(s.nz * ccsx::kProfSlots, 0);
    if (s.nz)
        HIPCHK(c, hipMemcpy(s.h_prof.data(), s.d_prof.p, s.nz * ccsx::kProfSlots * 8, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < nslots; ++i) sums[i] = 0;
    for (size_t zi = 0; zi < s.nz; ++zi)
        for (int i = 0; i < ccsx::kProfSlots; ++i) sums[i] += s.h_prof[zi * ccsx::kProfSlots + i];
    return 0;
}

int ccsx_gpu_profile_zmw(ccsx_ctx *c, uint64_t *out, uint32_t nzmw, uint32_t nslots)
{
    if (!c || !c->profiling || nslots < (uint32_t)ccsx::kProfSlots || nzmw < c->slot[0].nz) return -1;
    HIPCHK(c, hipSetDevice(c->device));
    const Slot &s = c->slot[0];
    if (s.nz) HIPCHK(c, hipMemcpy(out, s.d_prof.p, s.nz * ccsx::kProfSlots * 8, hipMemcpyDeviceToHost));
    return 0;
}

uint64_t ccsx_gpu_staged_bytes(const ccsx_ctx *c)
{
    if (!c) return 0;
    const Slot &s = c->slot[0];
    return s.seq_bytes + s.ws_bytes + s.out_bytes + s.msa_bytes;
}

// single-POA path used by the bspoa-compatible API (bspoa_gpu.cpp)
int ccsx_gpu_single_poa(ccsx_ctx *c, const ccsx_zmw_in *z, const uint8_t **cns, uint32_t *ncns,
                        const uint8_t **msa, uint32_t *ncols)
{
    int r = ccsx_gpu_stage_ex(c, z, 1, 1, 1);
    if (r) return r;
    r = ccsx_gpu_launch_ex(c, ccsx::kSinglePoa, nullptr);
    if (r) return r;
    ccsx_zmw_out o;
    r = ccsx_gpu_fetch(c, &o);
    if (r) return r;
    Slot &s = c->slot[0];
    s.h_ncols.resize(1);
    HIPCHK(c, hipMemcpy(s.h_ncols.data(), s.d_ncols.p, 4, hipMemcpyDeviceToHost));
    const uint64_t mb = uint64_t(s.h_ncols[0]) * (z->nseg + 4);
    s.h_msa.resize(mb + 1);
    if (mb) HIPCHK(c, hipMemcpy(s.h_msa.data(), s.d_msa.p, mb, hipMemcpyDeviceToHost));
    *cns = reinterpret_cast<const uint8_t *>(o.ccs);
    *ncns = o.len;
    *msa = s.h_msa.data();
    *ncols = s.h_ncols[0];
    return 0;
}

}  // extern "C"
