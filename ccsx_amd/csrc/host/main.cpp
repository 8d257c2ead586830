// main.cpp -- the C host program: ccsx's CLI and 3-stage pipeline on top of the
// MI355X engine.
//
// Restates main.c:723-870 (options, I/O, chunked pipeline) and step 0 / step 2
// of worker_pipeline (main.c:649-720).  Step 1 -- kt_for(ccs_for2/ccs_for),
// which deals the chunk's ZMWs over CPU threads with work stealing
// (kthread.c:24-46) -- becomes:
//   * ccs_prepare + strand flip on -j CPU threads (main.c:520-536);
//   * the chunk's ZMWs cut into cost-balanced micro-batches in
//     longest-first order (host/dispatch.cpp), queued behind the previous
//     chunk's;
//   * one worker thread per device context pulls batches from the queue and
//     runs them through the batched C-ABI (include/ccsx_gpu.h); two contexts
//     per GPU by default (CCSX_SLOTS), whose batches overlap on the device;
//   * a writer thread emits each chunk in input order once its last batch is
//     back (main.c:707-717).
// A ZMW the device cannot finish is reported on stderr and skipped; the other
// ZMWs of the run are written (the reference has no per-ZMW failure).
#include <errno.h>
#include <getopt.h>
#include <malloc.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "ccsx_gpu.h"
#include "ccsx_host.h"
#include "ingest.h"

namespace {

// ZMWs the reader takes into the first chunk before it waits for the device
// contexts to fix the chunk sizes
constexpr size_t kChunkProvisional = 16384;

// Bases of a chunk's ZMWs live in one arena per chunk (an anonymous mapping
// with transparent huge pages), recycled through a pool: per-ZMW strings
// (~130 KB each, ~2 GB per 16,384-ZMW chunk) cost a page fault per 4 KB page
// when written and a page-table teardown when freed -- 0.55 s per chunk at
// the process exit, which the CLI's timed run pays for every chunk still held.
class ArenaPool {
public:
    struct Arena {
        char *p = nullptr;
        size_t cap = 0;
    };
    Arena get(size_t need)
    {
        {
            std::lock_guard<std::mutex> g(m_);
            for (size_t i = 0; i < free_.size(); ++i)
                if (free_[i].cap >= need) {
                    Arena a = free_[i];
                    free_.erase(free_.begin() + (long)i);
                    return a;
                }
        }
        Arena a;
        a.cap = std::max<size_t>((need + need / 8 + (2u << 20) - 1) & ~size_t((2u << 20) - 1), 2u << 20);
        void *p = mmap(nullptr, a.cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) {
            fprintf(stderr, "[ccsx] cannot map %zu bytes for a chunk's bases\n", a.cap);
            std::_Exit(1);
        }
        if (!getenv("CCSX_NO_THP")) (void)madvise(p, a.cap, MADV_HUGEPAGE);
        a.p = static_cast<char *>(p);
        return a;
    }
    // back to the pool; unmapped at once once the input has ended (drain):
    // tearing memory down costs ~50 ms per GB even with huge pages (13 GB of
    // arenas: 0.64 s), which the worker that returns an arena pays while the
    // device still runs the last batches, instead of the process exit
    void put(Arena a)
    {
        if (!a.p) return;
        {
            std::lock_guard<std::mutex> g(m_);
            if (!draining_) {
                free_.push_back(a);
                return;
            }
        }
        munmap(a.p, a.cap);
    }
    void drain()
    {
        std::vector<Arena> v;
        {
            std::lock_guard<std::mutex> g(m_);
            draining_ = true;
            v.swap(free_);
        }
        for (Arena &a : v) munmap(a.p, a.cap);
    }

private:
    std::mutex m_;
    std::vector<Arena> free_;
    bool draining_ = false;
};

struct Zmw {
    ccsx_ingest::ZmwRef ref;  // the subreads as spans of the input blocks (until assembled)
    std::string movie, hole;
    char *seqs = nullptr;     // the bases (in the chunk's arena)
    std::vector<uint32_t> lens;
    std::vector<uint32_t> seg_off, seg_len;
    std::vector<uint8_t> seg_rev;
    std::string ccs;
    int32_t status = 0;
    std::vector<uint32_t> bp;  // -v >= 3: (breakpoint, MSA columns) per shredding round
};

struct Chunk {
    size_t id = 0;
    std::vector<Zmw> zs;
    ArenaPool *pool = nullptr;
    ArenaPool::Arena arena;  // the ZMWs' bases (needed until every batch is staged)
    void release_arena()
    {
        if (pool) pool->put(arena);
        arena = ArenaPool::Arena{};
    }
    ~Chunk() { release_arena(); }
    std::atomic<size_t> pending{0};  // batches not yet back from a device
    double t_read0 = 0, t_read1 = 0;  // CCSX_TIMING: when step 0's reader read it
    bool last_input = false;           // the input ended inside this chunk
    const char *input_hi = nullptr;    // end of the last record read into it (ZmwSource::release)
};

struct Batch {
    std::shared_ptr<Chunk> chunk;
    std::vector<uint32_t> idx;  // ZMWs of the chunk
};

int usage()
{
    fprintf(stdout,
            "Program: ccsx\n"
            "Version: 1.0.0 (MI355X engine)\n"
            "Usage  : ccsx  [options] <INPUT> <OUTPUT>\n"
            "Generate circular consensus sequences (ccs) from subreads.\n"
            "\n"
            "Options:\n"
            "-h             Output this help \n"
            "-v             debug \n"
            "-m     <int>   Minimum total length of subreads in a hole to use for generating CCS. [5000] \n"
            "-M     <int>   Maximum total length of subreads in a hole to use for generating CCS. [500000] \n"
            "-c     <int>   Minimum number of subreads required to generate CCS. [3] \n"
            "-A             For fasta/fastq input,gzip allowed  \n"
            "-P             primitive bsalign,subread shred by default \n"
            "-X\t\t<str>   Exclude ZMWs from output file,a comma-separated list of ID \n"
            "-j     <int>   Number of CPU threads for subread preparation. [1] \n"
            "\n"
            "Environment:\n"
            "CCSX_NGPU      Number of GPU contexts groups [all visible GPUs]; more than the visible\n"
            "               GPUs places group g on GPU g %% visible (logical contexts)\n"
            "CCSX_SLOTS     Device contexts (worker threads) per group [2]\n"
            "CCSX_ASYNC     0: one ccsx_gpu_run per batch instead of pipelined submit / collect [1]\n"
            "CCSX_TIMING    1: per-chunk / per-batch timing on stderr\n"
            "CCSX_CHUNK     Largest chunk in ZMWs [16384 x contexts; 8192 x contexts with CCSX_ASYNC=0]\n"
            "CCSX_CHUNK0    First chunk in ZMWs [CCSX_CHUNK / 2], growing x4 up to CCSX_CHUNK\n"
            "CCSX_KCFG      Force a kernel configuration (0 latency, 1 occupancy, 2 throughput, 3 solo)\n"
            "CCSX_DEV_SHARE Processes sharing each GPU [1] (each context's memory share shrinks)\n"
            "CCSX_MEM_FRAC  Fraction of each GPU's memory its contexts size their slices from [0.85]\n"
            "\n"
            "Arguments:\n"
            "input          Input file.\n"
            "output         Output file.\n"
            "\n");
    return 1;
}

// Per ZMW of the chunk, on nthreads threads: the bases assembled from the
// input blocks (the copy step 0 of the reference makes, main.c:674-685), then
// ccs_prepare + strand flip (the CPU half of step 1, main.c:520-536, with its
// -v output)
void prepare_chunk(Chunk &ch, int nthreads, int verbose)
{
    std::vector<Zmw> &zs = ch.zs;
    // each ZMW's bases at its offset in the chunk's arena
    std::vector<size_t> at(zs.size() + 1, 0);
    for (size_t i = 0; i < zs.size(); ++i) at[i + 1] = at[i] + zs[i].ref.total();
    ch.arena = ch.pool->get(at.back());
    std::atomic<size_t> next(0);
    auto work = [&]() {
        std::string msg;
        for (size_t i; (i = next.fetch_add(1)) < zs.size();) {
            Zmw &z = zs[i];
            z.movie = std::move(z.ref.movie);
            z.hole = std::move(z.ref.hole);
            z.seqs = ch.arena.p + at[i];
            z.lens.resize(z.ref.recs.size());
            size_t o = 0;
            for (size_t k = 0; k < z.ref.recs.size(); ++k) {
                const ccsx_ingest::Rec &r = z.ref.recs[k];
                ccsx_ingest::write_bases(r, &z.seqs[o]);
                z.lens[k] = r.len;
                o += r.len;
            }
            ccsx_ingest::ZmwRef().recs.swap(z.ref.recs);
            std::vector<std::shared_ptr<ccsx_ingest::Block>>().swap(z.ref.keep);
            const uint32_t n = (uint32_t)z.lens.size();
            z.seg_off.resize(n);
            z.seg_len.resize(n);
            z.seg_rev.resize(n);
            const uint32_t ns = ccsx_prepare(z.seqs, z.lens.data(), n, z.seg_off.data(), z.seg_len.data(),
                                             z.seg_rev.data());
            z.seg_off.resize(ns);
            z.seg_len.resize(ns);
            z.seg_rev.resize(ns);
            msg.clear();
            if (verbose > 1) msg += "poa begin " + z.hole + "\n";
            for (uint32_t l = 0; l < ns; ++l) {
                if (z.seg_rev[l]) ccsx_revcomp(&z.seqs[z.seg_off[l]], z.seg_len[l]);
                if (verbose) {
                    // main.c:477-479 / 533-535
                    char h[160];
                    snprintf(h, sizeof h, ">%s_%u/%u strand=%d len=%u \n", z.hole.c_str(), l, ns, z.seg_rev[l],
                             z.seg_len[l]);
                    msg += h;
                    msg.append(z.seqs + z.seg_off[l], z.seg_len[l]);
                    msg += '\n';
                }
            }
            if (!msg.empty()) fwrite(msg.data(), 1, msg.size(), stderr);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
}

// the batch queue between step 0 and the device workers
class BatchQueue {
public:
    void push(std::vector<Batch> &&bs)
    {
        {
            std::lock_guard<std::mutex> g(m_);
            for (auto &b : bs) q_.push_back(std::move(b));
        }
        cv_.notify_all();
    }
    void close()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            closed_ = true;
        }
        cv_.notify_all();
    }
    bool pop(Batch &b)
    {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return closed_ || !q_.empty(); });
        if (q_.empty()) return false;
        b = std::move(q_.front());
        q_.pop_front();
        return true;
    }
    // without waiting: false if no batch is queued right now
    bool try_pop(Batch &b)
    {
        std::lock_guard<std::mutex> g(m_);
        if (q_.empty()) return false;
        b = std::move(q_.front());
        q_.pop_front();
        return true;
    }

private:
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<Batch> q_;
    bool closed_ = false;
};

// chunks of ZMW references from step 0's reader to the preparing thread,
// bounded (reading chunk k + 1 overlaps preparing chunk k); an empty chunk
// ends the input
class ReadQueue {
public:
    explicit ReadQueue(size_t limit) : limit_(limit) {}
    void push(std::shared_ptr<Chunk> c)
    {
        std::unique_lock<std::mutex> g(m_);
        space_.wait(g, [this] { return q_.size() < limit_ || stop_; });
        q_.push_back(std::move(c));
        ready_.notify_all();
    }
    std::shared_ptr<Chunk> pop()
    {
        std::unique_lock<std::mutex> g(m_);
        ready_.wait(g, [this] { return !q_.empty(); });
        auto c = std::move(q_.front());
        q_.pop_front();
        space_.notify_all();
        return c;
    }
    void stop()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        space_.notify_all();
    }

private:
    std::mutex m_;
    std::condition_variable space_, ready_;
    std::deque<std::shared_ptr<Chunk>> q_;
    size_t limit_;
    bool stop_ = false;
};

// chunks in input order, handed from step 0 to the writer; bounded so step 0
// runs at most `limit` chunks ahead of the output
class ChunkRing {
public:
    explicit ChunkRing(size_t limit) : limit_(limit) {}
    void add(const std::shared_ptr<Chunk> &c)
    {
        std::unique_lock<std::mutex> g(m_);
        space_.wait(g, [this] { return q_.size() < limit_ || stop_; });
        q_.push_back(c);
        ready_.notify_all();
    }
    void finish()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            eof_ = true;
        }
        ready_.notify_all();
    }
    void stop()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        space_.notify_all();
        ready_.notify_all();
    }
    void batch_done()
    {
        // the decrement happened outside the lock: take it once so a writer
        // between its predicate check and its wait cannot miss this wake-up
        { std::lock_guard<std::mutex> g(m_); }
        ready_.notify_all();
    }
    // the oldest chunk once every batch of it is back; null at the end
    std::shared_ptr<Chunk> next_done()
    {
        std::unique_lock<std::mutex> g(m_);
        ready_.wait(g, [this] { return stop_ || (!q_.empty() && q_.front()->pending == 0) || (q_.empty() && eof_); });
        if (stop_ || q_.empty()) return nullptr;
        auto c = q_.front();
        return c;
    }
    void pop()
    {
        std::lock_guard<std::mutex> g(m_);
        q_.pop_front();
        space_.notify_all();
    }

private:
    std::mutex m_;
    std::condition_variable space_, ready_;
    std::deque<std::shared_ptr<Chunk>> q_;
    size_t limit_;
    bool eof_ = false, stop_ = false;
};

// -X (main.c:772-782): each option kputs-appends its argument to one buffer,
// then ksplit(',') splits the buffer *as a C string* in place (kstring.c:
// 65-107: a field's end delimiter becomes NUL, empty fields are skipped) and
// a fresh hole set holds the fields.  So only the last -X's set counts, and
// after a first split the buffer's C string ends at the first field: `-X 3,5
// -X 7` excludes hole 3, `-X 3 -X 7` excludes hole 37.
std::unordered_set<std::string> exclude_holes(std::string &buf, const char *arg)
{
    buf.append(arg);
    const size_t l = strnlen(buf.data(), buf.size());
    std::unordered_set<std::string> set;
    std::vector<size_t> starts;
    char last = 0;
    size_t start = 0;
    for (size_t i = 0; i <= l; ++i) {
        const char ch = i < l ? buf[i] : '\0';
        if (ch == ',' || ch == '\0') {
            if (last != 0 && last != ',') {
                if (i < l) buf[i] = '\0';
                starts.push_back(start);
                last = '\0';
                continue;
            }
        } else if (last == ',' || last == 0) {
            start = i;
        }
        last = ch;
    }
    for (size_t st : starts) set.insert(std::string(buf.c_str() + st));
    return set;
}

}  // namespace

// CCSX_CHUNK / CCSX_CHUNK0 (measurement overrides) over the default last
// chunk size cm_def (0: not known yet -- the device count decides it): the
// last and first chunk sizes, computed the same way before and after the
// devices open, the first never above the last.  Unknown sizes
// come back 0.
static void env_chunk_sizes(size_t cm_def, size_t &cm, size_t &c0)
{
    size_t ecm = 0, ec0 = 0;
    if (const char *e = getenv("CCSX_CHUNK")) ecm = std::max<size_t>(1024, strtoull(e, nullptr, 10));
    if (const char *e = getenv("CCSX_CHUNK0")) ec0 = std::min<size_t>(131072, std::max<size_t>(1, strtoull(e, nullptr, 10)));
    cm = ecm ? ecm : cm_def;
    if (ec0) {
        c0 = ecm ? std::min(ec0, ecm) : ec0;
        if (cm) cm = std::max(cm, c0);
    } else {
        c0 = cm ? std::max<size_t>(1024, cm / 2) : 0;
    }
}

int main(int argc, char **argv)
{
    const auto tmain = std::chrono::steady_clock::now();
    // per-ZMW strings (~130 KB of subreads each, a few GB per chunk) from the
    // heap, not one mmap each: freed memory is reused by the next chunk with
    // no munmap / page-fault churn, and nothing is returned to the kernel
    // mid-run (freeing a 16,384-ZMW chunk of mmap'd strings took 0.7 s, and
    // the process exit paid the same for the chunks still held)
    if (!getenv("CCSX_MALLOC_DEFAULT")) {
        mallopt(M_MMAP_THRESHOLD, 32 << 20);
        mallopt(M_TRIM_THRESHOLD, 1 << 30);
    }
    int c, verbose = 0, min_subread_len = 5000, max_subread_len = 500000, min_fulllen_count = 3, nthreads = 1;
    int isbam = 1, split_subread = 1;
    std::unordered_set<std::string> hole_set;
    std::string xbuf;  // -X: kputs-appended, ksplit in place (exclude_holes)
    bool have_holes = false;
    while ((c = getopt(argc, argv, "hm:M:c:j:X:PAv")) != -1) {
        switch (c) {
        case 'm': min_subread_len = atoi(optarg); break;
        case 'M': max_subread_len = atoi(optarg); break;
        case 'P': split_subread = 0; break;
        case 'A': isbam = 0; break;
        case 'X':  // main.c:772-782
            have_holes = true;
            hole_set = exclude_holes(xbuf, optarg);
            break;
        case 'c':
            min_fulllen_count = atoi(optarg);
            if (min_fulllen_count < 3) {
                fprintf(stderr, "Error! min fulllen count=[%d] (>=3) !\n", min_fulllen_count);
                return -1;
            }
            break;
        case 'v': verbose++; break;
        case 'j': nthreads = atoi(optarg); break;
        default: return usage();
        }
    }
    // main.c:802-826
    const char *in_path = "-";
    FILE *fp_out = nullptr;
    if (argc - optind == 0) {
        fp_out = stdout;
    } else if (argc - optind == 1) {
        in_path = argv[optind];
        fp_out = stdout;
    } else if (argc - optind == 2) {
        in_path = argv[optind];
        fp_out = strcmp(argv[optind + 1], "-") == 0 ? stdout : fopen(argv[optind + 1], "w+");
    } else {
        return usage();
    }
    if (nthreads < 1) nthreads = 1;
    // step 0's input: blocks decompressed ahead on a producer thread (BGZF
    // members inflated on the -j threads), records parsed as spans
    auto rd = ccsx_ingest::ZmwSource::open(in_path, isbam != 0, nthreads);
    if (!rd) {
        fprintf(stderr, "Error: Failed to open infile!\n");
        return 1;
    }
    if (!fp_out) {
        fprintf(stderr, "Cannot open file for write!\n");
        return 1;
    }
    // step 1 pipelined per context (ccsx_gpu_submit / ccsx_gpu_collect: the
    // next batch is launched before the previous one is collected);
    // CCSX_ASYNC=0: one ccsx_gpu_run per batch (also for the -v >= 3
    // breakpoint log, which ccsx_gpu_run gathers)
    const bool async = !(getenv("CCSX_ASYNC") && atoi(getenv("CCSX_ASYNC")) == 0) && !(verbose > 2 && split_subread);
    // CCSX_NGPU groups of CCSX_SLOTS contexts; group g on device g % ndev
    // (more groups than devices: logical contexts sharing a device, which is
    // how the multi-GPU split is exercised on a one-GPU box).  Two contexts
    // per GPU: each pulls micro-batches on its own worker thread, so one
    // batch's staging and tail overlap the other's kernels (100k config-E
    // ZMWs: 10.66 s vs 12.12 s with one, profiles/r03); pipelined, each keeps
    // two launches in flight (200k config-E ZMWs: 9.4-9.7 s with two
    // contexts, 10.7 s with one, 9.9-10.0 s for two contexts of ccsx_gpu_run;
    // gpurun_out r04r/r04s)
    int nslot = 2;
    if (const char *e = getenv("CCSX_SLOTS")) nslot = std::max(1, std::min(8, atoi(e)));
    // processes sharing each device (bench.py's multi-rank rehearsal on one
    // GPU): each context's memory share shrinks by that factor
    int dev_share = 1;
    if (const char *e = getenv("CCSX_DEV_SHARE")) dev_share = std::max(1, std::min(64, atoi(e)));
    // measurement overrides of the engine (never set by default)
    const int kcfg = getenv("CCSX_KCFG") ? atoi(getenv("CCSX_KCFG")) : -1;
    const int wg_cap = getenv("CCSX_WG_PER_CU") ? atoi(getenv("CCSX_WG_PER_CU")) : 0;
    const int read_cap = getenv("CCSX_SHRED_READ_CAP") ? atoi(getenv("CCSX_SHRED_READ_CAP")) : 0;
    // the contexts size their slices from 85 % of the device memory (the
    // library's default is half): a context's 8,192-ZMW batch of a config-E
    // chunk then runs as one launch instead of two of 4,096, whose
    // longest-first order balances better (200k config-E ZMWs 11.0 s -> 10.0 s,
    // gpurun_out r04q); CCSX_MEM_FRAC overrides
    const float mem_frac = getenv("CCSX_MEM_FRAC") ? (float)atof(getenv("CCSX_MEM_FRAC")) : 0.85f;
    // micro-batches per context and chunk (CCSX_CTX_BATCHES, default 1: 100k
    // config-E ZMWs from the generator's pipe 15.2 s with 2, 11.8 s with 1,
    // r03o)
    uint32_t batches_per_ctx = 1;
    if (const char *e = getenv("CCSX_CTX_BATCHES")) batches_per_ctx = (uint32_t)std::max(1, std::min(64, atoi(e)));
    // consumed input pages unmapped as chunks are prepared (CCSX_INPUT_RELEASE=0: at the exit)
    const bool input_release = !(getenv("CCSX_INPUT_RELEASE") && atoi(getenv("CCSX_INPUT_RELEASE")) == 0);
    // a context with no more work releases its memory while the others run
    // (CCSX_EARLY_CLOSE=0: the exit releases everything)
    const bool early_close = !(getenv("CCSX_EARLY_CLOSE") && atoi(getenv("CCSX_EARLY_CLOSE")) == 0);
    // the last context too, while the writer emits the last chunks: the exit
    // then has less to release (62,500 config-E ZMWs at -j 8: 317-321 ms from
    // the last batch to the exit against 345-369, r06j; CCSX_LAST_CLOSE=0: off)
    const bool last_close = !(getenv("CCSX_LAST_CLOSE") && atoi(getenv("CCSX_LAST_CLOSE")) == 0);
    // the chunk the input ends in: batches per context (the run ends on its
    // slowest batch; smaller ones let the contexts end together)
    uint32_t last_batches_per_ctx = 1;
    if (const char *e = getenv("CCSX_LAST_BATCHES")) last_batches_per_ctx = (uint32_t)std::max(1, std::min(64, atoi(e)));
    const bool timing = getenv("CCSX_TIMING") && atoi(getenv("CCSX_TIMING"));
    const auto tstart = std::chrono::steady_clock::now();
    auto now_ms = [tstart]() {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tstart).count();
    };
    const int mode = split_subread ? CCSX_MODE_SHRED : CCSX_MODE_PRIMITIVE;
    // the device contexts, opened on their own thread (below) while step 0
    // reads and prepares the first chunk
    int nctx = 0;
    std::vector<ccsx_ctx *> ctx;
    uint64_t slot_bytes = 0;

    ArenaPool arenas;  // (declared before every holder of a chunk)
    BatchQueue queue;
    ChunkRing ring(3);
    std::atomic<bool> fatal(false);
    std::atomic<uint64_t> cells_total(0);  // DP cells the devices computed (CCSX_TIMING report)
    std::atomic<int> workers_busy(0);      // pipelined workers still running
    std::mutex err_m;

    // test hook: the device reports this hole as failed (tests/test_gpu_cli.py)
    const std::string fault_hole = getenv("CCSX_FAULT_HOLE") ? getenv("CCSX_FAULT_HOLE") : "";
    // test hook: batches after the first CCSX_FATAL_AFTER ones fail as a
    // context error does (the fatal path's teardown, tests/test_gpu_cli.py)
    const long fatal_after = getenv("CCSX_FATAL_AFTER") ? atol(getenv("CCSX_FATAL_AFTER")) : -1;
    std::atomic<long> batches_seen(0);

    // step 1, device side: one worker per context
    // a batch in flight on a context: its input arrays live until collected
    struct Flight {
        Batch b;
        std::vector<ccsx_zmw_in> in;
        std::vector<ccsx_zmw_out> out;
        int slot = -1;
        double t0 = 0;
    };
    auto prepare_in = [&](int w, Flight &f) {
        Chunk &ch = *f.b.chunk;
        f.in.resize(f.b.idx.size());
        f.out.assign(f.b.idx.size(), ccsx_zmw_out{});
        for (size_t i = 0; i < f.b.idx.size(); ++i) {
            const Zmw &z = ch.zs[f.b.idx[i]];
            f.in[i] = ccsx_zmw_in{z.seqs, z.seg_off.data(), z.seg_len.data(), (uint32_t)z.seg_len.size()};
            if (!fault_hole.empty() && z.hole == fault_hole) ccsx_gpu_set_fault(ctx[w], (int64_t)i);
        }
        f.t0 = now_ms();
    };
    // results of a batch (r: the run / collect status) into its chunk
    auto finish = [&](int w, Flight &f, int r) {
        Chunk &ch = *f.b.chunk;
        if (fatal_after >= 0 && batches_seen.fetch_add(1) >= fatal_after) r = -9;
        if (r == 0 || r == -2) {
            // -2: some ZMWs failed on the device, the rest are valid
            uint64_t cells = 0;
            for (size_t i = 0; i < f.b.idx.size(); ++i) cells += f.out[i].cells;
            cells_total += cells;
            for (size_t i = 0; i < f.b.idx.size(); ++i) {
                Zmw &z = ch.zs[f.b.idx[i]];
                z.status = f.out[i].status;
                if (!f.out[i].status) z.ccs.assign(f.out[i].ccs, f.out[i].len);
                const uint32_t *lg;
                uint32_t nr = 0;
                if (verbose > 2 && !f.out[i].status && ccsx_gpu_bp_log(ctx[w], i, &lg, &nr) == 0)
                    z.bp.assign(lg, lg + 2 * (size_t)nr);
            }
        } else if (!fatal.exchange(true)) {
            std::lock_guard<std::mutex> g(err_m);
            fprintf(stderr, "[ccsx] device context %d: %s\n", w, r == -9 ? "injected fatal error (test hook)" : ccsx_gpu_error(ctx[w]));
        }
        if (timing)
            fprintf(stderr, "[ccsx] chunk %zu batch of %zu ZMWs on context %d: %.0f-%.0f ms\n", ch.id, f.b.idx.size(),
                    w, f.t0, now_ms());
        const bool chunk_done = f.b.chunk->pending.fetch_sub(1) == 1;
        ring.batch_done();
        // the bases were staged: the arena goes back before the chunk is
        // written (the writer needs only names and CCS)
        if (chunk_done) f.b.chunk->release_arena();
        f.b.chunk.reset();
    };
    // workers whose batches are all finished (the output and the exit wait
    // for this, not for a worker's teardown of its context)
    std::mutex done_m;
    std::condition_variable done_cv;
    int nwork_done = 0;
    auto work_done = [&](int) {
        std::lock_guard<std::mutex> g(done_m);
        ++nwork_done;
        done_cv.notify_all();
    };
    auto worker = [&](int w) {
        if (!async) {
            Flight f;
            while (queue.pop(f.b)) {
                if (fatal) {
                    finish(w, f, -1);
                    continue;
                }
                prepare_in(w, f);
                finish(w, f, ccsx_gpu_run(ctx[w], mode, f.in.data(), f.in.size(), f.out.data()));
            }
            workers_busy.fetch_sub(1);
            work_done(w);
            return;
        }
        // pipelined: up to two batches in flight, the next one submitted
        // before the oldest is collected (include/ccsx_gpu.h).  First the
        // pinned staging of the first slot, sized for a batch (a config-E
        // batch's subreads are ~1/60 of a slot, its tight CCS slabs ~1/3 of
        // that), while step 0 still reads the first chunk
        if (slot_bytes) (void)ccsx_gpu_reserve_staging(ctx[w], slot_bytes / 56, slot_bytes / 160);
        std::deque<Flight> fl;
        for (;;) {
            Flight f;
            const bool got = fl.size() < 2 && (fl.empty() ? queue.pop(f.b) : queue.try_pop(f.b));
            if (got) {
                if (fatal) {
                    finish(w, f, -1);
                    continue;
                }
                prepare_in(w, f);
                const int r = ccsx_gpu_submit(ctx[w], mode, f.in.data(), f.in.size(), &f.slot);
                if (r == -4) {
                    // larger than a slot: collect what is in flight, then
                    // the batch through ccsx_gpu_run's slices
                    while (!fl.empty()) {
                        Flight &g = fl.front();
                        finish(w, g, ccsx_gpu_collect(ctx[w], g.slot, g.out.data()));
                        fl.pop_front();
                    }
                    finish(w, f, ccsx_gpu_run(ctx[w], mode, f.in.data(), f.in.size(), f.out.data()));
                } else if (r != 0) {
                    finish(w, f, r);
                } else {
                    fl.push_back(std::move(f));
                }
                continue;
            }
            if (fl.empty()) break;  // the queue is closed and empty
            Flight &g = fl.front();
            finish(w, g, ccsx_gpu_collect(ctx[w], g.slot, g.out.data()));
            fl.pop_front();
        }
        // a context with no more work releases its pinned staging and device
        // memory while the others run their last batches (≈ 0.2 s each that
        // the process exit would otherwise pay); the last one is left to it.
        // The output waits for the work, not for the release (work_done)
        const bool last = workers_busy.fetch_sub(1) == 1;
        work_done(w);
        if (!fatal && (!last || last_close) && early_close) {
            ccsx_gpu_close(ctx[w]);
            ctx[w] = nullptr;
        }
    };
    std::vector<std::thread> workers;

    // step 0 (main.c:652-697) on its own thread, one chunk ahead of the
    // preparation (the reference's step 0 does both in turn), started before
    // the devices open: HIP's initialisation (~0.1 s) overlaps the first
    // chunk's read.  The reference grows the chunk 1,024 -> 4,096 -> 16,384
    // ZMWs (main.c:686-690); here the sizes scale with the device contexts
    // (known once the devices are counted: until then the first chunk keeps
    // growing; the sizes change only how the work is cut, never the output)
    std::atomic<size_t> chunk_first(SIZE_MAX), chunk_last(SIZE_MAX);
    {
        // the sizes the environment fixes hold from the first record on (the
        // defaults depend on the device count, known once the devices open)
        size_t cm = 0, c0 = 0;
        env_chunk_sizes(0, cm, c0);
        if (cm) chunk_last = cm;
        if (c0) chunk_first = c0;
    }
    ReadQueue rq(1);
    std::thread reader([&]() {
        size_t chunk_size = 0;
        for (size_t id = 0;; ++id) {
            auto ch = std::make_shared<Chunk>();
            ch->id = id;
            ch->pool = &arenas;
            std::vector<Zmw> &zs = ch->zs;
            ch->t_read0 = now_ms();
            ccsx_ingest::ZmwRef zr;
            int l = 0;
            while (!fatal && (l = rd->next(zr)) >= 0) {
                for (const auto &rc : zr.recs) ch->input_hi = std::max(ch->input_hi, rc.seq + rc.span);
                if (l < min_fulllen_count + 2) continue;
                const uint64_t total = zr.total();
                if (total > (uint64_t)max_subread_len || total < (uint64_t)min_subread_len) continue;
                if (have_holes && hole_set.count(zr.hole)) continue;
                zs.emplace_back();
                zs.back().ref = std::move(zr);
                size_t lim = chunk_size ? chunk_size : chunk_first.load();
                if (lim == SIZE_MAX && zs.size() >= kChunkProvisional) {
                    // the devices are still opening: wait for the chunk sizes
                    // rather than grow the first chunk without bound (a slow
                    // HIP init or 16 contexts would put a page-cached input
                    // into one chunk and one arena, with no pipelining)
                    while ((lim = chunk_first.load()) == SIZE_MAX && !fatal)
                        std::this_thread::sleep_for(std::chrono::microseconds(200));
                }
                if (zs.size() >= lim) {
                    chunk_size = std::min(zs.size() * 4, chunk_last.load());
                    break;
                }
            }
            ch->t_read1 = now_ms();
            ch->last_input = l < 0;
            // kt_pipeline stops on an empty chunk (main.c:694-697); a chunk
            // cut short by -1 (end of input or an invalid name) is processed
            // and the next read goes on, as the reference's next step 0 does
            const bool last = zs.empty();
            rq.push(std::move(ch));
            if (last) {
                arenas.drain();
                break;
            }
        }
    });
    // the devices: contexts opened, their workers started (each reserves its
    // first pinned staging at once); a failure ends the process here, before
    // any output
    std::thread opener([&]() {
        auto die = [&](const char *what) {
            fprintf(stderr, "[ccsx] %s\n", what);
            fflush(stderr);
            std::_Exit(1);
        };
        const int ndev = ccsx_gpu_device_count();
        if (ndev <= 0) die("no HIP device: the MI355X engine needs a GPU");
        int ngroup = ndev;
        if (const char *e = getenv("CCSX_NGPU")) ngroup = std::max(1, std::min(64, atoi(e)));
        const int n = ngroup * nslot;
        // the last chunk size: 16,384 ZMWs per pipelined context (one launch
        // per chunk and context), 8,192 per ccsx_gpu_run context (two slices
        // of ~4,096, above the solo configuration's threshold, also with 8
        // GPUs x 2 contexts); the first half of it (the reference starts at
        // 1,024 ZMWs, main.c:686-690, which here only fed small launches on
        // the latency / occupancy objects while the device idled: 62,500
        // config-E ZMWs 6.3 s with 1,024, 5.4 s with 8,192, 5.8 s with 16,384,
        // r04e); CCSX_CHUNK / CCSX_CHUNK0 override
        size_t cmax = 0, c0 = 0;
        env_chunk_sizes(std::min<size_t>((async ? 16384u : 8192u) * (size_t)n, 131072u), cmax, c0);
        chunk_last = cmax;
        chunk_first = c0;  // (the same first size the reader may already be filling to)
        ctx.assign(n, nullptr);
        std::vector<int> per_dev(ndev, 0);
        for (int i = 0; i < n; ++i) per_dev[(i / nslot) % ndev]++;
        for (int i = 0; i < n; ++i) {
            const int dev = (i / nslot) % ndev;
            if (ccsx_gpu_open(dev, &ctx[i]) != 0) die("cannot open a device context");
            ccsx_gpu_set_mem_share(ctx[i], (uint32_t)(per_dev[dev] * dev_share));
            ccsx_gpu_set_prealloc(ctx[i], 1);
            if (verbose > 2 && split_subread) ccsx_gpu_set_bp_log(ctx[i], 1);
            if ((kcfg >= 0 && ccsx_gpu_set_kernel_cfg(ctx[i], kcfg) != 0) ||
                (wg_cap > 0 && ccsx_gpu_set_wg_cap(ctx[i], (uint32_t)wg_cap) != 0) ||
                (read_cap > 0 && ccsx_gpu_set_shred_read_cap(ctx[i], (uint32_t)read_cap) != 0) ||
                (mem_frac > 0.f && ccsx_gpu_set_mem_frac(ctx[i], mem_frac) != 0))
                die("invalid CCSX_KCFG / CCSX_WG_PER_CU / CCSX_SHRED_READ_CAP / CCSX_MEM_FRAC");
        }
        // pipelined: batches of at most ~95 % of a slot (ccsx_gpu_slot_bytes),
        // so a submitted batch always fits one launch
        if (async && ccsx_gpu_slot_bytes(ctx[0], &slot_bytes) != 0) die(ccsx_gpu_error(ctx[0]));
        if (timing)
            fprintf(stderr, "[ccsx] %d device context(s) open at %.0f ms (main at epoch %.3f s, %.0f ms before)\n", n,
                    now_ms(),
                    std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count() -
                        std::chrono::duration<double>(std::chrono::steady_clock::now() - tmain).count(),
                    std::chrono::duration<double, std::milli>(tstart - tmain).count());
        nctx = n;
        workers_busy = n;
        for (int w = 0; w < n; ++w) workers.emplace_back(worker, w);
    });
    bool opened = false;
    auto await_open = [&]() {
        if (!opened) opener.join();
        opened = true;
    };

    // step 2: ordered output (main.c:707-717)
    size_t nfail = 0;
    // the last chunk written stays referenced here and the ones before it are
    // freed on a thread of their own: freeing a chunk (its per-ZMW vectors and
    // strings, the input blocks it holds) takes up to a few hundred ms, which
    // would delay the next chunk's records and, at the end, the exit
    std::shared_ptr<Chunk> last_written;
    ReadQueue reap(1 << 20);
    std::thread reaper([&]() {
        while (auto ch = reap.pop()) ch.reset();
    });
    std::thread writer([&]() {
        while (auto ch = ring.next_done()) {
            if (!fatal && verbose > 2) {
                // main.c:619-620, printed by ccs_for2 during step 1 (so before
                // the chunk's records), to stdout
                for (auto &z : ch->zs)
                    for (size_t r = 0; r + 1 < z.bp.size(); r += 2)
                        fprintf(stdout, "breakpoint=%u maplen=%u nseq=%zu hole=%s\n", z.bp[r], z.bp[r + 1],
                                z.seg_len.size(), z.hole.c_str());
            }
            if (!fatal) {
                for (auto &z : ch->zs) {
                    if (z.status) {
                        ++nfail;
                        fprintf(stderr, "[ccsx] %s/%s: no CCS, the device could not finish this ZMW (%s)\n",
                                z.movie.c_str(), z.hole.c_str(), ccsx_gpu_status_str(z.status));
                        continue;
                    }
                    if (verbose > 1) fprintf(stderr, "poa end %s\n", z.hole.c_str());
                    if (!z.ccs.empty())
                        fprintf(fp_out, ">%s/%s/ccs\n%s\n", z.movie.c_str(), z.hole.c_str(), z.ccs.c_str());
                }
            }
            if (timing) fprintf(stderr, "[ccsx] chunk %zu written at %.0f ms\n", ch->id, now_ms());
            if (last_written) reap.push(std::move(last_written));
            last_written = ch;
            ring.pop();
        }
    });

    // the CPU half of step 1: each chunk prepared, cost-ordered and cut into
    // micro-batches for the workers
    for (;;) {
        auto ch = rq.pop();
        if (ch->zs.empty() || fatal) break;
        std::vector<Zmw> &zs = ch->zs;
        const size_t id = ch->id;
        const double t0 = ch->t_read0, t1 = ch->t_read1;
        prepare_chunk(*ch, nthreads, verbose);
        // the chunk's bases are in its arena: its input pages go (a mapped
        // file is unmapped behind the reader instead of all at the exit)
        if (input_release) rd->release(ch->input_hi);
        await_open();
        // cost-balanced micro-batches: cost ranks dealt round-robin, each
        // batch longest first (dispatch.cpp)
        const uint32_t n = (uint32_t)zs.size();
        std::vector<uint64_t> cost(n);
        for (uint32_t i = 0; i < n; ++i) cost[i] = ccsx_zmw_cost(zs[i].seg_len.data(), (uint32_t)zs[i].seg_len.size());
        std::vector<uint32_t> order(n), bounds(n + 1);
        uint32_t nparts = (uint32_t)nctx * (ch->last_input ? std::max(batches_per_ctx, last_batches_per_ctx) : batches_per_ctx);
        if (async) {
            uint64_t bytes = 0;
            for (uint32_t i = 0; i < n; ++i) {
                const ccsx_zmw_in zi{zs[i].seqs, zs[i].seg_off.data(), zs[i].seg_len.data(), (uint32_t)zs[i].seg_len.size()};
                bytes += ccsx_gpu_zmw_bytes(ctx[0], mode, &zi);
            }
            const uint64_t per = slot_bytes / 20 * 19;
            nparts = std::max<uint32_t>(nparts, (uint32_t)((bytes + per - 1) / std::max<uint64_t>(per, 1)));
        }
        const uint32_t nb = ccsx_partition(cost.data(), n, nparts, 256u, order.data(), bounds.data());
        std::vector<Batch> bs(nb);
        for (uint32_t b = 0; b < nb; ++b) {
            bs[b].chunk = ch;
            bs[b].idx.assign(order.begin() + bounds[b], order.begin() + bounds[b + 1]);
        }
        ch->pending = nb;
        if (timing)
            fprintf(stderr, "[ccsx] chunk %zu: %u ZMWs read %.0f-%.0f ms, prepared until %.0f ms, %u batches\n", id, n,
                    t0, t1, now_ms(), nb);
        ring.add(ch);  // blocks while 3 chunks are ahead of the writer
        queue.push(std::move(bs));
    }
    // at the end of the input the reader has pushed its empty chunk and
    // returned; after a fatal device error it stops at its next record and
    // pushes without waiting for space
    await_open();
    rq.stop();
    reader.join();
    ring.finish();
    queue.close();
    {
        std::unique_lock<std::mutex> g(done_m);
        done_cv.wait(g, [&] { return nwork_done == nctx; });
    }
    if (fatal) ring.stop();
    writer.join();
    const double tw = now_ms();
    if (!fatal) {
        // (a worker may still be releasing its context: the exit ends it)
        // every byte is written: flush and leave without tearing down the
        // device contexts (≈ 0.8 s of hipFree / hipHostFree for a 100k run)
        // or the last chunk; process exit releases both
        // a failed final write (ENOSPC, EPIPE on a FIFO) must not exit 0
        bool werr = fp_out != stdout && (ferror(fp_out) || fclose(fp_out) != 0);
        werr = (ferror(stdout) || fflush(stdout) != 0) || werr;  // (-v >= 3 breakpoint lines go to stdout)
        if (werr) fprintf(stderr, "[ccsx] error writing the output: %s\n", strerror(errno));
        if (getenv("CCSX_EXIT_CLOSE")) {  // measurement: the teardown steps the exit skips, timed
            const double a = now_ms();
            for (auto &t : workers) t.join();
            for (auto *x : ctx) ccsx_gpu_close(x);
            const double b = now_ms();
            rd.reset();
            const double d = now_ms();
            reap.push(nullptr);
            reaper.join();
            last_written.reset();
            std::string mem;
            if (FILE *f = fopen("/proc/self/smaps_rollup", "r")) {
                char ln[256];
                while (fgets(ln, sizeof ln, f))
                    if (!strncmp(ln, "AnonHugePages", 13) || !strncmp(ln, "Rss", 3) || !strncmp(ln, "Anonymous", 9))
                        mem += std::string(ln, strcspn(ln, "\n")) + "; ";
                fclose(f);
            }
            fprintf(stderr, "[ccsx] teardown: contexts %.0f ms, input %.0f ms, last chunk %.0f ms (then %s)\n", b - a,
                    d - b, now_ms() - d, mem.c_str());
        }
        if (timing)
            fprintf(stderr, "[ccsx] output done at %.0f ms; device cells %llu; exit at epoch %.3f s\n", tw,
                    (unsigned long long)cells_total.load(),
                    std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count());
        if (nfail) fprintf(stderr, "[ccsx] %zu ZMWs had no CCS (device status, see above)\n", nfail);
        fflush(stderr);
        std::_Exit(werr ? 1 : 0);
    }
    for (auto &t : workers) t.join();
    for (auto *x : ctx) ccsx_gpu_close(x);
    reap.push(nullptr);
    reaper.join();
    if (timing) fprintf(stderr, "[ccsx] output done at %.0f ms, contexts closed at %.0f ms\n", tw, now_ms());
    rd.reset();
    if (fp_out != stdout) (void)fclose(fp_out);
    else (void)fflush(stdout);
    if (nfail) fprintf(stderr, "[ccsx] %zu ZMWs had no CCS (device status, see above)\n", nfail);
    return fatal ? 1 : 0;
}
