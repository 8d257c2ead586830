// dispatch.cpp -- cost model and micro-batch partitioner of the C host
// program's multi-GPU step 1 (include/ccsx_host.h).
//
// The reference balances ZMWs over its CPU threads dynamically: kt_for deals
// indices round-robin and idle threads steal (kthread.c:24-46).  A GPU launch
// is only efficient with thousands of ZMWs in it, so here the unit a device
// context pulls is a micro-batch: the chunk's ZMWs ranked by estimated cost
// (largest first) and the ranks dealt round-robin over the batches, kt_for's
// dealing applied to cost ranks.  Every batch then holds the same mix of
// expensive and cheap ZMWs (batch costs differ by at most one ZMW's cost), so
// no batch is only a chunk's most expensive ZMWs -- whose launch would end
// on its slowest serial chains -- and each launch, ordered longest first on
// the device, ends on cheap ones.
#include <algorithm>
#include <numeric>
#include <vector>

#include "ccsx_host.h"

extern "C" {

uint64_t ccsx_zmw_cost(const uint32_t *seg_len, uint32_t nseg)
{
    // DP cells of a ZMW ~ sum over windows and reads of graph rows x band;
    // graph rows ~ window x (1 + ~0.035 reads): cost ~ S x (28 + n)
    uint64_t s = 0;
    for (uint32_t k = 0; k < nseg; ++k) s += seg_len[k];
    return s * (28u + nseg);
}

uint32_t ccsx_partition(const uint64_t *cost, uint32_t n, uint32_t nparts, uint32_t min_batch, uint32_t *order,
                        uint32_t *bounds)
{
    if (n == 0) {
        bounds[0] = 0;
        return 0;
    }
    std::vector<uint32_t> rank(n);
    for (uint32_t i = 0; i < n; ++i) rank[i] = i;
    // LPT ranks; equal costs keep input order (deterministic batches)
    std::stable_sort(rank.begin(), rank.end(), [cost](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
    if (nparts < 1) nparts = 1;
    if (min_batch < 1) min_batch = 1;
    // as many batches as asked, none below min_batch ZMWs (one if n is short)
    const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(nparts, n / min_batch));
    // batch b = ranks b, b + nb, b + 2 nb, ...: contiguous in `order`
    uint32_t o = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        bounds[b] = o;
        for (uint32_t r = b; r < n; r += nb) order[o++] = rank[r];
    }
    bounds[nb] = n;
    return nb;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Synthetic prepared batches for benchmarks (bench.py's end-to-end line):
// ccsx_synth_zmw + ccsx_prepare_apply per ZMW on worker threads.
#include <atomic>
#include <memory>
#include <string>
#include <thread>

#include "ccsx_gpu.h"

struct ccsx_synth_batch {
    std::vector<std::string> seqs;
    std::vector<std::vector<uint32_t>> off, len;
    std::vector<ccsx_zmw_in> in;
};

extern "C" {

ccsx_synth_batch *ccsx_synth_batch_make(uint64_t seed, const uint64_t *holes, const uint32_t *L, const uint32_t *passes,
                                        uint32_t n, int nthreads)
{
    auto *b = new ccsx_synth_batch();
    b->seqs.resize(n);
    b->off.resize(n);
    b->len.resize(n);
    b->in.resize(n);
    std::atomic<uint32_t> nx(0);
    auto work = [&]() {
        std::vector<uint32_t> lens;
        for (uint32_t i; (i = nx.fetch_add(1)) < n;) {
            std::string &s = b->seqs[i];
            s.resize((size_t)passes[i] * (2ull * L[i] + 16) + 16);
            lens.resize(passes[i]);
            const uint64_t tot = ccsx_synth_zmw(seed, holes[i], L[i], passes[i], &s[0], lens.data(), nullptr);
            s.resize(tot);
            b->off[i].resize(passes[i]);
            b->len[i].resize(passes[i]);
            const uint32_t ns = ccsx_prepare_apply(&s[0], lens.data(), passes[i], b->off[i].data(), b->len[i].data());
            b->off[i].resize(ns);
            b->len[i].resize(ns);
            b->in[i] = ccsx_zmw_in{s.data(), b->off[i].data(), b->len[i].data(), ns};
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    return b;
}

const ccsx_zmw_in *ccsx_synth_batch_zmws(const ccsx_synth_batch *b) { return b->in.data(); }

void ccsx_synth_batch_free(ccsx_synth_batch *b) { delete b; }

}  // extern "C"
