// dispatch.cpp -- cost model and micro-batch partitioner of the C host
// program's multi-GPU step 1 (include/ccsx_host.h).
//
// The reference balances ZMWs over its CPU threads dynamically: kt_for deals
// indices round-robin and idle threads steal (kthread.c:24-46).  A GPU launch
// is only efficient with ~1,000+ ZMWs in it, so here the unit a device context
// pulls is a micro-batch: the chunk's ZMWs in longest-processing-time order
// (largest estimated cost first), cut into consecutive runs of about equal
// cost.  Contexts pull batches in that order, so the expensive ZMWs start
// first and a chunk ends on batches of small ones.
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
    for (uint32_t i = 0; i < n; ++i) order[i] = i;
    // LPT order; equal costs keep input order (deterministic batches)
    std::stable_sort(order, order + n, [cost](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
    if (nparts < 1) nparts = 1;
    if (min_batch < 1) min_batch = 1;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += cost[i];
    const uint64_t target = (total + nparts - 1) / nparts;
    uint32_t nb = 0, start = 0;
    uint64_t acc = 0;
    bounds[nb++] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        acc += cost[order[i]];
        const uint32_t cnt = i + 1 - start, rest = n - (i + 1);
        // cut once the batch holds its share, but never leave a batch (this
        // one or the remainder) below min_batch ZMWs
        if (rest > 0 && acc >= target && cnt >= min_batch && rest >= min_batch) {
            bounds[nb++] = i + 1;
            start = i + 1;
            acc = 0;
        }
    }
    bounds[nb] = n;
    return nb;
}

}  // extern "C"
