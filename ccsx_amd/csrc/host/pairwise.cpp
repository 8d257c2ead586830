// pairwise.cpp -- strand_match's pairwise aligner and the synthetic ZMW source.
//
// ccsx_pairwise stands in for bsalign's kmer_striped_seqedit_pairwise(13, ...)
// (called at main.c:264), which is un-vendored.  SPEC.md §8 defines it: k=13
// exact-seed diagonal vote, then a banded local alignment (match +1,
// mismatch -2, gap -2) around the winning diagonal.  It only decides strand
// and trimming of abnormal-length subreads on the host; it is not on the GPU
// hot path.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "ccsx_host.h"

namespace {

constexpr int kK = 13;
constexpr int kBin = 32;
constexpr int kHalfBand = 256;

inline uint64_t splitmix64(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

extern "C" {

ccsx_pairaln ccsx_pairwise(const uint8_t *q, uint32_t qlen, const uint8_t *t, uint32_t tlen)
{
    ccsx_pairaln r;
    memset(&r, 0, sizeof r);
    if (qlen < (uint32_t)kK || tlen < (uint32_t)kK) return r;
    // 1. k-mer diagonal vote (diagonal d = tpos - qpos, binned by kBin)
    const uint32_t mask = (1u << (2 * kK)) - 1;
    std::unordered_map<uint32_t, std::vector<uint32_t>> idx;
    idx.reserve(tlen);
    uint32_t h = 0, valid = 0;
    for (uint32_t i = 0; i < tlen; ++i) {
        if (t[i] > 3) {
            valid = 0;
            continue;
        }
        h = ((h << 2) | t[i]) & mask;
        if (++valid >= (uint32_t)kK) idx[h].push_back(i + 1 - kK);
    }
    std::unordered_map<int64_t, uint32_t> votes;
    h = 0, valid = 0;
    for (uint32_t i = 0; i < qlen; ++i) {
        if (q[i] > 3) {
            valid = 0;
            continue;
        }
        h = ((h << 2) | q[i]) & mask;
        if (++valid < (uint32_t)kK) continue;
        auto it = idx.find(h);
        if (it == idx.end() || it->second.size() > 64) continue;
        const int64_t qp = i + 1 - kK;
        for (uint32_t tp : it->second) {
            const int64_t d = (int64_t)tp - qp;
            votes[d >= 0 ? d / kBin : -((-d + kBin - 1) / kBin)]++;
        }
    }
    if (votes.empty()) return r;
    int64_t best_bin = 0;
    uint32_t best_votes = 0;
    for (auto &kv : votes)
        if (kv.second > best_votes || (kv.second == best_votes && kv.first < best_bin))
            best_bin = kv.first, best_votes = kv.second;
    const int64_t d0 = best_bin * kBin + kBin / 2;
    // 2. banded local alignment over diagonals [d0 - kHalfBand, d0 + kHalfBand]
    const int BW = 2 * kHalfBand + 1;
    std::vector<int32_t> Hprev(BW + 2, 0), Hcur(BW + 2, 0);
    std::vector<uint8_t> tb((size_t)qlen * BW, 0);  // 0 stop, 1 diag, 2 up (q gap... del), 3 left (ins)
    int32_t best = 0;
    int64_t bi = -1, bk = -1;
    // cell (i, j) with j = i + d, band index k = d - (d0 - kHalfBand)
    for (uint32_t i = 0; i < qlen; ++i) {
        std::fill(Hcur.begin(), Hcur.end(), 0);
        for (int k = 0; k < BW; ++k) {
            const int64_t j = (int64_t)i + d0 - kHalfBand + k;
            if (j < 0 || j >= (int64_t)tlen) continue;
            // diag: (i-1, j-1) same k; up: (i-1, j) -> k+1; left: (i, j-1) -> k-1
            const int32_t diag = (i > 0 && j > 0 ? Hprev[k + 1] : 0) + (q[i] < 4 && q[i] == t[j] ? 1 : -2);
            const int32_t up = (i > 0 && k + 1 < BW ? Hprev[k + 2] : 0) - 2;
            const int32_t left = (k > 0 ? Hcur[k] : 0) - 2;
            int32_t v = 0;
            uint8_t dir = 0;
            if (diag > v) v = diag, dir = 1;
            if (up > v) v = up, dir = 2;
            if (left > v) v = left, dir = 3;
            Hcur[k + 1] = v;
            tb[(size_t)i * BW + k] = dir;
            if (v > best) best = v, bi = i, bk = k;
        }
        std::swap(Hprev, Hcur);
    }
    if (bi < 0) return r;
    // 3. traceback
    int64_t i = bi, k = bk;
    r.qe = (int32_t)bi + 1;
    r.te = (int32_t)(bi + d0 - kHalfBand + bk) + 1;
    r.score = best;
    for (;;) {
        const uint8_t dir = tb[(size_t)i * BW + k];
        if (dir == 0) break;
        const int64_t j = i + d0 - kHalfBand + k;
        if (dir == 1) {
            if (q[i] < 4 && q[i] == t[j]) ++r.mat;
            else ++r.mis;
            r.qb = (int32_t)i, r.tb = (int32_t)j;
            --i;
        } else if (dir == 2) {
            ++r.ins;  // query base not in target
            r.qb = (int32_t)i;
            --i, ++k;
        } else {
            ++r.del;
            r.tb = (int32_t)j;
            --k;
        }
        if (i < 0 || k < 0 || k >= BW) break;
    }
    r.aln = r.mat + r.mis + r.ins + r.del;
    return r;
}

uint64_t ccsx_synth_zmw(uint64_t seed, uint64_t hole, uint32_t L, uint32_t passes, char *out, uint32_t *lens,
                        char *insert)
{
    static const char B[4] = {'A', 'C', 'G', 'T'};
    uint64_t s = seed ^ hole;
    std::vector<uint8_t> ins(L), rc(L);
    for (uint32_t i = 0; i < L; ++i) ins[i] = (uint8_t)(splitmix64(s) >> 62);
    for (uint32_t i = 0; i < L; ++i) rc[i] = (uint8_t)(3 - ins[L - 1 - i]);
    if (insert)
        for (uint32_t i = 0; i < L; ++i) insert[i] = B[ins[i]];
    uint64_t o = 0;
    for (uint32_t p = 0; p < passes; ++p) {
        const std::vector<uint8_t> &tp = (p & 1) ? rc : ins;
        const uint64_t o0 = o;
        for (uint32_t i = 0; i < L; ++i) {
            const uint64_t u = splitmix64(s) % 1000;
            if (u >= 30) {
                if (u < 40) out[o++] = B[(tp[i] + 1 + splitmix64(s) % 3) & 3];
                else out[o++] = B[tp[i]];
            }
            if (splitmix64(s) % 1000 < 60) out[o++] = B[splitmix64(s) >> 62];
        }
        lens[p] = (uint32_t)(o - o0);
    }
    return o;
}

}  // extern "C"
