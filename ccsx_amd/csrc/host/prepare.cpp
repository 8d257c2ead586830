// prepare.cpp -- ccs_prepare and the strand flip (main.c:116-453, seqio.h:120-148).
//
// Host code of the C host program; the GPU engine consumes its output.  The
// pairwise aligner that bsalign's kmer_striped_seqedit_pairwise provides to
// strand_match is un-vendored; ccsx_pairwise restates it per SPEC.md §8.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ccsx_host.h"

namespace {

// seqio.h:120-137 complement table (identity outside IUPAC letters)
struct CompTable {
    unsigned char t[256];
    CompTable()
    {
        for (int i = 0; i < 256; ++i) t[i] = (unsigned char)i;
        const char *from = "ABCDGHKMNRSTUVWYabcdghkmnrstuvwy";
        const char *to = "TVGHCDMKNYSAABWRtvghcdmknysaabwr";
        for (int i = 0; from[i]; ++i) t[(unsigned char)from[i]] = (unsigned char)to[i];
    }
};
const CompTable kComp;

// bsalign dna.h base_bit_table as used by recap_base_bit_u1v (main.c:222-241)
inline uint8_t base_bit(unsigned char c)
{
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 4;
    }
}

// main.c:222-241: 2-bit copy, reverse = reverse complement (3 - code)
void recap(std::vector<uint8_t> &v, const char *buf, size_t len, bool reverse)
{
    v.resize(len);
    if (reverse)
        for (size_t i = 0; i < len; ++i) v[i] = (uint8_t)(3 - base_bit((unsigned char)buf[len - i - 1]));
    else
        for (size_t i = 0; i < len; ++i) v[i] = base_bit((unsigned char)buf[i]);
}

struct Group {
    std::vector<int> ids;
    size_t sum_len = 0;
};

// main.c:124-129
inline bool len_in_group(const Group &g, uint32_t len, int tol)
{
    size_t tmp = (size_t)len * g.ids.size();
    size_t diff = tmp > g.sum_len ? tmp - g.sum_len : g.sum_len - tmp;
    return diff * 100 < (size_t)tol * g.sum_len;
}

// main.c:131-137
inline bool group_in_group(const Group &g, const Group &q, int tol)
{
    size_t a = g.sum_len * q.ids.size(), b = q.sum_len * g.ids.size();
    size_t diff = a > b ? a - b : b - a;
    return diff * 100 < a * (size_t)tol;
}

// main.c:139-212.  bubble_sort_array's tie order is unknown offline (bsalign
// un-vendored): groups are stably sorted by size, largest first (SPEC.md §8).
std::vector<Group> init_group_lens(const uint32_t *a, int n, int tol)
{
    std::vector<Group> g(n);
    for (int i = 0; i < n; ++i) {
        int j;
        for (j = 0; j < i; ++j) {
            if (!g[j].sum_len) continue;
            if (len_in_group(g[j], a[i], tol)) {
                g[j].ids.push_back(i);
                g[j].sum_len += a[i];
                break;
            }
        }
        if (j < i) continue;
        g[j].ids.push_back(i);
        g[j].sum_len = a[i];
    }
    for (bool flag = true; flag;) {
        flag = false;
        for (int j = 0; j < n; ++j) {
            if (g[j].ids.empty()) continue;
            for (int k = 0; k < j; ++k) {
                if (!g[k].ids.empty() && group_in_group(g[k], g[j], tol)) {
                    g[k].ids.insert(g[k].ids.end(), g[j].ids.begin(), g[j].ids.end());
                    g[k].sum_len += g[j].sum_len;
                    g[j].ids.clear();
                    g[j].sum_len = 0;
                    flag = true;
                    break;
                }
            }
        }
    }
    std::vector<Group> out;
    for (auto &x : g)
        if (!x.ids.empty()) out.push_back(std::move(x));
    std::stable_sort(out.begin(), out.end(), [](const Group &x, const Group &y) { return x.ids.size() > y.ids.size(); });
    return out;
}

// main.c:255-290
bool strand_match(const std::vector<uint8_t> &q, const std::vector<uint8_t> &t, int sim, ccsx_pairaln *rs)
{
    ccsx_pairaln r = ccsx_pairwise(q.data(), (uint32_t)q.size(), t.data(), (uint32_t)t.size());
    const int qlen = (int)q.size(), tlen = (int)t.size();
    if (r.aln * 2 > (qlen > tlen ? tlen : qlen) && r.mat * 100 >= r.aln * sim) {
        if (rs) *rs = r;
        return true;
    }
    return false;
}

struct Seg {
    uint32_t offs, len;
    uint8_t reverse;
};

// main.c:300-342
uint32_t get_template_grp(const char *seqs, const uint32_t *lens, const uint32_t *offs, const std::vector<Group> &groups)
{
    uint32_t tg = 0;
    if (groups[tg].ids.size() < 2) return 0;
    std::vector<uint8_t> border, main_seq;
    for (uint32_t cg = 1; cg < groups.size(); ++cg) {
        if (groups[cg].ids.size() < 2 || groups[cg].ids.size() * 5 < 4 * groups[0].ids.size()) continue;
        const uint32_t ci = (uint32_t)groups[cg].ids[groups[cg].ids.size() / 2];
        const uint32_t clen = lens[ci];
        if (clen <= lens[groups[tg].ids[groups[tg].ids.size() / 2]] || clen <= 2000) continue;
        recap(border, seqs + offs[ci], 1000, true);
        recap(main_seq, seqs + offs[ci] + 1000, clen - 1000, false);
        if (strand_match(border, main_seq, 70, nullptr)) continue;
        recap(border, seqs + offs[ci] + clen - 1000, 1000, true);
        recap(main_seq, seqs + offs[ci], clen - 1000, false);
        if (strand_match(border, main_seq, 70, nullptr)) continue;
        tg = cg;
    }
    return tg;
}

}  // namespace

extern "C" {

void ccsx_revcomp(char *s, uint32_t l)
{
    unsigned char *seq = reinterpret_cast<unsigned char *>(s);
    for (uint32_t i = 0; i < l >> 1; ++i) {
        unsigned char t = seq[l - 1 - i];
        seq[l - i - 1] = kComp.t[seq[i]];
        seq[i] = kComp.t[t];
    }
    if (l & 1) seq[l >> 1] = kComp.t[seq[l >> 1]];
}

// main.c:344-453
uint32_t ccsx_prepare(const char *seqs, const uint32_t *lens, uint32_t n, uint32_t *seg_off, uint32_t *seg_len,
                      uint8_t *seg_rev)
{
    if (n == 0) return 0;
    const int tol = 10;
    std::vector<uint32_t> offs(n);
    for (uint32_t i = 0, o = 0; i < n; o += lens[i], ++i) offs[i] = o;
    std::vector<Group> groups = init_group_lens(lens, (int)n, tol);
    std::vector<uint32_t> map_group(n);
    for (uint32_t i = 0; i < groups.size(); ++i)
        for (int id : groups[i].ids) map_group[id] = i;
    const uint32_t tg = get_template_grp(seqs, lens, offs.data(), groups);
    const uint32_t ti = (uint32_t)groups[tg].ids[groups[tg].ids.size() / 2];
    const uint32_t toffs = offs[ti], tlen = lens[ti];
    std::vector<Seg> segs;
    segs.push_back(Seg{toffs, tlen, 0});
    std::vector<uint8_t> tseq, t2seq, qseq;
    bool have_t = false;
    ccsx_pairaln rs;
    auto visit = [&](uint32_t k, uint8_t &reverse, bool &strand_adjust) {
        reverse = reverse == 0 ? 1 : 0;
        Seg seg{offs[k], lens[k], reverse};
        if (map_group[k] != tg) {
            strand_adjust = true;
            if (seg.len < tlen) return;
        } else if (!strand_adjust) {
            segs.push_back(seg);
            return;
        }
        if (!have_t) {
            recap(tseq, seqs + toffs, tlen, false);
            recap(t2seq, seqs + toffs, tlen, true);
            have_t = true;
        }
        recap(qseq, seqs + seg.offs, seg.len, false);
        if (strand_match(qseq, tseq, 75, &rs)) {
            reverse = 0;
            seg.offs += rs.qb, seg.len = rs.qe - rs.qb, seg.reverse = reverse;
            if (len_in_group(groups[tg], seg.len, tol)) segs.push_back(seg);
            strand_adjust = map_group[k] != tg;
        } else if (strand_match(qseq, t2seq, 75, &rs)) {
            reverse = 1;
            seg.offs += rs.qb, seg.len = rs.qe - rs.qb, seg.reverse = reverse;
            if (len_in_group(groups[tg], seg.len, tol)) segs.push_back(seg);
            strand_adjust = map_group[k] != tg;
        } else {
            strand_adjust = true;
        }
    };
    uint8_t reverse = 0;
    bool strand_adjust = false;
    for (int k = (int)ti - 1; k >= 0; --k) visit((uint32_t)k, reverse, strand_adjust);
    reverse = 0, strand_adjust = false;
    for (uint32_t i = ti + 1; i < n; ++i) visit(i, reverse, strand_adjust);
    for (size_t i = 0; i < segs.size(); ++i) {
        seg_off[i] = segs[i].offs;
        seg_len[i] = segs[i].len;
        if (seg_rev) seg_rev[i] = segs[i].reverse;
    }
    return (uint32_t)segs.size();
}

uint32_t ccsx_prepare_apply(char *seqs, const uint32_t *lens, uint32_t n, uint32_t *seg_off, uint32_t *seg_len)
{
    std::vector<uint8_t> rev(n ? n : 1);
    uint32_t ns = ccsx_prepare(seqs, lens, n, seg_off, seg_len, rev.data());
    for (uint32_t l = 0; l < ns; ++l)
        if (rev[l]) ccsx_revcomp(seqs + seg_off[l], seg_len[l]);
    return ns;
}

}  // extern "C"
