/*
 * oracle/prep_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker of the host's
 * ccs_prepare; never linked into the product).
 *
 * An independent plain-C restatement of ccs_prepare and its helpers, written
 * from /root/reference/main.c:116-453 (not from the product's host/prepare.cpp,
 * which it is compared with):
 *   len_in_group / group_in_group      main.c:124-137
 *   init_group_lens (+ bubble sort)    main.c:139-212
 *   recap_base_bit_u1v                 main.c:222-241
 *   strand_match                       main.c:255-290
 *   get_template_grp                   main.c:300-342
 *   ccs_prepare                        main.c:344-453
 *   seq_reverse_comp (the strand flip) seqio.h:120-148
 * and of SPEC.md §8's stand-in for bsalign's kmer_striped_seqedit_pairwise
 * (main.c:264; bsalign is un-vendored, so this part is the builder's spec,
 * as the POA is: parity with bsalign unpinned).
 *
 * Where main.c depends on bsalign's un-vendored headers, SPEC.md §8 fixes the
 * choice: bubble_sort_array is a bubble sort that swaps neighbours when the
 * right one's group is strictly larger (stable, largest first);
 * base_bit_table maps A/C/G/T/U (either case) to 0-3 and anything else to 4.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "prep_oracle.h"

/* ------------------------------------------------------------------ groups */
typedef struct {
    int *ids;
    size_t n, cap;
    size_t sum_len;
} ogrp_t;

static void grp_push(ogrp_t *g, int id)
{
    if (g->n == g->cap) {
        g->cap = g->cap ? 2 * g->cap : 4;
        g->ids = realloc(g->ids, g->cap * sizeof(int));
    }
    g->ids[g->n++] = id;
}

/* main.c:124-129 */
static int len_in_group(const ogrp_t *g, uint32_t len, int tol)
{
    size_t tmp = (size_t)len * g->n;
    size_t diff = tmp > g->sum_len ? tmp - g->sum_len : g->sum_len - tmp;
    return diff * 100 < (size_t)tol * g->sum_len;
}

/* main.c:131-137 */
static int group_in_group(const ogrp_t *g, const ogrp_t *q, int tol)
{
    size_t a = g->sum_len * q->n, b = q->sum_len * g->n;
    size_t diff = a > b ? a - b : b - a;
    return diff * 100 < a * (size_t)tol;
}

/* main.c:139-212: returns the number of groups; *out holds them */
static int init_group_lens(const uint32_t *len, int n, int tol, ogrp_t **out)
{
    ogrp_t *g = calloc((size_t)(n ? n : 1), sizeof(ogrp_t));
    for (int i = 0; i < n; ++i) {
        int j;
        for (j = 0; j < i; ++j) {
            if (!g[j].sum_len) continue;
            if (len_in_group(&g[j], len[i], tol)) {
                grp_push(&g[j], i);
                g[j].sum_len += len[i];
                break;
            }
        }
        if (j < i) continue;
        grp_push(&g[j], i); /* j == i: a new group */
        g[j].sum_len = len[i];
    }
    int flag = 1;
    while (flag) {
        flag = 0;
        for (int j = 0; j < n; ++j) {
            if (g[j].n == 0) continue;
            for (int k = 0; k < j; ++k) {
                if (g[k].n && group_in_group(&g[k], &g[j], tol)) {
                    for (size_t x = 0; x < g[j].n; ++x) grp_push(&g[k], g[j].ids[x]);
                    g[k].sum_len += g[j].sum_len;
                    g[j].n = 0;
                    g[j].sum_len = 0;
                    flag = 1;
                    break;
                }
            }
        }
    }
    int m = 0;
    for (int j = 0; j < n; ++j) {
        if (g[j].n == 0) {
            free(g[j].ids);
            continue;
        }
        g[m++] = g[j];
    }
    /* bubble_sort_array(..., kv_size(b) > kv_size(a)) (main.c:208) */
    for (int i = 0; i + 1 < m; ++i)
        for (int j = 0; j + 1 < m - i; ++j)
            if (g[j + 1].n > g[j].n) {
                ogrp_t t = g[j];
                g[j] = g[j + 1];
                g[j + 1] = t;
            }
    *out = g;
    return m;
}

/* ----------------------------------------------------------- 2-bit copies */
static uint8_t base_bit(unsigned char c)
{
    switch (c | 0x20) {
    case 'a': return 0;
    case 'c': return 1;
    case 'g': return 2;
    case 't': case 'u': return 3;
    default: return 4;
    }
}

/* main.c:222-241 (reverse: reverse complement, 3 - code) */
static uint8_t *recap(uint8_t *v, const char *buf, size_t len, int reverse)
{
    v = realloc(v, len ? len : 1);
    for (size_t i = 0; i < len; ++i)
        v[i] = reverse ? (uint8_t)(3 - base_bit((unsigned char)buf[len - i - 1])) : base_bit((unsigned char)buf[i]);
    return v;
}

/* ---------------------------------------------- SPEC.md §8 pairwise aligner */
enum { PK = 13, PBIN = 32, PHALF = 256, PBW = 2 * PHALF + 1, PMAXOCC = 64 };

static int cmp_u64(const void *a, const void *b)
{
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

oprep_aln oprep_pairwise(const uint8_t *q, uint32_t qlen, const uint8_t *t, uint32_t tlen)
{
    oprep_aln r;
    memset(&r, 0, sizeof r);
    if (qlen < PK || tlen < PK) return r;
    /* target 13-mers as (kmer << 32 | position), sorted: per k-mer the
     * positions ascend */
    const uint32_t mask = (1u << (2 * PK)) - 1;
    uint64_t *tk = malloc((size_t)tlen * sizeof(uint64_t));
    size_t ntk = 0;
    uint32_t h = 0, run = 0;
    for (uint32_t i = 0; i < tlen; ++i) {
        if (t[i] > 3) {
            run = 0;
            continue;
        }
        h = ((h << 2) | t[i]) & mask;
        if (++run >= PK) tk[ntk++] = (uint64_t)h << 32 | (i + 1 - PK);
    }
    qsort(tk, ntk, sizeof(uint64_t), cmp_u64);
    /* diagonal votes, d = tpos - qpos in bins of 32 (floor), k-mers seen more
     * than 64 times in the target ignored */
    const int64_t bmin = floor_div(-(int64_t)qlen, PBIN) - 1, bmax = floor_div((int64_t)tlen, PBIN) + 1;
    uint32_t *votes = calloc((size_t)(bmax - bmin + 1), sizeof(uint32_t));
    int any = 0;
    h = 0, run = 0;
    for (uint32_t i = 0; i < qlen; ++i) {
        if (q[i] > 3) {
            run = 0;
            continue;
        }
        h = ((h << 2) | q[i]) & mask;
        if (++run < PK) continue;
        /* first entry of k-mer h */
        size_t lo = 0, hi = ntk;
        while (lo < hi) {
            size_t mid = (lo + hi) / 2;
            if ((tk[mid] >> 32) < h) lo = mid + 1;
            else hi = mid;
        }
        size_t e = lo;
        while (e < ntk && (tk[e] >> 32) == h) ++e;
        if (e == lo || e - lo > PMAXOCC) continue;
        const int64_t qp = (int64_t)i + 1 - PK;
        for (size_t x = lo; x < e; ++x) {
            votes[floor_div((int64_t)(uint32_t)tk[x] - qp, PBIN) - bmin]++;
            any = 1;
        }
    }
    free(tk);
    if (!any) {
        free(votes);
        return r;
    }
    /* the most votes; ties: the smallest bin */
    int64_t best_bin = 0;
    uint32_t bv = 0;
    for (int64_t b = bmin; b <= bmax; ++b)
        if (votes[b - bmin] > bv) bv = votes[b - bmin], best_bin = b;
    free(votes);
    const int64_t d0 = best_bin * PBIN + PBIN / 2;
    /* banded local alignment: cell (i, j), j = i + d0 - 256 + k, k in [0, 513);
     * match +1, mismatch (or a non-ACGT query base) -2, gap -2; the first of
     * diagonal, up (a query base not in the target), left (a target base not
     * in the query) that strictly beats the running value, which starts at 0
     * (local); the best cell is the first strict maximum in row-major order */
    int32_t *prev = calloc(PBW, sizeof(int32_t)), *cur = calloc(PBW, sizeof(int32_t));
    uint8_t *dirs = calloc((size_t)qlen * PBW, 1);
    int32_t best = 0;
    int64_t bi = -1, bk = -1;
    for (uint32_t i = 0; i < qlen; ++i) {
        memset(cur, 0, PBW * sizeof(int32_t));
        for (int k = 0; k < PBW; ++k) {
            const int64_t j = (int64_t)i + d0 - PHALF + k;
            if (j < 0 || j >= (int64_t)tlen) continue;
            const int32_t s = (q[i] < 4 && q[i] == t[j]) ? 1 : -2;
            const int32_t dg = (i > 0 && j > 0 ? prev[k] : 0) + s;
            const int32_t up = (i > 0 && k + 1 < PBW ? prev[k + 1] : 0) - 2;
            const int32_t lf = (k > 0 ? cur[k - 1] : 0) - 2;
            int32_t v = 0;
            uint8_t d = 0;
            if (dg > v) v = dg, d = 1;
            if (up > v) v = up, d = 2;
            if (lf > v) v = lf, d = 3;
            cur[k] = v;
            dirs[(size_t)i * PBW + k] = d;
            if (v > best) best = v, bi = i, bk = k;
        }
        int32_t *x = prev;
        prev = cur;
        cur = x;
    }
    free(prev);
    free(cur);
    if (bi < 0) {
        free(dirs);
        return r;
    }
    r.score = best;
    r.qe = (int32_t)bi + 1;
    r.te = (int32_t)(bi + d0 - PHALF + bk) + 1;
    int64_t i = bi, k = bk;
    while (i >= 0 && k >= 0 && k < PBW) {
        const uint8_t d = dirs[(size_t)i * PBW + k];
        if (!d) break;
        const int64_t j = i + d0 - PHALF + k;
        if (d == 1) {
            if (q[i] < 4 && q[i] == t[j]) r.mat++;
            else r.mis++;
            r.qb = (int32_t)i, r.tb = (int32_t)j;
            --i;
        } else if (d == 2) {
            r.ins++;
            r.qb = (int32_t)i;
            --i, ++k;
        } else {
            r.del++;
            r.tb = (int32_t)j;
            --k;
        }
    }
    free(dirs);
    r.aln = r.mat + r.mis + r.ins + r.del;
    return r;
}

/* main.c:255-290 */
static int strand_match(const uint8_t *q, uint32_t qlen, const uint8_t *t, uint32_t tlen, int sim, oprep_aln *rs)
{
    oprep_aln r = oprep_pairwise(q, qlen, t, tlen);
    if (r.aln * 2 > (qlen > tlen ? (int)tlen : (int)qlen) && r.mat * 100 >= r.aln * sim) {
        if (rs) *rs = r;
        return 1;
    }
    return 0;
}

/* main.c:300-342 */
static uint32_t get_template_grp(const char *seqs, const uint32_t *lens, const uint32_t *offs, const ogrp_t *g, int ng)
{
    uint32_t tg = 0;
    if (g[0].n < 2) return 0;
    uint8_t *border = NULL, *main_seq = NULL;
    for (int cg = 1; cg < ng; ++cg) {
        if (g[cg].n < 2 || g[cg].n * 5 < 4 * g[0].n) continue;
        const uint32_t ci = (uint32_t)g[cg].ids[g[cg].n / 2];
        const uint32_t clen = lens[ci];
        if (clen <= lens[g[tg].ids[g[tg].n / 2]] || clen <= 2000) continue;
        border = recap(border, seqs + offs[ci], 1000, 1);
        main_seq = recap(main_seq, seqs + offs[ci] + 1000, clen - 1000, 0);
        if (strand_match(border, 1000, main_seq, clen - 1000, 70, NULL)) continue; /* head match */
        border = recap(border, seqs + offs[ci] + clen - 1000, 1000, 1);
        main_seq = recap(main_seq, seqs + offs[ci], clen - 1000, 0);
        if (strand_match(border, 1000, main_seq, clen - 1000, 70, NULL)) continue; /* tail match */
        tg = (uint32_t)cg;
    }
    free(border);
    free(main_seq);
    return tg;
}

/* main.c:344-453.  n == 0 (never reached through the CLI, whose -c filter
 * keeps >= 5 subreads; main.c would index an empty group list) returns 0. */
uint32_t oprep_prepare(const char *seqs, const uint32_t *lens, uint32_t n, uint32_t *seg_off, uint32_t *seg_len,
                       uint8_t *seg_rev)
{
    if (n == 0) return 0;
    const int tol = 10;
    uint32_t *offs = malloc(n * sizeof(uint32_t));
    for (uint32_t i = 0, o = 0; i < n; o += lens[i], ++i) offs[i] = o;
    ogrp_t *g;
    const int ng = init_group_lens(lens, (int)n, tol, &g);
    uint32_t *map_group = malloc(n * sizeof(uint32_t));
    for (int i = 0; i < ng; ++i)
        for (size_t j = 0; j < g[i].n; ++j) map_group[g[i].ids[j]] = (uint32_t)i;
    const uint32_t tg = get_template_grp(seqs, lens, offs, g, ng);
    const uint32_t ti = (uint32_t)g[tg].ids[g[tg].n / 2];
    const uint32_t toffs = offs[ti], tlen = lens[ti];
    uint32_t ns = 0;
    seg_off[ns] = toffs, seg_len[ns] = tlen, seg_rev[ns] = 0, ++ns;
    uint8_t *tseq = NULL, *t2seq = NULL, *qseq = NULL;
    /* the two walks away from the template (main.c:374-412, 414-446) */
    for (int side = 0; side < 2; ++side) {
        uint8_t reverse = 0;
        int strand_adjust = 0;
        const int64_t step = side == 0 ? -1 : 1;
        for (int64_t k = (int64_t)ti + step; k >= 0 && k < (int64_t)n; k += step) {
            reverse = reverse == 0 ? 1 : 0;
            uint32_t so = offs[k], sl = lens[k];
            if (map_group[k] != tg) { /* abnormal length */
                strand_adjust = 1;
                if (sl < tlen) continue;
            } else if (!strand_adjust) {
                seg_off[ns] = so, seg_len[ns] = sl, seg_rev[ns] = reverse, ++ns;
                continue;
            }
            if (!tseq) {
                tseq = recap(NULL, seqs + toffs, tlen, 0);
                t2seq = recap(NULL, seqs + toffs, tlen, 1);
            }
            qseq = recap(qseq, seqs + so, sl, 0);
            oprep_aln rs;
            int hit = 0;
            if (strand_match(qseq, sl, tseq, tlen, 75, &rs)) hit = 1, reverse = 0;
            else if (strand_match(qseq, sl, t2seq, tlen, 75, &rs)) hit = 1, reverse = 1;
            if (hit) {
                so += (uint32_t)rs.qb, sl = (uint32_t)(rs.qe - rs.qb);
                if (len_in_group(&g[tg], sl, tol)) seg_off[ns] = so, seg_len[ns] = sl, seg_rev[ns] = reverse, ++ns;
                strand_adjust = map_group[k] != tg;
            } else {
                strand_adjust = 1; /* cannot be aligned */
            }
        }
    }
    free(tseq);
    free(t2seq);
    free(qseq);
    for (int i = 0; i < ng; ++i) free(g[i].ids);
    free(g);
    free(map_group);
    free(offs);
    return ns;
}

/* seqio.h:120-148: complement table (IUPAC pairs, identity elsewhere) and the
 * in-place reverse complement */
static unsigned char comp_of(unsigned char c)
{
    static const char from[] = "ACGTUMRWSYKVHDBNacgtumrwsykvhdbn";
    static const char to[] = "TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn";
    for (int i = 0; from[i]; ++i)
        if ((unsigned char)from[i] == c) return (unsigned char)to[i];
    return c;
}

void oprep_revcomp(char *s, uint32_t l)
{
    for (uint32_t i = 0, j = l ? l - 1 : 0; i < l / 2; ++i, --j) {
        const unsigned char a = (unsigned char)s[i], b = (unsigned char)s[j];
        s[i] = (char)comp_of(b);
        s[j] = (char)comp_of(a);
    }
    if (l & 1) s[l / 2] = (char)comp_of((unsigned char)s[l / 2]);
}

uint32_t oprep_prepare_apply(char *seqs, const uint32_t *lens, uint32_t n, uint32_t *seg_off, uint32_t *seg_len)
{
    uint8_t *rev = malloc(n ? n : 1);
    const uint32_t ns = oprep_prepare(seqs, lens, n, seg_off, seg_len, rev);
    for (uint32_t i = 0; i < ns; ++i)
        if (rev[i]) oprep_revcomp(seqs + seg_off[i], seg_len[i]);
    free(rev);
    return ns;
}
