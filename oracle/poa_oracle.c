/*
 * oracle/poa_oracle.c -- CPU restatement of SPEC.md (TEST INFRASTRUCTURE ONLY).
 *
 * Plain scalar C, written for clarity: every decision (band placement, max
 * tie-breaks, traceback codes, graph merge, column consensus) follows SPEC.md
 * section by section so the HIP kernel can be checked against it byte for
 * byte.  The shredding loop and the breakpoint scan restate main.c:541-641.
 *
 * Parity status: the POA itself (end_bspoa/tidy_msa_bspoa) follows SPEC.md,
 * not bsalign, which is not available anywhere in this pipeline
 * (SURVEY.md §0-1, §8c): "parity unpinned" for everything inside end_bspoa.
 */
#include "poa_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NEG (-(1 << 29))
#define NONE 0xFFFFFFFFu

enum { HC_MPRED = 0, HC_MSRC = 1, HC_DEL = 2, HC_INS = 3 };
enum { EV_ALN = 0u, EV_INS = 1u, EV_LEAD = 2u };
#define EV_ROW(e) ((e) & 0x3FFFFFFFu)
#define EV_KIND(e) ((e) >> 30)

typedef struct {
    uint32_t R, E, nw, rcap, ecap;
    uint8_t *nb;    /* base (bits 0-1) | column-start flag (bit 2) */
    uint64_t *mem;  /* R*nw read-membership bits */
    uint32_t *poff; /* R+1 */
    uint32_t *pred; /* E, per row in edge-creation order */
} graph_t;

struct opoa_s {
    int M, X, O, E, W;
    /* pushed reads */
    uint32_t nseq, seqcap;
    uint8_t **seqs;
    uint32_t *lens, *lcap;
    graph_t g, h;
    uint32_t *rfirst, *rlast, rcap_reads;
    /* DP scratch */
    uint32_t dpcap;
    int32_t *Hs, *Ds, *roff, *rmax, *rarg;
    uint8_t *code;
    uint16_t *ms, *ds;
    /* per-read scratch */
    uint32_t evcap;
    uint32_t *ev, *tgt, *ipt, *ifix;
    uint8_t *ibase, *ics;
    uint32_t shcap;
    uint32_t *shift, *addp;
    uint8_t *fixed;
    /* results */
    uint32_t ncns, ncols, ccap;
    uint8_t *cns, *ccons;
    uint32_t *msaidxs, msacap, idxcap;  /* msacols bytes, msaidxs entries */
    uint8_t *msacols;
    uint32_t mrow;
    uint64_t cells;
};

static void *xrealloc(void *p, size_t n)
{
    void *q = realloc(p, n ? n : 1);
    if (!q) {
        fprintf(stderr, "[poa_oracle] out of memory (%zu bytes)\n", n);
        abort();
    }
    return q;
}

/* ASCII -> 2-bit code (SPEC.md §1: A/a=0 C/c=1 G/g=2 T/t/U/u=3, others 0). */
static uint8_t enc(unsigned char c)
{
    switch (c) {
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 0;
    }
}

static void graph_reserve(graph_t *g, uint32_t R, uint32_t E, uint32_t nw)
{
    if (R + 1 > g->rcap || nw != g->nw) {
        uint32_t c = R + 1 > g->rcap ? (R + 1) * 2 : g->rcap;
        g->nb = xrealloc(g->nb, c);
        g->mem = xrealloc(g->mem, (size_t)c * nw * 8);
        g->poff = xrealloc(g->poff, (size_t)(c + 1) * 4);
        g->rcap = c;
    }
    if (E > g->ecap) {
        uint32_t c = E * 2 + 16;
        g->pred = xrealloc(g->pred, (size_t)c * 4);
        g->ecap = c;
    }
    g->nw = nw;
}

opoa_t *opoa_init(int M, int X, int O, int E, int bandwidth)
{
    opoa_t *g = calloc(1, sizeof(*g));
    g->M = M, g->X = X, g->O = O, g->E = E, g->W = bandwidth;
    return g;
}

void opoa_free(opoa_t *g)
{
    if (!g) return;
    for (uint32_t i = 0; i < g->seqcap; ++i) free(g->seqs[i]);
    free(g->seqs), free(g->lens), free(g->lcap);
    graph_t *gs[2] = {&g->g, &g->h};
    for (int i = 0; i < 2; ++i) free(gs[i]->nb), free(gs[i]->mem), free(gs[i]->poff), free(gs[i]->pred);
    free(g->rfirst), free(g->rlast);
    free(g->Hs), free(g->Ds), free(g->roff), free(g->rmax), free(g->rarg), free(g->code), free(g->ms), free(g->ds);
    free(g->ev), free(g->tgt), free(g->ipt), free(g->ifix), free(g->ibase), free(g->ics);
    free(g->shift), free(g->addp), free(g->fixed);
    free(g->cns), free(g->ccons), free(g->msaidxs), free(g->msacols);
    free(g);
}

/* main.c:486,552 -- reset for a new POA */
void opoa_beg(opoa_t *g)
{
    g->nseq = 0;
    g->ncns = 0;
    g->ncols = 0;
    g->g.R = g->g.E = 0;
}

/* main.c:490,563,568 -- the library keeps its own 2-bit copy */
void opoa_push(opoa_t *g, const char *seq, uint32_t len)
{
    if (g->nseq == g->seqcap) {
        uint32_t c = g->seqcap ? g->seqcap * 2 : 16;
        g->seqs = xrealloc(g->seqs, c * sizeof(uint8_t *));
        g->lens = xrealloc(g->lens, c * 4);
        g->lcap = xrealloc(g->lcap, c * 4);
        for (uint32_t i = g->seqcap; i < c; ++i) g->seqs[i] = NULL, g->lcap[i] = 0;
        g->seqcap = c;
    }
    uint32_t k = g->nseq++;
    if (len + 1 > g->lcap[k]) {
        g->seqs[k] = xrealloc(g->seqs[k], len + 1);
        g->lcap[k] = len + 1;
    }
    for (uint32_t i = 0; i < len; ++i) g->seqs[k][i] = enc((unsigned char)seq[i]);
    g->lens[k] = len;
}

static inline int32_t getH(const opoa_t *g, uint32_t p, int64_t j)
{
    if (j < 0) return NEG;
    int64_t t = j - g->roff[p];
    if (t < 0 || t >= g->W) return NEG;
    return g->Hs[(size_t)p * g->W + t];
}

static inline int32_t getD(const opoa_t *g, uint32_t p, int64_t j)
{
    if (j < 0) return NEG;
    int64_t t = j - g->roff[p];
    if (t < 0 || t >= g->W) return NEG;
    return g->Ds[(size_t)p * g->W + t];
}

/* Debug statistics (not part of the restatement): DP rows by the class the
 * one-wave kernel objects give them (ccsx_kernel.hip dpS_row / dpA_cold, ring
 * of OPOA_KRING rows).  Summed over every DP since the last reset; a process-
 * wide counter, read single-threaded by tools/row_kinds.py. */
#define OPOA_KRING 8
enum { RK_FAST0, RK_FAST1, RK_CHAIN, RK_NP1, RK_NP2, RK_GEN, RK_FAR, RK_SPILL, RK_N };
static uint64_t row_kinds[RK_N];
void opoa_row_kinds(uint64_t *out, int reset)
{
    memcpy(out, row_kinds, sizeof row_kinds);
    if (reset) memset(row_kinds, 0, sizeof row_kinds);
}

/* Debug statistics: the traceback's predecessor moves by the row distance
 * they cover (1, 2, 3, 4-8, far row) and M / D kind, and the traceback steps;
 * summed like row_kinds (tools/row_kinds.py --tb). */
enum { TB_D1, TB_D2, TB_D3, TB_D4_8, TB_FAR, TB_MOVES_D, TB_STEPS, TB_M4, TB_M5_8, TB_DD1, TB_DDFAR, TB_DDGE2, TB_N };
static uint64_t tb_moves[TB_N];
void opoa_tb_moves(uint64_t *out, int reset)
{
    memcpy(out, tb_moves, sizeof tb_moves);
    if (reset) memset(tb_moves, 0, sizeof tb_moves);
}

static void count_tb_move(const graph_t *G, uint32_t r, uint32_t p, int isD)
{
    const uint32_t np = G->poff[r + 1] - G->poff[r];
    int far = np > 4;
    for (uint32_t s = 0; s < np; ++s) far |= r - G->pred[G->poff[r] + s] > OPOA_KRING;
    const uint32_t d = r - p;
    tb_moves[far ? TB_FAR : d == 1 ? TB_D1 : d == 2 ? TB_D2 : d == 3 ? TB_D3 : TB_D4_8]++;
    if (isD) tb_moves[TB_MOVES_D]++;
    if (isD && !far) tb_moves[d == 1 ? TB_DD1 : TB_DDGE2]++;
    if (isD && far) tb_moves[TB_DDFAR]++;
    if (!isD && !far && d == 4) tb_moves[TB_M4]++;
    if (!isD && !far && d > 4) tb_moves[TB_M5_8]++;
}

static void count_row_kind(const graph_t *G, uint32_t r, int32_t off, int32_t poff, const uint8_t *spill)
{
    const uint32_t np = G->poff[r + 1] - G->poff[r];
    const uint32_t *pl = G->pred + G->poff[r];
    int far = np > 4;
    for (uint32_t s = 0; s < np; ++s) far |= r - pl[s] > OPOA_KRING;
    if (spill[r]) row_kinds[RK_SPILL]++;
    const int chain = np == 1 && pl[0] + 1 == r;
    const int32_t sh = off - poff;
    if (far) row_kinds[RK_FAR]++;
    else if (chain && !spill[r] && (sh == 0 || sh == 1)) row_kinds[sh ? RK_FAST1 : RK_FAST0]++;
    else if (chain && sh >= 0 && sh <= 2) row_kinds[RK_CHAIN]++;
    else if (np == 1) row_kinds[RK_NP1]++;
    else if (np == 2) row_kinds[RK_NP2]++;
    else row_kinds[RK_GEN]++;
}

/* SPEC.md §3: banded read-vs-graph DP, rows in graph row order. */
static void dp_align(opoa_t *g, const uint8_t *q, uint32_t m, uint32_t *er_out, uint32_t *ej_out)
{
    const graph_t *G = &g->g;
    const int W = g->W, O = g->O, E = g->E;
    const uint32_t R = G->R;
    if (R > g->dpcap) {
        uint32_t c = R * 2;
        g->Hs = xrealloc(g->Hs, (size_t)c * W * 4);
        g->Ds = xrealloc(g->Ds, (size_t)c * W * 4);
        g->code = xrealloc(g->code, (size_t)c * W);
        g->ms = xrealloc(g->ms, (size_t)c * W * 2);
        g->ds = xrealloc(g->ds, (size_t)c * W * 2);
        g->roff = xrealloc(g->roff, c * 4);
        g->rmax = xrealloc(g->rmax, c * 4);
        g->rarg = xrealloc(g->rarg, c * 4);
        g->dpcap = c;
    }
    int32_t Hp[1024], Xv[1024];
    const int32_t lim = m > (uint32_t)W ? (int32_t)(m - W) : 0;
    int32_t bestE = INT32_MIN;
    uint32_t er = 0, ej = 0;
    uint8_t *spill = calloc(R + 1, 1);
    for (uint32_t r = 0; r < R; ++r)
        for (uint32_t e = G->poff[r]; e < G->poff[r + 1]; ++e)
            if (r - G->pred[e] > OPOA_KRING) spill[G->pred[e]] = 1;
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t np = G->poff[r + 1] - G->poff[r];
        const uint32_t *pl = G->pred + G->poff[r];
        const uint8_t base = G->nb[r] & 3;
        int32_t off = 0;
        if (np) {
            int32_t bm = INT32_MIN;
            uint32_t bp = 0;
            for (uint32_t s = 0; s < np; ++s)
                if (g->rmax[pl[s]] > bm) bm = g->rmax[pl[s]], bp = pl[s];
            off = g->rarg[bp] + 1 - W / 2;
            if (off < 0) off = 0;
            if (off > lim) off = lim;
        }
        g->roff[r] = off;
        count_row_kind(G, r, off, r ? g->roff[r - 1] : 0, spill);
        int32_t *H = g->Hs + (size_t)r * W, *D = g->Ds + (size_t)r * W;
        uint8_t *cd = g->code + (size_t)r * W;
        uint16_t *msr = g->ms + (size_t)r * W, *dsr = g->ds + (size_t)r * W;
        for (int t = 0; t < W; ++t) {
            const int64_t j = (int64_t)off + t;
            if (j >= m) {
                H[t] = D[t] = NEG;
                Hp[t] = NEG;
                cd[t] = 0, msr[t] = 0, dsr[t] = 0;
                continue;
            }
            int32_t Mh = NEG;
            uint32_t msl = 0;
            for (uint32_t s = 0; s < np; ++s) {
                int32_t h = getH(g, pl[s], j - 1);
                if (h > Mh) Mh = h, msl = s;
            }
            const int32_t src = j == 0 ? 0 : O + E * (int32_t)j;
            int hc;
            int32_t mb;
            if (Mh >= src) mb = Mh, hc = HC_MPRED;
            else mb = src, hc = HC_MSRC, msl = 0;
            const int32_t Mv = mb + (base == q[j] ? g->M : g->X);
            int32_t Dv = NEG;
            uint32_t dsl = 0;
            int dx = 0;
            for (uint32_t s = 0; s < np; ++s) {
                int32_t a = getH(g, pl[s], j) + O + E;
                int32_t b = getD(g, pl[s], j) + E;
                int32_t c = b > a ? b : a;
                if (c > Dv) Dv = c, dsl = s, dx = b > a;
            }
            int32_t hp = Mv;
            if (Dv > Mv) hp = Dv, hc = HC_DEL;
            Hp[t] = hp;
            Xv[t] = hp - E * t;
            D[t] = Dv;
            cd[t] = (uint8_t)(hc | (dx << 2));
            msr[t] = (uint16_t)msl;
            dsr[t] = (uint16_t)dsl;
        }
        /* SPEC.md §3.4: in-row insertion as an exclusive prefix max */
        int32_t ex = NEG, ex_prev = NEG, rm = INT32_MIN, ra = 0;
        for (int t = 0; t < W; ++t) {
            const int64_t j = (int64_t)off + t;
            if (j >= m) break;
            if (t > 0) {
                ex_prev = ex;
                if (Xv[t - 1] > ex) ex = Xv[t - 1];
            }
            const int32_t I = t == 0 ? NEG : O + E * t + ex;
            const int iext = t > 0 && ex_prev > Xv[t - 1];
            int32_t h = Hp[t];
            if (I > h) h = I, cd[t] = (uint8_t)((cd[t] & ~3u) | HC_INS);
            cd[t] |= (uint8_t)(iext << 3);
            H[t] = h;
            if (h > rm) rm = h, ra = (int32_t)j;
            const int32_t e = h + (j == (int64_t)m - 1 ? 0 : O + E * (int32_t)(m - 1 - j));
            if (e > bestE) bestE = e, er = r, ej = (uint32_t)j;
        }
        g->rmax[r] = rm;
        g->rarg[r] = ra;
    }
    free(spill);
    g->cells += (uint64_t)R * (m < (uint32_t)W ? m : (uint32_t)W);
    *er_out = er;
    *ej_out = ej;
}

/* SPEC.md §4: traceback into per-read-base events. */
static void traceback(opoa_t *g, uint32_t m, uint32_t er, uint32_t ej)
{
    const graph_t *G = &g->g;
    const int W = g->W;
    for (uint32_t jj = ej + 1; jj < m; ++jj) g->ev[jj] = (EV_INS << 30) | er;
    uint32_t r = er;
    int64_t j = ej;
    int st = 0; /* 0 = H, 1 = D, 2 = I */
    uint64_t guard = 0, lim = (uint64_t)G->R * 2 + (uint64_t)m * 2 + 16;
    for (;;) {
        if (++guard > lim) {
            fprintf(stderr, "[poa_oracle] traceback did not terminate\n");
            abort();
        }
        const size_t cell = (size_t)r * W + (size_t)(j - g->roff[r]);
        const uint8_t c = g->code[cell];
        tb_moves[TB_STEPS]++;
        if (st == 0) {
            const int hc = c & 3;
            if (hc == HC_MPRED) {
                g->ev[j] = (EV_ALN << 30) | r;
                const uint32_t p = G->pred[G->poff[r] + g->ms[cell]];
                count_tb_move(G, r, p, 0);
                r = p;
                --j;
            } else if (hc == HC_MSRC) {
                g->ev[j] = (EV_ALN << 30) | r;
                for (int64_t jj = 0; jj < j; ++jj) g->ev[jj] = (EV_LEAD << 30) | r;
                break;
            } else if (hc == HC_DEL) {
                st = 1;
            } else {
                st = 2;
            }
        } else if (st == 1) {
            st = (c >> 2) & 1 ? 1 : 0;
            const uint32_t p = G->pred[G->poff[r] + g->ds[cell]];
            count_tb_move(G, r, p, 1);
            r = p;
        } else {
            g->ev[j] = (EV_INS << 30) | r;
            st = (c >> 3) & 1 ? 2 : 0;
            --j;
        }
    }
}

static inline uint32_t col_start(const graph_t *G, uint32_t v)
{
    while (!(G->nb[v] & 4)) --v;
    return v;
}

static inline uint32_t col_end(const graph_t *G, uint32_t v)
{
    ++v;
    while (v < G->R && !(G->nb[v] & 4)) ++v;
    return v;
}

/* SPEC.md §5: merge read k (events in g->ev) into the graph. */
static void merge(opoa_t *g, uint32_t k, const uint8_t *q, uint32_t m)
{
    graph_t *G = &g->g, *N = &g->h;
    const uint32_t R = G->R, nw = G->nw;
    uint32_t K = 0;
    for (uint32_t j = 0; j < m; ++j) {
        const uint8_t b = q[j];
        uint32_t pt = 0, cs = 1, fix = NONE;
        if (R == 0) {
            pt = 0;
        } else {
            const uint32_t e = g->ev[j], v = EV_ROW(e), kind = EV_KIND(e);
            if (kind == EV_ALN) {
                if ((G->nb[v] & 3) == b) {
                    g->tgt[j] = v;
                    continue;
                }
                const uint32_t a = col_start(G, v), z = col_end(G, v);
                uint32_t u = a;
                for (; u < z; ++u)
                    if ((G->nb[u] & 3) >= b) break;
                if (u < z && (G->nb[u] & 3) == b) {
                    g->tgt[j] = u;
                    continue;
                }
                pt = u;
                cs = u == a;
                if (cs) fix = a;
            } else if (kind == EV_INS) {
                pt = col_end(G, v);
            } else {
                pt = col_start(G, v);
            }
        }
        g->ipt[K] = pt, g->ibase[K] = b, g->ics[K] = (uint8_t)cs, g->ifix[K] = fix;
        g->tgt[j] = 0x80000000u | K;
        ++K;
    }
    /* shift[k] = number of new items at points <= k */
    memset(g->shift, 0, (size_t)(R + 1) * 4);
    for (uint32_t i = 0; i < K; ++i) g->shift[g->ipt[i]]++;
    for (uint32_t x = 1; x <= R; ++x) g->shift[x] += g->shift[x - 1];
    memset(g->fixed, 0, R + 1);
    for (uint32_t i = 0; i < K; ++i)
        if (g->ifix[i] != NONE) g->fixed[g->ifix[i]] = 1;
    const uint32_t R2 = R + K;
#define NEWIDX(t) (((t) & 0x80000000u) ? g->ipt[(t) & 0x7FFFFFFFu] + ((t) & 0x7FFFFFFFu) : (t) + g->shift[(t)])
    /* new in-edges: at most one per target of this read */
    for (uint32_t x = 0; x < R2; ++x) g->addp[x] = NONE;
    for (uint32_t j = 1; j < m; ++j) {
        const uint32_t s = g->tgt[j - 1], d = g->tgt[j];
        if (!(d & 0x80000000u) && !(s & 0x80000000u)) {
            int dup = 0;
            for (uint32_t e = G->poff[d]; e < G->poff[d + 1]; ++e)
                if (G->pred[e] == s) { dup = 1; break; }
            if (dup) continue;
        }
        g->addp[NEWIDX(d)] = NEWIDX(s);
    }
    graph_reserve(N, R2, G->E + m + 1, nw);
    for (uint32_t x = 0; x < R; ++x) {
        const uint32_t n = x + g->shift[x];
        N->nb[n] = g->fixed[x] ? (uint8_t)(G->nb[x] & 3) : G->nb[x];
        memcpy(N->mem + (size_t)n * nw, G->mem + (size_t)x * nw, nw * 8);
    }
    for (uint32_t i = 0; i < K; ++i) {
        const uint32_t n = g->ipt[i] + i;
        N->nb[n] = (uint8_t)(g->ibase[i] | (g->ics[i] << 2));
        memset(N->mem + (size_t)n * nw, 0, nw * 8);
    }
    for (uint32_t j = 0; j < m; ++j) {
        const uint32_t n = NEWIDX(g->tgt[j]);
        N->mem[(size_t)n * nw + (k >> 6)] |= 1ull << (k & 63);
    }
    /* CSR: old preds remapped (creation order kept), then the new edge */
    uint32_t e2 = 0;
    uint32_t x = 0; /* old row cursor */
    for (uint32_t n = 0; n < R2; ++n) {
        N->poff[n] = e2;
        if (x < R && x + g->shift[x] == n) {
            for (uint32_t e = G->poff[x]; e < G->poff[x + 1]; ++e) {
                const uint32_t p = G->pred[e];
                N->pred[e2++] = p + g->shift[p];
            }
            ++x;
        }
        if (g->addp[n] != NONE) N->pred[e2++] = g->addp[n];
    }
    N->poff[R2] = e2;
    N->R = R2;
    N->E = e2;
    for (uint32_t kk = 0; kk < k; ++kk)
        if (g->rfirst[kk] != NONE) {
            g->rfirst[kk] += g->shift[g->rfirst[kk]];
            g->rlast[kk] += g->shift[g->rlast[kk]];
        }
    g->rfirst[k] = NEWIDX(g->tgt[0]);
    g->rlast[k] = NEWIDX(g->tgt[m - 1]);
#undef NEWIDX
    graph_t t = g->g;
    g->g = g->h;
    g->h = t;
}

/* SPEC.md §6: column consensus. */
static void call_columns(opoa_t *g)
{
    const graph_t *G = &g->g;
    const uint32_t R = G->R, nw = G->nw, n = g->nseq;
    if (R + 1 > g->ccap) {
        g->ccap = (R + 1) * 2;
        g->ccons = xrealloc(g->ccons, g->ccap);
        g->cns = xrealloc(g->cns, g->ccap);
    }
    /* column index of each read's first/last row */
    uint32_t *colof = xrealloc(NULL, (size_t)(R + 1) * 4);
    uint32_t c = 0;
    for (uint32_t r = 0; r < R; ++r) {
        if (G->nb[r] & 4) ++c;
        colof[r] = c - 1;
    }
    g->ncols = c;
    g->ncns = 0;
    uint32_t col = 0;
    for (uint32_t r = 0; r < R; col++) {
        uint32_t z = r + 1;
        while (z < R && !(G->nb[z] & 4)) ++z;
        uint32_t cnt[4] = {0, 0, 0, 0}, tot = 0, cov = 0;
        for (uint32_t u = r; u < z; ++u) {
            uint32_t pc = 0;
            for (uint32_t w = 0; w < nw; ++w) pc += (uint32_t)__builtin_popcountll(G->mem[(size_t)u * nw + w]);
            cnt[G->nb[u] & 3] += pc;
            tot += pc;
        }
        for (uint32_t k = 0; k < n; ++k)
            if (g->rfirst[k] != NONE && colof[g->rfirst[k]] <= col && col <= colof[g->rlast[k]]) ++cov;
        uint32_t best = 0;
        for (uint32_t b = 1; b < 4; ++b)
            if (cnt[b] > cnt[best]) best = b;
        const uint32_t gap = cov - tot;
        const uint8_t cons = cnt[best] >= gap ? (uint8_t)best : 4;
        g->ccons[col] = cons;
        if (cons < 4) g->cns[g->ncns++] = cons;
        r = z;
    }
    free(colof);
}

/* main.c:492,571 -- end_bspoa: build the graph read by read, then call the consensus */
void opoa_end(opoa_t *g)
{
    const uint32_t n = g->nseq, nw = (n + 63) / 64 ? (n + 63) / 64 : 1;
    uint32_t tot = 0, maxm = 0;
    for (uint32_t k = 0; k < n; ++k) {
        tot += g->lens[k];
        if (g->lens[k] > maxm) maxm = g->lens[k];
    }
    g->g.R = g->g.E = 0;
    g->g.nw = 0;
    graph_reserve(&g->g, tot + 1, tot + n + 1, nw);
    graph_reserve(&g->h, tot + 1, tot + n + 1, nw);
    if (n > g->rcap_reads) {
        g->rcap_reads = n * 2;
        g->rfirst = xrealloc(g->rfirst, g->rcap_reads * 4);
        g->rlast = xrealloc(g->rlast, g->rcap_reads * 4);
    }
    if (maxm + 1 > g->evcap) {
        g->evcap = (maxm + 1) * 2;
        g->ev = xrealloc(g->ev, g->evcap * 4);
        g->tgt = xrealloc(g->tgt, g->evcap * 4);
        g->ipt = xrealloc(g->ipt, g->evcap * 4);
        g->ifix = xrealloc(g->ifix, g->evcap * 4);
        g->ibase = xrealloc(g->ibase, g->evcap);
        g->ics = xrealloc(g->ics, g->evcap);
    }
    if (tot + 2 > g->shcap) {
        g->shcap = (tot + 2) * 2;
        g->shift = xrealloc(g->shift, g->shcap * 4);
        g->addp = xrealloc(g->addp, g->shcap * 4);
        g->fixed = xrealloc(g->fixed, g->shcap);
    }
    for (uint32_t k = 0; k < n; ++k) {
        g->rfirst[k] = g->rlast[k] = NONE;
        const uint32_t m = g->lens[k];
        if (m == 0) continue;
        if (g->g.R) {
            uint32_t er, ej;
            dp_align(g, g->seqs[k], m, &er, &ej);
            traceback(g, m, er, ej);
        }
        merge(g, k, g->seqs[k], m);
    }
    call_columns(g);
}

/* main.c:572 -- tidy_msa_bspoa: column-major MSA, mrow = nseq + 4 bytes per
 * column; row 0 and rows n+2, n+3 are filler (4), rows 1..n the reads, row
 * n+1 the consensus. */
void opoa_tidy_msa(opoa_t *g)
{
    const graph_t *G = &g->g;
    const uint32_t n = g->nseq, nw = G->nw, mrow = n + 4, nc = g->ncols;
    g->mrow = mrow;
    if ((size_t)nc * mrow + 1 > g->msacap) {
        g->msacap = (uint32_t)((size_t)nc * mrow * 2 + 16);
        g->msacols = xrealloc(g->msacols, g->msacap);
    }
    /* its own capacity: a later POA with fewer reads (smaller mrow) can have
     * more columns in the same msacols bytes */
    if (nc + 1 > g->idxcap) {
        g->idxcap = nc * 2 + 16;
        g->msaidxs = xrealloc(g->msaidxs, (size_t)g->idxcap * 4);
    }
    memset(g->msacols, 4, (size_t)nc * mrow);
    uint32_t col = 0;
    for (uint32_t r = 0; r < G->R; col++) {
        uint32_t z = r + 1;
        while (z < G->R && !(G->nb[z] & 4)) ++z;
        uint8_t *cp = g->msacols + (size_t)col * mrow;
        for (uint32_t u = r; u < z; ++u)
            for (uint32_t k = 0; k < n; ++k)
                if (G->mem[(size_t)u * nw + (k >> 6)] >> (k & 63) & 1) cp[k + 1] = G->nb[u] & 3;
        cp[n + 1] = g->ccons[col];
        g->msaidxs[col] = col;
        r = z;
    }
}

uint32_t opoa_cns(const opoa_t *g, const uint8_t **cns)
{
    *cns = g->cns;
    return g->ncns;
}

uint32_t opoa_msa(const opoa_t *g, const uint32_t **idxs, const uint8_t **cols, uint32_t *mrow)
{
    *idxs = g->msaidxs;
    *cols = g->msacols;
    *mrow = g->mrow;
    return g->ncols;
}

uint64_t opoa_cells(const opoa_t *g) { return g->cells; }
uint32_t opoa_nrows(const opoa_t *g) { return g->g.R; }

static const char BIT_BASE[5] = {'A', 'C', 'G', 'T', 'N'};

/* ccs_for (main.c:455-508) and ccs_for2 (main.c:510-647) after ccs_prepare.
 * bplog (optional, shredded mode): per round the pair (breakpoint i,
 * msaidxs->size) that main.c:619-620 prints at -v >= 3, at most bpcap pairs;
 * *nbp = the number of rounds. */
size_t ocsx_zmw(opoa_t *g, int mode, const char *seqs, const uint32_t *offs,
                const uint32_t *lens, uint32_t n, char *out)
{
    return ocsx_zmw_log(g, mode, seqs, offs, lens, n, out, NULL, 0, NULL);
}

size_t ocsx_zmw_log(opoa_t *g, int mode, const char *seqs, const uint32_t *offs, const uint32_t *lens, uint32_t n,
                    char *out, uint32_t *bplog, uint32_t bpcap, uint32_t *nbp)
{
    uint32_t nround = 0;
    if (nbp) *nbp = 0;
    size_t ol = 0;
    if (mode == 1) {
        opoa_beg(g);
        for (uint32_t k = 0; k < n; ++k) opoa_push(g, seqs + offs[k], lens[k]);
        opoa_end(g);
        for (uint32_t l = 0; l < g->ncns; ++l) out[ol++] = BIT_BASE[g->cns[l]];
        out[ol] = 0;
        return ol;
    }
    const uint32_t window = 10, addlen = 2000, minlen = 1000, initlen = 2000, minwin = 5;
    const uint32_t rowrate = 80, colrate = n < 10 ? 60 : 80;
    const uint32_t nseq = n, mrow = nseq + 4;
    uint32_t *pos = calloc(n ? n : 1, 4);
    uint8_t *rowcnt = malloc(n ? n : 1);
    uint32_t flag = 1;
    while (flag) {
        uint32_t i;
        for (uint32_t ws = initlen;; ws += addlen) {
            opoa_beg(g);
            for (i = 0; i < n; ++i)
                if (pos[i] + ws + minlen >= lens[i]) break;
            if (i < n || n < 3) {
                flag = 0;
                for (i = 0; i < n; ++i) opoa_push(g, seqs + offs[i] + pos[i], lens[i] - pos[i]);
            } else {
                for (i = 0; i < n; ++i) opoa_push(g, seqs + offs[i] + pos[i], ws);
            }
            opoa_end(g);
            opoa_tidy_msa(g);
            if (!flag) {
                i = g->ncols;
                break;
            }
            /* main.c:580-612; an MSA of <= window columns has no breakpoint (SPEC.md §7) */
            i = 0;
            if (g->ncols > window) {
                for (i = g->ncols - window; i >= 1; i--) {
                    uint32_t j, k, nogwin = 0;
                    memset(rowcnt, 0, nseq);
                    for (j = i; j < i + window; ++j) {
                        const uint8_t *col = g->msacols + (size_t)g->msaidxs[j] * mrow;
                        if (col[nseq + 1] >= 4) {
                            if (nogwin) continue;
                            else break;
                        }
                        ++nogwin;
                        uint32_t colcnt = 0;
                        for (k = 0; k < nseq; k++)
                            if (col[k + 1] == col[nseq + 1]) colcnt++, rowcnt[k]++;
                        if (colcnt * 100 < colrate * nseq) break;
                    }
                    if (j < i + window || nogwin < minwin) continue;
                    for (k = 0; k < nseq; ++k)
                        if (rowcnt[k] * 100 < rowrate * nogwin) break;
                    if (k >= nseq) break;
                }
            }
            if (i >= 1) break;
        }
        /* main.c:619-620 (-v >= 3) */
        if (bplog && nround < bpcap) bplog[2 * nround] = i, bplog[2 * nround + 1] = g->ncols;
        ++nround;
        /* main.c:622-638 */
        for (uint32_t j = 0; j < i; j++) {
            const uint8_t *col = g->msacols + (size_t)g->msaidxs[j] * mrow;
            if (flag)
                for (uint32_t k = 0; k < n; ++k)
                    if (col[k + 1] < 4) ++pos[k];
            if (col[nseq + 1] < 4) out[ol++] = BIT_BASE[col[nseq + 1]];
        }
    }
    free(pos);
    free(rowcnt);
    out[ol] = 0;
    if (nbp) *nbp = nround;
    return ol;
}

/* ------------------------------------------------------------------------
 * ocsx_batch: kt_for-style CPU run of ocsx_zmw over many ZMWs with nthreads
 * pthreads (kthread.c:24-65 semantics: dynamic work sharing, one POA object per
 * thread).  This is what "ccsx -j N" spends its step-1 time on; bench.py's
 * cpu_baseline leg times it.
 * ------------------------------------------------------------------------ */
#include <pthread.h>

typedef struct {
    int mode;
    uint32_t nz;
    const char **seqs;
    const uint32_t **offs, **lens;
    const uint32_t *nseg;
    char **out;
    size_t *olen;
    uint64_t *cells;
    uint32_t next;
    pthread_mutex_t mu;
} batch_t;

static void *batch_worker(void *arg)
{
    batch_t *b = arg;
    opoa_t *g = opoa_init(2, -6, -3, -2, 128);
    for (;;) {
        pthread_mutex_lock(&b->mu);
        uint32_t i = b->next++;
        pthread_mutex_unlock(&b->mu);
        if (i >= b->nz) break;
        uint64_t c0 = g->cells;
        b->olen[i] = ocsx_zmw(g, b->mode, b->seqs[i], b->offs[i], b->lens[i], b->nseg[i], b->out[i]);
        b->cells[i] = g->cells - c0;
    }
    opoa_free(g);
    return NULL;
}

void ocsx_batch(int mode, int nthreads, uint32_t nz, const char **seqs, const uint32_t **offs,
                const uint32_t **lens, const uint32_t *nseg, char **out, size_t *olen, uint64_t *cells)
{
    batch_t b = {mode, nz, seqs, offs, lens, nseg, out, olen, cells, 0};
    pthread_mutex_init(&b.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t *tid = malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; ++t) pthread_create(&tid[t], NULL, batch_worker, &b);
    for (int t = 0; t < nthreads; ++t) pthread_join(tid[t], NULL);
    free(tid);
    pthread_mutex_destroy(&b.mu);
}

/* Debug statistics of the current graph: hist[0] = rows, [1] = rows with >1
 * predecessor, [2] = max in-degree, [3..] = rows having a predecessor further
 * than 8, 16, 32, 64, 128 rows back. */
void opoa_graph_stats(const opoa_t *g, uint64_t *hist)
{
    const graph_t *G = &g->g;
    memset(hist, 0, 8 * sizeof(uint64_t));
    hist[0] = G->R;
    for (uint32_t r = 0; r < G->R; ++r) {
        uint32_t np = G->poff[r + 1] - G->poff[r], far = 0;
        if (np > 1) hist[1]++;
        if (np > hist[2]) hist[2] = np;
        for (uint32_t e = G->poff[r]; e < G->poff[r + 1]; ++e)
            if (r - G->pred[e] > far) far = r - G->pred[e];
        const uint32_t th[5] = {8, 16, 32, 64, 128};
        for (int i = 0; i < 5; ++i)
            if (far > th[i]) hist[3 + i]++;
    }
}

/* Debug: rows of the current graph that have a successor further than `ring`
 * rows ahead (the rows a kernel with a `ring`-row LDS ring must spill). */
uint32_t opoa_spill_rows(const opoa_t *g, uint32_t ring)
{
    const graph_t *G = &g->g;
    uint8_t *f = calloc(G->R + 1, 1);
    for (uint32_t r = 0; r < G->R; ++r)
        for (uint32_t e = G->poff[r]; e < G->poff[r + 1]; ++e)
            if (r - G->pred[e] > ring) f[G->pred[e]] = 1;
    uint32_t n = 0;
    for (uint32_t r = 0; r < G->R; ++r) n += f[r];
    free(f);
    return n;
}
