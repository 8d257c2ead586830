/*
 * oracle/poa_oracle.h -- CPU restatement of the ccsx consensus hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (ccsx_amd/, include/) may
 * include, link or call this code; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker.
 *
 * What it restates:
 *   - the bspoa C API main.c drives (init/beg/push/end/tidy_msa/free,
 *     main.c:486-501,552-575,841-858) following SPEC.md, the written POA
 *     specification of this project (bsalign itself is un-vendored, see
 *     DESIGN.md "Parity"); and
 *   - ccs_for  (main.c:455-508, -P "primitive" mode) and
 *     ccs_for2 (main.c:510-647, default "shredded" mode) on segments that
 *     ccs_prepare() has already strand-normalised.
 */
#ifndef CCSX_POA_ORACLE_H
#define CCSX_POA_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct opoa_s opoa_t;

/* Scoring exactly as main.c:841-849 sets BSPOAPar (M, X, O, E; Q=P=0). */
opoa_t *opoa_init(int M, int X, int O, int E, int bandwidth);
void opoa_free(opoa_t *g);
void opoa_beg(opoa_t *g);
void opoa_push(opoa_t *g, const char *seq, uint32_t len);
void opoa_end(opoa_t *g);
void opoa_tidy_msa(opoa_t *g);

uint32_t opoa_cns(const opoa_t *g, const uint8_t **cns);
uint32_t opoa_msa(const opoa_t *g, const uint32_t **idxs, const uint8_t **cols, uint32_t *mrow);
uint64_t opoa_cells(const opoa_t *g);   /* DP cells since opoa_init */
uint32_t opoa_nrows(const opoa_t *g);   /* graph nodes after opoa_end */

/* One ZMW: mode 0 = shredded (ccs_for2), 1 = primitive (ccs_for).
 * seqs+offs[k] / lens[k] are the strand-normalised segments in push order.
 * Writes the ASCII CCS into out (capacity >= sum(lens)); returns its length. */
size_t ocsx_zmw(opoa_t *g, int mode, const char *seqs, const uint32_t *offs,
                const uint32_t *lens, uint32_t n, char *out);
/* The same, recording per shredding round (breakpoint, MSA columns) -- the
 * values main.c:619-620 prints at -v >= 3 -- into bplog (bpcap pairs). */
size_t ocsx_zmw_log(opoa_t *g, int mode, const char *seqs, const uint32_t *offs, const uint32_t *lens, uint32_t n,
                    char *out, uint32_t *bplog, uint32_t bpcap, uint32_t *nbp);

/* Many ZMWs on nthreads CPU threads (kt_for semantics); out[i] capacity
 * >= sum(lens[i]) + 1; cells[i] = DP cells of ZMW i. */
void ocsx_batch(int mode, int nthreads, uint32_t nz, const char **seqs, const uint32_t **offs,
                const uint32_t **lens, const uint32_t *nseg, char **out, size_t *olen, uint64_t *cells);

#ifdef __cplusplus
}
#endif
#endif
