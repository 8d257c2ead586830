/*
 * ccsx_host.h -- the C host program's per-ZMW preparation (CPU side).
 *
 * Restates, for the GPU engine's caller, what ccsx does on its CPU threads
 * before the hot path: ccs_prepare (main.c:344-453: subread length groups,
 * template choice, strand assignment, abnormal-subread re-alignment and
 * trimming) and the in-place strand flip (main.c:471-476 / 527-531, using
 * seq_reverse_comp, seqio.h:138-148).
 */
#ifndef CCSX_HOST_H
#define CCSX_HOST_H
#include <stddef.h>
#include <stdint.h>

#include "ccsx_gpu.h" /* ccsx_zmw_in */

#ifdef __cplusplus
extern "C" {
#endif

/* seqio.h:120-148 -- in-place reverse complement (IUPAC/lowercase aware). */
void ccsx_revcomp(char *seq, uint32_t len);

/* main.c:344-453.  seqs = the ZMW's subreads concatenated, lens[n] their
 * lengths.  Writes the push list (<= n segments) into seg_off/seg_len/seg_rev
 * and returns its length.  Does not modify seqs. */
uint32_t ccsx_prepare(const char *seqs, const uint32_t *lens, uint32_t n,
                      uint32_t *seg_off, uint32_t *seg_len, uint8_t *seg_rev);

/* ccsx_prepare + the strand flip of every reverse segment, in place in seqs
 * (what ccs_for/ccs_for2 do before the first push). */
uint32_t ccsx_prepare_apply(char *seqs, const uint32_t *lens, uint32_t n,
                            uint32_t *seg_off, uint32_t *seg_len);

/* The pairwise aligner used by strand_match (main.c:255-290), standing in for
 * bsalign's kmer_striped_seqedit_pairwise(13, ...) (SPEC.md §8).  q/t are
 * 2-bit codes (values >= 4 never match).  Returns aligned columns (aln). */
typedef struct {
    int32_t qb, qe, tb, te, mat, mis, ins, del, aln, score;
} ccsx_pairaln;
ccsx_pairaln ccsx_pairwise(const uint8_t *q, uint32_t qlen, const uint8_t *t, uint32_t tlen);

/* Multi-GPU step 1 of the host program (replaces kt_for's dynamic dealing of
 * ZMW indices over threads, kthread.c:24-46).
 * ccsx_zmw_cost: estimated POA work of one prepared ZMW, S x (28 + nseg) with
 * S = sum of segment lengths.
 * ccsx_partition: nb = min(nparts, n / min_batch) batches (at least one);
 * the ZMWs ranked by decreasing cost (ties in input order) and rank r dealt to
 * batch r % nb, so batch costs differ by at most one ZMW's cost.  Batch b is
 * order[bounds[b] .. bounds[b+1]), in decreasing cost.  bounds needs room for
 * n + 1 entries.  Returns nb. */
uint64_t ccsx_zmw_cost(const uint32_t *seg_len, uint32_t nseg);
uint32_t ccsx_partition(const uint64_t *cost, uint32_t n, uint32_t nparts, uint32_t min_batch,
                        uint32_t *order, uint32_t *bounds);

/* Synthetic PacBio-like ZMW: insert of length L drawn from
 * splitmix64(seed ^ hole), `passes` full passes on alternating strands with
 * 6% insertions / 3% deletions / 1% substitutions.  Writes the concatenated
 * subreads into out (capacity >= passes * (2L + 16)) and their lengths into
 * lens[passes]; if insert != NULL the true insert (L bytes) is written too.
 * Returns the total number of bases written. */
uint64_t ccsx_synth_zmw(uint64_t seed, uint64_t hole, uint32_t L, uint32_t passes,
                        char *out, uint32_t *lens, char *insert);

/* Benchmarks: n synthetic ZMWs (ccsx_synth_zmw(seed, holes[i], L[i],
 * passes[i]), then ccsx_prepare_apply) made on nthreads threads; the batch
 * owns the data, ccsx_synth_batch_zmws gives the n push lists
 * (ccsx_zmw_in, include/ccsx_gpu.h) ready for ccsx_gpu_run. */
typedef struct ccsx_synth_batch ccsx_synth_batch;
ccsx_synth_batch *ccsx_synth_batch_make(uint64_t seed, const uint64_t *holes, const uint32_t *L,
                                        const uint32_t *passes, uint32_t n, int nthreads);
const ccsx_zmw_in *ccsx_synth_batch_zmws(const ccsx_synth_batch *b);
void ccsx_synth_batch_free(ccsx_synth_batch *b);

#ifdef __cplusplus
}
#endif
#endif
