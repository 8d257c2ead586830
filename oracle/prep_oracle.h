/* oracle/prep_oracle.h -- TEST INFRASTRUCTURE ONLY: the checker's restatement
 * of ccs_prepare (main.c:116-453) and SPEC.md §8's pairwise aligner
 * (oracle/prep_oracle.c). */
#pragma once
#include <stdint.h>

typedef struct {
    int32_t qb, qe, tb, te, score, mat, mis, ins, del, aln;
} oprep_aln;

/* SPEC.md §8 (bsalign's kmer_striped_seqedit_pairwise(13, ...) stand-in, main.c:264) */
oprep_aln oprep_pairwise(const uint8_t *q, uint32_t qlen, const uint8_t *t, uint32_t tlen);
/* ccs_prepare: the push list (offsets into seqs, lengths, reverse flags), template first */
uint32_t oprep_prepare(const char *seqs, const uint32_t *lens, uint32_t n, uint32_t *seg_off, uint32_t *seg_len,
                       uint8_t *seg_rev);
/* seq_reverse_comp (seqio.h:138-148) */
void oprep_revcomp(char *s, uint32_t l);
/* oprep_prepare + the strand flip of every reverse segment, in place */
uint32_t oprep_prepare_apply(char *seqs, const uint32_t *lens, uint32_t n, uint32_t *seg_off, uint32_t *seg_len);
