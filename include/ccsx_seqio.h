/*
 * ccsx_seqio.h -- subread ingest of the C host program (CPU side).
 *
 * Restates seqio.h's kseq_zmw_read (seqio.h:152-201): consecutive records
 * whose names split on '/' into exactly three non-empty fields
 * (movie/hole/range) are grouped into one ZMW; a record name with any other
 * field count prints "invalid zmw name :<name>" and ends the input.  Records
 * come from FASTA/FASTQ (kseq.h:178-218 semantics; gzip allowed) or, when
 * is_bam != 0, from unaligned BAM (bamlite.c:78-165, nt16 decoding of
 * seqio.h:92-118).
 */
#ifndef CCSX_SEQIO_H
#define CCSX_SEQIO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ccsx_reader ccsx_reader;

/* path "-" reads stdin.  Returns NULL if the file cannot be opened. */
ccsx_reader *ccsx_reader_open(const char *path, int is_bam);

/* Next ZMW: returns its number of subreads (> 0), or -1 at end of input (or
 * after an invalid name).  Pointers stay valid until the next call. */
int ccsx_reader_next(ccsx_reader *r, const char **movie, const char **hole, const char **seqs,
                     const uint32_t **lens);

void ccsx_reader_close(ccsx_reader *r);

#ifdef __cplusplus
}
#endif
#endif
