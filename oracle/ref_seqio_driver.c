/*
 * ref_seqio_driver.c -- TEST INFRASTRUCTURE (oracle/_ref), never shipped.
 *
 * A driver of this project's own around the reference's UNMODIFIED subread
 * ingest, compiled from the reference sources where they lie
 * (/root/reference/{seqio.h,kseq.h,kstring.c,bamlite.c}, see ref_build.py).
 * It instantiates SEQIO_INIT(gzFile, gzread) exactly as main.c:23 does, opens
 * the input as main.c:808-811 does and loops kseq_zmw_read as step 0 does
 * (main.c:658-697: after a -1 the next chunk reads on; the input ends at
 * the first chunk that yields no ZMW), printing one line per call:
 *
 *   <ret> \t <movie> \t <hole> \t <len,len,...> \t <seqs> \t <revcomp(each subread) concatenated>
 *
 * and a line "<ret>" for every negative return.  Used to generate and
 * check tests/golden/host_seqio.json against ccsx_amd's restatement.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "kvec.h"
#include "kstring.h"
#include "bamlite.h"
#include "seqio.h"

SEQIO_INIT(gzFile, gzread)

int main(int argc, char **argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s <is_bam 0|1> <input>\n", argv[0]);
        return 2;
    }
    int isbam = atoi(argv[1]);
    gzFile fp = gzopen(argv[2], "rb");
    if (!fp) return 1;
    kseqs_zmw_t z;
    kseqs_zmw_initialize(&z, fp, isbam);
    int l, got;
    do {
    got = 0;
    while ((l = kseq_zmw_read(&z)) >= 0) {
        ++got;
        printf("%d\t%s\t%s\t", l, z.movie_name.s, z.hole.s);
        size_t tot = 0;
        for (size_t i = 0; i < kv_size(z.lens); ++i) {
            printf(i ? ",%d" : "%d", kv_A(z.lens, i));
            tot += (size_t)kv_A(z.lens, i);
        }
        printf("\t%.*s\t", (int)tot, z.seqs.s);
        char *buf = (char *)malloc(tot + 1);
        memcpy(buf, z.seqs.s, tot);
        size_t o = 0;
        for (size_t i = 0; i < kv_size(z.lens); ++i) {
            seq_reverse_comp(kv_A(z.lens, i), (unsigned char *)buf + o);
            o += (size_t)kv_A(z.lens, i);
        }
        printf("%.*s\n", (int)tot, buf);
        free(buf);
    }
    printf("%d\n", l);
    } while (got);
    zmw_seqs_release(&z);
    gzclose(fp);
    return 0;
}
