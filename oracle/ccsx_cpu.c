/*
 * oracle/ccsx_cpu.c -- a CPU-only ccsx: the host program's ingest (the
 * product library's C-ABI, include/ccsx_seqio.h, pinned by the reference's own
 * seqio.h on tests/golden/host) around the oracle's ccs_prepare
 * (oracle/prep_oracle.c, an independent restatement of main.c:116-453) and
 * POA (oracle/poa_oracle.c).
 *
 * TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it as the
 * stand-in for `ccsx -A -j N` (main.c:723-870), which is unbuildable here
 * (bsalign is not vendored).  It is a scalar C restatement, not bsalign's SIMD
 * code.  Same options and pipeline shape as the reference: step 0 reads a
 * chunk (1,024 -> 4,096 -> 16,384 ZMWs, filters -m/-M/-c/-X as main.c:659-672),
 * step 1 runs ccs_prepare + strand flip + ccs_for2 / ccs_for on -j threads with
 * dynamic sharing (kthread.c:24-46), step 2 writes in input order.
 *
 *   ccsx_cpu [-j N] [-P] [-A] [-m MIN] [-M MAX] [-c C] IN OUT
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../include/ccsx_seqio.h"
#include "poa_oracle.h"
#include "prep_oracle.h"

typedef struct {
    char *name;  /* movie/hole */
    char *seqs;
    uint32_t *lens, n;
    char *ccs;
    size_t ccs_len;
} zmw_t;

typedef struct {
    zmw_t *z;
    size_t nz;
    size_t next;
    int mode;
    pthread_mutex_t mu;
} step_t;

static void *worker(void *arg)
{
    step_t *s = arg;
    opoa_t *g = opoa_init(2, -6, -3, -2, 128); /* main.c:841-849 */
    uint32_t *off = NULL, *len = NULL, cap = 0;
    for (;;) {
        pthread_mutex_lock(&s->mu);
        size_t i = s->next++;
        pthread_mutex_unlock(&s->mu);
        if (i >= s->nz) break;
        zmw_t *z = &s->z[i];
        if (z->n > cap) {
            cap = z->n;
            off = realloc(off, cap * 4);
            len = realloc(len, cap * 4);
        }
        const uint32_t ns = oprep_prepare_apply(z->seqs, z->lens, z->n, off, len);
        size_t tot = 0;
        for (uint32_t k = 0; k < z->n; ++k) tot += z->lens[k];
        z->ccs = malloc(tot + 16);
        z->ccs_len = ocsx_zmw(g, s->mode, z->seqs, off, len, ns, z->ccs);
    }
    free(off);
    free(len);
    opoa_free(g);
    return NULL;
}

int main(int argc, char **argv)
{
    int c, nthreads = 1, mode = 0, isbam = 1, min_len = 5000, max_len = 500000, min_count = 3;
    while ((c = getopt(argc, argv, "j:PAm:M:c:")) != -1) {
        switch (c) {
        case 'j': nthreads = atoi(optarg); break;
        case 'P': mode = 1; break;
        case 'A': isbam = 0; break;
        case 'm': min_len = atoi(optarg); break;
        case 'M': max_len = atoi(optarg); break;
        case 'c': min_count = atoi(optarg); break;
        default: return 2;
        }
    }
    if (argc - optind != 2) return 2;
    ccsx_reader *rd = ccsx_reader_open(argv[optind], isbam);
    FILE *out = fopen(argv[optind + 1], "w");
    if (!rd || !out) return 1;
    if (nthreads < 1) nthreads = 1;
    size_t chunk = 1024;
    for (;;) {
        /* step 0 (main.c:652-697) */
        zmw_t *zs = calloc(chunk, sizeof(zmw_t));
        size_t nz = 0;
        const char *movie, *hole, *seqs;
        const uint32_t *lens;
        int l;
        while ((l = ccsx_reader_next(rd, &movie, &hole, &seqs, &lens)) >= 0) {
            if (l < min_count + 2) continue;
            size_t tot = 0;
            for (int k = 0; k < l; ++k) tot += lens[k];
            if (tot > (size_t)max_len || tot < (size_t)min_len) continue;
            zmw_t *z = &zs[nz++];
            z->name = malloc(strlen(movie) + strlen(hole) + 2);
            sprintf(z->name, "%s/%s", movie, hole);
            z->seqs = malloc(tot + 1);
            memcpy(z->seqs, seqs, tot);
            z->lens = malloc((size_t)l * 4);
            memcpy(z->lens, lens, (size_t)l * 4);
            z->n = (uint32_t)l;
            if (nz >= chunk) break;
        }
        if (!nz) {
            free(zs);
            break;
        }
        /* step 1 */
        step_t s = {zs, nz, 0, mode};
        pthread_mutex_init(&s.mu, NULL);
        pthread_t *tid = malloc(sizeof(pthread_t) * (size_t)nthreads);
        for (int t = 0; t < nthreads; ++t) pthread_create(&tid[t], NULL, worker, &s);
        for (int t = 0; t < nthreads; ++t) pthread_join(tid[t], NULL);
        free(tid);
        pthread_mutex_destroy(&s.mu);
        /* step 2 (main.c:707-717) */
        for (size_t i = 0; i < nz; ++i) {
            if (zs[i].ccs_len) fprintf(out, ">%s/ccs\n%.*s\n", zs[i].name, (int)zs[i].ccs_len, zs[i].ccs);
            free(zs[i].name), free(zs[i].seqs), free(zs[i].lens), free(zs[i].ccs);
        }
        free(zs);
        if (chunk < 16384) chunk *= 4;
    }
    ccsx_reader_close(rd);
    fclose(out);
    return 0;
}
