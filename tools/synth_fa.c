// synth_fa.c -- stream a synthetic subread FASTA to stdout,
// fast enough to feed the CLI on stdin (main.c:804-808: input "-") at
// config-E scale without a 10+ GB file.  Records are `synth/<hole>/<qs>_<qe>`,
// single-line uppercase, the same bytes tools/gen_synth.py writes (the
// generator is the product's ccsx_synth_zmw, include/ccsx_host.h).
//
//   synth_fa NZMW HOLE0 [L PASSES] [THREADS]   (no L/PASSES: config E shapes,
//                                               bench.py zmw_shape)
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ccsx_host.h"

static const uint64_t kSeed = 20201104ull;

// bench.py zmw_shape: config E's per-hole insert length and pass count
static void e_shape(uint64_t hole, uint32_t *L, uint32_t *passes)
{
    uint64_t x = hole * 0x9E3779B97F4A7C15ull + kSeed;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    *L = 5000u + (uint32_t)(x % 20001u);
    uint32_t p = 5u + (uint32_t)((x >> 20) % 8u);
    const uint32_t cap = 450000u / (*L * 11u / 10u);
    if (p > cap) p = cap;
    if (p < 5u) p = 5u;
    *passes = p;
}

typedef struct {
    uint64_t hole0, n;
    uint32_t L, passes;
    uint64_t next;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    uint64_t written;  // ZMWs written so far (in hole order)
} job_t;

enum { kBatch = 64 };

static void *worker(void *arg)
{
    job_t *j = arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const uint64_t b = j->next;
        j->next += kBatch;
        pthread_mutex_unlock(&j->mu);
        if (b >= j->n) break;
        const uint64_t e = b + kBatch < j->n ? b + kBatch : j->n;
        size_t cap = 1u << 20, len = 0;
        char *buf = malloc(cap);
        for (uint64_t i = b; i < e; ++i) {
            const uint64_t h = j->hole0 + i;
            uint32_t L = j->L, P = j->passes;
            if (!L) e_shape(h, &L, &P);
            const size_t most = (size_t)P * (2 * (size_t)L + 16) + 64;
            char *seq = malloc(most), *ins = malloc((size_t)L + 16);
            uint32_t *lens = malloc(sizeof(uint32_t) * (P + 1));
            const uint64_t tot = ccsx_synth_zmw(kSeed, h, L, P, seq, lens, ins);
            (void)tot;
            uint64_t off = 0;
            for (uint32_t k = 0; k < P; ++k) {
                const size_t need = len + lens[k] + 64;
                if (need > cap) {
                    while (cap < need) cap *= 2;
                    buf = realloc(buf, cap);
                }
                len += (size_t)sprintf(buf + len, ">synth/%llu/%llu_%llu\n", (unsigned long long)h,
                                       (unsigned long long)off, (unsigned long long)(off + lens[k]));
                memcpy(buf + len, seq + off, lens[k]);
                len += lens[k];
                buf[len++] = '\n';
                off += lens[k];
            }
            free(seq);
            free(ins);
            free(lens);
        }
        // write in hole order
        pthread_mutex_lock(&j->mu);
        while (j->written != b) pthread_cond_wait(&j->cv, &j->mu);
        pthread_mutex_unlock(&j->mu);
        fwrite(buf, 1, len, stdout);
        free(buf);
        pthread_mutex_lock(&j->mu);
        j->written = e;
        pthread_cond_broadcast(&j->cv);
        pthread_mutex_unlock(&j->mu);
    }
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: synth_fa NZMW HOLE0 [L PASSES] [THREADS]\n");
        return 1;
    }
    job_t j;
    memset(&j, 0, sizeof j);
    j.n = strtoull(argv[1], NULL, 10);
    j.hole0 = strtoull(argv[2], NULL, 10);
    int nt = 8;
    if (argc >= 5) j.L = (uint32_t)atoi(argv[3]), j.passes = (uint32_t)atoi(argv[4]);
    if (argc >= 6) nt = atoi(argv[5]);
    if (nt < 1) nt = 1;
    pthread_mutex_init(&j.mu, NULL);
    pthread_cond_init(&j.cv, NULL);
    static char obuf[1 << 22];
    setvbuf(stdout, obuf, _IOFBF, sizeof obuf);
    pthread_t *t = malloc(sizeof(pthread_t) * (size_t)nt);
    for (int i = 0; i < nt; ++i) pthread_create(&t[i], NULL, worker, &j);
    for (int i = 0; i < nt; ++i) pthread_join(t[i], NULL);
    fflush(stdout);
    free(t);
    return 0;
}
