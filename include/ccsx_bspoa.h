/*
 * ccsx_bspoa.h -- drop-in for the bsalign bspoa.h API that ccsx's main.c uses,
 * backed by the MI355X engine (one device launch per end_bspoa).
 *
 * Replaces (un-vendored bsalign):
 *   BSPOAPar par = DEFAULT_BSPOA_PAR; par.M = 2; ...     main.c:841-849
 *   BSPOA *init_bspoa(BSPOAPar)                          main.c:851
 *   void   beg_bspoa(BSPOA*)                             main.c:486,552
 *   void   push_bspoa(BSPOA*, char *seq, u4i len)        main.c:490,563,568
 *   void   end_bspoa(BSPOA*)                             main.c:492,571
 *   void   tidy_msa_bspoa(BSPOA*)                        main.c:572
 *   void   free_bspoa(BSPOA*)                            main.c:858
 * and the fields main.c reads directly: g->cns->{buffer,size} (2-bit codes,
 * main.c:495-500), g->msaidxs->{buffer,size} and g->msacols->buffer (column j
 * at msacols + msaidxs[j] * (nseq + 4); row 1..n = reads, n+1 = consensus,
 * codes >= 4 are gaps; main.c:575-623).
 *
 * Only main.c's parameter set is supported (M=2 X=-6 O=-3 E=-2 Q=P=0,
 * bandwidth=128); init_bspoa aborts with a message otherwise.  Errors from the
 * device are fatal (abort with a message), as the reference has no error path.
 * The fast path for whole chunks of ZMWs is include/ccsx_gpu.h.
 */
#ifndef CCSX_BSPOA_H
#define CCSX_BSPOA_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int refmode, shuffle, realn;
    int M, X, O, E, Q, P;
    int editbw, bandwidth;
} BSPOAPar;

#define DEFAULT_BSPOA_PAR {0, 0, 0, 2, -6, -3, -2, 0, 0, 32, 128}

typedef struct {
    uint8_t *buffer;
    uint64_t size, cap;
} ccsx_u1v;

typedef struct {
    uint32_t *buffer;
    uint64_t size, cap;
} ccsx_u4v;

typedef struct BSPOA {
    BSPOAPar par;
    ccsx_u1v *cns;      /* consensus, 2-bit codes */
    ccsx_u4v *msaidxs;  /* storage index of the j-th MSA column */
    ccsx_u1v *msacols;  /* column-major MSA, (nseq + 4) bytes per column */
    uint32_t nseq;
    void *impl;
} BSPOA;

BSPOA *init_bspoa(BSPOAPar par);
void beg_bspoa(BSPOA *g);
void push_bspoa(BSPOA *g, char *seq, uint32_t len);
void end_bspoa(BSPOA *g);
void tidy_msa_bspoa(BSPOA *g);
void free_bspoa(BSPOA *g);

#ifdef __cplusplus
}
#endif
#endif
