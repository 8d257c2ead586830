/*
 * ccsx_gpu.h -- batched C-ABI of the MI355X consensus engine.
 *
 * Replaces step 1 of ccsx's 3-stage pipeline (main.c:698-706):
 *
 *     kt_for(p->nthreads, split_subread ? ccs_for2 : ccs_for, in, n_zmws);
 *
 * with one call per chunk of ZMWs.  The caller runs ccs_prepare()
 * (main.c:344-453) and the strand flip (main.c:471-476 / 527-531) on its CPU
 * threads and passes, per ZMW, the strand-normalised segments in push order
 * (template, template-1 .. 0, template+1 .. n-1).  Everything from there
 * (shredding main.c:541-641 or the -P single POA main.c:486-502, i.e. every
 * beg/push/end/tidy_msa_bspoa call, the breakpoint scan and the CCS emission)
 * runs on the GPU.  Scoring is main.c:841-849's (M=2 X=-6 O=-3 E=-2,
 * bandwidth 128); SPEC.md defines the POA.
 *
 * Ownership: input buffers belong to the caller and are only read during the
 * call.  Output CCS strings live in a context-owned arena, valid until the
 * next ccsx_gpu_run / ccsx_gpu_fetch on the same context.
 * Errors: every function returns 0 on success, < 0 on error; the message is
 * ccsx_gpu_error(ctx).  -1 is a context error (allocation, launch): the
 * context's results are void.  ccsx_gpu_run / ccsx_gpu_fetch return -2 when
 * individual ZMWs failed on the device (out[i].status != 0, no CCS); every
 * other ZMW of the call is valid, and the host program skips only the failed
 * ones (the reference has no per-ZMW failure to mirror).
 * Threading: one context per device; a context is used by one host thread.
 */
#ifndef CCSX_GPU_H
#define CCSX_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ccsx_ctx ccsx_ctx;

enum { CCSX_MODE_SHRED = 0, CCSX_MODE_PRIMITIVE = 1 };

typedef struct {
    const char *seqs;         /* the ZMW's bases (ASCII), segments are slices of it */
    const uint32_t *seg_off;  /* nseg offsets into seqs, in push order */
    const uint32_t *seg_len;  /* nseg lengths */
    uint32_t nseg;
} ccsx_zmw_in;

typedef struct {
    const char *ccs;          /* ASCII CCS (not NUL-terminated), ctx-owned */
    uint32_t len;             /* 0 = no CCS (main.c:713 writes nothing) */
    int32_t status;           /* 0 ok; see ccsx_gpu_status_str */
    uint64_t cells;           /* DP cells computed for this ZMW */
} ccsx_zmw_out;

/* Number of HIP devices visible to this process (0 if none). */
int ccsx_gpu_device_count(void);

/* Open a context on HIP device `device`. */
int ccsx_gpu_open(int device, ccsx_ctx **ctx);
void ccsx_gpu_close(ccsx_ctx *ctx);
const char *ccsx_gpu_error(const ccsx_ctx *ctx);
const char *ccsx_gpu_status_str(int32_t status);

/* One chunk (replaces kt_for(ccs_for2/ccs_for)): stage + launch + fetch, in
 * slices that fit the device memory; a ZMW whose graph outgrows the default
 * (tight) workspace capacities is re-run with exact upper-bound capacities.
 * Returns 0, -2 (some ZMWs failed, see out[i].status) or -1. */
int ccsx_gpu_run(ccsx_ctx *ctx, int mode, const ccsx_zmw_in *z, size_t nz, ccsx_zmw_out *out);

/* Pipelined batches (the host program's step 1): ccsx_gpu_submit stages a
 * batch that fits one slot into a free slot of the context's two and launches
 * it without waiting; ccsx_gpu_collect waits for that slot's batch and
 * returns its results (ZMWs that outgrew a tight cap re-run with full caps
 * inside the collect).  Submitting the next batch before collecting the
 * previous keeps the device fed.  *slot: the ticket to collect.  The
 * caller's input arrays must stay valid until the collect; out[i].ccs is
 * valid until that slot's next collect.  submit returns -3 when both slots
 * hold uncollected batches and -4 when the batch does not fit one slot
 * (ccsx_gpu_slot_bytes; or mixes launch classes): run it with ccsx_gpu_run
 * once the submitted batches are collected (ccsx_gpu_run drops uncollected
 * ones).  collect returns 0, -2 (some ZMWs failed) or -1. */
int ccsx_gpu_slot_bytes(ccsx_ctx *ctx, uint64_t *bytes);
/* Reserve the pinned host staging (subreads, CCS; exactly these sizes) of
 * the slot the next submit takes, e.g. on a worker thread while the first
 * batch is still being read, instead of in that batch's staging (huge-page
 * mapping, touch, registration: ~0.1 s per GB).  The other slot's is sized by
 * its first batch, while the first one's kernel runs. */
int ccsx_gpu_reserve_staging(ccsx_ctx *ctx, uint64_t seq_bytes, uint64_t out_bytes);
int ccsx_gpu_submit(ccsx_ctx *ctx, int mode, const ccsx_zmw_in *z, size_t nz, int *slot);
int ccsx_gpu_collect(ccsx_ctx *ctx, int slot, ccsx_zmw_out *out);

/* Contexts sharing one device concurrently (the CLI keeps two chunks in flight
 * per GPU): cap this context's slices at total device memory / share
 * (default 1 = whatever is free). */
int ccsx_gpu_set_mem_share(ccsx_ctx *ctx, uint32_t share);
/* The fraction of the device memory all contexts sharing it may use together
 * (default 0.5; 0.05 < frac <= 0.95): each context's slices are sized from
 * total memory x frac / share, split over its two slots. */
int ccsx_gpu_set_mem_frac(ccsx_ctx *ctx, float frac);
/* on != 0: the first ccsx_gpu_run reserves the whole slice budget for the
 * workspace at once instead of growing it with the chunk size (re-allocating
 * a workspace a launch has touched costs ~30 ms per GB; a fresh one does
 * not).  For long runs such as the CLI's growing chunks. */
int ccsx_gpu_set_prealloc(ccsx_ctx *ctx, int on);

/* -v >= 3 (main.c:619-620): on != 0 makes the following ccsx_gpu_run calls
 * (shredded mode) record, per ZMW and shredding round, the breakpoint i and
 * the MSA's column count (msaidxs->size) that ccs_for2 prints.
 * ccsx_gpu_bp_log: the log of ZMW `zmw` (index into the last ccsx_gpu_run's
 * batch) as nrounds (i, ncols) pairs, ctx-owned until the next run. */
int ccsx_gpu_set_bp_log(ccsx_ctx *ctx, int on);
int ccsx_gpu_bp_log(const ccsx_ctx *ctx, size_t zmw, const uint32_t **pairs, uint32_t *nrounds);
/* The same in three steps (one slice, tight capacities, no re-run), so inputs
 * can stay resident in HBM across launches (used by bench.py).
 * ccsx_gpu_launch returns the kernel time measured with HIP events on the
 * context's stream. */
int ccsx_gpu_stage(ccsx_ctx *ctx, const ccsx_zmw_in *z, size_t nz);
/* ccsx_gpu_stage with the tight capacities ccsx_gpu_run uses for `mode`
 * (shredded: workspaces and the LDS read buffer sized for the pushed windows,
 * not whole segments), so a staged slice runs the same kernel instance a
 * ccsx_gpu_run slice would. */
int ccsx_gpu_stage_for(ccsx_ctx *ctx, int mode, const ccsx_zmw_in *z, size_t nz);
int ccsx_gpu_launch(ccsx_ctx *ctx, int mode, float *kernel_ms);
int ccsx_gpu_fetch(ccsx_ctx *ctx, ccsx_zmw_out *out);

/* Device bytes the staged batch occupies (workspace + arenas). */
uint64_t ccsx_gpu_staged_bytes(const ccsx_ctx *ctx);

/* Diagnostics: per-phase shader-clock counters (s_memtime) summed over the
 * ZMWs of the last launch: total, read staging, DP, traceback, merge,
 * columns, breakpoint+emission, DP rows.  Off by default.  Only the
 * diagnostic library (libccsx_amd_diag.so) carries the counters: with the
 * product library, turning them on returns -1 (ccsx_gpu_error says why). */
int ccsx_gpu_set_profiling(ccsx_ctx *ctx, int on);
/* Test hook: tight row capacity override (0 = default 3 x longest segment +
 * 4096, the segment capped at the 4,096-base window read buffer in shredded
 * mode). */
int ccsx_gpu_set_tight_rows(ccsx_ctx *ctx, uint32_t rows);
/* Test hook: tight output slab override in bytes (0 = default 2 x longest
 * segment + 1,024; a consensus beyond it re-runs the ZMW with full caps). */
int ccsx_gpu_set_tight_out(ccsx_ctx *ctx, uint32_t bytes);
/* Test hook: tight far slot record rows (0 = default rcap / 16 + 64; a DP
 * meeting more far rows -- more than four predecessors or one beyond the
 * ring -- re-runs the ZMW with full caps, a record per row). */
int ccsx_gpu_set_tight_far(ccsx_ctx *ctx, uint32_t rows);
/* Test hook: half size of the piecewise subread staging (0 = 64 MiB) that a
 * preallocating context sharing its device (ccsx_gpu_set_prealloc,
 * ccsx_gpu_set_mem_share > 1: the CLI's) uses for slices larger than two
 * halves: 128 MiB pinned per slot instead of the whole slice. */
int ccsx_gpu_set_stage_piece(ccsx_ctx *ctx, uint64_t bytes);
/* Kernel configuration of the next slices: -1 (default) = by slice size (the
 * latency configuration 0 -- three waves, 8-row DP blocks, 32-row LDS ring --
 * when it keeps the whole slice resident; for slices of at least 3x what the
 * occupancy one keeps resident a one-wave-per-ZMW configuration with an int16
 * ring: 5 (solo16w, 24 per CU) when the slice's ZMWs average fewer than 16
 * segments, else 4 (solo16, 20 per CU), or 3 (solo, int32 ring) where a
 * pushed read exceeds 16,256 bases or the slice runs the HBM-read instance;
 * else the occupancy configuration 1 -- 4-row blocks, 24-row ring); 0 .. 5
 * force one (2: the throughput configuration, two-wave workgroups, up to 8
 * per CU, only by this call; a forced 4 / 5 the int16 ring cannot take runs 3).
 * ccsx_gpu_kernel_cfg: the configuration of the last staged slice. */
int ccsx_gpu_set_kernel_cfg(ccsx_ctx *ctx, int cfg);
int ccsx_gpu_kernel_cfg(const ccsx_ctx *ctx);
/* ZMWs ccsx_gpu_run has re-run with full caps on this context so far. */
int64_t ccsx_gpu_rerun_count(const ccsx_ctx *ctx);
/* Counters of this context's ccsx_gpu_run calls so far, the first n of:
 * [0] ZMWs re-run with full caps, [1] slices launched, [2] ZMW lists dealt
 * into interleaved parts (a list of one launch class that needs k > 1 slots),
 * [3] the parts of those lists, [4] slices that waited for device memory a
 * neighbour still held, [5] slices cut below the plan to the free memory. */
int ccsx_gpu_run_stats(const ccsx_ctx *ctx, uint64_t *stats, uint32_t n);
/* How long a slice waits for device memory that another context or a just
 * exited process still holds before the call fails (default 60,000 ms).
 * ccsx_gpu_run first cuts its slices to the free memory, then waits only if
 * not even one ZMW fits; a ccsx_gpu_submit batch waits for its whole size. */
int ccsx_gpu_set_mem_wait(ccsx_ctx *ctx, uint32_t ms);
/* Device bytes ZMW *z occupies in a ccsx_gpu_run slice of `mode` (tight
 * capacities: workspace, subreads, output slab, tables). */
uint64_t ccsx_gpu_zmw_bytes(const ccsx_ctx *ctx, int mode, const ccsx_zmw_in *z);
/* Test hook: bytes per slot for ccsx_gpu_run's slices (0 = by device memory:
 * half of this context's share, ccsx_gpu_set_mem_share), so a small batch is
 * cut into several slices. */
int ccsx_gpu_set_slot_budget(ccsx_ctx *ctx, uint64_t bytes);
/* Measurement hooks (the host program maps CCSX_WG_PER_CU / CCSX_SHRED_READ_CAP
 * onto them): pad the LDS request so at most wg_per_cu workgroups share a CU
 * (0 = off); the LDS read buffer of tight-cap shredded slices in bases
 * (1,024-65,536, default 4,096; a longer pushed window re-runs the ZMW with
 * full caps). */
int ccsx_gpu_set_wg_cap(ccsx_ctx *ctx, uint32_t wg_per_cu);
int ccsx_gpu_set_shred_read_cap(ccsx_ctx *ctx, uint32_t bases);
/* Test hook: the next ccsx_gpu_run reports ZMW `zmw` (index into its batch)
 * as failed (status 8) after computing it, as a device failure would; the
 * run returns -2 and the other ZMWs are valid.  -1 = off. */
int ccsx_gpu_set_fault(ccsx_ctx *ctx, int64_t zmw);
int ccsx_gpu_profile(ccsx_ctx *ctx, uint64_t *sums, uint32_t nslots);
/* Diagnostics: the same counters per ZMW (staging order), nslots per ZMW;
 * out holds nzmw * nslots values. */
int ccsx_gpu_profile_zmw(ccsx_ctx *ctx, uint64_t *out, uint32_t nzmw, uint32_t nslots);

#ifdef __cplusplus
}
#endif
#endif
