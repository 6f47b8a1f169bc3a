/*
 * kfac_hip.h — C ABI of the MI355X (gfx950) KFAC curvature engine.
 *
 * Plain pointers and sizes only (no torch types): every buffer is device memory
 * owned by the caller, every call is asynchronous on the given HIP stream
 * (passed as an opaque `void*` = hipStream_t) and does no implicit sync, no
 * allocation and no host<->device copy of data, so calls can be captured into a
 * HIP graph.  Return value: 0 = launched, <0 = bad argument / launch failure
 * (kfac_strerror).  Numerical failure (a non-positive pivot) is reported in a
 * DEVICE int array `info`, LAPACK style, for the caller to read when it syncs.
 *
 * Each entry point names the reference interface it replaces
 * (paths under TianmingQiu/BNN_KFAC).  The Python binding (ctypes) lives in
 * bnn_kfac_amd/_native.py; INTEGRATION.md shows the binding a maintainer of the
 * reference would add.
 */
#ifndef KFAC_HIP_H
#define KFAC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#define KFAC_API __attribute__((visibility("default")))
#else
#define KFAC_API
#endif

typedef void* kfac_stream_t; /* hipStream_t */

enum kfac_status {
  KFAC_OK = 0,
  KFAC_EINVAL = -1,     /* bad argument (null pointer, bad shape, bad layout) */
  KFAC_ELAUNCH = -2,    /* a HIP launch failed */
  KFAC_EWORKSPACE = -3, /* workspace too small */
};

/* ------------------------------------------------------------------ factors
 * F = beta * F + alpha * X~^T X~, X~ = [X | 1] (ones column iff has_ones),
 * X the (rows x cols) input whose element (k, i) is addressed per `layout`:
 *   KFAC_ROWMAJOR: ptr[k*ld + i]                     (Linear a, Linear g_rec)
 *   KFAC_CHANNEL : ptr[(k/L)*sB + (k%L) + i*L]        (Conv2d g_rec (B,C,Ho*Wo))
 *   KFAC_PATCH   : implicit im2col of x (B,C,H,W):   k = b*L + oh*Wo + ow,
 *                  i = c*kh*kw + ki*kw + kj  ->  x[b, c, oh*sh+ki-ph, ow*sw+kj-pw]
 *                  (0 outside the image)           (Conv2d a, F.unfold order)
 * F is n x n row-major with n = cols + has_ones, written exactly symmetric.
 * Replaces models/curvatures.py:341-363 (unfold/permute + the two torch.mm
 * calls + the per-batch-mean `/ float(cols)` + the `+=` accumulation).     */
enum kfac_layout { KFAC_ROWMAJOR = 0, KFAC_CHANNEL = 1, KFAC_PATCH = 2 };

typedef struct kfac_operand {
  const float* ptr;
  int32_t layout;
  int32_t cols;
  int64_t rows;
  int32_t has_ones;
  /* Multi-batch ROWMAJOR job (nseg > 1): rows of its LAST batch when that batch is
   * shorter than `rows` (a pass's ragged last batch), 0 = every batch has `rows`.
   * That batch enters with its own per-batch mean, alpha * rows / last_rows (the
   * reference's `/ forward.shape[1]` per update, curvatures.py:349,356); the other
   * batches with alpha.                                                       */
  int32_t last_rows;
  int64_t ld;  /* ROWMAJOR row stride (elements) */
  int64_t L;   /* CHANNEL/PATCH: positions per sample (Ho*Wo) */
  int64_t sB;  /* CHANNEL/PATCH: sample stride (elements) */
  int32_t C, H, W, kh, kw, sh, sw, ph, pw, Ho, Wo, reserved1; /* PATCH geometry */
} kfac_operand;

typedef struct kfac_factor_job {
  kfac_operand x;
  float alpha; /* 1/cols = per-batch mean (curvatures.py:349,356); 1/B_global when sharded */
  float beta;  /* 0 = first update assigns, 1 = later updates add (curvatures.py:359-363) */
  float* F;
  int64_t ldF;
  /* Optional deferred reduction (NULL = reduce into F in this call).  With `acc`
   * set, kfac_factor_update leaves F alone and keeps this factor's split-K partial
   * tiles in the caller's accumulator instead:  acc = acc_beta*acc + alpha*partial
   * (acc_beta 0 on the first update after a flush, 1 after).  kfac_factor_flush
   * then writes F = beta*F + alpha*sum(acc) once, e.g. at the end of a data pass,
   * so a pass of U updates runs U MFMA launches + 1 reduce instead of U + U.
   * acc_splits and the size come from kfac_factor_accum_plan; F = sum of the
   * partials either way (floating-point summation order differs).            */
  float* acc;
  int32_t acc_splits;
  float acc_beta;
  /* Optional multi-batch job (nseg > 1): the update covers nseg batches of x's
   * shape at once, F += alpha * sum_s X_s~^T X_s~, X_s the operand x with
   * ptr = seg_ptrs[s].  seg_ptrs is a HOST array of nseg device pointers, read
   * during the call and passed to the kernel as launch arguments (no copy, no
   * device table; graph-capturable); every base must share x.ptr's alignment
   * modulo 16 bytes.  One launch then walks K across the batches in place
   * (K = nseg * x.rows, up to 64 bases per launch, more run as back-to-back
   * launches), so a pass of U equal batches costs about one MFMA launch instead
   * of U.  Equivalent to nseg jobs with the same alpha (the reference's per-batch
   * mean over equal batches).  nseg 0 or 1 = the single batch at x.ptr.  Every
   * layout: a KFAC_PATCH / KFAC_CHANNEL job's images are the nseg batches' B
   * images each, in order (one launch per conv factor for the queued batches when
   * an image fits the LDS-staged kernel; else one launch per batch).           */
  const void* seg_ptrs;
  int32_t nseg;
  /* Deferred reduction, several jobs of one factor in ONE call (e.g. a pass's full
   * batches as one multi-batch job and its short last batch as another): slabs per
   * tile of the accumulator `acc` points into, 0 = acc_splits.  Each job owns its
   * own slab range [s0, s0 + acc_splits) of an accumulator of acc_stride slabs per
   * tile and passes acc = base + s0 * 64*64*sizeof(float) bytes (ranges must not
   * overlap); kfac_factor_flush then takes acc = base, acc_splits = acc_stride =
   * the total.  kfac_factor_accum_plan's bytes are linear in the splits, so the
   * accumulator of such a factor is the sum of its jobs' planned bytes.          */
  int32_t acc_stride;
} kfac_factor_job;

/* Workspace (split-K slabs) needed by kfac_factor_update for these jobs. */
KFAC_API size_t kfac_factor_workspace_bytes(const kfac_factor_job* jobs, int njobs);
/* All jobs of one KFAC.update() in one grouped MFMA launch + one reduce launch.
 * Replaces KFAC.update, models/curvatures.py:325-365. */
KFAC_API int kfac_factor_update(const kfac_factor_job* jobs, int njobs, void* workspace,
                       size_t workspace_bytes, kfac_stream_t stream);

/* Accumulator layout for these jobs (acc ignored): splits[j] and bytes[j] of job
 * j's deferred-reduction accumulator, planned for this batch shape (later
 * batches of any row count may use it).                                    */
KFAC_API int kfac_factor_accum_plan(const kfac_factor_job* jobs, int njobs, int32_t* splits,
                           size_t* bytes);
/* F = beta*F + alpha*sum(acc) for every job (all must carry acc): the reduce
 * step of kfac_factor_update, deferred (x is only read for the factor size). */
KFAC_API int kfac_factor_flush(const kfac_factor_job* jobs, int njobs, kfac_stream_t stream);

/* Single-factor conveniences (same kernels). */
KFAC_API int kfac_syrk_linear(const float* x, int64_t B, int64_t d, int64_t ldx, int has_ones,
                     float alpha, float beta, float* F, int64_t ldF, void* workspace,
                     size_t workspace_bytes, kfac_stream_t stream);
KFAC_API int kfac_syrk_conv(const float* x, int64_t B, int C, int H, int W, int kh, int kw, int sh,
                   int sw, int ph, int pw, int has_ones, float alpha, float beta, float* F,
                   int64_t ldF, void* workspace, size_t workspace_bytes, kfac_stream_t stream);
KFAC_API int kfac_syrk_convgrad(const float* g, int64_t B, int C, int64_t L, float alpha, float beta,
                       float* F, int64_t ldF, void* workspace, size_t workspace_bytes,
                       kfac_stream_t stream);

/* ---------------------------------------------------------------- inversion
 * R = scale * (F + F^T)/2 + shift * I, computed in fp64 on the device, then
 *   KFAC_OUT_INV_CHOL: out = L, lower, L L^T = R^{-1}   (= cholesky(inverse(R)))
 *   KFAC_OUT_INVERSE : out = R^{-1} (full, symmetric)
 * via C = chol(P R P) (P the exchange matrix), X = C^{-1}, L = P X^T P.
 * KFAC.invert passes scale = sqrt(multiply), shift = sqrt(add)
 * (models/curvatures.py:367-398); the regression block passes scale = N,
 * shift = N*tau with KFAC_OUT_INVERSE (regression_ll_block.py:130-133).
 * info[j] (device) = 0, or the 1-based index of the first non-positive pivot
 * of job j (the reference's RuntimeError / LinAlgError condition).          */
enum kfac_inv_out { KFAC_OUT_INV_CHOL = 0, KFAC_OUT_INVERSE = 1 };

typedef struct kfac_invert_job {
  const float* F;
  int64_t ldF;
  int32_t n;
  int32_t out_kind;
  double scale;
  double shift;
  float* out;
  int64_t ldo;
} kfac_invert_job;

KFAC_API size_t kfac_invert_workspace_bytes(const kfac_invert_job* jobs, int njobs);
KFAC_API int kfac_invert(const kfac_invert_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
                int32_t* info, kfac_stream_t stream);
/* kfac_invert that also signals when the inputs are consumed: `inputs_read` (a
 * hipEvent_t, may be NULL) is recorded on `stream` right after the launches that
 * read the F factors (the first of each job group: R' is built from F there), so
 * the caller may overwrite F (e.g. accumulate the next data pass) once the event
 * completes while the rest of the inversion still runs.  Same results as
 * kfac_invert.                                                               */
KFAC_API int kfac_invert_ex(const kfac_invert_job* jobs, int njobs, void* workspace,
                   size_t workspace_bytes, int32_t* info, void* inputs_read, kfac_stream_t stream);
/* Single-factor convenience: KFAC.invert for one factor. */
KFAC_API int kfac_damped_inv_chol(const float* F, int n, int64_t ldF, double sqrt_s, double sqrt_n,
                         float* L, int64_t ldL, void* workspace, size_t workspace_bytes,
                         int32_t* info, kfac_stream_t stream);

/* ------------------------------------------------------------ eigenvalues
 * Symmetric eigendecomposition of (F + F^T)/2 (fp64 on device): evals ascending
 * (torch.symeig / eigvalsh order), evecs (optional, may be NULL) as columns,
 * row-major n x n fp32.  Replaces models/utilities.py:120-159.           */
typedef struct kfac_eig_job {
  const float* F;
  int64_t ldF;
  int32_t n;
  int32_t reserved;
  double* evals;
  float* evecs;
  int64_t ldv;
} kfac_eig_job;

KFAC_API size_t kfac_eig_workspace_bytes(const kfac_eig_job* jobs, int njobs);
KFAC_API int kfac_syev(const kfac_eig_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
              int32_t* info, kfac_stream_t stream);

/* ------------------------------------------------- predictive variance
 * v[j][b] = J_jb kron(K1_j, K2_j) J_jb^T without forming the Kronecker product:
 * with M = J_jb viewed (nA x nG) row-major (the reference's flat order
 * a*nG + g), v = <K1^T M, M K2^T>_F.  K1/K2 may be flagged lower-triangular
 * (Cholesky factors) to skip their zero blocks.
 * out[b] = sum_j |v[j][b]| if abs_sum else sum_j v[j][b].
 * Replaces classification_ll_block.py:126-132 (torch.kron + J H J^T) and
 * regression_ll_block.py:128-139 (kronecker_product + J H J^T).          */
typedef struct kfac_quad_job {
  const float* J;
  int64_t ldJ; /* stride between the nb rows of J (elements) */
  int32_t nA, nG;
  const float* K1;
  int64_t ld1;
  const float* K2;
  int64_t ld2;
  int32_t lower1, lower2;
  float* v; /* optional (may be NULL): nb raw values for this job */
} kfac_quad_job;

KFAC_API size_t kfac_quadform_workspace_bytes(const kfac_quad_job* jobs, int njobs, int64_t nb);
KFAC_API int kfac_kron_quadform(const kfac_quad_job* jobs, int njobs, int64_t nb, int abs_sum, float* out,
                       void* workspace, size_t workspace_bytes, kfac_stream_t stream);

/* -------------------------------------------------------- posterior samples
 * out_j = (LA_j Z_j LG_j^T)^T, shape (nG x nA): KFAC.sample, curvatures.py:400-405,
 * with Z (nA x nG row-major) supplied by the caller (torch.randn, the reference's
 * draw).  LA/LG are lower-triangular with zero upper triangles (KFAC.invert's
 * factors): tiles above the diagonal are skipped.  Columns a < wcols go to W[g*ldW + a]; when wcols == nA-1 column
 * nA-1 goes to bias[g] (Curvature._replace, curvatures.py:68-82; bias may be NULL
 * to drop it).  accumulate: W += sample (sample_and_replace) else W = sample.
 * At most 8 jobs per call.                                                    */
typedef struct kfac_sample_job {
  const float* LA;
  int64_t ldA;
  const float* LG;
  int64_t ldG;
  const float* Z;
  int32_t nA, nG;
  float* W;
  int64_t ldW;
  float* bias;
  int32_t wcols;
  int32_t dense; /* 1: LA/LG are full matrices (EFB eigenvectors, curvatures.py:466-473) */
} kfac_sample_job;

KFAC_API size_t kfac_sample_workspace_bytes(const kfac_sample_job* jobs, int njobs);
KFAC_API int kfac_sample(const kfac_sample_job* jobs, int njobs, int accumulate, void* workspace,
                size_t workspace_bytes, kfac_stream_t stream);

/* ------------------------------------------------ eigenbasis curvatures
 * kfac_efb_update: EFB.update (models/curvatures.py:427-449) for up to 8 layers:
 *   state = [state +] (VG^T grad VA) ** 2          (nG x nA, elementwise square)
 *   diag  = [diag  +] (grad ** 2) * scale           (scale = batch size; diag may be NULL)
 * grad is the layer's (nG x nA) weight gradient with the bias gradient as its last
 * column; VA (nA x nA) and VG (nG x nG) the factors' eigenvectors (columns).  "+"
 * when accumulate != 0, else the results are written.  Two launches; the projection
 * VG^T grad lives in the workspace (nG x nA floats per layer).                  */
typedef struct kfac_efb_job {
  const float* VA;
  int64_t ldA;
  const float* VG;
  int64_t ldG;
  const float* grad;
  int64_t ld_grad;
  float* state;
  int64_t ld_state;
  float* diag;
  int64_t ld_diag;
  int32_t nA, nG;
  int32_t accumulate;
  float scale;
} kfac_efb_job;

KFAC_API size_t kfac_efb_workspace_bytes(const kfac_efb_job* jobs, int njobs);
KFAC_API int kfac_efb_update(const kfac_efb_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
                             kfac_stream_t stream);

/* kfac_kron_gram: INF.pre_sampler's V_s^T V_s (curvatures.py:548-580), V_s =
 * c * kron(UA, UG) * sigma, without forming V_s ((nA*nG) x (la*lg)):
 *   out[(p*lg+q)*ldo + p2*lg+q2] = sigma[p*lg+q] * sum_{a,g} c[a*nG+g]^2 UA[a][p] UA[a][p2]
 *                                  UG[g][q] UG[g][q2] * sigma[p2*lg+q2]
 * UA (nA x la, ldA), UG (nG x lg, ldG), c (nA*nG), sigma (la*lg).  Symmetric up
 * to one rounding of the sigma scaling.  Workspace: nA x lg^2 floats per job; up
 * to 8 jobs.                                                                    */
typedef struct kfac_gram_job {
  const float* UA;
  int64_t ldA;
  const float* UG;
  int64_t ldG;
  const float* c;
  const float* sigma;
  float* out;
  int64_t ldo;
  int32_t nA, nG, la, lg;
} kfac_gram_job;

KFAC_API size_t kfac_gram_workspace_bytes(const kfac_gram_job* jobs, int njobs);
KFAC_API int kfac_kron_gram(const kfac_gram_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
                            kfac_stream_t stream);

/* ------------------------------------------------- packed lower triangles
 * For the data-parallel collectives (no reference counterpart: the reference is
 * single-device).  Row i of a factor's lower triangle lives at
 * packed[offset + i(i+1)/2 .. + i], so a factor takes n(n+1)/2 floats and the
 * caller lays the factors out back to back.
 *   kfac_tri_pack  : packed <- lower triangles of the F's (the all-reduce of the
 *                    per-rank factor sums, curvatures.py:359-363 summed over ranks)
 *   kfac_tri_unpack: F <- packed, upper triangle mirrored (KFAC_TRI_SYMMETRIC: the
 *                    reduced A, G) or zeroed (KFAC_TRI_LOWER: the L_A, L_G of a
 *                    sharded inversion, curvatures.py:391-398, after the gather). */
enum kfac_tri_mode { KFAC_TRI_SYMMETRIC = 0, KFAC_TRI_LOWER = 1 };

typedef struct kfac_tri_job {
  float* F;
  int64_t ldF;
  int32_t n;
  int32_t reserved;
  int64_t offset; /* elements into `packed` */
} kfac_tri_job;

KFAC_API int kfac_tri_pack(const kfac_tri_job* jobs, int njobs, float* packed, kfac_stream_t stream);
KFAC_API int kfac_tri_unpack(const kfac_tri_job* jobs, int njobs, const float* packed, int mode,
                             kfac_stream_t stream);

/* -------------------------------------------------------------- profiling
 * Optional HIP-event timing of the library's own launches, recorded on the
 * stream each kernel is launched on (off by default; not graph-capturable when
 * on).  One slot per kernel family, named as rocprofv3 names the kernels:
 *   0 kfac_factor_tiles_t (fp32-MFMA SYRK: row-major, LDS-DMA, register-staged conv),
 *   1 kfac_factor_reduce, 2 the whole invert call, 3 kfac_quad tiles,
 *   4 kfac_factor_syrk3 (bf16x3, split in the workgroup; largest n >= 2048),
 *   5 kfac_factor_tiles_x3 (bf16x3, split in registers; largest n >= 256),
 *   6 kfac_factor_conv (image-staged conv factors, both the im2col and the
 *     channel-major operand), 7 kfac_factor_channel_small (channel factors n <= 8),
 *   8 the whole kfac_syev call,
 *   9 kfac_factor_conv_x3 (im2col factors with n > 32, bf16x3 from an LDS im2col),
 *   10 kfac_factor_conv_x3s (im2col factors with 17 <= n <= 32, bf16x3 from
 *     column-shifted image copies),
 *   11 kfac_factor_conv_x3f (stride-1 im2col factors with 32 < n <= 160, bf16x3 from
 *     flattened column copies),
 *   12 kfac_factor_channel_x3 (channel-major factors with 8 < n <= 32, bf16x3 from
 *     fragments loaded straight from HBM).
 * kfac_profile_read syncs the recorded events.  kfac_profile_read_work also
 * returns the slot's algorithmic work: `work` = flops, for the factor slots (0, 4-7, 9-12)
 * sum_jobs K_rows * n (n + 1) (lower triangle incl. the diagonal, 2 flops per
 * product; curvatures.py:341-356); `bytes` = HBM bytes, for the factor slots each
 * operand read once (rows x cols x 4; an im2col operand: its images), for the syev
 * slot the tridiagonalisations' sum_k (n - k)^2 x 16 ~ 16 n^3 / 3 (n > 128). */
enum kfac_prof_id { KFAC_PROF_FACTOR_TILES = 0, KFAC_PROF_FACTOR_REDUCE = 1, KFAC_PROF_INVERT = 2,
                    KFAC_PROF_QUAD_TILES = 3, KFAC_PROF_FACTOR_SYRK3 = 4, KFAC_PROF_FACTOR_X3 = 5,
                    KFAC_PROF_FACTOR_CONV = 6, KFAC_PROF_FACTOR_CHANNEL_SMALL = 7, KFAC_PROF_SYEV = 8,
                    KFAC_PROF_FACTOR_CONV_X3 = 9, KFAC_PROF_FACTOR_CONV_X3S = 10,
                    KFAC_PROF_FACTOR_CONV_X3F = 11, KFAC_PROF_FACTOR_CHANNEL_X3 = 12, KFAC_PROF_COUNT = 13 };
KFAC_API int kfac_profile_enable(int on);
KFAC_API int kfac_profile_read(int id, double* total_ms, int64_t* launches);
KFAC_API int kfac_profile_read_work(int id, double* total_ms, int64_t* launches, double* work,
                                   double* bytes);
KFAC_API int kfac_profile_reset(void);

/* ------------------------------------------------------------------- misc */
/* KFAC.invert beside the next data pass (curvatures.py:367-398, overlapped), one call:
 * record `order` on `main`, make `side` wait for it, run kfac_invert_ex on `side`
 * (`inputs_read` recorded after the F-reading launch, may be NULL), copy the njobs
 * verdicts from `info` (device) to `info_host` (pinned host memory) and record `done`
 * on `side`.  Events come from kfac_event_create. */
KFAC_API int kfac_invert_pipelined(const kfac_invert_job* jobs, int njobs, void* workspace,
                                   size_t workspace_bytes, int32_t* info, int32_t* info_host,
                                   void* order, void* inputs_read, void* done, kfac_stream_t main,
                                   kfac_stream_t side);

/* Raw HIP events for the host side's stream ordering (no reference counterpart: the
 * reference is synchronous).  query: 1 complete, 0 pending, < 0 error. */
KFAC_API int kfac_event_create(void** event);
/* flags bit 0: ordering-only event (no system-scope fence when recorded / waited on):
 * for stream-to-stream order on one device, not for host reads after a sync. */
KFAC_API int kfac_event_create_ex(void** event, int flags);
KFAC_API int kfac_event_destroy(void* event);
KFAC_API int kfac_event_record(void* event, kfac_stream_t stream);
KFAC_API int kfac_stream_wait_event(kfac_stream_t stream, void* event);
KFAC_API int kfac_event_query(void* event);
KFAC_API int kfac_event_synchronize(void* event);

/* Release every HIP object the library keeps across calls (the inversion's cached
 * hipGraphs and their events, the profiling event pool), waiting for their last
 * use first.  Call before the HIP runtime shuts down (the Python binding registers
 * it with atexit); later calls simply rebuild what they need.  No reference
 * counterpart (the reference keeps no device state). */
KFAC_API int kfac_release(void);

/* Environment knobs, read once when the library is loaded.  get: any
 * knob's current value (KFAC_EINVAL for an unknown name).  set: only the per-call ones
 * (KFAC_INV_GRAPH, KFAC_INV_LOOKAHEAD, KFAC_EIG_G, KFAC_EIG_RB), between calls; the
 * kernel-selection knobs (KFAC_SYRK3, KFAC_TILES_X3, KFAC_CONV_*) are fixed at load. */
KFAC_API int kfac_set_knob(const char* name, int value);
KFAC_API int kfac_get_knob(const char* name, int* value);

KFAC_API const char* kfac_strerror(int status);
KFAC_API const char* kfac_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KFAC_HIP_H */
