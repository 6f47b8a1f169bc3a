// Damped inverse-Cholesky of Kronecker factors (KFAC.invert) on gfx950, fp64.
//
// Replaces models/curvatures.py:374-398:
//   R = sqrt(s) F + sqrt(n) I ; R = (R + R^T)/2 ; L = cholesky(inverse(R))
// without forming R^{-1}.  With P the exchange (flip) matrix:
//   C = chol(P R P) (lower),  X = C^{-1} (lower),  L = P X^T P
// satisfies L L^T = R^{-1}, L lower with a positive diagonal (= the unique
// Cholesky factor of R^{-1}).  One potrf whose elimination also yields the
// inverse, instead of getrf/getri + potrf; all arithmetic in fp64 (cond(R)
// reaches ~1e5 on the MLP).
//
// Blocked over 64x64 fp64 tiles; every launch is grouped over ALL factors:
//   inv_step(-1)    build R' = P R P (damped, symmetrised, identity padded), Z = 0,
//                   info = 0; its workgroup 0 factors tile (0,0): X[0][0] = chol^{-1}
//   for k = 0..T-1: inv_step(k), ONE launch per step, the panel folded in:
//                   C_i = R'[i][k] X[k][k]^T formed where needed (never stored)
//                   R'[i][j] -= C_i C_j^T                 (i >= j > k)
//                   Z[i][j]  -= C_i X[k][k] Z[k][j]        (i > k >= j)
//                   X[k][j]   = X[k][k] Z[k][j] -> W[k][j] (final, j < k)
//                   and the block owning (k+1,k+1) factors it right after its
//                   update -> X[k+1][k+1] (one factorisation per step).
//   [inv_xtx]       Y = X^T X (only for the full-inverse output)
//   L[i][j] = X[n-1-j][n-1-i] (fp32) is written by the step that finalises each X
//   tile (upper zero blocks by step -1): no separate output pass.  The full-inverse
//   output (R^{-1} = P Y P) and the two-launch path (below) keep inv_out.
// Z (the partially eliminated identity) lives in X's lower tiles.  Tile GEMMs
// use v_mfma_f64_16x16x4_f64; the 64x64 diagonal factorisation is blocked by 16
// (one wave eliminates each 16x16 diagonal block, MFMA for the rest).
#include <math.h>

#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "kfac_common.h"

namespace kfac {
namespace t64 {  // 64x64 fp64 tiles: the two-launch path of large factors (> 1536)
constexpr int NB = 64;
constexpr int MERGE_T = 24;
#include "invert_tiles.inc"
}  // namespace t64
namespace t32 {  // 32x32 fp64 tiles: latency-bound factors (<= 1536), see below
constexpr int NB = 32;
constexpr int MERGE_T = 48;
#include "invert_tiles.inc"
}  // namespace t32
}  // namespace kfac


using namespace kfac;

// Tile edge of a call: 32x32 fp64 tiles when every factor is at most 1536 (the merged
// one-launch steps: latency-bound, and a 32-tile workgroup needs 29 KB of LDS, so it
// fits on a CU beside the 4 resident workgroups of a running SYRK launch, which leave
// 32 KB: the inversion overlaps the next data pass instead of waiting for its
// launches to drain); 64x64 tiles for larger factors (throughput-bound two-launch
// steps).
static bool small_tiles(const kfac_invert_job* jobs, int njobs) {
  int m = 0;
  for (int i = 0; i < njobs; ++i) m = std::max(m, (int)jobs[i].n);
  return m <= 1536;
}

static size_t job_ws(const kfac_invert_job& j, bool small) {
  return small ? t32::job_ws(j) : t64::job_ws(j);
}

// every job has its own region (the groups' F-reading launches all run first)
extern "C" size_t kfac_invert_workspace_bytes(const kfac_invert_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  const bool small = small_tiles(jobs, njobs);
  size_t tot = 0;
  for (int i = 0; i < njobs; ++i) tot += job_ws(jobs[i], small);
  return tot;
}

static int check_jobs(const kfac_invert_job* jobs, int njobs) {
  if (njobs <= 0 || !jobs) return KFAC_EINVAL;
  for (int i = 0; i < njobs; ++i) {
    const kfac_invert_job& j = jobs[i];
    if (!j.F || !j.out || j.n <= 0 || j.ldF < j.n || j.ldo < j.n ||
        (j.out_kind != KFAC_OUT_INV_CHOL && j.out_kind != KFAC_OUT_INVERSE))
      return KFAC_EINVAL;
    if (j.n > 65536) return KFAC_EINVAL;
  }
  return KFAC_OK;
}

// phase 0: every group's F-reading launch; phase 1: the rest
static int invert_phase(const kfac_invert_job* jobs, int njobs, void* workspace, int32_t* info,
                        hipStream_t stream, int phase) {
  const bool small = small_tiles(jobs, njobs);
  constexpr int IMAXJ = t64::IMAXJ;
  static_assert(t32::IMAXJ == t64::IMAXJ, "group size");
  char* ws = (char*)workspace;
  for (int g = 0; g < njobs; g += IMAXJ) {
    const int ng = std::min(IMAXJ, njobs - g);
    int32_t* inf = info ? info + g : nullptr;
    const int rc = small ? t32::invert_group(jobs + g, ng, ws, inf, stream, phase)
                         : t64::invert_group(jobs + g, ng, ws, inf, stream, phase);
    if (rc) return rc;
    for (int i = g; i < g + ng; ++i) ws += job_ws(jobs[i], small);
  }
  return KFAC_OK;
}

extern "C" int kfac_invert_ex(const kfac_invert_job* jobs, int njobs, void* workspace,
                              size_t workspace_bytes, int32_t* info, void* inputs_read,
                              kfac_stream_t stream) {
  const int rc0 = check_jobs(jobs, njobs);
  if (rc0) return rc0;
  if (workspace_bytes < kfac_invert_workspace_bytes(jobs, njobs)) return KFAC_EWORKSPACE;
  ProfScope ps(KFAC_PROF_INVERT, (hipStream_t)stream);
  // every group's F-reading launch first, then the event, then the rest
  for (int phase = 0; phase < 2; ++phase) {
    const int rc = invert_phase(jobs, njobs, workspace, info, (hipStream_t)stream, phase);
    if (rc) return rc;
    if (phase == 0 && inputs_read &&
        hipEventRecord((hipEvent_t)inputs_read, (hipStream_t)stream) != hipSuccess)
      return KFAC_ELAUNCH;
  }
  return KFAC_OK;
}

// The overlapped inversion's whole host sequence in one call (KFAC.invert beside the
// next data pass): order `side` after `main`'s current work (event `order`), the grouped
// inversion on `side` with `inputs_read` recorded after its F-reading launch, the pivot
// verdict copied to pinned host memory, `done` recorded.  In Python the same sequence was
// ~10 torch.cuda calls (stream / event objects, the stream context, a non-blocking
// copy), ~100 us of the caller's thread per inversion on the bench host.
extern "C" int kfac_invert_pipelined(const kfac_invert_job* jobs, int njobs, void* workspace,
                                     size_t workspace_bytes, int32_t* info, int32_t* info_host,
                                     void* order, void* inputs_read, void* done, kfac_stream_t main,
                                     kfac_stream_t side) {
  if (!info || !info_host || !order || !done || njobs <= 0) return KFAC_EINVAL;
  if (hipEventRecord((hipEvent_t)order, (hipStream_t)main) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)side, (hipEvent_t)order, 0) != hipSuccess)
    return KFAC_ELAUNCH;
  const int rc = kfac_invert_ex(jobs, njobs, workspace, workspace_bytes, info, inputs_read, side);
  if (rc) return rc;
  if (hipMemcpyAsync(info_host, info, (size_t)njobs * sizeof(int32_t), hipMemcpyDeviceToHost,
                     (hipStream_t)side) != hipSuccess ||
      hipEventRecord((hipEvent_t)done, (hipStream_t)side) != hipSuccess)
    return KFAC_ELAUNCH;
  return KFAC_OK;
}

extern "C" int kfac_invert(const kfac_invert_job* jobs, int njobs, void* workspace,
                           size_t workspace_bytes, int32_t* info, kfac_stream_t stream) {
  return kfac_invert_ex(jobs, njobs, workspace, workspace_bytes, info, nullptr, stream);
}

// the inversion's cached hipGraphs (both tile sizes); see kfac_release (capi.hip)
int kfac_release_graphs() {
  t64::release_graphs();
  t32::release_graphs();
  t64::release_look_ahead();
  t32::release_look_ahead();
  return KFAC_OK;
}


extern "C" int kfac_damped_inv_chol(const float* F, int n, int64_t ldF, double sqrt_s, double sqrt_n,
                                    float* L, int64_t ldL, void* workspace, size_t workspace_bytes,
                                    int32_t* info, kfac_stream_t stream) {
  kfac_invert_job j{};
  j.F = F;
  j.ldF = ldF;
  j.n = n;
  j.out_kind = KFAC_OUT_INV_CHOL;
  j.scale = sqrt_s;
  j.shift = sqrt_n;
  j.out = L;
  j.ldo = ldL;
  return kfac_invert(&j, 1, workspace, workspace_bytes, info, stream);
}
