// Damped inverse-Cholesky of Kronecker factors (KFAC.invert) on gfx950, fp64.
//
// Replaces models/curvatures.py:374-398:
//   R = sqrt(s) F + sqrt(n) I ; R = (R + R^T)/2 ; L = cholesky(inverse(R))
// without forming R^{-1}.  With P the exchange (flip) matrix:
//   C = chol(P R P) (lower),  X = C^{-1} (lower),  L = P X^T P
// satisfies L L^T = R^{-1}, L lower with a positive diagonal (= the unique
// Cholesky factor of R^{-1}).  One potrf + one trtri instead of getrf/getri +
// potrf; all arithmetic in fp64 (cond(R) reaches ~1e5 on the MLP).
//
// Blocked over 64x64 fp64 tiles, every launch grouped over ALL factors:
//   inv_build            R' = P R P (damped, symmetrised, identity padded)
//   for k: inv_panel(k)  factor the diagonal tile in LDS (LDL^T sweep that also
//                        yields its inverse X[k][k]), then L[i][k] = W[i][k] X[k][k]^T
//          inv_update(k) W[i][j] -= L[i][k] L[j][k]^T   (trailing lower tiles)
//   for s = 1,2,4..: inv_trtri1/2 recursive doubling X21 = -X22 (C21 X11)
//   [inv_xtx]            Y = X^T X (only for the full-inverse output)
//   inv_out              L[i][j] = X[n-1-j][n-1-i]  (or R^{-1} = P Y P), fp32
#include <math.h>

#include <algorithm>

#include "kfac_common.h"

namespace kfac {

constexpr int NB = 64;       // fp64 tile edge
constexpr int DP = NB + 1;   // padded pitch (doubles)
constexpr int IMAXJ = 8;

struct InvJobDev {
  const float* F;
  int64_t ldF;
  float* out;
  int64_t ldo;
  double* W;   // Np x Np: R', then the Cholesky factor C (lower tiles)
  double* X;   // Np x Np: C^{-1} (lower tiles)
  double* Tm;  // Np x Np: scratch
  int* info;
  double scale, shift;
  int n, T, Np, kind;
  // per-launch task geometry (filled by the host for the current launch)
  int pairs_full, last_bottom;
};

struct InvArgs {
  int njobs;
  int step;  // k for panel/update, s (tiles per half) for trtri
  int begin[IMAXJ + 1];
  InvJobDev job[IMAXJ];
};

__device__ __forceinline__ int find_job(const InvArgs& a, int task) {
  int j = 0;
  while (j + 1 < a.njobs && task >= a.begin[j + 1]) ++j;
  return j;
}

__device__ __forceinline__ double* tile_ptr(double* base, int Np, int ti, int tj) {
  return base + ((int64_t)ti * NB) * Np + (int64_t)tj * NB;
}

__device__ __forceinline__ void load_tile(double* lds, const double* g, int Np) {
  for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
    const int r = e >> 6, c = e & 63;
    lds[r * DP + c] = g[(int64_t)r * Np + c];
  }
}

__device__ __forceinline__ void store_tile(double* g, const double* lds, int Np) {
  for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
    const int r = e >> 6, c = e & 63;
    g[(int64_t)r * Np + c] = lds[r * DP + c];
  }
}

// ------------------------------------------------------------------- build R'
__global__ __launch_bounds__(NTHREADS) void inv_build(InvArgs args) {
  const int j = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[j];
  int ti, tj;
  tri_decode(blockIdx.x - args.begin[j], ti, tj);
  const int n = J.n;
  for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
    const int i = ti * NB + (e >> 6), c = tj * NB + (e & 63);
    double v;
    if (i < n && c < n) {
      const int fi = n - 1 - i, fc = n - 1 - c;  // flip
      const double sym = 0.5 * ((double)J.F[(int64_t)fi * J.ldF + fc] +
                                (double)J.F[(int64_t)fc * J.ldF + fi]);
      v = J.scale * sym + (i == c ? J.shift : 0.0);
    } else {
      v = (i == c) ? 1.0 : 0.0;  // identity padding keeps the padded block trivial
    }
    J.W[(int64_t)i * J.Np + c] = v;
  }
}

// -------------------------------------------------------------- panel step k
// Every block of the panel factors the (k,k) tile in LDS (cheap, avoids a launch):
// LDL^T sweep with the unit-lower inverse carried along (Gaussian elimination on
// [S | I] gives [D L^T | L_unit^{-1}]), then
//   Lkk = L_unit D^{1/2},  Xkk = D^{-1/2} L_unit^{-1}.
__global__ __launch_bounds__(NTHREADS) void inv_panel(InvArgs args) {
  __shared__ double S[NB * DP];
  __shared__ double Y[NB * DP];
  __shared__ double P[NB * DP];
  __shared__ double dg[NB];
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int k = args.step;
  const int i = k + (blockIdx.x - args.begin[jb]);
  const int tid = threadIdx.x;

  load_tile(S, tile_ptr(J.W, J.Np, k, k), J.Np);
  for (int e = tid; e < NB * NB; e += NTHREADS) Y[(e >> 6) * DP + (e & 63)] = ((e >> 6) == (e & 63)) ? 1.0 : 0.0;
  if (i != k) load_tile(P, tile_ptr(J.W, J.Np, i, k), J.Np);
  __syncthreads();

  const int cc = tid & 63, r0 = tid >> 6;
  for (int jj = 0; jj < NB; ++jj) {
    const double d = S[jj * DP + jj];
    if (tid == 0) dg[jj] = d;
    const double inv = 1.0 / d;
    for (int r = jj + 1 + r0; r < NB; r += 4) {
      if (cc > r) continue;
      const double l = S[r * DP + jj] * inv;
      if (cc <= jj)
        Y[r * DP + cc] -= l * Y[jj * DP + cc];
      else
        S[r * DP + cc] -= l * S[cc * DP + jj];
    }
    __syncthreads();
  }
  // Xkk = D^{-1/2} L_unit^{-1} (zero upper).  The factored diagonal tile itself is
  // never needed again (the panel and the inverse only use Xkk), so W[k][k] is
  // left as is: the other blocks of this launch may still be reading it.
  for (int e = tid; e < NB * NB; e += NTHREADS) {
    const int r = e >> 6, c = e & 63;
    const double xv = (r > c) ? Y[r * DP + c] / sqrt(dg[r]) : (r == c ? 1.0 / sqrt(dg[r]) : 0.0);
    Y[r * DP + c] = xv;
  }
  __syncthreads();
  if (i == k) {
    if (tid == 0 && J.info) {
      for (int c = 0; c < NB; ++c) {
        const int g = k * NB + c;
        if (g < J.n && !(dg[c] > 0.0)) {
          atomicCAS(J.info, 0, g + 1);
          break;
        }
      }
    }
    store_tile(tile_ptr(J.X, J.Np, k, k), Y, J.Np);
    return;
  }
  // L[i][k] = W[i][k] * Xkk^T  (64x64x64 fp64, 4x4 outputs per thread)
  const int tr = tid >> 4, tc = tid & 15;
  double acc[4][4] = {};
  for (int m = 0; m < NB; ++m) {
    double a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = P[(tr * 4 + q) * DP + m];
#pragma unroll
    for (int p = 0; p < 4; ++p) b[p] = Y[(tc * 4 + p) * DP + m];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int p = 0; p < 4; ++p) acc[q][p] += a[q] * b[p];
  }
  double* dst = tile_ptr(J.W, J.Np, i, k);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) dst[(int64_t)(tr * 4 + q) * J.Np + tc * 4 + p] = acc[q][p];
}

// ------------------------------------------------------------- update step k
__global__ __launch_bounds__(NTHREADS) void inv_update(InvArgs args) {
  __shared__ double A[NB * DP];
  __shared__ double B[NB * DP];
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int k = args.step;
  int a, b;
  tri_decode(blockIdx.x - args.begin[jb], a, b);
  const int i = k + 1 + a, jj = k + 1 + b;
  load_tile(A, tile_ptr(J.W, J.Np, i, k), J.Np);
  load_tile(B, tile_ptr(J.W, J.Np, jj, k), J.Np);
  __syncthreads();
  const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  double acc[4][4] = {};
  for (int m = 0; m < NB; ++m) {
    double x[4], y[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = A[(tr * 4 + q) * DP + m];
#pragma unroll
    for (int p = 0; p < 4; ++p) y[p] = B[(tc * 4 + p) * DP + m];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int p = 0; p < 4; ++p) acc[q][p] += x[q] * y[p];
  }
  double* dst = tile_ptr(J.W, J.Np, i, jj);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) dst[(int64_t)(tr * 4 + q) * J.Np + tc * 4 + p] -= acc[q][p];
}

// ------------------------------------------- tile GEMM: C = alpha * sum_m A(.,m) B(m,.)
// transA: A tile (r, m) read as Abase tile (m, r) transposed.
__device__ void tile_gemm_sum(const double* Abase, const double* Bbase, int Np, int ar, int bc,
                              int m0, int m1, bool transA, double alpha, double* C, double* sA,
                              double* sB) {
  const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  double acc[4][4] = {};
  for (int m = m0; m < m1; ++m) {
    if (transA)
      load_tile(sA, Abase + ((int64_t)m * NB) * Np + (int64_t)ar * NB, Np);
    else
      load_tile(sA, Abase + ((int64_t)ar * NB) * Np + (int64_t)m * NB, Np);
    load_tile(sB, Bbase + ((int64_t)m * NB) * Np + (int64_t)bc * NB, Np);
    __syncthreads();
    for (int mm = 0; mm < NB; ++mm) {
      double x[4], y[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        x[q] = transA ? sA[mm * DP + tr * 4 + q] : sA[(tr * 4 + q) * DP + mm];
#pragma unroll
      for (int p = 0; p < 4; ++p) y[p] = sB[mm * DP + tc * 4 + p];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int p = 0; p < 4; ++p) acc[q][p] += x[q] * y[p];
    }
    __syncthreads();
  }
  double* dst = C + ((int64_t)ar * NB) * Np + (int64_t)bc * NB;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) dst[(int64_t)(tr * 4 + q) * Np + tc * 4 + p] = alpha * acc[q][p];
}

// task -> (t0, bottom tile bi, top tile aj) for pair geometry at half-size s
__device__ __forceinline__ void pair_decode(const InvJobDev& J, int s, int local, int& t0, int& bi,
                                            int& aj) {
  const int full = J.pairs_full * s * s;
  int p, rem;
  if (local < full) {
    p = local / (s * s);
    rem = local - p * s * s;
  } else {
    p = J.pairs_full;
    rem = local - full;
  }
  t0 = p * 2 * s;
  bi = t0 + s + rem / s;
  aj = t0 + rem % s;
}

// T1[bi][aj] = sum_{m in top, m >= aj} C[bi][m] X[m][aj]
__global__ __launch_bounds__(NTHREADS) void inv_trtri1(InvArgs args) {
  __shared__ double sA[NB * DP];
  __shared__ double sB[NB * DP];
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int s = args.step;
  int t0, bi, aj;
  pair_decode(J, s, blockIdx.x - args.begin[jb], t0, bi, aj);
  tile_gemm_sum(J.W, J.X, J.Np, bi, aj, aj, t0 + s, false, 1.0, J.Tm, sA, sB);
}

// X[bi][aj] = - sum_{m in bottom, m <= bi} X[bi][m] T1[m][aj]
__global__ __launch_bounds__(NTHREADS) void inv_trtri2(InvArgs args) {
  __shared__ double sA[NB * DP];
  __shared__ double sB[NB * DP];
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int s = args.step;
  int t0, bi, aj;
  pair_decode(J, s, blockIdx.x - args.begin[jb], t0, bi, aj);
  tile_gemm_sum(J.X, J.Tm, J.Np, bi, aj, t0 + s, bi + 1, false, -1.0, J.X, sA, sB);
}

// Y[a][b] = sum_{m >= a} X[m][a]^T X[m][b]   (lower tiles, a >= b)
__global__ __launch_bounds__(NTHREADS) void inv_xtx(InvArgs args) {
  __shared__ double sA[NB * DP];
  __shared__ double sB[NB * DP];
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  int a, b;
  tri_decode(blockIdx.x - args.begin[jb], a, b);
  tile_gemm_sum(J.X, J.X, J.Np, a, b, a, J.T, true, 1.0, J.Tm, sA, sB);
}

// ------------------------------------------------------------------- output
__global__ __launch_bounds__(NTHREADS) void inv_out(InvArgs args) {
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int local = blockIdx.x - args.begin[jb];
  const int ti = local / J.T, tj = local - ti * J.T;
  const int n = J.n;
  for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
    const int i = ti * NB + (e >> 6), c = tj * NB + (e & 63);
    if (i >= n || c >= n) continue;
    double v;
    if (J.kind == KFAC_OUT_INV_CHOL) {
      v = (i >= c) ? J.X[(int64_t)(n - 1 - c) * J.Np + (n - 1 - i)] : 0.0;
    } else {
      const int a = n - 1 - i, b = n - 1 - c;
      v = (a >= b) ? J.Tm[(int64_t)a * J.Np + b] : J.Tm[(int64_t)b * J.Np + a];
    }
    J.out[(int64_t)i * J.ldo + c] = (float)v;
  }
}

// ---------------------------------------------------------------- host side
static size_t job_ws(const kfac_invert_job& j) {
  const int64_t Np = cdiv(j.n, NB) * NB;
  return 3 * align_up((size_t)(Np * Np) * sizeof(double), 256);
}

template <typename Count>
static int launch(void (*kern)(InvArgs), InvArgs& args, Count count, hipStream_t s) {
  int total = 0;
  for (int j = 0; j < args.njobs; ++j) {
    args.begin[j] = total;
    total += count(args.job[j]);
  }
  args.begin[args.njobs] = total;
  if (total == 0) return KFAC_OK;
  hipLaunchKernelGGL(kern, dim3(total), dim3(NTHREADS), 0, s, args);
  KFAC_CHECK_LAUNCH();
  return KFAC_OK;
}

static int invert_group(const kfac_invert_job* jobs, int njobs, char* ws, int32_t* info,
                        hipStream_t s) {
  InvArgs args{};
  args.njobs = njobs;
  int Tmax = 0;
  bool any_inverse = false;
  for (int i = 0; i < njobs; ++i) {
    const kfac_invert_job& jb = jobs[i];
    InvJobDev& d = args.job[i];
    d.F = jb.F;
    d.ldF = jb.ldF;
    d.out = jb.out;
    d.ldo = jb.ldo;
    d.n = jb.n;
    d.T = (int)cdiv(jb.n, NB);
    d.Np = d.T * NB;
    d.kind = jb.out_kind;
    d.scale = jb.scale;
    d.shift = jb.shift;
    d.info = info ? info + i : nullptr;
    const size_t mat = align_up((size_t)d.Np * d.Np * sizeof(double), 256);
    d.W = reinterpret_cast<double*>(ws);
    d.X = reinterpret_cast<double*>(ws + mat);
    d.Tm = reinterpret_cast<double*>(ws + 2 * mat);
    ws += 3 * mat;
    Tmax = std::max(Tmax, d.T);
    any_inverse |= jb.out_kind == KFAC_OUT_INVERSE;
  }
  int rc;
  if (info) {
    if (hipMemsetAsync(info, 0, sizeof(int32_t) * njobs, s) != hipSuccess) return KFAC_ELAUNCH;
  }
  rc = launch(inv_build, args, [](const InvJobDev& d) { return d.T * (d.T + 1) / 2; }, s);
  if (rc) return rc;
  for (int k = 0; k < Tmax; ++k) {
    args.step = k;
    rc = launch(inv_panel, args, [k](const InvJobDev& d) { return k < d.T ? d.T - k : 0; }, s);
    if (rc) return rc;
    rc = launch(inv_update, args,
                [k](const InvJobDev& d) { return k < d.T ? (d.T - k - 1) * (d.T - k) / 2 : 0; }, s);
    if (rc) return rc;
  }
  for (int sz = 1; sz < Tmax; sz *= 2) {
    args.step = sz;
    for (int j = 0; j < njobs; ++j) {
      InvJobDev& d = args.job[j];
      d.pairs_full = d.T / (2 * sz);
      const int rest = d.T - d.pairs_full * 2 * sz;
      d.last_bottom = std::max(0, rest - sz);
    }
    auto count = [sz](const InvJobDev& d) { return d.pairs_full * sz * sz + d.last_bottom * sz; };
    rc = launch(inv_trtri1, args, count, s);
    if (rc) return rc;
    rc = launch(inv_trtri2, args, count, s);
    if (rc) return rc;
  }
  if (any_inverse) {
    rc = launch(inv_xtx, args,
                [](const InvJobDev& d) { return d.kind == KFAC_OUT_INVERSE ? d.T * (d.T + 1) / 2 : 0; }, s);
    if (rc) return rc;
  }
  return launch(inv_out, args, [](const InvJobDev& d) { return d.T * d.T; }, s);
}

}  // namespace kfac

using namespace kfac;

extern "C" size_t kfac_invert_workspace_bytes(const kfac_invert_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  size_t best = 0;
  for (int g = 0; g < njobs; g += IMAXJ) {
    size_t tot = 0;
    for (int i = g; i < std::min(njobs, g + IMAXJ); ++i) tot += job_ws(jobs[i]);
    best = std::max(best, tot);
  }
  return best;
}

extern "C" int kfac_invert(const kfac_invert_job* jobs, int njobs, void* workspace,
                           size_t workspace_bytes, int32_t* info, kfac_stream_t stream) {
  if (njobs <= 0 || !jobs) return KFAC_EINVAL;
  for (int i = 0; i < njobs; ++i) {
    const kfac_invert_job& j = jobs[i];
    if (!j.F || !j.out || j.n <= 0 || j.ldF < j.n || j.ldo < j.n ||
        (j.out_kind != KFAC_OUT_INV_CHOL && j.out_kind != KFAC_OUT_INVERSE))
      return KFAC_EINVAL;
    if (j.n > 65536) return KFAC_EINVAL;
  }
  if (workspace_bytes < kfac_invert_workspace_bytes(jobs, njobs)) return KFAC_EWORKSPACE;
  ProfScope ps(KFAC_PROF_INVERT, (hipStream_t)stream);
  for (int g = 0; g < njobs; g += IMAXJ) {
    const int rc = invert_group(jobs + g, std::min(IMAXJ, njobs - g), (char*)workspace,
                                info ? info + g : nullptr, (hipStream_t)stream);
    if (rc) return rc;
  }
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
