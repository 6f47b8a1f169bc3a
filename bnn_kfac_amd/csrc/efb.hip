// Eigenbasis curvatures (EFB / INF) on gfx950.
//
// EFB.update (models/curvatures.py:427-449), per layer and batch:
//     lambdas = (V_G^T grad V_A) ** 2 ;  state (+)= lambdas ;  diags (+)= grad ** 2 * B
// as two launches over every layer of the call:
//   1. kfac_efb_project : T = V_G^T grad            (nG x nA, workspace)
//                         epilogue also: diag = [diag +] (grad * grad) * B
//                         (the diag grid IS the T grid: element (g, a) of both)
//   2. kfac_efb_square  : state = [state +] (T V_A) * (T V_A)
//                         (projection, square and accumulate in one epilogue; no
//                         lambdas tensor is materialised)
// INF.pre_sampler's V_s^T V_s (curvatures.py:548-580; V_s = c * kron(U_A, U_G) diag(sigma),
// (nA*nG) x (la*lg)) without forming V_s, as two launches:
//   3. kfac_inf_tq   : Tq[a][(q,q')] = sum_g c[a,g]^2 U_G[g,q] U_G[g,q']      (nA x lg^2)
//   4. kfac_inf_gram : out[(p,q)][(p',q')] = sigma_pq * (sum_a U_A[a,p] U_A[a,p'] Tq[a][(q,q')]) * sigma_p'q'
//      computed as the (la^2 x lg^2) GEMM over a and scattered to the (p,q) x (p',q')
//      layout in the epilogue.  Operand elements are formed in the panel loaders
//      (Khatri-Rao products of eigenvector rows), so neither kron(U_A, U_G) nor the
//      (p,p') operand exists in memory.  The unscaled sum is exactly symmetric (element
//      ((p',q'),(p,q)) multiplies the same fp32 products in the same k order); the
//      sigma scaling, applied in the reference's order, rounds the two halves apart by
//      at most an ulp, which the reference's (vtv + vtv^T) / 2 then averages.
//
// One 64x64 output tile per workgroup (4 waves, a 32x32 quadrant each, fp32
// v_mfma_f32_32x32x2_f32), K staged 32 rows at a time through double-buffered LDS
// panels [k][m]; each operand's loader picks the lane direction along which its
// memory is contiguous.
#include "kfac_common.h"

namespace kfac {

constexpr int EMAXJ = 8;     // layers per call
constexpr int EP = TILE + 1;  // LDS panel pitch (floats): conflict-free stores both ways

// ------------------------------------------------------------------ operands
// element (k, m) of the K x M operand; lanes walk m (ML) or k (KL) when staging
struct RowOp {  // X[k * ld + m] (k < K, m < M)
  static constexpr bool ML = true;
  const float* p;
  int64_t ld;
  int K, M;
  __device__ __forceinline__ float at(int k, int m) const {
    return (k < K && m < M) ? p[(int64_t)k * ld + m] : 0.f;
  }
};
struct ColOp {  // X[m * ld + k]: the transpose of a row-major M x K matrix
  static constexpr bool ML = false;
  const float* p;
  int64_t ld;
  int K, M;
  __device__ __forceinline__ float at(int k, int m) const {
    return (k < K && m < M) ? p[(int64_t)m * ld + k] : 0.f;
  }
};
struct SqColOp {  // X[m * ld + k]^2: INF's c[a, g]^2 (k = g, m = a)
  static constexpr bool ML = false;
  const float* p;
  int64_t ld;
  int K, M;
  __device__ __forceinline__ float at(int k, int m) const {
    if (k >= K || m >= M) return 0.f;
    const float c = p[(int64_t)m * ld + k];
    return __fmul_rn(c, c);
  }
};
struct KrOp {  // U[k * ld + m / w] * U[k * ld + m % w]: row k's Khatri-Rao pair (m < w^2)
  static constexpr bool ML = true;
  const float* p;
  int64_t ld;
  int K, w;
  __device__ __forceinline__ float at(int k, int m) const {
    if (k >= K || m >= w * w) return 0.f;
    const int i = m / w, j = m - i * w;
    const float* r = p + (int64_t)k * ld;
    return __fmul_rn(r[i], r[j]);
  }
};

// stage rows [k, k + BK) x columns [m0, m0 + 64) of `op` into `dst` ([k][m], pitch EP)
template <class Op>
__device__ __forceinline__ void stage_load(const Op& op, int k, int m0, float (&v)[8]) {
  const int tid = threadIdx.x;
  if constexpr (Op::ML) {
    const int c = tid & 63, r0 = tid >> 6;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = op.at(k + r0 + 4 * i, m0 + c);
  } else {
    const int r = tid & 31, c0 = tid >> 5;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = op.at(k + r, m0 + c0 + 8 * i);
  }
}
template <class Op>
__device__ __forceinline__ void stage_store(float* dst, const float (&v)[8]) {
  const int tid = threadIdx.x;
  if constexpr (Op::ML) {
    const int c = tid & 63, r0 = tid >> 6;
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[(r0 + 4 * i) * EP + c] = v[i];
  } else {
    const int r = tid & 31, c0 = tid >> 5;
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[r * EP + c0 + 8 * i] = v[i];
  }
}

// acc (this wave's 32x32 quadrant of the tile) = sum_{k < K} A(k, m0 + .) B(k, n0 + .)
template <class OA, class OB>
__device__ __forceinline__ void tile_gemm(const OA& oa, const OB& ob, int m0, int n0, int K, float* lds,
                                          floatx16& acc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qi = wave >> 1, qj = wave & 1, h = lane >> 5, rr = lane & 31;
  constexpr int PB = BK * EP;  // floats of one panel
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  float va[8], vb[8];
  stage_load(oa, 0, m0, va);
  stage_load(ob, 0, n0, vb);
  stage_store<OA>(lds, va);
  stage_store<OB>(lds + PB, vb);
  __syncthreads();
  int cur = 0;
  for (int k = 0; k < K; k += BK) {
    const bool more = k + BK < K;
    if (more) {
      stage_load(oa, k + BK, m0, va);
      stage_load(ob, k + BK, n0, vb);
    }
    const float* a = lds + 2 * cur * PB + h * EP + qi * 32 + rr;
    const float* b = lds + 2 * cur * PB + PB + h * EP + qj * 32 + rr;
#pragma unroll
    for (int s = 0; s < BK / 2; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[2 * s * EP], b[2 * s * EP], acc, 0, 0, 0);
    if (more) {
      stage_store<OA>(lds + 2 * (cur ^ 1) * PB, va);
      stage_store<OB>(lds + 2 * (cur ^ 1) * PB + PB, vb);
    }
    __syncthreads();
    cur ^= 1;
  }
}

// (row, col) of accumulator register v of this lane in the tile at (m0, n0)
__device__ __forceinline__ void tile_rc(int m0, int n0, int v, int& row, int& col) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  row = m0 + (wave >> 1) * 32 + acc_row(v, lane);
  col = n0 + (wave & 1) * 32 + (lane & 31);
}

// ---------------------------------------------------------------------- EFB
struct EfbJobDev {
  const float *VA, *VG, *grad;
  int64_t ldA, ldG, ldgr, lds, ldd;
  float *T, *state, *diag;
  int nA, nG, accumulate;
  float scale;
  int tbegin;  // first tile of this job (both launches: the nG x nA grid)
};
struct EfbArgs {
  int njobs;
  int tend[EMAXJ];
  EfbJobDev job[EMAXJ];
};
static_assert(sizeof(EfbArgs) <= 4096, "kernel argument block");

__device__ __forceinline__ int efb_job(const EfbArgs& a, int task) {
  int j = 0;
  while (j + 1 < a.njobs && task >= a.tend[j]) ++j;
  return j;
}

__global__ __launch_bounds__(NTHREADS) void kfac_efb_project(EfbArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[4 * BK * EP];
  const int jb = efb_job(args, blockIdx.x);
  const EfbJobDev& J = args.job[jb];
  const int local = blockIdx.x - J.tbegin, ta = (J.nA + TILE - 1) / TILE;
  const int m0 = (local / ta) * TILE, n0 = (local % ta) * TILE;
  floatx16 acc;
  // T[g'][a] = sum_g VG[g][g'] grad[g][a]
  tile_gemm(RowOp{J.VG, J.ldG, J.nG, J.nG}, RowOp{J.grad, J.ldgr, J.nG, J.nA}, m0, n0, J.nG, lds, acc);
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    int r, c;
    tile_rc(m0, n0, v, r, c);
    if (r >= J.nG || c >= J.nA) continue;
    J.T[(int64_t)r * J.nA + c] = acc[v];
    if (J.diag) {  // diags (+)= grads ** 2 * batch_size, rounded as torch does it
      const float g = J.grad[(int64_t)r * J.ldgr + c];
      const float t = __fmul_rn(__fmul_rn(g, g), J.scale);
      float* d = J.diag + (int64_t)r * J.ldd + c;
      *d = J.accumulate ? __fadd_rn(*d, t) : t;
    }
  }
}

__global__ __launch_bounds__(NTHREADS) void kfac_efb_square(EfbArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[4 * BK * EP];
  const int jb = efb_job(args, blockIdx.x);
  const EfbJobDev& J = args.job[jb];
  const int local = blockIdx.x - J.tbegin, ta = (J.nA + TILE - 1) / TILE;
  const int m0 = (local / ta) * TILE, n0 = (local % ta) * TILE;
  floatx16 acc;
  // P[g'][a'] = sum_a T[g'][a] VA[a][a']
  tile_gemm(ColOp{J.T, J.nA, J.nA, J.nG}, RowOp{J.VA, J.ldA, J.nA, J.nA}, m0, n0, J.nA, lds, acc);
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    int r, c;
    tile_rc(m0, n0, v, r, c);
    if (r >= J.nG || c >= J.nA) continue;
    const float l = __fmul_rn(acc[v], acc[v]);
    float* s = J.state + (int64_t)r * J.lds + c;
    *s = J.accumulate ? __fadd_rn(*s, l) : l;
  }
}

// ---------------------------------------------------------------------- INF
struct GramJobDev {
  const float *UA, *UG, *c, *sigma;
  int64_t ldA, ldG, ldo;
  float *Tq, *out;
  int nA, nG, la, lg;
  int t1begin, t2begin;
};
struct GramArgs {
  int njobs;
  int t1end[EMAXJ], t2end[EMAXJ];
  GramJobDev job[EMAXJ];
};
static_assert(sizeof(GramArgs) <= 4096, "kernel argument block");

__global__ __launch_bounds__(NTHREADS) void kfac_inf_tq(GramArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[4 * BK * EP];
  int jb = 0;
  while (jb + 1 < args.njobs && (int)blockIdx.x >= args.t1end[jb]) ++jb;
  const GramJobDev& J = args.job[jb];
  const int L2 = J.lg * J.lg;
  const int local = blockIdx.x - J.t1begin, tn = (L2 + TILE - 1) / TILE;
  const int m0 = (local / tn) * TILE, n0 = (local % tn) * TILE;
  floatx16 acc;
  // Tq[a][(q,q')] = sum_g c[a][g]^2 * (UG[g][q] UG[g][q'])
  tile_gemm(SqColOp{J.c, J.nG, J.nG, J.nA}, KrOp{J.UG, J.ldG, J.nG, J.lg}, m0, n0, J.nG, lds, acc);
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    int r, c;
    tile_rc(m0, n0, v, r, c);
    if (r < J.nA && c < L2) J.Tq[(int64_t)r * L2 + c] = acc[v];
  }
}

__global__ __launch_bounds__(NTHREADS) void kfac_inf_gram(GramArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[4 * BK * EP];
  int jb = 0;
  while (jb + 1 < args.njobs && (int)blockIdx.x >= args.t2end[jb]) ++jb;
  const GramJobDev& J = args.job[jb];
  const int A2 = J.la * J.la, L2 = J.lg * J.lg;
  const int local = blockIdx.x - J.t2begin, tn = (L2 + TILE - 1) / TILE;
  const int m0 = (local / tn) * TILE, n0 = (local % tn) * TILE;
  floatx16 acc;
  // X[(p,p')][(q,q')] = sum_a (UA[a][p] UA[a][p']) Tq[a][(q,q')]
  tile_gemm(KrOp{J.UA, J.ldA, J.nA, J.la}, RowOp{J.Tq, L2, J.nA, L2}, m0, n0, J.nA, lds, acc);
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    int r, c;
    tile_rc(m0, n0, v, r, c);
    if (r >= A2 || c >= L2) continue;
    const int p = r / J.la, p2 = r - p * J.la, q = c / J.lg, q2 = c - q * J.lg;
    const int i = p * J.lg + q, j = p2 * J.lg + q2;
    // reg_lambda[:, None] * vtv * reg_lambda[None, :] (left to right)
    J.out[(int64_t)i * J.ldo + j] = __fmul_rn(__fmul_rn(J.sigma[i], acc[v]), J.sigma[j]);
  }
}

static size_t efb_t_bytes(const kfac_efb_job& j) {
  return align_up((size_t)j.nA * (size_t)j.nG * sizeof(float), 256);
}
static size_t gram_tq_bytes(const kfac_gram_job& j) {
  return align_up((size_t)j.nA * (size_t)j.lg * (size_t)j.lg * sizeof(float), 256);
}

}  // namespace kfac

using namespace kfac;

extern "C" size_t kfac_efb_workspace_bytes(const kfac_efb_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  size_t t = 0;
  for (int i = 0; i < njobs; ++i) t += efb_t_bytes(jobs[i]);
  return t;
}

extern "C" int kfac_efb_update(const kfac_efb_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
                               kfac_stream_t stream) {
  if (njobs <= 0 || njobs > EMAXJ || !jobs) return KFAC_EINVAL;
  if (!workspace || workspace_bytes < kfac_efb_workspace_bytes(jobs, njobs)) return KFAC_EWORKSPACE;
  EfbArgs args{};
  args.njobs = njobs;
  char* ws = (char*)workspace;
  int64_t tiles = 0;
  for (int i = 0; i < njobs; ++i) {
    const kfac_efb_job& q = jobs[i];
    if (!q.VA || !q.VG || !q.grad || !q.state || q.nA <= 0 || q.nG <= 0 || q.ldA < q.nA || q.ldG < q.nG ||
        q.ld_grad < q.nA || q.ld_state < q.nA || (q.diag && q.ld_diag < q.nA))
      return KFAC_EINVAL;
    EfbJobDev& d = args.job[i];
    d.VA = q.VA; d.ldA = q.ldA;
    d.VG = q.VG; d.ldG = q.ldG;
    d.grad = q.grad; d.ldgr = q.ld_grad;
    d.state = q.state; d.lds = q.ld_state;
    d.diag = q.diag; d.ldd = q.ld_diag;
    d.nA = q.nA; d.nG = q.nG;
    d.accumulate = q.accumulate != 0;
    d.scale = q.scale;
    d.T = reinterpret_cast<float*>(ws);
    ws += efb_t_bytes(q);
    d.tbegin = (int)tiles;
    tiles += cdiv(q.nG, TILE) * cdiv(q.nA, TILE);
    args.tend[i] = (int)tiles;
  }
  if (tiles >= (int64_t)1 << 31) return KFAC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(kfac_efb_project, dim3((unsigned)tiles), dim3(NTHREADS), 0, s, args);
  KFAC_CHECK_LAUNCH();
  hipLaunchKernelGGL(kfac_efb_square, dim3((unsigned)tiles), dim3(NTHREADS), 0, s, args);
  KFAC_CHECK_LAUNCH();
  return KFAC_OK;
}

extern "C" size_t kfac_gram_workspace_bytes(const kfac_gram_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  size_t t = 0;
  for (int i = 0; i < njobs; ++i) t += gram_tq_bytes(jobs[i]);
  return t;
}

extern "C" int kfac_kron_gram(const kfac_gram_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
                              kfac_stream_t stream) {
  if (njobs <= 0 || njobs > EMAXJ || !jobs) return KFAC_EINVAL;
  if (!workspace || workspace_bytes < kfac_gram_workspace_bytes(jobs, njobs)) return KFAC_EWORKSPACE;
  GramArgs args{};
  args.njobs = njobs;
  char* ws = (char*)workspace;
  int64_t t1 = 0, t2 = 0;
  for (int i = 0; i < njobs; ++i) {
    const kfac_gram_job& q = jobs[i];
    if (!q.UA || !q.UG || !q.c || !q.sigma || !q.out || q.nA <= 0 || q.nG <= 0 || q.la <= 0 || q.lg <= 0 ||
        q.ldA < q.la || q.ldG < q.lg || q.ldo < (int64_t)q.la * q.lg || (int64_t)q.la * q.la >= (1 << 30) ||
        (int64_t)q.lg * q.lg >= (1 << 30))
      return KFAC_EINVAL;
    GramJobDev& d = args.job[i];
    d.UA = q.UA; d.ldA = q.ldA;
    d.UG = q.UG; d.ldG = q.ldG;
    d.c = q.c; d.sigma = q.sigma;
    d.out = q.out; d.ldo = q.ldo;
    d.nA = q.nA; d.nG = q.nG; d.la = q.la; d.lg = q.lg;
    d.Tq = reinterpret_cast<float*>(ws);
    ws += gram_tq_bytes(q);
    const int64_t L2 = (int64_t)q.lg * q.lg, A2 = (int64_t)q.la * q.la;
    d.t1begin = (int)t1;
    t1 += cdiv(q.nA, TILE) * cdiv(L2, TILE);
    args.t1end[i] = (int)t1;
    d.t2begin = (int)t2;
    t2 += cdiv(A2, TILE) * cdiv(L2, TILE);
    args.t2end[i] = (int)t2;
  }
  if (t1 >= (int64_t)1 << 31 || t2 >= (int64_t)1 << 31) return KFAC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(kfac_inf_tq, dim3((unsigned)t1), dim3(NTHREADS), 0, s, args);
  KFAC_CHECK_LAUNCH();
  hipLaunchKernelGGL(kfac_inf_gram, dim3((unsigned)t2), dim3(NTHREADS), 0, s, args);
  KFAC_CHECK_LAUNCH();
  return KFAC_OK;
}
