// Kronecker-structured predictive variance on gfx950.
//
// Replaces the per-layer `J_i @ torch.kron(Q_i, H_i) @ J_i.t()` of
// sampling_free/classification/classification_ll_block.py:126-132 (and the
// `kronecker_product` variant of regression_ll_block.py:128-139), which
// materialises an (nA*nG)^2 matrix (40 GB for the MLP's first layer).
//
// With M = J viewed (nA x nG) row-major (the reference's flat index a*nG + g):
//   J kron(K1, K2) J^T = <K1^T M, M K2^T>_F .
// One task = one (layer, sample, 64x64 output tile): the WG contracts both
// tiles with fp32 MFMA into two accumulators held in the same lanes, multiplies
// them elementwise and reduces to one partial (no intermediate ever leaves the
// CU).  A second launch sums the partials per (layer, sample) in a fixed order
// and folds |v| over layers.  Lower-triangular K1/K2 (Cholesky factors from
// KFAC.invert) skip their zero K-blocks.
#include "kfac_common.h"

namespace kfac {

constexpr int QMAXJ = 8;

struct QuadJobDev {
  OpDev k1, m_row;  // P = K1^T M : A-operand K1 (ROWMAJOR), B-operand M (ROWMAJOR, ld nG)
  OpDev m_col, k2;  // Q = M K2^T : A-operand M (CHANNEL: M[a*nG + k]), B-operand K2 (CHANNEL)
  const float* J;
  int64_t ldJ;
  float* v;
  double* partial;  // nb x ta x tg partial sums
  int nA, nG, ta, tg, lower1, lower2;
  int task_begin;
};

struct QuadArgs {
  int njobs;
  int64_t nb;
  int abs_sum;
  float* out;
  int task_end[QMAXJ];
  QuadJobDev job[QMAXJ];
};

__global__ __launch_bounds__(NTHREADS) void kfac_quad_tiles(QuadArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[4 * PANEL];
  __shared__ double red[NTHREADS / 64];
  const int task = blockIdx.x;
  int j = 0;
  while (j + 1 < args.njobs && task >= args.task_end[j]) ++j;
  const QuadJobDev& Q = args.job[j];
  const int local = task - Q.task_begin;
  const int per_sample = Q.ta * Q.tg;
  const int64_t b = local / per_sample;
  const int t = local - (int)(b * per_sample);
  const int ta = t / Q.tg, tg = t - ta * Q.tg;
  const int a0 = ta * TILE, g0 = tg * TILE;

  OpDev mrow = Q.m_row, mcol = Q.m_col;
  mrow.ptr = Q.J + b * Q.ldJ;
  mcol.ptr = Q.J + b * Q.ldJ;

  floatx16 p, q;
#pragma unroll
  for (int v = 0; v < 16; ++v) { p[v] = 0.f; q[v] = 0.f; }
  // P[a][g] = sum_k K1[k][a] M[k][g]; K1 lower => k >= a0
  contract_tile<KFAC_ROWMAJOR, KFAC_ROWMAJOR>(Q.k1, a0, mrow, g0, Q.lower1 ? a0 : 0, Q.nA, false,
                                              true, lds, p);
  // Q[a][g] = sum_k M[a][k] K2[g][k]; K2 lower => k <= g
  const int64_t kq = Q.lower2 ? min(Q.nG, g0 + TILE) : Q.nG;
  contract_tile<KFAC_CHANNEL, KFAC_CHANNEL>(mcol, a0, Q.k2, g0, 0, kq, false, true, lds, q);
  double s = 0.0;
#pragma unroll
  for (int v = 0; v < 16; ++v) s += (double)p[v] * (double)q[v];  // padding: exact zeros
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) Q.partial[local] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(64) void kfac_quad_reduce(QuadArgs args) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  double total = 0.0;
  for (int j = 0; j < args.njobs; ++j) {
    const QuadJobDev& Q = args.job[j];
    const int per = Q.ta * Q.tg;
    const double* part = Q.partial + b * per;
    double s = 0.0;
    for (int i = lane; i < per; i += 64) s += part[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (Q.v && lane == 0) Q.v[b] = (float)s;
    total += args.abs_sum ? fabs(s) : s;
  }
  if (lane == 0) args.out[b] = (float)total;
}

static size_t quad_partial_bytes(const kfac_quad_job& j, int64_t nb) {
  const int64_t ta = cdiv(j.nA, TILE), tg = cdiv(j.nG, TILE);
  return align_up((size_t)(nb * ta * tg) * sizeof(double), 256);
}

}  // namespace kfac

using namespace kfac;

extern "C" size_t kfac_quadform_workspace_bytes(const kfac_quad_job* jobs, int njobs, int64_t nb) {
  if (!jobs || njobs <= 0 || nb <= 0) return 0;
  size_t total = 0;
  for (int i = 0; i < njobs; ++i) total += quad_partial_bytes(jobs[i], nb);
  return total;
}

extern "C" int kfac_kron_quadform(const kfac_quad_job* jobs, int njobs, int64_t nb, int abs_sum,
                                  float* out, void* workspace, size_t workspace_bytes,
                                  kfac_stream_t stream) {
  if (njobs <= 0 || !jobs || nb <= 0 || !out) return KFAC_EINVAL;
  if (njobs > QMAXJ) return KFAC_EINVAL;
  if (workspace_bytes < kfac_quadform_workspace_bytes(jobs, njobs, nb)) return KFAC_EWORKSPACE;
  QuadArgs args{};
  args.njobs = njobs;
  args.nb = nb;
  args.abs_sum = abs_sum;
  args.out = out;
  char* ws = (char*)workspace;
  int64_t tasks = 0;
  for (int i = 0; i < njobs; ++i) {
    const kfac_quad_job& q = jobs[i];
    if (!q.J || !q.K1 || !q.K2 || q.nA <= 0 || q.nG <= 0 || q.ld1 < q.nA || q.ld2 < q.nG ||
        q.ldJ < (int64_t)q.nA * q.nG)
      return KFAC_EINVAL;
    QuadJobDev& d = args.job[i];
    d.J = q.J;
    d.ldJ = q.ldJ;
    d.v = q.v;
    d.nA = q.nA;
    d.nG = q.nG;
    d.ta = (int)cdiv(q.nA, TILE);
    d.tg = (int)cdiv(q.nG, TILE);
    d.lower1 = q.lower1;
    d.lower2 = q.lower2;
    d.partial = reinterpret_cast<double*>(ws);
    ws += quad_partial_bytes(q, nb);
    // P = K1^T M
    d.k1 = OpDev{};
    d.k1.ptr = q.K1; d.k1.layout = KFAC_ROWMAJOR; d.k1.rows = q.nA; d.k1.cols = q.nA;
    d.k1.ld = q.ld1; d.k1.ones = -1;
    d.m_row = OpDev{};
    d.m_row.layout = KFAC_ROWMAJOR; d.m_row.rows = q.nA; d.m_row.cols = q.nG; d.m_row.ld = q.nG;
    d.m_row.ones = -1;
    // Q = M K2^T : element (k, a) of M = J[a*nG + k]; element (k, g) of K2 = K2[g*ld2 + k]
    d.m_col = OpDev{};
    d.m_col.layout = KFAC_CHANNEL; d.m_col.rows = q.nG; d.m_col.cols = q.nA; d.m_col.L = q.nG;
    d.m_col.sB = 0; d.m_col.ones = -1;
    d.k2 = OpDev{};
    d.k2.ptr = q.K2; d.k2.layout = KFAC_CHANNEL; d.k2.rows = q.nG; d.k2.cols = q.nG;
    d.k2.L = q.ld2; d.k2.sB = 0; d.k2.ones = -1;
    d.task_begin = (int)tasks;
    tasks += nb * d.ta * d.tg;
    args.task_end[i] = (int)tasks;
  }
  if (tasks >= (int64_t)1 << 31) return KFAC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  {
    ProfScope ps(KFAC_PROF_QUAD_TILES, s);
    hipLaunchKernelGGL(kfac_quad_tiles, dim3((unsigned)tasks), dim3(NTHREADS), 0, s, args);
  }
  KFAC_CHECK_LAUNCH();
  hipLaunchKernelGGL(kfac_quad_reduce, dim3((unsigned)nb), dim3(64), 0, s, args);
  KFAC_CHECK_LAUNCH();
  return KFAC_OK;
}
