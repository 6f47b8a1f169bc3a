// Laplace posterior weight samples on gfx950.
//
// Replaces KFAC.sample (models/curvatures.py:400-405)
//     (L_A @ z @ L_G.t()).t(),  z ~ N(0, 1) of shape (nA, nG)
// and the in-place add of Curvature._replace (curvatures.py:68-82), which splits the
// (nG x nA) sample into weight columns [0, nA-1) and the bias column nA-1.
//
// Two grouped launches over every layer of a call (fp32 MFMA, exact fp32 products
// as torch's fp32 matmul):
//   1. Y = L_A z                  (nA x nG)   Y[a][j] = sum_{i <= a} L_A[a][i] z[i][j]
//   2. out[g][a] (+)= sum_{j <= g} L_G[g][j] Y[a][j]   = (L_A z L_G^T)^T
// Both factors are lower-triangular (KFAC.invert's Cholesky factors), so each tile
// contracts only the K-range its triangle leaves non-zero; `dense` jobs (EFB.sample,
// curvatures.py:466-473: eigenvector matrices, z pre-scaled by the host) contract
// all of K.  Launch 2's output tile is indexed (g, a) so the MFMA lanes walk a:
// weight rows are written coalesced.  z is
// the caller's (torch.randn in the reference's order), so samples match the
// reference draw for draw.
#include "kfac_common.h"

namespace kfac {

constexpr int SMAXJ = 8;

struct SampleJobDev {
  OpDev la_t, z;    // launch 1: A-operand L_A^T (element (i, a) = L_A[a][i]), B-operand z
  OpDev lg_t, y_t;  // launch 2: A-operand L_G^T (element (j, g) = L_G[g][j]), B-operand Y^T
  float* Y;         // workspace, nA x nG row-major
  float* W;
  float* bias;
  int64_t ldW;
  int nA, nG, wcols, accumulate, dense;
  int t1_begin, t2_begin;  // first task of this job in launch 1 / launch 2
};

struct SampleArgs {
  int njobs;
  int t1_end[SMAXJ], t2_end[SMAXJ];
  SampleJobDev job[SMAXJ];
};
static_assert(sizeof(SampleArgs) <= 4096, "kernel argument block");

__device__ __forceinline__ int find_job(const int* ends, int njobs, int task) {
  int j = 0;
  while (j + 1 < njobs && task >= ends[j]) ++j;
  return j;
}

// Launch 1: one 64x64 tile of Y per workgroup.
__global__ __launch_bounds__(NTHREADS) void kfac_sample_ly(SampleArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[4 * PANEL];
  const int task = blockIdx.x;
  const int jb = find_job(args.t1_end, args.njobs, task);
  const SampleJobDev& S = args.job[jb];
  const int tg = (S.nG + TILE - 1) / TILE;
  const int local = task - S.t1_begin;
  const int a0 = (local / tg) * TILE, j0 = (local % tg) * TILE;
  floatx16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  // L_A lower: L_A[a][i] = 0 for i > a, so i < a0 + 64 suffices (dense: all i)
  const int64_t kend = S.dense ? (int64_t)S.nA : min((int64_t)S.nA, (int64_t)a0 + TILE);
  contract_tile<KFAC_CHANNEL, KFAC_ROWMAJOR>(S.la_t, a0, S.z, j0, 0, kend, false, true, lds, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = j0 + (wave & 1) * 32 + (lane & 31);
  if (col >= S.nG) return;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int row = a0 + (wave >> 1) * 32 + acc_row(v, lane);
    if (row < S.nA) S.Y[(int64_t)row * S.nG + col] = acc[v];
  }
}

// Launch 2: one 64x64 tile of the (nG x nA) sample, added into (or written to) the
// weight rows, the last column going to the bias.
__global__ __launch_bounds__(NTHREADS) void kfac_sample_out(SampleArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[4 * PANEL];
  const int task = blockIdx.x;
  const int jb = find_job(args.t2_end, args.njobs, task);
  const SampleJobDev& S = args.job[jb];
  const int ta = (S.nA + TILE - 1) / TILE;
  const int local = task - S.t2_begin;
  const int g0 = (local / ta) * TILE, a0 = (local % ta) * TILE;
  floatx16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  // L_G lower: j <= g, so j < g0 + 64 suffices (dense: all j)
  const int64_t kend = S.dense ? (int64_t)S.nG : min((int64_t)S.nG, (int64_t)g0 + TILE);
  contract_tile<KFAC_CHANNEL, KFAC_CHANNEL>(S.lg_t, g0, S.y_t, a0, 0, kend, false, true, lds, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a = a0 + (wave & 1) * 32 + (lane & 31);
  if (a >= S.nA) return;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int g = g0 + (wave >> 1) * 32 + acc_row(v, lane);
    if (g >= S.nG) continue;
    float* dst = a < S.wcols ? S.W + (int64_t)g * S.ldW + a : (S.bias ? S.bias + g : nullptr);
    if (!dst) continue;
    *dst = S.accumulate ? *dst + acc[v] : acc[v];
  }
}

static size_t sample_y_bytes(const kfac_sample_job& j) {
  return align_up((size_t)j.nA * (size_t)j.nG * sizeof(float), 256);
}

}  // namespace kfac

using namespace kfac;

extern "C" size_t kfac_sample_workspace_bytes(const kfac_sample_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  size_t total = 0;
  for (int i = 0; i < njobs; ++i) total += sample_y_bytes(jobs[i]);
  return total;
}

extern "C" int kfac_sample(const kfac_sample_job* jobs, int njobs, int accumulate, void* workspace,
                           size_t workspace_bytes, kfac_stream_t stream) {
  if (njobs <= 0 || njobs > SMAXJ || !jobs) return KFAC_EINVAL;
  if (!workspace || workspace_bytes < kfac_sample_workspace_bytes(jobs, njobs)) return KFAC_EWORKSPACE;
  SampleArgs args{};
  args.njobs = njobs;
  char* ws = (char*)workspace;
  int64_t t1 = 0, t2 = 0;
  for (int i = 0; i < njobs; ++i) {
    const kfac_sample_job& q = jobs[i];
    if (!q.LA || !q.LG || !q.Z || !q.W || q.nA <= 0 || q.nG <= 0 || q.ldA < q.nA || q.ldG < q.nG ||
        q.wcols < 0 || q.wcols > q.nA || q.ldW < q.wcols || (q.wcols < q.nA && q.wcols != q.nA - 1))
      return KFAC_EINVAL;
    SampleJobDev& d = args.job[i];
    d.Y = reinterpret_cast<float*>(ws);
    ws += sample_y_bytes(q);
    d.W = q.W;
    d.bias = q.bias;
    d.ldW = q.ldW;
    d.nA = q.nA;
    d.nG = q.nG;
    d.wcols = q.wcols;
    d.accumulate = accumulate;
    d.dense = q.dense != 0;
    // element (i, a) of L_A^T = LA[a*ldA + i]: CHANNEL with L = ldA (rows = K = nA)
    d.la_t = OpDev{};
    d.la_t.ptr = q.LA; d.la_t.layout = KFAC_CHANNEL; d.la_t.rows = q.nA; d.la_t.cols = q.nA;
    d.la_t.L = q.ldA; d.la_t.sB = 0; d.la_t.ones = -1;
    d.z = OpDev{};
    d.z.ptr = q.Z; d.z.layout = KFAC_ROWMAJOR; d.z.rows = q.nA; d.z.cols = q.nG; d.z.ld = q.nG;
    d.z.ones = -1;
    // element (j, g) of L_G^T = LG[g*ldG + j]; element (j, a) of Y^T = Y[a*nG + j]
    d.lg_t = OpDev{};
    d.lg_t.ptr = q.LG; d.lg_t.layout = KFAC_CHANNEL; d.lg_t.rows = q.nG; d.lg_t.cols = q.nG;
    d.lg_t.L = q.ldG; d.lg_t.sB = 0; d.lg_t.ones = -1;
    d.y_t = OpDev{};
    d.y_t.ptr = d.Y; d.y_t.layout = KFAC_CHANNEL; d.y_t.rows = q.nG; d.y_t.cols = q.nA;
    d.y_t.L = q.nG; d.y_t.sB = 0; d.y_t.ones = -1;
    const int64_t ta = cdiv(q.nA, TILE), tg = cdiv(q.nG, TILE);
    d.t1_begin = (int)t1;
    d.t2_begin = (int)t2;
    t1 += ta * tg;
    t2 += ta * tg;
    args.t1_end[i] = (int)t1;
    args.t2_end[i] = (int)t2;
  }
  if (t1 >= (int64_t)1 << 31) return KFAC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(kfac_sample_ly, dim3((unsigned)t1), dim3(NTHREADS), 0, s, args);
  KFAC_CHECK_LAUNCH();
  hipLaunchKernelGGL(kfac_sample_out, dim3((unsigned)t2), dim3(NTHREADS), 0, s, args);
  KFAC_CHECK_LAUNCH();
  return KFAC_OK;
}
