// Symmetric eigendecomposition of Kronecker factors on gfx950 (fp64).
//
// Replaces torch.symeig in models/utilities.py:120-159 (get_eigenvalues /
// get_eigenvectors; torch.symeig no longer exists in torch>=2.0, eigvalsh /
// eigh are its successors with the same ascending order).
//
// Two-sided cyclic Jacobi with the parallel (round-robin tournament) ordering:
// each round applies n/2 disjoint rotations — rows, barrier, columns, barrier —
// inside ONE workgroup per matrix, the matrix resident in LDS (fp64, n <= 128).
// Eigenvector columns accumulate in a fp64 workspace copy of V.  Converged when
// off(A)^2 <= (1e-15)^2 * ||A||_F^2 (checked once per sweep).  Output sorted
// ascending by a parallel rank pass.
#include <math.h>

#include <algorithm>

#include "kfac_common.h"

namespace kfac {

constexpr int EIG_LDS_MAX = 128;  // fp64 n x n in LDS: 128 KiB
constexpr int EMAXJ = 8;
constexpr int EIG_MAX_SWEEPS = 40;

struct EigJobDev {
  const float* F;
  int64_t ldF;
  double* evals;
  float* evecs;
  int64_t ldv;
  double* V;   // n x n fp64 workspace (eigenvector accumulation)
  int* info;
  int n;
};

struct EigArgs {
  int njobs;
  EigJobDev job[EMAXJ];
};

// tournament pairing for round r of a (m = even) player round robin: player 0 fixed
__device__ __forceinline__ void rr_pair(int m, int r, int slot, int& p, int& q) {
  // positions: 0 fixed, others rotate
  auto player = [&](int pos) { return pos == 0 ? 0 : 1 + (pos - 1 + r) % (m - 1); };
  p = player(slot);
  q = player(m - 1 - slot);
}

__global__ __launch_bounds__(NTHREADS) void eig_jacobi_lds(EigArgs args) {
  __shared__ double A[EIG_LDS_MAX * EIG_LDS_MAX];
  __shared__ double cs[EIG_LDS_MAX];  // c, s per pair slot (2 * 64)
  __shared__ int pq[EIG_LDS_MAX];     // p, q per pair slot
  __shared__ double red[NTHREADS / 64];
  __shared__ double red2[NTHREADS / 64];
  __shared__ int rank_of[EIG_LDS_MAX];
  const EigJobDev& J = args.job[blockIdx.x];
  const int n = J.n, tid = threadIdx.x;
  const int m = n + (n & 1);  // players (n odd: one bye, index n)
  const int slots = m / 2;

  for (int e = tid; e < n * n; e += NTHREADS) {
    const int r = e / n, c = e - r * n;
    A[e] = 0.5 * ((double)J.F[(int64_t)r * J.ldF + c] + (double)J.F[(int64_t)c * J.ldF + r]);
    if (J.V) J.V[e] = (r == c) ? 1.0 : 0.0;
  }
  __syncthreads();

  int sweep = 0;
  for (; sweep < EIG_MAX_SWEEPS; ++sweep) {
    // convergence: off-diagonal vs total Frobenius norm
    double off = 0.0, tot = 0.0;
    for (int e = tid; e < n * n; e += NTHREADS) {
      const double v = A[e] * A[e];
      tot += v;
      if (e / n != e % n) off += v;
    }
    for (int o = 32; o > 0; o >>= 1) off += __shfl_xor(off, o);
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    if ((tid & 63) == 0) { red[tid >> 6] = off; red2[tid >> 6] = tot; }
    __syncthreads();
    off = red[0] + red[1] + red[2] + red[3];
    tot = red2[0] + red2[1] + red2[2] + red2[3];
    __syncthreads();
    if (off <= 1e-30 * tot || off == 0.0) break;

    for (int r = 0; r < m - 1; ++r) {
      // rotation parameters, one thread per pair slot
      if (tid < slots) {
        int p, q;
        rr_pair(m, r, tid, p, q);
        if (p > q) { const int t = p; p = q; q = t; }
        double c = 1.0, s = 0.0;
        if (q < n) {
          const double apq = A[p * n + q];
          if (apq != 0.0) {
            const double tau = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
            const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
            c = 1.0 / sqrt(1.0 + t * t);
            s = t * c;
          }
        }
        cs[2 * tid] = c;
        cs[2 * tid + 1] = s;
        pq[2 * tid] = p;
        pq[2 * tid + 1] = q;
      }
      __syncthreads();
      // rows: A[p,:] = c A[p,:] - s A[q,:];  A[q,:] = s A[p,:] + c A[q,:]
      for (int e = tid; e < slots * n; e += NTHREADS) {
        const int sl = e / n, col = e - sl * n;
        const int p = pq[2 * sl], q = pq[2 * sl + 1];
        if (q >= n) continue;
        const double c = cs[2 * sl], s = cs[2 * sl + 1];
        const double ap = A[p * n + col], aq = A[q * n + col];
        A[p * n + col] = c * ap - s * aq;
        A[q * n + col] = s * ap + c * aq;
      }
      __syncthreads();
      // columns (and V's columns)
      for (int e = tid; e < slots * n; e += NTHREADS) {
        const int sl = e / n, row = e - sl * n;
        const int p = pq[2 * sl], q = pq[2 * sl + 1];
        if (q >= n) continue;
        const double c = cs[2 * sl], s = cs[2 * sl + 1];
        const double ap = A[row * n + p], aq = A[row * n + q];
        A[row * n + p] = c * ap - s * aq;
        A[row * n + q] = s * ap + c * aq;
        if (J.V) {
          const double vp = J.V[row * n + p], vq = J.V[row * n + q];
          J.V[row * n + p] = c * vp - s * vq;
          J.V[row * n + q] = s * vp + c * vq;
        }
      }
      __syncthreads();
    }
  }
  if (tid == 0 && J.info) *J.info = (sweep >= EIG_MAX_SWEEPS) ? 1 : 0;
  // ascending rank (ties by index)
  for (int i = tid; i < n; i += NTHREADS) {
    const double li = A[i * n + i];
    int rk = 0;
    for (int j = 0; j < n; ++j) {
      const double lj = A[j * n + j];
      rk += (lj < li) || (lj == li && j < i);
    }
    rank_of[i] = rk;
    J.evals[rk] = li;
  }
  __syncthreads();
  if (J.evecs) {
    for (int e = tid; e < n * n; e += NTHREADS) {
      const int row = e / n, col = e - row * n;
      J.evecs[(int64_t)row * J.ldv + rank_of[col]] = (float)J.V[e];
    }
  }
}

}  // namespace kfac

using namespace kfac;

extern "C" size_t kfac_eig_workspace_bytes(const kfac_eig_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  size_t best = 0;
  for (int g = 0; g < njobs; g += EMAXJ) {
    size_t tot = 0;
    for (int i = g; i < std::min(njobs, g + EMAXJ); ++i)
      tot += align_up((size_t)jobs[i].n * jobs[i].n * sizeof(double), 256);
    best = std::max(best, tot);
  }
  return best;
}

extern "C" int kfac_syev(const kfac_eig_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
                         int32_t* info, kfac_stream_t stream) {
  if (njobs <= 0 || !jobs) return KFAC_EINVAL;
  for (int i = 0; i < njobs; ++i) {
    const kfac_eig_job& j = jobs[i];
    if (!j.F || !j.evals || j.n <= 0 || j.ldF < j.n || (j.evecs && j.ldv < j.n)) return KFAC_EINVAL;
    if (j.n > EIG_LDS_MAX) return KFAC_EINVAL;  // larger factors: blocked solver (not yet)
  }
  if (workspace_bytes < kfac_eig_workspace_bytes(jobs, njobs)) return KFAC_EWORKSPACE;
  for (int g = 0; g < njobs; g += EMAXJ) {
    EigArgs args{};
    args.njobs = std::min(EMAXJ, njobs - g);
    char* ws = (char*)workspace;
    for (int i = 0; i < args.njobs; ++i) {
      const kfac_eig_job& j = jobs[g + i];
      EigJobDev& d = args.job[i];
      d.F = j.F; d.ldF = j.ldF; d.n = j.n; d.evals = j.evals; d.evecs = j.evecs; d.ldv = j.ldv;
      d.V = j.evecs ? reinterpret_cast<double*>(ws) : nullptr;
      ws += align_up((size_t)j.n * j.n * sizeof(double), 256);
      d.info = info ? info + g + i : nullptr;
    }
    hipLaunchKernelGGL(eig_jacobi_lds, dim3(args.njobs), dim3(NTHREADS), 0, (hipStream_t)stream,
                       args);
    KFAC_CHECK_LAUNCH();
  }
  return KFAC_OK;
}
