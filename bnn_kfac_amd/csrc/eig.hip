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

// ---------------------------------------------------------------------------
// n > 128: Householder tridiagonalisation + Sturm bisection (eigenvalues).
//
// eig_tridiag: ONE persistent launch per factor.  G workgroups, row i owned by
// workgroup i % G (slot i / G), the owned rows kept in LDS for the whole
// reduction (fp64, symmetrised).  Step k (reflector for column k):
//   phase A (row-local): p_i = tau * sum_j A[i][j] u_j, partial c = sum p_i u_i
//   -- grid barrier --
//   phase B (row-local): w = p - (tau c / 2) u ;  A[i][j] -= u_i w_j + w_i u_j,
//            then the next column A[i][k+1] (and its partial norm) is published
//   -- grid barrier --
// Every workgroup derives the reflector scalars redundantly from the published
// partials, so the only cross-workgroup data are u / p / two partial vectors.
// Grid barriers: agent-scope release (one lane, after the workgroup barrier) on
// an arrival counter, agent-scope acquire poll, bounded spins; a timeout sets
// `abort` and every workgroup leaves at its next barrier (the launch always
// drains; the host reports the timeout as info = -1).

struct TriArgs {
  const float* F;
  int64_t ldF;
  int n, G, R;         // rows per workgroup R = ceil(n / G)
  double* rows_g;      // G x R x n owned rows when they do not fit LDS (else null)
  double* x;           // 2 x n: published columns (double-buffered by step parity)
  double* p;           // n
  double* cpart;       // G
  double* spart;       // G
  double* d;           // n: diagonal of T
  double* e;           // n: off-diagonal of T (e[k] = T[k+1][k])
  unsigned* bar;       // arrival counter (zeroed before the launch)
  unsigned* abort;     // timeout flag (zeroed before the launch)
  double* U;           // n x n: row k = reflector u_k (entries k+1..n-1), or null
  double* tau;         // n: reflector scales (0: no reflection), or null
};

__device__ __forceinline__ bool grid_sync(unsigned* bar, unsigned* abort, unsigned target) {
  __syncthreads();  // every wave's stores issued and waited (vmcnt 0) before the release
  __shared__ int bail;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    for (unsigned spins = 0;; ++spins) {
      if (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
          spins > (1u << 22)) {
        __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    bail = !ok;
  }
  __syncthreads();
  return !bail;
}

// deterministic: same tree in every workgroup -> bit-identical scalars everywhere
__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

template <bool LDS_ROWS>
__global__ __launch_bounds__(NTHREADS) void eig_tridiag(TriArgs a) {
  extern __shared__ double lds[];  // [u n][w n][rows R x n if LDS_ROWS]
  __shared__ double red[NTHREADS / 64];
  const int n = a.n, G = a.G, wg = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  double* uS = lds;
  double* wS = lds + n;
  double* rows = LDS_ROWS ? lds + 2 * n : a.rows_g + (size_t)wg * a.R * n;
  unsigned epoch = 0;
  auto row_of = [&](int slot) { return slot * G + wg; };
  auto A = [&](int slot) { return rows + (size_t)slot * n; };

  // load + symmetrise the owned rows; publish column 0 (step 0's x)
  for (int s = 0; s < a.R; ++s) {
    const int i = row_of(s);
    if (i >= n) break;
    for (int j = tid; j < n; j += NTHREADS)
      A(s)[j] = 0.5 * ((double)a.F[(int64_t)i * a.ldF + j] + (double)a.F[(int64_t)j * a.ldF + i]);
  }
  __syncthreads();
  {
    double sig = 0.0;
    for (int s = tid; s < a.R; s += NTHREADS) {
      const int i = row_of(s);
      if (i >= n) continue;
      const double v = A(s)[0];
      if (i >= 1) a.x[i] = v;
      if (i >= 2) sig += v * v;
      if (i == 0) a.d[0] = v;
    }
    sig = block_sum(sig, red);
    if (tid == 0) a.spart[wg] = sig;
  }
  if (!grid_sync(a.bar, a.abort, (++epoch) * G)) return;

  for (int k = 0; k + 2 < n; ++k) {
    const double* xk = a.x + (size_t)(k & 1) * n;
    // reflector scalars (every workgroup, redundantly, same order -> same bits)
    const double sigma = block_sum(tid < G ? a.spart[tid] : 0.0, red);
    const double alpha = xk[k + 1];
    double tau = 0.0, u0 = 0.0, beta = alpha;
    if (sigma > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
      u0 = alpha - beta;
      tau = 2.0 / (u0 * u0 + sigma);
    }
    if (wg == 0 && tid == 0) a.e[k] = beta;
    const bool keep_u = a.U && wg == k % G;  // reflectors kept for the eigenvector back-transform
    if (a.U && wg == 0 && tid == 0) a.tau[k] = tau;
    for (int j = k + 1 + tid; j < n; j += NTHREADS) {
      const double uj = j == k + 1 ? u0 : xk[j];
      uS[j] = uj;
      if (keep_u) a.U[(size_t)k * n + j] = uj;
    }
    __syncthreads();

    // phase A: p_i = tau * A[i][k+1:] . u, one wave per owned row
    double cp = 0.0;
    for (int s = wave; s < a.R; s += NTHREADS / 64) {
      const int i = row_of(s);
      if (i >= n) break;
      if (i <= k) continue;
      double acc = 0.0;
      for (int j = k + 1 + lane; j < n; j += 64) acc += A(s)[j] * uS[j];
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
      acc *= tau;
      if (lane == 0) {
        a.p[i] = acc;
        cp += acc * uS[i];
      }
    }
    cp = block_sum(cp, red);
    if (tid == 0) a.cpart[wg] = cp;
    if (!grid_sync(a.bar, a.abort, (++epoch) * G)) return;

    // phase B: rank-2 update of the owned trailing rows, publish column k+1
    const double K = 0.5 * tau * block_sum(tid < G ? a.cpart[tid] : 0.0, red);
    for (int j = k + 1 + tid; j < n; j += NTHREADS) wS[j] = a.p[j] - K * uS[j];
    __syncthreads();
    for (int s = 0; s < a.R; ++s) {
      const int i = row_of(s);
      if (i >= n) break;
      if (i <= k) continue;
      const double ui = uS[i], wi = wS[i];
      for (int j = k + 1 + tid; j < n; j += NTHREADS) A(s)[j] -= ui * wS[j] + wi * uS[j];
    }
    __syncthreads();
    double* xn = a.x + (size_t)((k + 1) & 1) * n;
    double sig = 0.0;
    for (int s = tid; s < a.R; s += NTHREADS) {
      const int i = row_of(s);
      if (i >= n) continue;
      const double v = A(s)[k + 1];
      if (i == k + 1) a.d[k + 1] = v;
      if (i >= k + 2) xn[i] = v;
      if (i >= k + 3) sig += v * v;
    }
    sig = block_sum(sig, red);
    if (tid == 0) a.spart[wg] = sig;
    if (!grid_sync(a.bar, a.abort, (++epoch) * G)) return;
  }
  // tail: T[n-1][n-1] and T[n-1][n-2] from their owner
  if (n >= 2 && tid == 0) {
    for (int s = 0; s < a.R; ++s) {
      if (row_of(s) == n - 1) {
        a.d[n - 1] = A(s)[n - 1];
        a.e[n - 2] = A(s)[n - 2];
      }
    }
  }
}

// Eigenvalues of the symmetric tridiagonal (d, e) by Sturm-count bisection, one
// thread per eigenvalue index (k-th smallest -> ascending order for free).
__global__ __launch_bounds__(NTHREADS) void eig_bisect(const double* d, const double* e, int n,
                                                       double* evals, const unsigned* abort, int* info) {
  const int k = blockIdx.x * NTHREADS + threadIdx.x;
  if (k == 0 && info) *info = *abort ? -1 : 0;
  if (k >= n) return;
  double lo = 0.0, hi = 0.0, emax2 = 0.0;
  for (int i = 0; i < n; ++i) {
    const double r = (i > 0 ? fabs(e[i - 1]) : 0.0) + (i + 1 < n ? fabs(e[i]) : 0.0);
    lo = i ? fmin(lo, d[i] - r) : d[i] - r;
    hi = i ? fmax(hi, d[i] + r) : d[i] + r;
    if (i + 1 < n) emax2 = fmax(emax2, e[i] * e[i]);
  }
  const double pivmin = 1e-290 * fmax(1.0, emax2);
  const double span = fmax(fabs(lo), fabs(hi));
  lo -= 2.2e-16 * span + pivmin;
  hi += 2.2e-16 * span + pivmin;
  for (int it = 0; it < 200; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (hi - lo <= 2.0 * 2.2e-16 * fmax(fabs(lo), fabs(hi)) + pivmin || mid == lo || mid == hi) break;
    // count of eigenvalues < mid (LDL^T inertia)
    int cnt = 0;
    double q = d[0] - mid;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
    for (int i = 1; i < n; ++i) {
      q = d[i] - mid - e[i - 1] * e[i - 1] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    if (cnt > k) hi = mid; else lo = mid;
  }
  evals[k] = 0.5 * (lo + hi);
}

}  // namespace kfac

using namespace kfac;

// Eigenvectors of the symmetric tridiagonal (d, e) at the bisection eigenvalues w
// (ascending) by inverse iteration (LAPACK dstein's recipe): pivoted LU of
// T - lam I, three solves from a pseudo-random start, normalised each time.
// Eigenvalues closer than 1e-7 ||T||_1 form a cluster, handled by one thread in
// order: lam is nudged apart by 10 eps ||T||_1 and every iterate is
// Gram-Schmidt-orthogonalised against the cluster's earlier vectors.  (dstein's
// 1e-3 threshold would chain a dense spectrum into one serial cluster; in fp64
// inverse iteration keeps vectors with gap g orthogonal to ~eps ||T|| / g, i.e.
// 2e-9 at this threshold, far below the fp32 output's resolution.)
// Layouts are thread-interleaved for coalescing: Z[i * n + j] = element i of
// eigenvector j of T; scratch[a][i][t] (5 arrays, stride `st` threads).
__global__ __launch_bounds__(NTHREADS) void eig_tri_vectors(const double* d, const double* e,
                                                            const double* w, int n, double* Z,
                                                            double* scratch) {
  const int j0 = blockIdx.x * NTHREADS + threadIdx.x;
  const int64_t st = (int64_t)gridDim.x * NTHREADS;
  if (j0 >= n) return;
  double onenrm = 0.0;
  for (int i = 0; i < n; ++i)
    onenrm = fmax(onenrm, fabs(d[i]) + (i > 0 ? fabs(e[i - 1]) : 0.0) + (i + 1 < n ? fabs(e[i]) : 0.0));
  const double ortol = 1e-7 * onenrm, pertol = 10.0 * 2.2e-16 * fmax(onenrm, 1e-300);
  if (j0 > 0 && w[j0] - w[j0 - 1] <= ortol) return;  // a member, not the first of its cluster
  double* U0 = scratch + j0;
  double* U1 = U0 + (int64_t)n * st;
  double* U2 = U1 + (int64_t)n * st;
  double* Lm = U2 + (int64_t)n * st;
  double* Pv = Lm + (int64_t)n * st;
#define S_(a, i) a[(int64_t)(i) * st]
  double xjm = 0.0;
  for (int j = j0; j < n && (j == j0 || w[j] - w[j - 1] <= ortol); ++j) {
    double lam = w[j];
    if (j > j0 && lam - xjm < pertol) lam = xjm + pertol;
    xjm = lam;
    // Gaussian elimination with partial pivoting of T - lam I (U: 3 diagonals)
    double cd = d[0] - lam, cs = n > 1 ? e[0] : 0.0;
    for (int i = 0; i + 1 < n; ++i) {
      const double c = e[i], a1 = d[i + 1] - lam, b1 = i + 2 < n ? e[i + 1] : 0.0;
      double u0;
      if (fabs(c) > fabs(cd)) {
        const double m = cd / c;
        u0 = c; S_(U1, i) = a1; S_(U2, i) = b1; S_(Lm, i) = m; S_(Pv, i) = 1.0;
        cd = cs - m * a1;
        cs = -m * b1;
      } else {
        const double m = cd != 0.0 ? c / cd : 0.0;
        u0 = cd; S_(U1, i) = cs; S_(U2, i) = 0.0; S_(Lm, i) = m; S_(Pv, i) = 0.0;
        cd = a1 - m * cs;
        cs = b1;
      }
      S_(U0, i) = u0 != 0.0 ? u0 : pertol;
    }
    S_(U0, n - 1) = cd != 0.0 ? cd : pertol;
    double* z = Z + j;  // element i at z[i * n]
    for (int i = 0; i < n; ++i) {  // deterministic pseudo-random start in [-1, 1)
      unsigned h = (unsigned)i * 2654435761u ^ ((unsigned)j * 40503u + 0x9e3779b9u);
      h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
      z[(int64_t)i * n] = (double)(h >> 8) * (2.0 / 16777216.0) - 1.0;
    }
    for (int it = 0; it < 3; ++it) {
      double zi = z[0];
      for (int i = 0; i + 1 < n; ++i) {  // apply the row swaps and multipliers
        double zn = z[(int64_t)(i + 1) * n];
        if (S_(Pv, i) != 0.0) { const double t = zi; zi = zn; zn = t; }
        z[(int64_t)i * n] = zi;
        zi = zn - S_(Lm, i) * zi;
      }
      z[(int64_t)(n - 1) * n] = zi;
      double x2 = 0.0, x1 = zi / S_(U0, n - 1);  // back substitution
      z[(int64_t)(n - 1) * n] = x1;
      for (int i = n - 2; i >= 0; --i) {
        const double x = (z[(int64_t)i * n] - S_(U1, i) * x1 - S_(U2, i) * x2) / S_(U0, i);
        z[(int64_t)i * n] = x;
        x2 = x1;
        x1 = x;
      }
      for (int jj = j0; jj < j; ++jj) {  // orthogonalise against the cluster's earlier vectors
        const double* y = Z + jj;
        double dot = 0.0;
        for (int i = 0; i < n; ++i) dot += z[(int64_t)i * n] * y[(int64_t)i * n];
        for (int i = 0; i < n; ++i) z[(int64_t)i * n] -= dot * y[(int64_t)i * n];
      }
      double mx = 0.0;
      for (int i = 0; i < n; ++i) mx = fmax(mx, fabs(z[(int64_t)i * n]));
      const double s1 = mx > 0.0 ? 1.0 / mx : 1.0;
      double nrm = 0.0;
      for (int i = 0; i < n; ++i) {
        const double v = z[(int64_t)i * n] * s1;
        nrm += v * v;
      }
      const double s2 = s1 / sqrt(nrm);
      for (int i = 0; i < n; ++i) z[(int64_t)i * n] *= s2;
    }
  }
#undef S_
}

// Back-transform: v_j = H_0 H_1 ... H_{n-3} z_j (T = Q^T A Q, Q = H_0 ... H_{n-3}).
// Columns are independent, so each block carries 4 eigenvectors through all the
// reflectors in LDS with no grid synchronisation; output fp32 evecs[i][j].
constexpr int BT_VECS = 4;

__global__ __launch_bounds__(NTHREADS) void eig_backtransform(const double* U, const double* tau,
                                                              const double* Z, int n, float* evecs,
                                                              int64_t ldv) {
  extern __shared__ double vs[];  // BT_VECS x n
  __shared__ double red[BT_VECS][NTHREADS / 64];
  const int j0 = blockIdx.x * BT_VECS, tid = threadIdx.x;
  const int nv = min(BT_VECS, n - j0);
  for (int q = 0; q < BT_VECS; ++q)
    for (int i = tid; i < n; i += NTHREADS) vs[q * n + i] = q < nv ? Z[(size_t)i * n + j0 + q] : 0.0;
  __syncthreads();
  for (int k = n - 3; k >= 0; --k) {
    const double t = tau[k];
    if (t == 0.0) continue;  // uniform
    const double* u = U + (size_t)k * n;
    double s[BT_VECS] = {0.0, 0.0, 0.0, 0.0};
    for (int i = k + 1 + tid; i < n; i += NTHREADS) {
      const double ui = u[i];
#pragma unroll
      for (int q = 0; q < BT_VECS; ++q) s[q] += ui * vs[q * n + i];
    }
#pragma unroll
    for (int q = 0; q < BT_VECS; ++q) {
      for (int o = 32; o > 0; o >>= 1) s[q] += __shfl_xor(s[q], o);
      if ((tid & 63) == 0) red[q][tid >> 6] = s[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BT_VECS; ++q) s[q] = t * ((red[q][0] + red[q][1]) + (red[q][2] + red[q][3]));
    for (int i = k + 1 + tid; i < n; i += NTHREADS) {
      const double ui = u[i];
#pragma unroll
      for (int q = 0; q < BT_VECS; ++q) vs[q * n + i] -= s[q] * ui;
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += NTHREADS)
    for (int q = 0; q < nv; ++q) evecs[(int64_t)i * ldv + j0 + q] = (float)vs[q * n + i];
}

// n > EIG_LDS_MAX: tridiagonalisation plan (grid, rows per workgroup, row storage)
struct TriPlan {
  int G, R;
  bool lds_rows;
  size_t shmem, ws;
};
constexpr size_t TRI_LDS_BUDGET = 150 * 1024;

static TriPlan tri_plan(int n, bool vecs) {
  TriPlan p;
  p.G = std::min(256, std::max(1, (n + 7) / 8));
  p.R = (n + p.G - 1) / p.G;
  p.lds_rows = (size_t)(2 + p.R) * n * sizeof(double) <= TRI_LDS_BUDGET;
  p.shmem = (size_t)(p.lds_rows ? 2 + p.R : 2) * n * sizeof(double);
  p.ws = 256                                                    // bar, abort (+pad)
         + align_up((size_t)2 * n * sizeof(double), 256)        // x
         + 3 * align_up((size_t)n * sizeof(double), 256)        // p, d, e
         + 2 * align_up(256 * sizeof(double), 256)              // cpart, spart
         + (p.lds_rows ? 0 : align_up((size_t)p.G * p.R * n * sizeof(double), 256))
         + (vecs ? 2 * align_up((size_t)n * n * sizeof(double), 256)  // U, Z
                       + 5 * align_up((size_t)n * cdiv(n, NTHREADS) * NTHREADS * sizeof(double), 256)
                       + align_up((size_t)n * sizeof(double), 256)    // tau
                 : 0);
  return p;
}

static int tridiag_eig(const kfac_eig_job& j, char* ws, int32_t* info, hipStream_t stream) {
  const bool vecs = j.evecs != nullptr;
  const TriPlan pl = tri_plan(j.n, vecs);
  if (pl.shmem > TRI_LDS_BUDGET) return KFAC_EINVAL;
  TriArgs t{};
  t.F = j.F; t.ldF = j.ldF; t.n = j.n; t.G = pl.G; t.R = pl.R;
  t.bar = reinterpret_cast<unsigned*>(ws);
  t.abort = t.bar + 1;
  char* q = ws + 256;
  t.x = reinterpret_cast<double*>(q); q += align_up((size_t)2 * j.n * sizeof(double), 256);
  t.p = reinterpret_cast<double*>(q); q += align_up((size_t)j.n * sizeof(double), 256);
  t.d = reinterpret_cast<double*>(q); q += align_up((size_t)j.n * sizeof(double), 256);
  t.e = reinterpret_cast<double*>(q); q += align_up((size_t)j.n * sizeof(double), 256);
  t.cpart = reinterpret_cast<double*>(q); q += align_up(256 * sizeof(double), 256);
  t.spart = reinterpret_cast<double*>(q); q += align_up(256 * sizeof(double), 256);
  t.rows_g = pl.lds_rows ? nullptr : reinterpret_cast<double*>(q);
  if (!pl.lds_rows) q += align_up((size_t)pl.G * pl.R * j.n * sizeof(double), 256);
  double *Z = nullptr, *scratch = nullptr;
  if (vecs) {
    const size_t nn = align_up((size_t)j.n * j.n * sizeof(double), 256);
    t.U = reinterpret_cast<double*>(q); q += nn;
    Z = reinterpret_cast<double*>(q); q += nn;
    scratch = reinterpret_cast<double*>(q);
    q += 5 * align_up((size_t)j.n * cdiv(j.n, NTHREADS) * NTHREADS * sizeof(double), 256);
    t.tau = reinterpret_cast<double*>(q);
    // reflector rows start zero below their support (the back-transform reads u[k+1..])
    if (hipMemsetAsync(t.tau, 0, (size_t)j.n * sizeof(double), stream) != hipSuccess) return KFAC_ELAUNCH;
  }
  if (hipMemsetAsync(ws, 0, 16, stream) != hipSuccess) return KFAC_ELAUNCH;
  const void* fn = pl.lds_rows ? reinterpret_cast<const void*>(&eig_tridiag<true>)
                               : reinterpret_cast<const void*>(&eig_tridiag<false>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.shmem) != hipSuccess)
    return KFAC_ELAUNCH;
  void* kargs[] = {&t};
  // cooperative: the runtime rejects a grid that cannot be co-resident (no deadlock)
  if (hipLaunchCooperativeKernel(fn, dim3(pl.G), dim3(NTHREADS), kargs, (unsigned)pl.shmem, stream) !=
      hipSuccess)
    return KFAC_ELAUNCH;
  hipLaunchKernelGGL(eig_bisect, dim3((j.n + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, stream,
                     t.d, t.e, j.n, j.evals, t.abort, info);
  KFAC_CHECK_LAUNCH();
  if (vecs) {
    hipLaunchKernelGGL(eig_tri_vectors, dim3((j.n + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0,
                       stream, t.d, t.e, j.evals, j.n, Z, scratch);
    KFAC_CHECK_LAUNCH();
    const size_t sh = (size_t)BT_VECS * j.n * sizeof(double);
    if (sh > TRI_LDS_BUDGET) return KFAC_EINVAL;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&eig_backtransform),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh) != hipSuccess)
      return KFAC_ELAUNCH;
    hipLaunchKernelGGL(eig_backtransform, dim3((j.n + BT_VECS - 1) / BT_VECS), dim3(NTHREADS), sh,
                       stream, t.U, t.tau, Z, j.n, j.evecs, j.ldv);
    KFAC_CHECK_LAUNCH();
  }
  return KFAC_OK;
}

extern "C" size_t kfac_eig_workspace_bytes(const kfac_eig_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  // small factors run grouped (V per job); large ones one at a time (stream-ordered reuse)
  size_t best = 0, tot = 0;
  int in_group = 0;
  for (int i = 0; i < njobs; ++i) {
    if (jobs[i].n > EIG_LDS_MAX) {
      best = std::max(best, tri_plan(jobs[i].n, jobs[i].evecs != nullptr).ws);
      continue;
    }
    if (in_group == EMAXJ) { best = std::max(best, tot); tot = 0; in_group = 0; }
    tot += align_up((size_t)jobs[i].n * jobs[i].n * sizeof(double), 256);
    ++in_group;
  }
  return std::max(best, tot);
}

extern "C" int kfac_syev(const kfac_eig_job* jobs, int njobs, void* workspace, size_t workspace_bytes,
                         int32_t* info, kfac_stream_t stream) {
  if (njobs <= 0 || !jobs) return KFAC_EINVAL;
  for (int i = 0; i < njobs; ++i) {
    const kfac_eig_job& j = jobs[i];
    if (!j.F || !j.evals || j.n <= 0 || j.ldF < j.n || (j.evecs && j.ldv < j.n)) return KFAC_EINVAL;
  }
  if (workspace_bytes < kfac_eig_workspace_bytes(jobs, njobs)) return KFAC_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  EigArgs args{};
  char* ws = (char*)workspace;
  auto flush = [&]() -> int {
    if (args.njobs == 0) return KFAC_OK;
    hipLaunchKernelGGL(eig_jacobi_lds, dim3(args.njobs), dim3(NTHREADS), 0, st, args);
    KFAC_CHECK_LAUNCH();
    args = EigArgs{};
    ws = (char*)workspace;
    return KFAC_OK;
  };
  for (int i = 0; i < njobs; ++i) {
    const kfac_eig_job& j = jobs[i];
    if (j.n > EIG_LDS_MAX) {
      int rc = flush();  // the small group owns the workspace until its launch is queued
      if (rc != KFAC_OK) return rc;
      rc = tridiag_eig(j, (char*)workspace, info ? info + i : nullptr, st);
      if (rc != KFAC_OK) return rc;
      continue;
    }
    if (args.njobs == EMAXJ) {
      const int rc = flush();
      if (rc != KFAC_OK) return rc;
    }
    EigJobDev& d = args.job[args.njobs++];
    d.F = j.F; d.ldF = j.ldF; d.n = j.n; d.evals = j.evals; d.evecs = j.evecs; d.ldv = j.ldv;
    d.V = j.evecs ? reinterpret_cast<double*>(ws) : nullptr;
    ws += align_up((size_t)j.n * j.n * sizeof(double), 256);
    d.info = info ? info + i : nullptr;
  }
  const int rc = flush();
  if (rc != KFAC_OK) return rc;
  return KFAC_OK;
}
