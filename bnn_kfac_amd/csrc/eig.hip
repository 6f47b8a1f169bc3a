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
#include <stdlib.h>

#include <algorithm>
#include <vector>
#include <stdio.h>

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
// eig_tridiag: ONE persistent launch per factor, ONE grid-wide exchange per
// reflector.  G workgroups, row i owned by workgroup i % G (slot i / G), the owned
// rows kept in LDS (fp64, symmetrised) when they fit, else in a global slab only
// their owner touches.  Every workgroup holds the full vectors x (the column the
// next reflector comes from), u and w in LDS.  Step k:
//   1. (every workgroup, redundantly, same bits) reflector u, tau from x;
//   2. (own rows i > k) ONE pass over the row: apply the previous step's rank-2
//      update lazily (A[i][j] -= u'_i w'_j + w'_i u'_j), read a_i = A_k[i][k+1] and
//      p_i = tau * A_k[i][k+1:] . u;
//   3. exchange: publish (p_i, a_i) and c_wg = sum p_i u_i; read everyone's;
//   4. (every workgroup) w = p - (tau c / 2) u and the next column
//      x'_i = a_i - u_i w_{k+1} - w_i u_{k+1}, its sigma for step k+1.
// (The row pass of step k+1 applies (u, w) to the rows.)
//
// The exchange is the data-tagged granule form of the MI355X in-launch hand-off
// (no flag, no fence): every published 32-bit half of a fp64 value travels as ONE
// aligned 8-byte {tag = epoch, bits} granule written by one `sc1` store; a reader
// re-reads its granules with `sc1` loads until every tag equals the step's epoch.
// Granules are double-buffered by step parity (a workgroup publishes step k+1 only
// after it has seen every workgroup's step-k granules, i.e. after every workgroup
// finished reading step k-1's).  All granules are zeroed before the launch (epochs
// start at 1).  Waits are bounded (1 s): a timeout sets `abort`, and every
// workgroup leaves at its next wait (the launch drains; info = -1).

typedef __attribute__((address_space(1))) unsigned long long eg_u64;
typedef __attribute__((address_space(1))) unsigned eg_unsigned;
typedef unsigned long long gran_t;
__device__ __forceinline__ void st_gran(gran_t* g, unsigned tag, unsigned bits) {
  __hip_atomic_store((eg_u64*)g, ((gran_t)tag << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_gran_d(gran_t* g, unsigned tag, double v) {  // 2 granules
  const gran_t b = (gran_t)__double_as_longlong(v);
  st_gran(g, tag, (unsigned)b);
  st_gran(g + 1, tag, (unsigned)(b >> 32));
}
__device__ __forceinline__ gran_t ld_gran(const gran_t* g) {
  return __hip_atomic_load((eg_u64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Two granules (one fp64 value) by ONE 16-byte `sc1` buffer load (aux 16 = sc1);
// each 8-byte half is checked by its own tag.
typedef unsigned gv4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ld_gran2(__amdgpu_buffer_rsrc_t rs, int off_bytes, gran_t& g0, gran_t& g1) {
  const gv4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, off_bytes, 0, 16);
  g0 = ((gran_t)v.y << 32) | v.x;
  g1 = ((gran_t)v.w << 32) | v.z;
}
__device__ __forceinline__ double gran_d(gran_t lo, gran_t hi) {
  return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
}
__device__ __forceinline__ bool gran_ok(gran_t g, unsigned tag) { return (unsigned)(g >> 32) == tag; }
__device__ __forceinline__ unsigned ldu_ag(const unsigned* p) {
  return __hip_atomic_load((eg_unsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stu_ag(unsigned* p, unsigned v) {
  __hip_atomic_store((eg_unsigned*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave's spin bookkeeping (wave-uniform): false once the launch is aborted or
// this wave's deadline has passed (then it sets the abort word).
struct Spin {
  uint64_t deadline = 0;
  unsigned spins = 0;
  // the abort word and the clock are read every 8th spin only (a spin is one sweep
  // of the granules; the first deadline is set at the first check)
  __device__ bool again(unsigned* abort) {
    if ((++spins & 7u) == 0u) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (deadline == 0) deadline = now + 100000000ull;  // 1 s at 100 MHz
      if (__builtin_amdgcn_readfirstlane(ldu_ag(abort)) != 0u) return false;
      if (now > deadline) {
        stu_ag(abort, 1u);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
    return true;
  }
};

struct TriArgs {
  const float* F;
  int64_t ldF;
  int n, G, R;         // rows per workgroup R = ceil(n / G)
  double* rows_g;      // G x R x n owned rows when they do not fit LDS (else null)
  double* vecs_g;      // G x 3n: each workgroup's x / u / w vectors when 3n doubles do not
                       // fit LDS (n > 6400; else null)
  gran_t* pub;         // 2 (step parity) x n x 4 granules {p lo, p hi, a lo, a hi}
  unsigned* abort;     // timeout flag
  double* d;           // n: diagonal of T
  double* e;           // n: off-diagonal of T (e[k] = T[k+1][k])
  double* U;           // n x n: row k = reflector u_k (entries k+1..n-1), or null
  double* tau;         // n: reflector scales (0: no reflection), or null
};

// Wave sum in registers (no LDS crossbar): quad_perm xor 1 / xor 2 and row_ror 4 / 8
// DPP within each 16-lane row, then permlane16_swap / permlane32_swap across rows.
// Lane 0's value is the one used (lanes may associate differently); the same tree
// runs in every workgroup -> bit-identical scalars everywhere.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x124>(v);  // row_ror:4
  v += dpp_d<0x128>(v);  // row_ror:8
  unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const auto pl = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  const auto ph = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  v = __builtin_bit_cast(double, ((unsigned long long)ph[0] << 32) | pl[0]) +
      __builtin_bit_cast(double, ((unsigned long long)ph[1] << 32) | pl[1]);
  b = __builtin_bit_cast(unsigned long long, v);
  const auto ql = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto qh = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return __builtin_bit_cast(double, ((unsigned long long)qh[0] << 32) | ql[0]) +
         __builtin_bit_cast(double, ((unsigned long long)qh[1] << 32) | ql[1]);
}

// fixed pairwise tree over W per-wave values (the same in every workgroup)
template <int W, class F>
__device__ __forceinline__ double wsum(F f) {
  if constexpr (W == 4) {
    return (f(0) + f(1)) + (f(2) + f(3));
  } else {
    double t[W];
#pragma unroll
    for (int w = 0; w < W; ++w) t[w] = f(w);
#pragma unroll
    for (int h = W / 2; h > 0; h >>= 1)
#pragma unroll
      for (int w = 0; w < h; ++w) t[w] += t[w + h];
    return t[0];
  }
}
template <int W>
__device__ __forceinline__ double block_sum_w(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return wsum<W>([&](int w) { return red[w]; });
}
template <int W>
__device__ __forceinline__ double block_sum1_w(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return wsum<W>([&](int w) { return red[w]; });
}

// one barrier: the caller guarantees a barrier between the reads of `red` here and
// the next write of the same slot
__device__ __forceinline__ double block_sum1(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

constexpr int TRI_CH = 8;  // columns per thread per sweep (4 granules each)

template <bool LDS_ROWS, int RB, bool VEC_LDS = true>
__global__ __launch_bounds__(NTHREADS) void eig_tridiag(TriArgs a) {
  constexpr int TB = NTHREADS, W = TB / 64, CH = TRI_CH;
  // [v0 n][v1 n][w n][rows R x n if LDS_ROWS]; without VEC_LDS (n > 6400: 3n doubles
  // exceed the LDS budget) the vectors are this workgroup's private global slab
  extern __shared__ double lds_dyn[];
  double* lds = VEC_LDS ? lds_dyn : a.vecs_g + (size_t)blockIdx.x * 3 * a.n;
  __shared__ double red[TB / 64];
  __shared__ int fail_s;
  const int n = a.n, G = a.G, wg = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  // x / u share a slot (u is built in place from x); the previous u is the other
  // slot; w is rewritten after each row pass (the previous w is dead by then)
  double* vs[2] = {lds, lds + n};
  double* wS = lds + 2 * n;
  double* rows = LDS_ROWS ? lds_dyn + (VEC_LDS ? 3 * n : 0) : a.rows_g + (size_t)wg * a.R * n;
  auto row_of = [&](int slot) { return slot * G + wg; };
  auto A = [&](int slot) { return rows + (size_t)slot * n; };
  if (tid == 0) fail_s = 0;
  for (int j = tid; j < n; j += TB) {  // the "previous step" of step 0: u = w = 0
    vs[1][j] = 0.0;
    wS[j] = 0.0;
  }

  // load + symmetrise the owned rows; publish column 0 (epoch 1, parity 1: step 0
  // publishes into parity 0)
  for (int s = 0; s < a.R; ++s) {
    const int i = row_of(s);
    if (i >= n) break;
    for (int j = tid; j < n; j += TB)
      A(s)[j] = 0.5 * ((double)a.F[(int64_t)i * a.ldF + j] + (double)a.F[(int64_t)j * a.ldF + i]);
  }
  __syncthreads();
  gran_t* pub1 = a.pub + (size_t)4 * n;
  for (int s = tid; s < a.R; s += TB) {
    const int i = row_of(s);
    if (i < n) st_gran_d(pub1 + 4 * (size_t)i + 2, 1u, A(s)[0]);
  }
  double* x = vs[0];
  double sig = 0.0;
  {
    Spin sp;
    for (int j0 = 0; j0 < n; j0 += CH * TB) {
      gran_t g[CH][2];
      bool ok;
      for (;;) {
        ok = true;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const int j = j0 + c * TB + tid;
          if (j < n) {
            g[c][0] = ld_gran(pub1 + 4 * (size_t)j + 2);
            g[c][1] = ld_gran(pub1 + 4 * (size_t)j + 3);
            ok = ok && gran_ok(g[c][0], 1u) && gran_ok(g[c][1], 1u);
          }
        }
        if (__builtin_amdgcn_readfirstlane(__all(ok))) break;
        if (!sp.again(a.abort)) break;
      }
      if (!__builtin_amdgcn_readfirstlane(__all(ok))) {
        if (lane == 0) fail_s = 1;
        break;
      }
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int j = j0 + c * TB + tid;
        if (j < n) {
          const double v = gran_d(g[c][0], g[c][1]);
          x[j] = v;
          if (j >= 2) sig += v * v;
        }
      }
    }
  }
  double sigma = block_sum_w<W>(sig, red);  // (its barriers also publish x and fail_s)
  if (fail_s) return;
  if (wg == 0 && tid == 0) a.d[0] = x[0];
  double* up = vs[1];  // previous step's u (unused at k = 0)

  __shared__ double rp[2][TB / 64][RB];  // per-wave partial dots of a row batch (batch parity)
  __shared__ double p1_s;
  __shared__ double red2[TB / 64];           // block_sum slot of the sigma reduction
  const __amdgpu_buffer_rsrc_t pub_rs =
      __builtin_amdgcn_make_buffer_rsrc(a.pub, 0, (int)(2 * 4 * (size_t)n * sizeof(gran_t)), 0x00020000);
  for (int k = 0; k + 2 < n; ++k) {
    const unsigned tag = (unsigned)k + 2u;
    gran_t* pub = a.pub + (size_t)(k & 1) * 4 * n;
    // 1. reflector (every workgroup, redundantly, same order -> same bits)
    const double alpha = x[k + 1];
    double tau = 0.0, u0 = 0.0, beta = alpha;
    if (sigma > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
      u0 = alpha - beta;
      tau = 2.0 / (u0 * u0 + sigma);
    }
    // u_j = x_j for j >= k+2 (the x slot is read as u); u_{k+1} = u0 stays in a
    // register (no barrier: nothing reads u[k+1] from LDS, and the next step's row
    // pass reads its previous u only at rows / columns >= k+2)
    const double* u = x;
    auto u_at = [&](int j) { return j == k + 1 ? u0 : u[j]; };
    if (wg == 0 && tid == 0) {
      a.e[k] = beta;
      if (a.U) a.tau[k] = tau;
    }
    if (a.U && wg == k % G)  // reflectors kept for the eigenvector back-transform
      for (int j = k + 1 + tid; j < n; j += TB) a.U[(size_t)k * n + j] = u_at(j);

    // 2. row pass, thread per column, RB owned rows at a time: the lazy rank-2
    //    update of step k-1, then a_i (column k+1) and p_i = tau A_k[i][k+1:] . u
    //    (per-thread partials, wave shuffles, one barrier per batch)
    const int s_lo = k + 1 > wg ? (k + 1 - wg + G - 1) / G : 0;  // first slot with row > k
    for (int s0 = s_lo, bp = 0; s0 < a.R; s0 += RB, bp ^= 1) {
      // a batch past the last slot repeats the last slot (read-before-write per column,
      // so the repeat writes the same values); slots whose row is >= n hold unused
      // rows.  Their results are never published.  (up / wS start zero: the k = 0
      // "update" subtracts nothing.)
      double acc[RB], upi[RB], wsi[RB];
      double* Ar[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int sl = min(s0 + r, a.R - 1);
        const int i = min(row_of(sl), n - 1);  // (an unused slot's row: any valid index)
        Ar[r] = A(sl);
        upi[r] = up[i];
        wsi[r] = wS[i];
        acc[r] = 0.0;
      }
      for (int j = k + 1 + tid; j < n; j += TB) {
        const double uj = u_at(j), upj = up[j], wj = wS[j];
        double v[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) v[r] = Ar[r][j];  // every load first
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          v[r] -= upi[r] * wj + wsi[r] * upj;
          Ar[r][j] = v[r];
          acc[r] += v[r] * uj;
        }
      }
      if constexpr (W == 1) {
        // one wave: lane 0 holds the sums and wrote column k+1 itself; no barrier
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const double v = wave_sum(acc[r]);
          if (lane == 0 && s0 + r < a.R && row_of(s0 + r) < n) {
            const int i = row_of(s0 + r);
            st_gran_d(pub + 4 * (size_t)i, tag, tau * v);
            st_gran_d(pub + 4 * (size_t)i + 2, tag, Ar[r][k + 1]);
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const double v = wave_sum(acc[r]);
          if (lane == 0) rp[bp][wave][r] = v;
        }
        __syncthreads();  // (the next batch writes the other parity: one barrier per batch)
        if (tid < RB && s0 + tid < a.R && row_of(s0 + tid) < n) {
          const int i = row_of(s0 + tid);
          const double pi = tau * (wsum<W>([&](int w) { return rp[bp][w][tid]; }));
          st_gran_d(pub + 4 * (size_t)i, tag, pi);
          st_gran_d(pub + 4 * (size_t)i + 2, tag, A(s0 + tid)[k + 1]);
        }
      }
    }

    // 3. exchange: every (p_j, a_j), j > k; c = sum p_j u_j from the gathered p
    //    (same tree in every workgroup), then w_j, x'_j.  Up to CH columns per
    //    thread per sweep; the last sweep's granules stay in registers.
    gran_t g[CH][4];
    double cs = 0.0;
    const int nch = (n - (k + 1) + CH * TB - 1) / (CH * TB);
    {
      Spin sp;
      for (int ch = 0; ch < nch; ++ch) {
        const int j0 = k + 1 + ch * CH * TB;
        bool ok;
        for (;;) {
          ok = true;
#pragma unroll
          for (int cc = 0; cc < CH; ++cc) {
            const int j = j0 + cc * TB + tid;
            if (j < n) {
              const int off = (int)(((size_t)(k & 1) * 4 * n + 4 * (size_t)j) * sizeof(gran_t));
              ld_gran2(pub_rs, off, g[cc][0], g[cc][1]);
              ld_gran2(pub_rs, off + 16, g[cc][2], g[cc][3]);
#pragma unroll
              for (int h = 0; h < 4; ++h) ok = ok && gran_ok(g[cc][h], tag);
            }
          }
          if (__builtin_amdgcn_readfirstlane(__all(ok))) break;
          if (!sp.again(a.abort)) break;
        }
        if (!__builtin_amdgcn_readfirstlane(__all(ok))) {
          if (lane == 0) fail_s = 1;
          break;
        }
#pragma unroll
        for (int cc = 0; cc < CH; ++cc) {
          const int j = j0 + cc * TB + tid;
          if (j < n) {
            const double pj = gran_d(g[cc][0], g[cc][1]);
            cs += pj * u_at(j);
            if (j == k + 1) p1_s = pj;
          }
        }
      }
    }
    const double c = block_sum1_w<W>(cs, red);  // (its barrier also publishes p1_s and fail_s)
    if (fail_s) return;
    const double K = 0.5 * tau * c;
    const double u1 = u0;
    const double w1 = p1_s - K * u1;
    double* xn = up;  // the previous u's slot is dead now
    sig = 0.0;
    for (int q = 0; q < nch; ++q) {
      // the last chunk first (its granules are still in registers), then the others
      // reloaded (arrived and checked in the sweep)
      const int ch = q == 0 ? nch - 1 : q - 1;
      const int j0 = k + 1 + ch * CH * TB;
      if (q > 0) {
#pragma unroll
        for (int cc = 0; cc < CH; ++cc) {
          const int j = j0 + cc * TB + tid;
          if (j < n) {
            const int off = (int)(((size_t)(k & 1) * 4 * n + 4 * (size_t)j) * sizeof(gran_t));
            ld_gran2(pub_rs, off, g[cc][0], g[cc][1]);
            ld_gran2(pub_rs, off + 16, g[cc][2], g[cc][3]);
          }
        }
      }
#pragma unroll
      for (int cc = 0; cc < CH; ++cc) {
        const int j = j0 + cc * TB + tid;
        if (j < n) {
          const double uj = u_at(j);
          const double wj = gran_d(g[cc][0], g[cc][1]) - K * uj;
          const double xj = gran_d(g[cc][2], g[cc][3]) - (uj * w1 + wj * u1);
          wS[j] = wj;
          xn[j] = xj;
          if (j >= k + 3) sig += xj * xj;
        }
      }
    }
    // every wave is past its row pass (the c barrier), so wS / xn could be rewritten
    // above; the sigma barrier publishes them (and separates this step's reads of
    // `red` / `red2` from the next step's writes of the other slot)
    sigma = block_sum1_w<W>(sig, red2);
    if (wg == 0 && tid == 0) a.d[k + 1] = xn[k + 1];
    up = x;
    x = xn;
  }
  // tail: T[n-1][n-2] is the last column's sub-diagonal entry; T[n-1][n-1] is row
  // n-1's diagonal with the last step's update applied (by its owner)
  if (wg == 0 && tid == 0) a.e[n - 2] = x[n - 1];
  if (tid == 0) {
    for (int s = 0; s < a.R; ++s) {
      if (row_of(s) == n - 1) a.d[n - 1] = A(s)[n - 1] - 2.0 * up[n - 1] * wS[n - 1];
    }
  }
}

// Eigenvalues of the symmetric tridiagonal (d, e) by Sturm-count multisection:
// ONE wave per eigenvalue index k (the k-th smallest -> ascending order for free).
// Each round the 64 lanes count the eigenvalues below 64 interior points of the
// current interval [lo, hi] (LDL^T inertia, one lane per point) and the interval
// shrinks to the 1/65 slice where the count crosses k: ~9 rounds of one O(n)
// recurrence reach fp64 resolution, where one-point bisection needs ~55 (the
// recurrence is a chain of dependent fp64 divisions, so rounds, not flops, are the
// cost).  d and e^2 are staged in LDS once per workgroup.
template <bool SH>
__global__ __launch_bounds__(NTHREADS) void eig_bisect(const double* d, const double* e, int n,
                                                       double* evals, const unsigned* abort, int* info) {
  // [d n][e^2 n] in LDS; without SH (n > 9600) d and e are read from global memory
  // (every lane of a wave reads the same element: one broadcast access) and e^2 is
  // formed in the loop
  extern __shared__ double sh[];
  double* dS = sh;
  double* e2S = sh + n;
  __shared__ double red[2][NTHREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63;
  if (blockIdx.x == 0 && tid == 0 && info) *info = *abort ? -1 : 0;
  double lo = 0.0, hi = 0.0, emax2 = 0.0;
  for (int i = tid; i < n; i += NTHREADS) {
    const double di = d[i], ei = i + 1 < n ? e[i] : 0.0;
    if (SH) {
      dS[i] = di;
      e2S[i] = ei * ei;
    }
    const double r = (i > 0 ? fabs(e[i - 1]) : 0.0) + fabs(ei);
    lo = i == tid ? di - r : fmin(lo, di - r);
    hi = i == tid ? di + r : fmax(hi, di + r);
    emax2 = fmax(emax2, ei * ei);
  }
  // Gershgorin bounds over the whole matrix (lanes without rows contribute nothing)
  const bool any = tid < n;
  double glo = any ? lo : INFINITY, ghi = any ? hi : -INFINITY;
  for (int o = 32; o > 0; o >>= 1) {
    glo = fmin(glo, __shfl_xor(glo, o));
    ghi = fmax(ghi, __shfl_xor(ghi, o));
    emax2 = fmax(emax2, __shfl_xor(emax2, o));
  }
  if (lane == 0) {
    red[0][tid >> 6] = glo;
    red[1][tid >> 6] = ghi;
  }
  __shared__ double em_s[NTHREADS / 64];
  if (lane == 0) em_s[tid >> 6] = emax2;
  __syncthreads();
  lo = fmin(fmin(red[0][0], red[0][1]), fmin(red[0][2], red[0][3]));
  hi = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
  emax2 = fmax(fmax(em_s[0], em_s[1]), fmax(em_s[2], em_s[3]));
  const int k = blockIdx.x * (NTHREADS / 64) + (tid >> 6);
  if (k >= n) return;  // (wave-uniform; no barrier follows)
  const double pivmin = 1e-290 * fmax(1.0, emax2);
  const double span = fmax(fabs(lo), fabs(hi));
  lo -= 2.2e-16 * span + pivmin;
  hi += 2.2e-16 * span + pivmin;
  for (int it = 0; it < 40; ++it) {
    if (hi - lo <= 2.0 * 2.2e-16 * fmax(fabs(lo), fabs(hi)) + pivmin) break;
    const double step = (hi - lo) * (1.0 / 65.0);
    const double mid = lane == 63 ? hi - step : lo + step * (double)(lane + 1);
    // count of eigenvalues < mid (LDL^T inertia)
    int cnt = 0;
    double q = (SH ? dS[0] : d[0]) - mid;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
    for (int i = 1; i < n; ++i) {
      // e^2 / q by v_rcp_f64 + two Newton steps (|q| >= pivmin, so no 0 / inf
      // cases; the division's scaling / fixup steps are not needed): a few-ulp
      // quotient, under which the inertia count stays backward stable
      double r = __builtin_amdgcn_rcp(q);
      r = fma(r, fma(-q, r, 1.0), r);
      r = fma(r, fma(-q, r, 1.0), r);
      q = SH ? (dS[i] - mid) - e2S[i - 1] * r : (d[i] - mid) - (e[i - 1] * e[i - 1]) * r;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    const unsigned long long above = __ballot(cnt > k);  // lanes whose point is above eigenvalue k
    const int first = above ? __builtin_ctzll(above) : 64;
    const double nlo = first == 0 ? lo : __shfl(mid, first - 1);
    const double nhi = first == 64 ? hi : __shfl(mid, first == 64 ? 0 : first);
    if (nlo == lo && nhi == hi) break;  // no representable progress
    lo = nlo;
    hi = nhi;
  }
  if (lane == 0) evals[k] = 0.5 * (lo + hi);
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
// V vectors per block.  VS_LDS: the V columns staged in LDS (8 V n bytes: V = 4 up to
// n = 4800, 2 up to 9600, 1 up to 19200); beyond that the one column is updated in
// place in Z (strided, uncached -- n > 19200 is far past any layer the reference's
// scripts build)
template <int V, bool VS_LDS>
__global__ __launch_bounds__(NTHREADS) void eig_backtransform(const double* U, const double* tau,
                                                              double* Z, int n, float* evecs,
                                                              int64_t ldv) {
  extern __shared__ double vs_dyn[];
  __shared__ double red[V][NTHREADS / 64];
  const int j0 = blockIdx.x * V, tid = threadIdx.x;
  const int nv = min(V, n - j0);
  auto vs = [&](int q, int i) -> double& {
    return VS_LDS ? vs_dyn[q * n + i] : Z[(size_t)i * n + j0 + q];
  };
  if (VS_LDS) {
    for (int q = 0; q < V; ++q)
      for (int i = tid; i < n; i += NTHREADS) vs(q, i) = q < nv ? Z[(size_t)i * n + j0 + q] : 0.0;
    __syncthreads();
  }
  for (int k = n - 3; k >= 0; --k) {
    const double t = tau[k];
    if (t == 0.0) continue;  // uniform
    const double* u = U + (size_t)k * n;
    double s[V];
#pragma unroll
    for (int q = 0; q < V; ++q) s[q] = 0.0;
    for (int i = k + 1 + tid; i < n; i += NTHREADS) {
      const double ui = u[i];
#pragma unroll
      for (int q = 0; q < V; ++q) s[q] += ui * vs(q, i);
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
      for (int o = 32; o > 0; o >>= 1) s[q] += __shfl_xor(s[q], o);
      if ((tid & 63) == 0) red[q][tid >> 6] = s[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < V; ++q) s[q] = t * ((red[q][0] + red[q][1]) + (red[q][2] + red[q][3]));
    for (int i = k + 1 + tid; i < n; i += NTHREADS) {
      const double ui = u[i];
#pragma unroll
      for (int q = 0; q < V; ++q) vs(q, i) -= s[q] * ui;
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += NTHREADS)
    for (int q = 0; q < nv; ++q) evecs[(int64_t)i * ldv + j0 + q] = (float)vs(q, i);
}

// n > EIG_LDS_MAX: tridiagonalisation plan (grid, rows per workgroup, row storage).
// Rows in LDS when some G <= 256 fits them: the fewest workgroups that do (the
// exchange's cost grows with G, the row pass's shrinks; env KFAC_EIG_G overrides
// within what fits).  Otherwise 256 workgroups with the rows in a global slab.
struct TriPlan {
  int G, R, RB;  // workgroups, rows per workgroup, rows per row-pass batch
  bool lds_rows;
  bool vec_lds;  // the 3n vector doubles fit LDS (n <= 6400); else a global slab per workgroup
  size_t shmem, ws;
};
constexpr size_t TRI_LDS_BUDGET = 150 * 1024;


// the block zeroed before every launch: abort word, then the granules
static size_t tri_zero_bytes(int n) {
  return 256 + align_up((size_t)2 * 4 * n * sizeof(gran_t), 256);  // pub: 2 parities x n x 4
}

static TriPlan tri_plan(int n, bool vecs) {
  TriPlan p;
  const size_t vec_bytes = (size_t)3 * n * sizeof(double);
  p.vec_lds = vec_bytes <= TRI_LDS_BUDGET;
  const size_t vec = p.vec_lds ? vec_bytes : 0;
  const size_t row = (size_t)n * sizeof(double);
  // vectors in global memory (n > 6400) leave at most 2 rows per workgroup of LDS: the
  // rows go to the global slab too
  const int rmax = p.vec_lds && vec < TRI_LDS_BUDGET ? (int)((TRI_LDS_BUDGET - vec) / row) : 0;
  const int gmin = rmax > 0 ? (n + rmax - 1) / rmax : 1 << 30;
  p.lds_rows = gmin <= 256;
  if (p.lds_rows) {
    // ~8 rows per workgroup (two row-pass batches): n = 785 -> 99 workgroups.  Measured
    // per step at 785 (tools/gpu/eig_clk.sh): G = 64 / 96 / 128 / 160 / 256 ->
    // 5.1 / 4.8 / 4.8 / 5.2 / 5.2 us (fewer rows per workgroup shorten the row pass,
    // more workgroups lengthen the exchange)
    p.G = std::max(gmin, std::min(256, (n + 7) / 8));
    if (knobs().eig_g > 0) p.G = std::max(gmin, std::min(1024, knobs().eig_g));
  } else {
    p.G = 256;
  }
  p.R = (n + p.G - 1) / p.G;
  p.RB = knobs().eig_rb;  // 4 rows per batch (default) measured faster at every G tried
  p.shmem = vec + (p.lds_rows ? (size_t)p.R * row : 0);
  p.ws = tri_zero_bytes(n)                                       // abort + granules
         + 2 * align_up((size_t)n * sizeof(double), 256)         // d, e
         + (p.lds_rows ? 0 : align_up((size_t)p.G * p.R * n * sizeof(double), 256))
         + (p.vec_lds ? 0 : align_up((size_t)p.G * 3 * n * sizeof(double), 256))
         + (vecs ? 2 * align_up((size_t)n * n * sizeof(double), 256)  // U, Z
                       + 5 * align_up((size_t)n * cdiv(n, NTHREADS) * NTHREADS * sizeof(double), 256)
                       + align_up((size_t)n * sizeof(double), 256)    // tau
                 : 0);
  return p;
}

static int tridiag_eig(const kfac_eig_job& j, char* ws, int32_t* info, hipStream_t stream) {
  const bool vecs = j.evecs != nullptr;
  const TriPlan pl = tri_plan(j.n, vecs);
  if (pl.shmem > TRI_LDS_BUDGET) return KFAC_EINVAL;  // unreachable: vectors / rows fall back
  TriArgs t{};
  t.F = j.F; t.ldF = j.ldF; t.n = j.n; t.G = pl.G; t.R = pl.R;
  t.abort = reinterpret_cast<unsigned*>(ws);
  char* q = ws + 256;
  t.pub = reinterpret_cast<gran_t*>(q); q += align_up((size_t)2 * 4 * j.n * sizeof(gran_t), 256);
  t.d = reinterpret_cast<double*>(q); q += align_up((size_t)j.n * sizeof(double), 256);
  t.e = reinterpret_cast<double*>(q); q += align_up((size_t)j.n * sizeof(double), 256);
  t.rows_g = pl.lds_rows ? nullptr : reinterpret_cast<double*>(q);
  if (!pl.lds_rows) q += align_up((size_t)pl.G * pl.R * j.n * sizeof(double), 256);
  t.vecs_g = pl.vec_lds ? nullptr : reinterpret_cast<double*>(q);
  if (!pl.vec_lds) q += align_up((size_t)pl.G * 3 * j.n * sizeof(double), 256);
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
  // abort word and every granule start at zero (tag 0 never matches an epoch)
  if (hipMemsetAsync(ws, 0, tri_zero_bytes(j.n), stream) != hipSuccess) return KFAC_ELAUNCH;
  const bool rb8 = pl.RB == 8;
  const void* fn = !pl.vec_lds ? reinterpret_cast<const void*>(&eig_tridiag<false, 4, false>)
                  : pl.lds_rows ? (rb8 ? reinterpret_cast<const void*>(&eig_tridiag<true, 8>)
                                       : reinterpret_cast<const void*>(&eig_tridiag<true, 4>))
                                : (rb8 ? reinterpret_cast<const void*>(&eig_tridiag<false, 8>)
                                       : reinterpret_cast<const void*>(&eig_tridiag<false, 4>));
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.shmem) != hipSuccess)
    return KFAC_ELAUNCH;
  void* kargs[] = {&t};
  // cooperative: the runtime rejects a grid that cannot be co-resident (no deadlock)
  if (hipLaunchCooperativeKernel(fn, dim3(pl.G), dim3(NTHREADS), kargs, (unsigned)pl.shmem, stream) !=
      hipSuccess)
    return KFAC_ELAUNCH;
  // one wave per eigenvalue; d and e^2 in LDS while 2 n doubles fit (n <= 9600), else
  // read from global memory
  const size_t bsh2 = (size_t)2 * j.n * sizeof(double);
  const bool bsh_lds = bsh2 <= TRI_LDS_BUDGET;
  const size_t bsh = bsh_lds ? bsh2 : 0;
  const void* bfn = bsh_lds ? reinterpret_cast<const void*>(&eig_bisect<true>)
                            : reinterpret_cast<const void*>(&eig_bisect<false>);
  if (hipFuncSetAttribute(bfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bsh) != hipSuccess)
    return KFAC_ELAUNCH;
  if (bsh_lds)
    hipLaunchKernelGGL(eig_bisect<true>, dim3((j.n + NTHREADS / 64 - 1) / (NTHREADS / 64)), dim3(NTHREADS),
                       bsh, stream, t.d, t.e, j.n, j.evals, t.abort, info);
  else
    hipLaunchKernelGGL(eig_bisect<false>, dim3((j.n + NTHREADS / 64 - 1) / (NTHREADS / 64)), dim3(NTHREADS),
                       0, stream, t.d, t.e, j.n, j.evals, t.abort, info);
  KFAC_CHECK_LAUNCH();
  if (vecs) {
    hipLaunchKernelGGL(eig_tri_vectors, dim3((j.n + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0,
                       stream, t.d, t.e, j.evals, j.n, Z, scratch);
    KFAC_CHECK_LAUNCH();
    const size_t col = (size_t)j.n * sizeof(double);
    const int V = 4 * col <= TRI_LDS_BUDGET ? 4 : 2 * col <= TRI_LDS_BUDGET ? 2 : col <= TRI_LDS_BUDGET ? 1 : 0;
    const size_t sh = (size_t)V * col;
    const void* bt = V == 4 ? reinterpret_cast<const void*>(&eig_backtransform<4, true>)
                     : V == 2 ? reinterpret_cast<const void*>(&eig_backtransform<2, true>)
                     : V == 1 ? reinterpret_cast<const void*>(&eig_backtransform<1, true>)
                              : reinterpret_cast<const void*>(&eig_backtransform<1, false>);
    if (hipFuncSetAttribute(bt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh) != hipSuccess)
      return KFAC_ELAUNCH;
    const dim3 bg((j.n + std::max(V, 1) - 1) / std::max(V, 1));
    if (V == 4)
      hipLaunchKernelGGL((eig_backtransform<4, true>), bg, dim3(NTHREADS), sh, stream, t.U, t.tau, Z, j.n,
                         j.evecs, j.ldv);
    else if (V == 2)
      hipLaunchKernelGGL((eig_backtransform<2, true>), bg, dim3(NTHREADS), sh, stream, t.U, t.tau, Z, j.n,
                         j.evecs, j.ldv);
    else if (V == 1)
      hipLaunchKernelGGL((eig_backtransform<1, true>), bg, dim3(NTHREADS), sh, stream, t.U, t.tau, Z, j.n,
                         j.evecs, j.ldv);
    else
      hipLaunchKernelGGL((eig_backtransform<1, false>), bg, dim3(NTHREADS), 0, stream, t.U, t.tau, Z, j.n,
                         j.evecs, j.ldv);
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
  // profile slot with the tridiagonalisations' algorithmic bytes: each reflector reads
  // and rewrites the trailing rows once, sum_k (n - k)^2 x 16 B ~ 16 n^3 / 3
  double bytes = 0.0;
  if (prof_on())
    for (int i = 0; i < njobs; ++i)
      if (jobs[i].n > EIG_LDS_MAX) bytes += 16.0 * (double)jobs[i].n * jobs[i].n * jobs[i].n / 3.0;
  ProfScope ps(KFAC_PROF_SYEV, st, 0.0, bytes);
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
