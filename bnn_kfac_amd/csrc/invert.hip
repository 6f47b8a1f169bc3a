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

#include <algorithm>

#include "kfac_common.h"

namespace kfac {

constexpr int NB = 64;      // fp64 tile edge
constexpr int DP = NB + 2;  // LDS pitch (doubles): conflict-free MFMA operand reads
constexpr int IMAXJ = 8;
constexpr int MERGE_T = 24;  // <= this many 64-tiles per edge: merged (one-launch) steps

typedef double doublex4 __attribute__((ext_vector_type(4)));

struct InvJobDev {
  const float* F;
  unsigned* cnt;  // inv_flow dependency counters (verR[T*T], verZ[T*T], diag[T]) or null
  int64_t ldF;
  float* out;
  int64_t ldo;
  double* W;   // Np x Np: R', then C below the diagonal (lower tiles)
  double* X;   // Np x Np: Z accumulators, then C^{-1} (lower tiles)
  double* Tm;  // Np x Np: scratch (X^T X)
  int* info;
  double scale, shift;
  int n, T, Np, kind;
  int xw;      // final strictly-lower X tiles in W (merged step) instead of X
  int fout;    // merged step, inverse-Cholesky output: the steps write L (no inv_out)
};

struct InvArgs {
  unsigned* flow;  // inv_flow queue header {head, abort} (zeroed by the build step) or null
  int njobs;
  int step;
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

// Global access to the W / X workspace tiles.  C = true (inv_flow: tiles handed
// between workgroups of ONE launch) uses the write-through form of the MI355X
// hand-off recipe: every store `sc1` (global_store ... sc1, the line leaves the
// XCD's L2), every load `sc1` (bypasses this CU's L1), so no release/acquire
// fence is needed around the dependency counters.  C = false: plain accesses
// (tiles cross kernel boundaries only).
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) unsigned gunsigned;
template <bool C>
__device__ __forceinline__ double gld(const double* p) {
  if constexpr (C)
    return __hip_atomic_load((gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    return *p;
}
template <bool C>
__device__ __forceinline__ void gst(double* p, double v) {
  if constexpr (C)
    __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

// All 16 loads of a thread are issued before the first LDS write (a rolled loop
// would serialise 16 global-memory round trips).
template <bool C = false>
__device__ __forceinline__ void load_tile(double* lds, const double* g, int Np) {
  constexpr int PER = NB * NB / NTHREADS;
  const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  double v[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) v[q] = gld<C>(g + (int64_t)(r0 + 4 * q) * Np + c);
#pragma unroll
  for (int q = 0; q < PER; ++q) lds[(r0 + 4 * q) * DP + c] = v[q];
}

// Up to three tiles with every load in flight together (one memory round trip
// instead of one per tile); null destinations are skipped.
template <bool C = false>
__device__ __forceinline__ void load_tiles(double* l0, const double* g0, double* l1, const double* g1,
                                           double* l2, const double* g2, int Np) {
  constexpr int PER = NB * NB / NTHREADS;
  const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  double v0[PER], v1[PER], v2[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int64_t off = (int64_t)(r0 + 4 * q) * Np + c;
    v0[q] = gld<C>(g0 + off);
    if (l1) v1[q] = gld<C>(g1 + off);
    if (l2) v2[q] = gld<C>(g2 + off);
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int o = (r0 + 4 * q) * DP + c;
    l0[o] = v0[q];
    if (l1) l1[o] = v1[q];
    if (l2) l2[o] = v2[q];
  }
}

template <bool C = false>
__device__ __forceinline__ void store_tile(double* g, const double* lds, int Np) {
  for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
    const int r = e >> 6, c = e & 63;
    gst<C>(g + (int64_t)r * Np + c, lds[r * DP + c]);
  }
}

// ---------------------------------------------------------------- MFMA f64 blocks
// One wave accumulates a 16x16 block: acc += A(16xK) * op(B), A rows at `a` (pitch
// lda), B either (K x 16) at `b` (trans=false) or (16 x K) at `b` read as B^T.
// v_mfma_f64_16x16x4_f64: lane l holds A[l&15][k0 + (l>>4)], B[k0 + (l>>4)][l&15];
// result register v of lane l is C[(l>>4) + 4v][l&15].
template <bool TRANS_B>
__device__ __forceinline__ void mfma_block(const double* a, int lda, const double* b, int ldb, int K,
                                           doublex4& acc) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, kk = lane >> 4;
  for (int k0 = 0; k0 < K; k0 += 4) {
    const double av = a[i * lda + k0 + kk];
    const double bv = TRANS_B ? b[i * ldb + k0 + kk] : b[(k0 + kk) * ldb + i];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
}

__device__ __forceinline__ int acc_row64(int v) { return ((threadIdx.x & 63) >> 4) + 4 * v; }

// Full 64x64 tile product into registers: wave w owns block row w, acc[jb] = block (w, jb).
template <bool TRANS_B>
__device__ __forceinline__ void gemm64(const double* A, const double* B, doublex4 (&acc)[4]) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    acc[jb] = doublex4{0.0, 0.0, 0.0, 0.0};
    if (TRANS_B)
      mfma_block<true>(A + 16 * w * DP, DP, B + 16 * jb * DP, DP, NB, acc[jb]);
    else
      mfma_block<false>(A + 16 * w * DP, DP, B + 16 * jb, DP, NB, acc[jb]);
  }
}

// global[tile](r, c) = alpha * acc (+ global if accumulate)   (acc from gemm64)
template <bool C = false>
__device__ __forceinline__ void store_acc_global(double* g, int Np, const doublex4 (&acc)[4],
                                                 double alpha, bool accumulate) {
  const int w = threadIdx.x >> 6, col = threadIdx.x & 15;
  auto at = [&](int jb, int v) { return g + (int64_t)(16 * w + acc_row64(v)) * Np + 16 * jb + col; };
  // every old value loaded before the first store: atomic (C) accesses keep program
  // order, so an interleaved load/store per element would serialise 16 round trips
  double old[4][4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int v = 0; v < 4; ++v) old[jb][v] = accumulate ? gld<C>(at(jb, v)) : 0.0;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int v = 0; v < 4; ++v) gst<C>(at(jb, v), old[jb][v] + alpha * acc[jb][v]);
}

// 1/d: v_rcp_f64 + two Newton steps (~1 ulp) instead of the IEEE division sequence,
// which sits on the elimination's serial chain.
__device__ __forceinline__ double fast_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}

// --------------------------------------------------------- diagonal factorisation
// S (64x64 lower, LDS) -> Y = chol(S)^{-1} (lower, LDS); S is destroyed.
// Blocked by 16: wave 0 eliminates each 16x16 diagonal block [D | I] -> I_k =
// D^{-1/2} L_unit^{-1}; the panel (C = S I_k^T, X_k = I_k Z_k) and the trailing /
// Z updates are 16x16 MFMA blocks spread over the 4 waves.  dg (>= NB+352 doubles)
// receives the pivots; its tail is scratch.
template <int PARTS = 7>  // ablation: bit0 elimination, bit1 panel, bit2 trailing
__device__ __forceinline__ void diag_factor(double* S, double* Y, double* dg) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < NB * NB; e += NTHREADS) Y[(e >> 6) * DP + (e & 63)] = 0.0;
  __syncthreads();
  for (int kb = 0; kb < 4; ++kb) {
    const int o = 16 * kb;
    // (1) one wave: unit-lower elimination of the 16x16 diagonal block [D | I] -> I_k.
    // Lane (r, g) keeps D[r][4g..4g+3] and Y[r][4g..4g+3] in registers; per column
    // the owners publish column j of D and row j of Y to LDS (`bc`, `by`), and every
    // lane reads what it needs in one batch (LDS ops of one wave complete in order,
    // so no barrier), then updates with selects (no divergent branches).
    if ((PARTS & 1) && wave == 0) {
      double* Sb = S + o * DP + o;
      double* Yb = Y + o * DP + o;
      double* bc = dg + NB;       // column j of D: 16 slots + 64 dummy slots
      double* by = dg + NB + 80;  // row j of Y: 16 slots + 4*64 dummy slots
      const int r = lane & 15, g = lane >> 4;
      double sv[4], yv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sv[q] = Sb[r * DP + 4 * g + q];
        yv[q] = (r == 4 * g + q) ? 1.0 : 0.0;
      }
      double piv = 1.0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        // every lane writes (non-owners into private dummy slots): no divergent branches
        bc[(g == (j >> 2)) ? r : 16 + lane] = sv[j & 3];
        double* yw = by + ((r == j) ? 4 * g : 16 + 4 * lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) yw[q] = yv[q];
        const double d = bc[j];
        const double srj = bc[r];
        double sc[4], yj[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sc[q] = bc[4 * g + q];
          yj[q] = by[4 * g + q];
        }
        piv = (r == j) ? d : piv;
        const double l = srj / d;
        const bool below = r > j;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = 4 * g + q;
          const double ns = sv[q] - l * sc[q];
          const double ny = yv[q] - l * yj[q];
          sv[q] = (below && c > j) ? ns : sv[q];
          yv[q] = (below && c <= j) ? ny : yv[q];
        }
      }
      if (g == 0) dg[o + r] = piv;
      const double rs = 1.0 / sqrt(piv);
#pragma unroll
      for (int q = 0; q < 4; ++q) Yb[r * DP + 4 * g + q] = (4 * g + q <= r) ? yv[q] * rs : 0.0;
    }
    __syncthreads();
    // (2) panel: blocks ib > kb: C = S[ib][kb] I^T ;  blocks jb < kb: X = I Z[kb][jb]
    const int nC = 3 - kb, nX = kb;
    doublex4 acc = {0.0, 0.0, 0.0, 0.0};
    int mine = -1;
    if ((PARTS & 2) && wave < nC + nX) {  // nC + nX = 3: at most one block per wave
      mine = wave;
      if (wave < nC) {
        const int ib = kb + 1 + wave;
        mfma_block<true>(S + 16 * ib * DP + o, DP, Y + o * DP + o, DP, 16, acc);
      } else {
        const int jb = wave - nC;
        mfma_block<false>(Y + o * DP + o, DP, Y + o * DP + 16 * jb, DP, 16, acc);
      }
    }
    __syncthreads();
    if (mine >= 0) {
      const int col = lane & 15;
      double* dst = (mine < nC) ? S + 16 * (kb + 1 + mine) * DP + o : Y + o * DP + 16 * (mine - nC);
#pragma unroll
      for (int v = 0; v < 4; ++v) dst[acc_row64(v) * DP + col] = acc[v];
    }
    __syncthreads();
    if (kb == 3) break;
    // (3) trailing: S[ib][jb] -= C[ib] C[jb]^T (kb < jb <= ib); Z[ib][jb] -= C[ib] X[kb][jb] (jb <= kb)
    const int nT = (3 - kb) * (4 - kb) / 2, nZ = (3 - kb) * (kb + 1);
    for (int t = wave; (PARTS & 4) && t < nT + nZ; t += 4) {
      doublex4 a2 = {0.0, 0.0, 0.0, 0.0};
      double* dst;
      if (t < nT) {
        int i = 0;
        while ((i + 1) * (i + 2) / 2 <= t) ++i;
        const int ib = kb + 1 + i, jb = kb + 1 + (t - i * (i + 1) / 2);
        mfma_block<true>(S + 16 * ib * DP + o, DP, S + 16 * jb * DP + o, DP, 16, a2);
        dst = S + 16 * ib * DP + 16 * jb;
      } else {
        const int u = t - nT;
        const int ib = kb + 1 + u / (kb + 1), jb = u % (kb + 1);
        mfma_block<false>(S + 16 * ib * DP + o, DP, Y + o * DP + 16 * jb, DP, 16, a2);
        dst = Y + 16 * ib * DP + 16 * jb;
      }
      const int col = lane & 15;
#pragma unroll
      for (int v = 0; v < 4; ++v) dst[acc_row64(v) * DP + col] -= a2[v];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------- build R'
// R'[i][c] = scale*(F[fi][fc] + F[fc][fi])/2 + shift*[i==c], fi = n-1-i, fc = n-1-c.
// Both source blocks are read row-coalesced into LDS (fp32, P and Q: 64 x 65 floats
// each), then combined; tile (ti, tj) goes to W (and a copy to LDS `copy` when
// non-null: the step -1 workgroup factors tile (0,0) straight from it).
__device__ __forceinline__ void build_tile(const InvJobDev& J, int ti, int tj, float* P, float* Q,
                                           double* copy) {
  const int n = J.n, i0 = ti * NB, c0 = tj * NB;
  constexpr int PER = NB * NB / NTHREADS;
  const int cc = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  float pv[PER], qv[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int a = r0 + 4 * q;
    // row fi = n-1-(i0+a), column fc = n-1-(c0+cc): consecutive lanes -> consecutive fc (descending)
    const int i = i0 + a, c = c0 + cc;
    pv[q] = (i < n && c < n) ? J.F[(int64_t)(n - 1 - i) * J.ldF + (n - 1 - c)] : 0.f;
    const int ib = i0 + cc, cb = c0 + a;  // Q[a][cc] = F[n-1-(c0+a)][n-1-(i0+cc)]
    qv[q] = (ib < n && cb < n) ? J.F[(int64_t)(n - 1 - cb) * J.ldF + (n - 1 - ib)] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    P[(r0 + 4 * q) * (NB + 1) + cc] = pv[q];
    Q[(r0 + 4 * q) * (NB + 1) + cc] = qv[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int a = r0 + 4 * q, i = i0 + a, c = c0 + cc;
    double v;
    if (i < n && c < n) {
      const double sym = 0.5 * ((double)P[a * (NB + 1) + cc] + (double)Q[cc * (NB + 1) + a]);
      v = J.scale * sym + (i == c ? J.shift : 0.0);
    } else {
      v = (i == c) ? 1.0 : 0.0;  // identity padding keeps the padded block trivial
    }
    J.W[(int64_t)i * J.Np + c] = v;
    if (copy) copy[a * DP + cc] = v;
    if (ti != tj) J.X[(int64_t)i * J.Np + c] = 0.0;  // Z accumulators start at 0
  }
}

// Output block of the final inverse tile X(a, b), a >= b, from LDS (pitch DP):
// L[n-1-q][n-1-r] = X[r][q] (r in tile a, q in tile b).  Output rows are walked
// with consecutive lanes on consecutive output columns (descending r): coalesced
// stores.  zero = true writes the (all-zero) block of the upper tile X(b, a) instead.
__device__ __forceinline__ void emit_out(const InvJobDev& J, int a, int b, const double* lds,
                                         bool zero = false) {
  const int n = J.n;
  for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
    const int cl = e >> 6, rl = NB - 1 - (e & 63);
    const int r = a * NB + rl, q = b * NB + cl;
    if (r >= n || q >= n) continue;
    J.out[(int64_t)(n - 1 - q) * J.ldo + (n - 1 - r)] = zero ? 0.f : (float)lds[rl * DP + cl];
  }
}

// Upper zero block of L for the strictly-lower tile (ti, tj): X(tj, ti) = 0, i.e.
// L[n-1-q][n-1-r] = 0 for r in tile tj, q in tile ti.
__device__ __forceinline__ void emit_zero_block(const InvJobDev& J, int ti, int tj) {
  const int n = J.n;
  for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
    const int ql = e >> 6, rl = NB - 1 - (e & 63);
    const int r = tj * NB + rl, q = ti * NB + ql;
    if (r >= n || q >= n) continue;
    J.out[(int64_t)(n - 1 - q) * J.ldo + (n - 1 - r)] = 0.f;
  }
}

__global__ __launch_bounds__(NTHREADS) void inv_build(InvArgs args) {
  __shared__ float P[NB * (NB + 1)];  // P[a][b] = F[fi(a)][fc(b)]
  __shared__ float Q[NB * (NB + 1)];  // Q[b][a] = F[fc(b)][fi(a)]
  const int j = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[j];
  const int local = blockIdx.x - args.begin[j];
  if (local == 0 && threadIdx.x == 0 && J.info) *J.info = 0;
  int ti, tj;
  tri_decode(local, ti, tj);
  build_tile(J, ti, tj, P, Q, nullptr);
}

// Pivot check of the factored diagonal tile d: info = first global column whose
// pivot is not positive (+1), one ballot of wave 0 (no serial scan).
__device__ __forceinline__ void check_pivots(const InvJobDev& J, int d, const double* dg) {
  if (!J.info || threadIdx.x >= 64) return;
  const int c = threadIdx.x, g = d * NB + c;
  const unsigned long long bad = __ballot(g < J.n && !(dg[c] > 0.0));
  if (bad && c == 0) atomicCAS(J.info, 0, d * NB + __ffsll(bad));
}

// acc (gemm64 layout) -> LDS tile
__device__ __forceinline__ void store_acc_lds(double* S, const doublex4 (&acc)[4]) {
  const int w = threadIdx.x >> 6, col = threadIdx.x & 15;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int v = 0; v < 4; ++v) S[(16 * w + acc_row64(v)) * DP + 16 * jb + col] = acc[jb][v];
}

// C_i = R'[i][k] X[k][k]^T into Sdst (Xkk already in LDS; Sdst holds R'[i][k] on entry)
__device__ __forceinline__ void panel_tile_lds(double* Sdst, const double* Xkk) {
  doublex4 acc[4];
  gemm64<true>(Sdst, Xkk, acc);
  __syncthreads();  // every wave done reading R'[i][k] before it is overwritten
  store_acc_lds(Sdst, acc);
  __syncthreads();
}

// ------------------------------------------------------------------- step k
// One launch per elimination step (the panel is folded in: every workgroup forms
// the panel blocks it needs, C[i][k] = R'[i][k] X[k][k]^T, itself; C is never
// stored — column k is dead after step k).
//   k = -1        : factor tile (0,0)                      -> X[0][0]
//   k <= T-2      : trailing  R'[i][j] -= C_i C_j^T        (i >= j > k)
//                   the (k+1,k+1) workgroup then factors   -> X[k+1][k+1]
//                   Z[i][j] -= C_i B,  B = X[k][k] (j = k) or X[k][k] Z[k][j] (j < k)
//                   row k+1's Z workgroups also store X[k][j] = X[k][k] Z[k][j]
//                   (final) into W[k][j], dead since step j (Z[k][j] stays intact
//                   for the other readers of this launch)
//   k = T-1       : X[k][j] = X[k][k] Z[k][j] -> W[k][j]   (j < k)
// Final inverse X: diagonal tiles in X, strictly-lower tiles in W (x_tile()).
// trailing tile (i, j), i >= j > k: R'[i][j] -= C_i C_j^T.  Returns true for the
// (k+1, k+1) workgroup, which then holds the updated diagonal tile in S0.
template <bool C = false>
__device__ __forceinline__ bool step_trailing_ij(const InvJobDev& J, int k, int i, int j, double* S0,
                                                 double* S1, double* S2) {
  const bool diag = i == k + 1 && j == k + 1;
  // the (k+1,k+1) workgroup also prefetches its diagonal tile into the idle S2
  load_tiles<C>(S0, tile_ptr(J.X, J.Np, k, k), S1, tile_ptr(J.W, J.Np, i, k),
                (j != i || diag) ? S2 : nullptr, tile_ptr(J.W, J.Np, j != i ? j : i, j != i ? k : i), J.Np);
  __syncthreads();
  panel_tile_lds(S1, S0);              // C_i
  if (j != i) panel_tile_lds(S2, S0);  // C_j
  doublex4 acc[4];
  gemm64<true>(S1, j != i ? S2 : S1, acc);
  if (!diag) {
    store_acc_global<C>(tile_ptr(J.W, J.Np, i, j), J.Np, acc, -1.0, true);
    return false;
  }
  // the updated diagonal tile is consumed right here (never written back)
  const int w = threadIdx.x >> 6, col = threadIdx.x & 15;
#pragma unroll
  for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
    for (int v = 0; v < 4; ++v) S2[(16 * w + acc_row64(v)) * DP + 16 * b4 + col] -= acc[b4][v];
  __syncthreads();
  return true;
}

template <bool C = false>
__device__ __forceinline__ bool step_trailing(const InvJobDev& J, int k, int local, double* S0,
                                              double* S1, double* S2) {
  int a, b;
  tri_decode(local, a, b);
  return step_trailing_ij<C>(J, k, k + 1 + a, k + 1 + b, S0, S1, S2);
}

// Z tile (i, j), i > k >= j: Z[i][j] -= C_i B, B = X[k][k] (j = k) or
// X[k][k] Z[k][j] (j < k; row k+1's workgroup also stores it as the final X[k][j]).
template <bool C = false>
__device__ __forceinline__ void step_z_ij(const InvJobDev& J, int k, int i, int j, double* S0,
                                          double* S1, double* S2) {
  load_tiles<C>(S0, tile_ptr(J.X, J.Np, k, k), S1, tile_ptr(J.W, J.Np, i, k), j < k ? S2 : nullptr,
             tile_ptr(J.X, J.Np, k, j), J.Np);
  __syncthreads();
  panel_tile_lds(S1, S0);  // C_i
  doublex4 acc[4];
  const double* Bm = S0;
  if (j < k) {
    gemm64<false>(S0, S2, acc);
    __syncthreads();
    store_acc_lds(S2, acc);
    if (i == k + 1 && J.xw) store_acc_global<C>(tile_ptr(J.W, J.Np, k, j), J.Np, acc, 1.0, false);
    __syncthreads();
    Bm = S2;
  }
  gemm64<false>(S1, Bm, acc);
  store_acc_global<C>(tile_ptr(J.X, J.Np, i, j), J.Np, acc, -1.0, true);
  if (j < k && i == k + 1 && J.fout) emit_out(J, k, j, S2);  // final X[k][j]
}

template <bool C = false>
__device__ __forceinline__ void step_z(const InvJobDev& J, int k, int u, double* S0, double* S1,
                                       double* S2) {
  step_z_ij<C>(J, k, k + 1 + u / (k + 1), u % (k + 1), S0, S1, S2);
}

// last row of X (k = T-1): X[k][j] = X[k][k] Z[k][j] -> W[k][j]
template <bool C = false>
__device__ __forceinline__ void step_last_row(const InvJobDev& J, int k, int j, double* S0,
                                              double* S1) {
  load_tiles<C>(S0, tile_ptr(J.X, J.Np, k, k), S1, tile_ptr(J.X, J.Np, k, j), nullptr, nullptr, J.Np);
  __syncthreads();
  doublex4 acc[4];
  gemm64<false>(S0, S1, acc);
  if (J.xw) store_acc_global<C>(tile_ptr(J.W, J.Np, k, j), J.Np, acc, 1.0, false);
  if (J.fout) {
    __syncthreads();  // S1 fully read by the GEMM
    store_acc_lds(S1, acc);
    __syncthreads();
    emit_out(J, k, j, S1);
  }
}

__global__ __launch_bounds__(NTHREADS) void inv_step(InvArgs args) {
  __shared__ __attribute__((aligned(16))) double S0[NB * DP];
  __shared__ __attribute__((aligned(16))) double S1[NB * DP];
  __shared__ __attribute__((aligned(16))) double S2[NB * DP];
  __shared__ double dg[NB + 352];  // pivots + elimination broadcast buffers
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int k = args.step, T = J.T;
  const int local = blockIdx.x - args.begin[jb];
  const int nTrail = (T - k - 1) * (T - k) / 2;
  if (k < 0) {  // build R' (one tile per workgroup); workgroup 0 also factors tile (0,0)
    int ti, tj;
    tri_decode(local, ti, tj);
    if (local == 0 && threadIdx.x == 0 && J.info) *J.info = 0;
    if (J.cnt) {  // inv_flow follows: its counters start at 0 (diag[0] set below)
      if (threadIdx.x == 0) J.cnt[ti * T + tj] = J.cnt[T * T + ti * T + tj] = 0u;
      if (local == 0 && threadIdx.x < T) J.cnt[2 * T * T + threadIdx.x] = 0u;
      if (jb == 0 && local == 0 && threadIdx.x < 2 && args.flow) args.flow[threadIdx.x] = 0u;
    }
    build_tile(J, ti, tj, reinterpret_cast<float*>(S0), reinterpret_cast<float*>(S1),
               local == 0 ? S2 : nullptr);
    if (J.fout && ti != tj) emit_zero_block(J, ti, tj);
    if (local != 0) return;
    __syncthreads();
  } else if (k == T - 1) {
    step_last_row(J, k, local, S0, S1);
    return;
  } else if (local >= nTrail) {
    step_z(J, k, local - nTrail, S0, S1, S2);
    return;
  } else if (!step_trailing(J, k, local, S0, S1, S2)) {
    return;
  }
  // the one diagonal factorisation of this step (single call site: stays inlined)
  const int d = k + 1;
  diag_factor(S2, S1, dg);
  check_pivots(J, d, dg);
  store_tile(tile_ptr(J.X, J.Np, d, d), S1, J.Np);
  if (J.fout) emit_out(J, d, d, S1);
  if (J.cnt && d == 0 && threadIdx.x == 0) J.cnt[2 * T * T] = 1u;  // X[0][0] ready for inv_flow
}

// ------------------------------------------- dataflow steps (one persistent launch)
// inv_flow runs every step k >= 0 of the merged elimination (after the build launch,
// inv_step(-1)) as ONE launch of a few workgroups that dequeue tasks in step order
// from a counter and start each as soon as the tiles it reads are final, instead
// of one launch per step: no kernel boundary per step, and a handful of resident
// workgroups (not ~100 per step) — the inversion keeps its CUs while the next data
// pass's SYRK launches fill the rest of the chip.
// Per job, counters written only by the task that finalises the tile (one writer each):
//   verR[i*T+j] = k + 1 once R'[i][j] holds the trailing updates of steps 0..k
//   verZ[i*T+j] = k - j + 1 once Z[i][j] holds the updates of steps j..k
//   diag[k]     = 1 once X[k][k] is stored
// Task (k, ...) needs X[k][k] and its operand tiles updated through step k-1:
//   trailing (i, j): verR[i][k], verR[j][k], verR[i][j] >= k
//   Z (i, j):        verR[i][k] >= k, verZ[k][j] >= k - j (j < k), verZ[i][j] >= k - j
//   last row (j):    verZ[T-1][j] >= T - 1 - j
// Dequeue order (topological, so every awaited task is held by a running
// workgroup: any number of resident workgroups completes, no co-residency assumed):
// the diagonal chain runs one step ahead of the bulk.  With D_k = trailing (k+1, k+1)
// of step k (it factors X[k+1][k+1]) and F_k = trailing (k+2, k+1), (k+2, k+2) of
// step k (the tiles D_{k+1} reads), segment s holds, per job,
//   D_s,  the rest of step s-1,  F_s            (segment 0: D_0, F_0)
// (segment T: the last row), so D_{s+1} is queued right behind the step-s tasks it
// needs instead of behind all of step s, and the bulk of a step runs while the
// next diagonal tile is factored.
// (vmcnt(0) in every wave), meets the workgroup barrier, then one lane stores the
// counter.  Waits are bounded (1 s): a timeout sets the abort word and info = -1.
constexpr int FLOW_SEGS = MERGE_T + 1;

// tasks of step k (T tiles per edge); its critical ones (D_k and, if present, F_k);
// the rest of it (the last row, k = T-1, has no critical task)
__host__ __device__ inline int flow_step_tasks(int T, int k) {
  return k + 1 < T ? (T - k - 1) * (T - k) / 2 + (T - k - 1) * (k + 1) : (k + 1 == T ? k : 0);
}
__host__ __device__ inline int flow_crit(int T, int k) {
  return k + 1 < T ? ((T - k - 1) * (T - k) / 2 >= 3 ? 3 : 1) : 0;
}
__host__ __device__ inline int flow_rest(int T, int k) { return flow_step_tasks(T, k) - flow_crit(T, k); }

struct FlowArgs {
  InvArgs a;
  int total;  // tasks
  int nsegs;  // Tmax + 1
  int sbegin[FLOW_SEGS][IMAXJ + 1];  // first task of (segment s, job j); [s][njobs] = end of segment s
};

__device__ __forceinline__ unsigned cnt_ld(const unsigned* p) {
  return __hip_atomic_load((gunsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void cnt_st(unsigned* p, unsigned v) {
  __hip_atomic_store((gunsigned*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave (all lanes, one address): spin until *p >= need (false: aborted / timed
// out).  Every value is read back through readfirstlane, so the loop is uniform.
__device__ __forceinline__ unsigned cnt_ld_u(const unsigned* p) {
  return __builtin_amdgcn_readfirstlane(cnt_ld(p));
}
__device__ bool flow_wait(const unsigned* p, unsigned need, unsigned* abort_word) {
  if (cnt_ld_u(p) >= need) return true;
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + 100000000ull;  // 1 s at 100 MHz
  for (;;) {
    __builtin_amdgcn_s_sleep(1);
    if (cnt_ld_u(p) >= need) return true;
    if (cnt_ld_u(abort_word)) return false;
    if (__builtin_amdgcn_s_memrealtime() > deadline) {
      cnt_st(abort_word, 1u);
      return false;
    }
  }
}

__global__ __launch_bounds__(NTHREADS) void inv_flow(FlowArgs fa) {
  __shared__ __attribute__((aligned(16))) double S0[NB * DP];
  __shared__ __attribute__((aligned(16))) double S1[NB * DP];
  __shared__ __attribute__((aligned(16))) double S2[NB * DP];
  __shared__ double dg[NB + 352];
  __shared__ int s_task, s_ok;
  const InvArgs& args = fa.a;
  unsigned* head = args.flow;
  unsigned* abort_word = args.flow + 1;
  // All control below is wave-uniform (scalar conditions): wave 0 dequeues, waits
  // and publishes with all its lanes, so no divergent branch encloses a loop exit
  // or a barrier (a `threadIdx.x == 0` region at the loop head made the compiler
  // split wave 0's lanes over two loop nests and run its barriers twice: a hang).
  const bool lead = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  for (;;) {
    if (lead) {
      // lane 0 adds 1, the others 0: lane 0's old value is this workgroup's task
      const unsigned old = __hip_atomic_fetch_add((gunsigned*)head, (threadIdx.x == 0) ? 1u : 0u,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_task = (int)__builtin_amdgcn_readfirstlane(old);
    }
    __syncthreads();
    // uniform (scalar) loop control: with a VGPR task index the compiler treats the
    // loop exits as divergent and may run one wave's barriers on different trips for
    // different lanes (a barrier-count mismatch: the workgroup hangs)
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    if (t >= fa.total) break;
    int sg = 0;
    while (t >= fa.sbegin[sg][args.njobs]) ++sg;
    int jb = 0;
    while (jb + 1 < args.njobs && t >= fa.sbegin[sg][jb + 1]) ++jb;
    const InvJobDev& J = args.job[jb];
    const int T = J.T;
    int u = t - fa.sbegin[sg][jb];
    const unsigned* verR = J.cnt;
    const unsigned* verZ = J.cnt + T * T;
    unsigned* cnt = J.cnt;
    // (step k, step-local index lo) of the task, see the segment layout above
    int k, lo;
    const bool hasA = sg <= T - 2;
    if (hasA && u == 0) {
      k = sg;
      lo = 0;
    } else {
      u -= hasA ? 1 : 0;
      const int nB = sg >= 1 ? flow_rest(T, sg - 1) : 0;
      if (u < nB) {
        k = sg - 1;
        lo = u + flow_crit(T, k);
      } else {
        k = sg;
        lo = 1 + (u - nB);
      }
    }
    // task kind: 0 trailing, 1 Z, 2 last row; (i, j) its tile
    const int nTrail = (T - k - 1) * (T - k) / 2;
    int kind, i, j;
    if (k == T - 1) {
      kind = 2;
      i = k;
      j = lo;
    } else if (lo < nTrail) {
      int a, b;
      tri_decode(lo, a, b);
      kind = 0;
      i = k + 1 + a;
      j = k + 1 + b;
    } else {
      const int z = lo - nTrail;
      kind = 1;
      i = k + 1 + z / (k + 1);
      j = z % (k + 1);
    }
    if (lead) {
      bool ok = flow_wait(cnt + 2 * T * T + k, 1u, abort_word);
      if (kind == 0) {
        ok = ok && flow_wait(verR + i * T + k, k, abort_word);
        ok = ok && flow_wait(verR + j * T + k, k, abort_word);
        ok = ok && flow_wait(verR + i * T + j, k, abort_word);
      } else if (kind == 1) {
        ok = ok && flow_wait(verR + i * T + k, k, abort_word);
        if (j < k) ok = ok && flow_wait(verZ + k * T + j, k - j, abort_word);
        ok = ok && flow_wait(verZ + i * T + j, k - j, abort_word);
      } else {
        ok = ok && flow_wait(verZ + i * T + j, T - 1 - j, abort_word);
      }
      if (!ok)
        for (int q = 0; q < args.njobs; ++q)
          if (args.job[q].info) __hip_atomic_store(args.job[q].info, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_ok = ok;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(s_ok)) break;
    bool factored = false;
    if (kind == 0) {
      if (step_trailing<true>(J, k, lo, S0, S1, S2)) {
        const int d = k + 1;
        diag_factor(S2, S1, dg);
        check_pivots(J, d, dg);
        store_tile<true>(tile_ptr(J.X, J.Np, d, d), S1, J.Np);
        emit_out(J, d, d, S1);
        factored = true;
      }
    } else if (kind == 1) {
      step_z<true>(J, k, lo - nTrail, S0, S1, S2);
    } else {
      step_last_row<true>(J, k, j, S0, S1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's tile stores have landed
    __syncthreads();                                    // ... and every other wave's
    if (lead) {  // every lane of wave 0 stores the same word
      if (kind == 0) cnt_st(cnt + i * T + j, (unsigned)(k + 1));
      else if (kind == 1) cnt_st(cnt + T * T + i * T + j, (unsigned)(k - j + 1));
      if (factored) cnt_st(cnt + 2 * T * T + k + 1, 1u);
    }
  }
}

// ------------------------------------------- two-launch step (large factors)
// For many tiles per edge (T > MERGE_T) the panel is formed ONCE per step
// (inv_panel, C in place in W and the final X[k][j] in place in X) and
// inv_update applies it: the merged step's per-workgroup panel recomputation
// would triple the trailing GEMM work there.  Final X stays entirely in X.
// update k
__global__ __launch_bounds__(NTHREADS) void inv_update(InvArgs args) {
  __shared__ __attribute__((aligned(16))) double A[NB * DP];
  __shared__ __attribute__((aligned(16))) double B[NB * DP];
  __shared__ __attribute__((aligned(16))) double Y[NB * DP];
  __shared__ double dg[NB + 352];  // pivots + elimination broadcast buffers
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int k = args.step, T = J.T;
  const int local = blockIdx.x - args.begin[jb];
  const int nTrail = (T - k - 1) * (T - k) / 2;
  if (k < 0 || local < nTrail) {
    int i = k + 1, j = k + 1;
    if (k >= 0) {
      int a, b;
      tri_decode(local, a, b);
      i = k + 1 + a;
      j = k + 1 + b;
    }
    const bool factor = (i == k + 1 && j == k + 1);
    doublex4 acc[4];
    if (k >= 0) {
      // the factoring workgroup (i == j) prefetches its diagonal tile into Y
      load_tiles(A, tile_ptr(J.W, J.Np, i, k), B, tile_ptr(J.W, J.Np, j, k), factor ? Y : nullptr,
                 tile_ptr(J.W, J.Np, i, i), J.Np);
      __syncthreads();
      gemm64<true>(A, B, acc);
    }
    if (!factor) {
      store_acc_global(tile_ptr(J.W, J.Np, i, j), J.Np, acc, -1.0, true);
      return;
    }
    // the updated diagonal tile is consumed right here (never written back)
    __syncthreads();
    double* D = A;  // diagonal tile
    double* Yo = Y;  // its factor's inverse
    if (k >= 0) {
      D = Y;
      Yo = A;
    } else {
      load_tile(A, tile_ptr(J.W, J.Np, i, i), J.Np);
      __syncthreads();
    }
    if (k >= 0) {
      const int w = threadIdx.x >> 6, col = threadIdx.x & 15;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int v = 0; v < 4; ++v) D[(16 * w + acc_row64(v)) * DP + 16 * b4 + col] -= acc[b4][v];
      __syncthreads();
    }
    diag_factor(D, Yo, dg);
    check_pivots(J, i, dg);
    store_tile(tile_ptr(J.X, J.Np, i, i), Yo, J.Np);
    return;
  }
  // Z[i][j] -= C[i][k] X[k][j]   (i > k >= j)
  const int u = local - nTrail;
  const int i = k + 1 + u / (k + 1), j = u % (k + 1);
  load_tiles(A, tile_ptr(J.W, J.Np, i, k), B, tile_ptr(J.X, J.Np, k, j), nullptr, nullptr, J.Np);
  __syncthreads();
  doublex4 acc[4];
  gemm64<false>(A, B, acc);
  store_acc_global(tile_ptr(J.X, J.Np, i, j), J.Np, acc, -1.0, true);
}


// -------------------------------------------------------------------- panel k
__global__ __launch_bounds__(NTHREADS) void inv_panel(InvArgs args) {
  __shared__ __attribute__((aligned(16))) double A[NB * DP];
  __shared__ __attribute__((aligned(16))) double Xk[NB * DP];
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  const int k = args.step, T = J.T;
  const int local = blockIdx.x - args.begin[jb];
  const int nC = T - k - 1;
  doublex4 acc[4];
  if (local < nC) {  // C[i][k] = R'[i][k] X[k][k]^T
    const int i = k + 1 + local;
    double* t = tile_ptr(J.W, J.Np, i, k);
    load_tiles(Xk, tile_ptr(J.X, J.Np, k, k), A, t, nullptr, nullptr, J.Np);
    __syncthreads();
    gemm64<true>(A, Xk, acc);
    store_acc_global(t, J.Np, acc, 1.0, false);
  } else {           // X[k][j] = X[k][k] Z[k][j]
    const int j = local - nC;
    double* t = tile_ptr(J.X, J.Np, k, j);
    load_tiles(Xk, tile_ptr(J.X, J.Np, k, k), A, t, nullptr, nullptr, J.Np);
    __syncthreads();
    gemm64<false>(Xk, A, acc);
    store_acc_global(t, J.Np, acc, 1.0, false);
  }
}


// final inverse X tile (a >= b): with the merged step the strictly-lower tiles live
// in W (see inv_step), with the two-launch step everything is in X
__device__ __forceinline__ const double* x_tile(const InvJobDev& J, int a, int b) {
  return tile_ptr(a > b && J.xw ? J.W : J.X, J.Np, a, b);
}

// Y[a][b] = sum_{m >= a} X[m][a]^T X[m][b]   (lower tiles, a >= b)
__global__ __launch_bounds__(NTHREADS) void inv_xtx(InvArgs args) {
  __shared__ __attribute__((aligned(16))) double A[NB * DP];
  __shared__ __attribute__((aligned(16))) double B[NB * DP];
  const int jb = find_job(args, blockIdx.x);
  const InvJobDev& J = args.job[jb];
  int a, b;
  tri_decode(blockIdx.x - args.begin[jb], a, b);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  doublex4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = doublex4{0.0, 0.0, 0.0, 0.0};
  for (int m = a; m < J.T; ++m) {
    load_tiles(A, x_tile(J, m, a), B, x_tile(J, m, b), nullptr, nullptr, J.Np);  // A read transposed
    __syncthreads();
    const int i = lane & 15, kk = lane >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      for (int k0 = 0; k0 < NB; k0 += 4) {
        const double av = A[(k0 + kk) * DP + 16 * w + i];  // (X^T)[row][k] = X[k][row]
        const double bv = B[(k0 + kk) * DP + 16 * q + i];
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
      }
    __syncthreads();
  }
  store_acc_global(tile_ptr(J.Tm, J.Np, a, b), J.Np, acc, 1.0, false);
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
      const int r = n - 1 - c, q = n - 1 - i;  // L[i][c] = X[r][q], r >= q
      v = (i >= c) ? ((r >> 6) > (q >> 6) && J.xw ? J.W : J.X)[(int64_t)r * J.Np + q] : 0.0;
    } else {
      const int a = n - 1 - i, b = n - 1 - c;
      v = (a >= b) ? J.Tm[(int64_t)a * J.Np + b] : J.Tm[(int64_t)b * J.Np + a];
    }
    J.out[(int64_t)i * J.ldo + c] = (float)v;
  }
}

// ---------------------------------------------------------------- host side
// inv_flow counters of a job (verR, verZ, diag) + the group's queue header
static size_t flow_cnt_bytes(int64_t T) { return align_up((size_t)(2 * T * T + T + 2) * sizeof(unsigned), 256); }

static size_t job_ws(const kfac_invert_job& j) {
  const int64_t T = cdiv(j.n, NB), Np = T * NB;
  return 3 * align_up((size_t)(Np * Np) * sizeof(double), 256) + flow_cnt_bytes(T);
}

// inv_flow (KFAC_INV_FLOW=1) or one launch per step (default: on the MLP the
// per-step launches are as fast at >= 64 flow workgroups and faster below, since a
// merged-step task recomputes its panels: ~12 us per task); workgroups of the
// persistent launch: KFAC_INV_FLOW_WGS (default 64)
static int flow_wgs() {
  const char* e = getenv("KFAC_INV_FLOW");
  if (!e || e[0] != '1') return 0;
  const char* w = getenv("KFAC_INV_FLOW_WGS");
  const int n = w ? atoi(w) : 64;
  return n > 0 ? n : 64;
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

// Phase 0 = the launch that reads F (merged: step -1, which builds R' and factors
// tile (0,0); two-launch path: inv_build); phase 1 = everything after it.
static int invert_group(const kfac_invert_job* jobs, int njobs, char* ws, int32_t* info,
                        hipStream_t s, int phase) {
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
    d.cnt = reinterpret_cast<unsigned*>(ws + 3 * mat);
    ws += 3 * mat + flow_cnt_bytes(d.T);
    Tmax = std::max(Tmax, d.T);
    any_inverse |= jb.out_kind == KFAC_OUT_INVERSE;
  }
  // latency-bound (few tiles per edge): one launch per step; else panel once per step
  const bool merged = Tmax <= MERGE_T;
  bool all_fused = merged;
  for (int i = 0; i < njobs; ++i) {
    args.job[i].xw = merged;
    args.job[i].fout = merged && args.job[i].kind == KFAC_OUT_INV_CHOL;
    all_fused &= args.job[i].fout != 0;
  }
  int rc;
  const bool flow = all_fused && flow_wgs() > 0;
  if (flow) {  // build launch, then every step in one persistent dataflow launch
    // final X[k][j] tiles are never stored (the steps emit L directly): W[k][j] may
    // still be read as R'[k][j] by a step-j task still running
    for (int i = 0; i < njobs; ++i) args.job[i].xw = 0;
    args.flow = args.job[0].cnt + 2 * args.job[0].T * args.job[0].T + args.job[0].T;
    if (!phase) {
      args.step = -1;
      return launch(inv_step, args, [](const InvJobDev& d) { return d.T * (d.T + 1) / 2; }, s);
    }
    FlowArgs fa{};
    fa.a = args;
    fa.nsegs = Tmax + 1;
    int total = 0;
    for (int sg = 0; sg <= Tmax; ++sg) {
      for (int i = 0; i < njobs; ++i) {
        const int T = args.job[i].T;
        fa.sbegin[sg][i] = total;
        if (sg <= T - 2) total += flow_crit(T, sg);   // D_s (+ F_s)
        if (sg >= 1) total += flow_rest(T, sg - 1);   // the rest of step s-1
      }
      fa.sbegin[sg][njobs] = total;
    }
    fa.total = total;
    if (total == 0) return KFAC_OK;
    hipLaunchKernelGGL(inv_flow, dim3(std::min(total, flow_wgs())), dim3(NTHREADS), 0, s, fa);
    KFAC_CHECK_LAUNCH();
    return KFAC_OK;
  }
  for (int i = 0; i < njobs; ++i) args.job[i].cnt = nullptr;
  // info is zeroed by the first launch (workgroup 0 of each job)
  if (merged) {
    for (int k = phase ? 0 : -1; k < (phase ? Tmax : 0); ++k) {
      args.step = k;
      rc = launch(inv_step, args, [k](const InvJobDev& d) {
        if (k < 0) return d.T * (d.T + 1) / 2;  // build every tile; workgroup 0 factors (0,0)
        if (k + 1 < d.T) return (d.T - k - 1) * (d.T - k) / 2 + (d.T - k - 1) * (k + 1);
        return k + 1 == d.T ? k : 0;  // last row of X
      }, s);
      if (rc) return rc;
    }
    if (!phase) return KFAC_OK;
  } else {
    if (!phase) return launch(inv_build, args, [](const InvJobDev& d) { return d.T * (d.T + 1) / 2; }, s);
    args.step = -1;
    rc = launch(inv_update, args, [](const InvJobDev&) { return 1; }, s);
    if (rc) return rc;
    for (int k = 0; k < Tmax; ++k) {
      args.step = k;
      rc = launch(inv_panel, args, [k](const InvJobDev& d) { return k < d.T ? d.T - 1 : 0; }, s);
      if (rc) return rc;
      rc = launch(inv_update, args, [k](const InvJobDev& d) {
        return k + 1 < d.T ? (d.T - k - 1) * (d.T - k) / 2 + (d.T - k - 1) * (k + 1) : 0;
      }, s);
      if (rc) return rc;
    }
  }
  if (any_inverse) {
    rc = launch(inv_xtx, args,
                [](const InvJobDev& d) { return d.kind == KFAC_OUT_INVERSE ? d.T * (d.T + 1) / 2 : 0; }, s);
    if (rc) return rc;
  }
  if (all_fused) return KFAC_OK;  // the steps already wrote every L
  return launch(inv_out, args, [](const InvJobDev& d) { return d.fout ? 0 : d.T * d.T; }, s);
}

}  // namespace kfac

using namespace kfac;

// every job has its own region (the groups' F-reading launches all run first)
extern "C" size_t kfac_invert_workspace_bytes(const kfac_invert_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  size_t tot = 0;
  for (int i = 0; i < njobs; ++i) tot += job_ws(jobs[i]);
  return tot;
}

extern "C" int kfac_invert_ex(const kfac_invert_job* jobs, int njobs, void* workspace,
                              size_t workspace_bytes, int32_t* info, void* inputs_read,
                              kfac_stream_t stream) {
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
  // every group's F-reading launch first, then the event, then the rest
  for (int phase = 0; phase < 2; ++phase) {
    char* ws = (char*)workspace;
    for (int g = 0; g < njobs; g += IMAXJ) {
      const int ng = std::min(IMAXJ, njobs - g);
      const int rc = invert_group(jobs + g, ng, ws, info ? info + g : nullptr, (hipStream_t)stream,
                                  phase);
      if (rc) return rc;
      for (int i = g; i < g + ng; ++i) ws += job_ws(jobs[i]);
    }
    if (phase == 0 && inputs_read &&
        hipEventRecord((hipEvent_t)inputs_read, (hipStream_t)stream) != hipSuccess)
      return KFAC_ELAUNCH;
  }
  return KFAC_OK;
}

extern "C" int kfac_invert(const kfac_invert_job* jobs, int njobs, void* workspace,
                           size_t workspace_bytes, int32_t* info, kfac_stream_t stream) {
  return kfac_invert_ex(jobs, njobs, workspace, workspace_bytes, info, nullptr, stream);
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
