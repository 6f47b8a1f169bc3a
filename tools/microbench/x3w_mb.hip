// bf16x3 register-split SYRK: wave-tile shape A/B for kfac_factor_tiles_x3 (DESIGN.md
// §3.1c).  Every variant computes the same region -- the 15 off-diagonal 128 x 128
// macro tiles of a 768-column row-major fp32 operand (ld 784, the MNIST MLP's layer-1
// activations) over K = 30,720 rows -- as split-K partial slabs, with the exact
// three-part bf16 split made in registers (6 v_mfma_f32_32x32x16_bf16 per 32 x 32
// block and 16 k).  What differs is how many MFMAs one split fragment feeds:
//   x3_64   : the production shape, a 128-thread workgroup per 64 x 64 tile, each wave
//             the whole tile over its half of each 32-row stage (4 fragments / 24 MFMA)
//   w128    : ONE wave per 128 x 128 macro tile (8 fragments / 96 MFMA, 256 acc)
//   w128x64 : one wave per 128 x 64 half tile (6 fragments / 48 MFMA)
//   pair    : two waves per macro tile, each 128 x 64, the A fragments split once
//             and exchanged through LDS (4 fragments / 48 MFMA per wave, 1 barrier per
//             16-row substep)
// Prints per variant: kernel time (best of reps), TF/s (fp32-equivalent on the
// computed blocks), vs the 417 TF/s bf16x3 roofline, and the max relative error of
// one macro tile against an fp64 recompute.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o x3w_mb x3w_mb.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int K = 30720, COLS = 768, LD = 784, MT = 128;
constexpr int T3 = COLS / MT;                  // 6 macro tile rows
constexpr int NTILE = T3 * (T3 - 1) / 2;       // 15 off-diagonal macro tiles

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ void offdiag_decode(int t, int& I, int& J) {  // I > J
  int i = 1;
  while (t >= i) { t -= i; ++i; }
  I = i;
  J = t;
}

__device__ __forceinline__ int acc_row(int v, int lane) { return (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5); }

__device__ __forceinline__ uint32_t bf16_pair(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float sub_f32(float x, float y) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ void split3(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = bf16_pair(a, b);
  const float ra = sub_f32(a, __uint_as_float(h << 16)), rb = sub_f32(b, __uint_as_float(h & 0xffff0000u));
  m = bf16_pair(ra, rb);
  const float sa = sub_f32(ra, __uint_as_float(m << 16)), sb = sub_f32(rb, __uint_as_float(m & 0xffff0000u));
  l = bf16_pair(sa, sb);
}
struct Frag {
  bf16x8 p[3];
};
__device__ __forceinline__ Frag split8(const float (&x)[8]) {
  u32x4 h, m, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t a, b, c;
    split3(x[2 * i], x[2 * i + 1], a, b, c);
    h[i] = a;
    m[i] = b;
    l[i] = c;
  }
  Frag f;
  f.p[0] = __builtin_bit_cast(bf16x8, h);
  f.p[1] = __builtin_bit_cast(bf16x8, m);
  f.p[2] = __builtin_bit_cast(bf16x8, l);
  return f;
}
__device__ __forceinline__ void six(floatx16& acc, const Frag& A, const Frag& B) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[2], B.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[1], B.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[0], B.p[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[1], B.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[0], B.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.p[0], B.p[0], acc, 0, 0, 0);
}
// 8 k of one column: rows r0 .. r0+7 (byte offset voff of row r0 / column), buffer loads
__device__ __forceinline__ void load8(float (&x)[8], __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
#pragma unroll
  for (int r = 0; r < 8; ++r)
    x[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff + r * LD * 4, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* X) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), 0, K * LD * 4, 0x00020000);
}

// ---------------------------------------------------------------- x3_64 (production shape)
__global__ __launch_bounds__(128, 2) void k_x3_64(const float* X, int splits, float* slab) {
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile >> 2, I, J);
  const int ti = 2 * I + ((tile >> 1) & 1), tj = 2 * J + (tile & 1);
  const int chunk = K / splits, k0 = split * chunk;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const auto rs = rsrc(X);
  const int lr = 16 * w + 8 * (lane >> 5);
  int vo[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) vo[f] = (lr * LD + (f < 2 ? ti : tj) * 64 + (f & 1) * 32 + (lane & 31)) * 4;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float xn[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f) load8(xn[f], rs, vo[f], k0 * LD * 4);
  for (int k = k0; k < k0 + chunk; k += 32) {
    float x[4][8];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 8; ++r) x[f][r] = xn[f][r];
#pragma unroll
    for (int f = 0; f < 4; ++f) load8(xn[f], rs, vo[f], (k + 32) * LD * 4);  // (unconditional: no branch)
    const Frag A0 = split8(x[0]), B0 = split8(x[2]);
    six(acc[0][0], A0, B0);
    const Frag A1 = split8(x[1]);
    six(acc[1][0], A1, B0);
    const Frag B1 = split8(x[3]);
    six(acc[0][1], A0, B1);
    six(acc[1][1], A1, B1);
  }
  // (the two waves' partials are summed in the production kernel's epilogue; here
  // each wave writes its own half slab)
  float* o = slab + ((size_t)task * 2 + w) * 64 * 64;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[(a * 32 + acc_row(v, lane)) * 64 + b * 32 + (lane & 31)] = acc[a][b][v];
}

// ---------------------------------------------------------------- w128: one wave, 128 x 128
template <int NB>  // column blocks of the wave tile: 4 (128 x 128) or 2 (128 x 64)
__device__ __forceinline__ void wave_tile(const float* X, int I, int c0, int k0, int chunk, float* o) {
  const int lane = threadIdx.x & 63;
  const auto rs = rsrc(X);
  const int lr = 8 * (lane >> 5);
  int va[4], vb[NB];
#pragma unroll
  for (int f = 0; f < 4; ++f) va[f] = (lr * LD + I * MT + f * 32 + (lane & 31)) * 4;
#pragma unroll
  for (int f = 0; f < NB; ++f) vb[f] = (lr * LD + c0 + f * 32 + (lane & 31)) * 4;
  floatx16 acc[4][NB];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float na[4][8], nb[NB][8];
#pragma unroll
  for (int f = 0; f < 4; ++f) load8(na[f], rs, va[f], k0 * LD * 4);
#pragma unroll
  for (int f = 0; f < NB; ++f) load8(nb[f], rs, vb[f], k0 * LD * 4);
  for (int k = k0; k < k0 + chunk; k += 16) {
    Frag B[NB];
#pragma unroll
    for (int f = 0; f < NB; ++f) {
      B[f] = split8(nb[f]);
      load8(nb[f], rs, vb[f], (k + 16) * LD * 4);  // (unconditional: past the end reads 0)
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const Frag A = split8(na[a]);
      load8(na[a], rs, va[a], (k + 16) * LD * 4);
#pragma unroll
      for (int b = 0; b < NB; ++b) six(acc[a][b], A, B[b]);
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        o[(a * 32 + acc_row(v, lane)) * (32 * NB) + b * 32 + (lane & 31)] = acc[a][b][v];
}

__global__ __launch_bounds__(64, 1) void k_w128(const float* X, int splits, float* slab) {
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile, I, J);
  const int chunk = K / splits;
  wave_tile<4>(X, I, J * MT, split * chunk, chunk, slab + (size_t)task * MT * MT);
}

__global__ __launch_bounds__(64, 1) void k_w128x64(const float* X, int splits, float* slab) {
  const int task = blockIdx.x, half = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(half >> 1, I, J);
  const int chunk = K / splits;
  wave_tile<2>(X, I, J * MT + (half & 1) * 64, split * chunk, chunk, slab + (size_t)task * MT * 64);
}

// ---------------------------------------------------------------- pair: 2 waves, A via LDS
// wave w splits A fragments 2w, 2w+1 (rows 64w .. 64w+63 of the macro tile) and its own
// B fragments (columns 64w ..), writes its A parts to the LDS slot of the substep, and
// after the barrier reads the other wave's two.  Slots double-buffered by substep parity.
__global__ __launch_bounds__(128, 1) void k_pair(const float* X, int splits, float* slab) {
  __shared__ __attribute__((aligned(16))) char lds[2][4][3][64 * 16];  // slot, A frag, part, lanes
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile, I, J);
  const int chunk = K / splits, k0 = split * chunk;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const auto rs = rsrc(X);
  const int lr = 8 * (lane >> 5);
  int va[2], vb[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    va[f] = (lr * LD + I * MT + (2 * w + f) * 32 + (lane & 31)) * 4;
    vb[f] = (lr * LD + J * MT + (2 * w + f) * 32 + (lane & 31)) * 4;
  }
  floatx16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float na[2][8], nb[2][8];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    load8(na[f], rs, va[f], k0 * LD * 4);
    load8(nb[f], rs, vb[f], k0 * LD * 4);
  }
  int slot = 0;
  for (int k = k0; k < k0 + chunk; k += 16) {
    Frag A[4], B[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      A[2 * w + f] = split8(na[f]);  // (w is wave-uniform: the compiler keeps both arms)
      load8(na[f], rs, va[f], (k + 16) * LD * 4);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        *reinterpret_cast<bf16x8*>(&lds[slot][2 * w + f][p][lane * 16]) = A[2 * w + f].p[p];
    }
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      B[f] = split8(nb[f]);
      load8(nb[f], rs, vb[f], (k + 16) * LD * 4);
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        A[2 * (1 - w) + f].p[p] = *reinterpret_cast<const bf16x8*>(&lds[slot][2 * (1 - w) + f][p][lane * 16]);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) six(acc[a][b], A[a], B[b]);
    slot ^= 1;
  }
  float* o = slab + ((size_t)task * 2 + w) * MT * 64;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[(a * 32 + acc_row(v, lane)) * 64 + b * 32 + (lane & 31)] = acc[a][b][v];
}


// ---------------------------------------------------------------- w128d: one wave, 128 x 128,
// operand rows by LDS-DMA.  Per 16-row substep the wave issues 16 buffer_load_dwordx4 ... lds
// (row r of the substep: lanes 0-31 bring 4 columns each of the A panel, lanes 32-63 of the
// B panel: one 1 KB LDS row of [A 128 | B 128] floats), one substep ahead, into a 2-slot
// ring of 16 KB; no VGPRs hold in-flight data, so the next substep's loads are issued at
// the top of the iteration and waited for one iteration later (vmcnt(16)).  Fragments
// are gathered with ds_read_b32 (lanes l, l+32: rows i, 8+i of one column -- the two
// 32-lane halves never conflict), split in registers, 96 MFMAs.
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_read8(float (&x)[8], const float* base) {  // rows 0..7 of the lane's column
#pragma unroll
  for (int r = 0; r < 8; ++r) x[r] = base[r * 256];
}
__global__ __launch_bounds__(64, 1) void k_w128d(const float* X, int splits, float* slab) {
  extern __shared__ __attribute__((aligned(16))) float dl[];  // 2 slots x 16 rows x 256
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile, I, J);
  const int chunk = K / splits, k0 = split * chunk;
  const int lane = threadIdx.x & 63;
  const auto rs = rsrc(X);
  const int dvo = (lane < 32 ? I * MT + 4 * lane : J * MT + 4 * (lane - 32)) * 4;
  auto issue = [&](int k, int slot) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dl + slot * 4096 + r * 256, 16, dvo, (k + r) * LD * 4, 0, 0);
  };
  floatx16 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  const int rd = 8 * (lane >> 5) * 256 + (lane & 31);  // the lane's column, its first row
  issue(k0, 0);
  int slot = 0;
  for (int k = k0; k < k0 + chunk; k += 16) {
    issue(k + 16, slot ^ 1);  // (past the chunk: harmless reads of the next rows / OOB zeros)
    vm_wait_n<16>();          // this substep's 16 pieces have landed
    const float* sl = dl + slot * 4096 + rd;
    Frag B[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      float x[8];
      lds_read8(x, sl + 128 + 32 * f);
      B[f] = split8(x);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float x[8];
      lds_read8(x, sl + 32 * a);
      const Frag A = split8(x);
#pragma unroll
      for (int b = 0; b < 4; ++b) six(acc[a][b], A, B[b]);
    }
    slot ^= 1;
  }
  float* o = slab + (size_t)task * MT * MT;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[(a * 32 + acc_row(v, lane)) * MT + b * 32 + (lane & 31)] = acc[a][b][v];
}


// ---------------------------------------------------------------- pinned-prefetch variants:
// the next stage's loads go out at the TOP of the iteration into their own registers and a
// sched_barrier keeps the scheduler from sinking them next to their use (the compiled
// x3_64 / w128 loops issue every load at the END of the body and wait vmcnt(0) at the
// head: the whole L2 latency exposed per stage).  IL: also interleave 1 MFMA with VALU.
#define SB() __builtin_amdgcn_sched_barrier(0)
template <bool IL>
__global__ __launch_bounds__(128, 2) void k_x3_64p(const float* X, int splits, float* slab) {
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile >> 2, I, J);
  const int ti = 2 * I + ((tile >> 1) & 1), tj = 2 * J + (tile & 1);
  const int chunk = K / splits, k0 = split * chunk;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const auto rs = rsrc(X);
  const int lr = 16 * w + 8 * (lane >> 5);
  int vo[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) vo[f] = (lr * LD + (f < 2 ? ti : tj) * 64 + (f & 1) * 32 + (lane & 31)) * 4;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  // ping-pong register buffers, loop unrolled by two: no loop-carried copies (a copy
  // xn -> x makes the compiler wait for the fresh loads inside the same iteration)
  float x0[4][8], x1[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f) load8(x0[f], rs, vo[f], k0 * LD * 4);
  auto body = [&](float (&x)[4][8], float (&xn)[4][8], int k) {
#pragma unroll
    for (int f = 0; f < 4; ++f) load8(xn[f], rs, vo[f], (k + 32) * LD * 4);
    SB();
    const Frag A0 = split8(x[0]), B0 = split8(x[2]);
    six(acc[0][0], A0, B0);
    const Frag A1 = split8(x[1]);
    six(acc[1][0], A1, B0);
    const Frag B1 = split8(x[3]);
    six(acc[0][1], A0, B1);
    six(acc[1][1], A1, B1);
    if constexpr (IL) {
#pragma unroll
      for (int i = 0; i < 24; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, 6, 0);
      }
    }
    SB();
  };
  for (int k = k0; k < k0 + chunk; k += 64) {  // (chunk: a multiple of 64)
    body(x0, x1, k);
    body(x1, x0, k + 32);
  }
  float* o = slab + ((size_t)task * 2 + w) * 64 * 64;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[(a * 32 + acc_row(v, lane)) * 64 + b * 32 + (lane & 31)] = acc[a][b][v];
}

template <bool IL>
__global__ __launch_bounds__(64, 1) void k_w128p(const float* X, int splits, float* slab) {
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile, I, J);
  const int chunk = K / splits, k0 = split * chunk;
  const int lane = threadIdx.x & 63;
  const auto rs = rsrc(X);
  const int lr = 8 * (lane >> 5);
  int vo[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) vo[f] = (lr * LD + (f < 4 ? I : J) * MT + (f & 3) * 32 + (lane & 31)) * 4;
  floatx16 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float x0[8][8], x1[8][8];
#pragma unroll
  for (int f = 0; f < 8; ++f) load8(x0[f], rs, vo[f], k0 * LD * 4);
  auto body = [&](float (&x)[8][8], float (&xn)[8][8], int k) {
#pragma unroll
    for (int f = 0; f < 8; ++f) load8(xn[f], rs, vo[f], (k + 16) * LD * 4);
    SB();
    Frag B[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) B[f] = split8(x[4 + f]);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const Frag A = split8(x[a]);
#pragma unroll
      for (int b = 0; b < 4; ++b) six(acc[a][b], A, B[b]);
    }
    if constexpr (IL) {
#pragma unroll
      for (int i = 0; i < 96; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, 4, 0);
      }
    }
    SB();
  };
  for (int k = k0; k < k0 + chunk; k += 32) {  // (chunk: a multiple of 32)
    body(x0, x1, k);
    body(x1, x0, k + 16);
  }
  float* o = slab + (size_t)task * MT * MT;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[(a * 32 + acc_row(v, lane)) * MT + b * 32 + (lane & 31)] = acc[a][b][v];
}


// ---------------------------------------------------------------- x3_64s: software-pipelined
// segments.  The first block's fragments (A0, B0) are split during the previous stage;
// each segment = 6 MFMAs of one block interleaved (sched_group_barrier) with the split
// of the fragment a later block needs and the reload of that fragment's registers for
// the next stage:
//   seg1: MFMA(0,0) || split A1, reload x1      seg2: MFMA(1,0) || split B1, reload x3
//   seg3: MFMA(0,1) || split A0', reload x0     seg4: MFMA(1,1) || split B0', reload x2
// so every load is issued one whole stage before its split, no register set is copied
// and 5 fragments at most are live.
__device__ __forceinline__ void seg_pattern() {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x2, 7, 0);
    __builtin_amdgcn_sched_group_barrier(0x20, 2, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x2, 8, 0);
  }
}
template <bool PAT>
__global__ __launch_bounds__(128, 2) void k_x3_64s(const float* X, int splits, float* slab) {
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile >> 2, I, J);
  const int ti = 2 * I + ((tile >> 1) & 1), tj = 2 * J + (tile & 1);
  const int chunk = K / splits, k0 = split * chunk;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const auto rs = rsrc(X);
  const int lr = 16 * w + 8 * (lane >> 5);
  int vo[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) vo[f] = (lr * LD + (f < 2 ? ti : tj) * 64 + (f & 1) * 32 + (lane & 31)) * 4;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float x[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f) load8(x[f], rs, vo[f], k0 * LD * 4);
  // prologue: A0, B0 of stage 0; their registers reloaded with stage 1
  Frag A0 = split8(x[0]), B0 = split8(x[2]);
  load8(x[0], rs, vo[0], (k0 + 32) * LD * 4);
  load8(x[2], rs, vo[2], (k0 + 32) * LD * 4);
  for (int k = k0; k < k0 + chunk; k += 32) {
    const int kn = (k + 32) * LD * 4, knn = (k + 64) * LD * 4;  // (past the end: harmless)
    SB();
    // seg1
    const Frag A1 = split8(x[1]);
    load8(x[1], rs, vo[1], kn);
    six(acc[0][0], A0, B0);
    if (PAT) seg_pattern();
    SB();
    // seg2
    const Frag B1 = split8(x[3]);
    load8(x[3], rs, vo[3], kn);
    six(acc[1][0], A1, B0);
    if (PAT) seg_pattern();
    SB();
    // seg3: the next stage's A0 (its loads went out in the previous stage)
    const Frag A0n = split8(x[0]);
    load8(x[0], rs, vo[0], knn);
    six(acc[0][1], A0, B1);
    if (PAT) seg_pattern();
    SB();
    // seg4
    const Frag B0n = split8(x[2]);
    load8(x[2], rs, vo[2], knn);
    six(acc[1][1], A1, B1);
    if (PAT) seg_pattern();
    A0 = A0n;
    B0 = B0n;
  }
  float* o = slab + ((size_t)task * 2 + w) * 64 * 64;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[(a * 32 + acc_row(v, lane)) * 64 + b * 32 + (lane & 31)] = acc[a][b][v];
}


// ---------------------------------------------------------------- ablations: what bounds it?
// MODE bit 0: load the operand rows each stage (else the registers are made opaque by an
// empty asm, no instruction); bit 1: split them (else fixed fragments split once).
// The MFMA count and order are those of x3_64 (2 waves / SIMD) and w128 (1 wave / SIMD).
template <int MODE>
__global__ __launch_bounds__(128, 2) void k_x364m(const float* X, int splits, float* slab) {
  constexpr bool LOAD = MODE & 1, SPLIT = (MODE & 2) != 0;
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  offdiag_decode(tile >> 2, I, J);
  const int ti = 2 * I + ((tile >> 1) & 1), tj = 2 * J + (tile & 1);
  const int chunk = K / splits, k0 = split * chunk;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const auto rs = rsrc(X);
  const int lr = 16 * w + 8 * (lane >> 5);
  int vo[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) vo[f] = (lr * LD + (f < 2 ? ti : tj) * 64 + (f & 1) * 32 + (lane & 31)) * 4;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float x[4][8];
#pragma unroll
  for (int f = 0; f < 4; ++f) load8(x[f], rs, vo[f], k0 * LD * 4);
  Frag F0 = split8(x[0]), F1 = split8(x[1]), F2 = split8(x[2]), F3 = split8(x[3]);
  for (int k = k0; k < k0 + chunk; k += 32) {
    if (LOAD) {
#pragma unroll
      for (int f = 0; f < 4; ++f) load8(x[f], rs, vo[f], (k + 32) * LD * 4);
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(x[f][r]));
    }
    Frag A0 = F0, A1 = F1, B0 = F2, B1 = F3;
    if (SPLIT) {
      A0 = split8(x[0]);
      B0 = split8(x[2]);
      A1 = split8(x[1]);
      B1 = split8(x[3]);
    } else if (LOAD) {  // keep the loads alive: fold one value into the accumulator chain
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int r = 0; r < 8; ++r) asm volatile("" ::"v"(x[f][r]));
    }
    if constexpr ((MODE & 4) != 0) {  // the 24 MFMAs round-robin over the 4 accumulators
#define X4(pa, pb)                                                                          \
  acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0.p[pa], B0.p[pb], acc[0][0], 0, 0, 0); \
  acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1.p[pa], B0.p[pb], acc[1][0], 0, 0, 0); \
  acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0.p[pa], B1.p[pb], acc[0][1], 0, 0, 0); \
  acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1.p[pa], B1.p[pb], acc[1][1], 0, 0, 0);
      X4(2, 0) X4(1, 1) X4(0, 2) X4(1, 0) X4(0, 1) X4(0, 0)
#undef X4
    } else {
      six(acc[0][0], A0, B0);
      six(acc[1][0], A1, B0);
      six(acc[0][1], A0, B1);
      six(acc[1][1], A1, B1);
    }
  }
  float* o = slab + ((size_t)task * 2 + w) * 64 * 64;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[(a * 32 + acc_row(v, lane)) * 64 + b * 32 + (lane & 31)] = acc[a][b][v];
}

// fp64 reference of macro tile (I, J): out[r][c] = sum_k X[k][I*128+r] X[k][J*128+c]
__global__ void k_ref(const float* X, int I, int J, double* out) {
  const int r = blockIdx.x, c = threadIdx.x;
  double s = 0;
  for (int k = 0; k < K; ++k) s += (double)X[(size_t)k * LD + I * MT + r] * (double)X[(size_t)k * LD + J * MT + c];
  out[r * MT + c] = s;
}

int main() {
  std::vector<float> h((size_t)K * LD);
  uint64_t st = 88172645463325252ull;
  for (auto& v : h) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    v = (float)((st >> 11) * (1.0 / 9007199254740992.0));  // U[0,1): post-ReLU-like
  }
  float* X;
  CHECK(hipMalloc(&X, h.size() * 4));
  CHECK(hipMemcpy(X, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  float* slab;
  const size_t slab_bytes = (size_t)2048 * MT * MT * 4;
  CHECK(hipMalloc(&slab, slab_bytes));
  double* ref;
  CHECK(hipMalloc(&ref, MT * MT * 8));
  const int RI = 3, RJ = 1;  // the checked macro tile
  int tref = 0;
  for (int i = 1; i < RI; ++i) tref += i;
  tref += RJ;
  hipLaunchKernelGGL(k_ref, dim3(MT), dim3(MT), 0, 0, X, RI, RJ, ref);
  std::vector<double> href(MT * MT);
  CHECK(hipMemcpy(href.data(), ref, MT * MT * 8, hipMemcpyDeviceToHost));
  const double flops = 2.0 * K * NTILE * MT * MT;
  struct V {
    const char* name;
    int threads, splits, tasks;
  };
  // splits: one round of resident workgroups (x3_64 / w128 / w128x64: 4 per CU; pair: 2)
  const V vs[] = {{"x3_64", 128, 16, 4 * NTILE * 16}, {"w128", 64, 64, NTILE * 64},
                  {"w128x64", 64, 32, 2 * NTILE * 32}, {"pair", 128, 32, NTILE * 32},
                  {"w128d", 64, 64, NTILE * 64}, {"x3_64p", 128, 16, 4 * NTILE * 16},
                  {"x3_64pi", 128, 16, 4 * NTILE * 16}, {"w128p", 64, 64, NTILE * 64},
                  {"w128pi", 64, 64, NTILE * 64}, {"x3_64s", 128, 16, 4 * NTILE * 16},
                  {"x3_64sp", 128, 16, 4 * NTILE * 16}, {"m0_mfma", 128, 16, 4 * NTILE * 16},
                  {"m1_load", 128, 16, 4 * NTILE * 16}, {"m2_split", 128, 16, 4 * NTILE * 16},
                  {"m3_all", 128, 16, 4 * NTILE * 16}, {"m4_mfma_il", 128, 16, 4 * NTILE * 16},
                  {"m7_all_il", 128, 16, 4 * NTILE * 16}, {"m6_split_il", 128, 16, 4 * NTILE * 16}};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (const V& v : vs) {
    auto launch = [&]() {
      if (!strcmp(v.name, "m0_mfma")) hipLaunchKernelGGL(k_x364m<0>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "m1_load")) hipLaunchKernelGGL(k_x364m<1>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "m2_split")) hipLaunchKernelGGL(k_x364m<2>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "m3_all")) hipLaunchKernelGGL(k_x364m<3>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "m4_mfma_il")) hipLaunchKernelGGL(k_x364m<4>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "m6_split_il")) hipLaunchKernelGGL(k_x364m<6>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "m7_all_il")) hipLaunchKernelGGL(k_x364m<7>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "x3_64s")) hipLaunchKernelGGL(k_x3_64s<false>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "x3_64sp")) hipLaunchKernelGGL(k_x3_64s<true>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "x3_64")) hipLaunchKernelGGL(k_x3_64, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "x3_64p")) hipLaunchKernelGGL(k_x3_64p<false>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "x3_64pi")) hipLaunchKernelGGL(k_x3_64p<true>, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "w128p")) hipLaunchKernelGGL(k_w128p<false>, dim3(v.tasks), dim3(64), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "w128pi")) hipLaunchKernelGGL(k_w128p<true>, dim3(v.tasks), dim3(64), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "w128")) hipLaunchKernelGGL(k_w128, dim3(v.tasks), dim3(64), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "w128x64")) hipLaunchKernelGGL(k_w128x64, dim3(v.tasks), dim3(64), 0, 0, X, v.splits, slab);
      else if (!strcmp(v.name, "pair")) hipLaunchKernelGGL(k_pair, dim3(v.tasks), dim3(128), 0, 0, X, v.splits, slab);
      else hipLaunchKernelGGL(k_w128d, dim3(v.tasks), dim3(64), 32768, 0, X, v.splits, slab);
    };
    launch();
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 10; ++r) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    // sum the checked macro tile's partials on the host
    std::vector<float> hs(slab_bytes / 4);
    CHECK(hipMemcpy(hs.data(), slab, slab_bytes, hipMemcpyDeviceToHost));
    std::vector<double> got(MT * MT, 0.0);
    for (int s = 0; s < v.splits; ++s) {
      for (int r = 0; r < MT; ++r)
        for (int c = 0; c < MT; ++c) {
          double x = 0;
          if (v.name[0] == 'x' || v.name[0] == 'm') {  // 4 64-tiles x 2 waves (all x3_64 variants)
            const int q = (r / 64) * 2 + c / 64;
            const size_t task = (size_t)(tref * 4 + q) * v.splits + s;
            for (int w = 0; w < 2; ++w) x += hs[(task * 2 + w) * 4096 + (r % 64) * 64 + c % 64];
          } else if (!strncmp(v.name, "w128", 4) && strcmp(v.name, "w128x64")) {
            x = hs[((size_t)tref * v.splits + s) * MT * MT + r * MT + c];
          } else if (!strcmp(v.name, "w128x64")) {
            const size_t task = (size_t)(tref * 2 + c / 64) * v.splits + s;
            x = hs[task * MT * 64 + r * 64 + c % 64];
          } else {
            const size_t task = (size_t)tref * v.splits + s;
            x = hs[(task * 2 + c / 64) * MT * 64 + r * 64 + c % 64];
          }
          got[r * MT + c] += x;
        }
    }
    double err = 0;
    for (int i = 0; i < MT * MT; ++i) err = std::max(err, std::fabs(got[i] - href[i]) / std::fabs(href[i]));
    printf("%-8s %8.1f us  %6.1f TF/s  %.3f of 417  max rel err %.2e\n", v.name, best * 1e3,
           flops / (best * 1e-3) / 1e12, flops / (best * 1e-3) / 1e12 / 416.7, err);
  }
  return 0;
}
