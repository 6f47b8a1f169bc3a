// bf16x3 SYRK with CU-sized tiles: the operand panels of a 16-row stage are loaded and
// split ONCE per workgroup into an LDS image (3 bf16 parts, MFMA fragment layout), and
// the waves run their MFMAs from LDS.  Compared with kfac_factor_tiles_x3 (every wave
// splits the fragments of its own 64 x 64 tile: 7.3 split VALU per MFMA) the split
// costs ~1.8 VALU per MFMA here.  Region: the 3 off-diagonal 256 x 256 tiles of a
// 768-column fp32 operand (ld 784) over K rows, split-K partial slabs per task.
//   cu4 : 256 threads, 4 waves (1 per SIMD), wave tile 128 x 128 (16 blocks, 256 acc)
//   cu8 : 512 threads, 8 waves (2 per SIMD), wave tile  64 x 128 ( 8 blocks, 128 acc)
//   *_m : MFMA + LDS reads only (no loads, no split): the ceiling of the shape
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o cut_mb cut_mb.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int K = 61440, COLS = 768, LD = 784;
constexpr int CT = 256;           // CU tile edge
constexpr int NP = 2 * CT;        // panel columns staged per stage (A | B)
constexpr int PART = NP * 32;     // bytes of one part of a stage: NP cols x 16 k x 2 B
constexpr int STG = 3 * PART;     // one stage buffer (48 KB)
constexpr int NTILE = 3;          // (1,0) (2,0) (2,1)

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

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
__device__ __forceinline__ void tile_of(int t, int& I, int& J) {
  I = t == 0 ? 1 : 2;
  J = t == 2 ? 1 : 0;
}

template <int NW, bool MFMA_ONLY>
__global__ __launch_bounds__(64 * NW, 1) void k_cut(const float* X, int splits, float* slab) {
  constexpr int NT = 64 * NW;
  constexpr int U = 1024 / NT;           // (column, k-half) units per thread and stage
  constexpr int RB = NW == 4 ? 4 : 2;    // 32-row blocks per wave tile
  constexpr int CB = 4;                  // 32-column blocks per wave tile
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  tile_of(tile, I, J);
  const int chunk = K / splits, k0 = split * chunk, ns = chunk / 16;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;   // wave tile (wr, wc): rows RB*32*wr, cols 128*wc
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), 0, K * LD * 4, 0x00020000);
  // this thread's units: q = u * NT + t -> panel column c = q % 512, k-half h = q / 512
  int voff[U], woff[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = u * NT + t, c = q % NP, h = q / NP;
    const int gc = c < CT ? I * CT + c : J * CT + (c - CT);
    voff[u] = (8 * h * LD + gc) * 4;
    woff[u] = h * (NP * 16) + c * 16;
  }
  floatx16 acc[RB][CB];
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float L0[U][8], L1[U][8];
  auto load = [&](float (&L)[U][8], int kk) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < 8; ++r)
        L[u][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff[u], (kk + r) * LD * 4, 0));
  };
  auto put = [&](const float (&L)[U][8], char* buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u32x4 hp, mp, lp;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t a, b, c;
        split3(L[u][2 * i], L[u][2 * i + 1], a, b, c);
        hp[i] = a;
        mp[i] = b;
        lp[i] = c;
      }
      *reinterpret_cast<u32x4*>(buf + woff[u]) = hp;
      *reinterpret_cast<u32x4*>(buf + PART + woff[u]) = mp;
      *reinterpret_cast<u32x4*>(buf + 2 * PART + woff[u]) = lp;
    }
  };
  // fragment read offsets (part 0): A block a: panel column RB*32*wr + 32a, B block b: 256 + 128wc + 32b
  const int fo = (lane >> 5) * (NP * 16) + (lane & 31) * 16;
  const int ao = fo + (RB * 32 * wr) * 16, bo = fo + (CT + 128 * wc) * 16;
  auto frag = [&](const char* buf, int off) { return *reinterpret_cast<const bf16x8*>(buf + off); };
  if (MFMA_ONLY) {
    load(L0, k0);
    put(L0, lds);
    put(L0, lds + STG);
  } else {
    load(L0, k0);
    put(L0, lds);
    load(L1, k0 + 16);
  }
  __syncthreads();
  for (int s = 0; s < ns; ++s) {
    const char* cur = lds + (s & 1) * STG;
    char* nxt = lds + ((s + 1) & 1) * STG;
    bf16x8 B[CB][3];
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int p = 0; p < 3; ++p) B[b][p] = frag(cur, bo + p * PART + b * 32 * 16);
    if (!MFMA_ONLY) {
      // the stage after next into the registers the current stage was split from
      if (s & 1) load(L1, k0 + 16 * (s + 2));
      else load(L0, k0 + 16 * (s + 2));
    }
#pragma unroll
    for (int a = 0; a < RB; ++a) {
      bf16x8 A[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) A[p] = frag(cur, ao + p * PART + a * 32 * 16);
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[b][0], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[b][1], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[b][2], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[b][0], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[b][1], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[b][0], acc[a][b], 0, 0, 0);
      }
    }
    if (!MFMA_ONLY && s + 1 < ns) {
      // the next stage (loaded one stage ago) split into the other buffer; its loads
      // are older than the ones just issued
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * U) : "memory");
      if (s & 1) put(L0, nxt);
      else put(L1, nxt);
    }
    __syncthreads();
  }
  float* o = slab + (size_t)task * CT * CT;
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        o[(RB * 32 * wr + a * 32 + acc_row(v, lane)) * CT + 128 * wc + b * 32 + (lane & 31)] = acc[a][b][v];
}

// cuti: the split of the next stage interleaved with this stage's MFMAs: unit u (one
// column x 8 rows) is split and written during MFMA row a = u (24 MFMAs), NV VALU per
// MFMA in the pattern.  LZ: B fragments read just before their first use (else all at
// the top of the stage); VM: the stage-after-next loads spread one per MFMA (else all
// issued before the first MFMA).
#define SB() __builtin_amdgcn_sched_barrier(0)
template <int NW, int NV, bool LZ, bool VM>
__global__ __launch_bounds__(64 * NW, 1) void k_cuti(const float* X, int splits, float* slab) {
  constexpr int NT = 64 * NW;
  constexpr int U = 1024 / NT;
  constexpr int RB = NW == 4 ? 4 : 2;
  constexpr int CB = 4;
  static_assert(U == RB, "one unit split per MFMA row");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  tile_of(tile, I, J);
  const int chunk = K / splits, k0 = split * chunk, ns = chunk / 16;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), 0, K * LD * 4, 0x00020000);
  int voff[U], woff[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = u * NT + t, c = q % NP, h = q / NP;
    const int gc = c < CT ? I * CT + c : J * CT + (c - CT);
    voff[u] = (8 * h * LD + gc) * 4;
    woff[u] = h * (NP * 16) + c * 16;
  }
  floatx16 acc[RB][CB];
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  float L0[U][8], L1[U][8];
  auto load = [&](float (&L)[U][8], int kk) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < 8; ++r)
        L[u][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff[u], (kk + r) * LD * 4, 0));
  };
  auto put1 = [&](const float (&x)[8], char* buf, int wo) {
    u32x4 hp, mp, lp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t a, b, c;
      split3(x[2 * i], x[2 * i + 1], a, b, c);
      hp[i] = a;
      mp[i] = b;
      lp[i] = c;
    }
    *reinterpret_cast<u32x4*>(buf + wo) = hp;
    *reinterpret_cast<u32x4*>(buf + PART + wo) = mp;
    *reinterpret_cast<u32x4*>(buf + 2 * PART + wo) = lp;
  };
  const int fo = (lane >> 5) * (NP * 16) + (lane & 31) * 16;
  const int ao = fo + (RB * 32 * wr) * 16, bo = fo + (CT + 128 * wc) * 16;
  auto frag = [&](const char* buf, int off) { return *reinterpret_cast<const bf16x8*>(buf + off); };
  load(L0, k0);
#pragma unroll
  for (int u = 0; u < U; ++u) put1(L0[u], lds, woff[u]);
  load(L1, k0 + 16);
  __syncthreads();
  auto body = [&](int s, float (&Lsplit)[U][8], float (&Lload)[U][8]) {
    const char* cur = lds + (s & 1) * STG;
    char* nxt = lds + ((s + 1) & 1) * STG;
    bf16x8 B[CB][3], A[2][3];
    if (!LZ)
#pragma unroll
      for (int b = 0; b < CB; ++b)
#pragma unroll
        for (int p = 0; p < 3; ++p) B[b][p] = frag(cur, bo + p * PART + b * 32 * 16);
#pragma unroll
    for (int p = 0; p < 3; ++p) A[0][p] = frag(cur, ao + p * PART);
    if (!VM) load(Lload, k0 + 16 * (s + 2));  // (past the task's rows: harmless reads, never split)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM ? 0 : 8 * U) : "memory");  // Lsplit has landed
    SB();
#pragma unroll
    for (int a = 0; a < RB; ++a) {
      if (VM && a == 0) load(Lload, k0 + 16 * (s + 2));
      if (a + 1 < RB)
#pragma unroll
        for (int p = 0; p < 3; ++p) A[(a + 1) & 1][p] = frag(cur, ao + p * PART + (a + 1) * 32 * 16);
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        if (LZ && a == 0)
#pragma unroll
          for (int p = 0; p < 3; ++p) B[b][p] = frag(cur, bo + p * PART + b * 32 * 16);
        const bf16x8* Aa = A[a & 1];
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[2], B[b][0], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[1], B[b][1], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[0], B[b][2], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[1], B[b][0], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[0], B[b][1], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Aa[0], B[b][0], acc[a][b], 0, 0, 0);
      }
      if (s + 1 < ns) put1(Lsplit[a], nxt, woff[a]);
      if (LZ && a == 0) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      if (a + 1 < RB) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // the next A reads first
#pragma unroll
      for (int i = 0; i < 24; ++i) {
        if (VM && a == 0 && i < 8 * U) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (LZ && a == 0 && i % 6 == 5 && i < 18) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        if (i % 8 == 7) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
      SB();
    }
    __syncthreads();
  };
  for (int s = 0; s < ns; s += 2) {  // (ns even)
    body(s, L1, L0);
    body(s + 1, L0, L1);
  }
  float* o = slab + (size_t)task * CT * CT;
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        o[(RB * 32 * wr + a * 32 + acc_row(v, lane)) * CT + 128 * wc + b * 32 + (lane & 31)] = acc[a][b][v];
}

// cutk: cuti's structure (8 waves, split once per CU, interleaved) with
// v_mfma_f32_16x16x32_bf16 and the bf16x3 parts laid along K: the 32 k of one MFMA are
// [16 rows of part X | 16 rows of part Y], so per 16 x 16 block and 16-row stage
//   [h|m].[h|h] + [h|l].[m|h] + [h|m].[l|m] = hh + mh + hm + lh + hl + mm
// -- all six products of the exact split in three MFMAs of 16 cycles.  A lane's operand
// is 8 rows of one column of one part: its LDS address picks the part by lane >> 5.
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int NV, bool LZ, bool VM>
__global__ __launch_bounds__(512, 1) void k_cutk(const float* X, int splits, float* slab) {
  constexpr int NW = 8, NT = 512, U = 2;
  constexpr int RB = 4, CB = 8;  // 16 x 16 blocks of the 64 x 128 wave tile
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int I, J;
  tile_of(tile, I, J);
  const int chunk = K / splits, k0 = split * chunk, ns = chunk / 16;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), 0, K * LD * 4, 0x00020000);
  int voff[U], woff[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = u * NT + t, c = q % NP, h = q / NP;
    const int gc = c < CT ? I * CT + c : J * CT + (c - CT);
    voff[u] = (8 * h * LD + gc) * 4;
    woff[u] = h * (NP * 16) + c * 16;
  }
  floatx4 acc[RB][CB];
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[a][b][v] = 0.f;
  float L0[U][8], L1[U][8];
  auto load = [&](float (&L)[U][8], int kk) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < 8; ++r)
        L[u][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff[u], (kk + r) * LD * 4, 0));
  };
  auto put1 = [&](const float (&x)[8], char* buf, int wo) {
    u32x4 hp, mp, lp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t a, b, c;
      split3(x[2 * i], x[2 * i + 1], a, b, c);
      hp[i] = a;
      mp[i] = b;
      lp[i] = c;
    }
    *reinterpret_cast<u32x4*>(buf + wo) = hp;
    *reinterpret_cast<u32x4*>(buf + PART + wo) = mp;
    *reinterpret_cast<u32x4*>(buf + 2 * PART + wo) = lp;
  };
  // lane's column (lane & 15) and k-half ((lane >> 4) & 1) of part 0; hi = lane >> 5 picks
  // part Y of a fragment's second K half
  const int hi = lane >> 5;
  const int fo = ((lane >> 4) & 1) * (NP * 16) + (lane & 15) * 16;
  const int arow = fo + (64 * wr) * 16, bcol = fo + (CT + 128 * wc) * 16;
  const int a_hm = arow + hi * PART, a_hl = arow + hi * 2 * PART;
  const int b_hh = bcol, b_mh = bcol + (1 - hi) * PART, b_lm = bcol + (2 - hi) * PART;
  auto frag = [&](const char* buf, int off) { return *reinterpret_cast<const bf16x8*>(buf + off); };
  load(L0, k0);
#pragma unroll
  for (int u = 0; u < U; ++u) put1(L0[u], lds, woff[u]);
  load(L1, k0 + 16);
  __syncthreads();
  auto body = [&](int s, float (&Lsplit)[U][8], float (&Lload)[U][8]) {
    const char* cur = lds + (s & 1) * STG;
    char* nxt = lds + ((s + 1) & 1) * STG;
    bf16x8 A[RB][2], B[2][3];
#pragma unroll
    for (int a = 0; a < RB; ++a) {
      A[a][0] = frag(cur, a_hm + a * 16 * 16);
      A[a][1] = frag(cur, a_hl + a * 16 * 16);
    }
    auto readB = [&](int b, bf16x8 (&Bb)[3]) {
      Bb[0] = frag(cur, b_hh + b * 16 * 16);
      Bb[1] = frag(cur, b_mh + b * 16 * 16);
      Bb[2] = frag(cur, b_lm + b * 16 * 16);
    };
    readB(0, B[0]);
    if (!VM) load(Lload, k0 + 16 * (s + 2));
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM ? 0 : 8 * U) : "memory");  // Lsplit has landed
    SB();
#pragma unroll
    for (int half = 0; half < 2; ++half) {  // col blocks 4 half .. 4 half + 3: one unit split
      if (VM && half == 0) load(Lload, k0 + 16 * (s + 2));
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int b = 4 * half + bb;
        if (b + 1 < CB) readB(b + 1, B[(b + 1) & 1]);
        const bf16x8* Bb = B[b & 1];
#pragma unroll
        for (int a = 0; a < RB; ++a) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][0], Bb[0], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][1], Bb[1], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][0], Bb[2], acc[a][b], 0, 0, 0);
        }
      }
      if (s + 1 < ns) put1(Lsplit[half], nxt, woff[half]);
#pragma unroll
      for (int i = 0; i < 48; ++i) {
        if (VM && half == 0 && i < 8 * U) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if (i % 12 == 0 && (half == 0 || i < 36)) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (i % 2 == 1) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        if (i % 16 == 15) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
      SB();
    }
    __syncthreads();
  };
  for (int s = 0; s < ns; s += 2) {  // (ns even)
    body(s, L1, L0);
    body(s + 1, L0, L1);
  }
  float* o = slab + (size_t)task * CT * CT;
  // 16x16 accumulator: lane holds rows 4 (lane >> 4) + v of column lane & 15
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        o[(64 * wr + a * 16 + 4 * (lane >> 4) + v) * CT + 128 * wc + b * 16 + (lane & 15)] = acc[a][b][v];
}

__global__ void k_ref(const float* X, int I, int J, double* out) {
  const int r = blockIdx.x, c = threadIdx.x;
  double s = 0;
  for (int k = 0; k < K; ++k) s += (double)X[(size_t)k * LD + I * CT + r] * (double)X[(size_t)k * LD + J * CT + c];
  out[r * CT + c] = s;
}

int main() {
  std::vector<float> h((size_t)K * LD);
  uint64_t st = 88172645463325252ull;
  for (auto& v : h) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    v = (float)((st >> 11) * (1.0 / 9007199254740992.0));
  }
  float* X;
  CHECK(hipMalloc(&X, h.size() * 4));
  CHECK(hipMemcpy(X, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const int splits = 80;  // 240 tasks: one workgroup per CU, one round
  float* slab;
  const size_t slab_bytes = (size_t)NTILE * splits * CT * CT * 4;
  CHECK(hipMalloc(&slab, slab_bytes));
  double* ref;
  CHECK(hipMalloc(&ref, CT * CT * 8));
  const int RT = 2;  // checked tile: (2, 1)
  hipLaunchKernelGGL(k_ref, dim3(CT), dim3(CT), 0, 0, X, 2, 1, ref);
  std::vector<double> href(CT * CT);
  CHECK(hipMemcpy(href.data(), ref, CT * CT * 8, hipMemcpyDeviceToHost));
  const double flops = 2.0 * K * NTILE * CT * CT;
  CHECK(hipFuncSetAttribute((const void*)k_cut<4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG));
  CHECK(hipFuncSetAttribute((const void*)k_cut<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG));
  CHECK(hipFuncSetAttribute((const void*)k_cut<4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG));
  CHECK(hipFuncSetAttribute((const void*)k_cut<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG));
#define CUTI_VARIANTS(X) X(8, 4, false, false) X(8, 4, true, true)
#define ATTR(nw, nv, lz, vm) CHECK(hipFuncSetAttribute((const void*)k_cuti<nw, nv, lz, vm>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG));
  CUTI_VARIANTS(ATTR)
#define CUTK_VARIANTS(X) X(2, true, true) X(3, true, true) X(4, true, true) X(2, false, false)
#define ATTRK(nv, lz, vm) CHECK(hipFuncSetAttribute((const void*)k_cutk<nv, lz, vm>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG));
  CUTK_VARIANTS(ATTRK)
  std::vector<std::string> names = {"cu4", "cu8", "cu4_m", "cu8_m"};
#define NAME(nw, nv, lz, vm) names.push_back(std::string("cu") + #nw + "i" + #nv + (lz ? "L" : "") + (vm ? "V" : ""));
  CUTI_VARIANTS(NAME)
#define NAMEK(nv, lz, vm) names.push_back(std::string("k16_") + #nv + (lz ? "L" : "") + (vm ? "V" : ""));
  CUTK_VARIANTS(NAMEK)
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int vi = 0; vi < (int)names.size(); ++vi) {
    auto launch = [&]() {
      const int tasks = NTILE * splits;
      if (vi == 0) hipLaunchKernelGGL((k_cut<4, false>), dim3(tasks), dim3(256), 2 * STG, 0, X, splits, slab);
      if (vi == 1) hipLaunchKernelGGL((k_cut<8, false>), dim3(tasks), dim3(512), 2 * STG, 0, X, splits, slab);
      if (vi == 2) hipLaunchKernelGGL((k_cut<4, true>), dim3(tasks), dim3(256), 2 * STG, 0, X, splits, slab);
      if (vi == 3) hipLaunchKernelGGL((k_cut<8, true>), dim3(tasks), dim3(512), 2 * STG, 0, X, splits, slab);
      int vj = 4;
#define LAUNCH(nw, nv, lz, vm) if (vi == vj++) hipLaunchKernelGGL((k_cuti<nw, nv, lz, vm>), dim3(tasks), dim3(64 * nw), 2 * STG, 0, X, splits, slab);
      CUTI_VARIANTS(LAUNCH)
#define LAUNCHK(nv, lz, vm) if (vi == vj++) hipLaunchKernelGGL((k_cutk<nv, lz, vm>), dim3(tasks), dim3(512), 2 * STG, 0, X, splits, slab);
      CUTK_VARIANTS(LAUNCHK)
    };
    launch();
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    for (int r = 0; r < 20; ++r) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      sum += ms;
    }
    std::vector<float> hs(slab_bytes / 4);
    CHECK(hipMemcpy(hs.data(), slab, slab_bytes, hipMemcpyDeviceToHost));
    double err = 0;
    for (int i = 0; i < CT * CT; ++i) {
      double g = 0;
      for (int s = 0; s < splits; ++s) g += hs[((size_t)RT * splits + s) * CT * CT + i];
      err = std::max(err, std::fabs(g - href[i]) / std::fabs(href[i]));
    }
    printf("%-9s best %7.1f us mean %7.1f us  %6.1f TF/s  %.3f of 417  max rel err %.2e\n", names[vi].c_str(), best * 1e3,
           sum / 20 * 1e3, flops / (best * 1e-3) / 1e12, flops / (best * 1e-3) / 1e12 / 416.7, err);
  }
  return 0;
}
