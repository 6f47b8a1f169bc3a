// bf16x3 SYRK with 128 x 128 tiles split once per WORKGROUP (4 waves, 2 workgroups per
// CU), the cut_mb.hip k_cuti structure at half the tile edge: each 16-row stage of the
// tile's A | B panels (256 columns) is loaded and split once into a double-buffered LDS
// image (3 bf16 parts, 24 KB per stage), the next stage's split interleaved with this
// stage's MFMAs; every wave computes a 64 x 64 quadrant (2 x 2 blocks of 32 x 32, 64
// accumulator registers) from LDS fragments.  The question: does it keep cu8i's lower
// split cost (3.7 VALU per MFMA here, 7.3 in kfac_factor_tiles_x3) within the register
// budget that leaves an inversion wave room beside two SYRK waves per SIMD (<= ~200)?
// Region: the 3 off-diagonal 256-tiles of a 768-column fp32 operand = 12 tiles of 128.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o cutq_mb cutq_mb.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef WIDE
constexpr int K = 61440, LD = 784;
#else
constexpr int K = 16384, LD = 4096;
#endif
constexpr int CT = 128;           // workgroup tile edge
constexpr int NP = 2 * CT;        // panel columns per stage (A | B)
constexpr int PART = NP * 32;     // one part of a stage: NP cols x 16 k x 2 B
constexpr int STG = 3 * PART;     // one stage buffer (24 KB)
#ifndef WIDE
constexpr int NTILE = 12;         // 128-tiles of the 256-tiles (1,0) (2,0) (2,1)
#else
constexpr int NTILE = 32 * 33 / 2;  // every lower-triangle 128-tile of 4096 columns
#endif

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
// 128-tile t: 256-tile (1,0) (2,0) (2,1) by t / 4, quadrant (t % 4) / 2, t % 2
__device__ __host__ inline void tile_cols(int t, int& ca, int& cb) {
#ifndef WIDE
  const int T = t / 4, I = T == 0 ? 1 : 2, J = T == 2 ? 1 : 0;
  ca = I * 256 + ((t % 4) / 2) * CT;
  cb = J * 256 + (t % 2) * CT;
#else
  int i = 0;
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  ca = i * CT;
  cb = (t - i * (i + 1) / 2) * CT;
#endif
}

#define SB() __builtin_amdgcn_sched_barrier(0)
// NV: VALU per MFMA slot in the interleave pattern; LZ: B fragments read lazily; VM: the
// stage-after-next loads spread one per MFMA over the first block row (else all issued
// before the first MFMA)
template <int NV, bool LZ, bool MFMA_ONLY, bool VM = false>
__global__ __launch_bounds__(256, 2) void k_cutq(const float* X, int splits, float* slab) {
  constexpr int NT = 256, U = 2, RB = 2, CB = 2;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int ca, cb;
  tile_cols(tile, ca, cb);
  const int chunk = K / splits, k0 = split * chunk, ns = chunk / 16;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;  // quadrant rows 64 wr, cols 64 wc
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), 0, K * LD * 4, 0x00020000);
  int voff[U], woff[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = u * NT + t, c = q % NP, h = q / NP;
    const int gc = c < CT ? ca + c : cb + (c - CT);
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
  const int ao = fo + (64 * wr) * 16, bo = fo + (CT + 64 * wc) * 16;
  auto frag = [&](const char* buf, int off) { return *reinterpret_cast<const bf16x8*>(buf + off); };
  load(L0, k0);
#pragma unroll
  for (int u = 0; u < U; ++u) put1(L0[u], lds, woff[u]);
  if (MFMA_ONLY)
#pragma unroll
    for (int u = 0; u < U; ++u) put1(L0[u], lds + STG, woff[u]);
  else
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
    if (!MFMA_ONLY) {
      if (!VM) load(Lload, k0 + 16 * (s + 2));  // (past the task's rows: harmless reads, never split)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM ? 0 : 8 * U) : "memory");  // Lsplit has landed
    }
    SB();
#pragma unroll
    for (int a = 0; a < RB; ++a) {
      if (VM && !MFMA_ONLY && a == 0) load(Lload, k0 + 16 * (s + 2));
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
      if (!MFMA_ONLY && s + 1 < ns) put1(Lsplit[a], nxt, woff[a]);
      if (LZ && a == 0) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      if (a + 1 < RB) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // the next A reads first
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        if (VM && !MFMA_ONLY && a == 0) {  // 16 loads over 12 MFMAs
          if (i < 4) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
          else __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (LZ && a == 0 && i == 5) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        if (i % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
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
        o[(64 * wr + a * 32 + acc_row(v, lane)) * CT + 64 * wc + b * 32 + (lane & 31)] = acc[a][b][v];
}

__global__ void k_ref(const float* X, int ca, int cb, double* out) {
  const int r = blockIdx.x, c = threadIdx.x;
  double s = 0;
  for (int k = 0; k < K; ++k) s += (double)X[(size_t)k * LD + ca + r] * (double)X[(size_t)k * LD + cb + c];
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
#ifndef WIDE
  const int splits = 40;  // 480 tasks: two workgroups per CU, one round
#else
  const int splits = 2;   // 1056 tasks
#endif
  float* slab;
  const size_t slab_bytes = (size_t)NTILE * splits * CT * CT * 4;
  CHECK(hipMalloc(&slab, slab_bytes));
  double* ref;
  CHECK(hipMalloc(&ref, CT * CT * 8));
#ifndef WIDE
  const int RT = 7;  // checked tile
#else
  const int RT = 100;
#endif
  int rca, rcb;
  tile_cols(RT, rca, rcb);
  hipLaunchKernelGGL(k_ref, dim3(CT), dim3(CT), 0, 0, X, rca, rcb, ref);
  std::vector<double> href(CT * CT);
  CHECK(hipMemcpy(href.data(), ref, CT * CT * 8, hipMemcpyDeviceToHost));
  const double flops = 2.0 * K * NTILE * CT * CT;
#define VARIANTS(X) X(4, true, false, false) X(4, true, false, true) X(2, true, false, true) X(6, true, false, true) X(4, false, false, true) X(4, true, true, false)
#define ATTR(nv, lz, mo, vm) CHECK(hipFuncSetAttribute((const void*)k_cutq<nv, lz, mo, vm>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG));
  VARIANTS(ATTR)
  std::vector<std::string> names;
#define NAME(nv, lz, mo, vm) names.push_back(std::string("q128_") + #nv + (lz ? "L" : "") + (vm ? "V" : "") + (mo ? "_m" : ""));
  VARIANTS(NAME)
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int vi = 0; vi < (int)names.size(); ++vi) {
    auto launch = [&]() {
      const int tasks = NTILE * splits;
      int vj = 0;
#define LAUNCH(nv, lz, mo, vm) if (vi == vj++) hipLaunchKernelGGL((k_cutq<nv, lz, mo, vm>), dim3(tasks), dim3(256), 2 * STG, 0, X, splits, slab);
      VARIANTS(LAUNCH)
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
    printf("%-10s best %7.1f us mean %7.1f us  %6.1f TF/s  %.3f of 417  max rel err %.2e\n", names[vi].c_str(),
           best * 1e3, sum / 20 * 1e3, flops / (best * 1e-3) / 1e12, flops / (best * 1e-3) / 1e12 / 416.7, err);
  }
  return 0;
}
