// fp64 MFMA ceiling of the inversion's 64x64 tile product (inv_bulk's inner step).
// Every workgroup (256 threads, 4 waves) keeps a tile pair resident in LDS and runs
// R steps of acc += A * B^T (64x64x64, 524,288 flop), each step bracketed by the two
// barriers and the 16-double-per-thread LDS commit of the real K loop. Variants:
//   reg   4 independent MFMA chains in registers (the instruction's ceiling)
//   row   wave w owns block row w, block-major (acc[x] chain of 16 MFMAs, then x+1)
//         = invert_tiles.inc's mfma_block loop
//   rowi  block row w, k-major: per k0 one A fragment, 4 B fragments, 4 MFMAs
//   quad  wave w owns a 2x2 block square, k-major: 2 A + 2 B fragments per 4 MFMAs
//   rowR / regR: row / reg with random full-mantissa operands (power-limited clock)
//   glob / pipe / g128: the inv_bulk shape with global tiles (see k_glob, k_pipe, k_glob128)
// plus the pure-register issue ceilings (no LDS, no barriers) of the f64 16x16x4 and
// the f32 32x32x2 / 16x16x4 MFMAs with 1 or 4 independent accumulator chains per wave.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o f64_mb f64_mb.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef double doublex4 __attribute__((ext_vector_type(4)));
constexpr int NB = 64, DP = NB + 2, NT = 256, PER = NB * NB / NT;

__device__ __forceinline__ doublex4 mf(double a, double b, doublex4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int MODE, bool RND = false>
__global__ __launch_bounds__(NT) void k_tile(const double* g, double* out, int R) {
  __shared__ __attribute__((aligned(16))) double A[NB * DP];
  __shared__ __attribute__((aligned(16))) double B[NB * DP];
  const int c = threadIdx.x % NB, r0 = threadIdx.x / NB;
  double va[PER], vb[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    va[q] = g[(r0 + 4 * q) * NB + c];
    vb[q] = g[NB * NB + (r0 + 4 * q) * NB + c];
    if (RND) {  // full-entropy operands (random mantissas, both signs): the power draw of real data
      uint64_t x = 0x9E3779B97F4A7C15ull * (blockIdx.x * NT + threadIdx.x + 1) + q;
      x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
      va[q] = (double)(int64_t)x * 0x1p-63;
      x *= 0x94D049BB133111EBull; x ^= x >> 31;
      vb[q] = (double)(int64_t)x * 0x1p-63;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, kk = lane >> 4;
  doublex4 acc[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) acc[x] = doublex4{0, 0, 0, 0};
  for (int s = 0; s < R; ++s) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      A[(r0 + 4 * q) * DP + c] = va[q];
      B[(r0 + 4 * q) * DP + c] = vb[q];
    }
    __syncthreads();
    if (MODE == 0) {
      const double a = va[s & 15], b = vb[s & 15];
#pragma unroll
      for (int k0 = 0; k0 < 16; ++k0)
#pragma unroll
        for (int x = 0; x < 4; ++x) acc[x] = mf(a, b + k0, acc[x]);
    } else if (MODE == 1) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int k0 = 0; k0 < NB; k0 += 4)
          acc[x] = mf(A[(16 * w + i) * DP + k0 + kk], B[(16 * x + i) * DP + k0 + kk], acc[x]);
    } else if (MODE == 2) {
#pragma unroll
      for (int k0 = 0; k0 < NB; k0 += 4) {
        const double a = A[(16 * w + i) * DP + k0 + kk];
#pragma unroll
        for (int x = 0; x < 4; ++x) acc[x] = mf(a, B[(16 * x + i) * DP + k0 + kk], acc[x]);
      }
    } else {
      const int br = 2 * (w >> 1), bc = 2 * (w & 1);
#pragma unroll
      for (int k0 = 0; k0 < NB; k0 += 4) {
        const double a0 = A[(16 * br + i) * DP + k0 + kk], a1 = A[(16 * br + 16 + i) * DP + k0 + kk];
        const double b0 = B[(16 * bc + i) * DP + k0 + kk], b1 = B[(16 * bc + 16 + i) * DP + k0 + kk];
        acc[0] = mf(a0, b0, acc[0]);
        acc[1] = mf(a0, b1, acc[1]);
        acc[2] = mf(a1, b0, acc[2]);
        acc[3] = mf(a1, b1, acc[3]);
      }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (RND) { const double t = va[q]; va[q] = vb[q] * 0.999; vb[q] = -t; } else { va[q] += 1e-300; vb[q] -= 1e-300; }
    }
  }
  double s = 0;
#pragma unroll
  for (int x = 0; x < 4; ++x) s += acc[x][0] + acc[x][1] + acc[x][2] + acc[x][3];
  out[blockIdx.x * NT + threadIdx.x] = s;
}

// inv_bulk's shape: each workgroup owns one 64x64 output tile (i, j) of a T x T tile
// matrix (pitch Np doubles) and runs S steps acc += W[i][k] W[j][k]^T, k = k0.., tiles
// loaded global -> registers -> LDS per step (unpipelined, as blk_trailing), then
// out = old - acc.  Grid: 8192 workgroups (16 rounds of 512 slots) cycling over the
// lower triangle of rows/cols >= S (timing only: repeated tiles race on their output).
template <bool WIDE>
__global__ __launch_bounds__(NT) void k_glob(double* W, int Np, int S, int m, int tmod) {
  __shared__ __attribute__((aligned(16))) double A[NB * DP];
  __shared__ __attribute__((aligned(16))) double B[NB * DP];
  const int tb = blockIdx.x % (m * (m + 1) / 2);  // grid may exceed the triangle (timing)
  int a = (int)((sqrtf(8.f * tb + 1.f) - 1.f) * 0.5f);
  while ((a + 1) * (a + 2) / 2 <= tb) ++a;
  while (a * (a + 1) / 2 > tb) --a;
  int b = tb - a * (a + 1) / 2, i = S + a, j = S + b;
  if (tmod) { i %= tmod; j %= tmod; }  // small working set (timing only: tiles alias)
  const int c = threadIdx.x % NB, r0 = threadIdx.x / NB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, kk = lane >> 4;
  doublex4 acc[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) acc[x] = doublex4{0, 0, 0, 0};
  for (int k = 0; k < S; ++k) {
    const double* ga = W + (size_t)(i * NB) * Np + k * NB;
    const double* gb = W + (size_t)(j * NB) * Np + k * NB;
    if (WIDE) {  // 16-byte loads: thread = (row r2 = tid / 32, column pair c2 = tid % 32)
      typedef double d2 __attribute__((ext_vector_type(2)));
      const int c2 = threadIdx.x % 32, q0 = threadIdx.x / 32;
      d2 va[PER / 2], vb[PER / 2];
#pragma unroll
      for (int q = 0; q < PER / 2; ++q) {
        va[q] = *(const d2*)(ga + (size_t)(q0 + 8 * q) * Np + 2 * c2);
        vb[q] = *(const d2*)(gb + (size_t)(q0 + 8 * q) * Np + 2 * c2);
      }
#pragma unroll
      for (int q = 0; q < PER / 2; ++q) {
        *(d2*)(A + (q0 + 8 * q) * DP + 2 * c2) = va[q];
        *(d2*)(B + (q0 + 8 * q) * DP + 2 * c2) = vb[q];
      }
    } else {
    double va[PER], vb[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      va[q] = ga[(size_t)(r0 + 4 * q) * Np + c];
      vb[q] = gb[(size_t)(r0 + 4 * q) * Np + c];
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      A[(r0 + 4 * q) * DP + c] = va[q];
      B[(r0 + 4 * q) * DP + c] = vb[q];
    }
    }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int k0 = 0; k0 < NB; k0 += 4)
        acc[x] = mf(A[(16 * w + li) * DP + k0 + kk], B[(16 * x + li) * DP + k0 + kk], acc[x]);
    __syncthreads();
  }
  double* out = W + (size_t)(i * NB) * Np + j * NB;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      double* p = out + (size_t)(16 * w + (lane >> 4) + 4 * v) * Np + 16 * x + (lane & 15);
      *p = *p - acc[x][v];
    }
}

template <bool WIDE = false>
static void run_glob(double* W, int T, int S, int tmod = 0);

// k_glob, pipelined: step k+1's tiles are loaded into registers right after the
// barrier that publishes step k, so the loads fly during step k's MFMAs.  RAWB: raw
// s_barrier + explicit lgkmcnt(0) instead of __syncthreads() (whose workgroup-scope
// fences also wait for the in-flight global loads).
template <bool RAWB>
__global__ __launch_bounds__(NT) void k_pipe(double* W, int Np, int S, int m) {
  __shared__ __attribute__((aligned(16))) double A[NB * DP];
  __shared__ __attribute__((aligned(16))) double B[NB * DP];
  const int tb = blockIdx.x % (m * (m + 1) / 2);  // grid may exceed the triangle (timing)
  int a = (int)((sqrtf(8.f * tb + 1.f) - 1.f) * 0.5f);
  while ((a + 1) * (a + 2) / 2 <= tb) ++a;
  while (a * (a + 1) / 2 > tb) --a;
  const int b = tb - a * (a + 1) / 2, i = S + a, j = S + b;
  const int c = threadIdx.x % NB, r0 = threadIdx.x / NB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, kk = lane >> 4;
  doublex4 acc[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) acc[x] = doublex4{0, 0, 0, 0};
  const double* ga = W + (size_t)(i * NB) * Np;
  const double* gb = W + (size_t)(j * NB) * Np;
  double va[PER], vb[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    va[q] = ga[(size_t)(r0 + 4 * q) * Np + c];
    vb[q] = gb[(size_t)(r0 + 4 * q) * Np + c];
  }
  for (int k = 0; k < S; ++k) {
    if (RAWB) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); } else __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      A[(r0 + 4 * q) * DP + c] = va[q];
      B[(r0 + 4 * q) * DP + c] = vb[q];
    }
    if (RAWB) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); } else __syncthreads();
    const int kn = min(k + 1, S - 1);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      va[q] = ga[(size_t)(r0 + 4 * q) * Np + kn * NB + c];
      vb[q] = gb[(size_t)(r0 + 4 * q) * Np + kn * NB + c];
    }
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int k0 = 0; k0 < NB; k0 += 4)
        acc[x] = mf(A[(16 * w + li) * DP + k0 + kk], B[(16 * x + li) * DP + k0 + kk], acc[x]);
  }
  double* out = W + (size_t)(i * NB) * Np + j * NB;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      double* p = out + (size_t)(16 * w + (lane >> 4) + 4 * v) * Np + 16 * x + (lane & 15);
      *p = *p - acc[x][v];
    }
}

template <bool RAWB>
static void run_pipe(double* W, int T, int S) {
  const int Np = T * NB, m = T - S, grid = 8192;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<float> t;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_pipe<RAWB>, dim3(grid), dim3(NT), 0, 0, W, Np, S, m);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double flop = 2.0 * NB * NB * NB * (double)S * grid;
  printf("pipe%s T %d S %2d grid %5d  %8.3f ms  %6.2f TF/s fp64\n", RAWB ? "R" : " ", T, S, grid, t[2],
         flop / (t[2] * 1e-3) / 1e12);
}

template <bool WIDE>
static void run_glob(double* W, int T, int S, int tmod) {
  const int Np = T * NB, m = T - S, grid = 8192;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<float> t;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_glob<WIDE>, dim3(grid), dim3(NT), 0, 0, W, Np, S, m, tmod);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double flop = 2.0 * NB * NB * NB * (double)S * grid;
  printf("glob%s T %d S %2d mod %2d grid %5d  %8.3f ms  %6.2f TF/s fp64\n", WIDE ? "W" : " ", T, S, tmod, grid, t[2],
         flop / (t[2] * 1e-3) / 1e12);
}

// 128 x 128 output per workgroup (4 waves, each a 64 x 64 quadrant = 4 x 4 blocks of
// 16 x 16, 16 accumulators), one 128 x 64 A and B panel pair in LDS per 64-wide step
// (135 KB: 1 workgroup per CU), tiles loaded global -> registers -> LDS.  Grid cycles
// over the lower triangle of 128-tiles of rows/cols >= S.
constexpr int MB = 128;
__global__ __launch_bounds__(NT, 1) void k_glob128(double* W, int Np, int S, int m) {
  extern __shared__ double sh[];
  double* A = sh;
  double* B = sh + MB * DP;
  const int tb = blockIdx.x % (m * (m + 1) / 2);
  int a = (int)((sqrtf(8.f * tb + 1.f) - 1.f) * 0.5f);
  while ((a + 1) * (a + 2) / 2 <= tb) ++a;
  while (a * (a + 1) / 2 > tb) --a;
  const int b = tb - a * (a + 1) / 2;
  const size_t i0 = (size_t)S * NB + (size_t)a * MB, j0 = (size_t)S * NB + (size_t)b * MB;
  const int c = threadIdx.x % NB, r0 = threadIdx.x / NB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, kk = lane >> 4;
  const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
  doublex4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = doublex4{0, 0, 0, 0};
  for (int k = 0; k < S; ++k) {
    const double* ga = W + i0 * Np + k * NB;
    const double* gb = W + j0 * Np + k * NB;
#pragma unroll
    for (int q = 0; q < MB / 4; ++q) {  // 32 rows per pass of 4: 32 loads each
      A[(r0 + 4 * q) * DP + c] = ga[(size_t)(r0 + 4 * q) * Np + c];
      B[(r0 + 4 * q) * DP + c] = gb[(size_t)(r0 + 4 * q) * Np + c];
    }
    __syncthreads();
#pragma unroll 4
    for (int k0 = 0; k0 < NB; k0 += 4) {
      double av[4], bv[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        av[x] = A[(wr + 16 * x + li) * DP + k0 + kk];
        bv[x] = B[(wc + 16 * x + li) * DP + k0 + kk];
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = mf(av[x], bv[y], acc[x][y]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        double* p = W + (i0 + wr + 16 * x + (lane >> 4) + 4 * v) * Np + j0 + wc + 16 * y + (lane & 15);
        *p = *p - acc[x][y][v];
      }
}

static void run_glob128(double* W, int T, int S) {
  const int Np = T * NB, m = (T - S) * NB / MB, grid = 2048;
  const int shmem = 2 * MB * DP * sizeof(double);
  (void)hipFuncSetAttribute((const void*)k_glob128, hipFuncAttributeMaxDynamicSharedMemorySize, shmem);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<float> t;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_glob128, dim3(grid), dim3(NT), shmem, 0, W, Np, S, m);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double flop = 2.0 * MB * MB * NB * (double)S * grid;
  printf("g128  T %d S %2d grid %5d  %8.3f ms  %6.2f TF/s fp64\n", T, S, grid, t[2], flop / (t[2] * 1e-3) / 1e12);
}

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
// KIND 0: f64 16x16x4, 1: f32 32x32x2, 2: f32 16x16x4; CH independent chains; R x 16 MFMAs each
template <int KIND, int CH>
__global__ __launch_bounds__(NT) void k_reg(double* out, int R) {
  const float a = 1e-3f * (threadIdx.x & 7), b = 1e-3f * (threadIdx.x >> 5);
  double s = 0;
  if (KIND == 0) {
    doublex4 acc[CH];
    for (int x = 0; x < CH; ++x) acc[x] = doublex4{0, 0, 0, 0};
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int x = 0; x < CH; ++x) acc[x] = mf(a, b + x, acc[x]);
    for (int x = 0; x < CH; ++x) s += acc[x][0] + acc[x][3];
  } else if (KIND == 1) {
    floatx16 acc[CH];
    for (int x = 0; x < CH; ++x) for (int e = 0; e < 16; ++e) acc[x][e] = 0.f;
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int x = 0; x < CH; ++x) acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b + x, acc[x], 0, 0, 0);
    for (int x = 0; x < CH; ++x) s += acc[x][0] + acc[x][15];
  } else {
    floatx4 acc[CH];
    for (int x = 0; x < CH; ++x) for (int e = 0; e < 4; ++e) acc[x][e] = 0.f;
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int x = 0; x < CH; ++x) acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b + x, acc[x], 0, 0, 0);
    for (int x = 0; x < CH; ++x) s += acc[x][0] + acc[x][3];
  }
  out[blockIdx.x * NT + threadIdx.x] = s;
}

template <int KIND, int CH>
static void run_reg(const char* name, double* out, int grid, int R, double flop_per) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<float> t;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_reg<KIND, CH>), dim3(grid), dim3(NT), 0, 0, out, R);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double flop = flop_per * 16.0 * CH * R * (grid * NT / 64);
  printf("%-10s chains %d grid %5d  %8.3f ms  %7.2f TF/s\n", name, CH, grid, t[2], flop / (t[2] * 1e-3) / 1e12);
}

template <int MODE, bool RND = false>
static void run(const char* name, const double* g, double* out, int grid, int R) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<float> t;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_tile<MODE, RND>), dim3(grid), dim3(NT), 0, 0, g, out, R);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double flop = 2.0 * NB * NB * NB * (double)R * grid;
  printf("%-5s grid %5d R %4d  %8.3f ms  %6.2f TF/s fp64\n", name, grid, R, t[2], flop / (t[2] * 1e-3) / 1e12);
}

int main() {
  double *g, *out;
  const int grid = 2048, R = 200;
  (void)hipMalloc(&g, 2 * NB * NB * sizeof(double));
  (void)hipMalloc(&out, (size_t)grid * NT * sizeof(double));
  std::vector<double> h(2 * NB * NB);
  for (size_t k = 0; k < h.size(); ++k) h[k] = 1e-3 * (double)(k % 97);
  (void)hipMemcpy(g, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice);
  run<0>("reg", g, out, grid, R);
  run<1>("row", g, out, grid, R);
  run<2>("rowi", g, out, grid, R);
  run<3>("quad", g, out, grid, R);
  run<1>("row", g, out, 512, R);
  run<1, true>("rowR", g, out, grid, R);
  run<1, true>("rowR", g, out, grid, 4 * R);
  run<0, true>("regR", g, out, grid, R);
  run<3>("quad", g, out, 512, R);
  {
    const int T = 64;
    double* W;
    (void)hipMalloc(&W, (size_t)T * NB * T * NB * sizeof(double));
    (void)hipMemset(W, 0, (size_t)T * NB * T * NB * sizeof(double));
    run_glob(W, T, 4);
    run_glob(W, T, 8);
    run_glob(W, T, 16);
    run_glob(W, T, 8, 12);  // tiles mod 12: a 4.7 MB working set
    run_glob128(W, T, 4);
    run_glob128(W, T, 8);
    run_glob128(W, T, 16);
    run_pipe<false>(W, T, 4);
    run_pipe<false>(W, T, 8);
    run_pipe<false>(W, T, 16);
    run_pipe<true>(W, T, 4);
    run_pipe<true>(W, T, 8);
    run_pipe<true>(W, T, 16);
    (void)hipFree(W);
  }
  run_reg<0, 1>("f64_16x4", out, grid, 100, 2048);
  run_reg<0, 4>("f64_16x4", out, grid, 25, 2048);
  run_reg<1, 1>("f32_32x2", out, grid, 100, 4096);
  run_reg<1, 4>("f32_32x2", out, grid, 25, 4096);
  run_reg<2, 1>("f32_16x4", out, grid, 100, 2048);
  run_reg<2, 4>("f32_16x4", out, grid, 25, 2048);
  (void)hipDeviceSynchronize();
  return 0;
}
