// SYRK tile-size ablation at the wide MLP's shape (a 4096-column operand, 16,384 rows =
// one 4-batch launch): one workgroup (4 waves) per TSxTS lower tile and K-split,
// register-staged panels (the next 32-row stage is loaded while the current one's
// MFMAs run), one barrier pair per stage, v_mfma_f32_32x32x2f32.
//   TS =  64: wave = one 32x32 quadrant, 16 MFMAs per stage, 4 workgroups per CU
//   TS = 128: wave = one 64x64 quadrant (2x2 accumulators), 64 MFMAs per stage,
//             2 workgroups per CU, half the panel bytes per flop
// GBK: rows per stage (32: 16 MFMAs per wave per barrier pair, 64: 32, 128: 64).
// Prints time and TF/s over the computed (full-tile) flops.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o syrk_macro syrk_macro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int NT = 256;

__device__ __forceinline__ void tri_decode(int t, int& i, int& j) {
  i = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
  while (i * (i + 1) / 2 > t) --i;
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  j = t - i * (i + 1) / 2;
}

template <int TS, int GBK = 32>
__global__ __launch_bounds__(NT, TS == 64 ? 4 : 2) void k_syrk(const float* X, int N, int K, int splits,
                                                                float* slab) {
  constexpr int PER = 2 * GBK * TS / NT / 4;  // float4 loads per thread per stage
  constexpr int QS = TS / 2;                  // quadrant edge per wave
  constexpr int NA = QS / 32;                 // 32-blocks per quadrant edge
  __shared__ __attribute__((aligned(16))) float lds[2 * GBK * TS];
  const int task = blockIdx.x, tile = task / splits, split = task % splits;
  int ti, tj;
  tri_decode(tile, ti, tj);
  const int kc = K / splits / GBK * GBK, k0 = split * kc;  // (whole stages; a ragged tail is dropped)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wi = w >> 1, wj = w & 1;
  const int rr = lane & 31, h = lane >> 5;
  floatx16 acc[NA][NA];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NA; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  // thread's float4 e of a stage: panel p = e / (GBK*TS/4), row, col4
  f4 v[PER];
#define FETCH(K_)                                                                  \
  _Pragma("unroll") for (int q = 0; q < PER; ++q) {                                \
    const int e = q * NT + threadIdx.x;                                            \
    const int p = e / (GBK * TS / 4), r = (e / (TS / 4)) % GBK, c4 = e % (TS / 4); \
    const int col = (p ? tj : ti) * TS + 4 * c4;                                   \
    v[q] = *(const f4*)(X + (size_t)((K_) + r) * N + col);                     \
  }
  FETCH(k0);
  for (int k = k0; k < k0 + kc; k += GBK) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) *(f4*)(lds + 4 * (q * NT + threadIdx.x)) = v[q];
    __syncthreads();
    { const int kn = min(k + GBK, k0 + kc - GBK); FETCH(kn); }  // (last stage: a harmless reload)
    const float* A = lds;
    const float* B = lds + GBK * TS;
#pragma unroll
    for (int s2 = 0; s2 < GBK / 2; ++s2) {
      float av[NA], bv[NA];
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        av[a] = A[(2 * s2 + h) * TS + wi * QS + 32 * a + rr];
        bv[a] = B[(2 * s2 + h) * TS + wj * QS + 32 * a + rr];
      }
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int b = 0; b < NA; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }
  float* out = slab + (size_t)task * TS * TS;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NA; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wi * QS + 32 * a + (r / 4) * 8 + h * 4 + (r % 4), col = wj * QS + 32 * b + rr;
        out[row * TS + col] = acc[a][b][r];
      }
}

template <int TS, int GBK = 32>
static void run(const float* X, float* slab, int N, int K, int splits) {
  const int T = N / TS, tiles = T * (T + 1) / 2, tasks = tiles * splits;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<float> t;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_syrk<TS, GBK>), dim3(tasks), dim3(NT), 0, 0, X, N, K, splits, slab);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double Kr = (double)(K / splits / GBK * GBK) * splits;  // rows actually run
  const double flop = 2.0 * TS * TS * Kr * tiles;
  const double alg = (double)N * (N + 1) * Kr;
  printf("GBK %d TS %3d splits %2d tasks %5d  %8.3f ms  %7.2f TF/s computed, %7.2f TF/s algorithmic\n", GBK, TS, splits, tasks,
         t[2], flop / (t[2] * 1e-3) / 1e12, alg / (t[2] * 1e-3) / 1e12);
  (void)GBK;
}

int main(int argc, char** argv) {
  // default: the wide shape; "mlp": the MLP's A1 factor at an 8-batch launch (832 =
  // 13 tiles of 64, 32,768 rows)
  const bool mlp = argc > 1;
  const int N = mlp ? 832 : 4096, K = mlp ? 32768 : 16384;
  float *X, *slab;
  (void)hipMalloc(&X, (size_t)N * K * sizeof(float));
  (void)hipMalloc(&slab, (size_t)2080 * 4 * 64 * 64 * sizeof(float));  // >= tiles * splits * 64^2
  std::vector<float> h((size_t)N * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3f * (float)(i % 1013);
  (void)hipMemcpy(X, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
  if (mlp) {
    run<64>(X, slab, N, K, 8);
    run<64>(X, slab, N, K, 11);
    run<64, 64>(X, slab, N, K, 8);
    run<64, 64>(X, slab, N, K, 11);
    run<64, 128>(X, slab, N, K, 11);
  } else {
    run<64>(X, slab, N, K, 1);
    run<64>(X, slab, N, K, 2);
    run<64, 64>(X, slab, N, K, 1);
    run<64, 64>(X, slab, N, K, 2);
    run<128>(X, slab, N, K, 1);
    run<128>(X, slab, N, K, 2);
  }
  (void)hipDeviceSynchronize();
  return 0;
}
