// Ablation microbenchmark for invert.hip's diagonal-tile factorisation.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 diag_mb.hip -o diag_mb
// Each kernel runs one 256-thread block that repeats a phase `reps` times on an
// SPD 64x64 tile in LDS; time per rep = event time / reps.
#include "../../bnn_kfac_amd/csrc/invert.hip"
namespace kfac { void prof_begin(int, hipStream_t) {} void prof_end(int, hipStream_t) {} }
#include <cstdio>
#include <vector>

using namespace kfac;
using namespace kfac::t64;

template <int MODE>
__global__ __launch_bounds__(256) void mb(const double* src, double* dst, int reps) {
  __shared__ __attribute__((aligned(16))) double S[NB * DP];
  __shared__ __attribute__((aligned(16))) double Y[NB * DP];
  __shared__ double dg[NB + 352];
  for (int it = 0; it < reps; ++it) {
    load_tile(S, src, NB);
    __syncthreads();
    if (MODE == 0) diag_factor(S, Y, dg);
    if (MODE == 3) diag_factor<1>(S, Y, dg);
    if (MODE == 4) diag_factor<6>(S, Y, dg);
    if (MODE == 5) diag_factor<0>(S, Y, dg);
    if (MODE == 1) {  // load + barrier only
      for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) Y[(e >> 6) * DP + (e & 63)] = S[(e >> 6) * DP + (e & 63)];
    }
    if (MODE == 2 || MODE == 6) {  // 64x64x64 MFMA gemm only (6: B not transposed)
      doublex4 acc[4];
      if (MODE == 2) gemm64<true>(S, S, acc);
      else gemm64<false>(S, S, acc);
      const int w = threadIdx.x >> 6, col = threadIdx.x & 15;
      for (int b4 = 0; b4 < 4; ++b4)
        for (int v = 0; v < 4; ++v) Y[(16 * w + acc_row64(v)) * DP + 16 * b4 + col] = acc[b4][v];
    }
    __syncthreads();
  }
  store_tile(dst, Y, NB);
}

template <int MODE>
float run(const double* s, double* d, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL(mb<MODE>, dim3(1), dim3(256), 0, 0, s, d, 2);
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL(mb<MODE>, dim3(1), dim3(256), 0, 0, s, d, reps);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return 1000.f * ms / reps;
}

extern "C" int mb_invert_check(int n);
int main() {
  mb_invert_check(63);
  mb_invert_check(130);
  std::vector<double> h(NB * NB);
  // random Gram matrix X^T X / m + 1e-3 I (condition ~1e5, like the MLP's A factor)
  std::vector<double> Xr(96 * NB);
  unsigned st = 12345;
  for (auto& v : Xr) { st = st * 1664525u + 1013904223u; v = (st >> 8) / 16777216.0; }
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      double acc = 0;
      for (int m = 0; m < 96; ++m) acc += Xr[m * NB + i] * Xr[m * NB + j];
      h[i * NB + j] = acc / 96 + (i == j ? 1e-3 : 0.0);
    }
  double *s, *d;
  (void)hipMalloc(&s, sizeof(double) * NB * NB);
  (void)hipMalloc(&d, sizeof(double) * NB * NB);
  (void)hipMemcpy(s, h.data(), sizeof(double) * NB * NB, hipMemcpyHostToDevice);
  const int reps = 200;
  printf("load+copy      %8.2f us/rep\n", run<1>(s, d, reps));
  printf("gemm64 f64     %8.2f us/rep\n", run<2>(s, d, reps));
  printf("gemm64 f64 nn  %8.2f us/rep\n", run<6>(s, d, reps));
  printf("diag elim only %8.2f us/rep\n", run<3>(s, d, reps));
  printf("diag mfma only %8.2f us/rep\n", run<4>(s, d, reps));
  printf("diag skeleton  %8.2f us/rep\n", run<5>(s, d, reps));
  printf("diag_factor    %8.2f us/rep\n", run<0>(s, d, reps));
  // correctness: Y * chol(S) == I  ->  check (Y S Y^T) == I
  std::vector<double> y(NB * NB);
  (void)hipMemcpy(y.data(), d, sizeof(double) * NB * NB, hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      double acc = 0;
      for (int k = 0; k < NB; ++k)
        for (int l = 0; l < NB; ++l) acc += y[i * NB + k] * h[k * NB + l] * y[j * NB + l];
      err = std::max(err, std::abs(acc - (i == j)));
    }
  printf("max |Y S Y^T - I| = %.3e\n", err);
  return 0;
}

// ---- end-to-end check through the C entry point (debug aid)
extern "C" int mb_invert_check(int n) {
  std::vector<float> F(n * n);
  std::vector<double> X(n * 40);
  unsigned st = 777;
  for (auto& v : X) { st = st * 1664525u + 1013904223u; v = (st >> 8) / 16777216.0 - 0.5; }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double acc = 0;
      for (int m = 0; m < 40; ++m) acc += X[i * 40 + m] * X[j * 40 + m];
      F[i * n + j] = (float)acc;
    }
  float *dF, *dL; int* dinfo; void* ws;
  kfac_invert_job job{};
  job.n = n; job.ldF = n; job.ldo = n; job.scale = 14.142135623730951; job.shift = 0.2; job.out_kind = 0;
  size_t wsb = kfac_invert_workspace_bytes(&job, 1);
  (void)hipMalloc(&dF, 4 * n * n); (void)hipMalloc(&dL, 4 * n * n); (void)hipMalloc(&dinfo, 4);
  (void)hipMalloc(&ws, wsb);
  (void)hipMemcpy(dF, F.data(), 4 * n * n, hipMemcpyHostToDevice);
  job.F = dF; job.out = dL;
  int rc = kfac_invert(&job, 1, ws, wsb, dinfo, nullptr);
  (void)hipDeviceSynchronize();
  int info; (void)hipMemcpy(&info, dinfo, 4, hipMemcpyDeviceToHost);
  std::vector<float> L(n * n);
  (void)hipMemcpy(L.data(), dL, 4 * n * n, hipMemcpyDeviceToHost);
  // L^T R L == I
  double err = 0;
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      double acc = 0;
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          const double R = job.scale * F[i * n + j] + (i == j ? job.shift : 0.0);
          acc += L[i * n + a] * R * L[j * n + b];
        }
      err = std::max(err, std::abs(acc - (a == b)));
    }
  printf("kfac_invert n=%d rc=%d info=%d  max|L^T R L - I|=%.3e\n", n, rc, info, err);
  return info;
}
