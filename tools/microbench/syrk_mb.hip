// Ablation microbenchmark for factor.hip's grouped SYRK tiles kernel at the MLP
// bench shape (A1: 4096 x 784 + ones, G1, A2, G2).  Compares the register-staged
// and LDS-DMA ring variants (time and slab agreement).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
#include "../../bnn_kfac_amd/csrc/factor.hip"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
namespace kfac { void prof_begin(int, hipStream_t) {} void prof_end(int, hipStream_t) {} }
using namespace kfac;

typedef void (*TilesK)(FactorArgs);
float time_tiles(TilesK k, FactorArgs la, int tasks, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(tasks), dim3(NTHREADS), 0, 0, la);
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(tasks), dim3(NTHREADS), 0, 0, la);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return 1000.f * ms / reps;
}

// All-CU f32 MFMA burn (4 independent accumulators per wave, 4 waves per WG):
// achievable rate and the core clock under this load (s_memtime vs the 100 MHz
// s_memrealtime, sampled by wave 0 of block 0).
template <int NA>
__global__ __launch_bounds__(256) void mfma_burn(float* out, long long* clk, int iters) {
  floatx16 acc[4];
  for (int c = 0; c < 4; ++c)
    for (int v = 0; v < 16; ++v) acc[c][v] = 0.f;
  const float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c % NA] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c % NA], 0, 0, 0);
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int c = 0; c < 4; ++c)
    for (int v = 0; v < 16; ++v) s += acc[c][v];
  if (s == 1234.5f) out[0] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

int main(int argc, char** argv) {
  {
    float* o; long long* ck;
    (void)hipMalloc(&o, 4); (void)hipMalloc(&ck, 16);
    for (int cfg = 0; cfg < 6; ++cfg) {
      const int wgs = (cfg % 3 == 0) ? 256 : (cfg % 3 == 1) ? 512 : 1024, na = cfg < 3 ? 4 : 1;
      const int iters = 800 * 256 / wgs;
      auto k = na == 4 ? mfma_burn<4> : mfma_burn<1>;
      hipLaunchKernelGGL(k, dim3(wgs), dim3(256), 0, 0, o, ck, iters);
      hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(k, dim3(wgs), dim3(256), 0, 0, o, ck, iters);
      (void)hipEventRecord(b, 0); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      long long h[2]; (void)hipMemcpy(h, ck, 16, hipMemcpyDeviceToHost);
      const double fl = (double)wgs * 4 * iters * 4 * 32 * 32 * 2 * 2;
      printf("acc/wave %d ", na);
      printf("mfma burn %4d WGs: %7.2f us  %6.1f TF  clock %.2f GHz (wave0: %lld cyc / %lld ticks)\n", wgs,
             ms * 1e3, fl / (ms * 1e-3) / 1e12, 0.1 * (double)h[0] / (double)h[1], h[0], h[1]);
    }
  }
  const int B = 4096;
  const int dims[4][2] = {{784, 1}, {128, 0}, {128, 1}, {10, 0}};  // cols, ones
  std::vector<float*> xs(4), Fs(4);
  std::vector<kfac_factor_job> jobs(4);
  for (int i = 0; i < 4; ++i) {
    const int c = dims[i][0], n = c + dims[i][1];
    std::vector<float> h((size_t)B * c);
    for (size_t e = 0; e < h.size(); ++e) h[e] = (float)((e * 2654435761u) % 1000) / 1000.f;
    (void)hipMalloc(&xs[i], h.size() * 4);
    (void)hipMemcpy(xs[i], h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&Fs[i], (size_t)n * n * 4);
    kfac_factor_job& j = jobs[i];
    j = kfac_factor_job{};
    j.x.ptr = xs[i]; j.x.layout = KFAC_ROWMAJOR; j.x.rows = B; j.x.cols = c; j.x.ld = c;
    j.x.has_ones = dims[i][1];
    j.alpha = 1.f / B; j.beta = 0.f; j.F = Fs[i]; j.ldF = n;
  }
  size_t wsb = kfac_factor_workspace_bytes(jobs.data(), 4);
  void* ws; (void)hipMalloc(&ws, wsb);
  const double flops = 650402.0 * B;
  std::vector<int> targets = {768, 1024, 1152, 1280, 1536};
  if (argc > 1) targets = {atoi(argv[1])};
  for (int target : targets) {
    Plan plans[MAXJ];
    plan_jobs(jobs.data(), 4, plans, target);
    FactorArgs la{};
    int lt = 0; size_t off = 0;
    for (int i = 0; i < 4; ++i) {
      FactorJobDev& d = la.job[i];
      fill_dev(d, jobs[i]); d.beta = 0; d.splits = plans[i].splits; d.chunk = plans[i].chunk;
      d.slab = (float*)((char*)ws + off); off += plans[i].slab_bytes;
      d.task_begin = lt; d.tile_begin = 0; lt += plans[i].tiles * plans[i].splits; la.task_end[i] = lt;
    }
    la.njobs = 4;
    if (off > wsb) { (void)hipFree(ws); (void)hipMalloc(&ws, off); wsb = off; for (int i = 0; i < 4; ++i) {} }
    size_t o2 = 0;
    for (int i = 0; i < 4; ++i) { la.job[i].slab = (float*)((char*)ws + o2); o2 += plans[i].slab_bytes; }
    for (int i = 0; i < 4; ++i)
      la.job[i].glds = jobs[i].x.cols % 4 == 0;
    la.stagger = 5;
    struct V { const char* name; TilesK k; } vs[] = {
        {"prod (BK32 x2 sched)", kfac_factor_tiles}, {"no stagger", kfac_factor_tiles_t<32, 2, 2 + 32>},
        {"32x4 sub2", kfac_factor_tiles_t<32, 4, 2, 2>}};
    for (auto& v : vs) {
      float t0 = time_tiles(v.k, la, lt, 50);
      printf("target %5d tasks %5d | %-15s %6.2f us (%5.1f TF)\n", target, lt, v.name, t0, flops / t0 / 1e6);
    }
  }
  return 0;
}
