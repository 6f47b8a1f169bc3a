// Ablation microbenchmark for factor.hip's grouped SYRK tiles kernel at the MLP
// bench shape (A1: 4096 x 784 + ones, G1, A2, G2).  Compares the register-staged
// and LDS-DMA ring variants (time and slab agreement).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
#include "../../bnn_kfac_amd/csrc/factor.hip"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
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

int main(int argc, char** argv) {
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
      d.x = to_dev(jobs[i].x); d.alpha = jobs[i].alpha; d.beta = 0; d.F = jobs[i].F; d.ldF = jobs[i].ldF;
      d.n = factor_n(jobs[i]); d.t = (int)cdiv(d.n, TILE); d.splits = plans[i].splits; d.chunk = plans[i].chunk;
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
        {"prod (BK32 x2 sched)", kfac_factor_tiles}, {"no sched", kfac_factor_tiles_t<32, 2, 0>},
        {"setprio", kfac_factor_tiles_t<32, 2, 1>}, {"no stagger", kfac_factor_tiles_t<32, 2, 2 + 32>},
        {"16x5 sub2", kfac_factor_tiles_t<16, 5, 2, 2>}, {"32x3", kfac_factor_tiles_t<32, 3, 2>},
        {"no DMA", kfac_factor_tiles_t<32, 2, 2 + 4>}, {"no MFMA", kfac_factor_tiles_t<32, 2, 8>},
        {"no DMA, no LDS reads", kfac_factor_tiles_t<32, 2, 4 + 16>}};
    for (auto& v : vs) {
      float t0 = time_tiles(v.k, la, lt, 50);
      printf("target %5d tasks %5d | %-15s %6.2f us (%5.1f TF)\n", target, lt, v.name, t0, flops / t0 / 1e6);
    }
  }
  return 0;
}
