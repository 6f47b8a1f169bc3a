// Microbenchmark of the LDS-staged conv SYRK kernels at LeNet-5's shapes (batch 1024):
// conv1 A (PATCH 1x28x28, k5 p2, n 26), conv1 G (CHANNEL 6 x 784), conv2 A (PATCH
// 6x14x14, k5, n 151), conv2 G (CHANNEL 16 x 100).  Times one launch per job (median
// of 3 x 20) for the kernel variants V = 0 (per-row-group chains) and V = 1 (one
// pipeline per image), with the MFMA-bound time of the MFMAs each variant issues.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DKFAC_CONV_STAMPS -o conv_ab conv_ab.hip
#include "../../bnn_kfac_amd/csrc/factor.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
#include <cstdlib>
namespace kfac { void prof_begin(int, hipStream_t) {} void prof_end(int, hipStream_t) {} }
using namespace kfac;

template <int LAYOUT, int V>
static void launch_v(const FactorArgs& args, const ConvGeom& g, int tasks) {
  (void)V;
  launch_conv<LAYOUT>(args, g, tasks, 0);
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;  // one job (PMC passes)
  const int B = 1024;
  struct Spec { const char* name; int layout, C, H, W, k, pad, cols_ch; bool ones; };
  // CHANNEL specs: C = channels, H*W = positions
  const Spec specs[4] = {{"conv1 A", KFAC_PATCH, 1, 28, 28, 5, 2, 0, true},
                         {"conv1 G", KFAC_CHANNEL, 6, 28, 28, 0, 0, 6, false},
                         {"conv2 A", KFAC_PATCH, 6, 14, 14, 5, 0, 0, true},
                         {"conv2 G", KFAC_CHANNEL, 16, 10, 10, 0, 0, 16, false}};
  void* ws = nullptr;
  size_t wsb = 0;
  std::vector<float> ref;
  for (int si = 0; si < 4; ++si) {
    const Spec& sp = specs[si];
    if (only >= 0 && si != only) continue;
    kfac_factor_job j{};
    kfac_operand& o = j.x;
    size_t elems;
    if (sp.layout == KFAC_PATCH) {
      o.layout = KFAC_PATCH; o.C = sp.C; o.H = sp.H; o.W = sp.W; o.kh = o.kw = sp.k; o.sh = o.sw = 1;
      o.ph = o.pw = sp.pad; o.Ho = sp.H + 2 * sp.pad - sp.k + 1; o.Wo = sp.W + 2 * sp.pad - sp.k + 1;
      o.L = (int64_t)o.Ho * o.Wo; o.sB = (int64_t)sp.C * sp.H * sp.W; o.rows = (int64_t)B * o.L;
      o.cols = sp.C * sp.k * sp.k; o.has_ones = sp.ones;
      elems = (size_t)B * o.sB;
    } else {
      o.layout = KFAC_CHANNEL; o.cols = sp.C; o.L = (int64_t)sp.H * sp.W; o.sB = sp.C * o.L;
      o.rows = (int64_t)B * o.L;
      elems = (size_t)B * o.sB;
    }
    std::vector<float> h(elems);
    for (size_t e = 0; e < elems; ++e) h[e] = (float)((e * 2654435761u) % 1000) / 1000.f - 0.3f;
    float* x;
    (void)hipMalloc(&x, elems * 4);
    (void)hipMemcpy(x, h.data(), elems * 4, hipMemcpyHostToDevice);
    o.ptr = x;
    const int n = o.cols + o.has_ones;
    float* F;
    (void)hipMalloc(&F, (size_t)n * n * 4);
    j.alpha = 1.f / B; j.beta = 0.f; j.F = F; j.ldF = n;
    const size_t need = kfac_factor_workspace_bytes(&j, 1);
    if (need > wsb) { if (ws) (void)hipFree(ws); (void)hipMalloc(&ws, need); wsb = need; }
    GroupLaunch g;
    if (prepare_group(&j, 1, (char*)ws, wsb, g) != KFAC_OK) { printf("prep failed\n"); return 1; }
    ConvGeom cg;
    if (!conv_geom(j, cg)) { printf("%s: not staged\n", sp.name); continue; }
    const int nb32 = (int)cdiv(n, 32);
    // MFMAs issued per image: PATCH G row groups x T (x blocks); CHANNEL segments x Q
    double mfma = cg.mode == 0 ? (double)cg.nq * cg.G * cg.T : (double)cg.G * cg.T * (cg.mode ? 4 : 1);
    if (sp.layout == KFAC_CHANNEL) mfma = (cg.mode == 0 ? cg.nq * cg.KR : 4.0 * cg.KR) * cg.T / cg.KR * (cg.mode == 0 ? 1 : 1);
    (void)nb32;
    const double cyc = cg.mode == 2 ? 32.0 : 64.0;
    const double bound_us = mfma * B * cyc / 1024.0 / 2.4e3;
    for (int V = 0; V < 1; ++V) {
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      std::vector<float> t;
      for (int r = 0; r < 3; ++r) {
        auto go = [&]() {
          if (sp.layout == KFAC_PATCH) { if (V) launch_v<KFAC_PATCH, 1>(g.args, cg, g.tasks); else launch_v<KFAC_PATCH, 0>(g.args, cg, g.tasks); }
          else { if (V) launch_v<KFAC_CHANNEL, 1>(g.args, cg, g.tasks); else launch_v<KFAC_CHANNEL, 0>(g.args, cg, g.tasks); }
        };
        go();
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < 20; ++i) go();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        t.push_back(1000.f * ms / 20);
      }
      std::sort(t.begin(), t.end());
      // results: slab of the last launch (split partials) summed on the host for a checksum
      launch_reduce(g.red, g.rtiles, 0);
      (void)hipDeviceSynchronize();
      std::vector<float> Fh((size_t)n * n);
      (void)hipMemcpy(Fh.data(), F, Fh.size() * 4, hipMemcpyDeviceToHost);
      double cs = 0;
      for (float v : Fh) cs += v;
      printf("%-8s n %3d mode %d tasks %4d lds %5d | V%d %8.2f us  (MFMA-bound %6.2f us)  checksum %.6e\n", sp.name,
             n, cg.mode, g.tasks, cg.lds, V, t[1], bound_us, cs);
      {  // per-workgroup stamps of the last launch (the reduce ran after it)
        std::vector<unsigned long long> st(2 * 16384);
        (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_syrk_stamps), st.size() * 8);
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < g.tasks; ++b) t0 = std::min(t0, st[2 * b]);
        std::vector<double> s0, e0, d0;
        for (int b = 0; b < g.tasks; ++b) {
          s0.push_back((st[2 * b] - t0) / 100.0);
          e0.push_back((st[2 * b + 1] - t0) / 100.0);
          d0.push_back((st[2 * b + 1] - st[2 * b]) / 100.0);
        }
        auto pct = [](std::vector<double> x, double q) { std::sort(x.begin(), x.end()); return x[(size_t)(q * (x.size() - 1))]; };
        printf("    start p0 %.1f p50 %.1f p90 %.1f p100 %.1f | end p50 %.1f p100 %.1f | dur p0 %.1f p50 %.1f p100 %.1f us\n",
               pct(s0, 0), pct(s0, .5), pct(s0, .9), pct(s0, 1), pct(e0, .5), pct(e0, 1), pct(d0, 0), pct(d0, .5), pct(d0, 1));
      }
    }
  }
  return 0;
}
