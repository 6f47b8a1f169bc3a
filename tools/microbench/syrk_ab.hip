// Ablation microbenchmark of the grouped SYRK tiles launch at the MLP bench's
// job set (A1 4096k x 784 + ones, G1 x 128, A2 x 128 + ones, G2 x 10) as multi-batch
// jobs of nb batches of 4096 rows (the queued launches of a KFAC pass: 1, 2, 4, 8).
// Prints the tiles-launch time per variant (median of 3 x 20 launches), its TF/s on
// the algorithmic 650,402 flop/img, and the A1-only job.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o syrk_ab syrk_ab.hip
#include "../../bnn_kfac_amd/csrc/factor.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <map>
namespace kfac { void prof_begin(int, hipStream_t) {} void prof_end(int, hipStream_t) {} }
using namespace kfac;

typedef void (*TilesK)(FactorArgs);

static float time_k(TilesK k, const FactorArgs& a, int tasks, int reps = 20) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<float> t;
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k, dim3(tasks), dim3(NTHREADS), 0, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(tasks), dim3(NTHREADS), 0, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    t.push_back(1000.f * ms / reps);
  }
  std::sort(t.begin(), t.end());
  return t[1];
}

int main(int argc, char** argv) {
  const int B = 4096;
  const int dims[4][2] = {{784, 1}, {128, 0}, {128, 1}, {10, 0}};  // cols, ones
  const int maxnb = 15;
  std::vector<float*> xs(4), Fs(4);
  std::vector<std::vector<const float*>> bases(4);
  for (int i = 0; i < 4; ++i) {
    const int c = dims[i][0], n = c + dims[i][1];
    std::vector<float> h((size_t)B * maxnb * c);
    for (size_t e = 0; e < h.size(); ++e) h[e] = (float)((e * 2654435761u) % 1000) / 1000.f;
    (void)hipMalloc(&xs[i], h.size() * 4);
    (void)hipMemcpy(xs[i], h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&Fs[i], (size_t)n * n * 4);
    for (int b = 0; b < maxnb; ++b) bases[i].push_back(xs[i] + (size_t)b * B * c);
  }
  void* ws = nullptr;
  size_t wsb = 0;
  std::vector<int> nbs = {1, 8, 15};
  int only = -1;  // argv: [nb] [t64-variant index]: one configuration (for PMC passes)
  if (argc > 1) nbs = {atoi(argv[1])};
  if (argc > 2) only = atoi(argv[2]);
  for (int nb : nbs) {
    for (int only_a1 = 0; only_a1 < 2; ++only_a1) {
      std::vector<kfac_factor_job> jobs;
      for (int i = 0; i < (only_a1 ? 1 : 4); ++i) {
        kfac_factor_job j{};
        j.x.ptr = xs[i]; j.x.layout = KFAC_ROWMAJOR; j.x.rows = B; j.x.cols = dims[i][0];
        j.x.ld = dims[i][0]; j.x.has_ones = dims[i][1];
        j.alpha = 1.f / B; j.beta = 0.f; j.F = Fs[i]; j.ldF = dims[i][0] + dims[i][1];
        if (nb > 1) { j.seg_ptrs = bases[i].data(); j.nseg = nb; }
        jobs.push_back(j);
      }
      const double flops = (only_a1 ? 785.0 * 786 : 650402.0) * B * nb;
      {
        const size_t need = kfac_factor_workspace_bytes(jobs.data(), (int)jobs.size());
        if (need > wsb) { if (ws) (void)hipFree(ws); (void)hipMalloc(&ws, need); wsb = need; }
        GroupLaunch g;
        if (prepare_group(jobs.data(), (int)jobs.size(), (char*)ws, wsb, g) != KFAC_OK) { printf("prep failed\n"); return 1; }
        struct V { const char* name; TilesK k; };
        std::vector<V> vs = {{"t64", kfac_factor_tiles_t<32, 2, 2 | 256>},
                             {"t64 noDMA", kfac_factor_tiles_t<32, 2, 2 | 256 | 4>},
                             {"t64 regops", kfac_factor_tiles_t<32, 2, 2 | 256 | 16>},
                             {"t64 noDMA+regops", kfac_factor_tiles_t<32, 2, 2 | 256 | 20>},
                             {"t64 noloop", kfac_factor_tiles_t<32, 2, 2 | 256 | 64>},
                             {"t64 stamps", kfac_factor_tiles_t<32, 2, 2 | 256 | 512>}};
        if (only >= 0 && only_a1) continue;
        int vi = -1;
        for (auto& v : vs) {
          if (only >= 0 && ++vi != only) continue;
          const float us = time_k(v.k, g.args, g.tasks);
          printf("nb %d %-4s tasks %4d | %-20s %8.2f us  %6.1f TF\n", nb, only_a1 ? "A1" : "MLP", g.tasks, v.name,
                 us, flops / us / 1e6);
          if (v.k == kfac_factor_tiles_t<32, 2, 2 | 256 | 512> && g.tasks <= 16384) {
            // the last timed launch's per-workgroup stamps (100 MHz): when workgroups
            // start / end relative to the first start, and how long each one runs
            std::vector<unsigned long long> st(2 * 16384);
            (void)hipDeviceSynchronize();
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
            printf("    start us p0 %.1f p50 %.1f p100 %.1f | end p10 %.1f p50 %.1f p90 %.1f p100 %.1f | "
                   "dur p0 %.1f p50 %.1f p100 %.1f\n", pct(s0, 0), pct(s0, .5), pct(s0, 1), pct(e0, .1), pct(e0, .5),
                   pct(e0, .9), pct(e0, 1), pct(d0, 0), pct(d0, .5), pct(d0, 1));
            if (only_a1) {
              // A1 alone (one job, split-major): durations by tile kind, and by how many
              // workgroups share the CU
              std::vector<unsigned> hw(2 * 16384);
              (void)hipMemcpyFromSymbol(hw.data(), HIP_SYMBOL(g_syrk_hw), hw.size() * 4);
              const int T = 13, ntiles = T * (T + 1) / 2, n = g.tasks;
              std::vector<double> full, diag, edge;
              std::map<unsigned, std::vector<int>> cu;
              for (int b = 0; b < n; ++b) {
                const int x = b & 7, sl = b >> 3, per = n >> 3, rem = n & 7;
                const int task = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + sl;
                const int tile = task % ntiles;
                int ti = 0;
                while ((ti + 1) * (ti + 2) / 2 <= tile) ++ti;
                const int tj = tile - ti * (ti + 1) / 2;
                (ti == T - 1 ? edge : ti == tj ? diag : full).push_back(d0[b]);
                const unsigned id = hw[2 * b], cu_key = (hw[2 * b + 1] << 16) | (((id >> 13) & 7) << 8) |
                                                        (((id >> 12) & 1) << 4) | ((id >> 8) & 15);
                cu[cu_key].push_back(b);
              }
              printf("    full %zu dur p10 %.1f p50 %.1f p90 %.1f | diag %zu p50 %.1f | edge %zu p50 %.1f\n",
                     full.size(), pct(full, .1), pct(full, .5), pct(full, .9), diag.size(), pct(diag, .5),
                     edge.size(), pct(edge, .5));
              std::map<int, std::vector<double>> by_occ;
              for (auto& kv : cu)
                for (int b : kv.second) by_occ[(int)kv.second.size()].push_back(d0[b]);
              std::map<int, std::vector<double>> by_xcc, by_cu_end;
              for (auto& kv : cu)
                for (int b : kv.second) by_xcc[(int)(kv.first >> 16)].push_back(d0[b]);
              printf("    per XCC dur p50:");
              for (auto& kv : by_xcc) printf(" %d:%.0f", kv.first, pct(kv.second, .5));
              printf("\n    per CU (4 WG) mean dur, sorted p0/p25/p50/p75/p100:");
              std::vector<double> cum;
              for (auto& kv : cu) {
                if (kv.second.size() != 4) continue;
                double m = 0;
                for (int b : kv.second) m += d0[b] / 4;
                cum.push_back(m);
              }
              printf(" %.0f %.0f %.0f %.0f %.0f\n", pct(cum, 0), pct(cum, .25), pct(cum, .5), pct(cum, .75), pct(cum, 1));
              printf("    CUs used %zu;", cu.size());
              for (auto& kv : by_occ) printf(" %d WG/CU: %zu WGs dur p50 %.1f max %.1f;", kv.first, kv.second.size(),
                                             pct(kv.second, .5), pct(kv.second, 1));
              printf("\n");
            }
          }
        }
      }
    }
  }
  return 0;
}
