// Practical v_mfma_f32_32x32x16_bf16 throughput on this part: register-only loops, no
// memory traffic in the timed body, at 1 / 2 / 4 waves per SIMD and with the
// accumulator chains interleaved (ILV: acc0 acc1 acc2 acc3 ...) or in runs of six on
// one accumulator (the x3 kernels' x3_six order).  The ceiling the SYRK kernels'
// roofline fraction should be read against.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_peak tools/microbench/mfma_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NACC, bool RUNS>
__global__ __launch_bounds__(256) void k_peak(int iters, float* out, float seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(seed * (threadIdx.x + i));
    b[i] = (__bf16)(seed * (threadIdx.x - i));
  }
  floatx16 acc[NACC];
  for (int c = 0; c < NACC; ++c)
    for (int v = 0; v < 16; ++v) acc[c][v] = 0.f;
  for (int it = 0; it < iters; ++it) {
    if constexpr (RUNS) {
#pragma unroll
      for (int c = 0; c < NACC; ++c)
#pragma unroll
        for (int r = 0; r < 6; ++r) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
    } else {
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < NACC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int c = 0; c < NACC; ++c)
    for (int v = 0; v < 16; ++v) s += acc[c][v];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC, bool RUNS>
void run(const char* name, int wps, float* out) {
  const int iters = 4000;
  const int blocks = 256 * wps;  // 256-thread workgroups: one wave per SIMD each
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_peak<NACC, RUNS><<<blocks, 256>>>(10, out, 1e-3f);
  hipEventRecord(e0);
  k_peak<NACC, RUNS><<<blocks, 256>>>(iters, out, 1e-3f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)blocks * 4 * iters * 6 * NACC * 32.0 * 32 * 16 * 2;
  const double tf = flops / (ms * 1e-3) / 1e12;
  printf("%-10s waves/SIMD %d  %8.3f ms  %7.1f TF/s  %.3f of 2.5 PF\n", name, wps, ms, tf, tf / 2500.0);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4 * 256 * sizeof(float) * 4);
  for (int wps = 1; wps <= 4; wps *= 2) {
    run<4, false>("ilv4", wps, out);
    run<4, true>("runs6x4", wps, out);
    run<2, false>("ilv2", wps, out);
    run<1, false>("chain1", wps, out);
  }
  hipFree(out);
  return 0;
}
