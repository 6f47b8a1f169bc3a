// Where do workgroups of a CU-masked stream land?  Each workgroup records its
// XCC id and HW_ID (SE / SH / CU) once; the host prints the distinct (xcc, se, sh, cu)
// sets per mask.  hipcc --offload-arch=gfx950 -O2 cu_map.hip -o cu_map
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <set>
#include <tuple>
#include <vector>

__global__ void where(uint32_t* out) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    for (int i = 0; i < 20000; ++i) __builtin_amdgcn_s_sleep(1);  // keep the CU busy a while
  }
}

static void run(const char* name, const std::vector<uint32_t>& mask) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    printf("%s: stream create failed\n", name);
    return;
  }
  const int nb = 2048;
  uint32_t* d;
  hipMalloc(&d, nb * 8);
  hipLaunchKernelGGL(where, dim3(nb), dim3(64), 0, s, d);
  std::vector<uint32_t> h(nb * 2);
  hipMemcpyAsync(h.data(), d, nb * 8, hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  std::set<std::tuple<int, int, int, int>> cus;
  int per_xcc[16] = {0};
  for (int b = 0; b < nb; ++b) {
    const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    cus.insert({(int)xcc, se, sh, cu});
    per_xcc[xcc]++;
  }
  printf("%-28s distinct CUs %3zu  blocks per xcc:", name, cus.size());
  for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
  printf("\n   first CUs (xcc,se,sh,cu):");
  int k = 0;
  for (auto& t : cus) {
    if (k++ >= 12) break;
    printf(" (%d,%d,%d,%d)", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
  }
  printf("\n");
  hipFree(d);
  hipStreamDestroy(s);
}

int main() {
  std::vector<uint32_t> all(8, 0xffffffffu);
  run("all", all);
  std::vector<uint32_t> m(8, 0);
  m[0] = 1;
  run("bit 0", m);
  m.assign(8, 0); m[0] = 0xff;
  run("bits 0-7", m);
  m.assign(8, 0); m[0] = 0xffffffffu;
  run("bits 0-31", m);
  m.assign(8, 0); for (int i = 0; i < 256; i += 8) m[i / 32] |= 1u << (i % 32);
  run("every 8th bit (32)", m);
  m.assign(8, 0); for (int i = 0; i < 256; i += 16) m[i / 32] |= 1u << (i % 32);
  run("every 16th bit (16)", m);
  m.assign(8, 0xffffffffu); m[0] = 0;
  run("all but bits 0-31", m);
  m.assign(8, 0xffffffffu); for (int i = 0; i < 256; i += 8) m[i / 32] &= ~(1u << (i % 32));
  run("all but every 8th", m);
  return 0;
}
