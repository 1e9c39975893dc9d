// placement_probe.hip — where the waves of two-wave workgroups land (r5 diagnostic): each wave records its HW_ID
// (SIMD, CU, shader array / engine) and XCC_ID; the host prints per-CU tables of (workgroup, wave) -> SIMD for the first
// CUs and a summary of how often the two waves of one workgroup share a SIMD / how wave 0s spread over SIMDs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <map>
#include <vector>

__global__ __launch_bounds__(128) void probe(uint32_t* out) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  for (int i = 0; i < 200; ++i) __builtin_amdgcn_s_sleep(127);  // keep the workgroups co-resident
  if ((threadIdx.x & 63) == 0) {
    out[(blockIdx.x * 2 + (threadIdx.x >> 6)) * 2] = hw;
    out[(blockIdx.x * 2 + (threadIdx.x >> 6)) * 2 + 1] = xcc;
  }
}

int main() {
  const int wgs = 2048;
  uint32_t* d;
  if (hipMalloc(&d, wgs * 4 * sizeof(uint32_t)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(wgs), dim3(128), 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<uint32_t> h(wgs * 4);
  if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  // HW_ID (gfx9): wave_id [3:0], simd_id [5:4], pipe [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
  std::map<uint32_t, std::vector<int>> by_cu;  // key: xcc << 16 | se << 8 | sh << 4 | cu
  int same = 0;
  int w0_simd[4] = {0, 0, 0, 0}, w1_simd[4] = {0, 0, 0, 0};
  for (int b = 0; b < wgs; ++b) {
    int simd[2];
    uint32_t key = 0;
    for (int w = 0; w < 2; ++w) {
      const uint32_t hw = h[(b * 2 + w) * 2], xcc = h[(b * 2 + w) * 2 + 1];
      simd[w] = (hw >> 4) & 3;
      key = (xcc & 0xf) << 16 | ((hw >> 13) & 7) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15);
    }
    same += simd[0] == simd[1];
    ++w0_simd[simd[0]];
    ++w1_simd[simd[1]];
    by_cu[key].push_back(b * 16 + simd[0] * 4 + simd[1]);
  }
  printf("workgroups %d, CUs seen %zu, both waves on one SIMD: %d\n", wgs, by_cu.size(), same);
  printf("wave0 SIMD histogram %d %d %d %d; wave1 %d %d %d %d\n", w0_simd[0], w0_simd[1], w0_simd[2], w0_simd[3],
         w1_simd[0], w1_simd[1], w1_simd[2], w1_simd[3]);
  int shown = 0;
  for (auto& kv : by_cu) {
    if (shown++ >= 12) break;
    printf("cu %06x:", kv.first);
    for (int v : kv.second) printf(" wg%d(w0:s%d,w1:s%d)", v / 16, (v >> 2) & 3, v & 3);
    printf("\n");
  }
  // per-SIMD role mix under role = wave ^ parity(f(blockIdx)) for a few f
  const char* names[3] = {"wave", "wave^(b&1)", "wave^((b>>1)&1)"};
  for (int f = 0; f < 3; ++f) {
    std::map<uint64_t, std::pair<int, int>> mix;  // (cu key, simd) -> (#role0, #role1)
    for (auto& kv : by_cu)
      for (int v : kv.second) {
        const int b = v / 16, s0 = (v >> 2) & 3, s1 = v & 3;
        const int flip = f == 0 ? 0 : f == 1 ? (b & 1) : ((b >> 1) & 1);
        auto& a = mix[(uint64_t)kv.first << 4 | s0];
        auto& c = mix[(uint64_t)kv.first << 4 | s1];
        (flip ? a.second : a.first)++;
        (flip ? c.first : c.second)++;
      }
    int balanced = 0, total = 0;
    for (auto& m : mix) { ++total; balanced += m.second.first == m.second.second; }
    printf("%s: SIMDs with equal role counts %d of %d\n", names[f], balanced, total);
  }
  return 0;
}
