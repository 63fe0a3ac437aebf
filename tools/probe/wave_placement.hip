// Wave placement probe (diagnostic, not part of libzbot): where the hardware puts the two waves of a
// 128-thread workgroup that has the split step kernel's resources (21 888 B of LDS, 218 VGPRs), for
// 1024 workgroups (4096 envs). Each wave records {block, wave, HW_ID, XCC_ID, start, end}; the waves
// spin ~40 us so that the whole grid is resident at once.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probe/wave_placement tools/probe/wave_placement.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <map>
#include <set>

__global__ __launch_bounds__(128, 2) void probe(unsigned long long* rec, int spin) {
  extern __shared__ float lds[];
  asm volatile("" ::: "v217");  // 218 VGPRs, like zb_step_split_kernel
  const int w = threadIdx.x / 64;
  const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < (unsigned long long)spin) t = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (float)hw;
  if (threadIdx.x % 64 == 0) {
    unsigned long long* r = rec + (blockIdx.x * 2 + w) * 4;
    r[0] = hw; r[1] = xcc; r[2] = t0; r[3] = t;
  }
}

__global__ __launch_bounds__(64, 2) void probe1(unsigned long long* rec, int spin) {
  extern __shared__ float lds[];
  asm volatile("" ::: "v255");  // 256 VGPRs, like zb_step_kernel
  const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
  const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < (unsigned long long)spin) t = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (float)hw;
  if (threadIdx.x == 0) {
    unsigned long long* r = rec + blockIdx.x * 4;
    r[0] = hw; r[1] = xcc; r[2] = t0; r[3] = t;
  }
}

template <int T>
__global__ __launch_bounds__(T, 1) void probeT(unsigned long long* rec, int spin, int big) {
  extern __shared__ float lds[];
  asm volatile("" ::: "v255");
  if (big) asm volatile("" ::: "a255");  // (512 registers: one wave per SIMD)
  const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
  const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < (unsigned long long)spin) t = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (float)hw;
  if (threadIdx.x % 64 == 0) {
    unsigned long long* r = rec + (blockIdx.x * (T / 64) + threadIdx.x / 64) * 4;
    r[0] = hw; r[1] = xcc; r[2] = t0; r[3] = t;
  }
}

template <int T>
int mainT(int blocks, int lds, int big) {
  const int waves = blocks * (T / 64);
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * waves * 4);
  probeT<T><<<blocks, T, lds>>>(d, 4000, big);
  std::vector<unsigned long long> h(waves * 4);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  std::map<unsigned long long, int> per_simd;
  for (int b = 0; b < waves; ++b) {
    const unsigned long long hw = h[b * 4], xcc = h[b * 4 + 1];
    per_simd[(xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 8) | (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3)]++;
  }
  std::map<int, int> hist;
  for (auto& kv : per_simd) hist[kv.second]++;
  printf("%d-thread workgroups%s: blocks %d lds %d: SIMDs used %zu\n", T, big ? " (512 regs)" : "", blocks, lds, per_simd.size());
  for (auto& kv : hist) printf("  SIMDs holding %d waves: %d\n", kv.first, kv.second);
  return 0;
}

int main1(int blocks, int lds) {
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * blocks * 4);
  probe1<<<blocks, 64, lds>>>(d, 4000);
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  std::map<unsigned long long, int> per_simd;
  for (int b = 0; b < blocks; ++b) {
    const unsigned long long hw = h[b * 4], xcc = h[b * 4 + 1];
    per_simd[(xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 8) | (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3)]++;
  }
  std::map<int, int> hist;
  for (auto& kv : per_simd) hist[kv.second]++;
  printf("one-wave workgroups: blocks %d lds %d: SIMDs used %zu\n", blocks, lds, per_simd.size());
  for (auto& kv : hist) printf("  SIMDs holding %d waves: %d\n", kv.first, kv.second);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 3 && argv[3][0] == '1') return main1(atoi(argv[1]), atoi(argv[2]));
  if (argc > 3 && argv[3][0] == 'b') return mainT<64>(atoi(argv[1]), atoi(argv[2]), 1);
  if (argc > 3 && argv[3][0] == '2') return mainT<128>(atoi(argv[1]), atoi(argv[2]), 0);
  if (argc > 3 && argv[3][0] == '4') return mainT<256>(atoi(argv[1]), atoi(argv[2]), 0);
  const int blocks = argc > 1 ? atoi(argv[1]) : 1024, lds = argc > 2 ? atoi(argv[2]) : 21888;
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * blocks * 8);
  probe<<<blocks, 128, lds>>>(d, 4000);  // 40 us at 100 MHz
  std::vector<unsigned long long> h(blocks * 8);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  std::map<unsigned long long, int> per_simd;
  int same_simd = 0, same_cu = 0;
  for (int b = 0; b < blocks; ++b) {
    unsigned long long key[2];
    for (int w = 0; w < 2; ++w) {
      const unsigned long long hw = h[(b * 2 + w) * 4], xcc = h[(b * 2 + w) * 4 + 1];
      const unsigned simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      key[w] = (xcc << 16) | (se << 12) | (sh << 8) | (cu << 2) | simd;
      per_simd[key[w]]++;
    }
    same_simd += key[0] == key[1];
    same_cu += (key[0] >> 2) == (key[1] >> 2);
  }
  // which waves share a SIMD: by wave index in the workgroup (role 0: wave 0 = physics) and by the
  // split kernel's role 2 (wave 0 takes the physics iff its SIMD + slot parity is even)
  std::map<unsigned long long, std::vector<int>> role0, role2;
  for (int b = 0; b < blocks; ++b) {
    const unsigned long long hw0 = h[b * 8];
    const int want0 = (int)(((hw0 & 15) + ((hw0 >> 4) & 3)) & 1);  // 0: wave 0 is physics
    for (int w = 0; w < 2; ++w) {
      const unsigned long long hw = h[(b * 2 + w) * 4], xcc = h[(b * 2 + w) * 4 + 1];
      const unsigned long long key = (xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 8) | (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3);
      role0[key].push_back(w == 0);
      role2[key].push_back((w == 0) == (want0 == 0));
    }
  }
  for (int r = 0; r < 2; ++r) {
    std::map<int, int> ph;
    for (auto& kv : (r ? role2 : role0)) { int a = 0; for (int x : kv.second) a += x; ph[a]++; }
    printf("  role %d: SIMDs by physics waves held:", r ? 2 : 0);
    for (auto& kv : ph) printf(" %d->%d", kv.first, kv.second);
    printf("\n");
  }
  std::map<int, int> hist;
  for (auto& kv : per_simd) hist[kv.second]++;
  printf("blocks %d lds %d: SIMDs used %zu; workgroups with both waves on one SIMD %d, on one CU %d\n", blocks, lds,
         per_simd.size(), same_simd, same_cu);
  for (auto& kv : hist) printf("  SIMDs holding %d waves: %d\n", kv.first, kv.second);
  for (int b = 0; b < 8; ++b)
    printf("  block %d: wave0 hw %08llx xcc %llu, wave1 hw %08llx xcc %llu\n", b, h[b * 8], h[b * 8 + 1], h[b * 8 + 4], h[b * 8 + 5]);
  return 0;
}
