// FETCH_SIZE / WRITE_SIZE calibration for the step kernel's HBM access patterns (diagnostic only,
// not part of libzbot). Each kernel reads (or writes) `rows` SoA rows of N floats exactly once:
//   k_team   : one wave = 4 envs x 16 lanes, every lane of a team loads the same address (ST())
//   k_carry  : lane s of team e loads row s (+16k) of env e (carry_prefetch)
//   k_wide   : 16 B per lane streaming (the guide's calibrated pattern)
//   k_store  : staged_store's pattern (16 rows x 4 envs per wave instruction)
//   *_xcd    : the same with the step kernel's XCD-aware workgroup -> env-block mapping
// Known bytes = rows * N * 4; rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE gives the counter's view.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_team(const float* __restrict__ st, int N, int rows, float* __restrict__ out) {
  const int env = blockIdx.x * 4 + threadIdx.x / 16;
  float acc = 0.f;
  for (int f = 0; f < rows; ++f) acc += st[(size_t)f * N + env];
  if (acc == 123.456f) out[env] = acc;
}
__global__ void k_carry(const float* __restrict__ st, int N, int rows, float* __restrict__ out) {
  const int env = blockIdx.x * 4 + threadIdx.x / 16, s = threadIdx.x % 16;
  float acc = 0.f;
  for (int f = s; f < rows; f += 16) acc += st[(size_t)f * N + env];
  if (acc == 123.456f) out[env] = acc;
}
__device__ __forceinline__ int xcd_block(int b, int nb) { return nb % 8 ? b : (b % 8) * (nb / 8) + b / 8; }
__global__ void k_team_xcd(const float* __restrict__ st, int N, int rows, float* __restrict__ out) {
  const int env = xcd_block(blockIdx.x, gridDim.x) * 4 + threadIdx.x / 16;
  float acc = 0.f;
  for (int f = 0; f < rows; ++f) acc += st[(size_t)f * N + env];
  if (acc == 123.456f) out[env] = acc;
}
__global__ void k_store_xcd(float* __restrict__ st, int N, int rows) {
  const int e = threadIdx.x % 4, f0 = threadIdx.x / 4;
  const int env = xcd_block(blockIdx.x, gridDim.x) * 4 + e;
  for (int f = f0; f < rows; f += 16) st[(size_t)f * N + env] = (float)f;
}
__global__ void k_wide(const float4* __restrict__ st, size_t n4, float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) {
    const float4 v = st[i];
    if (v.x + v.y + v.z + v.w == 123.456f) out[0] = v.x;
  }
}
__global__ void k_store(float* __restrict__ st, int N, int rows) {
  const int e = threadIdx.x % 4, f0 = threadIdx.x / 4;
  const int env = blockIdx.x * 4 + e;
  for (int f = f0; f < rows; f += 16) st[(size_t)f * N + env] = (float)f;
}

extern "C" int calib_run(int N, int rows) {
  float *st, *out;
  const size_t n = (size_t)rows * N;
  if (hipMalloc(&st, n * 4) != hipSuccess || hipMalloc(&out, (size_t)N * 4) != hipSuccess) return -1;
  (void)hipMemset(st, 0, n * 4);
  for (int rep = 0; rep < 5; ++rep) {
    k_team<<<N / 4, 64>>>(st, N, rows, out);
    k_carry<<<N / 4, 64>>>(st, N, rows, out);
    k_wide<<<(unsigned)((n / 4 + 255) / 256), 256>>>(reinterpret_cast<const float4*>(st), n / 4, out);
    k_store<<<N / 4, 64>>>(st, N, rows);
    k_team_xcd<<<N / 4, 64>>>(st, N, rows, out);
    k_store_xcd<<<N / 4, 64>>>(st, N, rows);
  }
  (void)hipDeviceSynchronize();
  (void)hipFree(st);
  (void)hipFree(out);
  return 0;
}
