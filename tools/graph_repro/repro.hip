// Minimal HIP-graph repro for the kernel-argument symptom behind DEBUG_CLR_GRAPH_PACKET_CAPTURE
// (tools/graph_repro/run.sh). A graph captures one launch of fill(dst_a, 1.0); the
// program replays it four times, launching fill(dst_b, 2.0 + k) eagerly on the same stream many
// times after each replay. A correct replay writes 1.0 into dst_a and leaves dst_b alone. Prints
// the result and exits 1 if a replay used the arguments of an eager launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void fill(float* dst, float v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = v;
}
// the step kernels take their task configuration (zb_task_cfg, 568 B) by value, torch's fused Adam
// a multi-tensor-apply metadata block of a few KB: a large kernarg
struct Big { float v; float pad[895]; };  // 3.5 KB, like a multi-tensor-apply TensorListMetadata
__global__ void fill_big(float* dst, Big b, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = b.v + b.pad[895 - (i & 511)];
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
      return 2;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int n = 1 << 16, eager = argc > 1 ? std::atoi(argv[1]) : 4096;
  const bool big = argc > 2 && argv[2][0] == 'b';  // 3.5 KB by-value argument
  Big ba = {}, bb = {};
  ba.v = 1.f;
  float *a, *b;
  CK(hipMalloc(&a, n * sizeof(float)));
  CK(hipMalloc(&b, n * sizeof(float)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipMemsetAsync(a, 0, n * sizeof(float), s));
  CK(hipMemsetAsync(b, 0, n * sizeof(float), s));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  if (big) fill_big<<<(n + 255) / 256, 256, 0, s>>>(a, ba, n);
  else fill<<<(n + 255) / 256, 256, 0, s>>>(a, 1.f, n);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  // replay, check, then `eager` launches of the same kernel with other arguments; four rounds (the
  // PPO update graph went wrong from its second replay on, with eager launches in between)
  bool ok = true;
  float a0 = 0.f, b0 = 0.f;
  int bad_round = -1;
  for (int r = 0; r < 4 && ok; ++r) {
    CK(hipMemsetAsync(a, 0, n * sizeof(float), s));
    CK(hipMemsetAsync(b, 0, n * sizeof(float), s));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    std::vector<float> ha(n), hb(n);
    CK(hipMemcpy(ha.data(), a, n * sizeof(float), hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), b, n * sizeof(float), hipMemcpyDeviceToHost));
    a0 = ha[0]; b0 = hb[0];
    ok = ha[0] == 1.f && ha[n - 1] == 1.f && hb[0] == 0.f;
    if (!ok) bad_round = r;
    for (int k = 0; k < eager; ++k) {
      bb.v = 2.f + k;
      if (big) fill_big<<<(n + 255) / 256, 256, 0, s>>>(b, bb, n);
      else fill<<<(n + 255) / 256, 256, 0, s>>>(b, 2.f + k, n);
    }
    CK(hipStreamSynchronize(s));
  }
  const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
  std::printf("DEBUG_CLR_GRAPH_PACKET_CAPTURE=%s %s kernarg, %d eager launches after each of 4 replays: %s "
              "(last replay a[0]=%g b[0]=%g, first wrong replay %d)\n", pc ? pc : "(unset)", big ? "3.5 KB" : "small",
              eager, ok ? "correct" : "WRONG ARGUMENTS", a0, b0, bad_round);
  return ok ? 0 : 1;
}
