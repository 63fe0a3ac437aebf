// HIP graph: a captured hipMemsetAsync followed by a kernel that depends on it (the pattern of
// PyTorch's multi-block reductions, which zero a semaphore buffer before the reduce kernel; e.g.
// clip_grad_norm_'s total norm -- tools/graph_repro/update_repro.py). Per replay the counter must
// be re-zeroed by the memset node, then every block adds 1: after each replay counter == blocks.
// Usage: memset_repro [replays]; run with DEBUG_CLR_GRAPH_PACKET_CAPTURE unset / 1 and 0.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(2);                                                               \
    }                                                                             \
  } while (0)

__global__ void count_blocks(unsigned* counter, unsigned* last, unsigned blocks) {
  if (threadIdx.x == 0) {
    const unsigned old = atomicAdd(counter, 1u);
    if (old == blocks - 1) *last = old + 1;  // the last block sees every other block's add
  }
}

int main(int argc, char** argv) {
  const int replays = argc > 1 ? std::atoi(argv[1]) : 4;
  const unsigned blocks = 256;
  const char* mode = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
  unsigned *counter, *last;
  CHK(hipMalloc(&counter, sizeof(unsigned)));
  CHK(hipMalloc(&last, sizeof(unsigned)));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CHK(hipMemset(counter, 0xff, sizeof(unsigned)));  // garbage: the captured memset must clear it
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  CHK(hipMemsetAsync(counter, 0, sizeof(unsigned), s));
  CHK(hipMemsetAsync(last, 0, sizeof(unsigned), s));
  count_blocks<<<blocks, 64, 0, s>>>(counter, last, blocks);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  int bad = 0;
  for (int r = 0; r < replays; ++r) {
    CHK(hipGraphLaunch(ge, s));
    CHK(hipStreamSynchronize(s));
    unsigned c = 0, l = 0;
    CHK(hipMemcpy(&c, counter, sizeof(c), hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&l, last, sizeof(l), hipMemcpyDeviceToHost));
    const bool ok = c == blocks && l == blocks;
    bad += ok ? 0 : 1;
    std::printf("  replay %d: counter %u last %u (expect %u)%s\n", r, c, l, blocks, ok ? "" : "  <-- WRONG");
  }
  std::printf("DEBUG_CLR_GRAPH_PACKET_CAPTURE=%s: memset node + dependent kernel, %d of %d replays wrong\n",
              mode ? mode : "(unset)", bad, replays);
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(s));
  CHK(hipFree(counter));
  CHK(hipFree(last));
  return bad ? 1 : 0;
}
