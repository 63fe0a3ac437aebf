// HIP graph: a captured hipMemsetAsync followed by a kernel that depends on it (the pattern of
// PyTorch's multi-block reductions, which zero a semaphore buffer before the reduce kernel; e.g.
// clip_grad_norm_'s total norm -- tools/graph_repro/update_repro.py). Per replay the counter must
// be re-zeroed by the memset node, then every block adds 1: after each replay counter == blocks.
// Second case: producer kernel -> memset node -> consumer kernel reading the producer's output.
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

// A slow producer (writes v into every element of buf after some busy work), a memset node, and a
// consumer that counts the elements of buf that do not hold v: in stream order the consumer runs
// after the producer, so the count must be 0 on every replay.
__global__ void produce(float* buf, int n, const float* v, int spin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x = 0.f;
  for (int k = 0; k < spin; ++k) x = fmaf(x, 0.999f, 1e-3f);  // busy work
  buf[i] = *v + (x > 1e30f ? 1.f : 0.f);
}
__global__ void consume(const float* buf, int n, const float* v, unsigned* sem, unsigned* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && buf[i] != *v) atomicAdd(bad, 1u);
  if (threadIdx.x == 0) atomicAdd(sem, 1u);
}

static int producer_memset_consumer(int replays) {
  const int n = 1 << 22, spin = 2000;
  float *buf, *v;
  unsigned *sem, *bad;
  CHK(hipMalloc(&buf, sizeof(float) * n));
  CHK(hipMalloc(&v, sizeof(float)));
  CHK(hipMalloc(&sem, sizeof(unsigned)));
  CHK(hipMalloc(&bad, sizeof(unsigned)));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  produce<<<n / 256, 256, 0, s>>>(buf, n, v, spin);
  CHK(hipMemsetAsync(sem, 0, sizeof(unsigned), s));  // (PyTorch zeroes a reduction's semaphores here)
  CHK(hipMemsetAsync(bad, 0, sizeof(unsigned), s));
  consume<<<n / 256, 256, 0, s>>>(buf, n, v, sem, bad);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  int wrong = 0;
  for (int r = 0; r < replays; ++r) {
    const float val = (float)(r + 1);
    CHK(hipMemcpy(v, &val, sizeof(val), hipMemcpyHostToDevice));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipStreamSynchronize(s));
    unsigned b = 0;
    CHK(hipMemcpy(&b, bad, sizeof(b), hipMemcpyDeviceToHost));
    wrong += b ? 1 : 0;
    std::printf("  producer -> memset -> consumer, replay %d: %u of %d elements read before the producer wrote them%s\n",
                r, b, n, b ? "  <-- WRONG" : "");
  }
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(s));
  CHK(hipFree(buf)); CHK(hipFree(v)); CHK(hipFree(sem)); CHK(hipFree(bad));
  return wrong;
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
  const int bad2 = producer_memset_consumer(replays);
  std::printf("DEBUG_CLR_GRAPH_PACKET_CAPTURE=%s: memset node + dependent kernel, %d of %d replays wrong; "
              "producer kernel -> memset -> consumer kernel, %d of %d replays wrong\n",
              mode ? mode : "(unset)", bad, replays, bad2, replays);
  bad += bad2;
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(s));
  CHK(hipFree(counter));
  CHK(hipFree(last));
  return bad ? 1 : 0;
}
