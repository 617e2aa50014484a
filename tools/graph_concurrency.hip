// Does a hipGraph run independent kernel nodes concurrently on this ROCm?  (The dense-hier layer
// graph replayed as a hipGraph measured slower than its eager 8-stream launches: 16.3k vs 24.9k
// crops/s, bench extras dense_hier_b256.)  Eight independent kernels, each a few blocks that busy-
// wait ~200 us, run three ways: eager on 8 streams (fork / join by events), one hipGraph whose 8
// kernel nodes have no edges (built with hipGraphAddKernelNode), and one hipGraph captured from the
// eager 8-stream fork / join.  Concurrent execution takes ~1x the kernel time, serial ~8x.
//   hipcc --offload-arch=gfx950 -O3 tools/graph_concurrency.hip -o tools/bin/graph_concurrency
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

// busy-waits `cycles` shader clocks; writes one value per block so the work is observable
__global__ void spin(float* out, long long cycles) {
  const long long t0 = clock64();
  float a = threadIdx.x;
  while (clock64() - t0 < cycles) a = a * 0.999f + 1.f;
  if (threadIdx.x == 0) out[blockIdx.x] = a;
}

int main() {
  constexpr int K = 8, BLOCKS = 4;
  const long long cycles = 200000;   // ~100 us at ~2 GHz
  float* buf;
  CK(hipMalloc(&buf, K * BLOCKS * sizeof(float)));
  hipStream_t main_s, side[K];
  CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
  for (auto& s : side) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t fork, join[K], e0, e1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  for (auto& e : join) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto eager = [&](hipStream_t st) {
    CK(hipEventRecord(fork, st));
    for (int k = 0; k < K; ++k) {
      CK(hipStreamWaitEvent(side[k], fork, 0));
      hipLaunchKernelGGL(spin, dim3(BLOCKS), dim3(64), 0, side[k], buf + k * BLOCKS, cycles);
      CK(hipEventRecord(join[k], side[k]));
      CK(hipStreamWaitEvent(st, join[k], 0));
    }
  };
  auto timed = [&](auto f) {
    f();
    CK(hipStreamSynchronize(main_s));
    CK(hipEventRecord(e0, main_s));
    for (int r = 0; r < 5; ++r) f();
    CK(hipEventRecord(e1, main_s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 5;
  };
  // one kernel alone
  const float t1 = timed([&] { hipLaunchKernelGGL(spin, dim3(BLOCKS), dim3(64), 0, main_s, buf, cycles); });
  const float te = timed([&] { eager(main_s); });
  // explicit graph: K root kernel nodes, no edges
  hipGraph_t g;
  CK(hipGraphCreate(&g, 0));
  for (int k = 0; k < K; ++k) {
    float* p = buf + k * BLOCKS;
    long long c = cycles;
    void* args[] = {&p, &c};
    hipKernelNodeParams kp{};
    kp.func = reinterpret_cast<void*>(spin);
    kp.gridDim = dim3(BLOCKS);
    kp.blockDim = dim3(64);
    kp.kernelParams = args;
    hipGraphNode_t nd;
    CK(hipGraphAddKernelNode(&nd, g, nullptr, 0, &kp));
  }
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  const float tg = timed([&] { CK(hipGraphLaunch(ge, main_s)); });
  // captured graph of the eager fork / join
  hipGraph_t gc;
  CK(hipStreamBeginCapture(main_s, hipStreamCaptureModeGlobal));
  eager(main_s);
  CK(hipStreamEndCapture(main_s, &gc));
  hipGraphExec_t gce;
  CK(hipGraphInstantiate(&gce, gc, nullptr, nullptr, 0));
  const float tc = timed([&] { CK(hipGraphLaunch(gce, main_s)); });
  printf("{\"kernels\": %d, \"one_kernel_ms\": %.3f, \"eager_8_streams_ms\": %.3f, \"graph_root_nodes_ms\": %.3f, "
         "\"graph_captured_fork_join_ms\": %.3f}\n", K, t1, te, tg, tc);
  return 0;
}
