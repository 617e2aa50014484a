// HBM streaming ceilings on this box (read-only, write-only, copy; float4 per lane, grid-stride,
// 2 GiB buffers).  Not part of the product: the practical roof next to the 8 TB/s spec figure.
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_stream.hip -o tools/bin/hbm_stream && tools/bin/hbm_stream
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void rd(const f4* __restrict__ a, size_t n, float* out) {
  f4 s = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s.x + s.y + s.z + s.w == 12345.f) out[0] = 1.f;
}
__global__ void wr(f4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = f4{1.f, 2.f, 3.f, 4.f};
}
__global__ void cp(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

int main() {
  const size_t bytes = (size_t)2 << 30, n = bytes / 16;
  f4 *a, *b;
  float* o;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 4)) return 1;
  hipMemset(a, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int grid : {1024, 2048, 4096, 8192}) {
    float ms[3];
    for (int k = 0; k < 3; ++k) {
      auto run = [&] {
        if (k == 0) hipLaunchKernelGGL(rd, dim3(grid), dim3(256), 0, 0, a, n, o);
        if (k == 1) hipLaunchKernelGGL(wr, dim3(grid), dim3(256), 0, 0, b, n);
        if (k == 2) hipLaunchKernelGGL(cp, dim3(grid), dim3(256), 0, 0, a, b, n);
      };
      run();
      hipEventRecord(e0, 0);
      for (int r = 0; r < 5; ++r) run();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms[k], e0, e1);
      ms[k] /= 5;
    }
    printf("{\"grid\": %d, \"read_GBps\": %.1f, \"write_GBps\": %.1f, \"copy_GBps\": %.1f}\n", grid,
           bytes / (ms[0] * 1e-3) / 1e9, bytes / (ms[1] * 1e-3) / 1e9, 2 * bytes / (ms[2] * 1e-3) / 1e9);
  }
  return 0;
}
