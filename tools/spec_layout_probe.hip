// Access-pattern probe for the spectrum layout (k_fft.hip S / Y, B = 256 fp32).  Not part of the
// product.  The spectral GEMM runs at its data movement alone (its MFMAs hide: round-3 probe), so
// its time is the time of its access pattern; this times that pattern against the alternative
// layout, in both the GEMM's and the FFT kernels' shape:
//   image-major (today): [b][cq][f][32 B].  GEMM block (4 f x 32 images x 16 cq) = 512 lines of
//     128 B, one per (image, cq) run; FFT block (image, cq) = one contiguous 85 KiB run.
//   quad-major: [f / 4][b][cq][4 f x 32 B].  GEMM block = one contiguous 64 KiB run; FFT block =
//     666 lines of 128 B at a stride of B x 16 x 128 B.
// Kernels (no arithmetic): gemm_io<L> reads its S tile into LDS and writes a Y tile from LDS (the
// spec_gemm_kernel shape: 256 threads, 67.5 KB LDS, 2 blocks per CU, 5,328 blocks); fft_store<L>
// writes one S run per block from LDS (the fft_fwd3 S staging shape: 192 threads, 3 blocks per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/spec_layout_probe.hip -o tools/bin/spec_layout_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

constexpr int NF = 72 * 37, NQ = NF / 4, NCQ = 16;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(uint4* p, uint4 v) {   // k_fft.hip's non-temporal 16-B store
  __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(p));
}

// uint4 index of piece (0..7) of the 128-B line (quad q, image b, channel group cq)
template <int L>
__device__ __forceinline__ size_t line_at(int q, int b, int cq, int B) {
  return L == 0 ? (((size_t)b * NCQ + cq) * NF + 4 * q) * 2 : (((size_t)q * B + b) * NCQ + cq) * 8;
}

template <int L>
__global__ __launch_bounds__(256, 2) void gemm_io(const uint4* __restrict__ S, uint4* __restrict__ Y, int B) {
  __shared__ uint4 tile[16 * 2 * 4 * 33];
  const int ngrp = B / 32;
  const int q8 = blockIdx.x / (8 * ngrp), rem = blockIdx.x - q8 * 8 * ngrp;
  const int grp = rem >> 3, quad = q8 * 8 + (rem & 7);
  if (quad >= NQ) return;
  const int tid = threadIdx.x;
  uint4 pre[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 256 + tid, line = idx >> 3, piece = idx & 7;
    const int bl = line >> 4, cq = line & 15;
    pre[it] = S[line_at<L>(quad, grp * 32 + bl, cq, B) + piece];
  }
#pragma unroll
  for (int it = 0; it < 16; ++it) tile[it * 256 + tid] = pre[it];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 256 + tid, line = idx >> 3, piece = idx & 7;
    const int bl = line >> 4, cq = line & 15;
    const uint4 v = tile[(it * 256 + tid + 37) % (16 * 256)];
    st16(Y + line_at<L>(quad, grp * 32 + bl, cq, B) + piece, v);
  }
}

// image-major layout, 8 frequencies (two quads) per block: each (image, cq) run is 256 B instead of
// 128 B.  512 threads (8 waves, one per frequency in the real kernel), a 128 KiB S tile and a
// 128 KiB Y tile through LDS, one block per CU, 2,664 blocks at B = 256
__global__ __launch_bounds__(512, 1) void gemm_io_pair(const uint4* __restrict__ S, uint4* __restrict__ Y, int B) {
  extern __shared__ uint4 tile2[];   // 8,192 + pad
  const int ngrp = B / 32;
  const int p8 = blockIdx.x / (8 * ngrp), rem = blockIdx.x - p8 * 8 * ngrp;
  const int grp = rem >> 3, pair = p8 * 8 + (rem & 7);
  if (pair >= NQ / 2) return;
  const int tid = threadIdx.x;
  uint4 pre[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 512 + tid, line = idx >> 4, piece = idx & 15;   // line = (image, cq), 16 pieces
    const int bl = line >> 4, cq = line & 15;
    pre[it] = S[(((size_t)(grp * 32 + bl) * NCQ + cq) * NF + 8 * pair) * 2 + piece];
  }
#pragma unroll
  for (int it = 0; it < 16; ++it) tile2[it * 512 + tid] = pre[it];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 512 + tid, line = idx >> 4, piece = idx & 15;
    const int bl = line >> 4, cq = line & 15;
    const uint4 v = tile2[(it * 512 + tid + 37) % (16 * 512)];
    st16(Y + (((size_t)(grp * 32 + bl) * NCQ + cq) * NF + 8 * pair) * 2 + piece, v);
  }
}

// one block = (image b, channel group cq): its 2,664 frequencies' 32-B groups from LDS to S
template <int L>
__global__ __launch_bounds__(192, 3) void fft_store(uint4* __restrict__ S, int B) {
  __shared__ uint4 stg[37 * 74];
  const int b = blockIdx.x >> 4, cq = blockIdx.x & 15, tid = threadIdx.x;
  for (int i = tid; i < 37 * 74; i += 192) stg[i] = uint4{(unsigned)i, (unsigned)b, (unsigned)cq, 7u};
  __syncthreads();
  for (int half = 0; half < 2; ++half) {
    for (int i = tid; i < 37 * 72; i += 192) {
      const int fx = i / 72, w = i - fx * 72;          // 36 groups (72 pieces) of fy per half
      const int f = fx * 72 + 36 * half + (w >> 1);
      const size_t at = line_at<L>(f >> 2, b, cq, B) + 2 * (f & 3) + (w & 1);
      st16(S + at, stg[fx * 74 + w]);
    }
  }
}

template <typename F>
static float time_ms(F f, hipEvent_t a, hipEvent_t b, int reps = 10) {
  f();
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int B = 256;
  const size_t bytes = (size_t)B * NCQ * NF * 32;
  uint4 *S, *Y;
  CK(hipMalloc(&S, bytes));
  CK(hipMalloc(&Y, bytes));
  CK(hipMemset(S, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int nq8 = (NQ + 7) / 8, ngrp = B / 32;
  std::vector<float> g0, g1, g2, f0, f1;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_io_pair), hipFuncAttributeMaxDynamicSharedMemorySize,
                         16 * 512 * 16));
  for (int r = 0; r < 7; ++r) {
    g0.push_back(time_ms([&] { hipLaunchKernelGGL(gemm_io<0>, dim3(nq8 * 8 * ngrp), dim3(256), 0, 0, S, Y, B); }, e0, e1));
    g1.push_back(time_ms([&] { hipLaunchKernelGGL(gemm_io<1>, dim3(nq8 * 8 * ngrp), dim3(256), 0, 0, S, Y, B); }, e0, e1));
    g2.push_back(time_ms([&] { hipLaunchKernelGGL(gemm_io_pair, dim3((NQ / 2 + 7) / 8 * 8 * ngrp), dim3(512), 16 * 512 * 16, 0, S, Y, B); }, e0, e1));
    f0.push_back(time_ms([&] { hipLaunchKernelGGL(fft_store<0>, dim3(B * 16), dim3(192), 0, 0, S, B); }, e0, e1));
    f1.push_back(time_ms([&] { hipLaunchKernelGGL(fft_store<1>, dim3(B * 16), dim3(192), 0, 0, S, B); }, e0, e1));
  }
  CK(hipGetLastError());
  auto med = [](std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("{\"B\": %d, \"gemm_io_image_major_pair_ms\": %.4f, ", B, med(g2));
  printf("\"gemm_io_image_major_ms\": %.4f, \"gemm_io_quad_major_ms\": %.4f, "
         "\"fft_store_image_major_ms\": %.4f, \"fft_store_quad_major_ms\": %.4f, \"spectrum_MB\": %.1f}\n",
         med(g0), med(g1), med(f0), med(f1), bytes / 1e6);
  return 0;
}
