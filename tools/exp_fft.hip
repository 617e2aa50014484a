// Occupancy probe of the FFT-path kernels (k_fft.hip): each kernel timed at B = 256 with its
// static LDS only and with extra dynamic LDS that caps it at 1 block per CU (not product code).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Imonkey-pose_amd/csrc \
//         tools/exp_fft.hip -o tools/bin/exp_fft && tools/bin/exp_fft 256
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "k_fft.hip"

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

using namespace mp;

// ---- prototype: channel-pair blocks (128 threads, ~38 KB LDS -> 4 blocks / CU) ----
// block -> (image, pair): the 4 pairs of one C8 chunk share blockIdx % 8 (one XCD)
__device__ __forceinline__ int pair_of(int j) { return 4 * (j & 7) + (j >> 3); }

__global__ __launch_bounds__(128, 4) void fft_inv2_kernel(const void* __restrict__ Y, float* __restrict__ P, int H,
                                                          int W) {
  __shared__ cpx T[64 * 2 * FX];   // 37,888 B: inverse columns T[y][c][fx]; then parked rows
  const int b = blockIdx.x >> 5, cp = pair_of(blockIdx.x & 31);
  const int cq = cp >> 1, c0 = 2 * (cp & 1), q = cp >> 2, e0 = 2 * (cp & 3);
  const int tid = threadIdx.x;
  if (tid < 2 * FX) {
    const int fx = tid >> 1, c = tid & 1;
    const cpx* src = static_cast<const cpx*>(Y) + (((size_t)b * 16 + cq) * NF + fx * 72) * 4 + c0 + c;
    cpx v[72];
#pragma unroll
    for (int fy = 0; fy < 72; ++fy) v[fy] = src[fy * 4];
    fft72<1>(v);
#pragma unroll
    for (int y = 0; y < 64; ++y) T[(y * 2 + c) * FX + fx] = v[y];
  }
  lds_barrier();
  const bool live = tid < 64 && tid < H;
  {
    cpx v[72];
    if (live) {
      const cpx* ta = T + (tid * 2) * FX;
      const cpx* tb = ta + FX;
#pragma unroll
      for (int k = 0; k < FX; ++k) {
        const cpx A = ta[k], B = tb[k];
        v[k] = {A.x - B.y, A.y + B.x};
        if (k > 0 && k < FX - 1) v[72 - k] = {A.x + B.y, B.x - A.y};
      }
      fft72<1>(v);
    }
    lds_barrier();
    if (live) {
#pragma unroll
      for (int x = 0; x < 64; ++x) T[tid * RLD + x] = v[x];
    }
  }
  lds_barrier();
#pragma unroll 4
  for (int i = tid; i < H * W; i += 128) {
    const int yy = i / W, x = i - yy * W;
    const cpx a = T[yy * RLD + x];
    *reinterpret_cast<float2*>(P + c8_index(b, q, yy, x, e0, H, W)) = float2{a.x, a.y};
  }
}

static float* dalloc_rand(size_t n, std::mt19937& g, float lo, float hi) {
  std::vector<float> h(n);
  std::uniform_real_distribution<float> d(lo, hi);
  for (auto& v : h) v = d(g);
  float* p;
  CK(hipMalloc(&p, n * sizeof(float)));
  CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return p;
}

template <typename F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256;
  const int H = 64, W = 64, KS = 15;
  std::mt19937 g(1);
  float* act = dalloc_rand((size_t)B * 64 * H * W, g, -1.f, 1.f);
  float* w = dalloc_rand((size_t)KS * KS * 64 * 64, g, -0.02f, 0.02f);
  void *S, *Y, *Gx;
  float* P;
  CK(hipMalloc(&S, fft_spec_bytes(B)));
  CK(hipMalloc(&Y, fft_spec_bytes(B)));
  CK(hipMalloc(&Gx, fft_weight_bytes()));
  CK(hipMalloc(&P, (size_t)B * 64 * H * W * sizeof(float)));
  float unscale = 0.f;
  CK(build_spec_weights(w, KS, Gx, &unscale, false));
  float* X = dalloc_rand((size_t)B * 64 * H * W, g, -1.f, 1.f);
  float* O = dalloc_rand((size_t)B * 64 * H * W, g, -1.f, 1.f);
  float* I;
  CK(hipMalloc(&I, (size_t)B * 64 * H * W * sizeof(float)));
  float* vecs = dalloc_rand(V_COUNT * 64, g, 0.5f, 1.f);
  ConvArgs a{};
  a.H = H;
  a.W = W;
  a.X = X;
  a.O = O;
  a.dst = I;
  a.vecs = vecs;
  CK(launch_fft_fwd(act, S, B, H, W, 0, false));
  CK(launch_spec_gemm(S, Gx, Y, B, unscale, 0, false));
  CK(hipDeviceSynchronize());
  {
    float* P2;
    CK(hipMalloc(&P2, (size_t)B * 64 * H * W * sizeof(float)));
    hipLaunchKernelGGL((fft_inv_kernel<false, false>), dim3(B * 16), dim3(FNT), 0, 0, Y, P, H, W);
    hipLaunchKernelGGL(fft_inv2_kernel, dim3(B * 32), dim3(128), 0, 0, Y, P2, H, W);
    CK(hipDeviceSynchronize());
    std::vector<float> h1((size_t)B * 64 * H * W), h2(h1.size());
    CK(hipMemcpy(h1.data(), P, h1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), P2, h2.size() * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < h1.size(); ++i) diff += h1[i] != h2[i];
    const float t1 = time_ms([&] { hipLaunchKernelGGL((fft_inv_kernel<false, false>), dim3(B * 16), dim3(FNT), 0, 0, Y, P, H, W); }, 20);
    const float t2 = time_ms([&] { hipLaunchKernelGGL(fft_inv2_kernel, dim3(B * 32), dim3(128), 0, 0, Y, P2, H, W); }, 20);
    const float t1b = time_ms([&] { hipLaunchKernelGGL((fft_inv_kernel<false, false>), dim3(B * 16), dim3(FNT), 0, 0, Y, P, H, W); }, 20);
    const float t2b = time_ms([&] { hipLaunchKernelGGL(fft_inv2_kernel, dim3(B * 32), dim3(128), 0, 0, Y, P2, H, W); }, 20);
    printf("fft_inv (4-ch) %.4f %.4f ms   fft_inv2 (pair) %.4f %.4f ms   mismatches %zu\n", t1, t1b, t2, t2b, diff);
  }
  {
    const float tg = time_ms([&] { CK(launch_spec_gemm(S, Gx, Y, B, unscale, 0, false)); }, 20);
    printf("NT_ST %d: spec_gemm %.4f ms\n", FFT_NT_ST, tg);
  }
  for (int extra : {0}) {
    const float tf = time_ms([&] {
      hipLaunchKernelGGL((fft_fwd_kernel<false, false>), dim3(B * 16), dim3(FNT), extra, 0, act, S, H, W);
    }, 20);
    const float ti = time_ms([&] {
      hipLaunchKernelGGL((fft_inv_kernel<false, false>), dim3(B * 16), dim3(FNT), extra, 0, Y, P, H, W);
    }, 20);
    const float ta = time_ms([&] {
      hipLaunchKernelGGL((fft_inv_a_fwd_kernel<false, false>), dim3(B * 16), dim3(FNT), extra, 0, Y, a, S);
    }, 20);
    printf("NT_ST %d extra LDS %6d B: fft_fwd %.4f  fft_inv %.4f  inv_a_fwd %.4f ms\n", FFT_NT_ST, extra, tf, ti, ta);
  }
  return 0;
}
