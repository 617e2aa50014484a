// A/B microbenchmark of the FFT conv path kernels (k_fft.hip), interleaved in ONE process.
// Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I../monkey-pose_amd/csrc \
//         tools/bench_fft.hip -o tools/bin/bench_fft
//   ./bench_fft [batch=256] [rounds=5]
//
// Prints one JSON object: median ms per launch and algorithmic GB/s of fft_fwd, spec_gemm, fft_inv
// (numerics are covered by tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "k_fft.hip"

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

using namespace mp;

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
static float time_ms(F f, hipEvent_t a, hipEvent_t b, int reps) {
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) CK(f());
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
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
  CK(build_spec_weights(w, KS, Gx, &unscale));
  CK(launch_fft_fwd(act, S, B, H, W, 0));
  CK(hipDeviceSynchronize());

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
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
  std::vector<float> tf, tg, ti, ta, tp1, tp2, tp3, tp4;
  const int ngrp = (B + SG_NI - 1) / SG_NI, nq8 = (NQUAD + 7) / 8;
  auto probe = [&](int v) {
#define PRB(K)                                                                                          \
  if (v == K)                                                                                         \
    hipLaunchKernelGGL(spec_gemm_kernel<K>, dim3(nq8 * 8 * ngrp), dim3(256), 0, 0, (const uint4*)S, \
                       (const uint4*)Gx, (uint4*)Y, B, ngrp, unscale);
    PRB(1) PRB(2) PRB(3) PRB(4)
#undef PRB
    return hipGetLastError();
  };
  for (int r = 0; r < rounds; ++r) {
    tf.push_back(time_ms([&] { return launch_fft_fwd(act, S, B, H, W, 0); }, e0, e1, 10));
    tg.push_back(time_ms([&] { return launch_spec_gemm(S, Gx, Y, B, unscale, 0); }, e0, e1, 10));
    ti.push_back(time_ms([&] { return launch_fft_inv(Y, P, B, H, W, 0); }, e0, e1, 10));
    ta.push_back(time_ms([&] { return launch_fft_inv_a_fwd(Y, a, S, B, 0); }, e0, e1, 10));
    tp1.push_back(time_ms([&] { return probe(1); }, e0, e1, 10));
    tp2.push_back(time_ms([&] { return probe(2); }, e0, e1, 10));
    tp3.push_back(time_ms([&] { return probe(3); }, e0, e1, 10));
    tp4.push_back(time_ms([&] { return probe(4); }, e0, e1, 10));
  }
  auto med = [](std::vector<float> x) {
    std::sort(x.begin(), x.end());
    return x[x.size() / 2];
  };
  const double spec = (double)fft_spec_bytes(B), actb = (double)B * 64 * H * W * 4;
  printf("{\"batch\": %d, \"kernels\": [\n", B);
  printf("  {\"name\": \"fft_fwd\", \"median_ms\": %.4f, \"GBps\": %.1f},\n", med(tf), (spec + actb) / med(tf) / 1e6);
  printf("  {\"name\": \"spec_gemm\", \"median_ms\": %.4f, \"GBps\": %.1f},\n", med(tg),
         (2 * spec + (double)fft_weight_bytes()) / med(tg) / 1e6);
  printf("  {\"name\": \"fft_inv\", \"median_ms\": %.4f, \"GBps\": %.1f},\n", med(ti), (spec + actb) / med(ti) / 1e6);
  printf("  {\"name\": \"inv_a_fwd\", \"median_ms\": %.4f, \"GBps\": %.1f},\n", med(ta),
         (2 * spec + 3 * actb) / med(ta) / 1e6);
  printf("  {\"name\": \"PROBE gemm no-MFMA\", \"median_ms\": %.4f},\n", med(tp1));
  printf("  {\"name\": \"PROBE gemm no-S/W-loads\", \"median_ms\": %.4f},\n", med(tp2));
  printf("  {\"name\": \"PROBE gemm no-W-loads\", \"median_ms\": %.4f},\n", med(tp3));
  printf("  {\"name\": \"PROBE gemm no-S-loads\", \"median_ms\": %.4f}\n]}\n", med(tp4));
  return 0;
}
