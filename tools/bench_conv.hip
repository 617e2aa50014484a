// A/B microbenchmark of the hGRU eCRF conv kernel variants, interleaved in ONE process (per the
// CDNA guide: cross-process / cross-device timings are not comparable).  Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../monkey-pose_amd/csrc tools/bench_conv.hip -o build/bench_conv
//   ./bench_conv [batch=256] [rounds=5]
//
// Prints one JSON object: per variant the median ms per launch, algorithmic TFLOP/s, and the max
// |difference| of its output against variant 0 (all variants must agree bit-for-bit or to rounding).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "k_conv64.hip"
#include "k_conv64x3.hip"

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

using namespace mp;

struct Variant {
  const char* name;
  hipError_t (*launch)(const ConvArgs&, const void*, float, int, hipStream_t);
  int tile_rows;
};

template <int EPI, int NW, int SCHED>
hipError_t run_v(const ConvArgs& a0, const void* w, float us, int B, hipStream_t st) {
  ConvArgs a = a0;
  a.ascale = ACT_SCALE;
  a.tiles_x = a.W / TW;
  a.tiles_y = a.H / TH3;
  return launch_x3_t<15, EPI, NW, SCHED>(a, w, us, B, st);
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

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const int H = 64, W = 64, KS = 15;
  std::mt19937 g(1);
  const size_t act = (size_t)B * H * W * 64;
  float* src = dalloc_rand(act, g, -1.f, 1.f);
  float* X = dalloc_rand(act, g, -1.f, 1.f);
  float* O = dalloc_rand(act, g, -1.f, 1.f);
  float* vecs = dalloc_rand(V_COUNT * 64, g, -0.3f, 0.3f);
  float* wraw = dalloc_rand((size_t)KS * KS * 64 * 64, g, -0.0144f, 0.0144f);
  float* graw = dalloc_rand(64 * 64, g, -0.2f, 0.2f);
  void* wpk;
  CK(hipMalloc(&wpk, (size_t)KS * KS * 16 * 1024));
  f32x4* gpk;
  CK(hipMalloc(&gpk, 1024 * 16));
  const float wscale = 65536.f;   // max|w| 0.0144 -> ~944
  CK(launch_pack_conv64x3(wraw, wpk, KS, wscale, nullptr));
  hipLaunchKernelGGL(pack_gate_kernel, dim3(4), dim3(256), 0, nullptr, graw, gpk);
  const float unscale = 1.f / (wscale * ACT_SCALE);

  const Variant vs[] = {
      {"A nw4 sched0", run_v<EPI_HGRU_A, 4, 0>, 32}, {"A nw4 sched1", run_v<EPI_HGRU_A, 4, 1>, 32},
      {"A nw8 sched0", run_v<EPI_HGRU_A, 8, 0>, 32}, {"A nw8 sched1", run_v<EPI_HGRU_A, 8, 1>, 32},
      {"B nw4 sched0", run_v<EPI_HGRU_B, 4, 0>, 32}, {"B nw4 sched1", run_v<EPI_HGRU_B, 4, 1>, 32},
      {"B nw8 sched0", run_v<EPI_HGRU_B, 8, 0>, 32}, {"B nw8 sched1", run_v<EPI_HGRU_B, 8, 1>, 32},
  };
  const int NV = sizeof(vs) / sizeof(vs[0]);
  std::vector<float*> outs(NV), outs2(NV);
  for (int v = 0; v < NV; ++v) {
    CK(hipMalloc(&outs[v], act * sizeof(float)));
    CK(hipMalloc(&outs2[v], act * sizeof(float)));
  }
  auto args_for = [&](int v) {
    ConvArgs a{};
    a.H = H;
    a.W = W;
    a.src = src;
    a.dst = outs[v];
    a.X = X;
    a.O = O;
    a.I = src;
    a.vecs = vecs;
    a.gpk_or = gpk;
    a.gpk_ir = gpk;
    a.dst2 = outs2[v];
    a.rho = 1.f;
    a.mode = 0;
    return a;
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int v = 0; v < NV; ++v) CK(vs[v].launch(args_for(v), wpk, unscale, B, nullptr));   // warm-up
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> ms(NV);
  const int reps = 3;
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < NV; ++v) {
      CK(hipEventRecord(e0, nullptr));
      for (int k = 0; k < reps; ++k) CK(vs[v].launch(args_for(v), wpk, unscale, B, nullptr));
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / reps);
    }
  const double flop = 2.0 * H * W * KS * KS * 64.0 * 64.0 * B;
  std::vector<float> ref(act), got(act);
  printf("{\"batch\": %d, \"rounds\": %d, \"variants\": [\n", B, rounds);
  for (int v = 0; v < NV; ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const float med = ms[v][ms[v].size() / 2];
    const int base = v < 4 ? 0 : 4;
    CK(hipMemcpy(ref.data(), outs[base], act * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got.data(), outs[v], act * 4, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < act; ++i) md = std::max(md, (double)std::fabs(got[i] - ref[i]));
    printf("  {\"name\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"tflops\": %.1f, \"maxdiff_vs_first\": %.3g}%s\n",
           vs[v].name, med, ms[v][0], flop / (med * 1e-3) / 1e12, md, v + 1 < NV ? "," : "");
  }
  printf("]}\n");
  return 0;
}
