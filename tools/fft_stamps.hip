// Phase timing of the FFT-path kernels (k_fft.hip built with FFT_STAMP): thread 0 of every block
// records s_memtime at the phase boundaries; this prints, per kernel, the mean / median cycles of
// each phase, the mean block lifetime, the resident blocks per CU implied by lifetime x blocks /
// (kernel cycles x CUs), and the kernel time.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DFFT_STAMP -Imonkey-pose_amd/csrc \
//         tools/fft_stamps.hip -o tools/bin/fft_stamps && tools/bin/fft_stamps 256 [bf16]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static float* dalloc_rand(size_t n, std::mt19937& g, float lo, float hi) {
  std::vector<float> h(n);
  std::uniform_real_distribution<float> d(lo, hi);
  for (auto& v : h) v = d(g);
  float* p;
  CK(hipMalloc(&p, n * sizeof(float)));
  CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return p;
}

static void report(const char* name, int nblk, const std::vector<int>& marks, float ms) {
#ifndef FFT_STAMP
  (void)nblk;
  (void)marks;
  printf("%-10s %.4f ms\n", name, ms);
#else
  std::vector<unsigned long long> st(16384 * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(fft_stamp_buf), st.size() * sizeof(unsigned long long)));
  unsigned long long t0 = ~0ull, t1 = 0;
  double life = 0;
  for (int b = 0; b < nblk; ++b) {
    t0 = std::min(t0, st[b * 8 + marks.front()]);
    t1 = std::max(t1, st[b * 8 + marks.back()]);
    life += (double)(st[b * 8 + marks.back()] - st[b * 8 + marks.front()]);
  }
  life /= nblk;
  const double span = (double)(t1 - t0);
  printf("%-10s %.4f ms  span %.0f cyc (%.2f GHz)  block life %.0f cyc  resident/CU %.2f  phases:", name, ms, span,
         span / (ms * 1e6), life, life * nblk / (span * 256));
  for (size_t k = 1; k < marks.size(); ++k) {
    std::vector<double> d(nblk);
    for (int b = 0; b < nblk; ++b) d[b] = (double)(st[b * 8 + marks[k]] - st[b * 8 + marks[k - 1]]);
    std::sort(d.begin(), d.end());
    double m = 0;
    for (double x : d) m += x;
    printf("  [%d->%d] mean %.0f med %.0f", marks[k - 1], marks[k], m / nblk, d[nblk / 2]);
  }
  printf("\n");
#endif
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256;
  const bool bf = argc > 2 && !strcmp(argv[2], "bf16");
  const int H = 64, W = 64, KS = 15;
  std::mt19937 g(1);
  const size_t nmap = (size_t)B * 64 * H * W;
  float* act = dalloc_rand(nmap, g, -1.f, 1.f);
  float* w = dalloc_rand((size_t)KS * KS * 64 * 64, g, -0.02f, 0.02f);
  void *S, *Y, *Gx;
  float* P;
  CK(hipMalloc(&S, fft_spec_bytes(B)));
  CK(hipMalloc(&Y, fft_spec_bytes(B)));
  CK(hipMalloc(&Gx, fft_weight_bytes()));
  CK(hipMalloc(&P, nmap * sizeof(float)));
  float unscale = 0.f;
  CK(build_spec_weights(w, KS, Gx, &unscale, bf));
  float* X = dalloc_rand(nmap, g, -1.f, 1.f);
  float* O = dalloc_rand(nmap, g, -1.f, 1.f);
  float* I;
  CK(hipMalloc(&I, nmap * sizeof(float)));
  float* vecs = dalloc_rand(V_COUNT * 64, g, 0.5f, 1.f);
  ConvArgs a{};
  a.H = H;
  a.W = W;
  a.X = X;
  a.O = O;
  a.dst = I;
  a.vecs = vecs;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto f) {   // median of 21 single-launch event timings (the stamps: the last launch)
    for (int i = 0; i < 3; ++i) CK(f());
    std::vector<float> t;
    for (int r = 0; r < 21; ++r) {
      CK(hipEventRecord(e0, 0));
      CK(f());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  const bool lf = !bf && B <= lfft_maxb();   // the small-batch kernels (k_fft.hip lfft_*): 32 blocks per image
  const int nblk = B * (lf ? 32 : 16);
  float ms = timed([&] { return launch_fft_fwd(act, S, B, H, W, 0, bf); });
  if (lf) printf("fft_fwd    %.4f ms (lfft, no stamps)\n", ms);
  else report("fft_fwd", nblk, {0, 1, 5}, ms);
  ms = timed([&] { return launch_spec_gemm(S, Gx, Y, B, unscale, 0, bf); });
  printf("spec_gemm  %.4f ms\n", ms);
  ms = timed([&] { return launch_fft_inv(Y, P, B, H, W, 0, bf); });
  if (lf) printf("fft_inv    %.4f ms (lfft, no stamps)\n", ms);
  else report("fft_inv", nblk, {0, 1, 2, 5}, ms);
  ms = timed([&] { return launch_fft_inv_a_fwd(Y, a, S, B, 0, bf); });
  // lfft: 0 start, 1 Y in LDS, 2 inverse columns, 3 inverse rows, 4 epilogue, 5 forward rows,
  // 6 forward columns + S staging, 7 S stored
  if (lf) report("inv_a_fwd", nblk, {0, 1, 2, 3, 4, 5, 6, 7}, ms);
  else report("inv_a_fwd", nblk, {0, 1, 2, 3, 4, 5}, ms);
  return 0;
}
