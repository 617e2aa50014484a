// Bit-determinism probe of the FFT-path kernels (k_fft.hip): each kernel runs on a batch of B images
// and again on the images [B0, B) alone (offset pointers, batch B - B0), and twice on the full
// batch; prints the number of differing 32-bit words of each comparison.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Imonkey-pose_amd/csrc \
//         tools/fft_det.hip -o tools/bin/fft_det && tools/bin/fft_det 96 64 [bf16]
#include <hip/hip_runtime.h>

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
static std::vector<uint32_t> fetch(const void* p, size_t bytes) {
  std::vector<uint32_t> h(bytes / 4);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h.data(), p, bytes, hipMemcpyDeviceToHost));
  return h;
}
static size_t ndiff(const std::vector<uint32_t>& a, const std::vector<uint32_t>& b, size_t off) {
  size_t n = 0;
  for (size_t i = 0; i < b.size(); ++i) n += a[off + i] != b[i];
  return n;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 96;
  const int B0 = argc > 2 ? atoi(argv[2]) : 64;
  const bool bf = argc > 3 && !strcmp(argv[3], "bf16");
  const int H = 64, W = 64, KS = 15;
  std::mt19937 g(1);
  const size_t per = (size_t)64 * H * W, nmap = (size_t)B * per;
  const size_t mb = bf && fft_bf16_maps() ? 2 : 4;   // bytes per map element
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
  auto mapoff = [&](const float* p, int b) { return (float*)((char*)p + (size_t)b * per * mb); };
  auto specoff = [&](void* p, int b) { return (void*)((char*)p + fft_spec_bytes(b)); };
  const size_t sb = fft_spec_bytes(B), so = fft_spec_bytes(B0), sn = fft_spec_bytes(B - B0);
  // fft_fwd
  CK(launch_fft_fwd(act, S, B, H, W, 0, bf));
  auto s1 = fetch(S, sb);
  CK(launch_fft_fwd(act, S, B, H, W, 0, bf));
  auto s2 = fetch(S, sb);
  CK(launch_fft_fwd(mapoff(act, B0), specoff(S, B0), B - B0, H, W, 0, bf));
  auto s3 = fetch(specoff(S, B0), sn);
  printf("fft_fwd   rerun %zu  slice %zu\n", ndiff(s1, s2, 0), ndiff(s1, s3, so / 4));
  // spec_gemm (S = the full-batch forward spectra)
  CK(hipMemcpy(S, s1.data(), sb, hipMemcpyHostToDevice));
  CK(launch_spec_gemm(S, Gx, Y, B, unscale, 0, bf));
  auto y1 = fetch(Y, sb);
  CK(launch_spec_gemm(S, Gx, Y, B, unscale, 0, bf));
  auto y2 = fetch(Y, sb);
  CK(launch_spec_gemm(specoff(S, B0), Gx, specoff(Y, B0), B - B0, unscale, 0, bf));
  auto y3 = fetch(specoff(Y, B0), sn);
  printf("spec_gemm rerun %zu  slice %zu\n", ndiff(y1, y2, 0), ndiff(y1, y3, so / 4));
  // fft_inv
  CK(hipMemcpy(Y, y1.data(), sb, hipMemcpyHostToDevice));
  CK(launch_fft_inv(Y, P, B, H, W, 0, bf));
  auto p1 = fetch(P, nmap * mb);
  CK(launch_fft_inv(Y, P, B, H, W, 0, bf));
  auto p2 = fetch(P, nmap * mb);
  CK(launch_fft_inv(specoff(Y, B0), mapoff(P, B0), B - B0, H, W, 0, bf));
  auto p3 = fetch(mapoff(P, B0), (size_t)(B - B0) * per * mb);
  printf("fft_inv   rerun %zu  slice %zu\n", ndiff(p1, p2, 0), ndiff(p1, p3, (size_t)B0 * per * mb / 4));
  // inv_a_fwd: I and S
  ConvArgs a{};
  a.H = H;
  a.W = W;
  a.X = X;
  a.O = O;
  a.dst = I;
  a.vecs = vecs;
  CK(launch_fft_inv_a_fwd(Y, a, S, B, 0, bf));
  auto i1 = fetch(I, nmap * mb);
  auto t1 = fetch(S, sb);
  CK(launch_fft_inv_a_fwd(Y, a, S, B, 0, bf));
  auto i2 = fetch(I, nmap * mb);
  auto t2 = fetch(S, sb);
  ConvArgs a2 = a;
  a2.X = mapoff(X, B0);
  a2.O = mapoff(O, B0);
  a2.dst = mapoff(I, B0);
  CK(launch_fft_inv_a_fwd(specoff(Y, B0), a2, specoff(S, B0), B - B0, 0, bf));
  auto i3 = fetch(mapoff(I, B0), (size_t)(B - B0) * per * mb);
  auto t3 = fetch(specoff(S, B0), sn);
  printf("inv_a_fwd rerun I %zu S %zu  slice I %zu S %zu\n", ndiff(i1, i2, 0), ndiff(t1, t2, 0),
         ndiff(i1, i3, (size_t)B0 * per * mb / 4), ndiff(t1, t3, so / 4));
  // the same four kernels as two concurrent slices [0, B0) and [B0, B) on two streams, 5 times
  hipStream_t sa, sb2;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb2, hipStreamNonBlocking));
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemcpy(Y, y1.data(), sb, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    CK(launch_fft_fwd(act, S, B0, H, W, sa, bf));
    CK(launch_fft_fwd(mapoff(act, B0), specoff(S, B0), B - B0, H, W, sb2, bf));
    CK(launch_fft_inv(Y, P, B0, H, W, sa, bf));
    CK(launch_fft_inv(specoff(Y, B0), mapoff(P, B0), B - B0, H, W, sb2, bf));
    auto c1 = fetch(S, sb);
    auto c2 = fetch(P, nmap * mb);
    CK(launch_spec_gemm(S, Gx, Y, B0, unscale, sa, bf));
    CK(launch_spec_gemm(specoff(S, B0), Gx, specoff(Y, B0), B - B0, unscale, sb2, bf));
    auto c3 = fetch(Y, sb);
    CK(hipMemcpy(Y, y1.data(), sb, hipMemcpyHostToDevice));
    CK(launch_fft_inv_a_fwd(Y, a, S, B0, sa, bf));
    CK(launch_fft_inv_a_fwd(specoff(Y, B0), a2, specoff(S, B0), B - B0, sb2, bf));
    auto c4 = fetch(I, nmap * mb);
    auto c5 = fetch(S, sb);
    printf("concurrent %d: fft_fwd %zu fft_inv %zu spec_gemm %zu inv_a_fwd I %zu S %zu\n", rep, ndiff(s1, c1, 0),
           ndiff(p1, c2, 0), ndiff(y1, c3, 0), ndiff(i1, c4, 0), ndiff(t1, c5, 0));
  }
  // FFT kernels beside MFMA work: inv_a_fwd / fft_inv / fft_fwd on stream a while spec_gemm runs
  // on other buffers on stream b (5 times each)
  void *S2, *Y2;
  CK(hipMalloc(&S2, sb));
  CK(hipMalloc(&Y2, sb));
  CK(hipMemcpy(S2, s1.data(), sb, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemcpy(Y, y1.data(), sb, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    for (int k = 0; k < 4; ++k) CK(launch_spec_gemm(S2, Gx, Y2, B, unscale, sb2, bf));
    CK(launch_fft_inv_a_fwd(Y, a, S, B, sa, bf));
    CK(launch_fft_inv(Y, P, B, H, W, sa, bf));
    auto c4 = fetch(I, nmap * mb);
    auto c5 = fetch(S, sb);
    auto c2 = fetch(P, nmap * mb);
    for (int k = 0; k < 4; ++k) CK(launch_spec_gemm(S2, Gx, Y2, B, unscale, sb2, bf));
    CK(launch_fft_fwd(act, S, B, H, W, sa, bf));
    auto c1 = fetch(S, sb);
    auto g2 = fetch(Y2, sb);
    printf("beside spec_gemm %d: inv_a_fwd I %zu S %zu  fft_inv %zu  fft_fwd %zu  | spec_gemm beside FFT %zu\n", rep,
           ndiff(i1, c4, 0), ndiff(t1, c5, 0), ndiff(p1, c2, 0), ndiff(s1, c1, 0), ndiff(y1, g2, 0));
    // the reverse order: FFT kernels first, the GEMMs (on a private copy of the spectra) beside them
    void* S3;
    CK(hipMalloc(&S3, sb));
    CK(hipMemcpy(S3, s1.data(), sb, hipMemcpyHostToDevice));
    CK(hipMemcpy(Y, y1.data(), sb, hipMemcpyHostToDevice));
    CK(hipMemset(Y2, 0, sb));
    CK(hipDeviceSynchronize());
    for (int k = 0; k < 3; ++k) {
      CK(launch_fft_inv_a_fwd(Y, a, S, B, sa, bf));
      CK(launch_fft_inv(Y, P, B, H, W, sa, bf));
      CK(launch_fft_fwd(act, S, B, H, W, sa, bf));
    }
    for (int k = 0; k < 6; ++k) CK(launch_spec_gemm(S3, Gx, Y2, B, unscale, sb2, bf));
    auto g3 = fetch(Y2, sb);
    CK(hipFree(S3));
    const auto& g4 = y1;
    printf("   spec_gemm launched behind FFT kernels vs alone: %zu words differ\n", ndiff(g4, g3, 0));
  }
  return 0;
}
