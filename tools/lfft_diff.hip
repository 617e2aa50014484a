// Where the small-batch inverse FFT (lfft_inv_kernel) differs from the batched fft_inv_kernel: both
// on the same Y, prints the differing words by row, column and channel.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Imonkey-pose_amd/csrc tools/lfft_diff.hip -o tools/bin/lfft_diff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <vector>
#include "k_fft.hip"
using namespace mp;
int main() {
  const int B = 1, H = 64, W = 64;
  const size_t nmap = (size_t)B * 64 * H * W;
  std::mt19937 g(1);
  std::vector<float> hy(fft_spec_bytes(B) / 4);
  std::uniform_real_distribution<float> d(-1.f, 1.f);
  for (auto& v : hy) v = d(g);
  void* Y; float *P0, *P1;
  hipMalloc(&Y, fft_spec_bytes(B)); hipMalloc(&P0, nmap * 4); hipMalloc(&P1, nmap * 4);
  hipMemcpy(Y, hy.data(), fft_spec_bytes(B), hipMemcpyHostToDevice);
  hipLaunchKernelGGL((fft_inv_kernel<false, false>), dim3(B * 16), dim3(FNT), 0, 0, Y, P0, H, W);
  hipLaunchKernelGGL(lfft_inv_kernel, dim3(B * 32), dim3(LF_NT), 0, 0, Y, P1, H, W);
  hipDeviceSynchronize();
  std::vector<float> a(nmap), b(nmap);
  hipMemcpy(a.data(), P0, nmap * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), P1, nmap * 4, hipMemcpyDeviceToHost);
  std::vector<int> by_y(64), by_x(64), by_c(64);
  int n = 0; double mx = 0;
  for (int q = 0; q < 8; ++q)
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x)
        for (int e = 0; e < 8; ++e) {
          const size_t i = (((size_t)q * H + y) * W + x) * 8 + e;
          if (a[i] != b[i]) { ++n; by_y[y]++; by_x[x]++; by_c[8 * q + e]++; mx = std::max(mx, (double)std::fabs(a[i] - b[i]) / (std::fabs(a[i]) + 1e-30)); }
        }
  printf("differ %d of %zu, max rel %.3e\nby y:", n, nmap, mx);
  for (int i = 0; i < 64; ++i) printf(" %d", by_y[i]);
  printf("\nby x:"); for (int i = 0; i < 64; ++i) printf(" %d", by_x[i]);
  printf("\nby c:"); for (int i = 0; i < 64; ++i) printf(" %d", by_c[i]);
  printf("\n");
}
