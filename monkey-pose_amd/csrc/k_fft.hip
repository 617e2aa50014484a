// FFT path of the hGRU association-field convolution (MP_DTYPE_F32_FFT).
//
// The eCRF convolution of hgru_module.py:657 / 735 (tf.nn.conv2d, SAME, 15x15 taps, 64 -> 64
// channels) on a 64x64 map is a 2-D circular convolution on any grid N >= H + R (R = taps / 2):
// the wrapped tail [H, N) of the zero-padded input is zero, so no output in [0, H) sees wrap-around.
// With N = 72 the per-pixel work drops from 15*15*64*64 real MACs to 64*64 complex MACs per
// frequency (72*37 frequencies for 64*64 pixels) plus two 72-point FFT passes, ~50x fewer FLOPs.
//
//   fft_fwd   act (C8)          -> S[b][cq][f][4]    2-D real FFT per (image, 4-channel group)
//   spec_gemm S, G              -> Y[b][cq][f][4]    per frequency: Y[b][co] = sum_ci S[b][ci] G[ci][co]
//   fft_inv   Y                 -> P (C8)            2-D inverse (complex-to-real) FFT
//   spec_epi  P (+ X, O, I ...) -> the fused hGRU epilogue of conv_epi.hpp, unchanged
//
// G[f][ci][co] = (1/N^2) sum_{ky,kx} w[ky][kx][ci][co] exp(-2 pi i (fy (R-ky) + fx (R-kx)) / N)
// (cross-correlation written as a convolution with the flipped kernel, inverse-DFT scale folded in)
// is computed once per weight set in double precision.  Every stage is fp32 (FFT butterflies with
// fp32 twiddles rounded once from double; the spectral GEMM on v_mfma_f32_32x32x2_f32), so the
// path is fp32-class: error ~1e-6 of max|output| against the float64 oracle.
//
// Frequencies: f = fx * 72 + fy, fy in [0, 72), fx in [0, 37) (the real-input half spectrum), so
// the 72 values one FFT thread writes / reads sit at a 32-byte stride (immediate offsets).
// Spectra are stored [b][cq][f][c] (complex, c = channel % 4, cq = channel / 4): every FFT block
// reads / writes one contiguous 85 KiB run, and a spectral-GEMM lane reads one float4 per group.
#include "conv_epi.hpp"
#include "fft_consts.hpp"

namespace mp {

constexpr int FX = FFT_N / 2 + 1;      // 37
constexpr int NF = FFT_N * FX;         // 2664 frequencies

struct cpx {
  float x, y;
};
__device__ __forceinline__ cpx operator+(cpx a, cpx b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cpx operator-(cpx a, cpx b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cpx scale(cpx a, float s) { return {a.x * s, a.y * s}; }
// a * e^{S i 2 pi m / 72}  (S = -1 forward, +1 inverse)
template <int S>
__device__ __forceinline__ cpx twid(cpx a, int m) {
  const float c = TW72_COS[m], s = S * TW72_SIN[m];
  return {a.x * c - a.y * s, a.x * s + a.y * c};
}
// a * e^{S i pi / 2}
template <int S>
__device__ __forceinline__ cpx rotq(cpx a) {
  return {-S * a.y, S * a.x};
}

template <int S>
__device__ __forceinline__ void dft8(cpx (&x)[8]) {
  constexpr float H = 0.70710678118654752f;
  const cpx a0 = x[0] + x[4], a1 = x[0] - x[4], a2 = x[2] + x[6], a3 = rotq<S>(x[2] - x[6]);
  const cpx a4 = x[1] + x[5], a5 = x[1] - x[5], a6 = x[3] + x[7], a7 = rotq<S>(x[3] - x[7]);
  const cpx b0 = a0 + a2, b2 = a0 - a2, b1 = a1 + a3, b3 = a1 - a3;
  const cpx b4 = a4 + a6, b6 = a4 - a6, b5 = a5 + a7, b7 = a5 - a7;
  const cpx t6 = rotq<S>(b6);
  const cpx t5 = {H * (b5.x - S * b5.y), H * (S * b5.x + b5.y)};      // b5 * W8^1
  const cpx t7 = {-H * (b7.x + S * b7.y), H * (S * b7.x - b7.y)};     // b7 * W8^3
  x[0] = b0 + b4;
  x[4] = b0 - b4;
  x[2] = b2 + t6;
  x[6] = b2 - t6;
  x[1] = b1 + t5;
  x[5] = b1 - t5;
  x[3] = b3 + t7;
  x[7] = b3 - t7;
}

template <int S>
__device__ __forceinline__ void dft3(cpx& z0, cpx& z1, cpx& z2) {
  constexpr float R3 = 0.86602540378443865f;
  const cpx t = z1 + z2, d = z1 - z2;
  const cpx m = z0 - scale(t, 0.5f);
  const cpx s = {-S * R3 * d.y, S * R3 * d.x};
  z0 = z0 + t;
  z1 = m + s;
  z2 = m - s;
}

// 9-point DFT as 3 x 3 (n = 3a + b, k = c + 3d)
template <int S>
__device__ __forceinline__ void dft9(cpx (&x)[9]) {
  cpx y[3][3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    cpx z0 = x[b], z1 = x[3 + b], z2 = x[6 + b];
    dft3<S>(z0, z1, z2);
    y[b][0] = z0;
    y[b][1] = twid<S>(z1, 8 * b);        // W9^{b c} = W72^{8 b c}
    y[b][2] = twid<S>(z2, 16 * b);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    cpx z0 = y[0][c], z1 = y[1][c], z2 = y[2][c];
    dft3<S>(z0, z1, z2);
    x[c] = z0;
    x[c + 3] = z1;
    x[c + 6] = z2;
  }
}

// in-register 72-point DFT, X[k] = sum_n v[n] e^{S 2 pi i n k / 72} (unnormalised);
// 72 = 8 x 9: n = 9 n1 + n2, k = k1 + 8 k2
template <int S>
__device__ __forceinline__ void fft72(cpx (&v)[72]) {
  cpx a[9][8];
#pragma unroll
  for (int n2 = 0; n2 < 9; ++n2) {
    cpx t[8];
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) t[n1] = v[9 * n1 + n2];
    dft8<S>(t);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) a[n2][k1] = (n2 * k1 == 0) ? t[k1] : twid<S>(t[k1], n2 * k1);
  }
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) {
    cpx u[9];
#pragma unroll
    for (int n2 = 0; n2 < 9; ++n2) u[n2] = a[n2][k1];
    dft9<S>(u);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) v[k1 + 8 * k2] = u[k2];
  }
}

// ---------------------------------------------------------------------------------------------
// forward 2-D FFT: one block per (image b, channel group cq); 192 threads.
//   phase 1 (128 threads): row y, channel pair p: the two real rows packed as one complex FFT,
//            then separated into their half spectra (fx = 0..36) -> LDS T[fx][c][y]
//   phase 2 (148 threads): column (fx, c): 72-point FFT over y -> S[b][cq][fx*72+fy][c]
constexpr int FWD_LD = 65;    // LDS row pitch (complex) of T: conflict-free column reads
__global__ __launch_bounds__(192, 2) void fft_fwd_kernel(const float* __restrict__ src, cpx* __restrict__ S,
                                                      int H, int W) {
  __shared__ cpx T[FX * 4 * FWD_LD];
  const int cq = blockIdx.x & 15, b = blockIdx.x >> 4;
  const int q = cq >> 1, e0 = 4 * (cq & 1);
  const int tid = threadIdx.x;
  if (tid < 128) {
    const int y = tid >> 1, p = tid & 1;
    cpx v[72];
    const float* row = src + c8_index(b, q, y < H ? y : 0, 0, e0 + 2 * p, H, W);
#pragma unroll
    for (int x = 0; x < 72; ++x) {
      if (x < 64 && y < H && x < W) {
        const float2 t = *reinterpret_cast<const float2*>(row + 8 * x);
        v[x] = {t.x, t.y};
      } else {
        v[x] = {0.f, 0.f};
      }
    }
    fft72<-1>(v);
    // Z = FFT(a + i b):  A[k] = (Z[k] + conj Z[-k]) / 2,  B[k] = (Z[k] - conj Z[-k]) / (2i)
#pragma unroll
    for (int k = 0; k < FX; ++k) {
      const cpx zk = v[k], zm = v[(72 - k) % 72];
      const cpx A = {0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y)};
      const cpx B = {0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x)};
      T[(k * 4 + 2 * p) * FWD_LD + y] = A;
      T[(k * 4 + 2 * p + 1) * FWD_LD + y] = B;
    }
  }
  __syncthreads();
  if (tid < FX * 4) {
    const int fx = tid >> 2, c = tid & 3;
    cpx v[72];
#pragma unroll
    for (int y = 0; y < 72; ++y) v[y] = y < 64 ? T[tid * FWD_LD + y] : cpx{0.f, 0.f};
    fft72<-1>(v);
    cpx* dst = S + (((size_t)b * 16 + cq) * NF + fx * 72) * 4 + c;
#pragma unroll
    for (int fy = 0; fy < 72; ++fy) dst[fy * 4] = v[fy];
  }
}

// ---------------------------------------------------------------------------------------------
// inverse 2-D FFT (complex-to-real): one block per (image b, channel group cq); 192 threads.
//   phase 1 (148 threads): column (fx, c): inverse 72-point FFT over fy, rows y < H -> LDS
//   phase 2 (128 threads): row y, channel pair p: the Hermitian-extended half spectra of the two
//            real rows packed as C = A + iB, one inverse FFT, real / imaginary parts = the rows
__global__ __launch_bounds__(192, 2) void fft_inv_kernel(const cpx* __restrict__ Y, float* __restrict__ P,
                                                      int H, int W) {
  __shared__ cpx T[64 * 4 * FX];   // [y][c][fx]
  const int cq = blockIdx.x & 15, b = blockIdx.x >> 4;
  const int q = cq >> 1, e0 = 4 * (cq & 1);
  const int tid = threadIdx.x;
  if (tid < FX * 4) {
    const int fx = tid >> 2, c = tid & 3;
    const cpx* src = Y + (((size_t)b * 16 + cq) * NF + fx * 72) * 4 + c;
    cpx v[72];
#pragma unroll
    for (int fy = 0; fy < 72; ++fy) v[fy] = src[fy * 4];
    fft72<1>(v);
#pragma unroll
    for (int y = 0; y < 64; ++y) T[(y * 4 + c) * FX + fx] = v[y];   // rows >= H: unused
  }
  __syncthreads();
  if (tid < 128) {
    const int y = tid >> 1, p = tid & 1;
    if (y < H) {
      const cpx* ta = T + (y * 4 + 2 * p) * FX;
      const cpx* tb = ta + FX;
      cpx v[72];
#pragma unroll
      for (int k = 0; k < FX; ++k) {   // C[k] = A[k] + i B[k];  C[72-k] from A[72-k] = conj A[k] etc.
        const cpx A = ta[k], B = tb[k];
        v[k] = {A.x - B.y, A.y + B.x};
        if (k > 0 && k < FX - 1) v[72 - k] = {A.x + B.y, B.x - A.y};
      }
      fft72<1>(v);
      float* row = P + c8_index(b, q, y, 0, e0 + 2 * p, H, W);
#pragma unroll
      for (int x = 0; x < 32; ++x) *reinterpret_cast<float2*>(row + 8 * x) = make_float2(v[x].x, v[x].y);
      if (W > 32) {   // W is 32 or 64 (uniform branch; per-x predicates double the live registers)
#pragma unroll
        for (int x = 32; x < 64; ++x) *reinterpret_cast<float2*>(row + 8 * x) = make_float2(v[x].x, v[x].y);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// spectral GEMM: per frequency f, Y[b][co] = sum_ci S[b][ci] G[ci][co] (complex), as one real
// 128 x 128 x 128 product D[n][b] = sum_k A[n][k] Bm[k][b] on v_mfma_f32_32x32x2_f32:
//   n = 2 co + (re|im),  k-step s / lane half h  <->  input channel ci = 4 (s>>2) + 2h + ((s&3)>>1),
//   part (s & 1): each lane's four consecutive k-steps are one float4 of its S group, and each
//   lane's four accumulator rows 4h..4h+3 of a row group are one float4 of its Y group.
// A (the expanded spectral weights of f, 64 KiB, fragment order [s][lane][mb]) is staged in LDS;
// a block = NWV waves x 32 images, blocks of one frequency adjacent in launch order.
template <int NWV>
__global__ __launch_bounds__(NWV * 64, 2) void spec_gemm_kernel(const f32x4* __restrict__ S,
                                                                const f32x4* __restrict__ Gx,
                                                                f32x4* __restrict__ Y, int B, int groups) {
  __shared__ f32x4 wl[64 * 64];
  const int f = blockIdx.x / groups, grp = blockIdx.x - f * groups;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5;
  const f32x4* gsrc = Gx + (size_t)f * 4096;
#pragma unroll
  for (int i = 0; i < 4096 / (NWV * 64); ++i) wl[i * NWV * 64 + tid] = gsrc[i * NWV * 64 + tid];
  const int b = (grp * NWV + wv) * 32 + (lane & 31);
  const bool live = b < B;
  f32x4 sv[16];
#pragma unroll
  for (int cq = 0; cq < 16; ++cq)
    sv[cq] = live ? S[(((size_t)b * 16 + cq) * NF + f) * 2 + h] : f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  f32x16 acc[4] = {};
#pragma unroll 8
  for (int s = 0; s < 64; ++s) {
    const f32x4 a = wl[s * 64 + lane];
    const float bv = sv[s >> 2][s & 3];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc[mb] = mfma32(a[mb], bv, acc[mb]);
  }
  if (live) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        Y[(((size_t)b * 16 + 4 * mb + g) * NF + f) * 2 + h] =
            f32x4{acc[mb][4 * g], acc[mb][4 * g + 1], acc[mb][4 * g + 2], acc[mb][4 * g + 3]};
  }
}

// spectral weights, once per weight set: one thread per (f, ci, co), float64 accumulation
__global__ void spec_weights_kernel(const float* __restrict__ w, float* __restrict__ Gx, int KS) {
  __shared__ double tc[FFT_N], ts[FFT_N];
  for (int m = threadIdx.x; m < FFT_N; m += blockDim.x) {
    double s, c;
    sincospi(2.0 * m / FFT_N, &s, &c);
    tc[m] = c;
    ts[m] = s;
  }
  __syncthreads();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NF * 4096) return;
  const int co = idx & 63, ci = (idx >> 6) & 63, f = idx >> 12;
  const int fx = f / FFT_N, fy = f - fx * FFT_N, R = KS / 2;
  double gr = 0.0, gi = 0.0;
  for (int ky = 0; ky < KS; ++ky)
    for (int kx = 0; kx < KS; ++kx) {
      const double v = w[((size_t)(ky * KS + kx) * 64 + ci) * 64 + co];
      int m = (fy * (R - ky) + fx * (R - kx)) % FFT_N;
      if (m < 0) m += FFT_N;
      gr += v * tc[m];      // exp(-i theta) = cos - i sin
      gi -= v * ts[m];
    }
  const double inv = 1.0 / ((double)FFT_N * FFT_N);
  const float vr = (float)(gr * inv), vi = (float)(gi * inv);
  // expanded real form: A[(co, ro)][(ci, ri)] = ro == ri ? gr : (ro == 0 ? -gi : gi)
  const int c = ci & 3, hh = c >> 1, s0 = 4 * (ci >> 2) + 2 * (c & 1);
#pragma unroll
  for (int ro = 0; ro < 2; ++ro)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int n = 2 * co + ro, s = s0 + ri, lane = 32 * hh + (n & 31), mb = n >> 5;
      Gx[(((size_t)f * 64 + s) * 64 + lane) * 4 + mb] = ro == ri ? vr : (ro == 0 ? -vi : vi);
    }
}

// the fused epilogue on the spatial result P: one wave per 32-pixel row segment, P loaded in the
// v_mfma 32x32 accumulator layout conv_epilogue expects (cout 32n + 8g + 4h + j at lane col x)
template <int EPI>
__global__ __launch_bounds__(256) void spec_epi_kernel(ConvArgs p, const float* __restrict__ P, int nseg) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= nseg) return;
  const int xs = p.W / 32;
  const int x = (seg % xs) * 32 + (lane & 31);
  const int y = (seg / xs) % p.H, b = seg / xs / p.H;
  f32x16 acc[2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(P + c8_index(b, 4 * n + g, y, x, 4 * h, p.H, p.W));
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[n][4 * g + j] = v[j];
    }
  conv_epilogue<EPI>(p, acc[0], acc[1], b, y, x, h, lane, 1.0f);
}

// ------------------------------------------------------------------------------------ launchers
size_t fft_spec_bytes(int B) { return (size_t)B * 16 * NF * 4 * sizeof(cpx); }
size_t fft_weight_bytes() { return (size_t)NF * 4096 * 4 * sizeof(float); }

hipError_t launch_spec_weights(const float* w, float* Gx, int ks, hipStream_t st) {
  const int total = NF * 4096;
  hipLaunchKernelGGL(spec_weights_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, Gx, ks);
  return hipGetLastError();
}

hipError_t launch_fft_fwd(const float* act, void* S, int B, int H, int W, hipStream_t st) {
  hipLaunchKernelGGL(fft_fwd_kernel, dim3(B * 16), dim3(192), 0, st, act, static_cast<cpx*>(S), H, W);
  return hipGetLastError();
}

hipError_t launch_spec_gemm(const void* S, const float* Gx, void* Y, int B, hipStream_t st) {
  constexpr int NWV = 4;
  const int groups = (B + 32 * NWV - 1) / (32 * NWV);
  hipLaunchKernelGGL((spec_gemm_kernel<NWV>), dim3(NF * groups), dim3(NWV * 64), 0, st,
                     static_cast<const f32x4*>(S), reinterpret_cast<const f32x4*>(Gx), static_cast<f32x4*>(Y),
                     B, groups);
  return hipGetLastError();
}

hipError_t launch_fft_inv(const void* Y, float* P, int B, int H, int W, hipStream_t st) {
  hipLaunchKernelGGL(fft_inv_kernel, dim3(B * 16), dim3(192), 0, st, static_cast<const cpx*>(Y), P, H, W);
  return hipGetLastError();
}

hipError_t launch_spec_epi(int epi, const ConvArgs& a, const float* P, int B, hipStream_t st) {
  const int nseg = B * a.H * (a.W / 32);
  if (epi == EPI_HGRU_A)
    hipLaunchKernelGGL((spec_epi_kernel<EPI_HGRU_A>), dim3((nseg + 3) / 4), dim3(256), 0, st, a, P, nseg);
  else if (epi == EPI_HGRU_B)
    hipLaunchKernelGGL((spec_epi_kernel<EPI_HGRU_B>), dim3((nseg + 3) / 4), dim3(256), 0, st, a, P, nseg);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace mp
