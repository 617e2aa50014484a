// fp32-accurate 64->64 SAME convolution on f16 matrix cores ("f16x3" split precision), with the
// same fused hGRU / backbone epilogues as the exact-fp32 kernel (conv_epi.hpp).
//
// Every fp32 operand v is split into two f16 values, hi = f16(s*v) and lo = f16(s*v - hi), with a
// power-of-two scale s (weights: per tensor, chosen at finalize so max|w|*s is ~2^14; activations:
// 2^10).  hi+lo carries 22 mantissa bits, and because s is a power of two the residual error of a
// flushed or subnormal lo is below 2^-24 in unscaled units.  Each product is then
//   w*a ~= hi_w*hi_a + hi_w*lo_a + lo_w*hi_a       (the lo*lo term is < 2^-22 relative)
// = three v_mfma_f32_32x32x16_f16 (exact products, fp32 accumulation), 3/16 of the issue cycles of
// the v_mfma_f32_32x32x2_f32 path for the same FLOPs.  The result is unscaled by 1/(s_w*s_a)
// (exact) before the epilogue.
//
// Geometry: one 256-thread block (4 waves, 1 block per CU, up to 512 VGPR+AGPR per lane) owns a
// 32x32-pixel tile of one image; wave w owns rows 8w..8w+7 (8 M-blocks of 32 pixels) x all 64
// output channels (2 N-blocks) = 16 32x32 accumulators (256 AGPRs).  The input halo
// ((32+KS-1)^2 pixels) of one 16-channel chunk is staged in LDS as f16 [row][plane][col] cells of
// 8 channels (planes: hi c0-7, hi c8-15, lo c0-7, lo c8-15), so each B fragment is one
// conflict-free ds_read_b128 of 32 consecutive cells.  Weights stream from L2 pre-split and
// pre-packed in fragment order (two 16-byte loads per lane per tap per 32 output channels).
#include "conv_epi.hpp"

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace mp {

constexpr float ACT_SCALE = 1024.0f;     // 2^10

__device__ __forceinline__ f32x16 mfma16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int KS, int EPI>
__global__ __launch_bounds__(256, 1) void conv64x3_kernel(ConvArgs p, const f16x8* __restrict__ wpk,
                                                          float unscale) {
  constexpr int R = KS / 2;
  constexpr int HY = TH3 + KS - 1, HX = TW + KS - 1;
  constexpr int KK = KS * KS;
  constexpr int NQ16 = 4;                // 16-channel chunks
  __shared__ f16x8 halo[HY * 4 * HX];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int H = p.H, W = p.W;
  int bid = blockIdx.x;
  const int tx = bid % p.tiles_x;
  bid /= p.tiles_x;
  const int ty = bid % p.tiles_y;
  const int b = bid / p.tiles_y;
  const int y0 = ty * TH3, x0 = tx * TW;

  f32x16 acc[2][8];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[n][m] = f32x16{};

  for (int Q = 0; Q < NQ16; ++Q) {
    __syncthreads();
    // ---- stage + split the 16-channel halo chunk (zero outside the image = SAME padding) ----
    for (int it = tid; it < HY * HX * 2; it += 256) {
      const int hh = it & 1;
      const int pix = it >> 1;
      const int hy = pix / HX, hx = pix - hy * HX;
      const int gy = y0 + hy - R, gx = x0 + hx - R;
      f16x8 vh = {}, vl = {};
      if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
        const f32x4* src = reinterpret_cast<const f32x4*>(p.src + c8_index(b, 2 * Q + hh, gy, gx, 0, H, W));
        const f32x4 a0 = src[0], a1 = src[1];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = (j < 4 ? a0[j] : a1[j - 4]) * ACT_SCALE;
          const _Float16 hi = (_Float16)v;
          vh[j] = hi;
          vl[j] = (_Float16)(v - (float)hi);
        }
      }
      halo[(hy * 4 + hh) * HX + hx] = vh;
      halo[(hy * 4 + 2 + hh) * HX + hx] = vl;
    }
    __syncthreads();

    // software pipeline, one tap ahead: the next tap's 4 weight fragments (L2) and 16 halo
    // fragments (LDS) are in flight while this tap's 48 MFMAs issue (1 wave per SIMD here).
    const f16x8* wt = wpk + (size_t)Q * KK * 4 * 64 + lane;
    const f16x8* hb = halo + ((wv * 8) * 4 + h) * HX + col;
    f16x8 w[4], bh[8], bl[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = wt[i * 64];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      bh[m] = hb[m * 4 * HX];
      bl[m] = hb[m * 4 * HX + 2 * HX];
    }
    int ky = 0, kx = 0;
    for (int tap = 0; tap < KK; ++tap) {
      f16x8 cw[4], ch[8], cl[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) cw[i] = w[i];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        ch[m] = bh[m];
        cl[m] = bl[m];
      }
      if (++kx == KS) {
        kx = 0;
        ++ky;
      }
      if (tap + 1 < KK) {
        wt += 4 * 64;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = wt[i * 64];
        const f16x8* hn = hb + ky * 4 * HX + kx;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          bh[m] = hn[m * 4 * HX];
          bl[m] = hn[m * 4 * HX + 2 * HX];
        }
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        acc[0][m] = mfma16(cw[0], cl[m], acc[0][m]);
        acc[1][m] = mfma16(cw[2], cl[m], acc[1][m]);
        acc[0][m] = mfma16(cw[1], ch[m], acc[0][m]);
        acc[1][m] = mfma16(cw[3], ch[m], acc[1][m]);
        acc[0][m] = mfma16(cw[0], ch[m], acc[0][m]);
        acc[1][m] = mfma16(cw[2], ch[m], acc[1][m]);
      }
    }
  }

  const int x = x0 + col;
#pragma unroll
  for (int m = 0; m < 8; ++m) conv_epilogue<EPI>(p, acc[0][m], acc[1][m], b, y0 + wv * 8 + m, x, h, lane, unscale);
}

// HWIO [KS][KS][64][64] fp32 -> [Q][tap][n][hi|lo][lane] f16x8:
//   element j = split(W[tap][16Q+8h+j][32n+(lane&31)] * wscale), h = lane>>5
__global__ void pack_conv64x3_kernel(const float* __restrict__ w, f16x8* out, int KK, float wscale) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int total = 4 * KK * 2 * 64;
  if (i >= total) return;
  const int lane = i % 64, n = (i / 64) % 2, tap = (i / 128) % KK, Q = i / (128 * KK);
  const int co = 32 * n + (lane & 31);
  const int ci0 = 16 * Q + 8 * (lane >> 5);
  f16x8 hv, lv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = w[((size_t)tap * 64 + ci0 + j) * 64 + co] * wscale;
    const _Float16 hi = (_Float16)v;
    hv[j] = hi;
    lv[j] = (_Float16)(v - (float)hi);
  }
  f16x8* dst = out + (((size_t)Q * KK + tap) * 2 + n) * 2 * 64 + lane;
  dst[0] = hv;
  dst[64] = lv;
}

template <int KS, int EPI>
static hipError_t launch_x3_t(const ConvArgs& a, const void* wpk, float unscale, int B, hipStream_t st) {
  const int nblk = B * a.tiles_x * a.tiles_y;
  hipLaunchKernelGGL((conv64x3_kernel<KS, EPI>), dim3(nblk), dim3(256), 0, st, a,
                     static_cast<const f16x8*>(wpk), unscale);
  return hipGetLastError();
}

hipError_t launch_conv64x3(int ks, int epi, ConvArgs a, const void* wpk, float unscale, int B, hipStream_t st) {
  a.tiles_x = a.W / TW;
  a.tiles_y = a.H / TH3;
#define MP_CASE(K, E) \
  if (ks == K && epi == E) return launch_x3_t<K, E>(a, wpk, unscale, B, st);
  MP_CASE(15, EPI_HGRU_A)
  MP_CASE(15, EPI_HGRU_B)
  MP_CASE(5, EPI_HGRU_A)
  MP_CASE(5, EPI_HGRU_B)
  MP_CASE(3, EPI_HGRU_A)
  MP_CASE(3, EPI_HGRU_B)
#undef MP_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_pack_conv64x3(const float* w, void* out, int ks, float wscale, hipStream_t st) {
  const int total = 4 * ks * ks * 2 * 64;
  hipLaunchKernelGGL(pack_conv64x3_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w,
                     static_cast<f16x8*>(out), ks * ks, wscale);
  return hipGetLastError();
}

}  // namespace mp
