// 64->64-channel SAME convolutions on the C8 layout, with the hGRU half-step epilogues fused.
//
// Reference ops replaced (all /root/reference):
//   hgru_module.py:531-535/544-548  tf.nn.conv2d(data, p_r [15,15,64,64], SAME)  (p_convolution 615)
//   hgru_module.py:696-707/729-740  1x1 gate convs i_r / o_r + bias + sigmoid
//   hgru_module.py:795-823          input/output integration (tanh mixes), 847-849 rho
//   hgru_pose.py:139-154 + 62-80    conv_2 / conv_3 (3x3 + bias + relu) + folded inference BN
//
// Implicit GEMM per block: D[cout 64][pixel 512] = sum over (tap, cin) of W^T[cout][k] * In[k][pixel]
// on v_mfma_f32_32x32x2_f32 (exact fp32).  A block owns a 16x32 pixel tile of one image; its
// input halo ((16+KS-1) x (32+KS-1) pixels) is staged in LDS one 8-channel chunk at a time as
// [halo_row][half h][halo_col] float4 cells, so lanes 0-31 / 32-63 of a ds_read_b128 read 32
// consecutive cells (conflict-free for every tap shift).  Weights stream from L2 pre-packed in
// MFMA-fragment order (one 16-byte load per lane per tap per 32 output channels).
#include "conv_epi.hpp"

namespace mp {


template <int KS, int EPI>
__global__ __launch_bounds__(256, 2) void conv64_kernel(ConvArgs p) {
  constexpr int R = KS / 2;
  constexpr int HY = TH + KS - 1, HX = TW + KS - 1;
  constexpr int NCELL = HY * 2 * HX;
  constexpr int KK = KS * KS;
  __shared__ f32x4 halo[NCELL];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int H = p.H, W = p.W;
  int bid = blockIdx.x;
  const int tx = bid % p.tiles_x; bid /= p.tiles_x;
  const int ty = bid % p.tiles_y;
  const int b = bid / p.tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;

  f32x16 acc[2][4];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[n][m] = f32x16{};

  for (int q = 0; q < NQ; ++q) {
    __syncthreads();
    // ---- stage the 8-channel halo chunk (zero outside the image = SAME padding) ----
    for (int cell = tid; cell < NCELL; cell += 256) {
      const int hy = cell / (2 * HX);
      const int rem = cell - hy * (2 * HX);
      const int hh = rem / HX;
      const int hx = rem - hh * HX;
      const int gy = y0 + hy - R, gx = x0 + hx - R;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (gy >= 0 && gy < H && gx >= 0 && gx < W)
        v = *reinterpret_cast<const f32x4*>(p.src + c8_index(b, q, gy, gx, 4 * hh, H, W));
      halo[cell] = v;
    }
    __syncthreads();

    const f32x4* wq = p.wpk + (size_t)q * KK * 2 * 64 + lane;
    for (int ky = 0; ky < KS; ++ky) {
      const f32x4* hrow = halo + ((wv * 4 + ky) * 2 + h) * HX + col;
#pragma unroll 3
      for (int kx = 0; kx < KS; ++kx) {
        const int tap = ky * KS + kx;
        const f32x4 w0 = wq[(tap * 2 + 0) * 64];
        const f32x4 w1 = wq[(tap * 2 + 1) * 64];
        f32x4 a[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = hrow[m * 2 * HX + kx];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            acc[0][m] = mfma32(w0[s], a[m][s], acc[0][m]);
            acc[1][m] = mfma32(w1[s], a[m][s], acc[1][m]);
          }
      }
    }
  }

  // ------------------------------------ epilogues ------------------------------------------
  const int x = x0 + col;
#pragma unroll
  for (int m = 0; m < 4; ++m) conv_epilogue<EPI>(p, acc[0][m], acc[1][m], b, y0 + wv * 4 + m, x, h, lane, 1.0f);
}

// ---------------------------------------------------------------------------------------------
// hidden-state init: O (C8) <- O0 (NHWC), Og = O0 * sigmoid(O0 . i_r + i_b)
// (the first circuit_input, hgru_module.py:696-711).  One wave = 32 consecutive pixels.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gate_init_kernel(const float* __restrict__ O0, float* O,
                                                        float* Og, const f32x4* __restrict__ gpk_ir,
                                                        const float* __restrict__ vecs, int npix,
                                                        int H, int W) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int pix = blk * 32 + (lane & 31);
  if (blk * 32 >= npix) return;
  const bool ok = pix < npix;
  const int pp = ok ? pix : npix - 1;
  const int x = pp % W, y = (pp / W) % H, b = pp / (W * H);
  f32x16 V[2], Y[2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = 32 * n + 8 * g + 4 * h;
      const f32x4 v = *reinterpret_cast<const f32x4*>(O0 + (size_t)pp * C + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) V[n][4 * g + j] = v[j];
    }
  gate_mm(gpk_ir, V, Y, lane);
  if (!ok) return;
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = 32 * n + 8 * g + 4 * h;
      const f32x4 ib = *reinterpret_cast<const f32x4*>(vecs + V_IB * 64 + c);
      f32x4 o, og;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = V[n][4 * g + j];
        og[j] = o[j] * sigmoidf_(Y[n][4 * g + j] + ib[j]);
      }
      const size_t idx = c8_index(b, 4 * n + g, y, x, 4 * h, H, W);
      *reinterpret_cast<f32x4*>(O + idx) = o;
      *reinterpret_cast<f32x4*>(Og + idx) = og;
    }
}

// ---------------------------------------------------------------------------------------------
// conv_1 (3x3, 1 -> 64, SAME) + bias + relu + 2x2/2 max-pool + folded BN  ->  C8
// hgru_pose.py:50-60.  One thread = one pooled pixel x 8 channels (a C8 chunk).  C_in = 1 makes
// this HBM-bound on the C8 store; the 4x4 input patch comes from L1/L2.
// ---------------------------------------------------------------------------------------------
// One thread per pooled output pixel, all 64 channels: the 4x4 input patch is loaded once
// (unconditional clamped loads, zero-masked), and the filter / bias / BN vectors are
// thread-uniform, so they come through scalar loads and enter the FMAs as SGPR operands.
template <bool NHWC>   // output layout: C8 (hGRU backbone) or NHWC (attention net, aconv_1 + apool_1 + BN)
__global__ __launch_bounds__(256) void conv1_pool_bn_kernel(const float* __restrict__ in,
                                                            const float* __restrict__ w,   // [9][64]
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ bn_s,
                                                            const float* __restrict__ bn_t,
                                                            float* out, int B, int Hin, int Win) {
  const int Ho = Hin / 2, Wo = Win / 2;
  const size_t total = (size_t)B * Ho * Wo;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int x = i % Wo;
  const int y = (i / Wo) % Ho;
  const int b = i / ((size_t)Wo * Ho);
  float pt[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int yy = 2 * y - 1 + r, xx = 2 * x - 1 + c;
      const bool ok = yy >= 0 && yy < Hin && xx >= 0 && xx < Win;
      const float v = in[((size_t)b * Hin + min(max(yy, 0), Hin - 1)) * Win + min(max(xx, 0), Win - 1)];
      pt[r][c] = ok ? v : 0.f;
    }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ch = 8 * q + e;
      float best = 0.f;   // relu output >= 0, so 0 is the identity of the max
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          float sacc = 0.f;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) sacc = fmaf(pt[dy + ky][dx + kx], w[(ky * 3 + kx) * 64 + ch], sacc);
          best = fmaxf(best, fmaxf(sacc + bias[ch], 0.f));
        }
      o[e] = best * bn_s[ch] + bn_t[ch];
    }
    float* dst = NHWC ? out + (((size_t)b * Ho + y) * Wo + x) * 64 + 8 * q : out + c8_index(b, q, y, x, 0, Ho, Wo);
    *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{o[4], o[5], o[6], o[7]};
  }
}

// The same fused 1-channel conv_layer + 2x2/2 max pool for any Cout % 4 == 0 (the dense regressor's
// conv_0: 1 -> 12, train_dense_networks.py:229-236), written to an NHWC view (ldo, coff) -- the
// graph runtime's concat buffers.  Exact fp32 FMAs, relu before the max; one thread per pooled
// pixel and 4 output channels.
__global__ __launch_bounds__(256) void conv1_pool_any_kernel(const float* __restrict__ in,
                                                             const float* __restrict__ w,   // [9][Cout]
                                                             const float* __restrict__ bias, float* out,
                                                             int ldo, int coff, int B, int Hin, int Win, int Cout) {
  const int Ho = Hin / 2, Wo = Win / 2, nq = Cout / 4;
  const size_t total = (size_t)B * Ho * Wo * nq;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int q = i % nq;
  const size_t pix = i / nq;
  const int x = pix % Wo;
  const int y = (pix / Wo) % Ho;
  const int b = pix / ((size_t)Wo * Ho);
  float pt[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int yy = 2 * y - 1 + r, xx = 2 * x - 1 + c;
      const bool ok = yy >= 0 && yy < Hin && xx >= 0 && xx < Win;
      const float v = in[((size_t)b * Hin + min(max(yy, 0), Hin - 1)) * Win + min(max(xx, 0), Win - 1)];
      pt[r][c] = ok ? v : 0.f;
    }
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ch = 4 * q + e;
    float best = 0.f;   // relu output >= 0, so 0 is the identity of the max
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float sacc = 0.f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) sacc = fmaf(pt[dy + ky][dx + kx], w[(ky * 3 + kx) * Cout + ch], sacc);
        best = fmaxf(best, fmaxf(sacc + bias[ch], 0.f));
      }
    o[e] = best;
  }
  float* dst = out + pix * ldo + coff + 4 * q;
  if ((ldo | coff) % 4 == 0) {
    *reinterpret_cast<f32x4*>(dst) = o;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[e] = o[e];
  }
}

hipError_t launch_conv1_pool_any(const float* in, const float* w, const float* bias, float* out, int ldo, int coff,
                                 int B, int Hin, int Win, int Cout, hipStream_t st) {
  if (Cout % 4 || Hin % 2 || Win % 2) return hipErrorInvalidValue;
  const size_t total = (size_t)B * (Hin / 2) * (Win / 2) * (Cout / 4);
  hipLaunchKernelGGL(conv1_pool_any_kernel, dim3((total + 255) / 256), dim3(256), 0, st, in, w, bias, out, ldo, coff, B,
                     Hin, Win, Cout);
  return hipGetLastError();
}

// layout conversions (standalone ContextualCircuit API, debug taps)
__global__ void nhwc_to_c8_kernel(const float* __restrict__ in, float* out, int B, int H, int W, bool bf, bool c4) {
  const size_t total = (size_t)B * H * W * NQ;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int q = i % NQ;
  const size_t pix = i / NQ;
  const int x = pix % W, y = (pix / W) % H, b = pix / ((size_t)W * H);
  const f32x4* s = reinterpret_cast<const f32x4*>(in + pix * C + 8 * q);
  const size_t o0 = c4 ? c4_index(b, q, y, x, 0, H, W) : c8_index(b, q, y, x, 0, H, W);
  const size_t o1 = c4 ? c4_index(b, q, y, x, 4, H, W) : o0 + 4;
  if (bf) {
    uint16_t* d = reinterpret_cast<uint16_t*>(out);
    *reinterpret_cast<uint2*>(d + o0) = bf16x4_pack(s[0]);
    *reinterpret_cast<uint2*>(d + o1) = bf16x4_pack(s[1]);
  } else {
    *reinterpret_cast<f32x4*>(out + o0) = s[0];
    *reinterpret_cast<f32x4*>(out + o1) = s[1];
  }
}

// dst_img: elements between consecutive images of the NHWC output (H*W*C when dense; larger when
// writing one timestep of a [n, T, H, W, C] state stack)
__global__ void c8_to_nhwc_kernel(const float* __restrict__ in, float* out, int B, int H, int W, bool bf,
                                  size_t dst_img, bool c4) {
  const size_t total = (size_t)B * H * W * NQ;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int q = i % NQ;
  const size_t pix = i / NQ;
  const int x = pix % W, y = (pix / W) % H, b = pix / ((size_t)W * H);
  // the chunk's two 4-channel halves (adjacent in C8, separate runs in C4)
  const size_t o0 = c4 ? c4_index(b, q, y, x, 0, H, W) : c8_index(b, q, y, x, 0, H, W);
  const size_t o1 = c4 ? c4_index(b, q, y, x, 4, H, W) : o0 + 4;
  f32x4* d = reinterpret_cast<f32x4*>(out + b * dst_img + ((size_t)y * W + x) * C + 8 * q);
  if (bf) {
    const uint16_t* s = reinterpret_cast<const uint16_t*>(in);
    d[0] = bf16x4_unpack(*reinterpret_cast<const uint2*>(s + o0));
    d[1] = bf16x4_unpack(*reinterpret_cast<const uint2*>(s + o1));
  } else {
    d[0] = *reinterpret_cast<const f32x4*>(in + o0);
    d[1] = *reinterpret_cast<const f32x4*>(in + o1);
  }
}

// ---------------------------------------------------------------------------------------------
// weight packing (one-time, at finalize)
// ---------------------------------------------------------------------------------------------
// HWIO [KS][KS][64][64] -> [q][tap][n][lane] float4{ W[tap][8q+4h+s][32n+(lane&31)] }_s
__global__ void pack_conv64_kernel(const float* __restrict__ w, f32x4* out, int KK) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int total = NQ * KK * 2 * 64;
  if (i >= total) return;
  const int lane = i % 64, n = (i / 64) % 2, tap = (i / 128) % KK, q = i / (128 * KK);
  const int co = 32 * n + (lane & 31);
  const int ci0 = 8 * q + 4 * (lane >> 5);
  f32x4 v;
#pragma unroll
  for (int s = 0; s < 4; ++s) v[s] = w[((size_t)tap * 64 + ci0 + s) * 64 + co];
  out[i] = v;
}

// 1x1 gate weights [64 (c)][64 (c2)] -> [n2][nb][g][lane] float4{ G[32nb+8g+4h+j][32n2+(lane&31)] }_j
__global__ void pack_gate_kernel(const float* __restrict__ g, f32x4* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * 2 * 4 * 64) return;
  const int lane = i % 64, gg = (i / 64) % 4, nb = (i / 256) % 2, n2 = i / 512;
  const int c2 = 32 * n2 + (lane & 31);
  const int c0 = 32 * nb + 8 * gg + 4 * (lane >> 5);
  f32x4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = g[(c0 + j) * 64 + c2];
  out[i] = v;
}

}  // namespace mp

// ---------------------------------------------------------------------------------------------
// host launchers (called from mp_abi.cpp)
// ---------------------------------------------------------------------------------------------
namespace mp {

template <int KS, int EPI>
static hipError_t launch_conv64_t(const ConvArgs& a, int B, hipStream_t st) {
  const int nblk = B * a.tiles_x * a.tiles_y;
  hipLaunchKernelGGL((conv64_kernel<KS, EPI>), dim3(nblk), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_conv64(int ks, int epi, ConvArgs a, int B, hipStream_t st) {
  a.tiles_x = a.W / TW;
  a.tiles_y = a.H / TH;
#define MP_CASE(K, E) \
  if (ks == K && epi == E) return launch_conv64_t<K, E>(a, B, st);
  MP_CASE(3, EPI_BB)
  MP_CASE(15, EPI_HGRU_A)
  MP_CASE(15, EPI_HGRU_B)
  MP_CASE(5, EPI_HGRU_A)
  MP_CASE(5, EPI_HGRU_B)
  MP_CASE(3, EPI_HGRU_A)
  MP_CASE(3, EPI_HGRU_B)
#undef MP_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_gate_init(const float* O0, float* O, float* Og, const f32x4* gpk_ir,
                            const float* vecs, int B, int H, int W, hipStream_t st) {
  const int npix = B * H * W;
  const int nw = (npix + 31) / 32;
  hipLaunchKernelGGL(gate_init_kernel, dim3((nw + 3) / 4), dim3(256), 0, st, O0, O, Og, gpk_ir,
                     vecs, npix, H, W);
  return hipGetLastError();
}

hipError_t launch_conv1_pool_bn(const float* in, const float* w, const float* bias, const float* s,
                                const float* t, float* out, int B, int Hin, int Win, hipStream_t st, bool nhwc) {
  const size_t total = (size_t)B * (Hin / 2) * (Win / 2);
  if (nhwc)
    hipLaunchKernelGGL(conv1_pool_bn_kernel<true>, dim3((total + 255) / 256), dim3(256), 0, st, in, w, bias, s, t,
                       out, B, Hin, Win);
  else
    hipLaunchKernelGGL(conv1_pool_bn_kernel<false>, dim3((total + 255) / 256), dim3(256), 0, st, in, w, bias, s, t,
                       out, B, Hin, Win);
  return hipGetLastError();
}

hipError_t launch_nhwc_to_c8(const float* in, float* out, int B, int H, int W, hipStream_t st, bool bf, bool c4) {
  if (c4 && !c4_width_ok(W)) return hipErrorInvalidValue;   // the C4 swizzle needs a power-of-two width
  const size_t total = (size_t)B * H * W * NQ;
  hipLaunchKernelGGL(nhwc_to_c8_kernel, dim3((total + 255) / 256), dim3(256), 0, st, in, out, B, H, W, bf, c4);
  return hipGetLastError();
}

hipError_t launch_c8_to_nhwc(const float* in, float* out, int B, int H, int W, hipStream_t st, bool bf,
                             size_t dst_img, bool c4) {
  if (c4 && !c4_width_ok(W)) return hipErrorInvalidValue;
  const size_t total = (size_t)B * H * W * NQ;
  if (dst_img == 0) dst_img = (size_t)H * W * C;
  hipLaunchKernelGGL(c8_to_nhwc_kernel, dim3((total + 255) / 256), dim3(256), 0, st, in, out, B, H, W, bf,
                     dst_img, c4);
  return hipGetLastError();
}

hipError_t launch_pack_conv64(const float* w, f32x4* out, int ks, hipStream_t st) {
  const int total = NQ * ks * ks * 2 * 64;
  hipLaunchKernelGGL(pack_conv64_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, out, ks * ks);
  return hipGetLastError();
}

hipError_t launch_pack_gate(const float* g, f32x4* out, hipStream_t st) {
  hipLaunchKernelGGL(pack_gate_kernel, dim3(4), dim3(256), 0, st, g, out);
  return hipGetLastError();
}

}  // namespace mp
