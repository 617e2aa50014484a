// Fused epilogues of the 64-channel convolutions (shared by the fp32 and the split-f16 kernels).
// One call handles one 32-pixel row segment (an M-block): acc[n] holds D[cout 32n+(r&3)+8(r>>2)+4h]
// [pixel x] in v_mfma_*_32x32 accumulator layout (the layout is the same for every MFMA dtype).
#pragma once
#include "mp_kernels.hpp"

namespace mp {

// Y[n2] (cout2 block) = sum_c G[c][cout2] * V[c] for one 32-pixel block held in accumulator layout.
// The accumulator register r of lane l is row (r&3)+8(r>>2)+4h of its 32-row block, i.e. exactly
// the B operand of k-step r (k = h), so the 1x1 conv needs no lane movement.
__device__ __forceinline__ void gate_mm(const f32x4* __restrict__ gpk, const f32x16 (&V)[2],
                                        f32x16 (&Y)[2], int lane) {
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) {
    f32x16 acc = {};
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 a = gpk[((n2 * 2 + nb) * 4 + g) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = mfma32(a[j], V[nb][4 * g + j], acc);
      }
    Y[n2] = acc;
  }
}

// backbone epilogue of output block n (32 channels): relu(conv + b), folded BN, C8 store
__device__ __forceinline__ void bb_epilogue_n(const ConvArgs& p, const f32x16& acc, int n, int b, int y, int x,
                                              int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int c = 32 * n + 8 * g + 4 * h;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(p.bias + c);
    const f32x4 ss = *reinterpret_cast<const f32x4*>(p.bn_s + c);
    const f32x4 tt = *reinterpret_cast<const f32x4*>(p.bn_t + c);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = fmaxf(acc[4 * g + j] + bb[j], 0.f);   // relu(conv + b)
      o[j] = v * ss[j] + tt[j];                             // folded BN
    }
    const size_t idx = p.dst_c4 ? c4_index(b, 4 * n + g, y, x, 4 * h, p.H, p.W) : c8_index(b, 4 * n + g, y, x, 4 * h, p.H, p.W);
    if (p.dst_bf16)
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.dst) + idx) = bf16x4_pack(o);
    else
      *reinterpret_cast<f32x4*>(p.dst + idx) = o;
  }
}

template <int EPI>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& p, const f32x16& acc0, const f32x16& acc1,
                                              int b, int y, int x, int h, int lane, float scale) {
  const int H = p.H, W = p.W;
  f32x16 acc[2] = {acc0 * scale, acc1 * scale};
  if constexpr (EPI == EPI_BB) {
#pragma unroll
    for (int n = 0; n < 2; ++n) bb_epilogue_n(p, acc[n], n, b, y, x, h);
  } else if constexpr (EPI == EPI_HGRU_A) {
    // I = tanh(X - (beta*O + nu) * (P1 + lateral_bias))      hgru_module.py:657, 797-799
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * n + 8 * g + 4 * h;
        const size_t idx = c8_index(b, 4 * n + g, y, x, 4 * h, H, W);
        const f32x4 xv = *reinterpret_cast<const f32x4*>(p.X + idx);
        const f32x4 ov = *reinterpret_cast<const f32x4*>(p.O + idx);
        const f32x4 lat = *reinterpret_cast<const f32x4*>(p.vecs + V_LAT * 64 + c);
        const f32x4 be = *reinterpret_cast<const f32x4*>(p.vecs + V_BETA * 64 + c);
        const f32x4 nu = *reinterpret_cast<const f32x4*>(p.vecs + V_NU * 64 + c);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float P = acc[n][4 * g + j] + lat[j];
          o[j] = tanhf(xv[j] - (be[j] * ov[j] + nu[j]) * P);
        }
        *reinterpret_cast<f32x4*>(p.dst + idx) = o;
      }
  } else {
    // g2 = sigmoid(I . o_r + o_b); e = gamma*P2; S = tanh(kappa*(I+e) + omega*(I*e));
    // O' = (g2*O + (1-g2)*S) * rho[t]                          hgru_module.py:729-740, 806-849
    // Iv holds I for the o_r gate, then is overwritten in place with O' for the i_r gate, so the
    // epilogue keeps only 64 extra registers live beside the 128 accumulators.
    f32x16 Iv[2], Y[2];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 iv = *reinterpret_cast<const f32x4*>(p.I + c8_index(b, 4 * n + g, y, x, 4 * h, H, W));
#pragma unroll
        for (int j = 0; j < 4; ++j) Iv[n][4 * g + j] = iv[j];
      }
    gate_mm(p.gpk_or, Iv, Y, lane);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * n + 8 * g + 4 * h;
        const size_t idx = c8_index(b, 4 * n + g, y, x, 4 * h, H, W);
        const f32x4 ov = *reinterpret_cast<const f32x4*>(p.O + idx);
        const f32x4 lat = *reinterpret_cast<const f32x4*>(p.vecs + V_LAT * 64 + c);
        const f32x4 ga = *reinterpret_cast<const f32x4*>(p.vecs + V_GAMMA * 64 + c);
        const f32x4 ka = *reinterpret_cast<const f32x4*>(p.vecs + V_KAPPA * 64 + c);
        const f32x4 om = *reinterpret_cast<const f32x4*>(p.vecs + V_OMEGA * 64 + c);
        const f32x4 ob = *reinterpret_cast<const f32x4*>(p.vecs + V_OB * 64 + c);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g + j;
          const float P = acc[n][r] + lat[j];
          const float g2 = sigmoidf_(Y[n][r] + ob[j]);
          const float iv = Iv[n][r];
          const float e = ga[j] * P;
          const float a = ka[j] * (iv + e);
          const float mm = om[j] * (iv * e);
          const float S = tanhf(a + mm);
          const float on = (g2 * ov[j] + (1.f - g2) * S) * p.rho;
          o[j] = on;
          Iv[n][r] = on;
        }
        *reinterpret_cast<f32x4*>(p.dst + idx) = o;
      }
    f32x16 (&Ov)[2] = Iv;
    if (p.mode == 0) {
      // next step's gated input Og' = O' * sigmoid(O' . i_r + i_b)   hgru_module.py:696-711
      gate_mm(p.gpk_ir, Ov, Y, lane);
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 32 * n + 8 * g + 4 * h;
          const f32x4 ib = *reinterpret_cast<const f32x4*>(p.vecs + V_IB * 64 + c);
          f32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = Ov[n][4 * g + j] * sigmoidf_(Y[n][4 * g + j] + ib[j]);
          *reinterpret_cast<f32x4*>(p.dst2 + c8_index(b, 4 * n + g, y, x, 4 * h, H, W)) = o;
        }
    } else {
      // final step: affine(O') (the BN after the circuit, hgru_pose.py:82-90) in NHWC order,
      // i.e. exactly the row-major flatten fc_1 consumes (hgru_pose.py:160)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 32 * n + 8 * g + 4 * h;
          const f32x4 ss = *reinterpret_cast<const f32x4*>(p.vecs + V_OUTS * 64 + c);
          const f32x4 tt = *reinterpret_cast<const f32x4*>(p.vecs + V_OUTT * 64 + c);
          f32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = Ov[n][4 * g + j] * ss[j] + tt[j];
          *reinterpret_cast<f32x4*>(p.dst2 + (((size_t)b * H + y) * W + x) * C + c) = o;
        }
    }
  }
}

}  // namespace mp
