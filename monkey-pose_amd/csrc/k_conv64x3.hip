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

#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace mp {

constexpr float ACT_SCALE = 1024.0f;     // 2^10, default activation scale (hGRU maps are tanh / sigmoid-bounded)

__device__ __forceinline__ f32x16 mfma16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// NW waves per block (4: one wave per SIMD, 8 M-blocks each; 8: two waves per SIMD, 4 M-blocks
// each).  SCHED selects the tap-loop schedule: 0 = fragments loaded at the top of each tap and
// left to the compiler; 1 = one-tap-ahead prefetch with the halo reads of M-block m pinned right
// after its MFMAs (sched_group_barrier).
// NP = 3: the fp32-accurate split (hi*lo, lo*hi, hi*hi); NP = 1: hi*hi only (MP_DTYPE_BF16's
// backbone: one f16 product per MAC, 11-bit operands, fp32 accumulation)
// TH rows per tile (TH3 = 32; 8 for small backbone batches) and NN of the two 32-channel output
// blocks per block (1: the block's n-half is blockIdx.x % 2; EPI_BB only).  Each accumulator's
// MFMA sequence (chunks, taps, lo/hi order) is the same for every TH / NN, so the outputs are
// bit-identical across the variants and a batch-size-dependent choice keeps batch invariance.
template <int KS, int EPI, int NW, int SCHED, int NP = 3, int TH = TH3, int NN = 2, int DB = 0>
__global__ __launch_bounds__(NW * 64, 1) void conv64x3_kernel(ConvArgs p, const f16x8* __restrict__ wpk,
                                                              float unscale) {
  static_assert(NN == 2 || EPI == EPI_BB, "split output blocks only for the backbone epilogue");
  static_assert(DB == 0 || SCHED == 1, "the double-buffered halo runs the prefetching tap loop");
  constexpr int R = KS / 2;
  constexpr int HY = TH + KS - 1, HX = TW + KS - 1;
  constexpr int KK = KS * KS;
  constexpr int NQ16 = 4;                // 16-channel chunks
  constexpr int MB = TH / NW;            // M-blocks (rows of 32 pixels) per wave
  static_assert(MB >= 1 && MB * NW == TH, "rows per tile must be a multiple of the wave count");
  constexpr int NT = NW * 64;
  constexpr int HSZ = HY * 4 * HX;       // f16x8 cells of one halo chunk
  // DB: two halo buffers; chunk Q+1's global loads are issued before chunk Q's tap loop and split /
  // written into the other buffer after it, so the loads are in flight during the MFMAs
  __shared__ f16x8 halo_all[(DB ? 2 : 1) * HSZ];
  constexpr int NIT = (HY * HX * 2 + NT - 1) / NT;   // staging items per thread

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int H = p.H, W = p.W;
  int bid = blockIdx.x;
  const int n0 = NN == 2 ? 0 : bid % 2;   // first output block of this block
  if constexpr (NN == 1) bid >>= 1;
  const int tx = bid % p.tiles_x;
  bid /= p.tiles_x;
  const int ty = bid % p.tiles_y;
  const int b = bid / p.tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;

  f32x16 acc[NN][MB];
#pragma unroll
  for (int n = 0; n < NN; ++n)
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[n][m] = f32x16{};

  // staging of one 16-channel chunk: item it = (pixel, half); raw fp32 loads, then split + LDS write
  f32x4 pre[DB ? NIT : 1][2];
  auto load_chunk = [&](int Q) {
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int it = tid + k * NT;
      const int hh = it & 1, pix = min(it >> 1, HY * HX - 1);
      const int hy = pix / HX, hx = pix - hy * HX;
      const int gy = min(max(y0 + hy - R, 0), H - 1), gx = min(max(x0 + hx - R, 0), W - 1);   // clamped
      const f32x4* src = reinterpret_cast<const f32x4*>(p.src + c8_index(b, 2 * Q + hh, gy, gx, 0, H, W));
      pre[k][0] = src[0];
      pre[k][1] = src[1];
    }
  };
  auto write_chunk = [&](f16x8* halo) {
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int it = tid + k * NT;
      if (it >= HY * HX * 2) break;
      const int hh = it & 1, pix = it >> 1;
      const int hy = pix / HX, hx = pix - hy * HX;
      const int gy = y0 + hy - R, gx = x0 + hx - R;
      f16x8 vh = {}, vl = {};
      if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = (j < 4 ? pre[k][0][j] : pre[k][1][j - 4]) * p.ascale;
          const _Float16 hi = (_Float16)v;
          vh[j] = hi;
          vl[j] = (_Float16)(v - (float)hi);
        }
      }
      halo[(hy * 4 + hh) * HX + hx] = vh;
      if constexpr (NP == 3) halo[(hy * 4 + 2 + hh) * HX + hx] = vl;
    }
  };
  if constexpr (DB) {
    load_chunk(0);
    write_chunk(halo_all);
  }

  for (int Q = 0; Q < NQ16; ++Q) {
    f16x8* halo = halo_all + (DB ? (Q & 1) * HSZ : 0);
    if constexpr (DB) {
      __syncthreads();                        // chunk Q's halo written; chunk Q-1's reads done
      if (Q + 1 < NQ16) load_chunk(Q + 1);    // in flight during chunk Q's taps
    } else {
      __syncthreads();
      // ---- stage + split the 16-channel halo chunk (zero outside the image = SAME padding) ----
      for (int it = tid; it < HY * HX * 2; it += NT) {
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
            const float v = (j < 4 ? a0[j] : a1[j - 4]) * p.ascale;
            const _Float16 hi = (_Float16)v;
            vh[j] = hi;
            vl[j] = (_Float16)(v - (float)hi);
          }
        }
        halo[(hy * 4 + hh) * HX + hx] = vh;
        if constexpr (NP == 3) halo[(hy * 4 + 2 + hh) * HX + hx] = vl;
      }
      __syncthreads();
    }
    const f16x8* wq = wpk + (size_t)Q * KK * 4 * 64 + lane;
    const f16x8* hb = halo + ((wv * MB) * 4 + h) * HX + col;
    if constexpr (SCHED == 0) {
      static_assert(NN == 2, "the SCHED 0 tap loop covers both output blocks");
      for (int ky = 0; ky < KS; ++ky) {
        const f16x8* hrow = hb + ky * 4 * HX;
#pragma unroll 1
        for (int kx = 0; kx < KS; ++kx) {
          const f16x8* wt = wq + (ky * KS + kx) * 4 * 64;
          const f16x8 w0 = wt[0], w1 = wt[64], w2 = wt[128], w3 = wt[192];
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            const f16x8 ch = hrow[m * 4 * HX + kx];
            if constexpr (NP == 3) {
              const f16x8 cl = hrow[m * 4 * HX + 2 * HX + kx];
              acc[0][m] = mfma16(w0, cl, acc[0][m]);
              acc[1][m] = mfma16(w2, cl, acc[1][m]);
              acc[0][m] = mfma16(w1, ch, acc[0][m]);
              acc[1][m] = mfma16(w3, ch, acc[1][m]);
            }
            acc[0][m] = mfma16(w0, ch, acc[0][m]);
            acc[1][m] = mfma16(w2, ch, acc[1][m]);
          }
        }
      }
    } else {
      // one-tap-ahead prefetch: the weights of tap t+1 are requested at the top of tap t, the
      // halo fragments of M-block m for tap t+1 right after M-block m's MFMAs of tap t.  The "next
      // tap" of the last tap wraps to tap 0 so every address stays in bounds.
      constexpr int NWF = 2 * NN;   // weight fragments per tap: (hi, lo) of each output block
      f16x8 w[NWF], bh[MB], bl[MB];
      const f16x8* wq0 = wq + 2 * n0 * 64;
#pragma unroll
      for (int i = 0; i < NWF; ++i) w[i] = wq0[i * 64];
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        bh[m] = hb[m * 4 * HX];
        bl[m] = NP == 3 ? hb[m * 4 * HX + 2 * HX] : f16x8{};
      }
      int nky = 0, nkx = 0;
      for (int tap = 0; tap < KK; ++tap) {
        const int ntap = (tap + 1 < KK) ? tap + 1 : 0;
        if (++nkx == KS) {
          nkx = 0;
          nky = (nky + 1 == KS) ? 0 : nky + 1;
        }
        f16x8 cw[NWF];
#pragma unroll
        for (int i = 0; i < NWF; ++i) cw[i] = w[i];
        const f16x8* wn = wq0 + ntap * 4 * 64;
#pragma unroll
        for (int i = 0; i < NWF; ++i) w[i] = wn[i * 64];
        const f16x8* hn = hb + nky * 4 * HX + nkx;
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          const f16x8 ch = bh[m], cl = bl[m];
          if constexpr (NP == 3) {
#pragma unroll
            for (int n = 0; n < NN; ++n) acc[n][m] = mfma16(cw[2 * n], cl, acc[n][m]);
#pragma unroll
            for (int n = 0; n < NN; ++n) acc[n][m] = mfma16(cw[2 * n + 1], ch, acc[n][m]);
          }
#pragma unroll
          for (int n = 0; n < NN; ++n) acc[n][m] = mfma16(cw[2 * n], ch, acc[n][m]);
          bh[m] = hn[m * 4 * HX];
          if constexpr (NP == 3) bl[m] = hn[m * 4 * HX + 2 * HX];
          if (m == 0) __builtin_amdgcn_sched_group_barrier(0x020, NWF, 0);   // the weight loads
          __builtin_amdgcn_sched_group_barrier(0x008, NN * NP, 0);           // 6 (2) MFMA at NN = 2
          __builtin_amdgcn_sched_group_barrier(0x100, NP == 3 ? 2 : 1, 0);   // 2 (1) ds_read
        }
      }
    }
    if constexpr (DB) {
      if (Q + 1 < NQ16) write_chunk(halo_all + ((Q + 1) & 1) * HSZ);   // the other buffer
    }
  }

  const int x = x0 + col;
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    // one M-block at a time: keeps the scheduler from hoisting every block's epilogue loads
    // beside the live accumulators
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NN == 2)
      conv_epilogue<EPI>(p, acc[0][m], acc[1][m], b, y0 + wv * MB + m, x, h, lane, unscale);
    else
      bb_epilogue_n(p, acc[0][m] * unscale, n0, b, y0 + wv * MB + m, x, h);
  }
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

// MP_CONV_DB=0: the single-buffered halo (A/B); the double-buffered one is used for the backbone
static bool conv_db() {
  static const int on = [] {
    const char* e = std::getenv("MP_CONV_DB");
    return e ? std::atoi(e) : 1;
  }();
  return on;
}

template <int KS, int EPI, int NW, int SCHED, int NP = 3, int TH = TH3, int NN = 2>
static hipError_t launch_x3_t(ConvArgs a, const void* wpk, float unscale, int B, hipStream_t st) {
  a.tiles_y = a.H / TH;
  const int nblk = B * a.tiles_x * a.tiles_y * (2 / NN);
  if constexpr (EPI == EPI_BB && KS == 3 && SCHED == 1) {
    if (conv_db()) {
      hipLaunchKernelGGL((conv64x3_kernel<KS, EPI, NW, SCHED, NP, TH, NN, 1>), dim3(nblk), dim3(NW * 64), 0, st, a,
                         static_cast<const f16x8*>(wpk), unscale);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((conv64x3_kernel<KS, EPI, NW, SCHED, NP, TH, NN, 0>), dim3(nblk), dim3(NW * 64), 0, st, a,
                     static_cast<const f16x8*>(wpk), unscale);
  return hipGetLastError();
}

// the production variant per kernel size (chosen with tools/bench_conv.hip)
constexpr int X3_NW = 8, X3_SCHED = 1;

// Backbone convs of small batches: 8-row tiles with one 32-channel output block per workgroup (8x
// the workgroups: a batch-1 conv is 32 instead of 4), bit-identical to the 32-row tiles.  Measured
// (one MI355X, tools/ab_th.sh, backbone ms with 32 / 16 / 8 rows): B = 8 0.118 / - / 0.059, B = 16
// 0.125 / 0.088 / 0.068, B = 24 0.129 / 0.099 / 0.088, B = 32 0.133 / 0.108 / 0.105, B = 48
// 0.145 / 0.160 / -.  Hence 8 rows up to 128 workgroups of the 32-row tiling (B <= 32 at 64 x 64),
// else 32.  MP_CONV_SMALL=0 keeps 32.
static bool conv_small_tiles(const ConvArgs& a, int B) {
  static const int on = [] {
    const char* e = std::getenv("MP_CONV_SMALL");
    return e ? std::atoi(e) : 1;
  }();
  return on && a.H % 8 == 0 && (long)B * (a.W / TW) * (a.H / TH3) <= 128;
}

hipError_t launch_conv64x3(int ks, int epi, ConvArgs a, const void* wpk, float unscale, int B, hipStream_t st,
                           int nprod) {
  a.tiles_x = a.W / TW;
  a.tiles_y = a.H / TH3;
  if (a.ascale == 0.f) a.ascale = ACT_SCALE;
  const bool small = epi == EPI_BB && ks == 3 && conv_small_tiles(a, B);
  if (nprod == 1) {
    if (ks == 3 && epi == EPI_BB)
      return small ? launch_x3_t<3, EPI_BB, X3_NW, X3_SCHED, 1, 8, 1>(a, wpk, unscale, B, st)
                   : launch_x3_t<3, EPI_BB, X3_NW, X3_SCHED, 1>(a, wpk, unscale, B, st);
    return hipErrorInvalidValue;
  }
  if (small) return launch_x3_t<3, EPI_BB, X3_NW, X3_SCHED, 3, 8, 1>(a, wpk, unscale, B, st);
#define MP_CASE(K, E) \
  if (ks == K && epi == E) return launch_x3_t<K, E, X3_NW, X3_SCHED>(a, wpk, unscale, B, st);
  MP_CASE(15, EPI_HGRU_A)
  MP_CASE(15, EPI_HGRU_B)
  MP_CASE(5, EPI_HGRU_A)
  MP_CASE(5, EPI_HGRU_B)
  MP_CASE(3, EPI_HGRU_A)
  MP_CASE(3, EPI_HGRU_B)
  MP_CASE(3, EPI_BB)      // backbone conv_2 / conv_3 under MP_DTYPE_F32_SPLIT / _FFT
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
