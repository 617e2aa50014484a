// Generic NHWC convolution (any Cin/Cout, KxK, stride, TF SAME padding) as an implicit GEMM on
// exact-fp32 MFMA, plus 2x2/2 SAME max/avg pooling -- the op vocabulary of the dense and the
// hierarchical regressors (train_dense_networks.py:414-448, train_hier_networks.py:535-569:
// conv_layer = relu(conv2d(x, W, stride, 'SAME') + b); max_pool / avg_pool 2x2/2 SAME).
//
// Tensors are "views": a base pointer, a row stride `ld` (channels per pixel of the underlying
// buffer) and a channel offset, so tf.concat along channels is free: producers write their
// channel range of one wide buffer and consumers read a channel prefix of it.
//
// GEMM: D[cout][pixel] = sum_k W[k][cout] * im2col[pixel][k], k = (ky*KS + kx)*Cin + ci, i.e. the
// HWIO filter read as a [K][Cout] matrix, packed like an FC weight ([k/8][cout/32][lane] float4).
// Block = 4 waves = 128 output pixels (one 32-pixel M-block per wave) x NB*32 output channels;
// the im2col tile [128][32 k] is gathered into LDS (+4 float row pad: conflict-free b128 reads).
#include "mp_kernels.hpp"

#include <algorithm>
#include <cstdlib>

namespace mp {

constexpr int IG_BM = 128, IG_BK = 32, IG_LDA = IG_BK + 4;

template <int NB>
__global__ __launch_bounds__(256) void igemm_conv_kernel(IgemmArgs p) {
  __shared__ float As[IG_BM * IG_LDA];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int HWo = p.Ho * p.Wo;
  const int M = p.N * HWo;
  const int m0 = blockIdx.x * IG_BM;
  const int nb0 = blockIdx.y * NB;
  const int N32 = (p.Cout + 31) / 32;
  const int K8 = (p.K + 7) / 8;
  const bool vec = (p.Cin % 4 == 0) && (p.cix % 4 == 0) && (p.ldx % 4 == 0);

  // the 4 staging slots of this thread keep their pixel for the whole K loop
  int sn[4], sy[4], sx[4];
  bool sok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + (tid >> 3) + 32 * i;
    sok[i] = gm < M;
    const int g = sok[i] ? gm : 0;
    sn[i] = g / HWo;
    const int r = g - sn[i] * HWo;
    sy[i] = (r / p.Wo) * p.stride - p.pad_t;
    sx[i] = (r % p.Wo) * p.stride - p.pad_l;
  }
  const int k4 = (tid & 7) * 4;

  f32x16 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x16{};

  for (int k0 = 0; k0 < p.K; k0 += IG_BK) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const int kk = k0 + k4;
      if (sok[i]) {
        if (vec) {
          if (kk < p.K) {
            const int tap = kk / p.Cin, ci = kk - tap * p.Cin;
            const int iy = sy[i] + tap / p.KS, ix = sx[i] + tap % p.KS;
            if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
              v = *reinterpret_cast<const f32x4*>(p.x + (((size_t)sn[i] * p.H + iy) * p.W + ix) * p.ldx + p.cix + ci);
          }
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int k = kk + s;
            if (k < p.K) {
              const int tap = k / p.Cin, ci = k - tap * p.Cin;
              const int iy = sy[i] + tap / p.KS, ix = sx[i] + tap % p.KS;
              if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
                v[s] = p.x[(((size_t)sn[i] * p.H + iy) * p.W + ix) * p.ldx + p.cix + ci];
            }
          }
        }
      }
      *reinterpret_cast<f32x4*>(As + ((tid >> 3) + 32 * i) * IG_LDA + k4) = v;
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < IG_BK / 8; ++g) {
      const int kb = (k0 >> 3) + g;
      if (kb >= K8) break;
      const f32x4 a = *reinterpret_cast<const f32x4*>(As + (wv * 32 + col) * IG_LDA + 8 * g + 4 * h);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        if (nb0 + nb >= N32) break;   // block-uniform
        const f32x4 wf = p.wpk[((size_t)kb * N32 + nb0 + nb) * 64 + lane];
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[nb] = mfma32(wf[s], a[s], acc[nb]);
      }
    }
  }

  const int gm = m0 + wv * 32 + col;
  if (gm >= M) return;
  float* dst = p.out + (size_t)gm * p.ldo + p.coff;
  const bool vst = (p.ldo % 4 == 0) && (p.coff % 4 == 0) && (p.Cout % 4 == 0);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if (nb0 + nb >= N32) break;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = (nb0 + nb) * 32 + 8 * g + 4 * h;
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[nb][4 * g + j] + (c + j < p.Cout ? p.bias[c + j] : 0.f);
        o[j] = p.relu ? fmaxf(v, 0.f) : v;
      }
      if (vst) {
        if (c < p.Cout) *reinterpret_cast<f32x4*>(dst + c) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c + j < p.Cout) dst[c + j] = o[j];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// fp32-accurate f16x3 implicit GEMM (regressor contexts finalized with MP_DTYPE_F32_SPLIT): the
// same block geometry as igemm_conv_kernel (128 output pixels x NB*32 output channels, one
// 32-pixel M-block per wave), D^T = W^T im2col^T on v_mfma_f32_32x32x16_f16 with both operands
// split into f16 hi + lo (three products per MAC, fp32 accumulation).  Weights are packed like
// fc_1's (launch_pack_fc_x3: [k/16][cout/32][hi|lo][lane] f16x8, power-of-two scale from max|W|);
// activations are split when the im2col tile is staged into LDS (hi / lo planes [128][32 k]).
// The next K step's im2col float4s and weight fragments are loaded into registers while the
// current step's MFMAs run; the loads are unconditional (clamped addresses, then a select), so a
// step's loads are all in flight together.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// XCD-aware tile order for the wide / halo / position-major kernels.  Workgroups are dispatched in
// linear order round-robin over the 8 XCDs, each with its own L2; with the plain (blockIdx.x = M
// tile, blockIdx.y = N tile) order every XCD touched every weight panel and every input row, and
// the PMC counters showed the HBM reads at 2-8x the input (halo) and 80x the weights (hier con_6).
// Here XCD x takes the contiguous virtual range [x T/8, (x+1) T/8) of the T tiles: N-fastest
// (n_major = false: a block's neighbours share its input rows) or M-fastest (n_major = true: they
// share its weight panel).  Identity when T % 8 != 0 or p.xcd == 0.
__device__ __forceinline__ void xcd_tile(const IgemmArgs& p, bool n_major, int& mt, int& nt) {
  const int nM = (int)gridDim.x, nN = (int)gridDim.y, T = nM * nN;
  const int L = (int)blockIdx.x + nM * (int)blockIdx.y;
  const int v = (p.xcd && T % 8 == 0) ? (L % 8) * (T / 8) + L / 8 : L;
  if (n_major) {
    nt = v / nM;
    mt = v - nt * nM;
  } else {
    mt = v / nN;
    nt = v - mt * nN;
  }
}

constexpr int IGX_LD = IG_BK + 8;   // f16 pitch of the hi / lo planes (+16 B: conflict-free b128 reads)

// NP (every f16 split kernel below): 3 = the fp32-accurate hi*lo + lo*hi + hi*hi products; 1 = hi*hi
// only (MP_DTYPE_BF16 regressors: one f16 MFMA per MAC, the lo planes neither staged nor loaded)
template <int NB, int NP>
__global__ __launch_bounds__(256, NB == 4 ? 2 : 3) void igemm_x3_kernel(IgemmArgs p, const f16x8* __restrict__ wpk, float unscale) {
  __shared__ _Float16 Ah[IG_BM * IGX_LD], Al[IG_BM * IGX_LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int HWo = p.Ho * p.Wo;
  const int M = p.N * HWo;
  const int m0 = blockIdx.x * IG_BM;
  const int nb0 = blockIdx.y * NB;
  const int N32 = (p.Cout + 31) / 32;
  const int K16 = (p.K + 15) / 16;
  const bool vec = (p.Cin % 4 == 0) && (p.cix % 4 == 0) && (p.ldx % 4 == 0);

  int sn[4], sy[4], sx[4];
  bool sok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + (tid >> 3) + 32 * i;
    sok[i] = gm < M;
    const int g = sok[i] ? gm : 0;
    sn[i] = g / HWo;
    const int r = g - sn[i] * HWo;
    sy[i] = (r / p.Wo) * p.stride - p.pad_t;
    sx[i] = (r % p.Wo) * p.stride - p.pad_l;
  }
  const int k4 = (tid & 7) * 4;

  // this thread's im2col column k = k0 + k4 as (ky, kx, ci), advanced by one K step per load_act
  // call (the calls come in K order) instead of two integer divisions per step; past K the tap
  // runs off the image (clamped address, masked value)
  int ici = 0, ikx = 0, iky = 0;
  auto im2col_start = [&](int k) {
    const int tap = k / p.Cin;
    ici = k - tap * p.Cin;
    iky = tap / p.KS;
    ikx = tap - iky * p.KS;
  };
  uint32_t okm = 0;   // bit i: slot i of the last load_act is inside the image and K
  auto load_act = [&](int k0, f32x4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = k0 + k4;
      if (vec) {
        const int iy = sy[i] + iky, ix = sx[i] + ikx;
        const bool ok = sok[i] && kk < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        const int cy = min(max(iy, 0), p.H - 1), cx = min(max(ix, 0), p.W - 1);
        v[i] = *reinterpret_cast<const f32x4*>(p.x + (((size_t)sn[i] * p.H + cy) * p.W + cx) * p.ldx + p.cix + ici);
        okm = ok ? okm | (1u << i) : okm & ~(1u << i);   // applied at the LDS store
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = kk + s;
          const int kc = min(k, p.K - 1);
          const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
          const int iy = sy[i] + tap / p.KS, ix = sx[i] + tap % p.KS;
          const bool ok = sok[i] && k < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
          const int cy = min(max(iy, 0), p.H - 1), cx = min(max(ix, 0), p.W - 1);
          const float t = p.x[(((size_t)sn[i] * p.H + cy) * p.W + cx) * p.ldx + p.cix + ci];
          v[i][s] = ok ? t : 0.f;
        }
        okm |= 1u << i;
      }
    }
    if (vec) {   // the next K step: ci += 32, carrying into the tap (at most 32 / Cin carries)
      ici += IG_BK;
      while (ici >= p.Cin) {
        ici -= p.Cin;
        if (++ikx == p.KS) {
          ikx = 0;
          ++iky;
        }
      }
    }
  };
  auto load_w = [&](int k0, f16x8 (&w)[2][NB][2]) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int kb = min((k0 >> 4) + g, K16 - 1);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int nbc = min(nb0 + nb, N32 - 1);
        const f16x8* wp = wpk + (((size_t)kb * N32 + nbc) * 2) * 64 + lane;
        w[g][nb][0] = wp[0];
        if constexpr (NP == 3) w[g][nb][1] = wp[64];
      }
    }
  };

  f32x16 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x16{};
  f32x4 av[4];
  f16x8 wn[2][NB][2];
  im2col_start(k4);
  load_act(0, av);
  load_w(0, wn);
  for (int k0 = 0; k0 < p.K; k0 += IG_BK) {
    lds_barrier();   // the previous step's LDS reads are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // one 8-byte store per plane and slot
      const int row = (tid >> 3) + 32 * i;
      f16x4 hv, lv;
      // the padding / past-K mask of the load (a select at the load made hipcc wait for each load
      // before issuing the next: the one-step prefetch was four serial HBM round trips)
      const f32x4 a = ((okm >> i) & 1u) ? av[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        hv[s] = (_Float16)a[s];
        lv[s] = (_Float16)(a[s] - (float)hv[s]);
      }
      *reinterpret_cast<f16x4*>(Ah + row * IGX_LD + k4) = hv;
      if constexpr (NP == 3) *reinterpret_cast<f16x4*>(Al + row * IGX_LD + k4) = lv;
    }
    f16x8 wc[2][NB][2];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        wc[g][nb][0] = wn[g][nb][0];
        wc[g][nb][1] = wn[g][nb][1];
      }
    // prefetch the next step, past the end too (masked, clamped addresses): a conditional prefetch
    // made hipcc merge the two paths into vmcnt(0) waits
    load_act(k0 + IG_BK, av);
    load_w(k0 + IG_BK, wn);
    lds_barrier();
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if ((k0 >> 4) + g >= K16) break;   // block-uniform
      const int o = (wv * 32 + col) * IGX_LD + 16 * g + 8 * h;
      const f16x8 ah = *reinterpret_cast<const f16x8*>(Ah + o);
      const f16x8 al = *reinterpret_cast<const f16x8*>(Al + o);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        if (nb0 + nb >= N32) break;   // block-uniform
        if constexpr (NP == 3) {
          acc[nb] = mfma16(wc[g][nb][1], ah, acc[nb]);
          acc[nb] = mfma16(wc[g][nb][0], al, acc[nb]);
        }
        acc[nb] = mfma16(wc[g][nb][0], ah, acc[nb]);
      }
    }
  }

  const int gm = m0 + wv * 32 + col;
  if (gm >= M) return;
  float* dst = p.out + (size_t)gm * p.ldo + p.coff;
  const bool vst = (p.ldo % 4 == 0) && (p.coff % 4 == 0) && (p.Cout % 4 == 0);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if (nb0 + nb >= N32) break;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = (nb0 + nb) * 32 + 8 * g + 4 * h;
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = acc[nb][4 * g + j] * unscale + (c + j < p.Cout ? p.bias[c + j] : 0.f);
        o[j] = p.relu ? fmaxf(v, 0.f) : v;
      }
      if (vst) {
        if (c < p.Cout) *reinterpret_cast<f32x4*>(dst + c) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c + j < p.Cout) dst[c + j] = o[j];
      }
    }
  }
}

// Position-major variant of igemm_x3w_kernel (below) for small maps with many padding taps (p.pmajor):
// m = position * N + image, so a block's pixels share one (or a few) output positions and its K
// loop visits only the taps inside the image for them.  Separate from igemm_x3w_kernel: the extra
// index arithmetic costs the row-major kernel 1.5-3 % (measured same-box A/B).
constexpr bool PM = true;
template <int NP>
__global__ __launch_bounds__(256, 3) void igemm_x3w_pm_kernel(IgemmArgs p, const f16x8* __restrict__ wpk, float unscale) {
  __shared__ _Float16 Ah[IG_BM * IGX_LD], Al[IG_BM * IGX_LD];
  __shared__ f16x8 Ws[2 * 4 * 2 * 64];   // [k16 g][cout block nb][part][lane]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int wm = wv & 1, wn = wv >> 1;   // this wave: pixels 64 wm .. +63, cout blocks 2 wn, 2 wn + 1
  const int HWo = p.Ho * p.Wo;
  const int M = p.N * HWo;
  int mt_, nt_;
  xcd_tile(p, true, mt_, nt_);   // blocks of one weight panel share an L2
  const int m0 = mt_ * IG_BM;
  const int nb0 = nt_ * 4;
  const int N32 = (p.Cout + 31) / 32;
  const int K16 = (p.K + 15) / 16;
  const bool vec = (p.Cin % 4 == 0) && (p.cix % 4 == 0) && (p.ldx % 4 == 0);

  int sn[4], sy[4], sx[4];
  bool sok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + (tid >> 3) + 32 * i;
    sok[i] = gm < M;
    const int g = sok[i] ? gm : 0;
    int r;
    if (PM) {
      sn[i] = g % p.N;
      r = g / p.N;
    } else {
      sn[i] = g / HWo;
      r = g - sn[i] * HWo;
    }
    sy[i] = (r / p.Wo) * p.stride - p.pad_t;
    sx[i] = (r % p.Wo) * p.stride - p.pad_l;
  }
  // K steps: all of K, or (position-major tiles with Cin % IG_BK == 0) only the taps that are
  // inside the image for at least one of the block's output positions -- ky x kx rectangles of
  // whole IG_BK steps (a 5x5 conv on a 4x4 map keeps 9-16 of its 25 taps per position)
  int ky_lo = 0, kx_lo = 0, nky = 1, kxsteps = (p.K + IG_BK - 1) / IG_BK;
  const bool skip = PM;   // the launcher sets PM only with Cin % IG_BK == 0
  if (skip) {
    const int p0 = m0 / p.N, p1 = (min(m0 + IG_BM, M) - 1) / p.N;
    int y0 = 1 << 30, y1 = -1, x0 = 1 << 30, x1 = -1;
    for (int q = p0; q <= p1; ++q) {
      const int yy = q / p.Wo, xx = q % p.Wo;
      y0 = min(y0, yy);
      y1 = max(y1, yy);
      x0 = min(x0, xx);
      x1 = max(x1, xx);
    }
    ky_lo = max(0, p.pad_t - y1 * p.stride);
    const int ky_hi = min(p.KS - 1, p.H - 1 + p.pad_t - y0 * p.stride);
    kx_lo = max(0, p.pad_l - x1 * p.stride);
    const int kx_hi = min(p.KS - 1, p.W - 1 + p.pad_l - x0 * p.stride);
    nky = max(0, ky_hi - ky_lo + 1);
    kxsteps = max(0, kx_hi - kx_lo + 1) * (p.Cin / IG_BK);
  }
  // split-K (p.part, gridDim.z ranges): this block sums input channels [z cps, (z+1) cps) chunks of
  // every visited tap -- the grouping depends on the layer only, never on the batch
  const int nz = p.part ? (int)gridDim.z : 1, cps = p.Cin / IG_BK / nz, zc = (int)blockIdx.z * cps;
  if (nz > 1) kxsteps = kxsteps / (p.Cin / IG_BK) * cps;
  const int nsteps = nky * kxsteps;
  auto kof = [&](int st) {   // k0 of K step st
    if (!skip) return st * IG_BK;
    const int r = st / kxsteps;
    if (nz > 1) {
      const int rem = st - r * kxsteps, kxo = rem / cps;
      return ((ky_lo + r) * p.KS + kx_lo + kxo) * p.Cin + (zc + rem - kxo * cps) * IG_BK;
    }
    return ((ky_lo + r) * p.KS + kx_lo) * p.Cin + (st - r * kxsteps) * IG_BK;
  };
  const int k4 = (tid & 7) * 4;

  uint32_t okm = 0;   // bit i: slot i of the last load_act is inside the image and K
  auto load_act = [&](int k0, f32x4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = k0 + k4;
      if (vec) {
        const int kc = min(kk, p.K - 4);
        const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
        const int iy = sy[i] + tap / p.KS, ix = sx[i] + tap % p.KS;
        const bool ok = sok[i] && kk < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        const int cy = min(max(iy, 0), p.H - 1), cx = min(max(ix, 0), p.W - 1);
        v[i] = *reinterpret_cast<const f32x4*>(p.x + (((size_t)sn[i] * p.H + cy) * p.W + cx) * p.ldx + p.cix + ci);
        okm = ok ? okm | (1u << i) : okm & ~(1u << i);   // applied at the LDS store
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = kk + s;
          const int kc = min(k, p.K - 1);
          const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
          const int iy = sy[i] + tap / p.KS, ix = sx[i] + tap % p.KS;
          const bool ok = sok[i] && k < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
          const int cy = min(max(iy, 0), p.H - 1), cx = min(max(ix, 0), p.W - 1);
          const float t = p.x[(((size_t)sn[i] * p.H + cy) * p.W + cx) * p.ldx + p.cix + ci];
          v[i][s] = ok ? t : 0.f;
        }
        okm |= 1u << i;
      }
    }
  };
  // this thread's 4 of the step's 1,024 weight fragments (16 KiB; slot e = tid + 256 u of
  // [g][nb][part][lane]); cout blocks past N32 and k16 past K16 are clamped (their products are
  // never stored / multiply zero activations)
  auto load_w = [&](int k0, f16x8 (&w)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, l = e & 63, part = (e >> 6) & 1, nb = (e >> 7) & 3, g = e >> 9;
      const int kb = min((k0 >> 4) + g, K16 - 1), nbc = min(nb0 + nb, N32 - 1);
      if (NP == 3 || part == 0) w[u] = wpk[(((size_t)kb * N32 + nbc) * 2 + part) * 64 + l];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = f32x16{};
  f32x4 av[4];
  f16x8 wnx[4];
  if (nsteps > 0) {
    load_act(kof(0), av);
    load_w(kof(0), wnx);
  }
  const bool wave_on = nb0 + 2 * wn < N32;   // wave-uniform
  for (int st = 0; st < nsteps; ++st) {
    const int k0 = kof(st);
    lds_barrier();   // the previous step's LDS reads are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      f16x4 hv, lv;
      // the padding / past-K mask of the load (a select at the load made hipcc wait for each load
      // before issuing the next: the one-step prefetch was four serial HBM round trips)
      const f32x4 a = ((okm >> i) & 1u) ? av[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        hv[s] = (_Float16)a[s];
        lv[s] = (_Float16)(a[s] - (float)hv[s]);
      }
      *reinterpret_cast<f16x4*>(Ah + row * IGX_LD + k4) = hv;
      if constexpr (NP == 3) *reinterpret_cast<f16x4*>(Al + row * IGX_LD + k4) = lv;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) Ws[tid + 256 * u] = wnx[u];
    {   // the next step, past the end too (kof clamped, masked, clamped addresses)
      const int kn = kof(min(st + 1, nsteps - 1));
      load_act(kn, av);
      load_w(kn, wnx);
    }
    lds_barrier();
    if (wave_on) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        if ((k0 >> 4) + g >= K16) break;   // block-uniform
        f16x8 ah[2], al[2];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
          const int o = ((2 * wm + mb) * 32 + col) * IGX_LD + 16 * g + 8 * h;
          ah[mb] = *reinterpret_cast<const f16x8*>(Ah + o);
          al[mb] = *reinterpret_cast<const f16x8*>(Al + o);
        }
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const f16x8 wh = Ws[((g * 4 + 2 * wn + nb) * 2 + 0) * 64 + lane];
          const f16x8 wl = Ws[((g * 4 + 2 * wn + nb) * 2 + 1) * 64 + lane];
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {
            if constexpr (NP == 3) {
              acc[mb][nb] = mfma16(wl, ah[mb], acc[mb][nb]);
              acc[mb][nb] = mfma16(wh, al[mb], acc[mb][nb]);
            }
            acc[mb][nb] = mfma16(wh, ah[mb], acc[mb][nb]);
          }
        }
      }
    }
  }
  if (!wave_on) return;
  if (nz > 1) {   // raw partial sums [z][gm][N32 * 32]; the reduce applies the epilogue
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int gm = m0 + (2 * wm + mb) * 32 + col;
      if (gm >= M) continue;
      float* dst = p.part + ((size_t)blockIdx.z * M + gm) * (N32 * 32);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int cb = nb0 + 2 * wn + nb;
        if (cb >= N32) break;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(dst + cb * 32 + 8 * g + 4 * h) =
              f32x4{acc[mb][nb][4 * g], acc[mb][nb][4 * g + 1], acc[mb][nb][4 * g + 2], acc[mb][nb][4 * g + 3]};
      }
    }
    return;
  }
  const bool vst = (p.ldo % 4 == 0) && (p.coff % 4 == 0) && (p.Cout % 4 == 0);
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int gm = m0 + (2 * wm + mb) * 32 + col;
    if (gm >= M) continue;
    const size_t pix = PM ? (size_t)(gm % p.N) * HWo + gm / p.N : (size_t)gm;   // NHWC pixel index
    float* dst = p.out + pix * p.ldo + p.coff;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int cb = nb0 + 2 * wn + nb;
      if (cb >= N32) break;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = cb * 32 + 8 * g + 4 * h;
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = acc[mb][nb][4 * g + j] * unscale + (c + j < p.Cout ? p.bias[c + j] : 0.f);
          o[j] = p.relu ? fmaxf(v, 0.f) : v;
        }
        if (vst) {
          if (c < p.Cout) *reinterpret_cast<f32x4*>(dst + c) = o;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c + j < p.Cout) dst[c + j] = o[j];
        }
      }
    }
  }
}

// the split-K reduce of igemm_x3w_pm_kernel: out = relu?((sum_z part[z]) * unscale + bias), z in
// order; one thread per 4 output channels of one (position-major) row
__global__ __launch_bounds__(256) void igemm_pm_reduce_kernel(IgemmArgs p, int S, float unscale) {
  const int HWo = p.Ho * p.Wo, M = p.N * HWo, N32 = (p.Cout + 31) / 32, nq = N32 * 8;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * nq) return;
  const int gm = (int)(i / nq), c = (int)(i - (size_t)gm * nq) * 4;
  if (c >= p.Cout) return;
  auto sum = [&](int row) {
    const float* src = p.part + (size_t)row * (N32 * 32) + c;
    f32x4 s = *reinterpret_cast<const f32x4*>(src);
    for (int z = 1; z < S; ++z) s += *reinterpret_cast<const f32x4*>(src + (size_t)z * M * (N32 * 32));
    return s;
  };
  if (p.pool) {   // fused 2x2/2 max pool: this thread = pooled position q (the top-left window row)
    const int n = gm % p.N, pos = gm / p.N, y = pos / p.Wo, x = pos - y * p.Wo;
    if ((y & 1) || (x & 1)) return;
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const f32x4 s = sum(((y + (d >> 1)) * p.Wo + x + (d & 1)) * p.N + n);
#pragma unroll
      for (int j = 0; j < 4; ++j) best[j] = fmaxf(best[j], fmaxf(s[j] * unscale + (c + j < p.Cout ? p.bias[c + j] : 0.f), 0.f));
    }
    float* dst = p.out + (((size_t)n * (p.Ho / 2) + y / 2) * (p.Wo / 2) + x / 2) * p.ldo + p.coff + c;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (c + j < p.Cout) dst[j] = best[j];
    return;
  }
  const f32x4 s = sum(gm);
  float* dst = p.out + ((size_t)(gm % p.N) * HWo + gm / p.N) * p.ldo + p.coff + c;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (c + j >= p.Cout) break;
    const float v = s[j] * unscale + p.bias[c + j];
    dst[j] = p.relu ? fmaxf(v, 0.f) : v;
  }
}

// Wide-N f16x3 implicit GEMM (Cout > 64): block = 128 output pixels x 128 output channels with the
// four waves in a 2 x 2 grid, each wave 64 pixels x 64 channels (2 x 2 MFMA tiles).  The K step's
// weight fragments (2 k16 x 4 cout blocks x hi|lo = 16 KiB) are staged in LDS once per block
// instead of being loaded by every wave from L1 (4x fewer weight loads than igemm_x3_kernel, whose
// waves each own 32 pixels x 128 channels), and every weight fragment read from LDS feeds two
// pixel blocks.  Same operand split, packing, K pipeline and epilogue as igemm_x3_kernel.
template <int NP>
__global__ __launch_bounds__(256, 3) void igemm_x3w_kernel(IgemmArgs p, const f16x8* __restrict__ wpk, float unscale) {
  __shared__ _Float16 Ah[IG_BM * IGX_LD], Al[IG_BM * IGX_LD];
  __shared__ f16x8 Ws[2 * 4 * 2 * 64];   // [k16 g][cout block nb][part][lane]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int wm = wv & 1, wn = wv >> 1;   // this wave: pixels 64 wm .. +63, cout blocks 2 wn, 2 wn + 1
  const int HWo = p.Ho * p.Wo;
  const int M = p.N * HWo;
  int mt_, nt_;
  xcd_tile(p, false, mt_, nt_);   // neighbouring tiles share input rows
  const int m0 = mt_ * IG_BM;
  const int nb0 = nt_ * 4;
  const int N32 = (p.Cout + 31) / 32;
  const int K16 = (p.K + 15) / 16;
  const bool vec = (p.Cin % 4 == 0) && (p.cix % 4 == 0) && (p.ldx % 4 == 0);

  int sn[4], sy[4], sx[4];
  bool sok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + (tid >> 3) + 32 * i;
    sok[i] = gm < M;
    const int g = sok[i] ? gm : 0;
    sn[i] = g / HWo;
    const int r = g - sn[i] * HWo;
    sy[i] = (r / p.Wo) * p.stride - p.pad_t;
    sx[i] = (r % p.Wo) * p.stride - p.pad_l;
  }
  const int k4 = (tid & 7) * 4;

  // this thread's im2col column k = k0 + k4 as (ky, kx, ci), advanced by one K step per load_act
  // call (the calls come in K order) instead of two integer divisions per step; past K the tap
  // runs off the image (clamped address, masked value)
  int ici = 0, ikx = 0, iky = 0;
  auto im2col_start = [&](int k) {
    const int tap = k / p.Cin;
    ici = k - tap * p.Cin;
    iky = tap / p.KS;
    ikx = tap - iky * p.KS;
  };
  uint32_t okm = 0;   // bit i: slot i of the last load_act is inside the image and K
  auto load_act = [&](int k0, f32x4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = k0 + k4;
      if (vec) {
        const int iy = sy[i] + iky, ix = sx[i] + ikx;
        const bool ok = sok[i] && kk < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        const int cy = min(max(iy, 0), p.H - 1), cx = min(max(ix, 0), p.W - 1);
        v[i] = *reinterpret_cast<const f32x4*>(p.x + (((size_t)sn[i] * p.H + cy) * p.W + cx) * p.ldx + p.cix + ici);
        okm = ok ? okm | (1u << i) : okm & ~(1u << i);   // applied at the LDS store
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = kk + s;
          const int kc = min(k, p.K - 1);
          const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
          const int iy = sy[i] + tap / p.KS, ix = sx[i] + tap % p.KS;
          const bool ok = sok[i] && k < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
          const int cy = min(max(iy, 0), p.H - 1), cx = min(max(ix, 0), p.W - 1);
          const float t = p.x[(((size_t)sn[i] * p.H + cy) * p.W + cx) * p.ldx + p.cix + ci];
          v[i][s] = ok ? t : 0.f;
        }
        okm |= 1u << i;
      }
    }
    if (vec) {   // the next K step: ci += 32, carrying into the tap (at most 32 / Cin carries)
      ici += IG_BK;
      while (ici >= p.Cin) {
        ici -= p.Cin;
        if (++ikx == p.KS) {
          ikx = 0;
          ++iky;
        }
      }
    }
  };
  // this thread's 4 of the step's 1,024 weight fragments (16 KiB; slot e = tid + 256 u of
  // [g][nb][part][lane]); cout blocks past N32 and k16 past K16 are clamped (their products are
  // never stored / multiply zero activations)
  auto load_w = [&](int k0, f16x8 (&w)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, l = e & 63, part = (e >> 6) & 1, nb = (e >> 7) & 3, g = e >> 9;
      const int kb = min((k0 >> 4) + g, K16 - 1), nbc = min(nb0 + nb, N32 - 1);
      if (NP == 3 || part == 0) w[u] = wpk[(((size_t)kb * N32 + nbc) * 2 + part) * 64 + l];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = f32x16{};
  // split-K (p.part, gridDim.z ranges, tiny maps: igemm_x3w_splits): this block sums K steps
  // [kb0, kb1) into raw partials; igemm_split_reduce_kernel adds them in z order with the epilogue
  const int nz = p.part ? (int)gridDim.z : 1;
  const int kspan = ((p.K + nz - 1) / nz + IG_BK - 1) / IG_BK * IG_BK;
  const int kb0 = (int)blockIdx.z * kspan, kb1 = min(p.K, kb0 + kspan);
  f32x4 av[4];
  f16x8 wnx[4];
  im2col_start(kb0 + k4);
  load_act(kb0, av);
  load_w(kb0, wnx);
  const bool wave_on = nb0 + 2 * wn < N32;   // wave-uniform
  for (int k0 = kb0; k0 < kb1; k0 += IG_BK) {
    lds_barrier();   // the previous step's LDS reads are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      f16x4 hv, lv;
      // the padding / past-K mask of the load (a select at the load made hipcc wait for each load
      // before issuing the next: the one-step prefetch was four serial HBM round trips)
      const f32x4 a = ((okm >> i) & 1u) ? av[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        hv[s] = (_Float16)a[s];
        lv[s] = (_Float16)(a[s] - (float)hv[s]);
      }
      *reinterpret_cast<f16x4*>(Ah + row * IGX_LD + k4) = hv;
      if constexpr (NP == 3) *reinterpret_cast<f16x4*>(Al + row * IGX_LD + k4) = lv;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) Ws[tid + 256 * u] = wnx[u];
    load_act(k0 + IG_BK, av);   // the next step, past the end too (masked, clamped addresses)
    load_w(k0 + IG_BK, wnx);
    lds_barrier();
    if (wave_on) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        if ((k0 >> 4) + g >= K16) break;   // block-uniform
        f16x8 ah[2], al[2];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
          const int o = ((2 * wm + mb) * 32 + col) * IGX_LD + 16 * g + 8 * h;
          ah[mb] = *reinterpret_cast<const f16x8*>(Ah + o);
          al[mb] = *reinterpret_cast<const f16x8*>(Al + o);
        }
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const f16x8 wh = Ws[((g * 4 + 2 * wn + nb) * 2 + 0) * 64 + lane];
          const f16x8 wl = Ws[((g * 4 + 2 * wn + nb) * 2 + 1) * 64 + lane];
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {
            if constexpr (NP == 3) {
              acc[mb][nb] = mfma16(wl, ah[mb], acc[mb][nb]);
              acc[mb][nb] = mfma16(wh, al[mb], acc[mb][nb]);
            }
            acc[mb][nb] = mfma16(wh, ah[mb], acc[mb][nb]);
          }
        }
      }
    }
  }
  if (!wave_on) return;
  if (nz > 1) {   // raw partial sums [z][gm][N32 * 32]
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int gm = m0 + (2 * wm + mb) * 32 + col;
      if (gm >= M) continue;
      float* dst = p.part + ((size_t)blockIdx.z * M + gm) * (N32 * 32);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int cb = nb0 + 2 * wn + nb;
        if (cb >= N32) break;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(dst + cb * 32 + 8 * g + 4 * h) =
              f32x4{acc[mb][nb][4 * g], acc[mb][nb][4 * g + 1], acc[mb][nb][4 * g + 2], acc[mb][nb][4 * g + 3]};
      }
    }
    return;
  }
  const bool vst = (p.ldo % 4 == 0) && (p.coff % 4 == 0) && (p.Cout % 4 == 0);
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int gm = m0 + (2 * wm + mb) * 32 + col;
    if (gm >= M) continue;
    float* dst = p.out + (size_t)gm * p.ldo + p.coff;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int cb = nb0 + 2 * wn + nb;
      if (cb >= N32) break;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = cb * 32 + 8 * g + 4 * h;
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = acc[mb][nb][4 * g + j] * unscale + (c + j < p.Cout ? p.bias[c + j] : 0.f);
          o[j] = p.relu ? fmaxf(v, 0.f) : v;
        }
        if (vst) {
          if (c < p.Cout) *reinterpret_cast<f32x4*>(dst + c) = o;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c + j < p.Cout) dst[c + j] = o[j];
        }
      }
    }
  }
}

// the split-K reduce of igemm_x3w_kernel (row-major rows): out = relu?((sum_z part[z]) * unscale +
// bias), z in order; one thread per 4 output channels of one row
__global__ __launch_bounds__(256) void igemm_split_reduce_kernel(IgemmArgs p, int S, float unscale) {
  const int M = p.N * p.Ho * p.Wo, N32 = (p.Cout + 31) / 32, nq = N32 * 8;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * nq) return;
  const int gm = (int)(i / nq), c = (int)(i - (size_t)gm * nq) * 4;
  if (c >= p.Cout) return;
  const float* src = p.part + (size_t)gm * (N32 * 32) + c;
  f32x4 s = *reinterpret_cast<const f32x4*>(src);
  for (int z = 1; z < S; ++z) s += *reinterpret_cast<const f32x4*>(src + (size_t)z * M * (N32 * 32));
  float* dst = p.out + (size_t)gm * p.ldo + p.coff + c;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (c + j >= p.Cout) break;
    const float v = s[j] * unscale + p.bias[c + j];
    dst[j] = p.relu ? fmaxf(v, 0.f) : v;
  }
}

// Pointwise (1x1, stride 1) f16x3 conv for K = Cin <= 192 and Cout <= 256 (the dense regressors'
// bottlenecks, train_dense_networks.py:248-373: 40 .. 184 -> 24 .. 96 channels on 64 x 64 maps).
// These are HBM-bound GEMMs with a short K loop: the im2col kernels' one-step-ahead prefetch left a
// load latency exposed in every one of their 2 - 6 K steps.  Here every thread issues its whole
// K extent of the activation tile (NCH chunks x 4 float4) up front, then the chunk loop only splits,
// stages and multiplies; weights stay one chunk ahead (L2-resident).  Block / wave geometry, operand
// split and epilogue are igemm_x3w_kernel's (128 pixels x 128 couts, 2 x 2 waves of 64 x 64), and
// so are the per-output K order and the result, bit for bit.
template <int NP, int NCH>
__global__ __launch_bounds__(256, 2) void igemm_x3pw_kernel(IgemmArgs p, const f16x8* __restrict__ wpk, float unscale) {
  __shared__ _Float16 Ah[IG_BM * IGX_LD], Al[IG_BM * IGX_LD];
  __shared__ f16x8 Ws[2 * 4 * 2 * 64];   // [k16 g][cout block nb][part][lane]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int wm = wv & 1, wn = wv >> 1;
  const int M = p.N * p.Ho * p.Wo;
  int mt_, nt_;
  xcd_tile(p, false, mt_, nt_);   // the N tiles of one pixel tile run on one XCD: one HBM read of it
  const int m0 = mt_ * IG_BM;
  const int nb0 = nt_ * 4;        // first 32-channel block of this block's 128 output channels
  const int N32 = (p.Cout + 31) / 32;
  const int K16 = (p.K + 15) / 16;
  const int k4 = (tid & 7) * 4;
  f32x4 av[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = m0 + (tid >> 3) + 32 * i, k = 32 * c + k4;
      const f32x4 t =
          *reinterpret_cast<const f32x4*>(p.x + (size_t)min(gm, M - 1) * p.ldx + p.cix + min(k, p.K - 4));
      av[c][i] = (gm < M && k < p.K) ? t : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  auto load_w = [&](int k0, f16x8 (&w)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, l = e & 63, part = (e >> 6) & 1, nb = (e >> 7) & 3, g = e >> 9;
      const int kb = min((k0 >> 4) + g, K16 - 1), nbc = min(nb0 + nb, N32 - 1);
      if (NP == 3 || part == 0) w[u] = wpk[(((size_t)kb * N32 + nbc) * 2 + part) * 64 + l];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = f32x16{};
  f16x8 wnx[4];
  load_w(0, wnx);
  const bool wave_on = nb0 + 2 * wn < N32;   // wave-uniform
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k0 = 32 * c;
    lds_barrier();   // the previous chunk's LDS reads are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      f16x4 hv, lv;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        hv[s] = (_Float16)av[c][i][s];
        lv[s] = (_Float16)(av[c][i][s] - (float)hv[s]);
      }
      *reinterpret_cast<f16x4*>(Ah + row * IGX_LD + k4) = hv;
      if constexpr (NP == 3) *reinterpret_cast<f16x4*>(Al + row * IGX_LD + k4) = lv;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) Ws[tid + 256 * u] = wnx[u];
    if (c + 1 < NCH) load_w(k0 + IG_BK, wnx);
    lds_barrier();
    if (wave_on) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        if ((k0 >> 4) + g >= K16) break;   // block-uniform
        f16x8 ah[2], al[2];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
          const int o = ((2 * wm + mb) * 32 + col) * IGX_LD + 16 * g + 8 * h;
          ah[mb] = *reinterpret_cast<const f16x8*>(Ah + o);
          al[mb] = *reinterpret_cast<const f16x8*>(Al + o);
        }
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const f16x8 wh = Ws[((g * 4 + 2 * wn + nb) * 2 + 0) * 64 + lane];
          const f16x8 wl = Ws[((g * 4 + 2 * wn + nb) * 2 + 1) * 64 + lane];
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {
            if constexpr (NP == 3) {
              acc[mb][nb] = mfma16(wl, ah[mb], acc[mb][nb]);
              acc[mb][nb] = mfma16(wh, al[mb], acc[mb][nb]);
            }
            acc[mb][nb] = mfma16(wh, ah[mb], acc[mb][nb]);
          }
        }
      }
    }
  }
  if (!wave_on) return;
  const bool vst = (p.ldo % 4 == 0) && (p.coff % 4 == 0) && (p.Cout % 4 == 0);
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int gm = m0 + (2 * wm + mb) * 32 + col;
    if (gm >= M) continue;
    float* dst = p.out + (size_t)gm * p.ldo + p.coff;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int cb = nb0 + 2 * wn + nb;
      if (cb >= N32) break;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = cb * 32 + 8 * g + 4 * h;
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = acc[mb][nb][4 * g + j] * unscale + (c + j < p.Cout ? p.bias[c + j] : 0.f);
          o[j] = p.relu ? fmaxf(v, 0.f) : v;
        }
        if (vst) {
          if (c < p.Cout) *reinterpret_cast<f32x4*>(dst + c) = o;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c + j < p.Cout) dst[c + j] = o[j];
        }
      }
    }
  }
}

// The pointwise kernel for 5 or 6 cout blocks (161 .. 192 output channels; dense conv_6_1_1x1 fused
// with conv_6_2_1x1_1: 184 -> 64 + 96, train_dense_networks.py:343-349).  igemm_x3pw_kernel covers
// them with two 128-channel N tiles, so every pixel tile is loaded, split and staged twice and the
// second tile runs one real cout block beside a clamped copy.  Here one block owns all NB cout
// blocks of its 128 pixels: wave w runs pixel block w (32 px) x NB cout blocks, the K extent is
// loaded once.  Per output the MFMA sequence (chunk, k16 group, lo*hi, hi*lo, hi*hi) is
// igemm_x3pw_kernel's, so the result is bit for bit the same.
template <int NP, int NCH, int NB>
__global__ __launch_bounds__(256, 2) void igemm_x3pwn_kernel(IgemmArgs p, const f16x8* __restrict__ wpk, float unscale) {
  __shared__ _Float16 Ah[IG_BM * IGX_LD], Al[IG_BM * IGX_LD];
  __shared__ f16x8 Ws[2 * NB * 2 * 64];   // [k16 g][cout block nb][part][lane]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int M = p.N * p.Ho * p.Wo;
  int mt_, nt_;
  xcd_tile(p, false, mt_, nt_);
  const int m0 = mt_ * IG_BM;
  const int K16 = (p.K + 15) / 16;
  const int k4 = (tid & 7) * 4;
  f32x4 av[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = m0 + (tid >> 3) + 32 * i, k = 32 * c + k4;
      const f32x4 t =
          *reinterpret_cast<const f32x4*>(p.x + (size_t)min(gm, M - 1) * p.ldx + p.cix + min(k, p.K - 4));
      av[c][i] = (gm < M && k < p.K) ? t : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  auto load_w = [&](int k0, f16x8 (&w)[NB]) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = tid + 256 * u, l = e & 63, part = (e >> 6) & 1, q = e >> 7, g = q / NB, nb = q - g * NB;
      const int kb = min((k0 >> 4) + g, K16 - 1);
      if (NP == 3 || part == 0) w[u] = wpk[(((size_t)kb * NB + nb) * 2 + part) * 64 + l];
    }
  };
  f32x16 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x16{};
  f16x8 wnx[NB];
  load_w(0, wnx);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k0 = 32 * c;
    lds_barrier();   // the previous chunk's LDS reads are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      f16x4 hv, lv;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        hv[s] = (_Float16)av[c][i][s];
        lv[s] = (_Float16)(av[c][i][s] - (float)hv[s]);
      }
      *reinterpret_cast<f16x4*>(Ah + row * IGX_LD + k4) = hv;
      if constexpr (NP == 3) *reinterpret_cast<f16x4*>(Al + row * IGX_LD + k4) = lv;
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) Ws[tid + 256 * u] = wnx[u];
    if (c + 1 < NCH) load_w(k0 + IG_BK, wnx);
    lds_barrier();
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if ((k0 >> 4) + g >= K16) break;   // block-uniform
      const int o = (wv * 32 + col) * IGX_LD + 16 * g + 8 * h;
      const f16x8 ah = *reinterpret_cast<const f16x8*>(Ah + o);
      const f16x8 al = *reinterpret_cast<const f16x8*>(Al + o);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const f16x8 wh = Ws[((g * NB + nb) * 2 + 0) * 64 + lane];
        const f16x8 wl = Ws[((g * NB + nb) * 2 + 1) * 64 + lane];
        if constexpr (NP == 3) {
          acc[nb] = mfma16(wl, ah, acc[nb]);
          acc[nb] = mfma16(wh, al, acc[nb]);
        }
        acc[nb] = mfma16(wh, ah, acc[nb]);
      }
    }
  }
  const int gm = m0 + wv * 32 + col;
  if (gm >= M) return;
  const bool vst = (p.ldo % 4 == 0) && (p.coff % 4 == 0) && (p.Cout % 4 == 0);
  float* dst = p.out + (size_t)gm * p.ldo + p.coff;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = nb * 32 + 8 * g + 4 * h;
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = acc[nb][4 * g + j] * unscale + (c + j < p.Cout ? p.bias[c + j] : 0.f);
        o[j] = p.relu ? fmaxf(v, 0.f) : v;
      }
      if (vst) {
        if (c < p.Cout) *reinterpret_cast<f32x4*>(dst + c) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c + j < p.Cout) dst[c + j] = o[j];
      }
    }
  }
}

// Halo-tiled f16x3 convolution (stride 1, odd KS, SAME, Cin % 32 == 0, Cout > 64): the im2col
// kernels above gather, split and stage every input element once per tap (9x for 3x3); here a
// block's 128 output pixels are whole rows (NI images x R rows x W cols, 128 % W == 0) and the
// input rows they need, with their halo, are staged once per 32-channel chunk as split f16
// (pixel pitch 144 B: [hi 32][lo 32][pad], conflict-free b128 reads for a row of 32 pixels), so
// each element is converted ~1.4-2x instead of KS^2 times.  All KS^2 taps of a chunk then read
// their fragments from the same LDS image at a per-tap offset.  Double-buffered: chunk c+1's loads
// are in flight during chunk c's MFMAs and are written to the other buffer after them (one barrier
// per chunk).  Weight fragments come straight from L2 / L1 (packed [k/16][n/32][hi|lo][lane], each
// wave-load one contiguous KiB), one tap ahead.  Waves: 2 x 2 grid of 64 pixels x 64 couts.
constexpr int HX_ITEMS = 9;    // f32x4 halo items per thread per chunk (<= 2304 = 288 pixels)

struct HaloGeom {
  int R, NI, HH, WW, PH;   // rows per tile, images per tile, halo rows / cols per image, halo pixels
};

// The halo kernel's epilogue with the 2x2/2 max pool of relu(conv + bias) fused (hier: every conv
// feeds exactly one max_pool, train_hier_networks.py:536-569): the pre-pool map is never written.
// A tile is R (even) whole rows of W (even) pixels, so every pool window lies in one tile: lane
// pairs (col, col ^ 1) hold its two columns; its two rows are lanes (col, col ^ W) of one 32-pixel
// block (W <= 16), the two blocks of one wave (W = 32), or the two wave rows (W = 64, exchanged
// through LDS).  max is exact, so the pooled values are bit-identical to conv -> pool2_kernel.
__device__ __forceinline__ float dpp_xor1(float v) {   // lane ^ 1 (quad_perm [1,0,3,2])
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
// WR: the wave layout of igemm_x3h_kernel (wave rows; MBW 32-pixel blocks x NBW cout blocks per wave)
// WR = 8: NARROW1 (Cout <= 32): four waves of 32 px x 32 couts -- the NARROW layout's second cout
// block would be a clamped copy of the first (twice the MFMAs and weight loads for nothing)
template <int WR>
struct HaloLayout {
  static constexpr int MBW = WR == 8 ? 1 : 4 / WR;               // 32-pixel blocks per wave (the tile has 4)
  static constexpr int NBW = (WR == 1 || WR == 8) ? 1 : 2;       // 32-cout blocks per wave
  static constexpr int NT = WR == 8 ? 1 : (4 / WR) * NBW;        // 32-cout blocks per tile (WR = 4: 2, else 4)
};

template <int WR>
__device__ void halo_pool_epilogue(const IgemmArgs& p, f32x16 (&acc)[HaloLayout<WR>::MBW][HaloLayout<WR>::NBW],
                                   bool wave_on, float unscale, int m0, int nb0, _Float16* lds) {
  constexpr int MBW = HaloLayout<WR>::MBW, NBW = HaloLayout<WR>::NBW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int wm = wv % WR, wn = wv / WR;
  const int N32 = (p.Cout + 31) / 32, W = p.W, HW = p.H * W;
  // relu(acc * unscale + bias), then the max over the column pair
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int cb = min(nb0 + NBW * wn + nb, N32 - 1);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = cb * 32 + 8 * (e >> 2) + 4 * h + (e & 3);
        const float v = fmaxf(acc[mb][nb][e] * unscale + (c < p.Cout ? p.bias[c] : 0.f), 0.f);
        acc[mb][nb][e] = fmaxf(v, dpp_xor1(v));
      }
    }
  // the max over the row pair: lanes col ^ W (W <= 16), blocks b, b + 1 (W = 32) or b, b + 2 (W = 64)
  // of the tile's four 32-pixel blocks b = MBW wm + mb -- in-lane when one wave holds both
  if (W <= 16) {
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mb][nb][e] = fmaxf(acc[mb][nb][e], __shfl_xor(acc[mb][nb][e], W));
  } else if (W == 32) {
#pragma unroll
    for (int mb = 0; mb + 1 < MBW; mb += 2)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mb][nb][e] = fmaxf(acc[mb][nb][e], acc[mb + 1][nb][e]);
  } else if constexpr (MBW == 4) {   // W = 64, one wave holds both rows
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mb][nb][e] = fmaxf(acc[mb][nb][e], acc[mb + 2][nb][e]);
  } else {   // W = 64, 2 x 2 waves: wave row wm = 1 hands its values to wm = 0 through LDS (the halo
             // buffers are free once every wave is past its last MFMA)
    float* x = reinterpret_cast<float*>(lds);
    lds_barrier();
    if (wm == 1) {
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
          for (int e = 0; e < 16; ++e) x[(((wn * MBW + mb) * NBW + nb) * 16 + e) * 64 + lane] = acc[mb][nb][e];
    }
    lds_barrier();
    if (wm == 0) {
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            acc[mb][nb][e] = fmaxf(acc[mb][nb][e], x[(((wn * MBW + mb) * NBW + nb) * 16 + e) * 64 + lane]);
    }
  }
  if (!wave_on) return;
  const int Ho = p.H / 2, Wo = W / 2;
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    const int b = MBW * wm + mb, pp = b * 32 + col;   // block and pixel of the tile
    const int gm = m0 + pp;
    const int n = gm / HW, y = (gm - n * HW) / W, xx = gm % W;
    // the window's top-left lane writes: even column, even row (the first block of its pair)
    const bool top = (W <= 16) ? ((y & 1) == 0) : (W == 32 ? (b & 1) == 0 : b < 2);
    if ((xx & 1) || !top || gm >= p.N * HW) continue;
    float* dst = p.out + (((size_t)n * Ho + y / 2) * Wo + xx / 2) * p.ldo + p.coff;
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int cb = nb0 + NBW * wn + nb;
      if (cb >= N32) break;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = cb * 32 + 8 * g + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c + j < p.Cout) dst[c + j] = acc[mb][nb][4 * g + j];
      }
    }
  }
}

// Wave layouts (WR = wave rows along the 128 pixels): 2 = the 2 x 2 grid of 64 px x 64 couts;
// 4 = NARROW (Cout <= 64): four waves of 32 px x 64 couts, instead of a 2 x 2 grid whose second wave
// column would idle; 1 = TALL: four waves of 128 px x 32 couts -- every wave loads only its own
// cout block's weight fragments (the 2 x 2 grid has two waves load each), half the per-tap weight
// traffic from L2 / L1 for twice the LDS fragment reads
// CH: input channels per staged chunk, 32 or 16 (Cin 12 / 16 / 40 / 48 ...: the weights' per-tap rows
// padded to 16 instead of 32); a staged pixel is [hi CH][lo CH][8 pad] f16 (72 / 40: conflict-free
// b128 reads of 32 consecutive pixels either way)
template <int KS, int NP, int WR = 2, int CH = 32>
__global__ __launch_bounds__(256, 2) void igemm_x3h_kernel(IgemmArgs p, HaloGeom hg, const f16x8* __restrict__ wpk,
                                                          float unscale) {
  constexpr int MBW = HaloLayout<WR>::MBW, NBW = HaloLayout<WR>::NBW;
  constexpr int PITCH = 2 * CH + 8, QPP = CH / 4, NG = CH / 16;
  extern __shared__ _Float16 hs[];   // [2][PH][PITCH]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const int wm = wv % WR, wn = wv / WR;
  const int HW = p.H * p.W;
  const int M = p.N * HW;
  int mt_, nt_;
  xcd_tile(p, false, mt_, nt_);   // neighbouring row tiles share halo rows
  const int m0 = mt_ * IG_BM;
  const int nb0 = nt_ * HaloLayout<WR>::NT;
  const int N32 = (p.Cout + 31) / 32;
  const int pad = KS / 2;
  const int n0 = m0 / HW, y0 = (m0 - n0 * HW) / p.W;   // first image / row of the tile
  const int cinp = p.cinp ? p.cinp : p.Cin;   // channels per tap of the weight packing (% CH == 0)
  const int nchunk = cinp / CH;
  const int bufsz = hg.PH * PITCH;

  // halo staging: item e = (halo pixel e / QPP, channel quad e % QPP)
  auto load_halo = [&](int c, f32x4 (&v)[HX_ITEMS]) {
#pragma unroll
    for (int u = 0; u < HX_ITEMS; ++u) {
      const int e = tid + 256 * u;
      const int hp = e / QPP, q = e % QPP;
      const int i = hp / (hg.HH * hg.WW), r = hp - i * hg.HH * hg.WW;
      const int hy = r / hg.WW, hx = r - hy * hg.WW;
      const int n = n0 + i, y = y0 + hy - pad, x = hx - pad;
      const bool ok = hp < hg.PH && n < p.N && y >= 0 && y < p.H && x >= 0 && x < p.W && c * CH + 4 * q < p.Cin;
      const int cn = min(n, p.N - 1), cy = min(max(y, 0), p.H - 1), cx = min(max(x, 0), p.W - 1);
      const f32x4 t = *reinterpret_cast<const f32x4*>(p.x + (((size_t)cn * p.H + cy) * p.W + cx) * p.ldx + p.cix +
                                                      min(c * CH + 4 * q, p.Cin - 4));
      v[u] = ok ? t : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_halo = [&](int buf, const f32x4 (&v)[HX_ITEMS]) {
#pragma unroll
    for (int u = 0; u < HX_ITEMS; ++u) {
      const int e = tid + 256 * u;
      const int hp = e / QPP, q = e % QPP;
      if (hp >= hg.PH) continue;
      f16x4 hv, lv;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        hv[s] = (_Float16)v[u][s];
        lv[s] = (_Float16)(v[u][s] - (float)hv[s]);
      }
      _Float16* d = hs + buf * bufsz + hp * PITCH + 4 * q;
      *reinterpret_cast<f16x4*>(d) = hv;
      if constexpr (NP == 3) *reinterpret_cast<f16x4*>(d + CH) = lv;
    }
  };
  // this wave's weight fragments of (chunk c, tap t): [g][nb][hi|lo]
  auto load_w = [&](int c, int t, f16x8 (&w)[2][NBW][2]) {
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) {
        const int kb = (t * cinp + c * CH) / 16 + g, nbc = min(nb0 + NBW * wn + nb, N32 - 1);
        const f16x8* src = wpk + ((size_t)kb * N32 + nbc) * 2 * 64 + lane;
        w[g][nb][0] = src[0];
        if constexpr (NP == 3) w[g][nb][1] = src[64];
      }
  };

  // halo offset (in f16) of this lane's output pixel in each of its two 32-pixel blocks
  int pbase[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    const int pp = (MBW * wm + mb) * 32 + col;
    const int i = pp / (hg.R * p.W), r = (pp / p.W) % hg.R, x = pp % p.W;
    pbase[mb] = ((i * hg.HH + r) * hg.WW + x) * PITCH + 8 * h;
  }

  f32x16 acc[MBW][NBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) acc[mb][nb] = f32x16{};
  const bool wave_on = nb0 + NBW * wn < N32;   // wave-uniform

  f32x4 hv[HX_ITEMS];
  load_halo(0, hv);
  store_halo(0, hv);
  f16x8 wc[2][NBW][2], wnx[2][NBW][2];
  load_w(0, 0, wnx);
  lds_barrier();
  for (int c = 0; c < nchunk; ++c) {
    if (c + 1 < nchunk) load_halo(c + 1, hv);
    const _Float16* hb = hs + (c & 1) * bufsz;
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) {
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) {
          wc[g][nb][0] = wnx[g][nb][0];
          wc[g][nb][1] = wnx[g][nb][1];
        }
      if (t + 1 < KS * KS)
        load_w(c, t + 1, wnx);
      else if (c + 1 < nchunk)
        load_w(c + 1, 0, wnx);
      const int toff = ((t / KS) * hg.WW + t % KS) * PITCH;
      if (wave_on) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          f16x8 ah[MBW], al[MBW];
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) {
            ah[mb] = *reinterpret_cast<const f16x8*>(hb + pbase[mb] + toff + 16 * g);
            al[mb] = *reinterpret_cast<const f16x8*>(hb + pbase[mb] + toff + CH + 16 * g);
          }
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
            for (int mb = 0; mb < MBW; ++mb) {
              if constexpr (NP == 3) {
                acc[mb][nb] = mfma16(wc[g][nb][1], ah[mb], acc[mb][nb]);
                acc[mb][nb] = mfma16(wc[g][nb][0], al[mb], acc[mb][nb]);
              }
              acc[mb][nb] = mfma16(wc[g][nb][0], ah[mb], acc[mb][nb]);
            }
        }
      }
    }
    if (c + 1 < nchunk) {
      store_halo((c + 1) & 1, hv);   // that buffer was last read in chunk c - 1, before the last barrier
      lds_barrier();
    }
  }
  if constexpr (WR != 4 && WR != 8) {
    if (p.pool) {   // fused 2x2/2 max pool (uniform branch): the pooled map goes to the output view
      halo_pool_epilogue<WR>(p, acc, wave_on, unscale, m0, nb0, hs);
      return;
    }
  }
  if (!wave_on) return;
  const bool vst = (p.ldo % 4 == 0) && (p.coff % 4 == 0) && (p.Cout % 4 == 0);
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    const int gm = m0 + (MBW * wm + mb) * 32 + col;
    if (gm >= M) continue;
    float* dst = p.out + (size_t)gm * p.ldo + p.coff;
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int cb = nb0 + NBW * wn + nb;
      if (cb >= N32) break;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = cb * 32 + 8 * g + 4 * h;
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = acc[mb][nb][4 * g + j] * unscale + (c + j < p.Cout ? p.bias[c + j] : 0.f);
          o[j] = p.relu ? fmaxf(v, 0.f) : v;
        }
        if (vst) {
          if (c < p.Cout) *reinterpret_cast<f32x4*>(dst + c) = o;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c + j < p.Cout) dst[c + j] = o[j];
        }
      }
    }
  }
}

// 2x2 / stride 2, TF SAME (odd sizes pad one row/column after; max ignores it, avg divides by the
// in-image count), optionally followed by a per-channel affine (a folded inference BN).  One
// thread per output element; C innermost for coalescing.
__global__ void pool2_kernel(const float* __restrict__ x, int ldx, int cix, int N, int H, int W, int C,
                             float* out, int ldo, int coff, int mode, const float* __restrict__ aff_s,
                             const float* __restrict__ aff_t) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const size_t total = (size_t)N * Ho * Wo * C;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c = i % C;
  const size_t pix = i / C;
  const int ox = pix % Wo, oy = (pix / Wo) % Ho;
  const int n = pix / ((size_t)Wo * Ho);
  float best = -INFINITY, sum = 0.f;
  int cnt = 0;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int iy = 2 * oy + dy, ix = 2 * ox + dx;
      if (iy < H && ix < W) {
        const float v = x[(((size_t)n * H + iy) * W + ix) * ldx + cix + c];
        best = fmaxf(best, v);
        sum += v;
        ++cnt;
      }
    }
  float v = mode == 0 ? best : sum / (float)cnt;
  if (aff_s) v = v * aff_s[c] + aff_t[c];   // inference BN after the pool (attention net)
  out[pix * ldo + coff + c] = v;
}

hipError_t launch_igemm_conv(const IgemmArgs& a, hipStream_t st) {
  const int M = a.N * a.Ho * a.Wo;
  const int N32 = (a.Cout + 31) / 32;
  const int nb = N32 >= 4 ? 4 : (N32 >= 2 ? 2 : 1);
  dim3 grid((M + IG_BM - 1) / IG_BM, (N32 + nb - 1) / nb);
  if (nb == 4)
    hipLaunchKernelGGL(igemm_conv_kernel<4>, grid, dim3(256), 0, st, a);
  else if (nb == 2)
    hipLaunchKernelGGL(igemm_conv_kernel<2>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(igemm_conv_kernel<1>, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

namespace {
int env_flag(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// halo tiles: stride 1, SAME, odd KS in {3, 5}, Cin % 32 == 0, tiles of whole rows of one image (or
// whole images), halo within HX_ITEMS per thread and two buffers within 80 KiB
// channels per staged chunk of the halo kernel: 32 unless the weights are padded to a multiple of 16
// that is not one of 32
int halo_ch(const IgemmArgs& a) { return (a.Cin % 32 == 0 || a.cinp % 32 == 0) ? 32 : 16; }

bool halo_geom(const IgemmArgs& a, HaloGeom& hg, size_t& lds) {
  static const int halo = env_flag("MP_IGEMM_HALO", 1);
  if (!(halo && a.stride == 1 && (a.KS == 3 || a.KS == 5) && a.pad_t == a.KS / 2 && a.pad_l == a.KS / 2 &&
        a.Ho == a.H && a.Wo == a.W && a.ldx % 4 == 0 && a.cix % 4 == 0 && a.W <= IG_BM &&
        (a.Cin % 32 == 0 || (a.wpad && a.cinp % 16 == 0 && a.cinp >= a.Cin && a.Cin % 4 == 0)) &&
        IG_BM % a.W == 0))
    return false;
  const int HW = a.H * a.W;
  bool ok = true;
  if (HW >= IG_BM) {
    hg.NI = 1;
    hg.R = IG_BM / a.W;
    ok = a.H % hg.R == 0;
  } else {
    hg.NI = IG_BM / HW;
    hg.R = a.H;
    ok = IG_BM % HW == 0;
  }
  hg.HH = hg.R + a.KS - 1;
  hg.WW = a.W + a.KS - 1;
  hg.PH = hg.NI * hg.HH * hg.WW;
  const int ch = halo_ch(a);
  if (ch == 16 && a.Cout > 64) return false;   // 16-channel chunks exist for the NARROW layout only
  // the second halo buffer only exists for the next chunk: one chunk, one buffer (Cin <= 16 / 32:
  // half the LDS, so 4 instead of 3 NARROW / NARROW1 blocks fit a CU)
  const int nchunk = (a.cinp ? a.cinp : a.Cin) / ch;
  lds = (nchunk > 1 ? 2 : 1) * (size_t)hg.PH * (2 * ch + 8) * sizeof(_Float16);
  return ok && hg.PH * (ch / 4) <= 256 * HX_ITEMS && lds <= 80 * 1024;
}

// small maps (<= 8 x 8) where at least 40 % of the im2col taps are padding: position-major tiles so
// the padding taps can be skipped (measured: a 5x5 conv on 4x4 maps, 51 % padding, 1.4x faster; on
// 8x8 maps, 28 % padding, slower -- a position-major tile gathers 128 images' pixels and loses the
// neighbouring-pixel input reuse of a row-major tile)
bool pm_path(const IgemmArgs& a) {
  static const int tapskip = env_flag("MP_IGEMM_TAPSKIP", 1);
  if (!(tapskip && a.KS > 1 && a.Ho * a.Wo <= 64 && a.Cin % IG_BK == 0)) return false;
  long valid = 0;
  for (int y = 0; y < a.Ho; ++y)
    for (int x = 0; x < a.Wo; ++x)
      for (int ky = 0; ky < a.KS; ++ky)
        for (int kx = 0; kx < a.KS; ++kx) {
          const int iy = y * a.stride - a.pad_t + ky, ix = x * a.stride - a.pad_l + kx;
          valid += iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        }
  return valid * 10 <= 6L * a.Ho * a.Wo * a.KS * a.KS;
}

bool wide_path(const IgemmArgs& a) {
  static const int wide = env_flag("MP_IGEMM_WIDE", 1);
  return wide && (a.Cout + 31) / 32 >= 3;   // Cout > 64: 2 x 2 wave tiles, weights staged in LDS
}
}  // namespace

int igemm_pm_splits(const IgemmArgs& a) {
  // split K into 8 input-channel ranges by default: hier con_6 (5x5, 512 -> 1024 on 4x4 maps,
  // 256 blocks of 128 x 128 otherwise: one wave per SIMD) 0.76 -> 0.40 ms on one stream (4 splits
  // 0.42, 16 splits 0.43), and on the graph runtime's streams hier fp32 34.5k -> 37.7k crops/s,
  // bf16 53.0k -> 56.3k (round 1 had measured 4 splits slower there; MP_IGEMM_PM_SPLITS=1 for A/B)
  static const int maxs = std::max(1, env_flag("MP_IGEMM_PM_SPLITS", 8));
  if (a.K < 4 || !wide_path(a)) return 1;
  HaloGeom hg;
  size_t lds;
  if (halo_geom(a, hg, lds) || !pm_path(a)) return 1;
  int S = maxs;
  while (S > 1 && a.Cin % (S * IG_BK)) S /= 2;
  return S;
}

// K splits of the wide im2col kernel on tiny output maps (<= 4 x 4: the dense-hier scale-3 convs,
// whose Cin is often not a multiple of 32 so neither the halo nor the tap-skipping path applies:
// 32 pixel tiles x 2 cout tiles = 64 blocks at B = 256 otherwise).  A property of the layer alone
// (K, map size), never of the batch.
int igemm_x3w_splits(const IgemmArgs& a) {
  static const int on = env_flag("MP_IGEMM_SMALL_SPLITK", 1);
  if (!on || !wide_path(a) || a.Ho * a.Wo > 16 || pm_path(a)) return 1;
  HaloGeom hg;
  size_t lds;
  if (halo_geom(a, hg, lds)) return 1;
  // up to 8 slices of >= 256 (on 8 x 8 maps, up to 4 slices of >= 512 measured flat in the
  // multi-stream dense-hier schedule: 20.1k vs 20.0k crops/s)
  return std::max(1, std::min(8, a.K / 256));
}

size_t igemm_pm_part_floats(const IgemmArgs& a) {
  const int S = std::max(igemm_pm_splits(a), igemm_x3w_splits(a));
  return S > 1 ? (size_t)S * a.N * a.Ho * a.Wo * ((a.Cout + 31) / 32 * 32) : 0;
}

bool igemm_can_pool(const IgemmArgs& a) {
  if (!a.relu || a.Ho % 2 || a.Wo % 2 || !wide_path(a)) return false;
  HaloGeom hg;
  size_t lds;
  if (halo_geom(a, hg, lds)) return hg.R % 2 == 0 && a.W <= 64 && 4096 * sizeof(float) <= lds;   // W = 64 exchange
  return pm_path(a) && a.part && igemm_pm_splits(a) > 1;   // the split-K reduce pools
}

hipError_t launch_igemm_x3(const IgemmArgs& a, const void* wpk, float unscale, hipStream_t st) {
  if (a.K < 4) return hipErrorInvalidValue;   // the clamped vector load needs K >= 4
  if (a.pool && !igemm_can_pool(a)) return hipErrorInvalidValue;
  const int M = a.N * a.Ho * a.Wo;
  const int N32 = (a.Cout + 31) / 32;
  const int nb = N32 >= 4 ? 4 : (N32 >= 2 ? 2 : 1);
  dim3 grid((M + IG_BM - 1) / IG_BM, (N32 + nb - 1) / nb);
  const f16x8* w = static_cast<const f16x8*>(wpk);
  const bool one = a.nprod == 1;   // MP_DTYPE_BF16: one f16 product per MAC
  static const int xcd = env_flag("MP_IGEMM_XCD", 1);
  static const int pw = env_flag("MP_IGEMM_PW", 1);
  if (pw && a.KS == 1 && a.stride == 1 && a.Ho == a.H && a.Wo == a.W && a.pad_t == 0 && a.pad_l == 0 &&
      a.K == a.Cin && a.K <= 192 && a.Cin % 4 == 0 && a.cix % 4 == 0 && a.ldx % 4 == 0 && N32 <= 8 && !a.pool) {
    const int nch = (a.K + 31) / 32;
    const dim3 pgrid((M + IG_BM - 1) / IG_BM, (N32 + 3) / 4);   // 128-channel output tiles
    IgemmArgs pa = a;
    pa.xcd = xcd;
    // 2 .. 6 cout blocks: one block owns all of them (igemm_x3pwn_kernel).  MP_IGEMM_PWN for A/B:
    // 0 = the 2 x 2 wave grid everywhere; 1 = one block at 5 / 6 only (dense conv_6_1_1x1 0.630 ->
    // 0.420 ms); 2 = also 2 / 3, where the grid idles or clamps waves (conv_4_1_1x1 0.195 -> 0.176,
    // conv_3_1_1x1 0.127 -> 0.114, profiles/r3zp); 3 (default) = also 4 (conv_5_1_1x1 0.294 -> 0.254,
    // profiles/r3zw)
    static const int pwn = env_flag("MP_IGEMM_PWN", 3);
    if ((pwn && (N32 == 5 || N32 == 6) && nch >= 4) || (pwn >= 2 && (N32 == 2 || N32 == 3)) ||
        (pwn == 3 && N32 == 4)) {
      const dim3 ngrid((M + IG_BM - 1) / IG_BM, 1);
#define MP_PWX(NPV, NCHV, NBV) hipLaunchKernelGGL((igemm_x3pwn_kernel<NPV, NCHV, NBV>), ngrid, dim3(256), 0, st, pa, w, unscale)
#define MP_PWXB(NCHV, NBV) \
  if (one) MP_PWX(1, NCHV, NBV); else MP_PWX(3, NCHV, NBV)
#define MP_PWXN(NCHV)                  \
  switch (N32) {                       \
    case 2: MP_PWXB(NCHV, 2); break;   \
    case 3: MP_PWXB(NCHV, 3); break;   \
    case 4: MP_PWXB(NCHV, 4); break;   \
    case 5: MP_PWXB(NCHV, 5); break;   \
    default: MP_PWXB(NCHV, 6); break;  \
  }
      switch (nch) {
        case 1: MP_PWXN(1); break;
        case 2: MP_PWXN(2); break;
        case 3: MP_PWXN(3); break;
        case 4: MP_PWXN(4); break;
        case 5: MP_PWXN(5); break;
        default: MP_PWXN(6); break;
      }
#undef MP_PWXB
#undef MP_PWXN
#undef MP_PWX
      return hipGetLastError();
    }
#define MP_PW(NPV, NCHV) hipLaunchKernelGGL((igemm_x3pw_kernel<NPV, NCHV>), pgrid, dim3(256), 0, st, pa, w, unscale)
#define MP_PWN(NCHV)     \
  if (one) MP_PW(1, NCHV); \
  else MP_PW(3, NCHV)
    switch (nch) {
      case 1: MP_PWN(1); break;
      case 2: MP_PWN(2); break;
      case 3: MP_PWN(3); break;
      case 4: MP_PWN(4); break;
      case 5: MP_PWN(5); break;
      default: MP_PWN(6); break;
    }
#undef MP_PWN
#undef MP_PW
    return hipGetLastError();
  }
  HaloGeom hg;
  size_t lds = 0;
  // halo tiles for Cout > 64, and (MP_IGEMM_HALO_NARROW, on by default) for Cout <= 64 with the
  // four waves along the pixels (igemm_x3h_kernel<.., NARROW>): the im2col kernel gathers every
  // input element KS^2 times
  static const int narrow = env_flag("MP_IGEMM_HALO_NARROW", 1);
  // (zero-padded Cin costs MFMAs: Cin = 12 padded to 32 was 2.7x and lost; the narrow halo path is
  // taken where the padded channels are at most 4/3 of Cin -- 16-channel chunks make that 12 -> 16,
  // 24 -> 32, 40 / 48 -> 48)
  if ((wide_path(a) || (narrow && (a.Cin % 32 == 0 || 3 * (a.cinp ? a.cinp : a.Cin) <= 4 * a.Cin))) &&
      halo_geom(a, hg, lds)) {
    {
      static const bool attr = [] {
        for (const void* f : {reinterpret_cast<const void*>(igemm_x3h_kernel<3, 3, 2>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 3, 2>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 1, 2>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 1, 2>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 3, 4>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 3, 4>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 1, 4>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 1, 4>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 3, 1>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 3, 1>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 1, 1>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 1, 1>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 3, 4, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 3, 4, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 1, 4, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 1, 4, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 3, 8, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 1, 8, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 3, 8, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 1, 8, 16>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 3, 8>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<3, 1, 8>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 3, 8>),
                              reinterpret_cast<const void*>(igemm_x3h_kernel<5, 1, 8>)})
          (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
        return true;
      }();
      (void)attr;
      static const int tall = env_flag("MP_IGEMM_HALO_TALL", 1);
      const dim3 hgrid((M + IG_BM - 1) / IG_BM, N32 <= 2 ? 1 : (N32 + 3) / 4);
      IgemmArgs h = a;
      h.xcd = xcd;
      if (a.Cin % 32) {
        w = static_cast<const f16x8*>(a.wpad);   // per-tap Cin rows padded to cinp (halo_geom checked)
      } else {
        h.cinp = 0;
      }
#define MP_HALO(KSV, NPV, WRV, CHV) \
  hipLaunchKernelGGL((igemm_x3h_kernel<KSV, NPV, WRV, CHV>), hgrid, dim3(256), lds, st, h, hg, w, unscale)
#define MP_HALO_WRC(WRV, CHV)                    \
  if (a.KS == 3 && one) MP_HALO(3, 1, WRV, CHV); \
  else if (a.KS == 3) MP_HALO(3, 3, WRV, CHV);   \
  else if (one) MP_HALO(5, 1, WRV, CHV);         \
  else MP_HALO(5, 3, WRV, CHV)
#define MP_HALO_WR(WRV) MP_HALO_WRC(WRV, 32)
      static const int narrow1 = env_flag("MP_IGEMM_HALO_NARROW1", 1);
      if (narrow1 && N32 == 1 && !a.pool && halo_ch(a) == 16) {   // Cout <= 32 (NARROW1)
        MP_HALO_WRC(8, 16);
      } else if (narrow1 && N32 == 1 && !a.pool) {
        MP_HALO_WR(8);
      } else if (N32 <= 2 && halo_ch(a) == 16) {   // Cout <= 64, 16-channel chunks
        MP_HALO_WRC(4, 16);
      } else if (N32 <= 2) {   // Cout <= 64
        MP_HALO_WR(4);
      } else if (tall) {
        MP_HALO_WR(1);
      } else {
        MP_HALO_WR(2);
      }
#undef MP_HALO_WR
#undef MP_HALO_WRC
#undef MP_HALO
      return hipGetLastError();
    }
  }
  if (wide_path(a)) {
    IgemmArgs b = a;
    b.xcd = xcd;
    b.pmajor = pm_path(a) ? 1 : 0;
    const int S = b.pmajor && a.part ? igemm_pm_splits(a) : 1;
    if (S > 1) {
      // split-K over input-channel ranges (z = range): raw partial sums to a.part, then a fixed-order
      // reduce with the epilogue -- 4x the blocks for the under-filled small-map convs (hier con_6:
      // 256 blocks of 128 x 128 on 256 CUs otherwise)
      const dim3 sgrid((M + IG_BM - 1) / IG_BM, (N32 + 3) / 4, S);
      if (one)
        hipLaunchKernelGGL(igemm_x3w_pm_kernel<1>, sgrid, dim3(256), 0, st, b, w, unscale);
      else
        hipLaunchKernelGGL(igemm_x3w_pm_kernel<3>, sgrid, dim3(256), 0, st, b, w, unscale);
      const size_t total = (size_t)M * (N32 * 8);
      hipLaunchKernelGGL(igemm_pm_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, b, S, unscale);
      return hipGetLastError();
    }
    const int S2 = !b.pmajor && a.part ? igemm_x3w_splits(a) : 1;
    if (S2 > 1) {
      const dim3 sgrid((M + IG_BM - 1) / IG_BM, (N32 + 3) / 4, S2);
      if (one)
        hipLaunchKernelGGL(igemm_x3w_kernel<1>, sgrid, dim3(256), 0, st, b, w, unscale);
      else
        hipLaunchKernelGGL(igemm_x3w_kernel<3>, sgrid, dim3(256), 0, st, b, w, unscale);
      const size_t total = (size_t)M * (N32 * 8);
      hipLaunchKernelGGL(igemm_split_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, b, S2, unscale);
      return hipGetLastError();
    }
    b.part = nullptr;
    const dim3 wgrid((M + IG_BM - 1) / IG_BM, (N32 + 3) / 4);
    if (b.pmajor && one)
      hipLaunchKernelGGL(igemm_x3w_pm_kernel<1>, wgrid, dim3(256), 0, st, b, w, unscale);
    else if (b.pmajor)
      hipLaunchKernelGGL(igemm_x3w_pm_kernel<3>, wgrid, dim3(256), 0, st, b, w, unscale);
    else if (one)
      hipLaunchKernelGGL(igemm_x3w_kernel<1>, wgrid, dim3(256), 0, st, b, w, unscale);
    else
      hipLaunchKernelGGL(igemm_x3w_kernel<3>, wgrid, dim3(256), 0, st, b, w, unscale);
    return hipGetLastError();
  }
  if (nb == 4 && one)
    hipLaunchKernelGGL((igemm_x3_kernel<4, 1>), grid, dim3(256), 0, st, a, w, unscale);
  else if (nb == 4)
    hipLaunchKernelGGL((igemm_x3_kernel<4, 3>), grid, dim3(256), 0, st, a, w, unscale);
  else if (nb == 2 && one)
    hipLaunchKernelGGL((igemm_x3_kernel<2, 1>), grid, dim3(256), 0, st, a, w, unscale);
  else if (nb == 2)
    hipLaunchKernelGGL((igemm_x3_kernel<2, 3>), grid, dim3(256), 0, st, a, w, unscale);
  else if (one)
    hipLaunchKernelGGL((igemm_x3_kernel<1, 1>), grid, dim3(256), 0, st, a, w, unscale);
  else
    hipLaunchKernelGGL((igemm_x3_kernel<1, 3>), grid, dim3(256), 0, st, a, w, unscale);
  return hipGetLastError();
}

hipError_t launch_pool2(const float* x, int ldx, int cix, int N, int H, int W, int C, float* out, int ldo,
                        int coff, int mode, hipStream_t st, const float* aff_s, const float* aff_t) {
  const size_t total = (size_t)N * ((H + 1) / 2) * ((W + 1) / 2) * C;
  hipLaunchKernelGGL(pool2_kernel, dim3((total + 255) / 256), dim3(256), 0, st, x, ldx, cix, N, H, W, C, out,
                     ldo, coff, mode, aff_s, aff_t);
  return hipGetLastError();
}

}  // namespace mp
