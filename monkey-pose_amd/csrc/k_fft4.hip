// Four-step FFT loop of the hGRU association-field convolution: the fp32 FFT path's default loop
// (MP_DTYPE_F32_FFT; MP_FFT4=0 restores k_fft.hip's six-launch loop for A/B).
//
// The eCRF convolution (hgru_module.py:615-657 p_convolution / process_p: tf.nn.conv2d SAME, 15x15
// taps, 64 -> 64 channels, twice per timestep) on a 64x64 map is a 72 x 72 circular convolution
// (k_fft.hip's header: why that is exact).  Here the 72-point COLUMN transform is split in two
// (y = 8 n1 + n2, fy = k1 + 9 k2; W_N = e^{-2 pi i / N}):
//   X[k1 + 9 k2] = sum_{n2<8} W8^{n2 k2} W72^{n2 k1} sum_{n1<9} x[8 n1 + n2] W9^{n1 k1}
// so that the kernels on either side of the spectral GEMM each hold everything their math needs:
//   row kernel  (image b, row class n2): the 8 rows y = 8 n1 + n2 with ALL 64 channels -- the row
//               transforms, the 9-point sums over n1, and every per-pixel channel mix (the 1x1 gates
//               of hgru_module.py:696-711, 729-740), so the B half-step's epilogue runs between its
//               inverse and the next step's forward transform without a map round trip;
//   col kernel  (column fx, class k1, 16 images): the 8 frequencies fy = k1 + 9 k2 with all 64
//               channels -- the twiddles W72^{n2 k1}, the 8-point sums over n2 and the per-frequency
//               64 x 64 complex GEMM (f16x3, k_fft.hip spec_gemm_kernel's fragments).
// One timestep is four launches (hgru_module.py:825-857):
//   col: Z -> Z'   row_a: Z', X, O -> I, Z   col: Z -> Z'   row_b: Z', I, O -> O', Z
// Z = [b][fx][k1][n2][64 channels] complex64 (1.36 MB per image, a spectrum's size) carries the
// partial transforms between them IN PLACE: every block reads exactly the elements it writes.  Per
// image and step: 8 spectra + 6 maps of traffic (17.2 MB) instead of the six-launch loop's 8 + 10
// (22.1 MB): P2 and the gated state Og never reach HBM.  The numerics are the six-launch loop's (fp32
// transforms, twiddles rounded once from double, the same f16x3 spectral GEMM and gate GEMMs, the same
// epilogue expressions); only the transforms' association order differs (~1e-7 relative).
#include "fft_dev.hpp"

namespace mp {

constexpr int Z_CLS = FX * 9;                        // 333 (fx, k1) column classes
constexpr int RK_ITEMS = FX * 64;                    // (fx, channel) columns of the 9-point passes: 2368
constexpr int RK_T = 8 * FX * 64;                    // T[n1][fx][c] complex: 151,552 B of LDS
constexpr int RK_SP = 68;                            // staging pitch (floats) per pixel (16-B fragment reads)

// complex index of channel 0 of Z[b][fx][k1][n2] (ZLAYOUT 1, the default: a column block's 8 row
// classes of one image are one contiguous 4-KB run; interleaved same-box A/B 8.21 -> 8.15 ms per fp32
// forward, bf16 unchanged, profiles/r5_ab/r5s2) or of Z[b][n2][fx][k1] (ZLAYOUT 0: a row block's
// (b, n2) slice contiguous)
#ifndef ZLAYOUT
#define ZLAYOUT 1
#endif
__device__ __forceinline__ size_t z_off(int b, int n2, int fx, int k1) {
  if constexpr (ZLAYOUT == 1) return ((((size_t)b * FX + fx) * 9 + k1) * 8 + n2) * 64;
  return ((((size_t)b * 8 + n2) * FX + fx) * 9 + k1) * 64;
}
constexpr int Z_K1 = ZLAYOUT == 1 ? 8 * 64 : 64;   // complex stride between consecutive k1

enum { ROW_A = 0, ROW_B = 1, ROW_FINAL = 2, ROW_INIT = 3 };

// a value the compiler cannot see through: index math re-derived from it in a later phase is not
// CSE'd with an earlier phase's (which would hold 64-bit item addresses live across the whole kernel),
// and loads through a pointer passed through it are not hoisted out of their loop
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ int opaque_s(int v) {   // the same for a wave-uniform (SGPR) value
  asm volatile("" : "+s"(v));
  return v;
}
template <typename P>
__device__ __forceinline__ P* opaque_ptr(P* p) {
  asm volatile("" : "+s"(p));
  return p;
}

// an fp32 x4 load, non-temporal under NT (the maps' policy: fft_dev.hpp map_ld4)
template <bool NT>
__device__ __forceinline__ f32x4 ld4(const float* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  else return *reinterpret_cast<const f32x4*>(p);
}

// Packed-FP32 forms of the epilogues' elementwise math: two channels per v_pk_{add,mul,fma}_f32, the
// transcendentals (v_exp_f32, v_rcp_f32) per channel as in fsigmoid / ftanh.  Same operations and
// contractions per channel as the scalar expressions.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pr2(const f32x4& v, int i) { return f2v{v[2 * i], v[2 * i + 1]}; }
__device__ __forceinline__ f2v pr16(const f32x16& v, int i) { return f2v{v[2 * i], v[2 * i + 1]}; }
__device__ __forceinline__ f2v rcp2(f2v x) { return f2v{__builtin_amdgcn_rcpf(x[0]), __builtin_amdgcn_rcpf(x[1])}; }
__device__ __forceinline__ f2v exp2v(f2v x) { return f2v{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])}; }
constexpr float LOG2E = 1.44269504088896340736f;
__device__ __forceinline__ f2v fsigmoid2(f2v x) { return rcp2(1.f + exp2v(-x * LOG2E)); }
__device__ __forceinline__ f2v ftanh2(f2v x) { return 1.f - 2.f * rcp2(1.f + exp2v((2.f * x) * LOG2E)); }

// II: a wave's 32-pixel segments (columns xs + j of its row), lane (h, j), register r of block n =
// channel 32 n + 8 (r >> 2) + 4 h + (r & 3) -- k_fft.hip spec_epi_b_kernel's layout and expressions,
// P read from (and the epilogue's output written back to) the staging.  The segment's map loads
// (A: X, O; B: I, O; INIT: O0) in SegIn.
struct SegIn {
  f32x4 a[2][4], o[2][4];
};

// the segment at map row y, columns xs .. xs + 31 (lane (h, j): pixel xs + j); O is loaded here with
// the other map (B modes: before the o_r gate rather than eight dependent loads after it)
template <int MODE, bool BM = false, bool NT = false>
__device__ __forceinline__ void rk_load_seg(const ConvArgs& p, const float* __restrict__ O0, int b, int y, int xs,
                                            int lane, SegIn& L) {
  const int H = p.H, W = p.W;
  const int h = lane >> 5, x = xs + (lane & 31);
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if constexpr (MODE == ROW_INIT) {
        L.a[n][g] = ld4<NT>(O0 + (((size_t)b * H + y) * W + x) * C + 32 * n + 8 * g + 4 * h);
      } else {
        L.a[n][g] = MODE == ROW_A ? map_ld4<BM, NT>(p.X, xx_index(b, 4 * n + g, y, x, 4 * h, H, W))
                                  : map_ld4<BM, NT>(p.I, ii_index(b, 4 * n + g, y, x, 4 * h, H, W));
        if (!BM && p.o_nhwc)   // step 0: O0 as given (NHWC fp32), not copied into the C8 map first
          L.o[n][g] = ld4<NT>(p.O + (((size_t)b * H + y) * W + x) * C + 32 * n + 8 * g + 4 * h);
        else
          L.o[n][g] = map_ld4<BM, NT>(p.O, oo_index(b, 4 * n + g, y, x, 4 * h, H, W));
      }
    }
}

// seg: the segment's 32 staged pixels (pitch RK_SP floats); the output goes back over the input
// LEAN: a scheduling fence after every 4-channel group, so the compiler does not hoist all eight groups'
// address math and LDS reads at once (the register budget next to the row's 64 values)
template <int MODE, bool LEAN = false, bool BM = false, bool NT = false>
__device__ __forceinline__ void rk_segment(const ConvArgs& p, float* seg, int b, int y, int xs, int lane,
                                           const SegIn& L, const void* __restrict__ or_x3, float or_us,
                                           const void* __restrict__ ir_x3, float ir_us, const float* vec) {
  const int h = lane >> 5, j = lane & 31, H = p.H, W = p.W;
  const int x = xs + j;
  float* sp = seg + j * RK_SP;
  // LEAN: the gate weights (LDS) are re-read per segment instead of 128 registers held across the kernel
  // (an opaque OFFSET, not an opaque pointer: the pointer keeps its LDS provenance, so the loads stay
  // ds_read_b128 -- through an opaque pointer they became flat loads, each followed by an
  // s_waitcnt vmcnt(0) lgkmcnt(0) that drained the block's outstanding map loads and stores)
  const void* orw = LEAN ? static_cast<const void*>(static_cast<const char*>(or_x3) + opaque_s(0)) : or_x3;
  const void* irw = LEAN ? static_cast<const void*>(static_cast<const char*>(ir_x3) + opaque_s(0)) : ir_x3;
  if constexpr (MODE == ROW_A) {
    // hgru_module.py:797-799: I = tanh(X - (beta O + nu) (P1 + lateral_bias))
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * n + 8 * g + 4 * h;
        const f32x4 pv = *reinterpret_cast<const f32x4*>(sp + c);
        const f32x4 lat = *reinterpret_cast<const f32x4*>(vec + V_LAT * 64 + c);
        const f32x4 be = *reinterpret_cast<const f32x4*>(vec + V_BETA * 64 + c);
        const f32x4 nu = *reinterpret_cast<const f32x4*>(vec + V_NU * 64 + c);
        f32x4 iv;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f2v x = pr2(L.a[n][g], q), o = pr2(L.o[n][g], q);
          const f2v t = ftanh2(-(pr2(be, q) * o + pr2(nu, q)) * (pr2(pv, q) + pr2(lat, q)) + x);
          iv[2 * q] = t[0];
          iv[2 * q + 1] = t[1];
        }
        map_st4<BM, NT>(p.dst, ii_index(b, 4 * n + g, y, x, 4 * h, H, W), iv);
        *reinterpret_cast<f32x4*>(sp + c) = iv;
        if constexpr (LEAN) __builtin_amdgcn_sched_barrier(0);
      }
  } else if constexpr (MODE == ROW_INIT) {
    // hgru_module.py:696-711 on O0 (NHWC): O = O0, Og = O0 * sigmoid(O0 . i_r + i_b)
    f32x16 V[2], Y[2];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) V[n][4 * g + e] = L.a[n][g][e];
    gate_any<BM>(irw, V, Y, lane, ir_us);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * n + 8 * g + 4 * h;
        const f32x4 ib = *reinterpret_cast<const f32x4*>(vec + V_IB * 64 + c);
        f32x4 o, og;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f2v ov = pr16(V[n], 2 * g + q), t = ov * fsigmoid2(pr16(Y[n], 2 * g + q) + pr2(ib, q));
          o[2 * q] = ov[0];
          o[2 * q + 1] = ov[1];
          og[2 * q] = t[0];
          og[2 * q + 1] = t[1];
        }
        if (p.dst) map_st4<BM, NT>(p.dst, oo_index(b, 4 * n + g, y, x, 4 * h, H, W), o);   // (null: O0 read directly)
        *reinterpret_cast<f32x4*>(sp + c) = og;
        if constexpr (LEAN) __builtin_amdgcn_sched_barrier(0);
      }
  } else {
    // hgru_module.py:729-740, 806-849: g2 = sigmoid(I . o_r + o_b); e = gamma (P2 + lat);
    // O' = (g2 O + (1 - g2) tanh(kappa (I + e) + omega (I e))) rho[t];  then Og' = O' sigmoid(O' . i_r + i_b)
    f32x16 Iv[2], Y[2];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) Iv[n][4 * g + e] = L.a[n][g][e];
    gate_any<BM>(orw, Iv, Y, lane, or_us);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * n + 8 * g + 4 * h;
        const f32x4 pv = *reinterpret_cast<const f32x4*>(sp + c);
        const f32x4 ov = L.o[n][g];
        const f32x4 lat = *reinterpret_cast<const f32x4*>(vec + V_LAT * 64 + c);
        const f32x4 ga = *reinterpret_cast<const f32x4*>(vec + V_GAMMA * 64 + c);
        const f32x4 ka = *reinterpret_cast<const f32x4*>(vec + V_KAPPA * 64 + c);
        const f32x4 om = *reinterpret_cast<const f32x4*>(vec + V_OMEGA * 64 + c);
        const f32x4 ob = *reinterpret_cast<const f32x4*>(vec + V_OB * 64 + c);
        f32x4 o;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rr = 4 * g + 2 * q;
          const f2v g2 = fsigmoid2(pr16(Y[n], 2 * g + q) + pr2(ob, q));
          const f2v iv = pr16(Iv[n], 2 * g + q);
          const f2v ee = pr2(ga, q) * (pr2(pv, q) + pr2(lat, q));
          const f2v S = ftanh2(pr2(ka, q) * (iv + ee) + pr2(om, q) * (iv * ee));
          const f2v on = (g2 * pr2(ov, q) + (1.f - g2) * S) * p.rho;
          o[2 * q] = on[0];
          o[2 * q + 1] = on[1];
          Iv[n][rr] = on[0];
          Iv[n][rr + 1] = on[1];
        }
        // ROW_FINAL with p.dst == nullptr: O_T only feeds BN_3 (no per-step states asked for), so the
        // C8 state map is not written (wave-uniform)
        if (MODE != ROW_FINAL || p.dst) map_st4<BM, NT>(p.dst, oo_index(b, 4 * n + g, y, x, 4 * h, H, W), o);
        if constexpr (LEAN) __builtin_amdgcn_sched_barrier(0);
      }
    f32x16 (&Ov)[2] = Iv;
    if constexpr (MODE == ROW_B) {
      gate_any<BM>(irw, Ov, Y, lane, ir_us);
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 32 * n + 8 * g + 4 * h;
          const f32x4 ib = *reinterpret_cast<const f32x4*>(vec + V_IB * 64 + c);
          f32x4 o;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f2v t = pr16(Ov[n], 2 * g + q) * fsigmoid2(pr16(Y[n], 2 * g + q) + pr2(ib, q));
            o[2 * q] = t[0];
            o[2 * q + 1] = t[1];
          }
          *reinterpret_cast<f32x4*>(sp + c) = o;
          if constexpr (LEAN) __builtin_amdgcn_sched_barrier(0);
        }
    } else {
      // ROW_FINAL: BN_3(O_T) (hgru_pose.py:82-90) as the NHWC fp32 map fc_1 flattens (mode 1) or as
      // fc_1's f16 hi / lo planes (mode 2); the segment's 32 pixels x 64 channels are one contiguous
      // 8 KiB run of the output, staged here and stored with contiguous lanes
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 32 * n + 8 * g + 4 * h;
          const f32x4 ss = *reinterpret_cast<const f32x4*>(vec + V_OUTS * 64 + c);
          const f32x4 tt = *reinterpret_cast<const f32x4*>(vec + V_OUTT * 64 + c);
          f32x4 o;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f2v t = pr16(Ov[n], 2 * g + q) * pr2(ss, q) + pr2(tt, q);
            o[2 * q] = t[0];
            o[2 * q + 1] = t[1];
          }
          *reinterpret_cast<f32x4*>(sp + c) = o;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const float* run = seg;
      const size_t e0 = (((size_t)b * H + y) * W + xs) * C;
      if (p.mode != 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {   // 8 x 1 KiB
          const int q = k * 64 + lane, pp = q >> 4, c4 = (q & 15) * 4;
          *reinterpret_cast<f32x4*>(p.dst2 + e0 + pp * C + c4) = *reinterpret_cast<const f32x4*>(run + pp * RK_SP + c4);
        }
      } else {   // fc_1's split planes, split exactly as fc_gemm_x3_kernel splits (k_fc.hip)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = k * 64 + lane, pp = q >> 3, c8 = (q & 7) * 8;
          const f32x4 a = *reinterpret_cast<const f32x4*>(run + pp * RK_SP + c8);
          const f32x4 bq = *reinterpret_cast<const f32x4*>(run + pp * RK_SP + c8 + 4);
          f16x8 hv, lv;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = e < 4 ? a[e] : bq[e - 4];
            hv[e] = (_Float16)v;
            lv[e] = (_Float16)(v - (float)hv[e]);
          }
          *reinterpret_cast<f16x8*>(reinterpret_cast<_Float16*>(p.dst2) + e0 + pp * C + c8) = hv;
          if (p.dst3) *reinterpret_cast<f16x8*>(reinterpret_cast<_Float16*>(p.dst3) + e0 + pp * C + c8) = lv;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

// ---------------------------------------------------------------------------------------------
// one real row of 72 points per lane: a 36-point complex transform of the even / odd
// samples packed as z[m] = x[2m] + i x[2m+1] and the split by W72^k, half the registers of fft72 on a
// packed pair of rows (72 instead of 144 values)
// ---------------------------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void dft4(cpx (&x)[4]) {
  const cpx a0 = x[0] + x[2], a1 = x[0] - x[2], a2 = x[1] + x[3], v3 = swp(x[1] - x[3]);
  x[0] = a0 + a2;
  x[2] = a0 - a2;
  x[1] = cfma(v3, cpx{(float)-S, (float)S}, a1);   // a1 + rotq(x1 - x3), one fma (exact product)
  x[3] = cfma(v3, cpx{(float)S, (float)-S}, a1);
}

// 36-point DFT, X[k] = sum_n v[n] e^{S 2 pi i n k / 36}: Good-Thomas 36 = 4 x 9 (gcd 1),
// n = (9 n1 + 4 n2) mod 36, k = (9 k1 + 28 k2) mod 36 -- no twiddles between the passes
template <int S>
__device__ __forceinline__ void fft36(cpx (&v)[36]) {
  cpx a[9][4];
#pragma unroll
  for (int n2 = 0; n2 < 9; ++n2) {
    cpx t[4];
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) t[n1] = v[(9 * n1 + 4 * n2) % 36];
    dft4<S>(t);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) a[n2][k1] = t[k1];
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    cpx u[9];
#pragma unroll
    for (int n2 = 0; n2 < 9; ++n2) u[n2] = a[n2][k1];
    dft9<S>(u);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) v[(9 * k1 + 28 * k2) % 36] = u[k2];
  }
}

// forward real transform: x[0..63] (x[64..71] = 0) -> X[k] = sum_n x[n] W72^{nk}, k = 0..36
__device__ __forceinline__ void rfft72_fwd(const float (&x)[64], cpx (&X)[FX]) {
  cpx z[36];
#pragma unroll
  for (int m = 0; m < 36; ++m) z[m] = m < 32 ? cpx{x[2 * m], x[2 * m + 1]} : cpx{0.f, 0.f};
  fft36<-1>(z);
#pragma unroll
  for (int k = 0; k < FX; ++k) {
    // E[k] = (Z[k] + conj Z[36-k]) / 2, O[k] = (Z[k] - conj Z[36-k]) / 2i, X[k] = E[k] + W72^k O[k]
    // = E + d w with d = Z[k] - conj Z[36-k] and w = W72^k / 2i = (-sin / 2, -cos / 2) (k 2 pi / 72):
    // two fmas on d and swp(d) after E, no separate twiddle product
    const cpx zk = z[k % 36], zm = z[(36 - k) % 36];
    const cpx E = cfma(zm, cpx{0.5f, -0.5f}, zk * 0.5f);             // (zk + conj zm) / 2, exact halving
    const cpx d = cfma(zm, cpx{-1.f, 1.f}, zk);                       // zk - conj zm
    const float wc = 0.5f * TW72_COS[k], ws = 0.5f * TW72_SIN[k];
    X[k] = cfma(swp(d), cpx{wc, -wc}, cfma(d, cpx{-ws, -ws}, E));
  }
}

// inverse real transform: X[0..36] (Hermitian half spectrum) -> x[n] = sum_{k<72} X[k] W72^{-nk}, n < 64
__device__ __forceinline__ void rfft72_inv(const cpx (&X)[FX], float (&x)[64]) {
  cpx z[36];
#pragma unroll
  for (int k = 0; k < 36; ++k) {
    // x[2m] = IDFT36(E), x[2m+1] = IDFT36(O): E[k] = X[k] + conj X[36-k], O[k] = (X[k] - conj X[36-k]) W72^{-k}
    // E + i O = E + D (i W72^{-k}), D = a - conj c, i W72^{-k} = (-sin, cos) (k 2 pi / 72)
    const cpx a = X[k], c = X[36 - k];
    const cpx E = cfma(c, cpx{1.f, -1.f}, a);                         // (a.x + c.x, a.y - c.y)
    const cpx D = cfma(c, cpx{-1.f, 1.f}, a);                         // (a.x - c.x, a.y + c.y)
    const float wc = TW72_COS[k], ws = TW72_SIN[k];
    z[k] = cfma(swp(D), cpx{-wc, wc}, cfma(D, cpx{-ws, -ws}, E));
  }
  fft36<1>(z);
#pragma unroll
  for (int m = 0; m < 32; ++m) {
    x[2 * m] = z[m].x;
    x[2 * m + 1] = z[m].y;
  }
}

// Z element access: complex64 (fp32 path) or one bf16 (re, im) pair (MP_DTYPE_BF16: round to nearest
// even on store, exact on load), at the same complex index
// NT: non-temporal (streaming) access
template <bool BF, bool NT = false>
__device__ __forceinline__ cpx z_ld(const void* Z, size_t i) {
  if constexpr (BF) {
    const uint32_t* p = static_cast<const uint32_t*>(Z) + i;
    return unpack_bf2(NT ? __builtin_nontemporal_load(p) : *p);
  } else {
    const cpx* p = static_cast<const cpx*>(Z) + i;
    return NT ? __builtin_nontemporal_load(p) : *p;
  }
}
template <bool BF, bool NT = false>
__device__ __forceinline__ void z_st(void* Z, size_t i, cpx v) {
  if constexpr (BF) {
    uint32_t* p = static_cast<uint32_t*>(Z) + i;
    const uint32_t u = pack_bf2(v.x, v.y);
    if constexpr (NT) __builtin_nontemporal_store(u, p);
    else *p = u;
  } else {
    cpx* p = static_cast<cpx*>(Z) + i;
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
  }
}

// ---------------------------------------------------------------------------------------------
// row kernel (row8_kernel).  Block = (image b, row class n2), 512 threads; wave w owns row n1 = w
// (map row y = 8 w + n2), lane c its channel c; one block per CU (the whole T, 151.5 KB):
//   Ia  items (fx, c): inverse 9-point sums over k1 of Z'[b][n2][fx][.][c] -> T[n1][fx][c]
//   Ib  lane c: its row's inverse real transform (rfft72_inv) -> P[x]
//   II  the half-step's epilogue on two 32-pixel segments in the MFMA accumulator layout (rk_segment),
//       P staged through LDS, the 1x1 gates' weights read from LDS
//   III lane c: forward real transform of the epilogue's output -> T; items (fx, c): forward 9-point
//       sums over n1 -> Z[b][fx][k1][n2][c]
// Round 5 measured two other forms and removed them: a four-wave block with the whole T (one row
// pair per wave) and a two-blocks-per-CU block with half of T (two transpose rounds; register
// spills): B = 256 fp32 9.61 ms per forward against this kernel's 9.04 (profiles/r5d).
// ---------------------------------------------------------------------------------------------
constexpr int R8_NT = 512;
constexpr int R8_NIT = (RK_ITEMS + R8_NT - 1) / R8_NT;   // 5

// LDS of row8_kernel: T[n1][fx][c] (151.5 KB) for the two transposes; during the epilogue its first
// 69.6 KB hold one 32-pixel staging segment per wave and the next 32 KB the two gates' packed weights
// (read from L2 once per block instead of once per segment and wave: 0.5 MB less L2 traffic a block)
// (ROW_FINAL, one gate: a whole 64-pixel row per wave, so no row stays in registers across the epilogue)
constexpr int R8_GATE = 2 * 4 * 2 * 64;                  // f16x8 of one gate's f16x3 pack (gate_x3_bytes / 16)
constexpr int R8_T = (8 * 64 * RK_SP * 4 + R8_GATE * 16) / 8;   // 155,648 B: T grown by 512 B for FINAL
static_assert(R8_T >= RK_T && (8 * 32 * RK_SP * 4 + 2 * R8_GATE * 16) <= R8_T * 8, "staging + gate weights fit");

#ifndef R8_INIT_MNT   // (A/B) row(INIT) follows the maps' policy too
#define R8_INIT_MNT 0
#endif
#ifndef R8_SEGPF
#define R8_SEGPF 0
#endif
// BF: MP_DTYPE_BF16 -- Z and the hGRU maps in bf16, the gates one bf16 product (gate_bf); transforms,
// epilogue math and the NHWC output fp32
// ZNT: Z read and written non-temporal (MP_ROW8_ZNT); MNT: the fp32 maps (X, O, I, O0) too (MP_MAP_NT)
template <int MODE, bool BF = false, bool ZNT = false, bool MNT = false>
__global__ __launch_bounds__(R8_NT, 1) void row8_kernel(void* __restrict__ Z, ConvArgs p, const void* __restrict__ or_x3,
                                                        float or_us, const void* __restrict__ ir_x3, float ir_us,
                                                        const float* __restrict__ O0) {
  __shared__ cpx T[R8_T];
  __shared__ float vsh[V_COUNT * 64];
  const int b = blockIdx.x >> 3, n2 = blockIdx.x & 7;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < V_COUNT * 64; i += R8_NT) vsh[i] = p.vecs[i];
  const int H = p.H, W = p.W;
  const int y = 8 * w + n2;
  const bool live = y < H;
  cpx* slot = T + w * FX * 64;
  constexpr int SPIX = MODE == ROW_FINAL ? 64 : 32;                        // staged pixels per wave
  float* stg = reinterpret_cast<float*>(T) + w * SPIX * RK_SP;             // epilogue staging (after Ib)
  uint4* gsh = reinterpret_cast<uint4*>(reinterpret_cast<float*>(T) + 8 * SPIX * RK_SP);   // gate weights
  constexpr bool OR = MODE == ROW_B || MODE == ROW_FINAL, IR = MODE == ROW_B || MODE == ROW_INIT;
  constexpr int GN = BF ? R8_GATE / 2 : R8_GATE;   // uint4 per gate (bf16: one product, no lo plane)
  float P[64];
  constexpr bool SEGPF = R8_SEGPF && (MODE == ROW_A || MODE == ROW_B);
  constexpr bool MNTM = MNT && (R8_INIT_MNT || MODE != ROW_INIT);   // this mode's map policy
  SegIn L0;
  if constexpr (MODE != ROW_INIT) {
    {
      cpx u[R8_NIT][9];
#pragma unroll
      for (int it = 0; it < R8_NIT; ++it) {
        const int i = min(it * R8_NT + tid, RK_ITEMS - 1);
        const size_t src = z_off(b, n2, i >> 6, 0) + (i & 63);
#pragma unroll
        for (int k1 = 0; k1 < 9; ++k1) u[it][k1] = z_ld<BF, ZNT>(Z, src + k1 * Z_K1);
      }
#pragma unroll
      for (int it = 0; it < R8_NIT; ++it) {
        const int i = it * R8_NT + tid;
        dft9<1>(u[it]);
        if (i < RK_ITEMS) {
          const int fx = i >> 6, c = i & 63;
#pragma unroll
          for (int r = 0; r < 8; ++r) T[(r * FX + fx) * 64 + c] = u[it][r];
        }
      }
    }
    lds_barrier();
    // R8_SEGPF (A/B, default 0): the first epilogue segment's maps requested here, during the inverse
    // row transforms instead of in front of the segment.  Same box, B = 256: row A 0.272 ms either
    // way, row B 0.297 -> 0.312 (profiles/r6/ab/ab_row.jsonl): not kept
    if constexpr (SEGPF) {
      if (live) rk_load_seg<MODE, BF, MNTM>(p, O0, b, y, 0, lane, L0);
    }
    {
      cpx A[FX];
#pragma unroll
      for (int k = 0; k < FX; ++k) A[k] = slot[k * 64 + lane];
      rfft72_inv(A, P);
    }
  }
  lds_barrier();   // every wave has read its row of T (and vsh is in): T becomes staging + gate weights
  if constexpr (OR || IR) {
    const uint4* ow = static_cast<const uint4*>(or_x3);
    const uint4* iw = static_cast<const uint4*>(ir_x3);
    for (int i = tid; i < GN; i += R8_NT) {
      if constexpr (OR) gsh[i] = ow[i];
      if constexpr (IR) gsh[GN + i] = iw[i];
    }
    lds_barrier();
  }
  if constexpr (MODE == ROW_FINAL) {
    if (live) {
#pragma unroll
      for (int x = 0; x < 64; ++x) stg[x * RK_SP + lane] = P[x];
#pragma unroll 1
      for (int sg = 0; sg < 2; ++sg) {
        const int xs = 32 * sg;
        if (xs >= W) continue;   // wave-uniform
        SegIn L;
        rk_load_seg<MODE, BF, MNTM>(p, O0, b, y, xs, lane, L);
        rk_segment<MODE, true, BF, MNTM>(p, stg + xs * RK_SP, b, y, xs, lane, L, gsh, or_us, gsh, ir_us, vsh);
      }
    }
    return;
  }
  if (live) {
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      const int xs = 32 * sg;
      if (xs >= W) continue;   // wave-uniform
      SegIn L;
      if (SEGPF && sg == 0) L = L0;
      else rk_load_seg<MODE, BF, MNTM>(p, O0, b, y, xs, lane, L);
      if constexpr (MODE != ROW_INIT) {
#pragma unroll
        for (int q = 0; q < 32; ++q) stg[q * RK_SP + lane] = P[xs + q];
      }
      rk_segment<MODE, true, BF, MNTM>(p, stg, b, y, xs, lane, L, gsh, or_us, gsh + GN, ir_us, vsh);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int q = 0; q < 32; ++q) P[xs + q] = stg[q * RK_SP + lane];
    }
  }
#pragma unroll
  for (int x = 0; x < 64; ++x) P[x] = (live && x < W) ? P[x] : 0.f;
  {
    cpx X[FX];
    rfft72_fwd(P, X);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_barrier();   // every wave is done with the staging and gate weights
#pragma unroll
    for (int k = 0; k < FX; ++k) slot[k * 64 + lane] = X[k];
  }
  lds_barrier();
  const int ts = opaque(tid);
#pragma unroll
  for (int it = 0; it < R8_NIT; ++it) {
    const int i = it * R8_NT + ts;
    if (i >= RK_ITEMS) break;
    const int fx = i >> 6, c = i & 63;
    cpx u[9];
#pragma unroll
    for (int r = 0; r < 8; ++r) u[r] = T[(r * FX + fx) * 64 + c];
    u[8] = cpx{0.f, 0.f};
    dft9<-1>(u);
    const size_t dst = z_off(b, n2, fx, 0) + c;
#pragma unroll
    for (int k1 = 0; k1 < 9; ++k1) z_st<BF, ZNT>(Z, dst + k1 * Z_K1, u[k1]);
  }
}

// ---------------------------------------------------------------------------------------------
// row A on channel quarters (rowq_a_kernel, fp32, small batches).  Row A's math is channel-separable
// (the 9-point sums and row transforms act per channel, the A epilogue per element: no gate), so a
// block can take (image b, row class n2, 16 channels): 128 threads, thread (row n1 = tid / 16, channel
// 16 q + tid % 16) for the transforms, T[n1][fx][16] (37.9 KB), four blocks per CU: four times the
// blocks of row8_kernel, the same LDS (and so the same waves) per CU.  It pays where row8_kernel leaves
// CUs idle: B = 1 0.941 -> 0.930 ms per forward, B = 4 0.968 -> 0.958, B = 8 0.994 -> 0.985; from B = 16
// on it is slower (1.113 vs 1.098; B = 32 1.44 vs 1.41, B = 256 8.47 vs 8.17; profiles/r5_ab/rq).  The
// same functions on the same values in the same order as row8_kernel<ROW_A>: bit-identical.
// ---------------------------------------------------------------------------------------------
constexpr int RQ_NT = 128;
constexpr int RQ_ITEMS = FX * 16;                        // (fx, channel) items of the 9-point passes
constexpr int RQ_NIT = (RQ_ITEMS + RQ_NT - 1) / RQ_NT;   // 5
__device__ __forceinline__ int rq_stg(int r, int x, int c) { return (r * 64 + x) * 16 + c + 16 * r; }
static_assert(8 * 64 * 16 + 16 * 8 <= 2 * 8 * FX * 16, "row A staging fits T");

template <bool ZNT, bool MNT>
__global__ __launch_bounds__(RQ_NT, 2) void rowq_a_kernel(void* __restrict__ Z, ConvArgs p) {
  __shared__ cpx T[8 * FX * 16];
  const int q = blockIdx.x & 3, n2 = (blockIdx.x >> 2) & 7, b = blockIdx.x >> 5;
  const int tid = threadIdx.x, r = tid >> 4, cc = tid & 15, c0 = 16 * q;
  const int H = p.H, W = p.W;
  float P[64];
  {
    cpx u[RQ_NIT][9];
#pragma unroll
    for (int it = 0; it < RQ_NIT; ++it) {
      const int i = min(it * RQ_NT + tid, RQ_ITEMS - 1);
      const size_t src = z_off(b, n2, i >> 4, 0) + c0 + (i & 15);
#pragma unroll
      for (int k1 = 0; k1 < 9; ++k1) u[it][k1] = z_ld<false, ZNT>(Z, src + k1 * Z_K1);
    }
#pragma unroll
    for (int it = 0; it < RQ_NIT; ++it) {
      const int i = it * RQ_NT + tid;
      dft9<1>(u[it]);
      if (i < RQ_ITEMS) {
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) T[(rr * FX + (i >> 4)) * 16 + (i & 15)] = u[it][rr];
      }
    }
  }
  lds_barrier();
  {
    cpx A[FX];
#pragma unroll
    for (int k = 0; k < FX; ++k) A[k] = T[(r * FX + k) * 16 + cc];
    rfft72_inv(A, P);
  }
  lds_barrier();   // T becomes the epilogue staging [n1][x][16]
  float* stg = reinterpret_cast<float*>(T);
#pragma unroll
  for (int x = 0; x < 64; ++x) stg[rq_stg(r, x, cc)] = P[x];
  lds_barrier();
  // the A epilogue (rk_segment<ROW_A>'s expression on the same 4-channel vectors): task (n1, x, 4 channels)
  const float* vec = p.vecs;
#pragma unroll 4
  for (int k = 0; k < 8 * 64 * 4 / RQ_NT; ++k) {
    const int t = k * RQ_NT + tid, g4 = t & 3, x = (t >> 2) & 63, rr = t >> 8;
    const int y = 8 * rr + n2, c = c0 + 4 * g4;
    if (y >= H || x >= W) continue;
    float* sp = stg + rq_stg(rr, x, 4 * g4);
    const f32x4 pv = *reinterpret_cast<const f32x4*>(sp);
    const f32x4 lat = *reinterpret_cast<const f32x4*>(vec + V_LAT * 64 + c);
    const f32x4 be = *reinterpret_cast<const f32x4*>(vec + V_BETA * 64 + c);
    const f32x4 nu = *reinterpret_cast<const f32x4*>(vec + V_NU * 64 + c);
    const f32x4 xv = map_ld4<false, MNT>(p.X, xx_index(b, c >> 3, y, x, c & 4, H, W));
    const f32x4 ov = p.o_nhwc ? ld4<MNT>(p.O + (((size_t)b * H + y) * W + x) * C + c)
                              : map_ld4<false, MNT>(p.O, oo_index(b, c >> 3, y, x, c & 4, H, W));
    f32x4 iv;
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const f2v xx = pr2(xv, qq), o = pr2(ov, qq);
      const f2v tt = ftanh2(-(pr2(be, qq) * o + pr2(nu, qq)) * (pr2(pv, qq) + pr2(lat, qq)) + xx);
      iv[2 * qq] = tt[0];
      iv[2 * qq + 1] = tt[1];
    }
    map_st4<false, MNT>(p.dst, ii_index(b, c >> 3, y, x, c & 4, H, W), iv);
    *reinterpret_cast<f32x4*>(sp) = iv;
  }
  lds_barrier();
  const bool live = 8 * r + n2 < H;
#pragma unroll
  for (int x = 0; x < 64; ++x) P[x] = (live && x < W) ? stg[rq_stg(r, x, cc)] : 0.f;
  {
    cpx X[FX];
    rfft72_fwd(P, X);
    lds_barrier();   // every thread has read its staged row
#pragma unroll
    for (int k = 0; k < FX; ++k) T[(r * FX + k) * 16 + cc] = X[k];
  }
  lds_barrier();
  const int ts = opaque(tid);
#pragma unroll
  for (int it = 0; it < RQ_NIT; ++it) {
    const int i = it * RQ_NT + ts;
    if (i >= RQ_ITEMS) break;
    const int fx = i >> 4, c = i & 15;
    cpx u[9];
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) u[rr] = T[(rr * FX + fx) * 16 + c];
    u[8] = cpx{0.f, 0.f};
    dft9<-1>(u);
    const size_t dst = z_off(b, n2, fx, 0) + c0 + c;
#pragma unroll
    for (int k1 = 0; k1 < 9; ++k1) z_st<false, ZNT>(Z, dst + k1 * Z_K1, u[k1]);
  }
}

// ---------------------------------------------------------------------------------------------
// column kernel (the spectral GEMM).  Block = (column class (fx, k1), 16 images), 256 threads, two
// blocks per CU (68 KB of LDS).  Thread (image, channel pair a) holds channels 2a, 2a + 1 and
// 32 + 2a, 33 + 2a of its image (each wave instruction reads / writes contiguous 256-B runs of Z) and
// turns their 8 row-class partials Z[b][fx][k1][n2][.] into the class's 8 frequencies (twiddle, 8-point
// DFT, scale + f16 split into the S tile).  Wave w then computes frequency fy = k1 + 9 k2 for k2 = w and
// w + 4:  Y[b][co] = sum_ci S[b][ci] G[ci][co]  (complex), as a real 128 x 16 x 128 product on
// v_mfma_f32_16x16x32_f16 in the f16x3 split (k = 2 ci + re|im; rows n = 64 ro + co, the re / im rows'
// A fragments derived from the compact weights by a sign flip / half swap as in k_fft.hip's
// spec_gemm_kernel).  The first frequency's Y goes into the S tile half it no longer needs while the
// second is computed.  Finally the same thread takes its channels' 8 frequencies back to row-class
// partials (8-point inverse DFT, twiddle) and writes them over its inputs.  Blocks of one class run on
// one XCD (its 256 KiB of weights fetched from HBM once).
// ---------------------------------------------------------------------------------------------
constexpr int CG_NI = 16;                            // images per block
constexpr int CG_SLD = CG_NI + 1;                    // S tile pitch (16-B units) per (cq, part, k2 % 4) row
constexpr int CG_HALF = 16 * 2 * 4 * CG_SLD;         // one frequency half of the S tile: 34,816 B
constexpr int CG_YLD = 16 * 4 * 2 + 1;               // Y tile pitch (16-B units) per image, one half
static_assert(CG_NI * CG_YLD <= CG_HALF, "a half's Y tile fits the S tile half it replaces");
constexpr int CG_NC8 = (Z_CLS + 7) / 8;              // 42 groups of 8 classes (one per XCD)

// CG_SWZ (default 1): rows of 16 units with image column bl ^ cq, so that a DFT thread group's S
// writes (eight channel groups cq of one image at a 2,176-B stride: 4-way bank conflicts on the padded
// rows) and the GEMM's fragment reads (16 images of a row, or two rows' halves) both spread over the 64
// banks; and the Y tile's frequency slot rotated by the channel group, (q + cq) & 7, so the inverse
// DFT's reads (one frequency of 16 channel groups, a 256-B stride: 8-way) do too.  Placement only: the
// values and their arithmetic are unchanged.
#ifndef CG_SWZ
#define CG_SWZ 1
#endif
__device__ __forceinline__ int cg_s(int k2, int cq, int part, int bl) {   // S tile index (16-B units)
  if constexpr (CG_SWZ) return (k2 >> 2) * CG_HALF + ((cq * 2 + part) * 4 + (k2 & 3)) * 16 + (bl ^ cq);
  return (k2 >> 2) * CG_HALF + ((cq * 2 + part) * 4 + (k2 & 3)) * CG_SLD + bl;
}
__device__ __forceinline__ int cg_yq(int q, int cq) { return CG_SWZ ? (q + cq) & 7 : q; }   // Y tile slot
__device__ __forceinline__ f32x4 mfma16x16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// The three phases of one (class, 16-image group) item, shared by col8_kernel and col8p_kernel so
// that both compute every output with the same operations in the same order (bit-identical).
// Thread roles: DFT (image bl = tid / 32, channel pair a = tid % 32: channels 2a, 2a + 1); GEMM (wave
// k2 = frequency fy = k1 + 9 k2, lane (kq, jj)).
//
// cg_forward: the thread's 8 row-class partials zin[n2] (channels 2a, 2a + 1) -> twiddle W72^{-n2 k1},
// 8-point DFT over n2, scale + f16 hi / lo split into the S tile.  The split: v_pk_mul_f32,
// v_cvt_pk_f16_f32 for hi and lo (round to nearest even, as (_Float16)), v_pk_add_f32 (re - hi is
// exact).  Columns of images past B are not zeroed: an MFMA output column depends on its own S
// column only, and theirs are never stored (col8p stores them: the same bytes as image B - 1's).
__device__ __forceinline__ void cg_forward(const f32x4 (&zin)[8], int k1, uint4* tile, int cq, int hf, int bl) {
  cpx s[2][8];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) s[e][n2] = twid<-1>(cpx{zin[n2][2 * e], zin[n2][2 * e + 1]}, n2 * k1);
    dft8_fold<-1>(s[e]);
  }
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  uint2* t2 = reinterpret_cast<uint2*>(tile);
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    uint32_t hv[2], lv[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const cpx v = s[e][k2] * SPEC_SCALE;
      const h2 hi = __builtin_convertvector(v, h2);
      const h2 lo = __builtin_convertvector(v - __builtin_convertvector(hi, cpx), h2);
      hv[e] = __builtin_bit_cast(uint32_t, hi);
      lv[e] = __builtin_bit_cast(uint32_t, lo);
    }
    t2[cg_s(k2, cq, 0, bl) * 2 + hf] = uint2{hv[0], hv[1]};
    t2[cg_s(k2, cq, 1, bl) * 2 + hf] = uint2{lv[0], lv[1]};
  }
}

// cg_kstep: k-step t of wave k2's frequency, Y[b][co] = sum_ci S[b][ci] G[ci][co] (complex) as a real
// 128 x 16 x 128 product on v_mfma_f32_16x16x32_f16 in the f16x3 split.  The compact weights A =
// (gr, gi) pairs as stored; the S fragment supplies the two forms, (sr, -si) for the real rows
// (gr sr - gi si) and (si, sr) for the imaginary rows (gr si + gi sr): a sign flip and a half swap per S
// dword (16 VALU per k-step) instead of four weight forms (64).  w[mq][0 | 1] = the hi | lo planes.
template <bool LEAN = false>
__device__ __forceinline__ void cg_kstep(const uint4* tile, int k2, int t, int kq, int jj, const uint4 (&w)[4][2],
                                         f32x4 (&acc)[8]) {
  const uint4 m = {0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u};
  const uint4 uh = tile[cg_s(k2, 4 * t + kq, 0, jj)], ul = tile[cg_s(k2, 4 * t + kq, 1, jj)];
  if constexpr (LEAN) {   // the real rows' MFMAs, then the imaginary rows' (fewer S forms live at once)
    const f16x8 sh = __builtin_bit_cast(f16x8, uh ^ m), sl = __builtin_bit_cast(f16x8, ul ^ m);
#pragma unroll
    for (int mq = 0; mq < 4; ++mq) {
      const f16x8 ah = __builtin_bit_cast(f16x8, w[mq][0]), al = __builtin_bit_cast(f16x8, w[mq][1]);
      acc[mq] = mfma16x16(al, sh, acc[mq]);
      acc[mq] = mfma16x16(ah, sl, acc[mq]);
      acc[mq] = mfma16x16(ah, sh, acc[mq]);
    }
    const f16x8 sh2 = __builtin_bit_cast(f16x8, (uh >> 16) | (uh << 16));
    const f16x8 sl2 = __builtin_bit_cast(f16x8, (ul >> 16) | (ul << 16));
#pragma unroll
    for (int mq = 0; mq < 4; ++mq) {
      const f16x8 ah = __builtin_bit_cast(f16x8, w[mq][0]), al = __builtin_bit_cast(f16x8, w[mq][1]);
      acc[4 + mq] = mfma16x16(al, sh2, acc[4 + mq]);
      acc[4 + mq] = mfma16x16(ah, sl2, acc[4 + mq]);
      acc[4 + mq] = mfma16x16(ah, sh2, acc[4 + mq]);
    }
    return;
  }
  const f16x8 sh = __builtin_bit_cast(f16x8, uh ^ m), sl = __builtin_bit_cast(f16x8, ul ^ m);
  const f16x8 sh2 = __builtin_bit_cast(f16x8, (uh >> 16) | (uh << 16));
  const f16x8 sl2 = __builtin_bit_cast(f16x8, (ul >> 16) | (ul << 16));
#pragma unroll
  for (int mq = 0; mq < 4; ++mq) {
    const f16x8 ah = __builtin_bit_cast(f16x8, w[mq][0]), al = __builtin_bit_cast(f16x8, w[mq][1]);
    acc[mq] = mfma16x16(al, sh, acc[mq]);
    acc[mq] = mfma16x16(ah, sl, acc[mq]);
    acc[mq] = mfma16x16(ah, sh, acc[mq]);
    acc[4 + mq] = mfma16x16(al, sh2, acc[4 + mq]);
    acc[4 + mq] = mfma16x16(ah, sl2, acc[4 + mq]);
    acc[4 + mq] = mfma16x16(ah, sh2, acc[4 + mq]);
  }
}

// cg_kstep on S fragments already read (uh / ul: the hi / lo fragment of k-step t): the same MFMAs in
// the same order as cg_kstep
__device__ __forceinline__ void cg_kstep_frag(uint4 uh, uint4 ul, const uint4 (&w)[4][2], f32x4 (&acc)[8]) {
  const uint4 m = {0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u};
  const f16x8 sh = __builtin_bit_cast(f16x8, uh ^ m), sl = __builtin_bit_cast(f16x8, ul ^ m);
  const f16x8 sh2 = __builtin_bit_cast(f16x8, (uh >> 16) | (uh << 16));
  const f16x8 sl2 = __builtin_bit_cast(f16x8, (ul >> 16) | (ul << 16));
#pragma unroll
  for (int mq = 0; mq < 4; ++mq) {
    const f16x8 ah = __builtin_bit_cast(f16x8, w[mq][0]), al = __builtin_bit_cast(f16x8, w[mq][1]);
    acc[mq] = mfma16x16(al, sh, acc[mq]);
    acc[mq] = mfma16x16(ah, sl, acc[mq]);
    acc[mq] = mfma16x16(ah, sh, acc[mq]);
    acc[4 + mq] = mfma16x16(al, sh2, acc[4 + mq]);
    acc[4 + mq] = mfma16x16(ah, sl2, acc[4 + mq]);
    acc[4 + mq] = mfma16x16(ah, sh2, acc[4 + mq]);
  }
}

// weights of k-step t for wave k2 of class cls (both planes, the wave's four row blocks)
// CG_WNT (A/B, default 0): the weight loads non-temporal
#ifndef CG_WNT
#define CG_WNT 0
#endif
__device__ __forceinline__ void cg_wload(const uint4* __restrict__ Gc, int cls, int k2, int t, int kq, int jj,
                                         uint4 (&w)[4][2]) {
  const uint4* gw = Gc + (size_t)(cls * 8 + k2) * 2 * 16 * 64;
#pragma unroll
  for (int mq = 0; mq < 4; ++mq) {
#if CG_WNT
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    const u4v* gv = reinterpret_cast<const u4v*>(gw);
    w[mq][0] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(gv + (0 * 16 + 4 * t + kq) * 64 + 16 * mq + jj));
    w[mq][1] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(gv + (1 * 16 + 4 * t + kq) * 64 + 16 * mq + jj));
#else
    w[mq][0] = gw[(0 * 16 + 4 * t + kq) * 64 + 16 * mq + jj];
    w[mq][1] = gw[(1 * 16 + 4 * t + kq) * 64 + 16 * mq + jj];
#endif
  }
}

// the Y tile over the S tile's space: [image][cq][k2] (16-B units, pitch 16 * 8 * 2 + 1 per image)
constexpr int CG_YP = 16 * 8 * 2 + 1;
static_assert(CG_NI * CG_YP <= 2 * CG_HALF, "the Y tile fits the S tile's space");
__device__ __forceinline__ void cg_ystore(uint4* tile, int k2, int kq, int jj, const f32x4 (&acc)[8], float unscale) {
  f32x4* ytile = reinterpret_cast<f32x4*>(tile);
#pragma unroll
  for (int mq = 0; mq < 4; ++mq) {
    const int cqo = 4 * mq + kq;
    const f32x4 re = acc[mq], im = acc[4 + mq];
    ytile[jj * CG_YP + (cqo * 8 + cg_yq(k2, cqo)) * 2] = f32x4{re[0], im[0], re[1], im[1]} * unscale;
    ytile[jj * CG_YP + (cqo * 8 + cg_yq(k2, cqo)) * 2 + 1] = f32x4{re[2], im[2], re[3], im[3]} * unscale;
  }
}

// cg_inverse: the thread's channels' 8 frequencies from the Y tile -> 8-point inverse DFT, twiddle
// W72^{n2 k1} -> the row-class partials out[n2] (channels 2a, 2a + 1)
__device__ __forceinline__ void cg_yread(const uint4* tile, int cq, int hf, int bl, f32x4 (&y)[8]) {
  const f32x4* ytile = reinterpret_cast<const f32x4*>(tile);
#pragma unroll
  for (int q = 0; q < 8; ++q) y[q] = ytile[bl * CG_YP + (cq * 8 + cg_yq(q, cq)) * 2 + hf];
}
__device__ __forceinline__ void cg_inverse_regs(const f32x4 (&y)[8], int k1, f32x4 (&out)[8]) {
  cpx yv[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    yv[0][q] = cpx{y[q][0], y[q][1]};
    yv[1][q] = cpx{y[q][2], y[q][3]};
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    dft8_fold<1>(yv[e]);
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) yv[e][n2] = twid<1>(yv[e][n2], n2 * k1);
  }
#pragma unroll
  for (int n2 = 0; n2 < 8; ++n2) out[n2] = f32x4{yv[0][n2].x, yv[0][n2].y, yv[1][n2].x, yv[1][n2].y};
}
__device__ __forceinline__ void cg_inverse(const uint4* tile, int k1, int cq, int hf, int bl, f32x4 (&out)[8]) {
  f32x4 y[8];
  cg_yread(tile, cq, hf, bl, y);
  cg_inverse_regs(y, k1, out);
}

// col8_kernel: 512 threads, thread = image x channel pair (one contiguous 512-B run of Z per image
// and n2 per wave instruction pair) for the DFTs and the split; each wave computes ONE frequency
// (k2 = wave).  Two blocks per CU (16 waves) leave 128 VGPRs per wave.  Round 5 also measured a
// four-wave form (two frequencies per wave behind a weight reload: 0.212 vs 0.192 ms at B = 256) and
// a persistent form holding each wave's weights in registers over several image groups, one block
// per CU (0.207 ms; batch-1 forward 1.06 vs 0.98 ms): both removed.  Large batches run col8p_kernel
// (below), the same arithmetic with the next item's partials in flight during this one's GEMM.
// ZNT: the partials Z read and written non-temporal (the weights, re-read by the other batch slice's
// launch of the same convolution, keep the cache)
template <bool ZNT>
__global__ __launch_bounds__(512, 2) void col8_kernel(cpx* __restrict__ Z, const uint4* __restrict__ Gc, int B,
                                                      int ngrp, float unscale) {
  __shared__ uint4 tile[2 * CG_HALF];   // 69,632 B
  const int c8 = blockIdx.x / (8 * ngrp), rem = blockIdx.x - c8 * 8 * ngrp;
  const int grp = rem >> 3, cls = c8 * 8 + (rem & 7);
  if (cls >= Z_CLS) return;
  const int fx = cls / 9, k1 = cls - fx * 9;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int img0 = grp * CG_NI;
  const int bl = tid >> 5, a = tid & 31;   // DFT role: image bl, channels 2a, 2a + 1 (group a >> 1, half a & 1)
  const bool live = img0 + bl < B;
  const int b = min(img0 + bl, B - 1);
  const int cq = a >> 1, hf = a & 1;
  const int kq = lane >> 4, jj = lane & 15, k2 = wv;
  // weights of two k-steps in registers (64 VGPRs), a two-slot ring: k-step t + 2's loads go into step
  // t's slot right after step t's MFMAs, so step t + 1's MFMAs cover part of their latency (col8 0.196 ->
  // 0.185 ms against loading steps 2 and 3 together after step 1; profiles/r5l).  Requesting step 0's
  // weights before the partials measured slower (8.27 -> 8.33 ms per forward; profiles/r5o)
  uint4 wr[2][4][2];
  {
    f32x4 zin[8];
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) {
      const f32x4* zp = reinterpret_cast<const f32x4*>(Z + z_off(b, n2, fx, k1)) + a;
      zin[n2] = ZNT ? __builtin_nontemporal_load(zp) : *zp;
    }
    cg_forward(zin, k1, tile, cq, hf, bl);
  }
  cg_wload(Gc, cls, k2, 0, kq, jj, wr[0]);
  cg_wload(Gc, cls, k2, 1, kq, jj, wr[1]);
  lds_barrier();
  f32x4 acc[8] = {};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    cg_kstep(tile, k2, t, kq, jj, wr[t % 2], acc);
    if (t + 2 < 4) cg_wload(Gc, cls, k2, t + 2, kq, jj, wr[t % 2]);
  }
  lds_barrier();   // every wave has read the S tile
  cg_ystore(tile, k2, kq, jj, acc, unscale);
  lds_barrier();
  f32x4 out[8];
  cg_inverse(tile, k1, cq, hf, bl, out);
  if (live) {
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) {
      f32x4* zp = reinterpret_cast<f32x4*>(Z + z_off(b, n2, fx, k1)) + a;
      if constexpr (ZNT) __builtin_nontemporal_store(out[n2], zp);
      else *zp = out[n2];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// col8p_kernel: col8_kernel's items (class, 16-image group) with the HBM stream kept busy.  col8_kernel
// runs each block's phases in series -- load the partials, DFT, GEMM, inverse DFT, store -- so with two
// blocks per CU the partials stream idles while both are past their loads (waves parked 46 % of their
// cycles, 0.53 of 8 TB/s).  Here a block (one per CU, 512 threads) walks a contiguous range of items and
// keeps the NEXT item's 64 KiB of partials in flight during the current one's work: they go straight
// into the second of two LDS slots by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, no
// registers), and each slot serves an item as raw partials -> S tile -> Y tile in turn.  A wave's
// weights (its frequency's 4 k-steps, 128 VGPRs) stay in registers while the range stays in one class
// (an item range spans at most two or three classes), so no vector-memory load is waited for between
// the DMA's issue and its use: vmcnt counts loads, stores and LDS-DMA together in issue order, and a
// wait for a younger load would drain the prefetch.  The item math is cg_forward / cg_kstep /
// cg_ystore / cg_inverse, as in col8_kernel: bit-identical outputs.
// ---------------------------------------------------------------------------------------------
constexpr int CP_SLOT = 2 * CG_HALF;                 // uint4 per LDS slot (69,632 B)
static_assert(CG_NI * 8 * 64 * 8 <= CP_SLOT * 16, "an item's raw partials fit a slot");
static_assert(ZLAYOUT == 1, "col8p DMA: an image's 8 row classes are one contiguous 4-KiB run of Z");

// one LDS-DMA wave instruction: 64 lanes x 16 B from each lane's gsrc to LDS bytes [lds, lds + 1024)
// (M0 = the wave-uniform LDS base, written and restored in the same statement)
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

// Measured and removed (same box, B = 256; profiles/r6/ab/ab_col8.jsonl): item it + 2's DMA issued
// before item it's stores (0.186 vs 0.170 ms); an item's stores held in registers and issued before
// the next item's GEMM (0.178 vs 0.169) or two after each of its k-steps (0.212); every k-step's S
// fragments read before the first MFMA (0.1742 vs 0.1744).  Timing-only builds (tools/exp_lib.sh
// -DCOL8P_NO...): no DMA wait 0.166 vs 0.171, no stores 0.147, no GEMM 0.129, no DMA and no stores
// (the item arithmetic alone) 0.103 of which the GEMM phase is 0.053, every item on the first class's
// weights 0.152 (the 85 MB of weights not read).  A class change's weights requested right after the
// previous item's GEMM instead of behind a vmcnt(0) at the class's first item: 0.1687 vs 0.1676, not
// kept (profiles/r6/ab/ab_col8_phases.jsonl).
template <bool ZNT>
__global__ __launch_bounds__(512, 1) void col8p_kernel(cpx* __restrict__ Z, const uint4* __restrict__ Gc, int B,
                                                       int ngrp, int nitems, float unscale) {
  __shared__ uint4 slots[2 * CP_SLOT];   // 139,264 B
  // consecutive item ranges on one XCD (blockIdx % 8 under round-robin dispatch; a speed choice only):
  // a class's weights are then read by one L2
  const int nblk = gridDim.x, per = nblk / 8, r8 = nblk % 8, xg = blockIdx.x % 8, q = blockIdx.x / 8;
  const int v = (xg < r8 ? xg * (per + 1) : r8 * (per + 1) + (xg - r8) * per) + q;
  const int it0 = (int)((int64_t)v * nitems / nblk), it1 = (int)((int64_t)(v + 1) * nitems / nblk);
  if (it0 >= it1) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int bl = tid >> 5, a = tid & 31, cq = a >> 1, hf = a & 1;
  const int kq = lane >> 4, jj = lane & 15, k2 = wv;
  const uint32_t lds0 = (uint32_t)(uintptr_t)slots;
  // item it -> slot s: wave wv moves images 2 wv, 2 wv + 1 of the group (four 1-KiB quarters each)
  auto dma = [&](int it, int s) {
#ifdef COL8P_NODMA   // timing only (with COL8P_NOWAIT): no partials loaded
    if (it >= 0) return;
#endif
    const int cls = it / ngrp, grp = it - cls * ngrp;
    const int fx = cls / 9, k1 = cls - fx * 9;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int il = 2 * wv + (i >> 2);
      const int b = min(grp * CG_NI + il, B - 1);
      const char* src = reinterpret_cast<const char*>(Z + z_off(b, 0, fx, k1)) + (i & 3) * 1024 + lane * 16;
      const uint32_t dst = lds0 + (uint32_t)(s * CP_SLOT * 16 + il * 4096 + (i & 3) * 1024);
      glds16(src, __builtin_amdgcn_readfirstlane(dst));
    }
  };
  // the weight loads are waited for where they are issued (s_waitcnt vmcnt(0) through the builtin, so
  // hipcc's wait bookkeeping sees them complete): otherwise every item's GEMM would carry hipcc's waits
  // for them, which in issue order also wait for the next item's DMA
  constexpr unsigned VMCNT0 = 0x0F70;   // vmcnt(0) expcnt(7) lgkmcnt(15)
  uint4 w[4][4][2];
  int wcls = it0 / ngrp;
#pragma unroll
  for (int t = 0; t < 4; ++t) cg_wload(Gc, wcls, k2, t, kq, jj, w[t]);
  __builtin_amdgcn_s_waitcnt(VMCNT0);
  dma(it0, 0);
  if (it0 + 1 < it1) dma(it0 + 1, 1);
  for (int it = it0; it < it1; ++it) {
    const int s = (it - it0) & 1;
    uint4* tile = slots + s * CP_SLOT;
    const int cls = it / ngrp, grp = it - cls * ngrp;
    const int fx = cls / 9, k1 = cls - fx * 9;
    // this item's DMA is older than: the previous item's 8 stores and the next item's 8 DMA pieces (a
    // class change's weight loads only make the wait longer)
    const bool nx = it + 1 < it1;
#ifndef COL8P_NOWAIT   // (timing only when defined: no wait for the DMA, reads whatever has landed)
    if (it == it0) {
      if (nx) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (nx) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
#endif
    lds_barrier();   // every wave's pieces have landed
    {
      f32x4 zin[8];
      const f32x4* raw = reinterpret_cast<const f32x4*>(tile) + bl * 256 + a;   // [image][n2][64 complex]
#pragma unroll
      for (int n2 = 0; n2 < 8; ++n2) zin[n2] = raw[n2 * 32];
      lds_barrier();   // the raw partials are read: the slot becomes the S tile
#ifndef COL8P_NODFT   // (timing-only A/B builds: tools/exp_lib.sh ... -DCOL8P_NODFT etc.)
      cg_forward(zin, k1, tile, cq, hf, bl);
#else
      if (zin[0][0] == 12345.f) tile[tid] = uint4{};
#endif
    }
    if (cls != wcls) {   // block-uniform
      wcls = cls;
#pragma unroll
      for (int t = 0; t < 4; ++t) cg_wload(Gc, wcls, k2, t, kq, jj, w[t]);
      __builtin_amdgcn_s_waitcnt(VMCNT0);
    }
    lds_barrier();
    f32x4 acc[8] = {};
#ifndef COL8P_NOGEMM
#pragma unroll
    for (int t = 0; t < 4; ++t) cg_kstep(tile, k2, t, kq, jj, w[t], acc);
#endif
    lds_barrier();   // every wave has read the S tile
    cg_ystore(tile, k2, kq, jj, acc, unscale);
    lds_barrier();
    f32x4 out[8];
    cg_yread(tile, cq, hf, bl, out);
#ifndef COL8P_NOINV
    cg_inverse_regs(out, k1, out);
#endif
    // images past B (a partial last group) store image B - 1's values over it: the same bytes, since
    // their DMA read image B - 1 too -- every item issues exactly 8 stores, as the counted waits assume
    const int b = min(grp * CG_NI + bl, B - 1);
    f32x4* zb = reinterpret_cast<f32x4*>(Z + z_off(b, 0, fx, k1)) + a;
#ifndef COL8P_NOSTORE   // timing only: no stores
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) {
      f32x4* zp = zb + n2 * 32;   // z_off(b, n2, fx, k1) - z_off(b, 0, fx, k1) = 64 n2 complex = 32 n2 f32x4
      if constexpr (ZNT) __builtin_nontemporal_store(out[n2], zp);
      else *zp = out[n2];
    }
#else
    if (out[0][0] == 12345.f) zb[0] = out[0];
#endif
    if (it + 2 < it1) {
      lds_barrier();   // every thread has read its Y values: the slot takes item it + 2
      dma(it + 2, s);
    }
  }
}

// col8q_kernel: col8p_kernel's blocks and LDS-DMA prefetch, software-pipelined so that the matrix
// cores and the vector ALUs work at the same time: item k's GEMM (MFMA, weights in registers, S from
// the working slot) runs beside item k - 1's inverse DFT and stores (VALU on the thread's 8 Y values,
// read from the Y tile into registers at the end of item k - 1).  Per item:
//   GEMM(k) || inverse(k - 1) + stores(k - 1);  Y(k) -> W;  yv <- W;
//   wait DMA(k + 1) in P;  raw(k + 1) -> DFT -> S(k + 1) over it in P;  DMA(k + 2) -> W;  swap W, P.
// Item k + 2's DMA is issued one item ahead of its use.  The same item arithmetic (cg_*): bit-identical.
template <bool ZNT>
__global__ __launch_bounds__(512, 1) void col8q_kernel(cpx* __restrict__ Z, const uint4* __restrict__ Gc, int B,
                                                       int ngrp, int nitems, float unscale) {
  __shared__ uint4 slots[2 * CP_SLOT];   // 139,264 B
  const int nblk = gridDim.x, per = nblk / 8, r8 = nblk % 8, xg = blockIdx.x % 8, q = blockIdx.x / 8;
  const int v = (xg < r8 ? xg * (per + 1) : r8 * (per + 1) + (xg - r8) * per) + q;
  const int it0 = (int)((int64_t)v * nitems / nblk), it1 = (int)((int64_t)(v + 1) * nitems / nblk);
  if (it0 >= it1) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int kq = lane >> 4, jj = lane & 15, k2 = wv;
  const uint32_t lds0 = (uint32_t)(uintptr_t)slots;
  auto dma = [&](int it, int s) {
    const int cls = it / ngrp, grp = it - cls * ngrp;
    const int fx = cls / 9, k1 = cls - fx * 9;
    const int lq = opaque(lane);   // (not hoisted out of the item loop)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int il = 2 * wv + (i >> 2);
      const int b = min(grp * CG_NI + il, B - 1);
      const char* src = reinterpret_cast<const char*>(Z + z_off(b, 0, fx, k1)) + (i & 3) * 1024 + lq * 16;
      const uint32_t dst = lds0 + (uint32_t)(s * CP_SLOT * 16 + il * 4096 + (i & 3) * 1024);
      glds16(src, __builtin_amdgcn_readfirstlane(dst));
    }
  };
  // raw partials of the item in slot s -> S tile over them (two barriers)
  auto forward = [&](int it, int s) {
    // thread indices re-derived from an opaque tid: their address math is not hoisted out of the loop
    // (held live, or spilled, across the GEMM)
    const int tq = opaque(tid), bl = tq >> 5, a = tq & 31, cq = a >> 1, hf = a & 1;
    uint4* tile = slots + s * CP_SLOT;
    const int cls = it / ngrp, k1 = cls % 9;
    f32x4 zin[8];
    const f32x4* raw = reinterpret_cast<const f32x4*>(tile) + bl * 256 + a;
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) zin[n2] = raw[n2 * 32];
    lds_barrier();   // the raw partials are read: the slot becomes the S tile
    cg_forward(zin, k1, tile, cq, hf, bl);
  };
  constexpr unsigned VMCNT0 = 0x0F70;   // vmcnt(0) expcnt(7) lgkmcnt(15), seen by hipcc's bookkeeping
  uint4 w[4][4][2];
  int wcls = it0 / ngrp;
#pragma unroll
  for (int t = 0; t < 4; ++t) cg_wload(Gc, wcls, k2, t, kq, jj, w[t]);
  __builtin_amdgcn_s_waitcnt(VMCNT0);
  dma(it0, 0);
  if (it0 + 1 < it1) {
    dma(it0 + 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  lds_barrier();
  forward(it0, 0);
  lds_barrier();
  f32x4 yv[8];   // the previous item's Y values of this thread's channels
  // one item; WI: with the previous item's inverse DFT and stores beside the GEMM (every item but the
  // first: a branch there would put them in a block of their own, after the MFMAs)
  auto item = [&](int it, auto WI) {
    const int s = (it - it0) & 1;
    uint4* tile = slots + s * CP_SLOT;
    const int cls = it / ngrp;
    if (cls != wcls) {   // block-uniform: before this item's GEMM
      wcls = cls;
#pragma unroll
      for (int t = 0; t < 4; ++t) cg_wload(Gc, wcls, k2, t, kq, jj, w[t]);
      __builtin_amdgcn_s_waitcnt(VMCNT0);
    }
    f32x4 acc[8] = {};
#pragma unroll
    for (int t = 0; t < 4; ++t) cg_kstep<true>(tile, k2, t, kq, jj, w[t], acc);
    if constexpr (decltype(WI)::value) {
      const int pit = it - 1, pcls = pit / ngrp, pgrp = pit - pcls * ngrp;
      const int pfx = pcls / 9, pk1 = pcls - pfx * 9;
      f32x4 out[8];
      cg_inverse_regs(yv, pk1, out);
      const int tq = opaque(tid);
      const int b = min(pgrp * CG_NI + (tq >> 5), B - 1);   // (images past B: image B - 1's bytes again)
#pragma unroll
      for (int n2 = 0; n2 < 8; ++n2) {
        f32x4* zp = reinterpret_cast<f32x4*>(Z + z_off(b, n2, pfx, pk1)) + (tq & 31);
        if constexpr (ZNT) __builtin_nontemporal_store(out[n2], zp);
        else *zp = out[n2];
      }
    }
    lds_barrier();   // every wave has read the S tile
    {
      const int lq = opaque(lane);
      cg_ystore(tile, k2, lq >> 4, lq & 15, acc, unscale);
    }
    if (it + 1 < it1) {
      // item it + 1's DMA (issued one item ago) is older than this item's 8 stores only
      if constexpr (decltype(WI)::value) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();   // every wave's pieces have landed; the Y tile is complete
      forward(it + 1, s ^ 1);
      {
        const int tq = opaque(tid);   // after the forward DFT: fewer registers live beside it
        cg_yread(tile, (tq & 31) >> 1, tq & 1, tq >> 5, yv);
      }
      lds_barrier();   // the S tile of item it + 1 is complete; every thread has read its Y values
      if (it + 2 < it1) dma(it + 2, s);
    } else {
      lds_barrier();
      const int tq = opaque(tid);
      cg_yread(tile, (tq & 31) >> 1, tq & 1, tq >> 5, yv);
    }
  };
  item(it0, std::false_type{});
  for (int it = it0 + 1; it < it1; ++it) item(it, std::true_type{});
  {   // the last item's inverse DFT and stores
    const int pit = it1 - 1, pcls = pit / ngrp, pgrp = pit - pcls * ngrp;
    const int pfx = pcls / 9, pk1 = pcls - pfx * 9;
    f32x4 out[8];
    cg_inverse_regs(yv, pk1, out);
    const int b = min(pgrp * CG_NI + (tid >> 5), B - 1);
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) {
      f32x4* zp = reinterpret_cast<f32x4*>(Z + z_off(b, n2, pfx, pk1)) + (tid & 31);
      if constexpr (ZNT) __builtin_nontemporal_store(out[n2], zp);
      else *zp = out[n2];
    }
  }
}

// column kernel, bf16 (MP_DTYPE_BF16): col8_kernel's blocking with bf16 Z partials (8-B reads of a
// thread's two channels), a bf16 S tile (one (re, im) pair per channel, no lo plane: 34 KB), one
// v_mfma_f32_16x16x32_bf16 product per (k-step, row block, re|im) against the class-major bf16
// weights Gb[f][cq][co] (16 KiB per frequency), fp32 accumulation, DFTs and twiddles in fp32.
constexpr int CB_HALF = 16 * 4 * CG_SLD;             // one frequency half of the bf16 S tile (16-B units)
// (CG_SWZ: rows of 16 units, image column img ^ c, as cg_s)
__device__ __forceinline__ int cb_s(int k2, int c, int img) {
  if constexpr (CG_SWZ) return (k2 >> 2) * CB_HALF + (c * 4 + (k2 & 3)) * 16 + (img ^ c);
  return (k2 >> 2) * CB_HALF + (c * 4 + (k2 & 3)) * CG_SLD + img;
}
// the bf16 item phases, shared by col8_bf_kernel and col8p_bf_kernel (bit-identical): the thread's 8
// bf16 row-class partials (channels 2a, 2a + 1) -> twiddle, 8-point DFT -> bf16 S tile
__device__ __forceinline__ void cb_forward(const uint2 (&zin)[8], int k1, uint4* tile, int cq, int hf, int bl) {
  cpx s[2][8];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) s[e][n2] = twid<-1>(unpack_bf2(e ? zin[n2].y : zin[n2].x), n2 * k1);
    dft8_fold<-1>(s[e]);
  }
  uint2* t2 = reinterpret_cast<uint2*>(tile);
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2)   // (columns past B unmasked, as in col8_kernel)
    t2[cb_s(k2, cq, bl) * 2 + hf] = uint2{pack_bf2(s[0][k2].x, s[0][k2].y), pack_bf2(s[1][k2].x, s[1][k2].y)};
}
// one k-step: S-side forms as in cg_kstep, one bf16 product per (row block, re | im)
__device__ __forceinline__ void cb_kstep(const uint4* tile, int k2, int t, int kq, int jj, const uint4 (&w)[4],
                                         f32x4 (&acc)[8]) {
  const uint4 m = {0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u};
  const uint4 us = tile[cb_s(k2, 4 * t + kq, jj)];
  const bf16x8 sre = __builtin_bit_cast(bf16x8, us ^ m), sim = __builtin_bit_cast(bf16x8, (us >> 16) | (us << 16));
#pragma unroll
  for (int mq = 0; mq < 4; ++mq) {
    const bf16x8 g = __builtin_bit_cast(bf16x8, w[mq]);
    acc[mq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(g, sre, acc[mq], 0, 0, 0);
    acc[4 + mq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(g, sim, acc[4 + mq], 0, 0, 0);
  }
}
__device__ __forceinline__ void cb_wload(const uint4* __restrict__ Gb, int cls, int k2, int t, int kq, int jj,
                                         uint4 (&w)[4]) {
  const uint4* gw = Gb + (size_t)(cls * 8 + k2) * 16 * 64;
#pragma unroll
  for (int mq = 0; mq < 4; ++mq) w[mq] = gw[(4 * t + kq) * 64 + 16 * mq + jj];
}
typedef uint32_t u2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u2v_t cb_pack(f32x4 v) { return u2v_t{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])}; }

template <bool ZNT>
__global__ __launch_bounds__(512, 2) void col8_bf_kernel(void* __restrict__ Zv, const uint4* __restrict__ Gb, int B,
                                                         int ngrp) {
  __shared__ uint4 tile[2 * CG_HALF];   // the Y tile (fp32) needs the fp32 kernel's space
  const int c8 = blockIdx.x / (8 * ngrp), rem = blockIdx.x - c8 * 8 * ngrp;
  const int grp = rem >> 3, cls = c8 * 8 + (rem & 7);
  if (cls >= Z_CLS) return;
  const int fx = cls / 9, k1 = cls - fx * 9;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int img0 = grp * CG_NI;
  const int bl = tid >> 5, a = tid & 31;
  const bool live = img0 + bl < B;
  const int b = min(img0 + bl, B - 1);
  const int cq = a >> 1, hf = a & 1;
  uint32_t* Z = static_cast<uint32_t*>(Zv);
  {
    uint2 zin[8];
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) {
      const u2v_t* zp = reinterpret_cast<const u2v_t*>(Z + z_off(b, n2, fx, k1)) + a;
      const u2v_t v = ZNT ? __builtin_nontemporal_load(zp) : *zp;
      zin[n2] = uint2{v.x, v.y};
    }
    cb_forward(zin, k1, tile, cq, hf, bl);
  }
  const int kq = lane >> 4, jj = lane & 15, k2 = wv;
  uint4 wr[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) cb_wload(Gb, cls, k2, t, kq, jj, wr[t]);
  lds_barrier();
  f32x4 acc[8] = {};
#pragma unroll
  for (int t = 0; t < 4; ++t) cb_kstep(tile, k2, t, kq, jj, wr[t], acc);
  lds_barrier();
  cg_ystore(tile, k2, kq, jj, acc, 1.0f);   // (x 1.0f: exact)
  lds_barrier();
  f32x4 yo[8];
  cg_inverse(tile, k1, cq, hf, bl, yo);
  if (live) {
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) {
      u2v_t* zp = reinterpret_cast<u2v_t*>(Z + z_off(b, n2, fx, k1)) + a;
      if constexpr (ZNT) __builtin_nontemporal_store(cb_pack(yo[n2]), zp);
      else *zp = cb_pack(yo[n2]);
    }
  }
}

// col8p_bf_kernel: col8p_kernel's persistent LDS-DMA form for the bf16 path (32 KiB of bf16 partials per
// item, 4 DMA pieces per wave; the weights of a wave's frequency, 64 VGPRs, resident), the item math
// of col8_bf_kernel (cb_* / cg_ystore / cg_inverse): bit-identical to it
template <bool ZNT>
__global__ __launch_bounds__(512, 1) void col8p_bf_kernel(void* __restrict__ Zv, const uint4* __restrict__ Gb, int B,
                                                          int ngrp, int nitems) {
  __shared__ uint4 slots[2 * CP_SLOT];
  const int nblk = gridDim.x, per = nblk / 8, r8 = nblk % 8, xg = blockIdx.x % 8, q = blockIdx.x / 8;
  const int v = (xg < r8 ? xg * (per + 1) : r8 * (per + 1) + (xg - r8) * per) + q;
  const int it0 = (int)((int64_t)v * nitems / nblk), it1 = (int)((int64_t)(v + 1) * nitems / nblk);
  if (it0 >= it1) return;
  uint32_t* Z = static_cast<uint32_t*>(Zv);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int bl = tid >> 5, a = tid & 31, cq = a >> 1, hf = a & 1;
  const int kq = lane >> 4, jj = lane & 15, k2 = wv;
  const uint32_t lds0 = (uint32_t)(uintptr_t)slots;
  // item it -> slot s: wave wv moves images 2 wv, 2 wv + 1 (2 KiB each, two 1-KiB pieces)
  auto dma = [&](int it, int s) {
    const int cls = it / ngrp, grp = it - cls * ngrp;
    const int fx = cls / 9, k1 = cls - fx * 9;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int il = 2 * wv + (i >> 1);
      const int b = min(grp * CG_NI + il, B - 1);
      const char* src = reinterpret_cast<const char*>(Z + z_off(b, 0, fx, k1)) + (i & 1) * 1024 + lane * 16;
      const uint32_t dst = lds0 + (uint32_t)(s * CP_SLOT * 16 + il * 2048 + (i & 1) * 1024);
      glds16(src, __builtin_amdgcn_readfirstlane(dst));
    }
  };
  constexpr unsigned VMCNT0 = 0x0F70;   // vmcnt(0) expcnt(7) lgkmcnt(15), seen by hipcc's bookkeeping
  uint4 w[4][4];
  int wcls = it0 / ngrp;
#pragma unroll
  for (int t = 0; t < 4; ++t) cb_wload(Gb, wcls, k2, t, kq, jj, w[t]);
  __builtin_amdgcn_s_waitcnt(VMCNT0);
  dma(it0, 0);
  if (it0 + 1 < it1) dma(it0 + 1, 1);
  for (int it = it0; it < it1; ++it) {
    const int s = (it - it0) & 1;
    uint4* tile = slots + s * CP_SLOT;
    const int cls = it / ngrp, grp = it - cls * ngrp;
    const int fx = cls / 9, k1 = cls - fx * 9;
    // this item's DMA is older than the previous item's 8 stores and the next item's 4 DMA pieces
    const bool nx = it + 1 < it1;
    if (it == it0) {
      if (nx) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (nx) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
    lds_barrier();   // every wave's pieces have landed
    {
      uint2 zin[8];
      const uint2* raw = reinterpret_cast<const uint2*>(tile) + bl * 256 + a;   // [image][n2][64 bf16 pairs]
#pragma unroll
      for (int n2 = 0; n2 < 8; ++n2) zin[n2] = raw[n2 * 32];
      lds_barrier();   // the raw partials are read: the slot becomes the S tile
      cb_forward(zin, k1, tile, cq, hf, bl);
    }
    if (cls != wcls) {   // block-uniform
      wcls = cls;
#pragma unroll
      for (int t = 0; t < 4; ++t) cb_wload(Gb, wcls, k2, t, kq, jj, w[t]);
      __builtin_amdgcn_s_waitcnt(VMCNT0);
    }
    lds_barrier();
    f32x4 acc[8] = {};
#pragma unroll
    for (int t = 0; t < 4; ++t) cb_kstep(tile, k2, t, kq, jj, w[t], acc);
    lds_barrier();   // every wave has read the S tile
    cg_ystore(tile, k2, kq, jj, acc, 1.0f);
    lds_barrier();
    f32x4 yo[8];
    cg_inverse(tile, k1, cq, hf, bl, yo);
    // images past B: image B - 1's bytes again; exactly 8 stores per item, as the counted waits assume
    const int b = min(grp * CG_NI + bl, B - 1);
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) {
      u2v_t* zp = reinterpret_cast<u2v_t*>(Z + z_off(b, n2, fx, k1)) + a;
      if constexpr (ZNT) __builtin_nontemporal_store(cb_pack(yo[n2]), zp);
      else *zp = cb_pack(yo[n2]);
    }
    if (it + 2 < it1) {
      lds_barrier();   // every thread has read its Y values: the slot takes item it + 2
      dma(it + 2, s);
    }
  }
}

// ------------------------------------------------------------------------------------ launchers
bool fft4_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("MP_FFT4");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// MP_MAP_NT: row8_kernel / rowq_a_kernel's map loads and stores (X, O, I; fp32 or bf16) non-temporal (1)
// or default policy (0).  Default: on for forwards of >= 128 images, whose maps are far larger than the
// 256 MB Infinity Cache: they then stop evicting the two convolutions' spectral weights (fp32 2 x 87 MB,
// bf16 2 x 44 MB, read by every column launch) from it; row(INIT) keeps the default policy
// (R8_INIT_MNT).  Same box, bit-identical (profiles/r6/ab/ab_map_nt.jsonl): fp32 B = 256 7.92 -> 7.70 ms
// per forward (col8p 0.166 -> 0.151, row A 0.273 -> 0.266, row B 0.307 -> 0.304), B = 128 4.10 -> 4.05;
// bf16 B = 256 4.98 -> 4.72, B = 128 2.555 -> 2.518.  Not below 128: fp32 B = 64 (slices of 32) 2.364 ->
// 2.398, B = 32 1.40 -> 1.43; bf16 B = 64 1.495 -> 1.505
#ifndef MAP_NT_MINB
#define MAP_NT_MINB 128
#endif
#ifndef MAP_NT_MINB_BF
#define MAP_NT_MINB_BF 128
#endif
static bool map_nt(bool bf, int ntot) {
  static const int v = [] {
    const char* e = std::getenv("MP_MAP_NT");
    return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
  }();
  return v < 0 ? ntot >= (bf ? MAP_NT_MINB_BF : MAP_NT_MINB) : v != 0;
}

// MP_COL8_ZNT: the column kernels' Z loads and stores non-temporal (1) or default policy (0).  Default:
// on for fp32 (same box: 8.51 -> 8.38 ms per B = 256 forward, the same PMC bytes; profiles/r5l, r5m), off
// for bf16 (col8_bf 0.0995 -> 0.1085 ms with it; profiles/r5m_bf16).  `resident` (the forward's whole
// batch <= 32: its Z, maps and spectral weights fit the 256 MB Infinity Cache): default policy, so the next kernel's reads hit there (interleaved same-box
// timing, both Z switches off: B = 1 0.962 -> 0.945 ms, B = 32 1.445 -> 1.419, B = 64 2.41 -> 2.48;
// profiles/r5_ab/r5w).  Also default policy for slices of <= 64 images when the maps are streamed
// (MP_MAP_NT): a slice's Z (<= 87 MB) then shares the Infinity Cache with the resident spectral weights
// (B = 128, slices of 64: 4.048 -> 3.977 ms per forward, both Z switches; at B = 192 / 256 / 64 it loses:
// 6.04 -> 6.15, 7.87 -> 8.11, 2.368 -> 2.429; profiles/r6/ab/ab_map_nt.jsonl)
static bool z_default_policy(bool bf, int B, int ntot) { return ntot <= 32 || (map_nt(bf, ntot) && B <= 64); }
static bool col8_znt(bool bf, int B, int ntot) {
  static const int v = [] {
    const char* e = std::getenv("MP_COL8_ZNT");
    return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
  }();
  return v < 0 ? !bf && !z_default_policy(bf, B, ntot) : v != 0;
}

// MP_COL8P: slices of at least this many images run col8p_kernel (fp32; 0 = never); MP_COL8P_BLOCKS:
// its grid (default: one block per CU).  Same box (profiles/r6/ab/ab_col8_batches.jsonl): B = 256 (two
// slices of 128) 8.00 vs 8.05 ms per forward with col8_kernel; B = 128 (slices of 64) 4.35 vs 4.23 --
// a persistent launch holding every CU keeps the other slice's kernels off the chip until it ends
static int col8p_minb() {
  static const int v = [] {
    const char* e = std::getenv("MP_COL8P");
    return e ? std::atoi(e) : 128;
  }();
  return v;
}
// MP_COL8Q (default 0): 1 runs the software-pipelined form col8q_kernel instead of col8p_kernel (same
// box, B = 256: 0.179 vs 0.170 ms; profiles/r6/ab/ab_col8.jsonl)
static bool col8q_on() {
  static const bool v = [] {
    const char* e = std::getenv("MP_COL8Q");
    return e ? std::atoi(e) != 0 : false;
  }();
  return v;
}
// MP_COL8P_BF (default 1): the bf16 path's slices of >= MP_COL8P images run col8p_bf_kernel
static bool col8p_bf_on() {
  static const bool v = [] {
    const char* e = std::getenv("MP_COL8P_BF");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}
static int col8p_blocks() {
  static const int v = [] {
    const char* e = std::getenv("MP_COL8P_BLOCKS");
    if (e) return std::max(1, std::atoi(e));
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return std::max(1, ncu);
  }();
  return v;
}

hipError_t launch_col_gemm(void* Z, const void* Gc, int B, float unscale, hipStream_t st, bool bf, int ntot) {
  if (B <= 0) return hipSuccess;
  const int ngrp = (B + CG_NI - 1) / CG_NI;
  if (!bf && col8p_minb() > 0 && B >= col8p_minb()) {
    const int nitems = Z_CLS * ngrp, nblk = std::min(nitems, col8p_blocks());
    if (col8q_on()) {
      if (col8_znt(false, B, ntot))
        hipLaunchKernelGGL((col8q_kernel<true>), dim3(nblk), dim3(512), 0, st, static_cast<cpx*>(Z),
                           static_cast<const uint4*>(Gc), B, ngrp, nitems, unscale);
      else
        hipLaunchKernelGGL((col8q_kernel<false>), dim3(nblk), dim3(512), 0, st, static_cast<cpx*>(Z),
                           static_cast<const uint4*>(Gc), B, ngrp, nitems, unscale);
      return hipGetLastError();
    }
    if (col8_znt(false, B, ntot))
      hipLaunchKernelGGL((col8p_kernel<true>), dim3(nblk), dim3(512), 0, st, static_cast<cpx*>(Z),
                         static_cast<const uint4*>(Gc), B, ngrp, nitems, unscale);
    else
      hipLaunchKernelGGL((col8p_kernel<false>), dim3(nblk), dim3(512), 0, st, static_cast<cpx*>(Z),
                         static_cast<const uint4*>(Gc), B, ngrp, nitems, unscale);
    return hipGetLastError();
  }
  if (bf && col8p_minb() > 0 && B >= col8p_minb() && col8p_bf_on()) {
    const int nitems = Z_CLS * ngrp, nblk = std::min(nitems, col8p_blocks());
    if (col8_znt(true, B, ntot))
      hipLaunchKernelGGL((col8p_bf_kernel<true>), dim3(nblk), dim3(512), 0, st, Z, static_cast<const uint4*>(Gc), B,
                         ngrp, nitems);
    else
      hipLaunchKernelGGL((col8p_bf_kernel<false>), dim3(nblk), dim3(512), 0, st, Z, static_cast<const uint4*>(Gc), B,
                         ngrp, nitems);
    return hipGetLastError();
  }
  if (bf) {
#define MP_COL8B(N)                                                                                          \
  hipLaunchKernelGGL((col8_bf_kernel<N>), dim3(CG_NC8 * 8 * ngrp), dim3(512), 0, st, Z, static_cast<const uint4*>(Gc), \
                     B, ngrp)
    if (col8_znt(true, B, ntot)) MP_COL8B(true);
    else MP_COL8B(false);
#undef MP_COL8B
  } else {
#define MP_COL8(N)                                                                                       \
  hipLaunchKernelGGL((col8_kernel<N>), dim3(CG_NC8 * 8 * ngrp), dim3(512), 0, st, static_cast<cpx*>(Z), \
                     static_cast<const uint4*>(Gc), B, ngrp, unscale)
    if (col8_znt(false, B, ntot)) MP_COL8(true);
    else MP_COL8(false);
#undef MP_COL8
  }
  return hipGetLastError();
}

// MP_ROW8_ZNT: row8_kernel's Z loads and stores non-temporal (1) or default policy (0).  Default: on for
// fp32 (interleaved same-box timing 8.27 -> 8.21 ms per B = 256 forward; profiles/r5o), off for bf16
// (5.080 vs 5.079 ms); off where col8_znt is (z_default_policy)
static bool row8_znt(bool bf, int B, int ntot) {
  static const int v = [] {
    const char* e = std::getenv("MP_ROW8_ZNT");
    return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
  }();
  return v < 0 ? !bf && !z_default_policy(bf, B, ntot) : v != 0;
}

// MP_ROWQ_MAXB: batch slices up to this many images run row A as rowq_a_kernel (fp32; default 8)
static int rowq_maxb() {
  static const int v = [] {
    const char* e = std::getenv("MP_ROWQ_MAXB");
    return e ? std::atoi(e) : 8;
  }();
  return v;
}

hipError_t launch_row(int mode, void* Z, const ConvArgs& a, const void* or_x3, float or_us, const void* ir_x3,
                      float ir_us, const float* O0, int B, hipStream_t st, bool bf, int ntot) {
  if (B <= 0) return hipSuccess;
  if (a.H < 1 || a.H > 64 || (a.W != 32 && a.W != 64)) return hipErrorInvalidValue;
  const bool znt = row8_znt(bf, B, ntot), mnt = map_nt(bf, ntot);
  if (mode == ROW_A && !bf && B <= rowq_maxb()) {
#define MP_ROWQ(ZV, MV) hipLaunchKernelGGL((rowq_a_kernel<ZV, MV>), dim3(B * 32), dim3(RQ_NT), 0, st, Z, a)
    if (znt) {
      if (mnt) MP_ROWQ(true, true);
      else MP_ROWQ(true, false);
    } else {
      if (mnt) MP_ROWQ(false, true);
      else MP_ROWQ(false, false);
    }
#undef MP_ROWQ
    return hipGetLastError();
  }
  const dim3 g(B * 8), t(R8_NT);
#define MP_ROW8K(M, BFV, ZV, MV) \
  hipLaunchKernelGGL((row8_kernel<M, BFV, ZV, MV>), g, t, 0, st, Z, a, or_x3, or_us, ir_x3, ir_us, O0)
#define MP_ROW8(M, BFV)                            \
  if (znt) {                                       \
    if (mnt) MP_ROW8K(M, BFV, true, true);         \
    else MP_ROW8K(M, BFV, true, false);            \
  } else {                                         \
    if (mnt) MP_ROW8K(M, BFV, false, true);        \
    else MP_ROW8K(M, BFV, false, false);           \
  }
#define MP_ROW8S(BFV)                               \
  switch (mode) {                                   \
    case ROW_A: MP_ROW8(ROW_A, BFV); break;         \
    case ROW_B: MP_ROW8(ROW_B, BFV); break;         \
    case ROW_FINAL: MP_ROW8(ROW_FINAL, BFV); break; \
    case ROW_INIT: MP_ROW8(ROW_INIT, BFV); break;   \
    default: return hipErrorInvalidValue;           \
  }
  if (bf) {
    MP_ROW8S(true)
  } else {
    MP_ROW8S(false)
  }
#undef MP_ROW8S
#undef MP_ROW8
#undef MP_ROW8K
  return hipGetLastError();
}

}  // namespace mp
