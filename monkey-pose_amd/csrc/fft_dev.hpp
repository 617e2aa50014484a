// Device helpers shared by the FFT-path kernels (k_fft.hip: the 2-D FFT kernels of the bf16 path and
// the small-batch forms; k_fft4.hip: the fp32 four-step loop): complex fp32 arithmetic, the 8 / 9 /
// 72-point DFTs, the map load / store forms of the hGRU maps and the f16x3 / bf16 1x1 gate GEMMs.
#pragma once
#include "conv_epi.hpp"
#include "fft_consts.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace mp {

constexpr int FX = FFT_N / 2 + 1;      // 37
#ifndef FFT_NT
#define FFT_NT 192                     // threads per FFT block (row phase 128, column phase 148)
#endif
constexpr int FNT = FFT_NT;
// phase timestamps (tools/fft_stamps.hip only; compiled out of the library): thread 0 of every
// block records the shader clock at the phase boundaries of the FFT kernels
#ifdef FFT_STAMP
__device__ unsigned long long fft_stamp_buf[16384 * 8];
#define FFT_STAMP_AT(k) \
  do { \
    if (threadIdx.x == 0) fft_stamp_buf[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define FFT_STAMP_AT(k) \
  do { \
  } while (0)
#endif
#ifndef FFT_MINB
#define FFT_MINB 2                     // blocks per CU the FFT kernels are register-budgeted for
#endif
#ifndef FFT_MINB_BF
#define FFT_MINB_BF 3                  // the bf16 kernels (f16 LDS tiles, 38.5 KB): 3 blocks per CU
#endif
constexpr int NF = FFT_N * FX;         // 2664 frequencies
// frequency order of S, Y and the spectral weights, per dtype.  fy-major, f = fy * 37 + fx: at one
// fy a wave of column threads (16 fx x 4 channels) reads / writes 512 (bf16: 256) contiguous bytes,
// and the forward column phase stores straight from registers; fx-major, f = fx * 72 + fy: each
// column thread's 72 values are contiguous (a wave-instruction touches 16 separate pieces) and S is
// staged through LDS into 1-KiB stores.  Measured (same box, B = 256): bf16 inv_a_fwd 0.213 -> 0.200,
// fft_fwd 0.100 -> 0.096 ms fy-major; fp32 the other way (inv_a_fwd 0.343 -> 0.352, fft_inv 0.138 ->
// 0.144), so fp32 stays fx-major.  The spectral GEMM only sees quads of 4 consecutive f either way.
#ifndef FFT_FYMAJOR_F32
#define FFT_FYMAJOR_F32 0
#endif
#ifndef FFT_FYMAJOR_BF
#define FFT_FYMAJOR_BF 1
#endif
template <bool BF>
__host__ __device__ constexpr bool fy_major() { return BF ? FFT_FYMAJOR_BF : FFT_FYMAJOR_F32; }
template <bool BF>
__host__ __device__ constexpr int spec_f(int fx, int fy) { return fy_major<BF>() ? fy * FX + fx : fx * FFT_N + fy; }
// scale of the input spectra before the f16 split: |S| <= 4096 max|x|, so activations up to
// 1023 in magnitude stay inside f16 range (hGRU maps are tanh / sigmoid-gated, |x| <~ 1)
constexpr float SPEC_SCALE = 1.0f / 64.0f;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x16 mfma16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// MP_DTYPE_BF16: spectra S / Y hold one bf16 (re, im) pair per channel (16 B per 4-channel group
// and frequency instead of 32 B), the spectral and gate GEMMs are one v_mfma_f32_32x32x16_bf16
// product with fp32 accumulation, no scaling (bf16 has the fp32 exponent range)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x16 mfmab(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};   // round to nearest even (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(uint32_t, v);
}


// complex fp32: a 2-float vector, so a complex add is one v_pk_add_f32 and a twiddle product two
// v_pk_fma_f32 / v_pk_mul_f32.  The re/im half swap of swp() is one v_pk_mov_b32 (op_sel:[1,0], a
// plain 64-bit move with its halves exchanged) in inline asm, so the compiler cannot fold it into an
// op_sel half-select of a packed-FP32 source (round 5: it replaced two v_mov_b32 per swap, -11 % of
// the row kernels' VALU instructions, same bits).  The folded form
// (round 3's FFT_PACKED = 1: 7,902 such instructions in this file) gave results that differed from
// the scalar build's and, under the two-stream hGRU schedule, from run to run (13-19 of 256 crops,
// up to 2.1e-5, all in the batch's head / tail, where one slice runs alone:
// profiles/r3a/pk_probe_det_fp32_pk0_pk1_pk2.log); this form is bit-identical to the scalar build
// and deterministic.  The cause was not isolated: tools/pk_hazard.hip runs the exact folded
// instruction (v_pk_fma_f32 v[a:a+1], v[a:a+1], s[k:k+1], v[a:a+1] op_sel:[1,0,0]
// op_sel_hi:[0,1,1]) with and without destination overlap at 1-16 waves per SIMD and finds every
// lane exact (profiles/r4/pk_hazard.json), and the slice-boundary audit in DESIGN.md found no
// cross-slice address.  Guarded by tests/test_gpu_parity.py::test_stream_split_is_bit_identical and
// test_batch_invariance_and_determinism.  (Round 3, same box: this form against the scalar one,
// fft_fwd 0.168 -> 0.157 ms, inv_a_fwd 0.339 -> 0.329, fft_inv 0.130 -> 0.126, same bits.)
typedef float cpx __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cpx cfma(cpx a, cpx b, cpx c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ cpx swp(cpx a) {
  cpx r;
  asm("v_pk_mov_b32 %0, %1, %1 op_sel:[1,0]" : "=v"(r) : "v"(a));
  return r;
}

// streaming (non-temporal) access to the once-written, once-read spectra and P2 (A/B switches)
#ifndef FFT_NT_ST
#define FFT_NT_ST 1         // staged 16-B stores of S and Y (fft_fwd 0.198 -> 0.173 ms, spec_gemm -2 %)
#endif
#ifndef FFT_EPI_EU
#define FFT_EPI_EU 8        // inv_a_fwd epilogue, fp32 maps: pixels per thread per load chunk
#endif
#ifndef FFT_EPI_STAGE
#define FFT_EPI_STAGE 1     // last B epilogue: the NHWC output staged per wave in LDS, stored as contiguous runs
#endif
#ifndef FFT_EPI_PIPE
#define FFT_EPI_PIPE 1      // inv_a_fwd epilogue, bf16 maps: next chunk's X / O loads issued before this chunk's math
#endif
#ifndef FFT_EPI_EARLY
#define FFT_EPI_EARLY 1     // chunk 0's X / O loads issued before the inverse row phase (implies the pipelining)
#endif
// FFT_C4: the loop's P2 and I maps in the C4 layout (mp_common.hpp c4_index; bit 0: P2, bit 1: I), so
// the inverse kernels (fft_inv, inv_a_fwd, their latency forms) write each block's 4-channel group as
// one contiguous run instead of 16-B halves of 32-B C8 pixels; spec_epi_b and the state stacks read
// them there.  Probes of the two writes made contiguous: fft_inv 0.134 -> 0.125 ms, inv_a_fwd 0.340 ->
// 0.328 ms at B = 256.  Unswizzled C4 reads cost fp32 epi_b 0.259 -> 0.289 ms on one box; with the
// odd group's row halves swapped (C4_SWZ) the same-box A/B against C8 is fp32 10.65 -> 10.46 ms, bf16
// 6.20 -> 6.10, B = 64 3.34 -> 3.28 (profiles/r4o).  Bit 2 puts the state O there too (gate_init /
// epi_b write it, inv_a_fwd's A epilogue and epi_b read it): fp32 10.21-10.27 -> 10.03-10.04 ms
// (epi_b 0.279 -> 0.256, inv_a_fwd 0.314 -> 0.309), bf16 6.13-6.15 -> 6.11 (profiles/r4o/c4_state_ab.log).
// Bit 3 the drive X (conv_3's backbone epilogue writes it, ConvArgs::dst_c4): fp32 9.95 -> 9.89 ms
// (inv_a_fwd 0.307 -> 0.299), bf16 6.08-6.10 -> 6.05-6.06 (profiles/r4o/c4_drive_ab.log).  Og (read by
// the forward FFT's row loads, where the C4 probe gained nothing) stays C8.  0 restores C8 maps.
#ifndef FFT_C4
#define FFT_C4 15
#endif
// (bit 0: P2, bit 1: I)
__device__ __forceinline__ size_t pp_index(int b, int q, int y, int x, int e, int H, int W) {
  return (FFT_C4 & 1) ? c4_index(b, q, y, x, e, H, W) : c8_index(b, q, y, x, e, H, W);
}
__device__ __forceinline__ size_t ii_index(int b, int q, int y, int x, int e, int H, int W) {
  return (FFT_C4 & 2) ? c4_index(b, q, y, x, e, H, W) : c8_index(b, q, y, x, e, H, W);
}
// bit 3: the drive X (written by conv_3's backbone epilogue, ConvArgs::dst_c4; read by the A epilogue)
__device__ __forceinline__ size_t xx_index(int b, int q, int y, int x, int e, int H, int W) {
  return (FFT_C4 & 8) ? c4_index(b, q, y, x, e, H, W) : c8_index(b, q, y, x, e, H, W);
}
// bit 2: the state O (written by gate_init / epi_b, read by inv_a_fwd's A epilogue and epi_b)
__device__ __forceinline__ size_t oo_index(int b, int q, int y, int x, int e, int H, int W) {
  return (FFT_C4 & 4) ? c4_index(b, q, y, x, e, H, W) : c8_index(b, q, y, x, e, H, W);
}
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st16(uint4* p, uint4 v) {
  if constexpr (FFT_NT_ST) {
    __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(p));
  } else {
    *p = v;
  }
}
__device__ __forceinline__ cpx unpack_bf2(uint32_t u) {   // bf16 -> fp32 is exact: the high half
  return cpx{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
// hGRU maps of the FFT path (the drive X, the states O, I, Og and the B half-step's P2): fp32 C8,
// or -- BM, the MP_DTYPE_BF16 default -- bf16 C8 at the same element index (half the bytes; round
// to nearest even on store, exact on load).  The final NHWC output for fc_1 stays fp32.
// NT: non-temporal loads / stores -- the batch-streaming kernels of a batch that
// does not fit the Infinity Cache, so that the maps do not evict what is re-read there (the spectral
// weights, read by every column launch)
typedef unsigned map_u2 __attribute__((ext_vector_type(2)));
template <bool BM, bool NT = false>
__device__ __forceinline__ f32x4 map_ld4(const float* base, size_t idx) {
  if constexpr (BM) {
    const map_u2* p = reinterpret_cast<const map_u2*>(reinterpret_cast<const uint16_t*>(base) + idx);
    const map_u2 u = NT ? __builtin_nontemporal_load(p) : *p;
    const cpx a = unpack_bf2(u.x), b = unpack_bf2(u.y);
    return f32x4{a.x, a.y, b.x, b.y};
  } else if constexpr (NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(base + idx));
  } else {
    return *reinterpret_cast<const f32x4*>(base + idx);
  }
}
template <bool BM, bool NT = false>
__device__ __forceinline__ void map_st4(float* base, size_t idx, f32x4 v) {
  if constexpr (BM) {
    map_u2* p = reinterpret_cast<map_u2*>(reinterpret_cast<uint16_t*>(base) + idx);
    const map_u2 u = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
    if constexpr (NT) __builtin_nontemporal_store(u, p);
    else *p = u;
  } else if constexpr (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(base + idx));
  else
    *reinterpret_cast<f32x4*>(base + idx) = v;
}
// maps read exactly once by the next kernel (P2, I).  Plain stores: the non-temporal hint on them
// made fft_inv 0.142 -> 0.229 ms (round 2, tools/exp_fft.hip), and on the inverse column phase's Y
// loads +7-15 %; both forms were removed in round 4.
template <bool BM>
__device__ __forceinline__ void map_st4_stream(float* base, size_t idx, f32x4 v) {
  map_st4<BM>(base, idx, v);
}
template <bool BM>
__device__ __forceinline__ cpx map_ld2(const float* base, size_t idx) {
  if constexpr (BM) {
    return unpack_bf2(*reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(base) + idx));
  } else {
    const float2 t = *reinterpret_cast<const float2*>(base + idx);
    return cpx{t.x, t.y};
  }
}
// sigmoid / tanh on v_exp_f32 + v_rcp_f32 (absolute error ~1e-7).  The A epilogue uses ftanh too
// (ocml's tanhf branches per lane: a polynomial below |x| = 0.625, an exp form above, both run by a
// mixed wave; an odd rational minimax was also tried and removed in round 4)
__device__ __forceinline__ float fsigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)); }
// the A epilogue's tanh argument x - (beta o + nu) (p + lateral_bias) (hgru_module.py:797-799) with
// both contractions written out: left to -ffp-contract, whether a product was fused into the
// following add depended on the surrounding code, and the small-batch kernels rounded differently
__device__ __forceinline__ float epi_a(float x, float o, float p, float be, float nu, float lat) {
  return fmaf(-fmaf(be, o, nu), p + lat, x);
}
__device__ __forceinline__ float atanh_f(float x) { return ftanh(x); }   // the A epilogue's tanh
__device__ __forceinline__ cpx scale(cpx a, float s) { return a * s; }
// a * e^{S i 2 pi m / 72}  (S = -1 forward, +1 inverse)
template <int S>
__device__ __forceinline__ cpx twid(cpx a, int m) {
  const float c = TW72_COS[m], s = S * TW72_SIN[m];
  return cfma(swp(a), cpx{-s, s}, a * c);   // (x c - y s, y c + x s)
}
// a * e^{S i pi / 2}
template <int S>
__device__ __forceinline__ cpx rotq(cpx a) {
  return swp(a) * cpx{(float)-S, (float)S};
}

template <int S>
__device__ __forceinline__ void dft8(cpx (&x)[8]) {
  constexpr float H = 0.70710678118654752f;
  const cpx a0 = x[0] + x[4], a1 = x[0] - x[4], a2 = x[2] + x[6], a3 = rotq<S>(x[2] - x[6]);
  const cpx a4 = x[1] + x[5], a5 = x[1] - x[5], a6 = x[3] + x[7], a7 = rotq<S>(x[3] - x[7]);
  const cpx b0 = a0 + a2, b2 = a0 - a2, b1 = a1 + a3, b3 = a1 - a3;
  const cpx b4 = a4 + a6, b6 = a4 - a6, b5 = a5 + a7, b7 = a5 - a7;
  const cpx t6 = rotq<S>(b6);
  // b5 * W8^1 = H (b5 + rotq b5), b7 * W8^3 = H (rotq b7 - b7): the products by H fused into the
  // butterflies explicitly (contraction left to the compiler was decided per call site: the same
  // transform rounded differently in the batched and the small-batch kernels)
  const cpx u5 = cfma(swp(b5), cpx{(float)-S, (float)S}, b5);
  const cpx u7 = cfma(swp(b7), cpx{(float)-S, (float)S}, -b7);
  x[0] = b0 + b4;
  x[4] = b0 - b4;
  x[2] = b2 + t6;
  x[6] = b2 - t6;
  x[1] = cfma(u5, cpx{H, H}, b1);
  x[5] = cfma(u5, cpx{-H, -H}, b1);
  x[3] = cfma(u7, cpx{H, H}, b3);
  x[7] = cfma(u7, cpx{-H, -H}, b3);
}

// FOLD: a +- rotq(v) as one fma each on swp(v) (3 instructions fewer; the same bits).  k_fft.hip's
// 72-point transforms keep the unfolded form: folded, fft_inv_a_fwd_kernel spills (336 B / lane)
template <int S>
__device__ __forceinline__ void dft8_fold(cpx (&x)[8]) {
  constexpr float H = 0.70710678118654752f;
  constexpr cpx RP = {(float)-S, (float)S}, RM = {(float)S, (float)-S};
  const cpx a0 = x[0] + x[4], a1 = x[0] - x[4], a2 = x[2] + x[6], v3 = swp(x[2] - x[6]);
  const cpx a4 = x[1] + x[5], a5 = x[1] - x[5], a6 = x[3] + x[7], v7 = swp(x[3] - x[7]);
  const cpx b0 = a0 + a2, b2 = a0 - a2, b1 = cfma(v3, RP, a1), b3 = cfma(v3, RM, a1);
  const cpx b4 = a4 + a6, b6 = a4 - a6, b5 = cfma(v7, RP, a5), b7 = cfma(v7, RM, a5);
  const cpx v6 = swp(b6);
  // b5 * W8^1 = H (b5 + rotq b5), b7 * W8^3 = H (rotq b7 - b7): the products by H fused into the
  // butterflies explicitly (contraction left to the compiler was decided per call site: the same
  // transform rounded differently in the batched and the small-batch kernels)
  const cpx u5 = cfma(swp(b5), cpx{(float)-S, (float)S}, b5);
  const cpx u7 = cfma(swp(b7), cpx{(float)-S, (float)S}, -b7);
  x[0] = b0 + b4;
  x[4] = b0 - b4;
  x[2] = cfma(v6, RP, b2);
  x[6] = cfma(v6, RM, b2);
  x[1] = cfma(u5, cpx{H, H}, b1);
  x[5] = cfma(u5, cpx{-H, -H}, b1);
  x[3] = cfma(u7, cpx{H, H}, b3);
  x[7] = cfma(u7, cpx{-H, -H}, b3);
}

template <int S>
__device__ __forceinline__ void dft3(cpx& z0, cpx& z1, cpx& z2) {
  constexpr float R3 = 0.86602540378443865f;
  const cpx t = z1 + z2, d = z1 - z2;
  const cpx m = z0 - scale(t, 0.5f);
  z0 = z0 + t;
  z1 = cfma(swp(d), cpx{-S * R3, S * R3}, m);   // m + s, s = swp(d) (-S R3, S R3): fused explicitly
  z2 = cfma(swp(d), cpx{S * R3, -S * R3}, m);   // m - s (see dft8)
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

// in-register 72-point DFT, X[k] = sum_n v[n] e^{S 2 pi i n k / 72} (unnormalised).
// Good-Thomas prime-factor form of 72 = 8 x 9 (gcd 1): n = (9 n1 + 8 n2) mod 72,
// k = (9 k1 + 64 k2) mod 72 makes e^{2 pi i n k / 72} = e^{2 pi i n1 k1 / 8} e^{2 pi i n2 k2 / 9}, so
// the 8-point and 9-point passes need no twiddles between them (56 complex products fewer per
// transform than Cooley-Tukey n = 9 n1 + n2; both index maps are register renamings)
template <int S>
__device__ __forceinline__ void fft72(cpx (&v)[72]) {
#ifdef FFT_PROBE_NOFFT   // timing probe (tools/fft_stamps.hip): data movement without the transforms
  return;
#endif
  cpx a[9][8];
#pragma unroll
  for (int n2 = 0; n2 < 9; ++n2) {
    cpx t[8];
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) t[n1] = v[(9 * n1 + 8 * n2) % 72];
    dft8<S>(t);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) a[n2][k1] = t[k1];
  }
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) {
    cpx u[9];
#pragma unroll
    for (int n2 = 0; n2 < 9; ++n2) u[n2] = a[n2][k1];
    dft9<S>(u);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) v[(9 * k1 + 64 * k2) % 72] = u[k2];
  }
}

constexpr float GATE_VSCALE = 256.0f;   // activations entering a gate: |v| < 255 stays in f16 range

#ifndef GATE_IL
#define GATE_IL 1   // gate_x3: the two output blocks' MFMA chains interleaved (0: one after the other, A/B)
#endif


// Y[n2] = sum_cin G[cin][32 n2 + row] V[cin][pixel], f16x3; gpk = [n2][s][hi|lo][lane] f16x8
__device__ __forceinline__ void gate_x3(const f16x8* __restrict__ gpk, const f32x16 (&V)[2], f32x16 (&Y)[2],
                                        int lane, float unscale) {
  // the split in channel pairs: one v_pk_mul_f32, v_cvt_pk_f16_f32 for hi and lo, one v_pk_add_f32
  // (round to nearest even as (_Float16); v - hi is exact)
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  f16x8 bh[4], bl[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const int r = 8 * (s & 1) + e;
      const f2 v = f2{V[s >> 1][r], V[s >> 1][r + 1]} * GATE_VSCALE;
      const h2 hv = __builtin_convertvector(v, h2);
      const h2 lv = __builtin_convertvector(v - __builtin_convertvector(hv, f2), h2);
      bh[s][e] = hv[0];
      bh[s][e + 1] = hv[1];
      bl[s][e] = lv[0];
      bl[s][e + 1] = lv[1];
    }
#if GATE_IL
  // the two 32-channel output blocks' chains interleaved (each accumulator keeps its own product
  // order: bit-identical to the sequential form): one block's MFMA covers the other's fragment
  // reads, where the sequential second chain waited out an LDS read before each of its MFMAs
  f32x16 acc[2] = {};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    f16x8 ah[2], al[2];
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) {
      ah[n2] = gpk[((n2 * 4 + s) * 2) * 64 + lane];
      al[n2] = gpk[((n2 * 4 + s) * 2 + 1) * 64 + lane];
    }
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) acc[n2] = mfma16(al[n2], bh[s], acc[n2]);
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) acc[n2] = mfma16(ah[n2], bl[s], acc[n2]);
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) acc[n2] = mfma16(ah[n2], bh[s], acc[n2]);
  }
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) Y[n2] = acc[n2] * unscale;
#else
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f16x8 ah = gpk[((n2 * 4 + s) * 2) * 64 + lane], al = gpk[((n2 * 4 + s) * 2 + 1) * 64 + lane];
      acc = mfma16(al, bh[s], acc);
      acc = mfma16(ah, bl[s], acc);
      acc = mfma16(ah, bh[s], acc);
    }
    Y[n2] = acc * unscale;
  }
#endif
}

// bf16 variant (MP_DTYPE_BF16): one product, gpk = [n2][s][lane] bf16x8 in the same K order
__device__ __forceinline__ void gate_bf(const uint4* __restrict__ gpk, const f32x16 (&V)[2], f32x16 (&Y)[2],
                                       int lane) {
  bf16x8 bv[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[s][e] = (__bf16)V[s >> 1][8 * (s & 1) + e];
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfmab(__builtin_bit_cast(bf16x8, gpk[(n2 * 4 + s) * 64 + lane]), bv[s], acc);
    Y[n2] = acc;
  }
}

template <bool BF>
__device__ __forceinline__ void gate_any(const void* gpk, const f32x16 (&V)[2], f32x16 (&Y)[2], int lane, float us) {
  if constexpr (BF)
    gate_bf(static_cast<const uint4*>(gpk), V, Y, lane);
  else
    gate_x3(static_cast<const f16x8*>(gpk), V, Y, lane, us);
}

}  // namespace mp
