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
//   fft_inv   Y                 -> P (C4)            2-D inverse (complex-to-real) FFT
//   inv_a_fwd Y, X, O           -> I (C4), S         inverse FFT + A epilogue + forward FFT of I
//   epi_b     P, I, O           -> O', Og' (C8)      B epilogue with the 1x1 gates (all 64 channels)
//
// G[f][ci][co] = (1/N^2) sum_{ky,kx} w[ky][kx][ci][co] exp(-2 pi i (fy (R-ky) + fx (R-kx)) / N)
// (cross-correlation written as a convolution with the flipped kernel, inverse-DFT scale folded in)
// is computed once per weight set in double precision.  The FFTs are fp32 (twiddles rounded once
// from double); the spectral GEMM is fp32-accurate "f16x3" (each operand split into power-of-two
// scaled f16 hi + lo, three f16 MFMA products, fp32 accumulation, as k_conv64x3.hip), so the path
// is fp32-class: error ~1e-6 of max|output| against the float64 oracle.
//
// Frequencies: f = fy * 37 + fx, fy in [0, 72), fx in [0, 37) (the real-input half spectrum), so
// at one fy the column threads of a wave (16 fx x 4 channels) read / write 512 contiguous bytes
// (bf16; spec_f<BF>() below: fp32 keeps f = fx * 72 + fy).  Spectra live image-major in HBM,
// [b][cq][f][32 B] (cq = channel / 4, f fastest): every FFT block reads / writes one contiguous run.
//   S (input spectra): 32 B = 8 f16 hi (re/im of the 4 channels, interleaved) + 8 f16 lo;
//   Y (output spectra): 32 B = 4 x complex64.
// The spectral GEMM needs, for ONE frequency, 32 images of one operand half side by side (an MFMA
// fragment); it loads (4 frequencies x 32 images) tiles whole-line and transposes them in LDS.
#include "fft_dev.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace mp {


// ---------------------------------------------------------------------------------------------
// 2-D FFT phases.  One block per (image b, channel group cq = 4 channels), 192 threads; the
// 72 x 72 transform is two passes of 72-point FFTs in registers with one LDS transpose between:
//   row phase (128 threads): row y, channel pair p -- the two real rows packed as one complex FFT
//   column phase (148 threads): column (fx, c), fx = 0..36 (the real-input half spectrum)
constexpr int FWD_LD = 65;        // pitch (complex) of the forward transpose T[fx][c][y]
constexpr int STG_LD = 296;       // output staging pitch per fx, dwords (36 fy x 8 dwords + 8 pad)
constexpr int STG_LD_B = 148;     // the same for bf16 spectra (36 fy x 4 dwords + 4 pad)
constexpr int FFT_LDS = FX * 4 * FWD_LD;   // complex elements of the block's LDS (76,960 B)

// The block's LDS transpose / parking space.  fp32 path: complex64 entries.  bf16 path (H): complex
// f16 entries (4 B) -- the spectra it feeds are bf16 (8-bit mantissa), so the f16 (11-bit)
// intermediates add ~1/8 of that rounding, and the halved tile (38.5 KB) lets 3 blocks share a CU
// instead of 2.  Values stay far inside f16 range (row-FFT outputs <= 64 max|map|, |map| <~ 2).
template <bool H>
struct Lds;
template <>
struct Lds<false> {
  typedef cpx elem;
  cpx* p;
  __device__ __forceinline__ cpx get(int i) const { return p[i]; }
  __device__ __forceinline__ void set(int i, cpx v) const { p[i] = v; }
  __device__ __forceinline__ uint32_t* raw() const { return reinterpret_cast<uint32_t*>(p); }
};
template <>
struct Lds<true> {
  typedef uint32_t elem;
  uint32_t* p;
  __device__ __forceinline__ cpx get(int i) const {
    const f16x2 h = __builtin_bit_cast(f16x2, p[i]);
    return cpx{(float)h[0], (float)h[1]};
  }
  __device__ __forceinline__ void set(int i, cpx v) const {
    const f16x2 h = {(_Float16)v.x, (_Float16)v.y};
    p[i] = __builtin_bit_cast(uint32_t, h);
  }
  __device__ __forceinline__ uint32_t* raw() const { return p; }
};

// forward row phase: the packed row v (a + ib, zero padded) -> half spectra of a and b in T
template <bool H>
__device__ __forceinline__ void fwd_rows_to_T(cpx (&v)[72], int y, int p, Lds<H> T) {
  fft72<-1>(v);
  // Z = FFT(a + i b):  A[k] = (Z[k] + conj Z[-k]) / 2,  B[k] = (Z[k] - conj Z[-k]) / (2i)
#pragma unroll
  for (int k = 0; k < FX; ++k) {
    const cpx zk = v[k], zm = v[(72 - k) % 72];
    const cpx A = cfma(zm, cpx{1.f, -1.f}, zk) * 0.5f;               // (zk.x + zm.x, zk.y - zm.y) / 2
    const cpx B = cfma(swp(zk), cpx{1.f, -1.f}, swp(zm)) * 0.5f;     // (zk.y + zm.y, zm.x - zk.x) / 2
    T.set((k * 4 + 2 * p) * FWD_LD + y, A);
    T.set((k * 4 + 2 * p + 1) * FWD_LD + y, B);
  }
}

// forward column phase: T -> S[b][cq][f] (scaled, split to f16 hi / lo).  T must be complete on
// entry.  Fy-major (f = fy * 37 + fx, fy_major<BF>) the column threads store straight to HBM: at one fy
// the wave's 16 columns x 4 channels are 512 contiguous bytes (fp32: the quad's hi / lo halves are
// regrouped by two DPP quad_perms so each lane stores 8 contiguous bytes), no LDS staging and no
// barrier (the last phase of its kernels).  Otherwise (f = fx * 72 + fy) the block's contiguous
// 85 KiB S run is written through LDS (T's space) in two fy halves, 1 KiB per wave-instruction;
// that form is called by ALL threads (it contains barriers).
template <bool BF>
__device__ __forceinline__ void fwd_cols_to_S(Lds<BF> T, void* __restrict__ S, int b, int cq, int tid) {
  const bool col = tid < FX * 4;
  const int fx = tid >> 2, c = tid & 3;
  cpx v[72];
  if constexpr (fy_major<BF>()) {
    if (!col) return;
#pragma unroll
    for (int y = 0; y < 72; ++y) v[y] = y < 64 ? T.get(tid * FWD_LD + y) : cpx{0.f, 0.f};
    fft72<-1>(v);
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    if constexpr (BF) {
      uint32_t* dst = static_cast<uint32_t*>(S) + (((size_t)b * 16 + cq) * NF + fx) * 4 + c;
#pragma unroll
      for (int fy = 0; fy < 72; ++fy) {
        const uint32_t w = pack_bf2(v[fy].x, v[fy].y);
        if constexpr (FFT_NT_ST)
          __builtin_nontemporal_store(w, dst + fy * FX * 4);
        else
          dst[fy * FX * 4] = w;
      }
    } else {
      // 32-B group of (f, cq): [hi c0 | hi c1 | hi c2 | hi c3 | lo c0 | lo c1 | lo c2 | lo c3] (4 B
      // each = f16 re, im); lane c of the quad stores bytes 8c .. 8c+7
      u32x2_t* dst = reinterpret_cast<u32x2_t*>(S) + (((size_t)b * 16 + cq) * NF + fx) * 4 + c;
      const bool hi_half = c < 2;
#pragma unroll
      for (int fy = 0; fy < 72; ++fy) {
        const float re = v[fy].x * SPEC_SCALE, im = v[fy].y * SPEC_SCALE;
        const _Float16 hr = (_Float16)re, hm = (_Float16)im;
        const f16x2 hv = {hr, hm}, lv = {(_Float16)(re - (float)hr), (_Float16)(im - (float)hm)};
        const int hb = __builtin_bit_cast(int, hv), lb = __builtin_bit_cast(int, lv);
        const int h0 = __builtin_amdgcn_mov_dpp(hb, 0x88, 0xF, 0xF, false);   // quad_perm [0,2,0,2]
        const int l0 = __builtin_amdgcn_mov_dpp(lb, 0x88, 0xF, 0xF, false);
        const int h1 = __builtin_amdgcn_mov_dpp(hb, 0xDD, 0xF, 0xF, false);   // quad_perm [1,3,1,3]
        const int l1 = __builtin_amdgcn_mov_dpp(lb, 0xDD, 0xF, 0xF, false);
        const u32x2_t w = {(unsigned)(hi_half ? h0 : l0), (unsigned)(hi_half ? h1 : l1)};
        if constexpr (FFT_NT_ST)
          __builtin_nontemporal_store(w, dst + fy * FX * 4);
        else
          dst[fy * FX * 4] = w;
      }
    }
    return;
  }
  if (col) {
#pragma unroll
    for (int y = 0; y < 72; ++y) v[y] = y < 64 ? T.get(tid * FWD_LD + y) : cpx{0.f, 0.f};
    fft72<-1>(v);
  }
  uint32_t* stg = T.raw();
  if constexpr (BF) {
    uint4* dst = reinterpret_cast<uint4*>(S) + ((size_t)b * 16 + cq) * NF;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      lds_barrier();
      if (col) {
#pragma unroll
        for (int j = 0; j < 36; ++j) {
          const cpx z = v[36 * half + j];
          stg[fx * STG_LD_B + j * 4 + c] = pack_bf2(z.x, z.y);
        }
      }
      lds_barrier();
      for (int i = tid; i < FX * 36; i += FNT) {   // per fx: 36 groups x 16 B at f = fx*72 + 36*half
        const int ffx = i / 36, w = i - ffx * 36;
        st16(dst + ffx * 72 + 36 * half + w, *reinterpret_cast<const uint4*>(stg + ffx * STG_LD_B + w * 4));
      }
    }
    return;
  }
  uint4* dst = reinterpret_cast<uint4*>(S) + ((size_t)b * 16 + cq) * NF * 2;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    lds_barrier();   // T (half 0) / the previous half's staging is no longer read
    if (col) {
#pragma unroll
      for (int j = 0; j < 36; ++j) {
        const cpx z = v[36 * half + j];
        const float re = z.x * SPEC_SCALE, im = z.y * SPEC_SCALE;
        const _Float16 hr = (_Float16)re, hi = (_Float16)im;
        const f16x2 hv = {hr, hi}, lv = {(_Float16)(re - (float)hr), (_Float16)(im - (float)hi)};
        stg[fx * STG_LD + j * 8 + c] = __builtin_bit_cast(uint32_t, hv);
        stg[fx * STG_LD + j * 8 + 4 + c] = __builtin_bit_cast(uint32_t, lv);
      }
    }
    lds_barrier();
    // per fx: 36 groups x 32 B = 72 uint4 at f = fx*72 + 36*half
    for (int i = tid; i < FX * 72; i += FNT) {
      const int ffx = i / 72, w = i - ffx * 72;
      st16(dst + (ffx * 72 + 36 * half) * 2 + w, *reinterpret_cast<const uint4*>(stg + ffx * STG_LD + w * 4));
    }
  }
}

// inverse column phase: Y[b][cq][f] -> T[y][c][fx] (rows y < 64).  Direct per-thread loads (72
// independent 8-byte loads in flight per thread) measured faster than an LDS-staged read.
template <bool BF>
__device__ __forceinline__ void inv_cols_to_T(const void* __restrict__ Y, int b, int cq, int tid, Lds<BF> T) {
  if (tid < FX * 4) {
    const int fx = tid >> 2, c = tid & 3;
    const size_t off = (((size_t)b * 16 + cq) * NF + spec_f<BF>(fx, 0)) * 4 + c;
    constexpr int FS = spec_f<BF>(0, 1) * 4;   // element stride of one fy step
    cpx v[72];
    if constexpr (BF) {
      const uint32_t* src = static_cast<const uint32_t*>(Y) + off;
#pragma unroll
      for (int fy = 0; fy < 72; ++fy) v[fy] = unpack_bf2(src[fy * FS]);
    } else {
#ifdef FFT_PROBE_YCOAL   // timing probe (tools/bench_fft.hip): the block's Y run read wave-contiguously
      const cpx* src = static_cast<const cpx*>(Y) + ((size_t)b * 16 + cq) * NF * 4 + tid;
#pragma unroll
      for (int fy = 0; fy < 72; ++fy) v[fy] = src[fy * FX * 4];
#else
      const cpx* src = static_cast<const cpx*>(Y) + off;
#pragma unroll
      for (int fy = 0; fy < 72; ++fy) v[fy] = src[fy * FS];
#endif
    }
    fft72<1>(v);
#pragma unroll
    for (int y = 0; y < 64; ++y) T.set((y * 4 + c) * FX + fx, v[y]);   // rows >= H: unused
  }
}

// inverse row phase: the Hermitian-extended half spectra of rows (y, 2p) and (y, 2p+1) packed as
// C = A + iB, one inverse FFT: v[x].x / v[x].y = the two real output rows
template <bool H>
__device__ __forceinline__ void inv_row_from_T(Lds<H> T, int y, int p, cpx (&v)[72]) {
  const int ta = (y * 4 + 2 * p) * FX, tb = ta + FX;
#pragma unroll
  for (int k = 0; k < FX; ++k) {   // C[k] = A[k] + i B[k];  C[72-k] from A[72-k] = conj A[k] etc.
    const cpx A = T.get(ta + k), B = T.get(tb + k);
    v[k] = cfma(swp(B), cpx{-1.f, 1.f}, A);                               // (A.x - B.y, A.y + B.x)
    if (k > 0 && k < FX - 1) v[72 - k] = cfma(A, cpx{1.f, -1.f}, swp(B));   // (A.x + B.y, B.x - A.y)
  }
  fft72<1>(v);
}

// Rows of the block's 4-channel tile are "parked" in LDS (T's space) between the row transforms
// and global memory: R[(2y + p) * RLD + x] = channels (2p, 2p+1) of pixel (y, x).  Global reads and
// writes of the activation maps then run pixel-major (lane = pixel, one 16-byte float4 of 4
// channels), instead of one strided 8-byte access per row thread.
constexpr int RLD = 73;

// Block -> channel group, XCD-aware: the two 4-channel groups of one C8 chunk (cq = 2q, 2q+1) each
// touch half of every 32-byte pixel chunk.  Workgroups are dispatched round-robin over the 8 XCDs
// (separate L2s), so blocks i and i+8 share an XCD: giving them the two halves of a chunk lets one
// L2 fetch (or write back) each line once instead of two XCDs each moving the whole line
// (rocprofv3 FETCH/WRITE_SIZE showed 2x the algorithmic bytes on these maps otherwise).
__device__ __forceinline__ int fft_block_img(int blk) {
#ifdef FFT_PROBE_WRAP   // timing probe (tools/fft_stamps.hip): every block works on one of WRAP images
  return (blk >> 4) % FFT_PROBE_WRAP;
#else
  return blk >> 4;
#endif
}
__device__ __forceinline__ int fft_block_cq(int blk) {
  const int p = blk & 15;
  return 2 * (p & 7) + (p >> 3);
}

// forward 2-D FFT of one C8 activation map -> S.  The rows are read straight into registers (64
// independent 8-byte loads in flight per thread): staging the tile through LDS pixel-major measured
// slower (0.24 vs 0.18 ms at B = 256) -- the load pass and its barrier serialise ahead of the FFT.
template <bool BF, bool BM>
__global__ __launch_bounds__(FNT, BF ? FFT_MINB_BF : FFT_MINB) void fft_fwd_kernel(const float* __restrict__ src, void* __restrict__ S,
                                                      int H, int W) {
  __shared__ typename Lds<BF>::elem Tbuf[FFT_LDS];
  const Lds<BF> T{Tbuf};
  const int b = fft_block_img(blockIdx.x), cq = fft_block_cq(blockIdx.x);
  const int q = cq >> 1, e0 = 4 * (cq & 1);
  const int tid = threadIdx.x;
  FFT_STAMP_AT(0);
  if (tid < 128) {
    const int y = tid >> 1, p = tid & 1;
    cpx v[72];
    // lane p of the row's lane pair loads all 4 channels of pixel 2k + p (one 16-byte fp32 / 8-byte
    // bf16 load; the pair reads one contiguous run), then the pair swaps the channel pair the other
    // lane transforms (DPP quad_perm [1,0,3,2]): half the load instructions of per-pair loads
    const size_t row = c8_index(b, q, y < H ? y : 0, 0, e0, H, W);
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int x = 2 * k + p;
      const bool in = y < H && x < W;
      cpx lo, hi;   // channels (e0, e0+1) and (e0+2, e0+3) of pixel x
      if constexpr (BM) {
        // unconditional (clamped) loads keep all 32 in flight; out-of-map pixels are zeroed after
        uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(src) + row + 8 * min(x, W - 1));
        if (!in) u = uint2{0u, 0u};
        lo = unpack_bf2(u.x);
        hi = unpack_bf2(u.y);
      } else {
        f32x4 u = *reinterpret_cast<const f32x4*>(src + row + 8 * min(x, W - 1));
        if (!in) u = f32x4{0.f, 0.f, 0.f, 0.f};
        lo = {u[0], u[1]};
        hi = {u[2], u[3]};
      }
      const cpx mine = p ? hi : lo, send = p ? lo : hi;
      const cpx recv = {__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send.x), 0xB1, 0xF, 0xF, false)),
                        __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send.y), 0xB1, 0xF, 0xF, false))};
      v[2 * k] = p ? recv : mine;
      v[2 * k + 1] = p ? mine : recv;
    }
#pragma unroll
    for (int x = 64; x < 72; ++x) v[x] = {0.f, 0.f};
    fwd_rows_to_T(v, y, p, T);
  }
  lds_barrier();
  FFT_STAMP_AT(1);
  fwd_cols_to_S<BF>(T, S, b, cq, tid);
  FFT_STAMP_AT(5);
}

// fp32 forward FFT at three blocks per CU (fft_fwd3_kernel): the transpose runs through a tile of TWO
// channels (37 fx x 2 x 65 rows, 38.5 KB) in two rounds -- channel pair 0 (the p = 0 row threads'
// outputs), then pair 1 -- so the block's LDS is the S staging buffer (43.8 KB) instead of the
// 77 KB four-channel tile.  Every thread reads at most one column: round A's 74 readers are wave 2
// and the even row threads 0..18 (their own row already written), round B's the odd row threads
// and the even ones 20..38; all 148 then run the column FFT together.  Values and rounding are
// those of fft_fwd_kernel (bit-identical S).
constexpr int F3_TLD = 65;
constexpr int F3_LDS = FX * STG_LD;      // dwords: the staging buffer (>= the 2-channel tile)
static_assert(FX * 2 * F3_TLD * 2 <= F3_LDS, "the 2-channel tile fits in the staging buffer");
__device__ __forceinline__ int f3_reader(int tid, int& fx, int& c) {   // round (0 A, 1 B, -1 none)
  int j = -1, r = -1;
  if (tid >= 128) { j = tid - 128; r = 0; }
  else if (tid & 1) { j = tid >> 1; r = 1; }
  else if (tid < 20) { j = 64 + (tid >> 1); r = 0; }
  else if (tid < 40) { j = 64 + ((tid - 20) >> 1); r = 1; }
  if (r < 0) return -1;
  fx = j >> 1;
  c = 2 * r + (j & 1);
  return r;
}
// The forward half of the three-blocks-per-CU kernels, from the row FFT input on: the row threads
// (tid < 128: y = tid >> 1, pair p = tid & 1) hold the packed row v (channels 2p, 2p+1 of row y,
// zero padded); the forward row FFT, the two-round 2-channel transpose, the column FFT and the
// LDS-staged S stores.  Called by every thread of the block (it contains barriers); lds3's space must
// be free on entry (the caller's barrier).
__device__ __forceinline__ void fwd3_tail(cpx (&v)[72], uint32_t* lds3, void* __restrict__ S, int b, int cq, int tid) {
  cpx* T2 = reinterpret_cast<cpx*>(lds3);
  int rfx = 0, rc = 0;
  const int round = f3_reader(tid, rfx, rc);
  const int y = tid >> 1, p = tid & 1;
  if (tid < 128) fft72<-1>(v);
  // rounds: the row threads of pair `pr` write the half spectra of their two channels into T2
  auto write_pair = [&](int pr) {
    if (tid < 128 && p == pr) {
#pragma unroll
      for (int k = 0; k < FX; ++k) {
        const cpx zk = v[k], zm = v[(72 - k) % 72];
        const cpx A = cfma(zm, cpx{1.f, -1.f}, zk) * 0.5f;
        const cpx B = cfma(swp(zk), cpx{1.f, -1.f}, swp(zm)) * 0.5f;
        T2[(k * 2 + 0) * F3_TLD + y] = A;
        T2[(k * 2 + 1) * F3_TLD + y] = B;
      }
    }
  };
  auto read_col = [&](int r) {
    if (round == r) {
#pragma unroll
      for (int yy = 0; yy < 72; ++yy) v[yy] = yy < 64 ? T2[(rfx * 2 + (rc & 1)) * F3_TLD + yy] : cpx{0.f, 0.f};
    }
  };
  write_pair(0);
  lds_barrier();
  read_col(0);
  lds_barrier();
  write_pair(1);
  lds_barrier();
  read_col(1);
  if (round >= 0) fft72<-1>(v);
  uint4* dst = reinterpret_cast<uint4*>(S) + ((size_t)b * 16 + cq) * NF * 2;
  constexpr int NR = 2, NY = 72 / NR, LD = STG_LD, NW = 2 * NY;   // S staged in two fy halves
#pragma unroll
  for (int half = 0; half < NR; ++half) {
    lds_barrier();   // T2 (round 0) / the previous round's staging is no longer read
    if (round >= 0) {
#pragma unroll
      for (int j = 0; j < NY; ++j) {
        const cpx z = v[NY * half + j];
        const float re = z.x * SPEC_SCALE, im = z.y * SPEC_SCALE;
        const _Float16 hr = (_Float16)re, hi = (_Float16)im;
        const f16x2 hv = {hr, hi}, lv = {(_Float16)(re - (float)hr), (_Float16)(im - (float)hi)};
        lds3[rfx * LD + j * 8 + rc] = __builtin_bit_cast(uint32_t, hv);
        lds3[rfx * LD + j * 8 + 4 + rc] = __builtin_bit_cast(uint32_t, lv);
      }
    }
    lds_barrier();
    for (int i = tid; i < FX * NW; i += FNT) {
      const int ffx = i / NW, w = i - ffx * NW;
      st16(dst + (ffx * 72 + NY * half) * 2 + w, *reinterpret_cast<const uint4*>(lds3 + ffx * LD + w * 4));
    }
  }
}
__global__ __launch_bounds__(FNT, 3) void fft_fwd3_kernel(const float* __restrict__ src, void* __restrict__ S,
                                                            int H, int W) {
  __shared__ uint32_t lds3[F3_LDS];
  const int b = fft_block_img(blockIdx.x), cq = fft_block_cq(blockIdx.x);
  const int q = cq >> 1, e0 = 4 * (cq & 1);
  const int tid = threadIdx.x;
  cpx v[72];
  const int y = tid >> 1, p = tid & 1;
  if (tid < 128) {
#ifdef FFT_PROBE_OGC4   // timing probe (tools/bench_fft.hip): the map read as a C4 group (16-B pixels)
    const size_t row = ((size_t)(b * 16 + cq) * H + (y < H ? y : 0)) * W * 4;
    constexpr int PXS = 4;
#else
    const size_t row = c8_index(b, q, y < H ? y : 0, 0, e0, H, W);
    constexpr int PXS = 8;
#endif
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int x = 2 * k + p;
      const bool in = y < H && x < W;
      f32x4 u = *reinterpret_cast<const f32x4*>(src + row + PXS * min(x, W - 1));
      if (!in) u = f32x4{0.f, 0.f, 0.f, 0.f};
      const cpx lo = {u[0], u[1]}, hi = {u[2], u[3]};
      const cpx mine = p ? hi : lo, send = p ? lo : hi;
      const cpx recv = {__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send.x), 0xB1, 0xF, 0xF, false)),
                        __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send.y), 0xB1, 0xF, 0xF, false))};
      v[2 * k] = p ? recv : mine;
      v[2 * k + 1] = p ? mine : recv;
    }
#pragma unroll
    for (int x = 64; x < 72; ++x) v[x] = {0.f, 0.f};
  }
  fwd3_tail(v, lds3, S, b, cq, tid);
}


// inverse 2-D FFT of Y -> the spatial conv result P (C8)
template <bool BF, bool BM>
__global__ __launch_bounds__(FNT, BF ? FFT_MINB_BF : FFT_MINB) void fft_inv_kernel(const void* __restrict__ Y, float* __restrict__ P,
                                                      int H, int W) {
  __shared__ typename Lds<BF>::elem Tbuf[FFT_LDS];
  const Lds<BF> T{Tbuf};
  const int b = fft_block_img(blockIdx.x), cq = fft_block_cq(blockIdx.x);
  const int q = cq >> 1, e0 = 4 * (cq & 1);
  const int tid = threadIdx.x;
  FFT_STAMP_AT(0);
  inv_cols_to_T<BF>(Y, b, cq, tid, T);
  lds_barrier();
  FFT_STAMP_AT(1);
  const int y = tid >> 1, p = tid & 1;
  const bool live = tid < 128 && y < H;
  {
    cpx v[72];
    if (live) inv_row_from_T(T, y, p, v);
    lds_barrier();   // every inverse row has read T
    if (live) {
#pragma unroll
      for (int x = 0; x < 64; ++x) T.set(tid * RLD + x, v[x]);
    }
  }
  lds_barrier();
  FFT_STAMP_AT(2);
#pragma unroll 4
  for (int i = tid; i < H * W; i += FNT) {
    const int yy = i / W, x = i - yy * W;
    const cpx a = T.get((2 * yy) * RLD + x), c = T.get((2 * yy + 1) * RLD + x);
#ifdef FFT_PROBE_PCOAL   // timing probe (tools/bench_fft.hip): the block's P quarter written contiguously
    map_st4_stream<BM>(P, ((size_t)b * 16 + cq) * 4096 * 4 + 4 * i, f32x4{a.x, a.y, c.x, c.y});
#else
    map_st4_stream<BM>(P, pp_index(b, q, yy, x, e0, H, W), f32x4{a.x, a.y, c.x, c.y});
#endif
  }
  FFT_STAMP_AT(5);
}

// The A half-step's tail and the B half-step's head in one pass (hgru_module.py:657, 797-799):
//   P1 = IFFT(Y)  ->  I = tanh(X - (beta*O + nu) * (P1 + lateral_bias))  ->  S = FFT(I)
// P1 never leaves the block: the inverse rows are parked in LDS, the epilogue runs pixel-major
// over them (X, O in, I out: one float4 per lane), and the parked I rows are the forward row
// transform's input.  p: the A-epilogue arguments (X, O, vecs; dst = I).
template <bool BF, bool BM>
__global__ __launch_bounds__(FNT, BF ? FFT_MINB_BF : FFT_MINB) void fft_inv_a_fwd_kernel(const void* __restrict__ Y, ConvArgs p,
                                                            void* __restrict__ S) {
  __shared__ typename Lds<BF>::elem Tbuf[FFT_LDS];
  const Lds<BF> T{Tbuf};
  const int H = p.H, W = p.W;
  const int b = fft_block_img(blockIdx.x), cq = fft_block_cq(blockIdx.x);
  const int q = cq >> 1, e0 = 4 * (cq & 1);
  const int tid = threadIdx.x;
  FFT_STAMP_AT(0);
  // the A epilogue's X / O loads (see below); FFT_EPI_EARLY issues chunk 0's before the inverse row
  // phase, so they are in flight during the row transforms
  constexpr int EU = BM ? 8 : FFT_EPI_EU, ECH = EU * FNT, NECH = (64 * 64 + ECH - 1) / ECH;
  constexpr bool PIPE = FFT_EPI_PIPE && (BM || FFT_EPI_EARLY);
  f32x4 xv[2][EU], ov[2][EU];
  auto load_chunk = [&](int k, f32x4 (&xs)[EU], f32x4 (&os)[EU]) {
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      const int i = min(k * ECH + u * FNT + tid, 64 * 64 - 1);
      const int yy = min(i >> 6, H - 1), x = min(i & 63, W - 1);
#ifdef FFT_PROBE_XOC4   // timing probe (tools/bench_fft.hip): X / O read as C4 groups
      const size_t idx = c4_index(b, q, yy, x, e0, H, W);
#else
      const size_t idx = c8_index(b, q, yy, x, e0, H, W);
#endif
      xs[u] = map_ld4<BM>(p.X, (FFT_C4 & 8) ? xx_index(b, q, yy, x, e0, H, W) : idx);
      os[u] = map_ld4<BM>(p.O, (FFT_C4 & 4) ? oo_index(b, q, yy, x, e0, H, W) : idx);
    }
  };
  inv_cols_to_T<BF>(Y, b, cq, tid, T);
  lds_barrier();
  FFT_STAMP_AT(1);
  // (fp32 maps only: the bf16 kernels are held to 168 VGPRs for 3 blocks per CU, and the early set
  // made their inv_a_fwd 0.178 -> 0.216 ms, profiles/r3g)
  constexpr bool EARLY = FFT_EPI_EARLY && !BM;
  if constexpr (PIPE && EARLY) load_chunk(0, xv[0], ov[0]);
  const int y = tid >> 1, pp = tid & 1;
  const bool live = tid < 128 && y < H;
  {
    cpx v[72];
    if (live) inv_row_from_T(T, y, pp, v);
    lds_barrier();   // every inverse row has read T
    if (live) {
#pragma unroll
      for (int x = 0; x < 64; ++x) T.set(tid * RLD + x, v[x]);
    }
  }
  lds_barrier();
  FFT_STAMP_AT(2);
  {
    const int ch = 8 * q + e0;
    const f32x4 lat = *reinterpret_cast<const f32x4*>(p.vecs + V_LAT * 64 + ch);
    const f32x4 be = *reinterpret_cast<const f32x4*>(p.vecs + V_BETA * 64 + ch);
    const f32x4 nu = *reinterpret_cast<const f32x4*>(p.vecs + V_NU * 64 + ch);
    // 64 x 64 pixels (zero padding included) in chunks of EU per thread: the X / O loads of a
    // chunk are unconditional (clamped addresses) so all 2 EU are in flight together.  With bf16
    // maps (PIPE) the next chunk's loads are issued before this chunk's math: the phase is ~45k of
    // the block's ~100k cycles (tools/fft_stamps.hip); with fp32 maps the second register set
    // measured 2-4 % slower (inv_a_fwd 0.338 -> 0.351 ms), so there it stays one chunk at a time
    if constexpr (PIPE && !EARLY) load_chunk(0, xv[0], ov[0]);
#pragma unroll
    for (int k = 0; k < NECH; ++k) {
      const int cur = PIPE ? (k & 1) : 0;
      if constexpr (PIPE) {
        if (k + 1 < NECH) load_chunk(k + 1, xv[cur ^ 1], ov[cur ^ 1]);
      } else {
        load_chunk(k, xv[0], ov[0]);
      }
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int i = k * ECH + u * FNT + tid;
        if (i >= 64 * 64) break;
        const int yy = i >> 6, x = i & 63;
        const int ia = (2 * yy) * RLD + x, ic = (2 * yy + 1) * RLD + x;
        if (yy < H && x < W) {
          const cpx ra = T.get(ia), rc = T.get(ic);
          const f32x4 pv = {ra.x, ra.y, rc.x, rc.y};
          f32x4 iv;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
#ifdef FFT_PROBE_NOTANH   // timing probe: the A epilogue without tanhf
            iv[j] = xv[cur][u][j] - (be[j] * ov[cur][u][j] + nu[j]) * (pv[j] + lat[j]);
#else
            iv[j] = atanh_f(epi_a(xv[cur][u][j], ov[cur][u][j], pv[j], be[j], nu[j], lat[j]));
#endif
          }
#ifdef FFT_PROBE_ICOAL   // timing probe (tools/bench_fft.hip): the block's I quarter written contiguously
          map_st4_stream<BM>(p.dst, ((size_t)b * 16 + cq) * 4096 * 4 + 4 * i, iv);
#else
          map_st4_stream<BM>(p.dst, ii_index(b, q, yy, x, e0, H, W), iv);
#endif
          T.set(ia, {iv[0], iv[1]});
          T.set(ic, {iv[2], iv[3]});
        } else {
          T.set(ia, {0.f, 0.f});
          T.set(ic, {0.f, 0.f});
        }
      }
    }
  }
  lds_barrier();
  FFT_STAMP_AT(3);
  cpx v[72];
  if (tid < 128) {
#pragma unroll
    for (int x = 0; x < 72; ++x) v[x] = x < 64 ? T.get(tid * RLD + x) : cpx{0.f, 0.f};
  }
  lds_barrier();   // parked rows read: T's space is free
  if (tid < 128) fwd_rows_to_T(v, y, pp, T);
  lds_barrier();
  FFT_STAMP_AT(4);
  fwd_cols_to_S<BF>(T, S, b, cq, tid);
  FFT_STAMP_AT(5);
}

// pitch (complex) of a row y of a 2-channel inverse tile (odd: conflict-free row reads)
constexpr int I3_LD = 2 * FX + 1;

// ---------------------------------------------------------------------------------------------
// Small-batch (latency) forms of the three fp32 FFT kernels (FFT path, fp32 maps; B <= lfft_maxb()).
// At batch 1 the batched kernels run 16 blocks, each a chain of per-thread 72-point transforms
// (~7.4k cycles per row / column phase) and a 21-pixel-per-thread epilogue, so inv_a_fwd takes ~49k
// cycles (tools/fft_stamps.hip, profiles/r3u).  Here every 72-point transform is spread over 9 lanes
// exactly along fft72's prime-factor passes: lane n2 runs the 8-point DFT of inputs (9 n1 + 8 n2) % 72,
// the 8 x 9 intermediates cross through LDS, lane k1 runs the 9-point DFT and holds outputs
// (9 k1 + 64 k2) % 72.  A block is one (image, channel PAIR): 74 column / 64 row transforms x 9 lanes
// (704 threads), 32 blocks per image.  Every value is produced by the same dft8 / dft9 / pair-separation
// / epilogue operations on the same operands as in the batched kernels, so the results are
// bit-identical to them (tests/test_gpu_parity.py::test_batch_invariance_and_determinism runs a crop
// alone and inside a batch).
constexpr int LF_NT = 704;             // 11 waves of 7 transforms x 9 lanes: 74 column / 64 row transforms
constexpr int LF_T = 74;
constexpr int LF_ZLD = 73;             // pitch (complex) of a row of the P / I rows and the forward row outputs
constexpr int LF_BIG = NF * 2;         // complex: the pair's whole spectrum (Y in, or S staging out), 42.6 KB
static_assert(LF_BIG >= 64 * I3_LD && LF_BIG >= 64 * LF_ZLD && LF_BIG >= LF_T * 72, "LDS plan");
// block -> (image, channel pair): the four pairs of one C8 chunk (8 channels, 32 B per pixel) on one XCD
__device__ __forceinline__ void lfft_block(int blk, int& b, int& cp) {
  b = blk >> 5;
  const int r = blk & 31;
  cp = 4 * (r & 7) + (r >> 3);
}
// stage 1 of a 9-lane transform: lane j (< 9) = n2: in[n1] = x[(9 n1 + 8 n2) % 72] -> dft8 -> E
template <int SG>
__device__ __forceinline__ void lf_stage1(cpx (&in)[8], cpx* E, int t, int j) {
  dft8<SG>(in);
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) E[t * 72 + j * 8 + k1] = in[k1];
}
// stage 2: lane j (< 8) = k1: u[n2] = E[n2][k1] -> dft9 -> u[k2] = X[(9 k1 + 64 k2) % 72]
template <int SG>
__device__ __forceinline__ void lf_stage2(cpx (&u)[9], const cpx* E, int t, int j) {
#pragma unroll
  for (int n2 = 0; n2 < 9; ++n2) u[n2] = E[t * 72 + n2 * 8 + j];
  dft9<SG>(u);
}
__device__ __forceinline__ int lf_in(int n1, int j) { return (9 * n1 + 8 * j) % 72; }
__device__ __forceinline__ int lf_out(int j, int k2) { return (9 * j + 64 * k2) % 72; }
// the same index sets as lane tables built incrementally ((9 n1 + 8 j) steps by +9, (9 j + 64 k2) by
// -8, mod 72): a conditional add instead of a division per element
struct LfIdx {
  int in[8], out[9];
  __device__ __forceinline__ explicit LfIdx(int j) {
    int a = 8 * j;   // j <= 8: a < 72
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) {
      in[n1] = a;
      a += 9;
      a -= a >= 72 ? 72 : 0;
    }
    int b = 9 * j;
    b -= b >= 72 ? 72 : 0;
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) {
      out[k2] = b;
      b -= 8;
      b += b < 0 ? 72 : 0;
    }
  }
};
// thread -> (transform t, lane j): 7 transforms of 9 lanes per wave (lane 63 idle), so a transform's
// exchange between its two passes stays inside one wave and needs no workgroup barrier
__device__ __forceinline__ void lf_lane(int tid, int& t, int& j) {
  const int ln = tid & 63, tw = ln / 9;
  t = ln == 63 ? 1 << 20 : 7 * (tid >> 6) + tw;
  j = ln - 9 * tw;
}
// the wave's own LDS writes of pass 1 have landed (DS instructions of a wave complete in order)
__device__ __forceinline__ void lf_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Y's channel pair (2 cp, 2 cp + 1) -> the P rows in R[y][x] (y, x < 64).  The spectrum is first
// copied into LDS with one 16-byte load per frequency (both channels; the wave reads 64 consecutive
// 32-byte groups), since the transforms' own access order scatters over the whole 85 KB run.
// Big: LF_BIG complex of LDS (the Y copy, then the inverse tile).  Called by every thread.
__device__ __forceinline__ void lf_inverse(const void* __restrict__ Y, int b, int cp, int tid, cpx* E, cpx* Big,
                                           cpx* R) {
  const int cq = cp >> 1, pp = cp & 1;
  int t, j;
  lf_lane(tid, t, j);
  const LfIdx ix(min(j, 8));
  const float4* ysrc = reinterpret_cast<const float4*>(Y) + ((size_t)b * 16 + cq) * NF * 2 + pp;
  for (int f = tid; f < NF; f += LF_NT) {   // the Y copy goes to R's space (free until the P rows)
    const float4 v = ysrc[2 * f];
    R[2 * f] = cpx{v.x, v.y};
    R[2 * f + 1] = cpx{v.z, v.w};
  }
  lds_barrier();
  FFT_STAMP_AT(1);
  cpx in[8], u[9];
  // inverse column (fx, cc) = (t >> 1, t & 1) over fy (inv_cols_to_T)
  if (t < LF_T && j < 9) {
    const int fx = t >> 1, cc = t & 1;
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) in[n1] = R[2 * spec_f<false>(fx, ix.in[n1]) + cc];
    lf_stage1<1>(in, E, t, j);
  }
  lf_wave_sync();
  if (t < LF_T && j < 8) {
    const int fx = t >> 1, cc = t & 1;
    lf_stage2<1>(u, E, t, j);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) {
      const int y = ix.out[k2];
      if (y < 64) Big[y * I3_LD + cc * FX + fx] = u[k2];
    }
  }
  lds_barrier();
  FFT_STAMP_AT(2);
  // inverse row y = t: C[m] = A[m] + i B[m] from the Hermitian half spectra (inv_row_from_T)
  if (t < 64 && j < 9) {
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) {
      const int m = ix.in[n1], k = m <= 36 ? m : 72 - m;
      const cpx A = Big[t * I3_LD + k], B = Big[t * I3_LD + FX + k];
      in[n1] = m <= 36 ? cfma(swp(B), cpx{-1.f, 1.f}, A) : cfma(A, cpx{1.f, -1.f}, swp(B));
    }
    lf_stage1<1>(in, E, t, j);
  }
  lf_wave_sync();
  if (t < 64 && j < 8) {
    lf_stage2<1>(u, E, t, j);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) {
      const int x = ix.out[k2];
      if (x < 64) R[t * LF_ZLD + x] = u[k2];
    }
  }
  lds_barrier();
  FFT_STAMP_AT(3);
}

// the rows R[y][x] (x < 64; zero outside the map) -> S for the channel pair: forward rows, forward
// columns, and the pair's S entries (hi / lo, 8 B each per frequency) staged in LDS and stored in
// frequency order.  R must be complete on entry; Big's space is free (reused for the row outputs,
// then the staging).  Called by every thread.
__device__ __forceinline__ void lf_forward(const cpx* R, int b, int cp, int tid, cpx* E, cpx* Big,
                                           void* __restrict__ S) {
  const int cq = cp >> 1, pp = cp & 1;
  int t, j;
  lf_lane(tid, t, j);
  const LfIdx ix(min(j, 8));
  cpx in[8], u[9];
  if (t < 64 && j < 9) {
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) {
      const int x = ix.in[n1];
      in[n1] = x < 64 ? R[t * LF_ZLD + x] : cpx{0.f, 0.f};
    }
    lf_stage1<-1>(in, E, t, j);
  }
  lf_wave_sync();   // (R, read by pass 1, is not written here)
  if (t < 64 && j < 8) {
    lf_stage2<-1>(u, E, t, j);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) Big[t * LF_ZLD + ix.out[k2]] = u[k2];
  }
  lds_barrier();
  FFT_STAMP_AT(5);
  // forward column (fx, cc): the pair-separated half spectra of rows y (fwd_rows_to_T), then over y
  if (t < LF_T && j < 9) {
    const int fx = t >> 1, cc = t & 1;
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) {
      const int y = ix.in[n1];
      cpx v = {0.f, 0.f};
      if (y < 64) {
        const cpx zk = Big[y * LF_ZLD + fx], zm = Big[y * LF_ZLD + (72 - fx) % 72];
        v = cc == 0 ? cfma(zm, cpx{1.f, -1.f}, zk) * 0.5f : cfma(swp(zk), cpx{1.f, -1.f}, swp(zm)) * 0.5f;
      }
      in[n1] = v;
    }
    lf_stage1<-1>(in, E, t, j);
  }
  lf_wave_sync();
  // the S staging [f][hi cc0, hi cc1, lo cc0, lo cc1] in R's space (its rows were read before the
  // last barrier)
  uint32_t* stg = reinterpret_cast<uint32_t*>(const_cast<cpx*>(R));
  if (t < LF_T && j < 8) {
    const int fx = t >> 1, cc = t & 1;
    lf_stage2<-1>(u, E, t, j);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) {
      const cpx z = u[k2];
      const float re = z.x * SPEC_SCALE, im = z.y * SPEC_SCALE;
      const _Float16 hr = (_Float16)re, hi = (_Float16)im;
      const f16x2 hv = {hr, hi}, lv = {(_Float16)(re - (float)hr), (_Float16)(im - (float)hi)};
      const int f = spec_f<false>(fx, ix.out[k2]);
      stg[4 * f + cc] = __builtin_bit_cast(uint32_t, hv);
      stg[4 * f + 2 + cc] = __builtin_bit_cast(uint32_t, lv);
    }
  }
  lds_barrier();
  FFT_STAMP_AT(6);
  // S group (b, cq, f): [hi c0..c3 | lo c0..c3], 4 B each; this pair's hi at 8 pp, lo at 16 + 8 pp
  uint2* dst = reinterpret_cast<uint2*>(S) + ((size_t)b * 16 + cq) * NF * 4 + pp;
  for (int f = tid; f < NF; f += LF_NT) {
    const uint4 w = *reinterpret_cast<const uint4*>(stg + 4 * f);
    dst[4 * f] = uint2{w.x, w.y};
    dst[4 * f + 2] = uint2{w.z, w.w};
  }
  FFT_STAMP_AT(7);
}

// pixels of the pixel-major passes: thread tid takes pixels tid + LF_NT i (i < LF_PX)
constexpr int LF_PX = (64 * 64 + LF_NT - 1) / LF_NT;   // 6

__global__ __launch_bounds__(LF_NT, 1) void lfft_inv_a_fwd_kernel(const void* __restrict__ Y, ConvArgs pa,
                                                                 void* __restrict__ S) {
  __shared__ cpx E[LF_T * 72];
  __shared__ cpx Big[LF_BIG];
  __shared__ cpx R[LF_BIG];   // the Y copy, the P rows, the I rows, the S staging
  const int H = pa.H, W = pa.W;
  int b, cp;
  lfft_block(blockIdx.x, b, cp);
  const int q = cp >> 2, ec = 2 * (cp & 3);   // C8 chunk and the pair's first channel in it
  const int tid = threadIdx.x;
  FFT_STAMP_AT(0);
  // the A epilogue's X / O of this thread's pixels, issued first (clamped addresses)
  cpx xv[LF_PX], ov[LF_PX];
#pragma unroll
  for (int i = 0; i < LF_PX; ++i) {
    const int px = min(tid + LF_NT * i, 64 * 64 - 1), y = min(px >> 6, H - 1), x = min(px & 63, W - 1);
    xv[i] = map_ld2<false>(pa.X, xx_index(b, q, y, x, ec, H, W));
    ov[i] = map_ld2<false>(pa.O, oo_index(b, q, y, x, ec, H, W));
  }
  lf_inverse(Y, b, cp, tid, E, Big, R);
  // the A epilogue (hgru_module.py:797-799), pixel-major over the P rows; I back into R
  const int ch = 8 * q + ec;
  const cpx lat = {pa.vecs[V_LAT * 64 + ch], pa.vecs[V_LAT * 64 + ch + 1]};
  const cpx be = {pa.vecs[V_BETA * 64 + ch], pa.vecs[V_BETA * 64 + ch + 1]};
  const cpx nu = {pa.vecs[V_NU * 64 + ch], pa.vecs[V_NU * 64 + ch + 1]};
#pragma unroll
  for (int i = 0; i < LF_PX; ++i) {
    const int px = tid + LF_NT * i;
    if (px >= 64 * 64) break;
    const int y = px >> 6, x = px & 63;
    cpx iv = {0.f, 0.f};
    if (y < H && x < W) {
      const cpx pv = R[y * LF_ZLD + x];
      iv = {atanh_f(epi_a(xv[i].x, ov[i].x, pv.x, be.x, nu.x, lat.x)),
            atanh_f(epi_a(xv[i].y, ov[i].y, pv.y, be.y, nu.y, lat.y))};
      *reinterpret_cast<float2*>(pa.dst + ii_index(b, q, y, x, ec, H, W)) = float2{iv.x, iv.y};
    }
    R[y * LF_ZLD + x] = iv;
  }
  lds_barrier();
  FFT_STAMP_AT(4);
  lf_forward(R, b, cp, tid, E, Big, S);
}

__global__ __launch_bounds__(LF_NT, 1) void lfft_inv_kernel(const void* __restrict__ Y, float* __restrict__ P, int H,
                                                           int W) {
  __shared__ cpx E[LF_T * 72];
  __shared__ cpx Big[LF_BIG];
  __shared__ cpx R[LF_BIG];
  int b, cp;
  lfft_block(blockIdx.x, b, cp);
  const int q = cp >> 2, ec = 2 * (cp & 3);
  const int tid = threadIdx.x;
  lf_inverse(Y, b, cp, tid, E, Big, R);
  for (int px = tid; px < 64 * 64; px += LF_NT) {
    const int y = px >> 6, x = px & 63;
    if (y < H && x < W) {
      const cpx v = R[y * LF_ZLD + x];
      *reinterpret_cast<float2*>(P + pp_index(b, q, y, x, ec, H, W)) = float2{v.x, v.y};
    }
  }
}

__global__ __launch_bounds__(LF_NT, 1) void lfft_fwd_kernel(const float* __restrict__ src, void* __restrict__ S, int H,
                                                           int W) {
  __shared__ cpx E[LF_T * 72];
  __shared__ cpx Big[LF_BIG];
  __shared__ cpx R[LF_BIG];
  int b, cp;
  lfft_block(blockIdx.x, b, cp);
  const int q = cp >> 2, ec = 2 * (cp & 3);
  const int tid = threadIdx.x;
  for (int px = tid; px < 64 * 64; px += LF_NT) {   // the pair's map rows, zero outside the map
    const int y = px >> 6, x = px & 63;
    R[y * LF_ZLD + x] = (y < H && x < W) ? map_ld2<false>(src, c8_index(b, q, y, x, ec, H, W)) : cpx{0.f, 0.f};
  }
  lds_barrier();
  lf_forward(R, b, cp, tid, E, Big, S);
}

#ifndef LFFT_MAXB
#define LFFT_MAXB 8   // largest batch for the latency kernels (profiles/r3y: B = 8 1.166 -> 1.126 ms, B = 16 1.354 -> 1.645); MP_LFFT_MAXB overrides, 0 = off
#endif
static int lfft_maxb() {
  static const int v = [] {
    const char* e = std::getenv("MP_LFFT_MAXB");
    return e ? std::atoi(e) : LFFT_MAXB;
  }();
  return v;
}

// ---------------------------------------------------------------------------------------------
// spectral GEMM: per frequency f, Y[b][co] = sum_ci S[b][ci] G[ci][co] (complex), as one real
// 128 x 32 x 128 product per (f, 32 images), D[n][j] = sum_k A[n][k] Bm[k][j] on
// v_mfma_f32_32x32x16_f16 in the f16x3 split, with n = 64 ro + co (ro = re|im of the output) and
// k = 2 ci + ri (ri = re|im of the input):
//   B fragment (lane h, image j; k-step t): k = 16t + 8h + e = the 8 hi (lo) halves of S group
//     cq = 2t + h of image j;
//   A fragment (lane h, row i of M-block mb, ro = mb >> 1): re/im pairs of G[ci = 8t+4h..+3][co],
//     negated imaginary halves for ro = 0 (gr, -gi), swapped halves for ro = 1 (gi, gr), derived in
//     registers from the compact split weights Gc[f][part][cq][co] (f16x8 = 4 complex), 32 KiB per f.
// Block = 4 consecutive frequencies (one 128-B line of S / Y per (image, channel group)) x 32
// images, 4 waves (one frequency each).  The S tile is loaded whole-line (8 lines per
// wave-instruction) into LDS [cq][part][f][b], the Y tile leaves the same way through LDS
// [b][cq][f]; the weights stream from L2.  Blocks of one frequency quad are placed on one XCD so its
// weights are fetched from HBM once.
constexpr int SG_NI = 32;              // images per block
#ifndef SPEC_SMALLB
#define SPEC_SMALLB 8   // batches up to this run spec_gemm_kernel<0, 8> (8-image tiles); 0 = off
#endif
#ifndef SPEC_SMALL_HALF
#define SPEC_SMALL_HALF 1   // 8-image kernel: the weights in two halves of 4 k-steps (64 VGPRs instead of 128):
                            // 3 blocks per CU, B = 1 forward 0.925 -> 0.890-0.897 ms (profiles/r4s)
#endif
#ifndef SPEC_SMALL_MINB
// blocks per CU of the 8-image kernel.  Whole-weight registers at 3 spilled (168 B / lane of
// scratch, 0.029 vs 0.019 ms at B = 1, profiles/r3z); with SPEC_SMALL_HALF 3 fit, so the 666 blocks
// run as one round of 768 slots instead of 1.3 rounds of 512
#define SPEC_SMALL_MINB (SPEC_SMALL_HALF ? 3 : 2)
#endif
constexpr int NQUAD = NF / 4;          // 666 frequency quads
constexpr int NQ8 = (NQUAD + 7) / 8;
constexpr int SG_SLD = 33;             // S tile pitch (16-B units) per (cq, part, f) row
constexpr int SG_YLD = 16 * 4 * 2 + 1; // Y tile pitch (16-B units) per image
// NI: images per block -- 32, or 8 for batches <= SPEC_SMALLB (a quarter of the S tile's loads and
// LDS; the MFMA columns of images past NI are zero, the per-output product order is the same)
template <int PROBE = 0, int NI = SG_NI>   // timing probes (tools/bench_fft.hip): 1 = no MFMA, 2 = no S / weight loads,
                                          // 3 = no weight loads, 4 = no S loads
__global__ __launch_bounds__(256, NI == SG_NI ? 2 : SPEC_SMALL_MINB) void spec_gemm_kernel(const uint4* __restrict__ S, const uint4* __restrict__ Gc,
                                                           uint4* __restrict__ Y, int B, int ngrp, float unscale) {
  constexpr int SLD = NI + 1;               // S tile pitch (16-B units) per (cq, part, f) row
  constexpr int NLD = NI * 16 * 8 / 256;    // 16-B S / Y pieces per thread
  __shared__ uint4 tile[16 * 2 * 4 * SLD];   // 67,584 B (NI = 32)
  static_assert(NI * SG_YLD <= 16 * 2 * 4 * SLD, "the Y tile fits in the S tile's space");
  // block -> (quad, image group): the ngrp groups of quad q run on XCD q % 8 (round-robin dispatch)
  const int q8 = blockIdx.x / (8 * ngrp), rem = blockIdx.x - q8 * 8 * ngrp;
  const int grp = rem >> 3, quad = q8 * 8 + (rem & 7);
  if (quad >= NQUAD) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, j = lane & 31;
  const int img0 = grp * NI;
  // ---- S tile: 32 images x 16 cq lines of 128 B (4 f x [hi 16 B | lo 16 B]) ----
  // unconditional loads from clamped addresses: a per-lane "b < B ? load : 0" branch made the
  // compiler wait for each of the 16 loads before issuing the next
  uint4 pre[NLD];
#pragma unroll
  for (int it = 0; it < NLD; ++it) {
    const int idx = it * 256 + tid, line = idx >> 3, piece = idx & 7;
    const int bl = line >> 4, cq = line & 15;
    const int b = min(img0 + bl, B - 1);
    pre[it] = S[(PROBE == 2 || PROBE == 4) ? (tid & 63) : (((size_t)b * 16 + cq) * NF + 4 * quad) * 2 + piece];
  }
  // ---- weights of frequency f = 4 quad + wv: one f16x8 per (t, h, part, co block), all 32 issued
  // before the S tile is waited for, so their L2 latency overlaps the tile's HBM latency (the
  // 8-image kernel under SPEC_SMALL_HALF: 16 per half, the second half issued after the first
  // half's MFMAs; the per-output k-step order is unchanged) ----
  constexpr int TW = (NI != SG_NI && SPEC_SMALL_HALF) ? 4 : 8;   // k-steps per weight batch
  const int f = 4 * quad + wv;
  const uint4* gw = Gc + ((PROBE == 2 || PROBE == 3) ? 0 : (size_t)f * 2 * 16 * 64);
  uint4 wr[TW][2][2];
  auto load_w = [&](int t0) {
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        wr[t][cb][0] = gw[(0 * 16 + 2 * (t0 + t) + h) * 64 + 32 * cb + j];
        wr[t][cb][1] = gw[(1 * 16 + 2 * (t0 + t) + h) * 64 + 32 * cb + j];
      }
  };
  load_w(0);
#pragma unroll
  for (int it = 0; it < NLD; ++it) {
    const int idx = it * 256 + tid, line = idx >> 3, piece = idx & 7;
    const int bl = line >> 4, cq = line & 15, f = piece >> 1, part = piece & 1;
    tile[((cq * 2 + part) * 4 + f) * SLD + bl] = img0 + bl < B ? pre[it] : uint4{0, 0, 0, 0};
  }
  lds_barrier();
  f32x16 acc[4] = {};
  const uint4 m = {0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u};
#pragma unroll
  for (int t0 = 0; t0 < 8; t0 += TW) {
    if (t0 > 0) load_w(t0);
#pragma unroll
    for (int tt = 0; tt < TW; ++tt) {
      const int t = t0 + tt;
      const int cq = 2 * t + h;
      const int jj = NI == SG_NI ? j : min(j, NI - 1);   // columns past NI: zero operands (below)
      f16x8 sh = __builtin_bit_cast(f16x8, tile[((cq * 2 + 0) * 4 + wv) * SLD + jj]);
      f16x8 sl = __builtin_bit_cast(f16x8, tile[((cq * 2 + 1) * 4 + wv) * SLD + jj]);
      if (NI != SG_NI && j >= NI) sh = sl = f16x8{};
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const uint4 gh = wr[tt][cb][0], gl = wr[tt][cb][1];
        // ro = 0 rows: (gr, -gi) pairs; ro = 1 rows: (gi, gr) pairs
        const f16x8 ah0 = __builtin_bit_cast(f16x8, gh ^ m), al0 = __builtin_bit_cast(f16x8, gl ^ m);
        const f16x8 ah1 = __builtin_bit_cast(f16x8, (gh >> 16) | (gh << 16));
        const f16x8 al1 = __builtin_bit_cast(f16x8, (gl >> 16) | (gl << 16));
        if constexpr (PROBE == 1) {   // keep the operand loads alive, skip the matrix cores
          acc[cb][0] += (float)(sh[0] + sl[0] + ah0[0] + al0[0] + ah1[1] + al1[1]);
        } else {
          acc[cb] = mfma16(al0, sh, acc[cb]);
          acc[cb] = mfma16(ah0, sl, acc[cb]);
          acc[cb] = mfma16(ah0, sh, acc[cb]);
          acc[2 + cb] = mfma16(al1, sh, acc[2 + cb]);
          acc[2 + cb] = mfma16(ah1, sl, acc[2 + cb]);
          acc[2 + cb] = mfma16(ah1, sh, acc[2 + cb]);
        }
      }
    }
  }
  lds_barrier();   // every wave has read the S tile
  // ---- Y tile: lane (h, j), co block cb, row group g: channels 32cb + 8g + 4h + e, e < 4 ----
  f32x4* ytile = reinterpret_cast<f32x4*>(tile);
  if (NI == SG_NI || j < NI) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int cqo = 8 * cb + 2 * g + h;
        const f32x16& re = acc[cb];
        const f32x16& im = acc[2 + cb];
        const f32x4 lo = f32x4{re[4 * g], im[4 * g], re[4 * g + 1], im[4 * g + 1]} * unscale;
        const f32x4 hi = f32x4{re[4 * g + 2], im[4 * g + 2], re[4 * g + 3], im[4 * g + 3]} * unscale;
        ytile[j * SG_YLD + (cqo * 4 + wv) * 2] = lo;
        ytile[j * SG_YLD + (cqo * 4 + wv) * 2 + 1] = hi;
      }
  }
  lds_barrier();
#pragma unroll
  for (int it = 0; it < NLD; ++it) {
    const int idx = it * 256 + tid, line = idx >> 3, piece = idx & 7;
    const int bl = line >> 4, cqo = line & 15, b = img0 + bl;
    if (b < B) st16(Y + (((size_t)b * 16 + cqo) * NF + 4 * quad) * 2 + piece, tile[bl * SG_YLD + cqo * 8 + piece]);
  }
}

// bf16 spectral GEMM (MP_DTYPE_BF16): the same blocking, fragments and XCD placement as
// spec_gemm_kernel with 16-byte spectra entries (one bf16 (re, im) pair per channel): a block's S
// tile is 32 images x 16 cq x 64 B, one v_mfma_f32_32x32x16_bf16 per (k-step, co block, re|im row
// half), weights Gb[f][cq][co] (bf16x8 = 4 complex), Y written as bf16 pairs.  A quad's 64-B piece
// is half a 128-B line, so the two quads of a line (2k, 2k+1) run on one XCD, one after the other
// in dispatch order: with quad q on XCD q % 8 (the fp32 kernel's placement) every S / Y line was
// moved by two L2s (PMC: 1.76x the algorithmic reads).
constexpr int NQ16 = (NQUAD + 15) / 16;
constexpr int SGB_YLD = 16 * 4 + 1;    // Y tile pitch (16-B units) per image
__global__ __launch_bounds__(256, 2) void spec_gemm_bf_kernel(const uint4* __restrict__ S, const uint4* __restrict__ Gb,
                                                              uint4* __restrict__ Y, int B, int ngrp) {
  __shared__ uint4 tile[16 * 4 * SG_SLD];   // 33,792 B (S tile [cq][f][b]; Y tile [b][cq][f])
  // block -> (quad, image group): XCD x = rem % 8 takes the quad pair (2x, 2x+1) of each 16
  const int q16 = blockIdx.x / (16 * ngrp), rem = blockIdx.x - q16 * 16 * ngrp;
  const int sq = rem >> 3;
  const int grp = sq >> 1, quad = q16 * 16 + 2 * (rem & 7) + (sq & 1);
  if (quad >= NQUAD) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, j = lane & 31;
  const int img0 = grp * SG_NI;
  uint4 pre[8];
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 256 + tid, line = idx >> 2, piece = idx & 3;
    const int bl = line >> 4, cq = line & 15;
    const int b = min(img0 + bl, B - 1);
    pre[it] = S[((size_t)b * 16 + cq) * NF + 4 * quad + piece];
  }
  const int f = 4 * quad + wv;
  const uint4* gw = Gb + (size_t)f * 16 * 64;
  uint4 wr[8][2];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) wr[t][cb] = gw[(2 * t + h) * 64 + 32 * cb + j];
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 256 + tid, line = idx >> 2, piece = idx & 3;
    const int bl = line >> 4, cq = line & 15;
    tile[(cq * 4 + piece) * SG_SLD + bl] = img0 + bl < B ? pre[it] : uint4{0, 0, 0, 0};
  }
  lds_barrier();
  f32x16 acc[4] = {};
  const uint4 m = {0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u};
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const bf16x8 sb = __builtin_bit_cast(bf16x8, tile[((2 * t + h) * 4 + wv) * SG_SLD + j]);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const uint4 g = wr[t][cb];
      acc[cb] = mfmab(__builtin_bit_cast(bf16x8, g ^ m), sb, acc[cb]);                       // (gr, -gi)
      acc[2 + cb] = mfmab(__builtin_bit_cast(bf16x8, (g >> 16) | (g << 16)), sb, acc[2 + cb]); // (gi, gr)
    }
  }
  lds_barrier();   // every wave has read the S tile
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int cqo = 8 * cb + 2 * g + h;
      const f32x16& re = acc[cb];
      const f32x16& im = acc[2 + cb];
      tile[j * SGB_YLD + cqo * 4 + wv] = uint4{pack_bf2(re[4 * g], im[4 * g]), pack_bf2(re[4 * g + 1], im[4 * g + 1]),
                                             pack_bf2(re[4 * g + 2], im[4 * g + 2]),
                                             pack_bf2(re[4 * g + 3], im[4 * g + 3])};
    }
  lds_barrier();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 256 + tid, line = idx >> 2, piece = idx & 3;
    const int bl = line >> 4, cqo = line & 15, b = img0 + bl;
    if (b < B) st16(Y + ((size_t)b * 16 + cqo) * NF + 4 * quad + piece, tile[bl * SGB_YLD + cqo * 4 + piece]);
  }
}

// spectral weights, once per weight set: G[f][ci][co] (complex, 1/N^2 folded in), one thread per
// (f, ci, co), float64 accumulation
__global__ void spec_weights_kernel(const float* __restrict__ w, cpx* __restrict__ G, int KS, int fym) {
  __shared__ double tc[FFT_N], ts[FFT_N];
  for (int m = threadIdx.x; m < FFT_N; m += blockDim.x) {
    double s, c;
    sincospi(2.0 * m / FFT_N, &s, &c);
    tc[m] = c;
    ts[m] = s;
  }
  lds_barrier();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NF * 4096) return;
  const int co = idx & 63, ci = (idx >> 6) & 63, f = idx >> 12;
  // spec_f<BF> order (fym 0: fx-major, 1: fy-major), or fym 2: the four-step loop's class-major order
  // f = ((fx * 9 + k1) * 8 + k2), fy = k1 + 9 k2 (k_fft4.hip col_gemm_kernel)
  int fx, fy;
  if (fym == 2) {
    fx = f / FFT_N;
    const int r = f - fx * FFT_N;
    fy = (r >> 3) + 9 * (r & 7);
  } else {
    fx = fym ? f % FX : f / FFT_N;
    fy = fym ? f / FX : f % FFT_N;
  }
  const int R = KS / 2;
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
  G[idx] = {(float)(gr * inv), (float)(gi * inv)};
}

__global__ void absmax_kernel(const float* __restrict__ x, size_t n, unsigned* out) {
  float m = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(x[i]));
  atomicMax(out, __float_as_uint(m));   // non-negative floats order like their bit patterns
}

// compact split weights Gc[f][part][cq][co]: one f16x8 = re/im of G[ci = 4cq..4cq+3][co] x wscale,
// part 0 = hi, 1 = lo; thread = (f, cq, co)
__global__ void spec_pack_kernel(const cpx* __restrict__ G, f16x8* __restrict__ Gc, float wscale) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NF * 16 * 64) return;
  const int co = idx & 63, cq = (idx >> 6) & 15, f = idx >> 10;
  f16x8 hv, lv;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const cpx g = G[((size_t)f * 64 + 4 * cq + (e >> 1)) * 64 + co];
    const float v = ((e & 1) ? g.y : g.x) * wscale;
    const _Float16 hh = (_Float16)v;
    hv[e] = hh;
    lv[e] = (_Float16)(v - (float)hh);
  }
  Gc[(((size_t)f * 2 + 0) * 16 + cq) * 64 + co] = hv;
  Gc[(((size_t)f * 2 + 1) * 16 + cq) * 64 + co] = lv;
}

// bf16 compact weights Gb[f][cq][co]: one bf16x8 = re/im of G[ci = 4cq..4cq+3][co], unscaled
__global__ void spec_pack_bf_kernel(const cpx* __restrict__ G, uint4* __restrict__ Gb) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NF * 16 * 64) return;
  const int co = idx & 63, cq = (idx >> 6) & 15, f = idx >> 10;
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const cpx g = G[((size_t)f * 64 + 4 * cq + e) * 64 + co];
    w[e] = pack_bf2(g.x, g.y);
  }
  Gb[((size_t)f * 16 + cq) * 64 + co] = uint4{w[0], w[1], w[2], w[3]};
}

// ---------------------------------------------------------------------------------------------
// FFT-path B epilogue (hgru_module.py:729-740, 806-849, 696-711) on the spatial conv result P2:
//   g2 = sigmoid(I . o_r + o_b); e = gamma*(P2 + lat); S = tanh(kappa*(I+e) + omega*(I*e));
//   O' = (g2*O + (1-g2)*S) * rho[t];  then Og' = O' * sigmoid(O' . i_r + i_b)  (or BN_3(O') NHWC)
// One wave per 32-pixel row segment, values held in the v_mfma 32x32 accumulator layout
// (register r of lane (h, x) = channel 32n + 8(r>>2) + 4h + (r&3) of pixel x).  The two 1x1 gate
// GEMMs run on v_mfma_f32_32x32x16_f16 in the f16x3 split.  Their K order is permuted so that the B
// fragment of k-step s is accumulator registers 8(s&1)..8(s&1)+7 of block s>>1 as they stand:
//   k-step s, lane half h, element e  <->  input channel 32(s>>1) + 8(2(s&1) + (e>>2)) + 4h + (e&3)
// (pack_gate_x3_kernel packs the weights in the same order).  sigmoid / tanh use v_exp_f32 and
// v_rcp_f32 (abs error ~1e-7).

// FINAL: the last step's instantiation (p.mode 1 / 2: BN_3(O_T) as the NHWC fp32 map or as fc_1's
// split planes); the other steps' (p.mode 0: the next step's gated state) carries no final-step code,
// so its register budget stays under 128 VGPRs (4 waves per SIMD)
template <bool BF, bool BM, bool FINAL = false>
__global__ __launch_bounds__(256) void spec_epi_b_kernel(ConvArgs p, const float* __restrict__ P,
                                                         const void* __restrict__ or_x3, float or_us,
                                                         const void* __restrict__ ir_x3, float ir_us, int nseg,
                                                         int rev) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int seg0 = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg0 >= nseg) return;
  // rev: segments (images) in descending order, so the first blocks read the P2 lines fft_inv wrote
  // last (still in the Infinity Cache) and the last ones write the Og lines the next fft_fwd reads first
  const int seg = rev ? nseg - 1 - seg0 : seg0;
  const int H = p.H, W = p.W, xs = W / 32;
  const int x = (seg % xs) * 32 + (lane & 31);
  const int y = (seg / xs) % H, b = seg / xs / H;
  f32x16 Iv[2], Y[2];
  // bf16 maps: P2 and O are issued with I, in flight during the o_r gate GEMM (0.195 -> 0.181 ms
  // at B = 256); with fp32 maps the 64 extra live VGPRs cost more than they hide (0.268 -> 0.295)
  f32x4 pvs[2][4], ovs[2][4];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 iv = map_ld4<BM>(p.I, ii_index(b, 4 * n + g, y, x, 4 * h, H, W));
      if constexpr (BM) {
        pvs[n][g] = map_ld4<BM>(P, pp_index(b, 4 * n + g, y, x, 4 * h, H, W));
        ovs[n][g] = map_ld4<BM>(p.O, oo_index(b, 4 * n + g, y, x, 4 * h, H, W));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) Iv[n][4 * g + j] = iv[j];
    }
  gate_any<BF>(or_x3, Iv, Y, lane, or_us);
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = 32 * n + 8 * g + 4 * h;
      const f32x4 pv = BM ? pvs[n][g] : map_ld4<BM>(P, pp_index(b, 4 * n + g, y, x, 4 * h, H, W));
      const size_t odx = oo_index(b, 4 * n + g, y, x, 4 * h, H, W);
      const f32x4 ov = BM ? ovs[n][g] : map_ld4<BM>(p.O, odx);
      const f32x4 lat = *reinterpret_cast<const f32x4*>(p.vecs + V_LAT * 64 + c);
      const f32x4 ga = *reinterpret_cast<const f32x4*>(p.vecs + V_GAMMA * 64 + c);
      const f32x4 ka = *reinterpret_cast<const f32x4*>(p.vecs + V_KAPPA * 64 + c);
      const f32x4 om = *reinterpret_cast<const f32x4*>(p.vecs + V_OMEGA * 64 + c);
      const f32x4 ob = *reinterpret_cast<const f32x4*>(p.vecs + V_OB * 64 + c);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * g + j;
        const float g2 = fsigmoid(Y[n][r] + ob[j]);
        const float iv = Iv[n][r];
        const float e = ga[j] * (pv[j] + lat[j]);
        const float S = ftanh(ka[j] * (iv + e) + om[j] * (iv * e));
        const float on = (g2 * ov[j] + (1.f - g2) * S) * p.rho;
        o[j] = on;
        Iv[n][r] = on;
      }
      map_st4<BM>(p.dst, odx, o);
    }
  f32x16 (&Ov)[2] = Iv;
  if constexpr (!FINAL) {
    gate_any<BF>(ir_x3, Ov, Y, lane, ir_us);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * n + 8 * g + 4 * h;
        const f32x4 ib = *reinterpret_cast<const f32x4*>(p.vecs + V_IB * 64 + c);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = Ov[n][4 * g + j] * fsigmoid(Y[n][4 * g + j] + ib[j]);
        map_st4<BM>(p.dst2, c8_index(b, 4 * n + g, y, x, 4 * h, H, W), o);
      }
  } else if constexpr (FFT_EPI_STAGE) {
    // the wave's 32 pixels x 64 channels of BN_3(O_T) are one contiguous 8 KiB run of the NHWC
    // output (x0 .. x0 + 31 of row y): stage them in LDS ([pixel][channel], pitch 68 floats:
    // conflict-free 16-B writes) and store the run with contiguous lanes, instead of 32-B pieces at
    // a 256-B pixel stride (the final epi_b took 0.40 vs 0.27 ms for the others).  Only the wave's
    // own LDS region is touched, so in-wave ordering suffices.  Same values, same split: bit-identical.
    constexpr int SP = 68;
    __shared__ float stg[4][32 * SP];
    float* sw = stg[threadIdx.x >> 6];
    const int px = lane & 31;
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
        *reinterpret_cast<f32x4*>(sw + px * SP + c) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const size_t e0 = (((size_t)b * H + y) * W + (x - px)) * C;   // the run's first element
    if (p.mode != 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {   // 8 x 1 KiB
        const int q = k * 64 + lane, pp = q >> 4, c4 = (q & 15) * 4;
        *reinterpret_cast<f32x4*>(p.dst2 + e0 + pp * C + c4) = *reinterpret_cast<const f32x4*>(sw + pp * SP + c4);
      }
    } else {   // mode 2: fc_1's f16 hi / lo planes, split exactly as fc_gemm_x3_kernel splits (k_fc.hip)
      typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int k = 0; k < 4; ++k) {   // 4 x (1 KiB hi + 1 KiB lo)
        const int q = k * 64 + lane, pp = q >> 3, c8 = (q & 7) * 8;
        const f32x4 a = *reinterpret_cast<const f32x4*>(sw + pp * SP + c8);
        const f32x4 bq = *reinterpret_cast<const f32x4*>(sw + pp * SP + c8 + 4);
        f16x8_t hv, lv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = j < 4 ? a[j] : bq[j - 4];
          hv[j] = (_Float16)v;
          lv[j] = (_Float16)(v - (float)hv[j]);
        }
        *reinterpret_cast<f16x8_t*>(reinterpret_cast<_Float16*>(p.dst2) + e0 + pp * C + c8) = hv;
        if (p.dst3) *reinterpret_cast<f16x8_t*>(reinterpret_cast<_Float16*>(p.dst3) + e0 + pp * C + c8) = lv;
      }
    }
  } else {
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
        const size_t e = (((size_t)b * H + y) * W + x) * C + c;
        if (p.mode != 2) {
          *reinterpret_cast<f32x4*>(p.dst2 + e) = o;
        } else {   // mode 2: fc_1's f16 hi / lo planes, split exactly as fc_gemm_x3_kernel splits (k_fc.hip)
          typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
          f16x4_t hv, lv;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            hv[j] = (_Float16)o[j];
            lv[j] = (_Float16)(o[j] - (float)hv[j]);
          }
          *reinterpret_cast<f16x4_t*>(reinterpret_cast<_Float16*>(p.dst2) + e) = hv;
          if (p.dst3) *reinterpret_cast<f16x4_t*>(reinterpret_cast<_Float16*>(p.dst3) + e) = lv;
        }
      }
  }
}

// first circuit_input gate (hgru_module.py:696-711) for the FFT path: O0 (NHWC) -> O, and
// Og = O0 * sigmoid(O0 . i_r + i_b) (C8), the gate on f16x3 MFMA; one wave per 32 pixels
template <bool BF, bool BM>
__global__ __launch_bounds__(256) void gate_init_x3_kernel(const float* __restrict__ O0, float* O, float* Og,
                                                           const void* __restrict__ ir_x3, float ir_us,
                                                           const float* __restrict__ vecs, int npix, int H,
                                                           int W) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk * 32 >= npix) return;
  const int pix = blk * 32 + (lane & 31);
  const bool ok = pix < npix;
  const int pp = ok ? pix : npix - 1;
  const int x = pp % W, y = (pp / W) % H, b = pp / (W * H);
  f32x16 V[2], Y[2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(O0 + (size_t)pp * C + 32 * n + 8 * g + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) V[n][4 * g + j] = v[j];
    }
  gate_any<BF>(ir_x3, V, Y, lane, ir_us);
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
        og[j] = o[j] * fsigmoid(Y[n][4 * g + j] + ib[j]);
      }
      const size_t idx = c8_index(b, 4 * n + g, y, x, 4 * h, H, W);
      map_st4<BM>(O, oo_index(b, 4 * n + g, y, x, 4 * h, H, W), o);
      map_st4<BM>(Og, idx, og);
    }
}

// 1x1 gate weights [cin][cout] -> [n2][s][hi|lo][lane] f16x8 in gate_x3's K order; thread =
// (n2, s, lane)
__global__ void pack_gate_x3_kernel(const float* __restrict__ g, f16x8* __restrict__ out, float wscale) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * 4 * 64) return;
  const int lane = i & 63, s = (i >> 6) & 3, n2 = i >> 8, h = lane >> 5;
  const int co = 32 * n2 + (lane & 31);
  f16x8 hv, lv;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ci = 32 * (s >> 1) + 8 * (2 * (s & 1) + (e >> 2)) + 4 * h + (e & 3);
    const float v = g[ci * 64 + co] * wscale;
    const _Float16 hh = (_Float16)v;
    hv[e] = hh;
    lv[e] = (_Float16)(v - (float)hh);
  }
  out[((n2 * 4 + s) * 2) * 64 + lane] = hv;
  out[((n2 * 4 + s) * 2 + 1) * 64 + lane] = lv;
}

__global__ void pack_gate_bf_kernel(const float* __restrict__ g, uint4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * 4 * 64) return;
  const int lane = i & 63, s = (i >> 6) & 3, n2 = i >> 8, h = lane >> 5;
  const int co = 32 * n2 + (lane & 31);
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const int ci0 = 32 * (s >> 1) + 8 * (2 * (s & 1) + (e >> 2)) + 4 * h + (e & 3);
    w[e >> 1] = pack_bf2(g[ci0 * 64 + co], g[(ci0 + 1) * 64 + co]);
  }
  out[(n2 * 4 + s) * 64 + lane] = uint4{w[0], w[1], w[2], w[3]};
}

// ------------------------------------------------------------------------------------ launchers
bool fft_c4_maps() { return (FFT_C4 & 2) != 0; }
bool fft_c4_state() { return (FFT_C4 & 4) != 0; }
bool fft_c4_drive() { return (FFT_C4 & 8) != 0; }
bool fft_bf16_maps() {
  static const bool v = [] {
    const char* e = std::getenv("MP_BF16_MAPS");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}
size_t fft_spec_bytes(int B) { return (size_t)B * 16 * NF * 4 * sizeof(cpx); }
hipError_t device_absmax(const float* x, size_t n, float* out) {
  unsigned* mx = nullptr;
  hipError_t e = hipMalloc(&mx, sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(mx, 0, sizeof(unsigned));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(absmax_kernel, dim3(1024), dim3(256), 0, 0, x, n, mx);
    e = hipGetLastError();
  }
  unsigned bits = 0;
  if (e == hipSuccess) e = hipMemcpy(&bits, mx, sizeof(unsigned), hipMemcpyDeviceToHost);
  if (mx) (void)hipFree(mx);
  std::memcpy(out, &bits, sizeof bits);
  return e;
}

size_t fft_weight_bytes() { return (size_t)NF * 2 * 16 * 64 * sizeof(f16x8); }

hipError_t build_spec_weights(const float* w, int ks, void* Gx, float* unscale, bool bf, bool cls_major) {
  cpx* G = nullptr;
  unsigned* mx = nullptr;
  hipError_t e = hipMalloc(&G, (size_t)NF * 4096 * sizeof(cpx));
  if (e == hipSuccess) e = hipMalloc(&mx, sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(mx, 0, sizeof(unsigned));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(spec_weights_kernel, dim3(NF * 4096 / 256), dim3(256), 0, 0, w, G, ks,
                       cls_major ? 2 : (int)(bf ? fy_major<true>() : fy_major<false>()));
    hipLaunchKernelGGL(absmax_kernel, dim3(1024), dim3(256), 0, 0, reinterpret_cast<const float*>(G),
                       (size_t)NF * 4096 * 2, mx);
    e = hipGetLastError();
  }
  unsigned bits = 0;
  if (e == hipSuccess) e = hipMemcpy(&bits, mx, sizeof(unsigned), hipMemcpyDeviceToHost);
  if (e == hipSuccess && bf) {
    *unscale = 1.0f;
    hipLaunchKernelGGL(spec_pack_bf_kernel, dim3(NF * 16 * 64 / 256), dim3(256), 0, 0, G, static_cast<uint4*>(Gx));
    e = hipGetLastError();
  } else if (e == hipSuccess) {
    // power-of-two weight scale putting max|G| at 2^13..2^14 (f16 max is 65504)
    float m;
    std::memcpy(&m, &bits, sizeof m);
    int ex = 0;
    if (m > 0.f) std::frexp(m, &ex);
    const float wscale = std::ldexp(1.0f, 14 - ex);
    *unscale = 1.0f / (wscale * SPEC_SCALE);
    hipLaunchKernelGGL(spec_pack_kernel, dim3(NF * 16 * 64 / 256), dim3(256), 0, 0, G,
                       static_cast<f16x8*>(Gx), wscale);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (G) (void)hipFree(G);
  if (mx) (void)hipFree(mx);
  return e;
}

hipError_t launch_fft_fwd(const float* act, void* S, int B, int H, int W, hipStream_t st, bool bf) {
  if (!bf && !fy_major<false>() && B <= lfft_maxb())
    hipLaunchKernelGGL(lfft_fwd_kernel, dim3(B * 32), dim3(LF_NT), 0, st, act, S, H, W);
  else if (bf && fft_bf16_maps())
    hipLaunchKernelGGL((fft_fwd_kernel<true, true>), dim3(B * 16), dim3(FNT), 0, st, act, S, H, W);
  else if (bf)
    hipLaunchKernelGGL((fft_fwd_kernel<true, false>), dim3(B * 16), dim3(FNT), 0, st, act, S, H, W);
  else if (!fy_major<false>())
    hipLaunchKernelGGL(fft_fwd3_kernel, dim3(B * 16), dim3(FNT), 0, st, act, S, H, W);
  else
    hipLaunchKernelGGL((fft_fwd_kernel<false, false>), dim3(B * 16), dim3(FNT), 0, st, act, S, H, W);
  return hipGetLastError();
}

hipError_t launch_fft_inv_a_fwd(const void* Y, const ConvArgs& a, void* S, int B, hipStream_t st, bool bf) {
  if (!bf && !fy_major<false>() && B <= lfft_maxb())
    hipLaunchKernelGGL(lfft_inv_a_fwd_kernel, dim3(B * 32), dim3(LF_NT), 0, st, Y, a, S);
  else if (bf && fft_bf16_maps())
    hipLaunchKernelGGL((fft_inv_a_fwd_kernel<true, true>), dim3(B * 16), dim3(FNT), 0, st, Y, a, S);
  else if (bf)
    hipLaunchKernelGGL((fft_inv_a_fwd_kernel<true, false>), dim3(B * 16), dim3(FNT), 0, st, Y, a, S);
  else
    hipLaunchKernelGGL((fft_inv_a_fwd_kernel<false, false>), dim3(B * 16), dim3(FNT), 0, st, Y, a, S);
  return hipGetLastError();
}

// batches up to SPEC_SMALLB run the spectral GEMM on 8-image tiles (spec_gemm_kernel<0, 8>, ceil(B / 8)
// image groups; bit-identical to the 32-image tiles, which measured slower there)
static int spec_smallb() { return SPEC_SMALLB; }

hipError_t launch_spec_gemm(const void* S, const void* Gx, void* Y, int B, float unscale, hipStream_t st, bool bf) {
  const bool small = !bf && B <= spec_smallb();
  const int ngrp = small ? (B + 7) / 8 : (B + SG_NI - 1) / SG_NI;
  if (bf)
    hipLaunchKernelGGL(spec_gemm_bf_kernel, dim3(NQ16 * 16 * ngrp), dim3(256), 0, st, static_cast<const uint4*>(S),
                       static_cast<const uint4*>(Gx), static_cast<uint4*>(Y), B, ngrp);
  else if (small)
    hipLaunchKernelGGL((spec_gemm_kernel<0, 8>), dim3(NQ8 * 8 * ngrp), dim3(256), 0, st, static_cast<const uint4*>(S),
                       static_cast<const uint4*>(Gx), static_cast<uint4*>(Y), B, ngrp, unscale);
  else
    hipLaunchKernelGGL(spec_gemm_kernel<0>, dim3(NQ8 * 8 * ngrp), dim3(256), 0, st, static_cast<const uint4*>(S),
                       static_cast<const uint4*>(Gx), static_cast<uint4*>(Y), B, ngrp, unscale);
  return hipGetLastError();
}

hipError_t launch_fft_inv(const void* Y, float* P, int B, int H, int W, hipStream_t st, bool bf) {
  if (!bf && !fy_major<false>() && B <= lfft_maxb())
    hipLaunchKernelGGL(lfft_inv_kernel, dim3(B * 32), dim3(LF_NT), 0, st, Y, P, H, W);
  else if (bf && fft_bf16_maps())
    hipLaunchKernelGGL((fft_inv_kernel<true, true>), dim3(B * 16), dim3(FNT), 0, st, Y, P, H, W);
  else if (bf)
    hipLaunchKernelGGL((fft_inv_kernel<true, false>), dim3(B * 16), dim3(FNT), 0, st, Y, P, H, W);
  else
    hipLaunchKernelGGL((fft_inv_kernel<false, false>), dim3(B * 16), dim3(FNT), 0, st, Y, P, H, W);
  return hipGetLastError();
}

size_t gate_x3_bytes() { return (size_t)2 * 4 * 2 * 64 * sizeof(f16x8); }

hipError_t pack_gate_x3(const float* g, void* out, float* unscale, bool bf) {
  if (bf) {
    *unscale = 1.0f;
    hipLaunchKernelGGL(pack_gate_bf_kernel, dim3(2), dim3(256), 0, 0, g, static_cast<uint4*>(out));
    return hipGetLastError();
  }
  std::vector<float> h(64 * 64);
  hipError_t e = hipMemcpy(h.data(), g, h.size() * sizeof(float), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  float m = 0.f;
  for (float v : h) m = std::max(m, std::fabs(v));
  int ex = 0;
  if (m > 0.f) std::frexp(m, &ex);
  const float wscale = std::ldexp(1.0f, 14 - ex);   // max|g| at 2^13..2^14
  *unscale = 1.0f / (wscale * GATE_VSCALE);
  hipLaunchKernelGGL(pack_gate_x3_kernel, dim3(2), dim3(256), 0, 0, g, static_cast<f16x8*>(out), wscale);
  return hipGetLastError();
}

hipError_t launch_gate_init_x3(const float* O0, float* O, float* Og, const void* ir_x3, float ir_us, const float* vecs,
                               int B, int H, int W, hipStream_t st, bool bf) {
  const int npix = B * H * W, nw = (npix + 31) / 32;
  if (bf && fft_bf16_maps())
    hipLaunchKernelGGL((gate_init_x3_kernel<true, true>), dim3((nw + 3) / 4), dim3(256), 0, st, O0, O, Og, ir_x3, ir_us, vecs,
                       npix, H, W);
  else if (bf)
    hipLaunchKernelGGL((gate_init_x3_kernel<true, false>), dim3((nw + 3) / 4), dim3(256), 0, st, O0, O, Og, ir_x3, ir_us, vecs,
                       npix, H, W);
  else
    hipLaunchKernelGGL((gate_init_x3_kernel<false, false>), dim3((nw + 3) / 4), dim3(256), 0, st, O0, O, Og, ir_x3, ir_us,
                       vecs, npix, H, W);
  return hipGetLastError();
}

// the B epilogue walks its images last to first, so its first blocks read the P2 lines fft_inv wrote
// last and its last blocks write the Og lines the next fft_fwd reads first (B = 256 fp32 10.43 -> 10.37
// ms per forward against ascending order, profiles/r4o)
static int epi_rev() { return 1; }

hipError_t launch_spec_epi_b(const ConvArgs& a, const float* P, const void* or_x3, float or_us, const void* ir_x3,
                             float ir_us, int B, hipStream_t st, bool bf) {
  const int nseg = B * a.H * (a.W / 32);
#define MP_EPIB(BFV, BMV, FV)                                                                                     \
  hipLaunchKernelGGL((spec_epi_b_kernel<BFV, BMV, FV>), dim3((nseg + 3) / 4), dim3(256), 0, st, a, P, or_x3, or_us, \
                     ir_x3, ir_us, nseg, epi_rev())
  const bool fin = a.mode != 0;
  if (bf && fft_bf16_maps()) {
    if (fin) MP_EPIB(true, true, true);
    else MP_EPIB(true, true, false);
  } else if (bf) {
    if (fin) MP_EPIB(true, false, true);
    else MP_EPIB(true, false, false);
  } else {
    if (fin) MP_EPIB(false, false, true);
    else MP_EPIB(false, false, false);
  }
#undef MP_EPIB
  return hipGetLastError();
}

}  // namespace mp
