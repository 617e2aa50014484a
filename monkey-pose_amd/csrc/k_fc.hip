// Fully-connected layers: split-K fp32 GEMM on v_mfma_f32_32x32x2_f32 + a reduce/epilogue kernel.
//
// Reference: hgru_pose.fc_layer (hgru_pose.py:156-163) = reshape [-1,in] -> tf.matmul(x, W[in,out])
// -> bias_add; then relu (92) and inference BN (95-103, folded to an affine) for fc_1, plain
// bias for fc_out (104).  The same kernels serve every fc_* of the dense / hier heads.
//
// D^T[n][m] = sum_k W[k][n] A[m][k]: W is the MFMA A operand, streamed once from HBM in a packed
// fragment order ([k/8][n/32][lane] float4, one 16-byte load per lane per 8-deep k group); the
// activations (the small M side) are staged in LDS [128 m][32 k + 4] (the +4 pad makes the
// ds_read_b128 row reads conflict-free).  Partial sums per K slice go to a slab
// part[split][M][Npad]; fc_reduce sums the slabs in fixed order (bit-reproducible), then applies
// bias, relu and the per-feature affine.
#include "mp_kernels.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <utility>
#include <vector>

namespace mp {

constexpr int FC_BK = 32, FC_LDA = FC_BK + 4;

__global__ void pack_fc_kernel(const float* __restrict__ W, f32x4* out, int K, int N, int K8, int N32) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)K8 * N32 * 64;
  if (i >= total) return;
  const int lane = i % 64;
  const int nb = (i / 64) % N32;
  const size_t kb = i / ((size_t)64 * N32);
  const int n = 32 * nb + (lane & 31);
  const size_t k0 = 8 * kb + 4 * (lane >> 5);
  f32x4 v;
#pragma unroll
  for (int s = 0; s < 4; ++s) v[s] = (k0 + s < (size_t)K && n < N) ? W[(k0 + s) * N + n] : 0.f;
  out[i] = v;
}

// 1-D grid -> (m tile, n tile, K split), XCD-aware: workgroups are dispatched round-robin over the
// 8 XCDs (separate L2s), so the Mt*Nt blocks of one K split are given ids 8 apart -- one XCD, back
// to back -- and the split's activation rows and weight slab are fetched into that L2 once instead
// of once per tile on different XCDs.  Blocks past the last split exit at once.
struct FcTile {
  int mt, nt, split;
};
__device__ __forceinline__ FcTile fc_tile(int Mt, int Nt) {
  const int id = blockIdx.x, local = id >> 3, per = Mt * Nt;
  const int r = local % per;
  return {r / Nt, r % Nt, (local / per) * 8 + (id & 7)};
}
inline int fc_grid(int Mt, int Nt, int S) { return 8 * ((S + 7) / 8) * Mt * Nt; }

// MB: 32-row m-blocks per block (1 or 2 for M <= 32 / 64: a batch-1 fc_out 18.9 us with 4, the MFMAs
// of 96 empty rows).  Each output row's K sum is the same MFMA chain whatever MB is (bit-identical)
template <int MB>
__global__ __launch_bounds__(256) void fc_gemm_kernel(const float* __restrict__ A, int lda,
                                                      const f32x4* __restrict__ Wpk,
                                                      float* __restrict__ part, int M, int K,
                                                      int N32, int kslice, int S) {
  constexpr int BM = 32 * MB;
  __shared__ float As[BM * FC_LDA];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const FcTile tl = fc_tile((M + BM - 1) / BM, (N32 + 3) / 4);
  if (tl.split >= S) return;
  const int mt = tl.mt, ntile = tl.nt, split = tl.split;
  const int K8 = (K + 7) / 8;
  const int Npad = N32 * 32;
  const int nb = ntile * 4 + wv;
  const bool wave_on = nb < N32;   // wave-uniform
  const int kbeg = split * kslice;
  const int kend = min(K, kbeg + kslice);

  f32x16 acc[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) acc[m] = f32x16{};

  const int nbc = min(nb, N32 - 1);
  for (int k0 = kbeg; k0 < kend; k0 += FC_BK) {
    // the step's weight fragments requested with its activations (one memory latency per step, not
    // two); k groups past K8 load group K8 - 1 and are not used.  With the MB tile: fc_out at batch 1
    // 18.9 -> 7.2 us, at batch 32 13.7 -> 7.7 (profiles/r5_ab/r5y)
    f32x4 wf[FC_BK / 8];
#pragma unroll
    for (int g = 0; g < FC_BK / 8; ++g) wf[g] = Wpk[((size_t)min((k0 >> 3) + g, K8 - 1) * N32 + nbc) * 64 + lane];
    f32x4 v[MB];
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int e = tid + i * 256;          // float4 slots: row = e / 8, k4 = e % 8
      const int row = e >> 3, k4 = (e & 7) * 4;
      const int gm = mt * BM + row, gk = k0 + k4;
      v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (gm < M) {
        if (gk + 3 < kend) {
          v[i] = *reinterpret_cast<const f32x4*>(A + (size_t)gm * lda + gk);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) v[i][s] = (gk + s < kend) ? A[(size_t)gm * lda + gk + s] : 0.f;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int e = tid + i * 256;
      *reinterpret_cast<f32x4*>(As + (e >> 3) * FC_LDA + (e & 7) * 4) = v[i];
    }
    __syncthreads();
    if (wave_on) {
#pragma unroll
      for (int g = 0; g < FC_BK / 8; ++g) {
        const int kb = (k0 >> 3) + g;
        if (kb >= K8) break;
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(As + (m * 32 + col) * FC_LDA + 8 * g + 4 * h);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc[m] = mfma32(wf[g][s], a[s], acc[m]);
        }
      }
    }
  }
  if (!wave_on) return;
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int gm = mt * BM + m * 32 + col;
    if (gm >= M) continue;
    float* dst = part + ((size_t)split * M + gm) * Npad + 32 * nb + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(dst + 8 * g) =
          f32x4{acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]};
  }
}

__global__ void fc_reduce_kernel(const float* __restrict__ part, int S, int M, int N, int Npad,
                                 const float* __restrict__ bias, int relu,
                                 const float* __restrict__ aff_s, const float* __restrict__ aff_t,
                                 float* out, int ldo) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * N) return;
  const int m = i / N, n = i % N;
  // the S partial slabs summed in slab order; their loads issued 16 at a time (a plain loop left
  // one load's latency per slab exposed: 9.7 us for fc_1's 64 slabs at batch 1)
  float v = 0.f;
  const float* pp = part + (size_t)m * Npad + n;
  const size_t ss = (size_t)M * Npad;
  int s = 0;
  for (; s + 16 <= S; s += 16) {
    float t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) t[u] = pp[(size_t)(s + u) * ss];
#pragma unroll
    for (int u = 0; u < 16; ++u) v += t[u];
  }
  for (; s < S; ++s) v += pp[(size_t)s * ss];
  if (bias) v += bias[n];
  if (relu) v = fmaxf(v, 0.f);
  if (aff_s) v = v * aff_s[n] + aff_t[n];
  out[(size_t)m * ldo + n] = v;
}

// ---------------------------------------------------------------------------------------------
// fp32-accurate f16x3 variant (the hGRU pose head's fc_1 under MP_DTYPE_F32_SPLIT / _FFT): the
// same split-K decomposition and slabs (so the same batch invariance), D^T = W^T A^T on
// v_mfma_f32_32x32x16_f16 with both operands split into f16 hi + lo (three products per MAC).
// W is packed [k/16][n/32][hi|lo][lane] f16x8 with a per-tensor power-of-two scale (max|W| at
// 2^13..2^14, so the lo halves stay normal); activations are split unscaled when staged into LDS
// (hi / lo planes [128 m][32 k] f16).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__global__ void pack_fc_x3_kernel(const float* __restrict__ W, f16x8* out, int K, int N, int N32, size_t total,
                                  float wscale) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int lane = i % 64;
  const int nb = (i / 64) % N32;
  const size_t k16 = i / ((size_t)64 * N32);
  const int n = 32 * nb + (lane & 31);
  const size_t k0 = 16 * k16 + 8 * (lane >> 5);
  f16x8 hv, lv;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float v = (k0 + e < (size_t)K && n < N) ? W[(k0 + e) * N + n] * wscale : 0.f;
    const _Float16 hh = (_Float16)v;
    hv[e] = hh;
    lv[e] = (_Float16)(v - (float)hh);
  }
  f16x8* dst = out + ((k16 * N32 + nb) * 2) * 64 + lane;
  dst[0] = hv;
  dst[64] = lv;
}



// K steps are software-pipelined one step ahead: the activation float4s and the weight fragments
// of step k+1 are loaded into registers while step k's MFMAs run; loads are unconditional (row
// index clamped, K a multiple of FC_BK), so all eight loads of a step are in flight together.
// NP = 3: the fp32-accurate f16x3 product; NP = 1 (dtype bf16's fc_1): hi x hi only -- one MFMA per
// MAC and only the hi weight planes are read (half the weight bytes), f16 operands (11-bit
// mantissa, finer than bf16), fp32 accumulation
// MB: 32-row m-blocks per block (4 = 128 rows; small batches take 1 or 2 so the MFMAs of empty rows
// and their staging are not paid: fc_1 at batch 1 / 64)
template <int NP, int MB, int BK = FC_BK>
__global__ __launch_bounds__(256, 3) void fc_gemm_x3_kernel(const float* __restrict__ A, int lda,
                                                         const f16x8* __restrict__ Wpk,
                                                         float* __restrict__ part, int M, int K,
                                                         int N32, int kslice, float unscale, int S) {
  constexpr int BM = 32 * MB;
  constexpr int LD = BK + 8;            // f16 pitch of the planes (+16 B: conflict-free b128 reads)
  constexpr int RQ = BK / 4;            // float4s per activation row per K step
  constexpr int NA = MB * BK / 32;      // activation float4s per thread per K step
  __shared__ _Float16 Ah[BM * LD], Al[NP == 3 ? BM * LD : 1];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const FcTile tl = fc_tile((M + BM - 1) / BM, (N32 + 3) / 4);
  if (tl.split >= S) return;
  const int mt = tl.mt, ntile = tl.nt, split = tl.split;
  const int K16 = (K + 15) / 16;
  const int Npad = N32 * 32;
  const int nb = ntile * 4 + wv;
  const bool wave_on = nb < N32;   // wave-uniform
  const int nbc = min(nb, N32 - 1);
  const int kbeg = split * kslice;
  const int kend = min(K, kbeg + kslice);

  auto load_act = [&](int k0, f32x4 (&v)[NA]) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = tid + i * 256, row = e / RQ, k4 = (e % RQ) * 4;
      const int gm = mt * BM + row;   // K % BK == 0 (launcher): every step is interior
      v[i] = *reinterpret_cast<const f32x4*>(A + (size_t)min(gm, M - 1) * lda + k0 + k4);
      if (gm >= M) v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto load_w = [&](int k0, f16x8 (&w)[BK / 16][2]) {
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      const int kb = min((k0 >> 4) + g, K16 - 1);
      const f16x8* wp = Wpk + (((size_t)kb * N32 + nbc) * 2) * 64 + lane;
      w[g][0] = wp[0];
      if constexpr (NP == 3) w[g][1] = wp[64];
    }
  };

  f32x16 acc[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) acc[m] = f32x16{};
  f32x4 av[NA];
  f16x8 wn[BK / 16][2];
  if (kbeg < kend) {
    load_act(kbeg, av);
    load_w(kbeg, wn);
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    lds_barrier();   // the previous step's LDS reads are done
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = tid + i * 256, row = e / RQ, k4 = (e % RQ) * 4;
      f16x4 hv, lv;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        hv[s] = (_Float16)av[i][s];
        lv[s] = (_Float16)(av[i][s] - (float)hv[s]);
      }
      *reinterpret_cast<f16x4*>(Ah + row * LD + k4) = hv;   // one 8-byte LDS write per plane
      if constexpr (NP == 3) *reinterpret_cast<f16x4*>(Al + row * LD + k4) = lv;
    }
    f16x8 wc[BK / 16][2];
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      wc[g][0] = wn[g][0];
      if constexpr (NP == 3) wc[g][1] = wn[g][1];
    }
    if (k0 + BK < kend) {   // prefetch the next step
      load_act(k0 + BK, av);
      load_w(k0 + BK, wn);
    }
    lds_barrier();
    if (wave_on) {
#pragma unroll
      for (int g = 0; g < BK / 16; ++g) {
        if ((k0 >> 4) + g >= K16) break;
        const f16x8 wh = wc[g][0];
        [[maybe_unused]] const f16x8 wl = wc[g][1];
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          const int o = (m * 32 + col) * LD + 16 * g + 8 * h;
          const f16x8 ah = *reinterpret_cast<const f16x8*>(Ah + o);
          if constexpr (NP == 3) {
            const f16x8 al = *reinterpret_cast<const f16x8*>(Al + o);
            acc[m] = mfma16(wl, ah, acc[m]);
            acc[m] = mfma16(wh, al, acc[m]);
          }
          acc[m] = mfma16(wh, ah, acc[m]);
        }
      }
    }
  }
  if (!wave_on) return;
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int gm = mt * BM + m * 32 + col;
    if (gm >= M) continue;
    float* dst = part + ((size_t)split * M + gm) * Npad + 32 * nb + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(dst + 8 * g) =
          f32x4{acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]} * unscale;
  }
}

// ---------------------------------------------------------------------------------------------
// fc_1 on pre-split activations (the hGRU pose head, FFT dtypes): the last hGRU epilogue
// (k_fft.hip spec_epi_b_kernel, mode 2) writes the BN'd NHWC activations as f16 hi / lo planes
// Ah, Al [M][K] with exactly fc_gemm_x3_kernel's split (hi = (f16)a, lo = (f16)(a - hi)), so the K
// loop here has no conversion work and no register staging: every K step's activation tile is
// copied HBM -> LDS by global_load_lds_dwordx4 (1 KiB per wave-instruction, lane-linear in LDS),
// double-buffered, one barrier per step, while the weights stream to registers one step ahead as
// before.  The LDS image of a plane is [BM rows][BK k] f16 with the 16-byte chunks of each row
// XOR-swizzled by row (the swizzle is applied to the global source address, since the DMA writes
// LDS lane-linearly), so the 32 consecutive rows one ds_read_b128 fragment load touches hit
// distinct banks.  MFMA order per output is fc_gemm_x3_kernel's: bit-identical results.
#ifndef FC_P_MINB
#define FC_P_MINB 3   // blocks per CU the pre-split kernel is register-budgeted for (one product)
#endif
#ifndef FC_P_BK3
#define FC_P_BK3 32   // K step of the three-product kernel
#endif
#ifndef FC_P_MINB3
#define FC_P_MINB3 3
#endif
#ifndef FC_P_NW3
#define FC_P_NW3 4    // waves per block of the three-product kernel (each 32 output columns)
#endif
template <int BK>
__device__ __forceinline__ int fcp_swz(int row) {   // 16-B chunk swizzle of a row (BK = 32: 4 chunks, 64: 8)
  return BK == 32 ? (row >> 2) & 3 : (row >> 1) & 7;
}

#ifndef FC_P_BIG
#define FC_P_BIG 1    // the 256 x 256 tile (8 waves, one block per CU) for the three-product kernel above 128 rows
#endif
#ifndef FC_PB_NW
#define FC_PB_NW 8    // waves per 256-row block: 8 (256 columns, one block per CU) or 4 (128 columns, two)
#endif
#ifndef FC_PB_NST
#define FC_PB_NST 3   // its stages (32 KiB each)
#endif
#ifndef FC_PB_PIPE
#define FC_PB_PIPE 1  // 256-row tile: fragment reads one group ahead of the MFMAs
#endif
#ifndef FC_P_NST
#define FC_P_NST 3    // activation LDS stages / weight register slots: loads run NST - 1 K steps ahead
#endif
// The A fragments of one 16-deep k group: N = MB x planes ds_read_b128 at immediate offsets from the
// lane's base, issued together and waited for in the SAME asm statement.  Written as plain loads,
// LLVM's waitcnt pass cannot tell them from the LDS-DMA writes still in flight into the other
// stages and puts an s_waitcnt vmcnt(0) before them: every later step's loads -- the weights and the
// activation DMA issued one and two steps ahead -- were then waited for at each step, so nothing
// overlapped the MFMAs.  Stage reuse is ordered by the explicit vmcnt + barrier of the K loop.
#ifndef FC_P_ASMRD
#define FC_P_ASMRD 1
#endif
template <int N, class F, int... I>
__device__ __forceinline__ void fcp_unroll_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void fcp_unroll(F&& f) {   // f(integral_constant<0>) ... f(<N - 1>)
  fcp_unroll_<N>(f, std::make_integer_sequence<int, N>{});
}
// The weight fragments likewise load through asm (FC_P_ASMW): the compiler's own waits for them
// merged to vmcnt(0) at the loop head (the slot registers are renamed around the unrolled loop), so
// the loads are invisible to it and the K loop's explicit wait -- which names the slot's registers
// as in/out operands, so no use of them can be scheduled above it -- is the only one.
#ifndef FC_P_ASMW
#define FC_P_ASMW 1
#endif
// FC_P_NTW: the three-product kernel's weight stream (every packed weight read once, by one CU)
// loaded non-temporal, so it evicts less of the activation slices that the N tiles of a K slice
// share through their XCD's L2: fp32 fc_1 at B = 256 0.369 -> 0.359-0.362 ms, PMC 1,645 -> 1,571 MB
// (1.17x the algorithmic 1,342 instead of 1.22x; profiles/r4n).  The one-product (bf16) kernel keeps
// the default policy: nt made it 0.19 -> 0.23 ms.
#ifndef FC_P_NTW
#define FC_P_NTW 1
#endif
#if FC_P_NTW
#define FCP_WPOL " nt"
#else
#define FCP_WPOL ""
#endif
__device__ __forceinline__ void fcp_ldw2(f16x8& a, f16x8& b, const f16x8* p) {
  asm volatile("global_load_dwordx4 %0, %2, off" FCP_WPOL "\n\tglobal_load_dwordx4 %1, %2, off offset:1024" FCP_WPOL
               : "=&v"(a), "=&v"(b)
               : "v"(p)
               : "memory");
}
__device__ __forceinline__ void fcp_ldw1(f16x8& a, const f16x8* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(a) : "v"(p) : "memory");
}
template <int CNT, int NP, int G>
__device__ __forceinline__ void fcp_wait(f16x8 (&w)[G][2]) {
  if constexpr (NP == 3) {
    static_assert(G == 2, "three-product kernel: 32-deep K steps");
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[1][0]), "+v"(w[1][1]) : "n"(CNT) : "memory");
  } else {
    static_assert(G == 4, "one-product kernel: 64-deep K steps");
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0][0]), "+v"(w[1][0]), "+v"(w[2][0]), "+v"(w[3][0]) : "n"(CNT) : "memory");
  }
}

template <int O0, int O1, int O2, int O3>
__device__ __forceinline__ void fcp_read4(f16x8 (&a)[4], uint32_t base) {
  asm volatile("ds_read_b128 %0, %4 offset:%c5\n\tds_read_b128 %1, %4 offset:%c6\n\t"
               "ds_read_b128 %2, %4 offset:%c7\n\tds_read_b128 %3, %4 offset:%c8\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3])
               : "v"(base), "n"(O0), "n"(O1), "n"(O2), "n"(O3)
               : "memory");
}
template <int O0, int O1>
__device__ __forceinline__ void fcp_read2(f16x8 (&a)[4], uint32_t base) {
  asm volatile("ds_read_b128 %0, %2 offset:%c3\n\tds_read_b128 %1, %2 offset:%c4\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(a[0]), "=&v"(a[1])
               : "v"(base), "n"(O0), "n"(O1)
               : "memory");
}
template <int O0>
__device__ __forceinline__ void fcp_read1(f16x8 (&a)[4], uint32_t base) {
  asm volatile("ds_read_b128 %0, %1 offset:%c2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(a[0]) : "v"(base), "n"(O0) : "memory");
}

template <int NP, int MB, int BK, int MINB, int NW = 4, int NST = FC_P_NST>
__global__ __launch_bounds__(64 * NW, MINB) void fc_gemm_x3p_kernel(const _Float16* __restrict__ Ah,
                                                               const _Float16* __restrict__ Al, int lda,
                                                               const f16x8* __restrict__ Wpk,
                                                               float* __restrict__ part, int M, int K, int N32,
                                                               int kslice, float unscale, int S) {
  static_assert(NST >= 2 && NST <= 4, "stage count");
  constexpr int BM = 32 * MB;
  constexpr int NPL = NP == 3 ? 2 : 1;         // activation planes staged (hi, lo)
  constexpr int CH = BK / 8;                   // 16-B chunks per row
  constexpr int PLANE = BM * BK;               // f16 per plane per stage
  constexpr int STAGE = NPL * PLANE;
  constexpr int RPI = 1024 / (BK * 2);         // rows per glds wave-instruction
  constexpr int NI = NPL * BM / RPI;           // glds wave-instructions per stage
  constexpr int NIW = (NI + NW - 1) / NW;      // per wave
  constexpr int GRP = NIW + (BK / 16) * NPL;   // vector-memory instructions one K step issues per lane
  // asm weight loads for the 64- and 128-row tiles (B > 32: fc_1 0.477 -> 0.451 ms at B = 256); the
  // 32-row tile keeps hipcc's loads (0.190 vs 0.197 ms at B = 1).  Same arithmetic either way.
  constexpr bool ASMW = FC_P_ASMW && MB > 1;
  constexpr bool BIGOFF = NST * STAGE * 2 > 65536 - 32 * BK * 2 * MB;   // the 256-row tile's stages
  static_assert(!BIGOFF || MB > 1, "big-offset reads pair m-blocks");
  __shared__ _Float16 lds[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, col = lane & 31;
  const FcTile tl = fc_tile((M + BM - 1) / BM, (N32 + NW - 1) / NW);
  if (tl.split >= S) return;
  const int mt = tl.mt, ntile = tl.nt, split = tl.split;
  const int K16 = (K + 15) / 16;
  const int Npad = N32 * 32;
  const int nb = ntile * NW + wv;
  const bool wave_on = nb < N32;   // wave-uniform
  const int nbc = min(nb, N32 - 1);
  const int kbeg = split * kslice;
  const int kend = min(K, kbeg + kslice);
  const int nsteps = kend > kbeg ? (kend - kbeg) / BK : 0;   // K, kslice multiples of BK (launcher)

  // this lane's glds sources (k offset added per step) and the wave-uniform LDS destinations (a
  // wave past the NI-th instruction repeats the last one: the same bytes to the same place)
  const _Float16* src[NIW];
  int dst[NIW];
#pragma unroll
  for (int j = 0; j < NIW; ++j) {
    const int i = min(wv + NW * j, NI - 1);
    const int pl = i / (BM / RPI), r0 = (i % (BM / RPI)) * RPI;
    const int row = r0 + lane / CH, c = (lane % CH) ^ fcp_swz<BK>(row);
    const int gm = min(mt * BM + row, M - 1);   // rows past M: valid addresses, outputs never stored
    src[j] = (pl ? Al : Ah) + (size_t)gm * lda + 8 * c;
    dst[j] = pl * PLANE + r0 * BK;
  }
  // one K step's loads: the activation tile by LDS DMA into stage `stg`, the weight fragments into
  // register slot `w` (issued in this order, GRP instructions)
  auto issue = [&](int k0, int stg, f16x8 (&w)[BK / 16][2]) {
#pragma unroll
    for (int j = 0; j < NIW; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src[j] + k0),
                                       (__attribute__((address_space(3))) void*)(lds + stg * STAGE + dst[j]), 16, 0, 0);
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      const int kb = min((k0 >> 4) + g, K16 - 1);
      const f16x8* wp = Wpk + (((size_t)kb * N32 + nbc) * 2) * 64 + lane;
      if constexpr (ASMW) {
        if constexpr (NP == 3) fcp_ldw2(w[g][0], w[g][1], wp);
        else fcp_ldw1(w[g][0], wp);
      } else {
        w[g][0] = wp[0];
        if constexpr (NP == 3) w[g][1] = wp[64];
      }
    }
  };

  // this lane's fragment address in a stage (bytes; plane, m and stage are immediate offsets): row
  // col of each 32-row block (the swizzle depends on col only), chunk 2g + h
  const uint32_t lds_base = (uint32_t)(size_t)(__attribute__((address_space(3))) _Float16*)lds;
  uint32_t rd_off[BK / 16];
#pragma unroll
  for (int g = 0; g < BK / 16; ++g) rd_off[g] = (uint32_t)((col * BK + 8 * ((2 * g + h) ^ fcp_swz<BK>(col))) * 2);
  f32x16 acc[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) acc[m] = f32x16{};
  // K step s: activation stage s % NST, weight slot s % NST; step s + NST - 1 is issued at step s,
  // after the barrier that retires step s - 1 (the stage it overwrites)
  // Every step issues a group, past the end too (the last step's addresses again, into a stage
  // nobody reads any more): the number of groups in flight behind step s is then always NST - 2,
  // and the compiler's own wait for the weight registers is exact (a conditional issue made it
  // merge the two paths into vmcnt(0))
  f16x8 wr[NST][BK / 16][2];
  const int slast = max(nsteps - 1, 0);
#pragma unroll
  for (int d = 0; d < NST - 1; ++d) issue(kbeg + min(d, slast) * BK, d, wr[d]);
  // step s (stage / slot u = s % NST): wait, barrier, issue step s + NST - 1, MFMAs
  auto step = [&](auto U, int s) {
    constexpr int u = decltype(U)::value;
    // step s's tile and weights have landed; the NST - 2 later groups may stay in flight
    if constexpr (ASMW) fcp_wait<(NST - 2) * GRP, NP>(wr[u]);   // ties slot u's registers to the wait
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * GRP) : "memory");
    lds_barrier();   // every wave's DMA share of stage u landed; every wave is done with step s - 1
    issue(kbeg + min(s + NST - 1, slast) * BK, (u + NST - 1) % NST, wr[(u + NST - 1) % NST]);
    // no wave_on branch: a wave past N computes column block nbc again and stores nothing (a
    // branch here, like a conditional step, made the compiler's wait for the weight registers
    // merge to vmcnt(0))
    if constexpr (BIGOFF && FC_PB_PIPE && NP == 3) {
      // 256-row tile: the (k group, m pair) fragment groups of the step in sequence, group i + 1's four
      // ds_read_b128 issued before group i's MFMAs (two fragment sets), and the two m-blocks' MFMAs
      // interleaved (each accumulator keeps its own product order: bit-identical)
      constexpr int NPR = MB / 2, NGR = (BK / 16) * NPR;
      constexpr int OS = u * STAGE * 2, OP = PLANE * 2, OM = 32 * BK * 2;
      f16x8 fa[2][4];
      auto rd = [&](auto I) {
        constexpr int i = decltype(I)::value, g = i / NPR, m0 = 2 * (i % NPR), m1 = m0 + 1;
        const uint32_t base = lds_base + rd_off[g] + (uint32_t)OS;
        f16x8 (&a)[4] = fa[i & 1];
        asm volatile("ds_read_b128 %0, %4 offset:%c5\n\tds_read_b128 %1, %4 offset:%c6\n\t"
                     "ds_read_b128 %2, %4 offset:%c7\n\tds_read_b128 %3, %4 offset:%c8"
                     : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3])
                     : "v"(base), "n"(m0 * OM), "n"(m1 * OM), "n"(OP + m0 * OM), "n"(OP + m1 * OM)
                     : "memory");
      };
      rd(std::integral_constant<int, 0>{});
      fcp_unroll<NGR>([&](auto I) {
        constexpr int i = decltype(I)::value, g = i / NPR, m0 = 2 * (i % NPR), m1 = m0 + 1;
        f16x8 (&a)[4] = fa[i & 1];
        if constexpr (i + 1 < NGR) {
          rd(std::integral_constant<int, i + 1>{});
          asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]) :: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]) :: "memory");
        }
        const f16x8 wh = wr[u][g][0], wl = wr[u][g][1];
        acc[m0] = mfma16(wl, a[0], acc[m0]);
        acc[m1] = mfma16(wl, a[1], acc[m1]);
        acc[m0] = mfma16(wh, a[2], acc[m0]);
        acc[m1] = mfma16(wh, a[3], acc[m1]);
        acc[m0] = mfma16(wh, a[0], acc[m0]);
        acc[m1] = mfma16(wh, a[1], acc[m1]);
      });
      return;
    }
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      const f16x8 wh = wr[u][g][0];
      [[maybe_unused]] const f16x8 wl = wr[u][g][1];
      // m-blocks in pairs (one pair's hi / lo fragments live at a time: 16 VGPRs)
      fcp_unroll<(MB + 1) / 2>([&](auto P) {
        constexpr int m0 = 2 * decltype(P)::value, m1 = m0 + (MB > 1 ? 1 : 0);
        constexpr int OS = u * STAGE * 2, OP = PLANE * 2, OM = 32 * BK * 2;
        f16x8 a[4];   // ah(m0), ah(m1), al(m0), al(m1) (MB = 1: ah, al)
        if constexpr (FC_P_ASMRD && BIGOFF) {   // stage base in the address (ds_read offsets are 16-bit)
          const uint32_t base = lds_base + rd_off[g] + (uint32_t)OS;
          if constexpr (NP == 3) fcp_read4<m0 * OM, m1 * OM, OP + m0 * OM, OP + m1 * OM>(a, base);
          else fcp_read2<m0 * OM, m1 * OM>(a, base);
        } else if constexpr (FC_P_ASMRD) {
          const uint32_t base = lds_base + rd_off[g];
          if constexpr (MB > 1 && NP == 3) fcp_read4<OS + m0 * OM, OS + m1 * OM, OS + OP + m0 * OM, OS + OP + m1 * OM>(a, base);
          else if constexpr (MB > 1) fcp_read2<OS + m0 * OM, OS + m1 * OM>(a, base);
          else if constexpr (NP == 3) { fcp_read2<OS, OS + OP>(a, base); a[2] = a[1]; }
          else fcp_read1<OS>(a, base);
        } else {
          const _Float16* tile = lds + u * STAGE + rd_off[g] / 2;
          a[0] = *reinterpret_cast<const f16x8*>(tile + m0 * 32 * BK);
          a[1] = *reinterpret_cast<const f16x8*>(tile + m1 * 32 * BK);
          if constexpr (NP == 3) {
            a[2] = *reinterpret_cast<const f16x8*>(tile + PLANE + m0 * 32 * BK);
            a[3] = *reinterpret_cast<const f16x8*>(tile + PLANE + m1 * 32 * BK);
          }
        }
        fcp_unroll<(MB > 1 ? 2 : 1)>([&](auto Q) {
          constexpr int q = decltype(Q)::value, m = m0 + q;
          const f16x8 ah = a[q];
          if constexpr (NP == 3) {
            const f16x8 al = a[2 + q];
            acc[m] = mfma16(wl, ah, acc[m]);
            acc[m] = mfma16(wh, al, acc[m]);
          }
          acc[m] = mfma16(wh, ah, acc[m]);
        });
      });
    }
  };
  // whole rounds of NST steps (no conditional step inside the loop), then the remainder
  const int nfull = nsteps / NST * NST;
  for (int s0 = 0; s0 < nfull; s0 += NST) fcp_unroll<NST>([&](auto U) { step(U, s0 + decltype(U)::value); });
  fcp_unroll<NST>([&](auto U) {
    if (nfull + decltype(U)::value < nsteps) step(U, nfull + decltype(U)::value);
  });
  // the groups issued past the last step (weights and LDS DMA) land before the wave ends: a DMA
  // still in flight at s_endpgm could write into LDS handed to the next workgroup.  Under
  // FC_P_ASMW every weight slot is named in/out here, so the registers of the never-consumed
  // groups stay allocated until their loads have landed (hipcc takes an asm load's destination
  // as written at the statement: dead right away, it could hand the register to the epilogue)
  if constexpr (ASMW) {
    fcp_wait<0, NP>(wr[0]);
    fcp_wait<0, NP>(wr[1]);
    if constexpr (NST > 2) fcp_wait<0, NP>(wr[2]);
    if constexpr (NST > 3) fcp_wait<0, NP>(wr[3]);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (!wave_on) return;
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int gm = mt * BM + m * 32 + col;
    if (gm >= M) continue;
    float* dstp = part + ((size_t)split * M + gm) * Npad + 32 * nb + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(dstp + 8 * g) =
          f32x4{acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]} * unscale;
  }
}

hipError_t launch_fc_gemm_x3p(const void* Ah, const void* Al, int lda, const void* Wpk, float unscale, float* part,
                              int M, int K, int N, int S, int kslice, hipStream_t st, int nprod) {
  const int BK = nprod == 1 ? 64 : FC_P_BK3;
  if (K % BK || kslice % BK || lda % 8 || (nprod == 3 && !Al)) return hipErrorInvalidValue;
  const int N32 = (N + 31) / 32;
  // three products above 128 rows: one 256 x 256 tile per block (8 waves of 256 rows x 32 columns,
  // one block per CU).  Per 32-deep K step a CU then moves 32 KiB of activations (shared by the 8
  // waves through LDS) and 32 KiB of weights for 48 MFMAs per wave, 21 B per cycle of MFMA time,
  // where three 128 x 128 blocks per CU moved 43 B / cycle, ~2/3 of an XCD's L2 bandwidth per CU
  const bool big = nprod == 3 && M > 128 && FC_P_BIG;
  const int mb = M <= 32 ? 1 : (M <= 64 ? 2 : (big ? 8 : 4));
  const int nw = big ? FC_PB_NW : (nprod == 3 ? FC_P_NW3 : 4);   // waves (32-column groups) per block
  const int grid = fc_grid((M + 32 * mb - 1) / (32 * mb), (N32 + nw - 1) / nw, S);
  const _Float16* h = static_cast<const _Float16*>(Ah);
  const _Float16* l = static_cast<const _Float16*>(Al);
  const f16x8* w = static_cast<const f16x8*>(Wpk);
#define MP_FCP(NPV, MBV, BKV, MINBV)                                                                                   \
  hipLaunchKernelGGL((fc_gemm_x3p_kernel<NPV, MBV, BKV, MINBV>), dim3(grid), dim3(256), 0, st, h, l, lda, w, part, M, K, \
                     N32, kslice, unscale, S)
#define MP_FCP3(MBV)                                                                                                   \
  hipLaunchKernelGGL((fc_gemm_x3p_kernel<3, MBV, FC_P_BK3, FC_P_MINB3, FC_P_NW3>), dim3(grid), dim3(64 * FC_P_NW3), 0, \
                     st, h, l, lda, w, part, M, K, N32, kslice, unscale, S)
  if (nprod == 1) {
    if (mb == 1) MP_FCP(1, 1, 64, FC_P_MINB);
    else if (mb == 2) MP_FCP(1, 2, 64, FC_P_MINB);
    else MP_FCP(1, 4, 64, FC_P_MINB);
  } else {
    if (mb == 1) MP_FCP3(1);
    else if (mb == 2) MP_FCP3(2);
    else if (mb == 8)
      hipLaunchKernelGGL((fc_gemm_x3p_kernel<3, 8, FC_P_BK3, 8 / FC_PB_NW, FC_PB_NW, FC_PB_NST>), dim3(grid),
                         dim3(64 * FC_PB_NW), 0, st, h, l, lda, w, part,
                         M, K, N32, kslice, unscale, S);
    else MP_FCP3(4);
  }
#undef MP_FCP
#undef MP_FCP3
  return hipGetLastError();
}

__global__ void pad_cin_kernel(const float* __restrict__ w, float* __restrict__ out, int taps, int Cin, int cinp,
                               int Cout) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)taps * cinp * Cout) return;
  const int co = i % Cout;
  const size_t r = i / Cout;
  const int ci = r % cinp, t = r / cinp;
  out[i] = ci < Cin ? w[((size_t)t * Cin + ci) * Cout + co] : 0.f;
}

hipError_t launch_pad_cin(const float* w, float* out, int taps, int Cin, int cinp, int Cout, hipStream_t st) {
  const size_t total = (size_t)taps * cinp * Cout;
  hipLaunchKernelGGL(pad_cin_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, out, taps, Cin, cinp, Cout);
  return hipGetLastError();
}

size_t fc_x3_bytes(int K, int N) { return (size_t)(K + 15) / 16 * ((N + 31) / 32) * 2 * 64 * sizeof(f16x8); }

hipError_t launch_pack_fc_x3(const float* W, void* out, int K, int N, float* unscale, hipStream_t st) {
  // power-of-two weight scale from max|W|
  float mx = 0.f;
  hipError_t e = device_absmax(W, (size_t)K * N, &mx);
  if (e != hipSuccess) return e;
  int ex = 0;
  if (mx > 0.f) std::frexp(mx, &ex);
  const float wscale = std::ldexp(1.0f, 14 - ex);
  *unscale = 1.0f / wscale;
  const int N32 = (N + 31) / 32;
  const size_t total = (size_t)(K + 15) / 16 * N32 * 64;
  hipLaunchKernelGGL(pack_fc_x3_kernel, dim3((total + 255) / 256), dim3(256), 0, st, W, static_cast<f16x8*>(out),
                     K, N, N32, total, wscale);
  return hipGetLastError();
}

hipError_t launch_fc_gemm_x3(const float* A, int lda, const void* Wpk, float unscale, float* part, int M, int K,
                             int N, int S, int kslice, hipStream_t st, int nprod) {
  if (K % FC_BK || kslice % FC_BK || lda % 4) return hipErrorInvalidValue;
  const int N32 = (N + 31) / 32;
  const int mb = M <= 32 ? 1 : (M <= 64 ? 2 : 4);   // 32-row m-blocks per block
  const int grid = fc_grid((M + 32 * mb - 1) / (32 * mb), (N32 + 3) / 4, S);
  const f16x8* w = static_cast<const f16x8*>(Wpk);
#define MP_FC_X3(NPV, MBV)                                                                                   \
  hipLaunchKernelGGL((fc_gemm_x3_kernel<NPV, MBV>), dim3(grid), dim3(256), 0, st, A, lda, w, part, M, K, N32, \
                     kslice, unscale, S)
#define MP_FC_X3K(NPV, MBV, BKV)                                                                                   \
  hipLaunchKernelGGL((fc_gemm_x3_kernel<NPV, MBV, BKV>), dim3(grid), dim3(256), 0, st, A, lda, w, part, M, K, N32, \
                     kslice, unscale, S)
  static const int bk64 = [] {
    const char* e = std::getenv("MP_FC_BK64");
    return e ? std::atoi(e) : 1;
  }();
  // one product (bf16): 64-deep K steps, half the barriers and LDS staging passes per MFMA --
  // bf16 fc_1 0.320 -> 0.263 ms at batch 256, 0.161 -> 0.129 at 32, 0.153 -> 0.106 at 1
  if (nprod == 1 && bk64 && K % 64 == 0 && kslice % 64 == 0) {
    if (mb == 1) MP_FC_X3K(1, 1, 64);
    else if (mb == 2) MP_FC_X3K(1, 2, 64);
    else MP_FC_X3K(1, 4, 64);
  } else if (nprod == 1) {
    if (mb == 1) MP_FC_X3(1, 1);
    else if (mb == 2) MP_FC_X3(1, 2);
    else MP_FC_X3(1, 4);
  } else {   // three products: 64-deep steps spill at 128 rows (160 B / lane, fc_1 0.46 -> 1.47 ms)
    if (mb == 1) MP_FC_X3(3, 1);
    else if (mb == 2) MP_FC_X3(3, 2);
    else MP_FC_X3(3, 4);
  }
#undef MP_FC_X3
#undef MP_FC_X3K
  return hipGetLastError();
}

hipError_t launch_pack_fc(const float* W, f32x4* out, int K, int N, hipStream_t st) {
  const int K8 = (K + 7) / 8, N32 = (N + 31) / 32;
  const size_t total = (size_t)K8 * N32 * 64;
  hipLaunchKernelGGL(pack_fc_kernel, dim3((total + 255) / 256), dim3(256), 0, st, W, out, K, N, K8, N32);
  return hipGetLastError();
}

// K slices: a function of K only, so every output row is summed in the same order whatever the
// batch size (results are bit-identical between a crop alone and inside a batch).  Large K
// (fc_1: 262,144) in slices of ~4,096; small K in slices of 128 so a short GEMM still spreads
// over enough blocks (fc_out, K = 1,024: 8 slices instead of 1).
int fc_choose_splits(int M, int K, int N, int* kslice) {
  (void)M;
  // large K: slices of ~5.4k, i.e. 48 for fc_1 (K = 262,144): at batch 256 that is 2 x 8 x 48 = 768
  // blocks = one full round of 3 blocks on each of the 256 CUs (64 slices left a 1/3-full second
  // round); and at least 384 blocks per 128-row tile whatever N is (the dense head's fc_1_1 / fc_1_2,
  // N = 512: 18 / 12 slices gave 192 / 128 blocks at batch 256 and 0.25 ms each).  A function of
  // K and N only, so a crop's sums group the same way at every batch.  MP_FC_KSLICE (A/B only)
  // fixes the slice length.
  static const char* kenv = std::getenv("MP_FC_KSLICE");
  static const int ksz = kenv ? std::max(32, std::atoi(kenv)) : 5440;
  const int nt = ((N + 31) / 32 + 3) / 4;   // 128-column tiles
  static const int smallk = [] {   // K per slice below 32k (A/B knob MP_FC_SMALLK)
    const char* e = std::getenv("MP_FC_SMALLK");
    return e ? std::max(32, std::atoi(e)) : 128;
  }();
  int S = K >= 32768 ? std::max(1, K / ksz) : std::min(64, (K + smallk - 1) / smallk);
  if (K >= 32768 && !kenv) S = std::min(std::max(S, (384 + nt - 1) / nt), K / 512);
  // N a multiple of 256 (fc_1: 1,024): the 256 x 256 tiles of launch_fc_gemm_x3p's 256-row kernel,
  // 256 / (N / 256) K slices (64 for fc_1: one block on each of the 256 CUs at batch 256)
  if (K >= 32768 && !kenv && FC_P_BIG && N % 256 == 0) S = std::min(std::max(1, 256 / (N / 256)), K / 512);
  if (S < 1) S = 1;
  int ks = (K + S - 1) / S;
  const int q = K % 64 == 0 ? 64 : FC_BK;   // whole 64-deep steps where K allows (the one-product kernel)
  ks = (ks + q - 1) / q * q;
  S = (K + ks - 1) / ks;
  *kslice = ks;
  return S;
}

hipError_t launch_fc_gemm(const float* A, int lda, const f32x4* Wpk, float* part, int M, int K, int N,
                          int S, int kslice, hipStream_t st) {
  const int N32 = (N + 31) / 32;
  const int mb = M <= 32 ? 1 : (M <= 64 ? 2 : 4);
  const int grid = fc_grid((M + 32 * mb - 1) / (32 * mb), (N32 + 3) / 4, S);
  if (mb == 1)
    hipLaunchKernelGGL(fc_gemm_kernel<1>, dim3(grid), dim3(256), 0, st, A, lda, Wpk, part, M, K, N32, kslice, S);
  else if (mb == 2)
    hipLaunchKernelGGL(fc_gemm_kernel<2>, dim3(grid), dim3(256), 0, st, A, lda, Wpk, part, M, K, N32, kslice, S);
  else
    hipLaunchKernelGGL(fc_gemm_kernel<4>, dim3(grid), dim3(256), 0, st, A, lda, Wpk, part, M, K, N32, kslice, S);
  return hipGetLastError();
}

hipError_t launch_fc_reduce(const float* part, int S, int M, int N, const float* bias, int relu,
                            const float* aff_s, const float* aff_t, float* out, int ldo, hipStream_t st) {
  const int Npad = (N + 31) / 32 * 32;
  const size_t total = (size_t)M * N;
  hipLaunchKernelGGL(fc_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, part, S, M, N, Npad,
                     bias, relu, aff_s, aff_t, out, ldo);
  return hipGetLastError();
}

}  // namespace mp
