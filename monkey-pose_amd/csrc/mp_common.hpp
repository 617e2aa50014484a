// Shared definitions for the monkey-pose MI355X (gfx950) kernels.
//
// Activation layout ("C8"): every 64-channel feature map of the hot path is stored in HBM as
//   act[b][q][y][x][e],  q = c / 8 (8 channel chunks), e = c % 8
// so that one halo-chunk load of the association-field convolution reads 32 contiguous bytes
// per pixel and one epilogue store of a 32x32 fp32 MFMA tile is a contiguous 1 KiB run.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace mp {

constexpr int C = 64;      // channels of every hGRU / backbone map (hgru_pose.py:50-81)
constexpr int NQ = C / 8;  // channel chunks in the C8 layout

__device__ __forceinline__ size_t c8_index(int b, int q, int y, int x, int e, int H, int W) {
  return ((((size_t)b * NQ + q) * H + y) * W + x) * 8 + e;
}
// C4 [N][16 channel groups][H][W][4]: the FFT loop's P2, I, O and X maps (k_fft.hip pp_index, ii_index,
// oo_index, xx_index), written per 4-channel group by the inverse FFT kernels as one contiguous run;
// channel 8 q + e of the C8 naming.  W must be a power of two: the C4_SWZ swizzle x ^ (W / 2) maps
// [0, W) onto itself only then (the FFT path's maps are 32 or 64 wide; launchers check c4_width_ok)
#ifndef C4_SWZ
#define C4_SWZ 1
#endif
__host__ __device__ constexpr bool c4_width_ok(int W) { return W > 0 && (W & (W - 1)) == 0; }
__device__ __forceinline__ size_t c4_index(int b, int q, int y, int x, int e, int H, int W) {
  // C4_SWZ: the odd group's row halves swapped, so the two half-waves of a C8-pattern access (groups
  // 2q and 2q + 1 at the same 32 pixels) read runs 512 B apart modulo 64 KiB
  const int xs = (C4_SWZ && (e & 4)) ? (x ^ (W >> 1)) : x;
  return ((((size_t)b * (2 * NQ) + 2 * q + (e >> 2)) * H + y) * W + xs) * 4 + (e & 3);
}

// bf16 C8 maps (MP_DTYPE_BF16's hGRU maps): 4 channels = 8 bytes, round to nearest even on store
__device__ __forceinline__ uint2 bf16x4_pack(f32x4 v) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const bf2_t a = {(__bf16)v[0], (__bf16)v[1]}, b = {(__bf16)v[2], (__bf16)v[3]};
  return uint2{__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b)};
}
__device__ __forceinline__ f32x4 bf16x4_unpack(uint2 u) {
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}

// v_mfma_f32_32x32x2_f32: exact fp32 (fma chain), 64 cycles issue per SIMD.
// A lane l: A[i=l&31][k=l>>5];  B lane l: B[k=l>>5][j=l&31];
// D lane l: D[i=(r&3)+8(r>>2)+4(l>>5)][j=l&31], r = 0..15.
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, then s_barrier.
// __syncthreads() also carries a release fence, which drains every outstanding global load and
// store (s_waitcnt vmcnt(0)) -- including prefetches meant to stay in flight across the barrier.
// Use only where no global-memory ordering between the block's threads is needed.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// per-channel parameter vectors of the hGRU epilogues, each 64 floats, in this order
enum VecId {
  V_LAT = 0,   // lateral_bias        (hgru_module.py:498-503, added at 657)
  V_BETA,      // beta                (405-416)
  V_NU,        // nu                  (418-429)
  V_GAMMA,     // gamma               (439-447)
  V_KAPPA,     // kappa               (469-474)
  V_OMEGA,     // omega               (480-485)
  V_IB,        // i_b                 (344-357)
  V_OB,        // o_b                 (382-396)
  V_OUTS,      // output affine scale (BN after the circuit, hgru_pose.py:82-90; 1 standalone)
  V_OUTT,      // output affine shift
  V_COUNT
};

}  // namespace mp
