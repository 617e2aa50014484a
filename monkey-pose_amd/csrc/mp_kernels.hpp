// Launcher declarations shared by the kernel translation units and the C-ABI layer.
#pragma once
#include "mp_common.hpp"
#include "../../include/monkeypose.h"

namespace mp {

constexpr int TH = 16, TW = 32;   // conv64 output tile (pixels) per 256-thread block
enum Epi { EPI_BB = 0, EPI_HGRU_A = 1, EPI_HGRU_B = 2 };

struct ConvArgs {
  const float* src;       // conv input, C8
  const f32x4* wpk;       // packed conv weights [q][tap][n][lane]
  float* dst;             // BB: output C8; A: I (C8); B: O' (C8, in place over O)
  // backbone epilogue
  const float* bias;      // [64]
  const float* bn_s;      // [64]
  const float* bn_t;      // [64]
  // hGRU epilogues
  const float* X;         // A: feed-forward drive (C8)
  const float* O;         // A, B: current output state (C8)
  const float* I;         // B: I (C8) (also the conv input)
  const float* vecs;      // [V_COUNT][64]
  const f32x4* gpk_or;    // B: packed o_r
  const f32x4* gpk_ir;    // B: packed i_r (next step's input gate)
  float* dst2;            // B mode 0: Og' (C8);  mode 1: affine(O') NHWC;  mode 2: its f16 hi plane
  float* dst3;            // B mode 2 (FFT path): the f16 lo plane of affine(O') NHWC (null: hi only)
  float rho;              // B: rho[t]
  int mode;               // B: 0 = next-step gate, 1 = final step, 2 = final step as fc_1's split planes
  int H, W, tiles_x, tiles_y;
  float ascale;           // f16x3 kernel: activation split scale (0 = the hGRU default 2^10)
  int dst_bf16;           // BB: dst is a bf16 C8 map (MP_DTYPE_BF16's hGRU drive X)
  int dst_c4;             // BB: dst is a C4 map (the FFT loop's drive X, k_fft.hip FFT_C4 bit 3)
  int o_nhwc;             // four-step row A / B (fp32): O is the NHWC fp32 initial state O0 (step 0)
};

// k_conv64.hip
hipError_t launch_conv64(int ks, int epi, ConvArgs a, int B, hipStream_t st);
hipError_t launch_gate_init(const float* O0, float* O, float* Og, const f32x4* gpk_ir, const float* vecs,
                            int B, int H, int W, hipStream_t st);
hipError_t launch_conv1_pool_bn(const float* in, const float* w, const float* bias, const float* s,
                                const float* t, float* out, int B, int Hin, int Win, hipStream_t st,
                                bool nhwc = false);
// 1-channel 3x3 SAME conv + relu + 2x2/2 max pool for Cout % 4 == 0, NHWC output view (ldo, coff)
hipError_t launch_conv1_pool_any(const float* in, const float* w, const float* bias, float* out, int ldo, int coff,
                                 int B, int Hin, int Win, int Cout, hipStream_t st);
// bf: the C8 side is a bf16 map
hipError_t launch_nhwc_to_c8(const float* in, float* out, int B, int H, int W, hipStream_t st, bool bf = false,
                             bool c4 = false);
// c4: the source is a C4 map (mp_common.hpp c4_index: the FFT loop's I, fft_c4_maps())
hipError_t launch_c8_to_nhwc(const float* in, float* out, int B, int H, int W, hipStream_t st, bool bf = false,
                             size_t dst_img = 0, bool c4 = false);
hipError_t launch_pack_conv64(const float* w, f32x4* out, int ks, hipStream_t st);
hipError_t launch_pack_gate(const float* g, f32x4* out, hipStream_t st);
// k_conv64x3.hip (fp32-accurate split-f16 MFMA path)
constexpr int TH3 = 32;
// nprod = 1: one f16 product per MAC (EPI_BB only; MP_DTYPE_BF16's backbone)
hipError_t launch_conv64x3(int ks, int epi, ConvArgs a, const void* wpk, float unscale, int B, hipStream_t st,
                           int nprod = 3);
hipError_t launch_pack_conv64x3(const float* w, void* out, int ks, float wscale, hipStream_t st);
// k_fft.hip (FFT path of the association-field conv, MP_DTYPE_F32_FFT; maps up to 64x64)
constexpr int FFT_MAX_HW = 64;
hipError_t device_absmax(const float* x, size_t n, float* out);   // max |x| (synchronous)
// MP_DTYPE_BF16 keeps the hGRU state maps O, I, Og, P2 in bf16 (MP_BF16_MAPS=0: fp32, for A/B);
// their element offsets are unchanged, so a map pointer offset by m elements is (bf16*)base + m
bool fft_bf16_maps();
bool fft_c4_drive();  // the FFT loop's X map is C4 (k_fft.hip FFT_C4 bit 3)
bool fft_c4_state();  // the FFT loop's O map is C4 (k_fft.hip FFT_C4 bit 2)
bool fft_c4_maps();   // the FFT loop's I map is C4 (k_fft.hip FFT_C4)
size_t fft_spec_bytes(int B);      // one spectrum buffer (S or Y) for B images
size_t fft_weight_bytes();         // expanded split spectral weights
// HWIO [ks][ks][64][64] -> packed split spectral weights (synchronous, finalize time)
// cls_major: the four-step loop's class-major frequency order (k_fft4.hip)
hipError_t build_spec_weights(const float* w, int ks, void* Gx, float* unscale, bool bf = false, bool cls_major = false);
hipError_t launch_fft_fwd(const float* act, void* S, int B, int H, int W, hipStream_t st, bool bf = false);
hipError_t launch_spec_gemm(const void* S, const void* Gx, void* Y, int B, float unscale, hipStream_t st,
                            bool bf = false);
hipError_t launch_fft_inv(const void* Y, float* P, int B, int H, int W, hipStream_t st, bool bf = false);
// P1 = IFFT(Y); I = A-epilogue(P1) -> a.dst; S = FFT(I)   (the A half-step tail + B half-step head)
hipError_t launch_fft_inv_a_fwd(const void* Y, const ConvArgs& a, void* S, int B, hipStream_t st, bool bf = false);
// B epilogue with f16x3 gate GEMMs (FFT path); gate weights packed by pack_gate_x3 (synchronous)
size_t gate_x3_bytes();
hipError_t pack_gate_x3(const float* g, void* out, float* unscale, bool bf = false);
hipError_t launch_gate_init_x3(const float* O0, float* O, float* Og, const void* ir_x3, float ir_us, const float* vecs,
                               int B, int H, int W, hipStream_t st, bool bf = false);
hipError_t launch_spec_epi_b(const ConvArgs& a, const float* P, const void* or_x3, float or_us, const void* ir_x3,
                             float ir_us, int B, hipStream_t st, bool bf = false);
// k_fft4.hip: the fp32 FFT path's four-step loop (MP_FFT4, default on).  One spectrum-sized buffer Z
// carries the partial transforms; per timestep col -> row(A) -> col -> row(B | FINAL), after one
// row(INIT) per forward.  Row modes: 0 = A (a.X, a.O -> a.dst = I), 1 = B (a.I, a.O -> a.dst = O'),
// 2 = the last B (O' and BN_3(O') to a.dst2 / a.dst3 per a.mode), 3 = INIT (O0 NHWC -> a.dst = O).
bool fft4_enabled();
// bf: MP_DTYPE_BF16 (bf16 Z, maps and spectral / gate products; class-major bf16 weights)
// ntot: the forward's whole batch -- its cache policy: at most 32 images fit the Infinity Cache (Z and
// the maps accessed with the default policy); from 128 on the maps are streamed non-temporal too
hipError_t launch_col_gemm(void* Z, const void* Gc, int B, float unscale, hipStream_t st, bool bf = false,
                           int ntot = 1 << 30);
hipError_t launch_row(int mode, void* Z, const ConvArgs& a, const void* or_x3, float or_us, const void* ir_x3,
                      float ir_us, const float* O0, int B, hipStream_t st, bool bf = false, int ntot = 1 << 30);
// k_igemm.hip (dense / hierarchical regressors)
struct IgemmArgs {
  const float* x;      // input view: pixel (n,y,x) channel ci at x[((n*H+y)*W+x)*ldx + cix + ci]
  int ldx, cix;
  int N, H, W, Cin;
  const f32x4* wpk;    // HWIO filter as [K][Cout], packed like an FC weight
  int K;               // KS*KS*Cin
  const float* bias;
  float* out;          // output view: out[(pixel)*ldo + coff + co]
  int ldo, coff, Cout;
  int Ho, Wo, KS, stride, pad_t, pad_l;
  int relu;
  int pmajor;          // wide f16x3 kernel only: M ordered position-major (m = pos * N + n), each
                       // block's K loop skips the taps that are padding for all of its positions
  float* part = nullptr;   // position-major split-K workspace (igemm_pm_splits(a) x M x Cout32
                           // floats, caller-owned); null: no split
  int nprod = 3;           // f16 split kernels: 3 = fp32-accurate f16x3, 1 = hi x hi only (bf16 dtype)
  int xcd = 0;             // set by the launcher: XCD-aware tile order (k_igemm.hip xcd_tile)
  const void* wpad = nullptr;   // halo path for Cin % 32 != 0: the same weights packed with every
  int cinp = 0;                 // tap's Cin rows zero-padded to cinp (% 32 == 0; launch_pack_cin_pad)
  int pool = 0;            // 1: a 2x2/2 max pool of relu(conv) is fused into the epilogue, and the
                           // output view (out, ldo, coff) is the pooled (Ho/2 x Wo/2) map;
                           // only where igemm_can_pool(a) holds
};
// whether launch_igemm_x3 can fuse the conv's 2x2 max pool (the halo and the split-K position-major
// paths, even output sizes, relu on)
bool igemm_can_pool(const IgemmArgs& a);
// input-channel splits of the position-major tap-skipping path for this conv (1 = none); a property
// of the layer alone (never of the batch), so every crop's sums group the same way at any batch
int igemm_pm_splits(const IgemmArgs& a);
size_t igemm_pm_part_floats(const IgemmArgs& a);
hipError_t launch_igemm_conv(const IgemmArgs& a, hipStream_t st);
// f16x3 (fp32-accurate) variant; wpk packed by launch_pack_fc_x3 as a [K][Cout] matrix
hipError_t launch_igemm_x3(const IgemmArgs& a, const void* wpk, float unscale, hipStream_t st);
hipError_t launch_pool2(const float* x, int ldx, int cix, int N, int H, int W, int C, float* out, int ldo,
                        int coff, int mode, hipStream_t st, const float* aff_s = nullptr,
                        const float* aff_t = nullptr);
// k_fc.hip
hipError_t launch_pack_fc(const float* W, f32x4* out, int K, int N, hipStream_t st);
int fc_choose_splits(int M, int K, int N, int* kslice);
hipError_t launch_fc_gemm(const float* A, int lda, const f32x4* Wpk, float* part, int M, int K, int N, int S,
                          int kslice, hipStream_t st);
// f16x3 (fp32-accurate) fc GEMM, same slabs / splits as launch_fc_gemm; nprod = 1: the hi x hi
// product only (single f16 MFMA, hi weight planes only -- MP_DTYPE_BF16's fc_1)
size_t fc_x3_bytes(int K, int N);
hipError_t launch_pack_fc_x3(const float* W, void* out, int K, int N, float* unscale, hipStream_t st);
// HWIO [taps][Cin][Cout] -> [taps][cinp][Cout] with zero rows ci >= Cin (fp32, device)
hipError_t launch_pad_cin(const float* w, float* out, int taps, int Cin, int cinp, int Cout, hipStream_t st);
hipError_t launch_fc_gemm_x3(const float* A, int lda, const void* Wpk, float unscale, float* part, int M, int K,
                             int N, int S, int kslice, hipStream_t st, int nprod = 3);
// the same GEMM on activations already split into f16 hi / lo planes [M][lda] (Al unused when
// nprod = 1): bit-identical partial sums, no conversion in the K loop (LDS-DMA staging)
hipError_t launch_fc_gemm_x3p(const void* Ah, const void* Al, int lda, const void* Wpk, float unscale, float* part,
                              int M, int K, int N, int S, int kslice, hipStream_t st, int nprod = 3);
// k_frame.hip (frame -> CoM -> crop chain)
hipError_t launch_resize_bilinear(const float* x, int N, int H, int W, int C, float* out, int Ho, int Wo,
                                  hipStream_t st);
hipError_t launch_hidden_uniform(float* out, int64_t n, uint64_t seed, double limit, hipStream_t st);
hipError_t launch_crop3d(const mp_camera& cam, const float* frames, int N, int H, int W, float frame_scale,
                         const float* com_norm, const double com_scale[3], int dsz, float* patches, double* Ms,
                         double* coms_out, int32_t* status, hipStream_t st, bool docom = false);
hipError_t launch_fc_reduce(const float* part, int S, int M, int N, const float* bias, int relu,
                            const float* aff_s, const float* aff_t, float* out, int ldo, hipStream_t st);

}  // namespace mp
