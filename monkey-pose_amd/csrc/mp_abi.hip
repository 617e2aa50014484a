// C ABI of libmonkeypose.so (declared in include/monkeypose.h): contexts, weight registry,
// finalize (BN folding + fragment packing) and the forward orchestration of the hot path.
//
// Forward of hgru_pose.model.build (hgru_pose.py:47-105) as launched here, one stream, no host
// synchronisation:
//   conv1_pool_bn            conv_1 + relu + max_pool + BN            (50-60)     HBM-bound
//   conv64<3,BB>  x2         conv_2 / conv_3 + relu + BN              (61-80)     MFMA fp32
//   gate_init                O0 -> O, O0*sigmoid(O0.i_r+i_b)          hgru_module.py:696-711
//   T x { conv64<15,A>, conv64<15,B> }  the hGRU half-steps         hgru_module.py:825-857
//                            (last B also applies BN_3, writes NHWC) (82-90)
//   fc_gemm + fc_reduce      fc_1 + relu + BN_4                       (91-103)
//   fc_gemm + fc_reduce      fc_out                                   (104-105)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/monkeypose.h"

#include "mp_runtime.hpp"


using namespace mp;

namespace mpr {
thread_local std::string g_err;
}


namespace mpr {

void upload(DevBuf& d, const std::vector<float>& h) {
  d.alloc(h.size() * sizeof(float));
  hip_check(hipMemcpy(d.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy H2D");
}

void bn_fold(mp_ctx* c, const std::string& scope, int n, DevBuf& s_out, DevBuf& t_out, std::vector<float>* hs,
             std::vector<float>* ht) {
  const auto& g = c->need(scope + "/gamma", {n}).host;
  const auto& b = c->need(scope + "/beta", {n}).host;
  const auto& m = c->need(scope + "/moving_mean", {n}).host;
  const auto& v = c->need(scope + "/moving_variance", {n}).host;
  std::vector<float> s(n), t(n);
  for (int i = 0; i < n; ++i) {
    // inference BN: gamma * (x - mean) / sqrt(var + eps) + beta, eps = 1e-5 (hgru_pose.py:17)
    const double sc = (double)g[i] / std::sqrt((double)v[i] + 1e-5);
    s[i] = (float)sc;
    t[i] = (float)((double)b[i] - (double)m[i] * sc);
  }
  upload(s_out, s);
  upload(t_out, t);
  if (hs) *hs = s;
  if (ht) *ht = t;
}

}  // namespace mpr

namespace {

void copy_dev(DevBuf& d, const RawWeight& w) {
  d.alloc(w.numel() * sizeof(float));
  hip_check(hipMemcpy(d.p, w.dev->p, w.numel() * sizeof(float), hipMemcpyDeviceToDevice), "hipMemcpy D2D");
}

std::vector<float> vec64(mp_ctx* c, const std::string& n) {
  return c->need("contextual_circuit/" + n, {1, 1, 1, 64}).host;
}

// backbone activations (BN outputs) are not tanh-bounded like the hGRU maps: split them at 2^4
constexpr float BB_ASCALE = 16.0f;

// HWIO [ks][ks][64][64] -> f16x3 fragments with a power-of-two scale putting max|w| at 2^13..2^14
void pack_x3(const RawWeight& w, DevBuf& out, int ks, float ascale, float* unscale, const char* what) {
  float mx = 0.f;
  hip_check(device_absmax(w.dev->f(), w.numel(), &mx), what);
  int e = 0;
  if (mx > 0.f) std::frexp(mx, &e);
  const float wscale = std::ldexp(1.0f, 14 - e);
  *unscale = 1.0f / (wscale * ascale);
  hip_check(launch_pack_conv64x3(w.dev->f(), out.p, ks, wscale, nullptr), what);
}

void finalize_circuit(mp_ctx* c, const std::vector<float>* outs, const std::vector<float>* outt) {
  auto it = c->raw.find("contextual_circuit/p_r");
  if (it == c->raw.end()) fail(MP_ERR_STATE, "weight not set: contextual_circuit/p_r");
  const auto& ps = it->second.shape;
  if (ps.size() != 4 || ps[0] != ps[1] || ps[2] != 64 || ps[3] != 64 ||
      !(ps[0] == 3 || ps[0] == 5 || ps[0] == 15))
    fail(MP_ERR_WEIGHT, "contextual_circuit/p_r must be [S,S,64,64] with S in {3,5,15}");
  c->ssf = (int)ps[0];
  c->p_pk.alloc((size_t)8 * c->ssf * c->ssf * 2 * 64 * 16);
  c->fft4 = false;
  if (c->dtype == MP_DTYPE_F32_SPLIT) {
    pack_x3(it->second, c->p_pk, c->ssf, 1024.0f, &c->p_unscale, "pack p_r (f16x3)");
  } else if (is_fft(c->dtype)) {
    const bool bf = c->dtype == MP_DTYPE_BF16;
    c->spec_g.alloc(fft_weight_bytes());
    c->fft4 = fft4_enabled() && (c->dtype == MP_DTYPE_F32_FFT || (bf && fft_bf16_maps()));
    hip_check(build_spec_weights(it->second.dev->f(), c->ssf, c->spec_g.p, &c->p_unscale, bf, c->fft4), "p_r spectrum");
    c->or_x3.alloc(gate_x3_bytes());
    c->ir_x3.alloc(gate_x3_bytes());
    hip_check(pack_gate_x3(c->need("contextual_circuit/o_r", {1, 1, 64, 64}).dev->f(), c->or_x3.p, &c->or_us, bf),
              "pack o_r");
    hip_check(pack_gate_x3(c->need("contextual_circuit/i_r", {1, 1, 64, 64}).dev->f(), c->ir_x3.p, &c->ir_us, bf),
              "pack i_r");
  } else {
    hip_check(launch_pack_conv64(it->second.dev->f(), c->p_pk.v4(), c->ssf, nullptr), "pack p_r");
  }
  c->ir_pk.alloc(1024 * 16);
  c->or_pk.alloc(1024 * 16);
  hip_check(launch_pack_gate(c->need("contextual_circuit/i_r", {1, 1, 64, 64}).dev->f(), c->ir_pk.v4(), nullptr),
            "pack i_r");
  hip_check(launch_pack_gate(c->need("contextual_circuit/o_r", {1, 1, 64, 64}).dev->f(), c->or_pk.v4(), nullptr),
            "pack o_r");
  std::vector<float> v(V_COUNT * 64);
  const char* order[] = {"lateral_bias", "beta", "nu", "gamma", "kappa", "omega", "i_b", "o_b"};
  for (int k = 0; k < 8; ++k) {
    auto x = vec64(c, order[k]);
    std::copy(x.begin(), x.end(), v.begin() + k * 64);
  }
  for (int i = 0; i < 64; ++i) {
    v[V_OUTS * 64 + i] = outs ? (*outs)[i] : 1.f;
    v[V_OUTT * 64 + i] = outt ? (*outt)[i] : 0.f;
  }
  upload(c->vecs, v);
  auto rt = c->raw.find("contextual_circuit/rho");
  if (rt == c->raw.end() || rt->second.shape.size() != 1 || rt->second.shape[0] < 1)
    fail(MP_ERR_WEIGHT, "contextual_circuit/rho must be set with shape [timesteps]");
  c->rho = rt->second.host;
  c->timesteps = (int)c->rho.size();
}

void finalize_pose(mp_ctx* c) {
  const int k = 64;
  copy_dev(c->conv1_w, c->need("conv_1/conv_1_filters", {3, 3, 1, k}));
  copy_dev(c->conv1_b, c->need("conv_1/conv_1_biases", {k}));
  // conv_1 as a generic implicit-GEMM weight, for the pre-pool conv1 tap only (mp_pose_taps)
  c->conv1_ig.alloc((size_t)((9 + 7) / 8) * ((k + 31) / 32) * 64 * 16);
  hip_check(launch_pack_fc(c->conv1_w.f(), c->conv1_ig.v4(), 9, k, nullptr), "pack conv_1 tap");
  bn_fold(c, "batch_normalization", k, c->bn0_s, c->bn0_t);
  if (c->dtype == MP_DTYPE_F32) {
    c->conv2_pk.alloc((size_t)8 * 9 * 2 * 64 * 16);
    c->conv3_pk.alloc((size_t)8 * 9 * 2 * 64 * 16);
    hip_check(launch_pack_conv64(c->need("conv_2/conv_2_filters", {3, 3, k, k}).dev->f(), c->conv2_pk.v4(), 3, nullptr),
              "pack conv_2");
    hip_check(launch_pack_conv64(c->need("conv_3/conv_3_filters", {3, 3, k, k}).dev->f(), c->conv3_pk.v4(), 3, nullptr),
              "pack conv_3");
  } else {   // fp32-accurate f16x3 backbone convs (k_conv64x3.hip, BB epilogue)
    c->conv2_pk.alloc((size_t)8 * 9 * 2 * 64 * 16);
    c->conv3_pk.alloc((size_t)8 * 9 * 2 * 64 * 16);
    pack_x3(c->need("conv_2/conv_2_filters", {3, 3, k, k}), c->conv2_pk, 3, BB_ASCALE, &c->conv2_us, "pack conv_2");
    pack_x3(c->need("conv_3/conv_3_filters", {3, 3, k, k}), c->conv3_pk, 3, BB_ASCALE, &c->conv3_us, "pack conv_3");
  }
  copy_dev(c->conv2_b, c->need("conv_2/conv_2_biases", {k}));
  copy_dev(c->conv3_b, c->need("conv_3/conv_3_biases", {k}));
  bn_fold(c, "batch_normalization_1", k, c->bn1_s, c->bn1_t);
  bn_fold(c, "batch_normalization_2", k, c->bn2_s, c->bn2_t);
  DevBuf s3, t3;
  std::vector<float> hs3, ht3;
  bn_fold(c, "batch_normalization_3", k, s3, t3, &hs3, &ht3);
  finalize_circuit(c, &hs3, &ht3);

  auto f1 = c->raw.find("fc_1/fc_1_weights");
  if (f1 == c->raw.end()) fail(MP_ERR_STATE, "weight not set: fc_1/fc_1_weights");
  if (f1->second.shape.size() != 2 || f1->second.shape[0] % 64 != 0)
    fail(MP_ERR_WEIGHT, "fc_1/fc_1_weights must be [H*W*64, N]");
  c->fc1_in = (int)f1->second.shape[0];
  c->fc1_out = (int)f1->second.shape[1];
  const int K8 = (c->fc1_in + 7) / 8, N32 = (c->fc1_out + 31) / 32;
  if (c->dtype == MP_DTYPE_F32) {
    c->fc1_pk.alloc((size_t)K8 * N32 * 64 * 16);
    hip_check(launch_pack_fc(f1->second.dev->f(), c->fc1_pk.v4(), c->fc1_in, c->fc1_out, nullptr), "pack fc_1");
  } else {   // fp32-accurate f16x3 (same slabs, same batch invariance)
    c->fc1_pk.alloc(fc_x3_bytes(c->fc1_in, c->fc1_out));
    hip_check(launch_pack_fc_x3(f1->second.dev->f(), c->fc1_pk.p, c->fc1_in, c->fc1_out, &c->fc1_unscale, nullptr),
              "pack fc_1 (f16x3)");
  }
  copy_dev(c->fc1_b, c->need("fc_1/fc_1_biases", {c->fc1_out}));
  bn_fold(c, "batch_normalization_4", c->fc1_out, c->bn4_s, c->bn4_t);
  auto fo = c->raw.find("fc_out/fc_out_weights");
  if (fo == c->raw.end()) fail(MP_ERR_STATE, "weight not set: fc_out/fc_out_weights");
  if (fo->second.shape.size() != 2 || fo->second.shape[0] != c->fc1_out)
    fail(MP_ERR_WEIGHT, "fc_out/fc_out_weights must be [fc_1 out, output_shape]");
  c->nout = (int)fo->second.shape[1];
  const int K8o = (c->fc1_out + 7) / 8, N32o = (c->nout + 31) / 32;
  c->fco_pk.alloc((size_t)K8o * N32o * 64 * 16);
  hip_check(launch_pack_fc(fo->second.dev->f(), c->fco_pk.v4(), c->fc1_out, c->nout, nullptr), "pack fc_out");
  copy_dev(c->fco_b, c->need("fc_out/fc_out_biases", {c->nout}));
}

void ensure_ws(mp_ctx* c, int64_t n, int64_t H, int64_t W) {
  const int64_t px = n * H * W;
  if (n <= c->cap_batch && H * W <= c->cap_hw) return;
  const int64_t nb = std::max(n, c->cap_batch), hw = std::max(H * W, c->cap_hw);
  const size_t st = (size_t)nb * hw * 64 * sizeof(float);
  c->X.alloc(st);
  c->O.alloc(st);
  c->I.alloc(st);
  // the four-step loop (k_fft4.hip) keeps the gated state and P1 / P2 on chip and updates one
  // spectrum-sized buffer Z (specS) in place: Og, specY and specP are six-launch-loop buffers only
  if (!c->fft4) c->Og.alloc(st);
  if (is_fft(c->dtype)) {
    c->specS.alloc(fft_spec_bytes((int)nb));
    if (!c->fft4) {
      c->specY.alloc(fft_spec_bytes((int)nb));
      c->specP.alloc(st);
    }
  }
  if (c->model == MP_MODEL_HGRU_POSE) {
    c->bufA.alloc(st);
    c->bufB.alloc(st);
    c->fcin.alloc(st);
    int ks;
    const int S = fc_choose_splits((int)nb, c->fc1_in, c->fc1_out, &ks);
    const size_t p1 = (size_t)S * nb * ((c->fc1_out + 31) / 32 * 32) * sizeof(float);
    const int S2 = fc_choose_splits((int)nb, c->fc1_out, c->nout, &ks);
    const size_t p2 = (size_t)S2 * nb * ((c->nout + 31) / 32 * 32) * sizeof(float);
    c->part.alloc(std::max(p1, p2));
    c->part2.alloc(p2);
    c->h1.alloc((size_t)nb * c->fc1_out * sizeof(float));
  }
  (void)px;
  c->cap_batch = nb;
  c->cap_hw = hw;
}


// MP_DTYPE_BF16 keeps the FFT loop's maps (X, O, I, Og, P2) in bf16 (k_fft.hip map_ld4)
bool bf16_maps(const mp_ctx* c) { return c->dtype == MP_DTYPE_BF16 && fft_bf16_maps(); }

// the drive X of an FFT-path context is a C4 map (k_fft.hip FFT_C4 bit 3)
bool x_c4(const mp_ctx* c) { return is_fft(c->dtype) && fft_c4_drive(); }

// one association-field conv p_r * a.src with its fused hGRU epilogue, in the context's precision
void eCRF_conv(mp_ctx* c, int epi, const ConvArgs& a, int n, hipStream_t st) {
  if (c->dtype == MP_DTYPE_F32_SPLIT)
    hip_check(launch_conv64x3(c->ssf, epi, a, c->p_pk.p, c->p_unscale, n, st), "conv15 (f16x3)");
  else
    hip_check(launch_conv64(c->ssf, epi, a, n, st), "conv15");
}

// FFT path of one hGRU step (k_fft.hip): the A half-step's inverse transform, its epilogue and the
// B half-step's forward transform are one kernel, so per step:
//   fft_fwd(Og) -> S;  spec_gemm -> Y;  inv_a_fwd: I = A-epi(IFFT(Y)), S = FFT(I);
//   spec_gemm -> Y;  fft_inv -> P2;  epi_b(P2, I, O) -> O', Og'
void fft_step(mp_ctx* c, const ConvArgs& a, const ConvArgs& b, int n, hipStream_t st) {
  const bool bf = c->dtype == MP_DTYPE_BF16;
  {
    ProfScope pa(c, st, "conv15_a");
    {
      ProfScope ps(c, st, "fft_fwd");
      hip_check(launch_fft_fwd(a.src, c->specS.p, n, a.H, a.W, st, bf), "fft_fwd");
    }
    {
      ProfScope ps(c, st, "spec_gemm");
      hip_check(launch_spec_gemm(c->specS.p, c->spec_g.p, c->specY.p, n, c->p_unscale, st, bf), "spec_gemm");
    }
    ProfScope ps(c, st, "inv_a_fwd");
    hip_check(launch_fft_inv_a_fwd(c->specY.p, a, c->specS.p, n, st, bf), "fft_inv_a_fwd");
  }
  ProfScope pb(c, st, "conv15_b");
  {
    ProfScope ps(c, st, "spec_gemm");
    hip_check(launch_spec_gemm(c->specS.p, c->spec_g.p, c->specY.p, n, c->p_unscale, st, bf), "spec_gemm");
  }
  {
    ProfScope ps(c, st, "fft_inv");
    hip_check(launch_fft_inv(c->specY.p, c->specP.f(), n, b.H, b.W, st, bf), "fft_inv");
  }
  ProfScope ps(c, st, "epi_b");
  hip_check(launch_spec_epi_b(b, c->specP.f(), c->or_x3.p, c->or_us, c->ir_x3.p, c->ir_us, n, st, bf), "B epilogue");
}

// map-size rule of the context's association-field conv path (MP_ERR_SHAPE otherwise)
void check_map(mp_ctx* c, int64_t H, int64_t W, const char* what) {
  if (is_fft(c->dtype)) {
    if (H < 1 || H > FFT_MAX_HW || (W != 32 && W != 64))
      fail(MP_ERR_SHAPE, std::string(what) + ": the FFT path needs map height in [1, 64] and width 32 or 64");
    return;
  }
  const int th = c->dtype == MP_DTYPE_F32_SPLIT ? TH3 : TH;
  if (H % th || W % TW)
    fail(MP_ERR_SHAPE, std::string(what) + ": map height must be a multiple of " + std::to_string(th) +
                           " and width a multiple of 32");
}

// per-step state outputs (store_states, hgru_module.py:889-915): [batch][T][H][W][64] NHWC fp32,
// O_t after the rho gain and I_t of each step; NULL = not wanted
struct StateOut {
  float* O = nullptr;
  float* I = nullptr;
  int T = 0;
};

// copy step t's O / I maps (C8, bf16 under MP_DTYPE_BF16 maps; ic4: I is the FFT loop's C4 map) of images
// [b0, b0 + n) into the stacks
void store_step(const StateOut* so, const float* Omap, const float* Imap, int b0, int n, int H, int W, int t,
                bool bf, hipStream_t st, bool ic4 = false, bool oc4 = false) {
  if (!so) return;
  const size_t img = (size_t)H * W * 64, stride = img * so->T;
  const size_t off = (size_t)b0 * stride + (size_t)t * img;
  if (so->O) hip_check(launch_c8_to_nhwc(Omap, so->O + off, n, H, W, st, bf, stride, oc4), "store_states O");
  if (so->I) hip_check(launch_c8_to_nhwc(Imap, so->I + off, n, H, W, st, bf, stride, ic4), "store_states I");
}

// fc_1's pre-split activation planes (FFT path, k_fc.hip launch_fc_gemm_x3p): the last B epilogue
// writes the BN'd NHWC output as f16 hi (and, for the three-product fc_1, lo) planes [batch][K]
struct SplitOut {
  _Float16* hi = nullptr;
  _Float16* lo = nullptr;   // null: hi plane only (dtype bf16's one-product fc_1)
};

// final-step output arguments of the B epilogue for images from b0 on: NHWC fp32 (mode 1) or the
// split planes (mode 2)
void final_out(ConvArgs& b, float* final_dst2, const SplitOut* sp, int b0, int H, int W) {
  const size_t m = (size_t)b0 * 64 * H * W;
  if (sp) {
    b.mode = 2;
    b.dst2 = reinterpret_cast<float*>(sp->hi + m);
    b.dst3 = sp->lo ? reinterpret_cast<float*>(sp->lo + m) : nullptr;
  } else {
    b.mode = 1;
    b.dst2 = final_dst2 + m;
  }
}

// the hGRU loop of images [b0, b0 + n) on stream st (FFT path), all state pointers offset
void fft_circuit_range(mp_ctx* c, int b0, int n, int H, int W, int T, float* final_dst2, const StateOut* so,
                       const SplitOut* sp, hipStream_t st) {
  const size_t m = (size_t)b0 * 64 * H * W;              // elements per image of a C8 / NHWC map
  void* S = static_cast<char*>(c->specS.p) + fft_spec_bytes(b0);
  void* Y = static_cast<char*>(c->specY.p) + fft_spec_bytes(b0);
  // maps X, O, I, Og, P2 (bf16 under MP_DTYPE_BF16, k_fft.hip map_ld4): the same element offset,
  // in units of their element type; the NHWC output stays fp32
  const bool bm = bf16_maps(c);
  auto map = [&](DevBuf& buf) { return bm ? reinterpret_cast<float*>(reinterpret_cast<uint16_t*>(buf.p) + m) : buf.f() + m; };
  float* P = map(c->specP);
  for (int t = 0; t < T; ++t) {
    ConvArgs a{};
    a.H = H;
    a.W = W;
    a.src = map(c->Og);
    a.dst = map(c->I);
    a.X = map(c->X);
    a.O = map(c->O);
    a.vecs = c->vecs.f();
    ConvArgs b{};
    b.H = H;
    b.W = W;
    b.dst = map(c->O);
    b.O = map(c->O);
    b.I = map(c->I);
    b.vecs = c->vecs.f();
    b.rho = c->rho[t];
    b.mode = 0;
    b.dst2 = map(c->Og);
    if (t == T - 1) final_out(b, final_dst2, sp, b0, H, W);
    const bool bf = c->dtype == MP_DTYPE_BF16;
    hip_check(launch_fft_fwd(a.src, S, n, H, W, st, bf), "fft_fwd");
    hip_check(launch_spec_gemm(S, c->spec_g.p, Y, n, c->p_unscale, st, bf), "spec_gemm");
    hip_check(launch_fft_inv_a_fwd(Y, a, S, n, st, bf), "fft_inv_a_fwd");
    hip_check(launch_spec_gemm(S, c->spec_g.p, Y, n, c->p_unscale, st, bf), "spec_gemm");
    hip_check(launch_fft_inv(Y, P, n, H, W, st, bf), "fft_inv");
    hip_check(launch_spec_epi_b(b, P, c->or_x3.p, c->or_us, c->ir_x3.p, c->ir_us, n, st, bf), "B epilogue");
    store_step(so, b.O, b.I, b0, n, H, W, t, bm, st, fft_c4_maps(), fft_c4_state());
  }
}

// MP_O0_DIRECT (default 1): the fp32 four-step loop's first step reads O0 (NHWC) directly; 0: row(INIT)
// copies it into the C8 state map first (1 MB per image more)
bool o0_direct() {
  static const bool v = [] {
    const char* e = std::getenv("MP_O0_DIRECT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// the hGRU loop of images [b0, b0 + n) on stream st, four-step FFT path (k_fft4.hip): one row(INIT)
// (hgru_module.py:696-711 on O0, and the forward transform of the gated state), then per timestep
//   col -> row A (I = tanh(X - (beta O + nu) P1), hgru_module.py:797-799) -> col -> row B (O', the
//   next gated state; the last step: O' and BN_3(O_T))
// every launch in place on one spectrum-sized buffer Z
// ntot: the forward's whole batch (its cache policy: k_fft4.hip col8_znt, row8_znt, map_nt)
void fft4_circuit_range(mp_ctx* c, int b0, int n, int ntot, int H, int W, int T, const float* o0_nhwc,
                        float* final_dst2, const StateOut* so, const SplitOut* sp, hipStream_t st) {
  const size_t m = (size_t)b0 * 64 * H * W;
  const bool bf = c->dtype == MP_DTYPE_BF16;   // bf16 Z (half a spectrum's bytes per image) and maps
  void* Z = static_cast<char*>(c->specS.p) + fft_spec_bytes(b0) / (bf ? 2 : 1);
  auto map = [&](DevBuf& buf) { return bf ? reinterpret_cast<float*>(reinterpret_cast<uint16_t*>(buf.p) + m) : buf.f() + m; };
  float* X = map(c->X);
  float* O = map(c->O);
  float* I = map(c->I);
  // fp32: step 0's row A / B read O0 itself (NHWC) instead of a C8 copy that row(INIT) would write
  const bool o0d = !bf && o0_direct();
  {
    ConvArgs a0{};
    a0.H = H;
    a0.W = W;
    a0.dst = o0d ? nullptr : O;
    a0.vecs = c->vecs.f();
    ProfScope pa(c, st, "conv15_a");
    ProfScope ps(c, st, "row_init");
    hip_check(launch_row(3, Z, a0, c->or_x3.p, c->or_us, c->ir_x3.p, c->ir_us, o0_nhwc + m, n, st, bf, ntot), "row_init");
  }
  for (int t = 0; t < T; ++t) {
    ConvArgs a{};
    a.H = H;
    a.W = W;
    a.X = X;
    a.O = O;
    a.dst = I;
    a.vecs = c->vecs.f();
    ConvArgs b{};
    b.H = H;
    b.W = W;
    b.I = I;
    b.O = O;
    b.dst = O;
    if (o0d && t == 0) {
      a.O = b.O = o0_nhwc + m;
      a.o_nhwc = b.o_nhwc = 1;
    }
    b.vecs = c->vecs.f();
    b.rho = c->rho[t];
    b.mode = 0;
    const bool last = t == T - 1;
    if (last) {
      final_out(b, final_dst2, sp, b0, H, W);
      if (!so) b.dst = nullptr;   // O_T is read by nothing but BN_3 (row FINAL): no C8 map write
    }
    {
      ProfScope pa(c, st, "conv15_a");
      {
        ProfScope ps(c, st, "col_gemm");
        hip_check(launch_col_gemm(Z, c->spec_g.p, n, c->p_unscale, st, bf, ntot), "col_gemm");
      }
      ProfScope ps(c, st, "row_a");
      hip_check(launch_row(0, Z, a, c->or_x3.p, c->or_us, c->ir_x3.p, c->ir_us, nullptr, n, st, bf, ntot), "row_a");
    }
    {
      ProfScope pb(c, st, "conv15_b");
      {
        ProfScope ps(c, st, "col_gemm");
        hip_check(launch_col_gemm(Z, c->spec_g.p, n, c->p_unscale, st, bf, ntot), "col_gemm");
      }
      ProfScope ps(c, st, last ? "row_final" : "row_b");
      hip_check(launch_row(last ? 2 : 1, Z, b, c->or_x3.p, c->or_us, c->ir_x3.p, c->ir_us, nullptr, n, st, bf, ntot),
                last ? "row_final" : "row_b");
    }
    store_step(so, O, I, b0, n, H, W, t, bf, st, fft_c4_maps(), fft_c4_state());
  }
}


// fc_1 on pre-split activation planes (MP_FC_PRESPLIT=0: the fp32 map + in-loop split, for A/B)
bool fc_presplit() {
  static const bool v = [] {
    const char* e = std::getenv("MP_FC_PRESPLIT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// MP_FC_SLICE (A/B, default 0): 1 runs the pose head (fc_1, its reduce + BN_4, fc_out) per hGRU batch
// slice on the slice's stream, right after that slice's loop, instead of once for the whole batch after
// the join.  Bit-identical, but each slice streams fc_1's 1.07 GB of weights: same box, B = 256 8.16 vs
// 7.97 ms, B = 64 2.60 vs 2.36 (profiles/r6/ab/ab_fc_slice.jsonl)
bool fc_slice() {
  static const bool v = [] {
    const char* e = std::getenv("MP_FC_SLICE");
    return e ? std::atoi(e) != 0 : false;
  }();
  return v;
}

int stream_count() {
  static const int v = [] {
    const char* e = std::getenv("MP_STREAMS");
    return e ? std::max(1, std::min(4, std::atoi(e))) : 2;
  }();
  return v;
}

// MP_BB_PIPE (default 1): the backbone per batch slice on the slice's stream; 0: whole batch first
bool bb_pipeline() {
  static const bool v = [] {
    const char* e = std::getenv("MP_BB_PIPE");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// MP_BB_STAGGER (default 1): a slice's backbone waits for the previous slice's, so that it overlaps that
// slice's hGRU loop instead of the other backbone (same box, B = 256: 8.40 -> 8.28 ms; profiles/r5n)
bool bb_stagger() {
  static const bool v = [] {
    const char* e = std::getenv("MP_BB_STAGGER");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// smallest batch slice worth a stream of its own (MP_SLICE_MIN, A/B knob)
int slice_min() {
  static const int v = [] {
    const char* e = std::getenv("MP_SLICE_MIN");
    return e ? std::max(1, std::atoi(e)) : 32;
  }();
  return v;
}

// pre (optional): work a batch slice needs before its hGRU loop (the backbone of its images), run on the
// slice's stream so that one slice's backbone overlaps another's loop
using SliceFn = std::function<void(int b0, int cnt, hipStream_t s)>;
// post (optional): work a batch slice does after its hGRU loop (the pose head on its rows), on the
// slice's stream, so that the first slice's head overlaps the last slice's loop
void run_circuit(mp_ctx* c, int64_t n, int H, int W, int T, const float* o0_nhwc, float* final_dst2,
                 const StateOut* so, hipStream_t st, const SplitOut* sp = nullptr, const SliceFn* pre = nullptr,
                 const SliceFn* post = nullptr) {
  if (sp && !is_fft(c->dtype)) fail(MP_ERR_STATE, "split fc_1 planes are an FFT-path output");
  // FFT path, not profiling: batch slices are independent, so they run on separate streams and
  // their latency-bound kernels overlap (the per-kernel HIP-event profile keeps one stream)
  const int ns = std::min<int>(stream_count(), (int)(n / slice_min()));
  const bool multi = is_fft(c->dtype) && !c->prof && ns >= 2;
  if (pre && !multi) (*pre)(0, (int)n, st);
  if (c->fft4 && !multi) {
    fft4_circuit_range(c, 0, (int)n, (int)n, H, W, T, o0_nhwc, final_dst2, so, sp, st);
    if (post) (*post)(0, (int)n, st);
    return;
  }
  if (multi) {
    if (!c->fft4)
      hip_check(launch_gate_init_x3(o0_nhwc, c->O.f(), c->Og.f(), c->ir_x3.p, c->ir_us, c->vecs.f(), (int)n, H, W,
                                  st, c->dtype == MP_DTYPE_BF16),
              "gate_init");
    while ((int)c->sides.size() < ns - 1) {
      hipStream_t s;
      hipEvent_t e;
      hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
      hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
      c->sides.push_back(s);
      c->ev_join.push_back(e);
    }
    if (!c->ev_fork) hip_check(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(c->ev_fork, st), "hipEventRecord");
    // slices of whole GEMM groups (32 images; MP_SLICE_MIN below 32 splits a group)
    const int gs = std::min(32, slice_min());
    const int groups = (int)(n + gs - 1) / gs;
    int b0 = 0;
    for (int k = 0; k < ns; ++k) {
      const int g = groups / ns + (k < groups % ns ? 1 : 0);
      const int cnt = std::min<int>(g * gs, (int)n - b0);
      hipStream_t s = k == 0 ? st : c->sides[k - 1];
      if (k > 0) hip_check(hipStreamWaitEvent(s, c->ev_fork, 0), "hipStreamWaitEvent");
      if (pre && bb_stagger() && k > 0) {   // slice k's backbone after slice k - 1's
        if (!c->ev_pre) hip_check(hipEventCreateWithFlags(&c->ev_pre, hipEventDisableTiming), "hipEventCreate");
        hip_check(hipStreamWaitEvent(s, c->ev_pre, 0), "hipStreamWaitEvent");
      }
      if (pre) (*pre)(b0, cnt, s);
      if (pre && bb_stagger() && k + 1 < ns) {
        if (!c->ev_pre) hip_check(hipEventCreateWithFlags(&c->ev_pre, hipEventDisableTiming), "hipEventCreate");
        hip_check(hipEventRecord(c->ev_pre, s), "hipEventRecord");
      }
      if (c->fft4)
        fft4_circuit_range(c, b0, cnt, (int)n, H, W, T, o0_nhwc, final_dst2, so, sp, s);
      else
        fft_circuit_range(c, b0, cnt, H, W, T, final_dst2, so, sp, s);
      if (post) (*post)(b0, cnt, s);
      b0 += cnt;
    }
    for (int k = 1; k < ns; ++k) {
      hip_check(hipEventRecord(c->ev_join[k - 1], c->sides[k - 1]), "hipEventRecord");
      hip_check(hipStreamWaitEvent(st, c->ev_join[k - 1], 0), "hipStreamWaitEvent");
    }
    return;
  }
  hip_check(is_fft(c->dtype)
                ? launch_gate_init_x3(o0_nhwc, c->O.f(), c->Og.f(), c->ir_x3.p, c->ir_us, c->vecs.f(), (int)n, H, W, st,
                                      c->dtype == MP_DTYPE_BF16)
                : launch_gate_init(o0_nhwc, c->O.f(), c->Og.f(), c->ir_pk.v4(), c->vecs.f(), (int)n, H, W, st),
            "gate_init");
  for (int t = 0; t < T; ++t) {
    ConvArgs a{};
    a.H = H;
    a.W = W;
    a.src = c->Og.f();
    a.wpk = c->p_pk.v4();
    a.dst = c->I.f();
    a.X = c->X.f();
    a.O = c->O.f();
    a.vecs = c->vecs.f();
    ConvArgs b{};
    b.H = H;
    b.W = W;
    b.src = c->I.f();
    b.wpk = c->p_pk.v4();
    b.dst = c->O.f();
    b.O = c->O.f();
    b.I = c->I.f();
    b.vecs = c->vecs.f();
    b.gpk_or = c->or_pk.v4();
    b.gpk_ir = c->ir_pk.v4();
    b.rho = c->rho[t];
    b.mode = 0;
    b.dst2 = c->Og.f();
    if (t == T - 1) final_out(b, final_dst2, sp, 0, H, W);
    if (is_fft(c->dtype)) {
      fft_step(c, a, b, (int)n, st);
    } else {
      {
        ProfScope ps(c, st, "conv15_a");
        eCRF_conv(c, EPI_HGRU_A, a, (int)n, st);
      }
      ProfScope ps(c, st, "conv15_b");
      eCRF_conv(c, EPI_HGRU_B, b, (int)n, st);
    }
    store_step(so, c->O.f(), c->I.f(), 0, (int)n, H, W, t, bf16_maps(c), st, is_fft(c->dtype) && fft_c4_maps(),
               is_fft(c->dtype) && fft_c4_state());
  }
  if (post) (*post)(0, (int)n, st);
}

// the initial output state for hidden_init (hgru_module.py:875-892) as an NHWC fp32 pointer:
// MP_HIDDEN_GIVEN -> the caller's o0; ZEROS -> a zeroed workspace map; IDENTITY -> X (the
// caller's NHWC x for the circuit, the C8 drive converted into a workspace map for the pose model)
const float* hidden_state(mp_ctx* c, int hidden_init, const float* o0, const float* x_nhwc, int64_t n, int H, int W,
                          hipStream_t st, uint64_t rng_seed = 0) {
  const size_t bytes = (size_t)n * H * W * 64 * sizeof(float);
  switch (hidden_init) {
    case MP_HIDDEN_RANDOM:
      // a fresh xavier-uniform draw on the device (hgru_module.py:884-887), limit sqrt(6 / (k + k))
      c->h0.alloc(bytes);
      hip_check(launch_hidden_uniform(c->h0.f(), (int64_t)n * H * W * 64, rng_seed, std::sqrt(6.0 / (2 * 64)), st),
                "hidden_init random");
      return c->h0.f();
    case MP_HIDDEN_GIVEN:
      if (!o0) fail(MP_ERR_ARG, "o0 is NULL (hidden_init = MP_HIDDEN_GIVEN)");
      return o0;
    case MP_HIDDEN_ZEROS:
      c->h0.alloc(bytes);
      hip_check(hipMemsetAsync(c->h0.p, 0, bytes, st), "hidden_init zeros");
      return c->h0.f();
    case MP_HIDDEN_IDENTITY:
      if (x_nhwc) return x_nhwc;
      c->h0.alloc(bytes);
      hip_check(launch_c8_to_nhwc(c->X.f(), c->h0.f(), (int)n, H, W, st, bf16_maps(c), 0, x_c4(c)), "hidden_init identity");
      return c->h0.f();
    default:
      fail(MP_ERR_ARG, "hidden_init must be MP_HIDDEN_GIVEN, _ZEROS, _IDENTITY or _RANDOM");
  }
  return nullptr;
}

}  // namespace

// ================================================ C ABI ============================================


extern "C" {

// 0.2: mp_pose_taps back to its 0.1 layout (the 0.1 header's seven pointers); the per-step states,
// hidden_init and the device O0 draw moved to the size-checked mp_fwd_opts (mp_hgru_pose_fwd_ex,
// mp_hgru_circuit_fwd_opts); mp_crop3d_ex (docom)
// 0.3: mp_hbm_probe / mp_hbm_rates added; the "graph_captured" mp_info key removed (the hipGraph
// replay path it reported was deleted in round 4)
int mp_version(void) { return (0 << 16) | 3; }

const char* mp_last_error(void) { return g_err.c_str(); }

int mp_create(int device, int model_kind, mp_ctx** out) {
  return guard([&] {
    if (!out) fail(MP_ERR_ARG, "out is NULL");
    if (model_kind < MP_MODEL_HGRU_POSE || model_kind > MP_MODEL_GRAPH)
      fail(MP_ERR_ARG, "unknown model_kind " + std::to_string(model_kind));
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (device < 0 || device >= ndev) fail(MP_ERR_ARG, "device " + std::to_string(device) + " out of range");
    hip_check(hipSetDevice(device), "hipSetDevice");
    auto* c = new mp_ctx();
    c->device = device;
    c->model = model_kind;
    *out = c;
  });
}

void mp_destroy(mp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  delete ctx;
}

int mp_set_weight(mp_ctx* ctx, const char* name, const float* data, const int64_t* shape, int ndim,
                  int mem_kind) {
  return guard([&] {
    if (!ctx || !name || !data || (!shape && ndim > 0) || ndim < 0 || ndim > 8)
      fail(MP_ERR_ARG, "mp_set_weight: bad argument");
    if (mem_kind != MP_MEM_HOST && mem_kind != MP_MEM_DEVICE) fail(MP_ERR_ARG, "mp_set_weight: bad mem_kind");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    const std::string n = strip_scope(name);
    if (!known_name(ctx->model, n)) fail(MP_ERR_WEIGHT, "unknown weight name: " + std::string(name));
    RawWeight w;
    for (int i = 0; i < ndim; ++i) {
      if (shape[i] <= 0) fail(MP_ERR_WEIGHT, "non-positive dimension in " + n);
      w.shape.push_back(shape[i]);
    }
    const size_t cnt = w.numel(), bytes = cnt * sizeof(float);
    w.dev = std::make_unique<DevBuf>();
    w.dev->alloc(bytes);
    hip_check(hipMemcpy(w.dev->p, data, bytes,
                        mem_kind == MP_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice),
              "hipMemcpy weight");
    if (cnt <= (1u << 16)) {
      w.host.resize(cnt);
      hip_check(hipMemcpy(w.host.data(), w.dev->p, bytes, hipMemcpyDeviceToHost), "hipMemcpy D2H");
    }
    ctx->raw[n] = std::move(w);
    ctx->finalized = false;
  });
}

int mp_bcast_weights(mp_ctx* const* ctxs, int nctx, int root) {
  return guard([&] {
    if (!ctxs || nctx <= 0 || root < 0 || root >= nctx) fail(MP_ERR_ARG, "mp_bcast_weights: bad argument");
    mp_ctx* src = ctxs[root];
    std::vector<mp_ctx*> order{src};
    for (int i = 0; i < nctx; ++i) {
      if (!ctxs[i]) fail(MP_ERR_ARG, "mp_bcast_weights: null context");
      if (ctxs[i]->model != src->model) fail(MP_ERR_ARG, "mp_bcast_weights: contexts of different model kinds");
      for (int j = 0; j < i; ++j)
        if (ctxs[j] == ctxs[i]) fail(MP_ERR_ARG, "mp_bcast_weights: a context is listed twice");
      if (i != root) order.push_back(ctxs[i]);
    }
    if (src->raw.empty()) fail(MP_ERR_STATE, "mp_bcast_weights: the root context has no weights");
    hip_check(hipSetDevice(src->device), "hipSetDevice");
    hip_check(hipDeviceSynchronize(), "sync root");   // its mp_set_weight copies are complete
    // destination tensors, same names / shapes (small ones keep their host copy for BN folding)
    for (size_t k = 1; k < order.size(); ++k) {
      mp_ctx* c = order[k];
      hip_check(hipSetDevice(c->device), "hipSetDevice");
      c->raw.clear();
      for (const auto& kv : src->raw) {
        RawWeight w;
        w.shape = kv.second.shape;
        w.host = kv.second.host;
        w.dev = std::make_unique<DevBuf>();
        w.dev->alloc(w.numel() * sizeof(float));
        c->raw[kv.first] = std::move(w);
      }
      c->finalized = false;
    }
    // binomial tree: in round r, holders order[0 .. have) copy to order[have .. 2 have)
    for (size_t have = 1; have < order.size(); have *= 2) {
      std::vector<int> devs;
      for (size_t i = 0; i < have && i + have < order.size(); ++i) {
        mp_ctx *a = order[i], *b = order[i + have];
        hip_check(hipSetDevice(b->device), "hipSetDevice");
        if (a->device != b->device) {
          int can = 0;
          hip_check(hipDeviceCanAccessPeer(&can, b->device, a->device), "hipDeviceCanAccessPeer");
          if (can) {
            const hipError_t e = hipDeviceEnablePeerAccess(a->device, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) hip_check(e, "hipDeviceEnablePeerAccess");
            (void)hipGetLastError();
          }
        }
        hip_check(hipSetDevice(a->device), "hipSetDevice");
        for (const auto& kv : a->raw) {
          const auto& dst = b->raw.at(kv.first);
          hip_check(hipMemcpyPeerAsync(dst.dev->p, b->device, kv.second.dev->p, a->device,
                                       kv.second.numel() * sizeof(float), nullptr),
                    "hipMemcpyPeerAsync");
        }
        devs.push_back(a->device);
        devs.push_back(b->device);
      }
      for (int d : devs) {   // every copy of this round is complete before the next round reads them
        hip_check(hipSetDevice(d), "hipSetDevice");
        hip_check(hipDeviceSynchronize(), "bcast round sync");
      }
    }
    hip_check(hipSetDevice(src->device), "hipSetDevice");
  });
}

int mp_finalize_weights(mp_ctx* ctx, int compute_dtype) {
  return guard([&] {
    if (!ctx) fail(MP_ERR_ARG, "ctx is NULL");
    if (compute_dtype != MP_DTYPE_F32 && compute_dtype != MP_DTYPE_F32_SPLIT && compute_dtype != MP_DTYPE_F32_FFT &&
        compute_dtype != MP_DTYPE_BF16)
      fail(MP_ERR_UNSUPPORTED, "compute_dtype must be MP_DTYPE_F32, _F32_SPLIT, _F32_FFT or MP_DTYPE_BF16");
    if (ctx->model >= MP_MODEL_DENSE && compute_dtype != MP_DTYPE_F32 && compute_dtype != MP_DTYPE_F32_SPLIT &&
        compute_dtype != MP_DTYPE_BF16)
      fail(MP_ERR_UNSUPPORTED, "regressor contexts run MP_DTYPE_F32, MP_DTYPE_F32_SPLIT or MP_DTYPE_BF16");
    if (compute_dtype != ctx->dtype) {   // workspace layout depends on the path
      ctx->cap_batch = 0;
      ctx->cap_hw = 0;
    }
    ctx->dtype = compute_dtype;
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    if (ctx->model == MP_MODEL_HGRU_POSE)
      finalize_pose(ctx);
    else if (ctx->model == MP_MODEL_HGRU_CIRCUIT)
      finalize_circuit(ctx, nullptr, nullptr);
    else if (ctx->model == MP_MODEL_GRAPH)
      finalize_graph(ctx);
    else
      finalize_regressor(ctx);
    hip_check(hipDeviceSynchronize(), "finalize sync");
    ctx->finalized = true;
  });
}

int mp_reserve(mp_ctx* ctx, int64_t max_batch) {
  return guard([&] {
    if (!ctx || max_batch <= 0) fail(MP_ERR_ARG, "mp_reserve: bad argument");
    if (!ctx->finalized) fail(MP_ERR_STATE, "mp_reserve before mp_finalize_weights");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    if (ctx->model >= MP_MODEL_DENSE) return;   // regressors: sized at first call
    const int64_t hw = ctx->model == MP_MODEL_HGRU_POSE ? ctx->fc1_in / 64 : 64 * 64;
    ensure_ws(ctx, max_batch, hw, 1);
  });
}

}  // extern "C"

namespace {

// the per-call options of a forward, from mp_fwd_opts (or their 0.1 defaults)
struct FwdOpts {
  mp_pose_taps tp{};
  float* states_O = nullptr;
  float* states_I = nullptr;
  int hidden_init = MP_HIDDEN_GIVEN;
  uint64_t rng_seed = 0;
};

// mp_fwd_opts as the caller compiled it: only struct_size bytes are read (fields the caller does not
// know keep their defaults), so a smaller, older struct never makes the library read past it
FwdOpts read_opts(const mp_fwd_opts* o, bool pose) {
  FwdOpts f;
  if (!o) return f;
  if (o->struct_size < offsetof(mp_fwd_opts, rng_call) + sizeof(uint64_t))
    fail(MP_ERR_ARG, "mp_fwd_opts.struct_size is smaller than the 0.2 layout");
  mp_fwd_opts c{};
  std::memcpy(&c, o, std::min<size_t>((size_t)o->struct_size, sizeof(c)));
  f.hidden_init = c.hidden_init;
  f.rng_seed = c.rng_seed + c.rng_call;
  f.states_O = c.states_O;
  f.states_I = c.states_I;
  if (c.taps) {
    if (!pose) fail(MP_ERR_ARG, "mp_fwd_opts.taps is for the pose model only");
    f.tp = *c.taps;
  }
  return f;
}

int pose_fwd(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, const float* o0, float* out,
             const FwdOpts& fo, void* stream) {
  return guard([&] {
    const mp_pose_taps& tp = fo.tp;
    if (!ctx || !depth || !out || (!o0 && fo.hidden_init == MP_HIDDEN_GIVEN))
      fail(MP_ERR_ARG, "mp_hgru_pose_fwd: null pointer");
    if (ctx->model != MP_MODEL_HGRU_POSE) fail(MP_ERR_STATE, "context is not an hgru_pose model");
    if (!ctx->finalized) fail(MP_ERR_STATE, "weights not finalized");
    if (n <= 0 || n > (1 << 20)) fail(MP_ERR_SHAPE, "batch must be in [1, 2^20]");
    if (h % 2 || w % 2) fail(MP_ERR_SHAPE, "crop height/width must be even");
    const int H = (int)(h / 2), W = (int)(w / 2);
    if (H % TH || W % TW)
      fail(MP_ERR_SHAPE, "crop/2 must be a multiple of 16 (rows) and 32 (cols)");   // backbone tiles
    check_map(ctx, H, W, "crop/2");
    if ((int64_t)H * W * 64 != ctx->fc1_in)
      fail(MP_ERR_SHAPE, "crop size does not match fc_1 input (" + std::to_string(ctx->fc1_in) + ")");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t st = static_cast<hipStream_t>(stream);
    ensure_ws(ctx, n, H, W);
    const int N = (int)n;
    if (tp.conv1) {   // relu(conv_1) before the pool: never materialised by the fused kernel
      IgemmArgs g{};
      g.x = depth;
      g.ldx = 1;
      g.N = N;
      g.H = (int)h;
      g.W = (int)w;
      g.Cin = 1;
      g.wpk = ctx->conv1_ig.v4();
      g.K = 9;
      g.bias = ctx->conv1_b.f();
      g.out = tp.conv1;
      g.ldo = 64;
      g.Cout = 64;
      g.Ho = (int)h;
      g.Wo = (int)w;
      g.KS = 3;
      g.stride = 1;
      g.pad_t = 1;
      g.pad_l = 1;
      g.relu = 1;
      hip_check(launch_igemm_conv(g, st), "conv_1 tap");
    }
    // the backbone of images b0 .. b0 + cnt on stream s (every buffer is image-major)
    const bool x3 = ctx->dtype != MP_DTYPE_F32 && H % TH3 == 0;
    const int np = ctx->dtype == MP_DTYPE_BF16 ? 1 : 3;   // bf16: one f16 product per MAC
    const size_t px = (size_t)H * W * 64;                  // elements of one image's 64-channel map
    const SliceFn backbone = [&](int b0, int cnt, hipStream_t s) {
      ProfScope ps(ctx, s, "backbone");
      float* bA = ctx->bufA.f() + b0 * px;
      float* bB = ctx->bufB.f() + b0 * px;
      float* xm = bf16_maps(ctx) ? reinterpret_cast<float*>(reinterpret_cast<uint16_t*>(ctx->X.p) + b0 * px)
                                 : ctx->X.f() + b0 * px;
      hip_check(launch_conv1_pool_bn(depth + (size_t)b0 * h * w, ctx->conv1_w.f(), ctx->conv1_b.f(), ctx->bn0_s.f(),
                                     ctx->bn0_t.f(), bA, cnt, (int)h, (int)w, s),
                "conv_1");
      ConvArgs a{};
      a.H = H;
      a.W = W;
      a.src = bA;
      a.wpk = ctx->conv2_pk.v4();
      a.dst = bB;
      a.bias = ctx->conv2_b.f();
      a.bn_s = ctx->bn1_s.f();
      a.bn_t = ctx->bn1_t.f();
      if (x3) a.ascale = BB_ASCALE;
      hip_check(x3 ? launch_conv64x3(3, EPI_BB, a, ctx->conv2_pk.p, ctx->conv2_us, cnt, s, np)
                   : launch_conv64(3, EPI_BB, a, cnt, s),
                "conv_2");
      a.src = bB;
      a.wpk = ctx->conv3_pk.v4();
      a.dst = xm;
      a.dst_bf16 = bf16_maps(ctx) ? 1 : 0;
      a.dst_c4 = x_c4(ctx) ? 1 : 0;
      a.bias = ctx->conv3_b.f();
      a.bn_s = ctx->bn2_s.f();
      a.bn_t = ctx->bn2_t.f();
      hip_check(x3 ? launch_conv64x3(3, EPI_BB, a, ctx->conv3_pk.p, ctx->conv3_us, cnt, s, np)
                   : launch_conv64(3, EPI_BB, a, cnt, s),
                "conv_3");
    };
    // the backbone runs per batch slice on the slice's stream (MP_BB_PIPE) unless a tap needs its
    // intermediate maps or hidden_init = identity needs X (O0 = X) before the loop; otherwise
    // whole-batch on the caller's stream first
    const bool bb_pipe = bb_pipeline() && !tp.pool1 && !tp.conv2 && !tp.conv3 && fo.hidden_init != MP_HIDDEN_IDENTITY;
    if (!bb_pipe) backbone(0, N, st);
    if (tp.pool1) hip_check(launch_c8_to_nhwc(ctx->bufA.f(), tp.pool1, N, H, W, st), "pool1 tap");
    if (tp.conv2) hip_check(launch_c8_to_nhwc(ctx->bufB.f(), tp.conv2, N, H, W, st), "conv2 tap");
    if (tp.conv3) hip_check(launch_c8_to_nhwc(ctx->X.f(), tp.conv3, N, H, W, st, bf16_maps(ctx), 0, x_c4(ctx)), "conv3 tap");
    const float* h0 = hidden_state(ctx, fo.hidden_init, o0, nullptr, n, H, W, st, fo.rng_seed);
    StateOut so;
    so.O = fo.states_O;
    so.I = fo.states_I;
    so.T = ctx->timesteps;
    // FFT dtypes: the last B epilogue writes fc_1's f16 hi / lo activation planes into fcin (same
    // bytes as the fp32 map), so fc_1 stages them by LDS-DMA with no conversion (bit-identical); the
    // hgru tap needs the fp32 map, and MP_FC_PRESPLIT=0 restores that form for A/B
    SplitOut sp;
    const bool presplit = is_fft(ctx->dtype) && !tp.hgru && fc_presplit();
    const int fc_np = ctx->dtype == MP_DTYPE_BF16 ? 1 : 3;   // bf16: one f16 product
    if (presplit) {
      sp.hi = reinterpret_cast<_Float16*>(ctx->fcin.p);
      sp.lo = fc_np == 3 ? sp.hi + (size_t)N * ctx->fc1_in : nullptr;
    }
    // the head of rows b0 .. b0 + cnt on stream s: fc_1 on the split planes (partials in the slice's own
    // S x cnt x Npad region of part, so slices run at once), relu + BN_4 into h1, fc_out (part2), its
    // reduce into out.  Each row's sums are the same MFMA chains whatever the rows' count (the split
    // count and slice length are functions of K and N only): bit-identical to the whole-batch head
    int ks1, ks2;
    const int S1 = fc_choose_splits(N, ctx->fc1_in, ctx->fc1_out, &ks1);
    const int S2 = fc_choose_splits(N, ctx->fc1_out, ctx->nout, &ks2);
    const size_t np1 = (size_t)(ctx->fc1_out + 31) / 32 * 32, np2 = (size_t)(ctx->nout + 31) / 32 * 32;
    const SliceFn head = [&](int b0, int cnt, hipStream_t s) {
      float* h1 = ctx->h1.f() + (size_t)b0 * ctx->fc1_out;
      {
        ProfScope ps(ctx, s, "fc1");
        float* p1 = ctx->part.f() + (size_t)S1 * b0 * np1;
        hip_check(launch_fc_gemm_x3p(sp.hi + (size_t)b0 * ctx->fc1_in, sp.lo ? sp.lo + (size_t)b0 * ctx->fc1_in : nullptr,
                                     ctx->fc1_in, ctx->fc1_pk.p, ctx->fc1_unscale, p1, cnt, ctx->fc1_in, ctx->fc1_out,
                                     S1, ks1, s, fc_np),
                  "fc_1 gemm");
        hip_check(launch_fc_reduce(p1, S1, cnt, ctx->fc1_out, ctx->fc1_b.f(), 1, ctx->bn4_s.f(), ctx->bn4_t.f(), h1,
                                   ctx->fc1_out, s),
                  "fc_1 reduce");
      }
      ProfScope ps(ctx, s, "fc_out");
      float* p2 = ctx->part2.f() + (size_t)S2 * b0 * np2;
      hip_check(launch_fc_gemm(h1, ctx->fc1_out, ctx->fco_pk.v4(), p2, cnt, ctx->fc1_out, ctx->nout, S2, ks2, s),
                "fc_out gemm");
      hip_check(launch_fc_reduce(p2, S2, cnt, ctx->nout, ctx->fco_b.f(), 0, nullptr, nullptr, out + (size_t)b0 * ctx->nout,
                                 ctx->nout, s),
                "fc_out reduce");
    };
    const bool head_slices = presplit && fc_slice() && !tp.fc1 && !tp.relu1;
    run_circuit(ctx, n, H, W, ctx->timesteps, h0, ctx->fcin.f(), (so.O || so.I) ? &so : nullptr, st,
                presplit ? &sp : nullptr, bb_pipe ? &backbone : nullptr, head_slices ? &head : nullptr);
    if (head_slices) return;
    if (tp.hgru)
      hip_check(hipMemcpyAsync(tp.hgru, ctx->fcin.f(), (size_t)N * ctx->fc1_in * sizeof(float),
                               hipMemcpyDeviceToDevice, st),
                "hgru tap");
    {
      ProfScope ps(ctx, st, "fc1");
      int ks;
      const int S = fc_choose_splits(N, ctx->fc1_in, ctx->fc1_out, &ks);
      (void)S1;
      (void)S2;
      hip_check(ctx->dtype == MP_DTYPE_F32
                    ? launch_fc_gemm(ctx->fcin.f(), ctx->fc1_in, ctx->fc1_pk.v4(), ctx->part.f(), N, ctx->fc1_in,
                                     ctx->fc1_out, S, ks, st)
                : presplit ? launch_fc_gemm_x3p(sp.hi, sp.lo, ctx->fc1_in, ctx->fc1_pk.p, ctx->fc1_unscale,
                                                ctx->part.f(), N, ctx->fc1_in, ctx->fc1_out, S, ks, st, fc_np)
                           : launch_fc_gemm_x3(ctx->fcin.f(), ctx->fc1_in, ctx->fc1_pk.p, ctx->fc1_unscale,
                                               ctx->part.f(), N, ctx->fc1_in, ctx->fc1_out, S, ks, st, fc_np),
                "fc_1 gemm");
      if (tp.fc1)   // fc_1 + bias before the relu (same partial sums)
        hip_check(launch_fc_reduce(ctx->part.f(), S, N, ctx->fc1_out, ctx->fc1_b.f(), 0, nullptr, nullptr, tp.fc1,
                                   ctx->fc1_out, st),
                  "fc1 tap");
      hip_check(launch_fc_reduce(ctx->part.f(), S, N, ctx->fc1_out, ctx->fc1_b.f(), 1, ctx->bn4_s.f(),
                                 ctx->bn4_t.f(), ctx->h1.f(), ctx->fc1_out, st),
                "fc_1 reduce");
    }
    {
      ProfScope ps(ctx, st, "fc_out");
      int ks;
      const int S2 = fc_choose_splits(N, ctx->fc1_out, ctx->nout, &ks);
      hip_check(launch_fc_gemm(ctx->h1.f(), ctx->fc1_out, ctx->fco_pk.v4(), ctx->part.f(), N, ctx->fc1_out,
                               ctx->nout, S2, ks, st),
                "fc_out gemm");
      hip_check(launch_fc_reduce(ctx->part.f(), S2, N, ctx->nout, ctx->fco_b.f(), 0, nullptr, nullptr, out,
                                 ctx->nout, st),
                "fc_out reduce");
    }
    if (tp.relu1)
      hip_check(hipMemcpyAsync(tp.relu1, ctx->h1.f(), (size_t)N * ctx->fc1_out * sizeof(float),
                               hipMemcpyDeviceToDevice, st),
                "relu1 tap");
  });
}

}  // namespace

extern "C" {

int mp_hgru_pose_fwd_taps(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, const float* o0,
                          float* out, const mp_pose_taps* taps, void* stream) {
  FwdOpts fo;
  if (taps) fo.tp = *taps;   // the seven pointers of the 0.1 struct, nothing past them
  return pose_fwd(ctx, depth, n, h, w, o0, out, fo, stream);
}

int mp_hgru_pose_fwd_ex(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, const float* o0,
                        float* out, const mp_fwd_opts* opts, void* stream) {
  FwdOpts fo;
  const int rc = guard([&] { fo = read_opts(opts, true); });
  if (rc != MP_OK) return rc;
  return pose_fwd(ctx, depth, n, h, w, o0, out, fo, stream);
}

int mp_hgru_pose_fwd(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, const float* o0,
                     float* out, void* stream) {
  return mp_hgru_pose_fwd_taps(ctx, depth, n, h, w, o0, out, nullptr, stream);
}

int mp_hgru_circuit_fwd(mp_ctx* ctx, const float* x, const float* o0, int64_t n, int64_t h, int64_t w,
                        int64_t k, int timesteps, float* o_out, void* stream) {
  return mp_hgru_circuit_fwd_ex(ctx, x, o0, n, h, w, k, timesteps, MP_HIDDEN_GIVEN, o_out, nullptr, nullptr,
                                stream);
}

int mp_hgru_circuit_fwd_ex(mp_ctx* ctx, const float* x, const float* o0, int64_t n, int64_t h, int64_t w,
                           int64_t k, int timesteps, int hidden_init, float* o_out, float* states_O,
                           float* states_I, void* stream) {
  mp_fwd_opts o{};
  o.struct_size = sizeof(o);
  o.hidden_init = hidden_init;
  o.states_O = states_O;
  o.states_I = states_I;
  return mp_hgru_circuit_fwd_opts(ctx, x, o0, n, h, w, k, timesteps, o_out, &o, stream);
}

int mp_hgru_circuit_fwd_opts(mp_ctx* ctx, const float* x, const float* o0, int64_t n, int64_t h, int64_t w,
                             int64_t k, int timesteps, float* o_out, const mp_fwd_opts* opts, void* stream) {
  return guard([&] {
    const FwdOpts fo = read_opts(opts, false);
    const int hidden_init = fo.hidden_init;
    float* states_O = fo.states_O;
    float* states_I = fo.states_I;
    if (!ctx || !x || !o_out || (!o0 && hidden_init == MP_HIDDEN_GIVEN))
      fail(MP_ERR_ARG, "mp_hgru_circuit_fwd: null pointer");
    if (!ctx->finalized) fail(MP_ERR_STATE, "weights not finalized");
    if (k != 64) fail(MP_ERR_SHAPE, "channel count k must be 64");
    if (n <= 0 || h <= 0 || w <= 0) fail(MP_ERR_SHAPE, "empty input");
    check_map(ctx, h, w, "x");
    if (timesteps < 1 || timesteps > (int)ctx->rho.size())
      fail(MP_ERR_ARG, "timesteps must be in [1, len(rho)]");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t st = static_cast<hipStream_t>(stream);
    ensure_ws(ctx, n, h, w);
    hip_check(launch_nhwc_to_c8(x, ctx->X.f(), (int)n, (int)h, (int)w, st, bf16_maps(ctx), x_c4(ctx)), "nhwc_to_c8");
    if (ctx->model == MP_MODEL_HGRU_POSE) {
      // the pose context's output affine is BN_3: use identity by running with a temporary copy
      fail(MP_ERR_UNSUPPORTED, "use an MP_MODEL_HGRU_CIRCUIT context for the standalone circuit");
    }
    const float* h0 = hidden_state(ctx, hidden_init, o0, x, n, (int)h, (int)w, st, fo.rng_seed);
    StateOut so;
    so.O = states_O;
    so.I = states_I;
    so.T = timesteps;
    run_circuit(ctx, n, (int)h, (int)w, timesteps, h0, o_out, (states_O || states_I) ? &so : nullptr, st);
  });
}

int mp_info(mp_ctx* ctx, const char* key, int64_t* value) {
  return guard([&] {
    if (!ctx || !key || !value) fail(MP_ERR_ARG, "mp_info: null pointer");
    const std::string k(key);
    if (graph_info(ctx, k, value)) return;
    if (k == "output_shape")
      *value = ctx->nout;
    else if (k == "timesteps")
      *value = ctx->timesteps;
    else if (k == "ssf")
      *value = ctx->ssf;
    else if (k == "finalized")
      *value = ctx->finalized ? 1 : 0;
    else if (k == "fc1_in")
      *value = ctx->fc1_in;
    else if (k == "fft_loop")   // 4: the four-step loop (k_fft4.hip), 6: the six-launch loop, 0: no FFT path
      *value = is_fft(ctx->dtype) ? (ctx->fft4 ? 4 : 6) : 0;
    else if (k == "workspace_bytes")
      *value = (int64_t)(ctx->X.bytes + ctx->O.bytes + ctx->I.bytes + ctx->Og.bytes + ctx->bufA.bytes +
                         ctx->bufB.bytes + ctx->fcin.bytes + ctx->part.bytes + ctx->h1.bytes);
    else if (k == "weight_bytes") {
      size_t s = 0;
      for (auto& kv : ctx->raw) s += kv.second.numel() * sizeof(float);
      *value = (int64_t)s;
    } else
      fail(MP_ERR_ARG, "unknown info key: " + k);
  });
}

int mp_profile_enable(mp_ctx* ctx, int enable) {
  return guard([&] {
    if (!ctx) fail(MP_ERR_ARG, "ctx is NULL");
    ctx->prof = enable != 0;
  });
}

int mp_profile_read(mp_ctx* ctx, const char* name, double* total_ms, int64_t* launches) {
  return guard([&] {
    if (!ctx || !name || !total_ms || !launches) fail(MP_ERR_ARG, "mp_profile_read: null pointer");
    double tot = 0;
    int64_t cnt = 0;
    std::vector<ProfEvent> keep;
    for (auto& e : ctx->events) {
      if (e.name == name) {
        hip_check(hipEventSynchronize(e.b), "hipEventSynchronize");
        float ms = 0;
        hip_check(hipEventElapsedTime(&ms, e.a, e.b), "hipEventElapsedTime");
        tot += ms;
        ++cnt;
        ctx->pool.push_back(e.a);
        ctx->pool.push_back(e.b);
      } else {
        keep.push_back(e);
      }
    }
    ctx->events.swap(keep);
    *total_ms = tot;
    *launches = cnt;
  });
}

}  // extern "C"
