// Internal runtime types shared by the C-ABI translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/monkeypose.h"
#include "mp_kernels.hpp"

using namespace mp;

namespace mpr {

extern thread_local std::string g_err;

struct Fail {
  int code;
};

[[noreturn]] inline void fail(int code, const std::string& msg) {
  g_err = msg;
  throw Fail{code};
}

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) fail(MP_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void alloc(size_t n) {
    if (n <= bytes && p) return;
    release();
    hip_check(hipMalloc(&p, n ? n : 16), "hipMalloc");
    bytes = n;
  }
  float* f() const { return static_cast<float*>(p); }
  f32x4* v4() const { return static_cast<f32x4*>(p); }
};

struct RawWeight {
  std::vector<int64_t> shape;
  std::unique_ptr<DevBuf> dev;
  std::vector<float> host;  // kept for small tensors (host-side BN folding)
  size_t numel() const {
    size_t n = 1;
    for (auto s : shape) n *= (size_t)s;
    return n;
  }
};

struct ProfEvent {
  std::string name;
  hipEvent_t a, b;
};

// dtypes whose association-field conv runs on the FFT path (k_fft.hip)
inline bool is_fft(int dtype) { return dtype == MP_DTYPE_F32_FFT || dtype == MP_DTYPE_BF16; }

inline std::string strip_scope(const char* name) {
  std::string s(name);
  if (s.rfind("cnn/", 0) == 0) s = s.substr(4);
  return s;
}

inline bool known_name_hgru(int model, const std::string& n) {
  static const char* circuit[] = {"p_r", "i_r", "i_b", "o_r", "o_b", "beta", "nu", "gamma", "kappa",
                                  "omega", "rho", "lateral_bias"};
  for (auto c : circuit)
    if (n == std::string("contextual_circuit/") + c) return true;
  if (model == MP_MODEL_HGRU_CIRCUIT) return false;
  for (const char* l : {"conv_1", "conv_2", "conv_3"})
    if (n == std::string(l) + "/" + l + "_filters" || n == std::string(l) + "/" + l + "_biases") return true;
  for (const char* l : {"fc_1", "fc_out"})
    if (n == std::string(l) + "/" + l + "_weights" || n == std::string(l) + "/" + l + "_biases") return true;
  for (const char* b : {"batch_normalization", "batch_normalization_1", "batch_normalization_2",
                        "batch_normalization_3", "batch_normalization_4"})
    for (const char* v : {"gamma", "beta", "moving_mean", "moving_variance"})
      if (n == std::string(b) + "/" + v) return true;
  return false;
}

// dense / hierarchical regressor variable names (mp_regressors.hip)
bool known_name_regressor(int model, const std::string& n);

inline bool known_name(int model, const std::string& n) {
  if (model == MP_MODEL_GRAPH) return true;   // checked against the graph at mp_finalize_weights
  return (model == MP_MODEL_HGRU_POSE || model == MP_MODEL_HGRU_CIRCUIT) ? known_name_hgru(model, n)
                                                                         : known_name_regressor(model, n);
}

}  // namespace mpr

using namespace mpr;

struct mp_ctx {
  int device = 0;
  int model = 0;
  bool finalized = false;
  std::map<std::string, RawWeight> raw;

  // ---- finalized weights ----
  int ssf = 15, timesteps = 8, nout = 0, fc1_in = 0, fc1_out = 0;
  int dtype = MP_DTYPE_F32;
  float p_unscale = 1.f;   // F32_SPLIT / F32_FFT: 1 / (weight scale * activation or spectrum scale)
  std::vector<float> rho;
  DevBuf conv1_w, conv1_b, bn0_s, bn0_t;
  DevBuf conv1_ig;          // conv_1 packed for the generic igemm (conv1 tap of mp_hgru_pose_fwd_taps)
  DevBuf conv2_pk, conv2_b, bn1_s, bn1_t;
  float conv2_us = 1.f, conv3_us = 1.f;   // backbone packed f16x3 (dtype != F32): 1 / (wscale * BB_ASCALE)
  DevBuf conv3_pk, conv3_b, bn2_s, bn2_t;
  DevBuf p_pk, ir_pk, or_pk, vecs;
  DevBuf spec_g;            // MP_DTYPE_F32_FFT: compact split spectral weights of p_r (k_fft.hip)
  bool fft4 = false;        // the fp32 FFT path runs k_fft4.hip's four-step loop (class-major spec_g)
  DevBuf or_x3, ir_x3;      // MP_DTYPE_F32_FFT: o_r / i_r packed for the f16x3 gate GEMMs
  float or_us = 1.f, ir_us = 1.f;
  DevBuf fc1_pk, fc1_b, bn4_s, bn4_t, fco_pk, fco_b;
  float fc1_unscale = 1.f;   // fc_1 packed f16x3 (dtype F32_SPLIT / F32_FFT): 1 / weight scale

  // ---- workspace ----
  int64_t cap_batch = 0;
  int64_t cap_hw = 0;
  DevBuf bufA, bufB, X, O, I, Og, fcin, part, part2, h1;   // part2: fc_out's partials (per-slice heads)
  DevBuf h0;                // hidden_init zeros / identity: the NHWC initial state (allocated on use)
  DevBuf specS, specY, specP;   // MP_DTYPE_F32_FFT: input / output spectra, spatial conv result

  // ---- dense / hierarchical regressors (mp_regressors.hip) ----
  struct PackedLayer {
    DevBuf w, b;          // conv: HWIO as [K][Cout] packed like an FC weight; fc: [in][out] packed
    DevBuf bn_s, bn_t;    // attention net: the folded BN that follows this layer (after pool / relu)
    int k = 0, cin = 0, cout = 0, K = 0;
    bool x3 = false;      // MP_DTYPE_F32_SPLIT / _BF16: w holds the f16x3 packing (launch_pack_fc_x3)
    float wus = 1.f;      // its 1 / weight scale
    int nprod = 3;        // products per MAC: 3 (fp32-accurate split) or 1 (MP_DTYPE_BF16: hi x hi)
    DevBuf wpad;          // x3 convs with Cin % 32 != 0: the packing with Cin zero-padded to cinp per
    int cinp = 0;         // tap (the halo kernel's 32-channel chunks; same scale as w)
  };
  std::map<std::string, PackedLayer> layers;   // keyed by layer name ("conv_3_1", "p_fc_2", ...)
  std::map<std::string, DevBuf> ws;            // named activation buffers
  int64_t ws_batch = 0, ws_h = 0, ws_w = 0;
  std::vector<int> head_sizes;                 // outputs: dense {out}; hier {out, P, R, M, I, T}

  // ---- recorded layer graph (MP_MODEL_GRAPH, mp_graph.hip) ----
  std::shared_ptr<struct GraphState> graph;

  // ---- profiling ----
  bool prof = false;
  std::vector<ProfEvent> events;
  std::vector<hipEvent_t> pool;

  // ---- batch slices on extra streams (FFT circuit; MP_STREAMS=1 disables) ----
  std::vector<hipStream_t> sides;
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_pre = nullptr;   // a slice's backbone done (MP_BB_STAGGER)
  std::vector<hipEvent_t> ev_join;

  ~mp_ctx() {
    for (auto s : sides) (void)hipStreamDestroy(s);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_pre) (void)hipEventDestroy(ev_pre);
    for (auto e : ev_join) (void)hipEventDestroy(e);
    for (auto& e : events) {
      (void)hipEventDestroy(e.a);
      (void)hipEventDestroy(e.b);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
  }

  const RawWeight& need(const std::string& n, std::vector<int64_t> shape) {
    auto it = raw.find(n);
    if (it == raw.end()) fail(MP_ERR_STATE, "weight not set: " + n);
    if (!shape.empty() && it->second.shape != shape) {
      std::string s = "weight " + n + " has shape [";
      for (auto v : it->second.shape) s += std::to_string(v) + ",";
      s += "], expected [";
      for (auto v : shape) s += std::to_string(v) + ",";
      fail(MP_ERR_WEIGHT, s + "]");
    }
    return it->second;
  }

  hipEvent_t ev() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    hip_check(hipEventCreate(&e), "hipEventCreate");
    return e;
  }
};

namespace mpr {

// run f, converting a Fail / exception into a status code + thread-local message
inline int guard(const std::function<void()>& f) {
  try {
    g_err.clear();
    f();
    return MP_OK;
  } catch (const Fail& e) {
    return e.code;
  } catch (const std::exception& e) {
    g_err = std::string("internal error: ") + e.what();
    return MP_ERR_STATE;
  } catch (...) {
    g_err = "internal error";
    return MP_ERR_STATE;
  }
}

// HIP events around a launch sequence on its stream (mp_profile_*)
struct ProfScope {
  mp_ctx* c;
  hipStream_t st;
  const char* name;
  hipEvent_t a = nullptr;
  ProfScope(mp_ctx* c_, hipStream_t s, const char* n) : c(c_), st(s), name(n) {
    if (c->prof) {
      a = c->ev();
      hip_check(hipEventRecord(a, st), "hipEventRecord");
    }
  }
  ~ProfScope() noexcept(false) {
    if (a) {
      hipEvent_t b = c->ev();
      hip_check(hipEventRecord(b, st), "hipEventRecord");
      c->events.push_back({name, a, b});
    }
  }
};

// mp_abi.hip: host vector -> device; inference BN folded to a per-channel affine
// gamma * (x - mean) / sqrt(var + eps) + beta = x * s + t  (eps = 1e-5, hgru_pose.py:17)
void upload(DevBuf& d, const std::vector<float>& h);
void bn_fold(mp_ctx* c, const std::string& scope, int n, DevBuf& s_out, DevBuf& t_out,
             std::vector<float>* hs = nullptr, std::vector<float>* ht = nullptr);

// mp_regressors.hip
void finalize_regressor(mp_ctx* c);
// a conv ([K][Cout]) or fc ([K][N]) weight packed in the context's precision
void pack_matrix(mp_ctx* c, mp_ctx::PackedLayer& L, const float* w, bool x3_ok);

// mp_graph.hip
void finalize_graph(mp_ctx* c);
bool graph_info(mp_ctx* c, const std::string& key, int64_t* value);   // "graph_*" keys of mp_info

}  // namespace mpr
