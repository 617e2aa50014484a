// Dense (train_dense_networks.py:223-408) and hierarchical (train_hier_networks.py:338-530)
// pose regressors: weight packing and the forward schedule, on the generic implicit-GEMM conv,
// 2x2 pool and split-K FC kernels.  tf.concat is free: every concatenated tensor is a channel
// prefix of one wide NHWC buffer per scale, which its producers write at channel offsets.
#include "mp_runtime.hpp"

namespace {

struct ConvSpec {
  std::string name;
  int k, stride, cin, cout;
};

// train_dense_networks.py:226-373 (mirrors monkey-pose_amd/weights.py::dense_conv_specs)
const int kDenseW[4][10] = {{24, 32, 32, 48, 32, 48, 48, 64, 48, 64},
                            {32, 48, 48, 64, 48, 64, 64, 96, 64, 96},
                            {48, 64, 64, 96, 64, 96, 96, 128, 96, 128},
                            {64, 96, 96, 128, 96, 128, 128, 144, 128, 144}};

std::vector<ConvSpec> dense_convs() {
  std::vector<ConvSpec> s = {{"conv_0", 3, 1, 1, 12},     {"conv_1_1", 3, 1, 12, 16},   {"conv_1_2", 3, 2, 16, 24},
                             {"conv_1_3", 3, 2, 24, 32},  {"conv_2_1", 3, 1, 16, 24},   {"conv_2_2_1", 3, 2, 16, 24},
                             {"conv_2_2_2", 3, 1, 24, 32}, {"conv_2_3_2", 3, 2, 24, 32}, {"conv_2_3_3", 3, 1, 32, 48}};
  int w1 = 40, w2 = 80, w3 = 112;
  for (int L = 3; L <= 6; ++L) {
    const int* d = kDenseW[L - 3];
    const std::string p = "conv_" + std::to_string(L);
    s.push_back({p + "_1_1x1", 1, 1, w1, d[0]});
    s.push_back({p + "_1", 3, 1, d[0], d[1]});
    s.push_back({p + "_2_1x1_1", 1, 1, w1, d[2]});
    s.push_back({p + "_2_1", 3, 2, d[2], d[3]});
    s.push_back({p + "_2_1x1_2", 1, 1, w2, d[4]});
    s.push_back({p + "_2_2", 3, 1, d[4], d[5]});
    s.push_back({p + "_3_1x1_2", 1, 1, w2, d[6]});
    s.push_back({p + "_3_2", 3, 2, d[6], d[7]});
    s.push_back({p + "_3_1x1_3", 1, 1, w3, d[8]});
    s.push_back({p + "_3_3", 3, 1, d[8], d[9]});
    w1 += d[1];
    w2 += d[3] + d[5];
    w3 += d[7] + d[9];
  }
  return s;
}
const char* kDenseFc[] = {"fc_1_1", "fc_1_2", "fc_1_3", "fc_2", "fc_3", "fc_4"};

const char* kFingers[] = {"p", "r", "m", "i", "t"};

// train_hier_networks.py:341-469
std::vector<ConvSpec> hier_convs() {
  std::vector<ConvSpec> s = {{"conv_1", 3, 1, 1, 64}, {"conv_2", 3, 1, 64, 128}};
  for (const char* br : {"pr", "mi", "t"}) {
    s.push_back({std::string(br) + "_con_3", 3, 1, 128, 256});
    s.push_back({std::string(br) + "_con_4", 3, 1, 256, 512});
  }
  for (const char* f : kFingers) {
    s.push_back({std::string(f) + "_con_5", 3, 1, 512, 512});
    s.push_back({std::string(f) + "_con_6", 5, 1, 512, 1024});
  }
  return s;
}
std::vector<std::string> hier_fcs() {
  std::vector<std::string> v;
  for (const char* f : kFingers)
    for (const char* suf : {"_fc_1", "_fc_2", "_fc_3", "h_fc_1", "h_fc_2"}) v.push_back(std::string(f) + suf);
  v.push_back("final_fc_1");
  v.push_back("final_fc_2");
  return v;
}

// attn_model_struct (train_cnn_networks_hgru.py:440-475): five conv + 2x2 max pool + BN stages
std::vector<ConvSpec> attn_convs() {
  return {{"aconv_1", 3, 1, 1, 64},
          {"aconv_2", 3, 1, 64, 128},
          {"aconv_3", 3, 1, 128, 256},
          {"aconv_4", 3, 1, 256, 512},
          {"aconv_5", 5, 1, 512, 1024}};
}
// tf.layers.batch_normalization calls in build order: after apool_1, apool_2, pool_3, pool_4,
// apool_5 (442-476) and after relu(afc_1) (482-490); default scopes of a fresh "cnn" scope
const char* kAttnBn[] = {"batch_normalization",   "batch_normalization_1", "batch_normalization_2",
                         "batch_normalization_3", "batch_normalization_4", "batch_normalization_5"};
constexpr int ATTN_SIZE = 128;   // tf.image.resize_images(input_image, [128, 128]) (439)

std::vector<ConvSpec> convs_of(int model) {
  if (model == MP_MODEL_DENSE) return dense_convs();
  if (model == MP_MODEL_ATTN) return attn_convs();
  return hier_convs();
}
std::vector<std::string> fcs_of(int model) {
  if (model == MP_MODEL_HIER) return hier_fcs();
  if (model == MP_MODEL_ATTN) return {"afc_1", "afc_out"};
  return std::vector<std::string>(std::begin(kDenseFc), std::end(kDenseFc));
}

int same_out(int in, int s) { return (in + s - 1) / s; }
int same_pad_before(int in, int k, int s) {
  const int out = same_out(in, s);
  const int tot = std::max((out - 1) * s + k - in, 0);
  return tot / 2;
}

// a channel range of an NHWC buffer
struct View {
  float* p;
  int ld, coff, C, H, W;
};

float* buf(mp_ctx* c, const std::string& name, size_t floats) {
  DevBuf& d = c->ws[name];
  d.alloc(floats * sizeof(float));
  return d.f();
}

void conv(mp_ctx* c, const std::string& name, int n, const View& in, const View& out, int stride,
          hipStream_t st) {
  auto it = c->layers.find(name);
  if (it == c->layers.end()) fail(MP_ERR_STATE, "conv layer missing: " + name);
  const auto& L = it->second;
  if (L.cin != in.C || L.cout != out.C) fail(MP_ERR_SHAPE, "conv " + name + ": channel mismatch");
  IgemmArgs a{};
  a.x = in.p;
  a.ldx = in.ld;
  a.cix = in.coff;
  a.N = n;
  a.H = in.H;
  a.W = in.W;
  a.Cin = in.C;
  a.wpk = L.w.v4();
  a.K = L.K;
  a.bias = L.b.f();
  a.out = out.p;
  a.ldo = out.ld;
  a.coff = out.coff;
  a.Cout = out.C;
  a.KS = L.k;
  a.stride = stride;
  a.Ho = same_out(in.H, stride);
  a.Wo = same_out(in.W, stride);
  if (a.Ho != out.H || a.Wo != out.W) fail(MP_ERR_SHAPE, "conv " + name + ": spatial mismatch");
  a.pad_t = same_pad_before(in.H, L.k, stride);
  a.pad_l = same_pad_before(in.W, L.k, stride);
  a.relu = 1;
  a.nprod = L.nprod;
  if (L.cinp) {   // the Cin-padded packing for the halo kernel
    a.wpad = L.wpad.p;
    a.cinp = L.cinp;
  }
  hip_check(L.x3 ? launch_igemm_x3(a, L.w.p, L.wus, st) : launch_igemm_conv(a, st), name.c_str());
}

void pool(int n, const View& in, const View& out, int mode, hipStream_t st, const float* aff_s = nullptr,
          const float* aff_t = nullptr) {
  if (out.H != same_out(in.H, 2) || out.W != same_out(in.W, 2) || out.C != in.C)
    fail(MP_ERR_SHAPE, "pool shape mismatch");
  hip_check(launch_pool2(in.p, in.ld, in.coff, n, in.H, in.W, in.C, out.p, out.ld, out.coff, mode, st, aff_s, aff_t),
            "pool");
}

void fcl(mp_ctx* c, const std::string& name, int n, const float* in, int K, float* out, int ldo, bool relu,
         hipStream_t st, const float* aff_s = nullptr, const float* aff_t = nullptr) {
  auto it = c->layers.find(name);
  if (it == c->layers.end()) fail(MP_ERR_STATE, "fc layer missing: " + name);
  const auto& L = it->second;
  if (L.K != K) fail(MP_ERR_SHAPE, "fc " + name + ": input size " + std::to_string(K) + " != " + std::to_string(L.K));
  int ks;
  const int S = fc_choose_splits(n, K, L.cout, &ks);
  float* part = buf(c, "fc_part", (size_t)S * n * ((L.cout + 31) / 32 * 32));
  hip_check(L.x3 ? launch_fc_gemm_x3(in, K, L.w.p, L.wus, part, n, K, L.cout, S, ks, st, L.nprod)
                 : launch_fc_gemm(in, K, L.w.v4(), part, n, K, L.cout, S, ks, st),
            name.c_str());
  hip_check(launch_fc_reduce(part, S, n, L.cout, L.b.f(), relu ? 1 : 0, aff_s, aff_t, out, ldo, st),
            name.c_str());
}

View V(float* p, int ld, int coff, int C, int H, int W) { return View{p, ld, coff, C, H, W}; }

// ------------------------------------------------------------------------------- dense forward
void dense_forward(mp_ctx* c, const float* depth, int n, int H, int W, float* out, hipStream_t st) {
  const int H1 = same_out(H, 2), W1 = same_out(W, 2);
  const int H2 = same_out(H1, 2), W2 = same_out(W1, 2);
  const int H3 = same_out(H2, 2), W3 = same_out(W2, 2);
  const int S1C = 16 + 24 + 32 + 48 + 64 + 96;                            // 280
  const int S2C = 24 + 56 + 96 + 128 + 192 + 256;                         // 752
  const int S3C = 32 + 80 + 128 + 192 + 256 + 288;                        // 976
  float* c0 = buf(c, "c0", (size_t)n * H * W * 12);
  float* p0 = buf(c, "p0", (size_t)n * H1 * W1 * 12);
  float* s1 = buf(c, "s1", (size_t)n * H1 * W1 * S1C);
  float* s2 = buf(c, "s2", (size_t)n * H2 * W2 * S2C);
  float* s3 = buf(c, "s3", (size_t)n * H3 * W3 * S3C);
  float* tb = buf(c, "t", (size_t)n * H1 * W1 * 128);
  const View x = V(const_cast<float*>(depth), 1, 0, 1, H, W);
  conv(c, "conv_0", n, x, V(c0, 12, 0, 12, H, W), 1, st);                                   // 226
  pool(n, V(c0, 12, 0, 12, H, W), V(p0, 12, 0, 12, H1, W1), 0, st);                         // 227
  conv(c, "conv_1_1", n, V(p0, 12, 0, 12, H1, W1), V(s1, S1C, 0, 16, H1, W1), 1, st);       // 230
  conv(c, "conv_1_2", n, V(s1, S1C, 0, 16, H1, W1), V(s2, S2C, 0, 24, H2, W2), 2, st);      // 231
  conv(c, "conv_1_3", n, V(s2, S2C, 0, 24, H2, W2), V(s3, S3C, 0, 32, H3, W3), 2, st);      // 232
  conv(c, "conv_2_1", n, V(s1, S1C, 0, 16, H1, W1), V(s1, S1C, 16, 24, H1, W1), 1, st);     // 236
  conv(c, "conv_2_2_1", n, V(s1, S1C, 0, 16, H1, W1), V(s2, S2C, 24, 24, H2, W2), 2, st);   // 238
  conv(c, "conv_2_2_2", n, V(s2, S2C, 0, 24, H2, W2), V(s2, S2C, 48, 32, H2, W2), 1, st);   // 239
  conv(c, "conv_2_3_2", n, V(s2, S2C, 0, 24, H2, W2), V(s3, S3C, 32, 32, H3, W3), 2, st);   // 242
  conv(c, "conv_2_3_3", n, V(s3, S3C, 0, 32, H3, W3), V(s3, S3C, 64, 48, H3, W3), 1, st);   // 243
  int w1 = 40, w2 = 80, w3 = 112;
  for (int L = 3; L <= 6; ++L) {                                                             // 248-373
    const int* d = kDenseW[L - 3];
    const std::string p = "conv_" + std::to_string(L);
    conv(c, p + "_1_1x1", n, V(s1, S1C, 0, w1, H1, W1), V(tb, d[0], 0, d[0], H1, W1), 1, st);
    conv(c, p + "_1", n, V(tb, d[0], 0, d[0], H1, W1), V(s1, S1C, w1, d[1], H1, W1), 1, st);
    conv(c, p + "_2_1x1_1", n, V(s1, S1C, 0, w1, H1, W1), V(tb, d[2], 0, d[2], H1, W1), 1, st);
    conv(c, p + "_2_1", n, V(tb, d[2], 0, d[2], H1, W1), V(s2, S2C, w2, d[3], H2, W2), 2, st);
    conv(c, p + "_2_1x1_2", n, V(s2, S2C, 0, w2, H2, W2), V(tb, d[4], 0, d[4], H2, W2), 1, st);
    conv(c, p + "_2_2", n, V(tb, d[4], 0, d[4], H2, W2), V(s2, S2C, w2 + d[3], d[5], H2, W2), 1, st);
    conv(c, p + "_3_1x1_2", n, V(s2, S2C, 0, w2, H2, W2), V(tb, d[6], 0, d[6], H2, W2), 1, st);
    conv(c, p + "_3_2", n, V(tb, d[6], 0, d[6], H2, W2), V(s3, S3C, w3, d[7], H3, W3), 2, st);
    conv(c, p + "_3_1x1_3", n, V(s3, S3C, 0, w3, H3, W3), V(tb, d[8], 0, d[8], H3, W3), 1, st);
    conv(c, p + "_3_3", n, V(tb, d[8], 0, d[8], H3, W3), V(s3, S3C, w3 + d[7], d[9], H3, W3), 1, st);
    w1 += d[1];
    w2 += d[3] + d[5];
    w3 += d[7] + d[9];
  }
  // avg pools of conv6_{1,2,3} = the last 96 / 256 / 288 channels of each scale buffer (376-378)
  const int Q1 = same_out(H1, 2) * same_out(W1, 2), Q2 = same_out(H2, 2) * same_out(W2, 2),
            Q3 = same_out(H3, 2) * same_out(W3, 2);
  float* pl1 = buf(c, "pool1", (size_t)n * Q1 * 96);
  float* pl2 = buf(c, "pool2", (size_t)n * Q2 * 256);
  float* pl3 = buf(c, "pool3", (size_t)n * Q3 * 288);
  pool(n, V(s1, S1C, S1C - 96, 96, H1, W1), V(pl1, 96, 0, 96, same_out(H1, 2), same_out(W1, 2)), 1, st);
  pool(n, V(s2, S2C, S2C - 256, 256, H2, W2), V(pl2, 256, 0, 256, same_out(H2, 2), same_out(W2, 2)), 1, st);
  pool(n, V(s3, S3C, S3C - 288, 288, H3, W3), V(pl3, 288, 0, 288, same_out(H3, 2), same_out(W3, 2)), 1, st);
  float* cat = buf(c, "cat", (size_t)n * 1536);
  fcl(c, "fc_1_1", n, pl1, Q1 * 96, cat, 1536, true, st);                                    // 381-383
  fcl(c, "fc_1_2", n, pl2, Q2 * 256, cat + 512, 1536, true, st);                             // 386-388
  fcl(c, "fc_1_3", n, pl3, Q3 * 288, cat + 1024, 1536, true, st);                            // 391-393
  float* h2 = buf(c, "h2", (size_t)n * 1024);
  float* h3 = buf(c, "h3", (size_t)n * 512);
  fcl(c, "fc_2", n, cat, 1536, h2, 1024, true, st);                                          // 396-397
  fcl(c, "fc_3", n, h2, 1024, h3, 512, true, st);                                            // 401-402
  const int nout = c->layers["fc_4"].cout;
  fcl(c, "fc_4", n, h3, 512, out, nout, false, st);                                          // 406-408
}

// -------------------------------------------------------------------------------- hier forward
void hier_forward(mp_ctx* c, const float* depth, int n, int H, int W, float* const* outs, hipStream_t st) {
  int h = H, w = W;
  const View x = V(const_cast<float*>(depth), 1, 0, 1, h, w);
  float* a = buf(c, "c1", (size_t)n * h * w * 64);
  conv(c, "conv_1", n, x, V(a, 64, 0, 64, h, w), 1, st);                                     // 341
  int h2 = same_out(h, 2), w2 = same_out(w, 2);
  float* b = buf(c, "p1", (size_t)n * h2 * w2 * 64);
  pool(n, V(a, 64, 0, 64, h, w), V(b, 64, 0, 64, h2, w2), 0, st);
  float* c2 = buf(c, "c2", (size_t)n * h2 * w2 * 128);
  conv(c, "conv_2", n, V(b, 64, 0, 64, h2, w2), V(c2, 128, 0, 128, h2, w2), 1, st);          // 344
  const int h4 = same_out(h2, 2), w4 = same_out(w2, 2);
  float* p2 = buf(c, "p2", (size_t)n * h4 * w4 * 128);
  pool(n, V(c2, 128, 0, 128, h2, w2), V(p2, 128, 0, 128, h4, w4), 0, st);
  const int h8 = same_out(h4, 2), w8 = same_out(w4, 2), h16 = same_out(h8, 2), w16 = same_out(w8, 2);
  const int h32 = same_out(h16, 2), w32 = same_out(w16, 2), h64 = same_out(h32, 2), w64 = same_out(w32, 2);
  float* t3 = buf(c, "t3", (size_t)n * h4 * w4 * 256);
  float* t3p = buf(c, "t3p", (size_t)n * h8 * w8 * 256);
  float* t4 = buf(c, "t4", (size_t)n * h8 * w8 * 512);
  std::map<std::string, float*> trunk;
  for (const char* br : {"pr", "mi", "t"}) {                                                 // 347-352 ...
    float* o = buf(c, std::string("b4_") + br, (size_t)n * h16 * w16 * 512);
    conv(c, std::string(br) + "_con_3", n, V(p2, 128, 0, 128, h4, w4), V(t3, 256, 0, 256, h4, w4), 1, st);
    pool(n, V(t3, 256, 0, 256, h4, w4), V(t3p, 256, 0, 256, h8, w8), 0, st);
    conv(c, std::string(br) + "_con_4", n, V(t3p, 256, 0, 256, h8, w8), V(t4, 512, 0, 512, h8, w8), 1, st);
    pool(n, V(t4, 512, 0, 512, h8, w8), V(o, 512, 0, 512, h16, w16), 0, st);
    trunk[br] = o;
  }
  const char* src5[] = {"pr", "pr", "mi", "mi", "t"};
  float* t5 = buf(c, "t5", (size_t)n * h16 * w16 * 512);
  float* t5p = buf(c, "t5p", (size_t)n * h32 * w32 * 512);
  float* t6 = buf(c, "t6", (size_t)n * h32 * w32 * 1024);
  const int flat = h64 * w64 * 1024;
  float* a1 = buf(c, "a1", (size_t)n * 1024);
  float* a2 = buf(c, "a2", (size_t)n * 1024);
  float* hc = buf(c, "hc", (size_t)n * 5120);
  for (int f = 0; f < 5; ++f) {                                                              // 354-469
    const std::string F = kFingers[f];
    float* p6 = buf(c, "p6_" + F, (size_t)n * flat);
    conv(c, F + "_con_5", n, V(trunk[src5[f]], 512, 0, 512, h16, w16), V(t5, 512, 0, 512, h16, w16), 1, st);
    pool(n, V(t5, 512, 0, 512, h16, w16), V(t5p, 512, 0, 512, h32, w32), 0, st);
    conv(c, F + "_con_6", n, V(t5p, 512, 0, 512, h32, w32), V(t6, 1024, 0, 1024, h32, w32), 1, st);
    pool(n, V(t6, 1024, 0, 1024, h32, w32), V(p6, 1024, 0, 1024, h64, w64), 0, st);
    fcl(c, F + "_fc_1", n, p6, flat, a1, 1024, true, st);
    fcl(c, F + "_fc_2", n, a1, 1024, a2, 1024, true, st);
    fcl(c, F + "_fc_3", n, a2, 1024, outs[1 + f], c->layers[F + "_fc_3"].cout, false, st);
  }
  for (int f = 0; f < 5; ++f) {                                                              // 473-523
    const std::string F = kFingers[f];
    fcl(c, F + "h_fc_1", n, c->ws["p6_" + F].f(), flat, a1, 1024, true, st);
    fcl(c, F + "h_fc_2", n, a1, 1024, hc + 1024 * f, 5120, true, st);
  }
  fcl(c, "final_fc_1", n, hc, 5120, a1, 1024, true, st);                                     // 525-526
  fcl(c, "final_fc_2", n, a1, 1024, outs[0], c->layers["final_fc_2"].cout, false, st);       // 529-530
}

// ---------------------------------------------------------------------------- attention forward
// attn_model_struct.build (train_cnn_networks_hgru.py:436-525), inference: resize to 128x128,
// five [conv + relu -> 2x2 max pool -> BN] stages, afc_1 + relu -> BN, afc_out.  The BN of each
// stage runs in the pool kernel's epilogue, the last one in the afc_1 split-K reduction.
void attn_forward(mp_ctx* c, const float* frames, int n, int H, int W, float* out, hipStream_t st) {
  float* x = const_cast<float*>(frames);
  if (H != ATTN_SIZE || W != ATTN_SIZE) {
    x = buf(c, "resized", (size_t)n * ATTN_SIZE * ATTN_SIZE);
    hip_check(launch_resize_bilinear(frames, n, H, W, 1, x, ATTN_SIZE, ATTN_SIZE, st), "resize");
  }
  int h = ATTN_SIZE, w = ATTN_SIZE, cin = 1;
  View cur = V(x, 1, 0, 1, h, w);
  const auto specs = attn_convs();
  for (size_t i = 0; i < specs.size(); ++i) {                                                  // 440-476
    const auto& s = specs[i];
    const auto& L = c->layers[s.name];
    const int h2 = same_out(h, 2), w2 = same_out(w, 2);
    if (i == 0 && h % 2 == 0 && w % 2 == 0) {
      // aconv_1 (1 -> 64, 3x3) + apool_1 + BN in one pass (the hGRU backbone's conv_1 kernel, NHWC
      // out): the 4 MiB-per-frame pre-pool map is never written
      float* pl = buf(c, "attn_pool_a", (size_t)n * h2 * w2 * 64);
      hip_check(launch_conv1_pool_bn(x, c->raw.at("aconv_1/aconv_1_filters").dev->f(), L.b.f(), L.bn_s.f(),
                                     L.bn_t.f(), pl, n, h, w, st, true),
                "aconv_1 + apool_1");
      cur = V(pl, 64, 0, 64, h2, w2);
      h = h2;
      w = w2;
      cin = 64;
      continue;
    }
    float* cv = buf(c, "attn_conv", (size_t)n * h * w * s.cout);
    conv(c, s.name, n, cur, V(cv, s.cout, 0, s.cout, h, w), 1, st);
    float* pl = buf(c, i % 2 ? "attn_pool_b" : "attn_pool_a", (size_t)n * h2 * w2 * s.cout);
    pool(n, V(cv, s.cout, 0, s.cout, h, w), V(pl, s.cout, 0, s.cout, h2, w2), 0, st, L.bn_s.f(), L.bn_t.f());
    cur = V(pl, s.cout, 0, s.cout, h2, w2);
    h = h2;
    w = w2;
    cin = s.cout;
  }
  float* h1 = buf(c, "attn_fc1", (size_t)n * 1024);
  const auto& F1 = c->layers["afc_1"];
  fcl(c, "afc_1", n, cur.p, h * w * cin, h1, F1.cout, true, st, F1.bn_s.f(), F1.bn_t.f());     // 478-490
  fcl(c, "afc_out", n, h1, F1.cout, out, c->layers["afc_out"].cout, false, st);                // 502-503
}

}  // namespace

namespace mpr {

bool known_name_regressor(int model, const std::string& n) {
  for (const auto& s : convs_of(model))
    if (n == s.name + "/" + s.name + "_filters" || n == s.name + "/" + s.name + "_biases") return true;
  for (const auto& f : fcs_of(model))
    if (n == f + "/" + f + "_weights" || n == f + "/" + f + "_biases") return true;
  if (model == MP_MODEL_ATTN)
    for (const char* b : kAttnBn)
      for (const char* v : {"gamma", "beta", "moving_mean", "moving_variance"})
        if (n == std::string(b) + "/" + v) return true;
  return false;
}

// a conv (HWIO as [K][Cout]) or fc ([K][N]) weight in the context's precision: fp32 fragments, or
// the f16x3 split under MP_DTYPE_F32_SPLIT when the x3 kernel takes the shape (x3_ok)
void pack_matrix(mp_ctx* c, mp_ctx::PackedLayer& L, const float* w, bool x3_ok) {
  // MP_DTYPE_BF16 keeps the split packing and runs its hi x hi product only (L.nprod = 1)
  L.x3 = (c->dtype == MP_DTYPE_F32_SPLIT || c->dtype == MP_DTYPE_BF16) && x3_ok;
  L.nprod = c->dtype == MP_DTYPE_BF16 ? 1 : 3;
  if (L.x3) {
    L.w.alloc(fc_x3_bytes(L.K, L.cout));
    hip_check(launch_pack_fc_x3(w, L.w.p, L.K, L.cout, &L.wus, nullptr), "pack (f16x3)");
    // 3x3 / 5x5 convs whose Cin is not a multiple of 32: a second packing with each tap's rows
    // zero-padded to a multiple of 16 or 32, for the halo kernel (zero rows leave max|W|, so the scale, and
    // every real weight's hi / lo split unchanged)
    if ((L.k == 3 || L.k == 5) && L.cin % 32 && L.cin % 4 == 0 && L.K == L.k * L.k * L.cin) {
      // the smaller of the 16- and 32-multiples (16-channel halo chunks when that is not one of 32)
      L.cinp = (L.cin + 15) / 16 * 16 < (L.cin + 31) / 32 * 32 ? (L.cin + 15) / 16 * 16 : (L.cin + 31) / 32 * 32;
      const int taps = L.k * L.k, Kp = taps * L.cinp;
      DevBuf tmp;
      tmp.alloc((size_t)Kp * L.cout * sizeof(float));
      hip_check(launch_pad_cin(w, tmp.f(), taps, L.cin, L.cinp, L.cout, nullptr), "pad Cin");
      L.wpad.alloc(fc_x3_bytes(Kp, L.cout));
      float us = 0.f;
      hip_check(launch_pack_fc_x3(tmp.f(), L.wpad.p, Kp, L.cout, &us, nullptr), "pack (f16x3, Cin padded)");
      hip_check(hipDeviceSynchronize(), "pad Cin sync");
      if (us != L.wus) fail(MP_ERR_STATE, "padded packing changed the weight scale");
    }
  } else {
    L.w.alloc((size_t)((L.K + 7) / 8) * ((L.cout + 31) / 32) * 64 * 16);
    hip_check(launch_pack_fc(w, L.w.v4(), L.K, L.cout, nullptr), "pack");
  }
}

void finalize_regressor(mp_ctx* c) {
  c->layers.clear();
  for (const auto& s : convs_of(c->model)) {
    const auto& w = c->need(s.name + "/" + s.name + "_filters", {s.k, s.k, s.cin, s.cout});
    const auto& b = c->need(s.name + "/" + s.name + "_biases", {s.cout});
    auto& L = c->layers[s.name];
    L.k = s.k;
    L.cin = s.cin;
    L.cout = s.cout;
    L.K = s.k * s.k * s.cin;
    pack_matrix(c, L, w.dev->f(), L.K >= 4);
    L.b.alloc(s.cout * sizeof(float));
    hip_check(hipMemcpy(L.b.p, b.dev->p, s.cout * sizeof(float), hipMemcpyDeviceToDevice), "bias");
  }
  for (const auto& f : fcs_of(c->model)) {
    auto it = c->raw.find(f + "/" + f + "_weights");
    if (it == c->raw.end()) fail(MP_ERR_STATE, "weight not set: " + f + "/" + f + "_weights");
    if (it->second.shape.size() != 2) fail(MP_ERR_WEIGHT, f + " weights must be 2-D");
    const int K = (int)it->second.shape[0], N = (int)it->second.shape[1];
    const auto& b = c->need(f + "/" + f + "_biases", {N});
    auto& L = c->layers[f];
    L.K = K;
    L.cin = K;
    L.cout = N;
    pack_matrix(c, L, it->second.dev->f(), K % 32 == 0);
    L.b.alloc(N * sizeof(float));
    hip_check(hipMemcpy(L.b.p, b.dev->p, N * sizeof(float), hipMemcpyDeviceToDevice), "bias");
  }
  if (c->model == MP_MODEL_ATTN) {
    const auto specs = attn_convs();
    for (size_t i = 0; i < specs.size(); ++i) {
      auto& L = c->layers[specs[i].name];
      bn_fold(c, kAttnBn[i], L.cout, L.bn_s, L.bn_t);
    }
    auto& F1 = c->layers["afc_1"];
    if (F1.K != 4 * 4 * 1024) fail(MP_ERR_WEIGHT, "afc_1 must be [16384, N] (4x4x1024 after apool_5)");
    if (c->layers["afc_out"].K != F1.cout) fail(MP_ERR_WEIGHT, "afc_out input size != afc_1 output size");
    bn_fold(c, kAttnBn[5], F1.cout, F1.bn_s, F1.bn_t);
  }
  c->head_sizes.clear();
  if (c->model == MP_MODEL_ATTN) {
    c->head_sizes.push_back(c->layers["afc_out"].cout);
  } else if (c->model == MP_MODEL_DENSE) {
    c->head_sizes.push_back(c->layers["fc_4"].cout);
  } else {
    c->head_sizes.push_back(c->layers["final_fc_2"].cout);
    for (const char* f : kFingers) c->head_sizes.push_back(c->layers[std::string(f) + "_fc_3"].cout);
  }
}

}  // namespace mpr

extern "C" {

int mp_dense_fwd(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, float* out, void* stream) {
  return guard([&] {
    if (!ctx || !depth || !out) fail(MP_ERR_ARG, "mp_dense_fwd: null pointer");
    if (ctx->model != MP_MODEL_DENSE) fail(MP_ERR_STATE, "context is not a dense model");
    if (!ctx->finalized) fail(MP_ERR_STATE, "weights not finalized");
    if (n <= 0 || n > (1 << 20) || h < 8 || w < 8) fail(MP_ERR_SHAPE, "bad input shape");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    ProfScope ps(ctx, static_cast<hipStream_t>(stream), "dense");
    dense_forward(ctx, depth, (int)n, (int)h, (int)w, out, static_cast<hipStream_t>(stream));
  });
}

int mp_hier_fwd(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, float* const* outs,
                void* stream) {
  return guard([&] {
    if (!ctx || !depth || !outs) fail(MP_ERR_ARG, "mp_hier_fwd: null pointer");
    for (int i = 0; i < 6; ++i)
      if (!outs[i]) fail(MP_ERR_ARG, "mp_hier_fwd: null output pointer");
    if (ctx->model != MP_MODEL_HIER) fail(MP_ERR_STATE, "context is not a hierarchical model");
    if (!ctx->finalized) fail(MP_ERR_STATE, "weights not finalized");
    if (n <= 0 || n > (1 << 20) || h < 64 || w < 64) fail(MP_ERR_SHAPE, "bad input shape");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    ProfScope ps(ctx, static_cast<hipStream_t>(stream), "hier");
    hier_forward(ctx, depth, (int)n, (int)h, (int)w, outs, static_cast<hipStream_t>(stream));
  });
}

int mp_attn_fwd(mp_ctx* ctx, const float* frames, int64_t n, int64_t h, int64_t w, float* out, void* stream) {
  return guard([&] {
    if (!ctx || !frames || !out) fail(MP_ERR_ARG, "mp_attn_fwd: null pointer");
    if (ctx->model != MP_MODEL_ATTN) fail(MP_ERR_STATE, "context is not an attention model");
    if (!ctx->finalized) fail(MP_ERR_STATE, "weights not finalized");
    if (n <= 0 || n > (1 << 20) || h < 1 || w < 1 || h > 8192 || w > 8192) fail(MP_ERR_SHAPE, "bad input shape");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    ProfScope ps(ctx, static_cast<hipStream_t>(stream), "attn");
    attn_forward(ctx, frames, (int)n, (int)h, (int)w, out, static_cast<hipStream_t>(stream));
  });
}

int mp_resize_bilinear(const float* x, int64_t n, int64_t h, int64_t w, int64_t c, int64_t ho, int64_t wo,
                       float* out, void* stream) {
  return guard([&] {
    if (!x || !out) fail(MP_ERR_ARG, "mp_resize_bilinear: null pointer");
    if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || ho <= 0 || wo <= 0 || h > 65536 || w > 65536 || ho > 65536 ||
        wo > 65536 || n * ho * wo * c > ((int64_t)1 << 40))
      fail(MP_ERR_SHAPE, "mp_resize_bilinear: bad shape");
    hip_check(launch_resize_bilinear(x, (int)n, (int)h, (int)w, (int)c, out, (int)ho, (int)wo,
                                     static_cast<hipStream_t>(stream)),
              "resize");
  });
}

}  // extern "C"
