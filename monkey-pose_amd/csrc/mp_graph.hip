// Layer-graph runtime (MP_MODEL_GRAPH): plans and runs a graph recorded by a facade from the
// reference's TF1 graph-builder calls (conv_layer / max_pool / avg_pool / tf.concat / fc_layer /
// tf.nn.relu / tf.identity, train_dense_hier_networks.py:338-2382 and helpers 2416-2455).
//
// Planning, once per input shape (n, h, w):
//   1. shapes: SAME arithmetic (conv: ceil(h / stride); pool: ceil(h / k));
//   2. aliases: identity -> its source; relu of a conv / pool / concat of non-negative tensors ->
//      its source; relu of an fc output consumed only by it -> the fc with a relu epilogue;
//   3. placement: every tf.concat is a constraint "source i starts at channel offset o_i of the
//      output"; a weighted union-find merges the constraints into groups, one wide NHWC buffer per
//      group, so producers write straight into their channel range and concat launches nothing;
//   4. schedule: the kernel ops as a dependency DAG over up to MP_GRAPH_STREAMS (default 8)
//      streams: an op continues the stream whose last op it consumes, else takes the least
//      recently used stream; cross-stream edges become events, pruned by vector clocks.
//      (A hipGraph replay of the same DAG measured slower on this ROCm and was removed in round 4:
//      DESIGN.md section 3c.)
// Activations: x is copied into a graph-owned input buffer and outputs copied out, so the plan
// only ever sees its own pointers.
#include <algorithm>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <numeric>

#include "mp_runtime.hpp"

struct GraphState {
  struct Op {
    int kind, out, ksize, stride, cout;
    std::vector<int> src;
    std::string name;
  };
  std::vector<Op> ops;
  std::vector<int> outputs;
  int in_channels = 1;
  int n_tensors = 0;

  // ---- plan (valid for n, h, w) ----
  struct Tensor {
    int H = 0, W = 0, C = 0;
    bool rank2 = false;      // fc output [n, C]
    bool nonneg = false;     // relu'd values (a relu on it is the identity)
    int alias = -1;          // tensor whose storage this is
    int group = -1;          // placement group (buffer)
    int off = 0;             // channel offset inside the group
    std::vector<int> prod;   // kernel ops that write it
  };
  struct Group {
    int H = 0, W = 0, span = 0;
    bool rank2 = false;
    mpr::DevBuf buf;
  };
  struct Kern {
    int op;                  // index into ops
    int kind;                // MP_OP_CONV / MAXPOOL / AVGPOOL / FC
    bool relu = false;       // fc epilogue
    int stream = 0;
    bool record = false;     // a later op on another stream waits for it
    std::vector<int> waits;  // kernel indices on other streams to wait for
    IgemmArgs ia{};
    // pool
    const float* px = nullptr;
    int pld = 0, pcix = 0, pH = 0, pW = 0, pC = 0, pldo = 0, pcoff = 0;
    float* pout = nullptr;
    // fc
    const float* fa = nullptr;
    int fK = 0, fN = 0, fS = 1, fks = 0, fldo = 0;
    float* fout = nullptr;
    mpr::DevBuf part;
    const mp_ctx::PackedLayer* L = nullptr;
    // fused 1-channel 3x3 conv + relu + 2x2 max pool (KIND_CONV1_POOL)
    const float *cw = nullptr, *cb = nullptr;
    int cH = 0, cW = 0;
    mpr::DevBuf ones, zeros;
  };
  // concatenated packings of fused 1x1 sibling convs, keyed by their names; kept across re-plans
  std::map<std::string, std::unique_ptr<mp_ctx::PackedLayer>> fused1x1;
  int n_fused_1x1 = 0;   // this plan's 1x1 convs computed by a sibling's kernel
  int64_t pn = 0, ph = 0, pw = 0;
  bool planned = false;
  std::vector<Tensor> t;
  std::vector<std::unique_ptr<Group>> groups;
  std::vector<std::unique_ptr<Kern>> kerns;
  int n_streams = 1;
  mpr::DevBuf input;
  std::vector<hipStream_t> streams;     // [0] = capture / eager main stream owned by the graph
  std::vector<hipEvent_t> kev;          // per kernel (those with record)
  std::vector<hipEvent_t> joins;        // per side stream
  hipEvent_t fork = nullptr;
  ~GraphState() {
    for (auto e : kev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : joins) (void)hipEventDestroy(e);
    if (fork) (void)hipEventDestroy(fork);
    for (auto s : streams) (void)hipStreamDestroy(s);
  }
};

namespace mpr {
namespace {

int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : dflt;
}

bool dbg() {
  static const int v = env_int("MP_GRAPH_DEBUG", 0);
  return v != 0;
}
#define GDBG(...)                       \
  do {                                  \
    if (dbg()) {                        \
      fprintf(stderr, "[mp_graph] " __VA_ARGS__); \
      fputc('\n', stderr);             \
      fflush(stderr);                   \
    }                                   \
  } while (0)

int same_out(int in, int s) { return (in + s - 1) / s; }
int same_pad_before(int in, int k, int s) {
  const int tot = std::max((same_out(in, s) - 1) * s + k - in, 0);
  return tot / 2;
}

// weighted union-find: pos(x) = pos(root) + w[x]
struct UF {
  std::vector<int> p, w;
  explicit UF(int n) : p(n), w(n, 0) { std::iota(p.begin(), p.end(), 0); }
  int find(int x) {
    if (p[x] == x) return x;
    const int r = find(p[x]);
    w[x] += w[p[x]];
    p[x] = r;
    return r;
  }
  // require pos(a) = pos(b) + d; false on a contradiction
  bool unite(int a, int b, int d) {
    const int ra = find(a), rb = find(b);
    if (ra == rb) return w[a] == w[b] + d;
    // pos(ra) = pos(a) - w[a] = pos(b) + d - w[a] = pos(rb) + w[b] + d - w[a]
    p[ra] = rb;
    w[ra] = w[b] + d - w[a];
    return true;
  }
};

using G = GraphState;

// internal kernel kind: conv (1 -> 64 channels, 3x3, stride 1) + relu + 2x2 max pool in one pass,
// for a conv whose only consumer is that pool (hier conv_1 -> pool_1): the pre-pool map is never
// written (the hGRU backbone's conv_1 kernel, NHWC out, unit affine)
constexpr int KIND_CONV1_POOL = 100;

// 1x1 sibling fusion: the one packing of several 1x1 convs over the same input, output channels
// concatenated in member order (weights [Cin][sum Cout], one power-of-two scale from their joint
// max|W|: the split stays 22 bits relative to that max, i.e. fp32-accurate, but not bit-identical to
// the separate packings)
const mp_ctx::PackedLayer& fused_1x1_pack(mp_ctx* c, G& g, const std::vector<int>& mem) {
  std::string key;
  int tot = 0;
  for (int m : mem) {
    key += g.ops[m].name + "+";
    tot += g.ops[m].cout;
  }
  auto& slot = g.fused1x1[key];
  if (slot) return *slot;
  slot = std::make_unique<mp_ctx::PackedLayer>();
  auto& F = *slot;
  const auto& L0 = c->layers.at(g.ops[mem[0]].name);
  F.k = 1;
  F.cin = L0.cin;
  F.K = L0.cin;
  F.cout = tot;
  F.x3 = true;
  F.nprod = L0.nprod;
  mpr::DevBuf tmp;
  tmp.alloc((size_t)F.K * tot * sizeof(float));
  F.b.alloc((size_t)tot * sizeof(float));
  int off = 0;
  for (int m : mem) {
    const auto& op = g.ops[m];
    const float* w = c->raw.at(op.name + "/" + op.name + "_filters").dev->f();   // HWIO [1][1][Cin][Cout]
    hip_check(hipMemcpy2D(tmp.f() + off, (size_t)tot * sizeof(float), w, (size_t)op.cout * sizeof(float),
                          (size_t)op.cout * sizeof(float), F.K, hipMemcpyDeviceToDevice),
              "fused 1x1 weights");
    hip_check(hipMemcpy(F.b.f() + off, c->layers.at(op.name).b.p, (size_t)op.cout * sizeof(float),
                        hipMemcpyDeviceToDevice),
              "fused 1x1 bias");
    off += op.cout;
  }
  F.w.alloc(fc_x3_bytes(F.K, tot));
  hip_check(launch_pack_fc_x3(tmp.f(), F.w.p, F.K, tot, &F.wus, nullptr), "pack fused 1x1");
  hip_check(hipDeviceSynchronize(), "pack fused 1x1");
  return F;
}

void plan(mp_ctx* c, G& g, int64_t n, int64_t h, int64_t w) {
  g.planned = false;
  g.kerns.clear();
  g.groups.clear();
  const int NT = g.n_tensors;
  g.t.assign(NT, G::Tensor{});
  auto& T = g.t;
  T[0].H = (int)h;
  T[0].W = (int)w;
  T[0].C = g.in_channels;
  std::vector<int> uses(NT, 0), def(NT, -1);
  for (size_t i = 0; i < g.ops.size(); ++i) {
    def[g.ops[i].out] = (int)i;
    for (int s : g.ops[i].src) ++uses[s];
  }
  for (int o : g.outputs) ++uses[o];
  auto root = [&](int x) {
    while (T[x].alias >= 0) x = T[x].alias;
    return x;
  };
  std::vector<int> fc_relu(g.ops.size(), 0);
  // 1 + 2: shapes and aliases
  for (size_t i = 0; i < g.ops.size(); ++i) {
    const auto& op = g.ops[i];
    auto& o = T[op.out];
    const auto& s0 = T[op.src[0]];
    switch (op.kind) {
      case MP_OP_CONV: {
        if (s0.rank2) fail(MP_ERR_SHAPE, "conv " + op.name + " on a rank-2 tensor");
        o.H = same_out(s0.H, op.stride);
        o.W = same_out(s0.W, op.stride);
        o.C = op.cout;
        o.nonneg = true;
        break;
      }
      case MP_OP_MAXPOOL:
      case MP_OP_AVGPOOL:
        if (s0.rank2) fail(MP_ERR_SHAPE, "pool on a rank-2 tensor");
        o.H = same_out(s0.H, op.ksize);
        o.W = same_out(s0.W, op.ksize);
        o.C = s0.C;
        o.nonneg = s0.nonneg;
        break;
      case MP_OP_CONCAT: {
        o.H = s0.H;
        o.W = s0.W;
        o.rank2 = s0.rank2;
        o.nonneg = true;
        for (int s : op.src) {
          if (T[s].H != o.H || T[s].W != o.W || T[s].rank2 != o.rank2)
            fail(MP_ERR_SHAPE, "tf.concat of tensors with different spatial shapes (tensor " +
                                   std::to_string(op.out) + ")");
          o.C += T[s].C;
          o.nonneg = o.nonneg && T[s].nonneg;
        }
        break;
      }
      case MP_OP_FC:
        o.H = o.W = 1;
        o.rank2 = true;
        o.C = op.cout;
        break;
      case MP_OP_IDENTITY:
      case MP_OP_RELU: {
        o.H = s0.H;
        o.W = s0.W;
        o.C = s0.C;
        o.rank2 = s0.rank2;
        o.nonneg = s0.nonneg;
        o.alias = op.src[0];
        if (op.kind == MP_OP_RELU && !s0.nonneg) {
          const int r = root(op.src[0]);
          const int d = def[r];
          if (d < 0 || g.ops[d].kind != MP_OP_FC || uses[r] != 1 || r != op.src[0])
            fail(MP_ERR_UNSUPPORTED, "tf.nn.relu is supported after fc_layer (sole consumer) or on relu'd tensors");
          fc_relu[d] = 1;
        }
        o.nonneg = o.nonneg || op.kind == MP_OP_RELU;
        break;
      }
      default:
        fail(MP_ERR_ARG, "unknown graph op kind " + std::to_string(op.kind));
    }
    if (o.H <= 0 || o.W <= 0 || o.C <= 0) fail(MP_ERR_SHAPE, "empty tensor in the graph");
  }
  GDBG("plan: shapes done (%d tensors, %zu ops)", NT, g.ops.size());
  // 1x1 siblings: stride-1 1x1 f16x3 convs reading the same tensor (the dense regressors'
  // conv_L_1_1x1 / conv_L_2_1x1_1 and conv_L_2_1x1_2 / conv_L_3_1x1_2 pairs,
  // train_dense_networks.py:248-373) run as one conv over their concatenated weights while the
  // pointwise kernel takes it (Cin <= 192, Cout <= 256): the input is read once instead of once per
  // conv.  Their outputs become adjacent channel ranges of one buffer (placement constraints like a
  // concat's), so each consumer reads its slice in place.  MP_GRAPH_FUSE_1X1=0 keeps them apart.
  std::vector<int> sib_lead(g.ops.size(), -1);        // op -> the op whose kernel computes it
  std::vector<std::vector<int>> sib_mem(g.ops.size());  // lead -> members (lead first)
  g.n_fused_1x1 = 0;
  if (env_int("MP_GRAPH_FUSE_1X1", 1)) {
    std::vector<char> in_concat(NT, 0);
    for (const auto& op : g.ops)
      if (op.kind == MP_OP_CONCAT)
        for (int s : op.src) in_concat[root(s)] = 1;
    std::map<int, std::vector<int>> by_src;
    for (size_t i = 0; i < g.ops.size(); ++i) {
      const auto& op = g.ops[i];
      if (op.kind != MP_OP_CONV || op.ksize != 1 || op.stride != 1) continue;
      const auto it = c->layers.find(op.name);
      if (it == c->layers.end() || !it->second.x3 || in_concat[op.out] || root(op.out) != op.out) continue;
      const int s = root(op.src[0]);
      if (s == 0 || T[s].C > 192 || T[s].C % 4) continue;
      by_src[s].push_back((int)i);
    }
    for (auto& kv : by_src) {
      const auto& v = kv.second;
      for (size_t a = 0; a < v.size();) {   // runs in op order, at most 256 output channels each
        int tot = g.ops[v[a]].cout;
        size_t b = a + 1;
        while (b < v.size() && tot + g.ops[v[b]].cout <= 256) tot += g.ops[v[b++]].cout;
        if (b - a >= 2) g.n_fused_1x1 += (int)(b - a) - 1;
        if (b - a >= 2)
          for (size_t q = a; q < b; ++q) {
            sib_lead[v[q]] = v[a];
            sib_mem[v[a]].push_back(v[q]);
          }
        a = b;
      }
    }
  }
  // 3: placement of concat groups
  UF uf(NT);
  for (size_t i = 0; i < g.ops.size(); ++i) {
    if (sib_lead[i] != (int)i) continue;
    int off = 0;
    for (int m : sib_mem[i]) {
      if (m != (int)i && !uf.unite(g.ops[m].out, g.ops[i].out, off))
        fail(MP_ERR_UNSUPPORTED, "1x1 sibling placement conflict at " + g.ops[m].name);
      off += g.ops[m].cout;
    }
  }
  for (const auto& op : g.ops) {
    if (op.kind != MP_OP_CONCAT) continue;
    int off = 0;
    const int ro = root(op.out);
    for (int s : op.src) {
      const int rs = root(s);
      if (rs == 0) fail(MP_ERR_UNSUPPORTED, "tf.concat of the graph input");
      if (!uf.unite(rs, ro, off))
        fail(MP_ERR_UNSUPPORTED, "tf.concat placement conflict at tensor " + std::to_string(op.out) +
                                     " (a tensor would need two channel offsets)");
      off += T[s].C;
    }
  }
  std::map<int, int> gid;
  std::vector<int> lo(NT, 1 << 30), hi(NT, -(1 << 30));
  for (int x = 0; x < NT; ++x) {
    if (T[x].alias >= 0 || T[x].C == 0) continue;
    const int r = uf.find(x);
    lo[r] = std::min(lo[r], uf.w[x]);
    hi[r] = std::max(hi[r], uf.w[x] + T[x].C);
  }
  for (int x = 1; x < NT; ++x) {
    if (T[x].alias >= 0 || T[x].C == 0) continue;
    const int r = uf.find(x);
    auto it = gid.find(r);
    if (it == gid.end()) {
      it = gid.emplace(r, (int)g.groups.size()).first;
      auto grp = std::make_unique<G::Group>();
      grp->H = T[x].H;
      grp->W = T[x].W;
      grp->rank2 = T[x].rank2;
      grp->span = hi[r] - lo[r];
      g.groups.push_back(std::move(grp));
    }
    T[x].group = it->second;
    T[x].off = uf.w[x] - lo[r];
    const auto& grp = *g.groups[it->second];
    if (grp.H != T[x].H || grp.W != T[x].W || grp.rank2 != T[x].rank2)
      fail(MP_ERR_SHAPE, "concat group mixes spatial shapes");
  }
  GDBG("plan: %zu groups", g.groups.size());
  for (auto& grp : g.groups) grp->buf.alloc((size_t)n * grp->H * grp->W * grp->span * sizeof(float));
  g.input.alloc((size_t)n * h * w * g.in_channels * sizeof(float));
  auto base = [&](int x) -> float* {
    x = root(x);
    if (x == 0) return g.input.f();
    return g.groups[T[x].group]->buf.f();
  };
  auto ld = [&](int x) {
    x = root(x);
    return x == 0 ? g.in_channels : g.groups[T[x].group]->span;
  };
  auto coff = [&](int x) {
    x = root(x);
    return x == 0 ? 0 : T[x].off;
  };
  // conv_1 + pool fusion candidates: conv index -> pool index
  std::vector<int> fused_pool(g.ops.size(), -1);
  std::vector<char> fused_away(g.ops.size(), 0);
  if (env_int("MP_GRAPH_FUSE", 1))
    for (size_t i = 0; i < g.ops.size(); ++i) {
      const auto& op = g.ops[i];
      if (op.kind != MP_OP_CONV || op.ksize != 3 || op.stride != 1 || op.cout % 4 || op.cout > 64) continue;
      const int s = op.src[0];
      if (root(s) != s || T[s].C != 1 || T[s].H % 2 || T[s].W % 2 || ld(s) != 1 || coff(s) != 0) continue;
      if (uses[op.out] != 1) continue;
      for (size_t j = i + 1; j < g.ops.size(); ++j) {
        const auto& pj = g.ops[j];
        if (pj.kind == MP_OP_MAXPOOL && pj.ksize == 2 && pj.src[0] == op.out && root(pj.out) == pj.out) {
          fused_pool[i] = (int)j;
          fused_away[j] = 1;
          // the pre-pool map is never materialised: drop its (singleton) buffer
          g.groups[T[op.out].group]->buf.release();
        }
      }
    }
  // conv -> 2x2 max pool pairs where the pool is the conv's only consumer: the f16x3 conv kernels
  // can write the pooled map themselves (k_igemm.hip igemm_can_pool; decided per conv below)
  std::vector<int> pool_after(g.ops.size(), -1);
  if (env_int("MP_GRAPH_FUSE_POOL", 1))
    for (size_t i = 0; i < g.ops.size(); ++i) {
      const auto& op = g.ops[i];
      if (op.kind != MP_OP_CONV || fused_pool[i] >= 0 || uses[op.out] != 1 || sib_lead[i] >= 0) continue;
      for (size_t j = i + 1; j < g.ops.size(); ++j) {
        const auto& pj = g.ops[j];
        if (pj.kind == MP_OP_MAXPOOL && pj.ksize == 2 && pj.src[0] == op.out && root(pj.out) == pj.out) {
          pool_after[i] = (int)j;
          break;
        }
      }
    }
  // kernels and their producers
  for (size_t i = 0; i < g.ops.size(); ++i) {
    const auto& op = g.ops[i];
    auto& o = T[op.out];
    if (fused_away[i]) continue;   // produced by its conv's fused kernel (below)
    if (fused_pool[i] >= 0) {
      const auto& pj = g.ops[fused_pool[i]];
      auto k = std::make_unique<G::Kern>();
      k->op = (int)i;
      k->kind = KIND_CONV1_POOL;
      const auto& L = c->layers.at(op.name);
      if (L.cin != 1 || L.cout != op.cout || L.k != 3) fail(MP_ERR_SHAPE, "conv " + op.name + ": weights mismatch");
      k->L = &L;
      k->px = base(op.src[0]);
      k->cH = T[op.src[0]].H;
      k->cW = T[op.src[0]].W;
      k->cw = c->raw.at(op.name + "/" + op.name + "_filters").dev->f();
      k->cb = L.b.f();
      k->pout = base(pj.out);
      k->pldo = ld(pj.out);
      k->pcoff = coff(pj.out);
      k->pC = op.cout;
      std::vector<float> one(64, 1.f), zero(64, 0.f);
      upload(k->ones, one);
      upload(k->zeros, zero);
      T[pj.out].prod = {(int)g.kerns.size()};
      g.kerns.push_back(std::move(k));
      continue;
    }
    if (op.kind == MP_OP_CONCAT) {
      for (int s : op.src) {
        const auto& p = T[root(s)].prod;
        o.prod.insert(o.prod.end(), p.begin(), p.end());
      }
      continue;
    }
    if (op.kind == MP_OP_RELU || op.kind == MP_OP_IDENTITY) continue;
    if (sib_lead[i] >= 0 && sib_lead[i] != (int)i) {   // computed by its lead's kernel
      o.prod = T[g.ops[sib_lead[i]].out].prod;
      continue;
    }
    auto k = std::make_unique<G::Kern>();
    k->op = (int)i;
    k->kind = op.kind;
    const int s = op.src[0];
    const auto& S = T[root(s)];
    if (op.kind == MP_OP_CONV) {
      auto it = c->layers.find(op.name);
      if (it == c->layers.end()) fail(MP_ERR_STATE, "conv layer not finalized: " + op.name);
      const auto& L1 = it->second;
      if (L1.cin != S.C || L1.cout != op.cout || L1.k != op.ksize)
        fail(MP_ERR_SHAPE, "conv " + op.name + ": weights [" + std::to_string(L1.k) + "," + std::to_string(L1.k) + "," +
                               std::to_string(L1.cin) + "," + std::to_string(L1.cout) + "] vs input channels " +
                               std::to_string(S.C));
      const auto& L = sib_lead[i] == (int)i ? fused_1x1_pack(c, g, sib_mem[i]) : L1;
      IgemmArgs& a = k->ia;
      a.x = base(s);
      a.ldx = ld(s);
      a.cix = coff(s);
      a.N = (int)n;
      a.H = S.H;
      a.W = S.W;
      a.Cin = S.C;
      a.wpk = L.w.v4();
      a.K = L.K;
      a.bias = L.b.f();
      a.out = base(op.out);
      a.ldo = ld(op.out);
      a.coff = coff(op.out);
      a.Cout = L.cout;
      a.KS = L.k;
      a.stride = op.stride;
      a.Ho = o.H;
      a.Wo = o.W;
      a.pad_t = same_pad_before(S.H, L.k, op.stride);
      a.pad_l = same_pad_before(S.W, L.k, op.stride);
      a.relu = 1;
      a.nprod = L.nprod;
      if (L.cinp) {   // the Cin-padded packing for the halo kernel (k_igemm.hip halo_geom)
        a.wpad = L.wpad.p;
        a.cinp = L.cinp;
      }
      k->L = &L;
      if (L.x3) {   // split-K workspace of the position-major small-map path (k_igemm.hip)
        const size_t pf = igemm_pm_part_floats(a);
        if (pf) {
          k->part.alloc(pf * sizeof(float));
          a.part = k->part.f();
        }
      }
      const int pj = pool_after[i];
      if (L.x3 && pj >= 0 && igemm_can_pool(a)) {
        // conv + relu + max pool in one kernel: the pre-pool map is never written
        a.pool = 1;
        a.out = base(g.ops[pj].out);
        a.ldo = ld(g.ops[pj].out);
        a.coff = coff(g.ops[pj].out);
        fused_away[pj] = 1;
        T[g.ops[pj].out].prod = {(int)g.kerns.size()};
      }
    } else if (op.kind == MP_OP_MAXPOOL || op.kind == MP_OP_AVGPOOL) {
      if (op.ksize != 2) fail(MP_ERR_UNSUPPORTED, "pool window " + std::to_string(op.ksize) + " (only 2x2/2)");
      k->px = base(s);
      k->pld = ld(s);
      k->pcix = coff(s);
      k->pH = S.H;
      k->pW = S.W;
      k->pC = S.C;
      k->pout = base(op.out) + 0;
      k->pldo = ld(op.out);
      k->pcoff = coff(op.out);
    } else {   // FC
      auto it = c->layers.find(op.name);
      if (it == c->layers.end()) fail(MP_ERR_STATE, "fc layer not finalized: " + op.name);
      const auto& L = it->second;
      const int K = S.H * S.W * S.C;
      if (L.K != K || L.cout != op.cout)
        fail(MP_ERR_SHAPE, "fc " + op.name + ": weights [" + std::to_string(L.K) + "," + std::to_string(L.cout) +
                               "] vs input size " + std::to_string(K));
      if (ld(s) != S.C || coff(s) != 0)
        fail(MP_ERR_UNSUPPORTED, "fc " + op.name + " reads a channel slice of a concat group");
      k->fa = base(s);
      k->fK = K;
      k->fN = L.cout;
      k->fS = fc_choose_splits((int)n, K, L.cout, &k->fks);
      k->fout = base(op.out) + coff(op.out);
      k->fldo = ld(op.out);
      k->relu = fc_relu[i] != 0;
      k->part.alloc((size_t)k->fS * n * ((L.cout + 31) / 32 * 32) * sizeof(float));
      k->L = &L;
    }
    o.prod = {(int)g.kerns.size()};
    g.kerns.push_back(std::move(k));
  }
  for (int x = 0; x < NT; ++x)
    if (T[x].alias >= 0) T[x].prod = T[root(x)].prod;
  GDBG("plan: %zu kernels", g.kerns.size());
  // 4: stream assignment
  const int maxs = std::max(1, std::min(16, env_int("MP_GRAPH_STREAMS", 8)));
  std::vector<int> tail(maxs, -1), last_use(maxs, -1);
  // vector clocks: known[s][s2] = the last kernel of stream s2 that stream s is already ordered
  // after (directly or through other waits); kclock[k] = its stream's clock right after k.  A
  // dependency already covered by the clock adds no event, so the DAG carries no redundant edges.
  std::vector<std::vector<int>> known(maxs, std::vector<int>(maxs, -1)), kclock(g.kerns.size());
  int used = 1;
  for (size_t ki = 0; ki < g.kerns.size(); ++ki) {
    auto& k = *g.kerns[ki];
    const auto& op = g.ops[k.op];
    std::vector<int> deps;
    for (int s : op.src) {
      const auto& p = T[root(s)].prod;
      deps.insert(deps.end(), p.begin(), p.end());
    }
    std::sort(deps.begin(), deps.end());
    deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
    int st = -1;
    for (auto it = deps.rbegin(); it != deps.rend(); ++it)
      if (tail[g.kerns[*it]->stream] == *it) {
        st = g.kerns[*it]->stream;
        break;
      }
    if (st < 0) {
      if (used < maxs) {
        st = used++;
      } else {
        st = 0;
        for (int s = 1; s < maxs; ++s)
          if (last_use[s] < last_use[st]) st = s;
      }
    }
    k.stream = st;
    for (auto it = deps.rbegin(); it != deps.rend(); ++it) {   // latest first: it covers earlier ones
      const int d = *it, ds = g.kerns[d]->stream;
      if (known[st][ds] >= d) continue;
      g.kerns[d]->record = true;
      k.waits.push_back(d);
      for (int s2 = 0; s2 < maxs; ++s2) known[st][s2] = std::max(known[st][s2], kclock[d][s2]);
    }
    known[st][st] = (int)ki;
    kclock[ki] = known[st];
    tail[st] = (int)ki;
    last_use[st] = (int)ki;
  }
  g.n_streams = used;
  // streams / events
  while ((int)g.streams.size() < g.n_streams) {
    hipStream_t s;
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    g.streams.push_back(s);
  }
  while ((int)g.joins.size() < g.n_streams) {
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    g.joins.push_back(e);
  }
  if (!g.fork) hip_check(hipEventCreateWithFlags(&g.fork, hipEventDisableTiming), "hipEventCreate");
  for (auto e : g.kev)
    if (e) (void)hipEventDestroy(e);
  g.kev.assign(g.kerns.size(), nullptr);
  for (size_t ki = 0; ki < g.kerns.size(); ++ki)
    if (g.kerns[ki]->record)
      hip_check(hipEventCreateWithFlags(&g.kev[ki], hipEventDisableTiming), "hipEventCreate");
  g.pn = n;
  g.ph = h;
  g.pw = w;
  g.planned = true;
  GDBG("plan: %d streams, done", g.n_streams);
}

void launch_kern(mp_ctx* c, G& g, G::Kern& k, hipStream_t st) {
  switch (k.kind) {
    case KIND_CONV1_POOL: {
      ProfScope ps(c, st, "graph_conv");
      ProfScope pl(c, st, g.ops[k.op].name.c_str());
      // the hGRU backbone's conv_1 kernel for a dense 64-channel output (hier conv_1), else the
      // any-width form writing into the pool output's view (dense conv_0: 12 channels)
      if (k.pC == 64 && k.pldo == 64 && k.pcoff == 0)
        hip_check(launch_conv1_pool_bn(k.px, k.cw, k.cb, k.ones.f(), k.zeros.f(), k.pout, (int)g.pn, k.cH, k.cW, st,
                                       true),
                  g.ops[k.op].name.c_str());
      else
        hip_check(launch_conv1_pool_any(k.px, k.cw, k.cb, k.pout, k.pldo, k.pcoff, (int)g.pn, k.cH, k.cW, k.pC, st),
                  g.ops[k.op].name.c_str());
      break;
    }
    case MP_OP_CONV: {
      ProfScope ps(c, st, "graph_conv");
      ProfScope pl(c, st, g.ops[k.op].name.c_str());   // per layer, read back by its scope name
      hip_check(k.L->x3 ? launch_igemm_x3(k.ia, k.L->w.p, k.L->wus, st) : launch_igemm_conv(k.ia, st),
                g.ops[k.op].name.c_str());
      break;
    }
    case MP_OP_MAXPOOL:
    case MP_OP_AVGPOOL: {
      ProfScope ps(c, st, "graph_pool");
      hip_check(launch_pool2(k.px, k.pld, k.pcix, (int)g.pn, k.pH, k.pW, k.pC, k.pout, k.pldo, k.pcoff,
                             k.kind == MP_OP_AVGPOOL ? 1 : 0, st),
                "graph pool");
      break;
    }
    default: {
      ProfScope ps(c, st, "graph_fc");
      ProfScope pl(c, st, g.ops[k.op].name.c_str());
      const auto& L = *k.L;
      const int M = (int)g.pn;
      hip_check(L.x3 ? launch_fc_gemm_x3(k.fa, k.fK, L.w.p, L.wus, k.part.f(), M, k.fK, k.fN, k.fS, k.fks, st,
                                         L.nprod)
                     : launch_fc_gemm(k.fa, k.fK, L.w.v4(), k.part.f(), M, k.fK, k.fN, k.fS, k.fks, st),
                g.ops[k.op].name.c_str());
      hip_check(launch_fc_reduce(k.part.f(), k.fS, M, k.fN, L.b.f(), k.relu ? 1 : 0, nullptr, nullptr, k.fout,
                                 k.fldo, st),
                g.ops[k.op].name.c_str());
    }
  }
}

// the whole schedule, eager: over g.streams (stream 0 is where the caller's work joins), or every
// launch in order on `single` (profiling: each launch timed on its own)
void issue(mp_ctx* c, G& g, hipStream_t single_st = nullptr, bool single = false) {
  hipStream_t s0 = single ? single_st : g.streams[0];
  if (!single) {
    hip_check(hipEventRecord(g.fork, s0), "hipEventRecord");
    for (int s = 1; s < g.n_streams; ++s) hip_check(hipStreamWaitEvent(g.streams[s], g.fork, 0), "hipStreamWaitEvent");
  }
  for (size_t ki = 0; ki < g.kerns.size(); ++ki) {
    auto& k = *g.kerns[ki];
    hipStream_t st = single ? s0 : g.streams[k.stream];
    if (!single)
      for (int d : k.waits) hip_check(hipStreamWaitEvent(st, g.kev[d], 0), "hipStreamWaitEvent");
    GDBG("issue %zu/%zu kind %d stream %d waits %zu", ki, g.kerns.size(), k.kind, single ? -1 : k.stream,
         k.waits.size());
    launch_kern(c, g, k, st);
    if (!single && k.record) hip_check(hipEventRecord(g.kev[ki], st), "hipEventRecord");
  }
  if (!single)
    for (int s = 1; s < g.n_streams; ++s) {
      GDBG("join stream %d", s);
      hip_check(hipEventRecord(g.joins[s], g.streams[s]), "hipEventRecord");
      hip_check(hipStreamWaitEvent(s0, g.joins[s], 0), "hipStreamWaitEvent");
    }
  GDBG("issued");
}

}  // namespace

void finalize_graph(mp_ctx* c) {
  if (!c->graph) fail(MP_ERR_STATE, "mp_graph_set must precede mp_finalize_weights");
  auto& g = *c->graph;
  g.planned = false;
  g.kerns.clear();
  g.fused1x1.clear();   // packed from the previous weights
  c->layers.clear();
  // input channels per conv from a channel-only pass (spatial sizes come at plan time)
  std::vector<int> ch(g.n_tensors, 0);
  ch[0] = g.in_channels;
  for (const auto& op : g.ops) {
    int C = 0;
    if (op.kind == MP_OP_CONV || op.kind == MP_OP_FC) C = op.cout;
    else if (op.kind == MP_OP_CONCAT)
      for (int s : op.src) C += ch[s];
    else C = ch[op.src[0]];
    if (op.kind == MP_OP_CONV) {
      const int cin = ch[op.src[0]];
      const auto& w = c->need(op.name + "/" + op.name + "_filters", {op.ksize, op.ksize, cin, op.cout});
      const auto& b = c->need(op.name + "/" + op.name + "_biases", {op.cout});
      if (c->layers.count(op.name)) fail(MP_ERR_ARG, "layer scope used twice: " + op.name);
      auto& L = c->layers[op.name];
      L.k = op.ksize;
      L.cin = cin;
      L.cout = op.cout;
      L.K = op.ksize * op.ksize * cin;
      pack_matrix(c, L, w.dev->f(), L.K >= 4);
      L.b.alloc(op.cout * sizeof(float));
      hip_check(hipMemcpy(L.b.p, b.dev->p, op.cout * sizeof(float), hipMemcpyDeviceToDevice), "bias");
    } else if (op.kind == MP_OP_FC) {
      auto it = c->raw.find(op.name + "/" + op.name + "_weights");
      if (it == c->raw.end()) fail(MP_ERR_STATE, "weight not set: " + op.name + "/" + op.name + "_weights");
      if (it->second.shape.size() != 2 || it->second.shape[1] != op.cout)
        fail(MP_ERR_WEIGHT, op.name + "_weights must be [K, " + std::to_string(op.cout) + "]");
      const int K = (int)it->second.shape[0];
      const auto& b = c->need(op.name + "/" + op.name + "_biases", {op.cout});
      if (c->layers.count(op.name)) fail(MP_ERR_ARG, "layer scope used twice: " + op.name);
      auto& L = c->layers[op.name];
      L.K = L.cin = K;
      L.cout = op.cout;
      pack_matrix(c, L, it->second.dev->f(), K % 32 == 0);
      L.b.alloc(op.cout * sizeof(float));
      hip_check(hipMemcpy(L.b.p, b.dev->p, op.cout * sizeof(float), hipMemcpyDeviceToDevice), "bias");
    }
    ch[op.out] = C;
  }
  c->head_sizes.clear();
  for (int o : g.outputs) c->head_sizes.push_back(ch[o]);
}

bool graph_info(mp_ctx* c, const std::string& k, int64_t* v) {
  if (k.rfind("graph_", 0) != 0) return false;
  if (!c->graph || !c->graph->planned) fail(MP_ERR_STATE, "graph not planned yet (run mp_graph_fwd first)");
  const auto& g = *c->graph;
  size_t launches = 0;
  for (const auto& kk : g.kerns) launches += kk->kind == MP_OP_FC ? 2 : 1;
  if (k == "graph_kernels")
    *v = (int64_t)launches;
  else if (k == "graph_streams")
    *v = g.n_streams;
  else if (k == "graph_buffers")
    *v = (int64_t)g.groups.size();
  else if (k == "graph_fused_1x1") {   // 1x1 convs computed by a sibling's kernel
    *v = g.n_fused_1x1;
  } else if (k == "graph_fused_pools") {   // max pools computed inside their conv's kernel
    int64_t f = 0;
    for (const auto& kk : g.kerns) f += (kk->kind == MP_OP_CONV && kk->ia.pool) || kk->kind == KIND_CONV1_POOL;
    *v = f;
  }
  else
    fail(MP_ERR_ARG, "unknown info key: " + k);
  return true;
}

}  // namespace mpr

extern "C" {

int mp_graph_set(mp_ctx* ctx, const mp_graph_op* ops, int n_ops, int in_channels, const int32_t* outputs,
                 int n_outputs) {
  return guard([&] {
    if (!ctx || !ops || n_ops <= 0 || !outputs || n_outputs <= 0 || in_channels <= 0)
      fail(MP_ERR_ARG, "mp_graph_set: bad argument");
    if (ctx->model != MP_MODEL_GRAPH) fail(MP_ERR_STATE, "context is not an MP_MODEL_GRAPH context");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    auto g = std::make_shared<GraphState>();
    g->in_channels = in_channels;
    int next = 1;   // SSA: ids strictly increase, every source defined earlier
    std::vector<char> defined(1, 1);
    for (int i = 0; i < n_ops; ++i) {
      const auto& o = ops[i];
      if (o.out < next) fail(MP_ERR_ARG, "op " + std::to_string(i) + ": tensor ids must increase");
      if (o.n_src < 1 || o.n_src > MP_GRAPH_MAX_SRC) fail(MP_ERR_ARG, "op " + std::to_string(i) + ": bad n_src");
      if (o.kind != MP_OP_CONCAT && o.n_src != 1) fail(MP_ERR_ARG, "op " + std::to_string(i) + ": one source expected");
      GraphState::Op op{o.kind, o.out, o.ksize, o.stride, o.cout, {}, o.name ? o.name : ""};
      for (int j = 0; j < o.n_src; ++j) {
        const int s = o.src[j];
        if (s < 0 || s >= (int)defined.size() || !defined[s])
          fail(MP_ERR_ARG, "op " + std::to_string(i) + ": source " + std::to_string(s) + " undefined");
        op.src.push_back(s);
      }
      if (o.kind == MP_OP_CONV || o.kind == MP_OP_FC) {
        if (op.name.empty() || o.cout <= 0) fail(MP_ERR_ARG, "op " + std::to_string(i) + ": conv / fc needs name, cout");
        op.name = strip_scope(op.name.c_str());
      }
      if (o.kind == MP_OP_CONV && (o.ksize <= 0 || o.stride <= 0)) fail(MP_ERR_ARG, "conv needs ksize, stride");
      if ((o.kind == MP_OP_MAXPOOL || o.kind == MP_OP_AVGPOOL) && o.ksize <= 0) fail(MP_ERR_ARG, "pool needs ksize");
      if (o.kind < MP_OP_CONV || o.kind > MP_OP_IDENTITY) fail(MP_ERR_ARG, "unknown op kind");
      defined.resize(o.out + 1, 0);
      defined[o.out] = 1;
      next = o.out + 1;
      g->ops.push_back(std::move(op));
    }
    g->n_tensors = next;
    for (int i = 0; i < n_outputs; ++i) {
      const int o = outputs[i];
      if (o <= 0 || o >= next || !defined[o]) fail(MP_ERR_ARG, "output tensor " + std::to_string(o) + " undefined");
      g->outputs.push_back(o);
    }
    ctx->graph = std::move(g);
    ctx->finalized = false;
  });
}

int mp_graph_fwd(mp_ctx* ctx, const float* x, int64_t n, int64_t h, int64_t w, float* const* outs, void* stream) {
  return guard([&] {
    if (!ctx || !x || !outs) fail(MP_ERR_ARG, "mp_graph_fwd: null pointer");
    if (ctx->model != MP_MODEL_GRAPH || !ctx->graph) fail(MP_ERR_STATE, "context has no graph");
    if (!ctx->finalized) fail(MP_ERR_STATE, "weights not finalized");
    if (n <= 0 || n > (1 << 20) || h <= 0 || w <= 0 || h > 8192 || w > 8192) fail(MP_ERR_SHAPE, "bad input shape");
    auto& g = *ctx->graph;
    for (size_t i = 0; i < g.outputs.size(); ++i)
      if (!outs[i]) fail(MP_ERR_ARG, "output buffer " + std::to_string(i) + " is NULL");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (!g.planned || g.pn != n || g.ph != h || g.pw != w) {
      hip_check(hipDeviceSynchronize(), "sync before re-plan");   // buffers of the old plan may be in use
      plan(ctx, g, n, h, w);
    }
    hip_check(hipMemcpyAsync(g.input.p, x, (size_t)n * h * w * g.in_channels * sizeof(float),
                             hipMemcpyDeviceToDevice, st),
              "graph input copy");
    if (ctx->prof) {
      issue(ctx, g, st, true);
    } else {
      // eager: the graph's stream 0 joins the caller's stream on both ends
      hipEvent_t a = ctx->ev();
      hip_check(hipEventRecord(a, st), "hipEventRecord");
      hip_check(hipStreamWaitEvent(g.streams[0], a, 0), "hipStreamWaitEvent");
      issue(ctx, g);
      hipEvent_t b = ctx->ev();
      hip_check(hipEventRecord(b, g.streams[0]), "hipEventRecord");
      hip_check(hipStreamWaitEvent(st, b, 0), "hipStreamWaitEvent");
      ctx->pool.push_back(a);
      ctx->pool.push_back(b);
    }
    GDBG("launched");
    for (size_t i = 0; i < g.outputs.size(); ++i) {
      int o = g.outputs[i];
      while (g.t[o].alias >= 0) o = g.t[o].alias;
      const auto& T = g.t[o];
      const size_t rows = (size_t)n * T.H * T.W;
      if (o == 0) {
        hip_check(hipMemcpyAsync(outs[i], x, rows * T.C * sizeof(float), hipMemcpyDeviceToDevice, st), "graph out");
        continue;
      }
      const auto& grp = *g.groups[T.group];
      hip_check(hipMemcpy2DAsync(outs[i], T.C * sizeof(float), grp.buf.f() + T.off, grp.span * sizeof(float),
                                 T.C * sizeof(float), rows, hipMemcpyDeviceToDevice, st),
                "graph output copy");
    }
  });
}

}  // extern "C"
