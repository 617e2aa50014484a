"""dense_hier_model_struct (train_dense_hier_networks.py:327-2507) and the layer-graph runtime
(mp_graph_*): the recorded graph against the reference's own build() (AST extraction, here only)
and the committed structural digest; the oracle against the golden vectors; the GPU graph runtime
against oracle + golden (fp32 gate 1e-4), eager == hipGraph replay bit for bit, batch invariance."""
import os

import numpy as np
import pytest

from helpers import FP32_REL_TOL, MG, ROOT, golden_array, golden_meta, pkg, rel_inf
from oracle import regressors_ref as RR

REF = "/root/reference/train_dense_hier_networks.py"
HEADS = MG.HIER_HEADS


def _digest():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "dense_hier_graph_digest.json")) as f:
        return json.load(f)


def _recorded(crop=128):
    m = pkg().train_dense_hier_networks.dense_hier_model_struct()
    return m, m.record(crop, crop, *HEADS)


def _extract():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import extract_dense_hier as X
    return X.extract(HEADS)


@pytest.mark.skipif(not os.path.exists(REF), reason="reference sources not present (GPU box)")
def test_recorded_graph_is_the_reference_graph():
    ops, shapes = _extract()
    _, g = _recorded()
    rec = g.records()
    assert len(rec) == len(ops) == 666
    for i, (a, b) in enumerate(zip(rec, ops)):
        b = {k: v for k, v in b.items() if k != "line"}
        assert a == b, (i, a, b)
    # every tensor's static shape agrees (TF's get_shape)
    by_label = {}
    for o in g.ops:
        by_label[o["out"].label] = o["out"].shape
    for name, shp in shapes.items():
        if name in by_label:   # rank-2 [n, C] here, (1, 1, C) in the extraction
            got = list(by_label[name])
            assert (got if len(got) == 3 else [1, 1] + got) == list(shp), name


@pytest.mark.skipif(not os.path.exists(REF), reason="reference sources not present (GPU box)")
def test_oracle_layer_sequence_is_the_reference():
    ops, _ = _extract()
    want = [("conv", o["name"], o["k"], o["stride"], o["cin"], o["cout"]) if o["op"] == "conv"
            else ("fc", o["name"], o["cin"], o["cout"]) for o in ops if o["op"] in ("conv", "fc")]
    m = golden_meta()["dense_hier_c128"]
    wts, depth = MG.regressor_inputs("dense_hier", 1, 128, m["weight_seed"], m["crop_seed"])
    trace = []
    RR.dense_hier_forward(depth, wts, trace=trace)
    assert trace == want


def test_recorded_graph_digest():
    d = _digest()
    _, g = _recorded(d["crop"])
    rec = g.records()
    import collections
    assert dict(collections.Counter(r["op"] for r in rec)) == d["counts"]
    assert pkg()._graph.canonical_digest(rec) == d["sha256"]
    assert d["counts"]["conv"] == 365 and d["counts"]["fc"] == 52 and d["counts"]["concat"] == 169


def test_dense_hier_oracle_matches_golden():
    m = golden_meta()["dense_hier_c128"]
    wts, depth = MG.regressor_inputs("dense_hier", m["n"], m["crop"], m["weight_seed"], m["crop_seed"])
    out, parts = RR.dense_hier_forward(depth, wts)
    assert rel_inf(out, golden_array("dense_hier_c128", "out")) < 1e-9
    for f in RR.FINGERS:
        assert rel_inf(parts[f], golden_array("dense_hier_c128", f"{f}_out")) < 1e-9


def test_recorder_checks_shapes_like_tf():
    G = pkg()._graph
    g = G.GraphRecorder(16, 16, 1)
    a = g.conv(g.input, 1, 8, "a")
    with pytest.raises(ValueError):
        g.conv(a, 4, 8, "b")                       # in_channels mismatch
    b = g.conv(a, 8, 8, "b", stride=2)
    with pytest.raises(ValueError):
        g.concat([a, b])                           # spatial mismatch
    p = g.pool(a)
    with pytest.raises(ValueError):
        g.fc(p, 100, 4, "f")                       # in_size != 8*8*8
    f = g.fc(p, 512, 4, "f")
    assert f.shape == (4,) and b.shape == (8, 8, 8)


def test_reject_training():
    m = pkg().train_dense_hier_networks.dense_hier_model_struct()
    m.record(64, 64, *HEADS)
    with pytest.raises(NotImplementedError):
        m.conv_layer(m.conv1, 12, 16, "x", batchnorm=["x"])


# ---------------------------------------------------------------------------------------- GPU
def _gpu_model(dtype, wts):
    model = pkg().train_dense_hier_networks.dense_hier_model_struct()
    model.compute_dtype = dtype
    model.load_weights(wts)
    return model


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "fp32_split"])
def test_dense_hier_gpu_matches_golden_and_oracle(dtype):
    torch = pytest.importorskip("torch")
    m = golden_meta()["dense_hier_c128"]
    wts, depth = MG.regressor_inputs("dense_hier", m["n"], m["crop"], m["weight_seed"], m["crop_seed"])
    model = _gpu_model(dtype, wts)
    x = torch.from_numpy(depth).cuda()
    out = model.build(x, *HEADS, train_mode=False).cpu().numpy()
    assert rel_inf(out, golden_array("dense_hier_c128", "out")) <= FP32_REL_TOL
    for f in RR.FINGERS:
        got = getattr(model, f"{f}_output").cpu().numpy()
        assert rel_inf(got, golden_array("dense_hier_c128", f"{f}_out")) <= FP32_REL_TOL
    ctx = model._ctx
    assert ctx.info("graph_streams") > 1
    # 365 convs + 28 pools + 52 FC (gemm + reduce); pools fused into their conv's kernel and 1x1
    # convs computed by a sibling's kernel launch nothing
    assert (ctx.info("graph_kernels") + ctx.info("graph_fused_pools") + ctx.info("graph_fused_1x1")
            == 365 + 28 + 2 * 52)
    # 169 concats placed in place: fewer buffers than tensors
    assert ctx.info("graph_buffers") < 365 + 28 + 52
    again = model.forward(x).cpu().numpy()
    assert np.array_equal(out, again)
    one = model.forward(x[1:2]).cpu().numpy()      # re-plan for n = 1; batch invariance
    assert np.array_equal(one[0], out[1])


@pytest.mark.gpu
def test_graph_eager_equals_one_stream(monkeypatch):
    """eager multi-stream (default) == one stream, bit for bit"""
    torch = pytest.importorskip("torch")
    m = golden_meta()["dense_hier_c128"]
    wts, depth = MG.regressor_inputs("dense_hier", 3, 128, m["weight_seed"], m["crop_seed"])
    model = _gpu_model("fp32_split", wts)
    x = torch.from_numpy(depth).cuda()
    ref = model.build(x, *HEADS).cpu().numpy()
    assert model._ctx.info("graph_streams") > 1
    monkeypatch.setenv("MP_GRAPH_STREAMS", "1")
    model2 = _gpu_model("fp32_split", wts)
    one = model2.build(x, *HEADS).cpu().numpy()
    assert model2._ctx.info("graph_streams") == 1
    assert np.array_equal(ref, one)


@pytest.mark.gpu
def test_graph_runtime_small_graph():
    """A hand-built graph: conv -> relu (folded) -> concat with a pooled branch -> fc + relu ->
    fc, against numpy; exercises relu folding, concat placement and a rank-2 concat."""
    torch = pytest.importorskip("torch")
    mp = pkg()
    G, L = mp._graph, mp._lib
    from oracle.hgru_ref import conv2d_same, max_pool_same
    rng = np.random.default_rng(0)
    g = G.GraphRecorder(12, 12, 1)
    a = g.conv(g.input, 1, 8, "a")
    ar = g.relu(a)
    b = g.conv(ar, 8, 8, "b", k=1)
    c = g.concat([ar, b])
    p = g.pool(c, 2, avg=True)
    f1 = g.relu(g.fc(p, 6 * 6 * 16, 32, "f1"))
    f2 = g.fc(p, 6 * 6 * 16, 8, "f2")
    cat = g.concat([f1, f2])
    out = g.fc(cat, 40, 5, "f3")
    wts = {"a/a_filters": rng.standard_normal((3, 3, 1, 8)), "a/a_biases": rng.standard_normal(8) * .1,
           "b/b_filters": rng.standard_normal((1, 1, 8, 8)), "b/b_biases": rng.standard_normal(8) * .1,
           "f1/f1_weights": rng.standard_normal((576, 32)) * .05, "f1/f1_biases": rng.standard_normal(32) * .1,
           "f2/f2_weights": rng.standard_normal((576, 8)) * .05, "f2/f2_biases": rng.standard_normal(8) * .1,
           "f3/f3_weights": rng.standard_normal((40, 5)) * .1, "f3/f3_biases": rng.standard_normal(5) * .1}
    x = rng.standard_normal((3, 12, 12, 1))
    r = lambda v: np.maximum(v, 0)
    ra = r(conv2d_same(x, wts["a/a_filters"]) + wts["a/a_biases"])
    rb = r(conv2d_same(ra, wts["b/b_filters"]) + wts["b/b_biases"])
    from oracle.hgru_ref import avg_pool_same
    rp = avg_pool_same(np.concatenate([ra, rb], -1)).reshape(3, -1)
    rf = np.concatenate([r(rp @ wts["f1/f1_weights"] + wts["f1/f1_biases"]), rp @ wts["f2/f2_weights"] + wts["f2/f2_biases"]], -1)
    want = rf @ wts["f3/f3_weights"] + wts["f3/f3_biases"]
    for dt in (L.MP_DTYPE_F32, L.MP_DTYPE_F32_SPLIT):
        ctx = L.Context(L.MP_MODEL_GRAPH, 0)
        G.install(ctx, g, [out, c])
        for k, v in wts.items():
            ctx.set_weight(k, v.astype(np.float32))
        ctx.finalize(dt)
        xt = torch.from_numpy(x.astype(np.float32)).cuda()
        o = torch.empty((3, 5), device="cuda")
        oc = torch.empty((3, 12, 12, 16), device="cuda")
        ctx.graph_fwd(xt, [o, oc], L.current_stream())
        torch.cuda.synchronize()
        assert rel_inf(o.cpu().numpy(), want) < 1e-5
        assert rel_inf(oc.cpu().numpy(), np.concatenate([ra, rb], -1)) < 1e-5
        assert ctx.info("graph_buffers") == 4    # groups: {a, b, c}, p, {f1, f2, cat}, out


@pytest.mark.gpu
def test_graph_runtime_rejects_unsupported_graphs():
    """Planning errors surface as MonkeyPoseError before any launch: a tensor needed at two different
    channel offsets (concat placement conflict), a relu on an fc output that has another consumer,
    and an unknown layer scope at finalize."""
    torch = pytest.importorskip("torch")
    mp = pkg()
    G, L = mp._graph, mp._lib
    rng = np.random.default_rng(1)

    def ctx_for(g, outs, wts):
        ctx = L.Context(L.MP_MODEL_GRAPH, 0)
        G.install(ctx, g, outs)
        for k, v in wts.items():
            ctx.set_weight(k, v.astype(np.float32))
        ctx.finalize(L.MP_DTYPE_F32_SPLIT)
        return ctx

    conv_w = {"a/a_filters": rng.standard_normal((3, 3, 1, 8)), "a/a_biases": np.zeros(8),
              "b/b_filters": rng.standard_normal((3, 3, 1, 8)), "b/b_biases": np.zeros(8)}
    x = torch.zeros((1, 8, 8, 1), device="cuda")
    # a sits at offset 0 of cat(a, b) and at offset 8 of cat(b, a)
    g = G.GraphRecorder(8, 8, 1)
    a = g.conv(g.input, 1, 8, "a")
    b = g.conv(g.input, 1, 8, "b")
    c1, c2 = g.concat([a, b]), g.concat([b, a])
    ctx = ctx_for(g, [c1, c2], conv_w)
    with pytest.raises(L.MonkeyPoseError, match="placement conflict"):
        ctx.graph_fwd(x, [torch.empty((1, 8, 8, 16), device="cuda")] * 2, L.current_stream())
    # relu of an fc output that is also a graph output
    g = G.GraphRecorder(8, 8, 1)
    f = g.fc(g.conv(g.input, 1, 8, "a"), 512, 4, "f")
    r = g.relu(f)
    wts = dict(conv_w, **{"f/f_weights": rng.standard_normal((512, 4)), "f/f_biases": np.zeros(4)})
    ctx = ctx_for(g, [r, f], wts)
    with pytest.raises(L.MonkeyPoseError, match="relu"):
        ctx.graph_fwd(x, [torch.empty((1, 4), device="cuda")] * 2, L.current_stream())
    # a layer whose weights were never set
    g = G.GraphRecorder(8, 8, 1)
    z = g.conv(g.input, 1, 8, "zz")
    with pytest.raises(L.MonkeyPoseError, match="weight not set"):
        ctx_for(g, [z], {})
