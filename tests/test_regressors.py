"""Dense (train_dense_networks.py:223-408) and hierarchical (train_hier_networks.py:338-530)
regressors: CPU oracle pinned to the golden vectors, GPU path (C ABI) against oracle + golden."""
import numpy as np
import pytest

from helpers import BF16_REL_TOL, FP32_REL_TOL, MG, golden_array, golden_meta, pkg, rel_inf
from oracle import regressors_ref as RR


def _inputs(case):
    m = golden_meta()[case]
    return m, MG.regressor_inputs(m["kind"], m["n"], m["crop"], m["weight_seed"], m["crop_seed"])


def test_dense_oracle_matches_golden():
    m, (wts, depth) = _inputs("dense_c128")
    out, t = RR.dense_forward(depth, wts, keep=True)
    assert rel_inf(out, golden_array("dense_c128", "out")) < 1e-9
    # the concat widths the reference builds: pool1/2/3 flatten to 98304/65536/18432
    assert t["pool1"][0].size == 98304 and t["pool2"][0].size == 65536 and t["pool3"][0].size == 18432


def test_hier_oracle_matches_golden():
    m, (wts, depth) = _inputs("hier_c128")
    out, parts = RR.hier_forward(depth, wts)
    assert rel_inf(out, golden_array("hier_c128", "out")) < 1e-9
    for f in RR.FINGERS:
        assert rel_inf(parts[f], golden_array("hier_c128", f"{f}_out")) < 1e-9


def test_dense_conv_table_is_consistent():
    W = pkg().weights
    specs = W.dense_conv_specs()
    assert len(specs) == 49
    assert sum(1 for s in specs if s[1] == 3) == 29 and sum(1 for s in specs if s[1] == 1) == 20


REG_DTYPES = ["fp32", "fp32_split"]


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["graph", "mp_dense_fwd"])
@pytest.mark.parametrize("dtype", REG_DTYPES)
def test_dense_gpu_matches_golden_and_oracle(dtype, engine):
    torch = pytest.importorskip("torch")
    m, (wts, depth) = _inputs("dense_c128")
    model = pkg().train_dense_networks.dense_model_struct(use_graph=engine == "graph")
    model.compute_dtype = dtype
    model.load_weights(wts)
    out = model.build(torch.from_numpy(depth).cuda(), 69, train_mode=False).cpu().numpy()
    assert rel_inf(out, golden_array("dense_c128", "out")) <= FP32_REL_TOL
    again = model.forward(torch.from_numpy(depth).cuda()).cpu().numpy()
    assert np.array_equal(out, again)
    one = model.forward(torch.from_numpy(depth[1:2]).cuda()).cpu().numpy()
    assert np.array_equal(one[0], out[1])
    if engine == "graph" and dtype == "fp32_split":
        # the 1x1 sibling pairs over one input (conv_L_1_1x1 + conv_L_2_1x1_1 at L = 3..6, and
        # conv_L_2_1x1_2 + conv_L_3_1x1_2 where the 32x32 input is <= 192 channels: L = 3, 4) run
        # as one conv each (mp_graph.hip plan: 1x1 siblings)
        assert model._ctx.info("graph_fused_1x1") == 6


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["graph", "mp_hier_fwd"])
@pytest.mark.parametrize("dtype", REG_DTYPES)
def test_hier_gpu_matches_golden_and_oracle(dtype, engine):
    torch = pytest.importorskip("torch")
    m, (wts, depth) = _inputs("hier_c128")
    model = pkg().train_hier_networks.hier_model_struct(use_graph=engine == "graph")
    model.compute_dtype = dtype
    model.load_weights(wts)
    out = model.build(torch.from_numpy(depth).cuda(), *MG.HIER_HEADS, train_mode=False).cpu().numpy()
    assert rel_inf(out, golden_array("hier_c128", "out")) <= FP32_REL_TOL
    for f in RR.FINGERS:
        got = getattr(model, f"{f}_output").cpu().numpy()
        assert rel_inf(got, golden_array("hier_c128", f"{f}_out")) <= FP32_REL_TOL


@pytest.mark.gpu
def test_regressors_reject_training():
    torch = pytest.importorskip("torch")
    x = torch.zeros((1, 128, 128, 1), device="cuda")
    with pytest.raises(NotImplementedError):
        pkg().train_dense_networks.dense_model_struct().build(x, 69, train_mode=True)
    with pytest.raises(NotImplementedError):
        pkg().train_hier_networks.hier_model_struct().build(x, 108, 39, 39, 39, 39, 36, batch_norm=["conv_1"])


REF_HIER = "/root/reference/train_hier_networks.py"


@pytest.mark.skipif(not __import__("os").path.exists(REF_HIER), reason="reference sources not present")
def test_hier_recorded_graph_is_the_reference_graph():
    """hier_model_struct.record() op for op against the reference's own build (AST extraction)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import extract_dense_hier as X
    ops, _ = X.extract(MG.HIER_HEADS, path=X.REF_HIER)
    rec = pkg().train_hier_networks.hier_model_struct().record(128, 128, *MG.HIER_HEADS).records()
    assert len(rec) == len(ops) == 91
    for a, b in zip(rec, ops):
        assert a == {k: v for k, v in b.items() if k != "line"}


def test_hier_recorded_graph_uses_the_hier_variables():
    m = pkg().train_hier_networks.hier_model_struct()
    g = m.record(128, 128, *MG.HIER_HEADS)
    W = pkg().weights
    assert {v.name: v.shape for v in m._table(g)} == {v.name: v.shape for v in W.hier_vars()}


REF_DENSE = "/root/reference/train_dense_networks.py"


@pytest.mark.skipif(not __import__("os").path.exists(REF_DENSE), reason="reference sources not present")
def test_dense_recorded_graph_is_the_reference_graph():
    """dense_model_struct.record() op for op against the reference's own build (AST extraction)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import extract_dense_hier as X
    ops, _ = X.extract((69,), path=X.REF_DENSE)
    rec = pkg().train_dense_networks.dense_model_struct().record(128, 128, 69).records()
    assert len(rec) == len(ops) == 88
    for a, b in zip(rec, ops):
        assert a == {k: v for k, v in b.items() if k != "line"}


def test_dense_recorded_graph_uses_the_dense_variables():
    m = pkg().train_dense_networks.dense_model_struct()
    g = m.record(128, 128, 69)
    W = pkg().weights
    assert {v.name: v.shape for v in m._table(g)} == {v.name: v.shape for v in W.dense_vars()}


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["graph", "abi"])
@pytest.mark.parametrize("kind", ["dense", "hier"])
def test_regressors_bf16_within_bf16_gate(kind, engine):
    """compute_dtype='bf16': the split kernels' hi x hi product only (one f16 MFMA per MAC), fp32
    accumulation; stated gate 5e-3 like the hGRU bf16 path, batch invariance kept."""
    torch = pytest.importorskip("torch")
    case = f"{kind}_c128"
    m, (wts, depth) = _inputs(case)
    P = pkg()
    model = (P.train_dense_networks.dense_model_struct(use_graph=engine == "graph") if kind == "dense"
             else P.train_hier_networks.hier_model_struct(use_graph=engine == "graph"))
    model.compute_dtype = "bf16"
    model.load_weights(wts)
    args = (69,) if kind == "dense" else MG.HIER_HEADS
    out = model.build(torch.from_numpy(depth).cuda(), *args, train_mode=False).cpu().numpy()
    err = rel_inf(out, golden_array(case, "out"))
    print(f"bf16 {kind} {engine}: rel_inf {err:.3e}")
    assert err <= BF16_REL_TOL
    one = model.forward(torch.from_numpy(depth[1:2]).cuda()).cpu().numpy()
    assert np.array_equal(one[0], out[1])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32_split", "bf16"])
def test_hier_fused_conv_pool_bit_identical(dtype, monkeypatch):
    """The graph runtime fuses every hier conv -> 2x2 max pool pair into the conv kernel (halo
    epilogue for conv_2 / con_3 / con_4 / con_5 at W = 64 / 32 / 16 / 8, the split-K reduce for
    con_6): all six outputs are bit-identical to the unfused conv + pool2_kernel schedule
    (MP_GRAPH_FUSE_POOL=0), at an odd batch (a partial last tile of two-image con_5 tiles)."""
    torch = pytest.importorskip("torch")
    W = pkg().weights
    outs = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("MP_GRAPH_FUSE_POOL", fuse)
        model = pkg().train_hier_networks.hier_model_struct()
        model.compute_dtype = dtype
        g = model.record(128, 128, *MG.HIER_HEADS)
        model.load_weights(W.synth_weights(model._table(g), seed=21))
        depth = torch.from_numpy(W.synth_crops(5, seed=22, size=128)).cuda()
        main = model.build(depth, *MG.HIER_HEADS, train_mode=False)
        outs[fuse] = [main.cpu().numpy()] + [getattr(model, f"{f}_output").cpu().numpy() for f in "prmit"]
    for a, b in zip(outs["1"], outs["0"]):
        assert np.array_equal(a, b)
