"""cnn_model_struct (train_cnn_networks_hgru.py:626-760): the regressor the reference's hGRU driver
builds for its validation (169), test (291) and real-data evaluation (363) graphs.  Structure
against the reference's own build (AST extraction, or the committed digest where the reference is
absent), the float64 oracle against the golden vectors on the CPU, and the GPU graph runtime
against both (fp32 gate 1e-4, bf16 gate 5e-3), batch invariance and B = 256."""
import json
import os

import numpy as np
import pytest

from helpers import BF16_REL_TOL, FP32_REL_TOL, MG, ROOT, golden_array, golden_meta, pkg, rel_inf
from oracle import regressors_ref as RR

REF_CNN = "/root/reference/train_cnn_networks_hgru.py"


def _inputs():
    m = golden_meta()["cnn_c128"]
    return MG.regressor_inputs("cnn", m["n"], m["crop"], m["weight_seed"], m["crop_seed"])


def _record():
    return pkg().train_cnn_networks_hgru.cnn_model_struct().record(128, 128, 69)


def test_cnn_oracle_matches_golden():
    wts, depth = _inputs()
    out, t = RR.cnn_forward(depth, wts, keep=True)
    assert rel_inf(out, golden_array("cnn_c128", "out")) < 1e-9
    assert t["pool5"].shape == (2, 4, 4, 1024)          # fc_1's fan-in 16,384 (658)
    f32 = RR.cnn_forward(depth, wts, dtype=np.float32)
    assert rel_inf(f32, out) < 1e-5


def test_cnn_recorded_graph_digest():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "cnn_graph_digest.json")))
    rec = _record().records()
    assert len(rec) == d["ops"] == 18
    assert pkg()._graph.canonical_digest(rec) == d["sha256"]


@pytest.mark.skipif(not os.path.exists(REF_CNN), reason="reference sources not present")
def test_cnn_recorded_graph_is_the_reference_graph():
    """cnn_model_struct.record() op for op against the reference's own build (AST extraction)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import extract_dense_hier as X
    ops, _ = X.extract((69,), path=X.REF_CNN, cls="cnn_model_struct")
    rec = _record().records()
    assert len(rec) == len(ops) == 18
    for a, b in zip(rec, ops):
        assert a == {k: v for k, v in b.items() if k != "line"}


def test_cnn_recorded_graph_uses_the_cnn_variables():
    m = pkg().train_cnn_networks_hgru.cnn_model_struct()
    g = m.record(128, 128, 69)
    W = pkg().weights
    assert {v.name: v.shape for v in m._table(g)} == {v.name: v.shape for v in W.cnn_vars()}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32_split", "fp32", "bf16"])
def test_cnn_gpu_matches_golden_and_oracle(dtype):
    torch = pytest.importorskip("torch")
    wts, depth = _inputs()
    model = pkg().train_cnn_networks_hgru.cnn_model_struct()
    model.compute_dtype = dtype
    model.load_weights(wts)
    x = torch.from_numpy(depth).cuda()
    out = model.build(x, 69, train_mode=False).cpu().numpy()
    assert out.shape == (2, 69) and model.out_put.shape == (2, 69)
    err = rel_inf(out, golden_array("cnn_c128", "out"))
    print(f"cnn {dtype}: rel_inf vs fp64 golden {err:.3e}")
    assert err <= (BF16_REL_TOL if dtype == "bf16" else FP32_REL_TOL)
    assert np.array_equal(model.forward(x).cpu().numpy(), out)                   # deterministic
    one = model.forward(x[1:2].contiguous()).cpu().numpy()
    assert np.array_equal(one[0], out[1])                                      # batch invariant


@pytest.mark.gpu
def test_cnn_gpu_batch256():
    """The bench batch: crops from the start, middle and end of a batch of 256 against the fp64
    oracle, each bit-identical to its own batch-1 run."""
    torch = pytest.importorskip("torch")
    W = pkg().weights
    wts = W.synth_weights(W.cnn_vars(), seed=81)
    depth = W.synth_crops(256, seed=47, size=128)
    model = pkg().train_cnn_networks_hgru.cnn_model_struct()
    model.load_weights(wts)
    x = torch.from_numpy(depth).cuda()
    out = model.build(x, 69).cpu().numpy()
    assert np.isfinite(out).all()
    idx = [0, 127, 255]
    ref = RR.cnn_forward(depth[idx], wts)
    assert rel_inf(out[idx], ref) <= FP32_REL_TOL
    for i in idx:
        one = model.forward(x[i:i + 1].contiguous()).cpu().numpy()
        assert np.array_equal(one[0], out[i]), i


@pytest.mark.gpu
def test_cnn_rejects_training():
    torch = pytest.importorskip("torch")
    x = torch.zeros((1, 128, 128, 1), device="cuda")
    with pytest.raises(NotImplementedError):
        pkg().train_cnn_networks_hgru.cnn_model_struct().build(x, 69, train_mode=True)
