"""The regressors at the batch they are benched at (B = 256; SURVEY config 3 is hier at B = 256).

The graph runtime's B = 256 schedule differs from the small-batch one: 8 streams, the 8-way
split-K of ``con_6``, position-major tiles whose M order is ``position * N + image`` (so a tile
mixes images), XCD-aware tile orders.  Here: 3 crops sampled across the batch against the fp64
oracle (the fp32 gate 1e-4), each of them run alone bit-identical to its row (batch invariance of
the schedule), and a second run bit-identical (determinism).  dense-hier (5 GFLOP / crop in the
oracle) gets the properties only, plus a one-crop oracle check.
References: train_hier_networks.py:338-530, train_dense_networks.py:223-408,
train_dense_hier_networks.py:327-2507."""
import numpy as np
import pytest

from helpers import FP32_REL_TOL, MG, pkg, rel_inf
from oracle import regressors_ref as RR

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

B = 256
SAMPLE = (3, 130, 255)


def _run(kind, dtype="fp32_split"):
    P = pkg()
    wts, depth = MG.regressor_inputs(kind, B, 128, 91, 92)
    if kind == "dense":
        model = P.train_dense_networks.dense_model_struct()
        args = (69,)
    elif kind == "hier":
        model = P.train_hier_networks.hier_model_struct()
        args = MG.HIER_HEADS
    else:
        model = P.train_dense_hier_networks.dense_hier_model_struct()
        args = MG.HIER_HEADS
    model.compute_dtype = dtype
    model.load_weights(wts)
    x = torch.from_numpy(depth).cuda()
    out = model.build(x, *args, train_mode=False)
    outs = [out.cpu().numpy()]
    if kind != "dense":
        outs += [getattr(model, f"{f}_output").cpu().numpy() for f in RR.FINGERS]
    return model, wts, depth, x, outs


def _heads(model, kind):
    o = [model.output.cpu().numpy()]
    if kind != "dense":
        o += [getattr(model, f"{f}_output").cpu().numpy() for f in RR.FINGERS]
    return o


@pytest.mark.parametrize("kind", ["hier", "dense"])
def test_regressor_b256_against_oracle_and_batch_invariant(kind):
    model, wts, depth, x, outs = _run(kind)
    assert model._ctx.info("graph_streams") > 1
    sample = list(SAMPLE)
    if kind == "hier":
        out, parts = RR.hier_forward(depth[sample].astype(np.float64), wts)
        refs = [out] + [parts[f] for f in RR.FINGERS]
    else:
        refs = [RR.dense_forward(depth[sample].astype(np.float64), wts)]
    for got, ref in zip(outs, refs):
        assert rel_inf(got[sample], ref) <= FP32_REL_TOL
    # determinism of the B = 256 schedule
    model.forward(x)
    again = _heads(model, kind)
    for a, b in zip(outs, again):
        assert np.array_equal(a, b)
    # each sampled crop alone (the B = 1 plan) is bit-identical to its row in the batch
    for i in sample:
        model.forward(x[i:i + 1])
        for got, alone in zip(outs, _heads(model, kind)):
            assert np.array_equal(alone[0], got[i]), i


def test_dense_hier_b256_properties():
    model, wts, depth, x, outs = _run("dense_hier")
    model.forward(x)
    for a, b in zip(outs, _heads(model, "dense_hier")):
        assert np.array_equal(a, b)
    for i in SAMPLE:
        model.forward(x[i:i + 1])
        for got, alone in zip(outs, _heads(model, "dense_hier")):
            assert np.array_equal(alone[0], got[i]), i
    out, parts = RR.dense_hier_forward(depth[[SAMPLE[1]]].astype(np.float64), wts)
    assert rel_inf(outs[0][[SAMPLE[1]]], out) <= FP32_REL_TOL
