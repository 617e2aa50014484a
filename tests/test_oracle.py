"""CPU: the oracle against independent restatements of the TF op semantics, a naive per-pixel
restatement of one hGRU step, and the committed golden vectors (regression pin)."""
import math

import numpy as np
import pytest

from helpers import MG, golden_array, golden_meta, rel_inf
from oracle import hgru_ref as R

torch = pytest.importorskip("torch")
F = torch.nn.functional


def _tf_same_conv_torch(x, w, s):
    n, h, wd, ci = x.shape
    k = w.shape[0]
    ho = -(-h // s)
    wo = -(-wd // s)
    th = max((ho - 1) * s + k - h, 0)
    tw = max((wo - 1) * s + k - wd, 0)
    xt = torch.tensor(x).permute(0, 3, 1, 2)
    xt = F.pad(xt, (tw // 2, tw - tw // 2, th // 2, th - th // 2))
    return F.conv2d(xt, torch.tensor(w).permute(3, 2, 0, 1), stride=s).permute(0, 2, 3, 1).numpy()


@pytest.mark.parametrize("h,w,k,s,ci,co", [(16, 16, 3, 1, 5, 7), (16, 16, 3, 2, 5, 7), (15, 13, 3, 2, 4, 3),
                                          (17, 17, 5, 1, 3, 2), (16, 16, 15, 1, 4, 4), (9, 9, 1, 1, 3, 3),
                                          (32, 32, 5, 2, 2, 3)])
def test_conv2d_same_matches_independent(h, w, k, s, ci, co):
    rng = np.random.default_rng(h * 100 + k * 10 + s)
    x = rng.standard_normal((2, h, w, ci))
    wt = rng.standard_normal((k, k, ci, co))
    assert np.allclose(R.conv2d_same(x, wt, s), _tf_same_conv_torch(x, wt, s), atol=1e-11)


def test_same_padding_rule():
    # TF SAME: stride-2 on an even size pads 0 before / 1 after
    assert R.same_pads(64, 3, 2) == (32, 0, 1)
    assert R.same_pads(64, 3, 1) == (64, 1, 1)
    assert R.same_pads(64, 15, 1) == (64, 7, 7)
    assert R.same_pads(15, 2, 2) == (8, 0, 1)


def test_pools():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, 8, 8, 3))
    mp_ = R.max_pool_same(x)
    ref = F.max_pool2d(torch.tensor(x).permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1).numpy()
    assert np.array_equal(mp_, ref)
    ap = R.avg_pool_same(x)
    ref = F.avg_pool2d(torch.tensor(x).permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1).numpy()
    assert np.allclose(ap, ref)
    # odd size: TF SAME pads after; max ignores the pad, avg divides by the in-image count
    x = rng.standard_normal((1, 5, 5, 1))
    m = R.max_pool_same(x)
    assert m.shape == (1, 3, 3, 1) and m[0, 2, 2, 0] == x[0, 4, 4, 0]
    a = R.avg_pool_same(x)
    assert math.isclose(a[0, 2, 2, 0], x[0, 4, 4, 0]) and math.isclose(a[0, 0, 2, 0], x[0, 0:2, 4, 0].mean())


def test_batch_norm_inference():
    rng = np.random.default_rng(2)
    x = rng.standard_normal((3, 4, 4, 6))
    wts = {"s/gamma": rng.random(6) + 0.5, "s/beta": rng.standard_normal(6),
           "s/moving_mean": rng.standard_normal(6), "s/moving_variance": rng.random(6) + 0.1}
    y = R.batch_norm_inf(x, wts, "s")
    ref = (x - wts["s/moving_mean"]) / np.sqrt(wts["s/moving_variance"] + 1e-5) * wts["s/gamma"] + wts["s/beta"]
    assert np.allclose(y, ref)


def _naive_step(X, O, t, p):
    """Per-pixel loops straight from hgru_module.py:692-857 (gru_gates, multiplicative
    excitation, adaptation; SAME zero padding)."""
    n, h, w, k = X.shape
    S = p["p_r"].shape[0]
    r = S // 2
    sig = lambda v: 1.0 / (1.0 + math.exp(-v))

    def conv(inp, Wt):
        out = np.zeros_like(inp)
        for b in range(n):
            for y in range(h):
                for x in range(w):
                    for co in range(k):
                        s = 0.0
                        for ky in range(Wt.shape[0]):
                            for kx in range(Wt.shape[1]):
                                yy, xx = y + ky - Wt.shape[0] // 2, x + kx - Wt.shape[1] // 2
                                if 0 <= yy < h and 0 <= xx < w:
                                    for ci in range(k):
                                        s += inp[b, yy, xx, ci] * Wt[ky, kx, ci, co]
                        out[b, y, x, co] = s
        return out

    v = lambda nm: p[nm].reshape(-1)
    g1 = np.vectorize(sig)(conv(O, p["i_r"]) + v("i_b"))
    P1 = conv(O * g1, p["p_r"]) + v("lateral_bias")
    I = np.tanh(X - (v("beta") * O + v("nu")) * P1)
    g2 = np.vectorize(sig)(conv(I, p["o_r"]) + v("o_b"))
    P2 = conv(I, p["p_r"]) + v("lateral_bias")
    e = v("gamma") * P2
    Sx = np.tanh(v("kappa") * (I + e) + v("omega") * (I * e))
    return (g2 * O + (1 - g2) * Sx) * p["rho"][t]


def test_hgru_step_matches_naive_restatement():
    rng = np.random.default_rng(3)
    k, h, w = 3, 4, 5
    p = {"p_r": rng.standard_normal((3, 3, k, k)) * 0.3, "i_r": rng.standard_normal((1, 1, k, k)),
         "o_r": rng.standard_normal((1, 1, k, k)), "rho": np.array([0.9, 1.1])}
    for nm in ("i_b", "o_b", "beta", "nu", "gamma", "kappa", "omega", "lateral_bias"):
        p[nm] = rng.standard_normal((1, 1, 1, k)) * 0.5
    wts = {f"cnn/contextual_circuit/{a}": b for a, b in p.items()}
    X = rng.standard_normal((2, h, w, k))
    O = rng.standard_normal((2, h, w, k)) * 0.5
    for t in range(2):
        ref = _naive_step(X, O, t, p)
        got = R.hgru_step(X, O, t, wts)
        assert np.allclose(got, ref, atol=1e-12)
        O = ref


@pytest.mark.parametrize("case", [c[0] for c in MG.CIRCUIT_CASES])
def test_oracle_reproduces_golden_circuit(case):
    meta = golden_meta()[case]
    wts, X, O0 = MG.circuit_inputs(meta["n"], meta["h"], meta["w"], meta["ssf"], meta["timesteps"],
                                   meta["weight_seed"], meta["x_seed"], meta["o0_seed"])
    O, steps = R.hgru_forward(X.astype(np.float64), O0, wts, meta["timesteps"], keep_steps=True)
    assert rel_inf(O, golden_array(case, "O")) < 1e-6
    for s, cs in zip(steps, meta["step_checksums"]):
        assert np.allclose(MG.checksums(s), cs, rtol=1e-9)


@pytest.mark.parametrize("case", [c[0] for c in MG.POSE_CASES])
def test_oracle_reproduces_golden_pose(case):
    meta = golden_meta()[case]
    wts, depth, O0 = MG.pose_inputs(meta["n"], meta["crop"], meta["timesteps"], meta["weight_seed"],
                                    meta["crop_seed"], meta["o0_seed"])
    out = R.hgru_pose_forward(depth, wts, O0, meta["timesteps"], np.float64)
    assert rel_inf(out, golden_array(case, "out")) < 1e-9


def test_metric_and_joint_layout():
    rng = np.random.default_rng(4)
    out = rng.standard_normal((3, 69))
    j = R.to_joints_mm(out)
    assert j.shape == (3, 23, 3) and np.allclose(j[1, 5], out[1, 15:18] * 600.0)
    lab = j + np.array([3.0, 4.0, 0.0])
    assert math.isclose(R.mean_error(lab, j), 5.0)


def test_fp32_port_close_to_fp64():
    meta = golden_meta()["pose_c64_t8"]
    wts, depth, O0 = MG.pose_inputs(1, 64, 8, meta["weight_seed"], meta["crop_seed"], meta["o0_seed"])
    a = R.hgru_pose_forward(depth, wts, O0, 8, np.float32)
    b = golden_array("pose_c64_t8", "out")[:1]
    assert a.dtype == np.float32 and rel_inf(a, b) < 1e-4


@pytest.mark.parametrize("case", ["pose_c64_t8", "pose_c128_t8"])
def test_torch_cpu_baseline_matches_oracle(case):
    """bench.py's timed CPU baseline (oracle/hgru_torch_cpu.py, torch-CPU fp32, BASELINE.md's
    plan) computes the same forward as the float64 oracle: within the fp32 gate of the golden."""
    from oracle import hgru_torch_cpu as TC
    meta = golden_meta()[case]
    wts, depth, O0 = MG.pose_inputs(meta["n"], meta["crop"], meta["timesteps"], meta["weight_seed"],
                                    meta["crop_seed"], meta["o0_seed"])
    out = TC.forward(depth, TC.prepare(wts, meta["timesteps"]), O0, meta["timesteps"])
    assert rel_inf(out, golden_array(case, "out")) <= 1e-4
