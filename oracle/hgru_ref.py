"""CPU ORACLE -- test infrastructure only.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / timed CPU baseline.  The product path
(``monkey-pose_amd``) never imports it and fails loudly when its HIP library is missing.

A NumPy restatement, line by line, of the reference's hot path:

* ``hgru_pose.model.build``            -- ``/root/reference/hgru_pose.py:47-105``
* ``ContextualCircuit.full`` (1 step)  -- ``/root/reference/hgru_module.py:825-857`` with
  ``circuit_input`` 692-724, ``input_integration`` 795-804, ``circuit_output`` 726-756,
  ``output_integration`` 806-823, ``process_p`` 626-658 and ``conv_2d_op`` 505-548
* TF1 op semantics (third-party, not under /root/reference, TF1.x unpinned): ``Conv2D``
  SAME/HWIO cross-correlation, ``MaxPool``/``AvgPool`` SAME, inference ``FusedBatchNorm``
  ``gamma*(x-mean)/sqrt(var+eps)+beta``, ``MatMul`` + ``BiasAdd``.

PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors
and cannot be executed here (Python 2 sources, TensorFlow not installed, and the imported
modules ``utils.py_utils`` / ``ops.initialization`` do not exist: SURVEY.md 8c).  This oracle is
therefore checked only against (a) independent re-implementations of the TF op semantics
(``tests/test_oracle.py`` cross-checks the conv/pool primitives against torch.nn.functional)
and (b) the committed fixtures it generated itself (``tests/golden/``), which pin it against
regressions.  The resolutions of the reference's defects (tuple return, undefined
``self.relu3``, BN ``axis=3`` on a rank-2 tensor, random hidden state) are those of
SURVEY.md 8a and are marked ``DEFECT`` below.

All functions take ``dtype``: float64 is the accuracy reference; float32 is the timed CPU
baseline (``cpu_baseline.kind = "port"`` in bench.py).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

BN_EPS = 1e-5           # hgru_pose.py:17 _BATCH_NORM_EPSILON


# ---------------------------------------------------------------------------------------------
# TF1 primitives
# ---------------------------------------------------------------------------------------------
def same_pads(size: int, k: int, stride: int):
    """TF 'SAME': out = ceil(in/stride); pad_total = max((out-1)*stride + k - in, 0);
    pad_before = pad_total // 2 (stride-2 on even sizes pads 0 before / 1 after)."""
    out = -(-size // stride)
    tot = max((out - 1) * stride + k - size, 0)
    return out, tot // 2, tot - tot // 2


def conv2d_same(x: np.ndarray, w: np.ndarray, stride: int = 1) -> np.ndarray:
    """``tf.nn.conv2d(x, w, [1,s,s,1], 'SAME')``: NHWC input, HWIO filter, cross-correlation.
    Sums over (kx, cin) with one GEMM per filter row ky (im2col over kx)."""
    n, h, wd, cin = x.shape
    kh, kw, cin2, cout = w.shape
    assert cin == cin2
    ho, pt, pb = same_pads(h, kh, stride)
    wo, pl, pr = same_pads(wd, kw, stride)
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    out = np.zeros((n * ho * wo, cout), dtype=x.dtype)
    for ky in range(kh):
        rows = xp[:, ky:ky + stride * (ho - 1) + 1:stride]                 # [n, ho, Wp, cin]
        win = sliding_window_view(rows, kw, axis=2)[:, :, ::stride]        # [n, ho, wo, cin, kw]
        cols = np.ascontiguousarray(win.transpose(0, 1, 2, 4, 3)).reshape(n * ho * wo, kw * cin)
        out += cols @ w[ky].reshape(kw * cin, cout).astype(x.dtype)
    return out.reshape(n, ho, wo, cout)


def bias_relu(x, b):
    return np.maximum(x + b.astype(x.dtype), 0)


def max_pool_same(x: np.ndarray, k: int = 2, s: int = 2) -> np.ndarray:
    """``tf.nn.max_pool`` ksize k stride s SAME (padding never wins the max)."""
    n, h, w, c = x.shape
    ho, pt, pb = same_pads(h, k, s)
    wo, pl, pr = same_pads(w, k, s)
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)), constant_values=-np.inf)
    win = sliding_window_view(xp, (k, k), axis=(1, 2))[:, ::s, ::s]
    return win.max(axis=(-2, -1))


def avg_pool_same(x: np.ndarray, k: int = 2, s: int = 2) -> np.ndarray:
    """``tf.nn.avg_pool`` SAME: the divisor counts only in-image elements."""
    n, h, w, c = x.shape
    ho, pt, pb = same_pads(h, k, s)
    wo, pl, pr = same_pads(w, k, s)
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    ones = np.pad(np.ones((1, h, w, 1), x.dtype), ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    sm = sliding_window_view(xp, (k, k), axis=(1, 2))[:, ::s, ::s].sum(axis=(-2, -1))
    cnt = sliding_window_view(ones, (k, k), axis=(1, 2))[:, ::s, ::s].sum(axis=(-2, -1))
    return sm / cnt


def batch_norm_inf(x, wts: Dict[str, np.ndarray], scope: str, eps: float = BN_EPS):
    """Inference ``tf.layers.batch_normalization`` over the last axis."""
    dt = x.dtype
    g = wts[f"{scope}/gamma"].astype(dt)
    b = wts[f"{scope}/beta"].astype(dt)
    m = wts[f"{scope}/moving_mean"].astype(dt)
    v = wts[f"{scope}/moving_variance"].astype(dt)
    return g * (x - m) / np.sqrt(v + dt.type(eps)) + b


def fc(x, w, b):
    """``fc_layer``: reshape to [-1, in] (row-major NHWC flatten) then matmul + bias_add."""
    x2 = x.reshape(x.shape[0], -1)
    return x2 @ w.astype(x.dtype) + b.astype(x.dtype)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


# ---------------------------------------------------------------------------------------------
# hGRU contextual circuit (hgru_module.py) with the hgru_pose aux (hgru_pose.py:20-39)
# ---------------------------------------------------------------------------------------------
def _vec(wts, scope, nm, dt):
    return wts[f"{scope}/{nm}"].astype(dt).reshape(-1)


def hgru_step(X, O, t, wts, scope="cnn/contextual_circuit", return_all=False):
    """One ``full`` iteration (hgru_module.py:825-857).  aux: gru_gates=True, output_gru_gates=
    False, association_field=True, multiplicative_excitation=True, gamma=True, adapation=True,
    xi=zeta=1 (constants, 438/464), rectify_weights=None (no rectification, 721/753)."""
    dt = X.dtype
    p_r = wts[f"{scope}/p_r"].astype(dt)
    i_r = wts[f"{scope}/i_r"].astype(dt)
    o_r = wts[f"{scope}/o_r"].astype(dt)
    i_b, o_b = _vec(wts, scope, "i_b", dt), _vec(wts, scope, "o_b", dt)
    beta, nu = _vec(wts, scope, "beta", dt), _vec(wts, scope, "nu", dt)
    gamma, kappa, omega = (_vec(wts, scope, n, dt) for n in ("gamma", "kappa", "omega"))
    lat = _vec(wts, scope, "lateral_bias", dt)
    rho = wts[f"{scope}/rho"].astype(dt).reshape(-1)

    # circuit_input (692-724): gate conv (gate_filter=1 -> full conv branch of conv_2d_op 531-548)
    g1 = sigmoid(conv2d_same(O, i_r) + i_b)                      # 696-707
    Og = O * g1                                                   # 711: rebinds the *local* O
    P1 = conv2d_same(Og, p_r) + lat                               # 714-718 -> process_p 657
    # input_integration (795-804), gru_gates=True branch 804; uses the caller's un-gated O
    I = np.tanh(X - (beta * O + nu) * P1)
    # circuit_output (726-756): output_gru_gates=False so I is not gated
    g2 = sigmoid(conv2d_same(I, o_r) + o_b)
    P2 = conv2d_same(I, p_r) + lat
    # output_integration (806-823), multiplicative_excitation branch, zeta = 1
    e = gamma * P2
    a = kappa * (I + e)
    m = omega * (I * e)
    S = np.tanh(a + m)
    On = g2 * O + (1 - g2) * S
    On = On * rho[t]                                              # adapation, 847-849
    if return_all:
        return On, dict(g1=g1, P1=P1, I=I, g2=g2, P2=P2)
    return On


def hidden_init_state(X, hidden_init="random", O0=None):
    """The initial output state O0 of ``ContextualCircuit.build`` (hgru_module.py:875-890):
    'identity' -> X (876-878), 'zeros' -> zeros_like(X) (888-890), 'random' -> the externally
    supplied draw ``O0`` (879-887, DEFECT 2).  The initial I is never read (795-804)."""
    if hidden_init == "identity":
        return X
    if hidden_init == "zeros":
        return X * 0
    if hidden_init == "random":
        if O0 is None:
            raise ValueError("hidden_init='random' needs the drawn O0")
        return O0
    raise RuntimeError(hidden_init)     # hgru_module.py:891-892


def hgru_forward(X, O0, wts, timesteps=8, scope="cnn/contextual_circuit", keep_steps=False,
                 keep_inputs=False):
    """``ContextualCircuit.build`` (872-954) with hidden_init='random' made explicit: ``O0`` is
    the (DEFECT 2) externally supplied initial output state; the random I0 is dead because the
    gru_gates input integration ignores the previous I (795-804).  Returns O_T (DEFECT 3: the
    reference returns the tuple (O, weights, activities); only O is consumed).
    ``keep_steps``: also the per-step O_t after the rho gain, as ``store_states`` writes them
    (912-915); ``keep_inputs`` additionally the per-step I_t -> (O, O_steps, I_steps)."""
    O = O0.astype(X.dtype)
    steps, isteps = [], []
    for t in range(timesteps):
        if keep_inputs:
            O, parts = hgru_step(X, O, t, wts, scope, return_all=True)
            isteps.append(parts["I"].copy())
        else:
            O = hgru_step(X, O, t, wts, scope)
        if keep_steps or keep_inputs:
            steps.append(O.copy())
    if keep_inputs:
        return O, steps, isteps
    return (O, steps) if keep_steps else O


# ---------------------------------------------------------------------------------------------
# hgru_pose.model.build (hgru_pose.py:47-105), inference (train_mode falsy)
# ---------------------------------------------------------------------------------------------
def hgru_pose_forward(depth: np.ndarray, wts: Dict[str, np.ndarray], O0: Optional[np.ndarray],
                      timesteps: int = 8, dtype=np.float64, keep: bool = False,
                      hidden_init: str = "random"):
    x = depth.astype(dtype)
    inter = {}
    c1 = bias_relu(conv2d_same(x, wts["cnn/conv_1/conv_1_filters"].astype(dtype)),
                   wts["cnn/conv_1/conv_1_biases"])                                  # 50
    p1 = max_pool_same(c1)                                                            # 51
    p1 = batch_norm_inf(p1, wts, "cnn/batch_normalization")                           # 52-60
    c2 = bias_relu(conv2d_same(p1, wts["cnn/conv_2/conv_2_filters"].astype(dtype)),
                   wts["cnn/conv_2/conv_2_biases"])                                  # 61
    c2 = batch_norm_inf(c2, wts, "cnn/batch_normalization_1")                         # 62-70
    c3 = bias_relu(conv2d_same(c2, wts["cnn/conv_3/conv_3_filters"].astype(dtype)),
                   wts["cnn/conv_3/conv_3_biases"])                                  # 71
    c3 = batch_norm_inf(c3, wts, "cnn/batch_normalization_2")                         # 72-80
    if keep:
        inter.update(conv1=c1, pool1=p1, conv2=c2, conv3=c3)
    O0 = hidden_init_state(c3, hidden_init, O0)                                       # 81
    h = hgru_forward(c3, O0, wts, timesteps, keep_inputs=keep)
    if keep:
        h, steps, isteps = h
        inter["hgru_steps"] = steps
        inter["hgru_isteps"] = isteps
    h = batch_norm_inf(h, wts, "cnn/batch_normalization_3")                           # 82-90
    f1 = fc(h, wts["cnn/fc_1/fc_1_weights"], wts["cnn/fc_1/fc_1_biases"])             # 91
    r1 = np.maximum(f1, 0)                                                            # 92
    # DEFECT 5: axis=3 on a rank-2 tensor -> per-feature BN over the 1024 axis     # 95-103
    r1 = batch_norm_inf(r1, wts, "cnn/batch_normalization_4")
    # DEFECT 4: fc_out consumes the BN'd relu1 (self.relu3 is undefined at 104)
    out = fc(r1, wts["cnn/fc_out/fc_out_weights"], wts["cnn/fc_out/fc_out_biases"])   # 104-105
    if keep:
        inter.update(hgru_bn=h, fc1=f1, relu1_bn=r1)
        return out, inter
    return out


# ---------------------------------------------------------------------------------------------
# post-processing / metric
# ---------------------------------------------------------------------------------------------
def to_joints_mm(out: np.ndarray, cube_z: float = 1200.0) -> np.ndarray:
    """``tf.reshape(model.out_put, [B, J, 3]) * cube[2] / 2`` (train_cnn_networks_hgru.py:155)."""
    return out.reshape(out.shape[0], -1, 3) * (cube_z / 2.0)


def mean_error(labels: np.ndarray, results: np.ndarray) -> float:
    """``getMeanError_train`` (pose_evaluation.py:30-36): mean over batch of the mean over joints
    of the Euclidean joint error."""
    return float(np.mean(np.mean(np.sqrt(np.sum((labels - results) ** 2, axis=2)), axis=1)))


def hgru_pose_flops(batch: int, timesteps: int = 8, k: int = 64, hw: int = 64, ssf: int = 15,
                    crop: int = 128, nout: int = 69) -> Dict[str, float]:
    """Algorithmic FLOPs (multiply-add = 2), SURVEY.md 8d."""
    px = hw * hw
    conv15 = 2.0 * px * ssf * ssf * k * k
    gate = 2.0 * px * k * k
    hgru = timesteps * 2 * (conv15 + gate)
    backbone = 2.0 * crop * crop * 9 * 1 * k + 2 * (2.0 * px * 9 * k * k)
    fc1 = 2.0 * px * k * 1024
    fco = 2.0 * 1024 * nout
    return {k_: v * batch for k_, v in dict(conv15_per_launch=conv15, hgru=hgru,
                                             backbone=backbone, fc1=fc1, fc_out=fco,
                                             total=hgru + backbone + fc1 + fco).items()}
