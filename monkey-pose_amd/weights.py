"""Variable tables and deterministic synthetic initialisers for the pose regressors.

Every tensor is keyed by the TensorFlow variable name the reference creates, so a
checkpoint exported from the reference (``{name: ndarray}``) loads unchanged:

* ``cnn/conv_1/conv_1_filters`` ... -- ``hgru_pose.conv_layer`` -> ``get_conv_var``
  (``hgru_pose.py:139-180``; scope ``cnn`` from ``train_cnn_networks_hgru.py:95``)
* ``cnn/batch_normalization{,_1.._4}/{gamma,beta,moving_mean,moving_variance}`` --
  the five ``tf.layers.batch_normalization`` calls (``hgru_pose.py:52-103``)
* ``cnn/contextual_circuit/{p_r,i_r,i_b,o_r,o_b,beta,nu,gamma,kappa,omega,rho,lateral_bias}``
  -- ``hgru_module.ContextualCircuit.prepare_tensors`` (``hgru_module.py:262-503``)
* ``cnn/fc_1/fc_1_weights`` ... -- ``hgru_pose.fc_layer`` / ``get_fc_var`` (156-194)

The reference draws its initial values from TF1 initialisers (truncated normal xavier,
``hgru_module.py:5`` ``ops.initialization`` which is *not vendored*), so the synthetic
values here are NOT the reference's random draws -- they are a reproducible stand-in with
the same shapes and variance class (glorot-uniform), generated from a splitmix64 hash so
that the numpy oracle and the HIP path see bit-identical weights for a given seed.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np

# ---------------------------------------------------------------------------
# splitmix64 counter-based generator (vectorised, chunked)
# ---------------------------------------------------------------------------
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def uniform01(seed: int, name: str, n: int, out: np.ndarray | None = None,
              chunk: int = 1 << 22) -> np.ndarray:
    """``n`` doubles in [0,1) from splitmix64(key + i*golden); float64 unless ``out`` given."""
    key = np.uint64((_fnv1a64(name) ^ (seed * 0x2545F4914F6CDD1D)) & 0xFFFFFFFFFFFFFFFF)
    if out is None:
        out = np.empty(n, dtype=np.float64)
    with np.errstate(over="ignore"):
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            idx = np.arange(s, e, dtype=np.uint64)
            z = _mix(idx * _GOLDEN + key)
            out[s:e] = (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    return out


def sym_uniform(seed: int, name: str, shape: Sequence[int], limit: float,
                dtype=np.float32) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform01(seed, name, n)
    return ((2.0 * u - 1.0) * limit).astype(dtype).reshape(shape)


def glorot_limit(shape: Sequence[int]) -> float:
    """TF glorot fan rule: conv kernels [kh,kw,in,out] -> fans scaled by the receptive field."""
    shape = list(shape)
    if len(shape) == 2:
        fan_in, fan_out = shape
    elif len(shape) >= 3:
        rf = int(np.prod(shape[:-2]))
        fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
    else:
        fan_in = fan_out = shape[0]
    return math.sqrt(6.0 / (fan_in + fan_out))


# ---------------------------------------------------------------------------
# variable table
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class Var:
    name: str
    shape: Tuple[int, ...]
    init: str          # see synth_value


def _bn(scope: str, n: int) -> List[Var]:
    return [Var(f"{scope}/gamma", (n,), "bn_gamma"), Var(f"{scope}/beta", (n,), "bn_beta"),
            Var(f"{scope}/moving_mean", (n,), "bn_mean"),
            Var(f"{scope}/moving_variance", (n,), "bn_var")]


def _conv(scope: str, k: int, cin: int, cout: int) -> List[Var]:
    return [Var(f"{scope}/{scope.split('/')[-1]}_filters", (k, k, cin, cout), "glorot"),
            Var(f"{scope}/{scope.split('/')[-1]}_biases", (cout,), "bias")]


def _fc(scope: str, nin: int, nout: int) -> List[Var]:
    return [Var(f"{scope}/{scope.split('/')[-1]}_weights", (nin, nout), "glorot"),
            Var(f"{scope}/{scope.split('/')[-1]}_biases", (nout,), "bias")]


def hgru_circuit_vars(k: int = 64, ssf: int = 15, gate_filter: int = 1, timesteps: int = 8,
                      scope: str = "cnn/contextual_circuit") -> List[Var]:
    """``prepare_tensors`` with the hgru_pose aux (``hgru_pose.py:20-39``): association field,
    gru gates, gamma, multiplicative excitation, adaptation (rho); xi/zeta constant 1."""
    v = [Var(f"{scope}/p_r", (ssf, ssf, k, k), "glorot"),                    # 298-310
         Var(f"{scope}/i_r", (gate_filter, gate_filter, k, k), "glorot"),    # 322-332
         Var(f"{scope}/i_b", (1, 1, 1, k), "chronos"),                       # 344-357
         Var(f"{scope}/o_r", (gate_filter, gate_filter, k, k), "glorot"),    # 360-370
         Var(f"{scope}/o_b", (1, 1, 1, k), "neg_chronos")]                   # 382-396
    for nm in ("beta", "nu", "gamma", "kappa", "omega"):                    # 405-486
        v.append(Var(f"{scope}/{nm}", (1, 1, 1, k), "glorot"))
    v.append(Var(f"{scope}/rho", (timesteps,), "ones"))                      # 490-493
    v.append(Var(f"{scope}/lateral_bias", (1, 1, 1, k), "glorot"))           # 498-503
    return v


def hgru_pose_vars(output_shape: int = 69, timesteps: int = 8, crop=128,
                   k: int = 64) -> List[Var]:
    """All variables of ``hgru_pose.model.build`` (``hgru_pose.py:47-105``) in build order.
    ``crop`` is the input size (int or (h, w)); fc_1's fan-in is (h/2)*(w/2)*64."""
    ch, cw = (crop, crop) if isinstance(crop, int) else crop
    v: List[Var] = []
    v += _conv("cnn/conv_1", 3, 1, k)
    v += _bn("cnn/batch_normalization", k)
    v += _conv("cnn/conv_2", 3, k, k)
    v += _bn("cnn/batch_normalization_1", k)
    v += _conv("cnn/conv_3", 3, k, k)
    v += _bn("cnn/batch_normalization_2", k)
    v += hgru_circuit_vars(k=k, timesteps=timesteps)
    v += _bn("cnn/batch_normalization_3", k)
    v += _fc("cnn/fc_1", (ch // 2) * (cw // 2) * k, 1024)
    v += _bn("cnn/batch_normalization_4", 1024)
    v += _fc("cnn/fc_out", 1024, output_shape)
    return v


def _conv_b(name: str, k: int, cin: int, cout: int) -> List[Var]:
    return _conv(f"cnn/{name}", k, cin, cout)


# dense_model_struct widths per layer 3..6 (train_dense_networks.py:250-373):
# (scale-1 1x1, scale-1 3x3, s2-from-s1 1x1, s2 3x3/2, s2 1x1, s2 3x3, s3-from-s2 1x1, s3 3x3/2,
#  s3 1x1, s3 3x3)
DENSE_WIDTHS = {3: (24, 32, 32, 48, 32, 48, 48, 64, 48, 64),
                4: (32, 48, 48, 64, 48, 64, 64, 96, 64, 96),
                5: (48, 64, 64, 96, 64, 96, 96, 128, 96, 128),
                6: (64, 96, 96, 128, 96, 128, 128, 144, 128, 144)}


def dense_conv_specs():
    """[(name, k, stride, cin, cout)] of dense_model_struct.build in call order (49 convs)."""
    s = [("conv_0", 3, 1, 1, 12), ("conv_1_1", 3, 1, 12, 16), ("conv_1_2", 3, 2, 16, 24),
         ("conv_1_3", 3, 2, 24, 32), ("conv_2_1", 3, 1, 16, 24), ("conv_2_2_1", 3, 2, 16, 24),
         ("conv_2_2_2", 3, 1, 24, 32), ("conv_2_3_2", 3, 2, 24, 32), ("conv_2_3_3", 3, 1, 32, 48)]
    w1, w2, w3 = 16 + 24, 24 + 56, 32 + 80          # widths of conv{3}_{1,2,3}_in
    for L in (3, 4, 5, 6):
        a, b, c, d, e, f, g, h, i, j = DENSE_WIDTHS[L]
        s += [(f"conv_{L}_1_1x1", 1, 1, w1, a), (f"conv_{L}_1", 3, 1, a, b),
              (f"conv_{L}_2_1x1_1", 1, 1, w1, c), (f"conv_{L}_2_1", 3, 2, c, d),
              (f"conv_{L}_2_1x1_2", 1, 1, w2, e), (f"conv_{L}_2_2", 3, 1, e, f),
              (f"conv_{L}_3_1x1_2", 1, 1, w2, g), (f"conv_{L}_3_2", 3, 2, g, h),
              (f"conv_{L}_3_1x1_3", 1, 1, w3, i), (f"conv_{L}_3_3", 3, 1, i, j)]
        w1, w2, w3 = w1 + b, w2 + d + f, w3 + h + j
    return s


def dense_vars(output_shape: int = 69, crop: int = 128) -> List[Var]:
    """All variables of ``dense_model_struct.build`` (train_dense_networks.py:223-408)."""
    v: List[Var] = []
    for name, k, _, cin, cout in dense_conv_specs():
        v += _conv_b(name, k, cin, cout)
    q = crop // 4   # conv6_1 is at crop/2, avg-pooled to crop/4
    v += _fc("cnn/fc_1_1", q * q * 96, 512)
    v += _fc("cnn/fc_1_2", (q // 2) * (q // 2) * 256, 512)
    v += _fc("cnn/fc_1_3", (q // 4) * (q // 4) * 288, 512)
    v += _fc("cnn/fc_2", 1536, 1024)
    v += _fc("cnn/fc_3", 1024, 512)
    v += _fc("cnn/fc_4", 512, output_shape)
    return v


# cnn_model_struct.build (train_cnn_networks_hgru.py:639-673): the hGRU driver's validation / test
# regressor -- five conv + 2x2 max-pool stages, then fc_1 .. fc_4
CNN_CONV_SPECS = (("conv_1", 3, 1, 64), ("conv_2", 3, 64, 128), ("conv_3", 3, 128, 256),
                  ("conv_4", 3, 256, 512), ("conv_5", 5, 512, 1024))


def cnn_vars(output_shape: int = 69, crop: int = 128) -> List[Var]:
    """All variables of ``cnn_model_struct.build`` in build order; fc_1's fan-in is the flattened
    pool_5 (five 2x2 pools: (crop / 32)^2 x 1024, 16,384 at 128 x 128, 652)."""
    v: List[Var] = []
    for name, k, cin, cout in CNN_CONV_SPECS:
        v += _conv_b(name, k, cin, cout)
    q = -(-crop // 32)
    v += _fc("cnn/fc_1", q * q * 1024, 1024) + _fc("cnn/fc_2", 1024, 1024) + _fc("cnn/fc_3", 1024, 1024)
    v += _fc("cnn/fc_4", 1024, output_shape)
    return v


HIER_FINGERS = ("p", "r", "m", "i", "t")


def hier_conv_specs():
    """[(name, k, stride, cin, cout)] of hier_model_struct.build (train_hier_networks.py:341-469)."""
    s = [("conv_1", 3, 1, 1, 64), ("conv_2", 3, 1, 64, 128)]
    for br in ("pr", "mi", "t"):
        s += [(f"{br}_con_3", 3, 1, 128, 256), (f"{br}_con_4", 3, 1, 256, 512)]
    for f in HIER_FINGERS:
        s += [(f"{f}_con_5", 3, 1, 512, 512), (f"{f}_con_6", 5, 1, 512, 1024)]
    return s


def hier_vars(output_shape: int = 108, part_shapes=(39, 39, 39, 39, 36), crop: int = 128) -> List[Var]:
    """All variables of ``hier_model_struct.build``; head sizes as at its call site
    (train_hier_networks.py:263: num_classes, 13*3, 13*3, 13*3, 13*3, 12*3)."""
    v: List[Var] = []
    for name, k, _, cin, cout in hier_conv_specs():
        v += _conv_b(name, k, cin, cout)
    q = crop // 64                  # six 2x2 pools
    flat = q * q * 1024
    for f, ps in zip(HIER_FINGERS, part_shapes):
        v += _fc(f"cnn/{f}_fc_1", flat, 1024) + _fc(f"cnn/{f}_fc_2", 1024, 1024)
        v += _fc(f"cnn/{f}_fc_3", 1024, ps)
    for f in HIER_FINGERS:
        v += _fc(f"cnn/{f}h_fc_1", flat, 1024) + _fc(f"cnn/{f}h_fc_2", 1024, 1024)
    v += _fc("cnn/final_fc_1", 5120, 1024) + _fc("cnn/final_fc_2", 1024, output_shape)
    return v


ATTN_CONV_SPECS = (("aconv_1", 3, 1, 64), ("aconv_2", 3, 64, 128), ("aconv_3", 3, 128, 256),
                   ("aconv_4", 3, 256, 512), ("aconv_5", 5, 512, 1024))


def attn_vars(output_shape: int = 3) -> List[Var]:
    """All variables of ``attn_model_struct.build`` (train_cnn_networks_hgru.py:436-525) in build
    order.  Input is resized to 128x128 (439), so afc_1's fan-in is 4*4*1024 for any frame size.
    The six ``tf.layers.batch_normalization`` calls take the default scopes of a fresh ``cnn``
    scope (``batch_normalization`` .. ``_5``); in the reference's combined test graph (attention
    built first, train_cnn_networks_hgru.py:285-289) the pose model's BNs follow as ``_6`` ..."""
    bn = ["cnn/batch_normalization"] + [f"cnn/batch_normalization_{i}" for i in range(1, 6)]
    v: List[Var] = []
    for (name, k, cin, cout), b in zip(ATTN_CONV_SPECS, bn):
        v += _conv_b(name, k, cin, cout)
        v += _bn(b, cout)
    v += _fc("cnn/afc_1", 4 * 4 * 1024, 1024)
    v += _bn(bn[5], 1024)
    v += _fc("cnn/afc_out", 1024, output_shape)
    return v


def attn_synth_weights(seed: int = 1234, output_shape: int = 3) -> Dict[str, np.ndarray]:
    """Synthetic attention weights whose CoM output lands inside a 424x512 frame: the glorot draw
    for everything, then afc_out scaled by 1/64 with biases (0.5, 0.5, 0.15), i.e. a CoM near
    (212, 256, 1500 mm) +- a few pixels (com = out * (424, 512, 10000),
    train_cnn_networks_hgru.py:69).  Only the synthetic end-to-end chain needs this; a plain
    ``synth_weights(attn_vars())`` draw gives arbitrary CoMs, most of which crop nothing."""
    w = synth_weights(attn_vars(output_shape), seed)
    w["cnn/afc_out/afc_out_weights"] = (w["cnn/afc_out/afc_out_weights"] / 64.0).astype(np.float32)
    b = np.zeros(output_shape, np.float32)
    b[:3] = (0.5, 0.5, 0.15)[:min(3, output_shape)]
    w["cnn/afc_out/afc_out_biases"] = b
    return w


def synth_value(var: Var, seed: int, timesteps: int = 8) -> np.ndarray:
    """Deterministic stand-in for the reference's TF initialisers (see module docstring)."""
    s, nm, kind = var.shape, var.name, var.init
    n = int(np.prod(s))
    if kind == "glorot":
        return sym_uniform(seed, nm, s, glorot_limit(s))
    if kind == "bias":
        return sym_uniform(seed, nm, s, 1e-2)
    if kind == "bn_gamma":
        return (1.0 + sym_uniform(seed, nm, s, 0.1, np.float64)).astype(np.float32)
    if kind in ("bn_beta", "bn_mean"):
        return sym_uniform(seed, nm, s, 0.1)
    if kind == "bn_var":
        return (1.0 + sym_uniform(seed, nm, s, 0.1, np.float64)).astype(np.float32)
    if kind in ("chronos", "neg_chronos"):
        # i_b = -log(U(1, T-1)); o_b = -i_b   (hgru_module.py:344-347, 386)
        base = nm.rsplit("/", 1)[0] + "/i_b"
        u = uniform01(seed, base, n).reshape(s)
        ib = -np.log(1.0 + u * (timesteps - 2))
        return (ib if kind == "chronos" else -ib).astype(np.float32)
    if kind == "ones":
        return np.ones(s, np.float32)
    raise ValueError(kind)


def synth_weights(vars_: Sequence[Var], seed: int = 1234, timesteps: int = 8) -> Dict[str, np.ndarray]:
    return {v.name: synth_value(v, seed, timesteps) for v in vars_}


def synth_hidden(shape: Sequence[int], seed: int = 7, name: str = "h2_init",
                 limit: float | None = None) -> np.ndarray:
    """Default hGRU output-state init O0 (``hgru_module.py:879-887``: xavier tensor, re-drawn per
    run).  The reference's ``ops.initialization`` is missing, so the scale is unpinned; we use
    glorot-uniform with fan_in = fan_out = k."""
    k = shape[-1]
    if limit is None:
        limit = math.sqrt(6.0 / (2 * k))
    return sym_uniform(seed, name, shape, limit)


def synth_frames(n: int, seed: int = 11, h: int = 424, w: int = 512) -> np.ndarray:
    """Synthetic normalised full depth frames [n,h,w,1] float32 (mm / 10000, the attention net's
    input, train_cnn_networks_hgru.py:116): a far wall at 3000-4000 mm, one ellipsoid body at
    800-1500 mm, ~3 % zero dropout; depths are whole millimetres as from a Kinect."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    out = np.empty((n, h, w), np.float32)
    for i in range(n):
        u = uniform01(seed, f"frame{i}", 8)
        f = 3000.0 + 1000.0 * u[0] + 200.0 * np.sin(xx / 37.0) * np.cos(yy / 23.0)
        cy, cx = (0.3 + 0.4 * u[1]) * h, (0.3 + 0.4 * u[2]) * w
        ry, rx = 30 + 60 * u[3], 30 + 60 * u[4]
        r2 = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2
        f = np.where(r2 < 1.0, 800.0 + 700.0 * u[5] + 50.0 * r2, f)
        f[uniform01(seed, f"fdrop{i}", h * w).reshape(h, w) < 0.03] = 0.0
        out[i] = (np.round(f).astype(np.float32) / np.float32(10000.0))
    return out[..., None]


def synth_crops(n: int, seed: int = 42, size: int = 128) -> np.ndarray:
    """Synthetic normalised depth crops [n,size,size,1] float32: background 1.0 (the
    ``maxDepth`` canvas fill, ``tf_monkeydetector.py:353`` / 10000), a few ellipsoid blobs at
    depth 0.20-0.30, ~5 % dropout pixels at 0.0."""
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float64)
    out = np.ones((n, size, size), np.float64)
    for i in range(n):
        u = uniform01(seed, f"crop{i}", 64)
        nb = 3 + int(u[0] * 4)
        for b in range(nb):
            cy, cx = size * (0.2 + 0.6 * u[1 + 6 * b]), size * (0.2 + 0.6 * u[2 + 6 * b])
            ry, rx = size * (0.05 + 0.2 * u[3 + 6 * b]), size * (0.05 + 0.2 * u[4 + 6 * b])
            d0 = 0.20 + 0.10 * u[5 + 6 * b]
            r2 = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2
            m = r2 < 1.0
            out[i][m] = np.minimum(out[i][m], d0 + 0.02 * r2[m])
        drop = uniform01(seed, f"drop{i}", size * size).reshape(size, size) < 0.05
        out[i][drop] = 0.0
    return out.astype(np.float32)[..., None]
