"""CPU ORACLE (test infrastructure only; see oracle/hgru_ref.py for the import rule and the
"parity unpinned" statement, which applies here too).

NumPy restatements of the two other pose regressors on the north-star path, call for call:

* ``dense_model_struct.build``  -- /root/reference/train_dense_networks.py:223-408
  (helpers conv_layer 433-448 = relu(conv2d SAME + b), max_pool/avg_pool 2x2/2 SAME 414-426,
  fc_layer 450-457)
* ``hier_model_struct.build``   -- /root/reference/train_hier_networks.py:338-530
  (helpers 535-579, same semantics)
* ``dense_hier_model_struct.build`` -- /root/reference/train_dense_hier_networks.py:338-2382
  (helpers 2416-2455): nine three-scale dense blocks over one width ladder, four transitions,
  five finger heads and the whole-hand head; ``trace`` records every conv / fc (scope, shapes) in
  build order so tests/test_dense_hier.py can pin the restatement against the reference's AST
* ``attn_model_struct.build``   -- /root/reference/train_cnn_networks_hgru.py:436-525 (helpers
  541-570), the attention / centre-of-mass regressor, with ``tf.image.resize_images`` (439)
  restated from TF1's published bilinear kernel (third-party, TF 1.x not importable here:
  PARITY UNPINNED): BILINEAR, align_corners=False, scale = in/out (float32), source coordinate
  in = out * scale (legacy, no half-pixel offset), lower = floor(in), upper = min(ceil(in),
  size-1), lerp = in - floor(in); value = top + (bottom - top) * ylerp with top/bottom the
  x-lerps, all float32 without fused multiply-add.

Inference only (train_mode falsy: no dropout, BN from moving statistics); ``batchnorm=None`` at every call site the
reference's test paths use, so the conv_layer batch-moment branch is never taken.
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from .hgru_ref import avg_pool_same, batch_norm_inf, conv2d_same, fc, max_pool_same


def _conv(wts, x, name, stride=1):
    """conv_layer(bottom, ..., name, filter_size, stride): relu(conv2d(x, W, SAME) + b)."""
    w = wts[f"cnn/{name}/{name}_filters"].astype(x.dtype)
    b = wts[f"cnn/{name}/{name}_biases"].astype(x.dtype)
    return np.maximum(conv2d_same(x, w, stride) + b, 0)


def _fc(wts, x, name):
    return fc(x, wts[f"cnn/{name}/{name}_weights"], wts[f"cnn/{name}/{name}_biases"])


def _cat(*xs):
    return np.concatenate(xs, axis=-1)


def dense_forward(depth: np.ndarray, wts: Dict[str, np.ndarray], dtype=np.float64, keep=False):
    """train_dense_networks.py:223-408, line for line."""
    x = depth.astype(dtype)
    t = {}
    t["conv0"] = _conv(wts, x, "conv_0")                                          # 226
    t["pool0"] = max_pool_same(t["conv0"])                                        # 227
    # layer 1 (230-232)
    t["conv1_1"] = _conv(wts, t["pool0"], "conv_1_1")
    t["conv1_2"] = _conv(wts, t["conv1_1"], "conv_1_2", 2)
    t["conv1_3"] = _conv(wts, t["conv1_2"], "conv_1_3", 2)
    # layer 2 (236-245)
    t["conv2_1"] = _conv(wts, t["conv1_1"], "conv_2_1")
    t["conv2_2_1"] = _conv(wts, t["conv1_1"], "conv_2_2_1", 2)
    t["conv2_2_2"] = _conv(wts, t["conv1_2"], "conv_2_2_2")
    t["conv2_2"] = _cat(t["conv2_2_1"], t["conv2_2_2"])
    t["conv2_3_2"] = _conv(wts, t["conv1_2"], "conv_2_3_2", 2)
    t["conv2_3_3"] = _conv(wts, t["conv1_3"], "conv_2_3_3")
    t["conv2_3"] = _cat(t["conv2_3_2"], t["conv2_3_3"])
    # layers 3-6 share one pattern (250-373): per scale s, a 1x1 bottleneck then a 3x3 conv at the
    # same scale, and a 1x1 + stride-2 3x3 from the finer scale's dense input
    prev = {1: [t["conv1_1"], t["conv2_1"]], 2: [t["conv1_2"], t["conv2_2"]],
            3: [t["conv1_3"], t["conv2_3"]]}
    for L in (3, 4, 5, 6):
        in1 = _cat(*prev[1])                                   # conv{L}_1_in
        b1 = _conv(wts, in1, f"conv_{L}_1_1x1")
        o1 = _conv(wts, b1, f"conv_{L}_1")
        d21 = _conv(wts, _conv(wts, in1, f"conv_{L}_2_1x1_1"), f"conv_{L}_2_1", 2)
        in2 = _cat(*prev[2])                                   # conv{L}_2_in
        d22 = _conv(wts, _conv(wts, in2, f"conv_{L}_2_1x1_2"), f"conv_{L}_2_2")
        o2 = _cat(d21, d22)
        d32 = _conv(wts, _conv(wts, in2, f"conv_{L}_3_1x1_2"), f"conv_{L}_3_2", 2)
        in3 = _cat(*prev[3])                                   # conv{L}_3_in
        d33 = _conv(wts, _conv(wts, in3, f"conv_{L}_3_1x1_3"), f"conv_{L}_3_3")
        o3 = _cat(d32, d33)
        t[f"conv{L}_1"], t[f"conv{L}_2"], t[f"conv{L}_3"] = o1, o2, o3
        prev[1].append(o1)
        prev[2].append(o2)
        prev[3].append(o3)
    # pooling + fc (376-408)
    p1 = avg_pool_same(t["conv6_1"])
    p2 = avg_pool_same(t["conv6_2"])
    p3 = avg_pool_same(t["conv6_3"])
    r11 = np.maximum(_fc(wts, p1, "fc_1_1"), 0)
    r12 = np.maximum(_fc(wts, p2, "fc_1_2"), 0)
    r13 = np.maximum(_fc(wts, p3, "fc_1_3"), 0)
    r2 = np.maximum(_fc(wts, _cat(r11, r12, r13), "fc_2"), 0)
    r3 = np.maximum(_fc(wts, r2, "fc_3"), 0)
    out = _fc(wts, r3, "fc_4")
    if keep:
        t.update(pool1=p1, pool2=p2, pool3=p3, relu2=r2, relu3=r3)
        return out, t
    return out


FINGERS = ("p", "r", "m", "i", "t")


def hier_forward(depth: np.ndarray, wts: Dict[str, np.ndarray], dtype=np.float64):
    """train_hier_networks.py:338-530.  Returns (output, {p,r,m,i,t}_output)."""
    x = depth.astype(dtype)
    c1 = _conv(wts, x, "conv_1")                                       # 341
    p1 = max_pool_same(c1)
    c2 = _conv(wts, p1, "conv_2")                                      # 344
    p2 = max_pool_same(c2)
    trunk = {}
    for br in ("pr", "mi"):                                            # 347-352, 395-400
        a = max_pool_same(_conv(wts, p2, f"{br}_con_3"))
        trunk[br] = max_pool_same(_conv(wts, a, f"{br}_con_4"))
    a = max_pool_same(_conv(wts, p2, "t_con_3"))                       # 444-449
    t4 = max_pool_same(_conv(wts, a, "t_con_4"))
    src5 = {"p": trunk["pr"], "r": trunk["pr"], "m": trunk["mi"], "i": trunk["mi"], "t": t4}
    pool6, outs = {}, {}
    for f in FINGERS:                                                  # 354-469
        c5 = max_pool_same(_conv(wts, src5[f], f"{f}_con_5"))
        pool6[f] = max_pool_same(_conv(wts, c5, f"{f}_con_6"))
        r1 = np.maximum(_fc(wts, pool6[f], f"{f}_fc_1"), 0)
        r2 = np.maximum(_fc(wts, r1, f"{f}_fc_2"), 0)
        outs[f] = _fc(wts, r2, f"{f}_fc_3")
    hand = []
    for f in FINGERS:                                                  # 473-523
        r1 = np.maximum(_fc(wts, pool6[f], f"{f}h_fc_1"), 0)
        hand.append(np.maximum(_fc(wts, r1, f"{f}h_fc_2"), 0))
    f1 = np.maximum(_fc(wts, _cat(*hand), "final_fc_1"), 0)            # 525-528 (dropout ignored)
    out = _fc(wts, f1, "final_fc_2")                                   # 529-530
    return out, outs


def resize_bilinear_tf1(x: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """tf.image.resize_images(x, [oh, ow]) (TF1 defaults) of a float32 [n, h, w, c] batch, in
    float32 with the kernel's operation order (see module docstring)."""
    x = np.asarray(x, np.float32)
    n, h, w, c = x.shape
    f32 = np.float32
    hs, ws = f32(h) / f32(oh), f32(w) / f32(ow)

    def weights(out, scale, size):
        i = np.arange(out, dtype=np.float32) * scale
        fl = np.floor(i)
        lo = np.maximum(fl.astype(np.int64), 0)
        hi = np.minimum(np.ceil(i).astype(np.int64), size - 1)
        return lo, hi, (i - fl).astype(np.float32)

    y0, y1, ly = weights(oh, hs, h)
    x0, x1, lx = weights(ow, ws, w)
    tl, tr = x[:, y0][:, :, x0], x[:, y0][:, :, x1]
    bl, br = x[:, y1][:, :, x0], x[:, y1][:, :, x1]
    lx4 = lx[None, None, :, None]
    top = tl + (tr - tl) * lx4
    bot = bl + (br - bl) * lx4
    return (top + (bot - top) * ly[None, :, None, None]).astype(np.float32)


ATTN_BN = ["cnn/batch_normalization"] + [f"cnn/batch_normalization_{i}" for i in range(1, 6)]


def attn_forward(frames: np.ndarray, wts: Dict[str, np.ndarray], dtype=np.float64, keep=False):
    """train_cnn_networks_hgru.py:436-525 (inference).  ``frames`` [n, h, w, 1] float32 normalised
    depth (images / image_max_depth, 116).  Returns [n, output_shape] (u, v, d) / image size."""
    r = resize_bilinear_tf1(frames, 128, 128)                         # 439 (float32, as TF)
    x = r.astype(dtype)
    t = {"resized": r}
    for i, name in enumerate(("aconv_1", "aconv_2", "aconv_3", "aconv_4", "aconv_5")):  # 440-476
        x = batch_norm_inf(max_pool_same(_conv(wts, x, name)), wts, ATTN_BN[i])
        t[name] = x
    h = np.maximum(_fc(wts, x, "afc_1"), 0)                           # 478-479
    h = batch_norm_inf(h, wts, ATTN_BN[5])                            # 482-490 (per feature)
    out = _fc(wts, h, "afc_out")                                      # 502-503
    if keep:
        t["relu1"] = h
        return out, t
    return out


def cnn_forward(depth: np.ndarray, wts: Dict[str, np.ndarray], dtype=np.float64, keep=False):
    """cnn_model_struct.build (train_cnn_networks_hgru.py:639-673), inference: conv_1 .. conv_5
    (conv_layer = relu(conv2d SAME + b), 695-710; conv_5 is 5x5), each followed by a 2x2 max pool
    SAME (690-693); fc_1 on the NHWC flatten of pool_5 (663, 712-719) + relu, fc_2 + relu, fc_3 +
    relu, fc_4 = out_put (dropout only under train_mode == True)."""
    x = depth.astype(dtype)
    t = {}
    for i, name in enumerate(("conv_1", "conv_2", "conv_3", "conv_4", "conv_5"), 1):   # 641-656
        x = max_pool_same(_conv(wts, x, name))
        t[f"pool{i}"] = x
    for name in ("fc_1", "fc_2", "fc_3"):                                            # 658-671
        x = np.maximum(_fc(wts, x, name), 0)
        t[name] = x
    out = _fc(wts, x, "fc_4")                                                         # 672-673
    if keep:
        return out, t
    return out


# dense_hier_model_struct (train_dense_hier_networks.py:338-2382)
DH_LADDER = (12, 16, 24, 32, 48, 64, 96, 128, 164, 198, 230)


def dense_hier_forward(depth: np.ndarray, wts: Dict[str, np.ndarray], dtype=np.float64, trace=None):
    """Returns (output, {p,r,m,i,t}_output).  Head sizes come from the fc_4 / final_fc_2 weights."""
    L = DH_LADDER

    def conv(x, name, stride=1):
        w = wts[f"cnn/{name}/{name}_filters"]
        if trace is not None:
            trace.append(("conv", name, int(w.shape[0]), stride, x.shape[-1], int(w.shape[3])))
        assert w.shape[2] == x.shape[-1], name
        return _conv(wts, x, name, stride)

    def fcr(x, name, relu=True):
        w = wts[f"cnn/{name}/{name}_weights"]
        if trace is not None:
            trace.append(("fc", name, int(np.prod(x.shape[1:])), int(w.shape[1])))
        y = _fc(wts, x, name)
        return np.maximum(y, 0) if relu else y

    def block(b, s, nl, ins, chain):
        p = f"dense_{b}_conv"
        if chain:                                                       # 348-352
            x1 = conv(ins[0], f"{p}_1_scale_1")
            x2 = conv(x1, f"{p}_1_scale_2", 2)
            x3 = conv(x2, f"{p}_1_scale_3", 2)
        else:                                                           # e.g. 455-459
            x1, x2, x3 = (conv(ins[k], f"{p}_1_scale_{k + 1}") for k in range(3))
        h1, h2, h3 = [x1], [x2], [x3]
        h1.append(conv(x1, f"{p}_2_scale_1"))                           # 356-364
        h2.append(_cat(conv(x1, f"{p}_2_scale_2_1", 2), conv(x2, f"{p}_2_scale_2_2")))
        h3.append(_cat(conv(x2, f"{p}_2_scale_3_2", 2), conv(x3, f"{p}_2_scale_3_3")))
        for l in range(3, nl + 1):                                      # 367-437
            n = f"{p}_{l}_scale"
            i1, i2, i3 = _cat(*h1), _cat(*h2), _cat(*h3)
            o1 = conv(conv(i1, f"{n}_1_1x1"), f"{n}_1")
            o21 = conv(conv(i1, f"{n}_2_1x1_1"), f"{n}_2_1", 2)
            o22 = conv(conv(i2, f"{n}_2_1x1_2"), f"{n}_2_2")
            o32 = conv(conv(i2, f"{n}_3_1x1_2"), f"{n}_3_2", 2)
            o33 = conv(conv(i3, f"{n}_3_1x1_3"), f"{n}_3_3")
            h1.append(o1)
            h2.append(_cat(o21, o22))
            h3.append(_cat(o32, o33))
        return h1[-1], h2[-1], h3[-1]

    def transition(k, outs):                                            # 440-449
        return [max_pool_same(conv(x, f"tran_{k}_conv_{j + 1}")) for j, x in enumerate(outs)]

    def finger(f, outs):                                                # 824-857
        pools = [max_pool_same(x) for x in outs]
        r1 = [fcr(pl, f"fc_1_{f}_{j + 1}") for j, pl in enumerate(pools)]
        r3 = fcr(fcr(_cat(*r1), f"fc_2_{f}"), f"fc_3_{f}")
        return pools, fcr(r3, f"fc_4_{f}", relu=False)

    x = depth.astype(dtype)
    pool1 = max_pool_same(conv(x, "conv_1"))                            # 341-343
    t1 = transition(1, block(1, 0, 4, [pool1], True))
    t2 = transition(2, block(2, 1, 4, t1, False))
    pools, outs = {}, {}
    pools["p"], outs["p"] = finger("p", block(3, 2, 6, t2, False))
    pools["r"], outs["r"] = finger("r", block(4, 2, 6, t2, False))
    t3 = transition(3, block(5, 1, 4, t1, False))
    pools["m"], outs["m"] = finger("m", block(6, 2, 6, t3, False))
    pools["i"], outs["i"] = finger("i", block(7, 2, 6, t3, False))
    t4 = transition(4, block(8, 1, 4, t1, False))
    pools["t"], outs["t"] = finger("t", block(9, 2, 6, t4, False))
    hand = []
    for f in FINGERS:                                                   # 2245-2373
        r1 = [fcr(pl, f"fc_1_{f}h_{j + 1}") for j, pl in enumerate(pools[f])]
        hand.append(fcr(_cat(*r1), f"fc_2_{f}h"))
    out = fcr(fcr(_cat(*hand), "final_fc_1"), "final_fc_2", relu=False)    # 2376-2382
    return out, outs
