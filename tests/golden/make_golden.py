"""Regenerates the committed golden fixtures from the float64 oracle (run in the build container).

The reference ships no fixtures and cannot be executed here (Python 2 + TensorFlow 1.x, missing
``utils.py_utils`` / ``ops.initialization``: SURVEY.md 8c), so these vectors come from the oracle
(``oracle/hgru_ref.py``).  They pin the oracle against regressions and give the GPU tests a
fixed target.  Inputs are regenerated from seeds by ``monkey-pose_amd/weights.py`` (the weight
tensors are up to 1 GB and are not stored); the files hold only seeds, shapes and outputs.

    python tests/golden/make_golden.py
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import hgru_ref as R  # noqa: E402

W = importlib.import_module("monkey-pose_amd").weights
HERE = os.path.dirname(os.path.abspath(__file__))

# (name, n, h, w, ssf, timesteps, weight seed, x seed, o0 seed)
CIRCUIT_CASES = [
    ("circuit_s5_t3", 2, 16, 32, 5, 3, 11, 21, 31),
    ("circuit_s15_t2", 1, 32, 32, 15, 2, 12, 22, 32),
]
# (name, n, crop, timesteps, weight seed, crop seed, o0 seed)
POSE_CASES = [
    ("pose_c64_t8", 2, 64, 8, 1234, 42, 7),
    ("pose_c128_t8", 2, 128, 8, 1234, 42, 7),
]


def circuit_inputs(n, h, w, ssf, T, ws, xs, os_):
    wts = W.synth_weights(W.hgru_circuit_vars(k=64, ssf=ssf, timesteps=T), seed=ws, timesteps=T)
    # exercise the adaptation gain: rho != 1
    wts["cnn/contextual_circuit/rho"] = (1.0 + W.sym_uniform(ws, "rho_pert", (T,), 0.1)).astype(np.float32)
    X = W.sym_uniform(xs, "X", (n, h, w, 64), 1.0)
    O0 = W.sym_uniform(os_, "O0", (n, h, w, 64), 0.5)
    return wts, X, O0


def pose_inputs(n, crop, T, ws, cs, os_):
    wts = W.synth_weights(W.hgru_pose_vars(output_shape=69, timesteps=T, crop=crop), seed=ws, timesteps=T)
    depth = W.synth_crops(n, seed=cs, size=crop)
    O0 = W.synth_hidden((n, crop // 2, crop // 2, 64), seed=os_)
    return wts, depth, O0


# (name, kind, n, crop, weight seed, crop seed)
REGRESSOR_CASES = [
    ("dense_c128", "dense", 2, 128, 77, 43),
    ("hier_c128", "hier", 2, 128, 78, 44),
    ("dense_hier_c128", "dense_hier", 2, 128, 80, 45),
    ("cnn_c128", "cnn", 2, 128, 81, 46),   # cnn_model_struct (train_cnn_networks_hgru.py:639-673)
]
HIER_HEADS = (108, 39, 39, 39, 39, 36)     # train_hier_networks.py:263 with 36 joints


def regressor_inputs(kind, n, crop, ws, cs):
    if kind == "dense_hier":
        table = importlib.import_module("monkey-pose_amd").train_dense_hier_networks.dense_hier_vars(HIER_HEADS, crop)
    elif kind == "cnn":
        table = W.cnn_vars(output_shape=69, crop=crop)
    else:
        table = (W.dense_vars(output_shape=69, crop=crop) if kind == "dense"
                 else W.hier_vars(output_shape=HIER_HEADS[0], part_shapes=HIER_HEADS[1:], crop=crop))
    return W.synth_weights(table, seed=ws), W.synth_crops(n, seed=cs, size=crop)


# (name, n, frame h, frame w, weight seed, frame seed): attention CoM regressor
# (train_cnn_networks_hgru.py:436-525) on full frames + prepare_data_test (61-74) on its output
ATTN_CASES = [
    ("attn_f424", 2, 424, 512, 79, 11),
]


def attn_inputs(n, h, w, ws, fs):
    return W.attn_synth_weights(seed=ws), W.synth_frames(n, seed=fs, h=h, w=w)


def checksums(a):
    a = np.asarray(a, np.float64)
    return [float(a.sum()), float((a * a).sum()), float(np.abs(a).max())]


def main(which=None):
    meta = {}
    for (name, n, h, w, ssf, T, ws, xs, os_) in CIRCUIT_CASES:
        if which and name not in which:
            continue
        wts, X, O0 = circuit_inputs(n, h, w, ssf, T, ws, xs, os_)
        O, steps = R.hgru_forward(X.astype(np.float64), O0, wts, T, keep_steps=True)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), O=O.astype(np.float32))
        meta[name] = dict(kind="circuit", n=n, h=h, w=w, ssf=ssf, timesteps=T, weight_seed=ws,
                          x_seed=xs, o0_seed=os_, step_checksums=[checksums(s) for s in steps])
        print(name, checksums(O))
    for (name, n, crop, T, ws, cs, os_) in POSE_CASES:
        if which and name not in which:
            continue
        wts, depth, O0 = pose_inputs(n, crop, T, ws, cs, os_)
        out, inter = R.hgru_pose_forward(depth, wts, O0, T, np.float64, keep=True)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), out=out.astype(np.float64))
        meta[name] = dict(kind="pose", n=n, crop=crop, timesteps=T, weight_seed=ws, crop_seed=cs,
                          o0_seed=os_, output_shape=69,
                          step_checksums=[checksums(s) for s in inter["hgru_steps"]],
                          hgru_bn_checksum=checksums(inter["hgru_bn"]),
                          fc1_checksum=checksums(inter["fc1"]))
        print(name, out[:, :6])
    from oracle import regressors_ref as RR
    for (name, kind, n, crop, ws, cs) in REGRESSOR_CASES:
        if which and name not in which:
            continue
        wts, depth = regressor_inputs(kind, n, crop, ws, cs)
        if kind in ("dense", "cnn"):
            out = (RR.dense_forward if kind == "dense" else RR.cnn_forward)(depth, wts)
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), out=out)
        else:
            out, parts = (RR.hier_forward if kind == "hier" else RR.dense_hier_forward)(depth, wts)
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), out=out,
                                **{f"{k}_out": v for k, v in parts.items()})
        meta[name] = dict(kind=kind, n=n, crop=crop, weight_seed=ws, crop_seed=cs)
        print(name, out[:, :4])
    from oracle import crop_ref as CR
    for (name, n, h, w, ws, fs) in ATTN_CASES:
        if which and name not in which:
            continue
        wts, frames = attn_inputs(n, h, w, ws, fs)
        out = RR.attn_forward(frames, wts)
        patches, Ms, coms = CR.prepare_data_test(frames, out.astype(np.float32), CR.MonkeyDetectorRef())
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), out=out, patches=patches, Ms=Ms, coms=coms)
        meta[name] = dict(kind="attn", n=n, h=h, w=w, weight_seed=ws, frame_seed=fs)
        print(name, out, coms)
    path = os.path.join(HERE, "golden.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    old.update(meta)
    json.dump(old, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
