"""The A/B switches read once at library load or plan time (MP_BF16_MAPS, MP_FC_PRESPLIT,
MP_GRAPH_FUSE_POOL, MP_IGEMM_PM_SPLITS, MP_IGEMM_XCD, MP_IGEMM_HALO, MP_IGEMM_HALO_NARROW,
MP_IGEMM_HALO_TALL, MP_IGEMM_PW, MP_IGEMM_SMALL_SPLITK) keep their paths correct: each case runs in
one child process with the switch set (the parent's library already made its choice), against the
committed golden vectors."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import json, sys
sys.path.insert(0, {tests!r})
import torch
from helpers import MG, golden_array, golden_meta, pkg, rel_inf
kind, dtype = {kind!r}, {dtype!r}
meta = golden_meta()
P = pkg()
if kind == "pose":
    m = meta["pose_c64_t8"]
    wts, depth, O0 = MG.pose_inputs(m["n"], m["crop"], m["timesteps"], m["weight_seed"], m["crop_seed"], m["o0_seed"])
    model = P.hgru_pose.model()
    model.compute_dtype = dtype
    model.load_weights(wts)
    out = model.build(torch.from_numpy(depth).cuda(), m["output_shape"], train_mode=False,
                      h2_init=torch.from_numpy(O0).cuda()).cpu().numpy()
    ref = golden_array("pose_c64_t8", "out")
elif kind == "dense":
    m = meta["dense_c128"]
    wts, depth = MG.regressor_inputs(m["kind"], m["n"], m["crop"], m["weight_seed"], m["crop_seed"])
    model = P.train_dense_networks.dense_model_struct()
    model.compute_dtype = dtype
    model.load_weights(wts)
    out = model.build(torch.from_numpy(depth).cuda(), 69, train_mode=False).cpu().numpy()
    ref = golden_array("dense_c128", "out")
elif kind == "dense_hier":
    m = meta["dense_hier_c128"]
    wts, depth = MG.regressor_inputs("dense_hier", m["n"], m["crop"], m["weight_seed"], m["crop_seed"])
    model = P.train_dense_hier_networks.dense_hier_model_struct()
    model.compute_dtype = dtype
    model.load_weights(wts)
    out = model.build(torch.from_numpy(depth).cuda(), *MG.HIER_HEADS, train_mode=False).cpu().numpy()
    ref = golden_array("dense_hier_c128", "out")
else:
    m = meta["hier_c128"]
    wts, depth = MG.regressor_inputs(m["kind"], m["n"], m["crop"], m["weight_seed"], m["crop_seed"])
    model = P.train_hier_networks.hier_model_struct()
    model.compute_dtype = dtype
    model.load_weights(wts)
    out = model.build(torch.from_numpy(depth).cuda(), *MG.HIER_HEADS, train_mode=False).cpu().numpy()
    ref = golden_array("hier_c128", "out")
print(json.dumps({{"err": float(rel_inf(out, ref))}}))
"""

CASES = [
    # (env, model, dtype, gate)
    ({"MP_BF16_MAPS": "0"}, "pose", "bf16", 5e-3),
    ({"MP_FC_PRESPLIT": "0"}, "pose", "fp32_fft", 1e-4),
    ({"MP_CONV_SMALL": "0"}, "pose", "fp32_fft", 1e-4),
    ({"MP_FC_PRESPLIT": "0"}, "pose", "bf16", 5e-3),
    ({"MP_IGEMM_PM_SPLITS": "1"}, "hier", "fp32_split", 1e-4),
    ({"MP_IGEMM_PM_SPLITS": "1"}, "hier", "bf16", 5e-3),
    ({"MP_IGEMM_XCD": "0", "MP_IGEMM_HALO": "0"}, "hier", "fp32_split", 1e-4),
    ({"MP_GRAPH_FUSE_POOL": "0"}, "hier", "bf16", 5e-3),
    ({"MP_IGEMM_HALO_TALL": "0"}, "hier", "fp32_split", 1e-4),
    ({"MP_IGEMM_SMALL_SPLITK": "0"}, "dense_hier", "fp32_split", 1e-4),
    # the six-launch FFT loop and the one-block-per-CU row kernel (A/B forms of the four-step loop)
    ({"MP_FFT4": "0"}, "pose", "fp32_fft", 1e-4),
    ({"MP_FFT4": "0"}, "pose", "bf16", 5e-3),
    ({"MP_IGEMM_PW": "0", "MP_IGEMM_HALO_NARROW": "0"}, "dense", "fp32_split", 1e-4),
    ({"MP_IGEMM_PW": "0", "MP_IGEMM_HALO_NARROW": "0"}, "dense", "bf16", 5e-3),
    ({"MP_GRAPH_FUSE_1X1": "0"}, "dense", "fp32_split", 1e-4),
    ({"MP_GRAPH_FUSE_1X1": "0"}, "dense_hier", "fp32_split", 1e-4),
]


@pytest.mark.gpu
@pytest.mark.parametrize("env,kind,dtype,gate", CASES,
                         ids=[f"{'+'.join(f'{k}={v}' for k, v in e.items())}-{k}-{d}" for e, k, d, _ in CASES])
def test_switch_keeps_parity(env, kind, dtype, gate):
    code = _CHILD.format(tests=os.path.join(ROOT, "tests"), kind=kind, dtype=dtype)
    r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **env}, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    err = json.loads(r.stdout.strip().splitlines()[-1])["err"]
    print(f"{env} {kind} {dtype}: rel_inf {err:.3e}")
    assert err <= gate, err


_CHILD_BITS = r"""
import hashlib, json, sys
sys.path.insert(0, {tests!r})
import numpy as np, torch
from helpers import MG, pkg
P = pkg()
kind, dtype = {kind!r}, {dtype!r}
if kind == "dense":
    wts, depth = MG.regressor_inputs("dense", 12, 128, 5, 6)
    model = P.train_dense_networks.dense_model_struct()
    model.compute_dtype = dtype
    model.load_weights(wts)
    out = model.build(torch.from_numpy(depth).cuda(), 69, train_mode=False).cpu().numpy()
else:   # 12 crops: above the small-batch FFT kernels' B <= 8; pose80: three 32-image GEMM groups,
        # two hGRU slices (64 + 16 crops)
    wts, depth, O0 = MG.pose_inputs(12 if kind == "pose12" else 80, 64, 8, 5, 6, 7)
    model = P.hgru_pose.model()
    model.compute_dtype = dtype
    model.load_weights(wts)
    if kind == "pose80id":   # O0 = X of this call, after a forward on other crops in the same context
        model.build(torch.from_numpy(np.ascontiguousarray(depth[::-1])).cuda(), 69, train_mode=False,
                    h2_init=torch.from_numpy(O0).cuda())
        model.aux["hidden_init"] = "identity"
        out = model.build(torch.from_numpy(depth).cuda(), 69, train_mode=False).cpu().numpy()
    else:
        out = model.build(torch.from_numpy(depth).cuda(), 69, train_mode=False,
                          h2_init=torch.from_numpy(O0).cuda()).cpu().numpy()
print(json.dumps({{"sha": hashlib.sha256(np.ascontiguousarray(out).tobytes()).hexdigest()}}))
"""

BITS_CASES = [
    # igemm_x3pwn_kernel (one block over all 2 / 3 / 5 / 6 cout blocks of a 1x1 conv) runs each
    # output's MFMA sequence of igemm_x3pw_kernel: MP_IGEMM_PWN = 0 / 1 / 2 give the same bytes
    ("dense", "fp32_split", "MP_IGEMM_PWN", ("0", "1", "2", "3"), {}),
    ("dense", "bf16", "MP_IGEMM_PWN", ("0", "1", "2", "3"), {}),
    # four-step loop: non-temporal or default cache policy for the partials moves no value
    ("pose80", "fp32_fft", "MP_COL8_ZNT", ("0", "1"), {}),
    ("pose80", "bf16", "MP_COL8_ZNT", ("0", "1"), {}),
    ("pose80", "fp32_fft", "MP_ROW8_ZNT", ("0", "1"), {}),
    # col8p_kernel's partials stored non-temporal or not (MP_COL8_ZNT under MP_COL8P = 1); the row
    # kernels' fp32 maps non-temporal or not (MP_MAP_NT, default on from 128 images), row8_kernel and
    # row A on channel quarters
    ("pose80", "fp32_fft", "MP_COL8_ZNT", ("0", "1"), {"MP_COL8P": "1"}),
    ("pose80", "fp32_fft", "MP_MAP_NT", ("0", "1"), {}),
    ("pose80", "bf16", "MP_MAP_NT", ("0", "1"), {}),
    ("pose80", "fp32_fft", "MP_MAP_NT", ("0", "1"), {"MP_ROWQ_MAXB": "80"}),
    # the backbone per batch slice (two slices at 80 crops), staggered or not, or whole-batch first
    ("pose80", "fp32_fft", "MP_BB_PIPE", ("0", "1"), {}),
    ("pose80", "fp32_fft", "MP_BB_STAGGER", ("0", "1"), {}),
    ("pose80", "bf16", "MP_BB_PIPE", ("0", "1"), {}),
    # hidden_init = identity (O0 = X) keeps the whole-batch backbone first under either setting
    ("pose80id", "fp32_fft", "MP_BB_PIPE", ("0", "1"), {}),
    # the persistent column kernel (col8p_kernel, slices of >= MP_COL8P images) or col8_kernel: the
    # same item arithmetic (64 + 16: col8p on the first slice only at 64; on both at 1)
    ("pose80", "fp32_fft", "MP_COL8P", ("0", "64", "1"), {}),
    ("pose80", "bf16", "MP_COL8P", ("0", "64", "1"), {}),
    ("pose12", "fp32_fft", "MP_COL8P", ("0", "1"), {}),
    # step 0 reading O0 (NHWC) directly, or row(INIT) copying it into the C8 state map first
    ("pose80", "fp32_fft", "MP_O0_DIRECT", ("0", "1"), {}),
    ("pose12", "fp32_fft", "MP_O0_DIRECT", ("0", "1"), {}),
    # the pose head per batch slice on the slice's stream, or once after the join (64 + 16 crops)
    ("pose80", "fp32_fft", "MP_FC_SLICE", ("0", "1"), {}),
    ("pose80", "bf16", "MP_FC_SLICE", ("0", "1"), {}),
    # col8q_kernel (software-pipelined) or col8p_kernel: one item's arithmetic either way
    ("pose80", "fp32_fft", "MP_COL8Q", ("0", "1"), {"MP_COL8P": "1"}),
    ("pose12", "fp32_fft", "MP_COL8Q", ("0", "1"), {"MP_COL8P": "1"}),
    # row A on channel quarters (rowq_a_kernel) or as row8_kernel<ROW_A>: one batch slice of 12, and
    # two slices (64 + 16) all on rowq; and the cache policy of a cache-resident batch (12 crops)
    ("pose12", "fp32_fft", "MP_ROWQ_MAXB", ("0", "16"), {}),
    ("pose80", "fp32_fft", "MP_ROWQ_MAXB", ("0", "80"), {}),
    ("pose12", "fp32_fft", "MP_ROW8_ZNT", ("0", "1"), {}),
]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,dtype,var,values,base", BITS_CASES, ids=[f"{c[2]}-{c[0]}-{c[1]}" + "".join(f"-{k}{v}" for k, v in c[4].items()) for c in BITS_CASES])
def test_switch_is_bit_identical(kind, dtype, var, values, base):
    """Switches whose forms compute every output with the same operations in the same order: the
    model output is the same bytes under each setting (one child process per setting)."""
    shas = []
    for v in values:
        code = _CHILD_BITS.format(tests=os.path.join(ROOT, "tests"), kind=kind, dtype=dtype)
        r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **base, var: v},
                           capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr[-2000:]
        shas.append(json.loads(r.stdout.strip().splitlines()[-1])["sha"])
    assert len(set(shas)) == 1, shas
