"""Four-step loop (k_fft4.hip) vs the six-launch loop (MP_FFT4=0, a child process) and the float64
oracle, then timing: B = 256 forward (default streams) and a one-stream per-kernel HIP-event pass.
usage: python tools/fft4_check.py [--batch 256] [--steps 20] [--child OUT.npy]"""
import argparse
import importlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mp = importlib.import_module("monkey-pose_amd")
W = mp.weights
p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=256)
p.add_argument("--steps", type=int, default=20)
p.add_argument("--child", default=None)
p.add_argument("--dtype", default="f32_fft")
p.add_argument("--quick", action="store_true", help="skip the six-launch comparison and the B = 256 timing")
a = p.parse_args()
dev = torch.device("cuda:0")
T = 8
wts = {v.name: W.synth_value(v, 1234, T) for v in W.hgru_pose_vars(output_shape=69, timesteps=T, crop=128)}
ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
for k, v in wts.items():
    ctx.set_weight(k, v)
ctx.finalize(mp._lib.dtype_code(a.dtype))
st = mp._lib.current_stream(dev)
NB = 37   # odd: a partial 32-image group and partial slices
d = W.synth_crops(NB, seed=42, size=128)
o0 = W.synth_hidden((NB, 64, 64, 64), seed=7)
out = torch.empty((NB, 69), device=dev)
ctx.pose_fwd(torch.from_numpy(d).to(dev), torch.from_numpy(o0).to(dev), out, st)
torch.cuda.synchronize()
got = out.cpu().numpy()
if a.child:
    np.save(a.child, got)
    sys.exit(0)
res = {"fft4": os.environ.get("MP_FFT4", "1"), "dtype": a.dtype, "fft_loop": ctx.info("fft_loop")}
one = torch.empty((1, 69), device=dev)
ctx.pose_fwd(torch.from_numpy(d[5:6]).to(dev), torch.from_numpy(o0[5:6]).to(dev), one, st)
torch.cuda.synchronize()
res["batch1_bit_identical"] = bool(np.array_equal(one.cpu().numpy()[0], got[5]))
ctx.pose_fwd(torch.from_numpy(d).to(dev), torch.from_numpy(o0).to(dev), out, st)
torch.cuda.synchronize()
res["deterministic"] = bool(np.array_equal(out.cpu().numpy(), got))
sys.path.insert(0, ROOT)
from oracle import hgru_ref as R  # noqa: E402  (test infrastructure: the checker only)
r64 = R.hgru_pose_forward(d[:2], wts, o0[:2], T, np.float64)
res["rel_err_fp64_oracle"] = float(np.abs(got[:2] - r64).max() / np.abs(r64).max())
env = dict(os.environ, MP_FFT4="0")
if a.quick:
    print(json.dumps(res), flush=True)
tmp = "/tmp/fft4_old.npy"
r = None if a.quick else subprocess.run([sys.executable, os.path.abspath(__file__), "--child", tmp, "--dtype", a.dtype], env=env, capture_output=True,
                   text=True, timeout=300)
if r is None:
    pass
elif r.returncode == 0:
    old = np.load(tmp)
    res["rel_err_vs_six_launch"] = float(np.abs(got - old).max() / np.abs(old).max())
    res["old_rel_err_fp64_oracle"] = float(np.abs(old[:2] - r64).max() / np.abs(r64).max())
else:
    res["old_error"] = r.stderr[-2000:]
if not a.quick:
    print(json.dumps(res), flush=True)

B = a.batch
depth = torch.from_numpy(W.synth_crops(B, seed=42, size=128)).to(dev)
h0 = torch.from_numpy(W.synth_hidden((B, 64, 64, 64), seed=7)).to(dev)
if not a.quick:
    ob = torch.empty((B, 69), device=dev)
    for _ in range(3):
        ctx.pose_fwd(depth, h0, ob, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.pose_fwd(depth, h0, ob, st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"batch": B, "ms_per_step": round(dt * 1e3, 3), "crops_per_s": round(B / dt, 1)}), flush=True)
    ctx.profile(True)
    for _ in range(3):
        ctx.pose_fwd(depth, h0, ob, st)
    torch.cuda.synchronize()
    ctx.profile(False)
    prof = {}
    for name in ("row_init", "col_gemm", "row_a", "row_b", "row_final", "fft_fwd", "spec_gemm", "inv_a_fwd", "fft_inv",
                 "epi_b", "conv15_a", "conv15_b", "fc1", "backbone"):
        ms, n = ctx.profile_read(name)
        if n:
            prof[name] = {"avg_ms": round(ms / n, 4), "per_fwd_ms": round(ms / 3, 3), "launches_per_fwd": n / 3}
    print(json.dumps(prof), flush=True)
small = {}
for bs in (1, 8, 32, 64, 128):
    d1 = depth[:bs].contiguous()
    h1 = h0[:bs].contiguous()
    o1 = torch.empty((bs, 69), device=dev)
    for _ in range(3):
        ctx.pose_fwd(d1, h1, o1, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 20
    for _ in range(n):
        ctx.pose_fwd(d1, h1, o1, st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    small[bs] = {"ms": round(dt * 1e3, 3), "crops_per_s": round(bs / dt, 1)}
print(json.dumps({"small_batch": small}), flush=True)
