"""Times the hGRU pose forward at batch B (no profiling) -- for A/B runs of build options / env
(e.g. MP_STREAMS=1 vs 2).  Synthetic weights and crops."""
import argparse
import importlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")
p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=256)
p.add_argument("--steps", type=int, default=20)
p.add_argument("--dtype", default="f32_fft")
p.add_argument("--profile", action="store_true", help="also a single-stream HIP-event pass: ms per kernel class")
a = p.parse_args()
W = mp.weights
dev = torch.device("cuda:0")
ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
    ctx.set_weight(v.name, W.synth_value(v, 1234, 8))
ctx.finalize(mp._lib.dtype_code(a.dtype))
B = a.batch
depth = torch.from_numpy(W.synth_crops(B, seed=42, size=128)).to(dev)
o0 = torch.from_numpy(W.synth_hidden((B, 64, 64, 64), seed=7)).to(dev)
out = torch.empty((B, 69), device=dev)
st = mp._lib.current_stream(dev)
for _ in range(3):
    ctx.pose_fwd(depth, o0, out, st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    ctx.pose_fwd(depth, o0, out, st)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.steps
print(f"MP_STREAMS={os.environ.get('MP_STREAMS', 'default')} dtype={a.dtype} B={B}: {dt * 1e3:.3f} ms/step, "
      f"{B / dt:.1f} crops/s, out[0,:3]={out[0, :3].tolist()}")
if a.profile:
    ctx.profile(True)
    for _ in range(5):
        ctx.pose_fwd(depth, o0, out, st)
    torch.cuda.synchronize()
    ctx.profile(False)
    names = ["backbone", "fc1", "fft_fwd", "spec_gemm", "inv_a_fwd", "fft_inv", "epi_b"]
    res = {}
    for n in names:
        ms, cnt = ctx.profile_read(n)
        res[n] = round(ms / max(1, cnt), 4)
    print("profile ms/launch:", res)
