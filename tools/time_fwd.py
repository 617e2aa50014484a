"""B = 256 pose-forward timing for same-box A/B (default streams, synthetic inputs): the median of
--reps timings of --steps forwards each.  usage: [MP_X=..] python tools/time_fwd.py [--dtype f32_fft]"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mp = importlib.import_module("monkey-pose_amd")
W = mp.weights
p = argparse.ArgumentParser()
p.add_argument("--dtype", default="f32_fft")
p.add_argument("--batch", type=int, default=256)
p.add_argument("--steps", type=int, default=20)
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
dev = torch.device("cuda:0")
T = 8
ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
for v in W.hgru_pose_vars(output_shape=69, timesteps=T, crop=128):
    ctx.set_weight(v.name, W.synth_value(v, 1234, T))
ctx.finalize(mp._lib.dtype_code(a.dtype))
st = mp._lib.current_stream(dev)
B = a.batch
depth = torch.from_numpy(W.synth_crops(B, seed=42, size=128)).to(dev)
h0 = torch.from_numpy(W.synth_hidden((B, 64, 64, 64), seed=7)).to(dev)
out = torch.empty((B, 69), device=dev)
for _ in range(3):
    ctx.pose_fwd(depth, h0, out, st)
torch.cuda.synchronize()
ts = []
for _ in range(a.reps):
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.pose_fwd(depth, h0, out, st)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) / a.steps * 1e3)
ts.sort()
env = {k: v for k, v in os.environ.items() if k.startswith("MP_")}
print(json.dumps({"env": env, "dtype": a.dtype, "batch": B, "ms_median": round(ts[len(ts) // 2], 4),
                  "ms_min": round(ts[0], 4), "ms_all": [round(t, 4) for t in ts]}), flush=True)
