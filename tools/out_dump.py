"""Writes the pose forward's output at batch B (synthetic weights / crops, as tools/time_fwd.py) to a
.npy, so that two processes with different MP_* switches can be compared bit for bit.
usage: [MP_X=..] python tools/out_dump.py <out.npy> [--batch B] [--dtype f32_fft]"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")
W = mp.weights
ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--dtype", default="f32_fft")
a = ap.parse_args()
dev = torch.device("cuda:0")
ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
    ctx.set_weight(v.name, W.synth_value(v, 1234, 8))
ctx.finalize(mp._lib.dtype_code(a.dtype))
depth = torch.from_numpy(W.synth_crops(a.batch, seed=42, size=128)).to(dev)
h0 = torch.from_numpy(W.synth_hidden((a.batch, 64, 64, 64), seed=7)).to(dev)
out = torch.empty((a.batch, 69), device=dev)
ctx.pose_fwd(depth, h0, out, mp._lib.current_stream(dev))
torch.cuda.synchronize()
np.save(a.out, out.cpu().numpy())
