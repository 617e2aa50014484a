"""Writes the hGRU pose output (synthetic weights / crops, fixed seeds) of the library MP_LIB_PATH
points at (default: in-tree) to a .npy file -- for bit-identity checks between A/B library builds.
usage: python tools/lib_out.py out.npy [batch] [dtype]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")
path = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dtype = sys.argv[3] if len(sys.argv) > 3 else "f32_fft"
W = mp.weights
dev = torch.device("cuda:0")
ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
    ctx.set_weight(v.name, W.synth_value(v, 1234, 8))
ctx.finalize(mp._lib.dtype_code(dtype))
depth = torch.from_numpy(W.synth_crops(B, seed=42, size=128)).to(dev)
o0 = torch.from_numpy(W.synth_hidden((B, 64, 64, 64), seed=7)).to(dev)
out = torch.empty((B, 69), device=dev)
ctx.pose_fwd(depth, o0, out, mp._lib.current_stream(dev))
torch.cuda.synchronize()
np.save(path, out.cpu().numpy())
