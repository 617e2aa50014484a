"""Times fc_1 (fc_gemm_x3 + fc_reduce) of the pose head alone at batch B through the context's
HIP-event profile (one-stream forward), for A/B of k_fc.hip changes.  Synthetic weights."""
import argparse
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")
p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, nargs="+", default=[256, 32, 1])
p.add_argument("--dtype", default="f32_fft")
a = p.parse_args()
W = mp.weights
dev = torch.device("cuda:0")
ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
    ctx.set_weight(v.name, W.synth_value(v, 1234, 8))
ctx.finalize(mp._lib.dtype_code(a.dtype))
st = mp._lib.current_stream(dev)
for B in a.batch:
    depth = torch.from_numpy(W.synth_crops(B, seed=42, size=128)).to(dev)
    o0 = torch.from_numpy(W.synth_hidden((B, 64, 64, 64), seed=7)).to(dev)
    out = torch.empty((B, 69), device=dev)
    ctx.pose_fwd(depth, o0, out, st)
    ctx.profile(True)
    for _ in range(5):
        ctx.pose_fwd(depth, o0, out, st)
    torch.cuda.synchronize()
    ctx.profile(False)
    ms, n = ctx.profile_read("fc1")
    for k in ("backbone", "conv15_a", "conv15_b", "fc_out", "fft_fwd", "spec_gemm", "inv_a_fwd", "fft_inv", "epi_b"):
        ctx.profile_read(k)
    print(f"KSLICE={os.environ.get('MP_FC_KSLICE', 'default')} dtype={a.dtype} B={B}: fc1 {ms / n:.4f} ms/launch "
          f"out[0,:2]={out[0, :2].tolist()}")
