"""Runs the frame chain (attention -> device crop -> hGRU pose) at batch B a few times, for
rocprofv3 kernel traces of the N1 row (synthetic frames / weights, no oracle)."""
import argparse
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=256)
p.add_argument("--iters", type=int, default=5)
p.add_argument("--dtype", default="f32_fft")
a = p.parse_args()
W, T = mp.weights, mp.train_cnn_networks_hgru
dev = torch.device("cuda:0")
frames = torch.from_numpy(W.synth_frames(a.batch, seed=12)).to(dev)
attn = T.attn_model_struct()
attn.load_weights(W.attn_synth_weights(seed=21))
pose = mp.hgru_pose.model()
pose.compute_dtype = a.dtype
md = mp.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
pipe = T.FramePosePipeline(attn, pose, md, check_crops=False)
o0 = torch.from_numpy(W.synth_hidden((a.batch, 64, 64, 64), seed=7)).to(dev)
for _ in range(a.iters):
    out, coms, Ms = pipe.run(frames, h2_init=o0)
torch.cuda.synchronize()
print("ok", tuple(out.shape), float(out.abs().max()))
