"""Same-box A/B of MP_* environment settings on the B = 256 pose forward: for r in 1..reps, for each
setting, one child process times the default-stream forward (median of 5 x --steps), hashes the output
and reads the one-stream per-kernel HIP-event profile.  One JSON line per run.
usage: python tools/ab_env.py [--reps 2] [--batch 256] [--dtype f32_fft] -- "-" "MP_COL8P=0" "MP_X=1,MP_Y=2" """
import argparse
import hashlib
import importlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["col_gemm", "row_a", "row_b", "row_final", "row_init", "fc1", "fc_out", "backbone"]


def child(a):
    import torch
    sys.path.insert(0, ROOT)
    mp = importlib.import_module("monkey-pose_amd")
    W = mp.weights
    dev = torch.device("cuda:0")
    ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
    for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
        ctx.set_weight(v.name, W.synth_value(v, 1234, 8))
    ctx.finalize(mp._lib.dtype_code(a.dtype))
    B = a.batch
    depth = torch.from_numpy(W.synth_crops(B, seed=42, size=128)).to(dev)
    h0 = torch.from_numpy(W.synth_hidden((B, 64, 64, 64), seed=7)).to(dev)
    out = torch.empty((B, 69), device=dev)
    st = mp._lib.current_stream(dev)
    for _ in range(3):
        ctx.pose_fwd(depth, h0, out, st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ctx.pose_fwd(depth, h0, out, st)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / a.steps * 1e3)
    sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    ctx.profile(True)
    for _ in range(3):
        ctx.pose_fwd(depth, h0, out, st)
    torch.cuda.synchronize()
    ctx.profile(False)
    prof = {}
    for n in NAMES:
        ms, cnt = ctx.profile_read(n)
        if cnt:
            prof[n] = [round(ms / cnt, 4), cnt // 3]
    ts.sort()
    print(json.dumps({"ms": round(ts[len(ts) // 2], 4), "ms_all": [round(t, 4) for t in ts], "sha": sha,
                      "kernels": prof}))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--dtype", default="f32_fft")
    p.add_argument("--child", action="store_true")
    p.add_argument("settings", nargs="*")
    a = p.parse_args()
    if a.child:
        return child(a)
    for r in range(a.reps):
        for s in a.settings or ["-"]:
            env = dict(os.environ)
            if s != "-":
                env.update(kv.split("=", 1) for kv in s.split(","))
            cmd = [sys.executable, __file__, "--child", "--batch", str(a.batch), "--steps", str(a.steps), "--dtype", a.dtype]
            r_ = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            if r_.returncode != 0:
                print(json.dumps({"setting": s, "error": r_.stderr[-1500:]}), flush=True)
                sys.exit(1)
            d = json.loads(r_.stdout.strip().splitlines()[-1])
            d.update(setting=s, rep=r, batch=a.batch, dtype=a.dtype)
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
