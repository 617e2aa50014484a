"""Bit-identity probe of the FFT path's batch slicing (not a test): the pose forward of 96 crops with
the two-stream slices, with the one-stream profile schedule, and crop 70 alone; prints which crops differ."""
import importlib, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")
W = mp.weights
dtype = sys.argv[1] if len(sys.argv) > 1 else "fp32_fft"
n = int(os.environ.get("SPLIT_N", "96"))
reps = int(os.environ.get("SPLIT_REPS", "3"))
ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
    ctx.set_weight(v.name, W.synth_value(v, 1234, 8))
ctx.finalize(mp._lib.dtype_code(dtype))
dev = torch.device("cuda:0")
depth = torch.from_numpy(W.synth_crops(n, seed=3, size=128)).to(dev)
o0 = torch.from_numpy(W.synth_hidden((n, 64, 64, 64), seed=4)).to(dev)
st = mp._lib.current_stream(dev)
outs = {}
runs = [("split", False)] + [(f"split{r}", False) for r in range(2, reps + 1)] + [("prof", True), ("prof2", True)]
for name, prof in runs:
    o = torch.empty((n, 69), device=dev)
    ctx.profile(prof)
    ctx.pose_fwd(depth, o0, o, st)
    ctx.profile(False)
    torch.cuda.synchronize()
    outs[name] = o.cpu()
for a, b in [("split", f"split{r}") for r in range(2, reps + 1)] + [("prof", "prof2"), ("split", "prof")]:
    d = (outs[a] != outs[b]).any(dim=1).nonzero().flatten().tolist()
    m = (outs[a] - outs[b]).abs().max().item()
    print(f"{dtype} {a} vs {b}: {len(d)} crops differ (max |d| {m:.3e}) {d[:12]}")
for k in [0, 40, 70]:
    one = torch.empty((1, 69), device=dev)
    ctx.pose_fwd(depth[k:k + 1].contiguous(), o0[k:k + 1].contiguous(), one, st)
    torch.cuda.synchronize()
    print(f"{dtype} crop {k} alone == split: {torch.equal(one[0].cpu(), outs['split'][k])}  == prof: {torch.equal(one[0].cpu(), outs['prof'][k])}")
# per-step states of two split runs: the first step whose I_t / O_t differ, and where
if os.environ.get("SPLIT_QUICK"):
    sys.exit(0)
taps = []
for r in range(3):
    sO = torch.empty((n, 8, 64, 64, 64), device=dev)
    sI = torch.empty((n, 8, 64, 64, 64), device=dev)
    o = torch.empty((n, 69), device=dev)
    ctx.pose_fwd_taps(depth, o0, o, {"states_O": sO, "states_I": sI}, st)
    torch.cuda.synchronize()
    taps.append((sI, sO))
for r in (1, 2):
    for t in range(8):
        for nm, k in (("I", 0), ("O", 1)):
            a, b = taps[0][k][:, t], taps[r][k][:, t]
            d = (a != b)
            if d.any():
                idx = d.nonzero()
                m = (a - b).abs().max().item()
                crops = sorted(set(idx[:, 0].tolist()))
                chans = sorted(set(idx[:, 3].tolist()))
                print(f"run0 vs run{r}: first diff at step {t} {nm}: {int(d.sum())} values, max {m:.3e}, "
                      f"crops {crops[:10]} ({len(crops)}), channels {chans[:16]} ({len(chans)}), "
                      f"pixels e.g. {idx[:5, 1:3].tolist()}")
                break
        else:
            continue
        break
    else:
        print(f"run0 vs run{r}: all states identical")
