"""Per-layer HIP-event times of a graph façade (hier / dense / dense_hier) at batch B, one stream
(profiling mode), heaviest first.  usage: python tools/profile_graph.py [hier|dense|dense_hier] [B]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

mp = importlib.import_module("monkey-pose_amd")
kind = sys.argv[1] if len(sys.argv) > 1 else "hier"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W = mp.weights
heads = (108, 39, 39, 39, 39, 36)
if kind == "hier":
    m = mp.train_hier_networks.hier_model_struct()
    args = heads
elif kind == "dense":
    m = mp.train_dense_networks.dense_model_struct()
    args = (69,)
else:
    m = mp.train_dense_hier_networks.dense_hier_model_struct()
    args = heads
g = m.record(128, 128, *args)
m.load_weights(W.synth_weights(m._table(g), seed=3))
x = torch.from_numpy(W.synth_crops(B, seed=1, size=128)).cuda()
m.build(x, *args)
torch.cuda.synchronize()
ctx = m._ctx
ctx.profile(True)
for _ in range(3):
    m.forward(x)
torch.cuda.synchronize()
ctx.profile(False)
rows = []
for o in g.layers():
    ms, n = ctx.profile_read(o["name"])
    flop = 2.0 * B * (o["out"].shape[0] * o["out"].shape[1] * o["k"] ** 2 * o["cin"] * o["cout"]
                      if o["kind"] == 1 else o["cin"] * o["cout"])
    rows.append((ms / max(1, n), o["name"], flop / (ms / max(1, n) * 1e-3) / 1e12 if n else 0.0))
tot = {k: ctx.profile_read(k) for k in ("graph_conv", "graph_pool", "graph_fc")}
rows.sort(reverse=True)
print({k: round(v[0] / 3, 3) for k, v in tot.items()}, "ms per forward (one stream)")
for ms, name, tf in rows[:25]:
    print(f"{name:28s} {ms:8.4f} ms  {tf:7.1f} TFLOP/s")
