"""Time single convolutions of the graph runtime (f16x3 implicit GEMM) at batch B, one stream.

usage: python tools/conv_bench.py [B] [H,W,Cin,Cout,k[,stride]] ...
Default shapes: the hier trunk / branch / head convs (train_hier_networks.py:338-470).
Prints ms per launch and useful TFLOP/s (2·M·N·K, the f16x3 split's 3 MFMAs not counted)."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

mp = importlib.import_module("monkey-pose_amd")
G, L = mp._graph, mp._lib

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
specs = [tuple(int(v) for v in s.split(",")) for s in sys.argv[2:]] or [
    (64, 64, 64, 128, 3), (32, 32, 128, 256, 3), (16, 16, 256, 512, 3), (8, 8, 512, 512, 3), (4, 4, 512, 1024, 5)]
rng = np.random.default_rng(0)
for spec in specs:
    H, W, ci, co, k = spec[:5]
    s = spec[5] if len(spec) > 5 else 1
    g = G.GraphRecorder(H, W, ci)
    y = g.conv(g.input, ci, co, "c", k=k, stride=s)
    ctx = L.Context(L.MP_MODEL_GRAPH, 0)
    G.install(ctx, g, [y])
    ctx_w = (rng.standard_normal((k, k, ci, co)) * 0.05).astype(np.float32)
    ctx.set_weight("c/c_filters", ctx_w)
    ctx.set_weight("c/c_biases", np.zeros(co, np.float32))
    ctx.finalize(L.MP_DTYPE_F32_SPLIT)
    x = torch.randn(B, H, W, ci, device="cuda")
    Ho, Wo = -(-H // s), -(-W // s)
    o = torch.empty(B, Ho, Wo, co, device="cuda")
    st = L.current_stream()
    for _ in range(3):
        ctx.graph_fwd(x, [o], st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        ctx.graph_fwd(x, [o], st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    wt = torch.from_numpy(ctx_w).to("cuda", torch.float64).permute(3, 2, 0, 1)
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), wt, stride=s, padding=k // 2)
    ref = ref.clamp_min(0).permute(0, 2, 3, 1)[:, :Ho, :Wo]
    err = float((o.double() - ref).abs().max() / ref.abs().max())
    fl = 2.0 * B * Ho * Wo * k * k * ci * co
    print(f"B={B} {H}x{W} {ci}->{co} k{k} s{s}: {ms:.4f} ms  {fl / ms / 1e9:.1f} TFLOP/s  rel err {err:.2e}", flush=True)
