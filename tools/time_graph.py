"""A/B timing of the layer-graph runtime on dense_hier_model_struct: eager launches over 1 / 2 / 4 /
8 streams, batch 256 and batch 1.  usage: python tools/time_graph.py  (STREAMS=1,8 for a subset)"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

mp = importlib.import_module("monkey-pose_amd")


def t_gpu(fn, n, w):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    W = mp.weights
    DH = mp.train_dense_hier_networks
    res = {}
    for B in (256, 1):
        depth = torch.from_numpy(W.synth_crops(B, seed=99, size=128)).cuda()
        for streams in (int(s) for s in os.environ.get("STREAMS", "1,2,4,8").split(",")):
            os.environ["MP_GRAPH_STREAMS"] = str(streams)
            model = DH.dense_hier_model_struct()
            g = model.record(128, 128, 108, 39, 39, 39, 39, 36)
            model.load_weights(W.synth_weights(model._table(g), seed=8))
            model.build(depth, 108, 39, 39, 39, 39, 36)
            t = t_gpu(lambda: model.forward(depth), 10 if B > 1 else 30, 2)
            k = f"B{B}_eager_s{streams}"
            res[k] = {"ms": round(t * 1e3, 3), "crops_per_s": round(B / t, 1)}
            print(k, res[k], flush=True)
            del model
    print(json.dumps(res))


if __name__ == "__main__":
    main()
