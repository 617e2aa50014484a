"""(e) multi-GPU logic on CPU with gloo, world_size 2: shard ranges, the one-time weight broadcast,
and output gathering (the GPU path uses the same functions with the nccl = RCCL backend)."""
import os
import socket

import numpy as np
import pytest

from helpers import pkg

torch = pytest.importorskip("torch")


def test_shard_ranges_cover_batch():
    par = pkg().parallel
    for gb in (1, 7, 256, 2048, 2049):
        for world in (1, 2, 3, 8):
            rs = [par.shard_range(gb, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == gb
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in rs]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mp = importlib.import_module("monkey-pose_amd")
    W, par = mp.weights, mp.parallel
    table = W.hgru_circuit_vars(ssf=5, timesteps=3)
    wts = W.synth_weights(table, seed=9, timesteps=3) if rank == 0 else None
    flat, layout, secs = par.broadcast_weights(table, wts, torch.device("cpu"), rank, world)
    ref = W.synth_weights(table, seed=9, timesteps=3)
    ok = all(np.array_equal(flat[o:o + n].numpy().reshape(s), ref[nm]) for nm, s, o, n in layout)
    gb = 5
    s, e = par.shard_range(gb, rank, world)
    shard = torch.arange(s * 3, e * 3, dtype=torch.float32).view(-1, 3)
    full = par.gather_outputs(shard, gb, rank, world)
    ok = ok and torch.equal(full, torch.arange(gb * 3, dtype=torch.float32).view(gb, 3))
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_broadcast_and_gather_gloo_world2():
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


@pytest.mark.gpu
def test_replicate_weights_peer_tree():
    """mp_bcast_weights: weights set on one context reach three others (here all on device 0, so
    the tree's peer copies are device-local) and every replica computes bit-identical outputs."""
    P = pkg()
    L, W = P._lib, P.weights
    n, crop, T = 2, 64, 8
    table = W.hgru_pose_vars(output_shape=69, timesteps=T, crop=crop)
    ctxs = [L.Context(L.MP_MODEL_HGRU_POSE, 0) for _ in range(4)]
    for v in table:
        ctxs[2].set_weight(v.name, W.synth_value(v, 1234, T))
    P.parallel.replicate_weights(ctxs, root=2)
    depth = torch.from_numpy(W.synth_crops(n, seed=42, size=crop)).cuda()
    o0 = torch.from_numpy(W.synth_hidden((n, crop // 2, crop // 2, 64), seed=7)).cuda()
    outs = []
    for c in ctxs:
        assert c.info("weight_bytes") == ctxs[2].info("weight_bytes")
        c.finalize(L.MP_DTYPE_F32_FFT)
        o = torch.empty((n, 69), device="cuda")
        c.pose_fwd(depth, o0, o, L.current_stream())
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    other = L.Context(L.MP_MODEL_DENSE, 0)
    with pytest.raises(L.MonkeyPoseError):
        P.parallel.replicate_weights([ctxs[0], other])
    with pytest.raises(L.MonkeyPoseError):
        P.parallel.replicate_weights([L.Context(L.MP_MODEL_HGRU_POSE, 0), ctxs[0]])   # empty root
