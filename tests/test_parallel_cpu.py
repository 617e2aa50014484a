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


def test_fc_hi_plane_round_trip_keeps_scale_and_plane():
    """fc_1's hi plane (the bf16 fc_1 reads only it) survives the w -> hi -> w' round trip with the
    same power-of-two scale, including elements that round up to 2^14 (the scale's boundary)."""
    par = pkg().parallel
    rng = np.random.default_rng(3)
    w = rng.standard_normal(4096).astype(np.float32)
    m = float(np.abs(w).max())
    e = int(np.frexp(np.float32(m))[1])
    s = 2.0 ** (14 - e)
    w[7] = np.float32((2 ** 14 - 1) / s)            # max element: s * w rounds up to 2^14 in f16
    w[9] = -np.float32((2 ** 14 - 2) / s)           # another element rounding up in magnitude
    h, e0, idx, vals = par.fc_hi_plane(w)
    assert 7 in idx and 9 in idx
    w2 = par.fc_from_hi_plane(torch.from_numpy(h), e0, torch.from_numpy(idx), torch.from_numpy(vals)).numpy()
    h2, e2, _, _ = par.fc_hi_plane(w2)
    assert e2 == e0 and np.array_equal(h.view(np.uint16), h2.view(np.uint16))
    assert float(np.abs(w2).max()) == float(np.abs(w).max())


def test_fc_hi_plane_round_trip_max_rounding_down():
    """The max element rounds DOWN in f16: max|w'| < max|w|, but the frexp exponent -- hence the
    pack scale and the hi plane -- is unchanged (the invariant fc_from_hi_plane relies on)."""
    par = pkg().parallel
    rng = np.random.default_rng(4)
    w = (rng.standard_normal(4096) * 0.01).astype(np.float32)
    e = 1
    s = 2.0 ** (14 - e)
    w[11] = np.float32((2 ** 13 + 3) / s)           # s * w = 8195: the f16 grid there is 8, -> 8192
    h, e0, idx, vals = par.fc_hi_plane(w)
    assert e0 == e and 11 not in idx
    w2 = par.fc_from_hi_plane(torch.from_numpy(h), e0, torch.from_numpy(idx), torch.from_numpy(vals)).numpy()
    assert float(np.abs(w2).max()) < float(np.abs(w).max())
    h2, e2, _, _ = par.fc_hi_plane(w2)
    assert e2 == e0 and np.array_equal(h.view(np.uint16), h2.view(np.uint16))


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
    # dtype bf16: fc_1 travels as its f16 hi plane; the rebuilt blob packs to the same hi plane and
    # scale on every rank, every other weight arrives bit for bit
    ptab = W.hgru_pose_vars(output_shape=69, timesteps=3, crop=32)
    pw = {v.name: W.synth_value(v, 1234, 3) for v in ptab}
    info = {}
    pflat, play, _ = par.broadcast_weights(ptab, pw if rank == 0 else None, torch.device("cpu"), rank, world,
                                           dtype="bf16", info=info)
    for nm, sh, o, n in play:
        got = pflat[o:o + n].numpy().reshape(sh)
        if nm == par.FC1_NAME:
            h0, e0, _, _ = par.fc_hi_plane(pw[nm])
            h1, e1, _, _ = par.fc_hi_plane(got)
            ok = ok and e0 == e1 and np.array_equal(h0.view(np.uint16), h1.view(np.uint16))
        else:
            ok = ok and np.array_equal(got, pw[nm])
    ok = ok and info["bytes"] < 0.55 * pflat.numel() * 4   # fc_1 is ~all of the bytes
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
