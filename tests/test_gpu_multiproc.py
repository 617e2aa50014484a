"""The multi-GPU path end to end with the HIP library, as close to config 4 as one
GPU allows: two fresh processes (spawned, one rank each, gloo as the process group since both
share device 0 -- RCCL refuses two ranks on one device), rank 0 generates the weights and
broadcasts the flat blob once (``parallel.broadcast_weights``), every rank loads its own context
(``parallel.load_context`` -> mp_set_weight / mp_finalize_weights), runs ``mp_hgru_pose_fwd`` on
its ``shard_range`` of a 96-crop batch, and ``parallel.gather_outputs`` reassembles [96, 69].
The gathered output must equal a single-process run bit for bit (every crop's forward is
independent of its batch neighbours; batch invariance is pinned in test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest

from helpers import pkg

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GLOBAL_BATCH = 96


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, dtype, q):
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        mp = importlib.import_module("monkey-pose_amd")
        W, par = mp.weights, mp.parallel
        dev = torch.device("cuda", 0)
        table = W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128)
        wts = {v.name: W.synth_value(v, 1234, 8) for v in table} if rank == 0 else None
        flat, layout, _ = par.broadcast_weights(table, wts, torch.device("cpu"), rank, world)
        ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
        par.load_context(ctx, flat.to(dev), layout)
        ctx.finalize(mp._lib.dtype_code(dtype))
        s, e = par.shard_range(GLOBAL_BATCH, rank, world)
        depth = torch.from_numpy(W.synth_crops(GLOBAL_BATCH, seed=5, size=128)[s:e]).to(dev)
        o0 = torch.from_numpy(W.synth_hidden((GLOBAL_BATCH, 64, 64, 64), seed=6)[s:e]).to(dev)
        out = torch.empty((e - s, 69), device=dev)
        ctx.pose_fwd(depth, o0, out, mp._lib.current_stream(dev))
        torch.cuda.synchronize()
        full = par.gather_outputs(out.cpu(), GLOBAL_BATCH, rank, world)
        ctx.close()
        q.put((rank, full.numpy() if rank == 0 else None, None))
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001 -- reported to the parent
        q.put((rank, None, repr(ex)))


@pytest.mark.parametrize("dtype", ["fp32_fft", "bf16"])
def test_two_rank_shards_equal_single_process(dtype):
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, dtype, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, arr, err = q.get(timeout=240)
        assert err is None, f"rank {r}: {err}"
        got[r] = arr
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered = got[0]
    assert gathered.shape == (GLOBAL_BATCH, 69)

    mp = pkg()
    W = mp.weights
    dev = torch.device("cuda", 0)
    one = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
    for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
        one.set_weight(v.name, W.synth_value(v, 1234, 8))
    one.finalize(mp._lib.dtype_code(dtype))
    depth = torch.from_numpy(W.synth_crops(GLOBAL_BATCH, seed=5, size=128)).to(dev)
    o0 = torch.from_numpy(W.synth_hidden((GLOBAL_BATCH, 64, 64, 64), seed=6)).to(dev)
    ref = torch.empty((GLOBAL_BATCH, 69), device=dev)
    one.pose_fwd(depth, o0, ref, mp._lib.current_stream(dev))
    torch.cuda.synchronize()
    assert np.array_equal(gathered, ref.cpu().numpy())
