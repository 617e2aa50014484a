"""Multi-GPU inference: one process per GPU, crops sharded by batch, weights broadcast once.

Every crop's forward is independent (inference BN uses moving statistics), so the batch splits
into contiguous shards with no per-batch collective.  The only communication is one
``torch.distributed.broadcast`` of the flat fp32 weight blob from rank 0 (RCCL over xGMI with the
"nccl" backend; gloo on CPU for tests), after which each rank packs its own copy in its context.
Spatial sharding is deliberately not offered: each hGRU half-step would need a 7-pixel halo
exchange.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Sequence, Tuple

import numpy as np


def shard_range(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [start, end) of rank ``rank``; sizes differ by at most one crop."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def flat_layout(table) -> List[Tuple[str, Tuple[int, ...], int, int]]:
    """(name, shape, offset, size) of every variable in the flat blob, in table order."""
    out, off = [], 0
    for v in table:
        n = int(np.prod(v.shape))
        out.append((v.name, tuple(v.shape), off, n))
        off += n
    return out


def broadcast_weights(table, weights: Dict[str, np.ndarray] | None, device, rank: int, world: int,
                      group=None):
    """Rank 0 packs ``weights`` (TF name -> array) into one flat fp32 tensor on ``device`` and
    broadcasts it; returns (flat tensor, layout, seconds spent in the broadcast)."""
    import time

    import torch
    import torch.distributed as dist
    layout = flat_layout(table)
    total = layout[-1][2] + layout[-1][3] if layout else 0
    flat = torch.empty(total, dtype=torch.float32, device=device)
    if rank == 0:
        host = np.empty(total, np.float32)
        for name, shape, off, n in layout:
            host[off:off + n] = np.asarray(weights[name], np.float32).reshape(-1)
        flat.copy_(torch.from_numpy(host))
    secs = 0.0
    if world > 1:
        if flat.is_cuda:
            torch.cuda.synchronize(device)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        dist.broadcast(flat, src=0, group=group)
        if flat.is_cuda:
            torch.cuda.synchronize(device)
        secs = time.perf_counter() - t0
    return flat, layout, secs


def load_context(ctx, flat, layout) -> None:
    """mp_set_weight for every variable straight from the (device) flat blob."""
    for name, shape, off, n in layout:
        ctx.set_weight(name, flat[off:off + n].view(*shape))


def gather_outputs(out_shard, global_batch: int, rank: int, world: int, group=None):
    """Optional: all ranks' [shard, k] outputs -> [global_batch, k] on every rank (all_gather of
    equal-size padded shards; 276 B per crop, negligible beside the forward)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return out_shard
    per = -(-global_batch // world)
    k = out_shard.shape[1]
    pad = torch.zeros((per, k), dtype=out_shard.dtype, device=out_shard.device)
    pad[:out_shard.shape[0]] = out_shard
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    rows = []
    for r in range(world):
        s, e = shard_range(global_batch, r, world)
        rows.append(parts[r][:e - s])
    return torch.cat(rows, 0)


def replicate_weights(contexts: Sequence, root: int = 0) -> None:
    """One process driving several GPUs: copy the weights set on ``contexts[root]`` into every
    other context (``mp_bcast_weights``: a binomial tree of device-to-device peer copies over xGMI,
    nothing through the host).  Finalize each context afterwards."""
    from . import _lib
    if not contexts:
        return
    arr = (ctypes.c_void_p * len(contexts))(*[c.h for c in contexts])
    _lib.check(contexts[0].lib.mp_bcast_weights(arr, len(contexts), int(root)))
