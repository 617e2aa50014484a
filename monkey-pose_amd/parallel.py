"""Multi-GPU inference: one process per GPU, crops sharded by batch, weights broadcast once.

Every crop's forward is independent (inference BN uses moving statistics), so the batch splits
into contiguous shards with no per-batch collective.  The only communication is one
``torch.distributed.broadcast`` of the weights from rank 0 (RCCL over xGMI with the "nccl"
backend; gloo on CPU for tests): the flat fp32 blob, or for dtype bf16 the bytes a bf16 context
reads (fc_1 as its f16 hi plane, half the bytes), after which each rank packs its own copy.
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


FC1_NAME = "cnn/fc_1/fc_1_weights"


def fc_hi_plane(w: np.ndarray):
    """The f16 "hi" plane the one-product (dtype bf16) fc_1 reads, exactly as the library packs it
    (k_fc.hip launch_pack_fc_x3 / pack_fc_x3_kernel): power-of-two scale s = 2^(14 - e) with
    frexp(max|w|) = (f, e), hi = f16(w * s) (round to nearest even; w * s is exact in fp32).
    Returns (hi, e, idx, vals): ``idx`` / ``vals`` are the few elements whose hi / s exceeds max|w|
    in magnitude (s * w within half an f16 ulp below 2^14 rounds up to it), sent as fp32 so the
    receiver's max|w'| -- hence its scale -- equals the sender's."""
    w = np.ascontiguousarray(w, np.float32).reshape(-1)
    m = float(np.abs(w).max()) if w.size else 0.0
    e = int(np.frexp(np.float32(m))[1]) if m > 0 else 0
    s = np.float32(2.0 ** (14 - e))
    hi = (w * s).astype(np.float16)
    back = hi.astype(np.float32) / s
    idx = np.nonzero(np.abs(back) > np.float32(m))[0].astype(np.int64)
    return hi, e, idx, w[idx]


def fc_from_hi_plane(hi, e: int, idx, vals):
    """Inverse of ``fc_hi_plane`` on either side (torch tensors): w' = hi / s with the exceptions
    restored.  max|w'| has the same frexp exponent as max|w| (s * max|w| lies in [2^13, 2^14) and
    its f16 rounding stays >= 2^13; a max rounding up past max|w| is sent as an exception), so the
    library packs w' to the same scale and, since s * w' = hi exactly, to the same hi plane.
    max|w'| itself may be smaller than max|w| when the max element rounds down.  The lo plane
    differs, which the one-product fc_1 never reads."""
    import torch
    s = float(2.0 ** (14 - e))
    w = hi.to(torch.float32) / s
    if idx.numel():
        w[idx] = vals
    return w


def broadcast_weights(table, weights: Dict[str, np.ndarray] | None, device, rank: int, world: int,
                      group=None, dtype: str = "fp32", info: dict | None = None):
    """Rank 0 packs ``weights`` (TF name -> array) into one flat fp32 tensor on ``device`` and
    broadcasts it; returns (flat tensor, layout, seconds spent in the broadcast).

    ``dtype='bf16'`` broadcasts what the bf16 context reads instead of the fp32 blob: fc_1's
    weights (99.5 % of the bytes, hgru_pose.py:91) go as their f16 hi plane plus the scale exponent
    (``fc_hi_plane``), everything else as fp32.  Each rank rebuilds a flat fp32 blob whose packing
    in a bf16 context is bit-identical to the original's (fp32: 1.078 GB on the wire, bf16:
    0.541 GB for the 128x128 model).  ``info`` (a dict) receives the bytes moved and the form."""
    import time

    import torch
    import torch.distributed as dist
    layout = flat_layout(table)
    total = layout[-1][2] + layout[-1][3] if layout else 0
    flat = torch.empty(total, dtype=torch.float32, device=device)
    fc = next((l for l in layout if l[0] == FC1_NAME), None) if dtype == "bf16" else None
    hi = meta = idx = vals = None
    if rank == 0:
        host = np.empty(total, np.float32)
        for name, shape, off, n in layout:
            if fc is not None and name == FC1_NAME:
                h, e, ix, vv = fc_hi_plane(weights[name])
                hi = torch.from_numpy(h).to(device)
                meta = torch.tensor([e, ix.size], dtype=torch.int64, device=device)
                idx = torch.from_numpy(ix).to(device)
                vals = torch.from_numpy(vv).to(device)
                host[off:off + n] = 0.0   # rebuilt from the hi plane below, on every rank
            else:
                host[off:off + n] = np.asarray(weights[name], np.float32).reshape(-1)
        flat.copy_(torch.from_numpy(host))
    elif fc is not None:
        hi = torch.empty(fc[3], dtype=torch.float16, device=device)
        meta = torch.empty(2, dtype=torch.int64, device=device)
    nbytes = flat.numel() * 4
    secs = 0.0
    # any initialised group runs the collective, a one-rank one included (tests/test_gpu_bench_ranks.py
    # drives RCCL through this exact code on one GPU); without a group there is nothing to send
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        if flat.is_cuda:
            torch.cuda.synchronize(device)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        if fc is None:
            dist.broadcast(flat, src=0, group=group)
        else:
            # everything but fc_1 as fp32 (the fc_1 range is zeros: sent, but 0.4 % of the blob
            # would not be worth a second layout), fc_1 as its hi plane
            small = torch.cat([flat[:fc[2]], flat[fc[2] + fc[3]:]])
            dist.broadcast(small, src=0, group=group)
            dist.broadcast(meta, src=0, group=group)
            n_exc = int(meta[1].item())
            if rank != 0:
                idx = torch.empty(n_exc, dtype=torch.int64, device=device)
                vals = torch.empty(n_exc, dtype=torch.float32, device=device)
            if n_exc:
                dist.broadcast(idx, src=0, group=group)
                dist.broadcast(vals, src=0, group=group)
            dist.broadcast(hi, src=0, group=group)
            if rank != 0:
                flat[:fc[2]] = small[:fc[2]]
                flat[fc[2] + fc[3]:] = small[fc[2]:]
            nbytes = small.numel() * 4 + hi.numel() * 2 + meta.numel() * 8 + n_exc * 12
        if flat.is_cuda:
            torch.cuda.synchronize(device)
        secs = time.perf_counter() - t0
    elif fc is not None:
        nbytes = (flat.numel() - fc[3]) * 4 + fc[3] * 2
    if fc is not None:
        e = int(meta[0].item())
        flat[fc[2]:fc[2] + fc[3]] = fc_from_hi_plane(hi, e, idx, vals)
    if info is not None:
        info.update(bytes=int(nbytes), form="fc_1 as f16 hi plane + fp32 rest" if fc is not None else "fp32 blob")
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
