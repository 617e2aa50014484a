"""Benchmark: depth-crops/s of the hGRU-8T pose forward (hgru_pose.model.build, 128x128 crops,
batch 256 per GPU), one process per GPU, weak scaling (batch shards, no data-path collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one forward of the whole hot path (conv_1 ... hGRU x8 ... fc_out) over B synthetic crops
already resident in HBM.  Weights: synthetic (splitmix64 glorot stand-ins), generated on rank 0
and broadcast ONCE over RCCL (xGMI) as one flat fp32 blob before timing.  Rank 0 prints one JSON
line; value = all ranks' crops / max-over-ranks elapsed.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (MFMA = vector), MI355X_MICROARCH.md chip table
PEAK_F16_TFLOPS = 2516.6   # MI355X dense f16/bf16 MFMA (no sparsity)
PEAK_HBM_GBS = 8000.0


def roofline(dtype, achieved_tf, launch_ms, launches, flop_per_launch):
    """Roofline of the dominant kernel (the hGRU eCRF conv, both half-step variants).
    achieved = ALGORITHMIC conv FLOPs per launch (2*px*15*15*64*64*B) / avg launch time.
    For the f16x3 split path every fp32 multiply-add costs three f16 MFMA products, so its
    fp32-accurate ceiling is the dense f16 MFMA peak / 3; the executed f16 rate is also given."""
    r = {"bound": "mfma", "kernel": "conv64<15> (hGRU eCRF conv, A+B half-steps)",
         "achieved": round(achieved_tf, 3), "unit": "TFLOP/s", "traffic": None,
         "avg_launch_ms": round(launch_ms, 4), "launches": launches,
         "flop_per_launch": flop_per_launch}
    if dtype == "f32":
        r.update(peak=PEAK_FP32_TFLOPS, peak_basis="dense fp32 MFMA (v_mfma_f32_32x32x2_f32)")
    else:
        r.update(peak=round(PEAK_F16_TFLOPS / 3, 1),
                 peak_basis="dense f16 MFMA peak 2516.6 / 3 products per fp32-accurate MAC",
                 executed_f16_tflops=round(3 * achieved_tf, 3),
                 executed_frac_of_f16_peak=round(3 * achieved_tf / PEAK_F16_TFLOPS, 4))
    r["frac"] = round(achieved_tf / r["peak"], 4)
    return r


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=256, help="crops per GPU")
    p.add_argument("--crop", type=int, default=128)
    p.add_argument("--timesteps", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=8, help="crops timed on the CPU oracle")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--dtype", default="f32_split", choices=["f32", "f32_split"],
                   help="hGRU eCRF conv precision: exact fp32 MFMA or fp32-accurate f16x3 split")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    mp = importlib.import_module("monkey-pose_amd")
    W = mp.weights
    B, crop, T = args.batch, args.crop, args.timesteps

    # ---- weights: generate on rank 0, one RCCL broadcast of the flat blob ----
    table = W.hgru_pose_vars(output_shape=69, timesteps=T, crop=crop)
    sizes = [int(np.prod(v.shape)) for v in table]
    total = int(sum(sizes))
    flat = torch.empty(total, dtype=torch.float32, device=dev)
    if rank == 0:
        host = np.empty(total, np.float32)
        o = 0
        for v, s in zip(table, sizes):
            host[o:o + s] = W.synth_value(v, 1234, T).reshape(-1)
            o += s
        flat.copy_(torch.from_numpy(host))
        del host
    bcast_ms = 0.0
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        dist.broadcast(flat, src=0)
        torch.cuda.synchronize()
        bcast_ms = (time.perf_counter() - t0) * 1e3
    ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, dev.index)
    o = 0
    for v, s in zip(table, sizes):
        ctx.set_weight(v.name, flat[o:o + s].view(*v.shape))
        o += s
    ctx.finalize(mp._lib.dtype_code(args.dtype))
    del flat
    ctx.reserve(B)

    # ---- synthetic inputs resident in HBM (per-rank shard) ----
    depth = torch.from_numpy(W.synth_crops(B, seed=42 + rank, size=crop)).to(dev)
    o0 = torch.from_numpy(W.synth_hidden((B, crop // 2, crop // 2, 64), seed=7 + rank)).to(dev)
    out = torch.empty((B, 69), dtype=torch.float32, device=dev)
    stream = mp._lib.current_stream(dev)

    for _ in range(args.warmup):
        ctx.pose_fwd(depth, o0, out, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ctx.profile(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.pose_fwd(depth, o0, out, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.profile(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_a, na = ctx.profile_read("conv15_a")
    ms_b, nb = ctx.profile_read("conv15_b")
    ms_fc, nfc = ctx.profile_read("fc1")
    ms_bb, nbb = ctx.profile_read("backbone")
    conv_launch_ms = (ms_a + ms_b) / max(1, na + nb)
    px = (crop // 2) ** 2
    conv15_flop = 2.0 * px * 15 * 15 * 64 * 64 * B            # algorithmic, per launch
    achieved_tf = conv15_flop / (conv_launch_ms * 1e-3) / 1e12

    value = world * B * args.steps / elapsed
    rec = {
        "metric": "depth-crops/sec hGRU-8T fwd @batch256 per GPU (128x128 crops, fp32)",
        "value": round(value, 3),
        "unit": "crops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.dtype == "f32" else "f32 (f16x3 split MFMA, fp32 accumulate)",
        "data": "synthetic crops + synthetic weights (splitmix64 stand-ins; reference publishes none)",
        "config": {"workload": f"hgru_pose.model.build fwd, T={T}, {crop}x{crop} crops, "
                               f"batch {B} per GPU", "global_batch": world * B, "crop": crop,
                   "timesteps": T, "parallelism": f"dp{world} (batch shards, RCCL weight broadcast)"},
        "roofline": roofline(args.dtype, achieved_tf, conv_launch_ms, na + nb, conv15_flop),
        "breakdown_ms_per_step": {"conv15": round((ms_a + ms_b) / args.steps, 3),
                                  "fc1": round(ms_fc / max(1, nfc) if nfc else 0.0, 3),
                                  "backbone": round(ms_bb / max(1, nbb) if nbb else 0.0, 3)},
        "weight_bcast_ms": round(bcast_ms, 3),
    }

    if rank == 0 and world == 1:
        from oracle import hgru_ref as R
        if not args.no_parity:
            # parity of the measured path on its first 2 crops vs the float64 oracle
            wts = {v.name: W.synth_value(v, 1234, T) for v in table}
            d2 = depth[:2].cpu().numpy()
            o2 = o0[:2].cpu().numpy()
            ref = R.hgru_pose_forward(d2, wts, o2, T, np.float64)
            got = out[:2].cpu().numpy()
            rec["parity"] = {"rel_inf_err": float(np.abs(got - ref).max() / np.abs(ref).max()),
                             "mean_joint_err_mm": R.mean_error(R.to_joints_mm(ref), R.to_joints_mm(got)),
                             "crops": 2, "oracle": "oracle/hgru_ref.py float64"}
        if not args.no_cpu_baseline:
            from threadpoolctl import threadpool_info
            wts32 = {v.name: W.synth_value(v, 1234, T) for v in table}
            nc = args.cpu_sample
            d = depth[:nc].cpu().numpy()
            oo = o0[:nc].cpu().numpy()
            t0 = time.perf_counter()
            for i in range(0, nc, 4):
                R.hgru_pose_forward(d[i:i + 4], wts32, oo[i:i + 4], T, np.float32)
            cpu_s = time.perf_counter() - t0
            threads = max([t["num_threads"] for t in threadpool_info() if t["user_api"] == "blas"] or [1])
            rec["cpu_baseline"] = {"value": round(nc / cpu_s, 4), "unit": "crops/s", "cores": threads,
                                   "kind": "port",
                                   "sample": f"{nc} crops of the same workload (numpy fp32 oracle, "
                                             f"OpenBLAS, batches of 4), {cpu_s:.1f} s"}
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
