"""Benchmark: depth-crops/s of the hGRU-8T pose forward (hgru_pose.model.build, 128x128 crops),
one process per GPU, batch shards, no data-path collective.  Default: batch 256 per GPU (weak
scaling, SURVEY config 4's sharding); ``--global-batch 256`` reads the metric as one batch of 256
over N GPUs (strong scaling, 256 / N per GPU).  At N > 1 the line also carries the other reading
as ``other_scaling_row``.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B | --global-batch G] [--dtype ...]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one forward of the whole hot path (conv_1 ... hGRU x8 ... fc_out) over B synthetic crops
already resident in HBM.  Weights: synthetic (splitmix64 glorot stand-ins), generated on rank 0
and broadcast ONCE over RCCL (xGMI) as one flat fp32 blob before timing.  Rank 0 prints one JSON
line; value = all ranks' crops / max-over-ranks elapsed.  At N=1 the line also carries the parity
of the measured path vs the float64 oracle, the CPU baseline, and "extras" (the other BASELINE
configs: hierarchical regressor at batch 256, dense regressor, batch-1 end-to-end latency with the
host CoM crop).
"""
import argparse
import datetime
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
PEAK_HBM_GBPS = 8000.0     # MI355X HBM3E
HBM_ACHIEVABLE_GBPS = 6290.0   # MI355X_MICROARCH.md: "8 TB/s peak (spec); ~6.3 TB/s achievable"
BF16_REL_TOL = 5e-3        # stated gate of the bf16 path (bf16 cannot meet 1e-4; measured ~8e-4)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=256, help="crops per GPU (weak scaling, the default)")
    p.add_argument("--global-batch", type=int, default=None,
                   help="crops over all GPUs, sharded contiguously (strong scaling: each GPU gets "
                        "global/N; the metric's 'batch 256 at 1/2/4/8 GPU' reading)")
    p.add_argument("--crop", type=int, default=128)
    p.add_argument("--timesteps", type=int, default=8)
    p.add_argument("--dtype", default="f32_fft", choices=["f32", "f32_split", "f32_fft", "bf16"],
                   help="hGRU eCRF conv path: exact fp32 MFMA direct, fp32-accurate f16x3 split "
                        "direct, fp32 FFT convolution, or the FFT path with bf16 spectral GEMMs")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--no-extras", action="store_true")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    return p.parse_args()


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


def fft_kernels(ctx, B, hw, steps, bf16=False):
    """Per-kernel time / algorithmic traffic of the FFT conv path (k_fft.hip), per launch."""
    NF, act = 72 * 37, B * 64 * hw * 4                 # frequencies; one fp32 C8 activation map
    ent = 16 if bf16 else 32                           # bytes per (4-channel group, frequency)
    spec = B * 16 * NF * ent                           # one spectrum buffer [b][cq][f][ent]
    # the maps X, O, I, Og, P2 are bf16 under dtype bf16 (k_fft.hip map_ld4; MP_BF16_MAPS=0: fp32)
    sm = act // 2 if bf16 and os.environ.get("MP_BF16_MAPS", "1") != "0" else act
    algo = {   # name: (bytes, flops) per launch
        # the six-launch loop (k_fft.hip; dtype bf16, or MP_FFT4=0)
        "fft_fwd": (sm + spec, 0.0),                   # Og in; S out
        "spec_gemm": (2 * spec + NF * ent * 1024, 8.0 * B * NF * 64 * 64),   # S in, Y out, weights
        "inv_a_fwd": (2 * spec + 3 * sm, 0.0),         # Y, X, O in; I, S out
        "fft_inv": (spec + sm, 0.0),                   # Y in; P out
        "epi_b": (5 * sm, 0.0),                        # P, I, O in; O', Og' out
        # the four-step loop (k_fft4.hip, the fp32 default): Z is a spectrum-sized complex64 buffer
        "col_gemm": (2 * spec + NF * ent * 1024, 8.0 * B * NF * 64 * 64),    # Z in, Z' out, weights
        "row_a": (2 * spec + 3 * sm, 0.0),             # Z', X, O in; I, Z out
        "row_b": (2 * spec + 3 * sm, 0.0),             # Z', I, O in; O', Z out
        "row_final": (spec + 2 * sm + act, 0.0),       # Z', I, O in; BN_3(O_T) NHWC (fp32 / split planes) out
        # O0 (NHWC fp32) in; Z out, and the C8 state map O under bf16 (the fp32 loop's step 0 reads O0
        # itself: MP_O0_DIRECT)
        "row_init": (act + spec + (sm if bf16 or os.environ.get("MP_O0_DIRECT", "1") == "0" else 0), 0.0),
    }
    out = {}
    # the fp32 path's spectral GEMM is f16x3 (three f16 MFMA products per fp32-accurate MAC): its
    # ceiling is the dense f16 peak / 3, not the fp32 MFMA peak; bf16 is one product per MAC
    mfma_peak = PEAK_F16_TFLOPS if bf16 else round(PEAK_F16_TFLOPS / 3, 1)
    for name, (byt, flop) in algo.items():
        ms, n = ctx.profile_read(name)
        if n == 0:
            continue
        t = ms / n * 1e-3
        hbm = byt / t / 1e9
        k = {"ms_per_step": round(ms / steps, 3), "avg_launch_ms": round(ms / n, 4), "launches": n,
             "algo_bytes": byt, "achieved_GBps": round(hbm, 1), "hbm_frac": round(hbm / PEAK_HBM_GBPS, 4)}
        if flop:
            k.update(algo_flop=flop, achieved_tflops=round(flop / t / 1e12, 2),
                     mfma_frac=round(flop / t / 1e12 / mfma_peak, 4), mfma_peak=mfma_peak)
        out[name] = k
    return out


# per-kernel HBM bytes per launch from rocprofv3 PMC passes (FETCH_SIZE x2 on gfx950 + WRITE_SIZE,
# MI355X_MICROARCH.md), collected with the full-batch single-stream launches of this workload by
# tools/pmc_bytes.py and committed under profiles/ (bench cannot profile itself)
PROFILE_DIR = "profiles/r6"
PMC_TRAFFIC = {False: PROFILE_DIR + "/pmc_traffic_fp32_b256.csv",
               True: PROFILE_DIR + "/pmc_traffic_bf16_b256.csv"}
PMC_KERNEL = {   # name: (fp32 path's kernel, bf16 path's kernel) as rocprofv3 names them
    "fft_fwd": ("fft_fwd3_kernel", "fft_fwd_kernel<true, true>"),
    "spec_gemm": ("spec_gemm_kernel<0, 32>", "spec_gemm_bf_kernel"),
    "inv_a_fwd": ("fft_inv_a_fwd_kernel<false, false>", "fft_inv_a_fwd_kernel<true, true>"),
    "fft_inv": ("fft_inv_kernel<false, false>", "fft_inv_kernel<true, true>"),
    "epi_b": ("spec_epi_b_kernel<false, false, false>", "spec_epi_b_kernel<true, true, false>"),
    # the four-step loop's default kernels (k_fft4.hip: col8 / row8 forms)
    # (prefixes: the template arguments after the dtype flag are cache-policy switches)
    "col_gemm": ("col8p_kernel", "col8_bf_kernel"), "row_a": ("row8_kernel<0, false", "row8_kernel<0, true"),
    "row_b": ("row8_kernel<1, false", "row8_kernel<1, true"),
    "row_final": ("row8_kernel<2, false", "row8_kernel<2, true"),
    "row_init": ("row8_kernel<3, false", "row8_kernel<3, true")}


# MFMA utilisation per kernel from the committed PMC pass (tools/pmc_mfma.sh / .py: SQ_VALU_MFMA_BUSY_CYCLES
# over GRBM_GUI_ACTIVE x 1024 SIMDs, the gfx950 MfmaUtil), same one-stream B = 256 workload
PMC_MFMA = PROFILE_DIR + "/mfma_util_pose_fp32_b256.csv"
MFMA_KERNELS = {"col8p (four-step spectral GEMM, k_fft4.hip)": "col8p_kernel",
                "row8 B (gate GEMMs, k_fft4.hip)": "row8_kernel<1, false",
                "fc_gemm_x3p (fc_1 on split planes, k_fc.hip)": "fc_gemm_x3p_kernel", "conv64x3 (conv_2/3, k_conv64x3.hip)": "conv64x3_kernel",
                "spec_gemm (k_fft.hip)": "spec_gemm_kernel", "spec_epi_b (gate GEMMs, k_fft.hip)": "spec_epi_b_kernel<false, false, false>",
                "gate_init_x3 (k_fft.hip)": "gate_init_x3_kernel"}


def tree_stamp():
    """sha256 (16 hex digits) of the native sources libmonkeypose.so is built from (csrc/*.hip, *.hpp,
    the Makefile, include/monkeypose.h): which kernels a profile or a bench line was measured on."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "monkey-pose_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".hpp")) or f == "Makefile")
    for f in files + ["../../include/monkeypose.h"]:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def profile_stamp():
    """The STAMP.json of the committed profile directory the roofline's PMC figures come from (git
    head and source hash of the tree they were collected on; tools/stamp_tree.py), with whether its
    source hash equals this tree's."""
    path = os.path.join(ROOT, PROFILE_DIR, "STAMP.json")
    if not os.path.exists(path):
        return {"dir": PROFILE_DIR, "stamp": None, "matches_this_tree": False}
    st = json.load(open(path))
    cur = tree_stamp()
    ok = st.get("src_sha") == cur
    if not ok:
        sys.stderr.write(f"bench.py: WARNING the PMC figures in {PROFILE_DIR} were collected on sources "
                         f"{st.get('src_sha')} (git {st.get('git_head')}), this tree is {cur}\n")
    return {"dir": PROFILE_DIR, "git_head": st.get("git_head"), "src_sha": st.get("src_sha"),
            "this_tree_src_sha": cur, "matches_this_tree": ok}


def pmc_mfma_busy():
    """{kernel: MFMA-busy fraction} of the MFMA kernels of the pose forward (fp32 path, B = 256)."""
    import csv
    full = os.path.join(os.path.dirname(os.path.abspath(__file__)), PMC_MFMA)
    if not os.path.exists(full):
        return None
    rows = list(csv.DictReader(open(full)))
    out = {}
    for label, tag in MFMA_KERNELS.items():
        for r in rows:
            if tag in r["kernel"]:
                out[label] = float(r["mfma_util"])
                break
    return {"source": PMC_MFMA, "mfma_busy": out}


PMC_FORWARD = PROFILE_DIR + "/pmc_forward_bytes.json"


def pmc_forward_bytes(dtype, batch):
    """Summed PMC HBM bytes of one whole pose forward (every kernel, B = 256) from the committed pass."""
    full = os.path.join(os.path.dirname(os.path.abspath(__file__)), PMC_FORWARD)
    if batch != 256 or not os.path.exists(full):
        return None
    d = json.load(open(full))
    return dict(d.get(dtype, {}), source=d["source"]) if dtype in d else None


def pmc_traffic(name, bf16, batch):
    """(bytes per launch, source) of kernel `name` from the committed PMC summary, or (None, why)."""
    import csv
    path = PMC_TRAFFIC.get(bf16)
    full = os.path.join(os.path.dirname(os.path.abspath(__file__)), path) if path else None
    if batch != 256 or not full or not os.path.exists(full):
        return None, "no PMC summary for this dtype / batch"
    tag = PMC_KERNEL[name][1 if bf16 else 0]
    if tag is None:
        return None, "no kernel of this name on this dtype"
    for r in csv.DictReader(open(full)):
        if tag in r["kernel"]:
            return round(float(r["traffic_MB"]) * 1e6), path
    return None, "kernel not in the PMC summary"


def fft_roofline(kern, bf16=False, batch=256, hbm_meas=None):
    """Roofline of the dominant FFT-path kernel: its binding roof (HBM bytes or fp32 MFMA FLOPs,
    whichever bounds it tighter at peak) against its measured average launch time."""
    name = max(kern, key=lambda k: kern[k]["ms_per_step"])
    k = kern[name]
    traffic, src = pmc_traffic(name, bf16, batch)
    src_file = "k_fft4.hip" if name in ("col_gemm", "row_a", "row_b", "row_final", "row_init") else "k_fft.hip"
    r = {"kernel": f"{name} ({src_file})", "avg_launch_ms": k["avg_launch_ms"], "launches": k["launches"],
         "traffic": traffic, "traffic_source": src, "algo_bytes": k["algo_bytes"],
         # FETCH_SIZE x 2 + WRITE_SIZE count L2 misses whether the Infinity Cache or HBM serves them:
         # from 128 images the column launches' spectral weights are Infinity Cache hits (MP_MAP_NT,
         # DESIGN.md section 8), so this figure includes them
         "traffic_counts": "L2 misses (Infinity Cache hits included)"}
    t_hbm = k["algo_bytes"] / (PEAK_HBM_GBPS * 1e9)
    peak = k.get("mfma_peak", round(PEAK_F16_TFLOPS / 3, 1))
    t_mfma = k.get("algo_flop", 0.0) / (peak * 1e12)
    if t_mfma > t_hbm:
        r.update(bound="mfma", achieved=k["achieved_tflops"], peak=peak, unit="TFLOP/s",
                 peak_basis="dense MFMA peak of the GEMM's operand type", frac=k["mfma_frac"])
    else:
        r.update(bound="hbm", achieved=k["achieved_GBps"], peak=PEAK_HBM_GBPS, unit="GB/s",
                 peak_basis="HBM3E 8 TB/s", frac=k["hbm_frac"],
                 frac_of_guide_achievable=round(k["achieved_GBps"] / HBM_ACHIEVABLE_GBPS, 4),
                 guide_achievable_GBps=HBM_ACHIEVABLE_GBPS)
        if hbm_meas:
            r["measured_GBps"] = hbm_meas
            for kind in ("read", "write", "copy"):
                r[f"frac_of_measured_{kind}"] = round(k["achieved_GBps"] / hbm_meas[f"{kind}_GBps"], 4)
    return r


def hbm_rates(dev):
    """The box's streaming HBM ceilings from the library's own probe kernels (mp_hbm_probe: read-only,
    write-only and copy over 2 GiB buffers, best over grids, accesses in flight per thread and cache
    policy), the practical roof next to the 8 TB/s spec figure (re-measure the peaks)."""
    mp = importlib.import_module("monkey-pose_amd")
    return mp._lib.hbm_probe(dev.index, 2 << 30)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def time_gpu(fn, steps, warmup):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def extras(mp, dev, args):
    """The other BASELINE.json configs, measured on this GPU (not the headline)."""
    import torch
    W = mp.weights
    out = {}
    B = args.batch
    depth = torch.from_numpy(W.synth_crops(B, seed=99, size=128)).to(dev)
    stream = mp._lib.current_stream(dev)
    try:   # config 3 through the façade's default engine: the recorded graph, multi-stream
        hm = mp.train_hier_networks.hier_model_struct()
        hm.load_weights({v.name: W.synth_value(v, 5) for v in W.hier_vars()})
        hm.build(depth, 108, 39, 39, 39, 39, 36)
        t = time_gpu(lambda: hm.forward(depth), 20, 3)
        out["hier_b256"] = {"crops_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3),
                            "gflop_per_crop": 7.97, "tflops": round(7.97e9 * B / t / 1e12, 2),
                            "dtype": "fp32_split", "engine": "layer-graph runtime (mp_graph_fwd)",
                            "streams": hm._ctx.info("graph_streams")}
        hm._ctx.close()
    except Exception as e:  # noqa: BLE001
        out["hier_b256"] = {"error": repr(e)}
    for dt in ("fp32_split", "fp32"):   # config 3 on the one-stream C-ABI schedule (mp_hier_fwd)
        key = "hier_b256_abi" + ("" if dt == "fp32_split" else "_exact_fp32")
        try:
            ctx = mp._lib.Context(mp._lib.MP_MODEL_HIER, dev.index)
            for v in W.hier_vars():
                ctx.set_weight(v.name, W.synth_value(v, 5))
            ctx.finalize(mp._lib.dtype_code(dt))
            heads = [torch.empty((B, s), device=dev) for s in (108, 39, 39, 39, 39, 36)]
            t = time_gpu(lambda: ctx.hier_fwd(depth, heads, stream), 5, 1)
            out[key] = {"crops_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3),
                        "gflop_per_crop": 7.97, "tflops": round(7.97e9 * B / t / 1e12, 2), "dtype": dt}
            ctx.close()
        except Exception as e:  # noqa: BLE001
            out[key] = {"error": repr(e)}
    try:   # config 2 (B = 64) and the metric's strong-scaling per-GPU batches (256 / N for N = 2, 4, 8)
        ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, dev.index)
        T = args.timesteps
        for v in W.hgru_pose_vars(output_shape=69, timesteps=T, crop=128):
            ctx.set_weight(v.name, W.synth_value(v, 1234, T))
        ctx.finalize(mp._lib.dtype_code(args.dtype))
        o_all = torch.from_numpy(W.synth_hidden((128, 64, 64, 64), seed=7)).to(dev)
        pts = {}
        for b in (128, 64, 32):
            db, ob = depth[:b].contiguous(), o_all[:b].contiguous()
            outb = torch.empty((b, 69), device=dev)
            t = time_gpu(lambda: ctx.pose_fwd(db, ob, outb, stream), 10, 2)
            pts[f"b{b}"] = {"crops_per_s": round(b / t, 2), "ms_per_batch": round(t * 1e3, 3)}
        out["hgru_b64"] = dict(pts["b64"], dtype=args.dtype)
        out["strong_scaling_per_gpu"] = {"note": "one GPU at the per-GPU batch of global batch 256 over "
                                                 "N = 2, 4, 8 GPUs; 'efficiency' = per-crop rate / the B=256 rate",
                                         **pts}
        ctx.close()
    except Exception as e:  # noqa: BLE001
        out["hgru_b64"] = {"error": repr(e)}
    try:   # the façade's default call: hidden_init 'random' drawn on the device per call (no h2_init)
        pm = mp.hgru_pose.model()
        pm.compute_dtype = {"f32_fft": "fp32_fft", "bf16": "bf16", "f32_split": "fp32_split", "f32": "fp32"}[args.dtype]
        pm.build(depth, 69)
        t = time_gpu(lambda: pm.forward(depth), 10, 2)
        out["hgru_facade_default_o0_b256"] = {
            "crops_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3), "dtype": args.dtype,
            "path": "hgru_pose.model().forward(depth): O0 drawn on the device per call (MP_HIDDEN_RANDOM), "
                    "no host RNG, no H2D"}
        pm._ctx.close()
    except Exception as e:  # noqa: BLE001
        out["hgru_facade_default_o0_b256"] = {"error": repr(e)}
    try:   # config 1 plumbing model at batch 256, façade default engine (recorded graph)
        dm = mp.train_dense_networks.dense_model_struct()
        dm.load_weights({v.name: W.synth_value(v, 6) for v in W.dense_vars()})
        dm.build(depth, 69)
        t = time_gpu(lambda: dm.forward(depth), 20, 3)
        out["dense_b256"] = {"crops_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3),
                             "gflop_per_crop": 3.22, "tflops": round(3.22e9 * B / t / 1e12, 2),
                             "dtype": "fp32_split", "engine": "layer-graph runtime (mp_graph_fwd)"}
        dm._ctx.close()
    except Exception as e:  # noqa: BLE001
        out["dense_b256"] = {"error": repr(e)}
    try:   # the same on the one-stream C-ABI schedule (mp_dense_fwd)
        ctx = mp._lib.Context(mp._lib.MP_MODEL_DENSE, dev.index)
        for v in W.dense_vars():
            ctx.set_weight(v.name, W.synth_value(v, 6))
        ctx.finalize(mp._lib.MP_DTYPE_F32_SPLIT)
        o = torch.empty((B, 69), device=dev)
        t = time_gpu(lambda: ctx.dense_fwd(depth, o, stream), 5, 1)
        out["dense_b256_abi"] = {"crops_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3),
                                 "gflop_per_crop": 3.22, "tflops": round(3.22e9 * B / t / 1e12, 2),
                                 "dtype": "fp32_split"}
        ctx.close()
    except Exception as e:  # noqa: BLE001
        out["dense_b256_abi"] = {"error": repr(e)}
    try:   # cnn_model_struct: the regressor the reference's driver validates / tests with (169, 291, 363)
        cm = mp.train_cnn_networks_hgru.cnn_model_struct()
        g = cm.record(128, 128, 69)
        cm.load_weights(W.synth_weights(cm._table(g), seed=81))
        gf = mp._graph.flops_per_sample(g) / 1e9
        rec = {"gflop_per_crop": round(gf, 3), "engine": "layer-graph runtime (mp_graph_fwd)"}
        for dt in ("fp32_split", "bf16"):
            cm.compute_dtype = dt
            cm.build(depth, 69)
            t = time_gpu(lambda: cm.forward(depth), 20, 3)
            rec[dt] = {"crops_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3),
                       "tflops": round(gf * 1e9 * B / t / 1e12, 2)}
        rec.update(rec["fp32_split"], dtype="fp32_split")
        out["cnn_b256"] = rec
        cm._ctx.close()
    except Exception as e:  # noqa: BLE001
        out["cnn_b256"] = {"error": repr(e)}
    try:   # dense-hierarchical hybrid on the layer-graph runtime
        DH = mp.train_dense_hier_networks
        model = DH.dense_hier_model_struct()
        g = model.record(128, 128, 108, 39, 39, 39, 39, 36)
        model.load_weights(W.synth_weights(model._table(g), seed=8))
        model.build(depth, 108, 39, 39, 39, 39, 36)
        gf = mp._graph.flops_per_sample(g) / 1e9
        rec = {"gflop_per_crop": round(gf, 3), "dtype": "fp32_split",
               "kernels": model._ctx.info("graph_kernels"), "streams": model._ctx.info("graph_streams"),
               "buffers": model._ctx.info("graph_buffers")}
        t = time_gpu(lambda: model.forward(depth), 10, 2)   # eager multi-stream launches
        rec.update({"crops_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3),
                    "tflops": round(gf * 1e9 * B / t / 1e12, 2)})
        d1 = depth[:1].contiguous()
        t1 = time_gpu(lambda: model.forward(d1), 20, 3)
        rec["b1_latency_ms"] = round(t1 * 1e3, 3)
        out["dense_hier_b256"] = rec
        model._ctx.close()
    except Exception as e:  # noqa: BLE001
        out["dense_hier_b256"] = {"error": repr(e)}
    try:   # attention CoM regressor on full frames + the device chain to the pose
        out.update(frame_chain(mp, dev, args))
    except Exception as e:  # noqa: BLE001
        out["attn_b256"] = {"error": repr(e)}
    return out


def bf16_leg(mp, dev, wts, depth, o0, T, hbm_meas, steps=20):
    """BASELINE config 4's dtype at the headline's per-GPU batch: the same crops and weights through a
    bf16 context (bf16 spectra / maps / GEMM operands, fp32 accumulation and FFTs), timed like the
    headline (default streams), with its own per-kernel profile and roofline, and its parity against
    the float64 oracle on 2 crops under the stated bf16 gate."""
    import torch
    from oracle import hgru_ref as R
    B = depth.shape[0]
    ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, dev.index)
    for k, v in wts.items():
        ctx.set_weight(k, v)
    ctx.finalize(mp._lib.MP_DTYPE_BF16)
    ctx.reserve(B)
    out = torch.empty((B, 69), dtype=torch.float32, device=dev)
    stream = mp._lib.current_stream(dev)
    t = time_gpu(lambda: ctx.pose_fwd(depth, o0, out, stream), steps, 3)
    got = out[:2].cpu().numpy().astype(np.float64)
    prof_steps = 5
    ctx.profile(True)
    for _ in range(prof_steps):
        ctx.pose_fwd(depth, o0, out, stream)
    torch.cuda.synchronize()
    ctx.profile(False)
    px = (depth.shape[1] // 2) ** 2
    kern = fft_kernels(ctx, B, px, prof_steps, True)
    ms_fc, nfc = ctx.profile_read("fc1")
    ms_bb, nbb = ctx.profile_read("backbone")
    ms_fo, nfo = ctx.profile_read("fc_out")
    ctx.close()
    r64 = R.hgru_pose_forward(depth[:2].cpu().numpy(), wts, o0[:2].cpu().numpy(), T, np.float64)
    err = float(np.abs(got - r64).max() / np.abs(r64).max())
    one_stream = sum(k["ms_per_step"] for k in kern.values()) + (ms_fc + ms_bb + ms_fo) / prof_steps
    return {"crops_per_s": round(B / t, 2), "ms_per_step": round(t * 1e3, 3), "batch": B, "steps": steps,
            "dtype": "bf16 (bf16 spectra and hGRU maps, bf16 spectral / gate GEMMs, fp32 accumulate, fp32 FFTs "
                     "and elementwise math)",
            "roofline": fft_roofline(kern, True, B, hbm_meas), "fft_kernels": kern,
            "one_stream_kernel_sum_ms": round(one_stream, 3),
            "note": "ms_per_step runs two batch slices on two streams; one_stream_kernel_sum_ms is the "
                    "profiled single-stream sum of every kernel (FFT loop + fc_1 + fc_out + backbone)",
            "parity": {"rel_inf_err_fp64_oracle": err, "crops": 2, "gate": BF16_REL_TOL, "ok": err <= BF16_REL_TOL}}


ATTN_GFLOP = 3.5421   # per frame: 5 convs at 128/64/32/16/8 px (one 5x5) + afc_1 (bench docstring)


def frame_chain(mp, dev, args):
    """attn_model_struct on B full 424x512 frames, the device crop of prepare_data_test, and the
    whole test_model batch body (attention -> device crop -> hGRU pose), frames/s."""
    import torch
    W = mp.weights
    T = mp.train_cnn_networks_hgru
    B = args.batch
    frames = torch.from_numpy(W.synth_frames(B, seed=12)).to(dev)
    attn = T.attn_model_struct()
    attn.load_weights(W.attn_synth_weights(seed=21))
    com = attn.build(frames, 3)
    stream = mp._lib.current_stream(dev)
    t = time_gpu(lambda: attn.forward(frames, com), 5, 1)
    res = {"attn_b256": {"frames_per_s": round(B / t, 2), "ms_per_batch": round(t * 1e3, 3),
                         "gflop_per_frame": ATTN_GFLOP, "tflops": round(ATTN_GFLOP * 1e9 * B / t / 1e12, 2),
                         "input": "424x512 normalised frames, bilinear resize to 128x128 inside"}}
    md = mp.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    md.crop_batch_device(frames, com)          # raises if any synthetic crop failed
    tc = time_gpu(lambda: md.crop_batch_device(frames, com, check=False), 20, 2)
    res["device_crop_b256"] = {"frames_per_s": round(B / tc, 1), "ms_per_batch": round(tc * 1e3, 4),
                               "hbm_gbps_written": round(B * 128 * 128 * 4 / tc / 1e9, 1)}
    pose = mp.hgru_pose.model()
    pose.compute_dtype = args.dtype
    o0 = torch.from_numpy(W.synth_hidden((B, 64, 64, 64), seed=7)).to(dev)
    pipe = T.FramePosePipeline(attn, pose, md, check_crops=False)
    pipe.run(frames, h2_init=o0)
    tp = time_gpu(lambda: pipe.run(frames, h2_init=o0), 3, 1)
    res["frame_chain_b256"] = {"frames_per_s": round(B / tp, 2), "ms_per_batch": round(tp * 1e3, 3),
                               "path": "attention -> device crop -> hgru_pose (" + args.dtype + "), on device"}
    # batch-1 latency of the same chain: H2D of one frame, chain, D2H, absolute joints on the host
    f1 = W.synth_frames(8, seed=13)
    o1 = o0[:1].contiguous()
    lat = []
    for i in range(40):
        t0 = time.perf_counter()
        x = torch.from_numpy(f1[i % 8:i % 8 + 1]).to(dev)
        out, coms, _ = pipe.run(x, h2_init=o1)
        rel = out.cpu().numpy().reshape(23, 3) * 600.0
        md.getAbsoluteCoordinates(rel, coms.cpu().numpy()[0])
        lat.append(time.perf_counter() - t0)
    lat = np.array(lat[5:]) * 1e3
    res["e2e_batch1_gpu_chain"] = {"p50_ms": round(float(np.percentile(lat, 50)), 3),
                                   "p99_ms": round(float(np.percentile(lat, 99)), 3),
                                   "path": "H2D frame -> attention -> device crop -> hgru_pose B=1 -> D2H"}
    del stream
    return res


def e2e_latency(mp, ctx, dev, T, wts, dtype, frames=40):
    """Config 5: one 424x512 float32 depth frame per call -> native host CoM crop -> H2D -> hGRU pose
    forward at batch 1 -> D2H -> absolute joints; p50 / p99 wall latency.  The headline p50 / p99
    are the product class's default form (train_cnn_networks_hgru.StreamPosePipeline with pageable
    blocking copies, which measured no slower than pinned ones); the pinned-memory form with async
    H2D / D2H on the forward's stream is reported beside it under `pinned_async_copies`."""
    import torch
    md = mp.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    W = mp.weights
    o0 = torch.from_numpy(W.synth_hidden((1, 64, 64, 64), seed=3)).to(dev)
    fr = list(W.synth_frames(8, seed=14)[..., 0] * np.float32(10000.0))   # mm, as the crop sees it

    def pct(lat):
        lat = np.array(lat[5:]) * 1e3
        return round(float(np.percentile(lat, 50)), 3), round(float(np.percentile(lat, 99)), 3), len(lat)

    # pageable copies through the raw context (the round-2 measurement)
    out = torch.empty((1, 69), device=dev)
    stream = mp._lib.current_stream(dev)
    lat = []
    for i in range(frames):
        t0 = time.perf_counter()
        patch, M, com = md.crop_batch(fr[i % 8][None], None, nthreads=1)
        x = torch.from_numpy(patch).to(dev, non_blocking=False)
        ctx.pose_fwd(x, o0, out, stream)
        rel = out.cpu().numpy().reshape(23, 3) * 600.0
        md.getAbsoluteCoordinates(rel, com[0])
        lat.append(time.perf_counter() - t0)
    p50_raw, p99_raw, _ = pct(lat)
    # the pipeline class on a façade model with the same weights
    pm = mp.hgru_pose.model()
    pm.compute_dtype = {"f32_fft": "fp32_fft", "bf16": "bf16", "f32_split": "fp32_split", "f32": "fp32"}[dtype]
    pm.load_weights(wts)
    pm.build(torch.zeros((1, 128, 128, 1), device=dev), 69, h2_init=o0)
    res = {}
    for pinned in (False, True):
        pipe = mp.train_cnn_networks_hgru.StreamPosePipeline(pm, md, h2_init=o0, pinned=pinned)
        lat = []
        for i in range(frames):
            t0 = time.perf_counter()
            pipe.run(fr[i % 8])
            lat.append(time.perf_counter() - t0)
        res[pinned] = pct(lat)
    pm._ctx.close()
    p50, p99, n = res[False]
    return {"p50_ms": p50, "p99_ms": p99, "frames": n, "fps_capacity": round(1000.0 / p50, 1),
            "path": "StreamPosePipeline: native host crop (mp_crop3d_batch) into a reused buffer + H2D + "
                    "hgru_pose fwd B=1 (direct context call) + D2H + getAbsoluteCoordinates",
            "pinned_async_copies": {"p50_ms": res[True][0], "p99_ms": res[True][1]},
            "pageable_copies_raw_ctx": {"p50_ms": p50_raw, "p99_ms": p99_raw}}


def cpu_threads():
    """The CPUs this process may use: its affinity set, capped by a cgroup CPU quota if one is set
    (a container's cpu.max), so the baseline does not oversubscribe a CPU share."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_baseline(depth, o0, out, wts, T, args):
    """BASELINE.md's CPU-baseline plan: the torch-CPU fp32 restatement of the forward
    (oracle/hgru_torch_cpu.py, checked against the float64 oracle in tests/test_oracle.py) on every
    CPU the process may use, timed on a bounded sample of the same crops (batches of 8 until ~12 s
    have passed, at most the whole batch).  Its outputs double as the parity check of the measured GPU
    path; the float64 numpy oracle checks the first 2 crops as well."""
    import torch
    from oracle import hgru_ref as R
    from oracle import hgru_torch_cpu as TC
    threads, avail, quota = cpu_threads()
    torch.set_num_threads(threads)
    P = TC.prepare(wts, T)
    bs, cap, budget = 8, depth.shape[0], 12.0
    d = depth[:cap].cpu().numpy()
    oo = o0[:cap].cpu().numpy()
    TC.forward(d[:2], P, oo[:2], T)                       # warm-up (oneDNN primitive creation)
    refs, done = [], 0
    t0 = time.perf_counter()
    while done < cap and (time.perf_counter() - t0) < budget:
        refs.append(TC.forward(d[done:done + bs], P, oo[done:done + bs], T))
        done += bs
    cpu_s = time.perf_counter() - t0
    res = {"cpu_baseline": {"value": round(done / cpu_s, 4), "unit": "crops/s", "cores": threads,
                            "kind": "port", "cpu": cpu_model(), "cpus_available": avail, "cpu_quota": quota,
                            "sample": f"{done} crops of the same workload in batches of {bs} (torch-CPU fp32 "
                                      f"restatement, oracle/hgru_torch_cpu.py, {threads} threads), {cpu_s:.1f} s"}}
    if not args.no_parity:
        ref = np.concatenate(refs).astype(np.float64)
        got = out[:done].cpu().numpy().astype(np.float64)
        r64 = R.hgru_pose_forward(d[:2], wts, oo[:2], T, np.float64)
        res["parity"] = {"rel_inf_err": float(np.abs(got - ref).max() / np.abs(ref).max()),
                         "rel_inf_err_fp64_oracle": float(np.abs(got[:2] - r64).max() / np.abs(r64).max()),
                         "mean_joint_err_mm": R.mean_error(R.to_joints_mm(ref), R.to_joints_mm(got)),
                         "crops": done, "oracle": "torch-CPU fp32 (the CPU baseline run); float64 numpy oracle on 2",
                         "gate": 1e-4 if args.dtype != "bf16" else BF16_REL_TOL}
    return res


def launch_ranks(args) -> int:
    """``python bench.py --gpus N`` (N > 1) outside a torch.distributed launcher: start the N ranks
    as ``torch.distributed.run`` children (one process per GPU) and return their exit status.  Runs
    before anything touches the GPU -- this process only waits; it never initialises HIP."""
    import socket
    import subprocess
    with socket.socket() as s:   # a free rendezvous port on the loopback interface
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # the driver's scaling curve reads n_gpus from this line: a launch whose world differs from
        # --gpus (e.g. a launcher started with another --nproc-per-node) must not report either
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one rank per GPU; local % device_count only matters for --backend gloo rehearsals of the
        # multi-rank path with several ranks on one GPU (RCCL refuses two ranks per device)
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        # a bounded collective timeout: a rank that dies leaves the others failing, not hanging
        tmo = datetime.timedelta(seconds=300)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(args.backend, timeout=tmo)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {dist.get_world_size()} ranks")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    mp = importlib.import_module("monkey-pose_amd")
    W, par = mp.weights, mp.parallel
    B, crop, T = args.batch, args.crop, args.timesteps

    # ---- weights: generated on rank 0, ONE RCCL broadcast, packed per rank.  fp32: the flat fp32
    # blob; bf16: what a bf16 context reads (fc_1 as its f16 hi plane), half the bytes ----
    table = W.hgru_pose_vars(output_shape=69, timesteps=T, crop=crop)
    wts = {v.name: W.synth_value(v, 1234, T) for v in table} if rank == 0 else None
    binfo = {}
    flat, layout, bcast_s = par.broadcast_weights(table, wts, dev, rank, world,
                                                  dtype="bf16" if args.dtype == "bf16" else "fp32", info=binfo)
    ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, dev.index)
    par.load_context(ctx, flat, layout)
    ctx.finalize(mp._lib.dtype_code(args.dtype))
    del flat
    ctx.reserve(B)

    # ---- synthetic inputs resident in HBM (this rank's shard of the global batch) ----
    strong = args.global_batch is not None
    gb = args.global_batch if strong else world * B
    s0, s1 = par.shard_range(gb, rank, world) if strong else (rank * B, rank * B + B)
    B = s1 - s0
    if B <= 0:
        raise SystemExit("--global-batch must give every GPU at least one crop")
    depth = torch.from_numpy(W.synth_crops(B, seed=42 + rank, size=crop)).to(dev)
    o0 = torch.from_numpy(W.synth_hidden((B, crop // 2, crop // 2, 64), seed=7 + rank)).to(dev)
    out = torch.empty((B, 69), dtype=torch.float32, device=dev)
    stream = mp._lib.current_stream(dev)

    def timed(d, h, o, steps, warmup):
        """warmup, barrier + sync, `steps` forwards, sync + barrier; the max over ranks"""
        for _ in range(warmup):
            ctx.pose_fwd(d, h, o, stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.pose_fwd(d, h, o, stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    elapsed = timed(depth, o0, out, args.steps, args.warmup)
    # the other scaling reading of the metric, after the timed region (N > 1 only): the strong row
    # (global batch 256 sharded) next to a weak headline, or the weak row (256 per GPU) next to a
    # strong headline
    other = None
    if world > 1:
        if strong:
            ob = 256
        else:
            a0, a1 = par.shard_range(256, rank, world)
            ob = a1 - a0
        d2 = torch.from_numpy(W.synth_crops(ob, seed=142 + rank, size=crop)).to(dev)
        h2 = torch.from_numpy(W.synth_hidden((ob, crop // 2, crop // 2, 64), seed=107 + rank)).to(dev)
        o2 = torch.empty((ob, 69), dtype=torch.float32, device=dev)
        el2 = timed(d2, h2, o2, args.steps, 1)
        tot = world * 256 if strong else 256
        other = {"scaling": "weak" if strong else "strong", "global_batch": tot,
                 "per_gpu_batch": 256 if strong else f"{256 // world}-{-(-256 // world)}",
                 "value": round(tot * args.steps / el2, 3), "unit": "crops/s",
                 "ms_per_step": round(el2 / args.steps * 1e3, 3)}
        del d2, h2, o2
    # per-kernel HIP-event profile: a separate pass over the same inputs with profiling on.  The
    # timed pass runs the hGRU loop of the FFT path as two batch halves on two streams (their
    # kernels overlap); with profiling on the library keeps one stream, so each launch below is a
    # full-batch launch with its own duration (what the roofline and rocprof report).
    prof_steps = max(1, min(args.steps, 5))
    ctx.profile(True)
    for _ in range(prof_steps):
        ctx.pose_fwd(depth, o0, out, stream)
    torch.cuda.synchronize()
    ctx.profile(False)

    ms_a, na = ctx.profile_read("conv15_a")
    ms_b, nb = ctx.profile_read("conv15_b")
    ms_fc, nfc = ctx.profile_read("fc1")
    ms_bb, nbb = ctx.profile_read("backbone")
    conv_launch_ms = (ms_a + ms_b) / max(1, na + nb)
    px = (crop // 2) ** 2
    conv15_flop = 2.0 * px * 15 * 15 * 64 * 64 * B            # algorithmic, per launch
    achieved_tf = conv15_flop / (conv_launch_ms * 1e-3) / 1e12

    fft = args.dtype in ("f32_fft", "bf16")
    fft_loop = ctx.info("fft_loop")
    kern = fft_kernels(ctx, B, px, prof_steps, args.dtype == "bf16") if fft else None
    hbm_meas = hbm_rates(dev) if fft else None   # after the timed region
    value = gb * args.steps / elapsed
    dev_list = []
    if world > 1:   # which device each rank ran on (RCCL needs one rank per GPU; gloo rehearsals may share)
        dl = [None] * world
        dist.all_gather_object(dl, dev.index)
        dev_list = dl
    if strong:
        metric = (f"depth-crops/sec hGRU-8T fwd @global batch {gb} over {world} GPU (strong scaling, "
                  f"{crop}x{crop} crops)")
    else:
        metric = f"depth-crops/sec hGRU-8T fwd @batch{B} per GPU (weak scaling, {crop}x{crop} crops)"
    rec = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "crops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": {"f32": "f32", "f32_split": "f32 (f16x3 split MFMA, fp32 accumulate)",
                  "f32_fft": "f32 (fp32 FFT convolution, fp32-accurate f16x3 spectral GEMM)",
                  "bf16": "bf16 (bf16 spectra and hGRU maps, bf16 spectral / gate GEMMs, fp32 accumulate, fp32 FFTs and elementwise math)"}[args.dtype],
        "data": "synthetic crops + synthetic weights (splitmix64 stand-ins; reference publishes none)",
        "config": {"workload": f"hgru_pose.model.build fwd, T={T}, {crop}x{crop} crops, "
                               + (f"global batch {gb} sharded over {world} GPU" if strong else f"batch {B} per GPU"),
                   "global_batch": gb, "per_gpu_batch": B, "crop": crop,
                   "timesteps": T,
                   "parallelism": (f"dp{world} (contiguous batch shards, one {'RCCL' if args.backend == 'nccl' else 'gloo'} "
                                   "weight broadcast before timing, no collective in the timed region)") if world > 1
                   else "dp1 (single GPU, no collective)",
                   "hgru_streams": (int(os.environ.get("MP_STREAMS", "2")) if fft else 1),
                   "hgru_loop": {4: "four-step FFT loop (k_fft4.hip: 4 launches per timestep)",
                                 6: "six-launch FFT loop (k_fft.hip)", 0: "direct conv"}[fft_loop]},
        "roofline": (fft_roofline(kern, args.dtype == "bf16", B, hbm_meas) if fft else
                     roofline(args.dtype, achieved_tf, conv_launch_ms, na + nb, conv15_flop)),
        "breakdown_ms_per_step": {"conv15": round((ms_a + ms_b) / prof_steps, 3),
                                  "fc1": round(ms_fc / max(1, nfc), 3),
                                  "backbone": round(ms_bb / max(1, nbb), 3)},
        "ranks": dist.get_world_size() if world > 1 else 1,
        "backend": (dist.get_backend() if world > 1 else "none (one process)"),
        "devices": (dev_list if world > 1 else [dev.index]),
        "weight_bcast_ms": round(bcast_s * 1e3, 3),
        "weight_bcast_bytes": binfo.get("bytes"),
        "weight_bcast_form": binfo.get("form"),
    }
    if other:
        rec["other_scaling_row"] = other
    rec["src_sha"] = tree_stamp()
    if fft:
        rec["roofline"]["traffic_stamp"] = profile_stamp()
    if args.dtype == "f32_fft":
        mb = pmc_mfma_busy()
        if mb:
            rec["roofline"]["mfma_busy_pmc"] = mb
    if kern:
        rec["fft_kernels"] = kern
        pf = pmc_forward_bytes(args.dtype, B)
        if pf:
            rec["pmc_hbm_bytes_per_forward"] = pf
        # the direct 15x15 conv's FLOPs over the FFT path's time: a speed-up figure for the algorithm,
        # NOT an executed rate (the FFT path executes ~50x fewer FLOPs), so never read it against a peak
        rec["eCRF_direct_conv_flops_over_fft_time"] = {
            "value": round(achieved_tf, 2), "unit": "direct-conv TFLOP-equivalents/s",
            "note": "algorithmic 15x15 direct-conv FLOPs / FFT-path time; not executed FLOPs, not comparable to any MFMA peak"}

    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            rec.update(cpu_baseline(depth, o0, out, wts, T, args))
        if not args.no_extras:
            head_rate = value
            rec["extras"] = {}
            if args.dtype == "f32_fft":
                try:   # config 4's dtype (bf16) on the same crops at the same per-GPU batch
                    rec["extras"]["bf16_b256"] = bf16_leg(mp, dev, wts, depth, o0, T, hbm_meas)
                except Exception as e:  # noqa: BLE001
                    rec["extras"]["bf16_b256"] = {"error": repr(e)}
            try:
                rec["extras"]["e2e_batch1_latency"] = e2e_latency(mp, ctx, dev, T, wts, args.dtype)
            except Exception as e:  # noqa: BLE001
                rec["extras"]["e2e_batch1_latency"] = {"error": repr(e)}
            ctx.close()
            rec["extras"].update(extras(mp, dev, args))
            sp = rec["extras"].get("strong_scaling_per_gpu")
            if sp and not strong and B == 256:
                for k, v in sp.items():
                    if isinstance(v, dict):
                        v["efficiency"] = round(v["crops_per_s"] / head_rate, 3)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    _a = parse()
    if _a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's `python bench.py --gpus N`: one rank per GPU under torch.distributed.run
        sys.exit(launch_ranks(_a))
    try:
        main()
    except BaseException as exc:   # noqa: BLE001
        # any rank's failure fails the whole `bench.py --gpus N` job: report it and leave with a
        # non-zero status at once (no destroy_process_group, which could wait on the other ranks)
        if isinstance(exc, SystemExit) and exc.code in (0, None):
            raise
        import traceback
        traceback.print_exc()
        sys.stderr.write(f"bench.py: rank {os.environ.get('RANK', '0')} failed: {exc!r}\n")
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)
