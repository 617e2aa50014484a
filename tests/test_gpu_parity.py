"""GPU parity: the HIP path (through the C ABI via the reference-shaped facades) against the CPU
oracle and the committed golden vectors.  Tolerance: fp32 gate ||out-ref||_inf/||ref||_inf <= 1e-4
(SURVEY.md 8d); the integer / bit-level properties are exact."""
import numpy as np
import pytest

from helpers import BF16_REL_TOL, BF16_STATE_REL_TOL, FP32_REL_TOL, HGRU_POSE_AUX, MG, golden_array, golden_meta, pkg, rel_inf

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


DTYPES = ["fp32", "fp32_split", "fp32_fft"]


def _split_ok(h, w):
    return h % 32 == 0 and w % 32 == 0


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", [c[0] for c in MG.CIRCUIT_CASES])
def test_circuit_matches_oracle(case, dtype):
    from oracle import hgru_ref as R
    mp = pkg()
    meta = golden_meta()[case]
    n, h, w, ssf, T = meta["n"], meta["h"], meta["w"], meta["ssf"], meta["timesteps"]
    if dtype == "fp32_split" and not _split_ok(h, w):
        pytest.skip("split path tiles 32x32")
    wts, X, O0 = MG.circuit_inputs(n, h, w, ssf, T, meta["weight_seed"], meta["x_seed"], meta["o0_seed"])
    cc = mp.hgru_module.ContextualCircuit(_cuda(X), timesteps=T, SRF=1, SSN=ssf, SSF=ssf,
                                          aux=HGRU_POSE_AUX)
    O, weights, acts = cc.build(weights=wts, h2_init=_cuda(O0), compute_dtype=dtype)
    O = O.cpu().numpy()
    ref = golden_array(case, "O")
    assert rel_inf(O, ref) <= FP32_REL_TOL
    fresh = R.hgru_forward(X.astype(np.float64), O0, wts, T)
    assert rel_inf(O, fresh) <= FP32_REL_TOL
    assert set(weights) >= {"p_r", "i_r", "o_r", "rho", "p_t"}


def _pose(case, dtype="fp32"):
    mp = pkg()
    meta = golden_meta()[case]
    n, crop, T = meta["n"], meta["crop"], meta["timesteps"]
    wts, depth, O0 = MG.pose_inputs(n, crop, T, meta["weight_seed"], meta["crop_seed"], meta["o0_seed"])
    m = mp.hgru_pose.model()
    m.compute_dtype = dtype
    m.load_weights(wts)
    out = m.build(_cuda(depth), meta["output_shape"], train_mode=False, h2_init=_cuda(O0))
    torch.cuda.synchronize()
    return m, out.cpu().numpy(), wts, depth, O0


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", [c[0] for c in MG.POSE_CASES])
def test_pose_matches_golden(case, dtype):
    m, out, *_ = _pose(case, dtype)
    ref = golden_array(case, "out")
    assert out.shape == ref.shape
    err = rel_inf(out, ref)
    assert err <= FP32_REL_TOL, err


def test_pose_matches_fresh_oracle_and_metric():
    from oracle import hgru_ref as R
    m, out, wts, depth, O0 = _pose("pose_c64_t8")
    ref = R.hgru_pose_forward(depth, wts, O0, 8, np.float64)
    assert rel_inf(out, ref) <= FP32_REL_TOL
    # mean 3D joint error between the two paths in mm (getMeanError_train semantics)
    e = R.mean_error(R.to_joints_mm(ref), R.to_joints_mm(out))
    assert e < 0.1


@pytest.mark.parametrize("dtype", ["fp32", "fp32_fft"])
def test_pose_intermediates_match_oracle(dtype):
    """m.conv1 ... m.relu1 (hgru_pose.py:50-103), lazily on first access and eagerly with
    keep_intermediates=True; both leave out_put bit-identical."""
    from oracle import hgru_ref as R
    m, out, wts, depth, O0 = _pose("pose_c64_t8", dtype)
    ref, inter = R.hgru_pose_forward(depth, wts, O0, 8, np.float64, keep=True)
    want = {"conv1": inter["conv1"], "pool1": inter["pool1"], "conv2": inter["conv2"],
            "conv3": inter["conv3"], "hgru": inter["hgru_bn"], "fc1": inter["fc1"], "relu1": inter["relu1_bn"]}
    lazy = {k: getattr(m, k).cpu().numpy() for k in want}
    assert np.array_equal(m.out_put.cpu().numpy(), out)
    for k, v in want.items():
        assert lazy[k].shape == v.shape, k
        assert rel_inf(lazy[k], v) <= FP32_REL_TOL, k
    out2 = m.build(_cuda(depth), 69, h2_init=_cuda(O0), keep_intermediates=True).cpu().numpy()
    assert np.array_equal(out2, out)
    for k in want:
        assert np.array_equal(getattr(m, k).cpu().numpy(), lazy[k]), k


@pytest.mark.parametrize("n", [1, 33, 130])
@pytest.mark.parametrize("dtype", ["fp32_fft", "bf16"])
def test_fc1_presplit_planes_bit_identical(dtype, n):
    """fc_1 on the f16 hi / lo planes the last B epilogue writes (spec_epi_b mode 2 ->
    k_fc.hip fc_gemm_x3p_kernel, LDS-DMA staging) equals fc_1 on the fp32 map (the hgru-tap path,
    fc_gemm_x3_kernel's in-loop split) bit for bit: 32-, 64- and 128-row tiles, a partial tile."""
    mp = pkg()
    W = mp.weights
    crop = 64
    wts = W.synth_weights(W.hgru_pose_vars(crop=crop), seed=11)
    depth = W.synth_crops(n, seed=12, size=crop)
    O0 = W.synth_hidden((n, crop // 2, crop // 2, 64), seed=13)
    m = mp.hgru_pose.model()
    m.compute_dtype = dtype
    m.load_weights(wts)
    plain = m.build(_cuda(depth), 69, h2_init=_cuda(O0)).cpu().numpy()
    tapped = m.build(_cuda(depth), 69, h2_init=_cuda(O0), keep_intermediates=True).cpu().numpy()
    assert np.array_equal(plain, tapped)


@pytest.mark.parametrize("crop", [128, 64])
@pytest.mark.parametrize("dtype", DTYPES)
def test_batch_invariance_and_determinism(dtype, crop):
    """Each crop's output is bit-identical alone or inside a batch, and run to run.  For the FFT
    dtype a lone crop runs the small-batch 9-lane FFT kernels (k_fft.hip lfft_*, B <= 8) and the
    batch of 10 the batched ones, so this also pins those two kernel families to the same bits."""
    mp = pkg()
    W = mp.weights
    n = 10
    wts = W.synth_weights(W.hgru_pose_vars(crop=crop), seed=5)
    depth = W.synth_crops(n, seed=9, size=crop)
    O0 = W.synth_hidden((n, crop // 2, crop // 2, 64), seed=3)
    m = mp.hgru_pose.model()
    m.compute_dtype = dtype
    m.load_weights(wts)
    full = m.build(_cuda(depth), 69, h2_init=_cuda(O0)).cpu().numpy()
    again = m.forward(_cuda(depth), h2_init=_cuda(O0)).cpu().numpy()
    assert np.array_equal(full, again)
    for i in (0, 3, 9):
        one = m.forward(_cuda(depth[i:i + 1]), h2_init=_cuda(O0[i:i + 1])).cpu().numpy()
        assert np.array_equal(one[0], full[i])


@pytest.mark.parametrize("dtype", ["fp32_fft", "bf16"])
def test_backbone_small_batch_tiles_bit_identical(dtype):
    """Backbone conv_2 / conv_3 of batches <= 32 (at 64 x 64) run 8-row tiles with one 32-channel
    output block per workgroup (k_conv64x3.hip conv_small_tiles); a batch of 66 takes the 32-row
    tiles.  The conv2 / conv3 taps and the outputs of single crops and of a 20-crop slice equal
    their part of the batch bit for bit."""
    mp = pkg()
    W = mp.weights
    n, crop = 66, 128
    wts = W.synth_weights(W.hgru_pose_vars(crop=crop), seed=21)
    depth = W.synth_crops(n, seed=22, size=crop)
    O0 = W.synth_hidden((n, crop // 2, crop // 2, 64), seed=23)
    m = mp.hgru_pose.model()
    m.compute_dtype = dtype
    m.load_weights(wts)
    full = m.build(_cuda(depth), 69, h2_init=_cuda(O0), keep_intermediates=True).cpu().numpy()
    taps = {k: getattr(m, k).cpu().numpy() for k in ("conv2", "conv3")}
    for i in (0, 33, 65):
        one = m.build(_cuda(depth[i:i + 1]), 69, h2_init=_cuda(O0[i:i + 1]), keep_intermediates=True)
        for k, v in taps.items():
            assert np.array_equal(getattr(m, k).cpu().numpy()[0], v[i]), (k, i)
        assert np.array_equal(one.cpu().numpy()[0], full[i]), i
    part = m.build(_cuda(depth[40:60]), 69, h2_init=_cuda(O0[40:60]), keep_intermediates=True)
    for k, v in taps.items():
        assert np.array_equal(getattr(m, k).cpu().numpy(), v[40:60]), k
    assert np.array_equal(part.cpu().numpy(), full[40:60])


def test_rejects_training_and_bad_shapes():
    mp = pkg()
    m = mp.hgru_pose.model()
    x = torch.zeros((1, 128, 128, 1), device="cuda")
    with pytest.raises(NotImplementedError):
        m.build(x, 69, train_mode=True)
    m2 = mp.hgru_pose.model()
    with pytest.raises(Exception):
        m2.build(torch.zeros((1, 100, 100, 1), device="cuda"), 69)
    with pytest.raises(NotImplementedError):
        mp.hgru_module.ContextualCircuit(torch.zeros((1, 16, 32, 64), device="cuda"), timesteps=2,
                                         aux={'gru_gates': False})


def test_profile_counters():
    m, out, *_ = _pose("pose_c64_t8")
    m.profile(True)
    x = torch.from_numpy(MG.pose_inputs(2, 64, 8, 1234, 42, 7)[1]).cuda()
    m.forward(x)
    ms_a, na = m.profile_read("conv15_a")
    ms_b, nb = m.profile_read("conv15_b")
    assert na == 8 and nb == 8 and ms_a > 0 and ms_b > 0


def test_split_precision_is_fp32_class():
    """The f16x3 split path stays within a few fp32 ulps of the exact fp32 path."""
    _, a, *_ = _pose("pose_c128_t8", "fp32")
    _, b, *_ = _pose("pose_c128_t8", "fp32_split")
    ref = golden_array("pose_c128_t8", "out")
    ea, eb = rel_inf(a, ref), rel_inf(b, ref)
    print(f"rel_inf err: fp32 {ea:.3e}  fp32_split {eb:.3e}  (split vs fp32 {rel_inf(b, a):.3e})")
    assert eb <= max(10 * ea, 2e-6)




@pytest.mark.parametrize("case", [c[0] for c in MG.POSE_CASES])
def test_bf16_pose_within_bf16_gate(case):
    m, out, *_ = _pose(case, "bf16")
    ref = golden_array(case, "out")
    err = rel_inf(out, ref)
    print(f"bf16 {case}: rel_inf {err:.3e}")
    assert err <= BF16_REL_TOL, err
    # the façade's dtype kwarg selects the same path
    m2 = pkg().hgru_pose.model()
    m2.load_weights(m.weights)
    meta = golden_meta()[case]
    _, depth, O0 = MG.pose_inputs(meta["n"], meta["crop"], 8, meta["weight_seed"], meta["crop_seed"], meta["o0_seed"])
    out2 = m2.build(_cuda(depth), 69, h2_init=_cuda(O0), dtype="bf16").cpu().numpy()
    assert np.array_equal(out2, out)


@pytest.mark.parametrize("case", [c[0] for c in MG.CIRCUIT_CASES])
def test_bf16_circuit_within_bf16_gate(case):
    mp = pkg()
    meta = golden_meta()[case]
    n, h, w, ssf, T = meta["n"], meta["h"], meta["w"], meta["ssf"], meta["timesteps"]
    wts, X, O0 = MG.circuit_inputs(n, h, w, ssf, T, meta["weight_seed"], meta["x_seed"], meta["o0_seed"])
    cc = mp.hgru_module.ContextualCircuit(_cuda(X), timesteps=T, SRF=1, SSN=ssf, SSF=ssf, aux=HGRU_POSE_AUX)
    O, _, _ = cc.build(weights=wts, h2_init=_cuda(O0), compute_dtype="bf16")
    err = rel_inf(O.cpu().numpy(), golden_array(case, "O"))
    print(f"bf16 {case}: rel_inf {err:.3e}")
    assert err <= BF16_STATE_REL_TOL, err


@pytest.mark.parametrize("dtype", ["fp32_fft", "bf16"])
def test_stream_split_is_bit_identical(dtype):
    """The FFT path runs the hGRU loop as batch slices on two streams unless profiling is on; both
    schedules give the same bits (every reduction is per crop), run after run.  (The op_sel form of
    the packed FFT arithmetic, k_fft.hip FFT_PACKED = 1, failed exactly this at n = 256: 13-19 crops
    differed between two-stream runs.)"""
    mp = pkg()
    W = mp.weights
    n = 256
    ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
    for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128):
        ctx.set_weight(v.name, W.synth_value(v, 1234, 8))
    ctx.finalize(mp._lib.dtype_code(dtype))
    depth = _cuda(W.synth_crops(n, seed=3, size=128))
    o0 = _cuda(W.synth_hidden((n, 64, 64, 64), seed=4))
    st = mp._lib.current_stream(torch.device("cuda:0"))
    a = torch.empty((n, 69), device="cuda")
    b = torch.empty((n, 69), device="cuda")
    ctx.pose_fwd(depth, o0, a, st)
    for _ in range(2):
        c = torch.empty((n, 69), device="cuda")
        ctx.pose_fwd(depth, o0, c, st)
        assert torch.equal(a, c)
    ctx.profile(True)
    ctx.pose_fwd(depth, o0, b, st)
    ctx.profile(False)
    assert torch.equal(a, b)
    one = torch.empty((1, 69), device="cuda")
    ctx.pose_fwd(depth[70:71].contiguous(), o0[70:71].contiguous(), one, st)
    assert torch.equal(one[0], a[70])


def test_fft_precision_is_fp32_class():
    """The FFT path (fp32 72-point FFTs + fp32 spectral GEMM) stays fp32-class: its error against
    the float64 golden output is within a small multiple of the exact fp32 direct path's."""
    _, a, *_ = _pose("pose_c128_t8", "fp32")
    _, b, *_ = _pose("pose_c128_t8", "fp32_fft")
    ref = golden_array("pose_c128_t8", "out")
    ea, eb = rel_inf(a, ref), rel_inf(b, ref)
    print(f"rel_inf err: fp32 {ea:.3e}  fp32_fft {eb:.3e}  (fft vs fp32 {rel_inf(b, a):.3e})")
    assert eb <= max(10 * ea, 1e-5)


@pytest.mark.parametrize("n,dtype", [(32, "fp32_fft"), (64, "fp32_fft"), (128, "fp32_fft"), (300, "fp32_fft"),
                                     (1024, "fp32_fft"), (256, "bf16")])
def test_full_size_properties(n, dtype):
    """BASELINE config 2 (B = 64, train_cnn_networks_hgru.py:141-142) and the per-GPU batches of the
    metric's strong-scaling reading (256 / N = 128, 64, 32), and beyond the metric's batch (ragged
    300 = 9 GEMM groups + 12, and 1024).  The hGRU loop runs as batch slices on two streams from
    64 crops on (mp_abi.hip run_circuit: 32 + 32 at B = 64, 64 + 64 at B = 128; one slice at 32).
    Every sampled crop is bit-identical to its own batch-1 run (slices, streams and GEMM groups
    never mix crops), the whole batch is finite, and the last crop of EACH slice matches the
    float64 oracle within the fp32 gate.  bf16 at 256: BASELINE config 4's per-GPU batch (2,048
    over 8 GPUs), against the oracle within the bf16 gate."""
    from oracle import hgru_ref as R
    mp = pkg()
    W = mp.weights
    ctx = mp._lib.Context(mp._lib.MP_MODEL_HGRU_POSE, 0)
    wts = {v.name: W.synth_value(v, 1234, 8) for v in W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128)}
    for k, v in wts.items():
        ctx.set_weight(k, v)
    ctx.finalize(mp._lib.dtype_code(dtype))
    depth_np = W.synth_crops(n, seed=21, size=128)
    o0_np = W.synth_hidden((n, 64, 64, 64), seed=22)
    depth, o0 = _cuda(depth_np), _cuda(o0_np)
    st = mp._lib.current_stream(torch.device("cuda:0"))
    out = torch.empty((n, 69), device="cuda")
    ctx.pose_fwd(depth, o0, out, st)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(out).all())
    one = torch.empty((1, 69), device="cuda")
    # the two-slice split at these sizes: whole 32-crop GEMM groups, the first slice takes the
    # larger half (mp_abi.hip run_circuit)
    groups = (n + 31) // 32
    first = min(n, ((groups + 1) // 2) * 32) if n >= 64 else n
    for i in sorted({0, first - 1, first % n, n // 2, n - 1}):
        ctx.pose_fwd(depth[i:i + 1].contiguous(), o0[i:i + 1].contiguous(), one, st)
        torch.cuda.synchronize()
        assert torch.equal(one[0], out[i]), i
    idx = sorted({first - 1, n - 1})
    ref = R.hgru_pose_forward(depth_np[idx], wts, o0_np[idx], 8, np.float64)
    err = rel_inf(out[idx].cpu().numpy(), ref)
    print(f"n={n} {dtype}: crops {idx} vs fp64 oracle rel_inf {err:.3e}")
    assert err <= (BF16_REL_TOL if dtype == "bf16" else FP32_REL_TOL)


def test_hbm_probe_reports_plausible_rates():
    """mp_hbm_probe (bench.py's practical roof): read / write / copy of 64 MiB buffers on this GPU,
    each between 1 TB/s and the chip's ~10 TB/s ceiling, with the access form that reached it."""
    r = pkg()._lib.hbm_probe(0, 64 << 20)
    for k in ("read", "write", "copy"):
        assert 1000.0 < r[f"{k}_GBps"] < 12000.0, r
        f = r[f"{k}_form"]
        assert f["grid"] in (1024, 2048, 4096, 8192) and f["per_thread"] in (1, 4, 8)
    with pytest.raises(pkg()._lib.MonkeyPoseError):
        pkg()._lib.hbm_probe(0, 1 << 20)   # below the 64 MiB floor
