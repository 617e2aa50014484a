"""Attention CoM regressor (train_cnn_networks_hgru.py:422-525) and the device crop of
prepare_data_test (61-74): the frame -> CoM -> crop -> pose chain of test_model (284-321).

CPU: the oracle's TF1 bilinear resize against a direct per-pixel restatement and known values,
the oracle chain against the golden fixture, the native host batch crop against the oracle.
GPU: resize bit-exact, attention within the fp32 gate, device crop bit-exact (patches, M, CoM)
with the host crop and the oracle, including frames whose crop fails, and the whole chain."""
import numpy as np
import pytest

from helpers import FP32_REL_TOL, MG, golden_array, golden_meta, pkg, rel_inf
from oracle import crop_ref as CR
from oracle import regressors_ref as RR

SCALE = np.array([424.0, 512.0, 10000.0])


def _resize_loop(x, oh, ow):
    """Per-pixel restatement of TF1's legacy bilinear kernel (float32 scalars)."""
    f32 = np.float32
    n, h, w, c = x.shape
    hs, ws = f32(h) / f32(oh), f32(w) / f32(ow)
    out = np.empty((n, oh, ow, c), np.float32)
    for oy in range(oh):
        iy = f32(oy) * hs
        y0, y1 = max(int(np.floor(iy)), 0), min(int(np.ceil(iy)), h - 1)
        ly = f32(iy - f32(np.floor(iy)))
        for ox in range(ow):
            ix = f32(ox) * ws
            x0, x1 = max(int(np.floor(ix)), 0), min(int(np.ceil(ix)), w - 1)
            lx = f32(ix - f32(np.floor(ix)))
            tl, tr, bl, br = x[:, y0, x0], x[:, y0, x1], x[:, y1, x0], x[:, y1, x1]
            top = tl + (tr - tl) * lx
            bot = bl + (br - bl) * lx
            out[:, oy, ox] = top + (bot - top) * ly
    return out


def test_resize_oracle_matches_loop_and_known_values():
    rng = np.random.default_rng(0)
    for (h, w, oh, ow) in ((13, 17, 5, 7), (5, 6, 11, 9), (424, 512, 16, 16), (8, 8, 8, 8)):
        x = rng.standard_normal((2, h, w, 2)).astype(np.float32)
        assert np.array_equal(RR.resize_bilinear_tf1(x, oh, ow), _resize_loop(x, oh, ow))
    # identity size is a copy; 2x upsampling of a ramp interpolates midpoints, clamps the edge
    x = rng.standard_normal((1, 9, 9, 1)).astype(np.float32)
    assert np.array_equal(RR.resize_bilinear_tf1(x, 9, 9), x)
    r = np.arange(4, dtype=np.float32).reshape(1, 1, 4, 1).repeat(2, axis=1)
    up = RR.resize_bilinear_tf1(r, 2, 8)[0, 0, :, 0]
    assert np.array_equal(up, np.array([0, .5, 1, 1.5, 2, 2.5, 3, 3], np.float32))
    # 424 -> 128 uses scale 3.3125 exactly: row 1 samples rows 3 / 4 at lerp 0.3125
    col = np.arange(424, dtype=np.float32).reshape(1, 424, 1, 1)
    assert RR.resize_bilinear_tf1(col, 128, 1)[0, 1, 0, 0] == np.float32(3.3125)


def test_attn_oracle_matches_golden():
    m = golden_meta()["attn_f424"]
    wts, frames = MG.attn_inputs(m["n"], m["h"], m["w"], m["weight_seed"], m["frame_seed"])
    out = RR.attn_forward(frames, wts)
    assert rel_inf(out, golden_array("attn_f424", "out")) < 1e-9
    patches, Ms, coms = CR.prepare_data_test(frames, out.astype(np.float32), CR.MonkeyDetectorRef())
    assert np.array_equal(patches, golden_array("attn_f424", "patches"))
    assert np.array_equal(Ms, golden_array("attn_f424", "Ms"))
    assert np.array_equal(coms, golden_array("attn_f424", "coms"))


def test_attn_var_table_matches_reference_layout():
    W = pkg().weights
    table = W.attn_vars()
    names = [v.name for v in table]
    assert names[0] == "cnn/aconv_1/aconv_1_filters" and names[-1] == "cnn/afc_out/afc_out_biases"
    assert sum(1 for n in names if n.endswith("moving_variance")) == 6
    shapes = {v.name: v.shape for v in table}
    assert shapes["cnn/aconv_5/aconv_5_filters"] == (5, 5, 512, 1024)
    assert shapes["cnn/afc_1/afc_1_weights"] == (16384, 1024)
    assert shapes["cnn/batch_normalization_5/gamma"] == (1024,)


def _com_cases(n_extra=0):
    """Attention-like normalised CoMs: centre, near each border (padding), partly off-frame,
    near / far depth; the last rows hit the failure statuses (zero depth, negative depth)."""
    good = [(0.5, 0.5, 0.15), (0.02, 0.5, 0.12), (0.98, 0.97, 0.2), (0.5, 0.01, 0.09),
            (1.15, 0.6, 0.15), (-0.1, 0.4, 0.3), (0.31, 0.77, 0.5123), (0.6, 0.3, 0.0731)]
    bad = [(0.5, 0.5, 0.0), (0.5, 0.5, -0.15)]
    return np.array(good, np.float32), np.array(bad, np.float32)


def test_host_batch_crop_matches_oracle_prepare_data_test():
    """The native host batch crop (numpy path of prepare_data_test) against the oracle."""
    T = pkg().train_cnn_networks_hgru
    md = pkg().monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    good, _ = _com_cases()
    frames = pkg().weights.synth_frames(len(good), seed=5)
    patches, coms, Ms = T.prepare_data_test(frames, good, md, T.InferenceConfig())
    rp, rM, rc = CR.prepare_data_test(frames, good, CR.MonkeyDetectorRef())
    assert np.array_equal(patches[..., 0], rp)
    assert np.array_equal(np.stack([np.asarray(m) for m in Ms]), rM) and np.array_equal(np.stack(coms), rc)


# ------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_resize_gpu_bit_exact():
    torch = pytest.importorskip("torch")
    lib = pkg()._lib
    rng = np.random.default_rng(1)
    for (h, w, c, oh, ow) in ((424, 512, 1, 128, 128), (13, 17, 3, 5, 7), (5, 6, 2, 11, 9), (64, 64, 1, 64, 64)):
        x = rng.standard_normal((3, h, w, c)).astype(np.float32)
        got = lib.resize_bilinear(torch.from_numpy(x).cuda(), (oh, ow)).cpu().numpy()
        assert np.array_equal(got, RR.resize_bilinear_tf1(x, oh, ow)), (h, w, c, oh, ow)


def _attn_model(wts, dtype="auto"):
    m = pkg().train_cnn_networks_hgru.attn_model_struct()
    m.compute_dtype = dtype
    m.load_weights(wts)
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "fp32_split"])
def test_attn_gpu_matches_golden_and_oracle(dtype):
    torch = pytest.importorskip("torch")
    m = golden_meta()["attn_f424"]
    wts, frames = MG.attn_inputs(m["n"], m["h"], m["w"], m["weight_seed"], m["frame_seed"])
    model = _attn_model(wts, dtype)
    out = model.build(torch.from_numpy(frames).cuda(), 3, train_mode=False).cpu().numpy()
    assert rel_inf(out, golden_array("attn_f424", "out")) <= FP32_REL_TOL
    # batch invariance: one frame alone gives the same bits as inside the batch
    one = model.forward(torch.from_numpy(frames[1:2]).cuda()).cpu().numpy()
    assert np.array_equal(one[0], out[1])
    # a plain glorot draw (no calibration), intermediate activations large: still within the gate
    W = pkg().weights
    wts2 = W.synth_weights(W.attn_vars(), seed=3)
    fr2 = W.synth_frames(3, seed=8)
    out2 = _attn_model(wts2, dtype).build(torch.from_numpy(fr2).cuda(), 3).cpu().numpy()
    assert rel_inf(out2, RR.attn_forward(fr2, wts2)) <= FP32_REL_TOL
    # already 128 x 128 input: the resize is skipped (identity in TF as well)
    fr3 = W.synth_frames(2, seed=9, h=128, w=128)
    out3 = _attn_model(wts2, dtype).build(torch.from_numpy(fr3).cuda(), 3).cpu().numpy()
    assert rel_inf(out3, RR.attn_forward(fr3, wts2)) <= FP32_REL_TOL


@pytest.mark.gpu
def test_attn_rejects_training_mode():
    torch = pytest.importorskip("torch")
    m = pkg().train_cnn_networks_hgru.attn_model_struct()
    with pytest.raises(NotImplementedError):
        m.build(torch.zeros((1, 424, 512, 1), device="cuda"), 3, train_mode=True)


@pytest.mark.gpu
def test_device_crop_bit_exact_with_host_and_oracle():
    torch = pytest.importorskip("torch")
    P = pkg()
    md = P.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    good, bad = _com_cases()
    frames = P.weights.synth_frames(len(good), seed=5)
    fd = torch.from_numpy(frames).cuda()
    patches, Ms, coms = md.crop_batch_device(fd, torch.from_numpy(good).cuda())
    rp, rM, rc = CR.prepare_data_test(frames, good, CR.MonkeyDetectorRef())
    assert np.array_equal(patches.cpu().numpy()[..., 0], rp)
    assert np.array_equal(Ms.cpu().numpy(), rM)
    assert np.array_equal(coms.cpu().numpy(), rc)
    # the host native crop on the same inputs (shared geometry code, independent sampling loop)
    hp, hM, hc = md.crop_batch(frames[..., 0] * np.float32(10000), coms=good.astype(np.float32) * SCALE)
    assert np.array_equal(patches.cpu().numpy(), hp)
    # failing frames: status per frame, the good ones unaffected, and check=True raises
    allc = np.concatenate([good[:2], bad])
    fr4 = P.weights.synth_frames(len(allc), seed=6)
    p4, _, _ = md.crop_batch_device(torch.from_numpy(fr4).cuda(), torch.from_numpy(allc).cuda(), check=False)
    st = md.last_status.cpu().numpy()
    assert st[0] == 0 and st[1] == 0 and st[2] == 1 and st[3] != 0
    rp4, _, _ = CR.prepare_data_test(fr4[:2], allc[:2], CR.MonkeyDetectorRef())
    assert np.array_equal(p4.cpu().numpy()[:2, ..., 0], rp4)
    assert np.all(p4.cpu().numpy()[2:] == 1.0)
    with pytest.raises(P._lib.MonkeyPoseError):
        md.crop_batch_device(torch.from_numpy(fr4).cuda(), torch.from_numpy(allc).cuda())


@pytest.mark.gpu
def test_frame_pose_chain_matches_oracle():
    """test_model's batch body: attention -> device crop -> hGRU pose.  The crop is compared
    bit-exactly on the GPU's own CoM (a 1-ulp CoM change may move an integer bound), the pose
    output within the fp32 gate of the oracle run on those patches."""
    torch = pytest.importorskip("torch")
    from oracle import hgru_ref as R
    P = pkg()
    T = P.train_cnn_networks_hgru
    m = golden_meta()["attn_f424"]
    wts, frames = MG.attn_inputs(m["n"], m["h"], m["w"], m["weight_seed"], m["frame_seed"])
    attn = _attn_model(wts)
    pose = P.hgru_pose.model()
    pm = golden_meta()["pose_c128_t8"]
    pw, _, _ = MG.pose_inputs(pm["n"], pm["crop"], 8, pm["weight_seed"], pm["crop_seed"], pm["o0_seed"])
    pose.load_weights(pw)
    md = P.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    pipe = T.FramePosePipeline(attn, pose, md)
    n = frames.shape[0]
    O0 = P.weights.synth_hidden((n, 64, 64, 64), seed=7)
    out, coms, Ms = pipe.run(torch.from_numpy(frames).cuda(), h2_init=torch.from_numpy(O0).cuda())
    com_norm = attn.out_put.cpu().numpy()
    rp, rM, rc = CR.prepare_data_test(frames, com_norm, CR.MonkeyDetectorRef())
    assert np.array_equal(coms.cpu().numpy(), rc) and np.array_equal(Ms.cpu().numpy(), rM)
    ref = R.hgru_pose_forward(rp[..., None], pw, O0, 8, np.float64)
    assert rel_inf(out.cpu().numpy(), ref) <= FP32_REL_TOL
