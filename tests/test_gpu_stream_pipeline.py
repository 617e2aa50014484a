"""SURVEY config 5 product class (train_cnn_networks_hgru.StreamPosePipeline): one depth frame ->
native host CoM crop into the reused staging buffer -> hGRU pose forward at batch 1 -> absolute
joints.  Its result must be the same bits as the façade chain it replaces (crop_batch ->
hgru_pose.model().build -> getAbsoluteCoordinates, train_cnn_networks_hgru.py:284-321), for both the
pageable (default) and the pinned staging, and over repeated calls (the buffers are reused)."""
import numpy as np
import pytest
import torch

from helpers import pkg
from oracle import crop_ref as CR

CAM = (365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_stream_pipeline_matches_facade_chain(pinned):
    mp = pkg()
    W = mp.weights
    dev = torch.device("cuda", 0)
    md = mp.monkeydetector.MonkeyDetector(*CAM)
    wts = W.synth_weights(W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128), seed=21)
    o0 = torch.from_numpy(W.synth_hidden((1, 64, 64, 64), seed=3)).to(dev)
    pm = mp.hgru_pose.model()
    pm.load_weights(wts)
    pm.build(torch.zeros((1, 128, 128, 1), device=dev), 69, h2_init=o0)
    pipe = mp.train_cnn_networks_hgru.StreamPosePipeline(pm, md, h2_init=o0, pinned=pinned)
    for seed, com in ((1, None), (2, (250.0, 200.0, 1500.0)), (1, None)):
        frame = CR.synth_frame(seed)
        xyz, uvd, c = pipe.run(frame, com)
        patches, _, coms = md.crop_batch(frame[None], None if com is None else [com])
        out = pm.build(torch.from_numpy(patches).to(dev), 69, h2_init=o0).cpu().numpy()
        rel = out.reshape(23, 3) * np.float32(md.cube[2] / 2.0)
        xyz_e, uvd_e = md.getAbsoluteCoordinates(rel, coms[0])
        assert np.array_equal(c, coms[0])
        assert np.array_equal(np.asarray(xyz), np.asarray(xyz_e)) and np.array_equal(np.asarray(uvd), np.asarray(uvd_e))


@pytest.mark.gpu
def test_stream_pipeline_matches_oracle_chain():
    """The same pipeline against an independent chain built from the oracle alone: the numpy
    restatement of cropArea3D (oracle/crop_ref.py, monkeydetector.py:177-334) -> crop / maxDepth
    (train_cnn_networks_hgru.py:61-74) -> the float64 hGRU pose forward (oracle/hgru_ref.py,
    hgru_pose.py:47-105) -> getAbsoluteCoordinates (monkeydetector.py).  The crop must be bit-exact
    and the CoM equal; the joints within the fp32 gate (||out - ref||_inf / ||ref||_inf <= 1e-4 on the
    network output) and 0.1 mm on the absolute joints."""
    from oracle import hgru_ref as R
    mp = pkg()
    W = mp.weights
    dev = torch.device("cuda", 0)
    md = mp.monkeydetector.MonkeyDetector(*CAM)
    ref_md = CR.MonkeyDetectorRef(*CAM)
    wts = W.synth_weights(W.hgru_pose_vars(output_shape=69, timesteps=8, crop=128), seed=21)
    o0_np = W.synth_hidden((1, 64, 64, 64), seed=3)
    o0 = torch.from_numpy(o0_np).to(dev)
    pm = mp.hgru_pose.model()
    pm.load_weights(wts)
    pm.build(torch.zeros((1, 128, 128, 1), device=dev), 69, h2_init=o0)
    pipe = mp.train_cnn_networks_hgru.StreamPosePipeline(pm, md, h2_init=o0)
    frame = CR.synth_frame(5)
    xyz, uvd, c = pipe.run(frame, None)
    crop, _, com_ref, _ = ref_md.cropArea3D(frame, None, (128, 128))
    patches, _, coms = md.crop_batch(frame[None], None)
    assert np.array_equal(coms[0], np.asarray(com_ref, np.float64)) and np.array_equal(c, coms[0])
    depth = (crop / np.float32(ref_md.maxDepth)).astype(np.float32)[None, :, :, None]
    assert np.array_equal(patches, depth)
    ref = R.hgru_pose_forward(depth, wts, o0_np, 8, np.float64)
    out = pm.build(torch.from_numpy(patches).to(dev), 69, h2_init=o0).cpu().numpy()
    assert np.abs(out - ref).max() / np.abs(ref).max() <= 1e-4
    rel = (ref.reshape(23, 3) * (ref_md.cube[2] / 2.0)).astype(np.float32)
    xyz_ref, uvd_ref = ref_md.getAbsoluteCoordinates(rel, com_ref)
    assert np.abs(np.asarray(xyz) - xyz_ref).max() < 0.1
    assert np.abs(np.asarray(uvd)[:, 2] - uvd_ref[:, 2]).max() < 0.1
