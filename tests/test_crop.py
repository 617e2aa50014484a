"""A20 host crop (monkeydetector.py:66-334) and A19 geometry: the native crop (libmonkeypose.so,
host C++) against the numpy oracle.  Integer bounds / sizes / offsets and every crop pixel are
bit-exact; M within 1e-12 (the reference builds it with a BLAS matmul whose FMA use is unpinned).
Runs on the CPU (the crop is host code, no GPU call)."""
import math

import numpy as np
import pytest

from helpers import pkg
from oracle import crop_ref as CR

CAM = (365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)   # train_cnn_networks_hgru.py:77


def _mds():
    return pkg().monkeydetector.MonkeyDetector(*CAM), CR.MonkeyDetectorRef()


def _coms(n, seed):
    """CoMs across the frame, including near / past the borders and near / far depths."""
    rng = np.random.default_rng(seed)
    u = rng.uniform(-40, 552, n)
    v = rng.uniform(-40, 464, n)
    d = rng.uniform(500, 4000, n)
    return np.stack([u, v, d], 1)


def test_pairwise_sum_restatement():
    """The classic numpy pairwise float32 sum (the reference era's dc.sum()) agrees with this
    numpy's own 1-D float32 sum; on 2-D frames numpy 2.x may differ in the last place."""
    rng = np.random.default_rng(0)
    for n in (1, 7, 8, 9, 127, 128, 129, 1000, 4097, 70001):
        a = (rng.random(n) * 1e4).astype(np.float32)
        assert CR.np_pairwise_sum_f32(a) == a.sum()
    f = CR.synth_frame(3)
    assert abs(float(CR.np_pairwise_sum_f32(f)) - float(f.astype(np.float64).sum())) < 1e3


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_crop_bit_exact_against_oracle(seed):
    md, ref = _mds()
    frame = CR.synth_frame(seed)
    for com in _coms(20, seed):
        got, M, c = md.cropArea3D(frame, com=com)
        exp, Mr, cr, info = ref.cropArea3D(frame, com=com)
        assert md.last_crop_info["bounds"] == info["bounds"]
        assert md.last_crop_info["sz"] == tuple(info["sz"])
        assert md.last_crop_info["offset"] == info["offset"]
        assert got.dtype == np.float32 and np.array_equal(got, exp), com
        assert np.allclose(np.asarray(M), Mr, rtol=1e-12, atol=1e-9)
        assert np.array_equal(c, cr)


@pytest.mark.parametrize("seed", [4, 5])
def test_crop_with_computed_com(seed):
    md, ref = _mds()
    frame = CR.synth_frame(seed)
    com = md.calculateCoM(frame)
    com_ref = ref.calculateCoM(frame)
    # mean row/col: exact; depth: numpy float32 pairwise sum restated (see test above)
    assert com[0] == com_ref[0] and com[1] == com_ref[1]
    s = CR.np_pairwise_sum_f32(np.where((frame >= 200) & (frame <= 10000), frame, 0).astype(np.float32))
    assert com[2] == float(s) / np.count_nonzero((frame >= 200) & (frame <= 10000))
    got, M, c = md.cropArea3D(frame)           # com=None path
    exp, Mr, cr, _ = ref.cropArea3D(frame, com=c)
    assert np.array_equal(got, exp)


def test_uint16_frames_follow_numpy_semantics():
    md, ref = _mds()
    frame = CR.synth_frame(6).astype(np.uint16)
    com = md.calculateCoM(frame)
    assert np.array_equal(com, ref.calculateCoM(frame))       # exact integer sum for uint16
    for c in _coms(10, 6):
        got, M, _ = md.cropArea3D(frame, com=c)
        exp, _, _, _ = ref.cropArea3D(frame, com=c)             # near-plane clamp truncates
        assert np.array_equal(got, exp)


def test_batch_matches_single_and_normalises():
    md, ref = _mds()
    frames = np.stack([CR.synth_frame(s) for s in (7, 8, 9)])
    coms = _coms(3, 11)
    coms[:, 0] = np.clip(coms[:, 0], 100, 400)
    patches, Ms, c = md.crop_batch(frames, coms, nthreads=3)
    for i in range(3):
        single, M, _ = md.cropArea3D(frames[i], com=coms[i])
        assert np.array_equal(patches[i, :, :, 0], single / np.float32(10000))   # train_cnn_networks_hgru.py:71
        assert np.array_equal(Ms[i], np.asarray(M))
    # out=: the patches land in the caller's buffer (StreamPosePipeline's reused staging array)
    buf = np.full((3, 128, 128, 1), np.nan, np.float32)
    p2, Ms2, c2 = md.crop_batch(frames, coms, nthreads=2, out=buf)
    assert p2 is buf and np.array_equal(buf, patches) and np.array_equal(Ms2, Ms) and np.array_equal(c2, c)
    with pytest.raises(ValueError):
        md.crop_batch(frames, coms, out=np.empty((3, 128, 128), np.float32))


def test_crop_errors():
    md, _ = _mds()
    with pytest.raises(Exception):
        md.cropArea3D(np.zeros((424, 512), np.float32))          # no valid pixel -> CoM depth 0
    # docom=True is implemented (monkeydetector.py:287-300; fixtures in test_crop_reference.py)
    crop, _, com = md.cropArea3D(CR.synth_frame(1), com=(256, 212, 1000), docom=True)
    exp, _, cr, _ = CR.MonkeyDetectorRef().cropArea3D(CR.synth_frame(1), com=np.array([256., 212, 1000]),
                                                      docom=True)
    assert np.array_equal(crop, exp) and np.array_equal(com, cr)


def test_relative_absolute_round_trip():
    """sample_pipeline.py:15-42: crop -> relative -> absolute recovers the joints."""
    md, ref = _mds()
    rng = np.random.default_rng(0)
    jnts_xyz = np.c_[rng.uniform(-300, 300, 23), rng.uniform(-300, 300, 23), -rng.uniform(900, 1600, 23)]
    jnts_uvd = md.xyztouvd(jnts_xyz)
    assert np.allclose(jnts_uvd, ref.xyztouvd(jnts_xyz), rtol=1e-6)
    com_uvd = md.calcCoMRenders(jnts_uvd)
    frame = CR.synth_frame(2)
    _, M, com = md.cropArea3D(frame, com=com_uvd)
    rel_xyz, rel_uvd = md.getRelativeCoordinates(jnts_xyz, jnts_uvd, com_uvd, M)
    r2, u2 = ref.getRelativeCoordinates(jnts_xyz, jnts_uvd, com_uvd, np.asarray(M))
    assert np.allclose(rel_xyz, r2) and np.allclose(rel_uvd, u2, rtol=1e-6, atol=1e-4)
    back_xyz, back_uvd = md.getAbsoluteCoordinates(rel_xyz, com_uvd)
    assert np.allclose(back_xyz, jnts_xyz, atol=1e-3)
    assert np.allclose(back_uvd, jnts_uvd, rtol=1e-5, atol=1e-3)


def test_absolute_fast_path_is_the_general_path():
    """getAbsoluteCoordinates' one-joint-set path (float32 [n, 3] joints, one CoM: the config-5 loop)
    returns the bytes of the general uvdtoxyz / xyztouvd composition, for float64 and float32 CoMs
    and with a joint at z == 0 (the principal-point branch)."""
    md, _ = _mds()
    rng = np.random.default_rng(3)
    for com_dtype in (np.float64, np.float32):
        for zero in (False, True):
            rel = rng.uniform(-300, 300, (23, 3)).astype(np.float32)
            com = np.array([rng.uniform(100, 400), rng.uniform(100, 300), rng.uniform(800, 2000)], com_dtype)
            if zero:
                rel[5, 2] = -np.float32(md.uvdtoxyz(com)[2])
            a_xyz, a_uvd = md.getAbsoluteCoordinates(rel, com)
            e_xyz = rel + md.uvdtoxyz(com)
            e_uvd = md.xyztouvd(e_xyz)
            assert a_xyz.dtype == e_xyz.dtype and np.array_equal(a_xyz, e_xyz)
            assert a_uvd.dtype == e_uvd.dtype and np.array_equal(a_uvd, e_uvd)
            if zero:
                assert a_xyz[5, 2] == 0 and a_uvd[5, 0] == np.float32(md.ux)
