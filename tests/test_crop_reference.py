"""A19 / A20 against the reference's OWN numpy code, executed here (tests/golden/make_crop_fixtures.py):
``calculateCoM``, ``comToBounds``, ``getCrop``, ``cropArea3D`` (both ``docom`` branches),
``xyztouvd_np`` / ``uvdtoxyz`` / ``getAbsoluteCoordinates`` / ``getRelativeCoordinates``,
``prepare_data_test`` and ``getMeanError_np``, with the NumPy 1.x promotion rules of the era
patched in explicitly by the generator.  Only cv2's INTER_NEAREST index rule inside ``resizeCrop``
is a restatement (parity unpinned for that piece).

Bit-exact: every crop pixel, the CoM, the integer bounds; M within 1e-12 (the reference forms it
with BLAS 3x3 products whose FMA use is unpinned); joint transforms bit-exact; metrics to 1e-6.
The CPU tests run the native host crop (libmonkeypose.so, no GPU call) and the oracle; the
``-m gpu`` test runs the device crop."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import ROOT, pkg
from oracle import crop_ref as CR

FIX = os.path.join(ROOT, "tests", "golden", "crop_ref_fixtures.npz")
PREP = ("f1", "f2", "f3", "f1", "f2", "f3", "tiebig")   # make_crop_fixtures.PREP_FRAMES


@pytest.fixture(scope="module")
def fx():
    z = np.load(FIX, allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    return z, meta


def _frame(z, case):
    f = z["frame_" + case["frame"]]
    return f.astype(np.uint16) if case["dtype"] == "u16" else f


def _cam(meta, case):
    return meta["cameras"][case["camera"]]


def test_fixture_covers_the_edges(fx):
    z, meta = fx
    cases = meta["cases"]
    assert len(cases) >= 40
    assert any(c["docom"] and c["com"] is None for c in cases)
    assert any(c["docom"] and c["dtype"] == "u16" for c in cases)
    assert sum(c["frame"] == "tie" for c in cases) == 6
    assert {c["frame"] for c in cases if c["docom"]} >= {"cz", "c0"}   # the allclose / isclose fallbacks


def test_native_crop_matches_reference_execution(fx):
    z, meta = fx
    MD = pkg().monkeydetector.MonkeyDetector
    for i, c in enumerate(meta["cases"]):
        md = MD(*_cam(meta, c))
        com = None if c["com"] is None else np.array(c["com"])
        crop, M, com_out = md.cropArea3D(_frame(z, c), com=com, docom=c["docom"])
        assert crop.dtype == np.float32 and np.array_equal(crop, z[f"c{i}_crop"]), (i, c)
        assert np.array_equal(com_out, z[f"c{i}_com"]), (i, c)
        assert np.allclose(np.asarray(M), z[f"c{i}_M"], rtol=1e-12, atol=1e-9), (i, c)
        if not c["docom"]:
            b = md.last_crop_info["bounds"]
            assert list(b) == list(z[f"c{i}_bounds"]), (i, c)


def test_native_com_and_bounds_match_reference(fx):
    z, meta = fx
    MD = pkg().monkeydetector.MonkeyDetector
    for i, c in enumerate(meta["cases"]):
        if c["com"] is not None:
            continue
        md = MD(*_cam(meta, c))
        com = md.calculateCoM(_frame(z, c))
        assert np.array_equal(com, z[f"c{i}_com0"]), (i, c)
        xs, xe, ys, ye, zs, ze = md.comToBounds(com, md.cube)
        assert [xs, xe, ys, ye] == list(z[f"c{i}_bounds"]) and [zs, ze] == list(z[f"c{i}_z"])


def test_oracle_matches_reference_execution(fx):
    z, meta = fx
    for i, c in enumerate(meta["cases"]):
        cam = [tuple(v) if isinstance(v, list) else v for v in _cam(meta, c)]
        ref = CR.MonkeyDetectorRef(*cam)
        com = None if c["com"] is None else np.array(c["com"])
        crop, M, com_out, _ = ref.cropArea3D(_frame(z, c), com=com, docom=c["docom"])
        assert np.array_equal(crop, z[f"c{i}_crop"]) and np.array_equal(com_out, z[f"c{i}_com"]), (i, c)


@pytest.mark.parametrize("dtype", ["f32", "u16"])
def test_zend_tie_follows_the_era_promotion(fx, dtype):
    """com depth 2399.99995: zend = 2999.99995 < f32(zend) = 3000.  NumPy 1.x compares a float32
    crop with zend in float32, so a 3000 pixel is KEPT; a uint16 crop compares in float64 and the
    pixel is zeroed.  (NumPy 2 / NEP 50 would zero both.)"""
    z, meta = fx
    i = next(k for k, c in enumerate(meta["cases"])
             if c["frame"] == "tie" and c["dtype"] == dtype and c["camera"] == "cam")
    c = meta["cases"][i]
    md = pkg().monkeydetector.MonkeyDetector(*_cam(meta, c))
    zend = c["com"][2] + 600.0
    assert zend < 3000.0 and np.float32(zend) == np.float32(3000.0)
    crop, _, _ = md.cropArea3D(_frame(z, c), com=np.array(c["com"]))
    assert np.array_equal(crop, z[f"c{i}_crop"])
    if dtype == "f32":
        assert (crop == 3000.0).any()              # the tie pixels survive
    else:
        assert not (crop == 3000.0).any()          # zeroed (backface)
    assert (crop == 2999.0).any() and not (crop == 3001.0).any()


def test_joint_transforms_match_reference(fx):
    z, _ = fx
    md = pkg().monkeydetector.tfMonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    for tag in ("f32", "f64"):
        j = z[f"j_{tag}_xyz"]
        assert np.array_equal(md.xyztouvd_np(j), z[f"j_{tag}_uvd_np"]), tag
        assert np.array_equal(md.xyztouvd(j), z[f"j_{tag}_uvd_md"]), tag
        assert np.array_equal(md.xyztouvd_np(j[3]), z[f"j_{tag}_uvd_one"]), tag
        assert np.array_equal(md.uvdtoxyz(z[f"j_{tag}_com_uvd"]), z[f"j_{tag}_com_xyz"]), tag
        assert np.array_equal(md.uvdtoxyz(z[f"j_{tag}_uvd_in"]), z[f"j_{tag}_xyz_of_uvd"]), tag
        a_xyz, a_uvd = md.getAbsoluteCoordinates(z[f"j_{tag}_rel"], z[f"j_{tag}_com_uvd"])
        assert np.array_equal(a_xyz, z[f"j_{tag}_abs_xyz"]) and np.array_equal(a_uvd, z[f"j_{tag}_abs_uvd"]), tag
        r_xyz, r_uvd = md.getRelativeCoordinates(j, z[f"j_{tag}_uvd_np"], z[f"j_{tag}_com_uvd"], z["c0_M"])
        assert np.array_equal(r_xyz, z[f"j_{tag}_relc_xyz"]), tag
        assert np.allclose(r_uvd, z[f"j_{tag}_relc_uvd"], rtol=1e-6, atol=1e-4), tag


def test_metrics_match_reference(fx):
    z, _ = fx
    pe = pkg().pose_evaluation
    lab, res = z["err_labels"], z["err_results"]
    assert np.isclose(pe.getMeanError_np(lab, res), z["err_mean"], rtol=1e-6)
    assert pe.getMaxError_np(lab, res) == z["err_max"]
    assert np.isclose(pe.getMeanError_np(lab.astype(np.float64), res.astype(np.float64)), z["err_mean_f64"],
                      rtol=1e-12)


def test_host_prepare_data_test_matches_reference(fx):
    """train_cnn_networks_hgru.py:61-74 executed by the generator vs the façade's host batch crop."""
    z, _ = fx
    P = pkg()
    fr = np.stack([z[f"frame_{k}"] for k in PREP]) / np.float32(10000.)
    cfg = type("C", (), dict(image_target_size=[128, 128, 1], image_orig_size=[424, 512, 1],
                             image_max_depth=10000.))
    md = P.monkeydetector.tfMonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    patches, coms, Ms = P.train_cnn_networks_hgru.prepare_data_test(fr.astype(np.float32), z["prep_tr_res"], md, cfg)
    assert np.array_equal(patches, z["prep_patches"].astype(np.float32))
    assert (patches[-1] == np.float32(3000.) / np.float32(10000.)).any()   # the zend tie kept
    assert np.array_equal(np.stack(coms), z["prep_coms"])
    assert np.allclose(np.stack([np.asarray(m) for m in Ms]), z["prep_Ms"], rtol=1e-12, atol=1e-9)


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs the reference sources (build container)")
def test_fixtures_are_the_reference_output(tmp_path):
    """Regenerating the fixtures from the reference's source reproduces the committed file."""
    gen = os.path.join(ROOT, "tests", "golden", "make_crop_fixtures.py")
    subprocess.run([sys.executable, gen, str(tmp_path / "f.npz")], check=True, capture_output=True)
    a, b = np.load(FIX), np.load(tmp_path / "f.npz")
    assert sorted(a.files) == sorted(b.files)
    for k in a.files:
        assert np.array_equal(a[k], b[k], equal_nan=a[k].dtype.kind == "f"), k


@pytest.mark.gpu
def test_device_prepare_data_test_matches_reference(fx):
    """The device crop (mp_crop3d_dev) of the same batch is bit-exact with the reference's
    prepare_data_test."""
    import torch
    z, _ = fx
    P = pkg()
    fr = np.stack([z[f"frame_{k}"] for k in PREP]) / np.float32(10000.)
    cfg = type("C", (), dict(image_target_size=[128, 128, 1], image_orig_size=[424, 512, 1],
                             image_max_depth=10000.))
    md = P.monkeydetector.tfMonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    patches, coms, Ms = P.train_cnn_networks_hgru.prepare_data_test(
        torch.from_numpy(fr.astype(np.float32)).cuda(), torch.from_numpy(z["prep_tr_res"]).cuda(), md, cfg)
    torch.cuda.synchronize()
    assert np.array_equal(patches.cpu().numpy(), z["prep_patches"].astype(np.float32))
    assert np.array_equal(coms.cpu().numpy(), z["prep_coms"])
    assert np.allclose(Ms.cpu().numpy(), z["prep_Ms"], rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
def test_device_docom_matches_host_docom(fx):
    """cropArea3D(docom=True) on the device (mp_crop3d_dev_ex, MP_CROP_DOCOM) equals the host
    refinement (itself bit-exact with the reference's code, test_native_crop_matches_reference_execution)
    bit for bit: patches, refined CoMs, M.  Includes a frame whose first crop has no valid pixel (the
    allclose -> centre-pixel -> 300 mm fallback)."""
    import torch
    z, _ = fx
    P = pkg()
    keys = ("f1", "f2", "f3", "tiebig")
    frames = [z[f"frame_{k}"] for k in keys] + [np.zeros((424, 512), np.float32)]
    fr = (np.stack(frames) / np.float32(10000.)).astype(np.float32)
    rng = np.random.default_rng(5)
    tr = np.stack([np.array([rng.uniform(0.2, 0.8), rng.uniform(0.2, 0.8), rng.uniform(0.08, 0.3)], np.float32)
                   for _ in frames])
    tr[3] = np.array([0.5, 0.5, 0.24], np.float32)
    md = P.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    patches, Ms, coms = md.crop_batch_device(torch.from_numpy(fr).cuda(), torch.from_numpy(tr).cuda(), docom=True)
    torch.cuda.synchronize()
    patches, Ms, coms = patches.cpu().numpy(), Ms.cpu().numpy(), coms.cpu().numpy()
    scale = np.array([424., 512., 10000.])
    for i in range(len(frames)):
        com = tr[i].astype(np.float64) * scale
        crop, M, c = md.cropArea3D(fr[i] * np.float32(10000.), com=com, docom=True)
        assert np.array_equal(coms[i], c), i
        assert np.array_equal(patches[i, :, :, 0], crop / np.float32(10000.)), i
        assert np.allclose(Ms[i], np.asarray(M), rtol=1e-12, atol=1e-9), i
    assert coms[4][2] == 300.0
