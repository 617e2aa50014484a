"""TFRecord ingestion (data_loader.py:10-40, Datareader.py:13-27): the native
reader / writer (host code in libmonkeypose.so, no GPU needed) against the pure-Python oracle
(oracle/tfrecord_ref.py), a hand-assembled Example and the published CRC-32C check value."""
import numpy as np
import pytest

from helpers import pkg
from oracle import tfrecord_ref as TR


def test_oracle_pins():
    assert TR.crc32c(b"123456789") == 0xE3069283          # CRC-32C check value
    # Example{features{feature{key: "a", value{bytes_list{value: "xy"}}}}}, assembled by hand
    want = bytes([0x0A, 0x0D, 0x0A, 0x0B, 0x0A, 0x01, 0x61, 0x12, 0x06, 0x0A, 0x04, 0x0A, 0x02, 0x78, 0x79])
    assert TR.encode_example([("a", b"xy")]) == want
    assert TR.parse_example(want) == {"a": b"xy"}


def _data(n, seed=0):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((n, 12, 16, 1)).astype(np.float32),
            rng.standard_normal((n, 69)).astype(np.float32))


def test_native_writer_matches_oracle_bytes(tmp_path):
    D = pkg().data_loader
    im, lab = _data(5)
    p = tmp_path / "a.tfrecord"
    D.create_tf_record(im, lab, str(p))
    want = b"".join(TR.frame(TR.encode_example([("label", lab[i].tobytes()), ("image", im[i].tobytes())]))
                    for i in range(5))
    assert p.read_bytes() == want
    assert D.encode_example(im[0], lab[0]) == TR.encode_example([("label", lab[0].tobytes()),
                                                                   ("image", im[0].tobytes())])


def test_native_reader_decodes_oracle_file(tmp_path):
    D = pkg().data_loader
    im, lab = _data(7, 1)
    p = tmp_path / "b.tfrecord"
    # oracle-written, with the features in the other order and an extra feature
    p.write_bytes(b"".join(TR.frame(TR.encode_example([("image", im[i].tobytes()), ("x", b"q" * i),
                                                       ("label", lab[i].tobytes())])) for i in range(7)))
    r = D.TFRecordFile(str(p))
    assert len(r) == 7 and r.feature_size("image") == im[0].nbytes and r.feature_size("x", 3) == 3
    got = [(l, m) for l, m in D.read_and_decode(r, (12, 16, 1), 69)]
    for i, (l, m) in enumerate(got):
        assert np.array_equal(l, lab[i]) and np.array_equal(m, im[i])
    idx = [6, 0, 3]
    out = r.gather("image", idx, np.empty((3, 12, 16, 1), np.float32), nthreads=3)
    assert np.array_equal(out, im[idx])


def test_inputs_batches(tmp_path):
    D = pkg().data_loader
    im, lab = _data(10, 2)
    p = tmp_path / "c.tfrecord"
    D.create_tf_record(im[:6], lab[:6], str(p))
    D.create_tf_record(im[6:], lab[6:], str(p), append=True)
    seen = []
    for data, labels in D.inputs(str(p), 2, (12, 16, 1), 69, 4, seed=3):
        assert data.shape == (4, 12, 16, 1) and labels.shape == (4, 69)
        for d, l in zip(data, labels):
            i = int(np.where((lab == l).all(1))[0][0])
            assert np.array_equal(im[i], d)
            seen.append(i)
    assert len(seen) == 16 and len(set(seen)) >= 8            # 2 epochs x 2 full batches, shuffled
    plain = list(D.inputs(str(p), 1, (12, 16, 1), 69, 5, shuffle=False))
    assert np.array_equal(plain[1][0], im[5:10])


def test_reader_rejects_corruption(tmp_path):
    D, L = pkg().data_loader, pkg()._lib
    im, lab = _data(3, 4)
    p = tmp_path / "d.tfrecord"
    D.create_tf_record(im, lab, str(p))
    blob = bytearray(p.read_bytes())
    blob[40] ^= 1                                   # inside record 0's payload
    p.write_bytes(bytes(blob))
    with pytest.raises(L.MonkeyPoseError, match="crc"):
        D.TFRecordFile(str(p))
    D.TFRecordFile(str(p), verify=False)            # payload CRCs skipped on request
    p.write_bytes(bytes(blob[:-3]))
    with pytest.raises(L.MonkeyPoseError, match="truncated"):
        D.TFRecordFile(str(p), verify=False)
    q = tmp_path / "e.tfrecord"
    D.create_tf_record(im, lab, str(q))
    with pytest.raises(L.MonkeyPoseError, match="expected"):
        D.TFRecordFile(str(q)).gather("image", [0], np.empty((1, 10), np.float32))


@pytest.mark.gpu
def test_tfrecord_frames_feed_the_frame_chain(tmp_path):
    """TFRecord of full depth frames -> inputs(device='cuda') batches -> attention -> device crop ->
    hGRU pose: identical (bitwise) to feeding the same frames from memory."""
    torch = pytest.importorskip("torch")
    from helpers import MG, golden_meta
    from test_attn import _attn_model
    P = pkg()
    T = P.train_cnn_networks_hgru
    m = golden_meta()["attn_f424"]
    wts, frames = MG.attn_inputs(m["n"], m["h"], m["w"], m["weight_seed"], m["frame_seed"])
    labels = np.arange(frames.shape[0] * 69, dtype=np.float32).reshape(-1, 69)
    p = tmp_path / "frames.tfrecord"
    P.data_loader.create_tf_record(frames[..., None] if frames.ndim == 3 else frames, labels, str(p))
    pose = P.hgru_pose.model()
    pm = golden_meta()["pose_c128_t8"]
    pw, _, _ = MG.pose_inputs(pm["n"], pm["crop"], 8, pm["weight_seed"], pm["crop_seed"], pm["o0_seed"])
    pose.load_weights(pw)
    md = P.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
    pipe = T.FramePosePipeline(_attn_model(wts), pose, md)
    n = frames.shape[0]
    O0 = torch.from_numpy(P.weights.synth_hidden((n, 64, 64, 64), seed=7)).cuda()
    (data, lab), = list(P.data_loader.inputs(str(p), 1, (m["h"], m["w"], 1), 69, n, shuffle=False, device="cuda"))
    assert data.is_cuda and np.array_equal(lab.cpu().numpy(), labels)
    direct = torch.from_numpy(frames.reshape(n, m["h"], m["w"], 1)).cuda()
    assert torch.equal(data, direct)
    out, _, _ = pipe.run(data, h2_init=O0)
    ref, _, _ = pipe.run(direct, h2_init=O0)
    assert torch.equal(out, ref)
