"""TF1 V2 checkpoint reader (monkey-pose_amd/tf_checkpoint.py).

Parity unpinned (no TF-written checkpoint exists here): the checksum is pinned by the published
CRC-32C (iSCSI, RFC 3720 B.4) known answers, the snappy decoder by hand-assembled streams, the
table reader by hand-built blocks (prefix-compressed keys, several data blocks, a snappy block),
and the bundle layer by round trips and corruption checks."""
import os
import struct

import numpy as np
import pytest

from helpers import pkg


def C():
    return pkg().tf_checkpoint


def test_crc32c_known_answers():
    c = C()
    assert c.crc32c(b"") == 0
    assert c.crc32c(b"123456789") == 0xE3069283
    assert c.crc32c(bytes(32)) == 0x8A9136AA
    assert c.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert c.crc32c(bytes(range(32))) == 0x46DD794E
    assert c.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    # streaming (init = previous crc) and unaligned starts agree with one shot
    data = os.urandom(1000)
    assert c.crc32c(data[300:], c.crc32c(data[:300])) == c.crc32c(data)
    assert c.crc32c(np.frombuffer(data, np.uint8)[3:]) == c.crc32c(data[3:])
    # LevelDB masking
    assert c.mask_crc(0) == 0xA282EAD8
    for v in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert c.unmask_crc(c.mask_crc(v)) == v


def test_snappy_hand_assembled_streams():
    c = C()
    # literal "abc" + copy (1-byte offset 3, length 9)
    assert c.snappy_decompress(b"\x0c\x08abc\x15\x03") == b"abcabcabcabc"
    # a 70-byte literal (tag 60 + 1 length byte) then a 2-byte-offset copy of 20 bytes at offset 70
    lit = bytes(range(70))
    stream = bytes([90]) + bytes([60 << 2, 69]) + lit + bytes([(20 - 1) << 2 | 2]) + struct.pack("<H", 70)
    assert c.snappy_decompress(stream) == lit + lit[:20]
    # overlapping copy: "a" then copy offset 1 length 7 -> "aaaaaaaa"
    assert c.snappy_decompress(b"\x08\x00a\x0d\x01") == b"a" * 8
    with pytest.raises(c.CheckpointError):
        c.snappy_decompress(b"\x05\x00a\x0d\x05")          # copy before the start


def _snappy_literal(data: bytes) -> bytes:
    """Valid snappy stream made only of literals (<= 60 bytes each)."""
    c = C()
    out = c._put_varint(len(data))
    for i in range(0, len(data), 60):
        ch = data[i:i + 60]
        out += bytes([(len(ch) - 1) << 2]) + ch
    return out


def test_table_reader_blocks_restarts_and_snappy(tmp_path):
    c = C()
    entries = [(f"key{i:04d}".encode(), f"value-{i}".encode() * (i % 3 + 1)) for i in range(200)]
    p = str(tmp_path / "t.index")
    c.write_table(p, entries, block_size=256)          # many data blocks, restart every 16 keys
    assert c.read_table(p) == entries
    # hand-build a table whose single data block is snappy-compressed (type 1)
    blk = c._block(entries[:20], 4)
    comp = _snappy_literal(blk)
    out = bytearray(comp) + b"\x01" + struct.pack("<I", c.mask_crc(c.crc32c(comp + b"\x01")))
    handle = c._put_varint(0) + c._put_varint(len(comp))
    meta_off = len(out)
    meta = c._block([], 1)
    out += meta + b"\x00" + struct.pack("<I", c.mask_crc(c.crc32c(meta + b"\x00")))
    idx_off = len(out)
    idx = c._block([(entries[19][0], handle)], 1)
    out += idx + b"\x00" + struct.pack("<I", c.mask_crc(c.crc32c(idx + b"\x00")))
    foot = c._put_varint(meta_off) + c._put_varint(len(meta)) + c._put_varint(idx_off) + c._put_varint(len(idx))
    out += foot + b"\x00" * (40 - len(foot)) + struct.pack("<Q", 0xDB4775248B80FB57)
    q = str(tmp_path / "s.index")
    open(q, "wb").write(out)
    assert c.read_table(q) == entries[:20]
    # a flipped byte inside a block fails its checksum
    bad = bytearray(out)
    bad[5] ^= 0x40
    open(q, "wb").write(bad)
    with pytest.raises(c.CheckpointError):
        c.read_table(q)


def test_checkpoint_round_trip_dtypes_and_state_file(tmp_path):
    c = C()
    rng = np.random.default_rng(0)
    t = {"cnn/conv_1/conv_1_filters": rng.standard_normal((3, 3, 1, 64)).astype(np.float32),
         "cnn/fc_out/fc_out_biases": rng.standard_normal(69).astype(np.float32),
         "global_step": np.array(1234, np.int64),
         "d": rng.standard_normal((2, 5)), "i32": np.arange(7, dtype=np.int32), "flag": np.array([True, False]),
         "h": rng.standard_normal(9).astype(np.float16), "u8": np.arange(5, dtype=np.uint8),
         "empty": np.zeros((0, 4), np.float32)}
    prefix = str(tmp_path / "ckpt" / "model.ckpt-10")
    c.write_checkpoint(prefix, t)
    for path in (prefix, prefix + ".index", str(tmp_path / "ckpt")):
        got = c.read_checkpoint(path)
        assert set(got) == set(t)
        for k, v in t.items():
            assert got[k].dtype == v.dtype and got[k].shape == v.shape and np.array_equal(got[k], v), k
    names = dict((n, (s, d)) for n, s, d in c.list_variables(prefix))
    assert names["cnn/conv_1/conv_1_filters"] == ((3, 3, 1, 64), "float32") and names["global_step"][0] == ()
    # a corrupted tensor byte is detected by the entry checksum
    data = prefix + ".data-00000-of-00001"
    raw = bytearray(open(data, "rb").read())
    raw[10] ^= 1
    open(data, "wb").write(raw)
    with pytest.raises(c.CheckpointError):
        c.read_checkpoint(prefix)
    assert len(c.read_checkpoint(prefix, verify=False)) == len(t)


def test_bfloat16_entries_widen_to_float32(tmp_path):
    c = C()
    vals = np.array([1.0, -2.5, 3.140625, 65280.0], np.float32)
    bf = (vals.view(np.uint32) >> 16).astype("<u2").tobytes()
    prefix = str(tmp_path / "bf")
    open(prefix + ".data-00000-of-00001", "wb").write(bf)
    e = c.Entry(14, (4,), 0, 0, len(bf), c.mask_crc(c.crc32c(bf)))
    hdr = c._pb_key(1, 0) + c._put_varint(1)
    c.write_table(prefix + ".index", [(b"", hdr), (b"w", e.serialize())])
    assert np.array_equal(c.read_checkpoint(prefix)["w"], vals)


def test_split_training_graph_names():
    c = C()
    W = pkg().weights
    attn = W.synth_weights(W.attn_vars(), seed=1)
    pose = W.synth_weights(W.hgru_pose_vars(output_shape=69, timesteps=8, crop=64), seed=2)
    graph = dict(attn)
    for k, v in pose.items():        # the pose model's BNs follow the attention net's six
        m = c._bn_index(k)
        if m:
            k = f"cnn/batch_normalization_{m[0] + 6}/{m[1]}"
        graph[k] = v
    slots = {k + "/Adam": v for k, v in list(graph.items())[:5]}
    slots.update({k + "/Adam_1": v for k, v in list(graph.items())[:5]})
    graph.update(slots, **{"beta1_power": np.float32(0.9), "beta2_power": np.float32(0.99),
                           "global_step": np.int64(5)})
    a, p = c.split_hgru_train_checkpoint(graph)
    assert set(a) == set(attn) and set(p) == set(pose)
    assert all(np.array_equal(a[k], attn[k]) for k in attn)
    assert all(np.array_equal(p[k], pose[k]) for k in pose)


def test_facade_loads_checkpoint_strictly(tmp_path):
    c = C()
    P = pkg()
    W = P.weights
    pose = W.synth_weights(W.hgru_pose_vars(output_shape=69, timesteps=8, crop=64), seed=2)
    prefix = str(tmp_path / "pose.ckpt")
    c.write_checkpoint(prefix, dict(pose, **{"cnn/fc_1/fc_1_weights/Adam": pose["cnn/fc_1/fc_1_weights"]}))
    m = P.hgru_pose.model()
    m.load_checkpoint(prefix)
    res = m._resolve_weights(69, (64, 64))
    assert set(res) == set(pose) and all(np.array_equal(res[k], pose[k]) for k in pose)
    # strict: a missing variable raises instead of being synthesised
    del pose["cnn/contextual_circuit/p_r"]
    c.write_checkpoint(prefix, pose)
    m.load_checkpoint(prefix)
    with pytest.raises(KeyError):
        m._resolve_weights(69, (64, 64))


@pytest.mark.gpu
def test_checkpoint_weights_drive_the_gpu_path(tmp_path):
    """hgru_pose built from a checkpoint gives the same bits as from the in-memory weights, and the
    attention half of a training-graph checkpoint loads into attn_model_struct."""
    import torch
    c = C()
    P = pkg()
    W = P.weights
    pose = W.synth_weights(W.hgru_pose_vars(output_shape=69, timesteps=8, crop=64), seed=2)
    attn = W.attn_synth_weights(seed=3)
    graph = dict(attn)
    for k, v in pose.items():
        m = c._bn_index(k)
        graph[f"cnn/batch_normalization_{m[0] + 6}/{m[1]}" if m else k] = v
    prefix = str(tmp_path / "train" / "model.ckpt-100")
    c.write_checkpoint(prefix, graph)
    depth = torch.from_numpy(W.synth_crops(2, seed=4, size=64)).cuda()
    o0 = torch.from_numpy(W.synth_hidden((2, 32, 32, 64), seed=5)).cuda()
    m1 = P.hgru_pose.model()
    m1.load_weights(pose)
    m2 = P.hgru_pose.model()
    m2.load_checkpoint(str(tmp_path / "train"), remap=lambda t: c.split_hgru_train_checkpoint(t)[1])
    a = m1.build(depth, 69, h2_init=o0).cpu().numpy()
    b = m2.build(depth, 69, h2_init=o0).cpu().numpy()
    assert np.array_equal(a, b)
    at = P.train_cnn_networks_hgru.attn_model_struct()
    at.load_checkpoint(prefix, remap=lambda t: c.split_hgru_train_checkpoint(t)[0])
    at2 = P.train_cnn_networks_hgru.attn_model_struct()
    at2.load_weights(attn)
    fr = torch.from_numpy(W.synth_frames(2, seed=6)).cuda()
    assert np.array_equal(at.build(fr, 3).cpu().numpy(), at2.build(fr, 3).cpu().numpy())
