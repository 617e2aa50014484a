"""TF1 checkpoint reader / writer: the weights a reference user has are
``tf.train.Saver`` V2 checkpoints (``train_cnn_networks_hgru.py:188`` saver, ``248-250`` /
``312-313`` ``saver.restore``), i.e. a ``<prefix>.index`` table plus ``<prefix>.data-SSSSS-of-NNNNN``
shards.  This module reads them without TensorFlow:

* ``<prefix>.index`` is a LevelDB-format sorted string table (the format of
  ``tensorflow/core/lib/io/table``): data blocks of prefix-compressed key/value entries with a
  restart array, each followed by a 5-byte trailer (compression type, masked CRC-32C), an index
  block mapping separator keys to (offset, size) block handles, a metaindex block, and a 48-byte
  footer ending in the magic 0xdb4775248b80fb57.  Blocks may be snappy-compressed (type 1).
* Key ``""`` holds a ``BundleHeaderProto`` (num_shards, endianness, version); every other key is
  a variable name whose value is a ``BundleEntryProto`` (dtype, shape, shard_id, offset, size,
  masked crc32c of the raw bytes) -- ``tensorflow/core/protobuf/tensor_bundle.proto``.
* Tensor bytes are raw little-endian at ``offset`` in the shard file.

Third-party formats (TensorFlow 1.x, LevelDB table, snappy) are restated from their published
specifications: PARITY UNPINNED -- no TF-written checkpoint exists in the reference or this image.
The reader is checked against the CRC-32C known-answer vectors, hand-assembled snappy streams and
tables, and round trips through ``write_checkpoint`` (tests/test_tf_checkpoint.py).  CRC-32C runs
natively (``mp_crc32c`` in libmonkeypose.so, SSE4.2).

``split_hgru_train_checkpoint`` maps the variables of the reference's training graph (attention
net built first, then ``hgru_pose.model``, one ``cnn`` scope, Adam slots) onto the two façades:
the attention BNs are ``batch_normalization`` .. ``_5``, the pose model's ``_6`` .. ``_10``.
"""
from __future__ import annotations

import ctypes
import os
import re
import struct
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

_MAGIC = 0xDB4775248B80FB57
_MASK_DELTA = 0xA282EAD8

# tensorflow/core/framework/types.proto DataType -> numpy (bfloat16 handled separately)
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8,
           9: np.int64, 10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
_DT_BFLOAT16 = 14
_DT_STRING = 7
_NP_TO_DT = {np.dtype(v): k for k, v in _DTYPES.items()}


class CheckpointError(ValueError):
    pass


# ----------------------------------------------------------------------------------- checksums
def crc32c(data, init: int = 0) -> int:
    """CRC-32C of ``data`` (bytes-like or numpy array) continuing from ``init``; native."""
    from . import _lib
    fn = _lib.load().mp_crc32c
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data)
        return int(fn(init, a.ctypes.data_as(ctypes.c_void_p), a.nbytes))
    b = bytes(data)
    buf = ctypes.create_string_buffer(b, len(b))
    return int(fn(init, ctypes.cast(buf, ctypes.c_void_p), len(b)))


def mask_crc(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


def unmask_crc(masked: int) -> int:
    rot = (masked - _MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ------------------------------------------------------------------------------------- varints
def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    r, shift = 0, 0
    while True:
        if pos >= len(buf):
            raise CheckpointError("truncated varint")
        b = buf[pos]
        pos += 1
        r |= (b & 0x7F) << shift
        if b < 0x80:
            return r, pos
        shift += 7
        if shift > 63:
            raise CheckpointError("varint too long")


def _put_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


# ------------------------------------------------------------------------------------ protobuf
def _pb_fields(buf: bytes) -> Dict[int, list]:
    """Wire-format decode: field number -> list of values (int for varint / fixed, bytes for
    length-delimited)."""
    out: Dict[int, list] = {}
    pos = 0
    while pos < len(buf):
        key, pos = _varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise CheckpointError(f"unsupported protobuf wire type {wt}")
        out.setdefault(field, []).append(v)
    if pos != len(buf):
        raise CheckpointError("truncated protobuf message")
    return out


def _pb_key(field: int, wt: int) -> bytes:
    return _put_varint((field << 3) | wt)


class Entry:
    """A ``BundleEntryProto``."""

    __slots__ = ("dtype", "shape", "shard_id", "offset", "size", "crc32c")

    def __init__(self, dtype, shape, shard_id, offset, size, crc):
        self.dtype, self.shape, self.shard_id = dtype, shape, shard_id
        self.offset, self.size, self.crc32c = offset, size, crc

    @classmethod
    def parse(cls, raw: bytes) -> "Entry":
        f = _pb_fields(raw)
        if 7 in f:
            raise CheckpointError("partitioned (sliced) variables are not supported")
        shape: List[int] = []
        if 2 in f:
            sp = _pb_fields(f[2][0])
            if sp.get(3, [0])[0]:
                raise CheckpointError("unknown-rank tensor in checkpoint")
            for d in sp.get(2, []):
                size = _pb_fields(d).get(1, [0])[0]
                if size >= 1 << 63:       # int64 two's complement (-1 = unknown dim)
                    raise CheckpointError("unknown dimension in checkpoint shape")
                shape.append(size)
        return cls(f.get(1, [0])[0], tuple(shape), f.get(3, [0])[0], f.get(4, [0])[0], f.get(5, [0])[0],
                   f.get(6, [None])[0])

    def serialize(self) -> bytes:
        dims = b"".join(_pb_key(2, 2) + _put_varint(len(d)) + d
                        for d in (_pb_key(1, 0) + _put_varint(s) if s else b"" for s in self.shape))
        out = _pb_key(1, 0) + _put_varint(self.dtype)
        out += _pb_key(2, 2) + _put_varint(len(dims)) + dims
        if self.shard_id:
            out += _pb_key(3, 0) + _put_varint(self.shard_id)
        if self.offset:
            out += _pb_key(4, 0) + _put_varint(self.offset)
        if self.size:
            out += _pb_key(5, 0) + _put_varint(self.size)
        out += _pb_key(6, 5) + struct.pack("<I", self.crc32c)
        return out


# -------------------------------------------------------------------------------------- snappy
def snappy_decompress(buf: bytes) -> bytes:
    """Raw snappy block format: varint uncompressed length, then literal / copy elements."""
    n, pos = _varint(buf, 0)
    out = bytearray()
    while pos < len(buf):
        tag = buf[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:                                   # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += buf[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:                                   # copy, 1-byte offset
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | buf[pos]
            pos += 1
        elif kind == 2:                                 # copy, 2-byte offset
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 2], "little")
            pos += 2
        else:                                           # copy, 4-byte offset
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 4], "little")
            pos += 4
        if off == 0 or off > len(out):
            raise CheckpointError("corrupt snappy stream (bad copy offset)")
        start = len(out) - off
        for i in range(ln):                             # byte-wise: copies may overlap
            out.append(out[start + i])
    if len(out) != n:
        raise CheckpointError("corrupt snappy stream (length mismatch)")
    return bytes(out)


# -------------------------------------------------------------------------------------- tables
def _read_block(data: bytes, offset: int, size: int, verify: bool) -> bytes:
    if offset + size + 5 > len(data):
        raise CheckpointError("block handle outside the table file")
    contents = data[offset:offset + size]
    ctype = data[offset + size]
    if verify:
        stored = struct.unpack_from("<I", data, offset + size + 1)[0]
        if unmask_crc(stored) != crc32c(data[offset:offset + size + 1]):
            raise CheckpointError("table block checksum mismatch")
    if ctype == 0:
        return contents
    if ctype == 1:
        return snappy_decompress(contents)
    raise CheckpointError(f"unsupported table block compression {ctype}")


def _block_entries(block: bytes) -> Iterator[Tuple[bytes, bytes]]:
    if len(block) < 4:
        raise CheckpointError("table block too short")
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    limit = len(block) - 4 - 4 * nrest
    if limit < 0:
        raise CheckpointError("bad restart count")
    pos, key = 0, b""
    while pos < limit:
        shared, pos = _varint(block, pos)
        nonshared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        if shared > len(key):
            raise CheckpointError("bad key prefix length")
        key = key[:shared] + block[pos:pos + nonshared]
        pos += nonshared
        val = block[pos:pos + vlen]
        pos += vlen
        yield key, val


def read_table(path: str, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    """All (key, value) pairs of a LevelDB-format table file, in key order."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 48:
        raise CheckpointError(f"{path}: too short for a table footer")
    magic = struct.unpack_from("<Q", data, len(data) - 8)[0]
    if magic != _MAGIC:
        raise CheckpointError(f"{path}: bad table magic {magic:#x}")
    foot = data[len(data) - 48:len(data) - 8]
    _, p = _varint(foot, 0)
    _, p = _varint(foot, p)                             # metaindex handle (unused)
    ioff, p = _varint(foot, p)
    isz, p = _varint(foot, p)
    out = []
    for _, handle in _block_entries(_read_block(data, ioff, isz, verify)):
        boff, q = _varint(handle, 0)
        bsz, _ = _varint(handle, q)
        out.extend(_block_entries(_read_block(data, boff, bsz, verify)))
    return out


def _block(entries: List[Tuple[bytes, bytes]], restart_interval: int) -> bytes:
    buf, restarts, prev = bytearray(), [], b""
    for i, (k, v) in enumerate(entries):
        shared = 0
        if i % restart_interval == 0:
            restarts.append(len(buf))
        else:
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        buf += _put_varint(shared) + _put_varint(len(k) - shared) + _put_varint(len(v))
        buf += k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


def write_table(path: str, entries: List[Tuple[bytes, bytes]], block_size: int = 4096) -> None:
    """LevelDB-format table (no compression), keys must be sorted and unique."""
    keys = [k for k, _ in entries]
    if keys != sorted(keys) or len(set(keys)) != len(keys):
        raise CheckpointError("table keys must be sorted and unique")
    out = bytearray()
    index = []

    def emit(contents: bytes) -> bytes:
        off = len(out)
        out.extend(contents)
        t = b"\x00"
        out.extend(t + struct.pack("<I", mask_crc(crc32c(contents + t))))
        return _put_varint(off) + _put_varint(len(contents))

    chunk: List[Tuple[bytes, bytes]] = []
    size = 0
    for k, v in entries:
        chunk.append((k, v))
        size += len(k) + len(v) + 8
        if size >= block_size:
            index.append((chunk[-1][0], emit(_block(chunk, 16))))
            chunk, size = [], 0
    if chunk:
        index.append((chunk[-1][0], emit(_block(chunk, 16))))
    meta = emit(_block([], 1))
    idx = emit(_block(index, 1))
    foot = meta + idx
    foot += b"\x00" * (40 - len(foot))
    out.extend(foot + struct.pack("<Q", _MAGIC))
    with open(path, "wb") as f:
        f.write(out)


# ---------------------------------------------------------------------------------- checkpoints
def resolve_prefix(path: str) -> str:
    """A checkpoint prefix from a prefix, an ``.index`` path, or a directory holding the
    ``checkpoint`` state file (``tf.train.latest_checkpoint``, train_cnn_networks_hgru.py:311)."""
    if path.endswith(".index"):
        return path[:-len(".index")]
    if os.path.isdir(path):
        state = os.path.join(path, "checkpoint")
        if not os.path.exists(state):
            raise CheckpointError(f"{path}: no 'checkpoint' state file")
        m = re.search(r'^model_checkpoint_path:\s*"(.*)"\s*$', open(state).read(), re.M)
        if not m:
            raise CheckpointError(f"{state}: no model_checkpoint_path")
        p = m.group(1)
        return p if os.path.isabs(p) else os.path.join(path, p)
    return path


def _entries(prefix: str, verify: bool) -> Tuple[int, Dict[str, Entry]]:
    rows = read_table(prefix + ".index", verify)
    if not rows or rows[0][0] != b"":
        raise CheckpointError("checkpoint index has no bundle header")
    hdr = _pb_fields(rows[0][1])
    nshards = hdr.get(1, [1])[0]
    if hdr.get(2, [0])[0] != 0:
        raise CheckpointError("big-endian checkpoints are not supported")
    return nshards, {k.decode(): Entry.parse(v) for k, v in rows[1:]}


def list_variables(path: str) -> List[Tuple[str, Tuple[int, ...], str]]:
    """(name, shape, dtype name) of every variable, like tf.train.list_variables."""
    _, ents = _entries(resolve_prefix(path), verify=True)
    names = {v: k for k, v in {"bfloat16": _DT_BFLOAT16, "string": _DT_STRING}.items()}
    return [(n, e.shape, np.dtype(_DTYPES[e.dtype]).name if e.dtype in _DTYPES else names.get(e.dtype, str(e.dtype)))
            for n, e in sorted(ents.items())]


def read_checkpoint(path: str, names: Optional[List[str]] = None, verify: bool = True,
                    skip_unsupported: bool = True) -> Dict[str, np.ndarray]:
    """{variable name: array} of a V2 checkpoint (``tf.train.NewCheckpointReader`` semantics).
    bfloat16 tensors are widened to float32; string tensors are skipped (or raise)."""
    prefix = resolve_prefix(path)
    nshards, ents = _entries(prefix, verify)
    want = sorted(ents) if names is None else list(names)
    out: Dict[str, np.ndarray] = {}
    files: Dict[int, object] = {}
    try:
        for n in want:
            if n not in ents:
                raise CheckpointError(f"variable {n!r} not in checkpoint")
            e = ents[n]
            if e.dtype not in _DTYPES and e.dtype != _DT_BFLOAT16:
                if skip_unsupported:
                    continue
                raise CheckpointError(f"{n}: unsupported dtype {e.dtype}")
            if e.shard_id not in files:
                files[e.shard_id] = open(f"{prefix}.data-{e.shard_id:05d}-of-{nshards:05d}", "rb")
            f = files[e.shard_id]
            f.seek(e.offset)
            raw = np.fromfile(f, dtype=np.uint8, count=e.size)
            if raw.size != e.size:
                raise CheckpointError(f"{n}: data shard truncated")
            if verify and e.crc32c is not None and unmask_crc(e.crc32c) != crc32c(raw):
                raise CheckpointError(f"{n}: tensor checksum mismatch")
            if e.dtype == _DT_BFLOAT16:
                arr = (raw.view("<u2").astype(np.uint32) << 16).view(np.float32)
            else:
                arr = raw.view(np.dtype(_DTYPES[e.dtype]).newbyteorder("<")).astype(_DTYPES[e.dtype], copy=False)
            n_el = int(np.prod(e.shape)) if e.shape else 1
            if arr.size != n_el:
                raise CheckpointError(f"{n}: {arr.size} elements for shape {e.shape}")
            out[n] = arr.reshape(e.shape)
    finally:
        for f in files.values():
            f.close()
    return out


def write_checkpoint(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """A single-shard V2 checkpoint (``tf.train.Saver.save`` layout) -- for exporting weights and
    for tests.  Writes ``<prefix>.index`` and ``<prefix>.data-00000-of-00001``."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    rows = []
    off = 0
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        for name in sorted(tensors):
            a = np.asarray(tensors[name])
            if not a.flags.c_contiguous:   # (np.ascontiguousarray would turn a scalar into [1])
                a = a.copy(order="C")
            dt = _NP_TO_DT.get(a.dtype)
            if dt is None:
                raise CheckpointError(f"{name}: dtype {a.dtype} not supported")
            raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            f.write(raw)
            e = Entry(dt, tuple(int(s) for s in a.shape), 0, off, len(raw), mask_crc(crc32c(raw)))
            rows.append((name.encode(), e.serialize()))
            off += len(raw)
    header = _pb_key(1, 0) + _put_varint(1) + _pb_key(3, 2) + _put_varint(2) + _pb_key(1, 0) + _put_varint(1)
    write_table(prefix + ".index", [(b"", header)] + rows)
    state = os.path.join(os.path.dirname(os.path.abspath(prefix)), "checkpoint")
    with open(state, "w") as f:
        f.write(f'model_checkpoint_path: "{os.path.basename(prefix)}"\n'
                f'all_model_checkpoint_paths: "{os.path.basename(prefix)}"\n')


# ------------------------------------------------------------------------ reference graph maps
_OPT_SLOT = re.compile(r"/(Adam|Adam_\d+|Momentum|RMSProp(_\d+)?)$")


def model_variables(tensors: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Drop optimizer state (Adam slots, beta{1,2}_power) and global_step."""
    return {k: v for k, v in tensors.items()
            if not _OPT_SLOT.search(k) and not re.search(r"(^|/)beta[12]_power(_\d+)?$", k)
            and not k.endswith("global_step")}


def _bn_index(name: str) -> Optional[Tuple[int, str]]:
    m = re.match(r"^cnn/batch_normalization(?:_(\d+))?/(gamma|beta|moving_mean|moving_variance)$", name)
    if not m:
        return None
    return int(m.group(1) or 0), m.group(2)


def split_hgru_train_checkpoint(tensors: Dict[str, np.ndarray], n_attn_bn: int = 6
                                ) -> Tuple[Dict[str, np.ndarray], Dict[str, np.ndarray]]:
    """(attention weights, hgru_pose weights) of the reference's training graph
    (train_cnn_networks_hgru.py:111-143: attn_model_struct built first, then hgru_pose.model, in
    one ``cnn`` scope): BNs 0..5 belong to the attention net, 6..10 are the pose model's BN 0..4.
    Names are returned in the façades' (fresh-graph) form."""
    tv = model_variables(tensors)
    attn, pose = {}, {}
    for k, v in tv.items():
        bn = _bn_index(k)
        if bn is not None:
            i, leaf = bn
            if i < n_attn_bn:
                attn[k] = v
            else:
                j = i - n_attn_bn
                pose[f"cnn/batch_normalization{'' if j == 0 else '_' + str(j)}/{leaf}"] = v
        elif re.match(r"^cnn/(aconv_\d|afc_)", k):
            attn[k] = v
        else:
            pose[k] = v
    return attn, pose
