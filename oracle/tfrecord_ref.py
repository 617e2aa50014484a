"""CPU ORACLE (test infrastructure only: imported by tests/ and never by the product).

Pure-Python restatement of the TFRecord container and the tf.train.Example encoding the
reference writes and reads (Datareader.py:13-27 encode_example / create_tf_record;
data_loader.py:10-26 read_and_decode).  Third-party format (TensorFlow 1.x, unpinned; not
importable here): restated from the published TFRecord and protobuf wire formats --
  record  = uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data)
  mask(c) = ((c >> 15) | (c << 17)) + 0xa282ead8 (mod 2^32)
  Example{features=1: Features{feature=1: map<string, Feature>}}, Feature{bytes_list=1: BytesList{value=1}}
CRC-32C is the bitwise Castagnoli (reflected 0x82F63B78) definition, pinned by the standard check
value crc32c(b"123456789") = 0xE3069283.  The reference ships no TFRecord files: parity of the
container is pinned by these published constants and a hand-assembled Example (tests), otherwise
PARITY UNPINNED.
"""
from __future__ import annotations

import struct
from typing import Dict, Iterator, List, Sequence, Tuple


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def mask(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(field: int, body: bytes) -> bytes:
    return _varint(field << 3 | 2) + _varint(len(body)) + body


def encode_example(features: Sequence[Tuple[str, bytes]]) -> bytes:
    """tf.train.Example with one bytes_feature per (name, raw) in order (Datareader.py:13-19)."""
    feats = b"".join(_ld(1, _ld(1, name.encode()) + _ld(2, _ld(1, _ld(1, raw)))) for name, raw in features)
    return _ld(1, feats)


def frame(data: bytes) -> bytes:
    n = struct.pack("<Q", len(data))
    return n + struct.pack("<I", mask(crc32c(n))) + data + struct.pack("<I", mask(crc32c(data)))


def _fields(buf: bytes) -> Iterator[Tuple[int, bytes]]:
    p = 0
    while p < len(buf):
        key, p = _read_varint(buf, p)
        assert key & 7 == 2, "only length-delimited fields expected"
        n, p = _read_varint(buf, p)
        yield key >> 3, buf[p:p + n]
        p += n


def _read_varint(buf: bytes, p: int) -> Tuple[int, int]:
    v = s = 0
    while True:
        b = buf[p]
        p += 1
        v |= (b & 0x7F) << s
        s += 7
        if not b & 0x80:
            return v, p


def read_records(blob: bytes) -> List[bytes]:
    out, p = [], 0
    while p < len(blob):
        n = struct.unpack_from("<Q", blob, p)[0]
        assert struct.unpack_from("<I", blob, p + 8)[0] == mask(crc32c(blob[p:p + 8]))
        d = blob[p + 12:p + 12 + n]
        assert struct.unpack_from("<I", blob, p + 12 + n)[0] == mask(crc32c(d))
        out.append(d)
        p += 16 + n
    return out


def parse_example(data: bytes) -> Dict[str, bytes]:
    (f, feats), = list(_fields(data))
    out = {}
    for _, entry in _fields(feats):
        kv = dict(_fields(entry))
        (_, blist), = list(_fields(kv[2]))
        (_, raw), = list(_fields(blist))
        out[kv[1].decode()] = raw
    return out
