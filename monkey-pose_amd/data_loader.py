"""Drop-in for ``/root/reference/data_loader.py`` and the writer half of ``Datareader.py``
(TFRecord ingestion), without TensorFlow.

* ``read_and_decode(reader, target_size, label_shape)`` -- data_loader.py:10-26: every record's
  ``label`` / ``image`` bytes features through ``decode_raw(float32)``, the image reshaped to
  ``target_size``.
* ``inputs(tfrecord_file, num_epochs, image_target_size, label_shape, batch_size, ...)`` --
  data_loader.py:28-40: batches ``(data [B, *image_target_size], labels [B, *label_shape])``.  The
  reference's ``tf.train.shuffle_batch`` (capacity 100 + 3B, min_after_dequeue 1, two threads) has
  no reproducible order; here each epoch is a seeded permutation of the records (``shuffle=False``
  keeps file order), the last partial batch is dropped as shuffle_batch does, and ``device=``
  copies each batch from pinned host memory onto the GPU.
* ``encode_example`` / ``create_tf_record`` -- Datareader.py:13-27.

The container is parsed natively (``mp_tfrecord_*`` in libmonkeypose.so: memory-mapped, CRC-checked
index, threaded gather-decode into the batch buffer).  Data augmentation (``data_augment=True``)
is a training option and raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterator, Optional, Sequence, Tuple

import numpy as np

from . import _lib


class TFRecordFile:
    """A memory-mapped, indexed TFRecord file (mp_tfrecord_open)."""

    def __init__(self, path: str, verify: bool = True):
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        n = ctypes.c_int64()
        _lib.check(self.lib.mp_tfrecord_open(os.fsencode(path), 1 if verify else 0, ctypes.byref(h),
                                             ctypes.byref(n)))
        self.h, self.path = h, path
        self.n = int(n.value)

    def __len__(self):
        return self.n

    def close(self):
        if getattr(self, "h", None):
            self.lib.mp_tfrecord_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def feature_size(self, feature: str, record: int = 0) -> int:
        b = ctypes.c_int64()
        _lib.check(self.lib.mp_tfrecord_feature_size(self.h, int(record), feature.encode(), ctypes.byref(b)))
        return int(b.value)

    def gather(self, feature: str, indices, out: np.ndarray, nthreads: int = 8) -> np.ndarray:
        """decode_raw of ``feature`` for records ``indices`` into ``out`` (C-contiguous, one row per
        index, each row exactly the feature's byte size)."""
        idx = np.ascontiguousarray(np.asarray(indices, np.int64))
        if not out.flags.c_contiguous or out.shape[0] != idx.size:
            raise ValueError("out must be C-contiguous with one row per index")
        per = out.nbytes // max(1, idx.size)
        _lib.check(self.lib.mp_tfrecord_read(self.h, idx.ctypes.data_as(ctypes.c_void_p), idx.size,
                                             feature.encode(), out.ctypes.data_as(ctypes.c_void_p), per,
                                             int(nthreads)))
        return out


def read_and_decode(reader, target_size, label_shape, data_augment=False) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
    """data_loader.py:10-26, one record at a time: (label float32 [label_shape], image float32
    reshaped to target_size)."""
    if data_augment:
        raise NotImplementedError("data_augment is a training option")
    r = reader if isinstance(reader, TFRecordFile) else TFRecordFile(reader)
    tsz = tuple(int(s) for s in np.atleast_1d(target_size))
    lsz = tuple(int(s) for s in np.atleast_1d(label_shape))
    for i in range(len(r)):
        label = r.gather("label", [i], np.empty((1, int(np.prod(lsz))), np.float32))[0].reshape(lsz)
        image = r.gather("image", [i], np.empty((1, int(np.prod(tsz))), np.float32))[0].reshape(tsz)
        yield label, image


def inputs(tfrecord_file, num_epochs, image_target_size, label_shape, batch_size, data_augment=False,
           shuffle: bool = True, seed: int = 0, device=None, nthreads: int = 8,
           verify: bool = True) -> Iterator[Tuple[object, object]]:
    """data_loader.py:28-40 as an iterator of (data, labels) batches (see module docstring);
    ``num_epochs=None`` repeats forever like string_input_producer."""
    if data_augment:
        raise NotImplementedError("data_augment is a training option")
    if not os.path.exists(tfrecord_file):
        raise FileNotFoundError(f"{tfrecord_file} not exists")
    r = TFRecordFile(tfrecord_file, verify=verify)
    tsz = tuple(int(s) for s in np.atleast_1d(image_target_size))
    lsz = tuple(int(s) for s in np.atleast_1d(label_shape))
    B = int(batch_size)
    pinned = None
    if device is not None:
        import torch
        pinned = (torch.empty((B,) + tsz, dtype=torch.float32).pin_memory(),
                  torch.empty((B,) + lsz, dtype=torch.float32).pin_memory())
    rng = np.random.default_rng(seed)
    epoch = 0
    while num_epochs is None or epoch < num_epochs:
        order = rng.permutation(len(r)) if shuffle else np.arange(len(r))
        for s in range(0, len(order) - B + 1, B):
            idx = order[s:s + B]
            if pinned is None:
                data = r.gather("image", idx, np.empty((B,) + tsz, np.float32), nthreads)
                labels = r.gather("label", idx, np.empty((B,) + lsz, np.float32), nthreads)
                yield data, labels
            else:
                r.gather("image", idx, pinned[0].numpy(), nthreads)
                r.gather("label", idx, pinned[1].numpy(), nthreads)
                data = pinned[0].to(device, non_blocking=True)
                labels = pinned[1].to(device, non_blocking=True)
                # the next gather reuses the pinned buffers: wait for these copies first
                import torch
                torch.cuda.current_stream(device).synchronize()
                yield data, labels
        epoch += 1


def encode_example(im: np.ndarray, label: np.ndarray) -> bytes:
    """Datareader.py:13-19: one serialized Example {'label': raw bytes, 'image': raw bytes} (via the
    native writer, so the bytes are exactly what create_tf_record writes)."""
    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".tfrecord") as f:
        create_tf_record([im], [label], f.name)
        blob = open(f.name, "rb").read()
    return blob[12:-4]


def create_tf_record(depth_files: Sequence[np.ndarray], lable_files: Sequence[np.ndarray], tf_file: str,
                     config=None, append: bool = False) -> None:
    """Datareader.py:21-27: one Example per (depth, label) pair, raw float32 bytes (``tostring``),
    features in the reference's order ('label', 'image')."""
    depth = np.ascontiguousarray(np.asarray(depth_files, np.float32))
    label = np.ascontiguousarray(np.asarray(lable_files, np.float32))
    n = depth.shape[0]
    if label.shape[0] != n:
        raise ValueError("depth and label counts differ")
    names = (ctypes.c_char_p * 2)(b"label", b"image")
    data = (ctypes.c_void_p * 2)(label.ctypes.data, depth.ctypes.data)
    per = (ctypes.c_int64 * 2)(label[0].nbytes if n else 0, depth[0].nbytes if n else 0)
    _lib.check(_lib.load().mp_tfrecord_write(os.fsencode(tf_file), n, 2, names, data, per, 1 if append else 0))
