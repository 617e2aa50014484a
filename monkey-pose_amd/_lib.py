"""ctypes binding of ``libmonkeypose.so`` (C ABI in ``include/monkeypose.h``).

The library is loaded *after* ``import torch`` so that it binds to the HIP runtime torch already
loaded (both resolve the soname ``libamdhip64.so.7``): device pointers and streams from torch
tensors are then valid inside the library.  There is no CPU fallback: if the library is missing
or the GPU is unavailable every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MP_LIB_PATH") or os.path.join(_HERE, "libmonkeypose.so")

MP_OK = 0
MP_MODEL_HGRU_POSE = 1
MP_MODEL_HGRU_CIRCUIT = 2
MP_MODEL_DENSE = 3
MP_MODEL_HIER = 4
MP_MODEL_ATTN = 5
MP_MODEL_GRAPH = 6
MP_MEM_HOST = 0
MP_MEM_DEVICE = 1
MP_DTYPE_F32 = 0
MP_DTYPE_F32_SPLIT = 1
MP_DTYPE_F32_FFT = 2
MP_DTYPE_BF16 = 3
DTYPES = {'fp32': MP_DTYPE_F32, 'f32': MP_DTYPE_F32, 'fp32_split': MP_DTYPE_F32_SPLIT,
          'f32_split': MP_DTYPE_F32_SPLIT, 'fp32_fft': MP_DTYPE_F32_FFT, 'f32_fft': MP_DTYPE_F32_FFT,
          'bf16': MP_DTYPE_BF16}


def resolve_dtype(name: str, h: int, w: int) -> str:
    """'auto' -> the fastest fp32-class eCRF path supporting an h x w hGRU map: the FFT path for
    maps up to 64 x 64 with width 32 or 64 (the reference's 128^2 / 64^2 crops), else the f16x3
    direct path for multiples of 32, else exact fp32.  Explicit names pass through."""
    if name == 'bf16' and not (1 <= h <= 64 and w in (32, 64)):
        raise ValueError("compute dtype 'bf16' runs on the FFT path: hGRU map height <= 64, width 32 or 64")
    if name != 'auto':
        return name
    if 1 <= h <= 64 and w in (32, 64):
        return 'fp32_fft'
    if h % 32 == 0 and w % 32 == 0:
        return 'fp32_split'
    return 'fp32'


def dtype_code(name: str) -> int:
    if name not in DTYPES:
        raise ValueError(f"compute dtype must be one of {sorted(DTYPES)}, got {name!r}")
    return DTYPES[name]

# every function the header declares, with its ctypes signature
_SIGS = {
    "mp_version": (ctypes.c_int, []),
    "mp_last_error": (ctypes.c_char_p, []),
    "mp_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "mp_destroy": (None, [ctypes.c_void_p]),
    "mp_set_weight": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p,
                                     ctypes.POINTER(ctypes.c_int64), ctypes.c_int, ctypes.c_int]),
    "mp_finalize_weights": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mp_bcast_weights": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int]),
    "mp_reserve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "mp_hgru_pose_fwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "mp_hgru_pose_fwd_taps": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mp_hgru_circuit_fwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "mp_hgru_circuit_fwd_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mp_hgru_pose_fwd_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mp_hgru_circuit_fwd_opts": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p]),
    "mp_dense_fwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "mp_hier_fwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                   ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "mp_attn_fwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                   ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "mp_resize_bilinear": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "mp_graph_set": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_int]),
    "mp_graph_fwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "mp_tfrecord_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_int64)]),
    "mp_tfrecord_close": (None, [ctypes.c_void_p]),
    "mp_tfrecord_feature_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p,
                                                ctypes.POINTER(ctypes.c_int64)]),
    "mp_tfrecord_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]),
    "mp_tfrecord_write": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "mp_crc32c": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    "mp_hbm_probe": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p]),
    "mp_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "mp_profile_enable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mp_profile_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p,
                                       ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_int64)]),
}

_lib: Optional[ctypes.CDLL] = None

# mp_pose_taps field order (include/monkeypose.h)
TAP_NAMES = ("conv1", "pool1", "conv2", "conv3", "hgru", "fc1", "relu1")
STATE_NAMES = ("states_O", "states_I")      # store_states stacks [n, T, h/2, w/2, 64]

# ContextualCircuit aux 'hidden_init' (hgru_module.py:875-892) -> MP_HIDDEN_*: 'random' with an
# explicit draw is MP_HIDDEN_GIVEN; without one the library draws it on the device (MP_HIDDEN_RANDOM)
MP_HIDDEN = {"random": 0, "zeros": 1, "identity": 2}
MP_HIDDEN_GIVEN, MP_HIDDEN_RANDOM = 0, 3
MP_ABI_VERSION = (0, 2)


class PoseTaps(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in TAP_NAMES]


class FwdOpts(ctypes.Structure):
    """``mp_fwd_opts`` (include/monkeypose.h, since 0.2)."""
    _fields_ = [("struct_size", ctypes.c_uint64), ("hidden_init", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("rng_seed", ctypes.c_uint64), ("rng_call", ctypes.c_uint64), ("states_O", ctypes.c_void_p),
                ("states_I", ctypes.c_void_p), ("taps", ctypes.c_void_p)]


def fwd_opts(hidden_init: int = 0, rng_seed: int = 0, rng_call: int = 0, states_O=None, states_I=None,
             taps: Optional[PoseTaps] = None) -> FwdOpts:
    o = FwdOpts()
    o.struct_size = ctypes.sizeof(FwdOpts)
    o.hidden_init = int(hidden_init)
    o.rng_seed = int(rng_seed) & 0xFFFFFFFFFFFFFFFF
    o.rng_call = int(rng_call) & 0xFFFFFFFFFFFFFFFF
    o.states_O, o.states_I = _ptr(states_O), _ptr(states_I)
    o.taps = None if taps is None else ctypes.addressof(taps)
    return o


class MonkeyPoseError(RuntimeError):
    """A non-zero status from the C ABI; ``code`` is the MP_ERR_* value."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def load() -> ctypes.CDLL:
    """Load (once) and return the library; raises if it has not been built."""
    global _lib
    if _lib is None:
        import torch  # noqa: F401  -- binds the library to torch's HIP runtime
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import "
                               "__graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.mp_version()
        if (v >> 16, v & 0xFFFF) < MP_ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH} is ABI {v >> 16}.{v & 0xFFFF}, this package needs "
                               f"{MP_ABI_VERSION[0]}.{MP_ABI_VERSION[1]}: rebuild it")
        _lib = lib
    return _lib


def check(status: int) -> None:
    if status != MP_OK:
        raise MonkeyPoseError(status, load().mp_last_error().decode())


def _ptr(t):
    return None if t is None else int(t.data_ptr())


class Context:
    """One ``mp_ctx`` on one device (the unit the reference's tf.Session/device placement maps to)."""

    def __init__(self, model_kind: int, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("monkey-pose_amd needs a ROCm GPU; there is no CPU fallback")
        self.lib = load()
        self.device = device
        h = ctypes.c_void_p()
        check(self.lib.mp_create(device, model_kind, ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.mp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_weight(self, name: str, value) -> None:
        import torch
        if isinstance(value, torch.Tensor):
            t = value.detach()
            if t.dtype != torch.float32:
                t = t.float()
            t = t.contiguous()
            shape = (ctypes.c_int64 * t.dim())(*t.shape)
            mem = MP_MEM_DEVICE if t.is_cuda else MP_MEM_HOST
            if t.is_cuda:
                torch.cuda.synchronize(t.device)   # the copy below runs on the null stream
            check(self.lib.mp_set_weight(self.h, name.encode(), ctypes.c_void_p(t.data_ptr()), shape,
                                         t.dim(), mem))
        else:
            a = np.ascontiguousarray(np.asarray(value, dtype=np.float32))
            shape = (ctypes.c_int64 * a.ndim)(*a.shape)
            check(self.lib.mp_set_weight(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                         shape, a.ndim, MP_MEM_HOST))

    def finalize(self, dtype: int = MP_DTYPE_F32) -> None:
        check(self.lib.mp_finalize_weights(self.h, dtype))

    def reserve(self, max_batch: int) -> None:
        check(self.lib.mp_reserve(self.h, int(max_batch)))

    def info(self, key: str) -> int:
        v = ctypes.c_int64()
        check(self.lib.mp_info(self.h, key.encode(), ctypes.byref(v)))
        return int(v.value)

    def pose_fwd(self, depth, o0, out, stream: int) -> None:
        n, h, w, c = depth.shape
        check(self.lib.mp_hgru_pose_fwd(self.h, _ptr(depth), n, h, w, _ptr(o0), _ptr(out),
                                        ctypes.c_void_p(stream)))

    def pose_fwd_taps(self, depth, o0, out, taps: dict, stream: int, hidden_init: int = 0, rng_seed: int = 0,
                      rng_call: int = 0) -> None:
        """mp_hgru_pose_fwd_ex; ``taps`` maps names of TAP_NAMES / STATE_NAMES to CUDA output
        tensors; ``o0`` may be None unless ``hidden_init`` is MP_HIDDEN_GIVEN; MP_HIDDEN_RANDOM
        draws O0 on the device from (rng_seed + rng_call)."""
        n, h, w, c = depth.shape
        t = None
        if any(k in taps for k in TAP_NAMES):
            t = PoseTaps(*[ctypes.c_void_p(_ptr(taps[k]) if k in taps else None) for k in TAP_NAMES])
        o = fwd_opts(hidden_init, rng_seed, rng_call, taps.get("states_O"), taps.get("states_I"), t)
        check(self.lib.mp_hgru_pose_fwd_ex(self.h, _ptr(depth), n, h, w, _ptr(o0), _ptr(out), ctypes.byref(o),
                                           ctypes.c_void_p(stream)))

    def circuit_fwd(self, x, o0, out, timesteps: int, stream: int, hidden_init: int = 0, states_O=None,
                    states_I=None, rng_seed: int = 0, rng_call: int = 0) -> None:
        n, h, w, k = x.shape
        o = fwd_opts(hidden_init, rng_seed, rng_call, states_O, states_I)
        check(self.lib.mp_hgru_circuit_fwd_opts(self.h, _ptr(x), _ptr(o0), n, h, w, k, int(timesteps), _ptr(out),
                                                ctypes.byref(o), ctypes.c_void_p(stream)))

    def dense_fwd(self, depth, out, stream: int) -> None:
        n, h, w, c = depth.shape
        check(self.lib.mp_dense_fwd(self.h, _ptr(depth), n, h, w, _ptr(out), ctypes.c_void_p(stream)))

    def hier_fwd(self, depth, outs, stream: int) -> None:
        n, h, w, c = depth.shape
        arr = (ctypes.c_void_p * 6)(*[_ptr(o) for o in outs])
        check(self.lib.mp_hier_fwd(self.h, _ptr(depth), n, h, w, arr, ctypes.c_void_p(stream)))

    def graph_fwd(self, x, outs, stream: int) -> None:
        n, h, w, c = x.shape
        arr = (ctypes.c_void_p * len(outs))(*[_ptr(o) for o in outs])
        check(self.lib.mp_graph_fwd(self.h, _ptr(x), n, h, w, arr, ctypes.c_void_p(stream)))

    def attn_fwd(self, frames, out, stream: int) -> None:
        n, h, w, c = frames.shape
        check(self.lib.mp_attn_fwd(self.h, _ptr(frames), n, h, w, _ptr(out), ctypes.c_void_p(stream)))

    def profile(self, enable: bool) -> None:
        check(self.lib.mp_profile_enable(self.h, 1 if enable else 0))

    def profile_read(self, name: str):
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        check(self.lib.mp_profile_read(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(cnt)))
        return float(ms.value), int(cnt.value)


def resize_bilinear(x, size, stream: Optional[int] = None):
    """``tf.image.resize_images(x, size)`` (TF1 BILINEAR, align_corners=False) of a CUDA tensor
    [n, h, w, c] fp32 -> new tensor [n, size[0], size[1], c] (mp_resize_bilinear)."""
    import torch
    if not isinstance(x, torch.Tensor) or not x.is_cuda or x.dim() != 4:
        raise TypeError("x must be a 4-D CUDA (ROCm) tensor [n, h, w, c]")
    x = x.detach().float().contiguous()
    n, h, w, c = x.shape
    out = torch.empty((n, int(size[0]), int(size[1]), c), dtype=torch.float32, device=x.device)
    st = current_stream(x.device) if stream is None else stream
    check(load().mp_resize_bilinear(_ptr(x), n, h, w, c, int(size[0]), int(size[1]), _ptr(out),
                                    ctypes.c_void_p(st)))
    return out


def current_stream(device=None) -> int:
    import torch
    return int(torch.cuda.current_stream(device).cuda_stream)


class HbmRates(ctypes.Structure):
    """mp_hbm_rates (include/monkeypose.h)"""
    _fields_ = [("read_gbps", ctypes.c_double), ("write_gbps", ctypes.c_double), ("copy_gbps", ctypes.c_double)] + \
               [(f"{k}_{f}", ctypes.c_int32) for k in ("read", "write", "copy") for f in ("grid", "unroll", "nt")]


def hbm_probe(device: int = 0, nbytes: int = 2 << 30) -> dict:
    """The box's streaming HBM read / write / copy rates (GB/s) and the access form that reached
    each (mp_hbm_probe; synchronous, allocates two nbytes buffers)."""
    r = HbmRates()
    check(load().mp_hbm_probe(int(device), int(nbytes), ctypes.byref(r)))
    out = {}
    for k in ("read", "write", "copy"):
        out[f"{k}_GBps"] = round(getattr(r, f"{k}_gbps"), 1)
        out[f"{k}_form"] = {"grid": getattr(r, f"{k}_grid"), "per_thread": getattr(r, f"{k}_unroll"),
                            "nontemporal": bool(getattr(r, f"{k}_nt"))}
    return out
