"""Drop-in for ``/root/reference/monkeydetector.py`` / ``tf_monkeydetector.py`` (inference geometry).

``MonkeyDetector(fx, fy, ux, uy, cube, d1, d2).cropArea3D(dpt, com)`` -> (crop, M, com) runs in
native code (``mp_crop3d`` in libmonkeypose.so, host C++, bit-exact integer bounds / sizes /
offsets / nearest-neighbour indices); ``crop_batch`` is the reference's per-frame loop
(``prepare_data_test``, train_cnn_networks_hgru.py:61-74) in one call, producing the normalised
model input directly.  The small joint-coordinate transforms are vectorised numpy.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib


class _Camera(ctypes.Structure):
    _fields_ = [("fx", ctypes.c_double), ("fy", ctypes.c_double), ("ux", ctypes.c_double),
                ("uy", ctypes.c_double), ("cube", ctypes.c_double * 3),
                ("min_depth", ctypes.c_double), ("max_depth", ctypes.c_double)]


_CROP_SIGS = {
    "mp_center_of_mass": (ctypes.c_int, [ctypes.POINTER(_Camera), ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]),
    "mp_crop3d": (ctypes.c_int, [ctypes.POINTER(_Camera), ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                 ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mp_crop3d_ex": (ctypes.c_int, [ctypes.POINTER(_Camera), ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mp_crop3d_batch": (ctypes.c_int, [ctypes.POINTER(_Camera), ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int]),
    "mp_crop3d_dev": (ctypes.c_int, [ctypes.POINTER(_Camera), ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]),
    "mp_crop3d_dev_ex": (ctypes.c_int, [ctypes.POINTER(_Camera), ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
}

_CROP_MSG = {1: "CoM depth is zero or not finite (no valid pixel in range?)", 2: "empty crop",
             3: "degenerate bounds", 4: "resize target is empty"}


def _lib_crop():
    lib = _lib.load()
    if not getattr(lib, "_crop_bound", False):
        for name, (res, args) in _CROP_SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        lib._crop_bound = True
    return lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class MonkeyDetector(object):
    """``MonkeyDetector`` (monkeydetector.py:21-63)."""

    RESIZE_BILINEAR = 0
    RESIZE_CV2_NN = 1
    RESIZE_CV2_LINEAR = 2

    def __init__(self, fx, fy, ux, uy, cube, d1, d2, importer=None):
        if len(cube) != 3:
            raise ValueError("Volume must be 3D")
        self.maxDepth = d2
        self.minDepth = d1
        self.fx, self.fy, self.ux, self.uy = fx, fy, ux, uy
        self.cube = cube
        self.resizeMethod = self.RESIZE_CV2_NN

    def _cam(self) -> _Camera:
        return _Camera(float(self.fx), float(self.fy), float(self.ux), float(self.uy),
                       (ctypes.c_double * 3)(*[float(c) for c in self.cube]), float(self.minDepth),
                       float(self.maxDepth))

    @staticmethod
    def _frame(dpt, ndim=2):
        """(contiguous array, MP_DEPTH_* code): uint16 frames keep their numpy semantics (exact CoM
        sum, truncating near-plane clamp); anything else is computed as float32 like the
        reference's float32 frames."""
        a = np.asarray(dpt)
        if a.ndim != ndim:
            raise NotImplementedError(f"expected {ndim}-D single-channel depth, got shape {a.shape}")
        if a.dtype == np.uint16:
            return np.ascontiguousarray(a), 1
        return np.ascontiguousarray(a, dtype=np.float32), 0

    # ------------------------------------------------------------------ native
    def calculateCoM(self, dpt):
        """monkeydetector.py:66-83 (float32 frame in mm; a uint16 frame is converted exactly)."""
        f, dt = self._frame(dpt)
        com = np.zeros(3, np.float64)
        cam = self._cam()
        _lib.check(_lib_crop().mp_center_of_mass(ctypes.byref(cam), _p(f), dt, f.shape[0], f.shape[1], _p(com)))
        return com

    def cropArea3D(self, dpt, com=None, dsize=(128, 128), docom=False):
        """monkeydetector.py:261-334 -> (crop [dsize] float32 mm, M 3x3 numpy matrix, com);
        ``docom=True`` runs the second refinement (287-300): a CoM of the first crop, a second crop
        around it, and the refined CoM returned."""
        if self.resizeMethod != self.RESIZE_CV2_NN:
            raise NotImplementedError("only RESIZE_CV2_NN (the reference default) is implemented")
        if len(dsize) != 2 or dsize[0] != dsize[1]:
            raise ValueError("dsize must be a square 2D bounding box")
        f, dt = self._frame(dpt)
        out = np.empty((dsize[0], dsize[1]), np.float32)
        M = np.zeros(9, np.float64)
        com_out = np.zeros(3, np.float64)
        info = np.zeros(8, np.int32)
        c = None if com is None else np.ascontiguousarray(np.asarray(com, np.float64).reshape(3))
        cam = self._cam()
        _lib.check(_lib_crop().mp_crop3d_ex(ctypes.byref(cam), _p(f), dt, f.shape[0], f.shape[1],
                                            None if c is None else _p(c), 1 if docom else 0, dsize[0], _p(out),
                                            _p(M), _p(com_out), _p(info)))
        self.last_crop_info = dict(bounds=tuple(int(v) for v in info[:4]), sz=(int(info[4]), int(info[5])),
                                   offset=(int(info[6]), int(info[7])))
        return out, np.asmatrix(M.reshape(3, 3)), com_out

    def crop_batch(self, frames, coms=None, dsize=128, nthreads=None, out=None):
        """Per-frame crop of ``prepare_data_test`` (train_cnn_networks_hgru.py:61-74) in one native
        call: returns (patches [n, dsize, dsize, 1] = crop / maxDepth, Ms [n, 3, 3], coms [n, 3]).
        ``out``: a C-contiguous float32 [n, dsize, dsize, 1] array the patches are written into (and
        returned as ``patches``), e.g. a reused or pinned staging buffer."""
        fr, dt = self._frame(frames, ndim=3)
        n = fr.shape[0]
        if out is None:
            patches = np.empty((n, dsize, dsize, 1), np.float32)
        else:
            if not (isinstance(out, np.ndarray) and out.dtype == np.float32 and out.flags.c_contiguous
                    and out.shape == (n, dsize, dsize, 1)):
                raise ValueError(f"out must be a C-contiguous float32 array of shape {(n, dsize, dsize, 1)}")
            patches = out
        Ms = np.empty((n, 9), np.float64)
        com_out = np.empty((n, 3), np.float64)
        c = None if coms is None else np.ascontiguousarray(np.asarray(coms, np.float64).reshape(n, 3))
        nt = nthreads or min(16, len(os.sched_getaffinity(0)))
        cam = self._cam()
        _lib.check(_lib_crop().mp_crop3d_batch(ctypes.byref(cam), _p(fr), dt, n, fr.shape[1], fr.shape[2],
                                               None if c is None else _p(c), dsize, _p(patches), _p(Ms),
                                               _p(com_out), int(nt)))
        return patches, Ms.reshape(n, 3, 3), com_out

    def crop_batch_device(self, frames, com_norm, com_scale=(424, 512, 10000.), frame_scale=10000.,
                          dsize=128, check=True, stream=None, docom=False):
        """``prepare_data_test`` (train_cnn_networks_hgru.py:61-74) on the GPU for a batch, with
        ``tr_res`` = the attention output still on the device (``mp_crop3d_dev``, one launch):

        frames     CUDA [n, h, w] or [n, h, w, 1] fp32 as fed to the attention net (image / max depth)
        com_norm   CUDA [n, 3] fp32 attention output; com = com_norm * com_scale (float64)
        returns    (patches CUDA [n, dsize, dsize, 1] = crop / maxDepth, Ms CUDA [n, 3, 3] f64,
                    coms CUDA [n, 3] f64); with ``check`` the per-frame status is read back (one
                    sync) and a failed frame raises like the host ``cropArea3D``.  ``docom``: the
                    second CoM refinement of ``cropArea3D(docom=True)`` per frame, on the device."""
        import torch
        if not (isinstance(frames, torch.Tensor) and frames.is_cuda and isinstance(com_norm, torch.Tensor)
                and com_norm.is_cuda):
            raise TypeError("frames and com_norm must be CUDA (ROCm) tensors")
        if frames.dim() == 4:
            if frames.shape[-1] != 1:
                raise ValueError("frames must be single-channel")
            frames = frames[..., 0]
        if frames.dim() != 3:
            raise ValueError(f"frames must be [n, h, w], got {tuple(frames.shape)}")
        fr = frames.detach().float().contiguous()
        n, h, w = fr.shape
        cn = com_norm.detach().float().contiguous().view(n, 3)
        dev = fr.device
        patches = torch.empty((n, dsize, dsize, 1), dtype=torch.float32, device=dev)
        Ms = torch.empty((n, 3, 3), dtype=torch.float64, device=dev)
        coms = torch.empty((n, 3), dtype=torch.float64, device=dev)
        status = torch.empty((n,), dtype=torch.int32, device=dev)
        scale = (ctypes.c_double * 3)(*[float(v) for v in com_scale])   # host array (read at the call)
        st = _lib.current_stream(dev) if stream is None else stream
        cam = self._cam()
        _lib.check(_lib_crop().mp_crop3d_dev_ex(ctypes.byref(cam), ctypes.c_void_p(fr.data_ptr()), n, h, w,
                                                float(frame_scale), ctypes.c_void_p(cn.data_ptr()),
                                                ctypes.cast(scale, ctypes.c_void_p), 1 if docom else 0, int(dsize),
                                             ctypes.c_void_p(patches.data_ptr()), ctypes.c_void_p(Ms.data_ptr()),
                                             ctypes.c_void_p(coms.data_ptr()), ctypes.c_void_p(status.data_ptr()),
                                             ctypes.c_void_p(st)))
        self.last_status = status
        if check:
            bad = torch.nonzero(status).flatten().tolist()
            if bad:
                code = int(status[bad[0]].item())
                raise _lib.MonkeyPoseError(-1, f"frame {bad[0]}: cropArea3D: {_CROP_MSG.get(code, code)}")
        return patches, Ms, coms

    # ------------------------------------------------------------------ geometry (host numpy)
    def comToBounds(self, com, size):
        """monkeydetector.py:162-175."""
        zstart = com[2] - size[2] / 2.
        zend = com[2] + size[2] / 2.
        xstart = int(np.floor((com[0] * com[2] / self.fx - size[0] / 2.) / com[2] * self.fx))
        xend = int(np.floor((com[0] * com[2] / self.fx + size[0] / 2.) / com[2] * self.fx))
        ystart = int(np.floor((com[1] * com[2] / self.fy - size[1] / 2.) / com[2] * self.fy))
        yend = int(np.floor((com[1] * com[2] / self.fy + size[1] / 2.) / com[2] * self.fy))
        return xstart, xend, ystart, yend, zstart, zend

    def xyztouvd(self, jnts_xyz):
        """monkeydetector.py:85-112 / tf_monkeydetector.py:116-141 (float32 output; z == 0 maps to the
        principal point).  The reference's scalar arithmetic under NumPy 1.x: ``x / z`` in the joints'
        own dtype (float32 / float32 is a float32 division), then ``* fx`` and ``ux -`` in float64
        (a float32 scalar with a Python float promotes), one rounding to float32 on the store."""
        j = np.asarray(jnts_xyz)
        one = j.ndim == 1
        j = np.atleast_2d(j)
        if j.dtype.kind != "f":
            j = j.astype(np.float64)
        out = np.zeros((j.shape[0], 3), np.float32)
        z = j[:, 2]
        nz = z != 0.
        out[~nz, 0], out[~nz, 1] = self.ux, self.uy
        qx = (j[nz, 0] / z[nz]).astype(np.float64)
        qy = (j[nz, 1] / z[nz]).astype(np.float64)
        out[nz, 0] = self.ux - qx * self.fx
        out[nz, 1] = qy * self.fy + self.uy
        out[nz, 2] = -z[nz]
        return out[0] if one else out

    def xyztouvd_np(self, jnts_xyz):
        return self.xyztouvd(jnts_xyz)

    def uvdtoxyz(self, jnts_uvd):
        """monkeydetector.py:114-131."""
        u = np.asarray(jnts_uvd)
        one = u.ndim == 1
        u = np.atleast_2d(u).astype(np.float64)
        out = np.empty((u.shape[0], 3), np.float32)
        out[:, 0] = (self.ux - u[:, 0]) * u[:, 2] / (-self.fx)
        out[:, 1] = (u[:, 1] - self.uy) * u[:, 2] / (-self.fy)
        out[:, 2] = -u[:, 2]
        return out[0] if one else out

    def calcCoMRenders(self, jnts):
        assert jnts.ndim == 2, 'input must be the 3D coordinates of all monkey joints'
        return np.sum(jnts, axis=0) / jnts.shape[0]

    @staticmethod
    def transformPoint2D(pt, M):
        p = np.asarray(M, np.float64).reshape(3, 3) @ np.array([pt[0], pt[1], 1.0])
        return np.array([p[0] / p[2], p[1] / p[2]])

    def getRelativeCoordinates(self, jnts_xyz, jnts_uvd, com_uvd, M):
        """monkeydetector.py:341-354."""
        rel_xyz = jnts_xyz - self.uvdtoxyz(com_uvd)
        Mm = np.asarray(M, np.float64).reshape(3, 3)
        uv1 = np.c_[np.asarray(jnts_uvd, np.float64)[:, :2], np.ones(len(jnts_uvd))]
        t = uv1 @ Mm.T
        rel_uvd = np.zeros((len(jnts_uvd), 3), np.float32)
        rel_uvd[:, 0] = t[:, 0] / t[:, 2]
        rel_uvd[:, 1] = t[:, 1] / t[:, 2]
        rel_uvd[:, 2] = np.asarray(jnts_uvd)[:, 2]
        return rel_xyz, rel_uvd

    def getAbsoluteCoordinates(self, rel_jnts_xyz, com_uvd):
        """monkeydetector.py:356-360 / tf_monkeydetector.py:387-391 (A19 post-step)."""
        r = rel_jnts_xyz
        c = np.asarray(com_uvd)
        if (isinstance(r, np.ndarray) and r.dtype == np.float32 and r.ndim == 2 and r.shape[1] == 3
                and c.shape == (3,) and c.dtype.kind == "f"):
            # one joint set per frame (the config-5 loop): uvdtoxyz of the CoM as Python float64
            # scalars (the same IEEE double operations numpy runs elementwise), one float32 rounding
            # each, then xyztouvd's operations on whole columns when no joint has z == 0
            u0, u1, u2 = float(c[0]), float(c[1]), float(c[2])
            cxyz = np.array([(self.ux - u0) * u2 / (-self.fx), (u1 - self.uy) * u2 / (-self.fy), -u2], np.float32)
            jnts_xyz = r + cxyz
            z = jnts_xyz[:, 2]
            if z.all():
                q = (jnts_xyz[:, :2] / z[:, None]).astype(np.float64)
                uvd = np.empty((r.shape[0], 3), np.float32)
                uvd[:, 0] = self.ux - q[:, 0] * self.fx
                uvd[:, 1] = q[:, 1] * self.fy + self.uy
                uvd[:, 2] = -z
                return jnts_xyz, uvd
            return jnts_xyz, self.xyztouvd(jnts_xyz)
        jnts_xyz = rel_jnts_xyz + self.uvdtoxyz(com_uvd)
        return jnts_xyz, self.xyztouvd(jnts_xyz)


# tf_monkeydetector.tfMonkeyDetector shares this inference API (tf_monkeydetector.py:21-391)
tfMonkeyDetector = MonkeyDetector
