"""CPU ORACLE (test infrastructure only; import rule as in oracle/hgru_ref.py).

Restatement of the host crop / geometry path used around the pose regressors:

* ``MonkeyDetector.calculateCoM``   /root/reference/monkeydetector.py:66-83
* ``comToBounds``                   monkeydetector.py:162-175 (= tf_monkeydetector.py:193-206)
* ``getCrop``                       monkeydetector.py:177-213
* ``resizeCrop`` (RESIZE_CV2_NN)    monkeydetector.py:215-230
* ``cropArea3D``                    monkeydetector.py:261-334 (= tf_monkeydetector.py:292-365)
* ``xyztouvd`` / ``uvdtoxyz``       monkeydetector.py:85-131; ``transformPoint2D`` 336-339;
  ``getRelativeCoordinates`` 341-354; ``getAbsoluteCoordinates`` 356-360

Third-party arithmetic restated from its published algorithm (not importable here, PARITY
UNPINNED for these pieces):
* OpenCV ``cv2.resize(..., INTER_NEAREST)`` (resizeNN): ``inv = dst/src`` (double), ``ifx =
  1/inv``, ``sx = min(floor(x*ifx), src-1)``.
* SciPy ``ndimage.center_of_mass(mask)``: mean row / column index of the mask (exact in float64).
* NumPy float32 ``ndarray.sum()``: pairwise summation (blocks of 128, 8 partial sums) -- restated in
  ``np_pairwise_sum_f32`` and checked against numpy itself in the tests.
Python 2 integer division in ``sz`` (monkeydetector.py:296-299) is floor division.

The era's NumPy (<= 1.16, Python 2.7) casts scalars by value: a float32 array compared with a
float64 scalar (getCrop's ``cropped < zstart`` / ``cropped > zend``, 209-210; calculateCoM's
``dc < minDepth`` / ``dc > maxDepth``, 74-75) compares in float32 against f32(scalar) (``_lcmp``);
a uint16 array compares in float64.  NumPy 2 (NEP 50) would compare in float64 throughout.
Pinned by fixtures from the reference's own code, executed here (tests/golden/make_crop_fixtures.py).
"""
from __future__ import annotations

import math

import numpy as np
from scipy import ndimage

FX = FY = 365.456          # train_cnn_networks_hgru.py:77
UX, UY = 256.0, 212.0
CUBE = (800.0, 800.0, 1200.0)
MIN_DEPTH, MAX_DEPTH = 200.0, 10000.0


def _lscalar(arr: np.ndarray, s: float):
    """the scalar as NumPy 1.x value-based casting sees it against ``arr`` (see the header)"""
    if arr.dtype == np.float32 and -3.4e38 < s < 3.4e38:
        return np.float32(s)
    return np.float64(s)


def np_pairwise_sum_f32(a: np.ndarray) -> np.float32:
    """numpy 1.x's float32 pairwise summation over a contiguous array (loops_utils.h.src): blocks of
    <= 128 summed into 8 partial sums, halves split at multiples of 8."""
    flat = np.ascontiguousarray(a, dtype=np.float32).reshape(-1)

    def rec(lo, n):
        if n < 8:
            r = np.float32(0)
            for i in range(n):
                r = np.float32(r + flat[lo + i])
            return r
        if n <= 128:
            r = flat[lo:lo + 8].copy()            # the 8 partial sums, one float32 add per element
            i = 8
            while i < n - (n % 8):
                r += flat[lo + i:lo + i + 8]
                i += 8
            res = np.float32(np.float32(np.float32(r[0] + r[1]) + np.float32(r[2] + r[3])) +
                             np.float32(np.float32(r[4] + r[5]) + np.float32(r[6] + r[7])))
            while i < n:
                res = np.float32(res + flat[lo + i])
                i += 1
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return np.float32(rec(lo, n2) + rec(lo + n2, n - n2))

    return np.float32(np.float32(0) + rec(0, flat.size))


class MonkeyDetectorRef:
    def __init__(self, fx=FX, fy=FY, ux=UX, uy=UY, cube=CUBE, d1=MIN_DEPTH, d2=MAX_DEPTH):
        self.fx, self.fy, self.ux, self.uy = fx, fy, ux, uy
        self.cube = cube
        self.minDepth, self.maxDepth = d1, d2

    def calculateCoM(self, dpt):
        dc = dpt.copy()
        dc[dc < _lscalar(dc, self.minDepth)] = 0
        dc[dc > _lscalar(dc, self.maxDepth)] = 0
        cc = ndimage.center_of_mass(dc > 0)
        num = np.count_nonzero(dc)
        if num == 0:
            return np.array((0, 0, 0), np.float64)
        s = np_pairwise_sum_f32(dc) if dc.dtype == np.float32 else dc.sum()
        com = np.array((cc[1] * num, cc[0] * num, s), np.float64)
        return com / num

    def comToBounds(self, com, size):
        zstart = com[2] - size[2] / 2.
        zend = com[2] + size[2] / 2.
        xstart = int(math.floor((com[0] * com[2] / self.fx - size[0] / 2.) / com[2] * self.fx))
        xend = int(math.floor((com[0] * com[2] / self.fx + size[0] / 2.) / com[2] * self.fx))
        ystart = int(math.floor((com[1] * com[2] / self.fy - size[1] / 2.) / com[2] * self.fy))
        yend = int(math.floor((com[1] * com[2] / self.fy + size[1] / 2.) / com[2] * self.fy))
        return xstart, xend, ystart, yend, zstart, zend

    def getCrop(self, dpt, xstart, xend, ystart, yend, zstart, zend, thresh_z=True):
        cropped = dpt[max(ystart, 0):min(yend, dpt.shape[0]), max(xstart, 0):min(xend, dpt.shape[1])].copy()
        cropped = np.pad(cropped, ((abs(ystart) - max(ystart, 0), abs(yend) - min(yend, dpt.shape[0])),
                                   (abs(xstart) - max(xstart, 0), abs(xend) - min(xend, dpt.shape[1]))),
                         mode='constant', constant_values=0)
        if thresh_z is True:
            msk1 = np.bitwise_and(cropped < _lscalar(cropped, zstart), cropped != 0)
            msk2 = np.bitwise_and(cropped > _lscalar(cropped, zend), cropped != 0)
            cropped[msk1] = zstart
            cropped[msk2] = 0.
        return cropped

    @staticmethod
    def resize_nn(src, sz):
        """cv2.resize(src, sz=(width, height), interpolation=INTER_NEAREST)."""
        dw, dh = int(sz[0]), int(sz[1])
        sh, sw = src.shape[:2]
        ifx = 1.0 / (dw / sw)
        ify = 1.0 / (dh / sh)
        xs = np.array([min(int(math.floor(x * ifx)), sw - 1) for x in range(dw)], np.int64)
        ys = np.array([min(int(math.floor(y * ify)), sh - 1) for y in range(dh)], np.int64)
        return src[ys][:, xs]

    def cropArea3D(self, dpt, com=None, dsize=(128, 128), docom=False):
        if com is None:
            com = self.calculateCoM(dpt)
        xstart, xend, ystart, yend, zstart, zend = self.comToBounds(com, self.cube)
        cropped = self.getCrop(dpt, xstart, xend, ystart, yend, zstart, zend)
        if docom:                                           # monkeydetector.py:287-300
            com = self.calculateCoM(cropped)
            if np.allclose(com, 0.):
                com[2] = cropped[cropped.shape[0] // 2, cropped.shape[1] // 2]
                if np.isclose(com[2], 0):
                    com[2] = 300.
            com[0] += xstart
            com[1] += ystart
            xstart, xend, ystart, yend, zstart, zend = self.comToBounds(com, self.cube)
            cropped = self.getCrop(dpt, xstart, xend, ystart, yend, zstart, zend)
        wb = (xend - xstart)
        hb = (yend - ystart)
        trans = np.eye(3)
        trans[0, 2] = -xstart
        trans[1, 2] = -ystart
        if wb > hb:
            sz = (dsize[0], hb * dsize[0] // wb)             # Py2 integer '/'
        else:
            sz = (wb * dsize[1] // hb, dsize[1])
        if cropped.shape[0] > cropped.shape[1]:
            scale = np.eye(3) * sz[1] / float(cropped.shape[0])
        else:
            scale = np.eye(3) * sz[0] / float(cropped.shape[1])
        scale[2, 2] = 1
        rz = self.resize_nn(cropped, sz)
        ret = np.ones(dsize, np.float32) * self.maxDepth
        xs = int(math.floor(dsize[0] / 2. - rz.shape[1] / 2.))
        ys = int(math.floor(dsize[1] / 2. - rz.shape[0] / 2.))
        ret[ys:ys + rz.shape[0], xs:xs + rz.shape[1]] = rz
        off = np.eye(3)
        off[0, 2] = xs
        off[1, 2] = ys
        M = off @ scale @ trans
        info = dict(bounds=(xstart, xend, ystart, yend), sz=sz, offset=(xs, ys))
        return ret, M, com, info

    # ---- coordinate transforms (float32 outputs as in the reference) ----
    def xyztouvd(self, j):
        out = np.zeros((j.shape[0], 3), np.float32)
        for i in range(j.shape[0]):
            if j[i, 2] == 0.:
                out[i, 0], out[i, 1] = self.ux, self.uy
                continue
            out[i, 0] = self.ux - j[i, 0] / j[i, 2] * self.fx
            out[i, 1] = j[i, 1] / j[i, 2] * self.fy + self.uy
            out[i, 2] = -j[i, 2]
        return out

    def uvdtoxyz(self, u):
        if u.ndim == 1:
            o = np.zeros((3,), np.float32)
            o[0] = (self.ux - u[0]) * u[2] / (-self.fx)
            o[1] = (u[1] - self.uy) * u[2] / (-self.fy)
            o[2] = -u[2]
            return o
        o = np.zeros((u.shape[0], 3), np.float32)
        for i in range(u.shape[0]):
            o[i, 0] = (self.ux - u[i, 0]) * u[i, 2] / (-self.fx)
            o[i, 1] = (u[i, 1] - self.uy) * u[i, 2] / (-self.fy)
            o[i, 2] = -u[i, 2]
        return o

    @staticmethod
    def transformPoint2D(pt, M):
        p2 = M.reshape(3, 3) @ np.array([pt[0], pt[1], 1.0])
        return np.array([p2[0] / p2[2], p2[1] / p2[2]])

    def getRelativeCoordinates(self, jnts_xyz, jnts_uvd, com_uvd, M):
        rel_xyz = jnts_xyz - self.uvdtoxyz(com_uvd)
        rel_uvd = np.zeros((jnts_uvd.shape[0], 3), np.float32)
        for k in range(jnts_uvd.shape[0]):
            t = self.transformPoint2D(jnts_uvd[k], M)
            rel_uvd[k, 0], rel_uvd[k, 1], rel_uvd[k, 2] = t[0], t[1], jnts_uvd[k, 2]
        return rel_xyz, rel_uvd

    def getAbsoluteCoordinates(self, rel_jnts_xyz, com_uvd):
        jnts_xyz = rel_jnts_xyz + self.uvdtoxyz(com_uvd)
        return jnts_xyz, self.xyztouvd(jnts_xyz)


def synth_frame(seed: int, h: int = 424, w: int = 512, dtype=np.float32, integer=True):
    """A synthetic Kinect-like frame in mm: far wall ~3000-4000, a blob body at 800-1500, zero
    dropout, a few saturated (> maxDepth) pixels."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    f = 3000.0 + 1000.0 * rng.random() + 200.0 * np.sin(xx / 37.0) * np.cos(yy / 23.0)
    cy, cx = rng.uniform(0.2, 0.8) * h, rng.uniform(0.2, 0.8) * w
    ry, rx = rng.uniform(30, 90), rng.uniform(30, 90)
    body = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 < 1
    f = np.where(body, rng.uniform(800, 1500) + 50 * ((yy - cy) / ry) ** 2, f)
    f[rng.random((h, w)) < 0.03] = 0.0
    f[rng.random((h, w)) < 0.003] = 12000.0
    if integer:
        f = np.round(f)
    return f.astype(dtype)


def prepare_data_test(frames_norm: np.ndarray, tr_res: np.ndarray, md: "MonkeyDetectorRef",
                      orig_size=(424, 512), max_depth: float = 10000.0, dsize: int = 128):
    """train_cnn_networks_hgru.py:61-74 with float32 frames [n, h, w(, 1)] (image / max depth) and
    the attention output tr_res [n, 3]: per frame com = tr_res * [orig0, orig1, max_depth]
    (float32 * float64 list -> float64), crop of image * max_depth (float32), patch = crop /
    max_depth (float32).  Returns (patches [n, dsize, dsize] float32, Ms [n, 3, 3], coms [n, 3])."""
    fr = np.asarray(frames_norm, np.float32)
    if fr.ndim == 4:
        fr = fr[..., 0]
    tr = np.asarray(tr_res, np.float32)
    scale = np.array([orig_size[0], orig_size[1], max_depth])
    patches, Ms, coms = [], [], []
    for i in range(fr.shape[0]):
        com = tr[i] * scale
        crop, M, c, _ = md.cropArea3D(fr[i] * np.float32(max_depth), com=com, dsize=(dsize, dsize))
        patches.append(np.asarray(crop, np.float32) / np.float32(max_depth))
        Ms.append(np.asarray(M, np.float64))
        coms.append(np.asarray(c, np.float64))
    return np.stack(patches), np.stack(Ms), np.stack(coms)
