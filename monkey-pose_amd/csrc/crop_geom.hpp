// Geometry of MonkeyDetector.cropArea3D (monkeydetector.py:162-334; identical code in
// tf_monkeydetector.py:173-365), shared by the host crop (mp_crop.hip) and the device crop
// (k_frame.hip) so both produce the same integers: bounds, slice, padding, resize target size,
// canvas offset and nearest-neighbour indices, all in float64 with the reference's operation
// order and no FP contraction.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/monkeypose.h"

namespace mpgeom {

enum CropStatus : int32_t {
  CROP_OK = 0,
  CROP_BAD_COM = 1,      // CoM depth zero or a coordinate not finite
  CROP_EMPTY = 2,        // sliced + padded crop has no rows or columns
  CROP_DEGENERATE = 3,   // xend <= xstart or yend <= ystart
  CROP_EMPTY_RESIZE = 4  // resize target rounds to zero pixels
};

struct CropGeom {
  int64_t xstart, xend, ystart, yend;   // comToBounds (monkeydetector.py:162-175)
  double zstart, zend;
  int64_t r0, r1, c0, c1;               // numpy slice of the frame (getCrop 177-213)
  int64_t pt, pl;                       // zero padding before the slice (top, left)
  int64_t rows, cols;                   // padded crop size
  int64_t szw, szh;                     // cv2.resize target (cropArea3D 314-320)
  int64_t offx, offy;                   // canvas offset (resizeCrop / padding, 268-279)
  double s, ifx, ify;                   // scale of M; cv2 INTER_NEAREST inverse scales
};

__host__ __device__ inline int64_t gmin(int64_t a, int64_t b) { return a < b ? a : b; }
__host__ __device__ inline int64_t gmax(int64_t a, int64_t b) { return a > b ? a : b; }
__host__ __device__ inline bool gfinite(double v) { return v - v == 0.0; }   // false for inf / nan
__host__ __device__ inline int64_t gabs(int64_t a) { return a < 0 ? -a : a; }

// Python slice a[s:e] on a length-n axis with s >= 0: [lo, hi)
__host__ __device__ inline void py_slice(int64_t s, int64_t e, int64_t n, int64_t* lo, int64_t* hi) {
  if (e < 0) e += n;
  if (e < 0) e = 0;
  if (e > n) e = n;
  if (s > n) s = n;
  *lo = s;
  *hi = gmax(s, e);
}

// all integer / float64 quantities of one crop; returns a CropStatus
__host__ __device__ inline int crop_geometry(const mp_camera& cam, const double com[3], int64_t h, int64_t w,
                                             int64_t dsz, CropGeom* g) {
#pragma clang fp contract(off)
  if (!(com[2] != 0.0) || !gfinite(com[0]) || !gfinite(com[1]) || !gfinite(com[2])) return CROP_BAD_COM;
  // comToBounds (monkeydetector.py:162-175)
  g->zstart = com[2] - cam.cube[2] / 2.;
  g->zend = com[2] + cam.cube[2] / 2.;
  g->xstart = (int64_t)floor((com[0] * com[2] / cam.fx - cam.cube[0] / 2.) / com[2] * cam.fx);
  g->xend = (int64_t)floor((com[0] * com[2] / cam.fx + cam.cube[0] / 2.) / com[2] * cam.fx);
  g->ystart = (int64_t)floor((com[1] * com[2] / cam.fy - cam.cube[1] / 2.) / com[2] * cam.fy);
  g->yend = (int64_t)floor((com[1] * com[2] / cam.fy + cam.cube[1] / 2.) / com[2] * cam.fy);
  // getCrop (177-213): slice, zero pad to keep the aspect ratio
  py_slice(gmax(g->ystart, 0), gmin(g->yend, h), h, &g->r0, &g->r1);
  py_slice(gmax(g->xstart, 0), gmin(g->xend, w), w, &g->c0, &g->c1);
  g->pt = gabs(g->ystart) - gmax(g->ystart, 0);
  const int64_t pb = gabs(g->yend) - gmin(g->yend, h);
  g->pl = gabs(g->xstart) - gmax(g->xstart, 0);
  const int64_t pr = gabs(g->xend) - gmin(g->xend, w);
  g->rows = (g->r1 - g->r0) + g->pt + pb;
  g->cols = (g->c1 - g->c0) + g->pl + pr;
  if (g->rows <= 0 || g->cols <= 0) return CROP_EMPTY;
  // cropArea3D (282-334)
  const int64_t wb = g->xend - g->xstart, hb = g->yend - g->ystart;
  if (wb <= 0 || hb <= 0) return CROP_DEGENERATE;
  if (wb > hb) {
    g->szw = dsz;
    g->szh = hb * dsz / wb;   // Python 2 integer '/'
  } else {
    g->szw = wb * dsz / hb;
    g->szh = dsz;
  }
  if (g->szw <= 0 || g->szh <= 0) return CROP_EMPTY_RESIZE;
  g->s = g->rows > g->cols ? (double)g->szh / (double)g->rows : (double)g->szw / (double)g->cols;
  // cv2.resize(INTER_NEAREST): inv = dst/src, ifx = 1/inv, sx = min(floor(x*ifx), src-1)
  g->ifx = 1. / ((double)g->szw / (double)g->cols);
  g->ify = 1. / ((double)g->szh / (double)g->rows);
  g->offx = (int64_t)floor(dsz / 2. - g->szw / 2.);
  g->offy = (int64_t)floor(dsz / 2. - g->szh / 2.);
  return CROP_OK;
}

// The reference ran on Python 2.7, i.e. NumPy <= 1.16, whose value-based casting compares a float32
// array with a float64 scalar (getCrop's `cropped < zstart` / `cropped > zend`,
// monkeydetector.py:209-210; calculateCoM's `dc < self.minDepth` / `dc > self.maxDepth`, 74-75)
// IN FLOAT32, against f32(scalar), whenever min_scalar_type(scalar) is at most float32, i.e.
// -3.4e38 < scalar < 3.4e38 (numpy/core/src/multiarray/convert_datatype.c, min_scalar_type_num);
// otherwise (NaN, inf, beyond that range) in float64.  A uint16 frame against a float scalar
// promotes to float64 (the scalar's kind is higher), so those comparisons stay in double.
// (NumPy 2's NEP 50 would compare in float64: a pixel equal to f32(zend) with zend < f32(zend) is
// kept by the reference and would be zeroed.)
// The bound is NumPy 1.x's literal 3.4e38 (min_scalar_type_num: `value > -3.4e38 && value < 3.4e38`
// -> NPY_FLOAT), not FLT_MAX = 3.4028235e38: a scalar in [3.4e38, FLT_MAX] maps to NPY_DOUBLE there,
// so the compare is in double, as here.  Non-finite scalars map to NPY_HALF (float32 compare); the
// double compare below gives the same answer for +-inf and NaN.
__host__ __device__ inline bool legacy_in_f32(double s) { return s > -3.4e38 && s < 3.4e38; }
__host__ __device__ inline bool f32_lt(float v, double s) {
  return legacy_in_f32(s) ? v < (float)s : (double)v < s;
}
__host__ __device__ inline bool f32_gt(float v, double s) {
  return legacy_in_f32(s) ? v > (float)s : (double)v > s;
}

// nearest-neighbour source row / column of resized pixel y / x
__host__ __device__ inline int64_t nn_row(const CropGeom& g, int64_t y) {
  return gmin((int64_t)floor((double)y * g.ify), g.rows - 1);
}
__host__ __device__ inline int64_t nn_col(const CropGeom& g, int64_t x) {
  return gmin((int64_t)floor((double)x * g.ifx), g.cols - 1);
}

// M = off * scale * trans, evaluated as numpy does: (off @ scale) @ trans
__host__ __device__ inline void crop_matrix(const CropGeom& g, double M[9]) {
#pragma clang fp contract(off)
  M[0] = g.s;
  M[1] = 0.0;
  M[2] = g.s * (double)(-g.xstart) + (double)g.offx;
  M[3] = 0.0;
  M[4] = g.s;
  M[5] = g.s * (double)(-g.ystart) + (double)g.offy;
  M[6] = 0.0;
  M[7] = 0.0;
  M[8] = 1.0;
}

inline const char* crop_status_msg(int st) {
  switch (st) {
    case CROP_BAD_COM: return "cropArea3D: CoM depth is zero or not finite (no valid pixel in range?)";
    case CROP_EMPTY: return "cropArea3D: empty crop";
    case CROP_DEGENERATE: return "cropArea3D: degenerate bounds";
    case CROP_EMPTY_RESIZE: return "cropArea3D: resize target is empty";
    default: return "cropArea3D: ok";
  }
}

}  // namespace mpgeom
