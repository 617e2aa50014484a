// Host-side 3D CoM crop (MonkeyDetector, /root/reference/monkeydetector.py:66-334; identical code in
// tf_monkeydetector.py:73-365), the pre-step of the pose regressors in the reference's inference
// loop (train_cnn_networks_hgru.py:61-74).  Plain C++ on the host (no GPU): the integer bounds,
// sizes, offsets and nearest-neighbour indices are computed with the reference's float64
// operation order so they are bit-exact; FP contraction is disabled in this file.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "mp_runtime.hpp"

#pragma clang fp contract(off)

namespace {

// numpy 1.x float32 pairwise summation (numpy/core/src/umath/loops_utils.h.src), used by
// calculateCoM's dc.sum() on a float32 frame (monkeydetector.py:78)
float pairwise_sum_f32(const float* a, int64_t n) {
  if (n < 8) {
    float r = 0.f;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    float r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum_f32(a, n2) + pairwise_sum_f32(a + n2, n - n2);
}

// numpy sum of the thresholded frame: float32 pairwise for a float32 frame, exact for uint16
double frame_sum(const std::vector<float>& dc) { return (double)pairwise_sum_f32(dc.data(), (int64_t)dc.size()); }
double frame_sum(const std::vector<uint16_t>& dc) {
  uint64_t s = 0;
  for (uint16_t v : dc) s += v;
  return (double)s;
}

template <typename T>
void center_of_mass(const mp_camera& cam, const T* dpt, int64_t h, int64_t w, double com[3]) {
  std::vector<T> dc(dpt, dpt + h * w);
  double sr = 0, sc = 0;   // integer sums, exact in double (center_of_mass of the mask)
  int64_t num = 0, npos = 0;
  for (int64_t y = 0; y < h; ++y)
    for (int64_t x = 0; x < w; ++x) {
      T& v = dc[y * w + x];
      if ((double)v < cam.min_depth) v = 0;
      if ((double)v > cam.max_depth) v = 0;
      if (v > 0) {
        sr += (double)y;
        sc += (double)x;
        ++npos;
      }
      if (v != 0) ++num;
    }
  if (num == 0) {
    com[0] = com[1] = com[2] = 0.0;
    return;
  }
  const double cc0 = sr / (double)npos, cc1 = sc / (double)npos;   // ndimage.center_of_mass(dc > 0)
  const double s = frame_sum(dc);
  com[0] = (cc1 * (double)num) / (double)num;                       // numpy.array(...) / num
  com[1] = (cc0 * (double)num) / (double)num;
  com[2] = s / (double)num;
}

// Python slice a[s:e] on a length-n axis with s >= 0: [lo, hi)
void py_slice(int64_t s, int64_t e, int64_t n, int64_t* lo, int64_t* hi) {
  if (e < 0) e += n;
  if (e < 0) e = 0;
  if (e > n) e = n;
  if (s > n) s = n;
  *lo = s;
  *hi = std::max(s, e);
}

struct CropInfo {
  int32_t xstart, xend, ystart, yend, szw, szh, offx, offy;
};

// getCrop's "cropped[msk1] = zstart" stores zstart in the frame's dtype (float32 rounds, uint16
// truncates); the crop itself is float32 (ret = ones(dsize, float32) * maxDepth; ret[...] = rz)
inline float store_as(float, double z) { return (float)z; }
inline float store_as(uint16_t, double z) { return (float)(uint16_t)(int64_t)z; }

template <typename T>
void crop_one(const mp_camera& cam, const T* dpt, int64_t h, int64_t w, const double* com_in,
              int64_t dsz, float* out, double M[9], double com_out[3], CropInfo* info) {
  double com[3];
  if (com_in)
    std::memcpy(com, com_in, sizeof(com));
  else
    center_of_mass(cam, dpt, h, w, com);
  if (!(com[2] != 0.0) || !std::isfinite(com[0]) || !std::isfinite(com[1]) || !std::isfinite(com[2]))
    fail(MP_ERR_ARG, "cropArea3D: CoM depth is zero or not finite (no valid pixel in range?)");
  // comToBounds (monkeydetector.py:162-175)
  const double zstart = com[2] - cam.cube[2] / 2.;
  const double zend = com[2] + cam.cube[2] / 2.;
  const int64_t xstart = (int64_t)std::floor((com[0] * com[2] / cam.fx - cam.cube[0] / 2.) / com[2] * cam.fx);
  const int64_t xend = (int64_t)std::floor((com[0] * com[2] / cam.fx + cam.cube[0] / 2.) / com[2] * cam.fx);
  const int64_t ystart = (int64_t)std::floor((com[1] * com[2] / cam.fy - cam.cube[1] / 2.) / com[2] * cam.fy);
  const int64_t yend = (int64_t)std::floor((com[1] * com[2] / cam.fy + cam.cube[1] / 2.) / com[2] * cam.fy);
  // getCrop (177-213): slice, zero pad to keep the aspect ratio, z threshold
  int64_t r0, r1, c0, c1;
  py_slice(std::max<int64_t>(ystart, 0), std::min<int64_t>(yend, h), h, &r0, &r1);
  py_slice(std::max<int64_t>(xstart, 0), std::min<int64_t>(xend, w), w, &c0, &c1);
  const int64_t pt = std::llabs(ystart) - std::max<int64_t>(ystart, 0);
  const int64_t pb = std::llabs(yend) - std::min<int64_t>(yend, h);
  const int64_t pl = std::llabs(xstart) - std::max<int64_t>(xstart, 0);
  const int64_t pr = std::llabs(xend) - std::min<int64_t>(xend, w);
  const int64_t rows = (r1 - r0) + pt + pb, cols = (c1 - c0) + pl + pr;
  if (rows <= 0 || cols <= 0) fail(MP_ERR_ARG, "cropArea3D: empty crop");
  auto crop_at = [&](int64_t y, int64_t x) -> float {   // padded, thresholded crop value
    const int64_t sy = y - pt, sx = x - pl;
    if (sy < 0 || sy >= r1 - r0 || sx < 0 || sx >= c1 - c0) return 0.f;
    const T v = dpt[(r0 + sy) * w + (c0 + sx)];
    if ((double)v < zstart && v != 0) return store_as(v, zstart);
    if ((double)v > zend && v != 0) return 0.f;
    return (float)v;
  };
  // cropArea3D (282-334)
  const int64_t wb = xend - xstart, hb = yend - ystart;
  if (wb <= 0 || hb <= 0) fail(MP_ERR_ARG, "cropArea3D: degenerate bounds");
  int64_t szw, szh;
  if (wb > hb) {
    szw = dsz;
    szh = hb * dsz / wb;   // Python 2 integer '/'
  } else {
    szw = wb * dsz / hb;
    szh = dsz;
  }
  if (szw <= 0 || szh <= 0) fail(MP_ERR_ARG, "cropArea3D: resize target is empty");
  const double s = rows > cols ? (double)szh / (double)rows : (double)szw / (double)cols;
  // cv2.resize(INTER_NEAREST): inv = dst/src, ifx = 1/inv, sx = min(floor(x*ifx), src-1)
  const double ifx = 1. / ((double)szw / (double)cols), ify = 1. / ((double)szh / (double)rows);
  const int64_t offx = (int64_t)std::floor(dsz / 2. - szw / 2.);
  const int64_t offy = (int64_t)std::floor(dsz / 2. - szh / 2.);
  for (int64_t i = 0; i < dsz * dsz; ++i) out[i] = (float)cam.max_depth;
  for (int64_t y = 0; y < szh; ++y) {
    const int64_t sy = std::min<int64_t>((int64_t)std::floor((double)y * ify), rows - 1);
    for (int64_t x = 0; x < szw; ++x) {
      const int64_t sx = std::min<int64_t>((int64_t)std::floor((double)x * ifx), cols - 1);
      const int64_t oy = offy + y, ox = offx + x;
      if (oy >= 0 && oy < dsz && ox >= 0 && ox < dsz) out[oy * dsz + ox] = crop_at(sy, sx);
    }
  }
  // M = off * scale * trans, evaluated as numpy does: (off @ scale) @ trans
  M[0] = s;   M[1] = 0.0; M[2] = s * (double)(-xstart) + (double)offx;
  M[3] = 0.0; M[4] = s;   M[5] = s * (double)(-ystart) + (double)offy;
  M[6] = 0.0; M[7] = 0.0; M[8] = 1.0;
  std::memcpy(com_out, com, sizeof(com));
  if (info) *info = CropInfo{(int32_t)xstart, (int32_t)xend, (int32_t)ystart, (int32_t)yend,
                             (int32_t)szw, (int32_t)szh, (int32_t)offx, (int32_t)offy};
}

void check_cam(const mp_camera* cam) {
  if (!cam) fail(MP_ERR_ARG, "camera is NULL");
  if (!(cam->fx > 0) || !(cam->fy > 0) || !(cam->cube[0] > 0) || !(cam->cube[1] > 0) || !(cam->cube[2] > 0))
    fail(MP_ERR_ARG, "camera focal lengths and cube must be positive");
}

}  // namespace

extern "C" {

int mp_center_of_mass(const mp_camera* cam, const void* depth, int depth_dtype, int64_t h, int64_t w,
                      double com[3]) {
  return guard([&] {
    check_cam(cam);
    if (!depth || !com || h <= 0 || w <= 0) fail(MP_ERR_ARG, "mp_center_of_mass: bad argument");
    if (depth_dtype == MP_DEPTH_F32)
      center_of_mass(*cam, static_cast<const float*>(depth), h, w, com);
    else if (depth_dtype == MP_DEPTH_U16)
      center_of_mass(*cam, static_cast<const uint16_t*>(depth), h, w, com);
    else
      fail(MP_ERR_ARG, "unknown depth dtype");
  });
}

int mp_crop3d(const mp_camera* cam, const void* depth, int depth_dtype, int64_t h, int64_t w, const double* com,
              int64_t dsize, float* out, double M[9], double com_out[3], int32_t info[8]) {
  return guard([&] {
    check_cam(cam);
    if (!depth || !out || !M || !com_out || h <= 0 || w <= 0 || dsize <= 0)
      fail(MP_ERR_ARG, "mp_crop3d: bad argument");
    CropInfo ci;
    if (depth_dtype == MP_DEPTH_F32)
      crop_one(*cam, static_cast<const float*>(depth), h, w, com, dsize, out, M, com_out, &ci);
    else if (depth_dtype == MP_DEPTH_U16)
      crop_one(*cam, static_cast<const uint16_t*>(depth), h, w, com, dsize, out, M, com_out, &ci);
    else
      fail(MP_ERR_ARG, "unknown depth dtype");
    if (info) std::memcpy(info, &ci, sizeof(ci));
  });
}

int mp_crop3d_batch(const mp_camera* cam, const void* frames, int depth_dtype, int64_t n, int64_t h, int64_t w,
                    const double* coms, int64_t dsize, float* patches, double* Ms, double* coms_out, int nthreads) {
  return guard([&] {
    check_cam(cam);
    if (!frames || !patches || !Ms || !coms_out || n <= 0 || h <= 0 || w <= 0 || dsize <= 0)
      fail(MP_ERR_ARG, "mp_crop3d_batch: bad argument");
    if (depth_dtype != MP_DEPTH_F32 && depth_dtype != MP_DEPTH_U16) fail(MP_ERR_ARG, "unknown depth dtype");
    const int nt = std::max(1, std::min<int>(nthreads, (int)n));
    std::vector<std::string> errs(nt);
    std::vector<int> codes(nt, MP_OK);
    auto work = [&](int t) {
      for (int64_t i = t; i < n; i += nt) {
        float* dst = patches + i * dsize * dsize;
        codes[t] = guard([&] {
          const double* ci = coms ? coms + 3 * i : nullptr;
          if (depth_dtype == MP_DEPTH_F32)
            crop_one(*cam, static_cast<const float*>(frames) + i * h * w, h, w, ci, dsize, dst, Ms + 9 * i,
                     coms_out + 3 * i, nullptr);
          else
            crop_one(*cam, static_cast<const uint16_t*>(frames) + i * h * w, h, w, ci, dsize, dst, Ms + 9 * i,
                     coms_out + 3 * i, nullptr);
        });
        if (codes[t] != MP_OK) {
          errs[t] = "frame " + std::to_string(i) + ": " + g_err;
          return;
        }
        // normalisation of the model input: patch / maxDepth (train_cnn_networks_hgru.py:71)
        const float md = (float)cam->max_depth;
        for (int64_t k = 0; k < dsize * dsize; ++k) dst[k] = dst[k] / md;
      }
    };
    if (nt == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
      for (auto& x : th) x.join();
    }
    for (int t = 0; t < nt; ++t)
      if (codes[t] != MP_OK) fail(codes[t], errs[t]);
  });
}

}  // extern "C"
