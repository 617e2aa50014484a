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

#include "crop_geom.hpp"
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
  mpgeom::CropGeom g;
  const int st = mpgeom::crop_geometry(cam, com, h, w, dsz, &g);
  if (st != mpgeom::CROP_OK) fail(MP_ERR_ARG, mpgeom::crop_status_msg(st));
  auto crop_at = [&](int64_t y, int64_t x) -> float {   // padded, thresholded crop value (getCrop)
    const int64_t sy = y - g.pt, sx = x - g.pl;
    if (sy < 0 || sy >= g.r1 - g.r0 || sx < 0 || sx >= g.c1 - g.c0) return 0.f;
    const T v = dpt[(g.r0 + sy) * w + (g.c0 + sx)];
    if ((double)v < g.zstart && v != 0) return store_as(v, g.zstart);
    if ((double)v > g.zend && v != 0) return 0.f;
    return (float)v;
  };
  for (int64_t i = 0; i < dsz * dsz; ++i) out[i] = (float)cam.max_depth;
  for (int64_t y = 0; y < g.szh; ++y) {
    const int64_t sy = mpgeom::nn_row(g, y);
    for (int64_t x = 0; x < g.szw; ++x) {
      const int64_t sx = mpgeom::nn_col(g, x);
      const int64_t oy = g.offy + y, ox = g.offx + x;
      if (oy >= 0 && oy < dsz && ox >= 0 && ox < dsz) out[oy * dsz + ox] = crop_at(sy, sx);
    }
  }
  mpgeom::crop_matrix(g, M);
  std::memcpy(com_out, com, sizeof(com));
  if (info) *info = CropInfo{(int32_t)g.xstart, (int32_t)g.xend, (int32_t)g.ystart, (int32_t)g.yend,
                             (int32_t)g.szw, (int32_t)g.szh, (int32_t)g.offx, (int32_t)g.offy};
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

int mp_crop3d_dev(const mp_camera* cam, const float* frames, int64_t n, int64_t h, int64_t w, float frame_scale,
                  const float* com_norm, const double* com_scale, int64_t dsize, float* patches, double* Ms,
                  double* coms_out, int32_t* status, void* stream) {
  return guard([&] {
    check_cam(cam);
    if (!frames || !com_norm || !com_scale || !patches || !Ms || !coms_out || !status)
      fail(MP_ERR_ARG, "mp_crop3d_dev: null pointer");
    if (n <= 0 || n > 65535 || h <= 0 || w <= 0 || h * w > ((int64_t)1 << 30) || dsize <= 0 || dsize > 4096)
      fail(MP_ERR_SHAPE, "mp_crop3d_dev: bad shape");
    if (!(cam->max_depth != 0.0)) fail(MP_ERR_ARG, "camera max_depth must be non-zero");
    hip_check(launch_crop3d(*cam, frames, (int)n, (int)h, (int)w, frame_scale, com_norm, com_scale, (int)dsize,
                            patches, Ms, coms_out, status, static_cast<hipStream_t>(stream)),
              "crop3d");
  });
}

}  // extern "C"
