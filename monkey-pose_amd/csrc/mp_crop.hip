// Host-side 3D CoM crop (MonkeyDetector, /root/reference/monkeydetector.py:66-334; identical code in
// tf_monkeydetector.py:73-365), the pre-step of the pose regressors in the reference's inference
// loop (train_cnn_networks_hgru.py:61-74).  Plain C++ on the host (no GPU): the integer bounds,
// sizes, offsets and nearest-neighbour indices are computed with the reference's float64
// operation order so they are bit-exact; FP contraction is disabled in this file.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "crop_geom.hpp"
#include "mp_runtime.hpp"

#pragma clang fp contract(off)

namespace {

// numpy 1.x float32 pairwise summation (numpy/core/src/umath/loops_utils.h.src), used by
// calculateCoM's dc.sum() on a float32 frame (monkeydetector.py:78)
// The leaf (8 <= n <= 128) keeps numpy's 8 accumulators in one 8-lane vector: r[j] += a[i + j] lane
// by lane, then ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) -- the same additions in the same
// order, without the scalar array the compiler did not vectorise.
typedef float f32v8 __attribute__((ext_vector_type(8)));
inline f32v8 load_v8(const float* p) {
  f32v8 v;
  std::memcpy(&v, p, sizeof(v));
  return v;
}
float pairwise_sum_f32(const float* a, int64_t n) {
  if (n < 8) {
    float r = 0.f;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    f32v8 r = load_v8(a);
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8) r += load_v8(a + i);
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum_f32(a, n2) + pairwise_sum_f32(a + n2, n - n2);
}

// numpy sum of the thresholded frame: float32 pairwise for a float32 frame, exact for uint16
double frame_sum(const float* dc, int64_t n) { return (double)pairwise_sum_f32(dc, n); }
double frame_sum(const uint16_t* dc, int64_t n) {
  uint64_t s = 0;
  for (int64_t i = 0; i < n; ++i) s += dc[i];
  return (double)s;
}

// calculateCoM's `dc[dc < self.minDepth] = 0; dc[dc > self.maxDepth] = 0` (74-75).  A uint16 frame
// compares in double (NumPy 1.x promotes it with the float scalar to float64); a float32 frame
// compares in float32 against f32(threshold) (NumPy 1.x value-based casting, crop_geom.hpp), or,
// for a threshold beyond min_scalar_type's float32 range, in double -- expressed as the float
// bound equivalent to the double comparison (v < lo <=> v < the smallest float >= lo), so the
// row loop runs in float SIMD lanes either way.
inline float float_at_least(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, INFINITY);
  return f;
}
inline float float_at_most(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -INFINITY);
  return f;
}
template <typename T>
struct Thresh {
  double lo, hi;
  explicit Thresh(const mp_camera& c) : lo(c.min_depth), hi(c.max_depth) {}
  bool out(T v) const { return (double)v < lo || (double)v > hi; }
};
template <>
struct Thresh<float> {
  float lo, hi;
  explicit Thresh(const mp_camera& c)
      : lo(mpgeom::legacy_in_f32(c.min_depth) ? (float)c.min_depth : float_at_least(c.min_depth)),
        hi(mpgeom::legacy_in_f32(c.max_depth) ? (float)c.max_depth : float_at_most(c.max_depth)) {}
  bool out(float v) const { return v < lo || v > hi; }
};

// The float32 frame's threshold / mask-sum pass of center_of_mass below (w < 46000), as a plain
// function so the host build carries AVX-512 / AVX2 clones of it beside the baseline x86-64 one,
// picked at load time by the CPU (the device pass of hipcc does not take the attribute).
#ifdef __HIP_DEVICE_COMPILE__
#define MP_HOST_CLONES
#else
#define MP_HOST_CLONES __attribute__((target_clones("arch=x86-64-v4", "arch=x86-64-v3", "default")))
#endif
MP_HOST_CLONES void thresh_rows_f32(const float* dpt, float* dc, int64_t h, int64_t w, float lo, float hi,
                                    int64_t acc[4]) {
  int64_t sr = 0, sc = 0, npos = 0, num = 0;
  for (int64_t y = 0; y < h; ++y) {
    const float* src = dpt + y * w;
    float* d = dc + y * w;
    int32_t p32 = 0, x32 = 0, n32 = 0;
    for (int32_t x = 0; x < (int32_t)w; ++x) {
      const float v = (src[x] < lo || src[x] > hi) ? 0.f : src[x];
      d[x] = v;
      const int32_t pos = v > 0.f;
      p32 += pos;
      x32 += pos ? x : 0;
      n32 += v != 0.f;
    }
    sr += y * p32;
    sc += x32;
    npos += p32;
    num += n32;
  }
  acc[0] = sr;
  acc[1] = sc;
  acc[2] = npos;
  acc[3] = num;
}

// numpy's calculateCoM (monkeydetector.py:66-84) in one pass: the thresholded frame dc goes to a
// per-thread buffer reused across calls (no 0.9 MB allocation and page faults per frame), and the
// mask sums are integer per row (the original's double sums of integers are exact, so this is
// bit-identical), a branch-free loop the compiler vectorises.  frame_sum keeps numpy's pairwise
// float32 order.
template <typename T>
void center_of_mass(const mp_camera& cam, const T* dpt, int64_t h, int64_t w, double com[3]) {
  thread_local std::vector<T> buf;
  buf.resize((size_t)(h * w));
  T* dc = buf.data();
  const Thresh<T> th(cam);
  const bool narrow = w < 46000;   // a row's sum of x fits int32
  int64_t sr = 0, sc = 0, num = 0, npos = 0;
  int64_t rows = h;
  if constexpr (std::is_same<T, float>::value) {
    if (narrow) {
      int64_t acc[4];
      thresh_rows_f32(dpt, dc, h, w, th.lo, th.hi, acc);
      sr = acc[0];
      sc = acc[1];
      npos = acc[2];
      num = acc[3];
      rows = 0;   // the row loop below has nothing left to do
    }
  }
  for (int64_t y = 0; y < rows; ++y) {
    const T* src = dpt + y * w;
    T* d = dc + y * w;
    int64_t rpos = 0, rx = 0, rnum = 0;
    if (narrow) {
      int32_t p32 = 0, x32 = 0, n32 = 0;
      for (int32_t x = 0; x < (int32_t)w; ++x) {
        const T v = th.out(src[x]) ? T(0) : src[x];   // dc[dc < min] = 0; dc[dc > max] = 0
        d[x] = v;
        const int32_t pos = v > T(0);
        p32 += pos;
        x32 += pos ? x : 0;
        n32 += v != T(0);
      }
      rpos = p32;
      rx = x32;
      rnum = n32;
    } else {
      for (int64_t x = 0; x < w; ++x) {
        const T v = th.out(src[x]) ? T(0) : src[x];
        d[x] = v;
        const int64_t pos = v > T(0);
        rpos += pos;
        rx += pos ? x : 0;
        rnum += v != T(0);
      }
    }
    sr += y * rpos;
    sc += rx;
    npos += rpos;
    num += rnum;
  }
  if (num == 0) {
    com[0] = com[1] = com[2] = 0.0;
    return;
  }
  const double cc0 = (double)sr / (double)npos, cc1 = (double)sc / (double)npos;   // ndimage.center_of_mass(dc > 0)
  const double s = frame_sum(dc, h * w);
  com[0] = (cc1 * (double)num) / (double)num;                                       // numpy.array(...) / num
  com[1] = (cc0 * (double)num) / (double)num;
  com[2] = s / (double)num;
}

struct CropInfo {
  int32_t xstart, xend, ystart, yend, szw, szh, offx, offy;
};

// getCrop's thresholding (monkeydetector.py:208-212) of one frame pixel, in the frame's dtype:
// "cropped[msk1] = zstart" stores zstart as float32 (rounded) or uint16 (truncated); the
// comparisons run in float32 for a float32 frame (NumPy 1.x value-based casting, crop_geom.hpp)
// and in float64 for a uint16 frame
inline float crop_px(float v, const mpgeom::CropGeom& g) {
  if (mpgeom::f32_lt(v, g.zstart) && v != 0.f) return (float)g.zstart;
  if (mpgeom::f32_gt(v, g.zend) && v != 0.f) return 0.f;
  return v;
}
inline uint16_t crop_px(uint16_t v, const mpgeom::CropGeom& g) {
  if ((double)v < g.zstart && v != 0) return (uint16_t)(int64_t)g.zstart;
  if ((double)v > g.zend && v != 0) return 0;
  return v;
}

// the padded, thresholded crop (getCrop's return value) at crop row y, column x
template <typename T>
inline T crop_at(const mpgeom::CropGeom& g, const T* dpt, int64_t w, int64_t y, int64_t x) {
  const int64_t sy = y - g.pt, sx = x - g.pl;
  if (sy < 0 || sy >= g.r1 - g.r0 || sx < 0 || sx >= g.c1 - g.c0) return T(0);
  return crop_px(dpt[(g.r0 + sy) * w + (g.c0 + sx)], g);
}

// cropArea3D's docom refinement (monkeydetector.py:287-300): the CoM of the first crop, shifted back
// to frame coordinates; numpy.allclose(com, 0.) (|c| <= 1e-8 each) falls back to the crop's centre
// pixel as the depth and then to 300 mm (numpy.isclose(com[2], 0))
template <typename T>
void refine_com(const mp_camera& cam, const mpgeom::CropGeom& g, const T* dpt, int64_t w, double com[3]) {
  thread_local std::vector<T> cb;
  cb.resize((size_t)(g.rows * g.cols));
  for (int64_t y = 0; y < g.rows; ++y)
    for (int64_t x = 0; x < g.cols; ++x) cb[(size_t)(y * g.cols + x)] = crop_at(g, dpt, w, y, x);
  center_of_mass(cam, cb.data(), g.rows, g.cols, com);
  if (std::fabs(com[0]) <= 1e-8 && std::fabs(com[1]) <= 1e-8 && std::fabs(com[2]) <= 1e-8) {
    com[2] = (double)cb[(size_t)((g.rows / 2) * g.cols + g.cols / 2)];
    if (std::fabs(com[2]) <= 1e-8) com[2] = 300.;
  }
  com[0] += (double)g.xstart;
  com[1] += (double)g.ystart;
}

template <typename T>
void crop_one(const mp_camera& cam, const T* dpt, int64_t h, int64_t w, const double* com_in, bool docom,
              int64_t dsz, float* out, double M[9], double com_out[3], CropInfo* info) {
  double com[3];
  if (com_in)
    std::memcpy(com, com_in, sizeof(com));
  else
    center_of_mass(cam, dpt, h, w, com);
  mpgeom::CropGeom g;
  int st = mpgeom::crop_geometry(cam, com, h, w, dsz, &g);
  if (st != mpgeom::CROP_OK) fail(MP_ERR_ARG, mpgeom::crop_status_msg(st));
  if (docom) {
    refine_com(cam, g, dpt, w, com);
    st = mpgeom::crop_geometry(cam, com, h, w, dsz, &g);
    if (st != mpgeom::CROP_OK) fail(MP_ERR_ARG, mpgeom::crop_status_msg(st));
  }
  for (int64_t i = 0; i < dsz * dsz; ++i) out[i] = (float)cam.max_depth;
  // the output columns inside the patch and their nearest-neighbour source columns, once per crop
  const int64_t x0 = std::max<int64_t>(0, -g.offx), x1 = std::min<int64_t>(g.szw, dsz - g.offx);
  // per output column, the frame column its nearest-neighbour source pixel reads, or -1 where that
  // pixel is the crop's zero padding; then per output row one frame row (or none) -- the per-pixel
  // work is one gather and getCrop's two thresholds (crop_px, unchanged)
  // float32 frames with both getCrop bounds in float32 range (always, for finite depths) compare
  // against f32(zstart) / f32(zend) exactly as crop_px does
  const bool fast = std::is_same<T, float>::value && mpgeom::legacy_in_f32(g.zstart) && mpgeom::legacy_in_f32(g.zend);
  const float zs = (float)g.zstart, ze = (float)g.zend;
  thread_local std::vector<int64_t> srccol;
  srccol.resize((size_t)std::max<int64_t>(0, x1 - x0));
  for (int64_t x = x0; x < x1; ++x) {
    const int64_t sx = mpgeom::nn_col(g, x) - g.pl;
    srccol[x - x0] = (sx >= 0 && sx < g.c1 - g.c0) ? g.c0 + sx : -1;
  }
  for (int64_t y = 0; y < g.szh; ++y) {
    const int64_t oy = g.offy + y;
    if (oy < 0 || oy >= dsz) continue;
    const int64_t sy = mpgeom::nn_row(g, y) - g.pt;
    float* orow = out + oy * dsz + (g.offx + x0);   // in-range base: output column offx + x0 >= 0
    if (sy < 0 || sy >= g.r1 - g.r0) {
      for (int64_t x = x0; x < x1; ++x) orow[x - x0] = 0.f;
      continue;
    }
    const T* src = dpt + (g.r0 + sy) * w;
    if (fast) {   // crop_px with its float32 bounds hoisted
      for (int64_t x = x0; x < x1; ++x) {
        const int64_t c = srccol[x - x0];
        const float v = c >= 0 ? (float)src[c] : 0.f;
        orow[x - x0] = (v != 0.f && v < zs) ? zs : ((v != 0.f && v > ze) ? 0.f : v);
      }
    } else {
      for (int64_t x = x0; x < x1; ++x) {
        const int64_t c = srccol[x - x0];
        orow[x - x0] = c >= 0 ? (float)crop_px(src[c], g) : 0.f;
      }
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
  return mp_crop3d_ex(cam, depth, depth_dtype, h, w, com, 0, dsize, out, M, com_out, info);
}

int mp_crop3d_ex(const mp_camera* cam, const void* depth, int depth_dtype, int64_t h, int64_t w, const double* com,
                 int flags, int64_t dsize, float* out, double M[9], double com_out[3], int32_t info[8]) {
  return guard([&] {
    if (flags & ~MP_CROP_DOCOM) fail(MP_ERR_ARG, "mp_crop3d_ex: unknown flags");
    const bool docom = (flags & MP_CROP_DOCOM) != 0;
    check_cam(cam);
    if (!depth || !out || !M || !com_out || h <= 0 || w <= 0 || dsize <= 0)
      fail(MP_ERR_ARG, "mp_crop3d: bad argument");
    CropInfo ci;
    if (depth_dtype == MP_DEPTH_F32)
      crop_one(*cam, static_cast<const float*>(depth), h, w, com, docom, dsize, out, M, com_out, &ci);
    else if (depth_dtype == MP_DEPTH_U16)
      crop_one(*cam, static_cast<const uint16_t*>(depth), h, w, com, docom, dsize, out, M, com_out, &ci);
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
            crop_one(*cam, static_cast<const float*>(frames) + i * h * w, h, w, ci, false, dsize, dst,
                     Ms + 9 * i, coms_out + 3 * i, nullptr);
          else
            crop_one(*cam, static_cast<const uint16_t*>(frames) + i * h * w, h, w, ci, false, dsize, dst,
                     Ms + 9 * i, coms_out + 3 * i, nullptr);
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
  return mp_crop3d_dev_ex(cam, frames, n, h, w, frame_scale, com_norm, com_scale, 0, dsize, patches, Ms, coms_out,
                          status, stream);
}

int mp_crop3d_dev_ex(const mp_camera* cam, const float* frames, int64_t n, int64_t h, int64_t w, float frame_scale,
                     const float* com_norm, const double* com_scale, int flags, int64_t dsize, float* patches,
                     double* Ms, double* coms_out, int32_t* status, void* stream) {
  return guard([&] {
    check_cam(cam);
    if (flags & ~MP_CROP_DOCOM) fail(MP_ERR_ARG, "mp_crop3d_dev_ex: unknown flags");
    if (!frames || !com_norm || !com_scale || !patches || !Ms || !coms_out || !status)
      fail(MP_ERR_ARG, "mp_crop3d_dev: null pointer");
    if (n <= 0 || n > 65535 || h <= 0 || w <= 0 || h * w > ((int64_t)1 << 30) || dsize <= 0 || dsize > 4096)
      fail(MP_ERR_SHAPE, "mp_crop3d_dev: bad shape");
    if (!(cam->max_depth != 0.0)) fail(MP_ERR_ARG, "camera max_depth must be non-zero");
    hip_check(launch_crop3d(*cam, frames, (int)n, (int)h, (int)w, frame_scale, com_norm, com_scale, (int)dsize,
                            patches, Ms, coms_out, status, static_cast<hipStream_t>(stream),
                            (flags & MP_CROP_DOCOM) != 0),
              "crop3d");
  });
}

}  // extern "C"
