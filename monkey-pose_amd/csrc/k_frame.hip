// Frame-level kernels of the end-to-end chain frame -> CoM -> crop -> pose
// (train_cnn_networks_hgru.py:284-321 test_model, 61-74 prepare_data_test):
//
//   resize_bilinear_kernel  tf.image.resize_images(x, [128,128]) of the attention net
//                           (train_cnn_networks_hgru.py:439): TF1 BILINEAR, align_corners=False,
//                           legacy (non half-pixel) source coordinates.  Unfused float32 lerps in
//                           the TF kernel's order, so the result is bit-identical to it.
//   crop3d_kernel           cropArea3D(frame * max_depth, com = attention output * image size)
//                           / max_depth for every frame of the batch on the device -- the
//                           reference's per-image host loop (61-74) in one launch.  Geometry from
//                           crop_geom.hpp (shared with the host crop, so the integers agree).
//
// Both are HBM/latency bound byte movers: one thread per output element, coalesced along the
// innermost output axis.
#include "crop_geom.hpp"
#include "mp_kernels.hpp"

#pragma clang fp contract(off)

namespace mp {

__global__ void resize_bilinear_kernel(const float* __restrict__ x, int N, int H, int W, int C, float* out, int Ho,
                                       int Wo, float hs, float ws) {
  const size_t total = (size_t)N * Ho * Wo * C;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  size_t r = i / C;
  const int ox = (int)(r % Wo);
  r /= Wo;
  const int oy = (int)(r % Ho);
  const int n = (int)(r / Ho);
  // compute_interpolation_weights (LegacyScaler: in = out * scale)
  const float iy = (float)oy * hs, ix = (float)ox * ws;
  const float fy = floorf(iy), fx = floorf(ix);
  const int y0 = max((int)fy, 0), y1 = min((int)ceilf(iy), H - 1);
  const int x0 = max((int)fx, 0), x1 = min((int)ceilf(ix), W - 1);
  const float ly = iy - fy, lx = ix - fx;
  const float* b = x + (size_t)n * H * W * C + c;
  const float tl = b[((size_t)y0 * W + x0) * C], tr = b[((size_t)y0 * W + x1) * C];
  const float bl = b[((size_t)y1 * W + x0) * C], br = b[((size_t)y1 * W + x1) * C];
  // compute_lerp
  const float top = tl + (tr - tl) * lx;
  const float bot = bl + (br - bl) * lx;
  out[i] = top + (bot - top) * ly;
}

hipError_t launch_resize_bilinear(const float* x, int N, int H, int W, int C, float* out, int Ho, int Wo,
                                  hipStream_t st) {
  const size_t total = (size_t)N * Ho * Wo * C;
  // CalculateResizeScale(in, out, align_corners = false) = in / (float)out
  const float hs = (float)H / (float)Ho, ws = (float)W / (float)Wo;
  hipLaunchKernelGGL(resize_bilinear_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, N, H, W,
                     C, out, Ho, Wo, hs, ws);
  return hipGetLastError();
}

constexpr int CROP_PIX_PER_BLOCK = 1024;

__global__ __launch_bounds__(256) void crop3d_kernel(mp_camera cam, const float* __restrict__ frames, int H, int W,
                                                     float frame_scale, const float* __restrict__ com_norm,
                                                     double cs0, double cs1, double cs2, int dsz,
                                                     float* __restrict__ patches, double* __restrict__ Ms,
                                                     double* __restrict__ coms_out, int32_t* __restrict__ status) {
  __shared__ mpgeom::CropGeom g;
  __shared__ int st;
  const int f = blockIdx.y;
  if (threadIdx.x == 0) {
    // tr_res[im] * [image_orig_size[0], image_orig_size[1], image_max_depth] (float32 * float64)
    double com[3] = {(double)com_norm[3 * f] * cs0, (double)com_norm[3 * f + 1] * cs1,
                     (double)com_norm[3 * f + 2] * cs2};
    st = mpgeom::crop_geometry(cam, com, H, W, dsz, &g);
    if (blockIdx.x == 0) {
      status[f] = st;
      coms_out[3 * f] = com[0];
      coms_out[3 * f + 1] = com[1];
      coms_out[3 * f + 2] = com[2];
      double M[9];
      if (st == mpgeom::CROP_OK) {
        mpgeom::crop_matrix(g, M);
      } else {
        for (int k = 0; k < 9; ++k) M[k] = 0.0;
      }
      for (int k = 0; k < 9; ++k) Ms[9 * f + k] = M[k];
    }
  }
  __syncthreads();
  const float md = (float)cam.max_depth;
  const float* fr = frames + (size_t)f * H * W;
  float* dst = patches + (size_t)f * dsz * dsz;
  const int npix = dsz * dsz;
  for (int k = 0; k < CROP_PIX_PER_BLOCK / 256; ++k) {
    const int p = blockIdx.x * CROP_PIX_PER_BLOCK + k * 256 + threadIdx.x;
    if (p >= npix) break;
    float v = md;   // canvas: ones(dsize, float32) * maxDepth
    if (st == mpgeom::CROP_OK) {
      const int64_t y = p / dsz - g.offy, x = p % dsz - g.offx;
      if (y >= 0 && y < g.szh && x >= 0 && x < g.szw) {
        // getCrop value at the nearest-neighbour source pixel (padded region = 0, z threshold)
        const int64_t sy = mpgeom::nn_row(g, y) - g.pt, sx = mpgeom::nn_col(g, x) - g.pl;
        v = 0.f;
        if (sy >= 0 && sy < g.r1 - g.r0 && sx >= 0 && sx < g.c1 - g.c0) {
          const float d = fr[(g.r0 + sy) * W + (g.c0 + sx)] * frame_scale;   // image * max_depth (float32)
          // float32 frame vs float64 bounds: compared in float32 (NumPy 1.x rule, crop_geom.hpp)
          if (mpgeom::f32_lt(d, g.zstart) && d != 0.f)
            v = (float)g.zstart;
          else if (mpgeom::f32_gt(d, g.zend) && d != 0.f)
            v = 0.f;
          else
            v = d;
        }
      }
    }
    dst[p] = v / md;   // patches = crop / max_depth (train_cnn_networks_hgru.py:71)
  }
}

hipError_t launch_crop3d(const mp_camera& cam, const float* frames, int N, int H, int W, float frame_scale,
                         const float* com_norm, const double com_scale[3], int dsz, float* patches, double* Ms,
                         double* coms_out, int32_t* status, hipStream_t st) {
  const int nb = (dsz * dsz + CROP_PIX_PER_BLOCK - 1) / CROP_PIX_PER_BLOCK;
  hipLaunchKernelGGL(crop3d_kernel, dim3(nb, N), dim3(256), 0, st, cam, frames, H, W, frame_scale, com_norm,
                     com_scale[0], com_scale[1], com_scale[2], dsz, patches, Ms, coms_out, status);
  return hipGetLastError();
}

// hidden_init 'random' (hgru_module.py:879-887) drawn on the device: element i of O0 is
// f32((2u - 1) * limit), u = (splitmix64(i * golden + key) >> 11) * 2^-53 -- the counter-based
// generator of monkey-pose_amd/weights.py (uniform01 / sym_uniform), so a draw is reproducible on the
// host bit for bit.  Double arithmetic with contraction off, as numpy evaluates it.
__device__ __forceinline__ uint64_t splitmix_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void hidden_uniform_kernel(float* __restrict__ out, int64_t n, uint64_t key,
                                                             double limit) {
#pragma clang fp contract(off)
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= n) return;
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t z = splitmix_mix((uint64_t)(i0 + k) * 0x9E3779B97F4A7C15ull + key);
    const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
    v[k] = (float)((2.0 * u - 1.0) * limit);
  }
  if (i0 + 4 <= n) {
    *reinterpret_cast<float4*>(out + i0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int k = 0; i0 + k < n; ++k) out[i0 + k] = v[k];
  }
}

static uint64_t fnv1a64(const char* s) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (; *s; ++s) {
    h ^= (uint8_t)*s;
    h *= 0x100000001B3ull;
  }
  return h;
}

hipError_t launch_hidden_uniform(float* out, int64_t n, uint64_t seed, double limit, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const uint64_t key = fnv1a64("h2_init") ^ (seed * 0x2545F4914F6CDD1Dull);
  const int64_t nb = (n + 1023) / 1024;
  hipLaunchKernelGGL(hidden_uniform_kernel, dim3((unsigned)nb), dim3(256), 0, st, out, n, key, limit);
  return hipGetLastError();
}

}  // namespace mp
