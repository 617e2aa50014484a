// HBM streaming ceilings of the box (mp_hbm_probe): the practical roof the FFT-path kernels are
// read against, next to the 8 TB/s spec figure (MI355X_MICROARCH.md: ~6.3 TB/s achievable).
//
// Three access forms, each swept over grids, loads / stores per thread in flight and cache policy,
// best of each reported: read-only (a reduction that keeps every load live), write-only, and copy
// (half reads, half writes -- the mix of every FFT-path kernel, 40-60 % of whose bytes are writes).
// 16 bytes per lane, U independent accesses per lane per loop trip, grid-stride over the buffer.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mp_runtime.hpp"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void probe_read(const f4* __restrict__ a, size_t n, float* out) {
  f4 s = {0.f, 0.f, 0.f, 0.f};
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += stride * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t j = min(i + u * stride, n - 1);
      v[u] = NT ? __builtin_nontemporal_load(a + j) : a[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  if (s.x + s.y + s.z + s.w == 1.2345e-30f) out[threadIdx.x] = s.x;   // keeps the loads live
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void probe_write(f4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256;
  const f4 v = {1.f, 2.f, 3.f, 4.f};
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += stride * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t j = i + u * stride;
      if (j < n) {
        if constexpr (NT)
          __builtin_nontemporal_store(v, b + j);
        else
          b[j] = v;
      }
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void probe_copy(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += stride * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[min(i + u * stride, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t j = i + u * stride;
      if (j < n) {
        if constexpr (NT)
          __builtin_nontemporal_store(v[u], b + j);
        else
          b[j] = v[u];
      }
    }
  }
}

struct Best {
  double gbps = 0.0;
  int grid = 0, unroll = 0, nt = 0;
};

// `launch(grid)` timed over `reps` launches after one warm-up; bytes moved per launch
template <class F>
double time_gbps(F launch, int grid, double bytes, hipEvent_t e0, hipEvent_t e1, int reps = 4) {
  launch(grid);
  hip_check(hipEventRecord(e0, nullptr), "hipEventRecord");
  for (int r = 0; r < reps; ++r) launch(grid);
  hip_check(hipEventRecord(e1, nullptr), "hipEventRecord");
  hip_check(hipEventSynchronize(e1), "hipEventSynchronize");
  float ms = 0.f;
  hip_check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
  return bytes * reps / (ms * 1e-3) / 1e9;
}

template <int U, bool NT>
void sweep(const f4* a, f4* b, float* o, size_t n, hipEvent_t e0, hipEvent_t e1, Best& rd, Best& wr, Best& cp) {
  const double bytes = (double)n * 16.0;
  for (int grid : {1024, 2048, 4096, 8192}) {
    auto r = [&](int g) { hipLaunchKernelGGL((probe_read<U, NT>), dim3(g), dim3(256), 0, 0, a, n, o); };
    auto w = [&](int g) { hipLaunchKernelGGL((probe_write<U, NT>), dim3(g), dim3(256), 0, 0, b, n); };
    auto c = [&](int g) { hipLaunchKernelGGL((probe_copy<U, NT>), dim3(g), dim3(256), 0, 0, a, b, n); };
    const double gr = time_gbps(r, grid, bytes, e0, e1), gw = time_gbps(w, grid, bytes, e0, e1),
                 gc = time_gbps(c, grid, 2.0 * bytes, e0, e1);
    if (gr > rd.gbps) rd = {gr, grid, U, NT};
    if (gw > wr.gbps) wr = {gw, grid, U, NT};
    if (gc > cp.gbps) cp = {gc, grid, U, NT};
  }
  hip_check(hipGetLastError(), "hbm probe launch");
}

}  // namespace

extern "C" int mp_hbm_probe(int device, int64_t bytes, mp_hbm_rates* out) {
  return guard([&] {
    if (!out) fail(MP_ERR_ARG, "out is NULL");
    if (bytes < (int64_t)(64 << 20)) fail(MP_ERR_ARG, "bytes must be at least 64 MiB (past the caches)");
    hip_check(hipSetDevice(device), "hipSetDevice");
    const size_t n = (size_t)bytes / 16;
    DevBuf A, B, O;
    A.alloc(n * 16);
    B.alloc(n * 16);
    O.alloc(256 * sizeof(float));
    hip_check(hipMemset(A.p, 0, n * 16), "hipMemset");
    hipEvent_t e0, e1;
    hip_check(hipEventCreate(&e0), "hipEventCreate");
    hip_check(hipEventCreate(&e1), "hipEventCreate");
    Best rd, wr, cp;
    const f4* a = static_cast<const f4*>(A.p);
    f4* b = static_cast<f4*>(B.p);
    try {
      sweep<1, false>(a, b, O.f(), n, e0, e1, rd, wr, cp);
      sweep<4, false>(a, b, O.f(), n, e0, e1, rd, wr, cp);
      sweep<4, true>(a, b, O.f(), n, e0, e1, rd, wr, cp);
      sweep<8, true>(a, b, O.f(), n, e0, e1, rd, wr, cp);
    } catch (...) {
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      throw;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    *out = mp_hbm_rates{rd.gbps, wr.gbps, cp.gbps, rd.grid, rd.unroll, rd.nt, wr.grid, wr.unroll, wr.nt,
                        cp.grid, cp.unroll, cp.nt};
  });
}
