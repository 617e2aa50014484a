// Probe for the FFT_PACKED = 1 nondeterminism (k_fft.hip, DESIGN.md 3a''): does a packed-FP32
// VOP3P instruction whose destination pair is also its half-SWAPPED source pair read the swapped
// half before or after its own other half has been written?
//
//   v_pk_fma_f32 v[a:a+1], v[a:a+1], s[k:k+1], v[a:a+1] op_sel:[1,0,0] op_sel_hi:[0,1,1]
//     lo' = fma(v[a+1], s[k],   v[a])       (src0 lo lane reads the HI half: op_sel[0] = 1)
//     hi' = fma(v[a],   s[k+1], v[a+1])     (src0 hi lane reads the LO half: op_sel_hi[0] = 0)
//
// If the hardware ran the two halves as passes and the hi pass read v[a] after the lo pass wrote
// it, hi' would be fma(lo', s[k+1], v[a+1]).  The probe runs the exact instruction form the
// FFT_PACKED = 1 build emits (the half swap of swp() folded into op_sel, 7,902 such instructions in
// k_fft.hip; none in the default FFT_PACKED = 2 build), with the destination overlapping and --
// as the control -- not overlapping, at 1 .. 16 waves per SIMD, and counts lanes whose hi' is not
// the architectural result.
//   hipcc --offload-arch=gfx950 -O3 tools/pk_hazard.hip -o tools/bin/pk_hazard && tools/bin/pk_hazard
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

// ITER dependent instructions per lane; every iteration the pair is re-seeded from the lane's
// values so the expected result stays exactly computable on the host
template <bool OVERLAP>
__global__ __launch_bounds__(256) void probe(const float* __restrict__ in, float* __restrict__ out, int iters,
                                             float s0, float s1) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const float a = in[2 * i], b = in[2 * i + 1];
  float lo_sum = 0.f, hi_sum = 0.f;
  for (int k = 0; k < iters; ++k) {
    f2 x = {a + (float)k, b - (float)k};
    f2 d;
    if constexpr (OVERLAP) {
      d = x;
      asm volatile("v_pk_fma_f32 %0, %0, %1, %0 op_sel:[1,0,0] op_sel_hi:[0,1,1]" : "+v"(d) : "s"(f2{s0, s1}));
    } else {
      asm volatile("v_pk_fma_f32 %0, %1, %2, %1 op_sel:[1,0,0] op_sel_hi:[0,1,1]"
                   : "=&v"(d)
                   : "v"(x), "s"(f2{s0, s1}));
    }
    lo_sum += d.x;
    hi_sum += d.y;
  }
  out[2 * i] = lo_sum;
  out[2 * i + 1] = hi_sum;
}

int main() {
  const int iters = 256;
  const float s0 = 1.5f, s1 = -0.75f;
  for (int blocks_per_cu : {1, 4, 16}) {
    const int nb = 256 * blocks_per_cu, n = nb * 256;
    std::vector<float> h(2 * n), o(2 * n);
    for (int i = 0; i < 2 * n; ++i) h[i] = std::ldexp((float)((i * 2654435761u) % 1000u), -7);
    float *din, *dout;
    if (hipMalloc(&din, h.size() * 4) || hipMalloc(&dout, h.size() * 4)) return 1;
    if (hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice)) return 1;
    for (int ov = 0; ov < 2; ++ov) {
      if (ov)
        hipLaunchKernelGGL(probe<true>, dim3(nb), dim3(256), 0, 0, din, dout, iters, s0, s1);
      else
        hipLaunchKernelGGL(probe<false>, dim3(nb), dim3(256), 0, 0, din, dout, iters, s0, s1);
      if (hipDeviceSynchronize() || hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost)) return 1;
      long bad_lo = 0, bad_hi = 0, hazard_hi = 0;
      for (int i = 0; i < n; ++i) {
        const float a = h[2 * i], b = h[2 * i + 1];
        float lo = 0.f, hi = 0.f, hz = 0.f;
        for (int k = 0; k < iters; ++k) {
          const float xa = a + (float)k, xb = b - (float)k;
          const float l = std::fma(xb, s0, xa);
          lo += l;
          hi += std::fma(xa, s1, xb);
          hz += std::fma(l, s1, xb);   // what a hi pass reading the freshly written lo would give
        }
        bad_lo += o[2 * i] != lo;
        bad_hi += o[2 * i + 1] != hi;
        hazard_hi += o[2 * i + 1] == hz;
      }
      printf("{\"blocks_per_cu\": %d, \"dst_overlaps_swapped_src\": %s, \"lanes\": %d, \"lo_wrong\": %ld, "
             "\"hi_wrong\": %ld, \"hi_equals_read_after_write\": %ld}\n",
             blocks_per_cu, ov ? "true" : "false", n, bad_lo, bad_hi, hazard_hi);
    }
    (void)hipFree(din);
    (void)hipFree(dout);
  }
  return 0;
}
