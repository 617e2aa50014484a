/* A plain C client of libmonkeypose.so (include/monkeypose.h): no Python, no torch.
 *
 *   gcc -O2 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/abi_demo.c \
 *       -L monkey-pose_amd -lmonkeypose -L /opt/rocm/lib -lamdhip64 \
 *       -Wl,-rpath,$PWD/monkey-pose_amd -Wl,-rpath,/opt/rocm/lib -o tools/bin/abi_demo
 *   tools/bin/abi_demo <dir>
 *
 * <dir> holds manifest.txt ("n h w output_shape dtype" then one line per weight: "name ndim d0 d1
 * ..."), weights.bin (the weights' float32 bytes in manifest order), depth.bin ([n,h,w,1]) and
 * o0.bin ([n,h/2,w/2,64]).  Writes out.bin ([n,output_shape]).  Used by tests/test_abi_cpu.py's GPU
 * test to show the ABI is callable from C exactly as the ctypes binding calls it. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "monkeypose.h"

#define CK(call, what)                                                        \
  do {                                                                        \
    int rc_ = (call);                                                         \
    if (rc_ != 0) {                                                           \
      fprintf(stderr, "%s failed (%d): %s\n", what, rc_, mp_last_error());    \
      return 1;                                                               \
    }                                                                         \
  } while (0)

static float* read_all(const char* dir, const char* name, size_t count) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  float* p = (float*)malloc(count * sizeof(float));
  if (p && fread(p, sizeof(float), count, f) != count) {
    free(p);
    p = NULL;
  }
  fclose(f);
  return p;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <dir>\n", argv[0]);
    return 2;
  }
  const char* dir = argv[1];
  char path[4096];
  snprintf(path, sizeof path, "%s/manifest.txt", dir);
  FILE* mf = fopen(path, "r");
  if (!mf) return 2;
  long n, h, w, nout;
  int dtype;
  if (fscanf(mf, "%ld %ld %ld %ld %d", &n, &h, &w, &nout, &dtype) != 5) return 2;

  mp_ctx* ctx = NULL;
  CK(mp_create(0, MP_MODEL_HGRU_POSE, &ctx), "mp_create");
  snprintf(path, sizeof path, "%s/weights.bin", dir);
  FILE* wf = fopen(path, "rb");
  if (!wf) return 2;
  char name[512];
  int ndim;
  while (fscanf(mf, "%511s %d", name, &ndim) == 2) {
    int64_t shape[8];
    size_t cnt = 1;
    for (int i = 0; i < ndim; ++i) {
      long d;
      if (fscanf(mf, "%ld", &d) != 1) return 2;
      shape[i] = d;
      cnt *= (size_t)d;
    }
    float* buf = (float*)malloc(cnt * sizeof(float));
    if (!buf || fread(buf, sizeof(float), cnt, wf) != cnt) return 2;
    CK(mp_set_weight(ctx, name, buf, shape, ndim, MP_MEM_HOST), "mp_set_weight");
    free(buf);
  }
  fclose(wf);
  fclose(mf);
  CK(mp_finalize_weights(ctx, dtype), "mp_finalize_weights");

  const size_t nd = (size_t)n * h * w, no0 = (size_t)n * (h / 2) * (w / 2) * 64, nres = (size_t)n * nout;
  float* depth = read_all(dir, "depth.bin", nd);
  float* o0 = read_all(dir, "o0.bin", no0);
  if (!depth || !o0) return 2;
  float *d_depth, *d_o0, *d_out;
  if (hipMalloc((void**)&d_depth, nd * 4) || hipMalloc((void**)&d_o0, no0 * 4) || hipMalloc((void**)&d_out, nres * 4))
    return 3;
  if (hipMemcpy(d_depth, depth, nd * 4, hipMemcpyHostToDevice) || hipMemcpy(d_o0, o0, no0 * 4, hipMemcpyHostToDevice))
    return 3;
  hipStream_t st;
  if (hipStreamCreate(&st)) return 3;
  CK(mp_hgru_pose_fwd(ctx, d_depth, n, h, w, d_o0, d_out, st), "mp_hgru_pose_fwd");
  if (hipStreamSynchronize(st)) return 3;
  float* out = (float*)malloc(nres * 4);
  if (hipMemcpy(out, d_out, nres * 4, hipMemcpyDeviceToHost)) return 3;
  snprintf(path, sizeof path, "%s/out.bin", dir);
  FILE* of = fopen(path, "wb");
  if (!of || fwrite(out, 4, nres, of) != nres) return 2;
  fclose(of);
  printf("abi_demo: n=%ld out[0][0..2] = %g %g %g\n", n, out[0], out[1], out[2]);
  mp_destroy(ctx);
  return 0;
}
