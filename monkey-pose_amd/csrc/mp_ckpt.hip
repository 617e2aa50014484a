// Host-side helper of the TF1 checkpoint reader (monkey-pose_amd/tf_checkpoint.py):
// CRC-32C (Castagnoli) of tensor payloads, as tensorflow/core/util/tensor_bundle stores it
// (BundleEntryProto.crc32c, masked) and as LevelDB-format tables store per-block checksums.
// Plain host code (no GPU): SSE4.2 crc32 instructions, 8 bytes per step, on x86-64.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "../../include/monkeypose.h"

namespace {

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
  return ~(uint32_t)c;
}

}  // namespace

extern "C" {

uint32_t mp_crc32c(uint32_t init, const void* data, size_t n) {
  if (!data || !n) return init;
  return crc32c_hw(init, static_cast<const uint8_t*>(data), n);
}

}  // extern "C"
