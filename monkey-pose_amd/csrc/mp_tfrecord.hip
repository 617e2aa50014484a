// TFRecord ingestion, host code: the reader side of data_loader.py:10-40
// (tf.TFRecordReader -> tf.parse_single_example({'label', 'image': FixedLenFeature([], string)})
// -> tf.decode_raw(float32)) and the writer of Datareader.py:13-27 (encode_example ->
// TFRecordWriter), without TensorFlow.
//
// File format (TFRecord): per record  uint64 length | uint32 masked_crc32c(length bytes) |
// data[length] | uint32 masked_crc32c(data), little endian; mask(c) = ((c >> 15) | (c << 17)) +
// 0xa282ead8.  data = a serialized tf.train.Example:
//   Example { Features features = 1; }   Features { map<string, Feature> feature = 1; }
//   Feature { oneof { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3; } }
//   BytesList { repeated bytes value = 1; }
// The file is memory-mapped and indexed once (length CRCs always checked, payload CRCs on request);
// batches are gathered by record index (the caller's shuffle) and decoded by a pool of host
// threads straight into the caller's (pinned) buffer.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mp_runtime.hpp"

struct mp_tfrecord {
  int fd = -1;
  const uint8_t* base = nullptr;
  size_t size = 0;
  std::vector<size_t> off;   // payload offset of record i
  std::vector<size_t> len;   // payload length
  ~mp_tfrecord() {
    if (base) munmap(const_cast<uint8_t*>(base), size);
    if (fd >= 0) close(fd);
  }
};

namespace {

uint32_t mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

// protobuf wire format: varint / length-delimited fields
bool varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int s = 0; s < 64 && p < end; s += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) return true;
  }
  return false;
}

struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
};

// first length-delimited field `field` of a message (false if absent / malformed)
bool field_len(Span m, uint32_t field, Span& out, Span* rest = nullptr) {
  const uint8_t *p = m.p, *end = m.p + m.n;
  while (p < end) {
    uint64_t key;
    if (!varint(p, end, key)) return false;
    const uint32_t f = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    uint64_t v;
    switch (wt) {
      case 0:
        if (!varint(p, end, v)) return false;
        break;
      case 1:
        if (end - p < 8) return false;
        p += 8;
        break;
      case 5:
        if (end - p < 4) return false;
        p += 4;
        break;
      case 2:
        if (!varint(p, end, v) || v > (uint64_t)(end - p)) return false;
        if (f == field) {
          out = {p, (size_t)v};
          if (rest) *rest = {p + v, (size_t)(end - p - v)};
          return true;
        }
        p += v;
        break;
      default:
        return false;
    }
  }
  return false;
}

// Example -> the raw bytes of feature `name` (bytes_list value[0], or the packed float_list)
bool find_feature(Span ex, const std::string& name, Span& raw) {
  Span feats;
  if (!field_len(ex, 1, feats)) return false;
  Span rest = feats, entry;
  while (rest.n && field_len(rest, 1, entry, &rest)) {
    Span key, val;
    if (!field_len(entry, 1, key) || key.n != name.size() || std::memcmp(key.p, name.data(), key.n)) continue;
    if (!field_len(entry, 2, val)) return false;
    Span list;
    if (field_len(val, 1, list)) return field_len(list, 1, raw);   // BytesList.value[0]
    if (field_len(val, 2, list)) return field_len(list, 1, raw);   // FloatList.value (packed)
    return false;
  }
  return false;
}

void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)((v & 0x7f) | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}

void put_len(std::string& s, uint32_t field, const std::string& body) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, body.size());
  s += body;
}

// encode_example (Datareader.py:13-19): {name: bytes_feature(raw)} in the given order
std::string encode_example(int nf, const char* const* names, const uint8_t* const* raw, const int64_t* bytes) {
  std::string feats;
  for (int i = 0; i < nf; ++i) {
    std::string blist, feat, entry;
    put_len(blist, 1, std::string(reinterpret_cast<const char*>(raw[i]), (size_t)bytes[i]));
    put_len(feat, 1, blist);
    put_len(entry, 1, std::string(names[i]));
    put_len(entry, 2, feat);
    put_len(feats, 1, entry);
  }
  std::string ex;
  put_len(ex, 1, feats);
  return ex;
}

}  // namespace

extern "C" {

int mp_tfrecord_open(const char* path, int verify, mp_tfrecord** out, int64_t* n_records) {
  return guard([&] {
    if (!path || !out) fail(MP_ERR_ARG, "mp_tfrecord_open: null pointer");
    auto r = std::make_unique<mp_tfrecord>();
    r->fd = open(path, O_RDONLY);
    if (r->fd < 0) fail(MP_ERR_ARG, std::string("cannot open ") + path);
    struct stat st;
    if (fstat(r->fd, &st) != 0) fail(MP_ERR_ARG, std::string("cannot stat ") + path);
    r->size = (size_t)st.st_size;
    if (r->size) {
      void* m = mmap(nullptr, r->size, PROT_READ, MAP_PRIVATE, r->fd, 0);
      if (m == MAP_FAILED) fail(MP_ERR_ARG, std::string("cannot mmap ") + path);
      r->base = static_cast<const uint8_t*>(m);
    }
    size_t p = 0;
    while (p < r->size) {
      if (r->size - p < 12) fail(MP_ERR_ARG, "truncated record header at byte " + std::to_string(p));
      const uint64_t n = rd64(r->base + p);
      if (mask(mp_crc32c(0, r->base + p, 8)) != rd32(r->base + p + 8))
        fail(MP_ERR_ARG, "corrupted record length (crc) at byte " + std::to_string(p));
      if (n > r->size - p - 12 || r->size - p - 12 - n < 4)
        fail(MP_ERR_ARG, "truncated record at byte " + std::to_string(p));
      const uint8_t* d = r->base + p + 12;
      if (verify && mask(mp_crc32c(0, d, n)) != rd32(d + n))
        fail(MP_ERR_ARG, "corrupted record data (crc) in record " + std::to_string(r->off.size()));
      r->off.push_back(p + 12);
      r->len.push_back(n);
      p += 12 + n + 4;
    }
    if (n_records) *n_records = (int64_t)r->off.size();
    *out = r.release();
  });
}

void mp_tfrecord_close(mp_tfrecord* r) { delete r; }

int mp_tfrecord_feature_size(mp_tfrecord* r, int64_t rec, const char* feature, int64_t* bytes) {
  return guard([&] {
    if (!r || !feature || !bytes) fail(MP_ERR_ARG, "mp_tfrecord_feature_size: null pointer");
    if (rec < 0 || rec >= (int64_t)r->off.size()) fail(MP_ERR_ARG, "record index out of range");
    Span raw;
    if (!find_feature({r->base + r->off[rec], r->len[rec]}, feature, raw))
      fail(MP_ERR_ARG, "record " + std::to_string(rec) + " has no bytes feature '" + feature + "'");
    *bytes = (int64_t)raw.n;
  });
}

int mp_tfrecord_read(mp_tfrecord* r, const int64_t* indices, int64_t count, const char* feature, void* out,
                     int64_t bytes_per_record, int nthreads) {
  return guard([&] {
    if (!r || !indices || !feature || (!out && count > 0) || count < 0 || bytes_per_record <= 0)
      fail(MP_ERR_ARG, "mp_tfrecord_read: bad argument");
    const std::string name(feature);
    for (int64_t i = 0; i < count; ++i)
      if (indices[i] < 0 || indices[i] >= (int64_t)r->off.size())
        fail(MP_ERR_ARG, "record index " + std::to_string(indices[i]) + " out of range");
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(std::max(1, nthreads), count));
    std::vector<int64_t> bad(nt, -1);
    std::vector<int64_t> badsz(nt, 0);
    auto work = [&](int t) {
      for (int64_t i = t; i < count; i += nt) {
        const int64_t rec = indices[i];
        Span raw;
        if (!find_feature({r->base + r->off[rec], r->len[rec]}, name, raw) || (int64_t)raw.n != bytes_per_record) {
          bad[t] = rec;
          badsz[t] = (int64_t)raw.n;
          return;
        }
        std::memcpy(static_cast<uint8_t*>(out) + i * bytes_per_record, raw.p, raw.n);
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (int t = 0; t < nt; ++t)
      if (bad[t] >= 0)
        fail(MP_ERR_SHAPE, "record " + std::to_string(bad[t]) + ": feature '" + name + "' has " +
                               std::to_string(badsz[t]) + " bytes, expected " + std::to_string(bytes_per_record));
  });
}

int mp_tfrecord_write(const char* path, int64_t n_records, int n_features, const char* const* names,
                      const void* const* data, const int64_t* bytes_per_record, int append) {
  return guard([&] {
    if (!path || n_records < 0 || n_features <= 0 || !names || !data || !bytes_per_record)
      fail(MP_ERR_ARG, "mp_tfrecord_write: bad argument");
    FILE* f = std::fopen(path, append ? "ab" : "wb");
    if (!f) fail(MP_ERR_ARG, std::string("cannot open ") + path + " for writing");
    std::vector<const uint8_t*> raw(n_features);
    bool ok = true;
    for (int64_t i = 0; i < n_records && ok; ++i) {
      for (int k = 0; k < n_features; ++k)
        raw[k] = static_cast<const uint8_t*>(data[k]) + i * bytes_per_record[k];
      const std::string ex = encode_example(n_features, names, raw.data(), bytes_per_record);
      uint8_t hdr[12];
      const uint64_t n = ex.size();
      std::memcpy(hdr, &n, 8);
      const uint32_t hc = mask(mp_crc32c(0, hdr, 8));
      std::memcpy(hdr + 8, &hc, 4);
      const uint32_t dc = mask(mp_crc32c(0, ex.data(), ex.size()));
      ok = std::fwrite(hdr, 1, 12, f) == 12 && std::fwrite(ex.data(), 1, ex.size(), f) == ex.size() &&
           std::fwrite(&dc, 1, 4, f) == 4;
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) fail(MP_ERR_ARG, std::string("write failed: ") + path);
  });
}

}  // extern "C"
