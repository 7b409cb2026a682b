// Zero-copy PredictRequest / PredictResponse codec. See tensor_codec.h.
#include "tensor_codec.h"

#include <immintrin.h>

#include <algorithm>

#include <cmath>
#include <cstring>

namespace dtfs {
namespace wire {

namespace {

enum WireType { WT_VARINT = 0, WT_FIXED64 = 1, WT_LEN = 2, WT_FIXED32 = 5 };

struct Reader {
  const uint8_t* p;
  const uint8_t* end;

  bool eof() const { return p >= end; }

  bool varint(uint64_t* v) {
    uint64_t r = 0;
    int shift = 0;
    while (p < end) {
      uint8_t b = *p++;
      r |= uint64_t(b & 0x7F) << shift;
      if (!(b & 0x80)) {
        *v = r;
        return true;
      }
      shift += 7;
      if (shift >= 70) return false;
    }
    return false;
  }

  bool fixed32(uint32_t* v) {
    if (end - p < 4) return false;
    std::memcpy(v, p, 4);
    p += 4;
    return true;
  }

  bool fixed64(uint64_t* v) {
    if (end - p < 8) return false;
    std::memcpy(v, p, 8);
    p += 8;
    return true;
  }

  bool len_delim(Span* s) {
    uint64_t n;
    if (!varint(&n)) return false;
    if (n > uint64_t(end - p)) return false;
    s->p = p;
    s->n = size_t(n);
    p += n;
    return true;
  }

  bool skip(int wt) {
    uint64_t v;
    Span s;
    switch (wt) {
      case WT_VARINT: return varint(&v);
      case WT_FIXED64: return fixed64(&v);
      case WT_LEN: return len_delim(&s);
      case WT_FIXED32: {
        uint32_t x;
        return fixed32(&x);
      }
      default: return false;  // groups (3/4) are not used by any serving message
    }
  }
};

// Typed value field number for each dtype (reference tensor.proto:38-80).
int value_field_for(int dtype) {
  switch (dtype) {
    case DT_FLOAT: return 5;
    case DT_DOUBLE: return 6;
    case DT_INT32: case DT_UINT8: case DT_INT16: case DT_INT8: case DT_UINT16: return 7;
    case DT_INT64: return 10;
    case DT_BOOL: return 11;
    case DT_HALF: case DT_BFLOAT16: return 13;
    case DT_UINT32: return 16;
    case DT_UINT64: return 17;
    default: return 0;
  }
}

int field_wire_kind(int field) {  // 0 varint, 1 fixed64, 5 fixed32, -1 other
  switch (field) {
    case 5: case 9: return WT_FIXED32;
    case 6: case 12: return WT_FIXED64;
    case 7: case 10: case 11: case 13: case 16: case 17: return WT_VARINT;
    default: return -1;
  }
}

size_t dtype_size(int dtype) {
  switch (dtype) {
    case DT_FLOAT: case DT_INT32: case DT_UINT32: return 4;
    case DT_DOUBLE: case DT_INT64: case DT_UINT64: return 8;
    case DT_HALF: case DT_BFLOAT16: case DT_INT16: case DT_UINT16: return 2;
    case DT_UINT8: case DT_INT8: case DT_BOOL: return 1;
    default: return 0;
  }
}

bool is_float_dtype(int dtype) {
  return dtype == DT_FLOAT || dtype == DT_DOUBLE || dtype == DT_HALF || dtype == DT_BFLOAT16;
}

float half_to_f32(uint16_t h) {
  uint32_t sign = uint32_t(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1F;
  uint32_t mant = h & 0x3FF;
  uint32_t bits;
  if (exp == 0) {
    if (mant == 0) {
      bits = sign;
    } else {  // subnormal
      int e = -1;
      do {
        mant <<= 1;
        ++e;
      } while (!(mant & 0x400));
      mant &= 0x3FF;
      bits = sign | (uint32_t(127 - 15 - e) << 23) | (mant << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7F800000u | (mant << 13);
  } else {
    bits = sign | ((exp + 127 - 15) << 23) | (mant << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

float bf16_to_f32(uint16_t h) {
  uint32_t bits = uint32_t(h) << 16;
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

namespace {
int64_t count_terms_sse2(const uint8_t* p, size_t n) {
  // bytes with MSB clear compare > -1 as int8: subtract the 0xFF masks from a
  // per-byte counter (<= 255 steps), then sum the counters with SAD
  int64_t c = 0;
  size_t i = 0;
  const __m128i neg1 = _mm_set1_epi8(-1), zero = _mm_setzero_si128();
  while (i + 16 <= n) {
    __m128i acc = zero;
    const size_t stop = std::min(n - 15, i + 16 * 255);
    for (; i < stop; i += 16)
      acc = _mm_sub_epi8(acc, _mm_cmpgt_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i)), neg1));
    const __m128i s = _mm_sad_epu8(acc, zero);
    c += _mm_cvtsi128_si64(s) + _mm_cvtsi128_si64(_mm_unpackhi_epi64(s, s));
  }
  for (; i < n; ++i) c += (p[i] & 0x80) == 0;
  return c;
}

__attribute__((target("avx2"))) int64_t count_terms_avx2(const uint8_t* p, size_t n) {
  int64_t c = 0;
  size_t i = 0;
  const __m256i neg1 = _mm256_set1_epi8(-1), zero = _mm256_setzero_si256();
  while (i + 32 <= n) {
    __m256i acc = zero;
    const size_t stop = std::min(n - 31, i + 32 * 255);
    for (; i < stop; i += 32)
      acc = _mm256_sub_epi8(acc,
                            _mm256_cmpgt_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i)), neg1));
    const __m256i s = _mm256_sad_epu8(acc, zero);
    c += _mm256_extract_epi64(s, 0) + _mm256_extract_epi64(s, 1) + _mm256_extract_epi64(s, 2) +
         _mm256_extract_epi64(s, 3);
  }
  return c + count_terms_sse2(p + i, n - i);
}

const bool g_avx2 = __builtin_cpu_supports("avx2");
}  // namespace

int64_t count_terms(const uint8_t* p, size_t n) { return g_avx2 ? count_terms_avx2(p, n) : count_terms_sse2(p, n); }

int64_t count_varints(const Span& s) { return count_terms(s.p, s.n); }

bool parse_shape(Span s, TensorView* t, std::string* err) {
  Reader r{s.p, s.p + s.n};
  while (!r.eof()) {
    uint64_t tag;
    if (!r.varint(&tag)) return *err = "bad shape tag", false;
    int f = int(tag >> 3), wt = int(tag & 7);
    if (f == 2 && wt == WT_LEN) {
      Span ds;
      if (!r.len_delim(&ds)) return *err = "bad dim", false;
      Reader dr{ds.p, ds.p + ds.n};
      int64_t size = 0;
      while (!dr.eof()) {
        uint64_t dtag;
        if (!dr.varint(&dtag)) return *err = "bad dim tag", false;
        if ((dtag >> 3) == 1 && (dtag & 7) == WT_VARINT) {
          uint64_t v;
          if (!dr.varint(&v)) return *err = "bad dim size", false;
          size = int64_t(v);
        } else if (!dr.skip(int(dtag & 7))) {
          return *err = "bad dim field", false;
        }
      }
      t->shape.push_back(size);
    } else if (f == 3 && wt == WT_VARINT) {
      uint64_t v;
      if (!r.varint(&v)) return *err = "bad unknown_rank", false;
      t->unknown_rank = v != 0;
    } else if (!r.skip(wt)) {
      return *err = "bad shape field", false;
    }
  }
  return true;
}

struct RawChunk {
  int field;
  bool packed;
  Span span;
  uint64_t scalar;
};

bool parse_tensor_impl(Span s, TensorView* t, std::string* err, bool count_varints_ = true) {
  Reader r{s.p, s.p + s.n};
  std::vector<RawChunk> chunks;
  while (!r.eof()) {
    uint64_t tag;
    if (!r.varint(&tag)) return *err = "bad tensor tag", false;
    int f = int(tag >> 3), wt = int(tag & 7);
    if (f == 1 && wt == WT_VARINT) {
      uint64_t v;
      if (!r.varint(&v)) return *err = "bad dtype", false;
      t->dtype = int(v);
    } else if (f == 2 && wt == WT_LEN) {
      Span ss;
      if (!r.len_delim(&ss)) return *err = "bad tensor_shape", false;
      t->shape.clear();
      if (!parse_shape(ss, t, err)) return false;
    } else if (f == 4 && wt == WT_LEN) {
      if (!r.len_delim(&t->content)) return *err = "bad tensor_content", false;
    } else if (field_wire_kind(f) >= 0) {
      int kind = field_wire_kind(f);
      RawChunk c{f, false, {}, 0};
      if (wt == WT_LEN) {
        c.packed = true;
        if (!r.len_delim(&c.span)) return *err = "bad packed field", false;
      } else if (wt == kind) {
        if (wt == WT_VARINT) {
          if (!r.varint(&c.scalar)) return *err = "bad varint value", false;
        } else if (wt == WT_FIXED32) {
          uint32_t x;
          if (!r.fixed32(&x)) return *err = "bad fixed32 value", false;
          c.scalar = x;
        } else {
          if (!r.fixed64(&c.scalar)) return *err = "bad fixed64 value", false;
        }
      } else {
        return *err = "wire type mismatch in typed value field", false;
      }
      chunks.push_back(c);
    } else if (!r.skip(wt)) {
      return *err = "bad tensor field", false;
    }
  }
  // Keep only the typed field that belongs to the dtype.
  t->value_field = value_field_for(t->dtype);
  int kind = field_wire_kind(t->value_field);
  t->value_packed_varint = kind == WT_VARINT;
  t->value_fixed32 = kind == WT_FIXED32;
  t->value_fixed64 = kind == WT_FIXED64;
  t->num_values = 0;
  bool uncounted = false;  // packed varints left for the caller to count (see header)
  for (const RawChunk& c : chunks) {
    if (c.field != t->value_field) continue;
    if (c.packed) {
      t->packed.push_back(c.span);
      if (kind == WT_VARINT) {
        if (count_varints_) t->num_values += count_varints(c.span);
        else uncounted = true;
      }
      else if (kind == WT_FIXED32) {
        if (c.span.n % 4) return *err = "packed fixed32 length not a multiple of 4", false;
        t->num_values += int64_t(c.span.n / 4);
      } else {
        if (c.span.n % 8) return *err = "packed fixed64 length not a multiple of 8", false;
        t->num_values += int64_t(c.span.n / 8);
      }
    } else {
      // Unpacked singles: keep them in order relative to packed chunks by
      // materialising as a tiny 'packed' span is impossible (no backing
      // bytes), so unpacked values go to a side vector. Mixed packed+unpacked
      // encodings of one field do not occur in practice; if they do, unpacked
      // values are appended after the packed ones.
      t->unpacked.push_back(c.scalar);
      t->num_values += 1;
    }
  }
  if (uncounted) t->num_values = -1;
  return true;
}

// Value sources ----------------------------------------------------------
template <typename F>
bool for_each_int(const TensorView& t, F&& fn) {
  for (const Span& s : t.packed) {
    Reader r{s.p, s.p + s.n};
    while (!r.eof()) {
      uint64_t v;
      if (!r.varint(&v)) return false;
      fn(v);
    }
  }
  for (uint64_t v : t.unpacked) fn(v);
  return true;
}

template <typename F>
void for_each_f32(const TensorView& t, F&& fn) {
  for (const Span& s : t.packed) {
    const uint8_t* p = s.p;
    size_t n = s.n / 4;
    for (size_t i = 0; i < n; ++i) {
      float f;
      std::memcpy(&f, p + 4 * i, 4);
      fn(f);
    }
  }
  for (uint64_t v : t.unpacked) {
    uint32_t u = uint32_t(v);
    float f;
    std::memcpy(&f, &u, 4);
    fn(f);
  }
}

template <typename F>
void for_each_f64(const TensorView& t, F&& fn) {
  for (const Span& s : t.packed) {
    size_t n = s.n / 8;
    for (size_t i = 0; i < n; ++i) {
      double d;
      std::memcpy(&d, s.p + 8 * i, 8);
      fn(d);
    }
  }
  for (uint64_t v : t.unpacked) {
    double d;
    std::memcpy(&d, &v, 8);
    fn(d);
  }
}

inline int64_t int_from_varint(int dtype, uint64_t v) {
  switch (dtype) {
    case DT_INT32: case DT_INT16: case DT_INT8: return int64_t(int32_t(uint32_t(v)));
    case DT_UINT8: return int64_t(v & 0xFF);
    case DT_UINT16: return int64_t(v & 0xFFFF);
    case DT_UINT32: return int64_t(uint32_t(v));
    default: return int64_t(v);
  }
}

inline int64_t apply_mod(int64_t id, int64_t m) {
  if (m <= 0) return id;
  int64_t r = id % m;
  return r < 0 ? r + m : r;
}

// Writes logical element i of the destination. The destination is a row view:
// `cols` elements per row, rows `ld` elements apart (ld == cols: contiguous),
// so a packed request row [ids | wts | pad] can be filled in place.
struct Writer {
  void* dst;
  DstType type;
  int64_t mod;
  int64_t cols;
  int64_t ld;
  bool contiguous;
  int64_t next_i = 0, r = 0, c = 0;  // sequential-access cursor

  Writer(void* d, DstType t, int64_t m, int64_t cols_, int64_t ld_)
      : dst(d), type(t), mod(m), cols(cols_ > 0 ? cols_ : 1), ld(ld_ > 0 ? ld_ : cols_), contiguous(ld_ <= 0 || ld_ == cols_) {}

  inline int64_t at(int64_t i) {
    if (contiguous) return i;
    if (i != next_i) {
      r = i / cols;
      c = i % cols;
    }
    const int64_t p = r * ld + c;
    next_i = i + 1;
    if (++c == cols) {
      c = 0;
      ++r;
    }
    return p;
  }
  inline void put_int(int64_t i, int64_t v) {
    const int64_t p = at(i);
    switch (type) {
      case DstType::I32: static_cast<int32_t*>(dst)[p] = int32_t(apply_mod(v, mod)); break;
      case DstType::I64: static_cast<int64_t*>(dst)[p] = apply_mod(v, mod); break;
      case DstType::F32: static_cast<float*>(dst)[p] = float(v); break;
      case DstType::BF16: static_cast<uint16_t*>(dst)[p] = f32_to_bf16(float(v)); break;
    }
  }
  inline void put_float(int64_t i, float v) {
    const int64_t p = at(i);
    switch (type) {
      case DstType::F32: static_cast<float*>(dst)[p] = v; break;
      case DstType::BF16: static_cast<uint16_t*>(dst)[p] = f32_to_bf16(v); break;
      default: break;  // rejected earlier
    }
  }
  inline void put_bits16(int64_t i, uint16_t h) { static_cast<uint16_t*>(dst)[at(i)] = h; }
  size_t elem_size() const { return (type == DstType::I64) ? 8 : (type == DstType::BF16 ? 2 : 4); }
  // Row-wise copy of n same-typed source elements (memcpy path).
  void copy_rows(const uint8_t* src, int64_t n) {
    const size_t es = elem_size();
    if (contiguous) {
      std::memcpy(dst, src, size_t(n) * es);
      return;
    }
    for (int64_t i = 0, row = 0; i < n; i += cols, ++row) {
      const int64_t k = std::min<int64_t>(cols, n - i);
      std::memcpy(static_cast<char*>(dst) + size_t(row * ld) * es, src + size_t(i) * es, size_t(k) * es);
    }
  }
  void fill_from(int64_t from, int64_t i0, int64_t n) {  // elements [i0, n) = element `from`
    const size_t es = elem_size();
    int64_t pf = contiguous ? from : (from / cols) * ld + from % cols;
    char buf[8];
    std::memcpy(buf, static_cast<char*>(dst) + size_t(pf) * es, es);
    for (int64_t i = i0; i < n; ++i) std::memcpy(static_cast<char*>(dst) + size_t(at(i)) * es, buf, es);
  }
};

}  // namespace

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return uint16_t((u >> 16) | 0x40);  // keep NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

int64_t TensorView::num_elements() const {
  int64_t n = 1;
  for (int64_t d : shape) n *= d;
  return n;
}

const TensorView* PredictRequestView::find(const std::string& key) const {
  for (const auto& kv : inputs)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

bool parse_tensor(const uint8_t* buf, size_t len, TensorView* out, std::string* err) {
  return parse_tensor_impl(Span{buf, len}, out, err);
}

bool parse_predict_request(const uint8_t* buf, size_t len, PredictRequestView* out, std::string* err,
                           bool count_packed_varints) {
  Reader r{buf, buf + len};
  while (!r.eof()) {
    uint64_t tag;
    if (!r.varint(&tag)) return *err = "bad request tag", false;
    int f = int(tag >> 3), wt = int(tag & 7);
    if (f == 1 && wt == WT_LEN) {  // model_spec
      Span ms;
      if (!r.len_delim(&ms)) return *err = "bad model_spec", false;
      Reader mr{ms.p, ms.p + ms.n};
      while (!mr.eof()) {
        uint64_t mtag;
        if (!mr.varint(&mtag)) return *err = "bad model_spec tag", false;
        int mf = int(mtag >> 3), mwt = int(mtag & 7);
        Span v;
        if (mf == 1 && mwt == WT_LEN) {
          if (!mr.len_delim(&v)) return *err = "bad model name", false;
          out->model_name.assign(reinterpret_cast<const char*>(v.p), v.n);
        } else if (mf == 3 && mwt == WT_LEN) {
          if (!mr.len_delim(&v)) return *err = "bad signature", false;
          out->signature_name.assign(reinterpret_cast<const char*>(v.p), v.n);
        } else if (mf == 2 && mwt == WT_LEN) {  // google.protobuf.Int64Value
          if (!mr.len_delim(&v)) return *err = "bad version", false;
          out->has_version = true;
          out->version = 0;
          Reader vr{v.p, v.p + v.n};
          while (!vr.eof()) {
            uint64_t vtag, x;
            if (!vr.varint(&vtag)) return *err = "bad version tag", false;
            if ((vtag >> 3) == 1 && (vtag & 7) == WT_VARINT) {
              if (!vr.varint(&x)) return *err = "bad version value", false;
              out->version = int64_t(x);
            } else if (!vr.skip(int(vtag & 7))) {
              return *err = "bad version field", false;
            }
          }
        } else if (!mr.skip(mwt)) {
          return *err = "bad model_spec field", false;
        }
      }
    } else if (f == 2 && wt == WT_LEN) {  // inputs map entry
      Span es;
      if (!r.len_delim(&es)) return *err = "bad inputs entry", false;
      Reader er{es.p, es.p + es.n};
      std::string key;
      Span value{nullptr, 0};
      while (!er.eof()) {
        uint64_t etag;
        if (!er.varint(&etag)) return *err = "bad entry tag", false;
        int ef = int(etag >> 3), ewt = int(etag & 7);
        Span v;
        if (ef == 1 && ewt == WT_LEN) {
          if (!er.len_delim(&v)) return *err = "bad entry key", false;
          key.assign(reinterpret_cast<const char*>(v.p), v.n);
        } else if (ef == 2 && ewt == WT_LEN) {
          if (!er.len_delim(&value)) return *err = "bad entry value", false;
        } else if (!er.skip(ewt)) {
          return *err = "bad entry field", false;
        }
      }
      TensorView tv;
      if (!parse_tensor_impl(value, &tv, err, count_packed_varints)) return false;
      // Map semantics: the last entry for a key wins.
      bool replaced = false;
      for (auto& kv : out->inputs)
        if (kv.first == key) {
          kv.second = std::move(tv);
          replaced = true;
        }
      if (!replaced) out->inputs.emplace_back(std::move(key), std::move(tv));
    } else if (f == 3 && wt == WT_LEN) {
      Span v;
      if (!r.len_delim(&v)) return *err = "bad output_filter", false;
      out->output_filter.emplace_back(reinterpret_cast<const char*>(v.p), v.n);
    } else if (!r.skip(wt)) {
      return *err = "bad request field", false;
    }
  }
  return true;
}

bool decode_into(const TensorView& t, void* dst, int64_t n, const DecodeOpts& opts, std::string* err) {
  const bool dst_int = opts.dst == DstType::I32 || opts.dst == DstType::I64;
  if (dst_int && is_float_dtype(t.dtype)) return *err = "cannot decode a floating tensor into integer ids", false;
  if (t.dtype == DT_STRING || dtype_size(t.dtype) == 0) return *err = "unsupported tensor dtype", false;
  const int64_t mod = dst_int ? opts.id_modulo : 0;
  Writer w(dst, opts.dst, mod, opts.cols > 0 ? opts.cols : n, opts.ld);

  if (t.content.n > 0) {
    const size_t es = dtype_size(t.dtype);
    if (t.content.n != size_t(n) * es) return *err = "tensor_content size does not match shape", false;
    const uint8_t* p = t.content.p;
    switch (t.dtype) {
      case DT_FLOAT:
        if (opts.dst == DstType::F32) {
          w.copy_rows(p, n);
        } else {
          for (int64_t i = 0; i < n; ++i) {
            float f;
            std::memcpy(&f, p + 4 * i, 4);
            w.put_float(i, f);
          }
        }
        return true;
      case DT_DOUBLE:
        for (int64_t i = 0; i < n; ++i) {
          double d;
          std::memcpy(&d, p + 8 * i, 8);
          w.put_float(i, float(d));
        }
        return true;
      case DT_HALF:
        for (int64_t i = 0; i < n; ++i) {
          uint16_t h;
          std::memcpy(&h, p + 2 * i, 2);
          w.put_float(i, half_to_f32(h));
        }
        return true;
      case DT_BFLOAT16:
        if (opts.dst == DstType::BF16) {
          w.copy_rows(p, n);
          return true;
        }
        for (int64_t i = 0; i < n; ++i) {
          uint16_t h;
          std::memcpy(&h, p + 2 * i, 2);
          w.put_float(i, bf16_to_f32(h));
        }
        return true;
      case DT_INT64: case DT_UINT64:
        if (opts.dst == DstType::I64 && mod <= 0) {
          w.copy_rows(p, n);
          return true;
        }
        for (int64_t i = 0; i < n; ++i) {
          int64_t v;
          std::memcpy(&v, p + 8 * i, 8);
          w.put_int(i, v);
        }
        return true;
      case DT_INT32:
        if (opts.dst == DstType::I32 && mod <= 0) {
          w.copy_rows(p, n);
          return true;
        }
        for (int64_t i = 0; i < n; ++i) {
          int32_t v;
          std::memcpy(&v, p + 4 * i, 4);
          w.put_int(i, v);
        }
        return true;
      case DT_UINT32:
        for (int64_t i = 0; i < n; ++i) {
          uint32_t v;
          std::memcpy(&v, p + 4 * i, 4);
          w.put_int(i, int64_t(v));
        }
        return true;
      case DT_INT16:
        for (int64_t i = 0; i < n; ++i) {
          int16_t v;
          std::memcpy(&v, p + 2 * i, 2);
          w.put_int(i, v);
        }
        return true;
      case DT_UINT16:
        for (int64_t i = 0; i < n; ++i) {
          uint16_t v;
          std::memcpy(&v, p + 2 * i, 2);
          w.put_int(i, v);
        }
        return true;
      case DT_INT8:
        for (int64_t i = 0; i < n; ++i) w.put_int(i, int8_t(p[i]));
        return true;
      case DT_UINT8: case DT_BOOL:
        for (int64_t i = 0; i < n; ++i) w.put_int(i, p[i]);
        return true;
      default:
        return *err = "unsupported tensor dtype", false;
    }
  }

  // Typed field path with fill semantics.
  const int64_t k = t.num_values;
  if (k > n) return *err = "more values than the tensor shape holds", false;
  if (n == 0) return true;
  if (k == 0) {  // empty typed field: zero fill
    for (int64_t i = 0; i < n; ++i) w.put_int(i, 0);
    return true;
  }
  int64_t i = 0;
  if (t.value_packed_varint) {
    if (t.dtype == DT_HALF || t.dtype == DT_BFLOAT16) {
      const bool bf = t.dtype == DT_BFLOAT16;
      bool over = false;
      if (!for_each_int(t, [&](uint64_t v) {
            const uint16_t h = uint16_t(v);
            if (i >= n) over = true;
            else if (bf && opts.dst == DstType::BF16) w.put_bits16(i++, h);
            else w.put_float(i++, bf ? bf16_to_f32(h) : half_to_f32(h));
          }))
        return *err = "bad packed varint", false;
      if (over) return *err = "more values than the tensor shape holds", false;
    } else if (t.dtype == DT_INT64 && dst_int && t.packed.size() == 1 && t.unpacked.empty()) {
      // Hot path: reference feat_ids (int64_val packed) -> row ids.
      const uint8_t* p = t.packed[0].p;
      const uint8_t* e = p + t.packed[0].n;
      while (p < e) {
        uint64_t v = *p++;
        if (v & 0x80) {
          v &= 0x7F;
          int shift = 7;
          uint8_t b;
          do {
            if (p >= e) return *err = "truncated varint", false;
            if (shift >= 70) return *err = "varint longer than 10 bytes", false;
            b = *p++;
            v |= uint64_t(b & 0x7F) << shift;
            shift += 7;
          } while (b & 0x80);
        }
        if (i >= n) return *err = "more values than the tensor shape holds", false;
        w.put_int(i++, int64_t(v));
      }
    } else {
      const int dt = t.dtype;
      bool over = false;
      if (!for_each_int(t, [&](uint64_t v) {
            if (i < n) w.put_int(i++, int_from_varint(dt, v));
            else over = true;
          }))
        return *err = "bad packed varint", false;
      if (over) return *err = "more values than the tensor shape holds", false;
    }
  } else if (t.value_fixed32) {
    if (opts.dst == DstType::F32 && t.packed.size() == 1 && t.unpacked.empty()) {
      i = std::min<int64_t>(n, int64_t(t.packed[0].n / 4));  // reference feat_wts: float_val packed
      w.copy_rows(t.packed[0].p, i);
    } else {
      for_each_f32(t, [&](float f) {
        if (i < n) w.put_float(i++, f);
      });
    }
  } else if (t.value_fixed64) {
    for_each_f64(t, [&](double d) {
      if (i < n) w.put_float(i++, float(d));
    });
  } else {
    return *err = "tensor has no typed value field for its dtype", false;
  }
  if (i < n) w.fill_from(k - 1, i, n);  // fill: repeat the last value
  return true;
}

// ---------------------------------------------------------------- encoders
namespace {

struct Out {
  std::string s;
  void byte(uint8_t b) { s.push_back(char(b)); }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      byte(uint8_t(v | 0x80));
      v >>= 7;
    }
    byte(uint8_t(v));
  }
  void tag(int field, int wt) { varint((uint64_t(field) << 3) | uint64_t(wt)); }
  void bytes(const void* p, size_t n) { s.append(static_cast<const char*>(p), n); }
  void len_field(int field, const std::string& payload) {
    tag(field, WT_LEN);
    varint(payload.size());
    s += payload;
  }
};

size_t varint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

std::string encode_spec(const ModelSpecOut& spec) {
  Out o;
  if (!spec.name.empty()) {
    o.tag(1, WT_LEN);
    o.varint(spec.name.size());
    o.bytes(spec.name.data(), spec.name.size());
  }
  if (spec.has_version) {
    Out v;
    if (spec.version != 0) {
      v.tag(1, WT_VARINT);
      v.varint(uint64_t(spec.version));
    }
    o.len_field(2, v.s);
  }
  if (!spec.signature_name.empty()) {
    o.tag(3, WT_LEN);
    o.varint(spec.signature_name.size());
    o.bytes(spec.signature_name.data(), spec.signature_name.size());
  }
  return o.s;
}

std::string encode_tensor(const TensorOut& t) {
  Out o;
  if (t.dtype != 0) {
    o.tag(1, WT_VARINT);
    o.varint(uint64_t(t.dtype));
  }
  {
    Out sh;
    for (int64_t d : t.shape) {
      Out dim;
      if (d != 0) {
        dim.tag(1, WT_VARINT);
        dim.varint(uint64_t(d));
      }
      sh.len_field(2, dim.s);
    }
    o.len_field(2, sh.s);
  }
  size_t es = dtype_size(t.dtype);
  if (t.n == 0) return o.s;
  if (t.raw) {
    o.tag(4, WT_LEN);
    o.varint(size_t(t.n) * es);
    o.bytes(t.data, size_t(t.n) * es);
    return o.s;
  }
  switch (t.dtype) {
    case DT_FLOAT:
      o.tag(5, WT_LEN);
      o.varint(size_t(t.n) * 4);
      o.bytes(t.data, size_t(t.n) * 4);
      break;
    case DT_DOUBLE:
      o.tag(6, WT_LEN);
      o.varint(size_t(t.n) * 8);
      o.bytes(t.data, size_t(t.n) * 8);
      break;
    case DT_INT64: case DT_INT32: {
      const bool i64 = t.dtype == DT_INT64;
      auto val = [&](int64_t i) -> uint64_t {
        return i64 ? uint64_t(static_cast<const int64_t*>(t.data)[i])
                   : uint64_t(int64_t(static_cast<const int32_t*>(t.data)[i]));
      };
      size_t len = 0;
      for (int64_t i = 0; i < t.n; ++i) len += varint_size(val(i));
      o.tag(i64 ? 10 : 7, WT_LEN);
      o.varint(len);
      o.s.reserve(o.s.size() + len);
      for (int64_t i = 0; i < t.n; ++i) o.varint(val(i));
      break;
    }
    default:  // everything else goes raw
      o.tag(4, WT_LEN);
      o.varint(size_t(t.n) * es);
      o.bytes(t.data, size_t(t.n) * es);
  }
  return o.s;
}

std::string encode_map_entry(const std::string& key, const std::string& value) {
  Out e;
  e.tag(1, WT_LEN);
  e.varint(key.size());
  e.bytes(key.data(), key.size());
  e.len_field(2, value);
  return e.s;
}

}  // namespace

std::string encode_predict_response(const ModelSpecOut& spec, const std::vector<TensorOut>& outputs) {
  Out o;
  for (const TensorOut& t : outputs) o.len_field(1, encode_map_entry(t.key, encode_tensor(t)));
  o.len_field(2, encode_spec(spec));
  return o.s;
}

std::string encode_predict_request(const ModelSpecOut& spec, const std::vector<TensorOut>& inputs,
                                   const std::vector<std::string>& output_filter) {
  Out o;
  o.len_field(1, encode_spec(spec));
  for (const TensorOut& t : inputs) o.len_field(2, encode_map_entry(t.key, encode_tensor(t)));
  for (const std::string& f : output_filter) {
    o.tag(3, WT_LEN);
    o.varint(f.size());
    o.bytes(f.data(), f.size());
  }
  return o.s;
}

int64_t count_varint_terminators(const uint8_t* p, size_t n) { return count_terms(p, n); }

size_t element_size(int dtype) { return dtype_size(dtype); }

}  // namespace wire
}  // namespace dtfs
