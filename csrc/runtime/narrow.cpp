#include "narrow.h"

#include <immintrin.h>

#include <cstring>

namespace dtfs {
namespace runtime {

namespace {

inline int32_t mod_scalar(int64_t v, int64_t m) {
  int64_t r = v % m;
  if (r < 0) r += m;
  return int32_t(r);
}

void narrow_ids_scalar(const uint8_t* src, int32_t* dst, int64_t n, int64_t m) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t v;
    std::memcpy(&v, src + 8 * i, 8);
    dst[i] = mod_scalar(v, m);
  }
}

// 4 ids per iteration. For 0 <= v < 2^52: d = double(v) exactly (magic-number
// conversion), q = floor(d / m) is the quotient or one off, r = v - q*m is
// corrected into [0, m) with one compare each way. Lanes outside that range
// (negative or huge ids) are redone in scalar code.
__attribute__((target("avx2,fma"))) void narrow_ids_avx2(const uint8_t* src, int32_t* dst, int64_t n, int64_t m) {
  const __m256i magic_i = _mm256_set1_epi64x(0x4330000000000000LL);
  const __m256d magic_d = _mm256_set1_pd(4503599627370496.0);  // 2^52
  const __m256d inv_m = _mm256_set1_pd(1.0 / double(m));
  const __m256i mv = _mm256_set1_epi64x(m);
  const __m256i lim = _mm256_set1_epi64x((1LL << 52) - 1);
  const __m256i zero = _mm256_setzero_si256();
  const __m256i pick = _mm256_setr_epi32(0, 2, 4, 6, 0, 2, 4, 6);
  int64_t i = 0;
  for (; i + 4 <= n; i += 4) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + 8 * i));
    // range check: 0 <= v <= 2^52 - 1
    const __m256i bad = _mm256_or_si256(_mm256_cmpgt_epi64(zero, v), _mm256_cmpgt_epi64(v, lim));
    const __m256d d = _mm256_sub_pd(_mm256_castsi256_pd(_mm256_or_si256(v, magic_i)), magic_d);
    const __m256d qd = _mm256_floor_pd(_mm256_mul_pd(d, inv_m));
    // q (< 2^52) back to integer bits the same way
    const __m256i q = _mm256_sub_epi64(_mm256_castpd_si256(_mm256_add_pd(qd, magic_d)), magic_i);
    // q * m with 32x32->64 products: q = qh * 2^32 + ql, m < 2^31
    const __m256i lo = _mm256_mul_epu32(q, mv);
    const __m256i hi = _mm256_slli_epi64(_mm256_mul_epu32(_mm256_srli_epi64(q, 32), mv), 32);
    __m256i r = _mm256_sub_epi64(v, _mm256_add_epi64(lo, hi));
    r = _mm256_add_epi64(r, _mm256_and_si256(_mm256_cmpgt_epi64(zero, r), mv));                     // r < 0: += m
    r = _mm256_sub_epi64(r, _mm256_andnot_si256(_mm256_cmpgt_epi64(mv, r), mv));                     // r >= m: -= m
    const __m128i r32 = _mm256_castsi256_si128(_mm256_permutevar8x32_epi32(r, pick));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i), r32);
    if (!_mm256_testz_si256(bad, bad)) {
      for (int k = 0; k < 4; ++k) {
        int64_t x;
        std::memcpy(&x, src + 8 * (i + k), 8);
        dst[i + k] = mod_scalar(x, m);
      }
    }
  }
  narrow_ids_scalar(src + 8 * i, dst + i, n - i, m);
}

const bool g_avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");

// int32 rows (< 2^24) -> 3 bytes each: per 128-bit lane the low 3 bytes of its
// 4 rows shuffled to the front (12 bytes), each lane stored as 16 bytes at a
// 12-byte stride (the next store overwrites the 4 bytes of junk)
__attribute__((target("avx2"))) void pack24_avx2(const int32_t* rows, uint8_t* dst, int64_t n) {
  const __m256i shuf = _mm256_setr_epi8(0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -1, -1, -1, -1,
                                        0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -1, -1, -1, -1);
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    const __m256i v = _mm256_shuffle_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(rows + i)), shuf);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + 3 * i), _mm256_castsi256_si128(v));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + 3 * i + 12), _mm256_extracti128_si256(v, 1));
  }
  for (; i < n; ++i) {
    const uint32_t r = uint32_t(rows[i]);
    dst[3 * i] = uint8_t(r);
    dst[3 * i + 1] = uint8_t(r >> 8);
    dst[3 * i + 2] = uint8_t(r >> 16);
  }
}

}  // namespace

int classify_weights(const uint8_t* src, int64_t rows, int64_t fields, int64_t wcols) {
  bool ones = true, bf16 = true;
  for (int64_t r = 0; r < rows && (ones || bf16); ++r) {
    const uint8_t* p = src + 4 * r * fields;
    uint32_t all = 0, low = 0;
    for (int64_t c = 0; c < wcols; ++c) {
      uint32_t v;
      std::memcpy(&v, p + 4 * c, 4);
      all |= v ^ 0x3f800000u;  // 1.0f
      low |= v & 0xffffu;
    }
    ones = ones && all == 0;
    bf16 = bf16 && low == 0;
  }
  return ones ? kWtsOnes : bf16 ? kWtsBf16 : kWtsF32;
}

void store_weights(const uint8_t* src, int64_t rows, int64_t fields, int64_t wcols, int kind, uint8_t* dst) {
  if (kind == kWtsOnes) return;
  if (kind == kWtsF32) {
    if (wcols == fields) {
      std::memcpy(dst, src, size_t(4 * rows * fields));
    } else {
      for (int64_t r = 0; r < rows; ++r) std::memcpy(dst + 4 * r * wcols, src + 4 * r * fields, size_t(4 * wcols));
    }
    return;
  }
  uint16_t* d = reinterpret_cast<uint16_t*>(dst);  // bf16: the high half of each (exact) fp32
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t c = 0; c < wcols; ++c) {
      uint32_t v;
      std::memcpy(&v, src + 4 * (r * fields + c), 4);
      d[r * wcols + c] = uint16_t(v >> 16);
    }
}

void narrow_ids(const uint8_t* src, int32_t* dst, int64_t n, int64_t modulo) {
  if (g_avx2) narrow_ids_avx2(src, dst, n, modulo);
  else narrow_ids_scalar(src, dst, n, modulo);
}

void narrow_ids24(const uint8_t* src, uint8_t* dst, int64_t n, int64_t modulo) {
  // in blocks that stay in L1: narrow to int32, then pack
  constexpr int64_t kBlock = 2048;
  alignas(32) int32_t tmp[kBlock];
  for (int64_t i = 0; i < n; i += kBlock) {
    const int64_t m = n - i < kBlock ? n - i : kBlock;
    narrow_ids(src + 8 * i, tmp, m, modulo);
    if (g_avx2) {
      pack24_avx2(tmp, dst + 3 * i, m);
    } else {
      for (int64_t k = 0; k < m; ++k) {
        const uint32_t r = uint32_t(tmp[k]);
        dst[3 * (i + k)] = uint8_t(r);
        dst[3 * (i + k) + 1] = uint8_t(r >> 8);
        dst[3 * (i + k) + 2] = uint8_t(r >> 16);
      }
    }
  }
}

}  // namespace runtime
}  // namespace dtfs
