/*!
 * \file src/data/strtonum.h
 * \brief Fast, locale-free number parsing shared by the CPU parsers AND the
 *  CDNA4 HIP kernels: the same source is compiled for host and device, so
 *  the GPU CSR is bit-identical to the CPU CSR by construction.
 *
 * Arithmetic parity with reference `src/data/strtonum.h`:
 *  - strtof (:37-97): integer part accumulated in float (v*10 + d), fraction
 *    as uint64 digits / uint64 pow10 in double then added as float, exponent
 *    clamped to 38 and applied through float *1e8 / *10 loops — NOT correctly
 *    rounded; we reproduce those exact operations (no FMA contraction).
 *  - strtoint / strtouint (:104-150): base-10 accumulation; Str2T<uint32_t>
 *    accumulates in a 32-bit int (reference :184-189), reproduced with
 *    wrap-around unsigned arithmetic (same bits, no UB).
 *  - isspace / isblank / isdigit / isdigitchars (:14-31), ParsePair /
 *    ParseTriple (:228-303).
 *
 * Difference: every parser here is bounded by an explicit `end` pointer (the
 * reference's strtof could skip whitespace and read into the next token).
 */
#ifndef DMLC_DATA_STRTONUM_H_
#define DMLC_DATA_STRTONUM_H_

#include <cstdint>

#if defined(__HIPCC__)
#define DMLC_XINLINE __host__ __device__ inline
#else
#define DMLC_XINLINE inline
#endif

namespace dmlc {
namespace data {

DMLC_XINLINE bool isspace(char c) {
  return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f';
}
DMLC_XINLINE bool isblank(char c) { return c == ' ' || c == '\t'; }
DMLC_XINLINE bool iseol(char c) { return c == '\n' || c == '\r'; }
DMLC_XINLINE bool isdigit(char c) { return c >= '0' && c <= '9'; }
DMLC_XINLINE bool isdigitchars(char c) {
  return (c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.' || c == 'e' || c == 'E';
}

/*! \brief keeps a parameter out of template argument deduction */
template <typename T>
struct NonDeduced {
  typedef T type;
};

/*!
 * \brief parse a float from [p, end) with the reference arithmetic
 * \param endptr receives the first unconsumed position
 */
template <typename It>
DMLC_XINLINE float StrToFloatT(It p, It end, typename NonDeduced<It>::type* endptr) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  bool sign = true;
  if (p != end && *p == '-') {
    sign = false;
    ++p;
  } else if (p != end && *p == '+') {
    ++p;
  }
  float value = 0.0f;
  for (; p != end && isdigit(*p); ++p) {
    value = value * 10.0f + static_cast<float>(*p - '0');
  }
  if (p != end && *p == '.') {
    uint64_t pow10 = 1;
    uint64_t val2 = 0;
    ++p;
    for (; p != end && isdigit(*p); ++p) {
      val2 = val2 * 10 + static_cast<uint64_t>(*p - '0');
      pow10 *= 10;
    }
    value += static_cast<float>(static_cast<double>(val2) / static_cast<double>(pow10));
  }
  if (p != end && (*p == 'e' || *p == 'E')) {
    ++p;
    bool frac = false;
    float scale = 1.0f;
    unsigned expon = 0;
    if (p != end && *p == '-') {
      frac = true;
      ++p;
    } else if (p != end && *p == '+') {
      ++p;
    }
    for (; p != end && isdigit(*p); ++p) {
      expon = expon * 10 + static_cast<unsigned>(*p - '0');
    }
    if (expon > 38) expon = 38;
    while (expon >= 8) {
      scale = static_cast<float>(static_cast<double>(scale) * 1e8);
      expon -= 8;
    }
    while (expon > 0) {
      scale = static_cast<float>(static_cast<double>(scale) * 10.0);
      expon -= 1;
    }
    value = frac ? (value / scale) : (value * scale);
  }
  if (endptr != nullptr) *endptr = p;
  return sign ? value : -value;
}
DMLC_XINLINE float StrToFloat(const char* p, const char* end, const char** endptr) {
  return StrToFloatT<const char*>(p, end, endptr);
}

/*!
 * \brief parse an unsigned integer of type V from [p, end).
 *  A leading '-' sets *neg (the caller reports the error); '+' is accepted.
 *  Accumulation uses AccT, wrapping like the reference's 32-bit int.
 */
template <typename V, typename AccT, typename It = const char*>
DMLC_XINLINE V StrToUInt(It p, It end, typename NonDeduced<It>::type* endptr, bool* neg) {
  *neg = false;
  if (p != end && *p == '-') {
    *neg = true;
    ++p;
  } else if (p != end && *p == '+') {
    ++p;
  }
  AccT value = 0;
  for (; p != end && isdigit(*p); ++p) {
    value = value * static_cast<AccT>(10) + static_cast<AccT>(*p - '0');
  }
  if (endptr != nullptr) *endptr = p;
  return static_cast<V>(value);
}

/*! \brief signed integer from [p, end) (two's-complement wrap on overflow) */
template <typename V, typename It = const char*>
DMLC_XINLINE V StrToInt(It p, It end, typename NonDeduced<It>::type* endptr) {
  bool sign = true;
  if (p != end && *p == '-') {
    sign = false;
    ++p;
  } else if (p != end && *p == '+') {
    ++p;
  }
  uint64_t value = 0;
  for (; p != end && isdigit(*p); ++p) value = value * 10u + static_cast<uint64_t>(*p - '0');
  if (endptr != nullptr) *endptr = p;
  return static_cast<V>(sign ? value : (~value + 1u));
}

/*! \brief type-directed conversion of a digitchars run [begin, end) */
template <typename T>
struct Str2T;
template <>
struct Str2T<float> {
  template <typename It>
  DMLC_XINLINE static float get(It b, It e, bool* bad) {
    *bad = false;
    return StrToFloatT<It>(b, e, nullptr);
  }
};
template <>
struct Str2T<uint32_t> {
  // reference: strtouint<int> -> 32-bit accumulation
  template <typename It>
  DMLC_XINLINE static uint32_t get(It b, It e, bool* bad) {
    return StrToUInt<uint32_t, uint32_t, It>(b, e, nullptr, bad);
  }
};
template <>
struct Str2T<uint64_t> {
  template <typename It>
  DMLC_XINLINE static uint64_t get(It b, It e, bool* bad) {
    return StrToUInt<uint64_t, uint64_t, It>(b, e, nullptr, bad);
  }
};
template <>
struct Str2T<int32_t> {
  template <typename It>
  DMLC_XINLINE static int32_t get(It b, It e, bool* bad) {
    *bad = false;
    return StrToInt<int32_t, It>(b, e, nullptr);
  }
};
template <>
struct Str2T<int64_t> {
  template <typename It>
  DMLC_XINLINE static int64_t get(It b, It e, bool* bad) {
    *bad = false;
    return StrToInt<int64_t, It>(b, e, nullptr);
  }
};

/*!
 * \brief parse `v1[:v2]` inside [begin, end) (one token).
 * \return number of values parsed (0 when the token has no digitchar);
 *  *bad is set when an unsigned field had a minus sign
 */
template <typename T1, typename T2, typename It = const char*>
DMLC_XINLINE int ParsePair(It begin, It end, T1* v1, T2* v2, bool* bad) {
  *bad = false;
  It p = begin;
  while (p != end && !isdigitchars(*p)) ++p;
  if (p == end) return 0;
  It q = p;
  while (q != end && isdigitchars(*q)) ++q;
  bool b1 = false;
  *v1 = Str2T<T1>::get(p, q, &b1);
  p = q;
  while (p != end && isblank(*p)) ++p;
  if (p == end || *p != ':') {
    *bad = b1;
    return 1;
  }
  ++p;
  while (p != end && !isdigitchars(*p)) ++p;
  q = p;
  while (q != end && isdigitchars(*q)) ++q;
  bool b2 = false;
  *v2 = Str2T<T2>::get(p, q, &b2);
  *bad = b1 || b2;
  return 2;
}

/*! \brief parse `v1:v2[:v3]` inside [begin, end) (one LibFM token) */
template <typename T1, typename T2, typename T3, typename It = const char*>
DMLC_XINLINE int ParseTriple(It begin, It end, T1* v1, T2* v2, T3* v3, bool* bad) {
  *bad = false;
  It p = begin;
  while (p != end && !isdigitchars(*p)) ++p;
  if (p == end) return 0;
  It q = p;
  while (q != end && isdigitchars(*q)) ++q;
  bool b1 = false, b2 = false, b3 = false;
  *v1 = Str2T<T1>::get(p, q, &b1);
  p = q;
  while (p != end && isblank(*p)) ++p;
  if (p == end || *p != ':') {
    *bad = b1;
    return 1;
  }
  ++p;
  while (p != end && !isdigitchars(*p)) ++p;
  q = p;
  while (q != end && isdigitchars(*q)) ++q;
  *v2 = Str2T<T2>::get(p, q, &b2);
  p = q;
  while (p != end && isblank(*p)) ++p;
  if (p == end || *p != ':') {
    *bad = b1 || b2;
    return 2;
  }
  ++p;
  while (p != end && !isdigitchars(*p)) ++p;
  q = p;
  while (q != end && isdigitchars(*q)) ++q;
  *v3 = Str2T<T3>::get(p, q, &b3);
  *bad = b1 || b2 || b3;
  return 3;
}

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_STRTONUM_H_
