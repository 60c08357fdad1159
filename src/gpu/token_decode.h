/*!
 * \file src/gpu/token_decode.h
 * \brief Register-window decoding of one LibSVM / LibFM token on gfx950 (the
 *  fast path of the tile fill kernel, src/gpu/tile_kernels.hip).
 *
 *  A token's bytes are read from the LDS-staged text 16 at a time: two
 *  16-byte-aligned ds_read_b128 cover any 16-byte window, which is then
 *  funnel-shifted into place with v_alignbyte (ext16).  Lanes of a wave take
 *  consecutive tokens (about 16 B apart), so the four 16-lane groups of a
 *  ds_read_b128 read nearly disjoint bank quads -- the unaligned dword reads
 *  of the round-2 kernel were 4-way conflicted at that stride.
 *  Digit runs are decoded 4 bytes at a time (SWAR, lead_digits); every
 *  number takes one window, a value's fraction digits come out of the same
 *  window when they fit.
 *
 *  Arithmetic parity with src/data/strtonum.h (reference src/data/strtonum.h:
 *  37-97): an integer part of <= 7 digits accumulated in float is exact, so it
 *  equals the integer converted once; the fraction float(double(F) /
 *  double(10^k)) equals the correctly rounded float quotient F / 10^k for
 *  k <= 8 (the quotient's distance to a float rounding boundary exceeds the
 *  double rounding error), and for k <= 7 (F < 2^24, exact in float) that
 *  quotient is q0 = F * r, q1 = fma(F - q0 * 10^k, r, q0) with r = RN(1 / 10^k)
 *  -- checked exhaustively for every F < 10^k, k = 1..7.  Shapes outside the
 *  fast path (exponents, > 7 integer or fraction digits, over-long indices,
 *  signs on indices, tokens longer than the windows) return false and take
 *  the generic ParsePair / ParseTriple.
 */
#ifndef DMLC_SRC_GPU_TOKEN_DECODE_H_
#define DMLC_SRC_GPU_TOKEN_DECODE_H_

#include <hip/hip_runtime.h>

#include <cstdint>

#include "./kernels.h"

namespace dmlc {
namespace gpu {
namespace tok {

/*! \brief 16 bytes starting at byte `a` of a 16-byte-aligned LDS buffer
 *  (the buffer must hold 32 bytes from a & ~15): the five dwords covering
 *  them, read one by one, funnel-shifted into place.  LDS issue is cheap in
 *  the (VALU-bound) decode rounds; two aligned ds_read_b128 plus the 15
 *  selects of the dword window cost more VALU issue. */
__device__ __forceinline__ uint4 ext16(const uint4* lds, uint32_t a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds) + (a >> 2);
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  const uint32_t r = a & 3u;
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
                    __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r));
}

/*! \brief 10^k for k = 0..7 from its bits: three selects, two 24-bit multiplies */
__device__ __forceinline__ uint32_t pow10_u(uint32_t k) {
  const uint32_t a = (k & 1u) ? 10u : 1u;
  const uint32_t b = (k & 2u) ? 100u : 1u;
  const uint32_t c = (k & 4u) ? 10000u : 1u;
  return __umul24(__umul24(a, b), c);
}

/*!
 * \brief SWAR: number of leading ASCII digits (0..4) of the 4 bytes g (first
 *  byte = lowest) and their decimal value.
 */
__device__ __forceinline__ uint32_t lead_digits(uint32_t g, uint32_t* val) {
  const uint32_t lo4 = g & 0x0F0F0F0Fu;
  const uint32_t hi = (g & 0xF0F0F0F0u) ^ 0x30303030u;        // high nibble != 3
  const uint32_t lo = (lo4 + 0x06060606u) & 0x10101010u;      // low nibble > 9
  const uint32_t bad = hi | (lo << 3);
  // no non-digit byte: 4 digits
  const uint32_t k = static_cast<uint32_t>(__builtin_ctzg(bad, 32)) >> 3;
  // k digits right-aligned (a 64-bit shift: k = 0 shifts them all out)
  const uint32_t x = static_cast<uint32_t>((static_cast<uint64_t>(lo4) << (8u * (4u - k))));
  // digit pairs by byte dot products (v_dot4_u32_u8), then pair0 * 100 + pair1
  const uint32_t p0 = __builtin_amdgcn_udot4(x, 0x0000010Au, 0u, false);
  const uint32_t p1 = __builtin_amdgcn_udot4(x, 0x010A0000u, 0u, false);
  *val = __umul24(p0, 100u) + p1;
  return k;
}

/*!
 * \brief the value and digit count of a run split in two 4-byte groups:
 *  (k0, v0) the first group's lead_digits, (k1, v1) the second's, which
 *  counts only when the first is full.  The empty asm pins the second group
 *  as computed: left alone, hipcc sinks it into an exec-masked branch (an
 *  s_and_saveexec / s_cbranch_execz / exec restore per number, and no
 *  interleaving of independent numbers across it).  Both factors are below
 *  2^24: a full-rate v_mul_u32_u24, not the quarter-rate v_mul_lo_u32.
 */
__device__ __forceinline__ uint32_t join_groups(uint32_t k0, uint32_t v0, uint32_t k1, uint32_t v1,
                                                uint32_t* k) {
  // (an explicit v_mul_u32_u24: from __umul24 of operands it can bound,
  // hipcc emits the quarter-rate v_mul_lo_u32)
  uint32_t x;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(x) : "v"(v0), "v"(pow10_u(k1)));
  x += v1;
  asm("" : "+v"(x));
  const bool full = k0 == 4;
  *k = full ? 4u + k1 : k0;
  return full ? x : v0;
}

/*!
 * \brief RN(1 / 10^k) and 10^k in float, k = 0..7: a three-level select on
 *  the bits of k.  Each level is pinned by an empty asm -- written as a
 *  plain ternary chain, hipcc lowers the lookup to nested exec-masked
 *  branches (s_and_saveexec / s_xor / s_cbranch per level, every number).
 */
__device__ __forceinline__ void pow10f(uint32_t k, float* p, float* inv) {
  *p = static_cast<float>(pow10_u(k));
  const bool b0 = (k & 1u) != 0, b1 = (k & 2u) != 0, b2 = (k & 4u) != 0;
  float a0 = b0 ? 0.1f : 1.0f, a1 = b0 ? 0.001f : 0.01f;
  float a2 = b0 ? 1e-5f : 1e-4f, a3 = b0 ? 1e-7f : 1e-6f;
  asm("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
  float c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2;
  asm("" : "+v"(c0), "+v"(c1));
  *inv = b2 ? c1 : c0;
}

/*!
 * \brief 12 bytes starting at byte `a` of a 16-byte-aligned LDS buffer (four
 *  dwords read, three funnel shifts): enough for a sign, 8 digits and the
 *  byte after them
 */
__device__ __forceinline__ uint3 ext12(const uint4* lds, uint32_t a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds) + (a >> 2);
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
  const uint32_t r = a & 3u;
  return make_uint3(__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
                    __builtin_amdgcn_alignbyte(w3, w2, r));
}

/*!
 * \brief the leading decimal digits of the 8 bytes lo | hi (first byte
 *  lowest), all 8 at once: k = their count (0..8; 8 = all eight, more may
 *  follow), val = the value of those k digits (< 10^8), term = the byte after
 *  them (`next` = byte 8 when k is 8).
 *
 *  A byte is a digit iff (byte ^ '0') < 10: after the xor the digit bytes hold
 *  their values, and the high bit of ((t & 0x7F) + 0x76) | t marks every other
 *  byte (no carries between bytes).  The first such byte gives k; the k digits
 *  are right-aligned in 64 bits by a shift of 64 - 8 k (two halves, so k = 0
 *  and k = 8 need no select); byte dot products give the four digit pairs and
 *  three 24-bit multiply-adds join them.  About 25 VALU for up to 8 digits,
 *  where two 4-digit groups and their join took about 45.
 */
struct Run8 {
  uint32_t k, val, term;
};

__device__ __forceinline__ Run8 digit_run8(uint32_t lo, uint32_t hi, uint32_t next) {
  const uint32_t t0 = lo ^ 0x30303030u, t1 = hi ^ 0x30303030u;
  const uint32_t b0 = (((t0 & 0x7F7F7F7Fu) + 0x76767676u) | t0) & 0x80808080u;
  const uint32_t b1 = (((t1 & 0x7F7F7F7Fu) + 0x76767676u) | t1) & 0x80808080u;
  const uint64_t bad = (static_cast<uint64_t>(b1) << 32) | b0;
  // 8 k: the first non-digit's bit is 8 k + 7 (64 when all 8 are digits)
  const uint32_t c8 = static_cast<uint32_t>(__builtin_ctzg(bad, 64)) & ~7u;
  const uint32_t half = 32u - (c8 >> 1);  // (64 - 8 k) / 2
  const uint64_t t = (static_cast<uint64_t>(t1) << 32) | t0;
  const uint64_t x = (t << half) << half;
  const uint32_t xl = static_cast<uint32_t>(x), xh = static_cast<uint32_t>(x >> 32);
  const uint32_t p0 = __builtin_amdgcn_udot4(xl, 0x0000010Au, 0u, false);
  const uint32_t p1 = __builtin_amdgcn_udot4(xl, 0x010A0000u, 0u, false);
  const uint32_t p2 = __builtin_amdgcn_udot4(xh, 0x0000010Au, 0u, false);
  const uint32_t p3 = __builtin_amdgcn_udot4(xh, 0x010A0000u, 0u, false);
  // (explicit 24-bit multiply-adds: every partial value is < 10^6 < 2^24)
  // (no inline asm here: the compiler must see the dot products' consumers
  // to place the wait states a DOT result needs before a VALU reads it)
  // (every partial value is < 10^6 < 2^24; the compiler picks the multiply-add)
  const uint32_t v = __umul24(__umul24(__umul24(p0, 100u) + p1, 100u) + p2, 100u) + p3;
  Run8 r;
  r.k = c8 >> 3;
  r.val = v;
  const uint64_t raw = (static_cast<uint64_t>(hi) << 32) | lo;
  r.term = c8 < 64 ? static_cast<uint32_t>(raw >> c8) & 0xFFu : next;
  return r;
}

/*! \brief separator bytes and the zero padding: ' ' \t \n \r NUL, one 64-bit
 *  shift of a bit set instead of five compares */
__device__ __forceinline__ bool is_end(uint32_t c) {
  return c <= 32u && ((0x100002601ull >> c) & 1u) != 0;
}

/*!
 * \brief one number `[+-] digits [. digits]` at LDS byte a, decoded without
 *  branches (every lane of a wave runs the same instructions; the caller
 *  selects what it needs):
 *   ival  the integer digits (valid as an index when ok_uint)
 *   fval  the reference StrToFloat value (valid when ok_float)
 *   end / term  the byte after the number and its LDS offset
 */
struct Num {
  uint32_t ival;
  float fval;
  uint32_t end, term;
  bool ok_float, ok_uint;
};

__device__ __forceinline__ Num parse_num_g(uint4 g, uint32_t a);

/*!
 * \brief parse_num on LDS: the integer digits from a 12-byte window at the
 *  number, the fraction from a second one at the byte after the '.' (read
 *  unconditionally: branch-free), each decoded by digit_run8.  The same
 *  values and flags as parse_num_g on every number whose fraction fits its
 *  16-byte window; a longer fraction (<= 7 digits) is taken here as well.
 *  Two extensions run only when some lane of the wave needs them (wave-
 *  uniform branches: free on plain `0.dddddd` data), with parse_num_ext's
 *  arithmetic, so the values are the same bits: fractions of 8 to 15 digits
 *  (a second digit run, the reference's double quotient) and exponents of up
 *  to 3 digits with |e| <= 10 (10^e exact in float, one IEEE multiply or
 *  divide).  Other exponents stay not-ok (the queued extended decoder).
 */
__device__ __forceinline__ Num parse_num(const uint4* lds, uint32_t a) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  Num o;
  const uint3 g = ext12(lds, a);
  const uint32_t c0 = g.x & 0xFFu;
  const bool neg = c0 == '-';
  const uint32_t s = (neg || c0 == '+') ? 1u : 0u;
  const uint32_t h0 = __builtin_amdgcn_alignbyte(g.y, g.x, s);
  const uint32_t h1 = __builtin_amdgcn_alignbyte(g.z, g.y, s);
  const uint32_t nb = (__builtin_amdgcn_alignbyte(g.z, g.y, s + 1u) >> 24);  // byte 8 after the sign
  const Run8 ir = digit_run8(h0, h1, nb);
  const uint32_t k = ir.k;
  const bool dot = ir.term == '.';
  const uint32_t fa = a + s + k + 1u;
  const uint3 f = ext12(lds, fa);
  const Run8 fr = digit_run8(f.x, f.y, f.z & 0xFFu);
  uint32_t nf = fr.k;
  o.ok_float = (k <= 7) & (dot ? ((nf <= 7) & ((k | nf) != 0)) : k != 0);
  o.ok_uint = (s == 0) & !dot & (k != 0) & !((k == 8) & (ir.term - '0' < 10u));
  o.term = dot ? fr.term : ir.term;
  o.end = dot ? fa + nf : a + s + k;
  o.ival = ir.val;
  // StrToFloat: float(int digits) + float(F / 10^nf) (see file comment)
  float p, inv;
  pow10f(nf, &p, &inv);
  const float ff = static_cast<float>(fr.val);
  const float q0 = ff * inv;
  const float rem = __builtin_fmaf(-q0, p, ff);
  float frac = __builtin_fmaf(rem, inv, q0);
  const bool longf = dot & (nf == 8u);
  if (__any(longf)) {
    // 8 fraction digits read: up to 8 more from the window after them
    const uint3 f2 = ext12(lds, fa + 8u);
    const Run8 r2 = digit_run8(f2.x, f2.y, f2.z & 0xFFu);
    if (longf) {
      nf = 8u + r2.k;
      const uint64_t fv = static_cast<uint64_t>(fr.val) * pow10_u(r2.k) + r2.val;
      frac = static_cast<float>(static_cast<double>(fv) /
                                (1e8 * static_cast<double>(pow10_u(r2.k))));
      o.ok_float = (k <= 7) & (nf < 16u);
      o.term = r2.term;
      o.end = fa + nf;
    }
  }
  float v = static_cast<float>(ir.val);
  v = dot ? v + frac : v;
  const bool has_e = (o.term == 'e') | (o.term == 'E');
  if (__any(has_e & o.ok_float)) {
    const uint3 e = ext12(lds, o.end + 1u);
    const uint32_t cs = e.x & 0xFFu;
    const bool eneg = cs == '-';
    const uint32_t es = (cs == '-' || cs == '+') ? 1u : 0u;
    const Run8 er = digit_run8(__builtin_amdgcn_alignbyte(e.y, e.x, es),
                               __builtin_amdgcn_alignbyte(e.z, e.y, es), 0u);
    const uint32_t ex = er.val;
    if (has_e) {
      const float scale = ex <= 7u ? static_cast<float>(pow10_u(ex))
                                   : (ex == 8u ? 1e8f : (ex == 9u ? 1e9f : 1e10f));
      o.ok_float = o.ok_float & (er.k < 4u) & (ex <= 10u);
      o.end = o.end + 1u + es + er.k;
      o.term = er.term;
      v = eneg ? (v / scale) : (v * scale);
    }
  }
  o.fval = neg ? -v : v;
  return o;
}

/*! \brief parse_num on the 16 bytes g already read from LDS byte a */
__device__ __forceinline__ Num parse_num_g(uint4 g, uint32_t a) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  Num o;
  const uint32_t c0 = g.x & 0xFFu;
  const bool neg = c0 == '-';
  const uint32_t s = (neg || c0 == '+') ? 1u : 0u;
  const uint32_t h0 = __builtin_amdgcn_alignbyte(g.y, g.x, s);
  const uint32_t h1 = __builtin_amdgcn_alignbyte(g.z, g.y, s);
  const uint32_t h2 = __builtin_amdgcn_alignbyte(g.w, g.z, s);
  const uint32_t h3 = g.w >> (8u * s);
  // integer digits (<= 8) and the byte after them
  uint32_t v0, v1;
  const uint32_t k0 = lead_digits(h0, &v0);
  const uint32_t k1 = lead_digits(h1, &v1);
  uint32_t k;
  const uint32_t iv = join_groups(k0, v0, k1, v1, &k);
  const uint32_t tw = k < 4 ? h0 : (k < 8 ? h1 : h2);
  const uint32_t term = (tw >> (8u * (k & 3u))) & 0xFFu;
  // fraction digits: 8 bytes at fs = k + 1 (1..9) of h0..h3
  const uint32_t fs = k + 1u;
  const uint32_t q = fs >> 2, r = fs & 3u;
  const uint32_t a0 = q == 0 ? h0 : (q == 1 ? h1 : h2);
  const uint32_t a1 = q == 0 ? h1 : (q == 1 ? h2 : h3);
  const uint32_t a2 = q == 0 ? h2 : (q == 1 ? h3 : 0u);
  const uint32_t lo = __builtin_amdgcn_alignbyte(a1, a0, r);
  const uint32_t hi = __builtin_amdgcn_alignbyte(a2, a1, r);
  uint32_t w0, w1;
  const uint32_t f0 = lead_digits(lo, &w0);
  const uint32_t f1 = lead_digits(hi, &w1);
  uint32_t nf;
  const uint32_t fv = join_groups(f0, w0, f1, w1, &nf);
  const uint32_t fw = nf < 4 ? lo : hi;
  const uint32_t fterm = nf < 8 ? (fw >> (8u * (nf & 3u))) & 0xFFu : 0x30u;
  const bool dot = term == '.';
  // the fraction and its terminator must lie inside the 16 - s window bytes
  const bool frac_ok = (nf <= 7) & (fs + nf < 16u - s) & ((k | nf) != 0);
  o.ok_float = (k <= 7) & (dot ? frac_ok : k != 0);
  o.ok_uint = (s == 0) & !dot & (k != 0) & !((k == 8) & ((h2 & 0xFFu) - '0' < 10u));
  o.term = dot ? fterm : term;
  o.end = a + s + k + (dot ? 1u + nf : 0u);
  o.ival = iv;
  // StrToFloat: float(int digits) + float(F / 10^nf) (see file comment)
  float p, inv;
  pow10f(nf, &p, &inv);
  const float ff = static_cast<float>(fv);
  const float q0 = ff * inv;
  const float rem = __builtin_fmaf(-q0, p, ff);
  const float frac = __builtin_fmaf(rem, inv, q0);
  float v = static_cast<float>(iv);
  v = dot ? v + frac : v;
  o.fval = neg ? -v : v;
  return o;
}

/*!
 * \brief the integer head of a number: `[+-] digits` at LDS byte a -- the
 *  first half of parse_num, for fields that are indices (no fraction decode,
 *  about 60 % of parse_num's instructions).  Equal to parse_num whenever the
 *  digits are not followed by '.'; with a '.' (term == '.') ok_float and
 *  ok_uint are false and the caller re-decodes with parse_num.
 */
__device__ __forceinline__ Num parse_int(const uint4* lds, uint32_t a) {
  Num o;
  const uint3 g = ext12(lds, a);
  const uint32_t c0 = g.x & 0xFFu;
  const bool neg = c0 == '-';
  const uint32_t s = (neg || c0 == '+') ? 1u : 0u;
  const uint32_t h0 = __builtin_amdgcn_alignbyte(g.y, g.x, s);
  const uint32_t h1 = __builtin_amdgcn_alignbyte(g.z, g.y, s);
  const uint32_t nb = (__builtin_amdgcn_alignbyte(g.z, g.y, s + 1u) >> 24);
  const Run8 ir = digit_run8(h0, h1, nb);
  const uint32_t k = ir.k;
  const bool dot = ir.term == '.';
  o.ok_float = (k <= 7) & (k != 0) & !dot;
  o.ok_uint = (s == 0) & !dot & (k != 0) & !((k == 8) & (ir.term - '0' < 10u));
  o.term = ir.term;
  o.end = a + s + k;
  o.ival = ir.val;
  const float v = static_cast<float>(ir.val);
  o.fval = neg ? -v : v;
  return o;
}


/*! \brief fast-path result of one token */
struct Token {
  uint32_t u0, u1;        // LibSVM index / LibFM field, LibFM index
  uint32_t u0_hi, u1_hi;  // high words (generic path, 64-bit indices)
  float f0, f1;           // label & weight, or the feature value
  int r;                  // values parsed (ParsePair / ParseTriple convention)
};

/*! \brief the token shape from its decoded numbers (decode's last stage):
 *  n1 the first number, n2 the one after its ':' (if any), n3 the one after
 *  n2's ':' (LibFM) */
template <TextFormat F>
__device__ __forceinline__ bool assemble(const Num& n1, const Num& n2, const Num& n3,
                                         bool is_label, Token* t) {
  const bool c1 = n1.term == ':';
  // label f[:f] (either format) or LibSVM feature u[:f]
  const bool first = is_label ? n1.ok_float : n1.ok_uint;
  const bool pair_ok = first & (c1 ? (n2.ok_float & is_end(n2.term)) : is_end(n1.term));
  t->u0 = n1.ival;
  t->f1 = n2.fval;
  if (F == TextFormat::kLibSVM) {
    t->f0 = is_label ? n1.fval : n2.fval;
    t->r = c1 ? 2 : 1;
    return pair_ok;
  }
  // LibFM feature field:index[:value]
  const bool c2 = n2.term == ':';
  const bool triple_ok =
      c1 & n1.ok_uint & n2.ok_uint & (c2 ? (n3.ok_float & is_end(n3.term)) : is_end(n2.term));
  t->u1 = n2.ival;
  t->f0 = is_label ? n1.fval : n3.fval;
  t->r = is_label ? (c1 ? 2 : 1) : (c2 ? 3 : 2);
  return is_label ? pair_ok : triple_ok;
}

/*!
 * \brief decode a label `f[:f]`, LibSVM feature `u[:f]` or LibFM feature
 *  `u:u[:f]` starting at LDS byte a, branch-free: the numbers are decoded
 *  unconditionally (the next one from wherever the previous ended) and the
 *  token shape is selected afterwards.  false: the generic parser is needed.
 *  Integer fields (indices, LibFM fields, integer labels) use parse_int.
 */
template <TextFormat F>
__device__ __forceinline__ bool decode(const uint4* lds, uint32_t a, bool is_label, Token* t) {
  // indices take the integer-only decoder; a label with a fraction (any lane
  // of the wave: the branch is wave-uniform) takes the full one
  Num n1 = parse_int(lds, a);
  if (__any(is_label & (n1.term == '.'))) n1 = parse_num(lds, a);
  const bool c1 = n1.term == ':';
  Num n2, n3;
  if (F == TextFormat::kLibSVM) {
    n2 = parse_num(lds, n1.end + (c1 ? 1u : 0u));  // the value (or the label's weight)
    n3 = n2;
  } else {
    // LibFM: the index, or the label's weight
    n2 = parse_int(lds, n1.end + (c1 ? 1u : 0u));
    if (__any(is_label & c1 & (n2.term == '.'))) n2 = parse_num(lds, n1.end + (c1 ? 1u : 0u));
    const bool c2 = n2.term == ':';
    n3 = parse_num(lds, n2.end + (c2 ? 1u : 0u));
  }
  return assemble<F>(n1, n2, n3, is_label, t);
}

/*!
 * \brief decode() of two tokens per lane (a decode "pair round": lanes take
 *  token i and token i + 64 of the list).  The same instructions as two
 *  decode() calls, but the two tokens' LDS window reads and number decodes
 *  are independent chains inside the same basic blocks -- the wave-uniform
 *  label-fraction branches are shared -- so the compiler interleaves them and
 *  each LDS round trip is paid once per pair.  Identical results.
 */
template <TextFormat F>
__device__ __forceinline__ void decode2(const uint4* lds, uint32_t a0, uint32_t a1, bool lab0,
                                        bool lab1, Token* t0, Token* t1, bool* ok0, bool* ok1) {
  Num n1a = parse_int(lds, a0);
  Num n1b = parse_int(lds, a1);
  if (__any((lab0 & (n1a.term == '.')) | (lab1 & (n1b.term == '.')))) {
    // (parse_num equals parse_int on tokens without a fraction)
    n1a = parse_num(lds, a0);
    n1b = parse_num(lds, a1);
  }
  const uint32_t s2a = n1a.end + (n1a.term == ':' ? 1u : 0u);
  const uint32_t s2b = n1b.end + (n1b.term == ':' ? 1u : 0u);
  Num n2a, n2b, n3a, n3b;
  if (F == TextFormat::kLibSVM) {
    n2a = parse_num(lds, s2a);
    n2b = parse_num(lds, s2b);
    n3a = n2a;
    n3b = n2b;
  } else {
    n2a = parse_int(lds, s2a);
    n2b = parse_int(lds, s2b);
    if (__any((lab0 & (n1a.term == ':') & (n2a.term == '.')) |
              (lab1 & (n1b.term == ':') & (n2b.term == '.')))) {
      n2a = parse_num(lds, s2a);
      n2b = parse_num(lds, s2b);
    }
    n3a = parse_num(lds, n2a.end + (n2a.term == ':' ? 1u : 0u));
    n3b = parse_num(lds, n2b.end + (n2b.term == ':' ? 1u : 0u));
  }
  *ok0 = assemble<F>(n1a, n2a, n3a, lab0, t0);
  *ok1 = assemble<F>(n1b, n2b, n3b, lab1, t1);
}

/*! \brief the dword starting at byte 4q (q <= 7) of a 32-byte window g0|g1 */
__device__ __forceinline__ uint32_t win_dw(uint4 g0, uint4 g1, uint32_t q) {
  return q < 4 ? (q < 2 ? (q == 0 ? g0.x : g0.y) : (q == 2 ? g0.z : g0.w))
               : (q < 6 ? (q == 4 ? g1.x : g1.y) : (q == 6 ? g1.z : g1.w));
}

/*! \brief byte i (0..31) of the window (i lane-varying) */
__device__ __forceinline__ uint32_t win_byte(uint4 g0, uint4 g1, uint32_t i) {
  return (win_dw(g0, g1, i >> 2) >> (8u * (i & 3u))) & 0xFFu;
}

/*! \brief the 4 bytes starting at byte i (i <= 28) of the window */
__device__ __forceinline__ uint32_t win_word(uint4 g0, uint4 g1, uint32_t i) {
  const uint32_t q = i >> 2;
  return __builtin_amdgcn_alignbyte(win_dw(g0, g1, q < 7 ? q + 1 : 7u), win_dw(g0, g1, q), i & 3u);
}

/*!
 * \brief a float in the full reference grammar (strtonum.h StrToFloatT):
 *  `[+-] digits [. digits] [(e|E) [+-] digits]`, read from a 32-byte window at
 *  LDS byte a -- the numbers the 16-byte fast decoder leaves out: exponents
 *  (`1.5e-3`) and fractions of 8 to 16 digits.  Same arithmetic as the
 *  reference, so bit-identical: the integer part (<= 7 digits) is exact in
 *  float; the fraction is float(double(F) / double(10^n)) with F, 10^n exact
 *  (n <= 16); the exponent scale is built by the reference's loop of rounded
 *  double products, then one IEEE float multiply or divide.  ok is false for
 *  anything longer (the generic parser takes it); `limit` bounds the staged
 *  bytes the number may use.
 */
struct ExtNum {
  float fval;
  uint32_t end, term;
  bool ok;
};

__device__ __forceinline__ ExtNum parse_num_ext(const uint4* lds, uint32_t a, uint32_t limit) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  ExtNum o;
  // every digit run is read from a 12-byte LDS window at its own start and
  // decoded 8 digits at a time (digit_run8): no lane-varying selects over a
  // register window (the round-5 form spent ~60 % of its VALU on those)
  const uint3 g = ext12(lds, a);
  const uint32_t c0 = g.x & 0xFFu;
  const bool neg = c0 == '-';
  const uint32_t s = (neg || c0 == '+') ? 1u : 0u;
  const uint32_t h0 = __builtin_amdgcn_alignbyte(g.y, g.x, s);
  const uint32_t h1 = __builtin_amdgcn_alignbyte(g.z, g.y, s);
  const uint32_t nb = __builtin_amdgcn_alignbyte(g.z, g.y, s + 1u) >> 24;
  const Run8 ir = digit_run8(h0, h1, nb);  // integer digits (<= 7 for an exact float)
  const uint32_t k = ir.k;
  const bool dot = ir.term == '.';
  // fraction digits: two runs of up to 8 (<= 16 digits)
  const uint32_t fa = a + s + k + 1u;
  const uint3 f1 = ext12(lds, fa);
  const Run8 r1 = digit_run8(f1.x, f1.y, f1.z & 0xFFu);
  const uint3 f2 = ext12(lds, fa + 8u);
  const Run8 r2 = digit_run8(f2.x, f2.y, f2.z & 0xFFu);
  const bool two = r1.k == 8u;
  const uint32_t nf = dot ? (two ? 8u + r2.k : r1.k) : 0u;
  const uint32_t after = dot ? fa + nf : a + s + k;  // LDS byte after the mantissa
  const uint32_t cterm = dot ? (two ? r2.term : r1.term) : ir.term;
  // exponent: (e|E) [+-] digits (<= 3)
  const bool has_e = cterm == 'e' || cterm == 'E';
  const uint3 e = ext12(lds, after + 1u);
  const uint32_t cs = e.x & 0xFFu;
  const bool eneg = cs == '-';
  const uint32_t es = (cs == '-' || cs == '+') ? 1u : 0u;
  const Run8 er = digit_run8(__builtin_amdgcn_alignbyte(e.y, e.x, es),
                             __builtin_amdgcn_alignbyte(e.z, e.y, es), 0u);
  const uint32_t ne = has_e ? er.k : 0u;
  const uint32_t ex = er.val;
  const uint32_t end = has_e ? after + 1u + es + ne : after;
  const uint32_t pos = end - a;
  o.term = has_e ? er.term : cterm;
  o.end = end;
  o.ok = k <= 7 && (k | nf) != 0 && nf < 16 && ne < 4 && pos < 28 && end < limit;
  // the reference arithmetic (strtonum.h StrToFloatT)
  float value = static_cast<float>(ir.val);
  if (dot) {
    // F / 10^nf: the float form of parse_num for nf <= 7 (equal to the
    // rounded double quotient there, see the file comment), the double
    // quotient of the reference for longer fractions
    float p, inv;
    pow10f(nf < 8u ? nf : 7u, &p, &inv);
    const float ff = static_cast<float>(r1.val);
    const float q0 = ff * inv;
    const float rem = __builtin_fmaf(-q0, p, ff);
    float frac = __builtin_fmaf(rem, inv, q0);
    if (nf >= 8u) {
      const uint64_t fv = static_cast<uint64_t>(r1.val) * pow10_u(r2.k) + r2.val;
      const double pw = 1e8 * static_cast<double>(pow10_u(r2.k));  // 10^nf, exact
      frac = static_cast<float>(static_cast<double>(fv) / pw);
    }
    value += frac;
  }
  if (has_e) {
    float scale;
    if (ex <= 10u) {
      // 10^ex is exact in float up to 10^10: the reference loop's products
      // are all exact there
      scale = ex <= 7u ? static_cast<float>(pow10_u(ex)) : (ex == 8u ? 1e8f : (ex == 9u ? 1e9f : 1e10f));
    } else {
      scale = 1.0f;
      uint32_t m = ex > 38 ? 38u : ex;
      while (m >= 8) {
        scale = static_cast<float>(static_cast<double>(scale) * 1e8);
        m -= 8;
      }
      while (m > 0) {
        scale = static_cast<float>(static_cast<double>(scale) * 10.0);
        m -= 1;
      }
    }
    value = eneg ? (value / scale) : (value * scale);
  }
  o.fval = neg ? -value : value;
  return o;
}

/*!
 * \brief decode() for the tokens it declined, with parse_num_ext for every
 *  float field (labels, weights, values): exponents and long fractions stay
 *  on the lane instead of the generic global-memory parser.  Integer fields
 *  are parse_int's as in decode().  limit: end of the token's staging slot.
 */
struct ExtToken {
  Token t;
  bool ok;
};

template <TextFormat F>
__device__ __forceinline__ bool decode_ext_into(const uint4* lds, uint32_t a, bool is_label,
                                                uint32_t limit, Token* t) {
  if (is_label) {
    const ExtNum n1 = parse_num_ext(lds, a, limit);
    const bool c1 = n1.term == ':';
    ExtNum n2 = n1;
    if (c1) n2 = parse_num_ext(lds, n1.end + 1, limit);
    t->f0 = n1.fval;
    t->f1 = n2.fval;
    t->r = c1 ? 2 : 1;
    return n1.ok && (c1 ? (n2.ok && is_end(n2.term)) : is_end(n1.term));
  }
  const Num n1 = parse_int(lds, a);
  const bool c1 = n1.term == ':';
  t->u0 = n1.ival;
  if (F == TextFormat::kLibSVM) {
    if (!c1) {
      t->r = 1;
      t->f0 = 1.0f;
      return n1.ok_uint && is_end(n1.term);
    }
    const ExtNum v = parse_num_ext(lds, n1.end + 1, limit);
    t->f0 = v.fval;
    t->r = 2;
    return n1.ok_uint && v.ok && is_end(v.term);
  }
  // LibFM field:index[:value]
  const Num n2 = parse_int(lds, n1.end + 1);
  const bool c2 = n2.term == ':';
  t->u1 = n2.ival;
  if (!c2) {
    t->r = 2;
    t->f0 = 1.0f;
    return c1 && n1.ok_uint && n2.ok_uint && is_end(n2.term);
  }
  const ExtNum v = parse_num_ext(lds, n2.end + 1, limit);
  t->f0 = v.fval;
  t->r = 3;
  return c1 && n1.ok_uint && n2.ok_uint && v.ok && is_end(v.term);
}

/*! \brief out of line and by value (a result pointer into the caller's
 *  frame would put the token on the stack) */
template <TextFormat F>
__device__ __noinline__ ExtToken decode_ext(const uint4* lds, uint32_t a, bool is_label,
                                            uint32_t limit) {
  ExtToken r;
  r.t.u0 = r.t.u1 = r.t.u0_hi = r.t.u1_hi = 0;
  r.t.f0 = r.t.f1 = 0.0f;
  r.t.r = 0;
  r.ok = decode_ext_into<F>(lds, a, is_label, limit, &r.t);
  return r;
}

}  // namespace tok
}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_SRC_GPU_TOKEN_DECODE_H_
