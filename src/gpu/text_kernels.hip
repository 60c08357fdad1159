/*!
 * \file src/gpu/text_kernels.hip
 * \brief CDNA4 text -> CSR kernels: K1 line index, K2 per-line count,
 *  K4 per-line fill (LibSVM / LibFM / CSV), K8 max-index reduction.
 *
 * Design (MI355X-first):
 *  - K1 works on 4 KiB tiles: each lane of a 256-lane workgroup takes one
 *    16-byte vector (global_load_dwordx4), classifies EOL bytes with a SWAR
 *    compare, and line starts are compacted with a workgroup scan.
 *  - K2/K4 run ONE WAVE64 PER LINE.  The wave streams its line through a
 *    2 KiB LDS window (two 1 KiB pieces, 16 B per lane, ds_write_b128).  Per
 *    lane, SWAR compares of the 16 bytes just loaded give separator / digit /
 *    delimiter bit masks; token starts, token ends (next separator: own mask,
 *    else the first higher lane from a ballot + one shuffle, else the next
 *    piece) and "token has a digit" are pure bit arithmetic, token ordinals
 *    come from a wave prefix sum.  The owning lane then pulls the token's
 *    bytes out of LDS with 3 x ds_read_b128 and a funnel shift into 8 VGPRs
 *    and runs the shared parser on a register iterator (no dependent load per
 *    byte); tokens > 32 B use the LDS/HBM pointer path.  K4 writes index/value
 *    at offset + rank (a wave prefix sum over valid feature tokens) and
 *    reduces max(index) with one atomicMax per wave (K8).
 *  - Number parsing is the shared host/device code of src/data/strtonum.h,
 *    so the device CSR is bit-identical to the CPU parsers' output.
 */
#include <hip/hip_runtime.h>

#include "../data/strtonum.h"
#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {

namespace {
constexpr int kThreads = 256;
constexpr int kWavesPerBlock = kThreads / dev::kWave;
constexpr uint32_t kPiece = 1024;        // bytes per wave load step (64 x 16 B)
constexpr uint32_t kWindow = 2 * kPiece;  // LDS bytes per wave

__device__ __forceinline__ uint32_t eol_mask(uint4 v) {
  return dev::byte_eq_mask(v, '\n') | dev::byte_eq_mask(v, '\r');
}

// ------------------------------------------------------------------ K1
__device__ __forceinline__ uint32_t line_start_mask(const uint8_t* __restrict__ text, size_t n,
                                                    size_t pos, uint4* vout) {
  const int lane = dev::lane_id();
  uint4 v = make_uint4(0, 0, 0, 0);
  if (pos < n) v = *reinterpret_cast<const uint4*>(text + pos);
  *vout = v;
  const uint32_t eol = eol_mask(v);
  // previous byte: last byte of the left neighbour, or a load for lane 0
  uint32_t prev_last = __shfl_up(v.w >> 24, 1, dev::kWave);
  bool prev_eol;
  if (lane == 0) {
    prev_eol = pos == 0 ? true : (text[pos - 1] == '\n' || text[pos - 1] == '\r');
  } else {
    prev_eol = prev_last == '\n' || prev_last == '\r';
  }
  uint32_t valid = 0xFFFFu;
  if (pos >= n) {
    valid = 0;
  } else if (n - pos < 16) {
    valid = (1u << (n - pos)) - 1u;
  }
  const uint32_t starts = ~eol & ((eol << 1) | (prev_eol ? 1u : 0u)) & valid;
  return starts & 0xFFFFu;
}

__global__ __launch_bounds__(kThreads) void k_line_count(const uint8_t* __restrict__ text, size_t n,
                                                         uint64_t* __restrict__ tile_counts) {
  __shared__ uint64_t smem[4];
  const size_t pos = blockIdx.x * kLineTileBytes + threadIdx.x * 16;
  uint4 v;
  const uint32_t m = line_start_mask(text, n, pos, &v);
  const uint64_t cnt = dev::block_sum_256<uint64_t>(__popc(m), smem);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = cnt;
}

__global__ __launch_bounds__(kThreads) void k_line_emit(const uint8_t* __restrict__ text, size_t n,
                                                        const uint64_t* __restrict__ tile_base,
                                                        uint32_t* __restrict__ line_starts) {
  __shared__ uint64_t smem[4];
  const size_t pos = blockIdx.x * kLineTileBytes + threadIdx.x * 16;
  uint4 v;
  uint32_t m = line_start_mask(text, n, pos, &v);
  uint64_t tot;
  uint64_t idx = dev::block_excl_scan_256<uint64_t>(__popc(m), smem, &tot) + tile_base[blockIdx.x];
  while (m != 0) {
    const int j = __ffs(m) - 1;
    m &= m - 1;
    line_starts[idx++] = static_cast<uint32_t>(pos + j);
  }
}

// --------------------------------------------------------------- lines
constexpr uint32_t kNone = 0xFFFFFFFFu;

/*!
 * \brief up to 32 bytes of a token held in 8 VGPRs; operator++ funnel-shifts
 *  the window (v_alignbyte_b32), so the shared strtonum.h parsers run on
 *  registers without a dependent memory load per byte.
 */
struct RegIter {
  uint32_t w[8];
  uint32_t pos;
  __device__ __forceinline__ char operator*() const { return static_cast<char>(w[0] & 0xffu); }
  __device__ __forceinline__ RegIter& operator++() {
#pragma unroll
    for (int i = 0; i < 7; ++i) w[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], 1);
    w[7] >>= 8;
    ++pos;
    return *this;
  }
  __device__ __forceinline__ bool operator!=(const RegIter& o) const { return pos != o.pos; }
  __device__ __forceinline__ bool operator==(const RegIter& o) const { return pos == o.pos; }
};

/*! \brief one token of the current line: [p, q) in chunk coordinates */
struct TokenRef {
  const uint8_t* text;
  const uint8_t* win;  // LDS window (2 KiB), win[0] = text[wbase]
  uint32_t wbase;
  uint32_t p, q;
  bool has_digit;

  __device__ __forceinline__ uint32_t len() const { return q - p; }
  /*! \brief tokens of <= 32 bytes are parsed from registers */
  __device__ __forceinline__ bool fast() const { return q - p <= 32; }
  __device__ __forceinline__ RegIter reg() const {
    // 3 x ds_read_b128 from the 16-byte aligned LDS offset, then a byte funnel
    // shift by (offset & 15): bytes [p, p+32) land in w[0..7]
    const uint32_t o = p - wbase;
    const uint4* src = reinterpret_cast<const uint4*>(win + (o & ~15u));
    const uint4 a = src[0], b = src[1], c = src[2];
    uint32_t d[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    const uint32_t s = o & 15u;
    if (s & 8u) {
#pragma unroll
      for (int i = 0; i < 10; ++i) d[i] = d[i + 2];
    }
    if (s & 4u) {
#pragma unroll
      for (int i = 0; i < 9; ++i) d[i] = d[i + 1];
    }
    RegIter it;
#pragma unroll
    for (int i = 0; i < 8; ++i) it.w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], s & 3u);
    it.pos = 0;
    return it;
  }
  /*! \brief generic pointer to the token (LDS if inside the window, else HBM) */
  __device__ __forceinline__ const char* ptr() const {
    return (q - wbase <= kWindow) ? reinterpret_cast<const char*>(win + (p - wbase))
                                  : reinterpret_cast<const char*>(text + p);
  }
  /*! \brief call fn(begin, end) with register iterators (fast) or pointers */
  template <class Fn>
  __device__ __forceinline__ void with_bytes(Fn fn) const {
    if (fast()) {
      RegIter b = reg();
      RegIter e = b;
      e.pos = q - p;
      fn(b, e);
    } else {
      const char* b = ptr();
      fn(b, b + (q - p));
    }
  }
};

template <TextFormat F>
__device__ __forceinline__ bool is_sep_byte(uint8_t c, char delim) {
  if constexpr (F == TextFormat::kCSV) {
    return c == static_cast<uint8_t>(delim) || c == '\n' || c == '\r';
  } else {
    return c == ' ' || c == '\t' || c == '\n' || c == '\r';
  }
}

/*! \brief exact per-byte flags (bit j) of '0' <= byte <= '9' */
__device__ __forceinline__ uint32_t digit_mask(uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = w[i];
    const uint32_t lo7 = x & 0x7F7F7F7Fu;
    // hasbetween(x, '0'-1, '9'+1): high bit of each byte with 0x2F < c < 0x3A
    const uint32_t t =
        ((0x7F7F7F7Fu + 0x3A3A3A3Au) - lo7) & ~x & (lo7 + (0x7F7F7F7Fu - 0x2F2F2F2Fu)) & 0x80808080u;
    const uint32_t g = ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
    m |= g << (4 * i);
  }
  return m;
}

__device__ __forceinline__ uint32_t digitchar_mask(uint4 v) {
  return digit_mask(v) | dev::byte_eq_mask(v, '+') | dev::byte_eq_mask(v, '-') |
         dev::byte_eq_mask(v, '.') | dev::byte_eq_mask(v, 'e') | dev::byte_eq_mask(v, 'E');
}

/*! \brief per-lane masks of one 16-byte vector of a line [b, e) */
struct LaneMasks {
  uint32_t sep;    // separator bytes, plus every byte outside [b, e)
  uint32_t dig;    // digit characters inside [b, e)
  uint32_t delim;  // CSV delimiter bytes inside [b, e)
  uint32_t eol;    // EOL bytes
};

template <TextFormat F>
__device__ __forceinline__ LaneMasks lane_masks(uint4 v, uint32_t pos, uint32_t b, uint32_t e,
                                                char delim) {
  uint32_t valid = 0xFFFFu;
  if (pos + 16 > e) valid = pos >= e ? 0u : ((1u << (e - pos)) - 1u);
  if (pos < b) valid &= b - pos >= 16 ? 0u : ~((1u << (b - pos)) - 1u);
  LaneMasks m;
  m.eol = eol_mask(v);
  if constexpr (F == TextFormat::kCSV) {
    m.delim = dev::byte_eq_mask(v, static_cast<uint8_t>(delim)) & valid;
    m.sep = (m.eol | m.delim | ~valid) & 0xFFFFu;
  } else {
    m.delim = 0;
    m.sep = (m.eol | dev::byte_eq_mask(v, ' ') | dev::byte_eq_mask(v, '\t') | ~valid) & 0xFFFFu;
  }
  m.dig = digitchar_mask(v) & valid;
  return m;
}

/*!
 * \brief first set bit at or after each lane's 16-byte range, searched over
 *  the lanes above it and then the next piece: returns the chunk position or
 *  kNone.  Must be called by the whole (converged) wave.
 */
__device__ __forceinline__ uint32_t next_after_lane(uint32_t mask, uint32_t pstart,
                                                    uint32_t next_piece_first) {
  const int lane = dev::lane_id();
  const uint64_t bal = __ballot(mask != 0);
  const uint64_t higher = lane == 63 ? 0ull : (bal & (~0ull << (lane + 1)));
  const int nl = higher ? __ffsll(static_cast<long long>(higher)) - 1 : lane;
  const uint32_t m2 = __shfl(mask, nl, dev::kWave);
  if (higher == 0) return next_piece_first;
  return pstart + 16u * nl + static_cast<uint32_t>(__ffs(m2) - 1);
}

/*! \brief first set bit of a whole piece (wave-uniform), or kNone */
__device__ __forceinline__ uint32_t first_in_piece(uint32_t mask, uint32_t pstart) {
  const uint64_t bal = __ballot(mask != 0);
  if (bal == 0) return kNone;
  const int fl = __ffsll(static_cast<long long>(bal)) - 1;
  const uint32_t m2 = __shfl(mask, fl, dev::kWave);
  return pstart + 16u * fl + static_cast<uint32_t>(__ffs(m2) - 1);
}

/*!
 * \brief stream line [b, e) through the wave's LDS window and visit its
 *  tokens.  Token boundaries and "contains a digit" come from per-lane byte
 *  masks + ballots (no byte loops); numbers are parsed from registers.
 *  Phase 1 calls vis.classify(tok, ord) for every token; with kEmit, tokens
 *  for which vis.selected(tok, ord) holds are passed to vis.emit(tok, ord,
 *  rank), rank = number of earlier selected tokens of the line.
 */
template <TextFormat F, bool kEmit, class Visitor>
__device__ void walk_line(const uint8_t* __restrict__ text, uint32_t b, uint32_t e, uint8_t* win,
                          char delim, Visitor& vis) {
  const int lane = dev::lane_id();
  uint32_t wbase = b & ~15u;
  uint4* win4 = reinterpret_cast<uint4*>(win);
  auto load = [&](uint32_t addr) -> uint4 {
    return addr < e ? *reinterpret_cast<const uint4*>(text + addr) : make_uint4(0, 0, 0, 0);
  };
  uint4 vcur = load(wbase + 16 * lane);
  uint4 vnext = load(wbase + kPiece + 16 * lane);
  win4[lane] = vcur;
  win4[64 + lane] = vnext;
  LaneMasks mcur = lane_masks<F>(vcur, wbase + 16 * lane, b, e, delim);
  LaneMasks mnext = lane_masks<F>(vnext, wbase + kPiece + 16 * lane, b, e, delim);
  dev::wave_sync();
  uint32_t tok_base = 0, rank_base = 0;
  bool prev_sep = true;     // byte before the line start behaves as a separator
  bool prev_delim = false;  // CSV: previous byte was the delimiter
  for (uint32_t pstart = wbase; pstart < e; pstart += kPiece) {
    const uint32_t pos = pstart + 16 * lane;
    // token starts of this lane's 16 bytes
    uint32_t starts;
    {
      const uint32_t up_sep = __shfl_up(mcur.sep, 1, dev::kWave);
      const uint32_t up_delim = __shfl_up(mcur.delim, 1, dev::kWave);
      if constexpr (F == TextFormat::kCSV) {
        const uint32_t pd = lane == 0 ? (prev_delim ? 1u : 0u) : ((up_delim >> 15) & 1u);
        // every byte after a delimiter starts a field, up to the line end: a
        // trailing delimiter opens no empty last field (reference
        // csv_parser.h:83-96 stops when p reaches lend after the delimiter)
        // (e is the next line's start: the EOL bytes lie inside [b, e))
        starts = ((mcur.delim << 1) | pd) & ~mcur.eol;
        if (b >= pos && b < pos + 16) starts |= 1u << (b - pos);
        const uint32_t room = e > pos ? (e - pos < 16 ? e - pos : 16u) : 0u;
        starts &= room >= 16 ? 0xFFFFu : ((1u << room) - 1u);
      } else {
        const uint32_t ps = lane == 0 ? (prev_sep ? 1u : 0u) : ((up_sep >> 15) & 1u);
        starts = ~mcur.sep & ((mcur.sep << 1) | ps) & 0xFFFFu;
      }
    }
    const uint32_t next_sep_piece = first_in_piece(mnext.sep, pstart + kPiece);
    const uint32_t next_dig_piece = first_in_piece(mnext.dig, pstart + kPiece);
    const uint32_t nsep = next_after_lane(mcur.sep, pstart, next_sep_piece);
    const uint32_t ndig = next_after_lane(mcur.dig, pstart, next_dig_piece);
    uint32_t ntok_total;
    const uint32_t tok_excl = dev::wave_excl_scan<uint32_t>(__popc(starts), &ntok_total);

    auto make_token = [&](int j) -> TokenRef {
      TokenRef t;
      t.text = text;
      t.win = win;
      t.wbase = pstart;
      t.p = pos + j;
      const uint32_t own = mcur.sep & ~((1u << j) - 1u);
      uint32_t q = own ? pos + (__ffs(own) - 1) : nsep;
      bool scanned = false;
      if (q == kNone) {
        // token runs past the next piece: scan HBM (rare: > 1 KiB tokens)
        q = pstart + 2 * kPiece;
        while (q < e && !is_sep_byte<F>(text[q], delim)) ++q;
        scanned = true;
      }
      if (q > e) q = e;
      t.q = q;
      const uint32_t ownd = mcur.dig & ~((1u << j) - 1u);
      const uint32_t fd = ownd ? pos + (__ffs(ownd) - 1) : ndig;
      if (fd != kNone) {
        t.has_digit = fd < q;
      } else if (scanned) {
        bool hd = false;
        for (uint32_t r = pstart + 2 * kPiece; r < q; ++r) hd |= data::isdigitchars(text[r]);
        t.has_digit = hd;
      } else {
        t.has_digit = false;
      }
      return t;
    };

    // phase 1: classify
    uint32_t m = starts;
    uint32_t ord = tok_base + tok_excl;
    uint32_t nsel = 0;
    while (m != 0) {
      const int j = __ffs(m) - 1;
      m &= m - 1;
      nsel += vis.classify(make_token(j), ord);
      ++ord;
    }
    vis.after_classify(tok_base, ntok_total);
    if constexpr (kEmit) {
      uint32_t nsel_total;
      uint32_t rank = rank_base + dev::wave_excl_scan<uint32_t>(nsel, &nsel_total);
      if (vis.emit_enabled()) {
        m = starts;
        ord = tok_base + tok_excl;
        while (m != 0) {
          const int j = __ffs(m) - 1;
          m &= m - 1;
          const TokenRef t = make_token(j);
          if (vis.selected(t, ord)) vis.emit(t, ord, rank++);
          ++ord;
        }
      }
      rank_base += nsel_total;
    }
    tok_base += ntok_total;
    prev_sep = (__shfl(mcur.sep, 63, dev::kWave) >> 15) & 1u;
    prev_delim = (__shfl(mcur.delim, 63, dev::kWave) >> 15) & 1u;
    // slide the window by one piece
    dev::wave_sync();
    vcur = vnext;
    mcur = mnext;
    vnext = load(pstart + 2 * kPiece + 16 * lane);
    mnext = lane_masks<F>(vnext, pstart + 2 * kPiece + 16 * lane, b, e, delim);
    win4[lane] = vcur;
    win4[64 + lane] = vnext;
    dev::wave_sync();
  }
}

/*! \brief "qid:" prefix test on a token */
__device__ __forceinline__ bool tok_is_qid(const TokenRef& t) {
  if (t.len() < 4) return false;
  if (t.fast()) {
    const RegIter r = t.reg();
    return (r.w[0] & 0xFFFFFFFFu) == 0x3A646971u;  // "qid:" little-endian
  }
  const char* c = t.ptr();
  return c[0] == 'q' && c[1] == 'i' && c[2] == 'd' && c[3] == ':';
}

/*! \brief LibFM rule: the first digit-character run is followed by ':' */
__device__ __forceinline__ bool tok_two_parts(const TokenRef& t) {
  bool ok = false;
  t.with_bytes([&](auto p, auto end) {
    while (p != end && !data::isdigitchars(*p)) ++p;
    if (p == end) return;
    while (p != end && data::isdigitchars(*p)) ++p;
    ok = p != end && *p == ':';
  });
  return ok;
}

/*!
 * \brief per-line visitor: phase-1 classification of tokens by role
 *  (label / weight / qid / feature), phase-2 emission of feature tokens.
 */
template <TextFormat F, typename IndexType>
struct LineVisitor {
  int label_col, weight_col;
  // label-token state (only the lane owning token 0 / the label column sets it)
  bool is_label_lane{false}, label_ok{false}, has_weight{false};
  float label{0.0f}, weight{1.0f};
  bool is_qid_lane{false};
  uint64_t qid{0};
  int row_state{0};  // 0 unknown, 1 ok, -1 invalid (wave-uniform)
  // fill target (phase 2)
  IndexType* index{nullptr};
  float* value{nullptr};
  IndexType* field{nullptr};
  uint64_t nnz_pos{0};
  uint64_t nnz_limit{~0ull};
  uint64_t max_index{0}, max_field{0};
  bool any_value{false}, neg{false}, overflow{false};

  __device__ uint32_t classify(const TokenRef& t, uint32_t ord) {
    if constexpr (F == TextFormat::kCSV) {
      if (static_cast<int>(ord) == label_col || static_cast<int>(ord) == weight_col) {
        float v = 0.0f;
        t.with_bytes([&](auto p, auto end) {
          while (p != end && data::isspace(*p)) ++p;
          v = data::StrToFloatT(p, end, static_cast<decltype(p)*>(nullptr));
        });
        if (static_cast<int>(ord) == label_col) {
          is_label_lane = true;
          label_ok = true;
          label = v;
        } else {
          has_weight = true;
          weight = v;
        }
        return 0;
      }
      return 1;
    } else {
      if (ord == 0) {
        is_label_lane = true;
        float l = 0.0f, wgt = 0.0f;
        int r = 0;
        if (t.has_digit) {
          bool bad;
          t.with_bytes([&](auto p, auto end) { r = data::ParsePair<float, float>(p, end, &l, &wgt, &bad); });
        }
        label_ok = r >= 1;
        if (r >= 1) label = l;
        if (r == 2) {
          has_weight = true;
          weight = wgt;
        }
        return 0;
      }
      if constexpr (F == TextFormat::kLibSVM) {
        if (ord == 1 && tok_is_qid(t)) {
          is_qid_lane = true;
          t.with_bytes([&](auto p, auto end) {
            ++p; ++p; ++p; ++p;
            qid = static_cast<uint64_t>(
                data::StrToInt<int64_t>(p, end, static_cast<decltype(p)*>(nullptr)));
          });
          return 0;
        }
        return t.has_digit ? 1u : 0u;
      } else {
        return (t.has_digit && tok_two_parts(t)) ? 1u : 0u;
      }
    }
  }
  /*! \brief same decision as classify, without side effects (phase 2) */
  __device__ bool selected(const TokenRef& t, uint32_t ord) const {
    if constexpr (F == TextFormat::kCSV) {
      return static_cast<int>(ord) != label_col && static_cast<int>(ord) != weight_col;
    } else {
      if (ord == 0) return false;
      if constexpr (F == TextFormat::kLibSVM) {
        if (ord == 1 && tok_is_qid(t)) return false;
        return t.has_digit;
      } else {
        return t.has_digit && tok_two_parts(t);
      }
    }
  }
  __device__ void after_classify(uint32_t tok_base, uint32_t ntok) {
    if (row_state == 0 && tok_base + ntok > 0) {
      if constexpr (F == TextFormat::kCSV) {
        row_state = 1;
      } else {
        row_state = __ballot(label_ok) != 0 ? 1 : -1;
      }
    }
  }
  __device__ bool emit_enabled() const { return row_state == 1; }
  __device__ void emit(const TokenRef& t, uint32_t ord, uint32_t rank) {
    const uint64_t pos = nnz_pos + rank;
    // defensive bound: a count/fill disagreement must never write out of bounds
    if (pos >= nnz_limit) {
      overflow = true;
      return;
    }
    bool bad = false;
    if constexpr (F == TextFormat::kCSV) {
      float v = 0.0f;
      t.with_bytes([&](auto p, auto end) {
        while (p != end && data::isspace(*p)) ++p;
        v = data::StrToFloatT(p, end, static_cast<decltype(p)*>(nullptr));
      });
      index[pos] = static_cast<IndexType>(rank);
      value[pos] = v;
      if (rank > max_index) max_index = rank;
    } else if constexpr (F == TextFormat::kLibSVM) {
      IndexType idx = 0;
      float v = 0.0f;
      int r = 0;
      t.with_bytes([&](auto p, auto end) { r = data::ParsePair<IndexType, float>(p, end, &idx, &v, &bad); });
      index[pos] = idx;
      value[pos] = r == 2 ? v : 1.0f;
      any_value |= (r == 2);
      if (static_cast<uint64_t>(idx) > max_index) max_index = idx;
    } else {
      IndexType fid = 0, idx = 0;
      float v = 0.0f;
      int r = 0;
      t.with_bytes([&](auto p, auto end) {
        r = data::ParseTriple<IndexType, IndexType, float>(p, end, &fid, &idx, &v, &bad);
      });
      field[pos] = fid;
      index[pos] = idx;
      value[pos] = r == 3 ? v : 1.0f;
      any_value |= (r == 3);
      if (static_cast<uint64_t>(idx) > max_index) max_index = idx;
      if (static_cast<uint64_t>(fid) > max_field) max_field = fid;
    }
    neg |= bad;
  }
};

/*!
 * \brief K9 fused into the per-line walk: feature tokens are hashed straight
 *  into the wave's LDS row (dim floats, ds_add_f32) -- no CSR in between.
 */
template <TextFormat F, typename IndexType>
struct HashVisitor {
  float* row;  // this wave's LDS accumulator
  uint32_t dim, seed;
  bool is_label_lane{false}, label_ok{false};
  float label{0.0f};
  int row_state{0};
  bool neg{false};

  __device__ uint32_t classify(const TokenRef& t, uint32_t ord) {
    if (ord == 0) {
      is_label_lane = true;
      float l = 0.0f, wgt = 0.0f;
      int r = 0;
      if (t.has_digit) {
        bool bad;
        t.with_bytes([&](auto p, auto end) { r = data::ParsePair<float, float>(p, end, &l, &wgt, &bad); });
      }
      label_ok = r >= 1;
      if (r >= 1) label = l;
      return 0;
    }
    if (!t.has_digit) return 0;
    uint64_t key = 0;
    float v = 1.0f;
    bool bad = false;
    if constexpr (F == TextFormat::kLibSVM) {
      if (ord == 1 && tok_is_qid(t)) return 0;
      IndexType idx = 0;
      float val = 0.0f;
      int r = 0;
      t.with_bytes([&](auto p, auto end) {
        r = data::ParsePair<IndexType, float>(p, end, &idx, &val, &bad);
      });
      key = dev::hash_key(static_cast<uint64_t>(idx), 0, false);
      v = r == 2 ? val : 1.0f;
    } else {
      if (!tok_two_parts(t)) return 0;
      IndexType fid = 0, idx = 0;
      float val = 0.0f;
      int r = 0;
      t.with_bytes([&](auto p, auto end) {
        r = data::ParseTriple<IndexType, IndexType, float>(p, end, &fid, &idx, &val, &bad);
      });
      key = dev::hash_key(static_cast<uint64_t>(idx), static_cast<uint64_t>(fid), true);
      v = r == 3 ? val : 1.0f;
    }
    neg |= bad;
    const uint32_t h = dev::hash_u64(key, seed);
    atomicAdd(&row[h % dim], (h & 0x80000000u) ? -v : v);
    return 0;
  }
  __device__ bool selected(const TokenRef&, uint32_t) const { return false; }
  __device__ void after_classify(uint32_t tok_base, uint32_t ntok) {
    if (row_state == 0 && tok_base + ntok > 0) row_state = __ballot(label_ok) != 0 ? 1 : -1;
  }
  __device__ bool emit_enabled() const { return false; }
  __device__ void emit(const TokenRef&, uint32_t, uint32_t) {}
};

/*!
 * \brief fused LibSVM / LibFM text -> hashed dense batch (BASELINE config 5):
 *  one wave per line walks the line (exact tokenizer), hashes every feature
 *  into its LDS row, then writes the row once -- OCP fp8 e4m3 (gfx950
 *  v_cvt_pk_fp8_f32, 4 columns per 32-bit store) or f32 -- plus its label.
 *  Rows are the valid lines (line_info scanned by K3, as for the CSR fill).
 */
template <TextFormat F, typename IndexType, bool kFP8>
__global__ __launch_bounds__(kThreads) void k_text_hash(const uint8_t* __restrict__ text, size_t n,
                                                        const uint32_t* __restrict__ line_starts,
                                                        size_t nlines, const uint64_t* __restrict__ line_info,
                                                        uint64_t row_base, int dim, float scale,
                                                        uint32_t seed, void* __restrict__ out,
                                                        float* __restrict__ labels,
                                                        MetaPartial* __restrict__ partials) {
  __shared__ uint4 lds[kWavesPerBlock][kWindow / 16];
  extern __shared__ __attribute__((aligned(16))) float rows[];
  const int wid = threadIdx.x / dev::kWave;
  const int lane = dev::lane_id();
  uint8_t* win = reinterpret_cast<uint8_t*>(lds[wid]);
  float* row = rows + static_cast<size_t>(wid) * dim;
  for (int c = lane; c < dim; c += dev::kWave) row[c] = 0.0f;
  dev::wave_sync();
  const size_t nwaves = static_cast<size_t>(gridDim.x) * kWavesPerBlock;
  bool wneg = false;
  for (size_t line = static_cast<size_t>(blockIdx.x) * kWavesPerBlock + wid; line < nlines;
       line += nwaves) {
    const uint32_t b = line_starts[line];
    const uint32_t e = line + 1 < nlines ? line_starts[line + 1] : static_cast<uint32_t>(n);
    HashVisitor<F, IndexType> vis;
    vis.row = row;
    vis.dim = static_cast<uint32_t>(dim);
    vis.seed = seed;
    walk_line<F, false>(text, b, e, win, ' ', vis);
    wneg |= vis.neg;
    dev::wave_sync();  // every ds_add of the line is done
    if (vis.row_state == 1) {
      const uint64_t r = row_base + (line_info[line] >> 32);
      const uint64_t lmask = __ballot(vis.is_label_lane);
      const int ll = lmask ? __ffsll(static_cast<long long>(lmask)) - 1 : 0;
      const float label = lmask ? __shfl(vis.label, ll, dev::kWave) : 0.0f;
      if (lane == 0) labels[r] = label;
      if constexpr (kFP8) {
        uint32_t* o = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(out) + r * dim);
        for (int c = lane * 4; c < dim; c += dev::kWave * 4) {
          int packed = __builtin_amdgcn_cvt_pk_fp8_f32(row[c] * scale, row[c + 1] * scale, 0, false);
          packed = __builtin_amdgcn_cvt_pk_fp8_f32(row[c + 2] * scale, row[c + 3] * scale, packed,
                                                   true);
          o[c / 4] = static_cast<uint32_t>(packed);
        }
      } else {
        float* o = static_cast<float*>(out) + r * dim;
        for (int c = lane; c < dim; c += dev::kWave) o[c] = row[c];
      }
    }
    dev::wave_sync();
    for (int c = lane; c < dim; c += dev::kWave) row[c] = 0.0f;
    dev::wave_sync();
  }
  dev::block_store_partial(0ull, 0ull, wneg ? kFlagNegIndex : 0u, partials);
}

// ------------------------------------------------------------------ K2
template <TextFormat F>
__global__ __launch_bounds__(kThreads) void k_text_count(const uint8_t* __restrict__ text, size_t n,
                                                         const uint32_t* __restrict__ line_starts,
                                                         size_t nlines, TextParseConfig cfg,
                                                         uint64_t* __restrict__ line_info,
                                                         MetaPartial* __restrict__ partials) {
  __shared__ uint4 lds[kWavesPerBlock][kWindow / 16];
  const int wid = threadIdx.x / dev::kWave;
  const int lane = dev::lane_id();
  uint8_t* win = reinterpret_cast<uint8_t*>(lds[wid]);
  const size_t nwaves = static_cast<size_t>(gridDim.x) * kWavesPerBlock;
  unsigned wflags = 0;
  for (size_t line = static_cast<size_t>(blockIdx.x) * kWavesPerBlock + wid; line < nlines;
       line += nwaves) {
    const uint32_t b = line_starts[line];
    const uint32_t e = line + 1 < nlines ? line_starts[line + 1] : static_cast<uint32_t>(n);
    LineVisitor<F, uint32_t> vis;
    vis.label_col = cfg.label_column;
    vis.weight_col = cfg.weight_column;
    struct Counter {
      LineVisitor<F, uint32_t>* v;
      uint32_t nfeat{0};
      __device__ uint32_t classify(const TokenRef& t, uint32_t ord) {
        const uint32_t s = v->classify(t, ord);
        nfeat += s;
        return s;
      }
      __device__ void after_classify(uint32_t tb, uint32_t nt) { v->after_classify(tb, nt); }
      __device__ bool emit_enabled() const { return false; }
      __device__ bool selected(const TokenRef&, uint32_t) const { return false; }
      __device__ void emit(const TokenRef&, uint32_t, uint32_t) {}
    } counter{&vis};
    walk_line<F, false>(text, b, e, win, cfg.delimiter, counter);
    const uint32_t nfeat = dev::wave_sum(counter.nfeat);
    const bool row_ok = vis.row_state == 1;
    const bool w = __ballot(vis.has_weight) != 0;
    const bool qd = __ballot(vis.is_qid_lane) != 0;
    if (lane == 0) line_info[line] = row_ok ? ((1ull << 32) | nfeat) : 0ull;
    if (row_ok && w) wflags |= kFlagWeight;
    if (row_ok && qd) wflags |= kFlagQid;
  }
  dev::block_store_partial(0ull, 0ull, wflags, partials);
}

// ------------------------------------------------------------------ K4
template <TextFormat F, typename IndexType>
__global__ __launch_bounds__(kThreads) void k_text_fill(const uint8_t* __restrict__ text, size_t n,
                                                        const uint32_t* __restrict__ line_starts,
                                                        size_t nlines, TextParseConfig cfg,
                                                        const uint64_t* __restrict__ line_info,
                                                        FillTarget<IndexType> out,
                                                        MetaPartial* __restrict__ partials) {
  __shared__ uint4 lds[kWavesPerBlock][kWindow / 16];
  const int wid = threadIdx.x / dev::kWave;
  const int lane = dev::lane_id();
  uint8_t* win = reinterpret_cast<uint8_t*>(lds[wid]);
  const size_t nwaves = static_cast<size_t>(gridDim.x) * kWavesPerBlock;
  uint64_t wmax_index = 0, wmax_field = 0;
  bool wany_value = false, wneg = false, woverflow = false;
  for (size_t line = static_cast<size_t>(blockIdx.x) * kWavesPerBlock + wid; line < nlines;
       line += nwaves) {
    const uint32_t b = line_starts[line];
    const uint32_t e = line + 1 < nlines ? line_starts[line + 1] : static_cast<uint32_t>(n);
    const uint64_t info = line_info[line];
    const uint64_t row = out.row_base + (info >> 32);
    LineVisitor<F, IndexType> vis;
    vis.label_col = cfg.label_column;
    vis.weight_col = cfg.weight_column;
    vis.index = out.index;
    vis.value = out.value;
    vis.field = out.field;
    vis.nnz_pos = out.nnz_base + (info & 0xffffffffull);
    vis.nnz_limit = out.nnz_limit;
    walk_line<F, true>(text, b, e, win, cfg.delimiter, vis);
    wmax_index = vis.max_index > wmax_index ? vis.max_index : wmax_index;
    wmax_field = vis.max_field > wmax_field ? vis.max_field : wmax_field;
    wany_value |= vis.any_value;
    wneg |= vis.neg;
    woverflow |= vis.overflow;
    if (vis.row_state == 1 && row >= out.row_limit) woverflow = true;
    if (vis.row_state == 1 && row < out.row_limit) {
      // broadcast the label-token results to lane 0 and write the row arrays
      const uint64_t lmask = __ballot(vis.is_label_lane);
      const int ll = lmask ? __ffsll(static_cast<long long>(lmask)) - 1 : 0;
      const float label = lmask ? __shfl(vis.label, ll, dev::kWave) : 0.0f;
      const uint64_t wmask = __ballot(vis.has_weight);
      const int wl = wmask ? __ffsll(static_cast<long long>(wmask)) - 1 : 0;
      const float weight = wmask ? __shfl(vis.weight, wl, dev::kWave) : 1.0f;
      const uint64_t qmask = __ballot(vis.is_qid_lane);
      const int ql = qmask ? __ffsll(static_cast<long long>(qmask)) - 1 : 0;
      const uint64_t qid = qmask ? __shfl(vis.qid, ql, dev::kWave) : 0ull;
      if (lane == 0) {
        out.offset[row] = out.nnz_base + (info & 0xffffffffull);
        out.label[row] = label;
        if (out.weight != nullptr) out.weight[row] = weight;
        if (out.qid != nullptr) out.qid[row] = qid;
      }
    }
  }
  // K8: workgroup reduction into this block's slot (no same-address atomics)
  unsigned fl = 0;
  if (wany_value) fl |= kFlagValue;
  if (wneg) fl |= kFlagNegIndex;
  if (woverflow) fl |= kFlagOverflow;
  if (F == TextFormat::kLibFM) fl |= kFlagField;
  dev::block_store_partial(static_cast<unsigned long long>(wmax_index),
                           static_cast<unsigned long long>(wmax_field), fl, partials);
}

__global__ void k_close_offsets(uint64_t* offset, uint64_t row_end, uint64_t nnz_end) {
  offset[row_end] = nnz_end;
}

int LineGrid(size_t nlines) {
  // enough waves to fill 256 CUs x 8 waves/SIMD-ish, grid-stride beyond that
  const size_t blocks = (nlines + kWavesPerBlock - 1) / kWavesPerBlock;
  return static_cast<int>(blocks < 8192 ? (blocks == 0 ? 1 : blocks) : 8192);
}
}  // namespace

size_t LineIndexTiles(size_t nbytes) {
  const size_t ntiles = (nbytes + kLineTileBytes - 1) / kLineTileBytes;
  return ntiles + 1 + ScanPartials(ntiles) + 1;
}

void LaunchLineCount(const char* text, size_t nbytes, uint64_t* tile_scratch, ChunkMeta* meta,
                     hipStream_t stream) {
  const size_t ntiles = (nbytes + kLineTileBytes - 1) / kLineTileBytes;
  if (ntiles == 0) {
    (void)hipMemsetAsync(&meta->nlines, 0, sizeof(uint64_t), stream);
    return;
  }
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  hipLaunchKernelGGL(k_line_count, dim3(ntiles), dim3(kThreads), 0, stream, t, nbytes,
                     tile_scratch);
  LaunchScanU64(tile_scratch, ntiles, tile_scratch + ntiles + 1,
                reinterpret_cast<uint64_t*>(&meta->nlines), stream);
}

void LaunchLineEmit(const char* text, size_t nbytes, const uint64_t* tile_scratch,
                    uint32_t* line_starts, hipStream_t stream) {
  const size_t ntiles = (nbytes + kLineTileBytes - 1) / kLineTileBytes;
  if (ntiles == 0) return;
  hipLaunchKernelGGL(k_line_emit, dim3(ntiles), dim3(kThreads), 0, stream,
                     reinterpret_cast<const uint8_t*>(text), nbytes, tile_scratch, line_starts);
}

void LaunchTextCount(const char* text, size_t nbytes, const uint32_t* line_starts, size_t nlines,
                     const TextParseConfig& cfg, uint64_t* line_info, MetaPartial* partials,
                     ChunkMeta* meta, hipStream_t stream) {
  if (nlines == 0) return;
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  const dim3 grid(LineGrid(nlines)), block(kThreads);
  switch (cfg.format) {
    case TextFormat::kLibSVM:
      hipLaunchKernelGGL(k_text_count<TextFormat::kLibSVM>, grid, block, 0, stream, t, nbytes,
                         line_starts, nlines, cfg, line_info, partials);
      break;
    case TextFormat::kLibFM:
      hipLaunchKernelGGL(k_text_count<TextFormat::kLibFM>, grid, block, 0, stream, t, nbytes,
                         line_starts, nlines, cfg, line_info, partials);
      break;
    case TextFormat::kCSV:
      hipLaunchKernelGGL(k_text_count<TextFormat::kCSV>, grid, block, 0, stream, t, nbytes,
                         line_starts, nlines, cfg, line_info, partials);
      break;
  }
  LaunchReducePartials(partials, static_cast<int>(grid.x), meta, stream);
}

template <typename IndexType>
void LaunchTextFill(const char* text, size_t nbytes, const uint32_t* line_starts, size_t nlines,
                    const TextParseConfig& cfg, const uint64_t* line_info,
                    const FillTarget<IndexType>& out, uint64_t nrows, uint64_t nnz,
                    MetaPartial* partials, ChunkMeta* meta, hipStream_t stream) {
  if (nlines != 0) {
    const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
    const dim3 grid(LineGrid(nlines)), block(kThreads);
    switch (cfg.format) {
      case TextFormat::kLibSVM:
        hipLaunchKernelGGL((k_text_fill<TextFormat::kLibSVM, IndexType>), grid, block, 0, stream,
                           t, nbytes, line_starts, nlines, cfg, line_info, out, partials);
        break;
      case TextFormat::kLibFM:
        hipLaunchKernelGGL((k_text_fill<TextFormat::kLibFM, IndexType>), grid, block, 0, stream,
                           t, nbytes, line_starts, nlines, cfg, line_info, out, partials);
        break;
      case TextFormat::kCSV:
        hipLaunchKernelGGL((k_text_fill<TextFormat::kCSV, IndexType>), grid, block, 0, stream, t,
                           nbytes, line_starts, nlines, cfg, line_info, out, partials);
        break;
    }
    LaunchReducePartials(partials, static_cast<int>(grid.x), meta, stream);
  }
  LaunchCloseOffsets(out.offset, out.row_base + nrows, out.nnz_base + nnz, stream);
}

template <typename IndexType>
void LaunchTextHashed(const char* text, size_t nbytes, const uint32_t* line_starts, size_t nlines,
                      TextFormat format, const uint64_t* line_info, uint64_t row_base, int dim,
                      float scale, uint32_t seed, bool fp8, void* out, float* labels,
                      MetaPartial* partials, ChunkMeta* meta, hipStream_t stream) {
  if (nlines == 0) return;
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  const dim3 grid(LineGrid(nlines)), block(kThreads);
  const size_t smem = static_cast<size_t>(kWavesPerBlock) * dim * sizeof(float);
#define DMLC_HASH_LAUNCH(FMT, FP8)                                                              \
  hipLaunchKernelGGL((k_text_hash<FMT, IndexType, FP8>), grid, block, smem, stream, t, nbytes, \
                     line_starts, nlines, line_info, row_base, dim, scale, seed, out, labels,    \
                     partials)
  if (format == TextFormat::kLibFM) {
    if (fp8) {
      DMLC_HASH_LAUNCH(TextFormat::kLibFM, true);
    } else {
      DMLC_HASH_LAUNCH(TextFormat::kLibFM, false);
    }
  } else {
    if (fp8) {
      DMLC_HASH_LAUNCH(TextFormat::kLibSVM, true);
    } else {
      DMLC_HASH_LAUNCH(TextFormat::kLibSVM, false);
    }
  }
#undef DMLC_HASH_LAUNCH
  LaunchReducePartials(partials, static_cast<int>(grid.x), meta, stream);
}

template void LaunchTextHashed<uint32_t>(const char*, size_t, const uint32_t*, size_t, TextFormat,
                                         const uint64_t*, uint64_t, int, float, uint32_t, bool,
                                         void*, float*, MetaPartial*, ChunkMeta*, hipStream_t);
template void LaunchTextHashed<uint64_t>(const char*, size_t, const uint32_t*, size_t, TextFormat,
                                         const uint64_t*, uint64_t, int, float, uint32_t, bool,
                                         void*, float*, MetaPartial*, ChunkMeta*, hipStream_t);

void LaunchCloseOffsets(uint64_t* offset, uint64_t row_end, uint64_t nnz_end, hipStream_t stream) {
  hipLaunchKernelGGL(k_close_offsets, dim3(1), dim3(1), 0, stream, offset, row_end, nnz_end);
}

template void LaunchTextFill<uint32_t>(const char*, size_t, const uint32_t*, size_t,
                                       const TextParseConfig&, const uint64_t*,
                                       const FillTarget<uint32_t>&, uint64_t, uint64_t,
                                       MetaPartial*, ChunkMeta*, hipStream_t);
template void LaunchTextFill<uint64_t>(const char*, size_t, const uint32_t*, size_t,
                                       const TextParseConfig&, const uint64_t*,
                                       const FillTarget<uint64_t>&, uint64_t, uint64_t,
                                       MetaPartial*, ChunkMeta*, hipStream_t);

}  // namespace gpu
}  // namespace dmlc
