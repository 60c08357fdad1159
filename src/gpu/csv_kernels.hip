/*!
 * \file src/gpu/csv_kernels.hip
 * \brief K5 fast path: CSV -> CSR on the tile pipeline (count -> two-level
 *  scan -> fill -> finish, sizes via mapped pinned memory), lane per field.
 *
 * Reference loop: CSVParser::ParseBlock (`src/data/csv_parser.h:64-104`):
 * every delimiter-separated field of a line is StrToFloat'ed after skipping
 * leading blanks; the label (and weight) column leave the feature list and
 * the remaining columns are numbered 0, 1, 2, ...; blank lines are no rows.
 *
 * A wave owns the rows that START in its 8 KiB tile and walks the text in
 * 1 KiB steps, 16 bytes per lane, until the first row start of the next tile
 * (at most 4 KiB past its own; longer rows send the chunk to the exact
 * kernels).  Per step every lane turns its 16 bytes into field-start and
 * row-start masks; a segmented wave scan (reset at row starts) gives every
 * field its column, a packed wave scan its field / row / excluded-column
 * ordinals.  The column tells what a field is (label, weight, feature
 * `column - excluded columns before it`), the ordinals where it goes:
 *   S1 k_csv_tile_count : (rows << 32 | entries) per tile + irregular flag,
 *                         straight from global memory (no LDS);
 *   S1p k_csv_tile_count_pos (label / weight column <= 0): the same counts by
 *                         position -- line ends and delimiters only, 8 loads
 *                         in flight, no walk; the fill adds its tile's head
 *                         fields and does S1's checks;
 *   C2 (tile_kernels.hip, raw scan), then
 *   S2 k_csv_tile_fill  : the same walk over a two-step LDS ring (one step
 *                         prefetched, so a number's 16-byte window never
 *                         leaves LDS); the step's fields are listed in LDS and
 *                         decoded 64 per round with the register-window
 *                         decoder (token_decode.h; empty fields are 0, other
 *                         shapes go through strtonum.h's StrToFloat from
 *                         global memory); row starts write the row pointer,
 *                         a row's last field settles a missing label / weight;
 *   C4 (tile_kernels.hip) folds max index / flags and closes the offsets.
 */
#include <dmlc/logging.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "../data/strtonum.h"
#include "./device_common.h"
#include "./kernels.h"
#include "./token_decode.h"

namespace dmlc {
namespace gpu {
namespace {

using namespace dev;  // NOLINT(build/namespaces)

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kStep = 1024;
constexpr uint32_t kExt = 4096;
constexpr uint32_t kTileSteps = static_cast<uint32_t>(kTileBytes) / kStep;
constexpr uint32_t kMaxSteps = (static_cast<uint32_t>(kTileBytes) + kExt) / kStep;
constexpr uint32_t kListCap = 512;     // fields per step (avg field >= 2 bytes)
constexpr uint32_t kRingVecs = 2 * kStep / 16 + 2;  // two steps + a mirror of slot 0's head

struct CsvCfg {
  int label_col;
  int weight_col;   // -1, or a column other than label_col
  int has_weight;   // weight_column >= 0 (every row gets a weight)
  int zero_excl;    // label / weight columns equal to 0 (excluded field per row)
  uint32_t delim;
  int pos;          // positional tile counts (S1p; label / weight at most column 0)
};

/*! \brief bit 7 of every byte of x equal to the byte in c4 (exact SWAR test) */
__device__ __forceinline__ uint32_t hb_eq(uint32_t x, uint32_t c4) {
  const uint32_t y = x ^ c4;
  return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}

/*! \brief bit 7 of every byte of x below 0x20 */
__device__ __forceinline__ uint32_t hb_lt20(uint32_t x) {
  return ~(((x & 0x7F7F7F7Fu) + 0x60606060u) | x) & 0x80808080u;
}

/*! \brief the byte flags of hb_* of a 16-byte slice as a 16-bit mask (byte k
 *  -> bit k): bits 7 / 15 / 23 / 31 gathered by two shift-or steps, no
 *  (quarter-rate) multiply */
__device__ __forceinline__ uint32_t mask16(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3) {
  auto m4 = [](uint32_t h) {
    const uint32_t m = (h >> 7) | (h >> 14);  // b0 -> bit 0, b1 -> bit 1, b2 -> 16, b3 -> 17
    return (m | (m >> 14)) & 0xFu;            // b2 -> bit 2, b3 -> bit 3
  };
  return m4(h0) | (m4(h1) << 4) | (m4(h2) << 8) | (m4(h3) << 12);
}

/*! \brief mask16 by byte dot products: v_dot4_u32_u8 of each word's flag
 *  bytes (0x80 or 0) with the bit weights, two words per accumulator -- six
 *  VALU where the shift-or gather takes about twenty */
__device__ __forceinline__ uint32_t mask16_dot(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3) {
  const uint32_t a0 = __builtin_amdgcn_udot4(h0, 0x08040201u, 0u, false);
  const uint32_t a = __builtin_amdgcn_udot4(h1, 0x80402010u, a0, false);
  const uint32_t b0 = __builtin_amdgcn_udot4(h2, 0x08040201u, 0u, false);
  const uint32_t b = __builtin_amdgcn_udot4(h3, 0x80402010u, b0, false);
  return (a >> 7) | (b << 1);  // b = 128 x (bits 8..15): << 1 puts them at 8
}

/*! \brief the byte classes of a 16-byte slice the CSV walk needs: eol (\\n,
 *  \\r and NUL: past the chunk), the delimiter, and control bytes other than
 *  \\t \\n \\r (NUL included) -- each byte test once, in the byte-flag form,
 *  and one 16-bit gather per class */
struct Classes {
  uint32_t eol, delim, ctl;
};
__device__ __forceinline__ Classes classify16(uint4 g, uint32_t delim4) {
  const uint32_t w[4] = {g.x, g.y, g.z, g.w};
  uint32_t he[4], hd[4], hc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t n = hb_eq(w[k], 0x0A0A0A0Au), r = hb_eq(w[k], 0x0D0D0D0Du);
    const uint32_t z = hb_eq(w[k], 0u), t = hb_eq(w[k], 0x09090909u);
    he[k] = n | r | z;
    hd[k] = hb_eq(w[k], delim4);
    hc[k] = hb_lt20(w[k]) & ~(t | n | r);
  }
  Classes c;
  c.eol = mask16(he[0], he[1], he[2], he[3]);
  c.delim = mask16(hd[0], hd[1], hd[2], hd[3]);
  c.ctl = mask16(hc[0], hc[1], hc[2], hc[3]);
  return c;
}

/*! \brief 16 bytes of the chunk at pos, zero past its end (the buffer is 16-byte padded) */
__device__ __forceinline__ uint4 load16_clip(const uint8_t* __restrict__ text, size_t pos, size_t n) {
  const uint4 v = *reinterpret_cast<const uint4*>(text + (pos < n ? pos : 0));
  const uint32_t keep = pos < n ? static_cast<uint32_t>(n - pos < 16 ? n - pos : 16) : 0u;
  const uint64_t m_lo = keep >= 8 ? ~0ull : ((1ull << (8 * keep)) - 1ull);
  const uint64_t m_hi = keep >= 16 ? ~0ull : (keep <= 8 ? 0ull : ((1ull << (8 * (keep - 8))) - 1ull));
  return make_uint4(v.x & static_cast<uint32_t>(m_lo), v.y & static_cast<uint32_t>(m_lo >> 32),
                    v.z & static_cast<uint32_t>(m_hi), v.w & static_cast<uint32_t>(m_hi >> 32));
}

/*! \brief wave-uniform state of a tile walk */
struct Walk {
  uint32_t carry_eol, carry_delim;  // last byte of the previous step
  uint32_t col_carry;               // fields since the last row start
  uint32_t rows, fields, excl;      // owned so far
  uint32_t pre;                     // field starts of the tile before its first row start
  bool started, done, bad;
};

/*! \brief one lane's 16 bytes of a step after the wave scans */
struct Slice {
  uint32_t fm, lm;  // owned field starts / row starts (bit k = byte k)
  uint32_t col0;    // column of the first field when no row start precedes it in the slice
  uint64_t before;  // packed fields | rows << 21 | excluded << 42 of the earlier lanes
  uint64_t total;   // the same for the whole step
};

__device__ __forceinline__ bool excluded(uint32_t col, const CsvCfg& cfg) {
  return static_cast<int>(col) == cfg.label_col || static_cast<int>(col) == cfg.weight_col;
}

constexpr int kExclNone = 0;  // no label / weight column
constexpr int kExclRows = 1;  // label / weight only in column 0: counted per row
constexpr int kExclCols = 2;  // columns needed (per-field column numbers)
// the fill's walk when only column 0 can be excluded: the column scan for the
// listing, the excluded fields counted per row start (no per-field loop)
constexpr int kExclRowsCols = 3;

__device__ __forceinline__ void col_scan(const CsvCfg& cfg, bool count, int lane, Walk* w,
                                         Slice* o, uint32_t* nx);

/*!
 * \brief masks, ownership and scans of step `s` (g: the lane's 16 bytes at
 *  tile offset s * kStep + 16 * lane; nrem: chunk bytes from the tile start,
 *  capped at 4 GiB).  Updates the walk state (all lanes see the same values).
 */
__device__ __forceinline__ Slice step_slice(uint4 g, uint32_t s, uint32_t nrem, const CsvCfg& cfg,
                                            int excl_mode, Walk* w, int lane,
                                            const uint32_t* pub = nullptr) {
  uint32_t e, d;
  bool bad = false;
  if (pub != nullptr) {
    // S1p's published masks (line ends | delimiters << 16); it checked the
    // control bytes of the whole tile
    e = *pub & 0xFFFFu;
    d = *pub >> 16;
  } else {
    const uint32_t p = s * kStep + 16u * lane;
    const Classes cls = classify16(g, cfg.delim * 0x01010101u);
    e = cls.eol;  // NUL: past the chunk
    d = cls.delim;
    // control bytes, and NULs inside the chunk, are text to the reference
    const uint32_t inside = p >= nrem ? 0u : (nrem - p >= 16 ? 0xFFFFu : (1u << (nrem - p)) - 1u);
    bad = (cls.ctl & inside) != 0;
  }
  const uint32_t last_e = (e >> 15) & 1u, last_d = (d >> 15) & 1u;
  const uint32_t up_e = lane_shr1(last_e);
  const uint32_t up_d = lane_shr1(last_d);
  const uint32_t pe = lane == 0 ? w->carry_eol : up_e;
  const uint32_t pd = lane == 0 ? w->carry_delim : up_d;
  uint32_t lm = ~e & ((e << 1) | pe) & 0xFFFFu;
  // a delimiter opens a field unless the line (or the chunk) ends right after
  // it: no empty last field for a trailing delimiter (reference csv_parser.h:83-96)
  uint32_t fm = lm | (((d << 1) | pd) & ~e & 0xFFFFu);
  w->carry_eol = lane63(last_e);
  w->carry_delim = lane63(last_d);
  // ownership: from the first row start in the tile to the first one after it
  uint32_t own = 0xFFFFu;
  const bool was_started = w->started;
  const uint64_t any_ls = __ballot(lm != 0);
  const int first_lane = any_ls != 0 ? __builtin_ctzll(any_ls) : 0;
  const uint32_t first_lm = __builtin_amdgcn_readlane(lm, first_lane);  // (first_lane: uniform)
  const uint32_t first_bit = first_lm & (0u - first_lm);
  if (s < kTileSteps) {
    if (!w->started) {
      if (any_ls == 0) {
        own = 0;
      } else {
        own = lane < first_lane ? 0u : (lane == first_lane ? (~(first_bit - 1u) & 0xFFFFu) : 0xFFFFu);
        w->started = true;
      }
    }
    if (s + 1 == kTileSteps && !w->started) w->done = true;  // no row starts in this tile
  } else {
    if (!w->started) {
      own = 0;
      w->done = true;
    } else if (any_ls != 0) {
      own = lane < first_lane ? 0xFFFFu : (lane == first_lane ? first_bit - 1u : 0u);
      w->done = true;  // the next tile's first row
    }
  }
  if (s * kStep + kStep >= nrem) w->done = true;  // the chunk ends in this step
  // (S1p) the tile's field starts before its first row start: the rest of
  // the previous tile's last row (wave-uniform: only until the walk starts)
  if (s < kTileSteps && !was_started) w->pre += wave_sum(static_cast<uint32_t>(__popc(fm & ~own)));
  fm &= own;
  lm &= own;
  w->bad |= __any(bad && own != 0);
  Slice o;
  o.fm = fm;
  o.lm = lm;
  uint32_t nx = 0;  // excluded columns among the lane's fields
  if (excl_mode == kExclNone || excl_mode == kExclRows) {
    // label / weight only in column 0 (or none): one excluded field per row,
    // no columns needed (the count pass of the common `label_column=0`)
    nx = static_cast<uint32_t>(__popc(lm)) * static_cast<uint32_t>(cfg.zero_excl);
    o.col0 = 0;
  } else {
    col_scan(cfg, excl_mode == kExclCols, lane, w, &o, &nx);
    if (excl_mode == kExclRowsCols) {
      nx = static_cast<uint32_t>(__popc(lm)) * static_cast<uint32_t>(cfg.zero_excl);
    }
  }
  // fields / rows (<= 1024 each per step: 16-bit halves) and excluded
  // columns: two DPP scans, repacked to the 21-bit layout of f21
  const uint64_t packed = static_cast<uint64_t>(__popc(fm)) |
                          (static_cast<uint64_t>(__popc(lm)) << 16) |
                          (static_cast<uint64_t>(nx) << 32);
  uint64_t tot;
  const uint64_t bef = wave_excl_scan_2x32(packed, &tot);
  auto repack = [](uint64_t v) {
    return (v & 0xFFFFull) | (((v >> 16) & 0xFFFFull) << 21) | ((v >> 32) << 42);
  };
  o.before = repack(bef);
  o.total = repack(tot);
  return o;
}

/*! \brief column of each lane's first field (segmented scan, reset at row
 *  starts) and, with count, the excluded columns among its fields */
__device__ __forceinline__ void col_scan(const CsvCfg& cfg, bool count, int lane, Walk* w,
                                         Slice* o, uint32_t* nx) {
  const uint32_t fm = o->fm, lm = o->lm;
  uint32_t x;
  if (lm != 0) {
    const uint32_t hi = 31u - __builtin_clz(lm);
    x = static_cast<uint32_t>(__popc(fm >> hi)) | 0x80000000u;
  } else {
    x = static_cast<uint32_t>(__popc(fm));
  }
  // segmented sum (bit 31: a row starts in this lane), DPP ladder
  x = wave_incl_scan_op(x, [](uint32_t y, uint32_t v) {
    return (v & 0x80000000u) ? v : ((v + (y & 0x7FFFFFFFu)) | (y & 0x80000000u));
  });
  const uint32_t prev = lane_shr1(x);
  const uint32_t last = lane63(x);
  o->col0 = lane == 0 ? w->col_carry
                      : (prev & 0x7FFFFFFFu) + ((prev & 0x80000000u) ? 0u : w->col_carry);
  w->col_carry = (last & 0x7FFFFFFFu) + ((last & 0x80000000u) ? 0u : w->col_carry);
  if (count) {
    uint32_t col = o->col0;
    for (uint32_t m = fm; m != 0; m &= m - 1) {
      const uint32_t b = static_cast<uint32_t>(__builtin_ctz(m));
      if ((lm >> b) & 1u) col = 0;
      *nx += excluded(col, cfg) ? 1u : 0u;
      ++col;
    }
  }
}

__device__ __forceinline__ uint32_t f21(uint64_t v, int k) {
  return static_cast<uint32_t>((v >> (21 * k)) & 0x1FFFFFull);
}

__global__ __launch_bounds__(kThreads) void k_csv_tile_count(const uint8_t* __restrict__ text,
                                                             size_t n, size_t ntiles, CsvCfg cfg,
                                                             uint64_t* __restrict__ counts,
                                                             uint32_t* __restrict__ flags) {
  const int lane = lane_id();
  const size_t tile = static_cast<size_t>(blockIdx.x) * kWaves + threadIdx.x / kWave;
  if (tile >= ntiles) return;  // whole waves leave; nothing below synchronises waves
  const size_t tile0 = tile * kTileBytes;
  const uint32_t nrem = static_cast<uint32_t>(n - tile0 < 0xFFFFFFFFull ? n - tile0 : 0xFFFFFFFFull);
  Walk w{};
  w.carry_eol = 1u;
  if (tile0 != 0) {
    const uint32_t c = text[tile0 - 1];
    w.carry_eol = (c == '\n' || c == '\r') ? 1u : 0u;
  }
  const int excl_mode = (cfg.label_col > 0 || cfg.weight_col > 0) ? kExclCols
                        : (cfg.zero_excl != 0 ? kExclRows : kExclNone);
  bool over = false;
  uint4 g = load16_clip(text, tile0 + 16u * lane, n);
  for (uint32_t s = 0; s < kMaxSteps; ++s) {
    const uint4 nxt = load16_clip(text, tile0 + (s + 1) * kStep + 16u * lane, n);  // prefetch
    const Slice sl = step_slice(g, s, nrem, cfg, excl_mode, &w, lane);
    over |= f21(sl.total, 0) > kListCap;
    w.fields += f21(sl.total, 0);
    w.rows += f21(sl.total, 1);
    w.excl += f21(sl.total, 2);
    if (w.done) break;
    g = nxt;
  }
  // rows run past the extension while the chunk goes on: exact kernels
  const bool irregular = w.bad || over || (!w.done && tile0 + kTileBytes + kExt < n);
  if (lane == 0) {
    counts[tile] = (static_cast<uint64_t>(w.rows) << 32) | (w.fields - w.excl);
    flags[tile] = irregular ? kFlagIrregular : 0u;
  }
}

/*!
 * \brief S1p: positional tile counts -- the row starts and entries whose
 *  first byte lies in the tile (not the rows the tile owns), for a label /
 *  weight column of at most 0 (one excluded field per row, no columns
 *  needed).  A wave reads its 8 KiB with all 8 loads in flight and tests only
 *  line ends and delimiters: no ownership walk, no scans, no extension.  The
 *  fill adds the field starts before its first row start (Walk::pre) and
 *  flags what S1 flagged (control bytes, > kListCap fields per step, rows
 *  past the extension) itself, so a chunk is checked once.
 */
__global__ __launch_bounds__(kThreads) void k_csv_tile_count_pos(const uint8_t* __restrict__ text,
                                                                 size_t n, size_t ntiles,
                                                                 CsvCfg cfg,
                                                                 uint64_t* __restrict__ counts,
                                                                 uint32_t* __restrict__ flags,
                                                                 uint32_t* __restrict__ masks) {
  constexpr int kLoads = static_cast<int>(kTileBytes / 1024);
  const int lane = lane_id();
  const size_t tile = static_cast<size_t>(blockIdx.x) * kWaves + threadIdx.x / kWave;
  if (tile >= ntiles) return;  // whole waves leave; nothing below synchronises waves
  const size_t tile0 = tile * kTileBytes;
  uint4 v[kLoads];
#pragma unroll
  for (int j = 0; j < kLoads; ++j) v[j] = load16_clip(text, tile0 + j * 1024 + 16u * lane, n);
  uint32_t pe = 1u, pd = 0u;  // the byte before the tile: a line end / delimiter
  if (tile0 != 0) {
    const uint32_t c = text[tile0 - 1];
    pe = (c == '\n' || c == '\r') ? 1u : 0u;
    pd = c == cfg.delim ? 1u : 0u;
  }
  const uint32_t delim4 = cfg.delim * 0x01010101u;
  uint32_t rows = 0, fields = 0, ctl_any = 0;
  const bool full = tile0 + kTileBytes <= n;  // (else the bytes past n are no text)
  // full tiles (every tile but a chunk's last): no NUL-past-the-end test (a NUL
  // inside the text is a control byte: the chunk goes to the exact kernels)
  auto walk = [&](auto fullc) {
#pragma unroll
    for (int j = 0; j < kLoads; ++j) {
      const uint32_t w4[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
      uint32_t he[4], hd[4], hc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // line ends, and the zeros past the chunk (no field starts there)
        const uint32_t nl = hb_eq(w4[k], 0x0A0A0A0Au), cr = hb_eq(w4[k], 0x0D0D0D0Du);
        he[k] = decltype(fullc)::value ? (nl | cr) : (nl | cr | hb_eq(w4[k], 0u));
        hd[k] = hb_eq(w4[k], delim4);
        // control bytes other than \t \n \r (NUL included): text to the
        // reference, so the chunk goes to the exact kernels (the fill's check,
        // made here once for the whole tile)
        hc[k] = hb_lt20(w4[k]) & ~(hb_eq(w4[k], 0x09090909u) | nl | cr);
      }
      const uint32_t e = mask16_dot(he[0], he[1], he[2], he[3]);
      const uint32_t d = mask16_dot(hd[0], hd[1], hd[2], hd[3]);
      uint32_t c = hc[0] | hc[1] | hc[2] | hc[3];
      if (!decltype(fullc)::value) {  // only the chunk's last tile
        const size_t p = tile0 + j * 1024 + 16u * lane;
        c = p >= n ? 0u
                   : (n - p >= 16 ? c : mask16_dot(hc[0], hc[1], hc[2], hc[3]) & ((1u << (n - p)) - 1u));
      }
      ctl_any |= c;
      masks[(tile * kLoads + j) * kWave + lane] = e | (d << 16);
      const uint32_t last_e = (e >> 15) & 1u, last_d = (d >> 15) & 1u;
      // the byte before each lane's 16: lane - 1's last, lane 0 the previous load's lane 63
      const uint32_t up_e = lane_shr1(last_e), up_d = lane_shr1(last_d);
      const uint32_t le = lane == 0 ? pe : up_e, ld = lane == 0 ? pd : up_d;
      pe = lane63(last_e);
      pd = lane63(last_d);
      const uint32_t lm = ~e & ((e << 1) | le) & 0xFFFFu;
      const uint32_t fm = lm | (((d << 1) | ld) & ~e & 0xFFFFu);
      rows += static_cast<uint32_t>(__popc(lm));
      fields += static_cast<uint32_t>(__popc(fm));
    }
  };
  if (full) {
    walk(std::true_type{});
  } else {
    walk(std::false_type{});
  }
  const uint64_t c = wave_sum_2x32((static_cast<uint64_t>(rows) << 32) | fields);
  const bool any_ctl = __any(ctl_any != 0);
  if (lane == 0) {
    const uint32_t r = static_cast<uint32_t>(c >> 32);
    counts[tile] = (c & 0xFFFFFFFF00000000ull) |
                   (static_cast<uint32_t>(c) - r * static_cast<uint32_t>(cfg.zero_excl));
    flags[tile] = any_ctl ? kFlagIrregular : 0u;
  }
}

/*! \brief StrToFloat of the field at global position q (the generic path);
 *  returned by value -- an out-pointer into the caller's frame would put it on
 *  the stack (a scratch store + load per field round) */
struct GenericField {
  float v;
  bool last;
};
__device__ __noinline__ GenericField generic_field(const char* q, const char* end, char delim) {
  const char* fe = q;
  while (fe != end && *fe != delim && *fe != '\n' && *fe != '\r') ++fe;
  GenericField r;
  // the row's last field: EOL / chunk end, or a trailing delimiter before them
  r.last = fe == end || *fe != delim || fe + 1 == end || fe[1] == '\n' || fe[1] == '\r';
  while (q != fe && data::isspace(*q)) ++q;
  r.v = data::StrToFloat(q, fe, nullptr);
  return r;
}

// 6 waves per SIMD (the LDS allows 6 workgroups per CU): <= 84 VGPRs.
// kCol0: the common configuration compiled on its own -- positional counts
// (label column 0 or none), no weight column, no pricing experiments: the
// round loop loses the weight / short-row / experiment branches and the
// scalar registers they held (the general kernel sits at the SGPR limit)
template <typename IndexType, bool kCol0>
__global__ __launch_bounds__(kThreads)
__attribute__((amdgpu_waves_per_eu(6))) void k_csv_tile_fill(const uint8_t* __restrict__ text,
                                                            size_t n, size_t ntiles, CsvCfg cfg,
                                                            const uint64_t* __restrict__ prefix,
                                                            const uint32_t* __restrict__ masks,
                                                            FillTarget<IndexType> out,
                                                            MetaPartial* __restrict__ partials,
                                                            uint32_t exp_arg) {
  const uint32_t exp = kCol0 ? 0u : exp_arg;
  __shared__ uint4 s_ring[kWaves][kRingVecs];
  __shared__ uint2 s_list[kWaves][kListCap];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  const size_t tile = static_cast<size_t>(blockIdx.x) * kWaves + wave;
  if (tile >= ntiles) return;
  uint4* ring = s_ring[wave];
  uint2* list = s_list[wave];
  const size_t tile0 = tile * kTileBytes;
  const uint32_t nrem = static_cast<uint32_t>(n - tile0 < 0xFFFFFFFFull ? n - tile0 : 0xFFFFFFFFull);
  const uint64_t pre = prefix[tile];
  const uint64_t R = out.row_base + (pre >> 32);          // the tile's first row
  const uint64_t C = out.nnz_base + (pre & 0xffffffffull);  // and first entry
  // outputs addressed from the tile's first row / entry, rooms clamped to
  // int32 (a tile's rows and entries are < 2^16): 32-bit compares per field
  // and fewer live 64-bit scalars in the round loop
  auto room32 = [](uint64_t limit, uint64_t at) {
    return limit <= at ? 0 : (limit - at > 0x7FFFFFFFull ? 0x7FFFFFFF : static_cast<int32_t>(limit - at));
  };
  const int32_t row_room = room32(out.row_limit, R);
  const int32_t nnz_room = room32(out.nnz_limit, C);
  float* const lab_at = out.label + R;
  float* const wgt_at = out.weight + R;  // (used only with has_weight: allocated)
  uint64_t* const off_at = out.offset + R;
  IndexType* const idx_at = out.index + C;
  float* const val_at = out.value + C;
  Walk w{};
  w.carry_eol = 1u;
  if (tile0 != 0) {
    const uint32_t c = text[tile0 - 1];
    w.carry_eol = (c == '\n' || c == '\r') ? 1u : 0u;
    w.carry_delim = c == cfg.delim ? 1u : 0u;
  }
  const uint32_t delim = cfg.delim;
  const int fill_excl =
      (!kCol0 && (cfg.label_col > 0 || cfg.weight_col > 0)) ? kExclCols : kExclRowsCols;
  // kCol0: only a label in column 0 is excluded
  const bool zl = cfg.label_col == 0;
  auto excl_col = [&](uint32_t col) { return kCol0 ? (zl && col == 0) : excluded(col, cfg); };
  uint32_t mx = 0;  // the largest column index (< 2^16)
  // a field's "last in its row" matters only for short rows with a label /
  // weight column after it (wave-uniform: skipped for label_column <= 0)
  const bool need_last = !kCol0 && (cfg.label_col > 0 || cfg.has_weight);
  bool irregular = false, any_value = false;
  // slot 0 <- step 0 (+ mirror of its head past slot 1).  Step s + 1 is staged
  // during step s from `pv`, which was loaded during step s - 1 (the load
  // for step s + 2 then goes straight into `pv`: no copy of a load in flight,
  // so no wait right behind it); bytes past n are zeroed where staged
  {
    const uint4 v = load16_clip(text, tile0 + 16u * lane, n);
    ring[lane] = v;
    if (lane < 2) ring[2 * kStep / 16 + lane] = v;
  }
  const size_t at1 = tile0 + kStep + 16u * lane;
  uint4 pv = *reinterpret_cast<const uint4*>(text + (at1 + 16 <= n ? at1 : 0));
  // S1p published the line-end / delimiter masks of every 16 bytes: the walk
  // takes them instead of classifying the bytes again (buffer loads: steps
  // past the chunk's last tile read zeros)
  const bool pub = kCol0 || cfg.pos != 0;
  __amdgpu_buffer_rsrc_t mrs;
  uint32_t mk = 0;
  if (pub) {
    const size_t words = (ntiles - tile) * (kTileBytes / 16);
    mrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(masks) + tile * (kTileBytes / 16), 0,
                                            static_cast<uint32_t>(words * 4 > 0xFFFFFFF0ull
                                                                      ? 0xFFFFFFF0ull
                                                                      : words * 4),
                                            0x00020000);
    mk = __builtin_amdgcn_raw_buffer_load_b32(mrs, static_cast<uint32_t>(lane) * 4, 0, 0);
  }
  for (uint32_t s = 0; s < kMaxSteps; ++s) {
    const uint32_t slot = (s & 1u) * (kStep / 16);
    // stage step s + 1 in the other slot (its head mirrored when that is slot 0)
    if (s + 1 < kMaxSteps) {
      const size_t at = tile0 + (s + 1) * kStep + 16u * lane;
      const uint4 v = at + 16 <= n ? pv : load16_clip(text, at, n);
      const uint32_t nslot = ((s + 1) & 1u) * (kStep / 16);
      ring[nslot + lane] = v;
      if (nslot == 0 && lane < 2) ring[2 * kStep / 16 + lane] = v;
      if (s + 2 < kMaxSteps) {
        const size_t at2 = at + kStep;
        pv = *reinterpret_cast<const uint4*>(text + (at2 + 16 <= n ? at2 : 0));
      }
    }
    wave_sync();
    // the fill lists every field with its column: always the column scan
    const uint32_t mk_s = mk;
    if (pub && s + 1 < kMaxSteps) {
      mk = __builtin_amdgcn_raw_buffer_load_b32(mrs, static_cast<uint32_t>(lane) * 4,
                                                (s + 1) * kWave * 4, 0);
    }
    const Slice sl = step_slice(ring[slot + lane], s, nrem, cfg, fill_excl, &w, lane,
                                pub ? &mk_s : nullptr);
    // list the lane's fields: x = ring byte | row in tile << 16, y = column | entry in tile << 16
    {
      uint32_t col = sl.col0;
      uint32_t at = f21(sl.before, 0);
      uint32_t row = w.rows + f21(sl.before, 1);  // rows started before this lane, this tile
      uint32_t ent = (w.fields + f21(sl.before, 0)) - (w.excl + f21(sl.before, 2));
      for (uint32_t m = sl.fm; m != 0; m &= m - 1) {
        const uint32_t b = static_cast<uint32_t>(__builtin_ctz(m));
        if ((sl.lm >> b) & 1u) {
          col = 0;
          ++row;
        }
        if (at < kListCap) {
          list[at] = make_uint2((slot * 16u + 16u * lane + b) | ((row - 1u) << 16),
                                col | (ent << 16));
        }
        ++at;
        ent += excl_col(col) ? 0u : 1u;
        ++col;
      }
    }
    const uint32_t nf = f21(sl.total, 0);
    w.fields += nf;
    w.rows += f21(sl.total, 1);
    w.excl += f21(sl.total, 2);
    irregular |= nf > kListCap;
    wave_sync();
    // pricing experiments (DMLC_CSV_EXP, 0 in production): 4 skips the rounds
    const uint32_t nlist = (exp & 4u) ? 0u : (nf < kListCap ? nf : kListCap);
    for (uint32_t r0 = 0; r0 < nlist; r0 += kWave) {
      const uint32_t k = r0 + lane;
      if (k < nlist) {
        const uint2 en = list[k];
        const uint32_t off = en.x & 0xFFFFu;
        const uint32_t row_t = en.x >> 16;
        const uint32_t col = en.y & 0xFFFFu;
        const uint32_t ent = en.y >> 16;
        const uint8_t* rb = reinterpret_cast<const uint8_t*>(ring);
        // line end or the zeros past the chunk: one 64-bit shift of a bit set
        auto eol_c = [](uint32_t c) { return c <= 13u && ((0x2401u >> c) & 1u) != 0; };
        // a field ended by a delimiter is still the row's last one when the
        // line ends right after that delimiter (no empty trailing field):
        // single LDS byte reads (the ring mirrors slot 0's head past slot 1)
        const uint32_t c0 = rb[off];
        float v;
        bool last;
        if (exp & 1u) {  // pricing: no number decode
          v = static_cast<float>(c0);
          last = eol_c(rb[off + 8]);
        } else if (c0 == delim || eol_c(c0)) {
          v = 0.0f;  // empty field
          last = need_last && (c0 != delim || eol_c(rb[off + 1]));
        } else {
          // the 8-digit run decoder of the LibSVM fill (token_decode.h)
          const tok::Num x = tok::parse_num(ring, off);
          const bool t_eol = eol_c(x.term);
          const bool last_fast = need_last && (t_eol || eol_c(rb[x.end + 1]));
          if (x.ok_float && (x.term == delim || t_eol)) {
            v = x.fval;
            last = last_fast;
          } else {
            const size_t gpos = tile0 + s * kStep + (off - slot * 16u);
            const GenericField g = generic_field(reinterpret_cast<const char*>(text) + gpos,
                                                 reinterpret_cast<const char*>(text) + n,
                                                 static_cast<char>(delim));
            v = g.v;
            last = g.last;
          }
        }
        // S1p: the prefix counts entries by position; the tile's own start
        // after the rest of the previous tile's last row (e: entry in the tile)
        const uint32_t e = ent + (pub ? w.pre : 0u);
        if (exp & 2u) {  // pricing: no stores (a value sink the compiler keeps)
          mx = __float_as_uint(v) == 0x7FC00001u ? mx + 1 : mx;
        } else if (static_cast<int32_t>(row_t) >= row_room) {
          irregular = true;
        } else {
          if (static_cast<int>(col) == cfg.label_col) {
            lab_at[row_t] = v;
          } else if (!kCol0 && static_cast<int>(col) == cfg.weight_col) {
            wgt_at[row_t] = v;
          } else if (static_cast<int32_t>(e) < nnz_room) {
            uint32_t idx = col;
            if (kCol0) {
              idx -= zl ? 1u : 0u;  // col > 0 here when the label takes column 0
            } else {
              idx -= (cfg.label_col >= 0 && col > static_cast<uint32_t>(cfg.label_col)) ? 1u : 0u;
              idx -= (cfg.weight_col >= 0 && col > static_cast<uint32_t>(cfg.weight_col)) ? 1u : 0u;
            }
            idx_at[e] = static_cast<IndexType>(idx);
            val_at[e] = v;
            mx = idx > mx ? idx : mx;
            any_value = true;
          } else {
            irregular = true;
          }
          if (col == 0) {
            off_at[row_t] = C + e;
            if (cfg.label_col < 0) lab_at[row_t] = 0.0f;
          }
          if (!kCol0 && last) {
            // a short row: no label / weight field
            if (cfg.label_col >= 0 && col < static_cast<uint32_t>(cfg.label_col)) lab_at[row_t] = 0.0f;
            if (cfg.has_weight && (cfg.weight_col < 0 || col < static_cast<uint32_t>(cfg.weight_col))) {
              wgt_at[row_t] = 1.0f;
            }
          }
        }
      }
    }
    if (w.done) break;
    wave_sync();  // the next prefetch overwrites this step's slot
  }
  // rows run past the extension while the chunk goes on: exact kernels (S1
  // flags it too; S1p leaves it to the fill)
  if (!w.done && tile0 + kTileBytes + kExt < n) irregular = true;
  unsigned fl = 0;
  if (irregular || w.bad) fl |= kFlagIrregular;
  if (any_value) fl |= kFlagValue;
  if (!kCol0 && cfg.has_weight) fl |= kFlagWeight;
  const unsigned long long m = wave_max(static_cast<unsigned long long>(mx));
  fl = wave_or(fl);
  if (lane == 0) {
    MetaPartial p;
    p.max_index = m;
    p.max_field = 0;
    p.flags = fl;
    p.pad = 0;
    partials[tile] = p;
  }
}

CsvCfg MakeCfg(int label_column, int weight_column, char delimiter) {
  CsvCfg c;
  c.label_col = label_column < 0 ? -1 : label_column;
  // weight_column == label_column: the label takes the column (the reference
  // tests it first), rows still get weight 1.0
  c.weight_col = (weight_column < 0 || weight_column == label_column) ? -1 : weight_column;
  c.has_weight = weight_column >= 0 ? 1 : 0;
  c.zero_excl = (c.label_col == 0 ? 1 : 0) + (c.weight_col == 0 ? 1 : 0);
  c.delim = static_cast<uint8_t>(delimiter);
  // positional counts whenever no column numbers are needed
  // (DMLC_CSV_POSCOUNT=0: the owning-tile count S1 for every chunk)
  static const bool pos_ok = [] {
    const char* v = std::getenv("DMLC_CSV_POSCOUNT");
    return v == nullptr || std::atoi(v) != 0;
  }();
  c.pos = pos_ok && c.label_col <= 0 && c.weight_col <= 0 ? 1 : 0;
  return c;
}

}  // namespace

void LaunchCsvTileCount(const char* text, size_t nbytes, int label_column, int weight_column,
                        char delimiter, uint64_t* tile_counts, uint32_t* tile_flags,
                        uint32_t* tile_masks, hipStream_t stream) {
  const size_t ntiles = TileCount(nbytes);
  if (ntiles == 0) return;
  const CsvCfg cfg = MakeCfg(label_column, weight_column, delimiter);
  const dim3 grid((ntiles + kWaves - 1) / kWaves);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  if (cfg.pos) {
    CHECK(tile_masks != nullptr) << "LaunchCsvTileCount: positional counts publish tile_masks";
    hipLaunchKernelGGL(k_csv_tile_count_pos, grid, dim3(kThreads), 0, stream, t, nbytes, ntiles, cfg,
                       tile_counts, tile_flags, tile_masks);
  } else {
    hipLaunchKernelGGL(k_csv_tile_count, grid, dim3(kThreads), 0, stream, t, nbytes, ntiles, cfg,
                       tile_counts, tile_flags);
  }
}

template <typename IndexType>
void LaunchCsvTileFill(const char* text, size_t nbytes, int label_column, int weight_column,
                       char delimiter, const uint64_t* tile_prefix, const uint32_t* tile_masks,
                       const FillTarget<IndexType>& out, MetaPartial* partials,
                       hipStream_t stream) {
  const size_t ntiles = TileCount(nbytes);
  if (ntiles == 0) return;
  static const uint32_t exp = [] {
    const char* v = std::getenv("DMLC_CSV_EXP");
    return v != nullptr ? static_cast<uint32_t>(std::atoi(v)) : 0u;
  }();
  const CsvCfg cfg = MakeCfg(label_column, weight_column, delimiter);
  const dim3 grid((ntiles + kWaves - 1) / kWaves);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  if (cfg.pos && !cfg.has_weight && exp == 0) {
    hipLaunchKernelGGL((k_csv_tile_fill<IndexType, true>), grid, dim3(kThreads), 0, stream, t, nbytes,
                       ntiles, cfg, tile_prefix, tile_masks, out, partials, 0u);
  } else {
    hipLaunchKernelGGL((k_csv_tile_fill<IndexType, false>), grid, dim3(kThreads), 0, stream, t,
                       nbytes, ntiles, cfg, tile_prefix, tile_masks, out, partials, exp);
  }
}

template void LaunchCsvTileFill<uint32_t>(const char*, size_t, int, int, char, const uint64_t*,
                                          const uint32_t*, const FillTarget<uint32_t>&,
                                          MetaPartial*, hipStream_t);
template void LaunchCsvTileFill<uint64_t>(const char*, size_t, int, int, char, const uint64_t*,
                                          const uint32_t*, const FillTarget<uint64_t>&,
                                          MetaPartial*, hipStream_t);

}  // namespace gpu
}  // namespace dmlc
