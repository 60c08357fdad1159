/*!
 * \file src/gpu/tile_kernels.hip
 * \brief LDS-staged tile parser: the LibSVM / LibFM fast path in three launches
 *  and one host wait (mapped pinned memory) for the chunk sizes.
 *
 *  Every row of a regular chunk is one line whose first byte starts its label
 *  token, so with L(p) = line starts at or before byte p and T(p) = tokens
 *  before p, the CSR position of a token follows from two prefix counts:
 *      row(label token k of line l)   = l,        offset[l] = k - l
 *      nnz(feature token k of line l) = k - l - 1
 *  No per-line or per-token index arrays are materialised.
 *
 *  C1 k_tile_count (one wave per 8 KiB tile): SWAR byte masks of 16 B per
 *     lane, per tile (line starts << 32 | token starts) and an irregular bit (a
 *     line that starts with a blank, control bytes other than \t \n \r).
 *     Reads the chunk once.  A token that does not start with [0-9+-.] never
 *     passes the fill's register-window decoder; the fill (and the fused hash
 *     kernel) flags it irregular on that fallback path, at no fast-path cost.
 *  C2 k_tile_scan  (one 1024-lane workgroup): exclusive scan of the tile
 *     counts, OR of the flags; nlines / nrows / nnz / flags go to the
 *     ChunkMeta and to mapped pinned memory the host polls (no D2H copy).
 *  C3 k_tile_fill  (one wave per tile, no workgroup barrier): streams the tile
 *     in 2 KiB steps through two LDS slots (step s and s - 1) with the next
 *     step prefetched in registers, lists every token (staging offset, line
 *     start bit, tile line ordinal) in a wave-private LDS list, and decodes
 *     whole 64-token rounds only -- a step's remainder waits for the next
 *     step's rounds.  Lane i decodes token i from two aligned ds_read_b128 in
 *     registers (token_decode.h: integer fields with parse_int, values with
 *     parse_num; anything else through strtonum.h's ParsePair / ParseTriple
 *     from global memory, bit-identical to the CPU parser) and stores index /
 *     value / label / offset directly.  K8 (max index / field, flags) is a
 *     per-wave slot.
 *  (C2 and C4 become two-level -- many workgroups, then one -- above 8192
 *  tiles, i.e. for the 1 GiB passes over HBM-resident text.)
 *  C4 k_tile_finish (one workgroup): fold the slots into the ChunkMeta and
 *     write the chunk's closing row pointer.
 *  Traffic per chunk: text read twice (C1, C3) + the CSR written once.
 */
#include <dmlc/gpu/hip_utils.h>
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
constexpr int kThreads = 256;
constexpr int kSub = static_cast<int>(kTileBytes / 4096);  // 4 KiB sub-tiles per tile
constexpr unsigned kOffBits = 13;                            // tile offset < 8192
constexpr unsigned kMaxTileTokens = static_cast<unsigned>(kTileBytes / 2);
static_assert(kTileBytes == 8192, "entry packing assumes 8 KiB tiles");

/*! \brief the high bit of each byte of z (z & 0x80808080) as a 4-bit mask:
 *  one byte dot product (v_dot4_u32_u8, full rate), not the quarter-rate
 *  v_mul_lo_u32 of the multiply-gather */
__device__ __forceinline__ uint32_t gather_hi(uint32_t z) {
  return __builtin_amdgcn_udot4(z, 0x08040201u, 0u, false) >> 7;
}

/*!
 * \brief byte classes of 16 bytes, branch-free SWAR (no cross-byte carries):
 *  sep = byte <= 0x20, eol = sep with (byte & 6) != 0, ctl = byte < 0x20.
 *  On text whose control bytes are only \t \n \r (verified per chunk by
 *  k_tile_count through `ctl`), sep is exactly {' ', \t, \n, \r} and eol
 *  exactly {\n, \r}.
 */
__device__ __forceinline__ void classify16(uint4 v, uint32_t* sep, uint32_t* eol, uint32_t* ctl) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t s = 0, e = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = w[i];
    const uint32_t lo7 = x & 0x7F7F7F7Fu;
    const uint32_t le20 = ~((lo7 + 0x5F5F5F5Fu) | x) & 0x80808080u;    // <= 0x20
    const uint32_t lt20 = ~((lo7 + 0x60606060u) | x) & 0x80808080u;    // <  0x20
    const uint32_t b6 = ((x & 0x06060606u) + 0x7E7E7E7Eu) & 0x80808080u;  // (b & 6) != 0
    s |= gather_hi(le20) << (4 * i);
    e |= gather_hi(le20 & b6) << (4 * i);
    c |= gather_hi(lt20) << (4 * i);
  }
  *sep = s;
  *eol = e;
  *ctl = c;
}

/*! \brief bytes of v with bit 6 set (letters and the like: no number starts
 *  so), as a 16-bit mask -- the C1 test of letter-started tokens */
__device__ __forceinline__ uint32_t letter_mask(uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) m |= gather_hi((w[i] << 1) & 0x80808080u) << (4 * i);
  return m;
}

__device__ __forceinline__ bool num_start(uint32_t c) {
  return (c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.';
}

/*!
 * \brief line-start / token-start masks of the 16 bytes v at chunk offset pos;
 *  pc = the byte before pos ('\n' at 0).  Bytes at or past n are invalid.
 *  kCheck: also return true when the lane saw an irregular construct (a
 *  control byte other than \t \n \r, a line starting with a blank, a token
 *  starting outside [0-9+-.]).
 */
template <bool kCheck, bool kFull = false, bool kCheckTokens = true>
__device__ __forceinline__ bool lane_masks(uint4 v, uint32_t pc, size_t pos, size_t n,
                                           uint32_t* lm, uint32_t* tm) {
  uint32_t sep, eol, ctl;
  classify16(v, &sep, &eol, &ctl);
  const uint32_t prev_eol = (pc == '\n' || pc == '\r') ? 1u : 0u;
  const uint32_t prev_sep = (prev_eol || pc == ' ' || pc == '\t') ? 1u : 0u;
  uint32_t valid = 0xFFFFu;  // kFull: all 16 bytes are before n (no 64-bit compares)
  if (kFull) {
  } else if (pos >= n) {
    valid = 0;
  } else if (n - pos < 16) {
    valid = (1u << (n - pos)) - 1u;
  }
  *lm = ~eol & ((eol << 1) | prev_eol) & valid & 0xFFFFu;
  *tm = ~sep & ((sep << 1) | prev_sep) & valid & 0xFFFFu;
  if (!kCheck) return false;
  bool bad = (*lm & ~*tm) != 0;  // a line that starts with a blank
  uint32_t t = kCheckTokens ? *tm : 0u;  // (else: the decoder's fallback flags them)
  while (t != 0) {
    const int j = __ffs(t) - 1;
    t &= t - 1;
    bad |= !num_start(dev::vec_byte(v, j));
  }
  uint32_t c = ctl & valid;
  while (c != 0) {
    const int j = __ffs(c) - 1;
    c &= c - 1;
    bad |= !((0x2600u >> dev::vec_byte(v, j)) & 1u);  // only \t \n \r
  }
  return bad;
}

__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ text, size_t pos, size_t n) {
  // a 16 B load that starts before n stays inside n + kTextPadBytes
  if (pos < n) return *reinterpret_cast<const uint4*>(text + pos);
  return make_uint4(0, 0, 0, 0);
}

/*! \brief byte before `pos` of this lane: lane t-1's last byte, or memory for lane 0 */
__device__ __forceinline__ uint32_t prev_byte(const uint8_t* __restrict__ text, size_t pos,
                                              uint4 v) {
  const uint32_t from_left = dev::lane_shr1(v.w >> 24);
  if (dev::lane_id() != 0) return from_left;
  return pos == 0 ? static_cast<uint32_t>('\n') : text[pos - 1];
}

/*!
 * \brief C1 lane step: line / token starts of 16 bytes as per-byte high-bit
 *  masks (bit 7 of byte j), gathered into 16-bit masks by byte dot products
 *  and popcounted once per 16 bytes, plus the irregular checks of
 *  lane_masks<true>.  pc: the byte before the 16.
 */
template <bool kFull>
__device__ __forceinline__ bool count16(uint4 v, uint32_t pc, size_t pos, size_t n,
                                        uint32_t* lines, uint32_t* toks, uint32_t* qtoks,
                                        uint32_t* packed = nullptr) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  // the token / line start masks in the fill's form (bit j = byte j of the 16,
  // token starts in bits 0..15, line starts in 16..31): byte dot products
  // gather the per-byte high bits (0x80 = 128 x the weight), two words per
  // accumulator
  uint32_t acc_t[2] = {0u, 0u}, acc_l[2] = {0u, 0u};
  // bytes at or past n are "separators" (no starts there); kFull: the whole
  // tile lies before n (every tile but a chunk's last), no per-word masks
  const size_t room = kFull ? 16 : (pos >= n ? 0 : (n - pos < 16 ? n - pos : 16));
  uint32_t prev_sep = (pc <= 0x20u) ? 0x80u : 0u;  // sep bit of the byte before, at bit 7
  uint32_t prev_eol = (pc == '\n' || pc == '\r') ? 0x80u : 0u;
  bool bad = false;
  uint32_t blank = 0;  // line starts that are no token starts (a line starting with a blank)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = w[i];
    const uint32_t lo7 = x & 0x7F7F7F7Fu;
    const uint32_t le20 = ~((lo7 + 0x5F5F5F5Fu) | x) & 0x80808080u;
    const uint32_t lt20 = ~((lo7 + 0x60606060u) | x) & 0x80808080u;
    const uint32_t b6 = ((x & 0x06060606u) + 0x7E7E7E7Eu) & 0x80808080u;
    const int valid_bytes = static_cast<int>(room) - 4 * i;
    const uint32_t valid = valid_bytes >= 4 ? 0x80808080u
                           : (valid_bytes <= 0 ? 0u : (0x80808080u >> (8 * (4 - valid_bytes))));
    const uint32_t sep = le20 | (~valid & 0x80808080u);
    const uint32_t eol = le20 & b6;
    const uint32_t sep_before = (sep << 8) | prev_sep;
    const uint32_t eol_before = (eol << 8) | prev_eol;
    const uint32_t tm = ~sep & sep_before & 0x80808080u;
    const uint32_t lm = ~eol & eol_before & valid & 0x80808080u;
    // tokens starting with a letter (byte bit 6 set; digits, signs and '.'
    // have it clear) are no entries of the CSR: LibSVM `qid:` tokens, which
    // the fill decodes beside its list, or junk that sends the chunk to the
    // exact kernels.  Bit 6 of each byte, moved to bit 7: x << 1.
    *qtoks += __popc(tm & (x << 1));
    // the starts gathered into the 16-bit masks by byte dot products (0x80 =
    // 128 x the weight, two words per accumulator); the token / line counts
    // are their popcounts, once per 16 bytes
    const uint32_t wgt = (i & 1) ? 0x80402010u : 0x08040201u;
    acc_t[i >> 1] = __builtin_amdgcn_udot4(tm, wgt, acc_t[i >> 1], false);
    acc_l[i >> 1] = __builtin_amdgcn_udot4(lm, wgt, acc_l[i >> 1], false);
    blank |= lm & ~tm;
    // (token starts outside [0-9+-.] are flagged by the fill / hash kernels:
    // such a token never passes the register-window decoder, so the check
    // costs nothing on the fast path -- here it was ~40% of the count's VALU)
    // control bytes other than \t \n \r: rare (line ends), a short loop is cheaper
    // than three more byte tests per word (measured: 88.5 vs 103.5 us per call)
    uint32_t c = lt20 & valid;
    while (c != 0) {
      const int j = (__ffs(c) - 1) >> 3;
      c &= c - 1;
      bad |= !((0x2600u >> ((x >> (8 * j)) & 0xFFu)) & 1u);
    }
    prev_sep = (sep >> 24) & 0x80u;
    prev_eol = (eol >> 24) & 0x80u;
  }
  const uint32_t pt = (acc_t[0] >> 7) | (acc_t[1] << 1);  // token starts, bit j = byte j
  const uint32_t pl = (acc_l[0] >> 7) | (acc_l[1] << 1);  // line starts
  *toks += __popc(pt);
  *lines += __popc(pl);
  bad |= blank != 0;
  if (packed != nullptr) *packed = pt | (pl << 16);
  return bad;
}

/*! \brief line starts of 16 bytes (the lm of count16 alone); room: bytes before n */
template <bool kFull>
__device__ __forceinline__ uint32_t lines16(uint4 v, uint32_t pc, int room) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t prev_eol = (pc == '\n' || pc == '\r') ? 0x80u : 0u;
  uint32_t lines = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = w[i];
    const uint32_t lo7 = x & 0x7F7F7F7Fu;
    const uint32_t le20 = ~((lo7 + 0x5F5F5F5Fu) | x) & 0x80808080u;
    const uint32_t b6 = ((x & 0x06060606u) + 0x7E7E7E7Eu) & 0x80808080u;
    const uint32_t eol = le20 & b6;
    const int valid_bytes = room - 4 * i;
    const uint32_t valid = kFull || valid_bytes >= 4
                               ? 0x80808080u
                               : (valid_bytes <= 0 ? 0u : (0x80808080u >> (8 * (4 - valid_bytes))));
    lines += __popc(~eol & ((eol << 8) | prev_eol) & valid);
    prev_eol = (eol >> 24) & 0x80u;
  }
  return lines;
}

/*!
 * \brief decoupled look-back over per-tile line counts (one wave per tile):
 *  publish this tile's count, sum the predecessors' counts back to the first
 *  inclusive prefix (64 tiles per probe), publish the inclusive prefix, return
 *  the exclusive one.  Status word: tag (30 bits, one per launch, so the array
 *  needs no reset) << 34 | state (1: count, 2: inclusive) << 32 | value.
 *  Tiles run in ticket order (k_tile_hash), so every tile waited on is resident
 *  or done and the wait ends.
 */
__device__ __forceinline__ uint64_t lookback_lines(uint64_t* st, size_t tile, uint32_t own,
                                                   uint32_t tag, int lane) {
  const uint64_t tg = static_cast<uint64_t>(tag) << 34;
  if (lane == 0) {
    __hip_atomic_store(&st[tile], tg | ((tile == 0 ? 2ull : 1ull) << 32) | own, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tile == 0) return 0;
  uint64_t excl = 0;
  int64_t j = static_cast<int64_t>(tile) - 1;  // the nearest predecessor not summed yet
  for (;;) {
    const int64_t k = j - lane;
    const uint64_t v = k >= 0 ? __hip_atomic_load(&st[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : (tg | (2ull << 32));  // before the chunk: inclusive 0
    const uint32_t state = static_cast<uint32_t>(v >> 32) & 3u;
    const bool ready = (v >> 34) == tag && state != 0;
    const uint64_t inc = __ballot(ready && state == 2u);
    const uint64_t waiting = __ballot(!ready);
    const int first = inc != 0 ? __builtin_ctzll(inc) : dev::kWave - 1;
    const uint64_t need = first >= dev::kWave - 1 ? ~0ull : ((2ull << first) - 1ull);
    if ((waiting & need) != 0) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    excl += dev::wave_sum(lane <= first ? static_cast<uint32_t>(v) : 0u);
    if (inc != 0) break;
    j -= dev::kWave;
  }
  if (lane == 0) {
    __hip_atomic_store(&st[tile], tg | (2ull << 32) | (excl + own), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  return excl;
}

/*!
 * \brief C1: one wave per 8 KiB tile, 8 x 16 B loads per lane all in flight,
 *  wave-level reductions only (no LDS, no barrier).
 */
constexpr int kCountLoads = static_cast<int>(kTileBytes / 1024);
__global__ __launch_bounds__(kThreads) void k_tile_count(const uint8_t* __restrict__ text,
                                                         size_t n, size_t ntiles,
                                                         uint64_t* __restrict__ counts,
                                                         uint32_t* __restrict__ flags,
                                                         uint2* __restrict__ masks) {
  const int lane = dev::lane_id();
  const size_t tile = static_cast<size_t>(blockIdx.x) * (kThreads / dev::kWave) +
                      threadIdx.x / dev::kWave;
  if (tile >= ntiles) return;  // whole waves leave; no barrier below
  const size_t base = tile * kTileBytes;
  uint4 v[kCountLoads];
#pragma unroll
  for (int j = 0; j < kCountLoads; ++j) v[j] = load16(text, base + j * 1024 + lane * 16, n);
  const uint32_t first = base == 0 ? static_cast<uint32_t>('\n') : text[base - 1];
  uint32_t lines = 0, toks = 0, qtoks = 0;
  bool bad = false;
  // the fill's masks of slices 2 s and 2 s + 1 (its step s), one 8-byte store
  // per lane per step: [tile][step][lane]
  uint2* const mrow = masks + tile * (kTileBytes / 2048) * dev::kWave + lane;
  auto count_tile = [&](auto full) {
    uint32_t m0 = 0;
#pragma unroll
    for (int j = 0; j < kCountLoads; ++j) {
      const uint32_t left = dev::lane_shr1(v[j].w >> 24);
      const uint32_t wrap = j == 0 ? first : dev::lane63(v[j - 1].w >> 24);
      const uint32_t pc = lane == 0 ? wrap : left;
      uint32_t m;
      bad |= count16<decltype(full)::value>(v[j], pc, base + j * 1024 + lane * 16, n, &lines,
                                            &toks, &qtoks, &m);
      if (j & 1) {
        mrow[(j >> 1) * dev::kWave] = make_uint2(m0, m);
      } else {
        m0 = m;
      }
    }
  };
  if (base + kTileBytes <= n) {  // wave-uniform: every tile but a chunk's last
    count_tile(std::true_type{});
  } else {
    count_tile(std::false_type{});
  }
  lines = dev::wave_sum(lines);
  toks = dev::wave_sum(toks);
  qtoks = dev::wave_sum(qtoks);
  const bool any_bad = __any(bad);
  if (lane == 0) {
    // letter-started tokens (LibSVM `qid:`) are no CSR entries: out of the count
    counts[tile] = (static_cast<uint64_t>(lines) << 32) | (toks - qtoks);
    flags[tile] = (any_bad ? kFlagIrregular : 0u) | (qtoks != 0 ? kFlagQid : 0u);
  }
}

/*!
 * \brief copy the ChunkMeta to mapped pinned host memory, then raise its
 *  `pad` word (after a system-scope fence) so the host can poll for it
 *  instead of a blocking stream synchronise (DeviceParser::WaitMapped)
 */
__device__ __forceinline__ void publish_host_meta(ChunkMeta* host_meta, ChunkMeta m) {
  m.pad = 0;
  *host_meta = m;
  __threadfence_system();
  *reinterpret_cast<volatile unsigned*>(&host_meta->pad) = 1u;
}

constexpr int kScanThreads = 1024;
constexpr int kScanPer = 8;

/*! \brief exclusive scan of ntiles counts in place (one workgroup), meta totals */
__global__ __launch_bounds__(kScanThreads) void k_tile_scan(uint64_t* __restrict__ counts,
                                                            const uint32_t* __restrict__ flags,
                                                            size_t ntiles, ChunkMeta* meta,
                                                            ChunkMeta* host_meta, int raw) {
  __shared__ uint64_t swave[kScanThreads / 64];
  __shared__ uint32_t sflag[kScanThreads / 64];
  const int wid = threadIdx.x / dev::kWave;
  uint64_t carry = 0;
  uint32_t fl = 0;
  for (size_t t0 = 0; t0 < ntiles; t0 += static_cast<size_t>(kScanThreads) * kScanPer) {
    const size_t base = t0 + static_cast<size_t>(threadIdx.x) * kScanPer;
    uint64_t v[kScanPer];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
      v[i] = base + i < ntiles ? counts[base + i] : 0;
      if (base + i < ntiles) fl |= flags[base + i];
      s += v[i];
    }
    uint64_t wtot;
    const uint64_t wx = dev::wave_excl_scan(s, &wtot);
    if (dev::lane_id() == 0) swave[wid] = wtot;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
      const uint64_t t = swave[w];
      if (w < wid) before += t;
      all += t;
    }
    uint64_t x = carry + before + wx;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
      if (base + i < ntiles) counts[base + i] = x;
      x += v[i];
    }
    carry += all;
    __syncthreads();
  }
  fl = dev::wave_or(fl);
  if (dev::lane_id() == 0) sflag[wid] = fl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t f = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) f |= sflag[w];
    const uint64_t lines = carry >> 32, toks = carry & 0xffffffffull;
    // text: (lines << 32 | tokens); raw (RecordIO): (records << 32 | bytes)
    meta->nlines = lines;
    meta->nrows = lines;
    meta->nnz = raw ? toks : toks - lines;
    meta->max_index = 0;
    meta->max_field = 0;
    meta->flags = f;
    meta->pad = 0;
    if (host_meta != nullptr) publish_host_meta(host_meta, *meta);  // no D2H blit
  }
}

/*!
 * \brief two-level scan for large chunks (a 1 GiB HBM-resident pass has 131 K
 *  tiles; one workgroup reading them all is bound by a single CU's load path).
 *  Level 1: workgroup g scans tiles [4096 g, 4096 (g+1)) in place -- coalesced
 *  loads into LDS, a blocked 4-per-lane scan, coalesced stores -- and writes
 *  its total and flag OR.  Level 2 is k_tile_scan over the block totals (it
 *  also fills the ChunkMeta).  Level 3 adds each block's prefix to its tiles.
 */
constexpr int kScanBlockPer = 4;
constexpr size_t kScanBlockTiles = static_cast<size_t>(kScanThreads) * kScanBlockPer;
__global__ __launch_bounds__(kScanThreads) void k_tile_scan_local(uint64_t* __restrict__ counts,
                                                                  const uint32_t* __restrict__ flags,
                                                                  size_t ntiles,
                                                                  uint64_t* __restrict__ bsum,
                                                                  uint32_t* __restrict__ bflag) {
  __shared__ uint64_t sbuf[kScanBlockTiles];
  __shared__ uint64_t swave[kScanThreads / 64];
  __shared__ uint32_t sfl[kScanThreads / 64];
  const int wid = threadIdx.x / dev::kWave;
  const size_t t0 = static_cast<size_t>(blockIdx.x) * kScanBlockTiles;
  uint32_t fl = 0;
#pragma unroll
  for (int k = 0; k < kScanBlockPer; ++k) {
    const size_t idx = t0 + static_cast<size_t>(k) * kScanThreads + threadIdx.x;
    uint64_t c = 0;
    if (idx < ntiles) {
      c = counts[idx];
      fl |= flags[idx];
    }
    sbuf[k * kScanThreads + threadIdx.x] = c;
  }
  __syncthreads();
  uint64_t v[kScanBlockPer];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanBlockPer; ++i) {
    v[i] = sbuf[threadIdx.x * kScanBlockPer + i];
    s += v[i];
  }
  uint64_t wtot;
  const uint64_t wx = dev::wave_excl_scan(s, &wtot);
  fl = dev::wave_or(fl);
  if (dev::lane_id() == 0) {
    swave[wid] = wtot;
    sfl[wid] = fl;
  }
  __syncthreads();
  uint64_t before = 0, all = 0;
  uint32_t f = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) {
    const uint64_t t = swave[w];
    if (w < wid) before += t;
    all += t;
    f |= sfl[w];
  }
  uint64_t x = before + wx;
#pragma unroll
  for (int i = 0; i < kScanBlockPer; ++i) {  // each lane rewrites only its own 4 entries
    sbuf[threadIdx.x * kScanBlockPer + i] = x;
    x += v[i];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScanBlockPer; ++k) {
    const size_t idx = t0 + static_cast<size_t>(k) * kScanThreads + threadIdx.x;
    if (idx < ntiles) counts[idx] = sbuf[k * kScanThreads + threadIdx.x];
  }
  if (threadIdx.x == 0) {
    bsum[blockIdx.x] = all;
    bflag[blockIdx.x] = f;
  }
}

__global__ __launch_bounds__(kThreads) void k_tile_scan_add(uint64_t* __restrict__ counts,
                                                            size_t ntiles,
                                                            const uint64_t* __restrict__ bprefix) {
  const size_t t = static_cast<size_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (t < ntiles) counts[t] += bprefix[t / kScanBlockTiles];
}

/*!
 * \brief byte iterator whose end is "the next separator" (blank / EOL) or a
 *  hard limit.  strtonum.h's ParsePair / ParseTriple compare against an end
 *  iterator; a `sentinel` end makes them stop at the token's own end without
 *  knowing its length, so a token is parsed with one pass of byte loads
 *  (ds_read_u8 from the LDS tile, or global loads for the last token of a
 *  tile) instead of locating its end first.
 */
template <typename Ptr>
struct SepIter {
  Ptr p;
  Ptr limit;
  bool sentinel;
  __device__ __forceinline__ char operator*() const { return static_cast<char>(*p); }
  __device__ __forceinline__ SepIter& operator++() {
    ++p;
    return *this;
  }
  __device__ __forceinline__ bool at_end() const {
    if (p >= limit) return true;
    const uint8_t c = *p;
    return c == ' ' || c == '\t' || c == '\n' || c == '\r';
  }
  __device__ __forceinline__ bool operator!=(const SepIter& o) const {
    return o.sentinel ? !at_end() : p != o.p;
  }
  __device__ __forceinline__ bool operator==(const SepIter& o) const { return !(*this != o); }
};

template <typename Ptr>
__device__ __forceinline__ SepIter<Ptr> sep_begin(Ptr p, Ptr limit) {
  return SepIter<Ptr>{p, limit, false};
}
template <typename Ptr>
__device__ __forceinline__ SepIter<Ptr> sep_end(Ptr limit) {
  return SepIter<Ptr>{limit, limit, true};
}

/*!
 * \brief generic (strtonum.h ParsePair / ParseTriple) parse of the token at
 *  global offset gpos: tokens the register-window decoder does not cover.
 *  Out of line: it is rare, and inlined it would raise the register
 *  allocation of the whole fill kernel.
 */
struct GenericResult {
  tok::Token t;
  bool bad;
};

template <TextFormat F, typename IndexType>
__device__ __noinline__ GenericResult generic_token(const uint8_t* __restrict__ text, size_t n,
                                                    size_t gpos, bool is_label) {
  GenericResult res;
  tok::Token* const t = &res.t;
  bool* const bad = &res.bad;
  t->u0 = t->u1 = t->u0_hi = t->u1_hi = 0;
  t->f0 = t->f1 = 0.0f;
  const uint8_t* lim = text + n;
  auto beg = sep_begin(text + gpos, lim);
  auto end = sep_end(lim);
  float f0 = 0.0f, f1 = 0.0f;
  *bad = false;
  if (is_label) {
    t->r = data::ParsePair<float, float>(beg, end, &f0, &f1, bad);
    t->f0 = f0;
    t->f1 = f1;
  } else if constexpr (F == TextFormat::kLibSVM) {
    IndexType idx = 0;
    t->r = data::ParsePair<IndexType, float>(beg, end, &idx, &f0, bad);
    t->u0 = static_cast<uint32_t>(idx);
    t->u0_hi = static_cast<uint32_t>(static_cast<uint64_t>(idx) >> 32);
    t->f0 = f0;
  } else {
    IndexType fid = 0, idx = 0;
    t->r = data::ParseTriple<IndexType, IndexType, float>(beg, end, &fid, &idx, &f0, bad);
    t->u0 = static_cast<uint32_t>(fid);
    t->u0_hi = static_cast<uint32_t>(static_cast<uint64_t>(fid) >> 32);
    t->u1 = static_cast<uint32_t>(idx);
    t->u1_hi = static_cast<uint32_t>(static_cast<uint64_t>(idx) >> 32);
    t->f0 = f0;
  }
  return res;
}

/*!
 * \brief a letter-started token at chunk offset gp: true when it is the
 *  row's `qid:` token -- the second token of its line (only blanks and one
 *  token, the label, between the line start and it) spelled `qid:` + integer
 *  (the CPU parser's grammar, src/data/libsvm_parser.h) -- and *qid its
 *  value.  Anything else is for the exact kernels.  Rare path: byte loads from
 *  global memory (L2-resident text).
 */
struct QidResult {
  uint64_t value;
  bool ok;
};

__device__ __noinline__ QidResult qid_token(const uint8_t* __restrict__ text, size_t n, size_t gp) {
  QidResult r{0, false};
  auto blank = [](uint32_t c) { return c == ' ' || c == '\t'; };
  auto eol = [](uint32_t c) { return c == '\n' || c == '\r'; };
  if (gp + 4 > n || text[gp] != 'q' || text[gp + 1] != 'i' || text[gp + 2] != 'd' ||
      text[gp + 3] != ':') {
    return r;
  }
  // backward: blanks, then the label token, then the line start
  size_t p = gp;
  while (p > 0 && blank(text[p - 1])) --p;
  if (p == 0 || p == gp || eol(text[p - 1])) return r;  // no label before it
  while (p > 0 && !blank(text[p - 1]) && !eol(text[p - 1])) --p;
  if (p != 0 && !eol(text[p - 1])) return r;  // another token before the label
  // the value: StrToInt<int64_t> over the token's bytes after "qid:"
  size_t q = gp + 4;
  bool neg = false;
  if (q < n && (text[q] == '-' || text[q] == '+')) {
    neg = text[q] == '-';
    ++q;
  }
  uint64_t v = 0;
  for (int k = 0; k < 20 && q < n && text[q] >= '0' && text[q] <= '9'; ++k, ++q) {
    v = v * 10 + (text[q] - '0');
  }
  if (q < n && !blank(text[q]) && !eol(text[q])) return r;  // junk after the digits
  r.value = neg ? 0 - v : v;
  r.ok = true;
  return r;
}

/*!
 * \brief the `qid:` token at staged LDS byte a (the 32 bytes from a are
 *  staged: a step slot holds 64 bytes past the step), same grammar as
 *  qid_token; a zero byte (past the text end) ends the digits like the end of
 *  the text does.
 */
__device__ __forceinline__ QidResult qid_lds(const uint4* lds, uint32_t a) {
  QidResult r{0, false};
  const uint3 g = tok::ext12(lds, a);
  if (g.x != 0x3A646971u) return r;  // "qid:"
  const uint32_t c0 = g.y & 0xFFu;
  const bool neg = c0 == '-';
  const uint32_t s = (neg || c0 == '+') ? 1u : 0u;
  // the digits 8 at a time (digit_run8); 16 or more: the byte loop below
  const uint3 d1 = tok::ext12(lds, a + 4u + s);
  const tok::Run8 r1 = tok::digit_run8(d1.x, d1.y, d1.z & 0xFFu);
  uint64_t v = r1.val;
  uint32_t term = r1.term;
  if (r1.k == 8u) {
    const uint3 d2 = tok::ext12(lds, a + 12u + s);
    const tok::Run8 r2 = tok::digit_run8(d2.x, d2.y, d2.z & 0xFFu);
    if (r2.k == 8u) {
      // 16+ digits (StrToInt over up to 20, wrapping): byte by byte
      const uint4 g0 = tok::ext16(lds, a), g1 = tok::ext16(lds, a + 16);
      uint32_t i = 4u + s;
      v = 0;
      for (int k = 0; k < 20; ++k, ++i) {
        const uint32_t c = tok::win_byte(g0, g1, i);
        if (c - '0' > 9u) break;
        v = v * 10 + (c - '0');
      }
      term = tok::win_byte(g0, g1, i);
    } else {
      v = v * tok::pow10_u(r2.k) + r2.val;
      term = r2.term;
    }
  }
  if (term != ' ' && term != '\t' && term != '\n' && term != '\r' && term != 0) return r;
  r.value = neg ? 0 - v : v;
  r.ok = true;
  return r;
}

/*! \brief status of the last token start of a 16-byte slice: 0 none, 2 a token
 *  that does not start a line, 3 one that does (a label) */
__device__ __forceinline__ uint32_t slice_last(uint32_t tm, uint32_t lm) {
  return tm != 0 ? 2u | ((lm >> (31 - __builtin_clz(tm))) & 1u) : 0u;
}

/*!
 * \brief for a `qid:` token start: the status of the token start before it --
 *  a `qid:` is the line's second token iff that one starts the line (3).
 *  Slices of a step in text order are all lanes' a slices, then the b slices;
 *  `carried` is the status at the step start (0: no token yet in this tile,
 *  then the global-memory check decides).  Wave-uniform call.
 */
struct PrevTok {
  uint32_t a, b;
};
__device__ __forceinline__ PrevTok prev_token_status(uint32_t tm_a, uint32_t lm_a, uint32_t tm_b,
                                                     uint32_t lm_b, uint32_t carried, int lane) {
  // inclusive max over lanes <= lane: the DPP ladder (no LDS round trips)
  auto scan = [](uint32_t v) {
    return dev::wave_incl_scan_op(v, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
  };
  const uint32_t ia = scan(tm_a != 0 ? ((lane + 1u) << 2) | slice_last(tm_a, lm_a) : 0u);
  const uint32_t ib = scan(tm_b != 0 ? ((lane + 1u) << 2) | slice_last(tm_b, lm_b) : 0u);
  const uint32_t xa = dev::lane_shr1(ia), xb = dev::lane_shr1(ib);  // lane 0: 0
  const uint32_t ta = dev::lane63(ia);
  PrevTok r;
  r.a = xa != 0 ? (xa & 3u) : carried;
  r.b = xb != 0 ? (xb & 3u) : (ta != 0 ? (ta & 3u) : carried);
  return r;
}

/*! \brief the status after a step (its last token start's), or `carried` */
__device__ __forceinline__ uint32_t step_last_status(uint32_t tm_a, uint32_t lm_a, uint32_t tm_b,
                                                     uint32_t lm_b, uint32_t carried) {
  const uint64_t bb = __ballot(tm_b != 0), ba = __ballot(tm_a != 0);
  const uint32_t sb = __builtin_amdgcn_readlane(slice_last(tm_b, lm_b),
                                                bb ? 63 - __builtin_clzll(bb) : 0);
  const uint32_t sa = __builtin_amdgcn_readlane(slice_last(tm_a, lm_a),
                                                ba ? 63 - __builtin_clzll(ba) : 0);
  // wave-uniform: kept in a scalar register
  return __builtin_amdgcn_readfirstlane(bb ? sb : (ba ? sa : carried));
}

/*! \brief status of the token start before bit j of a slice, given the status
 *  before the slice */
__device__ __forceinline__ uint32_t status_before(uint32_t tm, uint32_t lm, uint32_t j,
                                                  uint32_t before_slice) {
  const uint32_t inside = tm & ((1u << j) - 1u);
  return inside != 0 ? slice_last(inside, lm) : before_slice;
}

/*!
 * \brief C3: wave-autonomous tile fill.  Each wave of the workgroup owns one
 *  8 KiB tile and never synchronises with the others (no __syncthreads):
 *   1. all 8 KiB (+ the 64 bytes after it) are loaded into registers at once;
 *   2. per 2 KiB step the step is staged in the wave's LDS region, the
 *      line / token start masks of each lane's two 16 B slices come from the
 *      same registers, and a wave scan (DPP) places each token's LDS offset
 *      (and its line-start bit) in a wave-private list, in text order;
 *   3. 64 list entries at a time, lane i decodes token i from the LDS text in
 *      registers (token_decode.h: two aligned ds_read_b128 per number), its
 *      line ordinal comes from a ballot of the line-start bits, and it writes
 *      index / value (consecutive lanes -> consecutive nnz slots) or label /
 *      offset / weight directly.
 *  Tokens the fast decoder does not take use the generic strtonum.h parser
 *  from global memory (bit-identical by construction).
 */
constexpr int kFillWaves = kThreads / 64;
constexpr uint32_t kDecodeCarry = 64;  // tokens a step may leave for the next one's rounds
#ifndef DMLC_FILL_WAVES
#define DMLC_FILL_WAVES 4  // measured best (profiles/r03_fill_ablation)
#endif
constexpr uint32_t kStepBytes = 2048;
constexpr int kSteps = static_cast<int>(kTileBytes / kStepBytes);
constexpr uint32_t kSlotBytes = kStepBytes + 64;           // a step + 64 B of the next
constexpr uint32_t kStageVecs = 2 * kSlotBytes / 16;       // two slots: step s and s - 1
constexpr uint32_t kListCap = kDecodeCarry + kStepBytes / 2;  // carried + a step's tokens
// deferred-token ring: < 64 left after a queue round + 128 from a pair round
constexpr uint32_t kQueueCap = 256;
// k_tile_hash: the tokens after a step's last whole round (< 64) are carried
// into the next step's rounds; their text moves with them into a 1 KiB carry
// area in front of the staged step (the window stays contiguous), so no step
// pays a mostly idle last round.  A step of more tokens than the list holds
// is listed in two halves.  LDS per workgroup at dim 1024: 4 x (3136 B text +
// 428 x 4 B list + 64 dummy slots) + 16 KiB rows: 4 workgroups per CU
constexpr uint32_t kHashListCap = 428;
constexpr uint32_t kHashCarry = 1024;  // carry area ahead of the staged step
constexpr uint32_t kHashText = kHashCarry + kSlotBytes;

/*!
 * \brief the 16 B at chunk offset pos, bytes at or past n zeroed (the
 *  decoder's end marker), without branches: lanes past n load from a clamped
 *  in-bounds address and mask everything
 */
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

/*! \brief a buffer resource over the text from base on (raw, gfx9 dword3):
 *  the address lives in scalar registers, loads take a 32-bit lane offset.
 *  The range check zeroes whole dwords past num_records, so the record count
 *  is the text rounded up to 16 bytes (every 16-byte load that starts inside
 *  the text returns all its bytes; text buffers carry kTextPadBytes of
 *  padding) and the caller zeroes the bytes past the text (clip16). */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t text_rsrc(const uint8_t* base, size_t avail) {
  const size_t up = (avail + 15) & ~static_cast<size_t>(15);
  const uint32_t nr = up > 0xFFFFFFF0ull ? 0xFFFFFFF0u : static_cast<uint32_t>(up);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, nr, 0x00020000);
}

/*! \brief the 16 bytes at byte voff of a text_rsrc (zeros past its records).
 *  The whole offset goes in voffset: the range check does not cover soffset */
__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}

typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

/*! \brief the published start masks from tile `tile` on (C1's [tile][step][lane]
 *  uint2 words), as a buffer resource: per step one 8-byte load whose lane
 *  offset is fixed and whose step offset is scalar (no address VALU) */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mask_rsrc(const uint32_t* masks, size_t tile,
                                                            size_t ntiles) {
  const size_t words = (ntiles - tile) * (kTileBytes / 16);
  const size_t bytes = words * 4 > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : words * 4;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(masks) + tile * (kTileBytes / 16),
                                           0, static_cast<uint32_t>(bytes), 0x00020000);
}

/*! \brief step s's two slice masks of this lane (x: slice a, y: slice b) */
__device__ __forceinline__ uint2 load_masks(__amdgpu_buffer_rsrc_t r, uint32_t lane_off, int s) {
  const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, lane_off, s * dev::kWave * 8, 0);
  return make_uint2(v.x, v.y);
}

__device__ __forceinline__ uint4 load16_clip(const uint8_t* __restrict__ text, size_t pos, size_t n) {
  const size_t at = pos < n ? pos : 0;
  const uint4 v = *reinterpret_cast<const uint4*>(text + at);
  const uint32_t keep = pos < n ? static_cast<uint32_t>(n - pos < 16 ? n - pos : 16) : 0u;
  // byte mask of the first `keep` bytes, per word
  const uint64_t m_lo = keep >= 8 ? ~0ull : ((1ull << (8 * keep)) - 1ull);
  const uint64_t m_hi = keep >= 16 ? ~0ull : (keep <= 8 ? 0ull : ((1ull << (8 * (keep - 8))) - 1ull));
  return make_uint4(v.x & static_cast<uint32_t>(m_lo), v.y & static_cast<uint32_t>(m_lo >> 32),
                    v.z & static_cast<uint32_t>(m_hi), v.w & static_cast<uint32_t>(m_hi >> 32));
}

/*! \brief v (the 16 bytes at pos) with the bytes at or past n zeroed */
__device__ __forceinline__ uint4 clip16(uint4 v, size_t pos, size_t n) {
  const uint32_t keep = pos < n ? static_cast<uint32_t>(n - pos < 16 ? n - pos : 16) : 0u;
  const uint64_t m_lo = keep >= 8 ? ~0ull : ((1ull << (8 * keep)) - 1ull);
  const uint64_t m_hi = keep >= 16 ? ~0ull : (keep <= 8 ? 0ull : ((1ull << (8 * (keep - 8))) - 1ull));
  return make_uint4(v.x & static_cast<uint32_t>(m_lo), v.y & static_cast<uint32_t>(m_lo >> 32),
                    v.z & static_cast<uint32_t>(m_hi), v.w & static_cast<uint32_t>(m_hi >> 32));
}

/*!
 * \brief append the token starts of one lane's 16 B slice to the wave's list
 *  (`at` = its first list position; `line0` = line starts of the tile before
 *  this slice).  An entry is  staging offset (13 bits: slot * kSlotBytes +
 *  byte in the step) | line start (bit 13) | line ordinal in the tile, this
 *  token's line included (bits 14..26), so a round can take the entries in
 *  any lane order and a token can be decoded a step after it was listed.
 *  The first two starts are written unconditionally -- a lane with fewer
 *  writes a private dummy slot past kListCap -- so the common case has no
 *  per-lane loop; slices with more starts (tokens shorter than 8 B) take the
 *  loop.
 */
__device__ __forceinline__ uint32_t list_entry(uint32_t tm_bit_j, uint32_t lm, uint32_t base,
                                               uint32_t line0) {
  const uint32_t j = tm_bit_j;
  const uint32_t upto = lm & ((2u << j) - 1u);  // line starts up to byte j of the slice
  return (base + j) | (((lm >> j) & 1u) << 13) | ((line0 + __popc(upto)) << 14);
}

template <uint32_t kCap = kListCap>
__device__ __forceinline__ void list_slice(uint32_t* sl, uint32_t tm, uint32_t lm, uint32_t at,
                                           uint32_t base, uint32_t line0, int lane) {
  uint32_t m = tm;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint32_t j = static_cast<uint32_t>(__builtin_ctz(m | 0x10000u));
    const bool has = m != 0;
    sl[has ? at : kCap + lane] = list_entry(j & 15u, lm, base, line0);  // (the list holds kCap + 64)
    at += has ? 1u : 0u;
    m &= m - 1;
  }
  if (__any(m != 0)) {
    for (; m != 0; m &= m - 1) {
      sl[at++] = list_entry(static_cast<uint32_t>(__builtin_ctz(m)), lm, base, line0);
    }
  }
}

/*!
 * \brief token slot of `lane` in a decode round: the four 16-lane groups of a
 *  ds_read_b128 ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32)
 *  take 16 consecutive tokens each, which start ~16 B apart -- distinct bank
 *  quads, where lane-ordered slots put tokens 256 B apart into one group
 */
__device__ __forceinline__ uint32_t round_slot(int lane) {
  // rank within its group + 16 * group, for lanes 0..31 (4 bits per entry)
  const uint32_t l = static_cast<uint32_t>(lane) & 31u;
  uint32_t k;
  if (l < 4) {
    k = l;
  } else if (l < 12) {
    k = 16u + (l - 4u);
  } else if (l < 16) {
    k = 4u + (l - 12u);
  } else if (l < 20) {
    k = 24u + (l - 16u);
  } else if (l < 28) {
    k = 8u + (l - 20u);
  } else {
    k = 28u + (l - 28u);
  }
  return (static_cast<uint32_t>(lane) & 32u) + k;
}

/*! \brief the one-pass fill's look-back state (kOnePass) */
struct FillPass {
  uint64_t* status;             // per-tile look-back words, zeroed before the launch
  unsigned long long* ticket;   // workgroup ticket counter
  unsigned long long ticket0;   // its value at this launch
  ChunkMeta* meta;              // nlines / nrows / nnz of the chunk (the last tile writes them)
  uint32_t exp;                 // pricing experiments (DMLC_FILL_EXP; 0 in production):
                                // 1 no CSR stores, 2 no token decode (outputs are wrong)
  const uint32_t* masks;        // counted path: C1's start masks (TileMaskWords)
};

/*! \brief the pricing experiments of a DMLC_FILL_PRICING build (scripts/
 *  fill_pricing.sh); a constant 0 otherwise, so production kernels hold no
 *  experiment flags in scalar registers (the fill is at the SGPR limit) */
__device__ __forceinline__ uint32_t fill_exp(const FillPass& op) {
#ifdef DMLC_FILL_PRICING
  return op.exp;
#else
  (void)op;
  return 0u;
#endif
}

// kLean: a target without qid / weight columns (the common case) compiled on
// its own -- no qid pass, no weight stores, one flag for "weights seen": the
// scalar registers those held are what the kernel spilled to VGPR lanes (it
// sits at the SGPR limit)
template <TextFormat F, typename IndexType, bool kOnePass, bool kLean = false>
__global__ __launch_bounds__(kThreads, DMLC_FILL_WAVES) void k_tile_fill(
    const uint8_t* __restrict__ text, size_t n, size_t ntiles, const uint64_t* __restrict__ prefix,
    FillTarget<IndexType> out, MetaPartial* __restrict__ partials, FillPass op) {
  __shared__ uint4 s_text[kFillWaves][kStageVecs];
  __shared__ uint32_t s_list[kFillWaves][kListCap + 64];  // + a dummy slot per lane
  __shared__ uint32_t s_dq[kFillWaves][kQueueCap];  // deferred tokens: list index ring
  // wave-uniform in a scalar register: the tile's buffer resource stays scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / dev::kWave);
  const int lane = dev::lane_id();
  size_t group = blockIdx.x;
  if constexpr (kOnePass) {
    // tiles in ticket order: a workgroup looks back only at tiles of
    // workgroups that started before it (whatever the dispatch order), so
    // every tile it waits on is resident or done
    __shared__ uint32_t s_ticket;
    if (threadIdx.x == 0) s_ticket = static_cast<uint32_t>(atomicAdd(op.ticket, 1ull) - op.ticket0);
    __syncthreads();
    group = s_ticket;
  }
  const size_t tile = group * kFillWaves + wave;
  if (tile >= ntiles) return;  // whole waves leave; nothing below synchronises waves
  uint4* const st = s_text[wave];
  uint32_t* const sl = s_list[wave];
  uint32_t* const dq = s_dq[wave];
  uint32_t qh = 0, qn = 0;  // queue head, queued tokens
  const uint32_t slot = round_slot(lane);
  const size_t tile0 = tile * kTileBytes;

  // ---- 1. the first step in flight.  Each step's loads go into the previous
  // step's registers once its masks are built (no register copies of loads
  // in flight, so no wait right behind the load), and the tail a step stages
  // -- the next step's first 64 B -- is loaded one step ahead in `t`.  Bytes
  // at or past n are zeroed where a step is staged (buffer loads past the
  // resource return zeros; clip16 handles the last partial dword).
  const __amdgpu_buffer_rsrc_t trs = text_rsrc(text + tile0, n - tile0);
  const uint32_t loff = static_cast<uint32_t>(lane) * 16;
  uint4 a = bload16(trs, loff);
  uint4 b = bload16(trs, loff + 1024);
  uint4 t = make_uint4(0, 0, 0, 0);
  if (!kOnePass && lane < 4) t = bload16(trs, loff + kStepBytes);
  // counted path: the step's start masks come from C1 (published per 16 B),
  // not from classifying the bytes again; one pass classifies here
  __amdgpu_buffer_rsrc_t mrs;
  const uint32_t moff = static_cast<uint32_t>(lane) * 8;
  uint2 mk = make_uint2(0, 0);
  if constexpr (!kOnePass) {
    mrs = mask_rsrc(op.masks, tile, ntiles);
    mk = load_masks(mrs, moff, 0);
  }
  uint32_t carry_pc = 0;
  if constexpr (kOnePass) carry_pc = tile0 == 0 ? static_cast<uint32_t>('\n') : text[tile0 - 1];
  uint64_t line_base, tok_base;
  unsigned count_flags = 0;  // one pass: what C1 would have flagged for this tile
  if constexpr (kOnePass) {
    // C1 in the fill: the tile's 8 KiB in flight at once (the steps below
    // re-read 2 KiB at a time, from L2), line / entry starts and the
    // irregular checks counted, then the look-back for the tiles before it
    uint4 v[kCountLoads];
    v[0] = a;
    v[1] = b;
#pragma unroll
    for (int j = 2; j < kCountLoads; ++j) v[j] = bload16(trs, loff + j * 1024);
    if (lane < 4) t = v[2];  // step 0's tail (the 64 B after it) is already here
    uint32_t lines = 0, toks = 0, qtoks = 0;
    bool bad = false;
    auto count_tile = [&](auto full) {
#pragma unroll
      for (int j = 0; j < kCountLoads; ++j) {
        const uint32_t left = dev::lane_shr1(v[j].w >> 24);
        const uint32_t wrap = j == 0 ? carry_pc : dev::lane63(v[j - 1].w >> 24);
        const uint32_t pc = lane == 0 ? wrap : left;
        bad |= count16<decltype(full)::value>(v[j], pc, tile0 + j * 1024 + lane * 16, n, &lines,
                                              &toks, &qtoks);
      }
    };
    if (tile0 + kTileBytes <= n) {  // wave-uniform: every tile but a chunk's last
      count_tile(std::true_type{});
    } else {
      count_tile(std::false_type{});
    }
    lines = dev::wave_sum(lines);
    const uint32_t ent = dev::wave_sum(toks - qtoks);  // letter tokens are no entries
    qtoks = dev::wave_sum(qtoks);
    count_flags = (__any(bad) ? kFlagIrregular : 0u) | (qtoks != 0 ? kFlagQid : 0u);
    const uint64_t own = (static_cast<uint64_t>(lines) << 31) | ent;
    // (lines, entries) as a 31 / 31-bit pair: a chunk is < 2 GiB, so both are
    // <= bytes / 2 and the packed sums never carry
    const uint64_t excl = dev::lookback_pairs<31>(op.status, tile, own, lane);
    line_base = excl >> 31;
    tok_base = excl & 0x7FFFFFFFull;
    if (tile + 1 == ntiles && lane == 0) {
      // the chunk's sizes (k_tile_finish, stream-ordered, adds the flags and
      // maxima, writes the closing row pointer and publishes the meta)
      ChunkMeta m;
      m.nlines = m.nrows = line_base + lines;
      m.nnz = tok_base + ent - (line_base + lines);
      m.max_index = m.max_field = 0;
      m.flags = 0;
      m.pad = 0;
      *op.meta = m;
    }
  } else {
    const uint64_t pre = prefix[tile];
    line_base = pre >> 32;
    tok_base = pre & 0xffffffffull;
  }
  // token k = tok_base + i of line l = line_base + lcnt - 1 goes to nnz
  // position C + (i - lcnt); its row is R + lcnt - 1 (as k_tile_scan defines)
  const uint64_t C = out.nnz_base + tok_base - line_base;
  const uint64_t R = out.row_base + line_base;
  // rooms clamped to int32 (a tile's ordinals are < 2^13): 32-bit compares per token
  auto clamp32 = [](int64_t v) {
    return static_cast<int32_t>(v > INT32_MAX ? INT32_MAX : (v < INT32_MIN ? INT32_MIN : v));
  };
  const int32_t nnz_room =
      clamp32(static_cast<int64_t>(out.nnz_limit) - static_cast<int64_t>(C));
  const int32_t row_room =
      clamp32(static_cast<int64_t>(out.row_limit) - static_cast<int64_t>(R));
  IndexType* const idx_at = out.index + C;
  float* const val_at = out.value + C;
  IndexType* const fld_at = out.field != nullptr ? out.field + C : nullptr;
  float* const lab_at = out.label + R - 1;
  uint64_t* const off_at = out.offset + R - 1;
  float* const wgt_at = !kLean && out.weight != nullptr ? out.weight + R - 1 : nullptr;
  uint64_t* const qid_at = !kLean && out.qid != nullptr ? out.qid + R - 1 : nullptr;
  // the count pass saw 'q' token starts in this chunk (the host then enables
  // the qid column): only such chunks look for `qid:` tokens
  const bool qid_chunk = !kLean && F == TextFormat::kLibSVM && out.qid != nullptr;

  uint32_t tok0 = 0;   // tile token ordinal of list position 0
  uint32_t lcnt = 0;   // line starts of this tile so far
  uint32_t carry = 0;  // list entries left for the next step's rounds (listed, not decoded)
  uint32_t qid_prev = 0;  // status of the last token start so far (prev_token_status)
  // maxima in the index width (32-bit compares for u32 indices)
  using MaxT = typename std::conditional<sizeof(IndexType) == 4, uint32_t, uint64_t>::type;
  MaxT mx_index = 0, mx_field = 0;
  bool any_value = false, any_weight = false, irregular = false, neg = false, need_w = false;
  bool over = false;
  uint32_t sink = 0;  // pricing experiments only

#pragma unroll 1
  for (int s = 0; s < kSteps; ++s) {
    const bool last = s + 1 == kSteps;
    const size_t pos_a = tile0 + s * kStepBytes + lane * 16;
    if (tile0 + static_cast<size_t>(s + 1) * kStepBytes + 64 > n) {  // wave-uniform: the text ends here
      a = clip16(a, pos_a, n);
      b = clip16(b, pos_a + 1024, n);
      t = clip16(t, pos_a + kStepBytes, n);
    }
    // ---- 2. stage the step (+ the next 64 B) in slot s & 1 -- the other slot
    // still holds step s - 1 for the tokens carried from it -- and list its tokens
    const uint32_t sbase = (static_cast<uint32_t>(s) & 1u) * kSlotBytes;
    uint4* const ss = st + sbase / 16;
    ss[lane] = a;
    ss[64 + lane] = b;
    if (lane < 4) ss[128 + lane] = t;
    uint32_t lm_a, tm_a, lm_b, tm_b;
    if constexpr (kOnePass) {
      const uint32_t left_a = dev::lane_shr1(a.w >> 24);
      const uint32_t pc_a = lane == 0 ? carry_pc : left_a;
      const uint32_t left_b = dev::lane_shr1(b.w >> 24);
      // cross-lane reads run in every lane (a shuffle inside `lane == 0 ? :`
      // would execute with only lane 0 active and read an inactive lane)
      const uint32_t last_a = dev::lane63(a.w >> 24);
      const uint32_t pc_b = lane == 0 ? last_a : left_b;
      carry_pc = dev::lane63(b.w >> 24);
      if (tile0 + static_cast<size_t>(s + 1) * kStepBytes <= n) {  // wave-uniform: a full step
        (void)lane_masks<false, true>(a, pc_a, pos_a, n, &lm_a, &tm_a);
        (void)lane_masks<false, true>(b, pc_b, pos_a + 1024, n, &lm_b, &tm_b);
      } else {
        (void)lane_masks<false>(a, pc_a, pos_a, n, &lm_a, &tm_a);
        (void)lane_masks<false>(b, pc_b, pos_a + 1024, n, &lm_b, &tm_b);
      }
    } else {
      // C1's masks: the same starts (its blank / control checks passed)
      tm_a = mk.x & 0xFFFFu;
      lm_a = mk.x >> 16;
      tm_b = mk.y & 0xFFFFu;
      lm_b = mk.y >> 16;
    }
    // `qid:` tokens (C1 left them out of the entry counts): taken out of the
    // list here, decoded by their lane after the scan (wave-uniform test:
    // only chunks that have them pay)
    uint32_t qa = 0, qb = 0;
    if (qid_chunk) {
      qa = tm_a & letter_mask(a);
      qb = tm_b & letter_mask(b);
      tm_a &= ~qa;
      tm_b &= ~qb;
    }
    // a, b, t (and the masks) are consumed: the next step's loads go straight into them
    if (!last) {
      const uint32_t so = static_cast<uint32_t>(s + 1) * kStepBytes;
      a = bload16(trs, loff + so);
      b = bload16(trs, loff + so + 1024);
      if (lane < 4) t = bload16(trs, loff + so + kStepBytes);
      if constexpr (!kOnePass) mk = load_masks(mrs, moff, s + 1);
    }
    // one 64-bit scan of four 16-bit counts: tokens / lines of both slices
    const uint64_t cnt = static_cast<uint64_t>(__popc(tm_a)) |
                         (static_cast<uint64_t>(__popc(tm_b)) << 16) |
                         (static_cast<uint64_t>(__popc(lm_a)) << 32) |
                         (static_cast<uint64_t>(__popc(lm_b)) << 48);
    uint64_t tot;
    const uint64_t before = dev::wave_excl_scan_2x32(cnt, &tot);  // 16-bit fields: no carries
    const uint32_t ntok_a = static_cast<uint32_t>(tot & 0xFFFFu);
    const uint32_t ntok = ntok_a + static_cast<uint32_t>((tot >> 16) & 0xFFFFu);
    const uint32_t nline_a = static_cast<uint32_t>((tot >> 32) & 0xFFFFu);
    const uint32_t nline = nline_a + static_cast<uint32_t>(tot >> 48);
    list_slice(sl, tm_a, lm_a, carry + static_cast<uint32_t>(before & 0xFFFFu), sbase + lane * 16,
               lcnt + static_cast<uint32_t>((before >> 32) & 0xFFFFu), lane);
    list_slice(sl, tm_b, lm_b, carry + ntok_a + static_cast<uint32_t>((before >> 16) & 0xFFFFu),
               sbase + 1024 + lane * 16, lcnt + nline_a + static_cast<uint32_t>(before >> 48), lane);
    dev::wave_sync();  // the staged text and the list are visible to every lane
    if (qid_chunk) {
      if (__any((qa | qb) != 0)) {
        const PrevTok pv = prev_token_status(tm_a | qa, lm_a, tm_b | qb, lm_b, qid_prev, lane);
        const uint32_t lbase[2] = {lcnt + static_cast<uint32_t>((before >> 32) & 0xFFFFu),
                                   lcnt + nline_a + static_cast<uint32_t>(before >> 48)};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          // token starts with the letter ones: a `qid:` after another letter
          // token is not the second token
          const uint32_t lmh = h == 0 ? lm_a : lm_b, tmh = h == 0 ? tm_a | qa : tm_b | qb;
          for (uint32_t m = h == 0 ? qa : qb; m != 0; m &= m - 1) {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctz(m));
            // its row: the tile's line starts up to this byte (a line that
            // starts with 'q' has no label: exact kernels)
            const uint32_t lc = lbase[h] + static_cast<uint32_t>(__popc(lmh & ((2u << j) - 1u)));
            // the second token of its line: the token start before it is the
            // line's label (from the masks; the tile's first token: global check)
            const uint32_t prev = status_before(tmh, lmh, j, h == 0 ? pv.a : pv.b);
            QidResult q{0, false};
            if (prev == 3u) {
              q = qid_lds(st, sbase + static_cast<uint32_t>(h) * 1024 + lane * 16 + j);
            } else if (prev == 0u) {
              q = qid_token(text, n, pos_a + static_cast<size_t>(h) * 1024 + j);
            }
            // (lc 0: the tile's first, unfinished line -- the row before R)
            const bool ok = q.ok && ((lmh >> j) & 1u) == 0 &&
                            static_cast<int32_t>(lc) - 1 < row_room && qid_at != nullptr;
            if (ok) qid_at[lc] = q.value;
            irregular |= !ok;
          }
        }
      }
      qid_prev = step_last_status(tm_a | qa, lm_a, tm_b | qb, lm_b, qid_prev);
    }

    // ---- 3. decode 64 listed tokens per round.  Only whole rounds run: the
    // rest of this step's tokens (< 64) wait for the next step's rounds, so a
    // step does not pay a mostly idle last round; every older token is
    // decoded now (its slot is restaged next step), and the last step takes all
    const uint32_t total = carry + ntok;
    const uint32_t rest = total % dev::kWave < ntok ? total % dev::kWave : ntok;
    const uint32_t ndec = last ? total : total - rest;
    // a decoded token's outputs (every write is at a position derived from
    // the token / line ordinals, so deferred tokens may write later)
    auto emit = [&](bool active, uint32_t e, uint32_t i, const tok::Token& t, bool bad) {
      const bool is_label = active && ((e >> 13) & 1u) != 0;
      const uint32_t lc = e >> 14;
      const int32_t rel = static_cast<int32_t>(i) - static_cast<int32_t>(lc);
      const bool row_ok = static_cast<int32_t>(lc) - 1 < row_room;
      const bool nnz_ok = rel < nnz_room;
      bool field_ok = true;
      if (F == TextFormat::kLibFM) field_ok = is_label || t.r >= 2;
      // past the target's rows / entries: with sizes from C1 + C2 that is a
      // C1 / C3 disagreement (irregular); one pass writes into the capacity
      // the host has and asks for more (kFlagOverflow: grow, run again)
      const bool room_ok = is_label ? row_ok : nnz_ok;
      irregular |= active & !is_label & !field_ok;
      if constexpr (kOnePass) {
        over |= active & !room_ok;
      } else {
        irregular |= active & !room_ok;
      }
      if (fill_exp(op) & 1u) {
        // pricing: everything but the stores (the values stay live)
        sink ^= (active ? __float_as_uint(t.f0) ^ t.u0 ^ t.u1 : 0u) + static_cast<uint32_t>(i);
        return;
      }
      if (active & is_label & row_ok) {
        lab_at[lc] = t.f0;
        off_at[lc] = C + 1 + (static_cast<int64_t>(i) - static_cast<int64_t>(lc));
        if (wgt_at != nullptr) wgt_at[lc] = t.r == 2 ? t.f1 : 1.0f;
        // (qid: zero-filled by the host, the qid token's lane writes it)
      }
      if constexpr (!kLean) need_w |= active & is_label & (wgt_at == nullptr) & (t.r == 2);
      any_weight |= active & is_label & (t.r == 2);
      const bool feat = active & !is_label & nnz_ok & field_ok;
      const uint64_t u0 = (static_cast<uint64_t>(t.u0_hi) << 32) | t.u0;
      // (a feature's rel = i - lc is >= 0 and < 2^13: a 32-bit byte offset
      // from the SGPR base, no 64-bit address arithmetic per store)
      const uint32_t boff = static_cast<uint32_t>(rel) * static_cast<uint32_t>(sizeof(IndexType));
      const uint32_t voff = static_cast<uint32_t>(rel) * 4u;
      auto at = [](auto* base, uint32_t off) {
        using T = typename std::remove_pointer<decltype(base)>::type;
        return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
      };
      if constexpr (F == TextFormat::kLibSVM) {
        if (feat) {
          *at(idx_at, boff) = static_cast<IndexType>(u0);
          *at(val_at, voff) = t.r == 2 ? t.f0 : 1.0f;
        }
        any_value |= feat && t.r == 2;
        const MaxT iu = static_cast<MaxT>(static_cast<IndexType>(u0));
        mx_index = feat && iu > mx_index ? iu : mx_index;
      } else {
        const uint64_t u1 = (static_cast<uint64_t>(t.u1_hi) << 32) | t.u1;
        if (feat) {
          *at(fld_at, boff) = static_cast<IndexType>(u0);
          *at(idx_at, boff) = static_cast<IndexType>(u1);
          *at(val_at, voff) = t.r == 3 ? t.f0 : 1.0f;
        }
        any_value |= feat && t.r == 3;
        const MaxT iu = static_cast<MaxT>(static_cast<IndexType>(u1));
        const MaxT fu = static_cast<MaxT>(static_cast<IndexType>(u0));
        mx_index = feat && iu > mx_index ? iu : mx_index;
        mx_field = feat && fu > mx_field ? fu : mx_field;
      }
      neg |= active && bad;
    };
    // tokens the register-window decoder declines (exponents, long fractions,
    // anything for the generic parser) are queued (their list index, in a
    // ring) and decoded 64 at a time in rounds of their own, so a round with
    // one such token does not pay the long decoder for all 64 lanes; the
    // queue is drained before the slots it points into are restaged (by the
    // end of every step).  While 128 listed tokens remain a round decodes two
    // per lane (tok::decode2: two independent dependency chains per lane).
    auto enqueue = [&](bool defer, uint32_t li) {
      const uint64_t dm = __ballot(defer);
      if (dm != 0) {
        const uint32_t rank = static_cast<uint32_t>(__popcll(dm & ((1ull << lane) - 1ull)));
        if (defer) dq[(qh + qn + rank) & (kQueueCap - 1)] = li;
        qn += static_cast<uint32_t>(__popcll(dm));
      }
    };
    for (uint32_t r0 = 0;;) {
      const bool qround = qn >= static_cast<uint32_t>(dev::kWave) || (r0 >= ndec && qn != 0);
      if (!qround && r0 >= ndec) break;
      if (!qround && r0 + 2 * dev::kWave <= ndec) {  // wave-uniform: a pair round
        const uint32_t la = r0 + slot, lb = la + dev::kWave;
        const uint32_t ea = sl[la], eb = sl[lb];
        tok::Token ta, tb;
        ta.u0_hi = ta.u1_hi = tb.u0_hi = tb.u1_hi = 0;
        ta.u1 = tb.u1 = 0;
        bool oka, okb;
        if (fill_exp(op) & 2u) {  // pricing: no decode
          ta.u0 = ea;
          tb.u0 = eb;
          ta.f0 = ta.f1 = tb.f0 = tb.f1 = 1.0f;
          ta.r = tb.r = 2;
          oka = okb = true;
        } else {
          tok::decode2<F>(st, ea & 0x1FFFu, eb & 0x1FFFu, ((ea >> 13) & 1u) != 0,
                          ((eb >> 13) & 1u) != 0, &ta, &tb, &oka, &okb);
        }
        enqueue(!oka, la);
        enqueue(!okb, lb);
        emit(oka, ea, tok0 + la, ta, false);
        emit(okb, eb, tok0 + lb, tb, false);
        r0 += 2 * dev::kWave;
        continue;
      }
      bool active;
      uint32_t e, i;
      tok::Token t;
      t.u0_hi = t.u1_hi = 0;
      t.u1 = 0;
      bool bad = false;
      if (!qround) {
        const uint32_t li = r0 + slot;
        active = li < ndec;
        e = active ? sl[li] : 0u;
        i = tok0 + li;
        const bool is_label = active && ((e >> 13) & 1u) != 0;
        // 0 in idle lanes: they decode harmless bytes
        const bool ok = tok::decode<F>(st, e & 0x1FFFu, is_label, &t);
        enqueue(active & !ok, li);
        active = active & ok;
        r0 += dev::kWave;
      } else {
        dev::wave_sync();  // queue entries visible
        const uint32_t cnt = qn < static_cast<uint32_t>(dev::kWave) ? qn : dev::kWave;
        active = slot < cnt;
        const uint32_t li = active ? dq[(qh + slot) & (kQueueCap - 1)] : 0u;
        qh += cnt;
        qn -= cnt;
        e = active ? sl[li] : 0u;
        i = tok0 + li;
        const bool is_label = active && ((e >> 13) & 1u) != 0;
        const uint32_t off = e & 0x1FFFu;
        bool ok = false;
        if (active) {
          const tok::ExtToken x = tok::decode_ext<F>(
              st, off, is_label, off >= kSlotBytes ? 2 * kSlotBytes : kSlotBytes);
          t = x.t;
          ok = x.ok;
        }
        if (active & !ok) {
          // the step a slot holds: s, or s - 1 for a carried token
          const uint32_t in_slot = off >= kSlotBytes ? 1u : 0u;
          const int step = in_slot == (static_cast<uint32_t>(s) & 1u) ? s : s - 1;
          // by value: result pointers into this frame would put t / bad on the
          // stack, with a scratch store + load (and a vmcnt(0) wait) every round
          const size_t gpos =
              tile0 + static_cast<size_t>(step) * kStepBytes + off - in_slot * kSlotBytes;
          const GenericResult g = generic_token<F, IndexType>(text, n, gpos, is_label);
          t = g.t;
          bad = g.bad;
          // qid:, comments, junk: the exact kernels own the reference semantics
          irregular |= !num_start(text[gpos]);
        }
      }
      emit(active, e, i, t, bad);
    }
    // the undecoded rest moves to the front of the list (all lanes read before any writes)
    const uint32_t left = total - ndec;
    const uint32_t moved = lane < static_cast<int>(left) ? sl[ndec + lane] : 0u;
    dev::wave_sync();
    if (lane < static_cast<int>(left)) sl[lane] = moved;
    tok0 += ndec;
    carry = left;
    lcnt += nline;
    dev::wave_sync();  // every lane is done with this step's text and list
  }
  unsigned fl = count_flags;
  if (sink == 0x9E3779B9u) fl |= kFlagIrregular;  // keeps a pricing run's values live
  if (any_value) fl |= kFlagValue;
  if (any_weight) fl |= kFlagWeight;
  if (irregular) fl |= kFlagIrregular;
  if (neg) fl |= kFlagNegIndex;
  if (kLean ? any_weight : need_w) fl |= kFlagNeedWeight;  // (lean: no weight column)
  if (over) fl |= kFlagOverflow;
  if (F == TextFormat::kLibFM) fl |= kFlagField;
  const unsigned long long mi = dev::wave_max(static_cast<unsigned long long>(mx_index));
  const unsigned long long mf = dev::wave_max(static_cast<unsigned long long>(mx_field));
  fl = dev::wave_or(fl);
  if (lane == 0) {
    MetaPartial p;
    p.max_index = mi;
    p.max_field = mf;
    p.flags = fl;
    p.pad = 0;
    partials[tile] = p;
  }
}

/*!
 * \brief fused tokenize -> hash -> dense row (BASELINE config 5) on the fill
 *  kernel's wave-autonomous pipeline.  Wave w OWNS the lines that start in its
 *  8 KiB tile (`own` of them, from the C2 prefix -- no per-tile host data):
 *   1. the tile streams through the two LDS slots in 2 KiB steps exactly as in
 *      k_tile_fill (register prefetch, SWAR masks, DPP scan, wave-private token
 *      list, 64-token decode rounds through tok::decode).  Only owned tokens
 *      are listed: the head of the tile (the rest of the previous tile's last
 *      line) and everything after the owned lines are masked out before the
 *      scan, in the first / last step only (wave-uniform test);
 *   2. the last owned line is followed past the tile end step by step until
 *      the next line start (or the end of the text) -- no extension cap and
 *      no fallback for long lines; steps after the first extension step
 *      prefetch only the 64 B tail (lines > 2 KiB past the tile are rare);
 *   3. every decoded feature adds +-value at bucket hash % dim of ONE f32 row
 *      in the wave's LDS (ds_add_f32); when a round moves past a line, that row
 *      is flushed: each lane reads a float4 per 256 columns (lane-interleaved,
 *      conflict-free), zeroes it, converts to OCP fp8 e4m3 (v_cvt_pk_fp8_f32)
 *      and stores 4 B -- 256 contiguous bytes per wave store, zero spans
 *      included, no separate memset pass.
 *  The label token's lane writes the label.  No CSR, no per-row LDS buffers
 *  per workgroup, no barrier.  Hash and bucket are K9's (dev::hash_u64), so
 *  the fp8 bytes equal tile CSR + K9.  Reference token loop:
 *  src/data/libfm_parser.h:36-93, libsvm_parser.h:36-99 (strtonum.h:266-303).
 */
struct HashTarget {
  void* x;            // [row_limit, dim] fp8 bytes or f32
  float* label;
  uint64_t row_base;  // global row of the chunk's first line
  uint64_t nlines;    // lines of the chunk (the C2 total; one-pass: unused)
  int dim;
  float scale;
  uint32_t seed;
  // one pass (no C1 / C2): line counts by look-back, rows checked against row_cap
  uint32_t tag;                 // this launch's status tag (!= 0)
  uint64_t* status;             // per-tile look-back words
  unsigned long long* ticket;   // workgroup ticket counter
  unsigned long long ticket0;   // its value at this launch
  uint64_t row_cap;             // rows of x / label
  ChunkMeta* meta;              // nlines / nrows of the chunk (the last tile writes them)
  const uint32_t* masks;        // counted path: C1's start masks (TileMaskWords)
};

/*! \brief keep the token starts of a slice whose line ordinals are in [1, own];
 *  L0 = ordinal at the slice start (line starts before it, this tile) */
__device__ __forceinline__ uint32_t owned_tokens(uint32_t tm, uint32_t lm, uint32_t L0,
                                                 uint32_t own) {
  uint32_t m = tm;
  if (L0 == 0) m &= lm != 0 ? ~((lm & (0u - lm)) - 1u) : 0u;  // from the first line start on
  const uint32_t nl = static_cast<uint32_t>(__popc(lm));
  if (L0 + nl > own) {
    if (L0 > own) return 0u;
    uint32_t x = lm;
    for (uint32_t k = own - L0; k != 0; --k) x &= x - 1u;  // drop the starts still owned
    m &= (x & (0u - x)) - 1u;  // bytes before the first line start past `own`
  }
  return m;
}

template <TextFormat F, typename IndexType, bool kFP8, bool kOnePass>
__global__ __launch_bounds__(kThreads, DMLC_FILL_WAVES) void k_tile_hash(
    const uint8_t* __restrict__ text, size_t n, size_t ntiles,
    const uint64_t* __restrict__ prefix, HashTarget out, MetaPartial* __restrict__ partials) {
  // one staging slot and a list without carried entries: every step decodes
  // all its tokens, so the LDS per wave (+ the dim-wide f32 row) leaves room
  // for 4 workgroups per CU up to dim 1024
  __shared__ uint4 s_text[kFillWaves][kHashText / 16];
  __shared__ uint32_t s_list[kFillWaves][kHashListCap + 64];
  extern __shared__ __attribute__((aligned(16))) float s_hrow[];  // kFillWaves x dim
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / dev::kWave);
  const int lane = dev::lane_id();
  size_t group = blockIdx.x;
  if constexpr (kOnePass) {
    // tiles in ticket order: a workgroup looks back only at tiles of
    // workgroups that started before it (whatever the dispatch order)
    __shared__ uint32_t s_ticket;
    if (threadIdx.x == 0) s_ticket = static_cast<uint32_t>(atomicAdd(out.ticket, 1ull) - out.ticket0);
    __syncthreads();
    group = s_ticket;
  }
  const size_t tile = group * kFillWaves + wave;
  if (tile >= ntiles) return;  // whole waves leave; nothing below synchronises waves
  uint4* const st = s_text[wave];
  uint32_t* const sl = s_list[wave];
  const int dim = out.dim;
  float* const row = s_hrow + static_cast<size_t>(wave) * dim;
  const uint32_t slot = round_slot(lane);
  const size_t tile0 = tile * kTileBytes;
  const __amdgpu_buffer_rsrc_t trs = text_rsrc(text + tile0, n - tile0);
  const uint32_t loff = static_cast<uint32_t>(lane) * 16;
  uint4 a = bload16(trs, loff);
  uint4 b = bload16(trs, loff + 1024);
  // counted path: C1's start masks per step (steps past the tile read the
  // next tiles' words: the layout is contiguous over the chunk)
  __amdgpu_buffer_rsrc_t mrs;
  const uint32_t moff = static_cast<uint32_t>(lane) * 8;
  uint2 mk = make_uint2(0, 0);
  if constexpr (!kOnePass) {
    mrs = mask_rsrc(out.masks, tile, ntiles);
    mk = load_masks(mrs, moff, 0);
  }
  uint32_t carry_pc = 0;
  if constexpr (kOnePass) carry_pc = tile0 == 0 ? static_cast<uint32_t>('\n') : text[tile0 - 1];
  uint64_t line_base;
  uint32_t own;
  if constexpr (kOnePass) {
    // the C1 line count of this tile (its other 6 KiB come into L2 for the
    // steps), then the look-back for the lines before it
    uint4 v[kCountLoads];
    v[0] = a;
    v[1] = b;
#pragma unroll
    for (int j = 2; j < kCountLoads; ++j) v[j] = bload16(trs, loff + j * 1024);
    const bool full = tile0 + kTileBytes <= n;
    uint32_t lines = 0;
#pragma unroll
    for (int j = 0; j < kCountLoads; ++j) {
      const uint32_t left = dev::lane_shr1(v[j].w >> 24);
      const uint32_t wrap = j == 0 ? carry_pc : dev::lane63(v[j - 1].w >> 24);
      const uint32_t pc = lane == 0 ? wrap : left;
      if (full) {
        lines += lines16<true>(v[j], pc, 16);
      } else {
        const size_t pos = tile0 + j * 1024 + lane * 16;
        const int room = pos >= n ? 0 : (n - pos < 16 ? static_cast<int>(n - pos) : 16);
        lines += lines16<false>(v[j], pc, room);
      }
    }
    own = dev::wave_sum(lines);
    line_base = lookback_lines(out.status, tile, own, out.tag, lane);
    if (tile + 1 == ntiles && lane == 0) {
      ChunkMeta m;
      m.nlines = m.nrows = line_base + own;
      m.nnz = 0;
      m.max_index = m.max_field = 0;
      m.flags = 0;
      m.pad = 0;
      *out.meta = m;  // k_tile_finish (stream-ordered) adds the flags
    }
  } else {
    line_base = prefix[tile] >> 32;
    const uint64_t line_next = tile + 1 < ntiles ? prefix[tile + 1] >> 32 : out.nlines;
    own = static_cast<uint32_t>(line_next - line_base);
  }
  const uint64_t row_cap = kOnePass ? out.row_cap : ~0ull;
  bool irregular = false, neg = false, over = false;
  if (own != 0) {
    const uint64_t R = out.row_base + line_base;  // global row of tile line ordinal 1
    float* const lab_at = out.label + R - 1;      // labels by tile line ordinal
    const bool pow2 = (dim & (dim - 1)) == 0;
    const uint32_t dmask = static_cast<uint32_t>(dim - 1);
    for (int c = lane * 4; c < dim; c += dev::kWave * 4) {
      *reinterpret_cast<float4*>(row + c) = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    // one row out: read + zero this lane's columns, convert, store
    auto flush = [&](uint32_t lc) {
      dev::wave_sync();  // the row's adds are done
      const uint64_t g = R + lc - 1;
      const bool ok = lc <= own && g < row_cap;
      over |= lc <= own && g >= row_cap;
      if constexpr (kFP8) {
        // lane-interleaved float4s (consecutive lanes, consecutive 16 B: no
        // bank conflicts on the b128 read / zero), 4 fp8 bytes per lane store
        uint8_t* o = static_cast<uint8_t*>(out.x) + g * static_cast<uint64_t>(dim);
#pragma unroll 4
        for (int c0 = 0; c0 < dim; c0 += dev::kWave * 4) {  // uniform trip count
          const int c = c0 + lane * 4;
          if (c < dim) {  // (no break: the loop exit stays uniform)
            float4* r4 = reinterpret_cast<float4*>(row + c);
            const float4 x = *r4;
            *r4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            int pk = __builtin_amdgcn_cvt_pk_fp8_f32(x.x * out.scale, x.y * out.scale, 0, false);
            pk = __builtin_amdgcn_cvt_pk_fp8_f32(x.z * out.scale, x.w * out.scale, pk, true);
            if (ok) *reinterpret_cast<uint32_t*>(o + c) = static_cast<uint32_t>(pk);
          }
        }
      } else {
        float* o = static_cast<float*>(out.x) + g * static_cast<uint64_t>(dim);
        for (int c0 = 0; c0 < dim; c0 += dev::kWave * 4) {
          const int c = c0 + lane * 4;
          if (c < dim) {
            float4* r4 = reinterpret_cast<float4*>(row + c);
            const float4 x = *r4;
            *r4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (ok) *reinterpret_cast<float4*>(o + c) = make_float4(x.x, x.y, x.z, x.w);
          }
        }
      }
      dev::wave_sync();  // zeros land before the next row's adds
    };

    // loads as in k_tile_fill: the next step's go into a / b / t once they are
    // consumed (no copies of loads in flight), clipped where staged
    uint4 t = make_uint4(0, 0, 0, 0);
    if (lane < 4) t = bload16(trs, loff + kStepBytes);
    uint32_t lcnt = 0;   // line starts seen so far (this tile's ordinals)
    uint32_t open = 0;   // ordinal of the row being accumulated (0: none yet)
    uint32_t carry = 0;  // list entries carried from the previous step (listed, not decoded)
    uint32_t qid_prev = 0;  // LibSVM: status of the last token start (prev_token_status)
#pragma unroll 1
    for (int s = 0;; ++s) {
      const size_t cur = tile0 + static_cast<size_t>(s) * kStepBytes;
      const size_t nxt = cur + kStepBytes;
      const size_t pos_a = cur + lane * 16;
      if (nxt + 64 > n) {  // wave-uniform: the text ends here
        a = clip16(a, pos_a, n);
        b = clip16(b, pos_a + 1024, n);
        t = clip16(t, pos_a + kStepBytes, n);
      }
      // the step at [kHashCarry, kHashText); carried tokens' text before it
      constexpr uint32_t sbase = kHashCarry;
      st[sbase / 16 + lane] = a;
      st[sbase / 16 + 64 + lane] = b;
      if (lane < 4) st[sbase / 16 + 128 + lane] = t;
      uint32_t lm_a, tm_a, lm_b, tm_b;
      if constexpr (kOnePass) {
        const uint32_t left_a = dev::lane_shr1(a.w >> 24);
        const uint32_t pc_a = lane == 0 ? carry_pc : left_a;
        const uint32_t left_b = dev::lane_shr1(b.w >> 24);
        const uint32_t last_a = dev::lane63(a.w >> 24);
        const uint32_t pc_b = lane == 0 ? last_a : left_b;
        // one pass: C1's checks of blank-started lines and control bytes here
        // (token starts outside [0-9+-.] fail the decoder and are flagged there)
        if (nxt <= n) {  // wave-uniform: a full step
          irregular |= lane_masks<true, true, false>(a, pc_a, pos_a, n, &lm_a, &tm_a);
          irregular |= lane_masks<true, true, false>(b, pc_b, pos_a + 1024, n, &lm_b, &tm_b);
        } else {
          irregular |= lane_masks<true, false, false>(a, pc_a, pos_a, n, &lm_a, &tm_a);
          irregular |= lane_masks<true, false, false>(b, pc_b, pos_a + 1024, n, &lm_b, &tm_b);
        }
      } else {
        tm_a = mk.x & 0xFFFFu;
        lm_a = mk.x >> 16;
        tm_b = mk.y & 0xFFFFu;
        lm_b = mk.y >> 16;
      }
      carry_pc = dev::lane63(b.w >> 24);  // the step's last byte (a line end?)
      if (F == TextFormat::kLibSVM) {
        // `qid:` tokens are no features of the batch: dropped (checked as in
        // the fill, from the staged text; any other letter token sends the
        // chunk to the exact kernels)
        const uint32_t qa = tm_a & letter_mask(a), qb = tm_b & letter_mask(b);
        if (__any((qa | qb) != 0)) {
          const PrevTok pv = prev_token_status(tm_a, lm_a, tm_b, lm_b, qid_prev, lane);
          dev::wave_sync();  // the staged step is visible to every lane
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t lmh = h == 0 ? lm_a : lm_b, tmh = h == 0 ? tm_a : tm_b;
            for (uint32_t m = h == 0 ? qa : qb; m != 0; m &= m - 1) {
              const uint32_t j = static_cast<uint32_t>(__builtin_ctz(m));
              const uint32_t prev = status_before(tmh, lmh, j, h == 0 ? pv.a : pv.b);
              bool ok = false;
              if (prev == 3u) {
                ok = qid_lds(st, sbase + static_cast<uint32_t>(h) * 1024 + lane * 16 + j).ok;
              } else if (prev == 0u) {
                ok = qid_token(text, n, pos_a + static_cast<size_t>(h) * 1024 + j).ok;
              }
              irregular |= ((lmh >> j) & 1u) != 0 || !ok;
            }
          }
        }
        qid_prev = step_last_status(tm_a, lm_a, tm_b, lm_b, qid_prev);
        tm_a &= ~qa;
        tm_b &= ~qb;
      }
      uint64_t cnt = static_cast<uint64_t>(__popc(tm_a)) |
                     (static_cast<uint64_t>(__popc(tm_b)) << 16) |
                     (static_cast<uint64_t>(__popc(lm_a)) << 32) |
                     (static_cast<uint64_t>(__popc(lm_b)) << 48);
      uint64_t tot;
      uint64_t before = dev::wave_excl_scan_2x32(cnt, &tot);  // 16-bit fields: no carries
      const uint32_t nline_a = static_cast<uint32_t>((tot >> 32) & 0xFFFFu);
      const uint32_t nline = nline_a + static_cast<uint32_t>(tot >> 48);
      const uint32_t la0 = lcnt + static_cast<uint32_t>((before >> 32) & 0xFFFFu);
      const uint32_t lb0 = lcnt + nline_a + static_cast<uint32_t>(before >> 48);
      if (lcnt == 0 || lcnt + nline > own) {
        // wave-uniform (first / last step): drop tokens outside the owned lines
        tm_a = owned_tokens(tm_a, lm_a, la0, own);
        tm_b = owned_tokens(tm_b, lm_b, lb0, own);
        cnt = static_cast<uint64_t>(__popc(tm_a)) | (static_cast<uint64_t>(__popc(tm_b)) << 16);
        uint32_t t32;
        const uint32_t b32 = dev::wave_excl_scan<uint32_t>(static_cast<uint32_t>(cnt), &t32);
        before = (before & ~0xFFFFFFFFull) | b32;
        tot = (tot & ~0xFFFFFFFFull) | t32;
      }
      const uint32_t ntok_a = static_cast<uint32_t>(tot & 0xFFFFu);
      const uint32_t ntok = ntok_a + static_cast<uint32_t>((tot >> 16) & 0xFFFFu);
      // a step of more tokens than the list holds is listed and decoded in
      // its two 1 KiB halves (a half of more: the exact kernels)
      const uint32_t ntok_b = ntok - ntok_a;
      const bool split = carry + ntok > kHashListCap;
      if (split && (carry + ntok_a > kHashListCap || ntok_b > kHashListCap)) {
        irregular = true;
        break;
      }
      lcnt += nline;
      const bool eol_end = carry_pc == '\n' || carry_pc == '\r';
      const bool last = nxt >= n || lcnt > own || (s + 1 >= kSteps && lcnt == own && eol_end);
      // a, b, t are consumed (staged, masks taken): the next step's loads go
      // straight into them (in flight during this step's rounds)
      if (!last) {
        const uint32_t so = static_cast<uint32_t>(s + 1) * kStepBytes;
        a = bload16(trs, loff + so);
        b = bload16(trs, loff + so + 1024);
        if (lane < 4) t = bload16(trs, loff + so + kStepBytes);
        if constexpr (!kOnePass) mk = load_masks(mrs, moff, s + 1);
      }

      list_slice<kHashListCap>(sl, tm_a, lm_a, carry + static_cast<uint32_t>(before & 0xFFFFu),
                               sbase + lane * 16, la0, lane);
      // split: the b half is listed after the a half's rounds, from two packed
      // registers (few live across the rounds)
      const uint32_t pk_m = tm_b | (lm_b << 16);
      const uint32_t pk_o = static_cast<uint32_t>((before >> 16) & 0xFFFFu) | (lb0 << 16);
      if (!split) {
        list_slice<kHashListCap>(sl, tm_b, lm_b,
                                 carry + ntok_a + static_cast<uint32_t>((before >> 16) & 0xFFFFu),
                                 sbase + 1024 + lane * 16, lb0, lane);
      }
      dev::wave_sync();
      uint32_t total = 0, ndec = 0;
#pragma unroll 1
      for (int part = 0;; ++part) {
        // the list: carried tokens, then this step's (or its halves'); only
        // whole rounds run unless this is the wave's last step, or the first
        // left-over token starts before the part of the step a carry keeps
        // (its text would not fit the carry area: decode it all now).  The
        // a half of a split step is decoded whole.
        total = !split ? carry + ntok : (part == 0 ? carry + ntok_a : ntok_b);
        uint32_t rest = (last || (split && part == 0)) ? 0u : total % dev::kWave;
        if (rest != 0 && (dev::uniform(sl[total - rest]) & 0x1FFFu) < kHashText - kHashCarry - 64u) {
          rest = 0;
        }
        ndec = total - rest;
        for (uint32_t r0 = 0; r0 < ndec; r0 += dev::kWave) {
          const uint32_t li = r0 + slot;
          const bool active = li < ndec;
          const uint32_t e = active ? sl[li] : 0u;
          const bool is_label = active && ((e >> 13) & 1u) != 0;
          const uint32_t off = e & 0x1FFFu;
          const uint32_t lc = e >> 14;
          tok::Token t;
          t.u0_hi = t.u1_hi = 0;
          t.u1 = 0;
          bool bad = false;
          bool ok = tok::decode<F>(st, off, is_label, &t);
          if (__any(active & !ok)) {
            if (active & !ok) {
              const tok::ExtToken x = tok::decode_ext<F>(st, off, is_label, kHashText);
              if (x.ok) t = x.t;
              ok = x.ok;
            }
          }
          if (active & !ok) {
            const size_t gpos = cur + off - sbase;  // (carried tokens: before cur)
            const GenericResult gr = generic_token<F, IndexType>(text, n, gpos, is_label);
            t = gr.t;
            bad = gr.bad;
            irregular |= !num_start(text[gpos]);  // qid:, comments, junk: the exact kernels
          }
          // (counted path: C2 sized the target, no row check)
          if (active & is_label && (!kOnePass || R + lc - 1 < row_cap)) lab_at[lc] = t.f0;
          bool feat = active & !is_label;
          uint64_t key;
          float val;
          const uint64_t u0 = (static_cast<uint64_t>(t.u0_hi) << 32) | t.u0;
          if constexpr (F == TextFormat::kLibSVM) {
            key = static_cast<uint64_t>(static_cast<IndexType>(u0));
            val = t.r == 2 ? t.f0 : 1.0f;
          } else {
            const uint64_t u1 = (static_cast<uint64_t>(t.u1_hi) << 32) | t.u1;
            feat &= t.r >= 2;  // not field:index: the CPU parser skips it too
            key = dev::hash_key(static_cast<uint64_t>(static_cast<IndexType>(u1)),
                                static_cast<uint64_t>(static_cast<IndexType>(u0)), true);
            val = t.r == 3 ? t.f0 : 1.0f;
          }
          neg |= active && bad;
          const uint32_t h = dev::hash_u64(key, out.seed);
          uint32_t bucket;
          if (pow2) {
            bucket = h & dmask;
          } else {
            bucket = h % static_cast<uint32_t>(dim);
          }
          const float sv = (h & 0x80000000u) ? -val : val;
          // the round's rows, in text order: list entries r0 .. r0 + 63
          const uint32_t lo = dev::uniform(sl[r0] >> 14);
          const uint32_t hi =
              dev::uniform(sl[r0 + dev::kWave - 1 < ndec ? r0 + dev::kWave - 1 : ndec - 1] >> 14);
          for (uint32_t rr = lo; rr <= hi; ++rr) {
            if (rr != open) {
              if (open != 0) flush(open);
              open = rr;
            }
            if (feat && lc == rr) atomicAdd(&row[bucket], sv);
          }
        }
        if (!split || part == 1) break;
        carry = 0;  // the a half's list (carried tokens included) is done
        dev::wave_sync();  // the a half's rounds are done with the list
        list_slice<kHashListCap>(sl, pk_m & 0xFFFFu, pk_m >> 16, pk_o & 0xFFFFu,
                                 sbase + 1024 + lane * 16, pk_o >> 16, lane);
        dev::wave_sync();
      }  // part
      if (last) break;
      // carry the rest: the step's last 1 KiB of text into the carry area (the
      // next step restages the 64 B after it), its entries to the list front
      // with offsets moved down by the 2 KiB the text shifts
      const uint32_t left = total - ndec;
      dev::wave_sync();  // every lane is done with this step's rounds
      if (left != 0) {
        const uint4 keep = st[(kHashText - kHashCarry - 64) / 16 + lane];
        const uint32_t moved = lane < static_cast<int>(left) ? sl[ndec + lane] : 0u;
        dev::wave_sync();
        st[lane] = keep;
        if (lane < static_cast<int>(left)) sl[lane] = moved - kStepBytes;
      }
      carry = left;
      dev::wave_sync();  // every lane is done with this step's text and list
    }
    if (open != 0) flush(open);
  }
  unsigned fl = 0;
  if (irregular) fl |= kFlagIrregular;
  if (neg) fl |= kFlagNegIndex;
  if (over) fl |= kFlagOverflow;
  fl = dev::wave_or(fl);
  if (lane == 0) {
    MetaPartial p;
    p.max_index = 0;
    p.max_field = 0;
    p.flags = fl;
    p.pad = 0;
    partials[tile] = p;
  }
}

/*!
 * \brief fold the per-workgroup slots into meta; closing row pointer.  One
 *  1024-lane workgroup, 8 independent slot loads per lane per step (a
 *  latency-bound single-workgroup pass otherwise dominates small chunks).
 */
constexpr int kFinishThreads = 1024;
constexpr int kFinishPer = 8;
__global__ __launch_bounds__(kFinishThreads) void k_tile_finish(
    const MetaPartial* __restrict__ p, int np, ChunkMeta* meta, ChunkMeta* host_meta,
    uint64_t* offset, uint64_t row_base, uint64_t nnz_base) {
  unsigned long long mi = 0, mf = 0;
  unsigned fl = 0;
  for (int i0 = threadIdx.x; i0 < np; i0 += kFinishThreads * kFinishPer) {
    MetaPartial q[kFinishPer];
#pragma unroll
    for (int u = 0; u < kFinishPer; ++u) {
      const int i = i0 + u * kFinishThreads;
      if (i < np) {
        q[u] = p[i];
      } else {
        q[u].max_index = q[u].max_field = 0;
        q[u].flags = 0;
      }
    }
#pragma unroll
    for (int u = 0; u < kFinishPer; ++u) {
      mi = q[u].max_index > mi ? q[u].max_index : mi;
      mf = q[u].max_field > mf ? q[u].max_field : mf;
      fl |= q[u].flags;
    }
  }
  __shared__ unsigned long long s_mi[kFinishThreads / 64], s_mf[kFinishThreads / 64];
  __shared__ unsigned s_fl[kFinishThreads / 64];
  mi = dev::wave_max(mi);
  mf = dev::wave_max(mf);
  fl = dev::wave_or(fl);
  const int wid = threadIdx.x / dev::kWave;
  if (dev::lane_id() == 0) {
    s_mi[wid] = mi;
    s_mf[wid] = mf;
    s_fl[wid] = fl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kFinishThreads / 64; ++w) {
      s_mi[0] = s_mi[w] > s_mi[0] ? s_mi[w] : s_mi[0];
      s_mf[0] = s_mf[w] > s_mf[0] ? s_mf[w] : s_mf[0];
      s_fl[0] |= s_fl[w];
    }
    meta->max_index = s_mi[0];
    meta->max_field = s_mf[0];
    meta->flags |= s_fl[0];
    // (an overflowed one-pass fill's rows reach past the target: no row pointer)
    if (offset != nullptr && !(meta->flags & kFlagOverflow)) {
      offset[row_base + meta->nrows] = nnz_base + meta->nnz;
    }
    if (host_meta != nullptr) publish_host_meta(host_meta, *meta);
  }
}
/*! \brief level 1 of the finish fold: workgroup g folds slots g, g+G, ... into out[g] */
__global__ __launch_bounds__(kFinishThreads) void k_tile_finish_partial(
    const MetaPartial* __restrict__ p, size_t np, MetaPartial* __restrict__ out) {
  unsigned long long mi = 0, mf = 0;
  unsigned fl = 0;
  const size_t stride = static_cast<size_t>(gridDim.x) * kFinishThreads;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kFinishThreads + threadIdx.x; i < np;
       i += stride) {
    const MetaPartial q = p[i];
    mi = q.max_index > mi ? q.max_index : mi;
    mf = q.max_field > mf ? q.max_field : mf;
    fl |= q.flags;
  }
  __shared__ unsigned long long s_mi[kFinishThreads / 64], s_mf[kFinishThreads / 64];
  __shared__ unsigned s_fl[kFinishThreads / 64];
  mi = dev::wave_max(mi);
  mf = dev::wave_max(mf);
  fl = dev::wave_or(fl);
  const int wid = threadIdx.x / dev::kWave;
  if (dev::lane_id() == 0) {
    s_mi[wid] = mi;
    s_mf[wid] = mf;
    s_fl[wid] = fl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kFinishThreads / 64; ++w) {
      mi = s_mi[w] > mi ? s_mi[w] : mi;
      mf = s_mf[w] > mf ? s_mf[w] : mf;
    }
    mi = s_mi[0] > mi ? s_mi[0] : mi;
    mf = s_mf[0] > mf ? s_mf[0] : mf;
    unsigned f = 0;
    for (int w = 0; w < kFinishThreads / 64; ++w) f |= s_fl[w];
    MetaPartial r;
    r.max_index = mi;
    r.max_field = mf;
    r.flags = f;
    r.pad = 0;
    out[blockIdx.x] = r;
  }
}

// chunks above this many tiles take the multi-workgroup scan / finish
constexpr size_t kTwoLevelTiles = 2 * kScanBlockTiles;
constexpr int kFinishGroups = 128;

void LaunchFinish(MetaPartial* partials, size_t ntiles, ChunkMeta* meta, ChunkMeta* host_meta,
                  uint64_t* offset, uint64_t row_base, uint64_t nnz_base, hipStream_t stream) {
  const MetaPartial* src = partials;
  int np = static_cast<int>(ntiles);
  if (ntiles > kTwoLevelTiles) {
    MetaPartial* folded = partials + ntiles;  // TileScratchSlots(ntiles) leaves room
    hipLaunchKernelGGL(k_tile_finish_partial, dim3(kFinishGroups), dim3(kFinishThreads), 0, stream,
                       partials, ntiles, folded);
    src = folded;
    np = kFinishGroups;
  }
  hipLaunchKernelGGL(k_tile_finish, dim3(1), dim3(kFinishThreads), 0, stream, src, np, meta,
                     host_meta, offset, row_base, nnz_base);
}
}  // namespace

size_t TileCount(size_t nbytes) { return (nbytes + kTileBytes - 1) / kTileBytes; }

namespace {
void TileScan(uint64_t* tile_counts, uint32_t* tile_flags, size_t ntiles, ChunkMeta* meta,
              ChunkMeta* host_meta, int raw, hipStream_t stream) {
  if (ntiles <= kTwoLevelTiles) {
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(kScanThreads), 0, stream, tile_counts,
                       tile_flags, ntiles, meta, host_meta, raw);
    return;
  }
  // block totals / flags live past the tiles (TileScratchWords reserves them)
  const size_t nblk = (ntiles + kScanBlockTiles - 1) / kScanBlockTiles;
  uint64_t* bsum = tile_counts + ntiles;
  uint32_t* bflag = tile_flags + ntiles;
  hipLaunchKernelGGL(k_tile_scan_local, dim3(nblk), dim3(kScanThreads), 0, stream, tile_counts,
                     tile_flags, ntiles, bsum, bflag);
  hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(kScanThreads), 0, stream, bsum, bflag, nblk, meta,
                     host_meta, raw);
  hipLaunchKernelGGL(k_tile_scan_add, dim3((ntiles + kThreads - 1) / kThreads), dim3(kThreads), 0,
                     stream, tile_counts, ntiles, bsum);
}
}  // namespace

void LaunchTileCountScan(const char* text, size_t nbytes, uint64_t* tile_counts,
                         uint32_t* tile_flags, uint32_t* tile_masks, ChunkMeta* meta,
                         ChunkMeta* host_meta, hipStream_t stream) {
  const size_t ntiles = TileCount(nbytes);
  CHECK(tile_masks != nullptr) << "LaunchTileCountScan: tile_masks (TileMaskWords) is required";
  if (ntiles != 0) {
    const size_t per_block = kThreads / dev::kWave;
    hipLaunchKernelGGL(k_tile_count, dim3((ntiles + per_block - 1) / per_block), dim3(kThreads), 0,
                       stream, reinterpret_cast<const uint8_t*>(text), nbytes, ntiles, tile_counts,
                       tile_flags, reinterpret_cast<uint2*>(tile_masks));
  }
  TileScan(tile_counts, tile_flags, ntiles, meta, host_meta, 0, stream);
}

void LaunchTileScanRaw(uint64_t* tile_counts, uint32_t* tile_flags, size_t ntiles,
                       ChunkMeta* meta, ChunkMeta* host_meta, hipStream_t stream) {
  TileScan(tile_counts, tile_flags, ntiles, meta, host_meta, 1, stream);
}

void LaunchTileFinish(MetaPartial* partials, size_t nslots, ChunkMeta* meta, ChunkMeta* host_meta,
                      uint64_t* offset, uint64_t row_base, uint64_t nnz_base, hipStream_t stream) {
  LaunchFinish(partials, nslots, meta, host_meta, offset, row_base, nnz_base, stream);
}

size_t TileScratchWords(size_t ntiles) {
  return ntiles + (ntiles + kScanBlockTiles - 1) / kScanBlockTiles + 64;
}

size_t TileScratchSlots(size_t ntiles) { return ntiles + kFinishGroups; }

size_t TileMaskWords(size_t ntiles) { return ntiles * (kTileBytes / 16); }

template <typename IndexType>
size_t LaunchTileFill(const char* text, size_t nbytes, TextFormat format,
                      const uint64_t* tile_prefix, const uint32_t* tile_masks,
                      const FillTarget<IndexType>& out, MetaPartial* partials, ChunkMeta* meta,
                      ChunkMeta* host_meta, hipStream_t stream, const FillOnePass* one_pass) {
  const size_t ntiles = TileCount(nbytes);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  const size_t groups = (ntiles + kFillWaves - 1) / kFillWaves;
  static const uint32_t exp = [] {
    const char* v = std::getenv("DMLC_FILL_EXP");
    return v != nullptr ? static_cast<uint32_t>(std::atoi(v)) : 0u;
  }();
  FillPass op{nullptr, nullptr, 0ull, meta, exp, tile_masks};
  CHECK(one_pass != nullptr || tile_masks != nullptr || ntiles == 0)
      << "LaunchTileFill: the counted path needs C1's tile_masks";
  if (one_pass != nullptr) {
    op.status = one_pass->status;
    op.ticket = one_pass->ticket;
    op.ticket0 = one_pass->ticket0;
    // every look-back word starts "not yet" (cdna_hip_programming.md G16:
    // zero every polled word before every launch)
    DMLC_HIP_CHECK(hipMemsetAsync(op.status, 0, ntiles * sizeof(uint64_t), stream));
  }
  if (ntiles != 0) {
    const dim3 grid(static_cast<unsigned>(groups));
#define DMLC_TILE_FILL(FMT, ONE, LEAN)                                                       \
  hipLaunchKernelGGL((k_tile_fill<FMT, IndexType, ONE, LEAN>), grid, dim3(kThreads), 0, stream, t, \
                     nbytes, ntiles, tile_prefix, out, partials, op)
    // counted path without qid / weight columns: the lean instantiation
    const bool lean = one_pass == nullptr && out.qid == nullptr && out.weight == nullptr;
    if (format == TextFormat::kLibFM) {
      if (one_pass != nullptr) {
        DMLC_TILE_FILL(TextFormat::kLibFM, true, false);
      } else if (lean) {
        DMLC_TILE_FILL(TextFormat::kLibFM, false, true);
      } else {
        DMLC_TILE_FILL(TextFormat::kLibFM, false, false);
      }
    } else if (one_pass != nullptr) {
      DMLC_TILE_FILL(TextFormat::kLibSVM, true, false);
    } else if (lean) {
      DMLC_TILE_FILL(TextFormat::kLibSVM, false, true);
    } else {
      DMLC_TILE_FILL(TextFormat::kLibSVM, false, false);
    }
#undef DMLC_TILE_FILL
  }
  LaunchFinish(partials, ntiles, meta, host_meta, out.offset, out.row_base, out.nnz_base, stream);
  return ntiles != 0 ? groups : 0;
}

template <typename IndexType>
size_t LaunchTileHashed(const char* text, size_t nbytes, TextFormat format,
                        const uint64_t* tile_prefix, const uint32_t* tile_masks,
                        uint64_t row_base, uint64_t nlines, int dim,
                        float scale, uint32_t seed, bool fp8, void* out, float* labels,
                        MetaPartial* partials, ChunkMeta* meta, ChunkMeta* host_meta,
                        hipStream_t stream, const HashOnePass* one_pass) {
  const size_t ntiles = TileCount(nbytes);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  const size_t smem = static_cast<size_t>(kFillWaves) * dim * sizeof(float);
  HashTarget tgt{out, labels, row_base, nlines, dim, scale, seed, 0u, nullptr, nullptr, 0ull, 0ull,
                 meta, tile_masks};
  CHECK(one_pass != nullptr || tile_masks != nullptr || ntiles == 0)
      << "LaunchTileHashed: the counted path needs C1's tile_masks";
  const size_t groups = (ntiles + kFillWaves - 1) / kFillWaves;
  if (one_pass != nullptr) {
    tgt.tag = one_pass->tag;
    tgt.status = one_pass->status;
    tgt.ticket = one_pass->ticket;
    tgt.ticket0 = one_pass->ticket0;
    tgt.row_cap = one_pass->row_cap;
  }
  if (ntiles != 0) {
    const dim3 grid(static_cast<unsigned>(groups));
#define DMLC_TILE_HASH(FMT, FP8, ONE)                                                          \
  hipLaunchKernelGGL((k_tile_hash<FMT, IndexType, FP8, ONE>), grid, dim3(kThreads), smem, stream, \
                     t, nbytes, ntiles, tile_prefix, tgt, partials)
#define DMLC_TILE_HASH_FMT(FMT)             \
  if (one_pass != nullptr) {                \
    if (fp8) {                              \
      DMLC_TILE_HASH(FMT, true, true);      \
    } else {                                \
      DMLC_TILE_HASH(FMT, false, true);     \
    }                                       \
  } else if (fp8) {                         \
    DMLC_TILE_HASH(FMT, true, false);       \
  } else {                                  \
    DMLC_TILE_HASH(FMT, false, false);      \
  }
    if (format == TextFormat::kLibFM) {
      DMLC_TILE_HASH_FMT(TextFormat::kLibFM)
    } else {
      DMLC_TILE_HASH_FMT(TextFormat::kLibSVM)
    }
#undef DMLC_TILE_HASH_FMT
#undef DMLC_TILE_HASH
  }
  LaunchFinish(partials, ntiles, meta, host_meta, nullptr, 0ull, 0ull, stream);
  return ntiles != 0 ? groups : 0;
}

template size_t LaunchTileHashed<uint32_t>(const char*, size_t, TextFormat, const uint64_t*,
                                           const uint32_t*, uint64_t, uint64_t, int, float, uint32_t,
                                           bool, void*, float*, MetaPartial*, ChunkMeta*, ChunkMeta*,
                                           hipStream_t, const HashOnePass*);
template size_t LaunchTileHashed<uint64_t>(const char*, size_t, TextFormat, const uint64_t*,
                                           const uint32_t*, uint64_t, uint64_t, int, float, uint32_t,
                                           bool, void*, float*, MetaPartial*, ChunkMeta*, ChunkMeta*,
                                           hipStream_t, const HashOnePass*);

template size_t LaunchTileFill<uint32_t>(const char*, size_t, TextFormat, const uint64_t*,
                                         const uint32_t*, const FillTarget<uint32_t>&, MetaPartial*,
                                         ChunkMeta*, ChunkMeta*, hipStream_t, const FillOnePass*);
template size_t LaunchTileFill<uint64_t>(const char*, size_t, TextFormat, const uint64_t*,
                                         const uint32_t*, const FillTarget<uint64_t>&, MetaPartial*,
                                         ChunkMeta*, ChunkMeta*, hipStream_t, const FillOnePass*);

}  // namespace gpu
}  // namespace dmlc
