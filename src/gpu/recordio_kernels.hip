/*!
 * \file src/gpu/recordio_kernels.hip
 * \brief K7: RecordIO decode on the GPU, on the tile pipeline of the text
 *  parser (count -> two-level scan -> fill -> finish, sizes published to
 *  mapped pinned memory).
 *
 * Replaces the host record walk of RecordIOSplitter::ExtractNextRecord /
 * RecordIOChunkReader (reference `src/io/recordio_split.cc:44-82`,
 * `src/recordio.cc:85-156`).  The writer escapes every 4-byte-aligned
 * occurrence of the magic word inside a payload (`src/recordio.cc:22-38`), so
 * in a chunk that starts at a record head every aligned magic word is a part
 * header (an lrec can never equal the magic: its cflag would be 6).  Each part
 * is self-describing -- cflag 0 whole record, 1 first / 2 middle / 3 last part
 * -- and contributes len payload bytes, plus the 4-byte magic the reader
 * re-inserts in front of a continuation part.  So with per-tile prefix sums
 * of (record heads, output bytes) every part knows where its bytes go,
 * without walking chains:
 *
 *   R1 k_rec_tile_count: one wave per 1024-word (4 KiB) tile, 4 coalesced
 *      16 B loads per lane in flight; (heads << 32 | bytes) per tile and
 *      error bits (a part running past the chunk, a bad cflag).
 *   C2 (tile_kernels.hip, raw mode): exclusive scan, totals published.
 *   R2 k_rec_tile_fill: the same tile walk; per 1 KiB sub-tile a wave scan
 *      places each part; head parts write their record's offset; parts up to
 *      64 B are copied by the lane that found them, longer ones go to a
 *      wave-private LDS list and are copied by the whole wave (16 B per lane
 *      when source and destination allow it).  Every part checks the part
 *      that follows it (a continuation must follow a first / middle part,
 *      a head must follow a whole / last part).
 *   C4 (tile_kernels.hip): error bits folded, closing offset, published.
 *   One pass (HBM-resident replays): R2 with R1 inside -- each wave counts
 *      its tile from the words it already holds and takes the tiles before it
 *      by decoupled look-back, so a replayed chunk is one launch that reads
 *      the text once (the payload copies read the LDS-staged tile).
 *   R3 k_rec_gather: device gather of whole records (header included) into a
 *      contiguous batch -- the shuffled indexed-RecordIO epochs gather their
 *      batches from the HBM-resident partition with it.
 */
#include <dmlc/gpu/hip_utils.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {
namespace {

using namespace dev;  // NOLINT(build/namespaces)

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kMagic = 0xced7230aU;
constexpr size_t kTileWords = 1024;  // 4 loads x 64 lanes x 4 words
constexpr int kLoads = static_cast<int>(kTileWords / 256);
constexpr uint32_t kSmallPart = 64;  // bytes copied lane-by-lane
// parts > 64 B whose header lies in a tile: headers >= 19 words apart (2 + 17),
// so at most 54 in 1024 words.  4 KiB tiles keep the fill at 20 KiB of LDS
// and 68 VGPRs per wave: 7 waves per SIMD (8 KiB tiles: 40 KiB, 88 VGPRs, 4)
constexpr int kBigCap = 56;
static_assert(kBigCap * 19 >= static_cast<int>(kTileWords) + 19, "kBigCap too small");

__device__ __forceinline__ uint32_t cflag_of(uint32_t lrec) { return lrec >> 29; }
__device__ __forceinline__ uint32_t len_of(uint32_t lrec) { return lrec & ((1U << 29) - 1U); }

__device__ __forceinline__ uint4 load_quad(const uint32_t* __restrict__ w, size_t n, size_t i0) {
  if (i0 + 4 <= n) return *reinterpret_cast<const uint4*>(w + i0);
  uint4 q = make_uint4(0, 0, 0, 0);
  if (i0 < n) q.x = w[i0];
  if (i0 + 1 < n) q.y = w[i0 + 1];
  if (i0 + 2 < n) q.z = w[i0 + 2];
  return q;
}

/*! \brief part headers of one lane's quad: bit k = word k is a part header */
__device__ __forceinline__ uint32_t header_bits(uint4 q, size_t i0, size_t n) {
  uint32_t m = 0;
  m |= (q.x == kMagic && i0 + 1 < n) ? 1u : 0u;
  m |= (q.y == kMagic && i0 + 2 < n) ? 2u : 0u;
  m |= (q.z == kMagic && i0 + 3 < n) ? 4u : 0u;
  m |= (q.w == kMagic && i0 + 4 < n) ? 8u : 0u;
  return m;
}

__device__ __forceinline__ uint32_t quad_word(uint4 q, uint32_t k) {
  return k == 0 ? q.x : (k == 1 ? q.y : (k == 2 ? q.z : q.w));
}

/*! \brief lrec of the header at word k of the quad (k < 3: same quad; 3: `after`) */
__device__ __forceinline__ uint32_t lrec_at(uint4 q, uint32_t k, uint32_t after) {
  return k == 0 ? q.y : (k == 1 ? q.z : (k == 2 ? q.w : after));
}

/*!
 * \brief the tile's 8 quads of this lane and, for each, the word after its
 *  last word (lane + 1's first word; lane 63 takes the next load's lane 0,
 *  the tile's last lane reads past the tile)
 */
struct TileQuads {
  uint4 q[kLoads];
  uint32_t after[kLoads];
};

__device__ __forceinline__ void load_tile(const uint32_t* __restrict__ w, size_t n, size_t base,
                                          int lane, TileQuads* t) {
#pragma unroll
  for (int j = 0; j < kLoads; ++j) t->q[j] = load_quad(w, n, base + j * 256 + lane * 4);
  const size_t past = base + kTileWords;
  const uint32_t tail = past < n ? w[past] : 0u;
#pragma unroll
  for (int j = 0; j < kLoads; ++j) {
    const uint32_t right = lane_shl1(t->q[j].x);
    // every lane runs the cross-lane ops (under a lane condition they would
    // read an inactive lane)
    const uint32_t next0 = __builtin_amdgcn_readlane(t->q[j + 1 < kLoads ? j + 1 : j].x, 0);
    const uint32_t wrap = j + 1 < kLoads ? next0 : tail;
    t->after[j] = lane == kWave - 1 ? wrap : right;
  }
}

/*! \brief (heads << 32 | bytes) and error bits of the parts headed in one quad */
__device__ __forceinline__ uint64_t quad_counts(uint4 q, uint32_t after, size_t i0, size_t n,
                                                uint32_t* err) {
  uint32_t m = header_bits(q, i0, n);
  uint32_t heads = 0, bytes = 0;
  while (m != 0) {
    const uint32_t k = static_cast<uint32_t>(__ffs(m) - 1);
    m &= m - 1;
    const uint32_t lrec = lrec_at(q, k, after);
    const uint32_t cf = cflag_of(lrec), len = len_of(lrec);
    heads += cf <= 1 ? 1u : 0u;
    bytes += len + (cf >= 2 ? 4u : 0u);
    if (cf > 3) *err |= kRecErrBadPart;
    if (i0 + k + 2 + (static_cast<size_t>(len) + 3) / 4 > n) *err |= kRecErrTruncated;
  }
  return (static_cast<uint64_t>(heads) << 32) | bytes;
}

__global__ __launch_bounds__(kThreads) void k_rec_tile_count(const uint32_t* __restrict__ w,
                                                             size_t n, size_t ntiles,
                                                             uint64_t* __restrict__ counts,
                                                             uint32_t* __restrict__ flags) {
  const int lane = lane_id();
  const size_t tile = static_cast<size_t>(blockIdx.x) * kWaves + threadIdx.x / kWave;
  if (tile >= ntiles) return;  // whole waves leave; nothing below synchronises waves
  const size_t base = tile * kTileWords;
  TileQuads t;
  load_tile(w, n, base, lane, &t);
  uint64_t c = 0;
  uint32_t err = 0;
#pragma unroll
  for (int j = 0; j < kLoads; ++j) c += quad_counts(t.q[j], t.after[j], base + j * 256 + lane * 4, n, &err);
  // a chunk starts at a record head
  if (tile == 0 && lane == 0 && n != 0 && !(t.q[0].x == kMagic && n > 1 && cflag_of(t.q[0].y) <= 1))
    err |= kRecErrBadPart;
  c = wave_sum_2x32(c);  // heads << 32 | bytes: no carries
  err = wave_or(err);
  if (lane == 0) {
    counts[tile] = c;
    flags[tile] = err;
  }
}

/*!
 * \brief R1c: the same (heads << 32 | bytes) per tile as R1 from the part
 *  headers alone.  Lane per tile: the first aligned magic at or after the
 *  tile start is a part header (the writer escapes aligned magics inside
 *  payloads), and each header gives the next (h + 2 + ceil(len / 4) words),
 *  so a tile costs its first-header search plus one 8-byte read per part
 *  instead of reading every word: 512-byte records read ~2 % of the chunk.
 *  Latency-bound (one dependent read per part), so the host takes it for
 *  parts of >= 128 bytes on average.  A chain that does not land on a magic
 *  word is an error (R1 would count a different set of headers); the fill
 *  checks its own tile totals against the prefix, so an R1c / R2 mismatch is
 *  an error too, never a misplaced write.
 */
__global__ __launch_bounds__(kThreads) void k_rec_tile_count_chain(const uint32_t* __restrict__ w,
                                                                   size_t n, size_t ntiles,
                                                                   uint32_t per_lane,
                                                                   uint64_t* __restrict__ counts,
                                                                   uint32_t* __restrict__ flags) {
  // a lane takes per_lane consecutive tiles: one first-header search, then the
  // chain runs on across its tiles (the header after a tile's last part is
  // the next tile's first), counts binned by the tile of each header
  const size_t t0 = (static_cast<size_t>(blockIdx.x) * kThreads + threadIdx.x) * per_lane;
  if (t0 >= ntiles) return;
  const size_t t1 = t0 + per_lane < ntiles ? t0 + per_lane : ntiles;
  const size_t base = t0 * kTileWords;
  const size_t end = t1 * kTileWords < n ? t1 * kTileWords : n;
  // the first header: 16 words (4 loads in flight) per step
  size_t h = end;
  for (size_t i = base; i < end && h == end; i += 16) {
    uint4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = load_quad(w, n, i + 4 * k);
#pragma unroll
    for (int k = 3; k >= 0; --k) {
      const uint32_t m = header_bits(q[k], i + 4 * k, n);
      if (m != 0) h = i + 4 * k + static_cast<uint32_t>(__ffs(m) - 1);
    }
    if (h > end) h = end;
  }
  size_t tile = t0;  // the tile being binned
  uint32_t heads = 0, bytes = 0, err = 0;
  auto emit_to = [&](size_t upto) {  // close tiles [tile, upto)
    for (; tile < upto; ++tile) {
      counts[tile] = (static_cast<uint64_t>(heads) << 32) | bytes;
      flags[tile] = err;
      heads = bytes = err = 0;
    }
  };
  // a chunk starts at a record head
  if (t0 == 0 && n != 0 && h != 0) err |= kRecErrBadPart;
  while (h < end) {  // h + 1 < n: a header (search) or checked below
    emit_to(h / kTileWords);
    const uint32_t magic = w[h], lrec = w[h + 1];
    if (magic != kMagic) {
      err |= kRecErrBadPart;
      break;
    }
    const uint32_t cf = cflag_of(lrec), len = len_of(lrec);
    if (h == 0 && cf > 1) err |= kRecErrBadPart;
    heads += cf <= 1 ? 1u : 0u;
    bytes += len + (cf >= 2 ? 4u : 0u);
    if (cf > 3) err |= kRecErrBadPart;
    const size_t q = h + 2 + (static_cast<size_t>(len) + 3) / 4;
    if (q > n) {
      err |= kRecErrTruncated;
      break;
    }
    // a successor inside the range must be a full header (R1 counts no
    // header in the chunk's last word; the fill flags that chain)
    if (q < end && q + 1 >= n) break;
    h = q;
  }
  emit_to(t1);
}

/*! \brief copy len payload bytes of words src to byte address dst (one lane) */
__device__ __forceinline__ void lane_copy(const uint32_t* __restrict__ src, uint32_t len,
                                          uint8_t* __restrict__ dst) {
  const uint32_t nw = len / 4;
  if ((reinterpret_cast<uintptr_t>(dst) & 3U) == 0) {
    for (uint32_t j = 0; j < nw; ++j) reinterpret_cast<uint32_t*>(dst)[j] = src[j];
  } else {
    for (uint32_t j = 0; j < nw; ++j) {
      const uint32_t v = src[j];
#pragma unroll
      for (int b = 0; b < 4; ++b) dst[4 * j + b] = static_cast<uint8_t>(v >> (8 * b));
    }
  }
  const uint32_t rest = len & 3U;
  if (rest != 0) {
    const uint32_t v = src[nw];
    for (uint32_t b = 0; b < rest; ++b) dst[4 * nw + b] = static_cast<uint8_t>(v >> (8 * b));
  }
}

struct BigPart {
  uint32_t word;  // chunk word index of the header
  uint32_t len;
  uint64_t dst;   // output byte position (chunk-relative, after the re-inserted magic)
};

/*! \brief the one-pass fill's look-back state (kOnePass) */
struct RecPass {
  uint64_t* status;            // per-tile look-back words, zeroed before the launch
  unsigned long long* ticket;  // workgroup ticket counter
  unsigned long long ticket0;  // its value at this launch
  ChunkMeta* meta;             // records / bytes of the chunk (the last tile writes them)
  uint64_t rec_cap, byte_cap;  // offset / data capacity: records / bytes past them are not
                               // written and set kFlagOverflow (grow, run again)
  uint32_t exp;                // pricing experiments (DMLC_REC_EXP; 0 in production): 1 no
                               // look-back wait (wrong positions), 2 no payload copies
};

template <bool kOnePass>
__global__ __launch_bounds__(kThreads) void k_rec_tile_fill(const uint32_t* __restrict__ w,
                                                            size_t n, size_t ntiles,
                                                            const uint64_t* __restrict__ prefix,
                                                            uint64_t* __restrict__ offset,
                                                            uint64_t rec_base,
                                                            uint8_t* __restrict__ data,
                                                            uint64_t byte_base,
                                                            MetaPartial* __restrict__ partials,
                                                            RecPass op) {
  __shared__ BigPart s_big[kWaves][kBigCap];
  // the tile's words (+ the one after it): a part's successor check reads its
  // header from here instead of a dependent global load per part, and the
  // payload copies read their source from here (the text is read from
  // memory once)
  __shared__ uint4 s_tw[kWaves][kTileWords / 4 + 1];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  size_t group = blockIdx.x;
  if constexpr (kOnePass) {
    // tiles in ticket order: a workgroup looks back only at tiles of
    // workgroups that started before it, so every tile it waits on is
    // resident or done
    __shared__ uint32_t s_ticket;
    if (threadIdx.x == 0) s_ticket = static_cast<uint32_t>(atomicAdd(op.ticket, 1ull) - op.ticket0);
    __syncthreads();
    group = s_ticket;
  }
  const size_t tile = group * kWaves + wave;
  if (tile >= ntiles) return;  // whole waves leave; nothing below synchronises waves
  BigPart* big = s_big[wave];
  const size_t base = tile * kTileWords;
  TileQuads t;
  load_tile(w, n, base, lane, &t);
  uint32_t* const tw = reinterpret_cast<uint32_t*>(s_tw[wave]);
#pragma unroll
  for (int j = 0; j < kLoads; ++j) s_tw[wave][j * 64 + lane] = t.q[j];
  if (lane == kWave - 1) tw[kTileWords] = t.after[kLoads - 1];
  wave_sync();
  // word q of the chunk (q < n): staged when inside the tile (+1), else global
  auto word_at = [&](size_t q) {
    const size_t r = q - base;
    return r <= kTileWords ? tw[r] : w[q];
  };
  uint64_t pre;
  uint32_t err = 0;
  if constexpr (kOnePass) {
    // R1 in the fill: the tile's (heads, bytes) from the registers it already
    // holds, then the look-back for the tiles before it (heads < 2^30 and
    // bytes < 2^32 in a chunk < 4 GiB: a 30 / 32-bit pair)
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < kLoads; ++j) {
      c += quad_counts(t.q[j], t.after[j], base + j * 256 + lane * 4, n, &err);
    }
    if (tile == 0 && lane == 0 && n != 0 && !(t.q[0].x == kMagic && n > 1 && cflag_of(t.q[0].y) <= 1))
      err |= kRecErrBadPart;  // a chunk starts at a record head
    c = wave_sum_2x32(c);
    if (op.exp & 1u) {
      pre = static_cast<uint64_t>(tile) * c;  // pricing: positions without the look-back
    } else {
      pre = lookback_pairs<32>(op.status, tile, c, lane);
    }
    if (tile + 1 == ntiles && lane == 0) {
      ChunkMeta m;
      m.nlines = m.nrows = (pre + c) >> 32;
      m.nnz = (pre + c) & 0xffffffffull;
      m.max_index = m.max_field = 0;
      m.flags = 0;
      m.pad = 0;
      *op.meta = m;  // k_tile_finish (stream-ordered) adds the error bits, publishes
    }
  } else {
    pre = prefix[tile];
  }
  uint64_t rec = pre >> 32;            // records before this 1 KiB sub-tile (chunk-relative)
  uint64_t pos = pre & 0xffffffffull;  // output bytes before it
  uint8_t* const out = data + byte_base;
  bool over = false;
  uint32_t nbig = 0;
#pragma unroll
  for (int j = 0; j < kLoads; ++j) {
    const size_t i0 = base + j * 256 + lane * 4;
    uint32_t unused = 0;
    const uint64_t c = quad_counts(t.q[j], t.after[j], i0, n, &unused);
    uint64_t tot;
    const uint64_t before = wave_excl_scan_2x32(c, &tot);  // heads << 32 | bytes
    uint64_t r = rec + (before >> 32);
    uint64_t p = pos + (before & 0xffffffffull);
    // parts of more than 64 B are > 16 words apart: at most one per quad
    bool has_big = false;
    BigPart mine{0, 0, 0};
    uint32_t m = header_bits(t.q[j], i0, n);
    while (m != 0) {
      const uint32_t k = static_cast<uint32_t>(__ffs(m) - 1);
      m &= m - 1;
      const uint32_t lrec = lrec_at(t.q[j], k, t.after[j]);
      const uint32_t cf = cflag_of(lrec), len = len_of(lrec);
      const size_t i = i0 + k;
      {
        // the part that follows: a continuation must follow a first / middle
        // part, a head a whole / last part (read from the staged words)
        const size_t q = i + 2 + (static_cast<size_t>(len) + 3) / 4;
        const bool ends_record = cf == 0 || cf == 3;
        if (q > n) {
          err |= kRecErrTruncated;
        } else if (q == n) {
          err |= ends_record ? 0u : kRecErrTruncated;
        } else if (q + 1 >= n || word_at(q) != kMagic) {
          err |= kRecErrBadPart;
        } else {
          const uint32_t next = cflag_of(word_at(q + 1));
          const bool next_continues = next == 2 || next == 3;
          err |= (ends_record == next_continues || next > 3) ? kRecErrBadPart : 0u;
        }
      }
      // writes stay inside the capacity given (one pass: overflow -> grow ->
      // rerun; counted: sized exactly, so a miss is a count / fill mismatch)
      // (a head takes an offset slot, a continuation its re-inserted magic)
      const bool fits = (cf >= 2 || rec_base + r < op.rec_cap) &&
                        byte_base + p + len + (cf >= 2 ? 4u : 0u) <= op.byte_cap;
      over |= !fits;
      if (cf <= 1) {
        if (fits) offset[rec_base + r] = byte_base + p;
        ++r;
      } else {
        // the reader re-inserts the escaped magic in front of a continuation
        if (fits) {
#pragma unroll
          for (int b = 0; b < 4; ++b) out[p + b] = static_cast<uint8_t>(kMagic >> (8 * b));
        }
        p += 4;
      }
      const bool whole = fits && i + 2 + (static_cast<size_t>(len) + 3) / 4 <= n;  // else: truncated
      if (whole && len <= kSmallPart) {
        lane_copy(w + i + 2, len, out + p);
      } else if (whole) {
        has_big = true;
        mine = BigPart{static_cast<uint32_t>(i), len, p};
      }
      p += len;
    }
    const uint64_t bigs = __ballot(has_big);
    if (has_big) {
      const uint32_t slot = nbig + __builtin_amdgcn_mbcnt_hi(
                                       static_cast<uint32_t>(bigs >> 32),
                                       __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bigs), 0u));
      big[slot] = mine;
    }
    nbig += static_cast<uint32_t>(__popcll(bigs));
    rec += tot >> 32;
    pos += tot & 0xffffffffull;
  }
  wave_sync();  // the list is visible to every lane
  // the listed parts (> 64 B), two at a time: half-wave h copies part e0 + h.
  // Destinations are any byte offset (a continuation's re-inserted magic
  // shifts every later part by 4, odd payload lengths by anything), so each
  // part is written as its head bytes up to the first 16-byte boundary, whole
  // aligned 16-byte blocks (one dwordx4 store per lane) and its tail bytes;
  // a block's 16 source bytes are five payload words funnel-shifted into
  // place, read from the LDS-staged tile (or from memory past the tile).
  const int hl = lane & 31;
  for (uint32_t e0 = 0; e0 < ((op.exp & 2u) ? 0u : nbig); e0 += 2) {
    const uint32_t e = e0 + static_cast<uint32_t>(lane >> 5);
    if (e < nbig) {
      const BigPart bp = big[e];
      uint8_t* const d = out + bp.dst;
      const uint32_t head = (16u - static_cast<uint32_t>(reinterpret_cast<uintptr_t>(d) & 15u)) & 15u;
      const uint32_t h = head < bp.len ? head : bp.len;
      const uint32_t nblk = (bp.len - h) / 16;
      const uint32_t tail = bp.len - h - nblk * 16;
      const size_t pw = static_cast<size_t>(bp.word) + 2;  // chunk word of payload byte 0
      // payload word j: staged when inside the tile (+1), else from memory
      auto pword = [&](uint32_t j) {
        const size_t q = pw + j;
        return q - base <= kTileWords ? tw[q - base] : w[q];
      };
      auto pbyte = [&](uint32_t o) { return static_cast<uint8_t>(pword(o >> 2) >> (8 * (o & 3u))); };
      for (uint32_t b = static_cast<uint32_t>(hl); b < nblk; b += 32) {
        const uint32_t o = h + 16 * b;  // payload byte of the block's first byte
        const uint32_t j = o >> 2, r = o & 3u;
        const uint32_t w0 = pword(j), w1 = pword(j + 1), w2 = pword(j + 2), w3 = pword(j + 3);
        // (the fifth word only when the block is not word-aligned: it may lie
        // past the payload's last word, so it is not read otherwise)
        const uint32_t w4 = r != 0 ? pword(j + 4) : 0u;
        *reinterpret_cast<uint4*>(d + o) =
            make_uint4(__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
                       __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r));
      }
      if (static_cast<uint32_t>(hl) < h) d[hl] = pbyte(static_cast<uint32_t>(hl));
      if (static_cast<uint32_t>(hl) < tail) {
        const uint32_t o = h + nblk * 16 + static_cast<uint32_t>(hl);
        d[o] = pbyte(o);
      }
    }
  }
  if constexpr (!kOnePass) {
    // the tile's own parts must end where the count said the next tile
    // starts (R1c follows chains; R2 sees every aligned magic)
    if (op.meta != nullptr && lane == 0) {
      const uint64_t want = tile + 1 < ntiles ? prefix[tile + 1]
                                              : ((static_cast<uint64_t>(op.meta->nrows) << 32) |
                                                 op.meta->nnz);
      if (((rec << 32) | pos) != want) err |= kRecErrBadPart;
    }
    if (over) err |= kRecErrBadPart;
    over = false;
  }
  err = wave_or(err | (over ? kFlagOverflow : 0u));
  if (lane == 0) {
    MetaPartial mp;
    mp.max_index = 0;
    mp.max_field = 0;
    mp.flags = err;
    mp.pad = 0;
    partials[tile] = mp;
  }
}

/*!
 * \brief R3: record k of the batch = the n_k bytes at src + src_off[k] (a
 *  whole RecordIO record: header, payload, padding -- 4-byte multiples),
 *  copied to dst + dst_off[k]; one wave per record, 16 B per lane when both
 *  ends are 16-byte aligned
 */
__global__ __launch_bounds__(kThreads) void k_rec_gather(const uint8_t* __restrict__ src,
                                                         const uint64_t* __restrict__ src_off,
                                                         const uint32_t* __restrict__ len,
                                                         const uint64_t* __restrict__ dst_off,
                                                         size_t nrec, uint8_t* __restrict__ dst) {
  const size_t k = static_cast<size_t>(blockIdx.x) * kWaves + threadIdx.x / kWave;
  if (k >= nrec) return;
  const int lane = lane_id();
  const uint8_t* s = src + src_off[k];
  uint8_t* d = dst + dst_off[k];
  const uint32_t n = len[k];
  if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15U) == 0) {
    for (uint32_t c = lane; c < n / 16; c += kWave) {
      reinterpret_cast<uint4*>(d)[c] = reinterpret_cast<const uint4*>(s)[c];
    }
    for (uint32_t c = (n / 16) * 4 + lane; c < n / 4; c += kWave) {
      reinterpret_cast<uint32_t*>(d)[c] = reinterpret_cast<const uint32_t*>(s)[c];
    }
  } else {
    for (uint32_t c = lane; c < n / 4; c += kWave) {
      reinterpret_cast<uint32_t*>(d)[c] = reinterpret_cast<const uint32_t*>(s)[c];
    }
  }
}

}  // namespace

size_t RecordIOTiles(size_t nwords) { return (nwords + kTileWords - 1) / kTileWords; }

void LaunchRecordIOTileCount(const uint32_t* words, size_t nwords, uint64_t* tile_counts,
                             uint32_t* tile_flags, hipStream_t stream) {
  const size_t tiles = RecordIOTiles(nwords);
  if (tiles == 0) return;
  hipLaunchKernelGGL(k_rec_tile_count, dim3((tiles + kWaves - 1) / kWaves), dim3(kThreads), 0,
                     stream, words, nwords, tiles, tile_counts, tile_flags);
}

void LaunchRecordIOTileCountChain(const uint32_t* words, size_t nwords, uint64_t* tile_counts,
                                  uint32_t* tile_flags, hipStream_t stream) {
  const size_t tiles = RecordIOTiles(nwords);
  if (tiles == 0) return;
  // large pieces (counted beside a fill): up to 16 tiles per lane, so the
  // latency-bound chain waves hold few CU slots; small ones: a lane per tile
  // (DMLC_REC_CHAIN_TILES forces a tiles-per-lane value: the tests' small
  // chunks exercise the multi-tile walk with it)
  static const size_t forced = [] {
    const char* v = std::getenv("DMLC_REC_CHAIN_TILES");
    return v != nullptr ? static_cast<size_t>(std::atoi(v)) : size_t(0);
  }();
  // (64 KiB of text per lane on pieces of >= 1 GiB)
  size_t per = 1;
  while (per < 16 && tiles >= per * 2 * 16384) per *= 2;
  if (forced != 0) per = forced;
  const size_t lanes = (tiles + per - 1) / per;
  hipLaunchKernelGGL(k_rec_tile_count_chain, dim3((lanes + kThreads - 1) / kThreads),
                     dim3(kThreads), 0, stream, words, nwords, tiles, static_cast<uint32_t>(per),
                     tile_counts, tile_flags);
}

size_t LaunchRecordIOTileFill(const uint32_t* words, size_t nwords, const uint64_t* tile_prefix,
                              uint64_t* offset, uint64_t rec_base, uint8_t* data,
                              uint64_t byte_base, MetaPartial* partials, hipStream_t stream,
                              const RecordIOOnePass* one_pass, const RecordIOCaps* caps) {
  const size_t tiles = RecordIOTiles(nwords);
  if (tiles == 0) return 0;
  const size_t groups = (tiles + kWaves - 1) / kWaves;
  static const uint32_t exp = [] {
    const char* v = std::getenv("DMLC_REC_EXP");
    return v != nullptr ? static_cast<uint32_t>(std::atoi(v)) : 0u;
  }();
  RecPass op{nullptr, nullptr, 0ull, nullptr, ~0ull, ~0ull, exp};
  if (caps != nullptr) {
    op.meta = caps->meta;
    op.rec_cap = caps->rec_cap;
    op.byte_cap = caps->byte_cap;
  }
  if (one_pass != nullptr) {
    op = RecPass{one_pass->status, one_pass->ticket, one_pass->ticket0, one_pass->meta,
                 one_pass->rec_cap, one_pass->byte_cap, exp};
    // every look-back word starts "not yet" (zeroed before every launch)
    DMLC_HIP_CHECK(hipMemsetAsync(op.status, 0, tiles * sizeof(uint64_t), stream));
    hipLaunchKernelGGL(k_rec_tile_fill<true>, dim3(groups), dim3(kThreads), 0, stream, words,
                       nwords, tiles, tile_prefix, offset, rec_base, data, byte_base, partials, op);
  } else {
    hipLaunchKernelGGL(k_rec_tile_fill<false>, dim3(groups), dim3(kThreads), 0, stream, words,
                       nwords, tiles, tile_prefix, offset, rec_base, data, byte_base, partials, op);
  }
  return groups;
}

void LaunchRecordIOGather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                          const uint64_t* dst_off, size_t nrec, uint8_t* dst, hipStream_t stream) {
  if (nrec == 0) return;
  hipLaunchKernelGGL(k_rec_gather, dim3((nrec + kWaves - 1) / kWaves), dim3(kThreads), 0, stream,
                     src, src_off, len, dst_off, nrec, dst);
}

}  // namespace gpu
}  // namespace dmlc
