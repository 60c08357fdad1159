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
 *   R1 k_rec_tile_count: one wave per 2048-word (8 KiB) tile, 8 coalesced
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
 *   R3 k_rec_gather: device gather of whole records (header included) into a
 *      contiguous batch -- the shuffled indexed-RecordIO epochs gather their
 *      batches from the HBM-resident partition with it.
 */
#include <hip/hip_runtime.h>

#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {
namespace {

using namespace dev;  // NOLINT(build/namespaces)

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kMagic = 0xced7230aU;
constexpr size_t kTileWords = 2048;  // 8 loads x 64 lanes x 4 words
constexpr int kLoads = static_cast<int>(kTileWords / 256);
constexpr uint32_t kSmallPart = 64;  // bytes copied lane-by-lane
// parts > 64 B whose header lies in a tile: headers >= 19 words apart (2 + 17),
// so at most 108 in 2048 words.  112 keeps the fill at 40 KiB of LDS per
// workgroup: 4 workgroups per CU (kTileWords / 16 = 128 made it 3)
constexpr int kBigCap = 112;
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

/*! \brief the whole wave copies len bytes of words src to byte address dst */
__device__ __forceinline__ void wave_copy(const uint32_t* __restrict__ src, uint32_t len,
                                          uint8_t* __restrict__ dst, int lane) {
  const uintptr_t da = reinterpret_cast<uintptr_t>(dst);
  const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
  uint32_t done = 0;
  if ((da & 15U) == 0 && (sa & 15U) == 0) {
    const uint32_t n16 = len / 16;
    for (uint32_t c = lane; c < n16; c += kWave) {
      reinterpret_cast<uint4*>(dst)[c] = reinterpret_cast<const uint4*>(src)[c];
    }
    done = n16 * 16;
  } else if ((da & 3U) == 0) {
    const uint32_t n4 = len / 4;
    for (uint32_t c = lane; c < n4; c += kWave) reinterpret_cast<uint32_t*>(dst)[c] = src[c];
    done = n4 * 4;
  }
  // the rest byte by byte (a misaligned destination, or the tail)
  for (uint32_t b = done + lane; b < len; b += kWave) {
    dst[b] = static_cast<uint8_t>(src[b / 4] >> (8 * (b & 3U)));
  }
}

struct BigPart {
  uint32_t word;  // chunk word index of the header
  uint32_t len;
  uint64_t dst;   // output byte position (chunk-relative, after the re-inserted magic)
};

__global__ __launch_bounds__(kThreads) void k_rec_tile_fill(const uint32_t* __restrict__ w,
                                                            size_t n, size_t ntiles,
                                                            const uint64_t* __restrict__ prefix,
                                                            uint64_t* __restrict__ offset,
                                                            uint64_t rec_base,
                                                            uint8_t* __restrict__ data,
                                                            uint64_t byte_base,
                                                            MetaPartial* __restrict__ partials) {
  __shared__ BigPart s_big[kWaves][kBigCap];
  // the tile's words (+ the one after it): a part's successor check reads its
  // header from here instead of a dependent global load per part
  __shared__ uint4 s_tw[kWaves][kTileWords / 4 + 1];
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  const size_t tile = static_cast<size_t>(blockIdx.x) * kWaves + wave;
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
  const uint64_t pre = prefix[tile];
  uint64_t rec = pre >> 32;            // records before this 1 KiB sub-tile (chunk-relative)
  uint64_t pos = pre & 0xffffffffull;  // output bytes before it
  uint8_t* const out = data + byte_base;
  uint32_t err = 0;
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
      if (cf <= 1) {
        offset[rec_base + r] = byte_base + p;
        ++r;
      } else {
        // the reader re-inserts the escaped magic in front of a continuation
#pragma unroll
        for (int b = 0; b < 4; ++b) out[p + b] = static_cast<uint8_t>(kMagic >> (8 * b));
        p += 4;
      }
      const bool whole = i + 2 + (static_cast<size_t>(len) + 3) / 4 <= n;  // else: truncated
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
  // parts up to 1 KiB into 16-byte-aligned destinations (the common shape):
  // kBatch parts per round, every lane's loads of all of them issued before
  // any store, so a round waits for one memory latency instead of one per
  // part; anything else takes the generic wave copy
  constexpr uint32_t kBatch = 4;
  for (uint32_t e0 = 0; e0 < nbig; e0 += kBatch) {
    uint32_t v[kBatch][4];
    BigPart bp[kBatch];
    bool fast[kBatch];
#pragma unroll
    for (uint32_t q = 0; q < kBatch; ++q) {
      fast[q] = false;
      if (e0 + q < nbig) {
        bp[q] = big[e0 + q];
        fast[q] = bp[q].len <= 1024 && ((reinterpret_cast<uintptr_t>(out + bp[q].dst) & 15U) == 0);
        const uint32_t b0 = static_cast<uint32_t>(lane) * 16;
        if (fast[q] && b0 < bp[q].len) {
          const uint32_t* src = w + bp[q].word + 2 + lane * 4;
          const uint32_t nw = (bp[q].len - b0 + 3) / 4;  // words of this lane (<= 4)
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) v[q][k] = k < nw ? src[k] : 0u;
        }
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < kBatch; ++q) {
      if (e0 + q >= nbig) break;
      if (!fast[q]) {
        wave_copy(w + bp[q].word + 2, bp[q].len, out + bp[q].dst, lane);
        continue;
      }
      const uint32_t b0 = static_cast<uint32_t>(lane) * 16;
      if (b0 >= bp[q].len) continue;
      uint8_t* d = out + bp[q].dst + b0;
      const uint32_t m = bp[q].len - b0;
      if (m >= 16) {
        *reinterpret_cast<uint4*>(d) = make_uint4(v[q][0], v[q][1], v[q][2], v[q][3]);
      } else {
        for (uint32_t k = 0; k < m; ++k) d[k] = static_cast<uint8_t>(v[q][k >> 2] >> (8 * (k & 3U)));
      }
    }
  }
  err = wave_or(err);
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

void LaunchRecordIOTileFill(const uint32_t* words, size_t nwords, const uint64_t* tile_prefix,
                            uint64_t* offset, uint64_t rec_base, uint8_t* data, uint64_t byte_base,
                            MetaPartial* partials, hipStream_t stream) {
  const size_t tiles = RecordIOTiles(nwords);
  if (tiles == 0) return;
  hipLaunchKernelGGL(k_rec_tile_fill, dim3((tiles + kWaves - 1) / kWaves), dim3(kThreads), 0,
                     stream, words, nwords, tiles, tile_prefix, offset, rec_base, data, byte_base,
                     partials);
}

void LaunchRecordIOGather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                          const uint64_t* dst_off, size_t nrec, uint8_t* dst, hipStream_t stream) {
  if (nrec == 0) return;
  hipLaunchKernelGGL(k_rec_gather, dim3((nrec + kWaves - 1) / kWaves), dim3(kThreads), 0, stream,
                     src, src_off, len, dst_off, nrec, dst);
}

}  // namespace gpu
}  // namespace dmlc
