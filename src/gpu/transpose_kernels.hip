/*!
 * \file src/gpu/transpose_kernels.hip
 * \brief CSR -> CSC (the transpose / inverted index of a device CSR) on gfx950:
 *  a stable two-level counting sort of the entries by feature id, so every
 *  column lists its rows in ascending order (deterministic gradient sums).
 *
 *  Reference demonstrator of the operation: the row loop of
 *  include/dmlc/data.h:143-157 (Row::SDot) -- the transpose turns X^T d into
 *  the same gather over columns.
 *
 *  Column c = (bucket c >> kB, low key c & (L - 1)), L = 2^kB columns per
 *  bucket (kB = 10 .. 12, LowBits: the narrowest that keeps at most
 *  kMaxBuckets buckets, so feature ids < 2^22; wider feature spaces, up to
 *  2^28, take the three-level sort of RunSort3 below):
 *   T1 k_bucket_hist  one workgroup per block of BlockSubs() sub-tiles (in CSR
 *      order): LDS histogram of buckets -> G[bucket][block].
 *   T2 exclusive scan of G (bucket-major): where each (bucket, block) run
 *      lands in the bucket-ordered intermediate arrays.
 *   T3 k_bucket_scatter  same blocks, in sub-tiles of kSubElems entries: the
 *      sub-tile is counted per bucket, scanned in (bucket, position) order and
 *      ranked into LDS -- ranks among equal buckets of a 64-entry group come
 *      from ballots over the bucket bits (no atomics, so the sort is stable);
 *      row ids come from a per-chunk row table (k_chunk_rows) and a lane
 *      binary search over 64 row ends -- then leaves in bucket runs, so one
 *      store instruction touches a few lines / pages instead of 64 (the
 *      direct scatter was bound by partial lines and TLB misses: 16 ms at
 *      400 M entries).  Writes the low key (u16) and the (row, value) pair
 *      (8 bytes; the row alone without values).  The next sub-tile's
 *      entries load while this one is sorted.
 *   T4a k_lowkey_hist  one workgroup per (bucket, segment) of the bucket: LDS
 *      histogram of the L low keys -> H[bucket][segment][L].
 *   T4b k_lowkey_scan  one workgroup per bucket: column totals over segments,
 *      exclusive scan over the bucket's columns -> col_ptr, and per-segment
 *      starting cursors (in place in H).
 *   T4c k_lowkey_scatter  one wave per (bucket, segment): cursors in LDS,
 *      the segment's entries in order (8 groups of 64 loaded a batch ahead),
 *      ranks by ballots over the low-key bits -> row / value at their final
 *      CSC position.
 *  Traffic for 400 M entries: keys read 3x + (row, value) written and read
 *  once through the intermediate arrays, ~17 GB, no global atomics.
 */
#include <dmlc/gpu/hip_utils.h>
#include <dmlc/logging.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {

namespace {
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / dev::kWave;
constexpr int kMinLowBits = 10;  // columns per bucket: 2^kB, kB = 10 .. 12 (LowBits)
constexpr int kMaxLowBits = 12;
constexpr int kDefaultLowBits = kMinLowBits;
constexpr uint32_t kMaxBuckets = 1024;
constexpr uint32_t kSubElems = 2048;        // T3 sub-tile, sorted in LDS (4 workgroups / CU)
constexpr int kBlockSubs = 15;  // sub-tiles per T1 / T3 block (a workgroup), BlockSubs()
constexpr uint32_t kChunk = kSubElems / kWaves;  // entries per wave per sub-tile
constexpr int kPerLane = kChunk / dev::kWave;
constexpr int kSegments = 16;              // T4 segments per bucket

/*! \brief a feature id as a column below num_features (out-of-range ids are
 *  clamped for memory safety and reported through the error word by T1) */
template <typename IndexType>
__device__ __forceinline__ uint32_t column(IndexType c, uint64_t num_features) {
  return static_cast<uint32_t>(static_cast<uint64_t>(c) < num_features ? static_cast<uint64_t>(c)
                                                                       : num_features - 1);
}

/*! \brief lanes of this wave whose `key` (low `bits` bits) equals mine, among `valid` */
__device__ __forceinline__ uint64_t match_lanes(uint32_t key, int bits, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll 1
  for (int i = 0; i < bits; ++i) {
    const bool b = (key >> i) & 1u;
    const uint64_t v = __ballot(b);
    m &= b ? v : ~v;
  }
  return m;
}

__device__ __forceinline__ uint64_t lanes_below() {
  const int lane = dev::lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

/*! \brief first row whose entries end after entry e (offsets relative to base) */
__device__ __forceinline__ uint32_t row_of(const uint64_t* __restrict__ offset, size_t nrows,
                                           uint64_t base, uint64_t e) {
  size_t lo = 0, hi = nrows;  // offset[lo] - base <= e < offset[hi] - base
  while (hi - lo > 1) {
    const size_t mid = (lo + hi) >> 1;
    if (offset[mid] - base <= e) {
      lo = mid;
    } else {
      hi = mid;
    }
  }
  return static_cast<uint32_t>(lo);
}

template <typename IndexType, int kB>
__global__ __launch_bounds__(kThreads) void k_bucket_hist(const IndexType* __restrict__ index,
                                                          uint64_t nnz, uint64_t num_features,
                                                          uint32_t nbuckets,
                                                          uint64_t* __restrict__ G,
                                                          size_t nblocks, uint64_t block_elems,
                                                          uint32_t* __restrict__ error) {
  __shared__ uint32_t hist[kMaxBuckets];
  for (uint32_t b = threadIdx.x; b < nbuckets; b += kThreads) hist[b] = 0;
  __syncthreads();
  const uint64_t e0 = static_cast<uint64_t>(blockIdx.x) * block_elems;
  const uint64_t e1 = e0 + block_elems < nnz ? e0 + block_elems : nnz;
  bool bad = false;
  auto add = [&](IndexType c) {
    bad |= static_cast<uint64_t>(c) >= num_features;
    atomicAdd(&hist[column(c, num_features) >> kB], 1u);
  };
  uint64_t e = e0 + threadIdx.x;
  if (sizeof(IndexType) == 4 && (reinterpret_cast<uintptr_t>(index + e0) & 15u) == 0) {
    // four ids per 16-byte load (block_elems is a multiple of 4): a quarter
    // of the load instructions of the one-id-per-lane walk
    const uint64_t n4 = (e1 - e0) / 4;
    const uint4* q = reinterpret_cast<const uint4*>(index + e0);
    for (uint64_t i = threadIdx.x; i < n4; i += kThreads) {
      const uint4 v = q[i];
      add(static_cast<IndexType>(v.x));
      add(static_cast<IndexType>(v.y));
      add(static_cast<IndexType>(v.z));
      add(static_cast<IndexType>(v.w));
    }
    e = e0 + n4 * 4 + threadIdx.x;
  }
  for (; e < e1; e += kThreads) add(index[e]);
  if (__any(bad) && dev::lane_id() == 0) atomicOr(error, 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbuckets; b += kThreads) {
    G[static_cast<size_t>(b) * nblocks + blockIdx.x] = hist[b];
  }
}

/*! \brief row of the first entry of every kChunk-entry chunk (T3 waves start
 *  at any chunk without a dependent binary search of their own) */
__global__ void k_chunk_rows(const uint64_t* __restrict__ offset, size_t nrows, uint64_t base,
                             uint64_t nnz, uint32_t* __restrict__ chunk_row) {
  const uint64_t c = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c * kChunk < nnz) chunk_row[c] = row_of(offset, nrows, base, c * kChunk);
}

template <typename IndexType, int kB, typename KeyT = uint16_t>
__global__ __launch_bounds__(kThreads) void k_bucket_scatter(
    const uint64_t* __restrict__ offset, size_t nrows, uint64_t base,
    const IndexType* __restrict__ index, const float* __restrict__ value, uint64_t nnz,
    uint64_t num_features, uint32_t nbuckets, int bucket_bits, const uint64_t* __restrict__ G,
    size_t nblocks, uint64_t block_elems, const uint32_t* __restrict__ chunk_row,
    KeyT* __restrict__ t_key, uint32_t* __restrict__ t_row, uint2* __restrict__ t_rv) {
  // the sub-tile, sorted by (bucket, position) in LDS before it leaves
  __shared__ uint32_t s_col[kSubElems];
  __shared__ uint32_t s_row[kSubElems];
  __shared__ float s_val[kSubElems];
  // per-wave counts, then LDS cursors (<= kSubElems: 16 bits); bucket starts
  // inside the sub-tile; the block's next output position per bucket (nnz <
  // 2^32: 32 bits)
  __shared__ uint16_t cnt[kWaves][kMaxBuckets];
  __shared__ uint16_t lstart[kMaxBuckets + 2];
  __shared__ uint32_t gcur[kMaxBuckets];
  __shared__ uint32_t swave[kWaves];
  __shared__ uint32_t s_ends[kWaves][dev::kWave];  // row ends per group position
  const int w = threadIdx.x / dev::kWave;
  const int lane = dev::lane_id();
  const uint64_t below = lanes_below();
  for (uint32_t b = threadIdx.x; b < nbuckets; b += kThreads) {
    for (int q = 0; q < kWaves; ++q) cnt[q][b] = 0;
    gcur[b] = static_cast<uint32_t>(G[static_cast<size_t>(b) * nblocks + blockIdx.x]);
  }
  __syncthreads();
  const uint64_t blk0 = static_cast<uint64_t>(blockIdx.x) * block_elems;
  const uint64_t blk1 = blk0 + block_elems < nnz ? blk0 + block_elems : nnz;
  // the next sub-tile's entries (and its chunk's first row) are loaded while
  // this one is sorted: a wave waits for memory once per block, not once per
  // sub-tile (round 4: 71 % of the cycles waiting)
  IndexType ci[kPerLane];
  float vi[kPerLane];
  uint32_t nwb = 0;
  auto fetch = [&](uint64_t s0n) {
    const uint64_t c0n = s0n + static_cast<uint64_t>(w) * kChunk;
    const uint64_t c1n = c0n + kChunk < blk1 ? c0n + kChunk : blk1;
#pragma unroll
    for (int i = 0; i < kPerLane; ++i) {
      const uint64_t e = c0n + static_cast<uint64_t>(i) * dev::kWave + lane;
      ci[i] = e < c1n ? index[e] : IndexType(0);
      vi[i] = (e < c1n && value != nullptr) ? value[e] : 0.0f;
    }
    nwb = c0n < c1n ? chunk_row[c0n / kChunk] : 0u;
  };
  fetch(blk0);
  for (uint64_t s0 = blk0; s0 < blk1; s0 += kSubElems) {
    const uint32_t nsub = static_cast<uint32_t>(blk1 - s0 < kSubElems ? blk1 - s0 : kSubElems);
    // ---- this wave's chunk: kPerLane coalesced groups (loaded a sub-tile ago)
    const uint64_t c0 = s0 + static_cast<uint64_t>(w) * kChunk;
    const uint64_t c1 = c0 + kChunk < blk1 ? c0 + kChunk : blk1;
    uint32_t col[kPerLane];
    float v[kPerLane];
#pragma unroll
    for (int i = 0; i < kPerLane; ++i) {
      const uint64_t e = c0 + static_cast<uint64_t>(i) * dev::kWave + lane;
      col[i] = e < c1 ? column(ci[i], num_features) : 0u;
      v[i] = vi[i];
    }
    // the row window of the rank phase below, in flight during count + scan
    uint32_t wbase = nwb;
    auto window = [&](uint32_t wb) {
      const size_t ri = static_cast<size_t>(wb) + 1 + lane;
      return ri <= nrows ? offset[ri] - base : ~0ull;
    };
    uint64_t wend = window(wbase);
    if (s0 + kSubElems < blk1) fetch(s0 + kSubElems);
    // ---- count per bucket: lanes of a group with equal buckets from ballots
    // over the bucket bits (no atomics); each group's rank among its equal
    // buckets and their number stay in registers for the rank phase
    uint32_t rk[kPerLane];  // rank | n << 8 (n <= 64)
#pragma unroll
    for (int i = 0; i < kPerLane; ++i) {
      const bool valid = c0 + static_cast<uint64_t>(i) * dev::kWave + lane < c1;
      const uint32_t bk = col[i] >> kB;
      const uint64_t m = match_lanes(bk, bucket_bits, valid);
      const uint32_t rank = static_cast<uint32_t>(__popcll(m & below));
      const uint32_t n = static_cast<uint32_t>(__popcll(m));
      rk[i] = rank | (n << 8);
      // the group's last lane of each bucket adds the group's count (one
      // lane per bucket: no conflicts; groups in program order)
      if (valid && rank + 1 == n) cnt[w][bk] = static_cast<uint16_t>(cnt[w][bk] + n);
    }
    __syncthreads();
    // ---- exclusive scan in (bucket, wave) order: thread t owns 4 buckets
    {
      constexpr uint32_t kOwn = kMaxBuckets / kThreads;
      const uint32_t b0 = threadIdx.x * kOwn;
      uint32_t sum = 0;
#pragma unroll
      for (uint32_t i = 0; i < kOwn; ++i) {
        if (b0 + i < nbuckets) {
          for (int q = 0; q < kWaves; ++q) sum += cnt[q][b0 + i];
        }
      }
      uint32_t wtot;
      const uint32_t wx = dev::wave_excl_scan(sum, &wtot);
      if (lane == 0) swave[w] = wtot;
      __syncthreads();
      uint32_t x = wx;
      for (int q = 0; q < w; ++q) x += swave[q];
#pragma unroll
      for (uint32_t i = 0; i < kOwn; ++i) {
        const uint32_t b = b0 + i;
        if (b < nbuckets) {
          lstart[b] = static_cast<uint16_t>(x);
          for (int q = 0; q < kWaves; ++q) {
            const uint32_t c = cnt[q][b];
            cnt[q][b] = static_cast<uint16_t>(x);
            x += c;
          }
        }
      }
      if (threadIdx.x == 0) lstart[nbuckets] = static_cast<uint16_t>(nsub);
    }
    __syncthreads();
    // ---- rank every group into the LDS sub-tile.  Rows: lane i holds the end
    // of row wbase + i (one coalesced load of 64 row ends, from the chunk's
    // first row); an entry's row is wbase + the number of those ends at or
    // before it: each end is counted at its position in the group (an LDS
    // add; empty rows stack on one position) and a DPP scan over the
    // positions gives every entry its count -- two LDS trips per group
    // instead of a chain of six bpermutes (a binary search over the lanes).
    // The window only moves forward (rows are monotone in entry order),
    // reloaded when a group runs past its 64 rows
#pragma unroll
    for (int i = 0; i < kPerLane; ++i) {
      const uint64_t g = c0 + static_cast<uint64_t>(i) * dev::kWave;
      const bool valid = g + lane < c1;
      if (!__any(valid)) continue;  // the tail of the last chunk
      const uint32_t pos = lane;
      uint32_t row = wbase;
      bool found = !valid;
      for (;;) {
        // (ends before the group start -- rows of earlier groups still in the
        // window -- count as at or before every entry)
        const uint32_t rel = wend <= g ? 0u
                             : wend - g >= 0xFFFFFFFFull ? 0xFFFFFFFFu
                                                         : static_cast<uint32_t>(wend - g);
        uint32_t* const ends = s_ends[w];
        ends[lane] = 0u;
        dev::wave_sync();
        if (rel < static_cast<uint32_t>(dev::kWave)) atomicAdd(&ends[rel], 1u);
        dev::wave_sync();
        // ends at or before position pos (64: the whole window ends before it)
        const uint32_t n = dev::wave_incl_scan_u32(ends[pos]);
        dev::wave_sync();  // every lane has read its count before the next reset
        if (!found && n < static_cast<uint32_t>(dev::kWave)) {
          row = wbase + n;
          found = true;
        }
        if (__all(found)) break;
        wbase += dev::kWave;  // more than 64 row ends before some entry (empty rows)
        wend = window(wbase);
      }
      const uint32_t bk = col[i] >> kB;
      const uint32_t rank = rk[i] & 0xFFu, n = rk[i] >> 8;
      const uint32_t before = valid ? cnt[w][bk] : 0u;
      dev::wave_sync();  // every lane has read its cursor
      if (valid) {
        const uint32_t slot = before + rank;
        s_col[slot] = col[i];
        s_row[slot] = row;
        s_val[slot] = v[i];
        if (rank + 1 == n) cnt[w][bk] = static_cast<uint16_t>(before + n);  // the group's last lane
      }
      dev::wave_sync();
    }
    __syncthreads();
    // ---- the sorted sub-tile leaves in runs: consecutive threads, consecutive
    // positions of one bucket's run
    for (uint32_t j = threadIdx.x; j < nsub; j += kThreads) {
      const uint32_t c = s_col[j];
      const uint32_t b = c >> kB;
      const uint64_t p = static_cast<uint64_t>(gcur[b]) + (j - lstart[b]);
      t_key[p] = static_cast<KeyT>(c & ((1u << kB) - 1u));
      // (row, value) as one 8-byte pair: two store streams per sub-tile
      // instead of three, one load per entry in T4c
      if (value != nullptr) {
        t_rv[p] = make_uint2(s_row[j], __float_as_uint(s_val[j]));
      } else {
        t_row[p] = s_row[j];
      }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbuckets; b += kThreads) {
      gcur[b] += static_cast<uint32_t>(lstart[b + 1] - lstart[b]);
      for (int q = 0; q < kWaves; ++q) cnt[q][b] = 0;
    }
    __syncthreads();
  }
}

/*! \brief [begin, end) of segment s of bucket b (T4), from the bucket starts */
__device__ __forceinline__ void segment(const uint64_t* __restrict__ bstart, uint32_t b, int s,
                                        uint64_t* begin, uint64_t* end) {
  const uint64_t b0 = bstart[b], b1 = bstart[b + 1];
  const uint64_t n = b1 - b0;
  *begin = b0 + n * static_cast<uint64_t>(s) / kSegments;
  *end = b0 + n * static_cast<uint64_t>(s + 1) / kSegments;
}

template <int kB>
__global__ __launch_bounds__(kThreads) void k_lowkey_hist(const uint16_t* __restrict__ t_key,
                                                          const uint64_t* __restrict__ bstart,
                                                          uint32_t* __restrict__ H) {
  constexpr uint32_t kLow = 1u << kB;
  // counts need no order: the whole workgroup shares one histogram
  __shared__ uint32_t hist[kLow];
  const uint32_t b = blockIdx.x / kSegments;
  const int s = static_cast<int>(blockIdx.x % kSegments);
  for (uint32_t c = threadIdx.x; c < kLow; c += kThreads) hist[c] = 0;
  __syncthreads();
  uint64_t e0, e1;
  segment(bstart, b, s, &e0, &e1);
  // eight keys per 16-byte load over the aligned middle of the segment, the
  // unaligned head and tail one key at a time
  const uint64_t a0 = (e0 + 7) & ~7ull, a1 = e1 & ~7ull;
  if (a0 >= a1) {
    for (uint64_t e = e0 + threadIdx.x; e < e1; e += kThreads) atomicAdd(&hist[t_key[e]], 1u);
  } else {
    for (uint64_t e = e0 + threadIdx.x; e < a0; e += kThreads) atomicAdd(&hist[t_key[e]], 1u);
    for (uint64_t e = a1 + threadIdx.x; e < e1; e += kThreads) atomicAdd(&hist[t_key[e]], 1u);
    const uint4* k8 = reinterpret_cast<const uint4*>(t_key + a0);
    const uint64_t n8 = (a1 - a0) / 8;
#pragma unroll 2
    for (uint64_t i = threadIdx.x; i < n8; i += kThreads) {
      const uint4 q = k8[i];
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        atomicAdd(&hist[w[j] & 0xFFFFu], 1u);
        atomicAdd(&hist[w[j] >> 16], 1u);
      }
    }
  }
  __syncthreads();
  uint32_t* out = H + static_cast<size_t>(blockIdx.x) * kLow;
  for (uint32_t c = threadIdx.x; c < kLow; c += kThreads) out[c] = hist[c];
}

/*! \brief per bucket: column totals over segments -> col_ptr; per-segment
 *  cursors in H.  Thread t walks columns t, t + 256, ... so every H access of
 *  a segment row is one coalesced 1 KiB line run (round 4 walked 16
 *  consecutive columns per thread: 64-byte-strided lanes, 354 us); the scan
 *  over the bucket's columns runs on the LDS copy of the totals. */
template <int kB>
__global__ __launch_bounds__(kThreads) void k_lowkey_scan(uint32_t* __restrict__ H,
                                                          const uint64_t* __restrict__ bstart,
                                                          uint64_t num_features,
                                                          uint64_t* __restrict__ col_ptr) {
  constexpr uint32_t kLow = 1u << kB;
  __shared__ uint32_t s_tot[kLow];  // column totals, then exclusive column starts (u32)
  __shared__ uint64_t swave[kWaves];
  constexpr uint32_t kPer = kLow / kThreads;  // columns per thread
  const uint32_t b = blockIdx.x;
  uint32_t* Hb = H + static_cast<size_t>(b) * kSegments * kLow;
  // 1. per column: the segments' counts -> offsets inside the column (in H)
  //    and the column total (coalesced: consecutive threads, consecutive columns)
#pragma unroll 4
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint32_t c = i * kThreads + threadIdx.x;
    uint32_t h[kSegments];
#pragma unroll
    for (int s = 0; s < kSegments; ++s) h[s] = Hb[static_cast<size_t>(s) * kLow + c];
    uint32_t acc = 0;
#pragma unroll
    for (int s = 0; s < kSegments; ++s) {
      Hb[static_cast<size_t>(s) * kLow + c] = acc;
      acc += h[s];
    }
    s_tot[c] = acc;
  }
  __syncthreads();
  // 2. exclusive scan of the 4096 totals: thread t owns columns 16 t .. 16 t + 15
  const uint32_t c0 = threadIdx.x * kPer;
  uint32_t tot[kPer];
  uint64_t sum = 0;
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    tot[i] = s_tot[c0 + i];
    sum += tot[i];
  }
  uint64_t wtot;
  const uint64_t wx = dev::wave_excl_scan(sum, &wtot);
  const int w = threadIdx.x / dev::kWave;
  if (dev::lane_id() == 0) swave[w] = wtot;
  __syncthreads();
  uint64_t before = wx;
  for (int q = 0; q < w; ++q) before += swave[q];
  const uint64_t base = bstart[b];
  uint64_t x = before;  // relative to the bucket base (< 2^32: nnz < 2^32)
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint64_t c = static_cast<uint64_t>(b) * kLow + c0 + i;
    if (c < num_features) col_ptr[c] = base + x;
    s_tot[c0 + i] = static_cast<uint32_t>(x);
    x += tot[i];
  }
  __syncthreads();
  // 3. cursors become absolute CSC positions (u32 offsets from the bucket base)
#pragma unroll 4
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint32_t c = i * kThreads + threadIdx.x;
    const uint32_t start = s_tot[c];
#pragma unroll
    for (int s = 0; s < kSegments; ++s) Hb[static_cast<size_t>(s) * kLow + c] += start;
  }
}


// kPair: the output is interleaved (row, value) pairs -- one 8-byte store per
// entry instead of a 4-byte store into each of two arrays (T4c is bound by
// the output lines its scattered stores touch)
// kDepth: 64-entry groups per batch (loads a batch ahead; 8: 74 VGPRs -- 4 took 89)
template <bool kPair, int kB, int kDepth>
__global__ __launch_bounds__(dev::kWave) void k_lowkey_scatter(
    const uint16_t* __restrict__ t_key, const uint32_t* __restrict__ t_row,
    const uint2* __restrict__ t_rv, const uint64_t* __restrict__ bstart,
    const uint32_t* __restrict__ H, uint32_t* __restrict__ row_out, float* __restrict__ val_out) {
  constexpr uint32_t kLow = 1u << kB;
  __shared__ uint32_t cur[kLow];
  const uint32_t b = blockIdx.x / kSegments;
  const int s = static_cast<int>(blockIdx.x % kSegments);
  const int lane = dev::lane_id();
  const uint32_t* Hs = H + static_cast<size_t>(blockIdx.x) * kLow;
  for (uint32_t c = lane; c < kLow; c += dev::kWave) cur[c] = Hs[c];
  dev::wave_sync();
  uint64_t e0, e1;
  segment(bstart, b, s, &e0, &e1);
  const uint64_t base = bstart[b];
  const uint64_t below = lanes_below();
  // The segment walks in batches of kDepth groups of 64 consecutive
  // entries (group j of a batch: entries + 64 j + lane, so groups stay in
  // entry order).  A batch's loads are issued a whole batch ahead, into the
  // other register set: a wave keeps 8 x 64 entries in flight instead of one
  // group (the round-4 kernel waited out the memory latency every 64
  // entries, at 10 waves per CU -- 72 % of its cycles waiting)
  struct Batch {
    uint32_t k[kDepth], r[kDepth];
    float v[kDepth];
  };
  auto load = [&](uint64_t at, Batch* x) {
#pragma unroll
    for (int j = 0; j < kDepth; ++j) {
      const uint64_t e = at + static_cast<uint64_t>(j) * dev::kWave + lane;
      const bool ok = e < e1;
      x->k[j] = ok ? t_key[e] : 0u;
      if (val_out != nullptr) {
        const uint2 rv = ok ? t_rv[e] : make_uint2(0u, 0u);
        x->r[j] = rv.x;
        x->v[j] = __uint_as_float(rv.y);
      } else {
        x->r[j] = ok ? t_row[e] : 0u;
        x->v[j] = 0.0f;
      }
    }
  };
  auto process = [&](uint64_t at, const Batch& x) {
    // the ranks need no LDS: every group's ballots first, then the cursor
    // updates group by group (the only dependent chain)
    uint32_t rk[kDepth];
#pragma unroll
    for (int j = 0; j < kDepth; ++j) {
      const bool valid = at + static_cast<uint64_t>(j) * dev::kWave + lane < e1;
      const uint64_t m = match_lanes(x.k[j], kB, valid);
      rk[j] = static_cast<uint32_t>(__popcll(m & below)) |
              (static_cast<uint32_t>(__popcll(m)) << 8);
      // one group's ballots at a time: interleaved, the kB ballots of all
      // kDepth groups (64-bit SGPR pairs) overflowed the SGPRs into hundreds
      // of v_writelane / v_readlane spills
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < kDepth; ++j) {
      const uint64_t g = at + static_cast<uint64_t>(j) * dev::kWave;
      if (g >= e1) break;  // wave-uniform
      const bool valid = g + lane < e1;
      const uint32_t k = x.k[j];
      const uint32_t rank = rk[j] & 0xFFu, n = rk[j] >> 8;
      const uint32_t before = valid ? cur[k] : 0u;
      dev::wave_sync();
      if (valid) {
        const uint64_t pos = base + before + rank;
        if constexpr (kPair) {
          reinterpret_cast<uint2*>(row_out)[pos] = make_uint2(x.r[j], __float_as_uint(x.v[j]));
        } else {
          row_out[pos] = x.r[j];
          if (val_out != nullptr) val_out[pos] = x.v[j];
        }
        if (rank + 1 == n) cur[k] = before + n;
      }
      dev::wave_sync();
    }
  };
  constexpr uint64_t kBatch = static_cast<uint64_t>(kDepth) * dev::kWave;
  Batch A, B;
  load(e0, &A);
  for (uint64_t at = e0; at < e1; at += 2 * kBatch) {
    load(at + kBatch, &B);
    process(at, A);
    if (at + kBatch >= e1) break;
    load(at + 2 * kBatch, &A);
    process(at + kBatch, B);
  }
}

// ---------------------------------------------------------------------------
// Three levels (feature spaces above 2^22, up to 2^28).  T1-T3 split the
// entries into <= 1024 buckets of 2^S columns (S = 16 .. 18, the low S bits
// kept as a u32 key); a bucket's 2^S columns are too many for one LDS cursor
// table, so two more stable counting-sort passes of T4's shape follow:
//   L2 per (bucket, segment): digit = key >> 8 (2^(S-8) values) -> the
//      entries in (bucket, mid) "super-bucket" order, the low 8 bits kept as
//      a u8 key; the super-bucket starts come from L2's scan;
//   L3 per super-bucket (~1500 entries each at 2^26 x 400 M), one wave:
//      digit = the low 8 bits -> the final CSC position, the column pointer
//      (k_local_sort256: counts, scan and placement without a global
//      histogram).
// Every pass scatters into at most 1024 (L2) / 256 (L3) open runs per wave
// (T4c's 1024 - 4096 in the two-level sort).

/*! \brief [begin, end) of segment s of kSeg segments of bucket b */
template <int kSeg>
__device__ __forceinline__ void seg_range(const uint64_t* __restrict__ bstart, uint32_t b, int s,
                                          uint64_t* begin, uint64_t* end) {
  const uint64_t b0 = bstart[b], b1 = bstart[b + 1];
  const uint64_t n = b1 - b0;
  *begin = b0 + n * static_cast<uint64_t>(s) / kSeg;
  *end = b0 + n * static_cast<uint64_t>(s + 1) / kSeg;
}

/*! \brief L2 / L3 histogram: per (bucket, segment), the digit (key >> kShift)
 *  & (2^kB - 1) of its entries -> H[bucket][segment][2^kB] */
template <typename KeyIn, int kShift, int kB, int kSeg>
__global__ __launch_bounds__(kThreads) void k_digit_hist(const KeyIn* __restrict__ key,
                                                         const uint64_t* __restrict__ bstart,
                                                         uint32_t* __restrict__ H) {
  constexpr uint32_t kLow = 1u << kB;
  __shared__ uint32_t hist[kLow];
  const uint32_t b = blockIdx.x / kSeg;
  const int s = static_cast<int>(blockIdx.x % kSeg);
  for (uint32_t c = threadIdx.x; c < kLow; c += kThreads) hist[c] = 0;
  __syncthreads();
  uint64_t e0, e1;
  seg_range<kSeg>(bstart, b, s, &e0, &e1);
  auto add = [&](uint32_t k) { atomicAdd(&hist[(k >> kShift) & (kLow - 1u)], 1u); };
  if constexpr (sizeof(KeyIn) == 4) {
    // four keys per 16-byte load over the aligned middle of the segment
    const uint64_t a0 = (e0 + 3) & ~3ull, a1 = e1 & ~3ull;
    if (a0 < a1) {
      for (uint64_t e = e0 + threadIdx.x; e < a0; e += kThreads) add(key[e]);
      for (uint64_t e = a1 + threadIdx.x; e < e1; e += kThreads) add(key[e]);
      const uint4* k4 = reinterpret_cast<const uint4*>(key + a0);
      const uint64_t n4 = (a1 - a0) / 4;
      for (uint64_t i = threadIdx.x; i < n4; i += kThreads) {
        const uint4 q = k4[i];
        add(q.x);
        add(q.y);
        add(q.z);
        add(q.w);
      }
      e0 = e1;  // done
    }
  }
  for (uint64_t e = e0 + threadIdx.x; e < e1; e += kThreads) add(static_cast<uint32_t>(key[e]));
  __syncthreads();
  uint32_t* out = H + static_cast<size_t>(blockIdx.x) * kLow;
  for (uint32_t c = threadIdx.x; c < kLow; c += kThreads) out[c] = hist[c];
}

/*! \brief L2 / L3 scan, per bucket: digit totals over the segments -> the
 *  exclusive starts `starts[b * 2^kB + digit]` (absolute positions; entries
 *  past nstarts are not written) and absolute per-segment cursors in H */
template <int kB, int kSeg>
__global__ __launch_bounds__(kThreads) void k_digit_scan(uint32_t* __restrict__ H,
                                                         const uint64_t* __restrict__ bstart,
                                                         uint64_t nstarts,
                                                         uint64_t* __restrict__ starts) {
  constexpr uint32_t kLow = 1u << kB;
  constexpr uint32_t kPer = (kLow + kThreads - 1) / kThreads;
  __shared__ uint32_t s_tot[kLow];
  __shared__ uint64_t swave[kWaves];
  const uint32_t b = blockIdx.x;
  uint32_t* Hb = H + static_cast<size_t>(b) * kSeg * kLow;
  for (uint32_t c = threadIdx.x; c < kLow; c += kThreads) {
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < kSeg; ++q) {
      const uint32_t h = Hb[static_cast<size_t>(q) * kLow + c];
      Hb[static_cast<size_t>(q) * kLow + c] = acc;
      acc += h;
    }
    s_tot[c] = acc;
  }
  __syncthreads();
  const uint32_t c0 = threadIdx.x * kPer;
  uint32_t tot[kPer];
  uint64_t sum = 0;
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    tot[i] = c0 + i < kLow ? s_tot[c0 + i] : 0u;
    sum += tot[i];
  }
  uint64_t wtot;
  const uint64_t wx = dev::wave_excl_scan(sum, &wtot);
  const int w = threadIdx.x / dev::kWave;
  if (dev::lane_id() == 0) swave[w] = wtot;
  __syncthreads();
  uint64_t x = wx;
  for (int q = 0; q < w; ++q) x += swave[q];
  const uint64_t base = bstart[b];
  __syncthreads();  // every thread has read s_tot
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint32_t c = c0 + i;
    if (c < kLow) {
      const uint64_t g = static_cast<uint64_t>(b) * kLow + c;
      if (g < nstarts) starts[g] = base + x;
      s_tot[c] = static_cast<uint32_t>(x);
      x += tot[i];
    }
  }
  __syncthreads();
  for (uint32_t c = threadIdx.x; c < kLow; c += kThreads) {
    const uint32_t start = s_tot[c];
#pragma unroll
    for (int q = 0; q < kSeg; ++q) Hb[static_cast<size_t>(q) * kLow + c] += start;
  }
}

/*!
 * \brief L2 / L3 stable scatter: one wave per (bucket, segment), digit ranks
 *  by ballots as in T4c; the (row, value) pair (or the row) moves to
 *  bucket base + cursor, and with key_out the key's low 8 bits go along (L2).
 *  Output pairs when kPair (row / value arrays of the final CSC, or L2's
 *  intermediate pair array); rows alone otherwise.
 */
template <typename KeyIn, int kShift, int kB, int kSeg, bool kPair>
__global__ __launch_bounds__(dev::kWave) void k_digit_scatter(
    const KeyIn* __restrict__ key, const uint32_t* __restrict__ t_row,
    const uint2* __restrict__ t_rv, const uint64_t* __restrict__ bstart,
    const uint32_t* __restrict__ H, uint8_t* __restrict__ key_out, uint32_t* __restrict__ row_out,
    float* __restrict__ val_out, bool with_values) {
  constexpr uint32_t kLow = 1u << kB;
  constexpr int kDepth = 8;
  __shared__ uint32_t cur[kLow];
  const uint32_t b = blockIdx.x / kSeg;
  const int s = static_cast<int>(blockIdx.x % kSeg);
  const int lane = dev::lane_id();
  const uint32_t* Hs = H + static_cast<size_t>(blockIdx.x) * kLow;
  for (uint32_t c = lane; c < kLow; c += dev::kWave) cur[c] = Hs[c];
  dev::wave_sync();
  uint64_t e0, e1;
  seg_range<kSeg>(bstart, b, s, &e0, &e1);
  const uint64_t base = bstart[b];
  const uint64_t below = lanes_below();
  struct Batch {
    uint32_t k[kDepth], r[kDepth], v[kDepth];
  };
  auto load = [&](uint64_t at, Batch* x) {
#pragma unroll
    for (int j = 0; j < kDepth; ++j) {
      const uint64_t e = at + static_cast<uint64_t>(j) * dev::kWave + lane;
      const bool ok = e < e1;
      x->k[j] = ok ? static_cast<uint32_t>(key[e]) : 0u;
      if (with_values) {
        const uint2 rv = ok ? t_rv[e] : make_uint2(0u, 0u);
        x->r[j] = rv.x;
        x->v[j] = rv.y;
      } else {
        x->r[j] = ok ? t_row[e] : 0u;
        x->v[j] = 0u;
      }
    }
  };
  auto process = [&](uint64_t at, const Batch& x) {
    uint32_t rk[kDepth];
#pragma unroll
    for (int j = 0; j < kDepth; ++j) {
      const bool valid = at + static_cast<uint64_t>(j) * dev::kWave + lane < e1;
      const uint64_t m = match_lanes((x.k[j] >> kShift) & (kLow - 1u), kB, valid);
      rk[j] = static_cast<uint32_t>(__popcll(m & below)) |
              (static_cast<uint32_t>(__popcll(m)) << 8);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < kDepth; ++j) {
      const uint64_t g = at + static_cast<uint64_t>(j) * dev::kWave;
      if (g >= e1) break;  // wave-uniform
      const bool valid = g + lane < e1;
      const uint32_t d = (x.k[j] >> kShift) & (kLow - 1u);
      const uint32_t rank = rk[j] & 0xFFu, n = rk[j] >> 8;
      const uint32_t before = valid ? cur[d] : 0u;
      dev::wave_sync();
      if (valid) {
        const uint64_t pos = base + before + rank;  // (cursors: from the bucket base)
        if (key_out != nullptr) key_out[pos] = static_cast<uint8_t>(x.k[j] & 0xFFu);
        if constexpr (kPair) {
          reinterpret_cast<uint2*>(row_out)[pos] = make_uint2(x.r[j], x.v[j]);
        } else {
          row_out[pos] = x.r[j];
          if (val_out != nullptr) val_out[pos] = __uint_as_float(x.v[j]);
        }
        if (rank + 1 == n) cur[d] = before + n;
      }
      dev::wave_sync();
    }
  };
  constexpr uint64_t kBatch = static_cast<uint64_t>(kDepth) * dev::kWave;
  Batch A, B;
  load(e0, &A);
  for (uint64_t at = e0; at < e1; at += 2 * kBatch) {
    load(at + kBatch, &B);
    process(at, A);
    if (at + kBatch >= e1) break;
    load(at + 2 * kBatch, &A);
    process(at + kBatch, B);
  }
}

/*!
 * \brief L3 in one pass over a super-bucket: one wave per super-bucket (4
 *  per workgroup) counts its low bytes in LDS, scans the 256 counts (the
 *  column pointer of its 256 columns), then places its entries in order with
 *  ballot ranks -- no histogram round trip through global memory, no
 *  per-super-bucket workgroup of its own for the count and the scan.
 */
__global__ __launch_bounds__(kThreads) void k_local_sort256(
    const uint8_t* __restrict__ key, const uint2* __restrict__ rv,
    const uint64_t* __restrict__ sstart, uint64_t nsuper, uint64_t num_features,
    uint64_t* __restrict__ col_ptr, uint32_t* __restrict__ row_out, float* __restrict__ val_out,
    bool paired) {
  __shared__ uint32_t s_cnt[kWaves][256];
  const int w = threadIdx.x / dev::kWave;
  const int lane = dev::lane_id();
  const uint64_t sb = static_cast<uint64_t>(blockIdx.x) * kWaves + w;
  if (sb >= nsuper) return;  // whole waves leave; nothing below synchronises waves
  uint32_t* cnt = s_cnt[w];
  const uint64_t b0 = sstart[sb], b1 = sstart[sb + 1];
#pragma unroll
  for (int i = 0; i < 4; ++i) cnt[lane * 4 + i] = 0u;
  dev::wave_sync();
  // pass 1: counts (4 keys per 4-byte load over the aligned middle)
  const uint64_t a0 = (b0 + 3) & ~3ull, a1 = b1 & ~3ull;
  if (a0 < a1) {
    for (uint64_t e = b0 + lane; e < a0; e += dev::kWave) atomicAdd(&cnt[key[e]], 1u);
    for (uint64_t e = a1 + lane; e < b1; e += dev::kWave) atomicAdd(&cnt[key[e]], 1u);
    const uint32_t* k4 = reinterpret_cast<const uint32_t*>(key + a0);
    const uint64_t n4 = (a1 - a0) / 4;
    for (uint64_t i = lane; i < n4; i += dev::kWave) {
      const uint32_t q = k4[i];
      atomicAdd(&cnt[q & 0xFFu], 1u);
      atomicAdd(&cnt[(q >> 8) & 0xFFu], 1u);
      atomicAdd(&cnt[(q >> 16) & 0xFFu], 1u);
      atomicAdd(&cnt[q >> 24], 1u);
    }
  } else {
    for (uint64_t e = b0 + lane; e < b1; e += dev::kWave) atomicAdd(&cnt[key[e]], 1u);
  }
  dev::wave_sync();
  // scan: lane l owns columns 4 l .. 4 l + 3
  uint32_t c4[4];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    c4[i] = cnt[lane * 4 + i];
    sum += c4[i];
  }
  uint32_t tot;
  uint32_t x = dev::wave_excl_scan(sum, &tot);
  dev::wave_sync();  // every lane has read its counts
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t c = (sb << 8) + static_cast<uint64_t>(lane * 4 + i);
    if (c < num_features) col_ptr[c] = b0 + x;
    cnt[lane * 4 + i] = x;
    x += c4[i];
  }
  dev::wave_sync();
  // pass 2: entries in order, 64 at a time, ranks among equal keys by ballots
  const uint64_t below = lanes_below();
  for (uint64_t g = b0; g < b1; g += dev::kWave) {
    const uint64_t e = g + lane;
    const bool valid = e < b1;
    const uint32_t k = valid ? key[e] : 0u;
    const uint2 p = valid ? rv[e] : make_uint2(0u, 0u);
    const uint64_t m = match_lanes(k, 8, valid);
    const uint32_t rank = static_cast<uint32_t>(__popcll(m & below));
    const uint32_t n = static_cast<uint32_t>(__popcll(m));
    const uint32_t before = valid ? cnt[k] : 0u;
    dev::wave_sync();
    if (valid) {
      const uint64_t pos = b0 + before + rank;
      if (paired) {
        reinterpret_cast<uint2*>(row_out)[pos] = p;
      } else {
        row_out[pos] = p.x;
        if (val_out != nullptr) val_out[pos] = __uint_as_float(p.y);
      }
      if (rank + 1 == n) cnt[k] = before + n;
    }
    dev::wave_sync();
  }
}

__global__ void k_starts_close(uint64_t* __restrict__ starts, uint64_t n, uint64_t nnz) {
  starts[n] = nnz;
}

__global__ void k_transpose_close(const uint64_t* __restrict__ bstart, uint32_t nbuckets,
                                  uint64_t num_features, uint64_t* __restrict__ col_ptr) {
  col_ptr[num_features] = bstart[nbuckets];
}

size_t AlignUp(size_t n) { return (n + 255) & ~size_t(255); }

struct TransposePlan {
  int low_bits;  // columns per bucket: 2^low_bits
  uint64_t block_elems;  // entries per T1 / T3 block
  uint32_t nbuckets;
  int bucket_bits;
  size_t nblocks;
  size_t g_words, partials_words, h_words, nchunks;
  size_t key_off, row_off, val_off, g_off, partials_off, h_off, chunk_off, total;
  // three levels (low_bits = S > kMaxLowBits): L2 digits 2^(S - 8), super-buckets
  bool three;
  uint64_t nsuper;
  size_t key2_off, rv2_off, super_off;
};

constexpr int kL2Seg = 16;  // L2 segments per bucket
constexpr int kL3Bits = 8;  // L3 digit: the low 8 bits
constexpr int kMaxBits3 = 18;  // S <= 18: 2^28 features

/*!
 * \brief columns per bucket for a feature space: the narrowest of 2^10 ..
 *  2^12 that keeps the buckets <= kMaxBuckets (DMLC_T_LOWBITS forces a
 *  width that fits).  Narrower buckets shrink T4c's LDS cursor table (more
 *  waves per CU) and its ballots, and widen T3's fan-out.
 */
int LowBits(uint64_t num_features) {
  static const int forced = [] {
    const char* v = std::getenv("DMLC_T_LOWBITS");
    return v != nullptr ? std::atoi(v) : 0;
  }();
  auto fits = [&](int b) { return num_features <= (static_cast<uint64_t>(kMaxBuckets) << b); };
  if (forced >= kMinLowBits && forced <= kMaxLowBits && fits(forced)) return forced;
  for (int b = kDefaultLowBits; b < kMaxLowBits; ++b) {
    if (fits(b)) return b;
  }
  return kMaxLowBits;
}

/*! \brief sub-tiles per T1 / T3 block (DMLC_T_BLOCK_SUBS overrides, 1 .. 64):
 *  fewer blocks shrink G (buckets x blocks, written by T1 column by column) */
int BlockSubs() {
  static const int subs = [] {
    const char* v = std::getenv("DMLC_T_BLOCK_SUBS");
    const int k = v != nullptr ? std::atoi(v) : 0;
    return k >= 1 && k <= 64 ? k : kBlockSubs;
  }();
  return subs;
}

TransposePlan Plan(uint64_t nnz, uint64_t num_features) {
  TransposePlan p;
  p.three = num_features > (static_cast<uint64_t>(kMaxBuckets) << kMaxLowBits);
  p.low_bits = LowBits(num_features);
  if (p.three) {
    // S = 16 .. 18: the narrowest bucket width that keeps <= kMaxBuckets buckets
    p.low_bits = 16;
    while (p.low_bits < kMaxBits3 &&
           num_features > (static_cast<uint64_t>(kMaxBuckets) << p.low_bits)) {
      ++p.low_bits;
    }
  }
  const uint64_t low = uint64_t(1) << p.low_bits;
  p.nbuckets = static_cast<uint32_t>((num_features + low - 1) / low);
  if (p.nbuckets == 0) p.nbuckets = 1;
  p.bucket_bits = 0;
  while ((1u << p.bucket_bits) < p.nbuckets) ++p.bucket_bits;
  p.block_elems = static_cast<uint64_t>(BlockSubs()) * kSubElems;
  p.nblocks = (nnz + p.block_elems - 1) / p.block_elems;
  if (p.nblocks == 0) p.nblocks = 1;
  p.g_words = static_cast<size_t>(p.nbuckets) * p.nblocks + 1;  // + the bucket-end sentinel
  p.partials_words = ScanPartials(p.g_words) + 2;
  p.h_words = static_cast<size_t>(p.nbuckets) * kSegments * low;
  p.nsuper = 0;
  if (p.three) {
    const uint64_t mid = uint64_t(1) << (p.low_bits - kL3Bits);
    p.nsuper = static_cast<uint64_t>(p.nbuckets) * mid;
    p.h_words = static_cast<size_t>(p.nbuckets) * kL2Seg * mid;  // (L3 keeps its counts in LDS)
  }
  p.nchunks = (nnz + kChunk - 1) / kChunk;
  size_t off = 0;
  p.key_off = off;
  off += AlignUp(nnz * (p.three ? sizeof(uint32_t) : sizeof(uint16_t)));
  p.row_off = off;
  off += AlignUp(nnz * sizeof(uint32_t));
  p.val_off = off;
  off += AlignUp(nnz * sizeof(float));
  p.g_off = off;
  off += AlignUp(p.g_words * sizeof(uint64_t));
  p.partials_off = off;
  off += AlignUp(p.partials_words * sizeof(uint64_t));
  p.h_off = off;
  off += AlignUp(p.h_words * sizeof(uint32_t));
  p.chunk_off = off;
  off += AlignUp((p.nchunks + 1) * sizeof(uint32_t));
  p.key2_off = p.rv2_off = p.super_off = 0;
  if (p.three) {
    p.key2_off = off;
    off += AlignUp(nnz * sizeof(uint8_t));
    p.rv2_off = off;
    off += AlignUp(nnz * sizeof(uint2));
    p.super_off = off;
    off += AlignUp((p.nsuper + 1) * sizeof(uint64_t));
  }
  p.total = off;
  return p;
}

/*! \brief bucket starts: bstart[b] = G[b * nblocks] after the scan; bstart[nb] = nnz */
__global__ void k_bucket_starts(const uint64_t* __restrict__ G, size_t nblocks, uint32_t nbuckets,
                                uint64_t nnz, uint64_t* __restrict__ bstart) {
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b <= nbuckets;
       b += gridDim.x * blockDim.x) {
    bstart[b] = b < nbuckets ? G[static_cast<size_t>(b) * nblocks] : nnz;
  }
}

/*! \brief T1 .. T4 at 2^kB columns per bucket */
template <typename IndexType, int kB>
void RunSort(const TransposePlan& p, const uint64_t* offset, size_t nrows, uint64_t base,
             uint64_t nnz, const IndexType* index, const float* value, uint64_t num_features,
             uint64_t* col_ptr, uint32_t* row_out, float* val_out, void* scratch,
             uint32_t* error, hipStream_t stream) {
  char* sc = static_cast<char*>(scratch);
  uint16_t* t_key = reinterpret_cast<uint16_t*>(sc + p.key_off);
  // rows alone, or (row, value) pairs over the row + value regions (>= 8 nnz bytes)
  uint32_t* t_row = reinterpret_cast<uint32_t*>(sc + p.row_off);
  uint2* t_rv = reinterpret_cast<uint2*>(sc + p.row_off);
  uint64_t* G = reinterpret_cast<uint64_t*>(sc + p.g_off);
  uint64_t* partials = reinterpret_cast<uint64_t*>(sc + p.partials_off);
  uint32_t* H = reinterpret_cast<uint32_t*>(sc + p.h_off);
  uint32_t* chunk_row = reinterpret_cast<uint32_t*>(sc + p.chunk_off);
  uint64_t* bstart = reinterpret_cast<uint64_t*>(sc + p.total);
  const IndexType* idx = index + base;  // entries [base, base + nnz) of the arrays
  const float* val = value != nullptr ? value + base : nullptr;
  // T1 + T2
  DMLC_HIP_CHECK(hipMemsetAsync(G, 0, p.g_words * sizeof(uint64_t), stream));
  if (nnz != 0) {
    hipLaunchKernelGGL((k_bucket_hist<IndexType, kB>), dim3(p.nblocks), dim3(kThreads), 0, stream,
                       idx, nnz, num_features, p.nbuckets, G, p.nblocks, p.block_elems, error);
  }
  LaunchScanU64(G, p.g_words, partials, partials + p.partials_words - 1, stream);
  hipLaunchKernelGGL(k_bucket_starts, dim3((p.nbuckets + kThreads) / kThreads), dim3(kThreads), 0,
                     stream, G, p.nblocks, p.nbuckets, nnz, bstart);
  // T3
  if (nnz != 0) {
    hipLaunchKernelGGL(k_chunk_rows, dim3((p.nchunks + kThreads - 1) / kThreads), dim3(kThreads),
                       0, stream, offset, nrows, base, nnz, chunk_row);
    hipLaunchKernelGGL((k_bucket_scatter<IndexType, kB>), dim3(p.nblocks), dim3(kThreads), 0,
                       stream, offset, nrows, base, idx, val, nnz, num_features, p.nbuckets,
                       p.bucket_bits, G, p.nblocks, p.block_elems, chunk_row, t_key, t_row,
                       t_rv);
  }
  // T4
  const unsigned nseg = p.nbuckets * kSegments;
  hipLaunchKernelGGL(k_lowkey_hist<kB>, dim3(nseg), dim3(kThreads), 0, stream, t_key, bstart, H);
  hipLaunchKernelGGL(k_lowkey_scan<kB>, dim3(p.nbuckets), dim3(kThreads), 0, stream, H, bstart,
                     num_features, col_ptr);
  // (row, value) pairs when val_out is the float after row_out (8-byte aligned)
  const bool paired = val_out != nullptr && val_out == reinterpret_cast<float*>(row_out) + 1;
  if (paired) {
    CHECK_EQ(reinterpret_cast<uintptr_t>(row_out) & 7u, 0u) << "transpose: pair output not 8-byte aligned";
    hipLaunchKernelGGL((k_lowkey_scatter<true, kB, 8>), dim3(nseg), dim3(dev::kWave), 0, stream,
                       t_key, t_row, t_rv, bstart, H, row_out, val_out);
  } else {
    hipLaunchKernelGGL((k_lowkey_scatter<false, kB, 8>), dim3(nseg), dim3(dev::kWave), 0, stream,
                       t_key, t_row, t_rv, bstart, H, row_out, val_out);
  }
  hipLaunchKernelGGL(k_transpose_close, dim3(1), dim3(1), 0, stream, bstart, p.nbuckets,
                     num_features, col_ptr);
}
/*! \brief the three-level sort (feature spaces above 2^22): T1-T3 into
 *  buckets of 2^S columns with u32 keys, L2 into super-buckets of 256
 *  columns, L3 into the CSC */
template <typename IndexType, int kS>
void RunSort3(const TransposePlan& p, const uint64_t* offset, size_t nrows, uint64_t base,
              uint64_t nnz, const IndexType* index, const float* value, uint64_t num_features,
              uint64_t* col_ptr, uint32_t* row_out, float* val_out, void* scratch,
              uint32_t* error, hipStream_t stream) {
  constexpr int kMid = kS - kL3Bits;  // L2 digit bits
  char* sc = static_cast<char*>(scratch);
  uint32_t* t_key = reinterpret_cast<uint32_t*>(sc + p.key_off);
  uint32_t* t_row = reinterpret_cast<uint32_t*>(sc + p.row_off);
  uint2* t_rv = reinterpret_cast<uint2*>(sc + p.row_off);
  uint64_t* G = reinterpret_cast<uint64_t*>(sc + p.g_off);
  uint64_t* partials = reinterpret_cast<uint64_t*>(sc + p.partials_off);
  uint32_t* H = reinterpret_cast<uint32_t*>(sc + p.h_off);
  uint32_t* chunk_row = reinterpret_cast<uint32_t*>(sc + p.chunk_off);
  uint8_t* t_key2 = reinterpret_cast<uint8_t*>(sc + p.key2_off);
  uint2* t_rv2 = reinterpret_cast<uint2*>(sc + p.rv2_off);
  uint32_t* t_row2 = reinterpret_cast<uint32_t*>(sc + p.rv2_off);
  uint64_t* sstart = reinterpret_cast<uint64_t*>(sc + p.super_off);
  uint64_t* bstart = reinterpret_cast<uint64_t*>(sc + p.total);
  const IndexType* idx = index + base;
  const float* val = value != nullptr ? value + base : nullptr;
  const bool with_values = value != nullptr;
  // L1 = T1 + T2 + T3 at 2^kS columns per bucket (u32 keys)
  DMLC_HIP_CHECK(hipMemsetAsync(G, 0, p.g_words * sizeof(uint64_t), stream));
  if (nnz != 0) {
    hipLaunchKernelGGL((k_bucket_hist<IndexType, kS>), dim3(p.nblocks), dim3(kThreads), 0, stream,
                       idx, nnz, num_features, p.nbuckets, G, p.nblocks, p.block_elems, error);
  }
  LaunchScanU64(G, p.g_words, partials, partials + p.partials_words - 1, stream);
  hipLaunchKernelGGL(k_bucket_starts, dim3((p.nbuckets + kThreads) / kThreads), dim3(kThreads), 0,
                     stream, G, p.nblocks, p.nbuckets, nnz, bstart);
  if (nnz != 0) {
    hipLaunchKernelGGL(k_chunk_rows, dim3((p.nchunks + kThreads - 1) / kThreads), dim3(kThreads),
                       0, stream, offset, nrows, base, nnz, chunk_row);
    hipLaunchKernelGGL((k_bucket_scatter<IndexType, kS, uint32_t>), dim3(p.nblocks),
                       dim3(kThreads), 0, stream, offset, nrows, base, idx, val, nnz,
                       num_features, p.nbuckets, p.bucket_bits, G, p.nblocks, p.block_elems,
                       chunk_row, t_key, t_row, t_rv);
  }
  // L2: per (bucket, segment), digit = key >> 8 -> super-bucket order
  const unsigned n2 = p.nbuckets * kL2Seg;
  hipLaunchKernelGGL((k_digit_hist<uint32_t, kL3Bits, kMid, kL2Seg>), dim3(n2), dim3(kThreads), 0,
                     stream, t_key, bstart, H);
  hipLaunchKernelGGL((k_digit_scan<kMid, kL2Seg>), dim3(p.nbuckets), dim3(kThreads), 0, stream, H,
                     bstart, p.nsuper, sstart);
  hipLaunchKernelGGL(k_starts_close, dim3(1), dim3(1), 0, stream, sstart, p.nsuper, nnz);
  // (L2 always writes (row, value) pairs -- (row, 0) without values -- which L3 reads)
  hipLaunchKernelGGL((k_digit_scatter<uint32_t, kL3Bits, kMid, kL2Seg, true>), dim3(n2),
                     dim3(dev::kWave), 0, stream, t_key, t_row, t_rv, bstart, H, t_key2,
                     with_values ? reinterpret_cast<uint32_t*>(t_rv2) : t_row2, nullptr,
                     with_values);
  // L3: one wave per super-bucket sorts it by the low 8 bits into the CSC
  // (counts, column pointer and placement in one kernel)
  const bool paired = val_out != nullptr && val_out == reinterpret_cast<float*>(row_out) + 1;
  if (paired) {
    CHECK_EQ(reinterpret_cast<uintptr_t>(row_out) & 7u, 0u) << "transpose: pair output not 8-byte aligned";
  }
  (void)t_row2;
  hipLaunchKernelGGL(k_local_sort256, dim3(static_cast<unsigned>((p.nsuper + kWaves - 1) / kWaves)),
                     dim3(kThreads), 0, stream, t_key2, t_rv2, sstart, p.nsuper, num_features,
                     col_ptr, row_out, val_out, paired);
  hipLaunchKernelGGL(k_transpose_close, dim3(1), dim3(1), 0, stream, bstart, p.nbuckets,
                     num_features, col_ptr);
}
}  // namespace

size_t CSRTransposeScratchBytes(uint64_t nnz, uint64_t num_features) {
  // + the bucket-start table
  return Plan(nnz, num_features).total + AlignUp((kMaxBuckets + 1) * sizeof(uint64_t));
}

uint64_t CSRTransposeMaxFeatures() { return static_cast<uint64_t>(kMaxBuckets) << kMaxBits3; }

template <typename IndexType>
void LaunchCSRTranspose(const uint64_t* offset, size_t nrows, uint64_t base, uint64_t nnz,
                        const IndexType* index, const float* value, uint64_t num_features,
                        uint64_t* col_ptr, uint32_t* row_out, float* val_out, void* scratch,
                        uint32_t* error, hipStream_t stream) {
  CHECK_GT(num_features, 0U);
  CHECK_LE(num_features, CSRTransposeMaxFeatures()) << "transpose: num_features above the limit";
  CHECK_LT(nnz, uint64_t(1) << 32) << "transpose: at most 2^32 - 1 entries";
  CHECK_LT(nrows, size_t(1) << 32) << "transpose: at most 2^32 - 1 rows";
  const TransposePlan p = Plan(nnz, num_features);
  if (p.three) {
    switch (p.low_bits) {
      case 16:
        RunSort3<IndexType, 16>(p, offset, nrows, base, nnz, index, value, num_features, col_ptr,
                                row_out, val_out, scratch, error, stream);
        break;
      case 17:
        RunSort3<IndexType, 17>(p, offset, nrows, base, nnz, index, value, num_features, col_ptr,
                                row_out, val_out, scratch, error, stream);
        break;
      default:
        RunSort3<IndexType, 18>(p, offset, nrows, base, nnz, index, value, num_features, col_ptr,
                                row_out, val_out, scratch, error, stream);
        break;
    }
    return;
  }
  switch (p.low_bits) {
    case 10:
      RunSort<IndexType, 10>(p, offset, nrows, base, nnz, index, value, num_features, col_ptr,
                             row_out, val_out, scratch, error, stream);
      break;
    case 11:
      RunSort<IndexType, 11>(p, offset, nrows, base, nnz, index, value, num_features, col_ptr,
                             row_out, val_out, scratch, error, stream);
      break;
    default:
      RunSort<IndexType, 12>(p, offset, nrows, base, nnz, index, value, num_features, col_ptr,
                             row_out, val_out, scratch, error, stream);
      break;
  }
}

template void LaunchCSRTranspose<uint32_t>(const uint64_t*, size_t, uint64_t, uint64_t,
                                           const uint32_t*, const float*, uint64_t, uint64_t*,
                                           uint32_t*, float*, void*, uint32_t*, hipStream_t);
template void LaunchCSRTranspose<uint64_t>(const uint64_t*, size_t, uint64_t, uint64_t,
                                           const uint64_t*, const float*, uint64_t, uint64_t*,
                                           uint32_t*, float*, void*, uint32_t*, hipStream_t);

}  // namespace gpu
}  // namespace dmlc
