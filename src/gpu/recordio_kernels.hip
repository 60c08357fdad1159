/*!
 * \file src/gpu/recordio_kernels.hip
 * \brief K7: RecordIO decode on the GPU.
 *
 * Replaces the host record walk of RecordIOSplitter::ExtractNextRecord /
 * RecordIOChunkReader (reference `src/io/recordio_split.cc:44-82`,
 * `src/recordio.cc:85-156`).  The writer escapes every 4-byte-aligned
 * occurrence of the magic word inside a payload (`src/recordio.cc:22-38`),
 * so in a chunk that starts at a record head, *every* aligned magic word is a
 * part header and a record head is one whose lrec carries cflag 0 (whole) or
 * 1 (first part).  That makes the index embarrassingly parallel:
 *
 *   K7a count  : 256 threads x 16 words per 4096-word tile, dwordx4 loads,
 *                block reduce -> tile counts, device scan (K3)
 *   K7b emit   : same tiling, 4 ordered block scans per tile -> head positions
 *   K7c lengths: one lane per record; multi-part chains (rare) are walked by
 *                that lane; continuation parts add len + 4 (re-inserted magic)
 *   K7d gather : one wave64 per record copies its parts to the packed output
 *                (u32 stores when the destination is aligned, bytes otherwise)
 */
#include <hip/hip_runtime.h>

#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {
namespace {

using namespace dev;  // NOLINT(build/namespaces)

constexpr int kThreads = 256;
constexpr uint32_t kMagic = 0xced7230aU;
constexpr size_t kTileWords = 4096;  // 256 threads x 4 iterations x uint4

__device__ __forceinline__ uint32_t cflag_of(uint32_t lrec) { return (lrec >> 29) & 7U; }
__device__ __forceinline__ uint32_t len_of(uint32_t lrec) { return lrec & ((1U << 29) - 1U); }

/*! \brief bit k set when word i0+k (k < 4) is a record head */
__device__ __forceinline__ uint32_t head_mask(const uint32_t* __restrict__ w, size_t n, size_t i0) {
  uint32_t v[4];
  if (i0 + 4 <= n) {
    uint4 q = *reinterpret_cast<const uint4*>(w + i0);
    v[0] = q.x;
    v[1] = q.y;
    v[2] = q.z;
    v[3] = q.w;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (i0 + k < n) ? w[i0 + k] : 0U;
  }
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (v[k] == kMagic && i0 + k + 1 < n && cflag_of(w[i0 + k + 1]) <= 1U) m |= 1U << k;
  }
  return m;
}

__global__ __launch_bounds__(kThreads) void k_rec_count(const uint32_t* __restrict__ w, size_t n,
                                                        uint64_t* __restrict__ tile_counts) {
  __shared__ uint64_t smem[4];
  const size_t base = blockIdx.x * kTileWords;
  uint64_t c = 0;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const size_t i0 = base + it * (kThreads * 4) + threadIdx.x * 4;
    if (i0 < n) c += __popc(head_mask(w, n, i0));
  }
  const uint64_t total = block_sum_256(c, smem);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

__global__ __launch_bounds__(kThreads) void k_rec_emit(const uint32_t* __restrict__ w, size_t n,
                                                       const uint64_t* __restrict__ tile_offsets,
                                                       uint32_t* __restrict__ head_pos) {
  __shared__ uint32_t smem[2][4];
  const size_t base = blockIdx.x * kTileWords;
  uint64_t out = tile_offsets[blockIdx.x];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const size_t i0 = base + it * (kThreads * 4) + threadIdx.x * 4;
    uint32_t m = i0 < n ? head_mask(w, n, i0) : 0U;
    uint32_t tot;
    // double-buffered scratch: the scan's barrier of iteration it+1 orders
    // every read of buffer it&1 before its reuse in iteration it+2
    uint32_t off = block_excl_scan_256(static_cast<uint32_t>(__popc(m)), smem[it & 1], &tot);
    while (m != 0) {
      const int k = __ffs(m) - 1;
      m &= m - 1;
      head_pos[out + off++] = static_cast<uint32_t>(i0 + k);
    }
    out += tot;
  }
}

__global__ __launch_bounds__(kThreads) void k_rec_lengths(const uint32_t* __restrict__ w, size_t n,
                                                          const uint32_t* __restrict__ head_pos,
                                                          size_t nrec, uint64_t* __restrict__ rec_len,
                                                          uint32_t* __restrict__ err) {
  const size_t r = blockIdx.x * static_cast<size_t>(kThreads) + threadIdx.x;
  if (r >= nrec) return;
  size_t p = head_pos[r];
  const uint32_t lrec = w[p + 1];
  uint64_t total = len_of(lrec);
  size_t q = p + 2 + (len_of(lrec) + 3) / 4;
  uint32_t e = q > n ? kRecErrTruncated : 0U;
  if (cflag_of(lrec) == 1U) {
    for (;;) {
      if (q + 2 > n) {
        e |= kRecErrTruncated;
        break;
      }
      const uint32_t l2 = w[q + 1];
      const uint32_t cf = cflag_of(l2);
      if (w[q] != kMagic || (cf != 2U && cf != 3U)) {
        e |= kRecErrBadPart;
        break;
      }
      total += 4 + len_of(l2);
      q += 2 + (len_of(l2) + 3) / 4;
      if (q > n) e |= kRecErrTruncated;
      if (cf == 3U) break;
    }
  }
  rec_len[r] = total;
  if (e != 0) atomicOr(err, e);
}

__device__ __forceinline__ void copy_part(const uint32_t* __restrict__ src, uint32_t len,
                                          uint8_t* __restrict__ dst, int lane) {
  const uint32_t nw = (len + 3) / 4;
  const bool aligned = (reinterpret_cast<uintptr_t>(dst) & 3U) == 0;
  for (uint32_t j = lane; j < nw; j += kWave) {
    const uint32_t v = src[j];
    const uint32_t nb = min(4U, len - 4 * j);
    if (aligned && nb == 4) {
      *reinterpret_cast<uint32_t*>(dst + 4 * j) = v;
    } else {
      for (uint32_t b = 0; b < nb; ++b) dst[4 * j + b] = static_cast<uint8_t>(v >> (8 * b));
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_rec_gather(const uint32_t* __restrict__ w, size_t n,
                                                         const uint32_t* __restrict__ head_pos,
                                                         size_t nrec,
                                                         const uint64_t* __restrict__ rec_off,
                                                         uint8_t* __restrict__ out) {
  const size_t r = blockIdx.x * static_cast<size_t>(kThreads / kWave) + threadIdx.x / kWave;
  if (r >= nrec) return;
  const int lane = lane_id();
  size_t p = head_pos[r];
  uint8_t* dst = out + rec_off[r];
  uint8_t* const end = out + rec_off[r + 1];
  bool first = true;
  for (;;) {
    if (p + 2 > n) return;  // truncated: flagged by k_rec_lengths
    const uint32_t lrec = w[p + 1];
    const uint32_t cf = cflag_of(lrec);
    const uint32_t len = len_of(lrec);
    if (!first) {
      if (lane < 4) dst[lane] = static_cast<uint8_t>(kMagic >> (8 * lane));
      dst += 4;
    }
    if (dst + len > end || p + 2 + (len + 3) / 4 > n) return;  // malformed: flagged
    copy_part(w + p + 2, len, dst, lane);
    dst += len;
    p += 2 + (len + 3) / 4;
    if (cf == 0U || cf == 3U || (!first && cf != 2U)) return;
    first = false;
  }
}

}  // namespace

size_t RecordIOTiles(size_t nwords) { return (nwords + kTileWords - 1) / kTileWords; }

void LaunchRecordIOCount(const uint32_t* words, size_t nwords, uint64_t* tile_counts,
                         uint64_t* partials, uint64_t* nrec, hipStream_t stream) {
  const size_t tiles = RecordIOTiles(nwords);
  if (tiles == 0) {
    (void)hipMemsetAsync(nrec, 0, sizeof(uint64_t), stream);
    return;
  }
  hipLaunchKernelGGL(k_rec_count, dim3(tiles), dim3(kThreads), 0, stream, words, nwords,
                     tile_counts);
  LaunchScanU64(tile_counts, tiles, partials, nrec, stream);
}

void LaunchRecordIOEmit(const uint32_t* words, size_t nwords, const uint64_t* tile_counts,
                        uint32_t* head_pos, hipStream_t stream) {
  const size_t tiles = RecordIOTiles(nwords);
  if (tiles == 0) return;
  hipLaunchKernelGGL(k_rec_emit, dim3(tiles), dim3(kThreads), 0, stream, words, nwords,
                     tile_counts, head_pos);
}

void LaunchRecordIOLengths(const uint32_t* words, size_t nwords, const uint32_t* head_pos,
                           size_t nrec, uint64_t* rec_len, uint32_t* err, hipStream_t stream) {
  if (nrec == 0) return;
  const size_t blocks = (nrec + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(k_rec_lengths, dim3(blocks), dim3(kThreads), 0, stream, words, nwords,
                     head_pos, nrec, rec_len, err);
}

void LaunchRecordIOGather(const uint32_t* words, size_t nwords, const uint32_t* head_pos,
                          size_t nrec, const uint64_t* rec_off, uint8_t* out,
                          hipStream_t stream) {
  if (nrec == 0) return;
  const size_t per_block = kThreads / kWave;
  const size_t blocks = (nrec + per_block - 1) / per_block;
  hipLaunchKernelGGL(k_rec_gather, dim3(blocks), dim3(kThreads), 0, stream, words, nwords,
                     head_pos, nrec, rec_off, out);
}

}  // namespace gpu
}  // namespace dmlc
