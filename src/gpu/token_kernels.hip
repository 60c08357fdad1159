/*!
 * \file src/gpu/token_kernels.hip
 * \brief Token-parallel fast path of the LibSVM / LibFM parse (one lane per
 *  token), used for every chunk whose lines are "regular" (first token =
 *  label, every later token a feature).  Irregular chunks (qid tokens,
 *  tokens without digits, label-less lines) are detected on device and
 *  re-parsed with the exact wave-per-line kernels of text_kernels.hip.
 *
 *  T1a k_tok_count : per 4 KiB tile, count line starts and token starts with
 *                    SWAR byte masks (16 B per lane, global_load_dwordx4);
 *                    the two counts are packed into one u64 and scanned.
 *  T1b k_tok_emit  : recompute the masks, workgroup-scan the packed counts
 *                    and write line_start[], line_first_tok[], tok_pos[],
 *                    tok_line[] (compaction without atomics).
 *  T2  k_rowinfo   : per line (row_valid << 32 | tokens - 1), scanned by K3
 *                    into (row, nnz) prefixes.
 *  T3  k_tok_fill  : one lane per token: 3 x 16 B loads around the token,
 *                    funnel shift into 8 VGPRs, separator mask -> length, the
 *                    shared strtonum.h ParsePair on a register iterator, and
 *                    coalesced index/value stores at offset[row] + ord - 1.
 *                    K8 max reduction: wave max + one atomicMax per wave.
 * All passes read the chunk at HBM rate; the parse itself has 4M independent
 * lanes per 64 MiB chunk instead of a per-line dependency chain.
 */
#include <hip/hip_runtime.h>

#include "../data/strtonum.h"
#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {

namespace {
constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t blank_eol_mask(uint4 v, uint32_t* eol_out) {
  const uint32_t eol = dev::byte_eq_mask(v, '\n') | dev::byte_eq_mask(v, '\r');
  *eol_out = eol;
  return eol | dev::byte_eq_mask(v, ' ') | dev::byte_eq_mask(v, '\t');
}

/*!
 * \brief line-start and token-start bits of the 16 bytes at pos.
 *  line start: non-EOL byte after an EOL (or at 0); token start: non-separator
 *  byte after a separator (or at 0).
 */
__device__ __forceinline__ void tile_masks(const uint8_t* __restrict__ text, size_t n, size_t pos,
                                           uint32_t* lmask, uint32_t* tmask) {
  const int lane = dev::lane_id();
  uint4 v = make_uint4(0, 0, 0, 0);
  if (pos < n) v = *reinterpret_cast<const uint4*>(text + pos);
  uint32_t eol;
  const uint32_t sep = blank_eol_mask(v, &eol);
  const uint32_t prev_last = __shfl_up(v.w >> 24, 1, dev::kWave);
  uint32_t pc;
  if (lane == 0) {
    pc = pos == 0 ? '\n' : text[pos - 1];
  } else {
    pc = prev_last;
  }
  const uint32_t prev_eol = (pc == '\n' || pc == '\r') ? 1u : 0u;
  const uint32_t prev_sep = (prev_eol || pc == ' ' || pc == '\t') ? 1u : 0u;
  uint32_t valid = 0xFFFFu;
  if (pos >= n) {
    valid = 0;
  } else if (n - pos < 16) {
    valid = (1u << (n - pos)) - 1u;
  }
  *lmask = ~eol & ((eol << 1) | prev_eol) & valid & 0xFFFFu;
  *tmask = ~sep & ((sep << 1) | prev_sep) & valid & 0xFFFFu;
}

__global__ __launch_bounds__(kThreads) void k_tok_count(const uint8_t* __restrict__ text, size_t n,
                                                        uint64_t* __restrict__ tile_counts) {
  __shared__ uint64_t smem[4];
  const size_t pos = blockIdx.x * kLineTileBytes + threadIdx.x * 16;
  uint32_t lm, tm;
  tile_masks(text, n, pos, &lm, &tm);
  const uint64_t packed = (static_cast<uint64_t>(__popc(lm)) << 32) | __popc(tm);
  const uint64_t s = dev::block_sum_256<uint64_t>(packed, smem);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void k_tok_emit(const uint8_t* __restrict__ text, size_t n,
                                                       const uint64_t* __restrict__ tile_base,
                                                       uint32_t* __restrict__ line_starts,
                                                       uint32_t* __restrict__ line_first_tok,
                                                       uint32_t* __restrict__ tok_pos,
                                                       uint32_t* __restrict__ tok_line) {
  __shared__ uint64_t smem[4];
  const size_t pos = blockIdx.x * kLineTileBytes + threadIdx.x * 16;
  uint32_t lm, tm;
  tile_masks(text, n, pos, &lm, &tm);
  const uint64_t packed = (static_cast<uint64_t>(__popc(lm)) << 32) | __popc(tm);
  uint64_t tot;
  const uint64_t base = dev::block_excl_scan_256<uint64_t>(packed, smem, &tot) + tile_base[blockIdx.x];
  uint32_t line = static_cast<uint32_t>(base >> 32);  // lines started before this lane
  uint32_t tok = static_cast<uint32_t>(base & 0xffffffffu);
  uint32_t all = lm | tm;
  while (all != 0) {
    const int j = __ffs(all) - 1;
    all &= all - 1;
    const uint32_t bit = 1u << j;
    if (lm & bit) {
      line_starts[line] = static_cast<uint32_t>(pos + j);
      line_first_tok[line] = tok;
      ++line;
    }
    if (tm & bit) {
      tok_pos[tok] = static_cast<uint32_t>(pos + j);
      tok_line[tok] = line - 1;  // tokens only occur inside lines
      ++tok;
    }
  }
}

__global__ void k_rowinfo(const uint32_t* __restrict__ line_first_tok, size_t nlines,
                          uint32_t ntok_total, uint64_t* __restrict__ line_info) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < nlines;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const uint32_t b = line_first_tok[i];
    const uint32_t e = i + 1 < nlines ? line_first_tok[i + 1] : ntok_total;
    const uint32_t nt = e - b;
    line_info[i] = nt != 0 ? ((1ull << 32) | (nt - 1)) : 0ull;
  }
}

/*! \brief register window iterator (same as text_kernels.hip) */
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

/*! \brief bytes [p, p+32) of the chunk into 8 VGPRs (3 aligned 16-byte loads) */
__device__ __forceinline__ RegIter load_window(const uint8_t* __restrict__ text, uint32_t p) {
  const uint4* src = reinterpret_cast<const uint4*>(text + (p & ~15u));
  const uint4 a = src[0], b = src[1], c = src[2];
  uint32_t d[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
  const uint32_t s = p & 15u;
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

/*! \brief bit i set when byte i of the 32-byte window is a blank / EOL */
__device__ __forceinline__ uint32_t window_sep_mask(const RegIter& r) {
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const uint4 v = make_uint4(r.w[4 * i], r.w[4 * i + 1], r.w[4 * i + 2], r.w[4 * i + 3]);
    uint32_t eol;
    m |= blank_eol_mask(v, &eol) << (16 * i);
  }
  return m;
}

template <TextFormat F, typename IndexType>
__global__ __launch_bounds__(kThreads) void k_tok_fill(
    const uint8_t* __restrict__ text, size_t n, const uint32_t* __restrict__ tok_pos,
    const uint32_t* __restrict__ tok_line, size_t ntok, const uint32_t* __restrict__ line_first_tok,
    const uint64_t* __restrict__ line_info, FillTarget<IndexType> out,
    MetaPartial* __restrict__ partials) {
  uint64_t mx_index = 0, mx_field = 0;
  bool any_value = false, any_weight = false, irregular = false, neg = false;
  for (size_t k = blockIdx.x * static_cast<size_t>(kThreads) + threadIdx.x; k < ntok;
       k += static_cast<size_t>(gridDim.x) * kThreads) {
    const uint32_t p = tok_pos[k];
    const uint32_t line = tok_line[k];
    const uint32_t ord = static_cast<uint32_t>(k) - line_first_tok[line];
    const uint64_t info = line_info[line];
    const uint64_t row = out.row_base + (info >> 32);
    const uint64_t nnz0 = out.nnz_base + (info & 0xffffffffull);
    RegIter b = load_window(text, p);
    const uint32_t sm = window_sep_mask(b);
    bool bad = false;
    auto parse = [&](auto beg, auto end) {
      if (ord == 0) {
        float l = 0.0f, wgt = 0.0f;
        const int r = data::ParsePair<float, float>(beg, end, &l, &wgt, &bad);
        if (r < 1) {
          irregular = true;
          return;
        }
        if (row < out.row_limit) {
          out.label[row] = l;
          out.offset[row] = nnz0;
          if (out.weight != nullptr) out.weight[row] = r == 2 ? wgt : 1.0f;
          if (out.qid != nullptr) out.qid[row] = 0;  // qid lines take the exact path
        }
        any_weight |= (r == 2);
        return;
      }
      const uint64_t pos = nnz0 + ord - 1;
      if (pos >= out.nnz_limit) {
        irregular = true;
        return;
      }
      if constexpr (F == TextFormat::kLibSVM) {
        if (ord == 1 && *beg == 'q') {
          // "qid:" tokens are not features: the exact path handles the chunk
          auto it = beg;
          ++it;
          if (it != end && *it == 'i') {
            irregular = true;
            return;
          }
        }
        IndexType idx = 0;
        float v = 0.0f;
        const int r = data::ParsePair<IndexType, float>(beg, end, &idx, &v, &bad);
        if (r < 1) {
          irregular = true;
          return;
        }
        out.index[pos] = idx;
        out.value[pos] = r == 2 ? v : 1.0f;
        any_value |= (r == 2);
        if (static_cast<uint64_t>(idx) > mx_index) mx_index = idx;
      } else {
        IndexType fid = 0, idx = 0;
        float v = 0.0f;
        const int r = data::ParseTriple<IndexType, IndexType, float>(beg, end, &fid, &idx, &v, &bad);
        if (r < 2) {
          irregular = true;
          return;
        }
        out.field[pos] = fid;
        out.index[pos] = idx;
        out.value[pos] = r == 3 ? v : 1.0f;
        any_value |= (r == 3);
        if (static_cast<uint64_t>(idx) > mx_index) mx_index = idx;
        if (static_cast<uint64_t>(fid) > mx_field) mx_field = fid;
      }
    };
    if (sm != 0) {
      RegIter e = b;
      e.pos = static_cast<uint32_t>(__ffs(sm) - 1);
      if (p + e.pos > n) e.pos = static_cast<uint32_t>(n - p);
      parse(b, e);
    } else {
      // token longer than 32 bytes: pointer path over HBM
      uint32_t q = p + 32;
      while (q < n && !(text[q] == ' ' || text[q] == '\t' || text[q] == '\n' || text[q] == '\r')) ++q;
      const char* cp = reinterpret_cast<const char*>(text + p);
      parse(cp, cp + (q - p));
    }
    neg |= bad;
  }
  // K8: workgroup reduction into this block's slot (no same-address atomics)
  unsigned fl = 0;
  if (any_value) fl |= kFlagValue;
  if (any_weight) fl |= kFlagWeight;
  if (irregular) fl |= kFlagIrregular;
  if (neg) fl |= kFlagNegIndex;
  if (F == TextFormat::kLibFM) fl |= kFlagField;
  dev::block_store_partial(static_cast<unsigned long long>(mx_index),
                           static_cast<unsigned long long>(mx_field), fl, partials);
}

int Grid(size_t work, size_t per_block, size_t cap) {
  size_t b = (work + per_block - 1) / per_block;
  if (b == 0) b = 1;
  return static_cast<int>(b < cap ? b : cap);
}
}  // namespace

void LaunchTokenCount(const char* text, size_t nbytes, uint64_t* tile_scratch,
                      uint64_t* packed_total, hipStream_t stream) {
  const size_t ntiles = (nbytes + kLineTileBytes - 1) / kLineTileBytes;
  if (ntiles == 0) {
    (void)hipMemsetAsync(packed_total, 0, sizeof(uint64_t), stream);
    return;
  }
  hipLaunchKernelGGL(k_tok_count, dim3(ntiles), dim3(kThreads), 0, stream,
                     reinterpret_cast<const uint8_t*>(text), nbytes, tile_scratch);
  LaunchScanU64(tile_scratch, ntiles, tile_scratch + ntiles + 1, packed_total, stream);
}

void LaunchTokenEmit(const char* text, size_t nbytes, const uint64_t* tile_scratch,
                     uint32_t* line_starts, uint32_t* line_first_tok, uint32_t* tok_pos,
                     uint32_t* tok_line, hipStream_t stream) {
  const size_t ntiles = (nbytes + kLineTileBytes - 1) / kLineTileBytes;
  if (ntiles == 0) return;
  hipLaunchKernelGGL(k_tok_emit, dim3(ntiles), dim3(kThreads), 0, stream,
                     reinterpret_cast<const uint8_t*>(text), nbytes, tile_scratch, line_starts,
                     line_first_tok, tok_pos, tok_line);
}

void LaunchRowInfo(const uint32_t* line_first_tok, size_t nlines, size_t ntok,
                   uint64_t* line_info, hipStream_t stream) {
  if (nlines == 0) return;
  hipLaunchKernelGGL(k_rowinfo, dim3(Grid(nlines, kThreads, 4096)), dim3(kThreads), 0, stream,
                     line_first_tok, nlines, static_cast<uint32_t>(ntok), line_info);
}

template <typename IndexType>
void LaunchTokenFill(const char* text, size_t nbytes, TextFormat format, const uint32_t* tok_pos,
                     const uint32_t* tok_line, size_t ntok, const uint32_t* line_first_tok,
                     const uint64_t* line_info, const FillTarget<IndexType>& out, uint64_t nrows,
                     uint64_t nnz, MetaPartial* partials, ChunkMeta* meta, hipStream_t stream) {
  if (ntok != 0) {
    // ~1000 workgroups x 4 tokens per lane: enough waves to fill 256 CUs,
    // few enough partial slots for the single-workgroup reduction
    const dim3 grid(Grid(ntok, kThreads * 4, 2048)), block(kThreads);
    const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
    if (format == TextFormat::kLibFM) {
      hipLaunchKernelGGL((k_tok_fill<TextFormat::kLibFM, IndexType>), grid, block, 0, stream, t,
                         nbytes, tok_pos, tok_line, ntok, line_first_tok, line_info, out, partials);
    } else {
      hipLaunchKernelGGL((k_tok_fill<TextFormat::kLibSVM, IndexType>), grid, block, 0, stream, t,
                         nbytes, tok_pos, tok_line, ntok, line_first_tok, line_info, out, partials);
    }
    LaunchReducePartials(partials, static_cast<int>(grid.x), meta, stream);
  }
  LaunchCloseOffsets(out.offset, out.row_base + nrows, out.nnz_base + nnz, stream);
}

template void LaunchTokenFill<uint32_t>(const char*, size_t, TextFormat, const uint32_t*,
                                        const uint32_t*, size_t, const uint32_t*, const uint64_t*,
                                        const FillTarget<uint32_t>&, uint64_t, uint64_t,
                                        MetaPartial*, ChunkMeta*, hipStream_t);
template void LaunchTokenFill<uint64_t>(const char*, size_t, TextFormat, const uint32_t*,
                                        const uint32_t*, size_t, const uint32_t*, const uint64_t*,
                                        const FillTarget<uint64_t>&, uint64_t, uint64_t,
                                        MetaPartial*, ChunkMeta*, hipStream_t);

}  // namespace gpu
}  // namespace dmlc
