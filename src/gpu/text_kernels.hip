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
 *    2 KiB LDS window (two 1 KiB pieces, 16 B per lane, ds_write_b128): token
 *    starts are found from the registers just loaded (blank/delimiter SWAR
 *    masks + a shuffle for the previous byte), token ordinals come from a wave
 *    prefix sum, and every lane parses the tokens that start in its 16 bytes
 *    straight out of LDS (tokens that run past the window fall back to global
 *    memory).  K4 writes index/value at offset + rank, where rank is a second
 *    wave prefix sum over valid feature tokens, and reduces max(index) with one
 *    atomicMax per wave (K8).
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
struct LineWindow {
  uint8_t* win;    // this wave's LDS window (kWindow bytes)
  uint32_t wbase;  // text position of win[0]
};

__device__ __forceinline__ uint8_t byte_at(const uint8_t* __restrict__ text, const LineWindow& w,
                                           uint32_t q) {
  const uint32_t off = q - w.wbase;
  return off < kWindow ? w.win[off] : text[q];
}

template <TextFormat F>
__device__ __forceinline__ bool is_sep(uint8_t c, char delim) {
  if constexpr (F == TextFormat::kCSV) {
    return c == static_cast<uint8_t>(delim) || c == '\n' || c == '\r';
  } else {
    return c == ' ' || c == '\t' || c == '\n' || c == '\r';
  }
}

/*! \brief token-start bits of the 16 bytes at `pos` (within line [b, e)) */
template <TextFormat F>
__device__ __forceinline__ uint32_t token_start_mask(uint4 v, uint8_t prevb, uint32_t pos,
                                                     uint32_t b, uint32_t e, char delim) {
  uint32_t valid = 0xFFFFu;
  if (pos + 16 > e) valid = pos >= e ? 0u : ((1u << (e - pos)) - 1u);
  if (pos < b) valid &= ~((1u << (b - pos)) - 1u);
  const uint32_t eol = eol_mask(v);
  if constexpr (F == TextFormat::kCSV) {
    const uint32_t dl = dev::byte_eq_mask(v, static_cast<uint8_t>(delim));
    const uint32_t prev_dl = prevb == static_cast<uint8_t>(delim) ? 1u : 0u;
    uint32_t starts = ~eol & ((dl << 1) | prev_dl);
    if (b >= pos && b < pos + 16) starts |= 1u << (b - pos);  // the line start is a field
    return starts & valid;
  } else {
    const uint32_t sep = eol | dev::byte_eq_mask(v, ' ') | dev::byte_eq_mask(v, '\t');
    const uint32_t prev_sep = (prevb == ' ' || prevb == '\t' || prevb == '\n' || prevb == '\r') ? 1u : 0u;
    return ~sep & ((sep << 1) | prev_sep) & valid;
  }
}

/*!
 * \brief stream line [b, e) through the wave's LDS window and call
 *  `vis.classify(...)` for every token (phase 1); when `kEmit`, tokens whose
 *  classify returned 1 are passed to `vis.emit(..., rank)` (phase 2) where rank
 *  counts the earlier such tokens of the line.
 */
template <TextFormat F, bool kEmit, class Visitor>
__device__ void walk_line(const uint8_t* __restrict__ text, uint32_t b, uint32_t e,
                          uint8_t* win, char delim, Visitor& vis) {
  const int lane = dev::lane_id();
  LineWindow w{win, b & ~15u};
  uint4* win4 = reinterpret_cast<uint4*>(win);
  auto load = [&](uint32_t addr) -> uint4 {
    return addr < e ? *reinterpret_cast<const uint4*>(text + addr) : make_uint4(0, 0, 0, 0);
  };
  uint4 vcur = load(w.wbase + 16 * lane);
  uint4 vnext = load(w.wbase + kPiece + 16 * lane);
  win4[lane] = vcur;
  win4[64 + lane] = vnext;
  dev::wave_sync();
  uint32_t tok_base = 0;   // tokens in earlier pieces (wave-uniform)
  uint32_t rank_base = 0;  // emitted tokens in earlier pieces (wave-uniform)
  uint8_t prev_last = '\n';
  for (uint32_t pstart = w.wbase; pstart < e; pstart += kPiece) {
    const uint32_t pos = pstart + 16 * lane;
    uint8_t prevb = static_cast<uint8_t>(__shfl_up(vcur.w >> 24, 1, dev::kWave));
    if (lane == 0) prevb = prev_last;
    const uint32_t smask = token_start_mask<F>(vcur, prevb, pos, b, e, delim);
    uint32_t ntok_total;
    const uint32_t tok_excl = dev::wave_excl_scan<uint32_t>(__popc(smask), &ntok_total);
    // phase 1: classify
    uint32_t m = smask;
    uint32_t ord = tok_base + tok_excl;
    uint32_t nsel = 0;
    while (m != 0) {
      const int j = __ffs(m) - 1;
      m &= m - 1;
      const uint32_t p = pos + j;
      uint32_t q = p;
      while (q < e && !is_sep<F>(byte_at(text, w, q), delim)) ++q;
      const char* tp = (q - w.wbase <= kWindow)
                           ? reinterpret_cast<const char*>(w.win + (p - w.wbase))
                           : reinterpret_cast<const char*>(text + p);
      nsel += vis.classify(tp, q - p, ord);
      ++ord;
    }
    vis.after_classify(tok_base, ntok_total);
    if constexpr (kEmit) {
      uint32_t nsel_total;
      uint32_t rank = rank_base + dev::wave_excl_scan<uint32_t>(nsel, &nsel_total);
      if (vis.emit_enabled()) {
        m = smask;
        ord = tok_base + tok_excl;
        while (m != 0) {
          const int j = __ffs(m) - 1;
          m &= m - 1;
          const uint32_t p = pos + j;
          uint32_t q = p;
          while (q < e && !is_sep<F>(byte_at(text, w, q), delim)) ++q;
          const char* tp = (q - w.wbase <= kWindow)
                               ? reinterpret_cast<const char*>(w.win + (p - w.wbase))
                               : reinterpret_cast<const char*>(text + p);
          if (vis.selected(tp, q - p, ord)) vis.emit(tp, q - p, ord, rank++);
          ++ord;
        }
      }
      rank_base += nsel_total;
    }
    tok_base += ntok_total;
    prev_last = static_cast<uint8_t>(__shfl(vcur.w >> 24, 63, dev::kWave));
    // slide the window by one piece
    dev::wave_sync();
    vcur = vnext;
    vnext = load(pstart + 2 * kPiece + 16 * lane);
    win4[lane] = vcur;
    win4[64 + lane] = vnext;
    w.wbase += kPiece;
    dev::wave_sync();
  }
}

__device__ __forceinline__ bool has_digitchar(const char* tp, uint32_t len) {
  for (uint32_t i = 0; i < len; ++i) {
    if (data::isdigitchars(tp[i])) return true;
  }
  return false;
}
__device__ __forceinline__ bool is_qid(const char* tp, uint32_t len) {
  return len >= 4 && tp[0] == 'q' && tp[1] == 'i' && tp[2] == 'd' && tp[3] == ':';
}
/*! \brief `a[:b[:c]]` has at least two parts (LibFM feature rule) */
__device__ __forceinline__ bool has_two_parts(const char* tp, uint32_t len) {
  uint32_t i = 0;
  while (i < len && !data::isdigitchars(tp[i])) ++i;
  if (i == len) return false;
  while (i < len && data::isdigitchars(tp[i])) ++i;
  return i < len && tp[i] == ':';
}

/*!
 * \brief per-line visitor: phase-1 classification of tokens by role
 *  (label / weight / qid / feature), phase-2 emission of feature tokens.
 */
template <TextFormat F, typename IndexType>
struct LineVisitor {
  // configuration
  int label_col, weight_col;
  // label-token state (only the lane owning token 0 / the label column sets it)
  bool is_label_lane{false}, label_ok{false}, has_weight{false};
  float label{0.0f}, weight{1.0f};
  bool is_qid_lane{false};
  uint64_t qid{0};
  // wave-uniform row validity
  int row_state{0};  // 0 unknown, 1 ok, -1 invalid
  // fill target (phase 2)
  IndexType* index{nullptr};
  float* value{nullptr};
  IndexType* field{nullptr};
  uint64_t nnz_pos{0};
  uint64_t nnz_limit{~0ull};
  uint64_t max_index{0}, max_field{0};
  bool any_value{false}, neg{false}, overflow{false};

  __device__ uint32_t classify(const char* tp, uint32_t len, uint32_t ord) {
    if constexpr (F == TextFormat::kCSV) {
      if (static_cast<int>(ord) == label_col) {
        is_label_lane = true;
        label_ok = true;
        uint32_t i = 0;
        while (i < len && data::isspace(tp[i])) ++i;
        label = data::StrToFloat(tp + i, tp + len, nullptr);
        return 0;
      }
      if (static_cast<int>(ord) == weight_col) {
        has_weight = true;
        uint32_t i = 0;
        while (i < len && data::isspace(tp[i])) ++i;
        weight = data::StrToFloat(tp + i, tp + len, nullptr);
        return 0;
      }
      return 1;
    } else {
      if (ord == 0) {
        is_label_lane = true;
        float l = 0.0f, wgt = 0.0f;
        bool bad;
        const int r = data::ParsePair<float, float>(tp, tp + len, &l, &wgt, &bad);
        label_ok = r >= 1;
        if (r >= 1) label = l;
        if (r == 2) {
          has_weight = true;
          weight = wgt;
        }
        return 0;
      }
      if constexpr (F == TextFormat::kLibSVM) {
        if (ord == 1 && is_qid(tp, len)) {
          is_qid_lane = true;
          qid = static_cast<uint64_t>(data::StrToInt<int64_t>(tp + 4, tp + len, nullptr));
          return 0;
        }
        return has_digitchar(tp, len) ? 1u : 0u;
      } else {
        return has_two_parts(tp, len) ? 1u : 0u;
      }
    }
  }
  /*! \brief same decision as classify, without side effects (phase 2) */
  __device__ bool selected(const char* tp, uint32_t len, uint32_t ord) const {
    if constexpr (F == TextFormat::kCSV) {
      return static_cast<int>(ord) != label_col && static_cast<int>(ord) != weight_col;
    } else {
      if (ord == 0) return false;
      if constexpr (F == TextFormat::kLibSVM) {
        if (ord == 1 && is_qid(tp, len)) return false;
        return has_digitchar(tp, len);
      } else {
        return has_two_parts(tp, len);
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
  __device__ void emit(const char* tp, uint32_t len, uint32_t ord, uint32_t rank) {
    const uint64_t pos = nnz_pos + rank;
    // defensive bound: a count/fill disagreement must never write out of bounds
    if (pos >= nnz_limit) {
      overflow = true;
      return;
    }
    bool bad = false;
    if constexpr (F == TextFormat::kCSV) {
      uint32_t i = 0;
      while (i < len && data::isspace(tp[i])) ++i;
      const float v = data::StrToFloat(tp + i, tp + len, nullptr);
      index[pos] = static_cast<IndexType>(rank);
      value[pos] = v;
      if (rank > max_index) max_index = rank;
    } else if constexpr (F == TextFormat::kLibSVM) {
      IndexType idx = 0;
      float v = 0.0f;
      const int r = data::ParsePair<IndexType, float>(tp, tp + len, &idx, &v, &bad);
      index[pos] = idx;
      value[pos] = r == 2 ? v : 1.0f;
      any_value |= (r == 2);
      if (static_cast<uint64_t>(idx) > max_index) max_index = idx;
    } else {
      IndexType fid = 0, idx = 0;
      float v = 0.0f;
      const int r = data::ParseTriple<IndexType, IndexType, float>(tp, tp + len, &fid, &idx, &v, &bad);
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

// ------------------------------------------------------------------ K2
template <TextFormat F>
__global__ __launch_bounds__(kThreads) void k_text_count(const uint8_t* __restrict__ text, size_t n,
                                                         const uint32_t* __restrict__ line_starts,
                                                         size_t nlines, TextParseConfig cfg,
                                                         uint64_t* __restrict__ line_info,
                                                         ChunkMeta* __restrict__ meta) {
  __shared__ uint4 lds[kWavesPerBlock][kWindow / 16];
  const int wid = threadIdx.x / dev::kWave;
  const int lane = dev::lane_id();
  uint8_t* win = reinterpret_cast<uint8_t*>(lds[wid]);
  const size_t nwaves = static_cast<size_t>(gridDim.x) * kWavesPerBlock;
  for (size_t line = static_cast<size_t>(blockIdx.x) * kWavesPerBlock + wid; line < nlines;
       line += nwaves) {
    const uint32_t b = line_starts[line];
    const uint32_t e = line + 1 < nlines ? line_starts[line + 1] : static_cast<uint32_t>(n);
    LineVisitor<F, uint32_t> vis;
    vis.label_col = cfg.label_column;
    vis.weight_col = cfg.weight_column;
    // count-only: classify returns 1 for feature tokens; sum them
    struct Counter {
      LineVisitor<F, uint32_t>* v;
      uint32_t nfeat{0};
      __device__ uint32_t classify(const char* tp, uint32_t len, uint32_t ord) {
        uint32_t s = v->classify(tp, len, ord);
        nfeat += s;
        return s;
      }
      __device__ void after_classify(uint32_t tb, uint32_t nt) { v->after_classify(tb, nt); }
      __device__ bool emit_enabled() const { return false; }
      __device__ bool selected(const char*, uint32_t, uint32_t) const { return false; }
      __device__ void emit(const char*, uint32_t, uint32_t, uint32_t) {}
    } counter{&vis};
    walk_line<F, false>(text, b, e, win, cfg.delimiter, counter);
    const uint32_t nfeat = dev::wave_sum(counter.nfeat);
    const bool row_ok = vis.row_state == 1;
    const bool w = __ballot(vis.has_weight) != 0;
    const bool qd = __ballot(vis.is_qid_lane) != 0;
    if (lane == 0) {
      line_info[line] = row_ok ? ((1ull << 32) | nfeat) : 0ull;
      if (row_ok && w) atomicOr(&meta->flags, kFlagWeight);
      if (row_ok && qd) atomicOr(&meta->flags, kFlagQid);
    }
  }
}

// ------------------------------------------------------------------ K4
template <TextFormat F, typename IndexType>
__global__ __launch_bounds__(kThreads) void k_text_fill(const uint8_t* __restrict__ text, size_t n,
                                                        const uint32_t* __restrict__ line_starts,
                                                        size_t nlines, TextParseConfig cfg,
                                                        const uint64_t* __restrict__ line_info,
                                                        FillTarget<IndexType> out,
                                                        ChunkMeta* __restrict__ meta) {
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
  // K8: one atomic per wave
  const uint64_t mi = dev::wave_max(wmax_index);
  const uint64_t mf = dev::wave_max(wmax_field);
  const bool av = __ballot(wany_value) != 0;
  const bool ng = __ballot(wneg) != 0;
  const bool ov = __ballot(woverflow) != 0;
  if (lane == 0) {
    if (mi != 0) atomicMax(&meta->max_index, static_cast<unsigned long long>(mi));
    if (mf != 0) atomicMax(&meta->max_field, static_cast<unsigned long long>(mf));
    unsigned fl = 0;
    if (av) fl |= kFlagValue;
    if (ng) fl |= kFlagNegIndex;
    if (ov) fl |= kFlagOverflow;
    if (F == TextFormat::kLibFM) fl |= kFlagField;
    if (fl != 0) atomicOr(&meta->flags, fl);
  }
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
                     const TextParseConfig& cfg, uint64_t* line_info, ChunkMeta* meta,
                     hipStream_t stream) {
  if (nlines == 0) return;
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  const dim3 grid(LineGrid(nlines)), block(kThreads);
  switch (cfg.format) {
    case TextFormat::kLibSVM:
      hipLaunchKernelGGL(k_text_count<TextFormat::kLibSVM>, grid, block, 0, stream, t, nbytes,
                         line_starts, nlines, cfg, line_info, meta);
      break;
    case TextFormat::kLibFM:
      hipLaunchKernelGGL(k_text_count<TextFormat::kLibFM>, grid, block, 0, stream, t, nbytes,
                         line_starts, nlines, cfg, line_info, meta);
      break;
    case TextFormat::kCSV:
      hipLaunchKernelGGL(k_text_count<TextFormat::kCSV>, grid, block, 0, stream, t, nbytes,
                         line_starts, nlines, cfg, line_info, meta);
      break;
  }
}

template <typename IndexType>
void LaunchTextFill(const char* text, size_t nbytes, const uint32_t* line_starts, size_t nlines,
                    const TextParseConfig& cfg, const uint64_t* line_info,
                    const FillTarget<IndexType>& out, uint64_t nrows, uint64_t nnz,
                    ChunkMeta* meta, hipStream_t stream) {
  if (nlines != 0) {
    const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
    const dim3 grid(LineGrid(nlines)), block(kThreads);
    switch (cfg.format) {
      case TextFormat::kLibSVM:
        hipLaunchKernelGGL((k_text_fill<TextFormat::kLibSVM, IndexType>), grid, block, 0, stream,
                           t, nbytes, line_starts, nlines, cfg, line_info, out, meta);
        break;
      case TextFormat::kLibFM:
        hipLaunchKernelGGL((k_text_fill<TextFormat::kLibFM, IndexType>), grid, block, 0, stream,
                           t, nbytes, line_starts, nlines, cfg, line_info, out, meta);
        break;
      case TextFormat::kCSV:
        hipLaunchKernelGGL((k_text_fill<TextFormat::kCSV, IndexType>), grid, block, 0, stream, t,
                           nbytes, line_starts, nlines, cfg, line_info, out, meta);
        break;
    }
  }
  hipLaunchKernelGGL(k_close_offsets, dim3(1), dim3(1), 0, stream, out.offset,
                     out.row_base + nrows, out.nnz_base + nnz);
}

template void LaunchTextFill<uint32_t>(const char*, size_t, const uint32_t*, size_t,
                                       const TextParseConfig&, const uint64_t*,
                                       const FillTarget<uint32_t>&, uint64_t, uint64_t,
                                       ChunkMeta*, hipStream_t);
template void LaunchTextFill<uint64_t>(const char*, size_t, const uint32_t*, size_t,
                                       const TextParseConfig&, const uint64_t*,
                                       const FillTarget<uint64_t>&, uint64_t, uint64_t,
                                       ChunkMeta*, hipStream_t);

}  // namespace gpu
}  // namespace dmlc
