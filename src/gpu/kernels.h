/*!
 * \file src/gpu/kernels.h
 * \brief Host-callable launchers of the CDNA4 (gfx950) ingestion kernels.
 *
 * Kernel inventory:
 *   K1 line index        LaunchLineIndex          (text_kernels.hip)
 *   K2 per-line count    LaunchTextCount          (text_kernels.hip)
 *   K3 offsets scan      LaunchScanU64            (scan_kernels.hip)
 *   K4 per-line fill     LaunchTextFill           (text_kernels.hip)
 *   K5 CSV / K6 LibFM    same launchers, TextFormat::kCSV / kLibFM
 *   K7 recordio decode   LaunchRecordIOTileCount / LaunchRecordIOTileFill, LaunchRecordIOGather
 *                        (recordio_kernels.hip)
 *   K8 max reduce        fused into K4 (wave max + one atomicMax per wave)
 *   K9 fp8 pack / hash   LaunchHashedDenseFP8     (feature_kernels.hip)
 *   K10 csr concat       LaunchCSRAppend          (feature_kernels.hip)
 *   K11 spmv / sdot      LaunchCSRSpMV, LaunchCSRSpMVT (feature_kernels.hip)
 * All launchers are asynchronous on `stream` and never allocate or
 * synchronise (graph-capture safe, cdna_hip_programming.md Guideline 9).
 */
#ifndef DMLC_GPU_KERNELS_H_
#define DMLC_GPU_KERNELS_H_

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace dmlc {
namespace gpu {

/*! \brief padding (bytes) every device text buffer must have past its end */
constexpr size_t kTextPadBytes = 4096;
/*! \brief bytes per workgroup tile of the line-index kernels (256 lanes x 16 B) */
constexpr size_t kLineTileBytes = 4096;

enum class TextFormat : int { kLibSVM = 0, kLibFM = 1, kCSV = 2 };

/*! \brief per-format knobs passed by value to the kernels */
struct TextParseConfig {
  TextFormat format{TextFormat::kLibSVM};
  int label_column{-1};   // CSV
  int weight_column{-1};  // CSV
  char delimiter{','};    // CSV
};

/*! \brief per-chunk results written by the device */
struct ChunkMeta {
  unsigned long long nlines;     // candidate lines (K1)
  unsigned long long nrows;      // valid rows (K3 total >> 32)
  unsigned long long nnz;        // entries (K3 total & 0xffffffff)
  unsigned long long max_index;  // K8
  unsigned long long max_field;  // K8 (LibFM)
  unsigned int flags;            // kFlag* bits
  unsigned int pad;
};
constexpr unsigned kFlagWeight = 1u;
constexpr unsigned kFlagQid = 2u;
constexpr unsigned kFlagValue = 4u;
constexpr unsigned kFlagField = 8u;
constexpr unsigned kFlagNegIndex = 256u;
constexpr unsigned kFlagOverflow = 512u;

/*!
 * \brief per-workgroup reduction slot.  Kernels never hit one global word from
 *  every wave (same-address atomics serialise at the memory side, ~10 ns each:
 *  62k waves x 3 atomics cost 1.5 ms per chunk); each workgroup reduces in
 *  LDS and writes its slot, then k_reduce_partials folds the slots into the
 *  ChunkMeta with one workgroup.
 */
struct MetaPartial {
  unsigned long long max_index;
  unsigned long long max_field;
  unsigned int flags;
  unsigned int pad;
};
/*! \brief max workgroups of any kernel that writes MetaPartial slots */
constexpr int kMaxPartialBlocks = 8192;
/*! \brief fold nblocks MetaPartial slots into meta (max / or) with one workgroup */
void LaunchReducePartials(const MetaPartial* partials, int nblocks, ChunkMeta* meta,
                          hipStream_t stream);

/*! \brief destination arrays of the fill pass (device pointers) */
template <typename IndexType>
struct FillTarget {
  uint64_t* offset;  // row pointer (global)
  float* label;
  float* weight;
  uint64_t* qid;
  IndexType* field;  // may be null unless LibFM
  IndexType* index;
  float* value;
  uint64_t row_base;   // first row written by this chunk
  uint64_t nnz_base;   // first entry written by this chunk
  uint64_t row_limit;  // rows [row_base, row_limit) may be written
  uint64_t nnz_limit;  // entries [nnz_base, nnz_limit) may be written
};

/*! \brief scratch sizes for a chunk of `nbytes` */
size_t LineIndexTiles(size_t nbytes);
size_t ScanPartials(size_t n);

/*!
 * \brief K1a: count line starts per 4 KiB tile and scan the tile counts.
 * \param tile_scratch >= LineIndexTiles(nbytes) u64
 * \param meta meta->nlines receives the number of lines
 */
void LaunchLineCount(const char* text, size_t nbytes, uint64_t* tile_scratch, ChunkMeta* meta,
                     hipStream_t stream);
/*!
 * \brief K1b: write the line start offsets (needs LaunchLineCount's scanned
 *  tile_scratch); line_starts needs meta->nlines entries.
 */
void LaunchLineEmit(const char* text, size_t nbytes, const uint64_t* tile_scratch,
                    uint32_t* line_starts, hipStream_t stream);

/*!
 * \brief K2: per-line (row_valid << 32 | nnz) into line_info[nlines]; sets
 *  weight/qid flags in meta.
 */
void LaunchTextCount(const char* text, size_t nbytes, const uint32_t* line_starts,
                     size_t nlines, const TextParseConfig& cfg, uint64_t* line_info,
                     MetaPartial* partials, ChunkMeta* meta, hipStream_t stream);

/*!
 * \brief K3: exclusive scan of n u64 values in place; *total receives the sum.
 * \param partials >= ScanPartials(n) + 1 u64
 */
void LaunchScanU64(uint64_t* data, size_t n, uint64_t* partials, uint64_t* total,
                   hipStream_t stream);

/*! \brief split the scan total into meta->nrows / meta->nnz */
void LaunchMetaFromTotal(const uint64_t* total, ChunkMeta* meta, hipStream_t stream);

/*!
 * \brief K4 (+K5/K6/K8): parse every line into the CSR target. line_info must
 *  hold the exclusive scan produced by K3.  Also writes the closing offset.
 */
template <typename IndexType>
void LaunchTextFill(const char* text, size_t nbytes, const uint32_t* line_starts,
                    size_t nlines, const TextParseConfig& cfg, const uint64_t* line_info,
                    const FillTarget<IndexType>& out, uint64_t nrows, uint64_t nnz,
                    MetaPartial* partials, ChunkMeta* meta, hipStream_t stream);

/*! \brief offset[row_end] = nnz_end (closing row pointer of a chunk) */
void LaunchCloseOffsets(uint64_t* offset, uint64_t row_end, uint64_t nnz_end, hipStream_t stream);

/*! \brief a chunk the tile parser cannot take (the exact per-line kernels re-parse it) */
constexpr unsigned kFlagIrregular = 1024u;

// --------------- LDS-staged tile parser (LibSVM/LibFM fast path) ---------------
/*! \brief bytes of text per workgroup of the tile kernels */
constexpr size_t kTileBytes = 8192;
/*! \brief a weighted row met a FillTarget without a weight column (re-run with one) */
constexpr unsigned kFlagNeedWeight = 2048u;
/*! \brief tiles of a chunk (size of the tile count / flag scratch and MetaPartial slots) */
size_t TileCount(size_t nbytes);
/*! \brief u64 tile_counts / u32 tile_flags entries to reserve for ntiles tiles (scan scratch) */
size_t TileScratchWords(size_t ntiles);
/*! \brief MetaPartial slots to reserve for ntiles tiles (finish-fold scratch) */
size_t TileScratchSlots(size_t ntiles);
/*!
 * \brief C1 + C2: per-tile (line starts << 32 | token starts) and irregular
 *  flags, exclusive-scanned in place; meta receives nlines, nrows = nlines,
 *  nnz = tokens - lines, flags (kFlagIrregular) and zeroed maxima; host_meta
 *  (mapped pinned memory, may be null) receives a copy the host reads after
 *  synchronising the stream, without a device-to-host copy.
 *  tile_counts / tile_flags need TileCount(nbytes) entries; tile_masks
 *  (TileMaskWords) receives the per-16-byte start masks the fill reads.
 */
void LaunchTileCountScan(const char* text, size_t nbytes, uint64_t* tile_counts,
                         uint32_t* tile_flags, uint32_t* tile_masks, ChunkMeta* meta,
                         ChunkMeta* host_meta, hipStream_t stream);
/*!
 * \brief u32 words of C1's published token / line start masks for ntiles
 *  tiles (one word per 16 text bytes: the fill and the fused hash kernel take
 *  them instead of classifying every byte a second time)
 */
size_t TileMaskWords(size_t ntiles);
/*!
 * \brief C3 + C4: parse every token of a regular chunk into out using the
 *  scanned tile prefixes; merges max index / field and flags into meta and
 *  writes offset[row_base + nrows].  partials needs TileCount(nbytes) slots.
 *  Sets kFlagNeedWeight if a row is weighted and out.weight is null.
 *
 *  One pass (one_pass != nullptr; tile_prefix unused, nbytes > 0): no C1 / C2
 *  -- each wave counts its tile's lines and entries itself (with C1's
 *  irregular checks) and takes the counts before it by decoupled look-back
 *  over one_pass->status (zeroed here, in the stream, before the launch).
 *  The chunk's nlines / nrows / nnz land in meta (and host_meta) with the
 *  flags.  out.row_limit / nnz_limit are the target's capacities: rows or
 *  entries past them are not written and set kFlagOverflow (grow the target
 *  to meta's sizes and run the chunk again; no closing row pointer is
 *  written).  kFlagQid: the chunk has `qid:` tokens, which only the counted
 *  path (LaunchTileCountScan first, qid column zeroed) writes -- run it so.
 *  Returns the workgroups launched: advance ticket0 by it.
 */
struct FillOnePass {
  uint64_t* status;            // >= TileCount(nbytes) words
  unsigned long long* ticket;  // counter, zeroed once
  unsigned long long ticket0;  // the counter's value before this launch
};
template <typename IndexType>
size_t LaunchTileFill(const char* text, size_t nbytes, TextFormat format,
                      const uint64_t* tile_prefix, const uint32_t* tile_masks,
                      const FillTarget<IndexType>& out, MetaPartial* partials, ChunkMeta* meta,
                      ChunkMeta* host_meta, hipStream_t stream,
                      const FillOnePass* one_pass = nullptr);

/*!
 * \brief fused tokenize -> hash -> dense rows on the tile parser (config 5):
 *  rows = the `nlines` lines of a regular chunk (tile_prefix from
 *  LaunchTileCountScan), row row_base + line of a [rows x dim] fp8 (x scale)
 *  or f32 batch, labels alongside; no CSR is written.  One wave per tile, the
 *  lines that start in it (followed past the tile end, any length).  Sets
 *  kFlagIrregular for tokens only the exact kernels parse (qid:, junk; re-run
 *  the chunk with LaunchTextHashed), merges kFlagNegIndex.  dim: multiple of
 *  16, <= 4096.
 */
/*!
 *  One pass (one_pass != nullptr; tile_prefix / nlines unused): no C1 / C2 --
 *  each wave counts its tile's lines itself and takes the lines before it by
 *  decoupled look-back; the chunk's nlines / nrows land in meta (and
 *  host_meta) with the flags.  Rows at or past row_cap are not written and set
 *  kFlagOverflow (grow the batch to meta->nrows and run the chunk again).
 *  nbytes > 0 (an empty chunk has no tile to write the sizes).
 *  Also sets kFlagIrregular for what C1 would have (blank-started lines,
 *  control bytes other than \t \n \r).  Returns the workgroups launched:
 *  advance ticket0 by it for the next launch on the same counter.
 */
struct HashOnePass {
  uint64_t* status;            // >= TileCount(nbytes) words, zeroed once at allocation
  unsigned long long* ticket;  // counter, zeroed once
  unsigned long long ticket0;  // the counter's value before this launch
  uint32_t tag;                // distinct per launch on the same status array, 1..2^30-1
  uint64_t row_cap;            // rows of out / labels
};
template <typename IndexType>
size_t LaunchTileHashed(const char* text, size_t nbytes, TextFormat format,
                        const uint64_t* tile_prefix, const uint32_t* tile_masks,
                        uint64_t row_base, uint64_t nlines, int dim,
                        float scale, uint32_t seed, bool fp8, void* out, float* labels,
                        MetaPartial* partials, ChunkMeta* meta, ChunkMeta* host_meta,
                        hipStream_t stream, const HashOnePass* one_pass = nullptr);

/*!
 * \brief C2 alone over caller-filled per-tile u64 counts (hi 32 bits: items,
 *  lo 32 bits: bytes): exclusive scan in place, meta->nrows = items,
 *  meta->nnz = bytes, OR of tile_flags into meta->flags, published to
 *  host_meta.  Scratch sizes as for LaunchTileCountScan (TileScratchWords).
 */
void LaunchTileScanRaw(uint64_t* tile_counts, uint32_t* tile_flags, size_t ntiles,
                       ChunkMeta* meta, ChunkMeta* host_meta, hipStream_t stream);
/*!
 * \brief C4 alone: fold nslots MetaPartial slots into meta (max / or), write
 *  offset[row_base + meta->nrows] = nnz_base + meta->nnz (offset may be null)
 *  and publish meta to host_meta.  partials needs TileScratchSlots(nslots).
 */
void LaunchTileFinish(MetaPartial* partials, size_t nslots, ChunkMeta* meta, ChunkMeta* host_meta,
                      uint64_t* offset, uint64_t row_base, uint64_t nnz_base, hipStream_t stream);

// ------------------------- CSV on the tile pipeline -------------------------
/*!
 * \brief S1: per 8 KiB tile (rows starting in it << 32 | their entries) and
 *  kFlagIrregular (a row running > 4 KiB past its tile, control bytes); scan
 *  them with LaunchTileScanRaw.  tile_counts / tile_flags: TileScratchWords.
 *  With label / weight columns of at most 0 the counts are positional (S1p:
 *  row starts and entries whose first byte is in the tile, no flags) and the
 *  fill flags irregular chunks; LaunchCsvTileFill takes the same columns, so
 *  both pick the same mode.  The positional count also publishes every 16
 *  bytes' line-end / delimiter masks into tile_masks (TileMaskWords) and
 *  flags control bytes; the fill then reads the masks instead of classifying.
 */
void LaunchCsvTileCount(const char* text, size_t nbytes, int label_column, int weight_column,
                        char delimiter, uint64_t* tile_counts, uint32_t* tile_flags,
                        uint32_t* tile_masks, hipStream_t stream);
/*!
 * \brief S2: every row of a regular chunk into out (index / value / label /
 *  weight / offset) from the scanned S1 prefixes; one MetaPartial per tile
 *  (max index, kFlagValue / kFlagWeight), folded by LaunchTileFinish.
 */
template <typename IndexType>
void LaunchCsvTileFill(const char* text, size_t nbytes, int label_column, int weight_column,
                       char delimiter, const uint64_t* tile_prefix, const uint32_t* tile_masks,
                       const FillTarget<IndexType>& out, MetaPartial* partials,
                       hipStream_t stream);

// ----------------------------- RecordIO (K7) -----------------------------
/*! \brief error bits reported by the RecordIO kernels */
constexpr uint32_t kRecErrTruncated = 1;   // a part runs past the chunk end
constexpr uint32_t kRecErrBadPart = 2;     // continuation part without its head
/*! \brief 2048-word tiles of a chunk of `nwords` words (scan scratch: TileScratchWords) */
size_t RecordIOTiles(size_t nwords);
/*!
 * \brief R1: per tile (record heads << 32 | output bytes) and error bits
 *  (kRecErr*); scan them with LaunchTileScanRaw.  The chunk must start at a
 *  record head and be < 4 GiB.
 */
void LaunchRecordIOTileCount(const uint32_t* words, size_t nwords, uint64_t* tile_counts,
                             uint32_t* tile_flags, hipStream_t stream);
/*!
 * \brief R2: decode every record of the chunk: record r (chunk-relative) gets
 *  offset[rec_base + r] = byte_base + its output position and its payload
 *  (multi-part records reassembled, escaped magic words re-inserted) at
 *  data + that position.  tile_prefix: the scanned R1 counts; partials: one
 *  MetaPartial per tile (error bits), folded by LaunchTileFinish, which also
 *  writes the closing offset.
 */
/*!
 *  One pass (one_pass != nullptr; tile_prefix unused, nwords > 0): R1 runs
 *  inside the fill (decoupled look-back over one_pass->status, zeroed here
 *  before the launch); the chunk's records / bytes land in one_pass->meta
 *  (nrows / nnz), for LaunchTileFinish.  Records at or past rec_cap (offset
 *  slots; the closing one needs one more) and bytes past byte_cap are not
 *  written and set kFlagOverflow: grow to rec_base + nrows / byte_base + nnz
 *  and run the chunk again.  Returns the workgroups launched (advance
 *  ticket0 by it).
 */
struct RecordIOOnePass {
  uint64_t* status;            // >= RecordIOTiles(nwords) words
  unsigned long long* ticket;  // counter, zeroed once
  unsigned long long ticket0;  // the counter's value before this launch
  ChunkMeta* meta;
  uint64_t rec_cap;            // offset slots - 1
  uint64_t byte_cap;           // data bytes
};
/*!
 * \brief counted fill's guards: writes past (rec_cap offset slots, byte_cap
 *  data bytes) are dropped, and each tile checks that its parts end at the
 *  next tile's prefix (the last one: meta's totals); either miss is
 *  kRecErrBadPart (a count that disagrees with the fill's header view)
 */
struct RecordIOCaps {
  ChunkMeta* meta;
  uint64_t rec_cap;
  uint64_t byte_cap;
};
size_t LaunchRecordIOTileFill(const uint32_t* words, size_t nwords, const uint64_t* tile_prefix,
                              uint64_t* offset, uint64_t rec_base, uint8_t* data,
                              uint64_t byte_base, MetaPartial* partials, hipStream_t stream,
                              const RecordIOOnePass* one_pass = nullptr,
                              const RecordIOCaps* caps = nullptr);
/*!
 * \brief R1c: LaunchRecordIOTileCount's per-tile counts by following part
 *  chains (one 8-byte read per part after each tile's first-header search):
 *  the same counts on a well-formed chunk for ~2 % of its reads at 512-byte
 *  records; latency-bound, for chunks of parts >= ~128 bytes
 */
void LaunchRecordIOTileCountChain(const uint32_t* words, size_t nwords, uint64_t* tile_counts,
                                  uint32_t* tile_flags, hipStream_t stream);
/*!
 * \brief R3: gather nrec whole records (src + src_off[k], len[k] bytes, 4-byte
 *  multiples) to dst + dst_off[k]
 */
void LaunchRecordIOGather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                          const uint64_t* dst_off, size_t nrec, uint8_t* dst, hipStream_t stream);

// --------------------------- features (K9-K11) ---------------------------
/*!
 * \brief K9: hashed dense batch in OCP fp8 e4m3: out[r, h(index) % dim] +=
 *  value * scale, accumulated in f32 in LDS and converted with gfx950
 *  v_cvt_pk_fp8_f32.  rows = nrows, dim <= 8192.
 */
template <typename IndexType>
void LaunchHashedDenseFP8(const uint64_t* offset, const IndexType* index, const float* value,
                          const IndexType* field, size_t nrows, int dim, float scale,
                          uint32_t seed, uint8_t* out, hipStream_t stream);
/*! \brief same but f32 output (reference for the fp8 path / bf16 consumers) */
template <typename IndexType>
void LaunchHashedDenseF32(const uint64_t* offset, const IndexType* index, const float* value,
                          const IndexType* field, size_t nrows, int dim, uint32_t seed,
                          float* out, hipStream_t stream);
/*!
 * \brief K9 fused with the text walk (BASELINE config 5): every valid line of a
 *  LibSVM / LibFM chunk becomes row row_base + (line_info >> 32) of a dense
 *  [rows x dim] batch -- OCP fp8 e4m3 (x scale) or f32 -- with features
 *  hashed exactly as LaunchHashedDense* does, plus its label; no CSR is
 *  written.  line_starts / line_info as for LaunchTextFill (K1, K2 + K3).
 *  dim: multiple of 4, <= 4096 (LDS row per wave).  Merges kFlagNegIndex.
 */
template <typename IndexType>
void LaunchTextHashed(const char* text, size_t nbytes, const uint32_t* line_starts, size_t nlines,
                      TextFormat format, const uint64_t* line_info, uint64_t row_base, int dim,
                      float scale, uint32_t seed, bool fp8, void* out, float* labels,
                      MetaPartial* partials, ChunkMeta* meta, hipStream_t stream);
/*! \brief K11: y[r] = sum_j value * w[index] (+ bias), 16 lanes per row; value ==
 *  (float*)index + 1 (u32 indices): interleaved (index, value) pairs */
template <typename IndexType>
void LaunchCSRSpMV(const uint64_t* offset, const IndexType* index, const float* value,
                   size_t nrows, const float* w, float bias, float* y, hipStream_t stream);
/*! \brief K11^T: g[index] += value * d[r] (f32 atomics) */
template <typename IndexType>
void LaunchCSRSpMVT(const uint64_t* offset, const IndexType* index, const float* value,
                    size_t nrows, const float* d, float* g, hipStream_t stream);
// ------------------------ HashedFM (fm_kernels.hip) ------------------------
/*! \brief factor rank of the HIP HashedFM kernels and the [w | V] column count */
constexpr int kFmRank = 16;
constexpr int kFmCols = kFmRank + 1;
/*! \brief dynamic LDS of LaunchFmForward for `dim` features */
size_t FmForwardSharedBytes(int dim);
/*!
 * \brief F1: y[r] = bias + sx x_r.w + 1/2 (|sx x_r V|^2 - sx^2 x_r^2.q) and
 *  xv[r] = sx x_r V for the fp8 e4m3 batch x [rows x dim]; wt_bf16 = [w | V]^T
 *  as bf16 [17 x dim], q[n] = sum_f V_nf^2.  dim: multiple of 128, <= 2048.
 */
void LaunchFmForward(const uint8_t* x, int64_t rows, int dim, const void* wt_bf16, const float* q,
                     const float* bias, float sx, float* y, float* xv, int num_cus,
                     hipStream_t stream);
/*!
 * \brief F2: per-block partials part[nblocks][18][dim] of Z = G^T x (G_r =
 *  [g_r, g_r xv_r], rows 0..16) and t = (x^2)^T g (row 17); the caller sums
 *  over blocks.  dim: multiple of 128.
 */
void LaunchFmBackward(const uint8_t* x, int64_t rows, int dim, const float* g, const float* xv,
                      int nblocks, float* part, hipStream_t stream);
/*! \brief [w | V]^T in bf16 ([kFmCols][dim]) and q = rowsum(V^2) for LaunchFmForward
 *  (w: [dim] f32, v: [dim][kFmRank] f32) */
void LaunchFmPrep(const float* w, const float* v, int dim, void* wt_bf16, float* q,
                  hipStream_t stream);
/*! \brief sum the LaunchFmBackward partials (z: [kFmCols + 1][dim] scratch)
 *  and write dw [dim] and dV [dim][kFmRank] (v: [dim][kFmRank] f32) */
void LaunchFmReduceGrads(const float* part, int nblocks, int dim, const float* v, float sx,
                         float* z, float* gw, float* gv, hipStream_t stream);
/*! \brief losses of the fused HashedFM step */
enum FmLoss : int { kFmLogistic = 0, kFmSquared = 1 };
/*! \brief largest dim of LaunchFmFused (one wave per 128 features, 8 waves) */
constexpr int kFmFusedMaxDim = 1024;
/*!
 * \brief F5: forward, loss and backward of one HashedFM step in one pass over
 *  the fp8 batch.  Per 32-row tile: F1's products (split over the
 *  workgroup's waves by feature block, summed through LDS), y, the loss and
 *  g = dloss/dy for the tile's labels (mean over `rows`: g is scaled by
 *  inv_n), then F2's G^T X products from the same registers.  Writes y
 *  (optional), part[nblocks][18][dim] as LaunchFmBackward, and
 *  lpart[nblocks][2] = (sum of weighted losses, sum of g) per block.
 *  dim: multiple of 128, <= kFmFusedMaxDim.  weight may be null.
 */
void LaunchFmFused(const uint8_t* x, int64_t rows, int dim, const void* wt_bf16, const float* q,
                   const float* bias, float sx, const float* label, const float* weight,
                   int loss, float inv_n, int nblocks, float* y, float* part, float* lpart,
                   hipStream_t stream);

/*! \brief K10: dst_offset[i] = src_offset[i] - src_base + dst_base for i<=nrows */
void LaunchOffsetRebase(const uint64_t* src_offset, size_t nrows, uint64_t src_base,
                        uint64_t dst_base, uint64_t* dst_offset, hipStream_t stream);
/*!
 * \brief page-cache row pointers: offset[r + 1] (r < nrows) holds the
 *  page-local end of row r; add its page's nnz base.  page_row_end[p] =
 *  rows of pages 0..p (cumulative), page_nnz_base[p] = entries before page p.
 */
void LaunchPageRebase(uint64_t* offset, size_t nrows, const uint64_t* page_row_end,
                      const uint64_t* page_nnz_base, int npages, hipStream_t stream);
/*!
 * \brief CSR -> CSC (transpose_kernels.hip): rows [0, nrows) of a CSR whose
 *  entries are [base, base + nnz) of index / value; writes col_ptr
 *  [num_features + 1] (u64, from 0), row_out [nnz] (u32 row ids, ascending
 *  within each column) and val_out [nnz] (when value != null).  With
 *  val_out == (float*)row_out + 1 (row_out 8-byte aligned) the output is
 *  interleaved (row, value) pairs, one 8-byte store per entry.  Feature ids
 *  >= num_features are clamped and set *error (device u32) to 1.
 *  num_features <= CSRTransposeMaxFeatures(); scratch of
 *  CSRTransposeScratchBytes(nnz, num_features) bytes (256-byte aligned).
 */
template <typename IndexType>
void LaunchCSRTranspose(const uint64_t* offset, size_t nrows, uint64_t base, uint64_t nnz,
                        const IndexType* index, const float* value, uint64_t num_features,
                        uint64_t* col_ptr, uint32_t* row_out, float* val_out, void* scratch,
                        uint32_t* error, hipStream_t stream);
size_t CSRTransposeScratchBytes(uint64_t nnz, uint64_t num_features);
uint64_t CSRTransposeMaxFeatures();
/*! \brief fill n floats with v */
void LaunchFill(float* p, size_t n, float v, hipStream_t stream);

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_GPU_KERNELS_H_
