/*!
 * \file dmlc/gpu/device_parser.h
 * \brief GPU ingestion: text shard -> pinned ring -> HBM -> CSR, on MI355X.
 *
 * Pipeline:
 *
 *   reader thread ── parallel pread ──> pinned slot ring (P slots, ThreadedIter)
 *        │                                     │ hipMemcpyAsync (copy stream)
 *        ▼                                     ▼
 *   InputSplit partition            device text ring (D slots, hipEvents)
 *                                              │ K1 line index, K2 count, K3 scan,
 *                                              │ K4 fill + K8 max (compute stream)
 *                                              ▼
 *                                   DeviceRowBlock / DeviceCSR in HBM
 *
 * The reference equivalent is Parser<I>::Create + ThreadedParser +
 * ThreadedInputSplit (`src/data.cc:21-34`, `src/data/parser.h:71-126`,
 * `src/io/threaded_input_split.h`), with OpenMP parsing replaced by the HIP
 * kernels and the prefetch queues replaced by the pinned/device rings.
 */
#ifndef DMLC_GPU_DEVICE_PARSER_H_
#define DMLC_GPU_DEVICE_PARSER_H_

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "./device_row_block.h"

namespace dmlc {
namespace gpu {

/*! \brief knobs of the GPU ingestion pipeline (also settable as `?k=v` URI args) */
struct DeviceParserConfig {
  /*! \brief libsvm | libfm | csv */
  std::string format{"libsvm"};
  /*! \brief bytes per pinned / device text slot */
  size_t chunk_bytes{64UL << 20};
  /*! \brief pinned host slots queued ahead of the GPU */
  int pinned_slots{3};
  /*! \brief device text slots (H2D of chunk k+1 overlaps parsing of chunk k) */
  int device_slots{3};
  /*! \brief parallel pread threads of the reader */
  int read_threads{8};
  /*! \brief HIP device (-1 = current) */
  int device{-1};
  /*! \brief CSV: label column (-1 none), weight column, delimiter */
  int label_column{-1};
  int weight_column{-1};
  char delimiter{','};
  /*! \brief LibSVM/LibFM: token-parallel kernels with exact per-line fallback */
  bool fast_path{true};
  /*!
   * \brief ParseAll over HBM-resident text: one launch per chunk (the fill
   *  counts its own tile and takes its prefix by decoupled look-back) instead
   *  of count + scan + fill with the next chunk's count prelaunched beside the
   *  current fill (`?one_pass=1`).  Off by default: measured slower, the fill
   *  waves serialise count -> look-back -> decode where the separate count
   *  kernel is hidden behind the previous fill (profiles/r05_one_pass).
   */
  bool one_pass{false};
  /*!
   * \brief ParseAllHashed into a reused batch over HBM-resident text: one
   *  k_tile_hash launch per merged chunk with look-back line counts
   *  (`?hash_one_pass=1`) instead of C1 + C2 + the counted k_tile_hash with
   *  the next chunk's count beside it.  Off by default: the look-back kernel
   *  measured 6,011 VALU per tile against 1,042 + 4,185 counted, 2.17 vs
   *  1.98 ms per 2 M x 1024 pass (profiles/r06_fill/hash_counted)
   */
  bool hash_one_pass{false};
  /*! \brief counted HBM replay: queue the next chunk's count + scan on a
   *  second stream beside the current fill (`?prelaunch=0`: in line, for
   *  pricing each kernel alone) */
  bool prelaunch{true};
  /*!
   * \brief zero-copy ingest: mmap the partition and hipHostRegister it so the
   *  DMA engines read the page cache directly (-1 auto with fallback to the
   *  pinned pread ring, 0 off, 1 required)
   */
  int zero_copy{-1};
  /*!
   * \brief zero-copy pinning: partitions up to zc_pin_budget bytes are
   *  registered whole, larger ones in sliding windows of zc_window_bytes (at
   *  most two pinned, the next prepared in the background)
   *  (`?zc_pin_budget_mb=`, `?zc_window_mb=`)
   */
  size_t zc_pin_budget{64UL << 30};
  size_t zc_window_bytes{1UL << 30};
  /*!
   * \brief HBM epoch cache: the first full pass also keeps every
   *  chunk's text resident in one device arena (partition bytes of HBM); later
   *  epochs (BeforeFirst, or Seek to a chunk boundary) parse straight from HBM
   *  with no host I/O and no PCIe traffic.
   */
  bool hbm_cache{false};
  /*!
   * \brief ParseAll over the HBM cache parses adjacent cached chunks together,
   *  up to this many bytes per kernel pass (`?replay_chunk_mb=`).  Default
   *  2 GiB - 64 MiB, the most the 32-bit chunk offsets allow: fewer host
   *  turnarounds per epoch, measured 1155 -> 1192 GB/s LibSVM and 1055 ->
   *  1081 LibFM against 1 GiB (profiles/r06_fill/replay_chunk)
   */
  size_t replay_chunk_bytes{(2UL << 30) - (64UL << 20)};
  /*! \brief the first merged chunk of a replay pass (`?replay_first_mb=`); each
   *  next one doubles up to replay_chunk_bytes.  0 (default, measured best
   *  since the count pass is cheap: 988 vs 969 GB/s at 64 MiB, profiles/r04_final):
   *  every merged chunk takes replay_chunk_bytes (no ramp) */
  size_t replay_first_bytes{0};
  /*!
   * \brief busy-poll budget (us) of a chunk-metadata wait before the host
   *  thread falls back to 20 us sleeps (src/gpu/host_wait.h)
   */
  double wait_spin_us{50};
  /*!
   * \brief coarse shuffling, the GPU twin of InputSplitShuffle (reference
   *  include/dmlc/input_split_shuffle.h): the shard is cut into shuffle_parts
   *  sub-shards (partition part * K + i of nparts * K) visited each epoch in
   *  the order of std::mt19937(666 + part + nparts + K + seed), reshuffled by
   *  every BeforeFirst.  One pipeline serves all sub-shards (its reader is
   *  re-targeted, never rebuilt); with hbm_cache every sub-shard's chunks are
   *  replayed from HBM in each epoch's order.  1 = off.
   *  (`?shuffle_parts=`, `?shuffle_seed=`)
   */
  unsigned shuffle_parts{1};
  int shuffle_seed{0};
  /*! \brief apply `?k=v` overrides (chunk_mb, pinned_slots, device_slots,
   *  read_threads, device, format, label_column, weight_column, delimiter,
   *  fast_path, one_pass, prelaunch, zero_copy, zc_pin_budget_mb, zc_window_mb, hbm_cache, replay_chunk_mb,
   *  replay_first_mb,
   *  shuffle_parts, shuffle_seed) */
  void Update(const std::map<std::string, std::string>& args);
};

/*!
 * \brief a hashed dense batch in HBM (BASELINE config 5): row r of `x` is the
 *  signed feature hash of line r into `dim` buckets, OCP fp8 e4m3 (1 byte) or
 *  f32, `label` its label.  Grows by doubling, like DeviceCSR.  The buffers
 *  are shared: a consumer that exported them (DLPack) keeps its own
 *  reference, so a Reserve that moves the batch to bigger buffers never frees
 *  memory a tensor still points at.
 */
struct DeviceHashedBatch {
  std::shared_ptr<DeviceBuffer> x{std::make_shared<DeviceBuffer>()};
  std::shared_ptr<DeviceBuffer> label{std::make_shared<DeviceBuffer>()};
  size_t rows{0}, row_cap{0};
  int dim{0};
  bool fp8{true};
  int device{0};
  /*! \brief capacity for `rows` rows, preserving the first this->rows */
  void Reserve(size_t rows, hipStream_t stream);
};

/*! \brief cumulative pipeline counters */
struct DeviceParserStats {
  size_t bytes{0};
  size_t chunks{0};
  size_t rows{0};
  size_t nnz{0};
  /*! \brief chunks the fast path handed to the exact per-line kernels */
  size_t exact_chunks{0};
  /*! \brief chunks built in one pass (look-back, no count kernel): hashed
   *  batches, and resident CSR chunks */
  size_t one_pass_chunks{0};
  /*! \brief one-pass CSR chunks written again (target grown / weight column added) */
  size_t one_pass_reruns{0};
  /*! \brief seconds the host waited for the reader (pinned ring empty) */
  double wait_reader_sec{0};
  /*! \brief seconds the host waited for GPU results */
  double wait_gpu_sec{0};
  /*! \brief zero-copy mode active, and the one-time mmap + register cost */
  bool zero_copy{false};
  double register_sec{0};
  /*! \brief zero-copy: this process's pin budget (the configured one shared
   *  among the host's ranks, bounded by MemAvailable) and the most bytes it
   *  has had registered at once */
  size_t zc_pin_budget{0}, zc_pinned_peak{0};
  /*! \brief the last ParseAll: its wall time, pipeline fill (start until the
   *  first chunk is parsed) and drain (the reader's last chunk handed in
   *  until the pass is done), host clock */
  double last_pass_sec{0}, last_fill_sec{0}, last_drain_sec{0};
  /*! \brief metadata waits that ended spinning / sleeping / at the bound */
  size_t waits_spun{0}, waits_slept{0}, waits_timed_out{0};
};

/*!
 * \brief GPU parser for one partition of a text dataset.
 *
 *  Streaming:   while (p->Next()) use(p->Value());   // one block per chunk
 *  Resident:    DeviceCSR<uint32_t> csr; p->ParseAll(&csr);  // whole shard in HBM
 */
template <typename IndexType>
class DeviceParser {
 public:
  /*!
   * \param uri data uri (`?k=v` args override cfg)
   * \param part_index / num_parts sharding as in InputSplit::Create
   */
  static DeviceParser* Create(const std::string& uri, unsigned part_index, unsigned num_parts,
                              const DeviceParserConfig& cfg = DeviceParserConfig());
  virtual ~DeviceParser() = default;
  /*! \brief rewind to the first chunk */
  virtual void BeforeFirst() = 0;
  /*!
   * \brief mid-epoch resume cursor: partition byte offset of the first record
   *  not yet delivered by Next() / ParseAll().  Serialise it with
   *  the model checkpoint; a new parser over the same (uri, part, nparts)
   *  continues from it with Seek().  Zero-copy and pinned-ring modes share
   *  the cursor space.
   */
  virtual size_t Tell() const = 0;
  /*! \brief continue from a Tell() cursor (drains in-flight work first) */
  virtual void Seek(size_t cursor) = 0;
  /*!
   * \brief shuffled mode: epochs started so far (0 after construction, +1 per
   *  BeforeFirst) -- the visiting order is a function of it, so a resume
   *  restores it with SetEpoch before Seek
   */
  virtual unsigned Epoch() const { return 0; }
  /*! \brief shuffled mode: switch to epoch e's visiting order, rewound */
  virtual void SetEpoch(unsigned /*e*/) {}
  /*! \brief shuffled mode: the current epoch's sub-shard visiting order */
  virtual std::vector<unsigned> VisitOrder() const { return {0}; }
  /*! \brief parse the next chunk; the block is ready on return */
  virtual bool Next() = 0;
  /*! \brief block of the last Next() (valid until the next call) */
  virtual const DeviceRowBlock<IndexType>& Value() const = 0;
  /*! \brief parse the rest of the partition, appending to `out` */
  virtual void ParseAll(DeviceCSR<IndexType>* out) = 0;
  /*!
   * \brief parse the rest of the partition straight into a hashed dense batch
   *  (tokenize -> hash -> fp8 in one kernel per chunk, no CSR materialised);
   *  the hash is the one of ops.hashed_dense / LaunchHashedDense*
   */
  virtual void ParseAllHashed(DeviceHashedBatch* out, int dim, float scale, uint32_t seed,
                              bool fp8) = 0;
  /*! \brief total bytes of this partition */
  virtual size_t PartitionBytes() const = 0;
  virtual const DeviceParserStats& Stats() const = 0;
  /*! \brief stream on which blocks are produced */
  virtual hipStream_t stream() const = 0;
};

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_GPU_DEVICE_PARSER_H_
