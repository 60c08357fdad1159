/*!
 * \file dmlc/gpu/device_recordio.h
 * \brief GPU RecordIO reader: record-aligned chunks -> HBM -> K7 decode ->
 *  packed payloads + offsets in device memory.
 *
 * Reference equivalent: InputSplit::Create(uri, part, nparts, "recordio") +
 * RecordIOSplitter::NextRecord / RecordIOChunkReader (`src/io.cc:113-116`,
 * `src/io/recordio_split.cc:44-82`, `src/recordio.cc:85-156`).  The record
 * walk moves to the K7 kernels (src/gpu/recordio_kernels.hip); the host only
 * cuts chunks at record heads (zero-copy mmap + hipHostRegister, or the
 * InputSplit chunk path through a pinned staging slot).
 *
 * A batch is a byte-CSR: record i is data[offset[i], offset[i+1]) -- the same
 * layout as a RowBlock's offset array, ready for a decode kernel or DLPack.
 */
#ifndef DMLC_GPU_DEVICE_RECORDIO_H_
#define DMLC_GPU_DEVICE_RECORDIO_H_

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>

namespace dmlc {
namespace gpu {

struct DeviceRecordIOConfig {
  /*! \brief bytes per chunk / batch (< 4 GiB; a record longer than this gets a chunk of its own) */
  size_t chunk_bytes{64UL << 20};
  /*! \brief HIP device (-1 = current) */
  int device{-1};
  /*! \brief -1 auto (mmap + hipHostRegister, fall back to pinned staging), 0 off, 1 required */
  int zero_copy{-1};
  /*! \brief chunks in flight on the device (H2D of later chunks overlaps the decode) */
  int device_slots{3};
  /*! \brief pinned host slots of the reader thread (staging path) */
  int pinned_slots{3};
  /*!
   * \brief keep the partition's bytes resident in HBM after the first epoch
   *  and decode later epochs from there (adjacent chunks merged up to
   *  replay_chunk_bytes: 2 GiB, so a resident epoch of ~2 GB pays one scan /
   *  finish / host turnaround; < 4 GiB for the 32-bit in-chunk byte offsets)
   */
  bool hbm_cache{false};
  size_t replay_chunk_bytes{2UL << 30};
  /*!
   * \brief ReadAll over the HBM cache decodes each merged chunk in ONE launch
   *  (R1 inside the fill, decoupled look-back; the text is read once) instead
   *  of count + scan + fill with the next chunk's count prelaunched beside
   *  the current fill (`?one_pass=1`).  Off by default: the look-back costs
   *  the fill waves 338 us per GiB, the prelaunched count hides behind the
   *  fill (profiles/r05_recordio)
   */
  bool one_pass{false};
  /*!
   * \brief R1c, the chain count (headers only, one read per part) instead of
   *  R1 (every word): -1 auto (once decoded chunks show >= 128 and <= 4096
   *  bytes per record on average), 0 never, 1 always (`?chain_count=`)
   */
  int chain_count{-1};
  /*!
   * \brief indexed RecordIO (reference "indexed_recordio" InputSplit): the
   *  index file ("key offset" lines); shards by record count; with shuffle,
   *  every epoch visits the shard's records in the std::mt19937(111 + seed)
   *  order of the CPU IndexedRecordIOSplitter.  The shard is read into HBM
   *  once and each batch is gathered on the device (LaunchRecordIOGather).
   */
  std::string index_uri;
  bool shuffle{false};
  int seed{0};
  /*! \brief busy-poll budget (us) of a metadata wait before sleeping (src/gpu/host_wait.h) */
  double wait_spin_us{50};
  /*!
   * \brief apply `?k=v` overrides: chunk_mb, chunk_bytes, device, zero_copy,
   *  device_slots, pinned_slots, hbm_cache, replay_chunk_mb, one_pass,
   *  chain_count, index, shuffle, seed, wait_spin_us
   */
  void Update(const std::map<std::string, std::string>& args);
};

/*! \brief records in device memory: record i = data[offset[i], offset[i+1]) */
struct DeviceRecordBatch {
  size_t size{0};
  size_t bytes{0};
  const uint64_t* offset{nullptr};
  const uint8_t* data{nullptr};
};

struct DeviceRecordIOStats {
  /*! \brief input bytes decoded (records with their headers) */
  size_t bytes{0};
  size_t chunks{0};
  size_t records{0};
  bool zero_copy{false};
  /*! \brief host seconds waiting for the reader thread / for device results */
  double wait_reader_sec{0};
  double wait_gpu_sec{0};
  /*! \brief chunks decoded from the HBM-resident copy (hbm_cache / indexed) */
  size_t replayed_chunks{0};
  /*! \brief of those, chunks decoded in one launch (look-back, no count kernel) */
  size_t one_pass_chunks{0};
  /*! \brief one-pass chunks decoded again after growing the output */
  size_t one_pass_reruns{0};
  /*! \brief chunks counted by following part chains (R1c) */
  size_t chain_counts{0};
};

class DeviceRecordIOReader {
 public:
  static DeviceRecordIOReader* Create(const std::string& uri, unsigned part_index,
                                      unsigned num_parts,
                                      const DeviceRecordIOConfig& cfg = DeviceRecordIOConfig());
  virtual ~DeviceRecordIOReader() = default;
  virtual void BeforeFirst() = 0;
  /*! \brief decode the next chunk; Value() is valid until the next call */
  virtual bool Next() = 0;
  virtual const DeviceRecordBatch& Value() const = 0;
  /*!
   * \brief decode the rest of the partition into one resident batch (kept in
   *  HBM until the next ReadAll / BeforeFirst)
   */
  virtual const DeviceRecordBatch& ReadAll() = 0;
  virtual size_t PartitionBytes() const = 0;
  virtual const DeviceRecordIOStats& Stats() const = 0;
  virtual hipStream_t stream() const = 0;
};

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_GPU_DEVICE_RECORDIO_H_
