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
  /*! \brief bytes per chunk (a record must fit in one chunk) */
  size_t chunk_bytes{64UL << 20};
  /*! \brief HIP device (-1 = current) */
  int device{-1};
  /*! \brief -1 auto (mmap + hipHostRegister, fall back to pinned staging), 0 off, 1 required */
  int zero_copy{-1};
  /*! \brief apply `?k=v` overrides: chunk_mb, chunk_bytes, device, zero_copy */
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
  size_t bytes{0};
  size_t chunks{0};
  size_t records{0};
  bool zero_copy{false};
  double wait_gpu_sec{0};
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
