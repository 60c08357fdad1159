/*!
 * \file dmlc/recordio.h
 * \brief RecordIO: a splittable binary record container.
 *
 * On-disk format (bit-exact with the reference, `include/dmlc/recordio.h:16-75`,
 * `src/recordio.cc:11-82`):
 *
 *     u32 kMagic = 0xced7230a | u32 lrec = (cflag << 29) | length | payload | pad to 4 B
 *
 * cflag 0 = whole record, 1/2/3 = first/middle/last part.  The writer cuts a
 * record at EVERY 4-byte-aligned occurrence of kMagic inside its payload, drops
 * that magic word and starts a new part; the reader re-inserts it.  Hence every
 * aligned kMagic in a file whose next word has cflag 0 or 1 is a record head —
 * the invariant that makes fully parallel decoding possible (GPU kernel
 * `recordio_decode`, src/gpu/recordio_kernels.hip).
 */
#ifndef DMLC_RECORDIO_H_
#define DMLC_RECORDIO_H_

#include <cstring>
#include <string>

#include "./io.h"
#include "./logging.h"

namespace dmlc {

/*! \brief writes records into a stream */
class RecordIOWriter {
 public:
  /*! \brief magic word marking a record head */
  static constexpr uint32_t kMagic = 0xced7230a;
  /*! \brief pack (cflag, length) into the lrec word */
  inline static uint32_t EncodeLRec(uint32_t cflag, uint32_t length) {
    return (cflag << 29U) | length;
  }
  inline static uint32_t DecodeFlag(uint32_t rec) { return (rec >> 29U) & 7U; }
  inline static uint32_t DecodeLength(uint32_t rec) { return rec & ((1U << 29U) - 1U); }

  explicit RecordIOWriter(Stream* stream) : stream_(stream) {
    static_assert(sizeof(uint32_t) == 4, "uint32_t must be 4 bytes");
  }
  /*! \brief append one record (< 2^29 bytes) */
  void WriteRecord(const void* buf, size_t size);
  inline void WriteRecord(const std::string& data) {
    this->WriteRecord(data.data(), data.length());
  }
  /*! \brief number of magic words escaped so far */
  inline size_t except_counter() const { return except_counter_; }
  /*! \brief bytes written so far (for building index files) */
  inline size_t Tell() const { return bytes_written_; }

 private:
  Stream* stream_;
  size_t except_counter_{0};
  size_t bytes_written_{0};
};

/*! \brief sequential record reader over a stream */
class RecordIOReader {
 public:
  explicit RecordIOReader(Stream* stream) : stream_(stream) {}
  /*! \brief next record into out_rec (multi-part records are re-joined) */
  bool NextRecord(std::string* out_rec);
  /*! \brief seek to a record head (seekable streams only) */
  inline void Seek(size_t pos) {
    auto* ss = dynamic_cast<SeekStream*>(stream_);
    CHECK(ss != nullptr) << "RecordIOReader::Seek needs a SeekStream";
    ss->Seek(pos);
    end_of_stream_ = false;
  }

 private:
  Stream* stream_;
  bool end_of_stream_{false};
};

/*!
 * \brief reader of records inside one in-memory chunk, optionally restricted
 *  to sub-partition `part_index` of `num_parts` (for multi-threaded decode).
 */
class RecordIOChunkReader {
 public:
  explicit RecordIOChunkReader(InputSplit::Blob chunk, unsigned part_index = 0,
                               unsigned num_parts = 1);
  /*! \brief next record; the blob points into the chunk or an internal buffer */
  bool NextRecord(InputSplit::Blob* out_rec);

 private:
  char* pbegin_;
  char* pend_;
  std::string temp_;
};

}  // namespace dmlc
#endif  // DMLC_RECORDIO_H_
