/*!
 * \file dmlc/io.h
 * \brief Byte streams, seekable streams, serializable objects and sharded
 *  record readers (InputSplit).
 *
 * Parity: reference `include/dmlc/io.h` — Stream (:29-86) incl. templated
 * Write/Read through the serializer (:428-437), SeekStream (:89-109),
 * Serializable (:112-126), InputSplit with Blob / HintChunkSize /
 * GetTotalSize / BeforeFirst / NextRecord / NextChunk / NextBatch /
 * ResetPartition / Create (:135-282), dmlc::ostream / dmlc::istream streambuf
 * adapters (:298-486).
 *
 * URIs: `[proto://host]/path[;more][?k=v&...][#cachefile]` with protocols
 * file:// (default), hdfs://, viewfs://, s3://, http(s)://, azure:// and the
 * special names "stdin" / "stdout".
 */
#ifndef DMLC_IO_H_
#define DMLC_IO_H_

#include <cstdio>
#include <istream>
#include <ostream>
#include <streambuf>
#include <string>
#include <vector>

#include "./base.h"
#include "./logging.h"
#include "./serializer.h"

namespace dmlc {

/*! \brief abstract byte stream */
class Stream {
 public:
  /*! \return bytes actually read; 0 means end of stream */
  virtual size_t Read(void* ptr, size_t size) = 0;
  /*! \brief write exactly `size` bytes (throws dmlc::Error on failure) */
  virtual void Write(const void* ptr, size_t size) = 0;
  virtual ~Stream() = default;

  /*!
   * \brief open a stream for `uri`.
   * \param flag "r" read, "w" write (truncate), "a" append
   * \param allow_null return nullptr instead of throwing when it cannot open
   */
  static Stream* Create(const char* uri, const char* const flag,
                        bool allow_null = false);

  /*! \brief serialize any supported object (see serializer.h) */
  template <typename T>
  inline void Write(const T& data) {
    serializer::Handler<T>::Write(this, data);
  }
  /*! \brief deserialize; false when the stream ended early */
  template <typename T>
  inline bool Read(T* out_data) {
    return serializer::Handler<T>::Read(this, out_data);
  }
  /*! \brief write `num_elems` objects one after another */
  template <typename T>
  inline void WriteArray(const T* data, size_t num_elems) {
    for (size_t i = 0; i < num_elems; ++i) this->Write<T>(data[i]);
  }
  /*! \brief read `num_elems` objects written by WriteArray */
  template <typename T>
  inline bool ReadArray(T* data, size_t num_elems) {
    for (size_t i = 0; i < num_elems; ++i) {
      if (!this->Read<T>(data + i)) return false;
    }
    return true;
  }
};

/*! \brief stream that supports random access reads */
class SeekStream : public Stream {
 public:
  virtual ~SeekStream() = default;
  virtual void Seek(size_t pos) = 0;
  virtual size_t Tell() = 0;
  /*! \brief open `uri` for reading with seek support */
  static SeekStream* CreateForRead(const char* uri, bool allow_null = false);
};

/*! \brief interface of objects that can save/load themselves */
class Serializable {
 public:
  virtual ~Serializable() = default;
  virtual void Load(Stream* fi) = 0;
  virtual void Save(Stream* fo) const = 0;
};

/*!
 * \brief sharded reader of records from one or many files.
 *
 *  A job with `num_parts` workers gives each worker a disjoint, record-aligned
 *  byte range (or, for indexed RecordIO, record range) of the concatenated
 *  inputs; together the parts cover every record exactly once.
 */
class InputSplit {
 public:
  /*! \brief a view of memory owned by the split, valid until the next call */
  struct Blob {
    void* dptr;
    size_t size;
  };
  /*! \brief request chunks of at least this many bytes (a hint) */
  virtual void HintChunkSize(size_t /*chunk_size*/) {}
  /*! \brief total bytes of all input files (not just this part) */
  virtual size_t GetTotalSize() = 0;
  /*! \brief rewind to the first record of this part */
  virtual void BeforeFirst() = 0;
  /*! \brief next single record; false at end of part */
  virtual bool NextRecord(Blob* out_rec) = 0;
  /*! \brief next chunk holding one or more whole records */
  virtual bool NextChunk(Blob* out_chunk) = 0;
  /*! \brief next chunk of up to `n_records` records (indexed splits honour n) */
  virtual bool NextBatch(Blob* out_chunk, size_t /*n_records*/) {
    return NextChunk(out_chunk);
  }
  /*! \brief re-partition: become part `part_index` of `num_parts` */
  virtual void ResetPartition(unsigned part_index, unsigned num_parts) = 0;
  virtual ~InputSplit() = default;

  /*!
   * \brief create a split.
   * \param uri ';'-separated list of files / directories / regexes,
   *        optionally `#cachefile` and `?k=v` arguments
   * \param type "text", "recordio" or "indexed_recordio"
   */
  static InputSplit* Create(const char* uri, unsigned part_index,
                            unsigned num_parts, const char* type);
  /*!
   * \brief create a split with index file / shuffling support.
   * \param index_uri index file for "indexed_recordio" (text "key offset" lines)
   * \param shuffle shuffle record order (indexed_recordio) every epoch
   * \param seed shuffle seed
   * \param batch_size records per NextChunk for indexed splits
   * \param recurse_directories descend into sub-directories
   */
  static InputSplit* Create(const char* uri, const char* index_uri,
                            unsigned part_index, unsigned num_parts,
                            const char* type, const bool shuffle = false,
                            const int seed = 0, const size_t batch_size = 256,
                            const bool recurse_directories = false);
};

/*!
 * \brief std::ostream over a dmlc::Stream (buffered).
 *  Parity: reference io.h:298-366.
 */
class ostream : public std::basic_ostream<char> {
 public:
  explicit ostream(Stream* stream, size_t buffer_size = (1 << 10))
      : std::basic_ostream<char>(nullptr), buf_(buffer_size) {
    this->set_stream(stream);
  }
  ~ostream() DMLC_NO_EXCEPTION { buf_.pubsync(); }
  /*! \brief redirect to another stream (flushes the current one) */
  inline void set_stream(Stream* stream) {
    buf_.set_stream(stream);
    this->rdbuf(&buf_);
  }
  /*! \brief bytes written through this ostream */
  inline size_t bytes_written() const { return buf_.bytes_out(); }

 private:
  class OutBuf : public std::streambuf {
   public:
    explicit OutBuf(size_t buffer_size) : buffer_(buffer_size) {
      if (buffer_.empty()) buffer_.resize(2);
    }
    inline void set_stream(Stream* stream) {
      if (stream_ != nullptr) this->pubsync();
      stream_ = stream;
      this->setp(buffer_.data(), buffer_.data() + buffer_.size() - 1);
    }
    size_t bytes_out() const { return bytes_out_ + (pptr() - pbase()); }

   private:
    Stream* stream_{nullptr};
    std::vector<char> buffer_;
    size_t bytes_out_{0};
    int sync() override {
      if (stream_ == nullptr) return -1;
      std::ptrdiff_t n = pptr() - pbase();
      if (n != 0) stream_->Write(pbase(), n);
      bytes_out_ += n;
      this->pbump(-static_cast<int>(n));
      return 0;
    }
    int_type overflow(int_type c) override {
      *(this->pptr()) = static_cast<char>(c);
      this->pbump(1);
      return this->sync() == 0 ? c : traits_type::eof();
    }
  };
  OutBuf buf_;
};

/*!
 * \brief std::istream over a dmlc::Stream (buffered).
 *  Parity: reference io.h:369-422.
 */
class istream : public std::basic_istream<char> {
 public:
  explicit istream(Stream* stream, size_t buffer_size = (1 << 10))
      : std::basic_istream<char>(nullptr), buf_(buffer_size) {
    this->set_stream(stream);
  }
  virtual ~istream() DMLC_NO_EXCEPTION {}
  inline void set_stream(Stream* stream) {
    buf_.set_stream(stream);
    this->rdbuf(&buf_);
  }
  /*! \brief bytes consumed from the underlying stream */
  inline size_t bytes_read() const { return buf_.bytes_read(); }

 private:
  class InBuf : public std::streambuf {
   public:
    explicit InBuf(size_t buffer_size) : buffer_(buffer_size) {
      if (buffer_.empty()) buffer_.resize(1);
    }
    inline void set_stream(Stream* stream) {
      stream_ = stream;
      this->setg(buffer_.data(), buffer_.data(), buffer_.data());
    }
    size_t bytes_read() const { return bytes_read_; }

   private:
    Stream* stream_{nullptr};
    std::vector<char> buffer_;
    size_t bytes_read_{0};
    int_type underflow() override {
      if (this->gptr() == this->egptr()) {
        if (stream_ == nullptr) return traits_type::eof();
        size_t n = stream_->Read(buffer_.data(), buffer_.size());
        bytes_read_ += n;
        this->setg(buffer_.data(), buffer_.data(), buffer_.data() + n);
      }
      if (this->gptr() != this->egptr()) {
        return traits_type::to_int_type(*this->gptr());
      }
      return traits_type::eof();
    }
  };
  InBuf buf_;
};

namespace serializer {
inline void WriteBytes(Stream* strm, const void* ptr, size_t size) {
  strm->Write(ptr, size);
}
inline bool ReadBytes(Stream* strm, void* ptr, size_t size) {
  return strm->Read(ptr, size) == size;
}
}  // namespace serializer
}  // namespace dmlc

#endif  // DMLC_IO_H_
