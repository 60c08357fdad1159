/*!
 * \file src/io/single_file_split.h
 * \brief Unpartitioned line reader over one stream (used for "stdin").
 * Parity: reference `src/io/single_file_split.h:27-174` (256 KiB buffer that
 * doubles when a line does not fit; partitioning unsupported).
 */
#ifndef DMLC_IO_SINGLE_FILE_SPLIT_H_
#define DMLC_IO_SINGLE_FILE_SPLIT_H_

#include <dmlc/io.h>
#include <dmlc/logging.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace dmlc {
namespace io {

class SingleFileSplit : public InputSplit {
 public:
  explicit SingleFileSplit(const char* fname) : use_stdin_(std::strcmp(fname, "stdin") == 0) {
    fp_ = use_stdin_ ? stdin : std::fopen(fname, "rb");
    CHECK(fp_ != nullptr) << "SingleFileSplit: fail to open " << fname;
    buffer_.resize(kBufferSize);
  }
  ~SingleFileSplit() override {
    if (!use_stdin_ && fp_ != nullptr) std::fclose(fp_);
  }
  void BeforeFirst() override {
    CHECK(!use_stdin_) << "cannot rewind stdin";
    std::fseek(fp_, 0, SEEK_SET);
    begin_ = end_ = 0;
    eof_ = false;
  }
  void HintChunkSize(size_t chunk_size) override {
    if (chunk_size > buffer_.size()) buffer_.resize(chunk_size);
  }
  size_t GetTotalSize() override {
    if (use_stdin_) return 0;
    const long cur = std::ftell(fp_);
    std::fseek(fp_, 0, SEEK_END);
    const long sz = std::ftell(fp_);
    std::fseek(fp_, cur, SEEK_SET);
    return static_cast<size_t>(sz);
  }
  void ResetPartition(unsigned part_index, unsigned num_parts) override {
    CHECK(part_index == 0 && num_parts == 1) << "stdin/single file split cannot be partitioned";
    BeforeFirst();
  }
  bool NextRecord(Blob* out_rec) override {
    while (true) {
      // find a complete line inside [begin_, end_)
      size_t p = begin_;
      while (p < end_ && buffer_[p] != '\n' && buffer_[p] != '\r') ++p;
      if (p < end_ || (eof_ && begin_ < end_)) {
        size_t q = p;
        while (q < end_ && (buffer_[q] == '\n' || buffer_[q] == '\r')) ++q;
        if (q == end_ && !eof_ && q == p) {
          // EOL run may continue in the next read; fall through to refill
        } else {
          buffer_[p < end_ ? p : end_] = '\0';
          out_rec->dptr = &buffer_[begin_];
          out_rec->size = q - begin_;
          begin_ = q;
          return true;
        }
      }
      if (eof_) return false;
      Refill();
    }
  }
  bool NextChunk(Blob* out_chunk) override {
    // a chunk = everything up to the last EOL currently buffered
    while (true) {
      if (begin_ < end_) {
        size_t last = end_;
        while (last > begin_ && buffer_[last - 1] != '\n' && buffer_[last - 1] != '\r') --last;
        if (last > begin_ || eof_) {
          const size_t stop = last > begin_ ? last : end_;
          out_chunk->dptr = &buffer_[begin_];
          out_chunk->size = stop - begin_;
          begin_ = stop;
          return true;
        }
      }
      if (eof_) return false;
      Refill();
    }
  }

 private:
  static const size_t kBufferSize = 256 << 10;
  void Refill() {
    // compact then grow if full
    if (begin_ != 0) {
      std::memmove(&buffer_[0], &buffer_[begin_], end_ - begin_);
      end_ -= begin_;
      begin_ = 0;
    }
    if (end_ + 1 >= buffer_.size()) buffer_.resize(buffer_.size() * 2);
    const size_t n = std::fread(&buffer_[end_], 1, buffer_.size() - 1 - end_, fp_);
    if (n == 0) eof_ = true;
    end_ += n;
  }
  bool use_stdin_;
  FILE* fp_;
  std::vector<char> buffer_;
  size_t begin_{0}, end_{0};
  bool eof_{false};
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_SINGLE_FILE_SPLIT_H_
