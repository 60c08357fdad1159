/*!
 * \file dmlc/memory_io.h
 * \brief In-memory streams.
 * Parity: reference `include/dmlc/memory_io.h` — MemoryFixedSizeStream
 * (:21-60, bounds CHECKed) and MemoryStringStream (:66-103, grows).
 */
#ifndef DMLC_MEMORY_IO_H_
#define DMLC_MEMORY_IO_H_

#include <algorithm>
#include <cstring>
#include <string>

#include "./base.h"
#include "./io.h"
#include "./logging.h"

namespace dmlc {

/*! \brief seek stream over a caller-owned fixed-size buffer */
class MemoryFixedSizeStream : public SeekStream {
 public:
  MemoryFixedSizeStream(void* p_buffer, size_t buffer_size)
      : p_buffer_(reinterpret_cast<char*>(p_buffer)),
        buffer_size_(buffer_size) {}
  using SeekStream::Read;
  using SeekStream::Write;
  size_t Read(void* ptr, size_t size) override {
    CHECK(curr_ptr_ <= buffer_size_) << "read position past end of fixed buffer";
    size_t nread = std::min(buffer_size_ - curr_ptr_, size);
    if (nread != 0) std::memcpy(ptr, p_buffer_ + curr_ptr_, nread);
    curr_ptr_ += nread;
    return nread;
  }
  void Write(const void* ptr, size_t size) override {
    if (size == 0) return;
    CHECK(curr_ptr_ + size <= buffer_size_)
        << "write of " << size << " bytes overflows fixed buffer of "
        << buffer_size_ << " (at " << curr_ptr_ << ")";
    std::memcpy(p_buffer_ + curr_ptr_, ptr, size);
    curr_ptr_ += size;
  }
  void Seek(size_t pos) override { curr_ptr_ = pos; }
  size_t Tell() override { return curr_ptr_; }

 private:
  char* p_buffer_;
  size_t buffer_size_;
  size_t curr_ptr_{0};
};

/*! \brief seek stream backed by a std::string that grows on write */
class MemoryStringStream : public SeekStream {
 public:
  explicit MemoryStringStream(std::string* p_buffer) : p_buffer_(p_buffer) {}
  using SeekStream::Read;
  using SeekStream::Write;
  size_t Read(void* ptr, size_t size) override {
    CHECK(curr_ptr_ <= p_buffer_->length());
    size_t nread = std::min(p_buffer_->length() - curr_ptr_, size);
    if (nread != 0) std::memcpy(ptr, p_buffer_->data() + curr_ptr_, nread);
    curr_ptr_ += nread;
    return nread;
  }
  void Write(const void* ptr, size_t size) override {
    if (size == 0) return;
    if (curr_ptr_ + size > p_buffer_->length()) {
      p_buffer_->resize(curr_ptr_ + size);
    }
    std::memcpy(&(*p_buffer_)[0] + curr_ptr_, ptr, size);
    curr_ptr_ += size;
  }
  void Seek(size_t pos) override { curr_ptr_ = pos; }
  size_t Tell() override { return curr_ptr_; }

 private:
  std::string* p_buffer_;
  size_t curr_ptr_{0};
};
}  // namespace dmlc
#endif  // DMLC_MEMORY_IO_H_
