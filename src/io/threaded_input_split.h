/*!
 * \file src/io/threaded_input_split.h
 * \brief Prefetch chunks of an InputSplitBase on a background I/O thread.
 * Parity: reference `src/io/threaded_input_split.h:23-101` (ThreadedIter of
 * Chunks, capacity 2, producer = NextBatchEx, record extraction on the
 * consumer side).
 */
#ifndef DMLC_IO_THREADED_INPUT_SPLIT_H_
#define DMLC_IO_THREADED_INPUT_SPLIT_H_

#include <dmlc/threadediter.h>

#include <algorithm>
#include <memory>

#include "./input_split_base.h"

namespace dmlc {
namespace io {

class ThreadedInputSplit : public InputSplit {
 public:
  ThreadedInputSplit(InputSplitBase* base, size_t batch_size)
      : base_(base), batch_size_(batch_size), buffer_size_(InputSplitBase::kBufferSize) {
    iter_.set_max_capacity(2);
    iter_.Init(
        [this](InputSplitBase::Chunk** dptr) {
          if (*dptr == nullptr) *dptr = new InputSplitBase::Chunk(buffer_size_);
          return base_->NextBatchEx(*dptr, batch_size_);
        },
        [this]() { base_->BeforeFirst(); });
  }
  ~ThreadedInputSplit() override {
    iter_.Destroy();
    delete tmp_chunk_;
  }
  void BeforeFirst() override {
    iter_.BeforeFirst();
    if (tmp_chunk_ != nullptr) iter_.Recycle(&tmp_chunk_);
  }
  void HintChunkSize(size_t chunk_size) override {
    buffer_size_ = std::max(chunk_size / sizeof(uint32_t), buffer_size_);
    base_->HintChunkSize(chunk_size);
  }
  size_t GetTotalSize() override { return base_->GetTotalSize(); }
  void ResetPartition(unsigned part_index, unsigned num_parts) override {
    iter_.Destroy();
    tmp_chunk_ = nullptr;
    base_->ResetPartition(part_index, num_parts);
    iter_.set_max_capacity(2);
    iter_.Init(
        [this](InputSplitBase::Chunk** dptr) {
          if (*dptr == nullptr) *dptr = new InputSplitBase::Chunk(buffer_size_);
          return base_->NextBatchEx(*dptr, batch_size_);
        },
        [this]() { base_->BeforeFirst(); });
  }
  bool NextRecord(Blob* out_rec) override {
    if (tmp_chunk_ == nullptr && !iter_.Next(&tmp_chunk_)) return false;
    while (!base_->ExtractNextRecord(out_rec, tmp_chunk_)) {
      iter_.Recycle(&tmp_chunk_);
      if (!iter_.Next(&tmp_chunk_)) return false;
    }
    return true;
  }
  bool NextChunk(Blob* out_chunk) override {
    if (tmp_chunk_ == nullptr && !iter_.Next(&tmp_chunk_)) return false;
    while (!base_->ExtractNextChunk(out_chunk, tmp_chunk_)) {
      iter_.Recycle(&tmp_chunk_);
      if (!iter_.Next(&tmp_chunk_)) return false;
    }
    return true;
  }

 private:
  std::unique_ptr<InputSplitBase> base_;
  size_t batch_size_;
  size_t buffer_size_;
  ThreadedIter<InputSplitBase::Chunk> iter_;
  InputSplitBase::Chunk* tmp_chunk_{nullptr};
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_THREADED_INPUT_SPLIT_H_
