/*!
 * \file src/io/cached_input_split.h
 * \brief `uri#cachefile`: the first epoch streams chunks from the base split
 *  and appends them to a local cache file; later epochs replay the cache.
 * Parity: reference `src/io/cached_input_split.h:28-188` (cache format =
 * repeated [size_t n][n bytes]; writer thread capacity 16; ResetPartition
 * unsupported).
 */
#ifndef DMLC_IO_CACHED_INPUT_SPLIT_H_
#define DMLC_IO_CACHED_INPUT_SPLIT_H_

#include <dmlc/threadediter.h>

#include <memory>
#include <string>

#include "./input_split_base.h"

namespace dmlc {
namespace io {

class CachedInputSplit : public InputSplit {
 public:
  /*!
   * \param base the split to cache (owned)
   * \param cache_file local cache path
   * \param reuse_exist_cache replay an existing cache instead of rebuilding
   */
  CachedInputSplit(InputSplitBase* base, const char* cache_file, bool reuse_exist_cache = true)
      : base_(base), cache_file_(cache_file) {
    if (!reuse_exist_cache || !InitCachedIter()) InitPreprocIter();
  }
  ~CachedInputSplit() override {
    iter_preproc_.reset();
    fo_.reset();
    iter_cached_.reset();
    delete tmp_chunk_;
  }
  void BeforeFirst() override {
    if (iter_preproc_ != nullptr) {
      // finish writing the cache first
      if (tmp_chunk_ != nullptr) iter_preproc_->Recycle(&tmp_chunk_);
      while (iter_preproc_->Next(&tmp_chunk_)) iter_preproc_->Recycle(&tmp_chunk_);
      iter_preproc_.reset();
      fo_.reset();
      CHECK(InitCachedIter()) << "failed to build cache " << cache_file_;
    } else {
      if (tmp_chunk_ != nullptr) iter_cached_->Recycle(&tmp_chunk_);
      iter_cached_->BeforeFirst();
    }
  }
  void HintChunkSize(size_t chunk_size) override { base_->HintChunkSize(chunk_size); }
  size_t GetTotalSize() override { return base_->GetTotalSize(); }
  void ResetPartition(unsigned, unsigned) override {
    LOG(FATAL) << "ResetPartition is not supported by CachedInputSplit";
  }
  bool NextRecord(Blob* out_rec) override {
    auto* iter = CurrentIter();
    if (tmp_chunk_ == nullptr && !iter->Next(&tmp_chunk_)) return false;
    while (!base_->ExtractNextRecord(out_rec, tmp_chunk_)) {
      iter->Recycle(&tmp_chunk_);
      if (!iter->Next(&tmp_chunk_)) return false;
    }
    return true;
  }
  bool NextChunk(Blob* out_chunk) override {
    auto* iter = CurrentIter();
    if (tmp_chunk_ == nullptr && !iter->Next(&tmp_chunk_)) return false;
    while (!base_->ExtractNextChunk(out_chunk, tmp_chunk_)) {
      iter->Recycle(&tmp_chunk_);
      if (!iter->Next(&tmp_chunk_)) return false;
    }
    return true;
  }

 private:
  using Chunk = InputSplitBase::Chunk;
  ThreadedIter<Chunk>* CurrentIter() {
    return iter_preproc_ != nullptr ? iter_preproc_.get() : iter_cached_.get();
  }
  void InitPreprocIter() {
    fo_.reset(Stream::Create(cache_file_.c_str(), "w"));
    iter_preproc_.reset(new ThreadedIter<Chunk>());
    iter_preproc_->set_max_capacity(16);
    iter_preproc_->Init([this](Chunk** dptr) {
      if (*dptr == nullptr) *dptr = new Chunk(InputSplitBase::kBufferSize);
      Chunk* p = *dptr;
      if (!base_->NextChunkEx(p)) return false;
      const size_t size = p->end - p->begin;
      fo_->Write(&size, sizeof(size));
      fo_->Write(p->begin, size);
      return true;
    });
  }
  bool InitCachedIter() {
    fi_.reset(SeekStream::CreateForRead(cache_file_.c_str(), true));
    if (fi_ == nullptr) return false;
    iter_cached_.reset(new ThreadedIter<Chunk>());
    iter_cached_->set_max_capacity(16);
    iter_cached_->Init(
        [this](Chunk** dptr) {
          if (*dptr == nullptr) *dptr = new Chunk(InputSplitBase::kBufferSize);
          Chunk* p = *dptr;
          size_t size;
          const size_t nread = fi_->Read(&size, sizeof(size));
          if (nread == 0) return false;
          CHECK_EQ(nread, sizeof(size)) << cache_file_ << " has invalid cache file format";
          p->data.resize(size / sizeof(uint32_t) + 1);
          p->begin = reinterpret_cast<char*>(p->data.data());
          p->end = p->begin + size;
          CHECK_EQ(fi_->Read(p->begin, size), size)
              << cache_file_ << " has invalid cache file format";
          return true;
        },
        [this]() { fi_->Seek(0); });
    return true;
  }
  std::unique_ptr<InputSplitBase> base_;
  std::string cache_file_;
  std::unique_ptr<Stream> fo_;
  std::unique_ptr<SeekStream> fi_;
  std::unique_ptr<ThreadedIter<Chunk>> iter_preproc_;
  std::unique_ptr<ThreadedIter<Chunk>> iter_cached_;
  Chunk* tmp_chunk_{nullptr};
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_CACHED_INPUT_SPLIT_H_
