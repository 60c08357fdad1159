/*!
 * \file src/data/disk_row_iter.h
 * \brief RowBlockIter paging through a binary cache file (`uri#cachefile`).
 * Parity: reference `src/data/disk_row_iter.h:29-139` — first use builds the
 * cache by flushing a RowBlockContainer every 64 MiB, later epochs stream the
 * pages back through a ThreadedIter; NumCol tracked over all pages.
 * Difference: the 64 MiB test runs after every row, not after every parser
 * block, so page boundaries do not depend on the parser's thread count (and
 * match the GPU route's DevicePageCache byte for byte).
 */
#ifndef DMLC_DATA_DISK_ROW_ITER_H_
#define DMLC_DATA_DISK_ROW_ITER_H_

#include <dmlc/data.h>
#include <dmlc/logging.h>
#include <dmlc/threadediter.h>
#include <dmlc/timer.h>

#include <algorithm>
#include <memory>
#include <string>

#include "./row_block.h"

namespace dmlc {
namespace data {

template <typename IndexType, typename DType = real_t>
class DiskRowIter : public RowBlockIter<IndexType, DType> {
 public:
  static const size_t kPageSize = 64UL << 20UL;

  DiskRowIter(Parser<IndexType, DType>* parser, const char* cache_file, bool reuse_cache)
      : cache_file_(cache_file) {
    if (reuse_cache) {
      if (!TryLoadCache()) {
        BuildCache(parser);
        CHECK(TryLoadCache()) << "failed to build cache file " << cache_file;
      }
    } else {
      BuildCache(parser);
      CHECK(TryLoadCache()) << "failed to build cache file " << cache_file;
    }
    delete parser;
  }
  ~DiskRowIter() override {
    iter_.Destroy();
    fi_.reset();
  }
  void BeforeFirst() override { iter_.BeforeFirst(); }
  bool Next() override {
    if (iter_.Next()) {
      row_ = iter_.Value().GetBlock();
      return true;
    }
    return false;
  }
  const RowBlock<IndexType, DType>& Value() const override { return row_; }
  size_t NumCol() const override { return num_col_; }

 private:
  bool TryLoadCache() {
    fi_.reset(SeekStream::CreateForRead(cache_file_.c_str(), true));
    if (fi_ == nullptr) return false;
    // scan once for NumCol (pages are small relative to the data)
    num_col_ = 0;
    {
      RowBlockContainer<IndexType, DType> page;
      while (page.Load(fi_.get())) {
        num_col_ = std::max(num_col_, static_cast<size_t>(page.max_index) + 1);
      }
      fi_->Seek(0);
    }
    iter_.Init(
        [this](RowBlockContainer<IndexType, DType>** dptr) {
          if (*dptr == nullptr) *dptr = new RowBlockContainer<IndexType, DType>();
          return (*dptr)->Load(fi_.get());
        },
        [this]() { fi_->Seek(0); });
    return true;
  }
  void BuildCache(Parser<IndexType, DType>* parser) {
    std::unique_ptr<Stream> fo(Stream::Create(cache_file_.c_str(), "w"));
    RowBlockContainer<IndexType, DType> page;
    const double tstart = GetTime();
    // the page-size test runs after every row (the reference tests after each
    // parser block, whose size depends on the thread count): page boundaries
    // are a function of the data alone, and the GPU route's DevicePageCache
    // writes the same pages
    while (parser->Next()) {
      const RowBlock<IndexType, DType> blk = parser->Value();
      for (size_t i = 0; i < blk.size; ++i) {
        page.Push(blk[i]);
        if (page.MemCostBytes() >= kPageSize) {
          page.Finalize();
          page.Save(fo.get());
          page.Clear();
          VLOG(1) << (parser->BytesRead() >> 20UL) << "MB read, "
                  << (parser->BytesRead() >> 20UL) / (GetTime() - tstart) << " MB/sec";
        }
      }
    }
    if (page.Size() != 0) {
      page.Finalize();
      page.Save(fo.get());
    }
  }
  std::string cache_file_;
  std::unique_ptr<SeekStream> fi_;
  size_t num_col_{0};
  ThreadedIter<RowBlockContainer<IndexType, DType>> iter_{4};
  RowBlock<IndexType, DType> row_;
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_DISK_ROW_ITER_H_
