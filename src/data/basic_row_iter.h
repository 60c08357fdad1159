/*!
 * \file src/data/basic_row_iter.h
 * \brief RowBlockIter that loads the whole dataset into one in-memory block.
 * Parity: reference `src/data/basic_row_iter.h:24-83` (progress log every
 * 10 MB, NumCol = max_index + 1).
 */
#ifndef DMLC_DATA_BASIC_ROW_ITER_H_
#define DMLC_DATA_BASIC_ROW_ITER_H_

#include <dmlc/data.h>
#include <dmlc/logging.h>
#include <dmlc/timer.h>

#include <memory>

#include "./row_block.h"

namespace dmlc {
namespace data {

template <typename IndexType, typename DType = real_t>
class BasicRowIter : public RowBlockIter<IndexType, DType> {
 public:
  explicit BasicRowIter(Parser<IndexType, DType>* parser) { this->Init(parser); }
  void BeforeFirst() override { at_head_ = true; }
  bool Next() override {
    if (at_head_) {
      at_head_ = false;
      return true;
    }
    return false;
  }
  const RowBlock<IndexType, DType>& Value() const override { return row_; }
  size_t NumCol() const override { return static_cast<size_t>(data_.max_index) + 1; }

 private:
  void Init(Parser<IndexType, DType>* parser) {
    std::unique_ptr<Parser<IndexType, DType>> owner(parser);
    data_.Clear();
    const double tstart = GetTime();
    size_t bytes_expect = 10UL << 20UL;
    while (parser->Next()) {
      data_.Push(parser->Value());
      const size_t bytes_read = parser->BytesRead();
      if (bytes_read >= bytes_expect) {
        const double tdiff = GetTime() - tstart;
        VLOG(1) << (bytes_read >> 20UL) << "MB read, " << (bytes_read >> 20UL) / tdiff
                << " MB/sec";
        bytes_expect += 10UL << 20UL;
      }
    }
    data_.Finalize();
    row_ = data_.GetBlock();
    VLOG(1) << "finish reading " << row_.size << " rows in " << GetTime() - tstart << " sec";
  }
  bool at_head_{true};
  RowBlockContainer<IndexType, DType> data_;
  RowBlock<IndexType, DType> row_;
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_BASIC_ROW_ITER_H_
