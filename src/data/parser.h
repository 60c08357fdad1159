/*!
 * \file src/data/parser.h
 * \brief ParserImpl (walks the per-thread RowBlockContainers of a parsed
 *  chunk) and ThreadedParser (parses ahead on a background thread).
 * Parity: reference `src/data/parser.h:30-126` (capacity-8 ThreadedIter of
 * vector<RowBlockContainer>, empty containers skipped).
 */
#ifndef DMLC_DATA_PARSER_H_
#define DMLC_DATA_PARSER_H_

#include <dmlc/data.h>
#include <dmlc/threadediter.h>

#include <memory>
#include <vector>

#include "./row_block.h"

namespace dmlc {
namespace data {

template <typename IndexType, typename DType>
class ThreadedParser;

template <typename IndexType, typename DType = real_t>
class ParserImpl : public Parser<IndexType, DType> {
 public:
  using Container = std::vector<RowBlockContainer<IndexType, DType>>;
  bool Next() override {
    while (true) {
      while (data_ptr_ < data_.size()) {
        const auto& c = data_[data_ptr_++];
        if (c.Size() != 0) {
          block_ = c.GetBlock();
          return true;
        }
      }
      if (!ParseNext(&data_)) return false;
      data_ptr_ = 0;
    }
  }
  const RowBlock<IndexType, DType>& Value() const override { return block_; }

 protected:
  friend class ThreadedParser<IndexType, DType>;
  /*! \brief parse the next chunk into one container per worker thread */
  virtual bool ParseNext(Container* data) = 0;
  size_t data_ptr_{0};
  Container data_;
  RowBlock<IndexType, DType> block_;
};

template <typename IndexType, typename DType = real_t>
class ThreadedParser : public ParserImpl<IndexType, DType> {
 public:
  using Container = typename ParserImpl<IndexType, DType>::Container;
  explicit ThreadedParser(ParserImpl<IndexType, DType>* base) : base_(base) {
    iter_.set_max_capacity(8);
    iter_.Init(
        [base](Container** dptr) {
          if (*dptr == nullptr) *dptr = new Container();
          return base->ParseNext(*dptr);
        },
        [base]() { base->BeforeFirst(); });
  }
  ~ThreadedParser() override {
    iter_.Destroy();
    delete tmp_;
  }
  void BeforeFirst() override {
    if (tmp_ != nullptr) iter_.Recycle(&tmp_);
    iter_.BeforeFirst();
    pos_ = 0;
  }
  bool Next() override {
    while (true) {
      while (tmp_ != nullptr && pos_ < tmp_->size()) {
        const auto& c = (*tmp_)[pos_++];
        if (c.Size() != 0) {
          this->block_ = c.GetBlock();
          return true;
        }
      }
      if (tmp_ != nullptr) iter_.Recycle(&tmp_);
      if (!iter_.Next(&tmp_)) return false;
      pos_ = 0;
    }
  }
  size_t BytesRead() const override { return base_->BytesRead(); }

 protected:
  bool ParseNext(Container*) override {
    LOG(FATAL) << "cannot call ParseNext on ThreadedParser";
    return false;
  }

 private:
  std::unique_ptr<ParserImpl<IndexType, DType>> base_;
  ThreadedIter<Container> iter_;
  Container* tmp_{nullptr};
  size_t pos_{0};
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_PARSER_H_
