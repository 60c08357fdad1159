/*!
 * \file src/data/text_parser.h
 * \brief Multi-threaded text chunk parsing shared by LibSVM / LibFM / CSV.
 *
 * Parity: reference `src/data/text_parser.h:25-136` — a chunk from the
 * InputSplit is cut into one byte range per thread, each range start moved
 * back to a line boundary, every range parsed into its own container, and
 * exceptions from worker threads rethrown on the caller.
 *
 * Difference: the `nthread` argument is honoured (URI arg
 * `?nthread=N`; default = OpenMP max threads) instead of being ignored.
 * Line iteration uses memchr, which is several times faster than a byte loop.
 */
#ifndef DMLC_DATA_TEXT_PARSER_H_
#define DMLC_DATA_TEXT_PARSER_H_

#include <dmlc/io.h>
#include <dmlc/omp.h>

#include <algorithm>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <vector>

#include "./parser.h"
#include "./strtonum.h"

namespace dmlc {
namespace data {

template <typename IndexType, typename DType = real_t>
class TextParserBase : public ParserImpl<IndexType, DType> {
 public:
  using Container = typename ParserImpl<IndexType, DType>::Container;
  TextParserBase(InputSplit* source, int nthread) : source_(source) {
    nthread_ = nthread > 0 ? nthread : std::max(1, omp_get_max_threads());
  }
  void BeforeFirst() override { source_->BeforeFirst(); }
  size_t BytesRead() const override { return bytes_read_; }
  bool ParseNext(Container* data) override { return FillData(data); }
  int nthread() const { return nthread_; }

 protected:
  /*! \brief parse every complete line in [begin, end) into out */
  virtual void ParseBlock(const char* begin, const char* end,
                          RowBlockContainer<IndexType, DType>* out) = 0;

  /*! \brief call fn(line_begin, line_end) for every non-empty line */
  template <typename Fn>
  static inline void ForEachLine(const char* begin, const char* end, Fn fn) {
    const char* p = begin;
    while (p != end) {
      while (p != end && iseol(*p)) ++p;
      if (p == end) break;
      const char* nl = static_cast<const char*>(std::memchr(p, '\n', end - p));
      const char* lend = nl == nullptr ? end : nl;
      const char* cr = static_cast<const char*>(std::memchr(p, '\r', lend - p));
      if (cr != nullptr) lend = cr;
      fn(p, lend);
      p = lend;
    }
  }
  /*! \brief next blank-separated token in [p, end): sets [*tb, *te) */
  static inline bool NextToken(const char** p, const char* end, const char** tb,
                               const char** te) {
    const char* q = *p;
    while (q != end && isblank(*q)) ++q;
    if (q == end) {
      *p = end;
      return false;
    }
    *tb = q;
    while (q != end && !isblank(*q)) ++q;
    *te = q;
    *p = q;
    return true;
  }

 private:
  bool FillData(Container* data) {
    InputSplit::Blob chunk;
    if (!source_->NextChunk(&chunk)) return false;
    const int nthread = nthread_;
    data->resize(nthread);
    bytes_read_ += chunk.size;
    CHECK_NE(chunk.size, 0U);
    const char* head = static_cast<const char*>(chunk.dptr);
    // range boundaries moved back to just after an EOL
    std::vector<const char*> cut(nthread + 1);
    cut[0] = head;
    cut[nthread] = head + chunk.size;
    const size_t nstep = (chunk.size + nthread - 1) / nthread;
    for (int t = 1; t < nthread; ++t) {
      const char* p = head + std::min(chunk.size, nstep * t);
      while (p != head && !iseol(*(p - 1))) --p;
      cut[t] = std::max(p, cut[t - 1]);
    }
    std::exception_ptr err = nullptr;
    std::mutex err_mu;
#pragma omp parallel for num_threads(nthread) schedule(static, 1)
    for (int t = 0; t < nthread; ++t) {
      try {
        // parse into a container on this thread's stack (the vectors move in
        // and out: O(1)): the threads' containers sit side by side in `data`,
        // and every push_back updates a vector's end pointer -- adjacent
        // containers share cache lines at their edges
        typename Container::value_type local;
        std::swap(local, (*data)[t]);
        ParseBlock(cut[t], cut[t + 1], &local);
        std::swap(local, (*data)[t]);
      } catch (...) {
        std::lock_guard<std::mutex> lock(err_mu);
        if (err == nullptr) err = std::current_exception();
      }
    }
    if (err != nullptr) std::rethrow_exception(err);
    this->data_ptr_ = 0;
    return true;
  }
  int nthread_;
  size_t bytes_read_{0};
  std::unique_ptr<InputSplit> source_;
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_TEXT_PARSER_H_
