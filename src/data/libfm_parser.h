/*!
 * \file src/data/libfm_parser.h
 * \brief LibFM text (`label[:weight] field:index[:value] ...`) -> CSR with
 *  field ids.
 * Parity: reference `src/data/libfm_parser.h:36-93` (ParseTriple per token,
 * tokens with fewer than two parts skipped, field.size() == index.size()).
 * Token rules are those of libsvm_parser.h; missing values become 1.0.
 */
#ifndef DMLC_DATA_LIBFM_PARSER_H_
#define DMLC_DATA_LIBFM_PARSER_H_

#include <string>

#include "./text_parser.h"

namespace dmlc {
namespace data {

template <typename IndexType, typename DType = real_t>
class LibFMParser : public TextParserBase<IndexType, DType> {
 public:
  using Base = TextParserBase<IndexType, DType>;
  LibFMParser(InputSplit* source, int nthread) : Base(source, nthread) {}

  /*!
   * \brief single-pass parse of the common `digits:digits[:number]` token;
   *  false (nothing consumed) when it needs the general ParseTriple grammar.
   *  Equivalent on the tokens it accepts: the unsigned / float parsers only
   *  consume digitchars, so they stop at the same byte whether bounded by the
   *  digitchars run or the token end, and ParseTriple ignores what follows
   *  the third number inside the token.
   */
  static inline bool FastTriple(const char* tb, const char* te,
                                RowBlockContainer<IndexType, DType>* out) {
    const char* p = tb;
    IndexType v[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
      if (p == te || !isdigit(*p)) return false;
      IndexType x = 0;
      do {
        x = static_cast<IndexType>(x * 10u + static_cast<IndexType>(*p - '0'));
        ++p;
      } while (p != te && isdigit(*p));
      v[k] = x;
      if (k == 0) {
        if (p == te || *p != ':') return false;
        ++p;
      }
    }
    if (p == te) {
      out->PushField(v[0]);
      out->PushFeature(v[1], DType(1.0f), false);
      return true;
    }
    if (*p != ':' || p + 1 == te || !isdigitchars(p[1])) return false;
    const real_t val = StrToFloat(p + 1, te, nullptr);
    out->PushField(v[0]);
    out->PushFeature(v[1], static_cast<DType>(val), true);
    return true;
  }

  static inline void ParseLine(const char* lb, const char* le,
                               RowBlockContainer<IndexType, DType>* out) {
    const char* p = lb;
    const char *tb, *te;
    if (!Base::NextToken(&p, le, &tb, &te)) return;
    real_t label = 0.0f, weight = 0.0f;
    bool bad = false;
    const int r = ParsePair<real_t, real_t>(tb, te, &label, &weight, &bad);
    if (r < 1) return;
    out->BeginRow(static_cast<DType>(label));
    if (r == 2) out->SetWeight(weight);
    while (Base::NextToken(&p, le, &tb, &te)) {
      IndexType fid = 0, idx = 0;
      real_t val = 0.0f;
      if (FastTriple(tb, te, out)) continue;
      const int rr = ParseTriple<IndexType, IndexType, real_t>(tb, te, &fid, &idx, &val, &bad);
      if (rr <= 1) continue;
      CHECK(!bad) << "negative field/index in LibFM token \"" << std::string(tb, te - tb) << "\"";
      out->PushField(fid);
      out->PushFeature(idx, static_cast<DType>(val), rr == 3);
    }
    out->EndRow();
  }

 protected:
  void ParseBlock(const char* begin, const char* end,
                  RowBlockContainer<IndexType, DType>* out) override {
    out->Clear();
    Base::ForEachLine(begin, end, [out](const char* lb, const char* le) {
      ParseLine(lb, le, out);
    });
    out->Finalize();
    CHECK_EQ(out->field.size(), out->index.size());
  }
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_LIBFM_PARSER_H_
