/*!
 * \file src/data/libsvm_parser.h
 * \brief LibSVM text -> CSR (CPU implementation and GPU parity oracle).
 *
 * Grammar (shared bit-for-bit with the HIP kernels in src/gpu/libsvm_kernels.hip):
 *   line    := bytes between EOL characters ('\n', '\r'); EOL-only stretches skipped
 *   token   := maximal run of non-blank bytes (blank = ' ' or '\t')
 *   row     := label_tok [qid_tok] feature_tok*
 *   label_tok   = `label[:weight]` via ParsePair<float,float>; a line whose
 *                 first token has no digit character is skipped
 *   qid_tok     = second token starting with "qid:"; value = int64 after it
 *   feature_tok = `index[:value]` via ParsePair<IndexType,float>; tokens
 *                 without a digit character are ignored; a '-' index is an error
 * Parity: reference `src/data/libsvm_parser.h:36-99` for well-formed input.
 * Fixes: `qid:` is no longer re-parsed as a feature;
 * missing per-row weights / per-feature values are backfilled with 1.0.
 */
#ifndef DMLC_DATA_LIBSVM_PARSER_H_
#define DMLC_DATA_LIBSVM_PARSER_H_

#include <cstring>
#include <map>
#include <string>

#include "./text_parser.h"

namespace dmlc {
namespace data {

template <typename IndexType, typename DType = real_t>
class LibSVMParser : public TextParserBase<IndexType, DType> {
 public:
  using Base = TextParserBase<IndexType, DType>;
  LibSVMParser(InputSplit* source, int nthread) : Base(source, nthread) {}

  /*!
   * \brief single-pass parse of the common `digits[:number]` feature token.
   *  Returns false (nothing consumed) when the token needs the general
   *  ParsePair grammar. Equivalent to ParsePair on the tokens it accepts:
   *  StrToUInt / StrToFloat only consume digitchars, so they stop at the same
   *  byte whether bounded by the digitchars run or by the token end, and
   *  ParsePair ignores whatever follows the value inside the token.
   */
  static inline bool FastFeature(const char* tb, const char* te, IndexType* idx, real_t* val,
                                 RowBlockContainer<IndexType, DType>* out) {
    const char* p = tb;
    if (!isdigit(*p)) return false;
    IndexType v = 0;
    do {
      v = static_cast<IndexType>(v * 10u + static_cast<IndexType>(*p - '0'));
      ++p;
    } while (p != te && isdigit(*p));
    if (p == te) {
      out->PushFeature(v, DType(1.0f), false);
      return true;
    }
    if (*p != ':' || p + 1 == te || !isdigitchars(p[1])) return false;
    *idx = v;
    *val = StrToFloat(p + 1, te, nullptr);
    out->PushFeature(v, static_cast<DType>(*val), true);
    return true;
  }

  /*! \brief parse one line into out (exposed for tests / the GPU oracle) */
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
    bool first = true;
    while (Base::NextToken(&p, le, &tb, &te)) {
      if (first) {
        first = false;
        if (te - tb >= 4 && std::strncmp(tb, "qid:", 4) == 0) {
          out->SetQid(static_cast<uint64_t>(StrToInt<int64_t>(tb + 4, te, nullptr)));
          continue;
        }
      }
      IndexType idx = 0;
      real_t val = 0.0f;
      if (FastFeature(tb, te, &idx, &val, out)) continue;
      const int rr = ParsePair<IndexType, real_t>(tb, te, &idx, &val, &bad);
      if (rr < 1) continue;
      CHECK(!bad) << "negative feature index in LibSVM token \""
                  << std::string(tb, te - tb) << "\"";
      out->PushFeature(idx, static_cast<DType>(val), rr == 2);
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
  }
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_LIBSVM_PARSER_H_
