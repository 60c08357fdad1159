/*!
 * \file src/data/csv_parser.h
 * \brief Dense CSV -> CSR (every column is a feature; one may be the label).
 *
 * Parity: reference `src/data/csv_parser.h` — CSVParserParam {format="csv",
 * label_column=-1} (:22-32); per line each ','-separated field is parsed with
 * strtof, the label column is removed from the features and the remaining
 * columns are numbered 0,1,2,... (:64-104); label 0 when there is no label
 * column.  Extensions: `delimiter` (single character, default ',') and
 * `weight_column` (-1 = none).  Registered for uint32 AND uint64 indices and
 * multi-threaded.
 */
#ifndef DMLC_DATA_CSV_PARSER_H_
#define DMLC_DATA_CSV_PARSER_H_

#include <dmlc/parameter.h>

#include <map>
#include <string>

#include "./text_parser.h"

namespace dmlc {
namespace data {

struct CSVParserParam : public Parameter<CSVParserParam> {
  std::string format;
  int label_column;
  int weight_column;
  std::string delimiter;
  int nthread;
  DMLC_DECLARE_PARAMETER(CSVParserParam) {
    DMLC_DECLARE_FIELD(format).set_default("csv").describe("File format.");
    DMLC_DECLARE_FIELD(label_column).set_default(-1).describe(
        "Column index that will put into label.");
    DMLC_DECLARE_FIELD(weight_column).set_default(-1).describe(
        "Column index that will put into instance weights (-1: none).");
    DMLC_DECLARE_FIELD(delimiter).set_default(",").describe("Single-character delimiter.");
    DMLC_DECLARE_FIELD(nthread).set_default(0).describe("Parser threads (0: all).");
  }
};

template <typename IndexType, typename DType = real_t>
class CSVParser : public TextParserBase<IndexType, DType> {
 public:
  using Base = TextParserBase<IndexType, DType>;
  CSVParser(InputSplit* source, const std::map<std::string, std::string>& args, int nthread)
      : Base(source, nthread) {
    param_.Init(args);
    CHECK_EQ(param_.format, "csv");
    CHECK_EQ(param_.delimiter.size(), 1U) << "CSV delimiter must be one character";
    CHECK(param_.label_column < 0 || param_.label_column != param_.weight_column)
        << "label_column and weight_column must differ";
  }

  static inline void ParseLine(const char* lb, const char* le, char delim, int label_col,
                               int weight_col, RowBlockContainer<IndexType, DType>* out) {
    const char* p = lb;
    int column = 0;
    IndexType idx = 0;
    real_t label = 0.0f, weight = 1.0f;
    bool has_weight = false;
    // A delimiter that no number can contain (not a digit, sign, '.', 'e' or
    // blank) ends the field's number by itself: the number is parsed against
    // the line end and the field ends right where it stopped when a delimiter
    // (or the line end) follows -- no memchr per field.  Otherwise (junk
    // after the number) the delimiter is searched from there; every byte the
    // parse consumed precedes it, so the value equals the reference's
    // StrToFloat over [field start, delimiter) (reference :64-104).
    const bool direct = !isdigitchars(delim) && !isspace(delim);
    while (true) {
      const char* q = p;
      const char* fe;
      real_t v;
      if (direct) {
        while (q != le && isspace(*q)) ++q;
        const char* e;
        v = StrToFloat(q, le, &e);
        if (e == le || *e == delim) {
          fe = e;
        } else {
          fe = static_cast<const char*>(std::memchr(e, delim, le - e));
          if (fe == nullptr) fe = le;
        }
      } else {
        fe = static_cast<const char*>(std::memchr(p, delim, le - p));
        if (fe == nullptr) fe = le;
        while (q != fe && isspace(*q)) ++q;
        v = StrToFloat(q, fe, nullptr);
      }
      if (column == label_col) {
        label = v;
      } else if (column == weight_col) {
        weight = v;
        has_weight = true;
      } else {
        out->index.push_back(idx);
        out->value.push_back(static_cast<DType>(v));
        if (idx > out->max_index) out->max_index = idx;
        ++idx;
      }
      ++column;
      if (fe == le) break;
      p = fe + 1;
      if (p == le) break;  // a trailing delimiter opens no empty field (reference :83-96)
    }
    out->label.push_back(static_cast<DType>(label));
    // a weight column gives every row a weight (1.0 when the row is short)
    if (weight_col >= 0) out->weight.push_back(has_weight ? weight : 1.0f);
    out->offset.push_back(out->index.size());
  }

 protected:
  void ParseBlock(const char* begin, const char* end,
                  RowBlockContainer<IndexType, DType>* out) override {
    out->Clear();
    // one up-front reservation per block (a field is at least 2 bytes with its
    // delimiter); push_back's geometric growth covers any underestimate
    const size_t est = static_cast<size_t>(end - begin) / 4;
    out->index.reserve(est);
    out->value.reserve(est);
    const char delim = param_.delimiter[0];
    const int lc = param_.label_column, wc = param_.weight_column;
    Base::ForEachLine(begin, end, [&](const char* lb, const char* le) {
      ParseLine(lb, le, delim, lc, wc, out);
    });
  }

 private:
  CSVParserParam param_;
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_CSV_PARSER_H_
