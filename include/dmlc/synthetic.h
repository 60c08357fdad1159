/*!
 * \file dmlc/synthetic.h
 * \brief Deterministic synthetic dataset writers (LibSVM / LibFM / CSV /
 *  RecordIO) used by tests and benchmarks — no network, no real datasets.
 *
 * The defaults reproduce the survey's benchmark shape: binary
 * labels, 20-60 non-zeros per row with sorted random indices below
 * `num_features`, 6-decimal values (~640 bytes per LibSVM line).  Row r is
 * generated from splitmix64(seed, r) alone, so a dataset split over several
 * files (or written by several processes) is identical to the single-file
 * version.
 */
#ifndef DMLC_SYNTHETIC_H_
#define DMLC_SYNTHETIC_H_

#include <cstdint>
#include <string>

namespace dmlc {
namespace synthetic {

struct Spec {
  /*! \brief libsvm | libfm | csv | recordio */
  std::string format{"libsvm"};
  uint64_t seed{0};
  uint32_t min_nnz{20};
  uint32_t max_nnz{60};
  uint64_t num_features{1000000};
  uint32_t num_fields{32};
  /*! \brief CSV columns (label is column 0) */
  uint32_t csv_columns{29};
  /*! \brief RecordIO payload bytes per record */
  uint32_t record_bytes{512};
  /*! \brief emit `:weight` on the label for every k-th row (0: never) */
  uint32_t weight_every{0};
  /*! \brief emit `qid:` tokens */
  bool qid{false};
  /*!
   * \brief row shape (text formats):
   *  uniform  min_nnz..max_nnz tokens per line, `0.dddddd` values (the
   *           benchmark shape above);
   *  skewed   power-law tokens per line (Pareto, alpha 1.1, 2 .. 4000 tokens:
   *           most lines short, ~0.5 % longer than 8 KiB) and Zipf-like
   *           feature ids (short index digits dominate);
   *  mixed    skewed lines whose values mix `0.dddddd` with `1.5e-3`-style
   *           exponents, 9-12-digit mantissas, integers and valueless binary
   *           features, plus a weight on every 13th label and (LibSVM)
   *           `qid:` on every 17th line.
   */
  std::string shape{"uniform"};
};

/*!
 * \brief write rows [row_begin, row_end) of the dataset to `path`
 * \param nthread generator threads
 * \return bytes written
 */
uint64_t WriteRows(const Spec& spec, const std::string& path, uint64_t row_begin,
                   uint64_t row_end, int nthread);

}  // namespace synthetic
}  // namespace dmlc
#endif  // DMLC_SYNTHETIC_H_
