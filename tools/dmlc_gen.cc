// dmlc_gen: deterministic synthetic datasets of the benchmark shapes
// (LibSVM 20-60 nnz/row, LibFM, CSV 29 columns, RecordIO 512 B).
//
//   dmlc_gen <format> <rows> <out_prefix> [parts=1] [seed=0] [threads=8] [shape=uniform]
//
// shape: uniform | skewed | mixed (dmlc/synthetic.h)
//
// Writes <out_prefix>-<k>.<format> for k < parts; rows are split evenly and
// the same (format, rows, seed) always produces the same bytes.
#include <dmlc/logging.h>
#include <dmlc/synthetic.h>
#include <dmlc/timer.h>

#include <cstdio>
#include <cstdlib>
#include <string>

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr,
                 "usage: %s libsvm|libfm|csv|recordio rows out_prefix [parts] [seed] [threads] "
                 "[uniform|skewed|mixed]\n",
                 argv[0]);
    return 2;
  }
  dmlc::synthetic::Spec spec;
  spec.format = argv[1];
  uint64_t rows = std::strtoull(argv[2], nullptr, 10);
  std::string prefix = argv[3];
  unsigned parts = argc > 4 ? std::atoi(argv[4]) : 1;
  spec.seed = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 0;
  int threads = argc > 6 ? std::atoi(argv[6]) : 8;
  if (argc > 7) spec.shape = argv[7];
  CHECK_GT(parts, 0U);
  double t0 = dmlc::GetTime();
  uint64_t bytes = 0, per = (rows + parts - 1) / parts;
  for (unsigned k = 0; k < parts; ++k) {
    uint64_t b = k * per, e = std::min<uint64_t>(rows, b + per);
    std::string ext = spec.format == "recordio" ? "rec" : spec.format;
    std::string path = prefix + "-" + std::to_string(k) + "." + ext;
    bytes += dmlc::synthetic::WriteRows(spec, path, b, e, threads);
  }
  double dt = dmlc::GetTime() - t0;
  std::printf("wrote %llu rows, %.1f MB in %u part(s), %.2f s (%.0f MB/s)\n",
              static_cast<unsigned long long>(rows), bytes / 1e6, parts, dt, bytes / 1e6 / dt);
  return 0;
}
