// dmlc_bench_cpu: CPU parser throughput through the public API, the same
// harness shape the reference baseline was measured with (SURVEY §6.2:
// Parser<uint32_t>::Create(uri, part, nparts, format) + Next() loop).
//
//   dmlc_bench_cpu <uri> [format=libsvm] [part=0] [nparts=1] [repeat=3]
//
// OMP_NUM_THREADS / ?nthread= control the parse team.  Prints one JSON line.
#include <dmlc/data.h>
#include <dmlc/logging.h>
#include <dmlc/timer.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s uri [format] [part] [nparts] [repeat]\n", argv[0]);
    return 2;
  }
  std::string uri = argv[1];
  std::string fmt = argc > 2 ? argv[2] : "libsvm";
  unsigned part = argc > 3 ? std::atoi(argv[3]) : 0;
  unsigned nparts = argc > 4 ? std::atoi(argv[4]) : 1;
  int repeat = argc > 5 ? std::atoi(argv[5]) : 3;
  double best = 1e30;
  size_t rows = 0, nnz = 0, bytes = 0;
  for (int r = 0; r < repeat; ++r) {
    double t0 = dmlc::GetTime();
    std::unique_ptr<dmlc::Parser<uint32_t>> p(
        dmlc::Parser<uint32_t>::Create(uri.c_str(), part, nparts, fmt.c_str()));
    rows = nnz = 0;
    while (p->Next()) {
      const auto& b = p->Value();
      rows += b.size;
      nnz += b.offset[b.size] - b.offset[0];
    }
    bytes = p->BytesRead();
    best = std::min(best, dmlc::GetTime() - t0);
  }
  std::printf("{\"uri\": \"%s\", \"format\": \"%s\", \"rows\": %zu, \"nnz\": %zu, "
              "\"sec\": %.4f, \"rows_per_sec\": %.1f, \"MBps\": %.1f}\n",
              uri.c_str(), fmt.c_str(), rows, nnz, best, rows / best, bytes / best / 1e6);
  return 0;
}
