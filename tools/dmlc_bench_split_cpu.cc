// dmlc_bench_split_cpu: CPU record-layer throughput through the public API
// (InputSplit / RecordIOChunkReader only), so the same file builds against
// this repo's libdmlc and against the reference's sources -- the same-host
// baseline of BASELINE.md's RecordIO rows (reference harness shape:
// /root/reference/test/split_read_test.cc, recordio_test.cc).
//
//   dmlc_bench_split_cpu <uri> <mode> [part=0] [nparts=1] [repeat=3]
//     mode  record   InputSplit(type="recordio")::NextRecord
//           chunk    InputSplit(type="recordio")::NextChunk + RecordIOChunkReader
//                    split over OMP threads (reference src/recordio.cc:101-156)
//           text     InputSplit(type="text")::NextRecord (lines)
//
// Prints one JSON line (best of `repeat`).
#include <dmlc/io.h>
#include <dmlc/recordio.h>
#include <dmlc/timer.h>
#include <omp.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s uri record|chunk|text [part] [nparts] [repeat]\n", argv[0]);
    return 2;
  }
  const std::string uri = argv[1], mode = argv[2];
  const unsigned part = argc > 3 ? std::atoi(argv[3]) : 0;
  const unsigned nparts = argc > 4 ? std::atoi(argv[4]) : 1;
  const int repeat = argc > 5 ? std::atoi(argv[5]) : 3;
  const char* type = mode == "text" ? "text" : "recordio";
  double best = 1e30;
  size_t recs = 0, bytes = 0;
  for (int r = 0; r < repeat; ++r) {
    std::unique_ptr<dmlc::InputSplit> split(dmlc::InputSplit::Create(uri.c_str(), part, nparts, type));
    const double t0 = dmlc::GetTime();
    recs = bytes = 0;
    dmlc::InputSplit::Blob blob;
    if (mode == "chunk") {
      const int nt = omp_get_max_threads();
      while (split->NextChunk(&blob)) {
        std::vector<size_t> n(nt, 0), b(nt, 0);
#pragma omp parallel num_threads(nt)
        {
          const int t = omp_get_thread_num();
          dmlc::RecordIOChunkReader rd(blob, t, nt);
          dmlc::InputSplit::Blob rec;
          while (rd.NextRecord(&rec)) {
            n[t] += 1;
            b[t] += rec.size;
          }
        }
        for (int t = 0; t < nt; ++t) {
          recs += n[t];
          bytes += b[t];
        }
      }
    } else {
      while (split->NextRecord(&blob)) {
        recs += 1;
        bytes += blob.size;
      }
    }
    best = std::min(best, dmlc::GetTime() - t0);
  }
  std::printf("{\"uri\": \"%s\", \"mode\": \"%s\", \"threads\": %d, \"records\": %zu, "
              "\"payload_bytes\": %zu, \"sec\": %.4f, \"records_per_sec\": %.1f, \"MBps\": %.1f}\n",
              uri.c_str(), mode.c_str(), omp_get_max_threads(), recs, bytes, best, recs / best,
              bytes / best / 1e6);
  return 0;
}
