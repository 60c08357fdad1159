/*!
 * \file tools/dmlc_bench_read.cc
 * \brief Host stage of the GPU ring alone: ShardReader::Fill of one
 *  partition into a page-locked-sized host buffer, timed per epoch.  Measures
 *  the remote ingest path (s3:// / http:// ranged GETs, native receive or
 *  libcurl) without the GPU, so loopback throughput can be priced by parts.
 *
 * usage: dmlc_bench_read URI [threads=16] [chunk_mb=64] [epochs=3] [text|recordio]
 * prints one JSON line.
 */
#include <dmlc/timer.h>
#include <sys/mman.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "io/filesys.h"
#include "io/http.h"
#include "io/line_split.h"
#include "io/recordio_split.h"
#include "io/shard_reader.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s URI [threads] [chunk_mb] [epochs] [text|recordio]\n", argv[0]);
    return 1;
  }
  const std::string uri = argv[1];
  const int threads = argc > 2 ? std::atoi(argv[2]) : 16;
  const size_t chunk = (argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 64) << 20;
  const int epochs = argc > 4 ? std::atoi(argv[4]) : 3;
  const std::string type = argc > 5 ? argv[5] : "text";
  using namespace dmlc::io;
  URI path(uri.c_str());
  FileSystem* fs = FileSystem::GetInstance(path);
  std::unique_ptr<InputSplitBase> split;
  if (type == "text") {
    split.reset(new LineSplitter(fs, uri.c_str(), 0, 1));
  } else {
    split.reset(new RecordIOSplitter(fs, uri.c_str(), 0, 1));
  }
  ShardReader reader(split.get(), threads);
  size_t cap = chunk;
  // anonymous, pre-faulted and locked like a pinned ring slot
  char* buf = static_cast<char*>(::mmap(nullptr, cap, PROT_READ | PROT_WRITE,
                                        MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
  double best = 1e30, total = 0;
  size_t bytes = 0;
  for (int e = 0; e <= epochs; ++e) {  // epoch 0 is the warm one
    reader.Reset();
    const double t0 = dmlc::GetTime();
    size_t got = 0;
    for (;;) {
      size_t n = reader.Fill(buf, cap);
      while (n == ShardReader::kNeedMore) {
        ::munmap(buf, cap);
        cap = reader.NeedCapacity();
        buf = static_cast<char*>(::mmap(nullptr, cap, PROT_READ | PROT_WRITE,
                                        MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
        n = reader.Fill(buf, cap);
      }
      if (n == 0) break;
      got += n;
    }
    const double dt = dmlc::GetTime() - t0;
    if (e > 0) {
      total += dt;
      if (dt < best) best = dt;
    }
    bytes = got;
  }
  std::printf(
      "{\"uri\": \"%s\", \"threads\": %d, \"chunk_mb\": %zu, \"bytes\": %zu, \"epochs\": %d, "
      "\"sec_per_epoch\": %.4f, \"GBps\": %.3f, \"best_GBps\": %.3f, \"native_gets\": %llu, "
      "\"native_fallbacks\": %llu}\n",
      uri.c_str(), threads, chunk >> 20, bytes, epochs, total / epochs,
      bytes * epochs / total / 1e9, bytes / best / 1e9,
      static_cast<unsigned long long>(Http::NativeGets()),
      static_cast<unsigned long long>(Http::NativeFallbacks()));
  ::munmap(buf, cap);
  return 0;
}
