// Reference behaviours of the InputSplit family pinned against independent
// oracles (std::mt19937 + std::shuffle, plain sequential reads):
//   * InputSplitShuffle visiting order, seed 666 + part + nparts + nshuffle + seed
//     (reference include/dmlc/input_split_shuffle.h:100-119, reshuffle :24-33)
//   * indexed_recordio shuffle, std::mt19937(111 + seed), a fresh permutation of
//     the part's records at every BeforeFirst (src/io/indexed_recordio_split.cc:158-232)
//   * `uri#cache`: later epochs and later splits replay an existing cache file
//     (src/io/cached_input_split.h:148-188)
#include <dmlc/input_split_shuffle.h>
#include <dmlc/io.h>
#include <dmlc/recordio.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <memory>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "./testing.h"

namespace {

std::string MakeDir() {
  char tmpl[] = "/tmp/dmlc_split_XXXXXX";
  char* d = mkdtemp(tmpl);
  return d != nullptr ? std::string(d) : std::string("/tmp");
}

std::string Strip(const dmlc::InputSplit::Blob& b) {
  std::string s(static_cast<const char*>(b.dptr), b.size);
  while (!s.empty() && (s.back() == '\n' || s.back() == '\r' || s.back() == '\0')) s.pop_back();
  return s;
}

std::vector<std::string> ReadAll(dmlc::InputSplit* sp) {
  std::vector<std::string> out;
  dmlc::InputSplit::Blob b;
  while (sp->NextRecord(&b)) out.push_back(Strip(b));
  return out;
}

std::vector<std::string> ReadPart(const std::string& uri, unsigned part, unsigned nparts,
                                  const char* type) {
  std::unique_ptr<dmlc::InputSplit> sp(dmlc::InputSplit::Create(uri.c_str(), part, nparts, type));
  return ReadAll(sp.get());
}

std::string WriteLines(const std::string& dir, int n) {
  std::string p = dir + "/lines.txt";
  FILE* fp = std::fopen(p.c_str(), "w");
  for (int i = 0; i < n; ++i) std::fprintf(fp, "line-%d-%s\n", i, std::string(i % 23, 'x').c_str());
  std::fclose(fp);
  return p;
}

}  // namespace

TEST(InputSplitShuffle, VisitingOrderMatchesReferenceSeeds) {
  const std::string dir = MakeDir();
  const std::string path = WriteLines(dir, 2000);
  const unsigned nshuf = 5;
  const int seed = 3;
  for (unsigned nparts : {1u, 2u}) {
    for (unsigned part = 0; part < nparts; ++part) {
      std::unique_ptr<dmlc::InputSplit> sp(
          dmlc::InputSplitShuffle::Create(path.c_str(), part, nparts, "text", nshuf, seed));
      // oracle: the reference's RNG and shuffle, applied to sub-shard ids
      std::mt19937 rnd(666 + part + nparts + nshuf + seed);
      std::vector<unsigned> order(nshuf);
      std::iota(order.begin(), order.end(), 0u);
      std::shuffle(order.begin(), order.end(), rnd);
      for (int epoch = 0; epoch < 3; ++epoch) {
        if (epoch > 0) {
          std::shuffle(order.begin(), order.end(), rnd);
          sp->BeforeFirst();
        }
        std::vector<std::string> expect;
        for (unsigned k : order) {
          auto sub = ReadPart(path, part * nshuf + k, nparts * nshuf, "text");
          expect.insert(expect.end(), sub.begin(), sub.end());
        }
        auto got = ReadAll(sp.get());
        ASSERT_EQ(got.size(), expect.size());
        EXPECT_TRUE(got == expect);
      }
    }
  }
  std::remove(path.c_str());
  rmdir(dir.c_str());
}

TEST(IndexedRecordIO, ShufflePermutationMatchesReference) {
  const std::string dir = MakeDir();
  const std::string rec = dir + "/d.rec", idx = dir + "/d.idx";
  const size_t n = 503;
  std::vector<std::string> recs;
  {
    std::unique_ptr<dmlc::Stream> fo(dmlc::Stream::Create(rec.c_str(), "w"));
    dmlc::RecordIOWriter w(fo.get());
    std::ofstream index(idx);
    for (size_t i = 0; i < n; ++i) {
      recs.push_back("record-" + std::to_string(i) + std::string(i % 13, 'r'));
      index << i << "\t" << w.Tell() << "\n";
      w.WriteRecord(recs.back());
    }
  }
  const int seed = 7;
  const size_t batch = 9;
  for (unsigned nparts : {1u, 3u}) {
    const size_t step = (n + nparts - 1) / nparts;
    for (unsigned part = 0; part < nparts; ++part) {
      std::unique_ptr<dmlc::InputSplit> sp(dmlc::InputSplit::Create(
          rec.c_str(), idx.c_str(), part, nparts, "indexed_recordio", true, seed, batch));
      const size_t begin = part * step, end = std::min(n, begin + step);
      std::mt19937 rnd(111 + seed);
      for (int epoch = 0; epoch < 3; ++epoch) {
        // the constructor's ResetPartition shuffles once; every BeforeFirst
        // shuffles a fresh identity permutation with the continuing RNG
        std::vector<size_t> perm(end - begin);
        std::iota(perm.begin(), perm.end(), begin);
        std::shuffle(perm.begin(), perm.end(), rnd);
        if (epoch > 0) sp->BeforeFirst();
        std::vector<std::string> got;
        dmlc::InputSplit::Blob chunk;
        while (sp->NextChunk(&chunk)) {
          dmlc::RecordIOChunkReader rd(chunk);
          dmlc::InputSplit::Blob r;
          size_t in_batch = 0;
          while (rd.NextRecord(&r)) {
            got.emplace_back(static_cast<const char*>(r.dptr), r.size);
            ++in_batch;
          }
          EXPECT_LE(in_batch, batch);
        }
        ASSERT_EQ(got.size(), perm.size());
        for (size_t i = 0; i < perm.size(); ++i) EXPECT_TRUE(got[i] == recs[perm[i]]);
      }
    }
  }
  std::remove(rec.c_str());
  std::remove(idx.c_str());
  rmdir(dir.c_str());
}

TEST(CachedInputSplit, ReplaysAnExistingCacheFile) {
  const std::string dir = MakeDir();
  const std::string path = WriteLines(dir, 3000);
  const std::string cache = dir + "/split.cache";
  const auto plain = ReadPart(path, 0, 1, "text");
  {
    std::unique_ptr<dmlc::InputSplit> sp(
        dmlc::InputSplit::Create((path + "#" + cache).c_str(), 0, 1, "text"));
    for (int epoch = 0; epoch < 2; ++epoch) {
      if (epoch > 0) sp->BeforeFirst();
      auto got = ReadAll(sp.get());
      EXPECT_TRUE(got == plain);
    }
  }
  std::ifstream c(cache, std::ios::binary | std::ios::ate);
  EXPECT_TRUE(c.good() && c.tellg() > 0);
  // an existing cache is replayed as is: rewrite the source with other
  // content, a new split over the same cache still returns the cached records
  // (the source must still exist: the base split extracts records)
  WriteLines(dir, 10);
  {
    std::unique_ptr<dmlc::InputSplit> sp(
        dmlc::InputSplit::Create((path + "#" + cache).c_str(), 0, 1, "text"));
    auto got = ReadAll(sp.get());
    EXPECT_TRUE(got == plain);
  }
  std::remove(cache.c_str());
  std::remove(path.c_str());
  rmdir(dir.c_str());
}
