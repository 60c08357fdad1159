// L3/L4 unit tests: RecordIO with injected magic words (reference
// test/recordio_test.cc logic), sharded InputSplit completeness and
// BeforeFirst replay (test/split_repeat_read_test.cc), memory streams and
// the fast number parser vs libc (test/strtonum_test.cc).
#include <dmlc/io.h>
#include <dmlc/memory_io.h>
#include <dmlc/recordio.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../src/data/strtonum.h"
#include "../../src/io/crypto.h"
#include "./testing.h"

TEST(Crypto, Sha256HmacBase64Vectors) {
  namespace c = dmlc::io::crypto;
  EXPECT_EQ(c::Hex(c::Sha256Digest("abc")),
            "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");
  EXPECT_EQ(c::Hex(c::Sha256Digest("")),
            "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");
  std::string million(1000000, 'a');
  EXPECT_EQ(c::Hex(c::Sha256Digest(million)),
            "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0");
  // RFC 4231 test case 2
  EXPECT_EQ(c::Hex(c::HmacSha256("Jefe", "what do ya want for nothing?")),
            "5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843");
  // RFC 4231 test case 6 (key longer than the block)
  EXPECT_EQ(c::Hex(c::HmacSha256(std::string(131, '\xaa'),
                                 "Test Using Larger Than Block-Size Key - Hash Key First")),
            "60e431591ee0b67f0d8a26aacbf5b77f8e0bc6213728c5140546040f0ee37f54");
  EXPECT_EQ(c::Base64Encode("foobar"), "Zm9vYmFy");
  EXPECT_EQ(c::Base64Encode("fooba"), "Zm9vYmE=");
  EXPECT_EQ(c::Base64Decode("Zm9vYg=="), "foob");
  EXPECT_EQ(c::UriEncode("a b/c~"), "a%20b%2Fc~");
  EXPECT_EQ(c::UriEncode("a b/c", false), "a%20b/c");
}

namespace {

std::string TempDir() {
  char tmpl[] = "/tmp/dmlc_cpptest_XXXXXX";
  char* d = mkdtemp(tmpl);
  if (d == nullptr) std::abort();
  return d;
}

std::vector<std::string> RandomRecords(size_t n, uint32_t seed) {
  std::mt19937 rng(seed);
  std::vector<std::string> recs(n);
  const uint32_t magic = dmlc::RecordIOWriter::kMagic;
  for (auto& r : recs) {
    size_t len = rng() % 300;
    r.resize(len);
    for (auto& c : r) c = static_cast<char>(rng());
    // inject aligned and unaligned magic words
    for (size_t k = 0; k + 4 <= len; k += 4 + (rng() % 64)) {
      if (rng() % 3 == 0) std::memcpy(&r[k], &magic, 4);
    }
    if (len >= 8 && rng() % 5 == 0) std::memcpy(&r[len - 5], &magic, 4);
  }
  return recs;
}

}  // namespace

TEST(RecordIO, RoundTripWithInjectedMagic) {
  std::string dir = TempDir();
  std::string path = dir + "/a.rec";
  auto recs = RandomRecords(3000, 7);
  {
    std::unique_ptr<dmlc::Stream> fo(dmlc::Stream::Create(path.c_str(), "w"));
    dmlc::RecordIOWriter w(fo.get());
    for (auto& r : recs) w.WriteRecord(r);
    EXPECT_GT(w.except_counter(), 0U);
  }
  {
    std::unique_ptr<dmlc::Stream> fi(dmlc::Stream::Create(path.c_str(), "r"));
    dmlc::RecordIOReader rd(fi.get());
    std::string s;
    size_t i = 0;
    while (rd.NextRecord(&s)) {
      ASSERT_LT(i, recs.size());
      EXPECT_TRUE(s == recs[i]);
      ++i;
    }
    EXPECT_EQ(i, recs.size());
  }
  // sharded reading covers every record exactly once, in order
  for (unsigned nparts : {1u, 2u, 3u, 7u}) {
    size_t i = 0;
    for (unsigned part = 0; part < nparts; ++part) {
      std::unique_ptr<dmlc::InputSplit> sp(
          dmlc::InputSplit::Create(path.c_str(), part, nparts, "recordio"));
      dmlc::InputSplit::Blob b;
      while (sp->NextRecord(&b)) {
        ASSERT_LT(i, recs.size());
        EXPECT_TRUE(std::string(static_cast<char*>(b.dptr), b.size) == recs[i]);
        ++i;
      }
    }
    EXPECT_EQ(i, recs.size());
  }
  // chunk + RecordIOChunkReader with sub-partitions
  {
    std::unique_ptr<dmlc::InputSplit> sp(dmlc::InputSplit::Create(path.c_str(), 0, 1, "recordio"));
    dmlc::InputSplit::Blob chunk;
    size_t total = 0;
    while (sp->NextChunk(&chunk)) {
      for (unsigned k = 0; k < 3; ++k) {
        dmlc::RecordIOChunkReader cr(chunk, k, 3);
        dmlc::InputSplit::Blob r;
        while (cr.NextRecord(&r)) ++total;
      }
    }
    EXPECT_EQ(total, recs.size());
  }
  std::remove(path.c_str());
  rmdir(dir.c_str());
}

TEST(InputSplit, TextShardsDisjointCompleteAndReplayable) {
  std::string dir = TempDir();
  std::vector<std::string> lines;
  for (int f = 0; f < 4; ++f) {
    std::string p = dir + "/part-" + std::to_string(f) + ".txt";
    FILE* fp = std::fopen(p.c_str(), "w");
    int n = 100 + 37 * f;
    for (int i = 0; i < n; ++i) {
      std::string l = "f" + std::to_string(f) + "_line" + std::to_string(i);
      lines.push_back(l);
      // last file without trailing newline, some CRLF line ends
      bool last = (f == 3 && i == n - 1);
      std::fprintf(fp, "%s%s", l.c_str(), last ? "" : (i % 7 == 0 ? "\r\n" : "\n"));
    }
    std::fclose(fp);
  }
  for (unsigned nparts : {1u, 2u, 5u, 16u}) {
    std::vector<std::string> got;
    for (unsigned part = 0; part < nparts; ++part) {
      std::unique_ptr<dmlc::InputSplit> sp(
          dmlc::InputSplit::Create(dir.c_str(), part, nparts, "text"));
      std::vector<std::string> first;
      for (int epoch = 0; epoch < 2; ++epoch) {
        std::vector<std::string> mine;
        dmlc::InputSplit::Blob b;
        while (sp->NextRecord(&b)) {
          std::string s(static_cast<char*>(b.dptr), b.size);
          while (!s.empty() && (s.back() == '\n' || s.back() == '\r' || s.back() == '\0'))
            s.pop_back();
          mine.push_back(s);
        }
        if (epoch == 0) {
          first = mine;
          got.insert(got.end(), mine.begin(), mine.end());
        } else {
          EXPECT_TRUE(mine == first);  // BeforeFirst replay is identical
        }
        sp->BeforeFirst();
      }
    }
    ASSERT_EQ(got.size(), lines.size());
    EXPECT_TRUE(got == lines);
  }
  for (int f = 0; f < 4; ++f) std::remove((dir + "/part-" + std::to_string(f) + ".txt").c_str());
  rmdir(dir.c_str());
}

TEST(MemoryIO, FixedAndStringStreams) {
  char buf[16];
  dmlc::MemoryFixedSizeStream fs(buf, sizeof(buf));
  uint64_t a = 0x1122334455667788ULL;
  fs.Write(&a, 8);
  EXPECT_EQ(fs.Tell(), 8U);
  fs.Seek(0);
  uint64_t b = 0;
  EXPECT_EQ(fs.Read(&b, 8), 8U);
  EXPECT_EQ(a, b);
  EXPECT_THROW(fs.Write(buf, 32), dmlc::Error);
  std::string s;
  dmlc::MemoryStringStream ss(&s);
  ss.Write(std::string("hello"));
  ss.Seek(0);
  std::string back;
  EXPECT_TRUE(ss.Read(&back));
  EXPECT_EQ(back, "hello");
  dmlc::ostream os(&ss);
  os << " world " << 42;
  os.flush();
  EXPECT_TRUE(s.find("world 42") != std::string::npos);
}

TEST(StrToNum, MatchesLibcOnSimpleInputs) {
  const char* floats[] = {"0",     "1",      "-1.5",  "3.25e2", "1e-5", "+7.",
                          "0.125", "123456", "1E+10", "-0.0",   ".5",   "2.5e-3"};
  for (const char* f : floats) {
    const char* end = nullptr;
    float v = dmlc::data::StrToFloat(f, f + std::strlen(f), &end);
    float ref = std::strtof(f, nullptr);
    EXPECT_NEAR(v, ref, std::fabs(ref) * 1e-6f + 1e-30f);
    EXPECT_TRUE(end == f + std::strlen(f));
  }
  const char* ints[] = {"0", "17", "-42", "4294967295", "+9"};
  for (const char* s : ints) {
    const char* end = nullptr;
    int64_t v = dmlc::data::StrToInt<int64_t>(s, s + std::strlen(s), &end);
    EXPECT_EQ(v, std::strtoll(s, nullptr, 10));
  }
  const char* u = "18446744073709551615";
  const char* end = nullptr;
  bool neg = false;
  uint64_t uv = dmlc::data::StrToUInt<uint64_t, uint64_t>(u, u + std::strlen(u), &end, &neg);
  EXPECT_EQ(uv, 18446744073709551615ULL);
  EXPECT_FALSE(neg);
}
