/*!
 * \file src/synthetic.cc
 * \brief Parallel deterministic synthetic data writer (see dmlc/synthetic.h).
 */
#include <dmlc/logging.h>
#include <dmlc/recordio.h>
#include <dmlc/memory_io.h>
#include <dmlc/synthetic.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

namespace dmlc {
namespace synthetic {

namespace {
inline uint64_t SplitMix(uint64_t* x) {
  uint64_t z = (*x += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

inline char* PutU64(char* p, uint64_t v) {
  char tmp[24];
  int n = 0;
  do {
    tmp[n++] = static_cast<char>('0' + v % 10);
    v /= 10;
  } while (v != 0);
  while (n > 0) *p++ = tmp[--n];
  return p;
}

/*! \brief "0.dddddd" from a 20-bit random number */
inline char* PutFrac6(char* p, uint64_t r) {
  const uint64_t v = r % 1000000;
  *p++ = '0';
  *p++ = '.';
  char digits[6];
  uint64_t x = v;
  for (int i = 5; i >= 0; --i) {
    digits[i] = static_cast<char>('0' + x % 10);
    x /= 10;
  }
  std::memcpy(p, digits, 6);
  return p + 6;
}

/*! \brief one text row into p (buffer large enough); returns end */
char* TextRow(const Spec& s, uint64_t row, char* p, std::vector<uint64_t>* idx) {
  uint64_t st = s.seed * 0x100000001b3ull + row * 0x9e3779b97f4a7c15ull + 1;
  const uint64_t r0 = SplitMix(&st);
  *p++ = (r0 & 1) ? '1' : '0';
  if (s.weight_every != 0 && row % s.weight_every == 0) {
    *p++ = ':';
    p = PutFrac6(p, SplitMix(&st));
  }
  if (s.format == "csv") {
    for (uint32_t c = 1; c < s.csv_columns; ++c) {
      *p++ = ',';
      p = PutFrac6(p, SplitMix(&st));
    }
    *p++ = '\n';
    return p;
  }
  if (s.qid && s.format == "libsvm") {
    std::memcpy(p, " qid:", 5);
    p = PutU64(p + 5, row / 16);
  }
  const uint32_t span = s.max_nnz - s.min_nnz + 1;
  const uint32_t nnz = s.min_nnz + static_cast<uint32_t>(SplitMix(&st) % span);
  idx->resize(nnz);
  for (uint32_t i = 0; i < nnz; ++i) (*idx)[i] = SplitMix(&st) % s.num_features;
  std::sort(idx->begin(), idx->end());
  for (uint32_t i = 0; i < nnz; ++i) {
    *p++ = ' ';
    if (s.format == "libfm") {
      p = PutU64(p, (*idx)[i] % s.num_fields);
      *p++ = ':';
    }
    p = PutU64(p, (*idx)[i]);
    *p++ = ':';
    p = PutFrac6(p, SplitMix(&st));
  }
  *p++ = '\n';
  return p;
}
}  // namespace

uint64_t WriteRows(const Spec& spec, const std::string& path, uint64_t row_begin,
                   uint64_t row_end, int nthread) {
  CHECK(spec.min_nnz <= spec.max_nnz) << "min_nnz > max_nnz";
  std::unique_ptr<Stream> fo(Stream::Create(path.c_str(), "w"));
  nthread = std::max(1, nthread);
  const uint64_t kBlockRows = 16384;
  uint64_t total = 0;
  const bool recordio = spec.format == "recordio";
  // generate blocks of rows in parallel, write them in order
  for (uint64_t base = row_begin; base < row_end; base += kBlockRows * nthread) {
    std::vector<std::string> out(nthread);
    std::vector<std::thread> workers;
    for (int t = 0; t < nthread; ++t) {
      workers.emplace_back([&, t]() {
        const uint64_t b = base + t * kBlockRows;
        const uint64_t e = std::min(row_end, b + kBlockRows);
        if (b >= e) return;
        std::string& buf = out[t];
        std::vector<uint64_t> idx;
        if (recordio) {
          MemoryStringStream ms(&buf);
          RecordIOWriter w(&ms);
          std::string payload(spec.record_bytes, '\0');
          for (uint64_t r = b; r < e; ++r) {
            uint64_t st = spec.seed * 0x100000001b3ull + r * 0x9e3779b97f4a7c15ull + 7;
            for (size_t i = 0; i + 8 <= payload.size(); i += 8) {
              const uint64_t v = SplitMix(&st);
              std::memcpy(&payload[i], &v, 8);
            }
            // plant an aligned magic word in every 64th record (escape path)
            if (r % 64 == 0 && payload.size() >= 8) {
              const uint32_t m = RecordIOWriter::kMagic;
              std::memcpy(&payload[4], &m, 4);
            }
            w.WriteRecord(payload.data(), payload.size());
          }
        } else {
          const size_t per_row = spec.format == "csv"
                                     ? 16 + 12 * spec.csv_columns
                                     : 64 + static_cast<size_t>(spec.max_nnz) * 48;
          buf.resize((e - b) * per_row);
          char* p = &buf[0];
          for (uint64_t r = b; r < e; ++r) p = TextRow(spec, r, p, &idx);
          buf.resize(p - &buf[0]);
        }
      });
    }
    for (auto& w : workers) w.join();
    for (auto& s : out) {
      if (!s.empty()) fo->Write(s.data(), s.size());
      total += s.size();
    }
  }
  return total;
}

}  // namespace synthetic
}  // namespace dmlc
