/*!
 * \file src/synthetic.cc
 * \brief Parallel deterministic synthetic data writer (see dmlc/synthetic.h).
 */
#include <dmlc/logging.h>
#include <dmlc/recordio.h>
#include <dmlc/memory_io.h>
#include <dmlc/synthetic.h>

#include <algorithm>
#include <cmath>
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

/*! \brief "0." + k digits (k <= 18) */
inline char* PutFracK(char* p, uint64_t r, int k) {
  *p++ = '0';
  *p++ = '.';
  for (int i = 0; i < k; ++i) {
    *p++ = static_cast<char>('0' + r % 10);
    r /= 10;
  }
  return p;
}

/*! \brief a value of the mixed shape: mostly 0.dddddd, else another spelling */
inline char* PutMixedValue(char* p, uint64_t r) {
  switch ((r >> 40) % 16) {
    case 10:
    case 11: {  // d.ddde-d  (exponent: the generic strtonum path)
      *p++ = static_cast<char>('1' + r % 9);
      *p++ = '.';
      for (int i = 0; i < 3; ++i) *p++ = static_cast<char>('0' + (r >> (4 * i + 8)) % 10);
      *p++ = 'e';
      *p++ = '-';
      *p++ = static_cast<char>('1' + (r >> 24) % 5);
      return p;
    }
    case 12:  // 9 - 12 fraction digits
      return PutFracK(p, r, 9 + static_cast<int>((r >> 20) % 4));
    case 15:  // integer value
      return PutU64(p, 1 + r % 9);
    default:
      return PutFrac6(p, r);
  }
}

/*! \brief tokens of a skewed line: Pareto(alpha = 1.1, x_min = 2), capped */
inline uint32_t ParetoNnz(uint64_t r) {
  const double u = (static_cast<double>(r >> 11) + 1.0) * (1.0 / 9007199254740992.0);
  const double x = 2.0 * std::pow(u, -1.0 / 1.1);
  return static_cast<uint32_t>(std::min(x, 4000.0));
}

/*! \brief Zipf-like feature id: log-uniform over [1, num_features) */
inline uint64_t SkewedIndex(uint64_t r, uint64_t num_features) {
  const double u = static_cast<double>(r >> 11) * (1.0 / 9007199254740992.0);
  const uint64_t v = static_cast<uint64_t>(std::exp(u * std::log(static_cast<double>(num_features))));
  return std::min<uint64_t>(v, num_features - 1);
}

/*! \brief longest line TextRow can write for this spec */
size_t MaxRowBytes(const Spec& s) {
  if (s.format == "csv") return 16 + 12 * s.csv_columns;
  const size_t tokens = s.shape == "uniform" ? s.max_nnz : 4000;
  return 96 + tokens * 56;
}

/*! \brief one text row into p (MaxRowBytes(s) of room); returns end */
char* TextRow(const Spec& s, uint64_t row, char* p, std::vector<uint64_t>* idx) {
  uint64_t st = s.seed * 0x100000001b3ull + row * 0x9e3779b97f4a7c15ull + 1;
  const uint64_t r0 = SplitMix(&st);
  const bool skewed = s.shape == "skewed" || s.shape == "mixed";
  const bool mixed = s.shape == "mixed";
  *p++ = (r0 & 1) ? '1' : '0';
  if ((s.weight_every != 0 && row % s.weight_every == 0) || (mixed && row % 13 == 0)) {
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
  if (s.format == "libsvm" && (s.qid || (mixed && row % 17 == 0))) {
    std::memcpy(p, " qid:", 5);
    p = PutU64(p + 5, row / 16);
  }
  uint32_t nnz;
  if (skewed) {
    nnz = ParetoNnz(SplitMix(&st));
  } else {
    const uint32_t span = s.max_nnz - s.min_nnz + 1;
    nnz = s.min_nnz + static_cast<uint32_t>(SplitMix(&st) % span);
  }
  idx->resize(nnz);
  for (uint32_t i = 0; i < nnz; ++i) {
    const uint64_t r = SplitMix(&st);
    (*idx)[i] = skewed ? SkewedIndex(r, s.num_features) : r % s.num_features;
  }
  std::sort(idx->begin(), idx->end());
  for (uint32_t i = 0; i < nnz; ++i) {
    *p++ = ' ';
    if (s.format == "libfm") {
      p = PutU64(p, (*idx)[i] % s.num_fields);
      *p++ = ':';
    }
    p = PutU64(p, (*idx)[i]);
    const uint64_t r = SplitMix(&st);
    if (mixed) {
      if ((r >> 40) % 16 == 13 || (r >> 40) % 16 == 14) continue;  // valueless binary feature
      *p++ = ':';
      p = PutMixedValue(p, r);
    } else {
      *p++ = ':';
      p = PutFrac6(p, r);
    }
  }
  *p++ = '\n';
  return p;
}
}  // namespace

uint64_t WriteRows(const Spec& spec, const std::string& path, uint64_t row_begin,
                   uint64_t row_end, int nthread) {
  CHECK(spec.min_nnz <= spec.max_nnz) << "min_nnz > max_nnz";
  CHECK(spec.shape == "uniform" || spec.shape == "skewed" || spec.shape == "mixed")
      << "shape must be uniform, skewed or mixed, not " << spec.shape;
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
          const size_t room = MaxRowBytes(spec);
          size_t used = 0;
          for (uint64_t r = b; r < e; ++r) {
            if (buf.size() < used + room) buf.resize(std::max(2 * buf.size(), used + room));
            used = TextRow(spec, r, &buf[0] + used, &idx) - &buf[0];
          }
          buf.resize(used);
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
