/*!
 * \file src/io/line_split.cc
 * \brief LineSplitter (see line_split.h).
 */
#include "./line_split.h"

#include <cstring>

namespace dmlc {
namespace io {

namespace {
inline bool IsEOL(char c) { return c == '\n' || c == '\r'; }
}  // namespace

size_t LineSplitter::SeekRecordBegin(Stream* fi) {
  // read in blocks; count bytes up to and including the first EOL run
  char buf[4096];
  size_t nstep = 0;
  bool seen_eol = false;
  while (true) {
    const size_t n = fi->Read(buf, sizeof(buf));
    if (n == 0) return nstep;
    for (size_t i = 0; i < n; ++i) {
      if (!seen_eol) {
        ++nstep;
        if (IsEOL(buf[i])) seen_eol = true;
      } else {
        if (!IsEOL(buf[i])) return nstep;
        ++nstep;
      }
    }
  }
}

const char* LineSplitter::FindLastRecordBegin(const char* begin, const char* end) {
  CHECK(begin != end);
  for (const char* p = end - 1; p != begin; --p) {
    if (IsEOL(*p)) return p + 1;
  }
  return begin;
}

bool LineSplitter::ExtractNextRecord(Blob* out_rec, Chunk* chunk) {
  if (chunk->begin == chunk->end) return false;
  char* p = static_cast<char*>(std::memchr(chunk->begin, '\n', chunk->end - chunk->begin));
  // honour '\r' line ends too
  char* r = static_cast<char*>(
      std::memchr(chunk->begin, '\r', (p == nullptr ? chunk->end : p) - chunk->begin));
  if (r != nullptr) p = r;
  if (p == nullptr) p = chunk->end;
  while (p != chunk->end && IsEOL(*p)) ++p;
  if (p == chunk->end) {
    *p = '\0';
  } else {
    *(p - 1) = '\0';
  }
  out_rec->dptr = chunk->begin;
  out_rec->size = p - chunk->begin;
  chunk->begin = p;
  return true;
}

}  // namespace io
}  // namespace dmlc
