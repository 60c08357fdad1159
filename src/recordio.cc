/*!
 * \file src/recordio.cc
 * \brief RecordIO writer / reader / chunk reader.
 * Parity: reference `src/recordio.cc:11-156` (format in dmlc/recordio.h).
 */
#include <dmlc/recordio.h>

#include <algorithm>

namespace dmlc {

namespace {
/*! \brief first aligned record head (magic + cflag 0/1) in [begin, end) */
inline char* NextHead(char* begin, char* end) {
  CHECK_EQ(reinterpret_cast<uintptr_t>(begin) & 3U, 0U);
  CHECK_EQ(reinterpret_cast<uintptr_t>(end) & 3U, 0U);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(begin);
  const uint32_t* pend = reinterpret_cast<const uint32_t*>(end);
  for (; p + 1 < pend; ++p) {
    if (p[0] != RecordIOWriter::kMagic) continue;
    uint32_t cflag = RecordIOWriter::DecodeFlag(p[1]);
    if (cflag == 0 || cflag == 1) return reinterpret_cast<char*>(const_cast<uint32_t*>(p));
  }
  return end;
}
}  // namespace

void RecordIOWriter::WriteRecord(const void* buf, size_t size) {
  CHECK(size < (1U << 29U)) << "RecordIO only accepts records smaller than 2^29 bytes";
  const uint32_t magic = kMagic;
  const char* data = static_cast<const char*>(buf);
  const uint32_t len = static_cast<uint32_t>(size);
  // scan the payload's aligned words for the magic; each hit closes a part
  uint32_t part_begin = 0;
  const uint32_t aligned_len = len & ~3U;
  for (uint32_t i = 0; i < aligned_len; i += 4) {
    uint32_t word;
    std::memcpy(&word, data + i, 4);
    if (word != magic) continue;
    const uint32_t cflag = part_begin == 0 ? 1U : 2U;
    const uint32_t header[2] = {magic, EncodeLRec(cflag, i - part_begin)};
    stream_->Write(header, sizeof(header));
    if (i != part_begin) stream_->Write(data + part_begin, i - part_begin);
    bytes_written_ += sizeof(header) + (i - part_begin);
    part_begin = i + 4;
    ++except_counter_;
  }
  const uint32_t cflag = part_begin != 0 ? 3U : 0U;
  const uint32_t header[2] = {magic, EncodeLRec(cflag, len - part_begin)};
  stream_->Write(header, sizeof(header));
  if (len != part_begin) stream_->Write(data + part_begin, len - part_begin);
  bytes_written_ += sizeof(header) + (len - part_begin);
  const uint32_t padded = (len + 3U) & ~3U;
  if (padded != len) {
    const uint32_t zero = 0;
    stream_->Write(&zero, padded - len);
    bytes_written_ += padded - len;
  }
}

bool RecordIOReader::NextRecord(std::string* out_rec) {
  if (end_of_stream_) return false;
  out_rec->clear();
  size_t size = 0;
  while (true) {
    uint32_t header[2];
    size_t nread = stream_->Read(header, sizeof(header));
    if (nread == 0) {
      end_of_stream_ = true;
      return false;
    }
    CHECK_EQ(nread, sizeof(header)) << "Invalid RecordIO file: truncated header";
    CHECK_EQ(header[0], RecordIOWriter::kMagic) << "Invalid RecordIO file: bad magic";
    const uint32_t cflag = RecordIOWriter::DecodeFlag(header[1]);
    const uint32_t len = RecordIOWriter::DecodeLength(header[1]);
    const uint32_t padded = (len + 3U) & ~3U;
    out_rec->resize(size + padded);
    if (padded != 0) {
      CHECK_EQ(stream_->Read(&(*out_rec)[size], padded), padded)
          << "Invalid RecordIO file: truncated payload";
    }
    size += len;
    out_rec->resize(size);
    if (cflag == 0U || cflag == 3U) break;
    // re-insert the magic word the writer removed
    const uint32_t magic = RecordIOWriter::kMagic;
    out_rec->append(reinterpret_cast<const char*>(&magic), sizeof(magic));
    size += sizeof(magic);
  }
  return true;
}

RecordIOChunkReader::RecordIOChunkReader(InputSplit::Blob chunk, unsigned part_index,
                                         unsigned num_parts) {
  size_t nstep = (chunk.size + num_parts - 1) / num_parts;
  nstep = (nstep + 3U) & ~size_t(3);
  const size_t begin = std::min(chunk.size, nstep * part_index);
  const size_t end = std::min(chunk.size, nstep * (part_index + 1));
  char* head = static_cast<char*>(chunk.dptr);
  pbegin_ = NextHead(head + begin, head + chunk.size);
  pend_ = NextHead(head + end, head + chunk.size);
}

bool RecordIOChunkReader::NextRecord(InputSplit::Blob* out_rec) {
  if (pbegin_ >= pend_) return false;
  uint32_t* p = reinterpret_cast<uint32_t*>(pbegin_);
  CHECK_EQ(p[0], RecordIOWriter::kMagic);
  uint32_t cflag = RecordIOWriter::DecodeFlag(p[1]);
  uint32_t clen = RecordIOWriter::DecodeLength(p[1]);
  if (cflag == 0) {
    out_rec->dptr = pbegin_ + 2 * sizeof(uint32_t);
    out_rec->size = clen;
    pbegin_ += 2 * sizeof(uint32_t) + ((clen + 3U) & ~3U);
    CHECK(pbegin_ <= pend_) << "Invalid RecordIO format";
    return true;
  }
  // multi-part record: gather into temp_
  CHECK_EQ(cflag, 1U) << "Invalid RecordIO format";
  temp_.clear();
  while (true) {
    CHECK(pbegin_ + 2 * sizeof(uint32_t) <= pend_) << "Invalid RecordIO format";
    p = reinterpret_cast<uint32_t*>(pbegin_);
    CHECK_EQ(p[0], RecordIOWriter::kMagic);
    cflag = RecordIOWriter::DecodeFlag(p[1]);
    clen = RecordIOWriter::DecodeLength(p[1]);
    temp_.append(pbegin_ + 2 * sizeof(uint32_t), clen);
    pbegin_ += 2 * sizeof(uint32_t) + ((clen + 3U) & ~3U);
    if (cflag == 3U) break;
    const uint32_t magic = RecordIOWriter::kMagic;
    temp_.append(reinterpret_cast<const char*>(&magic), sizeof(magic));
  }
  out_rec->dptr = BeginPtr(temp_);
  out_rec->size = temp_.length();
  return true;
}

}  // namespace dmlc
