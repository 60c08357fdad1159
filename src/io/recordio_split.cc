/*!
 * \file src/io/recordio_split.cc
 * \brief RecordIO splitters (see recordio_split.h).
 */
#include "./recordio_split.h"

#include <dmlc/common.h>
#include <dmlc/recordio.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <sstream>

namespace dmlc {
namespace io {

size_t RecordIOSplitterBase::SeekRecordBegin(Stream* fi) {
  size_t nstep = 0;
  uint32_t v, lrec;
  while (true) {
    if (fi->Read(&v, sizeof(v)) == 0) return nstep;
    nstep += sizeof(v);
    if (v == RecordIOWriter::kMagic) {
      CHECK(fi->Read(&lrec, sizeof(lrec)) != 0) << "invalid record io format";
      nstep += sizeof(lrec);
      const uint32_t cflag = RecordIOWriter::DecodeFlag(lrec);
      if (cflag == 0 || cflag == 1) break;
    }
  }
  return nstep - 2 * sizeof(uint32_t);
}

const char* RecordIOSplitterBase::FindLastRecordBegin(const char* begin, const char* end) {
  CHECK_EQ(reinterpret_cast<uintptr_t>(begin) & 3U, 0U);
  CHECK_EQ(reinterpret_cast<uintptr_t>(end) & 3U, 0U);
  const uint32_t* pbegin = reinterpret_cast<const uint32_t*>(begin);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(end);
  CHECK(p >= pbegin + 2);
  for (p = p - 2; p != pbegin; --p) {
    if (p[0] == RecordIOWriter::kMagic) {
      const uint32_t cflag = RecordIOWriter::DecodeFlag(p[1]);
      if (cflag == 0 || cflag == 1) return reinterpret_cast<const char*>(p);
    }
  }
  return begin;
}

bool RecordIOSplitterBase::ExtractNextRecord(Blob* out_rec, Chunk* chunk) {
  if (chunk->begin == chunk->end) return false;
  CHECK(chunk->begin + 2 * sizeof(uint32_t) <= chunk->end) << "Invalid RecordIO format";
  CHECK_EQ(reinterpret_cast<uintptr_t>(chunk->begin) & 3U, 0U);
  uint32_t* p = reinterpret_cast<uint32_t*>(chunk->begin);
  uint32_t cflag = RecordIOWriter::DecodeFlag(p[1]);
  uint32_t clen = RecordIOWriter::DecodeLength(p[1]);
  out_rec->dptr = chunk->begin + 2 * sizeof(uint32_t);
  out_rec->size = clen;
  chunk->begin += 2 * sizeof(uint32_t) + ((clen + 3U) & ~3U);
  CHECK(chunk->begin <= chunk->end) << "Invalid RecordIO format";
  if (cflag == 0) return true;
  CHECK_EQ(cflag, 1U) << "Invalid RecordIO format";
  // multi-part: compact the parts in place behind the first one
  char* dst = static_cast<char*>(out_rec->dptr);
  while (cflag != 3U) {
    CHECK(chunk->begin + 2 * sizeof(uint32_t) <= chunk->end) << "Invalid RecordIO format";
    p = reinterpret_cast<uint32_t*>(chunk->begin);
    CHECK_EQ(p[0], RecordIOWriter::kMagic);
    cflag = RecordIOWriter::DecodeFlag(p[1]);
    clen = RecordIOWriter::DecodeLength(p[1]);
    const uint32_t magic = RecordIOWriter::kMagic;
    std::memcpy(dst + out_rec->size, &magic, sizeof(magic));
    out_rec->size += sizeof(magic);
    if (clen != 0) {
      std::memmove(dst + out_rec->size, chunk->begin + 2 * sizeof(uint32_t), clen);
      out_rec->size += clen;
    }
    chunk->begin += 2 * sizeof(uint32_t) + ((clen + 3U) & ~3U);
  }
  return true;
}

// ---------------------------------------------------------------------------
IndexedRecordIOSplitter::IndexedRecordIOSplitter(FileSystem* fs, const char* uri,
                                                 const char* index_uri, unsigned rank,
                                                 unsigned nsplit, size_t batch_size,
                                                 bool shuffle, int seed)
    : shuffle_(shuffle), batch_size_(batch_size) {
  if (shuffle) SetRandomSeed(seed);
  this->Init(fs, uri, 4);
  this->ReadIndexFile(index_uri);
  this->ResetPartition(rank, nsplit);
}

void IndexedRecordIOSplitter::ReadIndexFile(const std::string& index_uri) {
  std::vector<std::string> uris = Split(index_uri, ';');
  CHECK_EQ(uris.size(), 1U) << "IndexedRecordIOSplitter supports exactly one index file";
  URI path(uris[0].c_str());
  std::unique_ptr<Stream> fi(FileSystem::GetInstance(path)->Open(path, "r", false));
  std::string content;
  char buf[1 << 16];
  size_t n;
  while ((n = fi->Read(buf, sizeof(buf))) != 0) content.append(buf, n);
  std::istringstream is(content);
  std::vector<size_t> offsets;
  size_t key, offset;
  while (is >> key >> offset) offsets.push_back(offset);
  CHECK(!offsets.empty()) << "empty index file " << index_uri;
  std::sort(offsets.begin(), offsets.end());
  index_.clear();
  const size_t total = file_offset_.back();
  for (size_t j = 0; j < offsets.size(); ++j) {
    const size_t next = j + 1 < offsets.size() ? offsets[j + 1] : total;
    CHECK(offsets[j] <= next && next <= total) << "index offset beyond data size";
    index_.emplace_back(offsets[j], next - offsets[j]);
  }
}

void IndexedRecordIOSplitter::ResetPartition(unsigned rank, unsigned nsplit) {
  const size_t ntotal = index_.size();
  const size_t nstep = (ntotal + nsplit - 1) / nsplit;
  index_begin_ = std::min(ntotal, rank * nstep);
  index_end_ = std::min(ntotal, (rank + 1) * nstep);
  offset_begin_ = index_begin_ < ntotal ? index_[index_begin_].first : file_offset_.back();
  offset_end_ = index_end_ < ntotal ? index_[index_end_].first : file_offset_.back();
  delete fs_;
  fs_ = nullptr;
  this->BeforeFirst();
}

void IndexedRecordIOSplitter::BeforeFirst() {
  if (shuffle_) {
    permutation_.clear();
    for (size_t i = index_begin_; i < index_end_; ++i) permutation_.push_back(i);
    std::shuffle(permutation_.begin(), permutation_.end(), rnd_);
    current_index_ = 0;
  } else {
    current_index_ = index_begin_;
  }
  InputSplitBase::BeforeFirst();
}

void IndexedRecordIOSplitter::ReadBytes(size_t offset, size_t n, char* dst) {
  size_t cur = offset, done = 0;
  while (done < n) {
    // the file holding byte `cur`, then as much of [cur, offset + n) as it has
    const size_t fp = static_cast<size_t>(
        std::upper_bound(file_offset_.begin(), file_offset_.end(), cur) - file_offset_.begin() - 1);
    CHECK_LT(fp, files_.size()) << "RecordIO byte range beyond the data";
    if (fs_ == nullptr || fp != file_ptr_) {
      delete fs_;
      file_ptr_ = fp;
      fs_ = filesys_->OpenForRead(files_[fp].path);
    }
    fs_->Seek(cur - file_offset_[fp]);
    const size_t can = std::min(n - done, file_offset_[fp + 1] - cur);
    for (size_t got = 0; got < can;) {
      const size_t k = fs_->Read(dst + done + got, can - got);
      CHECK(k != 0) << "unexpected end of RecordIO file";
      got += k;
    }
    done += can;
    cur += can;
  }
}

bool IndexedRecordIOSplitter::LoadRecords(Chunk* chunk, const std::vector<size_t>& ids) {
  size_t total = 0;
  for (size_t id : ids) total += index_[id].second;
  if (total == 0) return false;
  chunk->data.resize(total / sizeof(uint32_t) + 2);
  char* dst = reinterpret_cast<char*>(chunk->data.data());
  size_t pos = 0;
  // coalesce records that are adjacent in the file into one read
  for (size_t i = 0; i < ids.size();) {
    size_t j = i + 1;
    const size_t off = index_[ids[i]].first;
    size_t len = index_[ids[i]].second;
    while (j < ids.size() && index_[ids[j]].first == off + len) len += index_[ids[j++]].second;
    ReadBytes(off, len, dst + pos);
    pos += len;
    i = j;
  }
  chunk->begin = dst;
  chunk->end = dst + pos;
  return true;
}

bool IndexedRecordIOSplitter::NextBatchEx(Chunk* chunk, size_t n_records) {
  std::vector<size_t> ids;
  if (shuffle_) {
    while (ids.size() < n_records && current_index_ < permutation_.size()) {
      ids.push_back(permutation_[current_index_++]);
    }
  } else {
    while (ids.size() < n_records && current_index_ < index_end_) {
      ids.push_back(current_index_++);
    }
  }
  if (ids.empty()) return false;
  return LoadRecords(chunk, ids);
}

bool IndexedRecordIOSplitter::NextBatch(Blob* out_chunk, size_t n_records) {
  while (!ExtractNextChunk(out_chunk, &tmp_chunk_)) {
    if (!NextBatchEx(&tmp_chunk_, n_records)) return false;
  }
  return true;
}

bool IndexedRecordIOSplitter::NextRecord(Blob* out_rec) {
  while (!ExtractNextRecord(out_rec, &tmp_chunk_)) {
    if (!NextBatchEx(&tmp_chunk_, 1)) return false;
  }
  return true;
}

}  // namespace io
}  // namespace dmlc
