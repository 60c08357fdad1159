/*!
 * \file src/io/input_split_base.cc
 * \brief Partitioning and chunked reading (see input_split_base.h for parity).
 */
#include "./input_split_base.h"

#include <dmlc/common.h>
#include <dmlc/logging.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <regex>

#include "./local_filesys.h"

namespace dmlc {
namespace io {

namespace {
std::string StripTrailing(std::string s, char ch) {
  while (!s.empty() && s.back() == ch) s.pop_back();
  return s;
}
}  // namespace

void InputSplitBase::Init(FileSystem* fs, const char* uri, size_t align_bytes,
                          bool recurse_directories) {
  filesys_ = fs;
  InitInputFileInfo(uri, recurse_directories);
  file_offset_.assign(files_.size() + 1, 0);
  for (size_t i = 0; i < files_.size(); ++i) {
    file_offset_[i + 1] = file_offset_[i] + files_[i].size;
    CHECK(files_[i].size % align_bytes == 0)
        << "file " << files_[i].path.str() << " is not aligned to " << align_bytes
        << " bytes";
  }
  align_bytes_ = align_bytes;
}

InputSplitBase::~InputSplitBase() {
  Unmap();
  delete fs_;
}

void InputSplitBase::Unmap() {
  for (const auto& m : maps_) ::munmap(m.first, m.second);
  maps_.clear();
  map_base_ = nullptr;
  map_len_ = 0;
  map_file_ = static_cast<size_t>(-1);
}

int InputSplitBase::LoadMapped(Chunk* chunk, size_t buffer_words) {
  if (mmap_mode_ < 0) {
    // opt-in (DMLC_SPLIT_MMAP=1), local files only (not stdin): on the MI355X
    // hosts a mapped epoch measured 0.55x the buffered one (page faults and
    // unmap shootdowns cost more than the copy out of the page cache:
    // profiles/r06_cpu/rec_ab.txt), so buffered reads are the default
    const char* e = std::getenv("DMLC_SPLIT_MMAP");
    bool ok = e != nullptr && std::atoi(e) != 0 && MappableChunks() &&
              dynamic_cast<LocalFileSystem*>(filesys_) != nullptr;
    for (const FileInfo& f : files_) ok = ok && f.path.name != "stdin" && f.path.name != "-";
    mmap_mode_ = ok ? 1 : 0;
  }
  if (mmap_mode_ == 0) return -1;
  if (offset_curr_ >= offset_end_) return 0;
  const size_t fp = static_cast<size_t>(
      std::upper_bound(file_offset_.begin(), file_offset_.end(), offset_curr_) -
      file_offset_.begin() - 1);
  if (fp != map_file_) {
    const int fd = ::open(files_[fp].path.name.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      mmap_mode_ = 0;
      return -1;
    }
    const size_t len = files_[fp].size;
    void* m = ::mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) {
      mmap_mode_ = 0;
      return -1;
    }
    ::madvise(m, len, MADV_SEQUENTIAL);
    maps_.emplace_back(static_cast<char*>(m), len);
    map_base_ = static_cast<char*>(m);
    map_len_ = len;
    map_file_ = fp;
  }
  const size_t o = offset_curr_ - file_offset_[fp];
  const size_t limit = std::min(offset_end_, file_offset_[fp + 1]) - file_offset_[fp];
  char* const b = map_base_ + o;
  size_t want = buffer_words * sizeof(uint32_t);
  for (;;) {
    if (limit - o <= want) {  // the rest of this file's part of the partition
      chunk->begin = b;
      chunk->end = map_base_ + limit;
      break;
    }
    const char* e = FindLastRecordBegin(b, b + want);
    if (e != b) {
      chunk->begin = b;
      chunk->end = const_cast<char*>(e);
      break;
    }
    want *= 2;  // one record longer than the view: widen it
  }
  offset_curr_ += static_cast<size_t>(chunk->end - chunk->begin);
  return 1;
}

void InputSplitBase::ResetPartition(unsigned rank, unsigned nsplit) {
  CHECK(nsplit != 0 && rank < nsplit) << "invalid partition " << rank << "/" << nsplit;
  const size_t ntotal = file_offset_.back();
  size_t nstep = (ntotal + nsplit - 1) / nsplit;
  nstep = ((nstep + align_bytes_ - 1) / align_bytes_) * align_bytes_;
  offset_begin_ = std::min(nstep * rank, ntotal);
  offset_end_ = std::min(nstep * (rank + 1), ntotal);
  offset_curr_ = offset_begin_;
  delete fs_;
  fs_ = nullptr;
  overflow_.clear();
  Unmap();
  if (offset_begin_ == offset_end_) return;
  auto file_of = [this](size_t off) {
    return static_cast<size_t>(std::upper_bound(file_offset_.begin(), file_offset_.end(), off) -
                               file_offset_.begin() - 1);
  };
  file_ptr_ = file_of(offset_begin_);
  file_ptr_end_ = file_of(offset_end_);
  // move the end to the next record head (same rule as the next part's begin)
  if (offset_end_ != file_offset_[file_ptr_end_]) {
    CHECK(offset_end_ > file_offset_[file_ptr_end_]);
    CHECK(file_ptr_end_ < files_.size());
    SeekStream* s = filesys_->OpenForRead(files_[file_ptr_end_].path);
    s->Seek(offset_end_ - file_offset_[file_ptr_end_]);
    offset_end_ += SeekRecordBegin(s);
    delete s;
  }
  if (offset_begin_ != file_offset_[file_ptr_]) {
    SeekStream* s = filesys_->OpenForRead(files_[file_ptr_].path);
    s->Seek(offset_begin_ - file_offset_[file_ptr_]);
    offset_begin_ += SeekRecordBegin(s);
    delete s;
  }
  this->BeforeFirst();
}

void InputSplitBase::BeforeFirst() {
  Unmap();  // (a copy-on-write mapping may hold compacted records)
  overflow_.clear();
  tmp_chunk_.begin = tmp_chunk_.end = nullptr;
  last_byte_ = -1;
  pending_newline_ = false;
  offset_curr_ = offset_begin_;
  if (offset_begin_ >= offset_end_) return;
  const size_t fp = static_cast<size_t>(
      std::upper_bound(file_offset_.begin(), file_offset_.end(), offset_begin_) -
      file_offset_.begin() - 1);
  if (fs_ == nullptr || file_ptr_ != fp) {
    delete fs_;
    file_ptr_ = fp;
    fs_ = filesys_->OpenForRead(files_[file_ptr_].path);
  }
  fs_->Seek(offset_begin_ - file_offset_[file_ptr_]);
}

std::vector<InputSplitBase::Segment> InputSplitBase::ShardSegments() const {
  std::vector<Segment> segs;
  if (offset_begin_ >= offset_end_) return segs;
  for (size_t i = 0; i < files_.size(); ++i) {
    const size_t fb = file_offset_[i], fe = file_offset_[i + 1];
    const size_t b = std::max(fb, offset_begin_), e = std::min(fe, offset_end_);
    if (b < e) segs.push_back(Segment{i, b - fb, e - fb});
  }
  return segs;
}

std::vector<URI> InputSplitBase::ConvertToURIs(const std::string& uri) {
  std::vector<URI> expanded;
  for (const std::string& item : Split(uri, ';')) {
    if (item.empty()) continue;
    URI path(item.c_str());
    const size_t pos = path.name.rfind('/');
    if (pos == std::string::npos || pos + 1 == path.name.length()) {
      expanded.push_back(path);
      continue;
    }
    // does the exact name exist in its directory? otherwise treat it as a regex
    URI dir = path;
    dir.name = pos == 0 ? "/" : path.name.substr(0, pos);
    std::vector<FileInfo> dfiles;
    filesys_->ListDirectory(dir, &dfiles);
    bool exact = false;
    for (const auto& f : dfiles) {
      if (StripTrailing(f.path.name, '/') == StripTrailing(path.name, '/')) {
        expanded.push_back(f.path);
        exact = true;
        break;
      }
    }
    if (exact) continue;
    try {
      std::regex pattern(path.name);
      bool any = false;
      for (const auto& f : dfiles) {
        if (f.type != kFile || f.size == 0) continue;
        if (std::regex_match(StripTrailing(f.path.name, '/'), pattern)) {
          expanded.push_back(f.path);
          any = true;
        }
      }
      if (!any) expanded.push_back(path);  // let GetPathInfo report it
    } catch (const std::regex_error& e) {
      LOG(FATAL) << e.what() << " bad regex " << path.name;
    }
  }
  return expanded;
}

void InputSplitBase::InitInputFileInfo(const std::string& uri, bool recurse_directories) {
  for (const URI& path : ConvertToURIs(uri)) {
    FileInfo info = filesys_->GetPathInfo(path);
    if (info.type == kDirectory) {
      std::vector<FileInfo> dfiles;
      if (recurse_directories) {
        filesys_->ListDirectoryRecursive(info.path, &dfiles);
      } else {
        filesys_->ListDirectory(info.path, &dfiles);
      }
      for (const auto& f : dfiles) {
        if (f.size != 0 && f.type == kFile) files_.push_back(f);
      }
    } else if (info.size != 0) {
      files_.push_back(info);
    }
  }
  CHECK_NE(files_.size(), 0U) << "Cannot find any files that matches the URI pattern " << uri;
}

size_t InputSplitBase::Read(void* ptr, size_t size) {
  char* buf = static_cast<char*>(ptr);
  size_t nleft = size;
  while (nleft != 0) {
    if (pending_newline_) {
      *buf++ = '\n';
      --nleft;
      last_byte_ = '\n';
      pending_newline_ = false;
      continue;
    }
    if (offset_curr_ >= offset_end_) break;
    const size_t file_end = file_offset_[file_ptr_ + 1];
    const size_t want = std::min(nleft, std::min(offset_end_, file_end) - offset_curr_);
    const size_t n = want == 0 ? 0 : fs_->Read(buf, want);
    if (n != 0) {
      last_byte_ = static_cast<unsigned char>(buf[n - 1]);
      buf += n;
      nleft -= n;
      offset_curr_ += n;
    }
    if (offset_curr_ == file_end) {
      if (file_ptr_ + 1 >= files_.size() || offset_curr_ >= offset_end_) break;
      if (IsTextParser() && last_byte_ != '\n' && last_byte_ != '\r') {
        pending_newline_ = true;
      }
      ++file_ptr_;
      delete fs_;
      fs_ = filesys_->OpenForRead(files_[file_ptr_].path);
    } else if (n == 0) {
      LOG(FATAL) << "file " << files_[file_ptr_].path.str() << " ended at offset "
                 << (offset_curr_ - file_offset_[file_ptr_]) << " but its size is "
                 << files_[file_ptr_].size << " (modified while reading?)";
    }
  }
  return size - nleft;
}

bool InputSplitBase::ReadChunk(void* buf, size_t* size) {
  const size_t max_size = *size;
  if (max_size <= overflow_.length()) {
    *size = 0;
    return true;
  }
  const size_t olen = overflow_.length();
  if (olen != 0) std::memcpy(buf, overflow_.data(), olen);
  overflow_.clear();
  const size_t nread = olen + this->Read(static_cast<char*>(buf) + olen, max_size - olen);
  if (nread == 0) return false;
  if (nread != max_size) {
    *size = nread;
    return true;
  }
  const char* bptr = static_cast<const char*>(buf);
  const char* bend = this->FindLastRecordBegin(bptr, bptr + max_size);
  *size = bend - bptr;
  overflow_.assign(bend, bptr + max_size - bend);
  return true;
}

bool InputSplitBase::Chunk::Load(InputSplitBase* split, size_t buffer_size) {
  const int mapped = split->LoadMapped(this, buffer_size);
  if (mapped >= 0) return mapped == 1;
  if (data.size() < buffer_size + 1) data.resize(buffer_size + 1);
  while (true) {
    size_t size = (data.size() - 1) * sizeof(uint32_t);
    data.back() = 0;
    if (!split->ReadChunk(data.data(), &size)) return false;
    if (size != 0) {
      begin = reinterpret_cast<char*>(data.data());
      end = begin + size;
      return true;
    }
    data.resize(data.size() * 2);  // one record larger than the buffer
  }
}

bool InputSplitBase::Chunk::Append(InputSplitBase* split, size_t buffer_size) {
  const size_t previous_size = end - begin;
  data.resize(data.size() + buffer_size);
  while (true) {
    const size_t capacity = (data.size() - 1) * sizeof(uint32_t);
    size_t size = capacity - previous_size;
    data.back() = 0;
    if (!split->ReadChunk(reinterpret_cast<char*>(data.data()) + previous_size, &size)) {
      return false;
    }
    if (size != 0) {
      begin = reinterpret_cast<char*>(data.data());
      end = begin + previous_size + size;
      return true;
    }
    data.resize(data.size() * 2);
  }
}

}  // namespace io
}  // namespace dmlc
