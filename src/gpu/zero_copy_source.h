/*!
 * \file src/gpu/zero_copy_source.h
 * \brief Zero-copy chunk source for the GPU pipelines: the partition's file
 *  ranges are mmap'ed and registered with hipHostRegister(ReadOnly), so every
 *  H2D DMA reads the page cache directly -- no CPU memcpy into pinned slots
 *  (measured: 87.0M rows/s vs 55.3M with the pread ring, profiles/r01_zero_copy).
 *
 * Chunks never cross a file boundary and end on a record boundary (a record
 * longer than chunk_bytes makes its chunk longer):
 *  - text: after the last EOL of the window (reference LineSplitter,
 *    `src/io/line_split.cc:27-34`);
 *  - RecordIO: at the last aligned record head (magic word followed by an lrec
 *    with cflag 0 or 1) of the window (reference RecordIOSplitter,
 *    `src/io/recordio_split.cc:26-42`), so a multi-part record is never split.
 */
#ifndef DMLC_SRC_GPU_ZERO_COPY_SOURCE_H_
#define DMLC_SRC_GPU_ZERO_COPY_SOURCE_H_

#include <dmlc/gpu/hip_utils.h>
#include <dmlc/logging.h>
#include <dmlc/recordio.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../io/filesys.h"
#include "../io/input_split_base.h"

namespace dmlc {
namespace gpu {

class ZeroCopySource {
 public:
  enum class Cut { kLine, kRecordIO };
  struct Piece {
    const char* ptr;
    size_t size;
  };
  explicit ZeroCopySource(Cut cut = Cut::kLine) : cut_(cut) {}
  ~ZeroCopySource() { Release(); }
  ZeroCopySource(const ZeroCopySource&) = delete;
  ZeroCopySource& operator=(const ZeroCopySource&) = delete;

  /*! \brief map + register every segment; false (and unmapped) on failure */
  bool Init(io::InputSplitBase* split, size_t chunk_bytes) {
    chunk_bytes_ = chunk_bytes;
    const long page = sysconf(_SC_PAGESIZE);
    for (const auto& seg : split->ShardSegments()) {
      if (seg.end <= seg.begin) continue;
      const int fd = split->filesystem()->OpenRawFd(split->files()[seg.file_index].path);
      if (fd < 0) return Fail();
      const size_t map_off = seg.begin & ~static_cast<size_t>(page - 1);
      const size_t map_len = seg.end - map_off;
      void* p = mmap(nullptr, map_len, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, map_off);
      ::close(fd);
      if (p == MAP_FAILED) return Fail();
      maps_.push_back(Mapping{p, map_len, false});
      hipError_t err = hipHostRegister(p, map_len, hipHostRegisterReadOnly);
      if (err != hipSuccess) {
        (void)hipGetLastError();
        return Fail();
      }
      maps_.back().registered = true;
      segs_.push_back(Seg{static_cast<const char*>(p) + (seg.begin - map_off), seg.end - seg.begin});
    }
    return true;
  }
  void Reset() {
    seg_ = 0;
    off_ = 0;
  }
  /*! \brief next chunk of whole records; false at the end */
  bool Next(Piece* out) {
    while (seg_ < segs_.size() && off_ >= segs_[seg_].size) {
      ++seg_;
      off_ = 0;
    }
    if (seg_ >= segs_.size()) return false;
    const Seg& s = segs_[seg_];
    const char* b = s.ptr + off_;
    size_t len = std::min(chunk_bytes_, s.size - off_);
    if (off_ + len < s.size) {
      const size_t avail = s.size - off_;
      len = cut_ == Cut::kLine ? CutLine(b, len, avail) : CutRecord(b, len, avail);
    }
    out->ptr = b;
    out->size = len;
    off_ += len;
    return true;
  }
  /*!
   * \brief partition byte offset of the next piece (same cursor space as
   *  io::ShardReader::Tell: file bytes only, always a record boundary)
   */
  size_t Tell() const {
    size_t n = 0;
    for (size_t i = 0; i < seg_ && i < segs_.size(); ++i) n += segs_[i].size;
    return n + off_;
  }
  /*! \brief continue from a Tell() cursor */
  void Seek(size_t pos) {
    seg_ = 0;
    off_ = pos;
    while (seg_ < segs_.size() && off_ >= segs_[seg_].size) {
      off_ -= segs_[seg_].size;
      ++seg_;
    }
    CHECK(seg_ < segs_.size() || off_ == 0) << "cursor beyond the partition";
  }
  size_t PartitionBytes() const {
    size_t n = 0;
    for (const auto& s : segs_) n += s.size;
    return n;
  }

 private:
  /*!
   * \brief end of the last whole line in [b, b+len); a line longer than the
   *  window makes the piece longer instead (up to the line's end, or `avail`,
   *  the bytes left in the segment), as the reference's InputSplitBase grows
   *  its buffer for long records (src/io/input_split_base.cc:241-258)
   */
  size_t CutLine(const char* b, size_t len, size_t avail) const {
    size_t cut = len;
    while (cut > 0 && b[cut - 1] != '\n' && b[cut - 1] != '\r') --cut;
    if (cut != 0) return cut;
    cut = len;
    while (cut < avail && b[cut] != '\n' && b[cut] != '\r') ++cut;
    while (cut < avail && (b[cut] == '\n' || b[cut] == '\r')) ++cut;
    return cut;
  }
  static bool IsHead(const uint32_t* w, size_t p) {
    return w[p] == RecordIOWriter::kMagic && RecordIOWriter::DecodeFlag(w[p + 1]) <= 1U;
  }
  /*! \brief last record head in the window; past it when one record fills it */
  size_t CutRecord(const char* b, size_t len, size_t avail) const {
    // segments start 4-byte aligned (RecordIO partitions align to 4 bytes)
    const uint32_t* w = reinterpret_cast<const uint32_t*>(b);
    const size_t nw = len / 4;
    for (size_t p = nw >= 2 ? nw - 2 : 0; p > 0; --p) {
      if (IsHead(w, p)) return p * 4;
    }
    const size_t aw = avail / 4;
    for (size_t p = nw > 1 ? nw - 1 : 1; p + 1 < aw; ++p) {
      if (IsHead(w, p)) return p * 4;
    }
    return avail;
  }
  struct Mapping {
    void* ptr;
    size_t len;
    bool registered;
  };
  struct Seg {
    const char* ptr;
    size_t size;
  };
  bool Fail() {
    Release();
    return false;
  }
  void Release() {
    for (auto& m : maps_) {
      if (m.registered) (void)hipHostUnregister(m.ptr);
      munmap(m.ptr, m.len);
    }
    maps_.clear();
    segs_.clear();
  }
  Cut cut_;
  size_t chunk_bytes_{0};
  std::vector<Mapping> maps_;
  std::vector<Seg> segs_;
  size_t seg_{0}, off_{0};
};

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_SRC_GPU_ZERO_COPY_SOURCE_H_
