/*!
 * \file src/io/shard_reader.cc
 * \brief Parallel-pread partition reader (see shard_reader.h).
 */
#include "./shard_reader.h"

#include <dmlc/fault.h>
#include <dmlc/logging.h>
#include <errno.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace dmlc {
namespace io {

// ----------------------------------------------------------------- pool
ReadPool::ReadPool(int nthread) {
  for (int i = 0; i < std::max(1, nthread); ++i) workers_.emplace_back([this]() { Worker(); });
}

ReadPool::~ReadPool() {
  {
    std::lock_guard<std::mutex> lock(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ReadPool::Worker() {
  uint64_t seen = 0;
  while (true) {
    {
      std::unique_lock<std::mutex> lock(mu_);
      cv_.wait(lock, [&]() { return stop_ || generation_ != seen; });
      if (stop_) return;
      seen = generation_;
    }
    // jobs are claimed under the lock and only for the generation we woke
    // for, so a late worker can never touch a finished batch
    while (true) {
      const std::function<void()>* job = nullptr;
      {
        std::lock_guard<std::mutex> lock(mu_);
        if (generation_ != seen || jobs_ == nullptr || next_ >= jobs_->size()) break;
        job = &(*jobs_)[next_++];
      }
      try {
        (*job)();
      } catch (...) {
        std::lock_guard<std::mutex> lock(mu_);
        if (err_ == nullptr) err_ = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> lock(mu_);
        ++finished_;
      }
      done_cv_.notify_all();
    }
  }
}

void ReadPool::Run(const std::vector<std::function<void()>>& jobs) {
  if (jobs.empty()) return;
  if (jobs.size() == 1) {
    jobs[0]();
    return;
  }
  {
    std::lock_guard<std::mutex> lock(mu_);
    jobs_ = &jobs;
    next_ = 0;
    finished_ = 0;
    err_ = nullptr;
    ++generation_;
  }
  cv_.notify_all();
  std::exception_ptr err;
  {
    std::unique_lock<std::mutex> lock(mu_);
    done_cv_.wait(lock, [&]() { return finished_ == jobs.size(); });
    jobs_ = nullptr;
    err = err_;
  }
  if (err != nullptr) std::rethrow_exception(err);
}

// --------------------------------------------------------------- reader
namespace {
// smallest ranged GET of a remote Fill (DMLC_REMOTE_MIN_PIECE_KB overrides)
size_t RemoteMinPiece() {
  static const size_t v = [] {
    const char* e = std::getenv("DMLC_REMOTE_MIN_PIECE_KB");
    const size_t kb = e != nullptr ? std::strtoull(e, nullptr, 10) : 1024;
    return std::max<size_t>(kb, 64) << 10;
  }();
  return v;
}

void PreadFull(int fd, char* dst, size_t len, size_t off) {
  while (len != 0) {
    const ssize_t n = ::pread(fd, dst, len, static_cast<off_t>(off));
    if (n < 0) {
      if (errno == EINTR) continue;
      LOG(FATAL) << "pread failed: " << std::strerror(errno);
    }
    CHECK(n != 0) << "unexpected end of file at offset " << off;
    dst += n;
    len -= static_cast<size_t>(n);
    off += static_cast<size_t>(n);
  }
}
}  // namespace

ShardReader::ShardReader(InputSplitBase* split, int nthread)
    : split_(split), pool_(new ReadPool(nthread)) {
  fds_.assign(split->files().size(), -2);  // -2: not opened yet
  const auto segs = split->ShardSegments();
  SetSegments(segs, std::vector<bool>(segs.size(), false));
}

ShardReader::ShardReader(InputSplitBase* split, int nthread,
                         const std::vector<InputSplitBase::Segment>& segs,
                         const std::vector<bool>& stop_after)
    : split_(split), pool_(new ReadPool(nthread)) {
  fds_.assign(split->files().size(), -2);
  SetSegments(segs, stop_after);
}

void ShardReader::SetSegments(const std::vector<InputSplitBase::Segment>& segs,
                              const std::vector<bool>& stop_after) {
  CHECK_EQ(segs.size(), stop_after.size());
  segs_.clear();
  part_bytes_ = 0;
  for (size_t i = 0; i < segs.size(); ++i) {
    Seg s{segs[i].file_index, segs[i].begin, segs[i].end, false, stop_after[i]};
    part_bytes_ += s.end - s.begin;
    if (split_->IsTextParser() && i + 1 < segs.size()) {
      // '\n' after a segment whose last line has no EOL (a file end; as
      // InputSplitBase::Read between files)
      char last = '\n';
      const int fd = Fd(s.file);
      if (fd >= 0) {
        PreadFull(fd, &last, 1, s.end - 1);
      } else {
        std::unique_ptr<SeekStream> st(split_->filesystem()->OpenForReadSized(
            split_->files()[s.file].path, split_->files()[s.file].size));
        st->Seek(s.end - 1);
        CHECK_EQ(st->Read(&last, 1), 1U);
      }
      s.newline_after = last != '\n' && last != '\r';
    }
    segs_.push_back(s);
  }
  Reset();
}

ShardReader::~ShardReader() {
  for (int fd : fds_) {
    if (fd >= 0) ::close(fd);
  }
}

int ShardReader::Fd(size_t file) {
  if (fds_[file] == -2) fds_[file] = split_->filesystem()->OpenRawFd(split_->files()[file].path);
  return fds_[file];
}

void ShardReader::Seek(size_t pos) {
  CHECK_LE(pos, part_bytes_) << "cursor beyond the partition";
  Reset();
  size_t base = 0;
  seg_idx_ = segs_.size();
  for (size_t i = 0; i < segs_.size(); ++i) {
    const size_t len = segs_[i].end - segs_[i].begin;
    if (pos < base + len) {
      // a cursor on a segment boundary means "previous file fully consumed",
      // so no separator newline is pending here
      seg_idx_ = i;
      seg_off_ = pos - base;
      break;
    }
    base += len;
  }
  bytes_read_ = pos;
}

void ShardReader::Reset() {
  seg_idx_ = 0;
  seg_off_ = 0;
  pending_newline_ = false;
  stop_pending_ = false;
  carry_.clear();
  bytes_read_ = 0;
}

size_t ShardReader::Fill(char* buf, size_t cap) {
  DMLC_FAULT_POINT("read");
  if (carry_.size() >= cap) {
    // the pending record alone fills the buffer: ask for a bigger one
    need_cap_ = std::max(2 * cap, carry_.size() + 1);
    return kNeedMore;
  }
  size_t pos = carry_.size();
  if (pos != 0) std::memcpy(buf, carry_.data(), pos);
  carry_.clear();
  std::vector<std::function<void()>> jobs;
  const size_t min_piece = 4UL << 20;
  bool group_end = false;
  while (pos < cap) {
    if (pending_newline_) {
      buf[pos++] = '\n';
      pending_newline_ = false;
      if (stop_pending_) {  // that newline closed a group (buffer was full)
        stop_pending_ = false;
        group_end = true;
        break;
      }
      continue;
    }
    if (seg_idx_ >= segs_.size()) break;
    const Seg& s = segs_[seg_idx_];
    const size_t n = std::min(s.end - s.begin - seg_off_, cap - pos);
    const size_t file_off = s.begin + seg_off_;
    const int fd = Fd(s.file);
    if (fd >= 0) {
      const size_t piece =
          std::max(min_piece, ((n / std::max(1, pool_->size())) + 4095) & ~size_t(4095));
      for (size_t o = 0; o < n; o += piece) {
        const size_t len = std::min(piece, n - o);
        char* dst = buf + pos + o;
        const size_t off = file_off + o;
        jobs.emplace_back([fd, dst, len, off]() { PreadFull(fd, dst, len, off); });
      }
    } else {
      // remote filesystem: parallel ranged GETs, one stream per piece (size
      // known from the listing, so no HEAD per piece).  One piece per pool
      // worker, so every connection is busy for the whole Fill (round 3 had
      // an 8 MiB floor: a 64 MiB slot kept 8 connections busy whatever the
      // pool size, profiles/r03_remote); the floor bounds request overhead.
      FileSystem* fs = split_->filesystem();
      const URI path = split_->files()[s.file].path;
      const size_t fsize = split_->files()[s.file].size;
      const size_t piece =
          std::max(RemoteMinPiece(),
                   ((n + pool_->size() - 1) / std::max(1, pool_->size()) + 65535) & ~size_t(65535));
      for (size_t o = 0; o < n; o += piece) {
        const size_t len = std::min(piece, n - o);
        char* dst = buf + pos + o;
        const size_t off = file_off + o;
        jobs.emplace_back([fs, path, fsize, dst, len, off]() {
          std::unique_ptr<SeekStream> st(fs->OpenForReadSized(path, fsize));
          st->Seek(off);
          size_t got = 0;
          while (got < len) {
            const size_t r = st->Read(dst + got, len - got);
            CHECK(r != 0) << "unexpected end of " << path.str();
            got += r;
          }
        });
      }
    }
    pos += n;
    seg_off_ += n;
    bytes_read_ += n;
    if (seg_off_ == s.end - s.begin) {
      if (s.newline_after) pending_newline_ = true;
      ++seg_idx_;
      seg_off_ = 0;
      if (s.stop_after) {
        // end of a group: the buffer ends on a record boundary here
        if (pending_newline_ && pos < cap) {
          buf[pos++] = '\n';
          pending_newline_ = false;
        }
        group_end = !pending_newline_;
        stop_pending_ = pending_newline_;
        break;
      }
    }
  }
  pool_->Run(jobs);
  if (pos == 0) return 0;
  const bool at_end = seg_idx_ >= segs_.size() && !pending_newline_;
  if (at_end || group_end) return pos;
  const char* last = split_->FindLastRecordBegin(buf, buf + pos);
  if (last == buf) {
    // one record is longer than the buffer: keep what was read, grow, retry
    // (the reference doubles its chunk buffer, src/io/input_split_base.cc:241-258)
    carry_.assign(buf, pos);
    need_cap_ = 2 * cap;
    return kNeedMore;
  }
  carry_.assign(last, buf + pos - last);
  return static_cast<size_t>(last - buf);
}

}  // namespace io
}  // namespace dmlc
