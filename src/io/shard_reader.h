/*!
 * \file src/io/shard_reader.h
 * \brief High-throughput reader of one InputSplit partition into
 *  caller-provided (pinned) buffers: many parallel preads per buffer, cut at
 *  the last record boundary, the partial record carried to the next buffer.
 *
 * This is the host stage of the MI355X pinned ring: the
 * reference's ThreadedInputSplit reads 8 MiB with one fread at a time
 * (`src/io/threaded_input_split.h:33-41`) which caps a rank at a few GB/s;
 * here a 64-256 MiB pinned slot is filled by `nthread` concurrent preads of
 * page-cache / NVMe data so that PCIe (not the CPU) is the bottleneck.
 * Record semantics are exactly those of InputSplitBase (same partition
 * boundaries, same '\n' insertion between text files, same record cut).
 * Remote filesystems fall back to sequential Stream reads.
 */
#ifndef DMLC_IO_SHARD_READER_H_
#define DMLC_IO_SHARD_READER_H_

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "./input_split_base.h"

namespace dmlc {
namespace io {

/*! \brief fixed pool of worker threads running batches of jobs */
class ReadPool {
 public:
  explicit ReadPool(int nthread);
  ~ReadPool();
  /*! \brief run every job (possibly in parallel) and wait for all */
  void Run(const std::vector<std::function<void()>>& jobs);
  int size() const { return static_cast<int>(workers_.size()); }

 private:
  void Worker();
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::vector<std::function<void()>>* jobs_{nullptr};
  std::atomic<size_t> next_{0};
  size_t finished_{0};
  uint64_t generation_{0};
  bool stop_{false};
  std::exception_ptr err_{nullptr};
};

class ShardReader {
 public:
  /*!
   * \param split partition description (not owned; must outlive the reader)
   * \param nthread parallel reads per Fill
   */
  ShardReader(InputSplitBase* split, int nthread);
  /*!
   * \brief read an explicit list of segments of the split's files instead of
   *  its partition (the GPU parser's shuffled mode: sub-shards in an epoch's
   *  visiting order).  A Fill never crosses a segment whose `stop_after` is
   *  set: it returns at the end of such a segment (a record boundary), so no
   *  buffer mixes two groups.
   */
  ShardReader(InputSplitBase* split, int nthread, const std::vector<InputSplitBase::Segment>& segs,
              const std::vector<bool>& stop_after);
  ~ShardReader();
  /*! \brief replace the segment list (as the constructor above) and rewind */
  void SetSegments(const std::vector<InputSplitBase::Segment>& segs,
                   const std::vector<bool>& stop_after);
  /*!
   * \brief fill buf (capacity `cap`, multiple of the split's alignment) with
   *  whole records.
   * \return bytes written; 0 at the end of the partition; kNeedMore when a
   *  single record is longer than `cap`: nothing is lost (the bytes read so
   *  far are kept), call again with a buffer of at least NeedCapacity() bytes
   */
  size_t Fill(char* buf, size_t cap);
  static constexpr size_t kNeedMore = ~static_cast<size_t>(0);
  /*! \brief capacity the next Fill needs after it returned kNeedMore */
  size_t NeedCapacity() const { return need_cap_; }
  /*! \brief rewind to the start of the partition */
  void Reset();
  /*! \brief bytes of the partition (excluding inserted newlines) */
  size_t PartitionBytes() const { return part_bytes_; }
  /*! \brief bytes consumed so far */
  size_t BytesRead() const { return bytes_read_; }
  /*!
   * \brief resume cursor: partition byte offset (file bytes only, inserted
   *  newlines excluded) of the first record not yet returned by Fill.  Always
   *  a record boundary, so Seek(Tell()) in a new reader over the same
   *  partition continues exactly where this one stopped.
   */
  size_t Tell() const { return bytes_read_ - carry_.size(); }
  /*! \brief continue from a cursor returned by Tell() */
  void Seek(size_t pos);

 private:
  struct Seg {
    size_t file;
    size_t begin, end;
    bool newline_after;  // text: insert '\n' after this segment
    bool stop_after;     // Fill returns at the end of this segment
  };
  InputSplitBase* split_;
  std::unique_ptr<ReadPool> pool_;
  std::vector<Seg> segs_;
  std::vector<int> fds_;
  size_t part_bytes_{0};
  size_t seg_idx_{0}, seg_off_{0};
  bool pending_newline_{false};
  bool stop_pending_{false};  // the pending newline ends a group
  std::string carry_;
  size_t need_cap_{0};
  size_t bytes_read_{0};
  int Fd(size_t file);
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_SHARD_READER_H_
