/*!
 * \file src/io/recordio_split.h
 * \brief RecordIO splitters: byte-range ("recordio") and index-driven
 *  ("indexed_recordio", record-count sharding + per-epoch shuffle).
 *
 * Parity: reference `src/io/recordio_split.{h,cc}` (align 4, SeekRecordBegin
 * scanning for magic + cflag∈{0,1}, in-place re-assembly of multi-part
 * records :44-82) and `src/io/indexed_recordio_split.{h,cc}` (index file of
 * "key offset" lines sorted by offset :43-61; record-count partition
 * ceil(nrec/n) :12-41; sequential batches or shuffled per-record reads with
 * std::mt19937(111 + seed) re-shuffled at every BeforeFirst :158-232).
 *
 * Fix: the end sentinel is not re-appended to the index on
 * every ResetPartition.
 */
#ifndef DMLC_IO_RECORDIO_SPLIT_H_
#define DMLC_IO_RECORDIO_SPLIT_H_

#include <random>
#include <string>
#include <utility>
#include <vector>

#include "./input_split_base.h"

namespace dmlc {
namespace io {

/*! \brief shared RecordIO record extraction */
class RecordIOSplitterBase : public InputSplitBase {
 public:
  bool ExtractNextRecord(Blob* out_rec, Chunk* chunk) override;
  const char* FindLastRecordBegin(const char* begin, const char* end) override;
  /*! \brief local files: chunks are views of the file mapping (no copy) */
  bool MappableChunks() const override { return true; }

 protected:
  size_t SeekRecordBegin(Stream* fi) override;
};

class RecordIOSplitter : public RecordIOSplitterBase {
 public:
  RecordIOSplitter(FileSystem* fs, const char* uri, unsigned rank, unsigned nsplit,
                   bool recurse_directories = false) {
    this->Init(fs, uri, 4, recurse_directories);
    this->ResetPartition(rank, nsplit);
  }
};

class IndexedRecordIOSplitter : public RecordIOSplitterBase {
 public:
  IndexedRecordIOSplitter(FileSystem* fs, const char* uri, const char* index_uri,
                          unsigned rank, unsigned nsplit, size_t batch_size,
                          bool shuffle, int seed = 0);
  void ResetPartition(unsigned rank, unsigned nsplit) override;
  void BeforeFirst() override;
  bool NextRecord(Blob* out_rec) override;
  bool NextChunk(Blob* out_chunk) override { return NextBatch(out_chunk, batch_size_); }
  bool NextBatch(Blob* out_chunk, size_t n_records) override;
  bool NextChunkEx(Chunk* chunk) override { return NextBatchEx(chunk, batch_size_); }
  bool NextBatchEx(Chunk* chunk, size_t n_records) override;
  void SetRandomSeed(size_t seed) { rnd_.seed(kRandMagic + seed); }
  void SetBatchSize(size_t batch_size) { batch_size_ = batch_size; }
  /*! \brief number of records in this part */
  size_t NumRecords() const { return index_end_ - index_begin_; }
  /*! \brief (file offset, size) of record i (global index, sorted by offset) */
  const std::pair<size_t, size_t>& Record(size_t i) const { return index_[i]; }
  /*! \brief global index of this part's first record */
  size_t FirstRecord() const { return index_begin_; }
  /*!
   * \brief this epoch's k-th record (global index): the shuffled order drawn
   *  by the last BeforeFirst, or the sequential one -- the order NextRecord /
   *  NextChunk deliver (the GPU reader gathers batches in it)
   */
  size_t EpochRecord(size_t k) const {
    return shuffle_ ? permutation_[k] : index_begin_ + k;
  }
  /*! \brief bytes [offset, offset + n) of the concatenated input files */
  void ReadBytes(size_t offset, size_t n, char* dst);

 private:
  static const int kRandMagic = 111;
  void ReadIndexFile(const std::string& index_uri);
  /*! \brief read records [ids] into chunk (exact byte ranges) */
  bool LoadRecords(Chunk* chunk, const std::vector<size_t>& ids);
  /*! \brief (offset, size) of every record, sorted by offset */
  std::vector<std::pair<size_t, size_t>> index_;
  std::vector<size_t> permutation_;
  bool shuffle_;
  size_t batch_size_;
  size_t index_begin_{0}, index_end_{0}, current_index_{0};
  std::mt19937 rnd_;
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_RECORDIO_SPLIT_H_
