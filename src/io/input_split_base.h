/*!
 * \file src/io/input_split_base.h
 * \brief Multi-file, record-aligned byte-range sharding + chunked reading.
 *
 * Parity: reference `src/io/input_split_base.h` / `.cc`:
 *  - Init: cumulative file offsets, per-file alignment CHECK (:13-28)
 *  - ResetPartition: nstep = ceil(total / n) rounded up to align_bytes, range
 *    [nstep*r, nstep*(r+1)) clipped, both ends moved to the next record head
 *    with SeekRecordBegin (:30-64) — bit-identical shard boundaries
 *  - ConvertToURIs: ';' lists, exact names, std::regex_match on the last
 *    path component (:96-147); directories expanded, zero-size files dropped
 *    (:149-175)
 *  - Read across file boundaries (:177-209), ReadChunk cutting at the last
 *    record head with an overflow carry (:211-239), Chunk::Load doubling the
 *    buffer when a record does not fit (:241-279)
 *
 * Differences: directory listings are sorted (deterministic shards); text
 * splits insert a '\n' between files whose last line lacks one (otherwise the
 * last line of file i and the first line of file i+1 would merge); the default
 * chunk is 8 MiB (the reference comment claims 16 MB, the value is 8 MiB —
 * SURVEY §7.4 #5).
 *
 * GPU hook: ShardSegments() exposes the exact per-file byte ranges of this
 * part so that the pinned-ring reader (src/io/shard_reader.h) can fill pinned
 * host slots with many parallel preads instead of one sequential stream.
 */
#ifndef DMLC_IO_INPUT_SPLIT_BASE_H_
#define DMLC_IO_INPUT_SPLIT_BASE_H_

#include <dmlc/io.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "./filesys.h"

namespace dmlc {
namespace io {

class InputSplitBase : public InputSplit {
 public:
  /*! \brief a buffer of whole records; `data` has one spare sentinel word */
  struct Chunk {
    char* begin{nullptr};
    char* end{nullptr};
    std::vector<uint32_t> data;
    explicit Chunk(size_t buffer_size) : data(buffer_size + 1) {}
    /*! \brief replace contents with the next records (grows the buffer) */
    bool Load(InputSplitBase* split, size_t buffer_size);
    /*! \brief append the next records after the current contents */
    bool Append(InputSplitBase* split, size_t buffer_size);
  };
  /*! \brief one contiguous piece of the partition inside one file */
  struct Segment {
    size_t file_index;
    size_t begin;  // byte offset inside the file
    size_t end;
  };

  /*! \brief default chunk: 2M words = 8 MiB */
  static const size_t kBufferSize = 2UL << 20UL;

  ~InputSplitBase() override;
  void HintChunkSize(size_t chunk_size) override {
    buffer_size_ = std::max(chunk_size / sizeof(uint32_t), buffer_size_);
  }
  size_t GetTotalSize() override { return file_offset_.back(); }
  void BeforeFirst() override;
  void ResetPartition(unsigned rank, unsigned nsplit) override;
  bool NextRecord(Blob* out_rec) override {
    while (!ExtractNextRecord(out_rec, &tmp_chunk_)) {
      if (!NextChunkEx(&tmp_chunk_)) return false;
    }
    return true;
  }
  bool NextChunk(Blob* out_chunk) override {
    while (!ExtractNextChunk(out_chunk, &tmp_chunk_)) {
      if (!NextChunkEx(&tmp_chunk_)) return false;
    }
    return true;
  }
  /*! \brief load the next chunk into `chunk` */
  virtual bool NextChunkEx(Chunk* chunk) { return chunk->Load(this, buffer_size_); }
  /*! \brief load the next batch of up to n records (indexed splits) */
  virtual bool NextBatchEx(Chunk* chunk, size_t /*n_records*/) { return NextChunkEx(chunk); }
  /*! \brief take the next record out of a loaded chunk */
  virtual bool ExtractNextRecord(Blob* out_rec, Chunk* chunk) = 0;
  /*! \brief take everything left in a loaded chunk */
  virtual bool ExtractNextChunk(Blob* out_chunk, Chunk* chunk) {
    if (chunk->begin == chunk->end) return false;
    out_chunk->dptr = chunk->begin;
    out_chunk->size = chunk->end - chunk->begin;
    chunk->begin = chunk->end;
    return true;
  }
  /*! \brief text splits get '\n' inserted between files */
  virtual bool IsTextParser() const { return false; }
  /*! \brief chunks may be views of a file mapping (LoadMapped): only when
   *  record extraction writes nothing past a record (RecordIO; the line
   *  splitter's NextRecord terminates a line in the byte after it) */
  virtual bool MappableChunks() const { return false; }
  /*!
   * \brief start of the last (possibly incomplete) record in [begin, end);
   *  returns begin when no record head is found after begin
   */
  virtual const char* FindLastRecordBegin(const char* begin, const char* end) = 0;

  /*! \brief raw partition bytes (crosses files); 0 at end of partition */
  size_t Read(void* ptr, size_t size);
  /*!
   * \brief with DMLC_SPLIT_MMAP=1, local files: point `chunk` at the next
   *  whole records inside a private mapping of the current file -- no copy
   *  out of the page cache (the default, like the reference, reads every
   *  chunk into a buffer: faster on the MI355X hosts).  Chunks never span
   *  files (so no newline needs inserting between files); a record longer
   *  than the buffer widens the view.  The mapping is copy-on-write, so the
   *  in-place compaction of multi-part RecordIO records works, and it is
   *  dropped (a fresh one maps the file again) on BeforeFirst / ResetPartition.
   * \return 1 loaded, 0 end of partition, -1 not a mappable file (use Read)
   */
  int LoadMapped(Chunk* chunk, size_t buffer_words);
  /*!
   * \brief fill buf with whole records (< *size bytes); carries the tail
   * \return false at end; *size == 0 with true means "buffer too small"
   */
  virtual bool ReadChunk(void* buf, size_t* size);

  // ---- introspection used by the GPU pinned-ring reader ----
  const std::vector<FileInfo>& files() const { return files_; }
  FileSystem* filesystem() const { return filesys_; }
  size_t align_bytes() const { return align_bytes_; }
  size_t buffer_bytes() const { return buffer_size_ * sizeof(uint32_t); }
  /*! \brief byte ranges of this partition, file by file */
  std::vector<Segment> ShardSegments() const;
  /*! \brief [begin, end) of this partition in concatenated-file space */
  size_t offset_begin() const { return offset_begin_; }
  size_t offset_end() const { return offset_end_; }

 protected:
  InputSplitBase() = default;
  /*! \brief resolve uri into files; every file size must be a multiple of align */
  void Init(FileSystem* fs, const char* uri, size_t align_bytes,
            bool recurse_directories = false);
  /*! \brief bytes from the stream's position to the next record head */
  virtual size_t SeekRecordBegin(Stream* fi) = 0;

  FileSystem* filesys_{nullptr};
  std::vector<FileInfo> files_;
  /*! \brief file_offset_[i] = bytes of files before file i */
  std::vector<size_t> file_offset_;
  size_t offset_begin_{0}, offset_end_{0}, offset_curr_{0};
  size_t file_ptr_{0}, file_ptr_end_{0};
  SeekStream* fs_{nullptr};
  size_t align_bytes_{1};
  size_t buffer_size_{kBufferSize};
  Chunk tmp_chunk_{kBufferSize};
  /*! \brief incomplete record carried to the next ReadChunk */
  std::string overflow_;
  /*! \brief last byte emitted by Read (text: decide about inserting '\n') */
  int last_byte_{-1};
  /*! \brief a '\n' must be emitted before reading the current file */
  bool pending_newline_{false};
  /*! \brief LoadMapped state: whether this split's files may be mapped
   *  (-1 undecided), the current file's mapping */
  int mmap_mode_{-1};
  char* map_base_{nullptr};
  size_t map_len_{0};
  size_t map_file_{static_cast<size_t>(-1)};
  /*! \brief every mapping of this pass: a prefetching consumer
   *  (ThreadedInputSplit) may still hold chunks of earlier files, so they
   *  are dropped only at BeforeFirst / ResetPartition */
  std::vector<std::pair<char*, size_t>> maps_;
  void Unmap();

 private:
  std::vector<URI> ConvertToURIs(const std::string& uri);
  void InitInputFileInfo(const std::string& uri, bool recurse_directories);
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_INPUT_SPLIT_BASE_H_
