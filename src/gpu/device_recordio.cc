/*!
 * \file src/gpu/device_recordio.cc
 * \brief DeviceRecordIOReader (see dmlc/gpu/device_recordio.h).
 *
 * Sources of device-resident chunks ("pieces"), all starting at a record head:
 *  - sequential, zero-copy: mmap + hipHostRegister'ed partition cut at record
 *    heads (ZeroCopySource), one H2D per piece;
 *  - sequential, staging: a reader thread fills pinned slots with
 *    RecordIOSplitter chunks (ThreadedIter), one H2D per slot;
 *  - HBM replay (hbm_cache): the first epoch's pieces stay in an arena,
 *    later epochs decode straight from it (adjacent pieces merged);
 *  - indexed: the shard's bytes are read into HBM once; every batch is
 *    gathered on the device from the epoch order of the CPU
 *    IndexedRecordIOSplitter (shuffled with std::mt19937(111 + seed)).
 * Per piece, in stream order (device_slots pieces in flight):
 *   copy stream    : wait(parsed[d]) -> H2D / gather (piece d) -> record(copied[d])
 *   compute stream : wait(copied[d]) -> R1 count -> C2 scan -> [host: sizes]
 *                    -> R2 fill -> C4 finish -> [host: error bits] -> record(parsed[d])
 * The two host waits poll a flag the publishing kernel raises in mapped
 * pinned memory (spin, then short sleeps: host_wait.h), no stream
 * synchronisation and no device-to-host copies.
 */
#include <dmlc/fault.h>
#include <dmlc/gpu/device_recordio.h>
#include <dmlc/gpu/hip_utils.h>
#include <dmlc/logging.h>
#include <dmlc/threadediter.h>
#include <dmlc/timer.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <vector>

#include "../io/filesys.h"
#include "../io/recordio_split.h"
#include "../io/uri_spec.h"
#include "./host_wait.h"
#include "./kernels.h"
#include "./zero_copy_source.h"

namespace dmlc {
namespace gpu {

void DeviceRecordIOConfig::Update(const std::map<std::string, std::string>& args) {
  auto mb = [](const std::string& v) { return static_cast<size_t>(std::atof(v.c_str()) * (1 << 20)); };
  auto flag = [](const std::string& v) { return v != "0" && v != "false" && !v.empty(); };
  for (const auto& kv : args) {
    const std::string& k = kv.first;
    const std::string& v = kv.second;
    if (k == "chunk_mb") {
      chunk_bytes = mb(v);
    } else if (k == "chunk_bytes") {
      chunk_bytes = std::strtoull(v.c_str(), nullptr, 10);
    } else if (k == "device") {
      device = std::atoi(v.c_str());
    } else if (k == "zero_copy") {
      zero_copy = (v == "auto" || v == "-1") ? -1 : (flag(v) ? 1 : 0);
    } else if (k == "device_slots") {
      device_slots = std::atoi(v.c_str());
    } else if (k == "pinned_slots") {
      pinned_slots = std::atoi(v.c_str());
    } else if (k == "hbm_cache") {
      hbm_cache = flag(v);
    } else if (k == "replay_chunk_mb") {
      replay_chunk_bytes = mb(v);
    } else if (k == "one_pass") {
      one_pass = flag(v);
    } else if (k == "chain_count") {
      chain_count = (v == "auto" || v == "-1") ? -1 : (flag(v) ? 1 : 0);
    } else if (k == "index") {
      index_uri = v;
    } else if (k == "shuffle") {
      shuffle = flag(v);
    } else if (k == "seed") {
      seed = std::atoi(v.c_str());
    } else if (k == "wait_spin_us") {
      wait_spin_us = std::atof(v.c_str());
    }
  }
  chunk_bytes = (chunk_bytes + 4095) & ~size_t(4095);
  CHECK_GE(chunk_bytes, 4096U);
  // per-chunk output bytes and record counts are scanned as 32-bit halves
  CHECK_LT(chunk_bytes, size_t(1) << 32) << "chunk_bytes must be < 4 GiB";
  CHECK_LT(replay_chunk_bytes, size_t(1) << 32) << "replay_chunk_bytes must be < 4 GiB";
  CHECK_GE(device_slots, 1);
  CHECK_GE(pinned_slots, 1);
}

namespace {

/*! \brief a chunk read by the reader thread into pinned memory */
struct HostSlot {
  PinnedBuffer buf;
  size_t size{0};
};

/*! \brief a device slot: a chunk's bytes (or the extents of a gathered batch) */
struct DevSlot {
  DeviceBuffer text;
  Event copied, parsed;
  bool used{false};
  // indexed batches: extents in pinned memory and on the device
  PinnedBuffer h_ext;
  DeviceBuffer d_ext;
};

/*! \brief a device-resident chunk ready to decode once `slot`'s copy is done */
struct Piece {
  const uint32_t* words;
  size_t bytes;
  int slot;          // device slot (-1: HBM arena)
  HostSlot* host;    // pinned slot to recycle after the copy (staging path)
};

class DeviceRecordIOImpl : public DeviceRecordIOReader {
 public:
  DeviceRecordIOImpl(const std::string& uri, unsigned part, unsigned nparts,
                     const DeviceRecordIOConfig& cfg)
      : cfg_(cfg) {
    if (cfg_.device >= 0) SetDevice(cfg_.device);
    io::URI path(uri.c_str());
    io::FileSystem* fs = io::FileSystem::GetInstance(path);
    for (int d = 0; d < cfg_.device_slots; ++d) slots_.emplace_back(new DevSlot());
    hmap_.Reserve(sizeof(ChunkMeta), /*mapped=*/true);
    std::memset(hmap_.get(), 0, sizeof(ChunkMeta));
    meta_.Reserve(sizeof(ChunkMeta));
    // second R1 + scan scratch set: the next replayed piece's count runs on
    // count_ while the current piece's fill runs (PrelaunchCount)
    hmap_next_.Reserve(sizeof(ChunkMeta), /*mapped=*/true);
    std::memset(hmap_next_.get(), 0, sizeof(ChunkMeta));
    meta_next_.Reserve(sizeof(ChunkMeta));
    if (!cfg_.index_uri.empty()) {
      indexed_.reset(new io::IndexedRecordIOSplitter(fs, uri.c_str(), cfg_.index_uri.c_str(), part,
                                                     nparts, 1, cfg_.shuffle, cfg_.seed));
      return;
    }
    split_.reset(new io::RecordIOSplitter(fs, uri.c_str(), part, nparts));
    if (cfg_.zero_copy != 0) {
      zc_.reset(new ZeroCopySource(ZeroCopySource::Cut::kRecordIO));
      zc_->SetDrain([this]() { copy_.Synchronize(); });
      if (!zc_->Init(split_.get(), cfg_.chunk_bytes,
                     ZeroCopySource::ShardPinBudget(size_t(64) << 30))) {
        CHECK_NE(cfg_.zero_copy, 1) << "zero_copy=1 but mmap/hipHostRegister failed";
        zc_.reset();
      }
    }
    stats_.zero_copy = zc_ != nullptr;
    if (zc_ == nullptr) StartReader();
    if (cfg_.hbm_cache) caching_ = true;
  }

  ~DeviceRecordIOImpl() override {
    (void)hipStreamSynchronize(copy_.get());
    (void)hipStreamSynchronize(compute_.get());
    (void)hipStreamSynchronize(count_.get());
    for (auto& p : ready_) {
      if (p.host != nullptr) iter_.Recycle(&p.host);
    }
    ready_.clear();
    iter_.Destroy();
  }

  void BeforeFirst() override {
    // a replay keeps the next epoch's prelaunched first count (the arena
    // stays); anything else retires it
    Drain(/*keep_prelaunch=*/cache_complete_ && indexed_ == nullptr);
    exhausted_ = false;
    resident_rows_ = resident_bytes_ = 0;
    if (indexed_ != nullptr) {
      indexed_->BeforeFirst();  // the next epoch's order (re-shuffled)
      epoch_pos_ = 0;
      return;
    }
    if (cache_complete_) {
      replay_ = true;
      replay_idx_ = 0;
      return;
    }
    // a partial first pass cannot complete the cache: start it over
    if (cfg_.hbm_cache) {
      cached_.clear();
      arena_fill_ = 0;
      caching_ = true;
    }
    if (zc_ != nullptr) {
      zc_->Reset();
    } else {
      iter_.BeforeFirst();
    }
  }

  bool Next() override {
    Piece p;
    if (!NextPiece(&p)) return false;
    Decode(p, false);
    return true;
  }
  const DeviceRecordBatch& Value() const override { return batch_; }

  const DeviceRecordBatch& ReadAll() override {
    resident_rows_ = resident_bytes_ = 0;
    res_off_.Grow(sizeof(uint64_t), 0, compute_.get());
    DMLC_HIP_CHECK(hipMemsetAsync(res_off_.get<uint64_t>(), 0, sizeof(uint64_t), compute_.get()));
    Piece p;
    merge_replay_ = true;  // resident decode: adjacent cached chunks may merge
    while (NextPiece(&p)) Decode(p, true);
    merge_replay_ = false;
    compute_.Synchronize();
    PrelaunchNextEpoch();
    resident_.size = resident_rows_;
    resident_.bytes = resident_bytes_;
    resident_.offset = res_off_.get<uint64_t>();
    resident_.data = res_data_.get<uint8_t>();
    return resident_;
  }

  size_t PartitionBytes() const override {
    if (indexed_ != nullptr) return IndexedBytes();
    if (zc_ != nullptr) return zc_->PartitionBytes();
    return split_->offset_end() - split_->offset_begin();
  }
  const DeviceRecordIOStats& Stats() const override { return stats_; }
  hipStream_t stream() const override { return compute_.get(); }

 private:
  // ------------------------------------------------------------ sources
  void StartReader() {
    const size_t cap = cfg_.chunk_bytes;
    io::RecordIOSplitter* split = split_.get();
    split->HintChunkSize(cap);
    iter_.set_max_capacity(static_cast<size_t>(cfg_.pinned_slots));
    iter_.Init(
        [split, cap](HostSlot** dptr) {
          InputSplit::Blob blob;
          if (!split->NextChunk(&blob)) return false;
          if (*dptr == nullptr) *dptr = new HostSlot();
          HostSlot* s = *dptr;
          s->buf.Reserve(std::max(cap, blob.size) + 16);  // grows for a record longer than cap
          std::memcpy(s->buf.get<char>(), blob.dptr, blob.size);
          s->size = blob.size;
          return true;
        },
        [split]() { split->BeforeFirst(); });
  }

  size_t IndexedBytes() const {
    const size_t n = indexed_->NumRecords();
    if (n == 0) return 0;
    const size_t first = indexed_->FirstRecord();
    const auto& last = indexed_->Record(first + n - 1);
    return last.first + last.second - indexed_->Record(first).first;
  }

  /*! \brief the shard's bytes into HBM (once): records at arena + (offset - base) */
  void LoadIndexedArena() {
    if (arena_loaded_) return;
    const size_t total = IndexedBytes();
    const size_t base = indexed_->NumRecords() ? indexed_->Record(indexed_->FirstRecord()).first : 0;
    arena_.Reserve(total + 16);
    PinnedBuffer stage(std::min<size_t>(std::max<size_t>(total, 1), 64UL << 20));
    for (size_t off = 0; off < total;) {
      const size_t n = std::min(stage.bytes(), total - off);
      indexed_->ReadBytes(base + off, n, stage.get<char>());
      DMLC_HIP_CHECK(hipMemcpyAsync(arena_.get<char>() + off, stage.get(), n, hipMemcpyHostToDevice,
                                    copy_.get()));
      copy_.Synchronize();  // the stage is reused
      off += n;
    }
    arena_base_ = base;
    arena_loaded_ = true;
  }

  DevSlot& TakeSlot(int* d) {
    *d = next_slot_;
    next_slot_ = (next_slot_ + 1) % cfg_.device_slots;
    return *slots_[*d];
  }

  /*! \brief the device slot `s` must hold `bytes` (+ pad); waits until no stream uses it */
  void FitSlot(DevSlot* s, size_t bytes) {
    if (bytes + 16 <= s->text.bytes()) return;
    if (s->used) s->parsed.Synchronize();
    s->text.Reserve(bytes + 16);
  }

  /*! \brief queue the next pieces until device_slots are in flight */
  void FillPipeline() {
    while (!exhausted_ && static_cast<int>(ready_.size()) + busy_ < cfg_.device_slots) {
      DMLC_FAULT_POINT("recordio");
      Piece p{nullptr, 0, -1, nullptr};
      if (!(indexed_ != nullptr ? GatherBatch(&p) : (replay_ ? ReplayPiece(&p) : ReadPiece(&p)))) {
        exhausted_ = true;
        if (caching_) {
          caching_ = false;
          cache_complete_ = true;
        }
        break;
      }
      ready_.push_back(p);
    }
  }

  bool ReadPiece(Piece* p) {
    const char* src = nullptr;
    size_t n = 0;
    HostSlot* host = nullptr;
    if (zc_ != nullptr) {
      ZeroCopySource::Piece zp;
      if (!zc_->Next(&zp)) return false;
      src = zp.ptr;
      n = zp.size;
    } else {
      const double t0 = GetTime();
      if (!iter_.Next(&host)) return false;
      stats_.wait_reader_sec += GetTime() - t0;
      src = host->buf.get<char>();
      n = host->size;
    }
    CHECK_EQ(n % 4, 0U) << "RecordIO chunk not 4-byte aligned";
    int d;
    DevSlot& s = TakeSlot(&d);
    char* dst;
    if (caching_) {
      // first pass of an hbm_cache epoch: the chunk lands in its arena place
      if (arena_.bytes() == 0) arena_.Reserve(PartitionBytes() + 16);
      CHECK_LE(arena_fill_ + n, PartitionBytes()) << "RecordIO HBM cache overflow";
      dst = arena_.get<char>() + arena_fill_;
      cached_.push_back({arena_fill_, n});
      arena_fill_ += n;
    } else {
      FitSlot(&s, n);
      dst = s.text.get<char>();
    }
    if (s.used) DMLC_HIP_CHECK(hipStreamWaitEvent(copy_.get(), s.parsed.get(), 0));
    DMLC_HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, copy_.get()));
    s.copied.Record(copy_.get());
    s.used = true;
    *p = Piece{reinterpret_cast<const uint32_t*>(dst), n, d, host};
    return true;
  }

  bool ReplayPiece(Piece* p) {
    if (replay_idx_ >= cached_.size()) return false;
    size_t off = cached_[replay_idx_].first, n = cached_[replay_idx_].second;
    ++replay_idx_;
    // ReadAll: adjacent cached chunks decode as one (fewer launches and host
    // waits); Next() keeps the first epoch's batch boundaries (<= chunk_bytes)
    while (merge_replay_ && replay_idx_ < cached_.size() && cached_[replay_idx_].first == off + n &&
           n + cached_[replay_idx_].second <= cfg_.replay_chunk_bytes) {
      n += cached_[replay_idx_++].second;
    }
    *p = Piece{reinterpret_cast<const uint32_t*>(arena_.get<char>() + off), n, -1, nullptr};
    stats_.replayed_chunks += 1;
    return true;
  }

  /*! \brief the next batch of the epoch order, gathered from the HBM shard into a slot */
  bool GatherBatch(Piece* p) {
    const size_t nrec = indexed_->NumRecords();
    if (epoch_pos_ >= nrec) return false;
    LoadIndexedArena();
    // records of the epoch order until the batch holds chunk_bytes (at least one)
    std::vector<uint64_t>& so = tmp_src_;
    std::vector<uint32_t>& ln = tmp_len_;
    std::vector<uint64_t>& dof = tmp_dst_;
    so.clear();
    ln.clear();
    dof.clear();
    size_t total = 0;
    while (epoch_pos_ < nrec) {
      const auto& r = indexed_->Record(indexed_->EpochRecord(epoch_pos_));
      if (!so.empty() && total + r.second > cfg_.chunk_bytes) break;
      CHECK_EQ(r.second % 4, 0U) << "indexed RecordIO: record size not a multiple of 4";
      so.push_back(r.first - arena_base_);
      ln.push_back(static_cast<uint32_t>(r.second));
      dof.push_back(total);
      total += r.second;
      ++epoch_pos_;
    }
    const size_t k = so.size();
    int d;
    DevSlot& s = TakeSlot(&d);
    FitSlot(&s, total);
    const size_t ext_bytes = k * (2 * sizeof(uint64_t) + sizeof(uint32_t));
    if (s.used) s.copied.Synchronize();  // the previous extents of this slot were consumed
    s.h_ext.Reserve(ext_bytes);
    s.d_ext.Reserve(ext_bytes);
    char* h = s.h_ext.get<char>();
    std::memcpy(h, so.data(), k * 8);
    std::memcpy(h + k * 8, dof.data(), k * 8);
    std::memcpy(h + k * 16, ln.data(), k * 4);
    if (s.used) DMLC_HIP_CHECK(hipStreamWaitEvent(copy_.get(), s.parsed.get(), 0));
    DMLC_HIP_CHECK(hipMemcpyAsync(s.d_ext.get(), h, ext_bytes, hipMemcpyHostToDevice, copy_.get()));
    const char* dx = s.d_ext.get<char>();
    LaunchRecordIOGather(arena_.get<uint8_t>(), reinterpret_cast<const uint64_t*>(dx),
                         reinterpret_cast<const uint32_t*>(dx + k * 16),
                         reinterpret_cast<const uint64_t*>(dx + k * 8), k, s.text.get<uint8_t>(),
                         copy_.get());
    s.copied.Record(copy_.get());
    s.used = true;
    *p = Piece{s.text.get<uint32_t>(), total, d, nullptr};
    stats_.replayed_chunks += 1;
    return true;
  }

  bool NextPiece(Piece* p) {
    FillPipeline();
    if (ready_.empty()) return false;
    *p = ready_.front();
    ready_.pop_front();
    return true;
  }

  void Drain(bool keep_prelaunch = false) {
    copy_.Synchronize();
    compute_.Synchronize();
    if (!keep_prelaunch) DropPrelaunch();
    for (auto& p : ready_) {
      if (p.host != nullptr) iter_.Recycle(&p.host);
    }
    ready_.clear();
    busy_ = 0;
  }

  // ------------------------------------------------------------ decode
  ChunkMeta WaitMeta() {
    const double t0 = GetTime();
    ChunkMeta* hm = hmap_.get<ChunkMeta>();
    volatile unsigned* flag = &hm->pad;
    if (!WaitHostFlag(flag, cfg_.wait_spin_us, 0.05, &waits_)) {
      compute_.Synchronize();
      count_.Synchronize();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    ChunkMeta m;
    std::memcpy(&m, const_cast<const ChunkMeta*>(hm), sizeof(m));
    *flag = 0;  // re-armed before the next publishing kernel
    stats_.wait_gpu_sec += GetTime() - t0;
    return m;
  }

  static void CheckErrors(unsigned e) {
    CHECK_EQ(e & kRecErrTruncated, 0U) << "RecordIO: a record runs past its chunk (corrupt file?)";
    CHECK_EQ(e & kRecErrBadPart, 0U) << "RecordIO: malformed record (bad multi-part chain or header)";
  }

  /*!
   * \brief one launch for an HBM-resident piece of ReadAll: the fill counts
   *  its own tiles (look-back), writes into output sized by the piece's bound
   *  (nwords / 2 records, its bytes) -- no count kernel, no second read of
   *  the text, one host wait
   */
  void DecodeOnePass(const Piece& p) {
    hipStream_t st = compute_.get();
    DropPrelaunch();
    const size_t nwords = p.bytes / 4;
    const size_t tiles = RecordIOTiles(nwords);
    partials_.Reserve(TileScratchSlots(tiles) * sizeof(MetaPartial));
    status_.Reserve(tiles * sizeof(uint64_t));
    if (ticket_.bytes() == 0) {
      ticket_.Reserve(sizeof(unsigned long long));
      DMLC_HIP_CHECK(hipMemsetAsync(ticket_.get(), 0, ticket_.bytes(), st));
      ticket0_ = 0;
    }
    ChunkMeta* dmeta = meta_.get<ChunkMeta>();
    ChunkMeta* hm = hmap_.get<ChunkMeta>();
    ChunkMeta done;
    for (;;) {
      // into the capacity the resident output has (an earlier epoch sized it)
      uint64_t* off = res_off_.get<uint64_t>();
      uint8_t* dat = res_data_.get<uint8_t>();
      const size_t rec_cap = res_off_.bytes() / sizeof(uint64_t);
      const RecordIOOnePass op{status_.get<uint64_t>(), ticket_.get<unsigned long long>(),
                               ticket0_, dmeta, rec_cap > 0 ? rec_cap - 1 : 0, res_data_.bytes()};
      ticket0_ += LaunchRecordIOTileFill(p.words, nwords, nullptr, off, resident_rows_, dat,
                                         resident_bytes_, partials_.get<MetaPartial>(), st, &op);
      LaunchTileFinish(partials_.get<MetaPartial>(), tiles, dmeta, hm, off, resident_rows_,
                       resident_bytes_, st);
      done = WaitMeta();
      CheckErrors(done.flags);
      if (!(done.flags & kFlagOverflow)) break;
      GrowResident(done.nrows, done.nnz);  // did not fit: grow, run the piece again
      stats_.one_pass_reruns += 1;
    }
    busy_ = 0;
    resident_rows_ += done.nrows;
    resident_bytes_ += done.nnz;
    stats_.bytes += p.bytes;
    stats_.chunks += 1;
    stats_.records += done.nrows;
    stats_.one_pass_chunks += 1;
  }

  void Decode(Piece p, bool resident) {
    ScopedRange range("recordio_chunk");
    busy_ = 1;
    hipStream_t st = compute_.get();
    if (resident && cfg_.one_pass && p.slot < 0 && p.host == nullptr && indexed_ == nullptr &&
        replay_ && p.bytes != 0) {
      DecodeOnePass(p);
      FillPipeline();
      return;
    }
    if (p.slot >= 0) DMLC_HIP_CHECK(hipStreamWaitEvent(st, slots_[p.slot]->copied.get(), 0));
    const size_t nwords = p.bytes / 4;
    const size_t tiles = RecordIOTiles(nwords);
    if (pre_.valid && pre_.words == p.words && pre_.bytes == p.bytes) {
      // R1 + scan of this piece ran on count_ beside the previous fill: adopt
      // that scratch set; the fill waits for the scan that wrote its prefix
      tcounts_.swap(tcounts_next_);
      tflags_.swap(tflags_next_);
      meta_.swap(meta_next_);
      hmap_.swap(hmap_next_);
      pre_.valid = false;
      DMLC_HIP_CHECK(hipStreamWaitEvent(st, pre_done_.get(), 0));
    } else {
      DropPrelaunch();
      tcounts_.Reserve(TileScratchWords(tiles) * sizeof(uint64_t));
      tflags_.Reserve(TileScratchWords(tiles) * sizeof(uint32_t));
      LaunchCount(p.words, nwords, tcounts_.get<uint64_t>(), tflags_.get<uint32_t>(), st);
      LaunchTileScanRaw(tcounts_.get<uint64_t>(), tflags_.get<uint32_t>(), tiles,
                        meta_.get<ChunkMeta>(), hmap_.get<ChunkMeta>(), st);
    }
    partials_.Reserve(TileScratchSlots(tiles) * sizeof(MetaPartial));
    ChunkMeta* dmeta = meta_.get<ChunkMeta>();
    ChunkMeta* hm = hmap_.get<ChunkMeta>();
    const ChunkMeta sizes = WaitMeta();
    // the copy of this piece is complete: its pinned slot goes back to the reader
    if (p.host != nullptr) iter_.Recycle(&p.host);
    FillPipeline();  // keep PCIe busy while this piece decodes
    CheckErrors(sizes.flags);
    const size_t nrec = sizes.nrows, nbytes = sizes.nnz;
    uint64_t* off;
    uint8_t* dat;
    uint64_t rec_base = 0, byte_base = 0;
    if (resident) {
      GrowResident(nrec, nbytes);
      off = res_off_.get<uint64_t>();
      dat = res_data_.get<uint8_t>();
      rec_base = resident_rows_;
      byte_base = resident_bytes_;
    } else {
      out_off_.Reserve((nrec + 1) * sizeof(uint64_t));
      out_data_.Reserve(std::max<size_t>(nbytes, 1));
      off = out_off_.get<uint64_t>();
      dat = out_data_.get<uint8_t>();
    }
    // the fill's guards: writes inside the output, tile totals equal to the count's
    const RecordIOCaps caps{dmeta,
                            (resident ? res_off_.bytes() : out_off_.bytes()) / sizeof(uint64_t) - 1,
                            resident ? res_data_.bytes() : out_data_.bytes()};
    LaunchRecordIOTileFill(p.words, nwords, tcounts_.get<uint64_t>(), off, rec_base, dat, byte_base,
                           partials_.get<MetaPartial>(), st, nullptr, &caps);
    LaunchTileFinish(partials_.get<MetaPartial>(), tiles, dmeta, hm, off, rec_base, byte_base, st);
    if (resident) PrelaunchCount();
    const ChunkMeta done = WaitMeta();
    if (p.slot >= 0) slots_[p.slot]->parsed.Record(st);
    busy_ = 0;
    CheckErrors(done.flags);
    if (resident) {
      resident_rows_ += nrec;
      resident_bytes_ += nbytes;
    } else {
      batch_.size = nrec;
      batch_.bytes = nbytes;
      batch_.offset = off;
      batch_.data = dat;
    }
    stats_.bytes += p.bytes;
    stats_.chunks += 1;
    stats_.records += nrec;
  }

  /*!
   * \brief ReadAll over the HBM cache: start the next replayed piece's R1 +
   *  scan on count_ (second scratch set) so it overlaps the current fill
   *  instead of following the host's turnaround; the set it writes was last
   *  used by the piece before the current one, which is complete.
   */
  void PrelaunchCount() {
    if (!replay_ || indexed_ != nullptr || pre_.valid) return;
    if (ready_.empty()) {
      // the epoch's last piece is decoding: count the next epoch's first
      // one beside it (ReadAll over the cache replays the same pieces)
      if (exhausted_ && merge_replay_) PrelaunchNextEpoch();
      return;
    }
    const Piece& nx = ready_.front();
    if (nx.slot >= 0 || nx.host != nullptr) return;  // not an arena-resident piece
    PrelaunchFor(nx.words, nx.bytes);
  }

  /*!
   * \brief at the end of a ReadAll over the HBM cache: the next epoch's
   *  first piece (the same merge from the first cached chunk) is counted
   *  now, on count_, so the next ReadAll's first fill does not wait for its
   *  count.  A next pass that starts with another piece (Next() batches)
   *  drops it unused.
   */
  void PrelaunchNextEpoch() {
    if (!replay_ || indexed_ != nullptr || pre_.valid || cached_.empty()) return;
    size_t off = cached_[0].first, n = cached_[0].second;
    for (size_t i = 1; i < cached_.size() && cached_[i].first == off + n &&
                       n + cached_[i].second <= cfg_.replay_chunk_bytes;
         ++i) {
      n += cached_[i].second;
    }
    if (n == 0) return;
    PrelaunchFor(reinterpret_cast<const uint32_t*>(arena_.get<char>() + off), n);
  }

  void PrelaunchFor(const uint32_t* words, size_t bytes) {
    const size_t nwords = bytes / 4;
    const size_t tiles = RecordIOTiles(nwords);
    tcounts_next_.Reserve(TileScratchWords(tiles) * sizeof(uint64_t));
    tflags_next_.Reserve(TileScratchWords(tiles) * sizeof(uint32_t));
    LaunchCount(words, nwords, tcounts_next_.get<uint64_t>(), tflags_next_.get<uint32_t>(),
                count_.get());
    LaunchTileScanRaw(tcounts_next_.get<uint64_t>(), tflags_next_.get<uint32_t>(), tiles,
                      meta_next_.get<ChunkMeta>(), hmap_next_.get<ChunkMeta>(), count_.get());
    pre_done_.Record(count_.get());
    pre_.valid = true;
    pre_.words = words;
    pre_.bytes = bytes;
  }

  /*!
   * \brief R1 or, for chunks of large enough records, R1c (headers only):
   *  auto decides from the records decoded so far (the first chunk: R1)
   */
  void LaunchCount(const uint32_t* words, size_t nwords, uint64_t* counts, uint32_t* flags,
                   hipStream_t st) {
    bool chain = cfg_.chain_count == 1;
    if (cfg_.chain_count < 0 && stats_.records != 0) {
      const size_t per = stats_.bytes / stats_.records;
      chain = per >= 128 && per <= 4096;
    }
    if (chain) {
      LaunchRecordIOTileCountChain(words, nwords, counts, flags, st);
      stats_.chain_counts += 1;
    } else {
      LaunchRecordIOTileCount(words, nwords, counts, flags, st);
    }
  }

  /*! \brief retire a prelaunched count nobody adopts (its flag re-armed) */
  void DropPrelaunch() {
    if (!pre_.valid) return;
    count_.Synchronize();
    hmap_next_.get<ChunkMeta>()->pad = 0;
    pre_.valid = false;
  }

  void GrowResident(size_t nrec, size_t bytes) {
    const size_t need_off = (resident_rows_ + nrec + 1) * sizeof(uint64_t);
    if (need_off > res_off_.bytes()) {
      res_off_.Grow(need_off + need_off / 2, (resident_rows_ + 1) * sizeof(uint64_t), compute_.get());
    }
    const size_t need_data = resident_bytes_ + bytes;
    if (need_data > res_data_.bytes()) {
      res_data_.Grow(need_data + need_data / 2, resident_bytes_, compute_.get());
    }
  }

  DeviceRecordIOConfig cfg_;
  std::unique_ptr<io::RecordIOSplitter> split_;
  std::unique_ptr<io::IndexedRecordIOSplitter> indexed_;
  std::unique_ptr<ZeroCopySource> zc_;
  ThreadedIter<HostSlot> iter_;
  Stream copy_, compute_, count_;
  Event pre_done_;
  std::vector<std::unique_ptr<DevSlot>> slots_;
  std::deque<Piece> ready_;
  int next_slot_{0};
  int busy_{0};
  bool exhausted_{false};
  // HBM arena: the hbm_cache copy (sequential) or the indexed shard
  DeviceBuffer arena_;
  size_t arena_fill_{0}, arena_base_{0}, replay_idx_{0}, epoch_pos_{0};
  std::vector<std::pair<size_t, size_t>> cached_;
  bool caching_{false}, cache_complete_{false}, replay_{false}, arena_loaded_{false};
  bool merge_replay_{false};  // inside ReadAll: ReplayPiece may merge cached chunks
  std::vector<uint64_t> tmp_src_, tmp_dst_;
  std::vector<uint32_t> tmp_len_;
  // decode scratch and outputs
  DeviceBuffer tcounts_, tflags_, partials_, meta_;
  PinnedBuffer hmap_;
  // the prelaunched next piece's R1 + scan scratch (ReadAll over the HBM cache)
  DeviceBuffer tcounts_next_, tflags_next_, meta_next_;
  PinnedBuffer hmap_next_;
  struct Prelaunch {
    bool valid{false};
    const uint32_t* words{nullptr};
    size_t bytes{0};
  } pre_;
  HostWaitStats waits_;
  DeviceBuffer out_off_, out_data_, res_off_, res_data_;
  // one-pass replays: look-back words (zeroed per launch), workgroup tickets
  DeviceBuffer status_, ticket_;
  unsigned long long ticket0_{0};
  size_t resident_rows_{0}, resident_bytes_{0};
  DeviceRecordBatch batch_, resident_;
  DeviceRecordIOStats stats_;
};

}  // namespace

DeviceRecordIOReader* DeviceRecordIOReader::Create(const std::string& uri, unsigned part_index,
                                                   unsigned num_parts,
                                                   const DeviceRecordIOConfig& cfg) {
  io::URISpec spec(uri, part_index, num_parts);
  DeviceRecordIOConfig c = cfg;
  c.Update(spec.args);
  return new DeviceRecordIOImpl(spec.uri, part_index, num_parts, c);
}

}  // namespace gpu
}  // namespace dmlc
