/*!
 * \file src/gpu/device_parser.cc
 * \brief The MI355X ingestion pipeline (see dmlc/gpu/device_parser.h).
 *
 * Per chunk, in stream order:
 *   copy stream    : wait(parsed[d]) -> H2D(text[d]) -> record(copied[d])
 *   compute stream : wait(copied[d]) -> parse -> record(parsed[d])
 *
 * LibSVM / LibFM chunks take the LDS-staged tile parser (tile_kernels.hip:
 * C1 count, C2 scan, C3 fill, C4 finish; lane per token, SWAR number decode).
 * A chunk it flags as irregular (qid tokens, digit-less tokens, label-less
 * lines, control bytes), and every CSV chunk, is parsed by the exact
 * wave-per-line kernels (text_kernels.hip: K1 line index, K2 count, K3 scan,
 * K4 fill).  Both write bit-identical CSR for regular input.
 * The tile kernels write the chunk's sizes and flags into mapped pinned
 * memory (two stream synchronisations per chunk, no D2H copies); the H2D of
 * the next chunks is queued before the current chunk is parsed, so PCIe
 * transfers overlap the kernels and the reader thread fills pinned slots
 * further ahead.
 */
#include <dmlc/gpu/device_parser.h>
#include <dmlc/fault.h>
#include <dmlc/input_split_shuffle.h>
#include <dmlc/logging.h>
#include <dmlc/threadediter.h>
#include <dmlc/timer.h>

#include <cstdlib>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <memory>
#include <vector>

#include "../io/filesys.h"
#include "../io/line_split.h"
#include "../io/shard_reader.h"
#include "../io/uri_spec.h"
#include "./host_wait.h"
#include "./kernels.h"
#include "./zero_copy_source.h"

namespace dmlc {
namespace gpu {

void DeviceParserConfig::Update(const std::map<std::string, std::string>& args) {
  for (const auto& kv : args) {
    const std::string& k = kv.first;
    const std::string& v = kv.second;
    if (k == "chunk_mb") {
      chunk_bytes = static_cast<size_t>(std::atof(v.c_str()) * (1 << 20));
    } else if (k == "chunk_bytes") {
      chunk_bytes = std::strtoull(v.c_str(), nullptr, 10);
    } else if (k == "pinned_slots") {
      pinned_slots = std::atoi(v.c_str());
    } else if (k == "device_slots") {
      device_slots = std::atoi(v.c_str());
    } else if (k == "read_threads") {
      read_threads = std::atoi(v.c_str());
    } else if (k == "device") {
      device = std::atoi(v.c_str());
    } else if (k == "format") {
      format = v;
    } else if (k == "label_column") {
      label_column = std::atoi(v.c_str());
    } else if (k == "weight_column") {
      weight_column = std::atoi(v.c_str());
    } else if (k == "delimiter") {
      CHECK_EQ(v.size(), 1U) << "delimiter must be one character";
      delimiter = v[0];
    } else if (k == "fast_path") {
      fast_path = v != "0" && v != "false";
    } else if (k == "one_pass") {
      one_pass = v != "0" && v != "false";
    } else if (k == "hash_one_pass") {
      hash_one_pass = v != "0" && v != "false";
    } else if (k == "prelaunch") {
      prelaunch = v != "0" && v != "false";
    } else if (k == "replay_chunk_mb") {
      replay_chunk_bytes = static_cast<size_t>(std::atof(v.c_str()) * (1 << 20));
    } else if (k == "replay_first_mb") {
      replay_first_bytes = static_cast<size_t>(std::atof(v.c_str()) * (1 << 20));
    } else if (k == "zc_pin_budget_mb") {
      zc_pin_budget = static_cast<size_t>(std::atof(v.c_str()) * (1 << 20));
    } else if (k == "zc_window_mb") {
      zc_window_bytes = static_cast<size_t>(std::atof(v.c_str()) * (1 << 20));
    } else if (k == "hbm_cache") {
      hbm_cache = v != "0" && v != "false";
    } else if (k == "wait_spin_us") {
      wait_spin_us = std::atof(v.c_str());
    } else if (k == "shuffle_parts") {
      shuffle_parts = static_cast<unsigned>(std::atoi(v.c_str()));
    } else if (k == "shuffle_seed") {
      shuffle_seed = std::atoi(v.c_str());
    } else if (k == "zero_copy") {
      zero_copy = (v == "auto" || v == "-1") ? -1 : ((v == "0" || v == "false") ? 0 : 1);
    }
  }
  chunk_bytes = (chunk_bytes + 4095) & ~size_t(4095);
  CHECK_GE(chunk_bytes, 4096U) << "chunk_bytes too small";
  CHECK_LT(chunk_bytes, size_t(1) << 31) << "chunk_bytes must be < 2 GiB";
  // merged replay chunks go through the same kernels: 32-bit line offsets on
  // the exact path, 32-bit packed token counts on the tile path
  CHECK_LT(replay_chunk_bytes, size_t(1) << 31) << "replay_chunk_bytes must be < 2 GiB";
  CHECK_GE(pinned_slots, 1);
  CHECK_GE(device_slots, 1);
  CHECK_GE(shuffle_parts, 1U) << "shuffle_parts must be >= 1";
}

namespace {

/*! \brief a filled pinned host slot */
struct HostSlot {
  PinnedBuffer buf;
  /*! \brief usable bytes of buf (grows for records longer than chunk_bytes) */
  size_t cap{0};
  size_t size{0};
  /*! \brief partition cursor after this chunk (ShardReader::Tell) */
  size_t end_pos{0};
};

/*! \brief per-chunk sizes the host needs to place the output */
struct ChunkPlan {
  size_t nlines{0}, ntok{0};
  uint64_t nrows{0}, nnz{0};
  unsigned flags{0};
};

template <typename IndexType>
class DeviceParserImpl : public DeviceParser<IndexType> {
 public:
  DeviceParserImpl(const std::string& uri, unsigned part, unsigned nparts,
                   const DeviceParserConfig& cfg)
      : cfg_(cfg) {
    if (cfg_.device >= 0) SetDevice(cfg_.device);
    DMLC_HIP_CHECK(hipGetDevice(&device_));
    if (cfg_.format == "libsvm") {
      tcfg_.format = TextFormat::kLibSVM;
    } else if (cfg_.format == "libfm") {
      tcfg_.format = TextFormat::kLibFM;
    } else if (cfg_.format == "csv") {
      tcfg_.format = TextFormat::kCSV;
    } else {
      LOG(FATAL) << "DeviceParser: unsupported format " << cfg_.format;
    }
    CHECK(tcfg_.format != TextFormat::kCSV || cfg_.label_column < 0 ||
          cfg_.label_column != cfg_.weight_column)
        << "label_column and weight_column must differ";
    tcfg_.label_column = cfg_.label_column;
    tcfg_.weight_column = cfg_.weight_column;
    tcfg_.delimiter = cfg_.delimiter;
    io::URI path(uri.c_str());
    split_.reset(new io::LineSplitter(io::FileSystem::GetInstance(path), uri.c_str(), part, nparts));
    part_ = part;
    nparts_ = nparts;
    if (cfg_.shuffle_parts > 1) {
      // sub-shard i = partition part * K + i of nparts * K (record-aligned
      // byte ranges, as InputSplitShuffle's source splits); the pipeline reads
      // the epoch's concatenation of them
      const unsigned k = cfg_.shuffle_parts;
      for (unsigned i = 0; i < k; ++i) {
        split_->ResetPartition(part * k + i, nparts * k);
        sub_first_.push_back(all_segs_.size());
        size_t bytes = 0;
        for (const auto& sg : split_->ShardSegments()) {
          if (sg.end <= sg.begin) continue;
          all_segs_.push_back(sg);
          bytes += sg.end - sg.begin;
        }
        sub_bytes_.push_back(bytes);
      }
      sub_first_.push_back(all_segs_.size());
      ApplyOrder();  // epoch 0
      reader_.reset(new io::ShardReader(split_.get(), cfg_.read_threads, EpochSegments(),
                                        EpochStops()));
    } else {
      reader_.reset(new io::ShardReader(split_.get(), cfg_.read_threads));
    }
    // the parse kernels' stream outranks the prelaunched counts' (a fill's or
    // hash's closing kernels are not queued behind the next chunk's count)
    int least_prio = 0, greatest_prio = 0;
    DMLC_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least_prio, &greatest_prio));
    compute_.reset(new Stream(greatest_prio));
    copy_.reset(new Stream());
    for (int d = 0; d < cfg_.device_slots; ++d) {
      dtext_.emplace_back(new DeviceBuffer(cfg_.chunk_bytes + kTextPadBytes));
      // the pad is read (never used) by 16-byte loads past the chunk end.  The
      // memsets go on the copy stream: the streams are non-blocking, so a
      // null-stream hipMemset is not ordered before the H2D copy into the slot
      DMLC_HIP_CHECK(hipMemsetAsync(dtext_.back()->get(), 0, cfg_.chunk_bytes + kTextPadBytes,
                                    copy_->get()));
      copied_.emplace_back(new Event());
      parsed_.emplace_back(new Event());
      parsed_.back()->Record(compute_->get());
    }
    tiles_.Reserve(LineIndexTiles(cfg_.chunk_bytes) * sizeof(uint64_t));
    tcounts_.Reserve(TileScratchWords(TileCount(cfg_.chunk_bytes)) * sizeof(uint64_t));
    tflags_.Reserve(TileScratchWords(TileCount(cfg_.chunk_bytes)) * sizeof(uint32_t));
    tmasks_.Reserve(TileMaskWords(TileCount(cfg_.chunk_bytes)) * sizeof(uint32_t));
    meta_.Reserve(2 * sizeof(ChunkMeta));
    hmeta_.Reserve(2 * sizeof(ChunkMeta));
    hmap_.Reserve(sizeof(ChunkMeta), /*mapped=*/true);
    std::memset(hmap_.get(), 0, sizeof(ChunkMeta));  // WaitMapped polls its pad word
    if (cfg_.hbm_cache) {
      // second C1/C2 scratch set: the next resident chunk's count + scan runs
      // on its own stream, concurrently with the current fill (PrelaunchCount)
      count_stream_.reset(new Stream());
      pre_done_.reset(new Event());
      meta_next_.Reserve(2 * sizeof(ChunkMeta));
      hmap_next_.Reserve(sizeof(ChunkMeta), /*mapped=*/true);
      std::memset(hmap_next_.get(), 0, sizeof(ChunkMeta));
    }
    slots_.Reserve(std::max<size_t>(kMaxPartialBlocks, TileScratchSlots(TileCount(cfg_.chunk_bytes))) *
                   sizeof(MetaPartial));
    iter_.set_max_capacity(static_cast<size_t>(cfg_.pinned_slots));
    if (cfg_.zero_copy != 0) {
      zc_.reset(new ZeroCopySource());
      const double t0 = GetTime();
      zc_->SetDrain([this]() { copy_->Synchronize(); });
      stats_.zc_pin_budget = ZeroCopySource::ShardPinBudget(cfg_.zc_pin_budget);
      if (!zc_->Init(split_.get(), cfg_.chunk_bytes, stats_.zc_pin_budget, cfg_.zc_window_bytes,
                     cfg_.shuffle_parts > 1 ? &all_segs_ : nullptr)) {
        CHECK(cfg_.zero_copy != 1) << "zero_copy=1 but the input cannot be mmap'ed + registered";
        zc_.reset();
      } else {
        stats_.register_sec = GetTime() - t0;
        stats_.zero_copy = true;
        if (cfg_.shuffle_parts > 1) zc_->Reorder(EpochSegmentIndices());
      }
    }
    if (zc_ == nullptr) StartReader();
    if (cfg_.hbm_cache) StartCaching();
  }

  ~DeviceParserImpl() override {
    // make sure no transfer still reads a pinned slot we are about to free;
    // destructors never throw, so errors are ignored here
    if (copy_) (void)hipStreamSynchronize(copy_->get());
    if (compute_) (void)hipStreamSynchronize(compute_->get());
    if (count_stream_) (void)hipStreamSynchronize(count_stream_->get());
    for (auto& f : inflight_) {
      if (f.slot != nullptr) iter_.Recycle(&f.slot);
    }
    inflight_.clear();
    iter_.Destroy();
    zc_.reset();
  }

  void BeforeFirst() override {
    if (cfg_.shuffle_parts > 1) {
      SetEpoch(epoch_ + 1);  // reshuffle (reference InputSplitShuffle::BeforeFirst)
      return;
    }
    Seek(0);
  }

  unsigned Epoch() const override { return epoch_; }

  void SetEpoch(unsigned e) override {
    if (cfg_.shuffle_parts <= 1) {
      Seek(0);
      return;
    }
    DrainInflight();
    epoch_ = e;
    ApplyOrder();
    if (zc_ != nullptr) {
      zc_->Reorder(EpochSegmentIndices());
    } else {
      reorder_reader_ = true;  // applied by the reader thread's rewind (Seek)
    }
    Seek(0);
  }

  std::vector<unsigned> VisitOrder() const override { return order_; }

  size_t Tell() const override { return cursor_; }

  void Seek(size_t cursor) override {
    CHECK_LE(cursor, PartitionBytes()) << "DeviceParser::Seek: cursor beyond the partition";
    // a replay restarting at 0 keeps the next epoch's first count, prelaunched
    // beside the last fill (PrelaunchNextEpoch; dropped if the chunk differs)
    DrainInflight(/*keep_prelaunch=*/cursor == 0 && cache_complete_ && cfg_.shuffle_parts <= 1);
    replay_ = false;
    caching_ = false;
    if (cfg_.hbm_cache) {
      if (cache_complete_) {
        // replay from the cache when the cursor is a chunk boundary of this
        // epoch's order (sub-shards in visiting order, chunks in text order)
        BuildReplayList();
        for (size_t i = 0; i <= replay_list_.size(); ++i) {
          const size_t b = i < replay_list_.size() ? replay_begin_[i] : PartitionBytes();
          if (b == cursor) {
            replay_ = true;
            replay_idx_ = i;
            merge_cap_ = 0;
            cursor_ = cursor;
            return;
          }
        }
      } else if (cursor == 0) {
        StartCaching();
      } else {
        cached_.clear();  // a partial pass cannot complete the cache
        arena_fill_ = 0;
      }
    }
    if (zc_ != nullptr) {
      zc_->Seek(cursor);
    } else {
      seek_pos_ = cursor;
      iter_.BeforeFirst();
    }
    cursor_ = cursor;
  }

  // ---------------------------------------------------------- shuffled mode
  /*! \brief this epoch's visiting order and each sub-shard's epoch offset */
  void ApplyOrder() {
    order_ = InputSplitShuffle::VisitOrder(part_, nparts_, cfg_.shuffle_parts, cfg_.shuffle_seed,
                                           epoch_);
    sub_pos_.assign(cfg_.shuffle_parts, 0);
    size_t pos = 0;
    for (unsigned j : order_) {
      sub_pos_[j] = pos;
      pos += sub_bytes_[j];
    }
  }
  std::vector<size_t> EpochSegmentIndices() const {
    std::vector<size_t> idx;
    for (unsigned j : order_) {
      for (size_t g = sub_first_[j]; g < sub_first_[j + 1]; ++g) idx.push_back(g);
    }
    return idx;
  }
  std::vector<io::InputSplitBase::Segment> EpochSegments() const {
    std::vector<io::InputSplitBase::Segment> segs;
    for (size_t g : EpochSegmentIndices()) segs.push_back(all_segs_[g]);
    return segs;
  }
  /*! \brief a pinned fill ends with each sub-shard (chunks never mix two) */
  std::vector<bool> EpochStops() const {
    std::vector<bool> stop;
    for (unsigned j : order_) {
      for (size_t g = sub_first_[j]; g < sub_first_[j + 1]; ++g) {
        stop.push_back(g + 1 == sub_first_[j + 1]);
      }
    }
    return stop;
  }
  /*! \brief sub-shard holding epoch cursor `pos` (the first one starting at or
   *  before it with bytes left), and the offset inside it */
  unsigned SubOf(size_t pos, size_t* local) const {
    if (cfg_.shuffle_parts <= 1) {
      *local = pos;
      return 0;
    }
    for (unsigned j : order_) {
      if (pos >= sub_pos_[j] && pos < sub_pos_[j] + sub_bytes_[j]) {
        *local = pos - sub_pos_[j];
        return j;
      }
    }
    *local = 0;
    return order_.back();
  }
  /*! \brief cached chunks in this epoch's order, with their epoch cursors */
  void BuildReplayList() {
    replay_list_.clear();
    replay_begin_.clear();
    replay_end_.clear();
    if (cfg_.shuffle_parts <= 1) {
      for (size_t i = 0; i < cached_.size(); ++i) {
        replay_list_.push_back(i);
        replay_begin_.push_back(cached_[i].begin_pos);
        replay_end_.push_back(cached_[i].end_pos);
      }
      return;
    }
    for (unsigned j : order_) {
      for (size_t i = 0; i < cached_.size(); ++i) {
        if (cached_[i].sub != j) continue;
        replay_list_.push_back(i);
        replay_begin_.push_back(sub_pos_[j] + cached_[i].sub_begin);
        replay_end_.push_back(sub_pos_[j] + cached_[i].sub_end);
      }
    }
  }

  bool Next() override {
    block_.Clear();
    block_.device_ = device_;
    ResetEpoch();
    if (!ProcessOne(&block_, /*append=*/false)) return false;
    FinishEpoch(&block_);
    view_ = block_.View();
    return true;
  }

  const DeviceRowBlock<IndexType>& Value() const override { return view_; }

  void ParseAll(DeviceCSR<IndexType>* out) override {
    ScopedRange range("DeviceParser::ParseAll");
    out->device_ = device_;
    ResetEpoch();
    merge_replay_ = true;
    if (cfg_.one_pass && replay_ && cfg_.fast_path && tcfg_.format != TextFormat::kCSV &&
        !one_pass_off_) {
      // one pass per resident chunk (no count to hide behind a previous fill,
      // so no small first chunk): merge up to 2 x replay_chunk_bytes, below
      // 2 GiB (the exact fallback's 32-bit offsets and the look-back's 31-bit
      // counts)
      merge_limit_ = std::min(2 * cfg_.replay_chunk_bytes, (size_t(1) << 31) - (size_t(64) << 20));
      if (merge_cap_ == 0) merge_cap_ = merge_limit_;
    }
    // pipeline fill (start -> first chunk parsed) and drain (last chunk
    // handed to the pipeline -> pass done), host clock
    const double t0 = GetTime();
    double t_first = 0, t_last_in = 0;
    try {
      while (ProcessOne(out, /*append=*/true)) {
        const double t = GetTime();
        if (t_first == 0) t_first = t;
        if (reader_done_ && t_last_in == 0) t_last_in = t;
      }
    } catch (...) {
      merge_replay_ = false;
      merge_limit_ = 0;
      throw;
    }
    merge_replay_ = false;
    merge_limit_ = 0;
    FinishEpoch(out);
    const double t_end = GetTime();
    stats_.last_pass_sec = t_end - t0;
    stats_.last_fill_sec = t_first != 0 ? t_first - t0 : 0;
    stats_.last_drain_sec = t_last_in != 0 ? t_end - t_last_in : 0;
  }

  size_t PartitionBytes() const override {
    return zc_ != nullptr ? zc_->PartitionBytes() : reader_->PartitionBytes();
  }
  const DeviceParserStats& Stats() const override { return stats_; }
  hipStream_t stream() const override { return compute_->get(); }

 private:
  struct Inflight {
    HostSlot* slot;  // nullptr in zero-copy / replay mode
    int d;           // device slot (events), -1 when replayed from the HBM cache
    size_t size;
    size_t end_pos;  // resume cursor once this chunk is delivered
    const char* text;  // device text of the chunk
  };
  /*! \brief a chunk held in the HBM epoch cache */
  struct CachedChunk {
    size_t off, size, begin_pos, end_pos;
    unsigned sub;                // shuffled mode: its sub-shard
    size_t sub_begin, sub_end;   // and its cursor range inside it
    bool eol_end;                // its text ends with an EOL byte (mergeable with the next)
  };

  void StartReader() {
    const size_t cap = cfg_.chunk_bytes;
    io::ShardReader* reader = reader_.get();
    iter_.Init(
        [reader, cap](HostSlot** dptr) {
          if (*dptr == nullptr) {
            *dptr = new HostSlot();
            (*dptr)->buf.Reserve(cap + kTextPadBytes);
            (*dptr)->cap = cap;
          }
          ScopedRange r("pinned_fill");
          HostSlot* slot = *dptr;
          size_t n = reader->Fill(slot->buf.template get<char>(), slot->cap);
          while (n == io::ShardReader::kNeedMore) {
            // a record longer than the slot: grow it (the reader kept the bytes)
            slot->cap = reader->NeedCapacity();
            slot->buf.Free();
            slot->buf.Reserve(slot->cap + kTextPadBytes);
            n = reader->Fill(slot->buf.template get<char>(), slot->cap);
          }
          (*dptr)->size = n;
          (*dptr)->end_pos = reader->Tell();
          return (*dptr)->size != 0;
        },
        // BeforeFirst / Seek: the consumer sets seek_pos_ before the
        // ThreadedIter handshake, which orders it before this call
        [this, reader]() {
          if (reorder_reader_) {  // shuffled mode: this epoch's sub-shard order
            reader->SetSegments(EpochSegments(), EpochStops());
            reorder_reader_ = false;
          }
          reader->Seek(seek_pos_);
        });
  }

  /*!
   * \brief queue H2D transfers until every device slot is in use.  The chunk
   *  being parsed (busy_) still owns its slot: its parsed_ event has not been
   *  recorded yet, so a copy queued into that slot would not wait for it.
   */
  void FillPipeline() {
    if (replay_) {
      // HBM epoch cache: chunks are already resident, no copy and no slot
      while (static_cast<int>(inflight_.size()) < cfg_.device_slots &&
             replay_idx_ < replay_list_.size()) {
        const CachedChunk& c = cached_[replay_list_[replay_idx_]];
        size_t size = c.size, end_pos = replay_end_[replay_idx_];
        ++replay_idx_;
        // ParseAll over resident text: chunks adjacent in the arena and in
        // this epoch's order are parsed as one larger chunk (fewer launches
        // and host round trips per byte)
        // (a chunk whose text ends without EOL -- a file's unterminated last
        // line on the zero-copy path -- must stay its own chunk).  The merged
        // size doubles per chunk from replay_first_bytes: the first chunk's count +
        // scan is the only one not hidden behind a previous chunk's fill (the
        // next count runs on count_stream_ meanwhile, and next to a fill it
        // takes about half the fill's time per byte: 2x keeps it hidden)
        merge_cap_ = merge_cap_ == 0
                         ? (cfg_.replay_first_bytes != 0 ? cfg_.replay_first_bytes
                                                         : cfg_.replay_chunk_bytes)
                         : merge_cap_ * 2;
        const size_t cap =
            std::min(merge_cap_, merge_limit_ != 0 ? merge_limit_ : cfg_.replay_chunk_bytes);
        while (merge_replay_ && replay_idx_ < replay_list_.size() &&
               cached_[replay_list_[replay_idx_ - 1]].eol_end &&
               cached_[replay_list_[replay_idx_]].off == c.off + size &&
               size + cached_[replay_list_[replay_idx_]].size <= cap) {
          size += cached_[replay_list_[replay_idx_]].size;
          end_pos = replay_end_[replay_idx_];
          ++replay_idx_;
        }
        inflight_.push_back(Inflight{nullptr, -1, size, end_pos, arena_->get<char>() + c.off});
      }
      reader_done_ = replay_idx_ == replay_list_.size();
      return;
    }
    while (static_cast<int>(inflight_.size()) + busy_ < cfg_.device_slots && !reader_done_) {
      // fault points sit before a slot is taken, so a failure leaks nothing
      if (zc_ != nullptr) DMLC_FAULT_POINT("read");
      DMLC_FAULT_POINT("h2d");
      HostSlot* slot = nullptr;
      const void* src = nullptr;
      size_t size = 0, end_pos = 0;
      if (zc_ != nullptr) {
        ZeroCopySource::Piece piece;
        if (!zc_->Next(&piece)) {
          reader_done_ = true;
          if (caching_) cache_complete_ = true;
          break;
        }
        src = piece.ptr;
        size = piece.size;
        end_pos = zc_->Tell();
      } else {
        const double t0 = GetTime();
        if (!iter_.Next(&slot)) {
          reader_done_ = true;
          if (caching_) cache_complete_ = true;
          break;
        }
        stats_.wait_reader_sec += GetTime() - t0;
        src = slot->buf.get();
        size = slot->size;
        end_pos = slot->end_pos;
      }
      const int d = next_dslot_;
      next_dslot_ = (next_dslot_ + 1) % cfg_.device_slots;
      if (size + kTextPadBytes > dtext_[d]->bytes()) {
        // a chunk longer than chunk_bytes (one long record): grow this device
        // slot once the parse that last used it has finished
        parsed_[d]->Synchronize();
        dtext_[d].reset(new DeviceBuffer(size + kTextPadBytes));
        DMLC_HIP_CHECK(hipMemsetAsync(dtext_[d]->get(), 0, size + kTextPadBytes, copy_->get()));
      }
      char* dst = dtext_[d]->template get<char>();
      if (caching_) {
        // first pass of an hbm_cache epoch: the chunk lands in its arena slot
        const size_t begin_pos = cached_.empty() ? 0 : cached_.back().end_pos;
        CHECK_LE(arena_fill_ + size, arena_bytes_) << "HBM cache arena overflow";
        dst = arena_->get<char>() + arena_fill_;
        const char last = size != 0 ? static_cast<const char*>(src)[size - 1] : '\n';
        CachedChunk c{arena_fill_, size, begin_pos, end_pos, 0, begin_pos, end_pos,
                      last == '\n' || last == '\r'};
        if (cfg_.shuffle_parts > 1) {
          // the sub-shard the chunk belongs to (chunks never span two: the
          // zero-copy pieces stop at segment ends, the pinned fills at group ends)
          size_t local = 0;
          c.sub = SubOf(begin_pos, &local);
          c.sub_begin = local;
          c.sub_end = local + (end_pos - begin_pos);
          CHECK_LE(c.sub_end, sub_bytes_[c.sub]) << "internal error: a chunk spans two sub-shards";
        }
        cached_.push_back(c);
        arena_fill_ += size;
      }
      DMLC_HIP_CHECK(hipStreamWaitEvent(copy_->get(), parsed_[d]->get(), 0));
      DMLC_HIP_CHECK(hipMemcpyAsync(dst, src, size, hipMemcpyHostToDevice, copy_->get()));
      copied_[d]->Record(copy_->get());
      inflight_.push_back(Inflight{slot, d, size, end_pos, dst});
    }
  }

  void StartCaching() {
    cached_.clear();
    arena_fill_ = 0;
    cache_complete_ = false;
    if (arena_ == nullptr) {
      // + the '\n' the pinned reader inserts after a segment whose last line
      // has no EOL (one per segment at most)
      arena_bytes_ = PartitionBytes() + std::max(split_->files().size(), all_segs_.size()) + 16;
      arena_.reset(new DeviceBuffer(arena_bytes_ + kTextPadBytes));
      DMLC_HIP_CHECK(hipMemsetAsync(arena_->get(), 0, arena_bytes_ + kTextPadBytes, copy_->get()));
    }
    caching_ = true;
  }

  void DrainInflight(bool keep_prelaunch = false) {
    copy_->Synchronize();
    compute_->Synchronize();
    if (!keep_prelaunch) DropPrelaunch();
    while (!inflight_.empty()) {
      if (inflight_.front().slot != nullptr) iter_.Recycle(&inflight_.front().slot);
      inflight_.pop_front();
    }
    reader_done_ = false;
    busy_ = 0;
  }

  void ResetEpoch() {
    acc_max_index_ = acc_max_field_ = 0;
    acc_flags_ = 0;
  }

  /*! \brief the ChunkMeta a kernel wrote into mapped pinned memory (synchronises) */
  ChunkMeta WaitMapped(ChunkMeta* hm) {
    const double t0 = GetTime();
    // the publishing kernel raises hm->pad last (after a system fence): poll
    // it rather than pay a blocking stream synchronise per chunk -- a short
    // spin, then short sleeps (host_wait.h); bounded, so a kernel that never
    // publishes (a fault) still surfaces through the sync
    volatile unsigned* flag = &hm->pad;
    const bool seen = WaitHostFlag(flag, cfg_.wait_spin_us, 0.05, &wait_stats_);
    if (!seen) {
      compute_->Synchronize();
      if (count_stream_) count_stream_->Synchronize();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    stats_.wait_gpu_sec += GetTime() - t0;
    stats_.waits_spun = wait_stats_.spun;
    stats_.waits_slept = wait_stats_.slept;
    stats_.waits_timed_out = wait_stats_.timed_out;
    ChunkMeta v;
    std::memcpy(&v, const_cast<const ChunkMeta*>(hm), sizeof(v));
    *flag = 0;  // re-armed before the next publishing kernel is launched
    return v;
  }

  /*! \brief device -> host copy of `bytes` at `src` (synchronises the compute stream) */
  template <typename T>
  T ReadBack(const void* src) {
    const double t0 = GetTime();
    DMLC_HIP_CHECK(hipMemcpyAsync(hmeta_.get(), src, sizeof(T), hipMemcpyDeviceToHost,
                                  compute_->get()));
    compute_->Synchronize();
    stats_.wait_gpu_sec += GetTime() - t0;
    T v;
    std::memcpy(&v, hmeta_.get(), sizeof(T));
    return v;
  }

  /*! \brief per-chunk scratch for a chunk of nbytes (chunks may exceed chunk_bytes) */
  void EnsureScratch(size_t nbytes) {
    const size_t tiles = TileCount(nbytes);
    tcounts_.Reserve(TileScratchWords(tiles) * sizeof(uint64_t));
    tflags_.Reserve(TileScratchWords(tiles) * sizeof(uint32_t));
    tmasks_.Reserve(TileMaskWords(tiles) * sizeof(uint32_t));
    slots_.Reserve(std::max<size_t>(kMaxPartialBlocks, TileScratchSlots(tiles)) * sizeof(MetaPartial));
    tiles_.Reserve(LineIndexTiles(nbytes) * sizeof(uint64_t));
  }

  void EnsureLineBuffers(size_t nlines) {
    lines_.Reserve((nlines + 1) * sizeof(uint32_t));
    info_.Reserve((nlines + 1) * sizeof(uint64_t));
    partials_.Reserve((ScanPartials(nlines) + 2) * sizeof(uint64_t));
  }

  /*! \brief grow the output for this chunk and build the fill target */
  FillTarget<IndexType> PrepareOutput(DeviceCSR<IndexType>* out, size_t row_base, size_t nnz_base,
                                      const ChunkPlan& plan, bool need_weight, size_t nbytes) {
    hipStream_t s = compute_->get();
    const bool libfm = tcfg_.format == TextFormat::kLibFM;
    if (row_base == 0) {
      // first chunk: reserve for the whole partition from this chunk's density
      const double scale = static_cast<double>(reader_->PartitionBytes()) /
                           std::max<size_t>(nbytes, 1) * 1.05;
      out->Reserve(static_cast<size_t>(plan.nrows * scale) + 1,
                   static_cast<size_t>(plan.nnz * scale) + 1, libfm, s, 0, 0);
    }
    out->Reserve(row_base + plan.nrows, nnz_base + plan.nnz, libfm, s, row_base, nnz_base);
    if (need_weight) out->EnableWeight(s);
    if (plan.flags & kFlagQid) {
      out->EnableQid(s);
      out->has_qid_ = true;
    }
    FillTarget<IndexType> tgt;
    tgt.offset = out->offset();
    tgt.label = out->label();
    tgt.weight = out->weight_capacity() >= out->row_capacity() ? out->weight() : nullptr;
    tgt.qid = out->has_qid_ ? out->qid() : nullptr;
    tgt.field = libfm ? out->field() : nullptr;
    tgt.index = out->index();
    tgt.value = out->value();
    tgt.row_base = row_base;
    tgt.nnz_base = nnz_base;
    tgt.row_limit = row_base + plan.nrows;
    tgt.nnz_limit = nnz_base + plan.nnz;
    return tgt;
  }

  /*!
   * \brief LDS-staged tile parse (tile_kernels.hip); false when the chunk must
   *  take the exact path.  One blocking read-back (the chunk's sizes) before
   *  the fill, one for the maxima / flags after it.
   */
  /*! \brief the tile pipeline's count + scan (LibSVM / LibFM C1 + C2, or CSV S1 + scan) */
  void LaunchCountScan(const char* text, size_t nbytes, uint64_t* counts, uint32_t* flags,
                       uint32_t* masks, ChunkMeta* dmeta, ChunkMeta* hm, hipStream_t s) {
    if (tcfg_.format == TextFormat::kCSV) {
      LaunchCsvTileCount(text, nbytes, tcfg_.label_column, tcfg_.weight_column, tcfg_.delimiter,
                         counts, flags, masks, s);
      LaunchTileScanRaw(counts, flags, TileCount(nbytes), dmeta, hm, s);
    } else {
      LaunchTileCountScan(text, nbytes, counts, flags, masks, dmeta, hm, s);
    }
  }

  /*! \brief count + scan of this chunk into the current scratch set: adopt the
   *  prelaunched set when it holds this chunk, else launch them now */
  void CountScanCurrent(const char* text, size_t nbytes) {
    if (pre_.valid && pre_.text == text && pre_.nbytes == nbytes) {
      // queued behind the previous fill: take over that scratch set (its sizes
      // are published, or about to be, in hmap_next_)
      tcounts_.swap(tcounts_next_);
      tflags_.swap(tflags_next_);
      tmasks_.swap(tmasks_next_);
      meta_.swap(meta_next_);
      hmap_.swap(hmap_next_);
      pre_.valid = false;
      // the fill reads the tile prefix the other stream wrote
      DMLC_HIP_CHECK(hipStreamWaitEvent(compute_->get(), pre_done_->get(), 0));
      return;
    }
    DropPrelaunch();
    LaunchCountScan(text, nbytes, tcounts_.get<uint64_t>(), tflags_.get<uint32_t>(),
                    tmasks_.get<uint32_t>(), meta_.get<ChunkMeta>(), hmap_.get<ChunkMeta>(),
                    compute_->get());
  }

  bool FastParse(const char* text, size_t nbytes, DeviceCSR<IndexType>* out, size_t row_base,
                 size_t nnz_base, ChunkPlan* plan) {
    hipStream_t s = compute_->get();
    CountScanCurrent(text, nbytes);
    ChunkMeta* dmeta = meta_.get<ChunkMeta>();
    ChunkMeta* hm = hmap_.get<ChunkMeta>();
    const ChunkMeta sizes = WaitMapped(hm);
    AfterFirstSync();
    if (sizes.flags & kFlagIrregular) return false;
    plan->nlines = sizes.nlines;
    plan->nrows = sizes.nrows;
    plan->nnz = sizes.nnz;
    // LibSVM `qid:` tokens: the column is needed (LibFM has none: a 'q'
    // token there is irregular and the chunk goes to the exact kernels)
    if (tcfg_.format == TextFormat::kLibSVM) plan->flags |= sizes.flags & kFlagQid;
    bool need_weight = false;
    for (;;) {
      FillTarget<IndexType> tgt = PrepareOutput(out, row_base, nnz_base, *plan, need_weight, nbytes);
      if (tgt.qid != nullptr && plan->nrows != 0) {
        // rows without a `qid:` token have qid 0; the fill writes the others
        DMLC_HIP_CHECK(hipMemsetAsync(tgt.qid + row_base, 0, plan->nrows * sizeof(uint64_t), s));
      }
      LaunchTileFill<IndexType>(text, nbytes, tcfg_.format, tcounts_.get<uint64_t>(),
                                tmasks_.get<uint32_t>(), tgt,
                                slots_.get<MetaPartial>(), dmeta, hm, s);
      PrelaunchCount();
      ChunkMeta m = WaitMapped(hm);
      if (m.flags & kFlagIrregular) return false;
      if ((m.flags & kFlagNeedWeight) && !need_weight) {
        // first weighted row of the epoch: allocate the column (earlier rows
        // get 1.0) and write this chunk again with it
        need_weight = true;
        m.flags &= ~kFlagNeedWeight;
        DMLC_HIP_CHECK(hipMemcpyAsync(dmeta, &sizes, sizeof(ChunkMeta), hipMemcpyHostToDevice, s));
        continue;
      }
      CHECK(!(m.flags & kFlagNeedWeight)) << "internal error: weight column not allocated";
      Accumulate(m);
      return true;
    }
  }

  /*!
   * \brief CSV on the tile pipeline (csv_kernels.hip): lane-per-row count ->
   *  raw scan -> fill -> finish, both size read-outs through mapped pinned
   *  memory; false when the chunk must take the exact path (rows longer than
   *  the tile extension, control bytes), found by the count (S1) or, with
   *  positional counts (S1p), by the fill.
   */
  bool CsvFastParse(const char* text, size_t nbytes, DeviceCSR<IndexType>* out, size_t row_base,
                    size_t nnz_base, ChunkPlan* plan) {
    hipStream_t s = compute_->get();
    const size_t ntiles = TileCount(nbytes);
    CountScanCurrent(text, nbytes);
    ChunkMeta* dmeta = meta_.get<ChunkMeta>();
    ChunkMeta* hm = hmap_.get<ChunkMeta>();
    const ChunkMeta sizes = WaitMapped(hm);
    AfterFirstSync();
    if (sizes.flags & kFlagIrregular) return false;
    plan->nlines = sizes.nrows;
    plan->nrows = sizes.nrows;
    plan->nnz = sizes.nnz;
    const bool need_weight = tcfg_.weight_column >= 0;
    FillTarget<IndexType> tgt = PrepareOutput(out, row_base, nnz_base, *plan, need_weight, nbytes);
    LaunchCsvTileFill<IndexType>(text, nbytes, tcfg_.label_column, tcfg_.weight_column,
                                 tcfg_.delimiter, tcounts_.get<uint64_t>(),
                                 tmasks_.get<uint32_t>(), tgt,
                                 slots_.get<MetaPartial>(), s);
    LaunchTileFinish(slots_.get<MetaPartial>(), ntiles, dmeta, hm, tgt.offset, row_base, nnz_base,
                     s);
    PrelaunchCount();
    const ChunkMeta m = WaitMapped(hm);
    // with positional counts (S1p) the fill is where control bytes, crowded
    // steps and over-long rows are found: the exact kernels rewrite the chunk
    if (m.flags & kFlagIrregular) return false;
    Accumulate(m);
    return true;
  }

  /*! \brief exact wave-per-line parse (any input) */
  void ExactParse(const char* text, size_t nbytes, DeviceCSR<IndexType>* out, size_t row_base,
                  size_t nnz_base, ChunkPlan* plan, bool first_sync_done) {
    hipStream_t s = compute_->get();
    ChunkMeta* dmeta = meta_.get<ChunkMeta>();
    DMLC_HIP_CHECK(hipMemsetAsync(dmeta, 0, sizeof(ChunkMeta), s));
    LaunchLineCount(text, nbytes, tiles_.get<uint64_t>(), dmeta, s);
    plan->nlines = ReadBack<ChunkMeta>(dmeta).nlines;
    if (!first_sync_done) AfterFirstSync();
    EnsureLineBuffers(plan->nlines);
    LaunchLineEmit(text, nbytes, tiles_.get<uint64_t>(), lines_.get<uint32_t>(), s);
    LaunchTextCount(text, nbytes, lines_.get<uint32_t>(), plan->nlines, tcfg_,
                    info_.get<uint64_t>(), slots_.get<MetaPartial>(), dmeta, s);
    uint64_t* total = partials_.get<uint64_t>() + ScanPartials(plan->nlines) + 1;
    LaunchScanU64(info_.get<uint64_t>(), plan->nlines, partials_.get<uint64_t>(), total, s);
    LaunchMetaFromTotal(total, dmeta, s);
    const ChunkMeta hm = ReadBack<ChunkMeta>(dmeta);
    plan->nrows = hm.nrows;
    plan->nnz = hm.nnz;
    plan->flags = hm.flags;
    const bool csv = tcfg_.format == TextFormat::kCSV;
    const bool need_weight = (hm.flags & kFlagWeight) || (csv && tcfg_.weight_column >= 0);
    FillTarget<IndexType> tgt = PrepareOutput(out, row_base, nnz_base, *plan, need_weight, nbytes);
    DMLC_HIP_CHECK(hipMemsetAsync(dmeta, 0, sizeof(ChunkMeta), s));
    LaunchTextFill<IndexType>(text, nbytes, lines_.get<uint32_t>(), plan->nlines, tcfg_,
                              info_.get<uint64_t>(), tgt, plan->nrows, plan->nnz,
                              slots_.get<MetaPartial>(), dmeta, s);
    ChunkMeta m = ReadBack<ChunkMeta>(dmeta);
    m.flags |= plan->flags & (kFlagWeight | kFlagQid);
    if (csv && tcfg_.weight_column >= 0) m.flags |= kFlagWeight;
    Accumulate(m);
  }

  void Accumulate(const ChunkMeta& m) {
    CHECK(!(m.flags & kFlagNegIndex)) << "negative feature index in " << cfg_.format << " input";
    CHECK(!(m.flags & kFlagOverflow))
        << "internal error: GPU fill pass disagreed with the count pass (writes were dropped)";
    acc_max_index_ = std::max<uint64_t>(acc_max_index_, m.max_index);
    acc_max_field_ = std::max<uint64_t>(acc_max_field_, m.max_field);
    acc_flags_ |= m.flags;
  }

  /*!
   * \brief ParseAll over HBM-resident text: queue the next chunk's count +
   *  scan (C1 + C2) into the second scratch set right behind the current
   *  fill, so the GPU does not idle while the host reads the fill's result
   *  and turns around (~20-50 us per chunk in the trace).  The next FastParse
   *  adopts the set when its chunk is the one prelaunched.
   */
  void PrelaunchCount() {
    if (!(replay_ && merge_replay_) || pre_.valid || !cfg_.prelaunch) return;
    if (inflight_.empty()) {
      // the epoch's last chunk is being parsed: count the next epoch's first
      // one beside it (a ParseAll over the cache replays the same merge)
      if (reader_done_ && cfg_.shuffle_parts <= 1) PrelaunchNextEpoch();
      return;
    }
    const Inflight& nx = inflight_.front();
    if (nx.d >= 0) return;  // not resident (its copy would have to be waited for)
    PrelaunchFor(nx.text, nx.size);
  }

  /*!
   * \brief the next epoch's first merged chunk (replay_list_ from the start,
   *  the first merge cap FillPipeline will use), counted now on count_stream_
   *  so the next pass's first fill does not wait for its count.  A next pass
   *  that starts otherwise drops it unused (CountScanCurrent matches text and
   *  size).
   */
  void PrelaunchNextEpoch() {
    if (replay_list_.empty()) return;
    const CachedChunk& c = cached_[replay_list_[0]];
    const size_t limit = merge_limit_ != 0 ? merge_limit_ : cfg_.replay_chunk_bytes;
    const size_t first = merge_limit_ != 0 ? merge_limit_
                         : (cfg_.replay_first_bytes != 0 ? cfg_.replay_first_bytes
                                                         : cfg_.replay_chunk_bytes);
    const size_t cap = std::min(first, limit);
    size_t size = c.size;
    for (size_t i = 1; i < replay_list_.size() && cached_[replay_list_[i - 1]].eol_end &&
                       cached_[replay_list_[i]].off == c.off + size &&
                       size + cached_[replay_list_[i]].size <= cap;
         ++i) {
      size += cached_[replay_list_[i]].size;
    }
    if (size == 0) return;
    PrelaunchFor(arena_->get<char>() + c.off, size);
  }

  void PrelaunchFor(const char* text, size_t nbytes) {
    const size_t tiles = TileCount(nbytes);
    tcounts_next_.Reserve(TileScratchWords(tiles) * sizeof(uint64_t));
    tflags_next_.Reserve(TileScratchWords(tiles) * sizeof(uint32_t));
    tmasks_next_.Reserve(TileMaskWords(tiles) * sizeof(uint32_t));
    // its own stream: count + scan (HBM- and VALU-light next to the fill)
    // overlap the current fill instead of queueing behind it.  The set it
    // writes was last used by the chunk before the current one, which is done.
    LaunchCountScan(text, nbytes, tcounts_next_.get<uint64_t>(), tflags_next_.get<uint32_t>(),
                    tmasks_next_.get<uint32_t>(), meta_next_.get<ChunkMeta>(),
                    hmap_next_.get<ChunkMeta>(), count_stream_->get());
    pre_done_->Record(count_stream_->get());
    pre_.valid = true;
    pre_.text = text;
    pre_.nbytes = nbytes;
  }

  /*! \brief retire a prelaunched count nobody will adopt (its flag re-armed) */
  void DropPrelaunch() {
    if (!pre_.valid) return;
    count_stream_->Synchronize();
    static_cast<ChunkMeta*>(hmap_next_.get())->pad = 0;
    pre_.valid = false;
  }

  /*! \brief the H2D of the current chunk is complete: recycle and keep PCIe busy */
  void AfterFirstSync() {
    if (cur_slot_ != nullptr) iter_.Recycle(&cur_slot_);
    FillPipeline();
  }

  /*! \brief parse one chunk into out (append or replace); false at end */
  /*!
   * \brief pop the next device-resident chunk and run body(text, nbytes) on it
   *  (compute stream, after its H2D); false at the end.  Slot recycling and
   *  the resume cursor are handled here, also when body throws.
   */
  template <typename Body>
  bool WithNextChunk(Body body) {
    DMLC_FAULT_POINT("parse");
    FillPipeline();
    if (inflight_.empty()) return false;
    Inflight cur = inflight_.front();
    inflight_.pop_front();
    busy_ = 1;
    cur_slot_ = cur.slot;
    EnsureScratch(cur.size);
    hipStream_t s = compute_->get();
    ScopedRange range("parse_chunk");
    if (cur.d >= 0) DMLC_HIP_CHECK(hipStreamWaitEvent(s, copied_[cur.d]->get(), 0));
    try {
      body(cur.text, cur.size);
      DMLC_FAULT_POINT("parse_fill");
    } catch (...) {
      // the chunk was not delivered: the cursor stays at its start (a resume
      // from Tell() replays it), its slots go back to the pipeline.  The
      // event and busy_ are settled first, and a producer error Recycle may
      // rethrow is dropped: the parse error is the one the caller sees
      (void)hipStreamSynchronize(s);
      if (cur.d >= 0) (void)hipEventRecord(parsed_[cur.d]->get(), s);
      busy_ = 0;
      if (cur_slot_ != nullptr) {
        try {
          iter_.Recycle(&cur_slot_);
        } catch (...) {
        }
      }
      throw;
    }
    if (cur_slot_ != nullptr) iter_.Recycle(&cur_slot_);
    if (cur.d >= 0) parsed_[cur.d]->Record(s);
    busy_ = 0;
    cursor_ = cur.end_pos;  // only once the chunk is delivered
    stats_.bytes += cur.size;
    stats_.chunks += 1;
    if (zc_ != nullptr) stats_.zc_pinned_peak = zc_->PeakPinnedBytes();
    return true;
  }

  /*! \brief outcome of a one-pass chunk: written, needs the counted tile
   *  path (qid tokens), or needs the exact kernels (irregular text) */
  enum class OnePass { kDone, kCounted, kExact };

  /*!
   * \brief one-pass tile parse of a resident chunk (k_tile_fill<kOnePass>):
   *  look-back instead of C1 + C2, written straight into the target's
   *  capacity -- a single launch and one host wait per chunk.  Grows the
   *  target and runs again when the chunk did not fit (or met the first
   *  weighted row); chunks with letter-started tokens go to the counted path
   *  (`qid:` data: every later resident chunk too, see ProcessOne).
   */
  OnePass OnePassParse(const char* text, size_t nbytes, DeviceCSR<IndexType>* out, size_t row_base,
                       size_t nnz_base, ChunkPlan* plan) {
    hipStream_t s = compute_->get();
    DropPrelaunch();
    ChunkMeta* dmeta = meta_.get<ChunkMeta>();
    ChunkMeta* hm = hmap_.get<ChunkMeta>();
    const bool libfm = tcfg_.format == TextFormat::kLibFM;
    const size_t tiles = TileCount(nbytes);
    fstatus_.Reserve(tiles * sizeof(uint64_t));  // zeroed by the launcher, per launch
    if (hticket_.bytes() == 0) {
      hticket_.Reserve(sizeof(unsigned long long));
      DMLC_HIP_CHECK(hipMemsetAsync(hticket_.get(), 0, hticket_.bytes(), s));
      hticket0_ = 0;
    }
    bool first_wait = true;
    for (;;) {
      FillTarget<IndexType> tgt;
      tgt.offset = out->offset();
      tgt.label = out->label();
      tgt.weight = out->weight_capacity() >= out->row_capacity() && out->row_capacity() != 0
                       ? out->weight()
                       : nullptr;
      tgt.qid = nullptr;  // qid chunks take the counted path
      tgt.field = libfm ? out->field() : nullptr;
      tgt.index = out->index();
      tgt.value = out->value();
      tgt.row_base = row_base;
      tgt.nnz_base = nnz_base;
      // every row / entry the capacity holds (the row pointer has one slot more)
      tgt.row_limit = out->row_capacity();
      tgt.nnz_limit = out->nnz_capacity();
      if (libfm && tgt.field == nullptr) tgt.nnz_limit = 0;
      const FillOnePass op{fstatus_.get<uint64_t>(), hticket_.get<unsigned long long>(), hticket0_};
      hticket0_ += LaunchTileFill<IndexType>(text, nbytes, tcfg_.format, nullptr, nullptr, tgt,
                                             slots_.get<MetaPartial>(), dmeta, hm, s, &op);
      ChunkMeta m = WaitMapped(hm);
      if (first_wait) {
        AfterFirstSync();
        first_wait = false;
      }
      // letter-started tokens: `qid:` (the counted path writes the zeroed
      // qid column; ProcessOne makes that sticky once it finds real ones)
      // or junk (the counted path sends the chunk on to the exact kernels)
      if (m.flags & kFlagQid) return OnePass::kCounted;
      if (m.flags & kFlagIrregular) return OnePass::kExact;
      if (m.flags & kFlagOverflow) {
        // grow to the chunk's sizes -- for the whole partition at its density
        // when this is the pass's first chunk (a new target) -- and run again
        size_t want_rows = row_base + m.nrows, want_nnz = nnz_base + m.nnz;
        if (row_base == 0) {
          const double f = static_cast<double>(PartitionBytes()) / static_cast<double>(nbytes) * 1.05;
          want_rows = std::max(want_rows, static_cast<size_t>(static_cast<double>(m.nrows) * f) + 1);
          want_nnz = std::max(want_nnz, static_cast<size_t>(static_cast<double>(m.nnz) * f) + 1);
        }
        out->Reserve(want_rows, want_nnz, libfm, s, row_base, nnz_base);
        stats_.one_pass_reruns += 1;
        continue;
      }
      if ((m.flags & kFlagNeedWeight) && tgt.weight == nullptr) {
        out->EnableWeight(s);  // earlier rows get 1.0; write this chunk again with it
        stats_.one_pass_reruns += 1;
        continue;
      }
      m.flags &= ~kFlagNeedWeight;
      plan->nlines = m.nlines;
      plan->nrows = m.nrows;
      plan->nnz = m.nnz;
      Accumulate(m);
      stats_.one_pass_chunks += 1;
      return OnePass::kDone;
    }
  }

  bool ProcessOne(DeviceCSR<IndexType>* out, bool append) {
    const size_t row_base = append ? out->rows_ : 0;
    const size_t nnz_base = append ? out->nnz_ : 0;
    ChunkPlan plan;
    const bool csv = tcfg_.format == TextFormat::kCSV;
    const bool more = WithNextChunk([&](const char* text, size_t nbytes) {
      bool done = false;
      if (cfg_.fast_path) {
        // resident text (HBM replay) of a regular format: one pass, no count
        // kernel and no host turnaround between count and fill
        const OnePass r = cfg_.one_pass && !csv && replay_ && append && !one_pass_off_ && nbytes != 0
                              ? OnePassParse(text, nbytes, out, row_base, nnz_base, &plan)
                              : OnePass::kCounted;
        if (r == OnePass::kDone) {
          done = true;
        } else if (r == OnePass::kCounted) {
          done = csv ? CsvFastParse(text, nbytes, out, row_base, nnz_base, &plan)
                     : FastParse(text, nbytes, out, row_base, nnz_base, &plan);
          // qid data: every later resident chunk goes straight to this path
          if (done && replay_ && (plan.flags & kFlagQid)) one_pass_off_ = true;
        }
        if (!done) stats_.exact_chunks += 1;
      }
      if (!done) ExactParse(text, nbytes, out, row_base, nnz_base, &plan, cfg_.fast_path);
    });
    if (!more) return false;
    out->rows_ = row_base + plan.nrows;
    out->nnz_ = nnz_base + plan.nnz;
    if (acc_flags_ & kFlagWeight) out->has_weight_ = true;
    if (tcfg_.format == TextFormat::kCSV) out->has_value_ = out->nnz_ != 0;
    if (tcfg_.format == TextFormat::kLibFM) out->has_field_ = true;
    stats_.rows += plan.nrows;
    stats_.nnz += plan.nnz;
    return true;
  }

  void ParseAllHashed(DeviceHashedBatch* out, int dim, float scale, uint32_t seed,
                      bool fp8) override {
    CHECK(tcfg_.format != TextFormat::kCSV) << "hashed batches are built from LibSVM / LibFM";
    CHECK(dim > 0 && dim % 4 == 0 && dim <= 4096) << "dim must be a multiple of 4 in (0, 4096]";
    ScopedRange range("DeviceParser::ParseAllHashed");
    if (out->row_cap != 0 && (out->dim != dim || out->fp8 != fp8 || out->device != device_)) {
      *out = DeviceHashedBatch();  // a reused batch of another shape: reallocate
    }
    out->device = device_;
    out->dim = dim;
    out->fp8 = fp8;
    out->rows = 0;
    // the first chunk sizes the batch for the whole partition from its density
    // (no doubling copies of a multi-GB batch); a reused batch usually fits already
    auto reserve = [&](size_t chunk_rows, size_t nbytes) {
      if (out->rows == 0) {
        const double f = static_cast<double>(PartitionBytes()) / std::max<size_t>(nbytes, 1);
        out->Reserve(static_cast<size_t>(chunk_rows * f * 1.02) + 1, compute_->get());
      }
      out->Reserve(out->rows + chunk_rows, compute_->get());
    };
    hipStream_t s = compute_->get();
    merge_replay_ = true;  // resident text: parse adjacent cached chunks together
    struct Unmerge {
      bool* f;
      size_t* limit;
      ~Unmerge() {
        *f = false;
        *limit = 0;
      }
    } unmerge{&merge_replay_, &merge_limit_};
    // resident text and a batch that already has rows (a reused one): one pass
    // per chunk (k_tile_hash look-back, no C1 / C2) with hash_one_pass, else
    // the counted kernel; either way a merged chunk costs one host turnaround,
    // so merge up to 2 x replay_chunk_bytes from the start (measured: 1.97 ->
    // 1.91 ms per 1.49 GB pass with the whole pass in one chunk; below 2 GiB:
    // an irregular chunk falls back to the exact kernels' 32-bit offsets, as
    // DeviceParserConfig::Update checks for replay_chunk_bytes)
    const bool one_pass =
        cfg_.hash_one_pass && cfg_.fast_path && dim % 16 == 0 && replay_ && out->row_cap != 0;
    if (replay_ && out->row_cap != 0 && cfg_.fast_path && dim % 16 == 0) {
      merge_limit_ = std::min(2 * cfg_.replay_chunk_bytes, (size_t(1) << 31) - (size_t(64) << 20));
      if (merge_cap_ == 0) merge_cap_ = merge_limit_;
    }
    while (WithNextChunk([&](const char* text, size_t nbytes) {
      ChunkMeta* dmeta = meta_.get<ChunkMeta>();
      if (one_pass && nbytes != 0 && out->row_cap != 0) {
        DropPrelaunch();
        ChunkMeta* hm = hmap_.get<ChunkMeta>();
        const size_t tiles = TileCount(nbytes);
        if (hstatus_.bytes() < tiles * sizeof(uint64_t)) {
          hstatus_.Reserve(tiles * sizeof(uint64_t));
          DMLC_HIP_CHECK(hipMemsetAsync(hstatus_.get(), 0, hstatus_.bytes(), s));
        }
        if (hticket_.bytes() == 0) {
          hticket_.Reserve(sizeof(unsigned long long));
          DMLC_HIP_CHECK(hipMemsetAsync(hticket_.get(), 0, hticket_.bytes(), s));
          hticket0_ = 0;
        }
        for (;;) {
          if (++htag_ >= (1u << 30)) {  // tags wrapped: old words could match again
            htag_ = 1;
            DMLC_HIP_CHECK(hipMemsetAsync(hstatus_.get(), 0, hstatus_.bytes(), s));
          }
          const HashOnePass op{hstatus_.get<uint64_t>(), hticket_.get<unsigned long long>(),
                               hticket0_, htag_, out->row_cap};
          hticket0_ += LaunchTileHashed<IndexType>(
              text, nbytes, tcfg_.format, nullptr, nullptr, out->rows, 0, dim, scale, seed, fp8,
              out->x->get(), out->label->get<float>(), slots_.get<MetaPartial>(), dmeta, hm, s, &op);
          const ChunkMeta m = WaitMapped(hm);
          AfterFirstSync();
          CHECK(!(m.flags & kFlagNegIndex)) << "negative feature index in " << cfg_.format
                                            << " input";
          if (m.flags & kFlagIrregular) break;  // the exact kernels, below
          if (m.flags & kFlagOverflow) {
            // more rows than the batch holds: grow it, write the chunk again
            reserve(m.nrows, nbytes);
            continue;
          }
          out->rows += m.nrows;
          stats_.rows += m.nrows;
          stats_.one_pass_chunks += 1;
          return;
        }
        stats_.exact_chunks += 1;
      } else if (cfg_.fast_path && dim % 16 == 0) {
        // tile parser: C1 + C2 sizes, then the fused tile kernel builds the
        // rows of the lines each workgroup owns
        CountScanCurrent(text, nbytes);  // may adopt a prelaunched count + scan
        dmeta = meta_.get<ChunkMeta>();
        ChunkMeta* hm = hmap_.get<ChunkMeta>();
        const ChunkMeta sizes = WaitMapped(hm);
        AfterFirstSync();
        if (!(sizes.flags & kFlagIrregular)) {
          reserve(sizes.nrows, nbytes);
          LaunchTileHashed<IndexType>(text, nbytes, tcfg_.format, tcounts_.get<uint64_t>(),
                                      tmasks_.get<uint32_t>(), out->rows, sizes.nlines, dim, scale,
                                      seed, fp8, out->x->get(),
                                      out->label->get<float>(), slots_.get<MetaPartial>(), dmeta,
                                      hm, s);
          PrelaunchCount();
          const ChunkMeta m = WaitMapped(hm);
          CHECK(!(m.flags & kFlagNegIndex)) << "negative feature index in " << cfg_.format
                                            << " input";
          if (!(m.flags & kFlagIrregular)) {
            out->rows += sizes.nrows;
            stats_.rows += sizes.nrows;
            return;
          }
        }
        stats_.exact_chunks += 1;
      }
      // K1 line index, K2 row validity + K3 scan (as the exact CSR path), then
      // the fused per-line hash kernel writes rows straight into the batch
      DMLC_HIP_CHECK(hipMemsetAsync(dmeta, 0, sizeof(ChunkMeta), s));
      LaunchLineCount(text, nbytes, tiles_.get<uint64_t>(), dmeta, s);
      const size_t nlines = ReadBack<ChunkMeta>(dmeta).nlines;
      if (!(cfg_.fast_path && dim % 16 == 0)) AfterFirstSync();
      EnsureLineBuffers(nlines);
      LaunchLineEmit(text, nbytes, tiles_.get<uint64_t>(), lines_.get<uint32_t>(), s);
      LaunchTextCount(text, nbytes, lines_.get<uint32_t>(), nlines, tcfg_, info_.get<uint64_t>(),
                      slots_.get<MetaPartial>(), dmeta, s);
      uint64_t* total = partials_.get<uint64_t>() + ScanPartials(nlines) + 1;
      LaunchScanU64(info_.get<uint64_t>(), nlines, partials_.get<uint64_t>(), total, s);
      LaunchMetaFromTotal(total, dmeta, s);
      const size_t nrows = ReadBack<ChunkMeta>(dmeta).nrows;
      reserve(nrows, nbytes);
      DMLC_HIP_CHECK(hipMemsetAsync(dmeta, 0, sizeof(ChunkMeta), s));
      LaunchTextHashed<IndexType>(text, nbytes, lines_.get<uint32_t>(), nlines, tcfg_.format,
                                  info_.get<uint64_t>(), out->rows, dim, scale, seed, fp8,
                                  out->x->get(), out->label->get<float>(), slots_.get<MetaPartial>(),
                                  dmeta, s);
      const ChunkMeta m = ReadBack<ChunkMeta>(dmeta);
      CHECK(!(m.flags & kFlagNegIndex)) << "negative feature index in " << cfg_.format << " input";
      out->rows += nrows;
      stats_.rows += nrows;
    })) {
    }
    compute_->Synchronize();
  }

  /*! \brief publish the accumulated max / flags of this epoch */
  void FinishEpoch(DeviceCSR<IndexType>* out) {
    out->max_index_ = std::max<uint64_t>(out->max_index_, acc_max_index_);
    out->max_field_ = std::max<uint64_t>(out->max_field_, acc_max_field_);
    if (acc_flags_ & kFlagValue) out->has_value_ = true;
    if (acc_flags_ & kFlagWeight) out->has_weight_ = true;
    if (out->rows_ == 0) {
      // keep a valid (zero) closing offset for empty partitions
      out->Reserve(1, 1, false, compute_->get());
      DMLC_HIP_CHECK(hipMemsetAsync(out->offset(), 0, sizeof(uint64_t), compute_->get()));
    }
    compute_->Synchronize();
  }

  DeviceParserConfig cfg_;
  TextParseConfig tcfg_;
  int device_{0};
  std::unique_ptr<io::InputSplitBase> split_;
  std::unique_ptr<io::ShardReader> reader_;
  std::unique_ptr<Stream> compute_, copy_;
  std::vector<std::unique_ptr<DeviceBuffer>> dtext_;
  std::vector<std::unique_ptr<Event>> copied_, parsed_;
  DeviceBuffer tiles_, lines_, info_, partials_, meta_;
  /*! \brief tile parser scratch: per-tile counts (scanned in place) and flags */
  DeviceBuffer tcounts_, tflags_, tmasks_;
  // the prelaunched next chunk's C1 + C2 scratch (hbm_cache ParseAll only)
  DeviceBuffer tcounts_next_, tflags_next_, tmasks_next_, meta_next_;
  PinnedBuffer hmap_next_;
  std::unique_ptr<Stream> count_stream_;  // prelaunched counts (hbm_cache only)
  std::unique_ptr<Event> pre_done_;
  struct Prelaunch {
    bool valid{false};
    const char* text{nullptr};
    size_t nbytes{0};
  } pre_;
  /*! \brief per-workgroup reduction slots (MetaPartial) */
  DeviceBuffer slots_;
  PinnedBuffer hmeta_;
  /*! \brief mapped pinned ChunkMeta the tile kernels write directly */
  PinnedBuffer hmap_;
  ThreadedIter<HostSlot> iter_;
  std::unique_ptr<ZeroCopySource> zc_;
  std::deque<Inflight> inflight_;
  /*! \brief HBM epoch cache (cfg_.hbm_cache): the partition's chunks, resident */
  std::unique_ptr<DeviceBuffer> arena_;
  size_t arena_bytes_{0}, arena_fill_{0}, replay_idx_{0};
  /*! \brief merged replay chunk cap of the pass (0: the next is the first) */
  size_t merge_cap_{0};
  size_t merge_limit_{0};  // merged replay chunk limit (0: replay_chunk_bytes)
  // one-pass hashed batches: look-back words, workgroup tickets, launch tag
  DeviceBuffer hstatus_, hticket_;
  // one-pass CSR fill: look-back words (zeroed per launch; tickets shared)
  DeviceBuffer fstatus_;
  /*! \brief qid data met: resident chunks take the counted tile path */
  bool one_pass_off_{false};
  unsigned long long hticket0_{0};
  uint32_t htag_{0};
  std::vector<CachedChunk> cached_;
  bool caching_{false}, cache_complete_{false}, replay_{false}, merge_replay_{false};
  HostSlot* cur_slot_{nullptr};
  /*! \brief resume cursor (partition offset after the last delivered chunk) */
  size_t cursor_{0};
  // shuffled mode (cfg_.shuffle_parts > 1)
  unsigned part_{0}, nparts_{1}, epoch_{0};
  std::vector<unsigned> order_{0};
  std::vector<io::InputSplitBase::Segment> all_segs_;  // sub-shard 0's, 1's, ...
  std::vector<size_t> sub_first_, sub_bytes_, sub_pos_;
  std::vector<size_t> replay_list_, replay_begin_, replay_end_;
  bool reorder_reader_{false};
  /*! \brief where the reader restarts on the next BeforeFirst handshake */
  size_t seek_pos_{0};
  int next_dslot_{0};
  int busy_{0};
  bool reader_done_{false};
  uint64_t acc_max_index_{0}, acc_max_field_{0};
  unsigned acc_flags_{0};
  DeviceCSR<IndexType> block_;
  DeviceRowBlock<IndexType> view_;
  DeviceParserStats stats_;
  HostWaitStats wait_stats_;
};

}  // namespace

template <typename IndexType>
DeviceParser<IndexType>* DeviceParser<IndexType>::Create(const std::string& uri,
                                                         unsigned part_index, unsigned num_parts,
                                                         const DeviceParserConfig& cfg) {
  io::URISpec spec(uri, part_index, num_parts);
  DeviceParserConfig c = cfg;
  c.Update(spec.args);
  return new DeviceParserImpl<IndexType>(spec.uri, part_index, num_parts, c);
}

template class DeviceParser<uint32_t>;
template class DeviceParser<uint64_t>;

}  // namespace gpu
}  // namespace dmlc
