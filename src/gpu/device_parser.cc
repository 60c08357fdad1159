/*!
 * \file src/gpu/device_parser.cc
 * \brief The MI355X ingestion pipeline (see dmlc/gpu/device_parser.h).
 *
 * Per chunk, in stream order:
 *   copy stream    : wait(parsed[d]) -> H2D(text[d]) -> record(copied[d])
 *   compute stream : wait(copied[d]) -> K1a line count + scan
 *                    [host reads nlines]  -> K1b emit, K2 count, K3 scan
 *                    [host reads nrows/nnz/flags, sizes the output]
 *                    -> K4 fill (+K8) -> record(parsed[d])
 * H2D of chunk k+1 is queued before chunk k is parsed, so PCIe transfers
 * overlap the kernels; the reader thread fills pinned slots further ahead.
 */
#include <dmlc/gpu/device_parser.h>
#include <dmlc/logging.h>
#include <dmlc/threadediter.h>
#include <dmlc/timer.h>

#include <cstdlib>
#include <deque>
#include <memory>
#include <vector>

#include "../io/filesys.h"
#include "../io/line_split.h"
#include "../io/shard_reader.h"
#include "../io/uri_spec.h"
#include "./kernels.h"

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
    }
  }
  chunk_bytes = (chunk_bytes + 4095) & ~size_t(4095);
  CHECK_GE(chunk_bytes, 4096U) << "chunk_bytes too small";
  CHECK_LT(chunk_bytes, size_t(1) << 32) << "chunk_bytes must be < 4 GiB";
  CHECK_GE(pinned_slots, 1);
  CHECK_GE(device_slots, 1);
}

namespace {

/*! \brief a filled pinned host slot */
struct HostSlot {
  PinnedBuffer buf;
  size_t size{0};
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
    tcfg_.label_column = cfg_.label_column;
    tcfg_.weight_column = cfg_.weight_column;
    tcfg_.delimiter = cfg_.delimiter;
    io::URI path(uri.c_str());
    split_.reset(new io::LineSplitter(io::FileSystem::GetInstance(path), uri.c_str(), part, nparts));
    reader_.reset(new io::ShardReader(split_.get(), cfg_.read_threads));
    compute_.reset(new Stream());
    copy_.reset(new Stream());
    for (int d = 0; d < cfg_.device_slots; ++d) {
      dtext_.emplace_back(new DeviceBuffer(cfg_.chunk_bytes + kTextPadBytes));
      copied_.emplace_back(new Event());
      parsed_.emplace_back(new Event());
      parsed_.back()->Record(compute_->get());
    }
    tiles_.Reserve(LineIndexTiles(cfg_.chunk_bytes) * sizeof(uint64_t));
    meta_.Reserve(2 * sizeof(ChunkMeta));
    hmeta_.Reserve(2 * sizeof(ChunkMeta));
    iter_.set_max_capacity(static_cast<size_t>(cfg_.pinned_slots));
    StartReader();
  }

  ~DeviceParserImpl() override {
    // make sure no transfer still reads a pinned slot we are about to free;
    // destructors never throw, so errors are ignored here
    if (copy_) (void)hipStreamSynchronize(copy_->get());
    if (compute_) (void)hipStreamSynchronize(compute_->get());
    for (auto& f : inflight_) iter_.Recycle(&f.slot);
    inflight_.clear();
    iter_.Destroy();
  }

  void BeforeFirst() override {
    DrainInflight();
    iter_.BeforeFirst();
  }

  bool Next() override {
    block_.Clear();
    block_.device_ = device_;
    if (!ProcessOne(&block_, /*append=*/false)) return false;
    FinishEpochMeta(&block_);
    view_ = block_.View();
    return true;
  }

  const DeviceRowBlock<IndexType>& Value() const override { return view_; }

  void ParseAll(DeviceCSR<IndexType>* out) override {
    ScopedRange range("DeviceParser::ParseAll");
    out->device_ = device_;
    ResetAccum();
    while (ProcessOne(out, /*append=*/true)) {
    }
    FinishEpochMeta(out);
  }

  size_t PartitionBytes() const override { return reader_->PartitionBytes(); }
  const DeviceParserStats& Stats() const override { return stats_; }
  hipStream_t stream() const override { return compute_->get(); }

 private:
  struct Inflight {
    HostSlot* slot;
    int d;
  };

  void StartReader() {
    const size_t cap = cfg_.chunk_bytes;
    io::ShardReader* reader = reader_.get();
    iter_.Init(
        [reader, cap](HostSlot** dptr) {
          if (*dptr == nullptr) {
            *dptr = new HostSlot();
            (*dptr)->buf.Reserve(cap + kTextPadBytes);
          }
          ScopedRange r("pinned_fill");
          (*dptr)->size = reader->Fill((*dptr)->buf.template get<char>(), cap);
          return (*dptr)->size != 0;
        },
        [reader]() { reader->Reset(); });
  }

  /*!
   * \brief queue H2D transfers until every device slot is in use.  The chunk
   *  being parsed (busy_) still owns its slot: its parsed_ event has not been
   *  recorded yet, so a copy queued into that slot would not wait for it.
   */
  void FillPipeline() {
    while (static_cast<int>(inflight_.size()) + busy_ < cfg_.device_slots && !reader_done_) {
      HostSlot* slot = nullptr;
      const double t0 = GetTime();
      if (!iter_.Next(&slot)) {
        reader_done_ = true;
        break;
      }
      stats_.wait_reader_sec += GetTime() - t0;
      const int d = next_dslot_;
      next_dslot_ = (next_dslot_ + 1) % cfg_.device_slots;
      // the device slot is free once its previous chunk has been parsed
      DMLC_HIP_CHECK(hipStreamWaitEvent(copy_->get(), parsed_[d]->get(), 0));
      DMLC_HIP_CHECK(hipMemcpyAsync(dtext_[d]->get(), slot->buf.get(), slot->size,
                                    hipMemcpyHostToDevice, copy_->get()));
      copied_[d]->Record(copy_->get());
      inflight_.push_back(Inflight{slot, d});
    }
  }

  void DrainInflight() {
    copy_->Synchronize();
    compute_->Synchronize();
    while (!inflight_.empty()) {
      iter_.Recycle(&inflight_.front().slot);
      inflight_.pop_front();
    }
    reader_done_ = false;
  }

  void ResetAccum() {
    DMLC_HIP_CHECK(hipMemsetAsync(meta_.get<ChunkMeta>() + 1, 0, sizeof(ChunkMeta), compute_->get()));
  }

  /*! \brief copy device meta[which] to host (synchronising the compute stream) */
  const ChunkMeta& ReadMeta(int which) {
    const double t0 = GetTime();
    DMLC_HIP_CHECK(hipMemcpyAsync(hmeta_.get<ChunkMeta>() + which, meta_.get<ChunkMeta>() + which,
                                  sizeof(ChunkMeta), hipMemcpyDeviceToHost, compute_->get()));
    compute_->Synchronize();
    stats_.wait_gpu_sec += GetTime() - t0;
    return hmeta_.get<ChunkMeta>()[which];
  }

  /*! \brief parse one chunk into out (append or replace); false at end */
  bool ProcessOne(DeviceCSR<IndexType>* out, bool append) {
    FillPipeline();
    if (inflight_.empty()) return false;
    Inflight cur = inflight_.front();
    inflight_.pop_front();
    busy_ = 1;
    const size_t nbytes = cur.slot->size;
    const char* text = dtext_[cur.d]->template get<char>();
    hipStream_t s = compute_->get();
    ChunkMeta* dmeta = meta_.get<ChunkMeta>();
    ChunkMeta* accum = dmeta + 1;
    if (!append) ResetAccum();
    ScopedRange range("parse_chunk");
    DMLC_HIP_CHECK(hipStreamWaitEvent(s, copied_[cur.d]->get(), 0));
    DMLC_HIP_CHECK(hipMemsetAsync(dmeta, 0, sizeof(ChunkMeta), s));
    // K1a: count lines
    LaunchLineCount(text, nbytes, tiles_.get<uint64_t>(), dmeta, s);
    const size_t nlines = ReadMeta(0).nlines;
    // the H2D of this chunk is complete (the compute stream waited for it)
    iter_.Recycle(&cur.slot);
    // keep PCIe busy while we parse
    FillPipeline();
    lines_.Reserve((nlines + 1) * sizeof(uint32_t));
    info_.Reserve((nlines + 1) * sizeof(uint64_t));
    partials_.Reserve((ScanPartials(nlines) + 2) * sizeof(uint64_t));
    LaunchLineEmit(text, nbytes, tiles_.get<uint64_t>(), lines_.get<uint32_t>(), s);
    LaunchTextCount(text, nbytes, lines_.get<uint32_t>(), nlines, tcfg_, info_.get<uint64_t>(),
                    dmeta, s);
    uint64_t* total = partials_.get<uint64_t>() + ScanPartials(nlines) + 1;
    LaunchScanU64(info_.get<uint64_t>(), nlines, partials_.get<uint64_t>(), total, s);
    LaunchMetaFromTotal(total, dmeta, s);
    const ChunkMeta hm = ReadMeta(0);
    // size the output
    const size_t row_base = append ? out->rows_ : 0;
    const size_t nnz_base = append ? out->nnz_ : 0;
    const bool libfm = tcfg_.format == TextFormat::kLibFM;
    if (append && out->rows_ == 0 && stats_.bytes == 0) {
      // first chunk of a resident parse: reserve for the whole partition
      const double scale = static_cast<double>(reader_->PartitionBytes()) /
                           std::max<size_t>(nbytes, 1) * 1.05;
      out->Reserve(static_cast<size_t>(hm.nrows * scale) + 1,
                   static_cast<size_t>(hm.nnz * scale) + 1, libfm, s, 0, 0);
    }
    out->Reserve(row_base + hm.nrows, nnz_base + hm.nnz, libfm, s, row_base, nnz_base);
    const bool csv = tcfg_.format == TextFormat::kCSV;
    if ((hm.flags & kFlagWeight) || (csv && tcfg_.weight_column >= 0)) {
      out->EnableWeight(s);
      out->has_weight_ = true;
    }
    if (hm.flags & kFlagQid) {
      out->EnableQid(s);
      out->has_qid_ = true;
    }
    FillTarget<IndexType> tgt;
    tgt.offset = out->offset();
    tgt.label = out->label();
    tgt.weight = out->has_weight_ ? out->weight() : nullptr;
    tgt.qid = out->has_qid_ ? out->qid() : nullptr;
    tgt.field = libfm ? out->field() : nullptr;
    tgt.index = out->index();
    tgt.value = out->value();
    tgt.row_base = row_base;
    tgt.nnz_base = nnz_base;
    tgt.row_limit = row_base + hm.nrows;
    tgt.nnz_limit = nnz_base + hm.nnz;
    LaunchTextFill<IndexType>(text, nbytes, lines_.get<uint32_t>(), nlines, tcfg_,
                              info_.get<uint64_t>(), tgt, hm.nrows, hm.nnz, accum, s);
    parsed_[cur.d]->Record(s);
    busy_ = 0;
    out->rows_ = row_base + hm.nrows;
    out->nnz_ = nnz_base + hm.nnz;
    if (csv) out->has_value_ = out->nnz_ != 0;
    if (libfm) out->has_field_ = true;
    stats_.bytes += nbytes;
    stats_.chunks += 1;
    stats_.rows += hm.nrows;
    stats_.nnz += hm.nnz;
    return true;
  }

  /*! \brief read the accumulated max/flags after the last fill */
  void FinishEpochMeta(DeviceCSR<IndexType>* out) {
    const ChunkMeta& acc = ReadMeta(1);
    CHECK(!(acc.flags & kFlagNegIndex)) << "negative feature index in " << cfg_.format << " input";
    CHECK(!(acc.flags & kFlagOverflow))
        << "internal error: GPU fill pass disagreed with the count pass (writes were dropped)";
    out->max_index_ = std::max<uint64_t>(out->max_index_, acc.max_index);
    out->max_field_ = std::max<uint64_t>(out->max_field_, acc.max_field);
    if (acc.flags & kFlagValue) out->has_value_ = true;
    if (out->rows_ == 0) {
      // keep a valid (zero) closing offset for empty partitions
      out->Reserve(1, 1, false, compute_->get());
      DMLC_HIP_CHECK(hipMemsetAsync(out->offset(), 0, sizeof(uint64_t), compute_->get()));
      compute_->Synchronize();
    }
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
  PinnedBuffer hmeta_;
  ThreadedIter<HostSlot> iter_;
  std::deque<Inflight> inflight_;
  int next_dslot_{0};
  int busy_{0};
  bool reader_done_{false};
  DeviceCSR<IndexType> block_;
  DeviceRowBlock<IndexType> view_;
  DeviceParserStats stats_;
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
