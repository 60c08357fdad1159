/*!
 * \file src/gpu/device_recordio.cc
 * \brief DeviceRecordIOReader (see dmlc/gpu/device_recordio.h).
 *
 * Per chunk, in stream order:
 *   copy stream    : wait(parsed[d]) -> H2D(text[d]) -> record(copied[d])
 *   compute stream : wait(copied[d]) -> K7a count+scan -> [host: nrec]
 *                    -> K7b emit -> K7c lengths -> K3 scan -> [host: bytes, err]
 *                    -> K7d gather -> record(parsed[d])
 * The H2D of the next chunks is queued before the current chunk is decoded.
 */
#include <dmlc/fault.h>
#include <dmlc/gpu/device_recordio.h>
#include <dmlc/gpu/hip_utils.h>
#include <dmlc/logging.h>
#include <dmlc/timer.h>

#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <vector>

#include "../io/filesys.h"
#include "../io/recordio_split.h"
#include "../io/uri_spec.h"
#include "./kernels.h"
#include "./zero_copy_source.h"

namespace dmlc {
namespace gpu {

void DeviceRecordIOConfig::Update(const std::map<std::string, std::string>& args) {
  for (const auto& kv : args) {
    if (kv.first == "chunk_mb") {
      chunk_bytes = static_cast<size_t>(std::atof(kv.second.c_str()) * (1 << 20));
    } else if (kv.first == "chunk_bytes") {
      chunk_bytes = std::strtoull(kv.second.c_str(), nullptr, 10);
    } else if (kv.first == "device") {
      device = std::atoi(kv.second.c_str());
    } else if (kv.first == "zero_copy") {
      const std::string& v = kv.second;
      zero_copy = (v == "auto" || v == "-1") ? -1 : ((v == "0" || v == "false") ? 0 : 1);
    }
  }
  chunk_bytes = (chunk_bytes + 4095) & ~size_t(4095);
  CHECK_GE(chunk_bytes, 4096U);
  CHECK_LT(chunk_bytes, size_t(1) << 34) << "chunk_bytes must be < 16 GiB (u32 word positions)";
}

namespace {

constexpr int kSlots = 2;

class DeviceRecordIOImpl : public DeviceRecordIOReader {
 public:
  DeviceRecordIOImpl(const std::string& uri, unsigned part, unsigned nparts,
                     const DeviceRecordIOConfig& cfg)
      : cfg_(cfg) {
    if (cfg_.device >= 0) SetDevice(cfg_.device);
    io::URI path(uri.c_str());
    split_.reset(new io::RecordIOSplitter(io::FileSystem::GetInstance(path), uri.c_str(), part,
                                          nparts));
    if (cfg_.zero_copy != 0) {
      zc_.reset(new ZeroCopySource(ZeroCopySource::Cut::kRecordIO));
      zc_->SetDrain([this]() { (void)hipStreamSynchronize(copy_.get()); });
      if (!zc_->Init(split_.get(), cfg_.chunk_bytes)) {
        CHECK_NE(cfg_.zero_copy, 1) << "zero_copy=1 but mmap/hipHostRegister failed";
        zc_.reset();
      }
    }
    stats_.zero_copy = zc_ != nullptr;
    if (zc_ == nullptr) split_->HintChunkSize(cfg_.chunk_bytes);
    for (int d = 0; d < kSlots; ++d) {
      slots_[d].text.Reserve(cfg_.chunk_bytes + 16);
      if (zc_ == nullptr) slots_[d].staging.Reserve(cfg_.chunk_bytes + 16);
    }
    host_.Reserve(4 * sizeof(uint64_t));
    scratch_.Reserve(3 * sizeof(uint64_t));
  }
  ~DeviceRecordIOImpl() override {
    (void)hipStreamSynchronize(copy_.get());
    (void)hipStreamSynchronize(compute_.get());
  }

  void BeforeFirst() override {
    DrainInflight();
    if (zc_ != nullptr) {
      zc_->Reset();
    } else {
      split_->BeforeFirst();
    }
    exhausted_ = false;
    resident_rows_ = resident_bytes_ = 0;
  }

  bool Next() override {
    FillPipeline();
    if (inflight_.empty()) return false;
    const int d = inflight_.front();
    inflight_.pop_front();
    ProcessOne(d, false);
    return true;
  }
  const DeviceRecordBatch& Value() const override { return batch_; }

  const DeviceRecordBatch& ReadAll() override {
    resident_rows_ = resident_bytes_ = 0;
    res_off_.Grow(sizeof(uint64_t), 0, compute_.get());
    DMLC_HIP_CHECK(hipMemsetAsync(res_off_.get<uint64_t>(), 0, sizeof(uint64_t), compute_.get()));
    for (;;) {
      FillPipeline();
      if (inflight_.empty()) break;
      const int d = inflight_.front();
      inflight_.pop_front();
      ProcessOne(d, true);
    }
    DMLC_HIP_CHECK(hipStreamSynchronize(compute_.get()));
    resident_.size = resident_rows_;
    resident_.bytes = resident_bytes_;
    resident_.offset = res_off_.get<uint64_t>();
    resident_.data = res_data_.get<uint8_t>();
    return resident_;
  }

  size_t PartitionBytes() const override {
    if (zc_ != nullptr) return zc_->PartitionBytes();
    return split_->offset_end() - split_->offset_begin();
  }
  const DeviceRecordIOStats& Stats() const override { return stats_; }
  hipStream_t stream() const override { return compute_.get(); }

 private:
  struct Slot {
    DeviceBuffer text;
    PinnedBuffer staging;
    Event copied, parsed;
    size_t size{0};
    bool used{false};
  };

  /*! \brief queue H2D copies of the next chunks into free device slots */
  void FillPipeline() {
    while (!exhausted_ && static_cast<int>(inflight_.size()) < kSlots) {
      DMLC_FAULT_POINT("recordio");
      const int d = next_slot_;
      Slot& s = slots_[d];
      const char* src = nullptr;
      size_t n = 0;
      if (zc_ != nullptr) {
        ZeroCopySource::Piece piece;
        if (!zc_->Next(&piece)) {
          exhausted_ = true;
          break;
        }
        src = piece.ptr;
        n = piece.size;
      } else {
        InputSplit::Blob blob;
        if (!split_->NextChunk(&blob)) {
          exhausted_ = true;
          break;
        }
        if (blob.size + 16 > s.text.bytes() || blob.size + 16 > s.staging.bytes()) {
          // the split's chunks can exceed the hint: grow this slot once both
          // streams no longer touch it
          DMLC_HIP_CHECK(hipStreamSynchronize(copy_.get()));
          DMLC_HIP_CHECK(hipStreamSynchronize(compute_.get()));
          s.text.Reserve(blob.size + 16);
          s.staging.Reserve(blob.size + 16);
        }
        if (s.used) s.copied.Synchronize();  // staging[d] free again
        std::memcpy(s.staging.get<char>(), blob.dptr, blob.size);
        src = s.staging.get<char>();
        n = blob.size;
      }
      CHECK_EQ(n % 4, 0U) << "RecordIO chunk not 4-byte aligned";
      if (n + 16 > s.text.bytes()) {
        // a zero-copy piece holding one record longer than chunk_bytes
        DMLC_HIP_CHECK(hipStreamSynchronize(copy_.get()));
        DMLC_HIP_CHECK(hipStreamSynchronize(compute_.get()));
        s.text.Reserve(n + 16);
      }
      if (s.used) DMLC_HIP_CHECK(hipStreamWaitEvent(copy_.get(), s.parsed.get(), 0));
      DMLC_HIP_CHECK(hipMemcpyAsync(s.text.get<char>(), src, n, hipMemcpyHostToDevice, copy_.get()));
      s.copied.Record(copy_.get());
      s.size = n;
      s.used = true;
      inflight_.push_back(d);
      next_slot_ = (next_slot_ + 1) % kSlots;
      stats_.bytes += n;
    }
  }

  void DrainInflight() {
    inflight_.clear();
    DMLC_HIP_CHECK(hipStreamSynchronize(copy_.get()));
    DMLC_HIP_CHECK(hipStreamSynchronize(compute_.get()));
  }

  void SyncCompute() {
    double t0 = GetTime();
    DMLC_HIP_CHECK(hipStreamSynchronize(compute_.get()));
    stats_.wait_gpu_sec += GetTime() - t0;
  }

  void ProcessOne(int d, bool resident) {
    Slot& s = slots_[d];
    hipStream_t st = compute_.get();
    DMLC_HIP_CHECK(hipStreamWaitEvent(st, s.copied.get(), 0));
    const uint32_t* words = s.text.get<uint32_t>();
    const size_t nwords = s.size / 4;
    const size_t tiles = RecordIOTiles(nwords);
    tiles_.Reserve((tiles + 1) * sizeof(uint64_t));
    partials_.Reserve((ScanPartials(std::max<size_t>(tiles, 1)) + 1) * sizeof(uint64_t));
    uint64_t* dev = scratch_.get<uint64_t>();  // [0] nrec, [1] err
    DMLC_HIP_CHECK(hipMemsetAsync(dev, 0, 2 * sizeof(uint64_t), st));
    LaunchRecordIOCount(words, nwords, tiles_.get<uint64_t>(), partials_.get<uint64_t>(), dev, st);
    DMLC_HIP_CHECK(hipMemcpyAsync(host_.get<uint64_t>(), dev, sizeof(uint64_t),
                                  hipMemcpyDeviceToHost, st));
    SyncCompute();
    const size_t nrec = host_.get<uint64_t>()[0];
    head_.Reserve(std::max<size_t>(nrec, 1) * sizeof(uint32_t));
    len_.Reserve((nrec + 1) * sizeof(uint64_t));
    partials_.Reserve((ScanPartials(std::max<size_t>(nrec, 1)) + 1) * sizeof(uint64_t));
    uint64_t* rec_len = len_.get<uint64_t>();
    uint32_t* err = reinterpret_cast<uint32_t*>(dev + 1);
    LaunchRecordIOEmit(words, nwords, tiles_.get<uint64_t>(), head_.get<uint32_t>(), st);
    LaunchRecordIOLengths(words, nwords, head_.get<uint32_t>(), nrec, rec_len, err, st);
    if (nrec > 0) {
      LaunchScanU64(rec_len, nrec, partials_.get<uint64_t>(), rec_len + nrec, st);
    } else {
      DMLC_HIP_CHECK(hipMemsetAsync(rec_len, 0, sizeof(uint64_t), st));
    }
    DMLC_HIP_CHECK(hipMemcpyAsync(host_.get<uint64_t>() + 1, rec_len + nrec, sizeof(uint64_t),
                                  hipMemcpyDeviceToHost, st));
    DMLC_HIP_CHECK(hipMemcpyAsync(host_.get<uint64_t>() + 2, dev + 1, sizeof(uint64_t),
                                  hipMemcpyDeviceToHost, st));
    SyncCompute();
    const size_t bytes = host_.get<uint64_t>()[1];
    const uint32_t e = static_cast<uint32_t>(host_.get<uint64_t>()[2]);
    CHECK_EQ(e & kRecErrTruncated, 0U) << "RecordIO: a record runs past its chunk (corrupt file?)";
    CHECK_EQ(e & kRecErrBadPart, 0U) << "RecordIO: malformed multi-part record";
    if (!resident) {
      out_.Reserve(std::max<size_t>(bytes, 1));
      LaunchRecordIOGather(words, nwords, head_.get<uint32_t>(), nrec, rec_len, out_.get<uint8_t>(),
                           st);
      batch_.size = nrec;
      batch_.bytes = bytes;
      batch_.offset = rec_len;
      batch_.data = out_.get<uint8_t>();
    } else {
      GrowResident(nrec, bytes);
      LaunchOffsetRebase(rec_len, nrec, 0, resident_bytes_,
                         res_off_.get<uint64_t>() + resident_rows_, st);
      LaunchRecordIOGather(words, nwords, head_.get<uint32_t>(), nrec, rec_len,
                           res_data_.get<uint8_t>() + resident_bytes_, st);
      resident_rows_ += nrec;
      resident_bytes_ += bytes;
    }
    s.parsed.Record(st);
    stats_.chunks += 1;
    stats_.records += nrec;
  }

  void GrowResident(size_t nrec, size_t bytes) {
    const size_t need_off = (resident_rows_ + nrec + 1) * sizeof(uint64_t);
    if (need_off > res_off_.bytes()) {
      res_off_.Grow(need_off + need_off / 2, (resident_rows_ + 1) * sizeof(uint64_t),
                    compute_.get());
    }
    const size_t need_data = resident_bytes_ + bytes;
    if (need_data > res_data_.bytes()) {
      res_data_.Grow(need_data + need_data / 2, resident_bytes_, compute_.get());
    }
  }

  DeviceRecordIOConfig cfg_;
  std::unique_ptr<io::RecordIOSplitter> split_;
  std::unique_ptr<ZeroCopySource> zc_;
  Stream copy_, compute_;
  Slot slots_[kSlots];
  std::deque<int> inflight_;
  int next_slot_{0};
  bool exhausted_{false};
  DeviceBuffer tiles_, partials_, head_, len_, out_, scratch_;
  DeviceBuffer res_off_, res_data_;
  PinnedBuffer host_;
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
