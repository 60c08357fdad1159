/*!
 * \file src/gpu/device_row_iter.cc
 * \brief The reference's public data API on the MI355X path:
 *  `Parser<I>::Create(uri + "?device=gpu", part, nparts, type)` and
 *  `RowBlockIter<I>::Create(...)` (reference include/dmlc/data.h:246-311,
 *  src/data.cc:62-107) return parsers whose text is tokenised by the HIP
 *  kernels of DeviceParser.
 *
 *  URI arguments (besides every DeviceParserConfig key):
 *    device=gpu | gpu:<k>   route to the GPU path (current device / device k)
 *    device_ptrs=1          (or to_host=0) serve the HBM-resident blocks: the
 *                           RowBlock's pointers are DEVICE pointers (stream-
 *                           ordered and ready when Next() returns), `offset`
 *                           is 64-bit.  Default: every block is copied back
 *                           into host memory, so code written against the
 *                           reference's host RowBlock API (Row access, SGD
 *                           loops) runs unchanged and never dereferences a
 *                           device pointer by accident.
 *  GPUParser<I>   : one block per chunk (the reference's ThreadedParser shape).
 *  DeviceRowIter<I>: the whole partition parsed into one HBM-resident CSR
 *                   (ParseAll), served as a single block (also when it is
 *                   empty), NumCol = max index + 1 (the reference's
 *                   BasicRowIter, src/data/basic_row_iter.h:35-48).  With
 *                   `uri#cachefile` it is DiskRowIter's device twin: the
 *                   page file is DMA'd into HBM when it exists, else built
 *                   from the GPU parse (gpu/device_page_cache.h).
 */
#include <dmlc/data.h>
#include <dmlc/gpu/device_page_cache.h>
#include <dmlc/gpu/device_parser.h>
#include <dmlc/logging.h>

#include <cstdlib>
#include <map>
#include <memory>
#include <string>

#include "../data/device_route.h"

namespace dmlc {
namespace data {

namespace {

struct RouteArgs {
  gpu::DeviceParserConfig cfg;
  bool to_host{true};
};

RouteArgs ParseRoute(const std::map<std::string, std::string>& args, const std::string& type) {
  RouteArgs r;
  std::map<std::string, std::string> rest;
  for (const auto& kv : args) {
    if (kv.first == "device") {
      const std::string& v = kv.second;
      CHECK(v.compare(0, 3, "gpu") == 0) << "device=" << v << ": expected gpu or gpu:<k>";
      r.cfg.device = v.size() > 4 && v[3] == ':' ? std::atoi(v.c_str() + 4) : -1;
    } else if (kv.first == "to_host") {
      r.to_host = kv.second != "0" && kv.second != "false";
    } else if (kv.first == "device_ptrs") {
      r.to_host = kv.second == "0" || kv.second == "false";
    } else if (kv.first != "format" && kv.first != "nthread") {
      rest.insert(kv);
    }
  }
  r.cfg.format = type;
  r.cfg.Update(rest);
  return r;
}

/*! \brief RowBlock over a device block (device pointers) */
template <typename IndexType>
RowBlock<IndexType> DeviceView(const gpu::DeviceRowBlock<IndexType>& d) {
  static_assert(sizeof(size_t) == sizeof(uint64_t), "RowBlock::offset aliases the u64 offsets");
  RowBlock<IndexType> b;
  b.size = d.size;
  b.offset = reinterpret_cast<const size_t*>(d.offset);
  b.label = d.label;
  b.weight = d.weight;
  b.qid = d.qid;
  b.field = d.field;
  b.index = d.index;
  b.value = d.value;
  return b;
}

template <typename IndexType>
class GPUParser : public Parser<IndexType> {
 public:
  GPUParser(const std::string& uri, unsigned part, unsigned nparts, const RouteArgs& r)
      : to_host_(r.to_host) {
    p_.reset(gpu::DeviceParser<IndexType>::Create(uri, part, nparts, r.cfg));
  }
  void BeforeFirst() override { p_->BeforeFirst(); }
  bool Next() override {
    if (!p_->Next()) return false;
    const gpu::DeviceRowBlock<IndexType>& d = p_->Value();
    if (to_host_) {
      host_ = gpu::CopyToHost(d);
      block_ = host_.GetBlock();
    } else {
      block_ = DeviceView(d);
    }
    return true;
  }
  const RowBlock<IndexType>& Value() const override { return block_; }
  size_t BytesRead() const override { return p_->Stats().bytes; }

 private:
  bool to_host_;
  std::unique_ptr<gpu::DeviceParser<IndexType>> p_;
  gpu::HostCSR<IndexType> host_;
  RowBlock<IndexType> block_;
};

template <typename IndexType>
class DeviceRowIter : public RowBlockIter<IndexType> {
 public:
  DeviceRowIter(const std::string& uri, unsigned part, unsigned nparts, const RouteArgs& r,
                const std::string& cache_file) {
    const char* how = "parsed";
    if (!cache_file.empty()) {
      // DiskRowIter's protocol (reference src/data/disk_row_iter.h:94-141):
      // load the page file when it exists, else build it from this parse
      auto cache = gpu::DevicePageCache<IndexType>::Open(cache_file, r.cfg.device);
      if (cache != nullptr) {
        cache->Load(&csr_);
        how = cache->zero_copy() ? "loaded (zero-copy DMA) from cache" : "loaded from cache";
      } else {
        Parse(uri, part, nparts, r);
        const size_t pages = gpu::DevicePageCache<IndexType>::Write(csr_, cache_file);
        LOG(INFO) << "DeviceRowIter: wrote " << pages << " cache pages to " << cache_file;
        how = "parsed, cache built";
      }
    } else {
      Parse(uri, part, nparts, r);
    }
    const gpu::DeviceRowBlock<IndexType> d = csr_.View();
    num_col_ = static_cast<size_t>(d.max_index) + 1;
    if (r.to_host) {
      host_ = gpu::CopyToHost(d);
      block_ = host_.GetBlock();
    } else {
      block_ = DeviceView(d);
    }
    LOG(INFO) << "DeviceRowIter: " << d.size << " rows, " << d.nnz << " entries resident in HBM ("
              << how << ")" << (r.to_host ? ", host copy served" : "");
  }
  void BeforeFirst() override { at_ = 0; }
  bool Next() override {
    if (at_ != 0) return false;
    at_ = 1;
    return true;
  }
  const RowBlock<IndexType>& Value() const override { return block_; }
  size_t NumCol() const override { return num_col_; }

 private:
  void Parse(const std::string& uri, unsigned part, unsigned nparts, const RouteArgs& r) {
    std::unique_ptr<gpu::DeviceParser<IndexType>> p(
        gpu::DeviceParser<IndexType>::Create(uri, part, nparts, r.cfg));
    p->ParseAll(&csr_);
  }
  gpu::DeviceCSR<IndexType> csr_;
  gpu::HostCSR<IndexType> host_;
  RowBlock<IndexType> block_;
  size_t num_col_{0};
  int at_{0};
};

}  // namespace

template <typename IndexType>
Parser<IndexType>* CreateDeviceParser(const std::string& uri,
                                      const std::map<std::string, std::string>& args,
                                      unsigned part, unsigned nparts, const std::string& type) {
  return new GPUParser<IndexType>(uri, part, nparts, ParseRoute(args, type));
}

template <typename IndexType>
RowBlockIter<IndexType>* CreateDeviceRowIter(const std::string& uri,
                                             const std::map<std::string, std::string>& args,
                                             unsigned part, unsigned nparts,
                                             const std::string& type,
                                             const std::string& cache_file) {
  return new DeviceRowIter<IndexType>(uri, part, nparts, ParseRoute(args, type), cache_file);
}

namespace {
/*! \brief installs the GPU factories into src/data.cc's `device=gpu` route */
struct InstallDeviceRoute {
  InstallDeviceRoute() {
    DeviceRoute<uint32_t>::parser = &CreateDeviceParser<uint32_t>;
    DeviceRoute<uint64_t>::parser = &CreateDeviceParser<uint64_t>;
    DeviceRoute<uint32_t>::iter = &CreateDeviceRowIter<uint32_t>;
    DeviceRoute<uint64_t>::iter = &CreateDeviceRowIter<uint64_t>;
  }
} install_device_route;
}  // namespace

}  // namespace data
}  // namespace dmlc
