/*!
 * \file src/gpu/runtime.cc
 * \brief Device queries, roctx ranges, DeviceCSR storage management and
 *  device -> host copies.
 */
#include <dlfcn.h>
#include <dmlc/gpu/device_parser.h>
#include <dmlc/gpu/device_row_block.h>
#include <dmlc/gpu/hip_utils.h>

#include <algorithm>
#include <cstring>

#include "./kernels.h"

namespace dmlc {
namespace gpu {

int DeviceCount() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

bool Available() { return DeviceCount() > 0; }

void SetDevice(int device) { DMLC_HIP_CHECK(hipSetDevice(device)); }

std::string DeviceArchName(int device) {
  hipDeviceProp_t prop;
  DMLC_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  return std::string(prop.gcnArchName);
}

// ------------------------------------------------------------------ roctx
namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) return;
    push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    if (push == nullptr || pop == nullptr) push = nullptr;
  }
};
Roctx& GetRoctx() {
  static Roctx r;
  return r;
}
}  // namespace

ScopedRange::ScopedRange(const char* name) {
  Roctx& r = GetRoctx();
  if (r.push != nullptr) {
    r.push(name);
    active_ = true;
  }
}
ScopedRange::~ScopedRange() {
  if (active_) GetRoctx().pop();
}

// -------------------------------------------------------------- DeviceCSR
namespace {
size_t Grown(size_t want, size_t have) {
  if (want <= have) return have;
  return std::max(want, have + have / 2);
}
}  // namespace

template <typename IndexType>
void DeviceCSR<IndexType>::Reserve(size_t rows, size_t nnz, bool with_field, hipStream_t stream,
                                   size_t used_rows, size_t used_nnz) {
  if (rows > row_cap_) {
    const size_t cap = Grown(rows, row_cap_);
    offset_.Grow((cap + 1) * sizeof(uint64_t), (used_rows + 1) * sizeof(uint64_t), stream);
    label_.Grow(cap * sizeof(float), used_rows * sizeof(float), stream);
    if (weight_.bytes() != 0) weight_.Grow(cap * sizeof(float), used_rows * sizeof(float), stream);
    if (qid_.bytes() != 0) qid_.Grow(cap * sizeof(uint64_t), used_rows * sizeof(uint64_t), stream);
    row_cap_ = cap;
  }
  if (nnz > nnz_cap_) {
    const size_t cap = Grown(nnz, nnz_cap_);
    index_.Grow(cap * sizeof(IndexType), used_nnz * sizeof(IndexType), stream);
    value_.Grow(cap * sizeof(float), used_nnz * sizeof(float), stream);
    if (field_.bytes() != 0 || with_field) {
      field_.Grow(cap * sizeof(IndexType), used_nnz * sizeof(IndexType), stream);
    }
    nnz_cap_ = cap;
  } else if (with_field && field_.bytes() < nnz_cap_ * sizeof(IndexType)) {
    field_.Grow(nnz_cap_ * sizeof(IndexType), used_nnz * sizeof(IndexType), stream);
  }
}

void DeviceHashedBatch::Reserve(size_t want, hipStream_t stream) {
  if (want <= row_cap) return;
  const size_t cap = std::max(want, row_cap * 2);
  const size_t esize = fp8 ? 1 : sizeof(float);
  auto nx = std::make_shared<DeviceBuffer>(cap * static_cast<size_t>(dim) * esize);
  auto nl = std::make_shared<DeviceBuffer>(cap * sizeof(float));
  if (rows != 0) {
    DMLC_HIP_CHECK(hipMemcpyAsync(nx->get(), x->get(), rows * static_cast<size_t>(dim) * esize,
                                  hipMemcpyDeviceToDevice, stream));
    DMLC_HIP_CHECK(hipMemcpyAsync(nl->get(), label->get(), rows * sizeof(float),
                                  hipMemcpyDeviceToDevice, stream));
  }
  // the old buffers are freed once their last owner (this batch, or a DLPack
  // tensor exported from it) lets go -- after the copies (hipFree synchronises)
  x = std::move(nx);
  label = std::move(nl);
  row_cap = cap;
}

template <typename IndexType>
void DeviceCSR<IndexType>::EnableWeight(hipStream_t stream) {
  if (weight_.bytes() >= row_cap_ * sizeof(float) && weight_.bytes() != 0) return;
  weight_.Reserve(std::max<size_t>(row_cap_, 1) * sizeof(float));
  if (rows_ != 0) LaunchFill(weight_.get<float>(), rows_, 1.0f, stream);
}

template <typename IndexType>
void DeviceCSR<IndexType>::EnableQid(hipStream_t stream) {
  if (qid_.bytes() >= row_cap_ * sizeof(uint64_t) && qid_.bytes() != 0) return;
  qid_.Reserve(std::max<size_t>(row_cap_, 1) * sizeof(uint64_t));
  if (rows_ != 0) DMLC_HIP_CHECK(hipMemsetAsync(qid_.get(), 0, rows_ * sizeof(uint64_t), stream));
}

template <typename IndexType>
DeviceRowBlock<IndexType> DeviceCSR<IndexType>::View() const {
  DeviceRowBlock<IndexType> b;
  b.size = rows_;
  b.nnz = nnz_;
  b.offset = offset_.get<uint64_t>();
  b.label = label_.get<float>();
  b.weight = has_weight_ ? weight_.get<float>() : nullptr;
  b.qid = has_qid_ ? qid_.get<uint64_t>() : nullptr;
  b.field = has_field_ ? field_.get<IndexType>() : nullptr;
  b.index = index_.get<IndexType>();
  b.value = has_value_ ? value_.get<float>() : nullptr;
  b.max_index = max_index_;
  b.max_field = max_field_;
  b.device = device_;
  return b;
}

template <typename IndexType>
HostCSR<IndexType> CopyToHost(const DeviceRowBlock<IndexType>& blk) {
  HostCSR<IndexType> h;
  const size_t n = blk.size;
  std::vector<uint64_t> off(n + 1, 0);
  if (blk.offset != nullptr) {
    DMLC_HIP_CHECK(hipMemcpy(off.data(), blk.offset, (n + 1) * sizeof(uint64_t),
                             hipMemcpyDeviceToHost));
  }
  const uint64_t base = off[0];
  const size_t nnz = static_cast<size_t>(off[n] - base);
  h.offset.resize(n + 1);
  for (size_t i = 0; i <= n; ++i) h.offset[i] = static_cast<size_t>(off[i] - base);
  auto copy = [](auto* dst_vec, const auto* src, size_t count) {
    using T = typename std::remove_pointer<decltype(dst_vec->data())>::type;
    dst_vec->resize(count);
    if (count != 0 && src != nullptr) {
      DMLC_HIP_CHECK(hipMemcpy(dst_vec->data(), src, count * sizeof(T), hipMemcpyDeviceToHost));
    }
  };
  copy(&h.label, blk.label, n);
  if (blk.weight != nullptr) copy(&h.weight, blk.weight, n);
  if (blk.qid != nullptr) copy(&h.qid, blk.qid, n);
  copy(&h.index, blk.index + base, nnz);
  if (blk.value != nullptr) copy(&h.value, blk.value + base, nnz);
  if (blk.field != nullptr) copy(&h.field, blk.field + base, nnz);
  return h;
}

template class DeviceCSR<uint32_t>;
template class DeviceCSR<uint64_t>;
template HostCSR<uint32_t> CopyToHost<uint32_t>(const DeviceRowBlock<uint32_t>&);
template HostCSR<uint64_t> CopyToHost<uint64_t>(const DeviceRowBlock<uint64_t>&);

}  // namespace gpu
}  // namespace dmlc
