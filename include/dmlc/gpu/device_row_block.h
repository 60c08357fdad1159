/*!
 * \file dmlc/gpu/device_row_block.h
 * \brief CSR row batches resident in MI355X HBM.
 *
 * DeviceRowBlock<I> is the device twin of dmlc::RowBlock<I> (reference
 * `include/dmlc/data.h:170-231`): same field meaning, but every pointer is a
 * device pointer and `offset` is 64-bit.  DeviceCSR<I> owns the storage and
 * grows by doubling; with 288 GB of HBM3E per GPU a whole shard's CSR
 * normally stays resident (the HBM epoch cache, SURVEY §5.4 design).
 */
#ifndef DMLC_GPU_DEVICE_ROW_BLOCK_H_
#define DMLC_GPU_DEVICE_ROW_BLOCK_H_

#include <dmlc/data.h>

#include <cstdint>
#include <vector>

#include "./hip_utils.h"

namespace dmlc {
namespace gpu {

/*! \brief non-owning view of a device CSR block */
template <typename IndexType>
struct DeviceRowBlock {
  /*! \brief number of rows */
  size_t size{0};
  /*! \brief number of stored entries (offset[size] - offset[0]) */
  size_t nnz{0};
  /*! \brief row pointer, size+1 entries (device) */
  const uint64_t* offset{nullptr};
  /*! \brief labels (device) */
  const float* label{nullptr};
  /*! \brief weights or nullptr (every weight 1) */
  const float* weight{nullptr};
  /*! \brief query ids or nullptr (every qid 0) */
  const uint64_t* qid{nullptr};
  /*! \brief LibFM fields or nullptr */
  const IndexType* field{nullptr};
  /*! \brief feature indices (device) */
  const IndexType* index{nullptr};
  /*! \brief feature values or nullptr (every value 1) */
  const float* value{nullptr};
  /*! \brief max feature index seen (NumCol = max_index + 1) */
  uint64_t max_index{0};
  /*! \brief max field id seen (LibFM) */
  uint64_t max_field{0};
  /*! \brief device the memory lives on */
  int device{0};
};

/*!
 * \brief host copy of a device block (for tests / CPU consumers)
 * \return host RowBlock storage (offset converted to size_t)
 */
template <typename IndexType>
struct HostCSR {
  std::vector<size_t> offset;
  std::vector<float> label, weight, value;
  std::vector<uint64_t> qid;
  std::vector<IndexType> field, index;
  RowBlock<IndexType> GetBlock() const {
    RowBlock<IndexType> b;
    b.size = label.size();
    b.offset = offset.data();
    b.label = label.data();
    b.weight = weight.empty() ? nullptr : weight.data();
    b.qid = qid.empty() ? nullptr : qid.data();
    b.field = field.empty() ? nullptr : field.data();
    b.index = index.data();
    b.value = value.empty() ? nullptr : value.data();
    return b;
  }
};

/*! \brief copy a device block to the host (synchronous) */
template <typename IndexType>
HostCSR<IndexType> CopyToHost(const DeviceRowBlock<IndexType>& blk);

/*! \brief owning, growable device CSR */
template <typename IndexType>
class DeviceCSR {
 public:
  DeviceCSR() = default;
  DeviceCSR(const DeviceCSR&) = delete;
  DeviceCSR& operator=(const DeviceCSR&) = delete;
  DeviceCSR(DeviceCSR&&) = default;
  DeviceCSR& operator=(DeviceCSR&&) = default;
  /*! \brief capacity >= rows / nnz, preserving the first used_rows/used_nnz */
  void Reserve(size_t rows, size_t nnz, bool with_field, hipStream_t stream,
               size_t used_rows = 0, size_t used_nnz = 0);
  /*! \brief allocate the weight column; existing rows get weight 1 */
  void EnableWeight(hipStream_t stream);
  /*! \brief allocate the qid column; existing rows get qid 0 */
  void EnableQid(hipStream_t stream);
  /*! \brief forget contents (keeps capacity) */
  void Clear() {
    rows_ = nnz_ = 0;
    max_index_ = max_field_ = 0;
    has_weight_ = has_qid_ = has_value_ = has_field_ = false;
  }
  DeviceRowBlock<IndexType> View() const;

  uint64_t* offset() { return offset_.get<uint64_t>(); }
  float* label() { return label_.get<float>(); }
  float* weight() { return weight_.get<float>(); }
  uint64_t* qid() { return qid_.get<uint64_t>(); }
  IndexType* field() { return field_.get<IndexType>(); }
  IndexType* index() { return index_.get<IndexType>(); }
  float* value() { return value_.get<float>(); }
  size_t row_capacity() const { return row_cap_; }
  /*! \brief rows the weight column can hold (0 when not allocated) */
  size_t weight_capacity() const { return weight_.bytes() / sizeof(float); }
  size_t nnz_capacity() const { return nnz_cap_; }
  /*! \brief device bytes held */
  size_t AllocatedBytes() const {
    return offset_.bytes() + label_.bytes() + weight_.bytes() + qid_.bytes() + field_.bytes() +
           index_.bytes() + value_.bytes();
  }

  size_t rows_{0}, nnz_{0};
  uint64_t max_index_{0}, max_field_{0};
  bool has_weight_{false}, has_qid_{false}, has_value_{false}, has_field_{false};
  int device_{0};

 private:
  DeviceBuffer offset_, label_, weight_, qid_, field_, index_, value_;
  size_t row_cap_{0}, nnz_cap_{0};
};

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_GPU_DEVICE_ROW_BLOCK_H_
