/*!
 * \file src/data/row_block.h
 * \brief RowBlockContainer: growable host CSR storage behind RowBlock views.
 *
 * Parity: reference `src/data/row_block.h:27-216` — fields offset / label /
 * weight / qid / field / index / value / max_field / max_index, Clear,
 * MemCostBytes, Push(Row) and Push(RowBlock) with max tracking, GetBlock with
 * consistency CHECKs, binary Save / Load (the DiskRowIter page format:
 * serialized vectors offset(size_t), label, weight, qid, field, index, value,
 * then raw max_field, max_index).
 *
 * Difference: optional columns are "all or nothing" per
 * block. When some rows carry a weight (value, qid) and others do not, the
 * missing entries are backfilled with the neutral value (1.0 / 1.0 / 0)
 * instead of producing misaligned arrays as the reference does.
 */
#ifndef DMLC_DATA_ROW_BLOCK_H_
#define DMLC_DATA_ROW_BLOCK_H_

#include <dmlc/data.h>
#include <dmlc/io.h>
#include <dmlc/logging.h>

#include <algorithm>
#include <limits>
#include <vector>

namespace dmlc {
namespace data {

template <typename IndexType, typename DType = real_t>
struct RowBlockContainer {
  std::vector<size_t> offset;
  std::vector<DType> label;
  std::vector<real_t> weight;
  std::vector<uint64_t> qid;
  std::vector<IndexType> field;
  std::vector<IndexType> index;
  std::vector<DType> value;
  IndexType max_field;
  IndexType max_index;

  RowBlockContainer() { this->Clear(); }

  /*! \brief view of the current contents */
  inline RowBlock<IndexType, DType> GetBlock() const;
  /*! \brief binary save (DiskRowIter page) */
  inline void Save(Stream* fo) const {
    fo->Write(offset);
    fo->Write(label);
    fo->Write(weight);
    fo->Write(qid);
    fo->Write(field);
    fo->Write(index);
    fo->Write(value);
    fo->Write(&max_field, sizeof(IndexType));
    fo->Write(&max_index, sizeof(IndexType));
  }
  /*! \brief binary load; false at end of stream */
  inline bool Load(Stream* fi) {
    if (!fi->Read(&offset)) return false;
    CHECK(fi->Read(&label)) << "Bad RowBlock format";
    CHECK(fi->Read(&weight)) << "Bad RowBlock format";
    CHECK(fi->Read(&qid)) << "Bad RowBlock format";
    CHECK(fi->Read(&field)) << "Bad RowBlock format";
    CHECK(fi->Read(&index)) << "Bad RowBlock format";
    CHECK(fi->Read(&value)) << "Bad RowBlock format";
    CHECK(fi->Read(&max_field, sizeof(IndexType))) << "Bad RowBlock format";
    CHECK(fi->Read(&max_index, sizeof(IndexType))) << "Bad RowBlock format";
    return true;
  }
  inline void Clear() {
    offset.clear();
    offset.push_back(0);
    label.clear();
    weight.clear();
    qid.clear();
    field.clear();
    index.clear();
    value.clear();
    max_field = 0;
    max_index = 0;
  }
  /*! \brief number of rows */
  inline size_t Size() const { return offset.size() - 1; }
  inline size_t MemCostBytes() const {
    return offset.size() * sizeof(size_t) + label.size() * sizeof(DType) +
           weight.size() * sizeof(real_t) + qid.size() * sizeof(uint64_t) +
           field.size() * sizeof(IndexType) + index.size() * sizeof(IndexType) +
           value.size() * sizeof(DType);
  }

  // ---- incremental row building used by the text parsers ----
  /*! \brief open a new row */
  inline void BeginRow(DType lbl) { label.push_back(lbl); }
  /*! \brief set the weight of the open row (backfills earlier rows with 1) */
  inline void SetWeight(real_t w) {
    if (weight.size() + 1 < label.size()) weight.resize(label.size() - 1, 1.0f);
    weight.push_back(w);
  }
  /*! \brief set the qid of the open row (backfills earlier rows with 0) */
  inline void SetQid(uint64_t q) {
    if (qid.size() + 1 < label.size()) qid.resize(label.size() - 1, 0);
    qid.push_back(q);
  }
  /*! \brief append a feature to the open row; has_value=false means 1.0 */
  inline void PushFeature(IndexType idx, DType val, bool has_value) {
    if (has_value) {
      if (value.size() < index.size()) value.resize(index.size(), DType(1.0f));
      value.push_back(val);
    } else if (!value.empty()) {
      value.push_back(DType(1.0f));
    }
    index.push_back(idx);
    max_index = std::max(max_index, idx);
  }
  inline void PushField(IndexType f) {
    field.push_back(f);
    max_field = std::max(max_field, f);
  }
  /*! \brief close the open row; pads optional columns of the row */
  inline void EndRow() {
    if (!weight.empty() && weight.size() < label.size()) weight.resize(label.size(), 1.0f);
    if (!qid.empty() && qid.size() < label.size()) qid.resize(label.size(), 0);
    offset.push_back(index.size());
  }
  /*! \brief make optional columns full-length after the last row */
  inline void Finalize() {
    if (!weight.empty()) weight.resize(label.size(), 1.0f);
    if (!qid.empty()) qid.resize(label.size(), 0);
    if (!value.empty()) value.resize(index.size(), DType(1.0f));
  }

  /*! \brief append one row */
  template <typename I>
  inline void Push(Row<I, DType> row) {
    label.push_back(row.get_label());
    if (row.weight != nullptr) SetWeightAt(label.size() - 1, *row.weight);
    if (row.qid != nullptr) SetQidAt(label.size() - 1, *row.qid);
    for (size_t i = 0; i < row.length; ++i) {
      CHECK_LE(row.index[i], std::numeric_limits<IndexType>::max())
          << "index exceed numeric bound of current type";
      const IndexType idx = static_cast<IndexType>(row.index[i]);
      PushFeature(idx, row.value != nullptr ? row.value[i] : DType(1.0f), row.value != nullptr);
      if (row.field != nullptr) {
        CHECK_LE(row.field[i], std::numeric_limits<IndexType>::max())
            << "field exceed numeric bound of current type";
        PushField(static_cast<IndexType>(row.field[i]));
      }
    }
    EndRow();
  }
  /*! \brief append a whole block (offsets shifted) */
  template <typename I>
  inline void Push(RowBlock<I, DType> batch) {
    for (size_t i = 0; i < batch.size; ++i) this->Push<I>(batch[i]);
  }

 private:
  inline void SetWeightAt(size_t row, real_t w) {
    if (weight.size() < row) weight.resize(row, 1.0f);
    weight.push_back(w);
  }
  inline void SetQidAt(size_t row, uint64_t q) {
    if (qid.size() < row) qid.resize(row, 0);
    qid.push_back(q);
  }
};

template <typename IndexType, typename DType>
inline RowBlock<IndexType, DType> RowBlockContainer<IndexType, DType>::GetBlock() const {
  CHECK_EQ(label.size() + 1, offset.size());
  CHECK_EQ(offset.back(), index.size());
  CHECK(weight.empty() || weight.size() == label.size()) << "weight column misaligned";
  CHECK(qid.empty() || qid.size() == label.size()) << "qid column misaligned";
  CHECK(field.empty() || field.size() == index.size()) << "field column misaligned";
  CHECK(value.empty() || value.size() == index.size()) << "value column misaligned";
  RowBlock<IndexType, DType> out;
  out.size = offset.size() - 1;
  out.offset = BeginPtr(offset);
  out.label = BeginPtr(label);
  out.weight = BeginPtr(weight);
  out.qid = BeginPtr(qid);
  out.field = BeginPtr(field);
  out.index = BeginPtr(index);
  out.value = BeginPtr(value);
  return out;
}

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_ROW_BLOCK_H_
