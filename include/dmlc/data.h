/*!
 * \file dmlc/data.h
 * \brief Sparse row-batch data structures (CSR RowBlock), data iterators and
 *  the parser factory registry.
 *
 * Parity: reference `include/dmlc/data.h` — real_t / index_t (:23-29),
 * DataIter<T> (:53-63), Row<I> with get_value/get_weight/get_qid and SDot
 * (:70-158; NULL value/weight mean 1.0, NULL qid means 0), RowBlock<I> CSR view
 * {size, offset[size+1], label, weight?, qid?, field?, index, value?}
 * (:170-231) with MemCostBytes / Slice / operator[], RowBlockIter<I>::Create /
 * NumCol (:246-267), Parser<I>::Create / BytesRead (:283-311),
 * ParserFactoryReg (:317-320), DMLC_REGISTER_DATA_PARSER (:347-350).
 *
 * GPU twin: dmlc/gpu/device_row_block.h (DeviceRowBlock<I> lives in HBM).
 */
#ifndef DMLC_DATA_H_
#define DMLC_DATA_H_

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "./base.h"
#include "./io.h"
#include "./logging.h"
#include "./registry.h"

namespace dmlc {

/*! \brief feature value type */
typedef float real_t;
/*! \brief default feature index type */
typedef unsigned index_t;

/*! \brief generic pull iterator */
template <typename DType>
class DataIter {
 public:
  virtual ~DataIter() = default;
  /*! \brief rewind */
  virtual void BeforeFirst() = 0;
  /*! \brief advance; false at end */
  virtual bool Next() = 0;
  /*! \brief current element (valid until the next Next/BeforeFirst) */
  virtual const DType& Value() const = 0;
};

/*! \brief one sparse row (a view into a RowBlock) */
template <typename IndexType, typename DType = real_t>
class Row {
 public:
  /*! \brief label of the row */
  const DType* label;
  /*! \brief per-row weight; nullptr means 1 */
  const real_t* weight;
  /*! \brief query id; nullptr means 0 */
  const uint64_t* qid;
  /*! \brief number of non-zeros */
  size_t length;
  /*! \brief field ids (LibFM); nullptr when absent */
  const IndexType* field;
  /*! \brief feature indices */
  const IndexType* index;
  /*! \brief feature values; nullptr means every value is 1 */
  const DType* value;

  inline IndexType get_field(size_t i) const { return field[i]; }
  inline IndexType get_index(size_t i) const { return index[i]; }
  inline DType get_value(size_t i) const {
    return value == nullptr ? DType(1.0f) : value[i];
  }
  inline DType get_label() const { return *label; }
  inline real_t get_weight() const { return weight == nullptr ? 1.0f : *weight; }
  inline uint64_t get_qid() const { return qid == nullptr ? 0 : *qid; }
  /*! \brief sparse dot product with a dense vector of size >= max index + 1 */
  template <typename V>
  inline V SDot(const V* weight_vec, size_t size) const {
    V sum = static_cast<V>(0);
    if (value == nullptr) {
      for (size_t i = 0; i < length; ++i) {
        CHECK(index[i] < size) << "feature index exceed bound";
        sum += weight_vec[index[i]];
      }
    } else {
      for (size_t i = 0; i < length; ++i) {
        CHECK(index[i] < size) << "feature index exceed bound";
        sum += weight_vec[index[i]] * value[i];
      }
    }
    return sum;
  }
};

/*! \brief a batch of rows in CSR layout (non-owning view) */
template <typename IndexType, typename DType = real_t>
struct RowBlock {
  /*! \brief number of rows */
  size_t size;
  /*! \brief row pointer, size + 1 entries */
  const size_t* offset;
  /*! \brief labels, size entries */
  const DType* label;
  /*! \brief weights, size entries or nullptr */
  const real_t* weight;
  /*! \brief query ids, size entries or nullptr */
  const uint64_t* qid;
  /*! \brief field ids, offset[size] entries or nullptr */
  const IndexType* field;
  /*! \brief feature indices, offset[size] entries */
  const IndexType* index;
  /*! \brief feature values, offset[size] entries or nullptr */
  const DType* value;

  inline Row<IndexType, DType> operator[](size_t rowid) const;
  /*! \brief approximate bytes referenced by this block */
  inline size_t MemCostBytes() const {
    size_t cost = size * (sizeof(size_t) + sizeof(DType));
    if (weight != nullptr) cost += size * sizeof(real_t);
    if (qid != nullptr) cost += size * sizeof(uint64_t);
    size_t ndata = offset[size] - offset[0];
    if (field != nullptr) cost += ndata * sizeof(IndexType);
    if (index != nullptr) cost += ndata * sizeof(IndexType);
    if (value != nullptr) cost += ndata * sizeof(DType);
    return cost;
  }
  /*!
   * \brief rows [begin, end) as a new view.  index/value are shared and the
   *  offsets are NOT rebased (offset[0] may be non-zero), as in the reference.
   */
  inline RowBlock Slice(size_t begin, size_t end) const {
    CHECK(begin <= end && end <= size);
    RowBlock ret;
    ret.size = end - begin;
    ret.label = label + begin;
    ret.weight = weight != nullptr ? weight + begin : nullptr;
    ret.qid = qid != nullptr ? qid + begin : nullptr;
    ret.offset = offset + begin;
    ret.field = field;
    ret.index = index;
    ret.value = value;
    return ret;
  }
};

template <typename IndexType, typename DType>
inline Row<IndexType, DType> RowBlock<IndexType, DType>::operator[](size_t rowid) const {
  CHECK(rowid < size);
  Row<IndexType, DType> inst;
  inst.label = label + rowid;
  inst.weight = weight != nullptr ? weight + rowid : nullptr;
  inst.qid = qid != nullptr ? qid + rowid : nullptr;
  inst.length = offset[rowid + 1] - offset[rowid];
  inst.field = field != nullptr ? field + offset[rowid] : nullptr;
  inst.index = index + offset[rowid];
  inst.value = value != nullptr ? value + offset[rowid] : nullptr;
  return inst;
}

/*!
 * \brief iterator over RowBlocks of a whole dataset (kept in memory, or paged
 *  through a `#cachefile` on disk).
 */
template <typename IndexType, typename DType = real_t>
class RowBlockIter : public DataIter<RowBlock<IndexType, DType>> {
 public:
  /*!
   * \param uri data uri; `uri#cachefile` enables the disk page cache
   * \param type "libsvm", "libfm", "csv" or "auto" (`?format=`)
   */
  static RowBlockIter<IndexType, DType>* Create(const char* uri, unsigned part_index,
                                                unsigned num_parts, const char* type);
  /*! \brief number of feature columns (max index + 1) */
  virtual size_t NumCol() const = 0;
};

/*! \brief streaming parser producing RowBlocks */
template <typename IndexType, typename DType = real_t>
class Parser : public DataIter<RowBlock<IndexType, DType>> {
 public:
  /*!
   * \param uri input uri with optional `?k=v` arguments
   * \param type registered parser name, or "auto" (`?format=...`, else libsvm)
   */
  static Parser<IndexType, DType>* Create(const char* uri, unsigned part_index,
                                          unsigned num_parts, const char* type);
  /*! \brief bytes consumed so far */
  virtual size_t BytesRead() const = 0;
  /*! \brief factory signature stored in the registry */
  typedef Parser<IndexType, DType>* (*Factory)(
      const std::string& path, const std::map<std::string, std::string>& args,
      unsigned part_index, unsigned num_parts);
};

/*! \brief registry entry of a parser factory */
template <typename IndexType, typename DType = real_t>
struct ParserFactoryReg
    : public FunctionRegEntryBase<ParserFactoryReg<IndexType, DType>,
                                  typename Parser<IndexType, DType>::Factory> {};

/*!
 * \brief register a parser factory `FactoryFunction` under `TypeName` for
 *  index type `IndexType`, e.g.
 *  DMLC_REGISTER_DATA_PARSER(uint32_t, libsvm, CreateLibSVMParser<uint32_t>)
 */
#define DMLC_REGISTER_DATA_PARSER(IndexType, TypeName, FactoryFunction)             \
  DMLC_REGISTRY_REGISTER(::dmlc::ParserFactoryReg<IndexType>, ParserFactoryReg##_##IndexType, \
                         TypeName)                                                  \
      .set_body(FactoryFunction)

}  // namespace dmlc
#endif  // DMLC_DATA_H_
