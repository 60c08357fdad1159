/*!
 * \file dmlc/array_view.h
 * \brief Read-only contiguous view (std::span-like).
 * Parity: reference `include/dmlc/array_view.h:36-124`.
 */
#ifndef DMLC_ARRAY_VIEW_H_
#define DMLC_ARRAY_VIEW_H_

#include <array>
#include <cstddef>
#include <vector>

namespace dmlc {
template <typename ValueType>
class array_view {
 public:
  array_view() = default;
  array_view(const std::vector<ValueType>& other)  // NOLINT(runtime/explicit)
      : begin_(other.data()), size_(other.size()) {}
  template <std::size_t N>
  array_view(const std::array<ValueType, N>& other)  // NOLINT(runtime/explicit)
      : begin_(other.data()), size_(N) {}
  array_view(const ValueType* begin, const ValueType* end)
      : begin_(begin), size_(static_cast<size_t>(end - begin)) {}
  const ValueType* data() const { return begin_; }
  const ValueType* begin() const { return begin_; }
  const ValueType* end() const { return begin_ + size_; }
  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  const ValueType& operator[](size_t i) const { return begin_[i]; }

 private:
  const ValueType* begin_{nullptr};
  size_t size_{0};
};
}  // namespace dmlc
#endif  // DMLC_ARRAY_VIEW_H_
