/*!
 * \file dmlc/common.h
 * \brief String split and hash combine.
 * Parity: reference `include/dmlc/common.h:20-46` (Split, HashCombine).
 */
#ifndef DMLC_COMMON_H_
#define DMLC_COMMON_H_

#include <functional>
#include <string>
#include <vector>

namespace dmlc {
/*!
 * \brief split `s` on `delim`; an empty trailing field is dropped, matching
 *  std::getline semantics used by the reference.
 */
inline std::vector<std::string> Split(const std::string& s, char delim) {
  std::vector<std::string> out;
  size_t start = 0;
  while (start < s.size()) {
    size_t pos = s.find(delim, start);
    if (pos == std::string::npos) pos = s.size();
    out.emplace_back(s, start, pos - start);
    start = pos + 1;
  }
  return out;
}

/*! \brief boost-style hash mixing of `value` into `key` */
template <typename T>
inline size_t HashCombine(size_t key, const T& value) {
  std::hash<T> hash_func;
  return key ^ (hash_func(value) + 0x9e3779b9 + (key << 6) + (key >> 2));
}
template <>
inline size_t HashCombine<size_t>(size_t key, const size_t& value) {
  return key ^ (value + 0x9e3779b9 + (key << 6) + (key >> 2));
}
}  // namespace dmlc
#endif  // DMLC_COMMON_H_
