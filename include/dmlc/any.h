/*!
 * \file dmlc/any.h
 * \brief dmlc::any — type-erased value with checked access.
 *
 * Parity: reference `include/dmlc/any.h` — any with small-buffer storage
 * (:137), get<T> with a type CHECK that throws dmlc::Error (:284-305),
 * construct<T>(args...) (:221-236), type()/empty()/clear()/swap.  Built on
 * std::any (which already provides the small-buffer optimisation).
 */
#ifndef DMLC_ANY_H_
#define DMLC_ANY_H_

#include <any>
#include <typeinfo>
#include <utility>

#include "./base.h"
#include "./logging.h"

namespace dmlc {

class any {
 public:
  any() = default;
  any(const any&) = default;
  any(any&&) = default;
  template <typename T, typename = typename std::enable_if<!std::is_same<
                            typename std::decay<T>::type, any>::value>::type>
  any(T&& other) : v_(std::forward<T>(other)) {}  // NOLINT(runtime/explicit)
  any& operator=(const any&) = default;
  any& operator=(any&&) = default;
  template <typename T, typename = typename std::enable_if<!std::is_same<
                            typename std::decay<T>::type, any>::value>::type>
  any& operator=(T&& other) {
    v_ = std::forward<T>(other);
    return *this;
  }
  bool empty() const { return !v_.has_value(); }
  void clear() { v_.reset(); }
  void swap(any& other) { v_.swap(other.v_); }
  const std::type_info& type() const { return v_.type(); }
  /*! \brief in-place construct a T from args */
  template <typename T, typename... Args>
  void construct(Args&&... args) {
    v_.emplace<T>(std::forward<Args>(args)...);
  }

 private:
  template <typename T>
  friend const T& get(const any& src);
  template <typename T>
  friend T& get(any& src);  // NOLINT(runtime/references)
  template <typename T>
  friend T* unsafe_get(any* src);
  std::any v_;
};

namespace any_detail {
inline void CheckType(const any& src, const std::type_info& want) {
  CHECK(!src.empty()) << "The any container is empty"
                      << " requested=" << Demangle(want.name());
  CHECK(src.type() == want) << "The stored type mismatch"
                            << " stored=" << Demangle(src.type().name())
                            << " requested=" << Demangle(want.name());
}
}  // namespace any_detail

template <typename T>
inline const T& get(const any& src) {
  any_detail::CheckType(src, typeid(T));
  return *std::any_cast<T>(&src.v_);
}
template <typename T>
inline T& get(any& src) {  // NOLINT(runtime/references)
  any_detail::CheckType(src, typeid(T));
  return *std::any_cast<T>(&src.v_);
}
/*! \brief unchecked access (nullptr on mismatch) */
template <typename T>
inline T* unsafe_get(any* src) {
  return std::any_cast<T>(&src->v_);
}
}  // namespace dmlc
#endif  // DMLC_ANY_H_
