/*!
 * \file dmlc/optional.h
 * \brief dmlc::optional<T>: std::optional with dmlc text I/O conventions.
 *
 * Parity: reference `include/dmlc/optional.h` — nullopt (:22-33), optional<T>
 * (:43-125), operator<< printing "None" (:141-148), operator>> accepting
 * "None" and a trailing 'L' on integers (:168-184), optional<bool> parsing
 * true/false/1/0/None (:205-228), type names (:231-237), std::hash (:244-257).
 * Built on std::optional.
 */
#ifndef DMLC_OPTIONAL_H_
#define DMLC_OPTIONAL_H_

#include <algorithm>
#include <cctype>
#include <functional>
#include <iostream>
#include <optional>
#include <string>
#include <utility>

#include "./base.h"
#include "./logging.h"
#include "./type_traits.h"

namespace dmlc {

/*! \brief tag type of an empty optional */
struct nullopt_t {
  constexpr explicit nullopt_t(int) {}
};
/*! \brief the empty-optional constant */
constexpr nullopt_t nullopt{0};

/*! \brief optional value; prints/parses as "None" when empty */
template <typename T>
class optional {
 public:
  optional() = default;
  optional(nullopt_t) {}  // NOLINT(runtime/explicit)
  optional(const T& value) : val_(value) {}  // NOLINT(runtime/explicit)
  optional(T&& value) : val_(std::move(value)) {}  // NOLINT(runtime/explicit)
  optional(const optional&) = default;
  optional(optional&&) = default;
  optional& operator=(const optional&) = default;
  optional& operator=(optional&&) = default;
  optional& operator=(nullopt_t) {
    val_.reset();
    return *this;
  }
  optional& operator=(const T& value) {
    val_ = value;
    return *this;
  }
  void swap(optional& other) { val_.swap(other.val_); }

  T& operator*() {
    CHECK(val_.has_value()) << "dereferencing an empty optional";
    return *val_;
  }
  const T& operator*() const {
    CHECK(val_.has_value()) << "dereferencing an empty optional";
    return *val_;
  }
  T* operator->() { return &**this; }
  const T* operator->() const { return &**this; }
  /*! \brief value or throw std::bad_optional_access */
  const T& value() const { return val_.value(); }
  T& value() { return val_.value(); }
  template <typename U>
  T value_or(U&& def) const {
    return val_.value_or(std::forward<U>(def));
  }
  bool has_value() const { return val_.has_value(); }
  explicit operator bool() const { return val_.has_value(); }

  bool operator==(const optional& o) const { return val_ == o.val_; }
  bool operator!=(const optional& o) const { return val_ != o.val_; }
  bool operator==(const T& v) const { return val_.has_value() && *val_ == v; }
  bool operator==(nullopt_t) const { return !val_.has_value(); }
  bool operator!=(nullopt_t) const { return val_.has_value(); }

 private:
  std::optional<T> val_;
};

/*! \brief prints "None" when empty */
template <typename T>
std::ostream& operator<<(std::ostream& os, const optional<T>& t) {
  if (t) {
    os << *t;
  } else {
    os << "None";
  }
  return os;
}

/*! \brief parses "None" (case-sensitive) or a T; integers may end with 'L' */
template <typename T>
std::istream& operator>>(std::istream& is, optional<T>& t) {
  char buf[4];
  std::streampos origin = is.tellg();
  is.read(buf, 4);
  if (is.fail() || !(buf[0] == 'N' && buf[1] == 'o' && buf[2] == 'n' && buf[3] == 'e')) {
    is.clear();
    is.seekg(origin);
    T x;
    is >> x;
    t = x;
    if (std::is_integral<T>::value && !is.eof() && is.peek() == 'L') is.get();
  } else {
    t = nullopt;
  }
  return is;
}

/*! \brief optional<bool>: true / false / 1 / 0 / None (case-insensitive) */
inline std::istream& operator>>(std::istream& is, optional<bool>& t) {
  std::string s;
  is >> s;
  std::string lower = s;
  std::transform(lower.begin(), lower.end(), lower.begin(),
                 [](unsigned char c) { return std::tolower(c); });
  if (lower == "true" || lower == "1") {
    t = true;
  } else if (lower == "false" || lower == "0") {
    t = false;
  } else if (lower == "none") {
    t = nullopt;
  } else {
    is.setstate(std::ios::failbit);
  }
  return is;
}

DMLC_DECLARE_TYPE_NAME(optional<int>, "int or None");
DMLC_DECLARE_TYPE_NAME(optional<bool>, "boolean or None");
DMLC_DECLARE_TYPE_NAME(optional<float>, "float or None");
DMLC_DECLARE_TYPE_NAME(optional<double>, "double or None");
DMLC_DECLARE_TYPE_NAME(optional<int64_t>, "long or None");

}  // namespace dmlc

namespace std {
template <typename T>
struct hash<dmlc::optional<T>> {
  size_t operator()(const dmlc::optional<T>& v) const {
    return v ? std::hash<T>()(*v) : 0;
  }
};
}  // namespace std

#endif  // DMLC_OPTIONAL_H_
