/*!
 * \file dmlc/type_traits.h
 * \brief Opt-in type traits and human-readable type names.
 *
 * Parity: reference `include/dmlc/type_traits.h` — is_pod / is_integral /
 * is_floating_point / is_arithmetic (:21-76), type_name<T>() (:86-103),
 * has_saveload (:110-113), DMLC_DECLARE_TRAITS (:126-130),
 * DMLC_DECLARE_TYPE_NAME (:133-139), IfThenElseType (:180-188).
 * Users may specialise the traits (DMLC_DECLARE_TRAITS) so that custom structs
 * are serialized as raw bytes or through Save/Load.
 */
#ifndef DMLC_TYPE_TRAITS_H_
#define DMLC_TYPE_TRAITS_H_

#include <string>
#include <type_traits>

#include "./base.h"

namespace dmlc {

template <typename T>
struct is_pod {
  static const bool value =
      std::is_trivially_copyable<T>::value && std::is_standard_layout<T>::value;
};
template <typename T>
struct is_integral {
  static const bool value = std::is_integral<T>::value;
};
template <typename T>
struct is_floating_point {
  static const bool value = std::is_floating_point<T>::value;
};
template <typename T>
struct is_arithmetic {
  static const bool value = std::is_arithmetic<T>::value;
};
/*! \brief true when T has member Save(Stream*) / Load(Stream*) (opt-in) */
template <typename T>
struct has_saveload {
  static const bool value = false;
};

/*! \brief compile-time select between two types */
template <bool cond, typename Then, typename Else>
struct IfThenElseType {
  typedef Then Type;
};
template <typename Then, typename Else>
struct IfThenElseType<false, Then, Else> {
  typedef Else Type;
};

/*! \brief helper that yields "" for undeclared types */
template <typename T>
struct type_name_helper {
  static inline std::string value() { return ""; }
};
/*! \brief readable name of T; "" when never declared */
template <typename T>
inline std::string type_name() {
  return type_name_helper<T>::value();
}

#define DMLC_DECLARE_TRAITS(Trait, Type, Value) \
  template <>                                   \
  struct Trait<Type> {                          \
    static const bool value = Value;            \
  }

#define DMLC_DECLARE_TYPE_NAME(Type, Name)                 \
  template <>                                              \
  struct type_name_helper<Type> {                          \
    static inline std::string value() { return Name; }     \
  }

DMLC_DECLARE_TYPE_NAME(float, "float");
DMLC_DECLARE_TYPE_NAME(double, "double");
DMLC_DECLARE_TYPE_NAME(int, "int");
DMLC_DECLARE_TYPE_NAME(int64_t, "long");
DMLC_DECLARE_TYPE_NAME(uint32_t, "int (non-negative)");
DMLC_DECLARE_TYPE_NAME(uint64_t, "long (non-negative)");
DMLC_DECLARE_TYPE_NAME(std::string, "string");
DMLC_DECLARE_TYPE_NAME(bool, "boolean");
DMLC_DECLARE_TYPE_NAME(void*, "ptr");

}  // namespace dmlc
#endif  // DMLC_TYPE_TRAITS_H_
