/*!
 * \file dmlc/serializer.h
 * \brief Binary serialization of PODs, strings and STL containers through
 *  dmlc::Stream.
 *
 * Wire format (bit-compatible with the reference, `include/dmlc/serializer.h`
 * :70-206): POD = raw native bytes; std::string and vector<POD> = uint64 count
 * followed by the raw elements; every other container (vector<non-POD>, list,
 * deque, map, set, unordered_*) = uint64 count followed by each element through
 * its own handler; pair = first then second; classes with Save/Load (opted in
 * via has_saveload) call their own methods.  Native byte order (little-endian,
 * enforced by a static_assert in base.h).
 *
 * Implementation is new: a single constexpr dispatch instead of the
 * reference's tag-dispatch class hierarchy.
 */
#ifndef DMLC_SERIALIZER_H_
#define DMLC_SERIALIZER_H_

#include <deque>
#include <list>
#include <map>
#include <set>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "./base.h"
#include "./logging.h"
#include "./type_traits.h"

namespace dmlc {
class Stream;

namespace serializer {

template <typename T>
struct Handler;

namespace detail {
template <typename T>
struct is_std_vector : std::false_type {};
template <typename T, typename A>
struct is_std_vector<std::vector<T, A>> : std::true_type {};

template <typename T>
struct is_pair : std::false_type {};
template <typename A, typename B>
struct is_pair<std::pair<A, B>> : std::true_type {};

/*! \brief containers serialized as "count + elements", read back by insert */
template <typename T>
struct is_collection : std::false_type {};
template <typename K, typename V, typename C, typename A>
struct is_collection<std::map<K, V, C, A>> : std::true_type {};
template <typename K, typename V, typename C, typename A>
struct is_collection<std::multimap<K, V, C, A>> : std::true_type {};
template <typename K, typename C, typename A>
struct is_collection<std::set<K, C, A>> : std::true_type {};
template <typename K, typename C, typename A>
struct is_collection<std::multiset<K, C, A>> : std::true_type {};
template <typename K, typename V, typename H, typename E, typename A>
struct is_collection<std::unordered_map<K, V, H, E, A>> : std::true_type {};
template <typename K, typename V, typename H, typename E, typename A>
struct is_collection<std::unordered_multimap<K, V, H, E, A>> : std::true_type {};
template <typename K, typename H, typename E, typename A>
struct is_collection<std::unordered_set<K, H, E, A>> : std::true_type {};
template <typename K, typename H, typename E, typename A>
struct is_collection<std::unordered_multiset<K, H, E, A>> : std::true_type {};

/*! \brief sequences serialized as "count + elements", read back by push_back */
template <typename T>
struct is_sequence : std::false_type {};
template <typename T, typename A>
struct is_sequence<std::list<T, A>> : std::true_type {};
template <typename T, typename A>
struct is_sequence<std::deque<T, A>> : std::true_type {};

/*! \brief element type used when reading a collection (map keys are non-const) */
template <typename T>
struct collection_value {
  using type = typename T::value_type;
};
template <typename K, typename V, typename C, typename A>
struct collection_value<std::map<K, V, C, A>> {
  using type = std::pair<K, V>;
};
template <typename K, typename V, typename C, typename A>
struct collection_value<std::multimap<K, V, C, A>> {
  using type = std::pair<K, V>;
};
template <typename K, typename V, typename H, typename E, typename A>
struct collection_value<std::unordered_map<K, V, H, E, A>> {
  using type = std::pair<K, V>;
};
template <typename K, typename V, typename H, typename E, typename A>
struct collection_value<std::unordered_multimap<K, V, H, E, A>> {
  using type = std::pair<K, V>;
};
/*! \brief call data->Load(strm); a void-returning Load counts as success */
template <typename T>
inline bool CallLoad(Stream* strm, T* data) {
  if constexpr (std::is_void<decltype(data->Load(strm))>::value) {
    data->Load(strm);
    return true;
  } else {
    return data->Load(strm);
  }
}
}  // namespace detail

/*! \brief raw-byte write/read helpers (defined after Stream, in io.h) */
inline void WriteBytes(Stream* strm, const void* ptr, size_t size);
inline bool ReadBytes(Stream* strm, void* ptr, size_t size);

template <typename T>
struct Handler {
  inline static void Write(Stream* strm, const T& data) {
    if constexpr (has_saveload<T>::value) {
      data.Save(strm);
    } else if constexpr (std::is_same<T, std::string>::value) {
      uint64_t sz = data.length();
      WriteBytes(strm, &sz, sizeof(sz));
      if (sz != 0) WriteBytes(strm, data.data(), data.length());
    } else if constexpr (detail::is_std_vector<T>::value) {
      using E = typename T::value_type;
      uint64_t sz = data.size();
      WriteBytes(strm, &sz, sizeof(sz));
      if constexpr (is_pod<E>::value && !std::is_same<E, bool>::value) {
        if (sz != 0) WriteBytes(strm, data.data(), sizeof(E) * data.size());
      } else {
        for (const auto& e : data) Handler<E>::Write(strm, e);
      }
    } else if constexpr (detail::is_pair<T>::value) {
      Handler<typename T::first_type>::Write(strm, data.first);
      Handler<typename T::second_type>::Write(strm, data.second);
    } else if constexpr (detail::is_collection<T>::value ||
                         detail::is_sequence<T>::value) {
      using E = typename detail::collection_value<T>::type;
      uint64_t sz = data.size();
      WriteBytes(strm, &sz, sizeof(sz));
      for (const auto& e : data) Handler<E>::Write(strm, E(e));
    } else if constexpr (is_pod<T>::value) {
      WriteBytes(strm, &data, sizeof(T));
    } else {
      // classes with Save/Load that did not opt in through has_saveload
      data.Save(strm);
    }
  }

  inline static bool Read(Stream* strm, T* data) {
    if constexpr (has_saveload<T>::value) {
      return detail::CallLoad(strm, data);
    } else if constexpr (std::is_same<T, std::string>::value) {
      uint64_t sz;
      if (!ReadBytes(strm, &sz, sizeof(sz))) return false;
      data->resize(static_cast<size_t>(sz));
      if (sz != 0) return ReadBytes(strm, &(*data)[0], static_cast<size_t>(sz));
      return true;
    } else if constexpr (detail::is_std_vector<T>::value) {
      using E = typename T::value_type;
      uint64_t sz;
      if (!ReadBytes(strm, &sz, sizeof(sz))) return false;
      data->resize(static_cast<size_t>(sz));
      if constexpr (is_pod<E>::value && !std::is_same<E, bool>::value) {
        if (sz != 0) return ReadBytes(strm, data->data(), sizeof(E) * sz);
        return true;
      } else {
        for (size_t i = 0; i < sz; ++i) {
          E e;
          if (!Handler<E>::Read(strm, &e)) return false;
          (*data)[i] = std::move(e);
        }
        return true;
      }
    } else if constexpr (detail::is_pair<T>::value) {
      return Handler<typename T::first_type>::Read(strm, &data->first) &&
             Handler<typename T::second_type>::Read(strm, &data->second);
    } else if constexpr (detail::is_collection<T>::value) {
      using E = typename detail::collection_value<T>::type;
      uint64_t sz;
      if (!ReadBytes(strm, &sz, sizeof(sz))) return false;
      data->clear();
      for (uint64_t i = 0; i < sz; ++i) {
        E e;
        if (!Handler<E>::Read(strm, &e)) return false;
        data->insert(std::move(e));
      }
      return true;
    } else if constexpr (detail::is_sequence<T>::value) {
      using E = typename T::value_type;
      uint64_t sz;
      if (!ReadBytes(strm, &sz, sizeof(sz))) return false;
      data->clear();
      for (uint64_t i = 0; i < sz; ++i) {
        E e;
        if (!Handler<E>::Read(strm, &e)) return false;
        data->push_back(std::move(e));
      }
      return true;
    } else if constexpr (is_pod<T>::value) {
      return ReadBytes(strm, data, sizeof(T));
    } else {
      return detail::CallLoad(strm, data);
    }
  }
};

}  // namespace serializer
}  // namespace dmlc
#endif  // DMLC_SERIALIZER_H_
