/*!
 * \file dmlc/parameter.h
 * \brief Typed, self-documenting parameter structs filled from string
 *  key/value pairs (command lines, URI `?k=v` arguments, JSON, environment).
 *
 * Public surface kept from the reference (`include/dmlc/parameter.h`):
 * ParamError, ParamInitOption {kAllowUnknown, kAllMatch, kAllowHidden},
 * ParamFieldInfo, Parameter<P>::{Init, InitAllowUnknown, UpdateAllowUnknown,
 * UpdateDict, __DICT__, Save, Load, __FIELDS__, __DOC__}, the
 * DMLC_DECLARE_PARAMETER / DMLC_DECLARE_FIELD / DMLC_DECLARE_ALIAS /
 * DMLC_REGISTER_PARAMETER macros, the chainable field setters (set_default,
 * describe, set_range, set_lower_bound, add_enum) and GetEnv / SetEnv.
 *
 * Behaviour (reference RunInit :391-430, field parsers
 * :551-1028, env helpers :1036-1063): an unknown key raises ParamError with
 * the field documentation unless it is allowed (kAllowUnknown collects it,
 * kAllowHidden skips `__name__` keys); a field without a value takes its
 * default or raises ParamError; numeric bounds are checked after every
 * assignment; int and optional<int> fields may carry enum names; bool accepts
 * true/false/1/0 in any case; float/double go through std::stof/stod so an
 * out-of-range text (a float denormal) is a ParamError.
 *
 * Implementation (new): one field template, FieldEntry<T>, whose value codec
 * is chosen by `ValueCodec<T>` specialisations and whose bounds / enum table
 * are members used through `if constexpr`; the manager is a flat vector of
 * fields plus a name -> field map.  A field is located by its byte offset in
 * the struct, recorded by running the struct's declaration body once on a
 * default-constructed instance.
 *
 * \code
 *  struct MyParam : public dmlc::Parameter<MyParam> {
 *    float lr; int nthread; std::string name;
 *    DMLC_DECLARE_PARAMETER(MyParam) {
 *      DMLC_DECLARE_FIELD(lr).set_default(0.01f).set_range(0, 1).describe("lr");
 *      DMLC_DECLARE_FIELD(nthread).set_lower_bound(1).set_default(4);
 *      DMLC_DECLARE_FIELD(name);          // required
 *      DMLC_DECLARE_ALIAS(lr, eta);
 *    }
 *  };
 *  DMLC_REGISTER_PARAMETER(MyParam);     // in one .cc file
 * \endcode
 */
#ifndef DMLC_PARAMETER_H_
#define DMLC_PARAMETER_H_

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <limits>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_set>
#include <utility>
#include <vector>

#include "./base.h"
#include "./json.h"
#include "./logging.h"
#include "./optional.h"
#include "./type_traits.h"

namespace dmlc {

/*! \brief invalid parameter input (unknown key, bad text, value out of bounds) */
struct ParamError : dmlc::Error {
  explicit ParamError(const std::string& msg) : dmlc::Error(msg) {}
};

/*! \brief what Init does with a key that names no field */
enum ParamInitOption {
  /*! \brief collect / ignore it */
  kAllowUnknown,
  /*! \brief raise ParamError */
  kAllMatch,
  /*! \brief ignore `__name__` keys, raise ParamError for the others */
  kAllowHidden
};

/*! \brief documentation of one field */
struct ParamFieldInfo {
  std::string name;
  std::string type;
  /*! \brief type plus "required" or the default, e.g. "int, optional, default=4" */
  std::string type_info_str;
  std::string description;
};

template <typename ValueType>
inline ValueType GetEnv(const char* key, ValueType default_value);
template <typename ValueType>
inline void SetEnv(const char* key, ValueType value);

namespace parameter {

using KeyValues = std::vector<std::pair<std::string, std::string>>;

/*! \brief throw a ParamError built from stream-able pieces */
template <typename... Parts>
[[noreturn]] inline void Fail(const Parts&... parts) {
  std::ostringstream why;
  (why << ... << parts);
  throw ParamError(why.str());
}

/*!
 * \brief text <-> value for one C++ type.  Parse returns false on text that
 *  is not entirely a value (trailing blanks are tolerated).
 */
template <typename T, typename Enable = void>
struct ValueCodec {
  static bool Parse(const std::string& text, T* out) {
    std::istringstream in(text);
    in >> *out;
    if (in.fail()) return false;
    in >> std::ws;  // anything but blanks after the value is an error
    return in.eof();
  }
  static void Print(std::ostream& os, const T& v) { os << v; }
};

template <>
struct ValueCodec<std::string> {
  static bool Parse(const std::string& text, std::string* out) {
    *out = text;
    return true;
  }
  static void Print(std::ostream& os, const std::string& v) { os << v; }
};

template <>
struct ValueCodec<bool> {
  static bool Parse(const std::string& text, bool* out) {
    const size_t b = text.find_first_not_of(" \t\r\n");
    if (b == std::string::npos) return false;
    const size_t e = text.find_last_not_of(" \t\r\n");
    std::string word = text.substr(b, e - b + 1);
    for (char& c : word) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    if (word == "1" || word == "true") {
      *out = true;
    } else if (word == "0" || word == "false") {
      *out = false;
    } else {
      return false;
    }
    return true;
  }
  static void Print(std::ostream& os, bool v) { os << (v ? "True" : "False"); }
};

/*! \brief float / double: std::stof / std::stod semantics, full precision out */
template <typename T>
struct ValueCodec<T, typename std::enable_if<std::is_floating_point<T>::value>::type> {
  static bool Parse(const std::string& text, T* out) {
    size_t used = 0;
    try {
      *out = std::is_same<T, float>::value ? static_cast<T>(std::stof(text, &used))
                                           : static_cast<T>(std::stod(text, &used));
    } catch (const std::invalid_argument&) {
      return false;
    }  // std::out_of_range propagates: the caller reports it separately
    return text.find_first_not_of(" \t\r\n", used) == std::string::npos;
  }
  static void Print(std::ostream& os, T v) {
    os << std::setprecision(std::numeric_limits<T>::max_digits10) << v;
  }
};

/*! \brief type-erased view of one declared field (the manager's element) */
class FieldAccessEntry {
 public:
  virtual ~FieldAccessEntry() = default;
  /*! \brief parse `text` into the field of the struct at `obj` (ParamError on bad text) */
  virtual void Set(void* obj, const std::string& text) const = 0;
  /*! \brief bounds check of the current value (ParamError when violated) */
  virtual void Check(void* obj) const = 0;
  /*! \brief store the default (ParamError for a required field) */
  virtual void SetDefault(void* obj) const = 0;
  virtual std::string GetStringValue(void* obj) const = 0;
  [[nodiscard]] virtual ParamFieldInfo GetFieldInfo() const = 0;

  const std::string& key() const { return key_; }
  bool has_default() const { return defaulted_; }
  /*! \brief position of the field in declaration order */
  size_t index() const { return index_; }

 protected:
  friend class ParamManager;
  std::string key_, type_, doc_;
  std::ptrdiff_t offset_{0};
  size_t index_{0};
  bool defaulted_{false};
};

/*! \brief bounds of a numeric field */
template <typename T>
struct Bounds {
  bool has_lo{false}, has_hi{false};
  T lo{}, hi{};
};

/*! \brief enum names of an int / optional<int> field */
struct EnumTable {
  std::map<std::string, int> by_name;
  std::map<int, std::string> by_value;
  bool empty() const { return by_name.empty(); }
  std::string Listing(bool with_none) const {
    std::string text = with_none ? "{None" : "{";
    bool first = !with_none;
    for (const auto& kv : by_name) {
      text += first ? "'" : ", '";
      text += kv.first + "'";
      first = false;
    }
    return text + "}";
  }
};

template <typename T>
struct IsOptionalInt : std::false_type {};
template <>
struct IsOptionalInt<optional<int>> : std::true_type {};

/*!
 * \brief one declared field of type T.  Numeric types (bool excluded) take
 *  bounds; int and optional<int> take enum names.
 */
template <typename T>
class FieldEntry : public FieldAccessEntry {
 public:
  static constexpr bool kNumeric = std::is_arithmetic<T>::value && !std::is_same<T, bool>::value;
  static constexpr bool kEnumerable = std::is_same<T, int>::value || IsOptionalInt<T>::value;

  /*! \brief bind to `field`, a member of the struct that starts at `obj` */
  void Init(const std::string& key, void* obj, T& field) {  // NOLINT(runtime/references)
    key_ = key;
    if (type_.empty()) type_ = type_name<T>();
    offset_ = reinterpret_cast<char*>(&field) - static_cast<char*>(obj);
  }

  FieldEntry& set_default(const T& v) {
    default_ = v;
    defaulted_ = true;
    return *this;
  }
  FieldEntry& describe(const std::string& doc) {
    doc_ = doc;
    return *this;
  }
  FieldEntry& set_range(T lo, T hi) {
    static_assert(kNumeric, "set_range needs a numeric field");
    bounds_.has_lo = bounds_.has_hi = true;
    bounds_.lo = lo;
    bounds_.hi = hi;
    return *this;
  }
  FieldEntry& set_lower_bound(T lo) {
    static_assert(kNumeric, "set_lower_bound needs a numeric field");
    bounds_.has_lo = true;
    bounds_.lo = lo;
    return *this;
  }
  FieldEntry& add_enum(const std::string& name, int value) {
    static_assert(kEnumerable, "add_enum needs an int or optional<int> field");
    if (IsOptionalInt<T>::value && name == "None") {
      LOG(FATAL) << key_ << ": \"None\" is reserved for the empty optional<int>";
    }
    if (enums_.by_name.count(name) != 0 || enums_.by_value.count(value) != 0) {
      LOG(FATAL) << key_ << ": enum name '" << name << "' or value " << value
                 << " declared twice; declared so far: " << enums_.Listing(false);
    }
    enums_.by_name[name] = value;
    enums_.by_value[value] = name;
    return *this;
  }

  void Set(void* obj, const std::string& text) const override {
    T& slot = Ref(obj);
    if constexpr (kEnumerable) {
      if (!enums_.empty() && !(IsOptionalInt<T>::value && text == "None")) {
        auto hit = enums_.by_name.find(text);
        if (hit == enums_.by_name.end()) {
          Fail("parameter ", key_, ": '", text, "' is not one of ",
               enums_.Listing(IsOptionalInt<T>::value));
        }
        slot = hit->second;
        return;
      }
    }
    bool ok = false;
    try {
      ok = ValueCodec<T>::Parse(text, &slot);
    } catch (const std::out_of_range&) {
      Fail("parameter ", key_, ": value '", text, "' is out of the range of ", type_);
    }
    if (!ok) Fail("parameter ", key_, ": cannot read '", text, "' as ", type_);
  }

  void Check(void* obj) const override {
    if constexpr (kNumeric) {
      const T v = Ref(obj);
      const bool below = bounds_.has_lo && v < bounds_.lo;
      const bool above = bounds_.has_hi && v > bounds_.hi;
      if (below || above) {
        std::ostringstream why;
        why << "parameter " << key_ << " = " << v << " is outside ";
        if (bounds_.has_lo) {
          why << '[' << bounds_.lo;
        } else {
          why << "(-inf";
        }
        why << ", ";
        if (bounds_.has_hi) {
          why << bounds_.hi << ']';
        } else {
          why << "+inf)";
        }
        if (!doc_.empty()) why << " (" << doc_ << ')';
        throw ParamError(why.str());
      }
    } else {
      (void)obj;
    }
  }

  void SetDefault(void* obj) const override {
    if (!defaulted_) Fail("required parameter ", key_, " (", type_, ") was not given");
    Ref(obj) = default_;
  }

  std::string GetStringValue(void* obj) const override { return ValueText(Ref(obj)); }

  ParamFieldInfo GetFieldInfo() const override {
    bool enumerated = false;
    if constexpr (kEnumerable) enumerated = !enums_.empty();
    std::string summary = enumerated ? Listing() : type_;
    if (!defaulted_) {
      summary += ", required";
    } else if (std::is_same<T, std::string>::value) {
      summary += ", optional, default='" + ValueText(default_) + "'";
    } else {
      summary += ", optional, default=" + ValueText(default_);
    }
    return ParamFieldInfo{key_, type_, summary, doc_};
  }

 private:
  T& Ref(void* obj) const { return *reinterpret_cast<T*>(static_cast<char*>(obj) + offset_); }
  std::string Listing() const {
    if constexpr (kEnumerable) return enums_.Listing(IsOptionalInt<T>::value);
    return type_;
  }
  std::string ValueText(const T& v) const {
    std::ostringstream text;
    Show(text, v);
    return text.str();
  }
  void Show(std::ostream& out, const T& v) const {
    if constexpr (kEnumerable) {
      if (!enums_.empty()) {
        int raw = 0;
        if constexpr (IsOptionalInt<T>::value) {
          if (!v.has_value()) {
            out << "None";
            return;
          }
          raw = *v;
        } else {
          raw = v;
        }
        auto hit = enums_.by_value.find(raw);
        CHECK(hit != enums_.by_value.end())
            << "parameter " << key_ << " holds " << raw << ", which has no enum name";
        out << hit->second;
        return;
      }
    }
    ValueCodec<T>::Print(out, v);
  }

  T default_{};
  Bounds<T> bounds_;
  EnumTable enums_;
};

/*! \brief the fields of one parameter struct, in declaration order */
class ParamManager {
 public:
  ParamManager() = default;
  ParamManager(const ParamManager&) = delete;
  ParamManager& operator=(const ParamManager&) = delete;

  void set_name(const std::string& name) { title_ = name; }
  const std::string& name() const { return title_; }

  void AddEntry(const std::string& key, FieldAccessEntry* entry) {
    std::unique_ptr<FieldAccessEntry> owned(entry);
    if (by_key_.count(key) != 0) LOG(FATAL) << title_ << ": field '" << key << "' declared twice";
    owned->index_ = fields_.size();
    by_key_[key] = owned.get();
    fields_.push_back(std::move(owned));
  }
  void AddAlias(const std::string& field, const std::string& alias) {
    auto target = by_key_.find(field);
    if (target == by_key_.end()) LOG(FATAL) << title_ << ": alias of unknown field '" << field << "'";
    if (by_key_.count(alias) != 0) LOG(FATAL) << title_ << ": alias '" << alias << "' is taken";
    by_key_[alias] = target->second;
  }
  /*! \brief the field named `key` (or aliased so), nullptr if none */
  FieldAccessEntry* Find(const std::string& key) const {
    auto hit = by_key_.find(key);
    return hit == by_key_.end() ? nullptr : hit->second;
  }

  /*! \brief assign the given pairs, then defaults to every field left unset */
  template <typename It>
  void RunInit(void* obj, It first, It last, KeyValues* unknown, ParamInitOption option) const {
    const std::vector<bool> given = Assign(obj, first, last, unknown, option);
    for (size_t i = 0; i < fields_.size(); ++i) {
      if (!given[i]) fields_[i]->SetDefault(obj);
    }
  }
  /*! \brief assign the given pairs only */
  template <typename It>
  void RunUpdate(void* obj, It first, It last, KeyValues* unknown, ParamInitOption option) const {
    (void)Assign(obj, first, last, unknown, option);
  }

  std::vector<ParamFieldInfo> GetFieldInfo() const {
    std::vector<ParamFieldInfo> out;
    out.reserve(fields_.size());
    for (const auto& f : fields_) out.push_back(f->GetFieldInfo());
    return out;
  }
  void PrintDocString(std::ostream& out) const {
    for (const auto& f : fields_) {
      const ParamFieldInfo doc = f->GetFieldInfo();
      out << doc.name << " : " << doc.type_info_str << "\n";
      if (!doc.description.empty()) out << "    " << doc.description << "\n";
    }
  }
  KeyValues GetDict(void* obj) const {
    KeyValues out;
    for (const auto& f : fields_) out.emplace_back(f->key(), f->GetStringValue(obj));
    return out;
  }
  template <typename Map>
  void UpdateDict(void* obj, Map* dict) const {
    for (const auto& f : fields_) (*dict)[f->key()] = f->GetStringValue(obj);
  }

 private:
  static bool IsHidden(const std::string& key) {
    const size_t n = key.size();
    return n > 4 && key[0] == '_' && key[1] == '_' && key[n - 1] == '_' && key[n - 2] == '_';
  }
  template <typename It>
  std::vector<bool> Assign(void* obj, It first, It last, KeyValues* unknown,
                           ParamInitOption option) const {
    std::vector<bool> given(fields_.size(), false);
    for (It it = first; it != last; ++it) {
      const std::string key(it->first), text(it->second);
      FieldAccessEntry* f = Find(key);
      if (f != nullptr) {
        f->Set(obj, text);
        f->Check(obj);
        given[f->index()] = true;
        continue;
      }
      if (option == kAllowUnknown) {
        if (unknown != nullptr) unknown->emplace_back(key, text);
      } else if (!(option == kAllowHidden && IsHidden(key))) {
        std::ostringstream why;
        why << title_ << " has no parameter '" << key << "'; its parameters are:\n";
        PrintDocString(why);
        throw ParamError(why.str());
      }
    }
    return given;
  }

  std::string title_;
  std::vector<std::unique_ptr<FieldAccessEntry>> fields_;
  std::map<std::string, FieldAccessEntry*> by_key_;
};

/*! \brief builds a struct's ParamManager by declaring on a scratch instance */
template <typename PType>
struct ParamManagerSingleton {
  ParamManager manager;
  explicit ParamManagerSingleton(const std::string& name) {
    manager.set_name(name);
    PType scratch;
    scratch.__DECLARE__(this);
  }
};

}  // namespace parameter

/*! \brief CRTP base of every parameter struct */
template <typename PType>
struct Parameter {
 public:
  /*! \brief assign `kwargs` ((key, value) string pairs), defaults to the rest */
  template <typename Container>
  inline void Init(const Container& kwargs, ParamInitOption option = kAllowHidden) {
    Manager()->RunInit(Self(), kwargs.begin(), kwargs.end(), nullptr, option);
  }
  /*! \brief Init that returns the pairs naming no field instead of failing */
  template <typename Container>
  inline parameter::KeyValues InitAllowUnknown(const Container& kwargs) {
    parameter::KeyValues rest;
    Manager()->RunInit(Self(), kwargs.begin(), kwargs.end(), &rest, kAllowUnknown);
    return rest;
  }
  /*! \brief assign the given fields only (others keep their values); unknown pairs returned */
  template <typename Container>
  inline parameter::KeyValues UpdateAllowUnknown(const Container& kwargs) {
    parameter::KeyValues rest;
    Manager()->RunUpdate(Self(), kwargs.begin(), kwargs.end(), &rest, kAllowUnknown);
    return rest;
  }
  /*! \brief write every field's text into `dict` */
  template <typename Container>
  inline void UpdateDict(Container* dict) const {
    Manager()->UpdateDict(Self(), dict);
  }
  /*! \brief every field as text */
  inline std::map<std::string, std::string> __DICT__() const {
    const parameter::KeyValues kv = Manager()->GetDict(Self());
    return std::map<std::string, std::string>(kv.begin(), kv.end());
  }
  /*! \brief JSON object {field: text} */
  inline void Save(JSONWriter* writer) const { writer->Write(__DICT__()); }
  /*! \brief read the object written by Save (every key must name a field) */
  inline void Load(JSONReader* reader) {
    std::map<std::string, std::string> kv;
    reader->Read(&kv);
    Init(kv);
  }
  inline static std::vector<ParamFieldInfo> __FIELDS__() { return PType::__MANAGER__()->GetFieldInfo(); }
  inline static std::string __DOC__() {
    std::ostringstream doc;
    PType::__MANAGER__()->PrintDocString(doc);
    return doc.str();
  }

 protected:
  /*! \brief declare `field` under `key` (DMLC_DECLARE_FIELD expands to this) */
  template <typename DType>
  inline parameter::FieldEntry<DType>& DECLARE(parameter::ParamManagerSingleton<PType>* owner,
                                               const std::string& key,
                                               DType& field) {  // NOLINT(runtime/references)
    auto* entry = new parameter::FieldEntry<DType>();
    entry->Init(key, Self(), field);
    owner->manager.AddEntry(key, entry);
    return *entry;
  }

 private:
  static parameter::ParamManager* Manager() { return PType::__MANAGER__(); }
  PType* Self() const { return static_cast<PType*>(const_cast<Parameter*>(this)); }
};

/*! \brief start the field declarations of PType (a body follows) */
#define DMLC_DECLARE_PARAMETER(PType)                    \
  static ::dmlc::parameter::ParamManager* __MANAGER__(); \
  inline void __DECLARE__(::dmlc::parameter::ParamManagerSingleton<PType>* manager)

/*! \brief declare one field; chain set_default / describe / set_range / ... */
#define DMLC_DECLARE_FIELD(FieldName) this->DECLARE(manager, #FieldName, FieldName)

/*! \brief let `AliasName` name the field `FieldName` too */
#define DMLC_DECLARE_ALIAS(FieldName, AliasName) \
  manager->manager.AddAlias(#FieldName, #AliasName)

/*! \brief define PType's field table (exactly one .cc file) */
#define DMLC_REGISTER_PARAMETER(PType)                                       \
  ::dmlc::parameter::ParamManager* PType::__MANAGER__() {                    \
    static ::dmlc::parameter::ParamManagerSingleton<PType> table_(#PType);   \
    return &table_.manager;                                                  \
  }                                                                          \
  static DMLC_ATTRIBUTE_UNUSED ::dmlc::parameter::ParamManager&              \
      __make__##PType##ParamManager__ = (*PType::__MANAGER__())

template <typename ValueType>
inline ValueType GetEnv(const char* key, ValueType default_value) {
  const char* text = std::getenv(key);
  if (text == nullptr || text[0] == '\0') return default_value;  // unset or blank
  ValueType value = default_value;
  parameter::FieldEntry<ValueType> codec;
  codec.Init(key, &value, value);
  codec.Set(&value, text);
  return value;
}

template <typename ValueType>
inline void SetEnv(const char* key, ValueType value) {
  parameter::FieldEntry<ValueType> codec;
  codec.Init(key, &value, value);
  ::setenv(key, codec.GetStringValue(&value).c_str(), 1);
}

}  // namespace dmlc
#endif  // DMLC_PARAMETER_H_
