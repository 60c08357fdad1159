/*!
 * \file dmlc/parameter.h
 * \brief Typed, self-documenting parameter structs initialised from
 *  string key/value maps (command lines, URI `?k=v` args, JSON, env vars).
 *
 * Parity: reference `include/dmlc/parameter.h` — ParamError (:30),
 * ParamInitOption (:72-79), ParamFieldInfo (:84-96), Parameter<P>::Init /
 * InitAllowUnknown / UpdateDict / __DICT__ / Save / Load / __FIELDS__ / __DOC__
 * (:123-230), DMLC_DECLARE_PARAMETER / FIELD / ALIAS / REGISTER_PARAMETER
 * (:260-293), RunInit semantics (:391-430: unknown key -> ParamError listing
 * the documentation, `__key__` hidden keys skipped under kAllowHidden, missing
 * fields get their default or raise "Required parameter"), FieldEntry
 * specialisations for numbers (ranges), int / optional<int> enums, strings,
 * bool (true/false/1/0, case-insensitive), float/double via std::stof/stod with
 * out-of-range -> ParamError (:551-1028), GetEnv / SetEnv (:1036-1063).
 *
 * Usage:
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
 * Fields are located through their byte offset inside the struct, recorded by
 * running __DECLARE__ once on a default-constructed instance.
 */
#ifndef DMLC_PARAMETER_H_
#define DMLC_PARAMETER_H_

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "./base.h"
#include "./json.h"
#include "./logging.h"
#include "./optional.h"
#include "./type_traits.h"

namespace dmlc {

/*! \brief error raised on invalid parameter input */
struct ParamError : public dmlc::Error {
  explicit ParamError(const std::string& msg) : dmlc::Error(msg) {}
};

/*! \brief read env var `key` as T; unset or blank -> default_value */
template <typename ValueType>
inline ValueType GetEnv(const char* key, ValueType default_value);
/*! \brief set env var `key` to the text form of `value` */
template <typename ValueType>
inline void SetEnv(const char* key, ValueType value);

namespace parameter {
class ParamManager;
template <typename PType>
struct ParamManagerSingleton;
class FieldAccessEntry;
template <typename DType>
class FieldEntry;
}  // namespace parameter

/*! \brief how Init treats keys that match no field */
enum ParamInitOption {
  /*! \brief unknown keys are ignored */
  kAllowUnknown,
  /*! \brief every key must match a field */
  kAllMatch,
  /*! \brief unknown keys of the form __xxx__ are ignored, others are errors */
  kAllowHidden
};

/*! \brief documentation record of one field */
struct ParamFieldInfo {
  std::string name;
  std::string type;
  std::string type_info_str;
  std::string description;
};

/*! \brief CRTP base of every parameter struct */
template <typename PType>
struct Parameter {
 public:
  /*! \brief set fields from an iterable of (key, value) string pairs */
  template <typename Container>
  inline void Init(const Container& kwargs, ParamInitOption option = kAllowHidden) {
    PType::__MANAGER__()->RunInit(static_cast<PType*>(this), kwargs.begin(),
                                  kwargs.end(), nullptr, option);
  }
  /*! \brief like Init but returns the (key, value) pairs that matched no field */
  template <typename Container>
  inline std::vector<std::pair<std::string, std::string>> InitAllowUnknown(
      const Container& kwargs) {
    std::vector<std::pair<std::string, std::string>> unknown;
    PType::__MANAGER__()->RunInit(static_cast<PType*>(this), kwargs.begin(),
                                  kwargs.end(), &unknown, kAllowUnknown);
    return unknown;
  }
  /*!
   * \brief update only the given fields (no defaults applied to the others);
   *  returns unknown pairs
   */
  template <typename Container>
  inline std::vector<std::pair<std::string, std::string>> UpdateAllowUnknown(
      const Container& kwargs) {
    std::vector<std::pair<std::string, std::string>> unknown;
    PType::__MANAGER__()->RunUpdate(static_cast<PType*>(this), kwargs.begin(),
                                    kwargs.end(), &unknown, kAllowUnknown);
    return unknown;
  }
  /*! \brief write the current value of every field into `dict` */
  template <typename Container>
  inline void UpdateDict(Container* dict) const {
    PType::__MANAGER__()->UpdateDict(head(), dict);
  }
  /*! \brief all fields as strings */
  inline std::map<std::string, std::string> __DICT__() const {
    std::vector<std::pair<std::string, std::string>> vec =
        PType::__MANAGER__()->GetDict(head());
    return std::map<std::string, std::string>(vec.begin(), vec.end());
  }
  /*! \brief JSON object of all fields (as strings) */
  inline void Save(JSONWriter* writer) const { writer->Write(this->__DICT__()); }
  /*! \brief load from the JSON written by Save (every key must be known) */
  inline void Load(JSONReader* reader) {
    std::map<std::string, std::string> kwargs;
    reader->Read(&kwargs);
    this->Init(kwargs);
  }
  /*! \brief documentation of every field */
  inline static std::vector<ParamFieldInfo> __FIELDS__() {
    return PType::__MANAGER__()->GetFieldInfo();
  }
  /*! \brief formatted documentation string */
  inline static std::string __DOC__() {
    std::ostringstream os;
    PType::__MANAGER__()->PrintDocString(os);
    return os.str();
  }

 protected:
  /*! \brief register field `ref` under `key` (used by DMLC_DECLARE_FIELD) */
  template <typename DType>
  inline parameter::FieldEntry<DType>& DECLARE(
      parameter::ParamManagerSingleton<PType>* manager, const std::string& key,
      DType& ref) {  // NOLINT(runtime/references)
    auto* e = new parameter::FieldEntry<DType>();
    e->Init(key, this->head(), ref);
    manager->manager.AddEntry(key, e);
    return *e;
  }

 private:
  inline PType* head() const {
    return static_cast<PType*>(const_cast<Parameter<PType>*>(this));
  }
};

/*! \brief declare the parameter struct's field list: body follows */
#define DMLC_DECLARE_PARAMETER(PType)                 \
  static ::dmlc::parameter::ParamManager* __MANAGER__(); \
  inline void __DECLARE__(::dmlc::parameter::ParamManagerSingleton<PType>* manager)

/*! \brief declare one field inside DMLC_DECLARE_PARAMETER */
#define DMLC_DECLARE_FIELD(FieldName) this->DECLARE(manager, #FieldName, FieldName)

/*! \brief make `AliasName` an alternative key of field `FieldName` */
#define DMLC_DECLARE_ALIAS(FieldName, AliasName) \
  manager->manager.AddAlias(#FieldName, #AliasName)

/*! \brief define the manager of a parameter struct (one .cc file) */
#define DMLC_REGISTER_PARAMETER(PType)                                   \
  ::dmlc::parameter::ParamManager* PType::__MANAGER__() {                \
    static ::dmlc::parameter::ParamManagerSingleton<PType> inst(#PType); \
    return &inst.manager;                                                \
  }                                                                      \
  static DMLC_ATTRIBUTE_UNUSED ::dmlc::parameter::ParamManager&          \
      __make__##PType##ParamManager__ = (*PType::__MANAGER__())

namespace parameter {

/*! \brief type-erased access to one field */
class FieldAccessEntry {
 public:
  virtual ~FieldAccessEntry() = default;
  /*! \brief write the default into the field; ParamError if there is none */
  virtual void SetDefault(void* head) const = 0;
  /*! \brief parse `value` into the field */
  virtual void Set(void* head, const std::string& value) const = 0;
  /*! \brief validate the field's current value */
  virtual void Check(void* /*head*/) const {}
  virtual std::string GetStringValue(void* head) const = 0;
  virtual ParamFieldInfo GetFieldInfo() const = 0;
  /*! \brief has a default (or is optional) */
  bool has_default() const { return has_default_; }
  const std::string& key() const { return key_; }
  size_t index() const { return index_; }

 protected:
  friend class ParamManager;
  bool has_default_{false};
  size_t index_{0};
  std::string key_;
  std::string type_;
  std::string description_;
  virtual void PrintDefaultValueString(std::ostream& os) const = 0;
};

/*! \brief owns the field entries of one parameter struct */
class ParamManager {
 public:
  ~ParamManager() {
    for (auto* e : entry_) delete e;
  }
  /*! \brief find an entry by key or alias */
  inline FieldAccessEntry* Find(const std::string& key) const {
    auto it = entry_map_.find(key);
    return it == entry_map_.end() ? nullptr : it->second;
  }
  template <typename RandomAccessIterator>
  inline void RunInit(void* head, RandomAccessIterator begin, RandomAccessIterator end,
                      std::vector<std::pair<std::string, std::string>>* unknown_args,
                      ParamInitOption option) const {
    std::set<FieldAccessEntry*> selected;
    ApplyArgs(head, begin, end, unknown_args, option, &selected);
    for (auto* e : entry_) {
      if (selected.count(e) == 0) {
        if (!e->has_default()) {
          std::ostringstream os;
          os << "Required parameter " << e->key_ << " of " << e->type_
             << " is not presented";
          throw ParamError(os.str());
        }
        e->SetDefault(head);
      }
    }
  }
  template <typename RandomAccessIterator>
  inline void RunUpdate(void* head, RandomAccessIterator begin, RandomAccessIterator end,
                        std::vector<std::pair<std::string, std::string>>* unknown_args,
                        ParamInitOption option) const {
    std::set<FieldAccessEntry*> selected;
    ApplyArgs(head, begin, end, unknown_args, option, &selected);
  }
  inline void AddEntry(const std::string& key, FieldAccessEntry* e) {
    e->index_ = entry_.size();
    if (entry_map_.count(key) != 0) {
      LOG(FATAL) << "key " << key << " has already been registered in " << name_;
    }
    entry_.push_back(e);
    entry_map_[key] = e;
  }
  inline void AddAlias(const std::string& field, const std::string& alias) {
    if (entry_map_.count(field) == 0) {
      LOG(FATAL) << "key " << field << " has not been registered in " << name_;
    }
    if (entry_map_.count(alias) != 0) {
      LOG(FATAL) << "Alias " << alias << " has already been registered in " << name_;
    }
    entry_map_[alias] = entry_map_[field];
  }
  inline void set_name(const std::string& name) { name_ = name; }
  inline std::vector<ParamFieldInfo> GetFieldInfo() const {
    std::vector<ParamFieldInfo> ret(entry_.size());
    for (size_t i = 0; i < entry_.size(); ++i) ret[i] = entry_[i]->GetFieldInfo();
    return ret;
  }
  inline void PrintDocString(std::ostream& os) const {
    for (auto* e : entry_) {
      ParamFieldInfo info = e->GetFieldInfo();
      os << info.name << " : " << info.type_info_str << '\n';
      if (!info.description.empty()) os << "    " << info.description << '\n';
    }
  }
  inline std::vector<std::pair<std::string, std::string>> GetDict(void* head) const {
    std::vector<std::pair<std::string, std::string>> ret;
    for (auto* e : entry_) ret.emplace_back(e->key_, e->GetStringValue(head));
    return ret;
  }
  template <typename Container>
  inline void UpdateDict(void* head, Container* dict) const {
    for (auto* e : entry_) (*dict)[e->key_] = e->GetStringValue(head);
  }

 private:
  template <typename RandomAccessIterator>
  inline void ApplyArgs(void* head, RandomAccessIterator begin, RandomAccessIterator end,
                        std::vector<std::pair<std::string, std::string>>* unknown_args,
                        ParamInitOption option, std::set<FieldAccessEntry*>* selected) const {
    for (auto it = begin; it != end; ++it) {
      const std::string key = it->first;
      const std::string value = it->second;
      if (FieldAccessEntry* e = Find(key)) {
        e->Set(head, value);
        e->Check(head);
        selected->insert(e);
      } else if (option == kAllowUnknown) {
        if (unknown_args != nullptr) unknown_args->emplace_back(key, value);
      } else if (option == kAllowHidden && key.size() > 4 &&
                 key.compare(0, 2, "__") == 0 &&
                 key.compare(key.size() - 2, 2, "__") == 0) {
        // hidden key: skipped
      } else {
        std::ostringstream os;
        os << "Cannot find argument \'" << key << "\', Possible Arguments:\n";
        os << "----------------\n";
        PrintDocString(os);
        throw ParamError(os.str());
      }
    }
  }
  std::string name_;
  std::vector<FieldAccessEntry*> entry_;
  std::map<std::string, FieldAccessEntry*> entry_map_;
};

/*! \brief builds the field table once by declaring on a dummy instance */
template <typename PType>
struct ParamManagerSingleton {
  ParamManager manager;
  explicit ParamManagerSingleton(const std::string& param_name) {
    PType param;
    manager.set_name(param_name);
    param.__DECLARE__(this);
  }
};

/*! \brief common machinery of typed field entries (CRTP) */
template <typename TEntry, typename DType>
class FieldEntryBase : public FieldAccessEntry {
 public:
  using EntryType = TEntry;
  void Set(void* head, const std::string& value) const override {
    std::istringstream is(value);
    is >> this->Get(head);
    if (!is.fail()) {
      while (!is.eof()) {
        int ch = is.get();
        if (ch == EOF) {
          is.clear();
          break;
        }
        if (!std::isspace(ch)) {
          is.setstate(std::ios::failbit);
          break;
        }
      }
    }
    if (is.fail()) {
      std::ostringstream os;
      os << "Invalid Parameter format for " << key_ << " expect " << type_
         << " but value=\'" << value << '\'';
      throw ParamError(os.str());
    }
  }
  std::string GetStringValue(void* head) const override {
    std::ostringstream os;
    PrintValue(os, this->Get(head));
    return os.str();
  }
  ParamFieldInfo GetFieldInfo() const override {
    ParamFieldInfo info;
    std::ostringstream os;
    info.name = key_;
    info.type = type_;
    os << type_;
    if (has_default_) {
      os << ',' << " optional, default=";
      PrintDefaultValueString(os);
    } else {
      os << ", required";
    }
    info.type_info_str = os.str();
    info.description = description_;
    return info;
  }
  void SetDefault(void* head) const override {
    if (!has_default_) {
      std::ostringstream os;
      os << "Required parameter " << key_ << " of " << type_ << " is not presented";
      throw ParamError(os.str());
    }
    this->Get(head) = default_value_;
  }
  inline TEntry& self() { return *static_cast<TEntry*>(this); }
  inline TEntry& set_default(const DType& default_value) {
    default_value_ = default_value;
    has_default_ = true;
    return self();
  }
  inline TEntry& describe(const std::string& description) {
    description_ = description;
    return self();
  }
  inline void Init(const std::string& key, void* head, DType& ref) {  // NOLINT(*)
    key_ = key;
    if (type_.empty()) type_ = type_name<DType>();
    offset_ = reinterpret_cast<char*>(&ref) - reinterpret_cast<char*>(head);
  }

 protected:
  virtual void PrintValue(std::ostream& os, DType value) const { os << value; }  // NOLINT
  void PrintDefaultValueString(std::ostream& os) const override {
    PrintValue(os, default_value_);
  }
  inline DType& Get(void* head) const {
    return *reinterpret_cast<DType*>(reinterpret_cast<char*>(head) + offset_);
  }
  std::ptrdiff_t offset_{0};
  DType default_value_{};
};

/*! \brief numeric field with optional [lower, upper] range */
template <typename TEntry, typename DType>
class FieldEntryNumeric : public FieldEntryBase<TEntry, DType> {
 public:
  inline TEntry& set_range(DType begin, DType end) {
    begin_ = begin;
    end_ = end;
    has_begin_ = has_end_ = true;
    return this->self();
  }
  inline TEntry& set_lower_bound(DType begin) {
    begin_ = begin;
    has_begin_ = true;
    return this->self();
  }
  void Check(void* head) const override {
    FieldEntryBase<TEntry, DType>::Check(head);
    DType v = this->Get(head);
    if (has_begin_ && has_end_) {
      if (v < begin_ || v > end_) {
        std::ostringstream os;
        os << "value " << v << " for Parameter " << this->key_
           << " exceed bound [" << begin_ << ',' << end_ << ']' << '\n';
        os << this->key_ << ": " << this->description_;
        throw ParamError(os.str());
      }
    } else if (has_begin_ && v < begin_) {
      std::ostringstream os;
      os << "value " << v << " for Parameter " << this->key_
         << " should be greater equal to " << begin_ << '\n';
      os << this->key_ << ": " << this->description_;
      throw ParamError(os.str());
    } else if (has_end_ && v > end_) {
      std::ostringstream os;
      os << "value " << v << " for Parameter " << this->key_
         << " should be smaller equal to " << end_ << '\n';
      os << this->key_ << ": " << this->description_;
      throw ParamError(os.str());
    }
  }

 protected:
  bool has_begin_{false}, has_end_{false};
  DType begin_{}, end_{};
};

/*! \brief generic field: numeric types get ranges, others plain parsing */
template <typename DType>
class FieldEntry
    : public std::conditional<std::is_arithmetic<DType>::value,
                              FieldEntryNumeric<FieldEntry<DType>, DType>,
                              FieldEntryBase<FieldEntry<DType>, DType>>::type {};

/*! \brief int field with optional enum names (add_enum) */
template <>
class FieldEntry<int> : public FieldEntryNumeric<FieldEntry<int>, int> {
 public:
  FieldEntry() : is_enum_(false) {}
  using Parent = FieldEntryNumeric<FieldEntry<int>, int>;
  void Set(void* head, const std::string& value) const override {
    if (is_enum_) {
      auto it = enum_map_.find(value);
      if (it == enum_map_.end()) {
        std::ostringstream os;
        os << "Invalid Input: \'" << value << "\', valid values are: ";
        PrintEnums(os);
        throw ParamError(os.str());
      }
      Parent::Set(head, std::to_string(it->second));
    } else {
      Parent::Set(head, value);
    }
  }
  ParamFieldInfo GetFieldInfo() const override {
    if (!is_enum_) return Parent::GetFieldInfo();
    ParamFieldInfo info;
    std::ostringstream os;
    info.name = key_;
    info.type = type_;
    PrintEnums(os);
    if (has_default_) {
      os << ',' << "optional, default=";
      PrintDefaultValueString(os);
    } else {
      os << ", required";
    }
    info.type_info_str = os.str();
    info.description = description_;
    return info;
  }
  inline FieldEntry<int>& add_enum(const std::string& key, int value) {
    if ((enum_map_.size() != 0 && enum_map_.count(key) != 0) ||
        enum_back_map_.count(value) != 0) {
      std::ostringstream os;
      os << "Enum " << "(" << key << ": " << value << " exisit!" << ")\n";
      os << "Enums: ";
      for (const auto& kv : enum_map_) os << "(" << kv.first << ": " << kv.second << "), ";
      LOG(FATAL) << os.str();
    }
    enum_map_[key] = value;
    enum_back_map_[value] = key;
    is_enum_ = true;
    return this->self();
  }

 protected:
  void PrintValue(std::ostream& os, int value) const override {  // NOLINT(*)
    if (is_enum_) {
      CHECK_NE(enum_back_map_.count(value), 0U) << "Value not found in enum declared";
      os << enum_back_map_.at(value);
    } else {
      os << value;
    }
  }
  inline void PrintEnums(std::ostream& os) const {  // NOLINT(*)
    os << '{';
    for (auto it = enum_map_.begin(); it != enum_map_.end(); ++it) {
      if (it != enum_map_.begin()) os << ", ";
      os << "\'" << it->first << '\'';
    }
    os << '}';
  }

 private:
  bool is_enum_;
  std::map<std::string, int> enum_map_;
  std::map<int, std::string> enum_back_map_;
};

/*! \brief optional<int> field with optional enum names; "None" = empty */
template <>
class FieldEntry<optional<int>>
    : public FieldEntryBase<FieldEntry<optional<int>>, optional<int>> {
 public:
  FieldEntry() : is_enum_(false) {}
  using Parent = FieldEntryBase<FieldEntry<optional<int>>, optional<int>>;
  void Set(void* head, const std::string& value) const override {
    if (is_enum_ && value != "None") {
      auto it = enum_map_.find(value);
      if (it == enum_map_.end()) {
        std::ostringstream os;
        os << "Invalid Input: \'" << value << "\', valid values are: ";
        PrintEnums(os);
        throw ParamError(os.str());
      }
      Parent::Set(head, std::to_string(it->second));
    } else {
      Parent::Set(head, value);
    }
  }
  ParamFieldInfo GetFieldInfo() const override {
    if (!is_enum_) return Parent::GetFieldInfo();
    ParamFieldInfo info;
    std::ostringstream os;
    info.name = key_;
    info.type = type_;
    PrintEnums(os);
    if (has_default_) {
      os << ',' << "optional, default=";
      PrintDefaultValueString(os);
    } else {
      os << ", required";
    }
    info.type_info_str = os.str();
    info.description = description_;
    return info;
  }
  inline FieldEntry<optional<int>>& add_enum(const std::string& key, int value) {
    CHECK_NE(key, "None") << "None is reserved for empty optional<int>";
    if ((enum_map_.size() != 0 && enum_map_.count(key) != 0) ||
        enum_back_map_.count(value) != 0) {
      LOG(FATAL) << "Enum (" << key << ": " << value << ") exisit!";
    }
    enum_map_[key] = value;
    enum_back_map_[value] = key;
    is_enum_ = true;
    return this->self();
  }

 protected:
  void PrintValue(std::ostream& os, optional<int> value) const override {  // NOLINT
    if (is_enum_) {
      if (!value) {
        os << "None";
      } else {
        CHECK_NE(enum_back_map_.count(*value), 0U) << "Value not found in enum declared";
        os << enum_back_map_.at(*value);
      }
    } else {
      os << value;
    }
  }
  inline void PrintEnums(std::ostream& os) const {  // NOLINT(*)
    os << "{None";
    for (const auto& kv : enum_map_) os << ", \'" << kv.first << "\'";
    os << '}';
  }

 private:
  bool is_enum_;
  std::map<std::string, int> enum_map_;
  std::map<int, std::string> enum_back_map_;
};

/*! \brief string field: the whole value is taken verbatim */
template <>
class FieldEntry<std::string>
    : public FieldEntryBase<FieldEntry<std::string>, std::string> {
 public:
  void Set(void* head, const std::string& value) const override {
    this->Get(head) = value;
  }
  void PrintDefaultValueString(std::ostream& os) const override {  // NOLINT(*)
    os << '\'' << default_value_ << '\'';
  }
};

/*! \brief bool field: true/false/1/0, case-insensitive */
template <>
class FieldEntry<bool> : public FieldEntryBase<FieldEntry<bool>, bool> {
 public:
  void Set(void* head, const std::string& value) const override {
    std::string lower_case = value;
    std::transform(lower_case.begin(), lower_case.end(), lower_case.begin(),
                   [](unsigned char c) { return std::tolower(c); });
    // trim surrounding spaces
    size_t b = lower_case.find_first_not_of(" \t");
    size_t e = lower_case.find_last_not_of(" \t");
    lower_case = (b == std::string::npos) ? "" : lower_case.substr(b, e - b + 1);
    bool& ref = this->Get(head);
    if (lower_case == "true" || lower_case == "1") {
      ref = true;
    } else if (lower_case == "false" || lower_case == "0") {
      ref = false;
    } else {
      std::ostringstream os;
      os << "Invalid Parameter format for " << key_ << " expect " << type_
         << " but value=\'" << value << '\'';
      throw ParamError(os.str());
    }
  }

 protected:
  void PrintValue(std::ostream& os, bool value) const override {  // NOLINT(*)
    os << (value ? "True" : "False");
  }
};

/*! \brief float / double parsing through std::stof / std::stod */
template <typename DType>
class FieldEntryFloat : public FieldEntryNumeric<FieldEntry<DType>, DType> {
 public:
  void Set(void* head, const std::string& value) const override {
    size_t pos = 0;
    try {
      if constexpr (std::is_same<DType, float>::value) {
        this->Get(head) = std::stof(value, &pos);
      } else {
        this->Get(head) = std::stod(value, &pos);
      }
    } catch (const std::invalid_argument&) {
      std::ostringstream os;
      os << "Invalid Parameter format for " << this->key_ << " expect "
         << this->type_ << " but value=\'" << value << '\'';
      throw ParamError(os.str());
    } catch (const std::out_of_range&) {
      std::ostringstream os;
      os << "Out of range value for " << this->key_ << ", value=\'" << value << '\'';
      throw ParamError(os.str());
    }
    for (; pos < value.size(); ++pos) {
      if (!std::isspace(static_cast<unsigned char>(value[pos]))) {
        std::ostringstream os;
        os << "Some trailing characters could not be parsed: \'"
           << value.substr(pos) << "\' for " << this->key_;
        throw ParamError(os.str());
      }
    }
  }

 protected:
  void PrintValue(std::ostream& os, DType value) const override {  // NOLINT(*)
    os << std::setprecision(std::numeric_limits<DType>::max_digits10) << value;
  }
};

template <>
class FieldEntry<float> : public FieldEntryFloat<float> {};
template <>
class FieldEntry<double> : public FieldEntryFloat<double> {};

}  // namespace parameter

template <typename ValueType>
inline ValueType GetEnv(const char* key, ValueType default_value) {
  const char* val = std::getenv(key);
  // blank or unset environment variable -> default
  if (val == nullptr || std::strlen(val) == 0) return default_value;
  ValueType ret;
  parameter::FieldEntry<ValueType> e;
  e.Init(key, &ret, ret);
  e.Set(&ret, val);
  return ret;
}

template <typename ValueType>
inline void SetEnv(const char* key, ValueType value) {
  parameter::FieldEntry<ValueType> e;
  e.Init(key, &value, value);
  ::setenv(key, e.GetStringValue(&value).c_str(), 1);
}
}  // namespace dmlc

#endif  // DMLC_PARAMETER_H_
