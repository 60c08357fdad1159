/*!
 * \file dmlc/registry.h
 * \brief Global name -> entry registries (parsers, GPU kernels, filesystems,
 *  user factories) with aliases and self-documentation.
 *
 * Parity: reference `include/dmlc/registry.h` — Registry<E>::List /
 * ListAllNames / Find / AddAlias / __REGISTER__ / __REGISTER_OR_GET__ / Get
 * (:27-122), FunctionRegEntryBase with set_body / describe / add_argument(s) /
 * set_return_type (:147-222), DMLC_REGISTRY_ENABLE (:230-235),
 * DMLC_REGISTRY_REGISTER (:246-248), DMLC_REGISTRY_FILE_TAG / LINK_TAG
 * (:259-304) to force static-library objects to link.
 */
#ifndef DMLC_REGISTRY_H_
#define DMLC_REGISTRY_H_

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "./base.h"
#include "./logging.h"
#include "./parameter.h"

namespace dmlc {

/*! \brief registry of entries of type EntryType, one per template instance */
template <typename EntryType>
class Registry {
 public:
  /*! \brief all registered entries in registration order */
  inline static const std::vector<const EntryType*>& List() {
    return Get()->const_list_;
  }
  /*! \brief all names, aliases included */
  inline static std::vector<std::string> ListAllNames() {
    const auto& fmap = Get()->fmap_;
    std::vector<std::string> names;
    names.reserve(fmap.size());
    for (const auto& kv : fmap) names.push_back(kv.first);
    return names;
  }
  /*! \brief entry registered under name (or alias); nullptr when absent */
  inline static const EntryType* Find(const std::string& name) {
    const auto& fmap = Get()->fmap_;
    auto p = fmap.find(name);
    return p == fmap.end() ? nullptr : p->second;
  }
  /*! \brief add `alias` for the entry `key_name` */
  inline void AddAlias(const std::string& key_name, const std::string& alias) {
    std::lock_guard<std::mutex> lock(mutex_);
    EntryType* e = fmap_.at(key_name);
    if (fmap_.count(alias)) {
      CHECK_EQ(e, fmap_.at(alias)) << "Trying to register alias " << alias
                                   << " for key " << key_name << " but "
                                   << alias << " is already taken";
    } else {
      fmap_[alias] = e;
    }
  }
  /*! \brief create a new entry; fatal if the name exists */
  inline EntryType& __REGISTER__(const std::string& name) {
    std::lock_guard<std::mutex> lock(mutex_);
    CHECK_EQ(fmap_.count(name), 0U) << name << " already registered";
    EntryType* e = new EntryType();
    e->name = name;
    fmap_[name] = e;
    const_list_.push_back(e);
    entry_list_.emplace_back(e);
    return *e;
  }
  /*! \brief get the entry, creating it if needed */
  inline EntryType& __REGISTER_OR_GET__(const std::string& name) {
    {
      std::lock_guard<std::mutex> lock(mutex_);
      auto it = fmap_.find(name);
      if (it != fmap_.end()) return *it->second;
    }
    return __REGISTER__(name);
  }
  /*! \brief the singleton (defined by DMLC_REGISTRY_ENABLE) */
  static Registry* Get();

 private:
  std::vector<std::unique_ptr<EntryType>> entry_list_;
  std::vector<const EntryType*> const_list_;
  std::map<std::string, EntryType*> fmap_;
  std::mutex mutex_;

 public:
  // constructed only through RegistrySingleton (function-local static)
  Registry() = default;
  Registry(const Registry&) = delete;
  Registry& operator=(const Registry&) = delete;
};

/*! \brief constructs the singleton (private ctor) */
template <typename EntryType>
inline Registry<EntryType>* RegistrySingleton() {
  static Registry<EntryType> inst;
  return &inst;
}

/*!
 * \brief base of function-like registry entries
 * \tparam EntryType the derived entry (CRTP)
 * \tparam FunctionType the std::function type of the body
 */
template <typename EntryType, typename FunctionType>
class FunctionRegEntryBase {
 public:
  std::string name;
  std::string description;
  std::vector<ParamFieldInfo> arguments;
  FunctionType body;
  std::string return_type;

  inline EntryType& set_body(FunctionType body) {
    this->body = body;
    return this->self();
  }
  inline EntryType& describe(const std::string& description) {
    this->description = description;
    return this->self();
  }
  inline EntryType& add_argument(const std::string& name, const std::string& type,
                                 const std::string& description) {
    ParamFieldInfo info;
    info.name = name;
    info.type = type;
    info.type_info_str = info.type;
    info.description = description;
    arguments.push_back(info);
    return this->self();
  }
  inline EntryType& add_arguments(const std::vector<ParamFieldInfo>& args) {
    arguments.insert(arguments.end(), args.begin(), args.end());
    return this->self();
  }
  inline EntryType& set_return_type(const std::string& type) {
    return_type = type;
    return this->self();
  }

 protected:
  inline EntryType& self() { return *(static_cast<EntryType*>(this)); }
};

/*! \brief define Registry<EntryType>::Get (one .cc file per entry type) */
#define DMLC_REGISTRY_ENABLE(EntryType)                     \
  template <>                                               \
  ::dmlc::Registry<EntryType>* ::dmlc::Registry<EntryType>::Get() { \
    return ::dmlc::RegistrySingleton<EntryType>();          \
  }

/*! \brief register a new entry into the registry */
#define DMLC_REGISTRY_REGISTER(EntryType, EntryTypeName, Name)                \
  static DMLC_ATTRIBUTE_UNUSED EntryType& __make_##EntryTypeName##_##Name##__ = \
      ::dmlc::Registry<EntryType>::Get()->__REGISTER__(#Name)

/*! \brief mark a file so that DMLC_REGISTRY_LINK_TAG can force-link it */
#define DMLC_REGISTRY_FILE_TAG(UniqueTag) \
  int __dmlc_registry_file_tag_##UniqueTag##__() { return 0; }

/*! \brief reference a tagged file so the static linker keeps its registrations */
#define DMLC_REGISTRY_LINK_TAG(UniqueTag)                                 \
  int __dmlc_registry_file_tag_##UniqueTag##__();                         \
  static int DMLC_ATTRIBUTE_UNUSED __reg_file_tag_##UniqueTag##__ =       \
      __dmlc_registry_file_tag_##UniqueTag##__();

}  // namespace dmlc
#endif  // DMLC_REGISTRY_H_
