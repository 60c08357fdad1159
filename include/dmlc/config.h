/*!
 * \file dmlc/config.h
 * \brief `key = value` configuration files.
 *
 * Parity: reference `include/dmlc/config.h:40-182` and `src/config.cc`:
 * tokens are `[^\s=]+` or double-quoted strings (with \" escapes), `=`
 * separates key and value, `#` starts a comment (not inside quotes);
 * GetParam returns the last value of a key; iteration follows insertion order
 * and, unless multi_value is set, yields only the latest occurrence of each
 * key; ToProtoString prints `key : value` (strings quoted).  Syntax errors are
 * reported with dmlc::Error (the reference only logged them).
 */
#ifndef DMLC_CONFIG_H_
#define DMLC_CONFIG_H_

#include <iterator>
#include <map>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

namespace dmlc {

class Config {
 public:
  typedef std::pair<std::string, std::string> ConfigEntry;
  class ConfigIterator;

  explicit Config(bool multi_value = false);
  explicit Config(std::istream& is, bool multi_value = false);  // NOLINT(*)
  /*! \brief remove every entry */
  void Clear();
  /*! \brief parse and add the entries of a stream */
  void LoadFromStream(std::istream& is);  // NOLINT(*)
  /*! \brief add an entry; is_string marks a value to be quoted in proto output */
  template <class T>
  void SetParam(const std::string& key, const T& value, bool is_string = false) {
    std::ostringstream oss;
    oss << value;
    Insert(key, oss.str(), is_string);
  }
  /*! \brief last value of key (fatal if absent) */
  const std::string& GetParam(const std::string& key) const;
  /*! \brief whether the last value of key was a quoted string */
  bool IsGenuineString(const std::string& key) const;
  /*! \brief protobuf-text style dump */
  std::string ToProtoString() const;

  ConfigIterator begin() const;
  ConfigIterator end() const;

  class ConfigIterator {
   public:
    using iterator_category = std::input_iterator_tag;
    using value_type = ConfigEntry;
    using difference_type = std::ptrdiff_t;
    using pointer = const ConfigEntry*;
    using reference = ConfigEntry;
    ConfigIterator(const ConfigIterator& other) = default;
    ConfigIterator& operator++();
    ConfigIterator operator++(int);  // NOLINT(*)
    bool operator==(const ConfigIterator& rhs) const;
    bool operator!=(const ConfigIterator& rhs) const;
    ConfigEntry operator*() const;

   private:
    friend class Config;
    ConfigIterator(size_t index, const Config* config);
    void FindNextIndex();
    size_t index_;
    const Config* config_;
  };

 private:
  struct ConfigValue {
    std::vector<std::string> val;
    std::vector<size_t> insert_index;
    bool is_string{false};
  };
  void Insert(const std::string& key, const std::string& value, bool is_string);
  std::map<std::string, ConfigValue> config_map_;
  /*! \brief (key, position of that occurrence within the key's values) */
  std::vector<std::pair<std::string, size_t>> order_;
  bool multi_value_;
};

}  // namespace dmlc
#endif  // DMLC_CONFIG_H_
