/*!
 * \file dmlc/json.h
 * \brief Streaming JSON reader/writer with STL handlers and dmlc::any support.
 *
 * Parity: reference `include/dmlc/json.h` — JSONReader (:43-183) with
 * ReadString / ReadNumber / BeginObject / BeginArray / NextObjectItem /
 * NextArrayItem / line_info; JSONWriter (:188-292); JSONObjectReadHelper with
 * DeclareField / DeclareOptionalField / ReadAllFields (:310-368, unknown field
 * and missing required field are errors); handlers for numbers, strings,
 * vectors, lists, maps, pairs and classes with Save(JSONWriter*) /
 * Load(JSONReader*) (:393-525); AnyJSONManager + DMLC_JSON_ENABLE_ANY writing
 * `["TypeKey", value]` (:370-384, :530-613).
 *
 * New implementation: single constexpr-dispatch handler, no SFINAE class tree.
 */
#ifndef DMLC_JSON_H_
#define DMLC_JSON_H_

#include <cctype>
#include <cstdio>
#include <functional>
#include <istream>
#include <list>
#include <map>
#include <ostream>
#include <sstream>
#include <string>
#include <type_traits>
#include <typeindex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "./any.h"
#include "./base.h"
#include "./logging.h"
#include "./type_traits.h"

namespace dmlc {

class JSONReader;
class JSONWriter;

namespace json {
template <typename T>
struct Handler;
}  // namespace json

/*! \brief pull-style JSON reader over a std::istream */
class JSONReader {
 public:
  explicit JSONReader(std::istream* is) : is_(is) {}

  /*! \brief read a quoted string (supports \" \\ \/ \n \r \t \b \f \uXXXX<128) */
  inline void ReadString(std::string* out_str);
  /*! \brief read a number (or bool for ValueType=bool) */
  template <typename ValueType>
  inline void ReadNumber(ValueType* out_value);
  inline void BeginObject();
  inline void BeginArray();
  /*! \brief advance to the next key of the current object; false at '}' */
  inline bool NextObjectItem(std::string* out_key);
  /*! \brief advance to the next element of the current array; false at ']' */
  inline bool NextArrayItem();
  /*! \brief read any value with a registered handler */
  template <typename ValueType>
  inline void Read(ValueType* out_value);
  /*! \brief "Line N, around ^`...`" for error messages */
  inline std::string line_info() const {
    std::ostringstream os;
    os << " Line " << std::max(line_count_r_, line_count_n_)
       << ", around ^`" << last_chars_ << "`";
    return os.str();
  }
  /*! \brief peek next non-space char without consuming it */
  inline int PeekNextNonSpace() {
    int ch;
    while (true) {
      ch = is_->peek();
      if (ch == '\n') ++line_count_n_;
      if (ch == '\r') ++line_count_r_;
      if (!std::isspace(ch)) break;
      is_->get();
    }
    return ch;
  }
  /*! \brief consume and return next non-space char */
  inline int NextNonSpace() {
    int ch;
    do {
      ch = NextChar();
      if (ch == '\n') ++line_count_n_;
      if (ch == '\r') ++line_count_r_;
    } while (std::isspace(ch));
    return ch;
  }

 private:
  inline int NextChar() {
    int ch = is_->get();
    if (ch != EOF) {
      last_chars_.push_back(static_cast<char>(ch));
      if (last_chars_.size() > 32) last_chars_.erase(0, last_chars_.size() - 32);
    }
    return ch;
  }
  std::istream* is_;
  size_t line_count_r_{0};
  size_t line_count_n_{0};
  std::string last_chars_;
  /*! \brief element counters of the open scopes */
  std::vector<size_t> scope_counter_;
};

/*! \brief JSON writer with optional multi-line indentation */
class JSONWriter {
 public:
  explicit JSONWriter(std::ostream* os) : os_(os) {}
  inline void WriteNoEscape(const std::string& s) { *os_ << '\"' << s << '\"'; }
  inline void WriteString(const std::string& s);
  template <typename ValueType>
  inline void WriteNumber(const ValueType& v) {
    if constexpr (std::is_same<ValueType, bool>::value) {
      *os_ << (v ? "true" : "false");
    } else if constexpr (std::is_floating_point<ValueType>::value) {
      std::ostringstream tmp;
      tmp.precision(std::is_same<ValueType, float>::value ? 9 : 17);
      tmp << v;
      *os_ << tmp.str();
    } else {
      *os_ << v;
    }
  }
  inline void BeginArray(bool multi_line = true);
  inline void EndArray();
  inline void BeginObject(bool multi_line = true);
  inline void EndObject();
  template <typename ValueType>
  inline void WriteObjectKeyValue(const std::string& key, const ValueType& value);
  inline void WriteArraySeperator();
  template <typename ValueType>
  inline void WriteArrayItem(const ValueType& value);
  template <typename ValueType>
  inline void Write(const ValueType& value);

 private:
  inline void WriteSeperator() {
    if (scope_multi_line_.empty() || scope_multi_line_.back()) {
      *os_ << '\n' << std::string(scope_multi_line_.size() * 2, ' ');
    }
  }
  std::ostream* os_;
  std::vector<size_t> scope_counter_;
  std::vector<bool> scope_multi_line_;
};

/*! \brief declarative reader of a fixed set of object fields */
class JSONObjectReadHelper {
 public:
  template <typename T>
  inline void DeclareField(const std::string& key, T* addr) {
    DeclareFieldInternal(key, addr, false);
  }
  template <typename T>
  inline void DeclareOptionalField(const std::string& key, T* addr) {
    DeclareFieldInternal(key, addr, true);
  }
  /*! \brief read the object; unknown keys and missing required keys are fatal */
  inline void ReadAllFields(JSONReader* reader);

 private:
  template <typename T>
  inline void DeclareFieldInternal(const std::string& key, T* addr, bool optional) {
    CHECK(map_.count(key) == 0) << "Adding duplicate field " << key;
    Entry e;
    e.func = [](JSONReader* reader, void* a) { reader->Read(static_cast<T*>(a)); };
    e.addr = addr;
    e.optional = optional;
    map_[key] = e;
  }
  struct Entry {
    std::function<void(JSONReader*, void*)> func;
    void* addr;
    bool optional;
  };
  std::map<std::string, Entry> map_;
};

namespace json {

/*! \brief registry of types storable inside dmlc::any for JSON I/O */
class AnyJSONManager {
 public:
  template <typename T>
  inline AnyJSONManager& EnableType(const std::string& type_name) {
    std::type_index tp = std::type_index(typeid(T));
    if (type_name_.count(tp) != 0) {
      CHECK(type_name_.at(tp) == type_name)
          << "Type has already been registered as another typename "
          << type_name_.at(tp);
      return *this;
    }
    CHECK(type_map_.count(type_name) == 0)
        << "Type name " << type_name << " already registered in registry";
    Entry e;
    e.read = [](JSONReader* reader, any* data) {
      T v;
      reader->Read(&v);
      *data = std::move(v);
    };
    e.write = [](JSONWriter* writer, const any& data) {
      writer->Write(dmlc::get<T>(data));
    };
    type_name_[tp] = type_name;
    type_map_[type_name] = e;
    return *this;
  }
  static AnyJSONManager* Global() {
    static AnyJSONManager inst;
    return &inst;
  }
  struct Entry {
    std::function<void(JSONReader*, any*)> read;
    std::function<void(JSONWriter*, const any&)> write;
  };
  std::unordered_map<std::type_index, std::string> type_name_;
  std::unordered_map<std::string, Entry> type_map_;
};

template <typename T>
struct is_vector_like : std::false_type {};
template <typename T, typename A>
struct is_vector_like<std::vector<T, A>> : std::true_type {};
template <typename T, typename A>
struct is_vector_like<std::list<T, A>> : std::true_type {};

template <typename T>
struct is_str_map : std::false_type {};
template <typename V, typename C, typename A>
struct is_str_map<std::map<std::string, V, C, A>> : std::true_type {};
template <typename V, typename H, typename E, typename A>
struct is_str_map<std::unordered_map<std::string, V, H, E, A>> : std::true_type {};

template <typename T>
struct is_pair_t : std::false_type {};
template <typename A, typename B>
struct is_pair_t<std::pair<A, B>> : std::true_type {};

template <typename T>
struct Handler {
  inline static void Write(JSONWriter* writer, const T& value) {
    if constexpr (std::is_same<T, std::string>::value) {
      writer->WriteString(value);
    } else if constexpr (std::is_arithmetic<T>::value) {
      writer->WriteNumber(value);
    } else if constexpr (std::is_same<T, any>::value) {
      std::type_index tp(value.type());
      auto* mgr = AnyJSONManager::Global();
      CHECK(mgr->type_name_.count(tp) != 0)
          << "Type " << Demangle(value.type().name())
          << " has not been registered via DMLC_JSON_ENABLE_ANY";
      const std::string& name = mgr->type_name_.at(tp);
      writer->BeginArray(false);
      writer->WriteArrayItem(name);
      writer->WriteArraySeperator();
      mgr->type_map_.at(name).write(writer, value);
      writer->EndArray();
    } else if constexpr (is_vector_like<T>::value) {
      writer->BeginArray(std::is_class<typename T::value_type>::value);
      for (const auto& v : value) writer->WriteArrayItem(v);
      writer->EndArray();
    } else if constexpr (is_str_map<T>::value) {
      writer->BeginObject(true);
      for (const auto& kv : value) writer->WriteObjectKeyValue(kv.first, kv.second);
      writer->EndObject();
    } else if constexpr (is_pair_t<T>::value) {
      writer->BeginArray(false);
      writer->WriteArrayItem(value.first);
      writer->WriteArrayItem(value.second);
      writer->EndArray();
    } else {
      value.Save(writer);
    }
  }
  inline static void Read(JSONReader* reader, T* value) {
    if constexpr (std::is_same<T, std::string>::value) {
      reader->ReadString(value);
    } else if constexpr (std::is_arithmetic<T>::value) {
      reader->ReadNumber(value);
    } else if constexpr (std::is_same<T, any>::value) {
      std::string type_name;
      reader->BeginArray();
      CHECK(reader->NextArrayItem()) << "invalid any json format";
      reader->ReadString(&type_name);
      auto* mgr = AnyJSONManager::Global();
      auto it = mgr->type_map_.find(type_name);
      CHECK(it != mgr->type_map_.end())
          << "JSONReader: cannot find type " << type_name
          << " (register it with DMLC_JSON_ENABLE_ANY)";
      CHECK(reader->NextArrayItem()) << "invalid any json format";
      it->second.read(reader, value);
      CHECK(!reader->NextArrayItem()) << "invalid any json format";
    } else if constexpr (is_vector_like<T>::value) {
      using E = typename T::value_type;
      value->clear();
      reader->BeginArray();
      while (reader->NextArrayItem()) {
        E e;
        Handler<E>::Read(reader, &e);
        value->push_back(std::move(e));
      }
    } else if constexpr (is_str_map<T>::value) {
      using V = typename T::mapped_type;
      value->clear();
      reader->BeginObject();
      std::string key;
      while (reader->NextObjectItem(&key)) {
        V v;
        Handler<V>::Read(reader, &v);
        (*value)[key] = std::move(v);
      }
    } else if constexpr (is_pair_t<T>::value) {
      reader->BeginArray();
      CHECK(reader->NextArrayItem()) << "Expect array of length 2";
      Handler<typename T::first_type>::Read(reader, &value->first);
      CHECK(reader->NextArrayItem()) << "Expect array of length 2";
      Handler<typename T::second_type>::Read(reader, &value->second);
      CHECK(!reader->NextArrayItem()) << "Expect array of length 2";
    } else {
      value->Load(reader);
    }
  }
};
}  // namespace json

#define DMLC_JSON_ENABLE_ANY_VAR_DEF(KeyName) \
  static DMLC_ATTRIBUTE_UNUSED ::dmlc::json::AnyJSONManager& __make_AnyJSONType##_##KeyName##__

/*! \brief allow values of `Type` inside dmlc::any to be saved/loaded as JSON */
#define DMLC_JSON_ENABLE_ANY(Type, KeyName) \
  DMLC_JSON_ENABLE_ANY_VAR_DEF(KeyName) =   \
      ::dmlc::json::AnyJSONManager::Global()->EnableType<Type>(#KeyName)

// ---------------------------------------------------------------------------
// implementation
// ---------------------------------------------------------------------------
inline void JSONReader::ReadString(std::string* out_str) {
  int ch = NextNonSpace();
  CHECK_EQ(ch, '\"') << "Error at" << line_info() << ", Expect \'\"\' but get \'"
                     << static_cast<char>(ch) << '\'';
  std::string out;
  while (true) {
    ch = NextChar();
    if (ch == '\\') {
      int sch = NextChar();
      switch (sch) {
        case 'r': out.push_back('\r'); break;
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case '\\': out.push_back('\\'); break;
        case '\"': out.push_back('\"'); break;
        case '/': out.push_back('/'); break;
        case 'u': {
          unsigned code = 0;
          for (int i = 0; i < 4; ++i) {
            int h = NextChar();
            code = code * 16 + static_cast<unsigned>(
                std::isdigit(h) ? h - '0' : (std::tolower(h) - 'a' + 10));
          }
          if (code < 0x80) {
            out.push_back(static_cast<char>(code));
          } else if (code < 0x800) {
            out.push_back(static_cast<char>(0xC0 | (code >> 6)));
            out.push_back(static_cast<char>(0x80 | (code & 0x3F)));
          } else {
            out.push_back(static_cast<char>(0xE0 | (code >> 12)));
            out.push_back(static_cast<char>(0x80 | ((code >> 6) & 0x3F)));
            out.push_back(static_cast<char>(0x80 | (code & 0x3F)));
          }
          break;
        }
        default: LOG(FATAL) << "unknown string escape \\" << static_cast<char>(sch);
      }
    } else {
      if (ch == '\"') break;
      CHECK(ch != EOF && ch != '\r' && ch != '\n')
          << "Error at" << line_info() << ", string is not terminated";
      out.push_back(static_cast<char>(ch));
    }
  }
  *out_str = std::move(out);
}

template <typename ValueType>
inline void JSONReader::ReadNumber(ValueType* out_value) {
  if constexpr (std::is_same<ValueType, bool>::value) {
    int ch = NextNonSpace();
    std::string tok(1, static_cast<char>(ch));
    while (std::isalpha(is_->peek())) tok.push_back(static_cast<char>(NextChar()));
    if (tok == "true") {
      *out_value = true;
    } else if (tok == "false") {
      *out_value = false;
    } else {
      // also accept 0/1
      CHECK(tok == "1" || tok == "0") << "Error at" << line_info()
                                      << ", expect boolean, got " << tok;
      *out_value = tok == "1";
    }
  } else {
    PeekNextNonSpace();
    *is_ >> *out_value;
    CHECK(!is_->fail()) << "Error at" << line_info() << ", Expect number";
  }
}

inline void JSONReader::BeginObject() {
  int ch = NextNonSpace();
  CHECK_EQ(ch, '{') << "Error at" << line_info() << ", Expect \'{\' but get \'"
                    << static_cast<char>(ch) << '\'';
  scope_counter_.push_back(0);
}

inline void JSONReader::BeginArray() {
  int ch = NextNonSpace();
  CHECK_EQ(ch, '[') << "Error at" << line_info() << ", Expect \'[\' but get \'"
                    << static_cast<char>(ch) << '\'';
  scope_counter_.push_back(0);
}

inline bool JSONReader::NextObjectItem(std::string* out_key) {
  bool next = true;
  if (scope_counter_.back() != 0) {
    int ch = NextNonSpace();
    if (ch == EOF || ch == '}') {
      next = false;
    } else {
      CHECK_EQ(ch, ',') << "Error at" << line_info()
                        << ", JSON object expect \'}\' or \',\' but get \'"
                        << static_cast<char>(ch) << '\'';
    }
  } else {
    int ch = PeekNextNonSpace();
    if (ch == '}') {
      NextChar();
      next = false;
    }
  }
  if (!next) {
    scope_counter_.pop_back();
    return false;
  }
  scope_counter_.back() += 1;
  ReadString(out_key);
  int ch = NextNonSpace();
  CHECK_EQ(ch, ':') << "Error at" << line_info() << ", Expect \':\' but get \'"
                    << static_cast<char>(ch) << '\'';
  return true;
}

inline bool JSONReader::NextArrayItem() {
  bool next = true;
  if (scope_counter_.back() != 0) {
    int ch = NextNonSpace();
    if (ch == EOF || ch == ']') {
      next = false;
    } else {
      CHECK_EQ(ch, ',') << "Error at" << line_info()
                        << ", JSON array expect \']\' or \',\'. Get \'"
                        << static_cast<char>(ch) << "\' instead";
    }
  } else {
    int ch = PeekNextNonSpace();
    if (ch == ']') {
      NextChar();
      next = false;
    }
  }
  if (!next) {
    scope_counter_.pop_back();
    return false;
  }
  scope_counter_.back() += 1;
  return true;
}

template <typename ValueType>
inline void JSONReader::Read(ValueType* out_value) {
  json::Handler<ValueType>::Read(this, out_value);
}

inline void JSONWriter::WriteString(const std::string& s) {
  std::ostream& os = *os_;
  os << '\"';
  for (char c : s) {
    switch (c) {
      case '\r': os << "\\r"; break;
      case '\n': os << "\\n"; break;
      case '\t': os << "\\t"; break;
      case '\b': os << "\\b"; break;
      case '\f': os << "\\f"; break;
      case '\\': os << "\\\\"; break;
      case '\"': os << "\\\""; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", static_cast<unsigned>(c));
          os << buf;
        } else {
          os << c;
        }
    }
  }
  os << '\"';
}

inline void JSONWriter::BeginArray(bool multi_line) {
  *os_ << '[';
  scope_multi_line_.push_back(multi_line);
  scope_counter_.push_back(0);
}

inline void JSONWriter::EndArray() {
  CHECK_NE(scope_multi_line_.size(), 0U);
  CHECK_NE(scope_counter_.size(), 0U);
  bool newline = scope_multi_line_.back();
  size_t nelem = scope_counter_.back();
  scope_multi_line_.pop_back();
  scope_counter_.pop_back();
  if (newline && nelem != 0) WriteSeperator();
  *os_ << ']';
}

inline void JSONWriter::BeginObject(bool multi_line) {
  *os_ << '{';
  scope_multi_line_.push_back(multi_line);
  scope_counter_.push_back(0);
}

inline void JSONWriter::EndObject() {
  CHECK_NE(scope_multi_line_.size(), 0U);
  CHECK_NE(scope_counter_.size(), 0U);
  bool newline = scope_multi_line_.back();
  size_t nelem = scope_counter_.back();
  scope_multi_line_.pop_back();
  scope_counter_.pop_back();
  if (newline && nelem != 0) WriteSeperator();
  *os_ << '}';
}

template <typename ValueType>
inline void JSONWriter::WriteObjectKeyValue(const std::string& key,
                                           const ValueType& value) {
  std::ostream& os = *os_;
  if (scope_counter_.back() != 0) os << ",";
  WriteSeperator();
  WriteString(key);
  os << ": ";
  scope_counter_.back() += 1;
  json::Handler<ValueType>::Write(this, value);
}

inline void JSONWriter::WriteArraySeperator() {
  std::ostream& os = *os_;
  if (scope_counter_.back() != 0) os << ", ";
  scope_counter_.back() += 1;
  if (scope_multi_line_.back()) WriteSeperator();
}

template <typename ValueType>
inline void JSONWriter::WriteArrayItem(const ValueType& value) {
  this->WriteArraySeperator();
  json::Handler<ValueType>::Write(this, value);
}

template <typename ValueType>
inline void JSONWriter::Write(const ValueType& value) {
  size_t nscope = scope_multi_line_.size();
  json::Handler<ValueType>::Write(this, value);
  CHECK_EQ(nscope, scope_multi_line_.size()) << "Uneven scope, did you call EndArray/EndObject?";
}

inline void JSONObjectReadHelper::ReadAllFields(JSONReader* reader) {
  reader->BeginObject();
  std::map<std::string, int> visited;
  std::string key;
  while (reader->NextObjectItem(&key)) {
    auto it = map_.find(key);
    if (it != map_.end()) {
      it->second.func(reader, it->second.addr);
      visited[key] = 0;
    } else {
      std::ostringstream err;
      err << "JSONReader: Unknown field " << key << ", candidates are: \n";
      for (const auto& kv : map_) err << '\"' << kv.first << "\"\n";
      LOG(FATAL) << err.str();
    }
  }
  for (const auto& kv : map_) {
    if (!kv.second.optional) {
      CHECK(visited.count(kv.first) != 0)
          << "JSONReader: Missing field \"" << kv.first << "\"\n At "
          << reader->line_info();
    }
  }
}

}  // namespace dmlc
#endif  // DMLC_JSON_H_
