/*!
 * \file dmlc/json.h
 * \brief Streaming JSON reader / writer with STL handlers and dmlc::any.
 *
 * Public surface kept from the reference (`include/dmlc/json.h`): JSONReader
 * {ReadString, ReadNumber, BeginObject, BeginArray, NextObjectItem,
 * NextArrayItem, Read, line_info}, JSONWriter {WriteNoEscape, WriteString,
 * WriteNumber, BeginArray, EndArray, BeginObject, EndObject,
 * WriteObjectKeyValue, WriteArraySeperator (sic), WriteArrayItem, Write},
 * JSONObjectReadHelper {DeclareField, DeclareOptionalField, ReadAllFields:
 * an unknown key or a missing required key is an error}, and
 * DMLC_JSON_ENABLE_ANY(Type, Key) which stores an `any` as `["Key", value]`.
 *
 * Layout written: objects put each member on its own line,
 * indented two spaces per open scope; arrays of class-typed elements do the
 * same, arrays of scalars / strings stay on one line ("[1, 2, 3]"); pairs and
 * `any` are one-line two-element arrays.
 *
 * Implementation (new): the reader keeps a stack of open scopes and advances
 * arrays and objects through one routine (`Advance`); the writer keeps a
 * stack of frames {multi-line, members written}; values dispatch through one
 * `json::Handler<T>` with `if constexpr`.
 */
#ifndef DMLC_JSON_H_
#define DMLC_JSON_H_

#include <cctype>
#include <cstdio>
#include <functional>
#include <istream>
#include <limits>
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

/*! \brief pull parser over a std::istream */
class JSONReader {
 public:
  explicit JSONReader(std::istream* is) : in_(is) {}

  /*! \brief a quoted string; escapes \" \\ \/ \b \f \n \r \t and \uXXXX (BMP, as UTF-8) */
  inline void ReadString(std::string* out);
  /*! \brief a number (true / false / 1 / 0 for bool) */
  template <typename ValueType>
  inline void ReadNumber(ValueType* out);
  inline void BeginObject() { Open('{', '}'); }
  inline void BeginArray() { Open('[', ']'); }
  /*! \brief move to the next member of the innermost object; false once it closed */
  inline bool NextObjectItem(std::string* out_key);
  /*! \brief move to the next element of the innermost array; false once it closed */
  inline bool NextArrayItem() { return Advance(']'); }
  /*! \brief any value with a json::Handler */
  template <typename ValueType>
  inline void Read(ValueType* out);
  /*! \brief where the reader is, for error messages */
  inline std::string line_info() const {
    std::ostringstream os;
    os << " (line " << line_ + 1 << ", after \"" << recent_ << "\")";
    return os.str();
  }
  /*! \brief next non-blank character, not consumed */
  inline int PeekNextNonSpace() {
    SkipBlanks();
    return in_->peek();
  }
  /*! \brief next non-blank character, consumed */
  inline int NextNonSpace() {
    SkipBlanks();
    return Take();
  }

 private:
  struct Scope {
    char close;
    size_t items;
  };
  inline int Take() {
    const int c = in_->get();
    if (c == EOF) return c;
    if (c == '\n') ++line_;
    recent_.push_back(static_cast<char>(c));
    if (recent_.size() > 24) recent_.erase(0, recent_.size() - 24);
    return c;
  }
  inline void SkipBlanks() {
    while (std::isspace(in_->peek())) Take();
  }
  inline void Expect(int got, char want) {
    if (got != want) {
      LOG(FATAL) << "JSON: wanted '" << want << "' but read "
                 << (got == EOF ? std::string("end of input")
                                : std::string("'") + static_cast<char>(got) + "'")
                 << line_info();
    }
  }
  inline void Open(char open, char close) {
    Expect(NextNonSpace(), open);
    scopes_.push_back(Scope{close, 0});
  }
  /*!
   * \brief shared step of NextArrayItem / NextObjectItem: consume the closing
   *  bracket (scope done) or, after the first item, the separating comma
   */
  inline bool Advance(char close) {
    CHECK(!scopes_.empty() && scopes_.back().close == close)
        << "JSON: no open '" << (close == ']' ? '[' : '{') << "' to iterate" << line_info();
    Scope& sc = scopes_.back();
    const int c = PeekNextNonSpace();
    if (c == close || c == EOF) {
      Take();
      scopes_.pop_back();
      return false;
    }
    if (sc.items != 0) Expect(Take(), ',');
    ++sc.items;
    return true;
  }
  inline unsigned HexDigit() {
    const int h = Take();
    if (h >= '0' && h <= '9') return static_cast<unsigned>(h - '0');
    if (h >= 'a' && h <= 'f') return static_cast<unsigned>(h - 'a' + 10);
    if (h >= 'A' && h <= 'F') return static_cast<unsigned>(h - 'A' + 10);
    LOG(FATAL) << "JSON: bad \\u escape digit" << line_info();
    return 0;
  }
  static inline void AppendUtf8(unsigned cp, std::string* s) {
    if (cp < 0x80) {
      s->push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      s->push_back(static_cast<char>(0xC0 | (cp >> 6)));
      s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      s->push_back(static_cast<char>(0xE0 | (cp >> 12)));
      s->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      s->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }

  std::istream* in_;
  size_t line_{0};
  std::string recent_;
  std::vector<Scope> scopes_;
};

/*! \brief writer producing the layout described in the file comment */
class JSONWriter {
 public:
  explicit JSONWriter(std::ostream* os) : out_(os) {}
  inline void WriteNoEscape(const std::string& s) { *out_ << '"' << s << '"'; }
  inline void WriteString(const std::string& s);
  template <typename ValueType>
  inline void WriteNumber(const ValueType& v) {
    if constexpr (std::is_same<ValueType, bool>::value) {
      *out_ << (v ? "true" : "false");
    } else if constexpr (std::is_floating_point<ValueType>::value) {
      // enough digits to read the same value back
      std::ostringstream num;
      num.precision(std::numeric_limits<ValueType>::max_digits10);
      num << v;
      *out_ << num.str();
    } else {
      *out_ << v;
    }
  }
  inline void BeginArray(bool multi_line = true) { Push('[', multi_line); }
  inline void EndArray() { Pop(']'); }
  inline void BeginObject(bool multi_line = true) { Push('{', multi_line); }
  inline void EndObject() { Pop('}'); }
  template <typename ValueType>
  inline void WriteObjectKeyValue(const std::string& key, const ValueType& value);
  /*! \brief the separator before the next array element (name kept from the reference API) */
  inline void WriteArraySeperator();
  template <typename ValueType>
  inline void WriteArrayItem(const ValueType& value) {
    WriteArraySeperator();
    json::Handler<ValueType>::Write(this, value);
  }
  template <typename ValueType>
  inline void Write(const ValueType& value);

 private:
  struct Frame {
    char close;
    bool multi_line;
    size_t written;
  };
  inline void NewLine() {
    *out_ << '\n';
    for (size_t i = 0; i < frames_.size(); ++i) *out_ << "  ";
  }
  inline void Push(char open, bool multi_line) {
    *out_ << open;
    frames_.push_back(Frame{open == '[' ? ']' : '}', multi_line, 0});
  }
  inline void Pop(char close) {
    CHECK(!frames_.empty() && frames_.back().close == close)
        << "JSONWriter: '" << close << "' does not close the innermost scope";
    const Frame f = frames_.back();
    frames_.pop_back();
    if (f.multi_line && f.written != 0) NewLine();
    *out_ << close;
  }
  std::ostream* out_;
  std::vector<Frame> frames_;
};

/*! \brief reads one object into declared fields */
class JSONObjectReadHelper {
 public:
  template <typename T>
  inline void DeclareField(const std::string& key, T* addr) {
    Declare(key, addr, true);
  }
  template <typename T>
  inline void DeclareOptionalField(const std::string& key, T* addr) {
    Declare(key, addr, false);
  }
  /*! \brief read the object; an undeclared key or a missing required key is fatal */
  inline void ReadAllFields(JSONReader* reader);

 private:
  struct Slot {
    std::function<void(JSONReader*)> read;
    bool required;
  };
  template <typename T>
  inline void Declare(const std::string& key, T* addr, bool required) {
    CHECK(slots_.find(key) == slots_.end()) << "JSONObjectReadHelper: '" << key
                                            << "' declared twice";
    slots_[key] = Slot{[addr](JSONReader* r) { r->Read(addr); }, required};
  }
  std::map<std::string, Slot> slots_;
};

namespace json {

/*! \brief types allowed inside dmlc::any for JSON I/O, by key name */
class AnyJSONManager {
 public:
  struct Entry {
    std::function<void(JSONReader*, any*)> read;
    std::function<void(JSONWriter*, const any&)> write;
  };
  template <typename T>
  inline AnyJSONManager& EnableType(const std::string& key) {
    const std::type_index tid(typeid(T));
    auto known = key_of_.find(tid);
    if (known != key_of_.end()) {
      CHECK_EQ(known->second, key) << "type already enabled for JSON as " << known->second;
      return *this;
    }
    CHECK(by_key_.count(key) == 0) << "JSON any key " << key << " is taken by another type";
    key_of_[tid] = key;
    by_key_[key] = Entry{[](JSONReader* r, any* dst) {
                           T v;
                           r->Read(&v);
                           *dst = std::move(v);
                         },
                         [](JSONWriter* w, const any& src) { w->Write(dmlc::get<T>(src)); }};
    return *this;
  }
  static AnyJSONManager* Global() {
    static AnyJSONManager registry;
    return &registry;
  }
  /*! \brief key of a stored type; fatal if it was never enabled */
  const std::string& KeyOf(const std::type_info& t) const {
    auto hit = key_of_.find(std::type_index(t));
    CHECK(hit != key_of_.end()) << "type " << Demangle(t.name())
                                << " is not enabled for JSON (DMLC_JSON_ENABLE_ANY)";
    return hit->second;
  }
  const Entry& ByKey(const std::string& key) const {
    auto hit = by_key_.find(key);
    CHECK(hit != by_key_.end()) << "JSON any key " << key
                                << " is not enabled (DMLC_JSON_ENABLE_ANY)";
    return hit->second;
  }

 private:
  std::unordered_map<std::type_index, std::string> key_of_;
  std::unordered_map<std::string, Entry> by_key_;
};

template <typename T>
struct IsSequence : std::false_type {};
template <typename T, typename A>
struct IsSequence<std::vector<T, A>> : std::true_type {};
template <typename T, typename A>
struct IsSequence<std::list<T, A>> : std::true_type {};

template <typename T>
struct IsStringKeyed : std::false_type {};
template <typename V, typename C, typename A>
struct IsStringKeyed<std::map<std::string, V, C, A>> : std::true_type {};
template <typename V, typename H, typename E, typename A>
struct IsStringKeyed<std::unordered_map<std::string, V, H, E, A>> : std::true_type {};

template <typename T>
struct IsPair : std::false_type {};
template <typename A, typename B>
struct IsPair<std::pair<A, B>> : std::true_type {};

/*! \brief read one element of a two-element array (pair, any) */
template <typename E>
inline void ReadSlot(JSONReader* r, E* dst, const char* what) {
  CHECK(r->NextArrayItem()) << "JSON: " << what << " needs two elements" << r->line_info();
  r->Read(dst);
}

template <typename T>
struct Handler {
  static void Write(JSONWriter* w, const T& v) {
    if constexpr (std::is_same<T, std::string>::value) {
      w->WriteString(v);
    } else if constexpr (std::is_arithmetic<T>::value) {
      w->WriteNumber(v);
    } else if constexpr (std::is_same<T, any>::value) {
      AnyJSONManager* reg = AnyJSONManager::Global();
      const std::string& key = reg->KeyOf(v.type());
      w->BeginArray(false);
      w->WriteArrayItem(key);
      w->WriteArraySeperator();
      reg->ByKey(key).write(w, v);
      w->EndArray();
    } else if constexpr (IsSequence<T>::value) {
      w->BeginArray(std::is_class<typename T::value_type>::value);
      for (const auto& e : v) w->WriteArrayItem(e);
      w->EndArray();
    } else if constexpr (IsStringKeyed<T>::value) {
      w->BeginObject(true);
      for (const auto& kv : v) w->WriteObjectKeyValue(kv.first, kv.second);
      w->EndObject();
    } else if constexpr (IsPair<T>::value) {
      w->BeginArray(false);
      w->WriteArrayItem(v.first);
      w->WriteArrayItem(v.second);
      w->EndArray();
    } else {
      v.Save(w);
    }
  }
  static void Read(JSONReader* r, T* v) {
    if constexpr (std::is_same<T, std::string>::value) {
      r->ReadString(v);
    } else if constexpr (std::is_arithmetic<T>::value) {
      r->ReadNumber(v);
    } else if constexpr (std::is_same<T, any>::value) {
      r->BeginArray();
      std::string key;
      ReadSlot(r, &key, "an any value");
      CHECK(r->NextArrayItem()) << "JSON: an any value needs two elements" << r->line_info();
      AnyJSONManager::Global()->ByKey(key).read(r, v);
      CHECK(!r->NextArrayItem()) << "JSON: an any value has exactly two elements"
                                 << r->line_info();
    } else if constexpr (IsSequence<T>::value) {
      T out;
      r->BeginArray();
      while (r->NextArrayItem()) {
        typename T::value_type e;
        r->Read(&e);
        out.push_back(std::move(e));
      }
      *v = std::move(out);
    } else if constexpr (IsStringKeyed<T>::value) {
      T out;
      r->BeginObject();
      std::string key;
      while (r->NextObjectItem(&key)) {
        typename T::mapped_type e;
        r->Read(&e);
        out[key] = std::move(e);
      }
      *v = std::move(out);
    } else if constexpr (IsPair<T>::value) {
      r->BeginArray();
      ReadSlot(r, &v->first, "a pair");
      ReadSlot(r, &v->second, "a pair");
      CHECK(!r->NextArrayItem()) << "JSON: a pair has exactly two elements" << r->line_info();
    } else {
      v->Load(r);
    }
  }
};
}  // namespace json

#define DMLC_JSON_ENABLE_ANY_VAR_DEF(KeyName) \
  static DMLC_ATTRIBUTE_UNUSED ::dmlc::json::AnyJSONManager& __make_AnyJSONType##_##KeyName##__

/*! \brief let dmlc::any values of `Type` be written / read as ["KeyName", value] */
#define DMLC_JSON_ENABLE_ANY(Type, KeyName) \
  DMLC_JSON_ENABLE_ANY_VAR_DEF(KeyName) =   \
      ::dmlc::json::AnyJSONManager::Global()->EnableType<Type>(#KeyName)

// ------------------------------------------------------------------ reader
inline void JSONReader::ReadString(std::string* out) {
  Expect(NextNonSpace(), '"');
  std::string s;
  for (;;) {
    const int c = Take();
    if (c == '"') break;
    CHECK(c != EOF && c != '\n' && c != '\r') << "JSON: unterminated string" << line_info();
    if (c != '\\') {
      s.push_back(static_cast<char>(c));
      continue;
    }
    const int e = Take();
    switch (e) {
      case '"':
      case '\\':
      case '/':
        s.push_back(static_cast<char>(e));
        break;
      case 'b': s.push_back('\b'); break;
      case 'f': s.push_back('\f'); break;
      case 'n': s.push_back('\n'); break;
      case 'r': s.push_back('\r'); break;
      case 't': s.push_back('\t'); break;
      case 'u': {
        unsigned cp = 0;
        for (int i = 0; i < 4; ++i) cp = (cp << 4) | HexDigit();
        AppendUtf8(cp, &s);
        break;
      }
      default:
        LOG(FATAL) << "JSON: unknown escape \\" << static_cast<char>(e) << line_info();
    }
  }
  *out = std::move(s);
}

template <typename ValueType>
inline void JSONReader::ReadNumber(ValueType* out) {
  if constexpr (std::is_same<ValueType, bool>::value) {
    std::string word;
    word.push_back(static_cast<char>(NextNonSpace()));
    while (std::isalnum(in_->peek())) word.push_back(static_cast<char>(Take()));
    if (word == "true" || word == "1") {
      *out = true;
    } else if (word == "false" || word == "0") {
      *out = false;
    } else {
      LOG(FATAL) << "JSON: '" << word << "' is not a boolean" << line_info();
    }
  } else {
    SkipBlanks();
    *in_ >> *out;
    CHECK(!in_->fail()) << "JSON: expected a number" << line_info();
  }
}

inline bool JSONReader::NextObjectItem(std::string* out_key) {
  if (!Advance('}')) return false;
  ReadString(out_key);
  Expect(NextNonSpace(), ':');
  return true;
}

template <typename ValueType>
inline void JSONReader::Read(ValueType* out) {
  json::Handler<ValueType>::Read(this, out);
}

// ------------------------------------------------------------------ writer
inline void JSONWriter::WriteString(const std::string& s) {
  std::ostream& os = *out_;
  os << '"';
  for (const char c : s) {
    const unsigned char u = static_cast<unsigned char>(c);
    if (c == '"' || c == '\\') {
      os << '\\' << c;
    } else if (c == '\n') {
      os << "\\n";
    } else if (c == '\r') {
      os << "\\r";
    } else if (c == '\t') {
      os << "\\t";
    } else if (c == '\b') {
      os << "\\b";
    } else if (c == '\f') {
      os << "\\f";
    } else if (u < 0x20) {
      char hex[8];
      std::snprintf(hex, sizeof(hex), "\\u%04x", u);
      os << hex;
    } else {
      os << c;
    }
  }
  os << '"';
}

inline void JSONWriter::WriteArraySeperator() {
  CHECK(!frames_.empty()) << "JSONWriter: array element outside an array";
  Frame& f = frames_.back();
  if (f.written++ != 0) *out_ << ", ";
  if (f.multi_line) NewLine();
}

template <typename ValueType>
inline void JSONWriter::WriteObjectKeyValue(const std::string& key, const ValueType& value) {
  CHECK(!frames_.empty()) << "JSONWriter: object member outside an object";
  Frame& f = frames_.back();
  if (f.written++ != 0) *out_ << ',';
  if (f.multi_line) NewLine();
  WriteString(key);
  *out_ << ": ";
  json::Handler<ValueType>::Write(this, value);
}

template <typename ValueType>
inline void JSONWriter::Write(const ValueType& value) {
  const size_t depth = frames_.size();
  json::Handler<ValueType>::Write(this, value);
  CHECK_EQ(depth, frames_.size()) << "JSONWriter: a Begin* without its End*";
}

inline void JSONObjectReadHelper::ReadAllFields(JSONReader* reader) {
  std::map<std::string, bool> seen;
  reader->BeginObject();
  std::string key;
  while (reader->NextObjectItem(&key)) {
    auto slot = slots_.find(key);
    if (slot == slots_.end()) {
      std::ostringstream known;
      for (const auto& kv : slots_) known << " \"" << kv.first << '"';
      LOG(FATAL) << "JSON: unexpected member \"" << key << "\"; expected one of" << known.str()
                 << reader->line_info();
    }
    slot->second.read(reader);
    seen[key] = true;
  }
  for (const auto& kv : slots_) {
    CHECK(!kv.second.required || seen.count(kv.first) != 0)
        << "JSON: required member \"" << kv.first << "\" is missing" << reader->line_info();
  }
}

}  // namespace dmlc
#endif  // DMLC_JSON_H_
