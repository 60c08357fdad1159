/*!
 * \file src/config.cc
 * \brief Config file tokenizer and store (see dmlc/config.h).
 */
#include <dmlc/config.h>
#include <dmlc/logging.h>

#include <cctype>
#include <istream>

namespace dmlc {

namespace {
enum class TokType { kString, kQuoted, kEqual, kNewline, kEnd };
struct Token {
  TokType type;
  std::string text;
};

/*! \brief streaming tokenizer: words, quoted strings, '=', newlines; '#' comments */
class Tokenizer {
 public:
  explicit Tokenizer(std::istream* is) : is_(is) {}
  Token Next() {
    while (true) {
      int c = is_->peek();
      if (c == EOF) return Token{TokType::kEnd, ""};
      if (c == '\n') {
        is_->get();
        ++line_;
        return Token{TokType::kNewline, ""};
      }
      if (std::isspace(c)) {
        is_->get();
        continue;
      }
      if (c == '#') {
        while (is_->peek() != EOF && is_->peek() != '\n') is_->get();
        continue;
      }
      if (c == '=') {
        is_->get();
        return Token{TokType::kEqual, "="};
      }
      if (c == '"') {
        is_->get();
        std::string s;
        while (true) {
          int d = is_->get();
          if (d == EOF || d == '\n') {
            throw Error("config line " + std::to_string(line_) + ": unterminated string");
          }
          if (d == '\\' && is_->peek() == '"') {
            s.push_back(static_cast<char>(is_->get()));
            continue;
          }
          if (d == '"') break;
          s.push_back(static_cast<char>(d));
        }
        return Token{TokType::kQuoted, s};
      }
      std::string s;
      while (is_->peek() != EOF) {
        int d = is_->peek();
        if (std::isspace(d) || d == '=' || d == '#' || d == '"') break;
        s.push_back(static_cast<char>(is_->get()));
      }
      return Token{TokType::kString, s};
    }
  }
  size_t line() const { return line_; }

 private:
  std::istream* is_;
  size_t line_{1};
};
}  // namespace

Config::Config(bool multi_value) : multi_value_(multi_value) { Clear(); }

Config::Config(std::istream& is, bool multi_value) : multi_value_(multi_value) {
  Clear();
  LoadFromStream(is);
}

void Config::Clear() {
  config_map_.clear();
  order_.clear();
}

void Config::LoadFromStream(std::istream& is) {
  Tokenizer tok(&is);
  while (true) {
    Token key = tok.Next();
    if (key.type == TokType::kEnd) break;
    if (key.type == TokType::kNewline) continue;
    if (key.type != TokType::kString && key.type != TokType::kQuoted) {
      throw Error("config line " + std::to_string(tok.line()) + ": expected a key");
    }
    Token eq = tok.Next();
    if (eq.type != TokType::kEqual) {
      throw Error("config line " + std::to_string(tok.line()) + ": expected '=' after key " +
                  key.text);
    }
    Token val = tok.Next();
    if (val.type != TokType::kString && val.type != TokType::kQuoted) {
      throw Error("config line " + std::to_string(tok.line()) + ": expected a value for key " +
                  key.text);
    }
    Insert(key.text, val.text, val.type == TokType::kQuoted);
  }
}

void Config::Insert(const std::string& key, const std::string& value, bool is_string) {
  ConfigValue& cv = config_map_[key];
  cv.val.push_back(value);
  cv.is_string = is_string;
  cv.insert_index.push_back(order_.size());
  order_.emplace_back(key, cv.val.size() - 1);
}

const std::string& Config::GetParam(const std::string& key) const {
  auto it = config_map_.find(key);
  CHECK(it != config_map_.end()) << "key \"" << key << "\" not found in configure";
  return it->second.val.back();
}

bool Config::IsGenuineString(const std::string& key) const {
  auto it = config_map_.find(key);
  CHECK(it != config_map_.end()) << "key \"" << key << "\" not found in configure";
  return it->second.is_string;
}

std::string Config::ToProtoString() const {
  std::ostringstream os;
  for (const ConfigEntry& e : *this) {
    os << e.first << " : ";
    if (config_map_.at(e.first).is_string) {
      os << '"';
      for (char c : e.second) {
        if (c == '"') os << '\\';
        os << c;
      }
      os << '"';
    } else {
      os << e.second;
    }
    os << '\n';
  }
  return os.str();
}

Config::ConfigIterator Config::begin() const { return ConfigIterator(0, this); }
Config::ConfigIterator Config::end() const { return ConfigIterator(order_.size(), this); }

Config::ConfigIterator::ConfigIterator(size_t index, const Config* config)
    : index_(index), config_(config) {
  FindNextIndex();
}

void Config::ConfigIterator::FindNextIndex() {
  // without multi_value only the latest occurrence of a key is visited
  while (index_ < config_->order_.size()) {
    if (config_->multi_value_) return;
    const auto& ent = config_->order_[index_];
    const auto& cv = config_->config_map_.at(ent.first);
    if (ent.second + 1 == cv.val.size()) return;
    ++index_;
  }
}

Config::ConfigIterator& Config::ConfigIterator::operator++() {
  ++index_;
  FindNextIndex();
  return *this;
}

Config::ConfigIterator Config::ConfigIterator::operator++(int) {
  ConfigIterator tmp(*this);
  ++(*this);
  return tmp;
}

bool Config::ConfigIterator::operator==(const ConfigIterator& rhs) const {
  return index_ == rhs.index_ && config_ == rhs.config_;
}
bool Config::ConfigIterator::operator!=(const ConfigIterator& rhs) const {
  return !(*this == rhs);
}

Config::ConfigEntry Config::ConfigIterator::operator*() const {
  const auto& ent = config_->order_[index_];
  return ConfigEntry(ent.first, config_->config_map_.at(ent.first).val[ent.second]);
}

}  // namespace dmlc
