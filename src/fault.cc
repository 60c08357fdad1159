/*!
 * \file src/fault.cc
 * \brief DMLC_FAULT_INJECT parsing and per-point pass counters.
 */
#include <dmlc/fault.h>

#include <cstdlib>
#include <map>
#include <mutex>

namespace dmlc {
namespace fault {
namespace {

struct State {
  std::mutex mu;
  std::map<std::string, long> fire_at;  // point -> pass number that fails
  std::map<std::string, long> count;
  std::atomic<bool> enabled{false};

  State() {
    const char* env = std::getenv("DMLC_FAULT_INJECT");
    if (env != nullptr) Parse(env);
  }
  void Parse(const std::string& spec) {
    fire_at.clear();
    count.clear();
    size_t b = 0;
    while (b < spec.size()) {
      size_t e = spec.find(',', b);
      if (e == std::string::npos) e = spec.size();
      const std::string item = spec.substr(b, e - b);
      b = e + 1;
      if (item.empty()) continue;
      const size_t c = item.find(':');
      const std::string point = item.substr(0, c);
      const long at = c == std::string::npos ? 1 : std::atol(item.c_str() + c + 1);
      CHECK_GT(at, 0) << "DMLC_FAULT_INJECT: bad count in \"" << item << "\"";
      fire_at[point] = at;
    }
    enabled.store(!fire_at.empty(), std::memory_order_relaxed);
  }
};

State& S() {
  static State* s = new State();
  return *s;
}

}  // namespace

bool Enabled() { return S().enabled.load(std::memory_order_relaxed); }

bool Hit(const char* point) {
  State& s = S();
  std::lock_guard<std::mutex> lock(s.mu);
  const long n = ++s.count[point];
  auto it = s.fire_at.find(point);
  return it != s.fire_at.end() && it->second == n;
}

void Configure(const std::string& spec) {
  State& s = S();
  std::lock_guard<std::mutex> lock(s.mu);
  s.Parse(spec);
}

long Count(const std::string& point) {
  State& s = S();
  std::lock_guard<std::mutex> lock(s.mu);
  auto it = s.count.find(point);
  return it == s.count.end() ? 0 : it->second;
}

}  // namespace fault
}  // namespace dmlc
