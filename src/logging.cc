/*!
 * \file src/logging.cc
 * \brief Stack traces, demangling, rank prefix and verbosity for logging.h.
 * Parity: reference `include/dmlc/logging.h:297-339` (Demangle / StackTrace
 * via backtrace + abi::__cxa_demangle).
 */
#include <cxxabi.h>
#include <dmlc/logging.h>
#include <execinfo.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>

namespace dmlc {

std::string Demangle(const char* msg_str) {
  int status = 0;
  std::unique_ptr<char, void (*)(void*)> demangled(
      abi::__cxa_demangle(msg_str, nullptr, nullptr, &status), std::free);
  if (status == 0 && demangled) return std::string(demangled.get());
  return std::string(msg_str);
}

namespace {
/*! \brief "module(mangled+0x12) [0x...]" -> demangled symbol when possible */
std::string DemangleFrame(const std::string& frame) {
  const size_t open = frame.find('(');
  const size_t plus = frame.find('+', open == std::string::npos ? 0 : open);
  if (open == std::string::npos || plus == std::string::npos || plus <= open + 1) return frame;
  const std::string sym = frame.substr(open + 1, plus - open - 1);
  return frame.substr(0, open + 1) + Demangle(sym.c_str()) + frame.substr(plus);
}
}  // namespace

std::string StackTrace(size_t skip, size_t max_depth) {
  std::ostringstream os;
  std::unique_ptr<void*[]> stack(new void*[max_depth + skip + 1]);
  const int nframes = backtrace(stack.get(), static_cast<int>(max_depth + skip + 1));
  char** msgs = backtrace_symbols(stack.get(), nframes);
  if (msgs == nullptr) return "";
  for (int i = static_cast<int>(skip) + 1; i < nframes; ++i) {
    os << "  [bt] (" << (i - static_cast<int>(skip) - 1) << ") " << DemangleFrame(msgs[i])
       << "\n";
  }
  std::free(msgs);
  return os.str();
}

namespace log_detail {
const char* RankPrefix() {
  static const std::string prefix = []() {
    const char* r = std::getenv("DMLC_RANK");
    if (r == nullptr || *r == '\0') r = std::getenv("RANK");
    if (r == nullptr || *r == '\0') return std::string();
    return std::string("[rank ") + r + "] ";
  }();
  return prefix.c_str();
}

int VerboseLevel() {
  static const int level = []() {
    const char* v = std::getenv("DMLC_VLOG_LEVEL");
    return (v == nullptr || *v == '\0') ? 0 : std::atoi(v);
  }();
  return level;
}
}  // namespace log_detail
}  // namespace dmlc
