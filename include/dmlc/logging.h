/*!
 * \file dmlc/logging.h
 * \brief CHECK / LOG macros, dmlc::Error and stack traces.
 *
 * Parity: reference `include/dmlc/logging.h` — dmlc::Error (:31), CHECK_xx
 * (:70-130), CHECK_NOTNULL (:131), DCHECK (:134-157), LOG(sev) (:172),
 * LOG_IF (:174), DateLogger (:195), LogMessageFatal throwing from its
 * destructor (:379-405), CustomLogMessage hook (:253-272), stack traces
 * (:297-339).
 *
 * Divergences: VLOG(n) honours the DMLC_VLOG_LEVEL env var
 * and LOG_EVERY_N really logs every N-th call (the reference logs always).
 * New: every line carries a `[rank r]` prefix when DMLC_RANK / RANK is set, so
 * the 8 per-GPU processes of one job can be told apart in a merged log.
 */
#ifndef DMLC_LOGGING_H_
#define DMLC_LOGGING_H_

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>

#include "./base.h"

namespace dmlc {

/*! \brief exception thrown by LOG(FATAL) and failed CHECKs */
struct Error : public std::runtime_error {
  explicit Error(const std::string& s) : std::runtime_error(s) {}
};

/*! \brief demangled stack trace of the calling thread (skips `skip` frames) */
std::string StackTrace(size_t skip = 1,
                       size_t max_depth = DMLC_LOG_STACK_TRACE_SIZE);
/*! \brief demangle a C++ symbol name; returns the input when it is not mangled */
std::string Demangle(const char* name);

/*! \brief glog compatibility: no-op initialisation */
inline void InitLogging(const char* /*argv0*/) {}

namespace log_detail {
/*! \brief "[rank r] " prefix from DMLC_RANK / RANK, computed once */
const char* RankPrefix();
/*! \brief verbosity threshold from DMLC_VLOG_LEVEL (default 0) */
int VerboseLevel();
}  // namespace log_detail

/*! \brief wall-clock "HH:MM:SS" stamp for log lines */
class DateLogger {
 public:
  const char* HumanDate() {
    std::time_t t = std::time(nullptr);
    struct tm now;
    localtime_r(&t, &now);
    std::snprintf(buf_, sizeof(buf_), "%02d:%02d:%02d", now.tm_hour, now.tm_min,
                  now.tm_sec);
    return buf_;
  }

 private:
  char buf_[16];
};

#if DMLC_LOG_CUSTOMIZE
/*! \brief user hook: define CustomLogMessage::Log in one translation unit */
class CustomLogMessage {
 public:
  CustomLogMessage(const char* file, int line) {
    log_stream_ << "[" << DateLogger().HumanDate() << "] " << file << ":"
                << line << ": ";
  }
  ~CustomLogMessage() { Log(log_stream_.str()); }
  std::ostream& stream() { return log_stream_; }
  static void Log(const std::string& msg);

 private:
  std::ostringstream log_stream_;
};
#endif

/*! \brief one non-fatal log line written to stderr when destroyed */
class LogMessage {
 public:
  LogMessage(const char* file, int line) {
    stream_ << "[" << DateLogger().HumanDate() << "] "
            << log_detail::RankPrefix() << file << ":" << line << ": ";
  }
  ~LogMessage() {
    stream_ << '\n';
    const std::string s = stream_.str();
    std::fwrite(s.data(), 1, s.size(), stderr);
  }
  std::ostream& stream() { return stream_; }

 protected:
  std::ostringstream stream_;

 private:
  DISALLOW_COPY_AND_ASSIGN(LogMessage);
};

/*! \brief fatal log line: throws dmlc::Error (or aborts) when destroyed */
class LogMessageFatal {
 public:
  LogMessageFatal(const char* file, int line) {
    stream_ << "[" << DateLogger().HumanDate() << "] "
            << log_detail::RankPrefix() << file << ":" << line << ": ";
  }
  std::ostream& stream() { return stream_; }
  ~LogMessageFatal() DMLC_THROW_EXCEPTION {
#if DMLC_LOG_STACK_TRACE
    stream_ << "\n\nStack trace:\n" << StackTrace(1);
#endif
#if DMLC_LOG_FATAL_THROW
    // do not throw while another exception is already unwinding
    if (std::uncaught_exceptions() == 0) throw Error(stream_.str());
#endif
    const std::string s = stream_.str() + "\n";
    std::fwrite(s.data(), 1, s.size(), stderr);
    std::abort();
  }

 private:
  std::ostringstream stream_;
  DISALLOW_COPY_AND_ASSIGN(LogMessageFatal);
};

/*! \brief swallows a stream expression (used for disabled log statements) */
class LogMessageVoidify {
 public:
  LogMessageVoidify() {}
  // lower precedence than << but higher than ?:
  void operator&(std::ostream&) {}
};

/*! \brief result of a failed binary CHECK, carrying "(a vs. b)" text */
struct LogCheckError {
  LogCheckError() : str(nullptr) {}
  explicit LogCheckError(const std::string& s) : str(new std::string(s)) {}
  LogCheckError(const LogCheckError&) = delete;
  LogCheckError(LogCheckError&& o) noexcept : str(o.str) { o.str = nullptr; }
  ~LogCheckError() { delete str; }
  explicit operator bool() const { return str != nullptr; }
  std::string* str;
};

#define DMLC_DEFINE_CHECK_FUNC(name, op)                                  \
  template <typename X, typename Y>                                       \
  inline LogCheckError LogCheck##name(const X& x, const Y& y) {           \
    if (x op y) return LogCheckError();                                   \
    std::ostringstream os;                                                \
    os << " (" << x << " vs. " << y << ") ";                              \
    return LogCheckError(os.str());                                       \
  }                                                                       \
  inline LogCheckError LogCheck##name(int x, int y) {                     \
    return LogCheck##name<int, int>(x, y);                                \
  }

#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wsign-compare"
DMLC_DEFINE_CHECK_FUNC(_LT, <)
DMLC_DEFINE_CHECK_FUNC(_GT, >)
DMLC_DEFINE_CHECK_FUNC(_LE, <=)
DMLC_DEFINE_CHECK_FUNC(_GE, >=)
DMLC_DEFINE_CHECK_FUNC(_EQ, ==)
DMLC_DEFINE_CHECK_FUNC(_NE, !=)
#pragma GCC diagnostic pop

/*! \brief LOG_EVERY_N helper: true on calls 1, N+1, 2N+1, ... of one site */
inline bool LogEveryNCheck(std::atomic<uint64_t>* counter, uint64_t n) {
  return (counter->fetch_add(1, std::memory_order_relaxed) % (n == 0 ? 1 : n)) == 0;
}

}  // namespace dmlc

#if DMLC_LOG_CUSTOMIZE
#define LOG_INFO ::dmlc::CustomLogMessage(__FILE__, __LINE__)
#else
#define LOG_INFO ::dmlc::LogMessage(__FILE__, __LINE__)
#endif
#define LOG_DEBUG LOG_INFO
#define LOG_WARNING LOG_INFO
#define LOG_ERROR LOG_INFO
#define LOG_FATAL ::dmlc::LogMessageFatal(__FILE__, __LINE__)
#define LOG_QFATAL LOG_FATAL

#define LOG(severity) LOG_##severity.stream()
#define LG LOG_INFO.stream()
#define LOG_IF(severity, condition) \
  !(condition) ? (void)0 : ::dmlc::LogMessageVoidify() & LOG(severity)

#define VLOG(n) LOG_IF(INFO, (n) <= ::dmlc::log_detail::VerboseLevel())

#define LOG_EVERY_N(severity, n)                                          \
  static std::atomic<uint64_t> DMLC_STR_CONCAT(dmlc_every_n_, __LINE__){0}; \
  LOG_IF(severity, ::dmlc::LogEveryNCheck(                                \
                       &DMLC_STR_CONCAT(dmlc_every_n_, __LINE__), (n)))

#define CHECK(x)                                          \
  if (__builtin_expect(!(x), 0))                          \
  ::dmlc::LogMessageFatal(__FILE__, __LINE__).stream()    \
      << "Check failed: " #x << ": "

#define CHECK_BINARY_OP(name, op, x, y)                                \
  if (::dmlc::LogCheckError _check_err = ::dmlc::LogCheck##name(x, y)) \
  ::dmlc::LogMessageFatal(__FILE__, __LINE__).stream()                 \
      << "Check failed: " << #x " " #op " " #y << *(_check_err.str) << ": "

#define CHECK_LT(x, y) CHECK_BINARY_OP(_LT, <, x, y)
#define CHECK_GT(x, y) CHECK_BINARY_OP(_GT, >, x, y)
#define CHECK_LE(x, y) CHECK_BINARY_OP(_LE, <=, x, y)
#define CHECK_GE(x, y) CHECK_BINARY_OP(_GE, >=, x, y)
#define CHECK_EQ(x, y) CHECK_BINARY_OP(_EQ, ==, x, y)
#define CHECK_NE(x, y) CHECK_BINARY_OP(_NE, !=, x, y)
#define CHECK_NOTNULL(x)                                                    \
  ((x) == nullptr                                                           \
       ? (::dmlc::LogMessageFatal(__FILE__, __LINE__).stream()              \
              << "Check  notnull: " #x << ' ',                              \
          (x))                                                              \
       : (x))

#ifdef NDEBUG
#define DCHECK(x) \
  while (false) CHECK(x)
#define DCHECK_LT(x, y) \
  while (false) CHECK((x) < (y))
#define DCHECK_GT(x, y) \
  while (false) CHECK((x) > (y))
#define DCHECK_LE(x, y) \
  while (false) CHECK((x) <= (y))
#define DCHECK_GE(x, y) \
  while (false) CHECK((x) >= (y))
#define DCHECK_EQ(x, y) \
  while (false) CHECK((x) == (y))
#define DCHECK_NE(x, y) \
  while (false) CHECK((x) != (y))
#else
#define DCHECK(x) CHECK(x)
#define DCHECK_LT(x, y) CHECK((x) < (y))
#define DCHECK_GT(x, y) CHECK((x) > (y))
#define DCHECK_LE(x, y) CHECK((x) <= (y))
#define DCHECK_GE(x, y) CHECK((x) >= (y))
#define DCHECK_EQ(x, y) CHECK((x) == (y))
#define DCHECK_NE(x, y) CHECK((x) != (y))
#endif

#endif  // DMLC_LOGGING_H_
