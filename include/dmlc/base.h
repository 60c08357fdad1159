/*!
 * \file dmlc/base.h
 * \brief Compile-time feature switches and tiny helpers shared by every layer.
 *
 * Parity: reference `include/dmlc/base.h:9-275` (feature macros DMLC_USE_*,
 * DMLC_LOG_FATAL_THROW, DISALLOW_COPY_AND_ASSIGN, BeginPtr).  This build is
 * C++17-only and targets Linux + ROCm (MI355X / gfx950), so the pre-C++11 and
 * MSVC branches of the reference are intentionally absent.  New switches:
 * DMLC_USE_HIP / DMLC_USE_RCCL describe whether the GPU ingestion path and the
 * RCCL communicator are compiled into libdmlc.
 */
#ifndef DMLC_BASE_H_
#define DMLC_BASE_H_

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

/*! \brief use glog for logging (never in this build; kept for API parity) */
#ifndef DMLC_USE_GLOG
#define DMLC_USE_GLOG 0
#endif

/*! \brief LOG(FATAL) / failed CHECK throws dmlc::Error (1) or aborts (0) */
#ifndef DMLC_LOG_FATAL_THROW
#define DMLC_LOG_FATAL_THROW 1
#endif

/*! \brief route log lines through dmlc::CustomLogMessage::Log */
#ifndef DMLC_LOG_CUSTOMIZE
#define DMLC_LOG_CUSTOMIZE 0
#endif

/*! \brief append a demangled stack trace to fatal messages */
#ifndef DMLC_LOG_STACK_TRACE
#define DMLC_LOG_STACK_TRACE 1
#endif

/*! \brief depth of the stack trace printed for fatal errors */
#ifndef DMLC_LOG_STACK_TRACE_SIZE
#define DMLC_LOG_STACK_TRACE_SIZE 12
#endif

/*! \brief remote filesystems: loaded with dlopen at run time, so always on */
#ifndef DMLC_USE_HDFS
#define DMLC_USE_HDFS 1
#endif
#ifndef DMLC_USE_S3
#define DMLC_USE_S3 1
#endif
#ifndef DMLC_USE_AZURE
#define DMLC_USE_AZURE 1
#endif

/*! \brief parameter-server roles (launch-only, see tracker) */
#ifndef DMLC_USE_PS
#define DMLC_USE_PS 0
#endif

/*! \brief C++11 and newer always available here */
#define DMLC_USE_CXX11 1
#define DMLC_USE_CXX14 1
#define DMLC_USE_CXX17 1
#define DMLC_ENABLE_STD_THREAD 1
#define DMLC_USE_REGEX 1
#define DMLC_STRICT_CXX11 0
#define DMLC_CXX11_THREAD_LOCAL 1
#define DMLC_MODERN_THREAD_LOCAL 1

/*! \brief the GPU (HIP, gfx950) ingestion path is compiled in */
#ifndef DMLC_USE_HIP
#define DMLC_USE_HIP 1
#endif
/*! \brief RCCL communicator (xGMI collectives) compiled in */
#ifndef DMLC_USE_RCCL
#define DMLC_USE_RCCL 1
#endif

#define DMLC_ATTRIBUTE_UNUSED __attribute__((unused))
#define DMLC_NO_INLINE __attribute__((noinline))
#define DMLC_ALWAYS_INLINE inline __attribute__((__always_inline__))
#define DMLC_THROW_EXCEPTION noexcept(false)
#define DMLC_NO_EXCEPTION noexcept(true)
#define DMLC_STR_CONCAT_(a, b) a##b
#define DMLC_STR_CONCAT(a, b) DMLC_STR_CONCAT_(a, b)

#ifndef DISALLOW_COPY_AND_ASSIGN
#define DISALLOW_COPY_AND_ASSIGN(T) \
  T(const T&) = delete;             \
  T& operator=(const T&) = delete
#endif

#if defined(__GNUC__)
#define DMLC_SUPPRESS_UBSAN __attribute__((no_sanitize("undefined")))
#else
#define DMLC_SUPPRESS_UBSAN
#endif

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__,
              "dmlc serializes in native (little-endian) byte order");

namespace dmlc {
/*!
 * \brief Pointer to the first element of a vector, or nullptr when empty.
 *  Used everywhere raw buffers are handed to Stream::Read/Write.
 */
template <typename T>
inline T* BeginPtr(std::vector<T>& vec) {  // NOLINT(runtime/references)
  return vec.empty() ? nullptr : vec.data();
}
template <typename T>
inline const T* BeginPtr(const std::vector<T>& vec) {
  return vec.empty() ? nullptr : vec.data();
}
inline char* BeginPtr(std::string& str) {  // NOLINT(runtime/references)
  return str.empty() ? nullptr : &str[0];
}
inline const char* BeginPtr(const std::string& str) {
  return str.empty() ? nullptr : str.data();
}
}  // namespace dmlc

#endif  // DMLC_BASE_H_
