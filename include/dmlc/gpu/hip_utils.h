/*!
 * \file dmlc/gpu/hip_utils.h
 * \brief HIP error checking and RAII handles (streams, events, device and
 *  pinned buffers) for the MI355X ingestion path.
 *
 * Every HIP failure becomes a dmlc::Error carrying the device id and the
 * process rank (via the logging prefix), so GPU faults surface through the
 * same exception path as every other error (SURVEY §5.3 design).
 */
#ifndef DMLC_GPU_HIP_UTILS_H_
#define DMLC_GPU_HIP_UTILS_H_

#include <dmlc/logging.h>
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <string>
#include <utility>

/*! \brief throw dmlc::Error if a HIP call fails */
#define DMLC_HIP_CHECK(call)                                                    \
  do {                                                                          \
    hipError_t _e = (call);                                                     \
    if (_e != hipSuccess) {                                                     \
      int _dev = -1;                                                            \
      (void)hipGetDevice(&_dev);                                                \
      LOG(FATAL) << "HIP error " << hipGetErrorName(_e) << " (" << hipGetErrorString(_e) \
                 << ") on device " << _dev << " at " #call;                     \
    }                                                                           \
  } while (0)

namespace dmlc {
namespace gpu {

/*! \brief number of visible HIP devices (0 when no GPU / no driver) */
int DeviceCount();
/*! \brief true when at least one HIP device is usable */
bool Available();
/*! \brief hipSetDevice with error checking */
void SetDevice(int device);
/*! \brief "gfx950" etc. for device `device` */
std::string DeviceArchName(int device);

/*! \brief owning hipStream_t (non-blocking w.r.t. the null stream) */
class Stream {
 public:
  explicit Stream(int priority = 0) {
    DMLC_HIP_CHECK(hipStreamCreateWithPriority(&s_, hipStreamNonBlocking, priority));
  }
  ~Stream() {
    if (s_ != nullptr) (void)hipStreamDestroy(s_);
  }
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  hipStream_t get() const { return s_; }
  void Synchronize() const { DMLC_HIP_CHECK(hipStreamSynchronize(s_)); }

 private:
  hipStream_t s_{nullptr};
};

/*! \brief owning hipEvent_t */
class Event {
 public:
  explicit Event(bool timing = false) {
    DMLC_HIP_CHECK(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming));
  }
  ~Event() {
    if (e_ != nullptr) (void)hipEventDestroy(e_);
  }
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  hipEvent_t get() const { return e_; }
  void Record(hipStream_t s) { DMLC_HIP_CHECK(hipEventRecord(e_, s)); }
  void Synchronize() const { DMLC_HIP_CHECK(hipEventSynchronize(e_)); }
  bool Query() const {
    hipError_t r = hipEventQuery(e_);
    if (r == hipSuccess) return true;
    if (r == hipErrorNotReady) return false;
    DMLC_HIP_CHECK(r);
    return false;
  }

 private:
  hipEvent_t e_{nullptr};
};

/*! \brief device allocation of `bytes` (grow-only Reserve) */
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes) { Reserve(bytes); }
  ~DeviceBuffer() { Free(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept : ptr_(o.ptr_), bytes_(o.bytes_) {
    o.ptr_ = nullptr;
    o.bytes_ = 0;
  }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
      Free();
      std::swap(ptr_, o.ptr_);
      std::swap(bytes_, o.bytes_);
    }
    return *this;
  }
  /*! \brief ensure capacity >= bytes; contents are NOT preserved */
  void Reserve(size_t bytes) {
    if (bytes <= bytes_) return;
    Free();
    DMLC_HIP_CHECK(hipMalloc(&ptr_, bytes == 0 ? 1 : bytes));
    bytes_ = bytes;
  }
  /*! \brief ensure capacity >= bytes, preserving the first `keep` bytes */
  void Grow(size_t bytes, size_t keep, hipStream_t stream) {
    if (bytes <= bytes_) return;
    void* p = nullptr;
    DMLC_HIP_CHECK(hipMalloc(&p, bytes));
    if (keep != 0 && ptr_ != nullptr) {
      DMLC_HIP_CHECK(hipMemcpyAsync(p, ptr_, keep, hipMemcpyDeviceToDevice, stream));
      DMLC_HIP_CHECK(hipStreamSynchronize(stream));
    }
    Free();
    ptr_ = p;
    bytes_ = bytes;
  }
  void Free() {
    if (ptr_ != nullptr) (void)hipFree(ptr_);
    ptr_ = nullptr;
    bytes_ = 0;
  }
  template <typename T = void>
  T* get() const {
    return static_cast<T*>(ptr_);
  }
  size_t bytes() const { return bytes_; }
  void swap(DeviceBuffer& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(bytes_, o.bytes_);
  }

 private:
  void* ptr_{nullptr};
  size_t bytes_{0};
};

/*! \brief page-locked host allocation (DMA source for hipMemcpyAsync) */
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t bytes, bool mapped = false) { Reserve(bytes, mapped); }
  ~PinnedBuffer() { Free(); }
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  PinnedBuffer(PinnedBuffer&& o) noexcept : ptr_(o.ptr_), bytes_(o.bytes_) {
    o.ptr_ = nullptr;
    o.bytes_ = 0;
  }
  void Reserve(size_t bytes, bool mapped = false) {
    if (bytes <= bytes_) return;
    Free();
    unsigned flags = hipHostMallocDefault;
    // mapped buffers are polled by the host while kernels write them:
    // coherent explicitly, whatever HIP_HOST_COHERENT says
    if (mapped) flags |= hipHostMallocMapped | hipHostMallocCoherent;
    DMLC_HIP_CHECK(hipHostMalloc(&ptr_, bytes == 0 ? 1 : bytes, flags));
    bytes_ = bytes;
  }
  void Free() {
    if (ptr_ != nullptr) (void)hipHostFree(ptr_);
    ptr_ = nullptr;
    bytes_ = 0;
  }
  template <typename T = void>
  T* get() const {
    return static_cast<T*>(ptr_);
  }
  size_t bytes() const { return bytes_; }
  void swap(PinnedBuffer& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(bytes_, o.bytes_);
  }

 private:
  void* ptr_{nullptr};
  size_t bytes_{0};
};

/*! \brief roctx range for rocprofv3 marker traces (no-op if roctx missing) */
class ScopedRange {
 public:
  explicit ScopedRange(const char* name);
  ~ScopedRange();
  ScopedRange(const ScopedRange&) = delete;
  ScopedRange& operator=(const ScopedRange&) = delete;

 private:
  bool active_{false};
};

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_GPU_HIP_UTILS_H_
