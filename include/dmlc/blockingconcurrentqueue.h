/*!
 * \file dmlc/blockingconcurrentqueue.h
 * \brief ConcurrentQueue plus a counting semaphore: blocking / timed dequeue.
 *
 * Parity: reference `include/dmlc/blockingconcurrentqueue.h` (vendored, 991
 * lines) — BlockingConcurrentQueue with enqueue*, try_dequeue*, wait_dequeue,
 * wait_dequeue_timed, wait_dequeue_bulk(_timed), size_approx.  New design:
 * the semaphore is a "benaphore" — an atomic count that only falls back to a
 * kernel semaphore (POSIX sem_t) when it goes negative, after a short spin —
 * so an uncontended hand-off costs two atomics and no syscall.
 */
#ifndef DMLC_BLOCKINGCONCURRENTQUEUE_H_
#define DMLC_BLOCKINGCONCURRENTQUEUE_H_

#include <errno.h>
#include <semaphore.h>
#include <time.h>

#include <atomic>
#include <cstdint>

#include "./concurrentqueue.h"

namespace dmlc {
namespace lockfree_detail {

/*! \brief counting semaphore with a user-space fast path */
class LightweightSemaphore {
 public:
  explicit LightweightSemaphore(int64_t initial = 0) : count_(initial) {
    sem_init(&sem_, 0, 0);
  }
  ~LightweightSemaphore() { sem_destroy(&sem_); }
  LightweightSemaphore(const LightweightSemaphore&) = delete;
  LightweightSemaphore& operator=(const LightweightSemaphore&) = delete;

  bool try_wait() {
    int64_t c = count_.load(std::memory_order_relaxed);
    while (c > 0) {
      if (count_.compare_exchange_weak(c, c - 1, std::memory_order_acquire)) return true;
    }
    return false;
  }
  /*! \brief wait; timeout_usec < 0 waits forever */
  bool wait(int64_t timeout_usec = -1) {
    for (int spin = 0; spin < 1024; ++spin) {
      if (try_wait()) return true;
#if defined(__x86_64__) || defined(__i386__)
      __builtin_ia32_pause();
#endif
    }
    if (count_.fetch_sub(1, std::memory_order_acquire) > 0) return true;
    // we are now a registered sleeper (count < 0)
    if (timeout_usec < 0) {
      while (sem_wait(&sem_) != 0 && errno == EINTR) {
      }
      return true;
    }
    if (timeout_usec > 0) {
      struct timespec ts;
      clock_gettime(CLOCK_REALTIME, &ts);
      int64_t ns = ts.tv_nsec + (timeout_usec % 1000000) * 1000;
      ts.tv_sec += timeout_usec / 1000000 + ns / 1000000000;
      ts.tv_nsec = ns % 1000000000;
      for (;;) {
        if (sem_timedwait(&sem_, &ts) == 0) return true;
        if (errno != EINTR) break;
      }
    }
    // timed out: deregister, unless a signal already counted us in
    for (;;) {
      int64_t c = count_.load(std::memory_order_relaxed);
      if (c < 0 && count_.compare_exchange_strong(c, c + 1, std::memory_order_relaxed)) {
        return false;
      }
      if (c >= 0 && sem_trywait(&sem_) == 0) return true;
    }
  }
  /*! \brief take up to `max` units, waiting for at least one */
  int64_t wait_many(int64_t max, int64_t timeout_usec = -1) {
    int64_t c = count_.load(std::memory_order_relaxed);
    while (c > 0) {
      int64_t take = c < max ? c : max;
      if (count_.compare_exchange_weak(c, c - take, std::memory_order_acquire)) return take;
    }
    if (!wait(timeout_usec)) return 0;
    int64_t got = 1;
    while (got < max && try_wait()) ++got;
    return got;
  }
  void signal(int64_t n = 1) {
    int64_t old = count_.fetch_add(n, std::memory_order_release);
    int64_t sleepers = old < 0 ? -old : 0;
    int64_t wake = sleepers < n ? sleepers : n;
    while (wake-- > 0) sem_post(&sem_);
  }
  int64_t available() const {
    int64_t c = count_.load(std::memory_order_relaxed);
    return c > 0 ? c : 0;
  }

 private:
  std::atomic<int64_t> count_;
  sem_t sem_;
};

}  // namespace lockfree_detail

template <typename T>
class BlockingConcurrentQueue {
 public:
  using value_type = T;
  explicit BlockingConcurrentQueue(size_t initial_size_estimate = 6 * ConcurrentQueue<T>::kCells)
      : queue_(initial_size_estimate) {}
  BlockingConcurrentQueue(const BlockingConcurrentQueue&) = delete;
  BlockingConcurrentQueue& operator=(const BlockingConcurrentQueue&) = delete;

  template <typename U>
  bool enqueue(U&& item) {
    if (!queue_.enqueue(std::forward<U>(item))) return false;
    sema_.signal();
    return true;
  }
  template <typename U>
  bool enqueue(const ProducerToken&, U&& item) {
    return enqueue(std::forward<U>(item));
  }
  template <typename U>
  bool try_enqueue(U&& item) {
    if (!queue_.try_enqueue(std::forward<U>(item))) return false;
    sema_.signal();
    return true;
  }
  template <typename It>
  bool enqueue_bulk(It first, size_t count) {
    size_t done = 0;
    for (; done < count; ++done, ++first) {
      if (!queue_.enqueue(*first)) break;
    }
    if (done) sema_.signal(static_cast<int64_t>(done));
    return done == count;
  }

  template <typename U>
  bool try_dequeue(U& item) {
    if (!sema_.try_wait()) return false;
    Take(item);
    return true;
  }
  template <typename U>
  bool try_dequeue(const ConsumerToken&, U& item) {
    return try_dequeue(item);
  }
  /*! \brief block until an item is available */
  template <typename U>
  void wait_dequeue(U& item) {
    sema_.wait();
    Take(item);
  }
  template <typename U>
  void wait_dequeue(const ConsumerToken&, U& item) {
    wait_dequeue(item);
  }
  /*! \brief block at most timeout_usecs; false on timeout */
  template <typename U>
  bool wait_dequeue_timed(U& item, int64_t timeout_usecs) {
    if (!sema_.wait(timeout_usecs)) return false;
    Take(item);
    return true;
  }
  template <typename It>
  size_t try_dequeue_bulk(It out, size_t max) {
    size_t n = 0;
    while (n < max && sema_.try_wait()) {
      T tmp;
      Take(tmp);
      *out = std::move(tmp);
      ++out;
      ++n;
    }
    return n;
  }
  /*! \brief wait for at least one item, take up to max */
  template <typename It>
  size_t wait_dequeue_bulk(It out, size_t max) {
    return BulkTake(out, sema_.wait_many(static_cast<int64_t>(max)));
  }
  template <typename It>
  size_t wait_dequeue_bulk_timed(It out, size_t max, int64_t timeout_usecs) {
    return BulkTake(out, sema_.wait_many(static_cast<int64_t>(max), timeout_usecs));
  }
  size_t size_approx() const { return static_cast<size_t>(sema_.available()); }
  static constexpr bool is_lock_free() { return ConcurrentQueue<T>::is_lock_free(); }

 private:
  // a semaphore unit guarantees an item is published or about to be
  template <typename U>
  void Take(U& item) {
    int spins = 0;
    while (!queue_.try_dequeue(item)) lockfree_detail::CpuRelax(&spins);
  }
  template <typename It>
  size_t BulkTake(It out, int64_t n) {
    for (int64_t i = 0; i < n; ++i, ++out) {
      T tmp;
      Take(tmp);
      *out = std::move(tmp);
    }
    return static_cast<size_t>(n);
  }

  ConcurrentQueue<T> queue_;
  lockfree_detail::LightweightSemaphore sema_;
};

}  // namespace dmlc
#endif  // DMLC_BLOCKINGCONCURRENTQUEUE_H_
