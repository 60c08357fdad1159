/*!
 * \file dmlc/concurrency.h
 * \brief Spinlock and a blocking FIFO / priority queue with kill signalling.
 *
 * Parity: reference `include/dmlc/concurrency.h` — Spinlock on atomic_flag
 * (:24-53, :142-149), ConcurrentBlockingQueue<T, kFIFO|kPriority> with
 * Push / PushFront / Pop / SignalForKill / Size (:56-140, :151-255).
 *
 * New implementation: the spinlock backs off with the x86 `pause` hint and a
 * yield after a bounded spin (the reader threads of the GPU ingestion ring
 * share cores with OpenMP teams, so unbounded spinning starves them); the
 * queue keeps one condition variable and a waiter count so Push only notifies
 * when somebody sleeps.  The priority variant orders by `operator<` on
 * `std::pair<T, int>`-free storage (an explicit priority argument, highest
 * first, FIFO among equal priorities).
 */
#ifndef DMLC_CONCURRENCY_H_
#define DMLC_CONCURRENCY_H_

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <queue>
#include <thread>
#include <utility>
#include <vector>

#include "./base.h"

namespace dmlc {

/*! \brief test-and-test-and-set spinlock (BasicLockable) */
class Spinlock {
 public:
  Spinlock() = default;
  DISALLOW_COPY_AND_ASSIGN(Spinlock);

  inline void lock() noexcept {
    for (int spins = 0;; ++spins) {
      if (!flag_.exchange(true, std::memory_order_acquire)) return;
      while (flag_.load(std::memory_order_relaxed)) {
        if (spins++ < 64) {
          Pause();
        } else {
          std::this_thread::yield();
        }
      }
    }
  }
  inline bool try_lock() noexcept {
    return !flag_.load(std::memory_order_relaxed) &&
           !flag_.exchange(true, std::memory_order_acquire);
  }
  inline void unlock() noexcept { flag_.store(false, std::memory_order_release); }

 private:
  static inline void Pause() noexcept {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
  }
  std::atomic<bool> flag_{false};
};

/*! \brief queue discipline of ConcurrentBlockingQueue */
enum class ConcurrentQueueType { kFIFO, kPriority };

/*!
 * \brief multi-producer multi-consumer blocking queue.
 *
 *  Pop blocks until an element arrives or SignalForKill is called; after a
 *  kill, Pop drains nothing and returns false (matching the reference, where
 *  killed consumers exit immediately).
 */
template <typename T, ConcurrentQueueType type = ConcurrentQueueType::kFIFO>
class ConcurrentBlockingQueue {
 public:
  ConcurrentBlockingQueue() = default;
  DISALLOW_COPY_AND_ASSIGN(ConcurrentBlockingQueue);

  /*! \brief enqueue (priority is ignored for FIFO queues) */
  template <typename E>
  void Push(E&& e, int priority = 0) {
    bool wake;
    {
      std::lock_guard<std::mutex> lock(mutex_);
      if (type == ConcurrentQueueType::kFIFO) {
        fifo_.emplace_back(std::forward<E>(e));
      } else {
        prio_.push(Entry{priority, seq_++, T(std::forward<E>(e))});
      }
      wake = nwait_ != 0;
    }
    if (wake) cv_.notify_one();
  }
  /*! \brief enqueue at the head (FIFO) or with the highest priority so far */
  template <typename E>
  void PushFront(E&& e, int priority = 0) {
    bool wake;
    {
      std::lock_guard<std::mutex> lock(mutex_);
      if (type == ConcurrentQueueType::kFIFO) {
        fifo_.emplace_front(std::forward<E>(e));
      } else {
        prio_.push(Entry{priority, seq_++, T(std::forward<E>(e))});
      }
      wake = nwait_ != 0;
    }
    if (wake) cv_.notify_one();
  }
  /*!
   * \brief dequeue, blocking until data or kill
   * \return false if the queue was killed
   */
  bool Pop(T* rv) {
    std::unique_lock<std::mutex> lock(mutex_);
    ++nwait_;
    cv_.wait(lock, [this] { return exit_now_ || !EmptyLocked(); });
    --nwait_;
    if (exit_now_) return false;
    TakeLocked(rv);
    return true;
  }
  /*! \brief non-blocking dequeue */
  bool TryPop(T* rv) {
    std::lock_guard<std::mutex> lock(mutex_);
    if (exit_now_ || EmptyLocked()) return false;
    TakeLocked(rv);
    return true;
  }
  /*! \brief wake every blocked Pop; subsequent Pops return false */
  void SignalForKill() {
    {
      std::lock_guard<std::mutex> lock(mutex_);
      exit_now_ = true;
    }
    cv_.notify_all();
  }
  /*! \brief number of queued elements */
  size_t Size() {
    std::lock_guard<std::mutex> lock(mutex_);
    return type == ConcurrentQueueType::kFIFO ? fifo_.size() : prio_.size();
  }

 private:
  struct Entry {
    int priority;
    uint64_t seq;
    T data;
    // highest priority first, then FIFO (smaller seq first)
    bool operator<(const Entry& o) const {
      return priority != o.priority ? priority < o.priority : seq > o.seq;
    }
  };
  bool EmptyLocked() const {
    return type == ConcurrentQueueType::kFIFO ? fifo_.empty() : prio_.empty();
  }
  void TakeLocked(T* rv) {
    if (type == ConcurrentQueueType::kFIFO) {
      *rv = std::move(fifo_.front());
      fifo_.pop_front();
    } else {
      *rv = std::move(const_cast<Entry&>(prio_.top()).data);
      prio_.pop();
    }
  }

  std::mutex mutex_;
  std::condition_variable cv_;
  std::deque<T> fifo_;
  std::priority_queue<Entry> prio_;
  uint64_t seq_{0};
  int nwait_{0};
  bool exit_now_{false};
};

}  // namespace dmlc
#endif  // DMLC_CONCURRENCY_H_
