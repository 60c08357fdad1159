/*!
 * \file dmlc/concurrentqueue.h
 * \brief Unbounded multi-producer multi-consumer lock-free queue.
 *
 * Parity: reference `include/dmlc/concurrentqueue.h` (a vendored third-party
 * queue, 3,719 lines) — ConcurrentQueue<T> with ProducerToken/ConsumerToken
 * (:574-673), enqueue / try_enqueue / enqueue_bulk / try_dequeue /
 * try_dequeue_bulk / size_approx / is_lock_free (:928-1270).  SURVEY §2.9
 * asks for a from-scratch rewrite; this is a different (much smaller) design:
 *
 *  - storage is a singly linked list of fixed segments of kCells cells;
 *  - producers claim a cell with one fetch_add on the tail segment's enqueue
 *    index, construct the value, then publish the cell with a release store;
 *  - consumers claim with a CAS on the head segment's dequeue index, and only
 *    claim indices a producer already reserved, so an empty queue never burns
 *    cells and a claimed cell is always filled (the consumer spins only for a
 *    producer that is between its reservation and its publish);
 *  - a full segment is followed by a fresh one linked with one CAS (the
 *    producer that links it pre-fills its cell 0);
 *  - fully drained segments are retired and reclaimed with hazard pointers
 *    (one hazard slot per thread, process-wide registry), then recycled
 *    through a small per-queue spare pool.
 *
 * FIFO order holds per producer (and globally for cells of one segment), the
 * same guarantee the reference gives.  Tokens are accepted for API parity;
 * they carry no state here because there are no per-producer sub-queues.
 */
#ifndef DMLC_CONCURRENTQUEUE_H_
#define DMLC_CONCURRENTQUEUE_H_

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <new>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

namespace dmlc {
namespace lockfree_detail {

/*! \brief one published hazard pointer, owned by one thread at a time */
struct HazardRecord {
  std::atomic<void*> ptr{nullptr};
  std::atomic<bool> active{false};
  HazardRecord* next{nullptr};
};

/*! \brief process-wide, append-only list of hazard records (never freed) */
class HazardRegistry {
 public:
  static HazardRegistry& Get() {
    static HazardRegistry* inst = new HazardRegistry();  // intentionally leaked
    return *inst;
  }
  HazardRecord* Acquire() {
    for (HazardRecord* r = head_.load(std::memory_order_acquire); r != nullptr; r = r->next) {
      bool expected = false;
      if (!r->active.load(std::memory_order_relaxed) &&
          r->active.compare_exchange_strong(expected, true, std::memory_order_acq_rel)) {
        return r;
      }
    }
    HazardRecord* r = new HazardRecord();
    r->active.store(true, std::memory_order_relaxed);
    HazardRecord* old = head_.load(std::memory_order_relaxed);
    do {
      r->next = old;
    } while (!head_.compare_exchange_weak(old, r, std::memory_order_acq_rel));
    return r;
  }
  void Release(HazardRecord* r) {
    r->ptr.store(nullptr, std::memory_order_release);
    r->active.store(false, std::memory_order_release);
  }
  bool IsHazard(const void* p) const {
    for (HazardRecord* r = head_.load(std::memory_order_acquire); r != nullptr; r = r->next) {
      if (r->ptr.load(std::memory_order_seq_cst) == p) return true;
    }
    return false;
  }

 private:
  std::atomic<HazardRecord*> head_{nullptr};
};

/*! \brief this thread's hazard slot (released when the thread exits) */
inline HazardRecord* ThisThreadHazard() {
  struct Holder {
    HazardRecord* rec = HazardRegistry::Get().Acquire();
    ~Holder() { HazardRegistry::Get().Release(rec); }
  };
  thread_local Holder holder;
  return holder.rec;
}

inline void CpuRelax(int* spins) {
  if (++*spins < 128) {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
  } else {
    std::this_thread::yield();
  }
}

constexpr size_t kCacheLine = 64;

}  // namespace lockfree_detail

template <typename T>
class ConcurrentQueue;

/*! \brief API-parity producer token (stateless here) */
class ProducerToken {
 public:
  template <typename Q>
  explicit ProducerToken(Q& /*queue*/) {}
  bool valid() const { return true; }
};

/*! \brief API-parity consumer token (stateless here) */
class ConsumerToken {
 public:
  template <typename Q>
  explicit ConsumerToken(Q& /*queue*/) {}
  bool valid() const { return true; }
};

template <typename T>
class ConcurrentQueue {
 public:
  using value_type = T;
  using size_t = std::size_t;
  static constexpr size_t kCells = 512;

  /*! \param initial_size_estimate pre-allocate segments for about this many items */
  explicit ConcurrentQueue(size_t initial_size_estimate = 6 * kCells) {
    Segment* s = new Segment();
    head_.store(s, std::memory_order_relaxed);
    tail_.store(s, std::memory_order_relaxed);
    for (size_t n = kCells; n < initial_size_estimate; n += kCells) spares_.push_back(new Segment());
  }
  ~ConcurrentQueue() {
    Segment* s = head_.load(std::memory_order_relaxed);
    while (s != nullptr) {
      size_t end = std::min<size_t>(s->enq.load(std::memory_order_relaxed), kCells);
      for (size_t i = s->deq.load(std::memory_order_relaxed); i < end; ++i) {
        if (s->cells[i].state.load(std::memory_order_relaxed) == kFull) s->cells[i].ptr()->~T();
      }
      Segment* n = s->next.load(std::memory_order_relaxed);
      delete s;
      s = n;
    }
    for (Segment* r : retired_) delete r;
    for (Segment* r : spares_) delete r;
  }
  ConcurrentQueue(const ConcurrentQueue&) = delete;
  ConcurrentQueue& operator=(const ConcurrentQueue&) = delete;

  /*! \brief enqueue, allocating a segment when needed (fails only on OOM) */
  bool enqueue(const T& item) { return Emplace(true, item); }
  bool enqueue(T&& item) { return Emplace(true, std::move(item)); }
  bool enqueue(const ProducerToken&, const T& item) { return Emplace(true, item); }
  bool enqueue(const ProducerToken&, T&& item) { return Emplace(true, std::move(item)); }
  /*! \brief enqueue without allocating: fails when a new segment would be needed
   *  and the spare pool is empty */
  bool try_enqueue(const T& item) { return Emplace(false, item); }
  bool try_enqueue(T&& item) { return Emplace(false, std::move(item)); }
  bool try_enqueue(const ProducerToken&, const T& item) { return Emplace(false, item); }
  bool try_enqueue(const ProducerToken&, T&& item) { return Emplace(false, std::move(item)); }

  template <typename It>
  bool enqueue_bulk(It first, size_t count) {
    for (size_t i = 0; i < count; ++i, ++first) {
      if (!enqueue(*first)) return false;
    }
    return true;
  }
  template <typename It>
  bool enqueue_bulk(const ProducerToken&, It first, size_t count) {
    return enqueue_bulk(first, count);
  }
  template <typename It>
  bool try_enqueue_bulk(It first, size_t count) {
    for (size_t i = 0; i < count; ++i, ++first) {
      if (!try_enqueue(*first)) return false;
    }
    return true;
  }

  /*! \brief dequeue into `item`; false if the queue looked empty */
  template <typename U>
  bool try_dequeue(U& item) {
    lockfree_detail::HazardRecord* hp = lockfree_detail::ThisThreadHazard();
    for (;;) {
      Segment* s = Protect(head_, hp);
      size_t d = s->deq.load(std::memory_order_acquire);
      if (d >= kCells) {
        Segment* n = s->next.load(std::memory_order_acquire);
        if (n == nullptr) {
          hp->ptr.store(nullptr, std::memory_order_release);
          return false;  // producers of the next segment are mid-link
        }
        Segment* t = s;
        tail_.compare_exchange_strong(t, n, std::memory_order_seq_cst);  // never retire the tail
        Segment* h = s;
        if (head_.compare_exchange_strong(h, n, std::memory_order_seq_cst)) {
          hp->ptr.store(nullptr, std::memory_order_release);
          Retire(s);
        }
        continue;
      }
      size_t e = std::min<size_t>(s->enq.load(std::memory_order_acquire), kCells);
      if (d >= e) {
        hp->ptr.store(nullptr, std::memory_order_release);
        return false;
      }
      if (!s->deq.compare_exchange_weak(d, d + 1, std::memory_order_acq_rel)) continue;
      Cell& c = s->cells[d];
      int spins = 0;
      while (c.state.load(std::memory_order_acquire) != kFull) lockfree_detail::CpuRelax(&spins);
      item = std::move(*c.ptr());
      c.ptr()->~T();
      hp->ptr.store(nullptr, std::memory_order_release);
      size_.fetch_sub(1, std::memory_order_relaxed);
      return true;
    }
  }
  template <typename U>
  bool try_dequeue(const ConsumerToken&, U& item) {
    return try_dequeue(item);
  }
  /*! \brief dequeue up to `max` items; returns how many */
  template <typename It>
  size_t try_dequeue_bulk(It out, size_t max) {
    size_t n = 0;
    while (n < max) {
      T tmp;
      if (!try_dequeue(tmp)) break;
      *out = std::move(tmp);
      ++out;
      ++n;
    }
    return n;
  }
  template <typename It>
  size_t try_dequeue_bulk(const ConsumerToken&, It out, size_t max) {
    return try_dequeue_bulk(out, max);
  }

  /*! \brief approximate number of items (exact when quiescent) */
  size_t size_approx() const {
    int64_t s = size_.load(std::memory_order_relaxed);
    return s < 0 ? 0 : static_cast<size_t>(s);
  }
  static constexpr bool is_lock_free() {
    return std::atomic<size_t>::is_always_lock_free && std::atomic<void*>::is_always_lock_free;
  }

 private:
  enum : uint32_t { kEmpty = 0, kFull = 1 };
  struct Cell {
    std::atomic<uint32_t> state{kEmpty};
    alignas(T) unsigned char storage[sizeof(T)];
    T* ptr() { return reinterpret_cast<T*>(storage); }
  };
  struct Segment {
    alignas(lockfree_detail::kCacheLine) std::atomic<size_t> enq{0};
    alignas(lockfree_detail::kCacheLine) std::atomic<size_t> deq{0};
    alignas(lockfree_detail::kCacheLine) std::atomic<Segment*> next{nullptr};
    Cell cells[kCells];
    void Reset() {
      enq.store(0, std::memory_order_relaxed);
      deq.store(0, std::memory_order_relaxed);
      next.store(nullptr, std::memory_order_relaxed);
      for (Cell& c : cells) c.state.store(kEmpty, std::memory_order_relaxed);
    }
  };

  static Segment* Protect(const std::atomic<Segment*>& src, lockfree_detail::HazardRecord* hp) {
    Segment* p = src.load(std::memory_order_acquire);
    for (;;) {
      hp->ptr.store(p, std::memory_order_seq_cst);
      Segment* q = src.load(std::memory_order_seq_cst);
      if (q == p) return p;
      p = q;
    }
  }

  template <typename U>
  bool Emplace(bool can_alloc, U&& item) {
    lockfree_detail::HazardRecord* hp = lockfree_detail::ThisThreadHazard();
    for (;;) {
      Segment* s = Protect(tail_, hp);
      size_t i = s->enq.fetch_add(1, std::memory_order_acq_rel);
      if (i < kCells) {
        Cell& c = s->cells[i];
        new (c.storage) T(std::forward<U>(item));
        size_.fetch_add(1, std::memory_order_relaxed);
        c.state.store(kFull, std::memory_order_release);
        hp->ptr.store(nullptr, std::memory_order_release);
        return true;
      }
      Segment* n = s->next.load(std::memory_order_acquire);
      if (n == nullptr) {
        Segment* fresh = TakeSpare();
        if (fresh == nullptr) {
          if (!can_alloc) {
            hp->ptr.store(nullptr, std::memory_order_release);
            return false;
          }
          fresh = new (std::nothrow) Segment();
          if (fresh == nullptr) {
            hp->ptr.store(nullptr, std::memory_order_release);
            return false;
          }
        }
        // pre-fill cell 0 so the linking producer is done in one step
        new (fresh->cells[0].storage) T(std::forward<U>(item));
        fresh->cells[0].state.store(kFull, std::memory_order_relaxed);
        fresh->enq.store(1, std::memory_order_relaxed);
        Segment* expected = nullptr;
        if (s->next.compare_exchange_strong(expected, fresh, std::memory_order_acq_rel)) {
          size_.fetch_add(1, std::memory_order_relaxed);
          Segment* t = s;
          tail_.compare_exchange_strong(t, fresh, std::memory_order_seq_cst);
          hp->ptr.store(nullptr, std::memory_order_release);
          return true;
        }
        // lost the race: take the value back and recycle the segment
        fresh->cells[0].ptr()->~T();
        fresh->Reset();
        GiveSpare(fresh);
        n = expected;
      }
      Segment* t = s;
      tail_.compare_exchange_strong(t, n, std::memory_order_seq_cst);
    }
  }

  Segment* TakeSpare() {
    std::lock_guard<std::mutex> lock(pool_mutex_);
    if (spares_.empty()) return nullptr;
    Segment* s = spares_.back();
    spares_.pop_back();
    return s;
  }
  void GiveSpare(Segment* s) {
    std::lock_guard<std::mutex> lock(pool_mutex_);
    spares_.push_back(s);
  }
  /*! \brief park an unlinked segment; recycle those no thread still protects */
  void Retire(Segment* s) {
    std::lock_guard<std::mutex> lock(pool_mutex_);
    retired_.push_back(s);
    if (retired_.size() < 4) return;
    auto& reg = lockfree_detail::HazardRegistry::Get();
    size_t keep = 0;
    for (Segment* r : retired_) {
      if (reg.IsHazard(r)) {
        retired_[keep++] = r;
      } else if (spares_.size() < 8) {
        r->Reset();
        spares_.push_back(r);
      } else {
        delete r;
      }
    }
    retired_.resize(keep);
  }

  alignas(lockfree_detail::kCacheLine) std::atomic<Segment*> head_{nullptr};
  alignas(lockfree_detail::kCacheLine) std::atomic<Segment*> tail_{nullptr};
  alignas(lockfree_detail::kCacheLine) std::atomic<int64_t> size_{0};
  std::mutex pool_mutex_;
  std::vector<Segment*> retired_;
  std::vector<Segment*> spares_;
};

}  // namespace dmlc
#endif  // DMLC_CONCURRENTQUEUE_H_
