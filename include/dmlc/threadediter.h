/*!
 * \file dmlc/threadediter.h
 * \brief Bounded producer/consumer prefetcher: one background thread runs a
 *  Producer while the consumer takes finished cells and recycles them.
 *
 * Parity: reference `include/dmlc/threadediter.h` — Producer {BeforeFirst,
 * Next} (:53-75), default capacity 8 (:80), Init(Producer*, own) (:287-297),
 * Init(next, beforefirst) (:300-408), BeforeFirst handshake (:178-203,
 * :331-346), Next / Recycle (:411-454), exception capture in the producer and
 * rethrow in the consumer (:374-403, :456-466), Destroy (:251-283),
 * DataIter adapter Next()/Value() (:158-176).
 *
 * Implementation is new: one mutex + two condition variables, an explicit
 * state machine {kProduce, kBeforeFirst, kDestroy}, and any exception type
 * (not only dmlc::Error) is transported through std::exception_ptr.
 * The GPU ingestion path (src/gpu/device_parser.cc) runs its pinned-host
 * slots through this iterator and gates device-slot reuse on hipEvents.
 */
#ifndef DMLC_THREADEDITER_H_
#define DMLC_THREADEDITER_H_

#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "./base.h"
#include "./data.h"
#include "./logging.h"

namespace dmlc {

/*! \brief base for ThreadedIter so that the control enum is not templated */
class ScopedThreadedIterState {
 public:
  enum Signal { kProduce, kBeforeFirst, kDestroy };
};

template <typename DType>
class ThreadedIter : public DataIter<DType> {
 public:
  /*! \brief the work run on the background thread */
  class Producer {
   public:
    virtual ~Producer() = default;
    /*! \brief rewind the producer */
    virtual void BeforeFirst() { NotImplemented(); }
    /*!
     * \brief produce the next cell
     * \param inout_dptr a recycled cell to reuse, or nullptr (allocate one)
     * \return false at end of data
     */
    virtual bool Next(DType** inout_dptr) = 0;
  };

  explicit ThreadedIter(size_t max_capacity = 8) : max_capacity_(max_capacity) {}
  ~ThreadedIter() override { this->Destroy(); }

  /*! \brief stop the producer thread and free every cell */
  inline void Destroy();
  /*! \brief change the queue bound (before Init) */
  inline void set_max_capacity(size_t max_capacity) { max_capacity_ = max_capacity; }
  /*! \brief start with a Producer object (optionally owning it) */
  inline void Init(Producer* producer, bool pass_ownership = false) {
    StopThread();
    producer_owned_.reset(pass_ownership ? producer : nullptr);
    Producer* p = producer;
    this->Init([p](DType** dptr) { return p->Next(dptr); },
               [p]() { p->BeforeFirst(); });
  }
  inline void Init(std::shared_ptr<Producer> producer) {
    StopThread();
    producer_shared_ = producer;
    Producer* p = producer.get();
    this->Init([p](DType** dptr) { return p->Next(dptr); },
               [p]() { p->BeforeFirst(); });
  }
  /*! \brief start with callables */
  inline void Init(std::function<bool(DType**)> next,
                   std::function<void()> beforefirst = NotImplemented);
  /*!
   * \brief take the next produced cell (blocks).  The caller owns *out_dptr
   *  until it hands it back through Recycle.
   * \return false at end of data
   */
  inline bool Next(DType** out_dptr);
  /*! \brief give a cell back for reuse; sets *inout_dptr to nullptr */
  inline void Recycle(DType** inout_dptr);
  /*! \brief rethrow an exception raised by the producer, if any */
  inline void ThrowExceptionIfSet();
  /*! \brief forget a stored producer exception */
  inline void ClearException() {
    std::lock_guard<std::mutex> lock(mutex_);
    iter_exception_ = nullptr;
  }

  // DataIter interface: Value() is valid until the next Next()/BeforeFirst()
  inline bool Next() override {
    if (out_data_ != nullptr) this->Recycle(&out_data_);
    return this->Next(&out_data_);
  }
  inline const DType& Value() const override {
    CHECK(out_data_ != nullptr) << "Calling Value at beginning or end?";
    return *out_data_;
  }
  inline void BeforeFirst() override;

 private:
  /*! \brief join the producer thread, keeping cells for reuse */
  inline void StopThread();
  inline static void NotImplemented() { LOG(FATAL) << "BeforeFirst is not supported"; }
  inline void ProducerLoop(std::function<bool(DType**)> next,
                           std::function<void()> beforefirst);

  size_t max_capacity_;
  std::unique_ptr<Producer> producer_owned_;
  std::shared_ptr<Producer> producer_shared_;
  std::unique_ptr<std::thread> producer_thread_;
  std::mutex mutex_;
  std::condition_variable producer_cond_;
  std::condition_variable consumer_cond_;
  ScopedThreadedIterState::Signal producer_sig_{ScopedThreadedIterState::kProduce};
  bool producer_sig_processed_{false};
  bool produce_end_{false};
  int nwait_consumer_{0};
  int nwait_producer_{0};
  std::deque<DType*> queue_;
  std::deque<DType*> free_cells_;
  DType* out_data_{nullptr};
  std::exception_ptr iter_exception_{nullptr};
};

// ---------------------------------------------------------------------------
template <typename DType>
inline void ThreadedIter<DType>::StopThread() {
  if (producer_thread_ != nullptr) {
    {
      std::lock_guard<std::mutex> lock(mutex_);
      producer_sig_ = ScopedThreadedIterState::kDestroy;
      producer_cond_.notify_all();
    }
    producer_thread_->join();
    producer_thread_.reset();
  }
  while (!queue_.empty()) {
    free_cells_.push_back(queue_.front());
    queue_.pop_front();
  }
}

template <typename DType>
inline void ThreadedIter<DType>::Destroy() {
  StopThread();
  for (DType* p : free_cells_) delete p;
  for (DType* p : queue_) delete p;
  free_cells_.clear();
  queue_.clear();
  delete out_data_;
  out_data_ = nullptr;
  producer_owned_.reset();
  producer_shared_.reset();
  produce_end_ = false;
  producer_sig_ = ScopedThreadedIterState::kProduce;
  iter_exception_ = nullptr;
}

template <typename DType>
inline void ThreadedIter<DType>::Init(std::function<bool(DType**)> next,
                                      std::function<void()> beforefirst) {
  // re-Init restarts the producer thread; recycled cells are kept
  StopThread();
  iter_exception_ = nullptr;
  producer_sig_ = ScopedThreadedIterState::kProduce;
  producer_sig_processed_ = false;
  produce_end_ = false;
  producer_thread_.reset(new std::thread(
      [this, next, beforefirst]() { this->ProducerLoop(next, beforefirst); }));
}

template <typename DType>
inline void ThreadedIter<DType>::ProducerLoop(std::function<bool(DType**)> next,
                                              std::function<void()> beforefirst) {
  while (true) {
    DType* cell = nullptr;
    {
      std::unique_lock<std::mutex> lock(mutex_);
      ++nwait_producer_;
      producer_cond_.wait(lock, [this]() {
        if (producer_sig_ != ScopedThreadedIterState::kProduce) return true;
        return !produce_end_ && queue_.size() < max_capacity_;
      });
      --nwait_producer_;
      if (producer_sig_ == ScopedThreadedIterState::kDestroy) return;
      if (producer_sig_ == ScopedThreadedIterState::kBeforeFirst) {
        // rewind: everything queued becomes free, then reset the producer
        while (!queue_.empty()) {
          free_cells_.push_back(queue_.front());
          queue_.pop_front();
        }
        try {
          beforefirst();
        } catch (...) {
          iter_exception_ = std::current_exception();
        }
        produce_end_ = false;
        producer_sig_ = ScopedThreadedIterState::kProduce;
        producer_sig_processed_ = true;
        consumer_cond_.notify_all();
        continue;
      }
      if (!free_cells_.empty()) {
        cell = free_cells_.front();
        free_cells_.pop_front();
      }
    }
    // produce outside the lock
    bool has_next = false;
    std::exception_ptr err = nullptr;
    try {
      has_next = next(&cell);
    } catch (...) {
      err = std::current_exception();
    }
    {
      std::lock_guard<std::mutex> lock(mutex_);
      if (err != nullptr) {
        iter_exception_ = std::move(err);  // the consumer holds the only reference
        produce_end_ = true;
        if (cell != nullptr) free_cells_.push_back(cell);
      } else if (has_next) {
        CHECK(cell != nullptr) << "Producer::Next returned true with a null cell";
        queue_.push_back(cell);
      } else {
        produce_end_ = true;
        if (cell != nullptr) free_cells_.push_back(cell);
      }
      consumer_cond_.notify_all();
    }
  }
}

template <typename DType>
inline bool ThreadedIter<DType>::Next(DType** out_dptr) {
  ThrowExceptionIfSet();
  std::unique_lock<std::mutex> lock(mutex_);
  CHECK(producer_thread_ != nullptr) << "ThreadedIter used before Init";
  ++nwait_consumer_;
  consumer_cond_.wait(lock, [this]() {
    return !queue_.empty() || produce_end_ || iter_exception_ != nullptr;
  });
  --nwait_consumer_;
  if (!queue_.empty()) {
    *out_dptr = queue_.front();
    queue_.pop_front();
    producer_cond_.notify_one();
    return true;
  }
  lock.unlock();
  ThrowExceptionIfSet();
  return false;
}

template <typename DType>
inline void ThreadedIter<DType>::Recycle(DType** inout_dptr) {
  // take the cell back BEFORE reporting a producer failure: throwing first
  // (as the reference does) leaks the cell the consumer was handing back
  {
    std::lock_guard<std::mutex> lock(mutex_);
    if (*inout_dptr != nullptr) free_cells_.push_back(*inout_dptr);
    *inout_dptr = nullptr;
    producer_cond_.notify_one();
  }
  ThrowExceptionIfSet();
}

template <typename DType>
inline void ThreadedIter<DType>::BeforeFirst() {
  ThrowExceptionIfSet();
  std::unique_lock<std::mutex> lock(mutex_);
  if (out_data_ != nullptr) {
    free_cells_.push_back(out_data_);
    out_data_ = nullptr;
  }
  if (producer_sig_ == ScopedThreadedIterState::kDestroy) return;
  producer_sig_ = ScopedThreadedIterState::kBeforeFirst;
  producer_sig_processed_ = false;
  producer_cond_.notify_all();
  consumer_cond_.wait(lock, [this]() { return producer_sig_processed_; });
  producer_sig_processed_ = false;
  lock.unlock();
  ThrowExceptionIfSet();
}

template <typename DType>
inline void ThreadedIter<DType>::ThrowExceptionIfSet() {
  std::exception_ptr err = nullptr;
  {
    std::lock_guard<std::mutex> lock(mutex_);
    err = iter_exception_;
    iter_exception_ = nullptr;
  }
  if (err != nullptr) std::rethrow_exception(err);
}

}  // namespace dmlc
#endif  // DMLC_THREADEDITER_H_
