/*!
 * \file dmlc/thread_group.h
 * \brief Named, owned threads: ThreadGroup, BlockingQueueThread, TimerThread,
 *  ManualEvent and shared-mutex aliases.
 *
 * Parity: reference `include/dmlc/thread_group.h` — ManualEvent (:31-70),
 * SharedMutex/ReadLock/WriteLock (:72-86), ThreadGroup::Thread lifecycle with
 * names, auto-remove, request_shutdown, join and a ready/start handshake
 * (:98-304, :725-783), ThreadGroup add/remove/join_all/request_shutdown_all/
 * create/thread_by_name (:92-518), BlockingQueueThread that drains its queue
 * before quitting (:527-636), TimerThread + CreateTimer (:642-720).
 *
 * Implementation is new: each Thread owns its std::thread and a start gate;
 * an auto-remove thread unregisters itself when its body returns and, if it
 * drops the last reference from inside its own body, detaches instead of
 * self-joining.  Shutdown requests are a sticky atomic flag plus a condition
 * variable so waits (queue pops, timer sleeps) wake immediately.
 */
#ifndef DMLC_THREAD_GROUP_H_
#define DMLC_THREAD_GROUP_H_

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <utility>
#include <vector>

#include "./base.h"
#include "./logging.h"

namespace dmlc {

/*! \brief event that stays signalled until reset() */
class ManualEvent {
 public:
  ManualEvent() = default;
  /*! \brief block until signalled */
  void wait() {
    std::unique_lock<std::mutex> lock(mutex_);
    cv_.wait(lock, [this] { return signaled_; });
  }
  /*! \brief wait at most `d`; returns signalled state */
  template <typename Rep, typename Period>
  bool wait_for(const std::chrono::duration<Rep, Period>& d) {
    std::unique_lock<std::mutex> lock(mutex_);
    return cv_.wait_until(lock, SystemDeadline(d), [this] { return signaled_; });
  }

  /*!
   * \brief deadline on the system clock: waits on it use pthread_cond_timedwait,
   *  which thread sanitizers understand (steady-clock waits go through
   *  pthread_cond_clockwait, which older TSan runtimes do not intercept).
   */
  template <typename Rep, typename Period>
  static std::chrono::system_clock::time_point SystemDeadline(
      const std::chrono::duration<Rep, Period>& d) {
    return std::chrono::system_clock::now() +
           std::chrono::duration_cast<std::chrono::system_clock::duration>(d);
  }
  void signal() {
    {
      std::lock_guard<std::mutex> lock(mutex_);
      signaled_ = true;
    }
    cv_.notify_all();
  }
  void reset() {
    std::lock_guard<std::mutex> lock(mutex_);
    signaled_ = false;
  }
  bool signaled() const {
    std::lock_guard<std::mutex> lock(mutex_);
    return signaled_;
  }

 private:
  mutable std::mutex mutex_;
  std::condition_variable cv_;
  bool signaled_{false};
};

using SharedMutex = std::shared_timed_mutex;
using ReadLock = std::shared_lock<SharedMutex>;
using WriteLock = std::unique_lock<SharedMutex>;

/*! \brief a set of named threads that can be shut down and joined together */
class ThreadGroup {
 public:
  /*! \brief one managed thread */
  class Thread : public std::enable_shared_from_this<Thread> {
   public:
    using SharedPtr = std::shared_ptr<Thread>;

    Thread(std::string name, ThreadGroup* owner) : name_(std::move(name)), owner_(owner) {}
    virtual ~Thread() {
      request_shutdown();
      if (thread_.joinable()) {
        if (thread_.get_id() == std::this_thread::get_id()) {
          thread_.detach();  // last reference dropped by the thread itself
        } else {
          thread_.join();
        }
      }
    }
    DISALLOW_COPY_AND_ASSIGN(Thread);

    const char* name() const { return name_.c_str(); }
    ThreadGroup* owner() const { return owner_; }

    /*!
     * \brief start `pThis` running start_function(args...).  The body does
     *  not begin before launch() has recorded the std::thread.
     * \param auto_remove unregister from the owner when the body returns
     */
    template <typename StartFunction, typename... Args>
    static bool launch(SharedPtr pThis, bool auto_remove, StartFunction start_function,
                       Args... args) {
      CHECK(pThis != nullptr);
      CHECK(!pThis->thread_.joinable()) << "thread " << pThis->name_ << " already launched";
      pThis->auto_remove_ = auto_remove;
      Thread* self = pThis.get();
      // the body keeps the object alive while it runs
      self->thread_ = std::thread([pThis, start_function, args...]() mutable {
        pThis->started_.wait();
        try {
          start_function(args...);
        } catch (const std::exception& e) {
          LOG(WARNING) << "thread " << pThis->name_ << " exited with: " << e.what();
        }
        pThis->has_exited_.store(true);
        if (pThis->auto_remove_ && pThis->owner_ != nullptr) {
          pThis->owner_->remove_thread(pThis);
        }
        pThis.reset();
      });
      self->started_.signal();
      return true;
    }

    bool is_current_thread() const { return thread_.get_id() == std::this_thread::get_id(); }
    /*! \brief ask the body to stop (it polls is_shutdown_requested) */
    virtual void request_shutdown() { shutdown_requested_.store(true); }
    virtual bool is_shutdown_requested() const { return shutdown_requested_.load(); }
    bool is_auto_remove() const { return auto_remove_; }
    /*! \brief turn off auto-remove so the owner can join this thread */
    void make_joinable() { auto_remove_ = false; }
    bool joinable() const { return thread_.joinable(); }
    bool has_exited() const { return has_exited_.load(); }
    void join() {
      if (thread_.joinable() && !is_current_thread()) thread_.join();
    }
    std::thread::id get_id() const { return thread_.get_id(); }

   private:
    std::string name_;
    ThreadGroup* owner_;
    std::thread thread_;
    ManualEvent started_;
    std::atomic<bool> shutdown_requested_{false};
    std::atomic<bool> has_exited_{false};
    bool auto_remove_{false};
  };

  ThreadGroup() = default;
  virtual ~ThreadGroup() {
    request_shutdown_all();
    join_all();
  }
  DISALLOW_COPY_AND_ASSIGN(ThreadGroup);

  /*! \brief whether `thread` is a member */
  bool is_this_thread_in() const {
    ReadLock lock(mutex_);
    for (auto& t : threads_) {
      if (t->is_current_thread()) return true;
    }
    return false;
  }
  bool add_thread(Thread::SharedPtr thread) {
    if (thread == nullptr) return false;
    WriteLock lock(mutex_);
    return threads_.insert(std::move(thread)).second;
  }
  bool remove_thread(const Thread::SharedPtr& thread) {
    Thread::SharedPtr keep;  // destroyed after the lock is released
    WriteLock lock(mutex_);
    auto it = threads_.find(thread);
    if (it == threads_.end()) return false;
    keep = *it;
    threads_.erase(it);
    lock.unlock();
    return true;
  }
  /*! \brief join every member (auto-remove members are waited for too) */
  void join_all() {
    CHECK(!is_this_thread_in()) << "join_all called from a member thread";
    for (;;) {
      std::vector<Thread::SharedPtr> snapshot;
      {
        ReadLock lock(mutex_);
        snapshot.assign(threads_.begin(), threads_.end());
      }
      if (snapshot.empty()) return;
      for (auto& t : snapshot) {
        t->join();
        remove_thread(t);
      }
    }
  }
  void request_shutdown_all(bool make_all_joinable = true) {
    ReadLock lock(mutex_);
    for (auto& t : threads_) {
      if (make_all_joinable) t->make_joinable();
      t->request_shutdown();
    }
  }
  size_t size() const {
    ReadLock lock(mutex_);
    return threads_.size();
  }
  bool empty() const { return size() == 0; }
  Thread::SharedPtr thread_by_name(const std::string& name) const {
    ReadLock lock(mutex_);
    for (auto& t : threads_) {
      if (name == t->name()) return t;
    }
    return nullptr;
  }
  /*! \brief create, register and launch a plain thread running fn(args...) */
  template <typename StartFunction, typename... Args>
  Thread::SharedPtr create(const std::string& name, bool auto_remove, StartFunction fn,
                           Args... args) {
    auto t = std::make_shared<Thread>(name, this);
    add_thread(t);
    Thread::launch(t, auto_remove, fn, args...);
    return t;
  }

 private:
  mutable SharedMutex mutex_;
  std::unordered_set<Thread::SharedPtr> threads_;
};

/*!
 * \brief thread that feeds queued items to a handler; on shutdown it first
 *  drains what is already queued (reference `thread_group.h:527-636`).
 */
template <typename ObjectType>
class BlockingQueueThread : public ThreadGroup::Thread {
 public:
  using Handler = std::function<int(ObjectType)>;

  BlockingQueueThread(const std::string& name, ThreadGroup* owner)
      : ThreadGroup::Thread(name, owner) {}
  ~BlockingQueueThread() override {
    request_shutdown();
    join();
  }
  void request_shutdown() override {
    ThreadGroup::Thread::request_shutdown();
    std::lock_guard<std::mutex> lock(mutex_);
    cv_.notify_all();
  }
  void enqueue(ObjectType item) {
    {
      std::lock_guard<std::mutex> lock(mutex_);
      queue_.push_back(std::move(item));
    }
    cv_.notify_one();
  }
  size_t size_approx() const {
    std::lock_guard<std::mutex> lock(mutex_);
    return queue_.size();
  }
  /*!
   * \brief launch; handler(item) != 0 stops the thread early
   */
  static bool start(std::shared_ptr<BlockingQueueThread> pThis, Handler handler) {
    BlockingQueueThread* self = pThis.get();
    return ThreadGroup::Thread::launch(pThis, false, [self, handler]() { self->Run(handler); });
  }

 private:
  void Run(const Handler& handler) {
    for (;;) {
      ObjectType item;
      {
        std::unique_lock<std::mutex> lock(mutex_);
        cv_.wait(lock, [this] { return !queue_.empty() || is_shutdown_requested(); });
        if (queue_.empty()) return;  // shutdown requested and drained
        item = std::move(queue_.front());
        queue_.pop_front();
      }
      if (handler(std::move(item)) != 0) return;
    }
  }
  mutable std::mutex mutex_;
  std::condition_variable cv_;
  std::deque<ObjectType> queue_;
};

/*!
 * \brief thread that calls on_timer() every `duration` until shutdown or
 *  until on_timer returns non-zero (reference `thread_group.h:642-720`).
 */
template <typename Duration = std::chrono::milliseconds>
class TimerThread : public ThreadGroup::Thread {
 public:
  TimerThread(const std::string& name, ThreadGroup* owner) : ThreadGroup::Thread(name, owner) {}
  ~TimerThread() override {
    request_shutdown();
    join();
  }
  void request_shutdown() override {
    ThreadGroup::Thread::request_shutdown();
    std::lock_guard<std::mutex> lock(mutex_);
    cv_.notify_all();
  }
  static bool start(std::shared_ptr<TimerThread> pThis, Duration duration,
                    std::function<int()> on_timer) {
    TimerThread* self = pThis.get();
    return ThreadGroup::Thread::launch(pThis, false, [self, duration, on_timer]() {
      auto next = std::chrono::steady_clock::now() + duration;
      for (;;) {
        {
          std::unique_lock<std::mutex> lock(self->mutex_);
          auto deadline = ManualEvent::SystemDeadline(next - std::chrono::steady_clock::now());
          if (self->cv_.wait_until(lock, deadline,
                                   [self] { return self->is_shutdown_requested(); }))
            return;
        }
        if (on_timer() != 0) return;
        next += duration;  // fixed-rate schedule: no drift from handler time
        auto now = std::chrono::steady_clock::now();
        if (next < now) next = now;
      }
    });
  }

 private:
  std::mutex mutex_;
  std::condition_variable cv_;
};

/*! \brief create + register + start a timer thread in `owner` */
template <typename Duration>
inline std::shared_ptr<TimerThread<Duration>> CreateTimer(const std::string& name,
                                                          Duration duration, ThreadGroup* owner,
                                                          std::function<int()> on_timer) {
  auto t = std::make_shared<TimerThread<Duration>>(name, owner);
  owner->add_thread(t);
  TimerThread<Duration>::start(t, duration, std::move(on_timer));
  return t;
}

}  // namespace dmlc
#endif  // DMLC_THREAD_GROUP_H_
