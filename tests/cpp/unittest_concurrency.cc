// L2 unit tests: the behaviours pinned by the reference's
// test/unittest/unittest_{lockfree,thread_group,threaditer,
// threaditer_exc_handling}.cc, plus the blocking queue and the
// memory pool.  These are also the TSan targets (make tsan).
#include <dmlc/blockingconcurrentqueue.h>
#include <dmlc/concurrency.h>
#include <dmlc/concurrentqueue.h>
#include <dmlc/memory.h>
#include <dmlc/thread_group.h>
#include <dmlc/thread_local.h>
#include <dmlc/threadediter.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <numeric>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "./testing.h"

// ---------------------------------------------------------------- lock-free queue
TEST(LockFree, ManyProducersManyConsumersExactlyOnce) {
  dmlc::ConcurrentQueue<int64_t> q;
  constexpr int kProducers = 16, kConsumers = 16, kPer = 20000;
  std::atomic<int64_t> sum{0}, count{0};
  std::atomic<int> producers_done{0};
  std::vector<std::thread> th;
  for (int p = 0; p < kProducers; ++p) {
    th.emplace_back([&, p] {
      for (int i = 0; i < kPer; ++i) q.enqueue(int64_t(p) * kPer + i);
      producers_done.fetch_add(1);
    });
  }
  for (int c = 0; c < kConsumers; ++c) {
    th.emplace_back([&] {
      int64_t v;
      for (;;) {
        if (q.try_dequeue(v)) {
          sum.fetch_add(v);
          count.fetch_add(1);
        } else if (producers_done.load() == kProducers && q.size_approx() == 0) {
          if (!q.try_dequeue(v)) return;
          sum.fetch_add(v);
          count.fetch_add(1);
        }
      }
    });
  }
  for (auto& t : th) t.join();
  const int64_t n = int64_t(kProducers) * kPer;
  EXPECT_EQ(count.load(), n);
  EXPECT_EQ(sum.load(), n * (n - 1) / 2);
  EXPECT_EQ(q.size_approx(), 0U);
  EXPECT_TRUE(q.is_lock_free());
}

TEST(LockFree, PerProducerFifoAndBulk) {
  dmlc::ConcurrentQueue<std::string> q(0);
  dmlc::ProducerToken tok(q);
  std::vector<std::string> in;
  for (int i = 0; i < 3000; ++i) in.push_back(std::to_string(i));
  EXPECT_TRUE(q.enqueue_bulk(tok, in.begin(), in.size()));
  EXPECT_EQ(q.size_approx(), 3000U);
  std::vector<std::string> out(5000);
  dmlc::ConsumerToken ctok(q);
  size_t n = q.try_dequeue_bulk(ctok, out.begin(), out.size());
  ASSERT_EQ(n, 3000U);
  out.resize(n);
  EXPECT_TRUE(out == in);
  std::string s;
  EXPECT_FALSE(q.try_dequeue(s));
}

TEST(LockFree, TryEnqueueDoesNotAllocate) {
  dmlc::ConcurrentQueue<int> q(0);  // one segment, no spares
  size_t ok = 0;
  while (q.try_enqueue(1)) ++ok;
  EXPECT_EQ(ok, dmlc::ConcurrentQueue<int>::kCells);
  EXPECT_TRUE(q.enqueue(2));  // enqueue may allocate
}

TEST(LockFree, DestructorReleasesQueuedObjects) {
  auto tracker = std::make_shared<int>(0);
  {
    dmlc::ConcurrentQueue<std::shared_ptr<int>> q;
    for (int i = 0; i < 2000; ++i) q.enqueue(tracker);
    std::shared_ptr<int> x;
    for (int i = 0; i < 700; ++i) q.try_dequeue(x);
    EXPECT_EQ(tracker.use_count(), 1 + 1300 + 1);
  }
  EXPECT_EQ(tracker.use_count(), 1);
}

TEST(LockFree, BlockingQueueWaitAndTimeout) {
  dmlc::BlockingConcurrentQueue<int> q;
  int v = 0;
  auto t0 = std::chrono::steady_clock::now();
  EXPECT_FALSE(q.wait_dequeue_timed(v, 20000));
  auto waited = std::chrono::steady_clock::now() - t0;
  EXPECT_GE(std::chrono::duration_cast<std::chrono::milliseconds>(waited).count(), 15);
  constexpr int kProducers = 8, kPer = 5000;
  std::atomic<int64_t> sum{0};
  std::vector<std::thread> th;
  for (int c = 0; c < 4; ++c) {
    th.emplace_back([&] {
      int x;
      for (;;) {
        q.wait_dequeue(x);
        if (x < 0) return;
        sum.fetch_add(x);
      }
    });
  }
  std::vector<std::thread> prod;
  for (int p = 0; p < kProducers; ++p) {
    prod.emplace_back([&] {
      for (int i = 1; i <= kPer; ++i) q.enqueue(i);
    });
  }
  for (auto& t : prod) t.join();
  for (int c = 0; c < 4; ++c) q.enqueue(-1);
  for (auto& t : th) t.join();
  EXPECT_EQ(sum.load(), int64_t(kProducers) * kPer * (kPer + 1) / 2);
  std::vector<int> batch{1, 2, 3};
  q.enqueue_bulk(batch.begin(), batch.size());
  std::vector<int> got(8);
  EXPECT_EQ(q.wait_dequeue_bulk(got.begin(), got.size()), 3U);
}

// ---------------------------------------------------------------- blocking queue
TEST(Concurrency, BlockingQueueFifoPriorityKill) {
  dmlc::ConcurrentBlockingQueue<int> q;
  q.Push(1);
  q.Push(2);
  q.PushFront(0);
  int v;
  ASSERT_TRUE(q.Pop(&v));
  EXPECT_EQ(v, 0);
  EXPECT_EQ(q.Size(), 2U);
  dmlc::ConcurrentBlockingQueue<int, dmlc::ConcurrentQueueType::kPriority> pq;
  pq.Push(10, 1);
  pq.Push(20, 5);
  pq.Push(30, 5);
  ASSERT_TRUE(pq.Pop(&v));
  EXPECT_EQ(v, 20);  // highest priority, FIFO among equals
  ASSERT_TRUE(pq.Pop(&v));
  EXPECT_EQ(v, 30);
  dmlc::ConcurrentBlockingQueue<int> empty;
  std::thread waiter([&] {
    int x;
    EXPECT_FALSE(empty.Pop(&x));
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  empty.SignalForKill();
  waiter.join();
  dmlc::Spinlock lock;
  int counter = 0;
  std::vector<std::thread> th;
  for (int i = 0; i < 8; ++i) {
    th.emplace_back([&] {
      for (int k = 0; k < 10000; ++k) {
        std::lock_guard<dmlc::Spinlock> g(lock);
        ++counter;
      }
    });
  }
  for (auto& t : th) t.join();
  EXPECT_EQ(counter, 80000);
}

// ---------------------------------------------------------------- thread group
TEST(ThreadGroup, AutoRemoveAndJoinable) {
  dmlc::ThreadGroup group;
  std::atomic<int> ran{0};
  for (int i = 0; i < 200; ++i) {
    group.create("auto" + std::to_string(i), true, [&ran] { ran.fetch_add(1); });
  }
  for (int i = 0; i < 200 && !group.empty(); ++i) {
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  group.join_all();
  EXPECT_EQ(ran.load(), 200);
  EXPECT_TRUE(group.empty());

  std::atomic<int> stopped{0};
  for (int i = 0; i < 50; ++i) {
    auto t = std::make_shared<dmlc::ThreadGroup::Thread>("j" + std::to_string(i), &group);
    group.add_thread(t);
    dmlc::ThreadGroup::Thread* raw = t.get();
    dmlc::ThreadGroup::Thread::launch(t, false, [raw, &stopped] {
      while (!raw->is_shutdown_requested()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      stopped.fetch_add(1);
    });
  }
  EXPECT_EQ(group.size(), 50U);
  EXPECT_TRUE(group.thread_by_name("j7") != nullptr);
  EXPECT_TRUE(group.thread_by_name("nope") == nullptr);
  group.request_shutdown_all();
  group.join_all();
  EXPECT_EQ(stopped.load(), 50);
}

TEST(ThreadGroup, BlockingQueueThreadDrainsBeforeQuit) {
  dmlc::ThreadGroup group;
  auto q = std::make_shared<dmlc::BlockingQueueThread<int>>("queue", &group);
  group.add_thread(q);
  std::atomic<int> handled{0};
  for (int i = 0; i < 500; ++i) q->enqueue(i);
  dmlc::BlockingQueueThread<int>::start(q, [&handled](int) {
    std::this_thread::sleep_for(std::chrono::microseconds(10));
    handled.fetch_add(1);
    return 0;
  });
  q->request_shutdown();
  group.join_all();
  EXPECT_EQ(handled.load(), 500);
}

TEST(ThreadGroup, TimerPeriod) {
  dmlc::ThreadGroup group;
  std::atomic<int> ticks{0};
  auto timer = dmlc::CreateTimer("timer", std::chrono::milliseconds(5), &group, [&ticks] {
    ticks.fetch_add(1);
    return 0;
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(500));
  timer->request_shutdown();
  group.join_all();
  // reference bounds: 10..150 ticks in 500 ms at a 5 ms period
  EXPECT_GE(ticks.load(), 10);
  EXPECT_LE(ticks.load(), 150);
  dmlc::ManualEvent ev;
  EXPECT_FALSE(ev.wait_for(std::chrono::milliseconds(1)));
  ev.signal();
  ev.wait();
  EXPECT_TRUE(ev.signaled());
  ev.reset();
  EXPECT_FALSE(ev.signaled());
}

// ---------------------------------------------------------------- threaded iter
struct IntProducer : public dmlc::ThreadedIter<int>::Producer {
  int counter{0}, maxcap;
  explicit IntProducer(int maxcap) : maxcap(maxcap) {}
  void BeforeFirst() override { counter = 0; }
  bool Next(int** inout) override {
    if (counter == maxcap) return false;
    if (*inout == nullptr) *inout = new int();
    **inout = counter++;
    return true;
  }
};

TEST(ThreadedIter, CapacityOneRepeatedBeforeFirst) {
  dmlc::ThreadedIter<int> iter(1);
  iter.Init(new IntProducer(100), true);
  for (int epoch = 0; epoch < 5; ++epoch) {
    int expect = 0;
    int* v = nullptr;
    while (iter.Next(&v)) {
      EXPECT_EQ(*v, expect++);
      iter.Recycle(&v);
      EXPECT_TRUE(v == nullptr);
      if (epoch == 2 && expect == 37) break;  // rewind mid-epoch
    }
    if (epoch != 2) EXPECT_EQ(expect, 100);
    iter.BeforeFirst();
  }
  // DataIter adapter
  int total = 0;
  while (iter.Next()) total += iter.Value();
  EXPECT_EQ(total, 99 * 100 / 2);
}

struct ThrowingProducer : public dmlc::ThreadedIter<int>::Producer {
  int counter{0};
  bool throw_in_next, throw_in_before_first;
  ThrowingProducer(bool n, bool b) : throw_in_next(n), throw_in_before_first(b) {}
  void BeforeFirst() override {
    counter = 0;
    if (throw_in_before_first) LOG(FATAL) << "BeforeFirst failure";
  }
  bool Next(int** inout) override {
    if (throw_in_next && counter == 5) LOG(FATAL) << "Next failure";
    if (counter == 10) return false;
    if (*inout == nullptr) *inout = new int();
    **inout = counter++;
    return true;
  }
};

TEST(ThreadedIter, ExceptionInNextReachesConsumer) {
  dmlc::ThreadedIter<int> iter(2);
  iter.Init(std::make_shared<ThrowingProducer>(true, false));
  bool caught = false;
  try {
    int* v = nullptr;
    while (iter.Next(&v)) iter.Recycle(&v);
  } catch (const dmlc::Error& e) {
    caught = std::string(e.what()).find("Next failure") != std::string::npos;
  }
  EXPECT_TRUE(caught);
}

TEST(ThreadedIter, ExceptionInBeforeFirstReachesConsumer) {
  dmlc::ThreadedIter<int> iter(2);
  iter.Init(std::make_shared<ThrowingProducer>(false, true));
  int* v = nullptr;
  while (iter.Next(&v)) iter.Recycle(&v);
  bool caught = false;
  try {
    iter.BeforeFirst();
    while (iter.Next(&v)) iter.Recycle(&v);
  } catch (const dmlc::Error&) {
    caught = true;
  }
  EXPECT_TRUE(caught);
}

// ---------------------------------------------------------------- memory
TEST(Memory, PoolReusesBlocks) {
  dmlc::MemoryPool<24, 16> pool;
  std::set<void*> seen;
  std::vector<void*> blocks;
  for (int i = 0; i < 10000; ++i) {
    void* p = pool.allocate();
    EXPECT_EQ(reinterpret_cast<uintptr_t>(p) % 16, 0U);
    blocks.push_back(p);
    seen.insert(p);
  }
  EXPECT_EQ(seen.size(), 10000U);
  for (void* p : blocks) pool.deallocate(p);
  size_t pages = pool.num_pages();
  for (int i = 0; i < 10000; ++i) pool.allocate();
  EXPECT_EQ(pool.num_pages(), pages);
}

TEST(Memory, ThreadlocalSharedPtr) {
  struct Obj {
    int v;
    explicit Obj(int v) : v(v) {}
  };
  auto p = dmlc::ThreadlocalSharedPtr<Obj>::Create(5);
  EXPECT_EQ(p->v, 5);
  {
    auto q = p;
    EXPECT_EQ(p.use_count(), 2U);
    q->v = 6;
  }
  EXPECT_EQ(p.use_count(), 1U);
  EXPECT_EQ((*p).v, 6);
  p.reset();
  EXPECT_TRUE(p == nullptr);
  int* a = dmlc::ThreadlocalAllocator<int>().allocate(1);
  *a = 3;
  dmlc::ThreadlocalAllocator<int>().deallocate(a, 1);
  EXPECT_THROW(dmlc::ThreadlocalAllocator<int>().allocate(2), dmlc::Error);
  std::atomic<int> distinct{0};
  int* main_ptr = dmlc::ThreadLocalStore<int>::Get();
  std::thread t([&] { distinct = dmlc::ThreadLocalStore<int>::Get() != main_ptr; });
  t.join();
  EXPECT_EQ(distinct.load(), 1);
}
