/*!
 * \file dmlc/memory.h
 * \brief Fixed-size object pool, thread-local allocator and a thread-local
 *  (non-atomic) shared pointer.
 *
 * Parity: reference `include/dmlc/memory.h` — MemoryPool<size, align> with
 * 4 MiB pages and a free list (:22-77), ThreadlocalAllocator<T> (n == 1 only)
 * (:85-121), ThreadlocalSharedPtr<T> with a non-atomic reference count
 * (:132-256).
 *
 * The pinned-host / device slab pools used by the GPU pipeline live in
 * `dmlc/gpu/memory_pool.h`; this header stays CPU-only.
 */
#ifndef DMLC_MEMORY_H_
#define DMLC_MEMORY_H_

#include <cstddef>
#include <cstdlib>
#include <new>
#include <utility>
#include <vector>

#include "./logging.h"
#include "./thread_local.h"

namespace dmlc {

/*!
 * \brief pool of `size`-byte blocks aligned to `align`, carved from 4 MiB
 *  pages; freed blocks go on an intrusive free list.  Not thread-safe (use one
 *  pool per thread, see ThreadlocalAllocator).
 */
template <size_t size, size_t align>
class MemoryPool {
 public:
  static_assert(align != 0 && (align & (align - 1)) == 0, "align must be a power of 2");
  static constexpr size_t kBlock = ((size < sizeof(void*) ? sizeof(void*) : size) + align - 1) /
                                   align * align;
  static constexpr size_t kPageSize = 1UL << 22;
  static_assert(kBlock <= kPageSize, "block larger than a pool page");

  MemoryPool() = default;
  ~MemoryPool() {
    for (void* p : pages_) std::free(p);
  }
  MemoryPool(const MemoryPool&) = delete;
  MemoryPool& operator=(const MemoryPool&) = delete;

  /*! \brief one block */
  void* allocate() {
    if (free_ != nullptr) {
      FreeNode* n = free_;
      free_ = n->next;
      return n;
    }
    if (cursor_ + kBlock > page_end_) NewPage();
    void* p = cursor_;
    cursor_ += kBlock;
    return p;
  }
  /*! \brief return a block obtained from allocate() */
  void deallocate(void* p) {
    FreeNode* n = static_cast<FreeNode*>(p);
    n->next = free_;
    free_ = n;
  }
  size_t num_pages() const { return pages_.size(); }

 private:
  struct FreeNode {
    FreeNode* next;
  };
  void NewPage() {
    void* page = std::aligned_alloc(align < alignof(std::max_align_t) ? alignof(std::max_align_t)
                                                                      : align,
                                    kPageSize);
    if (page == nullptr) throw std::bad_alloc();
    pages_.push_back(page);
    cursor_ = static_cast<char*>(page);
    page_end_ = cursor_ + kPageSize;
  }
  FreeNode* free_{nullptr};
  char* cursor_{nullptr};
  char* page_end_{nullptr};
  std::vector<void*> pages_;
};

/*!
 * \brief allocator of single objects from a per-thread MemoryPool.  Only
 *  n == 1 is supported, like the reference; memory must be freed on the
 *  thread that allocated it.
 */
template <typename T>
class ThreadlocalAllocator {
 public:
  using pointer = T*;
  using const_pointer = const T*;
  using value_type = T;

  ThreadlocalAllocator() = default;
  template <typename U>
  ThreadlocalAllocator(const ThreadlocalAllocator<U>&) {}  // NOLINT(runtime/explicit)
  template <typename U>
  struct rebind {
    using other = ThreadlocalAllocator<U>;
  };

  T* allocate(size_t n) {
    CHECK_EQ(n, 1U) << "ThreadlocalAllocator can only allocate one object";
    return static_cast<T*>(Pool()->allocate());
  }
  void deallocate(T* p, size_t n) {
    CHECK_EQ(n, 1U) << "ThreadlocalAllocator can only free one object";
    Pool()->deallocate(p);
  }
  bool operator==(const ThreadlocalAllocator&) const { return true; }
  bool operator!=(const ThreadlocalAllocator&) const { return false; }

 private:
  using PoolT = MemoryPool<sizeof(T), alignof(T)>;
  static PoolT* Pool() { return ThreadLocalStore<PoolT>::Get(); }
};

/*!
 * \brief shared pointer with a plain (non-atomic) reference count whose
 *  control block + object come from ThreadlocalAllocator in one block.
 *  All copies must stay on the creating thread.
 */
template <typename T>
class ThreadlocalSharedPtr {
 public:
  ThreadlocalSharedPtr() noexcept = default;
  ThreadlocalSharedPtr(std::nullptr_t) noexcept {}  // NOLINT(runtime/explicit)
  ThreadlocalSharedPtr(const ThreadlocalSharedPtr& o) noexcept : block_(o.block_) {
    if (block_ != nullptr) ++block_->ref;
  }
  ThreadlocalSharedPtr(ThreadlocalSharedPtr&& o) noexcept : block_(o.block_) { o.block_ = nullptr; }
  ~ThreadlocalSharedPtr() { DecRef(); }
  ThreadlocalSharedPtr& operator=(ThreadlocalSharedPtr o) noexcept {
    std::swap(block_, o.block_);
    return *this;
  }

  /*! \brief construct a new object */
  template <typename... Args>
  static ThreadlocalSharedPtr<T> Create(Args&&... args) {
    ThreadlocalAllocator<Block> alloc;
    Block* b = alloc.allocate(1);
    try {
      new (b) Block(std::forward<Args>(args)...);
    } catch (...) {
      alloc.deallocate(b, 1);
      throw;
    }
    ThreadlocalSharedPtr<T> p;
    p.block_ = b;
    return p;
  }
  T* get() const { return block_ == nullptr ? nullptr : &block_->data; }
  T& operator*() const { return *get(); }
  T* operator->() const { return get(); }
  explicit operator bool() const { return block_ != nullptr; }
  size_t use_count() const { return block_ == nullptr ? 0 : block_->ref; }
  void reset() {
    DecRef();
    block_ = nullptr;
  }
  bool operator==(std::nullptr_t) const { return block_ == nullptr; }
  bool operator!=(std::nullptr_t) const { return block_ != nullptr; }

 private:
  struct Block {
    template <typename... Args>
    explicit Block(Args&&... args) : data(std::forward<Args>(args)...) {}
    size_t ref{1};
    T data;
  };
  void DecRef() {
    if (block_ != nullptr && --block_->ref == 0) {
      block_->~Block();
      ThreadlocalAllocator<Block>().deallocate(block_, 1);
    }
  }
  Block* block_{nullptr};
};

}  // namespace dmlc
#endif  // DMLC_MEMORY_H_
