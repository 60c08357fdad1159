/*!
 * \file dmlc/thread_local.h
 * \brief Per-thread singleton store.
 *
 * Parity: reference `include/dmlc/thread_local.h:35-80` —
 * ThreadLocalStore<T>::Get().  C++17 `thread_local` is always available with
 * our toolchains (g++ / amdclang++), so the `__thread` + registry fallback of
 * the reference is not needed; the object is destroyed at thread exit.
 */
#ifndef DMLC_THREAD_LOCAL_H_
#define DMLC_THREAD_LOCAL_H_

namespace dmlc {

template <typename T>
class ThreadLocalStore {
 public:
  /*! \brief this thread's instance (default-constructed on first use) */
  static T* Get() {
    static thread_local T inst;
    return &inst;
  }

 private:
  ThreadLocalStore() = default;
};

}  // namespace dmlc
#endif  // DMLC_THREAD_LOCAL_H_
