/*!
 * \file src/gpu/host_wait.h
 * \brief Host side of the "kernel raises a flag in mapped pinned memory"
 *  handshake the GPU pipelines use instead of a blocking stream synchronise
 *  per chunk.
 *
 *  A chunk's metadata wait has two very different lengths: a few microseconds
 *  when the kernel is already done (the fill after a scan), or a whole PCIe
 *  transfer (~1 ms per 64 MiB) when the kernel still waits for its H2D copy.
 *  Spinning through the long case would burn one core per rank -- 8 cores on
 *  an 8-GPU node, on the NUMA nodes whose cores also run the pread / window
 *  registration threads.  So: spin (with `pause`) for `spin_us`, then poll
 *  with short sleeps (timer slack lowered to 1 us for this thread, so a
 *  5 us nap costs ~5-7 us, not the default 50 us slack: the wake-up latency
 *  sits between a kernel finishing and the next launch), and give up after
 *  `bound_s` so a kernel that never publishes surfaces through the caller's
 *  stream synchronise instead of hanging here.
 */
#ifndef DMLC_SRC_GPU_HOST_WAIT_H_
#define DMLC_SRC_GPU_HOST_WAIT_H_

#include <sys/prctl.h>
#include <time.h>

#include <cstdint>

#include <dmlc/timer.h>

namespace dmlc {
namespace gpu {

struct HostWaitStats {
  /*! \brief waits that ended in the spin phase / in the sleep phase / timed out */
  uint64_t spun{0}, slept{0}, timed_out{0};
};

inline void CpuRelax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}

/*!
 * \brief wait until *flag != 0; true if seen, false after bound_s
 * \param spin_us busy-poll budget before the sleep phase (0: sleep at once)
 */
inline bool WaitHostFlag(const volatile unsigned* flag, double spin_us, double bound_s,
                         HostWaitStats* st) {
  const double t0 = GetTime();
  const double spin_end = t0 + spin_us * 1e-6;
  for (uint32_t i = 0;; ++i) {
    if (*flag != 0) {
      ++st->spun;
      return true;
    }
    CpuRelax();
    if ((i & 63u) == 63u && GetTime() >= spin_end) break;
  }
  // a tight timer slack for the sleep phase only: the caller's thread (often
  // the training loop) gets its own slack back before we return
  const int old_slack = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
  (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1 us
  struct Restore {
    int v;
    ~Restore() {
      if (v > 0) (void)prctl(PR_SET_TIMERSLACK, static_cast<unsigned long>(v), 0, 0, 0);
    }
  } restore{old_slack};
  const struct timespec nap = {0, 5000};  // 5 us
  for (;;) {
    if (*flag != 0) {
      ++st->slept;
      return true;
    }
    if (GetTime() - t0 > bound_s) {
      ++st->timed_out;
      return false;
    }
    nanosleep(&nap, nullptr);
  }
}

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_SRC_GPU_HOST_WAIT_H_
