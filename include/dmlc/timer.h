/*!
 * \file dmlc/timer.h
 * \brief Monotonic wall clock.  Parity: reference `include/dmlc/timer.h:27-47`.
 */
#ifndef DMLC_TIMER_H_
#define DMLC_TIMER_H_

#include <chrono>

namespace dmlc {
/*! \brief seconds since an arbitrary epoch (steady clock, ns resolution) */
inline double GetTime() {
  return std::chrono::duration<double>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace dmlc
#endif  // DMLC_TIMER_H_
