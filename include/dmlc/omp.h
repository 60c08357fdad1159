/*!
 * \file dmlc/omp.h
 * \brief OpenMP header with single-thread fallbacks.
 * Parity: reference `include/dmlc/omp.h:6-36`.
 */
#ifndef DMLC_OMP_H_
#define DMLC_OMP_H_

#if defined(_OPENMP)
#include <omp.h>
#else
inline int omp_get_thread_num() { return 0; }
inline int omp_get_num_threads() { return 1; }
inline int omp_get_max_threads() { return 1; }
inline int omp_get_num_procs() { return 1; }
inline void omp_set_num_threads(int) {}
#endif

namespace dmlc {
using omp_uint = unsigned;   // NOLINT
using omp_ulong = unsigned long;  // NOLINT
}  // namespace dmlc
#endif  // DMLC_OMP_H_
