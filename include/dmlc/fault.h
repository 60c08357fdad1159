/*!
 * \file dmlc/fault.h
 * \brief Deterministic fault injection for the ingestion pipeline and the
 *  distributed runtime (SURVEY §5.3 design: `DMLC_FAULT_INJECT=stage:count`).
 *
 * The reference injects faults only inside unit tests, with throwing
 * producers (`test/unittest/unittest_threaditer_exc_handling.cc:20-50`).
 * Here every pipeline stage carries a named fault point, so a test (or an
 * operator rehearsing failure handling on a real job) can make exactly the
 * k-th pass through a stage fail:
 *
 *   DMLC_FAULT_INJECT="read:3,h2d:1"   # 3rd reader fill and 1st H2D copy fail
 *
 * Points: read (host reader fill / zero-copy piece), h2d (host->device copy),
 * parse (GPU parse of a chunk, before it starts), parse_fill (after the
 * chunk's kernels ran, before it is delivered), recordio (GPU RecordIO chunk), http (one
 * ranged GET returns nothing -> exercises the retry loop), tracker (tracker
 * connection).  A fault is a dmlc::Error thrown from that stage ("http" is
 * soft: a transient failure the caller retries).  Off (one relaxed atomic
 * load per point) when the variable is unset.
 */
#ifndef DMLC_FAULT_H_
#define DMLC_FAULT_H_

#include <dmlc/logging.h>

#include <atomic>
#include <string>

namespace dmlc {
namespace fault {

/*! \brief true when any fault is armed (env or Configure) */
bool Enabled();
/*! \brief count one pass through `point`; true if this pass must fail */
bool Hit(const char* point);
/*! \brief replace the armed faults ("" disarms everything); resets counters */
void Configure(const std::string& spec);
/*! \brief passes through `point` since the last Configure */
long Count(const std::string& point);

}  // namespace fault
}  // namespace dmlc

/*! \brief throw dmlc::Error when the armed fault of `point` fires */
#define DMLC_FAULT_POINT(point)                                                       \
  do {                                                                                \
    if (::dmlc::fault::Enabled() && ::dmlc::fault::Hit(point)) {                      \
      LOG(FATAL) << "injected fault at \"" << (point) << "\" (DMLC_FAULT_INJECT)";    \
    }                                                                                 \
  } while (0)

/*! \brief true when the armed fault of `point` fires (caller simulates a soft failure) */
#define DMLC_FAULT_SOFT(point) (::dmlc::fault::Enabled() && ::dmlc::fault::Hit(point))

#endif  // DMLC_FAULT_H_
