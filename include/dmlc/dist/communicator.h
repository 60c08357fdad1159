/*!
 * \file dmlc/dist/communicator.h
 * \brief RCCL communicator: one process = one MI355X = one rank.
 *
 * The reference has no data-plane collectives; this is the
 * MI355X-native communication backend of §5.8: ncclUniqueId distributed by
 * the tracker, `hipSetDevice(local index)`, one communicator per process,
 * and the collectives of the §2.12 call-site table (control all-reduces,
 * all-gather of per-rank counts, broadcast of configs, gradient all-reduce,
 * grouped send/recv all-to-all-v for a global row shuffle).
 *
 * RCCL is resolved at run time: if the process already has an RCCL loaded
 * (PyTorch-ROCm bundles one) that copy is reused, otherwise
 * /opt/rocm/lib/librccl.so.1 is opened -- so a Python process never ends up
 * with two RCCL runtimes fighting over the same GPUs.
 *
 * Sizing for xGMI: each MI355X has 7 point-to-point links
 * (~153 GB/s each); a ring all-reduce is per-link bound, so callers batch
 * small control values into one message and keep gradient buckets large.
 */
#ifndef DMLC_DIST_COMMUNICATOR_H_
#define DMLC_DIST_COMMUNICATOR_H_

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <atomic>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

namespace dmlc {
namespace dist {

class TrackerClient;

enum class DataType : int {
  kInt8 = 0, kUInt8 = 1, kInt32 = 2, kUInt32 = 3, kInt64 = 4, kUInt64 = 5,
  kFloat16 = 6, kFloat32 = 7, kFloat64 = 8, kBFloat16 = 9
};
enum class ReduceOp : int { kSum = 0, kProd = 1, kMax = 2, kMin = 3, kAvg = 4 };

size_t DataTypeSize(DataType t);

class Communicator {
 public:
  static constexpr size_t kUniqueIdBytes = 128;
  /*! \brief whether an RCCL library can be loaded in this process */
  static bool Available();
  /*! \brief file the RCCL entry points were resolved from ("" if none) */
  static std::string LibraryPath();
  /*! \brief fresh ncclUniqueId bytes (call on rank 0 only) */
  static std::string NewUniqueId();
  /*!
   * \brief collective constructor: every rank calls it with the same id
   * \param device HIP device of this rank (its local index on the node)
   */
  Communicator(int rank, int world_size, int device, const std::string& unique_id);
  /*! \brief rank / world from the tracker; id exchanged through it */
  static std::unique_ptr<Communicator> FromTracker(TrackerClient* tracker, int device,
                                                   const std::string& key = "world");
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  int rank() const { return rank_; }
  int world_size() const { return world_; }
  int device() const { return device_; }

  void AllReduce(const void* send, void* recv, size_t count, DataType dt, ReduceOp op,
                 hipStream_t stream);
  void Broadcast(const void* send, void* recv, size_t count, DataType dt, int root,
                 hipStream_t stream);
  /*! \brief recv holds world * send_count elements */
  void AllGather(const void* send, void* recv, size_t send_count, DataType dt,
                 hipStream_t stream);
  /*! \brief send holds world * recv_count elements */
  void ReduceScatter(const void* send, void* recv, size_t recv_count, DataType dt, ReduceOp op,
                     hipStream_t stream);
  /*! \brief equal-size all-to-all: `count` elements to / from every peer */
  void AllToAll(const void* send, void* recv, size_t count, DataType dt, hipStream_t stream);
  /*!
   * \brief variable-size all-to-all as one grouped send/recv round
   *  (counts / displacements in elements, one entry per peer)
   */
  void AllToAllV(const void* send, const std::vector<size_t>& send_counts,
                 const std::vector<size_t>& send_displs, void* recv,
                 const std::vector<size_t>& recv_counts,
                 const std::vector<size_t>& recv_displs, DataType dt, hipStream_t stream);
  void Send(const void* buf, size_t count, DataType dt, int peer, hipStream_t stream);
  void Recv(void* buf, size_t count, DataType dt, int peer, hipStream_t stream);
  /*! \brief device-side barrier (a 1-element all-reduce), then stream sync */
  void Barrier(hipStream_t stream);
  /*!
   * \brief abort in-flight work (failure signalled by the tracker): safe to
   *  call from another thread while a collective is blocked; every later
   *  call throws dmlc::Error
   */
  void Abort();
  /*! \brief true once Abort() ran */
  bool aborted() const { return aborted_.load(); }
  /*!
   * \brief abort this communicator when `tracker` reports a job failure
   *  (peer missed heartbeats / aborted); cleared by the destructor.  The
   *  tracker's heartbeat thread must be running (StartHeartbeat).
   */
  void AbortOnTrackerFailure(TrackerClient* tracker);

 private:
  void Check(int result, const char* what) const;
  void* Live() const;
  void* comm_{nullptr};
  std::atomic<bool> aborted_{false};
  std::mutex abort_mutex_;
  // collectives hold it shared across their enqueue; Abort takes it exclusive
  // (bounded wait) so ncclCommAbort never frees a comm mid-enqueue
  mutable std::shared_timed_mutex use_mu_;
  TrackerClient* watched_{nullptr};
  int rank_, world_, device_;
  void* scratch_{nullptr};
};

}  // namespace dist
}  // namespace dmlc
#endif  // DMLC_DIST_COMMUNICATOR_H_
