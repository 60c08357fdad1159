/*!
 * \file dmlc/dist/tracker_client.h
 * \brief C++ worker side of the tracker protocol (no Python in the worker).
 *
 * The reference has no in-repo client: rabit's C++ engine talks to
 * `tracker/dmlc_tracker/tracker.py`.  SURVEY §2.9 / §5.8 ask for a native
 * client so a C++ process can obtain its rank, topology and the RCCL unique
 * id.  Wire format: native-endian int32, strings as
 * int32 length + bytes; each command is one TCP connection starting with
 * magic 0xff99, rank, world_size, jobid, cmd.  Commands: start / recover /
 * shutdown / print (reference protocol) and rccl / barrier / heartbeat
 * (this framework's tracker, dmlc_core_amd/parallel/tracker.py).
 *
 * The data plane is RCCL, so Start() reports every topology link as already
 * established and the tracker brokers no TCP peer connections.
 */
#ifndef DMLC_DIST_TRACKER_CLIENT_H_
#define DMLC_DIST_TRACKER_CLIENT_H_

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dmlc {
namespace dist {

/*! \brief what the tracker told this worker */
struct Topology {
  int rank{-1};
  int parent{-1};
  int world_size{-1};
  std::vector<int> tree;
  int ring_prev{-1};
  int ring_next{-1};
};

class TrackerClient {
 public:
  static constexpr int kMagic = 0xff99;
  /*!
   * \param uri / port tracker address ("" / 0: DMLC_TRACKER_URI / DMLC_TRACKER_PORT)
   * \param jobid restart key ("" : DMLC_TASK_ID or "NULL")
   */
  TrackerClient(std::string uri = "", int port = 0, std::string jobid = "", int rank = -1,
                int world_size = -1, double timeout_sec = 600.0);
  ~TrackerClient();
  TrackerClient(const TrackerClient&) = delete;
  TrackerClient& operator=(const TrackerClient&) = delete;

  /*! \brief join the job (cmd start, or recover with the current rank) */
  const Topology& Start(bool recover = false);
  /*! \brief relay a log line through the tracker */
  void Print(const std::string& msg);
  /*! \brief tell the tracker this rank finished */
  void Shutdown();
  /*!
   * \brief one liveness ping
   * \return true while the job is healthy; false (reason in `*reason`) once
   *  the tracker declared it failed (a rank missed heartbeats or aborted)
   */
  bool Heartbeat(std::string* reason = nullptr);
  /*! \brief report a fatal error of this rank: the tracker fails the job */
  void Abort(const std::string& msg);
  /*!
   * \brief ping every `period_sec` on a background thread until Shutdown; on
   *  job failure (or an unreachable tracker) the failure handler runs once
   */
  void StartHeartbeat(double period_sec = 5.0);
  void StopHeartbeat();
  /*!
   * \brief called (once, from the heartbeat thread) when the job fails, e.g.
   *  Communicator::Abort so no rank blocks in a collective whose peer died.
   *  nullptr clears it.
   */
  void SetFailureHandler(std::function<void(const std::string&)> handler);
  /*! \brief publish / fetch an opaque blob (RCCL unique id) under `key` */
  void RcclPut(const std::string& key, const std::string& blob);
  std::string RcclGet(const std::string& key);
  /*! \brief block until `count` workers (default world size) reached `key` */
  void Barrier(const std::string& key = "default", int count = -1);
  /*!
   * \brief this launch's attempt number for the task id `jobid`: 0 the first
   *  time the tracker hears it, then 1, 2, ... (DMLC_NUM_ATTEMPT for
   *  launchers that relaunch containers on their own)
   */
  int Attempt();
  /*!
   * \brief rank 0 creates the id with make_id() and uploads it; every rank
   *  (rank 0 included) returns the same bytes
   */
  template <typename MakeId>
  std::string ExchangeUniqueId(MakeId make_id, const std::string& key = "world") {
    if (topo_.rank == 0) {
      std::string blob = make_id();
      RcclPut(key, blob);
      return blob;
    }
    return RcclGet(key);
  }

  const Topology& topology() const { return topo_; }
  int rank() const { return topo_.rank; }
  int world_size() const { return topo_.world_size; }

 private:
  class Conn;
  std::unique_ptr<Conn> Connect(const std::string& cmd);

  std::string uri_;
  int port_;
  std::string jobid_;
  double timeout_sec_;
  Topology topo_;
  std::thread hb_thread_;
  std::mutex hb_mutex_;
  std::condition_variable hb_cv_;
  bool hb_stop_{false};
  std::mutex handler_mutex_;
  std::function<void(const std::string&)> on_failure_;
  void ReportFailure(const std::string& reason);
};

}  // namespace dist
}  // namespace dmlc
#endif  // DMLC_DIST_TRACKER_CLIENT_H_
