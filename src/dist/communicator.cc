/*!
 * \file src/dist/communicator.cc
 * \brief RCCL communicator with run-time symbol resolution (see the header).
 */
#include <dlfcn.h>
#include <dmlc/dist/communicator.h>
#include <dmlc/dist/tracker_client.h>
#include <dmlc/logging.h>
#include <rccl/rccl.h>

#include <chrono>
#include <mutex>
#include <shared_mutex>

#include <dmlc/gpu/hip_utils.h>

#include <cstring>

namespace dmlc {
namespace dist {
namespace {

/*! \brief the RCCL entry points we use, resolved once */
struct RcclApi {
  void* handle{nullptr};
  decltype(&ncclGetUniqueId) GetUniqueId{nullptr};
  decltype(&ncclCommInitRank) CommInitRank{nullptr};
  decltype(&ncclCommDestroy) CommDestroy{nullptr};
  decltype(&ncclCommAbort) CommAbort{nullptr};
  decltype(&ncclGetErrorString) GetErrorString{nullptr};
  decltype(&ncclAllReduce) AllReduce{nullptr};
  decltype(&ncclBroadcast) Broadcast{nullptr};
  decltype(&ncclAllGather) AllGather{nullptr};
  decltype(&ncclReduceScatter) ReduceScatter{nullptr};
  decltype(&ncclAllToAll) AllToAll{nullptr};
  decltype(&ncclSend) Send{nullptr};
  decltype(&ncclRecv) Recv{nullptr};
  decltype(&ncclGroupStart) GroupStart{nullptr};
  decltype(&ncclGroupEnd) GroupEnd{nullptr};
  std::string error;

  RcclApi() {
    // reuse an RCCL already in the process (e.g. PyTorch's) before loading ours
    const char* names[] = {"librccl.so", "librccl.so.1"};
    for (const char* n : names) {
      handle = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
      if (handle != nullptr) break;
    }
    if (handle == nullptr) handle = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (handle == nullptr) handle = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (handle == nullptr) {
      const char* e = dlerror();
      error = e != nullptr ? e : "librccl not found";
      return;
    }
#define DMLC_RCCL_SYM(field, name) \
  field = reinterpret_cast<decltype(field)>(dlsym(handle, #name)); \
  if (field == nullptr) error += std::string(" missing ") + #name;
    DMLC_RCCL_SYM(GetUniqueId, ncclGetUniqueId)
    DMLC_RCCL_SYM(CommInitRank, ncclCommInitRank)
    DMLC_RCCL_SYM(CommDestroy, ncclCommDestroy)
    DMLC_RCCL_SYM(CommAbort, ncclCommAbort)
    DMLC_RCCL_SYM(GetErrorString, ncclGetErrorString)
    DMLC_RCCL_SYM(AllReduce, ncclAllReduce)
    DMLC_RCCL_SYM(Broadcast, ncclBroadcast)
    DMLC_RCCL_SYM(AllGather, ncclAllGather)
    DMLC_RCCL_SYM(ReduceScatter, ncclReduceScatter)
    DMLC_RCCL_SYM(AllToAll, ncclAllToAll)
    DMLC_RCCL_SYM(Send, ncclSend)
    DMLC_RCCL_SYM(Recv, ncclRecv)
    DMLC_RCCL_SYM(GroupStart, ncclGroupStart)
    DMLC_RCCL_SYM(GroupEnd, ncclGroupEnd)
#undef DMLC_RCCL_SYM
  }
  bool ok() const { return handle != nullptr && error.empty(); }
};

RcclApi& Api() {
  static RcclApi* api = new RcclApi();  // never unloaded
  return *api;
}

RcclApi& CheckedApi() {
  RcclApi& a = Api();
  CHECK(a.ok()) << "RCCL is not available: " << a.error;
  return a;
}

ncclDataType_t ToNccl(DataType t) {
  switch (t) {
    case DataType::kInt8: return ncclInt8;
    case DataType::kUInt8: return ncclUint8;
    case DataType::kInt32: return ncclInt32;
    case DataType::kUInt32: return ncclUint32;
    case DataType::kInt64: return ncclInt64;
    case DataType::kUInt64: return ncclUint64;
    case DataType::kFloat16: return ncclFloat16;
    case DataType::kFloat32: return ncclFloat32;
    case DataType::kFloat64: return ncclFloat64;
    case DataType::kBFloat16: return ncclBfloat16;
  }
  LOG(FATAL) << "unknown data type";
  return ncclFloat32;
}

ncclRedOp_t ToNccl(ReduceOp op) {
  switch (op) {
    case ReduceOp::kSum: return ncclSum;
    case ReduceOp::kProd: return ncclProd;
    case ReduceOp::kMax: return ncclMax;
    case ReduceOp::kMin: return ncclMin;
    case ReduceOp::kAvg: return ncclAvg;
  }
  LOG(FATAL) << "unknown reduce op";
  return ncclSum;
}

ncclComm_t C(void* p) { return static_cast<ncclComm_t>(p); }

}  // namespace

size_t DataTypeSize(DataType t) {
  switch (t) {
    case DataType::kInt8:
    case DataType::kUInt8: return 1;
    case DataType::kFloat16:
    case DataType::kBFloat16: return 2;
    case DataType::kInt32:
    case DataType::kUInt32:
    case DataType::kFloat32: return 4;
    default: return 8;
  }
}

bool Communicator::Available() { return Api().ok(); }

std::string Communicator::LibraryPath() {
  RcclApi& a = Api();
  Dl_info info;
  if (a.AllReduce == nullptr ||
      dladdr(reinterpret_cast<void*>(a.AllReduce), &info) == 0 || info.dli_fname == nullptr) {
    return "";
  }
  return info.dli_fname;
}

std::string Communicator::NewUniqueId() {
  static_assert(sizeof(ncclUniqueId) == kUniqueIdBytes, "ncclUniqueId size changed");
  ncclUniqueId id;
  ncclResult_t r = CheckedApi().GetUniqueId(&id);
  CHECK_EQ(r, ncclSuccess) << "ncclGetUniqueId: " << CheckedApi().GetErrorString(r);
  return std::string(id.internal, sizeof(id.internal));
}

void Communicator::Check(int result, const char* what) const {
  if (result != ncclSuccess) {
    LOG(FATAL) << what << " failed on rank " << rank_ << "/" << world_ << " (device " << device_
               << "): " << CheckedApi().GetErrorString(static_cast<ncclResult_t>(result));
  }
}

Communicator::Communicator(int rank, int world_size, int device, const std::string& unique_id)
    : rank_(rank), world_(world_size), device_(device) {
  CHECK_EQ(unique_id.size(), kUniqueIdBytes) << "bad ncclUniqueId";
  CHECK(rank >= 0 && rank < world_size) << "rank " << rank << " outside world " << world_size;
  RcclApi& api = CheckedApi();
  DMLC_HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), kUniqueIdBytes);
  ncclComm_t comm = nullptr;
  Check(api.CommInitRank(&comm, world_size, id, rank), "ncclCommInitRank");
  comm_ = comm;
  DMLC_HIP_CHECK(hipMalloc(&scratch_, 64));
}

std::unique_ptr<Communicator> Communicator::FromTracker(TrackerClient* tracker, int device,
                                                        const std::string& key) {
  if (tracker->rank() < 0) tracker->Start();
  std::string id = tracker->ExchangeUniqueId([] { return NewUniqueId(); }, key);
  std::unique_ptr<Communicator> comm(
      new Communicator(tracker->rank(), tracker->world_size(), device, id));
  comm->AbortOnTrackerFailure(tracker);  // effective once StartHeartbeat runs
  return comm;
}

Communicator::~Communicator() {
  if (watched_ != nullptr) watched_->SetFailureHandler(nullptr);
  if (comm_ != nullptr && !aborted_.load()) {
    (void)hipSetDevice(device_);
    (void)Api().CommDestroy(C(comm_));
  }
  if (scratch_ != nullptr) (void)hipFree(scratch_);
}

void Communicator::AllReduce(const void* send, void* recv, size_t count, DataType dt,
                             ReduceOp op, hipStream_t stream) {
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);
  Check(CheckedApi().AllReduce(send, recv, count, ToNccl(dt), ToNccl(op), C(Live()), stream),
        "ncclAllReduce");
}

void Communicator::Broadcast(const void* send, void* recv, size_t count, DataType dt, int root,
                             hipStream_t stream) {
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);
  Check(CheckedApi().Broadcast(send, recv, count, ToNccl(dt), root, C(Live()), stream),
        "ncclBroadcast");
}

void Communicator::AllGather(const void* send, void* recv, size_t send_count, DataType dt,
                             hipStream_t stream) {
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);
  Check(CheckedApi().AllGather(send, recv, send_count, ToNccl(dt), C(Live()), stream),
        "ncclAllGather");
}

void Communicator::ReduceScatter(const void* send, void* recv, size_t recv_count, DataType dt,
                                 ReduceOp op, hipStream_t stream) {
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);
  Check(CheckedApi().ReduceScatter(send, recv, recv_count, ToNccl(dt), ToNccl(op), C(Live()),
                                   stream),
        "ncclReduceScatter");
}

void Communicator::AllToAll(const void* send, void* recv, size_t count, DataType dt,
                            hipStream_t stream) {
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);
  Check(CheckedApi().AllToAll(send, recv, count, ToNccl(dt), C(Live()), stream), "ncclAllToAll");
}

void Communicator::AllToAllV(const void* send, const std::vector<size_t>& send_counts,
                             const std::vector<size_t>& send_displs, void* recv,
                             const std::vector<size_t>& recv_counts,
                             const std::vector<size_t>& recv_displs, DataType dt,
                             hipStream_t stream) {
  CHECK_EQ(send_counts.size(), static_cast<size_t>(world_));
  CHECK_EQ(recv_counts.size(), static_cast<size_t>(world_));
  CHECK_EQ(send_displs.size(), static_cast<size_t>(world_));
  CHECK_EQ(recv_displs.size(), static_cast<size_t>(world_));
  RcclApi& api = CheckedApi();
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);  // whole group
  const size_t esize = DataTypeSize(dt);
  const char* s = static_cast<const char*>(send);
  char* r = static_cast<char*>(recv);
  Check(api.GroupStart(), "ncclGroupStart");
  for (int p = 0; p < world_; ++p) {
    if (send_counts[p] > 0) {
      Check(api.Send(s + send_displs[p] * esize, send_counts[p], ToNccl(dt), p, C(Live()), stream),
            "ncclSend");
    }
    if (recv_counts[p] > 0) {
      Check(api.Recv(r + recv_displs[p] * esize, recv_counts[p], ToNccl(dt), p, C(Live()), stream),
            "ncclRecv");
    }
  }
  Check(api.GroupEnd(), "ncclGroupEnd");
}

void Communicator::Send(const void* buf, size_t count, DataType dt, int peer, hipStream_t stream) {
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);
  Check(CheckedApi().Send(buf, count, ToNccl(dt), peer, C(Live()), stream), "ncclSend");
}

void Communicator::Recv(void* buf, size_t count, DataType dt, int peer, hipStream_t stream) {
  std::shared_lock<std::shared_timed_mutex> use(use_mu_);
  Check(CheckedApi().Recv(buf, count, ToNccl(dt), peer, C(Live()), stream), "ncclRecv");
}

void Communicator::Barrier(hipStream_t stream) {
  AllReduce(scratch_, scratch_, 1, DataType::kInt32, ReduceOp::kSum, stream);
  DMLC_HIP_CHECK(hipStreamSynchronize(stream));
}

void* Communicator::Live() const {
  if (aborted_.load()) LOG(FATAL) << "RCCL communicator (rank " << rank_ << ") was aborted";
  return comm_;
}

void Communicator::Abort() {
  std::lock_guard<std::mutex> lock(abort_mutex_);
  if (comm_ == nullptr || aborted_.exchange(true)) return;
  // aborted_ is set first, so no new collective starts; wait (bounded) for
  // collectives that are mid-enqueue to leave RCCL before freeing the comm
  std::unique_lock<std::shared_timed_mutex> ex(use_mu_, std::defer_lock);
  if (!ex.try_lock_for(std::chrono::seconds(2))) {
    // a call is blocked inside RCCL (e.g. lazy connection setup to a dead
    // peer): ncclCommAbort is the one RCCL call allowed concurrently with it
    // and is what makes that call return
    LOG(WARNING) << "rank " << rank_ << ": aborting RCCL while a collective is blocked in it";
  }
  (void)Api().CommAbort(C(comm_));
}

void Communicator::AbortOnTrackerFailure(TrackerClient* tracker) {
  watched_ = tracker;
  tracker->SetFailureHandler([this](const std::string& reason) {
    LOG(WARNING) << "aborting RCCL communicator of rank " << rank_ << ": " << reason;
    Abort();
  });
}

}  // namespace dist
}  // namespace dmlc
