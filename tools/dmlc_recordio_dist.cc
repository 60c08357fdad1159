// dmlc_recordio_dist: BASELINE config 3 as a pure C++ worker -- RecordIO
// decode + InputSplit sharded across N MI355X, launched by dmlc-submit, RCCL
// bootstrapped through the tracker.  No Python runs inside the worker.
//
//   dmlc-submit --cluster local --num-workers N --gpus-per-node N \
//       build/dmlc_recordio_dist <uri> [steps=5] [warmup=1] [chunk_mb=64]
//
// Per rank: TrackerClient::Start (rank from the tracker, arrival order) ->
// hipSetDevice(DMLC_LOCAL_RANK: GPU = local index, never tracker rank) ->
// Communicator::FromTracker (rank 0 makes the ncclUniqueId, the tracker's
// `rccl` command hands it to everyone) -> DeviceRecordIOReader on shard
// (part = rank, nparts = world) -> every step re-reads + decodes the whole
// shard into HBM (K7 kernels) -> RCCL all-reduce SUM of (records, bytes) and
// MAX of the step time.  Rank 0 prints one JSON line.
//
// Reference equivalents: InputSplit::Create(uri, part, nparts, "recordio")
// (`src/io.cc:75-131`), RecordIOChunkReader (`src/recordio.cc:85-156`) and
// the rabit tracker rendezvous (`tracker/dmlc_tracker/tracker.py:137-334`).
#include <dmlc/dist/communicator.h>
#include <dmlc/dist/tracker_client.h>
#include <dmlc/gpu/device_recordio.h>
#include <dmlc/gpu/hip_utils.h>
#include <dmlc/logging.h>
#include <dmlc/timer.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

namespace {
int LocalRank() {
  for (const char* k : {"DMLC_LOCAL_RANK", "LOCAL_RANK"}) {
    const char* v = std::getenv(k);
    if (v != nullptr && *v != '\0') return std::atoi(v);
  }
  return 0;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <recordio uri> [steps=5] [warmup=1] [chunk_mb=64]\n", argv[0]);
    return 2;
  }
  const std::string uri = argv[1];
  const int steps = argc > 2 ? std::atoi(argv[2]) : 5;
  const int warmup = argc > 3 ? std::atoi(argv[3]) : 1;
  const size_t chunk_mb = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 64;
  CHECK_GT(steps, 0);

  dmlc::dist::TrackerClient tracker;
  const dmlc::dist::Topology& topo = tracker.Start();
  const int device = LocalRank();
  dmlc::gpu::SetDevice(device);
  std::unique_ptr<dmlc::dist::Communicator> comm =
      dmlc::dist::Communicator::FromTracker(&tracker, device);
  // a dead peer fails the job at the tracker; our heartbeat thread then
  // aborts the communicator instead of leaving us blocked in a collective
  tracker.StartHeartbeat(2.0);

  dmlc::gpu::DeviceRecordIOConfig cfg;
  cfg.chunk_bytes = chunk_mb << 20;
  cfg.device = device;
  std::unique_ptr<dmlc::gpu::DeviceRecordIOReader> reader(
      dmlc::gpu::DeviceRecordIOReader::Create(uri, topo.rank, topo.world_size, cfg));
  hipStream_t s = reader->stream();

  // counters[0..1] SUM, counters[2] MAX (seconds), device-resident for RCCL
  dmlc::gpu::DeviceBuffer dcount(4 * sizeof(double)), dmax(sizeof(double));
  double host[4];
  auto step = [&]() {
    reader->BeforeFirst();
    const dmlc::gpu::DeviceRecordBatch& b = reader->ReadAll();
    return std::make_pair(b.size, b.bytes);
  };
  for (int i = 0; i < warmup; ++i) step();
  DMLC_HIP_CHECK(hipStreamSynchronize(s));
  comm->Barrier(s);
  DMLC_HIP_CHECK(hipStreamSynchronize(s));
  const double t0 = dmlc::GetTime();
  std::pair<size_t, size_t> last{0, 0};
  for (int i = 0; i < steps; ++i) last = step();
  DMLC_HIP_CHECK(hipStreamSynchronize(s));
  comm->Barrier(s);
  DMLC_HIP_CHECK(hipStreamSynchronize(s));
  const double elapsed = dmlc::GetTime() - t0;

  host[0] = static_cast<double>(last.first);
  host[1] = static_cast<double>(last.second);
  host[2] = static_cast<double>(reader->PartitionBytes());
  host[3] = 0;
  DMLC_HIP_CHECK(hipMemcpyAsync(dcount.get(), host, sizeof(host), hipMemcpyHostToDevice, s));
  DMLC_HIP_CHECK(hipMemcpyAsync(dmax.get(), &elapsed, sizeof(double), hipMemcpyHostToDevice, s));
  comm->AllReduce(dcount.get(), dcount.get(), 4, dmlc::dist::DataType::kFloat64,
                  dmlc::dist::ReduceOp::kSum, s);
  comm->AllReduce(dmax.get(), dmax.get(), 1, dmlc::dist::DataType::kFloat64,
                  dmlc::dist::ReduceOp::kMax, s);
  double tmax = 0;
  DMLC_HIP_CHECK(hipMemcpyAsync(host, dcount.get(), sizeof(host), hipMemcpyDeviceToHost, s));
  DMLC_HIP_CHECK(hipMemcpyAsync(&tmax, dmax.get(), sizeof(double), hipMemcpyDeviceToHost, s));
  DMLC_HIP_CHECK(hipStreamSynchronize(s));

  if (topo.rank == 0) {
    const double recs = host[0], bytes = host[1];
    std::printf(
        "{\"metric\": \"RecordIO records/sec decoded into HBM, aggregate over GPUs\", "
        "\"value\": %.1f, \"unit\": \"records/s\", \"n_gpus\": %d, \"steps\": %d, "
        "\"warmup\": %d, \"ms_per_step\": %.3f, \"higher_is_better\": true, "
        "\"scaling\": \"strong\", \"vs_baseline\": %.3f, \"records\": %.0f, "
        "\"payload_bytes\": %.0f, \"input_bytes\": %.0f, \"input_GBps\": %.3f, "
        "\"bootstrap\": \"dmlc tracker rccl command -> ncclUniqueId -> RCCL\", "
        "\"rccl\": \"%s\"}\n",
        recs * steps / tmax, topo.world_size, steps, warmup, tmax / steps * 1e3,
        recs * steps / tmax / 11.3e6, recs, bytes, host[2], host[2] * steps / tmax / 1e9,
        dmlc::dist::Communicator::LibraryPath().c_str());
    std::fflush(stdout);
  }
  comm.reset();
  tracker.Shutdown();
  return 0;
}
