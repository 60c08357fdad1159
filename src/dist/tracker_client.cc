/*!
 * \file src/dist/tracker_client.cc
 * \brief TrackerClient: POSIX sockets implementation of the tracker protocol.
 *  Parity with the Python tracker in dmlc_core_amd/parallel/tracker.py
 *  (which keeps the reference framing, `tracker/dmlc_tracker/tracker.py:24-135`).
 */
#include <dmlc/dist/tracker_client.h>
#include <dmlc/fault.h>
#include <dmlc/logging.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <set>

namespace dmlc {
namespace dist {

/*! \brief one blocking TCP connection with int32 / string framing */
class TrackerClient::Conn {
 public:
  Conn(const std::string& host, int port, double timeout_sec) {
    struct addrinfo hints;
    std::memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    struct addrinfo* res = nullptr;
    std::string port_s = std::to_string(port);
    int rc = getaddrinfo(host.c_str(), port_s.c_str(), &hints, &res);
    CHECK_EQ(rc, 0) << "tracker address " << host << ":" << port << ": " << gai_strerror(rc);
    // the tracker may not be listening yet: retry for up to timeout_sec
    auto deadline = std::chrono::steady_clock::now() +
                    std::chrono::milliseconds(static_cast<int64_t>(timeout_sec * 1000));
    for (;;) {
      for (struct addrinfo* ai = res; ai != nullptr && fd_ < 0; ai = ai->ai_next) {
        int fd = socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
        if (fd < 0) continue;
        if (connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
          fd_ = fd;
        } else {
          close(fd);
        }
      }
      if (fd_ >= 0 || std::chrono::steady_clock::now() > deadline) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    freeaddrinfo(res);
    CHECK_GE(fd_, 0) << "cannot connect to tracker " << host << ":" << port;
    int one = 1;
    setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    struct timeval tv;
    tv.tv_sec = static_cast<time_t>(timeout_sec);
    tv.tv_usec = static_cast<suseconds_t>((timeout_sec - tv.tv_sec) * 1e6);
    setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  }
  ~Conn() {
    if (fd_ >= 0) close(fd_);
  }
  void SendAll(const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n > 0) {
      ssize_t k = send(fd_, c, n, MSG_NOSIGNAL);
      if (k < 0 && errno == EINTR) continue;
      CHECK_GT(k, 0) << "tracker send failed: " << std::strerror(errno);
      c += k;
      n -= static_cast<size_t>(k);
    }
  }
  void RecvAll(void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n > 0) {
      ssize_t k = recv(fd_, c, n, 0);
      if (k < 0 && errno == EINTR) continue;
      CHECK_GT(k, 0) << "tracker recv failed: " << (k == 0 ? "connection closed" : std::strerror(errno));
      c += k;
      n -= static_cast<size_t>(k);
    }
  }
  /*! \brief block until the peer closes (EOF) or the socket times out */
  void WaitClosed() {
    char b;
    for (;;) {
      const ssize_t k = recv(fd_, &b, 1, 0);
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) return;
    }
  }
  void SendInt(int32_t v) { SendAll(&v, sizeof(v)); }
  int32_t RecvInt() {
    int32_t v;
    RecvAll(&v, sizeof(v));
    return v;
  }
  void SendStr(const std::string& s) {
    SendInt(static_cast<int32_t>(s.size()));
    SendAll(s.data(), s.size());
  }
  std::string RecvStr() {
    int32_t n = RecvInt();
    CHECK(n >= 0 && n < (1 << 30)) << "bad string length from tracker: " << n;
    std::string s(static_cast<size_t>(n), '\0');
    if (n > 0) RecvAll(&s[0], s.size());
    return s;
  }

 private:
  int fd_{-1};
};

TrackerClient::TrackerClient(std::string uri, int port, std::string jobid, int rank,
                             int world_size, double timeout_sec)
    : uri_(std::move(uri)), port_(port), jobid_(std::move(jobid)), timeout_sec_(timeout_sec) {
  if (uri_.empty()) {
    const char* e = std::getenv("DMLC_TRACKER_URI");
    uri_ = e != nullptr ? e : "127.0.0.1";
  }
  if (port_ == 0) {
    const char* e = std::getenv("DMLC_TRACKER_PORT");
    port_ = e != nullptr ? std::atoi(e) : 9091;
  }
  if (jobid_.empty()) {
    const char* e = std::getenv("DMLC_TASK_ID");
    jobid_ = e != nullptr ? e : "NULL";
  }
  topo_.rank = rank;
  topo_.world_size = world_size;
}

TrackerClient::~TrackerClient() { StopHeartbeat(); }

std::unique_ptr<TrackerClient::Conn> TrackerClient::Connect(const std::string& cmd) {
  DMLC_FAULT_POINT("tracker");
  std::unique_ptr<Conn> c(new Conn(uri_, port_, timeout_sec_));
  c->SendInt(kMagic);
  int32_t magic = c->RecvInt();
  CHECK_EQ(magic, kMagic) << "tracker answered an invalid magic number";
  c->SendInt(topo_.rank);
  c->SendInt(topo_.world_size);
  c->SendStr(jobid_);
  c->SendStr(cmd);
  return c;
}

const Topology& TrackerClient::Start(bool recover) {
  if (recover) CHECK_GE(topo_.rank, 0) << "recover needs the previous rank";
  auto c = Connect(recover ? "recover" : "start");
  Topology t;
  t.rank = c->RecvInt();
  t.parent = c->RecvInt();
  t.world_size = c->RecvInt();
  int nnbr = c->RecvInt();
  for (int i = 0; i < nnbr; ++i) t.tree.push_back(c->RecvInt());
  t.ring_prev = c->RecvInt();
  t.ring_next = c->RecvInt();
  std::set<int> links(t.tree.begin(), t.tree.end());
  if (t.ring_prev != -1) links.insert(t.ring_prev);
  if (t.ring_next != -1) links.insert(t.ring_next);
  c->SendInt(static_cast<int32_t>(links.size()));
  for (int r : links) c->SendInt(r);
  int nconn = c->RecvInt();
  (void)c->RecvInt();  // n_accept
  for (int i = 0; i < nconn; ++i) {
    c->RecvStr();
    c->RecvInt();
    c->RecvInt();
  }
  c->SendInt(0);  // no link errors
  c->SendInt(0);  // listen port: unused, RCCL is the data plane
  topo_ = t;
  return topo_;
}

void TrackerClient::Print(const std::string& msg) {
  auto c = Connect("print");
  c->SendStr(msg);
}

void TrackerClient::Shutdown() {
  StopHeartbeat();
  Connect("shutdown");
}

bool TrackerClient::Heartbeat(std::string* reason) {
  auto c = Connect("heartbeat");
  if (c->RecvInt() == 0) return true;
  std::string why = c->RecvStr();
  if (reason != nullptr) *reason = why;
  return false;
}

void TrackerClient::Abort(const std::string& msg) {
  auto c = Connect("abort");
  c->SendStr(msg);
  c->WaitClosed();  // the tracker closes once the failure is recorded
}

void TrackerClient::SetFailureHandler(std::function<void(const std::string&)> handler) {
  std::lock_guard<std::mutex> lock(handler_mutex_);
  on_failure_ = std::move(handler);
}

void TrackerClient::ReportFailure(const std::string& reason) {
  LOG(WARNING) << "job failure signalled by the tracker: " << reason;
  std::lock_guard<std::mutex> lock(handler_mutex_);
  if (on_failure_) on_failure_(reason);
}

void TrackerClient::StartHeartbeat(double period_sec) {
  StopHeartbeat();
  std::string reason;
  if (!Heartbeat(&reason)) {
    ReportFailure(reason);
    return;
  }
  hb_stop_ = false;
  hb_thread_ = std::thread([this, period_sec]() {
    std::unique_lock<std::mutex> lock(hb_mutex_);
    for (;;) {
      auto until = std::chrono::system_clock::now() +
                   std::chrono::milliseconds(static_cast<int64_t>(period_sec * 1000));
      if (hb_cv_.wait_until(lock, until, [this] { return hb_stop_; })) return;
      lock.unlock();
      std::string why;
      bool ok = false;
      try {
        ok = Heartbeat(&why);
      } catch (const dmlc::Error& e) {
        why = std::string("tracker unreachable: ") + e.what();
      }
      if (!ok) {
        ReportFailure(why);
        return;
      }
      lock.lock();
    }
  });
}

void TrackerClient::StopHeartbeat() {
  {
    std::lock_guard<std::mutex> lock(hb_mutex_);
    hb_stop_ = true;
  }
  hb_cv_.notify_all();
  if (hb_thread_.joinable()) hb_thread_.join();
}

void TrackerClient::RcclPut(const std::string& key, const std::string& blob) {
  auto c = Connect("rccl");
  c->SendInt(0);
  c->SendStr(key);
  c->SendStr(blob);
  c->RecvInt();
}

std::string TrackerClient::RcclGet(const std::string& key) {
  auto c = Connect("rccl");
  c->SendInt(1);
  c->SendStr(key);
  return c->RecvStr();
}

void TrackerClient::Barrier(const std::string& key, int count) {
  auto c = Connect("barrier");
  c->SendStr(key);
  c->SendInt(count > 0 ? count : topo_.world_size);
  c->RecvInt();
}

int TrackerClient::Attempt() {
  auto c = Connect("attempt");
  return c->RecvInt();
}

}  // namespace dist
}  // namespace dmlc
