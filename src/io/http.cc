/*!
 * \file src/io/http.cc
 * \brief libcurl (dlopen) HTTP client and the ranged read stream.
 */
#include "./http.h"

#include <arpa/inet.h>
#include <dlfcn.h>
#include <dmlc/fault.h>
#include <dmlc/logging.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <set>
#include <thread>

namespace dmlc {
namespace io {
namespace {

// libcurl ABI constants (stable since 7.x; headers are not installed here)
constexpr int kOptWriteData = 10001, kOptUrl = 10002, kOptTimeout = 13,
              kOptReadData = 10009, kOptPostFields = 10015, kOptHttpHeader = 10023,
              kOptHeaderData = 10029, kOptCustomRequest = 10036, kOptNoBody = 44,
              kOptUpload = 46, kOptFollow = 52, kOptSslVerifyPeer = 64, kOptCaInfo = 10065,
              kOptConnectTimeout = 78, kOptSslVerifyHost = 81, kOptNoSignal = 99,
              kOptWriteFunction = 20011, kOptReadFunction = 20012,
              kOptHeaderFunction = 20079, kOptInFileSizeLarge = 30115,
              kOptPostFieldSizeLarge = 30120;
constexpr int kInfoResponseCode = 0x200002;
constexpr long kGlobalDefault = 3;

struct curl_slist;
struct CurlApi {
  void* handle{nullptr};
  int (*global_init)(long){nullptr};
  void* (*easy_init)(){nullptr};
  int (*easy_setopt)(void*, int, ...){nullptr};
  int (*easy_perform)(void*){nullptr};
  int (*easy_getinfo)(void*, int, ...){nullptr};
  void (*easy_cleanup)(void*){nullptr};
  void (*easy_reset)(void*){nullptr};
  const char* (*easy_strerror)(int){nullptr};
  curl_slist* (*slist_append)(curl_slist*, const char*){nullptr};
  void (*slist_free_all)(curl_slist*){nullptr};
  std::string error;

  CurlApi() {
    for (const char* n : {"libcurl.so.4", "libcurl.so", "libcurl-gnutls.so.4"}) {
      handle = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (handle != nullptr) break;
    }
    if (handle == nullptr) {
      error = "libcurl not found";
      return;
    }
#define DMLC_CURL_SYM(f, name) \
  f = reinterpret_cast<decltype(f)>(dlsym(handle, name)); \
  if (f == nullptr) error += std::string(" missing ") + name;
    DMLC_CURL_SYM(global_init, "curl_global_init")
    DMLC_CURL_SYM(easy_init, "curl_easy_init")
    DMLC_CURL_SYM(easy_setopt, "curl_easy_setopt")
    DMLC_CURL_SYM(easy_perform, "curl_easy_perform")
    DMLC_CURL_SYM(easy_getinfo, "curl_easy_getinfo")
    DMLC_CURL_SYM(easy_cleanup, "curl_easy_cleanup")
    DMLC_CURL_SYM(easy_reset, "curl_easy_reset")
    DMLC_CURL_SYM(easy_strerror, "curl_easy_strerror")
    DMLC_CURL_SYM(slist_append, "curl_slist_append")
    DMLC_CURL_SYM(slist_free_all, "curl_slist_free_all")
#undef DMLC_CURL_SYM
    if (error.empty()) global_init(kGlobalDefault);
  }
  bool ok() const { return handle != nullptr && error.empty(); }
};

/*! \brief CURL_CA_BUNDLE, else SSL_CERT_FILE; nullptr: the built-in store */
const char* CaBundle() {
  static const std::string ca = [] {
    for (const char* e : {"CURL_CA_BUNDLE", "SSL_CERT_FILE"}) {
      const char* v = std::getenv(e);
      if (v != nullptr && *v != '\0') return std::string(v);
    }
    return std::string();
  }();
  return ca.empty() ? nullptr : ca.c_str();
}

CurlApi& Curl() {
  static CurlApi* api = new CurlApi();
  return *api;
}

/*! \brief per-thread easy handle: keep-alive connections survive between requests */
struct EasyHandle {
  void* h{nullptr};
  ~EasyHandle() {
    if (h != nullptr) Curl().easy_cleanup(h);
  }
};

void* ThreadHandle() {
  thread_local EasyHandle eh;
  if (eh.h == nullptr) eh.h = Curl().easy_init();
  return eh.h;
}

struct Transfer {
  const HttpRequest* req;
  HttpResponse* resp;
  size_t upload_pos{0};
};

size_t OnWrite(char* data, size_t size, size_t nmemb, void* user) {
  auto* t = static_cast<Transfer*>(user);
  const size_t n = size * nmemb;
  if (t->req->out != nullptr) {
    const size_t k = std::min(n, t->req->out_cap - t->resp->out_written);
    std::memcpy(t->req->out + t->resp->out_written, data, k);
    t->resp->out_written += k;
    if (k < n) t->resp->body.append(data + k, n - k);  // overflow kept for diagnostics
  } else {
    t->resp->body.append(data, n);
  }
  return n;
}

size_t OnRead(char* dst, size_t size, size_t nmemb, void* user) {
  auto* t = static_cast<Transfer*>(user);
  const size_t k = std::min(size * nmemb, t->req->body_len - t->upload_pos);
  std::memcpy(dst, t->req->body + t->upload_pos, k);
  t->upload_pos += k;
  return k;
}

size_t OnHeader(char* data, size_t size, size_t nmemb, void* user) {
  auto* t = static_cast<Transfer*>(user);
  const size_t n = size * nmemb;
  std::string line(data, n);
  const size_t colon = line.find(':');
  if (colon != std::string::npos) {
    std::string k = line.substr(0, colon);
    std::string v = line.substr(colon + 1);
    std::transform(k.begin(), k.end(), k.begin(), ::tolower);
    const size_t b = v.find_first_not_of(" \t");
    const size_t e = v.find_last_not_of(" \t\r\n");
    t->resp->headers[k] = b == std::string::npos ? "" : v.substr(b, e - b + 1);
  }
  return n;
}

// ------------------------------------------------------------------------
// GETs received straight into the caller's memory.  libcurl reads the socket
// into its own 16 KiB buffer and hands it to OnWrite, which copies it into
// req.out (the pinned ring slot): two copies of every byte, ~30 GB/s of
// loopback per host in round 3 (profiles/r03_remote).  Here a plain-http body
// is recv()ed with MSG_WAITALL directly into req.out -- the kernel's socket
// copy is the only one -- and an https body is SSL_read() into req.out
// (OpenSSL 3 by dlopen: it decrypts each record and copies it out once, where
// libcurl's OnWrite adds a second copy).  Keep-alive connections are per
// thread (one per pool worker).  Anything unusual (a non-2xx status, chunked
// or length-less bodies, a transport or handshake error) closes the
// connection and the request goes to libcurl instead.  Hosts libcurl would
// reach through a proxy (http_proxy / https_proxy / all_proxy minus no_proxy)
// never take the native path, the connect waits at most libcurl's 30 s, and
// an authority whose direct connect failed is remembered, so later requests
// go straight to libcurl.

/*! \brief the OpenSSL 3 calls of the native https path (libssl.so.3, dlopen) */
struct TlsApi {
  void* handle{nullptr};
  const SSL_METHOD* (*client_method)(){nullptr};
  SSL_CTX* (*ctx_new)(const SSL_METHOD*){nullptr};
  int (*ctx_default_paths)(SSL_CTX*){nullptr};
  void (*ctx_set_verify)(SSL_CTX*, int, SSL_verify_cb){nullptr};
  SSL* (*ssl_new)(SSL_CTX*){nullptr};
  void (*ssl_free)(SSL*){nullptr};
  int (*set_fd)(SSL*, int){nullptr};
  long (*ctrl)(SSL*, int, long, void*){nullptr};  // NOLINT(runtime/int): the OpenSSL ABI
  int (*set1_host)(SSL*, const char*){nullptr};
  X509_VERIFY_PARAM* (*get0_param)(SSL*){nullptr};
  int (*param_ip)(X509_VERIFY_PARAM*, const char*){nullptr};
  int (*connect)(SSL*){nullptr};
  int (*read)(SSL*, void*, int){nullptr};
  int (*write)(SSL*, const void*, int){nullptr};
  SSL_CTX* verify_ctx{nullptr};    // peer and host verified (libcurl's default)
  SSL_CTX* noverify_ctx{nullptr};  // verify_ssl = false (S3_VERIFY_SSL=0 ...)

  TlsApi() {
    handle = dlopen("libssl.so.3", RTLD_NOW | RTLD_LOCAL);
    if (handle == nullptr) return;
    bool ok = true;
#define DMLC_TLS_SYM(f, name) \
  f = reinterpret_cast<decltype(f)>(dlsym(handle, name)); \
  ok = ok && f != nullptr;
    DMLC_TLS_SYM(client_method, "TLS_client_method")
    DMLC_TLS_SYM(ctx_new, "SSL_CTX_new")
    DMLC_TLS_SYM(ctx_default_paths, "SSL_CTX_set_default_verify_paths")
    DMLC_TLS_SYM(ctx_set_verify, "SSL_CTX_set_verify")
    DMLC_TLS_SYM(ssl_new, "SSL_new")
    DMLC_TLS_SYM(ssl_free, "SSL_free")
    DMLC_TLS_SYM(set_fd, "SSL_set_fd")
    DMLC_TLS_SYM(ctrl, "SSL_ctrl")
    DMLC_TLS_SYM(set1_host, "SSL_set1_host")
    DMLC_TLS_SYM(get0_param, "SSL_get0_param")
    DMLC_TLS_SYM(param_ip, "X509_VERIFY_PARAM_set1_ip_asc")  // libcrypto, a dependency
    DMLC_TLS_SYM(connect, "SSL_connect")
    DMLC_TLS_SYM(read, "SSL_read")
    DMLC_TLS_SYM(write, "SSL_write")
#undef DMLC_TLS_SYM
    if (!ok) return;
    verify_ctx = ctx_new(client_method());
    noverify_ctx = ctx_new(client_method());
    if (verify_ctx == nullptr || noverify_ctx == nullptr) return;
    ctx_default_paths(verify_ctx);  // the system store; SSL_CERT_FILE / SSL_CERT_DIR honoured
    if (const char* ca = std::getenv("CURL_CA_BUNDLE")) {
      auto load = reinterpret_cast<int (*)(SSL_CTX*, const char*, const char*)>(
          dlsym(handle, "SSL_CTX_load_verify_locations"));
      if (load != nullptr && *ca != '\0') load(verify_ctx, ca, nullptr);
    }
    ctx_set_verify(verify_ctx, SSL_VERIFY_PEER, nullptr);
    ctx_set_verify(noverify_ctx, SSL_VERIFY_NONE, nullptr);
  }
  bool ok() const { return verify_ctx != nullptr && noverify_ctx != nullptr; }
};

TlsApi& Tls() {
  static TlsApi* api = new TlsApi();
  return *api;
}

struct NativeConn {
  std::string authority;  // scheme://host[:port] the socket is connected to
  bool verify{true};      // the TLS verification the connection was made with
  int fd{-1};
  SSL* ssl{nullptr};      // https: the TLS session over fd
  ~NativeConn() { Close(); }
  void Close() {
    if (ssl != nullptr) Tls().ssl_free(ssl);
    ssl = nullptr;
    if (fd >= 0) ::close(fd);
    fd = -1;
  }
};

NativeConn& ThreadConn() {
  thread_local NativeConn c;
  return c;
}

bool NativeEnabled() {
  static const bool on = [] {
    const char* e = std::getenv("DMLC_HTTP_NATIVE");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

std::atomic<uint64_t> g_native_gets{0}, g_native_fallbacks{0};

/*! \brief libcurl's connect timeout (Perform sets the same 30 s) */
constexpr int kConnectTimeoutMs = 30000;

std::string LowerEnv(const char* a, const char* b) {
  const char* v = std::getenv(a);
  if (v == nullptr || *v == '\0') v = std::getenv(b);
  std::string s = v == nullptr ? "" : v;
  std::transform(s.begin(), s.end(), s.begin(), ::tolower);
  return s;
}

/*!
 * \brief true if libcurl would send a plain-http request to `host` through a
 *  proxy: http_proxy / all_proxy set (either case) and the host not excluded
 *  by no_proxy ("*", an exact name, or a domain suffix with or without the
 *  leading dot).  The native path then stays off: it only speaks to origin
 *  servers directly.
 */
bool ProxyApplies(const std::string& host, bool https = false) {
  // curl reads only lowercase http_proxy; https_proxy in either case
  const std::string hp = https ? LowerEnv("https_proxy", "HTTPS_PROXY") : [] {
    const char* v = std::getenv("http_proxy");
    return std::string(v == nullptr ? "" : v);
  }();
  const std::string proxy = !hp.empty() ? hp : LowerEnv("all_proxy", "ALL_PROXY");
  if (proxy.empty()) return false;
  std::string h = host;
  std::transform(h.begin(), h.end(), h.begin(), ::tolower);
  const std::string np = LowerEnv("no_proxy", "NO_PROXY");
  size_t at = 0;
  while (at <= np.size()) {
    size_t e = np.find(',', at);
    if (e == std::string::npos) e = np.size();
    std::string d = np.substr(at, e - at);
    at = e + 1;
    d.erase(0, d.find_first_not_of(" \t"));
    const size_t z = d.find_last_not_of(" \t");
    d.erase(z == std::string::npos ? 0 : z + 1);
    const size_t c = d.rfind(':');  // "host:port" entries: the host part
    if (c != std::string::npos && d.find(']') == std::string::npos) d.erase(c);
    if (d.empty()) continue;
    if (d == "*") return false;
    if (d.front() == '.') d.erase(0, 1);
    if (h == d) return false;
    if (h.size() > d.size() && h.compare(h.size() - d.size(), d.size(), d) == 0 &&
        h[h.size() - d.size() - 1] == '.') {
      return false;
    }
  }
  return true;
}

/*!
 * \brief authorities whose direct connect failed once: later requests go to
 *  libcurl at once instead of paying the connect timeout again per request
 */
std::mutex g_unreachable_mu;
std::set<std::string> g_unreachable;

bool KnownUnreachable(const std::string& authority) {
  std::lock_guard<std::mutex> lk(g_unreachable_mu);
  return g_unreachable.count(authority) != 0;
}

void MarkUnreachable(const std::string& authority) {
  std::lock_guard<std::mutex> lk(g_unreachable_mu);
  g_unreachable.insert(authority);
}

/*! \brief connect with a bounded wait (non-blocking connect + poll) */
bool ConnectWithin(int fd, const sockaddr* addr, socklen_t len, int timeout_ms) {
  const int fl = ::fcntl(fd, F_GETFL, 0);
  if (fl < 0 || ::fcntl(fd, F_SETFL, fl | O_NONBLOCK) < 0) return false;
  int rc = ::connect(fd, addr, len);
  if (rc != 0) {
    if (errno != EINPROGRESS) return false;
    pollfd p{fd, POLLOUT, 0};
    do {
      rc = ::poll(&p, 1, timeout_ms);
    } while (rc < 0 && errno == EINTR);
    if (rc <= 0) return false;  // timed out
    int err = 0;
    socklen_t el = sizeof(err);
    if (::getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el) != 0 || err != 0) return false;
  }
  return ::fcntl(fd, F_SETFL, fl) == 0;  // blocking again for MSG_WAITALL receives
}

int ConnectTo(const std::string& host, const std::string& port, long timeout_sec) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  if (::getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0) return -1;
  int fd = -1;
  for (addrinfo* a = res; a != nullptr; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    if (ConnectWithin(fd, a->ai_addr, a->ai_addrlen, kConnectTimeoutMs)) break;
    ::close(fd);
    fd = -1;
  }
  ::freeaddrinfo(res);
  if (fd < 0) return -1;
  const int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  timeval tv{timeout_sec, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  return fd;
}

bool SendAll(int fd, const char* p, size_t n) {
  while (n > 0) {
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

/*! \brief recv exactly n bytes (MSG_WAITALL: one syscall for the whole body on loopback) */
bool RecvAll(int fd, char* p, size_t n) {
  while (n > 0) {
    const ssize_t k = ::recv(fd, p, n, MSG_WAITALL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

/*! \brief write all of p (TLS or plain) */
bool ConnSend(NativeConn& c, const char* p, size_t n) {
  if (c.ssl == nullptr) return SendAll(c.fd, p, n);
  while (n > 0) {
    const int k = Tls().write(c.ssl, p, static_cast<int>(std::min<size_t>(n, INT_MAX)));
    if (k <= 0) return false;
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

/*! \brief what is there, up to n bytes (<= 0: closed or failed) */
ssize_t ConnRecvSome(NativeConn& c, char* p, size_t n) {
  if (c.ssl != nullptr) return Tls().read(c.ssl, p, static_cast<int>(std::min<size_t>(n, INT_MAX)));
  for (;;) {
    const ssize_t k = ::recv(c.fd, p, n, 0);
    if (k < 0 && errno == EINTR) continue;
    return k;
  }
}

/*! \brief exactly n bytes: one MSG_WAITALL recv on plain sockets, record by
 *  record (SSL_read into p, no staging buffer of ours) on TLS */
bool ConnRecvAll(NativeConn& c, char* p, size_t n) {
  if (c.ssl == nullptr) return RecvAll(c.fd, p, n);
  while (n > 0) {
    const ssize_t k = ConnRecvSome(c, p, n);
    if (k <= 0) return false;
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

/*! \brief TLS over c.fd: SNI, the peer checked against host (name or IP
 *  literal) when verify is on */
bool StartTls(NativeConn& c, const std::string& host, bool verify) {
  TlsApi& t = Tls();
  c.ssl = t.ssl_new(verify ? t.verify_ctx : t.noverify_ctx);
  if (c.ssl == nullptr || t.set_fd(c.ssl, c.fd) != 1) return false;
  in6_addr a6;
  in_addr a4;
  const bool ip = inet_pton(AF_INET, host.c_str(), &a4) == 1 ||
                  inet_pton(AF_INET6, host.c_str(), &a6) == 1;
  if (!ip) {
    t.ctrl(c.ssl, SSL_CTRL_SET_TLSEXT_HOSTNAME, TLSEXT_NAMETYPE_host_name,
           const_cast<char*>(host.c_str()));
  }
  if (verify) {
    const int r = ip ? t.param_ip(t.get0_param(c.ssl), host.c_str()) : t.set1_host(c.ssl, host.c_str());
    if (r != 1) return false;
  }
  return t.connect(c.ssl) == 1;
}

/*!
 * \brief one GET on the thread's keep-alive connection into req.out.
 * \return true if `resp` holds the outcome; false = use libcurl (the
 *  connection is closed, nothing of `resp` is kept)
 */
bool NativeGet(const HttpRequest& req, HttpResponse* resp) {
  const bool https = req.url.compare(0, 8, "https://") == 0;
  if (!https && req.url.compare(0, 7, "http://") != 0) return false;
  if (https && !Tls().ok()) return false;  // no libssl.so.3: libcurl
  const size_t skip = https ? 8 : 7;
  const size_t slash = req.url.find('/', skip);
  const std::string authority =
      req.url.substr(skip, slash == std::string::npos ? std::string::npos : slash - skip);
  const std::string target = slash == std::string::npos ? "/" : req.url.substr(slash);
  if (authority.empty() || authority.find('@') != std::string::npos ||
      authority.front() == '[') {
    return false;  // userinfo / IPv6 literals: libcurl
  }
  const size_t colon = authority.rfind(':');
  const std::string host = authority.substr(0, colon);
  const std::string port =
      colon == std::string::npos ? (https ? "443" : "80") : authority.substr(colon + 1);
  const std::string key = req.url.substr(0, skip) + authority;  // connections per scheme
  // a proxied host, or one whose direct connect already failed: libcurl
  if (ProxyApplies(host, https) || KnownUnreachable(key)) return false;

  std::string head = "GET " + target + " HTTP/1.1\r\nHost: " + authority + "\r\n";
  for (const auto& h : req.headers) head += h + "\r\n";
  head += "\r\n";

  NativeConn& c = ThreadConn();
  if (c.fd >= 0 && (c.authority != key || c.verify != req.verify_ssl)) c.Close();
  char hdr[16384];
  size_t have = 0, hend = std::string::npos;
  for (int attempt = 0; attempt < 2; ++attempt) {
    const bool reused = c.fd >= 0;
    if (!reused) {
      c.fd = ConnectTo(host, port, req.timeout_sec);
      if (c.fd < 0) {
        MarkUnreachable(key);
        return false;
      }
      c.authority = key;
      c.verify = req.verify_ssl;
      if (https && !StartTls(c, host, req.verify_ssl)) {
        c.Close();  // handshake or verification failed: libcurl reports it
        return false;
      }
    }
    have = 0;
    bool ok = ConnSend(c, head.data(), head.size());
    while (ok && hend == std::string::npos) {
      const ssize_t k = ConnRecvSome(c, hdr + have, sizeof(hdr) - have);
      if (k <= 0) {
        ok = false;
        break;
      }
      have += static_cast<size_t>(k);
      const char* e = static_cast<const char*>(memmem(hdr, have, "\r\n\r\n", 4));
      if (e != nullptr) hend = static_cast<size_t>(e - hdr) + 4;
      else if (have == sizeof(hdr)) ok = false;  // oversized header block
    }
    if (ok) break;
    c.Close();
    // a reused keep-alive connection the server has since closed: one fresh try
    if (!reused || have != 0) return false;
  }
  if (hend == std::string::npos) return false;

  // status line + headers
  HttpResponse r;
  const std::string block(hdr, hend);
  size_t eol = block.find("\r\n");
  const std::string status_line = block.substr(0, eol);
  if (status_line.compare(0, 5, "HTTP/") != 0) {
    c.Close();
    return false;
  }
  const bool http10 = status_line.compare(0, 8, "HTTP/1.0") == 0;
  const size_t sp = status_line.find(' ');
  r.status = sp == std::string::npos ? 0 : std::strtol(status_line.c_str() + sp + 1, nullptr, 10);
  for (size_t p = eol + 2; p < hend - 2;) {
    const size_t e = block.find("\r\n", p);
    const std::string line = block.substr(p, e - p);
    p = e + 2;
    const size_t col = line.find(':');
    if (col == std::string::npos) continue;
    std::string k = line.substr(0, col);
    std::transform(k.begin(), k.end(), k.begin(), ::tolower);
    const size_t b = line.find_first_not_of(" \t", col + 1);
    r.headers[k] = b == std::string::npos ? "" : line.substr(b);
  }
  auto conn = r.headers.find("connection");
  std::string conn_v = conn == r.headers.end() ? "" : conn->second;
  std::transform(conn_v.begin(), conn_v.end(), conn_v.begin(), ::tolower);
  const bool close_after = conn_v == "close" || (http10 && conn_v != "keep-alive");
  auto cl = r.headers.find("content-length");
  if ((r.status != 200 && r.status != 206) || cl == r.headers.end() ||
      r.headers.count("transfer-encoding") != 0) {
    c.Close();  // errors, redirects, chunked bodies: libcurl re-issues the request
    return false;
  }
  const size_t len = std::strtoull(cl->second.c_str(), nullptr, 10);
  const size_t into = std::min(len, req.out_cap);
  const size_t early = std::min(have - hend, len);  // body bytes that came with the headers
  const size_t early_in = std::min(early, into);
  std::memcpy(req.out, hdr + hend, early_in);
  if (early > early_in) r.body.append(hdr + hend + early_in, early - early_in);
  bool ok = ConnRecvAll(c, req.out + early_in, into - early_in);
  bool drop = close_after;
  if (ok && len > std::max(early, into)) {
    // overflow beyond out_cap (e.g. a server that ignored Range): keep a
    // little for diagnostics; a large rest is not drained, the socket closes
    const size_t rest = len - std::max(early, into);
    if (rest <= (64u << 10)) {
      const size_t at = r.body.size();
      r.body.resize(at + rest);
      ok = ConnRecvAll(c, &r.body[at], rest);
    } else {
      drop = true;
    }
  }
  if (!ok || drop) c.Close();
  if (!ok) return false;
  r.out_written = into;
  *resp = std::move(r);
  return true;
}

}  // namespace

bool Http::Available() { return Curl().ok(); }

uint64_t Http::NativeGets() { return g_native_gets.load(); }
uint64_t Http::NativeFallbacks() { return g_native_fallbacks.load(); }

HttpResponse Http::Perform(const HttpRequest& req) {
  if (req.method == "GET" && req.out != nullptr && req.out_cap != 0 && NativeEnabled()) {
    HttpResponse r;
    if (NativeGet(req, &r)) {
      g_native_gets.fetch_add(1, std::memory_order_relaxed);
      return r;
    }
    g_native_fallbacks.fetch_add(1, std::memory_order_relaxed);
  }
  CurlApi& c = Curl();
  CHECK(c.ok()) << "HTTP filesystems need libcurl: " << c.error;
  HttpResponse resp;
  void* h = ThreadHandle();
  c.easy_reset(h);
  Transfer t{&req, &resp};
  curl_slist* hdrs = nullptr;
  for (const auto& s : req.headers) hdrs = c.slist_append(hdrs, s.c_str());
  // an explicit empty Expect avoids the 100-continue round trip on uploads
  hdrs = c.slist_append(hdrs, "Expect:");
  c.easy_setopt(h, kOptUrl, req.url.c_str());
  c.easy_setopt(h, kOptHttpHeader, hdrs);
  c.easy_setopt(h, kOptWriteFunction, &OnWrite);
  c.easy_setopt(h, kOptWriteData, &t);
  c.easy_setopt(h, kOptHeaderFunction, &OnHeader);
  c.easy_setopt(h, kOptHeaderData, &t);
  c.easy_setopt(h, kOptNoSignal, 1L);
  c.easy_setopt(h, kOptFollow, req.follow_redirects ? 1L : 0L);
  c.easy_setopt(h, kOptConnectTimeout, 30L);
  c.easy_setopt(h, kOptTimeout, req.timeout_sec);
  c.easy_setopt(h, kOptSslVerifyPeer, req.verify_ssl ? 1L : 0L);
  // one trust store for both https paths: a CA bundle named by CURL_CA_BUNDLE
  // or SSL_CERT_FILE (the native path's OpenSSL reads SSL_CERT_FILE itself)
  if (const char* ca = CaBundle()) c.easy_setopt(h, kOptCaInfo, ca);
  c.easy_setopt(h, kOptSslVerifyHost, req.verify_ssl ? 2L : 0L);
  if (req.method == "HEAD") {
    c.easy_setopt(h, kOptNoBody, 1L);
  } else if (req.method == "PUT") {
    c.easy_setopt(h, kOptUpload, 1L);
    c.easy_setopt(h, kOptReadFunction, &OnRead);
    c.easy_setopt(h, kOptReadData, &t);
    c.easy_setopt(h, kOptInFileSizeLarge, static_cast<int64_t>(req.body_len));
  } else if (req.method == "POST") {
    c.easy_setopt(h, kOptPostFields, req.body != nullptr ? req.body : "");
    c.easy_setopt(h, kOptPostFieldSizeLarge, static_cast<int64_t>(req.body_len));
  } else if (req.method != "GET") {
    c.easy_setopt(h, kOptCustomRequest, req.method.c_str());
  }
  const int rc = c.easy_perform(h);
  if (rc != 0) {
    resp.error = c.easy_strerror(rc);
  } else {
    long code = 0;
    c.easy_getinfo(h, kInfoResponseCode, &code);
    resp.status = code;
  }
  c.slist_free_all(hdrs);
  return resp;
}

HttpResponse Http::PerformRetry(const HttpRequest& req, int retries, int pause_ms) {
  HttpResponse r;
  for (int attempt = 0;; ++attempt) {
    r = Perform(req);
    const bool transient = !r.error.empty() || r.status >= 500 || r.status == 429;
    if (!transient || attempt >= retries) return r;
    LOG(WARNING) << req.method << " " << req.url << " failed ("
                 << (r.error.empty() ? std::to_string(r.status) : r.error) << "), retry "
                 << attempt + 1 << "/" << retries;
    std::this_thread::sleep_for(std::chrono::milliseconds(pause_ms));
  }
}

size_t RangedReadStream::FetchRetry(size_t offset, size_t len, char* dst) {
  size_t done = 0;
  for (int attempt = 0; done < len; ++attempt) {
    // an injected "http" fault is a transient failure: nothing arrives, retry
    const size_t got = DMLC_FAULT_SOFT("http") ? 0 : fetch_(offset + done, len - done, dst + done);
    done += got;
    if (got == 0) {
      CHECK_LT(attempt, 50) << "ranged read at offset " << offset + done << " failed 50 times";
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
  }
  return done;
}

size_t RangedReadStream::Read(void* ptr, size_t size) {
  char* out = static_cast<char*>(ptr);
  size_t total = 0;
  while (size > 0 && pos_ < size_) {
    const size_t avail_file = size_ - pos_;
    // serve from the read-ahead buffer
    if (pos_ >= buf_begin_ && pos_ < buf_begin_ + buf_.size()) {
      const size_t k = std::min({size, buf_begin_ + buf_.size() - pos_, avail_file});
      std::memcpy(out, buf_.data() + (pos_ - buf_begin_), k);
      out += k;
      pos_ += k;
      size -= k;
      total += k;
      continue;
    }
    if (size >= std::min(block_, kDirectRead)) {
      // large read (a shard reader's piece): one exact ranged GET straight
      // into the caller's memory -- never a block_-sized read-ahead GET and
      // a copy out of it
      const size_t k = std::min(size, avail_file);
      FetchRetry(pos_, k, out);
      out += k;
      pos_ += k;
      size -= k;
      total += k;
      continue;
    }
    const size_t k = std::min(block_, avail_file);
    buf_.resize(k);
    FetchRetry(pos_, k, &buf_[0]);
    buf_begin_ = pos_;
  }
  return total;
}

void RangedReadStream::Write(const void*, size_t) {
  LOG(FATAL) << "RangedReadStream is read-only";
}

std::string HttpDate() {
  std::time_t t = std::time(nullptr);
  struct tm g;
  gmtime_r(&t, &g);
  char buf[64];
  std::strftime(buf, sizeof(buf), "%a, %d %b %Y %H:%M:%S GMT", &g);
  return buf;
}

std::pair<std::string, std::string> AmzDate() {
  std::time_t t = std::time(nullptr);
  struct tm g;
  gmtime_r(&t, &g);
  char full[32], day[16];
  std::strftime(full, sizeof(full), "%Y%m%dT%H%M%SZ", &g);
  std::strftime(day, sizeof(day), "%Y%m%d", &g);
  return {full, day};
}

std::string XmlText(const std::string& xml, const std::string& tag, size_t* from) {
  const std::string open = "<" + tag + ">", close = "</" + tag + ">";
  size_t start = from != nullptr ? *from : 0;
  size_t b = xml.find(open, start);
  if (b == std::string::npos) {
    if (from != nullptr) *from = std::string::npos;
    return "";
  }
  b += open.size();
  size_t e = xml.find(close, b);
  if (e == std::string::npos) {
    if (from != nullptr) *from = std::string::npos;
    return "";
  }
  if (from != nullptr) *from = e + close.size();
  // minimal entity decoding
  std::string s = xml.substr(b, e - b), out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '&') {
      static const std::pair<const char*, char> ents[] = {
          {"&amp;", '&'}, {"&lt;", '<'}, {"&gt;", '>'}, {"&quot;", '"'}, {"&apos;", '\''}};
      bool hit = false;
      for (const auto& en : ents) {
        const size_t L = std::strlen(en.first);
        if (s.compare(i, L, en.first) == 0) {
          out.push_back(en.second);
          i += L - 1;
          hit = true;
          break;
        }
      }
      if (!hit) out.push_back('&');
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

}  // namespace io
}  // namespace dmlc
