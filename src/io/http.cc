/*!
 * \file src/io/http.cc
 * \brief libcurl (dlopen) HTTP client and the ranged read stream.
 */
#include "./http.h"

#include <dlfcn.h>
#include <dmlc/fault.h>
#include <dmlc/logging.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <ctime>
#include <thread>

namespace dmlc {
namespace io {
namespace {

// libcurl ABI constants (stable since 7.x; headers are not installed here)
constexpr int kOptWriteData = 10001, kOptUrl = 10002, kOptTimeout = 13,
              kOptReadData = 10009, kOptPostFields = 10015, kOptHttpHeader = 10023,
              kOptHeaderData = 10029, kOptCustomRequest = 10036, kOptNoBody = 44,
              kOptUpload = 46, kOptFollow = 52, kOptSslVerifyPeer = 64,
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

}  // namespace

bool Http::Available() { return Curl().ok(); }

HttpResponse Http::Perform(const HttpRequest& req) {
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
    if (size >= block_) {
      // large read: straight into the caller's memory
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
