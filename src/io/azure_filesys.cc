/*!
 * \file src/io/azure_filesys.cc
 * \brief azure://container/path backend over the Blob REST API (SharedKey).
 *
 * The reference's Azure backend is a stub (`src/io/azure_filesys.h:22-32`:
 * GetPathInfo empty, Open/OpenForRead return NULL; listing uses a hard-coded
 * container `"container"`, `.cc:61`).  This one works:
 *  - credentials AZURE_STORAGE_ACCOUNT / AZURE_STORAGE_ACCESS_KEY (reference
 *    `azure_filesys.cc:31-40`), endpoint https://<account>.blob.core.windows.net
 *    or AZURE_STORAGE_ENDPOINT (Azurite, proxies, tests);
 *  - List Blobs with prefix / delimiter and NextMarker pagination;
 *  - Get Blob Properties (HEAD) for sizes, ranged Get Blob for reads;
 *  - writes: Put Blob below 64 MiB, else Put Block + Put Block List.
 */
#include <dmlc/logging.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "./crypto.h"
#include "./filesys.h"
#include "./http.h"
#include "./remote_filesys.h"

namespace dmlc {
namespace io {
namespace {

std::string Env(const char* k, const char* dflt = "") {
  const char* v = std::getenv(k);
  return (v == nullptr || *v == '\0') ? dflt : v;
}

struct AzureConfig {
  std::string account, key, endpoint;
  static AzureConfig FromEnv() {
    AzureConfig c;
    c.account = Env("AZURE_STORAGE_ACCOUNT");
    c.key = Env("AZURE_STORAGE_ACCESS_KEY");
    CHECK(!c.account.empty()) << "azure:// needs AZURE_STORAGE_ACCOUNT";
    c.endpoint = Env("AZURE_STORAGE_ENDPOINT");
    if (c.endpoint.empty()) c.endpoint = "https://" + c.account + ".blob.core.windows.net";
    while (!c.endpoint.empty() && c.endpoint.back() == '/') c.endpoint.pop_back();
    return c;
  }
};

class AzureClient {
 public:
  AzureClient(AzureConfig cfg, std::string container)
      : cfg_(std::move(cfg)), container_(std::move(container)) {}

  /*!
   * \param blob blob name ("" for container-level operations)
   * \param x_ms extra x-ms-* headers (lower-case names)
   */
  HttpRequest Make(const std::string& method, const std::string& blob,
                   const std::map<std::string, std::string>& query,
                   std::map<std::string, std::string> x_ms = {}, const char* body = nullptr,
                   size_t body_len = 0, const std::string& content_type = "") const {
    std::string path = "/" + container_ + (blob.empty() ? "" : "/" + crypto::UriEncode(blob, false));
    std::string qs;
    for (const auto& kv : query) {
      qs += (qs.empty() ? "" : "&") + crypto::UriEncode(kv.first) + "=" + crypto::UriEncode(kv.second);
    }
    HttpRequest req;
    req.method = method;
    req.url = cfg_.endpoint + path + (qs.empty() ? "" : "?" + qs);
    req.body = body;
    req.body_len = body_len;
    x_ms["x-ms-date"] = HttpDate();
    x_ms["x-ms-version"] = "2020-10-02";
    std::string canon_hdrs;
    for (const auto& kv : x_ms) {
      canon_hdrs += kv.first + ":" + kv.second + "\n";
      req.headers.push_back(kv.first + ": " + kv.second);
    }
    if (!content_type.empty()) req.headers.push_back("Content-Type: " + content_type);
    if (cfg_.key.empty()) return req;  // anonymous (public container)
    // for a path-style endpoint (Azurite) the account is part of the URL path
    std::string canon_res = "/" + cfg_.account;
    const size_t scheme = cfg_.endpoint.find("://");
    const size_t slash = cfg_.endpoint.find('/', scheme == std::string::npos ? 0 : scheme + 3);
    if (slash != std::string::npos) canon_res += cfg_.endpoint.substr(slash);
    canon_res += path;
    for (const auto& kv : query) canon_res += "\n" + kv.first + ":" + kv.second;
    // Content-Length is signed as "" when zero (x-ms-version >= 2015-02-21)
    const std::string len = body_len > 0 ? std::to_string(body_len) : "";
    const std::string to_sign = method + "\n" /*Content-Encoding*/ + "\n" /*Content-Language*/ +
                                "\n" + len + "\n" /*Content-MD5*/ + "\n" +
                                content_type + "\n" /*Date*/ + "\n" /*If-Modified-Since*/ +
                                "\n" /*If-Match*/ + "\n" /*If-None-Match*/ +
                                "\n" /*If-Unmodified-Since*/ + "\n" /*Range*/ + "\n" + canon_hdrs +
                                canon_res;
    const std::string sig =
        crypto::Base64Encode(crypto::HmacSha256(crypto::Base64Decode(cfg_.key), to_sign));
    req.headers.push_back("Authorization: SharedKey " + cfg_.account + ":" + sig);
    return req;
  }
  const std::string& container() const { return container_; }

 private:
  AzureConfig cfg_;
  std::string container_;
};

std::string BlobOf(const URI& path) {
  std::string k = path.name;
  while (!k.empty() && k[0] == '/') k.erase(0, 1);
  return k;
}

[[noreturn]] void Fail(const std::string& what, const HttpResponse& r) {
  LOG(FATAL) << what << ": "
             << (r.error.empty() ? "HTTP " + std::to_string(r.status) + " " + r.body.substr(0, 400)
                                 : r.error);
  std::abort();
}

class AzureWriteStream : public Stream {
 public:
  static constexpr size_t kBlock = 64UL << 20;
  AzureWriteStream(std::shared_ptr<AzureClient> c, std::string blob)
      : c_(std::move(c)), blob_(std::move(blob)) {}
  ~AzureWriteStream() override {
    try {
      Finish();
    } catch (const dmlc::Error& e) {
      LOG(ERROR) << "Azure upload of " << blob_ << " failed: " << e.what();
    }
  }
  size_t Read(void*, size_t) override {
    LOG(FATAL) << "AzureWriteStream is write-only";
    return 0;
  }
  void Write(const void* ptr, size_t size) override {
    buf_.append(static_cast<const char*>(ptr), size);
    while (buf_.size() >= kBlock) {
      PutBlock(buf_.data(), kBlock);
      buf_.erase(0, kBlock);
    }
  }

 private:
  void PutBlock(const char* data, size_t n) {
    char id[32];
    std::snprintf(id, sizeof(id), "block-%010zu", ids_.size());
    const std::string bid = crypto::Base64Encode(id);
    auto r = Http::PerformRetry(
        c_->Make("PUT", blob_, {{"blockid", bid}, {"comp", "block"}}, {}, data, n), 3);
    if (!r.ok()) Fail("Azure Put Block " + blob_, r);
    ids_.push_back(bid);
  }
  void Finish() {
    if (done_) return;
    done_ = true;
    if (ids_.empty()) {
      auto r = Http::PerformRetry(c_->Make("PUT", blob_, {}, {{"x-ms-blob-type", "BlockBlob"}},
                                           buf_.data(), buf_.size()),
                                  3);
      if (!r.ok()) Fail("Azure Put Blob " + blob_, r);
      return;
    }
    if (!buf_.empty()) PutBlock(buf_.data(), buf_.size());
    std::string xml = "<?xml version=\"1.0\" encoding=\"utf-8\"?><BlockList>";
    for (const auto& id : ids_) xml += "<Latest>" + id + "</Latest>";
    xml += "</BlockList>";
    auto r = Http::PerformRetry(
        c_->Make("PUT", blob_, {{"comp", "blocklist"}}, {}, xml.data(), xml.size()), 3);
    if (!r.ok()) Fail("Azure Put Block List " + blob_, r);
  }
  std::shared_ptr<AzureClient> c_;
  std::string blob_, buf_;
  std::vector<std::string> ids_;
  bool done_{false};
};

class AzureFileSystem : public FileSystem {
 public:
  explicit AzureFileSystem(const URI& path)
      : c_(std::make_shared<AzureClient>(AzureConfig::FromEnv(), path.host)) {}

  FileInfo GetPathInfo(const URI& path) override {
    FileInfo info;
    info.path = path;
    const std::string blob = BlobOf(path);
    if (!blob.empty() && blob.back() != '/') {
      auto r = Http::PerformRetry(c_->Make("HEAD", blob, {}), 3);
      if (r.ok()) {
        info.size = std::strtoull(r.headers["content-length"].c_str(), nullptr, 10);
        return info;
      }
      if (!r.error.empty() || r.status != 404) Fail("Azure HEAD " + blob, r);
    }
    std::vector<FileInfo> items;
    const bool any = List(blob.empty() || blob.back() == '/' ? blob : blob + "/", &items, 1);
    CHECK(any || blob.empty()) << "azure://" << c_->container() << "/" << blob << " does not exist";
    info.type = kDirectory;
    return info;
  }
  void ListDirectory(const URI& path, std::vector<FileInfo>* out) override {
    std::string p = BlobOf(path);
    if (!p.empty() && p.back() != '/') p += '/';
    out->clear();
    List(p, out, 0);
  }
  Stream* Open(const URI& path, const char* const flag, bool allow_null) override {
    if (!std::strcmp(flag, "r") || !std::strcmp(flag, "rb")) return OpenForRead(path, allow_null);
    if (!std::strcmp(flag, "w") || !std::strcmp(flag, "wb")) {
      return new AzureWriteStream(c_, BlobOf(path));
    }
    LOG(FATAL) << "Azure: unsupported open mode " << flag;
    return nullptr;
  }
  SeekStream* OpenForRead(const URI& path, bool allow_null) override {
    const std::string blob = BlobOf(path);
    auto head = Http::PerformRetry(c_->Make("HEAD", blob, {}), 3);
    if (!head.ok()) {
      if (allow_null) return nullptr;
      Fail("Azure open " + blob, head);
    }
    const size_t size = std::strtoull(head.headers["content-length"].c_str(), nullptr, 10);
    return OpenForReadSized(path, size);
  }
  SeekStream* OpenForReadSized(const URI& path, size_t size) override {
    const std::string blob = BlobOf(path);
    auto c = c_;
    return new RangedReadStream(size, [c, blob](size_t off, size_t len, char* dst) -> size_t {
      auto req = c->Make("GET", blob, {},
                         {{"x-ms-range", "bytes=" + std::to_string(off) + "-" +
                                             std::to_string(off + len - 1)}});
      req.out = dst;
      req.out_cap = len;
      auto r = Http::Perform(req);
      if (r.status == 404 || r.status == 403) Fail("Azure GET " + blob, r);
      return (r.status == 206 || r.status == 200) ? r.out_written : 0;
    });
  }

 private:
  bool List(const std::string& prefix, std::vector<FileInfo>* out, int max_results) {
    std::string marker;
    bool any = false;
    for (;;) {
      std::map<std::string, std::string> q{
          {"restype", "container"}, {"comp", "list"}, {"prefix", prefix}, {"delimiter", "/"}};
      if (max_results > 0) q["maxresults"] = std::to_string(max_results);
      if (!marker.empty()) q["marker"] = marker;
      auto r = Http::PerformRetry(c_->Make("GET", "", q), 3);
      if (!r.ok()) Fail("Azure List Blobs " + prefix, r);
      size_t pos = 0;
      for (;;) {
        std::string item = XmlText(r.body, "Blob", &pos);
        if (pos == std::string::npos) break;
        FileInfo fi;
        fi.path.protocol = "azure://";
        fi.path.host = c_->container();
        fi.path.name = "/" + XmlText(item, "Name");
        fi.size = std::strtoull(XmlText(item, "Content-Length").c_str(), nullptr, 10);
        out->push_back(fi);
        any = true;
      }
      pos = 0;
      for (;;) {
        std::string item = XmlText(r.body, "BlobPrefix", &pos);
        if (pos == std::string::npos) break;
        std::string p = XmlText(item, "Name");
        while (!p.empty() && p.back() == '/') p.pop_back();
        FileInfo fi;
        fi.path.protocol = "azure://";
        fi.path.host = c_->container();
        fi.path.name = "/" + p;
        fi.type = kDirectory;
        out->push_back(fi);
        any = true;
      }
      marker = XmlText(r.body, "NextMarker");
      if (marker.empty() || max_results > 0) break;
    }
    return any;
  }
  std::shared_ptr<AzureClient> c_;
};

FileSystem* CreateAzure(const URI& path) { return new AzureFileSystem(path); }

}  // namespace

void RegisterAzureFileSystem() { RegisterFileSystem("azure://", &CreateAzure); }

}  // namespace io
}  // namespace dmlc
