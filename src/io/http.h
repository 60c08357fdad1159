/*!
 * \file src/io/http.h
 * \brief Minimal HTTP(S) client over libcurl loaded at run time, plus a
 *  ranged, read-ahead SeekStream shared by the S3 / HTTP / Azure backends.
 *
 * libcurl is `dlopen`ed (remote filesystems load their libraries
 * at run time), so libdmlc has no link-time dependency and the remote
 * backends fail with a clear error when libcurl is absent.  Each thread keeps
 * one easy handle, so keep-alive connections are reused across requests.
 * Plain-http GETs into caller memory (the ranged reads of the shard reader)
 * bypass libcurl: the body is recv()ed straight into the destination (see
 * NativeGet in http.cc), libcurl handles everything else.
 *
 * Retry policy follows the reference: reads reconnect up to 50 times with a
 * 100 ms pause (`src/io/s3_filesys.cc:318-342`), writes retry 3 times
 * (`:577, :712-751`).
 */
#ifndef DMLC_IO_HTTP_H_
#define DMLC_IO_HTTP_H_

#include <dmlc/io.h>

#include <functional>
#include <map>
#include <string>
#include <vector>

namespace dmlc {
namespace io {

struct HttpRequest {
  std::string method{"GET"};
  std::string url;
  std::vector<std::string> headers;  // "Name: value"
  const char* body{nullptr};
  size_t body_len{0};
  /*! \brief optional destination for the response body (else Response::body) */
  char* out{nullptr};
  size_t out_cap{0};
  bool verify_ssl{true};
  /*! \brief follow 3xx Location (off for WebHDFS, which re-sends the body itself) */
  bool follow_redirects{true};
  long timeout_sec{300};
};

struct HttpResponse {
  long status{0};
  std::map<std::string, std::string> headers;  // lower-cased names
  std::string body;
  size_t out_written{0};
  std::string error;  // transport error ("" on success)
  bool ok() const { return error.empty() && status >= 200 && status < 300; }
};

class Http {
 public:
  /*! \brief whether libcurl could be loaded */
  static bool Available();
  /*! \brief one request (no retries) */
  static HttpResponse Perform(const HttpRequest& req);
  /*!
   * \brief retry transport errors and 5xx/429 responses `retries` times,
   *  sleeping `pause_ms` between attempts
   */
  static HttpResponse PerformRetry(const HttpRequest& req, int retries, int pause_ms = 100);
  /*!
   * \brief process-wide counts of GETs into caller memory served by the
   *  native plain-http receive path (body recv()ed straight into req.out) and
   *  of those it handed to libcurl (https, non-2xx, chunked, transport error).
   *  DMLC_HTTP_NATIVE=0 sends everything to libcurl.
   */
  static uint64_t NativeGets();
  static uint64_t NativeFallbacks();
};

/*!
 * \brief SeekStream over ranged GETs: reads of at least min(`block`,
 *  kDirectRead) bytes go straight into the caller's buffer as one exact
 *  ranged GET, smaller ones are served from a read-ahead buffer of `block`
 *  bytes.
 */
class RangedReadStream : public SeekStream {
 public:
  static constexpr size_t kDirectRead = 256UL << 10;
  /*! \brief fetch [offset, offset+len) into dst; returns bytes written (0 = failure) */
  using Fetcher = std::function<size_t(size_t offset, size_t len, char* dst)>;
  RangedReadStream(size_t file_size, Fetcher fetch, size_t block = 8UL << 20)
      : size_(file_size), fetch_(std::move(fetch)), block_(block) {}
  size_t Read(void* ptr, size_t size) override;
  void Write(const void*, size_t) override;
  void Seek(size_t pos) override { pos_ = pos; }
  size_t Tell() override { return pos_; }

 private:
  size_t FetchRetry(size_t offset, size_t len, char* dst);
  size_t size_;
  Fetcher fetch_;
  size_t block_;
  size_t pos_{0};
  std::string buf_;
  size_t buf_begin_{0};
};

/*! \brief "Wed, 21 Oct 2015 07:28:00 GMT" for now */
std::string HttpDate();
/*! \brief ("20150830T123600Z", "20150830") for now */
std::pair<std::string, std::string> AmzDate();
/*! \brief text of the first <tag>...</tag> at or after `from`; npos-safe */
std::string XmlText(const std::string& xml, const std::string& tag, size_t* from = nullptr);

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_HTTP_H_
