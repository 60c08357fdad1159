/*!
 * \file tools/dmlc_objserver.cc
 * \brief Loopback object server for throughput tests of the remote readers
 *  (BASELINE config 4): S3 path-style and plain HTTP over one directory,
 *  object bodies sent with sendfile(2) from the page cache.
 *
 *   dmlc_objserver --root DIR [--port P] [--host 127.0.0.1] [--tls CERT KEY]
 *
 * --tls serves https (OpenSSL; bodies read with pread and written with
 * SSL_write -- no sendfile through TLS without kernel TLS).
 *
 * Prints "PORT <n>" on stdout once listening (port 0 picks a free one), then
 * serves until killed.  Requests (HTTP/1.1, keep-alive, thread per
 * connection):
 *   HEAD /bucket/key                       Content-Length of DIR/bucket/key
 *   GET  /bucket/key [Range: bytes=b-e]    200 / 206 body via sendfile
 *   GET  /bucket?list-type=2&prefix=..     ListObjectsV2 XML (delimiter,
 *        &delimiter=..&continuation-token  max-keys, continuation tokens)
 * The S3 reader's requests (src/io/s3_filesys.cc) and the plain http://
 * reader's map onto the same routes.  Signatures are not checked: this is a
 * load generator for the client, the SigV4 verifier lives in
 * tests/mock_remote.py.
 */
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/ssl.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <map>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace {

namespace fs = std::filesystem;

std::string g_root;
SSL_CTX* g_tls = nullptr;  // --tls: https

/*! \brief one client connection: a socket, and its TLS session under --tls */
struct Conn {
  int fd;
  SSL* ssl;
};

std::string UrlDecode(const std::string& s) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      o.push_back(static_cast<char>(std::strtol(s.substr(i + 1, 2).c_str(), nullptr, 16)));
      i += 2;
    } else if (s[i] == '+') {
      o.push_back(' ');
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

std::string XmlEscape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '&': o += "&amp;"; break;
      case '<': o += "&lt;"; break;
      case '>': o += "&gt;"; break;
      default: o.push_back(c);
    }
  }
  return o;
}

bool SendAll(const Conn& c, const char* p, size_t n) {
  while (n != 0) {
    const int chunk = static_cast<int>(std::min<size_t>(n, 1u << 30));
    const ssize_t k = c.ssl != nullptr ? ::SSL_write(c.ssl, p, chunk) : ::send(c.fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

ssize_t RecvSome(const Conn& c, char* p, size_t n) {
  return c.ssl != nullptr ? ::SSL_read(c.ssl, p, static_cast<int>(n)) : ::recv(c.fd, p, n, 0);
}

bool Reply(const Conn& fd, int code, const char* reason, const std::string& body,
           const std::vector<std::string>& headers, bool head_only) {
  std::string h = "HTTP/1.1 " + std::to_string(code) + " " + reason + "\r\n";
  for (const auto& x : headers) h += x + "\r\n";
  h += "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n";
  if (!head_only) h += body;
  return SendAll(fd, h.data(), h.size());
}

/*! \brief ListObjectsV2 over DIR/bucket (keys sorted, '/'-separated) */
std::string ListXml(const std::string& bucket, std::map<std::string, std::string> q) {
  const std::string prefix = q["prefix"], delim = q["delimiter"];
  size_t max_keys = q.count("max-keys") ? std::strtoul(q["max-keys"].c_str(), nullptr, 10) : 1000;
  if (max_keys == 0 || max_keys > 1000) max_keys = 1000;
  std::vector<std::pair<std::string, uint64_t>> keys;
  const fs::path base = fs::path(g_root) / bucket;
  std::error_code ec;
  if (fs::is_directory(base, ec)) {
    for (auto it = fs::recursive_directory_iterator(base, ec); it != fs::recursive_directory_iterator();
         it.increment(ec)) {
      if (ec) break;
      if (!it->is_regular_file(ec)) continue;
      const std::string k = fs::relative(it->path(), base, ec).generic_string();
      if (k.compare(0, prefix.size(), prefix) == 0) keys.emplace_back(k, it->file_size(ec));
    }
  }
  std::sort(keys.begin(), keys.end());
  // entries in order: keys, and common prefixes once each
  std::vector<std::pair<bool, std::string>> items;  // (is_prefix, name)
  std::map<std::string, uint64_t> size_of;
  for (const auto& kv : keys) {
    const std::string rest = kv.first.substr(prefix.size());
    const size_t d = delim.empty() ? std::string::npos : rest.find(delim);
    if (d != std::string::npos) {
      const std::string p = prefix + rest.substr(0, d + delim.size());
      if (items.empty() || items.back() != std::make_pair(true, p)) items.emplace_back(true, p);
    } else {
      items.emplace_back(false, kv.first);
      size_of[kv.first] = kv.second;
    }
  }
  const size_t start = q.count("continuation-token")
                           ? std::strtoul(q["continuation-token"].c_str(), nullptr, 10)
                           : 0;
  const size_t end = std::min(items.size(), start + max_keys);
  std::string x = "<?xml version=\"1.0\" encoding=\"UTF-8\"?><ListBucketResult><Name>" +
                  XmlEscape(bucket) + "</Name><Prefix>" + XmlEscape(prefix) + "</Prefix><KeyCount>" +
                  std::to_string(end > start ? end - start : 0) + "</KeyCount><IsTruncated>" +
                  (end < items.size() ? "true" : "false") + "</IsTruncated>";
  if (end < items.size()) x += "<NextContinuationToken>" + std::to_string(end) + "</NextContinuationToken>";
  for (size_t i = start; i < end; ++i) {
    if (items[i].first) {
      x += "<CommonPrefixes><Prefix>" + XmlEscape(items[i].second) + "</Prefix></CommonPrefixes>";
    } else {
      x += "<Contents><Key>" + XmlEscape(items[i].second) + "</Key><Size>" +
           std::to_string(size_of[items[i].second]) + "</Size></Contents>";
    }
  }
  return x + "</ListBucketResult>";
}

/*! \brief one request; false ends the connection */
bool Serve(const Conn& fd, const std::string& method, const std::string& target,
           const std::map<std::string, std::string>& hdr) {
  const bool head = method == "HEAD";
  if (method != "GET" && !head) return Reply(fd, 501, "Not Implemented", "", {}, false);
  std::string path = target, query;
  const size_t qm = target.find('?');
  if (qm != std::string::npos) {
    path = target.substr(0, qm);
    query = target.substr(qm + 1);
  }
  std::map<std::string, std::string> q;
  for (size_t a = 0; a < query.size();) {
    size_t b = query.find('&', a);
    if (b == std::string::npos) b = query.size();
    const std::string kv = query.substr(a, b - a);
    const size_t eq = kv.find('=');
    q[UrlDecode(kv.substr(0, eq))] = eq == std::string::npos ? "" : UrlDecode(kv.substr(eq + 1));
    a = b + 1;
  }
  path = UrlDecode(path);
  if (path.find("..") != std::string::npos) return Reply(fd, 400, "Bad Request", "", {}, head);
  while (!path.empty() && path[0] == '/') path.erase(0, 1);
  if (q.count("list-type")) {
    const std::string bucket = path.substr(0, path.find('/'));
    return Reply(fd, 200, "OK", ListXml(bucket, q), {"Content-Type: application/xml"}, head);
  }
  const std::string file = g_root + "/" + path;
  const int f = ::open(file.c_str(), O_RDONLY | O_CLOEXEC);
  struct stat st;
  if (f < 0 || ::fstat(f, &st) != 0 || !S_ISREG(st.st_mode)) {
    if (f >= 0) ::close(f);
    return Reply(fd, 404, "Not Found", "<Error><Code>NoSuchKey</Code></Error>", {}, head);
  }
  const uint64_t size = static_cast<uint64_t>(st.st_size);
  uint64_t b = 0, e = size == 0 ? 0 : size - 1;
  bool ranged = false;
  auto r = hdr.find("range");
  if (r != hdr.end() && r->second.compare(0, 6, "bytes=") == 0) {
    const std::string spec = r->second.substr(6);
    const size_t dash = spec.find('-');
    bool bad = dash == std::string::npos;
    if (!bad && dash == 0) {
      // suffix range bytes=-N: the last N bytes (as S3)
      const uint64_t want = std::strtoull(spec.c_str() + 1, nullptr, 10);
      bad = want == 0;
      b = size - std::min<uint64_t>(want, size);
    } else if (!bad) {
      b = std::strtoull(spec.substr(0, dash).c_str(), nullptr, 10);
      if (dash + 1 < spec.size()) {
        const uint64_t last = std::strtoull(spec.c_str() + dash + 1, nullptr, 10);
        bad = last < b;
        e = std::min<uint64_t>(e, last);
      }
    }
    ranged = true;
    if (bad || b >= size) {
      ::close(f);
      return Reply(fd, 416, "Range Not Satisfiable", "",
                   {"Content-Range: bytes */" + std::to_string(size)}, head);
    }
  }
  const uint64_t len = size == 0 ? 0 : e - b + 1;
  std::string h = ranged ? "HTTP/1.1 206 Partial Content\r\n" : "HTTP/1.1 200 OK\r\n";
  if (ranged) {
    h += "Content-Range: bytes " + std::to_string(b) + "-" + std::to_string(e) + "/" +
         std::to_string(size) + "\r\n";
  }
  h += "Accept-Ranges: bytes\r\nContent-Length: " + std::to_string(len) + "\r\n\r\n";
  bool ok = SendAll(fd, h.data(), h.size());
  if (ok && !head && fd.ssl != nullptr) {
    // TLS: read and encrypt 1 MiB at a time
    thread_local std::vector<char> buf(1u << 20);
    uint64_t off = b, left = len;
    while (ok && left != 0) {
      const ssize_t k = ::pread(f, buf.data(), std::min<uint64_t>(left, buf.size()), static_cast<off_t>(off));
      ok = k > 0 && SendAll(fd, buf.data(), static_cast<size_t>(k));
      off += static_cast<uint64_t>(k > 0 ? k : 0);
      left -= static_cast<uint64_t>(k > 0 ? k : 0);
    }
  } else if (ok && !head) {
    off_t off = static_cast<off_t>(b);
    uint64_t left = len;
    while (left != 0) {
      const ssize_t k = ::sendfile(fd.fd, f, &off, std::min<uint64_t>(left, 1u << 30));
      if (k <= 0) {
        ok = false;
        break;
      }
      left -= static_cast<uint64_t>(k);
    }
  }
  ::close(f);
  return ok;
}

void Connection(int sock) {
  const int one = 1;
  ::setsockopt(sock, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  Conn fd{sock, nullptr};
  if (g_tls != nullptr) {
    fd.ssl = ::SSL_new(g_tls);
    if (fd.ssl == nullptr || ::SSL_set_fd(fd.ssl, sock) != 1 || ::SSL_accept(fd.ssl) != 1) {
      if (fd.ssl != nullptr) ::SSL_free(fd.ssl);
      ::close(sock);
      return;
    }
  }
  auto finish = [&] {
    if (fd.ssl != nullptr) ::SSL_free(fd.ssl);
    ::close(sock);
  };
  std::string buf;
  char tmp[16384];
  for (;;) {
    size_t end;
    while ((end = buf.find("\r\n\r\n")) == std::string::npos) {
      const ssize_t k = RecvSome(fd, tmp, sizeof(tmp));
      if (k <= 0) {
        finish();
        return;
      }
      buf.append(tmp, static_cast<size_t>(k));
      if (buf.size() > (1u << 20)) {
        finish();
        return;
      }
    }
    const std::string head = buf.substr(0, end);
    buf.erase(0, end + 4);
    const size_t l0 = head.find("\r\n");
    const std::string line = head.substr(0, l0);
    const size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string::npos || s2 <= s1) break;
    std::map<std::string, std::string> hdr;
    for (size_t a = l0 == std::string::npos ? head.size() : l0 + 2; a < head.size();) {
      size_t b = head.find("\r\n", a);
      if (b == std::string::npos) b = head.size();
      const std::string kv = head.substr(a, b - a);
      const size_t c = kv.find(':');
      if (c != std::string::npos) {
        std::string k = kv.substr(0, c);
        std::transform(k.begin(), k.end(), k.begin(), ::tolower);
        size_t v = c + 1;
        while (v < kv.size() && kv[v] == ' ') ++v;
        hdr[k] = kv.substr(v);
      }
      a = b + 2;
    }
    // drop a request body (none expected for GET / HEAD)
    if (hdr.count("content-length")) {
      size_t n = std::strtoul(hdr["content-length"].c_str(), nullptr, 10);
      while (buf.size() < n) {
        const ssize_t k = RecvSome(fd, tmp, sizeof(tmp));
        if (k <= 0) {
          finish();
          return;
        }
        buf.append(tmp, static_cast<size_t>(k));
      }
      buf.erase(0, n);
    }
    if (!Serve(fd, line.substr(0, s1), line.substr(s1 + 1, s2 - s1 - 1), hdr)) break;
    if (hdr.count("connection") && hdr["connection"] == "close") break;
  }
  finish();
}

}  // namespace

int main(int argc, char** argv) {
  std::string host = "127.0.0.1";
  int port = 0;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--root" && i + 1 < argc) {
      g_root = argv[++i];
    } else if (a == "--port" && i + 1 < argc) {
      port = std::atoi(argv[++i]);
    } else if (a == "--host" && i + 1 < argc) {
      host = argv[++i];
    } else if (a == "--tls" && i + 2 < argc) {
      g_tls = ::SSL_CTX_new(::TLS_server_method());
      if (g_tls == nullptr || ::SSL_CTX_use_certificate_chain_file(g_tls, argv[i + 1]) != 1 ||
          ::SSL_CTX_use_PrivateKey_file(g_tls, argv[i + 2], SSL_FILETYPE_PEM) != 1) {
        std::fprintf(stderr, "--tls: cannot load %s / %s\n", argv[i + 1], argv[i + 2]);
        return 2;
      }
      i += 2;
    } else {
      std::fprintf(stderr, "usage: %s --root DIR [--port P] [--host ADDR] [--tls CERT KEY]\n", argv[0]);
      return 2;
    }
  }
  if (g_root.empty()) {
    std::fprintf(stderr, "--root is required\n");
    return 2;
  }
  std::signal(SIGPIPE, SIG_IGN);
  const int s = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  const int one = 1;
  ::setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  ::inet_pton(AF_INET, host.c_str(), &addr.sin_addr);
  if (::bind(s, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || ::listen(s, 256) != 0) {
    std::perror("bind/listen");
    return 1;
  }
  socklen_t len = sizeof(addr);
  ::getsockname(s, reinterpret_cast<sockaddr*>(&addr), &len);
  std::printf("PORT %d\n", ntohs(addr.sin_port));
  std::fflush(stdout);
  for (;;) {
    const int c = ::accept4(s, nullptr, nullptr, SOCK_CLOEXEC);
    if (c < 0) continue;
    std::thread(Connection, c).detach();
  }
}
