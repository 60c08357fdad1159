/*!
 * \file src/io/filesys.h
 * \brief URI parsing and the abstract FileSystem interface.
 * Parity: reference `src/io/filesys.h:18-125` (URI, FileType, FileInfo,
 * FileSystem::GetInstance / GetPathInfo / ListDirectory /
 * ListDirectoryRecursive / Open / OpenForRead) and `src/io/filesys.cc:9-25`.
 */
#ifndef DMLC_IO_FILESYS_H_
#define DMLC_IO_FILESYS_H_

#include <dmlc/io.h>
#include <dmlc/logging.h>

#include <cstring>
#include <string>
#include <vector>

namespace dmlc {
namespace io {

/*! \brief `protocol://host/name`; plain paths have empty protocol and host */
struct URI {
  /*! \brief protocol including "://", e.g. "s3://"; empty for local paths */
  std::string protocol;
  /*! \brief host / bucket / namenode */
  std::string host;
  /*! \brief path (starts with '/' for remote URIs) */
  std::string name;

  URI() = default;
  explicit URI(const char* uri) {
    const char* p = std::strstr(uri, "://");
    if (p == nullptr) {
      name = uri;
      return;
    }
    protocol = std::string(uri, p - uri + 3);
    const char* h = p + 3;
    const char* slash = std::strchr(h, '/');
    if (slash == nullptr) {
      host = h;
      name = "/";
    } else {
      host = std::string(h, slash - h);
      name = slash;
    }
  }
  /*! \brief the full URI string */
  inline std::string str() const { return protocol + host + name; }
};

enum FileType { kFile, kDirectory };

struct FileInfo {
  URI path;
  size_t size{0};
  FileType type{kFile};
};

/*! \brief filesystem backend (local, s3/http, hdfs, azure) */
class FileSystem {
 public:
  /*! \brief the backend serving `path.protocol` (singleton per protocol/host) */
  static FileSystem* GetInstance(const URI& path);
  virtual ~FileSystem() = default;
  virtual FileInfo GetPathInfo(const URI& path) = 0;
  virtual void ListDirectory(const URI& path, std::vector<FileInfo>* out_list) = 0;
  /*! \brief breadth-first listing of every file below `path` */
  virtual void ListDirectoryRecursive(const URI& path, std::vector<FileInfo>* out_list);
  virtual Stream* Open(const URI& path, const char* const flag, bool allow_null = false) = 0;
  virtual SeekStream* OpenForRead(const URI& path, bool allow_null = false) = 0;
  /*!
   * \brief a POSIX file descriptor for high-throughput parallel `pread`
   *  (local files only); -1 when the backend has none.
   */
  virtual int OpenRawFd(const URI& /*path*/) { return -1; }
  /*!
   * \brief open for reading when the size is already known (from a listing):
   *  remote backends skip their HEAD request, so a reader can issue many
   *  parallel ranged GETs on one object cheaply.  Default: OpenForRead.
   */
  virtual SeekStream* OpenForReadSized(const URI& path, size_t /*size*/) {
    return OpenForRead(path, false);
  }
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_FILESYS_H_
