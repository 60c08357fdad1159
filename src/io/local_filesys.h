/*!
 * \file src/io/local_filesys.h
 * \brief POSIX filesystem backend.
 * Parity: reference `src/io/local_filesys.h` / `.cc:28-169` (FILE* streams,
 * stat, opendir, "stdin"/"stdout" magic names, `file://` stripping).
 * Addition: OpenRawFd for the parallel pread path of the GPU pinned ring.
 */
#ifndef DMLC_IO_LOCAL_FILESYS_H_
#define DMLC_IO_LOCAL_FILESYS_H_

#include <vector>

#include "./filesys.h"

namespace dmlc {
namespace io {

class LocalFileSystem : public FileSystem {
 public:
  static LocalFileSystem* GetInstance() {
    static LocalFileSystem instance;
    return &instance;
  }
  FileInfo GetPathInfo(const URI& path) override;
  void ListDirectory(const URI& path, std::vector<FileInfo>* out_list) override;
  Stream* Open(const URI& path, const char* const flag, bool allow_null) override;
  SeekStream* OpenForRead(const URI& path, bool allow_null) override;
  int OpenRawFd(const URI& path) override;
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_LOCAL_FILESYS_H_
