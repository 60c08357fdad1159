/*!
 * \file src/io/remote_filesys.cc
 * \brief Registers the remote filesystem backends with the protocol table.
 *
 * Each backend lives in its own translation unit and exposes a
 * `Register*FileSystem()` hook; calling them here (instead of relying on
 * static initialisers) keeps registration working when libdmlc is linked
 * statically (the reference needed DMLC_REGISTRY_LINK_TAG for that).
 */
#include "./remote_filesys.h"

#include <mutex>

namespace dmlc {
namespace io {

// weak defaults: a backend's own translation unit provides the strong symbol
__attribute__((weak)) void RegisterS3FileSystem() {}
__attribute__((weak)) void RegisterHDFSFileSystem() {}
__attribute__((weak)) void RegisterAzureFileSystem() {}

void EnsureRemoteFileSystemsRegistered() {
  static std::once_flag once;
  std::call_once(once, []() {
    RegisterS3FileSystem();
    RegisterHDFSFileSystem();
    RegisterAzureFileSystem();
  });
}

}  // namespace io
}  // namespace dmlc
