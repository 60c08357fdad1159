/*!
 * \file src/io/remote_filesys.h
 * \brief Protocol table for remote filesystem backends.
 */
#ifndef DMLC_IO_REMOTE_FILESYS_H_
#define DMLC_IO_REMOTE_FILESYS_H_

#include <string>

#include "./filesys.h"

namespace dmlc {
namespace io {

/*! \brief creates the backend serving one protocol/host */
typedef FileSystem* (*FileSystemFactory)(const URI& path);
/*! \brief register `factory` for `protocol` (e.g. "s3://") */
bool RegisterFileSystem(const std::string& protocol, FileSystemFactory factory);
/*! \brief make sure the S3/HTTP/HDFS/Azure translation units registered */
void EnsureRemoteFileSystemsRegistered();

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_REMOTE_FILESYS_H_
