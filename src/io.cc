/*!
 * \file src/io.cc
 * \brief Filesystem dispatch and the Stream / SeekStream / InputSplit factories.
 *
 * Parity: reference `src/io.cc` — FileSystem::GetInstance by protocol (:31-72:
 * file:// or none -> local, hdfs:// and viewfs:// -> HDFS, s3:// http://
 * https:// -> S3/HTTP, azure:// -> Azure, anything else fatal),
 * InputSplit::Create (:75-131: "stdin" -> SingleFileSplit, `#cache` ->
 * CachedInputSplit, else the splitter wrapped in a ThreadedInputSplit),
 * Stream::Create (:133-139), SeekStream::CreateForRead (:141-145).
 *
 * Remote backends register themselves in a small protocol table
 * (RegisterFileSystem) so that each lives in its own translation unit and
 * loads its native client (libcurl, libhdfs) with dlopen on first use.
 */
#include <dmlc/io.h>
#include <dmlc/logging.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "./io/cached_input_split.h"
#include "./io/filesys.h"
#include "./io/line_split.h"
#include "./io/local_filesys.h"
#include "./io/recordio_split.h"
#include "./io/single_file_split.h"
#include "./io/threaded_input_split.h"
#include "./io/uri_spec.h"
#include "./io/remote_filesys.h"

namespace dmlc {
namespace io {

namespace {
struct FsTable {
  std::mutex mu;
  std::map<std::string, FileSystemFactory> factories;
  std::map<std::string, FileSystem*> instances;  // key: protocol + host
};
FsTable& Table() {
  static FsTable* t = new FsTable();
  return *t;
}
}  // namespace

bool RegisterFileSystem(const std::string& protocol, FileSystemFactory factory) {
  std::lock_guard<std::mutex> lock(Table().mu);
  Table().factories[protocol] = factory;
  return true;
}

FileSystem* FileSystem::GetInstance(const URI& path) {
  if (path.protocol.empty() || path.protocol == "file://") {
    return LocalFileSystem::GetInstance();
  }
  EnsureRemoteFileSystemsRegistered();
  FsTable& t = Table();
  std::lock_guard<std::mutex> lock(t.mu);
  auto it = t.factories.find(path.protocol);
  if (it == t.factories.end()) {
    LOG(FATAL) << "unknown filesystem protocol " + path.protocol;
  }
  const std::string key = path.protocol + path.host;
  auto inst = t.instances.find(key);
  if (inst != t.instances.end()) return inst->second;
  FileSystem* fs = it->second(path);
  t.instances[key] = fs;
  return fs;
}

}  // namespace io

InputSplit* InputSplit::Create(const char* uri_, unsigned part, unsigned nsplit,
                               const char* type) {
  return Create(uri_, nullptr, part, nsplit, type);
}

InputSplit* InputSplit::Create(const char* uri_, const char* index_uri_, unsigned part,
                               unsigned nsplit, const char* type, const bool shuffle,
                               const int seed, const size_t batch_size,
                               const bool recurse_directories) {
  using namespace io;  // NOLINT(*)
  URISpec spec(uri_, part, nsplit);
  if (spec.uri == "stdin") return new SingleFileSplit(spec.uri.c_str());
  CHECK(part < nsplit) << "invalid input parameter for InputSplit::Create";
  URI path(spec.uri.c_str());
  FileSystem* fs = FileSystem::GetInstance(path);
  InputSplitBase* split = nullptr;
  if (!std::strcmp(type, "text")) {
    split = new LineSplitter(fs, spec.uri.c_str(), part, nsplit, recurse_directories);
  } else if (!std::strcmp(type, "indexed_recordio")) {
    CHECK(index_uri_ != nullptr) << "need an index file to use indexed_recordio";
    URISpec index_spec(index_uri_, part, nsplit);
    split = new IndexedRecordIOSplitter(fs, spec.uri.c_str(), index_spec.uri.c_str(), part,
                                        nsplit, batch_size, shuffle, seed);
  } else if (!std::strcmp(type, "recordio")) {
    split = new RecordIOSplitter(fs, spec.uri.c_str(), part, nsplit, recurse_directories);
  } else {
    LOG(FATAL) << "unknown input split type " << type;
  }
  if (spec.cache_file.length() == 0) {
    return new ThreadedInputSplit(split, batch_size);
  }
  return new CachedInputSplit(split, spec.cache_file.c_str());
}

Stream* Stream::Create(const char* uri, const char* const flag, bool try_create) {
  io::URI path(uri);
  return io::FileSystem::GetInstance(path)->Open(path, flag, try_create);
}

SeekStream* SeekStream::CreateForRead(const char* uri, bool try_create) {
  io::URI path(uri);
  return io::FileSystem::GetInstance(path)->OpenForRead(path, try_create);
}

}  // namespace dmlc
