/*!
 * \file src/io/local_filesys.cc
 * \brief POSIX filesystem backend (see local_filesys.h).
 */
#include "./local_filesys.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <queue>

namespace dmlc {
namespace io {

namespace {
/*! \brief local path of a URI ("file://" stripped, host kept as path prefix) */
std::string LocalPath(const URI& path) {
  if (path.protocol == "file://") return path.host + path.name;
  return path.name;
}

/*! \brief FILE*-backed seekable stream with a large stdio buffer */
class FileStream : public SeekStream {
 public:
  FileStream(FILE* fp, bool use_stdio) : fp_(fp), use_stdio_(use_stdio) {
    if (!use_stdio_) std::setvbuf(fp_, nullptr, _IOFBF, 1 << 20);
  }
  ~FileStream() override {
    if (fp_ != nullptr && !use_stdio_) std::fclose(fp_);
  }
  size_t Read(void* ptr, size_t size) override { return std::fread(ptr, 1, size, fp_); }
  void Write(const void* ptr, size_t size) override {
    CHECK(std::fwrite(ptr, 1, size, fp_) == size)
        << "FileStream.Write incomplete: " << std::strerror(errno);
  }
  void Seek(size_t pos) override {
    CHECK(!fseeko(fp_, static_cast<off_t>(pos), SEEK_SET))
        << "FileStream.Seek failed: " << std::strerror(errno);
  }
  size_t Tell() override { return static_cast<size_t>(ftello(fp_)); }

 private:
  FILE* fp_;
  bool use_stdio_;
};
}  // namespace

FileInfo LocalFileSystem::GetPathInfo(const URI& path) {
  struct stat sb;
  const std::string p = LocalPath(path);
  if (stat(p.c_str(), &sb) == -1) {
    int errsv = errno;
    LOG(FATAL) << "LocalFileSystem.GetPathInfo: " << p << " error: " << std::strerror(errsv);
  }
  FileInfo ret;
  ret.path = path;
  ret.size = static_cast<size_t>(sb.st_size);
  ret.type = S_ISDIR(sb.st_mode) ? kDirectory : kFile;
  return ret;
}

void LocalFileSystem::ListDirectory(const URI& path, std::vector<FileInfo>* out_list) {
  const std::string dir = LocalPath(path);
  DIR* d = opendir(dir.c_str());
  if (d == nullptr) {
    int errsv = errno;
    LOG(FATAL) << "LocalFileSystem.ListDirectory " << dir << " error: " << std::strerror(errsv);
  }
  out_list->clear();
  std::vector<std::string> names;
  while (struct dirent* ent = readdir(d)) {
    if (!std::strcmp(ent->d_name, ".") || !std::strcmp(ent->d_name, "..")) continue;
    names.emplace_back(ent->d_name);
  }
  closedir(d);
  std::sort(names.begin(), names.end());
  for (const auto& n : names) {
    URI pp = path;
    if (!pp.name.empty() && pp.name.back() != '/') pp.name += '/';
    pp.name += n;
    out_list->push_back(this->GetPathInfo(pp));
  }
}

Stream* LocalFileSystem::Open(const URI& path, const char* const flag, bool allow_null) {
  bool use_stdio = false;
  FILE* fp = nullptr;
  const std::string fname = LocalPath(path);
  if (fname == "stdin") {
    use_stdio = true;
    fp = stdin;
  } else if (fname == "stdout") {
    use_stdio = true;
    fp = stdout;
  } else {
    std::string mode = flag;
    if (mode == "w") mode = "wb";
    if (mode == "r") mode = "rb";
    if (mode == "a") mode = "ab";
    fp = std::fopen(fname.c_str(), mode.c_str());
  }
  if (fp != nullptr) return new FileStream(fp, use_stdio);
  CHECK(allow_null) << " LocalFileSystem::Open \"" << fname << "\": " << std::strerror(errno);
  return nullptr;
}

SeekStream* LocalFileSystem::OpenForRead(const URI& path, bool allow_null) {
  return static_cast<SeekStream*>(this->Open(path, "r", allow_null));
}

int LocalFileSystem::OpenRawFd(const URI& path) {
  const std::string fname = LocalPath(path);
  int fd = ::open(fname.c_str(), O_RDONLY | O_CLOEXEC);
  CHECK(fd >= 0) << "open(" << fname << "): " << std::strerror(errno);
#ifdef POSIX_FADV_SEQUENTIAL
  posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
#endif
  return fd;
}

void FileSystem::ListDirectoryRecursive(const URI& path, std::vector<FileInfo>* out_list) {
  std::queue<URI> queue;
  out_list->clear();
  queue.push(path);
  while (!queue.empty()) {
    std::vector<FileInfo> dfiles;
    URI dir = queue.front();
    queue.pop();
    this->ListDirectory(dir, &dfiles);
    for (const auto& f : dfiles) {
      if (f.type == kDirectory) {
        queue.push(f.path);
      } else {
        out_list->push_back(f);
      }
    }
  }
}

}  // namespace io
}  // namespace dmlc
