// dmlc_fs: filesystem CLI over every URI scheme the runtime serves
// (local, s3://, http(s)://, azure://, hdfs://).
//
//   dmlc_fs ls   <uri>              list a directory (or stat a file)
//   dmlc_fs lsr  <uri>              recursive listing
//   dmlc_fs stat <uri>              type and size
//   dmlc_fs cat  <uri>              stream the object to stdout
//   dmlc_fs cp   <src-uri> <dst-uri> copy through Stream (any scheme -> any scheme)
//
// The reference ships the same functionality as a manual test driver
// (`test/filesys_test.cc:8-59`: ls / cat / cp); here it is a product tool.
// Copies use 64 MiB reads so remote sources take the direct-to-buffer
// ranged-GET path.
#include <dmlc/io.h>
#include <dmlc/logging.h>
#include <dmlc/timer.h>

#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../src/io/filesys.h"

namespace {
using dmlc::io::FileInfo;
using dmlc::io::FileSystem;
using dmlc::io::URI;

void PrintInfo(const FileInfo& f) {
  std::printf("%s\t%zu\t%s\n", f.type == dmlc::io::kDirectory ? "dir" : "file", f.size,
              f.path.str().c_str());
}

int Usage(const char* argv0) {
  std::fprintf(stderr, "usage: %s ls|lsr|stat|cat <uri>\n       %s cp <src> <dst>\n", argv0,
               argv0);
  return 2;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) return Usage(argv[0]);
  const std::string cmd = argv[1];
  try {
    URI path(argv[2]);
    if (cmd == "ls" || cmd == "lsr" || cmd == "stat") {
      FileSystem* fs = FileSystem::GetInstance(path);
      FileInfo info = fs->GetPathInfo(path);
      if (cmd == "stat" || info.type == dmlc::io::kFile) {
        PrintInfo(info);
        return 0;
      }
      std::vector<FileInfo> items;
      if (cmd == "lsr") {
        fs->ListDirectoryRecursive(path, &items);
      } else {
        fs->ListDirectory(path, &items);
      }
      for (const auto& f : items) PrintInfo(f);
      return 0;
    }
    std::vector<char> buf(64UL << 20);
    if (cmd == "cat") {
      std::unique_ptr<dmlc::Stream> in(dmlc::Stream::Create(argv[2], "r"));
      for (;;) {
        const size_t n = in->Read(buf.data(), buf.size());
        if (n == 0) break;
        CHECK_EQ(std::fwrite(buf.data(), 1, n, stdout), n) << "write to stdout failed";
      }
      std::fflush(stdout);
      return 0;
    }
    if (cmd == "cp") {
      if (argc < 4) return Usage(argv[0]);
      const double t0 = dmlc::GetTime();
      std::unique_ptr<dmlc::Stream> in(dmlc::Stream::Create(argv[2], "r"));
      std::unique_ptr<dmlc::Stream> out(dmlc::Stream::Create(argv[3], "w"));
      size_t total = 0;
      for (;;) {
        const size_t n = in->Read(buf.data(), buf.size());
        if (n == 0) break;
        out->Write(buf.data(), n);
        total += n;
      }
      out.reset();  // flush / complete multipart uploads
      const double dt = dmlc::GetTime() - t0;
      std::fprintf(stderr, "copied %zu bytes in %.3f s (%.1f MB/s)\n", total, dt,
                   dt > 0 ? total / dt / 1e6 : 0.0);
      return 0;
    }
    return Usage(argv[0]);
  } catch (const dmlc::Error& e) {
    std::fprintf(stderr, "dmlc_fs %s: %s\n", cmd.c_str(), e.what());
    return 1;
  }
}
