// dmlc_recordio: pack / unpack / index / count RecordIO files (any URI).
//
//   dmlc_recordio pack   <out.rec> <file>...       one record per input file
//   dmlc_recordio lines  <out.rec> <text-uri>      one record per text line
//   dmlc_recordio unpack <in.rec> <out-dir>        record k -> <out-dir>/<k>
//   dmlc_recordio index  <in.rec> <out.idx>        "key offset" per record, the
//                                                  input of indexed_recordio
//   dmlc_recordio count  <in.rec>                  records and payload bytes
//
// Format and escaping are dmlc's (`include/dmlc/recordio.h`, reference
// `src/recordio.cc:11-82`): payload words equal to the magic at 4-byte
// aligned positions are split into multi-part records.  The index format is
// the one IndexedRecordIOSplitter reads (`src/io/indexed_recordio_split.cc:43-61`).
#include <dmlc/io.h>
#include <dmlc/logging.h>
#include <dmlc/recordio.h>

#include <cstdio>
#include <memory>
#include <string>

namespace {
int Usage(const char* a) {
  std::fprintf(stderr,
               "usage: %s pack <out.rec> <file>... | lines <out.rec> <text-uri> |\n"
               "       %s unpack <in.rec> <out-dir> | index <in.rec> <out.idx> | count <in.rec>\n",
               a, a);
  return 2;
}

std::string ReadAll(const std::string& uri) {
  std::unique_ptr<dmlc::Stream> in(dmlc::Stream::Create(uri.c_str(), "r"));
  std::string out, buf(1 << 20, '\0');
  for (;;) {
    const size_t n = in->Read(&buf[0], buf.size());
    if (n == 0) return out;
    out.append(buf.data(), n);
  }
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) return Usage(argv[0]);
  const std::string cmd = argv[1];
  try {
    if (cmd == "pack" || cmd == "lines") {
      if (argc < 4) return Usage(argv[0]);
      std::unique_ptr<dmlc::Stream> out(dmlc::Stream::Create(argv[2], "w"));
      dmlc::RecordIOWriter w(out.get());
      size_t n = 0;
      if (cmd == "pack") {
        for (int i = 3; i < argc; ++i, ++n) w.WriteRecord(ReadAll(argv[i]));
      } else {
        const std::string text = ReadAll(argv[3]);
        size_t b = 0;
        while (b < text.size()) {
          size_t e = text.find('\n', b);
          if (e == std::string::npos) e = text.size();
          size_t t = e;
          if (t > b && text[t - 1] == '\r') --t;
          w.WriteRecord(text.data() + b, t - b);
          ++n;
          b = e + 1;
        }
      }
      std::fprintf(stderr, "packed %zu records (%zu escaped magic words)\n", n,
                   w.except_counter());
      return 0;
    }
    std::unique_ptr<dmlc::Stream> in(dmlc::Stream::Create(argv[2], "r"));
    dmlc::RecordIOReader r(in.get());
    std::string rec;
    if (cmd == "count") {
      size_t n = 0, bytes = 0;
      while (r.NextRecord(&rec)) {
        ++n;
        bytes += rec.size();
      }
      std::printf("%zu records, %zu payload bytes\n", n, bytes);
      return 0;
    }
    if (argc < 4) return Usage(argv[0]);
    if (cmd == "unpack") {
      size_t n = 0;
      while (r.NextRecord(&rec)) {
        const std::string path = std::string(argv[3]) + "/" + std::to_string(n++);
        std::unique_ptr<dmlc::Stream> o(dmlc::Stream::Create(path.c_str(), "w"));
        o->Write(rec.data(), rec.size());
      }
      std::fprintf(stderr, "unpacked %zu records\n", n);
      return 0;
    }
    if (cmd == "index") {
      // offsets come from a second reader over a seekable stream: the record
      // head is where the previous NextRecord stopped
      std::unique_ptr<dmlc::SeekStream> s(dmlc::SeekStream::CreateForRead(argv[2]));
      dmlc::RecordIOReader rs(s.get());
      std::unique_ptr<dmlc::Stream> o(dmlc::Stream::Create(argv[3], "w"));
      size_t key = 0;
      for (;;) {
        const size_t off = s->Tell();
        if (!rs.NextRecord(&rec)) break;
        const std::string line = std::to_string(key++) + "\t" + std::to_string(off) + "\n";
        o->Write(line.data(), line.size());
      }
      std::fprintf(stderr, "indexed %zu records\n", key);
      return 0;
    }
    return Usage(argv[0]);
  } catch (const dmlc::Error& e) {
    std::fprintf(stderr, "dmlc_recordio %s: %s\n", cmd.c_str(), e.what());
    return 1;
  }
}
