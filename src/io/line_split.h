/*!
 * \file src/io/line_split.h
 * \brief Text splitter: records are lines.
 * Parity: reference `src/io/line_split.h:20-35`, `src/io/line_split.cc:9-55`
 * (SeekRecordBegin skips to after the next EOL run; a record is a line plus
 * its EOL run whose last EOL byte is overwritten with '\0').
 */
#ifndef DMLC_IO_LINE_SPLIT_H_
#define DMLC_IO_LINE_SPLIT_H_

#include "./input_split_base.h"

namespace dmlc {
namespace io {

class LineSplitter : public InputSplitBase {
 public:
  LineSplitter(FileSystem* fs, const char* uri, unsigned rank, unsigned nsplit,
               bool recurse_directories = false) {
    this->Init(fs, uri, 1, recurse_directories);
    this->ResetPartition(rank, nsplit);
  }
  bool IsTextParser() const override { return true; }
  bool ExtractNextRecord(Blob* out_rec, Chunk* chunk) override;
  const char* FindLastRecordBegin(const char* begin, const char* end) override;

 protected:
  size_t SeekRecordBegin(Stream* fi) override;
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_LINE_SPLIT_H_
