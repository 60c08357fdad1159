/*!
 * \file src/data.cc
 * \brief Parser / RowBlockIter factories and the parser registry.
 *
 * Parity: reference `src/data.cc` — CreateLibSVMParser / CreateLibFMParser /
 * CreateCSVParser (:21-60), CreateParser_ with type "auto" -> `?format=` or
 * libsvm (:62-85), CreateIter_ choosing DiskRowIter for `#cache` else
 * BasicRowIter (:87-107), uint32/uint64 specialisations (:112-147), registry
 * entries (:150-158).
 * Differences: CSV is registered for uint64 as well and threaded (§7.4 #4);
 * `?device=gpu[:k]` routes both factories to the MI355X path
 * (src/gpu/device_row_iter.cc: GPUParser per chunk, DeviceRowIter whole shard,
 * `#cache` through the same binary page file as DiskRowIter);
 * `?nthread=N` is honoured; RowBlockIter keeps `?k=v` args when a cache file
 * is used (the reference dropped them).
 */
#include <dmlc/data.h>
#include <dmlc/io.h>
#include <dmlc/registry.h>

#include <cstdlib>
#include <string>

#include "./data/basic_row_iter.h"
#include "./data/csv_parser.h"
#include "./data/device_route.h"
#include "./data/disk_row_iter.h"
#include "./data/libfm_parser.h"
#include "./data/libsvm_parser.h"
#include "./data/parser.h"
#include "./io/uri_spec.h"

namespace dmlc {
namespace data {

namespace {
int NThreadArg(const std::map<std::string, std::string>& args) {
  auto it = args.find("nthread");
  return it == args.end() ? 0 : std::atoi(it->second.c_str());
}
}  // namespace

template <typename IndexType>
Parser<IndexType>* CreateLibSVMParser(const std::string& path,
                                      const std::map<std::string, std::string>& args,
                                      unsigned part_index, unsigned num_parts) {
  InputSplit* source = InputSplit::Create(path.c_str(), part_index, num_parts, "text");
  auto* parser = new LibSVMParser<IndexType>(source, NThreadArg(args));
  return new ThreadedParser<IndexType>(parser);
}

template <typename IndexType>
Parser<IndexType>* CreateLibFMParser(const std::string& path,
                                     const std::map<std::string, std::string>& args,
                                     unsigned part_index, unsigned num_parts) {
  InputSplit* source = InputSplit::Create(path.c_str(), part_index, num_parts, "text");
  auto* parser = new LibFMParser<IndexType>(source, NThreadArg(args));
  return new ThreadedParser<IndexType>(parser);
}

template <typename IndexType>
Parser<IndexType>* CreateCSVParser(const std::string& path,
                                   const std::map<std::string, std::string>& args,
                                   unsigned part_index, unsigned num_parts) {
  InputSplit* source = InputSplit::Create(path.c_str(), part_index, num_parts, "text");
  auto* parser = new CSVParser<IndexType>(source, args, NThreadArg(args));
  return new ThreadedParser<IndexType>(parser);
}

template <typename IndexType>
inline Parser<IndexType>* CreateParser_(const char* uri_, unsigned part_index,
                                        unsigned num_parts, const char* type) {
  std::string ptype = type;
  io::URISpec spec(uri_, part_index, num_parts);
  if (ptype == "auto") {
    auto it = spec.args.find("format");
    ptype = it != spec.args.end() ? it->second : "libsvm";
  }
  if (RoutesToDevice(spec.args)) {
    CHECK(DeviceRoute<IndexType>::parser != nullptr) << "device=gpu: the GPU path is not built in";
    return DeviceRoute<IndexType>::parser(spec.uri, spec.args, part_index, num_parts, ptype);
  }
  const ParserFactoryReg<IndexType>* e = Registry<ParserFactoryReg<IndexType>>::Find(ptype);
  if (e == nullptr) {
    LOG(FATAL) << "Unknown data type " << ptype;
  }
  return (*e->body)(spec.uri, spec.args, part_index, num_parts);
}

template <typename IndexType>
inline RowBlockIter<IndexType>* CreateIter_(const char* uri_, unsigned part_index,
                                            unsigned num_parts, const char* type) {
  io::URISpec spec(uri_, part_index, num_parts);
  if (RoutesToDevice(spec.args)) {
    std::string ptype = type;
    if (ptype == "auto") {
      auto it = spec.args.find("format");
      ptype = it != spec.args.end() ? it->second : "libsvm";
    }
    CHECK(DeviceRoute<IndexType>::iter != nullptr) << "device=gpu: the GPU path is not built in";
    // `#cache` is honoured on this route too (DevicePageCache: same page file)
    return DeviceRoute<IndexType>::iter(spec.uri, spec.args, part_index, num_parts, ptype,
                                        spec.cache_file);
  }
  std::string parser_uri = uri_;
  const size_t hash = parser_uri.find('#');
  if (hash != std::string::npos) parser_uri = parser_uri.substr(0, hash);
  Parser<IndexType>* parser =
      CreateParser_<IndexType>(parser_uri.c_str(), part_index, num_parts, type);
  if (!spec.cache_file.empty()) {
    return new DiskRowIter<IndexType>(parser, spec.cache_file.c_str(), true);
  }
  return new BasicRowIter<IndexType>(parser);
}

DMLC_REGISTER_PARAMETER(CSVParserParam);

bool RoutesToDevice(const std::map<std::string, std::string>& args) {
  auto it = args.find("device");
  return it != args.end() && it->second.compare(0, 3, "gpu") == 0;
}
template <typename I>
typename DeviceRoute<I>::ParserFn DeviceRoute<I>::parser = nullptr;
template <typename I>
typename DeviceRoute<I>::IterFn DeviceRoute<I>::iter = nullptr;
template struct DeviceRoute<uint32_t>;
template struct DeviceRoute<uint64_t>;
}  // namespace data

template <>
RowBlockIter<uint32_t>* RowBlockIter<uint32_t>::Create(const char* uri, unsigned part_index,
                                                       unsigned num_parts, const char* type) {
  return data::CreateIter_<uint32_t>(uri, part_index, num_parts, type);
}
template <>
RowBlockIter<uint64_t>* RowBlockIter<uint64_t>::Create(const char* uri, unsigned part_index,
                                                       unsigned num_parts, const char* type) {
  return data::CreateIter_<uint64_t>(uri, part_index, num_parts, type);
}
template <>
Parser<uint32_t>* Parser<uint32_t>::Create(const char* uri, unsigned part_index,
                                           unsigned num_parts, const char* type) {
  return data::CreateParser_<uint32_t>(uri, part_index, num_parts, type);
}
template <>
Parser<uint64_t>* Parser<uint64_t>::Create(const char* uri, unsigned part_index,
                                           unsigned num_parts, const char* type) {
  return data::CreateParser_<uint64_t>(uri, part_index, num_parts, type);
}

DMLC_REGISTRY_ENABLE(ParserFactoryReg<uint32_t>);
DMLC_REGISTRY_ENABLE(ParserFactoryReg<uint64_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, libsvm, data::CreateLibSVMParser<uint32_t>)
    .describe("LibSVM text: label[:weight] [qid:n] index[:value] ...");
DMLC_REGISTER_DATA_PARSER(uint64_t, libsvm, data::CreateLibSVMParser<uint64_t>)
    .describe("LibSVM text, 64-bit feature indices");
DMLC_REGISTER_DATA_PARSER(uint32_t, libfm, data::CreateLibFMParser<uint32_t>)
    .describe("LibFM text: label[:weight] field:index[:value] ...");
DMLC_REGISTER_DATA_PARSER(uint64_t, libfm, data::CreateLibFMParser<uint64_t>)
    .describe("LibFM text, 64-bit indices");
DMLC_REGISTER_DATA_PARSER(uint32_t, csv, data::CreateCSVParser<uint32_t>)
    .describe("dense CSV (?label_column=k&delimiter=,)");
DMLC_REGISTER_DATA_PARSER(uint64_t, csv, data::CreateCSVParser<uint64_t>)
    .describe("dense CSV, 64-bit indices");

}  // namespace dmlc
