/*!
 * \file src/io/uri_spec.h
 * \brief `path?k=v&k2=v2#cachefile` URI sugar.
 * Parity: reference `src/io/uri_spec.h:29-77` — `#cache` becomes cache_file
 * with `.split<N>.part<K>` appended when N != 1; `?k=v` pairs become args.
 */
#ifndef DMLC_IO_URI_SPEC_H_
#define DMLC_IO_URI_SPEC_H_

#include <dmlc/common.h>
#include <dmlc/logging.h>

#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace dmlc {
namespace io {

class URISpec {
 public:
  /*! \brief the plain uri (args and cache removed) */
  std::string uri;
  /*! \brief `?k=v` arguments */
  std::map<std::string, std::string> args;
  /*! \brief cache file name, empty when no `#` suffix */
  std::string cache_file;

  URISpec(const std::string& input, unsigned part_index, unsigned num_parts) {
    std::string rest = input;
    const size_t hash = rest.find('#');
    if (hash != std::string::npos) {
      std::string cache = rest.substr(hash + 1);
      rest = rest.substr(0, hash);
      CHECK(!cache.empty()) << "empty cache file name in uri " << input;
      if (num_parts != 1) {
        std::ostringstream os;
        os << cache << ".split" << num_parts << ".part" << part_index;
        cache = os.str();
      }
      cache_file = cache;
    }
    const size_t q = rest.find('?');
    if (q != std::string::npos) {
      const std::string query = rest.substr(q + 1);
      rest = rest.substr(0, q);
      for (const std::string& kv : Split(query, '&')) {
        if (kv.empty()) continue;
        const size_t eq = kv.find('=');
        CHECK(eq != std::string::npos && eq != 0)
            << "invalid uri argument \"" << kv << "\" in " << input
            << " (expected key=value)";
        args[kv.substr(0, eq)] = kv.substr(eq + 1);
      }
    }
    uri = rest;
  }
};

}  // namespace io
}  // namespace dmlc
#endif  // DMLC_IO_URI_SPEC_H_
