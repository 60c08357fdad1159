/*!
 * \file src/data/device_route.h
 * \brief `?device=gpu` routing of the public Parser / RowBlockIter factories
 *  to the MI355X ingestion path (implemented in src/gpu/device_row_iter.cc).
 */
#ifndef DMLC_DATA_DEVICE_ROUTE_H_
#define DMLC_DATA_DEVICE_ROUTE_H_

#include <dmlc/data.h>

#include <map>
#include <string>

namespace dmlc {
namespace data {

/*! \brief true when the URI args ask for the GPU path (device=gpu[:k]) */
bool RoutesToDevice(const std::map<std::string, std::string>& args);

/*!
 * \brief factories of the GPU path, installed by src/gpu/device_row_iter.cc at
 *  static-initialisation time (null in CPU-only / sanitizer builds, where
 *  `device=gpu` fails loudly instead)
 */
template <typename IndexType>
struct DeviceRoute {
  typedef Parser<IndexType>* (*ParserFn)(const std::string& uri,
                                         const std::map<std::string, std::string>& args,
                                         unsigned part, unsigned nparts, const std::string& type);
  /*! cache_file: the `#cache` page file ("" for none), as DiskRowIter's */
  typedef RowBlockIter<IndexType>* (*IterFn)(const std::string& uri,
                                             const std::map<std::string, std::string>& args,
                                             unsigned part, unsigned nparts,
                                             const std::string& type,
                                             const std::string& cache_file);
  static ParserFn parser;
  static IterFn iter;
};

}  // namespace data
}  // namespace dmlc
#endif  // DMLC_DATA_DEVICE_ROUTE_H_
