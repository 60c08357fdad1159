/*!
 * \file dmlc/gpu/device_page_cache.h
 * \brief The `#cache` file of the GPU route: DiskRowIter's binary page cache
 *  (reference src/data/disk_row_iter.h:94-141, page format
 *  src/data/row_block.h:191-215) written from and DMA'd back into HBM.
 *
 *  A cache file is a sequence of RowBlockContainer<I>::Save pages -- vectors
 *  offset(size_t, page-local), label, weight, qid, field, index, value (u64
 *  count + raw elements each), then max_field and max_index (I).  Both the
 *  CPU DiskRowIter and this class flush a page as soon as its MemCostBytes()
 *  reaches 64 MiB, checked after every row, so for the same shard the two
 *  builders write the same bytes when every optional column (weight / qid /
 *  value) is carried by every row of the shard or by none.  Otherwise they
 *  may differ: the GPU route decides the optional columns per shard and
 *  prices a page with full-length columns, while the CPU RowBlockContainer
 *  fills them lazily (its MemCostBytes is lower mid-page, so its pages can
 *  hold more rows).  Either builder's file loads in either reader.
 *
 *  Loading is the MI355X fast path of a cached epoch: the file is mmap'ed and
 *  registered with hipHostRegister once (zero-copy, as the text route), every
 *  array of every page is one DMA straight into its place in a DeviceCSR --
 *  no parse, no host copy -- and one kernel rebases the page-local row
 *  pointers.  A binary page is ~half the bytes of its text, so a cached epoch
 *  moves ~2x the rows per second over the same PCIe link.  Remote or
 *  unregistrable files are read through dmlc::Stream into pinned staging.
 */
#ifndef DMLC_GPU_DEVICE_PAGE_CACHE_H_
#define DMLC_GPU_DEVICE_PAGE_CACHE_H_

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "./device_row_block.h"

namespace dmlc {
namespace gpu {

/*! \brief DiskRowIter's page size (reference disk_row_iter.h:33) */
constexpr size_t kCachePageBytes = 64UL << 20;

/*! \brief where one page's arrays lie in the cache file */
struct CachePage {
  size_t rows{0}, nnz{0};
  /*! \brief the page's byte range in the file */
  size_t begin{0}, end{0};
  /*! \brief file offsets of the first element of each array */
  size_t off_offset{0}, off_label{0}, off_weight{0}, off_qid{0}, off_field{0}, off_index{0},
      off_value{0};
  bool has_weight{false}, has_qid{false}, has_field{false}, has_value{false};
  uint64_t max_index{0}, max_field{0};
};

template <typename IndexType>
class DevicePageCache {
 public:
  ~DevicePageCache();
  /*!
   * \brief open an existing cache file; nullptr when it does not exist.
   *  Fails loudly on a malformed file.
   * \param device HIP device of the DeviceCSRs it loads (-1: current)
   */
  static std::unique_ptr<DevicePageCache> Open(const std::string& path, int device = -1);
  /*!
   * \brief write `csr` as cache pages (the RowBlockContainer<I>::Save format;
   *  page boundaries by the row-granular 64 MiB rule of DiskRowIter)
   * \return number of pages written
   */
  static size_t Write(const DeviceCSR<IndexType>& csr, const std::string& path,
                      size_t page_bytes = kCachePageBytes);
  /*! \brief replace out's contents with every page (synchronised before returning) */
  void Load(DeviceCSR<IndexType>* out);
  size_t rows() const { return rows_; }
  size_t nnz() const { return nnz_; }
  /*! \brief bytes of the cache file */
  size_t bytes() const { return bytes_; }
  /*! \brief true when loads DMA straight from the registered file mapping */
  bool zero_copy() const { return map_ != nullptr; }
  const std::vector<CachePage>& pages() const { return pages_; }
  uint64_t max_index() const { return max_index_; }
  uint64_t max_field() const { return max_field_; }

 private:
  DevicePageCache() = default;
  bool Index();
  void LoadStaged(DeviceCSR<IndexType>* out, hipStream_t s);
  void CopyPage(const CachePage& pg, const char* hp, size_t hp_file_off, DeviceCSR<IndexType>* out,
                size_t r0, size_t z0, hipStream_t s);
  std::string path_;
  int device_{0};
  std::vector<CachePage> pages_;
  size_t rows_{0}, nnz_{0}, bytes_{0};
  uint64_t max_index_{0}, max_field_{0};
  bool has_weight_{false}, has_qid_{false}, has_field_{false}, has_value_{false};
  // zero-copy mapping (local files)
  int fd_{-1};
  void* map_{nullptr};
  size_t map_len_{0};
  std::unique_ptr<Stream> stream_;
  DeviceBuffer page_table_;
  PinnedBuffer page_table_host_;
};

}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_GPU_DEVICE_PAGE_CACHE_H_
