/*!
 * \file src/gpu/device_page_cache.cc
 * \brief DevicePageCache: DiskRowIter's page cache written from, and DMA'd
 *  straight back into, an HBM-resident DeviceCSR (see the header).
 *
 *  Reference: src/data/disk_row_iter.h:94-141 (BuildCache / TryLoadCache),
 *  src/data/row_block.h:191-215 (RowBlockContainer::Save / Load).
 */
#include <dmlc/gpu/device_page_cache.h>
#include <dmlc/io.h>
#include <dmlc/logging.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

#include "../io/filesys.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {

namespace {
/*! \brief DiskRowIter page MemCostBytes() of `rows` rows / `nnz` entries
 *  (RowBlockContainer<I>::MemCostBytes with the shard's column set) */
template <typename IndexType>
size_t PageCost(size_t rows, size_t nnz, bool w, bool q, bool f, bool v) {
  return (rows + 1) * sizeof(size_t) + rows * sizeof(float) + (w ? rows * sizeof(float) : 0) +
         (q ? rows * sizeof(uint64_t) : 0) + (f ? nnz * sizeof(IndexType) : 0) +
         nnz * sizeof(IndexType) + (v ? nnz * sizeof(float) : 0);
}

bool IsLocal(const std::string& path) {
  io::URI u(path.c_str());
  return u.protocol.empty() || u.protocol == "file://";
}
}  // namespace

template <typename IndexType>
DevicePageCache<IndexType>::~DevicePageCache() {
  if (stream_ != nullptr) (void)hipStreamSynchronize(stream_->get());
  if (map_ != nullptr) {
    (void)hipHostUnregister(map_);
    munmap(map_, map_len_);
  }
  if (fd_ >= 0) ::close(fd_);
}

template <typename IndexType>
std::unique_ptr<DevicePageCache<IndexType>> DevicePageCache<IndexType>::Open(
    const std::string& path, int device) {
  std::unique_ptr<DevicePageCache> c(new DevicePageCache());
  c->path_ = path;
  if (device < 0) DMLC_HIP_CHECK(hipGetDevice(&device));
  c->device_ = device;
  if (IsLocal(path)) {
    const std::string name = io::URI(path.c_str()).name;
    c->fd_ = ::open(name.c_str(), O_RDONLY);
    if (c->fd_ < 0) return nullptr;
    struct stat st;
    CHECK_EQ(fstat(c->fd_, &st), 0) << "cannot stat cache file " << path;
    c->bytes_ = static_cast<size_t>(st.st_size);
    if (c->bytes_ != 0) {
      void* m = mmap(nullptr, c->bytes_, PROT_READ, MAP_SHARED | MAP_POPULATE, c->fd_, 0);
      if (m != MAP_FAILED) {
        DMLC_HIP_CHECK(hipSetDevice(device));
        if (hipHostRegister(m, c->bytes_, hipHostRegisterReadOnly) == hipSuccess) {
          c->map_ = m;
          c->map_len_ = c->bytes_;
        } else {
          (void)hipGetLastError();
          munmap(m, c->bytes_);
        }
      }
    }
  } else {
    std::unique_ptr<SeekStream> fi(SeekStream::CreateForRead(path.c_str(), true));
    if (fi == nullptr) return nullptr;
  }
  CHECK(c->Index()) << "malformed page cache file " << path;
  DMLC_HIP_CHECK(hipSetDevice(device));
  c->stream_.reset(new Stream());
  return c;
}

/*!
 * \brief walk the page headers (a few reads per 64 MiB page): every array's
 *  file offset, counts checked against each other like RowBlockContainer::Load
 *  + GetBlock would
 */
template <typename IndexType>
bool DevicePageCache<IndexType>::Index() {
  std::unique_ptr<SeekStream> fi;
  if (map_ == nullptr) {
    fi.reset(SeekStream::CreateForRead(path_.c_str(), false));
    if (!IsLocal(path_)) {
      io::URI u(path_.c_str());
      bytes_ = io::FileSystem::GetInstance(u)->GetPathInfo(u).size;
    }
  }
  auto read_at = [&](size_t pos, void* dst, size_t n) -> bool {
    if (pos + n > bytes_) return false;
    if (map_ != nullptr) {
      std::memcpy(dst, static_cast<const char*>(map_) + pos, n);
      return true;
    }
    fi->Seek(pos);
    return fi->Read(dst, n) == n;
  };
  size_t pos = 0;
  pages_.clear();
  rows_ = nnz_ = 0;
  while (pos < bytes_) {
    CachePage pg;
    pg.begin = pos;
    uint64_t cnt = 0;
    // vector<T> = u64 count + count * sizeof(T)
    auto vec = [&](size_t esize, size_t* off) -> bool {
      if (!read_at(pos, &cnt, sizeof(cnt))) return false;
      *off = pos + sizeof(cnt);
      pos = *off + cnt * esize;
      return pos <= bytes_;
    };
    if (!vec(sizeof(size_t), &pg.off_offset) || cnt == 0) return false;
    pg.rows = cnt - 1;
    if (!vec(sizeof(float), &pg.off_label) || cnt != pg.rows) return false;
    if (!vec(sizeof(float), &pg.off_weight) || (cnt != 0 && cnt != pg.rows)) return false;
    pg.has_weight = cnt != 0 && pg.rows != 0;
    if (!vec(sizeof(uint64_t), &pg.off_qid) || (cnt != 0 && cnt != pg.rows)) return false;
    pg.has_qid = cnt != 0 && pg.rows != 0;
    if (!vec(sizeof(IndexType), &pg.off_field)) return false;
    const uint64_t nfield = cnt;
    if (!vec(sizeof(IndexType), &pg.off_index)) return false;
    pg.nnz = cnt;
    if (nfield != 0 && nfield != pg.nnz) return false;
    pg.has_field = nfield != 0 && pg.nnz != 0;
    if (!vec(sizeof(float), &pg.off_value) || (cnt != 0 && cnt != pg.nnz)) return false;
    pg.has_value = cnt != 0 && pg.nnz != 0;
    IndexType mf = 0, mi = 0;
    if (!read_at(pos, &mf, sizeof(mf)) || !read_at(pos + sizeof(mf), &mi, sizeof(mi))) return false;
    pos += 2 * sizeof(IndexType);
    pg.end = pos;
    uint64_t last = 0;
    if (!read_at(pg.off_offset + pg.rows * sizeof(size_t), &last, sizeof(last)) || last != pg.nnz) {
      return false;
    }
    pg.max_field = mf;
    pg.max_index = mi;
    rows_ += pg.rows;
    nnz_ += pg.nnz;
    max_index_ = std::max<uint64_t>(max_index_, mi);
    max_field_ = std::max<uint64_t>(max_field_, mf);
    has_weight_ |= pg.has_weight;
    has_qid_ |= pg.has_qid;
    has_field_ |= pg.has_field;
    has_value_ |= pg.has_value;
    pages_.push_back(pg);
  }
  return true;
}

template <typename IndexType>
void DevicePageCache<IndexType>::Load(DeviceCSR<IndexType>* out) {
  ScopedRange range("DevicePageCache::Load");
  DMLC_HIP_CHECK(hipSetDevice(device_));
  hipStream_t s = stream_->get();
  out->Clear();
  out->device_ = device_;
  out->Reserve(std::max<size_t>(rows_, 1), std::max<size_t>(nnz_, 1), has_field_, s);
  if (has_weight_) out->EnableWeight(s);
  if (has_qid_) out->EnableQid(s);
  // page table for the row-pointer rebase: cumulative row ends, nnz bases
  const size_t np = pages_.size();
  page_table_host_.Reserve(std::max<size_t>(2 * np, 1) * sizeof(uint64_t));
  page_table_.Reserve(std::max<size_t>(2 * np, 1) * sizeof(uint64_t));
  uint64_t* tab = page_table_host_.get<uint64_t>();
  DMLC_HIP_CHECK(hipStreamSynchronize(s));  // the host table is free to rewrite
  {
    uint64_t r = 0, z = 0;
    for (size_t p = 0; p < np; ++p) {
      tab[np + p] = z;
      r += pages_[p].rows;
      z += pages_[p].nnz;
      tab[p] = r;
    }
  }
  DMLC_HIP_CHECK(hipMemcpyAsync(page_table_.get(), tab, 2 * np * sizeof(uint64_t),
                                hipMemcpyHostToDevice, s));
  DMLC_HIP_CHECK(hipMemsetAsync(out->offset(), 0, sizeof(uint64_t), s));
  if (map_ == nullptr) {
    LoadStaged(out, s);
  } else {
    const char* base = static_cast<const char*>(map_);
    size_t r0 = 0, z0 = 0;
    for (const CachePage& pg : pages_) {
      CopyPage(pg, base, 0, out, r0, z0, s);
      r0 += pg.rows;
      z0 += pg.nnz;
    }
  }
  if (rows_ != 0) {
    LaunchPageRebase(out->offset(), rows_, page_table_.get<uint64_t>(),
                     page_table_.get<uint64_t>() + np, static_cast<int>(np), s);
  }
  out->rows_ = rows_;
  out->nnz_ = nnz_;
  out->max_index_ = max_index_;
  out->max_field_ = max_field_;
  out->has_weight_ = has_weight_;
  out->has_qid_ = has_qid_;
  out->has_field_ = has_field_;
  out->has_value_ = has_value_;
  DMLC_HIP_CHECK(hipStreamSynchronize(s));
}

/*!
 * \brief every array of one page into its place in `out`: host bytes of the
 *  page's file range [pg.begin, pg.end) start at hp + (pg.begin - hp_file_off).
 *  Columns the shard has but this page lacks get their neutral value.
 */
template <typename IndexType>
void DevicePageCache<IndexType>::CopyPage(const CachePage& pg, const char* hp, size_t hp_file_off,
                                          DeviceCSR<IndexType>* out, size_t r0, size_t z0,
                                          hipStream_t s) {
  auto h2d = [&](void* dst, size_t file_off, size_t bytes) {
    if (bytes == 0) return;
    DMLC_HIP_CHECK(hipMemcpyAsync(dst, hp + (file_off - hp_file_off), bytes,
                                  hipMemcpyHostToDevice, s));
  };
  // row pointers: the page's entries 1..rows (entry 0 is its 0); rebased later
  h2d(out->offset() + r0 + 1, pg.off_offset + sizeof(size_t), pg.rows * sizeof(size_t));
  h2d(out->label() + r0, pg.off_label, pg.rows * sizeof(float));
  if (has_weight_) {
    if (pg.has_weight) {
      h2d(out->weight() + r0, pg.off_weight, pg.rows * sizeof(float));
    } else if (pg.rows != 0) {
      LaunchFill(out->weight() + r0, pg.rows, 1.0f, s);
    }
  }
  if (has_qid_) {
    if (pg.has_qid) {
      h2d(out->qid() + r0, pg.off_qid, pg.rows * sizeof(uint64_t));
    } else if (pg.rows != 0) {
      DMLC_HIP_CHECK(hipMemsetAsync(out->qid() + r0, 0, pg.rows * sizeof(uint64_t), s));
    }
  }
  if (has_field_) {
    if (pg.has_field) {
      h2d(out->field() + z0, pg.off_field, pg.nnz * sizeof(IndexType));
    } else if (pg.nnz != 0) {
      DMLC_HIP_CHECK(hipMemsetAsync(out->field() + z0, 0, pg.nnz * sizeof(IndexType), s));
    }
  }
  h2d(out->index() + z0, pg.off_index, pg.nnz * sizeof(IndexType));
  if (has_value_) {
    if (pg.has_value) {
      h2d(out->value() + z0, pg.off_value, pg.nnz * sizeof(float));
    } else if (pg.nnz != 0) {
      LaunchFill(out->value() + z0, pg.nnz, 1.0f, s);
    }
  }
}

/*!
 * \brief remote / unregistrable files: pages are read through dmlc::Stream into
 *  two pinned staging buffers, page k + 1 read while page k's DMAs run
 */
template <typename IndexType>
void DevicePageCache<IndexType>::LoadStaged(DeviceCSR<IndexType>* out, hipStream_t s) {
  std::unique_ptr<SeekStream> fi(SeekStream::CreateForRead(path_.c_str(), false));
  size_t biggest = 0;
  for (const CachePage& pg : pages_) biggest = std::max(biggest, pg.end - pg.begin);
  PinnedBuffer stage[2];
  Event done[2];
  bool used[2] = {false, false};
  for (auto& b : stage) b.Reserve(std::max<size_t>(biggest, 1));
  size_t r0 = 0, z0 = 0;
  for (size_t p = 0; p < pages_.size(); ++p) {
    const CachePage& pg = pages_[p];
    const int k = static_cast<int>(p & 1);
    if (used[k]) done[k].Synchronize();  // its previous page's DMAs are complete
    fi->Seek(pg.begin);
    CHECK_EQ(fi->Read(stage[k].get(), pg.end - pg.begin), pg.end - pg.begin)
        << "short read of page cache " << path_;
    CopyPage(pg, stage[k].get<char>(), pg.begin, out, r0, z0, s);
    done[k].Record(s);
    used[k] = true;
    r0 += pg.rows;
    z0 += pg.nnz;
  }
  // the last pages' DMAs read from the staging buffers: done before they go
  for (int k = 0; k < 2; ++k) {
    if (used[k]) done[k].Synchronize();
  }
}

template <typename IndexType>
size_t DevicePageCache<IndexType>::Write(const DeviceCSR<IndexType>& csr, const std::string& path,
                                         size_t page_bytes) {
  ScopedRange range("DevicePageCache::Write");
  const DeviceRowBlock<IndexType> v = csr.View();
  const HostCSR<IndexType> h = CopyToHost(v);
  const bool w = !h.weight.empty(), q = !h.qid.empty(), f = v.field != nullptr,
             val = v.value != nullptr;
  std::unique_ptr<dmlc::Stream> fo(dmlc::Stream::Create(path.c_str(), "w"));
  const size_t n = h.label.size();
  std::vector<size_t> off;
  size_t pages = 0;
  auto put_vec = [&](const void* p, size_t count, size_t esize) {
    const uint64_t c = count;
    fo->Write(&c, sizeof(c));
    if (count != 0) fo->Write(p, count * esize);
  };
  auto flush = [&](size_t r0, size_t r1) {
    const size_t z0 = h.offset[r0], z1 = h.offset[r1];
    off.resize(r1 - r0 + 1);
    for (size_t r = r0; r <= r1; ++r) off[r - r0] = h.offset[r] - z0;
    IndexType mi = 0, mf = 0;
    for (size_t j = z0; j < z1; ++j) mi = std::max(mi, h.index[j]);
    if (f) {
      for (size_t j = z0; j < z1; ++j) mf = std::max(mf, h.field[j]);
    }
    put_vec(off.data(), off.size(), sizeof(size_t));
    put_vec(h.label.data() + r0, r1 - r0, sizeof(float));
    put_vec(w ? h.weight.data() + r0 : nullptr, w ? r1 - r0 : 0, sizeof(float));
    put_vec(q ? h.qid.data() + r0 : nullptr, q ? r1 - r0 : 0, sizeof(uint64_t));
    put_vec(f ? h.field.data() + z0 : nullptr, f ? z1 - z0 : 0, sizeof(IndexType));
    put_vec(h.index.data() + z0, z1 - z0, sizeof(IndexType));
    put_vec(val ? h.value.data() + z0 : nullptr, val ? z1 - z0 : 0, sizeof(float));
    fo->Write(&mf, sizeof(mf));
    fo->Write(&mi, sizeof(mi));
    ++pages;
  };
  // DiskRowIter's rule, row-granular: a page is flushed as soon as its
  // MemCostBytes() reaches page_bytes after a row is appended
  size_t r0 = 0;
  for (size_t r = 0; r < n; ++r) {
    if (PageCost<IndexType>(r + 1 - r0, h.offset[r + 1] - h.offset[r0], w, q, f, val) >=
        page_bytes) {
      flush(r0, r + 1);
      r0 = r + 1;
    }
  }
  if (r0 < n) flush(r0, n);
  return pages;
}

template class DevicePageCache<uint32_t>;
template class DevicePageCache<uint64_t>;

}  // namespace gpu
}  // namespace dmlc
