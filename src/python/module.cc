/*!
 * \file src/python/module.cc
 * \brief pybind11 bindings: `dmlc_core_amd._dmlc`.
 *
 * Exposes the native runtime to Python: CPU parsers / InputSplit / RecordIO /
 * streams (host RowBlocks as numpy arrays), the GPU DeviceParser whose HBM
 * CSR arrays are handed to PyTorch zero-copy through DLPack capsules, and the
 * HIP feature kernels.  No Python fallback exists for any of these: if the
 * extension cannot load, importing the ops fails loudly.
 */
#include <dmlc/data.h>
#include <dmlc/fault.h>
#include <dmlc/dist/communicator.h>
#include <dmlc/dist/tracker_client.h>
#include <dmlc/gpu/device_page_cache.h>
#include <dmlc/gpu/device_parser.h>
#include <dmlc/gpu/device_recordio.h>
#include <dmlc/gpu/hip_utils.h>
#include <dmlc/input_split_shuffle.h>
#include <dmlc/io.h>
#include <dmlc/logging.h>
#include <dmlc/recordio.h>
#include <dmlc/synthetic.h>
#include <dmlc/timer.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <string>
#include <vector>

#include "../gpu/kernels.h"
#include "../io/http.h"
#include "../io/line_split.h"
#include "../io/recordio_split.h"
#include "../io/shard_reader.h"
#include "./dlpack.h"

namespace py = pybind11;
using namespace dmlc;  // NOLINT

namespace {

// ------------------------------------------------------------------ dlpack
struct DLCtx {
  std::shared_ptr<void> owner;
  std::vector<int64_t> shape;
};

void DLDeleter(DLManagedTensor* t) {
  delete static_cast<DLCtx*>(t->manager_ctx);
  delete t;
}

void CapsuleDeleter(PyObject* cap) {
  // only delete if the consumer did not take ownership (renamed capsule)
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (t != nullptr && t->deleter != nullptr) t->deleter(t);
  }
}

template <typename T>
DLDataType DType() {
  DLDataType d;
  d.lanes = 1;
  d.bits = sizeof(T) * 8;
  d.code = std::is_floating_point<T>::value ? kDLFloat
                                            : (std::is_signed<T>::value ? kDLInt : kDLUInt);
  return d;
}

template <typename T>
py::object ToCapsule(const T* ptr, int64_t n, int device, std::shared_ptr<void> owner) {
  auto* ctx = new DLCtx();
  ctx->owner = std::move(owner);
  ctx->shape = {n};
  auto* t = new DLManagedTensor();
  t->dl_tensor.data = const_cast<T*>(ptr);
  t->dl_tensor.device = DLDevice{kDLROCM, device};
  t->dl_tensor.ndim = 1;
  t->dl_tensor.dtype = DType<T>();
  t->dl_tensor.shape = ctx->shape.data();
  t->dl_tensor.strides = nullptr;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = ctx;
  t->deleter = DLDeleter;
  return py::reinterpret_steal<py::object>(PyCapsule_New(t, "dltensor", CapsuleDeleter));
}

template <typename T>
py::array_t<T> ToNumpy(const T* ptr, size_t n) {
  py::array_t<T> a(n);
  if (n != 0) std::memcpy(a.mutable_data(), ptr, n * sizeof(T));
  return a;
}

// --------------------------------------------------------------- host data
template <typename I>
py::dict BlockToDict(const RowBlock<I>& b) {
  py::dict d;
  const size_t nnz = b.offset[b.size] - b.offset[0];
  std::vector<uint64_t> off(b.size + 1);
  for (size_t i = 0; i <= b.size; ++i) off[i] = b.offset[i] - b.offset[0];
  d["offset"] = ToNumpy(off.data(), off.size());
  d["label"] = ToNumpy(b.label, b.size);
  d["weight"] = b.weight ? py::object(ToNumpy(b.weight, b.size)) : py::none();
  d["qid"] = b.qid ? py::object(ToNumpy(b.qid, b.size)) : py::none();
  d["field"] = b.field ? py::object(ToNumpy(b.field + b.offset[0], nnz)) : py::none();
  d["index"] = ToNumpy(b.index + b.offset[0], nnz);
  d["value"] = b.value ? py::object(ToNumpy(b.value + b.offset[0], nnz)) : py::none();
  return d;
}

template <typename I>
class PyParser {
 public:
  PyParser(const std::string& uri, unsigned part, unsigned nparts, const std::string& type) {
    py::gil_scoped_release nogil;
    p_.reset(Parser<I>::Create(uri.c_str(), part, nparts, type.c_str()));
  }
  ~PyParser() {
    py::gil_scoped_release nogil;
    p_.reset();
  }
  bool Next() {
    py::gil_scoped_release nogil;
    return p_->Next();
  }
  py::dict Value() { return BlockToDict(p_->Value()); }
  void BeforeFirst() { p_->BeforeFirst(); }
  size_t BytesRead() const { return p_->BytesRead(); }
  /*! \brief parse everything, return (rows, nnz, seconds) without copying */
  py::tuple Drain() {
    size_t rows = 0, nnz = 0;
    double t0 = GetTime();
    {
      py::gil_scoped_release nogil;
      while (p_->Next()) {
        const auto& b = p_->Value();
        rows += b.size;
        nnz += b.offset[b.size] - b.offset[0];
      }
    }
    return py::make_tuple(rows, nnz, GetTime() - t0);
  }

 private:
  std::unique_ptr<Parser<I>> p_;
};

template <typename I>
class PyRowBlockIter {
 public:
  PyRowBlockIter(const std::string& uri, unsigned part, unsigned nparts, const std::string& type) {
    py::gil_scoped_release nogil;
    it_.reset(RowBlockIter<I>::Create(uri.c_str(), part, nparts, type.c_str()));
  }
  bool Next() {
    py::gil_scoped_release nogil;
    return it_->Next();
  }
  py::dict Value() { return BlockToDict(it_->Value()); }
  void BeforeFirst() { it_->BeforeFirst(); }
  size_t NumCol() const { return it_->NumCol(); }

 private:
  std::unique_ptr<RowBlockIter<I>> it_;
};

/*! \brief the GPU ring's host stage as a Python iterator with a resume cursor */
class PyPartitionReader {
 public:
  PyPartitionReader(const std::string& uri, unsigned part, unsigned nparts,
                    const std::string& type, int nthread, size_t chunk_bytes)
      : buf_(chunk_bytes, '\0') {
    CHECK(type == "text" || type == "recordio")
        << "PartitionReader: type must be text or recordio, got " << type;
    py::gil_scoped_release nogil;  // listing may hit an in-process (Python) server
    io::URI path(uri.c_str());
    io::FileSystem* fs = io::FileSystem::GetInstance(path);
    if (type == "text") {
      split_.reset(new io::LineSplitter(fs, uri.c_str(), part, nparts));
    } else {
      split_.reset(new io::RecordIOSplitter(fs, uri.c_str(), part, nparts));
    }
    reader_.reset(new io::ShardReader(split_.get(), nthread));
  }
  ~PyPartitionReader() {
    py::gil_scoped_release nogil;
    reader_.reset();
    split_.reset();
  }
  py::object Next() {
    size_t n;
    {
      py::gil_scoped_release nogil;
      n = reader_->Fill(&buf_[0], buf_.size());
      while (n == io::ShardReader::kNeedMore) {  // a record longer than the buffer
        buf_.resize(reader_->NeedCapacity());
        n = reader_->Fill(&buf_[0], buf_.size());
      }
    }
    if (n == 0) return py::none();
    return py::bytes(buf_.data(), n);
  }
  size_t Tell() const { return reader_->Tell(); }
  void Seek(size_t pos) { reader_->Seek(pos); }
  size_t PartitionBytes() const { return reader_->PartitionBytes(); }

 private:
  std::string buf_;
  std::unique_ptr<io::InputSplitBase> split_;
  std::unique_ptr<io::ShardReader> reader_;
};

class PyInputSplit {
 public:
  PyInputSplit(const std::string& uri, unsigned part, unsigned nparts, const std::string& type,
               const std::string& index_uri, bool shuffle, int seed, size_t batch_size,
               unsigned num_shuffle_parts) {
    py::gil_scoped_release nogil;
    if (num_shuffle_parts > 0) {
      // coarse chunk shuffling (include/dmlc/input_split_shuffle.h)
      CHECK(index_uri.empty()) << "num_shuffle_parts does not combine with an index file";
      s_.reset(InputSplitShuffle::Create(uri.c_str(), part, nparts, type.c_str(),
                                         num_shuffle_parts, seed));
      return;
    }
    s_.reset(index_uri.empty()
                 ? InputSplit::Create(uri.c_str(), part, nparts, type.c_str())
                 : InputSplit::Create(uri.c_str(), index_uri.c_str(), part, nparts, type.c_str(),
                                      shuffle, seed, batch_size));
  }
  ~PyInputSplit() {
    py::gil_scoped_release nogil;
    s_.reset();
  }
  py::object NextRecord() {
    InputSplit::Blob b;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = s_->NextRecord(&b);
    }
    if (!ok) return py::none();
    return py::bytes(static_cast<const char*>(b.dptr), b.size);
  }
  py::object NextChunk() {
    InputSplit::Blob b;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = s_->NextChunk(&b);
    }
    if (!ok) return py::none();
    return py::bytes(static_cast<const char*>(b.dptr), b.size);
  }
  py::object NextBatch(size_t n) {
    InputSplit::Blob b;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = s_->NextBatch(&b, n);
    }
    if (!ok) return py::none();
    return py::bytes(static_cast<const char*>(b.dptr), b.size);
  }
  void BeforeFirst() {
    py::gil_scoped_release nogil;
    s_->BeforeFirst();
  }
  void ResetPartition(unsigned part, unsigned nparts) { s_->ResetPartition(part, nparts); }
  size_t TotalSize() { return s_->GetTotalSize(); }
  void HintChunkSize(size_t n) { s_->HintChunkSize(n); }

 private:
  std::unique_ptr<InputSplit> s_;
};

class PyStream {
 public:
  // every call may block on I/O (remote filesystems): release the GIL
  PyStream(const std::string& uri, const std::string& mode) {
    py::gil_scoped_release nogil;
    s_.reset(Stream::Create(uri.c_str(), mode.c_str()));
  }
  ~PyStream() {
    py::gil_scoped_release nogil;
    s_.reset();
  }
  py::bytes Read(size_t n) {
    std::string buf(n, '\0');
    {
      py::gil_scoped_release nogil;
      size_t got = s_->Read(&buf[0], n);
      buf.resize(got);
    }
    return py::bytes(buf);
  }
  void Write(const std::string& data) {
    py::gil_scoped_release nogil;
    s_->Write(data.data(), data.size());
  }
  void Close() {
    py::gil_scoped_release nogil;
    s_.reset();
  }

 private:
  std::unique_ptr<Stream> s_;
};

class PyRecordIOWriter {
 public:
  explicit PyRecordIOWriter(const std::string& uri)
      : s_(Stream::Create(uri.c_str(), "w")), w_(new RecordIOWriter(s_.get())) {}
  void Write(const std::string& rec) { w_->WriteRecord(rec.data(), rec.size()); }
  size_t Tell() const { return w_->Tell(); }
  size_t ExceptCounter() const { return w_->except_counter(); }
  void Close() {
    w_.reset();
    s_.reset();
  }

 private:
  std::unique_ptr<Stream> s_;
  std::unique_ptr<RecordIOWriter> w_;
};

class PyRecordIOReader {
 public:
  explicit PyRecordIOReader(const std::string& uri)
      : s_(Stream::Create(uri.c_str(), "r")), r_(new RecordIOReader(s_.get())) {}
  py::object Next() {
    std::string rec;
    if (!r_->NextRecord(&rec)) return py::none();
    return py::bytes(rec);
  }

 private:
  std::unique_ptr<Stream> s_;
  std::unique_ptr<RecordIOReader> r_;
};

// ----------------------------------------------------------------- device
template <typename I>
class PyDeviceCSR {
 public:
  PyDeviceCSR() : csr_(std::make_shared<gpu::DeviceCSR<I>>()) {}
  std::shared_ptr<gpu::DeviceCSR<I>> csr_;
  size_t rows() const { return csr_->rows_; }
  size_t nnz() const { return csr_->nnz_; }
  uint64_t max_index() const { return csr_->max_index_; }
  uint64_t max_field() const { return csr_->max_field_; }
  size_t allocated_bytes() const { return csr_->AllocatedBytes(); }
  py::dict Capsules() {
    auto v = csr_->View();
    std::shared_ptr<void> owner = csr_;
    py::dict d;
    d["offset"] = ToCapsule(v.offset, static_cast<int64_t>(v.size + 1), v.device, owner);
    d["label"] = ToCapsule(v.label, static_cast<int64_t>(v.size), v.device, owner);
    d["index"] = ToCapsule(v.index, static_cast<int64_t>(v.nnz), v.device, owner);
    d["value"] = v.value ? ToCapsule(v.value, static_cast<int64_t>(v.nnz), v.device, owner)
                         : py::none();
    d["weight"] = v.weight ? ToCapsule(v.weight, static_cast<int64_t>(v.size), v.device, owner)
                           : py::none();
    d["qid"] = v.qid ? ToCapsule(v.qid, static_cast<int64_t>(v.size), v.device, owner)
                     : py::none();
    d["field"] = v.field ? ToCapsule(v.field, static_cast<int64_t>(v.nnz), v.device, owner)
                         : py::none();
    return d;
  }
  py::dict ToHost() {
    auto h = gpu::CopyToHost(csr_->View());
    return BlockToDict(h.GetBlock());
  }
  void Clear() { csr_->Clear(); }
};

template <typename I>
class PyDeviceParser {
 public:
  PyDeviceParser(const std::string& uri, unsigned part, unsigned nparts, py::dict cfg_dict) {
    gpu::DeviceParserConfig cfg;
    std::map<std::string, std::string> args;
    for (auto kv : cfg_dict) args[py::str(kv.first)] = py::str(kv.second);
    cfg.Update(args);
    py::gil_scoped_release nogil;  // opening a remote split lists / HEADs over HTTP
    p_.reset(gpu::DeviceParser<I>::Create(uri, part, nparts, cfg));
  }
  void ParseAll(PyDeviceCSR<I>& out) {  // NOLINT
    py::gil_scoped_release nogil;
    p_->ParseAll(out.csr_.get());
  }
  /*! \brief fused tokenize -> hash -> fp8/f32 dense batch; DLPack capsules.
   *  out: the "batch" handle of an earlier result whose tensors the caller is
   *  done with -- its HBM buffers are refilled instead of allocated again. */
  py::dict ParseAllHashed(int dim, float scale, uint32_t seed, bool fp8, py::object out) {
    std::shared_ptr<gpu::DeviceHashedBatch> batch;
    if (!out.is_none()) batch = out.cast<std::shared_ptr<gpu::DeviceHashedBatch>>();
    if (batch == nullptr) batch = std::make_shared<gpu::DeviceHashedBatch>();
    {
      py::gil_scoped_release nogil;
      p_->ParseAllHashed(batch.get(), dim, scale, seed, fp8);
    }
    py::dict d;
    const int64_t n = static_cast<int64_t>(batch->rows) * dim;
    // each capsule owns the buffer it exports (not the batch): a later refill
    // that reallocates leaves these tensors their own, still valid, memory
    if (fp8) {
      d["x"] = ToCapsule(batch->x->get<uint8_t>(), n, batch->device, batch->x);
    } else {
      d["x"] = ToCapsule(batch->x->get<float>(), n, batch->device, batch->x);
    }
    d["label"] = ToCapsule(batch->label->get<float>(), static_cast<int64_t>(batch->rows),
                           batch->device, batch->label);
    d["rows"] = batch->rows;
    d["dim"] = dim;
    d["x_ptr"] = reinterpret_cast<uintptr_t>(batch->x->get());
    d["label_ptr"] = reinterpret_cast<uintptr_t>(batch->label->get());
    d["batch"] = py::cast(batch);
    return d;
  }
  bool Next() {
    py::gil_scoped_release nogil;
    return p_->Next();
  }
  py::dict ValueToHost() {
    auto h = gpu::CopyToHost(p_->Value());
    return BlockToDict(h.GetBlock());
  }
  py::tuple ValueShape() const {
    const auto& v = p_->Value();
    return py::make_tuple(v.size, v.nnz, v.max_index);
  }
  void BeforeFirst() {
    py::gil_scoped_release nogil;
    p_->BeforeFirst();
  }
  size_t Tell() const { return p_->Tell(); }
  void Seek(size_t cursor) {
    py::gil_scoped_release nogil;
    p_->Seek(cursor);
  }
  unsigned Epoch() const { return p_->Epoch(); }
  void SetEpoch(unsigned e) {
    py::gil_scoped_release nogil;
    p_->SetEpoch(e);
  }
  std::vector<unsigned> VisitOrder() const { return p_->VisitOrder(); }
  size_t PartitionBytes() const { return p_->PartitionBytes(); }
  py::dict Stats() const {
    const auto& s = p_->Stats();
    py::dict d;
    d["bytes"] = s.bytes;
    d["chunks"] = s.chunks;
    d["rows"] = s.rows;
    d["nnz"] = s.nnz;
    d["exact_chunks"] = s.exact_chunks;
    d["one_pass_chunks"] = s.one_pass_chunks;
    d["one_pass_reruns"] = s.one_pass_reruns;
    d["wait_reader_sec"] = s.wait_reader_sec;
    d["wait_gpu_sec"] = s.wait_gpu_sec;
    d["zero_copy"] = s.zero_copy;
    d["register_sec"] = s.register_sec;
    d["zc_pin_budget"] = s.zc_pin_budget;
    d["zc_pinned_peak"] = s.zc_pinned_peak;
    d["last_pass_sec"] = s.last_pass_sec;
    d["last_fill_sec"] = s.last_fill_sec;
    d["last_drain_sec"] = s.last_drain_sec;
    d["waits_spun"] = s.waits_spun;
    d["waits_slept"] = s.waits_slept;
    d["waits_timed_out"] = s.waits_timed_out;
    return d;
  }
  uintptr_t Stream() const { return reinterpret_cast<uintptr_t>(p_->stream()); }
  /*! \brief DLPack capsules of the last Next() block (valid until the next call) */
  py::dict ValueCapsules() {
    const auto& v = p_->Value();
    std::shared_ptr<void> owner = p_;
    py::dict d;
    d["offset"] = ToCapsule(v.offset, static_cast<int64_t>(v.size + 1), v.device, owner);
    d["label"] = ToCapsule(v.label, static_cast<int64_t>(v.size), v.device, owner);
    d["index"] = ToCapsule(v.index, static_cast<int64_t>(v.nnz), v.device, owner);
    d["value"] = v.value ? ToCapsule(v.value, static_cast<int64_t>(v.nnz), v.device, owner)
                         : py::none();
    d["weight"] = v.weight ? ToCapsule(v.weight, static_cast<int64_t>(v.size), v.device, owner)
                           : py::none();
    d["qid"] = v.qid ? ToCapsule(v.qid, static_cast<int64_t>(v.size), v.device, owner) : py::none();
    d["field"] = v.field ? ToCapsule(v.field, static_cast<int64_t>(v.nnz), v.device, owner)
                         : py::none();
    return d;
  }

 private:
  std::shared_ptr<gpu::DeviceParser<I>> p_;
};

/*! \brief the `#cache` page file on the GPU route (gpu/device_page_cache.h) */
template <typename I>
class PyPageCache {
 public:
  explicit PyPageCache(std::unique_ptr<gpu::DevicePageCache<I>> c) : c_(std::move(c)) {}
  static py::object Open(const std::string& path, int device) {
    std::unique_ptr<gpu::DevicePageCache<I>> c;
    {
      py::gil_scoped_release nogil;
      c = gpu::DevicePageCache<I>::Open(path, device);
    }
    if (c == nullptr) return py::none();
    return py::cast(new PyPageCache<I>(std::move(c)), py::return_value_policy::take_ownership);
  }
  static size_t Write(PyDeviceCSR<I>& csr, const std::string& path, double page_mb) {  // NOLINT
    py::gil_scoped_release nogil;
    return gpu::DevicePageCache<I>::Write(*csr.csr_, path, static_cast<size_t>(page_mb * (1 << 20)));
  }
  void Load(PyDeviceCSR<I>& out) {  // NOLINT
    py::gil_scoped_release nogil;
    c_->Load(out.csr_.get());
  }
  py::list Pages() const {
    py::list l;
    for (const auto& p : c_->pages()) {
      py::dict d;
      d["rows"] = p.rows;
      d["nnz"] = p.nnz;
      d["begin"] = p.begin;
      d["end"] = p.end;
      d["max_index"] = p.max_index;
      l.append(d);
    }
    return l;
  }
  std::unique_ptr<gpu::DevicePageCache<I>> c_;
};

template <typename I>
void BindIndexType(py::module_& m, const std::string& suffix) {
  py::class_<PyParser<I>>(m, ("Parser" + suffix).c_str())
      .def(py::init<const std::string&, unsigned, unsigned, const std::string&>(),
           py::arg("uri"), py::arg("part") = 0, py::arg("nparts") = 1, py::arg("type") = "auto")
      .def("next", &PyParser<I>::Next)
      .def("value", &PyParser<I>::Value)
      .def("before_first", &PyParser<I>::BeforeFirst)
      .def("bytes_read", &PyParser<I>::BytesRead)
      .def("drain", &PyParser<I>::Drain);
  py::class_<PyRowBlockIter<I>>(m, ("RowBlockIter" + suffix).c_str())
      .def(py::init<const std::string&, unsigned, unsigned, const std::string&>(),
           py::arg("uri"), py::arg("part") = 0, py::arg("nparts") = 1, py::arg("type") = "auto")
      .def("next", &PyRowBlockIter<I>::Next)
      .def("value", &PyRowBlockIter<I>::Value)
      .def("before_first", &PyRowBlockIter<I>::BeforeFirst)
      .def("num_col", &PyRowBlockIter<I>::NumCol);
  py::class_<PyDeviceCSR<I>>(m, ("DeviceCSR" + suffix).c_str())
      .def(py::init<>())
      .def_property_readonly("rows", &PyDeviceCSR<I>::rows)
      .def_property_readonly("nnz", &PyDeviceCSR<I>::nnz)
      .def_property_readonly("max_index", &PyDeviceCSR<I>::max_index)
      .def_property_readonly("max_field", &PyDeviceCSR<I>::max_field)
      .def_property_readonly("allocated_bytes", &PyDeviceCSR<I>::allocated_bytes)
      .def("capsules", &PyDeviceCSR<I>::Capsules)
      .def("to_host", &PyDeviceCSR<I>::ToHost)
      .def("clear", &PyDeviceCSR<I>::Clear);
  py::class_<PyPageCache<I>>(m, ("PageCache" + suffix).c_str())
      .def_static("open", &PyPageCache<I>::Open, py::arg("path"), py::arg("device") = -1)
      .def_static("write", &PyPageCache<I>::Write, py::arg("csr"), py::arg("path"),
                  py::arg("page_mb") = 64.0)
      .def("load", &PyPageCache<I>::Load)
      .def("pages", &PyPageCache<I>::Pages)
      .def_property_readonly("rows", [](const PyPageCache<I>& c) { return c.c_->rows(); })
      .def_property_readonly("nnz", [](const PyPageCache<I>& c) { return c.c_->nnz(); })
      .def_property_readonly("bytes", [](const PyPageCache<I>& c) { return c.c_->bytes(); })
      .def_property_readonly("zero_copy", [](const PyPageCache<I>& c) { return c.c_->zero_copy(); });
  py::class_<PyDeviceParser<I>>(m, ("DeviceParser" + suffix).c_str())
      .def(py::init<const std::string&, unsigned, unsigned, py::dict>(), py::arg("uri"),
           py::arg("part") = 0, py::arg("nparts") = 1, py::arg("config") = py::dict())
      .def("parse_all", &PyDeviceParser<I>::ParseAll)
      .def("parse_all_hashed", &PyDeviceParser<I>::ParseAllHashed, py::arg("dim"),
           py::arg("scale") = 1.0f, py::arg("seed") = 0u, py::arg("fp8") = true,
           py::arg("out") = py::none())
      .def("next", &PyDeviceParser<I>::Next)
      .def("value_to_host", &PyDeviceParser<I>::ValueToHost)
      .def("value_shape", &PyDeviceParser<I>::ValueShape)
      .def("value_capsules", &PyDeviceParser<I>::ValueCapsules)
      .def("before_first", &PyDeviceParser<I>::BeforeFirst)
      .def("tell", &PyDeviceParser<I>::Tell)
      .def("seek", &PyDeviceParser<I>::Seek)
      .def("epoch", &PyDeviceParser<I>::Epoch)
      .def("set_epoch", &PyDeviceParser<I>::SetEpoch)
      .def("visit_order", &PyDeviceParser<I>::VisitOrder)
      .def("partition_bytes", &PyDeviceParser<I>::PartitionBytes)
      .def("stats", &PyDeviceParser<I>::Stats)
      .def("stream", &PyDeviceParser<I>::Stream);
}

// --------------------------------------------------------------- device recordio
class PyDeviceRecordIO {
 public:
  PyDeviceRecordIO(const std::string& uri, unsigned part, unsigned nparts, py::dict kwargs) {
    gpu::DeviceRecordIOConfig cfg;
    std::map<std::string, std::string> args;
    for (auto kv : kwargs) args[py::str(kv.first)] = py::str(kv.second);
    cfg.Update(args);
    {
      py::gil_scoped_release nogil;
      reader_.reset(gpu::DeviceRecordIOReader::Create(uri, part, nparts, cfg));
    }
    DMLC_HIP_CHECK(hipGetDevice(&device_));
  }
  bool Next() {
    py::gil_scoped_release nogil;
    return reader_->Next();
  }
  py::dict ValueCapsules() { return Batch(reader_->Value()); }
  /*! \brief (offsets numpy, payload bytes) of the last Next() */
  py::tuple ValueToHost() { return ToHost(reader_->Value()); }
  py::tuple ResidentToHost() { return ToHost(Resident()); }
  void BeforeFirst() { reader_->BeforeFirst(); }
  size_t PartitionBytes() const { return reader_->PartitionBytes(); }
  py::dict Stats() const {
    const auto& s = reader_->Stats();
    py::dict d;
    d["bytes"] = s.bytes;
    d["chunks"] = s.chunks;
    d["records"] = s.records;
    d["zero_copy"] = s.zero_copy;
    d["wait_reader_sec"] = s.wait_reader_sec;
    d["wait_gpu_sec"] = s.wait_gpu_sec;
    d["replayed_chunks"] = s.replayed_chunks;
    d["one_pass_chunks"] = s.one_pass_chunks;
    d["one_pass_reruns"] = s.one_pass_reruns;
    d["chain_counts"] = s.chain_counts;
    return d;
  }
  uintptr_t Stream() const { return reinterpret_cast<uintptr_t>(reader_->stream()); }

 private:
  const gpu::DeviceRecordBatch& Resident() { return resident_view_; }
  py::dict Batch(const gpu::DeviceRecordBatch& b) {
    py::dict d;
    d["size"] = b.size;
    d["bytes"] = b.bytes;
    d["offset"] = ToCapsule(b.offset, static_cast<int64_t>(b.size + 1), device_, reader_);
    d["data"] = ToCapsule(b.data, static_cast<int64_t>(b.bytes), device_, reader_);
    return d;
  }
  py::tuple ToHost(const gpu::DeviceRecordBatch& b) {
    std::vector<uint64_t> off(b.size + 1, 0);
    std::string data(b.bytes, '\0');
    DMLC_HIP_CHECK(hipStreamSynchronize(reader_->stream()));
    if (b.size > 0) {
      DMLC_HIP_CHECK(hipMemcpy(off.data(), b.offset, off.size() * 8, hipMemcpyDeviceToHost));
    }
    if (b.bytes > 0) DMLC_HIP_CHECK(hipMemcpy(&data[0], b.data, b.bytes, hipMemcpyDeviceToHost));
    return py::make_tuple(ToNumpy(off.data(), off.size()), py::bytes(data));
  }
  std::shared_ptr<gpu::DeviceRecordIOReader> reader_;
  gpu::DeviceRecordBatch resident_view_;
  int device_{0};

  friend void BindRecordIO(py::module_& m);
};

void BindRecordIO(py::module_& m) {
  py::class_<PyDeviceRecordIO>(m, "DeviceRecordIO")
      .def(py::init<const std::string&, unsigned, unsigned, py::dict>(), py::arg("uri"),
           py::arg("part") = 0, py::arg("nparts") = 1, py::arg("config") = py::dict())
      .def("next", &PyDeviceRecordIO::Next)
      .def("read_all",
           [](PyDeviceRecordIO& self) {
             {
               py::gil_scoped_release nogil;
               self.resident_view_ = self.reader_->ReadAll();
             }
             return self.Batch(self.resident_view_);
           })
      .def("value", &PyDeviceRecordIO::ValueCapsules)
      .def("value_to_host", &PyDeviceRecordIO::ValueToHost)
      .def("resident_to_host", &PyDeviceRecordIO::ResidentToHost)
      .def("before_first", &PyDeviceRecordIO::BeforeFirst)
      .def("partition_bytes", &PyDeviceRecordIO::PartitionBytes)
      .def("stats", &PyDeviceRecordIO::Stats)
      .def("stream", &PyDeviceRecordIO::Stream);
}

}  // namespace

PYBIND11_MODULE(_dmlc, m) {
  m.doc() = "dmlc-core for MI355X: native runtime bindings";
  py::register_exception<dmlc::Error>(m, "DMLCError");
  py::class_<gpu::DeviceHashedBatch, std::shared_ptr<gpu::DeviceHashedBatch>>(m, "HashedBatch")
      .def_readonly("rows", &gpu::DeviceHashedBatch::rows)
      .def_readonly("row_capacity", &gpu::DeviceHashedBatch::row_cap)
      .def_readonly("dim", &gpu::DeviceHashedBatch::dim);
  BindIndexType<uint32_t>(m, "");
  BindIndexType<uint64_t>(m, "64");
  BindRecordIO(m);
  py::class_<PyPartitionReader>(m, "PartitionReader")
      .def(py::init<const std::string&, unsigned, unsigned, const std::string&, int, size_t>(),
           py::arg("uri"), py::arg("part") = 0, py::arg("nparts") = 1, py::arg("type") = "text",
           py::arg("nthread") = 8, py::arg("chunk_bytes") = 64UL << 20)
      .def("next", &PyPartitionReader::Next)
      .def("tell", &PyPartitionReader::Tell)
      .def("seek", &PyPartitionReader::Seek)
      .def("partition_bytes", &PyPartitionReader::PartitionBytes);
  py::class_<PyInputSplit>(m, "InputSplit")
      .def(py::init<const std::string&, unsigned, unsigned, const std::string&,
                    const std::string&, bool, int, size_t, unsigned>(),
           py::arg("uri"), py::arg("part") = 0, py::arg("nparts") = 1, py::arg("type") = "text",
           py::arg("index_uri") = "", py::arg("shuffle") = false, py::arg("seed") = 0,
           py::arg("batch_size") = 256, py::arg("num_shuffle_parts") = 0)
      .def("next_record", &PyInputSplit::NextRecord)
      .def("next_chunk", &PyInputSplit::NextChunk)
      .def("next_batch", &PyInputSplit::NextBatch)
      .def("before_first", &PyInputSplit::BeforeFirst)
      .def("reset_partition", &PyInputSplit::ResetPartition)
      .def("total_size", &PyInputSplit::TotalSize)
      .def("hint_chunk_size", &PyInputSplit::HintChunkSize);
  py::class_<PyStream>(m, "Stream")
      .def(py::init<const std::string&, const std::string&>(), py::arg("uri"),
           py::arg("mode") = "r")
      .def("read", &PyStream::Read)
      .def("write", &PyStream::Write)
      .def("close", &PyStream::Close);
  py::class_<PyRecordIOWriter>(m, "RecordIOWriter")
      .def(py::init<const std::string&>())
      .def("write", &PyRecordIOWriter::Write)
      .def("tell", &PyRecordIOWriter::Tell)
      .def("except_counter", &PyRecordIOWriter::ExceptCounter)
      .def("close", &PyRecordIOWriter::Close);
  py::class_<PyRecordIOReader>(m, "RecordIOReader")
      .def(py::init<const std::string&>())
      .def("next", &PyRecordIOReader::Next);
  m.def(
      "write_synthetic",
      [](const std::string& path, uint64_t row_begin, uint64_t row_end, const std::string& format,
         uint64_t seed, uint32_t min_nnz, uint32_t max_nnz, uint64_t num_features,
         uint32_t num_fields, uint32_t csv_columns, uint32_t record_bytes, uint32_t weight_every,
         bool qid, int nthread, const std::string& shape) {
        synthetic::Spec s;
        s.format = format;
        s.seed = seed;
        s.min_nnz = min_nnz;
        s.max_nnz = max_nnz;
        s.num_features = num_features;
        s.num_fields = num_fields;
        s.csv_columns = csv_columns;
        s.record_bytes = record_bytes;
        s.weight_every = weight_every;
        s.qid = qid;
        s.shape = shape;
        py::gil_scoped_release nogil;
        return synthetic::WriteRows(s, path, row_begin, row_end, nthread);
      },
      py::arg("path"), py::arg("row_begin"), py::arg("row_end"), py::arg("format") = "libsvm",
      py::arg("seed") = 0, py::arg("min_nnz") = 20, py::arg("max_nnz") = 60,
      py::arg("num_features") = 1000000, py::arg("num_fields") = 32, py::arg("csv_columns") = 29,
      py::arg("record_bytes") = 512, py::arg("weight_every") = 0, py::arg("qid") = false,
      py::arg("nthread") = 8, py::arg("shape") = "uniform");
  // ---- HIP feature kernels on raw device pointers (torch tensors' data_ptr) ----
  auto stream_of = [](uintptr_t s) { return reinterpret_cast<hipStream_t>(s); };
  m.def(
      "fm_forward",
      [stream_of](uintptr_t x, int64_t rows, int dim, uintptr_t wt, uintptr_t q, uintptr_t bias,
                  float sx, uintptr_t y, uintptr_t xv, int num_cus, uintptr_t stream) {
        CHECK(dim > 0 && dim % 128 == 0 && dim <= 2048)
            << "HashedFM kernels need dim a multiple of 128, <= 2048 (got " << dim << ")";
        gpu::LaunchFmForward(reinterpret_cast<const uint8_t*>(x), rows, dim,
                             reinterpret_cast<const void*>(wt), reinterpret_cast<const float*>(q),
                             reinterpret_cast<const float*>(bias), sx, reinterpret_cast<float*>(y),
                             reinterpret_cast<float*>(xv), num_cus, stream_of(stream));
      },
      py::arg("x"), py::arg("rows"), py::arg("dim"), py::arg("wt"), py::arg("q"), py::arg("bias"),
      py::arg("sx"), py::arg("y"), py::arg("xv"), py::arg("num_cus"), py::arg("stream"));
  m.def(
      "fm_backward",
      [stream_of](uintptr_t x, int64_t rows, int dim, uintptr_t g, uintptr_t xv, int nblocks,
                  uintptr_t part, uintptr_t stream) {
        CHECK(dim > 0 && dim % 128 == 0) << "HashedFM kernels need dim a multiple of 128";
        gpu::LaunchFmBackward(reinterpret_cast<const uint8_t*>(x), rows, dim,
                              reinterpret_cast<const float*>(g), reinterpret_cast<const float*>(xv),
                              nblocks, reinterpret_cast<float*>(part), stream_of(stream));
      },
      py::arg("x"), py::arg("rows"), py::arg("dim"), py::arg("g"), py::arg("xv"),
      py::arg("nblocks"), py::arg("part"), py::arg("stream"));
  m.def(
      "fm_prep",
      [stream_of](uintptr_t w, uintptr_t v, int dim, uintptr_t wt, uintptr_t q, uintptr_t stream) {
        gpu::LaunchFmPrep(reinterpret_cast<const float*>(w), reinterpret_cast<const float*>(v),
                          dim, reinterpret_cast<void*>(wt), reinterpret_cast<float*>(q),
                          stream_of(stream));
      },
      py::arg("w"), py::arg("v"), py::arg("dim"), py::arg("wt"), py::arg("q"), py::arg("stream"));
  m.def(
      "fm_reduce_grads",
      [stream_of](uintptr_t part, int nblocks, int dim, uintptr_t v, float sx, uintptr_t z,
                  uintptr_t gw, uintptr_t gv, uintptr_t stream) {
        gpu::LaunchFmReduceGrads(reinterpret_cast<const float*>(part), nblocks, dim,
                                 reinterpret_cast<const float*>(v), sx, reinterpret_cast<float*>(z),
                                 reinterpret_cast<float*>(gw), reinterpret_cast<float*>(gv),
                                 stream_of(stream));
      },
      py::arg("part"), py::arg("nblocks"), py::arg("dim"), py::arg("v"), py::arg("sx"),
      py::arg("z"), py::arg("gw"), py::arg("gv"), py::arg("stream"));
  m.def(
      "fm_fused",
      [stream_of](uintptr_t x, int64_t rows, int dim, uintptr_t wt, uintptr_t q, uintptr_t bias,
                  float sx, uintptr_t label, uintptr_t weight, int loss, float inv_n, int nblocks,
                  uintptr_t y, uintptr_t part, uintptr_t lpart, uintptr_t stream) {
        CHECK(dim == 128 || dim == 256 || dim == 512 || dim == 1024)
            << "fused HashedFM step: dim must be 128, 256, 512 or 1024 (got " << dim << ")";
        CHECK(loss == gpu::kFmLogistic || loss == gpu::kFmSquared) << "unknown loss " << loss;
        gpu::LaunchFmFused(reinterpret_cast<const uint8_t*>(x), rows, dim,
                           reinterpret_cast<const void*>(wt), reinterpret_cast<const float*>(q),
                           reinterpret_cast<const float*>(bias), sx,
                           reinterpret_cast<const float*>(label),
                           reinterpret_cast<const float*>(weight), loss, inv_n, nblocks,
                           reinterpret_cast<float*>(y), reinterpret_cast<float*>(part),
                           reinterpret_cast<float*>(lpart), stream_of(stream));
      },
      py::arg("x"), py::arg("rows"), py::arg("dim"), py::arg("wt"), py::arg("q"), py::arg("bias"),
      py::arg("sx"), py::arg("label"), py::arg("weight"), py::arg("loss"), py::arg("inv_n"),
      py::arg("nblocks"), py::arg("y"), py::arg("part"), py::arg("lpart"), py::arg("stream"));
  m.attr("fm_rank") = gpu::kFmRank;
  m.def("shuffle_parts_order", &InputSplitShuffle::VisitOrder, py::arg("part"), py::arg("nparts"),
        py::arg("num_shuffle_parts"), py::arg("seed"), py::arg("epoch"),
        "sub-shard visiting order of InputSplitShuffle in a given epoch");
  m.def(
      "spmv",
      [stream_of](uintptr_t offset, uintptr_t index, uintptr_t value, size_t nrows, uintptr_t w,
                  float bias, uintptr_t y, uintptr_t stream, bool index64) {
        auto* off = reinterpret_cast<const uint64_t*>(offset);
        auto* val = reinterpret_cast<const float*>(value);
        if (index64) {
          gpu::LaunchCSRSpMV<uint64_t>(off, reinterpret_cast<const uint64_t*>(index), val, nrows,
                                       reinterpret_cast<const float*>(w), bias,
                                       reinterpret_cast<float*>(y), stream_of(stream));
        } else {
          gpu::LaunchCSRSpMV<uint32_t>(off, reinterpret_cast<const uint32_t*>(index), val, nrows,
                                       reinterpret_cast<const float*>(w), bias,
                                       reinterpret_cast<float*>(y), stream_of(stream));
        }
      },
      py::arg("offset"), py::arg("index"), py::arg("value"), py::arg("nrows"), py::arg("w"),
      py::arg("bias"), py::arg("y"), py::arg("stream"), py::arg("index64") = false);
  m.def(
      "spmv_t",
      [stream_of](uintptr_t offset, uintptr_t index, uintptr_t value, size_t nrows, uintptr_t d,
                  uintptr_t g, uintptr_t stream, bool index64) {
        auto* off = reinterpret_cast<const uint64_t*>(offset);
        auto* val = reinterpret_cast<const float*>(value);
        if (index64) {
          gpu::LaunchCSRSpMVT<uint64_t>(off, reinterpret_cast<const uint64_t*>(index), val, nrows,
                                        reinterpret_cast<const float*>(d),
                                        reinterpret_cast<float*>(g), stream_of(stream));
        } else {
          gpu::LaunchCSRSpMVT<uint32_t>(off, reinterpret_cast<const uint32_t*>(index), val, nrows,
                                        reinterpret_cast<const float*>(d),
                                        reinterpret_cast<float*>(g), stream_of(stream));
        }
      },
      py::arg("offset"), py::arg("index"), py::arg("value"), py::arg("nrows"), py::arg("d"),
      py::arg("g"), py::arg("stream"), py::arg("index64") = false);
  m.def(
      "csr_transpose",
      [stream_of](uintptr_t offset, size_t nrows, uint64_t base, uint64_t nnz, uintptr_t index,
                  uintptr_t value, uint64_t num_features, uintptr_t col_ptr, uintptr_t row_out,
                  uintptr_t val_out, uintptr_t scratch, uintptr_t error, uintptr_t stream,
                  bool index64) {
        auto* off = reinterpret_cast<const uint64_t*>(offset);
        auto* val = reinterpret_cast<const float*>(value);
        auto* cp = reinterpret_cast<uint64_t*>(col_ptr);
        auto* ro = reinterpret_cast<uint32_t*>(row_out);
        auto* vo = reinterpret_cast<float*>(val_out);
        auto* err = reinterpret_cast<uint32_t*>(error);
        void* sc = reinterpret_cast<void*>(scratch);
        if (index64) {
          gpu::LaunchCSRTranspose<uint64_t>(off, nrows, base, nnz,
                                            reinterpret_cast<const uint64_t*>(index), val,
                                            num_features, cp, ro, vo, sc, err, stream_of(stream));
        } else {
          gpu::LaunchCSRTranspose<uint32_t>(off, nrows, base, nnz,
                                            reinterpret_cast<const uint32_t*>(index), val,
                                            num_features, cp, ro, vo, sc, err, stream_of(stream));
        }
      },
      py::arg("offset"), py::arg("nrows"), py::arg("base"), py::arg("nnz"), py::arg("index"),
      py::arg("value"), py::arg("num_features"), py::arg("col_ptr"), py::arg("row_out"),
      py::arg("val_out"), py::arg("scratch"), py::arg("error"), py::arg("stream"),
      py::arg("index64") = false);
  m.def("csr_transpose_scratch_bytes", &gpu::CSRTransposeScratchBytes, py::arg("nnz"),
        py::arg("num_features"));
  m.def("csr_transpose_max_features", &gpu::CSRTransposeMaxFeatures);
  m.def(
      "hashed_dense",
      [stream_of](uintptr_t offset, uintptr_t index, uintptr_t value, uintptr_t field,
                  size_t nrows, int dim, float scale, uint32_t seed, uintptr_t out, bool fp8,
                  uintptr_t stream, bool index64) {
        CHECK(dim > 0 && dim <= 8192 && dim % 4 == 0) << "dim must be a multiple of 4 in (0, 8192]";
        auto* off = reinterpret_cast<const uint64_t*>(offset);
        auto* val = reinterpret_cast<const float*>(value);
        if (index64) {
          auto* idx = reinterpret_cast<const uint64_t*>(index);
          auto* fld = reinterpret_cast<const uint64_t*>(field);
          if (fp8) {
            gpu::LaunchHashedDenseFP8<uint64_t>(off, idx, val, fld, nrows, dim, scale, seed,
                                                reinterpret_cast<uint8_t*>(out), stream_of(stream));
          } else {
            gpu::LaunchHashedDenseF32<uint64_t>(off, idx, val, fld, nrows, dim, seed,
                                                reinterpret_cast<float*>(out), stream_of(stream));
          }
        } else {
          auto* idx = reinterpret_cast<const uint32_t*>(index);
          auto* fld = reinterpret_cast<const uint32_t*>(field);
          if (fp8) {
            gpu::LaunchHashedDenseFP8<uint32_t>(off, idx, val, fld, nrows, dim, scale, seed,
                                                reinterpret_cast<uint8_t*>(out), stream_of(stream));
          } else {
            gpu::LaunchHashedDenseF32<uint32_t>(off, idx, val, fld, nrows, dim, seed,
                                                reinterpret_cast<float*>(out), stream_of(stream));
          }
        }
      },
      py::arg("offset"), py::arg("index"), py::arg("value"), py::arg("field"), py::arg("nrows"),
      py::arg("dim"), py::arg("scale"), py::arg("seed"), py::arg("out"), py::arg("fp8"),
      py::arg("stream"), py::arg("index64") = false);
  m.def(
      "read_partition",
      [](const std::string& uri, unsigned part, unsigned nparts, const std::string& type,
         int nthread, size_t chunk_bytes) {
        // the host stage of the GPU ring (parallel pread / parallel ranged
        // GETs) as a plain API: whole-record chunks of one partition
        CHECK(type == "text" || type == "recordio")
            << "read_partition: type must be text or recordio, got " << type;
        std::vector<std::string> chunks;
        {
          py::gil_scoped_release nogil;  // listing + reads may hit a (Python) server
          io::URI path(uri.c_str());
          io::FileSystem* fs = io::FileSystem::GetInstance(path);
          std::unique_ptr<io::InputSplitBase> split;
          if (type == "text") {
            split.reset(new io::LineSplitter(fs, uri.c_str(), part, nparts));
          } else {
            split.reset(new io::RecordIOSplitter(fs, uri.c_str(), part, nparts));
          }
          io::ShardReader reader(split.get(), nthread);
          std::string buf(chunk_bytes, '\0');
          for (;;) {
            size_t n = reader.Fill(&buf[0], buf.size());
            while (n == io::ShardReader::kNeedMore) {
              buf.resize(reader.NeedCapacity());
              n = reader.Fill(&buf[0], buf.size());
            }
            if (n == 0) break;
            chunks.emplace_back(buf.data(), n);
          }
        }
        py::list out;
        for (auto& c : chunks) out.append(py::bytes(c));
        return out;
      },
      py::arg("uri"), py::arg("part") = 0, py::arg("nparts") = 1, py::arg("type") = "text",
      py::arg("nthread") = 8, py::arg("chunk_bytes") = 64UL << 20);
  m.def(
      "http_stats",
      []() {
        py::dict d;
        d["native_gets"] = io::Http::NativeGets();
        d["native_fallbacks"] = io::Http::NativeFallbacks();
        return d;
      },
      "process-wide counts of ranged GETs received natively / handed to libcurl");
  m.def("fault_configure", &fault::Configure, py::arg("spec"),
        "arm DMLC_FAULT_INJECT-style faults (\"\" disarms); resets pass counters");
  m.def("fault_count", &fault::Count, py::arg("point"));
  m.def("gpu_device_count", &gpu::DeviceCount);
  m.def("gpu_arch", &gpu::DeviceArchName);
  m.def("get_time", &GetTime);

  // ---------------------------------------------------------------- dist
  using dist::TrackerClient;
  py::class_<TrackerClient>(m, "TrackerClient")
      .def(py::init<std::string, int, std::string, int, int, double>(), py::arg("uri") = "",
           py::arg("port") = 0, py::arg("jobid") = "", py::arg("rank") = -1,
           py::arg("world_size") = -1, py::arg("timeout") = 600.0)
      .def("start",
           [](TrackerClient& c, bool recover) {
             dist::Topology t;
             {
               py::gil_scoped_release nogil;
               t = c.Start(recover);
             }
             return py::make_tuple(t.rank, t.parent, t.world_size, t.tree, t.ring_prev,
                                   t.ring_next);
           },
           py::arg("recover") = false)
      .def("print", &TrackerClient::Print, py::call_guard<py::gil_scoped_release>())
      .def("shutdown", &TrackerClient::Shutdown, py::call_guard<py::gil_scoped_release>())
      .def("heartbeat",
           [](TrackerClient& c) -> py::object {
             std::string reason;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = c.Heartbeat(&reason);
             }
             if (ok) return py::none();
             return py::str(reason);
           })
      .def("abort", &TrackerClient::Abort, py::call_guard<py::gil_scoped_release>())
      // the first heartbeat is synchronous: never hold the GIL across it (an
      // in-process Python tracker needs the GIL to answer)
      .def("start_heartbeat", &TrackerClient::StartHeartbeat, py::arg("period") = 5.0,
           py::call_guard<py::gil_scoped_release>())
      .def("stop_heartbeat", &TrackerClient::StopHeartbeat,
           py::call_guard<py::gil_scoped_release>())
      .def("rccl_put",
           [](TrackerClient& c, const std::string& key, py::bytes blob) {
             std::string b = blob;
             py::gil_scoped_release nogil;
             c.RcclPut(key, b);
           })
      .def("rccl_get",
           [](TrackerClient& c, const std::string& key) {
             std::string b;
             {
               py::gil_scoped_release nogil;
               b = c.RcclGet(key);
             }
             return py::bytes(b);
           })
      .def("attempt", &TrackerClient::Attempt, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &TrackerClient::Barrier, py::arg("key") = "default",
           py::arg("count") = -1, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &TrackerClient::rank)
      .def_property_readonly("world_size", &TrackerClient::world_size);

  using dist::Communicator;
  py::enum_<dist::DataType>(m, "DataType")
      .value("int8", dist::DataType::kInt8).value("uint8", dist::DataType::kUInt8)
      .value("int32", dist::DataType::kInt32).value("uint32", dist::DataType::kUInt32)
      .value("int64", dist::DataType::kInt64).value("uint64", dist::DataType::kUInt64)
      .value("float16", dist::DataType::kFloat16).value("float32", dist::DataType::kFloat32)
      .value("float64", dist::DataType::kFloat64).value("bfloat16", dist::DataType::kBFloat16);
  py::enum_<dist::ReduceOp>(m, "ReduceOp")
      .value("sum", dist::ReduceOp::kSum).value("prod", dist::ReduceOp::kProd)
      .value("max", dist::ReduceOp::kMax).value("min", dist::ReduceOp::kMin)
      .value("avg", dist::ReduceOp::kAvg);
  py::class_<Communicator>(m, "Communicator")
      .def(py::init([](int rank, int world, int device, py::bytes uid) {
             std::string id = uid;
             py::gil_scoped_release nogil;
             return new Communicator(rank, world, device, id);
           }),
           py::arg("rank"), py::arg("world_size"), py::arg("device"), py::arg("unique_id"))
      .def_static("available", &Communicator::Available)
      .def_static("library_path", &Communicator::LibraryPath)
      .def_static("new_unique_id", []() { return py::bytes(Communicator::NewUniqueId()); })
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world_size", &Communicator::world_size)
      .def_property_readonly("device", &Communicator::device)
      .def_property_readonly("aborted", &Communicator::aborted)
      .def("abort", &Communicator::Abort, py::call_guard<py::gil_scoped_release>())
      .def("abort_on_tracker_failure", &Communicator::AbortOnTrackerFailure,
           py::keep_alive<1, 2>())
      .def("all_reduce",
           [stream_of](Communicator& c, uintptr_t send, uintptr_t recv, size_t count,
                       dist::DataType dt, dist::ReduceOp op, uintptr_t stream) {
             c.AllReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                         dt, op, stream_of(stream));
           })
      .def("broadcast",
           [stream_of](Communicator& c, uintptr_t send, uintptr_t recv, size_t count,
                       dist::DataType dt, int root, uintptr_t stream) {
             c.Broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                         dt, root, stream_of(stream));
           })
      .def("all_gather",
           [stream_of](Communicator& c, uintptr_t send, uintptr_t recv, size_t count,
                       dist::DataType dt, uintptr_t stream) {
             c.AllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                         dt, stream_of(stream));
           })
      .def("reduce_scatter",
           [stream_of](Communicator& c, uintptr_t send, uintptr_t recv, size_t count,
                       dist::DataType dt, dist::ReduceOp op, uintptr_t stream) {
             c.ReduceScatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                             count, dt, op, stream_of(stream));
           })
      .def("all_to_all_v",
           [stream_of](Communicator& c, uintptr_t send, std::vector<size_t> sc,
                       std::vector<size_t> sd, uintptr_t recv, std::vector<size_t> rc,
                       std::vector<size_t> rd, dist::DataType dt, uintptr_t stream) {
             c.AllToAllV(reinterpret_cast<const void*>(send), sc, sd, reinterpret_cast<void*>(recv),
                         rc, rd, dt, stream_of(stream));
           })
      .def("barrier", [stream_of](Communicator& c, uintptr_t stream) {
        py::gil_scoped_release nogil;
        c.Barrier(stream_of(stream));
      })
      .def("abort", &Communicator::Abort);
}
