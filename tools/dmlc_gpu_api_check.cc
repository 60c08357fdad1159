// dmlc_gpu_api_check: the reference's public data API on the GPU path.
//   Parser<I>::Create(uri + "?device=gpu", part, nparts, type)   (host blocks; device
//                                                  blocks with &device_ptrs=1)
//   RowBlockIter<I>::Create(uri + "?device=gpu&device_ptrs=1", ...) (whole shard in HBM)
// Every block is copied back with hipMemcpy and compared value by value with
// the CPU parser over the same partition.  Exit 0 = identical.
//
//   dmlc_gpu_api_check <uri> <type> <nparts> [extra uri args, e.g. chunk_bytes=65536]
#include <dmlc/data.h>
#include <dmlc/logging.h>
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

namespace {

struct Rows {
  std::vector<float> label, weight, value;
  std::vector<uint64_t> qid;
  std::vector<uint32_t> index, field;
  std::vector<size_t> row_nnz;
};

template <typename T>
void Append(std::vector<T>* dst, const T* src, size_t n, bool device) {
  if (src == nullptr || n == 0) return;
  const size_t at = dst->size();
  dst->resize(at + n);
  if (device) {
    if (hipMemcpy(dst->data() + at, src, n * sizeof(T), hipMemcpyDeviceToHost) != hipSuccess) {
      std::fprintf(stderr, "hipMemcpy failed\n");
      std::exit(3);
    }
  } else {
    std::copy(src, src + n, dst->data() + at);
  }
}

void AddBlock(const dmlc::RowBlock<uint32_t>& b, bool device, Rows* r) {
  std::vector<size_t> off;
  Append(&off, b.offset, b.size + 1, device);
  const size_t base = off.empty() ? 0 : off[0];
  const size_t nnz = off.empty() ? 0 : off[b.size] - base;
  for (size_t i = 0; i < b.size; ++i) r->row_nnz.push_back(off[i + 1] - off[i]);
  Append(&r->label, b.label, b.size, device);
  // absent optional columns mean "every weight 1 / qid 0 / value 1"
  if (b.weight != nullptr) {
    Append(&r->weight, b.weight, b.size, device);
  } else {
    r->weight.insert(r->weight.end(), b.size, 1.0f);
  }
  if (b.qid != nullptr) {
    Append(&r->qid, b.qid, b.size, device);
  } else {
    r->qid.insert(r->qid.end(), b.size, 0);
  }
  Append(&r->index, b.index + base, nnz, device);
  if (b.value != nullptr) {
    Append(&r->value, b.value + base, nnz, device);
  } else {
    r->value.insert(r->value.end(), nnz, 1.0f);
  }
  if (b.field != nullptr) Append(&r->field, b.field + base, nnz, device);
}

template <typename Iter>
Rows Drain(Iter* it, bool device) {
  Rows r;
  it->BeforeFirst();
  while (it->Next()) AddBlock(it->Value(), device, &r);
  return r;
}

bool Same(const Rows& a, const Rows& b, const char* what) {
  bool ok = a.label == b.label && a.weight == b.weight && a.qid == b.qid && a.index == b.index &&
            a.value == b.value && a.field == b.field && a.row_nnz == b.row_nnz;
  std::printf("%s: %zu rows, %zu entries: %s\n", what, a.label.size(), a.index.size(),
              ok ? "identical" : "DIFFERENT");
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s uri type nparts [args]\n", argv[0]);
    return 2;
  }
  const std::string uri = argv[1], type = argv[2];
  const unsigned nparts = static_cast<unsigned>(std::atoi(argv[3]));
  const std::string extra = argc > 4 ? std::string("&") + argv[4] : "";
  const std::string sep = uri.find('?') == std::string::npos ? "?" : "&";
  bool ok = true;
  for (unsigned part = 0; part < nparts; ++part) {
    std::unique_ptr<dmlc::Parser<uint32_t>> cpu(
        dmlc::Parser<uint32_t>::Create(uri.c_str(), part, nparts, type.c_str()));
    const Rows ref = Drain(cpu.get(), false);
    const std::string g = uri + sep + "device=gpu" + extra;
    std::unique_ptr<dmlc::Parser<uint32_t>> gp(
        dmlc::Parser<uint32_t>::Create((g + "&device_ptrs=1").c_str(), part, nparts, type.c_str()));
    ok &= Same(Drain(gp.get(), true), ref, "Parser device=gpu&device_ptrs=1");
    std::unique_ptr<dmlc::Parser<uint32_t>> gh(
        dmlc::Parser<uint32_t>::Create(g.c_str(), part, nparts, type.c_str()));
    ok &= Same(Drain(gh.get(), false), ref, "Parser device=gpu (host blocks by default)");
    std::unique_ptr<dmlc::RowBlockIter<uint32_t>> it(
        dmlc::RowBlockIter<uint32_t>::Create((g + "&device_ptrs=1").c_str(), part, nparts,
                                             type.c_str()));
    ok &= Same(Drain(it.get(), true), ref, "RowBlockIter device=gpu&device_ptrs=1");
    std::unique_ptr<dmlc::RowBlockIter<uint32_t>> cit(
        dmlc::RowBlockIter<uint32_t>::Create(uri.c_str(), part, nparts, type.c_str()));
    if (it->NumCol() != cit->NumCol()) {
      std::printf("NumCol differs: gpu %zu cpu %zu\n", it->NumCol(), cit->NumCol());
      ok = false;
    }
  }
  std::printf("%s\n", ok ? "OK" : "FAILED");
  return ok ? 0 : 1;
}
