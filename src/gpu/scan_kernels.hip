/*!
 * \file src/gpu/scan_kernels.hip
 * \brief K3: device-wide exclusive scan of u64 (reduce -> scan partials ->
 *  down-sweep), used for line offsets and CSR row pointers.
 *
 * 256-thread workgroups, 8 elements per lane (2048 per tile), 16-byte loads.
 * The partial sums are scanned by a single workgroup that walks them in
 * 2048-wide tiles, so any n works without recursion.
 */
#include <hip/hip_runtime.h>

#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {

namespace {
constexpr int kThreads = 256;
constexpr int kPer = 8;
constexpr size_t kTile = kThreads * kPer;

__device__ __forceinline__ void load8(const uint64_t* in, size_t base, size_t n, uint64_t (&v)[kPer]) {
  if (base + kPer <= n) {
    const ulonglong2* p = reinterpret_cast<const ulonglong2*>(in + base);
#pragma unroll
    for (int i = 0; i < kPer / 2; ++i) {
      ulonglong2 t = p[i];
      v[2 * i] = t.x;
      v[2 * i + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kPer; ++i) v[i] = base + i < n ? in[base + i] : 0;
  }
}

__global__ __launch_bounds__(kThreads) void k_scan_reduce(const uint64_t* __restrict__ in, size_t n,
                                                          uint64_t* __restrict__ partials) {
  __shared__ uint64_t smem[4];
  const size_t base = blockIdx.x * kTile + threadIdx.x * kPer;
  uint64_t v[kPer];
  load8(in, base, n, v);
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) s += v[i];
  s = dev::block_sum_256(s, smem);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void k_scan_partials(uint64_t* __restrict__ partials,
                                                            size_t np, uint64_t* __restrict__ total) {
  __shared__ uint64_t smem[4];
  uint64_t carry = 0;
  for (size_t t = 0; t < np; t += kTile) {
    const size_t base = t + threadIdx.x * kPer;
    uint64_t v[kPer];
    load8(partials, base, np, v);
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) s += v[i];
    uint64_t tile_total;
    uint64_t x = dev::block_excl_scan_256(s, smem, &tile_total) + carry;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      if (base + i < np) partials[base + i] = x;
      x += v[i];
    }
    carry += tile_total;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(kThreads) void k_scan_down(uint64_t* __restrict__ data, size_t n,
                                                        const uint64_t* __restrict__ partials) {
  __shared__ uint64_t smem[4];
  const size_t base = blockIdx.x * kTile + threadIdx.x * kPer;
  uint64_t v[kPer];
  load8(data, base, n, v);
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) s += v[i];
  uint64_t tot;
  uint64_t x = dev::block_excl_scan_256(s, smem, &tot) + partials[blockIdx.x];
  if (base + kPer <= n) {
    uint64_t o[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      o[i] = x;
      x += v[i];
    }
    ulonglong2* p = reinterpret_cast<ulonglong2*>(data + base);
#pragma unroll
    for (int i = 0; i < kPer / 2; ++i) p[i] = make_ulonglong2(o[2 * i], o[2 * i + 1]);
  } else {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      if (base + i < n) data[base + i] = x;
      x += v[i];
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_reduce_partials(const MetaPartial* __restrict__ p,
                                                              int n, ChunkMeta* meta) {
  unsigned long long mi = 0, mf = 0;
  unsigned fl = 0;
  for (int i = threadIdx.x; i < n; i += kThreads) {
    const MetaPartial q = p[i];
    mi = q.max_index > mi ? q.max_index : mi;
    mf = q.max_field > mf ? q.max_field : mf;
    fl |= q.flags;
  }
  __shared__ unsigned long long s_mi[4], s_mf[4];
  __shared__ unsigned s_fl[4];
  mi = dev::wave_max(mi);
  mf = dev::wave_max(mf);
  fl = dev::wave_or(fl);
  const int wid = threadIdx.x / dev::kWave;
  if (dev::lane_id() == 0) {
    s_mi[wid] = mi;
    s_mf[wid] = mf;
    s_fl[wid] = fl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      s_mi[0] = s_mi[w] > s_mi[0] ? s_mi[w] : s_mi[0];
      s_mf[0] = s_mf[w] > s_mf[0] ? s_mf[w] : s_mf[0];
      s_fl[0] |= s_fl[w];
    }
    // single writer, stream ordered: merge into what earlier kernels stored
    meta->max_index = s_mi[0] > meta->max_index ? s_mi[0] : meta->max_index;
    meta->max_field = s_mf[0] > meta->max_field ? s_mf[0] : meta->max_field;
    meta->flags |= s_fl[0];
  }
}

__global__ void k_meta_from_total(const uint64_t* __restrict__ total, ChunkMeta* meta) {
  const uint64_t t = *total;
  meta->nrows = t >> 32;
  meta->nnz = t & 0xffffffffull;
}
}  // namespace

size_t ScanPartials(size_t n) { return (n + kTile - 1) / kTile; }

void LaunchScanU64(uint64_t* data, size_t n, uint64_t* partials, uint64_t* total,
                   hipStream_t stream) {
  if (n == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(uint64_t), stream);
    return;
  }
  const size_t np = ScanPartials(n);
  hipLaunchKernelGGL(k_scan_reduce, dim3(np), dim3(kThreads), 0, stream, data, n, partials);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(kThreads), 0, stream, partials, np, total);
  hipLaunchKernelGGL(k_scan_down, dim3(np), dim3(kThreads), 0, stream, data, n, partials);
}

void LaunchReducePartials(const MetaPartial* partials, int nblocks, ChunkMeta* meta,
                          hipStream_t stream) {
  hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kThreads), 0, stream, partials, nblocks,
                     meta);
}

void LaunchMetaFromTotal(const uint64_t* total, ChunkMeta* meta, hipStream_t stream) {
  hipLaunchKernelGGL(k_meta_from_total, dim3(1), dim3(1), 0, stream, total, meta);
}

}  // namespace gpu
}  // namespace dmlc
