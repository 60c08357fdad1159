/*!
 * \file src/gpu/device_common.h
 * \brief Wave64 / workgroup primitives shared by the gfx950 kernels.
 *
 * CDNA4 rules applied (cdna_hip_programming.md §1, §6): waves are 64 lanes,
 * ballots are 64-bit, all block sizes are multiples of 64, cross-lane data
 * moves through DPP/permute (__shfl*) rather than LDS where possible.
 */
#ifndef DMLC_GPU_DEVICE_COMMON_H_
#define DMLC_GPU_DEVICE_COMMON_H_

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace dmlc {
namespace gpu {
namespace dev {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

/*! \brief make LDS writes of this wave visible to the other lanes of the wave */
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/*! \brief x of lane - 1 (lane 0: 0): DPP wave_shr:1, no LDS crossbar trip */
__device__ __forceinline__ uint32_t lane_shr1(uint32_t x) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x138, 0xF, 0xF, false));
}

/*! \brief x of lane + 1 (lane 63: 0): DPP wave_shl:1 */
__device__ __forceinline__ uint32_t lane_shl1(uint32_t x) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x130, 0xF, 0xF, false));
}

/*! \brief x of lane 63, as a scalar (uniform to the compiler) */
__device__ __forceinline__ uint32_t lane63(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
}

/*! \brief a wave-uniform value made scalar (the compiler then keeps the
 *  control flow on it uniform: scalar branches, no exec-mask bookkeeping) */
__device__ __forceinline__ uint32_t uniform(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(x)));
}
__device__ __forceinline__ uint64_t uniform(uint64_t x) {
  return static_cast<uint64_t>(uniform(static_cast<uint32_t>(x))) |
         (static_cast<uint64_t>(uniform(static_cast<uint32_t>(x >> 32))) << 32);
}

/*!
 * \brief inclusive u32 prefix sum over the wave with DPP only: row_shr 1/2/4/8
 *  within each 16-lane row, then row_bcast:15 / row_bcast:31 across rows (the
 *  GFX9 / CDNA cross-row broadcasts) -- six VALU ops against six LDS-crossbar
 *  round trips of a __shfl_up ladder.  Lanes without a source add 0.
 */
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  int x = static_cast<int>(v);
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return static_cast<uint32_t>(x);
}

/*!
 * \brief inclusive scan under an associative op whose identity is 0
 *  (op(0, x) == x; op(earlier, later)), by the same DPP ladder as
 *  wave_incl_scan_u32 -- e.g. a segmented sum with a reset flag bit
 */
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_pull(uint32_t x) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(x), kCtrl, kRowMask, 0xF, false));
}
template <typename Op>
__device__ __forceinline__ uint32_t wave_incl_scan_op(uint32_t v, Op op) {
  uint32_t x = v;
  x = op(dpp_pull<0x111, 0xF>(x), x);  // row_shr:1
  x = op(dpp_pull<0x112, 0xF>(x), x);  // row_shr:2
  x = op(dpp_pull<0x114, 0xF>(x), x);  // row_shr:4
  x = op(dpp_pull<0x118, 0xF>(x), x);  // row_shr:8
  x = op(dpp_pull<0x142, 0xA>(x), x);  // row_bcast:15 -> rows 1, 3
  x = op(dpp_pull<0x143, 0xC>(x), x);  // row_bcast:31 -> rows 2, 3
  return x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  if constexpr (std::is_integral<T>::value && sizeof(T) == 4) {
    return static_cast<T>(lane63(wave_incl_scan_u32(static_cast<uint32_t>(v))));
  } else {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
  }
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    T o = __shfl_xor(v, d, kWave);
    v = o > v ? o : v;
  }
  return v;
}

/*! \brief exclusive prefix sum across the wave; *total = wave sum */
template <typename T>
__device__ __forceinline__ T wave_excl_scan(T v, T* total) {
  if constexpr (std::is_integral<T>::value && sizeof(T) == 4) {
    const uint32_t x = wave_incl_scan_u32(static_cast<uint32_t>(v));
    *total = static_cast<T>(lane63(x));
    return static_cast<T>(x - static_cast<uint32_t>(v));
  } else {
    const int lane = lane_id();
    T x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      T y = __shfl_up(x, d, kWave);
      if (lane >= d) x += y;
    }
    *total = __shfl(x, kWave - 1, kWave);
    return x - v;
  }
}

/*! \brief wave_sum of a u64 made of two u32 counters that never carry */
__device__ __forceinline__ uint64_t wave_sum_2x32(uint64_t v) {
  return (static_cast<uint64_t>(wave_sum(static_cast<uint32_t>(v >> 32))) << 32) |
         wave_sum(static_cast<uint32_t>(v));
}

/*! \brief wave_excl_scan of a u64 made of two u32 counters that never carry
 *  into each other (packed per-lane counts): two DPP scans */
__device__ __forceinline__ uint64_t wave_excl_scan_2x32(uint64_t v, uint64_t* total) {
  uint32_t tlo, thi;
  const uint32_t lo = wave_excl_scan(static_cast<uint32_t>(v), &tlo);
  const uint32_t hi = wave_excl_scan(static_cast<uint32_t>(v >> 32), &thi);
  *total = (static_cast<uint64_t>(thi) << 32) | tlo;
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

/*!
 * \brief exclusive prefix across a 256-thread block (4 waves); *total = sum.
 *  `smem` needs 4 elements; contains a __syncthreads.
 */
template <typename T>
__device__ __forceinline__ T block_excl_scan_256(T v, T* smem, T* total) {
  T wtotal;
  T x = wave_excl_scan(v, &wtotal);
  const int wid = threadIdx.x / kWave;
  if (lane_id() == 0) smem[wid] = wtotal;
  __syncthreads();
  T base = 0, sum = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    T t = smem[w];
    if (w < wid) base += t;
    sum += t;
  }
  *total = sum;
  return base + x;
}

template <typename T>
__device__ __forceinline__ T block_sum_256(T v, T* smem) {
  T t;
  (void)block_excl_scan_256(v, smem, &t);
  return t;
}

template <typename T>
__device__ __forceinline__ T wave_or(T v) {
  if constexpr (std::is_integral<T>::value && sizeof(T) == 4) {
    return static_cast<T>(lane63(wave_incl_scan_op(static_cast<uint32_t>(v),
                                                    [](uint32_t a, uint32_t b) { return a | b; })));
  } else {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d, kWave);
    return v;
  }
}

/*!
 * \brief reduce (max, max, or) over a 256-thread workgroup and store the
 *  result in slot blockIdx.x — every thread of the block must call it.
 */
template <typename Partial>
__device__ __forceinline__ void block_store_partial(unsigned long long mi, unsigned long long mf,
                                                    unsigned fl, Partial* partials) {
  __shared__ unsigned long long s_mi[4], s_mf[4];
  __shared__ unsigned s_fl[4];
  mi = wave_max(mi);
  mf = wave_max(mf);
  fl = wave_or(fl);
  const int wid = threadIdx.x / kWave;
  if (lane_id() == 0) {
    s_mi[wid] = mi;
    s_mf[wid] = mf;
    s_fl[wid] = fl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Partial p;
    p.max_index = s_mi[0];
    p.max_field = s_mf[0];
    p.flags = s_fl[0];
    p.pad = 0;
    for (int w = 1; w < static_cast<int>(blockDim.x) / kWave; ++w) {
      p.max_index = s_mi[w] > p.max_index ? s_mi[w] : p.max_index;
      p.max_field = s_mf[w] > p.max_field ? s_mf[w] : p.max_field;
      p.flags |= s_fl[w];
    }
    partials[blockIdx.x] = p;
  }
}

/*!
 * \brief decoupled look-back over per-tile count pairs -- the one-pass
 *  kernels' replacement of a count kernel + scan.  Word: state (1: this tile's
 *  own counts, 2: inclusive prefix; 0: not yet -- the array is zeroed by a
 *  hipMemsetAsync before every launch) << 62 | hi << kLoBits | lo; the caller
 *  guarantees that every prefix of hi fits 62 - kLoBits bits and of lo
 *  kLoBits (no carries between the packed fields).  The word is the data and
 *  the flag at once (one 8-byte agent-scope store, relaxed agent-scope polls:
 *  the granule form of cdna_hip_programming.md Guideline 16, R2).  Tiles run
 *  in ticket order, so every tile waited on is resident or done.  Returns the
 *  exclusive prefix (packed the same way).
 */
template <int kLoBits>
__device__ __forceinline__ uint64_t lookback_pairs(uint64_t* st, size_t tile, uint64_t own, int lane) {
  constexpr uint64_t kVal = (1ull << 62) - 1ull;
  constexpr uint64_t kLo = (1ull << kLoBits) - 1ull;
  if (lane == 0) {
    __hip_atomic_store(&st[tile], ((tile == 0 ? 2ull : 1ull) << 62) | own, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tile == 0) return 0;
  uint32_t ex_hi = 0, ex_lo = 0;
  int64_t j = static_cast<int64_t>(tile) - 1;  // the nearest predecessor not summed yet
  for (;;) {
    const int64_t k = j - lane;
    const uint64_t v = k >= 0 ? __hip_atomic_load(&st[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : (2ull << 62);  // before the chunk: inclusive 0
    const uint32_t state = static_cast<uint32_t>(v >> 62);
    const uint64_t inc = __ballot(state == 2u);
    const uint64_t waiting = __ballot(state == 0u);
    const int first = inc != 0 ? __builtin_ctzll(inc) : kWave - 1;
    const uint64_t need = first >= kWave - 1 ? ~0ull : ((2ull << first) - 1ull);
    if ((waiting & need) != 0) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint64_t x = lane <= first ? (v & kVal) : 0ull;
    ex_hi += wave_sum(static_cast<uint32_t>(x >> kLoBits));
    ex_lo += wave_sum(static_cast<uint32_t>(x & kLo));
    if (inc != 0) break;
    j -= kWave;
  }
  const uint64_t excl = (static_cast<uint64_t>(ex_hi) << kLoBits) | ex_lo;
  if (lane == 0) {
    __hip_atomic_store(&st[tile], (2ull << 62) | (excl + own), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  return excl;
}

/*!
 * \brief 16-bit mask of the bytes of a 16-byte vector equal to `c`
 *  (exact SWAR zero-byte test per 32-bit word).
 */
__device__ __forceinline__ uint32_t byte_eq_mask(uint4 v, uint32_t c) {
  const uint32_t pat = c * 0x01010101u;
  uint32_t m = 0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = w[i] ^ pat;
    // high bit of each byte set iff that byte of x is zero
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    // gather the 4 high bits into bits 0..3
    const uint32_t g = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
    m |= g << (4 * i);
  }
  return m;
}

/*!
 * \brief K9 feature hash (murmur3 fmix64 of the key mixed with the seed); the
 *  low bits pick the bucket (h % dim), bit 31 the sign.  Shared by the CSR ->
 *  dense kernel and the fused text -> dense kernel so both hash identically.
 */
__device__ __forceinline__ uint32_t hash_u64(uint64_t x, uint32_t seed) {
  x ^= static_cast<uint64_t>(seed) * 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 33)) * 0xff51afd7ed558ccdull;
  x = (x ^ (x >> 33)) * 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

/*! \brief the K9 key of a (field, index) pair: fields occupy bits 40+ */
__device__ __forceinline__ uint64_t hash_key(uint64_t index, uint64_t field, bool has_field) {
  return has_field ? (index ^ (field << 40)) : index;
}

__device__ __forceinline__ uint8_t vec_byte(uint4 v, int j) {
  const uint32_t w = j < 4 ? v.x : (j < 8 ? v.y : (j < 12 ? v.z : v.w));
  return static_cast<uint8_t>(w >> (8 * (j & 3)));
}

}  // namespace dev
}  // namespace gpu
}  // namespace dmlc
#endif  // DMLC_GPU_DEVICE_COMMON_H_
