/*!
 * \file src/gpu/fm_kernels.hip
 * \brief HashedFM (BASELINE config 5) forward / backward on the fp8 hashed
 *  batch, bf16 MFMA on gfx950, the batch read once per pass.
 *
 * Model: y_r = b + s x_r.w + 1/2 (sum_f (s x_r.V_f)^2 - s^2 x_r^2.q),
 * q_n = sum_f V_nf^2 (the x^2 V^2 term summed over f is one dot product with
 * q), x = fp8 e4m3 codes, s = 1 / quantisation scale.
 *
 * F1 k_fm_fwd: a wave takes 32 rows; per 128-feature block each lane loads
 *   64 contiguous bytes of its row (lanes l and l+32 the two halves of a
 *   128-byte line) and feeds them, 8 at a time, as the A fragment of
 *   v_mfma_f32_32x32x16_bf16 against B = [w | V] (bf16, LDS-resident,
 *   columns 17..31 zero).  The K order inside a block is permuted the same way
 *   for A and B, so no data moves between lanes.  x^2.q accumulates on the
 *   VALU from the same converted registers.  The epilogue reduces (xV)^2 over
 *   the 16 V lanes with xor-shuffles and writes y and xV (kept for F2).
 * F2 k_fm_bwd: with g = dL/dy and G_r = [g_r, g_r xV_r] (17 columns),
 *   Z = G^T X (summed over rows) and t = (x^2)^T g give every gradient:
 *   dw = s Z_0, dV_nf = s Z_{1+f,n} - V_nf s^2 t_n.  Rows are the reduction
 *   index, so X must arrive with rows along K: each wave writes its 32-row X
 *   tile to LDS and reads it back transposed (ds_read_b64_tr_b8: 8 rows of
 *   one feature per lane), the B operand of the MFMA with G^T from LDS in
 *   the same row order.  Eight waves share one G tile
 *   (double-buffered in LDS: one barrier per 32-row tile); each
 *   keeps 128 features of Z in 64 accumulator registers and writes one
 *   partial per workgroup.
 * F3 k_fm_reduce + F4 k_fm_grads: the partials summed in a fixed order and
 *   turned into dw, dV on the device (no torch reduction over the partials).
 */
#include <dmlc/logging.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "./device_common.h"
#include "./kernels.h"

namespace dmlc {
namespace gpu {
namespace {

using namespace dev;  // NOLINT(build/namespaces)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef int v2i __attribute__((ext_vector_type(2)));

constexpr int kFwdThreads = 256;
constexpr int kBwdThreads = 512;  // 8 waves x 128 features = 1024 features per workgroup
constexpr int kBwdWaveFeatures = 128;

/*! \brief two dwords of fp8 e4m3 codes -> 8 floats (exact) */
__device__ __forceinline__ void fp8x8(uint32_t lo, uint32_t hi, float f[8]) {
  const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(lo), false);
  const f32x2 b = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(lo), true);
  const f32x2 c = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(hi), false);
  const f32x2 d = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(hi), true);
  f[0] = a[0];
  f[1] = a[1];
  f[2] = b[0];
  f[3] = b[1];
  f[4] = c[0];
  f[5] = c[1];
  f[6] = d[0];
  f[7] = d[1];
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

/*! \brief two dwords of fp8 e4m3 codes -> 8 bf16 (exact: e4m3 fits bf16),
 *  gfx950's packed scaled conversion, 4 instructions */
__device__ __forceinline__ bf16x8 fp8x8_bf16(uint32_t lo, uint32_t hi) {
  const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(static_cast<int>(lo), 1.0f, false);
  const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(static_cast<int>(lo), 1.0f, true);
  const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(static_cast<int>(hi), 1.0f, false);
  const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(static_cast<int>(hi), 1.0f, true);
  bf16x8 v;
  v[0] = a[0];
  v[1] = a[1];
  v[2] = b[0];
  v[3] = b[1];
  v[4] = c[0];
  v[5] = c[1];
  v[6] = d[0];
  v[7] = d[1];
  return v;
}

__device__ __forceinline__ uint32_t word(const uint4 (&v)[4], int i) {
  const uint4 q = v[i >> 2];
  const int k = i & 3;
  return k == 0 ? q.x : (k == 1 ? q.y : (k == 2 ? q.z : q.w));
}

__device__ __forceinline__ void load64(const uint8_t* p, bool valid, uint4 (&v)[4]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = valid ? q[i] : make_uint4(0, 0, 0, 0);
}

/*!
 * F1.  LDS: [w | V]^T as bf16 [17][dim + 8] (the pad spreads the 17 B-lanes
 * over bank quads) then q as f32 [dim].
 */
__global__ __launch_bounds__(kFwdThreads) void k_fm_fwd(const uint8_t* __restrict__ x,
                                                        int64_t rows, int dim,
                                                        const __bf16* __restrict__ wt,
                                                        const float* __restrict__ q,
                                                        const float* __restrict__ bias, float sx,
                                                        float* __restrict__ y,
                                                        float* __restrict__ xv) {
  extern __shared__ uint4 smem[];
  const int ldw = dim + 8;
  __bf16* s_wt = reinterpret_cast<__bf16*>(smem);
  float* s_q = reinterpret_cast<float*>(s_wt + kFmCols * ldw);
  for (int i = threadIdx.x; i < kFmCols * dim / 8; i += kFwdThreads) {
    const int c = i / (dim / 8), k8 = i % (dim / 8);
    *reinterpret_cast<uint4*>(s_wt + c * ldw + 8 * k8) =
        reinterpret_cast<const uint4*>(wt + static_cast<size_t>(c) * dim)[k8];
  }
  for (int i = threadIdx.x; i < dim / 4; i += kFwdThreads) {
    reinterpret_cast<float4*>(s_q)[i] = reinterpret_cast<const float4*>(q)[i];
  }
  __syncthreads();
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  const int waves = kFwdThreads / kWave;
  const int64_t ntiles = (rows + 31) / 32;
  const float b0 = *bias;
  const int nblk = dim / 128;
  const bf16x8 zero8 = {};
  // The wave's (tile, block) pairs form one stream; blocks rotate through three
  // register buffers, each refilled (two blocks ahead, across row tiles too)
  // right after its MFMAs consumed it -- no register copies of loads in
  // flight, so a block's wait only covers what was issued before it.  Loads
  // are unconditional (clamped row, zeroed past the rows).
  const int64_t tfirst = static_cast<int64_t>(blockIdx.x) * waves + threadIdx.x / kWave;
  const int64_t tstride = static_cast<int64_t>(gridDim.x) * waves;
  const int64_t rlast = rows - 1;
  int64_t lt = tfirst;  // the load cursor: tile, block
  int lkb = 0;
  auto issue = [&](uint4 (&v)[4]) {
    const int64_t r = lt * 32 + col;
    const bool ok = lt < ntiles && r < rows;
    const int64_t rc = r < rlast ? r : rlast;
    const uint4* q = reinterpret_cast<const uint4*>(x + rc * dim + 64 * h + 128 * lkb);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 u = q[i];
      v[i] = ok ? u : make_uint4(0, 0, 0, 0);
    }
    if (++lkb == nblk) {
      lkb = 0;
      lt += tstride;
    }
  };
  int64_t t = tfirst;  // the compute cursor
  int kb = 0;
  f32x16 acc = {};
  f32x2 x2q2 = {0.0f, 0.0f};
  // one block of the current tile from buffer cur; the tile's epilogue after
  // its last block.  false once the wave's tiles are done
  auto step = [&](const uint4 (&cur)[4]) {
    if (t >= ntiles) return false;
    const int kbase = 128 * kb + 64 * h;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t lo = word(cur, 2 * i), hi = word(cur, 2 * i + 1);
      float f[8];
      fp8x8(lo, hi, f);
      const float4 q0 = *reinterpret_cast<const float4*>(s_q + kbase + 8 * i);
      const float4 q1 = *reinterpret_cast<const float4*>(s_q + kbase + 8 * i + 4);
      // x^2.q in packed f32 (v_pk_mul / v_pk_fma), two partial sums
      f32x2 sq[4] = {{f[0], f[1]}, {f[2], f[3]}, {f[4], f[5]}, {f[6], f[7]}};
      const f32x2 qq[4] = {{q0.x, q0.y}, {q0.z, q0.w}, {q1.x, q1.y}, {q1.z, q1.w}};
#pragma unroll
      for (int k = 0; k < 4; ++k) x2q2 = __builtin_elementwise_fma(sq[k] * sq[k], qq[k], x2q2);
      const bf16x8 b = col < kFmCols
                           ? *reinterpret_cast<const bf16x8*>(s_wt + col * ldw + kbase + 8 * i)
                           : zero8;
      // A straight from the fp8 codes (exact), not through f32
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fp8x8_bf16(lo, hi), b, acc, 0, 0, 0);
    }
    if (++kb == nblk) {
      // lanes r and r + 32 hold the two halves of row r's x^2.q
      float x2q = x2q2[0] + x2q2[1];
      x2q += __shfl_xor(x2q, 32, kWave);
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int m = (reg & 3) + 8 * (reg >> 2) + 4 * h;  // accumulator row (C/D map)
        const float v = acc[reg];
        float sq = (col >= 1 && col <= kFmRank) ? v * v : 0.0f;
#pragma unroll
        for (int d = 1; d < 32; d <<= 1) sq += __shfl_xor(sq, d, kWave);
        const float lin = __shfl(v, h * 32, kWave);
        const float xq = __shfl(x2q, m, kWave);
        const int64_t r = t * 32 + m;
        if (r < rows) {
          if (col == 0) {
            y[r] = b0 + sx * lin + 0.5f * sx * sx * (sq - xq);
          } else if (col <= kFmRank) {
            xv[r * kFmRank + (col - 1)] = sx * v;
          }
        }
      }
      acc = f32x16{};
      x2q2 = f32x2{0.0f, 0.0f};
      kb = 0;
      t += tstride;
    }
    return true;
  };
  uint4 bA[4], bB[4], bC[4];
  issue(bA);
  issue(bB);
  issue(bC);
  for (;;) {
    if (!step(bA)) break;
    issue(bA);
    if (!step(bB)) break;
    issue(bB);
    if (!step(bC)) break;
    issue(bC);
  }
}

/*!
 * F2.  Workgroup = 8 waves over rows [blockIdx.x * rows_per_block, ...) and
 * features [1024 * blockIdx.y, + 1024); wave w takes 128 of them.  Writes
 * part[blockIdx.x][c][n] for c < 17 (Z) and c = 17 (t), n < dim.
 */
__global__ __launch_bounds__(kBwdThreads) void k_fm_bwd(const uint8_t* __restrict__ x,
                                                        int64_t rows, int dim,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ xv,
                                                        int64_t rows_per_block,
                                                        float* __restrict__ part) {
  // G^T [column][row] (columns 17..31 zero) and g, double-buffered: the next
  // tile's G is written while this one is consumed, one barrier per tile
  __shared__ __attribute__((aligned(16))) __bf16 s_gt[2][32][32 + 8];
  __shared__ __attribute__((aligned(16))) float s_g[2][32];
  // each wave's X tile, read back transposed (as in F5: chunk (i, lane) at
  // i * 64 + (lane ^ 8 (i & 1)))
  __shared__ uint4 s_xb[kBwdThreads / kWave][4 * 64];
  const int lane = lane_id();
  const int h = lane >> 5, n = lane & 31;
  const int wave = threadIdx.x / kWave;
  const int fbase = 1024 * blockIdx.y + kBwdWaveFeatures * wave;
  const bool active = fbase < dim;
  for (int i = threadIdx.x; i < 2 * 32 * 40; i += kBwdThreads) {
    (&s_gt[0][0][0])[i] = static_cast<__bf16>(0.0f);
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  // transposed reads of the wave's X image (ds_read_b64_tr_b8, the map of F5)
  const int gr = lane >> 4, qq = (lane & 15) >> 1, pp = lane & 1;
  const uint32_t xt_base =
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&s_xb[wave][0])) +
      16u * static_cast<uint32_t>((gr & 1) * 64 + ((8 * (gr >> 1) + qq) ^ (8 * (gr & 1)))) +
      8u * static_cast<uint32_t>(pp);
  f32x16 acc[4] = {};
  f32x2 tacc[4] = {};
  // the next tile's X fragment and G inputs are loaded while this tile computes
  const int grow = threadIdx.x >> 3, gpart = threadIdx.x & 7;  // G producer (threads < 256)
  // loads are issued unconditionally (a clamped row, the value zeroed past
  // the block's rows): every tile issues the same memory ops, so the wait for
  // a load counts only the ops issued after it
  const int64_t rlast = r1 > r0 ? r1 - 1 : rows - 1;  // in the batch for an empty block too
  auto load_g = [&](int64_t t, float* gv, float2* v) {
    const int64_t r = t + grow;
    const bool ok = threadIdx.x < 256 && r < r1;
    const int64_t rc = r < rlast ? r : rlast;
    const float g0 = g[rc];
    const float2 v0 = *reinterpret_cast<const float2*>(xv + rc * kFmRank + 2 * gpart);
    *gv = ok ? g0 : 0.0f;
    *v = ok ? v0 : make_float2(0.0f, 0.0f);
  };
  auto load_x = [&](int64_t t, uint4 (&w)[4]) {
    const int64_t r = t + n;  // the row of this lane's X fragment
    const bool ok = active && r < r1;
    const int64_t rc = r < rlast ? r : rlast;
    const uint4* q = reinterpret_cast<const uint4*>(x + rc * dim + (active ? fbase : 0) + 64 * h);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 u = q[i];
      w[i] = ok ? u : make_uint4(0, 0, 0, 0);
    }
  };
  auto put_g = [&](int bf, float gv, float2 v) {
    if (threadIdx.x < 256) {
      s_gt[bf][1 + 2 * gpart][grow] = static_cast<__bf16>(gv * v.x);
      s_gt[bf][2 + 2 * gpart][grow] = static_cast<__bf16>(gv * v.y);
      if (gpart == 0) {
        s_gt[bf][0][grow] = static_cast<__bf16>(gv);
        s_g[bf][grow] = gv;
      }
    }
  };
  float gv_n = 0.0f;
  float2 v_n = make_float2(0.0f, 0.0f);
  // X tiles rotate through three register buffers: tile i's fragment is
  // loaded while tiles i - 2 and i - 1 compute, into the buffer tile i - 3
  // just released (no register copies of loads in flight)
  uint4 x0[4], x1[4], x2[4];
  load_g(r0, &gv_n, &v_n);
  load_x(r0, x0);
  load_x(r0 + 32, x1);
  load_x(r0 + 64, x2);
  __syncthreads();  // the zeroed buffers
  put_g(0, gv_n, v_n);
  load_g(r0 + 32, &gv_n, &v_n);
  __syncthreads();
  int cb = 0;
  // one 32-row tile: the next tile's G into the other buffer, this tile's
  // products, then its X buffer takes the tile three ahead.  Tiles past the
  // block's rows (to a multiple of three) see zero X and G: they add nothing
  auto tile = [&](int64_t t0, uint4 (&xw)[4]) {
    put_g(cb ^ 1, gv_n, v_n);  // the next tile's G (its buffer was consumed last tile)
    load_g(t0 + 64, &gv_n, &v_n);
    if (active) {  // wave-uniform (the transposed reads need every lane)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_xb[wave][i * 64 + (lane ^ (8 * (i & 1)))] = xw[i];
      wave_sync();
      // A = G^T rows 16 s + 8 h + j (natural order), B = X rows along K
      bf16x8 ga[2];
      f32x2 g2[2][4];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        ga[s] = *reinterpret_cast<const bf16x8*>(&s_gt[cb][n][16 * s + 8 * h]);
        const float4 ga4 = *reinterpret_cast<const float4*>(&s_g[cb][16 * s + 8 * h]);
        const float4 gb4 = *reinterpret_cast<const float4*>(&s_g[cb][16 * s + 8 * h + 4]);
        g2[s][0] = f32x2{ga4.x, ga4.y};
        g2[s][1] = f32x2{ga4.z, ga4.w};
        g2[s][2] = f32x2{gb4.x, gb4.y};
        g2[s][3] = f32x2{gb4.z, gb4.w};
      }
      typedef __attribute__((address_space(3))) v2i lds_v2i;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint32_t a = xt_base + 2048u * (b & 1) + 512u * (b >> 1) + 256u * s;
          const v2i raw = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(static_cast<uintptr_t>(a)));
          const uint32_t lo = static_cast<uint32_t>(raw.x), hi = static_cast<uint32_t>(raw.y);
          acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[s], fp8x8_bf16(lo, hi), acc[b], 0, 0, 0);
          float f[8];
          fp8x8(lo, hi, f);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const f32x2 x2 = f32x2{f[2 * k], f[2 * k + 1]};
            tacc[b] = __builtin_elementwise_fma(x2 * x2, g2[s][k], tacc[b]);
          }
        }
      }
    }
    load_x(t0 + 96, xw);
    __syncthreads();  // buffer cb consumed; buffer cb ^ 1 written
    cb ^= 1;
  };
  for (int64_t t0 = r0; t0 < r1; t0 += 96) {
    tile(t0, x0);
    tile(t0 + 32, x1);
    tile(t0 + 64, x2);
  }
  if (!active) return;
  float* out = part + static_cast<size_t>(blockIdx.x) * (kFmCols + 1) * dim;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int feat = fbase + 32 * b + n;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int c = (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (c < kFmCols) out[static_cast<size_t>(c) * dim + feat] = acc[b][reg];
    }
    const float t1 = tacc[b][0] + tacc[b][1];
    const float tt = t1 + __shfl_xor(t1, 32, kWave);
    if (h == 0) out[static_cast<size_t>(kFmCols) * dim + feat] = tt;
  }
}

/*!
 * F3.  Z[c][n] = sum over the F2 workgroups of part[b][c][n]: workgroup
 * (64 features, column c), wave w sums blocks w, w + 4, ... (8 loads in flight
 * per lane), LDS combine in a fixed order (deterministic).
 */
constexpr int kRedThreads = 256;
__global__ __launch_bounds__(kRedThreads) void k_fm_reduce(const float* __restrict__ part,
                                                           int nblk, int dim,
                                                           float* __restrict__ z) {
  __shared__ float s[kRedThreads / kWave][kWave];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int n = blockIdx.x * kWave + lane, c = blockIdx.y;
  const size_t stride = static_cast<size_t>(kFmCols + 1) * dim;
  const float* p = part + static_cast<size_t>(c) * dim + n;
  constexpr int kWaves = kRedThreads / kWave;
  float acc = 0.0f;
  if (n < dim) {
    int b = w;
    for (; b + 7 * kWaves < nblk; b += 8 * kWaves) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[static_cast<size_t>(b + u * kWaves) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < nblk; b += kWaves) acc += p[static_cast<size_t>(b) * stride];
  }
  s[w][lane] = acc;
  __syncthreads();
  if (w == 0 && n < dim) {
    float t = s[0][lane];
#pragma unroll
    for (int q = 1; q < kWaves; ++q) t += s[q][lane];
    z[static_cast<size_t>(c) * dim + n] = t;
  }
}

/*! \brief F4.  dw = s Z_0, dV_nf = s Z_{1+f,n} - V_nf s^2 t_n (t = Z_17) */
__global__ __launch_bounds__(kWave) void k_fm_grads(const float* __restrict__ z, int dim,
                                                    const float* __restrict__ v, float sx,
                                                    float* __restrict__ gw,
                                                    float* __restrict__ gv) {
  const int n = blockIdx.x * kWave + lane_id();
  if (n >= dim) return;
  gw[n] = sx * z[n];
  const float t = sx * sx * z[static_cast<size_t>(kFmCols) * dim + n];
  const float4* vr = reinterpret_cast<const float4*>(v + static_cast<size_t>(n) * kFmRank);
  float4* gr = reinterpret_cast<float4*>(gv + static_cast<size_t>(n) * kFmRank);
#pragma unroll
  for (int q = 0; q < kFmRank / 4; ++q) {
    const float4 a = vr[q];
    const float* zc = z + static_cast<size_t>(1 + 4 * q) * dim + n;
    gr[q] = make_float4(sx * zc[0] - a.x * t, sx * zc[dim] - a.y * t,
                        sx * zc[2 * static_cast<size_t>(dim)] - a.z * t,
                        sx * zc[3 * static_cast<size_t>(dim)] - a.w * t);
  }
}

/*! \brief F0: [w | V]^T as bf16 [kFmCols][dim] and q = rowsum(V^2) (f32) */
__global__ __launch_bounds__(256) void k_fm_prep(const float* __restrict__ w,
                                                 const float* __restrict__ v, int dim,
                                                 __bf16* __restrict__ wt, float* __restrict__ q) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= dim) return;
  wt[k] = static_cast<__bf16>(w[k]);
  const float4* vr = reinterpret_cast<const float4*>(v + static_cast<size_t>(k) * kFmRank);
  float acc = 0.0f;
#pragma unroll
  for (int j = 0; j < kFmRank / 4; ++j) {
    const float4 a = vr[j];
    wt[static_cast<size_t>(1 + 4 * j) * dim + k] = static_cast<__bf16>(a.x);
    wt[static_cast<size_t>(2 + 4 * j) * dim + k] = static_cast<__bf16>(a.y);
    wt[static_cast<size_t>(3 + 4 * j) * dim + k] = static_cast<__bf16>(a.z);
    wt[static_cast<size_t>(4 + 4 * j) * dim + k] = static_cast<__bf16>(a.w);
    acc += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
  }
  q[k] = acc;
}

/*!
 * F5.  The whole step over one read of the batch.  Workgroup = W = dim / 128
 * waves over rows [blockIdx.x * rows_per_block, ...); wave w owns features
 * [128 w, 128 w + 128) for both halves of the step.  Per 32-row tile, with
 * the tile's X fragment (F1's and F2's lane layout are the same: lane (col, h)
 * holds 64 bytes of row col) loaded once:
 *   P1  G^T X of the tile two back (its X image kept in LDS and read back
 *       transposed by ds_read_b64_tr_b8, rows along K, so F2's identity
 *       MFMA and its f32 -> bf16 repacking are gone; G^T from s_gt / s_g),
 *       then this tile's x.[w | V] block products (F1, [w | V] in LDS) and
 *       x^2.q; the 32 x 18 partial sums go to s_part.
 *                                                          barrier
 *   P2  16 threads per row sum the W partials of its 18 columns, form y, the
 *       loss and g, and write G^T = [g, g sx xV] (bf16) and g.
 * Partials, G^T and X are double-buffered by tile parity, so one barrier per
 * tile orders everything (the loop's comment); the next tile's X is loaded
 * one tile ahead.
 * Loss partials and dbias partials (sum g) per workgroup go to lpart.
 */
/*! \brief ds_swizzle in bit mode: lane ^ xor_mask within 32 (no address VGPR) */
template <int kXor>
__device__ __forceinline__ float swz_xor(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (kXor << 10) | 0x1F));
}
/*! \brief lane (lane & ~15) + kLane of the lane's 16-lane group */
template <int kLane>
__device__ __forceinline__ float swz_group(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x10 | (kLane << 5)));
}

template <int W>
__global__ __launch_bounds__(64 * W) void k_fm_fused(
    const uint8_t* __restrict__ x, int64_t rows, const __bf16* __restrict__ wt,
    const float* __restrict__ q, const float* __restrict__ bias, float sx,
    const float* __restrict__ label, const float* __restrict__ weight, int loss, float inv_n,
    int64_t rows_per_block, float* __restrict__ y, float* __restrict__ part,
    float* __restrict__ lpart) {
  // every shape is compile-time (dim = 128 W), so each LDS access is one base
  // register + an immediate offset: no per-address registers to keep live
  constexpr int D = 128 * W;
  constexpr int kLdw = D + 8;
  constexpr int P = W + 1;  // odd stride of the partials: conflict-free column writes
  constexpr int kThreads = 64 * W;
  // F1's [17][D + 8] plus one zero row, the B row of lanes 17..31
  __shared__ __attribute__((aligned(16))) __bf16 s_wt[(kFmCols + 1) * kLdw];
  __shared__ __attribute__((aligned(16))) float s_q[D];
  // double-buffered by tile parity: one barrier per tile (see the loop)
  __shared__ float s_part[2][32 * 18 * P];                             // [row][column][wave]
  __shared__ __attribute__((aligned(16))) __bf16 s_gt[2][32 * 40];     // G^T [column][row]
  __shared__ __attribute__((aligned(16))) float s_g[2][32];
  // each wave's X fragment of a tile, kept two tiles for its backward:
  // 16-byte chunk (wave, i, lane) at (wave * 4 + i) * 64 + (lane ^ 8 (i & 1))
  // (the swizzle keeps the backward's transposed reads conflict-free)
  __shared__ uint4 s_x[2][W * 4 * 64];
  __shared__ float s_red[2 * W];
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  const int wave = tid / kWave;
  for (int i = tid; i < kFmCols * D / 8; i += kThreads) {
    const int c = i / (D / 8), k8 = i % (D / 8);
    *reinterpret_cast<uint4*>(s_wt + c * kLdw + 8 * k8) =
        reinterpret_cast<const uint4*>(wt + static_cast<size_t>(c) * D)[k8];
  }
  for (int i = tid; i < kLdw / 8; i += kThreads) {
    reinterpret_cast<uint4*>(s_wt + kFmCols * kLdw)[i] = make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < D / 4; i += kThreads) {
    reinterpret_cast<float4*>(s_q)[i] = reinterpret_cast<const float4*>(q)[i];
  }
  for (int i = tid; i < 2 * 32 * 40; i += kThreads) (&s_gt[0][0])[i] = static_cast<__bf16>(0.0f);
  // zero X and G images: the backward runs from the first tile on (tiles -2
  // and -1 add 0 x 0), so no branch splits the accumulators' live ranges
  for (int i = tid; i < 2 * W * 4 * 64; i += kThreads) (&s_x[0][0])[i] = make_uint4(0, 0, 0, 0);
  if (tid < 64) (&s_g[0][0])[tid] = 0.0f;
  const int kbase = 128 * wave + 64 * h;
  // this lane's B row of [w | V] (lanes 17..31: the zero row)
  const __bf16* const wrow = s_wt + (col < kFmCols ? col : kFmCols) * kLdw + kbase;
  // F2's transposed X reads (ds_read_b64_tr_b8): in each 16-lane group gr,
  // lane 2 qq + pp supplies row 8 (gr >> 1) + qq (+ 16 s) and bytes 8 pp ..
  // 8 pp + 7 of the group's 16 features 16 (gr & 1) (+ 32 b); lane i of the
  // group receives feature i of those 8 rows, row qq in byte qq
  // (tools/tr8_probe.hip checks this map).  The chunk of (row, 16 features)
  // follows s_x's swizzle; (bf, b, s) add compile-time offsets
  const int gr = lane >> 4, qq = (lane & 15) >> 1, pp = lane & 1;
  const uint32_t xt_base =
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&s_x[0][0])) +
      16u * static_cast<uint32_t>((wave * 4 + (gr & 1)) * 64 +
                                  ((8 * (gr >> 1) + qq) ^ (8 * (gr & 1)))) +
      8u * static_cast<uint32_t>(pp);
  const float b0 = *bias;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  // the clamp row of the unconditional loads: inside the batch even for a
  // block that starts at or past the last row (rows_per_block is rounded up to
  // 32, so trailing blocks can be empty); such a block loads row rows - 1,
  // zeroes it and writes zero partials
  const int64_t rlast = r1 > r0 ? r1 - 1 : rows - 1;
  // rows past the block's end load the clamp row (finite codes): their g is
  // zero, so they add nothing to the backward, and P2 stores nothing for them
  auto load_x = [&](int64_t t, uint4 (&v)[4]) {
    const int64_t r = t + col;
    const int64_t rc = r < rlast ? r : rlast;
    const uint4* p = reinterpret_cast<const uint4*>(x + rc * D + kbase);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = p[i];
  };
  // labels / weights of a tile: lane l holds row (l & 31), loaded a tile ahead
  auto load_lw = [&](int64_t t, float* lab, float* wgt) {
    const int64_t r = t + col;
    const int64_t rc = r < rlast ? r : rlast;
    const float l = label[rc];
    const float w = weight != nullptr ? weight[rc] : 1.0f;
    *lab = l;
    *wgt = w;
  };
  f32x16 acc[4] = {};
  f32x2 tacc[4] = {};
  float lsum = 0.0f, gsum = 0.0f;
  // F2 on the tile of parity bf: B = X with rows along K straight from the
  // LDS image by transposed reads (element j: row 16 s + 8 h + j of feature
  // 128 wave + 32 b + col), A = G^T from s_gt in the same natural row order;
  // t = (x^2)^T g accumulates from the same bytes
  auto backward = [&](int bf) {
    bf16x8 ga[2];
    f32x2 g2[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      ga[s] = *reinterpret_cast<const bf16x8*>(s_gt[bf] + col * 40 + 16 * s + 8 * h);
      const float4 ga4 = *reinterpret_cast<const float4*>(s_g[bf] + 16 * s + 8 * h);
      const float4 gb4 = *reinterpret_cast<const float4*>(s_g[bf] + 16 * s + 8 * h + 4);
      g2[s][0] = f32x2{ga4.x, ga4.y};
      g2[s][1] = f32x2{ga4.z, ga4.w};
      g2[s][2] = f32x2{gb4.x, gb4.y};
      g2[s][3] = f32x2{gb4.z, gb4.w};
    }
    typedef __attribute__((address_space(3))) v2i lds_v2i;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t a = xt_base + static_cast<uint32_t>(bf) * (W * 4 * 64 * 16) +
                           2048u * (b & 1) + 512u * (b >> 1) + 256u * s;
        const v2i raw = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(static_cast<uintptr_t>(a)));
        const uint32_t lo = static_cast<uint32_t>(raw.x), hi = static_cast<uint32_t>(raw.y);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[s], fp8x8_bf16(lo, hi), acc[b], 0, 0, 0);
        float f[8];
        fp8x8(lo, hi, f);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 x2 = f32x2{f[2 * k], f[2 * k + 1]};
          tacc[b] = __builtin_elementwise_fma(x2 * x2, g2[s][k], tacc[b]);
        }
      }
    }
  };
  float lab_n = 0.0f, wgt_n = 1.0f;
  load_lw(r0, &lab_n, &wgt_n);
  __syncthreads();  // s_wt, s_q, s_gt, s_g
  // Tile j (parity bf = j & 1):
  //   backward of tile j - 2 (its X in s_x[bf], its G^T in s_gt[bf]: written
  //   by P2(j - 2), which every thread finished before barrier j - 1);
  //   X(j) from registers into s_x[bf], X(j + 1) in flight; forward of j ->
  //   s_part[bf];  barrier j;  P2(j): s_part[bf] -> s_gt[bf], s_g[bf].
  // s_part[bf] is next written by forward(j + 2), after barrier j + 1, which
  // every thread reaches only after its P2(j): one barrier per tile, and a
  // wave done with P2 runs on into the next tile's products
  // one tile: X(t0) in xc, X(t0 + 32) loaded into xn.  The loop runs two
  // tiles per trip with the register sets swapped (no copy of the prefetch);
  // a block of an odd number of tiles ends on one of rows past r1 (g = 0)
  auto step = [&](int64_t t0, int j, const uint4 (&xc)[4], uint4 (&xn)[4]) {
    const int bf = j & 1;
    const float lab_t = lab_n, wgt_t = wgt_n;
    load_lw(t0 + 32, &lab_n, &wgt_n);
    backward(bf);
#pragma unroll
    for (int i = 0; i < 4; ++i) s_x[bf][(wave * 4 + i) * 64 + (lane ^ (8 * (i & 1)))] = xc[i];
    load_x(t0 + 32, xn);
    __builtin_amdgcn_sched_barrier(0);
    f32x16 fa = {};
    f32x2 x2q2 = {0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t lo = word(xc, 2 * i), hi = word(xc, 2 * i + 1);
      float f[8];
      fp8x8(lo, hi, f);
      const float4 q0 = *reinterpret_cast<const float4*>(s_q + kbase + 8 * i);
      const float4 q1 = *reinterpret_cast<const float4*>(s_q + kbase + 8 * i + 4);
      f32x2 sq[4] = {{f[0], f[1]}, {f[2], f[3]}, {f[4], f[5]}, {f[6], f[7]}};
      const f32x2 qq[4] = {{q0.x, q0.y}, {q0.z, q0.w}, {q1.x, q1.y}, {q1.z, q1.w}};
#pragma unroll
      for (int k = 0; k < 4; ++k) x2q2 = __builtin_elementwise_fma(sq[k] * sq[k], qq[k], x2q2);
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(wrow + 8 * i);
      fa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fp8x8_bf16(lo, hi), b, fa, 0, 0, 0);
    }
    float x2q = x2q2[0] + x2q2[1];
    x2q += __shfl_xor(x2q, 32, kWave);
    float* const sp = s_part[bf];
    if (col < kFmCols) {
      float* pw = sp + (4 * h * 18 + col) * P + wave;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        // accumulator row m = (reg & 3) + 8 (reg >> 2) + 4 h (C/D map)
        pw[((reg & 3) + 8 * (reg >> 2)) * 18 * P] = fa[reg];
      }
    }
    if (h == 0) sp[(col * 18 + 17) * P + wave] = x2q;
    __syncthreads();
    // ---- P2: 16 threads per row; row rr = tid / 16 (+ 4 W per pass)
    const int k = tid & 15;
#pragma unroll
    for (int pass = 0; pass < 32 / (4 * W); ++pass) {
      const int rr = (tid >> 4) + pass * 4 * W;
      const float* p0 = sp + (rr * 18 + k) * P;
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int w2 = 0; w2 < W; ++w2) s0 += p0[w2];
      if (k < 2) {
#pragma unroll
        for (int w2 = 0; w2 < W; ++w2) s1 += p0[16 * P + w2];
      }
      // lane k: column k (0 = x.w, 1..15 = xV_1..15); lane 0 also column 16
      // (xV_16), lane 1 column 17 (x^2.q)
      float sq = (k >= 1 ? s0 * s0 : 0.0f) + (k == 0 ? s1 * s1 : 0.0f);
      sq += swz_xor<1>(sq);
      sq += swz_xor<2>(sq);
      sq += swz_xor<4>(sq);
      sq += swz_xor<8>(sq);
      const float lin = swz_group<0>(s0);
      const float xq = swz_group<1>(s1);
      const float yv = b0 + sx * lin + 0.5f * sx * sx * (sq - xq);
      const int64_t row = t0 + rr;
      const bool valid = row < r1;
      const float lab = __shfl(lab_t, rr, kWave);
      const float wg = __shfl(wgt_t, rr, kWave);
      float l, g;
      if (loss == kFmSquared) {
        const float d = yv - lab;
        l = d * d;
        g = 2.0f * d;
      } else {
        // e in (0, 1]: log(1 + e) and 1 / (1 + e) by the hardware
        // log / reciprocal (1 ulp; no libm range reduction needed)
        const float e = __expf(-fabsf(yv));
        const float ope = 1.0f + e;
        l = fmaxf(yv, 0.0f) - yv * lab + __logf(ope);
        const float rc = __builtin_amdgcn_rcpf(ope);
        const float sig = yv >= 0.0f ? rc : e * rc;
        g = sig - lab;
      }
      g = valid ? g * wg * inv_n : 0.0f;
      s_gt[bf][k * 40 + rr] = static_cast<__bf16>(k == 0 ? g : g * sx * s0);
      if (k == 0) {
        s_gt[bf][16 * 40 + rr] = static_cast<__bf16>(g * sx * s1);
        s_g[bf][rr] = g;
        if (valid) {
          lsum += wg * l;
          gsum += g;
          if (y != nullptr) y[row] = yv;
        }
      }
    }
  };
  uint4 xa[4], xb[4];
  load_x(r0, xa);
  int j = 0;
  for (int64_t t0 = r0; t0 < r1; t0 += 64, j += 2) {
    step(t0, j, xa, xb);
    step(t0 + 32, j + 1, xb, xa);
  }
  // the last two tiles' backward, after every thread's last P2
  __syncthreads();
  backward(0);
  backward(1);
  // ---- partials
  float* out = part + static_cast<size_t>(blockIdx.x) * (kFmCols + 1) * D;
  const int fbase = 128 * wave;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int feat = fbase + 32 * b + col;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int c = (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (c < kFmCols) out[static_cast<size_t>(c) * D + feat] = acc[b][reg];
    }
    const float t1 = tacc[b][0] + tacc[b][1];
    const float tt = t1 + __shfl_xor(t1, 32, kWave);
    if (h == 0) out[static_cast<size_t>(kFmCols) * D + feat] = tt;
  }
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    lsum += __shfl_xor(lsum, d, kWave);
    gsum += __shfl_xor(gsum, d, kWave);
  }
  if (lane == 0) {
    s_red[2 * wave] = lsum;
    s_red[2 * wave + 1] = gsum;
  }
  __syncthreads();
  if (tid == 0) {
    float a = 0.0f, c = 0.0f;
#pragma unroll
    for (int w2 = 0; w2 < W; ++w2) {
      a += s_red[2 * w2];
      c += s_red[2 * w2 + 1];
    }
    lpart[2 * blockIdx.x] = a;
    lpart[2 * blockIdx.x + 1] = c;
  }
}

}  // namespace

void LaunchFmPrep(const float* w, const float* v, int dim, void* wt_bf16, float* q,
                  hipStream_t stream) {
  if (dim == 0) return;
  hipLaunchKernelGGL(k_fm_prep, dim3((dim + 255) / 256), dim3(256), 0, stream, w, v, dim,
                     static_cast<__bf16*>(wt_bf16), q);
}

void LaunchFmReduceGrads(const float* part, int nblocks, int dim, const float* v, float sx,
                         float* z, float* gw, float* gv, hipStream_t stream) {
  if (dim == 0) return;
  const int fb = (dim + kWave - 1) / kWave;
  hipLaunchKernelGGL(k_fm_reduce, dim3(fb, kFmCols + 1), dim3(kRedThreads), 0, stream, part,
                     nblocks, dim, z);
  hipLaunchKernelGGL(k_fm_grads, dim3(fb), dim3(kWave), 0, stream, z, dim, v, sx, gw, gv);
}

size_t FmForwardSharedBytes(int dim) {
  return static_cast<size_t>(kFmCols) * (dim + 8) * sizeof(__bf16) + static_cast<size_t>(dim) * 4;
}

void LaunchFmForward(const uint8_t* x, int64_t rows, int dim, const void* wt_bf16, const float* q,
                     const float* bias, float sx, float* y, float* xv, int num_cus,
                     hipStream_t stream) {
  if (rows == 0) return;
  const int64_t ntiles = (rows + 31) / 32;
  const int64_t want = (ntiles + kFwdThreads / kWave - 1) / (kFwdThreads / kWave);
  const int64_t cap = static_cast<int64_t>(num_cus) * 4;  // persistent: LDS [w | V] loaded once per CU slot
  const int grid = static_cast<int>(want < cap ? want : cap);
  hipLaunchKernelGGL(k_fm_fwd, dim3(grid), dim3(kFwdThreads), FmForwardSharedBytes(dim), stream, x,
                     rows, dim, reinterpret_cast<const __bf16*>(wt_bf16), q, bias, sx, y, xv);
}


void LaunchFmFused(const uint8_t* x, int64_t rows, int dim, const void* wt_bf16, const float* q,
                   const float* bias, float sx, const float* label, const float* weight,
                   int loss, float inv_n, int nblocks, float* y, float* part, float* lpart,
                   hipStream_t stream) {
  if (nblocks == 0) return;
  CHECK_GT(rows, 0) << "fused HashedFM step: empty batch";
  const int64_t per = (((rows + nblocks - 1) / nblocks) + 31) / 32 * 32;
  const int w = dim / 128;
  auto kernel = w == 8 ? k_fm_fused<8> : w == 4 ? k_fm_fused<4> : w == 2 ? k_fm_fused<2>
                                                                         : k_fm_fused<1>;
  CHECK(dim % 128 == 0 && (w == 1 || w == 2 || w == 4 || w == 8))
      << "fused HashedFM step: dim must be 128, 256, 512 or 1024 (got " << dim << ")";
  hipLaunchKernelGGL(kernel, dim3(nblocks), dim3(64 * w), 0, stream, x, rows,
                     reinterpret_cast<const __bf16*>(wt_bf16), q, bias, sx, label, weight, loss,
                     inv_n, per, y, part, lpart);
}

void LaunchFmBackward(const uint8_t* x, int64_t rows, int dim, const float* g, const float* xv,
                      int nblocks, float* part, hipStream_t stream) {
  if (rows == 0 || nblocks == 0) return;
  const int64_t per = (((rows + nblocks - 1) / nblocks) + 31) / 32 * 32;
  hipLaunchKernelGGL(k_fm_bwd, dim3(nblocks, (dim + 1023) / 1024), dim3(kBwdThreads), 0, stream, x,
                     rows, dim, g, xv, per, part);
}

}  // namespace gpu
}  // namespace dmlc
