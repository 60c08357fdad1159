// VALU issue-rate probe for gfx950: per instruction kind, cycles per
// wave64 instruction per SIMD with W resident waves per SIMD, each wave
// running 8 independent chains of the instruction (inline asm, no other
// VALU in the loop).  Times with s_memtime (shader clock) per wave.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o build/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <string>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define R8(F) F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7)

template <int OP>
__global__ __launch_bounds__(256) void k_probe(uint64_t* out, int iters, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
           a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed * 3 + threadIdx.x, c = seed ^ 0x5555u;
  uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3;
  if constexpr (OP == 29 || OP == 31)
    asm volatile("v_cmp_gt_u32 s[20:21], %0, %1" : : "v"(a0), "v"(b) : "s20", "s21");
  if constexpr (OP == 27 || OP == 28 || OP == 30)
    asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a0), "v"(b) : "vcc");
  if constexpr (OP == 24) asm volatile("v_cmp_gt_u32 s[20:21], %0, %1" : : "v"(a0), "v"(b) : "s20", "s21");
  if constexpr (OP == 25) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a0), "v"(b) : "vcc");
  __builtin_amdgcn_s_barrier();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define BODY(I) \
    if constexpr (OP == 0) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 2) \
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 3) asm volatile("v_alignbyte_b32 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 4) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 5) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 6) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 7) asm volatile("v_dot4_u32_u8 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 8) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 9) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 10) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 11) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a##I)); \
    if constexpr (OP == 12) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 13) asm volatile("v_ffbl_b32 %0, %0" : "+v"(a##I)); \
    if constexpr (OP == 14) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 15) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 17) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 18) asm volatile("v_cmp_eq_u32 vcc, %0, %1" : : "v"(a##I), "v"(b) : "vcc"); \
    if constexpr (OP == 19) \
      asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a##I)); \
    if constexpr (OP == 20) asm volatile("v_readlane_b32 s0, %0, 1" : : "v"(a##I) : "s0"); \
    if constexpr (OP == 21) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 22) asm volatile("v_and_b32 %0, 0x7f7f7f7f, %0" : "+v"(a##I)); \
    if constexpr (OP == 23) asm volatile("v_and_b32_e64 %0, %0, %1" : "+v"(a##I) : "v"(b)); \
  if constexpr (OP == 24) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 25) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 26) asm volatile("v_and_b32 %0, 7, %0" : "+v"(a##I)); \
    if constexpr (OP == 27) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 28) \
      asm volatile("v_and_b32 %0, %0, %1\n" \
                   " v_and_b32 %0, %0, %1\n" \
                   " v_and_b32 %0, %0, %1\n" \
                   " v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 29) \
      asm volatile("v_and_b32 %0, %0, %1\n" \
                   " v_and_b32 %0, %0, %1\n" \
                   " v_and_b32 %0, %0, %1\n" \
                   " v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a##I) : "v"(b)); \
    if constexpr (OP == 30) \
      asm volatile("v_cmp_gt_u32 vcc, %0, %1\n" \
                   " v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##I) : "v"(b) : "vcc"); \
    if constexpr (OP == 31) \
      asm volatile("v_cmp_gt_u32 s[20:21], %0, %1\n" \
                   " v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a##I) : "v"(b) : "s20", "s21"); \
    if constexpr (OP == 33) \
      asm volatile("v_mad_u64_u32 v[40:41], s[22:23], %0, %1, v[42:43]\n" \
                   " v_mov_b32 %0, v40" : "+v"(a##I) : "v"(b) : "v40", "v41", "v42", "v43", "s22", "s23"); \
    if constexpr (OP == 34) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a##I) : "v"(b), "v"(c)); \
    if constexpr (OP == 32) \
      asm volatile("v_and_b32 %0, %0, %1\n" \
                   " v_and_b32 %0, %0, %1\n" \
                   " v_and_b32 %0, %0, %1\n" \
                   " v_and_b32 %0, %0, %1" : "+v"(a##I) : "v"(b));
    R8(BODY)
    R8(BODY)
    if constexpr (OP == 16) {
      asm volatile("v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n"
                   "v_lshlrev_b64 %3, 3, %3" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
      asm volatile("v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n"
                   "v_lshlrev_b64 %3, 3, %3" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
      asm volatile("v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n"
                   "v_lshlrev_b64 %3, 3, %3" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
      asm volatile("v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n"
                   "v_lshlrev_b64 %3, 3, %3" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint32_t sink = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(w0 ^ w1 ^ w2 ^ w3);
  if ((threadIdx.x & 63) == 0) {
    const size_t wv = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
    out[2 * wv] = t1 - t0;
    out[2 * wv + 1] = sink == 0x12345678u ? 1 : 0;
  }
}

typedef void (*KernelFn)(uint64_t*, int, uint32_t);
struct Probe { const char* name; KernelFn fn; };

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  Probe probes[] = {
      {"v_and_b32", k_probe<0>}, {"v_add_u32", k_probe<1>}, {"v_bitop3_b32", k_probe<2>},
      {"v_alignbyte_b32", k_probe<3>}, {"v_bcnt_u32_b32", k_probe<4>},
      {"v_mul_lo_u32", k_probe<5>}, {"v_mul_u32_u24", k_probe<6>},
      {"v_dot4_u32_u8", k_probe<7>}, {"v_fma_f32", k_probe<8>}, {"v_perm_b32", k_probe<9>},
      {"v_pk_add_u16", k_probe<10>}, {"v_cvt_f32_u32", k_probe<11>},
      {"v_lshlrev_b32", k_probe<12>}, {"v_ffbl_b32", k_probe<13>},
      {"v_lshl_or_b32", k_probe<14>}, {"v_cndmask_b32", k_probe<15>},
      {"v_lshlrev_b64", k_probe<16>}, {"v_mad_u32_u24", k_probe<17>},
      {"v_cmp_eq_u32", k_probe<18>}, {"v_mov_b32_dpp", k_probe<19>},
      {"v_readlane_b32", k_probe<20>}, {"v_add3_u32", k_probe<21>},
      {"v_and_b32_literal", k_probe<22>}, {"v_and_b32_e64", k_probe<23>},
      {"v_cndmask_e64_sgpr", k_probe<24>}, {"v_cndmask_vcc_set", k_probe<25>},
      {"v_and_b32_inline", k_probe<26>}, {"v_cndmask_e64_vcc", k_probe<27>},
      {"mix3and_cndmask_vcc", k_probe<28>}, {"mix3and_cndmask_sgpr", k_probe<29>},
      {"cmp_vcc_cndmask", k_probe<30>}, {"cmp_sgpr_cndmask", k_probe<31>},
      {"mix4and", k_probe<32>}, {"mad_u64_plus_mov", k_probe<33>}};
  const char* only = argc > 1 ? argv[1] : nullptr;
  const int iters = 4096;
  uint64_t* d;
  const int max_blocks = cus * 8;  // 8 blocks of 4 waves per CU
  CHECK(hipMalloc(&d, sizeof(uint64_t) * 2 * max_blocks * 4));
  std::vector<uint64_t> h(2 * max_blocks * 4);
  printf("{\"cus\": %d, \"iters\": %d, \"instr_per_iter\": 16, \"results\": [\n", cus, iters);
  bool first = true;
  for (const Probe& p : probes) {
    if (only != nullptr &&
        std::string(only).find(std::string(",") + p.name + ",") == std::string::npos) {
      continue;
    }
    for (int wps : {2, 4, 8}) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
      const int blocks = cus * wps;
      hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(256), 0, 0, d, 16, 1u);  // warm
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(256), 0, 0, d, iters, 7u);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      CHECK(hipMemcpy(h.data(), d, sizeof(uint64_t) * 2 * blocks * 4, hipMemcpyDeviceToHost));
      double cyc = 0;
      for (int w = 0; w < blocks * 4; ++w) cyc += static_cast<double>(h[2 * w]);
      cyc /= blocks * 4;
      const double instr = 16.0 * iters;
      // per-wave cycles per instruction; with wps waves sharing a SIMD the
      // SIMD's cost per instruction is that / wps
      const double per_wave = cyc / instr;
      const double total = instr * blocks * 4;
      const double rate = total / (ms * 1e-3) / 1e9;  // G wave-instr / s chip-wide
      printf("%s{\"op\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr_per_wave\": %.3f, "
             "\"simd_cyc_per_instr\": %.3f, \"chip_G_wave_instr_per_s\": %.1f, \"ms\": %.3f}",
             first ? "" : ",\n", p.name, wps, per_wave, per_wave / wps, rate, ms);
      first = false;
    }
  }
  printf("\n]}\n");
  CHECK(hipFree(d));
  return 0;
}
