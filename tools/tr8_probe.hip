// Probe of gfx950's ds_read_b64_tr_b8 lane mapping: every lane supplies an
// 8-byte-aligned LDS address, every lane receives 8 bytes; the host decodes
// which source byte landed where and checks the mapping the HashedFM kernel
// relies on: within each 16-lane group, lane 2q + p supplies row q
// (bytes 8p .. 8p + 7 of a 16-column block) and lane i receives byte
// (i & 7) of the row pieces of lanes 2q + (i >> 3), row q in byte q.
// Build: hipcc --offload-arch=gfx950 -O2 tools/tr8_probe.hip -o build/tr8_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v2i __attribute__((ext_vector_type(2)));

__global__ void k_probe(const int* addr, int hi, v2i* out) {
  __shared__ __attribute__((aligned(16))) unsigned char s[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) s[i] = hi ? (i >> 8) : (i & 255);
  __syncthreads();
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  out[threadIdx.x] = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(s + addr[threadIdx.x]));
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  int* d_addr;
  v2i* d_out;
  CK(hipMalloc(&d_addr, 64 * sizeof(int)));
  CK(hipMalloc(&d_out, 64 * sizeof(v2i)));
  int bad_total = 0;
  for (int test = 0; test < 3; ++test) {
    std::vector<int> addr(64);
    srand(7 + test);
    std::vector<int> perm(512);
    for (int i = 0; i < 512; ++i) perm[i] = i;
    for (int i = 511; i > 0; --i) std::swap(perm[i], perm[rand() % (i + 1)]);
    for (int l = 0; l < 64; ++l) addr[l] = test == 0 ? 8 * l : (test == 1 ? 8 * (63 - l) : 8 * perm[l]);
    CK(hipMemcpy(d_addr, addr.data(), 64 * sizeof(int), hipMemcpyHostToDevice));
    std::vector<v2i> lo(64), hi(64);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d_addr, 0, d_out);
    CK(hipMemcpy(lo.data(), d_out, 64 * sizeof(v2i), hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d_addr, 1, d_out);
    CK(hipMemcpy(hi.data(), d_out, 64 * sizeof(v2i), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
      const unsigned char* bl = reinterpret_cast<const unsigned char*>(&lo[l]);
      const unsigned char* bh = reinterpret_cast<const unsigned char*>(&hi[l]);
      const int g = l / 16, i = l % 16;
      if (test == 0) {
        std::printf("lane %2d:", l);
        for (int b = 0; b < 8; ++b) std::printf(" %4d", bl[b] | (bh[b] << 8));
        std::printf("\n");
      }
      for (int q = 0; q < 8; ++q) {
        const int want = addr[16 * g + 2 * q + (i >> 3)] + (i & 7);
        const int got = bl[q] | (bh[q] << 8);
        if (want != got) ++bad;
      }
    }
    std::printf("test %d: %d of 512 bytes differ from the assumed mapping\n", test, bad);
    bad_total += bad;
  }
  std::printf("tr8 mapping %s\n", bad_total == 0 ? "CONFIRMED" : "DIFFERS");
  return 0;
}
