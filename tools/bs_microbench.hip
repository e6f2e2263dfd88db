// bs_microbench.hip -- throughput of the bitsliced MMO hash of
// tools/bs_aes.h on one MI355X (VALU only, no LDS): 8 blocks per lane,
// normal form in and out (transposes included), key masks from the kernel
// arguments.  Also checks the GPU result against the T-table hash on the host.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bs_microbench.hip -o /tmp/bsmb
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../distributed_point_functions_amd/csrc/kernels/aes_core.h"
#include "bs_aes.h"

#ifndef BS_WAVES
#define BS_WAVES 4
#endif

__host__ __device__ inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

struct KernelMasks {
  uint32_t m[11][32];
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BS_WAVES, BS_WAVES)))
void bs_kernel(KernelMasks km, int iters, uint32_t* out, int full) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t w[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) w[i] = mix32(gid * 32u + i);
  for (int it = 0; it < iters; ++it) bsa::mmo8(w, bsa::ArrayMasks{km.m});
  if (full) {
#pragma unroll
    for (int i = 0; i < 32; ++i) out[(size_t)gid * 32 + i] = w[i];
  } else {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= w[i];
    out[gid] = acc;
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

int main() {
  const uint8_t key[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  uint32_t rk[44];
  dpf_aes::expand_key(key, rk);
  const bsa::BsKeyMasks hm = bsa::make_key_masks(rk);
  KernelMasks km;
  memcpy(km.m, hm.m, sizeof km.m);
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // Correctness: 256 threads x 8 blocks, one hash, all outputs.
  const int vt = 256;
  uint32_t* d;
  CK(hipMalloc(&d, (size_t)vt * 32 * 4));
  bs_kernel<<<1, vt>>>(km, 1, d, 1);
  CK(hipGetLastError());
  std::vector<uint32_t> h((size_t)vt * 32);
  CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
  dpf_aes::HostLookup lk;
  int bad = 0;
  for (int g = 0; g < vt; ++g)
    for (int b = 0; b < 8; ++b) {
      dpf_aes::Block4 x{mix32(g * 32u + 4 * b), mix32(g * 32u + 4 * b + 1),
                        mix32(g * 32u + 4 * b + 2), mix32(g * 32u + 4 * b + 3)};
      dpf_aes::Block4 o = dpf_aes::mmo_hash(x, lk, dpf_aes::ArrayRK{rk});
      const uint32_t* got = &h[(size_t)g * 32 + 4 * b];
      if (o.w0 != got[0] || o.w1 != got[1] || o.w2 != got[2] || o.w3 != got[3]) ++bad;
    }
  CK(hipFree(d));
  printf("gpu check: %d mismatching blocks of %d\n", bad, vt * 8);
  if (bad) return 1;
  const int block = 256, iters = 32;
  const int threads = cus * 4 * 64 * BS_WAVES * 2;  // two waves' worth of work per slot
  CK(hipMalloc(&d, (size_t)threads * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    bs_kernel<<<threads / block, block>>>(km, iters, d, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep && ms < best) best = ms;
  }
  const double blocks = (double)threads * 8 * iters;
  printf("{\"waves_per_simd\": %d, \"ms\": %.3f, \"g_aes_per_s\": %.2f}\n", BS_WAVES, best,
         blocks / best / 1e6);
  return 0;
}
