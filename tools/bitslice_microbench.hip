// bitslice_microbench.hip -- measures bitsliced AES-128 on the VALU of one
// MI355X (no LDS), the alternative to the T-table kernels' LDS bound
// (DESIGN.md section 8).  Each thread holds 32 blocks as 128 bit planes.
//   --cpu-check : S-box vs FIPS-197 for all 256 inputs, encryption vs the
//                 T-table reference (aes_core.h) and the FIPS-197 C.1 vector.
//   (default)   : GPU check against the host, then timing of
//                 mode 0: encryptions on resident planes (the cost inside a
//                         bitsliced tree expansion, where seeds stay sliced);
//                 mode 1: transpose in + encryption + transpose out per block.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bitslice_microbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../distributed_point_functions_amd/csrc/kernels/aes_core.h"
#include "bitslice_aes.h"

struct Keys {
  uint32_t rk[44];
};

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__host__ __device__ inline uint32_t mix32h(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

#if defined(BS_WAVES)
#define BS_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(BS_WAVES, BS_WAVES)))
#else
#define BS_WAVES_ATTR
#endif
template <int MODE>
__global__ __launch_bounds__(256) BS_WAVES_ATTR void bs_kernel(Keys kk, const uint32_t* rkg, int iters,
                                                 uint32_t* out, int full) {
  (void)kk;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t blk[128], s[128];
#pragma unroll
  for (int i = 0; i < 128; ++i) blk[i] = mix32(gid * 128u + i);
  bs::to_planes(blk, s);
  for (int it = 0; it < iters; ++it) {
    // Round keys re-read (scalar loads) every iteration: left loop-invariant,
    // the compiler hoists all 1280 key masks and spills them.
    asm volatile("" ::: "memory");
    Keys k;
#pragma unroll
    for (int i = 0; i < 44; ++i) k.rk[i] = rkg[i];
    if (MODE == 1 && it) bs::to_planes(blk, s);
#if defined(BS_LOWREG)
    bs::encrypt_lowreg(s, k.rk);
#elif defined(BS_LOOP1)
    bs::encrypt_loop1(s, k.rk);
#elif defined(BS_LOOP2)
    bs::encrypt_loop2(s, k.rk);
#elif defined(BS_INPLACE)
    bs::encrypt_inplace(s, k.rk);
#else
    bs::encrypt(s, k.rk);
#endif
    if (MODE == 1) bs::from_planes(s, blk);
  }
  if (MODE == 0) bs::from_planes(s, blk);
  if (full) {
#pragma unroll
    for (int i = 0; i < 128; ++i) out[(size_t)gid * 128 + i] = blk[i];
  } else {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 128; ++i) acc ^= blk[i];
    out[gid] = acc;
  }
}

static void host_blocks(uint32_t gid, uint32_t* blk) {
  for (int i = 0; i < 128; ++i) blk[i] = mix32h(gid * 128u + i);
}

static int cpu_check() {
  int bad = 0;
  // S-box, 8 batches of 32 inputs.
  for (int batch = 0; batch < 8; ++batch) {
    uint32_t x[8] = {0};
    for (int b = 0; b < 32; ++b)
      for (int i = 0; i < 8; ++i) x[i] |= (uint32_t)(((32 * batch + b) >> i) & 1) << b;
    bs::sbox(x);
    for (int b = 0; b < 32; ++b) {
      int v = 0;
      for (int i = 0; i < 8; ++i) v |= ((x[i] >> b) & 1) << i;
      if (v != dpf_aes::kSbox[32 * batch + b]) ++bad;
    }
  }
  printf("sbox mismatches: %d\n", bad);
  // Transpose round trip and definition.
  uint32_t blk[128], s[128], back[128];
  host_blocks(7, blk);
  bs::to_planes(blk, s);
  for (int c = 0; c < 4; ++c)
    for (int k = 0; k < 32; ++k)
      for (int b = 0; b < 32; ++b)
        if (((s[32 * c + k] >> b) & 1) != ((blk[4 * b + c] >> k) & 1)) { ++bad; goto tdone; }
tdone:
  bs::from_planes(s, back);
  if (memcmp(back, blk, sizeof blk)) ++bad;
  printf("after transpose checks: %d\n", bad);
  // Encryption vs the T-table reference.
  const uint8_t key[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  uint32_t rk[44];
  dpf_aes::expand_key(key, rk);
  dpf_aes::HostLookup lk;
  for (int g = 0; g < 4; ++g) {
    host_blocks(g, blk);
    bs::to_planes(blk, s);
    bs::encrypt(s, rk);
    bs::from_planes(s, back);
    {
      uint32_t s2[128], back2[128];
      bs::to_planes(blk, s2);
      bs::encrypt_inplace(s2, rk);
      bs::from_planes(s2, back2);
      if (memcmp(back, back2, sizeof back)) ++bad;
      bs::to_planes(blk, s2);
      bs::encrypt_loop2(s2, rk);
      bs::from_planes(s2, back2);
      if (memcmp(back, back2, sizeof back)) ++bad;
      bs::to_planes(blk, s2);
      bs::encrypt_loop1(s2, rk);
      bs::from_planes(s2, back2);
      if (memcmp(back, back2, sizeof back)) ++bad;
      bs::to_planes(blk, s2);
      bs::encrypt_lowreg(s2, rk);
      bs::from_planes(s2, back2);
      if (memcmp(back, back2, sizeof back)) ++bad;
    }
    for (int b = 0; b < 32; ++b) {
      dpf_aes::Block4 in{blk[4 * b], blk[4 * b + 1], blk[4 * b + 2], blk[4 * b + 3]};
      dpf_aes::Block4 o = dpf_aes::encrypt(in, lk, dpf_aes::ArrayRK{rk});
      if (o.w0 != back[4 * b] || o.w1 != back[4 * b + 1] || o.w2 != back[4 * b + 2] ||
          o.w3 != back[4 * b + 3])
        ++bad;
    }
  }
  // FIPS-197 C.1: 00112233..ff under 000102..0f -> 69c4e0d86a7b0430d8cdb78070b4c55a.
  const uint8_t pt[16] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77,
                          0x88, 0x99, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff};
  const uint8_t ct[16] = {0x69, 0xc4, 0xe0, 0xd8, 0x6a, 0x7b, 0x04, 0x30,
                          0xd8, 0xcd, 0xb7, 0x80, 0x70, 0xb4, 0xc5, 0x5a};
  memset(blk, 0, sizeof blk);
  memcpy(blk, pt, 16);
  bs::to_planes(blk, s);
  bs::encrypt(s, rk);
  bs::from_planes(s, back);
  if (memcmp(back, ct, 16)) ++bad;
  printf("total mismatches: %d\n", bad);
  return bad ? 1 : 0;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "--cpu-check")) return cpu_check();
  if (cpu_check()) return 1;
  Keys k;
  const uint8_t key[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  dpf_aes::expand_key(key, k.rk);
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // GPU correctness: 256 threads x 32 blocks, one encryption, all outputs.
  const int vt = 256;
  uint32_t* d;
  uint32_t* drk;
  CK(hipMalloc(&drk, sizeof k.rk));
  CK(hipMemcpy(drk, k.rk, sizeof k.rk, hipMemcpyHostToDevice));
  CK(hipMalloc(&d, (size_t)vt * 128 * 4));
  bs_kernel<0><<<1, vt>>>(k, drk, 1, d, 1);
  CK(hipGetLastError());
  std::vector<uint32_t> h((size_t)vt * 128);
  CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
  dpf_aes::HostLookup lk;
  int bad = 0;
  for (int g = 0; g < vt; ++g) {
    uint32_t blk[128];
    host_blocks(g, blk);
    for (int b = 0; b < 32; ++b) {
      dpf_aes::Block4 in{blk[4 * b], blk[4 * b + 1], blk[4 * b + 2], blk[4 * b + 3]};
      dpf_aes::Block4 o = dpf_aes::encrypt(in, lk, dpf_aes::ArrayRK{k.rk});
      const uint32_t* got = &h[(size_t)g * 128 + 4 * b];
      if (o.w0 != got[0] || o.w1 != got[1] || o.w2 != got[2] || o.w3 != got[3]) ++bad;
    }
  }
  CK(hipFree(d));
  printf("gpu check: %d mismatching blocks of %d\n", bad, vt * 32);
  if (bad) return 1;
  // Timing: enough threads for several waves per SIMD.
  const int threads = cus * 4 * 64 * 4, block = 256, iters = 16;
  CK(hipMalloc(&d, (size_t)threads * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int mode = 0; mode < 2; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(a));
      if (mode == 0) bs_kernel<0><<<threads / block, block>>>(k, drk, iters, d, 0);
      else bs_kernel<1><<<threads / block, block>>>(k, drk, iters, d, 0);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep && ms < best) best = ms;
    }
    const double blocks = (double)threads * 32 * iters;
    printf("{\"mode\": %d, \"what\": \"%s\", \"ms\": %.3f, \"g_aes_per_s\": %.2f}\n", mode,
           mode == 0 ? "encryptions on resident planes" : "transpose in + encrypt + transpose out",
           best, blocks / best / 1e6);
  }
  return 0;
}
