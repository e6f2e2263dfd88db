// fbs_microbench.hip -- throughput of the full-bitslice MMO hash of
// tools/fbs_aes.h (32 blocks per lane, 128 bit planes in VGPRs, ShiftRows by
// renaming) on one MI355X.  Each lane hashes its 32 blocks `iters` times in a
// chain (x <- H(x)), planes in and out (no transposes: the whole-DFS design
// keeps seeds in plane form and transposes only at leaf stores).
//
// Variants (FBS_MODE):
//   0  rounds rolled (one round per loop trip, MixColumns writes back to the
//      canonical phase), round-key masks as LDS broadcasts;
//   1  four rounds per loop trip (the ShiftRows phase cycles 0..3 inside the
//      body, no moves), round-key masks as LDS broadcasts;
//   2  all ten rounds unrolled, round keys folded into the truth tables.
// FBS_FF_LDS = planes of the feed-forward sigma(x) kept in LDS (per wave,
// [plane][lane]); the rest stay in VGPRs.
// FBS_WAVES = waves per SIMD (256-thread workgroups, 1 wave per SIMD each).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DFBS_MODE=1 tools/fbs_microbench.hip -o tools/fbsm_1
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../distributed_point_functions_amd/csrc/kernels/aes_core.h"
#include "fbs_aes.h"

#ifndef FBS_MODE
#define FBS_MODE 1
#endif
#ifndef FBS_FF_LDS
#define FBS_FF_LDS 72
#endif
#ifndef FBS_WAVES
#define FBS_WAVES 2
#endif
// FBS_FF_GLB = planes of the feed-forward kept in a per-wave global buffer
// (after the LDS ones); the rest stay in VGPRs.
#ifndef FBS_FF_GLB
#define FBS_FF_GLB 0
#endif
// FBS_NO_FF=1: drop the MMO feed-forward (x <- AES(sigma(x))): the engine's
// compute ceiling without the 128 planes of sigma(x) to keep.
#ifndef FBS_NO_FF
#define FBS_NO_FF 0
#endif

namespace {

constexpr uint8_t kKey[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
struct CKB {
  static constexpr fbs::KeyBytes kb = fbs::key_bytes_c(kKey);
};

__host__ __device__ inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

constexpr int kWavesPerBlock = 4;

struct alignas(16) SharedImage {
#if FBS_MODE != 2
  fbs::MaskTable mt;
#endif
  uint32_t ff[kWavesPerBlock][FBS_FF_LDS > 0 ? FBS_FF_LDS : 1][64];
};

// Feed-forward store: planes [0, FBS_FF_LDS) in the wave's LDS rows,
// [FBS_FF_LDS, FBS_FF_LDS + FBS_FF_GLB) in the wave's global rows, the rest
// in VGPRs.
constexpr int kFFReg = 128 - FBS_FF_LDS - FBS_FF_GLB;
#if FBS_NO_FF
struct FF {
  uint32_t (*lds)[64];
  uint32_t* glb;
  int lane;
  __device__ void put(int, uint32_t) {}
  __device__ uint32_t get(int) const { return 0; }
};
#else
struct FF {
  uint32_t (*lds)[64];
  uint32_t* glb;  // this lane's column of the wave's [plane][64] rows
  int lane;
  uint32_t reg[kFFReg > 0 ? kFFReg : 1];
  __device__ void put(int p, uint32_t v) {
    if (p < FBS_FF_LDS) lds[p][lane] = v;
    else if (p < FBS_FF_LDS + FBS_FF_GLB) glb[(p - FBS_FF_LDS) * 64] = v;
    else reg[p - FBS_FF_LDS - FBS_FF_GLB] = v;
  }
  __device__ uint32_t get(int p) const {
    if (p < FBS_FF_LDS) return lds[p][lane];
    if (p < FBS_FF_LDS + FBS_FF_GLB) return glb[(p - FBS_FF_LDS) * 64];
    return reg[p - FBS_FF_LDS - FBS_FF_GLB];
  }
};
#endif

struct CKeys {
  __device__ uint32_t first(int p) const { return ((CKB::kb.b[0][p / 8] >> (p % 8)) & 1) ? ~0u : 0u; }
  __device__ uint32_t last(int p) const { return ((CKB::kb.b[10][p / 8] >> (p % 8)) & 1) ? ~0u : 0u; }
};

template <int PIN, int R>
__device__ __forceinline__ void rounds_c(uint32_t* s) {
  if constexpr (R <= 9) {
    fbs::sub_bytes(s);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      fbs::mix_column_c<(PIN + 1) & 3, CKB, R>(s, c);
      FBS_FENCE();
    }
    rounds_c<(PIN + 1) & 3, R + 1>(s);
  }
}

// One middle round entered and left at phase 0 (moves left to the compiler).
__device__ __forceinline__ void round_canon(uint32_t* s, const fbs::MaskKeys& ks, int R) {
  uint32_t t[128];
#pragma unroll
  for (int p = 0; p < 128; ++p) t[p] = s[p];
  fbs::round_mid<0>(t, ks, R);
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) s[8 * fbs::phys(0, r, c) + i] = t[8 * fbs::phys(1, r, c) + i];
}

__device__ __forceinline__ void hash32(uint32_t* s, const fbs::MaskTable* mt, FF& ff) {
  uint32_t o[128];
#if FBS_MODE == 2
  CKeys ck;
  fbs::sigma_ark0(s, ck, ff);
  __asm__ volatile("" ::: "memory");  // the feed-forward really goes through LDS
  rounds_c<0, 1>(s);
  fbs::round_last<1>(s, ck, ff, o);  // 9 rounds from phase 0 -> phase 1
#else
  const fbs::MaskKeys ks{mt};
  fbs::sigma_ark0(s, ks, ff);
  __asm__ volatile("" ::: "memory");  // the feed-forward really goes through LDS
#if FBS_MODE == 0
#pragma unroll 1
  for (int R = 1; R <= 9; ++R) round_canon(s, ks, R);
  fbs::round_last<0>(s, ks, ff, o);
#else
#pragma unroll 1
  for (int R = 1; R <= 5; R += 4) {
    fbs::round_mid<0>(s, ks, R);
    fbs::round_mid<1>(s, ks, R + 1);
    fbs::round_mid<2>(s, ks, R + 2);
    fbs::round_mid<3>(s, ks, R + 3);
  }
  fbs::round_mid<0>(s, ks, 9);
  fbs::round_last<1>(s, ks, ff, o);
#endif
#endif
#pragma unroll
  for (int p = 0; p < 128; ++p) s[p] = o[p];
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FBS_WAVES, FBS_WAVES)))
void fbs_kernel(const fbs::MaskTable* gmt, int iters, uint32_t* out, int full, uint32_t* ffbuf) {
  __shared__ SharedImage sh;
#if FBS_MODE != 2
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(gmt);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&sh.mt);
    for (int i = threadIdx.x; i < (int)(sizeof(fbs::MaskTable) / 4); i += blockDim.x) dst[i] = src[i];
  }
#endif
  __syncthreads();
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  FF ff;
  ff.lds = sh.ff[threadIdx.x >> 6];
  ff.lane = threadIdx.x & 63;
  ff.glb = ffbuf + (size_t)(gid >> 6) * (FBS_FF_GLB > 0 ? FBS_FF_GLB : 1) * 64 + ff.lane;
  uint32_t s[128];
#pragma unroll
  for (int p = 0; p < 128; ++p) s[p] = mix32(gid * 128u + p);
  #if FBS_MODE != 2
  const fbs::MaskTable* mt = &sh.mt;
#else
  const fbs::MaskTable* mt = gmt;
#endif
  for (int it = 0; it < iters; ++it) hash32(s, mt, ff);
  if (full) {
#pragma unroll
    for (int p = 0; p < 128; ++p) out[(size_t)p * gridDim.x * blockDim.x + gid] = s[p];
  } else {
    uint32_t acc = 0;
#pragma unroll
    for (int p = 0; p < 128; ++p) acc ^= s[p];
    out[gid] = acc;
  }
}

}  // namespace

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 16;
  uint32_t rk[44];
  dpf_aes::expand_key(kKey, rk);
  const fbs::MaskTable hmt = fbs::make_mask_table(fbs::key_bytes(rk));
  fbs::MaskTable* dmt;
  CK(hipMalloc(&dmt, sizeof hmt));
  CK(hipMemcpy(dmt, &hmt, sizeof hmt, hipMemcpyHostToDevice));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

  uint32_t* ffb;
  CK(hipMalloc(&ffb, (size_t)cus * 4 * 64 * FBS_WAVES * 2 * (FBS_FF_GLB > 0 ? FBS_FF_GLB : 1) * 4));
  // Correctness: 256 lanes x 32 blocks, two chained hashes, all planes.
  const int vt = 256;
  uint32_t* d;
  CK(hipMalloc(&d, (size_t)vt * 128 * 4));
  fbs_kernel<<<1, vt>>>(dmt, 2, d, 1, ffb);
  CK(hipGetLastError());
  std::vector<uint32_t> h((size_t)vt * 128);
  CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
  dpf_aes::HostLookup lk;
  int bad = 0;
  for (int g = 0; g < vt; ++g)
    for (int b = 0; b < 32; ++b) {
      uint32_t w[4] = {0, 0, 0, 0}, e[4] = {0, 0, 0, 0};
      for (int p = 0; p < 128; ++p) {
        w[p / 32] |= ((mix32(g * 128u + p) >> b) & 1u) << (p % 32);
        e[p / 32] |= ((h[(size_t)p * vt + g] >> b) & 1u) << (p % 32);
      }
      dpf_aes::Block4 x{w[0], w[1], w[2], w[3]};
      for (int rep = 0; rep < 2; ++rep)
        x = FBS_NO_FF ? dpf_aes::encrypt(dpf_aes::sigma(x), lk, dpf_aes::ArrayRK{rk})
                      : dpf_aes::mmo_hash(x, lk, dpf_aes::ArrayRK{rk});
      if (x.w0 != e[0] || x.w1 != e[1] || x.w2 != e[2] || x.w3 != e[3]) ++bad;
    }
  CK(hipFree(d));
  printf("gpu check (mode %d, ff_lds %d): %d mismatching blocks of %d\n", FBS_MODE, FBS_FF_LDS,
         bad, vt * 32);
  if (bad) return 1;

  const int block = 256;
  const int threads = cus * 4 * 64 * FBS_WAVES * 2;  // two waves' worth of work per slot
  CK(hipMalloc(&d, (size_t)threads * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    fbs_kernel<<<threads / block, block>>>(dmt, iters, d, 0, ffb);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep && ms < best) best = ms;
  }
  const double blocks = (double)threads * 32 * iters;
  printf("{\"mode\": %d, \"ff_lds\": %d, \"ff_glb\": %d, \"sbox_group\": %d, \"waves_per_simd\": %d, "
         "\"iters\": %d, \"ms\": %.3f, \"g_aes_per_s\": %.2f}\n",
         FBS_MODE, FBS_FF_LDS, FBS_FF_GLB, FBS_SBOX_GROUP, FBS_WAVES, iters, best, blocks / best / 1e6);
  return 0;
}
