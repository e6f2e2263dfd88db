// aes_microbench.hip -- standalone throughput study of AES-128 on gfx950
// (T-table in bank-replicated LDS), used to choose the kernel design.
// Each thread runs `iters` dependent MMO hashes on register-resident blocks,
// so memory traffic is nil and the result isolates the AES core.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/aes_microbench.hip -o tools/aes_microbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../distributed_point_functions_amd/csrc/kernels/aes_core.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

using dpf_aes::Block4;

struct T0Table { uint32_t v[256]; };
constexpr T0Table make_t0() {
  T0Table t{};
  for (int i = 0; i < 256; ++i) {
    uint32_t s = dpf_aes::kSbox[i];
    uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
    t.v[i] = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
  }
  return t;
}
__constant__ T0Table c_t0 = make_t0();
struct RK { uint32_t k[44]; };

// ---- lookup flavours ------------------------------------------------------
struct L4 {  // 4 tables x 32 copies = 128 KiB
  const char* base; uint32_t l0, l2;
  template <int T, int K> __device__ __forceinline__ uint32_t lookup(uint32_t w) const {
    uint32_t idx = K == 0 ? (w << 7) & 0x7f80u : K == 1 ? (w >> 1) & 0x7f80u
                 : K == 2 ? (w >> 9) & 0x7f80u : (w >> 17) & 0x7f80u;
    uint32_t off = (idx | (T < 2 ? l0 : l2)) + ((T & 1) ? 32768u : 0u);
    return *reinterpret_cast<const uint32_t*>(base + off);
  }
  __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) const {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
};
struct L1 {  // 1 table x 32 copies = 32 KiB, rotations in VALU
  const char* base; uint32_t l0;
  template <int T, int K> __device__ __forceinline__ uint32_t lookup(uint32_t w) const {
    uint32_t idx = K == 0 ? (w << 7) & 0x7f80u : K == 1 ? (w >> 1) & 0x7f80u
                 : K == 2 ? (w >> 9) & 0x7f80u : (w >> 17) & 0x7f80u;
    uint32_t v = *reinterpret_cast<const uint32_t*>(base + (idx | l0));
    return T == 0 ? v : __builtin_amdgcn_alignbit(v, v, 32 - 8 * T);
  }
  __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) const {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
};
struct URK {
  const uint32_t* k;
  __device__ __forceinline__ uint32_t operator()(int i) const { return k[i]; }
  template <class LK>
  __device__ __forceinline__ uint32_t mix(const LK& lk, uint32_t a, uint32_t b, int i) const { return lk.xor3(a, b, k[i]); }
};
// 4 tables in 256-byte rows: row e = [A copies 0..31 | B copies 0..31], C|D at +64 KiB.
// Address = v_perm_b32(w, lane_reg[T], sel_K): byte0 = lane offset (+128 for B/D),
// byte1 = byte K of w (the entry), byte2 = 1 for C/D.
struct LP {
  const char* base; uint32_t lt[4];
  template <int T, int K> __device__ __forceinline__ uint32_t lookup(uint32_t w) const {
    constexpr uint32_t sel = 0x0c020000u | ((4u + K) << 8);
    uint32_t off = __builtin_amdgcn_perm(w, lt[T], sel);
    return *reinterpret_cast<const uint32_t*>(base + off);
  }
  __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) const {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
};
__device__ void fill_perm(uint32_t* tab) {
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
    int t = 2 * (i >> 14) + ((i >> 5) & 1), e = (i >> 6) & 255;
    uint32_t v = c_t0.v[e];
    tab[i] = t == 0 ? v : ((v << (8 * t)) | (v >> (32 - 8 * t)));
  }
  __syncthreads();
}
template <int ILP>
__global__ void k_aes_perm(int iters, uint4* out, RK rk) {
  __shared__ uint32_t tab[32768];
  fill_perm(tab);
  uint32_t l = (threadIdx.x & 31) * 4;
  LP lk{(const char*)tab, {l, l + 128, l + 65536, l + 65536 + 128}};
  Block4 s[ILP];
  for (int j = 0; j < ILP; ++j) s[j] = Block4{threadIdx.x + j, blockIdx.x, 7u * j, 99u};
  for (int it = 0; it < iters; ++it) {
    if constexpr (ILP == 1) s[0] = dpf_aes::mmo_hash(s[0], lk, URK{rk.k});
    else dpf_aes::mmo_hash2(s[0], s[1], lk, URK{rk.k}, URK{rk.k});
  }
  uint32_t x = 0;
  for (int j = 0; j < ILP; ++j) x ^= s[j].w0 ^ s[j].w1 ^ s[j].w2 ^ s[j].w3;
  if (x == 0x12345678u) out[0] = make_uint4(x, 0, 0, 0);
}
// correctness probe: one hash of a known block with each lookup flavour
__global__ void k_check(uint4* out, RK rk) {
  __shared__ uint32_t tab[32768];
  fill_perm(tab);
  uint32_t l = (threadIdx.x & 31) * 4;
  LP lk{(const char*)tab, {l, l + 128, l + 65536, l + 65536 + 128}};
  Block4 b{threadIdx.x, 0x01230123u, 0x01230123u ^ threadIdx.x, 0x01230123u};
  Block4 h = dpf_aes::mmo_hash(b, lk, URK{rk.k});
  out[threadIdx.x] = make_uint4(h.w0, h.w1, h.w2, h.w3);
}



template <int TABLES>
__device__ void fill(uint32_t* tab) {
  for (int i = threadIdx.x; i < TABLES * 8192; i += blockDim.x) {
    int t = i >> 13, e = (i >> 5) & 255;
    uint32_t v = c_t0.v[e];
    tab[i] = t == 0 ? v : ((v << (8 * t)) | (v >> (32 - 8 * t)));
  }
  __syncthreads();
}

// ILP chains per thread
template <int TABLES, int ILP>
__global__ void k_aes(int iters, uint4* out, RK rk) {
  __shared__ uint32_t tab[TABLES * 8192];
  fill<TABLES>(tab);
  uint32_t lane = threadIdx.x & 31;
  Block4 s[ILP];
  for (int j = 0; j < ILP; ++j) s[j] = Block4{threadIdx.x + j, blockIdx.x, 7u * j, 99u};
  if constexpr (TABLES == 4) {
    L4 lk{(const char*)tab, lane * 4, lane * 4 + 65536};
    for (int it = 0; it < iters; ++it) {
      if constexpr (ILP == 1) s[0] = dpf_aes::mmo_hash(s[0], lk, URK{rk.k});
      else dpf_aes::mmo_hash2(s[0], s[1], lk, URK{rk.k}, URK{rk.k});
    }
  } else {
    L1 lk{(const char*)tab, lane * 4};
    for (int it = 0; it < iters; ++it) {
      if constexpr (ILP == 1) s[0] = dpf_aes::mmo_hash(s[0], lk, URK{rk.k});
      else dpf_aes::mmo_hash2(s[0], s[1], lk, URK{rk.k}, URK{rk.k});
    }
  }
  uint32_t x = 0;
  for (int j = 0; j < ILP; ++j) x ^= s[j].w0 ^ s[j].w1 ^ s[j].w2 ^ s[j].w3;
  if (x == 0x12345678u) out[0] = make_uint4(x, 0, 0, 0);
}

// Ablation: same LDS reads, minimal VALU (address = previous read value masked).
__global__ void k_lds_only(int iters, uint4* out) {
  __shared__ uint32_t tab[4 * 8192];
  fill<4>(tab);
  uint32_t lane = (threadIdx.x & 31) * 4;
  uint32_t a[16];
  for (int j = 0; j < 16; ++j) a[j] = (threadIdx.x * 7 + j) & 0x7f80;
  for (int it = 0; it < iters * 10; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      a[j] = (*reinterpret_cast<const uint32_t*>((const char*)tab + (a[j] & 0x1ff80u) + lane)) ;
  }
  uint32_t x = 0;
  for (int j = 0; j < 16; ++j) x ^= a[j];
  if (x == 0x12345678u) out[0] = make_uint4(x, 0, 0, 0);
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint4* out;
  CK(hipMalloc(&out, 64));
  RK rk;
  uint8_t key[16] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
  dpf_aes::expand_key(key, rk.k);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 2000;
  auto run = [&](const char* name, auto kern, int block, int wgs_per_cu, double aes_per_thread_iter) {
    int grid = cus * wgs_per_cu;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, iters, out, rk);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double aes = (double)grid * block * iters * aes_per_thread_iter;
    printf("%-34s block=%4d wg/cu=%d  %8.3f ms  %7.2f G AES/s\n", name, block, wgs_per_cu, ms,
           aes / ms / 1e6);
  };
  {
    uint4* o; CK(hipMalloc(&o, 64 * 16));
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, o, rk);
    uint4 h[64]; CK(hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost));
    dpf_aes::HostLookup hl; int bad = 0;
    for (int t = 0; t < 64; ++t) {
      Block4 b{(uint32_t)t, 0x01230123u, 0x01230123u ^ (uint32_t)t, 0x01230123u};
      Block4 w = dpf_aes::mmo_hash(b, hl, dpf_aes::ArrayRK{rk.k});
      bad += (w.w0 != h[t].x || w.w1 != h[t].y || w.w2 != h[t].z || w.w3 != h[t].w);
    }
    printf("perm-lookup correctness: %s\n", bad ? "MISMATCH" : "ok");
  }
  run("perm ILP1", k_aes_perm<1>, 1024, 1, 1);
  run("perm ILP2", k_aes_perm<2>, 1024, 1, 2);
  run("perm ILP1 512thr", k_aes_perm<1>, 512, 1, 1);
  run("4tab ILP1", k_aes<4, 1>, 1024, 1, 1);
  run("4tab ILP2", k_aes<4, 2>, 1024, 1, 2);
  run("4tab ILP1 512thr", k_aes<4, 1>, 512, 1, 1);
  run("4tab ILP2 512thr", k_aes<4, 2>, 512, 1, 2);
  run("1tab ILP1 1024x2", k_aes<1, 1>, 1024, 2, 1);
  run("1tab ILP1 512x4", k_aes<1, 1>, 512, 4, 1);
  run("1tab ILP2 1024x2", k_aes<1, 2>, 1024, 2, 2);
  run("1tab ILP2 512x4", k_aes<1, 2>, 512, 4, 2);
  run("1tab ILP1 1024x1", k_aes<1, 1>, 1024, 1, 1);
  // LDS-only: 160 reads per "AES"
  {
    int grid = cus;
    hipEventRecord(a);
    hipLaunchKernelGGL(k_lds_only, dim3(grid), dim3(1024), 0, 0, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double reads = (double)grid * 1024 * iters * 160;
    printf("%-34s %8.3f ms  %7.2f G lane-reads/s = %6.1f TB/s (equiv %6.2f G AES/s)\n", "lds_only b32",
           ms, reads / ms / 1e6, reads * 4 / ms / 1e9, reads / 160 / ms / 1e6);
  }
  return 0;
}
