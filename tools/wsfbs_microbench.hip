// wsfbs_microbench.hip -- the one wave-specialised combination r13 left
// unmeasured: T-table tree waves beside full-bitslice
// value-hash waves (tools/fbs_aes.h) whose MMO feed-forward stays in registers.
//
// Register budget first (hipcc -Rpass-analysis=kernel-resource-usage, gfx950):
// the full-bitslice hash with sigma(x) in registers needs 256 VGPRs + 114 AGPRs
// = 370 of a SIMD lane's 512 registers at one wave per SIMD; the octet kernel's
// T-table waves need ~120.  So one SIMD holds one bitslice wave plus at most
// ONE T-table wave (370 + 120 <= 512); the "two T-table waves per SIMD plus one
// bitslice wave" split does not fit (2 x 120 + 370 = 610 > 512).  A kernel has
// one register allocation for all its waves, so the split runs as two kernels
// on two streams, each sized to one wave per SIMD, co-resident on every CU.
//
// Measured (one JSON line each, best of 4 after a warm-up):
//   T16    the T-table work alone, 16 waves per CU (the octet kernel's shape)
//   T4     the same work, 4 waves per CU (one per SIMD)
//   B4     the bitslice MMO hash alone, 4 waves per CU, feed-forward in registers
//   T4+B4  both kernels at once on two streams
// The T-table work is the octet kernel's per-octet step mix (2 + 4 + 8 child
// hashes and 8 value hashes, dpf_device.h); the bitslice work hashes 32 blocks
// per lane per iteration (x <- H(x)).  A host check compares one lane of each.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-sched-strategy=iterative-ilp \
//          tools/wsfbs_microbench.hip -o tools/wsfbs_microbench
#define FBS_MODE 2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../distributed_point_functions_amd/csrc/kernels/dpf_device.h"
#include "fbs_aes.h"

namespace {

// ---------------------------------------------------------------- T-table part
// The T-table kernel is compiled to the octet kernel's budget of 128 VGPRs
// (waves_per_eu(4, 4)), so a T-table wave and a ~377-register bitslice wave
// fit one SIMD lane's 512 registers together.
__device__ __forceinline__ void t_body(LdsImage& lds, const RoundKeys& rkl, const RoundKeys& rkr,
                                       const RoundKeys& rkv, int iters, uint32_t* out,
                                       int keep_waves) {
  fill_tables(lds.tab);
  if (threadIdx.x < 64) {
    lds.cw_seed[threadIdx.x] = make_uint4(threadIdx.x * 77u, 5u, 9u, threadIdx.x);
    lds.cw_ctrl[threadIdx.x] = threadIdx.x & 3u;
  }
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= keep_waves) return;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const LdsLookup lk = make_lookup(lds);
  const UniformRK rv[4] = {UniformRK{rkv.k}, UniformRK{rkv.k}, UniformRK{rkv.k}, UniformRK{rkv.k}};
  Block4 node{gid, gid * 3u, 7u, 11u};
  uint32_t nt = gid & 1u, acc = 0;
  for (int it = 0; it < iters; ++it) {
    const int lvl = it & 31;
    Block4 c[2], q[4];
    uint32_t ct[2], qt[4];
    children_step(lk, rkl.k, rkr.k, node, nt, lds.cw_seed[lvl], lds.cw_ctrl[lvl], c[0], ct[0],
                  c[1], ct[1]);
    children_step_x2(lk, rkl.k, rkr.k, c[0], ct[0], c[1], ct[1], lds.cw_seed[lvl + 1],
                     lds.cw_ctrl[lvl + 1], q, qt);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      Block4 l[4];
      uint32_t lt[4];
      children_step_x2(lk, rkl.k, rkr.k, q[2 * hf], qt[2 * hf], q[2 * hf + 1], qt[2 * hf + 1],
                       lds.cw_seed[lvl + 2], lds.cw_ctrl[lvl + 2], l, lt);
      if (hf == 1) { node = l[3]; nt = lt[3]; }
      dpf_aes::mmo_hashN<4>(l, lk, rv);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc ^= l[j].w0 ^ l[j].w1 ^ l[j].w2 ^ l[j].w3 ^ lt[j];
    }
  }
  out[gid] = acc;
}
// keep_waves < 16: waves keep_waves..15 leave right after the table fill, so
// their registers free up (one wave per SIMD stays with keep_waves = 4) and a
// co-launched bitslice kernel's waves can take them.
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4)))
void t_kernel(RoundKeys rkl, RoundKeys rkr, RoundKeys rkv, int iters, uint32_t* out,
              int keep_waves) {
  __shared__ LdsImage lds;
  t_body(lds, rkl, rkr, rkv, iters, out, keep_waves);
}
constexpr int kTAesPerIter = 2 + 4 + 8 + 8;

// ---------------------------------------------------------------- bitslice part
constexpr uint8_t kKey[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
struct CKB {
  static constexpr fbs::KeyBytes kb = fbs::key_bytes_c(kKey);
};
struct CKeys {
  __device__ uint32_t first(int p) const { return ((CKB::kb.b[0][p / 8] >> (p % 8)) & 1) ? ~0u : 0u; }
  __device__ uint32_t last(int p) const { return ((CKB::kb.b[10][p / 8] >> (p % 8)) & 1) ? ~0u : 0u; }
};
struct FFRegs {  // the 128 planes of sigma(x), in registers (the compiler's AGPRs)
  uint32_t reg[128];
  __device__ void put(int p, uint32_t v) { reg[p] = v; }
  __device__ uint32_t get(int p) const { return reg[p]; }
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
__host__ __device__ inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// 32 x 32 bit-matrix transpose of a[0..31] (a[i] bit j <-> a[j] bit i): the
// conversion between 32 blocks' words and their bit planes that a bitslice
// wave pays on its inputs (leaf seeds) and outputs (hashes).
__device__ __forceinline__ void transpose32(uint32_t* a) {
#pragma unroll
  for (int st = 0; st < 5; ++st) {
    const int j = 16 >> st;
    const uint32_t m = st == 0 ? 0x0000ffffu : st == 1 ? 0x00ff00ffu : st == 2 ? 0x0f0f0f0fu
                     : st == 3 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int blk = 0; blk < 32; blk += 2 * j)
#pragma unroll
      for (int i = 0; i < j; ++i) {
        const int k = blk + i;
        const uint32_t t = (a[k] ^ (a[k + j] >> j)) & m;
        a[k] ^= t;
        a[k + j] ^= t << j;
      }
  }
}

// TRANSPOSES = 1: every iteration also converts the 128 planes to words and
// back (4 + 4 transposes; net identity), the layout changes a bitslice wave
// fed by and feeding ordinary blocks pays.
template <int TRANSPOSES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void b_kernel(int iters, uint32_t* out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t s[128];
#pragma unroll
  for (int p = 0; p < 128; ++p) s[p] = mix32(gid * 128u + p);
  const CKeys ck;
  for (int it = 0; it < iters; ++it) {
    if (TRANSPOSES) {
#pragma unroll
      for (int q = 0; q < 4; ++q) transpose32(s + 32 * q);
#pragma unroll
      for (int q = 0; q < 4; ++q) transpose32(s + 32 * q);
    }
    FFRegs ff;
    uint32_t o[128];
    fbs::sigma_ark0(s, ck, ff);
    rounds_c<0, 1>(s);
    fbs::round_last<1>(s, ck, ff, o);
#pragma unroll
    for (int p = 0; p < 128; ++p) s[p] = o[p];
  }
  uint32_t acc = 0;
#pragma unroll
  for (int p = 0; p < 128; ++p) acc ^= s[p] * (uint32_t)(2 * p + 1);
  out[gid] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

// Host check of one bitslice lane: 32 blocks, `iters` chained MMO hashes.
uint32_t host_b(uint32_t gid, int iters) {
  uint32_t rk[44];
  dpf_aes::expand_key(kKey, rk);
  static dpf_aes::HostLookup lk;
  uint32_t planes[128] = {};
  for (int b = 0; b < 32; ++b) {
    uint32_t w[4] = {0, 0, 0, 0};
    for (int p = 0; p < 128; ++p) w[p / 32] |= ((mix32(gid * 128u + p) >> b) & 1u) << (p % 32);
    dpf_aes::Block4 x{w[0], w[1], w[2], w[3]};
    for (int i = 0; i < iters; ++i) x = dpf_aes::mmo_hash(x, lk, dpf_aes::ArrayRK{rk});
    const uint32_t o[4] = {x.w0, x.w1, x.w2, x.w3};
    for (int p = 0; p < 128; ++p) planes[p] |= ((o[p / 32] >> (p % 32)) & 1u) << b;
  }
  uint32_t acc = 0;
  for (int p = 0; p < 128; ++p) acc ^= planes[p] * (uint32_t)(2 * p + 1);
  return acc;
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  float ms() { float m; CK(hipEventElapsedTime(&m, a, b)); return m; }
};

}  // namespace

int main(int argc, char** argv) {
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  RoundKeys k[3];
  for (int j = 0; j < 3; ++j) {
    dpf_aes_key key;
    for (int i = 0; i < 16; ++i) key.bytes[i] = (uint8_t)(i * 13 + j);
    k[j] = expand_key(&key);
  }
  const int t_iters = argc > 1 ? atoi(argv[1]) : 200;
  int b_iters = argc > 2 ? atoi(argv[2]) : 40;
  uint32_t *dt, *db;
  CK(hipMalloc(&dt, (size_t)cus * 1024 * 4));
  CK(hipMalloc(&db, (size_t)cus * 256 * 4));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  // Bitslice correctness on two lanes.
  b_kernel<1><<<cus, 256, 0, s2>>>(2, db);
  CK(hipStreamSynchronize(s2));
  {
    std::vector<uint32_t> h((size_t)cus * 256);
    CK(hipMemcpy(h.data(), db, h.size() * 4, hipMemcpyDeviceToHost));
    const bool ok = h[0] == host_b(0, 2) && h[777] == host_b(777, 2);
    printf("{\"bitslice_check\": \"%s\"}\n", ok ? "ok" : "MISMATCH");
    if (!ok) return 1;
  }
  auto best = [&](auto launch) {
    float m = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      const float x = launch();
      if (rep && x < m) m = x;
    }
    return m;
  };
  Timer tm;
  auto run_t16 = [&] {
    CK(hipEventRecord(tm.a, s1));
    hipLaunchKernelGGL(t_kernel, dim3(cus), dim3(1024), 0, s1, k[0], k[1], k[2], t_iters, dt, 16);
    CK(hipEventRecord(tm.b, s1));
    CK(hipEventSynchronize(tm.b));
    return tm.ms();
  };
  auto run_t4 = [&](int it) {
    CK(hipEventRecord(tm.a, s1));
    hipLaunchKernelGGL(t_kernel, dim3(cus), dim3(1024), 0, s1, k[0], k[1], k[2], it, dt, 4);
    CK(hipEventRecord(tm.b, s1));
    CK(hipEventSynchronize(tm.b));
    return tm.ms();
  };
  int tr = 0;   // transposes in the bitslice kernel (second pass)
  auto run_b4 = [&](int it) {
    CK(hipEventRecord(tm.a, s2));
    if (tr) hipLaunchKernelGGL(b_kernel<1>, dim3(cus), dim3(256), 0, s2, it, db);
    else hipLaunchKernelGGL(b_kernel<0>, dim3(cus), dim3(256), 0, s2, it, db);
    CK(hipEventRecord(tm.b, s2));
    CK(hipEventSynchronize(tm.b));
    return tm.ms();
  };
  const double t16_aes = (double)cus * 1024 * t_iters * kTAesPerIter;
  const float t16 = best(run_t16);
  printf("{\"case\": \"T16\", \"ms\": %.3f, \"g_aes_per_s\": %.2f}\n", t16, t16_aes / t16 / 1e6);
  const int t4_iters = t_iters;
  const double t4_aes = (double)cus * 256 * t4_iters * kTAesPerIter;   // 4 of 16 waves work
  const float t4 = best([&] { return run_t4(t4_iters); });
  printf("{\"case\": \"T4\", \"ms\": %.3f, \"g_aes_per_s\": %.2f}\n", t4, t4_aes / t4 / 1e6);
  for (tr = 0; tr <= 1; ++tr) {
    const float b4 = best([&] { return run_b4(b_iters); });
    const double b_aes_per_iter = (double)cus * 256 * 32;
    printf("{\"case\": \"B4\", \"transposes\": %d, \"iters\": %d, \"ms\": %.3f, "
           "\"g_aes_per_s\": %.2f}\n", tr, b_iters, b4, b_aes_per_iter * b_iters / b4 / 1e6);
    // Both at once, the bitslice share swept around the balance point.
    for (int pct : {50, 75, 100, 125}) {
      const int bi = (int)(b_iters * t4 / b4 * pct / 100.0 + 0.5);
      Timer t2;
      float both = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(tm.a, s1));
        CK(hipStreamWaitEvent(s2, tm.a, 0));
        hipLaunchKernelGGL(t_kernel, dim3(cus), dim3(1024), 0, s1, k[0], k[1], k[2], t4_iters, dt, 4);
        if (tr) hipLaunchKernelGGL(b_kernel<1>, dim3(cus), dim3(256), 0, s2, bi, db);
        else hipLaunchKernelGGL(b_kernel<0>, dim3(cus), dim3(256), 0, s2, bi, db);
        CK(hipEventRecord(t2.b, s2));
        CK(hipStreamWaitEvent(s1, t2.b, 0));
        CK(hipEventRecord(tm.b, s1));
        CK(hipEventSynchronize(tm.b));
        const float x = tm.ms();
        if (rep && x < both) both = x;
      }
      const double tot = t4_aes + b_aes_per_iter * bi;
      printf("{\"case\": \"T4+B4\", \"transposes\": %d, \"b_share\": %.3f, \"b_iters\": %d, "
             "\"ms\": %.3f, \"g_aes_per_s\": %.2f, \"vs_T16\": %.3f}\n", tr,
             b_aes_per_iter * bi / tot, bi, both, tot / both / 1e6, tot / both / (t16_aes / t16));
    }
  }
  return 0;
}
