// ws_microbench.hip -- can a bitsliced-AES wave use the VALU cycles that the
// LDS-bound T-table waves leave idle?  One 1024-thread workgroup per CU (the
// 128 KiB LDS tables), waves 0..NT-1 run the octet expand kernel's T-table
// work (2 + 4 + 8 child hashes and 8 value hashes per octet, the exact
// dpf_device.h steps), waves NT..15 run the bitsliced 8-block MMO hash of
// bs_aes.h under the fixed value key.  Each part's iteration count is a
// kernel argument (0 = idle), so one binary measures T alone, BS alone and
// both together on the same CUs.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DWS_NT=12 tools/ws_microbench.hip -o tools/wsmb_12
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "bs_aes.h"
#include "../distributed_point_functions_amd/csrc/kernels/dpf_device.h"

#ifndef WS_NT
#define WS_NT 12
#endif

namespace {
constexpr uint8_t kValueKeyBytes[16] = {0x98, 0x1c, 0x1d, 0xb2, 0x01, 0x11, 0xa3, 0x46,
                                        0xe3, 0x23, 0x54, 0x8c, 0x58, 0xd1, 0xa5, 0x05};
struct ValueKeyMasks {
  static constexpr bsa::BsKeyMasks m = bsa::make_key_masks_c(kValueKeyBytes);
};

__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4)))
void ws_kernel(RoundKeys rkl, RoundKeys rkr, RoundKeys rkv, int t_iters, int b_iters,
               uint32_t* out) {
  __shared__ LdsImage lds;
  fill_tables(lds.tab);
  if (threadIdx.x < 64) {
    lds.cw_seed[threadIdx.x] = make_uint4(threadIdx.x * 77u, 5u, 9u, threadIdx.x);
    lds.cw_ctrl[threadIdx.x] = threadIdx.x & 3u;
  }
  __syncthreads();
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t gid = blockIdx.x * 1024u + threadIdx.x;
  uint32_t acc = 0;
  if (wid < WS_NT) {
    const LdsLookup lk = make_lookup(lds);
    const UniformRK rv[4] = {UniformRK{rkv.k}, UniformRK{rkv.k}, UniformRK{rkv.k},
                             UniformRK{rkv.k}};
    Block4 node{gid, gid * 3u, 7u, 11u};
    uint32_t nt = gid & 1u;
    for (int it = 0; it < t_iters; ++it) {
#if defined(WS_FIXLVL)
      const int lvl = 20;
#else
      const int lvl = it & 31;
#endif
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
        for (int j = 0; j < 4; ++j) {
#if defined(WS_CORRECT)
          Block4 h = l[j];
          if (lt[j]) h = lanes_add<64>(h, Block4{rkv.k[1], rkv.k[2], rkv.k[3], rkv.k[4]});
          if (t_iters == 12345) h = lanes_neg<64>(h);
          acc ^= h.w0 ^ h.w1 ^ h.w2 ^ h.w3;
#else
          acc ^= l[j].w0 ^ l[j].w1 ^ l[j].w2 ^ l[j].w3 ^ lt[j];
#endif
        }
      }
    }
  }
#if WS_NT < 16
  else {
    uint32_t w[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) w[i] = gid * 32u + i;
    for (int it = 0; it < b_iters; ++it) {
      uint32_t ff[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) ff[i] = w[i];
      bsa::aes8_c<ValueKeyMasks>(w);
#pragma unroll
      for (int i = 0; i < 32; ++i) w[i] ^= ff[i];
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= w[i];
  }
#endif
  out[gid] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

float run(int cus, RoundKeys* k, int t_iters, int b_iters, uint32_t* d) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(ws_kernel, dim3(cus), dim3(1024), 0, 0, k[0], k[1], k[2], t_iters, b_iters,
                       d);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep && ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return best;
}
// Host restatement of the T waves' chain for lane `gid` (correctness check).
uint32_t host_chain(uint32_t gid, int t_iters, const RoundKeys* k) {
  static dpf_aes::HostLookup lk;
  auto cs = [](int i) { return Block4{(uint32_t)i * 77u, 5u, 9u, (uint32_t)i}; };
  auto step = [&](Block4 s, uint32_t t, int lvl, Block4& c0, uint32_t& t0, Block4& c1,
                  uint32_t& t1) {
    Block4 h0 = dpf_aes::mmo_hash(s, lk, dpf_aes::ArrayRK{k[0].k});
    Block4 h1 = dpf_aes::mmo_hash(s, lk, dpf_aes::ArrayRK{k[1].k});
    const Block4 c = cs(lvl);
    const uint32_t m = 0u - t, cc = (uint32_t)lvl & 3u;
    h0 = Block4{h0.w0 ^ (c.w0 & m), h0.w1 ^ (c.w1 & m), h0.w2 ^ (c.w2 & m), h0.w3 ^ (c.w3 & m)};
    h1 = Block4{h1.w0 ^ (c.w0 & m), h1.w1 ^ (c.w1 & m), h1.w2 ^ (c.w2 & m), h1.w3 ^ (c.w3 & m)};
    t0 = (h0.w0 & 1u) ^ (t & (cc & 1u));
    t1 = (h1.w0 & 1u) ^ (t & ((cc >> 1) & 1u));
    h0.w0 &= ~1u;
    h1.w0 &= ~1u;
    c0 = h0;
    c1 = h1;
  };
  Block4 node{gid, gid * 3u, 7u, 11u};
  uint32_t nt = gid & 1u, acc = 0;
  for (int it = 0; it < t_iters; ++it) {
#if defined(WS_FIXLVL)
    const int lvl = 20;
#else
    const int lvl = it & 31;
#endif
    Block4 c[2], q[4];
    uint32_t ct[2], qt[4];
    step(node, nt, lvl, c[0], ct[0], c[1], ct[1]);
    step(c[0], ct[0], lvl + 1, q[0], qt[0], q[1], qt[1]);
    step(c[1], ct[1], lvl + 1, q[2], qt[2], q[3], qt[3]);
    for (int hf = 0; hf < 2; ++hf) {
      Block4 l[4];
      uint32_t lt[4];
      step(q[2 * hf], qt[2 * hf], lvl + 2, l[0], lt[0], l[1], lt[1]);
      step(q[2 * hf + 1], qt[2 * hf + 1], lvl + 2, l[2], lt[2], l[3], lt[3]);
      if (hf == 1) { node = l[3]; nt = lt[3]; }
      for (int j = 0; j < 4; ++j) {
        const Block4 h = dpf_aes::mmo_hash(l[j], lk, dpf_aes::ArrayRK{k[2].k});
        acc ^= h.w0 ^ h.w1 ^ h.w2 ^ h.w3 ^ lt[j];
      }
    }
  }
  return acc;
}
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
  uint32_t* d;
  CK(hipMalloc(&d, (size_t)cus * 1024 * 4));
  const int nt = WS_NT, nb = 16 - WS_NT;
  const int t_iters = argc > 1 ? atoi(argv[1]) : 400;
  const double t_aes = (double)cus * nt * 64 * t_iters * 22;
  const double per_b = (double)cus * nb * 64 * 8;
  const float tt = run(cus, k, t_iters, 0, d);
#if !defined(WS_CORRECT) && !defined(WS_NOCHECK)
  {
    std::vector<uint32_t> h((size_t)cus * 1024);
    CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    const uint32_t probe[4] = {0u, 1u, 777u, (uint32_t)cus * 1024u - 1u};
    for (uint32_t g : probe)
      if ((int)((g & 1023) >> 6) < nt && h[g] != host_chain(g, t_iters, k)) ++bad;
    printf("{\"check\": \"%s\"}\n", bad ? "MISMATCH" : "ok");
  }
#endif
  printf("{\"nt\": %d, \"nb\": %d, \"mode\": \"T only\", \"ms\": %.3f, \"t_gaes\": %.2f}\n", nt, nb,
         tt, t_aes / tt / 1e6);
  if (nb == 0) return 0;
  const int b1 = 100;
  const float bt = run(cus, k, 0, b1, d);
  printf("{\"nt\": %d, \"nb\": %d, \"mode\": \"BS only\", \"b_iters\": %d, \"ms\": %.3f, "
         "\"b_gaes\": %.2f}\n", nt, nb, b1, bt, per_b * b1 / bt / 1e6);
  // Both: BS iterations that would fill 25%..125% of the T-only time at its solo rate.
  for (int pct = 25; pct <= 150; pct += 25) {
    const int bi = (int)(b1 * (tt / bt) * pct / 100.0);
    const float ms = run(cus, k, t_iters, bi, d);
    printf("{\"nt\": %d, \"nb\": %d, \"mode\": \"both\", \"b_iters\": %d, \"ms\": %.3f, "
           "\"t_alone_ms\": %.3f, \"total_gaes\": %.2f, \"t_gaes\": %.2f, \"b_gaes\": %.2f}\n",
           nt, nb, bi, ms, tt, (t_aes + per_b * bi) / ms / 1e6, t_aes / ms / 1e6,
           per_b * bi / ms / 1e6);
  }
  return 0;
}
