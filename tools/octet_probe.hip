// octet_probe.hip -- where does the octet expand kernel lose against the bare
// octet AES chain of tools/ws_microbench.hip?  A copy of expand_octet_kernel
// (dpf_kernels.hip) at config 2's shape (one start seed, 29 levels, S = 11,
// 2^18 items, 2^30 uint64 outputs) whose parts can be switched off at compile
// time:
//   -DPROBE_NOSTORE  outputs folded into a register instead of stored
//   -DPROBE_NOWALK   no start walk (the item's root seed is derived directly)
//   -DPROBE_NODFS    no DFS stack: each octet's root is the previous octet's
//                    last leaf seed (the bare chain of ws_microbench)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 [-D...] tools/octet_probe.hip -o tools/op_X
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../distributed_point_functions_amd/csrc/kernels/dpf_device.h"

namespace {

__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void probe_kernel(
    ExpandParams p, FastIntLeaf<64, false> leaf, uint32_t* sink) {
  __shared__ LdsImage lds;
  leaf.vcw = Block4{0x12345u, 0x6789u, 0xabcdu, 0xef01u};
  fill_tables(lds.tab);
  fill_cws(lds, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  __syncthreads();
  const LdsLookup lk = make_lookup(lds);
  const int k0 = p.k0, S = p.S;
  const int G = S - 3;
  const int64_t ngroups = (int64_t)1 << G;
  const UniformRK rv[4] = {UniformRK{p.rkv.k}, UniformRK{p.rkv.k}, UniformRK{p.rkv.k},
                           UniformRK{p.rkv.k}};
  uint32_t acc = 0;
  for (int64_t item = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; item < p.num_items;
       item += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = item >> k0;
    Block4 s = load_block(p.seeds_in + r);
    uint32_t t = p.ctrl_in[r] & 1u;
#if defined(PROBE_NOWALK)
    s.w0 ^= (uint32_t)item;
    s.w1 ^= (uint32_t)(item >> 7);
#else
    for (int j = 0; j < k0; ++j) {
      const uint32_t bit = (uint32_t)((item >> (k0 - 1 - j)) & 1);
      path_step(lk, p.rkl, p.rkd, s, t, bit, lds.cw_seed[j], lds.cw_ctrl[j]);
    }
#endif
    const int64_t leaf_base = item << S;
#if !defined(PROBE_NODFS)
    Block4 sib[kGMax];
    uint32_t tb = 0;
#endif
    Block4 next = s;
    uint32_t nextt = t;
    for (int64_t g = 0; g < ngroups; ++g) {
      Block4 node = next;
      uint32_t nt = nextt;
#if !defined(PROBE_NODFS)
      int ds = 0;
      if (g != 0) {
        ds = G - (int)__builtin_ctzll((unsigned long long)g);
        nt = (tb >> ds) & 1u;
      }
      for (int d = ds; d < G; ++d) {
        Block4 c0, c1;
        uint32_t t0, t1;
        children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.cw_seed[k0 + d], lds.cw_ctrl[k0 + d],
                      c0, t0, c1, t1);
        sib[d] = c1;
        tb = (tb & ~(1u << (d + 1))) | (t1 << (d + 1));
        node = c0;
        nt = t0;
      }
      if (g + 1 < ngroups) next = sib[G - (int)__builtin_ctzll((unsigned long long)(g + 1)) - 1];
#endif
#if defined(PROBE_LVLVAR)
      const int lvl = (int)(g & 15);
#else
      const int lvl = k0 + G;
#endif
      Block4 c[2], q[4];
      uint32_t ct[2], qt[4];
      children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.cw_seed[lvl], lds.cw_ctrl[lvl], c[0],
                    ct[0], c[1], ct[1]);
      children_step_x2(lk, p.rkl.k, p.rkr.k, c[0], ct[0], c[1], ct[1], lds.cw_seed[lvl + 1],
                       lds.cw_ctrl[lvl + 1], q, qt);
      uint4* o = reinterpret_cast<uint4*>(p.out + (leaf_base + 8 * g) * 16);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        Block4 l[4];
        uint32_t lt[4];
        children_step_x2(lk, p.rkl.k, p.rkr.k, q[2 * hf], qt[2 * hf], q[2 * hf + 1],
                         qt[2 * hf + 1], lds.cw_seed[lvl + 2], lds.cw_ctrl[lvl + 2], l, lt);
#if defined(PROBE_NODFS)
        if (hf == 1) { next = l[3]; nextt = lt[3]; }
#endif
        dpf_aes::mmo_hashN<4>(l, lk, rv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#if defined(PROBE_NOCORRECT)
          const Block4 h = l[j];
          acc ^= lt[j];
#else
          const Block4 h = leaf.correct(l[j], lt[j]);
#endif
#if defined(PROBE_NOSTORE)
          acc ^= h.w0 ^ h.w1 ^ h.w2 ^ h.w3;
#else
          o[4 * hf + j] = make_uint4(h.w0, h.w1, h.w2, h.w3);
#endif
        }
      }
    }
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

}  // namespace

int num_cus_() {
  int c = 256;
  hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, 0);
  return c;
}

int main(int argc, char** argv) {
  const char* name = argc > 1 ? argv[1] : "probe";
  const int L = 29, S = 11, cus = num_cus_();
  ExpandParams p{};
  p.num_levels = L;
  p.S = S;
  p.k0 = L - S;
  p.num_items = (int64_t)1 << p.k0;
  dpf_block seed{0x243F6A8885A308D3ull, 0x13198A2E03707344ull};
  uint8_t ctrl = 1;
  dpf_block cws[L];
  uint8_t cl[L], cr[L];
  for (int i = 0; i < L; ++i) {
    cws[i] = dpf_block{0x9E3779B97F4A7C15ull * (i + 1), 0xC2B2AE3D27D4EB4Full * (i + 7)};
    cl[i] = i & 1;
    cr[i] = (i >> 1) & 1;
  }
  dpf_block* d_seed; uint8_t* d_ctrl; dpf_block* d_cw; uint8_t *d_cl, *d_cr; uint32_t* sink;
  CK(hipMalloc(&d_seed, 16)); CK(hipMalloc(&d_ctrl, 1)); CK(hipMalloc(&d_cw, sizeof cws));
  CK(hipMalloc(&d_cl, L)); CK(hipMalloc(&d_cr, L)); CK(hipMalloc(&sink, (size_t)cus * kBlock * 4));
  CK(hipMemcpy(d_seed, &seed, 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ctrl, &ctrl, 1, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_cw, cws, sizeof cws, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_cl, cl, L, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_cr, cr, L, hipMemcpyHostToDevice));
  char* out;
  CK(hipMalloc(&out, (size_t)16 << L));
  p.seeds_in = d_seed; p.ctrl_in = d_ctrl; p.cw_seed = d_cw; p.cw_left = d_cl; p.cw_right = d_cr;
  p.out = out;
  dpf_aes_key kl, kr, kv;
  for (int i = 0; i < 16; ++i) { kl.bytes[i] = i; kr.bytes[i] = 3 * i + 1; kv.bytes[i] = 7 * i + 2; }
  p.rkl = expand_key(&kl); p.rkr = expand_key(&kr); p.rkv = expand_key(&kv);
  p.rkd = p.rkl;
  for (int i = 0; i < 44; ++i) p.rkd.k[i] = p.rkl.k[i] ^ p.rkr.k[i];
  FastIntLeaf<64, false> leaf{nullptr, 1, 0, 16, {}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float best = 1e30f, sum = 0;
  const int reps = 6;
  for (int rep = 0; rep < reps; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(probe_kernel, dim3(cus), dim3(kBlock), 0, 0, p, leaf, sink);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) { sum += ms; if (ms < best) best = ms; }
  }
#if defined(PROBE_NODFS)
  const double aes = (double)p.num_items * (1 << (S - 3)) * 22;
#else
  const double aes = 2.0 * ((1ull << L) - 1) + (double)(1ull << L);
#endif
  printf("{\"probe\": \"%s\", \"best_ms\": %.3f, \"mean_ms\": %.3f, \"g_aes\": %.2f}\n", name, best,
         sum / (reps - 1), aes / best / 1e6);
  return 0;
}
