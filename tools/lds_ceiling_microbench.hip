// lds_ceiling_microbench.hip -- the practical ceiling of conflict-free random
// ds_read_b32 lookups on one MI355X, in the T-table layout of dpf_device.h
// (4 tables x 256 entries x 32 bank copies, lane l reads copy l & 31, one
// v_perm_b32 per address), with as little VALU per lookup as possible:
// per lookup one v_perm (address), one ds_read_b32, one XOR into the chain.
// CH independent chains per lane, one 1024-thread workgroup per CU (the
// expand kernel's shape).  Reports lane-lookups per clock per CU at the clock
// measured in-kernel (s_memtime / s_memrealtime at 100 MHz).
// DYN = 1 (r16): the same lookups, but each wave takes its iterations in
// chunks of 64 from an LDS counter instead of a fixed 1/16 of the
// workgroup's: the CU's arbiter favours its oldest waves, so with fixed
// shares the last part of the launch runs on fewer and fewer waves (the
// r11 figure of 26.3 lane-lookups per clock measured that tail too).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lds_ceiling_microbench.hip -o tools/ldsc
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

// MODE 0: the T-table layout (32 copies, lane l -> copy l & 31, v_perm address).
// MODE 1: 64 copies of one table, lane l -> copy l (lanes 32-63 on the other
//         32 banks of the 64-bank array), v_perm address.
// MODE 2: as 0 but ds_read_b64 (8-byte entries): instruction rate for 8 B/lane.
template <int CH, int MODE, int DYN>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4)))
void lds_kernel(int iters, uint32_t* out, unsigned long long* clk) {
  __shared__ uint32_t tab[4 * 256 * 32];
  __shared__ int next;
  for (int i = threadIdx.x; i < 4 * 256 * 32; i += blockDim.x) tab[i] = i * 2654435761u;
  if (threadIdx.x == 0) next = 0;
  __syncthreads();
  const uint32_t l = MODE == 1 ? (threadIdx.x & 63) * 4u : (MODE == 2 ? (threadIdx.x & 31) * 8u
                                                                      : (threadIdx.x & 31) * 4u);
  const char* base = reinterpret_cast<const char*>(tab);
  uint32_t x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = (threadIdx.x * 2654435761u) ^ (c * 0x9e3779b9u);
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  // DYN: the workgroup's 16 * iters iterations in chunks of 64, taken per wave.
  const int chunks = DYN ? (blockDim.x / 64) * iters / 64 : 1;
  for (int ch = 0;;) {
    int lo = 0, hi = iters;
    if (DYN) {
      int c0 = 0;
      if ((threadIdx.x & 63) == 0) c0 = atomicAdd(&next, 1);
      ch = __builtin_amdgcn_readfirstlane(c0);
      if (ch >= chunks) break;
      lo = 0;
      hi = 64;
    } else if (ch++ > 0) {
      break;
    }
  for (int it = lo; it < hi; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      // byte 2 of x as the entry, table T0 (low 64 KiB), copy l & 31
      if (MODE == 0) {
        const uint32_t off = __builtin_amdgcn_perm(x[c], l, 0x0c020600u);
        x[c] ^= *reinterpret_cast<const uint32_t*>(base + off);
      } else if (MODE == 1) {
        // 64 copies x 4 B = 256-byte rows: entry in bits 8-15 (128 rows: 32 KiB... x 2)
        const uint32_t off = __builtin_amdgcn_perm(x[c], l, 0x0c020600u) & 0xffffu;
        x[c] ^= *reinterpret_cast<const uint32_t*>(base + off);
      } else {
        // 32 copies x 8 B = 256-byte rows
        const uint32_t off = __builtin_amdgcn_perm(x[c], l, 0x0c020600u) & 0xfff8u;
        const uint2 v = *reinterpret_cast<const uint2*>(base + off);
        x[c] ^= v.x ^ v.y;
      }
    }
  }
  }
  uint32_t a = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) a ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
  if (threadIdx.x == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int CH, int MODE, int DYN>
void run(int cus) {
  uint32_t* d;
  unsigned long long* c;
  CK(hipMalloc(&d, (size_t)cus * 1024 * 4));
  CK(hipMalloc(&c, (size_t)cus * 16));
  const int iters = 4096 / CH * 16;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 4; ++r) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((lds_kernel<CH, MODE, DYN>), dim3(cus), dim3(1024), 0, 0, iters, d, c);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r && ms < best) best = ms;
  }
  unsigned long long h[2];
  CK(hipMemcpy(h, c, 16, hipMemcpyDeviceToHost));
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
  const double lookups = (double)cus * 1024 * iters * CH;
  const double per_s = lookups / (best * 1e-3);
  printf("{\"mode\": %d, \"dynamic\": %d, \"chains\": %d, \"ms\": %.3f, \"t_lookups_per_s\": %.2f, \"clock_ghz\": %.3f, "
         "\"lane_lookups_per_clk_per_cu\": %.2f}\n", MODE, DYN, CH, best, per_s / 1e12, ghz,
         per_s / cus / (ghz * 1e9));
  CK(hipFree(d));
  CK(hipFree(c));
}

int main() {
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  run<4, 0, 0>(cus);
  run<8, 0, 0>(cus);
  run<16, 0, 0>(cus);
  run<4, 0, 1>(cus);
  run<8, 0, 1>(cus);
  run<16, 0, 1>(cus);
  run<8, 1, 0>(cus);
  run<8, 1, 1>(cus);
  run<8, 2, 0>(cus);
  run<8, 2, 1>(cus);
  return 0;
}
