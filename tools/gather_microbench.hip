// gather_microbench.hip -- lookup rate of a 4 KiB table (one AES T-table set,
// 4 x 256 x 4 B) read with per-lane random addresses through the vector L1
// (global_load_dword), against the same lookups from LDS (ds_read_b32, the
// 32x bank-replicated layout of dpf_device.h).  Question: is the vector
// memory path a usable second lookup engine beside the LDS T-table?
// Each lane runs CH independent chains (index of the next lookup = bits of
// the previous result), so throughput with CH loads in flight per lane.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_microbench.hip -o tools/gmb
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

template <int CH>
__global__ __launch_bounds__(1024) void gather_global(const uint32_t* __restrict__ tab, int iters,
                                                      uint32_t* out) {
  uint32_t x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = (threadIdx.x * 2654435761u + c * 40503u) >> 5;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = tab[(x[c] ^ (it + c)) & 1023] + threadIdx.x;
  }
  uint32_t a = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) a ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

template <int CH>
__global__ __launch_bounds__(1024) void gather_lds(const uint32_t* __restrict__ tab, int iters,
                                                   uint32_t* out) {
  __shared__ uint32_t t[256 * 32 * 4];  // 4 tables x 256 entries x 32 copies
  for (int i = threadIdx.x; i < 256 * 32 * 4; i += blockDim.x) t[i] = tab[(i >> 5) & 1023];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 31;
  uint32_t x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = (threadIdx.x * 2654435761u + c * 40503u) >> 5;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = t[(((x[c] ^ (it + c)) & 1023) << 5) | lane] + threadIdx.x;
  }
  uint32_t a = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) a ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

template <class F>
float timeit(F f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 4; ++r) {
    CK(hipEventRecord(a));
    f();
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r && ms < best) best = ms;
  }
  return best;
}

int main() {
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = i * 2654435761u;
  uint32_t *tab, *out;
  CK(hipMalloc(&tab, sizeof h));
  CK(hipMemcpy(tab, h, sizeof h, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)cus * 1024 * 4));
  const int iters = 2000;
  const double lookups = (double)cus * 1024 * iters;
  float g4 = timeit([&] { gather_global<4><<<cus, 1024>>>(tab, iters, out); });
  float g8 = timeit([&] { gather_global<8><<<cus, 1024>>>(tab, iters, out); });
  float l4 = timeit([&] { gather_lds<4><<<cus, 1024>>>(tab, iters, out); });
  float l8 = timeit([&] { gather_lds<8><<<cus, 1024>>>(tab, iters, out); });
  printf("{\"global_ch4_glookups\": %.1f, \"global_ch8_glookups\": %.1f, \"lds_ch4_glookups\": %.1f, "
         "\"lds_ch8_glookups\": %.1f}\n", lookups * 4 / g4 / 1e6, lookups * 8 / g8 / 1e6,
         lookups * 4 / l4 / 1e6, lookups * 8 / l8 / 1e6);
  return 0;
}
