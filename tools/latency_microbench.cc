// latency_microbench.cc -- fixed costs of one small device round trip on the
// box (what a 2^12-output EvaluateUntil pays besides its few microseconds of
// AES): kernel launch + stream sync, small H2D/D2H copies, events, and a
// kernel that reads its inputs from / writes its outputs to page-locked host
// memory directly.  Median of 200 repetitions, microseconds, one JSON line each.
//
//   tools/latency_microbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <vector>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

__global__ void empty_kernel() {}

// Reads n words and writes n words (one per thread).
__global__ void copy_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] * 3u + 1u;
}

static double median_us(const std::function<void()>& f) {
  std::vector<double> t;
  for (int i = 0; i < 20; ++i) f();
  for (int i = 0; i < 200; ++i) {
    auto a = std::chrono::steady_clock::now();
    f();
    auto b = std::chrono::steady_clock::now();
    t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

static void line(const char* what, double us) {
  printf("{\"what\": \"%s\", \"median_us\": %.2f}\n", what, us);
  fflush(stdout);
}

int main() {
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n = 1024;  // 4 KiB
  uint32_t *d_in, *d_out, *h_in, *h_out;
  CHECK(hipMalloc(&d_in, n * 4));
  CHECK(hipMalloc(&d_out, n * 4));
  CHECK(hipHostMalloc(&h_in, n * 4, hipHostMallocDefault));
  CHECK(hipHostMalloc(&h_out, n * 4, hipHostMallocDefault));
  std::vector<uint32_t> v(n, 7);
  for (int i = 0; i < n; ++i) h_in[i] = i;
  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));

  line("empty kernel launch + hipStreamSynchronize", median_us([&] {
         hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
         CHECK(hipStreamSynchronize(s));
       }));
  line("hipEventRecord + hipEventSynchronize (idle stream)", median_us([&] {
         CHECK(hipEventRecord(ev, s));
         CHECK(hipEventSynchronize(ev));
       }));
  line("H2D 4 KiB async from pinned + sync", median_us([&] {
         CHECK(hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, s));
         CHECK(hipStreamSynchronize(s));
       }));
  line("D2H 4 KiB async into pinned + sync", median_us([&] {
         CHECK(hipMemcpyAsync(h_out, d_out, n * 4, hipMemcpyDeviceToHost, s));
         CHECK(hipStreamSynchronize(s));
       }));
  line("H2D 4 KiB + kernel + D2H 4 KiB + sync (device staging)", median_us([&] {
         CHECK(hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, s));
         hipLaunchKernelGGL(copy_kernel, dim3(16), dim3(64), 0, s, d_in, d_out, n);
         CHECK(hipMemcpyAsync(h_out, d_out, n * 4, hipMemcpyDeviceToHost, s));
         CHECK(hipStreamSynchronize(s));
         memcpy(v.data(), h_out, n * 4);
       }));
  line("kernel reading and writing pinned host memory + sync (zero-copy)", median_us([&] {
         hipLaunchKernelGGL(copy_kernel, dim3(16), dim3(64), 0, s, h_in, h_out, n);
         CHECK(hipStreamSynchronize(s));
         memcpy(v.data(), h_out, n * 4);
       }));
  bool ok = true;
  for (int i = 0; i < n; ++i) ok = ok && v[i] == (uint32_t)i * 3u + 1u;
  printf("{\"zero_copy_result_ok\": %s}\n", ok ? "true" : "false");
  return ok ? 0 : 1;
}
