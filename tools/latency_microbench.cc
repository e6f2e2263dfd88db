// latency_microbench.cc -- fixed costs of one small device round trip on the
// box (what a 2^12-output EvaluateUntil pays besides its few microseconds of
// AES): kernel launch + stream sync, small H2D/D2H copies, events, and a
// kernel that reads its inputs from / writes its outputs to page-locked host
// memory directly; and how the host learns a small launch is done: blocking
// stream sync, spinning on the launch's event, or spinning on a flag the
// kernel's last workgroup writes into page-locked memory.  Median of 200
// repetitions, microseconds, one JSON line each.
//
//   tools/latency_microbench [--spin]   (--spin: hipDeviceScheduleSpin first)
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

// The last workgroup to finish publishes `seq` to a page-locked flag (vector
// store at system scope after a system fence): the host may read everything
// the kernel wrote to page-locked memory once it sees the flag.
__global__ void flag_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int n,
                            unsigned int* done_count, unsigned int* flag, unsigned int seq) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] * 3u + seq;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int prev = atomicAdd(done_count, 1u);
    if (prev == gridDim.x - 1) {
      *done_count = 0u;
      __threadfence_system();
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Stream-ordered after the kernel whose completion it publishes.
__global__ void seq_copy_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int n,
                                unsigned int seq) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] * 3u + seq;
}
__global__ void publish_kernel(unsigned int* flag, unsigned int seq) {
  __threadfence_system();
  __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "--spin") == 0) CHECK(hipSetDeviceFlags(hipDeviceScheduleSpin));
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
  line("empty kernel launch only (host side of hipLaunchKernel)", median_us([&] {
         hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
       }));
  CHECK(hipStreamSynchronize(s));
  line("empty kernel + hipEventRecord + spin on hipEventQuery", median_us([&] {
         hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
         CHECK(hipEventRecord(ev, s));
         while (hipEventQuery(ev) == hipErrorNotReady) {
         }
       }));
  unsigned int *d_count, *h_flag;
  CHECK(hipMalloc(&d_count, 4));
  CHECK(hipMemset(d_count, 0, 4));
  CHECK(hipHostMalloc(&h_flag, 4, hipHostMallocDefault));
  *h_flag = 0;
  unsigned int seq = 0;
  long stale = 0;
  line("zero-copy kernel (16 workgroups) + spin on its page-locked done flag", median_us([&] {
         ++seq;
         hipLaunchKernelGGL(flag_kernel, dim3(16), dim3(64), 0, s, h_in, h_out, n, d_count, h_flag,
                            seq);
         while (__atomic_load_n(h_flag, __ATOMIC_ACQUIRE) != seq) {
         }
         memcpy(v.data(), h_out, n * 4);
         for (int i = 0; i < n; ++i) stale += v[i] != (uint32_t)i * 3u + seq;
       }));
  line("zero-copy kernel + a 1-thread publish kernel + spin on the page-locked flag", median_us([&] {
         ++seq;
         hipLaunchKernelGGL(seq_copy_kernel, dim3(16), dim3(64), 0, s, h_in, h_out, n, seq);
         hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(1), 0, s, h_flag, seq);
         while (__atomic_load_n(h_flag, __ATOMIC_ACQUIRE) != seq) {
         }
         memcpy(v.data(), h_out, n * 4);
         for (int i = 0; i < n; ++i) stale += v[i] != (uint32_t)i * 3u + seq;
       }));
  printf("{\"stale_words_after_flag\": %ld}\n", stale);
  CHECK(hipStreamSynchronize(s));
  line("zero-copy kernel (16 workgroups) + hipStreamSynchronize", median_us([&] {
         ++seq;
         hipLaunchKernelGGL(flag_kernel, dim3(16), dim3(64), 0, s, h_in, h_out, n, d_count, h_flag,
                            seq);
         CHECK(hipStreamSynchronize(s));
         memcpy(v.data(), h_out, n * 4);
       }));
  bool ok = stale == 0;
  for (int i = 0; i < n; ++i) ok = ok && v[i] == (uint32_t)i * 3u + seq;
  printf("{\"zero_copy_results_ok\": %s}\n", ok ? "true" : "false");
  return ok ? 0 : 1;
}
