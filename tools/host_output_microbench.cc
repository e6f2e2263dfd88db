// host_output_microbench.cc -- where the API-level EvaluateUntil<T> time goes
// when the result must land in a fresh host std::vector<T> (the reference's
// return type, dpf/distributed_point_function.h:790-821): page faults and the
// value-initialisation of the vector, the DMA rate from HBM, and the host copy
// out of page-locked staging.  Prints one JSON line per measurement.
//
//   tools/host_output_microbench [log2 bytes = 33]
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void advise(void* p, size_t bytes) {
  const uintptr_t h = uintptr_t{2} << 20;
  uintptr_t lo = (reinterpret_cast<uintptr_t>(p) + h - 1) & ~(h - 1);
  uintptr_t hi = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(h - 1);
  if (hi > lo) madvise(reinterpret_cast<void*>(lo), hi - lo, MADV_HUGEPAGE);
}

template <class F>
static void parallel(int threads, size_t bytes, F f) {
  std::vector<std::thread> t;
  for (int i = 0; i < threads; ++i) {
    const size_t lo = bytes * i / threads / 4096 * 4096, hi = i + 1 == threads ? bytes : bytes * (i + 1) / threads / 4096 * 4096;
    t.emplace_back([=] { f(lo, hi); });
  }
  for (auto& x : t) x.join();
}

static void line(const char* what, double s, size_t bytes, int threads) {
  printf("{\"what\": \"%s\", \"ms\": %.1f, \"gb_per_s\": %.2f, \"threads\": %d}\n", what, s * 1e3,
         bytes / s / 1e9, threads);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 33;
  const size_t bytes = size_t{1} << lg;
  const size_t n = bytes / 8;
  cpu_set_t cs;
  sched_getaffinity(0, sizeof(cs), &cs);
  int threads = CPU_COUNT(&cs);
  if (const char* o = getenv("OMP_NUM_THREADS")) threads = std::min(threads, atoi(o));
  if (threads > 16) threads = 16;
  void* dev = nullptr;
  CHECK(hipMalloc(&dev, bytes));
  CHECK(hipMemset(dev, 0x5a, bytes));
  CHECK(hipDeviceSynchronize());

  for (int rep = 0; rep < 2; ++rep) {
    // 1. std::vector<uint64_t>(n): value-initialisation on one thread, page faults included.
    double t0 = now();
    {
      std::vector<uint64_t> v;
      v.reserve(n);
      advise(v.data(), bytes);
      v.resize(n);
      line("vector resize (THP advised, serial zero-fill + faults)", now() - t0, bytes, 1);
      // 2. the same vector's pages are now mapped: memset again (serial, no faults).
      t0 = now();
      memset(v.data(), 1, bytes);
      line("memset of mapped vector (serial)", now() - t0, bytes, 1);
    }
    // 3. parallel pre-fault, then resize.
    t0 = now();
    {
      std::vector<uint64_t> v;
      v.reserve(n);
      advise(v.data(), bytes);
      char* p = reinterpret_cast<char*>(v.data());
      parallel(threads, bytes, [p](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; i += 4096) p[i] = 0;
      });
      const double t1 = now();
      line("parallel pre-fault", t1 - t0, bytes, threads);
      v.resize(n);
      line("resize after pre-fault", now() - t1, bytes, 1);
    }
    // 4. DMA into page-locked memory.
    void* pinned = nullptr;
    CHECK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
    t0 = now();
    CHECK(hipMemcpy(pinned, dev, bytes, hipMemcpyDeviceToHost));
    line("hipMemcpy D2H into hipHostMalloc memory", now() - t0, bytes, 1);
    // 5. parallel host copy pinned -> fresh vector (faults in parallel), and
    //    pinned -> mapped vector.
    {
      std::vector<uint64_t> v;
      v.reserve(n);
      advise(v.data(), bytes);
      char* d = reinterpret_cast<char*>(v.data());
      const char* s = reinterpret_cast<const char*>(pinned);
      t0 = now();
      parallel(threads, bytes, [=](size_t lo, size_t hi) { memcpy(d + lo, s + lo, hi - lo); });
      line("parallel memcpy pinned -> fresh memory", now() - t0, bytes, threads);
      t0 = now();
      parallel(threads, bytes, [=](size_t lo, size_t hi) { memcpy(d + lo, s + lo, hi - lo); });
      line("parallel memcpy pinned -> mapped memory", now() - t0, bytes, threads);
      // 6. hipHostRegister of the mapped vector, then DMA straight into it.
      t0 = now();
      CHECK(hipHostRegister(d, bytes, hipHostRegisterDefault));
      line("hipHostRegister of mapped memory", now() - t0, bytes, 1);
      t0 = now();
      CHECK(hipMemcpy(d, dev, bytes, hipMemcpyDeviceToHost));
      line("hipMemcpy D2H into registered memory", now() - t0, bytes, 1);
      t0 = now();
      CHECK(hipHostUnregister(d));
      line("hipHostUnregister", now() - t0, bytes, 1);
    }
    CHECK(hipHostFree(pinned));
  }
  CHECK(hipFree(dev));
  return 0;
}
