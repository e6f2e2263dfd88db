// fresh_output_microbench.cc -- the drop-in API's per-call host output cycle
// at mid sizes (VERDICT r3 "mid-size cliff"): every EvaluateUntil<T> call
// returns a FRESH std::vector<T> (dpf/distributed_point_function.h:790-821) that
// the caller destroys, so each call pays the allocation, first touch, the D2H
// copy and the unmap.  This times that cycle for 8..256 MiB under the
// strategies the library can choose between, median and max over 25 calls:
//   reg        hipHostRegister the fresh range, DMA straight in, unregister
//   reg+thp    the same with the range advised onto transparent huge pages
//   bounce     DMA into two page-locked 16 MiB buffers, memcpy on 8 threads
//   bounce+thp the same with huge pages advised
// Every variant value-initialises the vector chunk by chunk as the library's
// HostSink does (resize before each chunk lands).  One JSON line per case.
//
//   hipcc -O2 -std=c++17 tools/fresh_output_microbench.cc -o tools/fresh_output_microbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <malloc.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#define CHECK(x)                                                \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
      exit(1);                                                  \
    }                                                           \
  } while (0)

using clk = std::chrono::steady_clock;
static double secs(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

static void advise(void* p, size_t bytes) {
  const uintptr_t h = uintptr_t{2} << 20;
  uintptr_t lo = (reinterpret_cast<uintptr_t>(p) + h - 1) & ~(h - 1);
  uintptr_t hi = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(h - 1);
  if (hi > lo) madvise(reinterpret_cast<void*>(lo), hi - lo, MADV_HUGEPAGE);
}

static void pcopy(char* d, const char* s, size_t bytes, int threads) {
  if (threads <= 1 || bytes < (size_t{2} << 20)) {
    memcpy(d, s, bytes);
    return;
  }
  std::vector<std::thread> t;
  for (int i = 0; i < threads; ++i) {
    const size_t lo = bytes * i / threads, hi = bytes * (i + 1) / threads;
    t.emplace_back([=] { memcpy(d + lo, s + lo, hi - lo); });
  }
  for (auto& x : t) x.join();
}

constexpr size_t kChunk = size_t{16} << 20;

int main() {
  const size_t max_bytes = size_t{256} << 20;
  void* dev = nullptr;
  CHECK(hipMalloc(&dev, max_bytes));
  CHECK(hipMemset(dev, 0x5a, max_bytes));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  char* bounce[2];
  for (auto& b : bounce) CHECK(hipHostMalloc((void**)&b, kChunk, hipHostMallocDefault));
  CHECK(hipDeviceSynchronize());
  const char* names[] = {"reg", "reg+thp", "bounce", "bounce+thp", "bounce16", "reg_prefault",
                         "bounce+thp+prefault", "bounce+thp, malloc keeps pages"};
  for (size_t mib : {8, 16, 24, 32, 48, 64, 128, 256}) {
    const size_t bytes = mib << 20;
    for (int var = 0; var < 8; ++var) {
      const bool reg = var == 0 || var == 1 || var == 5, thp = var == 1 || var == 3 || var >= 6;
      // Variant 7: glibc serves large blocks from the heap and keeps freed
      // pages (no mmap/munmap per call): what the per-call cost is without
      // the allocator's fresh pages.
      if (var == 7) {
        mallopt(M_MMAP_MAX, 0);
        mallopt(M_TRIM_THRESHOLD, 1 << 30);
      }
      const int threads = var == 4 ? 16 : 8;
      std::vector<double> tot, t_alloc, t_copy, t_free;
      for (int it = 0; it < 27; ++it) {
        auto t0 = clk::now();
        auto* v = new std::vector<uint64_t>();
        v->reserve(bytes / 8);
        char* d = reinterpret_cast<char*>(v->data());
        if (thp) advise(d, bytes);
        if (var == 5 || var == 6) {
          std::vector<std::thread> t;
          for (int i = 0; i < 16; ++i) {
            const size_t lo = bytes * i / 16, hi = bytes * (i + 1) / 16;
            t.emplace_back([=] { for (size_t j = lo; j < hi; j += 4096) d[j] = 0; });
          }
          for (auto& x : t) x.join();
        }
        auto t1 = clk::now();
        if (reg) {
          CHECK(hipHostRegister(d, bytes, hipHostRegisterDefault));
          for (size_t off = 0; off < bytes; off += 4 * kChunk) {
            const size_t len = std::min(4 * kChunk, bytes - off);
            v->resize((off + len) / 8);
            CHECK(hipMemcpyAsync(d + off, (char*)dev + off, len, hipMemcpyDeviceToHost, st));
          }
          CHECK(hipStreamSynchronize(st));
          CHECK(hipHostUnregister(d));
        } else {
          const size_t n = (bytes + kChunk - 1) / kChunk;
          auto len = [&](size_t i) { return std::min(kChunk, bytes - i * kChunk); };
          CHECK(hipMemcpyAsync(bounce[0], dev, len(0), hipMemcpyDeviceToHost, st));
          for (size_t i = 0; i < n; ++i) {
            CHECK(hipStreamSynchronize(st));
            if (i + 1 < n)
              CHECK(hipMemcpyAsync(bounce[(i + 1) & 1], (char*)dev + (i + 1) * kChunk, len(i + 1),
                                   hipMemcpyDeviceToHost, st));
            v->resize((i * kChunk + len(i)) / 8);
            pcopy(d + i * kChunk, bounce[i & 1], len(i), threads);
          }
        }
        auto t2 = clk::now();
        if ((*v)[bytes / 8 - 1] != 0x5a5a5a5a5a5a5a5aull) {
          fprintf(stderr, "bad copy\n");
          return 1;
        }
        delete v;
        auto t3 = clk::now();
        if (it < 2) continue;
        t_alloc.push_back(secs(t0, t1));
        t_copy.push_back(secs(t1, t2));
        t_free.push_back(secs(t2, t3));
        tot.push_back(secs(t0, t3));
      }
      auto med = [](std::vector<double> x) {
        std::sort(x.begin(), x.end());
        return x[x.size() / 2] * 1e3;
      };
      auto mx = [](const std::vector<double>& x) { return *std::max_element(x.begin(), x.end()) * 1e3; };
      printf("{\"mib\": %zu, \"variant\": \"%s\", \"total_ms\": %.3f, \"max_ms\": %.3f, "
             "\"alloc_ms\": %.3f, \"copy_ms\": %.3f, \"free_ms\": %.3f, \"copy_max_ms\": %.3f, "
             "\"free_max_ms\": %.3f}\n",
             mib, names[var], med(tot), mx(tot), med(t_alloc), med(t_copy), med(t_free),
             mx(t_copy), mx(t_free));
      fflush(stdout);
      if (var == 7) {
        mallopt(M_MMAP_MAX, 65536);
        mallopt(M_TRIM_THRESHOLD, 128 * 1024);
      }
    }
  }
  return 0;
}
