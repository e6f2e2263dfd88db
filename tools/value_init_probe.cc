// How fast can one thread value-initialise a fresh std::vector of 16-byte
// elements?  Config 3's API-level call (2^31 uint128 -> host std::vector,
// 32 GiB) is bound by the resize() that value-initialises the result: the
// vector is the reference's return type (distributed_point_function.h:817-821),
// and only its own thread may construct its elements.  This probe times, on a
// range that is already mapped (prefaulted on 16 threads, as the library does
// before the DMA):
//   resize64   std::vector<U128>::resize in 64 MiB steps (the library's grow()
//              up to r15: libstdc++'s value-initialisation loop)
//   zero64     the same growth by insert() from a read-only mapping of the
//              zero page (the library's GrowZeroed(): a memmove per step)
//   memset     one memset of the whole range (glibc's large-size path)
//   memset16   the same range zeroed by 16 threads (what a vector cannot do)
// Build: g++ -O2 -pthread tools/value_init_probe.cc -o /tmp/value_init_probe
// Run:   /tmp/value_init_probe [GiB=32] [reps=3]   (one JSON line per rep)
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <thread>
#include <vector>

struct U128 {
  uint64_t lo, hi;
  U128() = default;   // trivial, so value-initialisation zeroes (like absl::uint128)
};

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void parallel(char* p, size_t bytes, int threads, int value) {
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([=] {
      const size_t lo = bytes * t / threads, hi = bytes * (t + 1) / threads;
      std::memset(p + lo, value, hi - lo);
    });
  for (auto& t : ts) t.join();
}

int main(int argc, char** argv) {
  const size_t gib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 32;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
  const size_t bytes = gib << 30, n = bytes / sizeof(U128);
  const size_t step = (size_t{64} << 20) / sizeof(U128);
  const U128* zeros = static_cast<const U128*>(
      mmap(nullptr, step * sizeof(U128), PROT_READ, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0));
  if (zeros == MAP_FAILED) return 1;
  for (int r = 0; r < reps; ++r) {
    std::vector<U128> v;
    v.reserve(n);
    char* p = reinterpret_cast<char*>(v.data());
    double t0 = now();
    parallel(p, bytes, 16, 1);   // map the pages (prefault)
    const double prefault = now() - t0;
    t0 = now();
    for (size_t k = 0; k < n; k += step) v.resize(k + step < n ? k + step : n);
    const double resize = now() - t0;
    std::vector<U128> w;
    w.reserve(n);
    parallel(reinterpret_cast<char*>(w.data()), bytes, 16, 1);
    t0 = now();
    for (size_t k = 0; k < n; k += step) {
      const size_t add = k + step < n ? step : n - k;
      w.insert(w.end(), zeros, zeros + add);
    }
    const double zero = now() - t0;
    w = std::vector<U128>();
    t0 = now();
    std::memset(p, 0, bytes);
    const double ms = now() - t0;
    t0 = now();
    parallel(p, bytes, 16, 0);
    const double ms16 = now() - t0;
    std::printf("{\"gib\": %zu, \"rep\": %d, \"prefault16_s\": %.3f, \"resize64_s\": %.3f, "
                "\"resize64_gb_s\": %.1f, \"zero64_s\": %.3f, \"zero64_gb_s\": %.1f, \"memset_s\": %.3f, \"memset_gb_s\": %.1f, "
                "\"memset16_s\": %.3f, \"memset16_gb_s\": %.1f}\n",
                gib, r, prefault, resize, bytes / resize / 1e9, zero, bytes / zero / 1e9, ms, bytes / ms / 1e9, ms16,
                bytes / ms16 / 1e9);
    std::fflush(stdout);
  }
  return 0;
}
