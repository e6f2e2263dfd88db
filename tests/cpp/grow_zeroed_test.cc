// GrowZeroed (include/dpf/internal/value_type_helpers.h): growing a host
// result vector by memmove from the zero page must equal resize() -- the new
// elements value-initialised, the old ones kept -- across the 64 MiB span of
// ZeroPages(), for integer, uint128 and non-integer element types, and
// through VectorSink's grow()/chunk() as the D2H copies call them.
#include <cstdio>
#include <cstring>
#include <vector>

#include "dpf/internal/value_type_helpers.h"

using namespace distributed_point_functions;
using namespace distributed_point_functions::dpf_internal;

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);  \
      ++failures;                                                 \
    }                                                             \
  } while (0)

template <typename T>
void Grow(size_t first, size_t n) {
  std::vector<T> v(first);
  for (size_t i = 0; i < first; ++i) v[i] = static_cast<T>(i * 7 + 1);
  v.reserve(n);
  GrowZeroed(&v, n);
  CHECK(v.size() == n);
  bool ok = true;
  for (size_t i = 0; i < n && ok; ++i) ok = v[i] == (i < first ? static_cast<T>(i * 7 + 1) : T{});
  CHECK(ok);
}

int main() {
  size_t span = 0;
  const void* z = ZeroPages(&span);
  CHECK(z != nullptr && span == (size_t{64} << 20));
  const size_t per128 = span / 16;
  Grow<uint128>(0, 0);
  Grow<uint128>(0, 1);
  Grow<uint128>(3, 1000);
  Grow<uint128>(5, per128 + 17);       // crosses the span: two inserts
  Grow<uint64_t>(1, 2 * (span / 8) + 3);
  Grow<uint8_t>(0, 4097);
  Grow<uint32_t>(10, 10);               // no growth
  {
    std::vector<uint64_t> v(100, 5);
    GrowZeroed(&v, 40);                 // shrinking falls back to resize()
    CHECK(v.size() == 40 && v[39] == 5);
  }
  {
    std::vector<uint128> v;             // no reserve: insert reallocates
    GrowZeroed(&v, 12345);
    CHECK(v.size() == 12345 && v[12344] == 0);
  }
  {
    using T = Tuple<uint32_t, uint64_t>;  // not an integer: resize()
    std::vector<T> v;
    GrowZeroed(&v, 77);
    CHECK(v.size() == 77 && std::get<1>(v[76].value()) == 0);
  }
  {
    // VectorSink: grow() ahead of each DMA chunk, chunk() from staging.
    std::vector<uint128> out;
    const HostSink s = VectorSink(&out);
    uint8_t* dst = static_cast<uint8_t*>(s.reserve(16 * 1000));
    CHECK(dst == reinterpret_cast<uint8_t*>(out.data()));
    s.grow(16 * 500);
    CHECK(out.size() == 500);
    std::vector<uint8_t> src(16 * 500, 0xab);
    s.chunk(src.data(), 16 * 500, 16 * 500);
    CHECK(out.size() == 1000 && out[499] == 0 && (out[999] & 0xff) == 0xab);
  }
  std::printf("%d failures\n", failures);
  return failures != 0;
}
