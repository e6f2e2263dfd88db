// EvaluateUntil's prefix dedup (csrc/host/host_util.h DedupTreeIndices;
// distributed_point_function.h:718-742): unique tree indices in first-seen
// order and, per prefix, (position of its tree index, block index) -- checked
// against a plain first-seen-order map for ascending inputs split over many
// chunks (the fused order + count pass), orders broken inside a chunk and
// exactly at a chunk boundary (hash-map path), random orders, and both
// position types; `ascending_out` reports which path ran.
#include <cstdio>
#include <map>
#include <random>
#include <utility>
#include <vector>

#include "host_util.h"

using distributed_point_functions::Span;
using distributed_point_functions::uint128;
using distributed_point_functions::dpf_internal::DedupTreeIndices;
using distributed_point_functions::dpf_internal::NumChunks;

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);  \
      ++failures;                                                 \
    }                                                             \
  } while (0)

template <typename Pos>
static void Check(const std::vector<uint128>& prefixes, int bib, bool want_ascending) {
  std::vector<uint128> want_ti;
  std::vector<std::pair<int64_t, int>> want_map;
  std::map<uint128, int64_t> seen;
  const uint128 bmask = (uint128{1} << bib) - 1;
  for (const uint128& p : prefixes) {
    auto [it, inserted] = seen.emplace(p >> bib, static_cast<int64_t>(want_ti.size()));
    if (inserted) want_ti.push_back(p >> bib);
    want_map.emplace_back(it->second, static_cast<int>(p & bmask));
  }
  // Outputs recycled from a larger earlier call must be overwritten, not appended to.
  std::vector<uint128> ti(prefixes.size() + 7, ~uint128{0});
  std::vector<std::pair<Pos, int>> map(prefixes.size() + 7, {Pos{-1}, -1});
  bool ascending = !want_ascending;
  DedupTreeIndices(Span<const uint128>(prefixes.data(), prefixes.size()), bib, &ti, &map,
                   &ascending);
  CHECK(ascending == want_ascending);
  CHECK(ti == want_ti);
  CHECK(map.size() == want_map.size());
  for (size_t i = 0; i < map.size() && i < want_map.size(); ++i)
    if (static_cast<int64_t>(map[i].first) != want_map[i].first ||
        map[i].second != want_map[i].second) {
      CHECK(false && "prefix map entry");
      break;
    }
}

int main() {
  std::mt19937_64 rng(7);
  const int64_t P = int64_t{1} << 18;   // 8 chunks of 2^15 with DPF_HOST_THREADS=8
  const int chunks = NumChunks(P);
  std::printf("chunks %d\n", chunks);
  // Ascending, several prefixes per tree index (bib 2), 128-bit values.
  std::vector<uint128> asc;
  uint128 x = (static_cast<uint128>(rng()) << 64) | rng();
  for (int64_t i = 0; i < P; ++i) {
    x += 1 + (rng() % 5);
    asc.push_back(x);
  }
  for (int bib : {0, 2, 5}) {
    Check<int64_t>(asc, bib, true);
    Check<int32_t>(asc, bib, true);
  }
  // Order broken exactly at a chunk boundary, and inside a chunk.
  if (chunks > 1) {
    std::vector<uint128> b = asc;
    const int64_t lo = P * 3 / chunks;
    std::swap(b[lo - 1], b[lo]);
    Check<int64_t>(b, 2, false);
    Check<int32_t>(b, 2, false);
  }
  {
    std::vector<uint128> b = asc;
    b[P / 2 + 3] = b[P / 2 + 2];   // equal neighbours: not strictly ascending
    Check<int64_t>(b, 2, false);
    std::vector<uint128> c = asc;
    std::swap(c[10], c[11]);
    Check<int32_t>(c, 0, false);
  }
  // Random order with repeats.
  std::vector<uint128> r;
  for (int64_t i = 0; i < 100000; ++i) r.push_back(rng() % 30000);
  Check<int64_t>(r, 1, false);
  Check<int32_t>(r, 3, false);
  // Tiny inputs.
  Check<int64_t>({uint128{5}}, 2, true);
  Check<int32_t>({uint128{9}, uint128{8}}, 0, false);
  std::vector<uint128> ti(3);
  std::vector<std::pair<int32_t, int>> map(3);
  bool asc_out = true;
  DedupTreeIndices(Span<const uint128>(), 2, &ti, &map, &asc_out);
  CHECK(ti.empty() && map.empty() && !asc_out);
  std::printf("%d failures\n", failures);
  return failures == 0 ? 0 : 1;
}
