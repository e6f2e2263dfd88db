// dpf_benchmark.cc -- the reference's benchmark suite
// (dpf/distributed_point_function_benchmark.cc, and BM_EvaluateDcf of
// dcf/distributed_comparison_function_benchmark.cc) restated against this build's
// drop-in C++ API: same benchmark names, value types and argument ranges, the
// same API calls in the timed loops, so a user of the reference can compare
// numbers case by case.  Evaluation runs on the GPU through the C ABI; key
// generation (BM_KeyGeneration) stays on the CPU, as in the north star.
//
// The reference's harness is google-benchmark, which is not in this image; a
// small runner below keeps its conventions: --benchmark_filter=<regex>,
// --benchmark_min_time=<seconds>, the "BM_Name<T>/arg" naming and one
// "name  time  iterations" row per case.  --json=<path> also writes the rows
// as JSON.
//
//   g++ -O2 -std=c++20 -Iinclude tools/dpf_benchmark.cc -Ldistributed_point_functions_amd/lib -ldpf
//   (built by distributed_point_functions_amd/build_native.py)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <malloc.h>
#include <functional>
#include <numeric>
#include <random>
#include <regex>
#include <set>
#include <string>
#include <vector>

#include "dcf/distributed_comparison_function.h"
#include "dpf/distributed_point_function.h"
#include "dpf/int_mod_n.h"
#include "dpf/tuple.h"
#include "dpf/xor_wrapper.h"

namespace dpf = distributed_point_functions;
using dpf::DistributedPointFunction;
using dpf::DpfKey;
using dpf::DpfParameters;
using dpf::EvaluationContext;
using dpf::IntModN;
using dpf::Tuple;
using dpf::uint128;
using dpf::XorWrapper;

namespace {

// ---------------------------------------------------------------------------
// Runner (google-benchmark conventions, minimal)
// ---------------------------------------------------------------------------
struct Row {
  std::string name;
  double ns_per_iter;
  int64_t iterations;
  std::string label;
};

struct Runner {
  std::regex filter{".*"};
  double min_time = 0.2;
  bool split = false;   // --split: per-phase times of BM_EvaluateRegularDpf instead
  std::vector<Row> rows;

  // `body(n)` runs n timed iterations; `label` is printed after the time.
  void Run(const std::string& name, const std::function<void(int64_t)>& body,
           const std::function<std::string(double)>& label = nullptr) {
    if (!std::regex_search(name, filter)) return;
    using clk = std::chrono::steady_clock;
    body(1);  // untimed: first-call costs (device init, buffer growth)
    int64_t n = 1;
    double secs = 0;
    for (;;) {
      auto t0 = clk::now();
      body(n);
      secs = std::chrono::duration<double>(clk::now() - t0).count();
      if (secs >= min_time || n >= (int64_t{1} << 30)) break;
      // Grow like google-benchmark: aim 40% past min_time, at most 10x per step.
      double want = secs > 0 ? min_time * 1.4 / secs * static_cast<double>(n) : n * 10.0;
      n = std::max<int64_t>(n + 1, std::min<int64_t>(n * 10, static_cast<int64_t>(want)));
    }
    Row r{name, secs * 1e9 / static_cast<double>(n), n, label ? label(secs / n) : ""};
    std::printf("%-72s %14.0f ns %10lld %s\n", r.name.c_str(), r.ns_per_iter,
                static_cast<long long>(r.iterations), r.label.c_str());
    std::fflush(stdout);
    rows.push_back(r);
  }
};

template <typename T>
volatile size_t g_sink;

template <typename T>
void Sink(const std::vector<T>& v) {
  g_sink<T> = v.size();
}

template <typename T>
T Must(dpf::StatusOr<T> s, const char* what) {
  if (!s.ok()) {
    std::fprintf(stderr, "%s: %s\n", what, s.status().ToString().c_str());
    std::exit(1);
  }
  return std::move(s).value();
}

void Must(const dpf::Status& s, const char* what) {
  if (!s.ok()) {
    std::fprintf(stderr, "%s: %s\n", what, s.ToString().c_str());
    std::exit(1);
  }
}

std::string Rate(double items, const char* unit, double secs) {
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.3g %s/s", items / secs, unit);
  return buf;
}

// --split: where one EvaluateNext<T>({}) call's time goes on the host, median
// of 30 calls: the context copy, the packed evaluation (kernel + D2H into a
// fresh byte vector), the unpack into a fresh std::vector<T>, and freeing both;
// and the whole EvaluateNext<T> call as the benchmark makes it.
template <typename T>
void SplitPhases(const DistributedPointFunction& f, const EvaluationContext& ctx0,
                 const std::string& name) {
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  const std::vector<uint128> none;
  const dpf::ValueType t = dpf::ToValueType<T>();
  constexpr int kReps = 30;
  std::vector<double> ph[5];
  for (int i = 0; i < kReps + 2; ++i) {
    auto t0 = clk::now();
    EvaluationContext ctx = ctx0;
    auto t1 = clk::now();
    std::vector<uint8_t> packed = Must(f.EvaluateUntilPacked(0, none, ctx, &t), "packed");
    auto t2 = clk::now();
    std::vector<T> out = dpf::dpf_internal::UnpackElements<T>(
        f.flat_value_type(0), packed.data(), static_cast<int64_t>(packed.size() /
                                                               f.flat_value_type(0).packed_size));
    auto t3 = clk::now();
    Sink(out);
    { std::vector<uint8_t>().swap(packed); std::vector<T>().swap(out); }
    auto t4 = clk::now();
    EvaluationContext ctx2 = ctx0;
    Sink(Must(f.template EvaluateNext<T>(none, ctx2), "EvaluateNext"));
    auto t5 = clk::now();
    if (i < 2) continue;
    ph[0].push_back(secs(t0, t1));
    ph[1].push_back(secs(t1, t2));
    ph[2].push_back(secs(t2, t3));
    ph[3].push_back(secs(t3, t4));
    ph[4].push_back(secs(t4, t5));
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2] * 1e3;
  };
  auto mx = [](const std::vector<double>& v) { return *std::max_element(v.begin(), v.end()) * 1e3; };
  std::printf("%-72s ctx %.3f  packed %.3f  unpack %.3f  free %.3f  | EvaluateNext %.3f "
              "(max %.3f) ms\n", name.c_str(), med(ph[0]), med(ph[1]), med(ph[2]), med(ph[3]),
              med(ph[4]), mx(ph[4]));
  std::fflush(stdout);
}

// ---------------------------------------------------------------------------
// BM_EvaluateRegularDpf<T>/log: EvaluateNext<T>({}) on a fresh copy of a
// single-level context (reference benchmark.cc:27-49), alpha = 0, beta = T{}.
// ---------------------------------------------------------------------------
template <typename T>
void EvaluateRegularDpf(Runner& r, const std::string& tname, int lo, int hi) {
  for (int log = lo; log <= hi; log += 2) {
    const std::string name = "BM_EvaluateRegularDpf<" + tname + ">/" + std::to_string(log);
    if (!std::regex_search(name, r.filter)) continue;
    DpfParameters p;
    p.set_log_domain_size(log);
    *p.mutable_value_type() = dpf::ToValueType<T>();
    auto f = Must(DistributedPointFunction::Create(p), "Create");
    Must(f->template RegisterValueType<T>(), "RegisterValueType");
    auto keys = Must(f->GenerateKeys(uint128{0}, T{}), "GenerateKeys");
    const EvaluationContext ctx0 = Must(f->CreateEvaluationContext(keys.first), "ctx");
    const std::vector<uint128> none;
    if (r.split) {
      SplitPhases<T>(*f, ctx0, name);
      continue;
    }
    r.Run(name, [&](int64_t n) {
      for (int64_t i = 0; i < n; ++i) {
        EvaluationContext ctx = ctx0;
        Sink(Must(f->template EvaluateNext<T>(none, ctx), "EvaluateNext"));
      }
    }, [&](double s) { return Rate(std::ldexp(1.0, log), "outputs", s); });
  }
}

// ---------------------------------------------------------------------------
// BM_EvaluateHierarchicalFull<T>/levels: `levels` hierarchy levels up to 2^20,
// every prefix of the previous level evaluated (benchmark.cc:84-131).
// ---------------------------------------------------------------------------
template <typename T>
void EvaluateHierarchicalFull(Runner& r, const std::string& tname) {
  constexpr int kMaxLog = 20;
  for (int levels = 1; levels <= 16; levels += 2) {
    const std::string name =
        "BM_EvaluateHierarchicalFull<" + tname + ">/" + std::to_string(levels);
    if (!std::regex_search(name, r.filter)) continue;
    std::vector<DpfParameters> ps(levels);
    for (int i = 0; i < levels; ++i) {
      ps[i].set_log_domain_size(
          static_cast<int>(static_cast<double>(i + 1) / levels * kMaxLog));
      ps[i].mutable_value_type()->mutable_integer()->set_bitsize(sizeof(T) * 8);
    }
    auto f = Must(DistributedPointFunction::CreateIncremental(ps), "CreateIncremental");
    std::vector<uint128> beta(levels);
    for (int i = 0; i < levels; ++i) beta[i] = i;
    auto keys = Must(f->GenerateKeysIncremental(uint128{12345}, beta), "GenerateKeysIncremental");
    const EvaluationContext ctx0 = Must(f->CreateEvaluationContext(keys.first), "ctx");
    std::vector<std::vector<uint128>> prefixes(levels);
    for (int i = 1; i < levels; ++i) {
      prefixes[i].resize(size_t{1} << ps[i - 1].log_domain_size());
      std::iota(prefixes[i].begin(), prefixes[i].end(), uint128{0});
    }
    r.Run(name, [&](int64_t n) {
      for (int64_t it = 0; it < n; ++it) {
        EvaluationContext ctx = ctx0;
        for (int i = 0; i < levels; ++i)
          Sink(Must(f->template EvaluateNext<T>(prefixes[i], ctx), "EvaluateNext"));
      }
    });
  }
}

// Random prefixes extending random parents (benchmark.cc:138-173), seeded.
std::vector<std::vector<uint128>> RandomPrefixes(const std::vector<DpfParameters>& ps,
                                                 const std::vector<int>& nonzeros,
                                                 uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::vector<std::vector<uint128>> out(ps.size());
  for (size_t i = 1; i < ps.size(); ++i) {
    int shift = ps[i - 1].log_domain_size() - (i > 1 ? ps[i - 2].log_domain_size() : 0);
    out[i].resize(nonzeros[i - 1]);
    for (auto& x : out[i]) {
      uint128 parent = i > 1 ? out[i - 1][rng() % out[i - 1].size()] << shift : 0;
      x = parent | (rng() & ((uint64_t{1} << shift) - 1));
    }
    std::sort(out[i].begin(), out[i].end());
  }
  return out;
}

// BM_IsrgExampleHierarchy: levels {12, 25}, uint32, 32 random prefixes
// (benchmark.cc:175-222).
void IsrgExampleHierarchy(Runner& r) {
  const std::string name = "BM_IsrgExampleHierarchy";
  if (!std::regex_search(name, r.filter)) return;
  std::vector<DpfParameters> ps(2);
  ps[0].set_log_domain_size(12);
  ps[1].set_log_domain_size(25);
  for (auto& p : ps) p.mutable_value_type()->mutable_integer()->set_bitsize(32);
  auto f = Must(DistributedPointFunction::CreateIncremental(ps), "CreateIncremental");
  auto keys = Must(f->GenerateKeysIncremental(uint128{1234567}, std::vector<uint128>(2, 1)),
                   "GenerateKeysIncremental");
  auto prefixes = RandomPrefixes(ps, {32}, 0x15A6);
  const EvaluationContext ctx0 = Must(f->CreateEvaluationContext(keys.first), "ctx");
  r.Run(name, [&](int64_t n) {
    for (int64_t it = 0; it < n; ++it) {
      EvaluationContext ctx = ctx0;
      for (int i = 0; i < 2; ++i)
        Sink(Must(f->EvaluateNext<uint32_t>(prefixes[i], ctx), "EvaluateNext"));
    }
  });
}

// BM_KeyGeneration<direct>/log (benchmark.cc:224-260): CPU keygen, random alpha.
template <bool kDirect>
void KeyGeneration(Runner& r) {
  for (int log = 1; log <= 128; log *= 2) {
    const std::string name = std::string("BM_KeyGeneration<") + (kDirect ? "true" : "false") +
                             ">/" + std::to_string(log);
    if (!std::regex_search(name, r.filter)) continue;
    std::vector<DpfParameters> ps(kDirect ? 1 : log);
    for (size_t i = 0; i < ps.size(); ++i) {
      ps[i].set_log_domain_size(kDirect ? log : static_cast<int>(i) + 1);
      ps[i].mutable_value_type()->mutable_integer()->set_bitsize(32);
    }
    auto f = Must(DistributedPointFunction::CreateIncremental(ps), "CreateIncremental");
    std::vector<uint128> beta(ps.size(), 23);
    const uint128 mask = log >= 128 ? dpf::Uint128Max() : (uint128{1} << log) - 1;
    std::mt19937_64 rng(log);
    size_t key_size = 0;
    r.Run(name, [&](int64_t n) {
      for (int64_t it = 0; it < n; ++it) {
        uint128 alpha = dpf::MakeUint128(rng(), rng()) & mask;
        auto keys = Must(f->GenerateKeysIncremental(alpha, beta), "GenerateKeysIncremental");
        key_size = keys.first.SerializeAsString().size();
      }
    }, [&](double) { return "key_size: " + std::to_string(key_size); });
  }
}

// BM_HeavyHitters/levels: one level per bit, uint64, 10000 uniform non-zeros
// at the last level and their prefixes above (benchmark.cc:262-340).
void HeavyHitters(Runner& r) {
  constexpr int kNonzeros = 10000;
  for (int levels = 16; levels <= 128; levels *= 2) {
    const std::string name = "BM_HeavyHitters/" + std::to_string(levels);
    if (!std::regex_search(name, r.filter)) continue;
    std::vector<DpfParameters> ps(levels);
    for (int i = 0; i < levels; ++i) {
      ps[i].set_log_domain_size(i + 1);
      ps[i].mutable_value_type()->mutable_integer()->set_bitsize(64);
    }
    auto f = Must(DistributedPointFunction::CreateIncremental(ps), "CreateIncremental");
    auto keys = Must(f->GenerateKeysIncremental(uint128{42}, std::vector<uint128>(levels, 23)),
                     "GenerateKeysIncremental");
    // Uniform non-zeros over the second-to-last level's domain, then their
    // prefixes level by level (GenerateUniformPrefixes, benchmark.cc:262-302).
    std::mt19937_64 rng(levels);
    std::vector<std::vector<uint128>> prefixes(levels);
    {
      const int top = ps[levels - 2].log_domain_size();
      const uint128 mask = top >= 128 ? dpf::Uint128Max() : (uint128{1} << top) - 1;
      std::set<uint128> last;
      while (static_cast<int>(last.size()) < kNonzeros)
        last.insert(dpf::MakeUint128(rng(), rng()) & mask);
      prefixes[levels - 1].assign(last.begin(), last.end());
      for (int i = levels - 1; i > 1; --i) {
        std::vector<uint128>& cur = prefixes[i - 1];
        for (uint128 x : prefixes[i]) {
          uint128 p = x >> 1;
          if (cur.empty() || cur.back() != p) cur.push_back(p);
        }
      }
    }
    const EvaluationContext ctx0 = Must(f->CreateEvaluationContext(keys.first), "ctx");
    r.Run(name, [&](int64_t n) {
      for (int64_t it = 0; it < n; ++it) {
        EvaluationContext ctx = ctx0;
        for (int i = 0; i < levels; ++i)
          Sink(Must(f->EvaluateNext<uint64_t>(prefixes[i], ctx), "EvaluateNext"));
      }
    });
  }
}

// BM_BatchEvaluation<XorWrapper<uint128>>/keys/points: EvaluateAt per key on
// a 2^56 domain (benchmark.cc:342-402).
void BatchEvaluation(Runner& r) {
  using T = XorWrapper<uint128>;
  constexpr int kLog = 63 - 7;
  const std::pair<int, int> cases[] = {{1, 400000}, {10, 40000}, {100, 4000}};
  for (auto [num_keys, ppk] : cases) {
    const std::string name = "BM_BatchEvaluation<XorWrapper<uint128>>/" +
                             std::to_string(num_keys) + "/" + std::to_string(ppk);
    if (!std::regex_search(name, r.filter)) continue;
    DpfParameters p;
    p.set_log_domain_size(kLog);
    *p.mutable_value_type() = dpf::ToValueType<T>();
    auto f = Must(DistributedPointFunction::Create(p), "Create");
    Must(f->RegisterValueType<T>(), "RegisterValueType");
    const uint128 mask = (uint128{1} << kLog) - 1;
    std::mt19937_64 rng(num_keys);
    std::vector<DpfKey> keys;
    std::vector<uint128> points(static_cast<size_t>(num_keys) * ppk);
    for (int i = 0; i < num_keys; ++i) {
      keys.push_back(
          Must(f->GenerateKeys(dpf::MakeUint128(rng(), rng()) & mask, T{}), "GenerateKeys").first);
      for (int j = 0; j < ppk; ++j) points[size_t(i) * ppk + j] = dpf::MakeUint128(rng(), rng()) & mask;
    }
    r.Run(name, [&](int64_t n) {
      for (int64_t it = 0; it < n; ++it)
        for (int i = 0; i < num_keys; ++i)
          Sink(Must(f->EvaluateAt<T>(keys[i], 0,
                                     dpf::MakeConstSpan(points.data() + size_t(i) * ppk, ppk)),
                    "EvaluateAt"));
    }, [&](double s) { return Rate(double(num_keys) * ppk, "points", s); });
  }
}

// BM_EvaluateDcf<T>/log: one Evaluate<T>(key, x) per iteration, x counting up
// (dcf/distributed_comparison_function_benchmark.cc:24-54), beta = 42.  Each
// call is one GPU launch, so this measures the per-call latency; the batched
// API (EvaluateBatchToDevice, bench.py --workload dcf) is the throughput path.
template <typename T>
void EvaluateDcf(Runner& r, const std::string& tname) {
  for (int log = 2; log <= 24; log += 2) {
    const std::string name = "BM_EvaluateDcf<" + tname + ">/" + std::to_string(log);
    if (!std::regex_search(name, r.filter)) continue;
    dpf::DcfParameters p;
    *p.mutable_parameters()->mutable_value_type() = dpf::ToValueType<T>();
    p.mutable_parameters()->set_log_domain_size(log);
    auto f = Must(dpf::DistributedComparisonFunction::Create(p), "DCF Create");
    const uint128 mask = (uint128{1} << log) - 1;
    std::mt19937_64 rng(log);
    const uint128 alpha = dpf::MakeUint128(rng(), rng()) & mask;
    auto keys = Must(f->GenerateKeys(alpha, T(42)), "DCF GenerateKeys");
    uint128 x = 0;
    r.Run(name, [&](int64_t n) {
      for (int64_t it = 0; it < n; ++it) {
        T v = Must(f->template Evaluate<T>(keys.first, x), "DCF Evaluate");
        g_sink<T> = static_cast<size_t>(v == T{});
        x = (x + 1) & mask;
      }
    });
  }
}

using MyIntModN = IntModN<uint32_t, 4294967291u>;                 // 2^32 - 5
using MyIntModN64 = IntModN<uint64_t, 18446744073709551557ull>;   // 2^64 - 59

}  // namespace

int main(int argc, char** argv) {
  Runner r;
  std::string json;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* k) -> const char* {
      size_t n = std::strlen(k);
      return a.compare(0, n, k) == 0 ? argv[i] + n : nullptr;
    };
    if (const char* v = val("--benchmark_filter=")) r.filter = std::regex(v);
    else if (const char* v = val("--benchmark_min_time=")) r.min_time = std::atof(v);
    else if (const char* v = val("--json=")) json = v;
    else if (a == "--split") r.split = true;
    else if (a == "--malloc_keep_pages") {
      // Harness option, off by default: glibc serves every block from its heap
      // and keeps freed pages, so a result vector of >= 32 MiB is not a fresh
      // mmap (page faults, zeroing) plus a munmap per call -- what the
      // mid-size per-call cost is without the allocator's fresh pages.
      mallopt(M_MMAP_MAX, 0);
      mallopt(M_TRIM_THRESHOLD, 1 << 30);
    }
    else {
      std::fprintf(stderr, "usage: %s [--benchmark_filter=RE] [--benchmark_min_time=S] [--json=PATH] [--split] [--malloc_keep_pages]\n",
                   argv[0]);
      return 2;
    }
  }
  std::printf("%-72s %17s %10s\n", "Benchmark", "Time", "Iterations");
  EvaluateRegularDpf<uint8_t>(r, "uint8_t", 12, 24);
  EvaluateRegularDpf<uint16_t>(r, "uint16_t", 12, 24);
  EvaluateRegularDpf<uint32_t>(r, "uint32_t", 12, 24);
  EvaluateRegularDpf<uint64_t>(r, "uint64_t", 12, 24);
  EvaluateRegularDpf<uint128>(r, "uint128", 12, 24);
  EvaluateRegularDpf<Tuple<uint32_t, uint32_t>>(r, "Tuple<uint32_t, uint32_t>", 12, 24);
  EvaluateRegularDpf<Tuple<uint32_t, uint64_t>>(r, "Tuple<uint32_t, uint64_t>", 12, 24);
  EvaluateRegularDpf<Tuple<uint64_t, uint64_t>>(r, "Tuple<uint64_t, uint64_t>", 12, 24);
  EvaluateRegularDpf<Tuple<uint32_t, uint32_t, uint32_t, uint32_t>>(
      r, "Tuple<uint32_t, uint32_t, uint32_t, uint32_t>", 12, 24);
  EvaluateRegularDpf<Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>>(
      r, "Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>", 12, 24);
  EvaluateRegularDpf<Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>>(
      r, "Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>", 12, 24);
  EvaluateRegularDpf<Tuple<MyIntModN, MyIntModN, MyIntModN, MyIntModN, MyIntModN>>(
      r, "Tuple<MyIntModN x5>", 12, 24);
  EvaluateRegularDpf<Tuple<MyIntModN64, MyIntModN64, MyIntModN64, MyIntModN64, MyIntModN64>>(
      r, "Tuple<MyIntModN64 x5>", 12, 22);
  EvaluateRegularDpf<XorWrapper<uint128>>(r, "XorWrapper<uint128>", 12, 24);
  EvaluateHierarchicalFull<uint8_t>(r, "uint8_t");
  EvaluateHierarchicalFull<uint16_t>(r, "uint16_t");
  EvaluateHierarchicalFull<uint32_t>(r, "uint32_t");
  EvaluateHierarchicalFull<uint64_t>(r, "uint64_t");
  EvaluateHierarchicalFull<uint128>(r, "uint128");
  IsrgExampleHierarchy(r);
  KeyGeneration<true>(r);
  KeyGeneration<false>(r);
  HeavyHitters(r);
  BatchEvaluation(r);
  EvaluateDcf<uint8_t>(r, "uint8_t");
  EvaluateDcf<uint16_t>(r, "uint16_t");
  EvaluateDcf<uint32_t>(r, "uint32_t");
  EvaluateDcf<uint64_t>(r, "uint64_t");
  EvaluateDcf<uint128>(r, "uint128");
  if (!json.empty()) {
    std::ofstream o(json);
    o << "[\n";
    for (size_t i = 0; i < r.rows.size(); ++i) {
      const Row& w = r.rows[i];
      o << "  {\"name\": \"" << w.name << "\", \"ns_per_iter\": " << w.ns_per_iter
        << ", \"iterations\": " << w.iterations << ", \"label\": \"" << w.label << "\"}"
        << (i + 1 < r.rows.size() ? ",\n" : "\n");
    }
    o << "]\n";
  }
  return 0;
}
