// dpf_api_test.cc -- the reference's typed correctness tests
// (dpf/distributed_point_function_test.cc:665-1030, two-party reconstruction
// over value types and domain sizes; EvaluateAt against EvaluateUntil) written
// against the C++ templates of include/dpf/*.h, so the template paths a C++
// caller uses are covered too (the Python tests go through the type-erased
// *Packed entry points): EvaluateUntil<T> copying plain integers straight into
// the returned vector, the threaded unpack of tuples, EvaluateNext over
// hierarchies, EvaluateAt<T> with and without a context, and DCF Evaluate<T>.
//
// Exit status 0 and "ALL OK" on success; the first mismatch is printed.
// Run by tests/test_cpp_api_gpu.py; built by build_native.build_tools.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "dcf/distributed_comparison_function.h"
#include "dpf/distributed_point_function.h"
#include "dpf/int_mod_n.h"
#include "dpf/tuple.h"
#include "dpf/xor_wrapper.h"
#include "dpf_hip.h"
// The library's internal D2H helpers (CopyToHostSink), for the grow-failure test.
#include "../../distributed_point_functions_amd/csrc/host/host_util.h"

namespace dpf = distributed_point_functions;
using dpf::DistributedPointFunction;
using dpf::DpfParameters;
using dpf::EvaluationContext;
using dpf::uint128;

namespace {

int g_checks = 0;

[[noreturn]] void Fail(const std::string& what) {
  std::fprintf(stderr, "FAIL: %s\n", what.c_str());
  std::exit(1);
}

template <typename T>
T Must(dpf::StatusOr<T> s, const std::string& what) {
  if (!s.ok()) Fail(what + ": " + s.status().ToString());
  return std::move(s).value();
}

using ModN32 = dpf::IntModN<uint32_t, 4294967291u>;
using ModN64 = dpf::IntModN<uint64_t, 18446744073709551557ull>;

// beta values per type (non-zero, exercising high bits).
template <typename T> T Beta();
template <> uint8_t Beta<uint8_t>() { return 0xA5; }
template <> uint16_t Beta<uint16_t>() { return 0xBEEF; }
template <> uint32_t Beta<uint32_t>() { return 0xDEADBEEFu; }
template <> uint64_t Beta<uint64_t>() { return 0xFEEDFACECAFEBEEFull; }
template <> uint128 Beta<uint128>() { return dpf::MakeUint128(0x0123456789ABCDEFull, 0xF0E1D2C3B4A59687ull); }
template <> dpf::XorWrapper<uint128> Beta<dpf::XorWrapper<uint128>>() {
  return dpf::XorWrapper<uint128>(dpf::MakeUint128(0xAAAA5555AAAA5555ull, 0x123456789ull));
}
template <> dpf::Tuple<uint32_t, uint64_t> Beta<dpf::Tuple<uint32_t, uint64_t>>() {
  return dpf::Tuple<uint32_t, uint64_t>(0x11223344u, 0x5566778899AABBCCull);
}
using U32x5 = dpf::Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>;
template <> U32x5 Beta<U32x5>() { return U32x5(1u, 0xFFFFFFFFu, 3u, 0x80000000u, 5u); }
template <> dpf::Tuple<ModN32, ModN32> Beta<dpf::Tuple<ModN32, ModN32>>() {
  return dpf::Tuple<ModN32, ModN32>(ModN32(123456789u), ModN32(4000000000u));
}
template <> dpf::Tuple<ModN64, ModN64, ModN64> Beta<dpf::Tuple<ModN64, ModN64, ModN64>>() {
  return dpf::Tuple<ModN64, ModN64, ModN64>(ModN64(1), ModN64(18446744073709551000ull), ModN64(42));
}

// Two-party full-domain reconstruction at one level
// (distributed_point_function_test.cc:665-745), plus EvaluateAt<T> at a few
// points against the full-domain outputs (:874-930).
template <typename T>
void FullDomain(const std::string& name, int log) {
  DpfParameters p;
  p.set_log_domain_size(log);
  *p.mutable_value_type() = dpf::ToValueType<T>();
  auto f = Must(DistributedPointFunction::Create(p), "Create");
  if (!f->template RegisterValueType<T>().ok()) Fail("RegisterValueType " + name);
  std::mt19937_64 rng(log * 7919 + name.size());
  const uint128 domain = uint128{1} << log;
  const uint128 alpha = dpf::MakeUint128(rng(), rng()) % domain;
  const T beta = Beta<T>();
  auto keys = Must(f->GenerateKeys(alpha, beta), "GenerateKeys " + name);
  EvaluationContext c0 = Must(f->CreateEvaluationContext(keys.first), "ctx");
  EvaluationContext c1 = Must(f->CreateEvaluationContext(keys.second), "ctx");
  std::vector<T> a = Must(f->template EvaluateUntil<T>(0, {}, c0), "EvaluateUntil " + name);
  std::vector<T> b = Must(f->template EvaluateNext<T>({}, c1), "EvaluateNext " + name);
  if (a.size() != static_cast<size_t>(domain) || b.size() != a.size())
    Fail(name + ": output size " + std::to_string(a.size()));
  for (size_t i = 0; i < a.size(); ++i) {
    const T want = (uint128{i} == alpha) ? beta : T{};
    if (!(static_cast<T>(a[i] + b[i]) == want))  // uint8/16 promote to int
      Fail(name + "/" + std::to_string(log) + ": reconstruction at " + std::to_string(i));
  }
  std::vector<uint128> pts = {alpha, 0, domain - 1, dpf::MakeUint128(rng(), rng()) % domain};
  std::vector<T> at0 = Must(f->template EvaluateAt<T>(keys.first, 0, pts), "EvaluateAt " + name);
  for (size_t j = 0; j < pts.size(); ++j)
    if (!(at0[j] == a[static_cast<size_t>(pts[j])]))
      Fail(name + ": EvaluateAt != EvaluateUntil at point " + std::to_string(j));
  g_checks += 2;
}

// EvaluateAt<T> with a 4-32 MiB result (the overlapped-growth range of
// CopyToHostSink; run with DPF_OVERLAP_GROW=0 and 1 by test_cpp_api_gpu.py):
// every point's value equals the full-domain output's.
template <typename T>
void LargeEvaluateAt(const std::string& name, int log, int64_t npts) {
  DpfParameters p;
  p.set_log_domain_size(log);
  *p.mutable_value_type() = dpf::ToValueType<T>();
  auto f = Must(DistributedPointFunction::Create(p), "Create");
  if (!f->template RegisterValueType<T>().ok()) Fail("RegisterValueType " + name);
  std::mt19937_64 rng(log * 104729 + npts);
  const uint128 domain = uint128{1} << log;
  auto keys = Must(f->GenerateKeys(dpf::MakeUint128(rng(), rng()) % domain, Beta<T>()), "keys");
  EvaluationContext c0 = Must(f->CreateEvaluationContext(keys.first), "ctx");
  std::vector<T> full = Must(f->template EvaluateUntil<T>(0, {}, c0), "EvaluateUntil " + name);
  f->ReleaseScratch();   // the next call reallocates what it needs
  std::vector<uint128> pts(static_cast<size_t>(npts));
  for (auto& x : pts) x = dpf::MakeUint128(rng(), rng()) % domain;
  std::vector<T> at = Must(f->template EvaluateAt<T>(keys.first, 0, pts), "EvaluateAt " + name);
  if (at.size() != pts.size()) Fail(name + ": EvaluateAt size");
  for (size_t j = 0; j < pts.size(); ++j)
    if (!(at[j] == full[static_cast<size_t>(pts[j])]))
      Fail(name + ": large EvaluateAt != EvaluateUntil at " + std::to_string(j));
  ++g_checks;
}

// A result sink whose growth throws (no memory for the result) makes the
// device-to-host copy fail with an error, on the overlapped path (grow on a
// helper thread, 4-32 MiB) and on the chunk-by-chunk path -- never terminate.
void GrowFailureIsAnError() {
  const size_t bytes = size_t{8} << 20;
  void* dev = nullptr;
  if (dpf_hip_alloc(&dev, bytes) != 0 || dpf_hip_memset(dev, 0x5A, bytes, nullptr) != 0)
    Fail("device buffer");
  std::vector<uint8_t> host(bytes);
  dpf::dpf_internal::HostSink sink;
  sink.reserve = [&](size_t) -> void* { return host.data(); };
  // As VectorSink: grow() sizes the result up front on the overlapped path,
  // and chunk() grows it chunk by chunk otherwise.
  sink.grow = [](size_t) { throw std::bad_alloc(); };
  sink.chunk = [&](const uint8_t* src, size_t off, size_t len) {
    sink.grow(off + len);
    std::memcpy(host.data() + off, src, len);
  };
  for (const char* mode : {"1", "0"}) {
    setenv("DPF_OVERLAP_GROW", mode, 1);
    const int rc = dpf::dpf_internal::CopyToHostSink(sink, host.data(), dev, bytes, nullptr);
    if (rc == 0) Fail(std::string("grow failure not reported, DPF_OVERLAP_GROW=") + mode);
    ++g_checks;
  }
  unsetenv("DPF_OVERLAP_GROW");
  dpf_hip_free(dev);
}

// Hierarchical evaluation (distributed_point_function_test.cc:932-1030):
// levels {4, 9, 15}, EvaluateNext at every prefix of the previous level for
// the first step and at a prefix subset afterwards; both parties reconstruct
// beta_h at alpha's prefix and 0 elsewhere.  Also EvaluateAt with a context.
void Hierarchical() {
  const int logs[3] = {4, 9, 15};
  std::vector<DpfParameters> ps(3);
  for (int i = 0; i < 3; ++i) {
    ps[i].set_log_domain_size(logs[i]);
    ps[i].mutable_value_type()->mutable_integer()->set_bitsize(i == 1 ? 128 : 64);
  }
  auto f = Must(DistributedPointFunction::CreateIncremental(ps), "CreateIncremental");
  const uint128 alpha = 0x5A3C;  // < 2^15
  const std::vector<uint128> beta = {7, dpf::MakeUint128(3, 9), 0xFFFFFFFFFFFFFFFFull};
  auto keys = Must(f->GenerateKeysIncremental(alpha, beta), "GenerateKeysIncremental");
  EvaluationContext c[2] = {Must(f->CreateEvaluationContext(keys.first), "ctx"),
                            Must(f->CreateEvaluationContext(keys.second), "ctx")};
  // Level 0: full domain.
  std::vector<uint64_t> l0[2];
  for (int s = 0; s < 2; ++s) l0[s] = Must(f->EvaluateNext<uint64_t>({}, c[s]), "level 0");
  for (uint64_t i = 0; i < 16; ++i)
    if (l0[0][i] + l0[1][i] != (i == (alpha >> 11) ? 7u : 0u)) Fail("hierarchy level 0");
  // Level 1: prefixes {alpha>>11, 3, 9}.
  std::vector<uint128> pre1 = {alpha >> 11, 3, 9};
  std::vector<uint128> l1[2];
  for (int s = 0; s < 2; ++s) l1[s] = Must(f->EvaluateNext<uint128>(pre1, c[s]), "level 1");
  for (size_t j = 0; j < pre1.size(); ++j)
    for (uint128 x = 0; x < 32; ++x) {
      const uint128 full = (pre1[j] << 5) | x;
      const uint128 got = l1[0][j * 32 + static_cast<size_t>(x)] + l1[1][j * 32 + static_cast<size_t>(x)];
      if (got != (full == (alpha >> 6) ? beta[1] : 0)) Fail("hierarchy level 1");
    }
  // Level 2: two level-1 prefixes, one of them alpha's.
  std::vector<uint128> pre2 = {alpha >> 6, (uint128{9} << 5) | 17};
  std::vector<uint64_t> l2[2];
  for (int s = 0; s < 2; ++s) l2[s] = Must(f->EvaluateNext<uint64_t>(pre2, c[s]), "level 2");
  for (size_t j = 0; j < pre2.size(); ++j)
    for (uint64_t x = 0; x < 64; ++x) {
      const uint128 full = (pre2[j] << 6) | x;
      if (l2[0][j * 64 + x] + l2[1][j * 64 + x] !=
          (full == alpha ? static_cast<uint64_t>(beta[2]) : 0))
        Fail("hierarchy level 2");
    }
  // EvaluateAt with a fresh context at level 2 equals the hierarchical output.
  EvaluationContext c2 = Must(f->CreateEvaluationContext(keys.first), "ctx");
  std::vector<uint128> pts = {alpha, (uint128{9} << 11) | (17 << 6) | 5};
  std::vector<uint64_t> at = Must(f->EvaluateAt<uint64_t>(2, pts, c2), "EvaluateAt ctx");
  if (at[0] != l2[0][static_cast<size_t>(alpha & 63)]) Fail("EvaluateAt(ctx) at alpha");
  if (at[1] != l2[0][64 + 5]) Fail("EvaluateAt(ctx) at second point");
  g_checks += 4;
}

// EvaluateUntilToDevice with a too-small device buffer fails before touching
// the context, so a retry with the same context and a large enough buffer
// succeeds and equals EvaluateUntil on a copy of that context.  Covers both
// the first call (no prefixes) and a prefixed call (partial evaluations).
void DeviceRetryAfterSmallBuffer() {
  std::vector<DpfParameters> ps(2);
  ps[0].set_log_domain_size(4);
  ps[1].set_log_domain_size(9);
  for (auto& p : ps) p.mutable_value_type()->mutable_integer()->set_bitsize(64);
  auto f = Must(DistributedPointFunction::CreateIncremental(ps), "CreateIncremental");
  auto keys = Must(f->GenerateKeysIncremental(uint128{0x1A5}, {uint128{3}, uint128{5}}),
                   "GenerateKeysIncremental");
  EvaluationContext ctx = Must(f->CreateEvaluationContext(keys.first), "ctx");
  void* dev = nullptr;
  if (dpf_hip_alloc(&dev, 64 * 8) != 0) Fail("dpf_hip_alloc");
  std::vector<uint128> none;
  auto small0 = f->EvaluateUntilToDevice(0, none, ctx, dev, 15 * 8, nullptr);
  if (small0.ok()) Fail("first call: small buffer accepted");
  if (ctx.previous_hierarchy_level() != -1) Fail("first call: ctx changed by a failed call");
  EvaluationContext ref = ctx;
  std::vector<uint64_t> want0 = Must(f->EvaluateUntil<uint64_t>(0, none, ref), "EvaluateUntil 0");
  if (Must(f->EvaluateUntilToDevice(0, none, ctx, dev, 16 * 8, nullptr), "retry 0") != 16)
    Fail("first call: element count");
  std::vector<uint64_t> got(64);
  if (dpf_hip_memcpy_d2h(got.data(), dev, 16 * 8, nullptr) != 0) Fail("d2h");
  for (int i = 0; i < 16; ++i)
    if (got[i] != want0[i]) Fail("first call: retry output differs");
  std::vector<uint128> pre = {3, 10};
  const EvaluationContext before = ctx;
  auto small1 = f->EvaluateUntilToDevice(1, pre, ctx, dev, 63 * 8, nullptr);
  if (small1.ok()) Fail("prefixed call: small buffer accepted");
  if (!(ctx == before)) Fail("prefixed call: ctx changed by a failed call");
  ref = ctx;
  std::vector<uint64_t> want1 = Must(f->EvaluateUntil<uint64_t>(1, pre, ref), "EvaluateUntil 1");
  if (Must(f->EvaluateUntilToDevice(1, pre, ctx, dev, 64 * 8, nullptr), "retry 1") != 64)
    Fail("prefixed call: element count");
  if (dpf_hip_memcpy_d2h(got.data(), dev, 64 * 8, nullptr) != 0) Fail("d2h");
  if (got != want1) Fail("prefixed call: retry output differs");
  dpf_hip_free(dev);
  g_checks += 2;
}

// DCF (dcf/distributed_comparison_function_test.cc): x < alpha -> beta.
template <typename T>
void Dcf(int log) {
  dpf::DcfParameters p;
  p.mutable_parameters()->set_log_domain_size(log);
  *p.mutable_parameters()->mutable_value_type() = dpf::ToValueType<T>();
  auto f = Must(dpf::DistributedComparisonFunction::Create(p), "DCF Create");
  const uint128 domain = uint128{1} << log;
  const uint128 alpha = domain / 3 + 1;
  const T beta = Beta<T>();
  auto keys = Must(f->GenerateKeys(alpha, beta), "DCF GenerateKeys");
  for (uint128 x : {uint128{0}, alpha - 1, alpha, alpha + 1, domain - 1}) {
    T a = Must(f->template Evaluate<T>(keys.first, x), "DCF Evaluate");
    T b = Must(f->template Evaluate<T>(keys.second, x), "DCF Evaluate");
    if (!(static_cast<T>(a + b) == (x < alpha ? beta : T{}))) Fail("DCF reconstruction");
  }
  g_checks += 1;
}

}  // namespace

int main() {
  for (int log : {1, 5, 12, 21}) {
    FullDomain<uint8_t>("uint8_t", log);
    FullDomain<uint16_t>("uint16_t", log);
    FullDomain<uint32_t>("uint32_t", log);
    FullDomain<uint64_t>("uint64_t", log);
    FullDomain<uint128>("uint128", log);
    FullDomain<dpf::XorWrapper<uint128>>("XorWrapper<uint128>", log);
    FullDomain<dpf::Tuple<uint32_t, uint64_t>>("Tuple<uint32_t, uint64_t>", log);
    FullDomain<dpf::Tuple<ModN32, ModN32>>("Tuple<IntModN32 x2>", log);
  }
  // 2^23 outputs: large enough for the bounce-buffered copies and the
  // huge-page output vectors of the host path.
  FullDomain<uint64_t>("uint64_t", 23);
  FullDomain<dpf::Tuple<uint32_t, uint64_t>>("Tuple<uint32_t, uint64_t>", 22);
  FullDomain<dpf::Tuple<ModN64, ModN64, ModN64>>("Tuple<IntModN64 x3>", 10);
  // Chunked unpacking out of the 16 MiB staging buffers (chunks that are not
  // a power of two: 20- and 12-byte packed elements), and the registered DMA
  // straight into a 512 MiB result vector.
  FullDomain<U32x5>("Tuple<uint32_t x5>", 20);
  FullDomain<dpf::Tuple<uint32_t, uint64_t>>("Tuple<uint32_t, uint64_t>", 23);
  FullDomain<dpf::Tuple<ModN32, ModN32>>("Tuple<IntModN32 x2>", 22);
  FullDomain<uint64_t>("uint64_t", 26);
  // EvaluateAt results of 8, 16, 20 and 16 MiB.
  LargeEvaluateAt<uint64_t>("uint64_t", 24, int64_t{1} << 20);
  LargeEvaluateAt<uint128>("uint128", 22, int64_t{1} << 20);
  LargeEvaluateAt<U32x5>("Tuple<uint32_t x5>", 20, int64_t{1} << 20);
  LargeEvaluateAt<dpf::Tuple<ModN32, ModN32>>("Tuple<IntModN32 x2>", 22, int64_t{1} << 21);
  GrowFailureIsAnError();
  Hierarchical();
  DeviceRetryAfterSmallBuffer();
  for (int log : {3, 16, 64}) {
    Dcf<uint32_t>(log);
    Dcf<uint128>(log);
  }
  std::printf("ALL OK (%d checks)\n", g_checks);
  return 0;
}
