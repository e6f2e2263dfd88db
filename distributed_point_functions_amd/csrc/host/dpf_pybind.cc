// dpf_pybind.cc -- Python binding of the host C++ DistributedPointFunction.
// Protos cross the boundary as serialized bytes (the reference's wire format);
// 128-bit integers as numpy uint64 arrays of shape (n, 2) = {low, high}.
// Errors raise _dpf_host.StatusError("<code>|<message>"); the Python wrapper
// (distributed_point_functions_amd/dpf.py) turns it into DpfStatusError.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "dcf/distributed_comparison_function.h"
#include "dpf/distributed_point_function.h"
#include "synthetic_data_benchmarks.h"

namespace py = pybind11;
using namespace distributed_point_functions;

namespace {

struct StatusError : std::exception {
  std::string what_;
  explicit StatusError(const Status& s) : what_(std::to_string(s.raw_code()) + "|" + s.message()) {}
  const char* what() const noexcept override { return what_.c_str(); }
};

void Check(const Status& s) {
  if (!s.ok()) throw StatusError(s);
}
template <typename T>
T Take(StatusOr<T> s) {
  if (!s.ok()) throw StatusError(s.status());
  return std::move(*s);
}

template <typename M>
M Parse(const py::bytes& b) {
  M m;
  std::string s = b;
  if (!m.ParseFromString(s)) throw StatusError(InvalidArgumentError("failed to parse proto bytes"));
  return m;
}
template <typename M>
py::bytes Ser(const M& m) {
  return py::bytes(m.SerializeAsString());
}

std::vector<uint128> ToU128(const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& a) {
  if (a.size() == 0) return {};
  if (a.ndim() != 2 || a.shape(1) != 2) throw std::invalid_argument("expected uint64 array (n, 2)");
  std::vector<uint128> r(a.shape(0));
  auto v = a.unchecked<2>();
  for (py::ssize_t i = 0; i < a.shape(0); ++i) r[i] = MakeUint128(v(i, 1), v(i, 0));
  return r;
}

uint128 IntToU128(const py::int_& x) {
  py::int_ mask((1ULL << 63) * 2 - 1);  // 2^64 - 1 via unsigned wrap
  uint64_t lo = PyLong_AsUnsignedLongLongMask(x.ptr());
  py::object hi_o = x.attr("__rshift__")(64);
  uint64_t hi = PyLong_AsUnsignedLongLongMask(hi_o.ptr());
  return MakeUint128(hi, lo);
}

// The result vector itself becomes the numpy array's storage (no copy: a
// multi-GiB output would otherwise be faulted in and copied on one thread).
py::array_t<uint8_t> ToArray(std::vector<uint8_t>&& v) {
  auto* owned = new std::vector<uint8_t>(std::move(v));
  py::capsule free_when_done(owned, [](void* p) { delete static_cast<std::vector<uint8_t>*>(p); });
  return py::array_t<uint8_t>({static_cast<py::ssize_t>(owned->size())}, {py::ssize_t{1}},
                              owned->data(), free_when_done);
}

std::unique_ptr<ValueType> OptType(const py::object& o) {
  if (o.is_none()) return nullptr;
  return std::make_unique<ValueType>(Parse<ValueType>(o.cast<py::bytes>()));
}

struct PyKeyBatch {
  std::shared_ptr<KeyBatch> b;
  int64_t NumKeys() const { return b->num_keys; }
  int NumLevels() const { return b->num_levels; }
  py::array_t<uint64_t> Seeds() const {
    py::array_t<uint64_t> a({static_cast<py::ssize_t>(b->num_keys), py::ssize_t{2}});
    if (b->num_keys) std::memcpy(a.mutable_data(), b->seed.data(), b->num_keys * 16);
    return a;
  }
  py::array_t<uint8_t> Party() const {
    py::array_t<uint8_t> a(static_cast<py::ssize_t>(b->num_keys));
    if (b->num_keys) std::memcpy(a.mutable_data(), b->party.data(), b->num_keys);
    return a;
  }
};

struct PyDeviceKeyBatch {
  std::shared_ptr<DeviceKeyBatch> d;
  int64_t NumKeys() const { return d->num_keys(); }
  int64_t FirstKey() const { return d->first_key(); }
};

// Holds the device key batch alive as long as its context.
struct PyBatchContext {
  std::shared_ptr<DeviceKeyBatch> keys;
  std::shared_ptr<DeviceBatchContext> ctx;
  int PreviousHierarchyLevel() const { return ctx->previous_hierarchy_level(); }
  int PartialEvaluationsLevel() const { return ctx->partial_evaluations_level(); }
  int ExpansionCacheLevel() const { return ctx->expansion_cache_level(); }
  int64_t NumPartialEvaluations() const {
    return static_cast<int64_t>(ctx->partial_prefixes().size());
  }
};

class PyDpf {
 public:
  static PyDpf CreateIncremental(const std::vector<py::bytes>& params) {
    std::vector<DpfParameters> p;
    for (const auto& b : params) p.push_back(Parse<DpfParameters>(b));
    PyDpf r;
    r.dpf_ = std::shared_ptr<DistributedPointFunction>(
        Take(DistributedPointFunction::CreateIncremental(MakeConstSpan(p))).release());
    return r;
  }
  void RegisterValueType(const py::bytes& vt) { Check(dpf_->RegisterValueType(Parse<ValueType>(vt))); }
  py::tuple GenerateKeys(const py::int_& alpha, const std::vector<py::bytes>& betas) {
    std::vector<Value> v;
    for (const auto& b : betas) v.push_back(Parse<Value>(b));
    auto keys = Take(dpf_->GenerateKeysIncremental(IntToU128(alpha), MakeConstSpan(v)));
    return py::make_tuple(Ser(keys.first), Ser(keys.second));
  }
  py::tuple GenerateKeysWithSeeds(const py::int_& alpha, const std::vector<py::bytes>& betas,
                                  const py::int_& s0, const py::int_& s1) {
    std::vector<Value> v;
    for (const auto& b : betas) v.push_back(Parse<Value>(b));
    auto keys = Take(dpf_->GenerateKeysIncrementalWithSeeds(IntToU128(alpha), MakeConstSpan(v),
                                                            IntToU128(s0), IntToU128(s1)));
    return py::make_tuple(Ser(keys.first), Ser(keys.second));
  }
  // API-level timing of the drop-in EvaluateUntil<T>(level, {}, ctx) that
  // returns std::vector<T> in host memory (uint64_t or absl::uint128 by
  // `bits`): `reps` calls on fresh copies of ctx, wall seconds each (the
  // vector's allocation, the kernel and the D2H copy included; freeing the
  // previous vector is not).  Returns (seconds list, elements, sample of the
  // last output: (index, low, high) at `probe` positions).
  py::tuple TimeEvaluateUntil(int level, const py::bytes& ctx_bytes, int bits, int reps,
                              const std::vector<int64_t>& probe) {
    const EvaluationContext ctx0 = Parse<EvaluationContext>(ctx_bytes);
    std::vector<double> secs;
    int64_t n = 0;
    std::vector<py::tuple> samples;
    auto run = [&](auto tag) {
      using T = decltype(tag);
      std::vector<T> out;
      for (int r = 0; r < reps; ++r) {
        EvaluationContext ctx = ctx0;
        out = std::vector<T>();  // free before the timed call
        const auto t0 = std::chrono::steady_clock::now();
        {
          py::gil_scoped_release nogil;
          out = Take(dpf_->EvaluateUntil<T>(level, {}, ctx));
        }
        secs.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      }
      n = static_cast<int64_t>(out.size());
      for (int64_t i : probe)
        if (i >= 0 && i < n)
          samples.push_back(py::make_tuple(i, static_cast<uint64_t>(out[i]),
                                           static_cast<uint64_t>(uint128(out[i]) >> 64)));
    };
    if (bits == 64) run(uint64_t{});
    else if (bits == 128) run(uint128{});
    else throw StatusError(InvalidArgumentError("bits must be 64 or 128"));
    return py::make_tuple(secs, n, samples);
  }
  py::bytes CreateEvaluationContext(const py::bytes& key) {
    return Ser(Take(dpf_->CreateEvaluationContext(Parse<DpfKey>(key))));
  }
  py::tuple EvaluateUntil(int level, const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& prefixes,
                          const py::bytes& ctx_bytes, const py::object& vt) {
    EvaluationContext ctx = Parse<EvaluationContext>(ctx_bytes);
    auto p = ToU128(prefixes);
    auto t = OptType(vt);
    std::vector<uint8_t> out;
    {
      py::gil_scoped_release nogil;
      auto r = dpf_->EvaluateUntilPacked(level, MakeConstSpan(p), ctx, t.get());
      if (!r.ok()) {
        py::gil_scoped_acquire g;
        throw StatusError(r.status());
      }
      out = std::move(*r);
    }
    return py::make_tuple(ToArray(std::move(out)), Ser(ctx));
  }
  py::tuple EvaluateUntilToDevice(int level,
                                  const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& prefixes,
                                  const py::bytes& ctx_bytes, uintptr_t out_ptr, int64_t capacity,
                                  uintptr_t stream, const py::object& vt) {
    EvaluationContext ctx = Parse<EvaluationContext>(ctx_bytes);
    auto p = ToU128(prefixes);
    auto t = OptType(vt);
    int64_t n = 0;
    {
      py::gil_scoped_release nogil;
      auto r = dpf_->EvaluateUntilToDevice(level, MakeConstSpan(p), ctx, reinterpret_cast<void*>(out_ptr),
                                           capacity, reinterpret_cast<void*>(stream), t.get());
      if (!r.ok()) {
        py::gil_scoped_acquire g;
        throw StatusError(r.status());
      }
      n = *r;
    }
    return py::make_tuple(n, Ser(ctx));
  }
  py::tuple EvaluateShardToDevice(int level, int64_t shard, int64_t num_shards,
                                  const py::bytes& ctx_bytes, uintptr_t out_ptr, int64_t capacity,
                                  uintptr_t stream) {
    EvaluationContext ctx = Parse<EvaluationContext>(ctx_bytes);
    int64_t n = 0;
    {
      py::gil_scoped_release nogil;
      auto r = dpf_->EvaluateShardToDevice(level, shard, num_shards, ctx,
                                           reinterpret_cast<void*>(out_ptr), capacity,
                                           reinterpret_cast<void*>(stream));
      if (!r.ok()) {
        py::gil_scoped_acquire g;
        throw StatusError(r.status());
      }
      n = *r;
    }
    return py::make_tuple(n, Ser(ctx));
  }
  py::array_t<uint8_t> EvaluateAt(const py::bytes& key_bytes, int level,
                                  const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& points,
                                  const py::object& vt) {
    DpfKey key = Parse<DpfKey>(key_bytes);
    auto p = ToU128(points);
    auto t = OptType(vt);
    return ToArray(Take(dpf_->EvaluateAtPacked(key, level, MakeConstSpan(p), nullptr, t.get())));
  }
  py::tuple EvaluateAtCtx(int level,
                          const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& points,
                          const py::bytes& ctx_bytes, const py::object& vt) {
    EvaluationContext ctx = Parse<EvaluationContext>(ctx_bytes);
    auto p = ToU128(points);
    auto t = OptType(vt);
    auto out = Take(dpf_->EvaluateAtPacked(ctx.key(), level, MakeConstSpan(p), &ctx, t.get()));
    return py::make_tuple(ToArray(std::move(out)), Ser(ctx));
  }
  py::array_t<uint8_t> EvaluateAtBatch(const std::vector<py::bytes>& keys, int level,
                                       const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& points,
                                       int64_t points_per_key) {
    std::vector<DpfKey> k;
    k.reserve(keys.size());
    for (const auto& b : keys) k.push_back(Parse<DpfKey>(b));
    std::vector<const DpfKey*> ptrs;
    for (const auto& x : k) ptrs.push_back(&x);
    auto p = ToU128(points);
    return ToArray(Take(dpf_->EvaluateAtBatchPacked(MakeConstSpan(ptrs), level, MakeConstSpan(p),
                                                    points_per_key)));
  }
  PyKeyBatch MakeKeyBatch(const std::vector<py::bytes>& keys) {
    std::vector<DpfKey> k;
    k.reserve(keys.size());
    for (const auto& b : keys) k.push_back(Parse<DpfKey>(b));
    std::vector<const DpfKey*> ptrs;
    for (const auto& x : k) ptrs.push_back(&x);
    return PyKeyBatch{std::make_shared<KeyBatch>(Take(dpf_->MakeKeyBatch(MakeConstSpan(ptrs))))};
  }
  py::bytes KeyFromBatch(const PyKeyBatch& b, int64_t k) { return Ser(Take(dpf_->KeyFromBatch(*b.b, k))); }
  py::list SerializeKeyBatch(const PyKeyBatch& b, int threads) {
    StatusOr<std::vector<std::string>> r = InternalError("unset");
    {
      py::gil_scoped_release nogil;
      r = dpf_->SerializeKeyBatch(*b.b, threads);
    }
    std::vector<std::string> v = Take(std::move(r));
    py::list out(v.size());
    for (size_t i = 0; i < v.size(); ++i) out[i] = py::bytes(v[i]);
    return out;
  }
  PyKeyBatch ParseKeyBatch(const std::vector<py::bytes>& keys, int threads) {
    std::vector<std::string_view> views;
    views.reserve(keys.size());
    for (const auto& b : keys)
      views.emplace_back(PyBytes_AS_STRING(b.ptr()), static_cast<size_t>(PyBytes_GET_SIZE(b.ptr())));
    StatusOr<KeyBatch> r = InternalError("unset");
    {
      py::gil_scoped_release nogil;
      r = dpf_->ParseKeyBatch(Span<const std::string_view>(views), threads);
    }
    return PyKeyBatch{std::make_shared<KeyBatch>(Take(std::move(r)))};
  }
  py::tuple GenerateKeyBatch(const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& alphas,
                             const std::vector<py::bytes>& betas, const py::object& root_seeds,
                             int threads) {
    std::vector<Value> v;
    for (const auto& b : betas) v.push_back(Parse<Value>(b));
    auto a = ToU128(alphas);
    std::vector<uint128> seeds;
    if (!root_seeds.is_none())
      seeds = ToU128(root_seeds.cast<py::array_t<uint64_t, py::array::c_style | py::array::forcecast>>());
    std::pair<KeyBatch, KeyBatch> r;
    {
      py::gil_scoped_release nogil;
      auto s = dpf_->GenerateKeyBatch(MakeConstSpan(a), MakeConstSpan(v), MakeConstSpan(seeds), threads);
      if (!s.ok()) {
        py::gil_scoped_acquire g;
        throw StatusError(s.status());
      }
      r = std::move(*s);
    }
    return py::make_tuple(PyKeyBatch{std::make_shared<KeyBatch>(std::move(r.first))},
                          PyKeyBatch{std::make_shared<KeyBatch>(std::move(r.second))});
  }
  int64_t EvaluateAtBatchToDevice(const PyDeviceKeyBatch& keys, int level, uintptr_t points,
                                  int64_t points_per_key, bool shared, uintptr_t out,
                                  int64_t capacity, uintptr_t stream) {
    py::gil_scoped_release nogil;
    auto r = dpf_->EvaluateAtBatchToDevice(*keys.d, level, reinterpret_cast<const void*>(points),
                                           points_per_key, shared, reinterpret_cast<void*>(out),
                                           capacity, reinterpret_cast<void*>(stream));
    if (!r.ok()) {
      py::gil_scoped_acquire g;
      throw StatusError(r.status());
    }
    return *r;
  }
  void EvaluateAtBatchSumToDevice(const PyDeviceKeyBatch& keys, int level, uintptr_t points,
                                  int64_t num_points, uintptr_t out, uintptr_t stream) {
    py::gil_scoped_release nogil;
    Status st = dpf_->EvaluateAtBatchSumToDevice(*keys.d, level, reinterpret_cast<const void*>(points),
                                                 num_points, reinterpret_cast<void*>(out),
                                                 reinterpret_cast<void*>(stream));
    if (!st.ok()) {
      py::gil_scoped_acquire g;
      throw StatusError(st);
    }
  }
  PyBatchContext CreateBatchEvaluationContext(const PyDeviceKeyBatch& keys) {
    auto c = Take(dpf_->CreateBatchEvaluationContext(*keys.d));
    return PyBatchContext{keys.d, std::shared_ptr<DeviceBatchContext>(c.release())};
  }
  int64_t EvaluateUntilBatchToDevice(int level,
                                     const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& prefixes,
                                     PyBatchContext& ctx, bool sum, uintptr_t out, int64_t capacity,
                                     uintptr_t stream) {
    auto p = ToU128(prefixes);
    py::gil_scoped_release nogil;
    auto r = sum ? dpf_->EvaluateUntilBatchSumToDevice(level, MakeConstSpan(p), *ctx.ctx,
                                                       reinterpret_cast<void*>(out), capacity,
                                                       reinterpret_cast<void*>(stream))
                 : dpf_->EvaluateUntilBatchToDevice(level, MakeConstSpan(p), *ctx.ctx,
                                                    reinterpret_cast<void*>(out), capacity,
                                                    reinterpret_cast<void*>(stream));
    if (!r.ok()) {
      py::gil_scoped_acquire g;
      throw StatusError(r.status());
    }
    return *r;
  }
  py::bytes ExportEvaluationContext(const PyBatchContext& ctx, const PyKeyBatch& host, int64_t k,
                                    uintptr_t stream) {
    return Ser(Take(dpf_->ExportEvaluationContext(*ctx.ctx, *host.b, k,
                                                  reinterpret_cast<void*>(stream))));
  }
  py::array_t<uint8_t> SumPackedShares(int level, const py::array_t<uint8_t, py::array::c_style>& shares,
                                       int64_t num_shares, int64_t count) {
    if (static_cast<int64_t>(shares.size()) != num_shares * count * dpf_->flat_value_type(level).packed_size)
      throw StatusError(InvalidArgumentError("shares has the wrong size"));
    return ToArray(Take(dpf_->SumPackedShares(level, shares.data(), num_shares, count)));
  }
  std::vector<py::bytes> Parameters() const {
    std::vector<py::bytes> r;
    for (const auto& p : dpf_->parameters()) r.push_back(Ser(p));
    return r;
  }
  int TreeLevelsNeeded() const { return dpf_->tree_levels_needed(); }
  std::vector<int> HierarchyToTree() const { return dpf_->hierarchy_to_tree(); }
  int BlocksNeeded(int h) const { return dpf_->blocks_needed(h); }
  int ElementsPerBlock(int h) const { return dpf_->flat_value_type(h).elements_per_block; }
  int PackedSize(int h) const { return dpf_->flat_value_type(h).packed_size; }
  int CorrectedElementsPerBlock(int h) const { return dpf_->corrected_elements_per_block(h); }
  int64_t OutputElements(int h, int64_t n, int prev) const {
    return Take(dpf_->OutputElements(h, n, prev));
  }

 private:
  std::shared_ptr<DistributedPointFunction> dpf_;
};

class PyDcf {
 public:
  static PyDcf Create(const py::bytes& params) {
    PyDcf r;
    r.dcf_ = std::shared_ptr<DistributedComparisonFunction>(
        Take(DistributedComparisonFunction::Create(Parse<DcfParameters>(params))).release());
    return r;
  }
  py::tuple GenerateKeys(const py::int_& alpha, const py::bytes& beta, const py::object& s0,
                         const py::object& s1) {
    std::pair<DcfKey, DcfKey> keys;
    if (s0.is_none())
      keys = Take(dcf_->GenerateKeys(IntToU128(alpha), Parse<Value>(beta)));
    else
      keys = Take(dcf_->GenerateKeysWithSeeds(IntToU128(alpha), Parse<Value>(beta),
                                              IntToU128(s0.cast<py::int_>()),
                                              IntToU128(s1.cast<py::int_>())));
    return py::make_tuple(Ser(keys.first), Ser(keys.second));
  }
  py::array_t<uint8_t> Evaluate(const py::bytes& key,
                                const py::array_t<uint64_t, py::array::c_style | py::array::forcecast>& xs,
                                const py::object& vt) {
    auto x = ToU128(xs);
    auto t = OptType(vt);
    return ToArray(Take(dcf_->EvaluatePacked(Parse<DcfKey>(key), MakeConstSpan(x), t.get())));
  }
  PyKeyBatch MakeKeyBatch(const std::vector<py::bytes>& keys) {
    std::vector<DcfKey> k;
    k.reserve(keys.size());
    for (const auto& b : keys) k.push_back(Parse<DcfKey>(b));
    std::vector<const DcfKey*> ptrs;
    for (const auto& x : k) ptrs.push_back(&x);
    return PyKeyBatch{std::make_shared<KeyBatch>(Take(dcf_->MakeKeyBatch(MakeConstSpan(ptrs))))};
  }
  int64_t EvaluateBatchToDevice(const PyDeviceKeyBatch& keys, uintptr_t points, int64_t ppk,
                                bool shared, uintptr_t out, int64_t capacity, uintptr_t stream) {
    py::gil_scoped_release nogil;
    auto r = dcf_->EvaluateBatchToDevice(*keys.d, reinterpret_cast<const void*>(points), ppk, shared,
                                         reinterpret_cast<void*>(out), capacity,
                                         reinterpret_cast<void*>(stream));
    if (!r.ok()) {
      py::gil_scoped_acquire g;
      throw StatusError(r.status());
    }
    return *r;
  }
  int PackedSize() const { return dcf_->dpf().flat_value_type(0).packed_size; }
  std::vector<int> HierarchyToTree() const { return dcf_->dpf().hierarchy_to_tree(); }

 private:
  std::shared_ptr<DistributedComparisonFunction> dcf_;
};

}  // namespace

PYBIND11_MODULE(_dpf_host, m) {
  m.doc() = "Host C++ DistributedPointFunction (MI355X engine) -- serialized-proto binding";
  py::register_exception<StatusError>(m, "StatusError");
  py::class_<PyDeviceKeyBatch>(m, "DeviceKeyBatch")
      .def_property_readonly("num_keys", &PyDeviceKeyBatch::NumKeys)
      .def_property_readonly("first_key", &PyDeviceKeyBatch::FirstKey);
  py::class_<PyBatchContext>(m, "DeviceBatchContext")
      .def_property_readonly("previous_hierarchy_level", &PyBatchContext::PreviousHierarchyLevel)
      .def_property_readonly("partial_evaluations_level", &PyBatchContext::PartialEvaluationsLevel)
      .def_property_readonly("expansion_cache_level", &PyBatchContext::ExpansionCacheLevel)
      .def_property_readonly("num_partial_evaluations", &PyBatchContext::NumPartialEvaluations)
      .def_property_readonly("device_bytes", [](const PyBatchContext& c) { return c.ctx->device_bytes(); })
      .def_property_readonly("cache_events", [](const PyBatchContext& c) {
        const auto& e = c.ctx->cache_events();
        py::dict d;
        d["cache_refused"] = e.cache_refused;
        d["spare_refused"] = e.spare_refused;
        d["in_place"] = e.in_place;
        d["permuted"] = e.permuted;
        d["evicted_spare"] = e.evicted_spare;
        d["evicted_cache"] = e.evicted_cache;
        d["alloc_failures"] = e.alloc_failures;
        return d;
      })
      .def("fail_next_allocations_for_testing",
           [](PyBatchContext& c, int n, int skip) { c.ctx->FailNextAllocationsForTesting(n, skip); },
           py::arg("n"), py::arg("skip") = 0)
      .def("reset", [](PyBatchContext& c, bool release) { c.ctx->Reset(release); },
           py::arg("release_expansion_cache") = false)
      .def("release_expansion_cache", [](PyBatchContext& c) { c.ctx->ReleaseExpansionCache(); });
  py::class_<PyKeyBatch>(m, "KeyBatch")
      .def_property_readonly("num_keys", &PyKeyBatch::NumKeys)
      .def_property_readonly("num_levels", &PyKeyBatch::NumLevels)
      .def("seeds", &PyKeyBatch::Seeds)
      .def("party", &PyKeyBatch::Party)
      .def("upload", [](const PyKeyBatch& b, int64_t begin, int64_t end, uintptr_t stream) {
        auto d = Take(DeviceKeyBatch::Upload(*b.b, begin, end, reinterpret_cast<void*>(stream)));
        return PyDeviceKeyBatch{std::shared_ptr<DeviceKeyBatch>(d.release())};
      });
  py::class_<PyDpf>(m, "DistributedPointFunction")
      .def_static("create_incremental", &PyDpf::CreateIncremental)
      .def("register_value_type", &PyDpf::RegisterValueType)
      .def("generate_keys_incremental", &PyDpf::GenerateKeys)
      .def("generate_keys_incremental_with_seeds", &PyDpf::GenerateKeysWithSeeds)
      .def("create_evaluation_context", &PyDpf::CreateEvaluationContext)
      .def("time_evaluate_until", &PyDpf::TimeEvaluateUntil)
      .def("evaluate_until", &PyDpf::EvaluateUntil)
      .def("evaluate_until_to_device", &PyDpf::EvaluateUntilToDevice)
      .def("evaluate_shard_to_device", &PyDpf::EvaluateShardToDevice)
      .def("evaluate_at", &PyDpf::EvaluateAt)
      .def("evaluate_at_ctx", &PyDpf::EvaluateAtCtx)
      .def("evaluate_at_batch", &PyDpf::EvaluateAtBatch)
      .def("make_key_batch", &PyDpf::MakeKeyBatch)
      .def("key_from_batch", &PyDpf::KeyFromBatch)
      .def("parse_key_batch", &PyDpf::ParseKeyBatch)
      .def("serialize_key_batch", &PyDpf::SerializeKeyBatch)
      .def("generate_key_batch", &PyDpf::GenerateKeyBatch)
      .def("evaluate_at_batch_to_device", &PyDpf::EvaluateAtBatchToDevice)
      .def("evaluate_at_batch_sum_to_device", &PyDpf::EvaluateAtBatchSumToDevice)
      .def("create_batch_evaluation_context", &PyDpf::CreateBatchEvaluationContext)
      .def("evaluate_until_batch_to_device", &PyDpf::EvaluateUntilBatchToDevice)
      .def("export_evaluation_context", &PyDpf::ExportEvaluationContext)
      .def("sum_packed_shares", &PyDpf::SumPackedShares)
      .def("parameters", &PyDpf::Parameters)
      .def("tree_levels_needed", &PyDpf::TreeLevelsNeeded)
      .def("hierarchy_to_tree", &PyDpf::HierarchyToTree)
      .def("blocks_needed", &PyDpf::BlocksNeeded)
      .def("elements_per_block", &PyDpf::ElementsPerBlock)
      .def("packed_size", &PyDpf::PackedSize)
      .def("corrected_elements_per_block", &PyDpf::CorrectedElementsPerBlock)
      .def("output_elements", &PyDpf::OutputElements);
  py::class_<PyDcf>(m, "DistributedComparisonFunction")
      .def_static("create", &PyDcf::Create)
      .def("generate_keys", &PyDcf::GenerateKeys, py::arg("alpha"), py::arg("beta"),
           py::arg("seed_0") = py::none(), py::arg("seed_1") = py::none())
      .def("evaluate", &PyDcf::Evaluate)
      .def("make_key_batch", &PyDcf::MakeKeyBatch)
      .def("evaluate_batch_to_device", &PyDcf::EvaluateBatchToDevice)
      .def("packed_size", &PyDcf::PackedSize)
      .def("hierarchy_to_tree", &PyDcf::HierarchyToTree);
  m.def("synthetic_levels", [](int log, int64_t count, double concentration, uint64_t seed, int mef) {
    auto nz = experiments::MakeSyntheticNonzeros(count, log, concentration, seed);
    auto prefixes = experiments::ComputePrefixes(nz, log);
    auto levels = experiments::ComputeLevelsToEvaluate(prefixes, log, mef);
    std::vector<int64_t> per_bit;
    for (const auto& p : prefixes) per_bit.push_back(static_cast<int64_t>(p.size()));
    py::array_t<uint64_t> a({static_cast<py::ssize_t>(nz.size()), py::ssize_t{2}});
    if (!nz.empty()) std::memcpy(a.mutable_data(), nz.data(), nz.size() * 16);
    return py::make_tuple(levels, per_bit, a);
  });
  m.def("run_synthetic_data_benchmark",
        [](int log, int64_t count, double concentration, uint64_t seed, int mef, int iters,
           bool only_nonzeros, bool verify, bool device_context) {
          experiments::BenchmarkOptions o;
          o.log_domain_size = log;
          o.num_nonzeros = count;
          o.concentration = concentration;
          o.seed = seed;
          o.max_expansion_factor = mef;
          o.num_iterations = iters;
          o.only_nonzeros = only_nonzeros;
          o.verify = verify;
          o.device_context = device_context;
          experiments::BenchmarkReport r;
          {
            py::gil_scoped_release nogil;
            auto s = experiments::RunSyntheticDataBenchmark(o);
            if (!s.ok()) {
              py::gil_scoped_acquire g;
              throw StatusError(s.status());
            }
            r = std::move(*s);
          }
          py::dict d;
          d["levels_to_evaluate"] = r.levels_to_evaluate;
          d["prefixes_per_level"] = r.prefixes_per_level;
          d["outputs_per_level"] = r.outputs_per_level;
          d["key_size_bytes"] = r.key_size_bytes;
          d["seconds_per_iteration"] = r.seconds_per_iteration;
          d["checksum_seconds_excluded"] = r.checksum_seconds;
          d["verified"] = r.verified;
          return d;
        },
        py::arg("log"), py::arg("count"), py::arg("concentration"), py::arg("seed"),
        py::arg("mef"), py::arg("iters"), py::arg("only_nonzeros"), py::arg("verify"),
        py::arg("device_context") = false);
  m.def("bits_needed", [](const py::bytes& vt, double sec) {
    return Take(dpf_internal::BitsNeeded(Parse<ValueType>(vt), sec));
  });
  m.def("value_types_are_equal", [](const py::bytes& a, const py::bytes& b) {
    return Take(dpf_internal::ValueTypesAreEqual(Parse<ValueType>(a), Parse<ValueType>(b)));
  });
  m.def("roundtrip", [](const std::string& name, const py::bytes& b) -> py::bytes {
    // Parses and re-serializes one message (wire-format conformance tests).
    if (name == "DpfKey") return Ser(Parse<DpfKey>(b));
    if (name == "EvaluationContext") return Ser(Parse<EvaluationContext>(b));
    if (name == "DpfParameters") return Ser(Parse<DpfParameters>(b));
    if (name == "Value") return Ser(Parse<Value>(b));
    if (name == "ValueType") return Ser(Parse<ValueType>(b));
    if (name == "CorrectionWord") return Ser(Parse<CorrectionWord>(b));
    if (name == "PartialEvaluation") return Ser(Parse<PartialEvaluation>(b));
    if (name == "Block") return Ser(Parse<Block>(b));
    throw std::invalid_argument("unknown message " + name);
  });
  m.def("debug_string", [](const std::string& name, const py::bytes& b) -> std::string {
    if (name == "DpfKey") return Parse<DpfKey>(b).DebugString();
    if (name == "EvaluationContext") return Parse<EvaluationContext>(b).DebugString();
    if (name == "ValueType") return Parse<ValueType>(b).DebugString();
    if (name == "Value") return Parse<Value>(b).DebugString();
    throw std::invalid_argument("unknown message " + name);
  });
  m.def("validate_context", [](const std::vector<py::bytes>& params, const py::bytes& ctx) {
    std::vector<DpfParameters> p;
    for (const auto& b : params) p.push_back(Parse<DpfParameters>(b));
    auto v = Take(dpf_internal::ProtoValidator::Create(MakeConstSpan(p)));
    Check(v->ValidateEvaluationContext(Parse<EvaluationContext>(ctx)));
  });
}
