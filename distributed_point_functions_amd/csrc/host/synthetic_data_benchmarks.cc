// synthetic_data_benchmarks.cc -- see synthetic_data_benchmarks.h.
#include "synthetic_data_benchmarks.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <random>
#include <set>

#include "dpf/key_batch.h"

namespace distributed_point_functions {
namespace experiments {

std::vector<uint128> MakeSyntheticNonzeros(int64_t count, int log_domain_size,
                                           double concentration, uint64_t seed) {
  std::mt19937_64 rng(seed);
  const uint128 domain_mask =
      log_domain_size >= 128 ? ~uint128{0} : (uint128{1} << log_domain_size) - 1;
  auto draw = [&]() { return MakeUint128(rng(), rng()) & domain_mask; };
  // Size of the dense region: the first `concentration` fraction of the domain.
  uint128 dense = 0;
  const bool skewed = concentration > 0 && concentration < 1;
  if (skewed) {
    // concentration * 2^log without floating-point overflow: scale 2^64 pieces.
    const double c = concentration;
    if (log_domain_size <= 64) {
      dense = static_cast<uint128>(static_cast<double>(uint128{1} << log_domain_size) * c);
    } else {
      const uint128 unit = uint128{1} << (log_domain_size - 64);
      dense = unit * static_cast<uint64_t>(c * 18446744073709551616.0);
    }
    if (dense == 0) dense = 1;
  }
  std::set<uint128> out;
  const int64_t n_dense = skewed ? static_cast<int64_t>(count * 0.9) : 0;
  while (static_cast<int64_t>(out.size()) < n_dense) out.insert(draw() % dense);
  while (static_cast<int64_t>(out.size()) < count) {
    uint128 x = draw();
    if (skewed && x < dense) continue;
    out.insert(x);
  }
  return std::vector<uint128>(out.begin(), out.end());
}

std::vector<std::vector<uint128>> ComputePrefixes(const std::vector<uint128>& nonzeros,
                                                  int log_domain_size) {
  std::vector<std::vector<uint128>> result(log_domain_size + 1);
  result.back() = nonzeros;
  for (int i = log_domain_size; i > 1; --i) {
    // Sorted input -> shifted values are sorted; drop adjacent duplicates.
    std::vector<uint128>& cur = result[i - 1];
    cur.reserve(result[i].size());
    for (const uint128& x : result[i]) {
      uint128 p = x >> 1;
      if (cur.empty() || cur.back() != p) cur.push_back(p);
    }
  }
  return result;
}

std::vector<int> ComputeLevelsToEvaluate(const std::vector<std::vector<uint128>>& prefixes,
                                         int log_domain_size, int max_expansion_factor) {
  const int64_t num_nonzeros = static_cast<int64_t>(prefixes.back().size());
  std::vector<int> levels;
  levels.push_back(std::min(log_domain_size,
                            static_cast<int>(std::log2(static_cast<double>(num_nonzeros)) +
                                             std::log2(static_cast<double>(max_expansion_factor)))) -
                   1);
  while (levels.back() < log_domain_size) {
    const double at_last = static_cast<double>(prefixes[levels.back() + 1].size());
    levels.push_back(std::min(
        log_domain_size,
        static_cast<int>(levels.back() + std::log2(static_cast<double>(num_nonzeros)) +
                         std::log2(static_cast<double>(max_expansion_factor)) - std::log2(at_last))));
  }
  return levels;
}

namespace {
uint64_t Fold(const uint32_t* v, int64_t n) {
  uint64_t h = 0;
  for (int64_t i = 0; i < n; ++i) h ^= (static_cast<uint64_t>(v[i]) << ((i & 1) * 32));
  return h;
}
uint64_t Fold(const std::vector<uint32_t>& v) {
  return Fold(v.data(), static_cast<int64_t>(v.size()));
}
// The checksum is this build's own cross-check (device context vs proto
// context); the reference's loop only returns the outputs
// (synthetic_data_benchmarks.cc:169-191), so its time is kept out of the
// timed iterations and reported apart (HierarchicalResult::checksum_seconds).
template <typename F>
uint64_t TimedFold(double* seconds, F&& fold) {
  const auto a = std::chrono::steady_clock::now();
  const uint64_t h = fold();
  *seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
  return h;
}
}  // namespace

StatusOr<HierarchicalResult> RunHierarchicalEvaluation(
    const DistributedPointFunction& dpf, const DpfKey& key,
    const std::vector<std::vector<uint128>>& prefixes_to_evaluate, int num_iterations) {
  DPF_ASSIGN_OR_RETURN(EvaluationContext ctx, dpf.CreateEvaluationContext(key));
  if (prefixes_to_evaluate.size() != static_cast<size_t>(ctx.parameters_size()))
    return InvalidArgumentError("one prefix list per hierarchy level expected");
  HierarchicalResult r;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < num_iterations; ++i) {
    EvaluationContext ctx_copy = ctx;
    r.outputs_per_level.clear();
    r.checksum = 0;
    for (int level = 0; level < static_cast<int>(prefixes_to_evaluate.size()); ++level) {
      DPF_ASSIGN_OR_RETURN(std::vector<uint32_t> result,
                           dpf.EvaluateUntil<uint32_t>(level, prefixes_to_evaluate[level], ctx_copy));
      r.outputs_per_level.push_back(static_cast<int64_t>(result.size()));
      r.checksum ^= TimedFold(&r.checksum_seconds, [&] { return Fold(result); });
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  r.checksum_seconds /= num_iterations;
  r.seconds_per_iteration =
      std::chrono::duration<double>(t1 - t0).count() / num_iterations - r.checksum_seconds;
  return r;
}

StatusOr<HierarchicalResult> RunHierarchicalEvaluationDeviceContext(
    const DistributedPointFunction& dpf, const DpfKey& key,
    const std::vector<std::vector<uint128>>& prefixes_to_evaluate, int num_iterations) {
  const int H = static_cast<int>(dpf.parameters().size());
  if (prefixes_to_evaluate.size() != static_cast<size_t>(H))
    return InvalidArgumentError("one prefix list per hierarchy level expected");
  const DpfKey* kp = &key;
  DPF_ASSIGN_OR_RETURN(KeyBatch batch, dpf.MakeKeyBatch(Span<const DpfKey* const>(&kp, 1)));
  DPF_ASSIGN_OR_RETURN(std::unique_ptr<DeviceKeyBatch> dev, DeviceKeyBatch::Upload(batch, nullptr));
  DPF_ASSIGN_OR_RETURN(std::unique_ptr<DeviceBatchContext> ctx,
                       dpf.CreateBatchEvaluationContext(*dev));
  int64_t max_bytes = 0;
  for (int level = 0; level < H; ++level) {
    DPF_ASSIGN_OR_RETURN(int64_t n, dpf.OutputElements(level,
                                                       static_cast<int64_t>(prefixes_to_evaluate[level].size()),
                                                       level - 1));
    max_bytes = std::max(max_bytes, n * 4);
  }
  void* out = nullptr;
  if (int rc = dpf_hip_alloc(&out, std::max<int64_t>(max_bytes, 16)))
    return Status(static_cast<StatusCode>(rc), dpf_hip_last_error());
  HierarchicalResult r;
  Status st = OkStatus();
  // The level's outputs go to host memory, as the reference API returns them:
  // one page-locked buffer reused across levels (the caller's choice of
  // destination; DMA straight into it), pageable if none can be had.
  void* pinned = nullptr;
  if (dpf_hip_host_alloc(&pinned, static_cast<size_t>(std::max<int64_t>(max_bytes, 16))) != 0)
    pinned = nullptr;
  std::unique_ptr<uint32_t[]> pageable(pinned ? nullptr
                                              : new uint32_t[std::max<int64_t>(max_bytes / 4, 1)]);
  uint32_t* const host = pinned ? static_cast<uint32_t*>(pinned) : pageable.get();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < num_iterations && st.ok(); ++i) {
    ctx->Reset();
    r.outputs_per_level.clear();
    r.checksum = 0;
    for (int level = 0; level < H && st.ok(); ++level) {
      StatusOr<int64_t> n = dpf.EvaluateUntilBatchToDevice(level, prefixes_to_evaluate[level], *ctx,
                                                           out, max_bytes, nullptr);
      if (!n.ok()) {
        st = n.status();
        break;
      }
      // The reference returns the level's outputs in host memory (one buffer
      // reused across levels here).
      if (int rc = dpf_hip_memcpy_d2h(host, out, *n * 4, nullptr)) {
        st = Status(static_cast<StatusCode>(rc), dpf_hip_last_error());
        break;
      }
      r.outputs_per_level.push_back(*n);
      r.checksum ^= TimedFold(&r.checksum_seconds, [&] { return Fold(host, *n); });
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  dpf_hip_free(out);
  if (pinned) dpf_hip_host_free(pinned);
  DPF_RETURN_IF_ERROR(st);
  r.checksum_seconds /= num_iterations;
  r.seconds_per_iteration =
      std::chrono::duration<double>(t1 - t0).count() / num_iterations - r.checksum_seconds;
  return r;
}

StatusOr<HierarchicalResult> RunDirectEvaluation(const DistributedPointFunction& dpf,
                                                 const DpfKey& key,
                                                 const std::vector<uint128>& nonzeros,
                                                 int num_iterations) {
  if (dpf.parameters().size() != 1) return InvalidArgumentError("direct evaluation needs one level");
  HierarchicalResult r;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < num_iterations; ++i) {
    DPF_ASSIGN_OR_RETURN(std::vector<uint32_t> result, dpf.EvaluateAt<uint32_t>(key, 0, nonzeros));
    if (result.size() != nonzeros.size()) return InternalError("wrong number of outputs");
    r.outputs_per_level = {static_cast<int64_t>(result.size())};
    r.checksum = TimedFold(&r.checksum_seconds, [&] { return Fold(result); });
  }
  const auto t1 = std::chrono::steady_clock::now();
  r.checksum_seconds /= num_iterations;
  r.seconds_per_iteration =
      std::chrono::duration<double>(t1 - t0).count() / num_iterations - r.checksum_seconds;
  return r;
}

Status VerifyHierarchicalEvaluation(const DistributedPointFunction& dpf, const DpfKey& key0,
                                    const DpfKey& key1,
                                    const std::vector<std::vector<uint128>>& prefixes_to_evaluate,
                                    uint128 alpha, uint32_t beta) {
  DPF_ASSIGN_OR_RETURN(EvaluationContext c0, dpf.CreateEvaluationContext(key0));
  DPF_ASSIGN_OR_RETURN(EvaluationContext c1, dpf.CreateEvaluationContext(key1));
  const auto& params = dpf.parameters();
  const int last_log = params.back().log_domain_size();
  for (int level = 0; level < static_cast<int>(prefixes_to_evaluate.size()); ++level) {
    const auto& prefixes = prefixes_to_evaluate[level];
    DPF_ASSIGN_OR_RETURN(std::vector<uint32_t> a, dpf.EvaluateUntil<uint32_t>(level, prefixes, c0));
    DPF_ASSIGN_OR_RETURN(std::vector<uint32_t> b, dpf.EvaluateUntil<uint32_t>(level, prefixes, c1));
    if (a.size() != b.size()) return InternalError("share vectors differ in length");
    const int log_h = params[level].log_domain_size();
    const int log_p = level == 0 ? 0 : params[level - 1].log_domain_size();
    const uint128 alpha_h = last_log - log_h >= 128 ? 0 : alpha >> (last_log - log_h);
    int64_t expect = -1;
    if (level == 0) {
      expect = static_cast<int64_t>(alpha_h);
    } else {
      const uint128 parent = alpha_h >> (log_h - log_p);
      auto it = std::lower_bound(prefixes.begin(), prefixes.end(), parent);
      if (it != prefixes.end() && *it == parent)
        expect = (static_cast<int64_t>(it - prefixes.begin()) << (log_h - log_p)) +
                 static_cast<int64_t>(alpha_h & ((uint128{1} << (log_h - log_p)) - 1));
    }
    for (size_t i = 0; i < a.size(); ++i) {
      const uint32_t sum = a[i] + b[i];
      const uint32_t want = static_cast<int64_t>(i) == expect ? beta : 0;
      if (sum != want)
        return InternalError("reconstruction failed at level " + std::to_string(level) +
                             ", output " + std::to_string(i));
    }
  }
  return OkStatus();
}

StatusOr<BenchmarkReport> RunSyntheticDataBenchmark(const BenchmarkOptions& o) {
  if (o.log_domain_size < 1 || o.log_domain_size > 128 || o.num_nonzeros < 1 ||
      o.num_iterations < 1 || o.max_expansion_factor < 2)
    return InvalidArgumentError("bad benchmark options");
  const std::vector<uint128> nonzeros =
      MakeSyntheticNonzeros(o.num_nonzeros, o.log_domain_size, o.concentration, o.seed);
  const std::vector<std::vector<uint128>> prefixes = ComputePrefixes(nonzeros, o.log_domain_size);
  BenchmarkReport rep;
  rep.levels_to_evaluate = o.only_nonzeros
                               ? std::vector<int>{o.log_domain_size}
                               : ComputeLevelsToEvaluate(prefixes, o.log_domain_size,
                                                         o.max_expansion_factor);
  std::vector<std::vector<uint128>> prefixes_to_evaluate(1);
  for (size_t i = 1; i < rep.levels_to_evaluate.size(); ++i)
    prefixes_to_evaluate.push_back(prefixes[rep.levels_to_evaluate[i - 1]]);
  for (const auto& p : prefixes_to_evaluate) rep.prefixes_per_level.push_back(static_cast<int64_t>(p.size()));
  std::vector<DpfParameters> parameters(rep.levels_to_evaluate.size());
  for (size_t i = 0; i < parameters.size(); ++i) {
    parameters[i].mutable_value_type()->mutable_integer()->set_bitsize(32);
    parameters[i].set_log_domain_size(rep.levels_to_evaluate[i]);
  }
  DPF_ASSIGN_OR_RETURN(std::unique_ptr<DistributedPointFunction> dpf,
                       DistributedPointFunction::CreateIncremental(parameters));
  // The reference draws alpha uniformly; here it is one of the nonzeros so the
  // reconstruction check sees a hit at every level.
  std::mt19937_64 rng(o.seed ^ 0x9E3779B97F4A7C15ULL);
  const uint128 alpha = nonzeros[rng() % nonzeros.size()];
  std::vector<uint128> beta(parameters.size(), 1);
  std::vector<Value> beta_values;
  for (uint128 b : beta) {
    DPF_ASSIGN_OR_RETURN(Value v, dpf->ToValue(b));
    beta_values.push_back(std::move(v));
  }
  DPF_ASSIGN_OR_RETURN(auto keys, dpf->GenerateKeysIncremental(alpha, beta_values));
  rep.key_size_bytes = static_cast<int64_t>(keys.first.SerializeAsString().size());
  HierarchicalResult r;
  if (o.only_nonzeros) {
    DPF_ASSIGN_OR_RETURN(r, RunDirectEvaluation(*dpf, keys.first, nonzeros, o.num_iterations));
  } else if (o.device_context) {
    DPF_ASSIGN_OR_RETURN(r, RunHierarchicalEvaluationDeviceContext(*dpf, keys.first,
                                                                   prefixes_to_evaluate,
                                                                   o.num_iterations));
  } else {
    DPF_ASSIGN_OR_RETURN(r, RunHierarchicalEvaluation(*dpf, keys.first, prefixes_to_evaluate,
                                                      o.num_iterations));
  }
  rep.outputs_per_level = r.outputs_per_level;
  rep.seconds_per_iteration = r.seconds_per_iteration;
  rep.checksum_seconds = r.checksum_seconds;
  if (o.verify) {
    if (o.only_nonzeros) {
      DPF_ASSIGN_OR_RETURN(std::vector<uint32_t> a, dpf->EvaluateAt<uint32_t>(keys.first, 0, nonzeros));
      DPF_ASSIGN_OR_RETURN(std::vector<uint32_t> b, dpf->EvaluateAt<uint32_t>(keys.second, 0, nonzeros));
      for (size_t i = 0; i < a.size(); ++i)
        if (a[i] + b[i] != (nonzeros[i] == alpha ? 1u : 0u))
          return InternalError("direct evaluation reconstruction failed at " + std::to_string(i));
    } else {
      DPF_RETURN_IF_ERROR(VerifyHierarchicalEvaluation(*dpf, keys.first, keys.second,
                                                       prefixes_to_evaluate, alpha, 1));
      if (o.device_context) {
        // The device-context outputs must equal the proto-context API's.
        DPF_ASSIGN_OR_RETURN(HierarchicalResult api,
                             RunHierarchicalEvaluation(*dpf, keys.first, prefixes_to_evaluate, 1));
        if (api.checksum != r.checksum || api.outputs_per_level != r.outputs_per_level)
          return InternalError("device-context outputs differ from EvaluateUntil's");
      }
    }
    rep.verified = true;
  }
  return rep;
}

}  // namespace experiments
}  // namespace distributed_point_functions
