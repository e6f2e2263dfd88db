// synthetic_data_benchmarks.h -- the reference's sparse-histogram benchmark
// driver (experiments/synthetic_data_benchmarks.cc), restated as library
// functions so bench.py can run it on the GPU-backed API.
//
// One server expands ONE DpfKey either hierarchically (EvaluateUntil at every
// level of a prefix hierarchy chosen so no level expands to more than
// max_expansion_factor x #nonzeros outputs) or directly (EvaluateAt at the
// nonzeros).  The nonzeros stand in for the reference's CSV inputs, which are
// git-LFS stubs in the checkout; MakeSyntheticNonzeros regenerates inputs of
// the same shape (experiments/README.md: 2^20 distinct buckets, power law with
// 90% of them in the first 10% / 50% of the domain, or uniform).
#ifndef DPF_HOST_SYNTHETIC_DATA_BENCHMARKS_H_
#define DPF_HOST_SYNTHETIC_DATA_BENCHMARKS_H_

#include <cstdint>
#include <vector>

#include "dpf/distributed_point_function.h"

namespace distributed_point_functions {
namespace experiments {

// Sorted distinct nonzeros in [0, 2^log_domain_size).  `concentration` in
// (0, 1) puts 90% of them in the first `concentration` fraction of the domain;
// concentration <= 0 or >= 1 means uniform.  Deterministic in `seed`.
std::vector<uint128> MakeSyntheticNonzeros(int64_t count, int log_domain_size,
                                           double concentration, uint64_t seed);

// ComputePrefixes (synthetic_data_benchmarks.cc:89-108): result[b] = sorted
// distinct b-bit prefixes of the (sorted, distinct) nonzeros, b = 0..log.
std::vector<std::vector<uint128>> ComputePrefixes(const std::vector<uint128>& nonzeros,
                                                  int log_domain_size);

// ComputeLevelsToEvaluate (synthetic_data_benchmarks.cc:135-165).
std::vector<int> ComputeLevelsToEvaluate(const std::vector<std::vector<uint128>>& prefixes,
                                         int log_domain_size, int max_expansion_factor);

struct HierarchicalResult {
  double seconds_per_iteration = 0;
  std::vector<int64_t> outputs_per_level;  // of the last iteration
  uint64_t checksum = 0;                   // XOR-fold of every output of the last iteration
  double checksum_seconds = 0;             // per iteration, spent in that fold: not in the above
};

// RunHierarchicalEvaluation<uint32_t> (synthetic_data_benchmarks.cc:167-190):
// `prefixes_to_evaluate[0]` is empty, entry i the prefixes at level i - 1.
StatusOr<HierarchicalResult> RunHierarchicalEvaluation(
    const DistributedPointFunction& dpf, const DpfKey& key,
    const std::vector<std::vector<uint128>>& prefixes_to_evaluate, int num_iterations);

// The same hierarchy through the device-resident context:
// EvaluateUntilBatchToDevice on a one-key batch, each level's outputs copied
// to a host vector like the reference returns them.
StatusOr<HierarchicalResult> RunHierarchicalEvaluationDeviceContext(
    const DistributedPointFunction& dpf, const DpfKey& key,
    const std::vector<std::vector<uint128>>& prefixes_to_evaluate, int num_iterations);

// RunBatchedSinglePointEvaluation<uint32_t> (synthetic_data_benchmarks.cc:192-205).
StatusOr<HierarchicalResult> RunDirectEvaluation(const DistributedPointFunction& dpf,
                                                 const DpfKey& key,
                                                 const std::vector<uint128>& nonzeros,
                                                 int num_iterations);

// Two-server check of a hierarchy: at every level the two parties' uint32
// shares must add up to `beta` exactly at alpha's prefix (when its parent is
// among the level's prefixes) and to 0 everywhere else.  Prefix lists must be
// sorted (ComputePrefixes output).
Status VerifyHierarchicalEvaluation(const DistributedPointFunction& dpf, const DpfKey& key0,
                                    const DpfKey& key1,
                                    const std::vector<std::vector<uint128>>& prefixes_to_evaluate,
                                    uint128 alpha, uint32_t beta);

// main() of synthetic_data_benchmarks.cc: nonzeros -> prefixes -> levels ->
// CreateIncremental(uint32 at every level) -> keys -> timed evaluation.
struct BenchmarkOptions {
  int log_domain_size = 32;
  int64_t num_nonzeros = int64_t{1} << 20;
  double concentration = 0;      // 0.1, 0.5 or uniform (0)
  uint64_t seed = 1;
  int max_expansion_factor = 4;  // experiments/README.md: 2^22 = 4 x 2^20 per level
  int num_iterations = 3;
  bool only_nonzeros = false;    // direct EvaluateAt instead of the hierarchy
  bool verify = true;            // two-server reconstruction check (untimed)
  bool device_context = false;   // hierarchical: device-resident context (8f.1)
};
struct BenchmarkReport {
  std::vector<int> levels_to_evaluate;
  std::vector<int64_t> prefixes_per_level;
  std::vector<int64_t> outputs_per_level;
  int64_t key_size_bytes = 0;
  double seconds_per_iteration = 0;
  double checksum_seconds = 0;  // per iteration, excluded from seconds_per_iteration
  bool verified = false;
};
StatusOr<BenchmarkReport> RunSyntheticDataBenchmark(const BenchmarkOptions& options);

}  // namespace experiments
}  // namespace distributed_point_functions

#endif  // DPF_HOST_SYNTHETIC_DATA_BENCHMARKS_H_
