// distributed_comparison_function.h -- the reference's
// DistributedComparisonFunction (dcf/distributed_comparison_function.h:30-105)
// as a drop-in over the MI355X DPF engine.
//
// A DCF with log domain n is an n-level incremental DPF (level i has log
// domain i) whose level-i value is beta when bit (n-1-i) of alpha is set and
// 0 otherwise (cc:79-101); Evaluate(key, x) sums the levels whose bit of x is
// clear (h:83-105).  Here every evaluation -- single point, many points, many
// keys -- is ONE walk down x's path per (key, point) in the gfx950 kernel
// dpf_hip_dcf_eval_batch, instead of n root-to-level EvaluateAt walks.
#ifndef DCF_DISTRIBUTED_COMPARISON_FUNCTION_H_
#define DCF_DISTRIBUTED_COMPARISON_FUNCTION_H_

#include <memory>
#include <utility>
#include <vector>

#include "dcf/distributed_comparison_function.pb.h"
#include "dpf/distributed_point_function.h"

namespace distributed_point_functions {

namespace dpf_internal {
class DeviceScratch;
}

class DistributedComparisonFunction {
 public:
  static StatusOr<std::unique_ptr<DistributedComparisonFunction>> Create(
      const DcfParameters& parameters);

  // Keys for x -> beta if x < alpha else 0 (cc:79-101).
  StatusOr<std::pair<DcfKey, DcfKey>> GenerateKeys(uint128 alpha, const Value& beta);
  template <typename T, typename = std::enable_if_t<!std::is_convertible_v<T, Value> &&
                                                    is_supported_type_v<T>>>
  StatusOr<std::pair<DcfKey, DcfKey>> GenerateKeys(uint128 alpha, const T& beta) {
    StatusOr<Value> value = dpf_->ToValue(beta);
    if (!value.ok()) return value.status();
    return GenerateKeys(alpha, *value);
  }

  // h:83-105.
  template <typename T>
  StatusOr<T> Evaluate(const DcfKey& key, uint128 x) {
    ValueType t = ToValueType<T>();
    StatusOr<std::vector<uint8_t>> packed = EvaluatePacked(key, Span<const uint128>(&x, 1), &t);
    if (!packed.ok()) return packed.status();
    std::vector<T> v = dpf_internal::UnpackElements<T>(dpf_->flat_value_type(0), packed->data(), 1);
    return v[0];
  }

  DistributedComparisonFunction(const DistributedComparisonFunction&) = delete;
  DistributedComparisonFunction& operator=(const DistributedComparisonFunction&) = delete;
  ~DistributedComparisonFunction();

  // ---- MI355X extensions ---------------------------------------------------
  // GenerateKeys with caller-supplied root seeds (reproducible fixtures).
  StatusOr<std::pair<DcfKey, DcfKey>> GenerateKeysWithSeeds(uint128 alpha, const Value& beta,
                                                            uint128 seed_0, uint128 seed_1);
  // Evaluate(key, x) for every x of `xs`, packed elements (one launch).
  // `requested_type` (may be null) plays the role of T.
  StatusOr<std::vector<uint8_t>> EvaluatePacked(const DcfKey& key, Span<const uint128> xs,
                                                const ValueType* requested_type = nullptr);
  // Evaluate for every key of a device batch (rows of the DCF keys' DpfKeys,
  // MakeKeyBatch) at device points: points_per_key per key ([key][point]), or
  // one shared set when `shared_points`.  Writes packed [key][point] outputs.
  StatusOr<int64_t> EvaluateBatchToDevice(const DeviceKeyBatch& keys, const void* device_points,
                                          int64_t points_per_key, bool shared_points,
                                          void* device_out, int64_t capacity_bytes,
                                          void* stream) const;
  // SoA batch of the DpfKeys inside `keys` (validated like EvaluateAt does).
  StatusOr<KeyBatch> MakeKeyBatch(Span<const DcfKey* const> keys) const;
  const DcfParameters& parameters() const { return parameters_; }
  const DistributedPointFunction& dpf() const { return *dpf_; }

 private:
  DistributedComparisonFunction(DcfParameters parameters,
                                std::unique_ptr<DistributedPointFunction> dpf);
  StatusOr<std::pair<DcfKey, DcfKey>> GenerateKeysImpl(uint128 alpha, const Value& beta,
                                                       const uint128* seeds);
  // Per-level EvaluateAt loop of the reference, for value types the kernel
  // does not take (more than 4 tuple leaves).
  StatusOr<std::vector<uint8_t>> EvaluateByLevels(const DcfKey& key, Span<const uint128> xs);

  // The kernel launch shared by the device-batch and host entry points.
  Status Launch(int64_t num_keys, int64_t points_per_key, bool shared_points,
                const dpf_block* seed, const uint8_t* party, const dpf_block* points,
                const dpf_block* cw_seed, const uint8_t* cw_left, const uint8_t* cw_right,
                int cw_stride, const std::vector<const dpf_block*>& vcw, void* device_out,
                void* stream) const;

  const DcfParameters parameters_;
  const std::unique_ptr<DistributedPointFunction> dpf_;
  // Reused device buffers and staged uploads of the host entry points.
  const std::unique_ptr<dpf_internal::DeviceScratch> scratch_;
};

}  // namespace distributed_point_functions

#endif  // DCF_DISTRIBUTED_COMPARISON_FUNCTION_H_
