// distributed_point_function.h -- the DistributedPointFunction API of the
// reference (dpf/distributed_point_function.h:77-585), kept as a drop-in, with
// evaluation executed by hand-written gfx950 kernels through the C ABI of
// include/dpf_hip.h.  Key generation stays on the CPU.
//
// Public surface (same names, argument meaning and error behaviour as the
// reference): Create, CreateIncremental, ToValue, RegisterValueType,
// GenerateKeys (3 overloads), GenerateKeysIncremental (3 overloads),
// CreateEvaluationContext, EvaluateUntil<T>, EvaluateNext<T>, both
// EvaluateAt<T> overloads, parameters(); free functions ToValue, FromValue,
// ToValueType.
//
// MI355X extensions (not in the reference):
//   * *Packed variants: the type-erased core used by the templates and the
//     Python binding; output = packed elements (leaves concatenated, little-endian).
//   * EvaluateUntilToDevice: leaves the output in device memory (HBM), which is
//     how full-domain evaluations at 2^30+ elements are meant to be consumed.
//   * EvaluateAtBatchPacked: one launch for many keys x points.
//   * GenerateKeysIncrementalWithSeeds: injected root seeds for reproducible
//     fixtures (the reference draws them with RAND_bytes, cc:656-662).
//
// Thread-compatible, not thread-safe (like the reference, whose
// Aes128FixedKeyHash shares one EVP context).
#ifndef DPF_DISTRIBUTED_POINT_FUNCTION_H_
#define DPF_DISTRIBUTED_POINT_FUNCTION_H_

#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <string_view>
#include <type_traits>
#include <utility>
#include <vector>

#include "dpf/aes_128_fixed_key_hash.h"
#include "dpf/distributed_point_function.pb.h"
#include "dpf/internal/proto_validator.h"
#include "dpf/internal/value_type_helpers.h"
#include "dpf/key_batch.h"
#include "dpf/span.h"
#include "dpf/status.h"
#include "dpf/uint128.h"

namespace distributed_point_functions {

template <typename T>
using is_supported_type = dpf_internal::is_supported_type<T>;
template <typename T>
constexpr bool is_supported_type_v = is_supported_type<T>::value;

// h:49-67
template <typename T, typename = std::enable_if_t<is_supported_type_v<T>>>
StatusOr<T> FromValue(const Value& value) {
  return dpf_internal::FromValueImpl<T>(value);
}
template <typename T, typename = std::enable_if_t<is_supported_type_v<T>>>
Value ToValue(const T& input) {
  return dpf_internal::ValueTypeHelper<T>::ToValue(input);
}
template <typename T, typename = std::enable_if_t<is_supported_type_v<T>>>
ValueType ToValueType() {
  return dpf_internal::ValueTypeHelper<T>::ToValueType();
}

namespace dpf_internal {
class DeviceScratch;
}

class DistributedPointFunction {
 public:
  static StatusOr<std::unique_ptr<DistributedPointFunction>> Create(const DpfParameters& parameters);
  static StatusOr<std::unique_ptr<DistributedPointFunction>> CreateIncremental(
      Span<const DpfParameters> parameters);

  DistributedPointFunction(const DistributedPointFunction&) = delete;
  DistributedPointFunction& operator=(const DistributedPointFunction&) = delete;
  ~DistributedPointFunction();

  template <typename T>
  StatusOr<Value> ToValue(const T& in) {
    Status status = RegisterValueType<T>();
    if (!status.ok()) return status;
    return distributed_point_functions::ToValue(in);
  }

  template <typename T>
  Status RegisterValueType() {
    return RegisterValueType(ToValueType<T>());
  }
  // Runtime form of RegisterValueType<T>() (registers the serialized type).
  Status RegisterValueType(const ValueType& value_type);

  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeys(uint128 alpha, uint128 beta) {
    return GenerateKeysIncremental(alpha, Span<const uint128>(&beta, 1));
  }
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeys(uint128 alpha, Value beta) {
    return GenerateKeysIncremental(alpha, Span<const Value>(&beta, 1));
  }
  template <typename T, typename = std::enable_if_t<!std::is_convertible_v<T, uint128> &&
                                                    !std::is_convertible_v<T, Value> &&
                                                    is_supported_type_v<T>>>
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeys(uint128 alpha, const T& beta) {
    StatusOr<Value> value = ToValue<T>(beta);
    if (!value.ok()) return value.status();
    return GenerateKeysIncremental(alpha, Span<const Value>(&*value, 1));
  }

  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncremental(uint128 alpha,
                                                              Span<const uint128> beta) {
    std::vector<Value> values(beta.size());
    for (size_t i = 0; i < beta.size(); ++i) {
      StatusOr<Value> v = ToValue(beta[i]);
      if (!v.ok()) return v.status();
      values[i] = std::move(*v);
    }
    return GenerateKeysIncremental(alpha, Span<const Value>(values));
  }
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncremental(uint128 alpha,
                                                              Span<const Value> beta);
  template <typename T0, typename... Tn,
            typename = std::enable_if_t<
                !std::is_convertible_v<T0, Span<const Value>> &&
                !std::is_convertible_v<T0, Span<const uint128>> &&
                is_supported_type_v<std::decay_t<T0>> &&
                (is_supported_type_v<std::decay_t<Tn>> && ...)>>
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncremental(uint128 alpha, T0&& beta_0,
                                                              Tn&&... beta_n) {
    std::vector<Value> values;
    Status status = OkStatus();
    auto add = [&](const auto& b) {
      if (!status.ok()) return;
      StatusOr<Value> v = ToValue(b);
      if (v.ok()) values.push_back(std::move(*v)); else status = v.status();
    };
    add(beta_0);
    (add(beta_n), ...);
    if (!status.ok()) return status;
    return GenerateKeysIncremental(alpha, Span<const Value>(values));
  }

  // Extension: root seeds supplied by the caller (reproducible fixtures).
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncrementalWithSeeds(
      uint128 alpha, Span<const Value> beta, uint128 seed_0, uint128 seed_1);

  StatusOr<EvaluationContext> CreateEvaluationContext(DpfKey key) const;

  template <typename T>
  StatusOr<std::vector<T>> EvaluateUntil(int hierarchy_level, Span<const uint128> prefixes,
                                         EvaluationContext& ctx) const {
    ValueType t = ToValueType<T>();
    if constexpr (dpf_internal::kPackedIsMemoryImage<T>) {
      // The packed elements are T's memory image: copy them from the device
      // straight into the result.
      std::vector<T> out;
      const HostSink sink = dpf_internal::VectorSink(&out);
      Status status = EvaluateUntilToHost(hierarchy_level, prefixes, ctx, &t, sink);
      if (!status.ok()) return status;
      return out;
    } else {
      // Packed tuples / IntModN / XorWrapper values are unpacked straight out
      // of the page-locked staging buffers into the result, chunk by chunk
      // (the sink reads flat_[hierarchy_level] only after validation).
      std::vector<T> out;
      const HostSink sink = dpf_internal::UnpackSink(&flat_, hierarchy_level, &out);
      Status status = EvaluateUntilToHost(hierarchy_level, prefixes, ctx, &t, sink);
      if (!status.ok()) return status;
      return out;
    }
  }

  template <typename T>
  StatusOr<std::vector<T>> EvaluateNext(Span<const uint128> prefixes,
                                        EvaluationContext& ctx) const {
    if (prefixes.empty()) return EvaluateUntil<T>(0, prefixes, ctx);
    return EvaluateUntil<T>(ctx.previous_hierarchy_level() + 1, prefixes, ctx);
  }

  template <typename T>
  StatusOr<std::vector<T>> EvaluateAt(const DpfKey& key, int hierarchy_level,
                                      Span<const uint128> evaluation_points) const {
    return EvaluateAtImpl<T>(key, hierarchy_level, evaluation_points, nullptr);
  }

  template <typename T>
  StatusOr<std::vector<T>> EvaluateAt(int hierarchy_level, Span<const uint128> evaluation_points,
                                      EvaluationContext& ctx) const {
    return EvaluateAtImpl<T>(ctx.key(), hierarchy_level, evaluation_points, &ctx);
  }

  Span<const DpfParameters> parameters() const { return validator_->parameters(); }

  // ---- type-erased core (packed elements) --------------------------------
  // `requested_type` (may be null) plays the role of T in the templates.
  // Where the packed output is copied (dpf_internal::HostSink: storage for it,
  // and how a fresh vector becomes valid chunk by chunk during the copy).
  using HostSink = dpf_internal::HostSink;
  Status EvaluateUntilToHost(int hierarchy_level, Span<const uint128> prefixes,
                             EvaluationContext& ctx, const ValueType* requested_type,
                             const HostSink& sink) const;
  StatusOr<std::vector<uint8_t>> EvaluateUntilPacked(int hierarchy_level,
                                                     Span<const uint128> prefixes,
                                                     EvaluationContext& ctx,
                                                     const ValueType* requested_type = nullptr) const;
  // Writes the packed output to device memory `device_out` (capacity in bytes)
  // on `stream`; returns the number of elements written.
  StatusOr<int64_t> EvaluateUntilToDevice(int hierarchy_level, Span<const uint128> prefixes,
                                          EvaluationContext& ctx, void* device_out,
                                          int64_t capacity_bytes, void* stream,
                                          const ValueType* requested_type = nullptr) const;
  // Multi-GPU sharding: the first (full-domain) evaluation of
  // `hierarchy_level` restricted to shard `shard` of `num_shards` (a power of
  // two): the outputs [shard * n / num_shards, (shard + 1) * n / num_shards) of
  // EvaluateUntil(hierarchy_level, {}, ctx), i.e. the subtree under the top
  // log2(num_shards) tree bits.  Writes packed elements to device memory and
  // advances ctx like EvaluateUntil; returns the number of elements written.
  StatusOr<int64_t> EvaluateShardToDevice(int hierarchy_level, int64_t shard, int64_t num_shards,
                                          EvaluationContext& ctx, void* device_out,
                                          int64_t capacity_bytes, void* stream) const;
  StatusOr<std::vector<uint8_t>> EvaluateAtPacked(const DpfKey& key, int hierarchy_level,
                                                  Span<const uint128> evaluation_points,
                                                  EvaluationContext* ctx,
                                                  const ValueType* requested_type = nullptr) const;
  // EvaluateAt's packed output copied into `sink` (EvaluateAt<T>: straight
  // into the returned std::vector<T>).
  Status EvaluateAtToHost(const DpfKey& key, int hierarchy_level,
                          Span<const uint128> evaluation_points, EvaluationContext* ctx,
                          const ValueType* requested_type, const HostSink& sink) const;
  // keys[k] is evaluated at points[k*points_per_key .. (k+1)*points_per_key).
  StatusOr<std::vector<uint8_t>> EvaluateAtBatchPacked(Span<const DpfKey* const> keys,
                                                       int hierarchy_level,
                                                       Span<const uint128> points,
                                                       int64_t points_per_key) const;

  // ---- key batches ------------------
  // SoA image of `keys` (each validated like CreateEvaluationContext does).
  StatusOr<KeyBatch> MakeKeyBatch(Span<const DpfKey* const> keys) const;
  // SoA image of serialized DpfKeys (the proto wire format), parsed and
  // validated on `num_threads` host threads (0 = hardware concurrency, at most
  // 16) -- the batched key ingestion of SURVEY.md 8f.2.  Errors name the first
  // failing key.
  StatusOr<KeyBatch> ParseKeyBatch(Span<const std::string_view> serialized_keys,
                                   int num_threads = 0) const;
  // Row k of `batch` as a DpfKey proto (inverse of MakeKeyBatch).
  StatusOr<DpfKey> KeyFromBatch(const KeyBatch& batch, int64_t k) const;
  // Every row as a serialized DpfKey (inverse of ParseKeyBatch), on
  // `num_threads` host threads (0 = hardware concurrency, at most 16).
  StatusOr<std::vector<std::string>> SerializeKeyBatch(const KeyBatch& batch,
                                                       int num_threads = 0) const;
  // Key generation for many alphas at once, straight into SoA form, on
  // `num_threads` host threads (0 = hardware concurrency).  Key k of the pair
  // is what GenerateKeysIncrementalWithSeeds(alphas[k], beta, root_seeds[2k],
  // root_seeds[2k+1]) returns; with empty root_seeds they are drawn like
  // GenerateKeysIncremental draws them.  `beta` is shared by all keys.
  StatusOr<std::pair<KeyBatch, KeyBatch>> GenerateKeyBatch(Span<const uint128> alphas,
                                                           Span<const Value> beta,
                                                           Span<const uint128> root_seeds,
                                                           int num_threads = 0) const;
  // EvaluateAt(key_k, hierarchy_level, points_k) for every key of a device
  // batch.  `device_points` are raw domain points (uint128 memory images) in
  // device memory: points_per_key per key ([key][point]), or one shared set of
  // points_per_key points when `shared_points`.  Writes num_keys *
  // points_per_key packed elements ([key][point]) to device_out.
  StatusOr<int64_t> EvaluateAtBatchToDevice(const DeviceKeyBatch& keys, int hierarchy_level,
                                            const void* device_points, int64_t points_per_key,
                                            bool shared_points, void* device_out,
                                            int64_t capacity_bytes, void* stream) const;
  // Aggregation variant: out[j] = sum over the batch's keys of
  // EvaluateAt(key_k, hierarchy_level, point_j), in the value type's group,
  // for one shared set of num_points device points (num_points packed elements).
  Status EvaluateAtBatchSumToDevice(const DeviceKeyBatch& keys, int hierarchy_level,
                                    const void* device_points, int64_t num_points,
                                    void* device_out, void* stream) const;
  // ---- device-resident incremental evaluation of a key batch (8f.1, cfg 5b)
  // A fresh context for every key of `keys` (previous_hierarchy_level -1), as
  // CreateEvaluationContext would make per key.  `keys` must outlive it.
  StatusOr<std::unique_ptr<DeviceBatchContext>> CreateBatchEvaluationContext(
      const DeviceKeyBatch& keys) const;
  // EvaluateUntil(hierarchy_level, prefixes, ctx_k) for every key k of the
  // batch, at the same prefixes for all keys (same validation and errors as
  // EvaluateUntil): writes num_keys rows of n packed elements ([key][element])
  // to device_out and returns n.
  StatusOr<int64_t> EvaluateUntilBatchToDevice(int hierarchy_level, Span<const uint128> prefixes,
                                               DeviceBatchContext& ctx, void* device_out,
                                               int64_t capacity_bytes, void* stream) const;
  // Aggregation variant: out[j] = group sum over the batch's keys of
  // EvaluateUntil(hierarchy_level, prefixes, ctx_k)[j] (n packed elements).
  StatusOr<int64_t> EvaluateUntilBatchSumToDevice(int hierarchy_level,
                                                  Span<const uint128> prefixes,
                                                  DeviceBatchContext& ctx, void* device_out,
                                                  int64_t capacity_bytes, void* stream) const;
  // Key k's context as the EvaluationContext proto EvaluateUntil would have
  // left (lazy serialization; `host_keys` is the batch `ctx` was uploaded from).
  StatusOr<EvaluationContext> ExportEvaluationContext(const DeviceBatchContext& ctx,
                                                      const KeyBatch& host_keys, int64_t k,
                                                      void* stream) const;

  // Gives back the per-object host and device scratch the evaluation calls
  // keep between calls (page-locked argument images, staging, device buffers,
  // the prefix dedup's vectors): hundreds of MB after one huge hierarchical
  // call.  Waits for work in flight that reads them; the next call
  // reallocates.  Must not run concurrently with a call on this object.
  void ReleaseScratch();

  // Group sum of `num_shares` packed output vectors of `count` elements each
  // (host memory), e.g. per-GPU partial sums after an all-gather.
  StatusOr<std::vector<uint8_t>> SumPackedShares(int hierarchy_level, const uint8_t* shares,
                                                 int64_t num_shares, int64_t count) const;

  // Introspection.
  int tree_levels_needed() const { return validator_->tree_levels_needed(); }
  const std::vector<int>& hierarchy_to_tree() const { return validator_->hierarchy_to_tree(); }
  int blocks_needed(int h) const { return blocks_needed_[h]; }
  const dpf_internal::FlatValueType& flat_value_type(int h) const { return flat_[h]; }
  int corrected_elements_per_block(int h) const {
    return 1 << (parameters()[h].log_domain_size() - hierarchy_to_tree()[h]);
  }
  // Number of output elements EvaluateUntil(h, prefixes) produces.
  StatusOr<int64_t> OutputElements(int hierarchy_level, int64_t num_prefixes,
                                   int previous_hierarchy_level) const;

 private:
  struct DeviceStart;  // seeds + control bits of the expansion starts, on device

  DistributedPointFunction(std::unique_ptr<dpf_internal::ProtoValidator> validator,
                           std::vector<int> blocks_needed, std::vector<dpf_internal::FlatValueType> flat,
                           Aes128FixedKeyHash prg_left, Aes128FixedKeyHash prg_right,
                           Aes128FixedKeyHash prg_value);

  // EvaluateAt<T> (h:839-1010): the packed output copied or unpacked into
  // the result chunk by chunk, as EvaluateUntil<T> does.
  template <typename T>
  StatusOr<std::vector<T>> EvaluateAtImpl(const DpfKey& key, int hierarchy_level,
                                          Span<const uint128> evaluation_points,
                                          EvaluationContext* ctx) const {
    ValueType t = ToValueType<T>();
    std::vector<T> out;
    if constexpr (dpf_internal::kPackedIsMemoryImage<T>) {
      const HostSink sink = dpf_internal::VectorSink(&out);
      Status status = EvaluateAtToHost(key, hierarchy_level, evaluation_points, ctx, &t, sink);
      if (!status.ok()) return status;
    } else {
      const HostSink sink = dpf_internal::UnpackSink(&flat_, hierarchy_level, &out);
      Status status = EvaluateAtToHost(key, hierarchy_level, evaluation_points, ctx, &t, sink);
      if (!status.ok()) return status;
    }
    return out;
  }

  template <typename T>
  StatusOr<std::vector<T>> Unpack(int h, const std::vector<uint8_t>& packed) const {
    const auto& flat = flat_[h];
    return dpf_internal::UnpackElements<T>(flat, packed.data(),
                                           static_cast<int64_t>(packed.size() / flat.packed_size));
  }

  // Key generation pieces (cc:63-204).
  StatusOr<std::vector<uint128>> ComputeValueCorrectionLeaves(int hierarchy_level,
                                                              const uint128 seeds[2], uint128 alpha,
                                                              Span<const uint128> beta_leaves,
                                                              bool invert) const;
  Status CheckValueCorrectionKnown(int hierarchy_level) const;
  Status GenerateNextCore(int tree_level, uint128 alpha, uint128 seeds[2], bool control_bits[2],
                          uint128* seed_correction, bool ccw[2]) const;
  StatusOr<std::vector<Value>> ComputeValueCorrection(int hierarchy_level, const uint128 seeds[2],
                                                      uint128 alpha, const Value& beta,
                                                      bool invert) const;
  Status GenerateNext(int tree_level, uint128 alpha, Span<const Value> beta, uint128 seeds[2],
                      bool control_bits[2], DpfKey keys[2]) const;

  // Shared evaluation core; output goes to device_out (caller-owned device
  // memory) or, when device_out is null, to *host_out.
  Status EvaluateUntilCore(int hierarchy_level, Span<const uint128> prefixes,
                           EvaluationContext& ctx, const ValueType* requested_type,
                           void* device_out, int64_t capacity_bytes, void* stream,
                           const HostSink* host_out, int64_t* num_elements) const;
  // ComputePartialEvaluations (cc:351-453), path walk on the GPU.
  // `before_device` (may be empty) runs after the host-side lookups and before
  // any device work, so host validation errors never leave work in flight.
  Status ComputePartialEvaluations(Span<const uint128> prefixes, int hierarchy_level,
                                   bool update_ctx, EvaluationContext& ctx,
                                   DeviceStart* out, void* stream,
                                   const std::function<Status()>& before_device) const;
  StatusOr<std::vector<uint128>> ValueCorrectionLeaves(const DpfKey& key, int h) const;
  // Sizes `b` for n keys, and fills row k from `key` (validated).
  void ResizeKeyBatch(int64_t n, KeyBatch* b) const;
  Status FillKeyBatchRow(const DpfKey& key, int64_t k, KeyBatch* b) const;
  // Shared core of the two batched EvaluateUntil entry points.
  StatusOr<int64_t> EvaluateUntilBatchCore(int hierarchy_level, Span<const uint128> prefixes,
                                           DeviceBatchContext& ctx, bool sum, void* device_out,
                                           int64_t capacity_bytes, void* stream) const;

  std::unique_ptr<dpf_internal::ProtoValidator> validator_;
  std::vector<int> blocks_needed_;
  std::vector<dpf_internal::FlatValueType> flat_;
  Aes128FixedKeyHash prg_left_, prg_right_, prg_value_;
  std::set<std::string> registered_types_;
  std::unique_ptr<dpf_internal::DeviceScratch> scratch_;
};

}  // namespace distributed_point_functions

#endif  // DPF_DISTRIBUTED_POINT_FUNCTION_H_
