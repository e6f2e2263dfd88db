// distributed_comparison_function.cc -- DistributedComparisonFunction
// (dcf/distributed_comparison_function.cc:15-102, .h:83-105) over the MI355X
// DPF engine; see the header.
#include "dcf/distributed_comparison_function.h"

#include <algorithm>

#include "dpf/key_batch.h"
#include "dpf_hip.h"
#include "host_util.h"

namespace distributed_point_functions {

using dpf_internal::AesKey;
using dpf_internal::FromHip;
using dpf_internal::kPrgKeyLeft;
using dpf_internal::kPrgKeyRight;
using dpf_internal::kPrgKeyValue;
using dpf_internal::MakeDesc;
using dpf_internal::ToBlock;

namespace {

// cc:21-32: integers, IntModN and tuples (recursively) become 0; other kinds
// (XorWrapper) are left as they are, exactly like the reference.
void SetToZero(Value& value) {
  if (value.value_case() == Value::kInteger) {
    value.mutable_integer()->set_value_uint64(0);
  } else if (value.value_case() == Value::kIntModN) {
    value.mutable_int_mod_n()->set_value_uint64(0);
  } else if (value.value_case() == Value::kTuple) {
    for (int i = 0; i < value.tuple().elements_size(); ++i)
      SetToZero(*value.mutable_tuple()->mutable_elements(i));
  }
}


}  // namespace

DistributedComparisonFunction::DistributedComparisonFunction(
    DcfParameters parameters, std::unique_ptr<DistributedPointFunction> dpf)
    : parameters_(std::move(parameters)),
      dpf_(std::move(dpf)),
      scratch_(new dpf_internal::DeviceScratch()) {}

DistributedComparisonFunction::~DistributedComparisonFunction() = default;

StatusOr<std::unique_ptr<DistributedComparisonFunction>> DistributedComparisonFunction::Create(
    const DcfParameters& parameters) {
  // cc:38-72
  if (parameters.parameters().log_domain_size() < 1)
    return InvalidArgumentError("A DCF must have log_domain_size >= 1");
  if (!parameters.parameters().has_value_type())
    return InvalidArgumentError(
        "parameters.value_type must be set for DistributedComparisonFunction::Create");
  std::vector<DpfParameters> dpf_parameters(parameters.parameters().log_domain_size());
  for (int i = 0; i < static_cast<int>(dpf_parameters.size()); ++i) {
    dpf_parameters[i].set_log_domain_size(i);
    *dpf_parameters[i].mutable_value_type() = parameters.parameters().value_type();
  }
  DPF_RETURN_IF_ERROR(dpf_internal::ProtoValidator::ValidateParameters(dpf_parameters));
  DPF_ASSIGN_OR_RETURN(std::unique_ptr<DistributedPointFunction> dpf,
                       DistributedPointFunction::CreateIncremental(dpf_parameters));
  DPF_RETURN_IF_ERROR(dpf->RegisterValueType(parameters.parameters().value_type()));
  return std::unique_ptr<DistributedComparisonFunction>(
      new DistributedComparisonFunction(parameters, std::move(dpf)));
}

StatusOr<std::pair<DcfKey, DcfKey>> DistributedComparisonFunction::GenerateKeys(
    uint128 alpha, const Value& beta) {
  return GenerateKeysImpl(alpha, beta, nullptr);
}

StatusOr<std::pair<DcfKey, DcfKey>> DistributedComparisonFunction::GenerateKeysWithSeeds(
    uint128 alpha, const Value& beta, uint128 seed_0, uint128 seed_1) {
  const uint128 seeds[2] = {seed_0, seed_1};
  return GenerateKeysImpl(alpha, beta, seeds);
}

StatusOr<std::pair<DcfKey, DcfKey>> DistributedComparisonFunction::GenerateKeysImpl(
    uint128 alpha, const Value& beta, const uint128* seeds) {
  // cc:79-101
  const int n = parameters_.parameters().log_domain_size();
  std::vector<Value> dpf_values(n, beta);
  for (int i = 0; i < n; ++i) {
    const bool current_bit = (alpha & (uint128{1} << (n - i - 1))) != 0;
    if (!current_bit) SetToZero(dpf_values[i]);
  }
  // The last bit of alpha is encoded in dpf_values.back() (cc:95-97).
  std::pair<DpfKey, DpfKey> keys;
  if (seeds) {
    DPF_ASSIGN_OR_RETURN(keys, dpf_->GenerateKeysIncrementalWithSeeds(
                                   alpha >> 1, Span<const Value>(dpf_values), seeds[0], seeds[1]));
  } else {
    DPF_ASSIGN_OR_RETURN(keys, dpf_->GenerateKeysIncremental(alpha >> 1, Span<const Value>(dpf_values)));
  }
  std::pair<DcfKey, DcfKey> result;
  *result.first.mutable_key() = std::move(keys.first);
  *result.second.mutable_key() = std::move(keys.second);
  return result;
}

StatusOr<KeyBatch> DistributedComparisonFunction::MakeKeyBatch(
    Span<const DcfKey* const> keys) const {
  std::vector<const DpfKey*> dpf_keys;
  dpf_keys.reserve(keys.size());
  for (const DcfKey* k : keys) dpf_keys.push_back(&k->key());
  return dpf_->MakeKeyBatch(Span<const DpfKey* const>(dpf_keys));
}

StatusOr<int64_t> DistributedComparisonFunction::EvaluateBatchToDevice(
    const DeviceKeyBatch& keys, const void* device_points, int64_t points_per_key,
    bool shared_points, void* device_out, int64_t capacity_bytes, void* stream) const {
  const int n = parameters_.parameters().log_domain_size();
  if (keys.num_levels() != dpf_->tree_levels_needed() - 1 || keys.num_hierarchy_levels() != n)
    return InvalidArgumentError("key batch does not match this DistributedComparisonFunction");
  if (points_per_key < 0) return InvalidArgumentError("points_per_key must be non-negative");
  const int64_t total = keys.num_keys() * points_per_key;
  if (total == 0) return int64_t{0};
  const auto& f = dpf_->flat_value_type(0);
  if (!device_out || capacity_bytes < total * f.packed_size)
    return InvalidArgumentError("device output buffer too small");
  // EvaluateAt(key, 0, {x >> n}) rejects x >= 2^n (h:861-874).
  const int64_t num_points = shared_points ? points_per_key : total;
  if (n < 128) {
    int64_t bad = 0;
    HIP_RETURN_IF_ERROR(dpf_hip_count_out_of_range(
        num_points, static_cast<const dpf_block*>(device_points), n, &bad, stream));
    if (bad)
      return InvalidArgumentError(
          "`evaluation_points[0]` larger than the domain size at hierarchy level 0");
  }
  std::vector<const dpf_block*> vcw(n);
  for (int i = 0; i < n; ++i) vcw[i] = keys.value_correction(i);
  DPF_RETURN_IF_ERROR(Launch(keys.num_keys(), points_per_key, shared_points, keys.seed(),
                             keys.party(), static_cast<const dpf_block*>(device_points),
                             keys.cw_seed(), keys.cw_left(), keys.cw_right(), keys.num_levels(),
                             vcw, device_out, stream));
  return total;
}

Status DistributedComparisonFunction::Launch(int64_t num_keys, int64_t points_per_key,
                                             bool shared_points, const dpf_block* seed,
                                             const uint8_t* party, const dpf_block* points,
                                             const dpf_block* cw_seed, const uint8_t* cw_left,
                                             const uint8_t* cw_right, int cw_stride,
                                             const std::vector<const dpf_block*>& vcw,
                                             void* device_out, void* stream) const {
  const int n = parameters_.parameters().log_domain_size();
  const auto& f = dpf_->flat_value_type(0);
  std::vector<int32_t> depth(n), blocks(n);
  for (int i = 0; i < n; ++i) {
    depth[i] = dpf_->hierarchy_to_tree()[i];
    blocks[i] = dpf_->blocks_needed(i);
  }
  const dpf_value_desc desc = MakeDesc(f, blocks[0]);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  HIP_RETURN_IF_ERROR(dpf_hip_dcf_eval_batch(
      num_keys, points_per_key, shared_points ? 1 : 0, n, depth.data(), blocks.data(), seed, party,
      points, cw_seed, cw_left, cw_right, cw_stride, vcw.data(), &kl, &kr, &kv, &desc, device_out,
      stream));
  return OkStatus();
}

StatusOr<std::vector<uint8_t>> DistributedComparisonFunction::EvaluateByLevels(
    const DcfKey& key, Span<const uint128> xs) {
  // h:83-105 verbatim: one EvaluateAt per level and point.
  const int n = parameters_.parameters().log_domain_size();
  const auto& f = dpf_->flat_value_type(0);
  const int nl = static_cast<int>(f.leaves.size());
  std::vector<uint8_t> out(xs.size() * f.packed_size);
  std::vector<uint128> acc(nl), v(nl);
  for (size_t j = 0; j < xs.size(); ++j) {
    std::fill(acc.begin(), acc.end(), 0);
    const uint128 x = xs[j];
    for (int i = 0; i < n; ++i) {
      const uint128 prefix = n < 128 ? x >> (n - i) : 0;
      DPF_ASSIGN_OR_RETURN(std::vector<uint8_t> e,
                           dpf_->EvaluateAtPacked(key.key(), i, Span<const uint128>(&prefix, 1), nullptr));
      if ((x & (uint128{1} << (n - i - 1))) == 0) {
        dpf_internal::UnpackLeaves(f, e.data(), v.data());
        for (int l = 0; l < nl; ++l) acc[l] = dpf_internal::LeafAdd(f.leaves[l], acc[l], v[l]);
      }
    }
    dpf_internal::PackLeaves(f, acc.data(), out.data() + j * f.packed_size);
  }
  return out;
}

StatusOr<std::vector<uint8_t>> DistributedComparisonFunction::EvaluatePacked(
    const DcfKey& key, Span<const uint128> xs, const ValueType* requested_type) {
  const int n = parameters_.parameters().log_domain_size();
  // The checks of the reference's first EvaluateAt (level 0, point x >> n).
  if (requested_type) {
    DPF_ASSIGN_OR_RETURN(bool eq, dpf_internal::ValueTypesAreEqual(
                                      *requested_type, parameters_.parameters().value_type()));
    if (!eq) return InvalidArgumentError("Value type T doesn't match parameters at `hierarchy_level`");
  }
  for (uint128 x : xs)
    if (n < 128 && (x >> n) != 0)
      return InvalidArgumentError(
          "`evaluation_points[0]` larger than the domain size at hierarchy level 0");
  const DcfKey* kp = &key;
  DPF_ASSIGN_OR_RETURN(KeyBatch batch, MakeKeyBatch(Span<const DcfKey* const>(&kp, 1)));
  if (xs.empty()) return std::vector<uint8_t>{};
  const auto& f = dpf_->flat_value_type(0);
  if (f.leaves.size() > 4) return EvaluateByLevels(key, xs);
  // One key: its arrays and the points go through the reused scratch buffers
  // (staged, no per-call allocation), then one launch and one copy back.
  auto* s = scratch_.get();
  std::lock_guard<std::recursive_mutex> scratch_lock(s->mu);  // one call at a time per object
  const int64_t m = static_cast<int64_t>(xs.size());
  std::vector<dpf_block> pts(m);
  for (int64_t i = 0; i < m; ++i) pts[i] = ToBlock(xs[i]);
  const int L = batch.num_levels;
  std::vector<dpf_block> vcw_all;
  std::vector<size_t> vcw_off(n);
  for (int i = 0; i < n; ++i) {
    vcw_off[i] = vcw_all.size();
    vcw_all.insert(vcw_all.end(), batch.value_correction[i].begin(),
                   batch.value_correction[i].end());
  }
  dpf_internal::PackedUploads& up = s->packed;
  DPF_RETURN_IF_ERROR(up.Reset());
  const size_t o_seed = up.Add(batch.seed.data(), 1);
  const size_t o_party = up.Add(batch.party.data(), 1);
  const size_t o_cws = up.Add(batch.cw_seed.data(), L);
  const size_t o_cwl = up.Add(batch.cw_left.data(), L);
  const size_t o_cwr = up.Add(batch.cw_right.data(), L);
  const size_t o_vcw = up.Add(vcw_all.data(), vcw_all.size());
  const size_t o_pts = up.Add(pts.data(), pts.size());
  DPF_RETURN_IF_ERROR(up.Commit(nullptr));
  const size_t bytes = static_cast<size_t>(m) * f.packed_size;
  void* small = s->small_out.Get(bytes);   // small results: written to page-locked memory
  if (!small) DPF_RETURN_IF_ERROR(s->out.Reserve(bytes));
  void* const dev_out = small ? small : s->out.get();
  std::vector<const dpf_block*> vcw(n);
  for (int i = 0; i < n; ++i) vcw[i] = up.Ptr<dpf_block>(o_vcw) + vcw_off[i];
  DPF_RETURN_IF_ERROR(Launch(1, m, false, up.Ptr<dpf_block>(o_seed), up.Ptr<uint8_t>(o_party),
                             up.Ptr<dpf_block>(o_pts), up.Ptr<dpf_block>(o_cws),
                             up.Ptr<uint8_t>(o_cwl), up.Ptr<uint8_t>(o_cwr), L, vcw,
                             dev_out, nullptr));
  DPF_RETURN_IF_ERROR(up.MarkUsed(nullptr));
  std::vector<uint8_t> out(bytes);
  if (small) {
    HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(nullptr));
    std::memcpy(out.data(), small, bytes);
  } else {
    HIP_RETURN_IF_ERROR(dpf_hip_memcpy_d2h(out.data(), s->out.get(), out.size(), nullptr));
  }
  return out;
}

}  // namespace distributed_point_functions
