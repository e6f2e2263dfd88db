// key_batch.cc -- key batches: SoA ingestion of DpfKeys,
// multi-threaded batched key generation (8f.4), and the batched EvaluateAt
// paths of configs 4 and 5 (8e) on the gfx950 kernels of include/dpf_hip.h.
//
// Semantics per key are exactly those of the single-key API:
//   * GenerateKeyBatch row k == GenerateKeysIncrementalWithSeeds(alphas[k], ...)
//     (distributed_point_function.cc:619-687; value corrections cc:63-99);
//   * EvaluateAtBatchToDevice element (k, j) == EvaluateAt(key_k, h, {p_kj})
//     (distributed_point_function.h:839-1010);
//   * EvaluateAtBatchSumToDevice element j == the group sum over k of those.
#include <sys/random.h>

#include <algorithm>
#include <thread>

#include "dpf/distributed_point_function.h"
#include "dpf/key_batch.h"
#include "dpf_hip.h"
#include "host_util.h"

namespace distributed_point_functions {

using dpf_internal::AesKey;
using dpf_internal::FromBlock;
using dpf_internal::FromHip;
using dpf_internal::FromProtoBlock;
using dpf_internal::kPrgKeyLeft;
using dpf_internal::kPrgKeyRight;
using dpf_internal::kPrgKeyValue;
using dpf_internal::MakeDesc;
using dpf_internal::SetProtoBlock;
using dpf_internal::ToBlock;

// ------------------------------------------------------------ DeviceKeyBatch
namespace {
Status UploadRows(void** dst, const void* src, size_t bytes, void* stream) {
  HIP_RETURN_IF_ERROR(dpf_hip_alloc(dst, std::max<size_t>(bytes, 16)));
  return FromHip(dpf_hip_memcpy_h2d(*dst, src, bytes, stream));
}
}  // namespace

StatusOr<std::unique_ptr<DeviceKeyBatch>> DeviceKeyBatch::Upload(const KeyBatch& b, int64_t begin,
                                                                 int64_t end, void* stream) {
  if (begin < 0 || end < begin || end > b.num_keys)
    return InvalidArgumentError("key range out of bounds");
  const int64_t n = end - begin;
  const int L = b.num_levels;
  std::unique_ptr<DeviceKeyBatch> d(new DeviceKeyBatch());
  d->num_keys_ = n;
  d->first_key_ = begin;
  d->num_levels_ = L;
  DPF_RETURN_IF_ERROR(UploadRows(&d->seed_, b.seed.data() + begin, n * sizeof(dpf_block), stream));
  DPF_RETURN_IF_ERROR(UploadRows(&d->party_, b.party.data() + begin, n, stream));
  DPF_RETURN_IF_ERROR(UploadRows(&d->cw_seed_, b.cw_seed.data() + begin * L,
                                 n * L * sizeof(dpf_block), stream));
  DPF_RETURN_IF_ERROR(UploadRows(&d->cw_left_, b.cw_left.data() + begin * L, n * L, stream));
  DPF_RETURN_IF_ERROR(UploadRows(&d->cw_right_, b.cw_right.data() + begin * L, n * L, stream));
  d->vcw_.assign(b.value_correction.size(), nullptr);
  for (size_t h = 0; h < b.value_correction.size(); ++h) {
    const auto& v = b.value_correction[h];
    const int64_t per_key = b.num_keys ? static_cast<int64_t>(v.size()) / b.num_keys : 0;
    DPF_RETURN_IF_ERROR(UploadRows(&d->vcw_[h], v.data() + begin * per_key,
                                   n * per_key * sizeof(dpf_block), stream));
  }
  return d;
}

DeviceKeyBatch::~DeviceKeyBatch() {
  for (void* p : {seed_, party_, cw_seed_, cw_left_, cw_right_})
    if (p) dpf_hip_free(p);
  for (void* p : vcw_)
    if (p) dpf_hip_free(p);
}

// ------------------------------------------------------------ ingestion
void DistributedPointFunction::ResizeKeyBatch(int64_t n, KeyBatch* b) const {
  const int H = static_cast<int>(parameters().size());
  const int L = tree_levels_needed() - 1;
  b->num_keys = n;
  b->num_levels = L;
  b->seed.resize(n);
  b->party.resize(n);
  b->cw_seed.resize(n * L);
  b->cw_left.resize(n * L);
  b->cw_right.resize(n * L);
  b->value_correction.resize(H);
  for (int h = 0; h < H; ++h) {
    const auto& f = flat_value_type(h);
    b->value_correction[h].resize(n * f.elements_per_block * f.leaves.size());
  }
}

Status DistributedPointFunction::FillKeyBatchRow(const DpfKey& key, int64_t k, KeyBatch* b) const {
  const int H = static_cast<int>(parameters().size());
  const int L = b->num_levels;
  DPF_RETURN_IF_ERROR(validator_->ValidateDpfKey(key));
  b->seed[k] = ToBlock(FromProtoBlock(key.seed()));
  b->party[k] = static_cast<uint8_t>(key.party() & 1);
  for (int j = 0; j < L; ++j) {
    const CorrectionWord& cw = key.correction_words(j);
    b->cw_seed[k * L + j] = ToBlock(FromProtoBlock(cw.seed()));
    b->cw_left[k * L + j] = cw.control_left();
    b->cw_right[k * L + j] = cw.control_right();
  }
  for (int h = 0; h < H; ++h) {
    DPF_ASSIGN_OR_RETURN(std::vector<uint128> v, ValueCorrectionLeaves(key, h));
    auto& dst = b->value_correction[h];
    for (size_t i = 0; i < v.size(); ++i) dst[k * v.size() + i] = ToBlock(v[i]);
  }
  return OkStatus();
}

namespace {
// Runs fill(k) for k < n on up to `threads` host threads; returns the status
// of the first (lowest k) failure.
template <typename F>
Status ParallelRows(int64_t n, int threads, F fill) {
  int t = threads > 0 ? threads : static_cast<int>(std::thread::hardware_concurrency());
  t = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({t, 16, (n + 1023) / 1024})));
  std::vector<Status> first(t, OkStatus());
  std::vector<int64_t> where(t, n);
  auto work = [&](int w) {
    for (int64_t k = n * w / t, hi = n * (w + 1) / t; k < hi; ++k) {
      Status st = fill(k);
      if (!st.ok()) {
        first[w] = st;
        where[w] = k;
        return;
      }
    }
  };
  if (t == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int w = 0; w < t; ++w) pool.emplace_back(work, w);
    for (auto& th : pool) th.join();
  }
  int best = -1;
  for (int w = 0; w < t; ++w)
    if (!first[w].ok() && (best < 0 || where[w] < where[best])) best = w;
  return best < 0 ? OkStatus() : first[best];
}
}  // namespace

StatusOr<KeyBatch> DistributedPointFunction::MakeKeyBatch(Span<const DpfKey* const> keys) const {
  KeyBatch b;
  const int64_t n = static_cast<int64_t>(keys.size());
  ResizeKeyBatch(n, &b);
  DPF_RETURN_IF_ERROR(ParallelRows(n, 0, [&](int64_t k) { return FillKeyBatchRow(*keys[k], k, &b); }));
  return b;
}

StatusOr<KeyBatch> DistributedPointFunction::ParseKeyBatch(Span<const std::string_view> serialized,
                                                           int num_threads) const {
  KeyBatch b;
  const int64_t n = static_cast<int64_t>(serialized.size());
  ResizeKeyBatch(n, &b);
  DPF_RETURN_IF_ERROR(ParallelRows(n, num_threads, [&](int64_t k) -> Status {
    DpfKey key;
    if (!key.ParseFromArray(serialized[k].data(), static_cast<int>(serialized[k].size())))
      return InvalidArgumentError("Failed to parse DpfKey " + std::to_string(k));
    return FillKeyBatchRow(key, k, &b);
  }));
  return b;
}

StatusOr<std::vector<std::string>> DistributedPointFunction::SerializeKeyBatch(
    const KeyBatch& b, int num_threads) const {
  std::vector<std::string> out(b.num_keys);
  DPF_RETURN_IF_ERROR(ParallelRows(b.num_keys, num_threads, [&](int64_t k) -> Status {
    DPF_ASSIGN_OR_RETURN(DpfKey key, KeyFromBatch(b, k));
    out[k] = key.SerializeAsString();
    return OkStatus();
  }));
  return out;
}

StatusOr<DpfKey> DistributedPointFunction::KeyFromBatch(const KeyBatch& b, int64_t k) const {
  if (k < 0 || k >= b.num_keys) return InvalidArgumentError("key index out of range");
  const int H = static_cast<int>(parameters().size());
  const int L = b.num_levels;
  if (L != tree_levels_needed() - 1 || static_cast<int>(b.value_correction.size()) != H)
    return InvalidArgumentError("key batch does not match this DistributedPointFunction");
  DpfKey key;
  SetProtoBlock(FromBlock(b.seed[k]), key.mutable_seed());
  key.set_party(b.party[k]);
  auto leaves_to_values = [&](int h, RepeatedField<Value>* out) {
    const auto& f = flat_value_type(h);
    const int nl = static_cast<int>(f.leaves.size()), E = f.elements_per_block;
    std::vector<uint128> leaves(E * nl);
    for (int i = 0; i < E * nl; ++i) leaves[i] = FromBlock(b.value_correction[h][k * E * nl + i]);
    for (int e = 0; e < E; ++e) {
      int pos = 0;
      *out->Add() = dpf_internal::LeavesToValue(parameters()[h].value_type(), leaves.data() + e * nl, &pos);
    }
  };
  for (int j = 0; j < L; ++j) {
    CorrectionWord* cw = key.add_correction_words();
    SetProtoBlock(FromBlock(b.cw_seed[k * L + j]), cw->mutable_seed());
    cw->set_control_left(b.cw_left[k * L + j] != 0);
    cw->set_control_right(b.cw_right[k * L + j] != 0);
  }
  for (int h = 0; h + 1 < H; ++h)
    leaves_to_values(h, key.mutable_correction_words(hierarchy_to_tree()[h])->mutable_value_correction());
  leaves_to_values(H - 1, key.mutable_last_level_value_correction());
  return key;
}

// ------------------------------------------------------------ batched keygen
StatusOr<std::pair<KeyBatch, KeyBatch>> DistributedPointFunction::GenerateKeyBatch(
    Span<const uint128> alphas, Span<const Value> beta, Span<const uint128> root_seeds,
    int num_threads) const {
  // Checks of GenerateKeysIncremental (cc:619-655), once for the shared beta.
  const int H = static_cast<int>(parameters().size());
  if (static_cast<int>(beta.size()) != H)
    return InvalidArgumentError(
        "`beta` has to have the same size as `parameters` passed at construction");
  for (int i = 0; i < H; ++i) DPF_RETURN_IF_ERROR(validator_->ValidateValue(beta[i], i));
  const int64_t n = static_cast<int64_t>(alphas.size());
  if (!root_seeds.empty() && static_cast<int64_t>(root_seeds.size()) != 2 * n)
    return InvalidArgumentError("root_seeds must be empty or hold two seeds per alpha");
  const int last_log = parameters().back().log_domain_size();
  for (int64_t k = 0; k < n; ++k)
    if (last_log < 128 && alphas[k] >= (static_cast<uint128>(1) << last_log))
      return InvalidArgumentError("`alpha` must be smaller than the output domain size");
  std::vector<std::vector<uint128>> beta_leaves(H);
  for (int h = 0; h < H; ++h) {
    DPF_RETURN_IF_ERROR(CheckValueCorrectionKnown(h));
    DPF_ASSIGN_OR_RETURN(beta_leaves[h], dpf_internal::ValueToLeaves(parameters()[h].value_type(), beta[h]));
  }
  std::vector<uint128> seeds(root_seeds.begin(), root_seeds.end());
  if (seeds.empty() && n > 0) {
    // RAND_bytes in the reference (cc:656-658); getrandom(2) here.
    seeds.resize(2 * n);
    size_t bytes = seeds.size() * sizeof(uint128), got = 0;
    auto* p = reinterpret_cast<uint8_t*>(seeds.data());
    while (got < bytes) {
      ssize_t r = getrandom(p + got, bytes - got, 0);
      if (r <= 0) return InternalError("getrandom failed");
      got += static_cast<size_t>(r);
    }
  }
  const int T = tree_levels_needed();
  const int L = T - 1;
  std::pair<KeyBatch, KeyBatch> out;
  for (KeyBatch* b : {&out.first, &out.second}) {
    b->num_keys = n;
    b->num_levels = L;
    b->seed.resize(n);
    b->party.assign(n, b == &out.first ? 0 : 1);
    b->cw_seed.resize(n * L);
    b->cw_left.resize(n * L);
    b->cw_right.resize(n * L);
    b->value_correction.resize(H);
    for (int h = 0; h < H; ++h)
      b->value_correction[h].resize(n * flat_[h].elements_per_block * flat_[h].leaves.size());
  }
  const auto& t2h = validator_->tree_to_hierarchy();
  // One key pair (cc:656-687), written straight into row k of both batches.
  auto one = [&](int64_t k) -> Status {
    const uint128 alpha = alphas[k];
    uint128 s[2] = {seeds[2 * k], seeds[2 * k + 1]};
    bool t[2] = {false, true};
    out.first.seed[k] = ToBlock(s[0]);
    out.second.seed[k] = ToBlock(s[1]);
    auto put_vc = [&](int h, const std::vector<uint128>& vc) {
      const size_t w = vc.size();
      for (size_t i = 0; i < w; ++i) {
        out.first.value_correction[h][k * w + i] = ToBlock(vc[i]);
        out.second.value_correction[h][k * w + i] = ToBlock(vc[i]);
      }
    };
    for (int i = 1; i < T; ++i) {
      auto it = t2h.find(i - 1);
      if (it != t2h.end()) {
        const int h = it->second;
        const int shift = last_log - parameters()[h].log_domain_size();
        const uint128 alpha_prefix = shift < 128 ? alpha >> shift : 0;
        DPF_ASSIGN_OR_RETURN(std::vector<uint128> vc,
                             ComputeValueCorrectionLeaves(h, s, alpha_prefix,
                                                          MakeConstSpan(beta_leaves[h]), t[1]));
        put_vc(h, vc);
      }
      uint128 sc;
      bool ccw[2];
      DPF_RETURN_IF_ERROR(GenerateNextCore(i, alpha, s, t, &sc, ccw));
      const int64_t o = k * L + (i - 1);
      out.first.cw_seed[o] = out.second.cw_seed[o] = ToBlock(sc);
      out.first.cw_left[o] = out.second.cw_left[o] = ccw[0];
      out.first.cw_right[o] = out.second.cw_right[o] = ccw[1];
    }
    DPF_ASSIGN_OR_RETURN(std::vector<uint128> last,
                         ComputeValueCorrectionLeaves(H - 1, s, alpha,
                                                      MakeConstSpan(beta_leaves[H - 1]), t[1]));
    put_vc(H - 1, last);
    return OkStatus();
  };
  int threads = num_threads > 0 ? num_threads : static_cast<int>(std::thread::hardware_concurrency());
  threads = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(threads, (n + 255) / 256)));
  std::vector<Status> status(threads);
  auto work = [&](int w) {
    const int64_t lo = n * w / threads, hi = n * (w + 1) / threads;
    for (int64_t k = lo; k < hi; ++k) {
      Status st = one(k);
      if (!st.ok()) {
        status[w] = st;
        return;
      }
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int w = 0; w < threads; ++w) pool.emplace_back(work, w);
    for (auto& th : pool) th.join();
  }
  for (const Status& st : status) DPF_RETURN_IF_ERROR(st);
  return out;
}

// ------------------------------------------------------------ batched evaluation
namespace {
Status CheckBatch(const DeviceKeyBatch& keys, int hierarchy_level, int num_levels_needed, int H) {
  if (hierarchy_level < 0 || hierarchy_level >= H)
    return InvalidArgumentError("`hierarchy_level` out of range");
  if (keys.num_levels() != num_levels_needed || keys.num_hierarchy_levels() != H)
    return InvalidArgumentError("key batch does not match this DistributedPointFunction");
  return OkStatus();
}
}  // namespace

StatusOr<int64_t> DistributedPointFunction::EvaluateAtBatchToDevice(
    const DeviceKeyBatch& keys, int hierarchy_level, const void* device_points,
    int64_t points_per_key, bool shared_points, void* device_out, int64_t capacity_bytes,
    void* stream) const {
  const int H = static_cast<int>(parameters().size());
  DPF_RETURN_IF_ERROR(CheckBatch(keys, hierarchy_level, tree_levels_needed() - 1, H));
  if (points_per_key < 0) return InvalidArgumentError("points_per_key must be non-negative");
  const int64_t n = keys.num_keys() * points_per_key;
  if (n == 0) return int64_t{0};
  const auto& f = flat_[hierarchy_level];
  if (!device_out || capacity_bytes < n * f.packed_size)
    return InvalidArgumentError("device output buffer too small");
  const int log_domain_size = parameters()[hierarchy_level].log_domain_size();
  const int L = hierarchy_to_tree()[hierarchy_level];
  const int64_t num_points = shared_points ? points_per_key : n;
  // EvaluateAt's range check (h:861-874), on the device copy of the points.
  int64_t bad = 0;
  HIP_RETURN_IF_ERROR(dpf_hip_count_out_of_range(num_points, static_cast<const dpf_block*>(device_points),
                                                 log_domain_size, &bad, stream));
  if (bad) return InvalidArgumentError("`evaluation_points` larger than the domain size at hierarchy level " +
                                       std::to_string(hierarchy_level));
  const dpf_value_desc desc = MakeDesc(f, blocks_needed_[hierarchy_level]);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  HIP_RETURN_IF_ERROR(dpf_hip_eval_points_batch(
      keys.num_keys(), points_per_key, shared_points ? 1 : 0, L, keys.num_levels(),
      log_domain_size - L, keys.seed(),
      keys.party(), static_cast<const dpf_block*>(device_points), keys.cw_seed(), keys.cw_left(),
      keys.cw_right(), &kl, &kr, &kv, &desc, keys.value_correction(hierarchy_level), device_out,
      stream));
  return n;
}

Status DistributedPointFunction::EvaluateAtBatchSumToDevice(const DeviceKeyBatch& keys,
                                                            int hierarchy_level,
                                                            const void* device_points,
                                                            int64_t num_points, void* device_out,
                                                            void* stream) const {
  const int H = static_cast<int>(parameters().size());
  DPF_RETURN_IF_ERROR(CheckBatch(keys, hierarchy_level, tree_levels_needed() - 1, H));
  if (num_points < 0) return InvalidArgumentError("num_points must be non-negative");
  if (num_points == 0) return OkStatus();
  if (!device_out) return InvalidArgumentError("device_out must not be null");
  const auto& f = flat_[hierarchy_level];
  const int log_domain_size = parameters()[hierarchy_level].log_domain_size();
  const int L = hierarchy_to_tree()[hierarchy_level];
  int64_t bad = 0;
  HIP_RETURN_IF_ERROR(dpf_hip_count_out_of_range(num_points, static_cast<const dpf_block*>(device_points),
                                                 log_domain_size, &bad, stream));
  if (bad) return InvalidArgumentError("`evaluation_points` larger than the domain size at hierarchy level " +
                                       std::to_string(hierarchy_level));
  auto* s = scratch_.get();
  std::lock_guard<std::recursive_mutex> scratch_lock(s->mu);  // one call at a time per object
  // The workspace is zeroed and accumulated into on `stream`: an earlier call
  // on another stream must have finished with it first (device-side wait).
  DPF_RETURN_IF_ERROR(s->workspace_fence.Acquire(
      s->workspace, num_points * f.leaves.size() * 3 * sizeof(uint64_t), stream));
  const dpf_value_desc desc = MakeDesc(f, blocks_needed_[hierarchy_level]);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  HIP_RETURN_IF_ERROR(dpf_hip_eval_points_sum(
      keys.num_keys(), num_points, L, keys.num_levels(), log_domain_size - L, keys.seed(), keys.party(),
      static_cast<const dpf_block*>(device_points), keys.cw_seed(), keys.cw_left(), keys.cw_right(),
      &kl, &kr, &kv, &desc, keys.value_correction(hierarchy_level), s->workspace.as<uint64_t>(),
      device_out, stream));
  return s->workspace_fence.Mark(stream);
}

StatusOr<std::vector<uint8_t>> DistributedPointFunction::SumPackedShares(int hierarchy_level,
                                                                         const uint8_t* shares,
                                                                         int64_t num_shares,
                                                                         int64_t count) const {
  if (hierarchy_level < 0 || hierarchy_level >= static_cast<int>(parameters().size()))
    return InvalidArgumentError("`hierarchy_level` out of range");
  if (num_shares < 0 || count < 0) return InvalidArgumentError("negative sizes");
  const auto& f = flat_[hierarchy_level];
  const int nl = static_cast<int>(f.leaves.size()), esz = f.packed_size;
  std::vector<uint8_t> out(count * esz, 0);
  std::vector<uint128> acc(nl), v(nl);
  for (int64_t j = 0; j < count; ++j) {
    std::fill(acc.begin(), acc.end(), 0);
    for (int64_t r = 0; r < num_shares; ++r) {
      dpf_internal::UnpackLeaves(f, shares + (r * count + j) * esz, v.data());
      for (int i = 0; i < nl; ++i) acc[i] = dpf_internal::LeafAdd(f.leaves[i], acc[i], v[i]);
    }
    dpf_internal::PackLeaves(f, acc.data(), out.data() + j * esz);
  }
  return out;
}

}  // namespace distributed_point_functions
