// distributed_point_function.cc -- host orchestration of the DPF API.
//
// Semantics follow dpf/distributed_point_function.{h,cc} of the reference
// (file:line references below: cc = .cc, h = .h).  The hot loops -- the
// path walk (EvaluateSeeds), the subtree expansion (ExpandSeeds), leaf hashing
// (HashExpandedSeeds) and the value-correction loop -- run on the GPU through
// the C ABI of include/dpf_hip.h.  There is no CPU evaluation fallback: a
// missing GPU surfaces as an INTERNAL status from the C ABI.
#include "dpf/distributed_point_function.h"

#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <unordered_map>

#include "dpf_hip.h"
#include "host_util.h"

namespace distributed_point_functions {

using dpf_internal::AesKey;
using dpf_internal::CopyToHostSink;
using dpf_internal::CopyToHostVector;
using dpf_internal::PackedUploads;
using dpf_internal::FromBlock;
using dpf_internal::FromHip;
using dpf_internal::FromProtoBlock;
using dpf_internal::kPrgKeyLeft;
using dpf_internal::kPrgKeyRight;
using dpf_internal::kPrgKeyValue;
using dpf_internal::MakeDesc;
using dpf_internal::SetProtoBlock;
using dpf_internal::ToBlock;
using dpf_internal::U128Hash;

// Expansion starts resident on the device.
struct DistributedPointFunction::DeviceStart {
  int64_t n = 0;
  dpf_block* seeds = nullptr;
  uint8_t* ctrl = nullptr;
};

DistributedPointFunction::DistributedPointFunction(
    std::unique_ptr<dpf_internal::ProtoValidator> validator, std::vector<int> blocks_needed,
    std::vector<dpf_internal::FlatValueType> flat, Aes128FixedKeyHash prg_left,
    Aes128FixedKeyHash prg_right, Aes128FixedKeyHash prg_value)
    : validator_(std::move(validator)),
      blocks_needed_(std::move(blocks_needed)),
      flat_(std::move(flat)),
      prg_left_(prg_left),
      prg_right_(prg_right),
      prg_value_(prg_value),
      scratch_(new dpf_internal::DeviceScratch()) {}

DistributedPointFunction::~DistributedPointFunction() = default;

StatusOr<std::unique_ptr<DistributedPointFunction>> DistributedPointFunction::Create(
    const DpfParameters& parameters) {
  return CreateIncremental(Span<const DpfParameters>(&parameters, 1));
}

StatusOr<std::unique_ptr<DistributedPointFunction>> DistributedPointFunction::CreateIncremental(
    Span<const DpfParameters> parameters) {
  // cc:566-617
  DPF_ASSIGN_OR_RETURN(std::unique_ptr<dpf_internal::ProtoValidator> validator,
                       dpf_internal::ProtoValidator::Create(parameters));
  std::vector<int> blocks_needed(parameters.size());
  std::vector<dpf_internal::FlatValueType> flat(parameters.size());
  for (size_t i = 0; i < parameters.size(); ++i) {
    DPF_ASSIGN_OR_RETURN(int bits, dpf_internal::BitsNeeded(parameters[i].value_type(),
                                                             validator->parameters()[i].security_parameter()));
    blocks_needed[i] = (bits + 127) / 128;
    DPF_ASSIGN_OR_RETURN(flat[i], dpf_internal::Flatten(parameters[i].value_type()));
  }
  DPF_ASSIGN_OR_RETURN(Aes128FixedKeyHash prg_left, Aes128FixedKeyHash::Create(kPrgKeyLeft));
  DPF_ASSIGN_OR_RETURN(Aes128FixedKeyHash prg_right, Aes128FixedKeyHash::Create(kPrgKeyRight));
  DPF_ASSIGN_OR_RETURN(Aes128FixedKeyHash prg_value, Aes128FixedKeyHash::Create(kPrgKeyValue));
  std::unique_ptr<DistributedPointFunction> dpf(new DistributedPointFunction(
      std::move(validator), std::move(blocks_needed), std::move(flat), prg_left, prg_right,
      prg_value));
  // All unsigned integers are registered for backwards compatibility (cc:597-610).
  DPF_RETURN_IF_ERROR(dpf->RegisterValueType<uint8_t>());
  DPF_RETURN_IF_ERROR(dpf->RegisterValueType<uint16_t>());
  DPF_RETURN_IF_ERROR(dpf->RegisterValueType<uint32_t>());
  DPF_RETURN_IF_ERROR(dpf->RegisterValueType<uint64_t>());
  DPF_RETURN_IF_ERROR(dpf->RegisterValueType<uint128>());
  return dpf;
}

Status DistributedPointFunction::RegisterValueType(const ValueType& value_type) {
  registered_types_.insert(dpf_internal::SerializeValueTypeDeterministically(value_type));
  return OkStatus();
}

// ============================================================ key generation
StatusOr<std::vector<uint128>> DistributedPointFunction::ComputeValueCorrectionLeaves(
    int hierarchy_level, const uint128 seeds[2], uint128 alpha, Span<const uint128> beta_leaves,
    bool invert) const {
  // cc:63-99 and ComputeValueCorrectionFor<T> (value_type_helpers.h:597-631),
  // on flattened leaves: E * num_leaves values, element-major.
  const int b = blocks_needed_[hierarchy_level];
  uint128 expanded[2 * 8];
  std::vector<uint128> big;
  uint128* ex = expanded;
  if (b > 8) {
    big.resize(2 * b);
    ex = big.data();
  }
  for (int j = 0; j < b; ++j) {
    ex[j] = seeds[0] + static_cast<uint128>(j);
    ex[b + j] = seeds[1] + static_cast<uint128>(j);
  }
  DPF_RETURN_IF_ERROR(prg_value_.Evaluate(Span<const uint128>(ex, 2 * b), Span<uint128>(ex, 2 * b)));
  const DpfParameters& params = parameters()[hierarchy_level];
  const int block_index_bits = params.log_domain_size() - hierarchy_to_tree()[hierarchy_level];
  const int index_in_block =
      static_cast<int>(alpha & ((static_cast<uint128>(1) << block_index_bits) - 1));
  const dpf_internal::FlatValueType& f = flat_[hierarchy_level];
  const int nl = static_cast<int>(f.leaves.size()), E = f.elements_per_block;
  std::vector<uint128> a(E * nl), c(E * nl);
  dpf_internal::ConvertBytesToLeaves(f, reinterpret_cast<const uint8_t*>(ex), a.data());
  dpf_internal::ConvertBytesToLeaves(f, reinterpret_cast<const uint8_t*>(ex + b), c.data());
  for (int k = 0; k < nl; ++k)
    c[index_in_block * nl + k] = dpf_internal::LeafAdd(f.leaves[k], c[index_in_block * nl + k], beta_leaves[k]);
  for (int i = 0; i < E * nl; ++i) {
    const auto& leaf = f.leaves[i % nl];
    uint128 v = dpf_internal::LeafSub(leaf, c[i], a[i]);
    c[i] = invert ? dpf_internal::LeafNeg(leaf, v) : v;
  }
  return c;
}

Status DistributedPointFunction::CheckValueCorrectionKnown(int hierarchy_level) const {
  // GetValueCorrectionFunction (cc:544-559)
  const DpfParameters& params = parameters()[hierarchy_level];
  if (!registered_types_.count(dpf_internal::SerializeValueTypeDeterministically(params.value_type())))
    return FailedPreconditionError(
        "No value correction function known for the following parameters:\n" +
        params.DebugString() + "Did you call RegisterValueType<T>() with your value type?");
  return OkStatus();
}

StatusOr<std::vector<Value>> DistributedPointFunction::ComputeValueCorrection(
    int hierarchy_level, const uint128 seeds[2], uint128 alpha, const Value& beta,
    bool invert) const {
  const DpfParameters& params = parameters()[hierarchy_level];
  DPF_RETURN_IF_ERROR(CheckValueCorrectionKnown(hierarchy_level));
  DPF_ASSIGN_OR_RETURN(std::vector<uint128> beta_leaves,
                       dpf_internal::ValueToLeaves(params.value_type(), beta));
  DPF_ASSIGN_OR_RETURN(std::vector<uint128> c,
                       ComputeValueCorrectionLeaves(hierarchy_level, seeds, alpha,
                                                    MakeConstSpan(beta_leaves), invert));
  const int nl = static_cast<int>(flat_[hierarchy_level].leaves.size());
  const int E = flat_[hierarchy_level].elements_per_block;
  std::vector<Value> result;
  result.reserve(E);
  for (int e = 0; e < E; ++e) {
    int pos = 0;
    result.push_back(dpf_internal::LeavesToValue(params.value_type(), c.data() + e * nl, &pos));
  }
  return result;
}

Status DistributedPointFunction::GenerateNextCore(int tree_level, uint128 alpha, uint128 seeds[2],
                                                  bool control_bits[2], uint128* seed_correction_out,
                                                  bool ccw[2]) const {
  // cc:138-201: expand both parties' seeds, keep the child on alpha's path,
  // correct the other one away.
  uint128 ex[2][2];
  DPF_RETURN_IF_ERROR(prg_left_.Evaluate(Span<const uint128>(seeds, 2), Span<uint128>(ex[0], 2)));
  DPF_RETURN_IF_ERROR(prg_right_.Evaluate(Span<const uint128>(seeds, 2), Span<uint128>(ex[1], 2)));
  bool ec[2][2];
  for (int br = 0; br < 2; ++br)
    for (int p = 0; p < 2; ++p) {
      ec[br][p] = (ex[br][p] & 1) != 0;
      ex[br][p] &= ~static_cast<uint128>(1);
    }
  const int last_log = parameters().back().log_domain_size();
  bool bit = false;
  if (last_log - tree_level < 128) bit = ((alpha >> (last_log - tree_level)) & 1) != 0;
  const int keep = bit ? 1 : 0, lose = bit ? 0 : 1;
  const uint128 seed_correction = ex[lose][0] ^ ex[lose][1];
  ccw[0] = ec[0][0] ^ ec[0][1] ^ bit ^ 1;
  ccw[1] = ec[1][0] ^ ec[1][1] ^ bit;
  for (int p = 0; p < 2; ++p) {
    seeds[p] = ex[keep][p] ^ (control_bits[p] ? seed_correction : 0);
    control_bits[p] = ec[keep][p] ^ (control_bits[p] && ccw[keep]);
  }
  *seed_correction_out = seed_correction;
  return OkStatus();
}

Status DistributedPointFunction::GenerateNext(int tree_level, uint128 alpha, Span<const Value> beta,
                                              uint128 seeds[2], bool control_bits[2],
                                              DpfKey keys[2]) const {
  // cc:103-204 (line numbers of arXiv 2012.14884 Fig. 11 in the reference comments)
  CorrectionWord* cw = keys[0].add_correction_words();
  const auto& t2h = validator_->tree_to_hierarchy();
  const int last_log = parameters().back().log_domain_size();
  auto it = t2h.find(tree_level - 1);
  if (it != t2h.end()) {
    const int h = it->second;
    uint128 alpha_prefix = 0;
    const int shift = last_log - parameters()[h].log_domain_size();
    if (shift < 128) alpha_prefix = alpha >> shift;
    DPF_ASSIGN_OR_RETURN(std::vector<Value> vc,
                         ComputeValueCorrection(h, seeds, alpha_prefix, beta[h], control_bits[1]));
    for (Value& v : vc) *cw->add_value_correction() = std::move(v);
  }
  uint128 seed_correction;
  bool ccw[2];
  DPF_RETURN_IF_ERROR(GenerateNextCore(tree_level, alpha, seeds, control_bits, &seed_correction, ccw));
  SetProtoBlock(seed_correction, cw->mutable_seed());
  cw->set_control_left(ccw[0]);
  cw->set_control_right(ccw[1]);
  *keys[1].add_correction_words() = *cw;
  return OkStatus();
}

StatusOr<std::pair<DpfKey, DpfKey>> DistributedPointFunction::GenerateKeysIncremental(
    uint128 alpha, Span<const Value> beta) {
  uint128 seeds[2];
  // RAND_bytes in the reference (cc:656-658); getrandom(2) here.
  if (getrandom(seeds, sizeof(seeds), 0) != static_cast<ssize_t>(sizeof(seeds)))
    return InternalError("getrandom failed");
  return GenerateKeysIncrementalWithSeeds(alpha, beta, seeds[0], seeds[1]);
}

StatusOr<std::pair<DpfKey, DpfKey>> DistributedPointFunction::GenerateKeysIncrementalWithSeeds(
    uint128 alpha, Span<const Value> beta, uint128 seed_0, uint128 seed_1) {
  // cc:619-687
  const int H = static_cast<int>(parameters().size());
  if (static_cast<int>(beta.size()) != H)
    return InvalidArgumentError(
        "`beta` has to have the same size as `parameters` passed at construction");
  for (int i = 0; i < H; ++i) DPF_RETURN_IF_ERROR(validator_->ValidateValue(beta[i], i));
  const int last_log = parameters().back().log_domain_size();
  if (last_log < 128 && alpha >= (static_cast<uint128>(1) << last_log))
    return InvalidArgumentError("`alpha` must be smaller than the output domain size");
  DpfKey keys[2];
  keys[0].set_party(0);
  keys[1].set_party(1);
  uint128 seeds[2] = {seed_0, seed_1};
  SetProtoBlock(seeds[0], keys[0].mutable_seed());
  SetProtoBlock(seeds[1], keys[1].mutable_seed());
  bool control_bits[2] = {false, true};
  const int T = tree_levels_needed();
  keys[0].mutable_correction_words()->Reserve(T - 1);
  keys[1].mutable_correction_words()->Reserve(T - 1);
  for (int i = 1; i < T; ++i)
    DPF_RETURN_IF_ERROR(GenerateNext(i, alpha, beta, seeds, control_bits, keys));
  DPF_ASSIGN_OR_RETURN(std::vector<Value> last,
                       ComputeValueCorrection(H - 1, seeds, alpha, beta.back(), control_bits[1]));
  for (const Value& v : last) {
    *keys[0].add_last_level_value_correction() = v;
    *keys[1].add_last_level_value_correction() = v;
  }
  return std::make_pair(std::move(keys[0]), std::move(keys[1]));
}

StatusOr<EvaluationContext> DistributedPointFunction::CreateEvaluationContext(DpfKey key) const {
  // cc:689-704
  DPF_RETURN_IF_ERROR(validator_->ValidateDpfKey(key));
  EvaluationContext result;
  for (const DpfParameters& p : parameters()) *result.add_parameters() = p;
  *result.mutable_key() = std::move(key);
  result.set_previous_hierarchy_level(-1);
  return result;
}

// ============================================================ evaluation
StatusOr<std::vector<uint128>> DistributedPointFunction::ValueCorrectionLeaves(const DpfKey& key,
                                                                               int h) const {
  // h:761-780 / h:883-902
  const RepeatedField<Value>* vc;
  if (h < static_cast<int>(parameters().size()) - 1) {
    vc = &key.correction_words(hierarchy_to_tree()[h]).value_correction();
  } else {
    vc = &key.last_level_value_correction();
  }
  return dpf_internal::ValuesToLeafArray(parameters()[h].value_type(), flat_[h], *vc);
}

namespace {

// Correction words [start, stop) of `key` added to a packed upload.
struct PackedCws {
  size_t seed, left, right;
};
PackedCws AddCorrectionWords(const DpfKey& key, int start, int stop, PackedUploads& up) {
  const int L = stop - start;
  std::vector<dpf_block> seeds(std::max(L, 1));
  std::vector<uint8_t> cl(std::max(L, 1)), cr(std::max(L, 1));
  for (int j = 0; j < L; ++j) {
    const CorrectionWord& cw = key.correction_words(start + j);
    seeds[j] = ToBlock(FromProtoBlock(cw.seed()));
    cl[j] = cw.control_left();
    cr[j] = cw.control_right();
  }
  PackedCws o;
  o.seed = up.Add(seeds.data(), seeds.size());
  o.left = up.Add(cl.data(), cl.size());
  o.right = up.Add(cr.data(), cr.size());
  return o;
}

// Phase split of the prefix walk (ComputePartialEvaluations), printed at exit
// with DPF_HOST_TIMING: the lookup of the stored evaluations, the image and
// its upload, the walk on the device (with the walked seeds' D2H), and the
// context rewrite.
struct WalkTiming {
  double t[4] = {0, 0, 0, 0};
  long calls = 0;
  ~WalkTiming() {
    if (calls > 0 && std::getenv("DPF_HOST_TIMING"))
      std::fprintf(stderr,
                   "[prefix walk host timing] calls=%ld per call: lookup=%.2fus upload=%.2fus "
                   "device=%.2fus context=%.2fus\n",
                   calls, t[0] * 1e6 / calls, t[1] * 1e6 / calls, t[2] * 1e6 / calls,
                   t[3] * 1e6 / calls);
  }
};
WalkTiming g_walk_timing;
std::mutex g_walk_timing_mu;
const bool g_walk_timing_on = std::getenv("DPF_HOST_TIMING") != nullptr;
struct WalkClock {
  std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
  double t[4] = {0, 0, 0, 0};
  void mark(int phase) {
    if (!g_walk_timing_on) return;
    auto now = std::chrono::steady_clock::now();
    t[phase] += std::chrono::duration<double>(now - last).count();
    last = now;
  }
  ~WalkClock() {
    if (!g_walk_timing_on) return;
    std::lock_guard<std::mutex> lock(g_walk_timing_mu);
    ++g_walk_timing.calls;
    for (int i = 0; i < 4; ++i) g_walk_timing.t[i] += t[i];
  }
};
}  // namespace

Status DistributedPointFunction::ComputePartialEvaluations(
    Span<const uint128> prefixes, int hierarchy_level, bool update_ctx, EvaluationContext& ctx,
    DeviceStart* out, void* stream, const std::function<Status()>& before_device) const {
  // cc:351-453
  const int64_t n = static_cast<int64_t>(prefixes.size());
  int start_level = hierarchy_to_tree()[ctx.partial_evaluations_level()];
  const int stop_level = hierarchy_to_tree()[hierarchy_level];
  auto* s = scratch_.get();
  std::lock_guard<std::recursive_mutex> scratch_lock(s->mu);  // one call at a time per object
  WalkClock wclk;
  // The walk's inputs -- start seeds, control bits, paths, correction words --
  // go up as ONE packed image (read in place by the kernel when small); the
  // start seeds and control bits are written straight into it.
  PackedUploads& pu = s->packed_pe;
  DPF_RETURN_IF_ERROR(pu.Reset());
  const int max_levels = std::max(stop_level - start_level, stop_level);
  pu.Prepare(static_cast<size_t>(std::max<int64_t>(n, 1)) * (2 * sizeof(dpf_block) + 1) +
             static_cast<size_t>(max_levels + 1) * (sizeof(dpf_block) + 2) + 6 * 256);
  size_t o_seed, o_ctrl, o_paths;
  dpf_block* seeds = pu.Reserve<dpf_block>(std::max<int64_t>(n, 1), &o_seed);
  uint8_t* ctrl = pu.Reserve<uint8_t>(std::max<int64_t>(n, 1), &o_ctrl);
  dpf_block* paths = pu.Reserve<dpf_block>(std::max<int64_t>(n, 1), &o_paths);
  if (ctx.partial_evaluations_size() > 0 && start_level <= stop_level) {
    const int shift = stop_level - start_level;
    auto parent_of = [&](int64_t i) -> uint128 { return shift < 128 ? prefixes[i] >> shift : 0; };
    const auto& pe = ctx.partial_evaluations();
    const int64_t m = pe.size();
    // Sorted fast path (the usual hierarchical case: both the stored prefixes
    // and the lookups come out of EvaluateUntil in ascending order): two
    // chunked passes on host threads instead of a hash map.  The first checks
    // that the stored prefixes ascend and applies the reference's duplicate
    // check (cc:365-383) to adjacent equal ones; the second checks that the
    // lookups' parents ascend and merges them against the stored prefixes,
    // with the reference's lookup error (cc:392-407).  Either order broken:
    // the hash map below redoes the lookup.
    auto stored_at = [&](int64_t j) -> uint128 { return FromProtoBlock(pe[j].prefix()); };
    const int chunks_m = dpf_internal::NumChunks(m), chunks_n = dpf_internal::NumChunks(n);
    std::vector<char> ok_m(chunks_m, 1), dup_ok(chunks_m, 1);
    dpf_internal::ParallelChunks(m, chunks_m, [&](int c, int64_t lo, int64_t hi) {
      if (lo >= hi) return;
      const int64_t first = std::max<int64_t>(lo, 1);
      uint128 prev = stored_at(first - 1);
      for (int64_t j = first; j < hi; ++j) {
        const uint128 cur = stored_at(j);
        if (prev > cur) { ok_m[c] = 0; return; }
        if (prev == cur && dup_ok[c] &&
            (FromProtoBlock(pe[j - 1].seed()) != FromProtoBlock(pe[j].seed()) ||
             pe[j - 1].control_bit() != pe[j].control_bit()))
          dup_ok[c] = 0;
        prev = cur;
      }
    });
    auto all = [](const std::vector<char>& v) {
      return std::all_of(v.begin(), v.end(), [](char x) { return x != 0; });
    };
    bool sorted = all(ok_m);
    if (sorted && !all(dup_ok))
      return InvalidArgumentError(
          "Duplicate prefix in `ctx.partial_evaluations()` with mismatching seed or control bit");
    std::vector<char> ok_n(chunks_n, 1), missing(chunks_n, 0);
    if (sorted) {
      dpf_internal::ParallelChunks(n, chunks_n, [&](int c, int64_t lo, int64_t hi) {
        if (lo >= hi) return;
        int64_t j = std::partition_point(pe.begin(), pe.end(),
                                         [&](const PartialEvaluation& e) {
                                           return FromProtoBlock(e.prefix()) < parent_of(lo);
                                         }) -
                    pe.begin();
        uint128 prev = lo > 0 ? parent_of(lo - 1) : 0;
        for (int64_t i = lo; i < hi; ++i) {
          const uint128 want = parent_of(i);
          if (want < prev) { ok_n[c] = 0; return; }
          prev = want;
          while (j < m && stored_at(j) < want) ++j;
          if (j == m || stored_at(j) != want) { missing[c] = 1; return; }
          seeds[i] = ToBlock(FromProtoBlock(pe[j].seed()));
          ctrl[i] = pe[j].control_bit();
        }
      });
      sorted = all(ok_n);
    }
    if (sorted) {
      if (std::any_of(missing.begin(), missing.end(), [](char x) { return x != 0; }))
        return InvalidArgumentError("Prefix not present in ctx.partial_evaluations at hierarchy level " +
                                    std::to_string(hierarchy_level));
    } else {
    std::unordered_map<uint128, std::pair<uint128, bool>, U128Hash> previous;
    previous.reserve(ctx.partial_evaluations_size() * 2);
    for (const PartialEvaluation& e : ctx.partial_evaluations()) {
      auto value = std::make_pair(FromProtoBlock(e.seed()), e.control_bit());
      auto [it, inserted] = previous.try_emplace(FromProtoBlock(e.prefix()), value);
      if (!inserted && it->second != value)
        return InvalidArgumentError(
            "Duplicate prefix in `ctx.partial_evaluations()` with mismatching seed or control bit");
    }
    for (int64_t i = 0; i < n; ++i) {
      uint128 previous_prefix = 0;
      if (stop_level - start_level < 128) previous_prefix = prefixes[i] >> (stop_level - start_level);
      auto it = previous.find(previous_prefix);
      if (it == previous.end())
        return InvalidArgumentError("Prefix not present in ctx.partial_evaluations at hierarchy level " +
                                    std::to_string(hierarchy_level));
      seeds[i] = ToBlock(it->second.first);
      ctrl[i] = it->second.second;
    }
    }
  } else {
    const dpf_block root = ToBlock(FromProtoBlock(ctx.key().seed()));
    const uint8_t party = static_cast<uint8_t>(ctx.key().party() & 1);
    for (int64_t i = 0; i < n; ++i) {
      seeds[i] = root;
      ctrl[i] = party;
    }
    start_level = 0;
  }
  // Everything that can fail on the host is checked before device work starts.
  if (before_device) DPF_RETURN_IF_ERROR(before_device());
  wclk.mark(0);
  dpf_internal::ParallelFor(n, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) paths[i] = ToBlock(prefixes[i]);
  });
  const PackedCws o_cw = AddCorrectionWords(ctx.key(), start_level, stop_level, pu);
  DPF_RETURN_IF_ERROR(pu.Commit(stream));
  wclk.mark(1);
  dpf_block* dev_seed = pu.Ptr<dpf_block>(o_seed);
  uint8_t* dev_ctrl = pu.Ptr<uint8_t>(o_ctrl);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight);
  HIP_RETURN_IF_ERROR(dpf_hip_eval_paths(
      n, stop_level - start_level, dev_seed, dev_ctrl, pu.Ptr<dpf_block>(o_paths),
      pu.Ptr<dpf_block>(o_cw.seed), pu.Ptr<uint8_t>(o_cw.left), pu.Ptr<uint8_t>(o_cw.right), &kl,
      &kr, dev_seed, dev_ctrl, stream));
  // Whatever reads the walked seeds later (the caller's expansion) is
  // ordered after this on `stream`; the caller marks the image used again
  // after its launches (MarkStartUsed) so the next call waits for them too.
  DPF_RETURN_IF_ERROR(pu.MarkUsed(stream));
  if (!update_ctx) ctx.clear_partial_evaluations();
  if (update_ctx) {
    // The walked seeds and control bits back into the host image (in place
    // when the kernel wrote them there), then into the context.
    const size_t span = o_ctrl + static_cast<size_t>(n) - o_seed;
    if (pu.zero_copy()) {
      HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(stream));
    } else {
      HIP_RETURN_IF_ERROR(dpf_hip_memcpy_d2h(seeds, dev_seed, span, stream));
    }
    wclk.mark(2);
    // Resized, not cleared first: a context whose previous level stored as
    // many partial evaluations constructs none, and every field is rewritten.
    auto& pes = ctx.mutable_partial_evaluations()->vec();
    pes.resize(n);
    dpf_internal::ParallelFor(n, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) {
        PartialEvaluation* e = &pes[i];
        SetProtoBlock(prefixes[i], e->mutable_prefix());
        SetProtoBlock(FromBlock(seeds[i]), e->mutable_seed());
        e->set_control_bit(ctrl[i] != 0);
      }
    });
    wclk.mark(3);
  }
  ctx.set_partial_evaluations_level(hierarchy_level);
  out->n = n;
  out->seeds = dev_seed;
  out->ctrl = dev_ctrl;
  return OkStatus();
}

StatusOr<int64_t> DistributedPointFunction::OutputElements(int hierarchy_level,
                                                           int64_t num_prefixes,
                                                           int previous_hierarchy_level) const {
  const int prev_log =
      num_prefixes == 0 ? 0 : parameters()[previous_hierarchy_level].log_domain_size();
  const int log = parameters()[hierarchy_level].log_domain_size();
  if (log - prev_log > 62)
    return InvalidArgumentError(
        "Output size would be larger than 2**62. Please evaluate fewer hierarchy levels at once.");
  return std::max<int64_t>(num_prefixes, 1) << (log - prev_log);
}

namespace {
// Host-phase timing of EvaluateUntil, printed at exit when DPF_HOST_TIMING is
// set: where a small call's microseconds go (validation, uploads, launch,
// output copy).
struct UntilTiming {
  double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long calls = 0;
  ~UntilTiming() {
    const double n = static_cast<double>(calls - 100);
    if (calls > 100 && std::getenv("DPF_HOST_TIMING"))
      std::fprintf(stderr,
                   "[EvaluateUntil host timing] calls=%ld per call: validate=%.2fus "
                   "dedup=%.2fus walk+vcw=%.2fus pack=%.2fus commit=%.2fus launch=%.2fus "
                   "reserve=%.2fus copy=%.2fus\n",
                   calls, t[7] * 1e6 / n, t[0] * 1e6 / n, t[5] * 1e6 / n, t[6] * 1e6 / n,
                   t[1] * 1e6 / n, t[2] * 1e6 / n, t[3] * 1e6 / n, t[4] * 1e6 / n);
  }
};
UntilTiming g_until_timing;
std::mutex g_until_timing_mu;  // the counters are process-wide; calls on several objects race
const bool g_until_timing_on = std::getenv("DPF_HOST_TIMING") != nullptr;
struct UntilClock {
  std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
  void count_call() {
    if (!g_until_timing_on) return;
    std::lock_guard<std::mutex> lock(g_until_timing_mu);
    ++g_until_timing.calls;
  }
  void mark(int phase) {
    if (!g_until_timing_on) return;
    auto now = std::chrono::steady_clock::now();
    // The first 100 calls (allocations, page-locked buffers) are not counted.
    std::lock_guard<std::mutex> lock(g_until_timing_mu);
    if (g_until_timing.calls > 100)
      g_until_timing.t[phase] += std::chrono::duration<double>(now - last).count();
    last = now;
  }
};
}  // namespace

namespace {
// The split first-call expansion (EvaluateUntilCore): 2^kSplitLevels subtree
// launches.  DPF_EVAL_SPLIT=0 (read per call) launches the whole tree at
// once: an A/B hook.
constexpr int kSplitLevels = 3;
constexpr int kSplitParts = 1 << kSplitLevels;
bool SplitOn() {
  const char* v = std::getenv("DPF_EVAL_SPLIT");
  return !(v && v[0] == '0');
}
}  // namespace

Status DistributedPointFunction::EvaluateUntilCore(int hierarchy_level, Span<const uint128> prefixes,
                                                   EvaluationContext& ctx,
                                                   const ValueType* requested_type,
                                                   void* device_out, int64_t capacity_bytes,
                                                   void* stream, const HostSink* host_out,
                                                   int64_t* num_elements) const {
  // h:641-837
  UntilClock clk;
  DPF_RETURN_IF_ERROR(validator_->ValidateEvaluationContext(ctx));
  const int H = static_cast<int>(parameters().size());
  if (hierarchy_level < 0 || hierarchy_level >= H)
    return InvalidArgumentError(
        "`hierarchy_level` must be non-negative and less than parameters_.size()");
  if (requested_type) {
    DPF_ASSIGN_OR_RETURN(bool eq, dpf_internal::ValueTypesAreEqual(
                                      *requested_type, parameters()[hierarchy_level].value_type()));
    if (!eq) return InvalidArgumentError("Value type T doesn't match parameters at `hierarchy_level`");
  }
  if (hierarchy_level <= ctx.previous_hierarchy_level())
    return InvalidArgumentError(
        "`hierarchy_level` must be greater than `ctx.previous_hierarchy_level`");
  if ((ctx.previous_hierarchy_level() < 0) != prefixes.empty())
    return InvalidArgumentError(
        "`prefixes` must be empty if and only if this is the first call with `ctx`.");
  int previous_log_domain_size = 0;
  const int previous_hierarchy_level = ctx.previous_hierarchy_level();
  if (!prefixes.empty()) {
    previous_log_domain_size = parameters()[previous_hierarchy_level].log_domain_size();
    if (previous_log_domain_size < 128) {
      // The first out-of-range prefix is the one reported, as the reference's
      // loop does; the scan runs on host threads.
      const uint128 limit = static_cast<uint128>(1) << previous_log_domain_size;
      const int64_t np = static_cast<int64_t>(prefixes.size());
      const int chunks = dpf_internal::NumChunks(np);
      std::vector<int64_t> first_bad(chunks, np);
      dpf_internal::ParallelChunks(np, chunks, [&](int c, int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i)
          if (prefixes[i] >= limit) { first_bad[c] = i; return; }
      });
      const int64_t bad = *std::min_element(first_bad.begin(), first_bad.end());
      if (bad < np)
        return InvalidArgumentError("Index " + Uint128ToString(prefixes[bad]) +
                                    " out of range for hierarchy level " +
                                    std::to_string(previous_hierarchy_level));
    }
  }
  const int log_domain_size = parameters()[hierarchy_level].log_domain_size();
  if (log_domain_size - previous_log_domain_size > 62)
    return InvalidArgumentError(
        "Output size would be larger than 2**62. Please evaluate fewer hierarchy levels at once.");

  // The output size is known before anything touches `ctx`: a too-small
  // device buffer is rejected here, so the caller can retry with the same
  // context and a larger buffer.
  const int64_t num_prefixes = static_cast<int64_t>(prefixes.size());
  {
    const int64_t per_prefix = int64_t{1} << (log_domain_size - previous_log_domain_size);
    const int64_t out_total =
        num_prefixes == 0
            ? (int64_t{1} << hierarchy_to_tree()[hierarchy_level]) *
                  corrected_elements_per_block(hierarchy_level)
            : num_prefixes * per_prefix;
    if (device_out && capacity_bytes < out_total * flat_[hierarchy_level].packed_size)
      return InvalidArgumentError("device output buffer too small");
  }

  clk.mark(7);
  auto* s = scratch_.get();
  std::lock_guard<std::recursive_mutex> scratch_lock(s->mu);  // one call at a time per object
  // Unique tree indices of the prefixes, in first-seen order (h:718-742).
  std::vector<uint128>& tree_indices = s->tree_indices;
  std::vector<std::pair<int64_t, int>>& prefix_map = s->prefix_map;
  if (num_prefixes > 0) {
    dpf_internal::DedupTreeIndices(prefixes,
                                   parameters()[previous_hierarchy_level].log_domain_size() -
                                       hierarchy_to_tree()[previous_hierarchy_level],
                                   &tree_indices, &prefix_map);
  } else {
    tree_indices.clear();
    prefix_map.clear();
  }

  // ExpandAndUpdateContext (cc:455-498): starting seeds on the device.  The
  // value correction of this level (h:761-780) is parsed before device work.
  clk.count_call();
  clk.mark(0);
  std::vector<uint128> vcw;
  auto parse_vcw = [&]() -> Status {
    DPF_ASSIGN_OR_RETURN(vcw, ValueCorrectionLeaves(ctx.key(), hierarchy_level));
    return OkStatus();
  };
  DeviceStart start;
  int start_level = 0;
  PackedUploads& up = s->packed;
  DPF_RETURN_IF_ERROR(up.Reset());
  size_t o_root = 0, o_party = 0;
  if (tree_indices.empty()) {
    DPF_RETURN_IF_ERROR(parse_vcw());
    const dpf_block root = ToBlock(FromProtoBlock(ctx.key().seed()));
    const uint8_t party = static_cast<uint8_t>(ctx.key().party() & 1);
    o_root = up.Add(&root, 1);
    o_party = up.Add(&party, 1);
    start.n = 1;
  } else {
    const bool update_ctx = hierarchy_level < H - 1;
    DPF_RETURN_IF_ERROR(ComputePartialEvaluations(MakeConstSpan(tree_indices),
                                                  previous_hierarchy_level, update_ctx, ctx,
                                                  &start, stream, parse_vcw));
    start_level = hierarchy_to_tree()[previous_hierarchy_level];
  }
  const int stop_level = hierarchy_to_tree()[hierarchy_level];
  ctx.set_previous_hierarchy_level(hierarchy_level);
  const dpf_internal::FlatValueType& f = flat_[hierarchy_level];
  const int cepb = corrected_elements_per_block(hierarchy_level);
  const int esz = f.packed_size;
  const int L = stop_level - start_level;
  const int64_t expansion = start.n << L;
  const int64_t corrected = expansion * cepb;
  const int64_t outputs_per_prefix = int64_t{1} << (log_domain_size - previous_log_domain_size);
  const int64_t total = num_prefixes == 0 ? corrected : num_prefixes * outputs_per_prefix;
  *num_elements = total;

  clk.mark(5);
  std::vector<dpf_block> vcw_blocks(vcw.size());
  for (size_t i = 0; i < vcw.size(); ++i) vcw_blocks[i] = ToBlock(vcw[i]);
  const size_t o_vcw = up.Add(vcw_blocks.data(), vcw_blocks.size());
  const PackedCws o_cw = AddCorrectionWords(ctx.key(), start_level, stop_level, up);
  // A first call's output of >= DPF_HIP_REGISTER_MIN_BYTES bound for a fresh
  // host vector: the expansion runs as kSplitParts subtree launches, each
  // followed by an event, and the copy of part j (dpf_hip_memcpy_d2h_staged_after)
  // overlaps the expansion of the later parts (2^30 uint64: the 17 ms kernel
  // no longer precedes the 150 ms DMA).
  const bool split = host_out && host_out->grow && tree_indices.empty() && SplitOn() &&
                     L >= kSplitLevels + 12 &&
                     static_cast<size_t>(total) * esz >= DPF_HIP_REGISTER_MIN_BYTES;
  size_t o_sub_seed = 0, o_sub_ctrl = 0, o_sub_path = 0;
  PackedCws o_top{}, o_sub{};
  if (split) {
    const dpf_block root = ToBlock(FromProtoBlock(ctx.key().seed()));
    const uint8_t party = static_cast<uint8_t>(ctx.key().party() & 1);
    std::vector<dpf_block> roots(kSplitParts, root), paths(kSplitParts);
    std::vector<uint8_t> parties(kSplitParts, party);
    for (int j = 0; j < kSplitParts; ++j) paths[j] = ToBlock(static_cast<uint128>(j));
    o_sub_seed = up.Add(roots.data(), roots.size());
    o_sub_ctrl = up.Add(parties.data(), parties.size());
    o_sub_path = up.Add(paths.data(), paths.size());
    o_top = AddCorrectionWords(ctx.key(), 0, kSplitLevels, up);
    o_sub = AddCorrectionWords(ctx.key(), kSplitLevels, stop_level, up);
  }
  clk.mark(6);
  DPF_RETURN_IF_ERROR(up.Commit(stream));
  if (tree_indices.empty()) {
    start.seeds = up.Ptr<dpf_block>(o_root);
    start.ctrl = up.Ptr<uint8_t>(o_party);
  }

  // Is the gather (h:822-835) the identity?  Yes when every prefix maps to its
  // own tree index in order and covers the whole expanded block range.
  const int64_t blocks_per_tree_prefix = num_prefixes ? (expansion / start.n) : 0;
  bool identity = true;
  if (num_prefixes > 0) {
    identity = (outputs_per_prefix == blocks_per_tree_prefix * cepb) &&
               static_cast<int64_t>(tree_indices.size()) == num_prefixes;
    if (identity) {
      const int chunks = dpf_internal::NumChunks(num_prefixes);
      std::vector<char> ok(chunks, 1);
      dpf_internal::ParallelChunks(num_prefixes, chunks, [&](int c, int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i)
          if (prefix_map[i].first != i || prefix_map[i].second != 0) { ok[c] = 0; return; }
      });
      identity = std::all_of(ok.begin(), ok.end(), [](char x) { return x != 0; });
    }
  }
  // A small host result is written by the kernels straight into page-locked
  // memory (PinnedOut): no D2H copy.
  void* small = (!device_out && host_out) ? s->small_out.Get(static_cast<size_t>(total) * esz)
                                          : nullptr;
  void* expand_out = nullptr;
  if (device_out && identity) {
    if (capacity_bytes < total * esz) return InvalidArgumentError("device output buffer too small");
    expand_out = device_out;
  } else if (small && identity) {
    expand_out = small;
  } else {
    DPF_RETURN_IF_ERROR(s->out.Reserve(static_cast<size_t>(corrected) * esz));
    expand_out = s->out.get();
  }
  const dpf_value_desc desc = MakeDesc(f, blocks_needed_[hierarchy_level]);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  clk.mark(1);
  dpf_internal::PartEvents parts;
  if (split) {
    // The subtree roots at depth kSplitLevels (EvaluateSeeds, in place), then
    // one expansion per subtree into its slice of the output.
    dpf_block* sub_seed = up.Ptr<dpf_block>(o_sub_seed);
    uint8_t* sub_ctrl = up.Ptr<uint8_t>(o_sub_ctrl);
    HIP_RETURN_IF_ERROR(dpf_hip_eval_paths(kSplitParts, kSplitLevels, sub_seed, sub_ctrl,
                                           up.Ptr<dpf_block>(o_sub_path), up.Ptr<dpf_block>(o_top.seed),
                                           up.Ptr<uint8_t>(o_top.left), up.Ptr<uint8_t>(o_top.right),
                                           &kl, &kr, sub_seed, sub_ctrl, stream));
    const size_t part_bytes = static_cast<size_t>(corrected / kSplitParts) * esz;
    for (int j = 0; j < kSplitParts; ++j) {
      HIP_RETURN_IF_ERROR(dpf_hip_expand(
          1, sub_seed + j, sub_ctrl + j, L - kSplitLevels, up.Ptr<dpf_block>(o_sub.seed),
          up.Ptr<uint8_t>(o_sub.left), up.Ptr<uint8_t>(o_sub.right), &kl, &kr, &kv, &desc, cepb,
          up.Ptr<dpf_block>(o_vcw), ctx.key().party() & 1,
          static_cast<char*>(expand_out) + j * part_bytes, stream));
      DPF_RETURN_IF_ERROR(parts.Record(part_bytes * (j + 1), stream));
    }
  } else {
    HIP_RETURN_IF_ERROR(dpf_hip_expand(start.n, start.seeds, start.ctrl, L,
                                       up.Ptr<dpf_block>(o_cw.seed), up.Ptr<uint8_t>(o_cw.left),
                                       up.Ptr<uint8_t>(o_cw.right), &kl, &kr, &kv, &desc, cepb,
                                       up.Ptr<dpf_block>(o_vcw), ctx.key().party() & 1, expand_out,
                                       stream));
  }
  DPF_RETURN_IF_ERROR(up.MarkUsed(stream));
  // The expansion read its start seeds out of the walk's image: the next
  // call's ComputePartialEvaluations must not rewrite it before that is done.
  if (!tree_indices.empty()) DPF_RETURN_IF_ERROR(s->packed_pe.MarkUsed(stream));
  void* result = expand_out;
  if (!identity) {
    std::vector<int64_t> offsets(num_prefixes);
    dpf_internal::ParallelFor(num_prefixes, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i)
        offsets[i] = prefix_map[i].first * blocks_per_tree_prefix * cepb +
                     prefix_map[i].second * outputs_per_prefix;
    });
    DPF_RETURN_IF_ERROR(s->Upload(s->offsets, offsets.data(), offsets.size(), stream));
    if (device_out) {
      if (capacity_bytes < total * esz) return InvalidArgumentError("device output buffer too small");
      result = device_out;
    } else if (small) {
      result = small;
    } else {
      DPF_RETURN_IF_ERROR(s->gathered.Reserve(static_cast<size_t>(total) * esz));
      result = s->gathered.get();
    }
    HIP_RETURN_IF_ERROR(dpf_hip_gather(num_prefixes, outputs_per_prefix, esz,
                                       s->offsets.as<int64_t>(), expand_out, result, stream));
  }
  clk.mark(2);
  if (!device_out) {
    const size_t bytes = static_cast<size_t>(total) * esz;
    if (small) {
      clk.mark(3);
      DPF_RETURN_IF_ERROR(dpf_internal::ConsumePinnedOut(*host_out, small, bytes, stream));
      clk.mark(4);
      return OkStatus();
    }
    void* dst = host_out->reserve(bytes);
    clk.mark(3);
    HIP_RETURN_IF_ERROR(CopyToHostSink(*host_out, dst, result, bytes, stream, &parts));
    clk.mark(4);
  }
  return OkStatus();
}

StatusOr<std::vector<uint8_t>> DistributedPointFunction::EvaluateUntilPacked(
    int hierarchy_level, Span<const uint128> prefixes, EvaluationContext& ctx,
    const ValueType* requested_type) const {
  std::vector<uint8_t> out;
  int64_t n = 0;
  const HostSink sink = dpf_internal::VectorSink(&out);
  DPF_RETURN_IF_ERROR(EvaluateUntilCore(hierarchy_level, prefixes, ctx, requested_type, nullptr, 0,
                                        nullptr, &sink, &n));
  return out;
}

Status DistributedPointFunction::EvaluateUntilToHost(int hierarchy_level,
                                                     Span<const uint128> prefixes,
                                                     EvaluationContext& ctx,
                                                     const ValueType* requested_type,
                                                     const HostSink& sink) const {
  int64_t n = 0;
  return EvaluateUntilCore(hierarchy_level, prefixes, ctx, requested_type, nullptr, 0, nullptr,
                           &sink, &n);
}

StatusOr<int64_t> DistributedPointFunction::EvaluateUntilToDevice(
    int hierarchy_level, Span<const uint128> prefixes, EvaluationContext& ctx, void* device_out,
    int64_t capacity_bytes, void* stream, const ValueType* requested_type) const {
  if (!device_out) return InvalidArgumentError("device_out must not be null");
  int64_t n = 0;
  DPF_RETURN_IF_ERROR(EvaluateUntilCore(hierarchy_level, prefixes, ctx, requested_type, device_out,
                                        capacity_bytes, stream, nullptr, &n));
  return n;
}

void DistributedPointFunction::ReleaseScratch() {
  // The old scratch's destructors wait for the events of its images and free
  // its buffers (long-lived objects kept their largest call's).
  std::unique_ptr<dpf_internal::DeviceScratch> fresh(new dpf_internal::DeviceScratch());
  {
    std::lock_guard<std::recursive_mutex> lock(scratch_->mu);
  }
  scratch_.swap(fresh);
}

StatusOr<int64_t> DistributedPointFunction::EvaluateShardToDevice(
    int hierarchy_level, int64_t shard, int64_t num_shards, EvaluationContext& ctx,
    void* device_out, int64_t capacity_bytes, void* stream) const {
  DPF_RETURN_IF_ERROR(validator_->ValidateEvaluationContext(ctx));
  const int H = static_cast<int>(parameters().size());
  if (hierarchy_level < 0 || hierarchy_level >= H)
    return InvalidArgumentError(
        "`hierarchy_level` must be non-negative and less than parameters_.size()");
  if (ctx.previous_hierarchy_level() >= 0)
    return InvalidArgumentError("sharded evaluation is only defined for the first call with `ctx`");
  if (num_shards < 1 || (num_shards & (num_shards - 1)) || shard < 0 || shard >= num_shards)
    return InvalidArgumentError("num_shards must be a power of two and 0 <= shard < num_shards");
  int k = 0;
  while ((int64_t{1} << k) < num_shards) ++k;
  const int stop_level = hierarchy_to_tree()[hierarchy_level];
  if (k > stop_level) return InvalidArgumentError("more shards than subtrees at this level");
  const int log_domain_size = parameters()[hierarchy_level].log_domain_size();
  if (log_domain_size - k > 62)
    return InvalidArgumentError(
        "Output size would be larger than 2**62. Please evaluate fewer hierarchy levels at once.");
  DPF_ASSIGN_OR_RETURN(std::vector<uint128> vcw, ValueCorrectionLeaves(ctx.key(), hierarchy_level));
  const dpf_internal::FlatValueType& f = flat_[hierarchy_level];
  const int cepb = corrected_elements_per_block(hierarchy_level);
  const int64_t total = (int64_t{1} << (stop_level - k)) * cepb;
  if (!device_out || capacity_bytes < total * f.packed_size)
    return InvalidArgumentError("device output buffer too small");
  auto* s = scratch_.get();
  std::lock_guard<std::recursive_mutex> scratch_lock(s->mu);  // one call at a time per object
  // Everything the launches read -- root, party, shard path, value correction
  // and both correction-word ranges -- goes up as ONE page-locked image and
  // one async H2D (seven synchronous uploads had cost ~30 us per call, as
  // much as config 1's whole expansion kernel).
  const dpf_block root = ToBlock(FromProtoBlock(ctx.key().seed()));
  const uint8_t party = static_cast<uint8_t>(ctx.key().party() & 1);
  const dpf_block path = ToBlock(static_cast<uint128>(shard));
  std::vector<dpf_block> vcw_blocks(vcw.size());
  for (size_t i = 0; i < vcw.size(); ++i) vcw_blocks[i] = ToBlock(vcw[i]);
  PackedUploads& up = s->shard_alt ? s->packed_alt : s->packed;
  s->shard_alt = !s->shard_alt;
  DPF_RETURN_IF_ERROR(up.Reset());
  const size_t o_seed = up.Add(&root, 1), o_ctrl = up.Add(&party, 1), o_path = up.Add(&path, 1);
  const size_t o_vcw = up.Add(vcw_blocks.data(), vcw_blocks.size());
  const PackedCws o_top = AddCorrectionWords(ctx.key(), 0, k, up);
  const PackedCws o_cw = AddCorrectionWords(ctx.key(), k, stop_level, up);
  DPF_RETURN_IF_ERROR(up.Commit(stream));
  dpf_block* seed = up.Ptr<dpf_block>(o_seed);
  uint8_t* ctrl = up.Ptr<uint8_t>(o_ctrl);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  if (k > 0) {
    // Walk the root to the shard's subtree root along the top k tree bits (in place).
    HIP_RETURN_IF_ERROR(dpf_hip_eval_paths(1, k, seed, ctrl, up.Ptr<dpf_block>(o_path),
                                           up.Ptr<dpf_block>(o_top.seed), up.Ptr<uint8_t>(o_top.left),
                                           up.Ptr<uint8_t>(o_top.right), &kl, &kr, seed, ctrl,
                                           stream));
  }
  const dpf_value_desc desc = MakeDesc(f, blocks_needed_[hierarchy_level]);
  HIP_RETURN_IF_ERROR(dpf_hip_expand(1, seed, ctrl, stop_level - k, up.Ptr<dpf_block>(o_cw.seed),
                                     up.Ptr<uint8_t>(o_cw.left), up.Ptr<uint8_t>(o_cw.right), &kl,
                                     &kr, &kv, &desc, cepb, up.Ptr<dpf_block>(o_vcw), party,
                                     device_out, stream));
  DPF_RETURN_IF_ERROR(up.MarkUsed(stream));
  ctx.set_previous_hierarchy_level(hierarchy_level);
  return total;
}

namespace {
// Host-phase timing of EvaluateAt, printed at exit when DPF_HOST_TIMING is
// set (the first 10 calls, allocations and page-locked buffers, not counted):
// checks = the fused domain check + path / block-index pass over the points,
// key = key validation, value correction, context lookups and correction
// words, upload = the one packed H2D, launch = the point kernel's launch,
// device = waiting for the upload and the kernel (timing runs only: the
// stream is synchronised there), copy = the D2H into the caller's vector
// (unpacked chunk by chunk).
struct AtTiming {
  double t[6] = {0, 0, 0, 0, 0, 0};
  long calls = 0;
  ~AtTiming() {
    const double n = static_cast<double>(calls - 10);
    if (calls > 10 && std::getenv("DPF_HOST_TIMING"))
      std::fprintf(stderr,
                   "[EvaluateAt host timing] calls=%ld per call: checks=%.2fus key=%.2fus "
                   "upload=%.2fus launch=%.2fus device=%.2fus copy=%.2fus\n",
                   calls, t[0] * 1e6 / n, t[1] * 1e6 / n, t[2] * 1e6 / n, t[3] * 1e6 / n,
                   t[4] * 1e6 / n, t[5] * 1e6 / n);
  }
};
AtTiming g_at_timing;
std::mutex g_at_timing_mu;
struct AtClock {
  std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
  AtClock() {
    if (!g_until_timing_on) return;
    std::lock_guard<std::mutex> lock(g_at_timing_mu);
    ++g_at_timing.calls;
  }
  void mark(int phase) {
    if (!g_until_timing_on) return;
    auto now = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> lock(g_at_timing_mu);
    if (g_at_timing.calls > 10)
      g_at_timing.t[phase] += std::chrono::duration<double>(now - last).count();
    last = now;
  }
};

// First index in [0, n) whose point exceeds max_point (n if none), found on
// host threads while `fill(lo, hi)` writes the kernel's per-point arrays.
template <typename Fill>
int64_t CheckAndFillPoints(Span<const uint128> points, uint128 max_point, Fill fill) {
  const int64_t n = static_cast<int64_t>(points.size());
  std::atomic<int64_t> bad{n};
  dpf_internal::ParallelFor(
      n,
      [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i)
          if (points[i] > max_point) {
            int64_t cur = bad.load();
            while (i < cur && !bad.compare_exchange_weak(cur, i)) {
            }
            return;
          }
        fill(lo, hi);
      },
      int64_t{1} << 16);
  return bad.load();
}
}  // namespace

Status DistributedPointFunction::EvaluateAtToHost(const DpfKey& key, int hierarchy_level,
                                                  Span<const uint128> evaluation_points,
                                                  EvaluationContext* ctx,
                                                  const ValueType* requested_type,
                                                  const HostSink& sink) const {
  // h:839-1010
  AtClock clk;
  if (ctx != nullptr && &key != &ctx->key())
    return InvalidArgumentError("`key` and `ctx->key()` must refer to the same object");
  if (hierarchy_level < 0) return InvalidArgumentError("`hierarchy_level` must be non-negative");
  if (hierarchy_level >= static_cast<int>(parameters().size()))
    return InvalidArgumentError(
        "`hierarchy_level` must be less than the number of parameters passed at construction");
  if (requested_type) {
    // EvaluateAt<T> converts with T; a mismatching T is reported like EvaluateUntil does.
    DPF_ASSIGN_OR_RETURN(bool eq, dpf_internal::ValueTypesAreEqual(
                                      *requested_type, parameters()[hierarchy_level].value_type()));
    if (!eq) return InvalidArgumentError("Value type T doesn't match parameters at `hierarchy_level`");
  }
  const int64_t n = static_cast<int64_t>(evaluation_points.size());
  const int log_domain_size = parameters()[hierarchy_level].log_domain_size();
  const uint128 max_point =
      log_domain_size < 128 ? (static_cast<uint128>(1) << log_domain_size) - 1 : Uint128Max();
  const dpf_internal::FlatValueType& f = flat_[hierarchy_level];
  const int E = f.elements_per_block;
  const int stop_level = hierarchy_to_tree()[hierarchy_level];
  const int bib = log_domain_size - stop_level;
  const int start_level = ctx ? stop_level : 0;
  const int L = stop_level - start_level;
  auto* s = scratch_.get();
  std::lock_guard<std::recursive_mutex> scratch_lock(s->mu);  // one call at a time per object
  PackedUploads& up = s->packed;
  DPF_RETURN_IF_ERROR(up.Reset());
  // The domain check (h:861-874), tree indices and block indices (h:907-925)
  // in ONE pass on host threads, written straight into the page-locked
  // upload image.
  const size_t nvcw = static_cast<size_t>(E) * f.leaves.size();
  up.Prepare(7 * 256 + static_cast<size_t>(n) * (sizeof(dpf_block) + sizeof(int32_t)) +
             static_cast<size_t>(L + 1) * (sizeof(dpf_block) + 2) + nvcw * sizeof(dpf_block) + 32);
  size_t o_paths, o_bi;
  dpf_block* paths = up.Reserve<dpf_block>(n, &o_paths);
  int32_t* block_index = up.Reserve<int32_t>(n, &o_bi);
  const uint128 bmask = (static_cast<uint128>(1) << bib) - 1;
  const int64_t bad = CheckAndFillPoints(evaluation_points, max_point, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      const uint128 x = evaluation_points[i];
      paths[i] = ToBlock(E > 1 ? x >> bib : x);
      block_index[i] = E > 1 ? static_cast<int32_t>(x & bmask) : 0;
    }
  });
  if (bad < n)
    return InvalidArgumentError("`evaluation_points[" + std::to_string(bad) +
                                "]` larger than the domain size at hierarchy level " +
                                std::to_string(hierarchy_level));
  clk.mark(0);
  DPF_RETURN_IF_ERROR(validator_->ValidateDpfKey(key));
  if (n == 0) {
    (void)sink.reserve(0);
    return OkStatus();
  }
  DPF_ASSIGN_OR_RETURN(std::vector<uint128> vcw, ValueCorrectionLeaves(key, hierarchy_level));
  DeviceStart start;
  if (ctx) {
    // The tree indices, as uint128 memory images (paths is 256-byte aligned).
    const Span<const uint128> tree_indices(reinterpret_cast<const uint128*>(paths),
                                           static_cast<size_t>(n));
    DPF_RETURN_IF_ERROR(ComputePartialEvaluations(tree_indices, hierarchy_level,
                                                  /*update_ctx=*/true, *ctx, &start, nullptr,
                                                  nullptr));
  }
  std::vector<dpf_block> vcw_blocks(vcw.size());
  for (size_t i = 0; i < vcw.size(); ++i) vcw_blocks[i] = ToBlock(vcw[i]);
  const dpf_block root = ToBlock(FromProtoBlock(key.seed()));
  const uint8_t party = static_cast<uint8_t>(key.party() & 1);
  const PackedCws o_cw = AddCorrectionWords(key, start_level, stop_level, up);
  const size_t o_vcw = up.Add(vcw_blocks.data(), vcw_blocks.size());
  const size_t o_root = up.Add(&root, 1);
  const size_t o_party = up.Add(&party, 1);
  clk.mark(1);
  DPF_RETURN_IF_ERROR(up.Commit(nullptr));
  const size_t bytes = static_cast<size_t>(n) * f.packed_size;
  void* small = s->small_out.Get(bytes);   // small results: written to page-locked memory
  if (!small) DPF_RETURN_IF_ERROR(s->out.Reserve(bytes));
  void* const out = small ? small : s->out.get();
  clk.mark(2);
  const dpf_value_desc desc = MakeDesc(f, blocks_needed_[hierarchy_level]);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  HIP_RETURN_IF_ERROR(dpf_hip_eval_points(
      n, n, L, up.Ptr<dpf_block>(o_root), up.Ptr<uint8_t>(o_party),
      ctx ? start.seeds : nullptr, ctx ? start.ctrl : nullptr, up.Ptr<dpf_block>(o_paths),
      up.Ptr<int32_t>(o_bi), up.Ptr<dpf_block>(o_cw.seed), up.Ptr<uint8_t>(o_cw.left),
      up.Ptr<uint8_t>(o_cw.right), &kl, &kr, &kv, &desc, up.Ptr<dpf_block>(o_vcw), out, nullptr));
  DPF_RETURN_IF_ERROR(up.MarkUsed(nullptr));
  if (ctx) DPF_RETURN_IF_ERROR(s->packed_pe.MarkUsed(nullptr));   // start seeds read from it
  clk.mark(3);
  if (g_until_timing_on) {
    HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(nullptr));
    clk.mark(4);
  }
  // Packed elements straight into the caller's result (h:983-1003 outputs):
  // integers copied, tuples / IntModN / XorWrapper unpacked chunk by chunk out
  // of the page-locked staging buffers.
  if (small) {
    DPF_RETURN_IF_ERROR(dpf_internal::ConsumePinnedOut(sink, small, bytes, nullptr));
  } else {
    HIP_RETURN_IF_ERROR(dpf_internal::CopyToHostSink(sink, sink.reserve(bytes), s->out.get(), bytes,
                                                     nullptr));
  }
  clk.mark(5);
  if (ctx) ctx->set_previous_hierarchy_level(hierarchy_level);
  return OkStatus();
}

StatusOr<std::vector<uint8_t>> DistributedPointFunction::EvaluateAtPacked(
    const DpfKey& key, int hierarchy_level, Span<const uint128> evaluation_points,
    EvaluationContext* ctx, const ValueType* requested_type) const {
  std::vector<uint8_t> out;
  DPF_RETURN_IF_ERROR(EvaluateAtToHost(key, hierarchy_level, evaluation_points, ctx,
                                       requested_type, dpf_internal::VectorSink(&out)));
  return out;
}

StatusOr<std::vector<uint8_t>> DistributedPointFunction::EvaluateAtBatchPacked(
    Span<const DpfKey* const> keys, int hierarchy_level, Span<const uint128> points,
    int64_t points_per_key) const {
  if (hierarchy_level < 0 || hierarchy_level >= static_cast<int>(parameters().size()))
    return InvalidArgumentError("`hierarchy_level` out of range");
  const int64_t num_keys = static_cast<int64_t>(keys.size());
  if (points_per_key < 1 || static_cast<int64_t>(points.size()) != num_keys * points_per_key)
    return InvalidArgumentError("points.size() must equal keys.size() * points_per_key");
  const int log_domain_size = parameters()[hierarchy_level].log_domain_size();
  const uint128 max_point =
      log_domain_size < 128 ? (static_cast<uint128>(1) << log_domain_size) - 1 : Uint128Max();
  const int64_t n = static_cast<int64_t>(points.size());
  const dpf_internal::FlatValueType& f = flat_[hierarchy_level];
  const int E = f.elements_per_block, nl = static_cast<int>(f.leaves.size());
  const int L = hierarchy_to_tree()[hierarchy_level];
  const int bib = log_domain_size - L;
  auto* s = scratch_.get();
  std::lock_guard<std::recursive_mutex> scratch_lock(s->mu);  // one call at a time per object
  PackedUploads& up = s->packed;
  DPF_RETURN_IF_ERROR(up.Reset());
  const int64_t rows = std::max<int64_t>(num_keys * L, 1);
  up.Prepare(9 * 256 + static_cast<size_t>(n) * (sizeof(dpf_block) + sizeof(int32_t)) +
             static_cast<size_t>(num_keys) * (sizeof(dpf_block) + 1 + E * nl * sizeof(dpf_block)) +
             static_cast<size_t>(rows) * (sizeof(dpf_block) + 2) + 64);
  // The points: domain check, tree indices and block indices in one threaded
  // pass into the upload image (EvaluateAt's order: points before keys).
  size_t o_paths, o_bi;
  dpf_block* paths = up.Reserve<dpf_block>(n, &o_paths);
  int32_t* block_index = up.Reserve<int32_t>(n, &o_bi);
  const uint128 bmask = (static_cast<uint128>(1) << bib) - 1;
  const int64_t bad = CheckAndFillPoints(points, max_point, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      paths[i] = ToBlock(E > 1 ? points[i] >> bib : points[i]);
      block_index[i] = E > 1 ? static_cast<int32_t>(points[i] & bmask) : 0;
    }
  });
  if (bad < n)
    return InvalidArgumentError("`evaluation_points[" + std::to_string(bad) +
                                "]` larger than the domain size at hierarchy level " +
                                std::to_string(hierarchy_level));
  if (n == 0) return std::vector<uint8_t>{};
  // The keys: validated and flattened (SoA, [key][level]) on host threads;
  // the first failing key's error is returned.
  size_t o_seed, o_party, o_cws, o_cl, o_cr, o_vcw;
  dpf_block* seeds = up.Reserve<dpf_block>(num_keys, &o_seed);
  uint8_t* party = up.Reserve<uint8_t>(num_keys, &o_party);
  dpf_block* cw_seed = up.Reserve<dpf_block>(rows, &o_cws);
  uint8_t* cl = up.Reserve<uint8_t>(rows, &o_cl);
  uint8_t* cr = up.Reserve<uint8_t>(rows, &o_cr);
  dpf_block* vcw = up.Reserve<dpf_block>(std::max<int64_t>(num_keys * E * nl, 1), &o_vcw);
  std::atomic<int64_t> first_bad{num_keys};
  dpf_internal::ParallelFor(
      num_keys,
      [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; ++k) {
          const DpfKey& key = *keys[k];
          StatusOr<std::vector<uint128>> v = validator_->ValidateDpfKey(key).ok()
                                                 ? ValueCorrectionLeaves(key, hierarchy_level)
                                                 : StatusOr<std::vector<uint128>>(
                                                       InvalidArgumentError("invalid key"));
          if (!v.ok()) {
            int64_t cur = first_bad.load();
            while (k < cur && !first_bad.compare_exchange_weak(cur, k)) {
            }
            return;
          }
          seeds[k] = ToBlock(FromProtoBlock(key.seed()));
          party[k] = static_cast<uint8_t>(key.party() & 1);
          for (int j = 0; j < L; ++j) {
            const CorrectionWord& cw = key.correction_words(j);
            cw_seed[k * L + j] = ToBlock(FromProtoBlock(cw.seed()));
            cl[k * L + j] = cw.control_left();
            cr[k * L + j] = cw.control_right();
          }
          for (int i = 0; i < E * nl; ++i) vcw[k * E * nl + i] = ToBlock((*v)[i]);
        }
      },
      int64_t{256});
  if (first_bad.load() < num_keys) {
    // The failing key's own error, as the one-by-one loop reported it.
    const DpfKey& key = *keys[first_bad.load()];
    DPF_RETURN_IF_ERROR(validator_->ValidateDpfKey(key));
    return ValueCorrectionLeaves(key, hierarchy_level).status();
  }
  DPF_RETURN_IF_ERROR(up.Commit(nullptr));
  const size_t bytes = static_cast<size_t>(n) * f.packed_size;
  DPF_RETURN_IF_ERROR(s->out.Reserve(bytes));
  const dpf_value_desc desc = MakeDesc(f, blocks_needed_[hierarchy_level]);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  HIP_RETURN_IF_ERROR(dpf_hip_eval_points(
      n, points_per_key, L, up.Ptr<dpf_block>(o_seed), up.Ptr<uint8_t>(o_party), nullptr, nullptr,
      up.Ptr<dpf_block>(o_paths), up.Ptr<int32_t>(o_bi), up.Ptr<dpf_block>(o_cws),
      up.Ptr<uint8_t>(o_cl), up.Ptr<uint8_t>(o_cr), &kl, &kr, &kv, &desc,
      up.Ptr<dpf_block>(o_vcw), s->out.get(), nullptr));
  DPF_RETURN_IF_ERROR(up.MarkUsed(nullptr));
  std::vector<uint8_t> out;
  HIP_RETURN_IF_ERROR(CopyToHostVector(&out, s->out.get(), bytes, nullptr));
  return out;
}

}  // namespace distributed_point_functions
