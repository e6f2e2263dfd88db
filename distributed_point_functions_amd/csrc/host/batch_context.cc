// batch_context.cc -- incremental evaluation of a whole key batch with a
// device-resident EvaluationContext (config 5b, the
// heavy-hitters hierarchy over 2^20 client keys).
//
// EvaluateUntilBatch*(h, prefixes, ctx) computes, for every key k of the batch,
// exactly what EvaluateUntil<T>(h, prefixes, ctx_k)
// (distributed_point_function.h:641-837) returns, and leaves the batch
// context in the state the per-key contexts would be in:
//   * validation and error messages of EvaluateUntil (h:655-700);
//   * unique tree indices of the prefixes in first-seen order (h:718-742);
//   * ComputePartialEvaluations (cc:351-453): each tree index is found under
//     its parent among the stored partial evaluations (or walked from the
//     root), walked down on the GPU, and stored as the new partial evaluation
//     unless this is the last hierarchy level;
//   * ExpandSeeds + HashExpandedSeeds + correction (cc:271-349, 500-524;
//     h:745-808) and the per-prefix gather (h:817-836).
// The host does O(#prefixes) bookkeeping per call; every per-key step runs in
// one dpf_hip_eval_prefix_batch launch (csrc/kernels/dpf_batch.hip).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <unordered_map>

#include "dpf/distributed_point_function.h"
#include "dpf/key_batch.h"
#include "dpf_hip.h"
#include "host_util.h"

namespace distributed_point_functions {

using dpf_internal::AesKey;
using dpf_internal::FromBlock;
using dpf_internal::FromHip;
using dpf_internal::kPrgKeyLeft;
using dpf_internal::kPrgKeyRight;
using dpf_internal::kPrgKeyValue;
using dpf_internal::MakeDesc;
using dpf_internal::SetProtoBlock;
using dpf_internal::ToBlock;
using dpf_internal::U128Hash;

namespace {
// Host-phase timing of the batched path, printed at exit when
// DPF_BATCH_HOST_TIMING is set (diagnostics for config 5a's host-bound levels).
// Contexts on several threads add into it, so every update takes `mu`.
struct HostTiming {
  std::mutex mu;
  double t[6] = {0, 0, 0, 0, 0, 0};
  long calls = 0;
  void add(int phase, double s) {
    std::lock_guard<std::mutex> g(mu);
    t[phase] += s;
  }
  void call() {
    std::lock_guard<std::mutex> g(mu);
    ++calls;
  }
  ~HostTiming() {
    if (calls && std::getenv("DPF_BATCH_HOST_TIMING"))
      std::fprintf(stderr,
                   "[batch host timing] calls=%ld dedup=%.3fs lookup=%.3fs tables=%.3fs "
                   "upload=%.3fs device=%.3fs update=%.3fs\n",
                   calls, t[0], t[1], t[2], t[3], t[4], t[5]);
  }
};
HostTiming g_timing;
const bool g_timing_on = std::getenv("DPF_BATCH_HOST_TIMING") != nullptr;
// DPF_BATCH_NO_CACHE=1 turns the expansion cache off (every call walks down
// from the partial evaluations, as the reference does): an A/B and test hook.
bool CacheOn() {
  const char* v = std::getenv("DPF_BATCH_NO_CACHE");
  return !(v && v[0] == '1');
}
// How a call that reads the expansion cache writes the next one.  Default:
// into a spare buffer if one fits, else in place through a slot table, else
// (no slot table possible) in place after gathering the start seeds.
// DPF_BATCH_CACHE_MODE=spare|permute|gather forces one (a spare still only if
// it fits; permute falls back to gather when no slot table exists), and
// DPF_BATCH_CACHE_IN_PLACE=1 means gather: test and A/B hooks, read per call.
enum class CacheMode { kAuto, kSpare, kPermute, kGather };
CacheMode ForcedCacheMode() {
  const char* v = std::getenv("DPF_BATCH_CACHE_IN_PLACE");
  if (v && v[0] == '1') return CacheMode::kGather;
  const char* m = std::getenv("DPF_BATCH_CACHE_MODE");
  if (!m) return CacheMode::kAuto;
  const std::string s(m);
  if (s == "spare") return CacheMode::kSpare;
  if (s == "permute") return CacheMode::kPermute;
  if (s == "gather") return CacheMode::kGather;
  return CacheMode::kAuto;
}

// The slot table of an in-place rewrite (dpf_hip_eval_prefix_batch_cached_slots):
// start node u = (tree index u >> s, sub-node) reads physical slot
// start_slot[u >> s]; its 2^E leaves go to slot[(u << E) + l].  A slot read by
// exactly one start node (s == 0) takes that node's leaf 0; every other leaf
// takes the next slot no start node reads.  False if those run out.
bool BuildSlotTable(const std::vector<int64_t>& start_slot, int64_t T, int s, int E,
                    int64_t phys_stride, std::vector<int32_t>* slot) {
  static thread_local std::vector<uint8_t> tl_read;
  std::vector<uint8_t>& read = tl_read;
  read.assign(static_cast<size_t>(phys_stride), 0);
  for (int64_t i = 0; i < T; ++i) read[start_slot[i]] = 1;
  const int64_t leaves = (T << s) << E;
  slot->resize(static_cast<size_t>(leaves));
  int64_t g = 0;  // next unread slot candidate
  auto next_free = [&]() -> int64_t {
    while (g < phys_stride && read[g]) ++g;
    return g < phys_stride ? g++ : -1;
  };
  for (int64_t u = 0; u < (T << s); ++u) {
    for (int64_t l = 0; l < (int64_t{1} << E); ++l) {
      int64_t v;
      if (l == 0 && s == 0) {
        v = start_slot[u];
      } else if ((v = next_free()) < 0) {
        return false;
      }
      (*slot)[(u << E) + l] = static_cast<int32_t>(v);
    }
  }
  return true;
}
struct PhaseClock {
  std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
  void mark(int phase) {
    if (!g_timing_on) return;
    auto now = std::chrono::steady_clock::now();
    g_timing.add(phase, std::chrono::duration<double>(now - last).count());
    last = now;
  }
};
}  // namespace

// DPF_BATCH_ALLOC_LIMIT=<bytes>: a test hook that makes a batch context behave
// as if the device had only that much memory for it -- an allocation that
// would take the context's total above the limit fails like hipMalloc's
// out-of-memory, and MemInfo reports the limit -- so the expansion cache's
// fallbacks (no spare, eviction and retry, RESOURCE_EXHAUSTED) run
// deterministically.  Read per call.
size_t AllocLimit() {
  const char* v = std::getenv("DPF_BATCH_ALLOC_LIMIT");
  return v && *v ? static_cast<size_t>(std::strtoull(v, nullptr, 10)) : 0;
}

bool DeviceBatchContext::TryAlloc(void** p, size_t* cap, size_t bytes) {
  *p = nullptr;
  *cap = 0;
  const size_t limit = AllocLimit();
  if (limit && device_bytes_ + bytes > limit) return false;
  if (dpf_hip_alloc(p, bytes) != 0) {
    *p = nullptr;
    return false;
  }
  *cap = bytes;
  device_bytes_ += bytes;
  return true;
}

void DeviceBatchContext::Release(void** p, size_t* cap) {
  if (*p) dpf_hip_free(*p);
  device_bytes_ -= std::min(device_bytes_, *cap);
  *p = nullptr;
  *cap = 0;
}

void DeviceBatchContext::MemInfo(size_t* free_bytes, size_t* total_bytes) const {
  *free_bytes = *total_bytes = 0;
  if (const size_t limit = AllocLimit()) {
    *total_bytes = limit;
    *free_bytes = limit - std::min(limit, device_bytes_);
    return;
  }
  (void)dpf_hip_mem_info(free_bytes, total_bytes);
}

Status DeviceBatchContext::Ensure(void** p, size_t* cap, size_t bytes) {
  if (fail_next_ > 0 && fail_skip_ > 0) {
    --fail_skip_;
  } else if (fail_next_ > 0) {
    --fail_next_;
    Release(p, cap);
    ++events_.alloc_failures;
    return ResourceExhaustedError("Memory allocation error");
  }
  if (*p && *cap >= bytes) return OkStatus();
  Release(p, cap);
  if (!TryAlloc(p, cap, std::max<size_t>(bytes, 256))) {
    ++events_.alloc_failures;
    return ResourceExhaustedError("Memory allocation error");  // cc:289-291
  }
  return OkStatus();
}

void DeviceBatchContext::ReleaseExpansionCache() {
  // hipFree waits for the device work that may still read the buffers.
  Release(&leaf_seeds_, &leaf_seeds_cap_);
  Release(&leaf_spare_, &leaf_spare_cap_);
  Release(&slots_, &slots_cap_);
  Release(&leaf_slot_, &leaf_slot_cap_);
  leaf_phys_.clear();
  leaf_level_ = -1;
}

void DeviceBatchContext::Reset(bool release_expansion_cache) {
  previous_hierarchy_level_ = -1;
  partial_evaluations_level_ = -1;
  partial_prefixes_.clear();
  partial_sorted_ = false;
  leaf_level_ = -1;
  if (release_expansion_cache) {
    (void)dpf_hip_stream_sync(nullptr);  // work still reading the cache
    ReleaseExpansionCache();
  }
}

DeviceBatchContext::~DeviceBatchContext() {
  if (tables_pending_) (void)dpf_hip_event_sync(tables_event_);
  if (tables_event_) dpf_hip_event_destroy(tables_event_);
  if (pinned_tables_) dpf_hip_host_free(pinned_tables_);
  for (void* p : {seeds_, ctrl_, next_seeds_, next_ctrl_, parent_, path_, save_, offsets_,
                  workspace_, stage_, stage2_, leaf_seeds_, leaf_spare_, slots_, leaf_slot_})
    if (p) dpf_hip_free(p);
}

Status DeviceBatchContext::StageTables(size_t bytes) {
  if (tables_pending_) {
    HIP_RETURN_IF_ERROR(dpf_hip_event_sync(tables_event_));
    tables_pending_ = false;
  }
  if (pinned_tables_cap_ >= bytes && pinned_tables_) return OkStatus();
  if (pinned_tables_) dpf_hip_host_free(pinned_tables_);
  pinned_tables_ = nullptr;
  pinned_tables_cap_ = 0;
  const size_t want = std::max<size_t>(bytes + bytes / 2, size_t{1} << 16);
  if (dpf_hip_host_alloc(&pinned_tables_, want) != 0) {
    pinned_tables_ = nullptr;
    return ResourceExhaustedError("Memory allocation error");
  }
  pinned_tables_cap_ = want;
  return OkStatus();
}

Status DeviceBatchContext::TablesSent(void* stream) {
  if (!tables_event_) HIP_RETURN_IF_ERROR(dpf_hip_event_create(&tables_event_));
  HIP_RETURN_IF_ERROR(dpf_hip_event_record(tables_event_, stream));
  tables_pending_ = true;
  return OkStatus();
}

StatusOr<std::unique_ptr<DeviceBatchContext>> DistributedPointFunction::CreateBatchEvaluationContext(
    const DeviceKeyBatch& keys) const {
  if (keys.num_levels() != tree_levels_needed() - 1 ||
      keys.num_hierarchy_levels() != static_cast<int>(parameters().size()))
    return InvalidArgumentError("key batch does not match this DistributedPointFunction");
  std::unique_ptr<DeviceBatchContext> ctx(new DeviceBatchContext(&keys));
  // DPF_BATCH_KEY_MAJOR=1 (read at creation: one layout per context) keeps
  // the r15 key-major tables and lanes = start nodes (A/B and test hook).
  const char* km = std::getenv("DPF_BATCH_KEY_MAJOR");
  ctx->index_major_ = !(km && km[0] == '1');
  return ctx;
}

StatusOr<int64_t> DistributedPointFunction::EvaluateUntilBatchToDevice(
    int hierarchy_level, Span<const uint128> prefixes, DeviceBatchContext& ctx, void* device_out,
    int64_t capacity_bytes, void* stream) const {
  return EvaluateUntilBatchCore(hierarchy_level, prefixes, ctx, false, device_out, capacity_bytes,
                                stream);
}

StatusOr<int64_t> DistributedPointFunction::EvaluateUntilBatchSumToDevice(
    int hierarchy_level, Span<const uint128> prefixes, DeviceBatchContext& ctx, void* device_out,
    int64_t capacity_bytes, void* stream) const {
  return EvaluateUntilBatchCore(hierarchy_level, prefixes, ctx, true, device_out, capacity_bytes,
                                stream);
}

StatusOr<int64_t> DistributedPointFunction::EvaluateUntilBatchCore(
    int hierarchy_level, Span<const uint128> prefixes, DeviceBatchContext& ctx, bool sum,
    void* device_out, int64_t capacity_bytes, void* stream) const {
  const DeviceKeyBatch& keys = ctx.keys();
  const int H = static_cast<int>(parameters().size());
  if (keys.num_levels() != tree_levels_needed() - 1 || keys.num_hierarchy_levels() != H)
    return InvalidArgumentError("key batch does not match this DistributedPointFunction");
  // h:655-700, in the reference's order.
  if (hierarchy_level < 0 || hierarchy_level >= H)
    return InvalidArgumentError(
        "`hierarchy_level` must be non-negative and less than parameters_.size()");
  if (hierarchy_level <= ctx.previous_hierarchy_level_)
    return InvalidArgumentError(
        "`hierarchy_level` must be greater than `ctx.previous_hierarchy_level`");
  if ((ctx.previous_hierarchy_level_ < 0) != prefixes.empty())
    return InvalidArgumentError(
        "`prefixes` must be empty if and only if this is the first call with `ctx`.");
  const int prev = ctx.previous_hierarchy_level_;
  int prev_log = 0;
  if (!prefixes.empty()) {
    prev_log = parameters()[prev].log_domain_size();
    if (prev_log < 128) {
      const uint128 limit = static_cast<uint128>(1) << prev_log;
      const int64_t np = static_cast<int64_t>(prefixes.size());
      std::atomic<int64_t> bad{np};
      dpf_internal::ParallelFor(np, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i)
          if (prefixes[i] >= limit) {
            int64_t cur = bad.load();
            while (i < cur && !bad.compare_exchange_weak(cur, i)) {
            }
            return;
          }
      });
      if (bad.load() < np)
        return InvalidArgumentError("Index " + Uint128ToString(prefixes[bad.load()]) +
                                    " out of range for hierarchy level " + std::to_string(prev));
    }
  }
  const int log = parameters()[hierarchy_level].log_domain_size();
  if (log - prev_log > 62)
    return InvalidArgumentError(
        "Output size would be larger than 2**62. Please evaluate fewer hierarchy levels at once.");

  PhaseClock clk;
  if (g_timing_on) g_timing.call();
  // Unique tree indices in first-seen order and each prefix's (tree index,
  // block index) (h:718-742).
  const int64_t P = static_cast<int64_t>(prefixes.size());
  // Host buffers are recycled across calls: first touches of fresh pages cost
  // more than the bookkeeping itself at 1 M prefixes per level (config 5a).
  // Not cleared first: DedupTreeIndices overwrites every element, so vectors
  // kept from an earlier call of about this size value-initialise nothing
  // (clearing them had cost a 1 M-prefix level ~3.8 ms of single-threaded
  // zeroing, r16 DPF_BATCH_HOST_TIMING).
  // Start nodes are indexed by int32 on the device (checked below), so 32-bit
  // positions suffice: 8-byte (position, block index) entries.
  if (P > INT32_MAX)
    return ResourceExhaustedError(
        "Too many start nodes for one batched evaluation; evaluate fewer levels at once.");
  std::vector<uint128> tree_indices = std::move(ctx.spare_prefixes_);
  static thread_local std::vector<std::pair<int32_t, int>> tl_prefix_map;
  std::vector<std::pair<int32_t, int>>& prefix_map = tl_prefix_map;
  bool indices_ascending = false;   // tree_indices strictly ascending
  if (P > 0) {
    dpf_internal::DedupTreeIndices(prefixes, prev_log - hierarchy_to_tree()[prev], &tree_indices,
                                   &prefix_map, &indices_ascending);
  } else {
    tree_indices.clear();
    prefix_map.clear();
  }

  clk.mark(0);
  // Where each tree index starts: a stored partial evaluation or the root
  // (ExpandAndUpdateContext cc:455-498, ComputePartialEvaluations cc:351-453).
  const int Dh = hierarchy_to_tree()[hierarchy_level];
  int Dprev = 0, start_level = 0;
  bool from_root = true;
  static thread_local std::vector<int32_t> tl_parent_of;   // recycled: no per-call zeroing
  std::vector<int32_t>& parent_of = tl_parent_of;
  // Physical cache slot of each tree index's node (cached calls; see `cached`
  // below), filled in the parent lookup's own pass when there is one.
  static thread_local std::vector<int64_t> tl_start_slot;
  std::vector<int64_t>& start_slot = tl_start_slot;
  const bool g_cache_on = CacheOn();
  bool slots_done = false;
  if (P == 0) {
    tree_indices.assign(1, 0);  // the root, expanded to depth Dh
  } else {
    Dprev = hierarchy_to_tree()[prev];
    const auto& q = ctx.partial_prefixes_;
    if (ctx.partial_evaluations_level_ >= 0 && !q.empty() &&
        hierarchy_to_tree()[ctx.partial_evaluations_level_] <= Dprev) {
      start_level = hierarchy_to_tree()[ctx.partial_evaluations_level_];
      from_root = false;
      const int shift = Dprev - start_level;
      // Sortedness of the stored prefixes: known when they came from an
      // ascending dedup (the hierarchical case), else checked in chunks on
      // host threads.
      bool sorted = ctx.partial_sorted_;
      if (!sorted) {
        const int64_t nq = static_cast<int64_t>(q.size());
        const int qchunks = dpf_internal::NumChunks(nq);
        std::vector<char> q_ok(qchunks, 1);
        dpf_internal::ParallelChunks(nq, qchunks, [&](int c, int64_t lo, int64_t hi) {
          for (int64_t j = std::max<int64_t>(lo, 1); j < hi; ++j)
            if (q[j] < q[j - 1]) {
              q_ok[c] = 0;
              return;
            }
        });
        sorted = std::all_of(q_ok.begin(), q_ok.end(), [](char x) { return x != 0; });
      }
      std::unordered_map<uint128, int32_t, U128Hash> pos;
      if (!sorted) {
        pos.reserve(q.size() * 2);
        for (size_t j = 0; j < q.size(); ++j) pos.emplace(q[j], static_cast<int32_t>(j));
      }
      parent_of.resize(tree_indices.size());
      const int64_t nt = static_cast<int64_t>(tree_indices.size());
      // The same condition as `cached` below: the start slots come out of
      // this pass (one read of tree_indices instead of two).
      const int w1 = Dprev - start_level;
      slots_done = g_cache_on && ctx.leaf_seeds_ && ctx.leaf_level_ == prev &&
                   ctx.leaf_de_ == w1 && ctx.leaf_stride_ <= INT32_MAX;
      if (slots_done) start_slot.resize(nt);
      const uint128 slot_mask = slots_done ? (uint128{1} << w1) - 1 : 0;  // w1 <= 62 then
      const std::vector<int32_t>& phys = ctx.leaf_phys_;
      std::atomic<int64_t> first_missing{nt};
      dpf_internal::ParallelFor(nt, [&](int64_t lo, int64_t hi) {
        size_t cursor = 0;  // merge pointer while the lookups ascend too
        bool fresh = true;
        for (int64_t i = lo; i < hi; ++i) {
          const uint128 want = shift < 128 ? tree_indices[i] >> shift : 0;
          int64_t j = -1;
          if (sorted) {
            if (fresh || cursor >= q.size() || q[cursor] > want) {
              cursor = std::lower_bound(q.begin(), q.end(), want) - q.begin();
              fresh = false;
            } else if (want - q[cursor] < 64) {
              while (cursor < q.size() && q[cursor] < want) ++cursor;
            } else {
              cursor = std::lower_bound(q.begin() + cursor, q.end(), want) - q.begin();
            }
            if (cursor < q.size() && q[cursor] == want) j = static_cast<int64_t>(cursor);
          } else {
            auto it = pos.find(want);
            if (it != pos.end()) j = it->second;
          }
          if (j < 0) {
            int64_t cur = first_missing.load();
            while (i < cur && !first_missing.compare_exchange_weak(cur, i)) {
            }
            return;
          }
          parent_of[i] = static_cast<int32_t>(j);
          if (slots_done) {
            const int64_t logical = (j << w1) | static_cast<int64_t>(tree_indices[i] & slot_mask);
            start_slot[i] = phys.empty() ? logical : phys[logical];
          }
        }
      });
      if (first_missing.load() < nt)
        return InvalidArgumentError(
            "Prefix not present in ctx.partial_evaluations at hierarchy level " +
            std::to_string(prev));
    }
  }
  const int64_t T = static_cast<int64_t>(tree_indices.size());
  const int W1 = Dprev - start_level;
  const int dE = Dh - Dprev;

  const auto& f = flat_[hierarchy_level];
  const dpf_value_desc desc = MakeDesc(f, blocks_needed_[hierarchy_level]);
  int max_e = dpf_hip_prefix_batch_max_expand(&desc, sum ? 1 : 0);
  const bool native_sum = sum && max_e >= 0;
  if (max_e < 0) max_e = dpf_hip_prefix_batch_max_expand(&desc, 0);
  if (max_e < 0) return UnimplementedError("value type not supported by the batched GPU path");
  const int E = std::min(dE, max_e);
  const int s = dE - E;  // levels walked per start node below the tree index
  if (s > 30 || (T << s) > INT32_MAX)
    return ResourceExhaustedError(
        "Too many start nodes for one batched evaluation; evaluate fewer levels at once.");
  const int64_t U = T << s;
  const int64_t K = keys.num_keys();
  // The previous call's expansion cache holds this call's tree nodes (its
  // leaves are the children, W1 levels down, of the tree indices the
  // partial evaluations stand for): the kernel reads their seeds from it and
  // the W1-level path walk is skipped.  Outputs and the
  // partial evaluations are the same either way.
  const bool cached = g_cache_on && P > 0 && ctx.leaf_seeds_ && ctx.leaf_level_ == prev &&
                      ctx.leaf_de_ == W1 && ctx.leaf_stride_ <= INT32_MAX;
  const int Wk = cached ? 0 : W1;  // levels walked above each tree index
  const int cepb = corrected_elements_per_block(hierarchy_level);
  const int esz = f.packed_size;
  const int64_t block = (int64_t{1} << dE) * cepb;   // elements per tree index
  const int64_t n_blk = T * block;                  // elements per key before the gather
  const int64_t cnt = int64_t{1} << (log - prev_log);  // elements per prefix
  const int64_t n = P == 0 ? n_blk : P * cnt;
  bool identity = P == 0 || (T == P && cnt == block);
  for (int64_t i = 0; identity && P > 0 && i < P; ++i)
    identity = prefix_map[i].first == i && prefix_map[i].second == 0;
  const int64_t need = (sum ? n : K * n) * esz;
  if (!device_out || capacity_bytes < need) return InvalidArgumentError("device output buffer too small");
  const bool update_ctx = P > 0 && hierarchy_level < H - 1;

  // This call's leaves become the next call's expansion cache (not after the
  // last level).  Preferred: write them to the spare buffer while the kernel
  // reads the start seeds straight from the current cache, then swap.  With
  // no room for a spare, the start seeds are gathered first and the current
  // cache is rewritten in place; a failed allocation only turns the cache off.
  const int64_t leaf_stride = U << E;
  void* leaf_seeds = nullptr;
  int64_t cache_stride = leaf_stride;  // physical row stride of the cache written
  bool swap_cache = false;
  bool gather = false;
  bool permute = false;
  const uint128 leaf_mask = cached ? (uint128{1} << W1) - 1 : 0;  // W1 <= 62 when cached
  if (cached && !slots_done) {
    start_slot.resize(T);
    const std::vector<int32_t>& phys = ctx.leaf_phys_;
    dpf_internal::ParallelFor(T, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) {
        const int64_t logical = (static_cast<int64_t>(from_root ? 0 : parent_of[i]) << W1) |
                                static_cast<int64_t>(tree_indices[i] & leaf_mask);
        start_slot[i] = phys.empty() ? logical : phys[logical];
      }
    });
  }
  static thread_local std::vector<int32_t> tl_leaf_slot;
  std::vector<int32_t>& leaf_slot = tl_leaf_slot;
  // Headroom left on the device for everything else (the caller's buffers,
  // a second context): a quarter of it for the spare, an eighth for the cache.
  auto fits = [&](size_t bytes, size_t reserve_div) {
    size_t free_b = 0, total_b = 0;
    ctx.MemInfo(&free_b, &total_b);
    return free_b >= bytes + total_b / reserve_div;
  };
  if (g_cache_on && hierarchy_level < H - 1 && Dh > 0) {
    const size_t cache_need = static_cast<size_t>(K * leaf_stride) * sizeof(dpf_block);
    if (!cached) {
      // The current cache is not read by this call: rewrite (or regrow) it.
      ctx.leaf_level_ = -1;  // until this call has written it
      if (ctx.leaf_seeds_cap_ < cache_need) {
        HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(stream));
        ctx.Release(&ctx.leaf_seeds_, &ctx.leaf_seeds_cap_);
        if (!fits(cache_need, 8) || !ctx.TryAlloc(&ctx.leaf_seeds_, &ctx.leaf_seeds_cap_, cache_need))
          ++ctx.events_.cache_refused;
      }
      leaf_seeds = ctx.leaf_seeds_;
    } else {
      const CacheMode mode = ForcedCacheMode();
      const bool want_spare = mode == CacheMode::kAuto || mode == CacheMode::kSpare;
      if (want_spare && ctx.leaf_spare_cap_ < cache_need) {
        // The spare may still be read by work in flight on the stream.
        HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(stream));
        ctx.Release(&ctx.leaf_spare_, &ctx.leaf_spare_cap_);
        if (!fits(cache_need, 4) || !ctx.TryAlloc(&ctx.leaf_spare_, &ctx.leaf_spare_cap_, cache_need))
          ++ctx.events_.spare_refused;
      }
      if (want_spare && ctx.leaf_spare_ && ctx.leaf_spare_cap_ >= cache_need) {
        leaf_seeds = ctx.leaf_spare_;
        swap_cache = true;
      } else if (mode != CacheMode::kGather && leaf_stride <= ctx.leaf_stride_ &&
                 BuildSlotTable(start_slot, T, s, E, ctx.leaf_stride_, &leaf_slot)) {
        // In place through the slot table: no gather, no second buffer.
        permute = true;
        leaf_seeds = ctx.leaf_seeds_;
        cache_stride = ctx.leaf_stride_;
        ++ctx.events_.permuted;
      } else {
        gather = true;  // leaf_seeds is set once the gather is enqueued
        ++ctx.events_.in_place;
      }
    }
  }
  const bool direct = cached && !gather;  // start seeds read from the cache
  // The per-call buffers come first: when device memory runs out, the
  // expansion cache gives way (the spare, then -- unless this call reads it --
  // the cache itself) and the allocation is retried.
  bool cache_in_use = cached;  // read by this call's gather or kernel
  auto ensure = [&](void** p, size_t* cap, size_t bytes) -> Status {
    Status st = ctx.Ensure(p, cap, bytes);
    for (int step = 0; !st.ok() && step < 2; ++step) {
      void** victim = step == 0 ? &ctx.leaf_spare_ : &ctx.leaf_seeds_;
      size_t* victim_cap = step == 0 ? &ctx.leaf_spare_cap_ : &ctx.leaf_seeds_cap_;
      if (!*victim || (step == 1 && cache_in_use)) continue;
      HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(stream));
      if (leaf_seeds == *victim) {
        leaf_seeds = nullptr;  // this call writes no cache
        swap_cache = false;
      }
      ctx.Release(victim, victim_cap);
      ++(step == 0 ? ctx.events_.evicted_spare : ctx.events_.evicted_cache);
      if (step == 1) ctx.leaf_level_ = -1;
      st = ctx.Ensure(p, cap, bytes);
    }
    return st;
  };

  clk.mark(1);
  // Start-node tables (u = tree index i * 2^s + sub) and the output gather's
  // offsets, built in ONE page-locked image on host threads and sent with one
  // asynchronous H2D into one device buffer: parent[U] int32 | save[U] int32
  // (only with s > 0: with s == 0 start node u IS tree index u, save_index
  // NULL) | path[U] (only when the kernel walks, Wk + s > 0) | offsets[P]
  // int64 (non-identity gathers).  Three synchronous pageable copies of
  // 24 MiB had cost a 1 M-prefix level (config 5a) milliseconds.
  const bool need_path = Wk + s > 0;
  const bool need_save = s > 0;
  auto align = [](size_t b) { return (b + 255) & ~size_t{255}; };
  const size_t off_save = align(static_cast<size_t>(U) * sizeof(int32_t));
  const size_t off_path = off_save + (need_save ? align(static_cast<size_t>(U) * sizeof(int32_t)) : 0);
  const size_t off_offsets = off_path + (need_path ? align(static_cast<size_t>(U) * sizeof(dpf_block)) : 0);
  const size_t tables_bytes = off_offsets + (identity ? 0 : static_cast<size_t>(P) * sizeof(int64_t));
  DPF_RETURN_IF_ERROR(ctx.StageTables(tables_bytes));
  char* img = static_cast<char*>(ctx.pinned_tables_);
  int32_t* parent = reinterpret_cast<int32_t*>(img);
  int32_t* save = need_save ? reinterpret_cast<int32_t*>(img + off_save) : nullptr;
  dpf_block* path = need_path ? reinterpret_cast<dpf_block*>(img + off_path) : nullptr;
  const uint128 w1_mask = Wk >= 128 ? ~uint128{0} : ((uint128{1} << Wk) - 1);
  dpf_internal::ParallelFor(T, [&](int64_t lo, int64_t hi) {
    if (!path && s == 0) {
      // One start node per tree index and no walk (the cached steady state):
      // the parents alone, without reading the tree indices.
      for (int64_t i = lo; i < hi; ++i)
        parent[i] = direct ? static_cast<int32_t>(start_slot[i])
                    : gather ? static_cast<int32_t>(i)
                             : (from_root ? 0 : parent_of[i]);
      return;
    }
    for (int64_t i = lo; i < hi; ++i) {
      const uint128 low = tree_indices[i] & w1_mask;
      // Cached: the physical cache slot of tree index i.
      const int64_t slot = cached ? start_slot[i] : 0;
      const int32_t start = direct ? static_cast<int32_t>(slot)
                            : gather ? static_cast<int32_t>(i)
                                     : (from_root ? 0 : parent_of[i]);
      for (int64_t sub = 0; sub < (int64_t{1} << s); ++sub) {
        const int64_t u = (i << s) + sub;
        parent[u] = start;
        if (path) path[u] = ToBlock(s ? ((low << s) | static_cast<uint128>(sub)) : low);
        if (save) save[u] = sub == 0 ? static_cast<int32_t>(i) : -1;
      }
    }
  });
  if (!identity) {
    int64_t* offsets = reinterpret_cast<int64_t*>(img + off_offsets);
    dpf_internal::ParallelFor(P, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i)
        offsets[i] = prefix_map[i].first * block + prefix_map[i].second * cnt;
    });
  }
  clk.mark(2);
  DPF_RETURN_IF_ERROR(ensure(&ctx.parent_, &ctx.parent_cap_, tables_bytes));
  HIP_RETURN_IF_ERROR(dpf_hip_memcpy_h2d_async(ctx.parent_, img, tables_bytes, stream));
  DPF_RETURN_IF_ERROR(ctx.TablesSent(stream));
  char* dtab = static_cast<char*>(ctx.parent_);
  const int32_t* d_parent = reinterpret_cast<const int32_t*>(dtab);
  const int32_t* d_save = need_save ? reinterpret_cast<const int32_t*>(dtab + off_save) : nullptr;
  const dpf_block* d_path = need_path ? reinterpret_cast<const dpf_block*>(dtab + off_path) : nullptr;
  const int64_t* d_offsets = identity ? nullptr : reinterpret_cast<const int64_t*>(dtab + off_offsets);
  if (update_ctx || gather) {
    DPF_RETURN_IF_ERROR(ensure(&ctx.next_seeds_, &ctx.next_seeds_cap_,
                                                   K * T * sizeof(dpf_block)));
    DPF_RETURN_IF_ERROR(ensure(&ctx.next_ctrl_, &ctx.next_ctrl_cap_, K * T));
  }
  if (gather) {
    // The start seeds (and, with update_ctx, the new partial evaluations),
    // read before the kernel rewrites the cache.
    DPF_RETURN_IF_ERROR(ensure(&ctx.slots_, &ctx.slots_cap_, T * sizeof(int64_t)));
    HIP_RETURN_IF_ERROR(
        dpf_hip_memcpy_h2d(ctx.slots_, start_slot.data(), T * sizeof(int64_t), stream));
    HIP_RETURN_IF_ERROR(dpf_hip_gather_seeds_layout(
        K, T, static_cast<const int64_t*>(ctx.slots_), static_cast<const dpf_block*>(ctx.leaf_seeds_),
        ctx.leaf_stride_, static_cast<dpf_block*>(ctx.next_seeds_),
        static_cast<uint8_t*>(ctx.next_ctrl_), ctx.index_major_ ? 1 : 0, stream));
    cache_in_use = false;  // copied out; from here on only the write target
    ctx.leaf_level_ = -1;  // rewritten in place by this call's kernel
    const size_t cache_need = static_cast<size_t>(K * leaf_stride) * sizeof(dpf_block);
    if (ctx.leaf_seeds_cap_ < cache_need) {
      // Regrow once the gather has read the old cache.
      HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(stream));
      ctx.Release(&ctx.leaf_seeds_, &ctx.leaf_seeds_cap_);
      if (!fits(cache_need, 8) || !ctx.TryAlloc(&ctx.leaf_seeds_, &ctx.leaf_seeds_cap_, cache_need))
        ++ctx.events_.cache_refused;
    }
    leaf_seeds = ctx.leaf_seeds_;
  }
  if (permute) {
    const size_t bytes = leaf_slot.size() * sizeof(int32_t);
    DPF_RETURN_IF_ERROR(ensure(&ctx.leaf_slot_, &ctx.leaf_slot_cap_, bytes));
    HIP_RETURN_IF_ERROR(dpf_hip_memcpy_h2d(ctx.leaf_slot_, leaf_slot.data(), bytes, stream));
    ctx.leaf_level_ = -1;  // rewritten in place by this call's kernel
  }

  clk.mark(3);
  const dpf_aes_key kl = AesKey(kPrgKeyLeft), kr = AesKey(kPrgKeyRight), kv = AesKey(kPrgKeyValue);
  // Cached start seeds carry their control bit in bit 0 (control_in NULL).
  const dpf_block* start_seeds =
      direct   ? static_cast<const dpf_block*>(ctx.leaf_seeds_)
      : gather ? static_cast<const dpf_block*>(ctx.next_seeds_)
               : (from_root ? nullptr : ctx.partial_seeds());
  const uint8_t* start_ctrl = direct   ? nullptr
                              : gather ? static_cast<const uint8_t*>(ctx.next_ctrl_)
                                       : (from_root ? nullptr : ctx.partial_control());
  const int64_t start_stride = direct   ? ctx.leaf_stride_
                               : gather ? T
                                        : static_cast<int64_t>(ctx.partial_prefixes_.size());
  auto launch = [&](int sum_mode, void* out, uint64_t* workspace) {
    return FromHip(dpf_hip_eval_prefix_batch_layout(
        K, U, Wk + s, update_ctx && !gather ? Wk : -1, E, cached ? Dprev : start_level,
        keys.num_levels(), keys.seed(), keys.party(), start_seeds, start_ctrl, start_stride,
        d_parent, d_path, d_save, static_cast<dpf_block*>(ctx.next_seeds_),
        static_cast<uint8_t*>(ctx.next_ctrl_), T, keys.cw_seed(), keys.cw_left(), keys.cw_right(),
        &kl, &kr, &kv, &desc, cepb, keys.value_correction(hierarchy_level), sum_mode, workspace,
        out, static_cast<dpf_block*>(leaf_seeds), cache_stride,
        permute ? static_cast<const int32_t*>(ctx.leaf_slot_) : nullptr, ctx.index_major_ ? 1 : 0,
        stream));
  };
  if (native_sum) {
    void* target = device_out;
    if (!identity) {
      DPF_RETURN_IF_ERROR(ensure(&ctx.stage_, &ctx.stage_cap_, n_blk * esz));
      target = ctx.stage_;
    }
    DPF_RETURN_IF_ERROR(ensure(
        &ctx.workspace_, &ctx.workspace_cap_, n_blk * f.leaves.size() * 3 * sizeof(uint64_t)));
    DPF_RETURN_IF_ERROR(launch(1, target, static_cast<uint64_t*>(ctx.workspace_)));
    if (!identity)
      HIP_RETURN_IF_ERROR(dpf_hip_gather(P, cnt, esz, d_offsets,
                                         ctx.stage_, device_out, stream));
  } else if (sum) {
    // Value types without an on-device key sum in the kernel: per-key rows,
    // then a group sum over the rows.
    DPF_RETURN_IF_ERROR(ensure(&ctx.stage_, &ctx.stage_cap_, K * n_blk * esz));
    DPF_RETURN_IF_ERROR(launch(0, ctx.stage_, nullptr));
    void* target = device_out;
    if (!identity) {
      DPF_RETURN_IF_ERROR(ensure(&ctx.stage2_, &ctx.stage2_cap_, n_blk * esz));
      target = ctx.stage2_;
    }
    HIP_RETURN_IF_ERROR(dpf_hip_sum_rows(K, n_blk, &desc, ctx.stage_, target, stream));
    if (!identity)
      HIP_RETURN_IF_ERROR(dpf_hip_gather(P, cnt, esz, d_offsets,
                                         ctx.stage2_, device_out, stream));
  } else {
    void* target = device_out;
    if (!identity) {
      DPF_RETURN_IF_ERROR(ensure(&ctx.stage_, &ctx.stage_cap_, K * n_blk * esz));
      target = ctx.stage_;
    }
    DPF_RETURN_IF_ERROR(launch(0, target, nullptr));
    if (!identity)
      HIP_RETURN_IF_ERROR(dpf_hip_gather_batched(K, n_blk, P, cnt, esz,
                                                 d_offsets,
                                                 ctx.stage_, device_out, stream));
  }

  if (swap_cache) {
    std::swap(ctx.leaf_seeds_, ctx.leaf_spare_);
    std::swap(ctx.leaf_seeds_cap_, ctx.leaf_spare_cap_);
  }
  ctx.leaf_level_ = leaf_seeds ? hierarchy_level : -1;
  ctx.leaf_de_ = dE;
  ctx.leaf_stride_ = cache_stride;
  if (permute)
    ctx.leaf_phys_.assign(leaf_slot.begin(), leaf_slot.end());
  else
    ctx.leaf_phys_.clear();   // written in leaf order
  // After the last level nothing reads the cache; its buffers stay allocated
  // for the next pass over the hierarchy (Reset()), because giving them back
  // and regrowing them level by level (4, 16, 64 GiB for 2^20 heavy-hitters
  // clients) cost 3.7 s per 22 s pass (profiles/r14_ab.txt).  The 1/8-of-HBM
  // headroom rule above bounds what they take; callers that need the memory
  // call ReleaseExpansionCache() (or Reset(true)).
  if (hierarchy_level == H - 1) ctx.leaf_level_ = -1;
  if (g_timing_on) dpf_hip_stream_sync(stream);  // attribute device time to its phase
  clk.mark(4);
  // Context update (cc:435-451, 494-496).
  ctx.previous_hierarchy_level_ = hierarchy_level;
  if (P > 0) {
    if (update_ctx) {
      std::swap(ctx.partial_prefixes_, tree_indices);
      ctx.partial_sorted_ = indices_ascending;
      std::swap(ctx.seeds_, ctx.next_seeds_);
      std::swap(ctx.seeds_cap_, ctx.next_seeds_cap_);
      std::swap(ctx.ctrl_, ctx.next_ctrl_);
      std::swap(ctx.ctrl_cap_, ctx.next_ctrl_cap_);
    } else {
      ctx.partial_prefixes_.clear();
      ctx.partial_sorted_ = false;
    }
    ctx.partial_evaluations_level_ = prev;
  }
  ctx.spare_prefixes_ = std::move(tree_indices);
  clk.mark(5);
  return n;
}

StatusOr<EvaluationContext> DistributedPointFunction::ExportEvaluationContext(
    const DeviceBatchContext& ctx, const KeyBatch& host_keys, int64_t k, void* stream) const {
  const DeviceKeyBatch& keys = ctx.keys();
  if (k < 0 || k >= keys.num_keys()) return InvalidArgumentError("key index out of range");
  DPF_ASSIGN_OR_RETURN(DpfKey key, KeyFromBatch(host_keys, keys.first_key() + k));
  DPF_ASSIGN_OR_RETURN(EvaluationContext out, CreateEvaluationContext(std::move(key)));
  out.set_previous_hierarchy_level(ctx.previous_hierarchy_level());
  if (ctx.partial_evaluations_level() >= 0)
    out.set_partial_evaluations_level(ctx.partial_evaluations_level());
  const auto& q = ctx.partial_prefixes();
  if (!q.empty()) {
    const int64_t Q = static_cast<int64_t>(q.size());
    std::vector<dpf_block> seeds(Q);
    std::vector<uint8_t> ctrl(Q);
    if (ctx.index_major()) {
      // Key k's column of the [prefix][key] tables.
      const int64_t K = keys.num_keys();
      HIP_RETURN_IF_ERROR(dpf_hip_memcpy_d2h_strided(seeds.data(), ctx.partial_seeds() + k,
                                                     sizeof(dpf_block), K * sizeof(dpf_block), Q,
                                                     stream));
      HIP_RETURN_IF_ERROR(
          dpf_hip_memcpy_d2h_strided(ctrl.data(), ctx.partial_control() + k, 1, K, Q, stream));
    } else {
      HIP_RETURN_IF_ERROR(dpf_hip_memcpy_d2h(seeds.data(), ctx.partial_seeds() + k * Q,
                                             Q * sizeof(dpf_block), stream));
      HIP_RETURN_IF_ERROR(dpf_hip_memcpy_d2h(ctrl.data(), ctx.partial_control() + k * Q, Q, stream));
    }
    for (int64_t i = 0; i < Q; ++i) {
      PartialEvaluation* e = out.add_partial_evaluations();
      SetProtoBlock(q[i], e->mutable_prefix());
      SetProtoBlock(FromBlock(seeds[i]), e->mutable_seed());
      e->set_control_bit(ctrl[i] != 0);
    }
  }
  return out;
}

}  // namespace distributed_point_functions
