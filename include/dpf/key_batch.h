// key_batch.h -- many DpfKeys of one DistributedPointFunction as one
// structure-of-arrays image, the layout of the batched GPU paths.
//
// Not in the reference, which evaluates one DpfKey per call (the batched
// configurations of SURVEY.md section 8d -- 2^20 keys x 2^10 EvaluateAt points,
// and the 2^20-client heavy-hitters hierarchy -- loop over keys).  A KeyBatch
// holds exactly the fields of each DpfKey (distributed_point_function.proto:
// 114-140) that evaluation reads:
//   seed[k], party[k]                       DpfKey.seed, DpfKey.party
//   cw_seed/cw_left/cw_right[k * L + j]     DpfKey.correction_words[j]
//   value_correction[h][k * E_h * nl_h + i] the value correction of hierarchy
//                                           level h as flattened leaves
//                                           (correction_words[hierarchy_to_tree
//                                           [h]].value_correction, or
//                                           last_level_value_correction)
// with L = tree_levels_needed - 1 correction words per key.  Rows are keys, so
// a range of rows is one contiguous slice of every array (key-batch sharding
// across GPUs).
#ifndef DPF_KEY_BATCH_H_
#define DPF_KEY_BATCH_H_

#include <cstdint>
#include <memory>
#include <vector>

#include "dpf/status.h"
#include "dpf/uint128.h"
#include "dpf_hip.h"

namespace distributed_point_functions {

struct KeyBatch {
  int64_t num_keys = 0;
  int num_levels = 0;  // correction words per key
  std::vector<dpf_block> seed;
  std::vector<uint8_t> party;
  std::vector<dpf_block> cw_seed;
  std::vector<uint8_t> cw_left, cw_right;
  std::vector<std::vector<dpf_block>> value_correction;  // [hierarchy level]
};

// A KeyBatch (or a contiguous row range of one) resident in device memory,
// uploaded once and reused by every batched evaluation of those keys.
class DeviceKeyBatch {
 public:
  // Uploads rows [begin, end) of `batch` on `stream` (a hipStream_t, may be null).
  static StatusOr<std::unique_ptr<DeviceKeyBatch>> Upload(const KeyBatch& batch, int64_t begin,
                                                          int64_t end, void* stream);
  static StatusOr<std::unique_ptr<DeviceKeyBatch>> Upload(const KeyBatch& batch, void* stream) {
    return Upload(batch, 0, batch.num_keys, stream);
  }
  DeviceKeyBatch(const DeviceKeyBatch&) = delete;
  DeviceKeyBatch& operator=(const DeviceKeyBatch&) = delete;
  ~DeviceKeyBatch();

  int64_t num_keys() const { return num_keys_; }
  int num_levels() const { return num_levels_; }
  // First key of this range in the host batch it came from.
  int64_t first_key() const { return first_key_; }
  const dpf_block* seed() const { return static_cast<const dpf_block*>(seed_); }
  const uint8_t* party() const { return static_cast<const uint8_t*>(party_); }
  const dpf_block* cw_seed() const { return static_cast<const dpf_block*>(cw_seed_); }
  const uint8_t* cw_left() const { return static_cast<const uint8_t*>(cw_left_); }
  const uint8_t* cw_right() const { return static_cast<const uint8_t*>(cw_right_); }
  const dpf_block* value_correction(int h) const {
    return static_cast<const dpf_block*>(vcw_[h]);
  }
  int num_hierarchy_levels() const { return static_cast<int>(vcw_.size()); }

 private:
  DeviceKeyBatch() = default;
  int64_t num_keys_ = 0, first_key_ = 0;
  int num_levels_ = 0;
  void* seed_ = nullptr;
  void* party_ = nullptr;
  void* cw_seed_ = nullptr;
  void* cw_left_ = nullptr;
  void* cw_right_ = nullptr;
  std::vector<void*> vcw_;
};

// The EvaluationContext (distributed_point_function.proto:142-171) of every key
// of a DeviceKeyBatch, kept in device memory between incremental evaluations
// (SURVEY.md 8f.1): the batch is evaluated at the SAME prefixes for all keys
// (the heavy-hitters pattern of config 5b), so the context holds one shared
// list of partial-evaluation prefixes (tree indices at depth
// hierarchy_to_tree[partial_evaluations_level]) and, per key, the seed and
// control bit at each of them -- index-major, [prefix][key], so 64
// consecutive keys at one prefix are one 1 KiB access (DPF_BATCH_KEY_MAJOR=1
// at creation: key-major [key][prefix]) -- instead of a protobuf repeated
// field per key.  Created by
// DistributedPointFunction::CreateBatchEvaluationContext; serialized lazily to
// a per-key EvaluationContext proto by ExportEvaluationContext.
class DeviceBatchContext {
 public:
  DeviceBatchContext(const DeviceBatchContext&) = delete;
  DeviceBatchContext& operator=(const DeviceBatchContext&) = delete;
  ~DeviceBatchContext();

  const DeviceKeyBatch& keys() const { return *keys_; }
  int previous_hierarchy_level() const { return previous_hierarchy_level_; }
  int partial_evaluations_level() const { return partial_evaluations_level_; }
  // Shared partial-evaluation prefixes (tree indices), in evaluation order.
  const std::vector<uint128>& partial_prefixes() const { return partial_prefixes_; }
  // Device arrays [partial_prefixes().size()][num_keys] (index_major()), else
  // [num_keys][partial_prefixes().size()].
  const dpf_block* partial_seeds() const { return static_cast<const dpf_block*>(seeds_); }
  const uint8_t* partial_control() const { return static_cast<const uint8_t*>(ctrl_); }
  // Layout of the partial evaluations and the expansion cache.
  bool index_major() const { return index_major_; }
  // Back to the state CreateBatchEvaluationContext returns, keeping the
  // device allocations for the next pass over the hierarchy; with
  // `release_expansion_cache` the expansion cache (up to K x 4096 x 16 B per
  // buffer) is given back too.
  void Reset(bool release_expansion_cache = false);
  // Frees the expansion cache's buffers (the next call walks down from the
  // partial evaluations and rebuilds it).  Outputs are unaffected.
  void ReleaseExpansionCache();
  // Hierarchy level whose call wrote the expansion cache (-1: none).
  int expansion_cache_level() const { return leaf_level_; }
  // Device bytes this context holds (partial evaluations, expansion cache,
  // per-call scratch).
  size_t device_bytes() const { return device_bytes_; }
  // What the expansion cache did under memory pressure, since creation.
  struct CacheEvents {
    int64_t cache_refused = 0;   // no room for the cache: the call wrote none
    int64_t spare_refused = 0;   // no room for a spare: start seeds gathered, cache rewritten in place
    int64_t in_place = 0;        // calls that gathered their start seeds, then rewrote the cache
    int64_t permuted = 0;        // calls that rewrote the cache in place through a slot table (no gather)
    int64_t evicted_spare = 0;   // spare freed so a per-call buffer fits
    int64_t evicted_cache = 0;   // unread cache freed so a per-call buffer fits
    int64_t alloc_failures = 0;  // per-call allocations that failed (before any eviction)
  };
  const CacheEvents& cache_events() const { return events_; }
  // Test hook: after `skip` more per-call buffer requests, the next n fail as
  // if the device were out of memory (whether or not the buffer has to grow).
  void FailNextAllocationsForTesting(int n, int skip = 0) {
    fail_next_ = n;
    fail_skip_ = skip;
  }

 private:
  friend class DistributedPointFunction;
  explicit DeviceBatchContext(const DeviceKeyBatch* keys) : keys_(keys) {}
  // Grows a device allocation (contents are not preserved).  Failures are
  // RESOURCE_EXHAUSTED "Memory allocation error" (distributed_point_function.cc:289-291).
  Status Ensure(void** p, size_t* cap, size_t bytes);
  // Allocates exactly `bytes` into *p (*p must be null); false on failure.
  bool TryAlloc(void** p, size_t* cap, size_t bytes);
  void Release(void** p, size_t* cap);
  // Page-locked image of a call's start-node tables (and output offsets),
  // sent with one asynchronous H2D: StageTables waits for the previous
  // call's copy and makes room for `bytes`; TablesSent marks the copy.
  Status StageTables(size_t bytes);
  Status TablesSent(void* stream);
  // Free and total device memory as this context sees it (DPF_BATCH_ALLOC_LIMIT
  // replaces the device's figures with the limit, as a test hook).
  void MemInfo(size_t* free_bytes, size_t* total_bytes) const;

  const DeviceKeyBatch* keys_;
  int previous_hierarchy_level_ = -1;
  int partial_evaluations_level_ = -1;
  std::vector<uint128> partial_prefixes_;
  bool partial_sorted_ = false;  // partial_prefixes_ strictly ascending (skips a check)
  std::vector<uint128> spare_prefixes_;  // recycled storage for the next prefix list
  void* seeds_ = nullptr;  // current partial evaluations
  void* ctrl_ = nullptr;
  size_t seeds_cap_ = 0, ctrl_cap_ = 0;
  void* next_seeds_ = nullptr;  // written by the next evaluation, then swapped in
  void* next_ctrl_ = nullptr;
  size_t next_seeds_cap_ = 0, next_ctrl_cap_ = 0;
  bool index_major_ = true;
  // Expansion cache: the tree leaves of the last call ([leaf_stride_][key]
  // index-major, else [key][leaf_stride_]),
  // i.e. the next call's tree nodes (DistributedPointFunction's batched
  // EvaluateUntil reads its start seeds from it instead of walking down
  // from the partial evaluations two calls back).  leaf_de_: levels from a
  // tree index of that call to its leaves.  Double-buffered: a call reads
  // leaf_seeds_ and writes leaf_spare_, then the two swap; without room for
  // the spare the kernel rewrites the cache in place, each leaf into a slot
  // that only its own thread reads or nobody reads (leaf_phys_: logical leaf
  // -> physical slot, empty = identity), and when no such slot table exists
  // the start seeds are gathered first (slots_).  leaf_stride_ is the
  // physical row stride.
  std::vector<int32_t> leaf_phys_;
  void* leaf_slot_ = nullptr;  // device copy of the slot table of the running call
  size_t leaf_slot_cap_ = 0;
  void* leaf_seeds_ = nullptr;  // seed | control bit (bit 0)
  size_t leaf_seeds_cap_ = 0;
  void* leaf_spare_ = nullptr;
  size_t leaf_spare_cap_ = 0;
  int64_t leaf_stride_ = 0;
  int leaf_level_ = -1;
  int leaf_de_ = 0;
  void* slots_ = nullptr;
  size_t slots_cap_ = 0;
  size_t device_bytes_ = 0;  // sum of the caps below and above
  CacheEvents events_;
  int fail_next_ = 0, fail_skip_ = 0;
  void* pinned_tables_ = nullptr;
  size_t pinned_tables_cap_ = 0;
  void* tables_event_ = nullptr;
  bool tables_pending_ = false;
  // Per-call scratch: start-node tables (parent_: the device copy of the
  // whole table image), sums workspace, staging output.
  void* parent_ = nullptr;
  void* path_ = nullptr;
  void* save_ = nullptr;
  void* offsets_ = nullptr;
  void* workspace_ = nullptr;
  void* stage_ = nullptr;
  void* stage2_ = nullptr;
  size_t parent_cap_ = 0, path_cap_ = 0, save_cap_ = 0, offsets_cap_ = 0, workspace_cap_ = 0,
         stage_cap_ = 0, stage2_cap_ = 0;
};

}  // namespace distributed_point_functions

#endif  // DPF_KEY_BATCH_H_
