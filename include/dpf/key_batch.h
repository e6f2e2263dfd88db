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

}  // namespace distributed_point_functions

#endif  // DPF_KEY_BATCH_H_
