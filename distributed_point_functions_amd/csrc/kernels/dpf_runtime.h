// dpf_runtime.h -- host-side plumbing shared by the kernel translation units:
// absl status codes, the thread-local last-error message
// behind dpf_hip_last_error(), and launch-shape helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../../include/dpf_hip.h"

namespace dpf_rt {

constexpr int kOk = 0, kInvalidArgument = 3, kResourceExhausted = 8, kFailedPrecondition = 9,
              kUnimplemented = 12, kInternal = 13;

// Records `msg` as the calling thread's last error and returns `code`.
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

int num_cus();                                 // compute units of the current device
int block_for(int64_t work_items);             // threads per workgroup: kBlock, or fewer
                                               // (multiple of 64) to spread a small launch over more CUs
int grid_for(int64_t work_items, int block);   // workgroups of `block` threads, <= one per CU
// Chunks of 64 items per workgroup for take_chunk (dpf_device.h), or 0 (a
// fixed share per thread): dynamic when the launch gives every wave at least
// 4 chunks and `env` is not "0" (A/B and test hooks, read per launch).
int64_t dynamic_chunks_per_wg(int64_t items, int grid, int block, const char* env);
int validate_desc(const dpf_value_desc* d);    // kOk or the failure code
int packed_size(const dpf_value_desc* d);      // bytes of one packed element
bool fast_int(const dpf_value_desc* d);        // one plain/XOR integer leaf, direct, b == 1

// One steady-state heavy-hitters level (dpf_batch_hh.hip): start seeds from
// the expansion cache or gathered partial evaluations, no path walk, two
// expanded levels, Tuple/IntModN<uint32_t> values summed over the keys.
struct HHLevelArgs {
  int64_t num_keys, num_starts;
  int cw_level, cw_stride;
  const dpf_block* seeds_in;
  const uint8_t* ctrl_in;    // NULL: control bit in bit 0 of the seed
  int64_t in_stride;
  const int32_t* parent;
  int save;                   // 1: store each start node as the key's partial evaluation
  const int32_t* save_index;  // NULL (with save): start node u at index u
  dpf_block* seeds_out;
  uint8_t* ctrl_out;
  int64_t out_stride;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  const dpf_block* vcw;
  int vcw_stride;
  const uint8_t* party;
  unsigned long long* wide;
  dpf_block* leaf_seeds;
  int64_t leaf_stride;
  const int32_t* leaf_slot;  // NULL: leaf i of start node u at slot (u << 2) + i
  // 0: per-key tables key-major, element (k, j) at k*stride + j; sums into
  //    the 192-bit [slot][leaf][3] workspace (hh_level_kernel).
  // 1: index-major, element (k, j) at j*num_keys + k (the device batch
  //    context's layout); lanes are keys (hh_keys_kernel) and the sums go to
  //    one uint64 per [slot][leaf] (finalize with words == 1).
  int index_major;
  int nl, b;
  uint32_t mod[2];
  const dpf_aes_key* key_left;
  const dpf_aes_key* key_right;
  const dpf_aes_key* key_value;
};
int launch_hh_level(const HHLevelArgs& a, hipStream_t s);
int launch_hh_keys(const HHLevelArgs& a, hipStream_t s);   // index_major == 1

}  // namespace dpf_rt

#define HIP_TRY(expr)                                           \
  do {                                                          \
    hipError_t _e = (expr);                                     \
    if (_e != hipSuccess) return ::dpf_rt::hip_fail(_e, #expr); \
  } while (0)
