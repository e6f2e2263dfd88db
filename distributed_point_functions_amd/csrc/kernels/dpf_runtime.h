// dpf_runtime.h -- host-side plumbing shared by the kernel translation units:
// absl status codes, the thread-local last-error message
// behind dpf_hip_last_error(), and launch-shape helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../../include/dpf_hip.h"

namespace dpf_rt {

constexpr int kOk = 0, kInvalidArgument = 3, kResourceExhausted = 8, kUnimplemented = 12,
              kInternal = 13;

// Records `msg` as the calling thread's last error and returns `code`.
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

int num_cus();                                 // compute units of the current device
int block_for(int64_t work_items);             // threads per workgroup: kBlock, or fewer
                                               // (multiple of 64) to spread a small launch over more CUs
int grid_for(int64_t work_items, int block);   // workgroups of `block` threads, <= one per CU
int validate_desc(const dpf_value_desc* d);    // kOk or the failure code
int packed_size(const dpf_value_desc* d);      // bytes of one packed element
bool fast_int(const dpf_value_desc* d);        // one plain/XOR integer leaf, direct, b == 1

}  // namespace dpf_rt

#define HIP_TRY(expr)                                           \
  do {                                                          \
    hipError_t _e = (expr);                                     \
    if (_e != hipSuccess) return ::dpf_rt::hip_fail(_e, #expr); \
  } while (0)
