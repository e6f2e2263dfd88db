// aes_128_fixed_key_hash.h -- host-side fixed-key AES-128 MMO hash
//   H_k(x) = AES_k(sigma(x)) ^ sigma(x),  sigma(x) = MakeUint128(hi ^ lo, hi)
// (interface and semantics of the reference's dpf/aes_128_fixed_key_hash.h:27-85).
// Used on the host by key generation, which stays on the CPU; bulk evaluation
// runs on the GPU through dpf_hip_hash / the fused kernels (include/dpf_hip.h).
#ifndef DPF_AES_128_FIXED_KEY_HASH_H_
#define DPF_AES_128_FIXED_KEY_HASH_H_

#include <cstdint>

#include "dpf/span.h"
#include "dpf/status.h"
#include "dpf/uint128.h"

namespace distributed_point_functions {

class Aes128FixedKeyHash {
 public:
  static constexpr int kBatchSize = 64;  // aes_128_fixed_key_hash.h:69
  static StatusOr<Aes128FixedKeyHash> Create(uint128 key);
  // out[i] = H_key(in[i]); in and out may alias.
  Status Evaluate(Span<const uint128> in, Span<uint128> out) const;
  uint128 key() const { return key_; }
  const uint8_t* key_bytes() const { return reinterpret_cast<const uint8_t*>(&key_); }

 private:
  uint128 key_ = 0;
  alignas(16) uint32_t rk_[44];
  bool use_aesni_ = false;
};

}  // namespace distributed_point_functions

#endif  // DPF_AES_128_FIXED_KEY_HASH_H_
