// aes_128_fixed_key_hash.cc -- host MMO hash: AES-NI when the CPU has it,
// otherwise the portable 4-T-table formulation shared with the GPU kernels
// (csrc/kernels/aes_core.h, HostLookup).
#include "dpf/aes_128_fixed_key_hash.h"

#include <cpuid.h>
#include <immintrin.h>

#include <cstring>

#include "../kernels/aes_core.h"

namespace distributed_point_functions {
namespace {

bool CpuHasAesni() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c & bit_AES) != 0;
}

__attribute__((target("aes,sse4.1"))) void HashAesni(const uint32_t* rk, const uint128* in,
                                                     uint128* out, size_t n) {
  __m128i k[11];
  for (int i = 0; i < 11; ++i) k[i] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(rk + 4 * i));
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    __m128i s[4], x[4];
    for (int j = 0; j < 4; ++j) {
      __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(in + i + j));
      // sigma: low <- high, high <- high ^ low
      __m128i hi = _mm_unpackhi_epi64(v, v);
      s[j] = _mm_xor_si128(hi, _mm_slli_si128(v, 8));
      x[j] = _mm_xor_si128(s[j], k[0]);
    }
    for (int r = 1; r < 10; ++r)
      for (int j = 0; j < 4; ++j) x[j] = _mm_aesenc_si128(x[j], k[r]);
    for (int j = 0; j < 4; ++j) {
      x[j] = _mm_aesenclast_si128(x[j], k[10]);
      _mm_storeu_si128(reinterpret_cast<__m128i*>(out + i + j), _mm_xor_si128(x[j], s[j]));
    }
  }
  for (; i < n; ++i) {
    __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(in + i));
    __m128i s = _mm_xor_si128(_mm_unpackhi_epi64(v, v), _mm_slli_si128(v, 8));
    __m128i x = _mm_xor_si128(s, k[0]);
    for (int r = 1; r < 10; ++r) x = _mm_aesenc_si128(x, k[r]);
    x = _mm_aesenclast_si128(x, k[10]);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + i), _mm_xor_si128(x, s));
  }
}

const dpf_aes::HostLookup& Tables() {
  static const dpf_aes::HostLookup* t = new dpf_aes::HostLookup();
  return *t;
}

}  // namespace

StatusOr<Aes128FixedKeyHash> Aes128FixedKeyHash::Create(uint128 key) {
  Aes128FixedKeyHash h;
  h.key_ = key;
  uint8_t kb[16];
  std::memcpy(kb, &key, 16);  // memory image of the uint128 key (aes_128_fixed_key_hash.cc:38-40)
  dpf_aes::expand_key(kb, h.rk_);
  h.use_aesni_ = CpuHasAesni();
  return h;
}

Status Aes128FixedKeyHash::Evaluate(Span<const uint128> in, Span<uint128> out) const {
  if (in.size() != out.size()) return InvalidArgumentError("Input and output sizes don't match");
  if (in.empty()) return OkStatus();
  if (use_aesni_) {
    HashAesni(rk_, in.data(), out.data(), in.size());
    return OkStatus();
  }
  const dpf_aes::HostLookup& lk = Tables();
  for (size_t i = 0; i < in.size(); ++i) {
    dpf_aes::Block4 b;
    std::memcpy(&b, &in[i], 16);
    dpf_aes::Block4 h = dpf_aes::mmo_hash(b, lk, dpf_aes::ArrayRK{rk_});
    std::memcpy(&out[i], &h, 16);
  }
  return OkStatus();
}

}  // namespace distributed_point_functions
