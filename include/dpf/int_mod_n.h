// int_mod_n.h -- integers modulo a compile-time N stored in BaseInteger
// (semantics of the reference's dpf/int_mod_n.h:116-245 and int_mod_n.cc):
// a - b = a >= b ? a - b : N - b + a; a + b = a - (N - b); -a = 0 - a.
// The sampling API of the reference is here with the same signatures and
// Status messages: IntModNBase::{GetSecurityLevel, CheckParameters,
// GetNumBytesRequired, ConvertBytesTo} (dpf/int_mod_n.h:35-80, defined in
// csrc/host/value_type_helpers.cc after int_mod_n.cc:21-76) and
// IntModN::{GetNumBytesRequired, UnsafeSampleFromBytes, SampleFromBytes}
// (dpf/int_mod_n.h:136-205).
#ifndef DPF_INT_MOD_N_H_
#define DPF_INT_MOD_N_H_

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <type_traits>
#include <vector>

#include "dpf/span.h"
#include "dpf/status.h"
#include "dpf/uint128.h"

namespace distributed_point_functions {
namespace dpf_internal {

// Functions of IntModN independent of its template parameters
// (dpf/int_mod_n.h:35-80).
class IntModNBase {
 public:
  // Statistical security of sampling `num_samples` elements mod `modulus` from
  // one 128-bit block plus one BaseInteger per further sample (int_mod_n.cc:21-26).
  static double GetSecurityLevel(int num_samples, uint128 modulus);
  // OK for valid parameters, INVALID_ARGUMENT otherwise (int_mod_n.cc:28-61).
  static Status CheckParameters(int num_samples, int base_integer_bitsize, uint128 modulus,
                                double security_parameter);
  // 16 + bytes(BaseInteger) * (num_samples - 1), or CheckParameters' error
  // (int_mod_n.cc:63-76).
  static StatusOr<int> GetNumBytesRequired(int num_samples, int base_integer_bitsize,
                                           uint128 modulus, double security_parameter);
  // Little-endian bytes -> T; aborts if bytes.size() != sizeof(T) (h:66-79).
  template <typename T>
  static T ConvertBytesTo(std::string_view bytes) {
    if (bytes.size() != sizeof(T)) std::abort();
    T out{0};
    std::memcpy(&out, bytes.data(), sizeof(T));
    return out;
  }
};

template <typename BaseInteger, typename ModulusType, ModulusType kModulus>
class IntModNImpl : public IntModNBase {
  static_assert(sizeof(BaseInteger) <= 16, "BaseInteger may be at most 128 bits");
  static_assert(kModulus <= ModulusType(BaseInteger(-1)), "kModulus must fit in BaseInteger");

 public:
  using Base = BaseInteger;
  constexpr IntModNImpl() : value_(0) {}
  explicit constexpr IntModNImpl(BaseInteger v) : value_(static_cast<BaseInteger>(v % kModulus)) {}
  constexpr IntModNImpl& operator=(const BaseInteger& v) {
    value_ = static_cast<BaseInteger>(v % kModulus);
    return *this;
  }
  constexpr IntModNImpl& operator+=(const IntModNImpl& a) {
    Sub(static_cast<BaseInteger>(kModulus - a.value_));
    return *this;
  }
  constexpr IntModNImpl& operator-=(const IntModNImpl& a) {
    Sub(a.value_);
    return *this;
  }
  constexpr BaseInteger value() const { return value_; }
  static constexpr BaseInteger modulus() { return static_cast<BaseInteger>(kModulus); }

  // Bytes needed to sample `num_samples` elements within total variation
  // distance 2^-security_parameter (h:136-140).
  static StatusOr<int> GetNumBytesRequired(int num_samples, double security_parameter) {
    return IntModNBase::GetNumBytesRequired(num_samples, 8 * sizeof(BaseInteger),
                                            static_cast<uint128>(kModulus), security_parameter);
  }

  // r = first 16 bytes; sample i = r mod N, then r = (r / N) << bits(Base) |
  // next Base-sized bytes (h:154-177).  Does not check bytes.size().
  template <int kCompiledNumSamples = 1>
  static void UnsafeSampleFromBytes(std::string_view bytes, double security_parameter,
                                    Span<IntModNImpl> samples) {
    static_assert(kCompiledNumSamples >= 1, "kCompiledNumSamples must be positive");
    (void)security_parameter;
    uint128 r = ConvertBytesTo<uint128>(bytes.substr(0, 16));
    const int n = static_cast<int>(samples.size());
    for (int i = 0; i < n; ++i) {
      samples[i] = IntModNImpl(static_cast<BaseInteger>(r % static_cast<uint128>(kModulus)));
      if (i + 1 < n) {
        r /= static_cast<uint128>(kModulus);
        if constexpr (sizeof(BaseInteger) < sizeof(uint128)) r <<= (sizeof(BaseInteger) * 8);
        r |= static_cast<uint128>(ConvertBytesTo<BaseInteger>(
            bytes.substr(16 + i * sizeof(BaseInteger), sizeof(BaseInteger))));
      }
    }
  }

  // UnsafeSampleFromBytes after checking there are enough bytes (h:185-205).
  static Status SampleFromBytes(std::string_view bytes, double security_parameter,
                                Span<IntModNImpl> samples) {
    if (samples.empty()) return InvalidArgumentError("The number of samples required must be > 0");
    StatusOr<int> lower = GetNumBytesRequired(static_cast<int>(samples.size()), security_parameter);
    if (!lower.ok()) return lower.status();
    if (static_cast<size_t>(*lower) > bytes.size())
      return InvalidArgumentError("The number of bytes provided (" + std::to_string(bytes.size()) +
                                  ") is insufficient for the required statistical security and "
                                  "number of samples.");
    UnsafeSampleFromBytes(bytes, security_parameter, samples);
    return OkStatus();
  }

  friend constexpr IntModNImpl operator+(IntModNImpl a, const IntModNImpl& b) { return a += b; }
  friend constexpr IntModNImpl operator-(IntModNImpl a, const IntModNImpl& b) { return a -= b; }
  friend constexpr IntModNImpl operator-(const IntModNImpl& a) {
    IntModNImpl r(BaseInteger{0});
    r -= a;
    return r;
  }
  friend constexpr bool operator==(const IntModNImpl& a, const IntModNImpl& b) {
    return a.value_ == b.value_;
  }
  friend constexpr bool operator!=(const IntModNImpl& a, const IntModNImpl& b) { return !(a == b); }

 private:
  constexpr void Sub(BaseInteger a) {
    if (value_ >= a) value_ = static_cast<BaseInteger>(value_ - a);
    else value_ = static_cast<BaseInteger>(kModulus - a + value_);
  }
  BaseInteger value_;
};

}  // namespace dpf_internal

template <typename BaseInteger, uint128 kModulus>
using IntModN = dpf_internal::IntModNImpl<BaseInteger, uint128, kModulus>;

}  // namespace distributed_point_functions

#endif  // DPF_INT_MOD_N_H_
