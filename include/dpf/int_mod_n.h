// int_mod_n.h -- integers modulo a compile-time N stored in BaseInteger
// (semantics of the reference's dpf/int_mod_n.h:116-245 and int_mod_n.cc):
// a - b = a >= b ? a - b : N - b + a; a + b = a - (N - b); -a = 0 - a.
// Sampling parameters (GetSecurityLevel / GetNumBytesRequired) live in
// internal/value_type_helpers.h.
#ifndef DPF_INT_MOD_N_H_
#define DPF_INT_MOD_N_H_

#include <type_traits>

#include "dpf/uint128.h"

namespace distributed_point_functions {
namespace dpf_internal {

template <typename BaseInteger, typename ModulusType, ModulusType kModulus>
class IntModNImpl {
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
