// xor_wrapper.h -- group (T, XOR): + and - are XOR, negation is the identity
// (semantics of the reference's dpf/xor_wrapper.h:40-73).
#ifndef DPF_XOR_WRAPPER_H_
#define DPF_XOR_WRAPPER_H_

#include <utility>

namespace distributed_point_functions {

template <typename T>
class XorWrapper {
 public:
  using WrappedType = T;
  constexpr XorWrapper() : v_{} {}
  explicit constexpr XorWrapper(T v) : v_(std::move(v)) {}
  constexpr T& value() { return v_; }
  constexpr const T& value() const { return v_; }
  constexpr XorWrapper& operator+=(const XorWrapper& o) { v_ ^= o.v_; return *this; }
  constexpr XorWrapper& operator-=(const XorWrapper& o) { v_ ^= o.v_; return *this; }
  friend constexpr XorWrapper operator+(XorWrapper a, const XorWrapper& b) { return a += b; }
  friend constexpr XorWrapper operator-(XorWrapper a, const XorWrapper& b) { return a -= b; }
  friend constexpr XorWrapper operator-(const XorWrapper& a) { return a; }
  friend constexpr bool operator==(const XorWrapper& a, const XorWrapper& b) { return a.v_ == b.v_; }
  friend constexpr bool operator!=(const XorWrapper& a, const XorWrapper& b) { return !(a == b); }

 private:
  T v_;
};

}  // namespace distributed_point_functions

#endif  // DPF_XOR_WRAPPER_H_
