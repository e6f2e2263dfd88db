// tuple.h -- element-wise group over several value types (semantics of the
// reference's dpf/tuple.h:62-114: +, binary -, unary -, ==; constexpr like it).
#ifndef DPF_TUPLE_H_
#define DPF_TUPLE_H_

#include <tuple>
#include <utility>

namespace distributed_point_functions {

template <typename... T>
class Tuple {
 public:
  using Base = std::tuple<T...>;
  Tuple() = default;
  constexpr Tuple(T... elements) : value_(std::move(elements)...) {}  // NOLINT
  explicit constexpr Tuple(Base t) : value_(std::move(t)) {}
  constexpr Base& value() { return value_; }
  constexpr const Base& value() const { return value_; }

  friend constexpr Tuple operator+(const Tuple& a, const Tuple& b) {
    return Combine(a, b, [](const auto& x, const auto& y) { return x + y; },
                   std::index_sequence_for<T...>{});
  }
  friend constexpr Tuple operator-(const Tuple& a, const Tuple& b) { return a + (-b); }
  friend constexpr Tuple operator-(const Tuple& a) {
    return Map(a, [](const auto& x) { return -x; }, std::index_sequence_for<T...>{});
  }
  constexpr Tuple& operator+=(const Tuple& b) { return *this = *this + b; }
  constexpr Tuple& operator-=(const Tuple& b) { return *this = *this - b; }
  friend constexpr bool operator==(const Tuple& a, const Tuple& b) { return a.value_ == b.value_; }
  friend constexpr bool operator!=(const Tuple& a, const Tuple& b) { return !(a == b); }

 private:
  template <typename F, size_t... I>
  static constexpr Tuple Combine(const Tuple& a, const Tuple& b, F f, std::index_sequence<I...>) {
    return Tuple(Base(static_cast<T>(f(std::get<I>(a.value_), std::get<I>(b.value_)))...));
  }
  template <typename F, size_t... I>
  static constexpr Tuple Map(const Tuple& a, F f, std::index_sequence<I...>) {
    return Tuple(Base(static_cast<T>(f(std::get<I>(a.value_)))...));
  }
  Base value_;
};

}  // namespace distributed_point_functions

#endif  // DPF_TUPLE_H_
