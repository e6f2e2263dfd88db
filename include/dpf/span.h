// span.h -- a minimal absl::Span equivalent (constructible from containers,
// arrays, pointer+size and initializer lists), so that reference call sites like
// `dpf->EvaluateUntil<T>(1, {prefix}, ctx)` compile unchanged.
#ifndef DPF_SPAN_H_
#define DPF_SPAN_H_

#include <cstddef>
#include <initializer_list>
#include <type_traits>
#include <vector>

namespace distributed_point_functions {

template <typename T>
class Span {
 public:
  using element_type = T;
  using value_type = std::remove_cv_t<T>;
  using iterator = T*;

  constexpr Span() = default;
  constexpr Span(T* data, size_t size) : data_(data), size_(size) {}
  template <size_t N>
  constexpr Span(T (&a)[N]) : data_(a), size_(N) {}  // NOLINT
  template <typename C, typename = decltype(std::declval<C&>().data()),
            typename = std::enable_if_t<std::is_convertible_v<
                std::remove_pointer_t<decltype(std::declval<C&>().data())> (*)[], T (*)[]>>>
  constexpr Span(C& c) : data_(c.data()), size_(c.size()) {}  // NOLINT
  // Read-only spans also bind const containers and temporaries (absl::Span<const T>).
  template <typename C, typename U = T, typename = std::enable_if_t<std::is_const_v<U>>,
            typename = decltype(std::declval<const C&>().data()),
            typename = std::enable_if_t<std::is_convertible_v<
                std::remove_pointer_t<decltype(std::declval<const C&>().data())> (*)[], T (*)[]>>>
  constexpr Span(const C& c) : data_(c.data()), size_(c.size()) {}  // NOLINT
  template <typename U = T, typename = std::enable_if_t<std::is_const_v<U>>>
  Span(std::initializer_list<value_type> il) : data_(il.begin()), size_(il.size()) {}  // NOLINT

  constexpr T* data() const { return data_; }
  constexpr size_t size() const { return size_; }
  constexpr bool empty() const { return size_ == 0; }
  constexpr T& operator[](size_t i) const { return data_[i]; }
  constexpr T* begin() const { return data_; }
  constexpr T* end() const { return data_ + size_; }
  constexpr T& back() const { return data_[size_ - 1]; }
  constexpr Span subspan(size_t pos, size_t len) const { return Span(data_ + pos, len); }

 private:
  T* data_ = nullptr;
  size_t size_ = 0;
};

template <typename T>
Span<T> MakeSpan(T* p, size_t n) { return Span<T>(p, n); }
template <typename C>
auto MakeSpan(C& c) { return Span<std::remove_pointer_t<decltype(c.data())>>(c.data(), c.size()); }
template <typename T>
Span<const T> MakeConstSpan(const T* p, size_t n) { return Span<const T>(p, n); }
template <typename C>
auto MakeConstSpan(const C& c) {
  return Span<const std::remove_pointer_t<decltype(c.data())>>(c.data(), c.size());
}

}  // namespace distributed_point_functions

#endif  // DPF_SPAN_H_
