// uint128.h -- 128-bit unsigned integers for the host API.  The reference uses
// absl::uint128, whose memory image (low word first, little-endian) is the
// native unsigned __int128 on x86-64; the helpers mirror absl's names.
#ifndef DPF_UINT128_H_
#define DPF_UINT128_H_

#include <cstdint>
#include <string>

namespace distributed_point_functions {

using uint128 = unsigned __int128;

constexpr uint128 MakeUint128(uint64_t high, uint64_t low) {
  return (static_cast<uint128>(high) << 64) | low;
}
constexpr uint64_t Uint128High64(uint128 v) { return static_cast<uint64_t>(v >> 64); }
constexpr uint64_t Uint128Low64(uint128 v) { return static_cast<uint64_t>(v); }
constexpr uint128 Uint128Max() { return ~static_cast<uint128>(0); }

// Decimal rendering (absl's StrFormat("%d", uint128)).
inline std::string Uint128ToString(uint128 v) {
  if (v == 0) return "0";
  char buf[48];
  int i = 47;
  buf[i] = 0;
  while (v) {
    buf[--i] = static_cast<char>('0' + static_cast<int>(v % 10));
    v /= 10;
  }
  return std::string(buf + i);
}

}  // namespace distributed_point_functions

#endif  // DPF_UINT128_H_
