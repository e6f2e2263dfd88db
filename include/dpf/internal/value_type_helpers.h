// value_type_helpers.h -- value types of the DPF output groups.
//
// Restates the behaviour of the reference's dpf/internal/value_type_helpers.{h,cc}
// in a form suited to a GPU engine: every ValueType is *flattened* into its
// integer leaves (declaration order).  Flattening is exact for nested tuples:
// DirectlyFromBytes reads leaves at consecutive offsets (h:415-428) and
// SampleAndUpdateBytes updates after every leaf but the last (h:430-443).
// Templates (ValueTypeHelper<T>) only map C++ values <-> leaves; all semantics
// (validation messages, conversion, group ops) live in value_type_helpers.cc.
#ifndef DPF_INTERNAL_VALUE_TYPE_HELPERS_H_
#define DPF_INTERNAL_VALUE_TYPE_HELPERS_H_

#include <cstring>
#include <functional>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "dpf/distributed_point_function.pb.h"
#include "dpf/int_mod_n.h"
#include "dpf/status.h"
#include "dpf/tuple.h"
#include "dpf/uint128.h"
#include "dpf/xor_wrapper.h"

namespace distributed_point_functions {
namespace dpf_internal {

enum LeafKind { kLeafInt = 0, kLeafIntModN = 1, kLeafXor = 2 };

struct LeafSpec {
  int kind = kLeafInt;
  int bits = 0;
  uint128 modulus = 0;
};

// A ValueType flattened to its leaves.
struct FlatValueType {
  std::vector<LeafSpec> leaves;
  bool direct = true;          // CanBeConvertedDirectly (no IntModN leaf), h:342-344
  int total_bits = 0;          // TotalBitSize
  int packed_size = 0;         // bytes of one packed element (sum of leaf bytes)
  int elements_per_block = 1;  // ElementsPerBlock<T>(), h:508-520
};

// ---- free functions (value_type_helpers.cc) --------------------------------
StatusOr<FlatValueType> Flatten(const ValueType& value_type);
StatusOr<bool> ValueTypesAreEqual(const ValueType& lhs, const ValueType& rhs);
StatusOr<int> BitsNeeded(const ValueType& value_type, double security_parameter);
StatusOr<uint128> ValueIntegerToUint128(const Value::Integer& in);
Value::Integer Uint128ToValueInteger(uint128 in);
std::string SerializeValueTypeDeterministically(const ValueType& value_type);

// Shorthands for IntModNBase (dpf/int_mod_n.h, int_mod_n.cc).
inline double IntModNSecurityLevel(int num_samples, uint128 modulus) {
  return IntModNBase::GetSecurityLevel(num_samples, modulus);
}
inline Status IntModNCheckParameters(int num_samples, int base_integer_bitsize, uint128 modulus,
                                     double security_parameter) {
  return IntModNBase::CheckParameters(num_samples, base_integer_bitsize, modulus,
                                      security_parameter);
}
inline StatusOr<int> IntModNNumBytesRequired(int num_samples, int base_integer_bitsize,
                                             uint128 modulus, double security_parameter) {
  return IntModNBase::GetNumBytesRequired(num_samples, base_integer_bitsize, modulus,
                                          security_parameter);
}

// FromValue for a runtime ValueType, with the reference's error messages.
StatusOr<std::vector<uint128>> ValueToLeaves(const ValueType& type, const Value& value);
// ToValue for a runtime ValueType from flattened leaves (advances *pos).
Value LeavesToValue(const ValueType& type, const uint128* leaves, int* pos);
// ValuesToArray (h:544-563): exactly ElementsPerBlock values -> E * num_leaves leaves.
StatusOr<std::vector<uint128>> ValuesToLeafArray(const ValueType& type, const FlatValueType& flat,
                                                 const RepeatedField<Value>& values);
// ConvertBytesToArrayOf (h:569-589): bytes (blocks_needed * 16) -> E * num_leaves leaves.
void ConvertBytesToLeaves(const FlatValueType& flat, const uint8_t* bytes, uint128* out);
// Group operations on one leaf (int_mod_n.h, xor_wrapper.h, unsigned wrap-around).
uint128 LeafAdd(const LeafSpec& s, uint128 a, uint128 b);
uint128 LeafSub(const LeafSpec& s, uint128 a, uint128 b);
uint128 LeafNeg(const LeafSpec& s, uint128 a);
// Packed element bytes <-> leaves.
void PackLeaves(const FlatValueType& flat, const uint128* leaves, uint8_t* out);
void UnpackLeaves(const FlatValueType& flat, const uint8_t* in, uint128* leaves);

// ---- templates --------------------------------------------------------------
template <typename T>
using is_unsigned_integer =
    std::disjunction<std::is_same<T, uint8_t>, std::is_same<T, uint16_t>,
                     std::is_same<T, uint32_t>, std::is_same<T, uint64_t>,
                     std::is_same<T, uint128>>;

template <typename T, typename = void>
struct ValueTypeHelper {
  static constexpr bool IsSupportedType() { return false; }
};

template <typename T>
struct is_supported_type {
  static constexpr bool value = ValueTypeHelper<T>::IsSupportedType();
};
template <typename T>
constexpr bool is_supported_type_v = is_supported_type<T>::value;

// Unsigned integers.
template <typename T>
struct ValueTypeHelper<T, std::enable_if_t<is_unsigned_integer<T>::value>> {
  static constexpr bool IsSupportedType() { return true; }
  static constexpr int kNumLeaves = 1;
  static ValueType ToValueType() {
    ValueType r;
    r.mutable_integer()->set_bitsize(8 * sizeof(T));
    return r;
  }
  static Value ToValue(T v) {
    Value r;
    *r.mutable_integer() = Uint128ToValueInteger(static_cast<uint128>(v));
    return r;
  }
  static void ToLeaves(const T& v, uint128* out) { out[0] = static_cast<uint128>(v); }
  static T FromLeaves(const uint128* in) { return static_cast<T>(in[0]); }
  // Packed element image (little-endian, leaves back to back): sizeof(T) bytes.
  static constexpr int kPackedBytes = sizeof(T);
  static T FromPacked(const uint8_t* p) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    return v;
  }
};

// IntModN.
template <typename B, typename M, M kModulus>
struct ValueTypeHelper<IntModNImpl<B, M, kModulus>, void> {
  using Type = IntModNImpl<B, M, kModulus>;
  static constexpr bool IsSupportedType() { return is_unsigned_integer<B>::value; }
  static constexpr int kNumLeaves = 1;
  static ValueType ToValueType() {
    ValueType r;
    r.mutable_int_mod_n()->mutable_base_integer()->set_bitsize(8 * sizeof(B));
    *r.mutable_int_mod_n()->mutable_modulus() = Uint128ToValueInteger(static_cast<uint128>(kModulus));
    return r;
  }
  static Value ToValue(const Type& v) {
    Value r;
    *r.mutable_int_mod_n() = Uint128ToValueInteger(static_cast<uint128>(v.value()));
    return r;
  }
  static void ToLeaves(const Type& v, uint128* out) { out[0] = static_cast<uint128>(v.value()); }
  static Type FromLeaves(const uint128* in) { return Type(static_cast<B>(in[0])); }
  static constexpr int kPackedBytes = sizeof(B);
  static Type FromPacked(const uint8_t* p) {
    B v;
    std::memcpy(&v, p, sizeof(B));
    return Type(v);
  }
};

// XorWrapper.
template <typename T>
struct ValueTypeHelper<XorWrapper<T>, void> {
  static constexpr bool IsSupportedType() { return is_unsigned_integer<T>::value; }
  static constexpr int kNumLeaves = 1;
  static ValueType ToValueType() {
    ValueType r;
    r.mutable_xor_wrapper()->set_bitsize(8 * sizeof(T));
    return r;
  }
  static Value ToValue(const XorWrapper<T>& v) {
    Value r;
    *r.mutable_xor_wrapper() = Uint128ToValueInteger(static_cast<uint128>(v.value()));
    return r;
  }
  static void ToLeaves(const XorWrapper<T>& v, uint128* out) {
    out[0] = static_cast<uint128>(v.value());
  }
  static XorWrapper<T> FromLeaves(const uint128* in) {
    return XorWrapper<T>(static_cast<T>(in[0]));
  }
  static constexpr int kPackedBytes = sizeof(T);
  static XorWrapper<T> FromPacked(const uint8_t* p) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    return XorWrapper<T>(v);
  }
};

// Tuples.
template <typename... E>
struct ValueTypeHelper<Tuple<E...>, void> {
  using Type = Tuple<E...>;
  static constexpr bool IsSupportedType() { return (is_supported_type<E>::value && ...); }
  static constexpr int kNumLeaves = (ValueTypeHelper<E>::kNumLeaves + ... + 0);
  static ValueType ToValueType() {
    ValueType r;
    ValueType::Tuple* t = r.mutable_tuple();
    ((*t->add_elements() = ValueTypeHelper<E>::ToValueType()), ...);
    return r;
  }
  static Value ToValue(const Type& v) {
    Value r;
    Value::Tuple* t = r.mutable_tuple();
    std::apply([&](const E&... e) { ((*t->add_elements() = ValueTypeHelper<E>::ToValue(e)), ...); },
               v.value());
    return r;
  }
  static void ToLeaves(const Type& v, uint128* out) {
    int pos = 0;
    std::apply([&](const E&... e) {
      ((ValueTypeHelper<E>::ToLeaves(e, out + pos), pos += ValueTypeHelper<E>::kNumLeaves), ...);
    }, v.value());
  }
  static Type FromLeaves(const uint128* in) {
    int pos = 0;
    // Braced init list: left-to-right evaluation.
    return Type(typename Type::Base{Take<E>(in, pos)...});
  }
  static constexpr int kPackedBytes = (ValueTypeHelper<E>::kPackedBytes + ... + 0);
  static Type FromPacked(const uint8_t* p) {
    int off = 0;
    return Type(typename Type::Base{TakePacked<E>(p, off)...});
  }

 private:
  template <typename X>
  static X TakePacked(const uint8_t* p, int& off) {
    X x = ValueTypeHelper<X>::FromPacked(p + off);
    off += ValueTypeHelper<X>::kPackedBytes;
    return x;
  }
  template <typename X>
  static X Take(const uint128* in, int& pos) {
    X x = ValueTypeHelper<X>::FromLeaves(in + pos);
    pos += ValueTypeHelper<X>::kNumLeaves;
    return x;
  }
};

template <typename T>
ValueType ToValueTypeImpl() { return ValueTypeHelper<T>::ToValueType(); }

template <typename T>
StatusOr<T> FromValueImpl(const Value& value) {
  StatusOr<std::vector<uint128>> leaves = ValueToLeaves(ValueTypeHelper<T>::ToValueType(), value);
  if (!leaves.ok()) return leaves.status();
  return ValueTypeHelper<T>::FromLeaves(leaves->data());
}

// Plain unsigned integers: the packed image of n elements IS the array of T.
template <typename T>
constexpr bool kPackedIsMemoryImage =
    (std::is_integral_v<T> && std::is_unsigned_v<T> && !std::is_same_v<T, bool>) ||
    std::is_same_v<T, uint128>;

// Asks the kernel for transparent huge pages on [p, p + bytes) before it is
// first touched: a fresh 128 MiB output vector costs ~22 ms of 4 KiB page
// faults on the GPU box's host, ~7 ms with 2 MiB pages.  No-op below 4 MiB.
void AdviseHugePages(void* p, size_t bytes);

// Maps the pages of fresh storage [p, p + bytes) by touching them on up to 16
// host threads.  8 GiB: 30-47 ms, where the page faults of a one-thread
// first touch (value-initialisation) cost ~350 of the ~500 ms it takes
// (tools/host_output_microbench.cc).  No-op below 64 MiB.
void PrefaultPages(void* p, size_t bytes);

// Storage of a fresh std::vector<T> of n elements, reserved, advised onto huge
// pages and (with `prefault`) pre-faulted, but still empty (size 0).  The
// HostSinks below do not pre-fault: their copies map the pages as the data
// lands (dpf_hip_memcpy_d2h_staged maps and registers a large range piece by
// piece behind its DMA; below DPF_HIP_REGISTER_MIN_BYTES a 16-thread
// pre-fault measured slower than faulting chunk by chunk,
// profiles/r14b_fresh_output_microbench.jsonl).
template <typename T>
void ReserveOutputVector(std::vector<T>& out, int64_t n, bool prefault = true) {
  out.clear();
  out.reserve(n);
  AdviseHugePages(out.data(), static_cast<size_t>(n) * sizeof(T));
  if (prefault) PrefaultPages(out.data(), static_cast<size_t>(n) * sizeof(T));
}

// A read-only mapping of `*bytes` (64 MiB) bytes of the kernel's zero page,
// made on first use and kept for the life of the process.
const void* ZeroPages(size_t* bytes);

// out->resize(n) for a growing vector, with the value-initialisation of
// integer elements (absl::uint128 included) done by memmove from ZeroPages():
// libstdc++ value-initialises a 16-byte element with a load/store loop (34
// GB/s on the GPU box's host) where a large memmove or memset streams at 70-75
// GB/s -- the one-thread bound of config 3's 32 GiB host output
// (profiles/r15_value_init_probe.jsonl).  Other element types: resize().
template <typename T>
void GrowZeroed(std::vector<T>* out, size_t n) {
  if constexpr (std::is_arithmetic_v<T> || std::is_same_v<T, uint128>) {
    size_t span = 0;
    const T* zeros = static_cast<const T*>(ZeroPages(&span));
    const size_t per = span / sizeof(T);
    if (zeros && per > 0) {
      while (out->size() < n) {
        const size_t k = n - out->size() < per ? n - out->size() : per;
        out->insert(out->end(), zeros, zeros + k);
      }
      if (out->size() > n) out->resize(n);
      return;
    }
  }
  out->resize(n);
}

// A value-initialised std::vector<T> of n elements whose storage was advised
// onto huge pages and mapped on the host threads before the (one-thread)
// initialisation touched it.
template <typename T>
std::vector<T> MakeOutputVector(int64_t n) {
  std::vector<T> out;
  ReserveOutputVector(out, n);
  GrowZeroed(&out, static_cast<size_t>(n));
  return out;
}

// Where a packed device output is copied on the host (EvaluateUntilToHost):
// reserve(bytes) returns storage for it (or nullptr when the sink takes the
// bytes chunk by chunk); grow(bytes) (may be empty) makes its first `bytes`
// bytes valid and is called chunk by chunk right before each chunk's DMA, so a
// fresh vector's value-initialisation overlaps the copy
// (dpf_hip_memcpy_d2h_staged).  chunk(bytes, offset, len) (may be empty)
// receives [offset, offset + len) of the packed output from page-locked
// staging while the next chunk's DMA runs (dpf_hip_memcpy_d2h_chunked; len
// and offset multiples of `align`): used for every output below
// DPF_HIP_REGISTER_MIN_BYTES and whenever reserve() returned nullptr.
struct HostSink {
  std::function<void*(size_t bytes)> reserve;
  std::function<void(size_t bytes)> grow;
  std::function<void(const uint8_t* bytes, size_t offset, size_t len)> chunk;
  size_t align = 1;
};

// fn(lo, hi) over [0, n) in chunks of at least `grain`, on up to 16 host threads.
void ParallelRanges(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& fn);

// The HostSink that fills a fresh std::vector<T> (bytes: a multiple of sizeof(T)).
template <typename T>
HostSink VectorSink(std::vector<T>* out) {
  HostSink s;
  s.reserve = [out](size_t bytes) -> void* {
    ReserveOutputVector(*out, static_cast<int64_t>(bytes / sizeof(T)), false);
    return out->data();
  };
  s.grow = [out](size_t bytes) { GrowZeroed(out, (bytes + sizeof(T) - 1) / sizeof(T)); };
  s.chunk = [out](const uint8_t* src, size_t offset, size_t len) {
    // (Already grown when CopyToHostSink grew the whole result up front.)
    if (out->size() < (offset + len) / sizeof(T)) GrowZeroed(out, (offset + len) / sizeof(T));
    uint8_t* dst = reinterpret_cast<uint8_t*>(out->data()) + offset;
    ParallelRanges(static_cast<int64_t>(len), int64_t{2} << 20, [&](int64_t lo, int64_t hi) {
      std::memcpy(dst + lo, src + lo, static_cast<size_t>(hi - lo));
    });
  };
  s.align = sizeof(T);
  return s;
}

// Unpacks n packed elements of T into out[0, n) (value_type_helpers.h:526-589:
// the packed image is the kernels' little-endian leaf concatenation).
template <typename T>
void UnpackInto(const FlatValueType& flat, const uint8_t* data, int64_t n, T* out) {
  if (flat.packed_size == ValueTypeHelper<T>::kPackedBytes) {
    // The packed layout of T is known at compile time: fixed-width loads of
    // each leaf straight into the element (no per-leaf uint128 round trip).
    const int step = flat.packed_size;
    ParallelRanges(n, int64_t{1} << 15, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) out[i] = ValueTypeHelper<T>::FromPacked(data + i * step);
    });
    return;
  }
  ParallelRanges(n, int64_t{1} << 15, [&](int64_t lo, int64_t hi) {
    std::vector<uint128> leaves(flat.leaves.size());
    for (int64_t i = lo; i < hi; ++i) {
      UnpackLeaves(flat, data + i * flat.packed_size, leaves.data());
      out[i] = ValueTypeHelper<T>::FromLeaves(leaves.data());
    }
  });
}

// The HostSink that unpacks packed elements of T into a fresh std::vector<T>
// chunk by chunk, straight out of page-locked staging (no host copy of the
// packed bytes).
template <typename T>
HostSink UnpackSink(const std::vector<FlatValueType>* flats, int h, std::vector<T>* out) {
  HostSink s;
  s.reserve = [flats, h, out](size_t bytes) -> void* {
    ReserveOutputVector(*out, static_cast<int64_t>(bytes / (*flats)[h].packed_size), false);
    return nullptr;
  };
  // Value-initialises the whole result (CopyToHostSink runs it on a helper
  // thread while the DMA of the first chunk is in flight).
  s.grow = [flats, h, out](size_t bytes) {
    out->resize(bytes / static_cast<size_t>((*flats)[h].packed_size));
  };
  s.chunk = [flats, h, out](const uint8_t* src, size_t offset, size_t len) {
    const FlatValueType& flat = (*flats)[h];
    const int64_t first = static_cast<int64_t>(offset / flat.packed_size);
    const int64_t cnt = static_cast<int64_t>(len / flat.packed_size);
    if (static_cast<int64_t>(out->size()) < first + cnt) out->resize(first + cnt);
    UnpackInto<T>(flat, src, cnt, out->data() + first);
  };
  // Valid levels only (the sink is used after validation); 1 otherwise.
  s.align = h >= 0 && h < static_cast<int>(flats->size()) ? (*flats)[h].packed_size : 1;
  return s;
}

// Unpacks n packed elements of T.
template <typename T>
std::vector<T> UnpackElements(const FlatValueType& flat, const uint8_t* data, int64_t n) {
  if constexpr (kPackedIsMemoryImage<T>) {
    if (flat.leaves.size() == 1 && flat.packed_size == static_cast<int>(sizeof(T)) &&
        flat.leaves[0].bits == static_cast<int>(8 * sizeof(T)) && flat.leaves[0].kind == kLeafInt) {
      std::vector<T> out = MakeOutputVector<T>(n);
      if (n) std::memcpy(out.data(), data, n * sizeof(T));
      return out;
    }
  }
  std::vector<T> out = MakeOutputVector<T>(n);
  UnpackInto<T>(flat, data, n, out.data());
  return out;
}

}  // namespace dpf_internal
}  // namespace distributed_point_functions

#endif  // DPF_INTERNAL_VALUE_TYPE_HELPERS_H_
