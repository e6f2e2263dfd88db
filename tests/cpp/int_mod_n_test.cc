// Restates the reference's dpf/int_mod_n_test.cc:32-254 (and the constexpr
// checks of dpf/tuple.h) against the drop-in headers include/dpf/int_mod_n.h
// and include/dpf/tuple.h: the typed tests over IntModN<uint32_t, 2^32-5>,
// IntModN<uint64_t, 2^64-59> and IntModN<uint128, 2^80-65>, the sampling
// chain on "this is a length 32 test string." and the static_asserts that
// the operators are constexpr.  Self-contained (no gtest in this image):
// prints "<n> failures" and exits non-zero on any failure.
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "dpf/int_mod_n.h"
#include "dpf/tuple.h"

namespace dpf = distributed_point_functions;
using dpf::uint128;

namespace {

int g_failures = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      ++g_failures;                                                    \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);      \
    }                                                                  \
  } while (0)

constexpr double kFeasibleSecurityParameter = 40;
constexpr double kUnfeasibleSecurityParameter = 95;
constexpr int kNumSamples = 5;

std::string U128(uint128 v) {
  if (v == 0) return "0";
  std::string s;
  while (v) {
    s.insert(s.begin(), char('0' + int(v % 10)));
    v /= 10;
  }
  return s;
}

template <typename T>
void TypedTests() {
  {  // DefaultValueIsZero, SetValueWorks
    T a;
    EXPECT(a.value() == 0);
    a = 23;
    EXPECT(a.value() == 23);
  }
  {  // AdditionWithoutWrapAroundWorks
    T a, b;
    a += b;
    EXPECT(a.value() == 0);
    b = 23;
    a += b;
    EXPECT(a.value() == 23);
    b = 4294967200u;
    a += b;
    EXPECT(a.value() == 4294967223u);
  }
  {  // AdditionWithWrapAroundWorks
    T a, b;
    b = 23;
    a += b;
    b = T::modulus() - 10;
    a += b;
    EXPECT(a.value() == 13);
  }
  {  // SubtractionWithoutWrapAroundWorks / WithWrapAround / Negation
    T a(100), b(23);
    EXPECT((a - b).value() == 77);
    EXPECT((b - a).value() == T::modulus() - 77);
    T c(10);
    T d = -c;
    EXPECT(c + d == T(0));
  }
  {  // GetNumBytesRequiredFailsIfUnfeasible
    auto r = T::GetNumBytesRequired(kNumSamples, kUnfeasibleSecurityParameter);
    EXPECT(!r.ok());
    const std::string want = "For num_samples = 5 and kModulus = " + U128(uint128(T::modulus()));
    EXPECT(r.status().code() == dpf::StatusCode::kInvalidArgument);
    EXPECT(r.status().message().rfind(want, 0) == 0);
  }
  {  // GetNumBytesRequiredSucceedsIfFeasible
    auto r = T::GetNumBytesRequired(5, kFeasibleSecurityParameter);
    EXPECT(r.ok());
    EXPECT(*r == 16 + int(sizeof(typename T::Base)) * 4);
  }
  {  // SampleFailsIfUnfeasible
    auto r = T::GetNumBytesRequired(5, kFeasibleSecurityParameter);
    EXPECT(r.ok());
    std::string bytes(16, '#');
    EXPECT(size_t(*r) > bytes.size());
    std::vector<T> samples(5);
    dpf::Status s = T::SampleFromBytes(bytes, kFeasibleSecurityParameter,
                                       dpf::Span<T>(samples.data(), samples.size()));
    EXPECT(!s.ok());
    EXPECT(s.code() == dpf::StatusCode::kInvalidArgument);
    EXPECT(s.message() ==
           "The number of bytes provided (16) is insufficient for the required statistical "
           "security and number of samples.");
  }
  {  // SampleSucceedsIfFeasible, FirstEntryOfSamplesIsAsExpected
    auto r = T::GetNumBytesRequired(5, kFeasibleSecurityParameter);
    std::string bytes(*r, '#');
    std::vector<T> samples(5);
    dpf::Status s = T::SampleFromBytes(bytes, kFeasibleSecurityParameter,
                                       dpf::Span<T>(samples.data(), samples.size()));
    EXPECT(s.ok());
    EXPECT(samples[0].value() ==
           T::template ConvertBytesTo<uint128>(bytes.substr(0, 16)) % uint128(T::modulus()));
  }
  {  // zero samples (int_mod_n.h:188-191)
    std::vector<T> none;
    dpf::Status s = T::SampleFromBytes(std::string(64, 'x'), kFeasibleSecurityParameter,
                                       dpf::Span<T>(none.data(), 0));
    EXPECT(s.message() == "The number of samples required must be > 0");
  }
}

using MyIntModN = dpf::IntModN<uint32_t, 4294967291u>;  // 2**32 - 5

void ConcreteExample(bool corrupt_last) {
  auto r_getnum = MyIntModN::GetNumBytesRequired(5, kFeasibleSecurityParameter);
  EXPECT(r_getnum.ok());
  EXPECT(*r_getnum == 32);
  const std::string bytes = "this is a length 32 test string.";
  EXPECT(bytes.size() == 32);
  std::vector<MyIntModN> samples(5);
  dpf::Status st = MyIntModN::SampleFromBytes(bytes, kFeasibleSecurityParameter,
                                              dpf::Span<MyIntModN>(samples.data(), 5));
  EXPECT(st.ok());
  uint128 r = MyIntModN::ConvertBytesTo<uint128>("this is a length");
  EXPECT(samples[0].value() == r % MyIntModN::modulus());
  const char* words[4] = {" 32 ", "test", " str", corrupt_last ? "ing#" : "ing."};
  for (int i = 0; i < 4; ++i) {
    r /= MyIntModN::modulus();
    r <<= (sizeof(MyIntModN::Base) * 8);
    r |= MyIntModN::ConvertBytesTo<MyIntModN::Base>(words[i]);
    if (i == 3 && corrupt_last)
      EXPECT(samples[4].value() != r % MyIntModN::modulus());
    else
      EXPECT(samples[i + 1].value() == r % MyIntModN::modulus());
  }
}

void BaseChecks() {
  // IntModNBase used directly (int_mod_n.cc:21-76).
  using B = dpf::dpf_internal::IntModNBase;
  EXPECT(B::CheckParameters(0, 32, 7, 40).message() == "num_samples must be positive");
  EXPECT(B::CheckParameters(1, 0, 7, 40).message() == "base_integer_bitsize must be positive");
  EXPECT(B::CheckParameters(1, 129, 7, 40).message() == "base_integer_bitsize must be at most 128");
  EXPECT(B::CheckParameters(1, 8, 257, 40).message() ==
         "kModulus 257 out of range for base_integer_bitsize = 8");
  EXPECT(B::CheckParameters(1, 32, 4294967291u, 40).ok());
  const double sigma = B::GetSecurityLevel(5, 4294967291u);
  EXPECT(sigma > 90.0 && sigma < 95.0);  // 131 - (32 - 7e-9 + log2 5 + log2 6)
  auto n = B::GetNumBytesRequired(3, 64, uint128(1) << 63, 40);
  EXPECT(n.ok() && *n == 32);
}

// Constexpr operators (int_mod_n_test.cc:234-254; dpf/tuple.h:62-100).
constexpr MyIntModN TestAddition() { return MyIntModN(2) + MyIntModN(5); }
static_assert(TestAddition().value() == 7, "constexpr addition of IntModNs incorrect");
constexpr MyIntModN TestSubtraction() { return MyIntModN(5) - MyIntModN(2); }
static_assert(TestSubtraction().value() == 3, "constexpr subtraction of IntModNs incorrect");
constexpr MyIntModN TestAssignment() {
  MyIntModN x(0);
  x = 5;
  return x;
}
static_assert(TestAssignment().value() == 5, "constexpr assignment to IntModN incorrect");
constexpr unsigned __int128 kModulus128 = (unsigned __int128)(-1);
using MyIntModN128 = dpf::IntModN<unsigned __int128, kModulus128>;
constexpr MyIntModN128 TestAddition128() { return MyIntModN128(2) + MyIntModN128(5); }
static_assert(TestAddition128().value() == 7, "constexpr addition of IntModNs incorrect");

using T2 = dpf::Tuple<uint32_t, uint64_t>;
constexpr T2 TestTupleAdd() { return T2(1u, 2u) + T2(3u, 4u); }
static_assert(TestTupleAdd() == T2(4u, 6u), "constexpr Tuple addition incorrect");
constexpr T2 TestTupleNeg() { return -T2(1u, 1u); }
static_assert(std::get<0>(TestTupleNeg().value()) == 0xffffffffu, "constexpr Tuple negation");

}  // namespace

int main() {
  TypedTests<dpf::IntModN<uint32_t, 4294967291u>>();
  TypedTests<dpf::IntModN<uint64_t, 18446744073709551557ull>>();
  TypedTests<dpf::IntModN<uint128, (unsigned __int128)((uint128(65535) << 64) |
                                                       18446744073709551551ull)>>();
  ConcreteExample(false);
  ConcreteExample(true);
  BaseChecks();
  std::printf("%d failures\n", g_failures);
  return g_failures ? 1 : 0;
}
