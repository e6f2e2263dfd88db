// Host checks of the bitsliced AES engine (tools/bs_aes.h) against the
// FIPS-197 S-box and the T-table MMO hash of aes_core.h (itself pinned by the
// reference KAT, tests/test_oracle.py).  Built and run by tests/test_bs_aes_cpu.py.
#include <stdio.h>
#include <string.h>

#include <random>

#include "../../distributed_point_functions_amd/csrc/kernels/aes_core.h"
#include "../../tools/bs_aes.h"

static int g_bad = 0;

// The value PRG key (distributed_point_function.cc:37-42) as a memory image.
static constexpr uint8_t kv[16] = {0x98, 0x1c, 0x1d, 0xb2, 0x01, 0x11, 0xa3, 0x46,
                                   0xe3, 0x23, 0x54, 0x8c, 0x58, 0xd1, 0xa5, 0x05};
struct KM {
  static constexpr bsa::BsKeyMasks m = bsa::make_key_masks_c(kv);
};
#define CHECK(c, ...)                  \
  do {                                 \
    if (!(c)) {                        \
      ++g_bad;                         \
      if (g_bad < 20) {                \
        printf("FAIL %s:%d: ", __FILE__, __LINE__); \
        printf(__VA_ARGS__);           \
        printf("\n");                  \
      }                                \
    }                                  \
  } while (0)

int main() {
  std::mt19937_64 rng(0xB17511CEu);
  // 1. S-box: 32 inputs per plane word, all 256 values.
  for (int batch = 0; batch < 8; ++batch) {
    uint32_t x[8] = {0};
    for (int b = 0; b < 32; ++b)
      for (int i = 0; i < 8; ++i) x[i] |= (uint32_t)(((32 * batch + b) >> i) & 1) << b;
    bsa::sbox_planes(x[7], x[6], x[5], x[4], x[3], x[2], x[1], x[0]);
    for (int b = 0; b < 32; ++b) {
      int v = 0;
      for (int i = 0; i < 8; ++i) v |= ((x[i] >> b) & 1) << i;
      CHECK(v == dpf_aes::kSbox[32 * batch + b], "sbox(%d) = %02x", 32 * batch + b, v);
    }
  }
  // 2. Transposes: definition and round trip.
  for (int it = 0; it < 16; ++it) {
    uint32_t w[32], p[32];
    for (auto& v : w) v = (uint32_t)rng();
    memcpy(p, w, sizeof w);
    bsa::to_planes(p);
    for (int b = 0; b < 8; ++b)
      for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
          for (int i = 0; i < 8; ++i) {
            const uint32_t want = (w[4 * b + c] >> (8 * r + i)) & 1;
            const uint32_t got = (p[4 * i + r] >> (8 * c + b)) & 1;
            CHECK(want == got, "plane bit b=%d c=%d r=%d i=%d", b, c, r, i);
          }
    bsa::from_planes(p);
    CHECK(!memcmp(p, w, sizeof w), "transpose round trip");
  }
  // 3. MMO hash vs the T-table hash: the reference's three PRG keys
  //    (distributed_point_function.cc:37-42) and the KAT keys.
  const uint64_t keys[][2] = {{0x0000000000000000ull, 0x0000000000000000ull},
                              {0x1111111111111111ull, 0x1111111111111111ull},
                              {0x5be037ccf6a03de5ull, 0x935f08e19ab2b1ccull},
                              {0xef55d2f1bdf1e6b5ull, 0x2d5c2f5d7f6b4e5bull},
                              {0x0123456789abcdefull, 0xfedcba9876543210ull}};
  dpf_aes::HostLookup lk;
  for (const auto& k : keys) {
    uint8_t kb[16];
    memcpy(kb, &k[1], 8);  // low 64 first (absl::uint128 memory image)
    memcpy(kb + 8, &k[0], 8);
    uint32_t rk[44];
    dpf_aes::expand_key(kb, rk);
    const bsa::BsKeyMasks km = bsa::make_key_masks(rk);
    for (int it = 0; it < 64; ++it) {
      uint32_t w[32], ref[32];
      for (auto& v : w) v = (uint32_t)rng();
      if (it == 0) memset(w, 0, sizeof w);
      for (int b = 0; b < 8; ++b) {
        dpf_aes::Block4 x{w[4 * b], w[4 * b + 1], w[4 * b + 2], w[4 * b + 3]};
        dpf_aes::Block4 h = dpf_aes::mmo_hash(x, lk, dpf_aes::ArrayRK{rk});
        ref[4 * b] = h.w0; ref[4 * b + 1] = h.w1; ref[4 * b + 2] = h.w2; ref[4 * b + 3] = h.w3;
      }
      bsa::mmo8(w, bsa::ArrayMasks{km.m});
      CHECK(!memcmp(w, ref, sizeof w), "mmo8 vs T-table, key %016llx, it %d",
            (unsigned long long)k[0], it);
    }
  }
  // 4. Compile-time masks (make_key_masks_c) equal the run-time ones, and the
  //    unrolled literal-mask AES (aes8_c, used by dpf_expand_hybrid.hip) plus
  //    the MMO feed-forward equals the T-table hash under the value PRG key.
  {
    uint32_t rk[44];
    dpf_aes::expand_key(kv, rk);
    const bsa::BsKeyMasks km = bsa::make_key_masks(rk);
    CHECK(!memcmp(km.m, KM::m.m, sizeof km.m), "constexpr key masks");
    for (int it = 0; it < 64; ++it) {
      uint32_t w[32], ref[32], sg[32];
      for (auto& v : w) v = (uint32_t)rng();
      for (int b = 0; b < 8; ++b) {
        dpf_aes::Block4 x{w[4 * b], w[4 * b + 1], w[4 * b + 2], w[4 * b + 3]};
        dpf_aes::Block4 h = dpf_aes::mmo_hash(x, lk, dpf_aes::ArrayRK{rk});
        ref[4 * b] = h.w0; ref[4 * b + 1] = h.w1; ref[4 * b + 2] = h.w2; ref[4 * b + 3] = h.w3;
        dpf_aes::Block4 s = dpf_aes::sigma(x);
        sg[4 * b] = s.w0; sg[4 * b + 1] = s.w1; sg[4 * b + 2] = s.w2; sg[4 * b + 3] = s.w3;
      }
      uint32_t e[32];
      memcpy(e, sg, sizeof e);
      bsa::aes8_c<KM>(e);
      for (int j = 0; j < 32; ++j) e[j] ^= sg[j];
      CHECK(!memcmp(e, ref, sizeof e), "aes8_c + feed-forward vs T-table, it %d", it);
    }
  }
  printf("bs_aes_test: %d failures\n", g_bad);
  return g_bad ? 1 : 0;
}
