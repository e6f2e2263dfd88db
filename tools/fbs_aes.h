// fbs_aes.h -- "full bitslice" fixed-key AES-128 MMO hash for gfx950: 32
// blocks per lane, one 32-bit register per bit plane (128 planes), the form
// SURVEY.md §7.3.1 names for a whole-DFS bitsliced expansion.
//
// Semantics: H_k(x) = AES_k(sigma(x)) ^ sigma(x), sigma(x) = MakeUint128(hi ^ lo,
// hi) (dpf/aes_128_fixed_key_hash.cc:47-85), bit-exact with aes_core.h.
//
// Layout: plane p = 8 * k + i holds, in bit b, bit i of byte k of block b's
// 16-byte little-endian image (AES state byte k = (row k & 3, column k >> 2)).
//   * SubBytes: the 82-gate v_bitop3 S-box (bs_sbox_gen.h) on each byte's 8
//     planes: 16 x 82 full-rate VALU per round for the lane's 32 blocks.
//   * ShiftRows: register renaming.  "Phase" P says where the bytes are: the
//     logical byte (r, c) sits in physical column (c + P * r) & 3.  A round
//     reads at phase P + 1 after its ShiftRows and writes its MixColumns output
//     back in place, so the phase advances by one per round (period 4).
//   * MixColumns: b_r = xtime(u_r) ^ T ^ a_r with u_r = a_r ^ a_{r+1} and
//     T = u_0 ^ u_2 (all full-rate 2/3-input XORs); AddRoundKey folded in.
//   * Round keys: either compile-time (every mask an immediate truth table, no
//     instruction: `CKeys`) or run-time plane masks read from LDS as 16-byte
//     broadcasts (`MaskKeys`), folded into the u_r / T XORs, +4 VALU per
//     column over the compile-time form.
// Per block and round: 41 S-box + ~2.8 MixColumns(+key) VALU lane-ops.
#pragma once
#include <stdint.h>

#include "bs_aes.h"

namespace fbs {

using bsa::kXor3;
constexpr int kXnor3 = 0x69;

BS_HD constexpr int phys(int P, int r, int c) { return 4 * ((c + P * r) & 3) + r; }

BS_HD uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return BS3(a, b, c, kXor3); }

// x ^ y ^ (kbit ? ~0 : 0) with kbit known at compile time.
BS_HD uint32_t x2k(uint32_t a, uint32_t b, bool kbit) { return kbit ? ~(a ^ b) : (a ^ b); }
BS_HD uint32_t x3k(uint32_t a, uint32_t b, uint32_t c, bool kbit) {
  return kbit ? BS3(a, b, c, kXnor3) : BS3(a, b, c, kXor3);
}

// FBS_SBOX_GROUP: S-boxes the scheduler may interleave (a sched_barrier after
// every group keeps the live temporaries of at most that many S-boxes).
#ifndef FBS_SBOX_GROUP
#define FBS_SBOX_GROUP 2
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define FBS_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define FBS_FENCE() ((void)0)
#endif

BS_HD void sub_bytes(uint32_t* s) {
BS_UNROLL
  for (int k = 0; k < 16; ++k) {
    bsa::sbox_planes(s[8 * k + 7], s[8 * k + 6], s[8 * k + 5], s[8 * k + 4], s[8 * k + 3],
                     s[8 * k + 2], s[8 * k + 1], s[8 * k + 0]);
    if ((k + 1) % FBS_SBOX_GROUP == 0) FBS_FENCE();
  }
}

// Round-key bytes for compile-time keys: bytes[R][k] = byte k of round key R.
struct KeyBytes {
  uint8_t b[11][16];
};
constexpr KeyBytes key_bytes_c(const uint8_t (&key)[16]) {
  const bsa::RoundKeyWords rk = bsa::expand_key_c(key);
  KeyBytes kb{};
  for (int R = 0; R < 11; ++R)
    for (int k = 0; k < 16; ++k) kb.b[R][k] = (uint8_t)(rk.w[4 * R + k / 4] >> (8 * (k % 4)));
  return kb;
}
inline KeyBytes key_bytes(const uint32_t rk[44]) {
  KeyBytes kb{};
  for (int R = 0; R < 11; ++R)
    for (int k = 0; k < 16; ++k) kb.b[R][k] = (uint8_t)(rk[4 * R + k / 4] >> (8 * (k % 4)));
  return kb;
}

// ---------------------------------------------------------------------------
// Run-time key masks.  Per middle round R = 1..9 and logical column c, 40
// words (10 x 16-byte broadcast reads):
//   [0, 28): uk[r * 7 + m] = key bit m + 1 of output byte (r, c)  (folded into
//            u_r bit m, m = 0..6)
//   [28, 35): tk[j] = uk of row 0 ^ uk of row 2 at bit j (undoes the two keys
//            T = u_0 ^ u_2 picked up), j = 0..6
//   [35, 39): k0[r] = key bit 0 of output byte (r, c)
//   39: pad.
// Round 0 and round 10: 128 plane masks each.
// ---------------------------------------------------------------------------
constexpr int kColWords = 40;
struct MaskTable {
  uint32_t mid[9][4][kColWords];
  uint32_t first[128];
  uint32_t last[128];
};
inline uint32_t bitmask(const KeyBytes& kb, int R, int k, int i) {
  return ((kb.b[R][k] >> i) & 1) ? 0xffffffffu : 0u;
}
inline MaskTable make_mask_table(const KeyBytes& kb) {
  MaskTable t{};
  for (int R = 1; R <= 9; ++R)
    for (int c = 0; c < 4; ++c) {
      uint32_t* w = t.mid[R - 1][c];
      for (int r = 0; r < 4; ++r)
        for (int m = 0; m < 7; ++m) w[r * 7 + m] = bitmask(kb, R, 4 * c + r, m + 1);
      for (int j = 0; j < 7; ++j) w[28 + j] = w[0 * 7 + j] ^ w[2 * 7 + j];
      for (int r = 0; r < 4; ++r) w[35 + r] = bitmask(kb, R, 4 * c + r, 0);
      w[39] = 0;
    }
  for (int p = 0; p < 128; ++p) {
    t.first[p] = bitmask(kb, 0, p / 8, p % 8);
    t.last[p] = bitmask(kb, 10, p / 8, p % 8);
  }
  return t;
}

// MixColumns + AddRoundKey of logical column c, inputs/outputs at phase P
// (i.e. after the round's ShiftRows renaming).  `kw` = the column's 40 mask
// words (run-time keys) or nullptr with KB/R set (compile-time keys).
template <int P>
BS_HD void mix_column_masks(uint32_t* s, int c, const uint32_t* kw) {
  const int p0 = 8 * phys(P, 0, c), p1 = 8 * phys(P, 1, c), p2 = 8 * phys(P, 2, c),
            p3 = 8 * phys(P, 3, c);
  const int pr[4] = {p0, p1, p2, p3};
  uint32_t u[4][8];
BS_UNROLL
  for (int r = 0; r < 4; ++r) {
BS_UNROLL
    for (int m = 0; m < 7; ++m) u[r][m] = x3(s[pr[r] + m], s[pr[(r + 1) & 3] + m], kw[r * 7 + m]);
    u[r][7] = s[pr[r] + 7] ^ s[pr[(r + 1) & 3] + 7];
  }
  uint32_t T[8];
BS_UNROLL
  for (int j = 0; j < 7; ++j) T[j] = x3(u[0][j], u[2][j], kw[28 + j]);
  T[7] = u[0][7] ^ u[2][7];
BS_UNROLL
  for (int r = 0; r < 4; ++r) {
    uint32_t* a = s + pr[r];
    const uint32_t* v = u[r];
    const uint32_t o0 = x3(v[7], T[0], a[0]) ^ kw[35 + r];
    const uint32_t o1 = x3(v[0], v[7], T[1]) ^ a[1];
    const uint32_t o2 = x3(v[1], T[2], a[2]);
    const uint32_t o3 = x3(v[2], v[7], T[3]) ^ a[3];
    const uint32_t o4 = x3(v[3], v[7], T[4]) ^ a[4];
    const uint32_t o5 = x3(v[4], T[5], a[5]);
    const uint32_t o6 = x3(v[5], T[6], a[6]);
    const uint32_t o7 = x3(v[6], T[7], a[7]);
    a[0] = o0; a[1] = o1; a[2] = o2; a[3] = o3; a[4] = o4; a[5] = o5; a[6] = o6; a[7] = o7;
  }
}

// The same with compile-time key bytes KB::kb.b[R].
template <int P, class KB, int R>
BS_HD void mix_column_c(uint32_t* s, int c) {
  const int p0 = 8 * phys(P, 0, c), p1 = 8 * phys(P, 1, c), p2 = 8 * phys(P, 2, c),
            p3 = 8 * phys(P, 3, c);
  const int pr[4] = {p0, p1, p2, p3};
  uint32_t u[4][8];
BS_UNROLL
  for (int r = 0; r < 4; ++r)
BS_UNROLL
    for (int m = 0; m < 8; ++m) u[r][m] = s[pr[r] + m] ^ s[pr[(r + 1) & 3] + m];
  uint32_t T[8];
BS_UNROLL
  for (int j = 0; j < 8; ++j) T[j] = u[0][j] ^ u[2][j];
BS_UNROLL
  for (int r = 0; r < 4; ++r) {
    uint32_t* a = s + pr[r];
    const uint32_t* v = u[r];
    const uint8_t kb = KB::kb.b[R][4 * c + r];
    auto K = [&](int j) { return ((kb >> j) & 1) != 0; };
    const uint32_t o0 = x3k(v[7], T[0], a[0], K(0));
    const uint32_t o1 = x2k(x3(v[0], v[7], T[1]), a[1], K(1));
    const uint32_t o2 = x3k(v[1], T[2], a[2], K(2));
    const uint32_t o3 = x2k(x3(v[2], v[7], T[3]), a[3], K(3));
    const uint32_t o4 = x2k(x3(v[3], v[7], T[4]), a[4], K(4));
    const uint32_t o5 = x3k(v[4], T[5], a[5], K(5));
    const uint32_t o6 = x3k(v[5], T[6], a[6], K(6));
    const uint32_t o7 = x3k(v[6], T[7], a[7], K(7));
    a[0] = o0; a[1] = o1; a[2] = o2; a[3] = o3; a[4] = o4; a[5] = o5; a[6] = o6; a[7] = o7;
  }
}

// One middle round R (1..9) entered at phase PIN; leaves the state at PIN + 1.
template <int PIN, class KeySrc>
BS_HD void round_mid(uint32_t* s, const KeySrc& ks, int R) {
  sub_bytes(s);
BS_UNROLL
  for (int c = 0; c < 4; ++c) {
    ks.template mix<(PIN + 1) & 3>(s, c, R);
    FBS_FENCE();
  }
}

// Key sources.  MaskKeys reads the column's 40 words from a (LDS) table.
struct MaskKeys {
  const MaskTable* t;
  template <int P>
  BS_HD void mix(uint32_t* s, int c, int R) const {
    uint32_t kw[kColWords];
    const uint4* src = reinterpret_cast<const uint4*>(t->mid[R - 1][c]);
BS_UNROLL
    for (int q = 0; q < kColWords / 4; ++q) {
      const uint4 v = src[q];
      kw[4 * q] = v.x; kw[4 * q + 1] = v.y; kw[4 * q + 2] = v.z; kw[4 * q + 3] = v.w;
    }
    mix_column_masks<P>(s, c, kw);
  }
  BS_HD uint32_t first(int p) const { return t->first[p]; }
  BS_HD uint32_t last(int p) const { return t->last[p]; }
};

// sigma + round-0 key: ff = sigma(x) (what the MMO feed-forward XORs back in),
// s = sigma(x) ^ k0.  x and s may alias.  ff_store(p, v) receives plane p of
// sigma(x).
template <class KeySrc, class FF>
BS_HD void sigma_ark0(uint32_t* s, const KeySrc& ks, FF& ff) {
BS_UNROLL
  for (int j = 0; j < 64; ++j) {
    const uint32_t lo = s[j], hi = s[64 + j];
    const uint32_t slo = hi, shi = hi ^ lo;
    ff.put(j, slo);
    ff.put(64 + j, shi);
    s[j] = slo ^ ks.first(j);
    s[64 + j] = x3(hi, lo, ks.first(64 + j));
  }
}

// Final round at phase PIN (= 9 rounds after phase 0, i.e. 1): SubBytes,
// ShiftRows renaming, then out = s ^ k10 ^ ff, written to logical order.
template <int PIN, class KeySrc, class FF>
BS_HD void round_last(uint32_t* s, const KeySrc& ks, FF& ff, uint32_t* out) {
  sub_bytes(s);
  constexpr int P = (PIN + 1) & 3;
BS_UNROLL
  for (int c = 0; c < 4; ++c)
BS_UNROLL
    for (int r = 0; r < 4; ++r)
BS_UNROLL
      for (int i = 0; i < 8; ++i) {
        const int lp = 8 * (4 * c + r) + i;
        out[lp] = x3(s[8 * phys(P, r, c) + i], ff.get(lp), ks.last(lp));
      }
}

}  // namespace fbs
