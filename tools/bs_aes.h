// bs_aes.h -- bitsliced fixed-key AES-128 MMO hash on the VALU (gfx950), for
// the leaf value hashes of the full-domain expansion: the LDS T-table AES of
// aes_core.h is bound by the LDS pipe (5 clk per block per CU) while the VALU
// sits ~65% idle, so hashing a share of the blocks here puts both pipes to work.
//
// Semantics: H_k(x) = AES_k(sigma(x)) ^ sigma(x), sigma(x) = MakeUint128(hi ^ lo,
// hi) (dpf/aes_128_fixed_key_hash.cc:47-85), bit-exact with aes_core.h.
//
// Layout ("row groups", 8 blocks per lane): a batch is 8 blocks b = 0..7 held
// in 32 registers p[4*i + r], i = bit 0..7 of a state byte, r = AES row 0..3.
// Byte-lane c of p[4*i + r] holds, in its bit b, bit i of state byte (row r,
// column c) of block b -- i.e. of byte 4*c + r of the block's 16-byte
// little-endian memory image (aes_core.h: column word c = bytes 4c..4c+3).
//   * SubBytes: the S-box circuit on the 8 planes of a row group computes 32
//     S-boxes (4 columns x 8 blocks) at once: 4 x 82 v_bitop3 per round.
//   * ShiftRows: row r rotates right by 8r bits (v_alignbit): 24 per round.
//   * MixColumns: XORs between row groups (same byte-lane = same column), the
//     round key folded in: 96 per round.
//   * AddRoundKey: per plane a mask whose byte-lane c is 0xff where the key bit
//     is set -- uniform over the wave (scalar registers, `BsKeyMasks`).
// Per block: ~560 VALU lane-ops for the ten rounds plus 64 for the transposes
// in and out, i.e. ~4.9 clk per block per CU at 128 lane-ops/clk -- on the
// VALU, in parallel with the T-table's LDS work.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define BS_HD __host__ __device__ __forceinline__
#define BS_UNROLL _Pragma("unroll")
#else
#define BS_HD inline
#define BS_UNROLL
#endif

namespace bsa {

#if defined(__HIP_DEVICE_COMPILE__)
#define BS3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))
BS_HD uint32_t rotr(uint32_t x, uint32_t s) { return __builtin_amdgcn_alignbit(x, x, s); }
// v_perm_b32: byte k of the result = byte sel[k] of the 64-bit {hi, lo}.
BS_HD uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
#else
// Host emulation (unit checks): truth-table index = S0 * 4 + S1 * 2 + S2.
inline uint32_t bs3_host(uint32_t a, uint32_t b, uint32_t c, int imm) {
  uint32_t r = 0;
  for (int idx = 0; idx < 8; ++idx)
    if ((imm >> idx) & 1)
      r |= ((idx & 4) ? a : ~a) & ((idx & 2) ? b : ~b) & ((idx & 1) ? c : ~c);
  return r;
}
#define BS3(a, b, c, imm) ::bsa::bs3_host((a), (b), (c), (imm))
inline uint32_t rotr(uint32_t x, uint32_t s) { return s ? (x >> s) | (x << (32 - s)) : x; }
inline uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int k = 0; k < 4; ++k) {
    const uint32_t s = (sel >> (8 * k)) & 0xff;
    const uint32_t byte = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xff : 0;  // 0x0c -> 0x00
    r |= byte << (8 * k);
  }
  return r;
}
#endif

#include "bs_sbox_gen.h"

// bitop3 truth tables used below (index = S0 * 4 + S1 * 2 + S2).
constexpr int kXor3 = 0x96;    // S0 ^ S1 ^ S2
constexpr int kSelect = 0xe4;  // S2 ? S0 : S1

// ---------------------------------------------------------------------------
// Transposes between 8 blocks in normal form (w[4*b + c] = column word c of
// block b) and the planes p[4*i + r], in place on the same 32 registers.
// ---------------------------------------------------------------------------

// 4x4 byte transpose of the four column words of every block: afterwards
// w[4*b + r] has, in byte-lane c, byte r of (old) column word c.  An involution.
BS_HD void byte_transpose(uint32_t* w) {
BS_UNROLL
  for (int b = 0; b < 8; ++b) {
    uint32_t* a = w + 4 * b;
    const uint32_t t0 = perm(a[1], a[0], 0x05010400u), t1 = perm(a[1], a[0], 0x07030602u);
    const uint32_t t2 = perm(a[3], a[2], 0x05010400u), t3 = perm(a[3], a[2], 0x07030602u);
    a[0] = perm(t2, t0, 0x05040100u);
    a[1] = perm(t2, t0, 0x07060302u);
    a[2] = perm(t3, t1, 0x05040100u);
    a[3] = perm(t3, t1, 0x07060302u);
  }
}

// Per byte-lane 8x8 bit transpose of the 8 registers w[4*k + r] (k = 0..7) of
// each row r: afterwards bit q of byte-lane c of w[4*k + r] = (old) bit k of
// byte-lane c of w[4*q + r].  Recursive block swap; an involution.
template <int J>
BS_HD void bit_swap_stage(uint32_t* w, int r) {
  constexpr uint32_t m = J == 4 ? 0x0f0f0f0fu : (J == 2 ? 0x33333333u : 0x55555555u);
BS_UNROLL
  for (int q = 0; q < 4; ++q) {
    const int k = (q / J) * 2 * J + (q % J);  // the k in 0..7 with (k & J) == 0
    const uint32_t x = w[4 * k + r], y = w[4 * (k + J) + r];
    w[4 * k + r] = BS3(x, y << J, m, kSelect);
    w[4 * (k + J) + r] = BS3(x >> J, y, m, kSelect);
  }
}
BS_HD void bit_transpose(uint32_t* w) {
BS_UNROLL
  for (int r = 0; r < 4; ++r) {
    bit_swap_stage<4>(w, r);
    bit_swap_stage<2>(w, r);
    bit_swap_stage<1>(w, r);
  }
}

BS_HD void to_planes(uint32_t* w) {
  byte_transpose(w);
  bit_transpose(w);
}
BS_HD void from_planes(uint32_t* w) {
  bit_transpose(w);
  byte_transpose(w);
}

// ---------------------------------------------------------------------------
// Round keys as plane masks: mask[R][4*i + r] has byte-lane c = 0xff iff bit i
// of byte r of round-key word 4R + c is set (dpf_aes::expand_key's words).
// ---------------------------------------------------------------------------
struct BsKeyMasks {
  uint32_t m[11][32];
};

inline BsKeyMasks make_key_masks(const uint32_t rk[44]) {
  BsKeyMasks km{};
  for (int R = 0; R < 11; ++R)
    for (int i = 0; i < 8; ++i)
      for (int r = 0; r < 4; ++r) {
        uint32_t v = 0;
        for (int c = 0; c < 4; ++c)
          if ((rk[4 * R + c] >> (8 * r + i)) & 1u) v |= 0xffu << (8 * c);
        km.m[R][4 * i + r] = v;
      }
  return km;
}

// The same masks computed at compile time, for keys known when the kernel is
// built (the reference's fixed PRG keys, distributed_point_function.cc:37-42):
// with the rounds unrolled every mask is an immediate, so AddRoundKey costs a
// literal XOR (VOP2, full rate) or nothing, never an SGPR operand (half rate,
// profiles/r10_valu_issue_microbench.txt).
constexpr uint8_t kSboxC[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

// AES-128 key expansion (FIPS-197 5.2) on the little-endian column image of
// the 16 key bytes, as dpf_aes::expand_key, usable in constant expressions.
struct RoundKeyWords {
  uint32_t w[44];
};
constexpr RoundKeyWords expand_key_c(const uint8_t (&key)[16]) {
  RoundKeyWords r{};
  const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
  for (int i = 0; i < 4; ++i)
    r.w[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) |
             ((uint32_t)key[4 * i + 2] << 16) | ((uint32_t)key[4 * i + 3] << 24);
  for (int i = 4; i < 44; ++i) {
    uint32_t t = r.w[i - 1];
    if (i % 4 == 0) {
      t = (t >> 8) | (t << 24);
      t = (uint32_t)kSboxC[t & 0xff] | ((uint32_t)kSboxC[(t >> 8) & 0xff] << 8) |
          ((uint32_t)kSboxC[(t >> 16) & 0xff] << 16) | ((uint32_t)kSboxC[(t >> 24) & 0xff] << 24);
      t ^= rcon[i / 4 - 1];
    }
    r.w[i] = r.w[i - 4] ^ t;
  }
  return r;
}
constexpr BsKeyMasks make_key_masks_c(const uint8_t (&key)[16]) {
  const RoundKeyWords rk = expand_key_c(key);
  BsKeyMasks km{};
  for (int R = 0; R < 11; ++R)
    for (int i = 0; i < 8; ++i)
      for (int r = 0; r < 4; ++r) {
        uint32_t v = 0;
        for (int c = 0; c < 4; ++c)
          if ((rk.w[4 * R + c] >> (8 * r + i)) & 1u) v |= 0xffu << (8 * c);
        km.m[R][4 * i + r] = v;
      }
  return km;
}

// x ^ k for a mask k known at compile time after unrolling: nothing for 0, a
// NOT for ~0, otherwise a literal XOR.
BS_HD uint32_t xor_mask(uint32_t x, uint32_t k) {
  return k == 0 ? x : (k == 0xffffffffu ? ~x : x ^ k);
}

BS_HD void sub_bytes(uint32_t* p) {
BS_UNROLL
  for (int r = 0; r < 4; ++r)
    sbox_planes(p[28 + r], p[24 + r], p[20 + r], p[16 + r], p[12 + r], p[8 + r], p[4 + r], p[r]);
}

BS_HD void shift_rows(uint32_t* p) {
BS_UNROLL
  for (int i = 0; i < 8; ++i) {
    p[4 * i + 1] = rotr(p[4 * i + 1], 8);
    p[4 * i + 2] = rotr(p[4 * i + 2], 16);
    p[4 * i + 3] = rotr(p[4 * i + 3], 24);
  }
}

// MixColumns then AddRoundKey with masks k[32]:
//   out_r = xtime(a_r ^ a_{r+1}) ^ (a_{r+1} ^ a_{r+2}) ^ a_{r+3} ^ k_r.
BS_HD void mix_columns_ark(uint32_t* p, const uint32_t* k) {
  uint32_t d[32];  // d[4*i + r] = a_r ^ a_{r+1}
BS_UNROLL
  for (int i = 0; i < 8; ++i)
BS_UNROLL
    for (int r = 0; r < 4; ++r) d[4 * i + r] = p[4 * i + r] ^ p[4 * i + ((r + 1) & 3)];
  uint32_t o[32];
BS_UNROLL
  for (int r = 0; r < 4; ++r) {
    const int r1 = (r + 1) & 3, r3 = (r + 3) & 3;
BS_UNROLL
    for (int i = 0; i < 8; ++i) {
      const uint32_t a3 = p[4 * i + r3], d1 = d[4 * i + r1], kk = k[4 * i + r];
      if (i == 1 || i == 3 || i == 4) {
        // xtime bit i = d[i-1] ^ d[7]
        const uint32_t e = BS3(d[4 * (i - 1) + r], d[28 + r], d1, kXor3);
        o[4 * i + r] = BS3(e, a3, kk, kXor3);
      } else {
        const uint32_t x = i == 0 ? d[28 + r] : d[4 * (i - 1) + r];
        o[4 * i + r] = BS3(x, d1, a3, kXor3) ^ kk;
      }
    }
  }
BS_UNROLL
  for (int j = 0; j < 32; ++j) p[j] = o[j];
}

// MixColumns then AddRoundKey with masks known at compile time (KM::m).
template <class KM, int R>
BS_HD void mix_columns_ark_c(uint32_t* p) {
  uint32_t d[32];  // d[4*i + r] = a_r ^ a_{r+1}
BS_UNROLL
  for (int i = 0; i < 8; ++i)
BS_UNROLL
    for (int r = 0; r < 4; ++r) d[4 * i + r] = p[4 * i + r] ^ p[4 * i + ((r + 1) & 3)];
  uint32_t o[32];
BS_UNROLL
  for (int r = 0; r < 4; ++r) {
    const int r1 = (r + 1) & 3, r3 = (r + 3) & 3;
BS_UNROLL
    for (int i = 0; i < 8; ++i) {
      const uint32_t a3 = p[4 * i + r3], d1 = d[4 * i + r1];
      const uint32_t kk = KM::m.m[R][4 * i + r];
      if (i == 1 || i == 3 || i == 4) {
        // xtime bit i = d[i-1] ^ d[7]: five inputs with the key
        const uint32_t e = BS3(d[4 * (i - 1) + r], d[28 + r], d1, kXor3);
        o[4 * i + r] = kk == 0 ? (e ^ a3) : (kk == 0xffffffffu ? ~(e ^ a3) : BS3(e, a3, kk, kXor3));
      } else {
        const uint32_t x = i == 0 ? d[28 + r] : d[4 * (i - 1) + r];
        o[4 * i + r] = xor_mask(BS3(x, d1, a3, kXor3), kk);
      }
    }
  }
BS_UNROLL
  for (int j = 0; j < 32; ++j) p[j] = o[j];
}

template <class KM, int R>
BS_HD void round_c(uint32_t* w) {
  sub_bytes(w);
  shift_rows(w);
  if constexpr (R < 10) {
    mix_columns_ark_c<KM, R>(w);
  } else {
BS_UNROLL
    for (int j = 0; j < 32; ++j) w[j] = xor_mask(w[j], KM::m.m[10][j]);
  }
}
template <class KM, int R>
BS_HD void rounds_c(uint32_t* w) {
  round_c<KM, R>(w);
  if constexpr (R < 10) rounds_c<KM, R + 1>(w);
}

// AES-128 encryption (no MMO feed-forward) of 8 blocks in normal form, in
// place, under the compile-time key KM (KM::m = make_key_masks_c(key)).  All
// ten rounds unrolled: ~470 VALU per round for the 8 blocks of a lane.
template <class KM>
BS_HD void aes8_c(uint32_t* w) {
  to_planes(w);
BS_UNROLL
  for (int j = 0; j < 32; ++j) w[j] = xor_mask(w[j], KM::m.m[0][j]);
  rounds_c<KM, 1>(w);
  from_planes(w);
}

// Key-mask provider: km(R, j) = mask of round R, plane j.
struct ArrayMasks {
  const uint32_t (*m)[32];
  BS_HD uint32_t operator()(int R, int j) const { return m[R][j]; }
};

// H_k on 8 blocks, in place on w[32] (normal form in and out).
template <class KM>
BS_HD void mmo8(uint32_t* w, const KM& km) {
  // sigma in normal form: (w0, w1, w2, w3) -> (w2, w3, w2 ^ w0, w3 ^ w1).
BS_UNROLL
  for (int b = 0; b < 8; ++b) {
    uint32_t* a = w + 4 * b;
    const uint32_t w0 = a[0], w1 = a[1];
    a[0] = a[2];
    a[1] = a[3];
    a[2] = a[2] ^ w0;
    a[3] = a[3] ^ w1;
  }
  to_planes(w);
  uint32_t sp[32];
BS_UNROLL
  for (int j = 0; j < 32; ++j) {
    sp[j] = w[j];
    w[j] ^= km(0, j);
  }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int R = 1; R < 10; ++R) {
    uint32_t k[32];
BS_UNROLL
    for (int j = 0; j < 32; ++j) {
      k[j] = km(R, j);
#if defined(__HIP_DEVICE_COMPILE__) && defined(BS_KEY_VGPR)
      asm volatile("v_mov_b32 %0, %1" : "=v"(k[j]) : "s"(k[j]));
#endif
    }
    sub_bytes(w);
    shift_rows(w);
    mix_columns_ark(w, k);
  }
  sub_bytes(w);
  shift_rows(w);
BS_UNROLL
  for (int j = 0; j < 32; ++j) w[j] = BS3(w[j], km(10, j), sp[j], kXor3);
  from_planes(w);
}

}  // namespace bsa
