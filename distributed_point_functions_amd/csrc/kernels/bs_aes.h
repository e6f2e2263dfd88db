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
