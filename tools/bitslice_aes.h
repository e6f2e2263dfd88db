// bitslice_aes.h -- bitsliced AES-128 (32 blocks per 32-bit lane word) for the
// VALU-side measurement of DESIGN.md section 8 (tools/bitslice_microbench.hip).
//
// Layout: 128 planes per group of 32 blocks; plane 32*c + k holds bit k of
// column word c (the little-endian 32-bit column of dpf_aes::Block4) of every
// block, block b in bit b.  Equivalently plane 8*j + i is bit i of state byte
// j = 4*c + r (row r, column c).  In this layout ShiftRows is a renaming of
// planes, AddRoundKey is a XOR with 0 or ~0 per plane, the control bit of a
// DPF seed is plane 0 and clearing it zeroes that plane.
//
// S-box: the Boyar-Peralta 113-gate circuit (32 AND, 77 XOR, 4 XNOR; "A depth-16
// circuit for the AES S-box", 2011), checked against FIPS-197 for all 256
// inputs by `bitslice_microbench --cpu-check`.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define BS_HD __host__ __device__ __forceinline__
#define BS_UNROLL _Pragma("unroll")
#else
#define BS_HD inline
#define BS_UNROLL
#endif

namespace bs {

// x[0] = least significant bit plane of the byte, x[7] = most significant.
BS_HD void sbox(uint32_t* x) {
  const uint32_t U0 = x[7], U1 = x[6], U2 = x[5], U3 = x[4], U4 = x[3], U5 = x[2], U6 = x[1],
                 U7 = x[0];
  // Top linear layer.
  const uint32_t T1 = U0 ^ U3, T2 = U0 ^ U5, T3 = U0 ^ U6, T4 = U3 ^ U5, T5 = U4 ^ U6;
  const uint32_t T6 = T1 ^ T5, T7 = U1 ^ U2, T8 = U7 ^ T6, T9 = U7 ^ T7, T10 = T6 ^ T7;
  const uint32_t T11 = U1 ^ U5, T12 = U2 ^ U5, T13 = T3 ^ T4, T14 = T6 ^ T11, T15 = T5 ^ T11;
  const uint32_t T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = U3 ^ U7, T19 = T7 ^ T18, T20 = T1 ^ T19;
  const uint32_t T21 = U6 ^ U7, T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10, T25 = T20 ^ T17;
  const uint32_t T26 = T3 ^ T16, T27 = T1 ^ T12;
  // Shared non-linear middle (GF(2^4) inversion).
  const uint32_t M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7, M5 = M4 ^ M1;
  const uint32_t M6 = T3 & T16, M7 = T22 & T9, M8 = T26 ^ M6, M9 = T20 & T17, M10 = M9 ^ M6;
  const uint32_t M11 = T1 & T15, M12 = T4 & T27, M13 = M12 ^ M11, M14 = T2 & T10,
                 M15 = M14 ^ M11;
  const uint32_t M16 = M3 ^ M2, M17 = M5 ^ T24, M18 = M8 ^ M7, M19 = M10 ^ M15, M20 = M16 ^ M13;
  const uint32_t M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25, M24 = M22 ^ M23;
  const uint32_t M25 = M22 & M20, M26 = M21 ^ M25, M27 = M20 ^ M21, M28 = M23 ^ M25;
  const uint32_t M29 = M28 & M27, M30 = M26 & M24, M31 = M20 & M23, M32 = M27 & M31;
  const uint32_t M33 = M27 ^ M25, M34 = M21 & M22, M35 = M24 & M34, M36 = M24 ^ M25;
  const uint32_t M37 = M21 ^ M29, M38 = M32 ^ M33, M39 = M23 ^ M30, M40 = M35 ^ M36;
  const uint32_t M41 = M38 ^ M40, M42 = M37 ^ M39, M43 = M37 ^ M38, M44 = M39 ^ M40,
                 M45 = M42 ^ M41;
  const uint32_t M46 = M44 & T6, M47 = M40 & T8, M48 = M39 & U7, M49 = M43 & T16, M50 = M38 & T9;
  const uint32_t M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27, M54 = M41 & T10,
                 M55 = M44 & T13;
  const uint32_t M56 = M40 & T23, M57 = M39 & T19, M58 = M43 & T3, M59 = M38 & T22,
                 M60 = M37 & T20;
  const uint32_t M61 = M42 & T1, M62 = M45 & T4, M63 = M41 & T2;
  // Bottom linear layer.
  const uint32_t L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48, L3 = M47 ^ M55, L4 = M54 ^ M58;
  const uint32_t L5 = M49 ^ M61, L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59, L9 = M52 ^ M53;
  const uint32_t L10 = M53 ^ L4, L11 = M60 ^ L2, L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61;
  const uint32_t L15 = M55 ^ L1, L16 = M56 ^ L0, L17 = M57 ^ L1, L18 = M58 ^ L8, L19 = M63 ^ L4;
  const uint32_t L20 = L0 ^ L1, L21 = L1 ^ L7, L22 = L3 ^ L12, L23 = L18 ^ L2, L24 = L15 ^ L9;
  const uint32_t L25 = L6 ^ L10, L26 = L7 ^ L9, L27 = L8 ^ L10, L28 = L11 ^ L14, L29 = L11 ^ L17;
  x[7] = L6 ^ L24;
  x[6] = ~(L16 ^ L26);
  x[5] = ~(L19 ^ L28);
  x[4] = L6 ^ L21;
  x[3] = L20 ^ L22;
  x[2] = L25 ^ L29;
  x[1] = ~(L13 ^ L27);
  x[0] = ~(L6 ^ L23);
}

// 32x32 bit-matrix transpose in place: afterwards a[k] bit b = (old a[b]) bit k.
BS_HD void transpose32(uint32_t* a) {
  uint32_t m = 0x0000FFFFu;
BS_UNROLL
  for (int j = 16; j != 0; j >>= 1, m ^= m << j) {
BS_UNROLL
    for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
      const uint32_t t = ((a[k] >> j) ^ a[k + j]) & m;
      a[k + j] ^= t;
      a[k] ^= t << j;
    }
  }
}

// Blocks (4 column words each, blk[4*b + c]) of 32 blocks -> 128 planes, and back.
BS_HD void to_planes(const uint32_t* blk, uint32_t* s) {
BS_UNROLL
  for (int c = 0; c < 4; ++c) {
BS_UNROLL
    for (int b = 0; b < 32; ++b) s[32 * c + b] = blk[4 * b + c];
    transpose32(s + 32 * c);
  }
}
BS_HD void from_planes(uint32_t* s, uint32_t* blk) {
BS_UNROLL
  for (int c = 0; c < 4; ++c) {
    transpose32(s + 32 * c);
BS_UNROLL
    for (int b = 0; b < 32; ++b) blk[4 * b + c] = s[32 * c + b];
  }
}

BS_HD void add_round_key(uint32_t* s, const uint32_t* rk4) {
BS_UNROLL
  for (int c = 0; c < 4; ++c)
BS_UNROLL
    for (int k = 0; k < 32; ++k) s[32 * c + k] ^= 0u - ((rk4[c] >> k) & 1u);
}

// Scheduling fence between S-boxes and MixColumns columns: left alone the
// scheduler interleaves all 16 S-boxes, keeps ~30 temporaries of each live,
// spills to AGPRs and rematerialises gates (2x the VALU of the circuit).
#if defined(__HIP_DEVICE_COMPILE__) && defined(BS_FENCE)
#define BS_FENCE_POINT() __builtin_amdgcn_sched_barrier(0)
#else
#define BS_FENCE_POINT() ((void)0)
#endif

BS_HD void sub_bytes(uint32_t* s) {
BS_UNROLL
  for (int j = 0; j < 16; ++j) {
    sbox(s + 8 * j);
#if defined(__HIP_DEVICE_COMPILE__) && defined(BS_OPAQUE)
    // Opaque S-box outputs: stop IR reassociation from merging the S-box's
    // last XORs with MixColumns' XOR trees across all 16 bytes.
BS_UNROLL
    for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(s[8 * j + i]));
#endif
    BS_FENCE_POINT();
  }
}

// Byte j = 4c + r of the ShiftRows output is byte 4((c + r) & 3) + r of its input.
BS_HD int shift_src(int j) { return 4 * (((j >> 2) + (j & 3)) & 3) + (j & 3); }

// xtime on the 8 planes of one byte: out = 2a in GF(2^8) mod 0x11b.
BS_HD void xtime8(const uint32_t* a, uint32_t* o) {
  o[0] = a[7];
  o[1] = a[0] ^ a[7];
  o[2] = a[1];
  o[3] = a[2] ^ a[7];
  o[4] = a[3] ^ a[7];
  o[5] = a[4];
  o[6] = a[5];
  o[7] = a[6];
}

// ShiftRows + MixColumns from s into t.
BS_HD void shift_mix(const uint32_t* s, uint32_t* t) {
BS_UNROLL
  for (int c = 0; c < 4; ++c) {
    const uint32_t* a0 = s + 8 * shift_src(4 * c + 0);
    const uint32_t* a1 = s + 8 * shift_src(4 * c + 1);
    const uint32_t* a2 = s + 8 * shift_src(4 * c + 2);
    const uint32_t* a3 = s + 8 * shift_src(4 * c + 3);
    uint32_t d01[8], d12[8], d23[8], d30[8];
    uint32_t x01[8], x12[8], x23[8], x30[8];
BS_UNROLL
    for (int i = 0; i < 8; ++i) {
      x01[i] = a0[i] ^ a1[i];
      x12[i] = a1[i] ^ a2[i];
      x23[i] = a2[i] ^ a3[i];
      x30[i] = a3[i] ^ a0[i];
    }
    xtime8(x01, d01);
    xtime8(x12, d12);
    xtime8(x23, d23);
    xtime8(x30, d30);
    // o_r = 2a_r ^ 3a_{r+1} ^ a_{r+2} ^ a_{r+3} = 2(a_r ^ a_{r+1}) ^ a_{r+1} ^ (a_{r+2} ^ a_{r+3}).
    uint32_t* o0 = t + 8 * (4 * c + 0);
    uint32_t* o1 = t + 8 * (4 * c + 1);
    uint32_t* o2 = t + 8 * (4 * c + 2);
    uint32_t* o3 = t + 8 * (4 * c + 3);
BS_UNROLL
    for (int i = 0; i < 8; ++i) {
      o0[i] = d01[i] ^ a1[i] ^ x23[i];
      o1[i] = d12[i] ^ a2[i] ^ x30[i];
      o2[i] = d23[i] ^ a3[i] ^ x01[i];
      o3[i] = d30[i] ^ a0[i] ^ x12[i];
    }
  }
}

BS_HD void shift_rows(const uint32_t* s, uint32_t* t) {
BS_UNROLL
  for (int j = 0; j < 16; ++j)
BS_UNROLL
    for (int i = 0; i < 8; ++i) t[8 * j + i] = s[8 * shift_src(j) + i];
}

// AES-128 encryption of the 32 blocks held in s (planes), round keys as the 44
// little-endian column words of dpf_aes::expand_key.
BS_HD void encrypt(uint32_t* s, const uint32_t* rk) {
  uint32_t t[128];
  add_round_key(s, rk);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int r = 1; r < 10; ++r) {
    sub_bytes(s);
    shift_mix(s, t);
    add_round_key(t, rk + 4 * r);
BS_UNROLL
    for (int i = 0; i < 128; ++i) s[i] = t[i];
  }
  sub_bytes(s);
  shift_rows(s, t);
  add_round_key(t, rk + 40);
BS_UNROLL
  for (int i = 0; i < 128; ++i) s[i] = t[i];
}

}  // namespace bs

namespace bs {

// In-place variant: ShiftRows is never executed.  After R rounds logical byte
// (row r, column c) lives in physical byte slot 4*((c + R*r) & 3) + r, so each
// MixColumns writes its outputs over its own inputs (every physical byte feeds
// exactly one output column) and only 128 state planes are live.
template <int R>
BS_HD constexpr int phys(int r, int c) { return 4 * ((c + R * r) & 3) + r; }

template <int R>
BS_HD void ark_phys(uint32_t* s, const uint32_t* rk4) {
BS_UNROLL
  for (int c = 0; c < 4; ++c)
BS_UNROLL
    for (int r = 0; r < 4; ++r)
BS_UNROLL
      for (int i = 0; i < 8; ++i) s[8 * phys<R>(r, c) + i] ^= 0u - ((rk4[c] >> (8 * r + i)) & 1u);
}

template <int R>
BS_HD void mix_inplace(uint32_t* s) {
BS_UNROLL
  for (int c = 0; c < 4; ++c) {
    uint32_t* a0 = s + 8 * phys<R>(0, c);
    uint32_t* a1 = s + 8 * phys<R>(1, c);
    uint32_t* a2 = s + 8 * phys<R>(2, c);
    uint32_t* a3 = s + 8 * phys<R>(3, c);
    uint32_t x01[8], x12[8], x23[8], x30[8], d01[8], d12[8], d23[8], d30[8];
BS_UNROLL
    for (int i = 0; i < 8; ++i) {
      x01[i] = a0[i] ^ a1[i];
      x12[i] = a1[i] ^ a2[i];
      x23[i] = a2[i] ^ a3[i];
      x30[i] = a3[i] ^ a0[i];
    }
    xtime8(x01, d01);
    xtime8(x12, d12);
    xtime8(x23, d23);
    xtime8(x30, d30);
BS_UNROLL
    for (int i = 0; i < 8; ++i) {
      const uint32_t b0 = a0[i], b1 = a1[i], b2 = a2[i], b3 = a3[i];
      a0[i] = d01[i] ^ b1 ^ x23[i];
      a1[i] = d12[i] ^ b2 ^ x30[i];
      a2[i] = d23[i] ^ b3 ^ x01[i];
      a3[i] = d30[i] ^ b0 ^ x12[i];
    }
    BS_FENCE_POINT();
  }
}

template <int R>
BS_HD void rounds_inplace(uint32_t* s, const uint32_t* rk) {
  if constexpr (R <= 9) {
    sub_bytes(s);
    mix_inplace<R>(s);
    ark_phys<R>(s, rk + 4 * R);
    rounds_inplace<R + 1>(s, rk);
  } else {
    sub_bytes(s);
    ark_phys<10>(s, rk + 40);
    // Back to logical order (a renaming once unrolled).
    uint32_t t[128];
BS_UNROLL
    for (int c = 0; c < 4; ++c)
BS_UNROLL
      for (int r = 0; r < 4; ++r)
BS_UNROLL
        for (int i = 0; i < 8; ++i) t[8 * (4 * c + r) + i] = s[8 * phys<10>(r, c) + i];
BS_UNROLL
    for (int i = 0; i < 128; ++i) s[i] = t[i];
  }
}

BS_HD void encrypt_inplace(uint32_t* s, const uint32_t* rk) {
  add_round_key(s, rk);
  rounds_inplace<1>(s, rk);
}

}  // namespace bs

namespace bs {

// Two rounds per loop iteration: after rounds R=1,2 from the identity layout
// rows 1 and 3 sit rotated by two columns (row 2 is back in place), so 64
// plane moves restore the identity and the loop body stays small enough for
// the instruction cache (the fully unrolled encrypt_inplace does not).
BS_HD void restore_after2(uint32_t* s) {
BS_UNROLL
  for (int r = 1; r < 4; r += 2)
BS_UNROLL
    for (int c = 0; c < 2; ++c)
BS_UNROLL
      for (int i = 0; i < 8; ++i) {
        const uint32_t a = s[8 * (4 * c + r) + i];
        s[8 * (4 * c + r) + i] = s[8 * (4 * (c + 2) + r) + i];
        s[8 * (4 * (c + 2) + r) + i] = a;
      }
}

BS_HD void encrypt_loop2(uint32_t* s, const uint32_t* rk) {
  add_round_key(s, rk);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int it = 0; it < 4; ++it) {
    const uint32_t* k = rk + 8 * it;
    sub_bytes(s);
    mix_inplace<1>(s);
    ark_phys<1>(s, k + 4);
    sub_bytes(s);
    mix_inplace<2>(s);
    ark_phys<2>(s, k + 8);
    restore_after2(s);
  }
  // Round 9 from the identity layout, then the last round.
  sub_bytes(s);
  mix_inplace<1>(s);
  ark_phys<1>(s, rk + 36);
  sub_bytes(s);
  ark_phys<2>(s, rk + 40);
  uint32_t t[128];
BS_UNROLL
  for (int c = 0; c < 4; ++c)
BS_UNROLL
    for (int r = 0; r < 4; ++r)
BS_UNROLL
      for (int i = 0; i < 8; ++i) t[8 * (4 * c + r) + i] = s[8 * phys<2>(r, c) + i];
BS_UNROLL
  for (int i = 0; i < 128; ++i) s[i] = t[i];
}

}  // namespace bs

namespace bs {

// One round per loop iteration: smallest loop body (~2.7 K instructions),
// paying 96 plane moves per round to undo the row rotation of mix_inplace<1>.
BS_HD void restore_after1(uint32_t* s) {
  uint32_t t[96];
BS_UNROLL
  for (int r = 1; r < 4; ++r)
BS_UNROLL
    for (int c = 0; c < 4; ++c)
BS_UNROLL
      for (int i = 0; i < 8; ++i) t[32 * (r - 1) + 8 * c + i] = s[8 * phys<1>(r, c) + i];
BS_UNROLL
  for (int r = 1; r < 4; ++r)
BS_UNROLL
    for (int c = 0; c < 4; ++c)
BS_UNROLL
      for (int i = 0; i < 8; ++i) s[8 * (4 * c + r) + i] = t[32 * (r - 1) + 8 * c + i];
}

BS_HD void encrypt_loop1(uint32_t* s, const uint32_t* rk) {
  add_round_key(s, rk);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int r = 1; r < 10; ++r) {
    sub_bytes(s);
    mix_inplace<1>(s);
    ark_phys<1>(s, rk + 4 * r);
    restore_after1(s);
  }
  sub_bytes(s);
  ark_phys<1>(s, rk + 40);
  restore_after1(s);
}

}  // namespace bs

namespace bs {

// Lower-pressure round for 2 waves/SIMD: key masks from a VGPR key word
// (v_bfe_i32 per plane, consumed at once) and the row moves as in-place
// cycles with one temporary each.
BS_HD uint32_t key_mask(uint32_t kw, int bit) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_sbfe((int)kw, bit, 1);
#else
  return 0u - ((kw >> bit) & 1u);
#endif
}

template <int R>
BS_HD void ark_phys_v(uint32_t* s, const uint32_t* rk4) {
BS_UNROLL
  for (int c = 0; c < 4; ++c) {
#if defined(__HIP_DEVICE_COMPILE__)
    // Keep the word in a VGPR so the masks are VALU ops, not 32 live SGPRs.
    uint32_t kw = rk4[c];
    asm volatile("v_mov_b32 %0, %1" : "=v"(kw) : "s"(kw));
#else
    const uint32_t kw = rk4[c];
#endif
BS_UNROLL
    for (int r = 0; r < 4; ++r)
BS_UNROLL
      for (int i = 0; i < 8; ++i) s[8 * phys<R>(r, c) + i] ^= key_mask(kw, 8 * r + i);
  }
}

BS_HD void restore_after1_cycles(uint32_t* s) {
BS_UNROLL
  for (int i = 0; i < 8; ++i) {
    // Row 1: logical (1,c) sits at physical column c+1: rotate left by one.
    uint32_t t = s[8 * (4 * 0 + 1) + i];
    s[8 * (4 * 0 + 1) + i] = s[8 * (4 * 1 + 1) + i];
    s[8 * (4 * 1 + 1) + i] = s[8 * (4 * 2 + 1) + i];
    s[8 * (4 * 2 + 1) + i] = s[8 * (4 * 3 + 1) + i];
    s[8 * (4 * 3 + 1) + i] = t;
    // Row 2: two swaps.
    t = s[8 * (4 * 0 + 2) + i];
    s[8 * (4 * 0 + 2) + i] = s[8 * (4 * 2 + 2) + i];
    s[8 * (4 * 2 + 2) + i] = t;
    t = s[8 * (4 * 1 + 2) + i];
    s[8 * (4 * 1 + 2) + i] = s[8 * (4 * 3 + 2) + i];
    s[8 * (4 * 3 + 2) + i] = t;
    // Row 3: logical (3,c) at physical column c+3: rotate right by one.
    t = s[8 * (4 * 3 + 3) + i];
    s[8 * (4 * 3 + 3) + i] = s[8 * (4 * 2 + 3) + i];
    s[8 * (4 * 2 + 3) + i] = s[8 * (4 * 1 + 3) + i];
    s[8 * (4 * 1 + 3) + i] = s[8 * (4 * 0 + 3) + i];
    s[8 * (4 * 0 + 3) + i] = t;
  }
}

BS_HD void encrypt_lowreg(uint32_t* s, const uint32_t* rk) {
  add_round_key(s, rk);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int r = 1; r < 10; ++r) {
    sub_bytes(s);
    mix_inplace<1>(s);
    ark_phys_v<1>(s, rk + 4 * r);
    restore_after1_cycles(s);
  }
  sub_bytes(s);
  ark_phys_v<1>(s, rk + 40);
  restore_after1_cycles(s);
}

}  // namespace bs
