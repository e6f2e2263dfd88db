// aes_core.h -- fixed-key AES-128 MMO hash, written once for gfx950 kernels
// (tables in bank-replicated LDS) and for host-side unit checks (plain arrays).
//
// Semantics restated from the reference:
//   H_k(x) = AES_k(sigma(x)) ^ sigma(x),  sigma(x) = MakeUint128(hi ^ lo, hi)
//   (dpf/aes_128_fixed_key_hash.cc:47-85, aes_128_fixed_key_hash.h:27-38).
// A 128-bit block is the absl::uint128 memory image: 16 bytes, little-endian
// {low64, high64}; as four little-endian 32-bit AES columns w0..w3 that is
//   w0 = low[31:0], w1 = low[63:32], w2 = high[31:0], w3 = high[63:32].
// Keys are the memory image of the uint128 key (aes_128_fixed_key_hash.cc:38-40).
//
// Round function: the classic 4-table formulation on little-endian columns,
//   out_c = T0[b0(w_c)] ^ T1[b1(w_c+1)] ^ T2[b2(w_c+2)] ^ T3[b3(w_c+3)] ^ rk_c,
// with T0[x] = {2S, S, S, 3S} (byte 0 = row 0) and Tk = rotl(T0, 8k).  The last
// round takes S[x] out of the tables: byte r of T_{(r+2)&3}[x] equals S[x].
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define DPF_HD __host__ __device__ __forceinline__
#else
#define DPF_HD inline
#endif

// Rounds 1-9 stay a loop by default (code size); -DDPF_AES_UNROLL_ROUNDS
// unrolls them for scheduling experiments (tools/variant_bench.py).
#if defined(__HIPCC__)
#define DPF_UNROLL _Pragma("unroll")
#else
#define DPF_UNROLL
#endif
// Last-round scheduling fence every DPF_LAST_ROUND_FENCE chains (encryptN).
#ifndef DPF_LAST_ROUND_FENCE
#define DPF_LAST_ROUND_FENCE 2
#endif
#if defined(DPF_AES_UNROLL_ROUNDS)
#define DPF_ROUND_LOOP _Pragma("unroll")
#else
#define DPF_ROUND_LOOP _Pragma("unroll 1")
#endif
// Rounds 1..DPF_L1_ROUNDS read their T-table entries through the vector L1
// (lk.l1: one 1 KiB T0 table in global memory, rotated per table) instead of
// LDS, so the two lookup engines work side by side (an
// A/B variant, 0 = every round from LDS).
#ifndef DPF_L1_ROUNDS
#define DPF_L1_ROUNDS 0
#endif
#ifndef DPF_L1_AB
#define DPF_L1_AB 1   // 0: the ILP-N chains (encryptAB) keep every round in LDS
#endif
#if defined(__HIP_DEVICE_COMPILE__) && DPF_L1_ROUNDS > 0
#define DPF_L1_FIRST (1 + DPF_L1_ROUNDS)
#else
#define DPF_L1_FIRST 1
#endif

namespace dpf_aes {

// FIPS-197 S-box.
constexpr uint8_t kSbox[256] = {
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

DPF_HD uint32_t xtime(uint32_t x) { return ((x << 1) ^ ((x & 0x80) ? 0x1b : 0)) & 0xff; }

// T0[x] = {2S, S, S, 3S} packed little-endian.
DPF_HD uint32_t t0_entry(int x) {
  uint32_t s = kSbox[x], s2 = xtime(s), s3 = s2 ^ s;
  return s2 | (s << 8) | (s << 16) | (s3 << 24);
}
DPF_HD uint32_t rotl32(uint32_t x, int r) { return r == 0 ? x : (x << r) | (x >> (32 - r)); }

// AES-128 key expansion into 44 little-endian column words.
inline void expand_key(const uint8_t key[16], uint32_t rk[44]) {
  static const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
  for (int i = 0; i < 4; ++i)
    rk[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) |
            ((uint32_t)key[4 * i + 2] << 16) | ((uint32_t)key[4 * i + 3] << 24);
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      // RotWord then SubWord then Rcon, on the little-endian column image.
      t = (t >> 8) | (t << 24);
      t = (uint32_t)kSbox[t & 0xff] | ((uint32_t)kSbox[(t >> 8) & 0xff] << 8) |
          ((uint32_t)kSbox[(t >> 16) & 0xff] << 16) | ((uint32_t)kSbox[(t >> 24) & 0xff] << 24);
      t ^= rcon[i / 4 - 1];
    }
    rk[i] = rk[i - 4] ^ t;
  }
}

struct Block4 {
  uint32_t w0, w1, w2, w3;
};

// sigma(x) = MakeUint128(hi ^ lo, hi): new low = hi, new high = hi ^ lo.
DPF_HD Block4 sigma(Block4 x) { return Block4{x.w2, x.w3, x.w2 ^ x.w0, x.w3 ^ x.w1}; }

// Generic AES-128 encryption.  `LK` provides lookup<T, K>(w) = T_T[byte K of w]
// and xor3(a, b, c).  `RK` provides rk(i) for round-key word i (0..43) and
// rk.mix(lk, a, b, i) = a ^ b ^ rk(i) (the round's last XOR, where a key
// choice can be folded in: SelectRK in dpf_device.h).
template <class LK, class RK>
DPF_HD Block4 encrypt(Block4 s, const LK& lk, const RK& rk) {
  uint32_t w0 = s.w0 ^ rk(0), w1 = s.w1 ^ rk(1), w2 = s.w2 ^ rk(2), w3 = s.w3 ^ rk(3);
#if DPF_L1_FIRST > 1
  DPF_UNROLL
  for (int r = 1; r < DPF_L1_FIRST; ++r) {
    uint32_t n0 = lk.xor3(lk.template l1<0, 0>(w0), lk.template l1<1, 1>(w1), lk.template l1<2, 2>(w2));
    uint32_t n1 = lk.xor3(lk.template l1<0, 0>(w1), lk.template l1<1, 1>(w2), lk.template l1<2, 2>(w3));
    uint32_t n2 = lk.xor3(lk.template l1<0, 0>(w2), lk.template l1<1, 1>(w3), lk.template l1<2, 2>(w0));
    uint32_t n3 = lk.xor3(lk.template l1<0, 0>(w3), lk.template l1<1, 1>(w0), lk.template l1<2, 2>(w1));
    n0 = rk.mix(lk, n0, lk.template l1<3, 3>(w3), 4 * r + 0);
    n1 = rk.mix(lk, n1, lk.template l1<3, 3>(w0), 4 * r + 1);
    n2 = rk.mix(lk, n2, lk.template l1<3, 3>(w1), 4 * r + 2);
    n3 = rk.mix(lk, n3, lk.template l1<3, 3>(w2), 4 * r + 3);
    w0 = n0; w1 = n1; w2 = n2; w3 = n3;
  }
  __builtin_amdgcn_sched_barrier(0);  // hipcc's iterative-ilp RA crashes without it
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  DPF_ROUND_LOOP
#endif
  for (int r = DPF_L1_FIRST; r < 10; ++r) {
    uint32_t n0 = lk.xor3(lk.template lookup<0, 0>(w0), lk.template lookup<1, 1>(w1),
                          lk.template lookup<2, 2>(w2));
    uint32_t n1 = lk.xor3(lk.template lookup<0, 0>(w1), lk.template lookup<1, 1>(w2),
                          lk.template lookup<2, 2>(w3));
    uint32_t n2 = lk.xor3(lk.template lookup<0, 0>(w2), lk.template lookup<1, 1>(w3),
                          lk.template lookup<2, 2>(w0));
    uint32_t n3 = lk.xor3(lk.template lookup<0, 0>(w3), lk.template lookup<1, 1>(w0),
                          lk.template lookup<2, 2>(w1));
    n0 = rk.mix(lk, n0, lk.template lookup<3, 3>(w3), 4 * r + 0);
    n1 = rk.mix(lk, n1, lk.template lookup<3, 3>(w0), 4 * r + 1);
    n2 = rk.mix(lk, n2, lk.template lookup<3, 3>(w1), 4 * r + 2);
    n3 = rk.mix(lk, n3, lk.template lookup<3, 3>(w2), 4 * r + 3);
    w0 = n0; w1 = n1; w2 = n2; w3 = n3;
  }
  // Last round: S-box bytes pulled out of T2/T3/T0/T1 for rows 0/1/2/3.
  auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    uint32_t x = lk.template lookup<2, 0>(a), y = lk.template lookup<3, 1>(b);
    uint32_t z = lk.template lookup<0, 2>(c), u = lk.template lookup<1, 3>(d);
    uint32_t xy = (x & 0x000000ffu) | (y & 0xffffff00u);
    uint32_t zu = (z & 0x00ff0000u) | (u & 0xff00ffffu);
    return ((xy & 0x0000ffffu) | (zu & 0xffff0000u)) ^ k;
  };
  Block4 o;
  o.w0 = last(w0, w1, w2, w3, rk(40));
  o.w1 = last(w1, w2, w3, w0, rk(41));
  o.w2 = last(w2, w3, w0, w1, rk(42));
  o.w3 = last(w3, w0, w1, w2, rk(43));
  return o;
}

// MMO hash: AES_k(sigma(x)) ^ sigma(x).
template <class LK, class RK>
DPF_HD Block4 mmo_hash(Block4 x, const LK& lk, const RK& rk) {
  Block4 s = sigma(x);
  Block4 e = encrypt(s, lk, rk);
  return Block4{e.w0 ^ s.w0, e.w1 ^ s.w1, e.w2 ^ s.w2, e.w3 ^ s.w3};
}


// Two independent encryptions interleaved round by round (instruction-level
// parallelism: one chain's LDS latency hides under the other's VALU work).
template <class LK, class RKA, class RKB>
DPF_HD void encrypt2(Block4& sa, Block4& sb, const LK& lk, const RKA& ra, const RKB& rb) {
  uint32_t a0 = sa.w0 ^ ra(0), a1 = sa.w1 ^ ra(1), a2 = sa.w2 ^ ra(2), a3 = sa.w3 ^ ra(3);
  uint32_t b0 = sb.w0 ^ rb(0), b1 = sb.w1 ^ rb(1), b2 = sb.w2 ^ rb(2), b3 = sb.w3 ^ rb(3);
#if DPF_L1_FIRST > 1
  DPF_UNROLL
  for (int r = 1; r < DPF_L1_FIRST; ++r) {
    uint32_t n0 = lk.xor3(lk.template l1<0, 0>(a0), lk.template l1<1, 1>(a1), lk.template l1<2, 2>(a2));
    uint32_t n1 = lk.xor3(lk.template l1<0, 0>(a1), lk.template l1<1, 1>(a2), lk.template l1<2, 2>(a3));
    uint32_t n2 = lk.xor3(lk.template l1<0, 0>(a2), lk.template l1<1, 1>(a3), lk.template l1<2, 2>(a0));
    uint32_t n3 = lk.xor3(lk.template l1<0, 0>(a3), lk.template l1<1, 1>(a0), lk.template l1<2, 2>(a1));
    uint32_t m0 = lk.xor3(lk.template l1<0, 0>(b0), lk.template l1<1, 1>(b1), lk.template l1<2, 2>(b2));
    uint32_t m1 = lk.xor3(lk.template l1<0, 0>(b1), lk.template l1<1, 1>(b2), lk.template l1<2, 2>(b3));
    uint32_t m2 = lk.xor3(lk.template l1<0, 0>(b2), lk.template l1<1, 1>(b3), lk.template l1<2, 2>(b0));
    uint32_t m3 = lk.xor3(lk.template l1<0, 0>(b3), lk.template l1<1, 1>(b0), lk.template l1<2, 2>(b1));
    n0 = ra.mix(lk, n0, lk.template l1<3, 3>(a3), 4 * r + 0);
    n1 = ra.mix(lk, n1, lk.template l1<3, 3>(a0), 4 * r + 1);
    n2 = ra.mix(lk, n2, lk.template l1<3, 3>(a1), 4 * r + 2);
    n3 = ra.mix(lk, n3, lk.template l1<3, 3>(a2), 4 * r + 3);
    m0 = rb.mix(lk, m0, lk.template l1<3, 3>(b3), 4 * r + 0);
    m1 = rb.mix(lk, m1, lk.template l1<3, 3>(b0), 4 * r + 1);
    m2 = rb.mix(lk, m2, lk.template l1<3, 3>(b1), 4 * r + 2);
    m3 = rb.mix(lk, m3, lk.template l1<3, 3>(b2), 4 * r + 3);
    a0 = n0; a1 = n1; a2 = n2; a3 = n3;
    b0 = m0; b1 = m1; b2 = m2; b3 = m3;
  }
  __builtin_amdgcn_sched_barrier(0);  // hipcc's iterative-ilp RA crashes without it
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  DPF_ROUND_LOOP
#endif
  for (int r = DPF_L1_FIRST; r < 10; ++r) {
    uint32_t n0 = lk.xor3(lk.template lookup<0, 0>(a0), lk.template lookup<1, 1>(a1),
                          lk.template lookup<2, 2>(a2));
    uint32_t n1 = lk.xor3(lk.template lookup<0, 0>(a1), lk.template lookup<1, 1>(a2),
                          lk.template lookup<2, 2>(a3));
    uint32_t n2 = lk.xor3(lk.template lookup<0, 0>(a2), lk.template lookup<1, 1>(a3),
                          lk.template lookup<2, 2>(a0));
    uint32_t n3 = lk.xor3(lk.template lookup<0, 0>(a3), lk.template lookup<1, 1>(a0),
                          lk.template lookup<2, 2>(a1));
    uint32_t m0 = lk.xor3(lk.template lookup<0, 0>(b0), lk.template lookup<1, 1>(b1),
                          lk.template lookup<2, 2>(b2));
    uint32_t m1 = lk.xor3(lk.template lookup<0, 0>(b1), lk.template lookup<1, 1>(b2),
                          lk.template lookup<2, 2>(b3));
    uint32_t m2 = lk.xor3(lk.template lookup<0, 0>(b2), lk.template lookup<1, 1>(b3),
                          lk.template lookup<2, 2>(b0));
    uint32_t m3 = lk.xor3(lk.template lookup<0, 0>(b3), lk.template lookup<1, 1>(b0),
                          lk.template lookup<2, 2>(b1));
    n0 = ra.mix(lk, n0, lk.template lookup<3, 3>(a3), 4 * r + 0);
    n1 = ra.mix(lk, n1, lk.template lookup<3, 3>(a0), 4 * r + 1);
    n2 = ra.mix(lk, n2, lk.template lookup<3, 3>(a1), 4 * r + 2);
    n3 = ra.mix(lk, n3, lk.template lookup<3, 3>(a2), 4 * r + 3);
    m0 = rb.mix(lk, m0, lk.template lookup<3, 3>(b3), 4 * r + 0);
    m1 = rb.mix(lk, m1, lk.template lookup<3, 3>(b0), 4 * r + 1);
    m2 = rb.mix(lk, m2, lk.template lookup<3, 3>(b1), 4 * r + 2);
    m3 = rb.mix(lk, m3, lk.template lookup<3, 3>(b2), 4 * r + 3);
    a0 = n0; a1 = n1; a2 = n2; a3 = n3;
    b0 = m0; b1 = m1; b2 = m2; b3 = m3;
  }
  auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    uint32_t x = lk.template lookup<2, 0>(a), y = lk.template lookup<3, 1>(b);
    uint32_t z = lk.template lookup<0, 2>(c), u = lk.template lookup<1, 3>(d);
    uint32_t xy = (x & 0x000000ffu) | (y & 0xffffff00u);
    uint32_t zu = (z & 0x00ff0000u) | (u & 0xff00ffffu);
    return ((xy & 0x0000ffffu) | (zu & 0xffff0000u)) ^ k;
  };
  sa = Block4{last(a0, a1, a2, a3, ra(40)), last(a1, a2, a3, a0, ra(41)),
              last(a2, a3, a0, a1, ra(42)), last(a3, a0, a1, a2, ra(43))};
  sb = Block4{last(b0, b1, b2, b3, rb(40)), last(b1, b2, b3, b0, rb(41)),
              last(b2, b3, b0, b1, rb(42)), last(b3, b0, b1, b2, rb(43))};
}

// Two MMO hashes interleaved.
template <class LK, class RKA, class RKB>
DPF_HD void mmo_hash2(Block4& xa, Block4& xb, const LK& lk, const RKA& ra, const RKB& rb) {
  Block4 sa = sigma(xa), sb = sigma(xb);
  Block4 ea = sa, eb = sb;
  encrypt2(ea, eb, lk, ra, rb);
  xa = Block4{ea.w0 ^ sa.w0, ea.w1 ^ sa.w1, ea.w2 ^ sa.w2, ea.w3 ^ sa.w3};
  xb = Block4{eb.w0 ^ sb.w0, eb.w1 ^ sb.w1, eb.w2 ^ sb.w2, eb.w3 ^ sb.w3};
}

// NA + NB independent encryptions interleaved round by round (ILP NA + NB):
// chain i < NA takes its round keys from ra[i], chain NA + j from rb[j] (two
// key providers, e.g. a uniform value key beside a per-lane key select).
template <int NA, int NB, class LK, class RKA, class RKB>
DPF_HD void encryptAB(Block4* st, const LK& lk, const RKA* ra, const RKB* rb) {
  constexpr int N = NA + NB;
  // After full unrolling `i` is a constant, so each chain binds one provider.
  auto key = [&](int i, int j) { return i < NA ? ra[i < NA ? i : 0](j) : rb[i < NA ? 0 : i - NA](j); };
  auto mix = [&](int i, uint32_t a, uint32_t b, int j) {
    return i < NA ? ra[i < NA ? i : 0].mix(lk, a, b, j) : rb[i < NA ? 0 : i - NA].mix(lk, a, b, j);
  };
  uint32_t w[N][4];
DPF_UNROLL
  for (int i = 0; i < N; ++i) {
    w[i][0] = st[i].w0 ^ key(i, 0);
    w[i][1] = st[i].w1 ^ key(i, 1);
    w[i][2] = st[i].w2 ^ key(i, 2);
    w[i][3] = st[i].w3 ^ key(i, 3);
  }
#if DPF_L1_FIRST > 1 && DPF_L1_AB
  DPF_UNROLL
  for (int r = 1; r < DPF_L1_FIRST; ++r) {
    // Two chains at a time (a scheduling region each): the whole ILP-N round
    // at once crashes hipcc's register allocator under iterative-ilp.
DPF_UNROLL
    for (int i = 0; i < N; ++i) {
      uint32_t n[4];
DPF_UNROLL
      for (int c = 0; c < 4; ++c)
        n[c] = mix(i, lk.xor3(lk.template l1<0, 0>(w[i][c]), lk.template l1<1, 1>(w[i][(c + 1) & 3]),
                              lk.template l1<2, 2>(w[i][(c + 2) & 3])),
                   lk.template l1<3, 3>(w[i][(c + 3) & 3]), 4 * r + c);
DPF_UNROLL
      for (int c = 0; c < 4; ++c) w[i][c] = n[c];
      if (i % 2 == 1) __builtin_amdgcn_sched_barrier(0);
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // hipcc's iterative-ilp RA crashes without it
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  DPF_ROUND_LOOP
#endif
  for (int r = DPF_L1_AB ? DPF_L1_FIRST : 1; r < 10; ++r) {
    uint32_t n[N][4];
DPF_UNROLL
    for (int i = 0; i < N; ++i) {
DPF_UNROLL
      for (int c = 0; c < 4; ++c)
        n[i][c] = lk.xor3(lk.template lookup<0, 0>(w[i][c]), lk.template lookup<1, 1>(w[i][(c + 1) & 3]),
                          lk.template lookup<2, 2>(w[i][(c + 2) & 3]));
    }
DPF_UNROLL
    for (int i = 0; i < N; ++i) {
DPF_UNROLL
      for (int c = 0; c < 4; ++c)
        n[i][c] = mix(i, n[i][c], lk.template lookup<3, 3>(w[i][(c + 3) & 3]), 4 * r + c);
    }
DPF_UNROLL
    for (int i = 0; i < N; ++i)
DPF_UNROLL
      for (int c = 0; c < 4; ++c) w[i][c] = n[i][c];
  }
  auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    uint32_t x = lk.template lookup<2, 0>(a), y = lk.template lookup<3, 1>(b);
    uint32_t z = lk.template lookup<0, 2>(c), u = lk.template lookup<1, 3>(d);
    uint32_t xy = (x & 0x000000ffu) | (y & 0xffffff00u);
    uint32_t zu = (z & 0x00ff0000u) | (u & 0xff00ffffu);
    return ((xy & 0x0000ffffu) | (zu & 0xffff0000u)) ^ k;
  };
DPF_UNROLL
  for (int i = 0; i < N; ++i) {
    st[i] = Block4{last(w[i][0], w[i][1], w[i][2], w[i][3], key(i, 40)),
                   last(w[i][1], w[i][2], w[i][3], w[i][0], key(i, 41)),
                   last(w[i][2], w[i][3], w[i][0], w[i][1], key(i, 42)),
                   last(w[i][3], w[i][0], w[i][1], w[i][2], key(i, 43))};
#if defined(__HIP_DEVICE_COMPILE__)
    // Keeps the scheduler from issuing all N chains' last-round lookups before
    // any is consumed: at ILP4 the 64 live results spilled at 128 VGPRs (the
    // octet kernel: 37 -> 23 spilled VGPRs, HBM traffic 21.5 -> 17.7 GB per
    // config-2 launch, same speed; profiles/r11_ws_ab.txt).
    if (i % DPF_LAST_ROUND_FENCE == DPF_LAST_ROUND_FENCE - 1) __builtin_amdgcn_sched_barrier(0);
#endif
  }
}

// N independent encryptions interleaved round by round (ILP N): rk[i]
// provides chain i's round keys.
template <int N, class LK, class RK>
DPF_HD void encryptN(Block4* st, const LK& lk, const RK* rk) {
  encryptAB<N, 0>(st, lk, rk, rk);
}

// N MMO hashes interleaved.
template <int N, class LK, class RK>
DPF_HD void mmo_hashN(Block4* x, const LK& lk, const RK* rk) {
  Block4 s[N], e[N];
DPF_UNROLL
  for (int i = 0; i < N; ++i) e[i] = s[i] = sigma(x[i]);
  encryptN<N>(e, lk, rk);
DPF_UNROLL
  for (int i = 0; i < N; ++i)
    x[i] = Block4{e[i].w0 ^ s[i].w0, e[i].w1 ^ s[i].w1, e[i].w2 ^ s[i].w2, e[i].w3 ^ s[i].w3};
}

// NA + NB MMO hashes interleaved (encryptAB's key providers).
template <int NA, int NB, class LK, class RKA, class RKB>
DPF_HD void mmo_hashAB(Block4* x, const LK& lk, const RKA* ra, const RKB* rb) {
  constexpr int N = NA + NB;
  Block4 s[N], e[N];
DPF_UNROLL
  for (int i = 0; i < N; ++i) e[i] = s[i] = sigma(x[i]);
  encryptAB<NA, NB>(e, lk, ra, rb);
DPF_UNROLL
  for (int i = 0; i < N; ++i)
    x[i] = Block4{e[i].w0 ^ s[i].w0, e[i].w1 ^ s[i].w1, e[i].w2 ^ s[i].w2, e[i].w3 ^ s[i].w3};
}

// Host-side lookup over four plain 256-entry tables (unit checks only).
struct HostLookup {
  uint32_t t[4][256];
  HostLookup() {
    for (int x = 0; x < 256; ++x)
      for (int k = 0; k < 4; ++k) t[k][x] = rotl32(t0_entry(x), 8 * k);
  }
  template <int T, int K>
  uint32_t lookup(uint32_t w) const { return t[T][(w >> (8 * K)) & 0xff]; }
  template <int T, int K>
  uint32_t l1(uint32_t w) const { return lookup<T, K>(w); }
  uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) const { return a ^ b ^ c; }
};

struct ArrayRK {
  const uint32_t* k;
  DPF_HD uint32_t operator()(int i) const { return k[i]; }
  template <class LK>
  DPF_HD uint32_t mix(const LK& lk, uint32_t a, uint32_t b, int i) const { return lk.xor3(a, b, k[i]); }
};

}  // namespace dpf_aes
