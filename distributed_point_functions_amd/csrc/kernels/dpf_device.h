// dpf_device.h -- device-side building blocks shared by the gfx950 kernel
// translation units (dpf_kernels.hip, dpf_batch.hip): the bank-replicated LDS
// T-table AES, tree steps (distributed_point_function.cc:315-343,
// evaluate_prg_hwy.cc:452-486), leaf conversion/correction (value_type_helpers.h,
// int_mod_n.h) and the exact wide accumulators of the sum paths.
// Everything lives in an anonymous namespace: each TU gets private copies of
// the kernels' helpers and of the constant T-table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../../include/dpf_hip.h"
#include "aes_core.h"

namespace {

// ------------------------------------------------------------------------
// Tables and keys
// ------------------------------------------------------------------------
struct T0Table {
  uint32_t v[256];
};
constexpr T0Table make_t0() {
  T0Table t{};
  for (int i = 0; i < 256; ++i) {
    uint32_t s = dpf_aes::kSbox[i];
    uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
    t.v[i] = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
  }
  return t;
}
__constant__ T0Table c_t0 = make_t0();

struct RoundKeys {
  uint32_t k[44];
};

RoundKeys expand_key(const dpf_aes_key* key) {
  RoundKeys rk;
  dpf_aes::expand_key(key->bytes, rk.k);
  return rk;
}

constexpr int kBlock = 1024;             // threads per workgroup (16 waves)
constexpr int kWgPerCu = 1;              // one 128 KiB-table workgroup per CU
constexpr int kTabWords = 4 * 256 * 32;  // 4 tables x 256 entries x 32 bank copies = 128 KiB
#define DPF_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(4, 4)))
constexpr int kMaxCwLevels = 128;
#ifndef DPF_SMAX
#define DPF_SMAX 12
#endif
constexpr int kSMax = DPF_SMAX;          // max subtree depth handled per thread
constexpr int kGMax = kSMax - 1;         // max depth of the DFS stack above leaf pairs
constexpr int kBMax = 8;                 // max AES blocks hashed per leaf (generic path)

// LDS image: [tables 128 KiB][cw seeds 128 x 16 B][cw control 128 x 4 B]
struct LdsImage {
  uint32_t tab[kTabWords];
  uint4 cw_seed[kMaxCwLevels];
  uint32_t cw_ctrl[kMaxCwLevels];
};

// Table image: 256-byte rows.  Row e of the low 64 KiB = [T0[e] x 32 copies |
// T1[e] x 32 copies], of the high 64 KiB = [T2[e] x 32 | T3[e] x 32].  Lane l
// reads copy (l & 31), so every ds_read_b32 of a wave is bank-conflict-free.
// Filled 16 bytes (4 copies) per store: 8192 ds_write_b128 per workgroup, so a
// small workgroup (block_for) fills its tables in a few microseconds.
// The T0 loads of 16 stores are issued together: a 64-thread workgroup (small
// launches, block_for) makes 128 stores per thread, and one dependent
// constant-memory load per store cost ~40 us of a 2^12-output EvaluateUntil.
__device__ __forceinline__ void fill_tables(uint32_t* tab) {
  constexpr int kQuads = kTabWords / 4, kBatch = 16;
  for (int q0 = threadIdx.x; q0 < kQuads; q0 += kBatch * blockDim.x) {
    uint32_t v0[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int q = q0 + j * blockDim.x;
      v0[j] = q < kQuads ? c_t0.v[q >> 5] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      // q = (entry e, table t, quad k): words [half * 16384 + e * 64 + (t & 1) * 32 + 4k, +4)
      const int q = q0 + j * blockDim.x;
      if (q >= kQuads) break;
      const int e = q >> 5, t = (q >> 3) & 3, k = q & 7;
      const uint32_t v = t == 0 ? v0[j] : ((v0[j] << (8 * t)) | (v0[j] >> (32 - 8 * t)));
      *reinterpret_cast<uint4*>(tab + (t >> 1) * 16384 + e * 64 + (t & 1) * 32 + 4 * k) =
          make_uint4(v, v, v, v);
    }
  }
}

__device__ __forceinline__ void fill_cws(LdsImage& lds, const dpf_block* cw_seed,
                                         const uint8_t* cw_left, const uint8_t* cw_right,
                                         int num_levels) {
  for (int i = threadIdx.x; i < num_levels; i += blockDim.x) {
    dpf_block b = cw_seed[i];
    lds.cw_seed[i] = make_uint4((uint32_t)b.low, (uint32_t)(b.low >> 32), (uint32_t)b.high,
                                (uint32_t)(b.high >> 32));
    lds.cw_ctrl[i] = (uint32_t)(cw_left[i] & 1) | ((uint32_t)(cw_right[i] & 1) << 1);
  }
}

// Round keys of one AES key held as ONE VGPR: lane i keeps word i (i < 44),
// read as a wave-uniform value with v_readlane (an SGPR; no memory access).
// The kernel-argument form (DPF_RK_LANES=0) reloads a round's words with
// s_load inside the rolled round loops, and SMEM returns out of order behind
// the same lgkmcnt as the table lookups, so every first use of a reloaded
// word waited lgkmcnt(0) for all lookups in flight.
// key_ref must run where all lanes 0..43 of the wave are active (kernel
// entry; workgroups are whole waves).
#ifndef DPF_RK_LANES
#define DPF_RK_LANES 0
#endif
#if DPF_RK_LANES
struct KeyRef {
  uint32_t v;
};
__device__ __forceinline__ KeyRef key_ref(const RoundKeys& rk) {
  const int l = threadIdx.x & 63;
  uint32_t v = rk.k[l < 44 ? l : 43];
  // Pins the load at kernel entry (every lane active): without it the
  // compiler sank it into divergent code, where inactive lanes never loaded
  // their word and v_readlane read garbage (wrong outputs, r15).
  asm volatile("" : "+v"(v));
  return KeyRef{v};
}
__device__ __forceinline__ uint32_t rk_word(KeyRef k, int i) {
  return __builtin_amdgcn_readlane(k.v, i);
}
#else
struct KeyRef {
  const uint32_t* k;
};
__device__ __forceinline__ KeyRef key_ref(const RoundKeys& rk) { return KeyRef{rk.k}; }
__device__ __forceinline__ uint32_t rk_word(KeyRef k, int i) { return k.k[i]; }
#endif

// The four keys of a launch (left, right, value, left ^ right) as KeyRefs.
struct KeySet {
  KeyRef l, r, v, d;
};

// Conflict-free LDS T-table lookup with ONE VALU of addressing: v_perm_b32
// builds the byte address {lane offset, byte K of w, table half, 0}, i.e.
// (entry << 8) | lt[T] with lt[T] = (lane & 31) * 4 (+128 for T1/T3, +64 KiB
// for T2/T3).
//
// Byte 1 of w already sits at bits 8-15, where the address wants it: that
// lookup's address is (w & 0xff00) | lt[T], one v_bitop3_b32 -- a full-rate
// VALU op, where v_perm_b32 is half rate (profiles/r10_valu_issue_microbench.txt)
// -- with the mask held in a VGPR (an SGPR operand would make it half rate too).
struct LdsLookup {
  const char* base;
  uint32_t lt[4];
  uint32_t m1;  // 0xff00 in a VGPR
  KeySet ks;    // the launch's round keys (set by make_lookup(lds, keys))
  template <int T, int K>
  __device__ __forceinline__ uint32_t lookup(uint32_t w) const {
    uint32_t off;
#if !defined(DPF_NO_BYTE1_BITOP3)
    if constexpr (K == 1) {
      off = __builtin_amdgcn_bitop3_b32(w, m1, lt[T], 0xEA);  // (S0 & S1) | S2
    } else
#endif
    {
      constexpr uint32_t sel = 0x0c020000u | ((4u + K) << 8);
      off = __builtin_amdgcn_perm(w, lt[T], sel);
    }
    return *reinterpret_cast<const uint32_t*>(base + off);
  }
  __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) const {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
  // The same lookup through the vector memory pipe (aes_core.h DPF_L1_ROUNDS):
  // T0 from a 1 KiB constant table (L1-resident after the first touches),
  // T1..T3 as its byte rotations.
  template <int T, int K>
  __device__ __forceinline__ uint32_t l1(uint32_t w) const {
    const uint32_t v = c_t0.v[(w >> (8 * K)) & 0xffu];
    return T == 0 ? v : __builtin_amdgcn_alignbit(v, v, 32 - 8 * T);
  }
};

__device__ __forceinline__ LdsLookup make_lookup(const LdsImage& lds) {
  uint32_t l = (threadIdx.x & 31) * 4u;
  uint32_t m1;
  asm volatile("v_mov_b32 %0, 0xff00" : "=v"(m1));
  return LdsLookup{reinterpret_cast<const char*>(lds.tab), {l, l + 128u, l + 65536u, l + 65664u},
                   m1, KeySet{}};
}
__device__ __forceinline__ LdsLookup make_lookup(const LdsImage& lds, KeySet ks) {
  LdsLookup lk = make_lookup(lds);
  lk.ks = ks;
  return lk;
}

// Round keys shared by the whole wave.
struct UniformRK {
  KeyRef k;
  __device__ __forceinline__ uint32_t operator()(int i) const { return rk_word(k, i); }
  template <class LK>
  __device__ __forceinline__ uint32_t mix(const LK& lk, uint32_t a, uint32_t b, int i) const {
    return lk.xor3(a, b, rk_word(k, i));
  }
};
// Per-lane key choice: rk = left ^ (mask & (left ^ right)).  In a round's last
// XOR the choice costs one bitop3: (a ^ b ^ left) ^ (mask & diff), each
// instruction reading one scalar key word (a VALU op reads at most one SGPR;
// the plain form needed a v_mov of the key word first).
struct SelectRK {
  KeyRef left;
  KeyRef diff;
  uint32_t mask;
  __device__ __forceinline__ uint32_t operator()(int i) const {
    return rk_word(left, i) ^ (mask & rk_word(diff, i));
  }
  template <class LK>
  __device__ __forceinline__ uint32_t mix(const LK& lk, uint32_t a, uint32_t b, int i) const {
    // bitop3 truth table index = S0*4 + S1*2 + S2; 0x78 = S0 ^ (S1 & S2).
    return __builtin_amdgcn_bitop3_b32(lk.xor3(a, b, rk_word(left, i)), mask, rk_word(diff, i),
                                       0x78);
  }
};

using dpf_aes::Block4;
using u128 = unsigned __int128;

__device__ __forceinline__ u128 block_u128(Block4 h) {
  return ((u128)h.w3 << 96) | ((u128)h.w2 << 64) | ((u128)h.w1 << 32) | h.w0;
}
__device__ __forceinline__ u128 dpf_u128(dpf_block c) { return ((u128)c.high << 64) | c.low; }

// Full-domain expansion launch (dpf_hip_expand): items are subtrees.
struct ExpandParams {
  int64_t num_items;  // num_starts << k0
  int num_levels;     // L = k0 + S
  int k0;             // levels walked per item (per-lane direction)
  int S;              // subtree depth visited per item
  const dpf_block* seeds_in;
  const uint8_t* ctrl_in;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  char* out;
  RoundKeys rkl, rkr, rkv, rkd;
  // Octet kernel only: 0 = item u on thread u (grid stride); > 0 = workgroup b
  // owns items [b, b + 1) * dyn_chunks * 64 and its waves take them 64 at a
  // time from an LDS counter (dynamic distribution, dpf_kernels.hip).
  int dyn_chunks;
  // Clock probe (dpf_hip_clock_probe): NULL, or [shader clocks, 100 MHz ticks,
  // workgroups] that wave 0 of every workgroup adds its s_memtime /
  // s_memrealtime deltas around its work into.  Nothing reads it back in the
  // kernel; no output depends on it.
  unsigned long long* clock;
};

// Dynamic distribution of 64-item chunks over a workgroup's waves (r16).
// A CU's arbiter favours its oldest waves, so with a fixed share per thread
// the first waves of a workgroup finish long before the last (config 2's
// octet kernel: wave 0 at 7.8 ms, wave 15 at 16.6 ms of a 16.9 ms launch) and
// the end of every launch runs on fewer and fewer waves.  Taken one chunk
// at a time instead, the favoured waves do more of the work and all finish
// together.  Workgroup b owns chunks [b * per_wg, (b + 1) * per_wg) below
// `chunks`; the wave's lane 0 takes the next from `counter` (LDS, zeroed
// before the workgroup's first take).  Returns chunk * 64 + lane, or `done`
// once the workgroup's chunks are used up; wave-uniform.
__device__ __forceinline__ int64_t take_chunk(int* counter, int64_t per_wg, int64_t chunks,
                                              int64_t done) {
  int c = 0;
  if ((threadIdx.x & 63) == 0) c = atomicAdd(counter, 1);
  c = __builtin_amdgcn_readfirstlane(c);
  const int64_t g = (int64_t)blockIdx.x * per_wg + c;
  return c < per_wg && g < chunks ? g * 64 + (int64_t)(threadIdx.x & 63) : done;
}

// Stamps of the clock probe: wave-uniform (wave 0 of the workgroup), two
// reads per workgroup, so the probe costs nothing measurable in a launch of
// milliseconds (MI355X_MICROARCH.md: in-kernel clock = delta s_memtime /
// delta s_memrealtime x 100 MHz).
#ifndef DPF_CLOCK_PROBE
#define DPF_CLOCK_PROBE 1   // 0: stamps compiled out (A/B variant builds)
#endif
#ifndef DPF_CLOCK_PROBE_WAVE
#define DPF_CLOCK_PROBE_WAVE 0   // the stamped wave of each workgroup (variant builds: the last)
#endif
struct ClockStamp {
  unsigned long long c0 = 0, r0 = 0;
  __device__ __forceinline__ void begin(const unsigned long long* acc) {
    if (DPF_CLOCK_PROBE && acc != nullptr && (threadIdx.x >> 6) == DPF_CLOCK_PROBE_WAVE) {
      c0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) before the LDS loop
    }
  }
  __device__ __forceinline__ void end(unsigned long long* acc) {
    if (DPF_CLOCK_PROBE && acc != nullptr && (threadIdx.x >> 6) == DPF_CLOCK_PROBE_WAVE) {
      const unsigned long long c1 = __builtin_amdgcn_s_memtime();
      const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if ((threadIdx.x & 63) == 0) {
        atomicAdd(acc + 0, c1 - c0);
        atomicAdd(acc + 1, r1 - r0);
        atomicAdd(acc + 2, 1ull);
      }
    }
  }
};

__device__ __forceinline__ Block4 load_block(const dpf_block* p) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  return Block4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void store_block(dpf_block* p, Block4 b) {
  *reinterpret_cast<uint4*>(p) = make_uint4(b.w0, b.w1, b.w2, b.w3);
}
__device__ __forceinline__ Block4 add_small(Block4 s, uint32_t j) {
  // seed + j as absl::uint128 (distributed_point_function.cc:512)
  uint64_t lo = ((uint64_t)s.w1 << 32) | s.w0, hi = ((uint64_t)s.w3 << 32) | s.w2;
  uint64_t nlo = lo + j;
  hi += (nlo < lo) ? 1 : 0;
  return Block4{(uint32_t)nlo, (uint32_t)(nlo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

// One tree step for a uniformly chosen child: seed/control correction and
// control-bit extraction in the order of distributed_point_function.cc:323-343.
__device__ __forceinline__ void child_step(const LdsLookup& lk, KeyRef rk, Block4 s,
                                           uint32_t t, uint32_t dir, uint4 cs, uint32_t cctl,
                                           Block4& out, uint32_t& tout) {
  Block4 h = dpf_aes::mmo_hash(s, lk, UniformRK{rk});
  uint32_t m = 0u - t;
  h.w0 ^= cs.x & m; h.w1 ^= cs.y & m; h.w2 ^= cs.z & m; h.w3 ^= cs.w & m;
  uint32_t nt = h.w0 & 1u;
  h.w0 &= ~1u;
  nt ^= t & ((cctl >> dir) & 1u);
  out = h;
  tout = nt;
}

// Both children of one node: two interleaved MMO hashes (left key, right key).
__device__ __forceinline__ void children_step(const LdsLookup& lk, KeyRef rkl,
                                              KeyRef rkr, Block4 s, uint32_t t, uint4 cs,
                                              uint32_t cctl, Block4& c0, uint32_t& t0, Block4& c1,
                                              uint32_t& t1) {
  Block4 h0 = s, h1 = s;
  dpf_aes::mmo_hash2(h0, h1, lk, UniformRK{rkl}, UniformRK{rkr});
  uint32_t m = 0u - t;
  h0.w0 ^= cs.x & m; h0.w1 ^= cs.y & m; h0.w2 ^= cs.z & m; h0.w3 ^= cs.w & m;
  h1.w0 ^= cs.x & m; h1.w1 ^= cs.y & m; h1.w2 ^= cs.z & m; h1.w3 ^= cs.w & m;
  t0 = (h0.w0 & 1u) ^ (t & (cctl & 1u));
  t1 = (h1.w0 & 1u) ^ (t & ((cctl >> 1) & 1u));
  h0.w0 &= ~1u;
  h1.w0 &= ~1u;
  c0 = h0;
  c1 = h1;
}

// children_step for two nodes of the same level (same correction word): the
// four child hashes interleaved (ILP4).
__device__ __forceinline__ void children_step_x2(const LdsLookup& lk, KeyRef rkl,
                                                 KeyRef rkr, Block4 sa, uint32_t ta,
                                                 Block4 sb, uint32_t tb, uint4 cs, uint32_t cctl,
                                                 Block4* c, uint32_t* t) {
  Block4 h[4] = {sa, sa, sb, sb};
  const UniformRK rk[4] = {UniformRK{rkl}, UniformRK{rkr}, UniformRK{rkl}, UniformRK{rkr}};
  dpf_aes::mmo_hashN<4>(h, lk, rk);
  const uint32_t pt[4] = {ta, ta, tb, tb};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t m = 0u - pt[i];
    h[i].w0 ^= cs.x & m; h[i].w1 ^= cs.y & m; h[i].w2 ^= cs.z & m; h[i].w3 ^= cs.w & m;
    t[i] = (h[i].w0 & 1u) ^ (pt[i] & ((cctl >> (i & 1)) & 1u));
    h[i].w0 &= ~1u;
    c[i] = h[i];
  }
}

// Path step with a per-lane direction bit (evaluate_prg_hwy.cc:452-486).
__device__ __forceinline__ void path_step(const LdsLookup& lk, KeyRef rkl,
                                          KeyRef rkd, Block4& s, uint32_t& t,
                                          uint32_t bit, uint4 cs, uint32_t cctl) {
  Block4 h = dpf_aes::mmo_hash(s, lk, SelectRK{rkl, rkd, 0u - bit});
  uint32_t m = 0u - t;
  h.w0 ^= cs.x & m; h.w1 ^= cs.y & m; h.w2 ^= cs.z & m; h.w3 ^= cs.w & m;
  uint32_t nt = h.w0 & 1u;
  h.w0 &= ~1u;
  nt ^= t & ((cctl >> bit) & 1u);
  s = h;
  t = nt;
}

// ------------------------------------------------------------------------
// Leaf conversion + correction (a12/a13)
// ------------------------------------------------------------------------

// Element-wise add/neg of a 128-bit block viewed as 128/BITS little-endian lanes.
template <int BITS>
__device__ __forceinline__ Block4 lanes_add(Block4 a, Block4 b) {
  if constexpr (BITS == 128) {
    uint64_t alo = ((uint64_t)a.w1 << 32) | a.w0, ahi = ((uint64_t)a.w3 << 32) | a.w2;
    uint64_t blo = ((uint64_t)b.w1 << 32) | b.w0, bhi = ((uint64_t)b.w3 << 32) | b.w2;
    uint64_t lo = alo + blo, hi = ahi + bhi + (lo < alo ? 1 : 0);
    return Block4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  } else if constexpr (BITS == 64) {
    uint64_t lo = (((uint64_t)a.w1 << 32) | a.w0) + (((uint64_t)b.w1 << 32) | b.w0);
    uint64_t hi = (((uint64_t)a.w3 << 32) | a.w2) + (((uint64_t)b.w3 << 32) | b.w2);
    return Block4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  } else if constexpr (BITS == 32) {
    return Block4{a.w0 + b.w0, a.w1 + b.w1, a.w2 + b.w2, a.w3 + b.w3};
  } else {
    constexpr uint32_t H = BITS == 16 ? 0x80008000u : 0x80808080u;
    auto f = [](uint32_t x, uint32_t y) { return ((x & ~H) + (y & ~H)) ^ ((x ^ y) & H); };
    return Block4{f(a.w0, b.w0), f(a.w1, b.w1), f(a.w2, b.w2), f(a.w3, b.w3)};
  }
}
template <int BITS>
__device__ __forceinline__ Block4 lanes_neg(Block4 a) {
  if constexpr (BITS == 128) {
    uint64_t lo = ((uint64_t)a.w1 << 32) | a.w0, hi = ((uint64_t)a.w3 << 32) | a.w2;
    uint64_t nlo = 0 - lo, nhi = 0 - hi - (lo != 0 ? 1 : 0);
    return Block4{(uint32_t)nlo, (uint32_t)(nlo >> 32), (uint32_t)nhi, (uint32_t)(nhi >> 32)};
  } else if constexpr (BITS == 64) {
    uint64_t lo = 0 - (((uint64_t)a.w1 << 32) | a.w0);
    uint64_t hi = 0 - (((uint64_t)a.w3 << 32) | a.w2);
    return Block4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  } else if constexpr (BITS == 32) {
    return Block4{0u - a.w0, 0u - a.w1, 0u - a.w2, 0u - a.w3};
  } else {
    constexpr uint32_t H = BITS == 16 ? 0x80008000u : 0x80808080u;
    auto f = [](uint32_t x) { return (H - (x & ~H)) ^ (~x & H); };
    return Block4{f(a.w0), f(a.w1), f(a.w2), f(a.w3)};
  }
}

// Stores `bytes` (1..16) of a little-endian 128-bit value with the widest
// stores the alignment of `p` (a multiple of the packed element size) allows.
__device__ __forceinline__ void store_packed(char* p, Block4 v, int bytes) {
  switch (bytes) {
    case 16: *reinterpret_cast<uint4*>(p) = make_uint4(v.w0, v.w1, v.w2, v.w3); return;
    case 8: *reinterpret_cast<uint2*>(p) = make_uint2(v.w0, v.w1); return;
    case 4: *reinterpret_cast<uint32_t*>(p) = v.w0; return;
    case 2: *reinterpret_cast<uint16_t*>(p) = (uint16_t)v.w0; return;
    case 1: *reinterpret_cast<uint8_t*>(p) = (uint8_t)v.w0; return;
    case 12: {
      uint32_t* q = reinterpret_cast<uint32_t*>(p);
      q[0] = v.w0; q[1] = v.w1; q[2] = v.w2;
      return;
    }
    default: {
      const uint32_t w[4] = {v.w0, v.w1, v.w2, v.w3};
      for (int i = 0; i < bytes; ++i) p[i] = (char)(uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
  }
}

// Plain unsigned integers and XorWrapper of them with b == 1: the hashed block
// *is* the element array (value_type_helpers.h:199-211), the correction word is
// one block in the same layout.
template <int BITS, bool XOR>
struct FastIntLeaf {
  const dpf_block* vcw_elems;  // E elements, one dpf_block each (device)
  int E;
  int party;
  int store_bytes;    // elements_per_leaf * BITS / 8 (1..16)
  Block4 vcw;         // value correction packed as E lanes of BITS (set by init)

  // Packs the per-element correction into one block (value_type_helpers.h:597-631
  // produces E elements whose concatenation has the hashed block's layout).
  __device__ __forceinline__ void init() {
    unsigned __int128 packed = 0;
    for (int e = E - 1; e >= 0; --e) {
      dpf_block c = vcw_elems[e];
      unsigned __int128 v = ((unsigned __int128)c.high << 64) | c.low;
      if (BITS < 128) {
        v &= (((unsigned __int128)1 << (BITS & 127)) - 1);
        packed = (packed << (BITS & 127)) | v;
      } else {
        packed = v;
      }
    }
    vcw = Block4{(uint32_t)packed, (uint32_t)(packed >> 32), (uint32_t)(packed >> 64),
                 (uint32_t)(packed >> 96)};
  }

  __device__ __forceinline__ Block4 correct(Block4 h, uint32_t t) const {
    if (XOR) {
      uint32_t m = 0u - t;
      return Block4{h.w0 ^ (vcw.w0 & m), h.w1 ^ (vcw.w1 & m), h.w2 ^ (vcw.w2 & m),
                    h.w3 ^ (vcw.w3 & m)};
    }
    if (t) h = lanes_add<BITS>(h, vcw);
    if (party == 1) h = lanes_neg<BITS>(h);
    return h;
  }

  __device__ __forceinline__ void store(Block4 h, int64_t leaf, char* out) const {
    store_packed(out + leaf * (int64_t)store_bytes, h, store_bytes);
  }

  // Full-domain leaf: write elements_per_leaf elements.
  __device__ __forceinline__ void emit(const LdsLookup& lk, KeyRef rkv, Block4 seed,
                                       uint32_t t, int64_t leaf, char* out) const {
    store(correct(dpf_aes::mmo_hash(seed, lk, UniformRK{rkv}), t), leaf, out);
  }
  // Two sibling leaves (leaf, leaf + 1), hashed as one interleaved pair.
  __device__ __forceinline__ void emit2(const LdsLookup& lk, KeyRef rkv, Block4 s0,
                                        uint32_t t0, Block4 s1, uint32_t t1, int64_t leaf,
                                        char* out) const {
    dpf_aes::mmo_hash2(s0, s1, lk, UniformRK{rkv}, UniformRK{rkv});
    s0 = correct(s0, t0);
    s1 = correct(s1, t1);
    if (store_bytes == 16) {
      uint4* p = reinterpret_cast<uint4*>(out + leaf * 16);
      p[0] = make_uint4(s0.w0, s0.w1, s0.w2, s0.w3);
      p[1] = make_uint4(s1.w0, s1.w1, s1.w2, s1.w3);
    } else {
      store(s0, leaf, out);
      store(s1, leaf + 1, out);
    }
  }
  // Four consecutive leaves, hashed as one interleaved quadruple.
  __device__ __forceinline__ void emit4(const LdsLookup& lk, KeyRef rkv, Block4* s,
                                        const uint32_t* t, int64_t leaf, char* out) const {
    const UniformRK rk[4] = {UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}};
    dpf_aes::mmo_hashN<4>(s, lk, rk);
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = correct(s[i], t[i]);
    if (store_bytes == 16) {
      uint4* p = reinterpret_cast<uint4*>(out + leaf * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) p[i] = make_uint4(s[i].w0, s[i].w1, s[i].w2, s[i].w3);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) store(s[i], leaf + i, out);
    }
  }
};

// Invariant-divisor division of a 64-bit value by a 32-bit modulus
// (Moller & Granlund, "Improved division by invariant integers", Alg. 4):
// dn = N << sh is normalised (top bit set) and v = floor((2^64-1)/dn) - 2^32.
struct Div32 {
  uint32_t dn, v;
  int sh;
  uint32_t n;
};

// (u1:u0) / d for u1 < d, d normalised.  Returns the quotient word, r = remainder.
__device__ __forceinline__ uint32_t div_2by1(uint32_t u1, uint32_t u0, uint32_t d, uint32_t v,
                                             uint32_t& r) {
  uint64_t q = (uint64_t)v * u1;
  q += ((uint64_t)(u1 + 1u) << 32) | u0;
  uint32_t q1 = (uint32_t)(q >> 32), q0 = (uint32_t)q;
  uint32_t rr = u0 - q1 * d;
  if (rr > q0) { --q1; rr += d; }
  if (rr >= d) { ++q1; rr -= d; }
  r = rr;
  return q1;
}

// 128-bit block w (little-endian words) -> remainder mod N, and the low three
// quotient words (what `quotient << 32` keeps of it, int_mod_n.h:167-176).
__device__ __forceinline__ uint32_t divmod128(const uint32_t w[4], const Div32& d, uint32_t q[3]) {
  if (d.sh == 0) {
    // N >= 2^31 (e.g. 2^32 - 5): no normalisation shifts, and the top word's
    // quotient digit (0 or 1, shifted out) is one compare.  `d` is a kernel
    // argument, so the branch is wave-uniform.  Heavy hitters +1.5%,
    // Tuple<IntModN32 x 2> full domain +2.5% (profiles/r13_ab.txt).
    uint32_t r = w[3] >= d.dn ? w[3] - d.dn : w[3];
    q[2] = div_2by1(r, w[2], d.dn, d.v, r);
    q[1] = div_2by1(r, w[1], d.dn, d.v, r);
    q[0] = div_2by1(r, w[0], d.dn, d.v, r);
    return r;
  }
  const int sh = d.sh;
  uint32_t u4 = sh ? (w[3] >> (32 - sh)) : 0u;
  uint32_t u3 = (w[3] << sh) | (sh ? (w[2] >> (32 - sh)) : 0u);
  uint32_t u2 = (w[2] << sh) | (sh ? (w[1] >> (32 - sh)) : 0u);
  uint32_t u1 = (w[1] << sh) | (sh ? (w[0] >> (32 - sh)) : 0u);
  uint32_t u0 = w[0] << sh;
  uint32_t r = u4;
  (void)div_2by1(r, u3, d.dn, d.v, r);  // top quotient word: shifted out by `<< 32`
  q[2] = div_2by1(r, u2, d.dn, d.v, r);
  q[1] = div_2by1(r, u1, d.dn, d.v, r);
  q[0] = div_2by1(r, u0, d.dn, d.v, r);
  return r >> sh;
}


inline Div32 make_div32(uint32_t n) {
  Div32 d;
  d.n = n;
  d.sh = __builtin_clz(n);
  d.dn = n << d.sh;
  d.v = (uint32_t)(~0ull / d.dn - (1ull << 32));
  return d;
}



// Tuples of IntModN<uint32_t, N < 2^32> sampled from <= 2 blocks: 16 + 4 (nl - 1)
// bytes <= 32, so at most five leaves (the reference benchmark's
// Tuple<IntModN<uint32_t, 2^32 - 5> x5> among them).
constexpr int kMod32MaxLeaves = 5;
inline bool mod32_eligible(const dpf_value_desc* d, int* blocks_read) {
  if (d->direct || d->elements_per_block != 1 || d->num_leaves > kMod32MaxLeaves) return false;
  for (int k = 0; k < d->num_leaves; ++k)
    if (d->kind[k] != DPF_LEAF_INTMODN || d->bits[k] != 32 || d->mod_high[k] != 0 ||
        d->mod_low[k] == 0 || d->mod_low[k] > 0xffffffffull)
      return false;
  const int bytes = 16 + 4 * (d->num_leaves - 1);
  if (bytes > 16 * d->blocks_needed) return false;
  *blocks_read = (bytes + 15) / 16;
  return true;
}

// Direct conversion of a tuple of plain integers / XorWrappers of MIXED widths
// (value_type_helpers.h:199-211, 286-311 with CanBeConvertedDirectly): the
// hashed block is E packed elements, each the concatenation of its leaves, so
// the correction is a lane-wise add (XOR for XorWrapper lanes) on the 128-bit
// block with lanes of the leaves' widths -- SWAR on one u128: carries stop at
// the lane top bits `top`, XorWrapper lanes (`xmask`) take a ^ b.  Tuples whose
// leaves all have one width and kind go to FastIntLeaf instead.
#ifndef DPF_SWAR_ILP4
#define DPF_SWAR_ILP4 1
#endif
struct SwarLeaf {
  const dpf_block* vcw_elems;  // lanes = E * num_leaves values (device)
  int lanes;
  int party;
  int store_bytes;             // elements_per_leaf * packed element size
  uint8_t lane_off[16];        // bit offset of lane i in the block (lanes <= 16)
  uint8_t lane_bits[16];
  u128 top, xmask;             // lane top bits (all lanes) / XorWrapper lane bits
  u128 vcw;                    // packed correction, set by init

  __device__ __forceinline__ void init() {
    u128 packed = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // unrolled: no dynamic index into the struct
      if (i < lanes) {
        const int b = lane_bits[i];
        u128 v = dpf_u128(vcw_elems[i]);
        if (b < 128) v &= (((u128)1 << b) - 1);
        packed |= v << (lane_off[i] & 127);
      }
    }
    vcw = packed;
  }
  __device__ __forceinline__ u128 add(u128 a, u128 b) const {
    const u128 s = ((a & ~top) + (b & ~top)) ^ ((a ^ b) & top);
    return (s & ~xmask) | ((a ^ b) & xmask);
  }
  __device__ __forceinline__ u128 neg(u128 a) const {
    const u128 n = (top - (a & ~top)) ^ (~a & top);
    return (n & ~xmask) | (a & xmask);
  }
  __device__ __forceinline__ Block4 correct(Block4 h, uint32_t t) const {
    u128 x = block_u128(h);
    if (t) x = add(x, vcw);
    if (party == 1) x = neg(x);
    return Block4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)};
  }
  __device__ __forceinline__ void emit(const LdsLookup& lk, KeyRef rkv, Block4 seed,
                                       uint32_t t, int64_t leaf, char* out) const {
    store_packed(out + leaf * (int64_t)store_bytes,
                 correct(dpf_aes::mmo_hash(seed, lk, UniformRK{rkv}), t), store_bytes);
  }
  __device__ __forceinline__ void emit2(const LdsLookup& lk, KeyRef rkv, Block4 s0,
                                        uint32_t t0, Block4 s1, uint32_t t1, int64_t leaf,
                                        char* out) const {
    dpf_aes::mmo_hash2(s0, s1, lk, UniformRK{rkv}, UniformRK{rkv});
    store_packed(out + leaf * (int64_t)store_bytes, correct(s0, t0), store_bytes);
    store_packed(out + (leaf + 1) * (int64_t)store_bytes, correct(s1, t1), store_bytes);
  }
  // The half-octet's four value hashes as one ILP4 group, then the stores
  // (Tuple<u32, u64>: 18.65 -> 18.12 ms per 2^30 outputs vs two ILP2 pairs,
  // profiles/r11_ws_ab.txt).
  __device__ __forceinline__ void emit4(const LdsLookup& lk, KeyRef rkv, Block4* s,
                                        const uint32_t* t, int64_t leaf, char* out) const {
#if DPF_SWAR_ILP4
    const UniformRK rk[4] = {UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}};
    dpf_aes::mmo_hashN<4>(s, lk, rk);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      store_packed(out + (leaf + j) * (int64_t)store_bytes, correct(s[j], t[j]), store_bytes);
#else
    emit2(lk, rkv, s[0], t[0], s[1], t[1], leaf, out);
    emit2(lk, rkv, s[2], t[2], s[3], t[3], leaf + 2, out);
#endif
  }
};

// Tuples of IntModN<uint32_t, N_i < 2^32> (and a single IntModN<uint32_t, N>),
// full domain (E == 1): sampled from the first `b` hashed blocks of seed, seed+1
// (value_type_helpers.h:415-443, int_mod_n.h:155-177): r = the first 16 bytes;
// value_i = r mod N_i; r = (r / N_i) << 32 | the next 4 bytes.  Division by
// the invariant N_i is Div32's 2-by-1 word algorithm (no 128-bit division);
// only the b <= 2 blocks the sampling reads are hashed (blocks_needed may be
// more: the bytes past them never reach an output).
template <int NLMAX>
struct Mod32Leaf {
  const dpf_block* vcw_elems;  // num_leaves values (E == 1)
  int nl;
  int b;                       // hashed blocks read by the sampling: 1 or 2
  int party;
  Div32 div[NLMAX];
  uint32_t c[NLMAX];           // value correction per leaf, set by init

  __device__ __forceinline__ void init() {
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) c[i] = i < nl ? (uint32_t)vcw_elems[i].low : 0u;
  }
  __device__ __forceinline__ void convert_store(const uint32_t* w, uint32_t t, char* o) const {
    uint32_t x[NLMAX];
    convert(w, t, x);
    if (NLMAX >= 2 && nl == 2) {
      *reinterpret_cast<uint2*>(o) = make_uint2(x[0], x[NLMAX >= 2 ? 1 : 0]);
    } else {
#pragma unroll
      for (int i = 0; i < NLMAX; ++i)
        if (i < nl) reinterpret_cast<uint32_t*>(o)[i] = x[i];
    }
  }
  __device__ __forceinline__ void convert(const uint32_t* w, uint32_t t, uint32_t* x) const {
    uint32_t blk[4] = {w[0], w[1], w[2], w[3]};
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) {
      if (i < nl) {
        uint32_t q[3];
        const uint32_t n = div[i].n;
        uint32_t r = divmod128(blk, div[i], q);
        if (t) {  // IntModN += (int_mod_n.h:116-120)
          const uint32_t s = r + c[i];
          r = (s < r || s >= n) ? s - n : s;
        }
        if (party == 1) r = r == 0 ? 0u : n - r;
        x[i] = r;
        if (i + 1 < NLMAX) {   // the next leaf's block (w[4 + i]: at most w[7])
          blk[0] = w[4 + i]; blk[1] = q[0]; blk[2] = q[1]; blk[3] = q[2];
        }
      } else {
        x[i] = 0;
      }
    }
  }
  __device__ __forceinline__ void emit(const LdsLookup& lk, KeyRef rkv, Block4 seed,
                                       uint32_t t, int64_t leaf, char* out) const {
    uint32_t w[8];
    Block4 h0 = seed, h1 = add_small(seed, 1u);
    if (b == 2) {
      dpf_aes::mmo_hash2(h0, h1, lk, UniformRK{rkv}, UniformRK{rkv});
    } else {
      h0 = dpf_aes::mmo_hash(h0, lk, UniformRK{rkv});
      h1 = Block4{0, 0, 0, 0};
    }
    w[0] = h0.w0; w[1] = h0.w1; w[2] = h0.w2; w[3] = h0.w3;
    w[4] = h1.w0; w[5] = h1.w1; w[6] = h1.w2; w[7] = h1.w3;
    convert_store(w, t, out + leaf * 4 * nl);
  }
  // The value blocks (seed, seed + 1) of two leaves as words w0[8], w1[8]
  // (b == 2: one interleaved quadruple of hashes).
  __device__ __forceinline__ void hash2(const LdsLookup& lk, KeyRef rkv, Block4 s0,
                                        Block4 s1, uint32_t (&w0)[8], uint32_t (&w1)[8]) const {
    Block4 h[4] = {s0, add_small(s0, 1u), s1, add_small(s1, 1u)};
    if (b == 2) {
      const UniformRK rk[4] = {UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}};
      dpf_aes::mmo_hashN<4>(h, lk, rk);
    } else {
      dpf_aes::mmo_hash2(h[0], h[2], lk, UniformRK{rkv}, UniformRK{rkv});
      h[1] = h[3] = Block4{0, 0, 0, 0};
    }
    w0[0] = h[0].w0; w0[1] = h[0].w1; w0[2] = h[0].w2; w0[3] = h[0].w3;
    w0[4] = h[1].w0; w0[5] = h[1].w1; w0[6] = h[1].w2; w0[7] = h[1].w3;
    w1[0] = h[2].w0; w1[1] = h[2].w1; w1[2] = h[2].w2; w1[3] = h[2].w3;
    w1[4] = h[3].w0; w1[5] = h[3].w1; w1[6] = h[3].w2; w1[7] = h[3].w3;
  }
  __device__ __forceinline__ void emit2(const LdsLookup& lk, KeyRef rkv, Block4 s0,
                                        uint32_t t0, Block4 s1, uint32_t t1, int64_t leaf,
                                        char* out) const {
    uint32_t w0[8], w1[8];
    hash2(lk, rkv, s0, s1, w0, w1);
    convert_store(w0, t0, out + leaf * 4 * nl);
    convert_store(w1, t1, out + (leaf + 1) * 4 * nl);
  }
  // Four consecutive leaves (leaf % 4 == 0), converted first and stored as
  // whole 16-byte pieces: 32 contiguous bytes per lane for pairs (nl == 2),
  // 16 for single elements -- not four 8-byte stores spread over the AES work.
  __device__ __forceinline__ void emit4(const LdsLookup& lk, KeyRef rkv, Block4* s,
                                        const uint32_t* t, int64_t leaf, char* out) const {
    uint32_t x[4][NLMAX];
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      uint32_t w0[8], w1[8];
      hash2(lk, rkv, s[j], s[j + 1], w0, w1);
      convert(w0, t[j], x[j]);
      convert(w1, t[j + 1], x[j + 1]);
    }
    store4(x, leaf, out);
  }
  __device__ __forceinline__ void store4(const uint32_t (&x)[4][NLMAX], int64_t leaf,
                                         char* out) const {
    if (NLMAX >= 2 && nl == 2) {
      constexpr int i1 = NLMAX >= 2 ? 1 : 0;
      uint4* o = reinterpret_cast<uint4*>(out + leaf * 8);
      o[0] = make_uint4(x[0][0], x[0][i1], x[1][0], x[1][i1]);
      o[1] = make_uint4(x[2][0], x[2][i1], x[3][0], x[3][i1]);
    } else if (nl == 1) {
      *reinterpret_cast<uint4*>(out + leaf * 4) = make_uint4(x[0][0], x[1][0], x[2][0], x[3][0]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < NLMAX; ++i)
          if (i < nl) reinterpret_cast<uint32_t*>(out + (leaf + j) * 4 * nl)[i] = x[j][i];
    }
  }
};

// Descriptor-driven conversion for Tuple / IntModN / multi-block types
// (value_type_helpers.h:286-311, 415-443, 526-589).
struct GenericLeaf {
  dpf_value_desc d;
  const dpf_block* vcw;   // E * num_leaves blocks
  int party;
  int elements_per_leaf;  // full domain: corrected elements per block
  int esz;                // packed element size in bytes

  __device__ __forceinline__ void init() {}

  __device__ static unsigned __int128 load_le(const uint8_t* p, int n) {
    unsigned __int128 v = 0;
    for (int i = n - 1; i >= 0; --i) v = (v << 8) | p[i];
    return v;
  }
  __device__ static unsigned __int128 mask(int bits) {
    return bits >= 128 ? ~(unsigned __int128)0 : (((unsigned __int128)1 << bits) - 1);
  }
  __device__ unsigned __int128 modulus(int k) const {
    return ((unsigned __int128)d.mod_high[k] << 64) | d.mod_low[k];
  }
  __device__ unsigned __int128 add(int k, unsigned __int128 a, unsigned __int128 b) const {
    if (d.kind[k] == DPF_LEAF_XOR) return a ^ b;
    if (d.kind[k] == DPF_LEAF_INTMODN) {
      // IntModN += (int_mod_n.h:116-120, 208-223)
      unsigned __int128 n = modulus(k), c = n - b;
      return a >= c ? a - c : n - c + a;
    }
    return (a + b) & mask(d.bits[k]);
  }
  __device__ unsigned __int128 neg(int k, unsigned __int128 a) const {
    if (d.kind[k] == DPF_LEAF_XOR) return a;
    if (d.kind[k] == DPF_LEAF_INTMODN) return a == 0 ? 0 : modulus(k) - a;
    return (0 - a) & mask(d.bits[k]);
  }
  __device__ static void store_le(char* p, unsigned __int128 v, int n) {
    for (int i = 0; i < n; ++i) { p[i] = (char)(uint8_t)v; v >>= 8; }
  }

  // Hashes `seed` into b blocks and writes element `first .. first+count` of the
  // converted array (after correction) to out_elem.
  __device__ void convert_store(const LdsLookup& lk, KeyRef rkv, Block4 seed,
                                uint32_t t, int first, int count, char* out_elem) const {
    uint8_t bytes[16 * kBMax];
    const int b = d.blocks_needed;
    for (int j = 0; j < b; ++j) {
      Block4 h = dpf_aes::mmo_hash(add_small(seed, (uint32_t)j), lk, UniformRK{rkv});
      uint32_t w[4] = {h.w0, h.w1, h.w2, h.w3};
      for (int q = 0; q < 16; ++q) bytes[16 * j + q] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
    }
    const int nl = d.num_leaves;
    if (d.direct) {
      for (int e = first; e < first + count; ++e) {
        int off = e * esz;
        char* o = out_elem + (e - first) * esz;
        for (int k = 0; k < nl; ++k) {
          int lb = d.bits[k] >> 3;
          unsigned __int128 v = load_le(bytes + off, lb);
          if (t) {
            dpf_block c = vcw[e * nl + k];
            v = add(k, v, ((unsigned __int128)c.high << 64) | c.low);
          }
          if (party == 1) v = neg(k, v);
          store_le(o, v, lb);
          o += lb;
          off += lb;
        }
      }
      return;
    }
    // Sampling conversion: E == 1, every leaf but the last refills the block.
    unsigned __int128 block = load_le(bytes, 16);
    int rem = 16;
    char* o = out_elem;
    for (int k = 0; k < nl; ++k) {
      int lb = d.bits[k] >> 3;
      bool update = k + 1 < nl;
      unsigned __int128 v;
      if (d.kind[k] == DPF_LEAF_INTMODN) {
        unsigned __int128 n = modulus(k);
        unsigned __int128 q = block / n;
        v = block - q * n;
        if (update) {
          block = lb < 16 ? (q << (8 * lb)) : 0;
          block |= load_le(bytes + rem, lb);
          rem += lb;
        }
      } else {
        v = block & mask(d.bits[k]);
        if (update) {
          if (lb < 16) block &= ~mask(d.bits[k]); else block = 0;
          block |= load_le(bytes + rem, lb);
          rem += lb;
        }
      }
      if (t) {
        dpf_block c = vcw[k];
        v = add(k, v, ((unsigned __int128)c.high << 64) | c.low);
      }
      if (party == 1) v = neg(k, v);
      store_le(o, v, lb);
      o += lb;
    }
  }

  __device__ __forceinline__ void emit(const LdsLookup& lk, KeyRef rkv, Block4 seed,
                                       uint32_t t, int64_t leaf, char* out) const {
    convert_store(lk, rkv, seed, t, 0, elements_per_leaf,
                  out + leaf * (int64_t)elements_per_leaf * esz);
  }
  __device__ __forceinline__ void emit2(const LdsLookup& lk, KeyRef rkv, Block4 s0,
                                        uint32_t t0, Block4 s1, uint32_t t1, int64_t leaf,
                                        char* out) const {
    emit(lk, rkv, s0, t0, leaf, out);
    emit(lk, rkv, s1, t1, leaf + 1, out);
  }
  __device__ __forceinline__ void emit4(const LdsLookup& lk, KeyRef rkv, Block4* s,
                                        const uint32_t* t, int64_t leaf, char* out) const {
    for (int i = 0; i < 4; ++i) emit(lk, rkv, s[i], t[i], leaf + i, out);
  }
};

// ------------------------------------------------------------------------
// Latency mode: one AES chain per lane QUAD.  A launch far below one wave per
// SIMD (a small EvaluateAt call) is bound by how fast ONE chain walks its
// path, and a lone wave issues a VALU op only every ~5 clk: the ~40
// instructions of a one-lane round cost ~390 clk.  Here lane c of a quad
// holds column c of the state and computes output column c of every round
// (4 lookups, the other three columns fetched from its neighbours with DPP
// quad permutes), so a round is ~12 instructions per lane.  Same arithmetic
// as aes_core.h's encrypt: n_c = T0[b0(w_c)] ^ T1[b1(w_c+1)] ^ T2[b2(w_c+2)]
// ^ T3[b3(w_c+3)] ^ rk_c.  Every lane of a quad must be active.
// ------------------------------------------------------------------------
namespace quad {
// Lane c of a quad gets the value of lane (c + k) mod 4.
template <int K>
__device__ __forceinline__ uint32_t from_next(uint32_t v) {
  constexpr int ctrl = K == 0 ? 0xE4
                       : K == 1 ? (1 | 2 << 2 | 3 << 4 | 0 << 6)
                       : K == 2 ? (2 | 3 << 2 | 0 << 4 | 1 << 6)
                                : (3 | 0 << 2 | 1 << 4 | 2 << 6);
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xf, 0xf, false);
}
// Lane 0's value in every lane of the quad.
__device__ __forceinline__ uint32_t from_lane0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xf, 0xf, false);
}
__device__ __forceinline__ int column() { return (int)(threadIdx.x & 3); }

// Column c's word of every round key, one VGPR per round (rounds unrolled).
struct Keys {
  uint32_t k[11];
};
__device__ __forceinline__ Keys keys_of(const RoundKeys& rk) {
  Keys q;
  const int c = column();
#pragma unroll
  for (int r = 0; r < 11; ++r) q.k[r] = rk.k[4 * r + c];
  return q;
}

// sigma(x) = (x2, x3, x2 ^ x0, x3 ^ x1), column by column.
__device__ __forceinline__ uint32_t sigma(uint32_t x) {
  const uint32_t y = from_next<2>(x);
  return column() < 2 ? y : (x ^ y);
}

// DPF_QUAD_LOOKUP_FIRST=1: lane c looks up all four bytes of its OWN column
// (T0[b0(w_c)], T1[b1(w_c)], T2[b2(w_c)], T3[b3(w_c)]) and the quad permutes
// the looked-up words instead of the state: n_c = A_c ^ B_c+1 ^ C_c+2 ^ D_c+3.
// The lookups' addresses then depend on w directly (no DPP move and its
// wait states ahead of the LDS reads), and the moves fold into the XORs
// after them.  =0: permute the state, then look up (r15 first version).
#ifndef DPF_QUAD_LOOKUP_FIRST
#define DPF_QUAD_LOOKUP_FIRST 1
#endif
// from_next for a value the next instruction XORs: bound_ctrl set and no
// `old` operand, so the compiler can fold the move into that XOR as its DPP
// source (every lane of a quad_perm is valid, so bound_ctrl changes nothing).
template <int K>
__device__ __forceinline__ uint32_t xfrom_next(uint32_t v) {
  constexpr int ctrl = K == 1 ? (1 | 2 << 2 | 3 << 4 | 0 << 6)
                       : K == 2 ? (2 | 3 << 2 | 0 << 4 | 1 << 6)
                                : (3 | 0 << 2 | 1 << 4 | 2 << 6);
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, 0xf, 0xf, true);
}
// One middle round of column c; k: this column's round-key word.
__device__ __forceinline__ uint32_t round_mid(uint32_t w, const LdsLookup& lk, uint32_t k) {
#if DPF_QUAD_LOOKUP_FIRST
  const uint32_t a = lk.template lookup<0, 0>(w), b = lk.template lookup<1, 1>(w);
  const uint32_t c = lk.template lookup<2, 2>(w), d = lk.template lookup<3, 3>(w);
  return ((a ^ k) ^ xfrom_next<1>(b)) ^ xfrom_next<2>(c) ^ xfrom_next<3>(d);
#else
  const uint32_t b = from_next<1>(w), c = from_next<2>(w), d = from_next<3>(w);
  return lk.xor3(lk.xor3(lk.template lookup<0, 0>(w), lk.template lookup<1, 1>(b),
                         lk.template lookup<2, 2>(c)),
                 lk.template lookup<3, 3>(d), k);
#endif
}
// The last round of column c (SubBytes + ShiftRows), without the round key.
__device__ __forceinline__ uint32_t round_last(uint32_t w, const LdsLookup& lk) {
#if DPF_QUAD_LOOKUP_FIRST
  const uint32_t x = lk.template lookup<2, 0>(w);
  const uint32_t y = xfrom_next<1>(lk.template lookup<3, 1>(w));
  const uint32_t z = xfrom_next<2>(lk.template lookup<0, 2>(w));
  const uint32_t u = xfrom_next<3>(lk.template lookup<1, 3>(w));
#else
  const uint32_t b = from_next<1>(w), c = from_next<2>(w), d = from_next<3>(w);
  const uint32_t x = lk.template lookup<2, 0>(w), y = lk.template lookup<3, 1>(b);
  const uint32_t z = lk.template lookup<0, 2>(c), u = lk.template lookup<1, 3>(d);
#endif
  const uint32_t xy = (x & 0x000000ffu) | (y & 0xffffff00u);
  const uint32_t zu = (z & 0x00ff0000u) | (u & 0xff00ffffu);
  return (xy & 0x0000ffffu) | (zu & 0xffff0000u);
}

// AES-128 of the quad's state (this lane: column c); round key word r of
// this column = left.k[r] ^ (mask & diff.k[r]) (mask 0: left alone).
__device__ __forceinline__ uint32_t encrypt(uint32_t w, const LdsLookup& lk, const Keys& left,
                                            const Keys& diff, uint32_t mask) {
  // The round keys of this chain first (they depend on the mask only), so
  // each round ends in one XOR.
  uint32_t k[11];
#pragma unroll
  for (int r = 0; r < 11; ++r) k[r] = __builtin_amdgcn_bitop3_b32(left.k[r], mask, diff.k[r], 0x78);
  w ^= k[0];
#pragma unroll
  for (int r = 1; r < 10; ++r) w = round_mid(w, lk, k[r]);
  return round_last(w, lk) ^ k[10];
}
__device__ __forceinline__ uint32_t mmo(uint32_t x, const LdsLookup& lk, const Keys& left,
                                        const Keys& diff, uint32_t mask) {
  const uint32_t s = sigma(x);
  return encrypt(s, lk, left, diff, mask) ^ s;
}
// One path step (evaluate_prg_hwy.cc:452-486) of the quad's chain: bit,
// t, cs (this column's word of the correction seed) and cctl are
// quad-uniform.
__device__ __forceinline__ void path_step(const LdsLookup& lk, const Keys& left, const Keys& diff,
                                          uint32_t& s, uint32_t& t, uint32_t bit, uint32_t cs,
                                          uint32_t cctl) {
  uint32_t h = mmo(s, lk, left, diff, 0u - bit);
  h ^= cs & (0u - t);
  const uint32_t nt = (from_lane0(h) & 1u) ^ (t & ((cctl >> bit) & 1u));
  if (column() == 0) h &= ~1u;
  s = h;
  t = nt;
}
// Two chains of the quad interleaved round by round: `a` with keys ka, `b`
// with kb ^ (mask & kd) (DCF: a level's value hash beside its path step).
__device__ __forceinline__ void encrypt2(uint32_t& a, uint32_t& b, const LdsLookup& lk,
                                         const Keys& ka, const Keys& kb, const Keys& kd,
                                         uint32_t mask) {
  uint32_t k[11];
#pragma unroll
  for (int r = 0; r < 11; ++r) k[r] = __builtin_amdgcn_bitop3_b32(kb.k[r], mask, kd.k[r], 0x78);
  a ^= ka.k[0];
  b ^= k[0];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    const uint32_t na = round_mid(a, lk, ka.k[r]), nb = round_mid(b, lk, k[r]);
    a = na;
    b = nb;
  }
  a = round_last(a, lk) ^ ka.k[10];
  b = round_last(b, lk) ^ k[10];
}
// The quad's four columns in every lane, as a block (lane 0: in order).
__device__ __forceinline__ Block4 gather(uint32_t w) {
  return Block4{w, from_next<1>(w), from_next<2>(w), from_next<3>(w)};
}
// Both children of the quad's node (children_step above, one column per
// lane): the left and right hashes interleaved round by round.
__device__ __forceinline__ void children(const LdsLookup& lk, const Keys& left, const Keys& diff,
                                         uint32_t s, uint32_t t, uint32_t cs, uint32_t cctl,
                                         uint32_t& c0, uint32_t& t0, uint32_t& c1, uint32_t& t1) {
  const uint32_t x = sigma(s);
  uint32_t a = x, b = x;
  encrypt2(a, b, lk, left, left, diff, ~0u);
  const uint32_t m = cs & (0u - t);
  a ^= x ^ m;
  b ^= x ^ m;
  t0 = (from_lane0(a) & 1u) ^ (t & (cctl & 1u));
  t1 = (from_lane0(b) & 1u) ^ (t & ((cctl >> 1) & 1u));
  if (column() == 0) {
    a &= ~1u;
    b &= ~1u;
  }
  c0 = a;
  c1 = b;
}
// The value hashes of two seeds (mmo with the value key), interleaved.
__device__ __forceinline__ void hash2(const LdsLookup& lk, const Keys& value, uint32_t& a,
                                      uint32_t& b) {
  const uint32_t xa = sigma(a), xb = sigma(b);
  a = xa;
  b = xb;
  encrypt2(a, b, lk, value, value, value, 0u);
  a ^= xa;
  b ^= xb;
}
}  // namespace quad

// Path bit `pos` of a 128-bit path.
__device__ __forceinline__ uint32_t path_bit(Block4 p, int pos) {
  uint32_t w = pos < 32 ? p.w0 : pos < 64 ? p.w1 : pos < 96 ? p.w2 : p.w3;
  return (w >> (pos & 31)) & 1u;
}

// Two path steps with per-lane directions, interleaved (evaluate_prg_hwy.cc:452-486).
__device__ __forceinline__ void path_step2(const LdsLookup& lk, KeyRef rkl,
                                           KeyRef rkd, Block4& s0, uint32_t& t0,
                                           uint32_t b0, Block4& s1, uint32_t& t1, uint32_t b1,
                                           uint4 cs, uint32_t cctl) {
  Block4 h0 = s0, h1 = s1;
  dpf_aes::mmo_hash2(h0, h1, lk, SelectRK{rkl, rkd, 0u - b0}, SelectRK{rkl, rkd, 0u - b1});
  uint32_t m0 = 0u - t0, m1 = 0u - t1;
  h0.w0 ^= cs.x & m0; h0.w1 ^= cs.y & m0; h0.w2 ^= cs.z & m0; h0.w3 ^= cs.w & m0;
  h1.w0 ^= cs.x & m1; h1.w1 ^= cs.y & m1; h1.w2 ^= cs.z & m1; h1.w3 ^= cs.w & m1;
  uint32_t n0 = (h0.w0 & 1u) ^ (t0 & ((cctl >> b0) & 1u));
  uint32_t n1 = (h1.w0 & 1u) ^ (t1 & ((cctl >> b1) & 1u));
  h0.w0 &= ~1u;
  h1.w0 &= ~1u;
  s0 = h0; t0 = n0;
  s1 = h1; t1 = n1;
}


// Element `bi` of a directly converted integer block, corrected and negated
// (distributed_point_function.h:993-1002; value_type_helpers.h:199-211).
template <int BITS>
__device__ __forceinline__ u128 fast_point_value(Block4 h, uint32_t t, int bi, u128 cv, int party,
                                                 int xor_mode) {
  u128 x = block_u128(h);
  if (BITS < 128) x >>= (bi * BITS) & 127;
  if (xor_mode) {
    if (t) x ^= cv;
  } else {
    if (t) x += cv;
    if (party == 1) x = 0 - x;
  }
  if (BITS < 128) x &= (((u128)1 << (BITS & 127)) - 1);
  return x;
}

template <int BITS>
__device__ __forceinline__ void store_bits(char* o, u128 x) {
  if (BITS == 128) {
    *reinterpret_cast<uint4*>(o) = make_uint4((uint32_t)x, (uint32_t)(x >> 32),
                                              (uint32_t)(x >> 64), (uint32_t)(x >> 96));
  } else if (BITS == 64) {
    *reinterpret_cast<uint64_t*>(o) = (uint64_t)x;
  } else if (BITS == 32) {
    *reinterpret_cast<uint32_t*>(o) = (uint32_t)x;
  } else if (BITS == 16) {
    *reinterpret_cast<uint16_t*>(o) = (uint16_t)x;
  } else {
    *reinterpret_cast<uint8_t*>(o) = (uint8_t)x;
  }
}

// Adds v to a 192-bit little-endian accumulator held in three u64 words.
// Exact under any interleaving of concurrent adders: each word's carry-out is
// derived from the value the atomic returned.
__device__ __forceinline__ void wide_add(unsigned long long* w, u128 v) {
  unsigned long long lo = (unsigned long long)v, hi = (unsigned long long)(v >> 64);
  unsigned long long old = atomicAdd(w, lo);
  unsigned long long c = (old + lo) < old ? 1ull : 0ull;
  unsigned long long h = hi + c;
  unsigned long long c2 = (h < hi) ? 1ull : 0ull;
  if (h) {
    unsigned long long old2 = atomicAdd(w + 1, h);
    c2 += (old2 + h) < old2 ? 1ull : 0ull;
  }
  if (c2) atomicAdd(w + 2, c2);
}
__device__ __forceinline__ void wide_xor(unsigned long long* w, u128 v) {
  atomicXor(w, (unsigned long long)v);
  atomicXor(w + 1, (unsigned long long)(v >> 64));
}

// Packed-element conversion for the generic path: element `e` of the hashed
// leaf, corrected and negated, as per-leaf values.
__device__ void generic_point_values(const GenericLeaf& g, const LdsLookup& lk, KeyRef rkv,
                                     Block4 seed, uint32_t t, int e, const dpf_block* vcw,
                                     int party, u128* vals) {
  char buf[16 * DPF_MAX_LEAVES];
  GenericLeaf lf = g;
  lf.vcw = vcw;
  lf.party = party;
  lf.convert_store(lk, rkv, seed, t, e, 1, buf);
  int off = 0;
  for (int k = 0; k < g.d.num_leaves; ++k) {
    int lb = g.d.bits[k] >> 3;
    vals[k] = GenericLeaf::load_le(reinterpret_cast<const uint8_t*>(buf) + off, lb);
    off += lb;
  }
}

__device__ __forceinline__ u128 leaf_group_add(const dpf_value_desc& d, int k, u128 a, u128 b) {
  if (d.kind[k] == DPF_LEAF_XOR) return a ^ b;
  if (d.kind[k] == DPF_LEAF_INTMODN) {
    u128 n = ((u128)d.mod_high[k] << 64) | d.mod_low[k], c = n - b;
    return a >= c ? a - c : n - c + a;
  }
  u128 m = d.bits[k] >= 128 ? ~(u128)0 : (((u128)1 << d.bits[k]) - 1);
  return (a + b) & m;
}


// Round keys of (a ^ b), for the per-lane key select of path steps.
inline RoundKeys xor_keys(const RoundKeys& a, const RoundKeys& b) {
  RoundKeys r;
  for (int i = 0; i < 44; ++i) r.k[i] = a.k[i] ^ b.k[i];
  return r;
}

// Turns the 192-bit exact per-leaf sums into group elements and packs them:
// plain integers keep the low `bits`, XorWrapper is already reduced, IntModN
// takes the sum mod N (int_mod_n.h:116-120).
// `words` = 3: [point][leaf][3] 192-bit sums; 1: one uint64 per [point][leaf]
// (hh_keys_kernel, whose sums of < 2^32 values over <= 2^31 keys fit).
__global__ void finalize_sums_kernel(int64_t num_points, dpf_value_desc d,
                                     const unsigned long long* __restrict__ wide,
                                     char* __restrict__ out, int words) {
  const int nl = d.num_leaves;
  int esz = 0;
  for (int k = 0; k < nl; ++k) esz += d.bits[k] >> 3;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < num_points;
       i += (int64_t)gridDim.x * blockDim.x) {
    char* o = out + i * esz;
    for (int k = 0; k < nl; ++k) {
      const unsigned long long* w = wide + (i * nl + k) * words;
      const unsigned long long w2 = words == 3 ? w[2] : 0ull;
      u128 v = words == 3 ? (((u128)w[1] << 64) | w[0]) : (u128)w[0];
      if (d.kind[k] == DPF_LEAF_INTMODN) {
        const u128 n = ((u128)d.mod_high[k] << 64) | d.mod_low[k];
        // r = (w2 * 2^128 + v) mod n, one bit at a time (r < n throughout).
        u128 r = 0;
        for (int b = 191; b >= 0; --b) {
          const unsigned bit = b >= 128 ? (unsigned)((w2 >> (b - 128)) & 1)
                                        : (unsigned)((v >> b) & 1);
          r = (r >= n - r) ? r - (n - r) : r + r;  // 2r mod n
          if (bit) r = (r >= n - 1) ? 0 : r + 1;   // +1 mod n
        }
        v = r;
      }
      const int lb = d.bits[k] >> 3;
      for (int b = 0; b < lb; ++b) { o[b] = (char)(uint8_t)v; v >>= 8; }
      o += lb;
    }
  }
}

}  // namespace
