// dpf_batch.hip -- incremental (hierarchical) evaluation of a KEY BATCH at
// shared prefixes: SURVEY.md config 5b (2^20 heavy-hitters client keys, 61
// levels) and the device-resident EvaluationContext of section 8f.1.
//
// One call evaluates, for every key k of a batch and every start node u, what
// EvaluateUntil (distributed_point_function.h:641-837) computes for the prefix
// that start node stands for:
//   1. ComputePartialEvaluations (distributed_point_function.cc:351-453): start
//      from key k's partial evaluation seeds_in[k][parent[u]] (or its root),
//      walk `walk_levels` tree levels along path[u] (EvaluateSeeds,
//      evaluate_prg_hwy.cc:452-486) and, after `save_after` of them, store the
//      node as key k's new partial evaluation seeds_out[k][save_index[u]];
//   2. ExpandSeeds (cc:271-349) of the `expand_levels` levels below it, held in
//      VGPRs (at most 8 nodes);
//   3. HashExpandedSeeds (cc:500-524), ConvertBytesToArrayOf
//      (value_type_helpers.h:526-589), value correction and party negation
//      (h:785-808) of every leaf;
//   4. either stores the corrected elements per key, or sums them over the keys
//      in the value type's group (the per-prefix share aggregation of the
//      heavy-hitters protocol).
//
// Work decomposition: lanes of a wavefront are 64 consecutive start nodes of
// ONE key chunk, so the key index is wave-uniform -- correction words, value
// corrections and the party bit are scalar loads -- and a lane loops over the
// keys of its chunk.  Seeds are stored key-major ([k][slot]) so the lanes'
// loads and stores of one key are contiguous.  Keys are walked in pairs (two
// interleaved AES chains); expansion and leaf hashing are pairs of siblings.
// In sum mode each lane accumulates its leaves' values over the chunk in
// registers, then adds them once into exact 192-bit per-element sums.
// No last-round scheduling fence in this TU (aes_core.h, encryptN): the
// heavy-hitters kernel measured 0.35% slower with it (24.26 vs 24.18 s per pass).
#ifndef DPF_LAST_ROUND_FENCE
#define DPF_LAST_ROUND_FENCE 1024
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <vector>

#include "../../../include/dpf_hip.h"
#include "dpf_device.h"
#include "dpf_runtime.h"

using namespace dpf_rt;

namespace {

// Which kernel the calling thread's last dpf_hip_eval_prefix_batch_cached ran
// (dpf_hip_last_batch_kernel: dispatch checks in the tests).
thread_local const char* g_last_batch_kernel = "";

struct BatchLevelParams {
  int64_t num_keys;
  int64_t num_starts;       // U
  int64_t chunk_keys;
  int64_t waves_per_chunk;  // ceil(U / 64)
  int64_t num_threads;      // num_chunks * waves_per_chunk * 64
  int64_t dyn_per_wg;       // take_chunk's per_wg (0: grid stride)
  int walk_levels;
  int save_after;           // -1: no partial evaluations are stored
  int expand_levels;        // <= kMaxExpand
  int cw_first;             // correction word of the first walk level
  int cw_stride;            // correction words per key row
  const dpf_block* key_seed;
  const uint8_t* party;
  const dpf_block* seeds_in;  // NULL: start at the key's root
  const uint8_t* ctrl_in;
  int64_t in_stride;
  const int32_t* parent;
  const dpf_block* path;
  const int32_t* save_index;
  dpf_block* seeds_out;
  uint8_t* ctrl_out;
  int64_t out_stride;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  const dpf_block* vcw;
  int vcw_stride;           // E * num_leaves
  int E;                    // elements per block
  int epl;                  // corrected elements kept per tree leaf
  int esz;                  // packed element size
  int nl;                   // leaves per element
  int64_t out_row;          // STORE: bytes per key row
  char* out;
  unsigned long long* wide;  // SUM: [slot][leaf][3]
  // Expansion cache (optional): every tree leaf of this call, [key][u << E + l],
  // the start nodes of the next level's call (no path re-derivation).  A
  // non-root node's seed has bit 0 clear (distributed_point_function.cc:
  // 323-343), so the cache keeps the control bit there: one 16-byte store.
  dpf_block* leaf_seeds;
  int64_t leaf_stride;
  const int32_t* leaf_slot;   // NULL: leaf l of start node u at slot (u << E) + l
  // Layout of seeds_in / ctrl_in, seeds_out / ctrl_out and leaf_seeds:
  // 0 = key-major (element (k, j) at k * stride + j), 1 = index-major (at
  // j * num_keys + k, the device batch context's layout).
  int index_major;
  RoundKeys rkl, rkr, rkd, rkv;
};

// Element (key k, slot j) of a per-key table with `stride` slots per key.
__device__ __forceinline__ int64_t tab_at(const BatchLevelParams& p, int64_t k, int64_t j,
                                          int64_t stride) {
  return p.index_major ? j * p.num_keys + k : k * stride + j;
}

__device__ __forceinline__ uint4 cw_block(const dpf_block* p) {
  const dpf_block c = *p;
  return make_uint4((uint32_t)c.low, (uint32_t)(c.low >> 32), (uint32_t)c.high,
                    (uint32_t)(c.high >> 32));
}

// Two path steps of two different keys (own correction words), interleaved.
__device__ __forceinline__ void path_step2k(const LdsLookup& lk, KeyRef rkl,
                                            KeyRef rkd, Block4& s0, uint32_t& t0,
                                            uint4 cs0, uint32_t cc0, Block4& s1, uint32_t& t1,
                                            uint4 cs1, uint32_t cc1, uint32_t bit) {
  Block4 h0 = s0, h1 = s1;
  const SelectRK rk{rkl, rkd, 0u - bit};
  dpf_aes::mmo_hash2(h0, h1, lk, rk, rk);
  uint32_t m0 = 0u - t0, m1 = 0u - t1;
  h0.w0 ^= cs0.x & m0; h0.w1 ^= cs0.y & m0; h0.w2 ^= cs0.z & m0; h0.w3 ^= cs0.w & m0;
  h1.w0 ^= cs1.x & m1; h1.w1 ^= cs1.y & m1; h1.w2 ^= cs1.z & m1; h1.w3 ^= cs1.w & m1;
  uint32_t n0 = (h0.w0 & 1u) ^ (t0 & ((cc0 >> bit) & 1u));
  uint32_t n1 = (h1.w0 & 1u) ^ (t1 & ((cc1 >> bit) & 1u));
  h0.w0 &= ~1u;
  h1.w0 &= ~1u;
  s0 = h0; t0 = n0;
  s1 = h1; t1 = n1;
}

// ---------------------------------------------------------------- leaf policies
// Each policy converts hashed tree leaves of ONE key into corrected values:
//   key(p, k)                       per-key state (value correction, party)
//   pair(lk, p, s0, t0, s1, t1, ..) two sibling leaves, hashed interleaved
//   one(lk, p, s, t, ..)            a single leaf
//   acc_add / flush / store         sum mode and store mode.

// Plain integers and XorWrapper, one block per leaf: the hashed block IS the
// element array (value_type_helpers.h:199-211); all cepb elements of a leaf
// are corrected at once as SIMD lanes of one 128-bit word.
template <int BITS>
struct FastV {
  using Val = Block4;
  int xor_mode;
  int party;
  Block4 vcw;

  __device__ __forceinline__ void key(const BatchLevelParams& p, int64_t k) {
    party = p.party[k] & 1;
    const dpf_block* c = p.vcw + k * p.vcw_stride;
    u128 packed = 0;
    for (int e = p.E - 1; e >= 0; --e) {
      u128 v = dpf_u128(c[e]);
      if (BITS < 128) {
        v &= (((u128)1 << (BITS & 127)) - 1);
        packed = (packed << (BITS & 127)) | v;
      } else {
        packed = v;
      }
    }
    vcw = Block4{(uint32_t)packed, (uint32_t)(packed >> 32), (uint32_t)(packed >> 64),
                 (uint32_t)(packed >> 96)};
  }
  __device__ __forceinline__ Block4 correct(Block4 h, uint32_t t) const {
    if (xor_mode) {
      uint32_t m = 0u - t;
      return Block4{h.w0 ^ (vcw.w0 & m), h.w1 ^ (vcw.w1 & m), h.w2 ^ (vcw.w2 & m),
                    h.w3 ^ (vcw.w3 & m)};
    }
    if (t) h = lanes_add<BITS>(h, vcw);
    if (party == 1) h = lanes_neg<BITS>(h);
    return h;
  }
  __device__ __forceinline__ void pair(const LdsLookup& lk, const BatchLevelParams& p, Block4 s0,
                                       uint32_t t0, Block4 s1, uint32_t t1, Val& v0,
                                       Val& v1) const {
    dpf_aes::mmo_hash2(s0, s1, lk, UniformRK{lk.ks.v}, UniformRK{lk.ks.v});
    v0 = correct(s0, t0);
    v1 = correct(s1, t1);
  }
  __device__ __forceinline__ void one(const LdsLookup& lk, const BatchLevelParams& p, Block4 s,
                                      uint32_t t, Val& v) const {
    v = correct(dpf_aes::mmo_hash(s, lk, UniformRK{lk.ks.v}), t);
  }
  __device__ __forceinline__ static void zero(Val& a) { a = Block4{0, 0, 0, 0}; }
  __device__ __forceinline__ void acc_add(Val& a, const Val& v) const {
    if (xor_mode)
      a = Block4{a.w0 ^ v.w0, a.w1 ^ v.w1, a.w2 ^ v.w2, a.w3 ^ v.w3};
    else
      a = lanes_add<BITS>(a, v);
  }
  // Element e of the packed accumulator into the exact per-element sum.
  __device__ __forceinline__ void flush(const BatchLevelParams& p, int64_t slot0, const Val& a) const {
    u128 x = block_u128(a);
    for (int e = 0; e < p.epl; ++e) {
      u128 v = BITS < 128 ? ((x >> ((e * BITS) & 127)) & (((u128)1 << (BITS & 127)) - 1)) : x;
      unsigned long long* w = p.wide + (slot0 + e) * 3;
      if (xor_mode) wide_xor(w, v); else wide_add(w, v);
    }
  }
  __device__ __forceinline__ void store(const LdsLookup&, const BatchLevelParams& p, char* o,
                                        const Val& v) const {
    const int bytes = p.epl * (BITS / 8);
    switch (bytes) {
      case 16: *reinterpret_cast<uint4*>(o) = make_uint4(v.w0, v.w1, v.w2, v.w3); break;
      case 8: *reinterpret_cast<uint2*>(o) = make_uint2(v.w0, v.w1); break;
      case 4: *reinterpret_cast<uint32_t*>(o) = v.w0; break;
      case 2: *reinterpret_cast<uint16_t*>(o) = (uint16_t)v.w0; break;
      case 1: *reinterpret_cast<uint8_t*>(o) = (uint8_t)v.w0; break;
      default: {
        const uint32_t w[4] = {v.w0, v.w1, v.w2, v.w3};
        for (int i = 0; i < bytes; ++i) o[i] = (char)(uint8_t)(w[i >> 2] >> (8 * (i & 3)));
      }
    }
  }
};

// Tuples of IntModN<uint32_t, N_i> (and single IntModN<uint32_t, N>): sampled
// from b hashed blocks (value_type_helpers.h:286-311, 415-443;
// int_mod_n.h:155-177): r = first 16 bytes; value_i = r mod N_i; then
// r = (r / N_i) << 32 | next 4 bytes.  Division by the invariant N_i is the
// 2-by-1 word algorithm above -- no 128-bit division loop.
template <int NLMAX, bool ILP4>
struct Mod32V {
  struct Val {
    uint32_t x[NLMAX];
  };
  int nl;
  int b;  // blocks the sampling reads: 1 (one leaf) or 2 (<= 4 leaves of 4 bytes)
  Div32 div[NLMAX];
  int party;
  uint32_t c[NLMAX];

  __device__ __forceinline__ void key(const BatchLevelParams& p, int64_t k) {
    party = p.party[k] & 1;
    const dpf_block* v = p.vcw + k * p.vcw_stride;
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) c[i] = i < nl ? (uint32_t)v[i].low : 0u;
  }
  __device__ __forceinline__ void convert(const uint32_t* w, uint32_t t, Val& out) const {
#if defined(DPF_PROBE_NO_CONVERT)
    // Probe build only (tools/): the sampling's divisions left out, so a run
    // measures what the rest of the kernel costs.  Outputs are NOT the DPF's.
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) out.x[i] = (w[i] + (t ? c[i] : 0u)) ^ (uint32_t)party;
    return;
#endif
    uint32_t blk[4] = {w[0], w[1], w[2], w[3]};
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) {
      if (i < nl) {
        uint32_t q[3];
        const uint32_t n = div[i].n;
        uint32_t r = divmod128(blk, div[i], q);
        if (t) {  // IntModN += (int_mod_n.h:116-120)
          uint32_t s = r + c[i];
          r = (s < r || s >= n) ? s - n : s;
        }
        if (party == 1) r = r == 0 ? 0u : n - r;
        out.x[i] = r;
        blk[0] = w[4 + i]; blk[1] = q[0]; blk[2] = q[1]; blk[3] = q[2];
      } else {
        out.x[i] = 0;
      }
    }
  }
  __device__ __forceinline__ void pair(const LdsLookup& lk, const BatchLevelParams& p, Block4 s0,
                                       uint32_t t0, Block4 s1, uint32_t t1, Val& v0,
                                       Val& v1) const {
    uint32_t w0[8], w1[8];
    if (ILP4 && b == 2) {
      // Both leaves' two blocks as one interleaved quadruple.
      Block4 h[4] = {s0, add_small(s0, 1u), s1, add_small(s1, 1u)};
      const UniformRK rk[4] = {UniformRK{lk.ks.v}, UniformRK{lk.ks.v}, UniformRK{lk.ks.v},
                               UniformRK{lk.ks.v}};
      dpf_aes::mmo_hashN<4>(h, lk, rk);
      w0[0] = h[0].w0; w0[1] = h[0].w1; w0[2] = h[0].w2; w0[3] = h[0].w3;
      w0[4] = h[1].w0; w0[5] = h[1].w1; w0[6] = h[1].w2; w0[7] = h[1].w3;
      w1[0] = h[2].w0; w1[1] = h[2].w1; w1[2] = h[2].w2; w1[3] = h[2].w3;
      w1[4] = h[3].w0; w1[5] = h[3].w1; w1[6] = h[3].w2; w1[7] = h[3].w3;
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (j < b) {
          Block4 h0 = add_small(s0, (uint32_t)j), h1 = add_small(s1, (uint32_t)j);
          dpf_aes::mmo_hash2(h0, h1, lk, UniformRK{lk.ks.v}, UniformRK{lk.ks.v});
          w0[4 * j] = h0.w0; w0[4 * j + 1] = h0.w1; w0[4 * j + 2] = h0.w2; w0[4 * j + 3] = h0.w3;
          w1[4 * j] = h1.w0; w1[4 * j + 1] = h1.w1; w1[4 * j + 2] = h1.w2; w1[4 * j + 3] = h1.w3;
        } else {
          w0[4 * j] = w0[4 * j + 1] = w0[4 * j + 2] = w0[4 * j + 3] = 0;
          w1[4 * j] = w1[4 * j + 1] = w1[4 * j + 2] = w1[4 * j + 3] = 0;
        }
      }
    }
    convert(w0, t0, v0);
    convert(w1, t1, v1);
  }
  __device__ __forceinline__ void one(const LdsLookup& lk, const BatchLevelParams& p, Block4 s,
                                      uint32_t t, Val& v) const {
    uint32_t w[8];
    if (b == 2) {
      Block4 h0 = s, h1 = add_small(s, 1u);
      dpf_aes::mmo_hash2(h0, h1, lk, UniformRK{lk.ks.v}, UniformRK{lk.ks.v});
      w[0] = h0.w0; w[1] = h0.w1; w[2] = h0.w2; w[3] = h0.w3;
      w[4] = h1.w0; w[5] = h1.w1; w[6] = h1.w2; w[7] = h1.w3;
    } else {
      Block4 h0 = dpf_aes::mmo_hash(s, lk, UniformRK{lk.ks.v});
      w[0] = h0.w0; w[1] = h0.w1; w[2] = h0.w2; w[3] = h0.w3;
      w[4] = w[5] = w[6] = w[7] = 0;
    }
    convert(w, t, v);
  }
  __device__ __forceinline__ static void zero(Val& a) {
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) a.x[i] = 0;
  }
  __device__ __forceinline__ void acc_add(Val& a, const Val& v) const {
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) {
      if (i < nl) {
        uint32_t s = a.x[i] + v.x[i];
        a.x[i] = (s < a.x[i] || s >= div[i].n) ? s - div[i].n : s;
      }
    }
  }
  __device__ __forceinline__ void flush(const BatchLevelParams& p, int64_t slot0, const Val& a) const {
#pragma unroll
    for (int i = 0; i < NLMAX; ++i)
      if (i < nl && a.x[i]) wide_add(p.wide + (slot0 * nl + i) * 3, (u128)a.x[i]);
  }
  __device__ __forceinline__ void store(const LdsLookup&, const BatchLevelParams& p, char* o,
                                        const Val& v) const {
#pragma unroll
    for (int i = 0; i < NLMAX; ++i)
      if (i < nl) *reinterpret_cast<uint32_t*>(o + 4 * i) = v.x[i];
  }
};

// Any other value type (store mode only): the descriptor-driven conversion of
// the full-domain path (GenericLeaf::convert_store hashes the leaf itself).
struct GenericV {
  struct Val {
    Block4 s;
    uint32_t t;
  };
  GenericLeaf g;

  __device__ __forceinline__ void key(const BatchLevelParams& p, int64_t k) {
    g.party = p.party[k] & 1;
    g.vcw = p.vcw + k * p.vcw_stride;
  }
  __device__ __forceinline__ void pair(const LdsLookup&, const BatchLevelParams&, Block4 s0,
                                       uint32_t t0, Block4 s1, uint32_t t1, Val& v0,
                                       Val& v1) const {
    v0 = Val{s0, t0};
    v1 = Val{s1, t1};
  }
  __device__ __forceinline__ void one(const LdsLookup&, const BatchLevelParams&, Block4 s,
                                      uint32_t t, Val& v) const {
    v = Val{s, t};
  }
  __device__ __forceinline__ static void zero(Val& a) { a = Val{Block4{0, 0, 0, 0}, 0}; }
  __device__ __forceinline__ void acc_add(Val&, const Val&) const {}
  __device__ __forceinline__ void flush(const BatchLevelParams&, int64_t, const Val&) const {}
  __device__ __forceinline__ void store(const LdsLookup& lk, const BatchLevelParams& p, char* o,
                                        const Val& v) const {
    g.convert_store(lk, lk.ks.v, v.s, v.t, 0, p.epl, o);
  }
};

// --------------------------------------------------------------------- kernel

// Expands `node` by p.expand_levels levels in registers (children 2i, 2i+1 of
// node i, distributed_point_function.cc:324-330), then converts every leaf.
// `sink(l, val)` receives leaf l's value (sum or store).
template <int MAXE, class V, class Sink>
__device__ __forceinline__ void expand_and_convert(const LdsLookup& lk, const BatchLevelParams& p,
                                                   const V& v, int64_t k, Block4 node,
                                                   uint32_t t, bool store_leaves,
                                                   int64_t leaf_first, Sink&& sink) {
  Block4 N[1 << MAXE];
  uint32_t T = 0;  // bit i = control bit of N[i]
  N[0] = node;
  T = t & 1u;
  const int E = p.expand_levels;
  const dpf_block* cws = p.cw_seed + k * p.cw_stride + p.cw_first + p.walk_levels;
  const uint8_t* cl = p.cw_left + k * p.cw_stride + p.cw_first + p.walk_levels;
  const uint8_t* cr = p.cw_right + k * p.cw_stride + p.cw_first + p.walk_levels;
#pragma unroll
  for (int d = 0; d < MAXE; ++d) {
    if (d < E) {
      const uint4 cs = cw_block(cws + d);
      const uint32_t cc = (uint32_t)(cl[d] & 1) | ((uint32_t)(cr[d] & 1) << 1);
      if (d == 0) {
        Block4 c0, c1;
        uint32_t t0, t1;
        children_step(lk, lk.ks.l, lk.ks.r, N[0], T & 1u, cs, cc, c0, t0, c1, t1);
        N[0] = c0;
        N[1] = c1;
        T = t0 | (t1 << 1);
      } else {
        // Nodes i and i - 1 together (ILP4); descending i never overwrites an
        // unread node.
#pragma unroll
        for (int i = (1 << d) - 1; i >= 1; i -= 2) {
          Block4 c[4];
          uint32_t t[4];
          children_step_x2(lk, lk.ks.l, lk.ks.r, N[i], (T >> i) & 1u, N[i - 1], (T >> (i - 1)) & 1u,
                           cs, cc, c, t);
          N[2 * i] = c[0];
          N[2 * i + 1] = c[1];
          N[2 * i - 2] = c[2];
          N[2 * i - 1] = c[3];
          T = (T & ~(15u << (2 * i - 2))) | (t[2] << (2 * i - 2)) | (t[3] << (2 * i - 1)) |
              (t[0] << (2 * i)) | (t[1] << (2 * i + 1));
        }
      }
    }
  }
  // The expansion cache: this start node's 2^E leaves (node and control bit),
  // 2^E consecutive entries per lane.
  // With a slot table (the cache rewritten in place, permuted) leaf i goes
  // to its own slot; this thread has already read every cache entry it reads.
  if (store_leaves) {
#pragma unroll
    for (int i = 0; i < (1 << MAXE); ++i) {
      if (i < (1 << E)) {
        Block4 c = N[i];
        c.w0 |= (T >> i) & 1u;
        const int64_t slot = p.leaf_slot ? p.leaf_slot[leaf_first + i] : leaf_first + i;
        store_block(p.leaf_seeds + tab_at(p, k, slot, p.leaf_stride), c);
      }
    }
  }
  if (E == 0) {
    typename V::Val val;
    v.one(lk, p, N[0], T & 1u, val);
    sink(0, val);
    return;
  }
#pragma unroll
  for (int i = 0; i < (1 << MAXE); i += 2) {
    if (i < (1 << E)) {
      typename V::Val a, b;
      v.pair(lk, p, N[i], (T >> i) & 1u, N[i + 1], (T >> (i + 1)) & 1u, a, b);
      sink(i, a);
      sink(i + 1, b);
    }
  }
}

template <class V, int MAXE, bool SUM>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void batch_level_kernel(
    BatchLevelParams p, V v) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h)
  fill_tables(lds.tab);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const LdsLookup lk = make_lookup(
      lds, KeySet{key_ref(p.rkl), key_ref(p.rkr), key_ref(p.rkv), key_ref(p.rkd)});
  const int64_t U = p.num_starts;
  const int W = p.walk_levels;
  const int NL = 1 << p.expand_levels;
  // Wave tasks (key chunk x 64 start nodes) by grid stride, or taken one at a
  // time per wave (dyn_per_wg > 0).
  const int64_t tasks = p.num_threads >> 6;
  for (int64_t g = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, tasks, p.num_threads)
                                : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       g < p.num_threads;
       g = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, tasks, p.num_threads)
                        : g + (int64_t)gridDim.x * blockDim.x) {
    const int64_t wave = g >> 6;
    const int64_t chunk = (int64_t)__builtin_amdgcn_readfirstlane((int)(wave / p.waves_per_chunk));
    const int64_t u_raw = (wave - chunk * p.waves_per_chunk) * 64 + (g & 63);
    const bool valid = u_raw < U;
    const int64_t u = valid ? u_raw : U - 1;
    const int64_t k_begin = chunk * p.chunk_keys;
    const int64_t k_end = k_begin + p.chunk_keys < p.num_keys ? k_begin + p.chunk_keys : p.num_keys;
    const Block4 path = W > 0 ? load_block(p.path + u) : Block4{0, 0, 0, 0};
    const int32_t par = p.seeds_in ? p.parent[u] : 0;
    const int32_t save = (p.save_after >= 0 && p.seeds_out)
                             ? (p.save_index ? p.save_index[u] : (int32_t)u) : -1;
    typename V::Val acc[1 << MAXE];
#pragma unroll
    for (int i = 0; i < (1 << MAXE); ++i) V::zero(acc[i]);
    for (int64_t ka = k_begin; ka < k_end; ka += 2) {
      const bool has_b = ka + 1 < k_end;
      const int64_t kb = has_b ? ka + 1 : ka;
      Block4 sa, sb;
      uint32_t ta, tb;
      if (p.seeds_in) {
        const int64_t ia = tab_at(p, ka, par, p.in_stride), ib = tab_at(p, kb, par, p.in_stride);
        sa = load_block(p.seeds_in + ia);
        sb = load_block(p.seeds_in + ib);
        if (p.ctrl_in) {
          ta = p.ctrl_in[ia] & 1u;
          tb = p.ctrl_in[ib] & 1u;
        } else {
          // Expansion cache layout: the control bit rides in bit 0 of the seed.
          ta = sa.w0 & 1u;
          tb = sb.w0 & 1u;
          sa.w0 &= ~1u;
          sb.w0 &= ~1u;
        }
      } else {
        sa = load_block(p.key_seed + ka);
        ta = p.party[ka] & 1u;
        sb = load_block(p.key_seed + kb);
        tb = p.party[kb] & 1u;
      }
      // 1. path walk of both keys (ComputePartialEvaluations), saving the
      //    partial evaluation after save_after levels.
      const dpf_block* ca = p.cw_seed + ka * p.cw_stride + p.cw_first;
      const dpf_block* cb = p.cw_seed + kb * p.cw_stride + p.cw_first;
      const uint8_t* la = p.cw_left + ka * p.cw_stride + p.cw_first;
      const uint8_t* lb = p.cw_left + kb * p.cw_stride + p.cw_first;
      const uint8_t* ra = p.cw_right + ka * p.cw_stride + p.cw_first;
      const uint8_t* rb = p.cw_right + kb * p.cw_stride + p.cw_first;
      for (int j = 0; j <= W; ++j) {
        if (j == p.save_after && save >= 0 && valid) {
          const int64_t oa = tab_at(p, ka, save, p.out_stride);
          store_block(p.seeds_out + oa, sa);
          p.ctrl_out[oa] = (uint8_t)ta;
          if (has_b) {
            const int64_t ob = tab_at(p, kb, save, p.out_stride);
            store_block(p.seeds_out + ob, sb);
            p.ctrl_out[ob] = (uint8_t)tb;
          }
        }
        if (j == W) break;
        const uint32_t bit = path_bit(path, W - 1 - j);
        const uint32_t cca = (uint32_t)(la[j] & 1) | ((uint32_t)(ra[j] & 1) << 1);
        const uint32_t ccb = (uint32_t)(lb[j] & 1) | ((uint32_t)(rb[j] & 1) << 1);
        path_step2k(lk, lk.ks.l, lk.ks.d, sa, ta, cw_block(ca + j), cca, sb, tb, cw_block(cb + j), ccb,
                    bit);
      }
      // 2.-4. expansion, conversion and sum/store, one key at a time.
      for (int which = 0; which < 2; ++which) {
        if (which == 1 && !has_b) break;
        const int64_t k = which ? kb : ka;
        V vk = v;
        vk.key(p, k);
        const Block4 node = which ? sb : sa;
        const uint32_t tn = which ? tb : ta;
        const bool store_leaves = p.leaf_seeds && valid;
        const int64_t leaf_first = u << p.expand_levels;
        if constexpr (SUM) {
          expand_and_convert<MAXE>(lk, p, vk, k, node, tn, store_leaves, leaf_first,
                                   [&](int l, const typename V::Val& val) {
#pragma unroll
            for (int i = 0; i < (1 << MAXE); ++i)
              if (i == l) vk.acc_add(acc[i], val);
          });
        } else {
          char* row = p.out + k * p.out_row + (u << p.expand_levels) * (int64_t)p.epl * p.esz;
          expand_and_convert<MAXE>(lk, p, vk, k, node, tn, store_leaves, leaf_first,
                                   [&](int l, const typename V::Val& val) {
            if (valid) vk.store(lk, p, row + (int64_t)l * p.epl * p.esz, val);
          });
        }
      }
    }
    if constexpr (SUM) {
      if (valid && k_begin < k_end) {
        V vf = v;
        for (int i = 0; i < (1 << MAXE); ++i)
          if (i < NL) vf.flush(p, ((u << p.expand_levels) + i) * (int64_t)p.epl, acc[i]);
      }
    }
  }
}

}  // namespace

namespace {

// out[j] = group sum over rows r of in[r][j] (packed elements; integers mod
// 2^bits, IntModN mod N, XorWrapper by XOR -- tuple leaves element-wise).
__global__ void sum_rows_kernel(int64_t rows, int64_t row_len, dpf_value_desc d,
                                const char* __restrict__ in, char* __restrict__ out) {
  const int nl = d.num_leaves;
  int esz = 0;
  for (int k = 0; k < nl; ++k) esz += d.bits[k] >> 3;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < row_len;
       j += (int64_t)gridDim.x * blockDim.x) {
    u128 acc[DPF_MAX_LEAVES];
    for (int k = 0; k < nl; ++k) acc[k] = 0;
    for (int64_t r = 0; r < rows; ++r) {
      const uint8_t* p = reinterpret_cast<const uint8_t*>(in + (r * row_len + j) * esz);
      for (int k = 0; k < nl; ++k) {
        const int lb = d.bits[k] >> 3;
        acc[k] = leaf_group_add(d, k, acc[k], GenericLeaf::load_le(p, lb));
        p += lb;
      }
    }
    char* o = out + j * esz;
    for (int k = 0; k < nl; ++k) {
      const int lb = d.bits[k] >> 3;
      GenericLeaf::store_le(o, acc[k], lb);
      o += lb;
    }
  }
}

// Start seeds of a call from the previous call's expansion cache:
// seeds_out[k*T + i] = cache[k*cache_stride + slot[i]] (and the control bits);
// index_major: seeds_out[i*keys + k] = cache[slot[i]*keys + k].
__global__ void gather_seeds_kernel(int64_t keys, int64_t T, const int64_t* __restrict__ slot,
                                    const dpf_block* __restrict__ cache, int64_t cache_stride,
                                    dpf_block* __restrict__ seeds_out,
                                    uint8_t* __restrict__ ctrl_out, int keys_per_lane) {
  // blockIdx.y walks the keys, blockIdx.x the rows: no division per element.
  // Up to four keys' loads are issued before their stores (the scattered
  // 16-byte reads are latency-bound at one load in flight per lane).
  constexpr int kKeys = 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < T;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t si = slot[i];
    for (int64_t k0 = blockIdx.y; k0 < keys; k0 += (int64_t)gridDim.y * keys_per_lane) {
      Block4 c[kKeys];
#pragma unroll
      for (int j = 0; j < kKeys; ++j) {
        const int64_t k = k0 + j * (int64_t)gridDim.y;
        if (j < keys_per_lane && k < keys) c[j] = load_block(cache + k * cache_stride + si);
      }
#pragma unroll
      for (int j = 0; j < kKeys; ++j) {
        const int64_t k = k0 + j * (int64_t)gridDim.y;
        if (j < keys_per_lane && k < keys) {
          ctrl_out[k * T + i] = (uint8_t)(c[j].w0 & 1u);
          c[j].w0 &= ~1u;
          store_block(seeds_out + k * T + i, c[j]);
        }
      }
    }
  }
}

// Index-major form of gather_seeds_kernel: thread = one (row i, key k) pair
// with k fastest, so a wave reads one 1 KiB run of cache row slot[i] and
// writes one 1 KiB run of output row i.
__global__ void gather_seeds_im_kernel(int64_t keys, int64_t T, const int64_t* __restrict__ slot,
                                       const dpf_block* __restrict__ cache,
                                       dpf_block* __restrict__ seeds_out,
                                       uint8_t* __restrict__ ctrl_out) {
  const int64_t total = keys * T;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = x / keys, k = x - i * keys;
    Block4 c = load_block(cache + slot[i] * keys + k);
    ctrl_out[x] = (uint8_t)(c.w0 & 1u);
    c.w0 &= ~1u;
    store_block(seeds_out + x, c);
  }
}

// out[k][i*count + j] = in[k*in_row + src[i] + j], elements of elem_size bytes.
__global__ void gather_batched_kernel(int64_t keys, int64_t in_row, int64_t rows, int64_t count,
                                      int elem_size, const int64_t* __restrict__ src,
                                      const char* __restrict__ in, char* __restrict__ out) {
  const int64_t row_bytes = count * elem_size;
  const int64_t key_bytes = rows * row_bytes;
  const int64_t total = keys * key_bytes;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i / key_bytes, rem = i - k * key_bytes;
    const int64_t r = rem / row_bytes, c = rem - r * row_bytes;
    out[i] = in[(k * in_row + src[r]) * elem_size + c];
  }
}

template <class V, int MAXE, bool SUM>
int launch_batch(const BatchLevelParams& p0, const V& v, hipStream_t s) {
  BatchLevelParams p = p0;
  const int blk = block_for(p.num_threads);
  const int grid = grid_for(p.num_threads, blk);
  // DPF_BATCH_DYNAMIC=0: a fixed share of wave tasks per wave (A/B hook).
  p.dyn_per_wg = dynamic_chunks_per_wg(p.num_threads, grid, blk, "DPF_BATCH_DYNAMIC");
  hipLaunchKernelGGL((batch_level_kernel<V, MAXE, SUM>), dim3(grid), dim3(blk), 0, s, p, v);
  HIP_TRY(hipGetLastError());
  return kOk;
}

template <int NLMAX, bool ILP4>
int launch_mod32(const BatchLevelParams& p, const dpf_value_desc* desc, int b, int sum,
                 hipStream_t s) {
  using V = Mod32V<NLMAX, ILP4>;
  V v;
  memset(&v, 0, sizeof(v));
  v.nl = desc->num_leaves;
  v.b = b;
  for (int k = 0; k < desc->num_leaves; ++k) v.div[k] = make_div32((uint32_t)desc->mod_low[k]);
  return sum ? launch_batch<V, 2, true>(p, v, s) : launch_batch<V, 2, false>(p, v, s);
}

template <bool SUM>
int launch_batch_fast(const BatchLevelParams& p, int bits, int xor_mode, hipStream_t s) {
  switch (bits) {
    case 8: return launch_batch<FastV<8>, 2, SUM>(p, FastV<8>{xor_mode, 0, {}}, s);
    case 16: return launch_batch<FastV<16>, 2, SUM>(p, FastV<16>{xor_mode, 0, {}}, s);
    case 32: return launch_batch<FastV<32>, 2, SUM>(p, FastV<32>{xor_mode, 0, {}}, s);
    case 64: return launch_batch<FastV<64>, 2, SUM>(p, FastV<64>{xor_mode, 0, {}}, s);
    default: return launch_batch<FastV<128>, 2, SUM>(p, FastV<128>{xor_mode, 0, {}}, s);
  }
}

}  // namespace

extern "C" {

int dpf_hip_prefix_batch_max_expand(const dpf_value_desc* desc, int sum) {
  if (!desc || validate_desc(desc) != kOk) return -1;
  int b = 0;
  if (fast_int(desc)) return 2;
  if (mod32_eligible(desc, &b)) return 2;
  return sum ? -1 : 3;
}

int dpf_hip_eval_prefix_batch(int64_t num_keys, int64_t num_starts, int walk_levels,
                              int save_after, int expand_levels, int cw_first, int cw_stride,
                              const dpf_block* key_seed, const uint8_t* party,
                              const dpf_block* seeds_in, const uint8_t* control_in,
                              int64_t in_stride, const int32_t* parent, const dpf_block* path,
                              const int32_t* save_index, dpf_block* seeds_out,
                              uint8_t* control_out, int64_t out_stride, const dpf_block* cw_seed,
                              const uint8_t* cw_left, const uint8_t* cw_right,
                              const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                              const dpf_aes_key* key_value, const dpf_value_desc* desc,
                              int elements_per_leaf, const dpf_block* value_correction, int sum,
                              uint64_t* workspace, void* out, void* stream) {
  return dpf_hip_eval_prefix_batch_cached(
      num_keys, num_starts, walk_levels, save_after, expand_levels, cw_first, cw_stride, key_seed,
      party, seeds_in, control_in, in_stride, parent, path, save_index, seeds_out, control_out,
      out_stride, cw_seed, cw_left, cw_right, key_left, key_right, key_value, desc,
      elements_per_leaf, value_correction, sum, workspace, out, nullptr, 0, stream);
}

int dpf_hip_gather_seeds(int64_t num_keys, int64_t num_rows, const int64_t* slot,
                         const dpf_block* cache, int64_t cache_stride, dpf_block* seeds_out,
                         uint8_t* control_out, void* stream) {
  return dpf_hip_gather_seeds_layout(num_keys, num_rows, slot, cache, cache_stride, seeds_out,
                                     control_out, 0, stream);
}

int dpf_hip_gather_seeds_layout(int64_t num_keys, int64_t num_rows, const int64_t* slot,
                                const dpf_block* cache, int64_t cache_stride, dpf_block* seeds_out,
                                uint8_t* control_out, int index_major, void* stream) {
  if (num_keys < 0 || num_rows < 0 || cache_stride < 0) return fail(kInvalidArgument, "bad sizes");
  const int64_t total = num_keys * num_rows;
  if (total == 0) return kOk;
  if (!slot || !cache || !seeds_out || !control_out) return fail(kInvalidArgument, "NULL pointer");
  if (index_major) {
    int64_t g = (total + 255) / 256;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(gather_seeds_im_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                       num_keys, num_rows, slot, cache, seeds_out, control_out);
    HIP_TRY(hipGetLastError());
    return kOk;
  }
  int64_t gx = (num_rows + 255) / 256;
  if (gx > 64) gx = 64;
  // DPF_BATCH_GATHER_KEYS=1|2|4 (read per call; default 4): keys per lane and
  // pass, an A/B hook.
  const char* kv = getenv("DPF_BATCH_GATHER_KEYS");
  const int kpl = kv && (kv[0] == '1' || kv[0] == '2') ? kv[0] - '0' : 4;
  const int64_t ky = (num_keys + kpl - 1) / kpl;
  int64_t gy = ky < 65535 ? ky : 65535;
  if (gx * gy > 262144) gy = (262144 + gx - 1) / gx;
  hipLaunchKernelGGL(gather_seeds_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0,
                     (hipStream_t)stream,
                     num_keys, num_rows, slot, cache, cache_stride, seeds_out, control_out, kpl);
  HIP_TRY(hipGetLastError());
  return kOk;
}

int dpf_hip_eval_prefix_batch_cached(
    int64_t num_keys, int64_t num_starts, int walk_levels, int save_after, int expand_levels,
    int cw_first, int cw_stride, const dpf_block* key_seed, const uint8_t* party,
    const dpf_block* seeds_in, const uint8_t* control_in, int64_t in_stride,
    const int32_t* parent, const dpf_block* path, const int32_t* save_index, dpf_block* seeds_out,
    uint8_t* control_out, int64_t out_stride, const dpf_block* cw_seed, const uint8_t* cw_left,
    const uint8_t* cw_right, const dpf_aes_key* key_left, const dpf_aes_key* key_right,
    const dpf_aes_key* key_value, const dpf_value_desc* desc, int elements_per_leaf,
    const dpf_block* value_correction, int sum, uint64_t* workspace, void* out,
    dpf_block* leaf_cache, int64_t leaf_stride, void* stream) {
  return dpf_hip_eval_prefix_batch_cached_slots(
      num_keys, num_starts, walk_levels, save_after, expand_levels, cw_first, cw_stride, key_seed,
      party, seeds_in, control_in, in_stride, parent, path, save_index, seeds_out, control_out,
      out_stride, cw_seed, cw_left, cw_right, key_left, key_right, key_value, desc,
      elements_per_leaf, value_correction, sum, workspace, out, leaf_cache, leaf_stride, nullptr,
      stream);
}

int dpf_hip_eval_prefix_batch_cached_slots(
    int64_t num_keys, int64_t num_starts, int walk_levels, int save_after, int expand_levels,
    int cw_first, int cw_stride, const dpf_block* key_seed, const uint8_t* party,
    const dpf_block* seeds_in, const uint8_t* control_in, int64_t in_stride,
    const int32_t* parent, const dpf_block* path, const int32_t* save_index, dpf_block* seeds_out,
    uint8_t* control_out, int64_t out_stride, const dpf_block* cw_seed, const uint8_t* cw_left,
    const uint8_t* cw_right, const dpf_aes_key* key_left, const dpf_aes_key* key_right,
    const dpf_aes_key* key_value, const dpf_value_desc* desc, int elements_per_leaf,
    const dpf_block* value_correction, int sum, uint64_t* workspace, void* out,
    dpf_block* leaf_cache, int64_t leaf_stride, const int32_t* leaf_slot, void* stream) {
  return dpf_hip_eval_prefix_batch_layout(
      num_keys, num_starts, walk_levels, save_after, expand_levels, cw_first, cw_stride, key_seed,
      party, seeds_in, control_in, in_stride, parent, path, save_index, seeds_out, control_out,
      out_stride, cw_seed, cw_left, cw_right, key_left, key_right, key_value, desc,
      elements_per_leaf, value_correction, sum, workspace, out, leaf_cache, leaf_stride, leaf_slot,
      0, stream);
}

namespace {
// DPF_HIP_CHECK_SLOTS=1 (read per call): the slot table's contract
// (include/dpf_hip.h) checked on the host before the launch -- every slot
// below leaf_stride, no slot written twice, and a slot some start node reads
// written only as a leaf of that node and only if no other node reads it.
// A table breaking it would overwrite start seeds before they are read, or
// write out of bounds.  Costs two D2H copies; a debugging aid.
int check_slot_table(int64_t num_starts, int expand_levels, const int32_t* parent,
                     const int32_t* leaf_slot, int64_t leaf_stride) {
  const int64_t U = num_starts, n = U << expand_levels;
  std::vector<int32_t> par(U), slot(n);
  HIP_TRY(hipMemcpy(par.data(), parent, U * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(slot.data(), leaf_slot, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::vector<int64_t> reader(leaf_stride, -1);   // start node reading each slot (-2: several)
  for (int64_t u = 0; u < U; ++u) {
    if (par[u] < 0 || par[u] >= leaf_stride) return fail(kInvalidArgument, "slot table: parent out of range");
    reader[par[u]] = reader[par[u]] == -1 ? u : -2;
  }
  std::vector<char> written(leaf_stride, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t v = slot[i];
    if (v < 0 || v >= leaf_stride) return fail(kInvalidArgument, "slot table: slot out of range");
    if (written[v]++) return fail(kInvalidArgument, "slot table: slot written twice");
    const int64_t r = reader[v];
    if (r == -2 || (r >= 0 && r != (i >> expand_levels)))
      return fail(kInvalidArgument, "slot table: a slot another start node reads is overwritten");
  }
  return kOk;
}
}  // namespace

int dpf_hip_eval_prefix_batch_layout(
    int64_t num_keys, int64_t num_starts, int walk_levels, int save_after, int expand_levels,
    int cw_first, int cw_stride, const dpf_block* key_seed, const uint8_t* party,
    const dpf_block* seeds_in, const uint8_t* control_in, int64_t in_stride,
    const int32_t* parent, const dpf_block* path, const int32_t* save_index, dpf_block* seeds_out,
    uint8_t* control_out, int64_t out_stride, const dpf_block* cw_seed, const uint8_t* cw_left,
    const uint8_t* cw_right, const dpf_aes_key* key_left, const dpf_aes_key* key_right,
    const dpf_aes_key* key_value, const dpf_value_desc* desc, int elements_per_leaf,
    const dpf_block* value_correction, int sum, uint64_t* workspace, void* out,
    dpf_block* leaf_cache, int64_t leaf_stride, const int32_t* leaf_slot, int index_major,
    void* stream) {
  int st = validate_desc(desc);
  if (st) return st;
  const int max_e = dpf_hip_prefix_batch_max_expand(desc, sum);
  if (max_e < 0)
    return fail(kUnimplemented, "no on-device key sum for this value type (use store mode)");
  if (num_keys < 0 || num_starts < 0 || num_starts > INT32_MAX || walk_levels < 0 ||
      expand_levels < 0 || expand_levels > max_e || save_after < -1 || save_after > walk_levels ||
      cw_first < 0 || cw_first + walk_levels + expand_levels > cw_stride ||
      walk_levels > 128 || cw_stride > 4096)
    return fail(kInvalidArgument, "level arguments out of range");
  if (elements_per_leaf < 1 || elements_per_leaf > desc->elements_per_block)
    return fail(kInvalidArgument, "elements_per_leaf must be in [1, elements_per_block]");
  hipStream_t s = (hipStream_t)stream;
  const int64_t slots = (num_starts << expand_levels) * elements_per_leaf;
  const int nl = desc->num_leaves;
  int sum_words = 3;   // hh_keys_kernel (index-major) sums into one uint64 per element
  if (sum) {
    if (!workspace || !out) return fail(kInvalidArgument, "NULL pointer");
    HIP_TRY(hipMemsetAsync(workspace, 0, (size_t)slots * nl * 3 * sizeof(uint64_t), s));
  }
  if (num_keys > 0 && num_starts > 0) {
    if (!party || !value_correction || !key_left || !key_right || !key_value ||
        (!sum && !out) || (!seeds_in && !key_seed) || (seeds_in && !parent) ||
        (walk_levels > 0 && !path) || (save_after >= 0 && (!seeds_out || !control_out)) ||
        (walk_levels + expand_levels > 0 && (!cw_seed || !cw_left || !cw_right)))
      return fail(kInvalidArgument, "NULL pointer");
    BatchLevelParams p;
    memset(&p, 0, sizeof(p));
    p.num_keys = num_keys;
    p.num_starts = num_starts;
    p.waves_per_chunk = (num_starts + 63) / 64;
    // ~4 wave tasks per wave slot, 16 when they are taken dynamically.
    const char* dyn = std::getenv("DPF_BATCH_DYNAMIC");
    const int64_t want_waves = (int64_t)num_cus() * (kBlock / 64) * (dyn && dyn[0] == '0' ? 4 : 16);
    int64_t chunks = (want_waves + p.waves_per_chunk - 1) / p.waves_per_chunk;
    if (chunks > num_keys) chunks = num_keys;
    if (chunks < 1) chunks = 1;
    p.chunk_keys = (num_keys + chunks - 1) / chunks;
    chunks = (num_keys + p.chunk_keys - 1) / p.chunk_keys;
    p.num_threads = chunks * p.waves_per_chunk * 64;
    p.walk_levels = walk_levels;
    p.save_after = save_after;
    p.expand_levels = expand_levels;
    p.cw_first = cw_first;
    p.cw_stride = cw_stride;
    p.key_seed = key_seed;
    p.party = party;
    p.seeds_in = seeds_in;
    p.ctrl_in = control_in;
    p.in_stride = in_stride;
    p.parent = parent;
    p.path = path;
    p.save_index = save_index;
    p.seeds_out = save_after >= 0 ? seeds_out : nullptr;
    p.ctrl_out = control_out;
    p.out_stride = out_stride;
    p.cw_seed = cw_seed;
    p.cw_left = cw_left;
    p.cw_right = cw_right;
    p.vcw = value_correction;
    p.vcw_stride = desc->elements_per_block * nl;
    p.E = desc->elements_per_block;
    p.epl = elements_per_leaf;
    p.esz = packed_size(desc);
    p.nl = nl;
    p.out_row = slots * p.esz;
    p.out = (char*)out;
    p.wide = reinterpret_cast<unsigned long long*>(workspace);
    p.index_major = index_major ? 1 : 0;
    if (leaf_cache) {
      if (leaf_stride < (num_starts << expand_levels))
        return fail(kInvalidArgument, "expansion cache too small");
      // In place (leaf_cache == seeds_in) only through a slot table, whose
      // contract (include/dpf_hip.h) keeps every entry's read before its write.
      const bool in_place =
          leaf_slot && leaf_cache == seeds_in && in_stride == leaf_stride && !control_in;
      if (seeds_in && !in_place &&
          (const void*)leaf_cache < (const void*)(seeds_in + num_keys * in_stride) &&
          (const void*)seeds_in < (const void*)(leaf_cache + num_keys * leaf_stride))
        return fail(kInvalidArgument, "expansion cache overlaps the start seeds");
      p.leaf_seeds = leaf_cache;
      p.leaf_stride = leaf_stride;
      p.leaf_slot = leaf_slot;
      const char* chk = getenv("DPF_HIP_CHECK_SLOTS");
      if (leaf_slot && seeds_in && chk && chk[0] == '1') {
        HIP_TRY(hipStreamSynchronize(s));
        if (int e = check_slot_table(num_starts, expand_levels, parent, leaf_slot, leaf_stride))
          return e;
      }
    }
    p.rkl = expand_key(key_left);
    p.rkr = expand_key(key_right);
    p.rkv = expand_key(key_value);
    p.rkd = xor_keys(p.rkl, p.rkr);
    int b = 0;
    // The steady state of heavy hitters (start seeds from the expansion cache
    // or a gather, no walk, two expanded levels, IntModN<uint32_t> sums): the
    // lean kernel of dpf_batch_hh.hip.  DPF_BATCH_NO_LEAN=1 keeps the general
    // kernel (A/B and test hook).
    const char* no_lean_env = getenv("DPF_BATCH_NO_LEAN");
    const bool no_lean = no_lean_env && no_lean_env[0] == '1';
    if (sum && !no_lean && walk_levels == 0 && expand_levels == 2 && seeds_in &&
        elements_per_leaf == 1 && mod32_eligible(desc, &b) && nl <= 2 && (nl == 1 || b == 2)) {
      HHLevelArgs a;
      memset(&a, 0, sizeof(a));
      a.num_keys = num_keys;
      a.num_starts = num_starts;
      a.cw_level = cw_first;
      a.cw_stride = cw_stride;
      a.seeds_in = seeds_in;
      a.ctrl_in = control_in;
      a.in_stride = in_stride;
      a.parent = parent;
      a.save = save_after == 0 && seeds_out;
      a.save_index = save_index;
      a.seeds_out = seeds_out;
      a.ctrl_out = control_out;
      a.out_stride = out_stride;
      a.cw_seed = cw_seed;
      a.cw_left = cw_left;
      a.cw_right = cw_right;
      a.vcw = value_correction;
      a.vcw_stride = p.vcw_stride;
      a.party = party;
      a.wide = p.wide;
      a.leaf_seeds = p.leaf_seeds;
      a.leaf_stride = p.leaf_stride;
      a.leaf_slot = p.leaf_slot;
      a.nl = nl;
      a.b = b;
      a.index_major = p.index_major;
      for (int k = 0; k < nl; ++k) a.mod[k] = (uint32_t)desc->mod_low[k];
      a.key_left = key_left;
      a.key_right = key_right;
      a.key_value = key_value;
      st = launch_hh_level(a, s);
      if (a.index_major) sum_words = 1;
      g_last_batch_kernel = a.index_major ? "hh_keys" : "hh_level";
    } else if (fast_int(desc)) {
      g_last_batch_kernel = "batch_level/fast";
      const int xm = desc->kind[0] == DPF_LEAF_XOR;
      st = sum ? launch_batch_fast<true>(p, desc->bits[0], xm, s)
               : launch_batch_fast<false>(p, desc->bits[0], xm, s);
    } else if (mod32_eligible(desc, &b)) {
      // Leaf pairs hash their four blocks as one ILP4 group (r05: +0.8% over
      // two ILP2 pairs on heavy hitters); tuples of <= 2 leaves use 2-wide
      // accumulators (117 instead of 128 VGPRs).
      st = nl <= 2 ? launch_mod32<2, true>(p, desc, b, sum, s) : launch_mod32<4, true>(p, desc, b, sum, s);
      g_last_batch_kernel = "batch_level/mod32";
    } else {
      g_last_batch_kernel = "batch_level/generic";
      GenericV v;
      memset(&v, 0, sizeof(v));
      v.g.d = *desc;
      v.g.elements_per_leaf = elements_per_leaf;
      v.g.esz = p.esz;
      st = launch_batch<GenericV, 3, false>(p, v, s);
    }
    if (st) return st;
  }
  if (sum && slots > 0) {
    int64_t g = (slots + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(finalize_sums_kernel, dim3((unsigned)g), dim3(256), 0, s, slots, *desc,
                       reinterpret_cast<const unsigned long long*>(workspace), (char*)out,
                       sum_words);
    HIP_TRY(hipGetLastError());
  }
  return kOk;
}

const char* dpf_hip_last_batch_kernel(void) { return g_last_batch_kernel; }

int dpf_hip_sum_rows(int64_t num_rows, int64_t row_len, const dpf_value_desc* desc,
                     const void* in, void* out, void* stream) {
  int st = validate_desc(desc);
  if (st) return st;
  if (num_rows < 0 || row_len < 0) return fail(kInvalidArgument, "bad sizes");
  if (row_len == 0) return kOk;
  if (!out || (num_rows > 0 && !in)) return fail(kInvalidArgument, "NULL pointer");
  int64_t g = (row_len + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                     num_rows, row_len, *desc, (const char*)in, (char*)out);
  HIP_TRY(hipGetLastError());
  return kOk;
}

int dpf_hip_gather_batched(int64_t num_keys, int64_t in_row_elems, int64_t num_rows, int64_t count,
                           int elem_size, const int64_t* src_offset, const void* in, void* out,
                           void* stream) {
  if (num_keys < 0 || in_row_elems < 0 || num_rows < 0 || count < 0 || elem_size < 1)
    return fail(kInvalidArgument, "bad sizes");
  const int64_t total = num_keys * num_rows * count * elem_size;
  if (total == 0) return kOk;
  if (!src_offset || !in || !out) return fail(kInvalidArgument, "NULL pointer");
  int64_t g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(gather_batched_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                     num_keys, in_row_elems, num_rows, count, elem_size, src_offset,
                     (const char*)in, (char*)out);
  HIP_TRY(hipGetLastError());
  return kOk;
}

}  // extern "C"
