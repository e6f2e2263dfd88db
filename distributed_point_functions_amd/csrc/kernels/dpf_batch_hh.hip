// dpf_batch_hh.hip -- the heavy-hitters level of a key batch (SURVEY.md config
// 5b) in its steady state: every key's start seeds come from the previous
// call's expansion cache (no path walk), each start node is expanded two tree
// levels, its four leaves are hashed, sampled as Tuple<IntModN<uint32_t, N>...>
// / IntModN<uint32_t, N> values, corrected, and summed over the keys.  This is
// what batch_level_kernel<Mod32V, 2, true> (dpf_batch.hip) computes for
// walk_levels == 0 and expand_levels == 2 -- ExpandSeeds (distributed_point_
// function.cc:271-349) + HashExpandedSeeds (cc:500-524) + the correction loop
// (h:785-808) + the sampling of value_type_helpers.h:286-311, 415-443 -- in a
// kernel stripped to that shape: one key at a time (no second key's node held
// across the first's work), no path state, a small argument block, so the AES
// chains keep many more LDS lookups in flight at 4 waves per SIMD (r13: the
// general kernel's schedule waited on LDS every ~2 lookups, VGPR-bound).
// Built with the iterative-ilp scheduler (build_native.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/dpf_hip.h"
#include "dpf_device.h"
#include "dpf_runtime.h"

using namespace dpf_rt;

// Waves per SIMD: 4 = 1024-thread workgroups at <= 128 VGPRs (the other
// kernels' shape); 3 = 768 threads at <= 168 VGPRs (more lookups in flight
// per wave, fewer waves).
#ifndef DPF_HH_WAVES
#define DPF_HH_WAVES 4
#endif
// 1: the MMO feed-forward sigma(x) is recomputed from the leaf seed after the
// encryption instead of being held through it (8 fewer live VGPRs per leaf pair).
#ifndef DPF_HH_RESIGMA
#define DPF_HH_RESIGMA 1
#endif

// 1: the second leaf pair waits in LDS (32 B per thread beside the 128 KiB of
// tables) while the first pair is hashed, instead of in 10 VGPRs.
// DPF_HH_PREFETCH=1: the next key's start seed is loaded before this key's
// value hashes (the start seeds come from scattered rows of the expansion
// cache since the slot-table rewrite).  Measured slower (128 VGPRs; 2^20
// clients 20.68 vs 20.52 s per pass, 2^18 5.41 vs 5.33 s, profiles/r15_ab.txt
// part 17): the other 15 waves of the CU already hide the load.  Off.
#ifndef DPF_HH_PREFETCH
#define DPF_HH_PREFETCH 0
#endif
#ifndef DPF_HH_STASH
#define DPF_HH_STASH 1
#endif

namespace {

constexpr int kHHBlock = 256 * DPF_HH_WAVES;

struct HHLds {
  uint32_t tab[kTabWords];
#if DPF_HH_STASH
  uint4 stash[2][kHHBlock];  // [leaf 2 / 3][thread]: seed | control bit
#endif
};

struct HHParams {
  int64_t num_keys;
  int64_t num_starts;
  int64_t chunk_keys;
  int64_t waves_per_chunk;
  int64_t num_threads;
  int cw_level;    // correction word of the first expanded level
  int cw_stride;   // correction words per key row
  int save;        // 1: store each start node as the key's new partial evaluation
  int nl;          // tuple leaves (1 or 2)
  int b;           // value blocks hashed per leaf (1 or 2)
  const dpf_block* seeds_in;  // [k][in_stride]
  const uint8_t* ctrl_in;     // NULL: control bit in bit 0 of the seed (expansion cache)
  int64_t in_stride;
  const int32_t* parent;
  const int32_t* save_index;
  dpf_block* seeds_out;
  uint8_t* ctrl_out;
  int64_t out_stride;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  const dpf_block* vcw;
  int vcw_stride;
  const uint8_t* party;
  unsigned long long* wide;  // [start << 2 | leaf][nl][3]
  dpf_block* leaf_seeds;     // NULL: no expansion cache written
  int64_t leaf_stride;
  const int32_t* leaf_slot;  // NULL: leaf i of start node u at slot (u << 2) + i
  Div32 div[2];
  RoundKeys rkl, rkr, rkv;
  unsigned int* task_counter;  // non-NULL: waves take their 64-thread tasks from this
};

// value = sampled IntModN elements of one leaf (value_type_helpers.h:286-311):
// r0 = block mod N0; r1 = ((block / N0) << 32 | next 4 bytes) mod N1.
__device__ __forceinline__ void sample2(const HHParams& p, const Div32 (&div)[2], const Block4& h0,
                                        uint32_t w4, uint32_t out[2]) {
  const uint32_t blk[4] = {h0.w0, h0.w1, h0.w2, h0.w3};
  uint32_t q[3];
  out[0] = divmod128(blk, div[0], q);
  if (p.nl > 1) {
    const uint32_t nb[4] = {w4, q[0], q[1], q[2]};
    uint32_t q2[3];
    out[1] = divmod128(nb, div[1], q2);
  } else {
    out[1] = 0;
  }
}

// sample2 with the divisors passed directly (hh_keys_kernel).
__device__ __forceinline__ void sample2_nl(int nl, const Div32& d0, const Div32& d1,
                                           const Block4& h0, uint32_t w4, uint32_t out[2]) {
  const uint32_t blk[4] = {h0.w0, h0.w1, h0.w2, h0.w3};
  uint32_t q[3];
  out[0] = divmod128(blk, d0, q);
  if (nl > 1) {
    const uint32_t nb[4] = {w4, q[0], q[1], q[2]};
    uint32_t q2[3];
    out[1] = divmod128(nb, d1, q2);
  } else {
    out[1] = 0;
  }
}

// DPF_HH_PIN_DIV=1: wave-uniform kernel arguments copied into SGPRs by an
// instruction the compiler cannot rematerialise, so under SGPR pressure it
// spills the copy to a VGPR lane (v_writelane / v_readlane, no wait) instead
// of reloading the argument with s_load, whose lgkmcnt(0) wait drains the
// LDS lookups in flight (party / leaf_seeds / leaf_stride were reloaded 10x
// per key, r15 ISA).  Measured slower (2^20 clients 20.57 vs 20.45 s per
// pass, 2^18 5.39 / 5.37 vs 5.32 / 5.33 s; profiles/r15_ab.txt part 18): off.
#ifndef DPF_HH_PIN_DIV
#define DPF_HH_PIN_DIV 0
#endif
__device__ __forceinline__ uint32_t pin_sgpr(uint32_t x) {
#if DPF_HH_PIN_DIV
  uint32_t r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(x));
  return r;
#else
  return x;
#endif
}
__device__ __forceinline__ uint64_t pin_sgpr64(uint64_t x) {
#if DPF_HH_PIN_DIV
  uint64_t r;
  asm volatile("s_mov_b64 %0, %1" : "=s"(r) : "s"(x));
  return r;
#else
  return x;
#endif
}
template <typename T>
__device__ __forceinline__ T* pin_ptr(T* x) {
  return reinterpret_cast<T*>(pin_sgpr64(reinterpret_cast<uint64_t>(x)));
}

__device__ __forceinline__ uint32_t mod_add(uint32_t a, uint32_t b, uint32_t n) {
  const uint32_t s = a + b;
  return (s < a || s >= n) ? s - n : s;
}

// MMO hashes of two leaves' blocks x0, x0 + 1, x1, x1 + 1 (cc:500-524), ILP4.
__device__ __forceinline__ void hash_leaf_pair(const LdsLookup& lk, KeyRef rkv, Block4 x0,
                                               Block4 x1, Block4 h[4]) {
  const UniformRK rk[4] = {UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}};
#if DPF_HH_RESIGMA
  h[0] = dpf_aes::sigma(x0);
  h[1] = dpf_aes::sigma(add_small(x0, 1u));
  h[2] = dpf_aes::sigma(x1);
  h[3] = dpf_aes::sigma(add_small(x1, 1u));
  dpf_aes::encryptN<4>(h, lk, rk);
  const Block4 s[4] = {dpf_aes::sigma(x0), dpf_aes::sigma(add_small(x0, 1u)), dpf_aes::sigma(x1),
                       dpf_aes::sigma(add_small(x1, 1u))};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    h[i] = Block4{h[i].w0 ^ s[i].w0, h[i].w1 ^ s[i].w1, h[i].w2 ^ s[i].w2, h[i].w3 ^ s[i].w3};
#else
  h[0] = x0;
  h[1] = add_small(x0, 1u);
  h[2] = x1;
  h[3] = add_small(x1, 1u);
  dpf_aes::mmo_hashN<4>(h, lk, rk);
#endif
}

__global__ __launch_bounds__(kHHBlock) __attribute__((amdgpu_waves_per_eu(DPF_HH_WAVES, DPF_HH_WAVES)))
void hh_level_kernel(HHParams p) {
  __shared__ HHLds lds;
  fill_tables(lds.tab);
  __syncthreads();
  const uint32_t lt = (threadIdx.x & 31) * 4u;
  uint32_t m1;
  asm volatile("v_mov_b32 %0, 0xff00" : "=v"(m1));
  const LdsLookup lk{reinterpret_cast<const char*>(lds.tab),
                     {lt, lt + 128u, lt + 65536u, lt + 65664u}, m1,
                     KeySet{key_ref(p.rkl), key_ref(p.rkr), key_ref(p.rkv), KeyRef{}}};
  const int64_t U = p.num_starts;
  // The arguments the key loop reads every key (the s_load_dwordx8 of
  // party / wide / leaf_seeds / leaf_stride was reloaded 10x per key).
  const uint8_t* const party_p = pin_ptr(p.party);
  dpf_block* const leaf_seeds = pin_ptr(p.leaf_seeds);
  const int64_t leaf_stride = (int64_t)pin_sgpr64((uint64_t)p.leaf_stride);
  Div32 div[2];
#pragma unroll
  for (int e = 0; e < 2; ++e)
    div[e] = Div32{pin_sgpr(p.div[e].dn), pin_sgpr(p.div[e].v), (int)pin_sgpr((uint32_t)p.div[e].sh),
                   pin_sgpr(p.div[e].n)};
  // Tasks (64 threads each) by grid stride, or one at a time per wave from
  // the global counter (task_counter, as hh_keys_kernel).
  const int64_t num_tasks = p.num_threads >> 6;
  auto next = [&](int64_t g) -> int64_t {
    if (!p.task_counter) return g + (int64_t)gridDim.x * blockDim.x;
    unsigned int c = 0;
    if ((threadIdx.x & 63) == 0) c = atomicAdd(p.task_counter, 1u);
    c = __builtin_amdgcn_readfirstlane(c);
    return (int64_t)c < num_tasks ? (int64_t)c * 64 + (threadIdx.x & 63) : p.num_threads;
  };
  for (int64_t g = p.task_counter ? next(0) : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       g < p.num_threads; g = next(g)) {
    const int64_t wave = g >> 6;
    const int64_t chunk = (int64_t)__builtin_amdgcn_readfirstlane((int)(wave / p.waves_per_chunk));
    const int64_t u_raw = (wave - chunk * p.waves_per_chunk) * 64 + (g & 63);
    const bool valid = u_raw < U;
    const int64_t u = valid ? u_raw : U - 1;
    const int64_t k_begin = chunk * p.chunk_keys;
    const int64_t k_end = k_begin + p.chunk_keys < p.num_keys ? k_begin + p.chunk_keys : p.num_keys;
    const int32_t par = p.parent[u];
    const int32_t save = p.save && valid ? (p.save_index ? p.save_index[u] : (int32_t)u) : -1;
    uint32_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = 0;
    // The node's four leaf slots (the same for every key), loaded once: inside
    // the key loop the compiler reloaded them every key (the leaf stores may
    // alias the table), one more wait per key.
    int4 sl = make_int4((int)(u << 2), (int)(u << 2) + 1, (int)(u << 2) + 2, (int)(u << 2) + 3);
    if (p.leaf_slot && leaf_seeds && valid)
      sl = *reinterpret_cast<const int4*>(p.leaf_slot + (u << 2));
#if DPF_HH_PREFETCH
    Block4 s_next{};
    uint32_t c_next = 0;
    if (k_begin < k_end) {
      s_next = load_block(p.seeds_in + k_begin * p.in_stride + par);
      if (p.ctrl_in) c_next = p.ctrl_in[k_begin * p.in_stride + par];
    }
#endif
    for (int64_t k = k_begin; k < k_end; ++k) {
#if DPF_HH_PREFETCH
      Block4 s = s_next;
      const uint32_t c_in = c_next;
#else
      // Padding lanes (u clamped to U - 1) read nothing: that node's own
      // lane may be rewriting the slot in place.
      Block4 s = valid ? load_block(p.seeds_in + k * p.in_stride + par) : Block4{0, 0, 0, 0};
      const uint32_t c_in = p.ctrl_in && valid ? p.ctrl_in[k * p.in_stride + par] : 0u;
#endif
      uint32_t t;
      if (p.ctrl_in) {
        t = c_in & 1u;
      } else {
        t = s.w0 & 1u;
        s.w0 &= ~1u;
      }
      if (save >= 0) {
        store_block(p.seeds_out + k * p.out_stride + save, s);
        p.ctrl_out[k * p.out_stride + save] = (uint8_t)t;
      }
      // Two tree levels (cc:304-347): the node's children (ILP2), then both
      // children's children (ILP4); leaf order 0..3 = LL, LR, RL, RR.
      const int64_t cwi = k * p.cw_stride + p.cw_level;
      const uint4 cs0 = make_uint4((uint32_t)p.cw_seed[cwi].low, (uint32_t)(p.cw_seed[cwi].low >> 32),
                                   (uint32_t)p.cw_seed[cwi].high, (uint32_t)(p.cw_seed[cwi].high >> 32));
      const uint32_t cc0 = (uint32_t)(p.cw_left[cwi] & 1) | ((uint32_t)(p.cw_right[cwi] & 1) << 1);
      Block4 c0, c1;
      uint32_t t0, t1;
      children_step(lk, lk.ks.l, lk.ks.r, s, t, cs0, cc0, c0, t0, c1, t1);
      const uint4 cs1 = make_uint4(
          (uint32_t)p.cw_seed[cwi + 1].low, (uint32_t)(p.cw_seed[cwi + 1].low >> 32),
          (uint32_t)p.cw_seed[cwi + 1].high, (uint32_t)(p.cw_seed[cwi + 1].high >> 32));
      const uint32_t cc1 =
          (uint32_t)(p.cw_left[cwi + 1] & 1) | ((uint32_t)(p.cw_right[cwi + 1] & 1) << 1);
      Block4 L[4];
      uint32_t tl[4];
      children_step_x2(lk, lk.ks.l, lk.ks.r, c0, t0, c1, t1, cs1, cc1, L, tl);
      if (leaf_seeds && valid) {
        // A slot table places the leaves when the cache is rewritten in place:
        // leaf 0 in this node's own slot (read above by this thread), the
        // others in slots no start node reads.
        dpf_block* o = leaf_seeds + k * leaf_stride;
        const int slot[4] = {sl.x, sl.y, sl.z, sl.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          Block4 c = L[i];
          c.w0 |= tl[i];
          store_block(o + slot[i], c);
        }
      }
      // Value hashes (cc:500-524): two leaves' b blocks per ILP4 group.
      const int party = party_p[k] & 1;
      const dpf_block* vc = p.vcw + k * p.vcw_stride;
      const uint32_t corr[2] = {(uint32_t)vc[0].low, p.nl > 1 ? (uint32_t)vc[1].low : 0u};
      const UniformRK rk[4] = {UniformRK{lk.ks.v}, UniformRK{lk.ks.v}, UniformRK{lk.ks.v},
                               UniformRK{lk.ks.v}};
#if DPF_HH_PREFETCH
      {
        // In-place rewrites are safe: the next key's row is not written until
        // that key's own iteration (leaf stores go to row k only).
        const int64_t kn = k + 1 < k_end ? k + 1 : k;
        s_next = load_block(p.seeds_in + kn * p.in_stride + par);
        if (p.ctrl_in) c_next = p.ctrl_in[kn * p.in_stride + par];
      }
#endif
#if DPF_HH_STASH
      lds.stash[0][threadIdx.x] = make_uint4(L[2].w0 | tl[2], L[2].w1, L[2].w2, L[2].w3);
      lds.stash[1][threadIdx.x] = make_uint4(L[3].w0 | tl[3], L[3].w1, L[3].w2, L[3].w3);
#endif
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
#if DPF_HH_STASH
        if (pr == 1) {
          // Same thread wrote these: no barrier needed.
          const uint4 a = lds.stash[0][threadIdx.x], c = lds.stash[1][threadIdx.x];
          tl[2] = a.x & 1u;
          tl[3] = c.x & 1u;
          L[2] = Block4{a.x & ~1u, a.y, a.z, a.w};
          L[3] = Block4{c.x & ~1u, c.y, c.z, c.w};
        }
#endif
        Block4 h[4];
        if (p.b == 2) {
          hash_leaf_pair(lk, lk.ks.v, L[2 * pr], L[2 * pr + 1], h);
        } else {
          h[0] = L[2 * pr];
          h[2] = L[2 * pr + 1];
          Block4 two[2] = {h[0], h[2]};
          dpf_aes::mmo_hashN<2>(two, lk, rk);
          h[0] = two[0];
          h[2] = two[1];
          h[1] = h[3] = Block4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int leaf = 2 * pr + j;
          uint32_t v[2];
          sample2(p, div, h[2 * j], h[2 * j + 1].w0, v);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            if (e < p.nl) {
              const uint32_t n = div[e].n;
              uint32_t r = v[e];
              if (tl[leaf]) r = mod_add(r, corr[e], n);          // int_mod_n.h:116-120
              if (party == 1) r = r == 0 ? 0u : n - r;            // int_mod_n.h:208-218
              acc[leaf][e] = mod_add(acc[leaf][e], r, n);
            }
          }
        }
      }
    }
    if (valid && k_begin < k_end) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          if (e < p.nl && acc[i][e]) wide_add(p.wide + (((u << 2) + i) * p.nl + e) * 3, (u128)acc[i][e]);
    }
  }
}

// ---------------------------------------------------------------------------
// hh_keys_kernel: the same level with LANES = KEYS (r16, the default).
//
// The device batch context keeps its per-key tables index-major -- the
// expansion cache, the partial evaluations and the gathered start seeds hold
// element (key k, slot j) at j * K + k -- so one wave = 64 consecutive keys at
// ONE (wave-uniform) start node u reads its start seeds as one 1 KiB access
// and writes each of its four cache leaves and its partial evaluation as one
// 1 KiB access, whatever slots the level selected.  (hh_level_kernel, lanes =
// start nodes of one key, read 16-byte entries scattered across a 64 KiB
// key-major cache row: 4.1x read amplification, waves waiting 20% of their
// life)  The key's correction words, value correction and party
// are loaded once per wave into VGPRs and serve every start node; the wave's
// 64 keys' values of the node's 4 leaves x nl elements are summed mod N
// across the lanes by a transpose-reduction (10 lane exchanges for 8 sums)
// and added with ONE atomic instruction of 8 lanes into 64 contiguous bytes
// of uint64 sums (sums of < N < 2^32 values over <= 2^31 keys fit), reduced
// mod N by finalize_sums_kernel (words = 1).  Waves start their start-node
// loop at different nodes so the atomics of resident waves spread over the
// level's nodes.
struct HHKeysParams {
  int64_t num_keys;     // K
  int64_t num_starts;   // U
  int64_t u_ranges;     // start-node ranges per 64-key group
  int64_t u_per_range;
  int64_t num_waves;    // ceil(K / 64) * u_ranges
  unsigned int* task_counter;  // non-NULL: waves take tasks one at a time from this
                               // zeroed counter (dynamic); NULL: grid stride
  int cw_level;
  int cw_stride;
  int nl;
  int b;
  const dpf_block* seeds_in;   // [j][K]
  const uint8_t* ctrl_in;      // [j][K]; NULL: control bit in bit 0 of the seed
  const int32_t* parent;
  int save;                    // 1: store each start node as the key's partial evaluation
  const int32_t* save_index;   // NULL (with save): start node u at index u
  dpf_block* seeds_out;        // [save][K]
  uint8_t* ctrl_out;
  const dpf_block* cw_seed;    // [k][cw_stride] (the key batch's own layout)
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  const dpf_block* vcw;
  int vcw_stride;
  const uint8_t* party;
  const uint4* key_tab;        // DPF_HH_KEYS_MODE 2: [3][K], hh_key_table_kernel
  unsigned long long* sums;    // [(u << 2 | leaf) * nl + e]
  dpf_block* leaf_seeds;       // [slot][K]; NULL: no expansion cache written
  const int32_t* leaf_slot;    // NULL: leaf i of start node u at slot (u << 2) + i
  Div32 div[2];
  RoundKeys rkl, rkr, rkv;
};

// Sum over the wave's 64 lanes of eight u32 values v[i] (element i & 1: mod
// n0 or n1), in VALU lane permutes (no LDS, no address registers): three
// halving exchanges -- lanes ^ 32 (v_permlane32_swap), ^ 16
// (v_permlane16_swap), ^ 8 (DPP row_ror:8) -- after which lane L holds a
// partial sum of value L >> 3, completed over lanes ^ 4 (ds_swizzle), ^ 2 and
// ^ 1 (DPP quad_perm).  Lanes 8i return the sum of value i.  A slot's value
// index keeps the parity of the slot, so slot parity picks the modulus.
__device__ __forceinline__ uint32_t wave_sum8_mod(uint32_t v[8], uint32_t n0, uint32_t n1) {
  // The swaps exchange vdst's upper half (rows) with vsrc's lower: per lane
  // the two results are its own kept value and its partner's matching one.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(v[i], v[4 + i], false, false);
    v[i] = mod_add(r[0], r[1], (i & 1) ? n1 : n0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(v[i], v[2 + i], false, false);
    v[i] = mod_add(r[0], r[1], (i & 1) ? n1 : n0);
  }
  const bool hi8 = (threadIdx.x & 8) != 0;
  const uint32_t n = hi8 ? n1 : n0;
  const uint32_t keep = hi8 ? v[1] : v[0], give = hi8 ? v[0] : v[1];
  uint32_t x = mod_add(keep, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)give, 0x128, 0xF, 0xF, false), n);
  x = mod_add(x, (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x101F), n);        // lane ^ 4
  x = mod_add(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false), n);  // ^ 2
  x = mod_add(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false), n);  // ^ 1
  return x;
}

// Where hh_keys_kernel gets each key's two levels of correction words, its
// value correction and its party (DPF_HH_KEYS_MODE):
//   2 (default): a per-call key table built by hh_key_table_kernel, [3][K]
//     uint4 (cs0, cs1, {cc bits | party << 4, corr0, corr1}), re-read for
//     every start node next to its use as three coalesced 1 KiB loads per
//     wave (L2 hits), at 4 waves per SIMD;
//   1: loaded ONCE per wave into 11 VGPRs (135 VGPRs: 3 waves per SIMD):
//     22.8 vs 20.3 s per 2^20-client pass (profiles/r16/hh_ab.txt);
//   0: re-read for every start node straight from the key batch's
//     [key][level] rows (scattered 16-byte reads, ~60 TB of fetches per
//     2^20 pass), 4 waves per SIMD.
#ifndef DPF_HH_KEYS_MODE
#define DPF_HH_KEYS_MODE 2
#endif
#define DPF_HH_KEYS_HOIST (DPF_HH_KEYS_MODE == 1)
#ifndef DPF_HH_KEYS_WAVES
#define DPF_HH_KEYS_WAVES (DPF_HH_KEYS_HOIST ? 3 : 4)
#endif
constexpr int kHHKeysBlock = 256 * DPF_HH_KEYS_WAVES;
struct HHKeysLds {
  uint32_t tab[kTabWords];
#if DPF_HH_STASH
  uint4 stash[2][kHHKeysBlock];  // [leaf 2 / 3][thread]: seed | control bit
#endif
};

// DPF_HH_NT=1 (default): the streamed start seeds, cache leaves and partial
// evaluations are non-temporal (they are not read again within the call),
// leaving L2 to the waves' key tables: 2^20-client pass 19.03 / 19.23 /
// 19.25 vs 19.16 / 19.37 / 19.34 s with temporal accesses, three same-box
// pairs (profiles/r16/hh_nt_ab.txt).
#ifndef DPF_HH_NT
#define DPF_HH_NT 1
#endif
__device__ __forceinline__ Block4 stream_load(const dpf_block* p) {
#if DPF_HH_NT
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return Block4{v.x, v.y, v.z, v.w};
#else
  return load_block(p);
#endif
}
__device__ __forceinline__ void stream_store(dpf_block* p, Block4 b) {
#if DPF_HH_NT
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = {b.w0, b.w1, b.w2, b.w3};
  __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
#else
  store_block(p, b);
#endif
}

__device__ __forceinline__ uint4 cw_u4(const dpf_block& c) {
  return make_uint4((uint32_t)c.low, (uint32_t)(c.low >> 32), (uint32_t)c.high,
                    (uint32_t)(c.high >> 32));
}

__global__ __launch_bounds__(kHHKeysBlock)
__attribute__((amdgpu_waves_per_eu(DPF_HH_KEYS_WAVES, DPF_HH_KEYS_WAVES)))
void hh_keys_kernel(HHKeysParams p) {
  __shared__ HHKeysLds lds;
  fill_tables(lds.tab);
  __syncthreads();
  const uint32_t lt = (threadIdx.x & 31) * 4u;
  uint32_t m1;
  asm volatile("v_mov_b32 %0, 0xff00" : "=v"(m1));
  const LdsLookup lk{reinterpret_cast<const char*>(lds.tab),
                     {lt, lt + 128u, lt + 65536u, lt + 65664u}, m1,
                     KeySet{key_ref(p.rkl), key_ref(p.rkr), key_ref(p.rkv), KeyRef{}}};
  const int64_t K = p.num_keys, U = p.num_starts;
  const int lane = (int)(threadIdx.x & 63);
  const int64_t waves_per_block = kHHKeysBlock / 64;
  const int64_t wave0 = (int64_t)blockIdx.x * waves_per_block +
                        __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nl = p.nl;
  const Div32 div0 = p.div[0], div1 = p.div[1];
  // Tasks (64 keys x a range of start nodes) by grid stride, or -- with a
  // task counter -- taken one at a time in order, so the waves the CU's
  // arbiter favours take more of them and all finish together (the octet
  // kernel's items, dpf_kernels.hip; the LDS here is full, so the counter is
  // in global memory).  Neighbouring tasks share their 64 keys.
  auto take = [&]() -> int64_t {
    unsigned int c = 0;
    if (lane == 0) c = atomicAdd(p.task_counter, 1u);
    c = __builtin_amdgcn_readfirstlane(c);
    return (int64_t)c < p.num_waves ? (int64_t)c : p.num_waves;
  };
  for (int64_t w = p.task_counter ? take() : wave0; w < p.num_waves;
       w = p.task_counter ? take() : w + (int64_t)gridDim.x * waves_per_block) {
    const int64_t grp = w / p.u_ranges;
    const int64_t rng = w - grp * p.u_ranges;
    const int64_t k_raw = grp * 64 + lane;
    const bool valid = k_raw < K;
    const int64_t k = valid ? k_raw : K - 1;
    const int64_t cwi = k * p.cw_stride + p.cw_level;
    const dpf_block* vc = p.vcw + k * p.vcw_stride;
#if DPF_HH_KEYS_HOIST
    // The key's two levels of correction words, value correction and party.
    const uint4 key_cs0 = cw_u4(p.cw_seed[cwi]), key_cs1 = cw_u4(p.cw_seed[cwi + 1]);
    const uint32_t key_cc = (uint32_t)(p.cw_left[cwi] & 1) | ((uint32_t)(p.cw_right[cwi] & 1) << 1) |
                            ((uint32_t)(p.cw_left[cwi + 1] & 1) << 2) |
                            ((uint32_t)(p.cw_right[cwi + 1] & 1) << 3) |
                            ((uint32_t)(p.party[k] & 1) << 4);
    const uint32_t key_corr0 = (uint32_t)vc[0].low, key_corr1 = nl > 1 ? (uint32_t)vc[1].low : 0u;
#endif
    const int64_t u_begin = rng * p.u_per_range;
    const int64_t u_end = u_begin + p.u_per_range < U ? u_begin + p.u_per_range : U;
    const int64_t len = u_end - u_begin;
    const int64_t rot = len > 0 ? grp % len : 0;
    for (int64_t i = 0; i < len; ++i) {
      int64_t ui = i + rot;
      if (ui >= len) ui -= len;
      const int64_t u = u_begin + ui;   // wave-uniform
      const int64_t par = p.parent[u];
      Block4 s = stream_load(p.seeds_in + par * K + k);
      uint32_t t;
      if (p.ctrl_in) {
        t = p.ctrl_in[par * K + k] & 1u;
      } else {
        t = s.w0 & 1u;
        s.w0 &= ~1u;
      }
      if (p.save) {
        const int64_t save = p.save_index ? p.save_index[u] : u;
        if (save >= 0 && valid) {
          stream_store(p.seeds_out + save * K + k, s);
          p.ctrl_out[save * K + k] = (uint8_t)t;
        }
      }
      // Two tree levels (cc:304-347): children (ILP2), grandchildren (ILP4);
      // leaf order 0..3 = LL, LR, RL, RR.
      Block4 c0, c1;
      uint32_t t0, t1;
      {
#if DPF_HH_KEYS_HOIST
        const uint4 cs0 = key_cs0;
        const uint32_t cc0 = key_cc & 3u;
#elif DPF_HH_KEYS_MODE == 2
        const uint4 cs0 = p.key_tab[k];
        const uint32_t cc0 = p.key_tab[2 * K + k].x & 3u;
#else
        const uint4 cs0 = cw_u4(p.cw_seed[cwi]);
        const uint32_t cc0 = (uint32_t)(p.cw_left[cwi] & 1) | ((uint32_t)(p.cw_right[cwi] & 1) << 1);
#endif
        children_step(lk, lk.ks.l, lk.ks.r, s, t, cs0, cc0, c0, t0, c1, t1);
      }
      Block4 L[4];
      uint32_t tl[4];
      {
#if DPF_HH_KEYS_HOIST
        const uint4 cs1 = key_cs1;
        const uint32_t cc1 = (key_cc >> 2) & 3u;
#elif DPF_HH_KEYS_MODE == 2
        const uint4 cs1 = p.key_tab[K + k];
        const uint32_t cc1 = (p.key_tab[2 * K + k].x >> 2) & 3u;
#else
        const uint4 cs1 = cw_u4(p.cw_seed[cwi + 1]);
        const uint32_t cc1 =
            (uint32_t)(p.cw_left[cwi + 1] & 1) | ((uint32_t)(p.cw_right[cwi + 1] & 1) << 1);
#endif
        children_step_x2(lk, lk.ks.l, lk.ks.r, c0, t0, c1, t1, cs1, cc1, L, tl);
      }
      if (p.leaf_seeds && valid) {
        int4 sl = make_int4((int)(u << 2), (int)(u << 2) + 1, (int)(u << 2) + 2, (int)(u << 2) + 3);
        if (p.leaf_slot) sl = *reinterpret_cast<const int4*>(p.leaf_slot + (u << 2));
        const int slot[4] = {sl.x, sl.y, sl.z, sl.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          Block4 c = L[j];
          c.w0 |= tl[j];
          stream_store(p.leaf_seeds + slot[j] * K + k, c);
        }
      }
#if DPF_HH_STASH
      lds.stash[0][threadIdx.x] = make_uint4(L[2].w0 | tl[2], L[2].w1, L[2].w2, L[2].w3);
      lds.stash[1][threadIdx.x] = make_uint4(L[3].w0 | tl[3], L[3].w1, L[3].w2, L[3].w3);
#endif
      // Value hashes (cc:500-524), sampling, correction, party negation.
      uint32_t v[8];   // [leaf * 2 + element]
      // Leaves 0 and 1 are sampled before leaves 2 and 3 are hashed; the
      // correction and negation of all four wait until after (the value
      // correction and party are read there): fewer live registers across
      // the second pair's hashes.
      uint32_t tb = tl[0] | (tl[1] << 1);
      const UniformRK rk[4] = {UniformRK{lk.ks.v}, UniformRK{lk.ks.v}, UniformRK{lk.ks.v},
                               UniformRK{lk.ks.v}};
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
#if DPF_HH_STASH
        if (pr == 1) {
          // Same thread wrote these: no barrier needed.
          const uint4 a = lds.stash[0][threadIdx.x], c = lds.stash[1][threadIdx.x];
          tb |= ((a.x & 1u) << 2) | ((c.x & 1u) << 3);
          L[2] = Block4{a.x & ~1u, a.y, a.z, a.w};
          L[3] = Block4{c.x & ~1u, c.y, c.z, c.w};
        }
#else
        if (pr == 1) tb |= (tl[2] << 2) | (tl[3] << 3);
#endif
        Block4 h[4];
        if (p.b == 2) {
          hash_leaf_pair(lk, lk.ks.v, L[2 * pr], L[2 * pr + 1], h);
        } else {
          Block4 two[2] = {L[2 * pr], L[2 * pr + 1]};
          dpf_aes::mmo_hashN<2>(two, lk, rk);
          h[0] = two[0];
          h[2] = two[1];
          h[1] = h[3] = Block4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int leaf = 2 * pr + j;
          sample2_nl(nl, div0, div1, h[2 * j], h[2 * j + 1].w0, &v[leaf * 2]);
        }
      }
      {
#if DPF_HH_KEYS_HOIST
        const uint32_t corr[2] = {key_corr0, key_corr1};
        const bool neg = (key_cc & 16u) != 0;
#elif DPF_HH_KEYS_MODE == 2
        const uint4 meta = p.key_tab[2 * K + k];
        const uint32_t corr[2] = {meta.y, meta.z};
        const bool neg = (meta.x & 16u) != 0;
#else
        const uint32_t corr[2] = {(uint32_t)vc[0].low, nl > 1 ? (uint32_t)vc[1].low : 0u};
        const bool neg = (p.party[k] & 1u) != 0;
#endif
#pragma unroll
        for (int leaf = 0; leaf < 4; ++leaf) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint32_t n = e ? div1.n : div0.n;
            uint32_t r = v[leaf * 2 + e];
            if ((tb >> leaf) & 1u) r = mod_add(r, corr[e], n);   // int_mod_n.h:116-120
            if (neg) r = r == 0 ? 0u : n - r;                     // int_mod_n.h:208-218
            v[leaf * 2 + e] = (e < nl && valid) ? r : 0u;
          }
        }
      }
      const uint32_t total = wave_sum8_mod(v, div0.n, nl > 1 ? div1.n : div0.n);
      const int idx = lane >> 3, e = idx & 1;
      if ((lane & 7) == 0 && e < nl && total)
        atomicAdd(p.sums + ((u << 2) + (idx >> 1)) * nl + e, (unsigned long long)total);
    }
  }
}

// The per-call key table of hh_keys_kernel (DPF_HH_KEYS_MODE 2): key k's
// correction words of levels cw_level, cw_level + 1 and its control-bit
// corrections, value correction and party, index-major so that a wave of 64
// keys reads each part as one 1 KiB access.
__global__ void hh_key_table_kernel(int64_t K, int cw_level, int cw_stride,
                                    const dpf_block* __restrict__ cw_seed,
                                    const uint8_t* __restrict__ cw_left,
                                    const uint8_t* __restrict__ cw_right,
                                    const dpf_block* __restrict__ vcw, int vcw_stride, int nl,
                                    const uint8_t* __restrict__ party, uint4* __restrict__ tab) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < K;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cwi = k * cw_stride + cw_level;
    tab[k] = cw_u4(cw_seed[cwi]);
    tab[K + k] = cw_u4(cw_seed[cwi + 1]);
    const uint32_t cc = (uint32_t)(cw_left[cwi] & 1) | ((uint32_t)(cw_right[cwi] & 1) << 1) |
                        ((uint32_t)(cw_left[cwi + 1] & 1) << 2) |
                        ((uint32_t)(cw_right[cwi + 1] & 1) << 3) | ((uint32_t)(party[k] & 1) << 4);
    const dpf_block* vc = vcw + k * vcw_stride;
    tab[2 * K + k] = make_uint4(cc, (uint32_t)vc[0].low, nl > 1 ? (uint32_t)vc[1].low : 0u, 0u);
  }
}

}  // namespace

namespace dpf_rt {

int launch_hh_keys(const HHLevelArgs& a, hipStream_t s) {
  HHKeysParams p;
  memset(&p, 0, sizeof(p));
  p.num_keys = a.num_keys;
  p.num_starts = a.num_starts;
  const int64_t groups = (a.num_keys + 63) / 64;
  // At least ~4 tasks per wave slot of the chip (64 when they are taken
  // dynamically -- 2^20-client pass 17.16 / 16.71 / 16.39 / 16.28 s at 8 /
  // 16 / 32 / 64, profiles/r16/hh_dynamic_ab.txt; DPF_HH_DYNAMIC=0 turns that
  // off): split the start nodes when there are few 64-key groups.
  // DPF_HH_DYNAMIC=<n>: n tasks per wave slot (A/B hook).
  const char* dyn_env = std::getenv("DPF_HH_DYNAMIC");
  const int per_slot = dyn_env && *dyn_env ? std::atoi(dyn_env) : 64;
  const bool dynamic = per_slot > 0;
  const int64_t want_waves = (int64_t)num_cus() * (kHHKeysBlock / 64) * (dynamic ? per_slot : 4);
  int64_t ranges = (want_waves + groups - 1) / groups;
  if (ranges > a.num_starts) ranges = a.num_starts;
  if (ranges < 1) ranges = 1;
  p.u_per_range = (a.num_starts + ranges - 1) / ranges;
  p.u_ranges = (a.num_starts + p.u_per_range - 1) / p.u_per_range;
  p.num_waves = groups * p.u_ranges;
  p.cw_level = a.cw_level;
  p.cw_stride = a.cw_stride;
  p.nl = a.nl;
  p.b = a.b;
  p.seeds_in = a.seeds_in;
  p.ctrl_in = a.ctrl_in;
  p.parent = a.parent;
  p.save = a.save;
  p.save_index = a.save_index;
  p.seeds_out = a.seeds_out;
  p.ctrl_out = a.ctrl_out;
  p.cw_seed = a.cw_seed;
  p.cw_left = a.cw_left;
  p.cw_right = a.cw_right;
  p.vcw = a.vcw;
  p.vcw_stride = a.vcw_stride;
  p.party = a.party;
  p.sums = a.wide;
  p.leaf_seeds = a.leaf_seeds;
  p.leaf_slot = a.leaf_slot;
  for (int i = 0; i < 2; ++i) p.div[i] = make_div32(a.mod[i < a.nl ? i : 0]);
  p.rkl = expand_key(a.key_left);
  p.rkr = expand_key(a.key_right);
  p.rkv = expand_key(a.key_value);
  int64_t grid = (p.num_waves * 64 + kHHKeysBlock - 1) / kHHKeysBlock;
  if (grid > num_cus()) grid = num_cus();   // one 128 KiB-table workgroup per CU
  if (grid < 1) grid = 1;
  if (p.num_waves > (int64_t)UINT32_MAX / 2) return fail(kInvalidArgument, "too many tasks");
  void* tab = nullptr;
  if (DPF_HH_KEYS_MODE == 2) {
    // Stream-ordered scratch (48 B per key), freed behind the kernel; the
    // device's default pool keeps it for the next level's call.
    static const bool pool_kept = [] {
      int dev = 0;
      hipMemPool_t pool;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetDefaultMemPool(&pool, dev) != hipSuccess)
        return false;
      uint64_t keep = UINT64_MAX;
      return hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep) == hipSuccess;
    }();
    (void)pool_kept;
    // The key table, then the dynamic task counter.
    HIP_TRY(hipMallocAsync(&tab, (size_t)a.num_keys * 3 * sizeof(uint4) + 256, s));
    int64_t g = (a.num_keys + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(hh_key_table_kernel, dim3((unsigned)g), dim3(256), 0, s, a.num_keys,
                       a.cw_level, a.cw_stride, a.cw_seed, a.cw_left, a.cw_right, a.vcw,
                       a.vcw_stride, a.nl, a.party, static_cast<uint4*>(tab));
    p.key_tab = static_cast<const uint4*>(tab);
  } else {
    HIP_TRY(hipMallocAsync(&tab, 256, s));
  }
  if (dynamic) {
    p.task_counter = reinterpret_cast<unsigned int*>(
        static_cast<char*>(tab) + (DPF_HH_KEYS_MODE == 2 ? (size_t)a.num_keys * 3 * sizeof(uint4) : 0));
    HIP_TRY(hipMemsetAsync(p.task_counter, 0, sizeof(unsigned int), s));
  }
  hipLaunchKernelGGL(hh_keys_kernel, dim3((unsigned)grid), dim3(kHHKeysBlock), 0, s, p);
  const hipError_t e = hipGetLastError();
  if (tab) HIP_TRY(hipFreeAsync(tab, s));
  HIP_TRY(e);
  return kOk;
}

int launch_hh_level(const HHLevelArgs& a, hipStream_t s) {
  if (a.nl < 1 || a.nl > 2 || (a.b != 1 && a.b != 2) || (a.nl == 2 && a.b != 2))
    return fail(kUnimplemented, "hh_level_kernel: unsupported value type");
  if (a.index_major) return launch_hh_keys(a, s);
  HHParams p;
  memset(&p, 0, sizeof(p));
  p.num_keys = a.num_keys;
  p.num_starts = a.num_starts;
  p.waves_per_chunk = (a.num_starts + 63) / 64;
  // ~4 tasks per wave slot, or DPF_HH_DYNAMIC (default 64) taken dynamically
  // (0: the fixed grid-stride share).
  const char* dyn_env = std::getenv("DPF_HH_DYNAMIC");
  const int per_slot = dyn_env && *dyn_env ? std::atoi(dyn_env) : 64;
  const bool dynamic = per_slot > 0;
  const int64_t want_waves = (int64_t)num_cus() * (kBlock / 64) * (dynamic ? per_slot : 4);
  int64_t chunks = (want_waves + p.waves_per_chunk - 1) / p.waves_per_chunk;
  if (chunks > a.num_keys) chunks = a.num_keys;
  if (chunks < 1) chunks = 1;
  p.chunk_keys = (a.num_keys + chunks - 1) / chunks;
  chunks = (a.num_keys + p.chunk_keys - 1) / p.chunk_keys;
  p.num_threads = chunks * p.waves_per_chunk * 64;
  p.cw_level = a.cw_level;
  p.cw_stride = a.cw_stride;
  p.save = a.save;
  p.nl = a.nl;
  p.b = a.b;
  p.seeds_in = a.seeds_in;
  p.ctrl_in = a.ctrl_in;
  p.in_stride = a.in_stride;
  p.parent = a.parent;
  p.save_index = a.save_index;
  p.seeds_out = a.seeds_out;
  p.ctrl_out = a.ctrl_out;
  p.out_stride = a.out_stride;
  p.cw_seed = a.cw_seed;
  p.cw_left = a.cw_left;
  p.cw_right = a.cw_right;
  p.vcw = a.vcw;
  p.vcw_stride = a.vcw_stride;
  p.party = a.party;
  p.wide = a.wide;
  p.leaf_seeds = a.leaf_seeds;
  p.leaf_stride = a.leaf_stride;
  p.leaf_slot = a.leaf_slot;
  for (int i = 0; i < a.nl; ++i) p.div[i] = make_div32(a.mod[i]);
  p.rkl = expand_key(a.key_left);
  p.rkr = expand_key(a.key_right);
  p.rkv = expand_key(a.key_value);
  int64_t grid = (p.num_threads + kHHBlock - 1) / kHHBlock;
  if (grid > num_cus()) grid = num_cus();   // one 128 KiB-LDS workgroup per CU
  if (grid < 1) grid = 1;
  void* counter = nullptr;
  if (dynamic) {
    HIP_TRY(hipMallocAsync(&counter, 256, s));
    HIP_TRY(hipMemsetAsync(counter, 0, sizeof(unsigned int), s));
    p.task_counter = static_cast<unsigned int*>(counter);
  }
  hipLaunchKernelGGL(hh_level_kernel, dim3((unsigned)grid), dim3(kHHBlock), 0, s, p);
  const hipError_t e = hipGetLastError();
  if (counter) HIP_TRY(hipFreeAsync(counter, s));
  HIP_TRY(e);
  return kOk;
}

}  // namespace dpf_rt
