// dpf_kernels.hip -- MI355X (gfx950) kernels for incremental-DPF evaluation and
// the C ABI declared in include/dpf_hip.h.
//
// Hot path:
//   * AES-128 MMO hash with the four T-tables replicated 32x across LDS banks
//     (128 KiB): lane l reads copy (l & 31), so every ds_read_b32 of a wave is
//     bank-conflict-free whatever the table index.  Tables are laid out in
//     256-byte rows so one v_perm_b32 forms each lookup address; 3-input XORs
//     are single v_bitop3_b32 (gfx950).  One 1024-thread workgroup per CU.
//     Measured (tools/aes_microbench.hip): 97 G AES/s with two interleaved
//     chains, 88% of the chip's ds_read_b32 ceiling.
//   * expand_kernel: one thread = one subtree.  It walks from its start seed to
//     the subtree root along the bits of its work-item index (per-lane key
//     select), then visits the subtree depth-first with the path stack held in
//     VGPRs (uniform control flow: every lane of a wave is at the same leaf
//     pair), hashing each leaf with the value key, converting, correcting and
//     storing it.  Intermediate seeds never touch HBM; only leaves are written.
//   * eval_points_kernel: one thread = one (key, point) path walk, fused with the
//     leaf hash, conversion, correction and the store of the selected element.
//   * Correction words live in LDS (broadcast reads).
// All arithmetic is integer/bitwise; no MFMA (nothing here is a contraction).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <type_traits>
#include <thread>
#include <vector>
#include <string>

#include "../../../include/dpf_hip.h"
#include "dpf_device.h"
#include "dpf_runtime.h"

namespace dpf_rt {
thread_local std::string g_last_error;
thread_local const char* g_last_expand = "";
thread_local int g_last_expand_s = -1;
// dpf_hip_clock_probe's device accumulator (NULL: off), read by every
// dpf_hip_expand launch.
std::atomic<unsigned long long*> g_clock_acc{nullptr};

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? kResourceExhausted : kInternal,
              std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace dpf_rt

using namespace dpf_rt;

namespace {

// ------------------------------------------------------------------------
// Kernels
// ------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void hash_kernel(int64_t n, const dpf_block* __restrict__ in,
                                                      dpf_block* __restrict__ out,
                                                      RoundKeys rk, int64_t dyn_per_wg) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h); dyn_per_wg 0: grid stride
  fill_tables(lds.tab);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const KeyRef kr = key_ref(rk);
  LdsLookup lk = make_lookup(lds, KeySet{kr, kr, kr, kr});
  const int64_t nch = (n + 63) / 64;
  for (int64_t i = dyn_per_wg ? take_chunk(&next_chunk, dyn_per_wg, nch, n)
                              : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < n;
       i = dyn_per_wg ? take_chunk(&next_chunk, dyn_per_wg, nch, n)
                      : i + (int64_t)gridDim.x * blockDim.x) {
    store_block(out + i, dpf_aes::mmo_hash(load_block(in + i), lk, UniformRK{lk.ks.v}));
  }
}

struct PathParams {
  int64_t n;
  int num_levels;
  const dpf_block* seeds_in;
  const uint8_t* ctrl_in;
  const dpf_block* paths;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  dpf_block* seeds_out;
  uint8_t* ctrl_out;
  RoundKeys rkl, rkd;
  int64_t dyn_per_wg;  // take_chunk's per_wg (0: grid stride)
};


__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void eval_paths_kernel(PathParams p) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h)
  fill_tables(lds.tab);
  fill_cws(lds, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  LdsLookup lk = make_lookup(lds, KeySet{key_ref(p.rkl), KeyRef{}, KeyRef{}, key_ref(p.rkd)});
  const int64_t nch = (p.n + 63) / 64;
  for (int64_t i = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.n)
                                : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < p.n;
       i = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.n)
                        : i + (int64_t)gridDim.x * blockDim.x) {
    Block4 s = load_block(p.seeds_in + i);
    uint32_t t = p.ctrl_in[i] & 1u;
    Block4 path = load_block(p.paths + i);
    for (int j = 0; j < p.num_levels; ++j) {
      uint32_t bit = path_bit(path, p.num_levels - 1 - j);
      path_step(lk, lk.ks.l, lk.ks.d, s, t, bit, lds.cw_seed[j], lds.cw_ctrl[j]);
    }
    store_block(p.seeds_out + i, s);
    p.ctrl_out[i] = (uint8_t)t;
  }
}

template <class Leaf>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void expand_kernel(ExpandParams p, Leaf leaf) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h), p.dyn_chunks > 0
  leaf.init();
  fill_tables(lds.tab);
  fill_cws(lds, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const LdsLookup lk = make_lookup(lds, KeySet{key_ref(p.rkl), key_ref(p.rkr), key_ref(p.rkv), key_ref(p.rkd)});
  const int k0 = p.k0, S = p.S;
  const int B = S >= 1 ? 1 : 0;  // leaf pairs share their parent
  const int G = S - B;            // depth of the DFS stack
  const int64_t ngroups = (int64_t)1 << G;
  // Items by grid stride, or 64 at a time per wave (dyn_chunks > 0, as the
  // octet kernel).
  const int64_t nch = (p.num_items + 63) / 64;
  for (int64_t item = p.dyn_chunks ? take_chunk(&next_chunk, p.dyn_chunks, nch, p.num_items)
                                   : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       item < p.num_items;
       item = p.dyn_chunks ? take_chunk(&next_chunk, p.dyn_chunks, nch, p.num_items)
                           : item + (int64_t)gridDim.x * blockDim.x) {
    // 1. walk from the start seed to this item's subtree root.
    const int64_t r = item >> k0;
    Block4 s = load_block(p.seeds_in + r);
    uint32_t t = p.ctrl_in[r] & 1u;
    for (int j = 0; j < k0; ++j) {
      uint32_t bit = (uint32_t)((item >> (k0 - 1 - j)) & 1);
      path_step(lk, lk.ks.l, lk.ks.d, s, t, bit, lds.cw_seed[j], lds.cw_ctrl[j]);
    }
    // 2. depth-first over the subtree.  Every inner node is expanded into both
    //    children at once (two interleaved hashes); the left child is descended
    //    into and the right one parked in sib[d] until the walk returns to it,
    //    so each node is hashed exactly once and always in a pair.
    Block4 sib[kGMax];  // sib[d - 1] = parked right child at depth d
    uint32_t tb = 0;  // bit d = control bit of sib[d]
    const int64_t leaf_base = item << S;
    for (int64_t g = 0; g < ngroups; ++g) {
      Block4 node = s;
      uint32_t nt = t;
      int ds = 0;  // depth of `node` (wave-uniform)
      if (g != 0) {
        ds = G - (int)__builtin_ctzll((unsigned long long)g);
#pragma unroll
        for (int d = 1; d <= kGMax; ++d)
          if (d == ds) { node = sib[d - 1]; nt = (tb >> d) & 1u; }
      }
      for (int d = ds; d < G; ++d) {
        Block4 c0, c1;
        uint32_t t0, t1;
        children_step(lk, lk.ks.l, lk.ks.r, node, nt, lds.cw_seed[k0 + d], lds.cw_ctrl[k0 + d],
                      c0, t0, c1, t1);
#pragma unroll
        for (int e = 1; e <= kGMax; ++e)
          if (e == d + 1) sib[e - 1] = c1;
        tb = (tb & ~(1u << (d + 1))) | (t1 << (d + 1));
        node = c0;
        nt = t0;
      }
      if (B == 0) {
        leaf.emit(lk, lk.ks.v, node, nt, leaf_base + g, p.out);
      } else {
        const int lvl = k0 + G;
        Block4 c0, c1;
        uint32_t t0, t1;
        children_step(lk, lk.ks.l, lk.ks.r, node, nt, lds.cw_seed[lvl], lds.cw_ctrl[lvl], c0, t0,
                      c1, t1);
        leaf.emit2(lk, lk.ks.v, c0, t0, c1, t1, leaf_base + 2 * g, p.out);
      }
    }
  }
}

// Octet form of expand_kernel for integer leaves that fill whole 16-byte
// blocks (uint64, uint128, XorWrapper, uniform tuples; the default for them):
// the bottom three levels of every subtree are expanded breadth-first as an
// octet -- the node's 2 children (ILP2), its 4 grandchildren (ILP4), then per
// half its 4 leaf seeds and their 4 value hashes (ILP4 each) -- and each lane
// writes its 8 corrected blocks as 2 x 64 contiguous bytes, i.e. whole
// 128-byte lines (expand_kernel's 32-byte leaf-pair pieces measured write
// amplification 1.25).  The DFS stack above the octets lives in scratch (one
// 16-byte store per push, one load per octet, issued an octet ahead) so the
// VGPRs go to the ILP4 chains (128 VGPRs plus 160 B/lane of spills remain;
// that scratch traffic, not the outputs, is most of its HBM bytes beyond the
// 8 GiB written).  Measured same-box at config 2: 18.58 vs 18.87-18.98 ms per
// 2^30 outputs with identical outputs (tools/octet_check.py); in the bench
// 17.9 ms per step (59.95 G leaves/s).
// Half an octet's leaves (4 consecutive leaf blocks): integer leaves filling
// whole blocks store 4 x 16 contiguous bytes; other policies use their emit4.
template <int BITS, bool XOR>
__device__ __forceinline__ void octet_half(const FastIntLeaf<BITS, XOR>& leaf, const LdsLookup& lk,
                                           KeyRef rkv, Block4* l, const uint32_t* lt,
                                           int64_t first_leaf, char* out, Block4*) {
  const UniformRK rv[4] = {UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}, UniformRK{rkv}};
  dpf_aes::mmo_hashN<4>(l, lk, rv);
  uint4* o = reinterpret_cast<uint4*>(out + first_leaf * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const Block4 h = leaf.correct(l[j], lt[j]);
    o[j] = make_uint4(h.w0, h.w1, h.w2, h.w3);
  }
}
template <class Leaf>
__device__ __forceinline__ void octet_half(const Leaf& leaf, const LdsLookup& lk,
                                           KeyRef rkv, Block4* l, const uint32_t* lt,
                                           int64_t first_leaf, char* out, Block4* park) {
  leaf.emit4(lk, rkv, l, lt, first_leaf, out);
}
#ifndef DPF_MOD32_PARK
#define DPF_MOD32_PARK 1
#endif
// Tuples of IntModN<uint32_t>: the half's second leaf pair (seed | control
// bit in bit 0) waits in two scratch slots beside the DFS stack while the
// first pair's four value hashes run, instead of in 8 + 2 VGPRs -- that group
// was the register-starved one (~3 lookups in flight, r15 ISA).
template <class Leaf> struct OctetStash;
template <int NL>
__device__ __forceinline__ void octet_half(const Mod32Leaf<NL>& leaf, const LdsLookup& lk,
                                           KeyRef rkv, Block4* l, const uint32_t* lt,
                                           int64_t first_leaf, char* out, Block4* park) {
#if DPF_MOD32_PARK
  static_assert(OctetStash<Mod32Leaf<NL>>::value >= 2, "park slots hold the octet stash");
  park[0] = Block4{l[2].w0 | lt[2], l[2].w1, l[2].w2, l[2].w3};
  park[1] = Block4{l[3].w0 | lt[3], l[3].w1, l[3].w2, l[3].w3};
  asm volatile("" ::: "memory");   // read them back from scratch, not from registers
  uint32_t x[4][NL];
  {
    uint32_t w0[8], w1[8];
    leaf.hash2(lk, rkv, l[0], l[1], w0, w1);
    leaf.convert(w0, lt[0], x[0]);
    leaf.convert(w1, lt[1], x[1]);
  }
  asm volatile("" ::: "memory");
  {
    const Block4 a = park[0], b = park[1];
    uint32_t w0[8], w1[8];
    leaf.hash2(lk, rkv, Block4{a.w0 & ~1u, a.w1, a.w2, a.w3}, Block4{b.w0 & ~1u, b.w1, b.w2, b.w3},
               w0, w1);
    leaf.convert(w0, a.w0 & 1u, x[2]);
    leaf.convert(w1, b.w0 & 1u, x[3]);
  }
  leaf.store4(x, first_leaf, out);
#else
  leaf.emit4(lk, rkv, l, lt, first_leaf, out);
#endif
}

// Where the octet keeps its second half's two grandchildren during the first
// half: 0 = both in scratch beside the DFS stack, 1 = q[3] in LDS (16 B per
// lane), 2 = also q[2]'s upper 12 bytes in LDS, its low word in a VGPR -- the
// LDS left over by the T-tables and correction words (150 + 12 KiB of 160).
// Config 2: 17.21 -> 17.08 (1) -> 16.96 ms (2), WRITE_SIZE 1.30 -> 1.21 -> 1.18x
// the 8 GiB written; SwarLeaf runs out of VGPRs at 2 (profiles/r11_ws_ab.txt).
#ifndef DPF_OCTET_LDS_STASH
#define DPF_OCTET_LDS_STASH 2
#endif
template <class Leaf> struct OctetStash { static constexpr int value = DPF_OCTET_LDS_STASH; };
template <> struct OctetStash<SwarLeaf> {
  static constexpr int value = DPF_OCTET_LDS_STASH < 1 ? DPF_OCTET_LDS_STASH : 1;
};

template <class Leaf>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void expand_octet_kernel(ExpandParams p,
                                                                             Leaf leaf) {
  __shared__ LdsImage lds;
  constexpr int kStash = OctetStash<Leaf>::value;
  __shared__ uint4 stash[kStash >= 1 ? kBlock : 1];
  __shared__ uint3 stash2[kStash >= 2 ? kBlock : 1];
  __shared__ int next_chunk;   // dynamic distribution: the workgroup's next 64 items
  static_assert(sizeof(LdsImage) + (kStash >= 1 ? 16 * kBlock : 0) +
                    (kStash >= 2 ? 12 * kBlock : 0) + 16 <= 160 * 1024, "LDS over 160 KiB");
  leaf.init();
  fill_tables(lds.tab);
  fill_cws(lds, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const LdsLookup lk = make_lookup(lds, KeySet{key_ref(p.rkl), key_ref(p.rkr), key_ref(p.rkv), key_ref(p.rkd)});
  const int k0 = p.k0, S = p.S;
  const int G = S - 3;
  const int64_t ngroups = (int64_t)1 << G;
  ClockStamp stamp;
  stamp.begin(p.clock);
  // Items: thread u takes u, u + threads, ... (static), or -- dyn_chunks > 0
  // -- each wave takes the workgroup's next 64 items from next_chunk until
  // its range is used up.  The CU's arbiter favours its oldest waves (in
  // config 2 wave 0 of a workgroup finished in 7.8 ms, wave 15 in 16.6 ms of
  // a 16.9 ms launch): with a fixed share the last third of a launch runs on
  // fewer and fewer waves, while taken dynamically the fast waves do more
  // and all finish together.  Every lane of a wave holds the same chunk, so
  // the DFS stays wave-uniform.
  const int lane = (int)(threadIdx.x & 63);
  auto take = [&]() -> int64_t {
    int c = 0;
    if (lane == 0) c = atomicAdd(&next_chunk, 1);
    c = __builtin_amdgcn_readfirstlane(c);
    return c < p.dyn_chunks ? ((int64_t)blockIdx.x * p.dyn_chunks + c) * 64 + lane : p.num_items;
  };
  for (int64_t item = p.dyn_chunks ? take() : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       item < p.num_items;
       item = p.dyn_chunks ? take() : item + (int64_t)gridDim.x * blockDim.x) {
    // 1. walk from the start seed to this item's subtree root.
    const int64_t r = item >> k0;
    Block4 s = load_block(p.seeds_in + r);
    uint32_t t = p.ctrl_in[r] & 1u;
    for (int j = 0; j < k0; ++j) {
      const uint32_t bit = (uint32_t)((item >> (k0 - 1 - j)) & 1);
      path_step(lk, lk.ks.l, lk.ks.d, s, t, bit, lds.cw_seed[j], lds.cw_ctrl[j]);
    }
    // 2. depth-first down to the octet roots; right children parked in
    //    sib[d] (scratch), their control bits in tb.
    Block4 sib[kGMax];
    uint32_t tb = 0;
    const int64_t leaf_base = item << S;
    Block4 next = s;
    for (int64_t g = 0; g < ngroups; ++g) {
      Block4 node = next;
      uint32_t nt = t;
      int ds = 0;
      if (g != 0) {
        ds = G - (int)__builtin_ctzll((unsigned long long)g);
        nt = (tb >> ds) & 1u;
      }
      for (int d = ds; d < G; ++d) {
        Block4 c0, c1;
        uint32_t t0, t1;
        children_step(lk, lk.ks.l, lk.ks.r, node, nt, lds.cw_seed[k0 + d], lds.cw_ctrl[k0 + d],
                      c0, t0, c1, t1);
        sib[d] = c1;
        tb = (tb & ~(1u << (d + 1))) | (t1 << (d + 1));
        node = c0;
        nt = t0;
      }
      // The next octet's root (written by now), loaded an octet ahead.
      if (g + 1 < ngroups) next = sib[G - (int)__builtin_ctzll((unsigned long long)(g + 1)) - 1];
      // 3. the octet.
      const int lvl = k0 + G;
      Block4 c[2], q[4];
      uint32_t ct[2], qt[4];
      children_step(lk, lk.ks.l, lk.ks.r, node, nt, lds.cw_seed[lvl], lds.cw_ctrl[lvl], c[0],
                    ct[0], c[1], ct[1]);
      children_step_x2(lk, lk.ks.l, lk.ks.r, c[0], ct[0], c[1], ct[1], lds.cw_seed[lvl + 1],
                       lds.cw_ctrl[lvl + 1], q, qt);
      // The second half's two grandchildren wait outside the VGPRs during the
      // first half (OctetStash: lane-private LDS slots, else scratch beside
      // the DFS stack) instead of 8 VGPRs: 128 VGPRs with 37 spilled -> 110
      // with none, +3.5%, HBM traffic 17.7 -> 12.1 GB per config-2 launch in
      // scratch, 10.9 GB in LDS (profiles/r11_ws_ab.txt).  The DFS uses
      // sib[0 .. S-4], S <= kSMax.  Each lane reads back only its own slot.
      static_assert(kSMax - 3 <= kGMax - 2, "stash overlaps the DFS stack");
      uint32_t q2w0 = 0;
      if constexpr (kStash >= 2) {
        q2w0 = q[2].w0;
        stash2[threadIdx.x] = make_uint3(q[2].w1, q[2].w2, q[2].w3);
      } else {
        sib[kGMax - 2] = q[2];
      }
      if constexpr (kStash >= 1)
        stash[threadIdx.x] = make_uint4(q[3].w0, q[3].w1, q[3].w2, q[3].w3);
      else
        sib[kGMax - 1] = q[3];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        Block4 l[4];
        uint32_t lt[4];
        if (hf == 1) {
          if constexpr (kStash >= 2) {
            const uint3 u = stash2[threadIdx.x];
            q[2] = Block4{q2w0, u.x, u.y, u.z};
          } else {
            q[2] = sib[kGMax - 2];
          }
          if constexpr (kStash >= 1) {
            const uint4 v = stash[threadIdx.x];
            q[3] = Block4{v.x, v.y, v.z, v.w};
          } else {
            q[3] = sib[kGMax - 1];
          }
        }
        children_step_x2(lk, lk.ks.l, lk.ks.r, q[2 * hf], qt[2 * hf], q[2 * hf + 1],
                         qt[2 * hf + 1], lds.cw_seed[lvl + 2], lds.cw_ctrl[lvl + 2], l, lt);
        // The half's four value hashes (ILP4), conversion, correction, stores
        // (integer leaves: 64 contiguous bytes per lane).
        // sib[kGMax - 2 ..] is free when the stash lives in LDS (kStash == 2):
        // Mod32Leaf parks a leaf pair there.
        octet_half(leaf, lk, lk.ks.v, l, lt, leaf_base + 8 * g + 4 * hf, p.out, &sib[kGMax - 2]);
      }
    }
  }
  stamp.end(p.clock);
}

// Batched point evaluation (row a11).  Work item u covers
// key k and the point PAIR (q, q + half) of that key, hashed as two
// interleaved chains (ILP2).  With UNIFORM, half % 64 == 0, so all 64 lanes of
// a wave share k: `k` is made wave-uniform and the key's correction words come
// through scalar loads.  In sum mode (SUM) item u covers the pair for a chunk
// of `chunk_keys` consecutive keys and accumulates the shares in the value
// type's group before one wide atomic add per point.
struct PointParams {
  int64_t num_keys;
  int64_t points_per_key;   // P
  int64_t half;             // ceil(P / 2)
  int64_t num_items;
  int64_t chunk_keys;       // SUM: keys per item
  int shared_points;        // tree_index/block_index indexed by point only
  int num_levels;
  int cw_stride;            // correction words per key row (>= num_levels)
  int bib;                  // block-index bits: tree_index holds raw domain points
                            // (path = point >> bib, element = point & (2^bib - 1))
  const dpf_block* key_seed;
  const uint8_t* party;
  const dpf_block* seeds_in;
  const uint8_t* ctrl_in;
  const dpf_block* tree_index;
  const int32_t* block_index;
  const dpf_block* cw_seed;   // [key][level]
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  const dpf_block* vcw;       // [key][E * num_leaves]
  int vcw_stride;             // E * num_leaves
  char* out;
  unsigned long long* wide;   // SUM: [point][leaf][3] 192-bit exact sums
  int esz;
  int xor_mode;               // fast leaves: XorWrapper
  RoundKeys rkl, rkd, rkv;
  int64_t dyn_per_wg;         // eval_points4_kernel: take_chunk's per_wg (0: grid stride)
  int top_levels;             // eval_points4_kernel: nonzero: the TOP instance (6 / 4 levels walked once per wave)
};

// Latency mode of full-domain expansion for small trees (r15; config 1 and
// the reference's BM_EvaluateRegularDpf below ~2^20 outputs).  expand_kernel /
// the octet kernel give every lane its own subtree and walk each one from the
// start seed: at 2^19 leaves that is 262144 walks of 18 levels, 3.7x the
// algorithmic AES, and each lane's chain is latency-bound.  Here workgroup w
// owns the subtree at depth t = p.k0 under start w >> t (one workgroup per CU
// at most) and expands its D = p.S levels breadth-first through LDS, so every
// node is hashed once:
//   * wave 0 walks the t levels to the subtree root, one chain per lane QUAD
//     (quad::path_step);
//   * a level of <= 256 parents: quad q expands parent q into both children
//     (quad::children, the two hashes interleaved);
//   * a wider level: lane i expands parent i (children_step, ILP2);
//   * level D: lane i expands parent i and value-hashes its two leaves
//     (Leaf::emit2), stored side by side at (w << D) + 2i; integer leaves of
//     a level of <= 256 parents do that in quads.
// Nodes live in nodes[] / tbits[] (<= 1024 per level, so D <= 11), read into
// registers before a barrier and rewritten after it.
constexpr int kSmallMaxD = 11;
template <class Leaf> struct IsFastInt : std::false_type {};
template <int BITS, bool XOR> struct IsFastInt<FastIntLeaf<BITS, XOR>> : std::true_type {};
template <class Leaf>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void expand_small_kernel(ExpandParams p, Leaf leaf) {
  __shared__ LdsImage lds;
  __shared__ uint4 nodes[kBlock];
  __shared__ uint32_t tbits[kBlock];
  leaf.init();
  fill_tables(lds.tab);
  fill_cws(lds, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  __syncthreads();
  const LdsLookup lk =
      make_lookup(lds, KeySet{key_ref(p.rkl), key_ref(p.rkr), key_ref(p.rkv), key_ref(p.rkd)});
  const quad::Keys ql = quad::keys_of(p.rkl), qd = quad::keys_of(p.rkd);
  const int t = p.k0, D = p.S;
  const int64_t w = blockIdx.x;
  const int tid = threadIdx.x, c = quad::column(), q = tid >> 2;
  auto word = [](const uint4& v, int i) { return reinterpret_cast<const uint32_t*>(&v)[i]; };
  if (tid < 64) {
    const int64_t r = w >> t;
    uint32_t s = reinterpret_cast<const uint32_t*>(p.seeds_in + r)[c];
    uint32_t tt = p.ctrl_in[r] & 1u;
    for (int j = 0; j < t; ++j) {
      const uint32_t bit = (uint32_t)((w >> (t - 1 - j)) & 1);
      quad::path_step(lk, ql, qd, s, tt, bit, word(lds.cw_seed[j], c), lds.cw_ctrl[j]);
    }
    if (tid < 4) {
      reinterpret_cast<uint32_t*>(&nodes[0])[c] = s;
      if (c == 0) tbits[0] = tt;
    }
  }
  __syncthreads();
  for (int j = 1; j < D; ++j) {
    const int lvl = t + j - 1, npar = 1 << (j - 1);
    if (npar <= kBlock / 4) {
      const bool on = q < npar;
      uint32_t c0 = 0, c1 = 0, t0 = 0, t1 = 0;
      if (on)
        quad::children(lk, ql, qd, word(nodes[q], c), tbits[q], word(lds.cw_seed[lvl], c),
                       lds.cw_ctrl[lvl], c0, t0, c1, t1);
      __syncthreads();
      if (on) {
        reinterpret_cast<uint32_t*>(&nodes[2 * q])[c] = c0;
        reinterpret_cast<uint32_t*>(&nodes[2 * q + 1])[c] = c1;
        if (c == 0) {
          tbits[2 * q] = t0;
          tbits[2 * q + 1] = t1;
        }
      }
      __syncthreads();
    } else {
      const bool on = tid < npar;
      Block4 c0{}, c1{};
      uint32_t t0 = 0, t1 = 0;
      if (on) {
        const uint4 v = nodes[tid];
        children_step(lk, lk.ks.l, lk.ks.r, Block4{v.x, v.y, v.z, v.w}, tbits[tid],
                      lds.cw_seed[lvl], lds.cw_ctrl[lvl], c0, t0, c1, t1);
      }
      __syncthreads();
      if (on) {
        nodes[2 * tid] = make_uint4(c0.w0, c0.w1, c0.w2, c0.w3);
        nodes[2 * tid + 1] = make_uint4(c1.w0, c1.w1, c1.w2, c1.w3);
        tbits[2 * tid] = t0;
        tbits[2 * tid + 1] = t1;
      }
      __syncthreads();
    }
  }
  const int lvl = t + D - 1, npar = 1 << (D - 1);
  const int64_t leaf0 = w << D;
  bool quad_last = false;
  if constexpr (IsFastInt<Leaf>::value) quad_last = npar <= kBlock / 4;
  if (quad_last) {
    if constexpr (IsFastInt<Leaf>::value) if (q < npar) {
      const quad::Keys qv = quad::keys_of(p.rkv);
      uint32_t c0, c1, t0, t1;
      quad::children(lk, ql, qd, word(nodes[q], c), tbits[q], word(lds.cw_seed[lvl], c),
                     lds.cw_ctrl[lvl], c0, t0, c1, t1);
      quad::hash2(lk, qv, c0, c1);
      const Block4 h0 = quad::gather(c0), h1 = quad::gather(c1);
      if (c == 0) {
        leaf.store(leaf.correct(h0, t0), leaf0 + 2 * q, p.out);
        leaf.store(leaf.correct(h1, t1), leaf0 + 2 * q + 1, p.out);
      }
    }
  } else if (tid < npar) {
    const uint4 v = nodes[tid];
    Block4 c0, c1;
    uint32_t t0, t1;
    children_step(lk, lk.ks.l, lk.ks.r, Block4{v.x, v.y, v.z, v.w}, tbits[tid], lds.cw_seed[lvl],
                  lds.cw_ctrl[lvl], c0, t0, c1, t1);
    leaf.emit2(lk, lk.ks.v, c0, t0, c1, t1, leaf0 + 2 * tid, p.out);
  }
}

// Leaf policy of the tree-top pass (expand_top, below): expand_small_kernel's
// last breadth-first level is not hashed; its nodes are stored as the start
// seeds (seed, control bit) of the octet kernel's items.
struct SeedLeaf {
  dpf_block* seeds;
  uint8_t* ctrl;
  __device__ __forceinline__ void init() const {}
  __device__ __forceinline__ void emit2(const LdsLookup&, KeyRef, Block4 s0, uint32_t t0, Block4 s1,
                                        uint32_t t1, int64_t first, char*) const {
    store_block(seeds + first, s0);
    store_block(seeds + first + 1, s1);
    ctrl[first] = (uint8_t)t0;
    ctrl[first + 1] = (uint8_t)t1;
  }
};

// PAIRED = false (launches below one wave per CU, never in sum mode): one
// chain per lane, half = P, so a small call spreads over twice the CUs and each
// wave's dependent AES chain issues half the LDS reads per round.
template <class Leaf, int BITS, bool FAST, bool UNIFORM, bool SUM, bool PAIRED = true>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void eval_points_kernel(PointParams p, Leaf leaf) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h)
  fill_tables(lds.tab);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const LdsLookup lk = make_lookup(lds, KeySet{key_ref(p.rkl), KeyRef{}, key_ref(p.rkv), key_ref(p.rkd)});
  const int L = p.num_levels;
  const int64_t P = p.points_per_key, half = p.half;
  // Items by grid stride, or 64 at a time per wave (dyn_per_wg > 0; a chunk
  // cut off by num_items is the range's last, after which no lane takes more).
  const int64_t nch = (p.num_items + 63) / 64;
  for (int64_t u = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.num_items)
                                : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       u < p.num_items;
       u = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.num_items)
                        : u + (int64_t)gridDim.x * blockDim.x) {
    int64_t grp = u / half;
    if (UNIFORM) grp = (int64_t)__builtin_amdgcn_readfirstlane((int)grp);
    const int64_t q0 = u - grp * half;
    const int64_t q1raw = q0 + half;
    const bool has1 = q1raw < P;
    const int64_t q1 = has1 ? q1raw : q0;
    int64_t k_begin = grp, k_end = grp + 1;
    if (SUM) {
      k_begin = grp * p.chunk_keys;
      k_end = k_begin + p.chunk_keys < p.num_keys ? k_begin + p.chunk_keys : p.num_keys;
    }
    // Points are shared by all keys (sum mode always) or per key.
    const int64_t pi0 = p.shared_points ? q0 : grp * P + q0;
    const int64_t pi1 = p.shared_points ? q1 : grp * P + q1;
    const Block4 path0 = load_block(p.tree_index + pi0);
    const Block4 path1 = load_block(p.tree_index + pi1);
    const int bb = p.bib;
    const uint32_t bmask = (1u << bb) - 1u;
    const int bi0 = p.block_index ? p.block_index[pi0] : (int)(path0.w0 & bmask);
    const int bi1 = p.block_index ? p.block_index[pi1] : (int)(path1.w0 & bmask);
    u128 acc0[FAST ? 1 : DPF_MAX_LEAVES], acc1[FAST ? 1 : DPF_MAX_LEAVES];
    const int nl = FAST ? 1 : leaf.d.num_leaves;
    for (int k = 0; k < nl; ++k) { acc0[k] = 0; acc1[k] = 0; }
    for (int64_t k = k_begin; k < k_end; ++k) {
      const int party = p.party[k] & 1;
      Block4 s0, s1;
      uint32_t t0, t1;
      if (p.seeds_in) {
        const int64_t o0 = k * P + q0, o1 = k * P + q1;
        s0 = load_block(p.seeds_in + o0);
        t0 = p.ctrl_in[o0] & 1u;
        s1 = load_block(p.seeds_in + o1);
        t1 = p.ctrl_in[o1] & 1u;
      } else {
        s0 = s1 = load_block(p.key_seed + k);
        t0 = t1 = (uint32_t)party;
      }
      const dpf_block* cws = p.cw_seed + k * p.cw_stride;
      const uint8_t* cl = p.cw_left + k * p.cw_stride;
      const uint8_t* cr = p.cw_right + k * p.cw_stride;
      for (int j = 0; j < L; ++j) {
        const uint32_t b0 = path_bit(path0, L - 1 - j + bb), b1 = path_bit(path1, L - 1 - j + bb);
        const dpf_block c = cws[j];
        const uint32_t cctl = (uint32_t)(cl[j] & 1) | ((uint32_t)(cr[j] & 1) << 1);
        const uint4 cs = make_uint4((uint32_t)c.low, (uint32_t)(c.low >> 32), (uint32_t)c.high,
                                    (uint32_t)(c.high >> 32));
        if constexpr (PAIRED)
          path_step2(lk, lk.ks.l, lk.ks.d, s0, t0, b0, s1, t1, b1, cs, cctl);
        else
          path_step(lk, lk.ks.l, lk.ks.d, s0, t0, b0, cs, cctl);
      }
      const dpf_block* vcw = p.vcw + k * p.vcw_stride;
      if constexpr (FAST) {
        Block4 h0 = s0, h1 = s1;
        if constexpr (PAIRED)
          dpf_aes::mmo_hash2(h0, h1, lk, UniformRK{lk.ks.v}, UniformRK{lk.ks.v});
        else
          h0 = dpf_aes::mmo_hash(h0, lk, UniformRK{lk.ks.v});
        const u128 v0 = fast_point_value<BITS>(h0, t0, bi0, dpf_u128(vcw[bi0]), party, p.xor_mode);
        const u128 v1 =
            PAIRED ? fast_point_value<BITS>(h1, t1, bi1, dpf_u128(vcw[bi1]), party, p.xor_mode) : v0;
        if (SUM) {
          acc0[0] = p.xor_mode ? (acc0[0] ^ v0) : (acc0[0] + v0);
          acc1[0] = p.xor_mode ? (acc1[0] ^ v1) : (acc1[0] + v1);
        } else {
          store_bits<BITS>(p.out + (k * P + q0) * (int64_t)p.esz, v0);
          if (has1) store_bits<BITS>(p.out + (k * P + q1) * (int64_t)p.esz, v1);
        }
      } else {
        if (SUM) {
          u128 v[DPF_MAX_LEAVES];
          generic_point_values(leaf, lk, lk.ks.v, s0, t0, bi0, vcw, party, v);
          for (int e = 0; e < nl; ++e) acc0[e] = leaf_group_add(leaf.d, e, acc0[e], v[e]);
          generic_point_values(leaf, lk, lk.ks.v, s1, t1, bi1, vcw, party, v);
          for (int e = 0; e < nl; ++e) acc1[e] = leaf_group_add(leaf.d, e, acc1[e], v[e]);
        } else {
          GenericLeaf lf = leaf;
          lf.vcw = vcw;
          lf.party = party;
          lf.convert_store(lk, lk.ks.v, s0, t0, bi0, 1, p.out + (k * P + q0) * (int64_t)p.esz);
          if (has1)
            lf.convert_store(lk, lk.ks.v, s1, t1, bi1, 1, p.out + (k * P + q1) * (int64_t)p.esz);
        }
      }
    }
    if (SUM && k_begin < k_end) {
      for (int e = 0; e < nl; ++e) {
        const bool x = FAST ? p.xor_mode != 0 : leaf.d.kind[e] == DPF_LEAF_XOR;
        unsigned long long* w0 = p.wide + (q0 * nl + e) * 3;
        if (x) wide_xor(w0, acc0[e]); else wide_add(w0, acc0[e]);
        if (has1) {
          unsigned long long* w1 = p.wide + (q1 * nl + e) * 3;
          if (x) wide_xor(w1, acc1[e]); else wide_add(w1, acc1[e]);
        }
      }
    }
  }
}

// Counts points >= 2^log_domain_size (EvaluateAt's range check, h:861-874).
__global__ void count_out_of_range_kernel(int64_t n, const dpf_block* __restrict__ pts, int log,
                                          unsigned long long* __restrict__ bad) {
  unsigned long long c = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const dpf_block b = pts[i];
    bool out;
    if (log >= 128) out = false;
    else if (log >= 64) out = (b.high >> (log - 64)) != 0;
    else out = b.high != 0 || (b.low >> log) != 0;
    c += out ? 1 : 0;
  }
  // Wave-level reduction, one atomic per wave.
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, c);
}

__global__ void gather_kernel(int64_t rows, int64_t count, int elem_size,
                              const int64_t* __restrict__ src, const char* __restrict__ in,
                              char* __restrict__ out) {
  const int64_t total = rows * count * elem_size;
  const int64_t row_bytes = count * elem_size;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i / row_bytes, c = i - r * row_bytes;
    out[i] = in[src[r] * elem_size + c];
  }
}

__global__ void sum_shares_kernel(int64_t num_keys, int64_t row_len, int bits, int xor_mode,
                                  const char* __restrict__ shares, uint64_t* __restrict__ sums) {
  const int eb = bits / 8;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < row_len;
       j += (int64_t)gridDim.x * blockDim.x) {
    uint64_t acc = 0;
    for (int64_t k = 0; k < num_keys; ++k) {
      const char* p = shares + (k * row_len + j) * eb;
      uint64_t v = 0;
      if (eb == 8) v = *reinterpret_cast<const uint64_t*>(p);
      else if (eb == 4) v = *reinterpret_cast<const uint32_t*>(p);
      else if (eb == 2) v = *reinterpret_cast<const uint16_t*>(p);
      else v = *reinterpret_cast<const uint8_t*>(p);
      acc = xor_mode ? (acc ^ v) : (acc + v);
    }
    sums[j] = acc;
  }
}

// ------------------------------------------------------------------------
// Host-side launch helpers
// ------------------------------------------------------------------------
}  // namespace

namespace dpf_rt {
int num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

int block_for(int64_t work_items) {
  // A launch smaller than one full workgroup per CU runs LDS-bound on the few
  // CUs it occupies: give each CU a smaller workgroup instead (the tables cost
  // ~1 us to fill whatever the workgroup size).
  const int64_t cus = num_cus();
  int64_t per_cu = (work_items + cus - 1) / cus;
  int64_t b = (per_cu + 63) / 64 * 64;
  if (b < 64) b = 64;
  if (b > kBlock) b = kBlock;
  return (int)b;
}

int64_t dynamic_chunks_per_wg(int64_t items, int grid, int block, const char* env) {
  const char* v = env ? std::getenv(env) : nullptr;
  if (v && v[0] == '0') return 0;
  const int64_t chunks = (items + 63) / 64;
  if (chunks < (int64_t)grid * (block / 64) * 4) return 0;
  return (chunks + grid - 1) / grid;
}

int grid_for(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  int64_t cap = num_cus() * kWgPerCu;  // one 128 KiB-LDS workgroup per CU
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

int validate_desc(const dpf_value_desc* d) {
  if (!d) return fail(kInvalidArgument, "value descriptor is NULL");
  if (d->num_leaves < 1 || d->num_leaves > DPF_MAX_LEAVES)
    return fail(kUnimplemented, "value type has too many leaves for the GPU path");
  if (d->blocks_needed < 1 || d->blocks_needed > kBMax)
    return fail(kUnimplemented, "value type needs too many AES blocks for the GPU path");
  if (d->elements_per_block < 1) return fail(kInvalidArgument, "elements_per_block < 1");
  for (int k = 0; k < d->num_leaves; ++k) {
    int b = d->bits[k];
    if (b < 8 || b > 128 || (b & (b - 1)))
      return fail(kUnimplemented, "leaf bit size must be a power of two in [8, 128]");
    if (d->kind[k] == DPF_LEAF_INTMODN && d->mod_low[k] == 0 && d->mod_high[k] == 0)
      return fail(kInvalidArgument, "IntModN modulus is zero");
  }
  return kOk;
}

int packed_size(const dpf_value_desc* d) {
  int s = 0;
  for (int k = 0; k < d->num_leaves; ++k) s += d->bits[k] / 8;
  return s;
}

bool fast_int(const dpf_value_desc* d) {
  return d->num_leaves == 1 && d->direct && d->blocks_needed == 1 &&
         d->kind[0] != DPF_LEAF_INTMODN;
}


}  // namespace dpf_rt

namespace {

template <class Leaf>
const char* leaf_name() {
  if constexpr (std::is_same_v<Leaf, SwarLeaf>) return "swar";
  else if constexpr (std::is_same_v<Leaf, GenericLeaf>) return "generic";
  else if constexpr (std::is_same_v<Leaf, Mod32Leaf<2>> || std::is_same_v<Leaf, Mod32Leaf<4>> ||
                     std::is_same_v<Leaf, Mod32Leaf<kMod32MaxLeaves>>) return "mod32";
  else return "fast";
}

// Records the launch for dpf_hip_last_expand_kernel().
template <class Leaf>
void note_expand(const ExpandParams& p, bool octet) {
  static const std::string pair = std::string("pair/") + leaf_name<Leaf>();
  static const std::string oct = std::string("octet/") + leaf_name<Leaf>();
  g_last_expand = octet ? oct.c_str() : pair.c_str();
  g_last_expand_s = p.S;
}

// Latency mode for small trees (expand_small_kernel): num_starts << t
// workgroups, t as large as keeps them within one per CU, and D = L - t
// levels breadth-first in each; D must be 1..kSmallMaxD.  Returns false (and
// launches nothing) when the tree does not fit that shape.  DPF_EXPAND_SMALL=0
// (read per launch) turns it off: the A/B and test hook.
bool small_on() {
  const char* v = std::getenv("DPF_EXPAND_SMALL");
  return !(v && v[0] == '0');
}
bool small_shape(int64_t num_starts, int num_levels, int* t, int* D) {
  const int64_t cus = num_cus();
  if (!small_on() || num_levels < 1 || num_starts < 1 || num_starts > cus) return false;
  int tt = 0;
  while (tt < num_levels - 1 && (num_starts << (tt + 1)) <= cus) ++tt;
  const int d = num_levels - tt;
  if (d < 1 || d > kSmallMaxD) return false;
  *t = tt;
  *D = d;
  return true;
}
// Launches expand_small_kernel<Leaf> when the tree has the small shape.
template <class Leaf>
bool try_small(const ExpandParams& p0, const Leaf& leaf, hipStream_t s) {
  int t = 0, D = 0;
  const int64_t starts = p0.num_items >> p0.k0;
  if (!small_shape(starts, p0.num_levels, &t, &D)) return false;
  ExpandParams p = p0;
  p.k0 = t;
  p.S = D;
  p.num_items = starts << t;
  static const std::string name = std::string("small/") + leaf_name<Leaf>();
  g_last_expand = name.c_str();
  g_last_expand_s = D;
  hipLaunchKernelGGL((expand_small_kernel<Leaf>), dim3((unsigned)p.num_items), dim3(kBlock), 0, s,
                     p, leaf);
  return true;
}


// Tree-top pass of an octet launch (r16).  Every octet-kernel item walks k0
// levels from its start seed to its subtree root, one dependent AES per level
// per lane: at config 2's 2^30 outputs 18 of each lane's ~6160 AES, but at
// the 2^27-output shard a rank evaluates in an 8-GPU run (784 AES per lane)
// the walk is ~4.5% of the kernel.  Instead, expand_small_kernel<SeedLeaf>
// expands the top of the tree breadth-first -- each workgroup's wave 0 walks
// to its subtree root in lane quads, then up to 11 levels through LDS, every
// node hashed once -- and writes the 2^k0-per-start item roots (17 B each,
// stream-ordered scratch); the octet kernel then starts at them (k0 = 0).
// DPF_EXPAND_TOP=0 (read per launch) keeps the per-lane walk.
bool top_on() {
  const char* v = std::getenv("DPF_EXPAND_TOP");
  return !(v && v[0] == '0');
}
struct TopScratch {
  void* mem = nullptr;
  hipStream_t s = nullptr;
  ~TopScratch() {
    if (mem) (void)hipFreeAsync(mem, s);
  }
};
// Returns the error of a failed launch, else kOk (p rewritten when the pass ran).
int expand_top(ExpandParams& p, hipStream_t s, TopScratch& scratch) {
  const int64_t starts = p.num_items >> p.k0;
  // Few start seeds (full-domain calls and their shards): with many starts
  // every item's walk is short and a workgroup per start would idle.
  if (!top_on() || p.k0 < 8 || starts > num_cus() || p.num_items < 4 * (int64_t)num_cus())
    return kOk;
  // Workgroups: one per subtree at depth t under each start, at least one
  // per CU; D = k0 - t levels breadth-first (1..kSmallMaxD).
  int t = 0;
  while ((starts << t) < num_cus() && t < p.k0 - 1) ++t;
  if (p.k0 - t > kSmallMaxD) t = p.k0 - kSmallMaxD;
  const int D = p.k0 - t;
  if (D < 1 || (starts << t) > INT32_MAX) return kOk;
  static const bool pool_kept = [] {
    int dev = 0;
    hipMemPool_t pool;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetDefaultMemPool(&pool, dev) != hipSuccess)
      return false;
    uint64_t keep = UINT64_MAX;
    return hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep) == hipSuccess;
  }();
  (void)pool_kept;
  const size_t items = (size_t)p.num_items;
  void* mem = nullptr;
  HIP_TRY(hipMallocAsync(&mem, items * (sizeof(dpf_block) + 1), s));
  scratch.mem = mem;
  scratch.s = s;
  SeedLeaf leaf{static_cast<dpf_block*>(mem),
                static_cast<uint8_t*>(mem) + items * sizeof(dpf_block)};
  ExpandParams q = p;
  q.k0 = t;
  q.S = D;
  q.num_levels = p.k0;
  q.num_items = starts << t;
  q.clock = nullptr;
  hipLaunchKernelGGL((expand_small_kernel<SeedLeaf>), dim3((unsigned)q.num_items), dim3(kBlock), 0,
                     s, q, leaf);
  HIP_TRY(hipGetLastError());
  // The octet kernel starts at the item roots: k0 = 0, correction words from
  // level k0 on.
  p.seeds_in = leaf.seeds;
  p.ctrl_in = leaf.ctrl;
  p.cw_seed += p.k0;
  p.cw_left += p.k0;
  p.cw_right += p.k0;
  p.num_levels = p.S;
  p.k0 = 0;
  return kOk;
}

// Dynamic item distribution for the octet kernel (ExpandParams::dyn_chunks):
// a launch with at least 4 items per thread of one full workgroup per CU
// gets subtrees two levels shallower (4x the items, the two levels above
// them done by the tree-top pass) so every wave can take several chunks of
// 64 items from its workgroup's counter.  Applied only when the tree-top
// pass starts the items (k0 = 0 after it): otherwise every item would walk
// two more levels.  DPF_OCTET_DYNAMIC=0 (read per launch) keeps the static
// one-item-per-thread shape, =<1..4> sets the levels taken off the subtrees
// (2^that items per thread; A/B and test hook).  Default: 4 levels off
// subtrees of >= 11 (config 2 15.00 vs 15.05-15.17 ms, config 3's uint128
// shard 58.2 vs 60.9 ms, Tuple<IntModN32 x 2> 39.2 vs 40.9 ms), else 2 (the
// 2^27 / 2^28 shards 1.96 / 3.82 ms at 2 vs 2.04 / 3.90 at 4; 3 was worse than
// both everywhere; profiles/r16/octet_dynamic_ab.txt).
int octet_dynamic_shift(int S) {
  const char* v = std::getenv("DPF_OCTET_DYNAMIC");
  if (!v || !*v) return S >= 11 ? 4 : 2;
  const int k = std::atoi(v);
  return k <= 0 ? 0 : (k > 4 ? 4 : k);
}
// Levels each dynamically taken item walks below the tree-top pass's roots
// (DPF_OCTET_WALK=<n>, read per launch; 0: the pass goes down to the items).
int octet_walk_levels() {
  const char* v = std::getenv("DPF_OCTET_WALK");
  if (!v || !*v) return 2;
  const int k = std::atoi(v);
  return k < 0 ? 0 : (k > 4 ? 4 : k);
}
// Runs the tree-top pass and sets p's shape (and *grid, *blk) for the octet
// kernel launch.
int subtree_shape(ExpandParams& p, int min_S, hipStream_t s, TopScratch& top, int* grid,
                  int* blk) {
  p.dyn_chunks = 0;
  const int64_t cus = num_cus();
  const int sh = octet_dynamic_shift(p.S);
  if (sh > 0 && p.S - sh >= min_S && p.k0 + sh <= 62 &&
      (p.num_items << sh) % (cus * 64) == 0 && (p.num_items << sh) >= 4 * cus * kBlock) {
    ExpandParams q = p;
    q.S -= sh;
    q.k0 += sh;
    q.num_items <<= sh;
    q.dyn_chunks = (int)(q.num_items / (cus * 64));
    // The tree-top pass stops `w` levels above the items (a quarter of the
    // roots for w = 2: fewer rounds of its latency-bound workgroups), and
    // every item walks those levels itself (one path step per level, in the
    // octet kernel's throughput mode).
    const int w = octet_walk_levels();
    if (w > 0 && q.k0 - w >= 8) {
      ExpandParams t = q;
      t.k0 = q.k0 - w;
      t.S = q.S + w;
      t.num_items = q.num_items >> w;
      if (int st = expand_top(t, s, top)) return st;
      if (t.k0 == 0) {
        q.seeds_in = t.seeds_in;
        q.ctrl_in = t.ctrl_in;
        q.cw_seed = t.cw_seed;
        q.cw_left = t.cw_left;
        q.cw_right = t.cw_right;
        q.num_levels = q.S + w;
        q.k0 = w;
        p = q;
        *grid = (int)cus;
        *blk = kBlock;
        return kOk;
      }
    }
    if (int st = expand_top(q, s, top)) return st;
    if (q.k0 == 0) {
      p = q;
      *grid = (int)cus;
      *blk = kBlock;
      return kOk;
    }
  }
  if (int st = expand_top(p, s, top)) return st;
  *blk = block_for(p.num_items);
  *grid = grid_for(p.num_items, *blk);
  return kOk;
}
int octet_shape(ExpandParams& p, hipStream_t s, TopScratch& top, int* grid, int* blk) {
  return subtree_shape(p, 3, s, top, grid, blk);
}

template <class Leaf>
int launch_expand(const ExpandParams& p0, const Leaf& leaf, hipStream_t s) {
  // GenericLeaf's conversion spills in the small kernel's register budget and
  // measured 0.93-1.07x there (profiles/r15_ab.txt part 13): not dispatched.
  if (!std::is_same_v<Leaf, GenericLeaf> && try_small(p0, leaf, s)) {
    HIP_TRY(hipGetLastError());
    return kOk;
  }
  note_expand<Leaf>(p0, false);
  // The octet kernel's shape (tree-top pass, dynamic 64-item chunks) with
  // pair leaves: subtrees of >= 1 level.
  ExpandParams p = p0;
  TopScratch top;
  int grid = 0, blk = 0;
  if (int st = subtree_shape(p, 1, s, top, &grid, &blk)) return st;
  hipLaunchKernelGGL(expand_kernel<Leaf>, dim3(grid), dim3(blk), 0, s, p, leaf);
  HIP_TRY(hipGetLastError());
  return kOk;
}

// The octet kernel takes integer leaves filling whole blocks whenever the
// subtrees have >= 8 leaves (DPF_EXPAND_NO_OCTET=1 forces expand_kernel).
template <int BITS, bool XOR>
bool launch_octet(const ExpandParams& p0, const dpf_block* vcw, int E, int party, int store_bytes,
                  hipStream_t s, int* st) {
  const char* off = getenv("DPF_EXPAND_NO_OCTET");
  if ((off && off[0] == '1') || store_bytes != 16 || p0.S < 3) return false;
  note_expand<FastIntLeaf<BITS, XOR>>(p0, true);
  ExpandParams p = p0;
  TopScratch top;
  int grid = 0, blk = 0;
  if ((*st = octet_shape(p, s, top, &grid, &blk)) != kOk) return true;
  hipLaunchKernelGGL((expand_octet_kernel<FastIntLeaf<BITS, XOR>>), dim3(grid), dim3(blk), 0, s, p,
                     FastIntLeaf<BITS, XOR>{vcw, E, party, store_bytes, {}});
  return true;
}

template <int BITS>
int launch_expand_fast(const ExpandParams& p, const dpf_value_desc* d, const dpf_block* vcw,
                       int E, int party, int store_bytes, hipStream_t s) {
  if (d->kind[0] == DPF_LEAF_XOR ? try_small(p, FastIntLeaf<BITS, true>{vcw, E, party, store_bytes, {}}, s)
                                 : try_small(p, FastIntLeaf<BITS, false>{vcw, E, party, store_bytes, {}}, s)) {
    HIP_TRY(hipGetLastError());
    return kOk;
  }
  int st = kOk;
  if (d->kind[0] == DPF_LEAF_XOR ? launch_octet<BITS, true>(p, vcw, E, party, store_bytes, s, &st)
                                 : launch_octet<BITS, false>(p, vcw, E, party, store_bytes, s, &st)) {
    if (st != kOk) return st;
    HIP_TRY(hipGetLastError());
    return kOk;
  }
  if (d->kind[0] == DPF_LEAF_XOR)
    return launch_expand(p, FastIntLeaf<BITS, true>{vcw, E, party, store_bytes, {}}, s);
  return launch_expand(p, FastIntLeaf<BITS, false>{vcw, E, party, store_bytes, {}}, s);
}

// Integer leaves, four path chains per lane (ILP4): item u covers key grp and
// the points q + j * quarter, j < 4 (p.half holds the quarter).  Same
// arithmetic as eval_points_kernel<GenericLeaf, BITS, true, ...>, one more
// pair of chains in flight per wave (points_ilp below picks it).
template <int BITS, bool UNIFORM, bool SUM, bool TOP>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void eval_points4_kernel(PointParams p) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h)
  fill_tables(lds.tab);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const LdsLookup lk = make_lookup(lds, KeySet{key_ref(p.rkl), KeyRef{}, key_ref(p.rkv), key_ref(p.rkd)});
  const int L = p.num_levels;
  const int64_t P = p.points_per_key, quarter = p.half;
  // Sums of <= 64-bit values wrap mod 2^64 exactly (the group is mod 2^BITS).
  using Acc = typename std::conditional<(BITS <= 64), uint64_t, u128>::type;
  // Items by grid stride, or 64 at a time per wave (dyn_per_wg > 0).
  const int64_t nch = (p.num_items + 63) / 64;
  for (int64_t u = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.num_items)
                                : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       u < p.num_items;
       u = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.num_items)
                        : u + (int64_t)gridDim.x * blockDim.x) {
    int64_t grp = u / quarter;
    if (UNIFORM) grp = (int64_t)__builtin_amdgcn_readfirstlane((int)grp);
    const int64_t q0 = u - grp * quarter;
    // Point i of the item: q0 + i * quarter (clamped to q0 past the key's last point).
    auto qi = [&](int i) { return q0 + i * quarter < P ? q0 + i * quarter : q0; };
    auto pidx = [&](int i) { return p.shared_points ? qi(i) : grp * P + qi(i); };
    int64_t k_begin = grp, k_end = grp + 1;
    if (SUM) {
      k_begin = grp * p.chunk_keys;
      k_end = k_begin + p.chunk_keys < p.num_keys ? k_begin + p.chunk_keys : p.num_keys;
    }
    Block4 path[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) path[i] = load_block(p.tree_index + pidx(i));
    Acc acc[4] = {0, 0, 0, 0};
    for (int64_t k = k_begin; k < k_end; ++k) {
      const int party = p.party[k] & 1;
      Block4 st[4];
      uint32_t t[4];
      if (p.seeds_in) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          st[i] = load_block(p.seeds_in + k * P + qi(i));
          t[i] = p.ctrl_in[k * P + qi(i)] & 1u;
        }
      } else {
        const Block4 root = load_block(p.key_seed + k);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          st[i] = root;
          t[i] = (uint32_t)party;
        }
      }
      const dpf_block* cws = p.cw_seed + k * p.cw_stride;
      const uint8_t* cl = p.cw_left + k * p.cw_stride;
      const uint8_t* cr = p.cw_right + k * p.cw_stride;
      // Shared top (top_levels = 6, walks from the root): the wave's 256
      // points of this key share its top 6 levels, so lane l walks them once
      // for the prefix whose 6 path bits are l (one AES per level instead of
      // four), and each chain takes its depth-6 node from the lane its own
      // top bits name (ds_bpermute, no LDS allocation).
      // 6 levels in the key sum; 4 per key, whose instance schedules its path
      // loop as the full walk does only with the shorter top (ISA: 9 waits in
      // the round block vs 40 with 6 levels).
      constexpr int j0 = TOP ? (SUM ? 6 : 4) : 0;
      if (TOP) {
        const uint32_t lane = threadIdx.x & 63;
        Block4 ts = st[0];
        uint32_t tt = t[0];
        for (int j = 0; j < j0; ++j) {
          const dpf_block c = cws[j];
          const uint32_t cctl = (uint32_t)(cl[j] & 1) | ((uint32_t)(cr[j] & 1) << 1);
          const uint32_t b = (lane >> (j0 - 1 - j)) & 1u;
          Block4 h = dpf_aes::mmo_hash(ts, lk, SelectRK{lk.ks.l, lk.ks.d, 0u - b});
          const uint32_t m = 0u - tt;
          h.w0 ^= (uint32_t)c.low & m;
          h.w1 ^= (uint32_t)(c.low >> 32) & m;
          h.w2 ^= (uint32_t)c.high & m;
          h.w3 ^= (uint32_t)(c.high >> 32) & m;
          tt = (h.w0 & 1u) ^ (tt & ((cctl >> b) & 1u));
          h.w0 &= ~1u;
          ts = h;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint32_t src = 0;
          for (int j = 0; j < j0; ++j) src = (src << 1) | path_bit(path[i], L - 1 - j + p.bib);
          const int a = (int)(src << 2);
          st[i] = Block4{(uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)ts.w0),
                         (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)ts.w1),
                         (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)ts.w2),
                         (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)ts.w3)};
          t[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)tt);
        }
      }
      for (int j = j0; j < L; ++j) {
        const dpf_block c = cws[j];
        const uint32_t cctl = (uint32_t)(cl[j] & 1) | ((uint32_t)(cr[j] & 1) << 1);
        uint32_t b[4];
        SelectRK rk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          b[i] = path_bit(path[i], L - 1 - j + p.bib);
          rk[i] = SelectRK{lk.ks.l, lk.ks.d, 0u - b[i]};
        }
        Block4 h[4] = {st[0], st[1], st[2], st[3]};
        dpf_aes::mmo_hashN<4>(h, lk, rk);
        const uint32_t cw[4] = {(uint32_t)c.low, (uint32_t)(c.low >> 32), (uint32_t)c.high,
                                (uint32_t)(c.high >> 32)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t m = 0u - t[i];
          h[i].w0 ^= cw[0] & m; h[i].w1 ^= cw[1] & m; h[i].w2 ^= cw[2] & m; h[i].w3 ^= cw[3] & m;
          t[i] = (h[i].w0 & 1u) ^ (t[i] & ((cctl >> b[i]) & 1u));
          h[i].w0 &= ~1u;
          st[i] = h[i];
        }
      }
      const dpf_block* vcw = p.vcw + k * p.vcw_stride;
      const UniformRK vk[4] = {UniformRK{lk.ks.v}, UniformRK{lk.ks.v}, UniformRK{lk.ks.v},
                               UniformRK{lk.ks.v}};
      dpf_aes::mmo_hashN<4>(st, lk, vk);
      const uint32_t bmask = (1u << p.bib) - 1u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int bi = p.block_index ? p.block_index[pidx(i)] : (int)(path[i].w0 & bmask);
        const u128 v = fast_point_value<BITS>(st[i], t[i], bi, dpf_u128(vcw[bi]), party, p.xor_mode);
        if (SUM)
          acc[i] = p.xor_mode ? (acc[i] ^ (Acc)v) : (acc[i] + (Acc)v);
        else if (q0 + i * quarter < P)
          store_bits<BITS>(p.out + (k * P + qi(i)) * (int64_t)p.esz, v);
      }
    }
    if (SUM && k_begin < k_end) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (q0 + i * quarter >= P) continue;
        unsigned long long* w = p.wide + qi(i) * 3;
        if (p.xor_mode) wide_xor(w, (u128)acc[i]); else wide_add(w, (u128)acc[i]);
      }
    }
  }
}

// Latency mode of eval_points_kernel<GenericLeaf, BITS, true, ..> for small
// calls (no sum): one (key, point) per lane QUAD, lane c computing column c
// of every AES (dpf_device.h quad::), so one path walk runs ~2x faster than
// on one lane when the launch is far below a wave per SIMD.
template <int BITS>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void eval_points_quad_kernel(PointParams p) {
  __shared__ LdsImage lds;
  fill_tables(lds.tab);
  __syncthreads();
  const LdsLookup lk = make_lookup(lds);
  const quad::Keys kl = quad::keys_of(p.rkl), kd = quad::keys_of(p.rkd), kv = quad::keys_of(p.rkv);
  const int L = p.num_levels;
  const int64_t P = p.points_per_key;
  const int c = quad::column();
  const uint32_t bmask = (1u << p.bib) - 1u;
  // The stride is a multiple of 64, so the four lanes of a quad stay together.
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; (g >> 2) < p.num_items;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = g >> 2;  // item = key k, point q
    const int64_t k = u / P, q = u - k * P;
    const int64_t pi = p.shared_points ? q : u;
    const Block4 path = load_block(p.tree_index + pi);
    const int bi = p.block_index ? p.block_index[pi] : (int)(path.w0 & bmask);
    const int party = p.party[k] & 1;
    uint32_t s, t;
    if (p.seeds_in) {
      s = reinterpret_cast<const uint32_t*>(p.seeds_in + u)[c];
      t = p.ctrl_in[u] & 1u;
    } else {
      s = reinterpret_cast<const uint32_t*>(p.key_seed + k)[c];
      t = (uint32_t)party;
    }
    const dpf_block* cws = p.cw_seed + k * p.cw_stride;
    const uint8_t* cl = p.cw_left + k * p.cw_stride;
    const uint8_t* cr = p.cw_right + k * p.cw_stride;
    for (int j = 0; j < L; ++j) {
      const uint32_t bit = path_bit(path, L - 1 - j + p.bib);
      const uint32_t cs = reinterpret_cast<const uint32_t*>(cws + j)[c];
      const uint32_t cctl = (uint32_t)(cl[j] & 1) | ((uint32_t)(cr[j] & 1) << 1);
      quad::path_step(lk, kl, kd, s, t, bit, cs, cctl);
    }
    const Block4 h = quad::gather(quad::mmo(s, lk, kv, kv, 0u));
    if (c == 0) {
      const dpf_block* vcw = p.vcw + k * p.vcw_stride;
      store_bits<BITS>(p.out + u * (int64_t)p.esz,
                       fast_point_value<BITS>(h, t, bi, dpf_u128(vcw[bi]), party, p.xor_mode));
    }
  }
}

// DPF_POINTS_QUAD=0 (read per launch) turns the latency mode off (A/B hook).
bool points_quad_on() {
  const char* v = std::getenv("DPF_POINTS_QUAD");
  return !(v && v[0] == '0');
}
// Launches of at most this many points run in latency mode: num_cus x 256 by
// default, i.e. as many lane quads as one pass of 1024-thread workgroups on
// every CU holds.  BatchEvaluation/10/40000 (40000 points per call) 2.54-2.63
// -> 1.46-1.58 ms; /1/400000 stays on the lane chains (the quads would loop:
// 1.01-1.17 vs 0.97-1.00 ms); profiles/r15_ab.txt part 19.
// DPF_POINTS_QUAD_MAX=<points> (read per launch) moves the cut-over (A/B hook).
int64_t points_quad_max() {
  const char* v = std::getenv("DPF_POINTS_QUAD_MAX");
  const long long m = v && *v ? std::strtoll(v, nullptr, 10) : 0;
  return m > 0 ? (int64_t)m : (int64_t)num_cus() * 256;
}

// DPF_POINTS_ILP=2|4 (read per launch) forces two or four chains per lane
// (four only where a quarter of a key's points is a whole number of waves);
// by default integer leaves take four chains when the launch fills every CU
// with 1024-thread workgroups (config 4: +0.7% per key, +1.4% summed over
// keys, profiles/r14_ab.txt) and two otherwise.
int points_ilp() {
  const char* v = std::getenv("DPF_POINTS_ILP");
  return v && (v[0] == '2' || v[0] == '4') ? v[0] - '0' : 0;
}
thread_local const char* g_last_points_kernel = "";

template <class Leaf, int BITS, bool FAST, bool SUM>
int launch_points_t(const PointParams& pp, const Leaf& leaf, hipStream_t s) {
  if constexpr (FAST) {
    // ILP4: quarter = ceil(P / 4) points per chain row; enough items to fill the chip.
    const int64_t quarter = (pp.points_per_key + 3) / 4;
    const int64_t items = SUM ? pp.num_items / pp.half * quarter : pp.num_keys * quarter;
    const int ilp = points_ilp();
    if (quarter % 64 == 0 &&
        (ilp == 4 || (ilp == 0 && items >= (int64_t)num_cus() * 1024))) {
      g_last_points_kernel = "points/ilp4";
      PointParams p = pp;
      p.half = quarter;
      p.num_items = items;
      const int blk = block_for(p.num_items);
      const int grid = grid_for(p.num_items, blk);
      // DPF_POINTS_DYNAMIC=0: a fixed share of items per thread (A/B hook).
      p.dyn_per_wg = dynamic_chunks_per_wg(p.num_items, grid, blk, "DPF_POINTS_DYNAMIC");
      // The shared top (profiles/r16/points_shared_top_ab.txt): summed over
      // keys 6 levels, 1236 vs 1275 ms; per key 4 levels (6 measured 1358 vs
      // 1258 ms, r16h).  DPF_POINTS_SHARED_TOP=0 turns it off (A/B hook).
      const char* top = std::getenv("DPF_POINTS_SHARED_TOP");
      const bool want_top = !(top && top[0] == '0');
      p.top_levels = want_top && !p.seeds_in && p.num_levels >= 6 ? 6 : 0;
      if (p.top_levels)
        hipLaunchKernelGGL((eval_points4_kernel<BITS, true, SUM, true>), dim3(grid), dim3(blk), 0, s, p);
      else
        hipLaunchKernelGGL((eval_points4_kernel<BITS, true, SUM, false>), dim3(grid), dim3(blk), 0, s, p);
      HIP_TRY(hipGetLastError());
      return kOk;
    }
  }
  if constexpr (!SUM) {
    // Up to one pass of lane quads over every CU: one lane quad per point.
    const int64_t points = pp.num_keys * pp.points_per_key;
    if (FAST && points <= points_quad_max() && points_ilp() == 0 && points_quad_on()) {
      g_last_points_kernel = "points/quad";
      PointParams p = pp;
      p.num_items = points;
      const int blk = block_for(points * 4);
      hipLaunchKernelGGL((eval_points_quad_kernel<BITS>), dim3(grid_for(points * 4, blk)),
                         dim3(blk), 0, s, p);
      HIP_TRY(hipGetLastError());
      return kOk;
    }
    // Fewer paired items than one wave per CU: latency-bound, run unpaired.
    if (pp.num_items < (int64_t)num_cus() * 64 && points_ilp() != 2) {
      g_last_points_kernel = "points/single";
      PointParams p = pp;
      p.half = p.points_per_key;
      p.num_items = p.num_keys * p.points_per_key;
      const int blk = block_for(p.num_items);
      const dim3 grid(grid_for(p.num_items, blk)), block(blk);
      if (p.half % 64 == 0)
        hipLaunchKernelGGL((eval_points_kernel<Leaf, BITS, FAST, true, false, false>), grid, block,
                           0, s, p, leaf);
      else
        hipLaunchKernelGGL((eval_points_kernel<Leaf, BITS, FAST, false, false, false>), grid,
                           block, 0, s, p, leaf);
      HIP_TRY(hipGetLastError());
      return kOk;
    }
  }
  g_last_points_kernel = "points/ilp2";
  PointParams p = pp;
  const int blk = block_for(p.num_items);
  const dim3 grid(grid_for(p.num_items, blk)), block(blk);
  p.dyn_per_wg = dynamic_chunks_per_wg(p.num_items, (int)grid.x, blk, "DPF_POINTS_DYNAMIC");
  if (p.half % 64 == 0)
    hipLaunchKernelGGL((eval_points_kernel<Leaf, BITS, FAST, true, SUM>), grid, block, 0, s, p, leaf);
  else
    hipLaunchKernelGGL((eval_points_kernel<Leaf, BITS, FAST, false, SUM>), grid, block, 0, s, p, leaf);
  HIP_TRY(hipGetLastError());
  return kOk;
}

template <bool SUM>
int launch_points(const PointParams& p, const dpf_value_desc* desc, const dpf_block* vcw,
                  hipStream_t s) {
  if (fast_int(desc)) {
    switch (desc->bits[0]) {
      case 8: return launch_points_t<GenericLeaf, 8, true, SUM>(p, GenericLeaf{}, s);
      case 16: return launch_points_t<GenericLeaf, 16, true, SUM>(p, GenericLeaf{}, s);
      case 32: return launch_points_t<GenericLeaf, 32, true, SUM>(p, GenericLeaf{}, s);
      case 64: return launch_points_t<GenericLeaf, 64, true, SUM>(p, GenericLeaf{}, s);
      default: return launch_points_t<GenericLeaf, 128, true, SUM>(p, GenericLeaf{}, s);
    }
  }
  GenericLeaf g;
  g.d = *desc;
  g.vcw = vcw;
  g.party = 0;
  g.elements_per_leaf = 1;
  g.esz = packed_size(desc);
  return launch_points_t<GenericLeaf, 8, false, SUM>(p, g, s);
}

// Shared argument checks and parameter block of the two point entry points.
int make_point_params(int64_t num_keys, int64_t points_per_key, int num_levels,
                      const dpf_block* key_seed, const uint8_t* party, const dpf_block* seeds_in,
                      const uint8_t* control_in, const dpf_block* tree_index,
                      const int32_t* block_index, const dpf_block* cw_seed,
                      const uint8_t* cw_left, const uint8_t* cw_right,
                      const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                      const dpf_aes_key* key_value, const dpf_value_desc* desc,
                      const dpf_block* value_correction, PointParams* p) {
  int st = validate_desc(desc);
  if (st) return st;
  if (num_keys < 0 || points_per_key < 1 || num_levels < 0 || num_levels > 128)
    return fail(kInvalidArgument, "num_keys, points_per_key or num_levels out of range");
  if (!party || !tree_index || !key_left || !key_right || !key_value || !value_correction ||
      (!seeds_in && !key_seed) || (seeds_in && !control_in) ||
      (num_levels > 0 && (!cw_seed || !cw_left || !cw_right)))
    return fail(kInvalidArgument, "NULL pointer");
  memset(p, 0, sizeof(*p));
  p->num_keys = num_keys;
  p->points_per_key = points_per_key;
  p->half = (points_per_key + 1) / 2;
  p->num_levels = num_levels;
  p->cw_stride = num_levels;
  p->key_seed = key_seed;
  p->party = party;
  p->seeds_in = seeds_in;
  p->ctrl_in = control_in;
  p->tree_index = tree_index;
  p->block_index = block_index;
  p->cw_seed = cw_seed;
  p->cw_left = cw_left;
  p->cw_right = cw_right;
  p->vcw = value_correction;
  p->vcw_stride = desc->elements_per_block * desc->num_leaves;
  p->esz = packed_size(desc);
  p->xor_mode = desc->kind[0] == DPF_LEAF_XOR;
  p->dyn_per_wg = 0;
  p->top_levels = 0;
  p->rkl = expand_key(key_left);
  p->rkd = xor_keys(p->rkl, expand_key(key_right));
  p->rkv = expand_key(key_value);
  return kOk;
}

}  // namespace

// ==========================================================================
// C ABI
// ==========================================================================
extern "C" {

int dpf_hip_abi_version(void) { return DPF_HIP_ABI_VERSION; }
const char* dpf_hip_last_error(void) { return dpf_rt::g_last_error.c_str(); }

const char* dpf_hip_last_points_kernel(void) { return g_last_points_kernel; }
const char* dpf_hip_last_expand_kernel(int* subtree_depth) {
  if (subtree_depth) *subtree_depth = dpf_rt::g_last_expand_s;
  return dpf_rt::g_last_expand;
}

int dpf_hip_clock_probe(int on) {
  unsigned long long* old = dpf_rt::g_clock_acc.exchange(nullptr);
  if (old) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree(old));
  }
  if (!on) return kOk;
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, 4 * sizeof(unsigned long long)));
  HIP_TRY(hipMemset(p, 0, 4 * sizeof(unsigned long long)));
  HIP_TRY(hipDeviceSynchronize());
  dpf_rt::g_clock_acc.store(static_cast<unsigned long long*>(p));
  return kOk;
}

int dpf_hip_clock_probe_read(double* clock_ghz, int64_t* workgroups, double* mean_workgroup_s) {
  unsigned long long* acc = dpf_rt::g_clock_acc.load();
  if (!acc) return fail(kFailedPrecondition, "clock probe is off (dpf_hip_clock_probe(1))");
  unsigned long long h[4] = {0, 0, 0, 0};
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h, acc, sizeof(h), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemset(acc, 0, sizeof(h)));
  HIP_TRY(hipDeviceSynchronize());
  // s_memtime counts shader clocks, s_memrealtime a constant 100 MHz.
  if (clock_ghz) *clock_ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0.0;
  if (workgroups) *workgroups = (int64_t)h[2];
  if (mean_workgroup_s) *mean_workgroup_s = h[2] ? (double)h[1] / (double)h[2] * 1e-8 : 0.0;
  return kOk;
}

int dpf_hip_device_count(int* count) {
  HIP_TRY(hipGetDeviceCount(count));
  return kOk;
}
int dpf_hip_set_device(int device) {
  HIP_TRY(hipSetDevice(device));
  return kOk;
}
}  // extern "C"

namespace {
// Large copies between the device and pageable host memory: the runtime pins
// the user pages for each such copy, which measured ~28 ms per call for
// 4-128 MiB (tools/dpf_benchmark, BM_EvaluateRegularDpf at 2^22+ outputs)
// against ~0.3 ms for 16 MiB through page-locked memory.  They go through two
// page-locked 16 MiB bounce buffers instead, the DMA of one chunk overlapping
// the host copy of the other.
constexpr size_t kBounceMin = size_t{2} << 20;
constexpr size_t kBounceChunk = size_t{16} << 20;

// memcpy on up to 8 host threads for pieces of >= 2 MiB (the host side of a
// bounce runs at ~28 GB/s on 8 threads vs ~5 on one, page faults included).
void host_copy(void* dst, const void* src, size_t bytes) {
  const size_t piece = size_t{2} << 20;
  size_t t = bytes / piece;
  static const size_t hw = [] {
    const char* e = std::getenv("DPF_HOST_THREADS");   // as host_util.h HostThreads()
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 ? static_cast<size_t>(v) : static_cast<size_t>(std::thread::hardware_concurrency());
  }();
  if (t > 8) t = 8;
  if (hw && t > hw) t = hw;
  if (t <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> pool;
  for (size_t i = 0; i < t; ++i) {
    const size_t lo = bytes * i / t, hi = bytes * (i + 1) / t;
    pool.emplace_back([=] { memcpy((char*)dst + lo, (const char*)src + lo, hi - lo); });
  }
  for (auto& th : pool) th.join();
}
std::mutex g_bounce_mu;
char* g_bounce[2] = {nullptr, nullptr};

bool page_locked(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice ||
         a.type == hipMemoryTypeManaged;
}

int bounce_buffers() {
  for (auto& b : g_bounce)
    if (!b) HIP_TRY(hipHostMalloc((void**)&b, kBounceChunk, hipHostMallocDefault));
  return kOk;
}

int bounce_d2h(void* dst, const void* src, size_t bytes, void* stream) {
  std::lock_guard<std::mutex> lock(g_bounce_mu);
  if (int rc = bounce_buffers()) return rc;
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (bytes + kBounceChunk - 1) / kBounceChunk;
  auto len = [&](size_t i) { return i + 1 < n ? kBounceChunk : bytes - i * kBounceChunk; };
  HIP_TRY(hipMemcpyAsync(g_bounce[0], src, len(0), hipMemcpyDeviceToHost, s));
  for (size_t i = 0; i < n; ++i) {
    HIP_TRY(hipStreamSynchronize(s));   // chunk i is in g_bounce[i & 1]
    if (i + 1 < n)
      HIP_TRY(hipMemcpyAsync(g_bounce[(i + 1) & 1], (const char*)src + (i + 1) * kBounceChunk,
                             len(i + 1), hipMemcpyDeviceToHost, s));
    host_copy((char*)dst + i * kBounceChunk, g_bounce[i & 1], len(i));
  }
  return kOk;
}

// Large copies to or from pageable host memory: register the host range for
// the copy (16 ms for 8 GiB of mapped pages, tools/host_output_microbench.cc)
// and DMA straight into / out of it at the link rate (57 GB/s vs ~12 through
// the bounce buffers); the bounce path stays as the fallback when the
// registration is refused.
// Registering a fresh range (and unmapping it after) costs more than the
// page-locked staging below ~0.5 GiB (tools/fresh_output_microbench.cc,
// profiles/r14_fresh_output_microbench.jsonl): 32 MiB 4.5 vs 3.9 ms, 256 MiB
// 26.3 vs 25.9 ms; at 8 GiB the DMA straight into the range wins (42 vs ~28 GB/s).
constexpr size_t kRegisterMin = DPF_HIP_REGISTER_MIN_BYTES;
// The 512 MiB threshold prices the page faults of FRESH destinations.  A host
// range whose pages are already mapped -- every H2D source, and D2H
// destinations the caller has touched -- costs ~2 us/MiB to register (16 ms
// for 8 GiB, tools/host_output_microbench.cc) against a DMA at ~57 GB/s
// instead of ~12 GB/s through the bounce buffers, so those register from
// 32 MiB (the r13 threshold); profiles/r15_ab.txt (3), r15_mapped_register_ab.jsonl.
// DPF_HIP_REGISTER_MAPPED_MIB=<n> (read per call) overrides it: the A/B hook.
size_t register_min_mapped() {
  const char* v = std::getenv("DPF_HIP_REGISTER_MAPPED_MIB");
  const long m = v && *v ? std::strtol(v, nullptr, 10) : 0;
  return m > 0 ? static_cast<size_t>(m) << 20 : size_t{32} << 20;
}
// First, middle and last page of [p, p + bytes) resident (mincore): the
// range was touched before, so registering it maps no fresh pages.
bool pages_mapped(const void* p, size_t bytes) {
  const uintptr_t pg = 4096, lo = reinterpret_cast<uintptr_t>(p);
  for (uintptr_t a : {lo, lo + bytes / 2, lo + bytes - 1}) {
    unsigned char v = 0;
    if (mincore(reinterpret_cast<void*>(a & ~(pg - 1)), pg, &v) != 0 || !(v & 1)) return false;
  }
  return true;
}
constexpr size_t kStagedChunk = size_t{64} << 20;

// The library's own transient registrations, reference-counted: a second
// thread copying from or into a range another thread has registered for its
// copy shares that registration (page_locked() would report the range as
// page-locked and a plain async copy could outlive the first thread's
// hipHostUnregister); the last user unregisters.  A request that overlaps a
// registration without lying inside it takes the bounce path.
struct Registration {
  size_t bytes;
  int users;
};
std::mutex g_reg_mu;
std::map<uintptr_t, Registration> g_regs;   // base address -> registration
std::atomic<int> g_reg_count{0};            // g_regs.size(), readable without the lock

// Covers [p, p + bytes) with a library registration held by the caller (to be
// released with release_host(*base)): an existing one that contains the range,
// or -- for new ranges of >= kRegisterMin unless `reuse_only` -- a fresh one.
enum Acquire { kNotOurs, kAcquired, kOverlaps };
// kOverlaps: part of the range is in a registration of ours -- the copy must
// take the bounce path (HIP would take the partly registered range as
// page-locked).  kNotOurs: use the page-locked test / bounce path.
Acquire acquire_host(void* p, size_t bytes, bool reuse_only, uintptr_t* base,
                     size_t min_bytes = kRegisterMin) {
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + bytes;
  std::lock_guard<std::mutex> lock(g_reg_mu);
  auto it = g_regs.upper_bound(lo);
  if (it != g_regs.begin()) {
    auto prev = std::prev(it);
    if (prev->first + prev->second.bytes > lo) {          // overlaps the one below
      if (prev->first + prev->second.bytes >= hi) {        // contains the range
        ++prev->second.users;
        *base = prev->first;
        return kAcquired;
      }
      return kOverlaps;
    }
  }
  if (it != g_regs.end() && it->first < hi) return kOverlaps;  // overlaps the one above
  if (reuse_only || bytes < min_bytes) return kNotOurs;
  if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return kNotOurs;
  }
  g_regs[lo] = Registration{bytes, 1};
  g_reg_count.store(static_cast<int>(g_regs.size()));
  *base = lo;
  return kAcquired;
}

// True if [lo, hi) overlaps a registration of ours (g_reg_mu held).
bool overlaps_registration(uintptr_t lo, uintptr_t hi) {
  auto it = g_regs.upper_bound(lo);
  if (it != g_regs.begin()) {
    auto prev = std::prev(it);
    if (prev->first + prev->second.bytes > lo) return true;
  }
  return it != g_regs.end() && it->first < hi;
}

void release_host(uintptr_t base) {
  std::lock_guard<std::mutex> lock(g_reg_mu);
  auto it = g_regs.find(base);
  if (it == g_regs.end() || --it->second.users > 0) return;
  (void)hipHostUnregister(reinterpret_cast<void*>(base));
  g_regs.erase(it);
  g_reg_count.store(static_cast<int>(g_regs.size()));
}

// Copies chunk by chunk on `s`, calling before(ctx, end) ahead of each chunk's
// DMA (D2H: the destination chunk becomes valid while the previous chunk's
// DMA runs).  `h` lies in the registration acquired at `base`, released here.
int registered_copy(char* h, char* d, size_t bytes, bool to_host, void (*before)(void*, size_t),
                    void* ctx, hipStream_t s, uintptr_t base) {
  int rc = kOk;
  for (size_t off = 0; off < bytes && rc == kOk; off += kStagedChunk) {
    const size_t len = bytes - off < kStagedChunk ? bytes - off : kStagedChunk;
    if (before) before(ctx, off + len);
    const hipError_t e = to_host ? hipMemcpyAsync(h + off, d + off, len, hipMemcpyDeviceToHost, s)
                                 : hipMemcpyAsync(d + off, h + off, len, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) rc = hip_fail(e, "hipMemcpyAsync (registered host memory)");
  }
  const hipError_t e = hipStreamSynchronize(s);
  if (rc == kOk && e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
  release_host(base);
  return rc;
}

// Maps the pages of fresh host storage [p, p + bytes) by touching one byte per
// 4 KiB page on up to `threads` threads (a one-thread first touch of a fresh
// 8 GiB vector costs ~350 ms of page faults, tools/host_output_microbench.cc;
// registering unmapped pages would fault them in on one thread too).
void prefault(char* p, size_t bytes, int threads) {
  constexpr size_t kPage = 4096;
  const size_t pages = bytes / kPage + 1;
  size_t t = bytes >> 24;   // one thread per 16 MiB
  if (t > static_cast<size_t>(threads)) t = threads;
  auto touch = [p, bytes](size_t lo, size_t hi) {
    volatile char* v = p;
    for (size_t i = lo; i < hi; ++i)
      if (i * kPage < bytes) v[i * kPage] = 0;
  };
  if (t <= 1) {
    touch(0, pages);
    return;
  }
  std::vector<std::thread> pool;
  size_t done = 0;   // ranges [0, done) handed to threads
  try {
    for (; done < t; ++done) pool.emplace_back(touch, pages * done / t, pages * (done + 1) / t);
  } catch (...) {
    // No thread to spare: the rest on this one.
  }
  if (done < t) touch(pages * done / t, pages);
  for (auto& th : pool) th.join();
}

// A fresh destination of >= kRegisterMin is mapped and registered piece by
// piece behind the DMA (see piece_bytes below for the piece sizes).
// DPF_HIP_D2H_PIPELINE=0 (read per call) maps and registers the whole range
// before the first DMA instead (the r13 path): the A/B and test hook.
constexpr size_t kPipelineMax = size_t{16} << 30;   // above: a few large pieces
bool d2h_pipeline_on(size_t) {
  const char* v = std::getenv("DPF_HIP_D2H_PIPELINE");
  return !(v && v[0] == '0');
}
// DPF_HIP_D2H_REGISTER_PIECES=<n> (read per call): the pipelined copy acts as
// if the registration of its piece n (and every later one) were refused -- a
// test hook for the bounce fallback of the rest of the range.
long register_pieces_limit() {
  const char* v = std::getenv("DPF_HIP_D2H_REGISTER_PIECES");
  return v && *v ? std::strtol(v, nullptr, 10) : -1;
}

// A fresh pageable destination of >= kRegisterMin (no registration of ours
// overlaps it): a helper thread maps (prefault, 8 threads) and registers it in
// pieces (256 MiB, or 1/32 of the range) while this thread initialises (before) and DMAs the pieces
// already registered, so the ~45 ms of mapping and registering 8 GiB runs
// under the DMA instead of ahead of it.  Piece boundaries are 2 MiB-aligned
// (no page in two registrations) and every DMA chunk lies in one piece.  A
// piece whose registration is refused, and everything after it, goes through
// the bounce buffers.
constexpr size_t kPiece = size_t{256} << 20;
constexpr int kNoHelperThread = -1000;   // pipelined_d2h could not start its helper
// Up to kPipelineMax: ~32 pieces (256 MiB up to 8 GiB; 8 GiB copies 164-171
// ms pipelined vs 199-209 ms registered whole).  Above it, 8 GiB pieces: a
// 32 GiB copy (config 3's 2^31 uint128) in 33 or 129 pieces ran its DMA at
// ~13 GB/s in 1 of 4 calls (r14) and 3 of 6 (r15), in 5 pieces never in 6
// calls (3 pieces: never in 6), 682-758 ms per copy against 801-938 ms
// registered whole first (profiles/r15_ab.txt part 12).  A/B hooks (read per
// call): DPF_HIP_D2H_PIECE_MIB (a multiple of 64) and
// DPF_HIP_D2H_PREFAULT_THREADS (default 8).

size_t piece_bytes(size_t bytes) {
  const char* v = std::getenv("DPF_HIP_D2H_PIECE_MIB");
  const long m = v && *v ? std::strtol(v, nullptr, 10) : 0;
  if (m >= 64 && m % 64 == 0) return static_cast<size_t>(m) << 20;
  const size_t step = size_t{64} << 20;
  if (bytes > kPipelineMax) return size_t{8} << 30;
  const size_t want = (bytes / 32 + step - 1) / step * step;
  return want > kPiece ? want : kPiece;
}
int prefault_threads() {
  const char* v = std::getenv("DPF_HIP_D2H_PREFAULT_THREADS");
  const long t = v && *v ? std::strtol(v, nullptr, 10) : 0;
  return t >= 1 && t <= 64 ? static_cast<int>(t) : 8;
}

// With parts (nparts > 0) the DMAs run on `s` = a copy stream of their own:
// [0, ends[j]) of `d` is ready once events[j] (recorded on the producing
// stream) has completed, and each chunk's DMA waits on the device for the
// first part that covers it, so the copy of part j overlaps the work that
// produces the later parts.
int pipelined_d2h(char* h, const char* d, size_t bytes, void (*before)(void*, size_t), void* ctx,
                  hipStream_t s, int nparts = 0, void* const* events = nullptr,
                  const size_t* ends = nullptr) {
  const uintptr_t h0 = reinterpret_cast<uintptr_t>(h), h1 = h0 + bytes;
  const size_t piece = piece_bytes(bytes);
  const int pf_threads = prefault_threads();
  std::vector<uintptr_t> cut{h0};   // piece i = [cut[i], cut[i + 1])
  for (uintptr_t c = (h0 + piece) & ~((uintptr_t{2} << 20) - 1); c < h1; c += piece)
    if (c > cut.back()) cut.push_back(c);
  cut.push_back(h1);
  const size_t n = cut.size() - 1;
  std::vector<int> state(n, 0);   // 0 pending, 1 registered (in g_regs), -1 refused
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<bool> stop{false};
  int device = 0;
  (void)hipGetDevice(&device);
  const long limit = register_pieces_limit();
  // DPF_HIP_D2H_TRACE=1: per-call seconds spent mapping, registering and
  // waiting for the helper thread, on stderr (a diagnostic).
  const bool trace = std::getenv("DPF_HIP_D2H_TRACE") != nullptr;
  using clk = std::chrono::steady_clock;
  double t_fault = 0, t_reg = 0, t_wait = 0, t_before = 0;
  const auto t_start = clk::now();
  std::thread worker;
  auto helper = [&] {
    (void)hipSetDevice(device);
    for (size_t i = 0; i < n && !stop.load(); ++i) {
      char* p = reinterpret_cast<char*>(cut[i]);
      const size_t len = cut[i + 1] - cut[i];
      const auto a = clk::now();
      prefault(p, len, pf_threads);
      const auto b = clk::now();
      int st = -1;
      if (limit >= 0 && static_cast<long>(i) >= limit) {
        // test hook: refused
      } else {
        // Under g_reg_mu from the overlap check to the insert: another thread
        // may have registered part of this piece since acquire_host said
        // kNotOurs.  An overlapping piece is refused (the bounce path).
        std::lock_guard<std::mutex> lock(g_reg_mu);
        if (!overlaps_registration(cut[i], cut[i + 1])) {
          if (hipHostRegister(p, len, hipHostRegisterDefault) == hipSuccess) {
            g_regs[cut[i]] = Registration{len, 1};
            g_reg_count.store(static_cast<int>(g_regs.size()));
            st = 1;
          } else {
            (void)hipGetLastError();
          }
        }
      }
      t_fault += std::chrono::duration<double>(b - a).count();
      t_reg += std::chrono::duration<double>(clk::now() - b).count();
      {
        std::lock_guard<std::mutex> lock(mu);
        state[i] = st;
      }
      cv.notify_all();
      if (st < 0) break;
    }
  };
  try {
    worker = std::thread(helper);
  } catch (...) {
    return kNoHelperThread;   // nothing done yet: the caller copies another way
  }
  int rc = kOk;
  int waited = -1;   // parts whose event `s` already waits for: [0, waited]
  auto wait_parts = [&](size_t end) {
    int j = waited + 1;
    while (j < nparts - 1 && ends[j] < end) ++j;
    if (j >= nparts || j <= waited) return;
    const hipError_t e = hipStreamWaitEvent(s, (hipEvent_t)events[j], 0);
    if (e != hipSuccess) rc = hip_fail(e, "hipStreamWaitEvent");
    waited = j;
  };
  size_t i = 0;
  for (; i < n && rc == kOk; ++i) {
    int st;
    {
      const auto w = clk::now();
      std::unique_lock<std::mutex> lock(mu);
      cv.wait(lock, [&] { return state[i] != 0; });
      st = state[i];
      t_wait += std::chrono::duration<double>(clk::now() - w).count();
    }
    if (st < 0) break;
    for (uintptr_t off = cut[i]; off < cut[i + 1] && rc == kOk; off += kStagedChunk) {
      const size_t len = cut[i + 1] - off < kStagedChunk ? cut[i + 1] - off : kStagedChunk;
      wait_parts(off + len - h0);
      if (rc != kOk) break;
      if (before) {
        // The helper thread must be joined on every path out of here.
        try {
          const auto bt = clk::now();
          before(ctx, off + len - h0);
          t_before += std::chrono::duration<double>(clk::now() - bt).count();
        } catch (...) {
          rc = fail(kInternal, "dpf_hip_memcpy_d2h_staged: before_chunk threw");
          break;
        }
      }
      const hipError_t e = hipMemcpyAsync(reinterpret_cast<char*>(off), d + (off - h0), len,
                                          hipMemcpyDeviceToHost, s);
      if (e != hipSuccess) rc = hip_fail(e, "hipMemcpyAsync (registered host memory)");
    }
  }
  stop.store(true);
  worker.join();
  if (rc == kOk && i < n) {
    // Registration refused from piece i on: the rest through the bounce buffers.
    const size_t off = cut[i] - h0;
    prefault(h + off, bytes - off, 8);
    try {
      if (before) before(ctx, bytes);
    } catch (...) {
      rc = fail(kInternal, "dpf_hip_memcpy_d2h_staged: before_chunk threw");
    }
    if (rc == kOk) wait_parts(bytes);
    if (rc == kOk) rc = bounce_d2h(h + off, d + off, bytes - off, s);
  }
  const auto t_issue = clk::now();
  const hipError_t e = hipStreamSynchronize(s);
  if (rc == kOk && e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
  const auto t_sync = clk::now();
  for (size_t j = 0; j < n; ++j)
    if (state[j] > 0) release_host(cut[j]);
  if (trace)
    fprintf(stderr, "[pipelined_d2h] %zu MiB in %zu pieces: total %.1f ms, map %.1f ms, register "
            "%.1f ms (helper), wait %.1f ms, before_chunk %.1f ms, issue %.1f ms, final sync "
            "%.1f ms, unregister %.1f ms\n", bytes >> 20, n,
            1e3 * std::chrono::duration<double>(clk::now() - t_start).count(), 1e3 * t_fault,
            1e3 * t_reg, 1e3 * t_wait, 1e3 * t_before,
            1e3 * std::chrono::duration<double>(t_issue - t_start).count(),
            1e3 * std::chrono::duration<double>(t_sync - t_issue).count(),
            1e3 * std::chrono::duration<double>(clk::now() - t_sync).count());
  return rc;
}

int bounce_h2d(void* dst, const void* src, size_t bytes, void* stream) {
  std::lock_guard<std::mutex> lock(g_bounce_mu);
  if (int rc = bounce_buffers()) return rc;
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (bytes + kBounceChunk - 1) / kBounceChunk;
  for (size_t i = 0; i < n; ++i) {
    const size_t l = i + 1 < n ? kBounceChunk : bytes - i * kBounceChunk;
    if (i >= 2) HIP_TRY(hipStreamSynchronize(s));   // chunk i - 2 has left g_bounce[i & 1]
    host_copy(g_bounce[i & 1], (const char*)src + i * kBounceChunk, l);
    HIP_TRY(hipMemcpyAsync((char*)dst + i * kBounceChunk, g_bounce[i & 1], l,
                           hipMemcpyHostToDevice, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return kOk;
}
}  // namespace

extern "C" {

int dpf_hip_alloc(void** ptr, size_t bytes) {
  if (!ptr) return fail(kInvalidArgument, "ptr is NULL");
  *ptr = nullptr;
  if (bytes == 0) bytes = 1;
  const hipError_t e = hipMalloc(ptr, bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // an allocation failure must not fail the next launch check
    *ptr = nullptr;
  }
  HIP_TRY(e);
  return kOk;
}
int dpf_hip_mem_info(size_t* free_bytes, size_t* total_bytes) {
  if (!free_bytes || !total_bytes) return fail(kInvalidArgument, "NULL pointer");
  HIP_TRY(hipMemGetInfo(free_bytes, total_bytes));
  return kOk;
}
int dpf_hip_free(void* ptr) {
  if (ptr) HIP_TRY(hipFree(ptr));
  return kOk;
}
int dpf_hip_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return kOk;
  uintptr_t base = 0;
  if (bytes >= kBounceMin || g_reg_count.load() > 0) {
    // Inside a registration of ours (another thread's copy), or large and new.
    const Acquire a = acquire_host(const_cast<void*>(src), bytes,
                                   bytes < kBounceMin || page_locked(src), &base,
                                   register_min_mapped());
    if (a == kAcquired)
      return registered_copy((char*)const_cast<void*>(src), (char*)dst, bytes, false, nullptr,
                             nullptr, (hipStream_t)stream, base);
    if (a == kOverlaps || (bytes >= kBounceMin && !page_locked(src)))
      return bounce_h2d(dst, src, bytes, stream);
  }
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return kOk;
}
int dpf_hip_host_alloc(void** ptr, size_t bytes) {
  if (!ptr) return fail(kInvalidArgument, "ptr is NULL");
  *ptr = nullptr;
  if (bytes == 0) bytes = 1;
  HIP_TRY(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
  return kOk;
}
int dpf_hip_host_free(void* ptr) {
  if (ptr) HIP_TRY(hipHostFree(ptr));
  return kOk;
}
int dpf_hip_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return kOk;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return kOk;
}
int dpf_hip_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return kOk;
  uintptr_t base = 0;
  if (bytes >= kBounceMin || g_reg_count.load() > 0) {
    const bool reuse_only = bytes < kBounceMin || page_locked(dst);
    const Acquire a =
        acquire_host(dst, bytes, reuse_only, &base,
                     !reuse_only && pages_mapped(dst, bytes) ? register_min_mapped() : kRegisterMin);
    if (a == kAcquired)
      return registered_copy((char*)dst, (char*)const_cast<void*>(src), bytes, true, nullptr,
                             nullptr, (hipStream_t)stream, base);
    if (a == kOverlaps || (bytes >= kBounceMin && !page_locked(dst)))
      return bounce_d2h(dst, src, bytes, stream);
  }
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return kOk;
}
int dpf_hip_memcpy_d2h_strided(void* dst, const void* src, size_t elem_bytes,
                               size_t src_stride_bytes, int64_t count, void* stream) {
  if (count < 0 || src_stride_bytes < elem_bytes) return fail(kInvalidArgument, "bad sizes");
  if (count == 0 || elem_bytes == 0) return kOk;
  if (!dst || !src) return fail(kInvalidArgument, "NULL pointer");
  HIP_TRY(hipMemcpy2DAsync(dst, elem_bytes, src, src_stride_bytes, elem_bytes, (size_t)count,
                           hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return kOk;
}
int dpf_hip_memcpy_d2h_staged(void* dst, const void* src, size_t bytes,
                              void (*before_chunk)(void* ctx, size_t bytes_ready), void* ctx,
                              void* stream) {
  return dpf_hip_memcpy_d2h_staged_after(dst, src, bytes, before_chunk, ctx, 0, nullptr, nullptr,
                                         stream);
}
int dpf_hip_memcpy_d2h_staged_after(void* dst, const void* src, size_t bytes,
                                    void (*before_chunk)(void* ctx, size_t bytes_ready), void* ctx,
                                    int num_parts, void* const* part_events,
                                    const size_t* part_end_bytes, void* stream) {
  if (num_parts < 0 || (num_parts > 0 && (!part_events || !part_end_bytes)))
    return fail(kInvalidArgument, "dpf_hip_memcpy_d2h_staged_after: bad parts");
  for (int j = 0; j < num_parts; ++j)
    if (!part_events[j] || (j > 0 && part_end_bytes[j] < part_end_bytes[j - 1]) ||
        (j == num_parts - 1 && part_end_bytes[j] < bytes))
      return fail(kInvalidArgument, "dpf_hip_memcpy_d2h_staged_after: bad parts");
  // Every path but the pipelined one copies on `stream`, after all its parts.
  if (!before_chunk) return dpf_hip_memcpy_d2h(dst, src, bytes, stream);
  uintptr_t base = 0;
  if (bytes >= kRegisterMin) {
    const bool locked = page_locked(dst);
    // An existing registration of ours that contains the range is shared;
    // a fresh pageable range is mapped and registered piece by piece.
    const Acquire a = acquire_host(dst, bytes, true, &base);
    if (a == kAcquired)
      return registered_copy((char*)dst, (char*)const_cast<void*>(src), bytes, true, before_chunk,
                             ctx, (hipStream_t)stream, base);
    if (a == kNotOurs && !locked) {
      if (d2h_pipeline_on(bytes)) {
        int rc;
        if (num_parts == 0) {
          rc = pipelined_d2h((char*)dst, (const char*)src, bytes, before_chunk, ctx,
                             (hipStream_t)stream);
        } else {
          hipStream_t copy;
          HIP_TRY(hipStreamCreateWithFlags(&copy, hipStreamNonBlocking));
          rc = pipelined_d2h((char*)dst, (const char*)src, bytes, before_chunk, ctx, copy,
                             num_parts, part_events, part_end_bytes);
          (void)hipStreamDestroy(copy);
        }
        if (rc != kNoHelperThread) return rc;
        // No helper thread: map and register the whole range first.
      }
      using clk = std::chrono::steady_clock;
      const auto t0 = clk::now();
      prefault((char*)dst, bytes, 16);
      const auto t1 = clk::now();
      if (acquire_host(dst, bytes, false, &base) == kAcquired) {
        const auto t2 = clk::now();
        const int rc = registered_copy((char*)dst, (char*)const_cast<void*>(src), bytes, true,
                                       before_chunk, ctx, (hipStream_t)stream, base);
        if (std::getenv("DPF_HIP_D2H_TRACE"))
          fprintf(stderr, "[whole_d2h] %zu MiB: total %.1f ms, map %.1f ms, register %.1f ms, "
                  "copy+unregister %.1f ms\n", bytes >> 20,
                  1e3 * std::chrono::duration<double>(clk::now() - t0).count(),
                  1e3 * std::chrono::duration<double>(t1 - t0).count(),
                  1e3 * std::chrono::duration<double>(t2 - t1).count(),
                  1e3 * std::chrono::duration<double>(clk::now() - t2).count());
        return rc;
      }
    }
  }
  before_chunk(ctx, bytes);
  return dpf_hip_memcpy_d2h(dst, src, bytes, stream);
}
int dpf_hip_memcpy_d2h_chunked(const void* src, size_t bytes, size_t align,
                               void (*consume)(void* ctx, const void* chunk, size_t offset,
                                               size_t len),
                               void* ctx, void* stream) {
  if (!bytes) return kOk;
  if (!src || !consume || align == 0 || align > kBounceChunk)
    return fail(kInvalidArgument, "dpf_hip_memcpy_d2h_chunked: bad arguments");
  std::lock_guard<std::mutex> lock(g_bounce_mu);
  if (int rc = bounce_buffers()) return rc;
  hipStream_t s = (hipStream_t)stream;
  const size_t chunk = kBounceChunk / align * align;
  const size_t n = (bytes + chunk - 1) / chunk;
  auto len = [&](size_t i) { return i + 1 < n ? chunk : bytes - i * chunk; };
  HIP_TRY(hipMemcpyAsync(g_bounce[0], src, len(0), hipMemcpyDeviceToHost, s));
  for (size_t i = 0; i < n; ++i) {
    HIP_TRY(hipStreamSynchronize(s));   // chunk i is in g_bounce[i & 1]
    if (i + 1 < n)
      HIP_TRY(hipMemcpyAsync(g_bounce[(i + 1) & 1], (const char*)src + (i + 1) * chunk, len(i + 1),
                             hipMemcpyDeviceToHost, s));
    // The next chunk's DMA into the other bounce buffer must have finished
    // before the buffers (and g_bounce_mu) are given up on any path out.
    try {
      consume(ctx, g_bounce[i & 1], i * chunk, len(i));
    } catch (...) {
      (void)hipStreamSynchronize(s);
      return fail(kInternal, "dpf_hip_memcpy_d2h_chunked: consume threw");
    }
  }
  return kOk;
}
int dpf_hip_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return kOk;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return kOk;
}
int dpf_hip_memset(void* dst, int value, size_t bytes, void* stream) {
  if (!bytes) return kOk;
  HIP_TRY(hipMemsetAsync(dst, value, bytes, (hipStream_t)stream));
  return kOk;
}
int dpf_hip_stream_sync(void* stream) {
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return kOk;
}
int dpf_hip_event_sync(void* event) {
  HIP_TRY(hipEventSynchronize((hipEvent_t)event));
  return kOk;
}
int dpf_hip_stream_wait_event(void* stream, void* event) {
  HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
  return kOk;
}
int dpf_hip_packed_element_size(const dpf_value_desc* desc) {
  if (!desc) return -1;
  return packed_size(desc);
}

int dpf_hip_hash(int64_t n, const dpf_block* in, const dpf_aes_key* key, dpf_block* out,
                 void* stream) {
  if (n < 0) return fail(kInvalidArgument, "n < 0");
  if (n == 0) return kOk;
  if (!in || !out || !key) return fail(kInvalidArgument, "NULL pointer");
  const int blk = block_for(n);
  const int grid = grid_for(n, blk);
  // DPF_HASH_DYNAMIC=0: a fixed share of blocks per thread (A/B hook).
  hipLaunchKernelGGL(hash_kernel, dim3(grid), dim3(blk), 0, (hipStream_t)stream, n, in, out,
                     expand_key(key), dynamic_chunks_per_wg(n, grid, blk, "DPF_HASH_DYNAMIC"));
  HIP_TRY(hipGetLastError());
  return kOk;
}

int dpf_hip_eval_paths(int64_t num_seeds, int num_levels, const dpf_block* seeds_in,
                       const uint8_t* control_in, const dpf_block* paths,
                       const dpf_block* cw_seed, const uint8_t* cw_left, const uint8_t* cw_right,
                       const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                       dpf_block* seeds_out, uint8_t* control_out, void* stream) {
  if (num_seeds < 0 || num_levels < 0 || num_levels > kMaxCwLevels)
    return fail(kInvalidArgument, "num_seeds or num_levels out of range");
  if (num_seeds == 0) return kOk;
  hipStream_t s = (hipStream_t)stream;
  if (num_levels == 0) {
    if (seeds_out != seeds_in)
      HIP_TRY(hipMemcpyAsync(seeds_out, seeds_in, num_seeds * sizeof(dpf_block),
                             hipMemcpyDeviceToDevice, s));
    if (control_out != control_in)
      HIP_TRY(hipMemcpyAsync(control_out, control_in, num_seeds, hipMemcpyDeviceToDevice, s));
    return kOk;
  }
  if (!seeds_in || !control_in || !paths || !cw_seed || !cw_left || !cw_right || !key_left ||
      !key_right || !seeds_out || !control_out)
    return fail(kInvalidArgument, "NULL pointer");
  PathParams p;
  p.n = num_seeds;
  p.num_levels = num_levels;
  p.seeds_in = seeds_in;
  p.ctrl_in = control_in;
  p.paths = paths;
  p.cw_seed = cw_seed;
  p.cw_left = cw_left;
  p.cw_right = cw_right;
  p.seeds_out = seeds_out;
  p.ctrl_out = control_out;
  p.rkl = expand_key(key_left);
  p.rkd = xor_keys(p.rkl, expand_key(key_right));
  const int blk = block_for(num_seeds);
  const int grid = grid_for(num_seeds, blk);
  p.dyn_per_wg = dynamic_chunks_per_wg(num_seeds, grid, blk, "DPF_PATHS_DYNAMIC");
  hipLaunchKernelGGL(eval_paths_kernel, dim3(grid), dim3(blk), 0, s, p);
  HIP_TRY(hipGetLastError());
  return kOk;
}

int dpf_hip_expand(int64_t num_starts, const dpf_block* seeds_in, const uint8_t* control_in,
                   int num_levels, const dpf_block* cw_seed, const uint8_t* cw_left,
                   const uint8_t* cw_right, const dpf_aes_key* key_left,
                   const dpf_aes_key* key_right, const dpf_aes_key* key_value,
                   const dpf_value_desc* desc, int elements_per_leaf,
                   const dpf_block* value_correction, int party, void* out, void* stream) {
  int st = validate_desc(desc);
  if (st) return st;
  if (num_starts < 0 || num_levels < 0 || num_levels > 62)
    return fail(kInvalidArgument, "num_starts or num_levels out of range");
  if (elements_per_leaf < 1 || elements_per_leaf > desc->elements_per_block)
    return fail(kInvalidArgument, "elements_per_leaf must be in [1, elements_per_block]");
  if (num_starts == 0) return kOk;
  if (!seeds_in || !control_in || !key_left || !key_right || !key_value || !value_correction ||
      !out || (num_levels > 0 && (!cw_seed || !cw_left || !cw_right)))
    return fail(kInvalidArgument, "NULL pointer");
  if (num_starts > (INT64_MAX >> num_levels))
    return fail(kInvalidArgument, "expansion too large");
  // Choose the depth-first subtree depth S (items = num_starts * 2^(L - S)
  // subtrees, each walked k0 = L - S levels from its start seed) by the
  // per-thread critical path: rounds of items over the launch's threads times
  // the AES of one item, the ILP1 walk counted twice.  Small trees get shallow
  // subtrees and more items, so a launch far below one workgroup per CU is not
  // serialised on a few lanes' DFS; start counts that are not powers of two
  // (5 starts x 2^27: 1.25 subtrees of depth 11 per thread = 2 rounds) get
  // subtrees shallow enough to divide evenly (depth 9: 5 rounds of 1, +53%).
  int S = num_levels < kSMax ? num_levels : kSMax;
  {
    double best = -1;
    int best_s = S;
    for (int cand = S; cand >= (num_levels > 0 ? 1 : 0); --cand) {
      const int64_t items = num_starts << (num_levels - cand);
      const int blk = block_for(items);
      const int64_t threads = (int64_t)grid_for(items, blk) * blk;
      const int64_t rounds = (items + threads - 1) / threads;
      const double cost = (double)rounds * (2.0 * (num_levels - cand) + 3.0 * (double)(1ll << cand));
      if (best < 0 || cost < best * 0.999) {
        best = cost;
        best_s = cand;
      }
    }
    S = best_s;
  }
#if defined(DPF_FORCE_S)
  if (num_levels >= DPF_FORCE_S) S = DPF_FORCE_S;  // variant builds (tools/variant_bench.py)
#endif
  ExpandParams p;
  p.dyn_chunks = 0;
  p.num_levels = num_levels;
  p.S = S;
  p.k0 = num_levels - S;
  p.num_items = num_starts << p.k0;
  p.seeds_in = seeds_in;
  p.ctrl_in = control_in;
  p.cw_seed = cw_seed;
  p.cw_left = cw_left;
  p.cw_right = cw_right;
  p.out = (char*)out;
  p.rkl = expand_key(key_left);
  p.rkr = expand_key(key_right);
  p.rkv = expand_key(key_value);
  p.rkd = xor_keys(p.rkl, p.rkr);
  p.clock = dpf_rt::g_clock_acc.load(std::memory_order_relaxed);
  hipStream_t s = (hipStream_t)stream;
  if (fast_int(desc)) {
    const int bits = desc->bits[0], E = desc->elements_per_block;
    const int store_bytes = elements_per_leaf * bits / 8;
    switch (bits) {
      case 8: return launch_expand_fast<8>(p, desc, value_correction, E, party, store_bytes, s);
      case 16: return launch_expand_fast<16>(p, desc, value_correction, E, party, store_bytes, s);
      case 32: return launch_expand_fast<32>(p, desc, value_correction, E, party, store_bytes, s);
      case 64: return launch_expand_fast<64>(p, desc, value_correction, E, party, store_bytes, s);
      default: return launch_expand_fast<128>(p, desc, value_correction, E, party, store_bytes, s);
    }
  }
  const int esz = packed_size(desc);
  if (desc->direct && desc->blocks_needed == 1) {
    // Direct tuples of plain integers / XorWrappers: the hashed block is E
    // packed elements (value_type_helpers.h:199-211).
    const int nl = desc->num_leaves, bits = desc->bits[0], kind = desc->kind[0];
    bool uniform = true;
    for (int k = 1; k < nl; ++k) uniform = uniform && desc->bits[k] == bits && desc->kind[k] == kind;
    const int lanes = desc->elements_per_block * nl;
    if (uniform && lanes * bits <= 128) {
      // Every lane the same width and kind: the integer fast path with E * nl lanes.
      const int store_bytes = elements_per_leaf * esz;
      switch (bits) {
        case 8: return launch_expand_fast<8>(p, desc, value_correction, lanes, party, store_bytes, s);
        case 16: return launch_expand_fast<16>(p, desc, value_correction, lanes, party, store_bytes, s);
        case 32: return launch_expand_fast<32>(p, desc, value_correction, lanes, party, store_bytes, s);
        case 64: return launch_expand_fast<64>(p, desc, value_correction, lanes, party, store_bytes, s);
        default: return launch_expand_fast<128>(p, desc, value_correction, lanes, party, store_bytes, s);
      }
    }
    if (lanes <= 16 && desc->elements_per_block * esz <= 16) {
      SwarLeaf w;
      memset(&w, 0, sizeof(w));
      w.vcw_elems = value_correction;
      w.lanes = lanes;
      w.party = party;
      w.store_bytes = elements_per_leaf * esz;
      int off = 0;
      for (int i = 0; i < lanes; ++i) {
        const int b = desc->bits[i % nl];
        w.lane_off[i] = (uint8_t)off;
        w.lane_bits[i] = (uint8_t)b;
        w.top |= (u128)1 << (off + b - 1);
        if (desc->kind[i % nl] == DPF_LEAF_XOR)
          w.xmask |= (b >= 128 ? ~(u128)0 : (((u128)1 << b) - 1)) << off;
        off += b;
      }
      const char* off_env = getenv("DPF_EXPAND_NO_OCTET");
      if (try_small(p, w, s)) {
        HIP_TRY(hipGetLastError());
        return kOk;
      }
      if (p.S >= 3 && !(off_env && off_env[0] == '1')) {
        note_expand<SwarLeaf>(p, true);
        TopScratch top;
        int grid = 0, blk = 0;
        if (int st = octet_shape(p, s, top, &grid, &blk)) return st;
        hipLaunchKernelGGL((expand_octet_kernel<SwarLeaf>), dim3(grid), dim3(blk), 0, s, p, w);
        HIP_TRY(hipGetLastError());
        return kOk;
      }
      return launch_expand(p, w, s);
    }
  }
  int b = 0;
  if (elements_per_leaf == 1 && mod32_eligible(desc, &b)) {
    // Tuples of IntModN<uint32_t, N>: Moller-Granlund sampling.
    auto fill = [&](auto& m) {
      memset(&m, 0, sizeof(m));
      m.vcw_elems = value_correction;
      m.nl = desc->num_leaves;
      m.b = b;
      m.party = party;
      for (int k = 0; k < desc->num_leaves; ++k) m.div[k] = make_div32((uint32_t)desc->mod_low[k]);
    };
    if (desc->num_leaves <= 2) {
      Mod32Leaf<2> m;
      fill(m);
      const char* off = getenv("DPF_EXPAND_NO_OCTET");
      if (try_small(p, m, s)) {
        HIP_TRY(hipGetLastError());
        return kOk;
      }
      if (p.S >= 3 && !(off && off[0] == '1')) {
        // Octet form (the half's four leaves hashed as two ILP4 groups).
        note_expand<Mod32Leaf<2>>(p, true);
        TopScratch top;
        int grid = 0, blk = 0;
        if (int st = octet_shape(p, s, top, &grid, &blk)) return st;
        hipLaunchKernelGGL((expand_octet_kernel<Mod32Leaf<2>>), dim3(grid), dim3(blk), 0, s, p, m);
        HIP_TRY(hipGetLastError());
        return kOk;
      }
      return launch_expand(p, m, s);
    }
    if (desc->num_leaves <= 4) {   // no spills (Mod32Leaf<5> in expand_kernel: 36 B)
      Mod32Leaf<4> m;
      fill(m);
      return launch_expand(p, m, s);
    }
    Mod32Leaf<kMod32MaxLeaves> m;
    fill(m);
    return launch_expand(p, m, s);
  }
  GenericLeaf g;
  g.d = *desc;
  g.vcw = value_correction;
  g.party = party;
  g.elements_per_leaf = elements_per_leaf;
  g.esz = esz;
  return launch_expand(p, g, s);
}

int dpf_hip_eval_points(int64_t num_points, int64_t points_per_key, int num_levels,
                        const dpf_block* key_seed, const uint8_t* party,
                        const dpf_block* seeds_in, const uint8_t* control_in,
                        const dpf_block* tree_index, const int32_t* block_index,
                        const dpf_block* cw_seed, const uint8_t* cw_left, const uint8_t* cw_right,
                        const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                        const dpf_aes_key* key_value, const dpf_value_desc* desc,
                        const dpf_block* value_correction, void* out, void* stream) {
  if (num_points < 0 || points_per_key < 1 || num_points % points_per_key != 0)
    return fail(kInvalidArgument, "num_points must be a non-negative multiple of points_per_key");
  PointParams p;
  int st = make_point_params(num_points / points_per_key, points_per_key, num_levels, key_seed,
                             party, seeds_in, control_in, tree_index, block_index, cw_seed,
                             cw_left, cw_right, key_left, key_right, key_value, desc,
                             value_correction, &p);
  if (st) return st;
  if (num_points == 0) return kOk;
  if (!out) return fail(kInvalidArgument, "NULL pointer");
  p.num_items = p.num_keys * p.half;
  p.out = (char*)out;
  return launch_points<false>(p, desc, value_correction, (hipStream_t)stream);
}

int dpf_hip_eval_points_batch(int64_t num_keys, int64_t points_per_key, int shared_points,
                              int num_levels, int cw_stride, int block_index_bits,
                              const dpf_block* key_seed,
                              const uint8_t* party, const dpf_block* points,
                              const dpf_block* cw_seed, const uint8_t* cw_left,
                              const uint8_t* cw_right, const dpf_aes_key* key_left,
                              const dpf_aes_key* key_right, const dpf_aes_key* key_value,
                              const dpf_value_desc* desc, const dpf_block* value_correction,
                              void* out, void* stream) {
  if (block_index_bits < 0 || block_index_bits > 7 || num_levels + block_index_bits > 128)
    return fail(kInvalidArgument, "block_index_bits out of range");
  PointParams p;
  int st = make_point_params(num_keys, points_per_key, num_levels, key_seed, party, nullptr,
                             nullptr, points, nullptr, cw_seed, cw_left, cw_right, key_left,
                             key_right, key_value, desc, value_correction, &p);
  if (st) return st;
  if (!key_seed) return fail(kInvalidArgument, "NULL pointer");
  if (cw_stride < num_levels) return fail(kInvalidArgument, "cw_stride < num_levels");
  if (num_keys == 0) return kOk;
  if (!out) return fail(kInvalidArgument, "NULL pointer");
  p.cw_stride = cw_stride;
  p.bib = block_index_bits;
  p.shared_points = shared_points ? 1 : 0;
  p.num_items = p.num_keys * p.half;
  p.out = (char*)out;
  return launch_points<false>(p, desc, value_correction, (hipStream_t)stream);
}

int dpf_hip_eval_points_sum(int64_t num_keys, int64_t num_points, int num_levels, int cw_stride,
                            int block_index_bits, const dpf_block* key_seed, const uint8_t* party,
                            const dpf_block* points, const dpf_block* cw_seed,
                            const uint8_t* cw_left, const uint8_t* cw_right,
                            const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                            const dpf_aes_key* key_value, const dpf_value_desc* desc,
                            const dpf_block* value_correction, uint64_t* workspace, void* out,
                            void* stream) {
  if (num_points == 0 && num_keys >= 0) return kOk;
  if (block_index_bits < 0 || block_index_bits > 7 || num_levels + block_index_bits > 128)
    return fail(kInvalidArgument, "block_index_bits out of range");
  PointParams p;
  int st = make_point_params(num_keys, num_points, num_levels, key_seed, party, nullptr, nullptr,
                             points, nullptr, cw_seed, cw_left, cw_right, key_left, key_right,
                             key_value, desc, value_correction, &p);
  if (st) return st;
  if (!key_seed) return fail(kInvalidArgument, "NULL pointer");
  if (cw_stride < num_levels) return fail(kInvalidArgument, "cw_stride < num_levels");
  p.cw_stride = cw_stride;
  p.bib = block_index_bits;
  if (!out || !workspace) return fail(kInvalidArgument, "NULL pointer");
  hipStream_t s = (hipStream_t)stream;
  const size_t wide_bytes = (size_t)num_points * desc->num_leaves * 3 * sizeof(uint64_t);
  HIP_TRY(hipMemsetAsync(workspace, 0, wide_bytes, s));
  if (num_keys > 0) {
    // Enough (chunk, pair) items to fill every CU's 1024 threads a few times
    // (16 times when the waves take them dynamically: enough chunks per wave
    // for take_chunk; each item then sums fewer keys before its atomics).
    const char* dyn = std::getenv("DPF_POINTS_DYNAMIC");
    const int64_t want = (int64_t)num_cus() * kBlock * (dyn && dyn[0] == '0' ? 4 : 16);
    int64_t chunks = (want + p.half - 1) / p.half;
    if (chunks > num_keys) chunks = num_keys;
    p.chunk_keys = (num_keys + chunks - 1) / chunks;
    chunks = (num_keys + p.chunk_keys - 1) / p.chunk_keys;
    p.shared_points = 1;
    p.num_items = chunks * p.half;
    p.wide = reinterpret_cast<unsigned long long*>(workspace);
    st = launch_points<true>(p, desc, value_correction, s);
    if (st) return st;
  }
  int64_t g = (num_points + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(finalize_sums_kernel, dim3((unsigned)g), dim3(256), 0, s, num_points, *desc,
                     reinterpret_cast<const unsigned long long*>(workspace), (char*)out, 3);
  HIP_TRY(hipGetLastError());
  return kOk;
}

int dpf_hip_count_out_of_range(int64_t n, const dpf_block* points, int log_domain_size,
                               int64_t* count, void* stream) {
  if (!count || n < 0 || log_domain_size < 0 || log_domain_size > 128)
    return fail(kInvalidArgument, "bad arguments");
  *count = 0;
  if (n == 0 || log_domain_size == 128) return kOk;
  if (!points) return fail(kInvalidArgument, "NULL pointer");
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* d = nullptr;
  HIP_TRY(hipMallocAsync((void**)&d, sizeof(*d), s));
  HIP_TRY(hipMemsetAsync(d, 0, sizeof(*d), s));
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(count_out_of_range_kernel, dim3((unsigned)g), dim3(256), 0, s, n, points,
                     log_domain_size, d);
  HIP_TRY(hipGetLastError());
  unsigned long long h = 0;
  HIP_TRY(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(d, s));
  HIP_TRY(hipStreamSynchronize(s));
  *count = (int64_t)h;
  return kOk;
}

int dpf_hip_gather(int64_t num_rows, int64_t count, int elem_size, const int64_t* src_offset,
                   const void* in, void* out, void* stream) {
  if (num_rows < 0 || count < 0 || elem_size < 1) return fail(kInvalidArgument, "bad sizes");
  int64_t total = num_rows * count * elem_size;
  if (total == 0) return kOk;
  int64_t g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                     num_rows, count, elem_size, src_offset, (const char*)in, (char*)out);
  HIP_TRY(hipGetLastError());
  return kOk;
}

int dpf_hip_sum_shares_u64(int64_t num_keys, int64_t row_len, int bits, int xor_mode,
                           const void* shares, uint64_t* sums, void* stream) {
  if (num_keys < 0 || row_len < 0 || !(bits == 8 || bits == 16 || bits == 32 || bits == 64))
    return fail(kInvalidArgument, "bad arguments");
  if (row_len == 0) return kOk;
  int64_t g = (row_len + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(sum_shares_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                     num_keys, row_len, bits, xor_mode, (const char*)shares, sums);
  HIP_TRY(hipGetLastError());
  return kOk;
}

int dpf_hip_event_create(void** ev) {
  HIP_TRY(hipEventCreate((hipEvent_t*)ev));
  return kOk;
}
int dpf_hip_event_destroy(void* ev) {
  HIP_TRY(hipEventDestroy((hipEvent_t)ev));
  return kOk;
}
int dpf_hip_event_record(void* ev, void* stream) {
  HIP_TRY(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
  return kOk;
}
int dpf_hip_event_elapsed_ms(void* start, void* stop, float* ms) {
  HIP_TRY(hipEventSynchronize((hipEvent_t)stop));
  HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return kOk;
}

}  // extern "C"
