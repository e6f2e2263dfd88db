// dpf_expand_ws.hip -- full-domain expansion (dpf_hip_expand; SURVEY.md section 8
// rows a3-a6, a12-a13) with WAVE-SPECIALISED workgroups: the CU's two AES
// engines run in different waves at the same time instead of in phases of one
// wave (dpf_expand_hybrid.hip, measured slower).
//
//   * 12 "tree" waves (3 per SIMD) expand the tree on the LDS T-table AES of
//     aes_core.h (ExpandSeeds, distributed_point_function.cc:271-349): per
//     lane the depth-first walk of expand_octet_kernel down to octets, and per
//     octet the 2 + 4 + 8 child hashes down to its eight leaf seeds.
//   * 4 "value" waves (1 per SIMD) hash leaf seeds with the fixed value key
//     (HashExpandedSeeds, cc:500-524), 8 blocks per lane as one bitsliced
//     AES-128 on the VALU (bs_aes.h: the 82-gate v_bitop3 S-box, every
//     round-key mask an immediate), correct them (h:785-808) and store each
//     lane's eight blocks as one 128-byte line.
//
// Opt-in (DPF_EXPAND_WS=1): bit-exact, but measured 2-4% SLOWER than the octet
// kernel at config 2 (18.2-18.5 vs 17.5-18.0 ms, same box):
// with 3 tree waves per SIMD the T-table chains are latency-bound (the tree
// waves alone reach 74 G AES/s, 16 octet-kernel waves 90), and the bitsliced
// waves (715 VALU lane-ops per block against the T-table's 269) slow them by a
// fifth while adding 29 G AES/s of their own.
//
// Tree waves hand each half-octet's four leaf seeds per lane (4 KiB per wave)
// to the value waves through six LDS slots beside the 128 KiB of tables; a
// tree wave that finds no free slot hashes that half itself on the T-table
// (the octet kernel's path), so the split between the engines balances itself.  Measured
// (tools/ws_microbench.hip, same box): 12 T-table waves alone 85 G AES/s, with
// 4 bitsliced waves beside them 78 + 36 = 114 G AES/s.
//
// Work: 768 tree lanes per CU do not divide the power-of-two subtree counts,
// so work is handed out in rounds of one subtree per tree lane; the subtrees
// left over after a round (1/4 of the lanes' worth) are split four ways for the
// next round (1 + 1/4 + 1/16 + ... of a round: within 0.3% of an even split).
// Every round's subtrees share one depth, so each wave's lanes stay in lockstep.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../../include/dpf_hip.h"
#include "bs_aes.h"
#include "dpf_device.h"
#include "dpf_runtime.h"

using namespace dpf_rt;

namespace {

// Memory image of the reference's value PRG key kPrgKeyValue
// (distributed_point_function.cc:37-42), low 64 bits first.
constexpr uint8_t kWsValueKey[16] = {0x98, 0x1c, 0x1d, 0xb2, 0x01, 0x11, 0xa3, 0x46,
                                     0xe3, 0x23, 0x54, 0x8c, 0x58, 0xd1, 0xa5, 0x05};
struct WsValueMasks {
  static constexpr bsa::BsKeyMasks m = bsa::make_key_masks_c(kWsValueKey);
};

#ifndef DPF_WS_TREE_WAVES
#define DPF_WS_TREE_WAVES 12
#endif
constexpr int kWsTree = DPF_WS_TREE_WAVES;  // tree waves per workgroup
constexpr int kWsValue = 16 - kWsTree;      // value waves per workgroup
constexpr int kWsTreeLanes = kWsTree * 64;  // 768
constexpr int kWsSlots = 6;

// One hand-off: half an octet (four leaf seeds) per lane, [leaf][lane] so that
// every ds_write_b128 / ds_read_b128 of a wave is one contiguous KiB.  A value
// wave takes two halves (from any tree waves) as one 8-block bitsliced batch.
struct WsSlot {
  uint4 seed[4][64];
  uint32_t half[64];   // output half-octet index (leaf block / 4) per lane
  uint32_t ctrl[64];   // bit j = control bit of leaf j; bit 31 = lane valid
};
enum : uint32_t { kSlotFree = 0, kSlotFilling = 1, kSlotFull = 2, kSlotDraining = 3 };

struct WsLds {
  LdsImage img;
  WsSlot slot[kWsSlots];
  uint32_t state[kWsSlots];
  uint32_t tree_done;
#if defined(DPF_WS_STATS)
  uint32_t stat[4];  // halves handed off, halves hashed by tree waves, value batches, value sleeps
#endif
};
#if defined(DPF_WS_STATS)
#define WS_STAT(i) (threadIdx.x & 63 ? 0 : atomicAdd(&lds.stat[i], 1u))
#else
#define WS_STAT(i) 0
#endif
static_assert(sizeof(WsLds) <= 160 * 1024, "LDS budget");

// Moves one slot from `from` to `to`: lanes 0..kWsSlots-1 read one slot state
// each (one LDS read for the scan), then lane 0 tries a compare-and-swap on the
// candidates.  Returns the slot index (or -1) to the whole wave.
__device__ __forceinline__ int ws_claim(uint32_t* state, uint32_t from, uint32_t to) {
  const int lane = threadIdx.x & 63;
  const uint32_t st = lane < kWsSlots
                          ? __hip_atomic_load(&state[lane], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP)
                          : ~0u;
  uint64_t cand = __ballot(st == from);
  while (cand) {
    const int s = __builtin_ctzll(cand);
    int won = 0;
    if (lane == 0) {
      uint32_t e = from;
      won = __hip_atomic_compare_exchange_strong(&state[s], &e, to, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (__builtin_amdgcn_readfirstlane(won)) return s;
    cand &= cand - 1;
  }
  return -1;
}
__device__ __forceinline__ void ws_set(uint32_t* state, int s, uint32_t v) {
  // LDS-only release: the slot's data reads/writes have completed (lgkmcnt).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store(&state[s], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct WsParams {
  int64_t num_items;  // subtrees of depth S in round 1
  int num_levels;
  int S;
  const dpf_block* seeds_in;
  const uint8_t* ctrl_in;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  char* out;
  int self_period;  // > 0: tree waves hash every self_period-th half themselves (A/B knob)
  RoundKeys rkl, rkr, rkv, rkd;
};

// One subtree of depth S (item index at that depth), all lanes of the wave in
// lockstep; `valid` = false lanes shadow another lane's item and store nothing.
template <int BITS, bool XOR>
__device__ __forceinline__ void ws_tree_item(WsLds& lds, const LdsLookup& lk, const WsParams& p,
                                             const FastIntLeaf<BITS, XOR>& leaf, int64_t item,
                                             int S, bool valid) {
  const int k0 = p.num_levels - S;
  const int G = S - 3;
  const int64_t ngroups = (int64_t)1 << G;
  const int lane = threadIdx.x & 63;
  const int64_t r = item >> k0;
  Block4 s = load_block(p.seeds_in + r);
  uint32_t t = p.ctrl_in[r] & 1u;
  for (int j = 0; j < k0; ++j) {
    const uint32_t bit = (uint32_t)((item >> (k0 - 1 - j)) & 1);
    path_step(lk, p.rkl, p.rkd, s, t, bit, lds.img.cw_seed[j], lds.img.cw_ctrl[j]);
  }
  const UniformRK rv[4] = {UniformRK{p.rkv.k}, UniformRK{p.rkv.k}, UniformRK{p.rkv.k},
                           UniformRK{p.rkv.k}};
  Block4 sib[kGMax];
  uint32_t tb = 0;
  const int64_t octet_base = item << G;
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
      children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.img.cw_seed[k0 + d],
                    lds.img.cw_ctrl[k0 + d], c0, t0, c1, t1);
      sib[d] = c1;
      tb = (tb & ~(1u << (d + 1))) | (t1 << (d + 1));
      node = c0;
      nt = t0;
    }
    if (g + 1 < ngroups) next = sib[G - (int)__builtin_ctzll((unsigned long long)(g + 1)) - 1];
    // The octet: 2 + 4 child hashes, then per half its 4 leaf seeds, handed
    // to a value wave or, with no slot free, hashed here on the T-table.
    const int lvl = k0 + G;
    Block4 c[2], q[4];
    uint32_t ct[2], qt[4];
    children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.img.cw_seed[lvl], lds.img.cw_ctrl[lvl],
                  c[0], ct[0], c[1], ct[1]);
    children_step_x2(lk, p.rkl.k, p.rkr.k, c[0], ct[0], c[1], ct[1], lds.img.cw_seed[lvl + 1],
                     lds.img.cw_ctrl[lvl + 1], q, qt);
    const int64_t octet = octet_base + g;
    // The second half's grandchildren wait in scratch (as in expand_octet_kernel).
    static_assert(12 - 3 <= kGMax - 2, "stash overlaps the DFS stack");
    sib[kGMax - 2] = q[2];
    sib[kGMax - 1] = q[3];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      Block4 l[4];
      uint32_t lt[4];
      if (hf == 1) {
        q[2] = sib[kGMax - 2];
        q[3] = sib[kGMax - 1];
      }
      children_step_x2(lk, p.rkl.k, p.rkr.k, q[2 * hf], qt[2 * hf], q[2 * hf + 1], qt[2 * hf + 1],
                       lds.img.cw_seed[lvl + 2], lds.img.cw_ctrl[lvl + 2], l, lt);
      const bool self = p.self_period > 0 && ((2 * g + hf) % p.self_period) == p.self_period - 1;
      const int sl = self ? -1 : ws_claim(lds.state, kSlotFree, kSlotFilling);
      if (sl >= 0) {
        WsSlot& w = lds.slot[sl];
        uint32_t bits = valid ? 0x80000000u : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          w.seed[j][lane] = make_uint4(l[j].w0, l[j].w1, l[j].w2, l[j].w3);
          bits |= lt[j] << j;
        }
        w.half[lane] = (uint32_t)(2 * octet + hf);
        w.ctrl[lane] = bits;
        ws_set(lds.state, sl, kSlotFull);
        (void)WS_STAT(0);
      } else {
        (void)WS_STAT(1);
        dpf_aes::mmo_hashN<4>(l, lk, rv);
        uint4* o = reinterpret_cast<uint4*>(p.out + octet * 128 + hf * 64);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const Block4 h = leaf.correct(l[j], lt[j]);
          if (valid) o[j] = make_uint4(h.w0, h.w1, h.w2, h.w3);
        }
      }
    }
  }
}

// Takes a full half-slot, waiting while none is full; -1 once every tree wave
// has finished and no full half-slot is left.
__device__ __forceinline__ int ws_take(WsLds& lds) {
  for (;;) {
    int sl = ws_claim(lds.state, kSlotFull, kSlotDraining);
    if (sl >= 0) return sl;
    const uint32_t done =
        __hip_atomic_load(&lds.tree_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (done == kWsTree) return ws_claim(lds.state, kSlotFull, kSlotDraining);
    (void)WS_STAT(3);
    __builtin_amdgcn_s_sleep(1);
  }
}

template <int BITS, bool XOR>
__device__ __forceinline__ void ws_value_wave(WsLds& lds, const WsParams& p,
                                              const FastIntLeaf<BITS, XOR>& leaf) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    const int sa = ws_take(lds);
    if (sa < 0) break;
    const int sb = ws_take(lds);  // -1 at the very end: a batch of one half
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    uint32_t x[32];
    uint32_t half[2], bits[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const WsSlot& w = lds.slot[h == 0 ? sa : (sb < 0 ? sa : sb)];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 v = w.seed[j][lane];
        const Block4 sg = dpf_aes::sigma(Block4{v.x, v.y, v.z, v.w});
        uint32_t* xj = x + 16 * h + 4 * j;
        xj[0] = sg.w0; xj[1] = sg.w1; xj[2] = sg.w2; xj[3] = sg.w3;
      }
      half[h] = w.half[lane];
      bits[h] = w.ctrl[lane];
    }
    if (sb < 0) bits[1] = 0;  // second half invalid
    (void)WS_STAT(2);
    ws_set(lds.state, sa, kSlotFree);
    if (sb >= 0) ws_set(lds.state, sb, kSlotFree);
    uint32_t ff[32];  // sigma(x), the MMO feed-forward
#pragma unroll
    for (int j = 0; j < 32; ++j) ff[j] = x[j];
    bsa::aes8_c<WsValueMasks>(x);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint4* o = reinterpret_cast<uint4*>(p.out + (int64_t)half[h] * 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = 16 * h + 4 * j;
        Block4 v{x[b] ^ ff[b], x[b + 1] ^ ff[b + 1], x[b + 2] ^ ff[b + 2], x[b + 3] ^ ff[b + 3]};
        v = leaf.correct(v, (bits[h] >> j) & 1u);
        if (bits[h] >> 31) o[j] = make_uint4(v.w0, v.w1, v.w2, v.w3);
      }
    }
  }
}

#if defined(DPF_WS_STATS)
__device__ __forceinline__ void ws_stats_report(WsLds& lds) {
  __syncthreads();
  if (threadIdx.x == 0 && (blockIdx.x % 64) == 0)
    printf("ws wg %d: halves handed off %u, hashed by tree waves %u, value batches %u, value sleeps %u\n",
           (int)blockIdx.x, lds.stat[0], lds.stat[1], lds.stat[2], lds.stat[3]);
}
#endif

template <int BITS, bool XOR>
__global__ __launch_bounds__(64 * (kWsTree + kWsValue)) __attribute__((amdgpu_waves_per_eu(4, 4)))
void expand_ws_kernel(WsParams p, FastIntLeaf<BITS, XOR> leaf) {
  __shared__ WsLds lds;
  leaf.init();
  fill_tables(lds.img.tab);
  fill_cws(lds.img, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  if (threadIdx.x < kWsSlots) lds.state[threadIdx.x] = kSlotFree;
  if (threadIdx.x == 0) lds.tree_done = 0;
#if defined(DPF_WS_STATS)
  if (threadIdx.x < 4) lds.stat[threadIdx.x] = 0;
#endif
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave >= kWsTree) {
#if defined(DPF_WS_VALUE_PRIO)
    __builtin_amdgcn_s_setprio(DPF_WS_VALUE_PRIO);
#endif
#if !defined(DPF_WS_NO_VALUE_WAVES)  // timing experiment: tree waves alone
    ws_value_wave(lds, p, leaf);
#endif
#if defined(DPF_WS_STATS)
    ws_stats_report(lds);
#endif
    return;
  }
#if defined(DPF_WS_TREE_PRIO)
  __builtin_amdgcn_s_setprio(DPF_WS_TREE_PRIO);
#endif
  const LdsLookup lk = make_lookup(lds.img);
  const int64_t lanes = (int64_t)gridDim.x * kWsTreeLanes;
  const int64_t gl = (int64_t)blockIdx.x * kWsTreeLanes + threadIdx.x;
  const int64_t wave_first = gl - (threadIdx.x & 63);
  int S = p.S;
  int64_t base = 0, count = p.num_items;  // items [base, base + count) of depth S
  for (;;) {
    const int64_t n = count < lanes ? count : lanes;
    if (wave_first < n) {
      const bool valid = gl < n;
      ws_tree_item(lds, lk, p, leaf, base + (valid ? gl : wave_first), S, valid);
    }
    if (count <= lanes) break;
    // The leftover subtrees, split for the next round.
    const int f = S - 2 >= 3 ? 2 : S - 3;
    base = (base + lanes) << f;
    count = (count - lanes) << f;
    S -= f;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(&lds.tree_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#if defined(DPF_WS_STATS)
  ws_stats_report(lds);
#endif
}

template <int BITS, bool XOR>
int launch(const WsParams& p, const dpf_block* vcw, int E, int party, hipStream_t s) {
  const FastIntLeaf<BITS, XOR> leaf{vcw, E, party, 16, {}};
  hipLaunchKernelGGL((expand_ws_kernel<BITS, XOR>), dim3((unsigned)num_cus()),
                     dim3(64 * (kWsTree + kWsValue)), 0, s,
                     p, leaf);
  HIP_TRY(hipGetLastError());
  return kOk;
}

}  // namespace

namespace dpf_rt {

int ws_subtree_depth(int64_t num_starts, int num_levels) {
  const int64_t lanes = (int64_t)num_cus() * kWsTreeLanes;
  if (num_levels < 6) return -1;
  int S = num_levels < 12 ? num_levels : 12;
  while (S > 5 && (num_starts << (num_levels - S)) < lanes) --S;
  if ((num_starts << (num_levels - S)) < lanes) return -1;
  // Half-octet indices are 32-bit in the hand-off slots.
  if (((num_starts << num_levels) >> 2) > 0xffffffffll) return -1;
  return S;
}

bool expand_ws_applies(int64_t num_starts, int num_levels, const dpf_aes_key* key_value) {
  const char* on = getenv("DPF_EXPAND_WS");  // opt-in: measured 2-4% slower than the octet kernel
  if (!on || on[0] != '1') return false;
  if (__builtin_memcmp(key_value->bytes, kWsValueKey, 16) != 0) return false;
  return ws_subtree_depth(num_starts, num_levels) > 0;
}

int launch_expand_ws(int64_t num_starts, const dpf_block* seeds_in, const uint8_t* control_in,
                     int num_levels, const dpf_block* cw_seed, const uint8_t* cw_left,
                     const uint8_t* cw_right, const dpf_aes_key* key_left,
                     const dpf_aes_key* key_right, const dpf_aes_key* key_value, int bits,
                     bool xor_leaf, int elements, const dpf_block* value_correction, int party,
                     void* out, hipStream_t s) {
  const int S = ws_subtree_depth(num_starts, num_levels);
  if (S < 0) return fail(kInternal, "launch_expand_ws: shape not supported");
  WsParams p;
  p.num_levels = num_levels;
  p.S = S;
  p.num_items = num_starts << (num_levels - S);
  p.seeds_in = seeds_in;
  p.ctrl_in = control_in;
  p.cw_seed = cw_seed;
  p.cw_left = cw_left;
  p.cw_right = cw_right;
  p.out = (char*)out;
  const char* sp = getenv("DPF_WS_SELF_PERIOD");
  p.self_period = sp ? atoi(sp) : 0;
  p.rkl = expand_key(key_left);
  p.rkr = expand_key(key_right);
  p.rkv = expand_key(key_value);
  p.rkd = p.rkl;
  for (int i = 0; i < 44; ++i) p.rkd.k[i] ^= p.rkr.k[i];
  switch (bits) {
    case 8: return xor_leaf ? launch<8, true>(p, value_correction, elements, party, s)
                            : launch<8, false>(p, value_correction, elements, party, s);
    case 16: return xor_leaf ? launch<16, true>(p, value_correction, elements, party, s)
                             : launch<16, false>(p, value_correction, elements, party, s);
    case 32: return xor_leaf ? launch<32, true>(p, value_correction, elements, party, s)
                             : launch<32, false>(p, value_correction, elements, party, s);
    case 64: return xor_leaf ? launch<64, true>(p, value_correction, elements, party, s)
                             : launch<64, false>(p, value_correction, elements, party, s);
    default: return xor_leaf ? launch<128, true>(p, value_correction, elements, party, s)
                             : launch<128, false>(p, value_correction, elements, party, s);
  }
}

}  // namespace dpf_rt
