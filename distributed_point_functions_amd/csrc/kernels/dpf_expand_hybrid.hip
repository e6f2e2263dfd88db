// dpf_expand_hybrid.hip -- full-domain expansion (dpf_hip_expand, rows a3-a6 and
// a12-a13 of SURVEY.md section 8) with the AES work split over BOTH of the
// CU's pipes: the tree's inner hashes (ExpandSeeds, distributed_point_function
// .cc:271-349) run on the LDS T-table AES of aes_core.h, the leaf value hashes
// (HashExpandedSeeds, cc:500-524, one third of all AES) run bitsliced on the
// VALU (bs_aes.h).  The T-table kernel is bound by the LDS pipe (160 lookups
// per block) with the VALU about half idle; this kernel puts the idle VALU to
// work on a third of the blocks.
//
// Work item = one subtree of depth S, as in expand_kernel: a path walk of k0
// levels to its root, then a depth-first visit whose bottom three levels are
// an OCTET: the node's two children (T-table, ILP2), its four grandchildren
// (ILP4) and its eight leaf seeds (2 x ILP4), whose value hashes are computed
// together as one 8-block bitsliced AES-128 under the fixed value key (every
// round-key mask an immediate).  The eight corrected leaf blocks of a lane
// are 128 contiguous bytes: every lane writes whole cache lines.
//
// Opt-in (DPF_EXPAND_HYBRID=1): measured 11% SLOWER than the T-table kernel at
// config 2 (20.6 vs 18.3-18.6 ms per 2^30 uint64 outputs, same box, bit-exact
// either way); DESIGN.md section 8 has the A/B table and the PMC reading.  The
// octet needs ~190 VGPRs (two waves per SIMD): the T-table phase then lacks
// the waves that hide its LDS latency, and a lone wave issues VALU at half rate.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../../include/dpf_hip.h"
#include "bs_aes.h"
#include "dpf_device.h"
#include "dpf_runtime.h"

using namespace dpf_rt;

namespace {

// Memory image of the reference's value PRG key kPrgKeyValue
// (distributed_point_function.cc:37-42: MakeUint128(0x05a5d1588c5423e3,
// 0x46a31101b21d1c98)), low 64 bits first.
constexpr uint8_t kValueKeyBytes[16] = {0x98, 0x1c, 0x1d, 0xb2, 0x01, 0x11, 0xa3, 0x46,
                                        0xe3, 0x23, 0x54, 0x8c, 0x58, 0xd1, 0xa5, 0x05};
struct ValueKeyMasks {
  static constexpr bsa::BsKeyMasks m = bsa::make_key_masks_c(kValueKeyBytes);
};

#ifndef DPF_HYB_WAVES
#define DPF_HYB_WAVES 2
#endif
#ifndef DPF_HYB_SMAX
#define DPF_HYB_SMAX 11
#endif
constexpr int kHybBlock = 256 * DPF_HYB_WAVES;  // 4 SIMDs x 64 lanes x waves per SIMD
constexpr int kHybSMax = DPF_HYB_SMAX;
constexpr int kHybGMax = kHybSMax - 3;          // DFS stack depth above the octets

// ---------------------------------------------------------------------------
// Software-pipelined variant (DPF_HYB_PIPE): the bitsliced rounds of octet
// g - 1 are spread over the T-table rounds of octet g's 2 + 4 + 8 inner
// hashes, all in one unrolled basic block, so every wave always has LDS
// lookups and independent VALU work in flight (the plain hybrid alternates
// an LDS-latency-bound phase with a VALU-bound one).
// ---------------------------------------------------------------------------
template <int First, int Last, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (First < Last) {
    f(std::integral_constant<int, First>{});
    static_for<First + 1, Last>(f);
  }
}

// Bitsliced rounds [A, B) (1..10; round 10 ends with the last AddRoundKey).
template <int A, int B>
__device__ __forceinline__ void bs_rounds(uint32_t* w) {
  static_for<A, B>([&](auto R) { bsa::round_c<ValueKeyMasks, decltype(R)::value>(w); });
}

// N MMO hashes on the T-table (x[i] under rk[i]) with bitsliced rounds
// [RB0, RB1) of the carried state bsw interleaved between the T-table rounds.
template <int N, int RB0, int RB1>
__device__ __forceinline__ void mmo_fused(Block4* x, const LdsLookup& lk, const UniformRK* rk,
                                          uint32_t* bsw) {
  Block4 s[N];
  uint32_t w[N][4];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    s[i] = dpf_aes::sigma(x[i]);
    w[i][0] = s[i].w0 ^ rk[i](0);
    w[i][1] = s[i].w1 ^ rk[i](1);
    w[i][2] = s[i].w2 ^ rk[i](2);
    w[i][3] = s[i].w3 ^ rk[i](3);
  }
  static_for<1, 10>([&](auto RR) {
    constexpr int r = decltype(RR)::value;
    uint32_t n[N][4];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        n[i][c] = lk.xor3(lk.template lookup<0, 0>(w[i][c]), lk.template lookup<1, 1>(w[i][(c + 1) & 3]),
                          lk.template lookup<2, 2>(w[i][(c + 2) & 3]));
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        n[i][c] = rk[i].mix(lk, n[i][c], lk.template lookup<3, 3>(w[i][(c + 3) & 3]), 4 * r + c);
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) w[i][c] = n[i][c];
    constexpr int nb = RB1 - RB0;
    bs_rounds<RB0 + (r - 1) * nb / 9, RB0 + r * nb / 9>(bsw);
#if !defined(DPF_HYB_NO_SCHED_FENCE)
    // Schedule each T-table round with its share of bitsliced work as one
    // window: interleaving stays within it and register pressure bounded.
    __builtin_amdgcn_sched_barrier(0);
#endif
  });
  auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    uint32_t xa = lk.template lookup<2, 0>(a), ya = lk.template lookup<3, 1>(b);
    uint32_t za = lk.template lookup<0, 2>(c), ua = lk.template lookup<1, 3>(d);
    uint32_t xy = (xa & 0x000000ffu) | (ya & 0xffffff00u);
    uint32_t zu = (za & 0x00ff0000u) | (ua & 0xff00ffffu);
    return ((xy & 0x0000ffffu) | (zu & 0xffff0000u)) ^ k;
  };
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const Block4 e{last(w[i][0], w[i][1], w[i][2], w[i][3], rk[i](40)),
                   last(w[i][1], w[i][2], w[i][3], w[i][0], rk[i](41)),
                   last(w[i][2], w[i][3], w[i][0], w[i][1], rk[i](42)),
                   last(w[i][3], w[i][0], w[i][1], w[i][2], rk[i](43))};
    x[i] = Block4{e.w0 ^ s[i].w0, e.w1 ^ s[i].w1, e.w2 ^ s[i].w2, e.w3 ^ s[i].w3};
  }
}

// Seed/control correction and control-bit extraction of hashed children
// (distributed_point_function.cc:323-343); par[i] is child i's parent bit,
// dir[i] its direction.
template <int N>
__device__ __forceinline__ void correct_children(Block4* h, const uint32_t* par, uint4 cs,
                                                 uint32_t cctl, uint32_t* t) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t m = 0u - par[i];
    h[i].w0 ^= cs.x & m; h[i].w1 ^= cs.y & m; h[i].w2 ^= cs.z & m; h[i].w3 ^= cs.w & m;
    t[i] = (h[i].w0 & 1u) ^ (par[i] & ((cctl >> (i & 1)) & 1u));
    h[i].w0 &= ~1u;
  }
}

template <int RB0, int RB1>
__device__ __forceinline__ void children_fused(const LdsLookup& lk, const uint32_t* rkl,
                                               const uint32_t* rkr, Block4 s, uint32_t t, uint4 cs,
                                               uint32_t cctl, Block4* c, uint32_t* ct,
                                               uint32_t* bsw) {
  c[0] = s;
  c[1] = s;
  const UniformRK rk[2] = {UniformRK{rkl}, UniformRK{rkr}};
  mmo_fused<2, RB0, RB1>(c, lk, rk, bsw);
  const uint32_t par[2] = {t, t};
  correct_children<2>(c, par, cs, cctl, ct);
}

template <int RB0, int RB1>
__device__ __forceinline__ void children_x2_fused(const LdsLookup& lk, const uint32_t* rkl,
                                                  const uint32_t* rkr, Block4 sa, uint32_t ta,
                                                  Block4 sb, uint32_t tb, uint4 cs, uint32_t cctl,
                                                  Block4* c, uint32_t* ct, uint32_t* bsw) {
  c[0] = sa; c[1] = sa; c[2] = sb; c[3] = sb;
  const UniformRK rk[4] = {UniformRK{rkl}, UniformRK{rkr}, UniformRK{rkl}, UniformRK{rkr}};
  mmo_fused<4, RB0, RB1>(c, lk, rk, bsw);
  const uint32_t par[4] = {ta, ta, tb, tb};
  correct_children<4>(c, par, cs, cctl, ct);
}

template <int BITS, bool XOR>
__global__ __launch_bounds__(kHybBlock)
__attribute__((amdgpu_waves_per_eu(DPF_HYB_WAVES, DPF_HYB_WAVES)))
void expand_hybrid_kernel(ExpandParams p, FastIntLeaf<BITS, XOR> leaf) {
  __shared__ LdsImage lds;
  leaf.init();
  fill_tables(lds.tab);
  fill_cws(lds, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  __syncthreads();
  const LdsLookup lk = make_lookup(lds);
  const int k0 = p.k0, S = p.S;
  const int G = S - 3;
  const int64_t ngroups = (int64_t)1 << G;
  for (int64_t item = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; item < p.num_items;
       item += (int64_t)gridDim.x * blockDim.x) {
    // 1. walk from the start seed to this item's subtree root.
    const int64_t r = item >> k0;
    Block4 s = load_block(p.seeds_in + r);
    uint32_t t = p.ctrl_in[r] & 1u;
    for (int j = 0; j < k0; ++j) {
      const uint32_t bit = (uint32_t)((item >> (k0 - 1 - j)) & 1);
      path_step(lk, p.rkl, p.rkd, s, t, bit, lds.cw_seed[j], lds.cw_ctrl[j]);
    }
    // 2. depth-first down to the octet roots (depth G), right children parked
    //    in sib[] exactly as in expand_kernel.
    Block4 sib[kHybGMax > 0 ? kHybGMax : 1];
    uint32_t tb = 0;
    const int64_t leaf_base = item << S;
    for (int64_t g = 0; g < ngroups; ++g) {
      Block4 node = s;
      uint32_t nt = t;
      int ds = 0;
      if (g != 0) {
        ds = G - (int)__builtin_ctzll((unsigned long long)g);
#pragma unroll
        for (int d = 1; d <= kHybGMax; ++d)
          if (d == ds) { node = sib[d - 1]; nt = (tb >> d) & 1u; }
      }
      for (int d = ds; d < G; ++d) {
        Block4 c0, c1;
        uint32_t t0, t1;
        children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.cw_seed[k0 + d], lds.cw_ctrl[k0 + d],
                      c0, t0, c1, t1);
#pragma unroll
        for (int e = 1; e <= kHybGMax; ++e)
          if (e == d + 1) sib[e - 1] = c1;
        tb = (tb & ~(1u << (d + 1))) | (t1 << (d + 1));
        node = c0;
        nt = t0;
      }
      // 3. the octet: 2 + 4 + 8 T-table hashes down to the eight leaf seeds.
      const int lvl = k0 + G;
      Block4 c[2], q[4], l[8];
      uint32_t ct[2], qt[4], lt[8];
      children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.cw_seed[lvl], lds.cw_ctrl[lvl], c[0],
                    ct[0], c[1], ct[1]);
      children_step_x2(lk, p.rkl.k, p.rkr.k, c[0], ct[0], c[1], ct[1], lds.cw_seed[lvl + 1],
                       lds.cw_ctrl[lvl + 1], q, qt);
      children_step_x2(lk, p.rkl.k, p.rkr.k, q[0], qt[0], q[1], qt[1], lds.cw_seed[lvl + 2],
                       lds.cw_ctrl[lvl + 2], l, lt);
      children_step_x2(lk, p.rkl.k, p.rkr.k, q[2], qt[2], q[3], qt[3], lds.cw_seed[lvl + 2],
                       lds.cw_ctrl[lvl + 2], l + 4, lt + 4);
      uint4* o = reinterpret_cast<uint4*>(p.out + (leaf_base + 8 * g) * 16);
      uint32_t tbits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) tbits |= lt[j] << j;
      // 4. the eight value hashes, bitsliced: w = sigma(leaf seeds).
      uint32_t w[32];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const Block4 sg = dpf_aes::sigma(l[j]);
        w[4 * j] = sg.w0; w[4 * j + 1] = sg.w1; w[4 * j + 2] = sg.w2; w[4 * j + 3] = sg.w3;
      }
      uint32_t ff[32];   // sigma(x) for the MMO feed-forward
#pragma unroll
      for (int j = 0; j < 32; ++j) ff[j] = w[j];
      bsa::aes8_c<ValueKeyMasks>(w);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint4 sv = make_uint4(ff[4 * j], ff[4 * j + 1], ff[4 * j + 2], ff[4 * j + 3]);
        Block4 h{w[4 * j] ^ sv.x, w[4 * j + 1] ^ sv.y, w[4 * j + 2] ^ sv.z, w[4 * j + 3] ^ sv.w};
        h = leaf.correct(h, (tbits >> j) & 1u);
        o[j] = make_uint4(h.w0, h.w1, h.w2, h.w3);
      }
    }
  }
}

// The pipelined kernel: octet g's inner hashes carry octet g - 1's bitsliced
// value hashes (rounds 1-2 in the ILP2 step, 3-5, 6-8 and 9-10 in the three
// ILP4 steps); octet g's own leaves are then transposed into the carried
// planes.  The last octet of a lane is finished after its last item.
template <int BITS, bool XOR>
__global__ __launch_bounds__(kHybBlock)
__attribute__((amdgpu_waves_per_eu(DPF_HYB_WAVES, DPF_HYB_WAVES)))
void expand_hybrid_pipe_kernel(ExpandParams p, FastIntLeaf<BITS, XOR> leaf) {
  __shared__ LdsImage lds;
  leaf.init();
  fill_tables(lds.tab);
  fill_cws(lds, p.cw_seed, p.cw_left, p.cw_right, p.num_levels);
  __syncthreads();
  const LdsLookup lk = make_lookup(lds);
  const int k0 = p.k0, S = p.S;
  const int G = S - 3;
  const int64_t ngroups = (int64_t)1 << G;
  // Carried: the pending octet's planes; its sigma(x) for the MMO feed-forward
  // is parked in its own 128 output bytes (written back a whole octet later,
  // so the reload's latency is hidden), unless DPF_HYB_PIPE_REG_FF.
  uint32_t bsw[32];
#if defined(DPF_HYB_PIPE_REG_FF)
  uint32_t ff[32];
#endif
  uint32_t ptbits = 0;        // control bits of the pending octet's leaves
  uint4* pout = nullptr;      // its 128 output bytes; NULL = nothing pending
#pragma unroll
  for (int j = 0; j < 32; ++j) bsw[j] = 0;
  auto finish = [&]() {       // from planes, feed-forward, correct, store the pending octet
    bsa::from_planes(bsw);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#if defined(DPF_HYB_PIPE_REG_FF)
      const uint4 f = make_uint4(ff[4 * j], ff[4 * j + 1], ff[4 * j + 2], ff[4 * j + 3]);
#else
      const uint4 f = pout[j];
#endif
      Block4 h{bsw[4 * j] ^ f.x, bsw[4 * j + 1] ^ f.y, bsw[4 * j + 2] ^ f.z, bsw[4 * j + 3] ^ f.w};
      h = leaf.correct(h, (ptbits >> j) & 1u);
      pout[j] = make_uint4(h.w0, h.w1, h.w2, h.w3);
    }
  };
  for (int64_t item = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; item < p.num_items;
       item += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = item >> k0;
    Block4 s = load_block(p.seeds_in + r);
    uint32_t t = p.ctrl_in[r] & 1u;
    for (int j = 0; j < k0; ++j) {
      const uint32_t bit = (uint32_t)((item >> (k0 - 1 - j)) & 1);
      path_step(lk, p.rkl, p.rkd, s, t, bit, lds.cw_seed[j], lds.cw_ctrl[j]);
    }
    // The DFS stack lives in scratch (dynamically indexed: one 16-byte store
    // per push, one load per octet), not in the VGPRs the pipelined octet
    // needs; the next octet's root is loaded one octet ahead.
    Block4 sib[kHybGMax > 0 ? kHybGMax : 1];
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
        children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.cw_seed[k0 + d], lds.cw_ctrl[k0 + d],
                      c0, t0, c1, t1);
        sib[d] = c1;
        tb = (tb & ~(1u << (d + 1))) | (t1 << (d + 1));
        node = c0;
        nt = t0;
      }
      if (g + 1 < ngroups) next = sib[G - (int)__builtin_ctzll((unsigned long long)(g + 1)) - 1];
      const int lvl = k0 + G;
      Block4 c[2], q[4], l[8];
      uint32_t ct[2], qt[4], lt[8];
      if (pout) {
        children_fused<1, 3>(lk, p.rkl.k, p.rkr.k, node, nt, lds.cw_seed[lvl], lds.cw_ctrl[lvl], c,
                             ct, bsw);
        children_x2_fused<3, 6>(lk, p.rkl.k, p.rkr.k, c[0], ct[0], c[1], ct[1],
                                lds.cw_seed[lvl + 1], lds.cw_ctrl[lvl + 1], q, qt, bsw);
        children_x2_fused<6, 9>(lk, p.rkl.k, p.rkr.k, q[0], qt[0], q[1], qt[1],
                                lds.cw_seed[lvl + 2], lds.cw_ctrl[lvl + 2], l, lt, bsw);
        children_x2_fused<9, 11>(lk, p.rkl.k, p.rkr.k, q[2], qt[2], q[3], qt[3],
                                 lds.cw_seed[lvl + 2], lds.cw_ctrl[lvl + 2], l + 4, lt + 4, bsw);
        finish();
      } else {
        children_step(lk, p.rkl.k, p.rkr.k, node, nt, lds.cw_seed[lvl], lds.cw_ctrl[lvl], c[0],
                      ct[0], c[1], ct[1]);
        children_step_x2(lk, p.rkl.k, p.rkr.k, c[0], ct[0], c[1], ct[1], lds.cw_seed[lvl + 1],
                         lds.cw_ctrl[lvl + 1], q, qt);
        children_step_x2(lk, p.rkl.k, p.rkr.k, q[0], qt[0], q[1], qt[1], lds.cw_seed[lvl + 2],
                         lds.cw_ctrl[lvl + 2], l, lt);
        children_step_x2(lk, p.rkl.k, p.rkr.k, q[2], qt[2], q[3], qt[3], lds.cw_seed[lvl + 2],
                         lds.cw_ctrl[lvl + 2], l + 4, lt + 4);
      }
      // This octet's leaves become the pending bitsliced state.
      pout = reinterpret_cast<uint4*>(p.out + (leaf_base + 8 * g) * 16);
      ptbits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ptbits |= lt[j] << j;
        const Block4 sg = dpf_aes::sigma(l[j]);
        bsw[4 * j] = sg.w0;
        bsw[4 * j + 1] = sg.w1;
        bsw[4 * j + 2] = sg.w2;
        bsw[4 * j + 3] = sg.w3;
#if defined(DPF_HYB_PIPE_REG_FF)
        ff[4 * j] = sg.w0; ff[4 * j + 1] = sg.w1; ff[4 * j + 2] = sg.w2; ff[4 * j + 3] = sg.w3;
#else
        pout[j] = make_uint4(sg.w0, sg.w1, sg.w2, sg.w3);
#endif
      }
      bsa::to_planes(bsw);
#pragma unroll
      for (int j = 0; j < 32; ++j) bsw[j] = bsa::xor_mask(bsw[j], ValueKeyMasks::m.m[0][j]);
    }
  }
  if (pout) {
    bs_rounds<1, 11>(bsw);
    finish();
  }
}

template <int BITS, bool XOR>
int launch(const ExpandParams& p, const dpf_block* vcw, int E, int party, hipStream_t s) {
  const FastIntLeaf<BITS, XOR> leaf{vcw, E, party, 16, {}};
  int64_t g = (p.num_items + kHybBlock - 1) / kHybBlock;
  if (g > num_cus()) g = num_cus();   // one 128 KiB-table workgroup per CU
#if defined(DPF_HYB_NOPIPE)
  hipLaunchKernelGGL((expand_hybrid_kernel<BITS, XOR>), dim3((unsigned)g), dim3(kHybBlock), 0, s,
                     p, leaf);
#else
  hipLaunchKernelGGL((expand_hybrid_pipe_kernel<BITS, XOR>), dim3((unsigned)g), dim3(kHybBlock), 0,
                     s, p, leaf);
#endif
  HIP_TRY(hipGetLastError());
  return kOk;
}

}  // namespace

namespace dpf_rt {

bool expand_hybrid_applies(int64_t num_starts, int num_levels, const dpf_aes_key* key_value,
                           const dpf_value_desc* desc, int elements_per_leaf) {
  const char* on = getenv("DPF_EXPAND_HYBRID");
  if (!on || on[0] != '1') return false;
  if (!fast_int(desc) || elements_per_leaf != desc->elements_per_block) return false;
  if (__builtin_memcmp(key_value->bytes, kValueKeyBytes, 16) != 0) return false;
  // At least one octet (eight leaves) per lane of a full launch.
  if (num_levels < 3) return false;
  const int64_t lanes = (int64_t)num_cus() * kHybBlock;
  return (num_starts << num_levels) >= lanes * 8;
}

int launch_expand_hybrid(int64_t num_starts, const dpf_block* seeds_in, const uint8_t* control_in,
                         int num_levels, const dpf_block* cw_seed, const uint8_t* cw_left,
                         const uint8_t* cw_right, const dpf_aes_key* key_left,
                         const dpf_aes_key* key_right, const dpf_aes_key* key_value,
                         const dpf_value_desc* desc, const dpf_block* value_correction, int party,
                         void* out, hipStream_t s) {
  const int64_t lanes = (int64_t)num_cus() * kHybBlock;
  int S = num_levels < kHybSMax ? num_levels : kHybSMax;
  while (S > 3 && (num_starts << (num_levels - S)) < lanes) --S;
  ExpandParams p;
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
  const int E = desc->elements_per_block;
  const bool x = desc->kind[0] == DPF_LEAF_XOR;
  switch (desc->bits[0]) {
    case 8: return x ? launch<8, true>(p, value_correction, E, party, s)
                     : launch<8, false>(p, value_correction, E, party, s);
    case 16: return x ? launch<16, true>(p, value_correction, E, party, s)
                      : launch<16, false>(p, value_correction, E, party, s);
    case 32: return x ? launch<32, true>(p, value_correction, E, party, s)
                      : launch<32, false>(p, value_correction, E, party, s);
    case 64: return x ? launch<64, true>(p, value_correction, E, party, s)
                      : launch<64, false>(p, value_correction, E, party, s);
    default: return x ? launch<128, true>(p, value_correction, E, party, s)
                      : launch<128, false>(p, value_correction, E, party, s);
  }
}

}  // namespace dpf_rt
