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

template <int BITS, bool XOR>
int launch(const ExpandParams& p, const dpf_block* vcw, int E, int party, hipStream_t s) {
  const FastIntLeaf<BITS, XOR> leaf{vcw, E, party, 16, {}};
  int64_t g = (p.num_items + kHybBlock - 1) / kHybBlock;
  if (g > num_cus()) g = num_cus();   // one 128 KiB-table workgroup per CU
  hipLaunchKernelGGL((expand_hybrid_kernel<BITS, XOR>), dim3((unsigned)g), dim3(kHybBlock), 0, s,
                     p, leaf);
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
