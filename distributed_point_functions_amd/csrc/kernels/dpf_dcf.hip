// dpf_dcf.hip -- batched DistributedComparisonFunction::Evaluate on gfx950
// (dcf/distributed_comparison_function.h:83-105): one walk
// down x's tree path per (key, x) serves every hierarchy level.
//
// Its own translation unit so that it is built with the iterative-ilp
// scheduler (build_native.py) whatever dpf_batch.hip needs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "../../../include/dpf_hip.h"
#include "dpf_device.h"
#include "dpf_runtime.h"

using namespace dpf_rt;

// DistributedComparisonFunction::Evaluate (dcf/distributed_comparison_function
// .h:83-105) sums, over the hierarchy levels i < n with bit (n-1-i) of x
// clear, EvaluateAt(key, i, {x >> (n - i)}) of an n-level incremental DPF
// whose level i has log domain i.
namespace {

constexpr int kDcfMaxLevels = 128;
constexpr int kDcfMaxLeaves = 4;

struct DcfLevels {
  int n;                              // hierarchy levels = DCF log domain size
  uint8_t depth[kDcfMaxLevels];       // hierarchy_to_tree
  uint8_t blocks[kDcfMaxLevels];      // blocks_needed per level
  const dpf_block* vcw[kDcfMaxLevels];  // per level: [key][E * num_leaves]
};

struct DcfParams {
  int64_t num_keys, points_per_key, num_items;
  int shared_points;
  int cw_stride;
  int vcw_stride;  // E * num_leaves
  int esz;
  int xor_mode;
  const dpf_block* key_seed;
  const uint8_t* party;
  const dpf_block* points;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  char* out;
  RoundKeys rkl, rkd, rkv;
  int64_t dyn_per_wg;  // take_chunk's per_wg (0: grid stride)
};

__device__ __forceinline__ u128 shr128(u128 x, int s) { return s >= 128 ? (u128)0 : x >> s; }

template <int BITS, bool FAST>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void dcf_eval_kernel(
    DcfParams p, DcfLevels lv, GenericLeaf g) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h)
  fill_tables(lds.tab);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const LdsLookup lk = make_lookup(lds, KeySet{key_ref(p.rkl), KeyRef{}, key_ref(p.rkv), key_ref(p.rkd)});
  const int n = lv.n;
  const int dmax = lv.depth[n - 1];
  // Items by grid stride, or 64 at a time per wave (dyn_per_wg > 0).
  const int64_t nch = (p.num_items + 63) / 64;
  for (int64_t u = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.num_items)
                                : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       u < p.num_items;
       u = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, nch, p.num_items)
                        : u + (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = u / p.points_per_key, j = u - k * p.points_per_key;
    const u128 x = dpf_u128(p.points[p.shared_points ? j : u]);
    const int party = p.party[k] & 1;
    Block4 s = load_block(p.key_seed + k);
    uint32_t t = (uint32_t)party;
    const dpf_block* cws = p.cw_seed + k * p.cw_stride;
    const uint8_t* cl = p.cw_left + k * p.cw_stride;
    const uint8_t* cr = p.cw_right + k * p.cw_stride;
    u128 acc[FAST ? 1 : kDcfMaxLeaves];
    const int nl = FAST ? 1 : g.d.num_leaves;
    for (int e = 0; e < nl; ++e) acc[e] = 0;
    int level = 0;
    for (int d = 0; d <= dmax; ++d) {
      // Next node on x's path (computed beside the value hash when FAST).
      const uint32_t bit = d < dmax && n < 128 ? (uint32_t)(shr128(x, n - d - 1) & 1) : 0u;
      Block4 hv = s, hn = s;
      if (FAST) {
        if (d < dmax)
          dpf_aes::mmo_hash2(hv, hn, lk, UniformRK{lk.ks.v}, SelectRK{lk.ks.l, lk.ks.d, 0u - bit});
        else
          hv = dpf_aes::mmo_hash(s, lk, UniformRK{lk.ks.v});
      }
      for (; level < n && lv.depth[level] == d; ++level) {
        const bool take = ((shr128(x, n - 1 - level)) & 1) == 0;  // current_bit == 0
        const u128 prefix = n < 128 ? shr128(x, n - level) : (u128)0;
        const int bi = (int)(prefix & (((u128)1 << (level - d)) - 1));
        const dpf_block* vcw = lv.vcw[level] + k * p.vcw_stride;
        if (FAST) {
          const u128 v = fast_point_value<BITS>(hv, t, bi, dpf_u128(vcw[bi]), party, p.xor_mode);
          if (take) {
            if (p.xor_mode) acc[0] ^= v; else acc[0] += v;
          }
        } else {
          GenericLeaf lf = g;
          lf.d.blocks_needed = lv.blocks[level];
          lf.vcw = vcw;
          lf.party = party;
          char buf[16 * kDcfMaxLeaves];
          lf.convert_store(lk, lk.ks.v, s, t, bi, 1, buf);
          int off = 0;
          for (int e = 0; e < nl; ++e) {
            const int lb = g.d.bits[e] >> 3;
            const u128 v = GenericLeaf::load_le(reinterpret_cast<const uint8_t*>(buf) + off, lb);
            off += lb;
            if (take) acc[e] = leaf_group_add(g.d, e, acc[e], v);
          }
        }
      }
      if (d == dmax) break;
      const dpf_block c = cws[d];
      const uint4 cs = make_uint4((uint32_t)c.low, (uint32_t)(c.low >> 32), (uint32_t)c.high,
                                  (uint32_t)(c.high >> 32));
      const uint32_t cctl = (uint32_t)(cl[d] & 1) | ((uint32_t)(cr[d] & 1) << 1);
      if (FAST) {
        const uint32_t m = 0u - t;
        hn.w0 ^= cs.x & m; hn.w1 ^= cs.y & m; hn.w2 ^= cs.z & m; hn.w3 ^= cs.w & m;
        const uint32_t nt = (hn.w0 & 1u) ^ (t & ((cctl >> bit) & 1u));
        hn.w0 &= ~1u;
        s = hn;
        t = nt;
      } else {
        path_step(lk, lk.ks.l, lk.ks.d, s, t, bit, cs, cctl);
      }
    }
    char* o = p.out + u * (int64_t)p.esz;
    if (FAST) {
      store_bits<BITS>(o, acc[0]);
    } else {
      for (int e = 0; e < nl; ++e) {
        const int lb = g.d.bits[e] >> 3;
        GenericLeaf::store_le(o, acc[e], lb);
        o += lb;
      }
    }
  }
}


// ---------------------------------------------------------------------------
// dcf_fast_kernel: the DCF every DistributedComparisonFunction builds with a
// plain integer / XorWrapper value type.  Its DPF maps hierarchy level i to
// tree depth i (proto_validator.cc:131-136: tree_level = max(levels so far,
// ...), and level i has log domain i), so level i's point x >> (n - i) is x's
// depth-i node itself and its block index is 0
// (distributed_point_function.h:993-1002):
//   value_i = element 0 of H_value(node_i), + cw_i's element 0 if t_i,
//   summed iff bit (n-1-i) of x is 0 -- the bit that also steers the walk
//   from node_i to node_{i+1} (for n == 128 the reference evaluates every
//   level at prefix 0, so the walk always goes left).
// Party 1's negation is linear and applied once to the sum.  At every depth
// the value hashes and path steps of ITEMS (key, x) pairs run as one
// interleaved group of 2 * ITEMS AES chains (value key | per-lane key select).
// With UNIFORM (points_per_key % (64 * ITEMS) == 0) a wave's items share one
// key, whose correction words are then wave-uniform loads.  Each level's
// correction words are loaded one level ahead of their use.
struct DcfFastParams {
  int64_t num_items, points_per_key, num_groups;  // groups of 64 * ITEMS items
  int n;
  int shared_points;
  int cw_stride;
  int vcw_stride;  // dpf_blocks per key row of a level's value correction
  int esz;
  const dpf_block* key_seed;
  const uint8_t* party;
  const dpf_block* points;
  const dpf_block* cw_seed;
  const uint8_t* cw_left;
  const uint8_t* cw_right;
  char* out;
  RoundKeys rkl, rkd, rkv;
  int64_t dyn_per_wg;  // dcf_fast_kernel: take_chunk's per_wg (0: grid stride)
};

struct DcfVcw {
  const dpf_block* level[kDcfMaxLevels];  // per level: [key][E] value corrections
};

template <int BITS, bool XOR, bool UNIFORM, int ITEMS>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void dcf_fast_kernel(DcfFastParams p,
                                                                         DcfVcw vc) {
  __shared__ LdsImage lds;
  __shared__ int next_chunk;   // take_chunk (dpf_device.h)
  fill_tables(lds.tab);
  if (threadIdx.x == 0) next_chunk = 0;
  __syncthreads();
  const LdsLookup lk = make_lookup(lds, KeySet{key_ref(p.rkl), KeyRef{}, key_ref(p.rkv), key_ref(p.rkd)});
  const int n = p.n;
  using Acc = typename std::conditional<BITS == 128, u128, uint64_t>::type;
  // Groups of 64 lanes by grid stride, or taken one at a time per wave
  // (dyn_per_wg > 0).
  const int64_t done = p.num_groups * 64;
  for (int64_t g = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, p.num_groups, done)
                                : blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       (g >> 6) < p.num_groups;
       g = p.dyn_per_wg ? take_chunk(&next_chunk, p.dyn_per_wg, p.num_groups, done)
                        : g + (int64_t)gridDim.x * blockDim.x) {
    const int64_t base = (g >> 6) * (64 * ITEMS) + (g & 63);
    int64_t u[ITEMS], k[ITEMS];
    bool valid[ITEMS];
    Block4 s[ITEMS], x[ITEMS];
    uint32_t t[ITEMS], party[ITEMS];
    Acc acc[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int64_t uj = base + 64 * j;
      valid[j] = uj < p.num_items;
      u[j] = valid[j] ? uj : p.num_items - 1;
      k[j] = u[j] / p.points_per_key;
      if (UNIFORM) k[j] = (int64_t)__builtin_amdgcn_readfirstlane((int)k[j]);
      x[j] = load_block(p.points + (p.shared_points ? u[j] - k[j] * p.points_per_key : u[j]));
      party[j] = p.party[k[j]] & 1u;
      s[j] = load_block(p.key_seed + k[j]);
      t[j] = party[j];
      acc[j] = 0;
    }
    // Level d's correction words, loaded one level ahead.
    uint4 cw[ITEMS];
    uint32_t cc[ITEMS];
    Acc cv[ITEMS];
    auto load_level = [&](int d) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int64_t row = k[j] * p.cw_stride + d;
        cw[j] = d + 1 < n ? *reinterpret_cast<const uint4*>(p.cw_seed + row) : make_uint4(0, 0, 0, 0);
        cc[j] = d + 1 < n ? ((uint32_t)(p.cw_left[row] & 1) | ((uint32_t)(p.cw_right[row] & 1) << 1))
                          : 0u;
        const dpf_block c = vc.level[d][k[j] * p.vcw_stride];
        if constexpr (BITS == 128) cv[j] = dpf_u128(c); else cv[j] = c.low;
      }
    };
    load_level(0);
    for (int d = 0; d < n; ++d) {
      uint4 cwd[ITEMS];
      uint32_t ccd[ITEMS];
      Acc cvd[ITEMS];
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) { cwd[j] = cw[j]; ccd[j] = cc[j]; cvd[j] = cv[j]; }
      if (d + 1 < n) load_level(d + 1);
      const int pos = n - 1 - d;  // bit of x deciding level d's sum and the next step
      uint32_t xb[ITEMS], pb[ITEMS];
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        xb[j] = path_bit(x[j], pos);
        pb[j] = n < 128 ? xb[j] : 0u;
      }
      Block4 h[2 * ITEMS];
      if (d + 1 < n) {
        UniformRK rv[ITEMS];
        SelectRK rs[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
          h[j] = s[j];
          h[ITEMS + j] = s[j];
          rv[j] = UniformRK{lk.ks.v};
          rs[j] = SelectRK{lk.ks.l, lk.ks.d, 0u - pb[j]};
        }
        dpf_aes::mmo_hashAB<ITEMS, ITEMS>(h, lk, rv, rs);
      } else {
        UniformRK rv[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
          h[j] = s[j];
          rv[j] = UniformRK{lk.ks.v};
        }
        dpf_aes::mmo_hashN<ITEMS>(h, lk, rv);
      }
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        // Level d's value: element 0 of the value hash, corrected if t.
        Acc v;
        if constexpr (BITS == 128) v = block_u128(h[j]);
        else v = ((uint64_t)h[j].w1 << 32) | h[j].w0;
        const Acc tc = t[j] ? cvd[j] : (Acc)0;
        const Acc take = xb[j] ? (Acc)0 : ~(Acc)0;
        if constexpr (XOR) acc[j] ^= (v ^ tc) & take;
        else acc[j] += (v + tc) & take;
        // Step to node d + 1 (distributed_point_function.cc:323-343).
        if (d + 1 < n) {
          Block4 hn = h[ITEMS + j];
          const uint32_t m = 0u - t[j];
          hn.w0 ^= cwd[j].x & m; hn.w1 ^= cwd[j].y & m; hn.w2 ^= cwd[j].z & m; hn.w3 ^= cwd[j].w & m;
          t[j] = (hn.w0 & 1u) ^ (t[j] & ((ccd[j] >> pb[j]) & 1u));
          hn.w0 &= ~1u;
          s[j] = hn;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      Acc r = acc[j];
      if (!XOR && party[j]) r = (Acc)0 - r;
      if (valid[j]) store_bits<BITS>(p.out + u[j] * (int64_t)p.esz, (u128)r);
    }
  }
}

// Latency mode of dcf_fast_kernel (small calls: BM_EvaluateDcf evaluates one
// x per call): one (key, x) per lane QUAD, lane c computing AES column c of
// the level's value hash and path step together (dpf_device.h quad::).
template <int BITS, bool XOR>
__global__ __launch_bounds__(kBlock) DPF_WAVES_ATTR void dcf_fast_quad_kernel(DcfFastParams p,
                                                                              DcfVcw vc) {
  __shared__ LdsImage lds;
  fill_tables(lds.tab);
  __syncthreads();
  const LdsLookup lk = make_lookup(lds);
  const quad::Keys kl = quad::keys_of(p.rkl), kd = quad::keys_of(p.rkd), kv = quad::keys_of(p.rkv);
  const int n = p.n;
  const int c = quad::column();
  using Acc = typename std::conditional<BITS == 128, u128, uint64_t>::type;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; (g >> 2) < p.num_items;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = g >> 2;
    const int64_t k = u / p.points_per_key;
    const Block4 x = load_block(p.points + (p.shared_points ? u - k * p.points_per_key : u));
    const uint32_t party = p.party[k] & 1u;
    uint32_t s = reinterpret_cast<const uint32_t*>(p.key_seed + k)[c];
    uint32_t t = party;
    Acc acc = 0;
    for (int d = 0; d < n; ++d) {
      const int64_t row = k * p.cw_stride + d;
      const int pos = n - 1 - d;  // bit of x deciding level d's sum and the next step
      const uint32_t xb = path_bit(x, pos), pb = n < 128 ? xb : 0u;
      const uint32_t sg = quad::sigma(s);
      uint32_t hv = sg, hn = sg;
      if (d + 1 < n)
        quad::encrypt2(hv, hn, lk, kv, kl, kd, 0u - pb);
      else
        hv = quad::encrypt(hv, lk, kv, kv, 0u);
      hv ^= sg;
      hn ^= sg;
      // Level d's value: element 0 of the value hash, corrected if t, summed
      // iff bit pos of x is 0 (lane 0 holds the quad's columns in order).
      const Block4 h = quad::gather(hv);
      const dpf_block cvb = vc.level[d][k * p.vcw_stride];
      Acc v, cv;
      if constexpr (BITS == 128) {
        v = block_u128(h);
        cv = dpf_u128(cvb);
      } else {
        v = ((uint64_t)h.w1 << 32) | h.w0;
        cv = cvb.low;
      }
      const Acc tc = t ? cv : (Acc)0;
      const Acc take = xb ? (Acc)0 : ~(Acc)0;
      if constexpr (XOR) acc ^= (v ^ tc) & take;
      else acc += (v + tc) & take;
      if (d + 1 < n) {  // step to node d + 1 (distributed_point_function.cc:323-343)
        const uint32_t cs = reinterpret_cast<const uint32_t*>(p.cw_seed + row)[c];
        const uint32_t cc = (uint32_t)(p.cw_left[row] & 1) | ((uint32_t)(p.cw_right[row] & 1) << 1);
        hn ^= cs & (0u - t);
        const uint32_t nt = (quad::from_lane0(hn) & 1u) ^ (t & ((cc >> pb) & 1u));
        if (c == 0) hn &= ~1u;
        s = hn;
        t = nt;
      }
    }
    if (c == 0) {
      if (!XOR && party) acc = (Acc)0 - acc;
      store_bits<BITS>(p.out + u * (int64_t)p.esz, (u128)acc);
    }
  }
}

// DPF_DCF_QUAD=0 (read per launch) turns the latency mode off (A/B hook).
bool dcf_quad_on() {
  const char* v = getenv("DPF_DCF_QUAD");
  return !(v && v[0] == '0');
}

template <int BITS, bool XOR>
void launch_dcf_fast(const DcfFastParams& p0, const DcfVcw& vc, hipStream_t s) {
  if (p0.num_items <= (int64_t)num_cus() * 64 && dcf_quad_on()) {
    const int blk = block_for(p0.num_items * 4);
    hipLaunchKernelGGL((dcf_fast_quad_kernel<BITS, XOR>), dim3(grid_for(p0.num_items * 4, blk)),
                       dim3(blk), 0, s, p0, vc);
    return;
  }
  // One (key, x) pair per lane: two pairs (ILP4, 119-123 VGPRs) measured
  // 11% slower at the bench size (profiles/r13_ab.txt).
  DcfFastParams p = p0;
  p.num_groups = (p.num_items + 63) / 64;
  const int blk = block_for(p.num_groups * 64);
  const dim3 grid(grid_for(p.num_groups * 64, blk)), block(blk);
  // DPF_DCF_DYNAMIC=0: a fixed share of groups per thread (A/B hook).
  p.dyn_per_wg = dynamic_chunks_per_wg(p.num_groups * 64, (int)grid.x, blk, "DPF_DCF_DYNAMIC");
  if (p.points_per_key % 64 == 0)
    hipLaunchKernelGGL((dcf_fast_kernel<BITS, XOR, true, 1>), grid, block, 0, s, p, vc);
  else
    hipLaunchKernelGGL((dcf_fast_kernel<BITS, XOR, false, 1>), grid, block, 0, s, p, vc);
}
}  // namespace

extern "C" int dpf_hip_dcf_eval_batch(int64_t num_keys, int64_t points_per_key, int shared_points,
                                      int num_levels, const int32_t* level_depth,
                                      const int32_t* level_blocks, const dpf_block* key_seed,
                                      const uint8_t* party, const dpf_block* points,
                                      const dpf_block* cw_seed, const uint8_t* cw_left,
                                      const uint8_t* cw_right, int cw_stride,
                                      const dpf_block* const* value_correction,
                                      const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                                      const dpf_aes_key* key_value, const dpf_value_desc* desc,
                                      void* out, void* stream) {
  int st = validate_desc(desc);
  if (st) return st;
  if (num_keys < 0 || points_per_key < 0 || num_levels < 1 || num_levels > kDcfMaxLevels)
    return fail(kInvalidArgument, "num_keys, points_per_key or num_levels out of range");
  if (!level_depth || !level_blocks || !value_correction)
    return fail(kInvalidArgument, "NULL level table");
  DcfLevels lv;
  memset(&lv, 0, sizeof(lv));
  lv.n = num_levels;
  for (int i = 0; i < num_levels; ++i) {
    const int dep = level_depth[i];
    if (dep < 0 || dep > i || (i > 0 && (dep < level_depth[i - 1] || dep > level_depth[i - 1] + 1)) ||
        (i == 0 && dep != 0) || dep >= cw_stride + 1 || i - dep > 7)
      return fail(kInvalidArgument, "level depths are not a DCF hierarchy");
    if (level_blocks[i] < 1 || level_blocks[i] > kBMax)
      return fail(kUnimplemented, "value type needs too many AES blocks for the GPU path");
    if (!value_correction[i]) return fail(kInvalidArgument, "NULL value correction");
    lv.depth[i] = (uint8_t)dep;
    lv.blocks[i] = (uint8_t)level_blocks[i];
    lv.vcw[i] = value_correction[i];
  }
  if (lv.depth[num_levels - 1] > cw_stride) return fail(kInvalidArgument, "cw_stride too small");
  const bool fast = fast_int(desc);
  if (!fast && desc->num_leaves > kDcfMaxLeaves)
    return fail(kUnimplemented, "DCF value type has too many leaves for the GPU path");
  const int64_t items = num_keys * points_per_key;
  if (items == 0) return kOk;
  if (!key_seed || !party || !points || !out || !key_left || !key_right || !key_value ||
      (lv.depth[num_levels - 1] > 0 && (!cw_seed || !cw_left || !cw_right)))
    return fail(kInvalidArgument, "NULL pointer");
  DcfParams p;
  memset(&p, 0, sizeof(p));
  p.num_keys = num_keys;
  p.points_per_key = points_per_key;
  p.num_items = items;
  p.shared_points = shared_points ? 1 : 0;
  p.cw_stride = cw_stride;
  p.vcw_stride = desc->elements_per_block * desc->num_leaves;
  p.esz = packed_size(desc);
  p.xor_mode = desc->kind[0] == DPF_LEAF_XOR;
  p.key_seed = key_seed;
  p.party = party;
  p.points = points;
  p.cw_seed = cw_seed;
  p.cw_left = cw_left;
  p.cw_right = cw_right;
  p.out = (char*)out;
  p.rkl = expand_key(key_left);
  p.rkd = xor_keys(p.rkl, expand_key(key_right));
  p.rkv = expand_key(key_value);
  GenericLeaf g;
  memset(&g, 0, sizeof(g));
  g.d = *desc;
  g.elements_per_leaf = 1;
  g.esz = p.esz;
  hipStream_t s = (hipStream_t)stream;
  // Depth i == level i (what the validator builds for every DCF) with an
  // integer / XorWrapper value: dcf_fast_kernel.  DPF_DCF_GENERAL=1 forces
  // the general kernel (parity tests run both).
  bool identity = true;
  for (int i = 0; i < num_levels; ++i) identity = identity && level_depth[i] == i;
  const char* general = getenv("DPF_DCF_GENERAL");
  if (fast && identity && !(general && general[0] == '1')) {
    DcfFastParams f;
    memset(&f, 0, sizeof(f));
    f.num_items = items;
    f.points_per_key = points_per_key;
    f.n = num_levels;
    f.shared_points = p.shared_points;
    f.cw_stride = cw_stride;
    f.vcw_stride = p.vcw_stride;
    f.esz = p.esz;
    f.key_seed = key_seed;
    f.party = party;
    f.points = points;
    f.cw_seed = cw_seed;
    f.cw_left = cw_left;
    f.cw_right = cw_right;
    f.out = (char*)out;
    f.rkl = p.rkl;
    f.rkd = p.rkd;
    f.rkv = p.rkv;
    DcfVcw vc;
    memset(&vc, 0, sizeof(vc));
    for (int i = 0; i < num_levels; ++i) vc.level[i] = value_correction[i];
    const bool x = p.xor_mode != 0;
    switch (desc->bits[0]) {
      case 8: x ? launch_dcf_fast<8, true>(f, vc, s) : launch_dcf_fast<8, false>(f, vc, s); break;
      case 16: x ? launch_dcf_fast<16, true>(f, vc, s) : launch_dcf_fast<16, false>(f, vc, s); break;
      case 32: x ? launch_dcf_fast<32, true>(f, vc, s) : launch_dcf_fast<32, false>(f, vc, s); break;
      case 64: x ? launch_dcf_fast<64, true>(f, vc, s) : launch_dcf_fast<64, false>(f, vc, s); break;
      default: x ? launch_dcf_fast<128, true>(f, vc, s) : launch_dcf_fast<128, false>(f, vc, s); break;
    }
    HIP_TRY(hipGetLastError());
    return kOk;
  }
  const int blk = block_for(items);
  const dim3 grid(grid_for(items, blk)), block(blk);
  p.dyn_per_wg = dynamic_chunks_per_wg(items, (int)grid.x, blk, "DPF_DCF_DYNAMIC");
  if (fast) {
    switch (desc->bits[0]) {
      case 8: hipLaunchKernelGGL((dcf_eval_kernel<8, true>), grid, block, 0, s, p, lv, g); break;
      case 16: hipLaunchKernelGGL((dcf_eval_kernel<16, true>), grid, block, 0, s, p, lv, g); break;
      case 32: hipLaunchKernelGGL((dcf_eval_kernel<32, true>), grid, block, 0, s, p, lv, g); break;
      case 64: hipLaunchKernelGGL((dcf_eval_kernel<64, true>), grid, block, 0, s, p, lv, g); break;
      default: hipLaunchKernelGGL((dcf_eval_kernel<128, true>), grid, block, 0, s, p, lv, g); break;
    }
  } else {
    hipLaunchKernelGGL((dcf_eval_kernel<8, false>), grid, block, 0, s, p, lv, g);
  }
  HIP_TRY(hipGetLastError());
  return kOk;
}
