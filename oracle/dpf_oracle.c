/*
 * dpf_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's CPU evaluation path for incremental
 * DPFs, used as the parity checker for the MI355X HIP kernels.  Nothing in the
 * product (distributed_point_functions_amd/, include/) links or calls this
 * file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it (via oracle/oracle.py).
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference repository root).  The AES primitive is OpenSSL's EVP
 * AES-128-ECB -- the same EVP interface the reference drives through BoringSSL
 * (dpf/aes_128_fixed_key_hash.cc:38-40) -- and is pinned by the reference's
 * known-answer test (dpf/aes_128_fixed_key_hash_test.cc:114-135), which
 * tests/test_oracle.py re-checks.
 *
 * Conventions: a 128-bit block is the memory image of absl::uint128, i.e. two
 * little-endian uint64 words {low, high}; on x86-64 that is exactly
 * `unsigned __int128`.  Booleans are one byte each (0/1).
 */
#include <openssl/evp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

#define ORACLE_MAX_LEAVES 64
#define ORACLE_BATCH 64 /* Aes128FixedKeyHash::kBatchSize, aes_128_fixed_key_hash.h:69 */

/* ------------------------------------------------------------------------- */
/* a1: fixed-key AES-128 MMO hash  (dpf/aes_128_fixed_key_hash.cc:47-85)      */
/* ------------------------------------------------------------------------- */

typedef struct {
  EVP_CIPHER_CTX* ctx;
} oracle_prg;

static int prg_init(oracle_prg* p, const uint8_t key[16]) {
  /* aes_128_fixed_key_hash.cc:27-45 */
  p->ctx = EVP_CIPHER_CTX_new();
  if (!p->ctx) return 13;
  if (EVP_EncryptInit_ex(p->ctx, EVP_aes_128_ecb(), NULL, key, NULL) != 1) return 13;
  EVP_CIPHER_CTX_set_padding(p->ctx, 0);
  return 0;
}

static void prg_free(oracle_prg* p) {
  if (p->ctx) EVP_CIPHER_CTX_free(p->ctx);
  p->ctx = NULL;
}

static inline u128 sigma(u128 x) {
  /* sigma(x) = MakeUint128(high ^ low, high)  (aes_128_fixed_key_hash.cc:64-67) */
  uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
  return ((u128)(hi ^ lo) << 64) | (u128)hi;
}

/* out[i] = AES_k(sigma(in[i])) ^ sigma(in[i]); in/out may alias. */
static int prg_eval(const oracle_prg* p, const u128* in, u128* out, int64_t n) {
  u128 sig[ORACLE_BATCH];
  for (int64_t start = 0; start < n; start += ORACLE_BATCH) {
    int64_t bs = n - start < ORACLE_BATCH ? n - start : ORACLE_BATCH;
    for (int64_t i = 0; i < bs; ++i) sig[i] = sigma(in[start + i]);
    int out_len = 0;
    if (EVP_EncryptUpdate(p->ctx, (uint8_t*)(out + start), &out_len,
                          (const uint8_t*)sig, (int)(bs * 16)) != 1)
      return 13;
    if (out_len != (int)(bs * 16)) return 13;
    for (int64_t i = 0; i < bs; ++i) out[start + i] ^= sig[i];
  }
  return 0;
}

int oracle_aes_hash(const uint8_t key[16], int64_t n, const u128* in, u128* out) {
  oracle_prg p;
  int st = prg_init(&p, key);
  if (!st) st = prg_eval(&p, in, out, n);
  prg_free(&p);
  return st;
}

/* ------------------------------------------------------------------------- */
/* a3/a4: ExpandSeeds (dpf/distributed_point_function.cc:271-349)             */
/* ------------------------------------------------------------------------- */

/* Breadth-first expansion of n0 (seed, control) pairs through L levels.
 * Output index of node (r, path) is (r << L) | path; child 2j = left,
 * 2j+1 = right (cc:324-330).  seeds_out/ctrl_out hold n0 << L entries. */
int oracle_expand_seeds(const uint8_t key_left[16], const uint8_t key_right[16],
                        int64_t n0, const u128* seeds_in, const uint8_t* ctrl_in,
                        int L, const u128* cw_seeds, const uint8_t* cw_cl,
                        const uint8_t* cw_cr, u128* seeds_out, uint8_t* ctrl_out) {
  oracle_prg pl, pr;
  int st = prg_init(&pl, key_left);
  if (!st) st = prg_init(&pr, key_right);
  if (st) return st;
  int64_t out_n = n0 << L;
  u128* cur = (u128*)malloc(sizeof(u128) * (out_n ? out_n : 1));
  u128* nxt = (u128*)malloc(sizeof(u128) * (out_n ? out_n : 1));
  uint8_t* ccur = (uint8_t*)malloc(out_n ? out_n : 1);
  uint8_t* cnxt = (uint8_t*)malloc(out_n ? out_n : 1);
  if (!cur || !nxt || !ccur || !cnxt) { st = 8; goto done; }
  memcpy(cur, seeds_in, sizeof(u128) * n0);
  memcpy(ccur, ctrl_in, n0);
  int64_t size = n0;
  u128 bl[ORACLE_BATCH], br[ORACLE_BATCH];
  for (int i = 0; i < L; ++i) { /* cc:304-347 */
    u128 cs = cw_seeds[i];
    uint8_t cl = cw_cl[i] & 1, cr = cw_cr[i] & 1;
    for (int64_t start = 0; start < size; start += ORACLE_BATCH) {
      int64_t bs = size - start < ORACLE_BATCH ? size - start : ORACLE_BATCH;
      if ((st = prg_eval(&pl, cur + start, bl, bs))) goto done;
      if ((st = prg_eval(&pr, cur + start, br, bs))) goto done;
      for (int64_t j = 0; j < bs; ++j) { /* cc:323-343 */
        int64_t e = 2 * (start + j);
        uint8_t t = ccur[start + j] & 1;
        if (t) { bl[j] ^= cs; br[j] ^= cs; }
        uint8_t tl = (uint8_t)(bl[j] & 1), tr = (uint8_t)(br[j] & 1);
        nxt[e] = bl[j] & ~(u128)1;
        nxt[e + 1] = br[j] & ~(u128)1;
        if (t) { tl ^= cl; tr ^= cr; }
        cnxt[e] = tl;
        cnxt[e + 1] = tr;
      }
    }
    u128* ts = cur; cur = nxt; nxt = ts;
    uint8_t* tc = ccur; ccur = cnxt; cnxt = tc;
    size *= 2;
  }
  memcpy(seeds_out, cur, sizeof(u128) * size);
  memcpy(ctrl_out, ccur, size);
done:
  free(cur); free(nxt); free(ccur); free(cnxt);
  prg_free(&pl); prg_free(&pr);
  return st;
}

/* ------------------------------------------------------------------------- */
/* a9: EvaluateSeeds (dpf/internal/evaluate_prg_hwy.cc:415-491).  The scalar    */
/* fallback hashes both children and keeps one; the Highway kernel             */
/* (:205-304) hashes each seed once, with the key its path bit selects.  The   */
/* outputs are the same; this restatement does the latter (seeds grouped by    */
/* path bit, one EVP batch per key), so the oracle-based CPU baselines run the */
/* reference's one-AES-per-level work.                                         */
/* ------------------------------------------------------------------------- */

int oracle_evaluate_seeds(const uint8_t key_left[16], const uint8_t key_right[16],
                          int64_t n, int L, const u128* seeds_in,
                          const uint8_t* ctrl_in, const u128* paths,
                          const u128* cw_seeds, const uint8_t* cw_cl,
                          const uint8_t* cw_cr, u128* seeds_out, uint8_t* ctrl_out) {
  if (n == 0 || L == 0) { /* distributed_point_function.cc:238-240 */
    if (seeds_out != seeds_in) memmove(seeds_out, seeds_in, sizeof(u128) * n);
    if (ctrl_out != ctrl_in) memmove(ctrl_out, ctrl_in, n);
    return 0;
  }
  oracle_prg pl, pr;
  int st = prg_init(&pl, key_left);
  if (!st) st = prg_init(&pr, key_right);
  if (st) return st;
  u128 bl[ORACLE_BATCH], br[ORACLE_BATCH];
  int64_t il[ORACLE_BATCH], ir[ORACLE_BATCH];
  uint8_t pb[ORACLE_BATCH], cb[ORACLE_BATCH];
  for (int64_t start = 0; start < n; start += ORACLE_BATCH) {
    int64_t bs = n - start < ORACLE_BATCH ? n - start : ORACLE_BATCH;
    for (int level = 0; level < L; ++level) {
      const u128* src = (level == 0 ? seeds_in : seeds_out) + start;
      int bit_index = L - level - 1; /* evaluate_prg_hwy.cc:452 */
      int64_t nl = 0, nr = 0;
      for (int64_t i = 0; i < bs; ++i) {
        pb[i] = 0;
        if (bit_index < 128) pb[i] = (uint8_t)((paths[start + i] >> bit_index) & 1);
        if (pb[i]) { br[nr] = src[i]; ir[nr++] = i; }
        else { bl[nl] = src[i]; il[nl++] = i; }
      }
      if (nl && (st = prg_eval(&pl, bl, bl, nl))) goto done;
      if (nr && (st = prg_eval(&pr, br, br, nr))) goto done;
      for (int64_t j = 0; j < nl; ++j) seeds_out[start + il[j]] = bl[j];
      for (int64_t j = 0; j < nr; ++j) seeds_out[start + ir[j]] = br[j];
      memcpy(cb, (level == 0 ? ctrl_in : ctrl_out) + start, bs);
      for (int64_t i = 0; i < bs; ++i) { /* :470-486 */
        uint8_t t = cb[i] & 1;
        if (t) seeds_out[start + i] ^= cw_seeds[level];
        uint8_t c = (uint8_t)(seeds_out[start + i] & 1);
        seeds_out[start + i] &= ~(u128)1;
        if (t) c ^= pb[i] ? (cw_cr[level] & 1) : (cw_cl[level] & 1);
        ctrl_out[start + i] = c;
      }
    }
  }
done:
  prg_free(&pl); prg_free(&pr);
  return st;
}

/* ------------------------------------------------------------------------- */
/* Value types (dpf/internal/value_type_helpers.{h,cc}, dpf/int_mod_n.h,      */
/* dpf/tuple.h, dpf/xor_wrapper.h).  A value type is flattened into its       */
/* leaves in declaration order; tests/ prove flattening exact for nested      */
/* tuples (value_type_helpers.h:430-443: every leaf but the last updates).    */
/* ------------------------------------------------------------------------- */

enum { LEAF_INT = 0, LEAF_INTMODN = 1, LEAF_XOR = 2 };

typedef struct {
  int32_t num_leaves;
  int32_t direct; /* 1 iff no IntModN leaf: CanBeConvertedDirectly (h:342-344) */
  int32_t kind[ORACLE_MAX_LEAVES];
  int32_t bits[ORACLE_MAX_LEAVES];
  uint64_t mod_lo[ORACLE_MAX_LEAVES];
  uint64_t mod_hi[ORACLE_MAX_LEAVES];
} oracle_vtype;

static inline u128 leaf_mask(int bits) {
  return bits >= 128 ? ~(u128)0 : (((u128)1 << bits) - 1);
}
static inline u128 leaf_mod(const oracle_vtype* vt, int k) {
  return ((u128)vt->mod_hi[k] << 64) | vt->mod_lo[k];
}
static int total_bits(const oracle_vtype* vt) {
  int s = 0;
  for (int k = 0; k < vt->num_leaves; ++k) s += vt->bits[k];
  return s;
}

/* ElementsPerBlock<T>() (value_type_helpers.h:508-520) */
int oracle_elements_per_block(const oracle_vtype* vt) {
  if (!vt->direct) return 1;
  int tb = total_bits(vt);
  return tb <= 128 ? 128 / tb : 1;
}

static inline u128 load_le(const uint8_t* p, int nbytes) {
  u128 v = 0;
  for (int i = nbytes - 1; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

/* ConvertBytesToArrayOf<T> (value_type_helpers.h:569-589).  `bytes` holds
 * b*16 bytes; writes E elements * num_leaves leaves to `el`. */
static void convert_bytes(const oracle_vtype* vt, const uint8_t* bytes, u128* el) {
  int nl = vt->num_leaves;
  if (vt->direct) {
    /* DirectlyFromBytes for ints (h:199-211) and tuples (h:415-428) */
    int E = oracle_elements_per_block(vt);
    int esz = (total_bits(vt) + 7) / 8;
    for (int i = 0; i < E; ++i) {
      int off = i * esz;
      for (int k = 0; k < nl; ++k) {
        int lb = vt->bits[k] / 8;
        el[i * nl + k] = load_le(bytes + off, lb);
        off += lb;
      }
    }
    return;
  }
  /* FromBytes via SampleAndUpdateBytes (h:531-538, 213-234, 286-311, 430-443) */
  u128 block = load_le(bytes, 16);
  const uint8_t* rem = bytes + 16;
  for (int k = 0; k < nl; ++k) {
    int update = (k + 1 < nl);
    int lb = vt->bits[k] / 8;
    if (vt->kind[k] == LEAF_INTMODN) {
      u128 n = leaf_mod(vt, k);
      u128 q = block / n, r = block % n;
      el[k] = r;
      if (update) {
        block = (lb < 16) ? (q << (8 * lb)) : 0;
        block |= load_le(rem, lb);
        rem += lb;
      }
    } else {
      el[k] = block & leaf_mask(vt->bits[k]);
      if (update) {
        if (lb < 16) block &= ~leaf_mask(vt->bits[k]); else block = 0;
        block |= load_le(rem, lb);
        rem += lb;
      }
    }
  }
}

/* Group operations on one leaf (int_mod_n.h:116-245, xor_wrapper.h:40-73,
 * tuple.h:62-114; built-in unsigned ints wrap modulo 2^bits). */
static inline u128 leaf_sub_modn(u128 a, u128 b, u128 n) {
  /* SubtractBaseInteger (int_mod_n.h:208-215) */
  return a >= b ? a - b : n - b + a;
}
static inline u128 leaf_add(const oracle_vtype* vt, int k, u128 a, u128 b) {
  switch (vt->kind[k]) {
    case LEAF_XOR: return a ^ b;
    case LEAF_INTMODN: { u128 n = leaf_mod(vt, k); return leaf_sub_modn(a, n - b, n); }
    default: return (a + b) & leaf_mask(vt->bits[k]);
  }
}
static inline u128 leaf_sub(const oracle_vtype* vt, int k, u128 a, u128 b) {
  switch (vt->kind[k]) {
    case LEAF_XOR: return a ^ b;
    case LEAF_INTMODN: return leaf_sub_modn(a, b, leaf_mod(vt, k));
    default: return (a - b) & leaf_mask(vt->bits[k]);
  }
}
static inline u128 leaf_neg(const oracle_vtype* vt, int k, u128 a) {
  switch (vt->kind[k]) {
    case LEAF_XOR: return a;
    case LEAF_INTMODN: return leaf_sub_modn(0, a, leaf_mod(vt, k));
    default: return (0 - a) & leaf_mask(vt->bits[k]);
  }
}

static int packed_size(const oracle_vtype* vt) {
  int s = 0;
  for (int k = 0; k < vt->num_leaves; ++k) s += vt->bits[k] / 8;
  return s;
}
static void store_packed(const oracle_vtype* vt, const u128* leaves, uint8_t* out) {
  for (int k = 0; k < vt->num_leaves; ++k) {
    int lb = vt->bits[k] / 8;
    u128 v = leaves[k];
    for (int i = 0; i < lb; ++i) { out[i] = (uint8_t)v; v >>= 8; }
    out += lb;
  }
}

int oracle_packed_element_size(const oracle_vtype* vt) { return packed_size(vt); }

/* Raw conversion for the reference's FromBytes examples
 * (value_type_helpers_test.cc:217-240, int_mod_n_test.cc:158-186).
 * Writes E*num_leaves leaves. */
void oracle_convert_bytes(const oracle_vtype* vt, const uint8_t* bytes, u128* leaves_out) {
  convert_bytes(vt, bytes, leaves_out);
}

/* ------------------------------------------------------------------------- */
/* a5+a6+a12+a13: HashExpandedSeeds + value-correction loop                  */
/* (distributed_point_function.cc:500-524, distributed_point_function.h:785-808) */
/* ------------------------------------------------------------------------- */

/* For each of n seeds: hashed_j = H_value(seed + j), j < b; elements =
 * ConvertBytesToArrayOf; for e < cepb: +cw[e] if ctrl; negate if party 1.
 * Writes n*cepb packed elements to out. */
int oracle_hash_correct(const uint8_t key_value[16], const oracle_vtype* vt,
                        int64_t n, int b, int cepb, const u128* seeds,
                        const uint8_t* ctrl, const u128* cw_leaves, int party,
                        uint8_t* out) {
  oracle_prg pv;
  int st = prg_init(&pv, key_value);
  if (st) return st;
  int nl = vt->num_leaves, E = oracle_elements_per_block(vt), ps = packed_size(vt);
  u128* hashed = (u128*)malloc(sizeof(u128) * ((n * b) > 0 ? n * b : 1));
  u128* el = (u128*)malloc(sizeof(u128) * E * nl);
  if (!hashed || !el) { st = 8; goto done; }
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < b; ++j) hashed[i * b + j] = seeds[i] + (u128)j; /* cc:510-514 */
  if ((st = prg_eval(&pv, hashed, hashed, n * b))) goto done;
  for (int64_t i = 0; i < n; ++i) {
    convert_bytes(vt, (const uint8_t*)(hashed + i * b), el);
    for (int e = 0; e < cepb; ++e) {
      u128* x = el + e * nl;
      for (int k = 0; k < nl; ++k) {
        if (ctrl[i] & 1) x[k] = leaf_add(vt, k, x[k], cw_leaves[e * nl + k]);
        if (party == 1) x[k] = leaf_neg(vt, k, x[k]);
      }
      store_packed(vt, x, out + (i * cepb + e) * ps);
    }
  }
done:
  free(hashed); free(el);
  prg_free(&pv);
  return st;
}

/* EvaluateAtImpl's final loop (distributed_point_function.h:976-1003): the
 * element at block_index[i] of seed i's hashed block. */
int oracle_hash_select_correct(const uint8_t key_value[16], const oracle_vtype* vt,
                               int64_t n, int b, const u128* seeds,
                               const uint8_t* ctrl, const int32_t* block_index,
                               const u128* cw_leaves, int party, uint8_t* out) {
  oracle_prg pv;
  int st = prg_init(&pv, key_value);
  if (st) return st;
  int nl = vt->num_leaves, E = oracle_elements_per_block(vt), ps = packed_size(vt);
  u128* hashed = (u128*)malloc(sizeof(u128) * ((n * b) > 0 ? n * b : 1));
  u128* el = (u128*)malloc(sizeof(u128) * E * nl);
  if (!hashed || !el) { st = 8; goto done; }
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < b; ++j) hashed[i * b + j] = seeds[i] + (u128)j;
  if ((st = prg_eval(&pv, hashed, hashed, n * b))) goto done;
  for (int64_t i = 0; i < n; ++i) {
    convert_bytes(vt, (const uint8_t*)(hashed + i * b), el);
    int bi = block_index[i];
    u128* x = el + bi * nl;
    for (int k = 0; k < nl; ++k) {
      if (ctrl[i] & 1) x[k] = leaf_add(vt, k, x[k], cw_leaves[bi * nl + k]);
      if (party == 1) x[k] = leaf_neg(vt, k, x[k]);
    }
    store_packed(vt, x, out + i * ps);
  }
done:
  free(hashed); free(el);
  prg_free(&pv);
  return st;
}

/* Element-wise sum of two packed element arrays (the two-party reconstruction
 * the reference tests perform, distributed_point_function_test.cc:986-992). */
void oracle_add_packed(const oracle_vtype* vt, int64_t n, const uint8_t* a,
                       const uint8_t* b, uint8_t* out) {
  int nl = vt->num_leaves, ps = packed_size(vt);
  u128 la[ORACLE_MAX_LEAVES], lb[ORACLE_MAX_LEAVES];
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t* pa = a + i * ps;
    const uint8_t* pb = b + i * ps;
    for (int k = 0; k < nl; ++k) {
      int w = vt->bits[k] / 8;
      la[k] = load_le(pa, w); lb[k] = load_le(pb, w);
      pa += w; pb += w;
      la[k] = leaf_add(vt, k, la[k], lb[k]);
    }
    store_packed(vt, la, out + i * ps);
  }
}

/* ------------------------------------------------------------------------- */
/* a15: key generation with injected root seeds                               */
/* (distributed_point_function.cc:63-204, 619-687;                            */
/*  value_type_helpers.h:597-631 ComputeValueCorrectionFor)                   */
/* ------------------------------------------------------------------------- */

typedef struct {
  int32_t num_levels;               /* hierarchy levels H */
  int32_t tree_levels_needed;       /* proto_validator.cc:116-137 */
  int32_t last_log_domain_size;     /* parameters_.back().log_domain_size() */
  int32_t log_domain_size[130];
  int32_t hierarchy_to_tree[130];
  int32_t blocks_needed[130];       /* distributed_point_function.cc:578-587 */
} oracle_dpf_params;

/* ComputeValueCorrection (cc:63-99) for one hierarchy level.
 * seeds[2]; beta = num_leaves leaves; writes E*num_leaves leaves. */
static int value_correction(const oracle_prg* pv, const oracle_dpf_params* P,
                            const oracle_vtype* vt, int h, const u128 seeds[2],
                            u128 alpha_prefix, const u128* beta, int invert,
                            u128* vc_out) {
  int b = P->blocks_needed[h];
  int nl = vt->num_leaves, E = oracle_elements_per_block(vt);
  u128 buf[2 * 16];
  if (b > 16) return 3;
  for (int j = 0; j < b; ++j) { buf[j] = seeds[0] + (u128)j; buf[b + j] = seeds[1] + (u128)j; }
  int st = prg_eval(pv, buf, buf, 2 * b);
  if (st) return st;
  /* DomainToBlockIndex (cc:214-221) */
  int bits = P->log_domain_size[h] - P->hierarchy_to_tree[h];
  int index = (int)(alpha_prefix & (((u128)1 << bits) - 1));
  u128 ints_a[ORACLE_MAX_LEAVES * 128 / 8], ints_b[ORACLE_MAX_LEAVES * 128 / 8];
  convert_bytes(vt, (const uint8_t*)buf, ints_a);
  convert_bytes(vt, (const uint8_t*)(buf + b), ints_b);
  for (int k = 0; k < nl; ++k)
    ints_b[index * nl + k] = leaf_add(vt, k, ints_b[index * nl + k], beta[k]);
  for (int i = 0; i < E; ++i)
    for (int k = 0; k < nl; ++k) {
      u128 v = leaf_sub(vt, k, ints_b[i * nl + k], ints_a[i * nl + k]);
      if (invert) v = leaf_neg(vt, k, v);
      vc_out[i * nl + k] = v;
    }
  return 0;
}

/* GenerateKeysIncremental with the two root seeds supplied by the caller
 * instead of RAND_bytes (cc:656-662).  betas: concatenated leaves per level.
 * vc_out: concatenated E_h*num_leaves_h leaves per level (value correction of
 * level h; the last level's is last_level_value_correction). */
int oracle_generate_keys(const uint8_t key_left[16], const uint8_t key_right[16],
                         const uint8_t key_value[16], const oracle_dpf_params* P,
                         const oracle_vtype* vtypes, uint64_t alpha_lo, uint64_t alpha_hi,
                         const u128* betas, uint64_t seed0_lo, uint64_t seed0_hi,
                         uint64_t seed1_lo, uint64_t seed1_hi, u128* cw_seeds,
                         uint8_t* cw_cl, uint8_t* cw_cr, u128* vc_out) {
  u128 alpha = ((u128)alpha_hi << 64) | alpha_lo;
  u128 seed0 = ((u128)seed0_hi << 64) | seed0_lo;
  u128 seed1 = ((u128)seed1_hi << 64) | seed1_lo;
  oracle_prg pl, pr, pv;
  int st = prg_init(&pl, key_left);
  if (!st) st = prg_init(&pr, key_right);
  if (!st) st = prg_init(&pv, key_value);
  if (st) return st;
  int H = P->num_levels;
  int beta_off[131], vc_off[131];
  beta_off[0] = vc_off[0] = 0;
  for (int h = 0; h < H; ++h) {
    beta_off[h + 1] = beta_off[h] + vtypes[h].num_leaves;
    vc_off[h + 1] = vc_off[h] + oracle_elements_per_block(&vtypes[h]) * vtypes[h].num_leaves;
  }
  u128 seeds[2] = {seed0, seed1};
  uint8_t ctrl[2] = {0, 1}; /* cc:665 */
  int last_log = P->last_log_domain_size;
  for (int tl = 1; tl < P->tree_levels_needed; ++tl) { /* cc:670-674, GenerateNext cc:103-204 */
    int h = -1;
    for (int i = 0; i < H; ++i) if (P->hierarchy_to_tree[i] == tl - 1) h = i;
    if (h >= 0) {
      u128 prefix = 0;
      int shift = last_log - P->log_domain_size[h];
      if (shift < 128) prefix = alpha >> shift;
      st = value_correction(&pv, P, &vtypes[h], h, seeds, prefix, betas + beta_off[h],
                            ctrl[1], vc_out + vc_off[h]);
      if (st) goto done;
    }
    u128 ex[2][2];
    if ((st = prg_eval(&pl, seeds, ex[0], 2))) goto done;
    if ((st = prg_eval(&pr, seeds, ex[1], 2))) goto done;
    uint8_t ec[2][2];
    for (int br = 0; br < 2; ++br)
      for (int p = 0; p < 2; ++p) { ec[br][p] = (uint8_t)(ex[br][p] & 1); ex[br][p] &= ~(u128)1; }
    uint8_t bit = 0;
    if (last_log - tl < 128) bit = (uint8_t)((alpha >> (last_log - tl)) & 1);
    int keep = bit, lose = !bit;
    u128 sc = ex[lose][0] ^ ex[lose][1];
    uint8_t cc[2];
    cc[0] = ec[0][0] ^ ec[0][1] ^ bit ^ 1;
    cc[1] = ec[1][0] ^ ec[1][1] ^ bit;
    for (int p = 0; p < 2; ++p) {
      u128 ns = ex[keep][p];
      if (ctrl[p]) ns ^= sc;
      uint8_t nc = ec[keep][p] ^ (ctrl[p] & cc[keep]);
      seeds[p] = ns;
      ctrl[p] = nc;
    }
    cw_seeds[tl - 1] = sc;
    cw_cl[tl - 1] = cc[0];
    cw_cr[tl - 1] = cc[1];
  }
  /* last level value correction (cc:676-684) */
  st = value_correction(&pv, P, &vtypes[H - 1], H - 1, seeds, alpha, betas + beta_off[H - 1],
                        ctrl[1], vc_out + vc_off[H - 1]);
done:
  prg_free(&pl); prg_free(&pr); prg_free(&pv);
  return st;
}
