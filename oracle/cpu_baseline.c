/*
 * cpu_baseline.c -- TEST / BENCH INFRASTRUCTURE ONLY (like dpf_oracle.c):
 * bench.py's cpu_baseline leg for batched EvaluateAt and
 * a checker in tests/.  Never linked or called by the product path.
 *
 * The reference's CPU path for EvaluateAt, restated with AES-NI intrinsics:
 * EvaluateAtImpl (dpf/distributed_point_function.h:839-1010) walks every
 * evaluation point down its tree path with ONE fixed-key AES per level -- the
 * Highway EvaluateSeeds kernel (dpf/internal/evaluate_prg_hwy.cc:205-304)
 * hashes each seed with the key its path bit selects -- then hashes the leaf
 * seed with the value key (HashExpandedSeeds, cc:500-524), selects the
 * element of the block, corrects it and negates it for party 1
 * (h:993-1002).  dpf_oracle.c's oracle_evaluate_seeds restates the scalar
 * fallback instead (both children hashed per level, evaluate_prg_hwy.cc:
 * 446-449); the outputs are identical (tests/test_oracle.py checks this file
 * against the oracle).
 *
 * H_k(x) = AES_k(sigma(x)) ^ sigma(x), sigma(x) = MakeUint128(hi ^ lo, hi)
 * (dpf/aes_128_fixed_key_hash.cc:47-85).  Eight points are walked interleaved
 * so the AES unit's pipeline stays full (AESENC latency ~4 cycles); each
 * point's round keys are the schedule its path bit picks.
 */
#include <smmintrin.h>
#include <stdint.h>
#include <string.h>
#include <wmmintrin.h>

typedef unsigned __int128 u128;

static __m128i expand_step(__m128i k, __m128i g) {
  g = _mm_shuffle_epi32(g, 0xff);
  k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
  k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
  k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
  return _mm_xor_si128(k, g);
}

/* AES-128 key schedule (FIPS-197 5.2) of the 16-byte key memory image. */
static void key_schedule(const uint8_t key[16], __m128i rk[11]) {
  rk[0] = _mm_loadu_si128((const __m128i*)key);
#define KS(i, rc) rk[i] = expand_step(rk[i - 1], _mm_aeskeygenassist_si128(rk[i - 1], rc))
  KS(1, 0x01); KS(2, 0x02); KS(3, 0x04); KS(4, 0x08); KS(5, 0x10);
  KS(6, 0x20); KS(7, 0x40); KS(8, 0x80); KS(9, 0x1b); KS(10, 0x36);
#undef KS
}

/* sigma on the {low64, high64} lanes: (lo, hi) -> (hi, hi ^ lo). */
static inline __m128i sigma(__m128i x) {
  return _mm_xor_si128(_mm_unpackhi_epi64(x, x), _mm_slli_si128(x, 8));
}

#define NB 8

/* H_{k_i}(x_i) for NB blocks, each with its own schedule k[i]. */
static inline void mmo8(__m128i* x, const __m128i* const* k) {
  __m128i s[NB], e[NB];
  for (int i = 0; i < NB; ++i) {
    s[i] = sigma(x[i]);
    e[i] = _mm_xor_si128(s[i], k[i][0]);
  }
  for (int r = 1; r < 10; ++r)
    for (int i = 0; i < NB; ++i) e[i] = _mm_aesenc_si128(e[i], k[i][r]);
  for (int i = 0; i < NB; ++i) x[i] = _mm_xor_si128(_mm_aesenclast_si128(e[i], k[i][10]), s[i]);
}

/*
 * Batched EvaluateAt of uint64 values (ElementsPerBlock = 2, one hashed block
 * per leaf): key k < num_keys has root seed key_seed[k], party[k], correction
 * words cw_seed/cw_left/cw_right[k * cw_stride + j] (j < L tree levels) and
 * value corrections vcw[k * 2 + e] (the low 64 bits count).  Point j of key k
 * is points[k * ppk + j]: tree path = point >> bib, element = point & (2^bib-1).
 * out[k * ppk + j] = the party's uint64 share.  Returns 0.
 */
int baseline_evaluate_at_u64(const uint8_t key_left[16], const uint8_t key_right[16],
                             const uint8_t key_value[16], int64_t num_keys, int64_t ppk, int L,
                             int bib, const u128* key_seed, const uint8_t* party,
                             const u128* cw_seed, const uint8_t* cw_left, const uint8_t* cw_right,
                             int64_t cw_stride, const u128* vcw, const u128* points,
                             uint64_t* out) {
  __m128i sched[3][11];
  key_schedule(key_left, sched[0]);
  key_schedule(key_right, sched[1]);
  key_schedule(key_value, sched[2]);
  const __m128i* kv[NB];
  for (int i = 0; i < NB; ++i) kv[i] = sched[2];
  for (int64_t k = 0; k < num_keys; ++k) {
    const u128* cws = cw_seed + k * cw_stride;
    const uint8_t* cl = cw_left + k * cw_stride;
    const uint8_t* cr = cw_right + k * cw_stride;
    const uint8_t pk = party[k] & 1;
    const uint64_t vc[2] = {(uint64_t)vcw[2 * k], (uint64_t)vcw[2 * k + 1]};
    for (int64_t j0 = 0; j0 < ppk; j0 += NB) {
      const int nb = ppk - j0 < NB ? (int)(ppk - j0) : NB;
      __m128i s[NB];
      uint8_t t[NB];
      u128 path[NB];
      int el[NB];
      for (int i = 0; i < NB; ++i) {
        const u128 x = points[k * ppk + j0 + (i < nb ? i : 0)];
        path[i] = x >> bib;
        el[i] = (int)(x & (((u128)1 << bib) - 1));
        s[i] = _mm_loadu_si128((const __m128i*)&key_seed[k]);
        t[i] = pk;
      }
      for (int lvl = 0; lvl < L; ++lvl) {
        const int bit_index = L - 1 - lvl;  /* evaluate_prg_hwy.cc:452 */
        const __m128i* ks[NB];
        uint8_t bit[NB];
        for (int i = 0; i < NB; ++i) {
          bit[i] = (uint8_t)((path[i] >> bit_index) & 1);
          ks[i] = sched[bit[i]];
        }
        mmo8(s, ks);
        const __m128i cw = _mm_loadu_si128((const __m128i*)&cws[lvl]);
        for (int i = 0; i < NB; ++i) {  /* :470-486 */
          if (t[i]) s[i] = _mm_xor_si128(s[i], cw);
          const uint8_t c = (uint8_t)(_mm_cvtsi128_si32(s[i]) & 1);
          s[i] = _mm_andnot_si128(_mm_cvtsi32_si128(1), s[i]);
          t[i] = t[i] ? (uint8_t)(c ^ ((bit[i] ? cr[lvl] : cl[lvl]) & 1)) : c;
        }
      }
      mmo8(s, kv);
      for (int i = 0; i < nb; ++i) {
        uint64_t w[2];
        _mm_storeu_si128((__m128i*)w, s[i]);
        uint64_t v = w[el[i] & 1];
        if (t[i]) v += vc[el[i] & 1];
        if (pk) v = (uint64_t)0 - v;
        out[k * ppk + j0 + i] = v;
      }
    }
  }
  return 0;
}
