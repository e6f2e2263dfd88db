/*
 * dpf_hip.h -- C ABI of the MI355X (gfx950) DPF evaluation engine.
 *
 * This is the drop-in seam between a host DistributedPointFunction and the
 * HIP kernels.  It replaces the reference's CPU hot loops:
 *
 *   dpf_hip_hash        <- Aes128FixedKeyHash::Evaluate
 *                          (dpf/aes_128_fixed_key_hash.h:51-52, .cc:47-85)
 *   dpf_hip_eval_paths  <- dpf_internal::EvaluateSeeds
 *                          (dpf/internal/evaluate_prg_hwy.h:58-64, .cc:495-506)
 *   dpf_hip_expand      <- DistributedPointFunction::ExpandSeeds + HashExpandedSeeds
 *                          + the EvaluateUntil value-correction loop, fused
 *                          (dpf/distributed_point_function.cc:271-349, 500-524;
 *                           dpf/distributed_point_function.h:785-808)
 *   dpf_hip_eval_points <- EvaluateAtImpl's EvaluateSeeds + HashExpandedSeeds +
 *                          per-point correction, fused, for one or many keys
 *                          (dpf/distributed_point_function.h:839-1010)
 *
 * Conventions
 *   - Every function returns an int status: 0 = OK, otherwise the absl status
 *     code number (3 INVALID_ARGUMENT, 8 RESOURCE_EXHAUSTED, 12 UNIMPLEMENTED,
 *     13 INTERNAL).  dpf_hip_last_error() returns a message for the last failure
 *     on the calling thread.
 *   - All array pointers passed to compute entry points are DEVICE pointers,
 *     caller-owned.  Allocation only crosses the ABI through dpf_hip_alloc /
 *     dpf_hip_free; copies through dpf_hip_memcpy_*.
 *   - A 128-bit block (dpf_block) is the absl::uint128 memory image:
 *     {low, high}, little-endian.  Booleans are one byte (0/1).
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  Compute
 *     entry points are asynchronous on that stream (no host synchronisation);
 *     dpf_hip_stream_sync() waits.
 *   - Not thread-safe per stream (the reference is single-threaded too,
 *     dpf/aes_128_fixed_key_hash.h:77).
 */
#ifndef DPF_HIP_H_
#define DPF_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPF_HIP_ABI_VERSION 1
#define DPF_MAX_LEAVES 16

typedef struct dpf_block {
  uint64_t low;
  uint64_t high;
} dpf_block;

/* One fixed AES-128 key: the 16-byte memory image of the uint128 key
 * (aes_128_fixed_key_hash.cc:38-40). */
typedef struct dpf_aes_key {
  uint8_t bytes[16];
} dpf_aes_key;

/* Leaf kinds of a flattened ValueType (distributed_point_function.proto:25-60). */
enum dpf_leaf_kind { DPF_LEAF_INT = 0, DPF_LEAF_INTMODN = 1, DPF_LEAF_XOR = 2 };

/* A ValueType flattened into its integer leaves in declaration order, plus the
 * per-hierarchy-level sampling parameters the host computed:
 *   direct            CanBeConvertedDirectly (value_type_helpers.h:342-344)
 *   elements_per_block ElementsPerBlock<T>() (value_type_helpers.h:508-520)
 *   blocks_needed     ceil(BitsNeeded / 128) (distributed_point_function.cc:578-587) */
typedef struct dpf_value_desc {
  int32_t num_leaves;
  int32_t direct;
  int32_t elements_per_block;
  int32_t blocks_needed;
  int32_t kind[DPF_MAX_LEAVES];
  int32_t bits[DPF_MAX_LEAVES];
  uint64_t mod_low[DPF_MAX_LEAVES];
  uint64_t mod_high[DPF_MAX_LEAVES];
} dpf_value_desc;

/* ---- runtime / memory ---------------------------------------------------- */
int dpf_hip_abi_version(void);
const char* dpf_hip_last_error(void);
int dpf_hip_device_count(int* count);
int dpf_hip_set_device(int device);
int dpf_hip_alloc(void** ptr, size_t bytes);
int dpf_hip_free(void* ptr);
/* Free and total device memory of the current device (hipMemGetInfo). */
int dpf_hip_mem_info(size_t* free_bytes, size_t* total_bytes);
int dpf_hip_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
/* Page-locked host memory, and an H2D copy that does not wait: `src` must be
 * page-locked (dpf_hip_host_alloc) and stay unchanged until `stream` has run
 * the copy.  The host API stages its small per-call uploads this way. */
int dpf_hip_host_alloc(void** ptr, size_t bytes);
int dpf_hip_host_free(void* ptr);
int dpf_hip_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream);
int dpf_hip_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
/* D2H copy into FRESH host storage that the caller initialises chunk by chunk
 * (e.g. a std::vector<T> being value-initialised by resize): before each
 * chunk's DMA, `before_chunk(ctx, bytes_ready)` is called and must make
 * [0, bytes_ready) of `dst` valid; the DMA of one chunk overlaps the
 * initialisation of the next.  Large copies DMA straight into `dst`
 * (registered for the copy; a fresh pageable range is mapped and registered
 * piece by piece on a helper thread while the DMA fills the pieces already
 * registered), others go through page-locked staging.  The drop-in
 * EvaluateUntil<T> returns its std::vector<T> this way. */
/* FRESH host ranges (pages not yet mapped) of at least this many bytes are
 * registered (page-locked) for a copy and DMAed straight into; smaller ones go
 * through page-locked staging.  Ranges whose pages are already mapped (every
 * dpf_hip_memcpy_h2d source; dpf_hip_memcpy_d2h destinations the caller has
 * touched) are registered from 32 MiB. */
#define DPF_HIP_REGISTER_MIN_BYTES ((size_t)512 << 20)

/* D2H copy handed to the host chunk by chunk: the bytes arrive in the
 * library's page-locked staging buffers, and `consume(ctx, chunk, offset,
 * len)` gets [offset, offset + len) of the source (len a multiple of `align`,
 * <= 16 MiB) while the next chunk's DMA runs.  Returns after the last
 * consume.  The drop-in EvaluateUntil<T> unpacks packed tuples / IntModN
 * values straight into its result vector this way (no host copy of the packed
 * bytes), and mid-sized integer outputs are copied into theirs. */
int dpf_hip_memcpy_d2h_chunked(const void* src, size_t bytes, size_t align,
                               void (*consume)(void* ctx, const void* chunk, size_t offset,
                                               size_t len),
                               void* ctx, void* stream);
int dpf_hip_memcpy_d2h_staged(void* dst, const void* src, size_t bytes,
                              void (*before_chunk)(void* ctx, size_t bytes_ready), void* ctx,
                              void* stream);
/* _staged for a source produced in parts on `stream`: [0, part_end_bytes[j])
 * of `src` is complete once part_events[j] (dpf_hip_event_record on `stream`)
 * has completed (ends non-decreasing, the last >= bytes).  A fresh pageable
 * `dst` of >= DPF_HIP_REGISTER_MIN_BYTES is copied on a stream of the call's
 * own, each DMA chunk waiting on the device for the first part that covers
 * it, so the copy of part j overlaps the kernels producing the later parts;
 * every other destination is copied on `stream` after all parts.  The
 * drop-in EvaluateUntil<T> returns a >= 512 MiB first-call output this way,
 * its expansion launched as 8 subtrees. */
int dpf_hip_memcpy_d2h_staged_after(void* dst, const void* src, size_t bytes,
                                    void (*before_chunk)(void* ctx, size_t bytes_ready), void* ctx,
                                    int num_parts, void* const* part_events,
                                    const size_t* part_end_bytes, void* stream);
int dpf_hip_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);
int dpf_hip_memset(void* dst, int value, size_t bytes, void* stream);
int dpf_hip_stream_sync(void* stream);
/* Waits for an event (dpf_hip_event_create/record, declared with the timing
 * helpers below).  The host API marks the end of the work that reads its
 * staging buffers with one, so reusing them never depends on the caller's
 * stream still existing. */
int dpf_hip_event_sync(void* event);
/* Makes later work on `stream` wait for `event` on the device (no host wait). */
int dpf_hip_stream_wait_event(void* stream, void* event);
/* Packed size in bytes of one output element: sum of leaf bits / 8. */
int dpf_hip_packed_element_size(const dpf_value_desc* desc);

/* ---- a1: out[i] = AES_key(sigma(in[i])) ^ sigma(in[i]) --------------------
 * Replaces Aes128FixedKeyHash::Evaluate (aes_128_fixed_key_hash.cc:47-85).
 * in/out may alias. */
int dpf_hip_hash(int64_t n, const dpf_block* in, const dpf_aes_key* key,
                 dpf_block* out, void* stream);

/* ---- a9: path evaluation --------------------------------------------------
 * Replaces dpf_internal::EvaluateSeeds (evaluate_prg_hwy.h:58-64).  For each
 * seed i and level j < num_levels: bit = (paths[i] >> (num_levels-1-j)) & 1,
 * s = H_{bit ? right : left}(s); if t: s ^= cw_seed[j]; t' = s & 1; s &= ~1;
 * if t: t' ^= bit ? cw_right[j] : cw_left[j].  Outputs may alias inputs.
 * With num_levels == 0 the inputs are copied to the outputs. */
int dpf_hip_eval_paths(int64_t num_seeds, int num_levels, const dpf_block* seeds_in,
                       const uint8_t* control_in, const dpf_block* paths,
                       const dpf_block* cw_seed, const uint8_t* cw_left,
                       const uint8_t* cw_right, const dpf_aes_key* key_left,
                       const dpf_aes_key* key_right, dpf_block* seeds_out,
                       uint8_t* control_out, void* stream);

/* ---- a4+a5+a6+a12+a13: fused subtree expansion + leaf hashing/correction ---
 * Replaces ExpandSeeds (cc:271-349) + HashExpandedSeeds (cc:500-524) + the
 * EvaluateUntil correction loop (h:785-808).  Expands each of num_starts
 * (seed, control) pairs through num_levels levels (child 2j = left, 2j+1 =
 * right), hashes every leaf seed with key_value into desc->blocks_needed blocks
 * (seed + j), converts them to desc->elements_per_block elements, keeps the
 * first `elements_per_leaf` (= corrected_elements_per_block), adds
 * value_correction (elements_per_block * num_leaves dpf_blocks, one per leaf
 * value) when the leaf's control bit is set and negates when party == 1.
 * Writes (num_starts << num_levels) * elements_per_leaf packed elements to
 * `out` in expansion order. */
int dpf_hip_expand(int64_t num_starts, const dpf_block* seeds_in, const uint8_t* control_in,
                   int num_levels, const dpf_block* cw_seed, const uint8_t* cw_left,
                   const uint8_t* cw_right, const dpf_aes_key* key_left,
                   const dpf_aes_key* key_right, const dpf_aes_key* key_value,
                   const dpf_value_desc* desc, int elements_per_leaf,
                   const dpf_block* value_correction, int party, void* out, void* stream);

/* Diagnostic: which kernel the calling thread's last successful dpf_hip_expand
 * launched ("octet/<leaf>" or "pair/<leaf>", leaf = fast, swar, mod32,
 * generic; "" before the first call), and the depth-first subtree depth it
 * chose.  Tests use it to pin the dispatch. */
const char* dpf_hip_last_expand_kernel(int* subtree_depth);

/* Diagnostic (bench.py): the sustained shader clock of the expand launches
 * themselves.  dpf_hip_clock_probe(1) allocates and zeroes a device
 * accumulator on the current device; from then on wave 0 of every
 * workgroup of every octet expand launch (the full-domain kernel) adds its
 * s_memtime (shader clocks) and s_memrealtime (100 MHz) deltas around its
 * work into it -- two stamps per workgroup, nothing on the outputs' path.
 * dpf_hip_clock_probe_read waits for the device, returns the clock in GHz
 * (sum of shader-clock deltas / sum of real-time deltas), the number of
 * stamped workgroups and their mean duration in seconds, and zeroes the
 * accumulator.  dpf_hip_clock_probe(0) turns it off.  No reference
 * counterpart (SURVEY.md 8d asks for the sustained clock). */
int dpf_hip_clock_probe(int on);
int dpf_hip_clock_probe_read(double* clock_ghz, int64_t* workgroups, double* mean_workgroup_s);

/* Diagnostic: which kernel the calling thread's last
 * dpf_hip_eval_prefix_batch(_cached) launched: "hh_level" (the lean
 * heavy-hitters kernel: cached or gathered start seeds, two expanded levels,
 * IntModN<uint32_t> sums), "batch_level/fast", "batch_level/mod32" or
 * "batch_level/generic"; "" before the first call. */
const char* dpf_hip_last_batch_kernel(void);

/* Diagnostic: which point kernel the calling thread's last point evaluation
 * (dpf_hip_eval_points*, per key or summed) launched: "points/ilp4" (integer
 * leaves, four path chains per lane), "points/ilp2" (two) or "points/single"
 * (one, for launches below one wave per CU); "" before the first call. */
const char* dpf_hip_last_points_kernel(void);

/* ---- a11: fused point evaluation for many keys ----------------------------
 * Replaces EvaluateAtImpl's path walk + hash + correction (h:930-1003).
 * Point i belongs to key k = i / points_per_key.  Its walk starts at
 * (seeds_in[i], control_in[i]) if seeds_in != NULL, else at the key's root
 * (key_seed[k], party[k]).  The path is tree_index[i] over num_levels levels
 * using key k's correction words cw_seed[k*num_levels + j], cw_left[...],
 * cw_right[...].  The element block_index[i] (NULL = 0) of the hashed leaf is
 * corrected with value_correction[k * E*num_leaves ...] and negated if
 * party[k] == 1, then written packed to out[i]. */
int dpf_hip_eval_points(int64_t num_points, int64_t points_per_key, int num_levels,
                        const dpf_block* key_seed, const uint8_t* party,
                        const dpf_block* seeds_in, const uint8_t* control_in,
                        const dpf_block* tree_index, const int32_t* block_index,
                        const dpf_block* cw_seed, const uint8_t* cw_left,
                        const uint8_t* cw_right, const dpf_aes_key* key_left,
                        const dpf_aes_key* key_right, const dpf_aes_key* key_value,
                        const dpf_value_desc* desc, const dpf_block* value_correction,
                        void* out, void* stream);

/* ---- a11 + SURVEY 8e: batched point evaluation over a key batch ------------
 * Config 4 (2^20 keys x 2^10 points).  Key k < num_keys is the SoA row k of a
 * key batch: root key_seed[k], party[k], correction words cw_seed[k*cw_stride
 * + j], cw_left[...], cw_right[...] (j < num_levels = the hierarchy level's
 * tree depth <= cw_stride, the key's correction-word count) and value
 * corrections value_correction[k*E*num_leaves ...].
 * `points` are raw domain points (dpf_block = uint128): the tree path is
 * point >> block_index_bits and the element index point & (2^bits - 1)
 * (distributed_point_function.cc:206-221).  Point j of key k is
 * points[shared_points ? j : k*points_per_key + j]; the output element
 * k*points_per_key + j (packed) equals EvaluateAt(key_k, {point}).
 * When points_per_key is even and (points_per_key / 2) % 64 == 0 every
 * wavefront works on one key (scalar correction-word loads). */
int dpf_hip_eval_points_batch(int64_t num_keys, int64_t points_per_key, int shared_points,
                              int num_levels, int cw_stride, int block_index_bits,
                              const dpf_block* key_seed,
                              const uint8_t* party, const dpf_block* points,
                              const dpf_block* cw_seed, const uint8_t* cw_left,
                              const uint8_t* cw_right, const dpf_aes_key* key_left,
                              const dpf_aes_key* key_right, const dpf_aes_key* key_value,
                              const dpf_value_desc* desc, const dpf_block* value_correction,
                              void* out, void* stream);

/* Aggregation variant: every key is evaluated at the SAME num_points points
 * and   out[j] = sum over k < num_keys of EvaluateAt(key_k, points[j])
 * is written packed, the sum taken in the value type's group (integers mod
 * 2^bits, IntModN mod N, XorWrapper by XOR; tuples element-wise).
 * `workspace` (device) holds num_points * desc->num_leaves * 3 uint64 (192-bit
 * exact per-leaf sums) and is cleared by the call. */
int dpf_hip_eval_points_sum(int64_t num_keys, int64_t num_points, int num_levels, int cw_stride,
                            int block_index_bits, const dpf_block* key_seed, const uint8_t* party,
                            const dpf_block* points, const dpf_block* cw_seed,
                            const uint8_t* cw_left, const uint8_t* cw_right,
                            const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                            const dpf_aes_key* key_value, const dpf_value_desc* desc,
                            const dpf_block* value_correction, uint64_t* workspace, void* out,
                            void* stream);

/* Number of points[i] >= 2^log_domain_size (the EvaluateAt range check,
 * distributed_point_function.h:861-874, for device-resident points).
 * Synchronous: *count is a host int64. */
int dpf_hip_count_out_of_range(int64_t n, const dpf_block* points, int log_domain_size,
                               int64_t* count, void* stream);

/* ---- gather for EvaluateUntil with prefixes (h:822-835) -------------------
 * out[i*count + j] = in[src_offset[i] + j], elements of elem_size bytes. */
int dpf_hip_gather(int64_t num_rows, int64_t count, int elem_size, const int64_t* src_offset,
                   const void* in, void* out, void* stream);

/* ---- multi-key share aggregation ------------------------------
 * sums[j] = sum over k < num_keys of shares[k*row_len + j] for plain integer
 * leaves of `bits` (8..64) widened to uint64 (mod 2^64), or XOR for xor != 0. */
int dpf_hip_sum_shares_u64(int64_t num_keys, int64_t row_len, int bits, int xor_mode,
                           const void* shares, uint64_t* sums, void* stream);

/* ---- a7+a8+a9+a4+a5+a6 over a key batch at shared prefixes ----------------
 * One EvaluateUntil step (distributed_point_function.h:641-837) of every key
 * of a batch with a device-resident context: the
 * path walk of ComputePartialEvaluations (cc:351-453, EvaluateSeeds
 * evaluate_prg_hwy.cc:452-486), ExpandSeeds (cc:271-349), HashExpandedSeeds
 * (cc:500-524) and the value correction (h:785-808), fused.
 *
 * For key k < num_keys and start node u < num_starts:
 *   start  = (seeds_in[k*in_stride + parent[u]], control_in[...]), or key k's
 *            root (key_seed[k], party[k]) when seeds_in == NULL; with
 *            control_in == NULL the control bit is bit 0 of the seed (the
 *            expansion cache layout below) and is cleared before use;
 *   walk   walk_levels levels along path[u] (bit walk_levels-1-j at step j)
 *          with key k's correction words cw_first + j (rows of cw_stride);
 *          after save_after steps (-1 = never) the node is stored at
 *          seeds_out/control_out[k*out_stride + save_index[u]] when
 *          save_index[u] >= 0 (save_index == NULL: at index u);
 *   expand expand_levels (<= dpf_hip_prefix_batch_max_expand) full levels
 *          below it (correction words cw_first + walk_levels + d), hash
 *          every leaf, convert it and keep its first elements_per_leaf
 *          corrected elements (value_correction[k*E*num_leaves ...], party
 *          negation).
 * Slot (u << expand_levels) + leaf, element e is output element
 * ((u << expand_levels) + leaf) * elements_per_leaf + e.
 * sum == 0: out[k][slot] packed, one row of num_starts << expand_levels
 *           elements per key (== EvaluateUntil's block for that node).
 * sum != 0: out[slot] = group sum over keys (integers mod 2^bits, IntModN mod
 *           N, XorWrapper by XOR); workspace holds slots * num_leaves * 3
 *           uint64 and is cleared by the call.  Returns 12 UNIMPLEMENTED for
 *           value types without an on-device key sum
 *           (dpf_hip_prefix_batch_max_expand(desc, 1) < 0): use sum == 0 and
 *           dpf_hip_sum_rows. */
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
                              uint64_t* workspace, void* out, void* stream);

/* dpf_hip_eval_prefix_batch that also writes the expansion cache: every tree
 * leaf of the call (2^expand_levels per start node u) to
 * leaf_cache[k*leaf_stride + (u << expand_levels) + l] (leaf_stride >=
 * num_starts << expand_levels), the node's seed with its control bit in bit 0
 * (clear in every non-root seed).  The next level's tree nodes are among these
 * leaves, so the next call reads its start seeds straight from them
 * (seeds_in = the cache, control_in = NULL, parent[u] = the node's cache slot)
 * instead of re-deriving them by a path walk from the partial evaluations two
 * calls back (distributed_point_function.cc:351-453).
 * The leaves must not be the root (depth > 0).  leaf_cache must not overlap
 * seeds_in (the caller double-buffers).  leaf_cache == NULL: no cache. */
int dpf_hip_eval_prefix_batch_cached(
    int64_t num_keys, int64_t num_starts, int walk_levels, int save_after, int expand_levels,
    int cw_first, int cw_stride, const dpf_block* key_seed, const uint8_t* party,
    const dpf_block* seeds_in, const uint8_t* control_in, int64_t in_stride,
    const int32_t* parent, const dpf_block* path, const int32_t* save_index, dpf_block* seeds_out,
    uint8_t* control_out, int64_t out_stride, const dpf_block* cw_seed, const uint8_t* cw_left,
    const uint8_t* cw_right, const dpf_aes_key* key_left, const dpf_aes_key* key_right,
    const dpf_aes_key* key_value, const dpf_value_desc* desc, int elements_per_leaf,
    const dpf_block* value_correction, int sum, uint64_t* workspace, void* out,
    dpf_block* leaf_cache, int64_t leaf_stride, void* stream);

/* dpf_hip_eval_prefix_batch_cached with the cache rewritten IN PLACE:
 * leaf l of start node u goes to leaf_cache[k*leaf_stride + leaf_slot[(u <<
 * expand_levels) + l]] (leaf_slot: device, num_starts << expand_levels
 * entries), and leaf_cache may be seeds_in itself (in_stride == leaf_stride,
 * control_in == NULL).  Contract on the table: a slot that
 * some start node reads (parent[u]) may appear only among the leaves of that
 * start node, and only if no other start node reads it; every other entry is
 * a slot no start node reads.  Each (key, start node) is one thread that
 * reads its start seed before it writes any leaf, so no entry is overwritten
 * before it has been read -- no gather of the start seeds and no second
 * cache buffer (the heavy-hitters steady state at 2^20
 * clients, where a 64 GiB spare does not fit).  leaf_slot == NULL: exactly
 * dpf_hip_eval_prefix_batch_cached.  DPF_HIP_CHECK_SLOTS=1 checks the table
 * against this contract on the host first (INVALID_ARGUMENT if broken). */
int dpf_hip_eval_prefix_batch_cached_slots(
    int64_t num_keys, int64_t num_starts, int walk_levels, int save_after, int expand_levels,
    int cw_first, int cw_stride, const dpf_block* key_seed, const uint8_t* party,
    const dpf_block* seeds_in, const uint8_t* control_in, int64_t in_stride,
    const int32_t* parent, const dpf_block* path, const int32_t* save_index, dpf_block* seeds_out,
    uint8_t* control_out, int64_t out_stride, const dpf_block* cw_seed, const uint8_t* cw_left,
    const uint8_t* cw_right, const dpf_aes_key* key_left, const dpf_aes_key* key_right,
    const dpf_aes_key* key_value, const dpf_value_desc* desc, int elements_per_leaf,
    const dpf_block* value_correction, int sum, uint64_t* workspace, void* out,
    dpf_block* leaf_cache, int64_t leaf_stride, const int32_t* leaf_slot, void* stream);

/* dpf_hip_eval_prefix_batch_cached_slots with the layout of its per-key
 * tables chosen.  index_major == 0 is exactly that function: element (key k,
 * slot j) of seeds_in / control_in, seeds_out / control_out and leaf_cache at
 * k*stride + j.  index_major == 1 puts it at j*num_keys + k for all three
 * (in_stride, out_stride and leaf_stride then only give the slots per key):
 * the layout of the device batch context (DeviceBatchContext), in which 64
 * consecutive keys at one slot are one 1 KiB access.  With index_major == 1
 * the heavy-hitters steady state (no walk, two expanded levels, sum mode,
 * IntModN<uint32_t> tuples) runs with lanes = keys ("hh_keys" in
 * dpf_hip_last_batch_kernel); outputs are identical in both layouts. */
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
    void* stream);

/* seeds_out[k*num_rows + i] / control_out[k*num_rows + i] = the seed (bit 0
 * cleared) and control bit (bit 0) of cache[k*cache_stride + slot[i]]: a
 * call's start seeds from the previous call's expansion cache. */
int dpf_hip_gather_seeds(int64_t num_keys, int64_t num_rows, const int64_t* slot,
                         const dpf_block* cache, int64_t cache_stride, dpf_block* seeds_out,
                         uint8_t* control_out, void* stream);
/* dpf_hip_gather_seeds with index_major == 1: seeds_out / control_out[i*num_keys
 * + k] from cache[slot[i]*num_keys + k] (cache_stride unused). */
int dpf_hip_gather_seeds_layout(int64_t num_keys, int64_t num_rows, const int64_t* slot,
                                const dpf_block* cache, int64_t cache_stride, dpf_block* seeds_out,
                                uint8_t* control_out, int index_major, void* stream);

/* Device-to-host copy of `count` elements of `elem_bytes` each, element i
 * read at src + i*src_stride_bytes and written packed to dst (a column of an
 * index-major table: one key's partial evaluations, ExportEvaluationContext). */
int dpf_hip_memcpy_d2h_strided(void* dst, const void* src, size_t elem_bytes,
                               size_t src_stride_bytes, int64_t count, void* stream);

/* Largest expand_levels dpf_hip_eval_prefix_batch accepts for this value type
 * (register-resident subtree), or -1 if `sum` mode is not available. */
int dpf_hip_prefix_batch_max_expand(const dpf_value_desc* desc, int sum);

/* out[j] = group sum over r < num_rows of in[r*row_len + j], packed elements of
 * the value type (the generic on-device key sum). */
int dpf_hip_sum_rows(int64_t num_rows, int64_t row_len, const dpf_value_desc* desc,
                     const void* in, void* out, void* stream);

/* Per-key gather (h:822-835 for a key batch):
 * out[k*num_rows*count + i*count + j] = in[k*in_row_elems + src_offset[i] + j]. */
int dpf_hip_gather_batched(int64_t num_keys, int64_t in_row_elems, int64_t num_rows,
                           int64_t count, int elem_size, const int64_t* src_offset,
                           const void* in, void* out, void* stream);

/* ---- batched DCF evaluation ------------------------------
 * DistributedComparisonFunction::Evaluate (dcf/distributed_comparison_function
 * .h:83-105) for every (key, point) of a key batch of the DCF's incremental
 * DPF (num_levels = the DCF's log domain size n, level i has log domain i):
 *   out[k*points_per_key + j] = sum over levels i with bit (n-1-i) of x == 0
 *                               of EvaluateAt(key_k, i, {x >> (n - i)})
 * (for n == 128 the reference uses prefix 0 at every level; mirrored), with
 * x = points[shared_points ? j : k*points_per_key + j] and the sum in the
 * value type's group.  level_depth / level_blocks (host arrays of n) are
 * hierarchy_to_tree and blocks_needed; value_correction (host array of n
 * device pointers) holds level i's value corrections [key][E*num_leaves]. */
int dpf_hip_dcf_eval_batch(int64_t num_keys, int64_t points_per_key, int shared_points,
                           int num_levels, const int32_t* level_depth,
                           const int32_t* level_blocks, const dpf_block* key_seed,
                           const uint8_t* party, const dpf_block* points,
                           const dpf_block* cw_seed, const uint8_t* cw_left,
                           const uint8_t* cw_right, int cw_stride,
                           const dpf_block* const* value_correction,
                           const dpf_aes_key* key_left, const dpf_aes_key* key_right,
                           const dpf_aes_key* key_value, const dpf_value_desc* desc,
                           void* out, void* stream);

/* ---- timing helpers (hipEvents on the given stream) ------------------------ */
int dpf_hip_event_create(void** ev);
int dpf_hip_event_destroy(void* ev);
int dpf_hip_event_record(void* ev, void* stream);
int dpf_hip_event_elapsed_ms(void* start, void* stop, float* ms);

#ifdef __cplusplus
}
#endif

#endif /* DPF_HIP_H_ */
