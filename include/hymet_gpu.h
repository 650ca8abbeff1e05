/* hymet_gpu.h -- C ABI of libhymet_gpu.so, the MI355X (gfx950) implementation of HYMET's
 * contig-classification hot path (Mash screen -> candidate limit -> minimizer
 * seed-chain mapping -> PAF -> weighted LCA).
 *
 * Drop-in boundary.  The reference calls each stage as a subprocess:
 *   scripts/mash.sh:14              mash screen -p 8 -v 0.9 DB input/ *.fna      -> hymet_screen_*
 *   scripts/minimap2.sh:12          minimap2 -I2g -d reference.mmi refs.fasta    -> hymet_mm_index_*
 *   scripts/minimap2.sh:23          minimap2 -x asm10 reference.mmi input/ *.fna -> hymet_mm_map_*
 *   scripts/classification_cami.py:290-308 (_process_one / _weighted_lca)      -> hymet_lca_*
 *   scripts/classification.py:141-157      (process_query / determine_lca)     -> hymet_lca_*
 * The Python drop-ins in scripts/ keep those scripts' argv/file/exit-code contracts and
 * bind this ABI with ctypes (hymet_amd/_lib.py); INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every entry point returns 0 on success, a negative HYMET_E* code on failure;
 *     hymet_last_error() returns a thread-local message for the last failure.
 *   - pointers named d_* are DEVICE pointers (HBM), owned by the caller (the Python host
 *     allocates them through torch); h_* pointers are host pointers.
 *   - all device work is enqueued on the context's stream (hymet_set_stream) and is
 *     asynchronous unless the function says it synchronises.
 *   - no torch / HIP types appear in signatures; a stream is passed as void*.
 */
#ifndef HYMET_GPU_H
#define HYMET_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HYMET_OK 0
#define HYMET_E_HIP (-1)       /* a HIP runtime call failed */
#define HYMET_E_ARG (-2)       /* invalid argument / unsupported parameter */
#define HYMET_E_CAPACITY (-3)  /* caller-provided buffer too small; retry with the size reported */
#define HYMET_E_INTERNAL (-4)  /* a device-side consistency check failed (no out-of-range access was made) */

typedef struct hymet_ctx hymet_ctx;

/* ---------------------------------------------------------------- context */
int hymet_init(int device, hymet_ctx **out);
int hymet_destroy(hymet_ctx *ctx);
const char *hymet_last_error(void);
int hymet_set_stream(hymet_ctx *ctx, void *hip_stream);
int hymet_sync(hymet_ctx *ctx);
int hymet_version(void);
/* Live kernel timing: while enabled, HIP events are recorded on the context stream around
 * every hot-path kernel launch; query returns the summed elapsed ms, the launch count and
 * the summed ALGORITHMIC bytes for a kernel name; bench.py reports
 * the dominant kernel's roofline from these. */
int hymet_prof_enable(hymet_ctx *ctx, int on);
int hymet_prof_reset(hymet_ctx *ctx);
int hymet_prof_query(hymet_ctx *ctx, const char *name, double *total_ms, int64_t *count, double *alg_bytes);
/* newline-separated names of every timed kernel */
int hymet_prof_names(hymet_ctx *ctx, char *buf, int64_t cap);
/* The library's kernel scratch is a caching allocator keyed by (device, stream, size class)
 * (best fit up to twice the request) and capped at HYMET_SCRATCH_CAP_GB (default 160) of
 * cached blocks.  trim synchronises the
 * device and returns every cached block of the device to HIP (e.g. before torch
 * allocates large tensors); cached reports the bytes held. */
int hymet_scratch_trim(hymet_ctx *ctx, int64_t *freed_bytes);
int hymet_scratch_cached(hymet_ctx *ctx, int64_t *bytes);
/* Allocates `bytes` of scratch on the context's stream and returns them to the cache at once
 * (warms the pool before a run; a cached block is reused by later requests of up to that size). */
int hymet_scratch_reserve(hymet_ctx *ctx, int64_t bytes);
/* Process-wide: when hipMalloc fails even after the scratch cache was dropped, call
 * hook(user) once and retry.  The Python host sets it to torch.cuda.empty_cache, so the
 * library's pool and torch's yield to each other (torch's side: hymet_amd._lib.Gpu.empty).
 * NULL clears it. */
int hymet_set_oom_hook(void (*hook)(void *user), void *user);
/* counts[0..2]: the allocator's hipMalloc calls (cache misses), out-of-memory retries (each
 * synchronises the device and drops the cache) and frees past the cap (hipFree), since load. */
int hymet_scratch_stats(hymet_ctx *ctx, int64_t *counts);
/* n bytes of device memory (written by this context's stream) into pageable host memory,
 * through two pinned 64 MiB staging chunks (PCIe and `threads` host copy threads overlap).
 * Synchronous.
 * (The PAF / TSV text copy-out: resultados.paf is written by minimap2.sh:23, the TSV by
 * classification_cami.py:333-339.) */
int hymet_copy_to_host(hymet_ctx *ctx, void *dst, const void *src, int64_t n, int threads);
/* host -> device copy of n bytes through the same double-buffered pinned staging (threads
 * copy chunk k while chunk k-1 is in flight); returns when the bytes are in HBM.  Uploads the
 * FASTA bytes (ingest; classification's input is a host buffer like the reference's file). */
int hymet_copy_to_device(hymet_ctx *ctx, void *dst, const void *src, int64_t n, int threads);

/* ------------------------------------------------------- sequence packing
 * ASCII bases (device) -> 2-bit codes (16 bases per uint32, base i at bits 2*(i%16)) and an
 * invalid-base bitmask (32 bases per uint32).  `alphabet`: 0 = Mash ACGT with upper-casing
 * (CommandScreen hashSequence), 1 = Mash with preserveCase, 2 = minimap2 seq_nt4_table
 * (ACGTU, either case).  n_words2b = ceil(n/16), n_words_mask = ceil(n/32). */
int hymet_pack(hymet_ctx *ctx, const uint8_t *d_ascii, int64_t n, int alphabet,
               uint32_t *d_2b, uint32_t *d_mask);

/* ------------------------------------------------------------------ FASTA ingest
 * The reference hands the pooled contigs to Mash and minimap2 as FASTA files (mash.sh:14,
 * minimap2.sh:23; kseq: a record starts at '>' at the start of a line, the name is the
 * header's first whitespace-delimited token, line breaks are not sequence).  Host half:
 * the record table of a FASTA file in host memory (threads host threads, no copy).  cap =
 * capacity of the h_* arrays; HYMET_E_CAPACITY with *n_rec set when it is too small.
 * Offsets are byte offsets into h_buf; seq [h_seq_off, h_seq_end) includes line breaks,
 * h_nbases excludes them. */
int hymet_fasta_index(const char *h_buf, int64_t n, int threads, int64_t cap, int64_t *n_rec, int64_t *h_name_off,
                      int32_t *h_name_len, int64_t *h_seq_off, int64_t *h_seq_end, int64_t *h_nbases);
/* the names of n records (from the table above) gathered into h_pool (capacity sum of
 * h_name_len), with n + 1 offsets into it */
int hymet_fasta_names(const char *h_buf, const int64_t *h_name_off, const int32_t *h_name_len, int64_t n, char *h_pool,
                      int64_t *h_pool_off);
/* Device half: d_raw holds file bytes [raw_base, raw_base + raw_len) covering n_rec whole
 * records (host tables of those records); writes their sequences joined by one 'N' to
 * d_pool (pool_len = sum(nbases) + n_rec - 1, 16-byte aligned for hymet_pack) and each
 * record's pool offset to d_pool_start.  Synchronises the context stream. */
int hymet_fasta_compact(hymet_ctx *ctx, const uint8_t *d_raw, int64_t raw_len, int64_t raw_base, const int64_t *h_seq_off,
                        const int64_t *h_seq_end, const int64_t *h_nbases, int64_t n_rec, uint8_t *d_pool,
                        int64_t pool_len, int64_t *d_pool_start);
/* khash X31 hash of every name (d_raw + d_name_off[i], d_name_len[i] bytes): the per-query
 * seed of minimap2's hash tie-break (map.c mm_map_frag). */
int hymet_name_hash(hymet_ctx *ctx, const uint8_t *d_raw, const int64_t *d_name_off, const int32_t *d_name_len, int64_t n,
                    uint32_t *d_hash);

/* ------------------------------------------------------------ Mash screen
 * Replaces `mash screen` (scripts/mash.sh:14): one open-addressing table of the distinct
 * sketch hashes of a DB, counts of every pooled canonical k-mer hash that hits it, and the
 * per-reference shared / median-depth statistics. */
int64_t hymet_screen_table_slots(int64_t n_hashes);
/* d_table: n_slots uint64 slots, each key word << 32 | the smallest input index holding the
 * key (its canonical index), all ones when empty.  key_bits 64 (Mash's 64-bit sketches, k > 16):
 * the key word is the key's high 32 bits and a probe matching it checks the full key at
 * d_hashes[index], so d_hashes must stay allocated while the table is used; key_bits 32 (the
 * 32-bit sketches, k <= 16, the only tables hymet_screen_count probes for such k): the word is
 * the whole key and d_hashes is not read after the build;
 * d_scratch: n_hashes + 1 int64 (the duplicate keys' list); d_canon_of: n_hashes int32, each
 * input hash's canonical index (n_hashes for the reserved all-ones key).  Hits are counted per
 * canonical index, so counts are in the DB's own order on every rank whatever slots parallel
 * insertion chose, and the ranks' partial counts add up as they are.  Resets
 * d_table. */
int hymet_screen_table_build(hymet_ctx *ctx, const uint64_t *d_hashes, int64_t n_hashes,
                             uint64_t *d_table, int64_t n_slots, int64_t *d_scratch, int32_t *d_canon_of,
                             int key_bits);
/* The library's stable LSD radix sort (8-bit digits) of device (key, value) pairs by key bits
 * [begin_bit, end_bit), in place (the sort behind the mapper's minimizer, group, chain and
 * anchor-segment orders and the LCA row order; no rocPRIM on the mapping path). */
int hymet_sort_pairs_u64(hymet_ctx *ctx, uint64_t *d_keys, uint32_t *d_vals, int64_t n, int begin_bit, int end_bit);

/* The library's exclusive scan of n device uint32 counts into n int64 offsets (the scan
 * behind every count-then-write pass); *total = the sum (host).  mode 1: the running
 * maximum instead (inclusive, int32 in and out; total unused). */
int hymet_scan_u32(hymet_ctx *ctx, const uint32_t *d_in, int64_t *d_out, int64_t n, int mode, int64_t *total);

/* ---- Mash sketch databases (.msh) ----
 * Replaces the .msh load inside `mash screen` (scripts/mash.sh:14; the DB files of
 * run_hymet_cami.sh:52,85-97 and main.pl:44-46): the Cap'n Proto MinHash message is mapped
 * and parsed natively.  hymet_msh_open maps + parses; hymet_msh_info_get
 * reports the header and sizes; hymet_msh_copy fills any of: hashes (n_hashes uint64, each
 * reference's list ascending, 32-bit hashes widened), offsets (n_refs + 1), lengths
 * (n_refs), names / comments (NUL-separated, names_bytes / comments_bytes), alphabet
 * (alphabet_len bytes, no NUL).  `threads` host threads gather the hashes. */
typedef struct hymet_msh hymet_msh;
typedef struct {
    int32_t k, window_size, sketch_size;
    uint32_t seed;
    int32_t noncanonical, preserve_case, use64;
    int64_t n_refs, n_hashes, names_bytes, comments_bytes, alphabet_len;
} hymet_msh_info;
int hymet_msh_open(const char *path, hymet_msh **out);
int hymet_msh_info_get(const hymet_msh *m, hymet_msh_info *info);
int hymet_msh_copy(const hymet_msh *m, int threads, uint64_t *hashes, int64_t *offsets, int64_t *lengths,
                   char *names, char *comments, char *alphabet);
/* Where each reference's name and comment start in hymet_msh_copy's NUL-separated pools
 * (n_refs + 1 entries each, the last = the pool size): the host reader indexes the pools
 * without scanning them for NULs. */
int hymet_msh_text_offsets(const hymet_msh *m, int64_t *name_start, int64_t *comment_start);
/* The hashes of every reference (as hymet_msh_copy's `hashes`) gathered into the pinned host
 * array `pinned` in n_chunks chunks of equal hash counts, each chunk's host-to-device DMA into
 * `d_hashes` queued on ctx's stream as soon as it is gathered, so the copy of one chunk
 * overlaps the gather of the next.  Returns once every DMA is queued (work queued on the
 * stream afterwards sees the hashes in HBM).  Replaces the gather + one whole upload before
 * the screen table build of `mash screen`'s DB load (scripts/mash.sh:14). */
int hymet_msh_upload(hymet_ctx *ctx, const hymet_msh *m, int threads, uint64_t *pinned, uint64_t *d_hashes,
                     int n_chunks);
/* hymet_msh_upload restricted to hashes [lo_h, hi_h) of the concatenation: pinned[lo_h, hi_h)
 * and d_hashes[lo_h, hi_h) are written, nothing else (references cut by the bounds are copied
 * in part).  A multi-GPU job's ranks each load one slice of the DB and all-gather the slices
 * over xGMI instead of every rank parsing the whole file. */
int hymet_msh_upload_range(hymet_ctx *ctx, const hymet_msh *m, int threads, uint64_t *pinned, uint64_t *d_hashes,
                           int n_chunks, int64_t lo_h, int64_t hi_h);
void hymet_msh_close(hymet_msh *m);
/* Hash every valid canonical k-mer of the packed pool (k in 1..32: MurmurHash3_x64_128
 * word 0 with `seed` for k > 16, MurmurHash3_x86_32 widened to 64 bits for k <= 16, as
 * Mash's 64- / 32-bit sketches), probe ndb (<= 4) tables (hymet_screen_table_build's), count
 * hits into d_counts[i] at the hit key's canonical index (n_hashes[i]+1 uint32 each,
 * caller-zeroed, the last for the all-ones hash), and append every hash < cand_thr to d_cand (bottom-s
 * candidates; d_cand_n counts appends, may exceed cand_cap).  d_nkmers += valid k-mers.
 * seq_begin/seq_end limit the k-mer START positions processed (for sharding). */
int hymet_screen_count(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask,
                       int64_t n_bases, int64_t pos_begin, int64_t pos_end, int k, uint32_t seed,
                       int ndb, const uint64_t *const *h_d_tables, const int64_t *h_n_slots,
                       const uint64_t *const *h_d_hashes, const int64_t *h_n_hashes,
                       uint32_t *const *h_d_counts, uint64_t cand_thr, uint64_t *d_cand,
                       int64_t cand_cap, unsigned long long *d_cand_n,
                       unsigned long long *d_nkmers);
/* Per reference r (hashes d_ref_off[r]..d_ref_off[r+1] of the table input, each counted at
 * d_canon_of[j]): shared[r] = #hashes with count > 0; median[r] = sorted positive
 * counts[shared/2]. */
int hymet_screen_stats(hymet_ctx *ctx, const int64_t *d_ref_off, int64_t n_refs,
                       const int32_t *d_canon_of, const uint32_t *d_counts, uint32_t *d_shared,
                       uint32_t *d_median);

/* --------------------------------------------------- minimizer index (minimap2 -d)
 * Replaces `minimap2 -I2g -d reference.mmi combined_genomes.fasta` (scripts/minimap2.sh:12):
 * default indexing parameters k=15, w=10 (no -x at build time), one handle per -I part.
 * Sequences are given as a packed pool (hymet_pack, alphabet 2) + host start/length arrays
 * (pool offsets); rid = position of the sequence in the arrays. */
typedef struct hymet_mm_index hymet_mm_index;
/* Minimizers (sketch.c mm_sketch semantics) of every sequence, copied to host arrays of
 * capacity cap; rid_mode 0 -> rid 0 (queries), 1 -> rid = sequence index. */
int hymet_mm_sketch(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask, const int64_t *h_starts,
                    const int64_t *h_lens, int32_t n_seq, int w, int k, int rid_mode, uint64_t *h_x,
                    uint64_t *h_y, int64_t cap, int64_t *n_out);
int hymet_mm_index_build(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask, const int64_t *h_starts,
                         const int64_t *h_lens, int32_t n_seq, int w, int k, hymet_mm_index **out);
int hymet_mm_index_destroy(hymet_mm_index *idx);
int hymet_mm_index_info(const hymet_mm_index *idx, int32_t *w, int32_t *k, int32_t *n_seq, int64_t *n_pos);
/* index.c mm_idx_cal_max_occ: the occurrence threshold for a fraction f (-f 2e-4) */
int hymet_mm_index_max_occ(hymet_ctx *ctx, const hymet_mm_index *idx, float frac, int32_t *out);
/* The GPU index persisted beside reference.mmi (minimap2.sh:10 reuses a non-empty index):
 * save writes (append != 0: appends) one part -- header, sequence lengths, the sorted
 * (bucket, y) arrays -- and reports the file offset after it; load reads the part at
 * `offset` and rebuilds the direct-address offsets on the device (no sketching, no sort). */
int hymet_mm_index_save(hymet_ctx *ctx, const hymet_mm_index *idx, const char *path, int append, int64_t *end_offset);
int hymet_mm_index_load(hymet_ctx *ctx, const char *path, int64_t offset, hymet_mm_index **out, int64_t *end_offset);
/* sorted (bucket = minimizer hash, y) arrays, n_pos entries each (tests / persistence) */
int hymet_mm_index_export(hymet_ctx *ctx, const hymet_mm_index *idx, uint32_t *h_hash, uint64_t *h_pos);

/* ------------------------------------------------ mapping (minimap2 -x asm10)
 * Replaces `minimap2 -x asm10 reference.mmi input/ *.fna > resultados.paf`
 * (scripts/minimap2.sh:23).  Options mirror mm_mapopt_t after mm_set_opt("asm10") and
 * mm_mapopt_update (mid_occ resolved by the caller from hymet_mm_index_max_occ). */
typedef struct {
    int32_t mid_occ;
    float q_occ_frac;
    int32_t max_max_occ, occ_dist;
    int32_t min_cnt, min_chain_score;
    int32_t bw, bw_long, max_gap, max_chain_skip;
    int32_t rmq_inner_dist, rmq_size_cap, rmq_rescue_size;
    float rmq_rescue_ratio;
    float chain_gap_scale, chain_skip_scale;
    float mask_level, pri_ratio;
    int32_t mask_len, best_n, a, b, seed;
} hymet_mm_opt;

/* one PAF record before formatting (hit.c mm_reg1_t fields that PAF prints) */
typedef struct {
    int32_t qs, qe, rs, re, rid, rev;
    int32_t mlen, blen, mapq, cnt, score, subsc, parent, id, n_sub, strand_retained;
    float div;
    int32_t as;
    uint32_t hash;
    int32_t pad;
} hymet_mm_reg;

typedef struct hymet_mm_result hymet_mm_result;
/* Map n_q queries (packed pool + host pool offsets/lengths) against one index part.
 * h_name_hash[q] = khash X31 hash of the query name (map.c mm_map_frag). */
int hymet_mm_map(hymet_ctx *ctx, const hymet_mm_index *idx, const hymet_mm_opt *opt,
                 const uint32_t *d_2b, const uint32_t *d_mask, const int64_t *h_starts,
                 const int64_t *h_lens, const uint32_t *h_name_hash, int32_t n_q,
                 hymet_mm_result **out);
/* n_regs total; h_off: n_q+1 per-query offsets; h_rep_len: n_q; h_regs: n_regs records */
int hymet_mm_result_size(const hymet_mm_result *res, int64_t *n_regs);
int hymet_mm_result_copy(const hymet_mm_result *res, int64_t *h_off, int32_t *h_rep_len,
                         hymet_mm_reg *h_regs);
int hymet_mm_result_destroy(hymet_mm_result *res);
/* Device-resident resultados.paf of a run: hymet_mm_map_acc appends one batch's lines
 * (query q_base + q, index part part_id, target t_base + rid), so after every part x batch
 * the accumulator holds minimap2's output order (part-major, queries in input order).  The
 * classifier and the PAF text writer read it in place; nothing returns to the host. */
typedef struct hymet_paf_acc hymet_paf_acc;
int hymet_paf_acc_create(hymet_ctx *ctx, hymet_paf_acc **out);
int hymet_paf_acc_reset(hymet_paf_acc *acc);
int hymet_paf_acc_destroy(hymet_paf_acc *acc);
/* line count and the device arrays (hymet_mm_reg, int32 query, part, rep_len, target) */
int hymet_paf_acc_info(const hymet_paf_acc *acc, int64_t *n_lines, void **d_regs, void **d_q, void **d_part, void **d_rl,
                       void **d_t);
/* append lines [begin, end) of src to dst (device copies on ctx's stream; src's producing
 * work must be complete -- hymet_mm_map_acc returns synchronised) */
int hymet_paf_acc_append(hymet_ctx *ctx, hymet_paf_acc *dst, const hymet_paf_acc *src, int64_t begin, int64_t end);
/* query, part and target index of every line, copied to host arrays of n_lines (synchronous) */
int hymet_paf_acc_copy(hymet_ctx *ctx, const hymet_paf_acc *acc, int32_t *h_q, int32_t *h_part, int32_t *h_t);
/* one int32 field of every line's hymet_mm_reg record (field = word index, e.g. 9 = cnt, the
 * chain's minimizer count that PAF prints as cm:i), copied to a host array of n_lines */
int hymet_paf_acc_field(hymet_ctx *ctx, const hymet_paf_acc *acc, int field, int32_t *h_out);
int hymet_mm_map_acc(hymet_ctx *ctx, const hymet_mm_index *idx, const hymet_mm_opt *opt, const uint32_t *d_2b,
                     const uint32_t *d_mask, const int64_t *h_starts, const int64_t *h_lens, const uint32_t *d_name_hash,
                     int32_t n_q, int32_t q_base, int32_t part_id, int32_t t_base, hymet_paf_acc *acc);
/* resultados.paf text of the accumulator's lines (format.c mm_write_paf3 + write_tags, no
 * CIGAR): query names d_qname[d_qname_off[q] .. d_qname_off[q+1]), d_qlen[q]; target names
 * and lengths likewise.  *n_bytes = text size; HYMET_E_CAPACITY when > cap (nothing
 * written).  d_line_off (optional, n_lines + 1): byte offset of every line. */
int hymet_emit_paf(hymet_ctx *ctx, const hymet_paf_acc *acc, const uint8_t *d_qname, const int64_t *d_qname_off,
                   const int64_t *d_qlen, const uint8_t *d_tname, const int64_t *d_tname_off, const int64_t *d_tlen,
                   char *d_out, int64_t cap, int64_t *n_bytes, int64_t *d_line_off);
/* Chaining DP alone (lchain.c mg_lchain_rmq's f[]/p[], the stage inside hymet_mm_map), for
 * parity tests and kernel timing: n anchors (x, y as minimap2 packs them) of ONE query,
 * sorted by x; groups are runs of equal x>>32.  max_dist/bw are given as mg_lchain_rmq
 * receives them (first pass: max_gap, bw; long join: max_gap, bw_long).  Host arrays,
 * synchronous; h_p holds anchor indices or -1. */
int hymet_mm_chain_dp(hymet_ctx *ctx, const uint64_t *h_x, const uint64_t *h_y, int64_t n, int max_dist,
                      int max_dist_inner, int bw, int max_chn_skip, int cap_rmq_size, float pen_gap,
                      float pen_skip, int32_t *h_f, int64_t *h_p);

/* --------------------------------------------------- weighted LCA (classify)
 * Replaces the per-query loop of scripts/classification_cami.py:290-308 (+ _weighted_lca
 * :251-288; mode 0) and scripts/classification.py:141-157 (mode 1).  PAF lines are given
 * per query in PAF order (d_q_off CSR); targets/taxids are integer-encoded by the host.
 * hymet_lca_ref_counts: d_counts[t] += #lines with target t (ref_abundance, caller-zeroed;
 * all-reduced across ranks by the caller). */
int hymet_lca_ref_counts(hymet_ctx *ctx, const int32_t *d_line_t, int64_t n_lines, int32_t *d_counts);
/* The same over a hymet_paf_acc (the fused path): ref_counts of its lines, then rows = the
 * queries with >= 1 line in classification_cami.py's output order (first appearance in
 * the PAF: by index part of the first line, then query index), each classified over its
 * lines in PAF order.  Row outputs hold n_q entries; *n_rows is set (synchronises).  Query
 * lengths d_qlen[q]; the legacy mode's exact-match test compares query and target names. */
int hymet_acc_ref_counts(hymet_ctx *ctx, const hymet_paf_acc *acc, int32_t *d_counts);
int hymet_acc_classify(hymet_ctx *ctx, const hymet_paf_acc *acc, int mode, int32_t n_q, const int64_t *d_qlen,
                       const int32_t *d_ref_counts, const int32_t *d_t_tax, const int32_t *d_tax_names,
                       const uint8_t *d_tax_in_hier, const uint8_t *d_qname_pool, const int64_t *d_qname_off,
                       const uint8_t *d_tname_pool, const int64_t *d_tname_off, int32_t *d_row_q, int32_t *d_row_part,
                       int32_t *d_row_depth, int32_t *d_row_names, double *d_row_conf, int32_t *d_row_tax,
                       int32_t *n_rows);
/* classified_sequences.tsv rows (no header) for LCA rows (csv.writer: tab, minimal quoting,
 * CRLF, "%.4f"): query names by row_q from the name pool; CAMI lineages "rank:name" joined
 * by "; " from the label pool, legacy ones ";"-joined raw parts, the legacy exact shortcut
 * the taxid's raw lineage / level strings.  Two-call capacity protocol as hymet_emit_paf. */
int hymet_emit_tsv(hymet_ctx *ctx, int mode, int32_t n_rows, const int32_t *d_row_q, const int32_t *d_row_depth,
                   const int32_t *d_row_names, const double *d_row_conf, const int32_t *d_row_tax, const uint8_t *d_qname,
                   const int64_t *d_qname_off, const uint8_t *d_label, const int64_t *d_label_off, const uint8_t *d_taxlin,
                   const int64_t *d_taxlin_off, const uint8_t *d_taxlvl, const int64_t *d_taxlvl_off, char *d_out,
                   int64_t cap, int64_t *n_bytes);
int hymet_lca(hymet_ctx *ctx, int mode, int32_t n_q, const int64_t *d_q_off, const int32_t *d_line_t,
              const int64_t *d_line_blen, const int64_t *d_line_qlen, const uint8_t *d_line_exact,
              const int32_t *d_ref_counts, const int32_t *d_t_tax, const int32_t *d_tax_names,
              const uint8_t *d_tax_in_hier, int32_t *d_scr_tid, double *d_scr_w, int32_t *d_scr_nm,
              double *d_scr_nw, int32_t *d_out_depth, int32_t *d_out_names, double *d_out_conf,
              int32_t *d_out_tax);

#ifdef __cplusplus
}
#endif
#endif
