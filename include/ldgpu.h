/* ldgpu.h -- C ABI of libldgpu.so, the MI355X (gfx950) hot path of
 * spark-languagedetector: FIT byte n-gram counting into per-language gram
 * probability tables, and SCORE (window scan, gram->row lookup, fp64
 * accumulation, argmax).
 *
 * Plain C, POD arguments only.  Every entry point returns an int status
 * (LDGPU_OK = 0) and leaves a thread-local message for ldgpu_last_error().
 * All entry points are thread-safe; calls on one ldgpu_ctx are serialised on
 * that context's HIP stream.
 *
 * Reference interfaces replaced (Scala, /root/reference/src/main/scala/org/
 * apache/spark/ml/feature/languagedetection/):
 *   ldgpu_model_create  -- new LanguageDetectorModel(gramProbabilities,
 *                          gramLengths, languages)  LanguageDetectorModel.scala:178-198
 *                          + the table broadcast of transform  :222
 *   ldgpu_score[_device]-- LanguageDetectorModel.detect(Array[Byte], map, langs,
 *                          grams) :131-156, batched over documents (the per-row
 *                          map of transform :225-238)
 *   ldgpu_count[_device]-- LanguageDetector computeGrams + reduceGrams
 *                          LanguageDetector.scala:25-66
 *   ldgpu_fit_table_*   -- computeProbabilities + filterTopGrams + collect.toMap
 *                          LanguageDetector.scala:75-132, :252-254
 *
 * Encodings are the caller's job (as in the reference): FIT documents are
 * UTF-8 bytes (String.getBytes(UTF-8), LanguageDetector.scala:37); SCORE
 * documents are the low byte of every UTF-16 code unit
 * (text.toCharArray.map(_.toByte), LanguageDetectorModel.scala:161).
 *
 * Documents are packed: bytes[offsets[d] .. offsets[d+1]) is document d;
 * offsets has n_docs + 1 non-decreasing entries.
 */
#ifndef LDGPU_H
#define LDGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ldgpu_status {
    LDGPU_OK = 0,
    LDGPU_EINVAL = 1,        /* bad argument: gram length <= 0, bad offsets, null pointer, L < 1 */
    LDGPU_EROWLEN = 2,       /* a scored window hit a row whose length != #languages
                                (BLAS.axpy require, LanguageDetectorModel.scala:149) */
    LDGPU_ENOMEM = 3,        /* device or host allocation failed / count table full */
    LDGPU_EDEVICE = 4,       /* HIP runtime error */
    LDGPU_EUNSUPPORTED = 5,  /* outside the device path's limits (see below) */
    LDGPU_ENODEV = 6         /* no HIP device */
};

/* Device-path limits.  Gram lengths 1..LDGPU_MAX_GRAM for SCORE tables and
 * LDGPU_MAX_FIT_GRAM for FIT counting: keys of up to 7 bytes pack into one
 * u64 (7 payload bytes + a length byte); keys of 8..15 bytes take two words,
 * in a table of their own (SCORE and FIT alike); a SCORE table with a gram
 * length beyond 15 keeps every key in a general table (hash + key bytes
 * compared on the device: any length, as the reference), and FIT counts grams
 * of more than 15 bytes in a table of such keys (up to 2^24 - 1 bytes).  1..LDGPU_MAX_LANGS
 * languages (SCORE scores more than 256 in blocks of 256 languages). */
#define LDGPU_MAX_GRAM 2147483647  /* SCORE tables: any gram length */
#define LDGPU_MAX_FIT_GRAM 16777215  /* FIT counting: lengths beyond 15 in a general-key table */
#define LDGPU_MAX_LANGS 4096
#define LDGPU_MAX_GRAM_LENGTHS 32

const char* ldgpu_version(void);
/* build provenance: sha256 (first 16 hex digits) of the sources this library
 * was compiled from (spark-languagedetector_amd/Makefile, PROV) */
const char* ldgpu_build_id(void);
const char* ldgpu_last_error(void);          /* thread-local, never NULL */
int ldgpu_device_count(int32_t* out_count);

/* ---------------------------------------------------------------- context */
typedef struct ldgpu_ctx ldgpu_ctx;
int ldgpu_ctx_create(int32_t device, ldgpu_ctx** out);
int ldgpu_ctx_destroy(ldgpu_ctx* ctx);
int ldgpu_ctx_synchronize(ldgpu_ctx* ctx);
void* ldgpu_ctx_stream(ldgpu_ctx* ctx);      /* the context's hipStream_t */

/* Page-locked host memory for the host-buffer APIs: documents packed straight
 * into it (a JNI shim wraps it in direct ByteBuffers) are copied to the device
 * without a staging copy; labels written into it skip one too.  Replaces the
 * JVM-owned row buffers of transform (LanguageDetectorModel.scala:225-238). */
int ldgpu_host_alloc(ldgpu_ctx* ctx, int64_t n_bytes, void** out);
int ldgpu_host_free(ldgpu_ctx* ctx, void* p);

/* ------------------------------------------------------------------ SCORE */
typedef struct ldgpu_model ldgpu_model;

/* The gram -> probability-row map.  Key i is key_bytes[key_offsets[i] ..
 * key_offsets[i+1]); its row is rows[i*n_langs .. (i+1)*n_langs) in
 * supported-language order.  row_ok (nullable) marks rows whose length in the
 * caller's map differs from n_langs: scoring a document that hits such a row
 * fails with LDGPU_EROWLEN, as BLAS.axpy does in the reference.  A later
 * duplicate key replaces an earlier one (Scala toMap).  gram_lengths is kept
 * in order, duplicates included (each repeat scans the document again). */
int ldgpu_model_create(ldgpu_ctx* ctx, int64_t n_rows, const uint8_t* key_bytes,
                       const int64_t* key_offsets, const double* rows, const uint8_t* row_ok,
                       int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                       ldgpu_model** out);
/* Mask form of the same table (what a fit produces, and what a table too
 * large for dense rows is carried in): row i is vals[i] at the languages set
 * in masks[i*S .. (i+1)*S), S = ceil(n_langs / 64), 0.0 elsewhere. */
int ldgpu_model_create_masks(ldgpu_ctx* ctx, int64_t n_rows, const uint8_t* key_bytes,
                             const int64_t* key_offsets, const uint64_t* masks, const double* vals,
                             int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                             ldgpu_model** out);
int ldgpu_model_destroy(ldgpu_model* model);

/* mode: 0 = every row is one value times a language bitmask, 1 = dense fp64
 * rows, 2 = mask form where every row shares ONE finite value (fit-produced
 * tables whose grams all have the same presence class, e.g. all unique to one
 * language): scored from per-language hit counts.  n_keys: keys resident on
 * the device. */
int ldgpu_model_info(const ldgpu_model* model, int32_t* mode, int64_t* n_keys,
                     int64_t* table_slots, int64_t* filter_bits, int64_t* device_bytes);

/* The device layout the model's scoring kernel takes (bit set = in use), so a
 * caller (and the parity tests) can tell which product path scores it:
 * the window filter (LDS prefix Bloom, or a keyed bloom in L2 / Infinity Cache,
 * one word per key or one 64-B line per window position), the key table
 * (cuckoo slots, or 4-slot buckets for count-mode tables beyond 2^20 keys),
 * packs of short documents (labels-only count mode). */
#define LDGPU_LAYOUT_LDS_BLOOM          0x01
#define LDGPU_LAYOUT_KEYED_BLOOM        0x02
#define LDGPU_LAYOUT_KEYED_BLOOM_LINES  0x04
#define LDGPU_LAYOUT_BUCKETS            0x08
#define LDGPU_LAYOUT_WIDE_KEYS          0x10
#define LDGPU_LAYOUT_DIRECT             0x20
#define LDGPU_LAYOUT_PACKS              0x40
#define LDGPU_LAYOUT_LANG_BLOCKS        0x80
#define LDGPU_LAYOUT_GENERAL_KEYS       0x100  /* keys of any length (a gram length > 15) */
#define LDGPU_LAYOUT_KEYED_BLOOM_CHUNKS 0x200  /* count mode: one 16-B bloom chunk per window position */
#define LDGPU_LAYOUT_CLASSES            0x400  /* labels-only calls on a mask table of at most 4 distinct
                                                  finite values: per-(value, language) hit counts and a
                                                  rounding bound; documents the bound cannot separate
                                                  replayed in reference order */
int ldgpu_model_layout(const ldgpu_model* model, int32_t* flags);
/* The model's language count (a caller sizing score buffers, e.g. the JNI
 * shim, takes it from the model rather than trusting its own). */
int ldgpu_model_langs(const ldgpu_model* model, int32_t* n_langs);

/* Host buffers in, host buffers out; synchronous.  out_scores is nullable
 * ([n_docs][n_langs] fp64).  out_labels[d] is the index into the supported
 * languages of argmax(scores of d): first maximum, all-zero -> 0.  Chunks of
 * documents are pipelined over two streams (copy-in / score / copy-out of one
 * chunk overlap the host staging of the next); buffers from ldgpu_host_alloc
 * are copied from / to directly, pageable ones through pinned staging.  (A
 * class-mode table's replay of ambiguous documents is sized on the device, so
 * the pipeline never waits for the GPU between chunks.) */
int ldgpu_score(ldgpu_model* model, const uint8_t* bytes, const int64_t* offsets,
                int64_t n_docs, int32_t* out_labels, double* out_scores);

/* Device-resident variant, asynchronous on `stream` (a hipStream_t used as
 * given: NULL is HIP's null stream; ldgpu_ctx_stream() gives the context's).
 * d_bytes must be 4-byte aligned and n_bytes >= d_offsets[n_docs].
 * d_scores is nullable.  Offsets are trusted (validate with the host API);
 * documents must be shorter than 2^28 bytes (the host API checks this).
 * A labels-only call (d_scores NULL) on a model in class mode
 * (LDGPU_LAYOUT_CLASSES) replays the documents its rounding bound left
 * ambiguous on the same stream, sized on the device: it is asynchronous too. */
int ldgpu_score_device(ldgpu_model* model, const uint8_t* d_bytes, int64_t n_bytes,
                       const int64_t* d_offsets, int64_t n_docs, int32_t* d_labels,
                       double* d_scores, void* stream);

/* -------------------------------------------------------------------- FIT */
typedef struct ldgpu_counts ldgpu_counts;

/* A device count table for n_langs languages and the given gram lengths.
 * capacity_hint: expected distinct grams (0 = default); the table grows when
 * it passes half full between batches. */
int ldgpu_counts_create(ldgpu_ctx* ctx, int32_t n_langs, const int32_t* gram_lengths,
                        int32_t n_grams, int64_t capacity_hint, ldgpu_counts** out);
int ldgpu_counts_destroy(ldgpu_counts* counts);
/* The table's language count. */
int ldgpu_counts_langs(const ldgpu_counts* counts, int32_t* n_langs);

/* Accumulate one batch of documents: every window of every gram length is
 * counted for doc_lang[d] (documents whose doc_lang is outside [0, n_langs)
 * are skipped, as reduceGrams filters unsupported languages).  Device
 * scratch per call: the records of up to ~512 MB of corpus at a time (~16 GB,
 * kept by the context for the next call) and a table of the call's maximal
 * windows (one per byte position), from which every gram length's counts are
 * derived before the call returns (FIT v4). */
int ldgpu_count(ldgpu_counts* counts, const uint8_t* bytes, const int64_t* offsets,
                const int32_t* doc_lang, int64_t n_docs);
int ldgpu_count_device(ldgpu_counts* counts, const uint8_t* d_bytes, int64_t n_bytes,
                       const int64_t* d_offsets, const int32_t* d_doc_lang, int64_t n_docs,
                       void* stream);

/* Distinct grams and their total key bytes. */
int ldgpu_counts_size(ldgpu_counts* counts, int64_t* n_grams, int64_t* key_bytes);
/* Distinct grams, distinct (gram, language) pairs -- the rows reduceGrams
 * emits (LanguageDetector.scala:57-65) -- and the sum of all counts (= the
 * windows counted).  Any output pointer may be NULL. */
int ldgpu_counts_stats(ldgpu_counts* counts, int64_t* n_grams, int64_t* n_pairs, int64_t* total);
/* Export sorted by (length, unsigned bytes): key_bytes, key_offsets[n+1],
 * counts[n][n_langs] (raw int64 sums; the JVM sums wrap at 2^31). */
int ldgpu_counts_export(ldgpu_counts* counts, uint8_t* key_bytes, int64_t* key_offsets,
                        int64_t* counts_out);

/* Merge a dense (keys, counts[n][n_langs]) block into the table (used by the
 * multi-GPU merge after an all-reduce over a common key list).  Keys are
 * given packed as in ldgpu_counts_export. */
int ldgpu_counts_add(ldgpu_counts* counts, int64_t n, const uint8_t* key_bytes,
                     const int64_t* key_offsets, const int64_t* counts_in);

/* Sparse form of the table, what crosses a Spark shuffle: the grams
 * [first, first + n) of the (length, bytes) order (0 <= first <= first + n <=
 * n_grams) with their nonzero (language, count) pairs in language order --
 * ~1.3 pairs per gram on the fit corpora against n_langs dense counters.
 * _sparse_size gives the range's key bytes and pairs; _export_sparse writes
 * key_bytes, key_offsets[n + 1] and pair_offsets[n + 1] (both relative to the
 * range), pair_langs and pair_counts.  Exporting in ranges keeps every buffer
 * as small as the caller wants (a JVM direct buffer holds < 2 GiB).
 * _add_sparse adds such a block (keys of 1..15 bytes, counts >= 0). */
int ldgpu_counts_sparse_size(ldgpu_counts* counts, int64_t first, int64_t n, int64_t* key_bytes,
                             int64_t* n_pairs);
int ldgpu_counts_export_sparse(ldgpu_counts* counts, int64_t first, int64_t n, uint8_t* key_bytes,
                               int64_t* key_offsets, int64_t* pair_offsets, int32_t* pair_langs,
                               int64_t* pair_counts);
int ldgpu_counts_add_sparse(ldgpu_counts* counts, int64_t n, const uint8_t* key_bytes,
                            const int64_t* key_offsets, const int64_t* pair_offsets,
                            const int32_t* pair_langs, const int64_t* pair_counts);

/* Device-resident forms of export / add (the multi-GPU merge keeps counts in
 * HBM and exchanges them with RCCL).  Keys are packed u64: bytes little-endian
 * in bits 0..55, length (1..7) in bits 56..63 (a table holding grams of 8..15
 * bytes fails export_device with LDGPU_EUNSUPPORTED: use ldgpu_counts_export).  export_device writes the
 * distinct grams (unordered) into caller buffers of `capacity` entries
 * (keys[capacity], counts[capacity][n_langs] int64) and their number to
 * *n_out; it fails with LDGPU_EINVAL if capacity is too small.  Both are
 * synchronous with respect to `stream` (NULL = HIP's null stream). */
int ldgpu_counts_export_device(ldgpu_counts* counts, int64_t capacity, uint64_t* d_keys,
                               int64_t* d_counts, int64_t* n_out, void* stream);
int ldgpu_counts_add_device(ldgpu_counts* counts, int64_t n, const uint64_t* d_keys,
                            const int64_t* d_counts, void* stream);

/* ------------------------------------------------------- multi-GPU FIT merge
 * Replaces the reference's shuffles of reduceGrams / computeProbabilities /
 * filterTopGrams (LanguageDetector.scala:57-65, :79-81, :110-126) when the
 * corpus is sharded over executors, one GPU each.  A communicator spans the
 * ranks of one fit; two transports run the same merge:
 *   RCCL over xGMI  -- ldgpu_comm_create_rccl; rank 0 makes the id with
 *                      ldgpu_comm_unique_id and the caller hands it to every
 *                      rank (Spark: a driver broadcast);
 *   host callbacks  -- ldgpu_comm_create_host; the caller provides an
 *                      all-gather and an all-to-all over host memory (an
 *                      executor's own transport; gloo in the tests). */
typedef struct ldgpu_comm ldgpu_comm;
#define LDGPU_COMM_ID_BYTES 128

typedef struct {
    void* user;
    /* recv = world * bytes, rank r's block at r * bytes; returns 0 on success */
    int (*allgather)(void* user, const void* send, int64_t bytes, void* recv);
    /* send_bytes[r] bytes to rank r (blocks in rank order), recv_bytes[r]
     * from rank r (blocks in rank order); returns 0 on success */
    int (*alltoallv)(void* user, const void* send, const int64_t* send_bytes, void* recv,
                     const int64_t* recv_bytes);
} ldgpu_host_coll;

int ldgpu_comm_unique_id(uint8_t* out_id /* LDGPU_COMM_ID_BYTES */);
int ldgpu_comm_create_rccl(ldgpu_ctx* ctx, const uint8_t* id, int32_t rank, int32_t world, ldgpu_comm** out);
int ldgpu_comm_create_host(ldgpu_ctx* ctx, int32_t rank, int32_t world, const ldgpu_host_coll* coll,
                           ldgpu_comm** out);
int ldgpu_comm_destroy(ldgpu_comm* comm);

/* Owner-partitioned exchange: gram g belongs to rank owner(g) (a hash of its
 * key), every rank sends its counts of the grams it does not own to their
 * owners (one all-to-all), and afterwards holds the GLOBAL counts (sums over
 * all ranks, bit-exact) of exactly the grams it owns.  ldgpu_counts_export /
 * _size / _stats then describe the owned shard; ldgpu_fit_table_size on the
 * merged table runs the global top-K through the communicator (a (language,
 * class) histogram all-reduce, an all-gather of each rank's tie candidates,
 * an all-gather of the chosen rows), and every rank exports the same table.
 * Grams of 8..15 bytes (their own table) travel by an all-gather of every
 * rank's entries instead, each rank keeping those it owns, and a merged table
 * holding any takes the top-K over every rank's presence rows on the host.
 * Collective: every rank calls it.  Counting more documents into a merged
 * table is an error (LDGPU_EINVAL). */
int ldgpu_counts_merge(ldgpu_counts* counts, ldgpu_comm* comm);

/* computeProbabilities + filterTopGrams: v_l = log(1 + [g in l] / k_g);
 * per language the profile_size largest v_l (ties: ascending (length, bytes));
 * the union of the chosen grams with their full rows.  Two calls: _size
 * computes and caches the table, _export copies it (sorted by (length, bytes)). */
int ldgpu_fit_table_size(ldgpu_counts* counts, int32_t profile_size, int64_t* n_rows,
                         int64_t* key_bytes);
int ldgpu_fit_table_export(ldgpu_counts* counts, uint8_t* key_bytes, int64_t* key_offsets,
                           double* rows);
/* The cached table's rows and key bytes (what the last _size returned);
 * LDGPU_EINVAL before any _size. */
int ldgpu_fit_table_info(ldgpu_counts* counts, int64_t* n_rows, int64_t* key_bytes);
/* The same table in mask form (masks [n_rows][ceil(L/64)], vals [n_rows]):
 * 8 (S + 1) bytes per row instead of 8 L -- what ldgpu_model_create_masks
 * takes (config-5 tables: 10M rows x 200 languages). */
int ldgpu_fit_table_export_masks(ldgpu_counts* counts, uint8_t* key_bytes, int64_t* key_offsets,
                                 uint64_t* masks, double* vals);

/* ----------------------------------------------------------- PREPROCESS */
/* The caller-side preprocessors on the device, over Java strings (UTF-16 code
 * units, offsets in units):
 *   LDGPU_PRE_LOWER  LowerCasePreprocessor (LowerCasePreprocessor.scala:44-76):
 *                    String.toLowerCase(Locale.forLanguageTag(label)) -- each
 *                    unit through the host language's 1:1 mapping (`lower`,
 *                    e.g. Character.toLowerCase), the 1:1 locale rules of
 *                    tr / az (I -> U+0131, U+0130 -> i) applied on the device;
 *   LDGPU_PRE_CLEAN  SpecialCharPreprocessor's documented intent
 *                    (SpecialCharPreprocessor.scala:40-70): the symbols
 *                    / _ [ ] * ( ) % ^ & @ $ # : | { } < > ~ ` " \ and every
 *                    space removed (the reference's own pattern never
 *                    compiles: the JVM throws PatternSyntaxException);
 *   LDGPU_PRE_LOW_BYTES  the output is the SCORE encoding (the low byte of each
 *                    unit, LanguageDetectorModel.scala:226) instead of units:
 *                    ldgpu_score_device's input.
 * A document whose lower-casing is not 1:1 or needs context -- a unit marked
 * in `special` (U+0130 outside tr / az, capital sigma's Final_Sigma rule, the
 * high surrogates of cased supplementary planes), tr / az "I" + U+0307, lt
 * I / J / U+012E before a mark above, U+00CC / U+00CD / U+0128 -- is not
 * processed: host[d] = 1 and its output is empty; the caller lower-cases it
 * itself (the Java locale rules stay on the host). */
#define LDGPU_PRE_LOWER      1
#define LDGPU_PRE_CLEAN      2
#define LDGPU_PRE_LOW_BYTES  4
#define LDGPU_LOCALE_ROOT    0  /* per-document locale class of the label */
#define LDGPU_LOCALE_TR_AZ   1  /* Locale.forLanguageTag(label).getLanguage() is tr or az */
#define LDGPU_LOCALE_LT      2  /* ... lt */

typedef struct ldgpu_casemap ldgpu_casemap;
/* lower: [65536] the lower-case unit of each unit (1:1); special: [8192]
 * bytes, bit u set = unit u sends its document to the host. */
int ldgpu_casemap_create(ldgpu_ctx* ctx, const uint16_t* lower, const uint8_t* special, ldgpu_casemap** out);
int ldgpu_casemap_destroy(ldgpu_casemap* map);
/* Device buffers, asynchronous on `stream` (NULL: the default stream).
 * d_out holds up to d_offsets[n_docs] - d_offsets[0] units (bytes with
 * LDGPU_PRE_LOW_BYTES); d_out_offsets [n_docs + 1] receives the output's
 * offsets (from 0); d_host [n_docs]; d_locale (nullable: root) [n_docs]. */
int ldgpu_preprocess_device(ldgpu_casemap* map, const uint16_t* d_units, const int64_t* d_offsets,
                            int64_t n_docs, const uint8_t* d_locale, int32_t flags, void* d_out,
                            int64_t* d_out_offsets, uint8_t* d_host, void* stream);
/* The same over host buffers (copied in and out; returns when done). */
int ldgpu_preprocess(ldgpu_casemap* map, const uint16_t* units, const int64_t* offsets, int64_t n_docs,
                     const uint8_t* locale, int32_t flags, void* out, int64_t* out_offsets, uint8_t* host);

#ifdef __cplusplus
}
#endif

#endif /* LDGPU_H */
