// ldgpu_internal.h -- kernel parameter blocks and launchers shared between the
// kernels (ldgpu_score.hip, ldgpu_fit.hip) and the host runtime (ldgpu_api.hip).
#pragma once

#include "ldgpu_common.h"

// Diagnostics build (lib/libldgpu_diag.so, -DLDGPU_DIAG=1): only there does
// the library read the LDGPU_* environment switches (path selection for tests,
// timing ablations, statistics).  The product library (lib/libldgpu.so) never
// consults the environment, and its kernels contain no ablation branch.
#ifndef LDGPU_DIAG
#define LDGPU_DIAG 0
#endif

namespace ldgpu {

// ------------------------------------------------------------------ SCORE
struct ScoreParams {
    const uint8_t* bytes;       // 4-byte aligned
    int64_t n_bytes;            // readable bytes of `bytes`
    int64_t last_dword;         // index of the last readable dword of bytes
    const int64_t* offsets;     // [n_docs + 1]
    int64_t n_docs;
    int32_t group;              // documents per staged group (1..63)
    int32_t* labels;            // [n_docs]
    double* scores;             // nullable [n_docs][L]
    const Slot* slots;          // open-addressed key -> row table (modes 0-2)
    const Bucket* buckets;      // count mode: bucketed key -> (row, language) table; slot_shift/mask index it
    uint32_t slot_shift;        // bucket = mix64(key) >> slot_shift (or & slot_mask)
    uint64_t slot_mask;
    uint32_t slot_shift32;      // cuckoo slot = h1 (h2) >> slot_shift32 of slot_hash
    const WideSlot* wslots;     // wide keys (8..15 bytes), nullptr: none
    uint32_t wslot_shift32;     // wide slot = h1 (h2) >> wslot_shift32 of wide_hash
    const uint32_t* filter;     // image: bmp1 | bmp2 | bloom (ldgpu_common.h)
    uint32_t bloom_words;       // power of two
    uint32_t bloom_shift;       // bloom word = hash >> bloom_shift (>= 10)
    int32_t kb_lines;           // keyed bloom in the line layout (kb_line16: blooms beyond kKbLineBytes)
    uint32_t len_mask;          // bit k set: the table holds keys of k bytes
    const uint64_t* masks;      // mask mode: [rows][S] language bitmasks
    const double* vals;         // mask mode: [rows] the row's one nonzero value
    const double* rows;         // dense mode: [rows][L]
    const double* fold;         // count mode: fold[c] = c left-folded adds of the value, c <= fold_max
    uint32_t fold_max;
    int32_t count_sign;         // count mode: sign of the value (fold[c] strictly monotone)
    int64_t count_argmax_len;   // count mode: documents up to this length take count_argmax (-1: none)
    int32_t* err;               // bit 0: a window hit a wrong-length row; bit 1: doc too long
    unsigned long long* stats;  // diagnostics build (-DLDGPU_STATS, env LDGPU_STATS): [0] candidates verified, [1] hits
    int32_t L;
    int32_t ablate;             // diagnostics build only (LDGPU_ABLATE; compiled out otherwise): bit 0 skip
                                // verify/accumulate, bit 1 skip probe, bit 2 skip the hit replay, bit 3
                                // skip count-mode 1-/2-byte direct counts, bit 4 skip count-mode >= 3-byte
                                // tests, bit 5 skip the count argmax (labels 0)
    int32_t nG;
    int32_t G[kMaxGramLengths];
    // fast path (documents of maxg..256 bytes: every window full-length):
    // the gram lengths with a table key, 4 bits each in order (16 per word);
    // count mode: each distinct length once
    uint64_t gpack[2];
    int32_t n_fast;             // entries in gpack
    int32_t maxg;               // max(G)
    uint32_t fast_mask;         // count mode fast path: bit n = n is in G and some key has n bytes
    uint8_t mult[16];           // count mode: multiplicity of n in G (the fast path tests n once)
    // count mode, direct tables (every 1-/2-byte key names one language):
    // image words [direct_off, + direct_words) = lang1[256] u8 (0xff: no key),
    // base2[2048] u16 (rank of each 2-byte bitmap word), lang2[n2] u8
    uint32_t direct_off;
    uint32_t direct_words;      // 0: no direct tables
    // count mode: consecutive short documents are scored in packs
    // (score_pack; the hit area holds kPackDocs counter blocks)
    int32_t pack;
    // language blocks (L > kBlockLangs: one launch per block of languages,
    // ldgpu_api.hip): per document this block's maximum score (block 0 with
    // a NaN first score: +inf, the reference keeps index 0), the block index
    // (the NaN-first rule is block 0's only) and the scores' row stride
    double* best;
    int32_t block;
    int64_t score_stride;       // 0: L
};

// languages per block of a blocked model (L > kBlockLangs)
constexpr int kBlockLangs = 256;

// Launch configuration of the score kernel.
#ifndef LDGPU_SCORE_WAVES
#define LDGPU_SCORE_WAVES 12
#endif
constexpr int kScoreWaves = LDGPU_SCORE_WAVES;  // waves per workgroup (768 threads)
// occupancy target (HIP launch bound: waves per SIMD = WGs x waves / 4):
// 2 workgroups = 24 waves per CU (6 per SIMD) caps the kernel at 80 VGPRs;
// two copies of the filter image + 24 waves' queues, hit areas and
// double-buffered group staging fit the 160 KiB LDS (score_lds_bytes)
#ifndef LDGPU_SCORE_MIN_WG
#define LDGPU_SCORE_MIN_WG 2
#endif
constexpr int kScoreMinWgPerCu = LDGPU_SCORE_MIN_WG;
constexpr int kQueueCap = 288;             // candidate entries (u32) per wave (>= 256 + slack)
constexpr int kBufBytes = 1024;            // staged bytes of a document group per wave (one 64 x 16-B LDS-DMA)
constexpr int kBufWords = kBufBytes / 4 + 4;
constexpr int kMaxLdsBloomLog2 = 14;       // bloom words in LDS up to 64 KiB
constexpr int kMaxBloomLog2 = 22;          // bloom_shift >= 10
// keyed blooms of more than this many bytes take the line layout (every
// length >= 4 of a position in one 64-B line): an XCD's 4 MiB L2 holds half of
// one or less, so lines saved are HBM / Infinity Cache lines; a smaller bloom
// stays L2-resident and keeps one word per key
constexpr uint64_t kKbLineBytes = 2ull << 20;

// documents per pack of short documents (count mode, score_pack)
constexpr uint32_t kPackDocs = 4;

// per-wave hit area (u32 words): ordered modes hold 64 verified hits of
// (S + 2) / 2 uint4 each; count mode (3) holds the 64 S u32 per-language
// counters (packing: 64 words for the pack probe's non-candidate stores, then
// kPackDocs blocks of 64 S u16 counters)
constexpr uint32_t hit_area_words(int slices, int mode, bool pack = false) {
    return mode == 3 ? (pack ? 64u + 64u * (kPackDocs / 2u) * (uint32_t)slices : 64u * (uint32_t)slices)
                     : 64u * 4u * (((uint32_t)slices + 2u) / 2u);
}

// bytes of dynamic LDS the score kernel needs; image_words = the filter image
// staged in LDS (bitmaps, the bloom when it fits, direct tables)
inline size_t score_lds_bytes(int slices, int mode, uint32_t image_words, bool pack = false) {
    return (size_t)image_words * 4u + (size_t)kScoreWaves * (kQueueCap * 4u + hit_area_words(slices, mode, pack) * 4u +
                                                              2u * kBufWords * 4u + 64u * 4u);
}

// slices = ceil(L / 64); mode 0 = mask rows, 1 = mask rows with finite values
// (fma accumulate), 2 = dense fp64 rows, 3 = mask rows sharing one finite
// value (per-language hit counts); lds_bloom = bloom staged in LDS
hipError_t launch_score(const ScoreParams& p, int slices, int mode, bool lds_bloom, int grid, hipStream_t stream);
// label[i] = the first block maximum over nb language blocks (block b's
// labels / maxima at lab + b n, best + b n)
hipError_t launch_combine_blocks(int64_t n, int nb, const int32_t* lab, const double* best, int32_t* out,
                                 hipStream_t stream);
// sets the dynamic-LDS limit and returns the resident workgroups per CU
hipError_t score_prepare(int slices, int mode, bool lds_bloom, size_t lds_bytes, int* blocks_per_cu);

// -------------------------------------------------------------------- FIT
struct CountParams {
    const uint8_t* bytes;       // 4-byte aligned
    int64_t last_dword;
    const int64_t* offsets;
    const int32_t* doc_lang;
    int64_t n_docs;
    uint64_t* keys;             // [cap] gram keys (0 = empty)
    unsigned long long* counts; // [cap][L]
    uint32_t shift;             // slot = mix64(key) >> shift
    uint64_t mask;              // cap - 1
    unsigned long long* size;   // distinct keys inserted
    uint64_t* ovf_keys;         // overflow (probe limit reached): key, lang, count
    int32_t* ovf_lang;
    unsigned long long* ovf_cnt;
    unsigned int* ovf_n;
    uint32_t ovf_cap;
    uint32_t max_probe;         // probe limit of an insert (kMaxProbe; re-inserts of overflow entries: more)
    int32_t L;
    int32_t nG;
    int32_t G[kMaxGramLengths];
};

constexpr int kCountWaves = 16;
constexpr uint32_t kMaxProbe = 128;
constexpr uint32_t kReinsertProbe = 1u << 16;

hipError_t launch_count(const CountParams& p, int grid, hipStream_t stream);
// insert keys[i] with counts rows[i][L] (add) into the table; n entries
hipError_t launch_counts_add(const CountParams& p, const uint64_t* keys, const unsigned long long* rows,
                             const int32_t* lang_of /*nullable: row is one count cnt_of[i] at lang_of[i]*/,
                             const unsigned long long* cnt_of, int64_t n, hipStream_t stream);

// ---- FIT v3: language-grouped LDS aggregation + radix-partitioned record
// aggregation (ldgpu_count.hip) -- every gram length, every language count.
// A window that no workgroup table absorbs (or a table entry at the end of a
// workgroup's documents) becomes one record of K u64 words:
//   K = 1 (compact; 8 max(G) + 1 + lb + cb <= 64 with cb >= 8):
//        ((sentinel << lb | lang) << cb) | count, sentinel = 1 << 8 klen | bytes
//   K = 2 (grams of <= 7 bytes, any L): {packed key (ldgpu_common.h),
//        lang << 52 | count}
//   K = 3 (some gram length of 8..15 bytes): {lo, hi, lang << 52 | count};
//        a key of <= 7 bytes is lo = its packed key, hi = 0, a wide key is
//        lo = bytes 0..7, hi = bytes 8.. | klen << 56
// h = route hash of the (gram, language) pair: q1 = h >> 58, q2 = bits
// 52..57 (4096 buckets), LDS slot = low 32 bits (reduce).
constexpr int kQBits = 6;
constexpr int kQ = 1 << kQBits;                 // buckets per level
constexpr int kBlkWords = 6144;                 // u64 words of records per emit block (LDS, 48 KiB)
constexpr int kHdr = 68;                        // u32 per block header (kQ + 1 used)
constexpr int kEmitWaves = 16;
constexpr int kSplits = 4;                      // emit workgroup groups (part2 inputs)
constexpr int kT23 = 8192;                      // emit: workgroup LDS table of 2- and 3-byte grams
constexpr uint64_t kCntBits = 52;               // K >= 2: count bits of the last record word
// emit rounds: a wave step adds at most 64 x sub records (sub = 4 positions per
// lane for K = 1, 1 otherwise); a block is flushed once it could not take
// another round
constexpr int emit_sub(int K) { return K == 1 ? 4 : 1; }
constexpr int emit_blk_recs(int K) { return kBlkWords / K; }
constexpr int emit_round_recs(int K) { return kEmitWaves * 64 * emit_sub(K); }

struct PartParams {
    // corpus of the batch
    const uint8_t* bytes;
    int64_t last_dword;
    const int64_t* offsets;
    const int32_t* doc_lang;
    int32_t L;
    int32_t nG;
    int32_t G[kMaxGramLengths];
    uint32_t lb, cb;            // K = 1: language / count bit widths of a record
    int32_t ablate;             // diagnostics build only (LDGPU_FIT_EMIT_ABLATE; compiled out otherwise):
                                // bit 0 2-/3-byte windows skip the workgroup table (records instead),
                                // bit 1 the block flush skips its global stores, bit 2 no records at all
    // emit (phase A): the batch's documents in language order (perm, a
    // permutation of 0 .. n-1); workgroup w owns perm[wg_doc[w] .. wg_doc[w+1]),
    // all of language wg_lang[w], records [wg_rec[w], ...) (capacity: its
    // windows) and block ids [wg_dir[w], ...); blocks are sorted by q1 with a
    // kHdr header
    int32_t grid_a;             // emit workgroups (a multiple of kSplits)
    const int32_t* perm;
    const int32_t* wg_lang;
    const int64_t* wg_doc;
    const int64_t* wg_rec;
    const int64_t* wg_dir;
    uint64_t* rec;              // K words per record
    int64_t* blk_start;         // [blocks] record offset of the block
    uint32_t* blk_hdr;          // [blocks][kHdr] exclusive q1 starts (+ total)
    int32_t* nblk;              // [grid_a] blocks written
    uint32_t* cnt3;             // [kQ][kQ][kSplits] records per (q1, q2, emit group)
    CountParams direct;         // global table: K = 1 counts too large for a record
    // part2: q1 bucket of emit group s -> q2 sub-buckets at exact offsets
    const uint64_t* p2off;      // [kQ][kQ][kSplits]
    uint64_t* rec2;             // K words per record
    // reduce: bucket (q1, q2) = rec2[boff[b] .. boff[b+1]) -> (key, count)
    // entries at out[boff[b] ..] (at most one per record; equal keys summed
    // as far as the LDS hash holds them), nout[b] of them
    const uint64_t* boff;       // [kQ * kQ + 1]
    uint64_t* out;              // K words per entry (the record form, the count field a batch sum)
    uint32_t* nout;             // [kQ * kQ]
    const uint64_t* epre;       // merge: exclusive prefix of nout [kQ * kQ + 1]
};

size_t emit_lds_bytes(int K);
size_t reduce_lds_bytes(int K);
hipError_t fit3_prepare(int K);
hipError_t launch_emit(int K, const PartParams& p, hipStream_t stream);
hipError_t launch_part2(int K, const PartParams& p, hipStream_t stream);
hipError_t launch_reduce(int K, const PartParams& p, hipStream_t stream);
struct WideCountParams;
// add the reduce output entries e0 .. e0 + n into the global tables (K = 3:
// keys of 8..15 bytes into the wide table)
hipError_t launch_merge(int K, const PartParams& p, const CountParams& c, const WideCountParams& w, int64_t e0,
                        int64_t n, hipStream_t stream);
// rehash all occupied slots of `from` into `to` (keys unique), moving the count rows
hipError_t launch_rehash(const CountParams& from, const CountParams& to, uint64_t from_cap,
                         hipStream_t stream);
// out[0] += distinct (gram, language) pairs, out[1] += sum of all counts
hipError_t launch_stats(const CountParams& p, uint64_t cap, unsigned long long* out, hipStream_t stream);
// compact occupied slots: out_keys[i], out_counts[i][L]; *out_n = number written
hipError_t launch_compact(const CountParams& p, uint64_t cap, uint64_t* out_keys,
                          unsigned long long* out_counts, unsigned long long* out_n, hipStream_t stream);

// ---- FIT of gram lengths 8..15 (ldgpu_fit.hip): a table of two-word keys
// (lo = bytes 0..7, hi = bytes 8.. | klen << 56; hi = 0: empty slot) with a
// u64 counter row per slot
struct WideCountParams {
    const uint8_t* bytes;       // 4-byte aligned
    int64_t last_dword;
    const int64_t* offsets;
    const int32_t* doc_lang;
    int64_t n_docs;
    uint64_t* klo;              // [cap]
    uint64_t* khi;              // [cap]
    unsigned long long* counts; // [cap][L]
    uint32_t shift;             // slot = wide_slot(lo, hi) >> shift
    uint64_t mask;              // cap - 1
    unsigned long long* size;   // distinct keys inserted
    unsigned int* full;         // set when an insert found no slot (the host keeps load <= 1/2)
    int32_t L;
    int32_t nG;                 // the wide gram lengths, in gramLengths order
    int32_t G[kMaxGramLengths];
    CountParams narrow;         // partial windows of documents shorter than 8 bytes: one-word keys
};

hipError_t launch_wide_count(const WideCountParams& p, int grid, hipStream_t stream);
hipError_t launch_wide_rehash(const WideCountParams& from, const WideCountParams& to, uint64_t from_cap,
                              hipStream_t stream);
hipError_t launch_wide_add(const WideCountParams& p, const uint64_t* lo, const uint64_t* hi,
                           const unsigned long long* rows, int64_t n, hipStream_t stream);
hipError_t launch_wide_compact(const WideCountParams& p, uint64_t cap, uint64_t* out_lo, uint64_t* out_hi,
                               unsigned long long* out_counts, unsigned long long* out_n, hipStream_t stream);

// ---- device probability / top-K (computeProbabilities + filterTopGrams)
// presence: compact occupied slots into keys[n], masks[n][S] (count > 0 per
// language) and k[n] (= popcount), and histogram hist[l][k] over (gram, l).
hipError_t launch_presence(const CountParams& p, uint64_t cap, int S, uint64_t* out_keys, uint64_t* out_masks,
                           int32_t* out_k, unsigned long long* out_n, unsigned int* hist, hipStream_t stream);
// select: chosen[j] = 1 when k_j < kstar[l] for some l in the gram's mask;
// grams with k_j == kstar[l] (need[l] > 0) are appended as threshold
// candidates (lang, sort key, index).
hipError_t launch_select(int64_t n, int L, int S, const uint64_t* keys, const uint64_t* masks, const int32_t* ks,
                         const int32_t* kstar, const int32_t* need, uint8_t* chosen, int32_t* cand_lang,
                         uint64_t* cand_key, uint32_t* cand_idx, unsigned int* cand_n, hipStream_t stream);
// chosen[idx[i]] = 1
// sorted_keys (nullable): instead of marking, write the candidates' sort keys
// in (language, key) order (the distributed top-K takes each segment's prefix)
hipError_t launch_topk_candidates(int64_t cn, int L, const int32_t* cand_lang, const uint64_t* cand_key,
                                  const uint32_t* cand_idx, const int64_t* seg_start, const int32_t* need,
                                  uint8_t* chosen, uint64_t* sorted_keys, hipStream_t stream);
// chosen[cand_idx[i]] = 1 when cand_key[i] <= thr[cand_lang[i]]
hipError_t launch_mark_threshold(int64_t n, const int32_t* cand_lang, const uint64_t* cand_key,
                                 const uint32_t* cand_idx, const uint64_t* thr, uint8_t* chosen, hipStream_t stream);
// multi-GPU merge: n_of[r] += occupied slots owned by rank r; scatter them
// (keys, count rows) to out at cursor[owner]++
hipError_t launch_owner_count(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* n_of,
                              hipStream_t stream);
hipError_t launch_owner_scatter(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* cursor,
                                uint64_t* out_keys, unsigned long long* out_rows, hipStream_t stream);
// sparse owner exchange: n_of[r] += nonzero (gram, language) pairs owned by
// rank r; scatter them as (key, lang << kPairCntBits | count) to out at
// cursor[owner]++; add such pairs into a table
constexpr uint32_t kPairCntBits = 52;
hipError_t launch_owner_pair_count(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* n_of,
                                   hipStream_t stream);
hipError_t launch_owner_pair_scatter(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* cursor,
                                     uint64_t* out, hipStream_t stream);
hipError_t launch_pairs_add(const CountParams& p, const uint64_t* pairs, int64_t n, hipStream_t stream);
hipError_t launch_mark(const uint32_t* idx, int64_t n, uint8_t* chosen, hipStream_t stream);
// gather the chosen grams: out_keys[m], out_masks[m][S], out_k[m]
hipError_t launch_gather_chosen(int64_t n, int S, const uint8_t* chosen, const uint64_t* keys, const uint64_t* masks,
                                const int32_t* ks, uint64_t* out_keys, uint64_t* out_masks, int32_t* out_k,
                                unsigned long long* out_n, hipStream_t stream);

}  // namespace ldgpu
