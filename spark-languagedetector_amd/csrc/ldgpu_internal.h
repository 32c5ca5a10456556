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
    const Bucket* buckets;      // count mode: bucketed key -> (row, language) table of slot_mask buckets
    uint32_t slot_shift;        // (bucket_index of mix64(key)'s high / low half)
    uint64_t slot_mask;
    uint32_t slot_shift32;      // cuckoo slot = h1 (h2) >> slot_shift32 of slot_hash
    const WideSlot* wslots;     // wide keys (8..15 bytes), nullptr: none
    uint32_t wslot_shift32;     // wide slot = h1 (h2) >> wslot_shift32 of wide_hash
    const uint32_t* filter;     // image: bmp1 | bmp2 | bloom (ldgpu_common.h)
    uint32_t bloom_words;       // power of two
    uint32_t bloom_shift;       // bloom word = hash >> bloom_shift (>= 10)
    int32_t kb_lines;           // keyed bloom in the line layout (kb_line16: blooms beyond kKbLineBytes)
    int32_t kb_chunks;          // count mode: keyed bloom in the chunk layout (kb_chunk; chunk = kb_chunk >> bloom_shift)
    uint32_t len_mask;          // bit k set: the table holds keys of k bytes
    const uint64_t* masks;      // mask mode: [rows][S] language bitmasks
    const double* vals;         // mask mode: [rows] the row's one nonzero value
    const double* rows;         // dense mode: [rows][L]
    const double* fold;         // count mode: fold[c] = c left-folded adds of the value, c <= fold_max
    uint32_t fold_max;
    int32_t count_sign;         // count mode: sign of the value (fold[c] strictly monotone)
    int64_t count_argmax_len;   // count mode: documents up to this length take count_argmax (-1: none)
    // class mode (4, labels only): the table's distinct row values; counters
    // per (class, language); a document whose top two languages are not
    // separated by the rounding bound gets label -1 (exact replay after)
    double cls[4];
    int32_t n_cls;
    uint32_t hit_words;         // class mode: the hit area per wave (64 S n_cls words), sized by the table
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
    // indirect launch (class mode's exact replay, mode 1): document i of the
    // launch is document doc_idx[i] of the corpus, i < *n_docs_dev (a count
    // the device wrote: no readback), its label stored to labels[doc_idx[i]]
    const int64_t* doc_idx;     // nullptr: document i is document i
    const unsigned long long* n_docs_dev;
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

// class mode (4): at most this many distinct row values, so that its
// (class, language) counters fit the ordered modes' hit area (same LDS)
constexpr int class_max(int slices) { return (int)(4u * (((uint32_t)slices + 2u) / 2u) / (uint32_t)slices); }

// bytes of dynamic LDS the score kernel needs; image_words = the filter image
// staged in LDS (bitmaps, the bloom when it fits, direct tables)
// (hit_words: class mode's area, 64 S counters per class; 0 = the mode's)
inline size_t score_lds_bytes(int slices, int mode, uint32_t image_words, bool pack = false, uint32_t hit_words = 0) {
    const uint32_t hw = hit_words ? hit_words : hit_area_words(slices, mode, pack);
    return (size_t)image_words * 4u + (size_t)kScoreWaves * (kQueueCap * 4u + hw * 4u + 2u * kBufWords * 4u + 64u * 4u);
}

// slices = ceil(L / 64); mode 0 = mask rows, 1 = mask rows with finite values
// (fma accumulate), 2 = dense fp64 rows, 3 = mask rows sharing one finite
// value (per-language hit counts), 4 = mask rows of at most class_max(S)
// finite values, labels only (per-(class, language) hit counts and a rounding
// bound; ambiguous documents labelled -1); lds_bloom = bloom staged in LDS
hipError_t launch_score(const ScoreParams& p, int slices, int mode, bool lds_bloom, int grid, hipStream_t stream);
// the per-(mode, slices) entry points behind launch_score / score_prepare
// (ldgpu_score.hip compiled once per pair: launch_score_<mode>_<slices>)
#define LDGPU_SCORE_PAIR_DECL(m, s)                                                                              \
    hipError_t launch_score_##m##_##s(const ScoreParams& p, bool lds_bloom, int grid, hipStream_t stream);        \
    hipError_t prepare_score_##m##_##s(bool lds_bloom, bool chunks, size_t lds, int* blocks);
LDGPU_SCORE_PAIR_DECL(0, 1) LDGPU_SCORE_PAIR_DECL(0, 2) LDGPU_SCORE_PAIR_DECL(0, 3) LDGPU_SCORE_PAIR_DECL(0, 4)
LDGPU_SCORE_PAIR_DECL(1, 1) LDGPU_SCORE_PAIR_DECL(1, 2) LDGPU_SCORE_PAIR_DECL(1, 3) LDGPU_SCORE_PAIR_DECL(1, 4)
LDGPU_SCORE_PAIR_DECL(2, 1) LDGPU_SCORE_PAIR_DECL(2, 2) LDGPU_SCORE_PAIR_DECL(2, 3) LDGPU_SCORE_PAIR_DECL(2, 4)
LDGPU_SCORE_PAIR_DECL(3, 1) LDGPU_SCORE_PAIR_DECL(3, 2) LDGPU_SCORE_PAIR_DECL(3, 3) LDGPU_SCORE_PAIR_DECL(3, 4)
LDGPU_SCORE_PAIR_DECL(4, 1) LDGPU_SCORE_PAIR_DECL(4, 2) LDGPU_SCORE_PAIR_DECL(4, 3) LDGPU_SCORE_PAIR_DECL(4, 4)
#undef LDGPU_SCORE_PAIR_DECL
// class mode's ambiguous documents (ldgpu_replay.hip): idx[0 .. *n_out) = the
// documents labelled -1 (then replayed by an indirect mode-1 launch)
hipError_t launch_amb_compact(const int32_t* labels, int64_t n, int64_t* idx, unsigned long long* n_out,
                              hipStream_t stream);

// General-key scoring (ldgpu_general.hip): models with a gram length beyond
// kMaxWideGram -- keys of any length in one table (GenSlot), compared byte for
// byte against the key arena on a hash match.  One wave per document; the
// reference's loop order (n outer, window position inner), each hit's row
// added in that order by the lanes (language l: lane l mod 64), the scores in
// LDS; the breeze argmax.
struct GenScoreParams {
    const uint8_t* bytes;
    const int64_t* offsets;     // [n_docs + 1]
    int64_t n_docs;
    int32_t* labels;
    double* scores;             // nullable [n_docs][L]
    const GenSlot* slots;
    uint64_t slot_mask;         // slots - 1 (power of two)
    uint32_t slot_shift;        // first slot = h >> slot_shift
    const uint8_t* arena;       // key bytes
    const int64_t* koff;        // [rows + 1] key offsets into the arena
    const uint64_t* masks;      // mask form: [rows][S] (null: dense rows)
    const double* vals;         // mask form: [rows]
    const double* rows;         // dense form: [rows][L]
    int32_t* err;               // bit 0: a window hit a wrong-length row
    int32_t L;
    int32_t nG;
    int32_t G[kMaxGramLengths];
    // indirect launch (mixed tables: the documents the long-gram pass listed):
    // document i of the launch is doc_idx[i], i < *n_docs_dev
    const int64_t* doc_idx;     // nullptr: document i is document i
    const unsigned long long* n_docs_dev;
};
constexpr int kGenWaves = 2;    // waves per workgroup (LDS: 2 x L doubles)
hipError_t launch_general_score(const GenScoreParams& p, int grid, hipStream_t stream);

// Mixed tables (gram lengths beyond kMaxWideGram next to shorter ones): the
// shorter lengths are scored by the LDS-filtered kernels over the keys of <=
// 15 bytes; this pass lists the documents that the longer lengths can hit --
// a window of a long length n whose bits of the long-key prefilter (long_bits)
// are set and which is a key of the general table, or (a document shorter
// than some long n: Scala's partial window) the whole document if it is a key
// -- and those documents are then rescored exactly by the general kernel.
struct LongFlagParams {
    const uint8_t* bytes;       // 4-byte aligned
    const int64_t* offsets;
    int64_t n_docs;
    const uint32_t* bitmap;     // 2^lb bits
    uint32_t lb;
    int32_t n_long;             // distinct long gram lengths
    int32_t Glong[kMaxGramLengths];
    int32_t max_long;
    const GenSlot* slots;       // the general table (every key)
    uint64_t slot_mask;
    uint32_t slot_shift;
    const uint8_t* arena;
    const int64_t* koff;
    int64_t* idx;               // out: listed documents
    unsigned long long* n_out;  // out: their count (zeroed by the caller)
};
hipError_t launch_long_flag(const LongFlagParams& p, int cus, hipStream_t stream);

// label[i] = the first block maximum over nb language blocks (block b's
// labels / maxima at lab + b n, best + b n)
hipError_t launch_combine_blocks(int64_t n, int nb, const int32_t* lab, const double* best, int32_t* out,
                                 hipStream_t stream);
// sets the dynamic-LDS limit and returns the resident workgroups per CU
// (chunks: a count-mode table's keyed bloom in the chunk layout)
hipError_t score_prepare(int slices, int mode, bool lds_bloom, bool chunks, size_t lds_bytes, int* blocks_per_cu);

// ------------------------------------------------------------- PREPROCESS
// The caller-side preprocessors (ldgpu_pre.hip; flags and locale classes:
// LDGPU_PRE_* / LDGPU_LOCALE_* of include/ldgpu.h)
struct PreParams {
    const uint16_t* units;      // UTF-16 code units
    const int64_t* offsets;     // [n_docs + 1], in units
    int64_t n_docs;
    const uint8_t* locale;      // nullable [n_docs]
    int32_t flags;
    const uint16_t* map;        // [65536] 1:1 lower-case unit
    const uint32_t* special;    // [2048] words: units whose document goes to the host
    void* out;                  // units (u16) or, LDGPU_PRE_LOW_BYTES, bytes
    uint8_t* host;              // [n_docs] 1 = redo on the host (empty output)
};
// pass 1 (kept units per document: len_tmp [n_docs + 1]), the scan into
// out_off [n_docs + 1], pass 2 (the output); scan_tmp == nullptr: *scan_bytes =
// the scan's scratch, nothing launched
hipError_t launch_preprocess(const PreParams& p, int64_t* len_tmp, int64_t* out_off, void* scan_tmp, size_t* scan_bytes,
                             int cus, hipStream_t stream);

}  // namespace ldgpu
