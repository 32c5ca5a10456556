// ldgpu_fit.h -- FIT kernel parameter blocks and launchers shared between
// ldgpu_fit.hip and the host runtime (ldgpu_api.hip).  (Kept apart from
// ldgpu_internal.h so the SCORE objects do not depend on it.)
#pragma once

#include "ldgpu_internal.h"

namespace ldgpu {

// -------------------------------------------------------------------- FIT
struct CountParams {
    const uint8_t* bytes;       // 4-byte aligned
    int64_t last_dword;
    const int64_t* offsets;
    const int32_t* doc_lang;
    int64_t n_docs;
    uint64_t* keys;             // [cap] gram keys (0 = empty)
    unsigned long long* counts; // [cap][L]
    uint32_t shift;             // slot = fit_hash(key) >> shift
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

    // Sparse table (the final count table T of ldgpu_counts; pkeys != null,
    // counts == null): the reference's reduceGrams rows (LanguageDetector.
    // scala:57-65) -- one (gram, language) -> count pair per row, not a dense
    // row of L counters per gram.  keys[cap] holds the grams with kcnt[cap],
    // the number of languages each occurs in (its pairs: k of
    // computeProbabilities) MINUS ONE, mod 2^32 (gram_k): the thread that
    // creates a gram and its first pair -- most grams' only one -- adds
    // nothing, every other new pair adds 1, a creator whose pair is not new
    // subtracts 1 (kcnt_delta);
    // the pair table pkeys[pcap] / pcounts[pcap] is keyed (gram slot + 1) << 12 | lang.
    uint32_t* kcnt;
    uint64_t* pkeys;
    unsigned long long* pcounts;
    uint32_t pshift;            // pair slot = fit_hash(pair key) >> pshift
    uint64_t pmask;             // pcap - 1
    unsigned long long* psize;  // distinct pairs inserted
    // pair entry i: key pkeys[i << pinter], count pcounts[i << pinter].  T's
    // pair table interleaves them (pinter 1, pcounts = pkeys + 1: an insert's
    // key claim and count add touch one 64-B line); 0 = separate arrays (the
    // long-gram table's views)
    uint32_t pinter;
};

__host__ __device__ __forceinline__ uint64_t* pkey_at(const CountParams& p, uint64_t i) { return p.pkeys + (i << p.pinter); }
__host__ __device__ __forceinline__ unsigned long long* pcnt_at(const CountParams& p, uint64_t i) {
    return p.pcounts + (i << p.pinter);
}

constexpr uint32_t kPairLangBits = 12;  // pair key: (gram slot + 1) << 12 | lang (L <= 4096)

constexpr int kCountWaves = 16;
constexpr uint32_t kMaxProbe = 128;
constexpr uint32_t kReinsertProbe = 1u << 16;

hipError_t launch_count(const CountParams& p, int grid, hipStream_t stream);
// insert keys[i] with counts rows[i][L] (add) into the table; n entries
hipError_t launch_counts_add(const CountParams& p, const uint64_t* keys, const unsigned long long* rows,
                             const int32_t* lang_of /*nullable: row is one count cnt_of[i] at lang_of[i]*/,
                             const unsigned long long* cnt_of, int64_t n, hipStream_t stream);

// ---- FIT v4: maximal-window records, radix-partitioned record aggregation
// and prefix derivation (ldgpu_fit.hip) -- every gram length, every language
// count.  Every byte position of a document makes ONE record: its maximal
// window, min(N, len - pos) bytes (N = max(G)); the records of a batch are
// summed per (window, language) into a table T1, and T1 derives every gram
// length's counts (the n-gram at a position is the n-byte prefix of its
// maximal window).  A record is K u64 words:
//   K = 1 (compact; 8 max(G) + 1 + lb + cb <= 64 with cb >= 8):
//        ((sentinel << lb | lang) << cb) | count, sentinel = 1 << 8 klen | bytes
//   K = 2 (grams of <= 7 bytes, any L): {packed key (ldgpu_common.h),
//        lang << 52 | count}
//   K = 3 (some gram length of 8..15 bytes): {lo, hi, lang << 52 | count};
//        a key of <= 7 bytes is lo = its packed key, hi = 0, a wide key is
//        lo = bytes 0..7, hi = bytes 8.. | klen << 56
// h = route hash of the (window, language) pair: q1 = h >> 58, q2 = bits
// 52..57 (4096 buckets), LDS slot = low 32 bits (reduce).
constexpr int kQBits = 6;
constexpr int kQ = 1 << kQBits;                 // buckets per level
constexpr int kBlkWords = 6144;                 // u64 words of records per emit block (LDS, 48 KiB)
constexpr int kHdr = 68;                        // u32 per block header (kQ + 1 used)
constexpr int kEmitWaves = 16;
constexpr int kSplits = 8;                      // emit workgroup groups (part2 inputs)
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
    int32_t maxg;               // N = max(G): the maximal window length
    int32_t ablate;             // diagnostics build only (LDGPU_FIT_EMIT_ABLATE; compiled out otherwise):
                                // bit 1 the block flush skips its global stores, bit 2 no records at all
    // emit (phase A): the batch's documents in language order (perm, a
    // permutation of 0 .. n-1); workgroup w owns perm[wg_doc[w] .. wg_doc[w+1]),
    // all of language wg_lang[w], records [wg_rec[w], ...) (capacity: its
    // windows) and block ids [wg_dir[w], ...); blocks are sorted by q1 with a
    // kHdr header
    int32_t grid_a;             // emit workgroups (a multiple of kSplits)
    const int64_t* dstart;      // perm order: each document's first byte (offsets[perm[i]]) ...
    const int32_t* dlen;        // ... and length (> 0): a wave prefetches its next document's without a
                                // dependent load
    const int32_t* wg_lang;
    const int64_t* wg_doc;
    const int64_t* wg_rec;
    const int64_t* wg_dir;
    uint64_t* rec;              // K words per record
    int64_t* blk_start;         // [blocks] record offset of the block
    uint32_t* blk_hdr;          // [blocks][kHdr] exclusive q1 starts (+ total)
    int32_t* nblk;              // [grid_a] blocks written
    uint32_t* cnt3;             // [kQ][kQ][kSplits] records per (q1, q2, emit group)
    // part2: q1 bucket of emit group s -> q2 sub-buckets at exact offsets
    const uint64_t* p2off;      // [kQ][kQ][kSplits]
    uint64_t* rec2;             // K words per record
    // reduce: bucket (q1, q2) = rec2[boff[b] .. boff[b+1]) -> (key, count)
    // entries at out[boff[b] ..] (at most one per record; equal keys summed
    // as far as the LDS hash holds them), nout[b] of them
    const uint64_t* boff;       // [kQ * kQ + 1]
    uint64_t* out;              // K words per entry (the record form, the count field a batch sum)
    uint32_t* nout;             // [kQ * kQ]
};

size_t emit_lds_bytes(int K);
size_t reduce_lds_bytes(int K);
hipError_t fit3_prepare(int K);
hipError_t launch_emit(int K, const PartParams& p, hipStream_t stream);
// p2off / boff from cnt3 on the device (one workgroup)
hipError_t launch_fit_offsets(const PartParams& p, hipStream_t stream);
hipError_t launch_part2(int K, const PartParams& p, hipStream_t stream);
hipError_t launch_reduce(int K, const PartParams& p, hipStream_t stream);
struct WideCountParams;
// add the reduce output entries of buckets b0 .. b1 into the tables of T1
// (K = 3: windows of 8..15 bytes into the wide table)
// (buckets b0 .. b1; pairs: T1 of (window, language) pairs with one counter
// each -- K = 1 keyed by the entries' kl, K = 2 a wide table of (packed key,
// lang + 1))
hipError_t launch_merge(int K, const PartParams& p, const CountParams& c, const WideCountParams& w, int b0, int b1,
                        bool pairs, hipStream_t stream);
// rehash all occupied slots of `from` into `to` (keys unique), moving the count rows
hipError_t launch_rehash(const CountParams& from, const CountParams& to, uint64_t from_cap,
                         hipStream_t stream);
// sparse table: grams of `from` into `to` with their presence masks,
// remap[old slot] = new slot; then every pair of `from` into the pair table of
// `to` (gram slots through remap, or kept when remap is null)
hipError_t launch_sparse_rehash(const CountParams& from, const CountParams& to, uint64_t from_cap, uint64_t* remap,
                                hipStream_t stream);
hipError_t launch_pair_rehash(const CountParams& from, const CountParams& to, uint64_t from_pcap,
                              const uint64_t* remap, hipStream_t stream);
// sparse table exports: the grams (out_keys[o], out_slot[o] = gram slot);
// rank_of[slot[r]] = r; every pair as (rank_of[gram] << 12 | lang, count)
// (sort_keys: out_keys holds each gram's sort_key, ldgpu_common.h)
hipError_t launch_gram_compact(const CountParams& p, uint64_t cap, uint64_t* out_keys, uint64_t* out_slot,
                               unsigned long long* out_n, bool sort_keys, hipStream_t stream);
hipError_t launch_rank_scatter(int64_t n, const uint64_t* slot, uint32_t* rank_of, hipStream_t stream);
hipError_t launch_pair_compact(const CountParams& p, uint64_t pcap, const uint32_t* rank_of, uint64_t* out_pk,
                               unsigned long long* out_cnt, unsigned long long* out_n, hipStream_t stream);
// every pair's count into dense rows: rows[rank_of[gram]][lang] (rows zeroed by the caller)
hipError_t launch_pair_dense(const CountParams& p, uint64_t pcap, const uint32_t* rank_of, unsigned long long* rows,
                             hipStream_t stream);
// sort (key, value) u64 pairs by the low `bits` bits of the key (hipcub radix;
// scratch allocated and freed here; synchronises `stream`)
hipError_t sort_pairs_u64(int64_t n, uint64_t* keys, unsigned long long* vals, int bits, hipStream_t stream);
// nonzero entries of n u64 counters: *out += them
hipError_t launch_nnz(const unsigned long long* v, int64_t n, unsigned long long* out, hipStream_t stream);
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

// ---- FIT v4: the distinct gram lengths (ascending) and their multiplicity
// in gramLengths (partial windows: partial_kernel)
struct DeriveParams {
    int32_t n;
    int32_t len[kMaxGramLengths];
    uint32_t mult[kMaxGramLengths];
};
// level lev of the derive: T1's entries of lev bytes in slots [s0, s1) of its
// one-word (wide = false) or wide table add mult c to T and c to their
// (lev - 1)-byte prefix (flagged) in T1
hipError_t launch_derive_level(const CountParams& t1, const WideCountParams& t1w, bool wide, uint64_t s0, uint64_t s1,
                               int lev, uint32_t mt, const CountParams& to, const WideCountParams& tow,
                               hipStream_t stream);
// the same for a pair table T1 (K = 1: keys kl, one counter; lb language bits)
// (ablate: diagnostics build only, bit 0 no adds to T, bit 1 no prefix adds)
hipError_t launch_derive_pairs_level(const CountParams& t1, uint32_t lb, uint64_t s0, uint64_t s1, int lev, uint32_t mt,
                                     const CountParams& to, int ablate, hipStream_t stream);
// the same for a two-word pair table T1 (K = 2: wide table, one counter,
// lo = packed key, hi = lang + 1)
// nx.khi != null (split): the prefixes and T1's shorter entries go to nx, the
// next level's T1 (t1w is then read only); else the prefixes go to t1w
hipError_t launch_derive_pairs2_level(const WideCountParams& t1w, uint64_t s0, uint64_t s1, int lev, uint32_t mt,
                                      const CountParams& to, const WideCountParams& nx, int ablate,
                                      hipStream_t stream);
// out[t] += occupied T1 slots of t-byte keys (16 counters); pairs: 0 dense
// T1, 1 one-word pairs (lb language bits), 2 two-word pairs
hipError_t launch_len_hist(const CountParams& t1, const WideCountParams& t1w, int pairs, uint32_t lb,
                           unsigned long long* out, hipStream_t stream);
// partial windows of docs[0 .. n) (documents shorter than some gram length)
hipError_t launch_partial(const uint8_t* bytes, const int64_t* offsets, const int32_t* doc_lang, const int64_t* docs,
                          int64_t n_docs, const CountParams& to, const WideCountParams& tow, const DeriveParams& d,
                          hipStream_t stream);

// ---- FIT v5 (ldgpu_fit.hip, count_launch_sorted in ldgpu_api.hip): tables
// of two-word records (grams of <= 7 bytes with many languages: config 5's
// fit, L = 200, grams 1-7) counted by SORTING instead of through T1.  Every
// byte position whose maximal window is a full N-byte window (N = max(G))
// makes one u64 sort key, lang << 8N | the window's bytes big-endian (first
// byte most significant).  Sorted, the positions of one (language, n-byte
// prefix) form one contiguous run for EVERY n <= N, so one pass per gram
// length finds the batch's (n-gram, language) counts as run lengths
// (LanguageDetector.scala:32-43 counts every window once per n; :57-65 sums
// them per (gram, language)); they go into T as one add each.  The last N - 1
// positions of a document (windows shorter than N) add their grams to T
// directly in the emit.  Positions without a full window and documents of
// unsupported languages hold kSortNone, which sorts after every key: language
// codes stay below 2^lbs - 1, lbs = ceil(log2(L + 1)), 8 N + lbs <= 64.
constexpr uint64_t kSortNone = ~0ull;

struct SortFitParams {
    const uint8_t* bytes;       // 4-byte aligned
    int64_t last_dword;
    const int64_t* offsets;     // the batch's documents [0, n_docs]
    const int32_t* doc_lang;
    int64_t n_docs;
    int64_t base;               // offsets[0]: key i belongs to byte position base + i
    int32_t N;                  // max(G) <= 7
    int32_t L;
    uint64_t* keys;             // [offsets[n_docs] - base]
    DeriveParams d;             // distinct gram lengths (ascending) and multiplicities: the tail adds
};

// keys of every position of the batch; the tail positions' grams into T
hipError_t launch_sort_emit(const SortFitParams& p, const CountParams& to, hipStream_t stream);
// radix sort of n u64 keys by bits [0, bits) (hipcub onesweep) between keys
// and alt; tmp == nullptr: *tmp_bytes = the scratch it needs.  *in_alt: the
// sorted keys are in alt
hipError_t sort_keys_u64(int64_t n, uint64_t* keys, uint64_t* alt, int bits, void* tmp, size_t* tmp_bytes,
                         bool* in_alt, hipStream_t stream);
// the gram lengths of one runs pass (bit n of mask) and their multiplicities
// in gramLengths
struct RunLens {
    uint32_t mask;
    uint32_t mult[kMaxGram + 1];
};
// runs[n] (n = 1..N) += the runs of gram length n in sorted keys[0, R) (one
// pass for every length: a run of length n starts where a key's common prefix
// with the previous key, language included, is shorter than n bytes)
hipError_t launch_runs_count(const uint64_t* keys, int64_t R, int N, unsigned long long* runs, hipStream_t stream);
// the runs of the gram lengths in lens in sorted keys[0, R), read once for
// all of them: one entry per distinct (language, n-byte prefix) -- packed
// key, language, run length x mult -- appended at out_n (block-level
// compaction)
hipError_t launch_sort_runs(const uint64_t* keys, int64_t R, int N, const RunLens& lens, uint64_t* out_key,
                            int32_t* out_lang, unsigned long long* out_cnt, unsigned long long* out_n,
                            hipStream_t stream);
// n (key, language, count) entries into T (sparse or dense), grid-stride:
// one counter update per thread, not per wave and entry
hipError_t launch_runs_add(const CountParams& p, const uint64_t* keys, const int32_t* lang, const unsigned long long* cnt,
                           int64_t n, int cus, hipStream_t stream);

// ---- FIT of gram lengths beyond kMaxWideGram (ldgpu_long.hip): keys of any
// length in a table of their own -- a slot per gram holds the hash of its
// bytes and length (gen_hash, ldgpu_common.h) and where its bytes sit in the
// table's key arena -- with a pair table of (gram slot, language) -> count as
// the sparse T (CountParams).  The host sizes every
// table and the arena for a launch up front, so an insert always finds room.
struct alignas(16) LongSlot {
    uint64_t h;       // gen_hash | 1 (0: empty)
    uint64_t meta;    // arena offset << 24 | length (0: being written)
};
constexpr uint64_t kLongLenBits = 24;  // gram lengths < 2^24

struct LongCountParams {
    LongSlot* slots;
    uint32_t shift;             // slot = h >> shift
    uint64_t mask;              // cap - 1
    unsigned long long* size;   // distinct grams
    uint8_t* arena;             // key bytes
    unsigned long long* arena_n;  // arena bytes used
    uint64_t arena_cap;
    uint64_t* pkeys;            // pair table: (slot + 1) << kPairLangBits | lang
    unsigned long long* pcounts;
    uint32_t pshift;
    uint64_t pmask;
    unsigned long long* psize;
    unsigned int* full;         // set if an insert found no room (never: the host sizes the tables)
    int32_t L;
};

// every window of the long gram lengths d (duplicates: mult) of documents
// [0, n_docs), and the partial window (the whole text) of each document of
// 16 <= len < n, counted for its language
hipError_t launch_long_count(const LongCountParams& p, const uint8_t* bytes, const int64_t* offsets,
                             const int32_t* doc_lang, int64_t n_docs, const DeriveParams& d, hipStream_t stream);
// add n (key, language, count) triples: key i = kbytes[koff[i] .. koff[i + 1])
hipError_t launch_long_add(const LongCountParams& p, const uint8_t* kbytes, const int64_t* koff, const int32_t* lang,
                           const unsigned long long* cnt, int64_t n, hipStream_t stream);
// grow: slots of `from` into `to`, remap[old] = new slot
hipError_t launch_long_rehash(const LongCountParams& from, const LongCountParams& to, uint64_t from_cap,
                              uint64_t* remap, hipStream_t stream);

// ---- top-K over the sparse table's pairs (computeProbabilities +
// filterTopGrams, LanguageDetector.scala:75-132): the grams compacted
// (out_keys[o], out_k[o] = k, rk[slot] = o | k << 32); the (language, k) histogram,
// the selection and the chosen rows' presence masks all from the pairs
// rk[g] = row | k << 32 of every occupied gram slot g (its compacted row and
// its language count: one 8-B gather per pair in the pair scans below)
hipError_t launch_gram_rows(const CountParams& p, uint64_t cap, uint64_t* out_keys, int32_t* out_k, uint64_t* rk,
                            unsigned long long* out_n, hipStream_t stream);
hipError_t launch_pair_hist(const CountParams& p, uint64_t pcap, int L, const uint64_t* rk, unsigned int* hist, int cus,
                            hipStream_t stream);
// chosen[j] = 1 when the gram is below its language's threshold class; the
// threshold-class pairs (need[l] > 0) appended as candidates (lang, sort key, j);
// lenhist (nullable, [L][16]) += the candidates per (language, key length)
hipError_t launch_pair_select(const CountParams& p, uint64_t pcap, const uint64_t* rk, const uint64_t* keys,
                              const int32_t* kstar, const int32_t* need, uint8_t* chosen, int32_t* cand_lang,
                              uint64_t* cand_key, uint32_t* cand_idx, unsigned int* cand_n, int L,
                              unsigned int* lenhist, hipStream_t stream);
// the length split of the threshold class: candidates shorter than
// thr_len[l] chosen, those of thr_len[l] bytes compacted into out_*, longer
// ones dropped (thr_len[l] = 0: all kept)
hipError_t launch_cand_filter(int64_t n, const int32_t* cand_lang, const uint64_t* cand_key, const uint32_t* cand_idx,
                              const int32_t* thr_len, uint8_t* chosen, int32_t* out_lang, uint64_t* out_key,
                              uint32_t* out_idx, unsigned int* out_n, hipStream_t stream);
// the chosen rows: out_keys[r], out_k[r], outrow[j] = r (0xffffffff: not
// chosen); rows from out_cap on are counted in out_n, not written
hipError_t launch_gather_rows(int64_t n, const uint8_t* chosen, const uint64_t* keys, const int32_t* ks,
                              uint64_t* out_keys, int32_t* out_k, uint32_t* outrow, unsigned long long* out_n,
                              int64_t out_cap, hipStream_t stream);
// the chosen rows in (length, bytes) order: sk[i] = sort_key(keys[i]), idx[i]
// = i (then sort_pairs_u64), and rows r of the permutation gathered
hipError_t launch_sort_keys_of(int64_t n, const uint64_t* keys, uint64_t* sk, unsigned long long* idx,
                               hipStream_t stream);
hipError_t launch_rows_permute(int64_t n, int S, const unsigned long long* idx, const uint64_t* keys, const int32_t* ks,
                               const uint64_t* masks, uint64_t* out_keys, int32_t* out_k, uint64_t* out_masks,
                               hipStream_t stream);
// rk[g]'s row replaced by outrow[row] for every occupied gram slot (then
// launch_pair_masks with outrow null)
hipError_t launch_rows_final(const CountParams& p, uint64_t cap, const uint32_t* outrow, uint64_t* rk,
                             hipStream_t stream);
// presence masks: masks[row][l / 64] |= bit l for every pair, row = outrow[(uint32_t)rk[g]]
// (outrow null: the row itself); masks zeroed by the caller
hipError_t launch_pair_masks(const CountParams& p, uint64_t pcap, const uint64_t* rk, const uint32_t* outrow, int S,
                             uint64_t* masks, hipStream_t stream);

// threshold-class ties: per language the need[l] smallest (length, bytes)
// candidates get chosen[idx] = 1
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

// Slot hash of the FIT count tables (T's grams and pairs, T1's K = 1 pairs) and route
// hash of K = 1 records: one 64-bit multiply (Fibonacci hashing) after a fold
// of the high half into the low one; callers take its TOP bits (slot = h >>
// shift, the records' q1 / q2), or bits 20..51 (reduce's LDS slot), which
// depend on every key bit.  Against mix64 (two multiplies): config 3's count
// 28.6 -> 26.8 ms per GiB (same-box A/B).
#ifndef LDGPU_FIT_FIB
#define LDGPU_FIT_FIB 1
#endif
__device__ __forceinline__ uint64_t fit_hash(uint64_t k) {
    if (LDGPU_FIT_FIB) return (k ^ (k >> 29)) * 0x9E3779B97F4A7C15ull;
    return mix64(k);
}

}  // namespace ldgpu
