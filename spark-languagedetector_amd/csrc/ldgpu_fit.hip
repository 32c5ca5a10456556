// ldgpu_fit.hip -- FIT counting kernels for gfx950.
//
// Semantic target: computeGrams + reduceGrams (LanguageDetector.scala:25-66):
// for every training document (lang, text), for every n in gramLengths (order,
// duplicates included), every window of the Scala sliding(n) over the UTF-8
// bytes (0 < len < n -> the whole text) adds 1 to count(lang, window).
//
// Table: one open-addressed hash table keyed by the packed gram key with a
// row of L u64 counters per slot (keys[cap], counts[cap][L]).  Integer atomics
// are order-independent, so the counts are bit-exact whatever the schedule.
//
// The counting path is FIT v3 (emit / part2 / reduce / merge, end of file:
// language-grouped LDS aggregation and radix-partitioned records, one table
// add per distinct (gram, language) per bucket and batch) for every gram
// length and language count.  The single-pass count_kernel here and the
// wide_count_kernel below are the round-1 atomic kernels, kept for A/B timing
// in diagnostics builds only (LDGPU_FIT_LEGACY).  count_kernel:
// one wave per document, lanes = 64 consecutive window positions of one gram
// length; 1-gram windows aggregated in a per-wave 256-bin LDS histogram, 2-
// and 3-byte keys in a per-wave LDS hash (kH2 slots, flushed after each gram
// length; a key that finds no slot goes global), longer keys straight into
// the global table: find-or-CAS the key (relaxed agent-scope loads,
// device-scope CAS), then one u64 atomic add on the (slot, lang) counter.  An
// insert that exceeds kMaxProbe probes appends (key, lang, count) to an
// overflow list that the host re-inserts after growing the table.  Gram
// lengths 8..15 count in a table of two-word keys of their own (end of file).
#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "ldgpu_fit.h"

namespace ldgpu {

namespace {

__device__ __forceinline__ uint32_t ld_dw(const uint32_t* w, int64_t i, int64_t last) {
    return w[i < last ? i : last];
}

// Block-level compaction: the block's occupied slots of one chunk get
// consecutive output positions from ONE global atomic (a per-wave atomic on
// the one counter serialises ~cap/64 of them at an L2 channel: 12.6 ms of a
// 64M-slot table); returns this thread's output index (valid if occ).
constexpr int kScanThreads = 1024;

// grid of the grid-stride compaction kernels: up to 2048 blocks of kScanThreads
unsigned scan_grid(uint64_t n) {
    return (unsigned)std::min<uint64_t>(2048, std::max<uint64_t>(1, (n + kScanThreads - 1) / kScanThreads));
}

template <typename C = unsigned long long>
__device__ __forceinline__ unsigned long long block_compact(bool occ, C* out_n, unsigned int* wcnt,
                                                            unsigned long long* bbase) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = __ballot(occ);
    if (lane == 0) wcnt[wave] = (unsigned int)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned int acc = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) {
            const unsigned int c = wcnt[w];
            wcnt[w] = acc;
            acc += c;
        }
        *bbase = acc ? (unsigned long long)atomicAdd(out_n, (C)acc) : 0ull;
    }
    __syncthreads();
    const unsigned long long o = *bbase + wcnt[wave] +
                                 __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    __syncthreads();  // wcnt / bbase are reused by the next chunk
    return o;
}

// block_compact for chunks of several items per thread (kScanIpt items,
// kScanThreads apart): bit j of sm flags this thread's item j.  The block's
// flagged items of one chunk get consecutive output positions from ONE global
// atomic, in (item, wave, lane) order -- so each item's writes stay coalesced
// across the wave, as with block_compact; rel[j] + base is item j's index.
// Each chunk costs the block three barriers and the round trip of its atomic
// on the single counter, so the scans over ~1G positions (FIT v5 runs, the
// top-K's pair and gram scans) take kScanIpt items per thread per chunk.
constexpr int kScanIpt = 8;
static_assert(kScanIpt * (kScanThreads / 64) == 128, "block_place scans 2 counters per lane");

template <typename C = unsigned long long>
__device__ __forceinline__ void block_place(uint32_t sm, C* out_n, unsigned int* wcnt, unsigned long long* bbase,
                                            uint32_t (&rel)[kScanIpt], unsigned long long& base) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < kScanIpt; ++j) {
        const uint64_t m = __ballot((sm >> j) & 1u);
        if (lane == 0) wcnt[j * (kScanThreads / 64) + wave] = (unsigned int)__popcll(m);
        rel[j] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    __syncthreads();
    if (wave == 0) {  // exclusive scan of the 128 counters, two per lane
        const uint32_t a = wcnt[2 * lane], b = wcnt[2 * lane + 1], t = a + b;
        uint32_t incl = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        wcnt[2 * lane] = incl - t;
        wcnt[2 * lane + 1] = incl - t + a;
        const uint32_t tot = __shfl(incl, 63);
        if (lane == 0) *bbase = tot ? (unsigned long long)atomicAdd(out_n, (C)tot) : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kScanIpt; ++j) rel[j] += wcnt[j * (kScanThreads / 64) + wave];
    base = *bbase;
    __syncthreads();  // wcnt / bbase are reused by the next chunk
}

// grid of a scan placing kScanIpt items per thread per chunk
unsigned scan_grid_ipt(uint64_t n) { return scan_grid((n + kScanIpt - 1) / kScanIpt); }

// FIT v4 derive: flag of the prefix aggregates a level adds to T1 (never a
// key bit: klen <= 15 in bits 56..59; pair keys use <= 57 bits)
constexpr uint64_t kDerived = 1ull << 62;

// the packed key (ldgpu_common.h) of a K = 1 record's kl = record >> cb
__device__ __forceinline__ uint64_t kl_key(uint64_t kl, uint32_t lb) {
    const uint64_t sent = kl >> lb;
    const int klen = (63 - __builtin_clzll(sent)) >> 3;
    return (sent ^ (1ull << (8 * klen))) | ((uint64_t)klen << 56);
}

// find-or-insert; returns the slot or -1 when the probe limit is reached.
// PRE: k0 is keys[s] already loaded by the caller (the first probes of a
// thread's several inserts issued together: one memory round trip for all of
// them).  A stale k0 is harmless: keys are never removed, an empty one is
// claimed by CAS (whose result decides), and another key stays there.
template <bool PRE = false>
__device__ __forceinline__ int64_t find_or_insert_at(const CountParams& p, uint64_t key, uint64_t s, uint64_t k0,
                                                     bool& new_key) {
    for (uint32_t probe = 0; probe < p.max_probe; ++probe) {
        uint64_t k = (PRE && probe == 0) ? k0 : __hip_atomic_load(&p.keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return (int64_t)s;
        if (k == kEmpty) {
            const unsigned long long old =
                atomicCAS(reinterpret_cast<unsigned long long*>(&p.keys[s]), 0ull, (unsigned long long)key);
            if (old == 0ull) {
                new_key = true;
                return (int64_t)s;
            }
            if (old == key) return (int64_t)s;
        }
        s = (s + 1) & p.mask;
    }
    return -1;
}

__device__ __forceinline__ int64_t find_or_insert(const CountParams& p, uint64_t key, bool& new_key) {
    return find_or_insert_at<false>(p, key, fit_hash(key) >> p.shift, 0ull, new_key);
}

// the table's distinct-key counter: one atomic per ballot of the lanes calling
// together (a single same-address atomic per new key would serialise)
__device__ __forceinline__ void count_new_keys(const CountParams& p, bool new_key) {
    const uint64_t m = __ballot(new_key);
    if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd(p.size, (unsigned long long)__popcll(m));
}

// Diagnostics build only (tools/build_variant.sh ... -DLDGPU_FIT_ABLATE=n):
// bit 0 skips the counter add, bit 1 skips the whole global update, bit 2
// adds 32-bit instead of 64-bit (timing only).
#ifndef LDGPU_FIT_ABLATE
#define LDGPU_FIT_ABLATE 0
#endif

// The table's distinct-key counter, for kernels whose threads make many
// inserts: each thread counts its new keys and the wave adds them with ONE
// atomic when the thread is done (every lane of the wave must call it) --
// one atomic per insert ballot on the single counter serialises at its L2
// channel (~1M atomics in a 60M-key derive level).
__device__ __forceinline__ void flush_new_keys(unsigned long long* size, unsigned int n) {
    unsigned int v = n;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(size, (unsigned long long)v);
}

// Sparse table T (CountParams::pkeys): find-or-insert of a pair key in the
// pair table; the slot or -1 at the probe limit
template <bool PRE = false>
__device__ __forceinline__ int64_t pair_find_or_insert_at(const CountParams& p, uint64_t pk, uint64_t s, uint64_t k0,
                                                          bool& new_pair) {
    for (uint32_t probe = 0; probe < p.max_probe; ++probe) {
        uint64_t k = (PRE && probe == 0) ? k0 : __hip_atomic_load(pkey_at(p, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == pk) return (int64_t)s;
        if (k == kEmpty) {
            const unsigned long long old =
                atomicCAS(reinterpret_cast<unsigned long long*>(pkey_at(p, s)), 0ull, (unsigned long long)pk);
            if (old == 0ull) {
                new_pair = true;
                return (int64_t)s;
            }
            if (old == pk) return (int64_t)s;
        }
        s = (s + 1) & p.pmask;
    }
    return -1;
}

__device__ __forceinline__ int64_t pair_find_or_insert(const CountParams& p, uint64_t pk, bool& new_pair) {
    return pair_find_or_insert_at<false>(p, pk, fit_hash(pk) >> p.pshift, 0ull, new_pair);
}

// kcnt (ldgpu_fit.h) of one add: +1 for a new pair, -1 for a new gram (its
// creator's pair is counted by the encoding) -- 0, no atomic, for the usual
// new gram with its new pair
__device__ __forceinline__ void kcnt_delta(const CountParams& p, int64_t g, bool new_gram, bool new_pair) {
    const int d = (int)new_pair - (int)new_gram;
    if (g >= 0 && d) atomicAdd(&p.kcnt[g], (uint32_t)d);
}

// the language count k of the gram at occupied slot g
__device__ __forceinline__ int gram_k(const CountParams& p, uint64_t g) { return (int)(p.kcnt[g] + 1u); }

// c of (key, lang) into the sparse table: the gram's slot (its language
// count up when the pair is new), then the pair's counter.  An add that reaches a
// probe limit in either table goes to the overflow list as (key, lang, c) --
// re-adding it finds the gram if it was placed.  A zero count adds nothing
// (a reduceGrams row has count >= 1).  Returns new gram | new pair << 32.
// UNIQ: no other thread of the launch adds this (key, lang) (FIT v5's run
// entries: one per (gram, language) per launch), so a pair this thread
// claimed takes its count by a plain store, not an atomic add.
template <bool UNIQ = false>
__device__ __forceinline__ uint64_t sparse_add_q(const CountParams& p, uint64_t key, int lang, unsigned long long c) {
    if (!c) return 0;
    bool new_gram = false, new_pair = false;
    const int64_t g = find_or_insert(p, key, new_gram);
    int64_t s = -1;
    if (g >= 0) {
        s = pair_find_or_insert(p, ((uint64_t)(g + 1) << kPairLangBits) | (uint64_t)lang, new_pair);
        if (s >= 0) {
            if (UNIQ && new_pair) *pcnt_at(p, s) = c;
            else atomicAdd(pcnt_at(p, s), c);
        }
        kcnt_delta(p, g, new_gram, new_pair);
    }
    if (s < 0) {
        const unsigned int at = atomicAdd(p.ovf_n, 1u);
        if (at < p.ovf_cap) {
            p.ovf_keys[at] = key;
            p.ovf_lang[at] = lang;
            p.ovf_cnt[at] = c;
        }
    }
    return (uint64_t)new_gram | ((uint64_t)new_pair << 32);
}

// c into (slot sl, lang) of a count table, or (sl < 0: probe limit) into the
// overflow list
__device__ __forceinline__ void count_add_slot(const CountParams& p, int64_t sl, uint64_t key, int lang,
                                               unsigned long long c) {
    if (sl >= 0) {
        atomicAdd(&p.counts[(size_t)sl * p.L + lang], c);
        return;
    }
    const unsigned int at = atomicAdd(p.ovf_n, 1u);
    if (at < p.ovf_cap) {
        p.ovf_keys[at] = key;
        p.ovf_lang[at] = lang;
        p.ovf_cnt[at] = c;
    }
}

// add_count without the counter update: returns whether the key is new
__device__ __forceinline__ bool add_count_q(const CountParams& p, uint64_t key, int lang, unsigned long long c) {
    bool new_key = false;
    const int64_t s = find_or_insert(p, key, new_key);
    if (s >= 0) {
        atomicAdd(&p.counts[(size_t)s * p.L + lang], c);
    } else {
        const unsigned int at = atomicAdd(p.ovf_n, 1u);
        if (at < p.ovf_cap) {
            p.ovf_keys[at] = key;
            p.ovf_lang[at] = lang;
            p.ovf_cnt[at] = c;
        }
    }
    return new_key;
}

// an add into T (sparse) or a dense table without the counter updates: new
// keys | new pairs << 32 (t_flush adds them up)
template <bool UNIQ = false>
__device__ __forceinline__ uint64_t t_add_q(const CountParams& p, uint64_t key, int lang, unsigned long long c) {
    if (p.pkeys) return sparse_add_q<UNIQ>(p, key, lang, c);
    return add_count_q(p, key, lang, c) ? 1ull : 0ull;
}

// a thread's t_add_q results into the table's counters (every lane of the wave calls it)
__device__ __forceinline__ void t_flush(const CountParams& p, uint64_t n) {
    flush_new_keys(p.size, (unsigned int)n);
    if (p.pkeys) flush_new_keys(p.psize, (unsigned int)(n >> 32));
}

__device__ __forceinline__ void add_count(const CountParams& p, uint64_t key, int lang, unsigned long long c) {
    if (LDGPU_FIT_ABLATE & 2) return;
    if (p.pkeys) {  // sparse T: one atomic per ballot on each counter
        const uint64_t r = sparse_add_q(p, key, lang, c);
        const uint64_t mg = __ballot(r & 1ull), mp = __ballot(r >> 32);
        const uint32_t lane = threadIdx.x & 63;
        if (mg && lane == (uint32_t)__builtin_ctzll(mg)) atomicAdd(p.size, (unsigned long long)__popcll(mg));
        if (mp && lane == (uint32_t)__builtin_ctzll(mp)) atomicAdd(p.psize, (unsigned long long)__popcll(mp));
        return;
    }
    bool new_key = false;
    const int64_t s = find_or_insert(p, key, new_key);
    count_new_keys(p, new_key);
    if (s >= 0) {
        if (LDGPU_FIT_ABLATE & 4)  // timing probe: a 32-bit add on the counter's low word
            atomicAdd(reinterpret_cast<unsigned int*>(&p.counts[(size_t)s * p.L + lang]), (unsigned int)c);
        else if (!(LDGPU_FIT_ABLATE & 1))
            atomicAdd(&p.counts[(size_t)s * p.L + lang], c);
    } else {
        // overflow (probe limit): the host grows the table and re-adds the entry
        const unsigned int at = atomicAdd(p.ovf_n, 1u);
        if (at < p.ovf_cap) {
            p.ovf_keys[at] = key;
            p.ovf_lang[at] = lang;
            p.ovf_cnt[at] = c;
        }
    }
}

// per-wave LDS aggregation of a document's 2- and 3-byte keys (one language
// per document): open-addressed, kH2 slots, tag = bytes | length << 24 (0 = empty)
constexpr uint32_t kH2 = 384;
constexpr int kH2Probe = 8;

__global__ __launch_bounds__(kCountWaves * 64) void count_kernel(const CountParams p) {
    __shared__ unsigned int hist[kCountWaves][256];
    __shared__ unsigned int tag2[kCountWaves][kH2];
    __shared__ unsigned int cnt2[kCountWaves][kH2];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned int* h1 = hist[wave];
    unsigned int* k2 = tag2[wave];
    unsigned int* c2 = cnt2[wave];
    for (int i = lane; i < 256; i += 64) h1[i] = 0u;
    for (int i = lane; i < (int)kH2; i += 64) k2[i] = c2[i] = 0u;
    const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
    const int64_t stride = (int64_t)gridDim.x * kCountWaves;
    for (int64_t doc = (int64_t)blockIdx.x * kCountWaves + wave; doc < p.n_docs; doc += stride) {
        const int lang = p.doc_lang[doc];
        if (lang < 0 || lang >= p.L) continue;
        const int64_t b = p.offsets[doc];
        const int64_t len = p.offsets[doc + 1] - b;
        bool used_hist = false, used2 = false;
        for (int gi = 0; gi < p.nG; ++gi) {
            const int n = p.G[gi];
            const int64_t nwin = n_windows(len, n);
            const int klen = len < n ? (int)len : n;
            const uint32_t lomask = klen >= 4 ? 0xffffffffu : ((1u << (8 * klen)) - 1u);
            const uint32_t himask = klen <= 4 ? 0u : ((1u << (8 * (klen - 4))) - 1u);
            const uint32_t hitag = (uint32_t)klen << 24;
            for (int64_t p0 = 0; p0 < nwin; p0 += 64) {
                const int64_t pos = p0 + lane;
                if (pos >= nwin) continue;
                const int64_t a = b + pos;
                const int64_t i = a >> 2;
                const uint32_t sh = (uint32_t)(a & 3);
                const uint32_t w0 = ld_dw(W, i, p.last_dword);
                const uint32_t w1 = ld_dw(W, i + 1, p.last_dword);
                const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh) & lomask;
                if (klen == 1) {
                    atomicAdd(&h1[lo], 1u);
                    used_hist = true;
                    continue;
                }
                if (klen == 2 || klen == 3) {
                    const uint32_t tag = lo | ((uint32_t)klen << 24);  // never 0
                    uint32_t slot = (uint32_t)(((uint64_t)(lo * 0x9E3779B1u) * kH2) >> 32);
                    bool done = false;
                    for (int t = 0; t < kH2Probe; ++t) {
                        const unsigned int old = atomicCAS(&k2[slot], 0u, tag);
                        if (old == 0u || old == tag) {
                            atomicAdd(&c2[slot], 1u);
                            done = true;
                            break;
                        }
                        slot = slot + 1u == kH2 ? 0u : slot + 1u;
                    }
                    used2 = true;
                    if (done) continue;
                }
                uint32_t hi = hitag;
                if (klen > 4) {
                    const uint32_t w2 = ld_dw(W, i + 2, p.last_dword);
                    hi |= __builtin_amdgcn_alignbyte(w2, w1, sh) & himask;
                }
                add_count(p, ((uint64_t)hi << 32) | lo, lang, 1ull);
            }
            if (__ballot(used2)) {  // flush this length's LDS-aggregated keys
                used2 = false;
                __builtin_amdgcn_wave_barrier();
                for (int i = lane; i < (int)kH2; i += 64) {
                    const unsigned int tag = k2[i];
                    if (tag) {
                        const unsigned int c = c2[i];
                        k2[i] = 0u;
                        c2[i] = 0u;
                        add_count(p, ((uint64_t)(tag >> 24) << 56) | (uint64_t)(tag & 0xffffffu), lang,
                                  (unsigned long long)c);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (__ballot(used_hist)) {
            __builtin_amdgcn_wave_barrier();
            for (int i = lane; i < 256; i += 64) {
                const unsigned int c = h1[i];
                if (c) {
                    h1[i] = 0u;
                    add_count(p, ((uint64_t)1 << 56) | (uint64_t)i, lang, (unsigned long long)c);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

__global__ void counts_add_kernel(const CountParams p, const uint64_t* keys, const unsigned long long* rows,
                                  const int32_t* lang_of, const unsigned long long* cnt_of, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (p.pkeys) {  // sparse T: every nonzero (key, language, count) as one add (overflow: the list)
        if (lang_of) {
            add_count(p, keys[i], lang_of[i], cnt_of ? cnt_of[i] : 1ull);
        } else {
            uint64_t r = 0;
            for (int l = 0; l < p.L; ++l) r += sparse_add_q(p, keys[i], l, rows[(size_t)i * p.L + l]);
            if (r & 0xffffffffull) atomicAdd(p.size, (unsigned long long)(r & 0xffffffffull));
            if (r >> 32) atomicAdd(p.psize, (unsigned long long)(r >> 32));
        }
        return;
    }
    bool new_key = false;
    const int64_t s = find_or_insert(p, keys[i], new_key);
    count_new_keys(p, new_key);
    if (s < 0) {
        // no slot: entries of the (key, language, count) form go to the
        // overflow list (re-inserted after a grow, after_batch); a row form
        // entry is reported as table full
        const unsigned int at = atomicAdd(p.ovf_n, 1u);
        if (lang_of && at < p.ovf_cap) {
            p.ovf_keys[at] = keys[i];
            p.ovf_lang[at] = lang_of[i];
            p.ovf_cnt[at] = cnt_of ? cnt_of[i] : 1ull;
        }
        return;
    }
    if (lang_of) {
        atomicAdd(&p.counts[(size_t)s * p.L + lang_of[i]], cnt_of ? cnt_of[i] : 1ull);
    } else {
        for (int l = 0; l < p.L; ++l) {
            const unsigned long long c = rows[(size_t)i * p.L + l];
            if (c) atomicAdd(&p.counts[(size_t)s * p.L + l], c);
        }
    }
}

// table statistics: [0] distinct (gram, language) pairs, [1] sum of counts
// (grid-stride, one pair of global atomics per block)
__global__ __launch_bounds__(256) void stats_kernel(const CountParams p, uint64_t cap, unsigned long long* out) {
    __shared__ unsigned long long red[2][4];
    unsigned long long pairs = 0, total = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        if (p.pkeys) {  // a pair table
            if (*pkey_at(p, i) == kEmpty) continue;
            const unsigned long long c = *pcnt_at(p, i);
            pairs += c != 0ull;
            total += c;
            continue;
        }
        if (p.keys[i] == kEmpty) continue;
        for (int l = 0; l < p.L; ++l) {
            const unsigned long long c = p.counts[i * p.L + l];
            pairs += c != 0ull;
            total += c;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        pairs += __shfl_xor(pairs, o);
        total += __shfl_xor(total, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = pairs;
        red[1][threadIdx.x >> 6] = total;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        const unsigned long long b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        if (a | b) {
            atomicAdd(&out[0], a);
            atomicAdd(&out[1], b);
        }
    }
}

__global__ void rehash_kernel(const CountParams from, const CountParams to, uint64_t from_cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= from_cap) return;
    const uint64_t key = from.keys[i];
    if (key == kEmpty) return;
    uint64_t s = fit_hash(key) >> to.shift;
    for (;;) {
        const unsigned long long old =
            atomicCAS(reinterpret_cast<unsigned long long*>(&to.keys[s]), 0ull, (unsigned long long)key);
        if (old == 0ull) break;
        s = (s + 1) & to.mask;
    }
    for (int l = 0; l < from.L; ++l) to.counts[(size_t)s * to.L + l] = from.counts[(size_t)i * from.L + l];
}

__global__ __launch_bounds__(kScanThreads) void compact_kernel(const CountParams p, uint64_t cap, uint64_t* out_keys,
                                                               unsigned long long* out_counts,
                                                               unsigned long long* out_n) {
    __shared__ unsigned int wcnt[kScanThreads / 64];
    __shared__ unsigned long long bbase;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kScanThreads; c0 < cap; c0 += (uint64_t)gridDim.x * kScanThreads) {
        const uint64_t i = c0 + threadIdx.x;
        const bool occ = i < cap && p.keys[i] != kEmpty;
        const unsigned long long o = block_compact(occ, out_n, wcnt, &bbase);
        if (!occ) continue;
        out_keys[o] = p.keys[i];
        for (int l = 0; l < p.L; ++l) out_counts[o * p.L + l] = p.counts[i * p.L + l];
    }
}

// ---- sparse table T (CountParams::pkeys): grow, export
__global__ void sparse_rehash_kernel(const CountParams from, const CountParams to, uint64_t from_cap, uint64_t* remap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= from_cap) return;
    const uint64_t key = from.keys[i];
    if (key == kEmpty) return;
    uint64_t s = fit_hash(key) >> to.shift;
    while (atomicCAS(reinterpret_cast<unsigned long long*>(&to.keys[s]), 0ull, (unsigned long long)key) != 0ull)
        s = (s + 1) & to.mask;
    to.kcnt[s] = from.kcnt[i];
    remap[i] = s;
}

__global__ void pair_rehash_kernel(const CountParams from, const CountParams to, uint64_t from_pcap,
                                   const uint64_t* remap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= from_pcap) return;
    uint64_t pk = *pkey_at(from, i);
    if (pk == kEmpty) return;
    if (remap) {
        const uint64_t g = (pk >> kPairLangBits) - 1ull;
        pk = ((remap[g] + 1ull) << kPairLangBits) | (pk & ((1ull << kPairLangBits) - 1ull));
    }
    uint64_t s = fit_hash(pk) >> to.pshift;
    while (atomicCAS(reinterpret_cast<unsigned long long*>(pkey_at(to, s)), 0ull, (unsigned long long)pk) != 0ull)
        s = (s + 1) & to.pmask;
    *pcnt_at(to, s) = *pcnt_at(from, i);
}

__global__ __launch_bounds__(kScanThreads) void gram_compact_kernel(const CountParams p, uint64_t cap,
                                                                    uint64_t* out_keys, uint64_t* out_slot,
                                                                    unsigned long long* out_n, int sort_keys) {
    __shared__ unsigned int wcnt[kScanThreads / 64];
    __shared__ unsigned long long bbase;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kScanThreads; c0 < cap; c0 += (uint64_t)gridDim.x * kScanThreads) {
        const uint64_t i = c0 + threadIdx.x;
        const bool occ = i < cap && p.keys[i] != kEmpty;
        const unsigned long long o = block_compact(occ, out_n, wcnt, &bbase);
        if (!occ) continue;
        out_keys[o] = sort_keys ? sort_key(p.keys[i]) : p.keys[i];
        out_slot[o] = i;
    }
}

__global__ void rank_scatter_kernel(int64_t n, const uint64_t* slot, uint32_t* rank_of) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) rank_of[slot[r]] = (uint32_t)r;
}

__global__ __launch_bounds__(kScanThreads) void pair_compact_kernel(const CountParams p, uint64_t pcap,
                                                                    const uint32_t* rank_of, uint64_t* out_pk,
                                                                    unsigned long long* out_cnt,
                                                                    unsigned long long* out_n) {
    __shared__ unsigned int wcnt[kScanThreads / 64];
    __shared__ unsigned long long bbase;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kScanThreads; c0 < pcap; c0 += (uint64_t)gridDim.x * kScanThreads) {
        const uint64_t i = c0 + threadIdx.x;
        const uint64_t pk = i < pcap ? *pkey_at(p, i) : kEmpty;
        const bool occ = pk != kEmpty;
        const unsigned long long o = block_compact(occ, out_n, wcnt, &bbase);
        if (!occ) continue;
        const uint64_t g = (pk >> kPairLangBits) - 1ull;
        out_pk[o] = ((uint64_t)rank_of[g] << kPairLangBits) | (pk & ((1ull << kPairLangBits) - 1ull));
        out_cnt[o] = *pcnt_at(p, i);
    }
}

__global__ void pair_dense_kernel(const CountParams p, uint64_t pcap, const uint32_t* rank_of,
                                  unsigned long long* rows) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= pcap) return;
    const uint64_t pk = *pkey_at(p, i);
    if (pk == kEmpty) return;
    const uint64_t g = (pk >> kPairLangBits) - 1ull;
    rows[(uint64_t)rank_of[g] * p.L + (pk & ((1ull << kPairLangBits) - 1ull))] = *pcnt_at(p, i);
}

__global__ __launch_bounds__(256) void nnz_kernel(const unsigned long long* v, int64_t n, unsigned long long* out) {
    unsigned long long k = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        k += v[i] != 0ull;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) k += __shfl_xor(k, o);
    if ((threadIdx.x & 63) == 0 && k) atomicAdd(out, k);
}

}  // namespace

hipError_t launch_sparse_rehash(const CountParams& from, const CountParams& to, uint64_t from_cap, uint64_t* remap,
                                hipStream_t stream) {
    if (from_cap == 0) return hipSuccess;
    hipLaunchKernelGGL(sparse_rehash_kernel, dim3((unsigned)((from_cap + 255) / 256)), dim3(256), 0, stream, from, to,
                       from_cap, remap);
    return hipGetLastError();
}

hipError_t launch_pair_rehash(const CountParams& from, const CountParams& to, uint64_t from_pcap,
                              const uint64_t* remap, hipStream_t stream) {
    if (from_pcap == 0) return hipSuccess;
    hipLaunchKernelGGL(pair_rehash_kernel, dim3((unsigned)((from_pcap + 255) / 256)), dim3(256), 0, stream, from, to,
                       from_pcap, remap);
    return hipGetLastError();
}

hipError_t launch_gram_compact(const CountParams& p, uint64_t cap, uint64_t* out_keys, uint64_t* out_slot,
                               unsigned long long* out_n, bool sort_keys, hipStream_t stream) {
    hipLaunchKernelGGL(gram_compact_kernel, dim3(scan_grid(cap)), dim3(kScanThreads), 0, stream, p, cap, out_keys,
                       out_slot, out_n, (int)sort_keys);
    return hipGetLastError();
}

hipError_t launch_rank_scatter(int64_t n, const uint64_t* slot, uint32_t* rank_of, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(rank_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, n, slot, rank_of);
    return hipGetLastError();
}

hipError_t launch_pair_compact(const CountParams& p, uint64_t pcap, const uint32_t* rank_of, uint64_t* out_pk,
                               unsigned long long* out_cnt, unsigned long long* out_n, hipStream_t stream) {
    hipLaunchKernelGGL(pair_compact_kernel, dim3(scan_grid(pcap)), dim3(kScanThreads), 0, stream, p, pcap, rank_of,
                       out_pk, out_cnt, out_n);
    return hipGetLastError();
}

hipError_t launch_pair_dense(const CountParams& p, uint64_t pcap, const uint32_t* rank_of, unsigned long long* rows,
                             hipStream_t stream) {
    if (pcap == 0) return hipSuccess;
    hipLaunchKernelGGL(pair_dense_kernel, dim3((unsigned)((pcap + 255) / 256)), dim3(256), 0, stream, p, pcap, rank_of,
                       rows);
    return hipGetLastError();
}

hipError_t launch_nnz(const unsigned long long* v, int64_t n, unsigned long long* out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(nnz_kernel, dim3(g), dim3(256), 0, stream, v, n, out);
    return hipGetLastError();
}

hipError_t sort_pairs_u64(int64_t n, uint64_t* keys, unsigned long long* vals, int bits, hipStream_t stream) {
    if (n <= 1) return hipSuccess;
    uint64_t* k2 = nullptr;
    unsigned long long* v2 = nullptr;
    void* tmp = nullptr;
    size_t tb = 0;
    hipcub::DoubleBuffer<uint64_t> kb(keys, nullptr);
    hipcub::DoubleBuffer<unsigned long long> vb(vals, nullptr);
    hipError_t e = hipMalloc((void**)&k2, sizeof(uint64_t) * n);
    if (e == hipSuccess) e = hipMalloc((void**)&v2, sizeof(unsigned long long) * n);
    if (e == hipSuccess) {
        kb = hipcub::DoubleBuffer<uint64_t>(keys, k2);
        vb = hipcub::DoubleBuffer<unsigned long long>(vals, v2);
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kb, vb, (int)n, 0, bits, stream);
    }
    if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tb, 16));
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, kb, vb, (int)n, 0, bits, stream);
    if (e == hipSuccess && kb.Current() != keys)
        e = hipMemcpyAsync(keys, kb.Current(), sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess && vb.Current() != vals)
        e = hipMemcpyAsync(vals, vb.Current(), sizeof(unsigned long long) * n, hipMemcpyDeviceToDevice, stream);
    const hipError_t s = hipStreamSynchronize(stream);
    if (e == hipSuccess) e = s;
    for (void* q : {(void*)k2, (void*)v2, tmp})
        if (q) (void)hipFree(q);
    return e;
}

hipError_t launch_count(const CountParams& p, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(count_kernel, dim3(grid), dim3(kCountWaves * 64), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_counts_add(const CountParams& p, const uint64_t* keys, const unsigned long long* rows,
                             const int32_t* lang_of, const unsigned long long* cnt_of, int64_t n,
                             hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(counts_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, p, keys, rows,
                       lang_of, cnt_of, n);
    return hipGetLastError();
}

hipError_t launch_stats(const CountParams& p, uint64_t cap, unsigned long long* out, hipStream_t stream) {
    hipLaunchKernelGGL(stats_kernel, dim3((unsigned)std::min<uint64_t>(4096, (cap + 255) / 256)), dim3(256), 0, stream,
                       p, cap, out);
    return hipGetLastError();
}

hipError_t launch_rehash(const CountParams& from, const CountParams& to, uint64_t from_cap, hipStream_t stream) {
    hipLaunchKernelGGL(rehash_kernel, dim3((unsigned)((from_cap + 255) / 256)), dim3(256), 0, stream, from, to,
                       from_cap);
    return hipGetLastError();
}

hipError_t launch_compact(const CountParams& p, uint64_t cap, uint64_t* out_keys, unsigned long long* out_counts,
                          unsigned long long* out_n, hipStream_t stream) {
    hipLaunchKernelGGL(compact_kernel, dim3(scan_grid(cap)), dim3(kScanThreads), 0, stream, p, cap, out_keys,
                       out_counts, out_n);
    return hipGetLastError();
}

}  // namespace ldgpu

// ---------------------------------------------------------------------------
// Device probability / top-K table (LanguageDetector.scala:75-132).
//
// computeProbabilities gives gram g the row v_l = log(1 + [g in l] / k_g),
// k_g = #languages with g (:85-87), so a row is fully described by the
// language mask of g.  filterTopGrams ranks, per language l, ALL grams by v_l
// descending and keeps K (:113-119); since log(1 + 1/k) falls with k, the
// order is: present grams by k ascending, then absent ones; ties by the
// build's (length, bytes) rule.  From the sparse table's pairs the device
// builds the (language, k) histogram (k kept per gram by the count kernels);
// the host turns it into a threshold class per language; the device flags
// every gram below a threshold and sorts the threshold-class candidates by
// (language, length, bytes), then builds the chosen rows' masks.
namespace ldgpu {
namespace {

__global__ void mark_kernel(const uint32_t* idx, int64_t n, uint8_t* chosen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) chosen[idx[i]] = 1;
}

unsigned grid_of(int64_t n, int b) { return (unsigned)std::max<int64_t>(1, (n + b - 1) / b); }

__global__ void iota_kernel(int64_t n, uint32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)i;
}

__global__ void cand_lang_kernel(int64_t n, const uint32_t* perm, const int32_t* cand_lang, uint32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)cand_lang[perm[i]];
}

// candidates grouped by language, ascending (length, bytes) within a group:
// the first need[l] of group l are language l's picks
__global__ void cand_mark_kernel(int64_t n, const uint32_t* lang_sorted, const uint32_t* perm,
                                 const int64_t* seg_start, const int32_t* need, const uint32_t* cand_idx,
                                 uint8_t* chosen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t l = lang_sorted[i];
    if (i - seg_start[l] < (int64_t)need[l]) chosen[cand_idx[perm[i]]] = 1;
}

// ---- top-K over the sparse table's pairs
__global__ __launch_bounds__(kScanThreads) void gram_rows_kernel(const CountParams p, uint64_t cap, uint64_t* out_keys,
                                                                 int32_t* out_k, uint64_t* rk,
                                                                 unsigned long long* out_n) {
    __shared__ unsigned int wcnt[kScanIpt * (kScanThreads / 64)];
    __shared__ unsigned long long bbase;
    constexpr uint64_t kChunk = (uint64_t)kScanIpt * kScanThreads;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kChunk; c0 < cap; c0 += (uint64_t)gridDim.x * kChunk) {
        uint64_t key[kScanIpt];
        uint32_t om = 0;
#pragma unroll
        for (int j = 0; j < kScanIpt; ++j) {
            const uint64_t i = c0 + (uint64_t)j * kScanThreads + threadIdx.x;
            key[j] = i < cap ? p.keys[i] : kEmpty;
            if (key[j] != kEmpty) om |= 1u << j;
        }
        uint32_t rel[kScanIpt];
        unsigned long long base;
        block_place(om, out_n, wcnt, &bbase, rel, base);
#pragma unroll
        for (int j = 0; j < kScanIpt; ++j) {
            if (!((om >> j) & 1u)) continue;
            const uint64_t i = c0 + (uint64_t)j * kScanThreads + threadIdx.x;
            const unsigned long long o = base + rel[j];
            const uint32_t k = (uint32_t)gram_k(p, i);
            out_keys[o] = key[j];
            out_k[o] = (int32_t)k;
            rk[i] = o | ((uint64_t)k << 32);
        }
    }
}

__device__ __forceinline__ uint32_t pair_lang(uint64_t pk) { return (uint32_t)(pk & ((1ull << kPairLangBits) - 1ull)); }
__device__ __forceinline__ uint64_t pair_slot(uint64_t pk) { return (pk >> kPairLangBits) - 1ull; }

// (language, k) histogram of the pairs, k = the gram's language count (rk
// at its slot: one random 8-B read per pair, kScanIpt in flight per thread).  Classes k <= kl count in LDS
// ([L][kl + 1], kl = L when it fits), the rest -- rare: most grams are in
// few languages -- in global memory; each block flushes its nonzero LDS
// counters once.  (Global atomics on the ~L hot counters of k = 1: 152 ms on
// config 5's 1.39G pairs.)
__global__ __launch_bounds__(kScanThreads) void pair_hist_kernel(const CountParams p, uint64_t pcap, int L, int kl,
                                                                 const uint64_t* rk, unsigned int* hist) {
    extern __shared__ unsigned int lh[];
    const int kw = kl + 1;
    for (int i = threadIdx.x; i < L * kw; i += blockDim.x) lh[i] = 0u;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < pcap; i0 += kScanIpt * stride) {
        uint64_t pk[kScanIpt];
#pragma unroll
        for (int q = 0; q < kScanIpt; ++q) {
            const uint64_t i = i0 + q * stride;
            pk[q] = i < pcap ? *pkey_at(p, i) : kEmpty;
        }
        int k[kScanIpt];
#pragma unroll
        for (int q = 0; q < kScanIpt; ++q) k[q] = pk[q] != kEmpty ? (int)(rk[pair_slot(pk[q])] >> 32) : 0;
#pragma unroll
        for (int q = 0; q < kScanIpt; ++q) {
            if (pk[q] == kEmpty) continue;
            const uint32_t l = pair_lang(pk[q]);
            if (k[q] <= kl) atomicAdd(&lh[l * kw + k[q]], 1u);
            else atomicAdd(&hist[l * (L + 1) + k[q]], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < L * kw; i += blockDim.x) {
        const unsigned int v = lh[i];
        if (v) atomicAdd(&hist[(i / kw) * (L + 1) + i % kw], v);
    }
}

// grid-stride with block-level compaction of the candidates: the threshold
// class can hold most pairs (config 3: nearly every gram is in one language),
// and one counter add per wave serialised ~1M atomics on cand_n (47 ms of a
// 72M-pair table)
// lenhist (nullable): the candidates per (language, key length) ([L][16],
// in LDS, flushed once per block) -- the threshold class's length split
__global__ __launch_bounds__(kScanThreads) void pair_select_kernel(const CountParams p, uint64_t pcap,
                                                                   const uint64_t* rk, const uint64_t* keys,
                                                                   const int32_t* kstar, const int32_t* need,
                                                                   uint8_t* chosen, int32_t* cand_lang,
                                                                   uint64_t* cand_key, uint32_t* cand_idx,
                                                                   unsigned int* cand_n, int L, unsigned int* lenhist) {
    __shared__ unsigned int wcnt[kScanIpt * (kScanThreads / 64)];
    __shared__ unsigned long long bbase;
    extern __shared__ unsigned int lh[];
    if (lenhist) {
        for (int i = threadIdx.x; i < 16 * L; i += blockDim.x) lh[i] = 0u;
        __syncthreads();
    }
    constexpr uint64_t kChunk = (uint64_t)kScanIpt * kScanThreads;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kChunk; c0 < pcap; c0 += (uint64_t)gridDim.x * kChunk) {
        // kScanIpt pairs per thread: their random gram-slot reads in flight together
        uint64_t pk[kScanIpt];
#pragma unroll
        for (int q = 0; q < kScanIpt; ++q) {
            const uint64_t i = c0 + (uint64_t)q * kScanThreads + threadIdx.x;
            pk[q] = i < pcap ? *pkey_at(p, i) : kEmpty;
        }
        uint32_t j[kScanIpt];
        int k[kScanIpt];
#pragma unroll
        for (int q = 0; q < kScanIpt; ++q) {
            j[q] = 0;
            k[q] = 0;
            if (pk[q] != kEmpty) {
                const uint64_t v = rk[pair_slot(pk[q])];
                j[q] = (uint32_t)v;
                k[q] = (int)(v >> 32);
            }
        }
        uint32_t cm = 0;
#pragma unroll
        for (int q = 0; q < kScanIpt; ++q) {
            if (pk[q] == kEmpty) continue;
            const uint32_t l = pair_lang(pk[q]);
            const int ksl = kstar[l];
            if (k[q] < ksl) chosen[j[q]] = 1;
            if (k[q] == ksl && need[l] > 0) cm |= 1u << q;
        }
        uint32_t rel[kScanIpt];
        unsigned long long base;
        block_place<unsigned int>(cm, cand_n, wcnt, &bbase, rel, base);
#pragma unroll
        for (int q = 0; q < kScanIpt; ++q) {
            if (!((cm >> q) & 1u)) continue;
            const unsigned long long at = base + rel[q];
            const uint32_t l = pair_lang(pk[q]);
            const uint64_t sk = sort_key(keys[j[q]]);
            cand_lang[at] = (int32_t)l;
            cand_key[at] = sk;
            cand_idx[at] = j[q];
            if (lenhist) atomicAdd(&lh[16 * l + (int)(sk >> 56)], 1u);
        }
    }
    if (lenhist) {
        __syncthreads();
        for (int i = threadIdx.x; i < 16 * L; i += blockDim.x) {
            const unsigned int v = lh[i];
            if (v) atomicAdd(&lenhist[i], v);
        }
    }
}

// the threshold class's length split (fit_table_device): a candidate of
// language l shorter than thr_len[l] is chosen outright, one of exactly
// thr_len[l] bytes stays a candidate (compacted into out_*), a longer one
// drops out; thr_len[l] = 0 keeps every candidate of l
__global__ __launch_bounds__(kScanThreads) void cand_filter_kernel(int64_t n, const int32_t* cand_lang,
                                                                   const uint64_t* cand_key, const uint32_t* cand_idx,
                                                                   const int32_t* thr_len, uint8_t* chosen,
                                                                   int32_t* out_lang, uint64_t* out_key,
                                                                   uint32_t* out_idx, unsigned int* out_n) {
    __shared__ unsigned int wcnt[kScanThreads / 64];
    __shared__ unsigned long long bbase;
    for (int64_t c0 = (int64_t)blockIdx.x * kScanThreads; c0 < n; c0 += (int64_t)gridDim.x * kScanThreads) {
        const int64_t i = c0 + threadIdx.x;
        bool keep = false;
        int32_t l = 0;
        uint64_t sk = 0;
        if (i < n) {
            l = cand_lang[i];
            sk = cand_key[i];
            const int t = thr_len[l];
            const int len = (int)(sk >> 56);
            keep = t == 0 || len == t;
            if (t && len < t) chosen[cand_idx[i]] = 1;
        }
        const unsigned long long at = block_compact<unsigned int>(keep, out_n, wcnt, &bbase);
        if (!keep) continue;
        out_lang[at] = l;
        out_key[at] = sk;
        out_idx[at] = cand_idx[i];
    }
}

__global__ __launch_bounds__(kScanThreads) void gather_rows_kernel(int64_t n, const uint8_t* chosen,
                                                                   const uint64_t* keys, const int32_t* ks,
                                                                   uint64_t* out_keys, int32_t* out_k,
                                                                   uint32_t* outrow, unsigned long long* out_n,
                                                                   int64_t out_cap) {
    __shared__ unsigned int wcnt[kScanThreads / 64];
    __shared__ unsigned long long bbase;
    for (int64_t c0 = (int64_t)blockIdx.x * kScanThreads; c0 < n; c0 += (int64_t)gridDim.x * kScanThreads) {
        const int64_t j = c0 + threadIdx.x;
        const bool c = j < n && chosen[j];
        const unsigned long long o = block_compact(c, out_n, wcnt, &bbase);
        if (j >= n) continue;
        outrow[j] = c && (int64_t)o < out_cap ? (uint32_t)o : 0xffffffffu;
        if (!c || (int64_t)o >= out_cap) continue;  // more than out_cap: the caller fails
        out_keys[o] = keys[j];
        out_k[o] = ks[j];
    }
}

// rk[g]'s row -> outrow[row] (0xffffffff: not chosen) for every occupied gram
// slot: rows follow slot order, so the outrow reads are near-sequential here,
// and the pair scan after it gathers one word per pair instead of two
__global__ void rows_final_kernel(const CountParams p, uint64_t cap, const uint32_t* outrow, uint64_t* rk) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= cap || p.keys[g] == kEmpty) return;
    const uint64_t v = rk[g];
    rk[g] = (v & ~0xffffffffull) | outrow[(uint32_t)v];
}

__global__ void pair_masks_kernel(const CountParams p, uint64_t pcap, const uint64_t* rk, const uint32_t* outrow,
                                  int S, uint64_t* masks) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= pcap) return;
    const uint64_t pk = *pkey_at(p, i);
    if (pk == kEmpty) return;
    const uint32_t l = pair_lang(pk);
    uint32_t r = (uint32_t)rk[pair_slot(pk)];
    if (outrow) r = outrow[r];
    if (r == 0xffffffffu) return;
    atomicOr(reinterpret_cast<unsigned long long*>(&masks[(size_t)r * S + (l >> 6)]), 1ull << (l & 63));
}

__global__ void sort_keys_of_kernel(int64_t n, const uint64_t* keys, uint64_t* sk, unsigned long long* idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sk[i] = sort_key(keys[i]);
    idx[i] = (unsigned long long)i;
}

__global__ void rows_permute_kernel(int64_t n, int S, const unsigned long long* idx, const uint64_t* keys,
                                    const int32_t* ks, const uint64_t* masks, uint64_t* out_keys, int32_t* out_k,
                                    uint64_t* out_masks) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t i = idx[r];
    out_keys[r] = keys[i];
    out_k[r] = ks[i];
    for (int s = 0; s < S; ++s) out_masks[(size_t)r * S + s] = masks[i * S + s];
}

// ---- multi-GPU merge: owner partition of the table (ldgpu_counts_merge)
__device__ __forceinline__ uint32_t owner_of(uint64_t key, uint32_t world) {
    return (uint32_t)(((mix64(key) & 0xffffffffull) * world) >> 32);
}

__global__ void owner_count_kernel(const CountParams p, uint64_t cap, uint32_t world, unsigned long long* n_of) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap && p.keys[i] != kEmpty) atomicAdd(&n_of[owner_of(p.keys[i], world)], 1ull);
}

__global__ void owner_scatter_kernel(const CountParams p, uint64_t cap, uint32_t world, unsigned long long* cursor,
                                     uint64_t* out_keys, unsigned long long* out_rows) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap || p.keys[i] == kEmpty) return;
    const uint64_t key = p.keys[i];
    const unsigned long long o = atomicAdd(&cursor[owner_of(key, world)], 1ull);
    out_keys[o] = key;
    for (int l = 0; l < p.L; ++l) out_rows[o * p.L + l] = p.counts[i * p.L + l];
}

// sparse exchange (ldgpu_counts_merge): a slot's nonzero (language, count)
// pairs, 16 B each -- (key, lang << 52 | count) -- instead of its dense row of
// L counters (1.3 pairs per gram against L = 20..200 counters on the fit
// corpora)
// (sparse T: cap is the pair table's; one thread per pair)
__device__ __forceinline__ uint64_t pair_gram(const CountParams& p, uint64_t pk) {
    return p.keys[(pk >> kPairLangBits) - 1ull];
}

__global__ void owner_pair_count_kernel(const CountParams p, uint64_t cap, uint32_t world, unsigned long long* n_of) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p.pkeys) {
        if (i < cap && *pkey_at(p, i) != kEmpty) atomicAdd(&n_of[owner_of(pair_gram(p, *pkey_at(p, i)), world)], 1ull);
        return;
    }
    if (i >= cap || p.keys[i] == kEmpty) return;
    unsigned long long k = 0;
    for (int l = 0; l < p.L; ++l) k += p.counts[i * p.L + l] != 0ull;
    if (k) atomicAdd(&n_of[owner_of(p.keys[i], world)], k);
}

__global__ void owner_pair_scatter_kernel(const CountParams p, uint64_t cap, uint32_t world, unsigned long long* cursor,
                                          uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p.pkeys) {
        if (i >= cap || *pkey_at(p, i) == kEmpty) return;
        const uint64_t pk = *pkey_at(p, i), key = pair_gram(p, pk);
        const unsigned long long o = atomicAdd(&cursor[owner_of(key, world)], 1ull);
        out[2 * o] = key;
        out[2 * o + 1] = ((pk & ((1ull << kPairLangBits) - 1ull)) << kPairCntBits) | *pcnt_at(p, i);
        return;
    }
    if (i >= cap || p.keys[i] == kEmpty) return;
    const uint64_t key = p.keys[i];
    const unsigned long long* row = p.counts + i * p.L;
    unsigned long long k = 0;
    for (int l = 0; l < p.L; ++l) k += row[l] != 0ull;
    if (!k) return;
    unsigned long long o = atomicAdd(&cursor[owner_of(key, world)], k);
    for (int l = 0; l < p.L; ++l) {
        if (!row[l]) continue;
        out[2 * o] = key;
        out[2 * o + 1] = ((uint64_t)l << kPairCntBits) | row[l];
        ++o;
    }
}

// add received (key, lang << 52 | count) pairs into the table (probe-limit
// overflows go to the overflow list, re-inserted by the host)
__global__ void pairs_add_kernel(const CountParams p, const uint64_t* pairs, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t v = pairs[2 * i + 1];
    add_count(p, pairs[2 * i], (int)(v >> kPairCntBits), (unsigned long long)(v & ((1ull << kPairCntBits) - 1ull)));
}

// distributed top-K: a candidate is chosen when its (length, bytes) sort key
// is at most its language's global threshold
__global__ void mark_threshold_kernel(int64_t n, const int32_t* cand_lang, const uint64_t* cand_key,
                                      const uint32_t* cand_idx, const uint64_t* thr, uint8_t* chosen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && cand_key[i] <= thr[cand_lang[i]]) chosen[cand_idx[i]] = 1;
}

__global__ void gather_u64_kernel(int64_t n, const uint32_t* idx, const uint64_t* src, uint64_t* dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}

}  // namespace

hipError_t launch_gram_rows(const CountParams& p, uint64_t cap, uint64_t* out_keys, int32_t* out_k, uint64_t* rk,
                            unsigned long long* out_n, hipStream_t stream) {
    hipLaunchKernelGGL(gram_rows_kernel, dim3(scan_grid_ipt(cap)), dim3(kScanThreads), 0, stream, p, cap, out_keys, out_k,
                       rk, out_n);
    return hipGetLastError();
}

hipError_t launch_pair_hist(const CountParams& p, uint64_t pcap, int L, const uint64_t* rk, unsigned int* hist, int cus,
                            hipStream_t stream) {
    if (pcap == 0) return hipSuccess;
    // LDS classes: every k when L (L + 1) counters fit 48 KiB, else as many
    // as fit (at least k = 1)
    const int kl = std::max(1, std::min(L, (int)(12288 / L) - 1));
    const size_t lds = (size_t)L * (kl + 1) * 4;
    const unsigned g = (unsigned)std::min<uint64_t>((uint64_t)cus * 2, (pcap + kScanThreads - 1) / kScanThreads);
    hipLaunchKernelGGL(pair_hist_kernel, dim3(std::max(1u, g)), dim3(kScanThreads), lds, stream, p, pcap, L, kl, rk, hist);
    return hipGetLastError();
}

hipError_t launch_pair_select(const CountParams& p, uint64_t pcap, const uint64_t* rk, const uint64_t* keys,
                              const int32_t* kstar, const int32_t* need, uint8_t* chosen, int32_t* cand_lang,
                              uint64_t* cand_key, uint32_t* cand_idx, unsigned int* cand_n, int L,
                              unsigned int* lenhist, hipStream_t stream) {
    if (pcap == 0) return hipSuccess;
    const size_t lds = lenhist ? (size_t)16 * L * 4 : 0;
    hipLaunchKernelGGL(pair_select_kernel, dim3(scan_grid_ipt(pcap)), dim3(kScanThreads), lds, stream, p, pcap, rk,
                       keys, kstar, need, chosen, cand_lang, cand_key, cand_idx, cand_n, L, lenhist);
    return hipGetLastError();
}

hipError_t launch_cand_filter(int64_t n, const int32_t* cand_lang, const uint64_t* cand_key, const uint32_t* cand_idx,
                              const int32_t* thr_len, uint8_t* chosen, int32_t* out_lang, uint64_t* out_key,
                              uint32_t* out_idx, unsigned int* out_n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cand_filter_kernel, dim3(scan_grid((uint64_t)n)), dim3(kScanThreads), 0, stream, n, cand_lang,
                       cand_key, cand_idx, thr_len, chosen, out_lang, out_key, out_idx, out_n);
    return hipGetLastError();
}

hipError_t launch_gather_rows(int64_t n, const uint8_t* chosen, const uint64_t* keys, const int32_t* ks,
                              uint64_t* out_keys, int32_t* out_k, uint32_t* outrow, unsigned long long* out_n,
                              int64_t out_cap, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(scan_grid((uint64_t)n)), dim3(kScanThreads), 0, stream, n, chosen, keys,
                       ks, out_keys, out_k, outrow, out_n, out_cap);
    return hipGetLastError();
}

hipError_t launch_sort_keys_of(int64_t n, const uint64_t* keys, uint64_t* sk, unsigned long long* idx,
                               hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(sort_keys_of_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, n, keys, sk, idx);
    return hipGetLastError();
}

hipError_t launch_rows_permute(int64_t n, int S, const unsigned long long* idx, const uint64_t* keys, const int32_t* ks,
                               const uint64_t* masks, uint64_t* out_keys, int32_t* out_k, uint64_t* out_masks,
                               hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(rows_permute_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, n, S, idx, keys, ks, masks,
                       out_keys, out_k, out_masks);
    return hipGetLastError();
}

hipError_t launch_rows_final(const CountParams& p, uint64_t cap, const uint32_t* outrow, uint64_t* rk,
                             hipStream_t stream) {
    if (cap == 0) return hipSuccess;
    hipLaunchKernelGGL(rows_final_kernel, dim3(grid_of((int64_t)cap, 256)), dim3(256), 0, stream, p, cap, outrow, rk);
    return hipGetLastError();
}

hipError_t launch_pair_masks(const CountParams& p, uint64_t pcap, const uint64_t* rk, const uint32_t* outrow, int S,
                             uint64_t* masks, hipStream_t stream) {
    if (pcap == 0) return hipSuccess;
    hipLaunchKernelGGL(pair_masks_kernel, dim3(grid_of((int64_t)pcap, 256)), dim3(256), 0, stream, p, pcap, rk,
                       outrow, S, masks);
    return hipGetLastError();
}

hipError_t launch_owner_count(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* n_of,
                              hipStream_t stream) {
    hipLaunchKernelGGL(owner_count_kernel, dim3(grid_of((int64_t)cap, 256)), dim3(256), 0, stream, p, cap, world, n_of);
    return hipGetLastError();
}

hipError_t launch_owner_scatter(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* cursor,
                                uint64_t* out_keys, unsigned long long* out_rows, hipStream_t stream) {
    hipLaunchKernelGGL(owner_scatter_kernel, dim3(grid_of((int64_t)cap, 256)), dim3(256), 0, stream, p, cap, world,
                       cursor, out_keys, out_rows);
    return hipGetLastError();
}

hipError_t launch_owner_pair_count(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* n_of,
                                   hipStream_t stream) {
    hipLaunchKernelGGL(owner_pair_count_kernel, dim3(grid_of((int64_t)cap, 256)), dim3(256), 0, stream, p, cap, world,
                       n_of);
    return hipGetLastError();
}

hipError_t launch_owner_pair_scatter(const CountParams& p, uint64_t cap, uint32_t world, unsigned long long* cursor,
                                     uint64_t* out, hipStream_t stream) {
    hipLaunchKernelGGL(owner_pair_scatter_kernel, dim3(grid_of((int64_t)cap, 256)), dim3(256), 0, stream, p, cap,
                       world, cursor, out);
    return hipGetLastError();
}

hipError_t launch_pairs_add(const CountParams& p, const uint64_t* pairs, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(pairs_add_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, p, pairs, n);
    return hipGetLastError();
}

hipError_t launch_mark_threshold(int64_t n, const int32_t* cand_lang, const uint64_t* cand_key,
                                 const uint32_t* cand_idx, const uint64_t* thr, uint8_t* chosen, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mark_threshold_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, n, cand_lang, cand_key,
                       cand_idx, thr, chosen);
    return hipGetLastError();
}

// Threshold-class tie resolution on the device (filterTopGrams' take(K),
// LanguageDetector.scala:113-119, under the build's (length, bytes) tie rule):
// two stable LSD radix sorts -- by sort_key (59 bits), then by language
// (ceil(log2 L) bits) -- leave each language's candidates contiguous and in
// tie order.
// Sort keys are unique per gram, so this picks exactly the set nth_element
// picked on the host.  Synchronises `stream` before returning (scratch freed).
hipError_t launch_topk_candidates(int64_t cn, int L, const int32_t* cand_lang, const uint64_t* cand_key,
                                  const uint32_t* cand_idx, const int64_t* seg_start, const int32_t* need,
                                  uint8_t* chosen, uint64_t* sorted_keys, hipStream_t stream) {
    if (cn <= 0) return hipSuccess;
    const int n = (int)cn;
    int lbits = 1;
    while ((1 << lbits) < L) ++lbits;
    uint64_t* key_out = nullptr;
    uint32_t *perm_a = nullptr, *perm_b = nullptr, *lang_a = nullptr, *lang_b = nullptr;
    void* tmp = nullptr;
    size_t tmp1 = 0, tmp2 = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp1, cand_key, key_out, perm_a, perm_b, n, 0, 59,
                                                      stream);
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp2, lang_a, lang_b, perm_b, perm_a, n, 0, lbits, stream);
    if (e == hipSuccess) e = hipMalloc((void**)&key_out, sizeof(uint64_t) * cn);
    if (e == hipSuccess) e = hipMalloc((void**)&perm_a, sizeof(uint32_t) * cn);
    if (e == hipSuccess) e = hipMalloc((void**)&perm_b, sizeof(uint32_t) * cn);
    if (e == hipSuccess) e = hipMalloc((void**)&lang_a, sizeof(uint32_t) * cn);
    if (e == hipSuccess) e = hipMalloc((void**)&lang_b, sizeof(uint32_t) * cn);
    if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(std::max(tmp1, tmp2), 16));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(iota_kernel, dim3(grid_of(cn, 256)), dim3(256), 0, stream, cn, perm_a);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp1, cand_key, key_out, perm_a, perm_b, n, 0, 59, stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(cand_lang_kernel, dim3(grid_of(cn, 256)), dim3(256), 0, stream, cn, perm_b, cand_lang,
                           lang_a);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp2, lang_a, lang_b, perm_b, perm_a, n, 0, lbits, stream);
    if (e == hipSuccess && sorted_keys) {  // distributed: each language's sorted candidate keys, no marking
        hipLaunchKernelGGL(gather_u64_kernel, dim3(grid_of(cn, 256)), dim3(256), 0, stream, cn, perm_a, cand_key,
                           sorted_keys);
        e = hipGetLastError();
    } else if (e == hipSuccess) {
        hipLaunchKernelGGL(cand_mark_kernel, dim3(grid_of(cn, 256)), dim3(256), 0, stream, cn, lang_b, perm_a,
                           seg_start, need, cand_idx, chosen);
        e = hipGetLastError();
    }
    const hipError_t s = hipStreamSynchronize(stream);
    if (e == hipSuccess) e = s;
    for (void* q : {(void*)key_out, (void*)perm_a, (void*)perm_b, (void*)lang_a, (void*)lang_b, tmp})
        if (q) (void)hipFree(q);
    return e;
}

hipError_t launch_mark(const uint32_t* idx, int64_t n, uint8_t* chosen, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mark_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, idx, n, chosen);
    return hipGetLastError();
}

}  // namespace ldgpu

// ---------------------------------------------------------------------------
// FIT of gram lengths 8..15 (computeGrams + reduceGrams, LanguageDetector.
// scala:25-66, for windows too long for a one-word key).  Such windows count
// into a table of two-word keys of their own -- lo = bytes 0..7, hi = bytes
// 8.. | klen << 56 (ldgpu_common.h) -- with one u64 counter row per slot, as
// the one-word table.  A wide gram length still makes one-word keys: the
// partial window of a document shorter than 8 bytes (Scala sliding gives the
// whole text), which goes to the one-word table.  One wave per document, a
// lane per window; an insert claims its slot by a CAS on hi carrying a
// "being written" bit, stores lo, then publishes hi, so a reader that finds
// the bit waits for the key before comparing it.  The host keeps the table at
// most half full (wide_ensure), so a probe always ends.
namespace ldgpu {
namespace {

constexpr uint64_t kWidePending = 1ull << 63;  // never set in hi (klen <= 15 in bits 56..59)

__device__ __forceinline__ uint64_t wide_slot(uint64_t lo, uint64_t hi) { return mix64(lo ^ mix64(hi)); }

// find-or-insert of (lo, hi); -1 if every slot is taken (or, never expected,
// a slot stays "being written" for 2^22 looks).  No lane ever waits inside a
// branch: a lane that wins a slot publishes lo and hi in the same pass of the
// loop body, in straight-line code that every lane passes before the loop's
// exits, and a lane that meets another insert in flight looks at the same
// slot again on its next pass -- so the wave makes progress whatever order
// the compiler gives the divergent paths (a winner and a waiter may share a
// wave: a wait nested in the loser's branch could run before the winner's
// stores and never end).
__device__ __forceinline__ int64_t wide_find_or_insert(const WideCountParams& p, uint64_t lo, uint64_t hi,
                                                       bool& new_key) {
    uint64_t s = wide_slot(lo, hi) >> p.shift;
    uint64_t probes = 0;
    for (uint32_t pass = 0; pass < (1u << 22); ++pass) {
        uint64_t h = __hip_atomic_load(&p.khi[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        bool won = false;
        if (h == kEmpty) {
            const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(&p.khi[s]), 0ull,
                                                     (unsigned long long)(hi | kWidePending));
            won = old == 0ull;
            h = won ? (hi | kWidePending) : old;
        }
        if (won) {  // publish: lo first, then hi without the pending bit
            __hip_atomic_store(&p.klo[s], lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&p.khi[s], hi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            h = hi;
        }
        if (h & kWidePending) continue;  // another insert in flight: look at this slot again
        if (h == hi && (won || __hip_atomic_load(&p.klo[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == lo)) {
            new_key = won;
            return (int64_t)s;
        }
        s = (s + 1) & p.mask;
        if (++probes > p.mask) return -1;
    }
    return -1;
}

__device__ __forceinline__ void wide_add(const WideCountParams& p, uint64_t lo, uint64_t hi, int lang,
                                         unsigned long long c) {
    bool new_key = false;
    const int64_t s = wide_find_or_insert(p, lo, hi, new_key);
    const uint64_t m = __ballot(new_key);
    if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd(p.size, (unsigned long long)__popcll(m));
    if (s >= 0)
        atomicAdd(&p.counts[(size_t)s * p.L + lang], c);
    else
        atomicOr(p.full, 1u);
}

// wide_add without the counter update (flush_new_keys): returns whether the key is new
__device__ __forceinline__ bool wide_add_q(const WideCountParams& p, uint64_t lo, uint64_t hi, int lang,
                                           unsigned long long c) {
    bool new_key = false;
    const int64_t s = wide_find_or_insert(p, lo, hi, new_key);
    if (s >= 0)
        atomicAdd(&p.counts[(size_t)s * p.L + lang], c);
    else
        atomicOr(p.full, 1u);
    return new_key;
}

__global__ __launch_bounds__(kCountWaves * 64) void wide_count_kernel(const WideCountParams p) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
    const int64_t stride = (int64_t)gridDim.x * kCountWaves;
    for (int64_t doc = (int64_t)blockIdx.x * kCountWaves + wave; doc < p.n_docs; doc += stride) {
        const int lang = p.doc_lang[doc];
        if (lang < 0 || lang >= p.L) continue;  // reduceGrams keeps supported languages only
        const int64_t b = p.offsets[doc];
        const int64_t len = p.offsets[doc + 1] - b;
        for (int gi = 0; gi < p.nG; ++gi) {
            const int n = p.G[gi];
            const int64_t nwin = n_windows(len, n);
            const int klen = len < n ? (int)len : n;
            for (int64_t p0 = 0; p0 < nwin; p0 += 64) {
                const int64_t pos = p0 + lane;
                if (pos >= nwin) continue;
                const int64_t a = b + pos;
                const int64_t i = a >> 2;
                const uint32_t sh = (uint32_t)(a & 3);
                uint32_t w[5];
#pragma unroll
                for (int t = 0; t < 5; ++t) w[t] = ld_dw(W, i + t, p.last_dword);
                const uint64_t lo = ((uint64_t)__builtin_amdgcn_alignbyte(w[2], w[1], sh) << 32) |
                                    __builtin_amdgcn_alignbyte(w[1], w[0], sh);
                if (klen <= kMaxGram) {  // a short document's whole text: a one-word key
                    add_count(p.narrow, (lo & (~0ull >> (64 - 8 * klen))) | ((uint64_t)klen << 56), lang, 1ull);
                    continue;
                }
                const uint64_t hw = ((uint64_t)__builtin_amdgcn_alignbyte(w[4], w[3], sh) << 32) |
                                    __builtin_amdgcn_alignbyte(w[3], w[2], sh);
                const uint64_t hi =
                    (klen == 8 ? 0ull : (hw & (~0ull >> (64 - 8 * (klen - 8))))) | ((uint64_t)klen << 56);
                wide_add(p, lo, hi, lang, 1ull);
            }
        }
    }
}

// grow: every occupied slot of `from` (keys unique) into `to`
__global__ void wide_rehash_kernel(const WideCountParams from, const WideCountParams to, uint64_t from_cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= from_cap) return;
    const uint64_t hi = from.khi[i];
    if (hi == kEmpty) return;
    const uint64_t lo = from.klo[i];
    uint64_t s = wide_slot(lo, hi) >> to.shift;
    while (atomicCAS(reinterpret_cast<unsigned long long*>(&to.khi[s]), 0ull, (unsigned long long)hi) != 0ull)
        s = (s + 1) & to.mask;
    to.klo[s] = lo;
    for (int l = 0; l < from.L; ++l) to.counts[(size_t)s * to.L + l] = from.counts[(size_t)i * from.L + l];
}

// ldgpu_counts_add of wide keys: rows[i][L] added at (lo[i], hi[i])
__global__ void wide_add_kernel(const WideCountParams p, const uint64_t* lo, const uint64_t* hi,
                                const unsigned long long* rows, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool new_key = false;
    const int64_t s = i < n ? wide_find_or_insert(p, lo[i], hi[i], new_key) : -1;
    const uint64_t m = __ballot(new_key);
    if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd(p.size, (unsigned long long)__popcll(m));
    if (i >= n) return;
    if (s < 0) {
        atomicOr(p.full, 1u);
        return;
    }
    for (int l = 0; l < p.L; ++l) {
        const unsigned long long c = rows[(size_t)i * p.L + l];
        if (c) atomicAdd(&p.counts[(size_t)s * p.L + l], c);
    }
}

__global__ void wide_compact_kernel(const WideCountParams p, uint64_t cap, uint64_t* out_lo, uint64_t* out_hi,
                                    unsigned long long* out_counts, unsigned long long* out_n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool occ = i < cap && p.khi[i] != kEmpty;
    const uint64_t m = __ballot(occ);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    const int leader = __builtin_ctzll(m);
    if (lane == leader) base = atomicAdd(out_n, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (!occ) return;
    const unsigned long long o =
        base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    out_lo[o] = p.klo[i];
    out_hi[o] = p.khi[i];
    for (int l = 0; l < p.L; ++l) out_counts[o * p.L + l] = p.counts[i * p.L + l];
}

}  // namespace

hipError_t launch_wide_count(const WideCountParams& p, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(wide_count_kernel, dim3(grid), dim3(kCountWaves * 64), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_wide_rehash(const WideCountParams& from, const WideCountParams& to, uint64_t from_cap,
                              hipStream_t stream) {
    if (from_cap == 0) return hipSuccess;
    hipLaunchKernelGGL(wide_rehash_kernel, dim3((unsigned)((from_cap + 255) / 256)), dim3(256), 0, stream, from, to,
                       from_cap);
    return hipGetLastError();
}

hipError_t launch_wide_add(const WideCountParams& p, const uint64_t* lo, const uint64_t* hi,
                           const unsigned long long* rows, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(wide_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, p, lo, hi, rows, n);
    return hipGetLastError();
}

hipError_t launch_wide_compact(const WideCountParams& p, uint64_t cap, uint64_t* out_lo, uint64_t* out_hi,
                               unsigned long long* out_counts, unsigned long long* out_n, hipStream_t stream) {
    if (cap == 0) return hipSuccess;
    hipLaunchKernelGGL(wide_compact_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, stream, p, cap, out_lo,
                       out_hi, out_counts, out_n);
    return hipGetLastError();
}

}  // namespace ldgpu

// ---------------------------------------------------------------------------
// FIT v3: language-grouped LDS aggregation + radix-partitioned record
// aggregation -- the north star's "LDS-privatised histogram, then a sort /
// segmented-reduce merge into HBM count tables" for every gram length (1..15)
// and language count (<= 4096).  The global table sees one add per distinct
// (gram, language) per bucket and batch instead of one device-scope atomic
// per window.  Per batch of documents:
//   emit    the host orders the batch's documents by language and gives each
//           workgroup documents of ONE language, so the workgroup's LDS tables
//           aggregate across its documents: 1-byte windows in a 256-bin
//           histogram, 2- and 3-byte windows in an 8192-slot hash (a window
//           that finds no slot within the probe limit becomes a record);
//           longer windows become records.  Records gather in a workgroup LDS
//           block; a full block is counting-sorted by q1 in LDS and written
//           once, coalesced, with a header of q1 starts.  At the end the tables
//           go out as counted records.  The workgroup also histograms (q1, q2).
//   part2   each q1 run is re-scattered by q2 to exact, host-scanned offsets --
//           4096 contiguous buckets.
//   reduce  one workgroup per bucket sums equal (gram, language) records in an
//           LDS hash and writes (key, count) entries (a record the hash cannot
//           place goes out as it is: the merge adds it all the same).
//   merge   each entry is one find-or-insert + one u64 add in the table.
// Integer sums are order-independent and nothing is dropped: counts are
// bit-exact whatever the schedule and whatever the LDS tables absorbed.
namespace ldgpu {
namespace {

__device__ __forceinline__ bool emit_ablated(const PartParams& p, int bit) { return LDGPU_DIAG && (p.ablate & bit); }

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

constexpr uint64_t kCntMask = (1ull << kCntBits) - 1ull;
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;

// ---- record forms (ldgpu_internal.h).  lo = the window's first min(klen, 8)
// bytes, hi = bytes 8.. (klen > 8), both masked to the window.
template <int K>
struct Rec {
    uint64_t w[K];
};

template <int K>
__device__ __forceinline__ Rec<K> make_rec(uint64_t lo, uint64_t hi, int klen, uint32_t lang, uint64_t c,
                                           const PartParams& p) {
    Rec<K> r;
    if constexpr (K == 1) {
        const uint64_t sent = (1ull << (8 * klen)) | lo;
        r.w[0] = (((sent << p.lb) | (uint64_t)lang) << p.cb) | c;
    } else if constexpr (K == 2) {
        r.w[0] = lo | ((uint64_t)klen << 56);
        r.w[1] = ((uint64_t)lang << kCntBits) | c;
    } else {
        if (klen <= kMaxGram) {
            r.w[0] = lo | ((uint64_t)klen << 56);
            r.w[1] = 0ull;
        } else {
            r.w[0] = lo;
            r.w[1] = hi | ((uint64_t)klen << 56);
        }
        r.w[2] = ((uint64_t)lang << kCntBits) | c;
    }
    return r;
}

template <int K>
__device__ __forceinline__ uint64_t rec_count(const Rec<K>& r, uint32_t cb) {
    if constexpr (K == 1) return r.w[0] & (cb >= 64 ? ~0ull : ((1ull << cb) - 1ull));
    else return r.w[K - 1] & kCntMask;
}

template <int K>
__device__ __forceinline__ uint32_t rec_lang(const Rec<K>& r, uint32_t lb, uint32_t cb) {
    if constexpr (K == 1) return (uint32_t)((r.w[0] >> cb) & ((1ull << lb) - 1ull));
    else return (uint32_t)(r.w[K - 1] >> kCntBits);
}

// route hash of the record's (gram, language) pair; K = 1: the T1 pair
// table's slot hash of the entry (fit_hash(kl)), so a bucket of records maps to
// one contiguous slice of T1 (the merge's inserts stay local)
template <int K>
__device__ __forceinline__ uint64_t rec_hash(const Rec<K>& r, uint32_t cb) {
    if constexpr (K == 1) return fit_hash(r.w[0] >> cb);
    else if constexpr (K == 2) return mix64(r.w[0] + (r.w[1] >> kCntBits) * kGolden);
    else return mix64(r.w[0] ^ mix64(r.w[1] + (r.w[2] >> kCntBits) * kGolden));
}

template <int K>
__device__ __forceinline__ bool rec_same_key(const Rec<K>& a, const Rec<K>& b, uint32_t cb) {
    if constexpr (K == 1) return (a.w[0] >> cb) == (b.w[0] >> cb);
    else if constexpr (K == 2) return a.w[0] == b.w[0] && (a.w[1] >> kCntBits) == (b.w[1] >> kCntBits);
    else return a.w[0] == b.w[0] && a.w[1] == b.w[1] && (a.w[2] >> kCntBits) == (b.w[2] >> kCntBits);
}

template <int K>
__device__ __forceinline__ Rec<K> load_rec(const uint64_t* base, int64_t i) {
    Rec<K> r;
#pragma unroll
    for (int k = 0; k < K; ++k) r.w[k] = base[i * K + k];
    return r;
}

template <int K>
__device__ __forceinline__ void store_rec(uint64_t* base, int64_t i, const Rec<K>& r) {
#pragma unroll
    for (int k = 0; k < K; ++k) base[i * K + k] = r.w[k];
}


// Workgroup barrier for LDS traffic only: waits for this wave's LDS operations
// (lgkmcnt), not for its outstanding global loads -- __syncthreads() would
// drain those too, and emit keeps the next step's window loads in flight
// across the round barriers.  Global stores before it need not be visible to
// the other waves (each flushed block is read by the next kernel only).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// wave inclusive scan (64 lanes)
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    return v;
}

template <int K>
struct EmitLds {
    uint64_t blk[kBlkWords];
    uint8_t bq1[emit_blk_recs(K)];  // q1 of each block record (computed once per record)
    uint32_t hist2[kQ * kQ];
    uint32_t pcnt[kQ];
    uint32_t pfill[kQ];
    uint32_t pstart[kQ + 1];
    uint32_t blk_n;
    uint32_t active;
    uint32_t next_doc;
};

enum { kNextDoc = 0, kWin = 1, kDone = 2 };

// one wave's position in its current document (wave-uniform)
template <int K>
struct WaveState {
    static constexpr int kW = K == 3 ? 5 : 3;  // dwords per window position
    int64_t b, len, p0;
    int64_t nb;                    // the next document (claimed a document early, its loads in flight)
    int32_t nlen;                  // 0: none
    int32_t phase;
    bool pf;                       // pw holds the words of the next WIN step (issued a round early)
    uint32_t pw[emit_sub(K)][kW];
};

// claim the wave's next document and issue the loads of its start / length
template <int K>
__device__ __forceinline__ void claim_next(const PartParams& p, EmitLds<K>& S, WaveState<K>& w, int lane, int64_t d0,
                                           int64_t d1) {
    uint32_t k = 0;
    if (lane == 0) k = __hip_atomic_fetch_add(&S.next_doc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // wave-uniform: scalar loads into SGPRs
    const int64_t i = d0 + (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(k, 0));
    w.nb = 0;
    w.nlen = 0;
    if (i < d1) {
        w.nb = p.dstart[i];
        w.nlen = p.dlen[i];
    }
}

// append the lanes' records (sub per lane) to the workgroup block with one
// reservation (the round bound keeps it from overflowing); every lane of the
// wave must be active
template <int K, int SUB>
__device__ __forceinline__ void emit_recs(EmitLds<K>& S, const bool (&has)[SUB], const Rec<K> (&r)[SUB],
                                          const PartParams& p, int lane) {
    uint64_t m[SUB];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < SUB; ++k) {
        m[k] = __ballot(has[k]);
        tot += (uint32_t)__popcll(m[k]);
    }
    if (!tot) return;
    uint32_t base = 0;
    if (lane == 0) base = __hip_atomic_fetch_add(&S.blk_n, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    base = __shfl(base, 0);
#pragma unroll
    for (int k = 0; k < SUB; ++k) {
        if (has[k]) {
            const uint32_t at = base + lane_rank(m[k]);
            store_rec<K>(S.blk, at, r[k]);
            const uint64_t h = rec_hash<K>(r[k], p.cb);
            const uint32_t q1 = (uint32_t)(h >> (64 - kQBits));
            const uint32_t q2 = (uint32_t)(h >> (64 - 2 * kQBits)) & (kQ - 1);
            S.bq1[at] = (uint8_t)q1;
            __hip_atomic_fetch_add(&S.pcnt[q1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(&S.hist2[q1 * kQ + q2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        base += (uint32_t)__popcll(m[k]);
    }
}

__device__ __forceinline__ uint32_t ld_dw3(const uint32_t* w, int64_t i, int64_t last) {
    return w[i < last ? i : last];
}

// the dwords of the positions of a WIN step at p0: 3 per position for
// windows of <= 7 bytes, 5 for wide ones (as many as max(G) needs)
template <int K>
__device__ __forceinline__ void window_loads(const PartParams& p, const WaveState<K>& w, int lane,
                                             uint32_t (&pw)[emit_sub(K)][WaveState<K>::kW]) {
    constexpr int SUB = emit_sub(K);
    const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
#pragma unroll
    for (int k = 0; k < SUB; ++k) {
        const int64_t pos = w.p0 + 64 * k + lane;
        const int64_t a = w.b + (pos < w.len ? pos : 0);
        const int64_t i = a >> 2;
        pw[k][0] = ld_dw3(W, i, p.last_dword);
        pw[k][1] = ld_dw3(W, i + 1, p.last_dword);
        pw[k][2] = p.maxg > 4 ? ld_dw3(W, i + 2, p.last_dword) : 0u;
        if constexpr (K == 3) {
            pw[k][3] = p.maxg > 8 ? ld_dw3(W, i + 3, p.last_dword) : 0u;
            pw[k][4] = p.maxg > 12 ? ld_dw3(W, i + 4, p.last_dword) : 0u;
        }
    }
}

__device__ __forceinline__ uint64_t byte_mask(int n) { return n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1ull); }

// One step of a wave: <= 64 sub positions of its document, one record each
// -- the maximal window at the position, min(N, len - pos) bytes (N =
// max(G)).  The positions' loads are all issued before any is used; the
// next step's (or the next document's first step's) loads are issued at the
// end, so they fly across the round barrier, and the document after the
// next is claimed as a document starts.
template <int K>
__device__ __forceinline__ void emit_step(const PartParams& p, EmitLds<K>& S, WaveState<K>& w, int lane, int64_t d0,
                                          int64_t d1, uint32_t lang) {
    constexpr int SUB = emit_sub(K);
    if (w.phase == kNextDoc) {  // the wave's first document
        claim_next<K>(p, S, w, lane, d0, d1);
        if (w.nlen == 0) {
            w.phase = kDone;
            if (lane == 0) __hip_atomic_fetch_sub(&S.active, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        w.b = w.nb;
        w.len = w.nlen;
        w.p0 = 0;
        w.pf = false;
        w.phase = kWin;
        claim_next<K>(p, S, w, lane, d0, d1);
    }
    if (!w.pf) window_loads<K>(p, w, lane, w.pw);
    w.pf = false;
    bool has[SUB];
    Rec<K> r[SUB];
#pragma unroll
    for (int k = 0; k < SUB; ++k) {
        const int64_t pos = w.p0 + 64 * k + lane;
        has[k] = pos < w.len;
        const int64_t rem = w.len - pos;
        const int klen = rem >= p.maxg ? p.maxg : (rem > 0 ? (int)rem : 1);
        const uint32_t sh = (uint32_t)((w.b + (has[k] ? pos : 0)) & 3);
        const uint32_t a0 = __builtin_amdgcn_alignbyte(w.pw[k][1], w.pw[k][0], sh);
        const uint32_t a1 = __builtin_amdgcn_alignbyte(w.pw[k][2], w.pw[k][1], sh);
        const uint64_t lo = (((uint64_t)a1 << 32) | a0) & byte_mask(klen);
        uint64_t hi = 0;
        if constexpr (K == 3) {
            if (klen > 8) {
                const uint32_t a2 = __builtin_amdgcn_alignbyte(w.pw[k][3], w.pw[k][2], sh);
                const uint32_t a3 = __builtin_amdgcn_alignbyte(w.pw[k][4], w.pw[k][3], sh);
                hi = (((uint64_t)a3 << 32) | a2) & byte_mask(klen - 8);
            }
        }
        r[k] = make_rec<K>(lo, hi, klen, lang, 1, p);
    }
    if (emit_ablated(p, 4)) {
#pragma unroll
        for (int k = 0; k < SUB; ++k) has[k] = false;
    }
    emit_recs<K, SUB>(S, has, r, p, lane);
    w.p0 += 64 * SUB;
    if (w.p0 >= w.len) {  // the next document (claimed a document ago)
        if (w.nlen == 0) {
            w.phase = kDone;
            if (lane == 0) __hip_atomic_fetch_sub(&S.active, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        w.b = w.nb;
        w.len = w.nlen;
        w.p0 = 0;
        claim_next<K>(p, S, w, lane, d0, d1);
    }
    window_loads<K>(p, w, lane, w.pw);  // the next step's loads fly across the round barrier
    w.pf = true;
}

// Write the block: counting sort by q1 in LDS, scattered stores into the
// block's own contiguous range (the lines fill in L2 and leave whole).
template <int K>
__device__ __forceinline__ void flush_block(const PartParams& p, EmitLds<K>& S, uint32_t n, int64_t rb, int64_t gid,
                                            int tid) {
    if (tid < 64) {
        const uint32_t v = S.pcnt[tid];
        const uint32_t inc = wave_inclusive_scan(v, tid);
        S.pstart[tid] = inc - v;
        S.pfill[tid] = inc - v;
        S.pcnt[tid] = 0u;
        if (tid == 63) S.pstart[kQ] = inc;
    }
    lds_barrier();
    for (uint32_t i = tid; i < n; i += kEmitWaves * 64) {
        const Rec<K> r = load_rec<K>(S.blk, i);
        const uint32_t at = __hip_atomic_fetch_add(&S.pfill[S.bq1[i]], 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        if (!emit_ablated(p, 2)) store_rec<K>(p.rec, rb + at, r);
    }
    if (tid <= kQ) p.blk_hdr[(size_t)gid * kHdr + tid] = S.pstart[tid];
    if (tid == 0) {
        p.blk_start[gid] = rb;
        S.blk_n = 0u;
    }
    lds_barrier();
}

// (HIP launch bound: >= 8 waves per SIMD, i.e. two workgroups per CU -- <= 64 VGPRs)
template <int K>
__global__ __launch_bounds__(kEmitWaves * 64, 8) void emit_kernel(const PartParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t emit_smem[];
    EmitLds<K>& S = *reinterpret_cast<EmitLds<K>*>(emit_smem);
    constexpr uint32_t kThresh = (uint32_t)(emit_blk_recs(K) - emit_round_recs(K));
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int bid = blockIdx.x;
    const int64_t d0 = p.wg_doc[bid], d1 = p.wg_doc[bid + 1];
    const int64_t rbase = p.wg_rec[bid], dbase = p.wg_dir[bid];
    const uint32_t lang = (uint32_t)p.wg_lang[bid];
    for (int i = tid; i < kQ * kQ; i += kEmitWaves * 64) S.hist2[i] = 0u;
    if (tid < kQ) S.pcnt[tid] = 0u;
    if (tid == 0) {
        S.blk_n = 0u;
        S.active = kEmitWaves;
        S.next_doc = 0u;
    }
    lds_barrier();
    WaveState<K> w{};
    w.phase = d0 < d1 ? kNextDoc : kDone;
    if (w.phase == kDone && lane == 0)
        __hip_atomic_fetch_sub(&S.active, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    int64_t written = 0;
    int64_t nb = 0;
    lds_barrier();
    for (;;) {
        // a round: every live wave takes one step (<= emit_round_recs records,
        // so the block, flushed above kThresh, never overflows)
        if (w.phase != kDone) emit_step<K>(p, S, w, lane, d0, d1, lang);
        lds_barrier();
        const uint32_t n = S.blk_n;
        const uint32_t act = S.active;
        lds_barrier();  // every thread has read n / act before the next round moves them
        if (n > kThresh || (act == 0u && n > 0u)) {
            flush_block<K>(p, S, n, rbase + written, dbase + nb, tid);
            written += n;
            ++nb;
        }
        if (act == 0u) break;
    }
    if (tid == 0) p.nblk[bid] = (int32_t)nb;
    const int grp = bid / (p.grid_a / kSplits);
    for (int i = tid; i < kQ * kQ; i += kEmitWaves * 64)
        if (S.hist2[i]) atomicAdd(&p.cnt3[i * kSplits + grp], S.hist2[i]);
}

// part2: the q1 runs of one emit group's blocks -> q2 sub-buckets at exact
// offsets.  Per round the workgroup gathers up to p2_cap records of
// consecutive runs into LDS (a run longer than the room continues in the next
// round), counting-sorts them by q2 there and writes each q2 segment
// contiguously at the workgroup's running cursor of that sub-bucket -- stores
// of consecutive addresses, where scattering each record to its sub-bucket
// straight from the run would touch 64 lines per store instruction.  (Order
// within a sub-bucket is free: reduce sums.)
template <int K>
constexpr int p2_cap() {
    return K == 1 ? 4096 : (K == 2 ? 2048 : 1024);
}

template <int K>
struct Part2Lds {
    uint64_t in[p2_cap<K>() * K];
    uint64_t out[p2_cap<K>() * K];
    uint8_t q2in[p2_cap<K>()];
    uint8_t q2out[p2_cap<K>()];
    int64_t rstart[64];    // the round's runs: first record (global index)
    uint32_t roff[65];     // their offsets in the round (exclusive prefix), roff[64] = total
    uint32_t hist[kQ];
    uint32_t fill[kQ];
    uint32_t lstart[kQ];
    uint64_t cur[kQ];      // records written per q2 sub-bucket so far
    int64_t base[kQ];      // global index of the round's first record of q2, minus its LDS start
    int32_t gpre[257];     // blocks of the group's emit workgroups (exclusive prefix)
    int64_t unit, uoff;    // next run and the records of it already taken
};

__device__ __forceinline__ int64_t rdlane_i64(int64_t v, int l) {
    return (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l) << 32));
}

template <int K>
__global__ __launch_bounds__(kEmitWaves * 64) void part2_kernel(const PartParams p) {
    constexpr int CAP = p2_cap<K>();
    constexpr int NT = kEmitWaves * 64;
    __shared__ Part2Lds<K> S;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t q1 = blockIdx.x / kSplits;
    const int s = blockIdx.x % kSplits;
    const int per = p.grid_a / kSplits;
    const int w0 = s * per;
    if (tid == 0) {
        int32_t acc = 0;
        for (int k = 0; k < per; ++k) {
            S.gpre[k] = acc;
            acc += p.nblk[w0 + k];
        }
        S.gpre[per] = acc;
        S.unit = 0;
        S.uoff = 0;
    }
    if (tid < kQ) {
        S.cur[tid] = 0;
        S.hist[tid] = 0u;
    }
    __syncthreads();
    const int64_t tb = S.gpre[per];
    for (;;) {
        if (tid < 64) {  // wave 0 plans the round: runs unit .. unit + 63
            const int64_t u0 = S.unit, o0 = S.uoff;
            const int64_t u = u0 + lane;
            int64_t st = 0;
            uint32_t ln = 0;
            if (u < tb) {
                int lo = 0, hi = per;  // emit workgroup of unit u: largest k with gpre[k] <= u
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (S.gpre[mid] <= u) lo = mid;
                    else hi = mid;
                }
                const int64_t gid = p.wg_dir[w0 + lo] + (u - S.gpre[lo]);
                const uint32_t a = p.blk_hdr[(size_t)gid * kHdr + q1];
                const uint32_t e = p.blk_hdr[(size_t)gid * kHdr + q1 + 1];
                st = p.blk_start[gid] + a;
                ln = e - a;
                if (lane == 0) {
                    st += o0;
                    ln -= (uint32_t)o0;
                }
            }
            const uint32_t inc = wave_inclusive_scan(ln, lane);
            const uint32_t exc = inc - ln;
            const uint64_t over = __ballot(inc > (uint32_t)CAP);
            S.rstart[lane] = st;
            S.roff[lane] = exc < (uint32_t)CAP ? exc : (uint32_t)CAP;
            if (lane == 63) {
                const int64_t nu = u0 + 64 < tb ? u0 + 64 : tb;
                if (!over) {
                    S.roff[64] = inc;
                    S.unit = nu;
                    S.uoff = 0;
                }
            }
            if (over) {
                const int l = __builtin_ctzll(over);  // the run the room ends in
                const uint32_t ex_l = (uint32_t)__shfl((int)exc, l);
                if (lane == 0) {
                    S.roff[64] = CAP;
                    S.unit = u0 + l;
                    S.uoff = (l == 0 ? o0 : 0) + (int64_t)(CAP - ex_l);
                }
            }
        }
        __syncthreads();
        const uint32_t T = S.roff[64];
        const bool done = S.unit >= tb;
        if (T == 0u) {  // 64 empty runs (or none left)
            __syncthreads();  // every thread has read T / unit before wave 0 plans again
            if (done) break;
            continue;
        }
        // gather: record i of the round from its run.  A thread's records of
        // the round (CAP / NT of them) are located first and their loads all
        // issued before any is used: one memory round trip per round, not one
        // per record.
        constexpr int PER = CAP / NT;
        static_assert(CAP % NT == 0 && PER >= 1, "part2 gather");
        Rec<K> r[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = (uint32_t)tid + (uint32_t)(u * NT);
            if (i < T) {
                int lo = 0;
#pragma unroll
                for (int step = 32; step >= 1; step >>= 1)
                    if (S.roff[lo + step] <= i) lo += step;
                r[u] = load_rec<K>(p.rec, S.rstart[lo] + (int64_t)(i - S.roff[lo]));
            }
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = (uint32_t)tid + (uint32_t)(u * NT);
            if (i < T) {
                const uint32_t q2 = (uint32_t)(rec_hash<K>(r[u], p.cb) >> (64 - 2 * kQBits)) & (kQ - 1);
                store_rec<K>(S.in, i, r[u]);
                S.q2in[i] = (uint8_t)q2;
                __hip_atomic_fetch_add(&S.hist[q2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        if (tid < 64) {
            const uint32_t v = S.hist[tid];
            const uint32_t inc = wave_inclusive_scan(v, tid);
            S.lstart[tid] = inc - v;
            S.fill[tid] = inc - v;
            S.base[tid] = (int64_t)p.p2off[((size_t)q1 * kQ + tid) * kSplits + s] + (int64_t)S.cur[tid] - (int64_t)(inc - v);
            S.cur[tid] += v;
            S.hist[tid] = 0u;
        }
        __syncthreads();
        for (uint32_t i = tid; i < T; i += NT) {
            const uint32_t q2 = S.q2in[i];
            const uint32_t at = __hip_atomic_fetch_add(&S.fill[q2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            store_rec<K>(S.out, at, load_rec<K>(S.in, i));
            S.q2out[at] = (uint8_t)q2;
        }
        __syncthreads();
        for (uint32_t i = tid; i < T; i += NT) store_rec<K>(p.rec2, S.base[S.q2out[i]] + (int64_t)i, load_rec<K>(S.out, i));
        __syncthreads();  // the next round's plan overwrites roff / rstart; its gather, in
    }
}

// Exact bucket offsets from the emit histograms, on the device (no host
// round trip between emit and part2): cnt3[(q1, q2)][group] counts ->
// p2off = their exclusive prefix in that order, boff[b] = p2off[b][0],
// boff[kQ * kQ] = the total.  One workgroup: each thread scans 32 counters.
__global__ __launch_bounds__(1024) void fit_offsets_kernel(const uint32_t* cnt3, uint64_t* p2off, uint64_t* boff) {
    constexpr int kN = kQ * kQ * kSplits, kPer = kN / 1024;
    static_assert(kN % 1024 == 0 && kPer % kSplits == 0, "fit offsets");
    __shared__ uint64_t part[1024];
    const int t = threadIdx.x;
    uint64_t sum = 0;
    for (int i = 0; i < kPer; ++i) sum += cnt3[t * kPer + i];
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan (Hillis-Steele)
        const uint64_t v = t >= o ? part[t - o] : 0ull;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t acc = part[t] - sum;
    for (int i = 0; i < kPer; ++i) {
        const int j = t * kPer + i;
        p2off[j] = acc;
        if (j % kSplits == 0) boff[j / kSplits] = acc;
        acc += cnt3[j];
    }
    if (t == 1023) boff[kQ * kQ] = acc;
}

// reduce: LDS hash slots per bucket (K u64 key words + a u32 count each, within
// one workgroup's LDS)
template <int K>
constexpr int agg_slots() {
    return K == 1 ? 12288 : (K == 2 ? 6144 : 4096);
}

// entries out: bucket b writes from boff[b] on (it has at most as many as
// records), through a workgroup-local counter -- one global counter for every
// bucket's appends would serialise ~0.5M atomics per batch on one address.
// An entry is out_words(K) words: K = 1 (kl, count) -- a bucket's sum may
// exceed a record's count bits --, K >= 2 the record form with the sum in its
// count field.
template <int K>
__device__ __forceinline__ void out_append(const PartParams& p, uint32_t* n_out, int64_t base, bool has,
                                           const Rec<K>& r, uint64_t c, int lane) {
    const uint64_t m = __ballot(has);
    if (!m) return;
    uint32_t at = 0;
    if (lane == 0) at = __hip_atomic_fetch_add(n_out, (uint32_t)__popcll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    at = __shfl(at, 0);
    if (!has) return;
    const int64_t o = base + at + lane_rank(m);
    if constexpr (K == 1) {
        p.out[2 * o] = r.w[0] >> p.cb;
        p.out[2 * o + 1] = c;
    } else {
        Rec<K> e = r;
        e.w[K - 1] = (e.w[K - 1] & ~kCntMask) | c;
        store_rec<K>(p.out, o, e);
    }
}

// LDS claim protocol for keys of several words (K >= 2): a slot is claimed
// by a CAS of its tag word from 0 to kBusy, the claimer stores the key words
// and then the tag (a nonzero hash of the key); a reader compares the key words
// only after it has seen the tag.  A reader that meets kBusy, or a tag that
// matches while the key differs, probes on: at worst one key gets two slots
// (two entries out, summed by the merge).
constexpr uint32_t kBusy = 1u;

constexpr int kRedRounds = 8;  // reduce: LDS probe rounds per record

// K = 1 reduce probes without divergent branches: every lane issues the round's
// LDS read, CAS and counter add, a lane with nothing to claim or add aiming
// them at a dummy word of its own (kRedDummy u64 words after the table) -- the
// exec-mask save / restore of each divergent branch cost ~1 SALU instruction
// per record on the CU's one scalar unit
#ifndef LDGPU_RED_BRANCHLESS
#define LDGPU_RED_BRANCHLESS 1
#endif
constexpr int kRedDummy = kEmitWaves * 64;

template <int K>
__global__ __launch_bounds__(kEmitWaves * 64, 1) void reduce_kernel(const PartParams p) {
    constexpr int N = agg_slots<K>();
    extern __shared__ __attribute__((aligned(16))) uint8_t red_smem[];
    // K = 1: keys[N] (kl, 0 = empty) + cnt[N]; K >= 2: kw[N][K - 1] key words,
    // lang[N], tag[N], cnt[N]
    uint64_t* kw = reinterpret_cast<uint64_t*>(red_smem);
    uint32_t* lg = reinterpret_cast<uint32_t*>(kw + (size_t)N * (K == 1 ? 1 : K - 1));
    uint32_t* tag = lg + (K == 1 ? 0 : N);
    uint32_t* cnt = tag + (K == 1 ? 0 : N);
    uint32_t* n_out = cnt + N;
    // K = 1, branch-light probes: a dummy u64 per thread (16-B aligned after n_out)
    uint64_t* dummy = reinterpret_cast<uint64_t*>(red_smem + (((size_t)N * 12 + 4 + 15) & ~(size_t)15));
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    for (int i = tid; i < N; i += kEmitWaves * 64) {
        cnt[i] = 0u;
        if (K == 1) kw[i] = 0ull;
        else tag[i] = 0u;
    }
    if (tid == 0) *n_out = 0u;
    __syncthreads();
    const int64_t beg = (int64_t)p.boff[blockIdx.x], end = (int64_t)p.boff[blockIdx.x + 1];
    constexpr int kU = 4;  // records per lane in flight (and 4 more loading); their probes advance together
    // software pipeline: the next chunk's records load while this chunk probes
    Rec<K> nx[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int64_t i = beg + (int64_t)wave * 64 * kU + 64 * u + lane;
        nx[u] = i < end ? load_rec<K>(p.rec2, i) : Rec<K>{};
    }
    for (int64_t i00 = beg + (int64_t)wave * 64 * kU; i00 < end; i00 += kEmitWaves * 64 * kU) {
        Rec<K> r[kU];
        uint32_t c[kU], slot[kU], tg[kU];
        bool pend[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            r[u] = nx[u];
            const int64_t j = i00 + kEmitWaves * 64 * kU + 64 * u + lane;
            nx[u] = j < end ? load_rec<K>(p.rec2, j) : Rec<K>{};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t i = i00 + 64 * u + lane;
            pend[u] = i < end;
            c[u] = (uint32_t)rec_count<K>(r[u], p.cb);
            const uint64_t h = rec_hash<K>(r[u], p.cb);
            // (K = 1: bits 20..51 of fit_hash -- its low bits see only the
            // key's low bits)
            slot[u] = (uint32_t)(((uint64_t)(uint32_t)(K == 1 && LDGPU_FIT_FIB ? h >> 20 : h) * (uint64_t)N) >> 32);
            tg[u] = (uint32_t)(h >> 32) | 2u;  // never 0 (empty) or kBusy
        }
        // a bounded number of probe rounds: the wave waits for its slowest
        // lane, and a record still unplaced goes out as it is
        for (int t = 0; t < kRedRounds; ++t) {
            bool any = false;
            if constexpr (K == 1 && LDGPU_RED_BRANCHLESS) {
                const uint4* KW2 = reinterpret_cast<const uint4*>(kw);
                uint4 cur[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) cur[u] = KW2[slot[u] >> 1];
                uint64_t* const dk = &dummy[tid];
                uint32_t* const dc = reinterpret_cast<uint32_t*>(dk);
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const uint64_t kl = r[u].w[0] >> p.cb;  // never 0 for a record: the sentinel bit
                    const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x;
                    const uint64_t k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                    const uint32_t pr = slot[u] & ~1u;
                    const bool h0 = k0 == kl, h1 = k1 == kl, e0 = k0 == 0ull, e1 = k1 == 0ull;
                    const bool hit = pend[u] && (h0 || h1);
                    const bool claim = pend[u] && !h0 && !h1 && (e0 || e1);
                    const uint32_t ca = pr + (e0 ? 0u : 1u);
                    const unsigned long long old = atomicCAS(
                        reinterpret_cast<unsigned long long*>(claim ? &kw[ca] : dk), 0ull, (unsigned long long)kl);
                    const bool won = claim && (old == 0ull || old == kl);
                    const bool add = hit || won;
                    const uint32_t at = hit ? pr + (h0 ? 0u : 1u) : ca;
                    __hip_atomic_fetch_add(add ? &cnt[at] : dc, add ? c[u] : 0u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    // a full pair without the key: the next pair; a lost claim:
                    // this pair again
                    const bool full = pend[u] && !h0 && !h1 && !e0 && !e1;
                    slot[u] = full ? (pr + 2u == (uint32_t)N ? 0u : pr + 2u) : slot[u];
                    pend[u] = pend[u] && !add;
                    any = any || pend[u];
                }
            } else if constexpr (K == 1) {
                // slot pairs: one ds_read_b128 reads both keys of a pair
                // (filled in slot order, never emptied)
                const uint4* KW2 = reinterpret_cast<const uint4*>(kw);
                uint4 cur[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) cur[u] = pend[u] ? KW2[slot[u] >> 1] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    if (!pend[u]) continue;
                    const uint64_t kl = r[u].w[0] >> p.cb;  // never 0 for a record: the sentinel bit
                    const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x;
                    const uint64_t k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                    const uint32_t pr = slot[u] & ~1u;
                    int hit = k0 == kl ? 0 : (k1 == kl ? 1 : -1);
                    if (hit < 0) {
                        const int emp = k0 == 0ull ? 0 : (k1 == 0ull ? 1 : -1);
                        if (emp >= 0) {
                            const unsigned long long old = atomicCAS(
                                reinterpret_cast<unsigned long long*>(&kw[pr + (uint32_t)emp]), 0ull, (unsigned long long)kl);
                            if (old == 0ull || old == kl) hit = emp;  // else: lost the slot, read the pair again
                        } else {
                            slot[u] = pr + 2u == (uint32_t)N ? 0u : pr + 2u;
                        }
                    }
                    if (hit >= 0) {
                        __hip_atomic_fetch_add(&cnt[pr + (uint32_t)hit], c[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        pend[u] = false;
                    } else {
                        any = true;
                    }
                }
            } else {
                uint32_t cur[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) cur[u] = pend[u] ? tag[slot[u]] : 0u;
                bool won[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    won[u] = false;
                    if (pend[u] && cur[u] == 0u) {
                        const uint32_t old = atomicCAS(&tag[slot[u]], 0u, kBusy);
                        won[u] = old == 0u;
                        cur[u] = won[u] ? kBusy : old;
                    }
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    if (!won[u]) continue;  // a claimed slot: key words, then the tag
#pragma unroll
                    for (int k = 0; k < K - 1; ++k) kw[(size_t)slot[u] * (K - 1) + k] = r[u].w[k];
                    lg[slot[u]] = (uint32_t)(r[u].w[K - 1] >> kCntBits);
                    __hip_atomic_fetch_add(&cnt[slot[u]], c[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&tag[slot[u]], tg[u], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    pend[u] = false;
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    if (!pend[u]) continue;
                    bool same = cur[u] == tg[u];
                    if (same) {
#pragma unroll
                        for (int k = 0; k < K - 1; ++k) same &= kw[(size_t)slot[u] * (K - 1) + k] == r[u].w[k];
                        same &= lg[slot[u]] == (uint32_t)(r[u].w[K - 1] >> kCntBits);
                    }
                    if (same) {
                        __hip_atomic_fetch_add(&cnt[slot[u]], c[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        pend[u] = false;
                    } else {
                        slot[u] = slot[u] + 1u == (uint32_t)N ? 0u : slot[u] + 1u;
                        any = true;
                    }
                }
            }
            if (!__ballot(any)) break;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)  // no LDS room: the record goes out as it is
            out_append<K>(p, n_out, beg, pend[u], r[u], c[u], lane);
    }
    __syncthreads();
    for (int i0 = wave * 64; i0 < N; i0 += kEmitWaves * 64) {
        const int i = i0 + lane;
        Rec<K> r{};
        bool has;
        if constexpr (K == 1) {
            has = kw[i] != 0ull;
            r.w[0] = kw[i] << p.cb;  // the record form of the entry's kl (out_append shifts it back)
        } else {
            has = tag[i] > kBusy;
#pragma unroll
            for (int k = 0; k < K - 1; ++k) r.w[k] = kw[(size_t)i * (K - 1) + k];
            r.w[K - 1] = (uint64_t)lg[i] << kCntBits;
        }
        out_append<K>(p, n_out, beg, has, r, cnt[i], lane);
    }
    __syncthreads();
    if (tid == 0) p.nout[blockIdx.x] = *n_out;
}

// merge: one workgroup per reduce bucket b (b0 + block) adds the bucket's
// nout[b] entries (at boff[b]) into T1 -- a bucket's keys share the top bits
// of their route hash, which (K = 1 pairs) are the top bits of their T1 slot:
// the workgroup's inserts stay within one slice of the table.
// pairs (K = 1): T1 is a table of (window, language) pairs -- key = the
// entry's kl (sentinel key << lb | lang), one counter (L = 1)
template <int K>
__global__ __launch_bounds__(1024) void merge_kernel(const PartParams p, const CountParams c, const WideCountParams w,
                                                     int b0, int pairs) {
    const int b = b0 + blockIdx.x;
    const int64_t n = p.nout[b];
    const int64_t base = (int64_t)p.boff[b];
    unsigned int nn = 0, nw = 0;
    if constexpr (K == 1) {
        // kMU entries per thread at a time: their loads, then their tables'
        // first probes, all issued before any is resolved (the merge waited
        // ~80 % of its cycles on one dependent chain per entry)
        constexpr int kMU = 4;
        for (int64_t i0 = threadIdx.x; i0 < n; i0 += kMU * (int64_t)blockDim.x) {
            uint64_t key[kMU], cn[kMU], sl[kMU], k0[kMU];
            int lg[kMU];
#pragma unroll
            for (int u = 0; u < kMU; ++u) {
                const int64_t i = i0 + (int64_t)u * blockDim.x;
                key[u] = kEmpty;
                cn[u] = 0;
                if (i < n) {
                    key[u] = p.out[2 * (base + i)];
                    cn[u] = p.out[2 * (base + i) + 1];
                }
            }
#pragma unroll
            for (int u = 0; u < kMU; ++u) {
                lg[u] = 0;
                if (key[u] != kEmpty && !pairs) {
                    lg[u] = (int)(key[u] & ((1ull << p.lb) - 1ull));
                    key[u] = kl_key(key[u], p.lb);
                }
                sl[u] = fit_hash(key[u]) >> c.shift;
                k0[u] = key[u] != kEmpty ? __hip_atomic_load(&c.keys[sl[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : 0ull;
            }
#pragma unroll
            for (int u = 0; u < kMU; ++u) {
                if (key[u] == kEmpty) continue;
                bool nk = false;
                const int64_t at = find_or_insert_at<true>(c, key[u], sl[u], k0[u], nk);
                nn += nk ? 1u : 0u;
                count_add_slot(c, at, key[u], lg[u], cn[u]);
            }
        }
    }
    for (int64_t i = threadIdx.x; i < (K == 1 ? 0 : n); i += blockDim.x) {
        const int64_t at = base + i;
        if constexpr (K == 1) {
        } else {
            const Rec<K> r = load_rec<K>(p.out, at);
            const int lang = (int)(r.w[K - 1] >> kCntBits);
            const unsigned long long cn = r.w[K - 1] & kCntMask;
            if (K == 2 && pairs) nw += wide_add_q(w, r.w[0], (uint64_t)lang + 1ull, 0, cn);  // (key, lang + 1)
            else if (K == 3 && r.w[1] != 0ull) nw += wide_add_q(w, r.w[0], r.w[1], lang, cn);
            else nn += add_count_q(c, r.w[0], lang, cn);
        }
    }
    flush_new_keys(c.size, nn);
    if (K >= 2 && w.size) flush_new_keys(w.size, nw);
}

}  // namespace

namespace {
// Derive (FIT v4), level by level.  T1 holds, per (maximal window w of t
// bytes, language), the number of positions whose maximal window is w.  With
// S_n(g) = the positions whose maximal window has g as prefix and >= n bytes
// -- the count of the n-gram g (LanguageDetector.scala:32-43) --
//   S_N = the windows of N bytes,   S_n(g) = sum_x S_{n+1}(g x) + A_n(g)
// (A_n: the maximal windows of exactly n bytes, the tails of documents).
// Level t: every T1 entry of t bytes -- a maximal window or an aggregate of
// level t made by level t + 1 (key flag kDerived) -- adds mult(t) c to its
// key in T when t is in gramLengths (duplicates count mult(t) times) and c to
// its (t-1)-byte prefix, flagged, in T1.  The entries a level inserts are one
// byte shorter than the ones it reads, so one pass per level sees each
// entry once; the host keeps T1 from growing during a level.  Compared with
// adding every maximal window to all its prefixes, a level adds only its own
// distinct keys to the next (the hot 1- and 2-byte prefixes receive a few
// thousand adds instead of one per window of the table).

__global__ __launch_bounds__(256) void derive_level_kernel(const CountParams t1, const WideCountParams t1w, int wide,
                                                           uint64_t s0, uint64_t s1, int lev, uint32_t mt,
                                                           const CountParams to, const WideCountParams tow) {
    const int L = t1.L;
    uint64_t n_to = 0;
    unsigned int n_tow = 0, n_t1 = 0, n_t1w = 0;
    for (uint64_t s = s0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < s1;
         s += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo, hi = 0;
        const unsigned long long* row;
        if (!wide) {
            const uint64_t key = t1.keys[s];
            if (key == kEmpty || (int)((key >> 56) & 15) != lev) continue;
            lo = key & 0x00ffffffffffffffull;
            row = t1.counts + s * (uint64_t)L;
        } else {
            const uint64_t h = t1w.khi[s];
            if (h == kEmpty || (int)((h >> 56) & 15) != lev) continue;
            lo = t1w.klo[s];
            hi = h & 0x00ffffffffffffffull;
            row = t1w.counts + s * (uint64_t)L;
        }
        const int n = lev - 1;
        for (int l = 0; l < L; ++l) {
            const unsigned long long c = row[l];
            if (!c) continue;
            if (mt) {
                if (lev <= kMaxGram) n_to += t_add_q(to, lo | ((uint64_t)lev << 56), l, c * mt);
                else n_tow += wide_add_q(tow, lo, hi | ((uint64_t)lev << 56), l, c * mt);
            }
            if (n >= 1) {
                if (n <= kMaxGram) n_t1 += add_count_q(t1, (lo & byte_mask(n)) | ((uint64_t)n << 56) | kDerived, l, c);
                else n_t1w += wide_add_q(t1w, lo, (hi & byte_mask(n - 8)) | ((uint64_t)n << 56) | kDerived, l, c);
            }
        }
    }
    t_flush(to, n_to);
    flush_new_keys(t1.size, n_t1);
    if (tow.size) flush_new_keys(tow.size, n_tow);
    if (t1w.size) flush_new_keys(t1w.size, n_t1w);
}

// the same level for a pair table T1 (K = 1 records: key = kl | kDerived,
// one counter): one thread per (window, language) entry
__device__ __forceinline__ int kl_len(uint64_t kl, uint32_t lb) {
    return (63 - __builtin_clzll(kl >> lb)) >> 3;
}

__global__ __launch_bounds__(256) void derive_pairs_level_kernel(const CountParams t1, uint32_t lb, uint64_t s0,
                                                                 uint64_t s1, int lev, uint32_t mt,
                                                                 const CountParams to, int ablate) {
    const uint64_t lmask = (1ull << lb) - 1ull;
    uint64_t n_to = 0;
    unsigned int n_t1 = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const int n = lev - 1;
    const bool to_t = mt && !(LDGPU_DIAG && (ablate & 1));
    const bool to_t1 = n >= 1 && !(LDGPU_DIAG && (ablate & 2));
    if (to.pkeys) {
        // sparse T: kDU slots per thread at a time -- their T1 entries, then
        // the first probes of their gram (T) and prefix (T1) inserts, then
        // those of their pairs, each batch issued before any is resolved
        constexpr int kDU = 4;
        for (uint64_t s = s0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < s1; s += kDU * stride) {
            uint64_t e[kDU];
#pragma unroll
            for (int u = 0; u < kDU; ++u) {
                const uint64_t su = s + u * stride;
                e[u] = su < s1 ? t1.keys[su] : kEmpty;
            }
            uint64_t gk[kDU], pk[kDU], gs[kDU], g0[kDU], ps[kDU], p0[kDU];
            unsigned long long c[kDU];
            int lang[kDU];
            bool v[kDU];
#pragma unroll
            for (int u = 0; u < kDU; ++u) {
                const uint64_t kl = e[u] & ~kDerived;
                v[u] = e[u] != kEmpty && kl_len(kl, lb) == lev;
                c[u] = v[u] ? t1.counts[s + u * stride] : 0ull;
                lang[u] = (int)(kl & lmask);
                const uint64_t bytes = (kl >> lb) ^ (1ull << (8 * lev));
                gk[u] = bytes | ((uint64_t)lev << 56);
                const uint64_t sent = (1ull << (8 * (n > 0 ? n : 0))) | (bytes & byte_mask(n > 0 ? n : 0));
                pk[u] = ((sent << lb) | (uint64_t)lang[u]) | kDerived;
                gs[u] = fit_hash(gk[u]) >> to.shift;
                ps[u] = fit_hash(pk[u]) >> t1.shift;
                g0[u] = v[u] && to_t ? __hip_atomic_load(&to.keys[gs[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                p0[u] = v[u] && to_t1 ? __hip_atomic_load(&t1.keys[ps[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : 0ull;
            }
            if (to_t) {
                int64_t g[kDU];
                bool ng[kDU];
#pragma unroll
                for (int u = 0; u < kDU; ++u) {
                    ng[u] = false;
                    // (a zero count adds nothing, as sparse_add_q: never the case
                    // for a T1 entry, whose counts are sums of records)
                    g[u] = v[u] && c[u] ? find_or_insert_at<true>(to, gk[u], gs[u], g0[u], ng[u]) : -1;
                }
                uint64_t pp[kDU], pa[kDU], pv[kDU];
#pragma unroll
                for (int u = 0; u < kDU; ++u) {
                    pp[u] = ((uint64_t)(g[u] + 1) << kPairLangBits) | (uint64_t)lang[u];
                    pa[u] = fit_hash(pp[u]) >> to.pshift;
                    pv[u] = g[u] >= 0 ? __hip_atomic_load(pkey_at(to, pa[u]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : 0ull;
                }
#pragma unroll
                for (int u = 0; u < kDU; ++u) {
                    if (!v[u] || !c[u]) continue;
                    const unsigned long long cm = c[u] * mt;
                    bool np = false;
                    int64_t sp = -1;
                    if (g[u] >= 0) {
                        sp = pair_find_or_insert_at<true>(to, pp[u], pa[u], pv[u], np);
                        if (sp >= 0) atomicAdd(pcnt_at(to, sp), cm);
                        kcnt_delta(to, g[u], ng[u], np);
                    }
                    if (sp < 0) {  // a probe limit: (key, lang, c) to the overflow list (sparse_add_q)
                        const unsigned int at = atomicAdd(to.ovf_n, 1u);
                        if (at < to.ovf_cap) {
                            to.ovf_keys[at] = gk[u];
                            to.ovf_lang[at] = lang[u];
                            to.ovf_cnt[at] = cm;
                        }
                    }
                    n_to += (uint64_t)ng[u] | ((uint64_t)np << 32);
                }
            }
            if (to_t1) {
#pragma unroll
                for (int u = 0; u < kDU; ++u) {
                    if (!v[u]) continue;
                    bool nk = false;
                    const int64_t at = find_or_insert_at<true>(t1, pk[u], ps[u], p0[u], nk);
                    n_t1 += nk ? 1u : 0u;
                    count_add_slot(t1, at, pk[u], 0, c[u]);
                }
            }
        }
        t_flush(to, n_to);
        flush_new_keys(t1.size, n_t1);
        return;
    }
    for (uint64_t s = s0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < s1;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = t1.keys[s];
        if (key == kEmpty) continue;
        const uint64_t kl = key & ~kDerived;
        const int klen = kl_len(kl, lb);
        if (klen != lev) continue;
        const unsigned long long c = t1.counts[s];
        const int lang = (int)(kl & lmask);
        const uint64_t bytes = (kl >> lb) ^ (1ull << (8 * klen));
        if (mt && !(LDGPU_DIAG && (ablate & 1))) n_to += t_add_q(to, bytes | ((uint64_t)klen << 56), lang, c * mt);
        const int n = lev - 1;
        if (n >= 1 && !(LDGPU_DIAG && (ablate & 2))) {
            const uint64_t sent = (1ull << (8 * n)) | (bytes & byte_mask(n));
            n_t1 += add_count_q(t1, ((sent << lb) | (uint64_t)lang) | kDerived, 0, c);
        }
    }
    t_flush(to, n_to);
    flush_new_keys(t1.size, n_t1);
}

// the same for a two-word pair table T1 (K = 2 records: a wide table with
// one counter, lo = the window's packed key, hi = lang + 1 | kDerived).
// Split (nx.khi set): the level's prefixes and the entries shorter than the
// level go to nx, a fresh table for the levels below, so T1 never holds more
// than two levels' entries at once (a 1 GB fit at L = 200 holds ~1.5G pairs
// per level).
__global__ __launch_bounds__(256) void derive_pairs2_level_kernel(const WideCountParams t1w, uint64_t s0, uint64_t s1,
                                                                  int lev, uint32_t mt, const CountParams to,
                                                                  const WideCountParams nx, int ablate) {
    const bool split = nx.khi != nullptr;
    const WideCountParams& dst = split ? nx : t1w;
    uint64_t n_to = 0;
    unsigned int n_t1 = 0;
    for (uint64_t s = s0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < s1;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t hi = t1w.khi[s];
        if (hi == kEmpty) continue;
        const uint64_t key = t1w.klo[s];
        const int klen = (int)(key >> 56);
        if (klen != lev) {
            if (split && klen < lev) n_t1 += wide_add_q(nx, key, hi, 0, t1w.counts[s]);
            continue;
        }
        const unsigned long long c = t1w.counts[s];
        const int lang = (int)((hi & ~kDerived) - 1ull);
        if (mt && !(LDGPU_DIAG && (ablate & 1))) n_to += t_add_q(to, key, lang, c * mt);
        const int n = lev - 1;
        if (n >= 1 && !(LDGPU_DIAG && (ablate & 2)))
            n_t1 += wide_add_q(dst, (key & byte_mask(n)) | ((uint64_t)n << 56), ((uint64_t)lang + 1ull) | kDerived, 0,
                               c);
    }
    t_flush(to, n_to);
    flush_new_keys(dst.size, n_t1);
}

// occupied T1 slots per key length (one-word and wide tables)
__global__ __launch_bounds__(256) void len_hist_kernel(const CountParams t1, const WideCountParams t1w, int pairs,
                                                       uint32_t lb, unsigned long long* out) {
    __shared__ unsigned int h[16];
    if (threadIdx.x < 16) h[threadIdx.x] = 0u;
    __syncthreads();
    const uint64_t cap = t1.mask + 1, wcap = t1w.klo ? t1w.mask + 1 : 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap + wcap;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = s < cap ? t1.keys[s] : t1w.khi[s - cap];
        if (k == kEmpty) continue;
        int t;
        if (pairs == 1) t = kl_len(k & ~kDerived, lb);
        else if (pairs == 2) t = (int)((t1w.klo[s - cap] >> 56) & 15);  // two-word pairs: (packed key, lang + 1)
        else t = (int)((k >> 56) & 15);
        atomicAdd(&h[t], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 16 && h[threadIdx.x]) atomicAdd(&out[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// Partial windows (Scala sliding: 0 < len < n gives the whole text once):
// a document shorter than some gram length adds, for every such n in
// gramLengths (duplicates included), one count of its whole text -- a key of
// len bytes, straight into T.  Its windows of lengths n <= len are its
// maximal windows' prefixes (emit / derive).
__global__ __launch_bounds__(256) void partial_kernel(const uint8_t* bytes, const int64_t* offsets, const int32_t* doc_lang,
                                                      const int64_t* docs, int64_t n_docs, const CountParams to,
                                                      const WideCountParams tow, const DeriveParams d) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_docs) return;
    const int64_t doc = docs[i];
    const int lang = doc_lang[doc];
    if (lang < 0 || lang >= to.L) return;
    const int64_t b = offsets[doc];
    const int len = (int)(offsets[doc + 1] - b);
    unsigned long long c = 0;
    for (int j = 0; j < d.n; ++j)
        if (d.len[j] > len) c += d.mult[j];
    if (len <= 0 || len > kMaxWideGram || !c) return;
    uint64_t lo = 0, hi = 0;
    for (int k = 0; k < len; ++k) {
        const uint64_t v = bytes[b + k];
        if (k < 8) lo |= v << (8 * k);
        else hi |= v << (8 * (k - 8));
    }
    if (len <= kMaxGram) add_count(to, lo | ((uint64_t)len << 56), lang, c);
    else wide_add(tow, lo, hi | ((uint64_t)len << 56), lang, c);
}

// ---- FIT v5: counting by sorting (ldgpu_fit.h SortFitParams).
// Emit: one wave per document (grid-stride), a lane per byte position; lanes
// read their window's 8 bytes from three dwords and store consecutive keys
// (coalesced).  A tail position (fewer than N bytes left) adds each gram
// length n <= its bytes left straight into T: about N^2 / 2 adds per
// document, next to the document's len sort keys.
__global__ __launch_bounds__(256) void sort_emit_kernel(const SortFitParams p, const CountParams to) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
    const int N = p.N;
    const int sh = 64 - 8 * N;
    uint64_t n_new = 0;
    for (int64_t doc = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; doc < p.n_docs; doc += nw) {
        const int64_t b = p.offsets[doc];
        const int64_t len = p.offsets[doc + 1] - b;
        const int lang = p.doc_lang[doc];
        const bool ok = lang >= 0 && lang < p.L;
        const uint64_t lk = ok ? (uint64_t)lang << (8 * N) : 0ull;
        uint64_t* out = p.keys + (b - p.base);
        for (int64_t q = lane; q < len; q += 64) {
            const int64_t a = b + q, i = a >> 2;
            const uint64_t lo = (uint64_t)ld_dw(W, i, p.last_dword) | ((uint64_t)ld_dw(W, i + 1, p.last_dword) << 32);
            const uint32_t s = (uint32_t)(a & 3) * 8u;
            const uint64_t v = s ? (lo >> s) | ((uint64_t)ld_dw(W, i + 2, p.last_dword) << (64u - s)) : lo;
            const int64_t rest = len - q;
            out[q] = ok && rest >= N ? lk | (__builtin_bswap64(v) >> sh) : kSortNone;
            if (ok && rest < N) {
                for (int j = 0; j < p.d.n && p.d.len[j] <= rest; ++j) {
                    const int n = p.d.len[j];
                    n_new += t_add_q(to, (v & byte_mask(n)) | ((uint64_t)n << 56), lang, p.d.mult[j]);
                }
            }
        }
    }
    t_flush(to, n_new);
}

// the common prefix of sorted keys a (at i) and b (at i - 1) in gram bytes:
// 0 when the language differs, N when the keys are equal.  Position i starts a
// run of every gram length n > common_prefix.
__device__ __forceinline__ int common_prefix(uint64_t a, uint64_t b, int N) {
    const uint64_t x = a ^ b;
    if (x >> (8 * N)) return 0;
    if (!x) return N;
    return (__builtin_clzll(x) - (64 - 8 * N)) >> 3;
}

__global__ __launch_bounds__(256) void runs_count_kernel(const uint64_t* keys, int64_t R, int N,
                                                         unsigned long long* runs) {
    __shared__ unsigned long long h[kMaxGram + 1];
    if (threadIdx.x <= kMaxGram) h[threadIdx.x] = 0ull;
    __syncthreads();
    uint32_t c[kMaxGram + 1] = {};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (int64_t)gridDim.x * blockDim.x) {
        const int cp = i == 0 ? 0 : common_prefix(keys[i], keys[i - 1], N);
#pragma unroll
        for (int n = 1; n <= kMaxGram; ++n) c[n] += cp < n ? 1u : 0u;
    }
#pragma unroll
    for (int n = 1; n <= kMaxGram; ++n) {
        uint32_t v = c[n];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&h[n], (unsigned long long)v);
    }
    __syncthreads();
    if (threadIdx.x >= 1 && threadIdx.x <= kMaxGram && threadIdx.x <= N && h[threadIdx.x])
        atomicAdd(&runs[threadIdx.x], h[threadIdx.x]);
}

// Runs of the gram lengths in lens: position i starts one of length n when
// its common prefix with position i - 1 (language included) is shorter than
// n bytes; the run ends at the next start.  The keys of a chunk of
// kScanIpt x kScanThreads positions are read once for every length of the
// pass.  Per length, the chunk keeps its starts as a bitmap in LDS, so most
// runs end within a few map words (the ~1-position runs of long grams, the
// short runs of middle lengths); a run that leaves the words searched is
// found by a galloping search from there (1, 2, 4, ... positions ahead, then
// bisection): O(log run) loads for the long runs of short grams.
// Compaction: one global atomic per chunk and length (block_place).
__global__ __launch_bounds__(kScanThreads) void sort_runs_kernel(const uint64_t* keys, int64_t R, int N,
                                                                 const RunLens lens, uint64_t* out_key,
                                                                 int32_t* out_lang, unsigned long long* out_cnt,
                                                                 unsigned long long* out_n) {
    constexpr int64_t kChunk = (int64_t)kScanIpt * kScanThreads;
    constexpr int kMapWords = (int)(kChunk / 32);
    constexpr int kScanWords = 8;  // map words searched for the next start before galloping
    __shared__ unsigned int wcnt[kScanIpt * (kScanThreads / 64)];
    __shared__ unsigned long long bbase;
    // one length's starts in the chunk, one bit per position (relative
    // position j * kScanThreads + thread), double-buffered: a wave still
    // reading one (chunk, length) step's map has passed no barrier of the next
    // step, which writes the other one
    __shared__ uint32_t smap[2][kMapWords];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int par = 0;
    for (int64_t c0 = (int64_t)blockIdx.x * kChunk; c0 < R; c0 += (int64_t)gridDim.x * kChunk) {
        // kScanIpt positions per thread, kScanThreads apart (coalesced)
        uint64_t key[kScanIpt];
        int cp[kScanIpt];
#pragma unroll
        for (int j = 0; j < kScanIpt; ++j) {
            const int64_t i = c0 + (int64_t)j * kScanThreads + threadIdx.x;
            key[j] = 0;
            cp[j] = N;  // past R: no start
            if (i < R) {
                key[j] = keys[i];
                cp[j] = i == 0 ? 0 : common_prefix(key[j], keys[i - 1], N);
            }
        }
        const int64_t cend = c0 + kChunk < R ? c0 + kChunk : R;
        for (int n = N; n >= 1; --n) {
            if (!((lens.mask >> n) & 1u)) continue;
            const int shift = 8 * (N - n);
            const uint32_t mult = lens.mult[n];
            uint32_t sm = 0;
#pragma unroll
            for (int j = 0; j < kScanIpt; ++j) sm |= cp[j] < n ? 1u << j : 0u;
            uint32_t* const map = smap[par];
            par ^= 1;
#pragma unroll
            for (int j = 0; j < kScanIpt; ++j) {
                const uint64_t m = __ballot((sm >> j) & 1u);
                if (lane < 2) map[(j * kScanThreads + wave * 64) / 32 + lane] = (uint32_t)(m >> (32 * lane));
            }
            uint32_t rel[kScanIpt];
            unsigned long long base;
            block_place(sm, out_n, wcnt, &bbase, rel, base);  // (its barriers publish the map)
#pragma unroll
            for (int j = 0; j < kScanIpt; ++j) {
                if (!((sm >> j) & 1u)) continue;
                const int r = j * kScanThreads + (int)threadIdx.x;
                const int64_t i = c0 + r;
                const uint64_t pk = key[j] >> shift;
                const unsigned long long o = base + rel[j];
                int64_t hi = -1;
                int w = r >> 5;
                uint32_t bits = (r & 31) == 31 ? 0u : map[w] & (~0u << ((r & 31) + 1));
                for (int k = 0;; ++k) {
                    if (bits) {
                        hi = c0 + 32 * w + __builtin_ctz(bits);
                        break;
                    }
                    if (++w == kMapWords || k == kScanWords) break;
                    bits = map[w];
                }
                if (hi < 0) {
                    // positions (i, c0 + 32 w) continue the run (no start among them)
                    int64_t lo = (c0 + 32 * (int64_t)w < cend ? c0 + 32 * (int64_t)w : cend) - 1;
                    hi = R;
                    for (int64_t step = 1; lo + step < R; step <<= 1) {
                        if ((keys[lo + step] >> shift) != pk) {
                            hi = lo + step;
                            break;
                        }
                        lo += step;
                    }
                    while (hi - lo > 1) {
                        const int64_t mid = lo + ((hi - lo) >> 1);
                        if ((keys[mid] >> shift) == pk) lo = mid;
                        else hi = mid;
                    }
                }
                out_key[o] = __builtin_bswap64((pk & byte_mask(n)) << (64 - 8 * n)) | ((uint64_t)n << 56);
                out_lang[o] = (int32_t)(pk >> (8 * n));
                out_cnt[o] = (unsigned long long)(hi - i) * mult;
            }
        }
    }
}

#ifndef LDGPU_RUNS_UNIQ
#define LDGPU_RUNS_UNIQ 1
#endif
// (key, language, count) entries into T, grid-stride; the new-key counters
// once per thread (t_flush)
__global__ __launch_bounds__(256) void runs_add_kernel(const CountParams p, const uint64_t* keys, const int32_t* lang,
                                                       const unsigned long long* cnt, int64_t n) {
    uint64_t n_new = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        n_new += t_add_q<LDGPU_RUNS_UNIQ>(p, keys[i], lang[i], cnt[i]);
    t_flush(p, n_new);
}

}  // namespace

hipError_t launch_sort_emit(const SortFitParams& p, const CountParams& to, hipStream_t stream) {
    if (p.n_docs <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>(65536, (p.n_docs + 3) / 4);
    hipLaunchKernelGGL(sort_emit_kernel, dim3(g), dim3(256), 0, stream, p, to);
    return hipGetLastError();
}

hipError_t sort_keys_u64(int64_t n, uint64_t* keys, uint64_t* alt, int bits, void* tmp, size_t* tmp_bytes,
                         bool* in_alt, hipStream_t stream) {
    hipcub::DoubleBuffer<uint64_t> kb(keys, alt);
    if (n > INT32_MAX) return hipErrorInvalidValue;
    hipError_t e = hipcub::DeviceRadixSort::SortKeys(tmp, *tmp_bytes, kb, (int)n, 0, bits, stream);
    if (in_alt) *in_alt = kb.Current() == alt;
    return e;
}

hipError_t launch_runs_count(const uint64_t* keys, int64_t R, int N, unsigned long long* runs, hipStream_t stream) {
    if (R <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>(4096, (R + 255) / 256);
    hipLaunchKernelGGL(runs_count_kernel, dim3(g), dim3(256), 0, stream, keys, R, N, runs);
    return hipGetLastError();
}

hipError_t launch_sort_runs(const uint64_t* keys, int64_t R, int N, const RunLens& lens, uint64_t* out_key,
                            int32_t* out_lang, unsigned long long* out_cnt, unsigned long long* out_n,
                            hipStream_t stream) {
    if (R <= 0) return hipSuccess;
    hipLaunchKernelGGL(sort_runs_kernel, dim3(scan_grid_ipt((uint64_t)R)), dim3(kScanThreads), 0, stream, keys, R, N,
                       lens, out_key, out_lang, out_cnt, out_n);
    return hipGetLastError();
}

hipError_t launch_runs_add(const CountParams& p, const uint64_t* keys, const int32_t* lang, const unsigned long long* cnt,
                           int64_t n, int cus, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>((int64_t)cus * 8, (n + 255) / 256);
    hipLaunchKernelGGL(runs_add_kernel, dim3(g), dim3(256), 0, stream, p, keys, lang, cnt, n);
    return hipGetLastError();
}

size_t emit_lds_bytes(int K) {
    return K == 1 ? sizeof(EmitLds<1>) : (K == 2 ? sizeof(EmitLds<2>) : sizeof(EmitLds<3>));
}

size_t reduce_lds_bytes(int K) {
    const size_t N = K == 1 ? agg_slots<1>() : (K == 2 ? agg_slots<2>() : agg_slots<3>());
    return K == 1 ? ((N * (8 + 4) + 4 + 15) & ~(size_t)15) + (LDGPU_RED_BRANCHLESS ? 8 * (size_t)kRedDummy : 16)
                  : N * (8 * (size_t)(K - 1) + 12) + 16;
}

hipError_t fit3_prepare(int K) {
    const void* e = K == 1 ? (const void*)&emit_kernel<1> : (K == 2 ? (const void*)&emit_kernel<2> : (const void*)&emit_kernel<3>);
    const void* r =
        K == 1 ? (const void*)&reduce_kernel<1> : (K == 2 ? (const void*)&reduce_kernel<2> : (const void*)&reduce_kernel<3>);
    hipError_t x = hipFuncSetAttribute(e, hipFuncAttributeMaxDynamicSharedMemorySize, (int)emit_lds_bytes(K));
    if (x == hipSuccess) x = hipFuncSetAttribute(r, hipFuncAttributeMaxDynamicSharedMemorySize, (int)reduce_lds_bytes(K));
    return x;
}

hipError_t launch_emit(int K, const PartParams& p, hipStream_t stream) {
    const dim3 g(p.grid_a), b(kEmitWaves * 64);
    if (K == 1) hipLaunchKernelGGL(emit_kernel<1>, g, b, emit_lds_bytes(1), stream, p);
    else if (K == 2) hipLaunchKernelGGL(emit_kernel<2>, g, b, emit_lds_bytes(2), stream, p);
    else hipLaunchKernelGGL(emit_kernel<3>, g, b, emit_lds_bytes(3), stream, p);
    return hipGetLastError();
}

hipError_t launch_fit_offsets(const PartParams& p, hipStream_t stream) {
    hipLaunchKernelGGL(fit_offsets_kernel, dim3(1), dim3(1024), 0, stream, p.cnt3, const_cast<uint64_t*>(p.p2off),
                       const_cast<uint64_t*>(p.boff));
    return hipGetLastError();
}

hipError_t launch_part2(int K, const PartParams& p, hipStream_t stream) {
    const dim3 g(kQ * kSplits), b(kEmitWaves * 64);
    if (K == 1) hipLaunchKernelGGL(part2_kernel<1>, g, b, 0, stream, p);
    else if (K == 2) hipLaunchKernelGGL(part2_kernel<2>, g, b, 0, stream, p);
    else hipLaunchKernelGGL(part2_kernel<3>, g, b, 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_reduce(int K, const PartParams& p, hipStream_t stream) {
    const dim3 g(kQ * kQ), b(kEmitWaves * 64);
    if (K == 1) hipLaunchKernelGGL(reduce_kernel<1>, g, b, reduce_lds_bytes(1), stream, p);
    else if (K == 2) hipLaunchKernelGGL(reduce_kernel<2>, g, b, reduce_lds_bytes(2), stream, p);
    else hipLaunchKernelGGL(reduce_kernel<3>, g, b, reduce_lds_bytes(3), stream, p);
    return hipGetLastError();
}

hipError_t launch_merge(int K, const PartParams& p, const CountParams& c, const WideCountParams& w, int b0, int b1,
                        bool pairs, hipStream_t stream) {
    if (b1 <= b0) return hipSuccess;
    const dim3 g((unsigned)(b1 - b0)), b(1024);
    const int pr = pairs && K <= 2;
    if (K == 1) hipLaunchKernelGGL(merge_kernel<1>, g, b, 0, stream, p, c, w, b0, pr);
    else if (K == 2) hipLaunchKernelGGL(merge_kernel<2>, g, b, 0, stream, p, c, w, b0, pr);
    else hipLaunchKernelGGL(merge_kernel<3>, g, b, 0, stream, p, c, w, b0, 0);
    return hipGetLastError();
}

hipError_t launch_derive_level(const CountParams& t1, const WideCountParams& t1w, bool wide, uint64_t s0, uint64_t s1,
                               int lev, uint32_t mt, const CountParams& to, const WideCountParams& tow,
                               hipStream_t stream) {
    if (s1 <= s0) return hipSuccess;
    const unsigned g = (unsigned)std::min<uint64_t>(16384, (s1 - s0 + 255) / 256);
    hipLaunchKernelGGL(derive_level_kernel, dim3(g), dim3(256), 0, stream, t1, t1w, (int)wide, s0, s1, lev, mt, to,
                       tow);
    return hipGetLastError();
}

hipError_t launch_len_hist(const CountParams& t1, const WideCountParams& t1w, int pairs, uint32_t lb,
                           unsigned long long* out, hipStream_t stream) {
    const uint64_t n = t1.mask + 1 + (t1w.klo ? t1w.mask + 1 : 0);
    const unsigned g = (unsigned)std::min<uint64_t>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(len_hist_kernel, dim3(g), dim3(256), 0, stream, t1, t1w, (int)pairs, lb, out);
    return hipGetLastError();
}

hipError_t launch_derive_pairs2_level(const WideCountParams& t1w, uint64_t s0, uint64_t s1, int lev, uint32_t mt,
                                      const CountParams& to, const WideCountParams& nx, int ablate,
                                      hipStream_t stream) {
    if (s1 <= s0) return hipSuccess;
    const unsigned g = (unsigned)std::min<uint64_t>(16384, (s1 - s0 + 255) / 256);
    hipLaunchKernelGGL(derive_pairs2_level_kernel, dim3(g), dim3(256), 0, stream, t1w, s0, s1, lev, mt, to, nx,
                       ablate);
    return hipGetLastError();
}

hipError_t launch_derive_pairs_level(const CountParams& t1, uint32_t lb, uint64_t s0, uint64_t s1, int lev, uint32_t mt,
                                     const CountParams& to, int ablate, hipStream_t stream) {
    if (s1 <= s0) return hipSuccess;
    const unsigned g = (unsigned)std::min<uint64_t>(16384, (s1 - s0 + 255) / 256);
    hipLaunchKernelGGL(derive_pairs_level_kernel, dim3(g), dim3(256), 0, stream, t1, lb, s0, s1, lev, mt, to, ablate);
    return hipGetLastError();
}

hipError_t launch_partial(const uint8_t* bytes, const int64_t* offsets, const int32_t* doc_lang, const int64_t* docs,
                          int64_t n_docs, const CountParams& to, const WideCountParams& tow, const DeriveParams& d,
                          hipStream_t stream) {
    if (n_docs <= 0) return hipSuccess;
    hipLaunchKernelGGL(partial_kernel, dim3((unsigned)((n_docs + 255) / 256)), dim3(256), 0, stream, bytes, offsets,
                       doc_lang, docs, n_docs, to, tow, d);
    return hipGetLastError();
}

}  // namespace ldgpu
