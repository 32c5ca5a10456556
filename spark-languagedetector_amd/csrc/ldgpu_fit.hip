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
// Two counting paths share the table: FIT v2 (emit / part2 / reduce /
// merge, below: radix-partitioned record aggregation, one table add per
// distinct (gram, language) per batch -- the path every table whose
// (gram, language, count) record fits 64 bits takes) and the single-pass
// count_kernel here (tables whose record does not fit, e.g. 7-byte grams with
// hundreds of languages; diagnostics builds force it: LDGPU_FIT_LEGACY).  count_kernel:
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

#include "ldgpu_internal.h"

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

__device__ __forceinline__ unsigned long long block_compact(bool occ, unsigned long long* out_n, unsigned int* wcnt,
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
        *bbase = acc ? atomicAdd(out_n, (unsigned long long)acc) : 0ull;
    }
    __syncthreads();
    const unsigned long long o = *bbase + wcnt[wave] +
                                 __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    __syncthreads();  // wcnt / bbase are reused by the next chunk
    return o;
}

// find-or-insert; returns the slot or -1 when the probe limit is reached
__device__ __forceinline__ int64_t find_or_insert(const CountParams& p, uint64_t key, bool& new_key) {
    uint64_t s = mix64(key) >> p.shift;
    for (int probe = 0; probe < kMaxProbe; ++probe) {
        uint64_t k = __hip_atomic_load(&p.keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

__device__ __forceinline__ void add_count(const CountParams& p, uint64_t key, int lang, unsigned long long c) {
    if (LDGPU_FIT_ABLATE & 2) return;
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
    uint64_t s = mix64(key) >> to.shift;
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

}  // namespace

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
// build's (length, bytes) rule.  The device computes masks, k and the
// (language, k) histogram; the host turns the histogram into a threshold
// class per language; the device flags every gram below a threshold and
// emits the threshold-class candidates, whose (length, bytes) order the host
// resolves with nth_element.
namespace ldgpu {
namespace {

// grid-stride over the table in chunks of kScanThreads slots; the (language,
// k) histogram in LDS (L <= 88), flushed once per block
__global__ __launch_bounds__(kScanThreads) void presence_kernel(const CountParams p, uint64_t cap, int S,
                                                                uint64_t* out_keys, uint64_t* out_masks,
                                                                int32_t* out_k, unsigned long long* out_n,
                                                                unsigned int* hist) {
    extern __shared__ unsigned int lhist[];
    __shared__ unsigned int wcnt[kScanThreads / 64];
    __shared__ unsigned long long bbase;
    const int L = p.L;
    const bool lds_hist = L <= 88;  // L * (L + 1) * 4 B <= 31 KiB
    if (lds_hist) {
        for (int i = threadIdx.x; i < L * (L + 1); i += blockDim.x) lhist[i] = 0u;
        __syncthreads();
    }
    for (uint64_t c0 = (uint64_t)blockIdx.x * kScanThreads; c0 < cap; c0 += (uint64_t)gridDim.x * kScanThreads) {
        const uint64_t i = c0 + threadIdx.x;
        const bool occ = i < cap && p.keys[i] != kEmpty;
        const unsigned long long o = block_compact(occ, out_n, wcnt, &bbase);
        if (!occ) continue;
        const unsigned long long* row = p.counts + i * L;
        // the row's presence bits, 64 languages a word, 8 counters per batch of
        // independent loads; then the histogram from the bits (one read of the row)
        int k = 0;
        for (int s = 0; s < S; ++s) {
            const int l0 = 64 * s, nl = min(64, L - l0);
            uint64_t w = 0;
            for (int b0 = 0; b0 < nl; b0 += 8) {
                unsigned long long v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = b0 + u < nl ? row[l0 + b0 + u] : 0ull;
#pragma unroll
                for (int u = 0; u < 8; ++u) w |= (uint64_t)(v[u] != 0ull) << (b0 + u);
            }
            out_masks[o * S + s] = w;
            k += __popcll(w);
        }
        out_keys[o] = p.keys[i];
        out_k[o] = k;
        for (int s = 0; s < S; ++s) {
            uint64_t w = out_masks[o * S + s];
            while (w) {
                const int l = 64 * s + __builtin_ctzll(w);
                w &= w - 1;
                if (lds_hist)
                    atomicAdd(&lhist[l * (L + 1) + k], 1u);
                else
                    atomicAdd(&hist[l * (L + 1) + k], 1u);
            }
        }
    }
    if (lds_hist) {
        __syncthreads();
        for (int t = threadIdx.x; t < L * (L + 1); t += blockDim.x)
            if (lhist[t]) atomicAdd(&hist[t], lhist[t]);
    }
}

__global__ void select_kernel(int64_t n, int L, int S, const uint64_t* keys, const uint64_t* masks, const int32_t* ks,
                              const int32_t* kstar, const int32_t* need, uint8_t* chosen, int32_t* cand_lang,
                              uint64_t* cand_key, uint32_t* cand_idx, unsigned int* cand_n) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int k = ks[j];
    uint8_t ch = 0;
    for (int s = 0; s < S; ++s) {
        uint64_t w = masks[j * S + s];
        while (w) {
            const int l = s * 64 + __builtin_ctzll(w);
            w &= w - 1;
            if (k < kstar[l]) {
                ch = 1;
            } else if (k == kstar[l] && need[l] > 0) {
                const unsigned int at = atomicAdd(cand_n, 1u);
                cand_lang[at] = l;
                cand_key[at] = sort_key(keys[j]);
                cand_idx[at] = (uint32_t)j;
            }
        }
    }
    chosen[j] = ch;
}

__global__ void mark_kernel(const uint32_t* idx, int64_t n, uint8_t* chosen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) chosen[idx[i]] = 1;
}

__global__ __launch_bounds__(kScanThreads) void gather_chosen_kernel(int64_t n, int S, const uint8_t* chosen,
                                                                     const uint64_t* keys, const uint64_t* masks,
                                                                     const int32_t* ks, uint64_t* out_keys,
                                                                     uint64_t* out_masks, int32_t* out_k,
                                                                     unsigned long long* out_n) {
    __shared__ unsigned int wcnt[kScanThreads / 64];
    __shared__ unsigned long long bbase;
    for (int64_t c0 = (int64_t)blockIdx.x * kScanThreads; c0 < n; c0 += (int64_t)gridDim.x * kScanThreads) {
        const int64_t j = c0 + threadIdx.x;
        const bool c = j < n && chosen[j];
        const unsigned long long o = block_compact(c, out_n, wcnt, &bbase);
        if (!c) continue;
        out_keys[o] = keys[j];
        out_k[o] = ks[j];
        for (int s = 0; s < S; ++s) out_masks[o * S + s] = masks[j * S + s];
    }
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

hipError_t launch_mark_threshold(int64_t n, const int32_t* cand_lang, const uint64_t* cand_key,
                                 const uint32_t* cand_idx, const uint64_t* thr, uint8_t* chosen, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mark_threshold_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, n, cand_lang, cand_key,
                       cand_idx, thr, chosen);
    return hipGetLastError();
}

hipError_t launch_presence(const CountParams& p, uint64_t cap, int S, uint64_t* out_keys, uint64_t* out_masks,
                           int32_t* out_k, unsigned long long* out_n, unsigned int* hist, hipStream_t stream) {
    const size_t lds = p.L <= 88 ? (size_t)p.L * (p.L + 1) * 4 : 0;
    hipLaunchKernelGGL(presence_kernel, dim3(scan_grid(cap)), dim3(kScanThreads), lds, stream, p, cap, S, out_keys, out_masks,
                       out_k, out_n, hist);
    return hipGetLastError();
}

hipError_t launch_select(int64_t n, int L, int S, const uint64_t* keys, const uint64_t* masks, const int32_t* ks,
                         const int32_t* kstar, const int32_t* need, uint8_t* chosen, int32_t* cand_lang,
                         uint64_t* cand_key, uint32_t* cand_idx, unsigned int* cand_n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(select_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, n, L, S, keys, masks, ks, kstar,
                       need, chosen, cand_lang, cand_key, cand_idx, cand_n);
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

hipError_t launch_gather_chosen(int64_t n, int S, const uint8_t* chosen, const uint64_t* keys, const uint64_t* masks,
                                const int32_t* ks, uint64_t* out_keys, uint64_t* out_masks, int32_t* out_k,
                                unsigned long long* out_n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_chosen_kernel, dim3(scan_grid((uint64_t)n)), dim3(kScanThreads), 0, stream, n, S, chosen,
                       keys, masks, ks, out_keys, out_masks, out_k, out_n);
    return hipGetLastError();
}

}  // namespace ldgpu

// ---------------------------------------------------------------------------
// FIT v2: radix-partitioned record aggregation -- the north star's "LDS-
// privatised histogram, then a sort / segmented-reduce merge into HBM count
// tables", built so that the global table sees ONE add per distinct
// (gram, language) per batch instead of one device-scope atomic per window
// (which bounded the single-pass count_kernel above: ~2.7e9 random atomics
// per GiB).  Per batch of documents:
//   emit    one wave per document: 1-byte windows into a per-wave LDS
//           histogram, 2-/3-byte windows into a per-wave LDS hash (both
//           flushed per document / gram length as counted records), longer
//           windows straight to records.  Records gather in a workgroup LDS
//           block; a full block is counting-sorted by q1 in LDS and written
//           once, coalesced, into the workgroup's own region with a header
//           of q1 starts.  The workgroup also histograms (q1, q2).
//   part2   bucket q1 of one emit group: the group's q1 runs (load-balanced
//           over a wave) are re-scattered by q2 to exact, host-scanned
//           offsets -- 4096 contiguous buckets (q1, q2).
//   reduce  one workgroup per bucket: an LDS hash (kAggSlots entries) sums
//           the counts of equal (gram, language) records; distinct entries
//           go out as (kl, count).
//   merge   each entry is one find-or-insert + one u64 add in the table.
// Integer sums are order-independent: counts stay bit-exact.
namespace ldgpu {
namespace {

__device__ __forceinline__ bool emit_ablated(const PartParams& p, int bit) { return LDGPU_DIAG && (p.ablate & bit); }

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t make_rec(uint64_t bytes, int klen, uint32_t lang, uint64_t c, uint32_t lb,
                                             uint32_t cb) {
    const uint64_t sent = (1ull << (8 * klen)) | bytes;
    return (((sent << lb) | (uint64_t)lang) << cb) | c;
}

// the packed gram key (ldgpu_common.h) of a record's kl = record >> cb
__device__ __forceinline__ uint64_t kl_key(uint64_t kl, uint32_t lb) {
    const uint64_t sent = kl >> lb;
    const int klen = (63 - __builtin_clzll(sent)) >> 3;
    return (sent ^ (1ull << (8 * klen))) | ((uint64_t)klen << 56);
}

__device__ __forceinline__ uint32_t q1_of(uint64_t r, uint32_t cb) { return (uint32_t)(mix64(r >> cb) >> (64 - kQBits)); }
__device__ __forceinline__ uint32_t q2_of(uint64_t r, uint32_t cb) {
    return (uint32_t)(mix64(r >> cb) >> (64 - 2 * kQBits)) & (kQ - 1);
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

// emit's per-wave LDS table of a document's 2-byte windows: 1024 packed
// slots (16-bit key, 16-bit count), so a document's few hundred distinct
// 2-grams probe short chains; documents of 64 Ki bytes or more skip it (a
// count must stay below 0xffff)
constexpr uint32_t kK2 = 1024;
constexpr uint32_t kK2Empty = 0xffffffffu;
constexpr int kK2Probe = 16;
constexpr int64_t kK2MaxDoc = 0xffff;

struct EmitLds {
    uint64_t blk[kBlkRecs];
    uint32_t hist2[kQ * kQ];
    uint32_t h1[kEmitWaves][256];
    uint32_t k2[kEmitWaves][kK2];      // per-document 2-gram counts: key << 16 | count, kK2Empty = free
    uint32_t pcnt[kQ];
    uint32_t pfill[kQ];
    uint32_t pstart[kQ + 1];
    uint32_t blk_n;
    uint32_t active;
    uint32_t next_doc;
};

enum { kNextDoc = 0, kWin = 1, kHFlush = 2, kH1Flush = 3, kDone = 4 };

// one wave's position in its current document (wave-uniform)
struct WaveState {
    int64_t b, len, p0;
    int32_t lang, gi, phase, cursor;
    uint32_t used1;
    bool pf;                     // pw holds the words of the next WIN step (issued a round early)
    uint32_t pw[4][3];
};

// append the lanes' records (kSub per lane) to the workgroup block with one
// reservation (the round bound keeps it from overflowing); every lane of the
// wave must be active
constexpr int kSubW = 4;  // window positions (or flushed slots) per lane per step

__device__ __forceinline__ void emit_recs(EmitLds& S, const bool (&has)[kSubW], const uint64_t (&r)[kSubW],
                                          int lane) {
    uint64_t m[kSubW];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < kSubW; ++k) {
        m[k] = __ballot(has[k]);
        tot += (uint32_t)__popcll(m[k]);
    }
    if (!tot) return;
    uint32_t base = 0;
    if (lane == 0) base = __hip_atomic_fetch_add(&S.blk_n, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    base = __shfl(base, 0);
#pragma unroll
    for (int k = 0; k < kSubW; ++k) {
        if (has[k]) S.blk[base + lane_rank(m[k])] = r[k];
        base += (uint32_t)__popcll(m[k]);
    }
}

__device__ __forceinline__ void next_gram(const PartParams& p, WaveState& w) {
    w.gi += 1;
    w.p0 = 0;
    w.cursor = 0;
    w.phase = w.gi < p.nG ? kWin : (w.used1 ? kH1Flush : kNextDoc);
}

// the dwords of the kSubW positions of a WIN step at (gi, p0)
__device__ __forceinline__ void window_loads(const PartParams& p, const WaveState& w, int lane,
                                             uint32_t (&pw)[4][3]) {
    const int n = p.G[w.gi];
    const int64_t nwin = n_windows(w.len, n);
    const int klen = w.len < n ? (int)w.len : n;
    const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
#pragma unroll
    for (int k = 0; k < kSubW; ++k) {
        const int64_t pos = w.p0 + 64 * k + lane;
        const int64_t a = w.b + (pos < nwin ? pos : 0);
        const int64_t i = a >> 2;
        pw[k][0] = ld_dw(W, i, p.last_dword);
        pw[k][1] = ld_dw(W, i + 1, p.last_dword);
        pw[k][2] = klen > 4 ? ld_dw(W, i + 2, p.last_dword) : 0u;
    }
}

// One step of a wave: <= 64 kSubW windows or flushed slots, <= 64 kSubW
// records.  The positions' loads are all issued before any is used.
__device__ __forceinline__ void emit_step(const PartParams& p, EmitLds& S, WaveState& w, int wave, int lane,
                                          int64_t d0, int64_t d1) {
    const uint64_t cmax = p.cb >= 32 ? 0xffffffffull : ((1ull << p.cb) - 1ull);
    uint32_t* h1 = S.h1[wave];
    uint32_t* k2 = S.k2[wave];
    if (w.phase == kNextDoc) {
        uint32_t k = 0;
        if (lane == 0) k = __hip_atomic_fetch_add(&S.next_doc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int64_t d = d0 + (int64_t)__shfl(k, 0);
        if (d >= d1) {
            w.phase = kDone;
            if (lane == 0) __hip_atomic_fetch_sub(&S.active, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        const int lang = p.doc_lang[d];
        if (lang < 0 || lang >= p.L) return;  // reduceGrams keeps supported languages only
        const int64_t b = p.offsets[d];
        const int64_t len = p.offsets[d + 1] - b;
        if (len <= 0 || p.nG == 0) return;
        w.b = b;
        w.len = len;
        w.lang = lang;
        w.gi = 0;
        w.p0 = 0;
        w.cursor = 0;
        w.used1 = 0;
        w.pf = false;
        w.phase = kWin;
        // fall through: the document's first windows in this step
    }
    bool has[kSubW];
    uint64_t r[kSubW];
#pragma unroll
    for (int k = 0; k < kSubW; ++k) {
        has[k] = false;
        r[k] = 0;
    }
    if (w.phase == kWin) {
        const int n = p.G[w.gi];
        const int64_t nwin = n_windows(w.len, n);
        const int klen = w.len < n ? (int)w.len : n;
        const uint32_t lomask = klen >= 4 ? 0xffffffffu : ((1u << (8 * klen)) - 1u);
        const uint32_t himask = klen <= 4 ? 0u : ((1u << (8 * (klen - 4))) - 1u);
        uint32_t lo[kSubW], hi[kSubW];
        bool valid[kSubW];
        if (!w.pf) window_loads(p, w, lane, w.pw);
        w.pf = false;
#pragma unroll
        for (int k = 0; k < kSubW; ++k) {
            const int64_t pos = w.p0 + 64 * k + lane;
            valid[k] = pos < nwin;
            const uint32_t sh = (uint32_t)((w.b + (valid[k] ? pos : 0)) & 3);
            lo[k] = __builtin_amdgcn_alignbyte(w.pw[k][1], w.pw[k][0], sh) & lomask;
            hi[k] = __builtin_amdgcn_alignbyte(w.pw[k][2], w.pw[k][1], sh) & himask;
        }
        if (klen == 1) {
#pragma unroll
            for (int k = 0; k < kSubW; ++k)
                if (valid[k]) __hip_atomic_fetch_add(&h1[lo[k]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            w.used1 = 1;
        } else if (klen == 2 && w.len < kK2MaxDoc && !emit_ablated(p, 1)) {
            // the kSubW positions probe together: one LDS round trip per
            // probe step for all of them (most find their key at once)
            uint32_t slot[kSubW];
            bool pend[kSubW];
#pragma unroll
            for (int k = 0; k < kSubW; ++k) {
                slot[k] = (uint32_t)(((uint64_t)(lo[k] * 0x9E3779B1u) * kK2) >> 32);
                pend[k] = valid[k];
            }
            for (int t = 0; t < kK2Probe; ++t) {
                uint32_t cur[kSubW];
#pragma unroll
                for (int k = 0; k < kSubW; ++k) cur[k] = pend[k] ? k2[slot[k]] : 0u;
                bool any = false;
#pragma unroll
                for (int k = 0; k < kSubW; ++k) {
                    if (!pend[k]) continue;
                    if (cur[k] == kK2Empty &&
                        atomicCAS(&k2[slot[k]], kK2Empty, (lo[k] << 16) | 1u) == kK2Empty) {
                        pend[k] = false;  // inserted with count 1
                        continue;
                    }
                    if (cur[k] == kK2Empty) cur[k] = k2[slot[k]];  // lost the race: see who won
                    if ((cur[k] >> 16) == lo[k]) {
                        __hip_atomic_fetch_add(&k2[slot[k]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        pend[k] = false;
                    } else {
                        slot[k] = (slot[k] + 1u) & (kK2 - 1u);
                        any = true;
                    }
                }
                if (!__ballot(any)) break;
            }
#pragma unroll
            for (int k = 0; k < kSubW; ++k) {
                if (pend[k]) {  // no slot: the window goes out as a record
                    has[k] = true;
                    r[k] = make_rec(lo[k], klen, (uint32_t)w.lang, 1, p.lb, p.cb);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < kSubW; ++k) {
                has[k] = valid[k];
                r[k] = make_rec(((uint64_t)hi[k] << 32) | lo[k], klen, (uint32_t)w.lang, 1, p.lb, p.cb);
            }
        }
        if (emit_ablated(p, 4)) {
#pragma unroll
            for (int k = 0; k < kSubW; ++k) has[k] = false;
        }
        emit_recs(S, has, r, lane);
        w.p0 += 64 * kSubW;
        if (w.p0 >= nwin) {
            __builtin_amdgcn_wave_barrier();
            if (klen == 2 && w.len < kK2MaxDoc && !emit_ablated(p, 1)) {
                w.phase = kHFlush;
                w.cursor = 0;
            } else {
                next_gram(p, w);
            }
        }
        if (w.phase == kWin) {  // the next step's loads fly across the round barrier
            window_loads(p, w, lane, w.pw);
            w.pf = true;
        }
        return;
    }
    if (w.phase == kHFlush) {  // this gram length's 2-byte keys, 64 kSubW slots a step
#pragma unroll
        for (int k = 0; k < kSubW; ++k) {
            const uint32_t slot = (uint32_t)w.cursor + 64u * k + lane;
            const uint32_t v = k2[slot];
            if (v == kK2Empty) continue;
            k2[slot] = kK2Empty;
            const uint32_t c = v & 0xffffu;
            if (c <= cmax) {
                has[k] = true;
                r[k] = make_rec(v >> 16, 2, (uint32_t)w.lang, c, p.lb, p.cb);
            } else {
                add_count(p.direct, (2ull << 56) | (uint64_t)(v >> 16), w.lang, c);
            }
        }
        emit_recs(S, has, r, lane);
        w.cursor += 64 * kSubW;
        if (w.cursor >= (int)kK2) {
            __builtin_amdgcn_wave_barrier();
            next_gram(p, w);
            if (w.phase == kWin) {
                window_loads(p, w, lane, w.pw);
                w.pf = true;
            }
        }
        return;
    }
    if (w.phase == kH1Flush) {  // the document's 1-byte keys (256 bins: one step)
#pragma unroll
        for (int k = 0; k < kSubW; ++k) {
            const int bin = 64 * k + lane;
            const uint32_t c = h1[bin];
            if (!c) continue;
            h1[bin] = 0u;
            if (c <= cmax) {
                has[k] = true;
                r[k] = make_rec((uint64_t)bin, 1, (uint32_t)w.lang, c, p.lb, p.cb);
            } else {
                add_count(p.direct, (1ull << 56) | (uint64_t)bin, w.lang, c);
            }
        }
        emit_recs(S, has, r, lane);
        __builtin_amdgcn_wave_barrier();
        w.used1 = 0;
        w.phase = kNextDoc;
    }
}

// Write the block: counting sort by q1 in LDS, scattered stores into the
// block's own contiguous range (the lines fill in L2 and leave whole).
__device__ __forceinline__ void flush_block(const PartParams& p, EmitLds& S, uint32_t n, int64_t rb, int64_t gid,
                                            int tid) {
    for (uint32_t i = tid; i < n; i += kEmitWaves * 64) {
        const uint64_t h = mix64(S.blk[i] >> p.cb);
        const uint32_t q1 = (uint32_t)(h >> (64 - kQBits));
        const uint32_t q2 = (uint32_t)(h >> (64 - 2 * kQBits)) & (kQ - 1);
        __hip_atomic_fetch_add(&S.pcnt[q1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&S.hist2[q1 * kQ + q2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    lds_barrier();
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
        const uint64_t r = S.blk[i];
        const uint32_t at =
            __hip_atomic_fetch_add(&S.pfill[q1_of(r, p.cb)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (!emit_ablated(p, 2)) p.rec[rb + at] = r;
    }
    if (tid <= kQ) p.blk_hdr[(size_t)gid * kHdr + tid] = S.pstart[tid];
    if (tid == 0) {
        p.blk_start[gid] = rb;
        S.blk_n = 0u;
    }
    lds_barrier();
}

__global__ __launch_bounds__(kEmitWaves * 64, 1) void emit_kernel(const PartParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t emit_smem[];
    EmitLds& S = *reinterpret_cast<EmitLds*>(emit_smem);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = blockIdx.x;
    const int64_t d0 = p.wg_doc[bid], d1 = p.wg_doc[bid + 1];
    const int64_t rbase = p.wg_rec[bid], dbase = p.wg_dir[bid];
    for (int i = tid; i < kQ * kQ; i += kEmitWaves * 64) S.hist2[i] = 0u;
    for (int i = lane; i < 256; i += 64) S.h1[wave][i] = 0u;
    for (int i = lane; i < (int)kK2; i += 64) S.k2[wave][i] = kK2Empty;
    if (tid < kQ) S.pcnt[tid] = 0u;
    if (tid == 0) {
        S.blk_n = 0u;
        S.active = kEmitWaves;
        S.next_doc = 0u;
    }
    lds_barrier();
    WaveState w{};
    w.phase = kNextDoc;
    int64_t written = 0;
    int64_t nb = 0;
    for (;;) {
        // a round: every live wave takes one step (<= 64 kSubW records, so the
        // block, flushed above kBlkRecs - kRoundRecs, never overflows)
        if (w.phase != kDone) emit_step(p, S, w, wave, lane, d0, d1);
        lds_barrier();
        const uint32_t n = S.blk_n;
        const uint32_t act = S.active;
        lds_barrier();  // every thread has read n / act before the next round moves them
        if (n > (uint32_t)(kBlkRecs - kRoundRecs) || (act == 0u && n > 0u)) {
            flush_block(p, S, n, rbase + written, dbase + nb, tid);
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

struct Part2Lds {
    uint32_t cur[kQ];
    int32_t gpre[257];
};

__device__ __forceinline__ int64_t rdlane_i64(int64_t v, int l) {
    return (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l) << 32));
}

__global__ __launch_bounds__(kEmitWaves * 64) void part2_kernel(const PartParams p) {
    __shared__ Part2Lds S;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
    }
    if (tid < kQ) S.cur[tid] = 0u;
    __syncthreads();
    const int64_t tb = S.gpre[per];
    for (int64_t u0 = (int64_t)wave * 64; u0 < tb; u0 += kEmitWaves * 64) {
        const int64_t u = u0 + lane;
        int64_t start = 0;
        uint32_t len = 0;
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
            start = p.blk_start[gid] + a;
            len = e - a;
        }
        // the chunk's 64 runs, kR at a time: the wave loads the runs' records
        // cooperatively (runs average kBlkRecs / kQ records), kR loads in flight
        constexpr int kR = 8;
        for (int i = 0; i < 64; i += kR) {
            int64_t st[kR];
            uint32_t ln[kR];
            uint32_t lm = 0;
#pragma unroll
            for (int k = 0; k < kR; ++k) {
                st[k] = rdlane_i64(start, i + k);
                ln[k] = (uint32_t)__builtin_amdgcn_readlane((int)len, i + k);
                lm = ln[k] > lm ? ln[k] : lm;
            }
            for (uint32_t j = lane; j < ((lm + 63u) & ~63u); j += 64) {
                uint64_t r[kR];
#pragma unroll
                for (int k = 0; k < kR; ++k) r[k] = j < ln[k] ? p.rec[st[k] + j] : 0ull;
#pragma unroll
                for (int k = 0; k < kR; ++k) {
                    if (j < ln[k]) {
                        const uint32_t q2 = q2_of(r[k], p.cb);
                        const uint32_t at =
                            __hip_atomic_fetch_add(&S.cur[q2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        p.rec2[p.p2off[(q1 * kQ + q2) * kSplits + s] + at] = r[k];
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// distinct (kl, count) out: bucket b writes its entries from boff[b] on (it
// has at most as many as records), through a workgroup-local counter -- one
// global counter for every bucket's appends would serialise ~0.5M atomics
// per batch on one address
__device__ __forceinline__ void out_append(const PartParams& p, uint32_t* n_out, int64_t base, bool has, uint64_t kl,
                                           uint32_t c, int lane) {
    const uint64_t m = __ballot(has);
    if (!m) return;
    uint32_t at = 0;
    if (lane == 0) at = __hip_atomic_fetch_add(n_out, (uint32_t)__popcll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    at = __shfl(at, 0);
    if (has) {
        const int64_t o = base + at + lane_rank(m);
        p.out_kl[o] = kl;
        p.out_cnt[o] = c;
    }
}

__global__ __launch_bounds__(kEmitWaves * 64, 1) void reduce_kernel(const PartParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t red_smem[];
    uint64_t* keys = reinterpret_cast<uint64_t*>(red_smem);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(keys + kAggSlots);
    uint32_t* n_out = cnt + kAggSlots;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    for (int i = tid; i < kAggSlots; i += kEmitWaves * 64) {
        keys[i] = 0ull;
        cnt[i] = 0u;
    }
    if (tid == 0) *n_out = 0u;
    __syncthreads();
    const int64_t beg = (int64_t)p.boff[blockIdx.x], end = (int64_t)p.boff[blockIdx.x + 1];
    const uint64_t cmask = p.cb >= 64 ? ~0ull : ((1ull << p.cb) - 1ull);
    constexpr int kU = 8;  // records per lane in flight; their probes advance together
    for (int64_t i00 = beg + (int64_t)wave * 64 * kU; i00 < end; i00 += kEmitWaves * 64 * kU) {
        uint64_t kl[kU];
        uint32_t c[kU], slot[kU];
        bool pend[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t i = i00 + 64 * u + lane;
            const uint64_t r = i < end ? p.rec2[i] : 0ull;
            pend[u] = i < end;
            kl[u] = r >> p.cb;  // never 0 for a record: the sentinel bit
            c[u] = (uint32_t)(r & cmask);
            slot[u] = (uint32_t)(((uint64_t)(uint32_t)mix64(kl[u]) * kAggSlots) >> 32);
        }
        for (int t = 0; t < 32; ++t) {
            uint64_t cur[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) cur[u] = pend[u] ? keys[slot[u]] : 0ull;  // read first: most records find their key
            bool any = false;
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                if (!pend[u]) continue;
                if (cur[u] == 0ull) {
                    const unsigned long long old =
                        atomicCAS(reinterpret_cast<unsigned long long*>(&keys[slot[u]]), 0ull, (unsigned long long)kl[u]);
                    cur[u] = old == 0ull ? kl[u] : old;
                }
                if (cur[u] == kl[u]) {
                    __hip_atomic_fetch_add(&cnt[slot[u]], c[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    pend[u] = false;
                } else {
                    slot[u] = (slot[u] + 1u) & (kAggSlots - 1u);
                    any = true;
                }
            }
            if (!__ballot(any)) break;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)  // no LDS room: the record goes out as it is
            out_append(p, n_out, beg, pend[u], kl[u], c[u], lane);
    }
    __syncthreads();
    for (int i0 = wave * 64; i0 < kAggSlots; i0 += kEmitWaves * 64) {
        const int i = i0 + lane;
        const uint64_t k = keys[i];
        out_append(p, n_out, beg, k != 0ull, k, cnt[i], lane);
    }
    __syncthreads();
    if (tid == 0) p.nout[blockIdx.x] = *n_out;
}

// entry i of the batch (buckets' outputs in bucket order, prefix epre) ->
// bucket b = the last with epre[b] <= i, stored at boff[b] + (i - epre[b])
__global__ __launch_bounds__(1024) void merge_kernel(const PartParams p, const CountParams c, int64_t n) {
    __shared__ uint64_t pre[kQ * kQ + 1];
    for (int i = threadIdx.x; i <= kQ * kQ; i += blockDim.x) pre[i] = p.epre[i];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int lo = 0;
#pragma unroll
    for (int step = 2048; step >= 1; step >>= 1)
        if (lo + step <= kQ * kQ && pre[lo + step] <= (uint64_t)i) lo += step;
    const int64_t at = (int64_t)p.boff[lo] + (i - (int64_t)pre[lo]);
    const uint64_t kl = p.out_kl[at];
    add_count(c, kl_key(kl, p.lb), (int)(kl & ((1ull << p.lb) - 1ull)), p.out_cnt[at]);
}

}  // namespace

size_t emit_lds_bytes() { return sizeof(EmitLds); }
size_t reduce_lds_bytes() { return (size_t)kAggSlots * (sizeof(uint64_t) + sizeof(uint32_t)) + 16; }

hipError_t fit2_prepare() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&emit_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)emit_lds_bytes());
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&reduce_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)reduce_lds_bytes());
    return e;
}

hipError_t launch_emit(const PartParams& p, hipStream_t stream) {
    hipLaunchKernelGGL(emit_kernel, dim3(p.grid_a), dim3(kEmitWaves * 64), emit_lds_bytes(), stream, p);
    return hipGetLastError();
}

hipError_t launch_part2(const PartParams& p, hipStream_t stream) {
    hipLaunchKernelGGL(part2_kernel, dim3(kQ * kSplits), dim3(kEmitWaves * 64), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_reduce(const PartParams& p, hipStream_t stream) {
    hipLaunchKernelGGL(reduce_kernel, dim3(kQ * kQ), dim3(kEmitWaves * 64), reduce_lds_bytes(), stream, p);
    return hipGetLastError();
}

hipError_t launch_merge(const PartParams& p, const CountParams& c, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(merge_kernel, dim3((unsigned)((n + 1023) / 1024)), dim3(1024), 0, stream, p, c, n);
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

// find-or-insert of (lo, hi); -1 only if every slot is taken
__device__ __forceinline__ int64_t wide_find_or_insert(const WideCountParams& p, uint64_t lo, uint64_t hi,
                                                       bool& new_key) {
    uint64_t s = wide_slot(lo, hi) >> p.shift;
    for (uint64_t probe = 0; probe <= p.mask; ++probe) {
        uint64_t h = __hip_atomic_load(&p.khi[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (h == kEmpty) {
            const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(&p.khi[s]), 0ull,
                                                     (unsigned long long)(hi | kWidePending));
            if (old == 0ull) {
                __hip_atomic_store(&p.klo[s], lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&p.khi[s], hi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                new_key = true;
                return (int64_t)s;
            }
            h = old;
        }
        // another lane's insert in flight: its lo is stored before hi is
        // published (a lane of this wave wrote it above, before this loop)
        while (h & kWidePending) h = __hip_atomic_load(&p.khi[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (h == hi && __hip_atomic_load(&p.klo[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == lo)
            return (int64_t)s;
        s = (s + 1) & p.mask;
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
