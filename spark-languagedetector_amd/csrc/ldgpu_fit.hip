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
// Kernel structure (one wave per document, persistent grid): lanes = 64
// consecutive window positions of one gram length.  1-gram windows (the
// hottest keys: every document hits ' ', 'e', ...) are first aggregated in a
// per-wave 256-bin LDS histogram and flushed once per document, so the global
// atomics on those rows drop from one per byte to one per distinct byte per
// document; 2- and 3-byte keys likewise go through a per-wave LDS hash (kH2
// slots, flushed after each gram length; a key that finds no slot goes global).  Longer keys insert straight into the global table: find-or-CAS
// the key (relaxed agent-scope loads, device-scope CAS), then one u64 atomic
// add on the (slot, lang) counter.  An insert that exceeds kMaxProbe probes
// appends (key, lang) to an overflow list that the host re-inserts after
// growing the table.
#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "ldgpu_internal.h"

namespace ldgpu {

namespace {

__device__ __forceinline__ uint32_t ld_dw(const uint32_t* w, int64_t i, int64_t last) {
    return w[i < last ? i : last];
}

// find-or-insert; returns the slot or -1 when the probe limit is reached
__device__ __forceinline__ int64_t find_or_insert(const CountParams& p, uint64_t key) {
    uint64_t s = mix64(key) >> p.shift;
    for (int probe = 0; probe < kMaxProbe; ++probe) {
        uint64_t k = __hip_atomic_load(&p.keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return (int64_t)s;
        if (k == kEmpty) {
            const unsigned long long old =
                atomicCAS(reinterpret_cast<unsigned long long*>(&p.keys[s]), 0ull, (unsigned long long)key);
            if (old == 0ull) {
                atomicAdd(p.size, 1ull);
                return (int64_t)s;
            }
            if (old == key) return (int64_t)s;
        }
        s = (s + 1) & p.mask;
    }
    return -1;
}

// Diagnostics build only (tools/build_variant.sh ... -DLDGPU_FIT_ABLATE=n):
// bit 0 skips the counter add, bit 1 skips the whole global update, bit 2
// adds 32-bit instead of 64-bit (timing only).
#ifndef LDGPU_FIT_ABLATE
#define LDGPU_FIT_ABLATE 0
#endif

__device__ __forceinline__ void add_count(const CountParams& p, uint64_t key, int lang, unsigned long long c) {
    if (LDGPU_FIT_ABLATE & 2) return;
    const int64_t s = find_or_insert(p, key);
    if (s >= 0) {
        if (LDGPU_FIT_ABLATE & 4)  // timing probe: a 32-bit add on the counter's low word
            atomicAdd(reinterpret_cast<unsigned int*>(&p.counts[(size_t)s * p.L + lang]), (unsigned int)c);
        else if (!(LDGPU_FIT_ABLATE & 1))
            atomicAdd(&p.counts[(size_t)s * p.L + lang], c);
    } else {
        // overflow: one entry per unit count -- an LDS flush (1-gram
        // histogram, 2-/3-byte hash) passes c > 1 and repeats the entry c times
        for (unsigned long long r = 0; r < c; ++r) {
            const unsigned int at = atomicAdd(p.ovf_n, 1u);
            if (at < p.ovf_cap) {
                p.ovf_keys[at] = key;
                p.ovf_lang[at] = lang;
            }
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
                                  const int32_t* lang_of, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t s = find_or_insert(p, keys[i]);
    if (s < 0) {
        atomicAdd(p.ovf_n, 1u);  // cannot happen after a grow; reported as table full
        return;
    }
    if (lang_of) {
        atomicAdd(&p.counts[(size_t)s * p.L + lang_of[i]], 1ull);
    } else {
        for (int l = 0; l < p.L; ++l) {
            const unsigned long long c = rows[(size_t)i * p.L + l];
            if (c) atomicAdd(&p.counts[(size_t)s * p.L + l], c);
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

__global__ void compact_kernel(const CountParams p, uint64_t cap, uint64_t* out_keys,
                               unsigned long long* out_counts, unsigned long long* out_n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool occ = i < cap && p.keys[i] != kEmpty;
    const uint64_t m = __ballot(occ);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    const int leader = __builtin_ctzll(m);
    if (lane == leader) base = atomicAdd(out_n, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (!occ) return;
    const int off = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const unsigned long long o = base + off;
    out_keys[o] = p.keys[i];
    for (int l = 0; l < p.L; ++l) out_counts[o * p.L + l] = p.counts[i * p.L + l];
}

}  // namespace

hipError_t launch_count(const CountParams& p, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(count_kernel, dim3(grid), dim3(kCountWaves * 64), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_counts_add(const CountParams& p, const uint64_t* keys, const unsigned long long* rows,
                             const int32_t* lang_of, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(counts_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, p, keys, rows,
                       lang_of, n);
    return hipGetLastError();
}

hipError_t launch_rehash(const CountParams& from, const CountParams& to, uint64_t from_cap, hipStream_t stream) {
    hipLaunchKernelGGL(rehash_kernel, dim3((unsigned)((from_cap + 255) / 256)), dim3(256), 0, stream, from, to,
                       from_cap);
    return hipGetLastError();
}

hipError_t launch_compact(const CountParams& p, uint64_t cap, uint64_t* out_keys, unsigned long long* out_counts,
                          unsigned long long* out_n, hipStream_t stream) {
    hipLaunchKernelGGL(compact_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, stream, p, cap, out_keys,
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

__global__ void presence_kernel(const CountParams p, uint64_t cap, int S, uint64_t* out_keys, uint64_t* out_masks,
                                int32_t* out_k, unsigned long long* out_n, unsigned int* hist) {
    extern __shared__ unsigned int lhist[];
    const int L = p.L;
    const bool lds_hist = L <= 88;  // L * (L + 1) * 4 B <= 31 KiB
    if (lds_hist) {
        for (int i = threadIdx.x; i < L * (L + 1); i += blockDim.x) lhist[i] = 0u;
        __syncthreads();
    }
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool occ = i < cap && p.keys[i] != kEmpty;
    const uint64_t m = __ballot(occ);
    const int lane = threadIdx.x & 63;
    if (m) {
        unsigned long long base = 0;
        const int leader = __builtin_ctzll(m);
        if (lane == leader) base = atomicAdd(out_n, (unsigned long long)__popcll(m));
        base = __shfl(base, leader);
        if (occ) {
            const uint32_t off =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const unsigned long long o = base + off;
            int k = 0;
            for (int s = 0; s < S; ++s) {
                uint64_t w = 0;
                for (int b = 0; b < 64 && s * 64 + b < L; ++b)
                    if (p.counts[i * L + s * 64 + b] != 0ull) w |= 1ull << b;
                out_masks[o * S + s] = w;
                k += __popcll(w);
            }
            out_keys[o] = p.keys[i];
            out_k[o] = k;
            for (int l = 0; l < L; ++l) {
                if (p.counts[i * L + l] != 0ull) {
                    if (lds_hist)
                        atomicAdd(&lhist[l * (L + 1) + k], 1u);
                    else
                        atomicAdd(&hist[l * (L + 1) + k], 1u);
                }
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

__global__ void gather_chosen_kernel(int64_t n, int S, const uint8_t* chosen, const uint64_t* keys,
                                     const uint64_t* masks, const int32_t* ks, uint64_t* out_keys,
                                     uint64_t* out_masks, int32_t* out_k, unsigned long long* out_n) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool c = j < n && chosen[j];
    const uint64_t m = __ballot(c);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    const int leader = __builtin_ctzll(m);
    if (lane == leader) base = atomicAdd(out_n, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (!c) return;
    const unsigned long long o =
        base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    out_keys[o] = keys[j];
    out_k[o] = ks[j];
    for (int s = 0; s < S; ++s) out_masks[o * S + s] = masks[j * S + s];
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

}  // namespace

hipError_t launch_presence(const CountParams& p, uint64_t cap, int S, uint64_t* out_keys, uint64_t* out_masks,
                           int32_t* out_k, unsigned long long* out_n, unsigned int* hist, hipStream_t stream) {
    const size_t lds = p.L <= 88 ? (size_t)p.L * (p.L + 1) * 4 : 0;
    hipLaunchKernelGGL(presence_kernel, dim3(grid_of((int64_t)cap, 256)), dim3(256), lds, stream, p, cap, S, out_keys,
                       out_masks, out_k, out_n, hist);
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
// (8 bits) -- leave each language's candidates contiguous and in tie order.
// Sort keys are unique per gram, so this picks exactly the set nth_element
// picked on the host.  Synchronises `stream` before returning (scratch freed).
hipError_t launch_topk_candidates(int64_t cn, const int32_t* cand_lang, const uint64_t* cand_key,
                                  const uint32_t* cand_idx, const int64_t* seg_start, const int32_t* need,
                                  uint8_t* chosen, hipStream_t stream) {
    if (cn <= 0) return hipSuccess;
    const int n = (int)cn;
    uint64_t* key_out = nullptr;
    uint32_t *perm_a = nullptr, *perm_b = nullptr, *lang_a = nullptr, *lang_b = nullptr;
    void* tmp = nullptr;
    size_t tmp1 = 0, tmp2 = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp1, cand_key, key_out, perm_a, perm_b, n, 0, 59,
                                                      stream);
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp2, lang_a, lang_b, perm_b, perm_a, n, 0, 8, stream);
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
        e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp2, lang_a, lang_b, perm_b, perm_a, n, 0, 8, stream);
    if (e == hipSuccess) {
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
    hipLaunchKernelGGL(gather_chosen_kernel, dim3(grid_of(n, 256)), dim3(256), 0, stream, n, S, chosen, keys, masks,
                       ks, out_keys, out_masks, out_k, out_n);
    return hipGetLastError();
}

}  // namespace ldgpu
