// ldgpu_long.hip -- FIT counting of gram lengths beyond 15 bytes (gfx950).
//
// Semantic target: computeGrams + reduceGrams (LanguageDetector.scala:25-66)
// for any n of gramLengths: every window of the Scala sliding(n) of a
// document's UTF-8 bytes (0 < len < n: the whole text, once) adds 1 to
// count(lang, window), once per occurrence of n in gramLengths.  Grams of up
// to 15 bytes take FIT v4 (ldgpu_fit.hip); this file counts the longer ones.
//
// Table: open addressing over LongSlot {hash | 1, arena offset << 24 | length};
// the gram's bytes are copied into the table's key arena by the insert that
// claims the slot (CAS on the hash word, then the bytes, then the meta word
// with release order); a reader that meets the slot's hash waits for the meta
// word, then compares length and bytes.  Counts go to a pair table keyed
// (slot + 1) << 12 | lang with one u64 counter (as the sparse T of
// ldgpu_fit.hip).
// Integer adds are order-free: the counts are bit-exact in any schedule.
// The host sizes the slots, the pair table and the arena for a launch's
// windows before it runs, so an insert always finds room.
#include "ldgpu_fit.h"

namespace ldgpu {
namespace {

constexpr uint64_t kLenMask = (1ull << kLongLenBits) - 1ull;

__device__ __forceinline__ bool bytes_equal(const uint8_t* a, const uint8_t* b, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

// find-or-insert of the gram w[0 .. len); its slot, or -1 (table full: never
// with the host's sizing).  A lane that wins a slot copies the bytes and
// publishes the meta word in the same pass of the loop; a lane that meets a
// slot being written looks at it again on its next pass (no wait nested in
// a branch: the winner may share the wave).
__device__ int64_t long_find_or_insert(const LongCountParams& p, const uint8_t* w, int64_t len, bool& new_gram) {
    const uint64_t h = gen_hash(w, len) | 1ull;
    uint64_t s = h >> p.shift;
    uint64_t probes = 0;
    for (uint32_t pass = 0; pass < (1u << 24); ++pass) {
        uint64_t cur = __hip_atomic_load(&p.slots[s].h, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        bool won = false;
        if (cur == 0ull) {
            const unsigned long long old =
                atomicCAS(reinterpret_cast<unsigned long long*>(&p.slots[s].h), 0ull, (unsigned long long)h);
            won = old == 0ull;
            cur = won ? h : old;
        }
        if (won) {
            uint64_t off = atomicAdd(p.arena_n, (unsigned long long)len);
            if (off + (uint64_t)len > p.arena_cap) {
                atomicOr(p.full, 1u);
                off = 0;
            } else {
                for (int64_t i = 0; i < len; ++i) p.arena[off + i] = w[i];
            }
            __hip_atomic_store(&p.slots[s].meta, (off << kLongLenBits) | (uint64_t)len, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
            new_gram = true;
            return (int64_t)s;
        }
        if (cur == h) {
            const uint64_t meta = __hip_atomic_load(&p.slots[s].meta, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (meta == 0ull) continue;  // being written: this slot again
            if ((int64_t)(meta & kLenMask) == len && bytes_equal(p.arena + (meta >> kLongLenBits), w, len))
                return (int64_t)s;
        }
        s = (s + 1) & p.mask;
        if (++probes > p.mask) break;
    }
    atomicOr(p.full, 1u);
    return -1;
}

// c of (gram slot g, lang) into the pair table; returns whether the pair is new
__device__ bool long_pair_add(const LongCountParams& p, int64_t g, int lang, unsigned long long c) {
    const uint64_t pk = ((uint64_t)(g + 1) << kPairLangBits) | (uint64_t)lang;
    uint64_t s = fit_hash(pk) >> p.pshift;  // (launch_pair_rehash grows this table)
    for (uint64_t probe = 0; probe <= p.pmask; ++probe) {
        const uint64_t k = __hip_atomic_load(&p.pkeys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool hit = k == pk, fresh = false;
        if (k == kEmpty) {
            const unsigned long long old =
                atomicCAS(reinterpret_cast<unsigned long long*>(&p.pkeys[s]), 0ull, (unsigned long long)pk);
            fresh = old == 0ull;
            hit = fresh || old == pk;
        }
        if (hit) {
            atomicAdd(&p.pcounts[s], c);
            return fresh;
        }
        s = (s + 1) & p.pmask;
    }
    atomicOr(p.full, 1u);
    return false;
}

__device__ __forceinline__ void wave_add(unsigned long long* ctr, unsigned int n) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd(ctr, (unsigned long long)n);
}

constexpr int kLongWaves = 4;

__global__ __launch_bounds__(kLongWaves * 64) void long_count_kernel(const LongCountParams p, const uint8_t* bytes,
                                                                     const int64_t* offsets, const int32_t* doc_lang,
                                                                     int64_t n_docs, const DeriveParams d) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    unsigned int ng = 0, np = 0;
    const int64_t stride = (int64_t)gridDim.x * kLongWaves;
    for (int64_t doc = (int64_t)blockIdx.x * kLongWaves + wave; doc < n_docs; doc += stride) {
        const int lang = doc_lang[doc];
        if (lang < 0 || lang >= p.L) continue;  // reduceGrams keeps supported languages only
        const int64_t b = offsets[doc];
        const int64_t len = offsets[doc + 1] - b;
        const uint8_t* t = bytes + b;
        unsigned long long partial = 0;
        for (int j = 0; j < d.n; ++j) {
            const int64_t n = d.len[j];
            if (len < n) {
                partial += d.mult[j];
                continue;
            }
            for (int64_t pos = lane; pos <= len - n; pos += 64) {
                bool fresh = false;
                const int64_t g = long_find_or_insert(p, t + pos, n, fresh);
                ng += fresh;
                if (g >= 0) np += long_pair_add(p, g, lang, d.mult[j]);
            }
        }
        // the Scala sliding partial window: the whole text, once per such n
        // (texts of <= 15 bytes take partial_kernel's one- and two-word keys)
        if (partial && len > kMaxWideGram && lane == 0) {
            bool fresh = false;
            const int64_t g = long_find_or_insert(p, t, len, fresh);
            ng += fresh;
            if (g >= 0) np += long_pair_add(p, g, lang, partial);
        }
    }
    wave_add(p.size, ng);
    wave_add(p.psize, np);
}

__global__ void long_add_kernel(const LongCountParams p, const uint8_t* kbytes, const int64_t* koff,
                                const int32_t* lang, const unsigned long long* cnt, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned int ng = 0, np = 0;
    if (i < n && cnt[i]) {
        bool fresh = false;
        const int64_t g = long_find_or_insert(p, kbytes + koff[i], koff[i + 1] - koff[i], fresh);
        ng = fresh;
        if (g >= 0) np = long_pair_add(p, g, lang[i], cnt[i]);
    }
    wave_add(p.size, ng);
    wave_add(p.psize, np);
}

__global__ void long_rehash_kernel(const LongCountParams from, const LongCountParams to, uint64_t from_cap,
                                   uint64_t* remap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= from_cap) return;
    const LongSlot e = from.slots[i];
    if (e.h == 0ull) return;
    uint64_t s = e.h >> to.shift;
    while (atomicCAS(reinterpret_cast<unsigned long long*>(&to.slots[s].h), 0ull, (unsigned long long)e.h) != 0ull)
        s = (s + 1) & to.mask;
    to.slots[s].meta = e.meta;
    remap[i] = s;
}

}  // namespace

hipError_t launch_long_count(const LongCountParams& p, const uint8_t* bytes, const int64_t* offsets,
                             const int32_t* doc_lang, int64_t n_docs, const DeriveParams& d, hipStream_t stream) {
    if (n_docs <= 0 || d.n == 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>(8192, (n_docs + kLongWaves - 1) / kLongWaves);
    hipLaunchKernelGGL(long_count_kernel, dim3(g), dim3(kLongWaves * 64), 0, stream, p, bytes, offsets, doc_lang,
                       n_docs, d);
    return hipGetLastError();
}

hipError_t launch_long_add(const LongCountParams& p, const uint8_t* kbytes, const int64_t* koff, const int32_t* lang,
                           const unsigned long long* cnt, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(long_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, p, kbytes, koff,
                       lang, cnt, n);
    return hipGetLastError();
}

hipError_t launch_long_rehash(const LongCountParams& from, const LongCountParams& to, uint64_t from_cap,
                              uint64_t* remap, hipStream_t stream) {
    if (from_cap == 0) return hipSuccess;
    hipLaunchKernelGGL(long_rehash_kernel, dim3((unsigned)((from_cap + 255) / 256)), dim3(256), 0, stream, from, to,
                       from_cap, remap);
    return hipGetLastError();
}

}  // namespace ldgpu
