// ldgpu_general.hip -- SCORE for tables with keys of any length (gfx950).
//
// Semantic target: LanguageDetectorModel.detect(Array[Byte], ...),
// LanguageDetectorModel.scala:131-156, for models whose gram lengths go beyond
// the packed one- and two-word keys (1..15 bytes): the reference accepts any n
// (:139-147).  For n in gramLengths (order, duplicates repeat), for every
// window of the Scala sliding(n) (0 < len < n: one window, the whole text) in
// position order, a table hit adds its row to the scores (s[l] = s[l] +
// row[l], F2J daxpy with a = 1.0); then breeze's argmax (first maximum; a NaN
// first score keeps index 0).
//
// One wave per document.  Lanes take 64 consecutive windows: each hashes its
// window (gen_hash), probes the key table (linear probes over GenSlot) and, on
// a hash and length match, compares the window with the key's bytes in the
// arena.  The hits of the 64 windows are then replayed in position order --
// the reference's order, so the fp64 sums are bit-identical: lane j adds
// row[l] for its languages l = j, j + 64, ... into the wave's score vector in
// LDS.  A mask-form row adds v at its set languages (adding 0.0 elsewhere is
// exact: a score is never -0.0).  This path favours generality over speed:
// tables with every gram length <= 15 take the LDS-filtered kernels of
// ldgpu_score.hip.  A document of up to kGenBuf bytes is first copied into the
// wave's LDS buffer: a window's hash then reads its bytes from LDS -- up to 12
// bytes as three byte-aligned words, the FNV steps unrolled in registers --
// instead of one dependent global load per byte.
//
// Mixed tables (long lengths next to lengths <= 15): the LDS-filtered kernels
// score the short lengths over the short keys, long_flag_kernel lists the
// documents a long length can hit, and this kernel rescores only those
// (indirect launch, every length, every key): a document no long window hits
// gets exactly the short lengths' adds, in the reference's order.
#include "ldgpu_internal.h"

namespace ldgpu {
namespace {

__device__ __forceinline__ bool key_equal(const uint8_t* a, const uint8_t* b, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

// the row of the key window[0 .. klen), or -1
__device__ __forceinline__ int64_t gen_lookup(const GenScoreParams& p, const uint8_t* w, int64_t klen) {
    const uint64_t h = gen_hash(w, klen);
    uint64_t s = h >> p.slot_shift;
    for (;;) {
        const GenSlot e = p.slots[s];
        if (e.len == 0) return -1;
        if (e.h == h && e.len == (uint32_t)klen) {
            const uint32_t r = e.row & ~kBadRow;
            if (key_equal(w, p.arena + p.koff[r], klen)) return (int64_t)e.row;
        }
        s = (s + 1) & p.slot_mask;
    }
}

constexpr int kGenBuf = 4096;  // staged document bytes per wave (+ 64 B of read slack)

__device__ __forceinline__ uint64_t fnv_step(uint64_t h, uint32_t byte) { return (h ^ byte) * 1099511628211ull; }

// gen_hash (ldgpu_common.h) of the klen-byte window at byte pos of the
// wave's staged document
__device__ __forceinline__ uint64_t gen_hash_staged(const uint8_t* buf, uint32_t pos, int64_t klen) {
    uint64_t h = 1469598103934665603ull ^ (uint64_t)klen;
    if (klen <= 12) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(buf) + (pos >> 2);
        const uint32_t sh = pos & 3u;
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
        const uint32_t x[3] = {__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                               __builtin_amdgcn_alignbyte(w3, w2, sh)};
#pragma unroll
        for (int i = 0; i < 12; ++i)
            if (i < klen) h = fnv_step(h, (x[i >> 2] >> (8 * (i & 3))) & 0xffu);
    } else {
        for (int64_t i = 0; i < klen; ++i) h = fnv_step(h, buf[pos + i]);
    }
    return mix64(h);
}

// gen_lookup of a window of the staged document
__device__ __forceinline__ int64_t gen_lookup_staged(const GenScoreParams& p, const uint8_t* buf, uint32_t pos,
                                                     int64_t klen) {
    const uint64_t h = gen_hash_staged(buf, pos, klen);
    uint64_t s = h >> p.slot_shift;
    for (;;) {
        const GenSlot e = p.slots[s];
        if (e.len == 0) return -1;
        if (e.h == h && e.len == (uint32_t)klen) {
            const uint32_t r = e.row & ~kBadRow;
            if (key_equal(buf + pos, p.arena + p.koff[r], klen)) return (int64_t)e.row;
        }
        s = (s + 1) & p.slot_mask;
    }
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const double u = __shfl_xor(v, o);
        v = u > v ? u : v;
    }
    return v;
}

__global__ __launch_bounds__(kGenWaves * 64) void general_score_kernel(const GenScoreParams p) {
    extern __shared__ double gen_acc[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    double* acc = gen_acc + (size_t)wave * p.L;
    uint8_t* const buf = reinterpret_cast<uint8_t*>(gen_acc + (size_t)kGenWaves * p.L) + wave * (kGenBuf + 64);
    const int S = (p.L + 63) / 64;
    const int64_t stride = (int64_t)gridDim.x * kGenWaves;
    const int64_t n_docs = p.doc_idx ? (int64_t)*p.n_docs_dev : p.n_docs;
    for (int64_t i = (int64_t)blockIdx.x * kGenWaves + wave; i < n_docs; i += stride) {
        const int64_t doc = p.doc_idx ? p.doc_idx[i] : i;
        for (int l = lane; l < p.L; l += 64) acc[l] = 0.0;
        const int64_t b = p.offsets[doc];
        const int64_t len = p.offsets[doc + 1] - b;
        const uint8_t* d = p.bytes + b;
        const bool staged = len <= kGenBuf;
        if (staged) {  // the document into the wave's buffer (LDS ops of a wave complete in order)
            __builtin_amdgcn_wave_barrier();
            for (int64_t i = lane; i < len; i += 64) buf[i] = d[i];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
        for (int gi = 0; gi < p.nG; ++gi) {
            const int64_t n = p.G[gi];
            const int64_t nw = n_windows(len, (int)(n > 0x7fffffff ? 0x7fffffff : n));
            const int64_t klen = len < n ? len : n;
            for (int64_t p0 = 0; p0 < nw; p0 += 64) {
                const int64_t pos = p0 + lane;
                const int64_t row = pos >= nw ? -1
                                    : (staged ? gen_lookup_staged(p, buf, (uint32_t)pos, klen) : gen_lookup(p, d + pos, klen));
                uint64_t hits = __ballot(row >= 0);
                while (hits) {  // in window order
                    const int j = __builtin_ctzll(hits);
                    hits &= hits - 1;
                    const uint32_t r = (uint32_t)__shfl((int)row, j);
                    if (r & kBadRow) {
                        if (lane == 0) atomicOr(p.err, 1);
                        continue;
                    }
                    if (p.masks) {
                        const double v = p.vals[r];
                        for (int s = 0; s < S; ++s) {
                            const int l = s * 64 + lane;
                            if (l < p.L && ((p.masks[(size_t)r * S + s] >> lane) & 1ull)) acc[l] = acc[l] + v;
                        }
                    } else {
                        const double* rw = p.rows + (size_t)r * p.L;
                        for (int l = lane; l < p.L; l += 64) acc[l] = acc[l] + rw[l];
                    }
                }
            }
        }
        // breeze argmax: the first index of the maximum of the non-NaN scores;
        // a NaN first score keeps index 0
        double lv = -__builtin_inf();
        for (int l = lane; l < p.L; l += 64)
            if (!__builtin_isnan(acc[l]) && acc[l] > lv) lv = acc[l];
        const double M = wave_max(lv);
        int first = 0x7fffffff;
        for (int l = lane; l < p.L; l += 64)
            if (acc[l] == M) {
                first = l;
                break;
            }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) first = min(first, __shfl_xor(first, o));
        const int label = (__builtin_isnan(acc[0]) || first == 0x7fffffff) ? 0 : first;
        if (lane == 0) p.labels[doc] = label;
        if (p.scores)
            for (int l = lane; l < p.L; l += 64) p.scores[doc * p.L + l] = acc[l];
    }
}

// Mixed tables: list the documents a long gram length can hit (LongFlagParams).
// One wave per document; lanes take 64 consecutive window positions of each
// long length n, read the window's first eight bytes (three dword loads and a
// byte align: n >= 16, so they lie inside the document) and test its two
// prefilter bits in the workgroup's LDS copy of the bitmap; a window passing
// both is looked up in the general table (hash of its n bytes, linear probes,
// byte compare).  A document shorter than some long n is also looked up whole
// (its one partial window, whatever its length).  The first hit lists the
// document (one atomic per listed document) and ends its scan.
constexpr int kFlagWaves = 4;

__global__ __launch_bounds__(kFlagWaves * 64) void long_flag_kernel(const LongFlagParams p) {
    extern __shared__ uint32_t bm[];
    for (uint32_t i = threadIdx.x; i < (1u << p.lb) / 32u; i += blockDim.x) bm[i] = p.bitmap[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    GenScoreParams g{};
    g.slots = p.slots;
    g.slot_mask = p.slot_mask;
    g.slot_shift = p.slot_shift;
    g.arena = p.arena;
    g.koff = p.koff;
    const int64_t stride = (int64_t)gridDim.x * kFlagWaves;
    for (int64_t doc = (int64_t)blockIdx.x * kFlagWaves + wave; doc < p.n_docs; doc += stride) {
        const int64_t b = p.offsets[doc];
        const int64_t len = p.offsets[doc + 1] - b;
        const uint8_t* d = p.bytes + b;
        bool hit = false;
        if (len > 0 && len < p.max_long && lane == 0) hit = gen_lookup(g, d, len) >= 0;
        uint64_t any = __ballot(hit);
        for (int gi = 0; gi < p.n_long && !any; ++gi) {
            const int64_t n = p.Glong[gi];
            const int64_t nw = len - n + 1;  // full windows (n > len: none)
            for (int64_t p0 = 0; p0 < nw && !any; p0 += 64) {
                const int64_t pos = p0 + lane;
                bool h = false;
                if (pos < nw) {
                    const uintptr_t a = (uintptr_t)(d + pos);
                    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
                    const uint32_t sh = (uint32_t)(a & 3), w0 = w[0], w1 = w[1], w2 = w[2];
                    uint32_t b1, b2;
                    long_bits(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                              (uint32_t)n, p.lb, b1, b2);
                    if (((bm[b1 >> 5] >> (b1 & 31)) & (bm[b2 >> 5] >> (b2 & 31)) & 1u) != 0u)
                        h = gen_lookup(g, d + pos, n) >= 0;
                }
                any = __ballot(h);
            }
        }
        if (any && lane == 0) p.idx[atomicAdd(p.n_out, 1ull)] = doc;
    }
}

}  // namespace

hipError_t launch_long_flag(const LongFlagParams& p, int cus, hipStream_t stream) {
    if (p.n_docs <= 0) return hipSuccess;
    const size_t lds = (size_t)(1u << p.lb) / 8u;
    hipError_t e = hipFuncSetAttribute((const void*)&long_flag_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    const int64_t want = (p.n_docs + kFlagWaves - 1) / kFlagWaves;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)cus * 8));
    hipLaunchKernelGGL(long_flag_kernel, dim3(grid), dim3(kFlagWaves * 64), lds, stream, p);
    return hipGetLastError();
}

hipError_t launch_general_score(const GenScoreParams& p, int grid, hipStream_t stream) {
    // scores (<= 64 KiB: L <= 4096) and the staged documents
    const size_t lds = sizeof(double) * kGenWaves * p.L + (size_t)kGenWaves * (kGenBuf + 64);
    hipError_t e = hipFuncSetAttribute((const void*)&general_score_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(general_score_kernel, dim3(grid), dim3(kGenWaves * 64), lds, stream, p);
    return hipGetLastError();
}

}  // namespace ldgpu
