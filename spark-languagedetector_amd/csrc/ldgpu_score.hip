// ldgpu_score.hip -- SCORE kernel for gfx950.
//
// Semantic target: LanguageDetectorModel.detect(Array[Byte], ...)
// (LanguageDetectorModel.scala:131-156):
//   s = zeros(L)
//   for n in gramLengths (order, duplicates repeat)
//     for window in sliding(n) (0 < len < n -> the whole text)      :139-144
//       if table contains window: s = s + row   (daxpy, a = 1.0)     :145-149
//   label = argmax(s), first maximum (breeze)                       :154
//
// Structure (one wave per document, persistent grid; each wave's groups of
// consecutive documents staged into its LDS by double-buffered LDS-DMA):
//   probe      a superblock = 256 window positions, 4 per lane at stride 64.
//              Each lane reads the 8 bytes at each of its positions once
//              (LDS words + v_alignbyte) and, once per superblock, the
//              prefix-Bloom word chosen by each position's first three bytes
//              (shared by every key length >= 3, ldgpu_common.h); a table
//              whose bloom exceeds LDS uses the keyed bloom in global memory
//              instead.  Each gram length n then tests one bit of a word (a
//              24-bit multiply and a bit extract), and a ballot appends the
//              candidates to a per-wave LDS queue with mbcnt, so the queue is
//              in reference order: n outer, position inner.
//   verify     64 queued keys at a time probe the global table (2-choice
//              cuckoo slots, 5-slot buckets for big count-mode tables, a
//              two-word table for keys of 8..15 bytes).
//   accumulate count mode (every row one shared value): per-language hit
//              counts in LDS (order-free; 1-/2-byte keys counted straight from
//              LDS direct tables, and the verify loads of the longer keys
//              issued before those direct counts), scores = a host-built fold
//              table.  Other mask tables: hits replayed in queue order, lane l
//              owns language l (slices of 64 for L > 64) and does s_l = s_l +
//              v or + 0.0; dense tables: s_l = s_l + row_l.  Every s_l sees
//              exactly the reference's sequence of fp64 adds: scores are
//              bit-identical, not just within tolerance.
//   argmax     DPP wave max, then the first index holding it (breeze rule).
// Documents of max(G)..256 bytes take a fast path (all windows full-length,
// one superblock); in count mode consecutive short ones share a superblock
// (packs).  Shorter documents (partial windows) and longer ones loop n outer,
// superblocks inner.
#include <type_traits>

//
// Build: this file is compiled once per (mode, slices) pair with
// -DLDGPU_SCORE_MODE=m -DLDGPU_SCORE_S=s (the Makefile's score_<m>_<s>
// objects: twenty translation units that compile in parallel), each defining
// that pair's launch / prepare entry points, and once without them for the
// dispatch (launch_score, score_prepare) and the language-block combine.
#include "ldgpu_internal.h"

namespace ldgpu {

#if defined(LDGPU_SCORE_MODE)
namespace {

constexpr int kSub = 4;  // 64-position sub-blocks per superblock

// tuning switch (build variants only): count mode issues its verify loads
// before the direct 1-/2-byte counts and completes them after (probe_count_all)
#ifndef LDGPU_SPLIT_VERIFY
#define LDGPU_SPLIT_VERIFY 1
#endif



// The launch's parameter block through an opaque pointer to the kernarg
// segment, for fields used off the hot path (long documents, score outputs,
// error flags): their loads stay at their use (s_load from the scalar cache)
// instead of being hoisted to the kernel start and held in SGPRs across the
// persistent loop (LDGPU_COLD_PARAMS; the score kernels spill ~30 SGPRs).
#ifndef LDGPU_COLD_PARAMS
#define LDGPU_COLD_PARAMS 1
#endif
typedef const __attribute__((address_space(4))) ScoreParams* ColdParams;
__device__ __forceinline__ ColdParams cold_params() {
    ColdParams q = (ColdParams)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));
    return q;
}
// f(params): with the cold pointer in the LDS-bloom kernels (KEYED == 0:
// config 2's table on either path), with p itself in the keyed-bloom ones
// (config 4's packs ran 5 % slower with it: same-box A/B)
#ifndef LDGPU_COLD_KEYED
#define LDGPU_COLD_KEYED 0
#endif
template <int KEYED, typename F>
__device__ __forceinline__ auto with_cold(const ScoreParams& p, F&& f) {
    if constexpr (LDGPU_COLD_PARAMS && (KEYED == 0 || LDGPU_COLD_KEYED)) return f(*cold_params());
    else return f(p);
}

// timing ablations exist only in the diagnostics build (LDGPU_DIAG)
__device__ __forceinline__ bool ablated(const ScoreParams& p, int bit) { return LDGPU_DIAG && (p.ablate & bit); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    return (uint64_t)rdlane((uint32_t)v, l) | ((uint64_t)rdlane((uint32_t)(v >> 32), l) << 32);
}
__device__ __forceinline__ double rdlaned(double v, int l) {
    return __longlong_as_double((long long)rdlane64((uint64_t)__double_as_longlong(v), l));
}

__device__ __forceinline__ uint32_t ld_dw(const uint32_t* w, int64_t i, int64_t last) {
    return w[i < last ? i : last];
}

struct Windows {
    uint32_t lo[kSub], hi[kSub];  // bytes [a, a+4) and [a+4, a+8) of each position
};

struct GramCtx {
    int32_t nwin;  // windows of this gram length (docs < 2^28 bytes)
    int32_t klen;  // key length: n, or len for a partial window
};

__device__ __forceinline__ GramCtx gram_ctx(int64_t len, int n) {
    GramCtx g;
    g.nwin = (int32_t)n_windows(len, n);
    g.klen = len < n ? (int)len : n;
    return g;
}

// Per-wave LDS regions.
struct WaveLds {
    uint32_t* queue;  // [kQueueCap] candidate entries (klen << 29 | position)
    uint64_t* hits;   // [64][S + 1] verified hits of one chunk: value bits, mask words
                      // (MODE 3: the document's per-language hit counters, count_area)
    uint32_t* buf;    // [2][kBufBytes / 4 + 4] staged bytes of document groups (double buffer)
    uint32_t* labels; // [64] labels of the current group
    uint32_t* cnt;    // MODE 3: per-language hit counters (count_area)
};

// MODE 3 per-language hit counters: the wave's hit area -- in the packing
// kernels after its first 64 words, which take the pack probe's non-candidate
// stores (append_pack); hit_area_words(S, 3, pack).
__device__ __forceinline__ uint32_t* count_area(const WaveLds& w) { return w.cnt; }

// counter idx += inc: u32 counters, or (PACK: packed short documents) u16
// counters two to a word -- a document of a pack has at most 256 windows per
// gram length, so no count carries into its neighbour
template <bool PACK>
__device__ __forceinline__ void count_inc(uint32_t* cnt, uint32_t idx, uint32_t inc) {
    if constexpr (PACK)
        __hip_atomic_fetch_add(&cnt[idx >> 1], inc << ((idx & 1u) << 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
        __hip_atomic_fetch_add(&cnt[idx], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Where a document's bytes are read from: the wave's LDS buffer (staged
// group: byte `base` of the buffer) or global memory (byte `base` of p.bytes).
struct DocSrc {
    const uint32_t* lds;  // nullptr = global
    int64_t base;
};

template <bool STAGED>
__device__ __forceinline__ void window_words(const ScoreParams& p, const DocSrc& src, int64_t pos, uint32_t& w0,
                                             uint32_t& w1, uint32_t& w2, uint32_t& sh) {
    const int64_t a = src.base + pos;
    sh = (uint32_t)(a & 3);
    if constexpr (STAGED) {
        const uint32_t i = (uint32_t)(a >> 2);
        w0 = src.lds[i];
        w1 = src.lds[i + 1];
        w2 = src.lds[i + 2];
    } else {
        const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
        const int64_t i = a >> 2;
        w0 = ld_dw(W, i, p.last_dword);
        w1 = ld_dw(W, i + 1, p.last_dword);
        w2 = ld_dw(W, i + 2, p.last_dword);
    }
}

// the window's bytes [pos, pos + 16) as 5 words + byte shift (wide keys)
template <bool STAGED>
__device__ __forceinline__ void window_words5(const ScoreParams& p, const DocSrc& src, int64_t pos, uint32_t (&w)[5],
                                              uint32_t& sh) {
    const int64_t a = src.base + pos;
    sh = (uint32_t)(a & 3);
    if constexpr (STAGED) {
        const uint32_t i = (uint32_t)(a >> 2);
#pragma unroll
        for (int t = 0; t < 5; ++t) w[t] = src.lds[i + t];
    } else {
        const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
        const int64_t i = a >> 2;
#pragma unroll
        for (int t = 0; t < 5; ++t) w[t] = ld_dw(W, i + t, p.last_dword);
    }
}

// Max over the wave of a non-NaN double, by DPP row shifts / broadcasts (no
// LDS traffic); the result is read from lane 63 and is wave-uniform.
__device__ __forceinline__ double dpp_max_step_impl(double v, int olo, int ohi) {
    const double o = __hiloint2double(ohi, olo);
    double r;
    asm volatile("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(v), "v"(o));
    return r;
}
#define LDGPU_DPP_MAX(v, CTRL, RM)                                                                      \
    do {                                                                                                \
        const int lo_ = __double2loint(v), hi_ = __double2hiint(v);                                   \
        const int olo_ = __builtin_amdgcn_update_dpp(0, lo_, CTRL, RM, 0xf, false);                     \
        const int ohi_ = __builtin_amdgcn_update_dpp((int)0xfff00000, hi_, CTRL, RM, 0xf, false);       \
        v = dpp_max_step_impl(v, olo_, ohi_);                                                           \
    } while (0)

__device__ __forceinline__ double wave_max_f64(double v) {
    LDGPU_DPP_MAX(v, 0x111, 0xf);  // row_shr:1
    LDGPU_DPP_MAX(v, 0x112, 0xf);  // row_shr:2
    LDGPU_DPP_MAX(v, 0x114, 0xf);  // row_shr:4
    LDGPU_DPP_MAX(v, 0x118, 0xf);  // row_shr:8
    LDGPU_DPP_MAX(v, 0x142, 0xa);  // row_bcast:15
    LDGPU_DPP_MAX(v, 0x143, 0xc);  // row_bcast:31
    return rdlaned(v, 63);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return rdlane(v, 63);
}

// One verified hit as LDS quads: {value, mask word 0}, {mask 1, mask 2}, ...
template <int S>
constexpr int kHitQuads = (S + 2) / 2;

// s_l = s_l + (bit l of the hit's mask ? value : 0.0) -- exact: x + 0.0 == x
// because no accumulator is ever -0.0.  FIN (every table value finite):
// s_l = fma(value, bit, s_l), where value * 1.0 and value * 0.0 are exact, so
// the single rounding is that of s_l + value (or of s_l + 0.0 == s_l).
template <int S, bool FIN>
__device__ __forceinline__ void hit_add(const uint4 (&e)[kHitQuads<S>], double (&acc)[S], int lane) {
    const double vv = __longlong_as_double((long long)(((uint64_t)e[0].y << 32) | e[0].x));
    const bool upper = lane >= 32;
    const uint32_t bit = (uint32_t)lane & 31u;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int w = 2 * (1 + s);  // 32-bit words w, w + 1 hold mask s
        const uint4& q = e[w >> 2];
        const uint32_t lo = (w & 3) == 0 ? q.x : q.z;
        const uint32_t hi = (w & 3) == 0 ? q.y : q.w;
        const uint32_t b = ((upper ? hi : lo) >> bit) & 1u;
        if constexpr (FIN) {
            acc[s] = __builtin_fma(vv, (double)b, acc[s]);
        } else {
            acc[s] = acc[s] + (b ? vv : 0.0);
        }
    }
}

// Verify + accumulate the queued candidates (in queue order).
// Look key up in one bucket (one 64-B line: 4 keys, then 4 payloads).
// one bucket (one 64-B line, four independent 16-B loads): whether the key
// is there (pay = its payload) and the bucket's overflow flag
__device__ __forceinline__ bool bucket_find(const Bucket* b, uint64_t key, uint32_t& pay, bool& ovf) {
    const u32x4* q = reinterpret_cast<const u32x4*>(b);
    const u32x4 a = q[0], c = q[1], d = q[2], e = q[3];
    const uint64_t k0 = ((uint64_t)a.y << 32) | a.x;
    const uint64_t k1 = ((uint64_t)a.w << 32) | a.z;
    const uint64_t k2 = ((uint64_t)c.y << 32) | c.x;
    const uint64_t k3 = ((uint64_t)c.w << 32) | c.z;
    const uint64_t k4 = ((uint64_t)d.y << 32) | d.x;
    // p[0..4] = d.z, d.w, e.x, e.y, e.z; flags = e.w
    ovf = (e.w & kBucketOverflow) != 0u;
    pay = k0 == key ? d.z : (k1 == key ? d.w : (k2 == key ? e.x : (k3 == key ? e.y : e.z)));
    return k0 == key || k1 == key || k2 == key || k3 == key || k4 == key;
}

// A wide candidate (8..15 bytes): its own 2-choice table (WideSlot); value
// and mask words from the row arrays.
template <bool STAGED, int MODE, int S>
__device__ __forceinline__ void wide_lookup(const ScoreParams& p, const DocSrc& src, int64_t pos, int klen,
                                         uint32_t& row, uint32_t& lang1, double& v, uint64_t& m0) {
    uint32_t w[5], sh;
    window_words5<STAGED>(p, src, pos, w, sh);
    const uint64_t lo = ((uint64_t)__builtin_amdgcn_alignbyte(w[2], w[1], sh) << 32) |
                        __builtin_amdgcn_alignbyte(w[1], w[0], sh);
    const uint64_t hw = ((uint64_t)__builtin_amdgcn_alignbyte(w[4], w[3], sh) << 32) |
                        __builtin_amdgcn_alignbyte(w[3], w[2], sh);
    const uint64_t hi = (klen == 8 ? 0ull : (hw & (~0ull >> (64 - 8 * (klen - 8))))) | ((uint64_t)klen << 56);
    uint32_t h1, h2;
    wide_hash(lo, hi, h1, h2);
    const u32x4* sl = reinterpret_cast<const u32x4*>(p.wslots);
    const uint64_t ia = h1 >> p.wslot_shift32, ic = h2 >> p.wslot_shift32;
    u32x4 a0 = sl[2 * ia], a1 = sl[2 * ia + 1], c0 = sl[2 * ic], c1 = sl[2 * ic + 1];
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(c0), "+v"(c1));
    const bool ha = ((((uint64_t)a0.y) << 32) | a0.x) == lo && ((((uint64_t)a0.w) << 32) | a0.z) == hi;
    const bool hc = ((((uint64_t)c0.y) << 32) | c0.x) == lo && ((((uint64_t)c0.w) << 32) | c0.z) == hi;
    if (ha || hc) {
        const u32x4 s1 = ha ? a1 : c1;  // WideSlot: row, lang1
        row = s1.x;
        lang1 = s1.y;
        if (MODE != 2 && MODE != 3 && !(row & kBadRow)) {
            v = p.vals[row];
            m0 = p.masks[(size_t)row * S];
        }
    }
}

// Count mode, split verify of the queue's first 64 candidates (one-word keys,
// cuckoo slots): verify_issue builds the keys and issues both slots' loads;
// the caller does independent LDS work (the direct 1-/2-byte counts) while
// they are in flight, and verify_complete compares and counts.  Counts are
// order-free, so the result is flush's.
struct VerifyIssue {
    u32x4 a0, c0;   // first halves of the key's two cuckoo slots (Slot: key, row, language)
    uint64_t key;
    uint32_t inc;   // the key length's multiplicity in gramLengths
    bool valid;
};

template <bool STAGED>
__device__ __forceinline__ void verify_issue(const ScoreParams& p, const WaveLds& w, int qn, const DocSrc& src,
                                             int lane, VerifyIssue& v) {
    __builtin_amdgcn_wave_barrier();
    v.valid = lane < qn;
    v.key = 0;
    v.inc = 0;
    v.a0 = v.c0 = u32x4{0u, 0u, 0u, 0u};
    if (v.valid) {
        const uint32_t e = w.queue[lane];
        const int klen = (int)(e >> kPosBits);
        v.inc = p.mult[klen];
        uint32_t w0, w1, w2, sh;
        window_words<STAGED>(p, src, (int64_t)(e & ((1u << kPosBits) - 1u)), w0, w1, w2, sh);
        const uint64_t win = ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) |
                             __builtin_amdgcn_alignbyte(w1, w0, sh);
        v.key = (win & (~0ull >> (64 - 8 * klen))) | ((uint64_t)klen << 56);
        const u32x4* sl = reinterpret_cast<const u32x4*>(p.slots);
        uint32_t h1, h2;
        slot_hash((uint32_t)v.key, (uint32_t)(v.key >> 32), h1, h2);
        v.a0 = sl[2 * (uint64_t)(h1 >> p.slot_shift32)];
        v.c0 = sl[2 * (uint64_t)(h2 >> p.slot_shift32)];
    }
}

template <int S, int MODE = 3>
__device__ __forceinline__ void verify_complete(const ScoreParams& p, const WaveLds& w, const VerifyIssue& v) {
    uint32_t row = 0xffffffffu, lang1 = 0xffffffffu;
    if (v.valid) {
        const bool ha = ((((uint64_t)v.a0.y) << 32) | v.a0.x) == v.key;
        const bool hc = ((((uint64_t)v.c0.y) << 32) | v.c0.x) == v.key;
        if (ha || hc) {
            row = ha ? v.a0.z : v.c0.z;
            lang1 = ha ? v.a0.w : v.c0.w;
        }
    }
    const bool hit = row != 0xffffffffu;
    const bool bad = hit && (row & kBadRow);
    if (__ballot(bad)) {
        if ((threadIdx.x & 63) == 0) atomicOr(p.err, 1);
    }
    const bool good = hit && !bad;
#ifdef LDGPU_STATS
    if (p.stats) {
        const int ng = __popcll(__ballot(good));
        const int nv = __popcll(__ballot(v.valid));
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&p.stats[0], (unsigned long long)nv);
            atomicAdd(&p.stats[1], (unsigned long long)ng);
        }
    }
#endif
    uint32_t* cnt = count_area(w);
    if (good && lang1 != 0xffffffffu) {
        count_inc<false>(cnt, lang1, v.inc);
    } else if (good) {
        if constexpr (MODE == 4) {  // class mode: the row's class from its value
            const double x = p.vals[row];
            cnt += (x == p.cls[1] ? 1u : (x == p.cls[2] ? 2u : (x == p.cls[3] ? 3u : 0u))) * 64u * S;
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            uint64_t mm = p.masks[(size_t)row * S + s];
            while (mm) {
                const int l = __builtin_ctzll(mm);
                mm &= mm - 1;
                count_inc<false>(cnt, 64 * s + l, v.inc);
            }
        }
    }
}

// weighted (MODE 3 fast path, distinct gram lengths): a hit of a k-byte key
// counts p.mult[k] times (k's multiplicity in gramLengths).
// PACK (MODE 3, packed short documents, score_pack): an entry's position is
// its low 8 bits and bits 8..9 name the document of the pack, whose (u16)
// counter block it counts into.
template <int S, int MODE, bool STAGED, int KEYED, bool PACK = false, bool WIDE = false>
__device__ __forceinline__ void flush(const ScoreParams& p, const WaveLds& w, int qn, const DocSrc& src,
                                      double (&acc)[S], int lane, bool weighted = false, int q_begin = 0) {
    __builtin_amdgcn_wave_barrier();
    for (int q0 = q_begin; q0 < qn; q0 += 64) {
        const int j = q0 + lane;
        uint32_t row = 0xffffffffu;
        double v = 0.0;
        uint64_t m0 = 0;
        uint32_t lang1 = 0xffffffffu;  // count mode: the row's one language (Slot::pad)
        uint32_t inc = 1;
        uint32_t coff = 0;  // PACK: the document's counter block
        if (j < qn) {
            const uint32_t e = w.queue[j];
            const int klen = (int)(e >> kPosBits);
            if ((MODE == 3 || MODE == 4) && weighted) inc = p.mult[klen];
            if (PACK) coff = ((e >> 8) & (kPackDocs - 1u)) * 64u * S;
            const int64_t pos = (int64_t)(e & (PACK ? 255u : (1u << kPosBits) - 1u));
            if (WIDE && klen > kMaxGram) {  // (WIDE kernels: tables holding wide keys)
                wide_lookup<STAGED, MODE, S>(p, src, pos, klen, row, lang1, v, m0);
            } else {
            uint32_t w0, w1, w2, sh;
            window_words<STAGED>(p, src, pos, w0, w1, w2, sh);
            const uint64_t win = ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) |
                                 __builtin_amdgcn_alignbyte(w1, w0, sh);
            const uint64_t key = (win & (~0ull >> (64 - 8 * klen))) | ((uint64_t)klen << 56);
            if (MODE == 3 && KEYED && p.buckets) {  // (buckets only for tables beyond the caches)
                const uint64_t h = mix64(key);
                // 5-slot buckets, one 64-B line each: the key is in its primary
                // bucket, or -- only if that bucket's overflow flag is set -- in
                // its secondary one (Bucket, ldgpu_common.h; slot_mask = buckets)
                uint32_t pay = 0;
                bool ovf = false;
                bool found = bucket_find(p.buckets + bucket_index((uint32_t)(h >> 32), p.slot_mask), key, pay, ovf);
                if (!found && ovf)
                    found = bucket_find(p.buckets + bucket_index((uint32_t)h, p.slot_mask), key, pay, ovf);
                if (found) {
                    const bool one = (pay & kPayLang) != 0u;
                    row = one ? (pay & kBadRow) : pay;
                    lang1 = one ? (pay & 0xffffu) : 0xffffffffu;
                }
            } else if constexpr (MODE == 3) {
                // count mode reads only the slots' first halves (key, row,
                // the row's one language): a multi-language row's mask words
                // come from p.masks, and the value is the table's one value
                const u32x4* sl = reinterpret_cast<const u32x4*>(p.slots);
                uint32_t h1, h2;
                slot_hash((uint32_t)key, (uint32_t)(key >> 32), h1, h2);
                const uint64_t ia = h1 >> p.slot_shift32, ic = h2 >> p.slot_shift32;
                u32x4 a0 = sl[2 * ia], c0 = sl[2 * ic];
                asm volatile("" : "+v"(a0), "+v"(c0));
                const bool ha = ((((uint64_t)a0.y) << 32) | a0.x) == key;
                const bool hc = ((((uint64_t)c0.y) << 32) | c0.x) == key;
                if (ha || hc) {
                    row = ha ? a0.z : c0.z;
                    lang1 = ha ? a0.w : c0.w;
                }
            } else {
                // 2-choice cuckoo table: the key is in one of two slots (or
                // absent).  Both slots' four 16-B loads are issued before any
                // compare (the register pin keeps the compiler from sinking
                // the second slot's loads behind the first one's key test), so
                // a candidate costs one L2 round trip, not three.
                const u32x4* sl = reinterpret_cast<const u32x4*>(p.slots);
                uint32_t h1, h2;
                slot_hash((uint32_t)key, (uint32_t)(key >> 32), h1, h2);
                const uint64_t ia = h1 >> p.slot_shift32, ic = h2 >> p.slot_shift32;
                u32x4 a0 = sl[2 * ia], a1 = sl[2 * ia + 1], c0 = sl[2 * ic], c1 = sl[2 * ic + 1];
                asm volatile("" : "+v"(a0), "+v"(a1), "+v"(c0), "+v"(c1));
                const bool ha = ((((uint64_t)a0.y) << 32) | a0.x) == key;
                const bool hc = ((((uint64_t)c0.y) << 32) | c0.x) == key;
                const u32x4 s0 = ha ? a0 : c0, s1 = ha ? a1 : c1;
                if (ha || hc) {  // Slot: key, row, pad | val, mask0
                    row = s0.z;
                    lang1 = s0.w;
                    v = __longlong_as_double((long long)((((uint64_t)s1.y) << 32) | s1.x));
                    m0 = (((uint64_t)s1.w) << 32) | s1.z;
                }
            }
            }  // narrow key
        }
        const bool hit = row != 0xffffffffu;
        const bool bad = hit && (row & kBadRow);
        if (__ballot(bad)) {
            if (lane == 0) with_cold<KEYED>(p, [](const auto& q) { atomicOr(q.err, 1); });
        }
        const bool good = hit && !bad;
#ifdef LDGPU_STATS
        if (p.stats) {  // diagnostics build: candidates verified, hits
            const int ng = __popcll(__ballot(good));
            if (lane == 0) {
                atomicAdd(&p.stats[0], (unsigned long long)min(64, qn - q0));
                atomicAdd(&p.stats[1], (unsigned long long)ng);
            }
        }
#endif
        if constexpr (MODE == 4) {
            // class mode: order-free per-(class, language) hit counts.  A
            // one-language row's slot holds its counter directly (class q,
            // language l: q 64 S + l, the host's encoding of class-mode
            // tables); another row's class is the index of its value among
            // p.cls (exact: the host took p.cls from the rows' values; unused
            // entries are NaN)
            if (good) {
                if (lang1 != 0xffffffffu) {
                    count_inc<false>(count_area(w), lang1, inc);
                } else {
                    const uint32_t q = v == p.cls[1] ? 1u : (v == p.cls[2] ? 2u : (v == p.cls[3] ? 3u : 0u));
                    uint32_t* cnt = count_area(w) + q * 64u * S;
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        uint64_t mm = s == 0 ? m0 : p.masks[(size_t)row * S + s];
                        while (mm) {
                            const int l = __builtin_ctzll(mm);
                            mm &= mm - 1;
                            count_inc<false>(cnt, 64 * s + l, inc);
                        }
                    }
                }
            }
            continue;
        }
        if constexpr (MODE == 3) {
            // uniform-value table: order-free per-language hit counts (the
            // score is the fold of that many adds of the one value, applied
            // at the end of the document: count_scores)
            if (good && lang1 != 0xffffffffu) {
                // single-language row: no mask words to read (no extra lines)
                count_inc<PACK>(count_area(w), coff + lang1, inc);
            } else if (good) {
                uint32_t* cnt = count_area(w);
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    // (a multi-language row: its mask words from the row arrays)
                    uint64_t mm = with_cold<KEYED>(p, [&](const auto& q) { return q.masks[(size_t)row * S + s]; });
                    while (mm) {
                        const int l = __builtin_ctzll(mm);
                        mm &= mm - 1;
                        count_inc<PACK>(cnt, coff + 64 * s + l, inc);
                    }
                }
            }
            continue;
        }
        const uint64_t hits = __ballot(good);
        if (!hits) continue;
        constexpr bool DENSE = MODE == 2;
        constexpr bool FIN = MODE == 1;
        if constexpr (!DENSE) {
            // compact the hits into LDS in queue order (entry: value, mask
            // words; 16-B aligned), then every lane (one language each)
            // replays them with broadcast ds_read_b128
            constexpr int kQ = kHitQuads<S>;  // uint4 per entry
            uint4* hq = reinterpret_cast<uint4*>(w.hits);
            if (good) {
                const uint32_t off =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(hits >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hits, 0u));
                uint64_t words[2 * kQ];
                words[0] = (uint64_t)__double_as_longlong(v);
                words[1] = m0;
#pragma unroll
                for (int s = 1; s < S; ++s) words[1 + s] = p.masks[(size_t)row * S + s];
#pragma unroll
                for (int s = S + 1; s < 2 * kQ; ++s) words[s] = 0;
#pragma unroll
                for (int q = 0; q < kQ; ++q)
                    hq[off * kQ + q] = make_uint4((uint32_t)words[2 * q], (uint32_t)(words[2 * q] >> 32),
                                                  (uint32_t)words[2 * q + 1], (uint32_t)(words[2 * q + 1] >> 32));
            }
            __builtin_amdgcn_wave_barrier();
            const int nh = ablated(p, 4) ? 0 : __popcll(hits);
            int t = 0;
            // 4 broadcast reads in flight, then 4 ordered adds
            for (; t + 4 <= nh; t += 4) {
                uint4 e[4][kQ];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int q = 0; q < kQ; ++q) e[u][q] = hq[(t + u) * kQ + q];
#pragma unroll
                for (int u = 0; u < 4; ++u) hit_add<S, FIN>(e[u], acc, lane);
            }
            for (; t < nh; ++t) {
                uint4 e[kQ];
#pragma unroll
                for (int q = 0; q < kQ; ++q) e[q] = hq[t * kQ + q];
                hit_add<S, FIN>(e, acc, lane);
            }
            __builtin_amdgcn_wave_barrier();
        } else {
            uint64_t hh = hits;
            while (hh) {
                const int h = __builtin_ctzll(hh);
                hh &= hh - 1;
                const uint32_t r = rdlane(row, h);
                const double* rp = p.rows + (size_t)r * p.L;
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const int l = s * 64 + lane;
                    if (l < p.L) acc[s] = acc[s] + rp[l];
                }
            }
        }
    }
}

// MODE 3: turn the document's per-language hit counts into scores and clear
// the counters for the next document.  Every add the reference makes to s_l
// is s_l + v (a member hit) or s_l + 0.0 (exact: s_l is never -0.0), so s_l is
// the left fold of c_l adds of v: fold[c] (host-computed, bit-identical),
// continued on the device past the table's end.
template <int S>
__device__ __forceinline__ void count_scores(const ScoreParams& p, const WaveLds& w, double (&acc)[S], int lane) {
    uint32_t* cnt = count_area(w);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int l = 64 * s + lane;
        if (l < p.L) {
            const uint32_t c = cnt[l];
            cnt[l] = 0;
            double v = 0.0;
            if (c) {
                v = p.fold[c < p.fold_max ? c : p.fold_max];
                for (uint32_t i = p.fold_max; i < c; ++i) v = v + p.fold[1];
            }
            acc[s] = v;
        }
    }
}

// MODE 3 label without scores: fold[c] is strictly monotone in c (host-checked:
// sign of the value p.count_sign, no overflow while c < 2^24), so the first
// maximum of the scores is the first maximum of c (value > 0), of -c
// (value < 0) or index 0 (value 0).  One integer DPP max over
// (key << 8 | 255 - l); clears the counters.
template <int S, typename C = uint32_t>
__device__ __forceinline__ int count_argmax(const ScoreParams& p, C* cnt, int lane) {
    uint32_t best = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int l = 64 * s + lane;
        if (l < p.L) {
            const uint32_t c = cnt[l];
            cnt[l] = 0;
            const uint32_t k = p.count_sign > 0 ? c : (p.count_sign < 0 ? 0xffffffu - c : 0u);
            best = max(best, (k << 8) | (uint32_t)(255 - l));
        }
    }
    return 255 - (int)(wave_max_u32(best) & 255u);
}

// MODE 4 label (labels only, at most 4 distinct row values v_q): per
// language l (lane l of slice s) the hit counts c_ql of each class give
// a_l = sum_q c_ql v_q and T_l = sum_q c_ql |v_q|; the reference's score f_l
// is the ordered left fold of those n_l = sum_q c_ql adds
// (LanguageDetectorModel.scala:139-154; adds of 0.0 are exact), and
// |f_l - a_l| <= (gamma(n_l - 1) + gamma(4)) T_l, gamma(k) = k u / (1 - k u),
// u = 2^-53; e_l = (n_l + 6) 2^-52 T_l bounds it with a margin that also
// covers the roundings of a_l, T_l, e_l and of the comparisons below.  The
// first maximum j of a is the reference's label when a_j - e_j > a_l + e_l for
// every other l (then f_j > f_l: no tie, breeze's argmax is j); otherwise the
// document is ambiguous: label -1, replayed exactly afterwards.  One class:
// f_l = fold(n_l) is the same fold for every l, so n_l == n_j is an exact tie
// and l > j loses it (j is the first maximum).  No hit at all: every f_l = 0.0,
// label 0.  Clears the counters.
template <int S>
__device__ __forceinline__ int class_label(const ScoreParams& p, uint32_t* cnt, int lane) {
    double a[S], e[S];
    uint32_t nn[S];
    uint32_t any = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int l = 64 * s + lane;
        a[s] = -__builtin_inf();
        e[s] = 0.0;
        nn[s] = 0;
        if (l < p.L) {
            double acc = 0.0, t = 0.0;
            uint32_t n = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q < p.n_cls) {
                    const uint32_t c = cnt[q * 64 * S + 64 * s + lane];
                    cnt[q * 64 * S + 64 * s + lane] = 0;
                    acc = acc + (double)c * p.cls[q];
                    t = t + (double)c * __builtin_fabs(p.cls[q]);
                    n += c;
                }
            }
            a[s] = acc;
            e[s] = (double)(n + 6u) * 0x1p-52 * t;
            nn[s] = n;
            any |= n;
        }
    }
    if (!__ballot(any != 0u)) return 0;
    double lv = -__builtin_inf();
#pragma unroll
    for (int s = 0; s < S; ++s) lv = a[s] > lv ? a[s] : lv;
    const double M = wave_max_f64(lv);
    int j = -1;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const uint64_t b = __ballot(64 * s + lane < p.L && a[s] == M);
        if (j < 0 && b) j = 64 * s + __builtin_ctzll(b);
    }
    double ej = 0.0;
    uint32_t nj = 0;
#pragma unroll
    for (int s = 0; s < S; ++s)
        if (j >> 6 == s) {
            ej = rdlaned(e[s], j & 63);
            nj = rdlane(nn[s], j & 63);
        }
    const double lo = M - ej;
    const bool one = p.n_cls == 1;
    bool clash = !__builtin_isfinite(lo);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int l = 64 * s + lane;
        if (l < p.L && l != j && !(a[s] + e[s] < lo) && !(one && nn[s] == nj)) clash = true;
    }
    return __ballot(clash) ? -1 : j;
}

// The prefix-Bloom words the positions of one superblock need (chosen by
// each position's first three bytes and shared by every key length >= 3,
// ldgpu_common.h): loaded once per superblock, they serve every gram length
// >= 3 of the document.  The 1-/2-byte bitmap words are read per test (one
// gram length each; caching them would cost 8 VGPRs of occupancy).
// Keyed tables (bloom too large for LDS, read from L2/MALL): one word per
// (position, length) chosen by the whole key instead (kb_hash,
// ldgpu_common.h) -- a big table's keys share few 3-byte prefixes, which
// would saturate prefix words; gb / gshift locate that bloom.
struct FWords {
    uint32_t w3[kSub];  // prefix bloom: the position's word; keyed line layout: its line << 4 (kb_line16)
    u32x4 ck[kSub];     // keyed chunk layout (KEYED == 2): the position's 16-B chunk
    const uint32_t* gb;
    uint32_t gshift;
    bool lines;         // keyed bloom in the line layout (ScoreParams::kb_lines)
};

// Bloom layout of a kernel instantiation (KEYED): 0 = prefix Bloom in LDS,
// 1 = keyed bloom in global memory (a word per key, or the line layout),
// 2 = keyed chunk layout (count mode: a 16-B chunk per window position, every
// length's bits in it, kb_chunk16).  kind_of: the filter_word KIND of keys
// of >= 3 bytes.
constexpr int kind_of(int keyed) { return keyed == 2 ? 5 : (keyed ? 4 : 3); }

template <int KEYED>
__device__ __forceinline__ void load_fwords(const ScoreParams& p, const uint32_t* bloom, const Windows& x,
                                            FWords& f) {
    if constexpr (KEYED == 2) {
        // one 16-B load per position: its chunk holds the bits of every key
        // length starting there
        const u32x4* c4 = reinterpret_cast<const u32x4*>(bloom);
#pragma unroll
        for (int k = 0; k < kSub; ++k) f.ck[k] = c4[kb_chunk(x.lo[k]) >> p.bloom_shift];
    } else if constexpr (KEYED) {
        f.gb = bloom;
        f.gshift = p.bloom_shift;
        f.lines = p.kb_lines != 0;
        if (f.lines) {  // (a scalar branch: the line hashes only for the line layout)
#pragma unroll
            for (int k = 0; k < kSub; ++k) f.w3[k] = kb_line16(x.lo[k], p.bloom_shift);
        } else {
#pragma unroll
            for (int k = 0; k < kSub; ++k) f.w3[k] = 0u;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kSub; ++k) f.w3[k] = bloom[pf_word(x.lo[k], p.bloom_shift)];
    }
}

// Filter-test the (up to) 256 windows of one superblock for one key length:
// m[k] = candidate mask of sub-block k < NSB (bit i = position p0 + 64k + i;
// NSB = sub-blocks holding a window).  Three bodies serve all lengths:
//   KIND 1 / 2 (1-/2-byte keys): bit (lo & 0xff) / (lo & 0xffff) of the exact
//   bitmaps;
//   KIND 3 (3..7 bytes): bit pf_bit_c(lo, hi, sh, mul) of the position's
//   prefix-Bloom word, already in a register (f);
//   KIND 4 (3..7 bytes, keyed bloom): the key's own word, loaded here.
// nw = windows left from the superblock's first position, in
// (64 (NSB - 1), 64 NSB] when NSB < 4: the last sub-block's ballot is cut to
// its first nw - 64 (NSB - 1) lanes by a scalar mask.
__device__ __forceinline__ uint64_t lanes_below(int32_t n) {  // n in [1, 64]
    return n >= 64 ? ~0ull : ((1ull << n) - 1ull);
}

// the filter word and bit positions of sub-block k's window: a candidate has
// bits bit and bit2 of w set (bit2 = bit except for a two-bit prefix Bloom)
template <int KIND>
__device__ __forceinline__ void filter_word(const uint32_t* img, uint32_t sh, uint32_t mul, const FWords& f,
                                            const Windows& x, int k, uint32_t& w, uint32_t& bit, uint32_t& bit2) {
    if constexpr (KIND == 1) {
        w = img[(x.lo[k] >> 5) & 7u];
        bit = bit2 = x.lo[k];
    } else if constexpr (KIND == 2) {
        w = img[kBmp1Words + bmp2_word(x.lo[k])];
        bit = bit2 = x.lo[k];
    } else if constexpr (KIND == 3) {
        w = f.w3[k];
        const uint32_t in = __builtin_amdgcn_alignbit(x.hi[k], x.lo[k], sh);
        bit = mulhi24(in, mul);
        bit2 = LDGPU_BLOOM_BITS == 2 ? mulhi24(in, pf_mult2_of(mul)) : bit;
    } else if constexpr (KIND == 5) {  // keyed chunk layout: sh = key length
        const uint32_t lo = sh >= 4 ? x.lo[k] : x.lo[k] & ((1u << (8 * sh)) - 1u);
        const uint32_t hi = sh <= 4 ? 0u : x.hi[k] & ((1u << (8 * (sh < 7 ? sh - 4 : 3))) - 1u);
        const uint32_t h = kb_hash(lo, hi, sh);
        const uint32_t q1 = h >> 25, q2 = (h >> 18) & 127u;
        const u32x4 c = f.ck[k];
        const uint32_t w1 = q1 < 64 ? (q1 < 32 ? c.x : c.y) : (q1 < 96 ? c.z : c.w);
        const uint32_t w2 = q2 < 64 ? (q2 < 32 ? c.x : c.y) : (q2 < 96 ? c.z : c.w);
        w = (w1 >> (q1 & 31u)) & (w2 >> (q2 & 31u));  // bit 0: both bits set
        bit = bit2 = 0;
    } else {  // KIND 4, keyed bloom: sh = key length, mul = unused
        const uint32_t lo = sh >= 4 ? x.lo[k] : x.lo[k] & ((1u << (8 * sh)) - 1u);
        // (a wide key hashes its first seven bytes)
        const uint32_t hi = sh <= 4 ? 0u : x.hi[k] & ((1u << (8 * (sh < 7 ? sh - 4 : 3))) - 1u);
        const uint32_t h = kb_hash(lo, hi, sh);
        // (f.w3 is 0 outside the line layout)
        w = f.gb[(sh >= 4 ? f.w3[k] : 0u) + (h >> kb_sword(sh, f.lines, f.gshift))];
        bit = bit2 = h >> kb_sbit(sh, f.lines, f.gshift);
    }
}

__device__ __forceinline__ bool filter_hit(uint32_t w, uint32_t bit, uint32_t bit2) {
    return (__builtin_amdgcn_ubfe(w, bit, 1) & __builtin_amdgcn_ubfe(w, bit2, 1)) != 0u;
}

template <int KIND, int NSB>
__device__ __forceinline__ void test_len(const uint32_t* img, uint32_t sh, uint32_t mul, const FWords& f,
                                         const Windows& x, int32_t nw, uint64_t (&m)[kSub]) {
    uint32_t w[NSB], bit[NSB], bit2[NSB];
#pragma unroll
    for (int k = 0; k < NSB; ++k) filter_word<KIND>(img, sh, mul, f, x, k, w[k], bit[k], bit2[k]);
#pragma unroll
    for (int k = 0; k < NSB; ++k) m[k] = __builtin_amdgcn_ballot_w64(filter_hit(w[k], bit[k], bit2[k]));
    m[NSB - 1] &= lanes_below(nw - 64 * (NSB - 1));
#pragma unroll
    for (int k = NSB; k < kSub; ++k) m[k] = 0;
}

template <int KIND>
__device__ __forceinline__ void test_nsb(const uint32_t* img, uint32_t sh, uint32_t mul, const FWords& f,
                                         const Windows& x, int32_t nw, uint64_t (&m)[kSub]) {
    if (nw > 192)
        test_len<KIND, 4>(img, sh, mul, f, x, nw, m);
    else if (nw > 128)
        test_len<KIND, 3>(img, sh, mul, f, x, nw, m);
    else if (nw > 64)
        test_len<KIND, 2>(img, sh, mul, f, x, nw, m);
    else
        test_len<KIND, 1>(img, sh, mul, f, x, nw, m);
}

// FULL: every length has more than 192 windows (NSB = 4, no dispatch)
template <bool FULL, int KEYED>
__device__ __forceinline__ void test_sb(const uint32_t* img, int klen, const FWords& f, const Windows& x, int32_t nw,
                                        uint64_t (&m)[kSub]) {
    const uint32_t sh = KEYED ? (uint32_t)klen : pf_shift(klen), mul = pf_mult(klen);
    constexpr int K3 = kind_of(KEYED);
    if (klen == 1) {
        if (FULL) test_len<1, 4>(img, sh, mul, f, x, nw, m); else test_nsb<1>(img, sh, mul, f, x, nw, m);
    } else if (klen == 2) {
        if (FULL) test_len<2, 4>(img, sh, mul, f, x, nw, m); else test_nsb<2>(img, sh, mul, f, x, nw, m);
    } else {
        if (FULL) test_len<K3, 4>(img, sh, mul, f, x, nw, m); else test_nsb<K3>(img, sh, mul, f, x, nw, m);
    }
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;

// Append the candidates of one superblock to the queue in position order;
// the caller guarantees room for every set bit.  Only the candidate lanes
// store (exec = the ballot itself, one s_and_saveexec: no per-lane select),
// each to the queue's next free word + its rank among them.
__device__ __forceinline__ void append_sb(uint32_t* queue, int& qn, const uint64_t (&m)[kSub], int klen, int32_t p0,
                                          int lane) {
    // opaque lane: the tags are then built here, not hoisted out of the
    // document loop as loop invariants (which the allocator spills)
    uint32_t l = (uint32_t)lane;
    asm volatile("" : "+v"(l));
    const uint32_t tag0 = ((uint32_t)klen << kPosBits) | ((uint32_t)p0 + l);
    const uint32_t qbase = (uint32_t)(uintptr_t)queue;  // LDS offset (low half of the flat address)
#pragma unroll
    for (int k = 0; k < kSub; ++k) {
        if (m[k]) {
            // rank among the candidates + the queue's fill, in entries
            const uint32_t at = __builtin_amdgcn_mbcnt_hi((uint32_t)(m[k] >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m[k], (uint32_t)qn));
            if (__builtin_amdgcn_inverse_ballot_w64(m[k])) *(lds_u32*)(size_t)(qbase + 4u * at) = tag0 + 64u * k;
            qn += __popcll(m[k]);
        }
    }
}

__device__ __forceinline__ int count_sb(const uint64_t (&m)[kSub]) {
    int t = 0;
#pragma unroll
    for (int k = 0; k < kSub; ++k) t += __popcll(m[k]);
    return t;
}

template <bool STAGED>
__device__ __forceinline__ void load_windows(const ScoreParams& p, const DocSrc& src, int32_t p0, int lane,
                                             Windows& x) {
    if constexpr (STAGED) {
        // the four positions of a lane are 64 B apart: one byte shift, and
        // their dwords at immediate offsets from one address
        const uint32_t a = (uint32_t)(src.base + p0) + (uint32_t)lane;
        const uint32_t sh = a & 3u;
        const uint32_t* w = src.lds + (a >> 2);
#pragma unroll
        for (int k = 0; k < kSub; ++k) {
            const uint32_t w0 = w[16 * k], w1 = w[16 * k + 1], w2 = w[16 * k + 2];
            x.lo[k] = __builtin_amdgcn_alignbyte(w1, w0, sh);
            x.hi[k] = __builtin_amdgcn_alignbyte(w2, w1, sh);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kSub; ++k) {
        uint32_t w0, w1, w2, sh;
        window_words<STAGED>(p, src, p0 + 64 * k + lane, w0, w1, w2, sh);
        x.lo[k] = __builtin_amdgcn_alignbyte(w1, w0, sh);
        x.hi[k] = __builtin_amdgcn_alignbyte(w2, w1, sh);
    }
}

// Count-mode direct tables (ScoreParams::direct_*): a 1-/2-byte window that is
// a key (exact bitmaps: never a false positive) names its one language in
// LDS, and its count is added there -- no queue, no verification.  Windows of
// the last sub-block past nw are masked per lane.
// PACK: position k of the lane is valid while N <= rem[k] (bytes to the end of
// its document) and counts into its document's block (tb[k] >> 8).
struct PackPos {
    int32_t rem[kSub];  // bytes from the position to the end of its document (<= 0: none)
    uint32_t tb[kSub];  // document index << 8 | position in the pack
};

// append_sb for packs: an entry is klen << kPosBits | the pack tag (tb).
// Every lane stores (measured faster here than an exec-masked store): a
// candidate to its queue rank, the others to their own word at dummy_a.
__device__ __forceinline__ void append_pack(uint32_t* queue, int& qn, const uint64_t (&m)[kSub], uint32_t klen,
                                            const PackPos& pk, uint32_t dummy_a) {
    const uint32_t qbase = (uint32_t)(uintptr_t)queue;
#pragma unroll
    for (int k = 0; k < kSub; ++k) {
        if (m[k]) {
            const uint32_t at = __builtin_amdgcn_mbcnt_hi((uint32_t)(m[k] >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m[k], (uint32_t)qn));
            uint32_t a;  // bit `lane` of m[k] ? queue word : dummy word (one v_cndmask on the mask)
            asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(a) : "v"(dummy_a), "v"(qbase + 4u * at), "s"(m[k]));
            *(lds_u32*)(size_t)a = (klen << kPosBits) | pk.tb[k];
            qn += __popcll(m[k]);
        }
    }
}

template <int N, bool FULL, int S = 1, bool PACK = false, int NK = kSub>
__device__ __forceinline__ void direct_count(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                             const Windows& x, int32_t nw, int lane, const PackPos* pk = nullptr) {
    const uint8_t* l1 = reinterpret_cast<const uint8_t*>(img + p.direct_off);
    const uint16_t* b2 = reinterpret_cast<const uint16_t*>(img + p.direct_off + 64);
    const uint8_t* l2 = reinterpret_cast<const uint8_t*>(img + p.direct_off + 64 + 1024);
    uint32_t* cnt = count_area(wl);
    const uint32_t inc = p.mult[N];
    uint32_t lang[kSub];
    bool hit[kSub];
    if constexpr (N == 1) {
#pragma unroll
        for (int k = 0; k < NK; ++k) lang[k] = l1[x.lo[k] & 0xffu];
        // (a zero-extended byte: 0xff is its only value >= 0xff)
#pragma unroll
        for (int k = 0; k < NK; ++k) hit[k] = lang[k] < 0xffu;
    } else {
        uint32_t w[kSub];
#pragma unroll
        for (int k = 0; k < NK; ++k) w[k] = img[kBmp1Words + bmp2_word(x.lo[k])];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            // bit (lo & 31) of the word; the offset / width operands of v_bfe
            // take their low 5 bits, so no masking
            hit[k] = __builtin_amdgcn_ubfe(w[k], x.lo[k], 1) != 0u;
            // the key's language by its rank among the 2-byte keys: read for
            // hits only (a missing window costs one LDS read, not three)
            lang[k] = 0;
            if (hit[k])
                lang[k] = l2[b2[bmp2_word(x.lo[k])] +
                             __builtin_popcount(__builtin_amdgcn_ubfe(w[k], 0, x.lo[k]))];
        }
    }
    if constexpr (PACK) {
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            hit[k] = hit[k] && pk->rem[k] >= N;
            lang[k] += (pk->tb[k] >> 8) * 64u * S;
        }
    } else {
        // FULL: more than 192 windows, so only the last sub-block is cut
#pragma unroll
        for (int k = FULL ? kSub - 1 : 0; k < kSub; ++k) hit[k] = hit[k] && 64 * k + lane < nw;
    }
#pragma unroll
    for (int k = 0; k < NK; ++k)
        if (hit[k]) count_inc<PACK>(cnt, lang[k], inc);
}

// Count-mode fast path, gram length N (straight-line code for N = 1..7, so
// the tests of consecutive lengths overlap): test the document's one
// superblock if N is a listed length with table keys, and queue the
// candidates unless the queue would overflow (then `over` is set and the
// document restarts on the general path).
// Count-mode verify of a full queue in the middle of a document's probe
// (hit-dense tables: config 5's 10M keys); counts are order-free, so the
// probe just continues.
template <int S, bool STAGED, int KEYED, bool WIDE, int MODE = 3>
__device__ __forceinline__ void flush_count(const ScoreParams& p, const WaveLds& wl, int qn, const DocSrc& src,
                                            int lane) {
    double acc[S];  // unused in count / class mode
    if (!ablated(p, 1)) flush<S, MODE, STAGED, KEYED, false, WIDE>(p, wl, qn, src, acc, lane, true);
}

// keyed Bloom hash of sub-block k's N-byte window (filter_word, KIND 4)
template <int N>
__device__ __forceinline__ uint32_t keyed_hash(const Windows& x, int k) {
    const uint32_t lo = N >= 4 ? x.lo[k] : x.lo[k] & ((1u << (8 * N)) - 1u);
    const uint32_t hi = N <= 4 ? 0u : x.hi[k] & ((1u << (8 * (N < 7 ? N - 4 : 3))) - 1u);
    return kb_hash(lo, hi, (uint32_t)N);
}

// keyed_hash of sub-block 0's window for a length n known only at run time
// (n in 3..7, after unrolling a constant)
__device__ __forceinline__ uint32_t kb_hash_n(const Windows& x, int n) {
    const uint32_t lo = n >= 4 ? x.lo[0] : x.lo[0] & ((1u << (8 * n)) - 1u);
    const uint32_t hi = n <= 4 ? 0u : x.hi[0] & ((1u << (8 * (n < 7 ? n - 4 : 3))) - 1u);
    return kb_hash(lo, hi, (uint32_t)n);
}

// keyed Bloom (global memory): the words of lengths 3 .. 2 + PRE are loaded
// before the first test, so a document (or pack) waits one memory round trip,
// not one per length; the tests recompute the bit position (VALU is cheap
// next to the latency).  Single documents preload every length 3..7 (config
// 5: 145 -> 121 ms per 10M documents, despite 6 VGPRs spilled), packs 3..5
// (their registers hold the pack's positions).  Longer lengths load at their
// test.  (Diagnostics of the single-document preload: LDGPU_SINGLE_PRELOAD=0
// builds.)
#ifndef LDGPU_SINGLE_PRELOAD
#define LDGPU_SINGLE_PRELOAD 1
#endif
constexpr int kPreN = 5;      // single documents
constexpr int kPackPreN = 3;  // packs

template <int N, int PRE = kPreN>
__device__ __forceinline__ void keyed_preload(const FWords& f, const Windows& x, uint32_t fm, uint32_t (&kw)[kPreN][kSub]) {
    if constexpr (N - 3 < PRE) {
        if ((fm >> N) & 1u) {
#pragma unroll
            for (int k = 0; k < kSub; ++k)
                kw[N - 3][k] = f.gb[(N >= 4 ? f.w3[k] : 0u) + (keyed_hash<N>(x, k) >> kb_sword(N, f.lines, f.gshift))];
        }
    }
}

// fm: p.fast_mask, bit kFmDirect = direct tables present (one SGPR, see
// probe_count_all)
constexpr int kFmDirect = 16;
// bit kFmArgmax: a labels-only count-mode launch (no score / best output):
// its fast-path documents take the count argmax without reading the cold
// parameters per document (config 2: 5.27 -> 5.15 ms, same-box A/B)
constexpr int kFmArgmax = 17;

// kw: the keyed bloom words of lengths 3 .. 2 + kPreN, preloaded together
// (keyed_preload; KEYED == 1 with LDGPU_SINGLE_PRELOAD)
template <int N, bool FULL, int S, bool STAGED, int KEYED, bool WIDE, int MODE = 3>
__device__ __forceinline__ void probe_count(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                            const FWords& f, const Windows& x, int32_t len, int lane, int& qn,
                                            const DocSrc& src, uint32_t fm, const uint32_t (&kw)[kPreN][kSub]) {
    if (!((fm >> N) & 1u)) return;
    if (ablated(p, N <= 2 ? 8 : 16)) return;
    if constexpr (N <= 2) {
        if ((fm >> kFmDirect) & 1u) {
            direct_count<N, FULL>(p, wl, img, x, len - N + 1, lane);
            return;
        }
    }
    constexpr int KIND = N < 3 ? N : kind_of(KEYED);
    constexpr uint32_t sh = N < 3 ? 0u : (KEYED ? (uint32_t)N : pf_shift(N)), mul = N < 3 ? 0u : pf_mult(N);
    uint64_t m[kSub];
    if constexpr (KIND == 4 && N - 3 < kPreN && LDGPU_SINGLE_PRELOAD) {
        // preloaded word: the bit position recomputed (VALU is cheap next to
        // the latency the preload hides)
        const int32_t nw = len - N + 1;
#pragma unroll
        for (int k = 0; k < kSub; ++k) {
            const uint32_t bit = keyed_hash<N>(x, k) >> kb_sbit(N, f.lines, f.gshift);
            m[k] = __builtin_amdgcn_ballot_w64(filter_hit(kw[N - 3][k], bit, bit) && 64 * k + lane < nw);
        }
    } else if constexpr (FULL) {
        test_len<KIND, 4>(img, sh, mul, f, x, len - N + 1, m);
    } else {
        test_nsb<KIND>(img, sh, mul, f, x, len - N + 1, m);
    }
    if (qn + count_sb(m) > kQueueCap) {
        flush_count<S, STAGED, KEYED, WIDE, MODE>(p, wl, qn, src, lane);
        qn = 0;
    }
    append_sb(wl.queue, qn, m, N, 0, lane);
}

template <bool FULL, int S, bool STAGED, int KEYED, bool WIDE, int MODE = 3>
__device__ __forceinline__ void probe_count_all(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                                const FWords& f, const Windows& x, int32_t len, int lane, int& qn,
                                                const DocSrc& src) {
    // the per-length switches as bits of one SGPR, re-read per document (the
    // compiler otherwise hoists seven lane-mask booleans out of the document
    // loop and spills them to VGPR lanes: two v_readlane per test)
    uint32_t fm = __builtin_amdgcn_readfirstlane(p.fast_mask | (p.direct_words ? 1u << kFmDirect : 0u));
    asm volatile("" : "+s"(fm));
    // With direct tables the 1-/2-byte counts never touch the queue: the
    // longer lengths are probed first, their first 64 candidates' slot loads
    // issued, and the direct counts run while those loads are in flight
    // (LDGPU_SPLIT_VERIFY; one-word keys in cuckoo slots only)
    const bool split = LDGPU_SPLIT_VERIFY && !WIDE && !(KEYED && p.buckets) && ((fm >> kFmDirect) & 1u);
    // keyed bloom (config 5): the words of lengths 3 .. 2 + kPreN loaded
    // together before the first test -- one memory round trip instead of one
    // per length (the 1-/2-byte tests run while they are in flight)
    uint32_t kw[kPreN][kSub];
    if constexpr (KEYED == 1 && LDGPU_SINGLE_PRELOAD) {
        keyed_preload<3>(f, x, fm, kw);
        keyed_preload<4>(f, x, fm, kw);
        keyed_preload<5>(f, x, fm, kw);
        keyed_preload<6>(f, x, fm, kw);
        keyed_preload<7>(f, x, fm, kw);
    }
    if (!split) {
        probe_count<1, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
        probe_count<2, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
    }
    probe_count<3, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
    probe_count<4, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
    probe_count<5, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
    probe_count<6, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
    probe_count<7, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
    // wide gram lengths 8..15: one loop, the length a scalar (their filter
    // bits use the first seven bytes: the same two tests as length 7)
    for (uint32_t wm = WIDE ? (fm >> 8) & 0xffu : 0u; wm; wm &= wm - 1u) {
        const int n = 8 + __builtin_ctz(wm);
        const uint32_t sh = KEYED ? (uint32_t)n : pf_shift(n), mul = pf_mult(n);
        constexpr int K3 = kind_of(KEYED);
        uint64_t m[kSub];
        if constexpr (FULL)
            test_len<K3, 4>(img, sh, mul, f, x, len - n + 1, m);
        else
            test_nsb<K3>(img, sh, mul, f, x, len - n + 1, m);
        if (qn + count_sb(m) > kQueueCap) {
            flush_count<S, STAGED, KEYED, WIDE, MODE>(p, wl, qn, src, lane);
            qn = 0;
        }
        append_sb(wl.queue, qn, m, n, 0, lane);
    }
    if (split) {
        VerifyIssue v;
        const bool pending = qn > 0 && !ablated(p, 1);
        if (pending) verify_issue<STAGED>(p, wl, qn, src, lane, v);
        probe_count<1, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
        probe_count<2, FULL, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, len, lane, qn, src, fm, kw);
        if (pending) {
            verify_complete<S, MODE>(p, wl, v);
            if (qn > 64) {
                double acc[S];  // unused in count mode
                flush<S, MODE, STAGED, KEYED, false, WIDE>(p, wl, qn, src, acc, lane, true, 64);
            }
        }
        qn = 0;
    }
}

// Packed short documents (count mode): up to kPackDocs consecutive documents
// of maxg..256 bytes, 256 bytes in all, share one superblock laid over their
// contiguous bytes -- position j is byte j of the pack.  A window is a window
// of the reference (LanguageDetectorModel.scala:139-144, all full-length as
// len >= maxg) iff it ends inside its own document: N <= rem (bytes from j to
// that document's end).  Hits count into the document's own counter block;
// each document's label is its block's count argmax.  Three 64-B documents
// per wave-pass instead of one: the lanes a lone short document leaves idle
// do the next documents' windows.
template <int N, int S, int KEYED, bool WIDE>
__device__ __forceinline__ void probe_pack(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                           const FWords& f, const Windows& x, const PackPos& pk, int lane, int& qn,
                                           const DocSrc& src, uint32_t dummy_a, uint32_t fm,
                                           const uint32_t (&kw)[kPreN][kSub]) {
    if (!((fm >> N) & 1u)) return;
    if (ablated(p, N <= 2 ? 8 : 16)) return;
    if constexpr (N <= 2) {
        if ((fm >> kFmDirect) & 1u) {
            direct_count<N, false, S, true>(p, wl, img, x, 0, lane, &pk);
            return;
        }
    }
    constexpr int KIND = N < 3 ? N : kind_of(KEYED);
    constexpr uint32_t sh = N < 3 ? 0u : (KEYED ? (uint32_t)N : pf_shift(N)), mul = N < 3 ? 0u : pf_mult(N);
    uint64_t m[kSub];
    uint32_t w[kSub], bit[kSub], bit2[kSub];
#pragma unroll
    for (int k = 0; k < kSub; ++k) {
        if constexpr (KIND == 4 && N - 3 < kPackPreN) {
            w[k] = kw[N - 3][k];
            bit[k] = bit2[k] = keyed_hash<N>(x, k) >> kb_sbit(N, f.lines, f.gshift);
        } else {
            filter_word<KIND>(img, sh, mul, f, x, k, w[k], bit[k], bit2[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < kSub; ++k) m[k] = __ballot(filter_hit(w[k], bit[k], bit2[k]) && pk.rem[k] >= N);
    if (qn + count_sb(m) > kQueueCap) {
        double acc[S];  // unused in count mode
        flush<S, 3, true, KEYED, true, WIDE>(p, wl, qn, src, acc, lane, true);
        qn = 0;
    }
    append_pack(wl.queue, qn, m, (uint32_t)N, pk, dummy_a);
}

#ifndef LDGPU_PACK_KOUTER
#define LDGPU_PACK_KOUTER 1
#endif

// Packs, one sub-block at a time (LDGPU_PACK_KOUTER): count mode is order-
// free, so the 64 positions of sub-block k are tested for every gram length
// before sub-block k + 1 is loaded -- only one position's window bytes, bloom
// chunk / word and pack position are live per lane (the pack kernel ran at
// the 80-VGPR cap with 14 VGPRs spilled when all four sub-blocks' were: config
// 4's scratch writes).  Sub-block k's tests of length N (x, f, pk hold the
// lane's position 64 k + lane in their index 0).
template <int N, int S, int KEYED, bool WIDE>
__device__ __forceinline__ void probe_pack1(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                            const FWords& f, const Windows& x, const PackPos& pk, int lane, int& qn,
                                            const DocSrc& src, uint32_t dummy_a, uint32_t fm,
                                            const uint32_t (&kw)[kPreN][kSub]) {
    if (!((fm >> N) & 1u)) return;
    if (ablated(p, N <= 2 ? 8 : 16)) return;
    if constexpr (N <= 2) {
        if ((fm >> kFmDirect) & 1u) {
            direct_count<N, false, S, true, 1>(p, wl, img, x, 0, lane, &pk);
            return;
        }
    }
    constexpr int KIND = N < 3 ? N : kind_of(KEYED);
    constexpr uint32_t sh = N < 3 ? 0u : (KEYED ? (uint32_t)N : pf_shift(N)), mul = N < 3 ? 0u : pf_mult(N);
    uint32_t w, bit, bit2;
    if constexpr (KIND == 4 && N - 3 < kPackPreN) {
        w = kw[N - 3][0];
        bit = bit2 = keyed_hash<N>(x, 0) >> kb_sbit(N, f.lines, f.gshift);
    } else {
        filter_word<KIND>(img, sh, mul, f, x, 0, w, bit, bit2);
    }
    uint64_t m[kSub] = {__ballot(filter_hit(w, bit, bit2) && pk.rem[0] >= N), 0, 0, 0};
    if (qn + __popcll(m[0]) > kQueueCap) {
        double acc[S];  // unused in count mode
        flush<S, 3, true, KEYED, true, WIDE>(p, wl, qn, src, acc, lane, true);
        qn = 0;
    }
    append_pack(wl.queue, qn, m, (uint32_t)N, pk, dummy_a);
}

template <int S, int KEYED, bool WIDE>
__device__ __forceinline__ void score_pack_kouter(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                                  const uint32_t* bloom, const DocSrc& src, int32_t e1, int32_t e2,
                                                  int32_t e3, int32_t tot, int nd, int i, int lane) {
    uint32_t fm = __builtin_amdgcn_readfirstlane(p.fast_mask | (p.direct_words ? 1u << kFmDirect : 0u));
    asm volatile("" : "+s"(fm));
    int qn = 0;
    if (ablated(p, 2)) fm = 0;
    const uint32_t dummy_a = (uint32_t)(uintptr_t)(reinterpret_cast<uint32_t*>(wl.hits) + lane);
#pragma unroll 1
    for (int k = 0; 64 * k < tot; ++k) {  // (uniform: tot <= 256)
        Windows x;
        {
            const uint32_t a = (uint32_t)src.base + 64u * k + (uint32_t)lane;
            const uint32_t sh = a & 3u;
            const uint32_t* w = src.lds + (a >> 2);
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
            x.lo[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
            x.hi[0] = __builtin_amdgcn_alignbyte(w2, w1, sh);
        }
        FWords f;
        if constexpr (KEYED == 2) {
            f.ck[0] = reinterpret_cast<const u32x4*>(bloom)[kb_chunk(x.lo[0]) >> p.bloom_shift];
        } else if constexpr (KEYED) {
            f.gb = bloom;
            f.gshift = p.bloom_shift;
            f.lines = p.kb_lines != 0;
            f.w3[0] = f.lines ? kb_line16(x.lo[0], p.bloom_shift) : 0u;
        } else {
            f.w3[0] = bloom[pf_word(x.lo[0], p.bloom_shift)];
        }
        PackPos pk;
        {
            const int32_t j = 64 * k + lane;
            const uint32_t d = (uint32_t)(j >= e1) + (uint32_t)(j >= e2) + (uint32_t)(j >= e3);
            const int32_t end = j < e1 ? e1 : (j < e2 ? e2 : (j < e3 ? e3 : tot));
            pk.rem[0] = end - j;
            pk.tb[0] = (d << 8) | (uint32_t)j;
        }
        uint32_t kw[kPreN][kSub];
        if constexpr (KEYED == 1) {
#pragma unroll
            for (int n = 3; n < 3 + kPackPreN; ++n)
                if ((fm >> n) & 1u)
                    kw[n - 3][0] = f.gb[(n >= 4 ? f.w3[0] : 0u) + (kb_hash_n(x, n) >> kb_sword(n, f.lines, f.gshift))];
        }
        probe_pack1<1, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
        probe_pack1<2, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
        probe_pack1<3, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
        probe_pack1<4, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
        probe_pack1<5, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
        probe_pack1<6, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
        probe_pack1<7, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
        for (uint32_t wm = WIDE ? (fm >> 8) & 0xffu : 0u; wm; wm &= wm - 1u) {  // wide lengths 8..15
            const int n = 8 + __builtin_ctz(wm);
            constexpr int K3 = kind_of(KEYED);
            const uint32_t sh = KEYED ? (uint32_t)n : pf_shift(n), mul = pf_mult(n);
            uint32_t w, bit, bit2;
            filter_word<K3>(img, sh, mul, f, x, 0, w, bit, bit2);
            uint64_t m[kSub] = {__ballot(filter_hit(w, bit, bit2) && pk.rem[0] >= n), 0, 0, 0};
            if (qn + __popcll(m[0]) > kQueueCap) {
                double acc[S];
                flush<S, 3, true, KEYED, true, WIDE>(p, wl, qn, src, acc, lane, true);
                qn = 0;
            }
            append_pack(wl.queue, qn, m, (uint32_t)n, pk, dummy_a);
        }
    }
    if (ablated(p, 1)) qn = 0;
    if (qn) {
        double acc[S];
        flush<S, 3, true, KEYED, true, WIDE>(p, wl, qn, src, acc, lane, true);
    }
    for (int q = 0; q < (ablated(p, 32) ? 0 : nd); ++q) {
        const int lab = count_argmax<S>(p, reinterpret_cast<uint16_t*>(count_area(wl)) + q * 64 * S, lane);
        if (lane == 0) wl.labels[i + q] = lab;
    }
}

// One pack: documents [i, i + nd) of the staged group, ends e1 < e2 < e3 <=
// tot relative to the pack's first byte (unused ends = tot); labels to
// wl.labels[i ..).
template <int S, int KEYED, bool WIDE>
__device__ __forceinline__ void score_pack(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                        const uint32_t* bloom, const DocSrc& src, int32_t e1, int32_t e2,
                                        int32_t e3, int32_t tot, int nd, int i, int lane) {
    Windows x;
    load_windows<true>(p, src, 0, lane, x);
    FWords f;
    load_fwords<KEYED>(p, bloom, x, f);
    PackPos pk;
#pragma unroll
    for (int k = 0; k < kSub; ++k) {
        const int32_t j = 64 * k + lane;
        const uint32_t d = (uint32_t)(j >= e1) + (uint32_t)(j >= e2) + (uint32_t)(j >= e3);
        const int32_t end = j < e1 ? e1 : (j < e2 ? e2 : (j < e3 ? e3 : tot));
        pk.rem[k] = end - j;
        pk.tb[k] = (d << 8) | (uint32_t)j;
    }
    uint32_t fm = __builtin_amdgcn_readfirstlane(p.fast_mask | (p.direct_words ? 1u << kFmDirect : 0u));
    asm volatile("" : "+s"(fm));
    int qn = 0;
    if (ablated(p, 2)) fm = 0;
    const uint32_t dummy_a = (uint32_t)(uintptr_t)(reinterpret_cast<uint32_t*>(wl.hits) + lane);
    uint32_t kw[kPreN][kSub];
    if constexpr (KEYED == 1) {
        keyed_preload<3, kPackPreN>(f, x, fm, kw);
        keyed_preload<4, kPackPreN>(f, x, fm, kw);
        keyed_preload<5, kPackPreN>(f, x, fm, kw);
    }
    probe_pack<1, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
    probe_pack<2, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
    probe_pack<3, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
    probe_pack<4, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
    probe_pack<5, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
    probe_pack<6, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
    probe_pack<7, S, KEYED, WIDE>(p, wl, img, f, x, pk, lane, qn, src, dummy_a, fm, kw);
    for (uint32_t wm = WIDE ? (fm >> 8) & 0xffu : 0u; wm; wm &= wm - 1u) {  // wide lengths 8..15
        const int n = 8 + __builtin_ctz(wm);
        constexpr int K3 = kind_of(KEYED);
        const uint32_t sh = KEYED ? (uint32_t)n : pf_shift(n), mul = pf_mult(n);
        uint64_t m[kSub];
        uint32_t w[kSub], bit[kSub], bit2[kSub];
#pragma unroll
        for (int k = 0; k < kSub; ++k) filter_word<K3>(img, sh, mul, f, x, k, w[k], bit[k], bit2[k]);
#pragma unroll
        for (int k = 0; k < kSub; ++k) m[k] = __ballot(filter_hit(w[k], bit[k], bit2[k]) && pk.rem[k] >= n);
        if (qn + count_sb(m) > kQueueCap) {
            double acc[S];
            flush<S, 3, true, KEYED, true, WIDE>(p, wl, qn, src, acc, lane, true);
            qn = 0;
        }
        append_pack(wl.queue, qn, m, (uint32_t)n, pk, dummy_a);
    }
    if (ablated(p, 1)) qn = 0;
    if (qn) {
        double acc[S];
        flush<S, 3, true, KEYED, true, WIDE>(p, wl, qn, src, acc, lane, true);
    }
    for (int q = 0; q < (ablated(p, 32) ? 0 : nd); ++q) {
        const int lab = count_argmax<S>(p, reinterpret_cast<uint16_t*>(count_area(wl)) + q * 64 * S, lane);
        if (lane == 0) wl.labels[i + q] = lab;
    }
}

// Score one document (probe -> verify/accumulate -> argmax -> outputs).
template <int S, int MODE, bool STAGED, int KEYED, bool WIDE>
__device__ __forceinline__ int score_doc(const ScoreParams& p, const WaveLds& wl, const uint32_t* img,
                                          const uint32_t* bloom, int64_t doc, int64_t b, int64_t len,
                                          const DocSrc& src, int lane) {
    double acc[S];
#pragma unroll
    for (int s = 0; s < S; ++s) acc[s] = 0.0;
    int qn = 0;
    bool general = !(len >= p.maxg && len <= 64 * kSub);
    if (!general) {
        // fast path: every window is full-length (klen = n) and one
        // superblock covers the document, so every gram length reuses the
        // same window bytes and prefix-Bloom words.  Count mode (hit order
        // free): the host packs each DISTINCT length once and its hits count
        // its multiplicity in gramLengths.  The candidates of all lengths
        // are verified together, or in order whenever the next length's
        // would overflow the queue.
        if (p.n_fast && !ablated(p, 2)) {
            Windows x;
            load_windows<STAGED>(p, src, 0, lane, x);
            FWords f;
            load_fwords<KEYED>(p, bloom, x, f);
            if constexpr (MODE == 3 || MODE == 4) {
                if (len >= 192 + p.maxg)
                    probe_count_all<true, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, (int32_t)len, lane, qn, src);
                else
                    probe_count_all<false, S, STAGED, KEYED, WIDE, MODE>(p, wl, img, f, x, (int32_t)len, lane, qn, src);
            }
            uint64_t gq = p.gpack[0];
            for (int gi = 0; gi < (MODE == 3 || MODE == 4 ? 0 : p.n_fast); ++gi) {
                const int n = (int)(gq & 15u);
                gq = (gi & 15) == 15 ? p.gpack[1] : gq >> 4;
                // pin the tests inside this loop: hoisted out of it (they are
                // loop-invariant), the tests of all lengths would run per doc
#pragma unroll
                for (int k = 0; k < kSub; ++k) asm volatile("" : "+v"(x.lo[k]), "+v"(x.hi[k]), "+v"(f.w3[k]));
                uint64_t m[kSub];
                if (len >= 192 + p.maxg)
                    test_sb<true, KEYED>(img, n, f, x, (int32_t)len - n + 1, m);
                else
                    test_sb<false, KEYED>(img, n, f, x, (int32_t)len - n + 1, m);
                if (qn + count_sb(m) > kQueueCap) {
                    // verify and replay the queued candidates (they precede
                    // this length's in reference order) and go on: a table
                    // holding the 1-/2-byte grams of the text queues ~510
                    // candidates per 256-B document, more than the queue
                    flush<S, MODE, STAGED, KEYED, false, WIDE>(p, wl, qn, src, acc, lane);
                    qn = 0;
                }
                append_sb(wl.queue, qn, m, n, 0, lane);
            }
            if (!general) {
                if (ablated(p, 1)) qn = 0;
                if (qn) flush<S, MODE, STAGED, KEYED, false, WIDE>(p, wl, qn, src, acc, lane, MODE == 3 || MODE == 4);
            }
            qn = 0;
        }
    }
    if (!general) {
    } else if (len >= kMaxDocBytes) {
        if (lane == 0) with_cold<KEYED>(p, [](const auto& q) { atomicOr(q.err, 2); });
    } else {
        // general path: partial windows (len < n) and long documents; n outer
        // (reference order), superblocks inner
        const int nG = with_cold<KEYED>(p, [](const auto& q) { return q.nG; });
        for (int gi = 0; gi < nG; ++gi) {
            const int n = with_cold<KEYED>(p, [&](const auto& q) { return q.G[gi]; });
            const uint32_t lm = with_cold<KEYED>(p, [](const auto& q) { return q.len_mask; });
            const GramCtx g = gram_ctx(len, n);
            if (!((lm >> g.klen) & 1u) || ablated(p, 2)) continue;
            for (int32_t p0 = 0; p0 < g.nwin; p0 += 64 * kSub) {
                Windows x;
                load_windows<STAGED>(p, src, p0, lane, x);
                FWords f;
                if (g.klen >= 3) load_fwords<KEYED>(p, bloom, x, f);
                uint64_t m[kSub];
                test_sb<false, KEYED>(img, g.klen, f, x, g.nwin - p0, m);
                if (qn + count_sb(m) > kQueueCap) {
                    flush<S, MODE, STAGED, KEYED, false, WIDE>(p, wl, qn, src, acc, lane);
                    qn = 0;
                }
                append_sb(wl.queue, qn, m, g.klen, p0, lane);
            }
        }
    }
    if (ablated(p, 1)) qn = 0;
    if (qn) flush<S, MODE, STAGED, KEYED, false, WIDE>(p, wl, qn, src, acc, lane);
    if constexpr (MODE == 4) return ablated(p, 32) ? 0 : class_label<S>(p, count_area(wl), lane);
    if constexpr (MODE == 3) {
        if (ablated(p, 32)) return 0;
        if (!general && ((p.fast_mask >> kFmArgmax) & 1u)) return count_argmax<S>(p, count_area(wl), lane);
        if (with_cold<KEYED>(p, [&](const auto& q) { return !q.scores && !q.best && len <= q.count_argmax_len; }))
            return count_argmax<S>(p, count_area(wl), lane);
        count_scores<S>(p, wl, acc, lane);
    }

    // argmax (breeze: first element, then strict '>' updates): the wave max M
    // of the non-NaN scores by DPP (no LDS), then the first index holding M;
    // a NaN first score keeps index 0.
    double lv = -__builtin_inf();
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int l = s * 64 + lane;
        if (l < p.L && !__builtin_isnan(acc[s]) && acc[s] > lv) lv = acc[s];
    }
    const double M = wave_max_f64(lv);
    int label = 0;
    bool found = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const uint64_t b = __ballot(s * 64 + lane < p.L && acc[s] == M);
        if (!found && b) {
            label = s * 64 + __builtin_ctzll(b);
            found = true;
        }
    }
    // breeze keeps index 0 when the first score is NaN (NaN never compares
    // greater); in a language block other than the first, a NaN is just
    // never the maximum
    const bool nan_first = with_cold<KEYED>(p, [](const auto& q) { return q.block == 0; }) &&
                           __builtin_isnan(rdlaned(acc[0], 0));
    if (nan_first) label = 0;
    double* const best = with_cold<KEYED>(p, [](const auto& q) { return q.best; });
    if (best && lane == 0) best[doc] = nan_first ? __builtin_inf() : M;
    double* const scores = with_cold<KEYED>(p, [](const auto& q) { return q.scores; });
    if (scores) {
        const int64_t stride = with_cold<KEYED>(p, [](const auto& q) { return q.score_stride; });
        double* out = scores + doc * (stride ? stride : (int64_t)p.L);
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int l = s * 64 + lane;
            if (l < p.L) out[l] = acc[s];
        }
    }
    return label;
}

__device__ __forceinline__ int64_t rdlane_i64(int64_t v, int l) { return (int64_t)rdlane64((uint64_t)v, l); }


// LDS-DMA of a group's bytes [s0, s0 + kBufBytes) into dst (wave-uniform LDS
// address; lane i's 16 B land at dst + 16 i), range-checked: bytes past
// n_bytes read as 0, never fault.
// lane id recomputed in place (mbcnt): never spilled, never a scratch reload
// (whose vmcnt wait would drain the in-flight group DMA)
__device__ __forceinline__ uint32_t fresh_lane() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ void group_dma(const ScoreParams& p, int64_t s0, uint32_t* dst) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(p.bytes + s0));
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)(p.bytes + s0) >> 32));
    const int64_t left = ((p.n_bytes + 3) & ~(int64_t)3) - s0;
    const uint32_t nrec =
        __builtin_amdgcn_readfirstlane((uint32_t)(left < 0 ? 0 : (left > 0x7ffffff0 ? 0x7ffffff0 : left)));
    void* base = (void*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)nrec, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, 16 * fresh_lane(), 0,
                                             0, 0);
}

// Issue the 16-B-per-lane buffer load of a group's bytes [s0, s0 + kBufBytes)
// (range-checked: bytes past n_bytes read as 0, never fault).
__device__ __forceinline__ void group_load(const ScoreParams& p, int64_t s0, int lane, uint4& r0) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(p.bytes + s0));
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)(p.bytes + s0) >> 32));
    // whole dwords: the range check zeroes a dword with ANY byte past the end
    const int64_t left = ((p.n_bytes + 3) & ~(int64_t)3) - s0;
    const uint32_t nrec =
        __builtin_amdgcn_readfirstlane((uint32_t)(left < 0 ? 0 : (left > 0x7ffffff0 ? 0x7ffffff0 : left)));
    void* base = (void*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)nrec, 0x00020000);
    r0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, 16 * lane, 0, 0));
}

// PACK (count mode only): a separate instantiation with the pack path, so the
// pack path's registers never burden the single-document kernels
// BL: the bloom layout (KEYED of the device functions): 0 = prefix Bloom in
// LDS, 1 = keyed bloom (words / lines), 2 = keyed chunks
// INVARIANT (cold_params): ScoreParams is the kernel's first and only explicit
// argument, so it sits at offset 0 of the kernarg segment; the static_assert
// after the kernel checks the signature.
// IND (mode 1 only): the indirect launch of class mode's exact replay -- wave w
// scores documents p.doc_idx[i], i = w, w + waves, ... < *p.n_docs_dev (count
// written by the device), each in place from global memory, its label stored
// to labels[doc_idx[i]]; workgroups with no document exit before staging.
#ifndef LDGPU_LATE_OFFSETS
#define LDGPU_LATE_OFFSETS 1
#endif
template <int S, int MODE, int BL, bool PACK = false, bool WIDE = false, bool IND = false>
__global__ __launch_bounds__(kScoreWaves * 64, kScoreMinWgPerCu * kScoreWaves / 4) void score_kernel(const ScoreParams p) {
    constexpr bool FLDS = BL == 0;
    // the kernels at the register cap (packs, global-memory blooms) load the
    // next group's offsets after the group's documents, not before
    constexpr bool kLateOffsets = LDGPU_LATE_OFFSETS && (PACK || BL != 0);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int64_t n_ind = 0;
    if constexpr (IND) {
        n_ind = (int64_t)*p.n_docs_dev;  // (uniform address: a scalar load)
        if ((int64_t)blockIdx.x * kScoreWaves >= n_ind) return;
    }
    const uint32_t img_words = kBloomBase + (FLDS ? p.bloom_words : 0u) + p.direct_words;
    {
        const uint4* src = reinterpret_cast<const uint4*>(p.filter);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = tid; i < (img_words >> 2); i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    const uint32_t* bloom = FLDS ? lds + kBloomBase : p.filter + kBloomBase;
    WaveLds wl;
    wl.queue = lds + img_words + wave * kQueueCap;
    // class mode: the hit area holds the table's classes' counters only
    const uint32_t kHitW = MODE == 4 ? __builtin_amdgcn_readfirstlane(p.hit_words) : hit_area_words(S, MODE, PACK);
    wl.hits = reinterpret_cast<uint64_t*>(lds + img_words + kScoreWaves * kQueueCap + wave * kHitW);
    wl.buf = lds + img_words + kScoreWaves * (kQueueCap + kHitW) + wave * 2 * kBufWords;
    wl.labels = lds + img_words + kScoreWaves * (kQueueCap + kHitW + 2 * kBufWords) + wave * 64;
    wl.cnt = reinterpret_cast<uint32_t*>(wl.hits) + (PACK ? 64 : 0);

    if constexpr (MODE == 3) {
        uint32_t* cnt = count_area(wl);
#pragma unroll
        for (int s = 0; s < S * (PACK ? (int)kPackDocs / 2 : 1); ++s) cnt[64 * s + lane] = 0;
        __builtin_amdgcn_wave_barrier();
    }
    if constexpr (MODE == 4) {  // (class, language) counters: the whole hit area
        uint32_t* cnt = count_area(wl);
        for (uint32_t i = (uint32_t)lane; i < kHitW; i += 64) cnt[i] = 0;
        __builtin_amdgcn_wave_barrier();
    }

    if constexpr (IND) {
        const int64_t nw = (int64_t)gridDim.x * kScoreWaves;
        for (int64_t i = (int64_t)blockIdx.x * kScoreWaves + wave; i < n_ind; i += nw) {
            const int64_t d = p.doc_idx[i];
            const int64_t b = p.offsets[d], len = p.offsets[d + 1] - b;
            const int lab = score_doc<S, MODE, false, BL, WIDE>(p, wl, lds, bloom, d, b, len, DocSrc{nullptr, b}, lane);
            if (lane == 0) p.labels[d] = lab;
        }
        return;
    }

    // this wave's contiguous range of documents, walked in groups of p.group
    const int64_t nwaves = (int64_t)gridDim.x * kScoreWaves;
    const int64_t wg = (int64_t)blockIdx.x * kScoreWaves + wave;
    const int64_t dbeg = (int64_t)((__int128)p.n_docs * wg / nwaves);
    const int64_t dend = (int64_t)((__int128)p.n_docs * (wg + 1) / nwaves);
    if (dbeg >= dend) return;
    const int G = p.group;

    // lane i <= G holds offsets[g0 + i] of the current group (clamped to dend).
    // Group bytes are staged by LDS-DMA into a double buffer: the next
    // group's load is in flight while this group is scored, and no VGPR
    // holds it.
    uint32_t* const buf0 = wl.buf;
    uint32_t* const buf1 = wl.buf + kBufWords;
    int64_t g0 = dbeg;
    int64_t offv = p.offsets[min(g0 + (int64_t)min(lane, G), dend)];
    group_dma(p, rdlane_i64(offv, 0) & ~(int64_t)15, buf0);
    bool par = false;
    int64_t prev_g0 = 0;
    int prev_cnt = 0;

    while (g0 < dend) {
        // this group's bytes (DMA issued one group ago) have landed, and the
        // previous group's label store has drained
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        // this group: as many consecutive whole documents as the staging
        // buffer holds from s0 (at least one; offsets never decrease, so
        // the lanes that fit are a prefix)
        const int64_t s0 = rdlane_i64(offv, 0) & ~(int64_t)15;
        const int lim = (int)min((int64_t)G, dend - g0);
        const int fl = (int)fresh_lane();
        const int cnt = max(1, (int)__popcll(__ballot(fl >= 1 && fl <= lim && offv - s0 <= (int64_t)kBufBytes)));
        const int64_t g1 = g0 + cnt;
        const int64_t send = rdlane_i64(offv, cnt);
        const bool staged = send - s0 <= kBufBytes;
        uint32_t* const cur = par ? buf1 : buf0;
        // bytes and offsets of the next group (hidden behind this group's work)
        if (g1 < dend) group_dma(p, send & ~(int64_t)15, par ? buf0 : buf1);
        const int64_t n1 = min(g1 + (int64_t)G, dend);
        int64_t offn = 0;
        if constexpr (!kLateOffsets) offn = p.offsets[min(g1 + (int64_t)min((int)fresh_lane(), G), n1)];
        // the previous group's labels: one coalesced store
        {
            const uint32_t l = fresh_lane();
            if ((int)l < prev_cnt) p.labels[prev_g0 + l] = (int32_t)wl.labels[l];
        }
        __builtin_amdgcn_wave_barrier();
        if (staged) {
            for (int i = 0; i < cnt;) {
                const int64_t b = rdlane_i64(offv, i);
                const int64_t len = rdlane_i64(offv, i + 1) - b;
                const DocSrc src{cur, b - s0};
                if constexpr (PACK) {
                    // a pack of consecutive short documents (score_pack);
                    // packing runs only without score output, with count
                    // argmax and fast lengths
                    if (len >= p.maxg && len <= 128) {
                        int32_t e[kPackDocs];
                        e[0] = (int32_t)len;
                        int nd = 1;
                        while (nd < kPackDocs && i + nd < cnt) {
                            const int64_t l2 = rdlane_i64(offv, i + nd + 1) - rdlane_i64(offv, i + nd);
                            if (l2 < p.maxg || e[nd - 1] + l2 > 64 * kSub) break;
                            e[nd] = e[nd - 1] + (int32_t)l2;
                            ++nd;
                        }
                        if (nd > 1) {
                            const int32_t tot = e[nd - 1];
                            if constexpr (LDGPU_PACK_KOUTER)
                                score_pack_kouter<S, BL, WIDE>(p, wl, lds, bloom, src, e[0], nd > 2 ? e[1] : tot,
                                                               nd > 3 ? e[2] : tot, tot, nd, i, lane);
                            else
                                score_pack<S, BL, WIDE>(p, wl, lds, bloom, src, e[0], nd > 2 ? e[1] : tot,
                                                     nd > 3 ? e[2] : tot, tot, nd, i, lane);
                            i += nd;
                            continue;
                        }
                    }
                }
                const int lab = score_doc<S, MODE, true, BL, WIDE>(p, wl, lds, bloom, g0 + i, b, len, src, lane);
                if (lane == 0) wl.labels[i] = lab;
                ++i;
            }
        } else {
            for (int i = 0; i < cnt; ++i) {
                const int64_t b = rdlane_i64(offv, i);
                const int64_t len = rdlane_i64(offv, i + 1) - b;
                const DocSrc src{nullptr, b};
                const int lab = score_doc<S, MODE, false, BL, WIDE>(p, wl, lds, bloom, g0 + i, b, len, src, lane);
                if (lane == 0) wl.labels[i] = lab;
            }
        }
        __builtin_amdgcn_wave_barrier();
        // (kLateOffsets: the next group's offsets loaded only now -- held in
        // registers across the group's documents they were spilled to
        // scratch, one 512-B store + reload per group: config 4's writes)
        if constexpr (kLateOffsets) offn = p.offsets[min(g1 + (int64_t)min((int)fresh_lane(), G), n1)];
        prev_g0 = g0;
        prev_cnt = cnt;
        offv = offn;
        g0 = g1;
        par = !par;
    }
    if (lane < prev_cnt) p.labels[prev_g0 + lane] = (int32_t)wl.labels[lane];
}

template <int S, int MODE, int BL, bool WIDE>
hipError_t launch_w(const ScoreParams& p, int grid, hipStream_t stream) {
    const bool pack = MODE == 3 && p.pack;
    const size_t lds = score_lds_bytes(S, MODE, kBloomBase + (BL == 0 ? p.bloom_words : 0u) + p.direct_words, pack,
                                       MODE == 4 ? p.hit_words : 0u);
    if constexpr (MODE == 1) {
        if (p.doc_idx) {
            hipLaunchKernelGGL((score_kernel<S, MODE, BL, false, WIDE, true>), dim3(grid), dim3(kScoreWaves * 64), lds,
                               stream, p);
            return hipGetLastError();
        }
    }
    if constexpr (MODE == 3) {
        if (pack) {
            hipLaunchKernelGGL((score_kernel<S, MODE, BL, true, WIDE>), dim3(grid), dim3(kScoreWaves * 64), lds,
                               stream, p);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((score_kernel<S, MODE, BL, false, WIDE>), dim3(grid), dim3(kScoreWaves * 64), lds, stream, p);
    return hipGetLastError();
}

// tables with wide keys (8..15 bytes) run the WIDE instantiations
template <int S, int MODE, int BL>
hipError_t launch_t(const ScoreParams& p, int grid, hipStream_t stream) {
    return p.wslots ? launch_w<S, MODE, BL, true>(p, grid, stream) : launch_w<S, MODE, BL, false>(p, grid, stream);
}

template <int S, int MODE, int BL, bool PACK = false, bool WIDE = false, bool IND = false>
hipError_t prepare_k(size_t lds, int* blocks) {
    const void* f = reinterpret_cast<const void*>(&score_kernel<S, MODE, BL, PACK, WIDE, IND>);
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, f, kScoreWaves * 64, lds);
}

// count mode prepares both instantiations (single documents, packs); the
// resident workgroups are the smaller of the two
template <int S, int MODE, int BL>
hipError_t prepare_t(size_t lds, int* blocks) {
    hipError_t e = prepare_k<S, MODE, BL>(lds, blocks);
    int b2 = 0;
    if (e == hipSuccess) e = prepare_k<S, MODE, BL, false, true>(lds, &b2);
    if (e == hipSuccess) *blocks = std::min(*blocks, b2);
    if constexpr (MODE == 1) {  // (the indirect replay: its LDS limit; it never sets the grid)
        int b3 = 0;
        if (e == hipSuccess) e = prepare_k<S, MODE, BL, false, false, true>(lds, &b3);
        if (e == hipSuccess) e = prepare_k<S, MODE, BL, false, true, true>(lds, &b3);
    }
    if constexpr (MODE == 3) {
        if (e == hipSuccess) e = prepare_k<S, MODE, BL, true>(lds, &b2);
        if (e == hipSuccess) *blocks = std::min(*blocks, b2);
        if (e == hipSuccess) e = prepare_k<S, MODE, BL, true, true>(lds, &b2);
        if (e == hipSuccess) *blocks = std::min(*blocks, b2);
    }
    return e;
}

// cold_params() reads the kernarg segment as a ScoreParams: any other
// argument list for score_kernel must change cold_params first
template <typename T>
struct ParamsOnlyKernel : std::false_type {};
template <>
struct ParamsOnlyKernel<void (*)(ScoreParams)> : std::true_type {};
static_assert(ParamsOnlyKernel<decltype(&score_kernel<1, 3, 0, false, false>)>::value &&
                  ParamsOnlyKernel<decltype(&score_kernel<4, 1, 1, true, true>)>::value &&
                  ParamsOnlyKernel<decltype(&score_kernel<2, 1, 0, false, true, true>)>::value,
              "score_kernel must take exactly one argument, ScoreParams (cold_params reads it at kernarg offset 0)");

constexpr int kM = LDGPU_SCORE_MODE, kS = LDGPU_SCORE_S;

// LDGPU_NARROW_VARIANT (tuning builds only, tools/build_variant.sh): just the
// kernels of one bench configuration, compiled in a minute instead of ten:
//   1: config 2 -- LDS bloom, one slice, count mode and the finite-value replay
//   4: config 4 -- keyed bloom in chunks, two slices (L = 100), count mode
//   5: config 5 -- keyed bloom in lines, four slices (L = 200), count mode
// kNarrowBl: the one bloom layout built (-1: every layout, a product build)
#if !defined(LDGPU_NARROW_VARIANT)
constexpr bool kBuilt = true;
constexpr int kNarrowBl = -1;
#elif LDGPU_NARROW_VARIANT == 4
constexpr bool kBuilt = kM == 3 && kS == 2;
constexpr int kNarrowBl = 2;
#elif LDGPU_NARROW_VARIANT == 5
constexpr bool kBuilt = kM == 3 && kS == 4;
constexpr int kNarrowBl = 1;
#else
constexpr bool kBuilt = (kM == 3 || kM == 1) && kS == 1;
constexpr int kNarrowBl = 0;
#endif

// the bloom layout of a launch: 0 = prefix Bloom in LDS, 2 = keyed chunks
// (built for count-mode tables only), 1 = keyed words / lines
int bloom_layout(bool lds_bloom, bool chunks) { return lds_bloom ? 0 : (kM == 3 && chunks ? 2 : 1); }

}  // namespace

#define LDGPU_CAT4(a, b, c, d) a##b##c##d
#define LDGPU_FN(pre, m, s) LDGPU_CAT4(pre, m, _, s)

hipError_t LDGPU_FN(launch_score_, LDGPU_SCORE_MODE, LDGPU_SCORE_S)(const ScoreParams& p, bool lds_bloom, int grid,
                                                                   hipStream_t stream) {
    if constexpr (!kBuilt) {
        return hipErrorInvalidValue;
    } else {
        const int bl = bloom_layout(lds_bloom, p.kb_chunks != 0);
        if constexpr (kNarrowBl < 0 || kNarrowBl == 0) {
            if (bl == 0) return launch_t<kS, kM, 0>(p, grid, stream);
        }
        if constexpr (kM == 3 && (kNarrowBl < 0 || kNarrowBl == 2)) {
            if (bl == 2) return launch_t<kS, kM, 2>(p, grid, stream);
        }
        if constexpr (kNarrowBl < 0 || kNarrowBl == 1) {
            if (bl == 1) return launch_t<kS, kM, 1>(p, grid, stream);
        }
        return hipErrorInvalidValue;
    }
}

hipError_t LDGPU_FN(prepare_score_, LDGPU_SCORE_MODE, LDGPU_SCORE_S)(bool lds_bloom, bool chunks, size_t lds,
                                                                    int* blocks) {
    if constexpr (!kBuilt) {
        return hipErrorInvalidValue;
    } else {
        const int bl = bloom_layout(lds_bloom, chunks);
        if constexpr (kNarrowBl < 0 || kNarrowBl == 0) {
            if (bl == 0) return prepare_t<kS, kM, 0>(lds, blocks);
        }
        if constexpr (kM == 3 && (kNarrowBl < 0 || kNarrowBl == 2)) {
            if (bl == 2) return prepare_t<kS, kM, 2>(lds, blocks);
        }
        if constexpr (kNarrowBl < 0 || kNarrowBl == 1) {
            if (bl == 1) return prepare_t<kS, kM, 1>(lds, blocks);
        }
        return hipErrorInvalidValue;
    }
}

#else  // the dispatch translation unit

namespace {

// first maximum across language blocks: block maxima compared with '>' in
// block order, as breeze's argmax compares scores in language order
__global__ void combine_blocks_kernel(int64_t n, int nb, const int32_t* lab, const double* best, int32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t l = lab[i];
    double m = best[i];
    for (int b = 1; b < nb; ++b) {
        const double v = best[(int64_t)b * n + i];
        if (v > m) {
            m = v;
            l = kBlockLangs * b + lab[(int64_t)b * n + i];
        }
    }
    out[i] = l;
}

}  // namespace

hipError_t launch_combine_blocks(int64_t n, int nb, const int32_t* lab, const double* best, int32_t* out,
                                 hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(combine_blocks_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, n, nb, lab, best,
                       out);
    return hipGetLastError();
}

#define LDGPU_SCORE_CASE(m, s, ...)  \
    case (m) * 8 + (s):                \
        return launch_score_##m##_##s(__VA_ARGS__);
#define LDGPU_PREPARE_CASE(m, s, ...)  \
    case (m) * 8 + (s):                  \
        return prepare_score_##m##_##s(__VA_ARGS__);
#define LDGPU_FOR_PAIRS(X, ...)                                                                              \
    X(0, 1, __VA_ARGS__) X(0, 2, __VA_ARGS__) X(0, 3, __VA_ARGS__) X(0, 4, __VA_ARGS__) X(1, 1, __VA_ARGS__) \
    X(1, 2, __VA_ARGS__) X(1, 3, __VA_ARGS__) X(1, 4, __VA_ARGS__) X(2, 1, __VA_ARGS__) X(2, 2, __VA_ARGS__) \
    X(2, 3, __VA_ARGS__) X(2, 4, __VA_ARGS__) X(3, 1, __VA_ARGS__) X(3, 2, __VA_ARGS__) X(3, 3, __VA_ARGS__) \
    X(3, 4, __VA_ARGS__) X(4, 1, __VA_ARGS__) X(4, 2, __VA_ARGS__) X(4, 3, __VA_ARGS__) X(4, 4, __VA_ARGS__)

hipError_t launch_score(const ScoreParams& p, int slices, int mode, bool lds_bloom, int grid, hipStream_t stream) {
    if (slices < 1 || slices > 4) return hipErrorInvalidValue;
    switch (mode * 8 + slices) {
        LDGPU_FOR_PAIRS(LDGPU_SCORE_CASE, p, lds_bloom, grid, stream)
        default: return hipErrorInvalidValue;
    }
}

hipError_t score_prepare(int slices, int mode, bool lds_bloom, bool chunks, size_t lds_bytes, int* blocks_per_cu) {
    if (slices < 1 || slices > 4) return hipErrorInvalidValue;
    switch (mode * 8 + slices) {
        LDGPU_FOR_PAIRS(LDGPU_PREPARE_CASE, lds_bloom, chunks, lds_bytes, blocks_per_cu)
        default: return hipErrorInvalidValue;
    }
}

#endif  // LDGPU_SCORE_MODE

}  // namespace ldgpu
