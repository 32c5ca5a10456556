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
// Structure (one wave per document, persistent grid):
//   probe phase    lanes = 64 consecutive window positions of one gram length;
//                  each lane loads its window (3 dwords + v_alignbyte), packs
//                  the u64 key, hashes it and tests one bit of the filter,
//                  which is staged in LDS (<= 64 KiB).  Candidates are
//                  appended to a per-wave LDS queue with ballot + mbcnt, so
//                  the queue is in reference order (n outer, position inner).
//   verify phase   (when the queue is nearly full and at the end of the
//                  document) 64 queued keys at a time probe the global
//                  open-addressed table (L2-resident); hits carry their row.
//   accumulate     hits are replayed in queue order; lane l owns language l
//                  (slices of 64 for L > 64) and does s_l = s_l + row_l, so
//                  every s_l sees exactly the reference's sequence of fp64
//                  adds: scores are bit-identical, not just within tolerance.
//                  Mask-form rows (all nonzeros equal: every fit-produced row)
//                  add v or skip (x + 0.0 == x since s never is -0.0).
//   argmax         lane-local over slices, then a 6-step xor-shuffle
//                  reduction on (value, index) with the breeze rule.
#include "ldgpu_internal.h"

namespace ldgpu {

namespace {

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

// Verify + accumulate the queued candidates (in queue order).
template <int S, bool DENSE>
__device__ __forceinline__ void flush(const ScoreParams& p, const uint64_t* queue, int qn, double (&acc)[S],
                                      int lane) {
    __builtin_amdgcn_wave_barrier();
    for (int q0 = 0; q0 < qn; q0 += 64) {
        const int j = q0 + lane;
        uint32_t row = 0xffffffffu;
        if (j < qn) {
            const uint64_t key = queue[j];
            uint64_t s = mix64(key) >> p.slot_shift;
            for (;;) {
                const Slot e = p.slots[s];
                if (e.key == key) { row = e.row; break; }
                if (e.key == kEmpty) break;
                s = (s + 1) & p.slot_mask;
            }
        }
        const bool hit = row != 0xffffffffu;
        const bool bad = hit && (row & kBadRow);
        if (__ballot(bad)) {
            if (lane == 0) atomicOr(p.err, 1);
        }
        uint64_t hits = __ballot(hit && !bad);
        if (!hits) continue;
        if constexpr (!DENSE) {
            uint64_t mw[S];
            double v = 0.0;
            if (hit && !bad) {
#pragma unroll
                for (int s = 0; s < S; ++s) mw[s] = p.masks[(size_t)row * S + s];
                v = p.vals[row];
            } else {
#pragma unroll
                for (int s = 0; s < S; ++s) mw[s] = 0;
            }
            while (hits) {
                const int h = __builtin_ctzll(hits);
                hits &= hits - 1;
                const double vv = rdlaned(v, h);
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const uint64_t ms = rdlane64(mw[s], h);
                    acc[s] = acc[s] + (((ms >> lane) & 1ull) ? vv : 0.0);
                }
            }
        } else {
            while (hits) {
                const int h = __builtin_ctzll(hits);
                hits &= hits - 1;
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

constexpr int kSub = 4;  // 64-position sub-blocks per superblock (loads issued together)

// Window bytes of one position: lo = bytes[a..a+4), hi = bytes[a+4..a+8)
// (dword loads + v_alignbyte; clamped at the last readable dword).
__device__ __forceinline__ void load_window(const uint32_t* W, int64_t a, int64_t last, bool need_hi, uint32_t& lo,
                                            uint32_t& hi) {
    const int64_t i = a >> 2;
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = ld_dw(W, i, last);
    const uint32_t w1 = ld_dw(W, i + 1, last);
    lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
    hi = 0;
    if (need_hi) hi = __builtin_amdgcn_alignbyte(ld_dw(W, i + 2, last), w1, sh);
}

struct GramCtx {
    int64_t nwin;
    uint32_t lomask, himask, hitag, himix_c;
    bool big;  // klen > 4
};

__device__ __forceinline__ GramCtx gram_ctx(int64_t len, int n) {
    GramCtx g;
    g.nwin = n_windows(len, n);
    const int klen = len < n ? (int)len : n;
    g.lomask = klen >= 4 ? 0xffffffffu : ((1u << (8 * klen)) - 1u);
    g.himask = klen <= 4 ? 0u : ((1u << (8 * (klen - 4))) - 1u);
    g.hitag = (uint32_t)klen << 24;
    g.himix_c = hi_mix(g.hitag);
    g.big = klen > 4;
    return g;
}

// Filter-test 64 windows (one per lane) and append the candidates to the
// wave's queue in lane (= position) order; flush when the queue is nearly full.
template <int S, bool DENSE>
__device__ __forceinline__ void probe_block(const ScoreParams& p, const uint32_t* filt, uint64_t* queue, int& qn,
                                            double (&acc)[S], int lane, const GramCtx& g, uint32_t xlo, uint32_t xhi,
                                            bool valid) {
    const uint32_t lo = xlo & g.lomask;
    uint32_t hi = g.hitag;
    uint32_t himix = g.himix_c;
    if (g.big) {
        hi |= xhi & g.himask;
        himix = hi_mix(hi);
    }
    const uint32_t bit = filter_hash(lo, himix) >> p.filter_shift;
    const bool cand = valid && ((filt[bit >> 5] >> (bit & 31)) & 1u);
    const uint64_t m = __ballot(cand);
    if (m) {
        const int off = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (cand) queue[qn + off] = ((uint64_t)hi << 32) | lo;
        qn += __popcll(m);
        if (qn > kQueueCap - 64) {
            flush<S, DENSE>(p, queue, qn, acc, lane);
            qn = 0;
        }
    }
}

template <int S, bool DENSE, bool FLDS>
__global__ __launch_bounds__(kScoreWaves * 64) void score_kernel(const ScoreParams p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t fwords = FLDS ? p.filter_words : 0u;
    uint64_t* queue = reinterpret_cast<uint64_t*>(lds + ((fwords + 3u) & ~3u)) + wave * kQueueCap;
    const uint32_t* filt = p.filter;
    if constexpr (FLDS) {
        const uint4* src = reinterpret_cast<const uint4*>(p.filter);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = tid; i < (fwords >> 2); i += blockDim.x) dst[i] = src[i];
        __syncthreads();
        filt = lds;
    }
    const uint32_t* W = reinterpret_cast<const uint32_t*>(p.bytes);
    const bool need_hi = p.max_gram > 4;
    const int64_t stride = (int64_t)gridDim.x * kScoreWaves;
    for (int64_t doc = (int64_t)blockIdx.x * kScoreWaves + wave; doc < p.n_docs; doc += stride) {
        const int64_t b = p.offsets[doc];
        const int64_t len = p.offsets[doc + 1] - b;
        double acc[S];
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s] = 0.0;
        int qn = 0;
        if (len <= 64 * kSub) {
            // one superblock: every gram length reuses the same window bytes
            uint32_t xlo[kSub], xhi[kSub];
#pragma unroll
            for (int k = 0; k < kSub; ++k) load_window(W, b + 64 * k + lane, p.last_dword, need_hi, xlo[k], xhi[k]);
            for (int gi = 0; gi < p.nG; ++gi) {
                const GramCtx g = gram_ctx(len, p.G[gi]);
#pragma unroll
                for (int k = 0; k < kSub; ++k) {
                    if (64 * k < g.nwin)
                        probe_block<S, DENSE>(p, filt, queue, qn, acc, lane, g, xlo[k], xhi[k],
                                              64 * k + lane < g.nwin);
                }
            }
        } else {
            // long documents: n outer (reference order), superblocks inner
            for (int gi = 0; gi < p.nG; ++gi) {
                const GramCtx g = gram_ctx(len, p.G[gi]);
                for (int64_t p0 = 0; p0 < g.nwin; p0 += 64 * kSub) {
                    uint32_t xlo[kSub], xhi[kSub];
#pragma unroll
                    for (int k = 0; k < kSub; ++k)
                        load_window(W, b + p0 + 64 * k + lane, p.last_dword, g.big, xlo[k], xhi[k]);
#pragma unroll
                    for (int k = 0; k < kSub; ++k) {
                        if (p0 + 64 * k < g.nwin)
                            probe_block<S, DENSE>(p, filt, queue, qn, acc, lane, g, xlo[k], xhi[k],
                                                  p0 + 64 * k + lane < g.nwin);
                    }
                }
            }
        }
        if (qn) flush<S, DENSE>(p, queue, qn, acc, lane);

        // argmax (breeze: first element, then strict '>' updates)
        double bv = acc[0];
        int bi = lane;
        bool bval = lane < p.L && !__builtin_isnan(bv);
#pragma unroll
        for (int s = 1; s < S; ++s) {
            const int l = s * 64 + lane;
            const double v = acc[s];
            if (l < p.L && !__builtin_isnan(v) && (!bval || v > bv)) {
                bv = v;
                bi = l;
                bval = true;
            }
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double ov = __shfl_xor(bv, d);
            const int oi = __shfl_xor(bi, d);
            const bool oval = __shfl_xor((int)bval, d) != 0;
            const bool better = oval && (!bval || ov > bv || (ov == bv && oi < bi));
            if (better) {
                bv = ov;
                bi = oi;
                bval = true;
            }
        }
        const double s0 = rdlaned(acc[0], 0);
        const int label = (!bval || __builtin_isnan(s0)) ? 0 : bi;
        if (lane == 0) p.labels[doc] = label;
        if (p.scores) {
            double* out = p.scores + doc * (int64_t)p.L;
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int l = s * 64 + lane;
                if (l < p.L) out[l] = acc[s];
            }
        }
    }
}

template <int S, bool DENSE, bool FLDS>
hipError_t launch_t(const ScoreParams& p, int grid, hipStream_t stream) {
    const size_t lds = (FLDS ? ((p.filter_words + 3u) & ~3u) * 4u : 0u) +
                       (size_t)kScoreWaves * kQueueCap * sizeof(uint64_t);
    hipLaunchKernelGGL((score_kernel<S, DENSE, FLDS>), dim3(grid), dim3(kScoreWaves * 64), lds, stream, p);
    return hipGetLastError();
}

template <int S, bool DENSE, bool FLDS>
hipError_t prepare_t(size_t lds) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&score_kernel<S, DENSE, FLDS>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

template <bool DENSE, bool FLDS>
hipError_t launch_s(const ScoreParams& p, int slices, int grid, hipStream_t stream) {
    switch (slices) {
        case 1: return launch_t<1, DENSE, FLDS>(p, grid, stream);
        case 2: return launch_t<2, DENSE, FLDS>(p, grid, stream);
        case 3: return launch_t<3, DENSE, FLDS>(p, grid, stream);
        case 4: return launch_t<4, DENSE, FLDS>(p, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

template <bool DENSE, bool FLDS>
hipError_t prepare_s(int slices, size_t lds) {
    switch (slices) {
        case 1: return prepare_t<1, DENSE, FLDS>(lds);
        case 2: return prepare_t<2, DENSE, FLDS>(lds);
        case 3: return prepare_t<3, DENSE, FLDS>(lds);
        case 4: return prepare_t<4, DENSE, FLDS>(lds);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_score(const ScoreParams& p, int slices, bool dense, bool lds_filter, int grid,
                        hipStream_t stream) {
    if (dense) {
        return lds_filter ? launch_s<true, true>(p, slices, grid, stream)
                          : launch_s<true, false>(p, slices, grid, stream);
    }
    return lds_filter ? launch_s<false, true>(p, slices, grid, stream)
                      : launch_s<false, false>(p, slices, grid, stream);
}

hipError_t score_prepare(int slices, bool dense, bool lds_filter, size_t lds_bytes) {
    if (dense) {
        return lds_filter ? prepare_s<true, true>(slices, lds_bytes) : prepare_s<true, false>(slices, lds_bytes);
    }
    return lds_filter ? prepare_s<false, true>(slices, lds_bytes) : prepare_s<false, false>(slices, lds_bytes);
}

}  // namespace ldgpu
