// ldgpu_pre.hip -- the caller-side preprocessors on the device (gfx950).
//
// Reference (org.apache.spark.ml.feature.languagedetection.preprocessing):
//   LowerCasePreprocessor.scala:44-76   text.toLowerCase(Locale.forLanguageTag(lang))
//   SpecialCharPreprocessor.scala:40-70 replaceAll(<symbol list>, "") then
//                                       replaceAll("  *", ""): the documented
//                                       intent (the reference's pattern never
//                                       compiles: languagedetection/preprocessing.py)
//
// Documents are Java strings: UTF-16 code units (u16) + offsets in units.  One
// wave per document, 64 units per step:
//   lower  unit u -> map[u], the host language's 1:1 lower-case mapping
//          (Character.toLowerCase / str.lower of one character), with the
//          locale rules of java.lang.ConditionalSpecialCasing that stay 1:1
//          (tr / az: I -> U+0131, U+0130 -> i).  A unit whose String.toLowerCase
//          is NOT 1:1 or depends on context -- U+0130 outside tr / az, capital
//          sigma (Final_Sigma), tr / az "I" + U+0307, lt I / J / U+012E before a
//          mark above and U+00CC / U+00CD / U+0128, the high surrogates of cased
//          supplementary planes (the host's `special` bitmap and the rules
//          below) -- sends its document back to the host (host[d] = 1, empty
//          output): those are rare outside Greek capitals and Turkish /
//          Lithuanian text.
//   clean  units of the symbol list and spaces dropped (a ballot + mbcnt
//          compaction).
// Output: units, or the SCORE encoding itself (the low byte of each unit,
// LanguageDetectorModel.scala:226's getBytes of the char's low byte), packed at
// offsets from a device scan of the per-document lengths -- ready for
// ldgpu_score_device without a host round trip.
#include <hipcub/hipcub.hpp>

#include "../../include/ldgpu.h"
#include "ldgpu_internal.h"

namespace ldgpu {
namespace {

constexpr int kPreWaves = 4;

// the symbols of SpecialCharPreprocessor.scala:55 and the space ("  *", :56)
__device__ __forceinline__ bool clean_drop(uint32_t u) {
    if (u >= 128u) return false;
    // / _ [ ] * ( ) % ^ & @ $ # : | { } < > ~ ` " \ and ' '
    const uint64_t lo = (1ull << '/') | (1ull << '*') | (1ull << '(') | (1ull << ')') | (1ull << '%') |
                        (1ull << '&') | (1ull << '$') | (1ull << '#') | (1ull << ':') | (1ull << '<') |
                        (1ull << '>') | (1ull << '"') | (1ull << ' ');
    const uint64_t hi = (1ull << ('_' - 64)) | (1ull << ('[' - 64)) | (1ull << (']' - 64)) | (1ull << ('^' - 64)) |
                        (1ull << ('@' - 64)) | (1ull << ('|' - 64)) | (1ull << ('{' - 64)) | (1ull << ('}' - 64)) |
                        (1ull << ('~' - 64)) | (1ull << ('`' - 64)) | (1ull << ('\\' - 64));
    return ((u < 64u ? lo >> u : hi >> (u - 64u)) & 1ull) != 0ull;
}

// combining marks of canonical class 230 (Above) that Java's Lithuanian rule
// tests for (ConditionalSpecialCasing "More_Above"; preprocessing.py
// _COMBINING_ABOVE)
__device__ __forceinline__ bool above_mark(uint32_t u) {
    return (u >= 0x300u && u <= 0x314u) || (u >= 0x33Du && u <= 0x344u) || u == 0x346u ||
           (u >= 0x34Au && u <= 0x34Cu) || (u >= 0x350u && u <= 0x352u) || u == 0x357u || u == 0x35Bu ||
           (u >= 0x363u && u <= 0x36Fu);
}

// unit i of the document (0 past its end)
__device__ __forceinline__ uint32_t unit_at(const uint16_t* d, int64_t len, int64_t i) {
    return i < len ? (uint32_t)d[i] : 0u;
}

// one unit: its lower-case unit (*out), whether it is kept (clean) and
// whether its document must go back to the host
__device__ __forceinline__ void pre_unit(const PreParams& p, const uint32_t* special, uint32_t u, uint32_t next,
                                         uint32_t loc, uint32_t& out, bool& keep, bool& host) {
    out = u;
    host = false;
    if (p.flags & LDGPU_PRE_LOWER) {
        if (loc == LDGPU_LOCALE_TR_AZ && (u == 'I' || u == 0x130u)) {
            host = u == 'I' && next == 0x307u;  // "I" + dot above -> "i": two units to one
            out = u == 'I' ? 0x131u : 'i';
        } else {
            host = ((special[u >> 5] >> (u & 31u)) & 1u) != 0u;
            if (loc == LDGPU_LOCALE_LT)
                host = host || ((u == 'I' || u == 'J' || u == 0x12Eu) && above_mark(next)) || u == 0xCCu ||
                       u == 0xCDu || u == 0x128u;
            out = p.map[u];
        }
    }
    keep = !((p.flags & LDGPU_PRE_CLEAN) && clean_drop(out));
}

// pass 1: kept units per document, and the documents that go to the host
__global__ __launch_bounds__(kPreWaves * 64) void pre_len_kernel(const PreParams p, int64_t* len_out) {
    __shared__ uint32_t special[65536 / 32];
    for (int i = threadIdx.x; i < 65536 / 32; i += blockDim.x) special[i] = p.special[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * kPreWaves;
    for (int64_t d = (int64_t)blockIdx.x * kPreWaves + (threadIdx.x >> 6); d < p.n_docs; d += stride) {
        const int64_t b = p.offsets[d], len = p.offsets[d + 1] - b;
        const uint16_t* s = p.units + b;
        const uint32_t loc = p.locale ? p.locale[d] : 0u;
        int64_t kept = 0;
        bool host = false;
        for (int64_t i0 = 0; i0 < len && !host; i0 += 64) {
            const int64_t i = i0 + lane;
            bool k = false, h = false;
            if (i < len) {
                uint32_t o;
                pre_unit(p, special, s[i], unit_at(s, len, i + 1), loc, o, k, h);
            }
            kept += __popcll(__ballot(k));
            host = __ballot(h) != 0ull;
        }
        if (lane == 0) {
            len_out[d] = host ? 0 : kept;
            p.host[d] = host ? 1 : 0;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) len_out[p.n_docs] = 0;
}

// pass 3: the kept (lower-cased) units of every document not sent to the host,
// at out_off[d]
__global__ __launch_bounds__(kPreWaves * 64) void pre_write_kernel(const PreParams p, const int64_t* out_off) {
    __shared__ uint32_t special[65536 / 32];
    for (int i = threadIdx.x; i < 65536 / 32; i += blockDim.x) special[i] = p.special[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * kPreWaves;
    for (int64_t d = (int64_t)blockIdx.x * kPreWaves + (threadIdx.x >> 6); d < p.n_docs; d += stride) {
        if (p.host[d]) continue;
        const int64_t b = p.offsets[d], len = p.offsets[d + 1] - b;
        const uint16_t* s = p.units + b;
        const uint32_t loc = p.locale ? p.locale[d] : 0u;
        int64_t o = out_off[d];
        for (int64_t i0 = 0; i0 < len; i0 += 64) {
            const int64_t i = i0 + lane;
            bool k = false, h = false;
            uint32_t u = 0;
            if (i < len) pre_unit(p, special, s[i], unit_at(s, len, i + 1), loc, u, k, h);
            const uint64_t m = __ballot(k);
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (k) {
                if (p.flags & LDGPU_PRE_LOW_BYTES)
                    static_cast<uint8_t*>(p.out)[o + r] = (uint8_t)u;
                else
                    static_cast<uint16_t*>(p.out)[o + r] = (uint16_t)u;
            }
            o += __popcll(m);
        }
    }
}

int pre_grid(int64_t n, int cus) {
    const int64_t want = (n + kPreWaves - 1) / kPreWaves;
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)cus * 8));
}

}  // namespace

hipError_t launch_preprocess(const PreParams& p, int64_t* len_tmp, int64_t* out_off, void* scan_tmp, size_t* scan_bytes,
                             int cus, hipStream_t stream) {
    if (!scan_tmp) return hipcub::DeviceScan::ExclusiveSum(nullptr, *scan_bytes, len_tmp, out_off, (int)(p.n_docs + 1), stream);
    if (p.n_docs <= 0) return hipMemsetAsync(out_off, 0, sizeof(int64_t), stream);
    hipLaunchKernelGGL(pre_len_kernel, dim3(pre_grid(p.n_docs, cus)), dim3(kPreWaves * 64), 0, stream, p, len_tmp);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, *scan_bytes, len_tmp, out_off, (int)(p.n_docs + 1), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pre_write_kernel, dim3(pre_grid(p.n_docs, cus)), dim3(kPreWaves * 64), 0, stream, p, out_off);
    return hipGetLastError();
}

}  // namespace ldgpu
