// ldgpu_replay.hip -- the list of class mode's ambiguous documents (gfx950).
//
// Class mode (score_kernel MODE 4, labels only) labels a document from its
// per-(class, language) hit counts when a rounding bound separates its top
// language from every other; a document it cannot separate (an exact tie or a
// near one) is labelled -1.  Those documents are listed here, and an indirect
// launch of the ordered mask-replay kernel (the reference's fp64 fold,
// LanguageDetectorModel.scala:139-154: bit-identical scores, breeze's first
// maximum) scores each of them in place and stores its label -- reading the
// list's length on the device, so the call stays asynchronous.
#include "ldgpu_internal.h"

namespace ldgpu {
namespace {

constexpr int kAmbThreads = 1024;

// the documents labelled -1, in index order within each block-chunk (the
// order of the list does not matter: each label goes back to its index)
__global__ __launch_bounds__(kAmbThreads) void amb_compact_kernel(const int32_t* labels, int64_t n, int64_t* idx,
                                                                  unsigned long long* n_out) {
    __shared__ unsigned int wcnt[kAmbThreads / 64];
    __shared__ unsigned long long bbase;
    for (int64_t c0 = (int64_t)blockIdx.x * kAmbThreads; c0 < n; c0 += (int64_t)gridDim.x * kAmbThreads) {
        const int64_t i = c0 + threadIdx.x;
        const bool amb = i < n && labels[i] < 0;
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const uint64_t m = __ballot(amb);
        if (lane == 0) wcnt[wave] = (unsigned int)__popcll(m);
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned int acc = 0;
            for (int w = 0; w < kAmbThreads / 64; ++w) {
                const unsigned int c = wcnt[w];
                wcnt[w] = acc;
                acc += c;
            }
            bbase = acc ? atomicAdd(n_out, (unsigned long long)acc) : 0ull;
        }
        __syncthreads();
        if (amb)
            idx[bbase + wcnt[wave] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = i;
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_amb_compact(const int32_t* labels, int64_t n, int64_t* idx, unsigned long long* n_out,
                              hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>(2048, (n + kAmbThreads - 1) / kAmbThreads);
    hipLaunchKernelGGL(amb_compact_kernel, dim3(g), dim3(kAmbThreads), 0, stream, labels, n, idx, n_out);
    return hipGetLastError();
}

}  // namespace ldgpu
