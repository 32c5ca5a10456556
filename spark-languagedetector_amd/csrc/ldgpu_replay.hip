// ldgpu_replay.hip -- the exact replay of class mode's ambiguous documents
// (gfx950).
//
// Class mode (score_kernel MODE 4, labels only) labels a document from its
// per-(class, language) hit counts when a rounding bound separates its top
// language from every other; a document it cannot separate (an exact tie or a
// near one) is labelled -1.  Those documents are gathered here into a packed
// sub-corpus, scored by the ordered mask-replay kernel (the reference's fp64
// fold, LanguageDetectorModel.scala:139-154: bit-identical scores, breeze's
// first maximum), and their labels scattered back.
#include <hipcub/hipcub.hpp>

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

__global__ void amb_lengths_kernel(const int64_t* idx, int64_t k, const int64_t* offsets, int64_t* len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) len[i] = offsets[idx[i] + 1] - offsets[idx[i]];
    if (i == k) len[i] = 0;
}

// one wave per document: its bytes to the sub-corpus
__global__ __launch_bounds__(256) void amb_gather_kernel(const int64_t* idx, int64_t k, const int64_t* offsets,
                                                         const uint8_t* bytes, const int64_t* sub_off, uint8_t* sub) {
    const int64_t d = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (d >= k) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = offsets[idx[d]], len = offsets[idx[d] + 1] - b, o = sub_off[d];
    for (int64_t j = lane; j < len; j += 64) sub[o + j] = bytes[b + j];
}

__global__ void amb_scatter_kernel(const int64_t* idx, int64_t k, const int32_t* sub_labels, int32_t* labels) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) labels[idx[i]] = sub_labels[i];
}

unsigned grid_for(int64_t n, int b) { return (unsigned)std::max<int64_t>(1, (n + b - 1) / b); }

}  // namespace

hipError_t launch_amb_compact(const int32_t* labels, int64_t n, int64_t* idx, unsigned long long* n_out,
                              hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>(2048, (n + kAmbThreads - 1) / kAmbThreads);
    hipLaunchKernelGGL(amb_compact_kernel, dim3(g), dim3(kAmbThreads), 0, stream, labels, n, idx, n_out);
    return hipGetLastError();
}

hipError_t amb_sub_corpus(const int64_t* idx, int64_t k, const int64_t* offsets, const uint8_t* bytes, int64_t* sub_off,
                          int64_t* len_tmp, void* scan_tmp, size_t* scan_bytes, uint8_t* sub, hipStream_t stream) {
    // exclusive scan of the k + 1 lengths (the last is 0): sub_off[0 .. k]
    if (!scan_tmp) return hipcub::DeviceScan::ExclusiveSum(nullptr, *scan_bytes, len_tmp, sub_off, (int)(k + 1), stream);
    hipLaunchKernelGGL(amb_lengths_kernel, dim3(grid_for(k + 1, 256)), dim3(256), 0, stream, idx, k, offsets, len_tmp);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, *scan_bytes, len_tmp, sub_off, (int)(k + 1), stream);
    if (e != hipSuccess || !sub) return e;
    hipLaunchKernelGGL(amb_gather_kernel, dim3(grid_for(64 * k, 256)), dim3(256), 0, stream, idx, k, offsets, bytes,
                       sub_off, sub);
    return hipGetLastError();
}

hipError_t launch_amb_scatter(const int64_t* idx, int64_t k, const int32_t* sub_labels, int32_t* labels,
                              hipStream_t stream) {
    if (k <= 0) return hipSuccess;
    hipLaunchKernelGGL(amb_scatter_kernel, dim3(grid_for(k, 256)), dim3(256), 0, stream, idx, k, sub_labels, labels);
    return hipGetLastError();
}

}  // namespace ldgpu
