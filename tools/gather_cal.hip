// gather_cal.hip -- known-byte kernels for calibrating the FETCH_SIZE PMC
// counter on gfx950 (profiles/README.md, DESIGN.md "Traffic").
//
// The score kernel's config-5 probes are random 4-B loads into a table far
// beyond the 256 MiB MALL.  The streaming-read correction of
// MI355X_MICROARCH.md (FETCH_SIZE counts half of 16-B/lane streaming reads)
// is calibrated for a different access pattern, so this program measures the
// counter on both patterns with exactly known demand:
//   stream_kernel  every lane reads 16 B, consecutive, over the whole buffer
//                  once: known bytes = buffer bytes.
//   gather_kernel  every lane does G random 4-B loads, one per 64-B line
//                  chosen by a hash: known lines = G x lanes (distinct lines
//                  expected: nlines (1 - exp(-loads / nlines)), printed).
// Each kernel keeps its loads live by a data-dependent vector store that
// never fires.  Run under rocprofv3 --pmc FETCH_SIZE (tools/gather_cal.sh);
// the printed JSON gives the known bytes and each kernel's time.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__global__ void stream_kernel(const uint4* a, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

__global__ void gather_kernel(const uint32_t* a, uint64_t nlines, int per_lane, uint32_t* sink) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int i = 0; i < per_lane; ++i) {
        const uint64_t line = mix(t * 0x100000001b3ull + (uint64_t)i) % nlines;
        acc += a[line * 16 + (t & 15)];  // one 4-B word of the 64-B line
    }
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 4ull << 30);
    const int per_lane = argc > 2 ? atoi(argv[2]) : 16;
    const int blocks = argc > 3 ? atoi(argv[3]) : 16384;
    const int threads = 256;
    uint32_t* a = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&sink, 4096));
    CHECK(hipMemset(a, 1, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint64_t n16 = bytes / 16, nlines = bytes / 64;
    float ms_stream = 0.f, ms_gather = 0.f;
    // one untimed launch of each, then the timed (profiled: last dispatch) one
    for (int rep = 0; rep < 2; ++rep) {
        CHECK(hipEventRecord(e0));
        stream_kernel<<<4096, 256>>>(reinterpret_cast<const uint4*>(a), n16, sink);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms_stream, e0, e1));
        CHECK(hipEventRecord(e0));
        gather_kernel<<<blocks, threads>>>(a, nlines, per_lane, sink);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms_gather, e0, e1));
    }
    CHECK(hipGetLastError());
    const double loads = (double)blocks * threads * per_lane;
    const double distinct = (double)nlines * (1.0 - std::exp(-loads / (double)nlines));
    printf("{\"buffer_bytes\": %llu, \"stream_known_bytes\": %llu, \"stream_ms\": %.4f, "
           "\"gather_loads\": %.0f, \"gather_distinct_lines_expected\": %.0f, \"line_bytes\": 64, "
           "\"gather_ms\": %.4f, \"gather_lines_per_s\": %.4e}\n",
           (unsigned long long)bytes, (unsigned long long)bytes, ms_stream, loads, distinct, ms_gather,
           loads / (ms_gather * 1e-3));
    CHECK(hipFree(a));
    CHECK(hipFree(sink));
    return 0;
}
