// Microbenchmark (round 6): random 64-bit atomic adds into a big table, fully
// random vs partitioned into regions (the inserts of one launch window confined
// to 1/R of the table) -- does locality (TLB / L2) bound FIT v5's inserts?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}

// entry i -> slot: random over the table, or (regions > 1) region r = i / (n / regions)
__global__ void add_kernel(unsigned long long* t, uint64_t cap_log2, uint64_t n, uint64_t regions, int chain) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + 1);
        uint64_t s;
        if (regions <= 1) {
            s = h >> (64 - cap_log2);
        } else {
            const uint64_t per = n / regions, r = i / per, rl = 64 - __builtin_ctzll(regions);
            (void)rl;
            const uint64_t region_slots = (1ull << cap_log2) / regions;
            s = (r % regions) * region_slots + (h % region_slots);
        }
        if (chain) {
            // a dependent chain like find_or_insert: read, then CAS, then add
            unsigned long long v = __hip_atomic_load(&t[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v == 0) atomicCAS(&t[s], 0ull, 1ull);
            atomicAdd(&t[(s ^ 1)], 1ull);
        } else {
            atomicAdd(&t[s], 1ull);
        }
    }
}

int main() {
    const uint64_t cap_log2 = 32;  // 2^32 x 8 B = 32 GiB
    unsigned long long* t = nullptr;
    if (hipMalloc(&t, sizeof(unsigned long long) << cap_log2) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(t, 0, sizeof(unsigned long long) << cap_log2);
    const uint64_t n = 1ull << 29;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int chain = 0; chain < 2; ++chain)
        for (uint64_t regions : {1ull, 16ull, 256ull, 4096ull, 65536ull}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                hipLaunchKernelGGL(add_kernel, dim3(256 * 8), dim3(256), 0, 0, t, cap_log2, n, regions, chain);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (rep) printf("chain %d regions %6llu (%8.1f MiB each): %.1f ms for %llu entries = %.2f G/s\n", chain,
                                (unsigned long long)regions, (double)(8ull << cap_log2) / regions / 1048576.0, ms,
                                (unsigned long long)n, n / (ms * 1e-3) / 1e9);
            }
        }
    hipFree(t);
    return 0;
}
