// ldgpu_api.hip -- host runtime of libldgpu.so: the C ABI declared in
// include/ldgpu.h (contexts, device tables, H2D/D2H staging, count-table
// growth, probability / top-K table build).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/ldgpu.h"
#include "ldgpu_fit.h"

using namespace ldgpu;

// LDGPU_* environment switches: read only by the diagnostics build
// (ldgpu_internal.h); the product library sees none of them.
static const char* diag_env(const char* name) { return LDGPU_DIAG ? getenv(name) : nullptr; }

// Diagnostics build: LDGPU_FIT_TRACE prints the FIT runtime's host-side phase
// times to stderr (a scope's time, its stream drained at the end).
namespace {
double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// consecutive phases of one function: mark("x") prints the time since the last mark
struct PhaseMarks {
    hipStream_t st;
    bool on;
    double t;
    explicit PhaseMarks(hipStream_t s) : st(s), on(diag_env("LDGPU_FIT_TRACE") != nullptr), t(on ? now_ms() : 0.0) {}
    void operator()(const char* what) {
        if (!on) return;
        (void)hipStreamSynchronize(st);
        const double u = now_ms();
        fprintf(stderr, "fit %s: %.3f ms\n", what, u - t);
        t = u;
    }
};
struct PhaseTrace {
    const char* what;
    unsigned long long a, b;
    hipStream_t st;
    double t0;
    bool on;
    PhaseTrace(const char* w, unsigned long long a_, unsigned long long b_, hipStream_t s)
        : what(w), a(a_), b(b_), st(s), t0(0.0), on(diag_env("LDGPU_FIT_TRACE") != nullptr) {
        if (on) t0 = now_ms();
    }
    ~PhaseTrace() {
        if (!on) return;
        (void)hipStreamSynchronize(st);
        fprintf(stderr, "fit %s (%llu, %llu): %.3f ms\n", what, a, b, now_ms() - t0);
    }
};
}  // namespace

// ------------------------------------------------------------------- errors
namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int ok() {
    g_err.clear();
    return LDGPU_OK;
}

// Diagnostics build: LDGPU_FAIL_AT=<point> makes the named point of the
// runtime fail (tests of the ranks' status agreement around collectives)
int injected(const char* point) {
    const char* f = diag_env("LDGPU_FAIL_AT");
    if (f && strcmp(f, point) == 0) return fail(LDGPU_EDEVICE, "injected failure at %s", point);
    return 0;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return fail(LDGPU_EDEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

int log2u(uint64_t p) {
    int l = 0;
    while ((1ull << l) < p) ++l;
    return l;
}

// device buffer that only grows
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 1 << 20);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// pinned (page-locked) host buffer that only grows: the H2D / D2H copies of
// the host-buffer API run from it at full PCIe rate, asynchronously
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(n, 1 << 20);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// true when host pointer q lies in page-locked memory (ldgpu_host_alloc,
// hipHostMalloc, hipHostRegister): then it is copied from / to directly
bool is_pinned(const void* q) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, q) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy split over up to 8 threads (pageable -> pinned staging is the host
// path's bound when the caller's buffers are pageable)
void par_memcpy(void* dst, const void* src, size_t n) {
    const size_t kMin = 4u << 20;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned t = (unsigned)std::min<size_t>(std::min(8u, hw), std::max<size_t>(1, n / kMin));
    if (t <= 1) {
        memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t part = (n + t - 1) / t;
    for (unsigned i = 1; i < t; ++i) {
        const size_t a = std::min(n, part * i), b = std::min(n, part * (i + 1));
        if (a < b) th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
    }
    memcpy(dst, src, std::min(n, part));
    for (auto& x : th) x.join();
}

// fn(i0, i1) over [0, n) split across up to 8 threads (host loops over a
// fit table's ~10M rows)
template <typename F>
void par_for(int64_t n, F fn) {
    const int64_t kMin = 1 << 16;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int64_t t = std::min<int64_t>(std::min<unsigned>(8u, hw), std::max<int64_t>(1, n / kMin));
    if (t <= 1) {
        fn((int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    const int64_t part = (n + t - 1) / t;
    for (int64_t i = 1; i < t; ++i) {
        const int64_t a = std::min(n, part * i), b = std::min(n, part * (i + 1));
        if (a < b) th.emplace_back([=] { fn(a, b); });
    }
    fn((int64_t)0, std::min(n, part));
    for (auto& x : th) x.join();
}

int check_grams(const int32_t* G, int32_t nG, int max_len = kMaxGram) {
    if (nG < 0 || nG > LDGPU_MAX_GRAM_LENGTHS)
        return fail(LDGPU_EINVAL, "number of gram lengths %d outside [0, %d]", nG, LDGPU_MAX_GRAM_LENGTHS);
    if (nG > 0 && !G) return fail(LDGPU_EINVAL, "gram_lengths is NULL");
    for (int i = 0; i < nG; ++i) {
        if (G[i] <= 0)
            return fail(LDGPU_EINVAL, "requirement failed: size=%d and step=1, but both must be positive", G[i]);
        if (G[i] > max_len)
            return fail(LDGPU_EUNSUPPORTED, "gram length %d exceeds the device path's limit of %d bytes", G[i],
                        max_len);
    }
    return LDGPU_OK;
}

int check_offsets(const int64_t* off, int64_t n_docs) {
    if (n_docs < 0) return fail(LDGPU_EINVAL, "n_docs < 0");
    if (!off) return fail(LDGPU_EINVAL, "offsets is NULL");
    if (off[0] < 0) return fail(LDGPU_EINVAL, "offsets[0] < 0");
    for (int64_t d = 0; d < n_docs; ++d)
        if (off[d + 1] < off[d]) return fail(LDGPU_EINVAL, "offsets decrease at document %lld", (long long)d);
    return LDGPU_OK;
}

}  // namespace

// ------------------------------------------------------------------ context
// one stage of the host-buffer scoring pipeline (ldgpu_score): pinned
// staging + device buffers of one chunk, on its own stream
struct ScoreStage {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    DevBuf bytes, offsets, labels, scores;
    HostBuf h_bytes, h_offsets, h_labels, h_scores;
    int64_t d0 = 0, nd = 0;
    bool busy = false;
};

// One ldgpu_score call's pipeline: two stages plus the call's own error word
// (a wrong-length row hit by THIS call's documents).  Contexts keep a pool:
// concurrent callers (Spark task threads of one executor, Spark.scala:11
// local[4]) each take a pipeline and run on their own streams.
struct ScorePipe {
    ScoreStage stage[2];
    int32_t* d_err = nullptr;
};

struct ldgpu_ctx {
    int device = 0;
    int cus = 256;
    hipStream_t stream = nullptr;
    std::mutex mu;                     // FIT calls and the ctx stream
    DevBuf bytes, offsets, labels, scores, langs;
    std::mutex pool_mu;                // guards `pipes` / `free_pipes` only
    std::vector<ScorePipe*> pipes, free_pipes;
    // FIT v2 batch scratch (records, buckets, reduce output), shared by the
    // context's count tables under `mu` and kept between fits: multi-GB
    // allocations per fit would cost more than the counting itself
    DevBuf f_rec, f_rec2, f_bstart, f_bhdr, f_nblk, f_cnt3, f_wg, f_p2, f_boff, f_okl, f_ocnt, f_on;
    DevBuf f_stmp;                     // FIT v5: the radix sort's scratch
    HostBuf h_fwg;                     // pinned staging of a batch's plan (one async copy to f_wg)
    HostBuf h_fon;                     // pinned landing of a batch's nout / boff (an async copy back)
    // pinned landing of a single-rank device fit table (keys, masks, k per
    // row: one DMA); it stays the table of h_tbl_owner until another count
    // table's build needs it (tbl_materialize moves the owner's into its own
    // vectors first)
    HostBuf h_tbl;
    struct ldgpu_counts* h_tbl_owner = nullptr;
    // device blocks of destroyed / grown count tables and overflow lists,
    // reused by exact size: a Spark executor fits partition after partition,
    // and freeing and re-mapping ~10 GB per fit stalls the allocator
    std::mutex cache_mu;
    std::vector<std::pair<size_t, void*>> cache;
    size_t cache_bytes = 0;
    size_t cache_max = 96ull << 30;  // half the device's memory (ldgpu_ctx_create)
    // FIT: T1 keys per corpus byte of the last count call on this context --
    // sizes the next call's T1 (of any count table: an executor fits
    // partition after partition of like text), so it is not grown by
    // doubling from a small start, rehashing ~its final size each time
    double t1_keys_per_byte = 0.0;
    int64_t t1_keys = 0;  // (and its keys: a hint is capped at twice them)
};

namespace {
// The block cache keeps freed device blocks for the next call of the same
// shape, up to half the device's memory: a config-5-sized fit frees ~90 GB per
// call (T, the top-K scratch), and a 96 GB cap evicted blocks the next fit
// then re-allocated -- 3.5 s of hipMalloc in one table phase of eight -- and
// up to 256 blocks (at 64, the big blocks a larger byte cap keeps pushed out
// the small top-K scratch blocks of config 3's fits instead).  An allocation
// that fails frees the whole cache and retries (cache_alloc).
constexpr size_t kCacheMaxBlocks = 256;

hipError_t cache_alloc(ldgpu_ctx* c, void** p, size_t bytes) {
    {
        std::lock_guard<std::mutex> g(c->cache_mu);
        for (size_t i = 0; i < c->cache.size(); ++i) {
            if (c->cache[i].first == bytes) {
                *p = c->cache[i].second;
                c->cache_bytes -= bytes;
                c->cache.erase(c->cache.begin() + (std::ptrdiff_t)i);
                return hipSuccess;
            }
        }
    }
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory) {  // give the cache back to the device and retry
        (void)hipGetLastError();
        std::lock_guard<std::mutex> g(c->cache_mu);
        for (auto& b : c->cache) (void)hipFree(b.second);
        c->cache.clear();
        c->cache_bytes = 0;
        e = hipMalloc(p, bytes);
    }
    return e;
}

void cache_free(ldgpu_ctx* c, void* p, size_t bytes) {
    if (!p) return;
    std::lock_guard<std::mutex> g(c->cache_mu);
    c->cache.emplace_back(bytes, p);
    c->cache_bytes += bytes;
    while (!c->cache.empty() && (c->cache_bytes > c->cache_max || c->cache.size() > kCacheMaxBlocks)) {
        (void)hipFree(c->cache.front().second);
        c->cache_bytes -= c->cache.front().first;
        c->cache.erase(c->cache.begin());
    }
}
}  // namespace

namespace {
void pipe_destroy(ScorePipe* pp) {
    for (auto& st : pp->stage) {
        if (st.stream) (void)hipStreamSynchronize(st.stream);
        for (DevBuf* b : {&st.bytes, &st.offsets, &st.labels, &st.scores}) b->release();
        for (HostBuf* b : {&st.h_bytes, &st.h_offsets, &st.h_labels, &st.h_scores}) b->release();
        if (st.done) (void)hipEventDestroy(st.done);
        if (st.stream) (void)hipStreamDestroy(st.stream);
    }
    if (pp->d_err) (void)hipFree(pp->d_err);
    delete pp;
}

// a free pipeline of the context, created on demand (nullptr + error on failure)
ScorePipe* pipe_acquire(ldgpu_ctx* c) {
    {
        std::lock_guard<std::mutex> g(c->pool_mu);
        if (!c->free_pipes.empty()) {
            ScorePipe* pp = c->free_pipes.back();
            c->free_pipes.pop_back();
            return pp;
        }
    }
    auto* pp = new ScorePipe();
    hipError_t e = hipSuccess;
    for (auto& st : pp->stage) {
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&st.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&st.done, hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipMalloc((void**)&pp->d_err, sizeof(int32_t));
    if (e == hipSuccess) e = hipMemset(pp->d_err, 0, sizeof(int32_t));
    if (e != hipSuccess) {
        pipe_destroy(pp);
        fail(LDGPU_EDEVICE, "score pipeline: %s", hipGetErrorString(e));
        return nullptr;
    }
    std::lock_guard<std::mutex> g(c->pool_mu);
    c->pipes.push_back(pp);
    return pp;
}

void pipe_release(ldgpu_ctx* c, ScorePipe* pp) {
    std::lock_guard<std::mutex> g(c->pool_mu);
    c->free_pipes.push_back(pp);
}
}  // namespace

extern "C" const char* ldgpu_version(void) { return "ldgpu 0.1.0 (gfx950)"; }
#ifndef LDGPU_SRC_HASH
#define LDGPU_SRC_HASH "unknown"
#endif
extern "C" const char* ldgpu_build_id(void) { return LDGPU_SRC_HASH; }
extern "C" const char* ldgpu_last_error(void) { return g_err.c_str(); }

extern "C" int ldgpu_device_count(int32_t* out) {
    if (!out) return fail(LDGPU_EINVAL, "out is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return ok();
}

extern "C" int ldgpu_ctx_create(int32_t device, ldgpu_ctx** out) {
    if (!out) return fail(LDGPU_EINVAL, "out is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(LDGPU_ENODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(LDGPU_EINVAL, "device %d outside [0, %d)", device, n);
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    auto* c = new ldgpu_ctx();
    c->device = device;
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->cache_max = std::max<size_t>(c->cache_max, prop.totalGlobalMem / 2);
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        (void)ldgpu_ctx_destroy(c);
        return fail(LDGPU_EDEVICE, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    *out = c;
    return ok();
}

extern "C" int ldgpu_ctx_destroy(ldgpu_ctx* c) {
    if (!c) return ok();
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->bytes.release();
    c->offsets.release();
    c->labels.release();
    c->scores.release();
    c->langs.release();
    for (DevBuf* b : {&c->f_rec, &c->f_rec2, &c->f_bstart, &c->f_bhdr, &c->f_nblk, &c->f_cnt3, &c->f_wg, &c->f_p2,
                      &c->f_boff, &c->f_okl, &c->f_ocnt, &c->f_on, &c->f_stmp})
        b->release();
    c->h_fwg.release();
    c->h_fon.release();
    c->h_tbl.release();
    for (ScorePipe* pp : c->pipes) pipe_destroy(pp);
    for (auto& b : c->cache) (void)hipFree(b.second);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return ok();
}

extern "C" int ldgpu_ctx_synchronize(ldgpu_ctx* c) {
    if (!c) return fail(LDGPU_EINVAL, "ctx is NULL");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ok();
}

extern "C" void* ldgpu_ctx_stream(ldgpu_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int ldgpu_host_alloc(ldgpu_ctx* c, int64_t n_bytes, void** out) {
    if (!c || !out) return fail(LDGPU_EINVAL, "ctx/out is NULL");
    if (n_bytes < 0) return fail(LDGPU_EINVAL, "n_bytes < 0");
    HIP_TRY(hipSetDevice(c->device));
    *out = nullptr;
    hipError_t e = hipHostMalloc(out, (size_t)std::max<int64_t>(n_bytes, 1), hipHostMallocDefault);
    if (e != hipSuccess) return fail(LDGPU_ENOMEM, "hipHostMalloc(%lld): %s", (long long)n_bytes, hipGetErrorString(e));
    return ok();
}

extern "C" int ldgpu_host_free(ldgpu_ctx* c, void* p) {
    if (!c) return fail(LDGPU_EINVAL, "ctx is NULL");
    if (p) HIP_TRY(hipHostFree(p));
    return ok();
}

// --------------------------------------------------------------- preprocess
// The caller-side preprocessors (ldgpu_pre.hip; include/ldgpu.h PREPROCESS):
// the host language's 1:1 lower-case mapping of UTF-16 units and the units
// whose documents stay on the host, resident on the context's device.
struct ldgpu_casemap {
    ldgpu_ctx* ctx = nullptr;
    uint16_t* d_map = nullptr;
    uint32_t* d_special = nullptr;
};

extern "C" int ldgpu_casemap_create(ldgpu_ctx* ctx, const uint16_t* lower, const uint8_t* special, ldgpu_casemap** out) {
    if (!ctx || !lower || !special || !out) return fail(LDGPU_EINVAL, "ctx/lower/special/out is NULL");
    HIP_TRY(hipSetDevice(ctx->device));
    auto* m = new ldgpu_casemap();
    m->ctx = ctx;
    hipError_t e = hipMalloc((void**)&m->d_map, 65536 * sizeof(uint16_t));
    if (e == hipSuccess) e = hipMalloc((void**)&m->d_special, 8192);
    if (e == hipSuccess) e = hipMemcpy(m->d_map, lower, 65536 * sizeof(uint16_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(m->d_special, special, 8192, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(m->d_map);
        (void)hipFree(m->d_special);
        delete m;
        return fail(e == hipErrorOutOfMemory ? LDGPU_ENOMEM : LDGPU_EDEVICE, "casemap upload: %s", hipGetErrorString(e));
    }
    *out = m;
    return ok();
}

extern "C" int ldgpu_casemap_destroy(ldgpu_casemap* m) {
    if (!m) return ok();
    (void)hipSetDevice(m->ctx->device);
    (void)hipFree(m->d_map);
    (void)hipFree(m->d_special);
    delete m;
    return ok();
}

extern "C" int ldgpu_preprocess_device(ldgpu_casemap* m, const uint16_t* d_units, const int64_t* d_offsets,
                                       int64_t n_docs, const uint8_t* d_locale, int32_t flags, void* d_out,
                                       int64_t* d_out_offsets, uint8_t* d_host, void* stream) {
    if (!m) return fail(LDGPU_EINVAL, "casemap is NULL");
    if (n_docs < 0) return fail(LDGPU_EINVAL, "n_docs < 0");
    if (flags & ~(LDGPU_PRE_LOWER | LDGPU_PRE_CLEAN | LDGPU_PRE_LOW_BYTES))
        return fail(LDGPU_EINVAL, "unknown preprocess flags 0x%x", flags);
    if (!d_out_offsets || (n_docs > 0 && (!d_offsets || !d_host || !d_out)))
        return fail(LDGPU_EINVAL, "device pointer is NULL");
    if (n_docs >= (int64_t)std::numeric_limits<int>::max())
        return fail(LDGPU_EUNSUPPORTED, "%lld documents in one call (the scan takes < 2^31)", (long long)n_docs);
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipSetDevice(m->ctx->device));
    PreParams p{};
    p.units = d_units;
    p.offsets = d_offsets;
    p.n_docs = n_docs;
    p.locale = d_locale;
    p.flags = flags;
    p.map = m->d_map;
    p.special = m->d_special;
    p.out = d_out;
    p.host = d_host;
    size_t scan_bytes = 0;
    HIP_TRY(launch_preprocess(p, nullptr, nullptr, nullptr, &scan_bytes, m->ctx->cus, st));
    int64_t* len_tmp = nullptr;
    HIP_TRY(hipMallocAsync((void**)&len_tmp, sizeof(int64_t) * (size_t)(n_docs + 1) + scan_bytes + 16, st));
    const hipError_t e = launch_preprocess(p, len_tmp, d_out_offsets, len_tmp + n_docs + 1, &scan_bytes, m->ctx->cus, st);
    (void)hipFreeAsync(len_tmp, st);
    HIP_TRY(e);
    return ok();
}

extern "C" int ldgpu_preprocess(ldgpu_casemap* m, const uint16_t* units, const int64_t* offsets, int64_t n_docs,
                                const uint8_t* locale, int32_t flags, void* out, int64_t* out_offsets, uint8_t* host) {
    if (!m) return fail(LDGPU_EINVAL, "casemap is NULL");
    if (int rc = check_offsets(offsets, n_docs)) return rc;
    if (!out_offsets || (n_docs > 0 && (!host || !out))) return fail(LDGPU_EINVAL, "output pointer is NULL");
    const int64_t b0 = n_docs > 0 ? offsets[0] : 0, nu = n_docs > 0 ? offsets[n_docs] - b0 : 0;
    if (nu > 0 && !units) return fail(LDGPU_EINVAL, "units is NULL");
    HIP_TRY(hipSetDevice(m->ctx->device));
    const size_t ob = (flags & LDGPU_PRE_LOW_BYTES) ? 1 : 2;
    std::vector<int64_t> off0((size_t)n_docs + 1);
    for (int64_t i = 0; i <= n_docs; ++i) off0[(size_t)i] = n_docs > 0 ? offsets[i] - b0 : 0;
    // one device block: units, offsets (in, out), locale, host flags, output
    const size_t a_units = ((size_t)nu * 2 + 15) & ~(size_t)15, a_off = sizeof(int64_t) * ((size_t)n_docs + 1);
    const size_t a_small = ((size_t)n_docs + 15) & ~(size_t)15, a_out = ((size_t)nu * ob + 15) & ~(size_t)15;
    uint8_t* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, a_units + 2 * a_off + 2 * a_small + a_out + 16));
    uint16_t* d_units = (uint16_t*)d;
    int64_t* d_off = (int64_t*)(d + a_units);
    int64_t* d_ooff = (int64_t*)(d + a_units + a_off);
    uint8_t* d_loc = d + a_units + 2 * a_off;
    uint8_t* d_host = d_loc + a_small;
    void* d_out = d_host + a_small;
    hipStream_t st = m->ctx->stream;
    int rc = LDGPU_OK;
    hipError_t e = hipSuccess;
    {
        std::lock_guard<std::mutex> lock(m->ctx->mu);  // the context's stream
        if (nu) e = hipMemcpyAsync(d_units, units + b0, (size_t)nu * 2, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(d_off, off0.data(), a_off, hipMemcpyHostToDevice, st);
        if (e == hipSuccess && locale && n_docs)
            e = hipMemcpyAsync(d_loc, locale, (size_t)n_docs, hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            rc = ldgpu_preprocess_device(m, d_units, d_off, n_docs, locale ? d_loc : nullptr, flags, d_out, d_ooff,
                                         d_host, st);
        if (e == hipSuccess && !rc) e = hipMemcpyAsync(out_offsets, d_ooff, a_off, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && !rc && n_docs) e = hipMemcpyAsync(host, d_host, (size_t)n_docs, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && !rc) e = hipStreamSynchronize(st);
        if (e == hipSuccess && !rc && out_offsets[n_docs] > 0)
            e = hipMemcpy(out, d_out, (size_t)out_offsets[n_docs] * ob, hipMemcpyDeviceToHost);
    }
    (void)hipFree(d);
    if (rc) return rc;
    HIP_TRY(e);
    return ok();
}

// -------------------------------------------------------------------- model
struct ldgpu_model {
    ldgpu_ctx* ctx = nullptr;
    int32_t L = 0, nG = 0;
    int32_t G[kMaxGramLengths] = {};
    int slices = 1;
    bool dense = false;
    int mode = 0;             // kernel mode: 0 mask, 1 mask + finite values, 2 dense, 3 mask + one finite value
    bool lds_filter = true;
    bool kb_lines = false;   // keyed bloom in the line layout (kKbLineBytes)
    bool kb_chunks = false;  // count mode: keyed bloom in the chunk layout (kb_chunk)
    bool has_bad = false;
    int64_t n_keys = 0;
    uint64_t slot_cap = 0;
    int filter_log2 = 10;     // bloom words (log2)
    uint32_t len_mask = 0;    // bit k: some key has k bytes
    size_t lds_bytes = 0;
    int wg_per_cu = 1;
    int ablate = 0;           // diagnostics build only: LDGPU_ABLATE
    size_t device_bytes = 0;
    Slot* d_slots = nullptr;
    WideSlot* d_wslots = nullptr;  // wide keys (8..15 bytes), nullptr: none
    uint64_t wslot_cap = 0;
    Bucket* d_buckets = nullptr;  // count mode key table
    uint64_t n_buckets = 0;
    uint32_t* d_filter = nullptr;
    uint64_t* d_masks = nullptr;
    double* d_vals = nullptr;
    double* d_rows = nullptr;
    double* d_fold = nullptr;  // mode 3: fold[c], c = 0..kFoldMax
    int count_sign = 0;        // mode 3: sign of the shared value
    uint32_t direct_off = 0, direct_words = 0;  // mode 3: direct tables in the image (ScoreParams)
    bool count_int_argmax = false;  // mode 3: label = first max of the counts (monotone fold)
    bool pack_ok = false;           // mode 3: short documents may be scored in packs (score_pack)
    // mode 1 with at most class_max(slices) distinct row values: labels-only
    // calls take class mode (kernel mode 4) with these values (unused: NaN)
    int n_cls = 0;
    double cls[4] = {};
    int32_t* d_err = nullptr;
    unsigned long long* d_stats = nullptr;  // LDGPU_STATS diagnostics (printed at destroy)
    // general keys (a gram length beyond kMaxWideGram: ldgpu_general.hip):
    // every key in one GenSlot table, its bytes in the arena
    bool general = false;
    GenSlot* d_gslots = nullptr;
    uint64_t gslot_cap = 0;
    uint8_t* d_arena = nullptr;
    int64_t* d_koff = nullptr;
    // mixed tables (general, and some gram length <= 15): the model of the
    // keys of <= 15 bytes over those lengths (nullptr: every length is long),
    // the long lengths and the long keys' prefilter bitmap (long_bits)
    ldgpu_model* short_m = nullptr;
    int n_long = 0;
    int32_t Glong[kMaxGramLengths] = {};
    int32_t max_long = 0;
    uint32_t* d_lbits = nullptr;
    uint32_t lbits_log2 = 0;
    // L > kBlockLangs: one sub-model per block of kBlockLangs languages
    // (model_build_blocked); this model then holds no table of its own
    std::vector<ldgpu_model*> blocks;
};

// mode 3 fold table: fold[c] = ((0.0 + v) + v) ... c times
constexpr uint32_t kFoldMax = 8191;

namespace {
void model_free(ldgpu_model* m) {
    if (!m) return;
    for (ldgpu_model* b : m->blocks) model_free(b);
    model_free(m->short_m);
    if (m->ctx) (void)hipSetDevice(m->ctx->device);
    if (m->d_stats) {
        unsigned long long st[2] = {0, 0};
        if (hipMemcpy(st, m->d_stats, sizeof st, hipMemcpyDeviceToHost) == hipSuccess)
            fprintf(stderr, "[ldgpu] stats: candidates verified %llu, hits %llu\n", st[0], st[1]);
        (void)hipFree(m->d_stats);
    }
    for (void* p : {(void*)m->d_slots, (void*)m->d_wslots, (void*)m->d_buckets, (void*)m->d_filter, (void*)m->d_masks, (void*)m->d_vals, (void*)m->d_rows,
                    (void*)m->d_fold, (void*)m->d_err, (void*)m->d_gslots, (void*)m->d_arena, (void*)m->d_koff,
                    (void*)m->d_lbits})
        if (p) (void)hipFree(p);
    delete m;
}

template <typename T>
hipError_t upload(T** dst, const std::vector<T>& src, size_t* total) {
    const size_t n = std::max<size_t>(src.size(), 1) * sizeof(T);
    hipError_t e = hipMalloc((void**)dst, n);
    if (e != hipSuccess) return e;
    *total += n;
    if (src.empty()) return hipMemset(*dst, 0, n);
    return hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
}
}  // namespace

namespace {
// A table parsed into device form: unique packed keys (Scala toMap semantics:
// a later duplicate key wins; keys longer than every window, which can never
// be hit, are dropped), per key a wrong-length flag, and either mask form
// (masks [n][S], vals [n]) or dense fp64 rows [n][L].
struct ParsedTable {
    std::vector<uint64_t> keys;          // one-word keys (<= 7 bytes), rows [0, keys.size())
    std::vector<uint64_t> wlo, whi;      // wide keys (8..15 bytes), rows keys.size() + j
    std::vector<uint8_t> bad;
    bool dense = false;
    std::vector<uint64_t> masks;
    std::vector<double> vals, drows;
};

int check_model_args(ldgpu_ctx* ctx, ldgpu_model** out, int64_t n_rows, int32_t n_langs,
                     const int32_t* gram_lengths, int32_t n_grams) {
    if (!ctx || !out) return fail(LDGPU_EINVAL, "ctx/out is NULL");
    if (n_langs < 1) return fail(LDGPU_EINVAL, "No values in array: the model has no supported languages");
    if (n_langs > LDGPU_MAX_LANGS)
        return fail(LDGPU_EUNSUPPORTED, "%d languages exceed the device path's limit of %d", n_langs,
                    LDGPU_MAX_LANGS);
    if (n_rows < 0) return fail(LDGPU_EINVAL, "n_rows < 0");
    return check_grams(gram_lengths, n_grams, LDGPU_MAX_GRAM);  // SCORE: any length (beyond 15: general keys)
}

// unique keys -> source row index (later duplicates win); wide keys (8..15
// bytes) into wlo / whi with their rows after the one-word keys' rows
struct PairHash {
    size_t operator()(const std::pair<uint64_t, uint64_t>& k) const { return (size_t)mix64(k.first ^ mix64(k.second)); }
};

int unique_keys(int64_t n_rows, const uint8_t* key_bytes, const int64_t* key_offsets, int maxg,
                std::vector<uint64_t>& keys, std::vector<int64_t>& src_row, std::vector<uint64_t>* wlo = nullptr,
                std::vector<uint64_t>* whi = nullptr) {
    std::unordered_map<uint64_t, int64_t> idx;
    idx.reserve((size_t)n_rows * 2 + 1);
    std::unordered_map<std::pair<uint64_t, uint64_t>, int64_t, PairHash> widx;
    std::vector<int64_t> wrow;
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t len = key_offsets[r + 1] - key_offsets[r];
        if (len < 0) return fail(LDGPU_EINVAL, "key_offsets decrease at row %lld", (long long)r);
        if (len == 0 || len > maxg) continue;
        if (len > kMaxGram) {
            if (!wlo) continue;
            const uint8_t* b = key_bytes + key_offsets[r];
            uint64_t lo = 0, hi = (uint64_t)len << 56;
            for (int i = 0; i < 8; ++i) lo |= (uint64_t)b[i] << (8 * i);
            for (int i = 8; i < len; ++i) hi |= (uint64_t)b[i] << (8 * (i - 8));
            auto it = widx.find({lo, hi});
            if (it == widx.end()) {
                widx.emplace(std::make_pair(lo, hi), (int64_t)wlo->size());
                wlo->push_back(lo);
                whi->push_back(hi);
                wrow.push_back(r);
            } else {
                wrow[it->second] = r;
            }
            continue;
        }
        const uint64_t k = pack_key_host(key_bytes + key_offsets[r], (int)len);
        auto it = idx.find(k);
        if (it == idx.end()) {
            idx.emplace(k, (int64_t)keys.size());
            keys.push_back(k);
            src_row.push_back(r);
        } else {
            src_row[it->second] = r;
        }
    }
    src_row.insert(src_row.end(), wrow.begin(), wrow.end());
    return LDGPU_OK;
}

int max_gram(const int32_t* G, int32_t nG) {
    int maxg = 0;
    for (int i = 0; i < nG; ++i) maxg = std::max(maxg, G[i]);
    return maxg;
}

int model_build(ldgpu_ctx* ctx, int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams, ParsedTable& t,
                ldgpu_model** out);

// Place every key in nb 5-slot buckets (count mode).  Primary bucket while it
// has room, else the secondary (raising the primary's overflow flag), else a
// bounded random walk of evictions; false when it does not settle.
bool bucket_place(const std::vector<uint64_t>& keys, const std::vector<uint64_t>& masks, int S,
                  const std::vector<uint8_t>& bad, uint64_t nb, std::vector<Bucket>& out) {
    out.assign(nb, Bucket{});
    auto prim = [&](uint64_t k) { return bucket_index((uint32_t)(mix64(k) >> 32), nb); };
    auto sec = [&](uint64_t k) { return bucket_index((uint32_t)mix64(k), nb); };
    auto put = [&](uint64_t b, int s, uint64_t k, uint32_t pay) {
        out[b].k[s] = k;
        out[b].p[s] = pay;
        if (b != prim(k)) out[prim(k)].flags |= kBucketOverflow;
    };
    auto free_slot = [&](uint64_t b) {
        for (int s = 0; s < 5; ++s)
            if (out[b].k[s] == kEmpty) return s;
        return -1;
    };
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < keys.size(); ++i) {
        uint32_t lang = 0xffffffffu;
        int bits = 0;
        for (int s = 0; s < S; ++s) {
            const uint64_t w = masks[i * S + s];
            if (w && !bits) lang = 64u * (uint32_t)s + (uint32_t)__builtin_ctzll(w);
            bits += __builtin_popcountll(w);
        }
        uint64_t k = keys[i];
        uint32_t pay = (bits == 1 ? (kPayLang | lang) : (uint32_t)i) | (bad[i] ? kBadRow : 0u);
        bool placed = false;
        for (int step = 0; step < 2000 && !placed; ++step) {
            const uint64_t b1 = prim(k), b2 = sec(k);
            int s;
            if ((s = free_slot(b1)) >= 0) {
                put(b1, s, k, pay);
                placed = true;
            } else if ((s = free_slot(b2)) >= 0) {
                put(b2, s, k, pay);
                placed = true;
            } else {
                // evict a random resident of the secondary bucket; it retries its own buckets
                rng = rng * 6364136223846793005ull + 1442695040888963407ull;
                s = (int)((rng >> 32) % 5u);
                const uint64_t vk = out[b2].k[s];
                const uint32_t vp = out[b2].p[s];
                put(b2, s, k, pay);
                k = vk;
                pay = vp;
            }
        }
        if (!placed) return false;
    }
    return true;
}
}  // namespace

extern "C" int ldgpu_model_create(ldgpu_ctx* ctx, int64_t n_rows, const uint8_t* key_bytes,
                                  const int64_t* key_offsets, const double* rows, const uint8_t* row_ok,
                                  int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                                  ldgpu_model** out);
extern "C" int ldgpu_model_create_masks(ldgpu_ctx* ctx, int64_t n_rows, const uint8_t* key_bytes,
                                        const int64_t* key_offsets, const uint64_t* masks, const double* vals,
                                        int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                                        ldgpu_model** out);

namespace {
// A model with a gram length beyond kMaxWideGram (ldgpu_general.hip): every
// key of 1..max(G) bytes (longer keys can never be hit) in one GenSlot table
// with its bytes in an arena; Scala toMap semantics (a later duplicate key
// wins).  Rows in mask form (masks [rows][S], vals) or dense (rows [rows][L]);
// row_ok (nullable) marks wrong-length rows.  src_row: row i of the table is
// source row src_row[i] of the caller's arrays.
int model_create_general(ldgpu_ctx* ctx, int64_t n_rows, const uint8_t* key_bytes, const int64_t* key_offsets,
                         const double* rows, const uint8_t* row_ok, const uint64_t* masks, const double* vals,
                         int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams, ldgpu_model** out) {
    const int maxg = max_gram(gram_lengths, n_grams);
    const int S = (n_langs + 63) / 64;
    std::unordered_map<std::string, int64_t> idx;
    idx.reserve((size_t)n_rows * 2 + 1);
    std::vector<int64_t> src;
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t len = key_offsets[r + 1] - key_offsets[r];
        if (len < 0) return fail(LDGPU_EINVAL, "key_offsets decrease at row %lld", (long long)r);
        if (len == 0 || len > maxg) continue;
        std::string k((const char*)key_bytes + key_offsets[r], (size_t)len);
        auto it = idx.find(k);
        if (it == idx.end()) {
            idx.emplace(std::move(k), (int64_t)src.size());
            src.push_back(r);
        } else {
            src[it->second] = r;
        }
    }
    const int64_t nk = (int64_t)src.size();
    if (nk >= (int64_t)kBadRow) return fail(LDGPU_EUNSUPPORTED, "%lld keys exceed the general table", (long long)nk);
    std::vector<uint8_t> arena;
    std::vector<int64_t> koff(1, 0);
    for (int64_t i = 0; i < nk; ++i) {
        const int64_t r = src[i];
        arena.insert(arena.end(), key_bytes + key_offsets[r], key_bytes + key_offsets[r + 1]);
        koff.push_back((int64_t)arena.size());
    }
    const uint64_t cap = next_pow2(std::max<uint64_t>(16, 2 * (uint64_t)nk + 1));
    std::vector<GenSlot> slots(cap, GenSlot{0, 0, 0});
    const uint32_t shift = (uint32_t)(64 - log2u(cap));
    for (int64_t i = 0; i < nk; ++i) {
        const int64_t len = koff[i + 1] - koff[i];
        const uint64_t h = gen_hash(arena.data() + koff[i], len);
        uint64_t sl = h >> shift;
        while (slots[sl].len) sl = (sl + 1) & (cap - 1);
        const bool bad = row_ok && !row_ok[src[i]];
        slots[sl] = GenSlot{h, (uint32_t)len, (uint32_t)i | (bad ? kBadRow : 0u)};
    }
    auto* m = new ldgpu_model();
    m->ctx = ctx;
    m->L = n_langs;
    m->nG = n_grams;
    for (int i = 0; i < n_grams; ++i) m->G[i] = gram_lengths[i];
    m->slices = S;
    m->general = true;
    m->n_keys = nk;
    m->gslot_cap = cap;
    m->slot_cap = cap;
    for (int64_t i = 0; i < nk; ++i) {
        const int64_t len = koff[i + 1] - koff[i];
        if (len < 32) m->len_mask |= 1u << len;
        m->has_bad |= row_ok && !row_ok[src[i]];
    }
    // mask form unless some row has two different nonzero values (as
    // ldgpu_model_create decides)
    std::vector<uint64_t> mk;
    std::vector<double> vv, dr;
    bool dense = false;
    if (rows) {
        for (int64_t i = 0; i < nk && !dense; ++i) {
            const double* rw = rows + src[i] * (int64_t)n_langs;
            uint64_t v = 0;
            bool have = false;
            for (int l = 0; l < n_langs && !dense; ++l) {
                if (rw[l] == 0.0) continue;
                uint64_t b;
                memcpy(&b, &rw[l], 8);
                if (!have) {
                    v = b;
                    have = true;
                } else {
                    dense = b != v;
                }
            }
        }
    }
    m->dense = dense;
    m->mode = dense ? 2 : 0;
    if (dense) {
        dr.resize((size_t)nk * n_langs);
        for (int64_t i = 0; i < nk; ++i)
            memcpy(&dr[(size_t)i * n_langs], rows + src[i] * (int64_t)n_langs, sizeof(double) * n_langs);
    } else {
        mk.assign((size_t)nk * S, 0);
        vv.assign((size_t)nk, 0.0);
        for (int64_t i = 0; i < nk; ++i) {
            if (rows) {
                const double* rw = rows + src[i] * (int64_t)n_langs;
                for (int l = 0; l < n_langs; ++l) {
                    if (rw[l] == 0.0) continue;
                    mk[(size_t)i * S + l / 64] |= 1ull << (l % 64);
                    vv[i] = rw[l];
                }
            } else {
                memcpy(&mk[(size_t)i * S], masks + src[i] * S, sizeof(uint64_t) * S);
                if (n_langs % 64) mk[(size_t)i * S + S - 1] &= (1ull << (n_langs % 64)) - 1ull;
                vv[i] = vals[src[i]];
                if (vv[i] == 0.0)  // the all-zero row
                    for (int w = 0; w < S; ++w) mk[(size_t)i * S + w] = 0;
            }
        }
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = upload(&m->d_gslots, slots, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_arena, arena, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_koff, koff, &m->device_bytes);
    if (e == hipSuccess && dense) e = upload(&m->d_rows, dr, &m->device_bytes);
    if (e == hipSuccess && !dense) e = upload(&m->d_masks, mk, &m->device_bytes);
    if (e == hipSuccess && !dense) e = upload(&m->d_vals, vv, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_err, std::vector<int32_t>{0}, &m->device_bytes);
    // mixed table: the long lengths (distinct), the prefilter bitmap of the
    // keys a full window of one of them can equal (2 bits per key, ~32 bits
    // per key: ~0.4 % of windows pass), and the short lengths' model
    std::vector<int32_t> gshort;
    for (int i = 0; i < n_grams; ++i) {
        const int32_t n = gram_lengths[i];
        if (n <= kMaxWideGram) {
            gshort.push_back(n);
            continue;
        }
        m->max_long = std::max(m->max_long, n);
        if (std::find(m->Glong, m->Glong + m->n_long, n) == m->Glong + m->n_long) m->Glong[m->n_long++] = n;
    }
    if (e == hipSuccess) {
        auto is_long = [&](int64_t len) { return std::find(m->Glong, m->Glong + m->n_long, (int32_t)len) != m->Glong + m->n_long; };
        int64_t nl = 0;
        for (int64_t i = 0; i < nk; ++i) nl += is_long(koff[i + 1] - koff[i]);
        uint32_t lb = 12;
        while (lb < 19 && ((uint64_t)1 << lb) < 32ull * (uint64_t)nl) ++lb;
        m->lbits_log2 = lb;
        std::vector<uint32_t> bits((size_t)1 << (lb - 5), 0u);
        for (int64_t i = 0; i < nk; ++i) {
            const int64_t len = koff[i + 1] - koff[i];
            if (!is_long(len)) continue;
            uint32_t w[2] = {0u, 0u};
            memcpy(w, arena.data() + koff[i], 8);
            uint32_t b1, b2;
            long_bits(w[0], w[1], (uint32_t)len, lb, b1, b2);
            bits[b1 >> 5] |= 1u << (b1 & 31);
            bits[b2 >> 5] |= 1u << (b2 & 31);
        }
        e = upload(&m->d_lbits, bits, &m->device_bytes);
    }
    if (e != hipSuccess) {
        model_free(m);
        return fail(LDGPU_ENOMEM, "model upload: %s", hipGetErrorString(e));
    }
    if (!gshort.empty()) {
        const int rc = rows ? ldgpu_model_create(ctx, n_rows, key_bytes, key_offsets, rows, row_ok, n_langs,
                                                 gshort.data(), (int32_t)gshort.size(), &m->short_m)
                            : ldgpu_model_create_masks(ctx, n_rows, key_bytes, key_offsets, masks, vals, n_langs,
                                                       gshort.data(), (int32_t)gshort.size(), &m->short_m);
        if (rc) {
            model_free(m);
            return rc;
        }
        m->device_bytes += m->short_m->device_bytes;
    }
    *out = m;
    return ok();
}
}  // namespace

extern "C" int ldgpu_model_create(ldgpu_ctx* ctx, int64_t n_rows, const uint8_t* key_bytes,
                                  const int64_t* key_offsets, const double* rows, const uint8_t* row_ok,
                                  int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                                  ldgpu_model** out) {
    if (int rc = check_model_args(ctx, out, n_rows, n_langs, gram_lengths, n_grams)) return rc;
    if (n_rows > 0 && (!key_bytes || !key_offsets || !rows)) return fail(LDGPU_EINVAL, "table pointer is NULL");
    if (max_gram(gram_lengths, n_grams) > kMaxWideGram)
        return model_create_general(ctx, n_rows, key_bytes, key_offsets, rows, row_ok, nullptr, nullptr, n_langs,
                                    gram_lengths, n_grams, out);
    ParsedTable t;
    std::vector<int64_t> src_row;
    if (int rc = unique_keys(n_rows, key_bytes, key_offsets, max_gram(gram_lengths, n_grams), t.keys, src_row,
                             &t.wlo, &t.whi))
        return rc;
    const int64_t nk = (int64_t)src_row.size();  // rows: one-word keys, then wide keys
    const int S = (n_langs + 63) / 64;
    t.bad.resize(nk);
    for (int64_t i = 0; i < nk; ++i) t.bad[i] = row_ok && !row_ok[src_row[i]];

    // mask form: every nonzero entry of every row bitwise equal within the row
    for (int64_t i = 0; i < nk && !t.dense; ++i) {
        const double* rw = rows + src_row[i] * (int64_t)n_langs;
        uint64_t v = 0;
        bool have = false;
        for (int l = 0; l < n_langs; ++l) {
            if (rw[l] == 0.0) continue;
            uint64_t b;
            memcpy(&b, &rw[l], 8);
            if (!have) {
                v = b;
                have = true;
            } else if (b != v) {
                t.dense = true;
                break;
            }
        }
    }
    if (!t.dense) {
        t.masks.assign((size_t)nk * S, 0);
        t.vals.assign((size_t)nk, 0.0);
        for (int64_t i = 0; i < nk; ++i) {
            const double* rw = rows + src_row[i] * (int64_t)n_langs;
            for (int l = 0; l < n_langs; ++l) {
                if (rw[l] == 0.0) continue;
                t.masks[(size_t)i * S + l / 64] |= 1ull << (l % 64);
                t.vals[i] = rw[l];
            }
        }
    } else {
        t.drows.resize((size_t)nk * n_langs);
        for (int64_t i = 0; i < nk; ++i)
            memcpy(&t.drows[(size_t)i * n_langs], rows + src_row[i] * (int64_t)n_langs, sizeof(double) * n_langs);
    }
    return model_build(ctx, n_langs, gram_lengths, n_grams, t, out);
}

extern "C" int ldgpu_model_create_masks(ldgpu_ctx* ctx, int64_t n_rows, const uint8_t* key_bytes,
                                        const int64_t* key_offsets, const uint64_t* masks, const double* vals,
                                        int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                                        ldgpu_model** out) {
    if (int rc = check_model_args(ctx, out, n_rows, n_langs, gram_lengths, n_grams)) return rc;
    if (n_rows > 0 && (!key_bytes || !key_offsets || !masks || !vals))
        return fail(LDGPU_EINVAL, "table pointer is NULL");
    if (max_gram(gram_lengths, n_grams) > kMaxWideGram)
        return model_create_general(ctx, n_rows, key_bytes, key_offsets, nullptr, nullptr, masks, vals, n_langs,
                                    gram_lengths, n_grams, out);
    ParsedTable t;
    std::vector<int64_t> src_row;
    if (int rc = unique_keys(n_rows, key_bytes, key_offsets, max_gram(gram_lengths, n_grams), t.keys, src_row,
                             &t.wlo, &t.whi))
        return rc;
    const int64_t nk = (int64_t)src_row.size();  // rows: one-word keys, then wide keys
    const int S = (n_langs + 63) / 64;
    t.bad.assign(nk, 0);
    t.masks.resize((size_t)nk * S);
    t.vals.resize(nk);
    for (int64_t i = 0; i < nk; ++i) {
        memcpy(&t.masks[(size_t)i * S], masks + src_row[i] * S, sizeof(uint64_t) * S);
        if (n_langs % 64) t.masks[(size_t)i * S + S - 1] &= (1ull << (n_langs % 64)) - 1ull;
        t.vals[i] = vals[src_row[i]];
        // a row whose value is 0.0 (or -0.0) is the all-zero row
        if (t.vals[i] == 0.0)
            for (int s = 0; s < S; ++s) t.masks[(size_t)i * S + s] = 0;
    }
    return model_build(ctx, n_langs, gram_lengths, n_grams, t, out);
}

namespace {
// L > kBlockLangs: the languages are scored in blocks of kBlockLangs, one
// sub-model per block holding that block's columns and only the keys with a
// nonzero entry there (a zero row adds exact zeros: no effect); wrong-length
// rows stay in every block so a hit still fails.  A document's label is the
// first maximum over the blocks' maxima (launch_combine_blocks).
int model_build_blocked(ldgpu_ctx* ctx, int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                        ParsedTable& t, ldgpu_model** out) {
    const int64_t nn = (int64_t)t.keys.size();
    const int64_t nk = nn + (int64_t)t.wlo.size();  // rows: one-word keys, then wide keys
    const int S = (n_langs + 63) / 64;
    const int nb = (n_langs + kBlockLangs - 1) / kBlockLangs;
    auto* m = new ldgpu_model();
    m->ctx = ctx;
    m->L = n_langs;
    m->nG = n_grams;
    for (int i = 0; i < n_grams; ++i) m->G[i] = gram_lengths[i];
    m->slices = S;
    m->dense = t.dense;
    m->n_keys = nk;
    for (int b = 0; b < nb; ++b) {
        const int l0 = b * kBlockLangs, lb = std::min(kBlockLangs, n_langs - l0);
        const int w0 = l0 / 64, sb = (lb + 63) / 64;
        ParsedTable tb;
        tb.dense = t.dense;
        for (int64_t i = 0; i < nk; ++i) {
            bool any = t.bad[i] != 0;
            if (t.dense) {
                for (int l = 0; l < lb && !any; ++l) any = t.drows[(size_t)i * n_langs + l0 + l] != 0.0;
            } else {
                for (int w = 0; w < sb && !any; ++w) any = t.masks[(size_t)i * S + w0 + w] != 0;
            }
            if (!any) continue;
            if (i < nn) {
                tb.keys.push_back(t.keys[i]);
            } else {
                tb.wlo.push_back(t.wlo[i - nn]);
                tb.whi.push_back(t.whi[i - nn]);
            }
            tb.bad.push_back(t.bad[i]);
            if (t.dense) {
                tb.drows.insert(tb.drows.end(), t.drows.begin() + (size_t)i * n_langs + l0,
                                t.drows.begin() + (size_t)i * n_langs + l0 + lb);
            } else {
                for (int w = 0; w < sb; ++w) tb.masks.push_back(t.masks[(size_t)i * S + w0 + w]);
                tb.vals.push_back(t.vals[i]);
            }
        }
        ldgpu_model* sub = nullptr;
        if (int rc = model_build(ctx, lb, gram_lengths, n_grams, tb, &sub)) {
            model_free(m);
            return rc;
        }
        m->blocks.push_back(sub);
        m->has_bad |= sub->has_bad;
        m->device_bytes += sub->device_bytes;
        m->slot_cap += sub->slot_cap;
    }
    m->mode = m->blocks[0]->mode;
    m->filter_log2 = m->blocks[0]->filter_log2;
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = upload(&m->d_err, std::vector<int32_t>{0}, &m->device_bytes);
    if (e != hipSuccess) {
        model_free(m);
        return fail(LDGPU_EDEVICE, "model upload: %s", hipGetErrorString(e));
    }
    *out = m;
    return ok();
}

int model_build(ldgpu_ctx* ctx, int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams, ParsedTable& t,
                ldgpu_model** out) {
    if (n_langs > kBlockLangs) return model_build_blocked(ctx, n_langs, gram_lengths, n_grams, t, out);
    const int64_t nn = (int64_t)t.keys.size();        // one-word keys: rows [0, nn)
    const int64_t nw = (int64_t)t.wlo.size();         // wide keys: rows [nn, nn + nw)
    const int64_t nk = nn + nw;
    const int S = (n_langs + 63) / 64;
    const bool dense = t.dense;
    std::vector<uint64_t>& keys = t.keys;
    std::vector<uint64_t>& masks = t.masks;
    std::vector<double>& vals = t.vals;
    std::vector<double>& drows = t.drows;
    std::vector<double> fold;

    auto* m = new ldgpu_model();
    m->ctx = ctx;
    m->L = n_langs;
    m->nG = n_grams;
    for (int i = 0; i < n_grams; ++i) m->G[i] = gram_lengths[i];
    m->slices = S;
    m->dense = dense;
    m->n_keys = nk;
    m->mode = dense ? 2 : 1;
    if (!dense) {
        for (int64_t i = 0; i < nk && m->mode == 1; ++i) {
            bool any = false;
            for (int s = 0; s < S; ++s) any |= masks[(size_t)i * S + s] != 0;
            if (any && !std::isfinite(vals[i])) m->mode = 0;
        }
        // one value shared by every row with a nonzero entry: order-free
        // per-language hit counts (mode 3) reproduce the fold exactly
        bool have_v = false, uniform = m->mode == 1;
        uint64_t vbits = 0;
        for (int64_t i = 0; i < nk && uniform; ++i) {
            bool any = false;
            for (int s = 0; s < S; ++s) any |= masks[(size_t)i * S + s] != 0;
            if (!any) continue;
            uint64_t b;
            memcpy(&b, &vals[i], 8);
            if (!have_v) {
                vbits = b;
                have_v = true;
            } else if (b != vbits) {
                uniform = false;
            }
        }
        if (const char* f = diag_env("LDGPU_NO_COUNT_MODE")) uniform &= atoi(f) == 0;  // tests cover both paths
        if (uniform) {
            m->mode = 3;
            double v;
            memcpy(&v, &vbits, 8);
            fold.resize(kFoldMax + 1);
            fold[0] = 0.0;
            for (uint32_t c = 1; c <= kFoldMax; ++c) fold[c] = fold[c - 1] + v;
            // |v| far from overflow: fold[c] (c < 2^24) is strictly monotone
            // (each add moves it: |v| >> ulp(c |v|) / 2), so argmax needs only c
            m->count_sign = v > 0.0 ? 1 : (v < 0.0 ? -1 : 0);
            m->count_int_argmax = std::fabs(v) < 1e300;
        }
        // a few distinct values (e.g. a fit table's presence classes):
        // labels-only calls count hits per (value, language) and replay only
        // the documents a rounding bound cannot separate (class_label)
        if (m->mode == 1 && !diag_env("LDGPU_NO_CLASS_MODE")) {
            int nc = 0;
            bool fits = true;
            for (int64_t i = 0; i < nk && fits; ++i) {
                bool any = false;
                for (int s = 0; s < S; ++s) any |= masks[(size_t)i * S + s] != 0;
                if (!any) continue;
                int q = 0;
                while (q < nc && !(m->cls[q] == vals[i])) ++q;  // == : 0.0 and -0.0 add alike
                if (q < nc) continue;
                if (nc == std::min(4, class_max(S))) fits = false;
                else m->cls[nc++] = vals[i];
            }
            if (fits && nc > 0) {
                m->n_cls = nc;
                for (int q = nc; q < 4; ++q) m->cls[q] = std::numeric_limits<double>::quiet_NaN();
            }
        }
    }

    // class mode: a one-language row's slot names its counter, class q and
    // language l -> q 64 S + l (class_label's layout); other modes: l
    auto lang_slot = [&](int64_t i, uint32_t l) -> uint32_t {
        if (!m->n_cls || l == 0xffffffffu) return l;
        uint32_t q = 0;
        while ((int)q + 1 < m->n_cls && !(m->cls[q] == vals[i])) ++q;
        return q * 64u * (uint32_t)S + l;
    };

    // key -> row slots (mask form: the row's value and first mask word inline),
    // 2-choice cuckoo hashing: a key sits in slot h >> (64 - log2 cap) or
    // slot h & (cap - 1) of h = mix64(key), so the device verifies a candidate
    // with two independent loads and no probe loop.  Load <= 0.4 (2.5 slots
    // per key) lets the cuckoo walk settle in a few steps; a walk that does
    // not settle doubles the table and starts over.
    std::vector<Slot> slots;
    std::vector<Bucket> buckets;
    // count mode with a table beyond the caches (> 2^20 keys: 32 MiB of slots):
    // 2-choice buckets of 5 slots (Bucket, ldgpu_common.h: one 64-B line) at
    // about 0.85 load, so most lookups read ONE HBM line instead of two slots;
    // cache-resident tables keep the two independent slot loads (one dependent
    // step less) (such a table's bloom never fits LDS: the keyed kernels, which
    // alone read buckets)
    // Also every other count-mode table whose bloom is keyed (those kernels
    // alone read buckets) once its cuckoo slots (2.5 per key, 32 B) would pass
    // kBucketL2Bytes: config 4's 100k keys take 8 MiB of slots, which an XCD's
    // 4 MiB L2 does not hold, against 1.5 MiB of buckets (one L2-resident line
    // per verify).  Diagnostics: LDGPU_BUCKETS=0/1 forces either layout.
    int64_t n_long = nw;
    for (int64_t i = 0; i < nn; ++i) n_long += key_len(keys[i]) >= 3;
    double kpw = 2.5;
    if (const char* s = diag_env("LDGPU_BLOOM_KPW")) kpw = std::max(0.05, atof(s));  // tuning experiments only
    uint64_t bwords = next_pow2(std::max<uint64_t>(64, (uint64_t)((double)n_long / kpw) + 1));
    bwords = std::min<uint64_t>(bwords, 1ull << kMaxBloomLog2);
    const bool keyed = bwords > (1ull << kMaxLdsBloomLog2);
    constexpr double kBucketL2Bytes = 2.0 * (1 << 20);
    bool use_buckets = m->mode == 3 && (nn > (1 << 20) || (keyed && 2.5 * 32.0 * (double)nn > kBucketL2Bytes));
    if (const char* b = diag_env("LDGPU_BUCKETS")) use_buckets = m->mode == 3 && keyed && atoi(b) != 0;
#ifdef LDGPU_BIG_BUCKETS_ONLY  // A/B builds (tools/build_variant.sh): round 4's rule
    use_buckets = m->mode == 3 && nn > (1 << 20);
#endif
    if (use_buckets && (uint64_t)nk >= (uint64_t)kPayLang) {
        // a bucket payload holds a multi-language row's index below kPayLang
        // (bit 30 marks a one-language payload, bit 31 a bad row)
        delete m;
        return fail(LDGPU_EUNSUPPORTED, "key table: %lld one-word keys, bucket payloads hold row indices < 2^30",
                    (long long)nk);
    }
    if (use_buckets) {
        // ~0.85 load (any bucket count); a placement that does not settle
        // retries with 10 % more buckets
        for (m->n_buckets = std::max<uint64_t>(16, (uint64_t)((double)nn / 4.25) + 1);;
             m->n_buckets += m->n_buckets / 10 + 1) {
            if (bucket_place(keys, masks, S, t.bad, m->n_buckets, buckets)) break;
            if (m->n_buckets >= (1ull << 31)) {
                delete m;
                return fail(LDGPU_ENOMEM, "key table: bucket placement failed");
            }
        }
        m->slot_cap = m->n_buckets * 5;
        for (int64_t i = 0; i < nk; ++i) m->has_bad |= t.bad[i] != 0;
    }
    for (m->slot_cap = use_buckets ? m->slot_cap
                                   : next_pow2(std::max<uint64_t>(16, (uint64_t)(2.5 * (double)nn) + 1));
         !use_buckets; m->slot_cap *= 2) {
        const int slog = log2u(m->slot_cap);
        const uint64_t cmask = m->slot_cap - 1;
        (void)cmask;
        if (slog > 32) {
            delete m;
            return fail(LDGPU_ENOMEM, "key table: more than 2^32 slots");
        }
        auto pos1 = [&](uint64_t k) {
            uint32_t h1, h2;
            slot_hash((uint32_t)k, (uint32_t)(k >> 32), h1, h2);
            return slog ? (uint64_t)(h1 >> (32 - slog)) : 0ull;
        };
        auto pos2 = [&](uint64_t k) {
            uint32_t h1, h2;
            slot_hash((uint32_t)k, (uint32_t)(k >> 32), h1, h2);
            return slog ? (uint64_t)(h2 >> (32 - slog)) : 0ull;
        };
        slots.assign(m->slot_cap, Slot{kEmpty, 0, 0xffffffffu, 0.0, 0});
        bool ok_all = true;
        for (int64_t i = 0; i < nn && ok_all; ++i) {
            Slot cur{keys[i], (uint32_t)i, 0xffffffffu, 0.0, 0};
            if (!dense) {
                cur.val = vals[i];
                cur.mask0 = masks[(size_t)i * S];
                // the row's one language, when it has exactly one (count mode reads it
                // instead of the mask words)
                int bits = 0;
                for (int s = 0; s < S; ++s) {
                    const uint64_t w = masks[(size_t)i * S + s];
                    if (w && !bits) cur.pad = 64u * (uint32_t)s + (uint32_t)__builtin_ctzll(w);
                    bits += __builtin_popcountll(w);
                }
                if (bits != 1) cur.pad = 0xffffffffu;
                cur.pad = lang_slot(i, cur.pad);
            }
            if (t.bad[i]) {
                cur.row |= kBadRow;
                m->has_bad = true;
            }
            uint64_t at = pos1(cur.key);
            if (slots[at].key != kEmpty && slots[pos2(cur.key)].key == kEmpty) at = pos2(cur.key);
            bool placed = false;
            for (int step = 0; step < 2000; ++step) {
                if (slots[at].key == kEmpty) {
                    slots[at] = cur;
                    placed = true;
                    break;
                }
                std::swap(cur, slots[at]);  // evict; the evicted key moves to its other slot
                const uint64_t a = pos1(cur.key), b = pos2(cur.key);
                at = at == a ? b : a;
            }
            ok_all = placed;
        }
        if (ok_all) break;
        if (m->slot_cap >= (1ull << 34)) {
            delete m;
            return fail(LDGPU_ENOMEM, "key table: cuckoo placement failed");
        }
    }

    // wide keys (8..15 bytes): their own 2-choice cuckoo table (WideSlot), rows
    // nn + j of the row arrays
    std::vector<WideSlot> wslots;
    if (nw > 0) {
        for (m->wslot_cap = next_pow2(std::max<uint64_t>(16, (uint64_t)(2.5 * (double)nw) + 1));;
             m->wslot_cap *= 2) {
            const int wlog = log2u(m->wslot_cap);
            if (wlog > 32) {
                delete m;
                return fail(LDGPU_ENOMEM, "wide key table: more than 2^32 slots");
            }
            auto wpos = [&](const WideSlot& w, int which) {
                uint32_t h1, h2;
                wide_hash(w.lo, w.hi, h1, h2);
                return (uint64_t)((which ? h2 : h1) >> (32 - wlog));
            };
            wslots.assign(m->wslot_cap, WideSlot{0, 0, 0, 0xffffffffu, {0, 0}});
            bool ok_all = true;
            for (int64_t j = 0; j < nw && ok_all; ++j) {
                const int64_t i = nn + j;
                WideSlot cur{t.wlo[j], t.whi[j], (uint32_t)i, 0xffffffffu, {0, 0}};
                if (!dense) {
                    int bits = 0;
                    for (int sidx = 0; sidx < S; ++sidx) {
                        const uint64_t w = masks[(size_t)i * S + sidx];
                        if (w && !bits) cur.lang1 = 64u * (uint32_t)sidx + (uint32_t)__builtin_ctzll(w);
                        bits += __builtin_popcountll(w);
                    }
                    if (bits != 1) cur.lang1 = 0xffffffffu;
                    cur.lang1 = lang_slot(i, cur.lang1);
                }
                if (t.bad[i]) {
                    cur.row |= kBadRow;
                    m->has_bad = true;
                }
                uint64_t at = wpos(cur, 0);
                if (wslots[at].hi != 0 && wslots[wpos(cur, 1)].hi == 0) at = wpos(cur, 1);
                bool placed = false;
                for (int step = 0; step < 2000; ++step) {
                    if (wslots[at].hi == 0) {  // (hi holds the length: never 0 in a key)
                        wslots[at] = cur;
                        placed = true;
                        break;
                    }
                    std::swap(cur, wslots[at]);
                    const uint64_t a = wpos(cur, 0), b = wpos(cur, 1);
                    at = at == a ? b : a;
                }
                ok_all = placed;
            }
            if (ok_all) break;
        }
    }

    // filter image: exact bitmaps of the 1- and 2-byte keys, then the prefix
    // Bloom filter of the longer ones (ldgpu_common.h).  The bloom is staged
    // in LDS up to 64 KiB, else read from global memory (L2 / Infinity Cache).
    // ~2 keys per 32-bit word (one bit each) keeps false positives at a few
    // percent: they only cost verification lanes (~1 VALU op each, batched 64
    // at a time), while LDS costs resident workgroups.
    // (n_long and bwords: computed with the key table's layout above)
    for (int64_t i = 0; i < nn; ++i) m->len_mask |= 1u << key_len(keys[i]);
    for (int64_t j = 0; j < nw; ++j) m->len_mask |= 1u << key_len(t.whi[j]);
    m->lds_filter = !keyed;
    m->kb_lines = !m->lds_filter && (4 * bwords > kKbLineBytes || diag_env("LDGPU_KB_LINES"));  // (tests: any keyed bloom)
    m->filter_log2 = log2u(bwords);
    const uint32_t bshift = 32u - (uint32_t)m->filter_log2;
    std::vector<uint32_t> filter(kBloomBase + bwords, 0u);
    for (int64_t i = 0; i < nn + nw; ++i) {
        // a wide key's filter bits: its first seven bytes and its length
        const int kl = i < nn ? key_len(keys[i]) : key_len(t.whi[i - nn]);
        const uint64_t kw = i < nn ? keys[i] : t.wlo[i - nn];
        if (kl == 1) {
            const uint32_t b0 = (uint32_t)(kw & 0xff);
            filter[b0 >> 5] |= 1u << (b0 & 31);
        } else if (kl == 2) {
            const uint32_t b01 = (uint32_t)(kw & 0xffff);
            filter[kBmp1Words + bmp2_word(b01)] |= 1u << (b01 & 31);
        } else {
            const uint32_t lo = (uint32_t)kw;
            const uint32_t hi = (uint32_t)(kw >> 32) & ((1u << (8 * std::min(3, std::max(0, kl - 4)))) - 1u);
            if (m->lds_filter) {  // prefix bloom (LDGPU_BLOOM_BITS bits per key)
                const uint32_t b = pf_bit(kl, lo, hi);
                filter[kBloomBase + pf_word(lo, bshift)] |= 1u << (b & 31u);
                if (LDGPU_BLOOM_BITS == 2) filter[kBloomBase + pf_word(lo, bshift)] |= 1u << (pf_bit2(kl, lo, hi) & 31u);
            } else {  // keyed bloom (kb_hash; keys of >= 4 bytes in their position's line)
                const uint32_t h = kb_hash(lo, hi, (uint32_t)kl);
                const bool ln = m->kb_lines && kl >= 4;
                const uint32_t w = (ln ? kb_line16(lo, bshift) : 0u) + (h >> kb_sword(kl, m->kb_lines, bshift));
                filter[kBloomBase + w] |= 1u << ((h >> kb_sbit(kl, m->kb_lines, bshift)) & 31u);
            }
        }
    }

    // Count mode, keyed bloom that stays L2-resident: the chunk layout
    // (kb_chunk, ldgpu_common.h) when its false-candidate estimate is at most
    // 1.5x the word layout's: a position then costs one L2 request for every
    // key length instead of one per length.  The estimates stand in for text
    // windows that are not keys: the word layout's, its overall fill (a
    // window's word is random); the chunk layout's, the mean of (filled bits /
    // 128)^2 over the chunks of the keys' distinct 3-byte prefixes (a window
    // whose prefix many keys share is mostly a key itself: weighting chunks
    // by key count overstates it ~6x on config 4's table).
    if (!m->lds_filter && !m->kb_lines && m->mode == 3 && bwords >= 8) {  // >= 2 chunks: cshift < 32
        const uint64_t chunks = bwords / 4;
        const uint32_t cshift = 32u - (uint32_t)log2u(chunks);
        std::vector<uint32_t> cf(bwords, 0u);
        std::unordered_set<uint32_t> prefixes;
        for (int64_t i = 0; i < nn + nw; ++i) {
            const int kl = i < nn ? key_len(keys[i]) : key_len(t.whi[i - nn]);
            if (kl < 3) continue;
            const uint64_t kw = i < nn ? keys[i] : t.wlo[i - nn];
            const uint32_t lo = (uint32_t)kw;
            const uint32_t hi = (uint32_t)(kw >> 32) & ((1u << (8 * std::min(3, std::max(0, kl - 4)))) - 1u);
            const uint32_t h = kb_hash(lo, hi, (uint32_t)kl);
            const uint32_t c = kb_chunk(lo) >> cshift;
            for (uint32_t q : {h >> 25, (h >> 18) & 127u}) cf[4 * c + (q >> 5)] |= 1u << (q & 31u);
            prefixes.insert(lo & 0xffffffu);
        }
        uint64_t set = 0;
        for (uint64_t w = 0; w < bwords; ++w) set += __builtin_popcount(filter[kBloomBase + w]);
        const double ew = (double)set / (32.0 * (double)bwords);
        double ec = 0.0;
        for (uint32_t pr : prefixes) {
            const uint32_t* q = &cf[4 * (kb_chunk(pr) >> cshift)];
            const double fc = (__builtin_popcount(q[0]) + __builtin_popcount(q[1]) + __builtin_popcount(q[2]) +
                               __builtin_popcount(q[3])) / 128.0;
            ec += fc * fc;
        }
        ec /= (double)std::max<size_t>(prefixes.size(), 1);
        m->kb_chunks = ec <= 1.5 * ew;
#ifdef LDGPU_NO_KB_CHUNKS  // A/B builds (tools/build_variant.sh)
        m->kb_chunks = false;
#endif
        if (const char* kc = diag_env("LDGPU_KB_CHUNKS")) m->kb_chunks = atoi(kc) != 0;  // tests: either layout
        if (m->kb_chunks) std::copy(cf.begin(), cf.end(), filter.begin() + kBloomBase);
    }

    // count mode with every 1-/2-byte key naming ONE language (fit tables of
    // grams unique to a language): direct tables after the image (see
    // ScoreParams::direct_*), so those keys are counted from LDS unverified.
    // Class mode too, for L <= 63 (one slice): an entry is the counter,
    // language | class << 6 (lang_slot; never 0xff)
    uint32_t image_words = kBloomBase + (m->lds_filter ? (uint32_t)bwords : 0u);
    const bool direct_mode = m->mode == 3 ? n_langs <= 255 : (m->n_cls > 0 && n_langs <= 63);
    if (direct_mode && m->lds_filter && !diag_env("LDGPU_NO_DIRECT")) {
        std::vector<uint8_t> lang1(256, 0xff), lang2of(65536, 0xff);
        bool ok = true;
        for (int64_t i = 0; i < nn && ok; ++i) {
            const int kl = key_len(keys[i]);
            if (kl > 2) continue;
            int bits = 0, lang = 0;
            for (int s = 0; s < S; ++s) {
                const uint64_t w = masks[(size_t)i * S + s];
                if (w && !bits) lang = 64 * s + __builtin_ctzll(w);
                bits += __builtin_popcountll(w);
            }
            ok = bits == 1 && !t.bad[i];
            const uint8_t e = (uint8_t)lang_slot(i, (uint32_t)lang);
            if (kl == 1) lang1[keys[i] & 0xff] = e;
            else lang2of[keys[i] & 0xffff] = e;
        }
        if (ok) {
            std::vector<uint16_t> base2(2048);
            std::vector<uint8_t> lang2;
            for (uint32_t wd = 0; wd < 2048; ++wd) {
                base2[wd] = (uint16_t)lang2.size();
                for (uint32_t b = 0; b < 32; ++b)
                    if ((filter[kBmp1Words + wd] >> b) & 1u) lang2.push_back(lang2of[bmp2_unword(wd) * 32 + b]);
            }
            const uint32_t dwords = 64u + 1024u + (uint32_t)((lang2.size() + 16) / 16) * 4u;  // uint4-padded
            const uint32_t hw4 = m->mode == 3 ? 0u : 64u * (uint32_t)S * (uint32_t)m->n_cls;
            if (score_lds_bytes(S, m->mode == 3 ? 3 : 4, image_words + dwords, false, hw4) * 2 <= 163840) {
                m->direct_off = image_words;
                m->direct_words = dwords;
                filter.resize(image_words + dwords, 0u);
                uint8_t* d = reinterpret_cast<uint8_t*>(filter.data() + image_words);
                memcpy(d, lang1.data(), 256);
                memcpy(d + 256, base2.data(), 4096);
                memcpy(d + 256 + 4096, lang2.data(), lang2.size());
                image_words += dwords;
            }
        }
    }

    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = upload(&m->d_slots, slots, &m->device_bytes);
    if (e == hipSuccess && nw > 0) e = upload(&m->d_wslots, wslots, &m->device_bytes);
    if (e == hipSuccess && use_buckets) e = upload(&m->d_buckets, buckets, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_filter, filter, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_masks, masks, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_vals, vals, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_rows, drows, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_fold, fold, &m->device_bytes);
    if (e == hipSuccess) e = upload(&m->d_err, std::vector<int32_t>{0}, &m->device_bytes);
    m->lds_bytes = score_lds_bytes(S, m->mode, image_words);
    // packs of short documents need kPackDocs counter blocks per wave: only
    // when that keeps the workgroups per CU (the prepared LDS limit is then
    // the packed size; a launch without packing asks for less)
    if (m->mode == 3 && m->count_int_argmax && !diag_env("LDGPU_NO_PACK")) {
        const size_t packed = score_lds_bytes(S, 3, image_words, true);
        if (packed <= 163840 && 163840 / packed >= 163840 / m->lds_bytes) {
            m->pack_ok = true;
            m->lds_bytes = packed;
        }
    }
    int resident = 0;
    if (m->n_cls) {
        // the ordered replay reads no direct tables; class mode's hit area
        // holds its classes' counters: the larger of the two launches
        const size_t l1 = score_lds_bytes(S, 1, image_words - m->direct_words);
        const size_t l4 = score_lds_bytes(S, 4, image_words, false, 64u * (uint32_t)S * (uint32_t)m->n_cls);
        m->lds_bytes = std::max(l1, l4);
        if (e == hipSuccess) e = score_prepare(S, 1, m->lds_filter, m->kb_chunks, l1, &resident);
        int r4 = 0;  // class mode shares the grid: the smaller occupancy
        if (e == hipSuccess) e = score_prepare(S, 4, m->lds_filter, m->kb_chunks, l4, &r4);
        if (r4 > 0) resident = resident > 0 ? std::min(resident, r4) : r4;
    } else if (e == hipSuccess) {
        e = score_prepare(S, m->mode, m->lds_filter, m->kb_chunks, m->lds_bytes, &resident);
    }
    // persistent grid = what is resident; never more workgroups than the LDS admits
    m->wg_per_cu = std::max<int>(1, std::min<int>(resident > 0 ? resident : 1, (int)(163840 / m->lds_bytes)));
    if (const char* ov = diag_env("LDGPU_WG_PER_CU")) m->wg_per_cu = std::max(1, atoi(ov));
    if (const char* ab = diag_env("LDGPU_ABLATE")) m->ablate = atoi(ab);
    if (diag_env("LDGPU_STATS") && e == hipSuccess) {
        e = hipMalloc((void**)&m->d_stats, 2 * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMemset(m->d_stats, 0, 2 * sizeof(unsigned long long));
    }
    if (diag_env("LDGPU_DEBUG"))
        fprintf(stderr, "[ldgpu] model: keys=%lld mode=%d direct=%u slices=%d bloom_words=%llu lds_bloom=%d lds=%zu B "
                        "resident_api=%d wg_per_cu=%d pack=%d classes=%d\n",
                (long long)nk, m->mode, m->direct_words, S, (unsigned long long)bwords, (int)m->lds_filter, m->lds_bytes, resident,
                m->wg_per_cu, (int)m->pack_ok, m->n_cls);
    if (e != hipSuccess) {
        model_free(m);
        return fail(e == hipErrorOutOfMemory ? LDGPU_ENOMEM : LDGPU_EDEVICE, "model upload: %s",
                    hipGetErrorString(e));
    }
    *out = m;
    return ok();
}

}  // namespace

extern "C" int ldgpu_model_destroy(ldgpu_model* m) {
    model_free(m);
    return ok();
}

extern "C" int ldgpu_model_info(const ldgpu_model* m, int32_t* mode, int64_t* n_keys, int64_t* table_slots,
                                int64_t* filter_bits, int64_t* device_bytes) {
    if (!m) return fail(LDGPU_EINVAL, "model is NULL");
    if (mode) *mode = m->dense ? 1 : (m->mode == 3 ? 2 : 0);
    if (n_keys) *n_keys = m->n_keys;
    if (table_slots) *table_slots = (int64_t)m->slot_cap;
    if (filter_bits) *filter_bits = ((int64_t)1 << m->filter_log2) * 32;  // bloom bits
    if (device_bytes) *device_bytes = (int64_t)m->device_bytes;
    return ok();
}

extern "C" int ldgpu_model_langs(const ldgpu_model* m, int32_t* n_langs) {
    if (!m || !n_langs) return fail(LDGPU_EINVAL, "model/n_langs is NULL");
    *n_langs = m->L;
    return ok();
}

extern "C" int ldgpu_model_layout(const ldgpu_model* m, int32_t* flags) {
    if (!m || !flags) return fail(LDGPU_EINVAL, "model/flags is NULL");
    const ldgpu_model* b = m->blocks.empty() ? m : m->blocks[0];  // blocks share one layout
    int32_t f = 0;
    if (b->lds_filter) f |= LDGPU_LAYOUT_LDS_BLOOM;
    if (!b->lds_filter && !b->kb_lines && !b->kb_chunks) f |= LDGPU_LAYOUT_KEYED_BLOOM;
    if (b->kb_chunks) f |= LDGPU_LAYOUT_KEYED_BLOOM_CHUNKS;
    if (b->kb_lines) f |= LDGPU_LAYOUT_KEYED_BLOOM_LINES;
    if (b->d_buckets) f |= LDGPU_LAYOUT_BUCKETS;
    if (b->d_wslots) f |= LDGPU_LAYOUT_WIDE_KEYS;
    if (b->direct_words) f |= LDGPU_LAYOUT_DIRECT;
    if (b->pack_ok) f |= LDGPU_LAYOUT_PACKS;
    if (b->n_cls && m->blocks.empty()) f |= LDGPU_LAYOUT_CLASSES;
    if (!m->blocks.empty()) f |= LDGPU_LAYOUT_LANG_BLOCKS;
    if (m->general) {  // (a mixed table: its short lengths' model's layout too)
        f = LDGPU_LAYOUT_GENERAL_KEYS;
        if (m->short_m) {
            int32_t fs = 0;
            if (int rc = ldgpu_model_layout(m->short_m, &fs)) return rc;
            f |= fs;
        }
    }
    *flags = f;
    return ok();
}

namespace {
// the gram lengths the kernel scans: maxg, fast_mask, gpack / n_fast; order-
// free modes (3, 4) scan a repeated length once (mult = its multiplicity)
void gram_lists(const ldgpu_model* m, ScoreParams& p, int mode) {
    p.maxg = 0;
    p.n_fast = 0;
    p.fast_mask = 0;
    for (auto& g : p.gpack) g = 0;
    for (auto& c : p.mult) c = 0;
    for (int i = 0; i < m->nG; ++i) {
        p.maxg = std::max(p.maxg, m->G[i]);
        if (!((m->len_mask >> m->G[i]) & 1u)) continue;  // no key of that length: never a hit
        p.fast_mask |= 1u << m->G[i];
        if ((mode == 3 || mode == 4) && p.mult[m->G[i]]++) continue;
        p.gpack[p.n_fast >> 4] |= (uint64_t)m->G[i] << (4 * (p.n_fast & 15));
        ++p.n_fast;
    }
}

// persistent grid: one wave per kScoreWaves documents, at most what is resident
int score_grid(const ldgpu_model* m, int64_t n_docs) {
    const int64_t want = (n_docs + kScoreWaves - 1) / kScoreWaves;
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)m->ctx->cus * m->wg_per_cu));
}

// class mode's second step: the documents class_label left ambiguous (-1)
// listed (amb_compact, their count written on the device) and scored in place
// by an indirect launch of the ordered replay (mode 1, the reference's fold bit
// for bit), which reads that count itself: nothing is read back, so the call
// stays asynchronous on its stream.  The list is stream-ordered scratch of the
// worst case (every document ambiguous).
int class_replay(ldgpu_model* m, const ScoreParams& p4, hipStream_t st) {
    const int64_t n = p4.n_docs;
    int64_t* idx = nullptr;
    HIP_TRY(hipMallocAsync((void**)&idx, sizeof(int64_t) * (size_t)(n + 1), st));
    unsigned long long* d_k = (unsigned long long*)(idx + n);
    hipError_t e = hipMemsetAsync(d_k, 0, sizeof *d_k, st);
    if (e == hipSuccess) e = launch_amb_compact(p4.labels, n, idx, d_k, st);
    if (e == hipSuccess) {
        ScoreParams p1 = p4;
        p1.doc_idx = idx;
        p1.n_docs_dev = d_k;
        p1.n_cls = 0;
        p1.hit_words = 0;
        p1.direct_words = 0;
        gram_lists(m, p1, 1);
        e = launch_score(p1, m->slices, 1, m->lds_filter, score_grid(m, n), st);
    }
    (void)hipFreeAsync(idx, st);
    HIP_TRY(e);
    return LDGPU_OK;
}

int score_launch(ldgpu_model* m, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets, int64_t n_docs,
                 int32_t* d_labels, double* d_scores, int32_t* d_err, hipStream_t st, double* d_best = nullptr,
                 int block = 0, int64_t score_stride = 0) {
    if (n_docs == 0) return LDGPU_OK;
    if (m->general) {
        // mixed table: the short lengths on the LDS-filtered kernels (or, with
        // none, label 0 and zero scores: the reference's result without a
        // hit), then the documents a long length hits rescored exactly
        int64_t* idx = nullptr;
        if (m->n_long > 0) {
            if (m->short_m) {
                if (int rc = score_launch(m->short_m, d_bytes, n_bytes, d_offsets, n_docs, d_labels, d_scores, d_err, st))
                    return rc;
            } else {
                HIP_TRY(hipMemsetAsync(d_labels, 0, sizeof(int32_t) * (size_t)n_docs, st));
                if (d_scores) HIP_TRY(hipMemsetAsync(d_scores, 0, sizeof(double) * (size_t)n_docs * m->L, st));
            }
            HIP_TRY(hipMallocAsync((void**)&idx, sizeof(int64_t) * (size_t)(n_docs + 1), st));
            LongFlagParams f{};
            f.bytes = d_bytes;
            f.offsets = d_offsets;
            f.n_docs = n_docs;
            f.bitmap = m->d_lbits;
            f.lb = m->lbits_log2;
            f.n_long = m->n_long;
            for (int i = 0; i < m->n_long; ++i) f.Glong[i] = m->Glong[i];
            f.max_long = m->max_long;
            f.slots = m->d_gslots;
            f.slot_mask = m->gslot_cap - 1;
            f.slot_shift = (uint32_t)(64 - log2u(m->gslot_cap));
            f.arena = m->d_arena;
            f.koff = m->d_koff;
            f.idx = idx;
            f.n_out = (unsigned long long*)(idx + n_docs);
            hipError_t e = hipMemsetAsync(f.n_out, 0, sizeof(unsigned long long), st);
            if (e == hipSuccess) e = launch_long_flag(f, m->ctx->cus, st);
            if (e != hipSuccess) {
                (void)hipFreeAsync(idx, st);
                HIP_TRY(e);
            }
        }
        GenScoreParams g{};
        g.doc_idx = idx;
        g.n_docs_dev = idx ? (const unsigned long long*)(idx + n_docs) : nullptr;
        g.bytes = d_bytes;
        g.offsets = d_offsets;
        g.n_docs = n_docs;
        g.labels = d_labels;
        g.scores = d_scores;
        g.slots = m->d_gslots;
        g.slot_mask = m->gslot_cap - 1;
        g.slot_shift = (uint32_t)(64 - log2u(m->gslot_cap));
        g.arena = m->d_arena;
        g.koff = m->d_koff;
        g.masks = m->dense ? nullptr : m->d_masks;
        g.vals = m->d_vals;
        g.rows = m->d_rows;
        g.err = d_err;
        g.L = m->L;
        g.nG = m->nG;
        for (int i = 0; i < m->nG; ++i) g.G[i] = m->G[i];
        const int64_t want = (n_docs + kGenWaves - 1) / kGenWaves;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)m->ctx->cus * 8));
        const hipError_t e = launch_general_score(g, grid, st);
        if (idx) (void)hipFreeAsync(idx, st);
        HIP_TRY(e);
        return LDGPU_OK;
    }
    if (!m->blocks.empty()) {
        // one launch per language block (block labels and maxima in stream-
        // ordered scratch), then the first maximum across blocks
        const int nb = (int)m->blocks.size();
        int32_t* lab = nullptr;
        double* best = nullptr;
        HIP_TRY(hipMallocAsync((void**)&lab, sizeof(int32_t) * (size_t)nb * n_docs, st));
        HIP_TRY(hipMallocAsync((void**)&best, sizeof(double) * (size_t)nb * n_docs, st));
        int rc = LDGPU_OK;
        for (int b = 0; b < nb && !rc; ++b)
            rc = score_launch(m->blocks[b], d_bytes, n_bytes, d_offsets, n_docs, lab + (size_t)b * n_docs,
                              d_scores ? d_scores + (size_t)b * kBlockLangs : nullptr, d_err, st,
                              best + (size_t)b * n_docs, b, m->L);
        hipError_t e = rc ? hipSuccess : launch_combine_blocks(n_docs, nb, lab, best, d_labels, st);
        (void)hipFreeAsync(lab, st);
        (void)hipFreeAsync(best, st);
        if (rc) return rc;
        HIP_TRY(e);
        return LDGPU_OK;
    }
    ScoreParams p{};
    p.best = d_best;
    p.block = block;
    p.score_stride = score_stride;
    p.bytes = d_bytes;
    p.n_bytes = n_bytes;
    p.last_dword = n_bytes > 0 ? (n_bytes - 1) >> 2 : 0;
    // documents per staged group: at most 63 (the lanes holding a group's
    // offsets); the kernel takes as many as fit the staging buffer
    p.group = 63;
    const double mean = (double)n_bytes / (double)std::max<int64_t>(n_docs, 1);
    p.offsets = d_offsets;
    p.n_docs = n_docs;
    p.labels = d_labels;
    p.scores = d_scores;
    p.slots = m->d_slots;
    p.buckets = m->d_buckets;
    // cuckoo slots: slot 1 = h >> slot_shift, slot 2 = h & slot_mask; buckets:
    // bucket_index of h's halves over slot_mask = the bucket count
    const uint64_t n_index = m->d_buckets ? m->n_buckets : m->slot_cap;
    p.slot_shift = (uint32_t)(64 - log2u(n_index));
    p.slot_mask = m->d_buckets ? m->n_buckets : n_index - 1;
    p.slot_shift32 = (uint32_t)(32 - log2u(n_index));  // cuckoo slots: slot_hash
    p.wslots = m->d_wslots;
    p.wslot_shift32 = m->d_wslots ? (uint32_t)(32 - log2u(m->wslot_cap)) : 0u;
    p.filter = m->d_filter;
    p.bloom_shift = (uint32_t)(32 - m->filter_log2);
    p.kb_lines = m->kb_lines ? 1 : 0;
    p.kb_chunks = m->kb_chunks ? 1 : 0;
    if (m->kb_chunks) p.bloom_shift += 2;  // chunk index = kb_chunk >> (32 - log2(words / 4))
    p.bloom_words = (uint32_t)((uint64_t)1 << m->filter_log2);
    p.len_mask = m->len_mask;
    p.masks = m->d_masks;
    p.vals = m->d_vals;
    p.rows = m->d_rows;
    p.fold = m->d_fold;
    p.fold_max = kFoldMax;
    p.direct_off = m->direct_off;
    p.direct_words = m->direct_words;  // (order-free modes only: set below)
    p.count_sign = m->count_sign;
    // counts stay below 2^24: c <= windows of a document <= len * n_grams
    p.count_argmax_len = m->count_int_argmax ? ((1 << 24) - 1) / std::max(1, m->nG) : -1;
    // packs of short documents (labels only; the kernel packs documents of
    // maxg..128 bytes)
    p.pack = m->pack_ok && !d_scores && !d_best && mean < 192.0;
    p.err = d_err;
    p.stats = m->d_stats;
    p.L = m->L;
    p.ablate = m->ablate;
    p.nG = m->nG;
    for (int i = 0; i < m->nG; ++i) p.G[i] = m->G[i];
    // class mode: labels only, on a table of at most class_max(S) values
    const bool classes = m->n_cls > 0 && !d_scores && !d_best && m->mode == 1;
    const int mode = classes ? 4 : m->mode;
    if (classes) {
        for (int q = 0; q < 4; ++q) p.cls[q] = m->cls[q];
        p.n_cls = m->n_cls;
        p.hit_words = 64u * (uint32_t)m->slices * (uint32_t)m->n_cls;
    }
    gram_lists(m, p, mode);
    if (mode != 3 && mode != 4) p.direct_words = 0;  // the ordered replay reads no direct tables
    // count mode, labels only: a fast-path document (<= 256 B, so far below
    // count_argmax_len) takes the count argmax (score kernel kFmArgmax)
    if (mode == 3 && p.count_argmax_len >= 256 && !d_scores && !d_best) p.fast_mask |= 1u << 17;
    HIP_TRY(launch_score(p, m->slices, mode, m->lds_filter, score_grid(m, n_docs), st));
    if (classes) return class_replay(m, p, st);
    return LDGPU_OK;
}

// the whole byte range the documents span lies in pinned memory
bool nb_total_pinned(const uint8_t* bytes, const int64_t* offsets, int64_t n_docs) {
    if (offsets[n_docs] <= offsets[0]) return true;
    return is_pinned(bytes + offsets[0]) && is_pinned(bytes + offsets[n_docs] - 1);
}

int check_row_error(ldgpu_model* m, int32_t* d_err, hipStream_t st) {
    int32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, d_err, sizeof err, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (err) {
        int32_t z = 0;
        HIP_TRY(hipMemcpy(d_err, &z, sizeof z, hipMemcpyHostToDevice));
        if (err & 2)
            return fail(LDGPU_EUNSUPPORTED, "a document of %lld bytes or more exceeds the device path's limit",
                        (long long)kMaxDocBytes);
        return fail(LDGPU_EROWLEN, "requirement failed: BLAS.axpy size mismatch (a hit gram's row length != %d)",
                    m->L);
    }
    return LDGPU_OK;
}
}  // namespace

extern "C" int ldgpu_score_device(ldgpu_model* m, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                                  int64_t n_docs, int32_t* d_labels, double* d_scores, void* stream) {
    if (!m) return fail(LDGPU_EINVAL, "model is NULL");
    if (n_docs < 0) return fail(LDGPU_EINVAL, "n_docs < 0");
    if (n_docs > 0 && (!d_offsets || !d_labels || (n_bytes > 0 && !d_bytes)))
        return fail(LDGPU_EINVAL, "device pointer is NULL");
    if (((uintptr_t)d_bytes & 3) != 0) return fail(LDGPU_EINVAL, "d_bytes must be 4-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipSetDevice(m->ctx->device));
    if (int rc = score_launch(m, d_bytes, n_bytes, d_offsets, n_docs, d_labels, d_scores, m->d_err, st)) return rc;
    if (m->has_bad) {
        if (int rc = check_row_error(m, m->d_err, st)) return rc;
    }
    return ok();
}

namespace {
int score_host(ldgpu_model* m, ScorePipe* pp, const uint8_t* bytes, const int64_t* offsets, int64_t n_docs,
               int32_t* out_labels, double* out_scores);
}  // namespace

// Thread-safe and concurrent: each call scores on a pipeline (two streams,
// pinned staging, its own error word) taken from the context's pool.
extern "C" int ldgpu_score(ldgpu_model* m, const uint8_t* bytes, const int64_t* offsets, int64_t n_docs,
                           int32_t* out_labels, double* out_scores) {
    if (!m) return fail(LDGPU_EINVAL, "model is NULL");
    if (int rc = check_offsets(offsets, n_docs)) return rc;
    if (n_docs == 0) return ok();
    if (!out_labels) return fail(LDGPU_EINVAL, "out_labels is NULL");
    if (!bytes && offsets[n_docs] > offsets[0]) return fail(LDGPU_EINVAL, "bytes is NULL");
    for (int64_t d = 0; d < n_docs; ++d)
        if (offsets[d + 1] - offsets[d] >= kMaxDocBytes)
            return fail(LDGPU_EUNSUPPORTED, "document %lld has %lld bytes: the device path's limit is %lld",
                        (long long)d, (long long)(offsets[d + 1] - offsets[d]), (long long)kMaxDocBytes - 1);
    ldgpu_ctx* c = m->ctx;
    HIP_TRY(hipSetDevice(c->device));
    ScorePipe* pp = pipe_acquire(c);
    if (!pp) return LDGPU_EDEVICE;
    const int rc = score_host(m, pp, bytes, offsets, n_docs, out_labels, out_scores);
    pipe_release(c, pp);
    if (rc) return rc;
    return ok();
}

namespace {
int score_host(ldgpu_model* m, ScorePipe* pp, const uint8_t* bytes, const int64_t* offsets, int64_t n_docs,
               int32_t* out_labels, double* out_scores) {
    // Two-stage pipeline over chunks of documents, one stream per stage: while
    // the GPU copies and scores chunk i, the host stages chunk i + 1 into the
    // other stage's pinned buffers (a caller buffer already in pinned memory is
    // copied from directly) and hands back the labels of chunk i - 1.
    const int64_t kChunkBytes = 64ll << 20, kChunkDocs = 1ll << 20;
    const bool pinned_in = nb_total_pinned(bytes, offsets, n_docs);
    const bool pinned_out = is_pinned(out_labels) && (!out_scores || is_pinned(out_scores));
    auto retire = [&](ScoreStage& st) -> int {
        if (!st.busy) return LDGPU_OK;
        HIP_TRY(hipEventSynchronize(st.done));
        st.busy = false;
        if (!pinned_out) {
            memcpy(out_labels + st.d0, st.h_labels.p, sizeof(int32_t) * st.nd);
            if (out_scores) par_memcpy(out_scores + st.d0 * m->L, st.h_scores.p, sizeof(double) * st.nd * m->L);
        }
        return LDGPU_OK;
    };
    // one chunk's copies and launch on stage st; an error returns without
    // leaving the loop's drain behind (the caller breaks, then drains)
    auto issue = [&](ScoreStage& st, int64_t d0, int64_t d1) -> int {
        const int64_t nd = d1 - d0, b0 = offsets[d0], nb = offsets[d1] - b0;
        HIP_TRY(st.bytes.ensure((size_t)nb + 16));
        HIP_TRY(st.offsets.ensure(sizeof(int64_t) * (nd + 1)));
        HIP_TRY(st.labels.ensure(sizeof(int32_t) * nd));
        if (out_scores) HIP_TRY(st.scores.ensure(sizeof(double) * nd * m->L));
        HIP_TRY(st.h_offsets.ensure(sizeof(int64_t) * (nd + 1)));
        int64_t* ho = (int64_t*)st.h_offsets.p;
        for (int64_t i = 0; i <= nd; ++i) ho[i] = offsets[d0 + i] - b0;
        const uint8_t* src = bytes + b0;
        if (nb && !pinned_in) {
            HIP_TRY(st.h_bytes.ensure((size_t)nb));
            par_memcpy(st.h_bytes.p, src, (size_t)nb);
            src = (const uint8_t*)st.h_bytes.p;
        }
        if (nb) HIP_TRY(hipMemcpyAsync(st.bytes.p, src, nb, hipMemcpyHostToDevice, st.stream));
        HIP_TRY(hipMemcpyAsync(st.offsets.p, ho, sizeof(int64_t) * (nd + 1), hipMemcpyHostToDevice, st.stream));
        // (class mode included: its replay of ambiguous documents reads no
        // count back, so the staging of the next chunk still overlaps)
        if (int r = score_launch(m, (const uint8_t*)st.bytes.p, nb, (const int64_t*)st.offsets.p, nd,
                                 (int32_t*)st.labels.p, out_scores ? (double*)st.scores.p : nullptr, pp->d_err,
                                 st.stream))
            return r;
        int32_t* lab_dst = out_labels + d0;
        double* sc_dst = out_scores ? out_scores + d0 * m->L : nullptr;
        if (!pinned_out) {
            HIP_TRY(st.h_labels.ensure(sizeof(int32_t) * nd));
            lab_dst = (int32_t*)st.h_labels.p;
            if (out_scores) {
                HIP_TRY(st.h_scores.ensure(sizeof(double) * nd * m->L));
                sc_dst = (double*)st.h_scores.p;
            }
        }
        HIP_TRY(hipMemcpyAsync(lab_dst, st.labels.p, sizeof(int32_t) * nd, hipMemcpyDeviceToHost, st.stream));
        if (out_scores)
            HIP_TRY(hipMemcpyAsync(sc_dst, st.scores.p, sizeof(double) * nd * m->L, hipMemcpyDeviceToHost,
                                   st.stream));
        HIP_TRY(hipEventRecord(st.done, st.stream));
        st.d0 = d0;
        st.nd = nd;
        st.busy = true;
        return LDGPU_OK;
    };
    // diagnostics build: fail after issuing this many chunks (error-path tests)
    const char* fail_at = diag_env("LDGPU_FAIL_CHUNK");
    int64_t d0 = 0;
    int k = 0;
    int rc = LDGPU_OK;
    while (d0 < n_docs && rc == LDGPU_OK) {
        int64_t d1 = d0 + 1;
        while (d1 < n_docs && d1 - d0 < kChunkDocs && offsets[d1 + 1] - offsets[d0] <= kChunkBytes) ++d1;
        ScoreStage& st = pp->stage[k & 1];
        if ((rc = retire(st))) break;
        if (fail_at && k == atoi(fail_at)) {
            rc = fail(LDGPU_EDEVICE, "injected failure at chunk %d (LDGPU_FAIL_CHUNK)", k);
            break;
        }
        if ((rc = issue(st, d0, d1))) break;
        d0 = d1;
        ++k;
    }
    // drain: every copy this call queued (also a half-issued chunk's, after an
    // error) completes before the call returns, in chunk order; a stage is
    // idle when the pipeline goes back to the pool
    for (auto& st : pp->stage) {
        const hipError_t e = hipStreamSynchronize(st.stream);
        if (!rc && e != hipSuccess) rc = fail(LDGPU_EDEVICE, "score pipeline: %s", hipGetErrorString(e));
    }
    for (int i = 0; i < 2; ++i) {
        ScoreStage& st = pp->stage[(k + i) & 1];
        if (rc) {
            st.busy = false;  // the call failed: its outputs are undefined
            continue;
        }
        rc = retire(st);
    }
    if (rc) {
        (void)hipMemset(pp->d_err, 0, sizeof(int32_t));  // no stale row error for the pipeline's next call
        return rc;
    }
    if (m->has_bad) {
        for (auto& st : pp->stage) HIP_TRY(hipStreamSynchronize(st.stream));
        if (int r = check_row_error(m, pp->d_err, pp->stage[0].stream)) return r;
    }
    return LDGPU_OK;
}
}  // namespace

// ---------------------------------------------------------------------- FIT
struct ldgpu_counts {
    ldgpu_ctx* ctx = nullptr;
    int32_t L = 0, nG = 0;
    int32_t G[kMaxGramLengths] = {};
    // gramLengths split: one-word lengths (1..7: the count kernels) and wide
    // lengths (8..15: wide_count_kernel), each in the caller's order
    int32_t nGn = 0, Gn[kMaxGramLengths] = {};
    int32_t nGw = 0, Gw[kMaxGramLengths] = {};
    uint64_t cap = 0;
    uint64_t* d_keys = nullptr;
    unsigned long long* d_counts = nullptr;  // [cap][L] (dense tables: T1 of the count calls)
    unsigned long long* d_size = nullptr;
    // The final table T of a count table is sparse (ldgpu_fit.h CountParams):
    // the grams in d_keys with their language counts d_kcnt[cap] (the pairs
    // each has), the counts in a table of (gram slot, language) pairs -- the
    // reduceGrams rows (LanguageDetector.scala:57-65), ~1.3 per gram on the fit
    // corpora, where a dense row of L counters per gram took 1.6 KB at L = 200.
    bool sparse = false;
    uint32_t* d_kcnt = nullptr;
    uint64_t pcap = 0, psize = 0;
    uint64_t* d_pkeys = nullptr;
    unsigned long long* d_pcounts = nullptr;
    unsigned long long* d_psize = nullptr;
    uint64_t* d_ovf_keys = nullptr;
    int32_t* d_ovf_lang = nullptr;
    unsigned long long* d_ovf_cnt = nullptr;
    unsigned int* d_ovf_n = nullptr;
    // second overflow list (allocated at the first overflow): re-inserting a
    // list after a grow may overflow again, into this one
    uint64_t* d_ovf2_keys = nullptr;
    int32_t* d_ovf2_lang = nullptr;
    unsigned long long* d_ovf2_cnt = nullptr;
    unsigned int* d_ovf2_n = nullptr;
    uint32_t ovf2_cap = 0;
    uint32_t ovf_cap = 1u << 20;  // windows per sub-launch; grown per call up to kOvfMax
    uint64_t size = 0;
    // FIT v3 (ldgpu_fit.hip): K = words per record (ldgpu_internal.h); K = 1
    // records are ((sentinel << lb | lang) << cb | count)
    bool v3 = true;
    int K = 1;
    uint32_t lb = 0, cb = 0;
    int64_t batch_recs = 0;     // kBatchRecords / K (diagnostics: LDGPU_FIT_BATCH_WINDOWS)
    ldgpu_counts* pend = nullptr; // FIT v4: T1, the table of maximal windows of a count call
    int64_t pend_hint = 0;      // T1's keys in the last call (sizes the next one)
    double new_per_entry = 1.0; // new keys per merged entry in the last batch (projected growth)
    // FIT v5 (count_launch_sorted): new grams / pairs per run entry of the last
    // insert into T (projected growth of the next)
    double run_new_grams = 1.0, run_new_pairs = 1.0;
    ldgpu_comm* comm = nullptr; // set by ldgpu_counts_merge: the table is this rank's owned shard
    // grams of 8..15 bytes: a two-word-key table of their own (ldgpu_fit.hip)
    uint64_t wcap = 0, wsize = 0;
    bool merged_wide = false;   // merged table: some rank held wide grams (the same on every rank)
    uint64_t* d_wlo = nullptr;
    uint64_t* d_whi = nullptr;
    unsigned long long* d_wcounts = nullptr;
    unsigned long long* d_wsize = nullptr;
    unsigned int* d_wfull = nullptr;
    // grams longer than kMaxWideGram (ldgpu_long.hip): gram slots with a key
    // arena and a pair table, as the sparse T; Gall = the
    // caller's gram lengths, G (above) its lengths <= 15 (FIT v4), Gl the
    // longer ones
    int32_t nGall = 0, Gall[kMaxGramLengths] = {};
    int32_t nGl = 0, Gl[kMaxGramLengths] = {};
    uint64_t lcap = 0, lsize = 0, lpcap = 0, lpsize = 0, larena_cap = 0, larena_n = 0;
    LongSlot* d_lslots = nullptr;
    uint8_t* d_larena = nullptr;
    uint64_t* d_lpkeys = nullptr;
    unsigned long long* d_lpcounts = nullptr;
    unsigned long long* d_lctr = nullptr;  // [0] grams, [1] pairs, [2] arena bytes, [3] full flag
    // the grams of 8 or more bytes (wide and long) in (length, bytes) order, as
    // of the last counts_pull: key kWideTag << 56 | r of a pulled key list is
    // ext_sorted[r]
    std::vector<std::string> ext_sorted;
    // cached fit table (ldgpu_fit_table_size -> _export)
    bool tbl_valid = false;
    // sparse host copy of the table for ranged exports (ldgpu_counts_export_sparse),
    // valid until the counts change: keys (one-word or wide stand-ins, see
    // counts_pull) in (length, bytes) order, their nonzero (language, count) pairs
    bool sp_valid = false;
    std::vector<uint64_t> sp_keys;
    std::vector<int64_t> sp_koff;   // key byte offsets [n + 1]
    std::vector<int64_t> sp_poff;   // pair offsets [n + 1]
    std::vector<int32_t> sp_lang;
    std::vector<int64_t> sp_cnt;
    std::vector<uint8_t> tbl_bytes;
    std::vector<int64_t> tbl_off;
    std::vector<uint64_t> tbl_masks;  // [rows][S] presence masks of the chosen grams
    std::vector<double> tbl_vals;     // [rows] log(1 + 1/k): the value of every nonzero entry
    // single-rank device build: the table is in ctx->h_tbl (keys [rows],
    // masks [rows][S], k [rows]) instead of the vectors above
    bool tbl_pin = false;
    int64_t tbl_rows = 0, tbl_kb = 0;
};

namespace {
// bytes per gram slot besides the key: dense rows of L u64 counters, or the
// sparse table's u32 language count
uint64_t row_bytes(const ldgpu_counts* c) { return c->sparse ? 4ull : 8ull * (uint64_t)c->L; }

CountParams count_params(const ldgpu_counts* c) {
    CountParams p{};
    p.keys = c->d_keys;
    p.counts = c->d_counts;
    p.shift = (uint32_t)(64 - log2u(c->cap));
    p.mask = c->cap - 1;
    p.size = c->d_size;
    p.ovf_keys = c->d_ovf_keys;
    p.ovf_lang = c->d_ovf_lang;
    p.ovf_cnt = c->d_ovf_cnt;
    p.ovf_n = c->d_ovf_n;
    p.ovf_cap = c->ovf_cap;
    p.max_probe = kMaxProbe;
    p.L = c->L;
    p.nG = c->nGn;
    for (int i = 0; i < c->nGn; ++i) p.G[i] = c->Gn[i];
    if (c->sparse) {
        p.kcnt = c->d_kcnt;
        p.pkeys = c->d_pkeys;
        p.pcounts = c->d_pcounts;
        p.pshift = (uint32_t)(64 - log2u(c->pcap));
        p.pmask = c->pcap - 1;
        p.psize = c->d_psize;
        p.pinter = 1;  // alloc_pairs: keys and counts interleaved
    }
    return p;
}

// a pair table for stats_kernel (occupied pairs and the sum of their counts);
// inter: keys and counts interleaved (T) or separate (the long-gram table)
CountParams pair_view_of(uint64_t* pkeys, unsigned long long* pcounts, uint32_t inter) {
    CountParams p{};
    p.pkeys = pkeys;
    p.pcounts = pcounts;
    p.pinter = inter;
    p.L = 1;
    return p;
}

CountParams pair_view(const ldgpu_counts* c) { return pair_view_of(c->d_pkeys, c->d_pcounts, 1); }

// T's pair table (alloc_pairs): one block of 16-B entries, pcounts = pkeys + 1
void free_pairs(ldgpu_ctx* ctx, uint64_t* pkeys, uint64_t pcap) { cache_free(ctx, pkeys, pcap * 16u); }

void counts_free(ldgpu_counts* c) {
    if (!c) return;
    if (c->ctx && c->ctx->h_tbl_owner == c) c->ctx->h_tbl_owner = nullptr;
    if (c->pend) counts_free(c->pend);
    for (void* p : {(void*)c->d_wlo, (void*)c->d_whi, (void*)c->d_wcounts, (void*)c->d_wsize, (void*)c->d_wfull,
                    (void*)c->d_lslots, (void*)c->d_larena, (void*)c->d_lpkeys,
                    (void*)c->d_lpcounts, (void*)c->d_lctr})
        if (p) (void)hipFree(p);
    if (c->ctx) {
        (void)hipSetDevice(c->ctx->device);
        // table and overflow lists back to the context's cache (no kernel
        // uses them once the stream drained)
        (void)hipStreamSynchronize(c->ctx->stream);
        cache_free(c->ctx, c->d_keys, c->cap * sizeof(uint64_t));
        cache_free(c->ctx, c->d_counts, c->cap * (size_t)c->L * sizeof(unsigned long long));
        cache_free(c->ctx, c->d_kcnt, c->cap * sizeof(uint32_t));
        free_pairs(c->ctx, c->d_pkeys, c->pcap);
        cache_free(c->ctx, c->d_ovf_keys, sizeof(uint64_t) * c->ovf_cap);
        cache_free(c->ctx, c->d_ovf_lang, sizeof(int32_t) * c->ovf_cap);
        cache_free(c->ctx, c->d_ovf_cnt, sizeof(unsigned long long) * c->ovf_cap);
    } else {
        for (void* p : {(void*)c->d_keys, (void*)c->d_counts, (void*)c->d_kcnt, (void*)c->d_pkeys,
                        (void*)c->d_ovf_keys, (void*)c->d_ovf_lang, (void*)c->d_ovf_cnt})
            if (p) (void)hipFree(p);
    }
    for (void* p : {(void*)c->d_size, (void*)c->d_psize, (void*)c->d_ovf_n, (void*)c->d_ovf2_keys,
                    (void*)c->d_ovf2_lang, (void*)c->d_ovf2_cnt, (void*)c->d_ovf2_n})
        if (p) (void)hipFree(p);
    delete c;
}

// a gram table of cap slots: keys and rows of row_bytes(c) (dense counters,
// or the sparse table's language counts), zeroed
int alloc_table(ldgpu_counts* c, uint64_t cap, uint64_t** keys, void** rows) {
    const size_t rb = cap * (size_t)row_bytes(c);
    HIP_TRY(cache_alloc(c->ctx, (void**)keys, cap * sizeof(uint64_t)));
    hipError_t e = cache_alloc(c->ctx, (void**)rows, rb);
    if (e != hipSuccess) {
        cache_free(c->ctx, *keys, cap * sizeof(uint64_t));
        *keys = nullptr;
        return fail(LDGPU_ENOMEM, "count table of %llu slots: %s", (unsigned long long)cap, hipGetErrorString(e));
    }
    HIP_TRY(hipMemsetAsync(*keys, 0, cap * sizeof(uint64_t), c->ctx->stream));
    HIP_TRY(hipMemsetAsync(*rows, 0, rb, c->ctx->stream));
    return LDGPU_OK;
}

// the sparse table's pair table of pcap slots, zeroed: 16-B entries {key,
// count} (CountParams::pinter), so a pair insert claims its key and adds its
// count in one 64-B line
int alloc_pairs(ldgpu_counts* c, uint64_t pcap, uint64_t** pkeys, unsigned long long** pcounts) {
    hipError_t e = cache_alloc(c->ctx, (void**)pkeys, pcap * 16u);
    if (e != hipSuccess) {
        *pkeys = nullptr;
        *pcounts = nullptr;
        return fail(LDGPU_ENOMEM, "pair table of %llu slots: %s", (unsigned long long)pcap, hipGetErrorString(e));
    }
    *pcounts = reinterpret_cast<unsigned long long*>(*pkeys) + 1;
    HIP_TRY(hipMemsetAsync(*pkeys, 0, pcap * 16u, c->ctx->stream));
    return LDGPU_OK;
}

// the sparse table's pairs into a fresh pair table of new_pcap slots, their
// gram slots through remap (a grown gram table) or kept (remap null)
int rebuild_pairs(ldgpu_counts* c, uint64_t new_pcap, const uint64_t* remap) {
    uint64_t* nk = nullptr;
    unsigned long long* nc = nullptr;
    if (int rc = alloc_pairs(c, new_pcap, &nk, &nc)) return rc;
    ldgpu_counts tmp;
    tmp.sparse = true;
    tmp.cap = c->cap;
    tmp.pcap = new_pcap;
    tmp.d_pkeys = nk;
    tmp.d_pcounts = nc;
    HIP_TRY(launch_pair_rehash(count_params(c), count_params(&tmp), c->pcap, remap, c->ctx->stream));
    HIP_TRY(hipStreamSynchronize(c->ctx->stream));
    free_pairs(c->ctx, c->d_pkeys, c->pcap);
    c->d_pkeys = nk;
    c->d_pcounts = nc;
    c->pcap = new_pcap;
    return LDGPU_OK;
}

// grow to new_cap (power of two) by rehashing on the device (the sparse
// table: its grams with their masks, then its pairs re-keyed by the grams'
// new slots)
int grow(ldgpu_counts* c, uint64_t new_cap) {
    if (new_cap <= c->cap) return LDGPU_OK;
    PhaseTrace tr("grow grams", c->cap, new_cap, c->ctx->stream);
    uint64_t* nk = nullptr;
    void* nr = nullptr;
    if (int rc = alloc_table(c, new_cap, &nk, &nr)) return rc;
    CountParams from = count_params(c);
    ldgpu_counts tmp;
    tmp.L = c->L;
    tmp.sparse = c->sparse;
    tmp.cap = new_cap;
    tmp.d_keys = nk;
    if (c->sparse) {
        // The new gram table, the slot remap and the new pair table are all
        // allocated and filled before the old ones are released: a failed
        // grow leaves the table as it was (callers may go on without it).
        tmp.d_kcnt = static_cast<uint32_t*>(nr);
        tmp.pcap = c->pcap;
        uint64_t* remap = nullptr;
        hipError_t e = cache_alloc(c->ctx, (void**)&remap, c->cap * sizeof(uint64_t));
        int rc = e == hipSuccess ? alloc_pairs(c, c->pcap, &tmp.d_pkeys, &tmp.d_pcounts) : LDGPU_ENOMEM;
        if (e == hipSuccess && !rc) e = launch_sparse_rehash(from, count_params(&tmp), c->cap, remap, c->ctx->stream);
        if (e == hipSuccess && !rc)
            e = launch_pair_rehash(from, count_params(&tmp), c->pcap, remap, c->ctx->stream);
        if (e == hipSuccess && !rc) e = hipStreamSynchronize(c->ctx->stream);
        if (e != hipSuccess || rc) {
            (void)hipGetLastError();
            if (remap) cache_free(c->ctx, remap, c->cap * sizeof(uint64_t));
            if (tmp.d_pkeys) free_pairs(c->ctx, tmp.d_pkeys, c->pcap);
            cache_free(c->ctx, nk, new_cap * sizeof(uint64_t));
            cache_free(c->ctx, nr, new_cap * sizeof(uint32_t));
            tmp.d_pkeys = nullptr;
            tmp.d_pcounts = nullptr;
            return fail(LDGPU_ENOMEM, "count table grow to %llu slots: %s", (unsigned long long)new_cap,
                        e != hipSuccess ? hipGetErrorString(e) : "pair table allocation failed");
        }
        cache_free(c->ctx, remap, c->cap * sizeof(uint64_t));
        cache_free(c->ctx, c->d_keys, c->cap * sizeof(uint64_t));
        cache_free(c->ctx, c->d_kcnt, c->cap * sizeof(uint32_t));
        free_pairs(c->ctx, c->d_pkeys, c->pcap);
        c->d_keys = nk;
        c->d_kcnt = tmp.d_kcnt;
        c->d_pkeys = tmp.d_pkeys;
        c->d_pcounts = tmp.d_pcounts;
        c->cap = new_cap;
        tmp.d_pkeys = nullptr;
        tmp.d_pcounts = nullptr;
        return LDGPU_OK;
    }
    tmp.d_counts = static_cast<unsigned long long*>(nr);
    CountParams to = count_params(&tmp);
    HIP_TRY(launch_rehash(from, to, c->cap, c->ctx->stream));
    HIP_TRY(hipStreamSynchronize(c->ctx->stream));
    cache_free(c->ctx, c->d_keys, c->cap * sizeof(uint64_t));
    cache_free(c->ctx, c->d_counts, c->cap * (size_t)c->L * sizeof(unsigned long long));
    c->d_keys = nk;
    c->d_counts = static_cast<unsigned long long*>(nr);
    c->cap = new_cap;
    return LDGPU_OK;
}

// the sparse table's pair table to new_pcap slots
int pgrow(ldgpu_counts* c, uint64_t new_pcap) {
    if (!c->sparse || new_pcap <= c->pcap) return LDGPU_OK;
    PhaseTrace tr("grow pairs", c->pcap, new_pcap, c->ctx->stream);
    return rebuild_pairs(c, new_pcap, nullptr);
}

// Load a table may reach before it doubles: 1/2, or 0.8 once the doubled
// table would pass kBigTableBytes -- the device must hold the old and the new
// table during a rehash, next to the others of the fit.  A dense slot holds a
// row of L counters (1.6 KB at L = 200: T1 of a K = 3 fit); the sparse T's
// gram slots are 12 B and its pairs 16 B, but a 1 GB fit at L = 200 holds
// ~1.4G grams and ~1.7G pairs (2^31 slots each at load 0.8: 26 + 34 GB;
// 2^32 at load 1/2 would take twice that, and three times during the grow).
// (A rare insert that meets a linear-probe cluster longer than kMaxProbe goes
// to the overflow list and is re-inserted by the host.)
constexpr uint64_t kBigTableBytes = 48ull << 30;

double load_limit(uint64_t cap, uint64_t slot_bytes) { return 2 * cap * slot_bytes >= kBigTableBytes ? 0.8 : 0.5; }

double max_load(const ldgpu_counts* c) { return load_limit(c->cap, 8ull + row_bytes(c)); }

// the sparse table's pair table (16-B slots)
double pair_load(const ldgpu_counts* c) { return load_limit(c->pcap, 16ull); }

// the smallest power-of-two table of slot_bytes slots that holds `need` keys
// within its load limit
uint64_t cap_for(double need, uint64_t slot_bytes) {
    uint64_t cap = 1ull << 12;
    while (need > load_limit(cap, slot_bytes) * (double)cap) cap <<= 1;
    return cap;
}

// room for `grams` more grams and `pairs` more pairs within the load limits
// (grow / pgrow to the next fitting power of two)
int reserve(ldgpu_counts* c, uint64_t grams, uint64_t pairs) {
    if ((double)(c->size + grams) > max_load(c) * (double)c->cap) {
        if (int rc = grow(c, cap_for((double)(c->size + grams) + 16, 8ull + row_bytes(c)))) return rc;
    }
    if (c->sparse && (double)(c->psize + pairs) > pair_load(c) * (double)c->pcap) {
        if (int rc = pgrow(c, cap_for((double)(c->psize + pairs) + 16, 16ull))) return rc;
    }
    return LDGPU_OK;
}

// after a batch: read size / overflow, grow, re-insert overflow entries
// (may_grow = false: a table being scanned -- the derive's T1 -- keeps its
// slots: entries are re-inserted in place; the caller keeps it within 0.9
// load)
int after_batch(ldgpu_counts* c, bool may_grow = true) {
    unsigned long long size = 0, psize = 0;
    unsigned int novf = 0;
    HIP_TRY(hipMemcpyAsync(&size, c->d_size, sizeof size, hipMemcpyDeviceToHost, c->ctx->stream));
    if (c->sparse) HIP_TRY(hipMemcpyAsync(&psize, c->d_psize, sizeof psize, hipMemcpyDeviceToHost, c->ctx->stream));
    HIP_TRY(hipMemcpyAsync(&novf, c->d_ovf_n, sizeof novf, hipMemcpyDeviceToHost, c->ctx->stream));
    HIP_TRY(hipStreamSynchronize(c->ctx->stream));
    if (novf > c->ovf_cap)  // cannot happen: sub-launches hold <= ovf_cap windows
        return fail(LDGPU_ENOMEM, "count table overflow (%u entries lost)", novf);
    c->size = size;
    c->psize = psize;
    c->tbl_valid = false;
    c->sp_valid = false;
    if (novf == 0) {
        while (may_grow && (double)c->size > max_load(c) * (double)c->cap) {  // past the load limit: double
            if (int rc = grow(c, 2 * c->cap)) return rc;
        }
        while (may_grow && c->sparse && (double)c->psize > pair_load(c) * (double)c->pcap) {
            if (int rc = pgrow(c, 2 * c->pcap)) return rc;
        }
        return LDGPU_OK;
    }
    // Entries whose key found no slot are on the overflow list: grow, then
    // re-insert them (into the second list when they overflow again) until
    // none is left.  The list may count windows, duplicates included (count
    // kernel), or distinct records (FIT v2 merge), so it sizes the first grow
    // only within 8x the table; later rounds double.  The second list needs
    // room for at most this list's entries.
    if (!c->d_ovf2_keys || c->ovf2_cap < novf) {
        HIP_TRY(hipStreamSynchronize(c->ctx->stream));
        for (void* q : {(void*)c->d_ovf2_keys, (void*)c->d_ovf2_lang, (void*)c->d_ovf2_cnt, (void*)c->d_ovf2_n})
            if (q) (void)hipFree(q);
        c->d_ovf2_keys = nullptr;
        c->d_ovf2_lang = nullptr;
        c->d_ovf2_cnt = nullptr;
        c->d_ovf2_n = nullptr;
        c->ovf2_cap = 0;
        hipError_t e = hipMalloc((void**)&c->d_ovf2_keys, sizeof(uint64_t) * novf);
        if (e == hipSuccess) e = hipMalloc((void**)&c->d_ovf2_lang, sizeof(int32_t) * novf);
        if (e == hipSuccess) e = hipMalloc((void**)&c->d_ovf2_cnt, sizeof(unsigned long long) * novf);
        if (e == hipSuccess) e = hipMalloc((void**)&c->d_ovf2_n, sizeof(unsigned int));
        if (e != hipSuccess) return fail(LDGPU_ENOMEM, "overflow list: %s", hipGetErrorString(e));
        c->ovf2_cap = novf;
    }
    uint64_t* src_k = c->d_ovf_keys;
    int32_t* src_l = c->d_ovf_lang;
    unsigned long long* src_c = c->d_ovf_cnt;
    uint64_t* dst_k = c->d_ovf2_keys;
    int32_t* dst_l = c->d_ovf2_lang;
    unsigned long long* dst_c = c->d_ovf2_cnt;
    unsigned int* dst_n = c->d_ovf2_n;
    unsigned int* src_n = c->d_ovf_n;
    uint32_t dst_cap = c->ovf2_cap, src_cap = c->ovf_cap;
    // While the table, with every overflow entry a new key, stays within 0.9
    // load, the entries are re-inserted in place with a long probe limit
    // (kReinsertProbe: an overflow is a long linear-probe cluster, not a full
    // table); otherwise the table grows to the load limit first.  The list may
    // count windows, duplicates included (legacy count kernel), so a grow is
    // sized within 8x the table.  (The sparse table: its gram and pair tables
    // alike.)
    auto target_of = [&](uint64_t sz, uint64_t cap, double load) {
        if (!may_grow || (double)(sz + novf) <= 0.9 * (double)cap) return cap;
        const uint64_t t = next_pow2((uint64_t)((double)(sz + novf) / load) + 16);
        return std::max<uint64_t>(std::min<uint64_t>(t, 8 * cap), 2 * cap);
    };
    uint64_t target = target_of(size, c->cap, max_load(c));
    uint64_t ptarget = c->sparse ? target_of(psize, c->pcap, pair_load(c)) : 0;
    for (unsigned int n = novf; n > 0;) {
        if (int rc = grow(c, target)) return rc;
        if (int rc = pgrow(c, ptarget)) return rc;
        CountParams p = count_params(c);
        p.max_probe = kReinsertProbe;
        p.ovf_keys = dst_k;
        p.ovf_lang = dst_l;
        p.ovf_cnt = dst_c;
        p.ovf_n = dst_n;
        p.ovf_cap = dst_cap;
        HIP_TRY(hipMemsetAsync(dst_n, 0, sizeof(unsigned int), c->ctx->stream));
        HIP_TRY(launch_counts_add(p, src_k, nullptr, src_l, src_c, n, c->ctx->stream));
        unsigned int again = 0;
        HIP_TRY(hipMemcpyAsync(&again, dst_n, sizeof again, hipMemcpyDeviceToHost, c->ctx->stream));
        HIP_TRY(hipMemcpyAsync(&size, c->d_size, sizeof size, hipMemcpyDeviceToHost, c->ctx->stream));
        if (c->sparse)
            HIP_TRY(hipMemcpyAsync(&psize, c->d_psize, sizeof psize, hipMemcpyDeviceToHost, c->ctx->stream));
        HIP_TRY(hipStreamSynchronize(c->ctx->stream));
        c->size = size;
        c->psize = psize;
        n = again;
        std::swap(src_k, dst_k);
        std::swap(src_l, dst_l);
        std::swap(src_c, dst_c);
        std::swap(src_n, dst_n);
        std::swap(src_cap, dst_cap);
        if (!may_grow && n > 0) return fail(LDGPU_EDEVICE, "count table: %u entries found no slot", n);
        target = 2 * c->cap;
        ptarget = 2 * c->pcap;
    }
    return LDGPU_OK;
}

// windows the count kernel visits for a document of len bytes
int64_t doc_windows(const ldgpu_counts* c, int64_t len) {
    int64_t w = 0;
    for (int i = 0; i < c->nGn; ++i) w += n_windows(len, c->Gn[i]);
    return w;
}

// Sub-launches hold <= ovf_cap windows (so the overflow list can never lose an
// entry), and one launch must carry enough documents to fill the chip: one
// wave per document, 2 x kCountWaves waves per CU => ~8k documents of 1-7 KB
// = ~1.6e8 windows at grams 1..5.  The list (12 B per window) is grown to the
// call's window count, capped at kOvfMax (1.5 GiB of HBM).
constexpr uint32_t kOvfMax = 1u << 27;

int ensure_ovf(ldgpu_counts* c, int64_t windows) {
    const uint64_t want = std::min<uint64_t>(kOvfMax, next_pow2((uint64_t)std::max<int64_t>(windows, 1)));
    if (want <= c->ovf_cap && c->d_ovf_keys && c->d_ovf_lang && c->d_ovf_cnt) return LDGPU_OK;
    HIP_TRY(hipStreamSynchronize(c->ctx->stream));
    auto drop = [&] {
        cache_free(c->ctx, c->d_ovf_keys, sizeof(uint64_t) * c->ovf_cap);
        cache_free(c->ctx, c->d_ovf_lang, sizeof(int32_t) * c->ovf_cap);
        cache_free(c->ctx, c->d_ovf_cnt, sizeof(unsigned long long) * c->ovf_cap);
        c->d_ovf_keys = nullptr;
        c->d_ovf_lang = nullptr;
        c->d_ovf_cnt = nullptr;
        c->ovf_cap = 0;
    };
    auto take = [&](uint64_t n) {
        hipError_t e = cache_alloc(c->ctx, (void**)&c->d_ovf_keys, sizeof(uint64_t) * n);
        if (e == hipSuccess) e = cache_alloc(c->ctx, (void**)&c->d_ovf_lang, sizeof(int32_t) * n);
        if (e == hipSuccess) e = cache_alloc(c->ctx, (void**)&c->d_ovf_cnt, sizeof(unsigned long long) * n);
        if (e == hipSuccess) c->ovf_cap = (uint32_t)n;
        else drop();
        return e;
    };
    drop();
    // fall back to the smallest list that still makes progress
    hipError_t e = take(std::max<uint64_t>(want, 1u << 20));
    if (e != hipSuccess) e = take(1u << 20);
    if (e != hipSuccess) return fail(LDGPU_ENOMEM, "overflow list: %s", hipGetErrorString(e));
    return LDGPU_OK;
}

// ---- grams of 8..15 bytes (wide_count_kernel, ldgpu_fit.hip)
WideCountParams wide_params(const ldgpu_counts* c) {
    WideCountParams p{};
    p.klo = c->d_wlo;
    p.khi = c->d_whi;
    p.counts = c->d_wcounts;
    p.shift = c->wcap ? (uint32_t)(64 - log2u(c->wcap)) : 63u;
    p.mask = c->wcap ? c->wcap - 1 : 0;
    p.size = c->d_wsize;
    p.full = c->d_wfull;
    p.L = c->L;
    p.nG = c->nGw;
    for (int i = 0; i < c->nGw; ++i) p.G[i] = c->Gw[i];
    p.narrow = count_params(c);
    return p;
}

// room for `extra` more wide keys within the load limit (1/2; 0.8 for a big
// table, as load_limit -- an insert's probe always ends, the table never
// fills): allocate or grow (device rehash) the wide table, to 4x the keys (a
// big table: to load <= 0.7)
int wide_ensure(ldgpu_counts* c, uint64_t extra) {
    hipStream_t st = c->ctx->stream;
    if (!c->d_wsize) {
        HIP_TRY(hipMalloc((void**)&c->d_wsize, sizeof(unsigned long long)));
        HIP_TRY(hipMalloc((void**)&c->d_wfull, sizeof(unsigned int)));
        HIP_TRY(hipMemsetAsync(c->d_wsize, 0, sizeof(unsigned long long), st));
        HIP_TRY(hipMemsetAsync(c->d_wfull, 0, sizeof(unsigned int), st));
    }
    const uint64_t slot = 16ull + 8ull * (uint64_t)c->L, need = c->wsize + extra;
    if (c->wcap && (double)need <= load_limit(c->wcap, slot) * (double)c->wcap) return LDGPU_OK;
    uint64_t cap = next_pow2(std::max<uint64_t>(1 << 12, 4 * need));
    if (cap * slot > kBigTableBytes) cap = std::max(c->wcap, next_pow2((uint64_t)((double)need / 0.7) + 1));
    ldgpu_counts t;
    t.L = c->L;
    t.wcap = cap;
    hipError_t e = hipMalloc((void**)&t.d_wlo, cap * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void**)&t.d_whi, cap * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void**)&t.d_wcounts, cap * (size_t)c->L * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemsetAsync(t.d_whi, 0, cap * sizeof(uint64_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(t.d_wcounts, 0, cap * (size_t)c->L * sizeof(unsigned long long), st);
    if (e == hipSuccess && c->wcap) e = launch_wide_rehash(wide_params(c), wide_params(&t), c->wcap, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        for (void* q : {(void*)t.d_wlo, (void*)t.d_whi, (void*)t.d_wcounts})
            if (q) (void)hipFree(q);
        return fail(LDGPU_ENOMEM, "wide count table of %llu slots: %s", (unsigned long long)cap, hipGetErrorString(e));
    }
    for (void* q : {(void*)c->d_wlo, (void*)c->d_whi, (void*)c->d_wcounts})
        if (q) (void)hipFree(q);
    c->d_wlo = t.d_wlo;
    c->d_whi = t.d_whi;
    c->d_wcounts = t.d_wcounts;
    c->wcap = cap;
    t.d_wlo = t.d_whi = nullptr;
    t.d_wcounts = nullptr;
    return LDGPU_OK;
}

// after a wide launch: the table's size, and no insert left without a slot
int wide_after(ldgpu_counts* c) {
    unsigned long long size = 0;
    unsigned int full = 0;
    HIP_TRY(hipMemcpyAsync(&size, c->d_wsize, sizeof size, hipMemcpyDeviceToHost, c->ctx->stream));
    HIP_TRY(hipMemcpyAsync(&full, c->d_wfull, sizeof full, hipMemcpyDeviceToHost, c->ctx->stream));
    HIP_TRY(hipStreamSynchronize(c->ctx->stream));
    if (full) return fail(LDGPU_EDEVICE, "wide count table: an insert found no slot");
    c->wsize = size;
    c->tbl_valid = false;
    c->sp_valid = false;
    return LDGPU_OK;
}

// ---- grams longer than kMaxWideGram (ldgpu_long.hip)
LongCountParams long_params(const ldgpu_counts* c) {
    LongCountParams p{};
    p.slots = c->d_lslots;
    p.shift = c->lcap ? (uint32_t)(64 - log2u(c->lcap)) : 63u;
    p.mask = c->lcap ? c->lcap - 1 : 0;
    p.size = c->d_lctr;
    p.psize = c->d_lctr ? c->d_lctr + 1 : nullptr;
    p.arena_n = c->d_lctr ? c->d_lctr + 2 : nullptr;
    p.full = c->d_lctr ? reinterpret_cast<unsigned int*>(c->d_lctr + 3) : nullptr;
    p.arena = c->d_larena;
    p.arena_cap = c->larena_cap;
    p.pkeys = c->d_lpkeys;
    p.pcounts = c->d_lpcounts;
    p.pshift = c->lpcap ? (uint32_t)(64 - log2u(c->lpcap)) : 63u;
    p.pmask = c->lpcap ? c->lpcap - 1 : 0;
    p.L = c->L;
    return p;
}

// the long table's pairs as a sparse-T pair view (launch_pair_rehash / _compact)
CountParams long_pair_view(const ldgpu_counts* c, uint64_t* pkeys, unsigned long long* pcounts, uint64_t pcap) {
    CountParams v{};
    v.pkeys = pkeys;
    v.pcounts = pcounts;
    v.pshift = pcap ? (uint32_t)(64 - log2u(pcap)) : 63u;
    v.pmask = pcap ? pcap - 1 : 0;
    v.L = 1;
    return v;
}

// room for `grams` more long grams, `pairs` more pairs (load <= 1/2) and
// `bytes` more arena bytes: allocate, or grow by device rehash (pairs re-keyed
// through the slot remap) / a copy of the arena
int long_reserve(ldgpu_counts* c, uint64_t grams, uint64_t pairs, uint64_t bytes) {
    hipStream_t st = c->ctx->stream;
    if (!c->d_lctr) {
        HIP_TRY(hipMalloc((void**)&c->d_lctr, 4 * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(c->d_lctr, 0, 4 * sizeof(unsigned long long), st));
    }
    // Every new table is allocated and filled before any old one is
    // released: a failure leaves the table as it was (a grown slot table
    // re-keys the pairs through its remap, so both move together).
    const bool gslots = 2 * (c->lsize + grams) > c->lcap;
    if (gslots || 2 * (c->lpsize + pairs) > c->lpcap) {
        const uint64_t cap = gslots ? next_pow2(std::max<uint64_t>(1 << 12, 4 * (c->lsize + grams))) : c->lcap;
        const uint64_t pcap = std::max<uint64_t>(c->lpcap, next_pow2(std::max<uint64_t>(1 << 12, 4 * (c->lpsize + pairs))));
        ldgpu_counts t;
        t.L = c->L;
        t.lcap = cap;
        uint64_t* remap = nullptr;
        uint64_t* nk = nullptr;
        unsigned long long* nc = nullptr;
        hipError_t e = hipSuccess;
        if (gslots) {
            e = hipMalloc((void**)&t.d_lslots, cap * sizeof(LongSlot));
            if (e == hipSuccess) e = hipMemsetAsync(t.d_lslots, 0, cap * sizeof(LongSlot), st);
            if (e == hipSuccess && c->lcap) e = hipMalloc((void**)&remap, c->lcap * sizeof(uint64_t));
        }
        if (e == hipSuccess) e = hipMalloc((void**)&nk, pcap * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMalloc((void**)&nc, pcap * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMemsetAsync(nk, 0, pcap * sizeof(uint64_t), st);
        if (e == hipSuccess) e = hipMemsetAsync(nc, 0, pcap * sizeof(unsigned long long), st);
        if (e == hipSuccess && gslots && c->lcap)
            e = launch_long_rehash(long_params(c), long_params(&t), c->lcap, remap, st);
        if (e == hipSuccess && c->lpcap)
            e = launch_pair_rehash(long_pair_view(c, c->d_lpkeys, c->d_lpcounts, c->lpcap),
                                   long_pair_view(c, nk, nc, pcap), c->lpcap, remap, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (remap) (void)hipFree(remap);
        if (e != hipSuccess) {
            for (void* q : {(void*)t.d_lslots, (void*)nk, (void*)nc})
                if (q) (void)hipFree(q);
            t.d_lslots = nullptr;
            return fail(LDGPU_ENOMEM, "long gram tables of %llu / %llu slots: %s", (unsigned long long)cap,
                        (unsigned long long)pcap, hipGetErrorString(e));
        }
        if (gslots) {
            if (c->d_lslots) (void)hipFree(c->d_lslots);
            c->d_lslots = t.d_lslots;
            c->lcap = cap;
        }
        t.d_lslots = nullptr;
        for (void* q : {(void*)c->d_lpkeys, (void*)c->d_lpcounts})
            if (q) (void)hipFree(q);
        c->d_lpkeys = nk;
        c->d_lpcounts = nc;
        c->lpcap = pcap;
    }
    if (c->larena_n + bytes > c->larena_cap) {
        const uint64_t cap = next_pow2(std::max<uint64_t>(1 << 16, 2 * (c->larena_n + bytes)));
        uint8_t* a = nullptr;
        hipError_t e = hipMalloc((void**)&a, cap);
        if (e == hipSuccess && c->larena_n) e = hipMemcpyAsync(a, c->d_larena, c->larena_n, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            if (a) (void)hipFree(a);
            return fail(LDGPU_ENOMEM, "long gram key arena of %llu bytes: %s", (unsigned long long)cap,
                        hipGetErrorString(e));
        }
        if (c->d_larena) (void)hipFree(c->d_larena);
        c->d_larena = a;
        c->larena_cap = cap;
    }
    return LDGPU_OK;
}

// after a long launch: the counters, and no insert left without room
int long_after(ldgpu_counts* c) {
    unsigned long long ctr[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(ctr, c->d_lctr, sizeof ctr, hipMemcpyDeviceToHost, c->ctx->stream));
    HIP_TRY(hipStreamSynchronize(c->ctx->stream));
    c->tbl_valid = false;
    c->sp_valid = false;
    if ((unsigned int)ctr[3]) return fail(LDGPU_EDEVICE, "long gram table: an insert found no room");
    c->lsize = ctr[0];
    c->lpsize = ctr[1];
    c->larena_n = ctr[2];
    return LDGPU_OK;
}

// the long gram lengths (distinct, with their multiplicity in gramLengths)
DeriveParams long_lengths(const ldgpu_counts* c) {
    DeriveParams d{};
    for (int i = 0; i < c->nGl; ++i) {
        int j = 0;
        while (j < d.n && d.len[j] != c->Gl[i]) ++j;
        if (j == d.n) {
            d.len[d.n] = c->Gl[i];
            d.mult[d.n++] = 0;
        }
        d.mult[j]++;
    }
    return d;
}

// Count the long gram lengths of documents [0, n_docs) (h_off, h_lang: their
// offsets and languages on the host): launches of at most kLongLaunchWindows
// windows, the tables sized for each up front.
constexpr int64_t kLongLaunchWindows = 1ll << 24;

int long_count_launch(ldgpu_counts* c, const uint8_t* d_bytes, const int64_t* d_offsets, const int32_t* d_lang,
                      int64_t n_docs, const int64_t* h_off, const int32_t* h_lang) {
    const DeriveParams d = long_lengths(c);
    if (!d.n) return LDGPU_OK;
    int64_t d0 = 0;
    while (d0 < n_docs) {
        int64_t d1 = d0, win = 0, bytes = 0;
        while (d1 < n_docs) {
            const int64_t len = h_off[d1 + 1] - h_off[d1];
            int64_t w = 0, b = 0;
            if (h_lang[d1] >= 0 && h_lang[d1] < c->L) {
                bool part = false;
                for (int j = 0; j < d.n; ++j) {
                    if (len >= d.len[j]) {
                        w += len - d.len[j] + 1;
                        b += (len - d.len[j] + 1) * (int64_t)d.len[j];
                    } else {
                        part = true;
                    }
                }
                if (part && len > kMaxWideGram) {
                    w += 1;
                    b += len;
                }
            }
            if (d1 > d0 && win + w > kLongLaunchWindows) break;
            win += w;
            bytes += b;
            ++d1;
        }
        if (win) {
            if (int rc = long_reserve(c, (uint64_t)win, (uint64_t)win, (uint64_t)bytes)) return rc;
            HIP_TRY(launch_long_count(long_params(c), d_bytes, d_offsets + d0, d_lang + d0, d1 - d0, d, c->ctx->stream));
            if (int rc = long_after(c)) return rc;
        }
        d0 = d1;
    }
    return LDGPU_OK;
}

// add (key, language, count) triples of long keys (their bytes: kb[ko[i] ..
// ko[i + 1]), host memory) to the long table
int long_add_triples(ldgpu_counts* c, const std::vector<uint8_t>& kb, const std::vector<int64_t>& ko,
                     const std::vector<int32_t>& tl, const std::vector<unsigned long long>& tc) {
    const int64_t n = (int64_t)tl.size();
    if (!n) return LDGPU_OK;
    if (int rc = long_reserve(c, (uint64_t)n, (uint64_t)n, (uint64_t)kb.size())) return rc;
    hipStream_t st = c->ctx->stream;
    uint8_t* d_kb = nullptr;
    int64_t* d_ko = nullptr;
    int32_t* d_l = nullptr;
    unsigned long long* d_c = nullptr;
    hipError_t e = hipMalloc((void**)&d_kb, std::max<size_t>(kb.size(), 1));
    if (e == hipSuccess) e = hipMalloc((void**)&d_ko, sizeof(int64_t) * (n + 1));
    if (e == hipSuccess) e = hipMalloc((void**)&d_l, sizeof(int32_t) * n);
    if (e == hipSuccess) e = hipMalloc((void**)&d_c, sizeof(unsigned long long) * n);
    if (e == hipSuccess && !kb.empty()) e = hipMemcpyAsync(d_kb, kb.data(), kb.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_ko, ko.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_l, tl.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_c, tc.data(), sizeof(unsigned long long) * n, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = launch_long_add(long_params(c), d_kb, d_ko, d_l, d_c, n, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    for (void* q : {(void*)d_kb, (void*)d_ko, (void*)d_l, (void*)d_c})
        if (q) (void)hipFree(q);
    if (e != hipSuccess) return fail(LDGPU_EDEVICE, "long gram add: %s", hipGetErrorString(e));
    return long_after(c);
}

// Count the wide gram lengths of documents [0, n_docs): sub-launches of at
// most kWideLaunchWindows wide windows, the table grown for each up front;
// partial windows shorter than 8 bytes go to the one-word table through its
// overflow-safe insert (so the overflow list must hold them all).
constexpr int64_t kWideLaunchWindows = 1ll << 25;

int wide_count_launch(ldgpu_counts* c, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                      const int32_t* d_lang, int64_t n_docs, const int64_t* h_off) {
    hipStream_t st = c->ctx->stream;
    int64_t d0 = 0;
    while (d0 < n_docs) {
        int64_t d1 = d0, wide = 0, part = 0;
        while (d1 < n_docs) {
            const int64_t len = h_off[d1 + 1] - h_off[d1];
            int64_t w = 0, q = 0;
            for (int i = 0; i < c->nGw; ++i) {
                if (len >= 8) w += n_windows(len, c->Gw[i]);
                else if (len > 0) q += 1;
            }
            if (d1 > d0 && wide + w > kWideLaunchWindows) break;
            wide += w;
            part += q;
            ++d1;
        }
        if (int rc = wide_ensure(c, (uint64_t)wide)) return rc;
        if (int rc = ensure_ovf(c, std::max<int64_t>(part, 1))) return rc;
        if (int rc = reserve(c, (uint64_t)part, (uint64_t)part)) return rc;
        WideCountParams p = wide_params(c);
        p.bytes = d_bytes;
        p.last_dword = n_bytes > 0 ? (n_bytes - 1) >> 2 : 0;
        p.offsets = d_offsets + d0;
        p.doc_lang = d_lang + d0;
        p.n_docs = d1 - d0;
        p.narrow.ovf_cap = c->ovf_cap;
        const int64_t want = (p.n_docs + kCountWaves - 1) / kCountWaves;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)c->ctx->cus * 2));
        HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
        HIP_TRY(launch_wide_count(p, grid, st));
        if (int rc = wide_after(c)) return rc;
        if (int rc = after_batch(c)) return rc;  // the one-word keys of short documents
        d0 = d1;
    }
    return LDGPU_OK;
}

// FIT v4 batches: at most batch_recs records (kBatchRecords / K: one per
// byte position, ~512 MB of corpus), so the record scratch (K words per
// record for the emit blocks and the buckets, out_words per record of reduce
// output) stays within ~16 GB of HBM.  Larger batches merge a frequent
// (window, language) pair into T1 fewer times.
constexpr int64_t kBatchRecords = 1ll << 29;

int out_words(int K) { return K == 1 ? 2 : K; }

int counts_new(ldgpu_ctx* ctx, int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams, int64_t capacity_hint,
               ldgpu_counts** out, bool sparse = false);

// distinct gram lengths, ascending, with their multiplicity in gramLengths
// (every gramLengths entry, long ones included: partial_kernel counts the
// partial window of a short document once per n above its length)
DeriveParams derive_params(const ldgpu_counts* c) {
    DeriveParams d{};
    std::vector<int32_t> lens(c->Gall, c->Gall + c->nGall);
    std::sort(lens.begin(), lens.end());
    for (size_t i = 0; i < lens.size(); ++i) {
        if (d.n && d.len[d.n - 1] == lens[i]) {
            d.mult[d.n - 1]++;
            continue;
        }
        d.len[d.n] = lens[i];
        d.mult[d.n] = 1;
        ++d.n;
    }
    return d;
}

// T1 (c->pend) -> T (c), level by level (derive_level_kernel): level t
// reads T1's entries of t bytes, adds them to T (t in gramLengths) and to
// their (t-1)-byte prefixes in T1.  A level's passes go in chunks of T1 slots
// small enough that the overflow lists hold every add of the chunk and T,
// even if every add were a new key, stays within 0.1 of its load limit (T
// grows with the keys actually inserted).  T1 may not move during a level:
// it is grown before the level to hold the level's new prefixes (at most its
// entries) within 0.1 of its load limit, and its overflow entries go back in
// place.
int derive_pending(ldgpu_counts* c) {
    ldgpu_counts* t = c->pend;
    if (!t || (t->size == 0 && t->wsize == 0)) return LDGPU_OK;
    hipStream_t st = c->ctx->stream;
    uint32_t mult[kMaxWideGram + 1] = {};
    int maxg = 0;
    for (int i = 0; i < c->nG; ++i) {
        mult[c->G[i]]++;
        maxg = std::max(maxg, c->G[i]);
    }
    const uint64_t L = (uint64_t)c->L;
    const char* dab = diag_env("LDGPU_FIT_DERIVE_ABLATE");  // timing only (counts wrong)
    const int derive_ablate = dab ? atoi(dab) : 0;
    // T1 of (window, language) pairs: one-word keys (K = 1) or a wide table of
    // (packed key, lang + 1) (K = 2); dense rows otherwise
    const int pairs = c->K == 1 ? 1 : (c->K == 2 ? 2 : 0);
    const uint64_t per_slot = pairs ? 1 : L;  // adds of one T1 slot (to T; to T1)
    // T1's occupied slots per key length
    unsigned long long cnt[16] = {};
    {
        void* d_h = nullptr;
        HIP_TRY(cache_alloc(c->ctx, &d_h, sizeof cnt));
        HIP_TRY(hipMemsetAsync(d_h, 0, sizeof cnt, st));
        HIP_TRY(launch_len_hist(count_params(t), wide_params(t), pairs, c->lb, (unsigned long long*)d_h, st));
        HIP_TRY(hipMemcpyAsync(cnt, d_h, sizeof cnt, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        cache_free(c->ctx, d_h, sizeof cnt);
    }
    // T's projected growth: the N-byte windows (most of T1) are new keys
    // (a pair table holds ~2 languages per window on multilingual corpora);
    // every T1 entry of a level is one (gram, language) pair of T
    {
        const double tn = (double)(t->size + t->wsize);
        const double est = (double)c->size + (pairs ? 0.55 : 1.1) * tn;
        if (est > max_load(c) * (double)c->cap) {
            const uint64_t target = cap_for(est, 8ull + row_bytes(c));
            if (target > c->cap && grow(c, target) != LDGPU_OK) {
                (void)hipGetLastError();
                (void)ok();
            }
        }
        const double pest = (double)c->psize + 1.1 * tn;
        if (c->sparse && pest > pair_load(c) * (double)c->pcap) {
            if (pgrow(c, cap_for(pest, 16ull)) != LDGPU_OK) {
                (void)hipGetLastError();
                (void)ok();
            }
        }
    }
    // two-word pair T1 (K = 2): each level writes its prefixes and the shorter
    // entries into another table (derive_pairs2_level_kernel's split), sized
    // for all of them: a level's scan reads only the entries still to derive,
    // and T1 never holds a grown table next to the old one.  The two tables
    // alternate (the one read by a level is cleared and written by the next,
    // when it holds them: no allocation per level -- 51 GB at L = 200 on 1 GB
    // of corpus).  Diagnostics: LDGPU_FIT_DERIVE_INPLACE keeps one T1.
    const bool split = pairs == 2 && !diag_env("LDGPU_FIT_DERIVE_INPLACE");
    struct Owned {
        ldgpu_counts* p = nullptr;
        ~Owned() {
            if (p) counts_free(p);
        }
        void reset(ldgpu_counts* q) {
            if (p) counts_free(p);
            p = q;
        }
    };
    Owned spare;  // the table the previous level read
    const bool trace = diag_env("LDGPU_FIT_TRACE") != nullptr;
    auto now_ms = [] {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    for (int lev = maxg; lev >= 1; --lev) {
        const double t_lev = trace ? now_ms() : 0.0;
        int chunks = 0;
        const uint32_t mt = mult[lev];
        const int n = lev - 1;
        if (!cnt[lev] || (!mt && n < 1)) continue;
        const bool wide = lev > kMaxGram || pairs == 2;  // the level's entries are in T1's wide table
        // T1 room for this level's prefixes (one per entry at most), within
        // 0.1 of its load limit (linear probes stay short)
        Owned nx;
        if (n >= 1 && split) {
            uint64_t keep = cnt[lev];
            for (int j = 1; j < lev; ++j) keep += cnt[j];
            ldgpu_counts* sp = spare.p;
            if (sp && sp->wcap && (double)keep <= load_limit(sp->wcap, 16ull + 8ull * (uint64_t)sp->L) * (double)sp->wcap) {
                // the spare, emptied (a key word of 0 is an empty slot; the
                // low words are written before a slot is published)
                HIP_TRY(hipMemsetAsync(sp->d_whi, 0, sp->wcap * sizeof(uint64_t), st));
                HIP_TRY(hipMemsetAsync(sp->d_wcounts, 0, sp->wcap * (size_t)sp->L * sizeof(unsigned long long), st));
                HIP_TRY(hipMemsetAsync(sp->d_wsize, 0, sizeof(unsigned long long), st));
                sp->wsize = 0;
                nx.p = sp;
                spare.p = nullptr;
            } else {
                spare.reset(nullptr);
                if (int rc = counts_new(c->ctx, 1, c->G, c->nG, 1 << 12, &nx.p)) return rc;
                if (int rc = wide_ensure(nx.p, keep)) return rc;
            }
            cnt[n] += cnt[lev];
        } else if (n >= 1) {
            if (n <= kMaxGram && pairs != 2) {
                const double need = (double)(t->size + cnt[lev]);
                if (need > (max_load(t) + 0.1) * (double)t->cap) {
                    if (int rc = grow(t, next_pow2((uint64_t)(need / max_load(t)) + 16))) return rc;
                }
            } else if (int rc = wide_ensure(t, cnt[lev])) {
                return rc;
            }
            cnt[n] += cnt[lev];
        }
        const uint64_t tcap = wide ? t->wcap : t->cap;
        const double tload = std::max(1e-6, (double)cnt[lev] / (double)tcap);
        for (uint64_t s0 = 0; s0 < tcap;) {
            while ((double)c->size > max_load(c) * (double)c->cap) {
                if (int rc = grow(c, 2 * c->cap)) return rc;
            }
            while (c->sparse && (double)c->psize > pair_load(c) * (double)c->pcap) {
                if (int rc = pgrow(c, 2 * c->pcap)) return rc;
            }
            uint64_t slots = kOvfMax / per_slot;
            if (mt) {
                // every occupied T1 slot adds at most one gram and per_slot pairs to T
                const double room = std::max(1.0, (max_load(c) + 0.1) * (double)c->cap - (double)c->size);
                slots = std::min<uint64_t>(slots, (uint64_t)(room / tload));
                if (c->sparse) {
                    const double proom = std::max(1.0, (pair_load(c) + 0.1) * (double)c->pcap - (double)c->psize);
                    slots = std::min<uint64_t>(slots, (uint64_t)(proom / (tload * (double)per_slot)));
                }
                if (lev > kMaxGram) {
                    const uint64_t occ = std::min<uint64_t>(cnt[lev], (uint64_t)(2.0 * tload * (double)slots) + 64);
                    if (int rc = wide_ensure(c, occ)) return rc;
                }
            }
            slots = std::min<uint64_t>(std::max<uint64_t>(slots, 1), tcap - s0);
            const int64_t adds = (int64_t)std::min<uint64_t>(slots * per_slot, kOvfMax);
            if (int rc = ensure_ovf(c, adds)) return rc;
            if (int rc = ensure_ovf(t, adds)) return rc;
            HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
            HIP_TRY(hipMemsetAsync(t->d_ovf_n, 0, sizeof(unsigned int), st));
            if (pairs == 2)
                HIP_TRY(launch_derive_pairs2_level(wide_params(t), s0, s0 + slots, lev, mt, count_params(c),
                                                   nx.p ? wide_params(nx.p) : WideCountParams{}, derive_ablate, st));
            else if (pairs)
                HIP_TRY(launch_derive_pairs_level(count_params(t), c->lb, s0, s0 + slots, lev, mt, count_params(c),
                                                  derive_ablate, st));
            else
                HIP_TRY(launch_derive_level(count_params(t), wide_params(t), wide, s0, s0 + slots, lev, mt,
                                            count_params(c), wide_params(c), st));
            if (lev > kMaxGram && mt) {
                if (int rc = wide_after(c)) return rc;
            }
            if (n > kMaxGram || (pairs == 2 && n >= 1)) {
                if (int rc = wide_after(nx.p ? nx.p : t)) return rc;
            }
            if (int rc = after_batch(c)) return rc;
            if (int rc = after_batch(t, false)) return rc;
            s0 += slots;
            ++chunks;
        }
        if (nx.p) {  // the next level's T1; this one the spare
            spare.reset(t);
            c->pend = t = nx.p;
            nx.p = nullptr;
        }
        if (trace) {
            HIP_TRY(hipStreamSynchronize(st));
            fprintf(stderr, "fit derive level %d: %llu entries, %d chunks, %.3f ms (T %llu grams / %llu slots, %llu pairs / %llu)\n",
                    lev, cnt[lev], chunks, now_ms() - t_lev, (unsigned long long)c->size, (unsigned long long)c->cap,
                    (unsigned long long)c->psize, (unsigned long long)c->pcap);
        }
    }
    return LDGPU_OK;
}

// Partial windows of the call's documents shorter than some gram length
// (partial_kernel): one add each, straight into T.
int count_partial(ldgpu_counts* c, const uint8_t* d_bytes, const int64_t* d_offsets, const int32_t* d_lang,
                  int64_t n_docs, const int64_t* h_off, const int32_t* h_lang) {
    int maxg = 0;
    for (int i = 0; i < c->nGall; ++i) maxg = std::max(maxg, c->Gall[i]);
    std::vector<int64_t> docs;
    bool any_wide = false;
    for (int64_t d = 0; d < n_docs; ++d) {
        const int64_t len = h_off[d + 1] - h_off[d];
        if (len <= 0 || len >= maxg || h_lang[d] < 0 || h_lang[d] >= c->L) continue;
        docs.push_back(d);
        any_wide |= len > kMaxGram;
    }
    if (docs.empty()) return LDGPU_OK;
    ldgpu_ctx* x = c->ctx;
    hipStream_t st = x->stream;
    const int64_t n = (int64_t)docs.size();
    if (int rc = ensure_ovf(c, n)) return rc;
    if (int rc = reserve(c, (uint64_t)n, (uint64_t)n)) return rc;
    if (any_wide) {
        if (int rc = wide_ensure(c, (uint64_t)n)) return rc;
    }
    HIP_TRY(x->f_ocnt.ensure(sizeof(int64_t) * (size_t)n));
    HIP_TRY(hipMemcpyAsync(x->f_ocnt.p, docs.data(), sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
    HIP_TRY(launch_partial(d_bytes, d_offsets, d_lang, (const int64_t*)x->f_ocnt.p, n, count_params(c), wide_params(c),
                           derive_params(c), st));
    if (any_wide) {
        if (int rc = wide_after(c)) return rc;
    }
    return after_batch(c);
}

// n (key, language, count) run entries into T (FIT v5).  T first grows to
// its projected size (new grams / pairs per entry as in the table's last
// insert; a failed grow leaves T as it was and the chunks grow it instead),
// then the entries go in chunks small enough that T stays within 0.1 of its
// load limits even if every entry were new and the overflow lists hold them
// all, T doubling whenever it passes a limit.
int insert_runs(ldgpu_counts* c, const uint64_t* d_k, const int32_t* d_l, const unsigned long long* d_c, int64_t n) {
    if (n <= 0) return LDGPU_OK;
    hipStream_t st = c->ctx->stream;
    const double eg = (double)c->size + c->run_new_grams * (double)n;
    if (eg > max_load(c) * (double)c->cap && grow(c, cap_for(eg, 8ull + row_bytes(c))) != LDGPU_OK) {
        (void)hipGetLastError();
        (void)ok();
    }
    const double ep = (double)c->psize + c->run_new_pairs * (double)n;
    if (c->sparse && ep > pair_load(c) * (double)c->pcap && pgrow(c, cap_for(ep, 16ull)) != LDGPU_OK) {
        (void)hipGetLastError();
        (void)ok();
    }
    const uint64_t g0 = c->size, p0 = c->psize;
    for (int64_t i0 = 0; i0 < n;) {
        while ((double)c->size > max_load(c) * (double)c->cap) {
            if (int rc = grow(c, 2 * c->cap)) return rc;
        }
        while (c->sparse && (double)c->psize > pair_load(c) * (double)c->pcap) {
            if (int rc = pgrow(c, 2 * c->pcap)) return rc;
        }
        double room = (max_load(c) + 0.1) * (double)c->cap - (double)c->size;
        if (c->sparse) room = std::min(room, (pair_load(c) + 0.1) * (double)c->pcap - (double)c->psize);
        const int64_t m = std::min<int64_t>(std::min<int64_t>(n - i0, (int64_t)kOvfMax), std::max<int64_t>(1, (int64_t)room));
        if (int rc = ensure_ovf(c, m)) return rc;
        HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
        HIP_TRY(launch_runs_add(count_params(c), d_k + i0, d_l + i0, d_c + i0, m, c->ctx->cus, st));
        if (int rc = after_batch(c)) return rc;
        i0 += m;
    }
    c->run_new_grams = std::max(0.02, (double)(c->size - g0) / (double)n);
    c->run_new_pairs = std::max(0.02, (double)(c->psize - p0) / (double)n);
    return LDGPU_OK;
}

// FIT v5 applies to a sparse count table of two-word records (grams of <= 7
// bytes whose one-word record has no room: many languages) whose sort key
// (8 max(G) bits of window, ceil(log2(L + 1)) of language) fits 64 bits.
// Diagnostics: LDGPU_FIT_NO_SORT keeps such tables on FIT v4 (A/B, tests).
bool sort_path(const ldgpu_counts* c) {
    if (!c->sparse || c->K != 2 || c->nG == 0 || diag_env("LDGPU_FIT_NO_SORT")) return false;
    int maxg = 0;
    for (int i = 0; i < c->nG; ++i) maxg = std::max(maxg, c->G[i]);
    return maxg <= kMaxGram && 8 * maxg + log2u((uint64_t)c->L + 1) <= 64;
}

// byte positions per FIT v5 batch: the keys and the sort's second buffer take
// 16 B each, the run entries of one gram length <= 20 B per position
constexpr int64_t kSortBatch = 1ll << 30;

// Count documents [0, n_docs) with FIT v5 (ldgpu_fit.h): per batch of
// documents, every position's sort key (the tail positions' grams straight
// into T), one radix sort, then per distinct gram length n one pass that
// turns the runs of equal (language, n-byte prefix) into (n-gram, language,
// count) entries, inserted into T.  Partial windows and grams longer than 15
// bytes take their own kernels, as in FIT v4.
int count_launch_sorted(ldgpu_counts* c, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                        const int32_t* d_lang, int64_t n_docs, const int64_t* h_off, const int32_t* h_lang) {
    ldgpu_ctx* x = c->ctx;
    hipStream_t st = x->stream;
    if (c->pend) {
        counts_free(c->pend);
        c->pend = nullptr;
    }
    if (int rc = count_partial(c, d_bytes, d_offsets, d_lang, n_docs, h_off, h_lang)) return rc;
    if (int rc = long_count_launch(c, d_bytes, d_offsets, d_lang, n_docs, h_off, h_lang)) return rc;
    int N = 0;
    uint32_t mult[kMaxGram + 1] = {};
    for (int i = 0; i < c->nG; ++i) {
        N = std::max(N, c->G[i]);
        mult[c->G[i]]++;
    }
    const int bits = 8 * N + log2u((uint64_t)c->L + 1);
    const DeriveParams d = derive_params(c);
    // tail adds of a document of len bytes: for each of its last min(N - 1,
    // len) positions (r bytes left), the gram lengths <= r
    int64_t tails_of[kMaxGram + 1] = {};
    for (int r = 1; r < N; ++r) {
        int64_t k = 0;
        for (int j = 0; j < d.n && d.len[j] <= r; ++j) ++k;
        tails_of[r] = tails_of[r - 1] + k;
    }
    // positions per batch: at most kSortBatch, and at most what half of the
    // device memory left (plus the scratch this context already holds) takes
    // at ~36 B per position -- the keys and the sort's second buffer (8 B
    // each), a length's run entries (20 B), the sort's scratch -- so a fit
    // that fits a smaller or shared device runs in more, smaller batches
    int64_t batch = kSortBatch;
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const double held = (double)(x->f_rec.cap + x->f_rec2.cap + x->f_okl.cap + x->f_stmp.cap);
            const int64_t fit = (int64_t)(0.5 * ((double)free_b + held) / 36.0);
            batch = std::max<int64_t>(1ll << 24, std::min<int64_t>(batch, fit));
        }
    }
    if (const char* b = diag_env("LDGPU_FIT_SORT_BATCH")) batch = std::max(1ll, atoll(b));
    const bool trace = diag_env("LDGPU_FIT_TRACE") != nullptr;
    auto now_ms = [] {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    HIP_TRY(x->f_on.ensure(sizeof(unsigned long long) * (kMaxGram + 2)));
    unsigned long long* d_n = (unsigned long long*)x->f_on.p;  // [0]: entries written, [1..7]: runs per length
    for (int64_t d0 = 0; d0 < n_docs;) {
        const double t0 = trace ? now_ms() : 0.0;
        int64_t d1 = d0, R = 0, tails = 0;
        while (d1 < n_docs) {
            const int64_t len = h_off[d1 + 1] - h_off[d1];
            const bool ok_doc = len > 0 && h_lang[d1] >= 0 && h_lang[d1] < c->L;
            const int64_t t = ok_doc ? tails_of[std::min<int64_t>(len, N - 1)] : 0;
            if (d1 > d0 && (h_off[d1 + 1] - h_off[d0] > batch || tails + t > (int64_t)kOvfMax)) break;
            if (ok_doc) R += std::max<int64_t>(0, len - N + 1);
            tails += t;
            ++d1;
        }
        const int64_t P = h_off[d1] - h_off[d0];
        if (P > INT32_MAX)
            return fail(LDGPU_EUNSUPPORTED, "FIT: a document of %lld bytes exceeds the sort batch", (long long)P);
        if (P > 0) {
            HIP_TRY(x->f_rec.ensure(sizeof(uint64_t) * (size_t)P));
            HIP_TRY(x->f_rec2.ensure(sizeof(uint64_t) * (size_t)P));
            uint64_t* keys = (uint64_t*)x->f_rec.p;
            uint64_t* alt = (uint64_t*)x->f_rec2.p;
            if (tails) {
                if (int rc = ensure_ovf(c, tails)) return rc;
                if (int rc = reserve(c, (uint64_t)tails, (uint64_t)tails)) return rc;
            }
            HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
            SortFitParams sp{};
            sp.bytes = d_bytes;
            sp.last_dword = n_bytes > 0 ? (n_bytes - 1) >> 2 : 0;
            sp.offsets = d_offsets + d0;
            sp.doc_lang = d_lang + d0;
            sp.n_docs = d1 - d0;
            sp.base = h_off[d0];
            sp.N = N;
            sp.L = c->L;
            sp.keys = keys;
            sp.d = d;
            HIP_TRY(launch_sort_emit(sp, count_params(c), st));
            if (int rc = after_batch(c)) return rc;  // the tail adds (overflow entries re-inserted)
            const double t1 = trace ? now_ms() : 0.0;
            size_t tb = 0;
            bool in_alt = false;
            HIP_TRY(sort_keys_u64(P, keys, alt, bits, nullptr, &tb, nullptr, st));
            HIP_TRY(x->f_stmp.ensure(tb + 16));
            HIP_TRY(sort_keys_u64(P, keys, alt, bits, x->f_stmp.p, &tb, &in_alt, st));
            const uint64_t* sorted = in_alt ? alt : keys;
            if (trace) HIP_TRY(hipStreamSynchronize(st));
            const double t2 = trace ? now_ms() : 0.0;
            // run entries (key, count, language: 20 B), room for R of them:
            // the runs of every gram length, counted in one pass, then
            // written by passes over groups of lengths whose entries fit
            // (each length has at most R runs), inserted into T per pass
            const size_t cap = (size_t)std::max<int64_t>(R, 1);
            HIP_TRY(x->f_okl.ensure(cap * (2 * sizeof(uint64_t) + sizeof(int32_t)) + 64));
            uint64_t* rk = (uint64_t*)x->f_okl.p;
            unsigned long long* rcnt = (unsigned long long*)(rk + cap);
            int32_t* rl = (int32_t*)(rcnt + cap);
            double t_runs = 0.0, t_ins = 0.0;
            unsigned long long runs[kMaxGram + 1] = {};
            if (R > 0) {
                const double ta = trace ? now_ms() : 0.0;
                HIP_TRY(hipMemsetAsync(d_n, 0, sizeof(unsigned long long) * (kMaxGram + 2), st));
                HIP_TRY(launch_runs_count(sorted, R, N, d_n + 1, st));
                HIP_TRY(hipMemcpyAsync(runs, d_n + 1, sizeof runs, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                if (trace) t_runs += now_ms() - ta;
            }
            for (int n = N; n >= 1 && R > 0;) {
                RunLens lens{};
                unsigned long long want = 0;
                for (; n >= 1; --n) {
                    if (!mult[n]) continue;
                    if (runs[n] > (unsigned long long)R)
                        return fail(LDGPU_EDEVICE, "FIT runs: %llu of length %d from %lld keys", runs[n], n, (long long)R);
                    if (want + runs[n] > (unsigned long long)R) break;
                    want += runs[n];
                    lens.mask |= 1u << n;
                    lens.mult[n] = mult[n];
                }
                if (!lens.mask) continue;
                const double ta = trace ? now_ms() : 0.0;
                HIP_TRY(hipMemsetAsync(d_n, 0, sizeof(unsigned long long), st));
                HIP_TRY(launch_sort_runs(sorted, R, N, lens, rk, rl, rcnt, d_n, st));
                unsigned long long rn = 0;
                HIP_TRY(hipMemcpyAsync(&rn, d_n, sizeof rn, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                if (rn != want)
                    return fail(LDGPU_EDEVICE, "FIT runs: %llu entries, %llu counted (lengths 0x%x)", rn, want, lens.mask);
                const double tb2 = trace ? now_ms() : 0.0;
                if (int rc = insert_runs(c, rk, rl, rcnt, (int64_t)rn)) return rc;
                if (trace) {
                    t_runs += tb2 - ta;
                    t_ins += now_ms() - tb2;
                    fprintf(stderr, "fit v5 lengths 0x%x: %llu runs\n", lens.mask, rn);
                }
            }
            if (trace)
                fprintf(stderr, "fit v5 batch: %lld positions, %lld keys, %lld tail adds: emit %.3f sort %.3f runs %.3f "
                                "insert %.3f ms (T %llu grams / %llu slots, %llu pairs / %llu)\n",
                        (long long)P, (long long)R, (long long)tails, t1 - t0, t2 - t1, t_runs, t_ins,
                        (unsigned long long)c->size, (unsigned long long)c->cap, (unsigned long long)c->psize,
                        (unsigned long long)c->pcap);
        }
        d0 = d1;
    }
    return LDGPU_OK;
}

// Count documents [0, n_docs) on the device with FIT v4 (ldgpu_fit.hip): per
// batch, the documents in language order (h_lang: their languages on the
// host), emit -> part2 -> reduce -> merge into T1 (c->pend, the per-call table
// of maximal windows); then T1 derives every gram length's counts into T.
int count_launch_v3(ldgpu_counts* c, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                    const int32_t* d_lang, int64_t n_docs, const int64_t* h_off, const int32_t* h_lang) {
    ldgpu_ctx* x = c->ctx;
    hipStream_t st = x->stream;
    const int K = c->K;
    const int64_t thresh = emit_blk_recs(K) - emit_round_recs(K);
    int maxg = 0;
    for (int i = 0; i < c->nG; ++i) maxg = std::max(maxg, c->G[i]);
    if (c->pend) {  // left by a call that failed part-way: its counts are not carried over
        counts_free(c->pend);
        c->pend = nullptr;
    }
    if (int rc = count_partial(c, d_bytes, d_offsets, d_lang, n_docs, h_off, h_lang)) return rc;
    // gram lengths beyond 15 bytes: their own table (ldgpu_long.hip)
    if (int rc = long_count_launch(c, d_bytes, d_offsets, d_lang, n_docs, h_off, h_lang)) return rc;
    if (c->nG == 0) return LDGPU_OK;  // no gram length of <= 15 bytes: no maximal windows
    // T1's expected keys: this table's last call, or (K = 1 pair tables of up
    // to 2^28 keys) this context's last call scaled to this call's bytes --
    // larger T1s keep growing from the table's own hint, under the load
    // limits of a device-filling fit (a hint of ~1G two-word pairs from a
    // high-entropy fit would claim its table at load 1/2 at once: 100 GB)
    const int64_t call_bytes = h_off[n_docs] - h_off[0];
    int64_t t1_hint = c->pend_hint;
    if (K == 1) {
        const double h = std::min(1.1 * x->t1_keys_per_byte * (double)call_bytes, 2.0 * (double)x->t1_keys);
        if (h <= (double)(1ll << 28)) t1_hint = std::max<int64_t>(t1_hint, (int64_t)h);
    }
    if (!c->pend) {
        // one- and two-word records: T1 keyed by (window, language) pairs, one
        // counter each (K = 2: in its wide table, key (packed key, lang + 1));
        // a dense row of L counters per window otherwise
        if (int rc = counts_new(x, K <= 2 ? 1 : c->L, c->G, c->nG, std::max<int64_t>(1 << 16, t1_hint), &c->pend))
            return rc;
    }
    ldgpu_counts* t1 = c->pend;
    if (int rc = ensure_ovf(t1, 1 << 20)) return rc;
    std::vector<uint32_t> cnt3((size_t)kQ * kQ * kSplits);
    std::vector<uint64_t> p2off((size_t)kQ * kQ * kSplits), boff((size_t)kQ * kQ + 1);
    const int L = c->L;
    std::vector<int64_t> lcnt(L + 1), lwin(L);
    std::vector<int32_t> perm;
    std::vector<int64_t> wg_doc, wg_rec, wg_dir;
    // A batch's plan (documents in language order, emit workgroups, the
    // documents' starts and lengths) is made on the host while the GPU runs
    // the previous batch.
    struct BatchPlan {
        int64_t d0 = 0, d1 = 0, nd = 0, acc = 0, dirs = 0;
        int grid_a = 0;
        std::vector<int64_t> meta;
        std::vector<int32_t> wg_lang, plen;
    };
    auto make_plan = [&](int64_t d0, BatchPlan& bp) {
        std::vector<int64_t>& meta = bp.meta;
        std::vector<int32_t>& wg_lang = bp.wg_lang;
        std::vector<int32_t>& plen = bp.plen;
        // records of a document: one per byte position
        int64_t d1 = d0, W = 0;
        while (d1 < n_docs) {
            const int64_t len = h_off[d1 + 1] - h_off[d1];
            if (d1 > d0 && W + len > c->batch_recs) break;
            W += len;
            ++d1;
        }
        // the batch's documents of supported languages, in language order
        // (a stable counting sort; reduceGrams drops the others)
        std::fill(lcnt.begin(), lcnt.end(), 0);
        std::fill(lwin.begin(), lwin.end(), 0);
        for (int64_t d = d0; d < d1; ++d) {
            const int32_t l = h_lang[d];
            const int64_t len = h_off[d + 1] - h_off[d];
            if (l < 0 || l >= L || len <= 0) continue;
            lcnt[l + 1]++;
            lwin[l] += len;
        }
        for (int l = 0; l < L; ++l) lcnt[l + 1] += lcnt[l];
        const int64_t nd = lcnt[L];
        perm.assign((size_t)std::max<int64_t>(nd, 1), 0);
        {
            std::vector<int64_t> at(lcnt.begin(), lcnt.end() - 1);
            for (int64_t d = d0; d < d1; ++d) {
                const int32_t l = h_lang[d];
                if (l < 0 || l >= L || h_off[d + 1] <= h_off[d]) continue;
                perm[at[l]++] = (int32_t)(d - d0);
            }
        }
        // emit workgroups: each language's documents split into ranges
        // balanced by records, about 4 workgroups per CU in all (2 resident:
        // the tail of the launch stays short); a
        // workgroup's record region holds its records, its block directory
        // records / threshold + 2 blocks
        const int64_t Wk = std::accumulate(lwin.begin(), lwin.end(), (int64_t)0);
        const int64_t target = std::max<int64_t>(1, (Wk + 4 * x->cus - 1) / (4 * x->cus));
        wg_doc.clear();
        wg_rec.clear();
        wg_dir.clear();
        wg_lang.clear();
        int64_t acc = 0, dirs = 0;
        for (int l = 0; l < L; ++l) {
            if (!lwin[l]) continue;
            const int64_t parts = std::max<int64_t>(1, (lwin[l] + target - 1) / target);
            int64_t i = lcnt[l], wacc = 0;
            for (int64_t k = 0; k < parts; ++k) {
                const int64_t start = i, start_acc = acc, goal = lwin[l] * (k + 1) / parts;
                while (i < lcnt[l + 1] && (wacc < goal || k + 1 == parts)) {
                    const int64_t dd = d0 + perm[i];
                    const int64_t w = h_off[dd + 1] - h_off[dd];
                    wacc += w;
                    acc += w;
                    ++i;
                }
                if (i == start) continue;
                wg_doc.push_back(start);
                wg_rec.push_back(start_acc);
                wg_dir.push_back(dirs);
                wg_lang.push_back(l);
                dirs += (acc - start_acc) / thresh + 2;
            }
        }
        while (wg_doc.empty() || wg_doc.size() % kSplits) {  // empty workgroups: a multiple of kSplits
            wg_doc.push_back(nd);
            wg_rec.push_back(acc);
            wg_dir.push_back(dirs);
            wg_lang.push_back(0);
        }
        const int grid_a = (int)wg_doc.size();
        wg_doc.push_back(nd);
        wg_rec.push_back(acc);
        wg_dir.push_back(dirs);
        meta.clear();
        meta.reserve(3 * wg_doc.size());
        meta.insert(meta.end(), wg_doc.begin(), wg_doc.end());
        meta.insert(meta.end(), wg_rec.begin(), wg_rec.end());
        meta.insert(meta.end(), wg_dir.begin(), wg_dir.end());
        // the documents' starts and lengths in perm order (emit prefetches a
        // wave's next document with two independent loads)
        const size_t n_perm = perm.size();
        for (size_t i = 0; i < n_perm; ++i) {
            const int64_t dd = d0 + (nd ? perm[i] : 0);
            meta.push_back(h_off[dd]);
        }
        plen.assign(n_perm, 0);
        for (size_t i = 0; i < n_perm; ++i) {
            const int64_t dd = d0 + (nd ? perm[i] : 0);
            plen[i] = (int32_t)(h_off[dd + 1] - h_off[dd]);
        }
        bp.d0 = d0;
        bp.d1 = d1;
        bp.nd = nd;
        bp.acc = acc;
        bp.dirs = dirs;
        bp.grid_a = grid_a;
    };
    BatchPlan cur, nxt;
    make_plan(0, cur);
    // The last merge of a batch is not waited for: its table size and
    // overflow count are read back after the next batch's reduce (the host
    // waits there anyway), so the next batch's emit follows the merge on the
    // stream without a host round trip.  (Tables with a wide part check it
    // after every merge.)
    bool t1_pending = false;
    uint64_t pend_size0 = 0;
    unsigned long long pend_E = 0;
    auto settle_t1 = [&]() -> int {
        if (!t1_pending) return LDGPU_OK;
        t1_pending = false;
        if (int rc = after_batch(t1)) return rc;
        if (pend_E) t1->new_per_entry = std::max(0.02, (double)(t1->size + t1->wsize - pend_size0) / (double)pend_E);
        return LDGPU_OK;
    };
    // diagnostics build: host-side phase times per batch (LDGPU_FIT_TRACE)
    const bool trace = diag_env("LDGPU_FIT_TRACE") != nullptr;
    auto now_ms = [] {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    double tt[6] = {};
    for (;;) {
        if (trace) tt[0] = now_ms();
        const int64_t d0 = cur.d0, d1 = cur.d1, acc = cur.acc, dirs = cur.dirs;
        const int grid_a = cur.grid_a;
        const std::vector<int64_t>& meta = cur.meta;
        const std::vector<int32_t>& wg_lang = cur.wg_lang;
        const std::vector<int32_t>& plen = cur.plen;
        const size_t n_lang = wg_lang.size(), n_perm = plen.size();
        const size_t wg_bytes = sizeof(int64_t) * meta.size() + sizeof(int32_t) * (n_lang + n_perm);
        HIP_TRY(x->f_wg.ensure(wg_bytes + 16));
        HIP_TRY(x->h_fwg.ensure(wg_bytes + 16));
        HIP_TRY(x->h_fon.ensure(sizeof(uint32_t) * kQ * kQ + sizeof(uint64_t) * (kQ * kQ + 1)));
        HIP_TRY(x->f_rec.ensure(sizeof(uint64_t) * K * (size_t)std::max<int64_t>(acc, 1)));
        HIP_TRY(x->f_bstart.ensure(sizeof(int64_t) * (size_t)dirs));
        HIP_TRY(x->f_bhdr.ensure(sizeof(uint32_t) * kHdr * (size_t)dirs));
        HIP_TRY(x->f_nblk.ensure(sizeof(int32_t) * (size_t)grid_a + sizeof(unsigned long long)));
        HIP_TRY(x->f_cnt3.ensure(sizeof(uint32_t) * cnt3.size()));
        uint8_t* wgp = (uint8_t*)x->f_wg.p;
        int32_t* d_wg_lang = (int32_t*)(wgp + sizeof(int64_t) * meta.size());
        int32_t* d_perm = d_wg_lang + n_lang;
        {  // the plan through pinned staging: one asynchronous copy (the
           // previous batch's copy completed before its kernels, which the
           // host waited for)
            uint8_t* h = (uint8_t*)x->h_fwg.p;
            memcpy(h, meta.data(), sizeof(int64_t) * meta.size());
            memcpy(h + sizeof(int64_t) * meta.size(), wg_lang.data(), sizeof(int32_t) * n_lang);
            memcpy(h + sizeof(int64_t) * meta.size() + sizeof(int32_t) * n_lang, plen.data(), sizeof(int32_t) * n_perm);
            HIP_TRY(hipMemcpyAsync(wgp, h, wg_bytes, hipMemcpyHostToDevice, st));
        }
        HIP_TRY(hipMemsetAsync(x->f_cnt3.p, 0, sizeof(uint32_t) * cnt3.size(), st));
        PartParams pp{};
        pp.bytes = d_bytes;
        pp.last_dword = n_bytes > 0 ? (n_bytes - 1) >> 2 : 0;
        pp.offsets = d_offsets + d0;
        pp.doc_lang = d_lang + d0;
        pp.L = c->L;
        pp.nG = c->nG;
        for (int i = 0; i < c->nG; ++i) pp.G[i] = c->G[i];
        pp.maxg = maxg;
        pp.lb = c->lb;
        pp.cb = c->cb;
        if (const char* ab = diag_env("LDGPU_FIT_EMIT_ABLATE")) pp.ablate = atoi(ab);
        pp.grid_a = grid_a;
        pp.dlen = d_perm;
        pp.wg_lang = d_wg_lang;
        pp.wg_doc = (const int64_t*)wgp;
        pp.wg_rec = pp.wg_doc + grid_a + 1;
        pp.wg_dir = pp.wg_rec + grid_a + 1;
        pp.dstart = pp.wg_dir + grid_a + 1;
        pp.rec = (uint64_t*)x->f_rec.p;
        pp.blk_start = (int64_t*)x->f_bstart.p;
        pp.blk_hdr = (uint32_t*)x->f_bhdr.p;
        pp.nblk = (int32_t*)x->f_nblk.p;
        pp.cnt3 = (uint32_t*)x->f_cnt3.p;
        // exact bucket offsets ((q1, q2) major, emit group minor) are scanned
        // on the device, so emit, part2 and reduce run back to back; the
        // bucket scratch is sized by the batch's positions (records <= them)
        HIP_TRY(x->f_p2.ensure(sizeof(uint64_t) * p2off.size()));
        HIP_TRY(x->f_boff.ensure(sizeof(uint64_t) * boff.size()));
        HIP_TRY(x->f_rec2.ensure(sizeof(uint64_t) * K * (size_t)std::max<int64_t>(acc, 1)));
        HIP_TRY(x->f_okl.ensure(sizeof(uint64_t) * out_words(K) * (size_t)std::max<int64_t>(acc, 1)));
        HIP_TRY(x->f_on.ensure(sizeof(uint32_t) * kQ * kQ + sizeof(uint64_t) * (kQ * kQ + 1)));
        pp.p2off = (const uint64_t*)x->f_p2.p;
        pp.rec2 = (uint64_t*)x->f_rec2.p;
        pp.boff = (const uint64_t*)x->f_boff.p;
        pp.out = (uint64_t*)x->f_okl.p;
        pp.nout = (uint32_t*)x->f_on.p;
        std::vector<uint32_t> nout((size_t)kQ * kQ, 0u);
        if (acc > 0) {
            HIP_TRY(launch_emit(K, pp, st));
            HIP_TRY(launch_fit_offsets(pp, st));
            HIP_TRY(launch_part2(K, pp, st));
            HIP_TRY(launch_reduce(K, pp, st));
            // into pinned memory: a copy to pageable memory would wait for the
            // kernels here, before the next batch's plan
            HIP_TRY(hipMemcpyAsync(x->h_fon.p, pp.nout, sizeof(uint32_t) * nout.size(), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync((uint8_t*)x->h_fon.p + sizeof(uint32_t) * nout.size(), pp.boff,
                                   sizeof(uint64_t) * boff.size(), hipMemcpyDeviceToHost, st));
        } else {
            std::fill(boff.begin(), boff.end(), 0ull);
        }
        const bool more = d1 < n_docs;
        if (trace) tt[1] = now_ms();
        if (more) make_plan(d1, nxt);  // (host work while the GPU runs this batch)
        if (trace) tt[2] = now_ms();
        HIP_TRY(hipStreamSynchronize(st));
        if (trace) tt[3] = now_ms();
        if (acc > 0) {
            memcpy(nout.data(), x->h_fon.p, sizeof(uint32_t) * nout.size());
            memcpy(boff.data(), (uint8_t*)x->h_fon.p + sizeof(uint32_t) * nout.size(), sizeof(uint64_t) * boff.size());
        }
        if (int rc = settle_t1()) return rc;  // the previous batch's last merge
        const int64_t R = (int64_t)boff[(size_t)kQ * kQ];
        if (R > acc) return fail(LDGPU_EDEVICE, "fit emit: %lld records from %lld positions", (long long)R, (long long)acc);
        unsigned long long E = 0;
        for (int b = 0; b < kQ * kQ; ++b) {
            if (nout[b] > boff[b + 1] - boff[b])
                return fail(LDGPU_EDEVICE, "fit reduce: bucket %d wrote %u entries from %llu records", b, nout[b],
                            (unsigned long long)(boff[b + 1] - boff[b]));
            E += nout[b];
        }
        // The merge into T1 in chunks, each small enough that even if every
        // entry of it were a new key a table would stay within 0.1 of its load
        // limit (probes stay short and rarely reach the overflow list -- which
        // catches them), doubling a table once it is past the limit: the table
        // grows with the keys actually inserted, not with the batch's entries
        // (most of which find their key; a slot holds a dense row of L
        // counters, 1.6 KB at L = 200).
        // T1's wide table: windows of 8..15 bytes, or every pair (K = 2)
        const bool wide = (K == 3 && maxg > kMaxGram) || K == 2;
        if (wide) {
            if (int rc = wide_ensure(t1, K == 2 ? (uint64_t)std::max<int64_t>(t1_hint, 1) : 1)) return rc;
        }
        // Projected growth: the batch adds about E x (the last batch's new
        // keys per entry) keys.  A table short of that grows once, here --
        // doubling through the chunks would rehash what it holds each time
        // (an empty table's first grow is only an allocation).  If the
        // projection cannot be allocated, the chunks grow as they need.
        {
            const double est = (double)t1->size + t1->new_per_entry * (double)E;
            if (est > max_load(t1) * (double)t1->cap) {
                const uint64_t slot = 8ull + 8ull * (uint64_t)t1->L;
                uint64_t target = next_pow2((uint64_t)(est / 0.5) + 1);
                if (target * slot > kBigTableBytes) target = next_pow2((uint64_t)(est / 0.8) + 1);
                if (target > t1->cap && grow(t1, target) != LDGPU_OK) {
                    (void)hipGetLastError();  // (a failed allocation's sticky error)
                    (void)ok();
                }
            }
        }
        const uint64_t size0 = t1->size + t1->wsize;
        // (no entries: nout on the device is the last batch's, reduce did not run)
        if (trace) tt[4] = now_ms();
        for (int b0 = E ? 0 : kQ * kQ; b0 < kQ * kQ;) {
            while ((double)t1->size > max_load(t1) * (double)t1->cap) {
                if (int rc = grow(t1, 2 * t1->cap)) return rc;
            }
            if (wide) {
                if (int rc = wide_ensure(t1, 0)) return rc;  // past its load limit: grows
            }
            // the wide table's ceiling for a chunk: 3/4 (load limit 1/2), 0.9 (0.8)
            const double wceil = wide ? std::min(0.9, 1.5 * load_limit(t1->wcap, 16ull + 8ull * (uint64_t)t1->L)) : 0.0;
            const double ceil_load = max_load(t1) + 0.1;
            int64_t room = (int64_t)(ceil_load * (double)t1->cap) - (int64_t)t1->size;
            if (wide) room = std::min<int64_t>(room, (int64_t)(wceil * (double)t1->wcap) - (int64_t)t1->wsize);
            // buckets b0 .. b1 (at least one) whose entries fit the room
            int b1 = b0;
            int64_t n = 0;
            while (b1 < kQ * kQ && (b1 == b0 || n + (int64_t)nout[b1] <= room)) n += nout[b1++];
            if (wide && (double)(t1->wsize + (uint64_t)n) > wceil * (double)t1->wcap) {  // one bucket beyond the room
                if (int rc = wide_ensure(t1, (uint64_t)n)) return rc;
            }
            if (int rc = ensure_ovf(t1, std::max<int64_t>(n, 1))) return rc;
            HIP_TRY(hipMemsetAsync(t1->d_ovf_n, 0, sizeof(unsigned int), st));
            HIP_TRY(launch_merge(K, pp, count_params(t1), wide_params(t1), b0, b1, K <= 2, st));
            if (wide) {
                if (int rc = wide_after(t1)) return rc;
            }
            if (!wide && more && b1 == kQ * kQ) {
                t1_pending = true;  // settled after the next batch's reduce
            } else if (int rc = after_batch(t1)) {
                return rc;
            }
            b0 = b1;
        }
        if (t1_pending) {
            pend_size0 = size0;
            pend_E = E;
        } else if (E) {
            t1->new_per_entry = std::max(0.02, (double)(t1->size + t1->wsize - size0) / (double)E);
        }
        if (trace) {
            tt[5] = now_ms();
            fprintf(stderr, "fit batch: upload+launch %.3f plan %.3f gpu-wait %.3f pre-merge %.3f merge %.3f ms\n",
                    tt[1] - tt[0], tt[2] - tt[1], tt[3] - tt[2], tt[4] - tt[3], tt[5] - tt[4]);
        }
        if (!more) break;
        std::swap(cur, nxt);
    }
    // every gram length from the call's maximal windows; T1 back to the
    // context's block cache (the next call starts an empty one, sized by this)
    c->pend_hint = (int64_t)(c->pend->size + c->pend->wsize);  // (before the derive's levels replace T1)
    if (call_bytes > 0) {
        x->t1_keys_per_byte = (double)c->pend_hint / (double)call_bytes;
        x->t1_keys = c->pend_hint;
    }
    // the cached top-K table and sparse export describe the table before this
    // call: invalid from here on, even if the derive fails part way through
    c->tbl_valid = false;
    c->sp_valid = false;
    const int rc = derive_pending(c);
    counts_free(c->pend);
    c->pend = nullptr;
    return rc;
}

// Count documents [0, n_docs) of d_offsets / d_lang (h_off / h_lang: the
// same offsets and languages on the host, used to plan the batches): FIT v3
// for every gram length; the diagnostics build's LDGPU_FIT_LEGACY runs the
// round-1 atomic kernels instead (one-word lengths, then the wide ones).
int count_launch_narrow(ldgpu_counts* c, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                        const int32_t* d_lang, int64_t n_docs, const int64_t* h_off, hipStream_t st);

int count_launch(ldgpu_counts* c, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                 const int32_t* d_lang, int64_t n_docs, const int64_t* h_off, const int32_t* h_lang, hipStream_t st) {
    if (st != c->ctx->stream) HIP_TRY(hipStreamSynchronize(st));  // inputs were written on the caller's stream
    // the cached fit table and sparse copy describe the counts before this
    // call, which may fail part-way through changing them
    c->tbl_valid = false;
    c->sp_valid = false;
    if (c->v3 && sort_path(c)) return count_launch_sorted(c, d_bytes, n_bytes, d_offsets, d_lang, n_docs, h_off, h_lang);
    if (c->v3) return count_launch_v3(c, d_bytes, n_bytes, d_offsets, d_lang, n_docs, h_off, h_lang);
    if (c->nGn > 0) {
        if (int rc = count_launch_narrow(c, d_bytes, n_bytes, d_offsets, d_lang, n_docs, h_off, c->ctx->stream))
            return rc;
    }
    if (c->nGw > 0) {
        if (int rc = wide_count_launch(c, d_bytes, n_bytes, d_offsets, d_lang, n_docs, h_off)) return rc;
    }
    return LDGPU_OK;
}

int count_launch_narrow(ldgpu_counts* c, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                        const int32_t* d_lang, int64_t n_docs, const int64_t* h_off, hipStream_t st) {
    int64_t total = 0;
    for (int64_t d = 0; d < n_docs; ++d) total += doc_windows(c, h_off[d + 1] - h_off[d]);
    if (int rc = ensure_ovf(c, total)) return rc;
    int64_t d0 = 0;
    while (d0 < n_docs) {
        // also keep a launch within ~8 windows per slot of the current table:
        // a launch much larger than the table overflows most of its new keys
        // (re-inserted after a grow sized by the overflow count, i.e. far too big)
        const int64_t limit = std::min<int64_t>((int64_t)c->ovf_cap, std::max<int64_t>(1 << 24, 8 * (int64_t)c->cap));
        int64_t d1 = d0, win = 0;
        while (d1 < n_docs) {
            const int64_t w = doc_windows(c, h_off[d1 + 1] - h_off[d1]);
            if (d1 > d0 && win + w > limit) break;
            win += w;
            ++d1;
        }
        // a single document larger than the overflow list: make room up front
        if (win > (int64_t)c->ovf_cap) {
            if (int rc = grow(c, next_pow2(4 * (c->size + (uint64_t)win) + 16))) return rc;
        }
        CountParams p = count_params(c);
        p.bytes = d_bytes;
        p.last_dword = n_bytes > 0 ? (n_bytes - 1) >> 2 : 0;
        p.offsets = d_offsets + d0;
        p.doc_lang = d_lang + d0;
        p.n_docs = d1 - d0;
        const int64_t want = (p.n_docs + kCountWaves - 1) / kCountWaves;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)c->ctx->cus * 2));
        HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
        HIP_TRY(launch_count(p, grid, st));
        if (st != c->ctx->stream) HIP_TRY(hipStreamSynchronize(st));
        if (int rc = after_batch(c)) return rc;
        d0 = d1;
    }
    return LDGPU_OK;
}
}  // namespace

extern "C" int ldgpu_counts_create(ldgpu_ctx* ctx, int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams,
                                   int64_t capacity_hint, ldgpu_counts** out) {
    if (!ctx || !out) return fail(LDGPU_EINVAL, "ctx/out is NULL");
    if (n_langs < 1 || n_langs > LDGPU_MAX_LANGS)
        return fail(n_langs < 1 ? LDGPU_EINVAL : LDGPU_EUNSUPPORTED, "n_langs %d outside [1, %d]", n_langs,
                    LDGPU_MAX_LANGS);
    if (int rc = check_grams(gram_lengths, n_grams, LDGPU_MAX_FIT_GRAM)) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = counts_new(ctx, n_langs, gram_lengths, n_grams, capacity_hint, out, true)) return rc;
    return ok();
}

namespace {
// a count table (validated arguments; the caller has set the device)
int counts_new(ldgpu_ctx* ctx, int32_t n_langs, const int32_t* gram_lengths, int32_t n_grams, int64_t capacity_hint,
               ldgpu_counts** out, bool sparse) {
    auto* c = new ldgpu_counts();
    c->ctx = ctx;
    c->L = n_langs;
    c->sparse = sparse;
    // G: the lengths of <= 15 bytes (FIT v4: maximal windows); Gl: longer
    // ones (ldgpu_long.hip); Gall: all, in the caller's order
    c->nGall = n_grams;
    for (int i = 0; i < n_grams; ++i) {
        c->Gall[i] = gram_lengths[i];
        if (gram_lengths[i] > kMaxWideGram) {
            c->Gl[c->nGl++] = gram_lengths[i];
            continue;
        }
        c->G[c->nG++] = gram_lengths[i];
        if (gram_lengths[i] <= kMaxGram)
            c->Gn[c->nGn++] = gram_lengths[i];
        else
            c->Gw[c->nGw++] = gram_lengths[i];
    }
    c->cap = next_pow2(std::max<int64_t>(1 << 12, 2 * std::max<int64_t>(capacity_hint, 0)));
    // FIT v3 record form (ldgpu_internal.h): the compact one-word record when
    // 8 max(G) + 1 sentinel-key bits + ceil(log2 L) language bits leave >= 8
    // count bits, two words for any other table of grams <= 7 bytes, three
    // with grams of 8..15 bytes
    {
        int maxg = 0;
        for (int i = 0; i < c->nG; ++i) maxg = std::max(maxg, c->G[i]);
        c->lb = (uint32_t)std::max(1, log2u((uint64_t)n_langs));
        const int cb = 64 - (8 * std::min(maxg, kMaxGram) + 1) - (int)c->lb;
        c->cb = (uint32_t)std::max(cb, 0);
        c->K = maxg > kMaxGram ? 3 : (cb >= 8 ? 1 : 2);
        if (const char* k = diag_env("LDGPU_FIT_K")) c->K = std::max(c->K, std::min(3, atoi(k)));  // tests: wider forms
        c->v3 = !diag_env("LDGPU_FIT_LEGACY");
        c->batch_recs = kBatchRecords / c->K;
        if (const char* bw = diag_env("LDGPU_FIT_BATCH_WINDOWS")) c->batch_recs = std::max(1ll, atoll(bw));
        if (c->v3) {
            const hipError_t pe = fit3_prepare(c->K);  // dynamic-LDS limits of this device's kernels
            if (pe != hipSuccess) {
                delete c;
                return fail(LDGPU_EDEVICE, "fit kernels: %s", hipGetErrorString(pe));
            }
        }
    }
    int rc = sparse ? alloc_table(c, c->cap, &c->d_keys, reinterpret_cast<void**>(&c->d_kcnt))
                    : alloc_table(c, c->cap, &c->d_keys, reinterpret_cast<void**>(&c->d_counts));
    if (!rc && sparse) {
        c->pcap = c->cap;
        rc = alloc_pairs(c, c->pcap, &c->d_pkeys, &c->d_pcounts);
    }
    hipError_t e = hipSuccess;
    if (!rc) e = hipMalloc((void**)&c->d_size, sizeof(unsigned long long));
    if (!rc && e == hipSuccess && sparse) e = hipMalloc((void**)&c->d_psize, sizeof(unsigned long long));
    if (!rc && e == hipSuccess && sparse) e = hipMemsetAsync(c->d_psize, 0, sizeof(unsigned long long), ctx->stream);
    if (!rc && e == hipSuccess) e = cache_alloc(c->ctx, (void**)&c->d_ovf_keys, sizeof(uint64_t) * c->ovf_cap);
    if (!rc && e == hipSuccess) e = cache_alloc(c->ctx, (void**)&c->d_ovf_lang, sizeof(int32_t) * c->ovf_cap);
    if (!rc && e == hipSuccess)
        e = cache_alloc(c->ctx, (void**)&c->d_ovf_cnt, sizeof(unsigned long long) * c->ovf_cap);
    if (!rc && e == hipSuccess) e = hipMalloc((void**)&c->d_ovf_n, sizeof(unsigned int));
    if (!rc && e == hipSuccess) e = hipMemsetAsync(c->d_size, 0, sizeof(unsigned long long), ctx->stream);
    if (!rc && e == hipSuccess) e = hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), ctx->stream);
    if (!rc && e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (rc || e != hipSuccess) {
        counts_free(c);
        return rc ? rc : fail(LDGPU_ENOMEM, "count table: %s", hipGetErrorString(e));
    }
    *out = c;
    return LDGPU_OK;
}
}  // namespace

extern "C" int ldgpu_counts_langs(const ldgpu_counts* c, int32_t* n_langs) {
    if (!c || !n_langs) return fail(LDGPU_EINVAL, "counts/n_langs is NULL");
    *n_langs = c->L;
    return ok();
}

extern "C" int ldgpu_counts_destroy(ldgpu_counts* c) {
    counts_free(c);
    return ok();
}

extern "C" int ldgpu_count_device(ldgpu_counts* c, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_offsets,
                                  const int32_t* d_doc_lang, int64_t n_docs, void* stream) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    if (c->comm) return fail(LDGPU_EINVAL, "the count table is merged (ldgpu_counts_merge): it takes no more counts");
    if (n_docs < 0) return fail(LDGPU_EINVAL, "n_docs < 0");
    if (n_docs > 0 && (!d_offsets || !d_doc_lang || (n_bytes > 0 && !d_bytes)))
        return fail(LDGPU_EINVAL, "device pointer is NULL");
    if (((uintptr_t)d_bytes & 3) != 0) return fail(LDGPU_EINVAL, "d_bytes must be 4-byte aligned");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    hipStream_t st = (hipStream_t)stream;
    if (n_docs == 0) return ok();
    c->tbl_valid = false;  // a count changes the table, whatever happens below
    c->sp_valid = false;
    std::vector<int64_t> h_off(n_docs + 1);
    std::vector<int32_t> h_lang(n_docs);
    HIP_TRY(hipMemcpyAsync(h_off.data(), d_offsets, sizeof(int64_t) * (n_docs + 1), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(h_lang.data(), d_doc_lang, sizeof(int32_t) * n_docs, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (int rc = count_launch(c, d_bytes, n_bytes, d_offsets, d_doc_lang, n_docs, h_off.data(), h_lang.data(), st))
        return rc;
    return ok();
}

extern "C" int ldgpu_count(ldgpu_counts* c, const uint8_t* bytes, const int64_t* offsets, const int32_t* doc_lang,
                           int64_t n_docs) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    if (c->comm) return fail(LDGPU_EINVAL, "the count table is merged (ldgpu_counts_merge): it takes no more counts");
    if (int rc = check_offsets(offsets, n_docs)) return rc;
    if (n_docs == 0) return ok();
    if (!doc_lang) return fail(LDGPU_EINVAL, "doc_lang is NULL");
    if (!bytes && offsets[n_docs] > offsets[0]) return fail(LDGPU_EINVAL, "bytes is NULL");
    ldgpu_ctx* x = c->ctx;
    std::lock_guard<std::mutex> lock(x->mu);
    HIP_TRY(hipSetDevice(x->device));
    c->tbl_valid = false;  // a count changes the table, whatever happens below
    c->sp_valid = false;
    const int64_t kChunkBytes = 64ll << 20, kChunkDocs = 4ll << 20;
    std::vector<int64_t> off;
    int64_t d0 = 0;
    while (d0 < n_docs) {
        int64_t d1 = d0 + 1;
        while (d1 < n_docs && d1 - d0 < kChunkDocs && offsets[d1 + 1] - offsets[d0] <= kChunkBytes) ++d1;
        const int64_t nd = d1 - d0, b0 = offsets[d0], nb = offsets[d1] - b0;
        off.resize(nd + 1);
        for (int64_t i = 0; i <= nd; ++i) off[i] = offsets[d0 + i] - b0;
        HIP_TRY(x->bytes.ensure((size_t)nb + 16));
        HIP_TRY(x->offsets.ensure(sizeof(int64_t) * (nd + 1)));
        HIP_TRY(x->langs.ensure(sizeof(int32_t) * nd));
        if (nb) HIP_TRY(hipMemcpyAsync(x->bytes.p, bytes + b0, nb, hipMemcpyHostToDevice, x->stream));
        HIP_TRY(hipMemcpyAsync(x->offsets.p, off.data(), sizeof(int64_t) * (nd + 1), hipMemcpyHostToDevice,
                               x->stream));
        HIP_TRY(hipMemcpyAsync(x->langs.p, doc_lang + d0, sizeof(int32_t) * nd, hipMemcpyHostToDevice, x->stream));
        if (int rc = count_launch(c, (const uint8_t*)x->bytes.p, nb, (const int64_t*)x->offsets.p,
                                  (const int32_t*)x->langs.p, nd, off.data(), doc_lang + d0, x->stream))
            return rc;
        d0 = d1;
    }
    return ok();
}

namespace {
// device scratch freed on scope exit; with a context, the blocks come from
// and go back to its cache (a fit's scratch has the same sizes fit after fit:
// no hipMalloc / hipFree per call).  Blocks go back once the caller's work on
// the context's stream is queued; later users of the stream run after it.
struct DevBufs {
    ldgpu_ctx* ctx = nullptr;
    std::vector<std::pair<void*, size_t>> p;
    ~DevBufs() {
        for (auto& x : p) {
            if (!x.first) continue;
            if (ctx)
                cache_free(ctx, x.first, x.second);
            else
                (void)hipFree(x.first);
        }
    }
    template <typename T>
    hipError_t alloc(T** out, size_t n) {
        void* x = nullptr;
        const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        hipError_t e = ctx ? cache_alloc(ctx, &x, bytes) : hipMalloc(&x, bytes);
        if (e == hipSuccess) p.emplace_back(x, bytes);
        *out = (T*)x;
        return e;
    }
};

// the wide table's occupied slots (unordered): lo, hi, counts rows
int wide_export(ldgpu_counts* c, std::vector<uint64_t>& wlo, std::vector<uint64_t>& whi,
                std::vector<unsigned long long>& wc) {
    const uint64_t nw = c->wsize;
    wlo.assign(nw, 0);
    whi.assign(nw, 0);
    wc.assign((size_t)nw * c->L, 0);
    if (!nw) return LDGPU_OK;
    DevBufs wb;
    uint64_t *d_lo, *d_hi;
    unsigned long long *d_wc, *d_wn;
    HIP_TRY(wb.alloc(&d_lo, nw));
    HIP_TRY(wb.alloc(&d_hi, nw));
    HIP_TRY(wb.alloc(&d_wc, (size_t)nw * c->L));
    HIP_TRY(wb.alloc(&d_wn, 1));
    hipStream_t st = c->ctx->stream;
    HIP_TRY(hipMemsetAsync(d_wn, 0, sizeof(unsigned long long), st));
    HIP_TRY(launch_wide_compact(wide_params(c), c->wcap, d_lo, d_hi, d_wc, d_wn, st));
    unsigned long long got = 0;
    HIP_TRY(hipMemcpyAsync(&got, d_wn, sizeof got, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(wlo.data(), d_lo, nw * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(whi.data(), d_hi, nw * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(wc.data(), d_wc, nw * c->L * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (got != nw)
        return fail(LDGPU_EDEVICE, "wide count export: %llu slots occupied, %llu expected", got, (unsigned long long)nw);
    return LDGPU_OK;
}

// the (length, bytes) order of wide keys: length, then bytes 0..7, then 8..
std::vector<uint64_t> wide_order(const std::vector<uint64_t>& wlo, const std::vector<uint64_t>& whi) {
    auto be = [](uint64_t x) { return __builtin_bswap64(x); };
    std::vector<uint64_t> word(wlo.size());
    for (uint64_t i = 0; i < word.size(); ++i) word[i] = i;
    std::sort(word.begin(), word.end(), [&](uint64_t a, uint64_t b) {
        const int la = key_len(whi[a]), lb = key_len(whi[b]);
        if (la != lb) return la < lb;
        if (wlo[a] != wlo[b]) return be(wlo[a]) < be(wlo[b]);
        return be(whi[a] << 8) < be(whi[b] << 8);
    });
    return word;
}

// the packed key of a sort_key (ldgpu_common.h): length in the top byte,
// bytes big-endian below it
uint64_t unsort_key(uint64_t s) {
    const int len = key_len(s);
    uint64_t k = (uint64_t)len << 56;
    for (int i = 0; i < len; ++i) k |= ((s >> (48 - 8 * i)) & 0xffull) << (8 * i);
    return k;
}

// The grams of 8 or more bytes (the wide table's, 8..15, and the long
// table's, 16..), unordered, as byte strings with their nonzero (language,
// count) pairs in language order (gram i: [poff[i], poff[i + 1])).
struct Ext {
    std::vector<std::string> keys;
    std::vector<int64_t> poff{0};
    std::vector<int32_t> lang;
    std::vector<int64_t> cnt;
};

std::string wide_bytes(uint64_t lo, uint64_t hi) {
    const int len = key_len(hi);
    std::string k((size_t)len, '\0');
    for (int j = 0; j < len; ++j) k[j] = (char)(uint8_t)((j < 8 ? lo : hi) >> (8 * (j & 7)));
    return k;
}

// the long table on the host: its grams (slot order) and pairs
int long_export(ldgpu_counts* c, Ext& x, bool with_pairs) {
    if (!c->lsize) return LDGPU_OK;
    hipStream_t st = c->ctx->stream;
    std::vector<LongSlot> slots(c->lcap);
    std::vector<uint8_t> arena(std::max<uint64_t>(c->larena_n, 1));
    HIP_TRY(hipMemcpyAsync(slots.data(), c->d_lslots, c->lcap * sizeof(LongSlot), hipMemcpyDeviceToHost, st));
    if (c->larena_n) HIP_TRY(hipMemcpyAsync(arena.data(), c->d_larena, c->larena_n, hipMemcpyDeviceToHost, st));
    std::vector<uint64_t> pk;
    std::vector<unsigned long long> pc;
    if (with_pairs) {
        pk.resize(c->lpcap);
        pc.resize(c->lpcap);
        HIP_TRY(hipMemcpyAsync(pk.data(), c->d_lpkeys, c->lpcap * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(pc.data(), c->d_lpcounts, c->lpcap * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<int64_t> idx(c->lcap, -1);
    const size_t base = x.keys.size();
    for (uint64_t s = 0; s < c->lcap; ++s) {
        if (!slots[s].h) continue;
        const uint64_t off = slots[s].meta >> kLongLenBits, len = slots[s].meta & ((1ull << kLongLenBits) - 1);
        if (off + len > c->larena_n) return fail(LDGPU_EDEVICE, "long gram table: slot %llu outside the arena",
                                                 (unsigned long long)s);
        idx[s] = (int64_t)(x.keys.size() - base);
        x.keys.emplace_back((const char*)arena.data() + off, (size_t)len);
    }
    const size_t ng = x.keys.size() - base;
    if (ng != c->lsize) return fail(LDGPU_EDEVICE, "long gram table: %zu grams, %llu expected", ng,
                                    (unsigned long long)c->lsize);
    std::vector<std::vector<std::pair<int32_t, int64_t>>> per(ng);
    for (uint64_t i = 0; i < pk.size(); ++i) {
        if (!pk[i]) continue;
        const uint64_t g = (pk[i] >> kPairLangBits) - 1;
        if (g >= c->lcap || idx[g] < 0) return fail(LDGPU_EDEVICE, "long gram table: pair of an empty slot");
        per[idx[g]].push_back({(int32_t)(pk[i] & ((1ull << kPairLangBits) - 1)), (int64_t)pc[i]});
    }
    for (size_t g = 0; g < ng; ++g) {
        std::sort(per[g].begin(), per[g].end());
        for (auto& q : per[g]) {
            x.lang.push_back(q.first);
            x.cnt.push_back(q.second);
        }
        x.poff.push_back((int64_t)x.lang.size());
    }
    return LDGPU_OK;
}

// the wide and long grams (unordered), with their pairs when with_pairs
int ext_export(ldgpu_counts* c, Ext& x, bool with_pairs) {
    std::vector<uint64_t> wlo, whi;
    std::vector<unsigned long long> wc;
    if (int rc = wide_export(c, wlo, whi, wc)) return rc;
    const int L = c->L;
    for (size_t i = 0; i < wlo.size(); ++i) {
        x.keys.push_back(wide_bytes(wlo[i], whi[i]));
        if (with_pairs)
            for (int l = 0; l < L; ++l) {
                if (!wc[i * L + l]) continue;
                x.lang.push_back(l);
                x.cnt.push_back((int64_t)wc[i * L + l]);
            }
        x.poff.push_back((int64_t)x.lang.size());
    }
    return long_export(c, x, with_pairs);
}

// The table pulled to the host in (length, bytes) order -- the rows of
// reduceGrams (LanguageDetector.scala:57-65): every gram (one-word key, or a
// stand-in kWideTag << 56 | rank, c->ext_sorted[rank]) and its nonzero
// (language, count) pairs in language order (pairs of gram i: [poff[i],
// poff[i + 1])).  with_pairs = false: the keys only.
struct Pulled {
    std::vector<uint64_t> keys;
    std::vector<int64_t> poff;
    std::vector<int32_t> lang;
    std::vector<int64_t> cnt;
};

int counts_pull(ldgpu_counts* c, Pulled& out, bool with_pairs = true) {
    const uint64_t n = c->size, np = c->psize;
    hipStream_t st = c->ctx->stream;
    std::vector<uint64_t> sk(n), pk;
    std::vector<unsigned long long> pc;
    if (n) {
        // the grams' sort keys ordered on the device, each gram slot's rank, then
        // the pairs keyed (rank, language) and ordered the same way
        DevBufs db;
        db.ctx = c->ctx;
        uint64_t *d_sk, *d_slot;
        uint32_t* d_rank;
        unsigned long long* d_n;
        HIP_TRY(db.alloc(&d_sk, n));
        HIP_TRY(db.alloc(&d_slot, n));
        HIP_TRY(db.alloc(&d_rank, c->cap));
        HIP_TRY(db.alloc(&d_n, 2));
        HIP_TRY(hipMemsetAsync(d_n, 0, 2 * sizeof(unsigned long long), st));
        HIP_TRY(launch_gram_compact(count_params(c), c->cap, d_sk, d_slot, d_n, true, st));
        unsigned long long got = 0;
        HIP_TRY(hipMemcpyAsync(&got, d_n, sizeof got, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (got != n)
            return fail(LDGPU_EDEVICE, "count export: %llu grams, %llu expected", got, (unsigned long long)n);
        HIP_TRY(sort_pairs_u64((int64_t)n, d_sk, reinterpret_cast<unsigned long long*>(d_slot), 59, st));
        HIP_TRY(hipMemcpyAsync(sk.data(), d_sk, n * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        if (with_pairs && np) {
            uint64_t* d_pk;
            unsigned long long* d_pc;
            HIP_TRY(db.alloc(&d_pk, np));
            HIP_TRY(db.alloc(&d_pc, np));
            HIP_TRY(launch_rank_scatter((int64_t)n, d_slot, d_rank, st));
            HIP_TRY(launch_pair_compact(count_params(c), c->pcap, d_rank, d_pk, d_pc, d_n + 1, st));
            HIP_TRY(hipMemcpyAsync(&got, d_n + 1, sizeof got, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (got != np)
                return fail(LDGPU_EDEVICE, "count export: %llu pairs, %llu expected", got, (unsigned long long)np);
            HIP_TRY(sort_pairs_u64((int64_t)np, d_pk, d_pc, (int)kPairLangBits + log2u(n + 1) + 1, st));
            pk.resize(np);
            pc.resize(np);
            HIP_TRY(hipMemcpyAsync(pk.data(), d_pk, np * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(pc.data(), d_pc, np * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        }
        HIP_TRY(hipStreamSynchronize(st));
    }
    // the grams of 8 or more bytes (wide: 8..15, long: 16..) after them, in
    // (length, bytes) order, as stand-in keys kWideTag << 56 | rank
    // (c->ext_sorted[rank])
    Ext ext;
    if (int rc = ext_export(c, ext, with_pairs)) return rc;
    const uint64_t nx = ext.keys.size();
    std::vector<uint64_t> ord(nx);
    for (uint64_t i = 0; i < nx; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) {
        const std::string &x = ext.keys[a], &y = ext.keys[b];
        return x.size() != y.size() ? x.size() < y.size() : x < y;  // unsigned bytes: char_traits compares as unsigned
    });
    c->ext_sorted.resize(nx);
    out.keys.resize(n + nx);
    for (uint64_t i = 0; i < n; ++i) out.keys[i] = unsort_key(sk[i]);
    for (uint64_t r = 0; r < nx; ++r) {
        c->ext_sorted[r] = ext.keys[ord[r]];
        out.keys[n + r] = (kWideTag << 56) | r;
    }
    out.poff.clear();
    out.lang.clear();
    out.cnt.clear();
    if (!with_pairs) return LDGPU_OK;
    out.poff.assign(n + nx + 1, 0);
    out.lang.resize(pk.size());
    out.cnt.resize(pk.size());
    for (size_t j = 0; j < pk.size(); ++j) {
        const uint64_t r = pk[j] >> kPairLangBits;
        if (r >= n) return fail(LDGPU_EDEVICE, "count export: pair of gram %llu, %llu grams", (unsigned long long)r,
                                (unsigned long long)n);
        out.poff[r + 1]++;
        out.lang[j] = (int32_t)(pk[j] & ((1ull << kPairLangBits) - 1ull));
        out.cnt[j] = (int64_t)pc[j];
    }
    for (uint64_t i = 0; i < n; ++i) out.poff[i + 1] += out.poff[i];
    for (uint64_t r = 0; r < nx; ++r) {
        const uint64_t i = ord[r];
        for (int64_t j = ext.poff[i]; j < ext.poff[i + 1]; ++j) {
            out.lang.push_back(ext.lang[j]);
            out.cnt.push_back(ext.cnt[j]);
        }
        out.poff[n + r + 1] = (int64_t)out.lang.size();
    }
    return LDGPU_OK;
}

// bytes of a pulled key (one-word, or a wide stand-in resolved through
// c->ext_sorted): returns the length, writes the bytes when out != nullptr
int gram_bytes(const ldgpu_counts* c, uint64_t k, uint8_t* out) {
    if (key_len(k) < (int)kWideTag) {
        const int len = key_len(k);
        if (out)
            for (int j = 0; j < len; ++j) out[j] = (uint8_t)(k >> (8 * j));
        return len;
    }
    const std::string& w = c->ext_sorted[k & ((1ull << 56) - 1)];
    if (out) memcpy(out, w.data(), w.size());
    return (int)w.size();
}

void write_keys(const ldgpu_counts* c, const std::vector<uint64_t>& keys, uint8_t* key_bytes, int64_t* key_offsets) {
    int64_t o = 0;
    key_offsets[0] = 0;
    for (size_t i = 0; i < keys.size(); ++i) {
        o += gram_bytes(c, keys[i], key_bytes + o);
        key_offsets[i + 1] = o;
    }
}

// write_keys for one-word keys (<= 7 bytes, no wide stand-ins) from a plain
// array: offsets by a serial prefix sum of the lengths, the bytes in parallel
void write_short_keys(const uint64_t* keys, int64_t n, std::vector<uint8_t>& key_bytes, std::vector<int64_t>& key_offsets) {
    key_offsets.resize((size_t)n + 1);
    key_offsets[0] = 0;
    for (int64_t i = 0; i < n; ++i) key_offsets[i + 1] = key_offsets[i] + key_len(keys[i]);
    key_bytes.resize((size_t)std::max<int64_t>(key_offsets[n], 1));
    uint8_t* kb = key_bytes.data();
    const int64_t* ko = key_offsets.data();
    par_for(n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const uint64_t k = keys[i];
            for (int64_t j = 0; j < ko[i + 1] - ko[i]; ++j) kb[ko[i] + j] = (uint8_t)(k >> (8 * j));
        }
    });
}
}  // namespace

namespace {
// the pinned table's arrays (tbl_pin: ctx->h_tbl, owned by c)
struct PinnedTable {
    const uint64_t* keys;
    const uint64_t* masks;
    const int32_t* k;
};
PinnedTable pinned_table(const ldgpu_counts* c) {
    const int S = (c->L + 63) / 64;
    const uint64_t* keys = (const uint64_t*)c->ctx->h_tbl.p;
    const uint64_t* masks = keys + c->tbl_rows;
    return {keys, masks, (const int32_t*)(masks + (size_t)c->tbl_rows * S)};
}

double row_value(int k) { return std::log(1.0 + 1.0 / (double)k); }

// rows, key bytes of the cached table
int64_t tbl_rows(const ldgpu_counts* c) { return c->tbl_pin ? c->tbl_rows : (int64_t)c->tbl_off.size() - 1; }
int64_t tbl_key_bytes(const ldgpu_counts* c) { return c->tbl_pin ? c->tbl_kb : c->tbl_off.back(); }

// the pinned table into c's own vectors (before another table's build
// reuses the context's pinned buffer, or for the dense export)
void tbl_materialize(ldgpu_counts* c) {
    if (!c->tbl_pin) return;
    const PinnedTable t = pinned_table(c);
    const int64_t m = c->tbl_rows;
    const int S = (c->L + 63) / 64;
    c->tbl_masks.assign(t.masks, t.masks + (size_t)m * S);
    c->tbl_vals.resize((size_t)m);
    for (int64_t r = 0; r < m; ++r) c->tbl_vals[r] = row_value(t.k[r]);
    write_short_keys(t.keys, m, c->tbl_bytes, c->tbl_off);
    c->tbl_pin = false;
    if (c->ctx->h_tbl_owner == c) c->ctx->h_tbl_owner = nullptr;
}
}  // namespace

extern "C" int ldgpu_counts_size(ldgpu_counts* c, int64_t* n_grams, int64_t* key_bytes) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    if (n_grams) *n_grams = (int64_t)(c->size + c->wsize + c->lsize);
    if (key_bytes) {
        Pulled t;
        if (int rc = counts_pull(c, t, false)) return rc;
        int64_t s = 0;
        for (uint64_t x : t.keys) s += gram_bytes(c, x, nullptr);
        *key_bytes = s;
    }
    return ok();
}

extern "C" int ldgpu_counts_stats(ldgpu_counts* c, int64_t* n_grams, int64_t* n_pairs, int64_t* total) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    unsigned long long* d = nullptr;
    unsigned long long h[2] = {0, 0};
    HIP_TRY(hipMalloc((void**)&d, sizeof h));
    hipError_t e = hipMemsetAsync(d, 0, sizeof h, c->ctx->stream);
    // the sparse table's pairs (one counter each), the wide table's rows
    if (e == hipSuccess) e = launch_stats(pair_view(c), c->pcap, d, c->ctx->stream);
    if (e == hipSuccess && c->lpcap)  // the long grams' pairs
        e = launch_stats(pair_view_of(c->d_lpkeys, c->d_lpcounts, 0), c->lpcap, d, c->ctx->stream);
    if (e == hipSuccess && c->wcap) {  // the wide table, through the same kernel (hi != 0: occupied)
        CountParams w{};
        w.keys = c->d_whi;
        w.counts = c->d_wcounts;
        w.L = c->L;
        e = launch_stats(w, c->wcap, d, c->ctx->stream);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, c->ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->ctx->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(LDGPU_EDEVICE, "counts_stats: %s", hipGetErrorString(e));
    if (n_grams) *n_grams = (int64_t)(c->size + c->wsize + c->lsize);
    if (n_pairs) *n_pairs = (int64_t)h[0];
    if (total) *total = (int64_t)h[1];
    return ok();
}

extern "C" int ldgpu_counts_export(ldgpu_counts* c, uint8_t* key_bytes, int64_t* key_offsets, int64_t* counts_out) {
    if (!c || !key_offsets || !counts_out) return fail(LDGPU_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    Pulled t;
    if (int rc = counts_pull(c, t)) return rc;
    write_keys(c, t.keys, key_bytes, key_offsets);
    const int L = c->L;
    const size_t n = t.keys.size();
    memset(counts_out, 0, sizeof(int64_t) * n * (size_t)L);
    for (size_t i = 0; i < n; ++i)
        for (int64_t j = t.poff[i]; j < t.poff[i + 1]; ++j) counts_out[i * L + t.lang[j]] = t.cnt[j];
    return ok();
}

namespace {
// the sparse host copy (ldgpu_counts::sp_*), pulled once per table state
int sparse_pull(ldgpu_counts* c) {
    if (c->sp_valid) return LDGPU_OK;
    Pulled t;
    if (int rc = counts_pull(c, t)) return rc;
    const size_t n = t.keys.size();
    c->sp_keys = std::move(t.keys);
    c->sp_koff.assign(n + 1, 0);
    for (size_t i = 0; i < n; ++i) c->sp_koff[i + 1] = c->sp_koff[i] + gram_bytes(c, c->sp_keys[i], nullptr);
    c->sp_poff = std::move(t.poff);
    c->sp_lang = std::move(t.lang);
    c->sp_cnt = std::move(t.cnt);
    c->sp_valid = true;
    return LDGPU_OK;
}

int check_range(const ldgpu_counts* c, int64_t first, int64_t n) {
    const int64_t total = (int64_t)c->sp_keys.size();
    if (first < 0 || n < 0 || first > total || n > total - first)
        return fail(LDGPU_EINVAL, "gram range [%lld, %lld) outside [0, %lld)", (long long)first,
                    (long long)(first + n), (long long)total);
    return LDGPU_OK;
}

// (key, language, count) triples of one-word keys into the sparse table
// (nonzero counts; probe-limit overflows are re-inserted by after_batch)
int add_triples(ldgpu_counts* c, const std::vector<uint64_t>& tk, const std::vector<int32_t>& tl,
                const std::vector<unsigned long long>& tc) {
    const int64_t nt = (int64_t)tk.size();
    if (!nt) return LDGPU_OK;
    hipStream_t st = c->ctx->stream;
    if (int rc = reserve(c, (uint64_t)nt, (uint64_t)nt)) return rc;
    if (int rc = ensure_ovf(c, nt)) return rc;
    DevBufs tb;
    uint64_t* d_k;
    int32_t* d_l;
    unsigned long long* d_c;
    HIP_TRY(tb.alloc(&d_k, nt));
    HIP_TRY(tb.alloc(&d_l, nt));
    HIP_TRY(tb.alloc(&d_c, nt));
    HIP_TRY(hipMemcpyAsync(d_k, tk.data(), nt * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_l, tl.data(), nt * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_c, tc.data(), nt * sizeof(unsigned long long), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
    HIP_TRY(launch_counts_add(count_params(c), d_k, nullptr, d_l, d_c, nt, st));
    HIP_TRY(hipStreamSynchronize(st));
    return after_batch(c);
}

// dense rows of wide keys (8..15 bytes) into the wide table
int add_wide_rows(ldgpu_counts* c, const std::vector<uint64_t>& wlo, const std::vector<uint64_t>& whi,
                  const std::vector<unsigned long long>& wrows) {
    const int64_t nw = (int64_t)wlo.size();
    if (!nw) return LDGPU_OK;
    hipStream_t st = c->ctx->stream;
    if (int rc = wide_ensure(c, (uint64_t)nw)) return rc;
    DevBufs wb;
    uint64_t *d_lo, *d_hi;
    unsigned long long* d_r;
    HIP_TRY(wb.alloc(&d_lo, nw));
    HIP_TRY(wb.alloc(&d_hi, nw));
    HIP_TRY(wb.alloc(&d_r, (size_t)nw * c->L));
    HIP_TRY(hipMemcpyAsync(d_lo, wlo.data(), nw * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_hi, whi.data(), nw * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_r, wrows.data(), wrows.size() * sizeof(unsigned long long), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_wide_add(wide_params(c), d_lo, d_hi, d_r, nw, st));
    return wide_after(c);
}

uint64_t wide_lo_host(const uint8_t* kb) { return (pack_key_host(kb, 8) & ((1ull << 56) - 1)) | ((uint64_t)kb[7] << 56); }
uint64_t wide_hi_host(const uint8_t* kb, int64_t len) {
    return (pack_key_host(kb + 8, (int)len - 8) & ((1ull << 56) - 1)) | ((uint64_t)len << 56);
}
}  // namespace

extern "C" int ldgpu_counts_sparse_size(ldgpu_counts* c, int64_t first, int64_t n, int64_t* key_bytes,
                                        int64_t* n_pairs) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    if (int rc = sparse_pull(c)) return rc;
    if (int rc = check_range(c, first, n)) return rc;
    if (key_bytes) *key_bytes = c->sp_koff[first + n] - c->sp_koff[first];
    if (n_pairs) *n_pairs = c->sp_poff[first + n] - c->sp_poff[first];
    return ok();
}

extern "C" int ldgpu_counts_export_sparse(ldgpu_counts* c, int64_t first, int64_t n, uint8_t* key_bytes,
                                          int64_t* key_offsets, int64_t* pair_offsets, int32_t* pair_langs,
                                          int64_t* pair_counts) {
    if (!c || !key_offsets || !pair_offsets) return fail(LDGPU_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    if (int rc = sparse_pull(c)) return rc;
    if (int rc = check_range(c, first, n)) return rc;
    const int64_t k0 = c->sp_koff[first], p0 = c->sp_poff[first];
    const int64_t nk = c->sp_koff[first + n] - k0, np = c->sp_poff[first + n] - p0;
    if ((nk && !key_bytes) || (np && (!pair_langs || !pair_counts))) return fail(LDGPU_EINVAL, "NULL argument");
    for (int64_t i = 0; i < n; ++i) gram_bytes(c, c->sp_keys[first + i], key_bytes + c->sp_koff[first + i] - k0);
    for (int64_t i = 0; i <= n; ++i) {
        key_offsets[i] = c->sp_koff[first + i] - k0;
        pair_offsets[i] = c->sp_poff[first + i] - p0;
    }
    if (np) {
        memcpy(pair_langs, c->sp_lang.data() + p0, sizeof(int32_t) * (size_t)np);
        memcpy(pair_counts, c->sp_cnt.data() + p0, sizeof(int64_t) * (size_t)np);
    }
    return ok();
}

extern "C" int ldgpu_counts_add_sparse(ldgpu_counts* c, int64_t n, const uint8_t* key_bytes,
                                       const int64_t* key_offsets, const int64_t* pair_offsets,
                                       const int32_t* pair_langs, const int64_t* pair_counts) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    if (c->comm) return fail(LDGPU_EINVAL, "the count table is merged (ldgpu_counts_merge): it takes no more counts");
    if (n < 0) return fail(LDGPU_EINVAL, "n < 0");
    if (n == 0) return ok();
    if (!key_bytes || !key_offsets || !pair_offsets) return fail(LDGPU_EINVAL, "NULL argument");
    const int64_t np = pair_offsets[n] - pair_offsets[0];
    if (np < 0 || (np && (!pair_langs || !pair_counts))) return fail(LDGPU_EINVAL, "bad pair offsets / NULL pairs");
    // one-word keys as (key, language, count) triples; wide keys as dense
    // rows; longer keys as triples with their bytes
    std::vector<uint64_t> tk, wlo, whi;
    std::vector<int32_t> tl, ll;
    std::vector<unsigned long long> tc, wrows, lc;
    std::vector<uint8_t> lkb;
    std::vector<int64_t> lko(1, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t len = key_offsets[i + 1] - key_offsets[i];
        if (len < 1 || len > LDGPU_MAX_FIT_GRAM)
            return fail(LDGPU_EINVAL, "key %lld has length %lld outside [1, %d]", (long long)i, (long long)len,
                        LDGPU_MAX_FIT_GRAM);
        if (pair_offsets[i + 1] < pair_offsets[i]) return fail(LDGPU_EINVAL, "pair offsets decrease at %lld", (long long)i);
        const uint8_t* kb = key_bytes + key_offsets[i];
        for (int64_t j = pair_offsets[i]; j < pair_offsets[i + 1]; ++j) {
            const int64_t q = j - pair_offsets[0];
            if (pair_langs[q] < 0 || pair_langs[q] >= c->L)
                return fail(LDGPU_EINVAL, "pair %lld: language %d outside [0, %d)", (long long)q, pair_langs[q], c->L);
            if (pair_counts[q] < 0) return fail(LDGPU_EINVAL, "pair %lld: negative count", (long long)q);
        }
        if (len <= kMaxGram) {
            const uint64_t key = pack_key_host(kb, (int)len);
            for (int64_t j = pair_offsets[i]; j < pair_offsets[i + 1]; ++j) {
                const int64_t q = j - pair_offsets[0];
                if (!pair_counts[q]) continue;
                tk.push_back(key);
                tl.push_back(pair_langs[q]);
                tc.push_back((unsigned long long)pair_counts[q]);
            }
        } else if (len > kMaxWideGram) {
            for (int64_t j = pair_offsets[i]; j < pair_offsets[i + 1]; ++j) {
                const int64_t q = j - pair_offsets[0];
                if (!pair_counts[q]) continue;
                lkb.insert(lkb.end(), kb, kb + len);
                lko.push_back((int64_t)lkb.size());
                ll.push_back(pair_langs[q]);
                lc.push_back((unsigned long long)pair_counts[q]);
            }
        } else {
            wlo.push_back(wide_lo_host(kb));
            whi.push_back(wide_hi_host(kb, len));
            wrows.resize(wrows.size() + c->L, 0ull);
            for (int64_t j = pair_offsets[i]; j < pair_offsets[i + 1]; ++j) {
                const int64_t q = j - pair_offsets[0];
                wrows[wrows.size() - c->L + pair_langs[q]] += (unsigned long long)pair_counts[q];
            }
        }
    }
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    c->tbl_valid = false;
    c->sp_valid = false;
    if (int rc = add_wide_rows(c, wlo, whi, wrows)) return rc;
    if (int rc = long_add_triples(c, lkb, lko, ll, lc)) return rc;
    if (int rc = add_triples(c, tk, tl, tc)) return rc;
    return ok();
}

extern "C" int ldgpu_counts_add(ldgpu_counts* c, int64_t n, const uint8_t* key_bytes, const int64_t* key_offsets,
                                const int64_t* counts_in) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    if (c->comm) return fail(LDGPU_EINVAL, "the count table is merged (ldgpu_counts_merge): it takes no more counts");
    if (n < 0) return fail(LDGPU_EINVAL, "n < 0");
    if (n == 0) return ok();
    if (!key_bytes || !key_offsets || !counts_in) return fail(LDGPU_EINVAL, "NULL argument");
    // one-word keys (1..7 bytes): their nonzero counts as (key, language,
    // count) triples; wide keys (8..15 bytes: two words) as dense rows
    const int L = c->L;
    std::vector<uint64_t> tk, wlo, whi;
    std::vector<int32_t> tl, ll;
    std::vector<unsigned long long> tc, wrows, lc;
    std::vector<uint8_t> lkb;
    std::vector<int64_t> lko(1, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t len = key_offsets[i + 1] - key_offsets[i];
        if (len < 1 || len > LDGPU_MAX_FIT_GRAM)
            return fail(LDGPU_EINVAL, "key %lld has length %lld outside [1, %d]", (long long)i, (long long)len,
                        LDGPU_MAX_FIT_GRAM);
        const uint8_t* kb = key_bytes + key_offsets[i];
        const int64_t* row = counts_in + (size_t)i * L;
        for (int l = 0; l < L; ++l)
            if (row[l] < 0) return fail(LDGPU_EINVAL, "key %lld: negative count", (long long)i);
        if (len <= kMaxGram) {
            const uint64_t key = pack_key_host(kb, (int)len);
            for (int l = 0; l < L; ++l) {
                if (!row[l]) continue;
                tk.push_back(key);
                tl.push_back(l);
                tc.push_back((unsigned long long)row[l]);
            }
        } else if (len > kMaxWideGram) {
            for (int l = 0; l < L; ++l) {
                if (!row[l]) continue;
                lkb.insert(lkb.end(), kb, kb + len);
                lko.push_back((int64_t)lkb.size());
                ll.push_back(l);
                lc.push_back((unsigned long long)row[l]);
            }
        } else {
            wlo.push_back(wide_lo_host(kb));
            whi.push_back(wide_hi_host(kb, len));
            wrows.insert(wrows.end(), row, row + L);
        }
    }
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    c->tbl_valid = false;
    c->sp_valid = false;
    if (int rc = add_wide_rows(c, wlo, whi, wrows)) return rc;
    if (int rc = long_add_triples(c, lkb, lko, ll, lc)) return rc;
    if (int rc = add_triples(c, tk, tl, tc)) return rc;
    return ok();
}

extern "C" int ldgpu_counts_export_device(ldgpu_counts* c, int64_t capacity, uint64_t* d_keys, int64_t* d_counts,
                                          int64_t* n_out, void* stream) {
    if (!c || !n_out) return fail(LDGPU_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    if (c->wsize || c->lsize)
        return fail(LDGPU_EUNSUPPORTED, "export_device: the table holds grams of 8 or more bytes, which have no packed "
                                        "u64 form (use ldgpu_counts_export)");
    *n_out = (int64_t)c->size;
    if ((int64_t)c->size > capacity)
        return fail(LDGPU_EINVAL, "export_device: %llu grams exceed the capacity %lld", (unsigned long long)c->size,
                    (long long)capacity);
    if (c->size && (!d_keys || !d_counts)) return fail(LDGPU_EINVAL, "device pointer is NULL");
    if (!c->size) return ok();
    hipStream_t st = (hipStream_t)stream;
    hipStream_t cs = c->ctx->stream;
    HIP_TRY(hipStreamSynchronize(st));  // the caller's buffers may be in use on its stream
    // the grams (unordered) with their slots, each slot's output row, then the
    // pairs into the zeroed dense rows
    DevBufs db;
    db.ctx = c->ctx;
    uint64_t* d_slot;
    uint32_t* d_rank;
    unsigned long long* d_n;
    HIP_TRY(db.alloc(&d_slot, c->size));
    HIP_TRY(db.alloc(&d_rank, c->cap));
    HIP_TRY(db.alloc(&d_n, 1));
    HIP_TRY(hipMemsetAsync(d_n, 0, sizeof(unsigned long long), cs));
    HIP_TRY(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * c->size * (size_t)c->L, cs));
    HIP_TRY(launch_gram_compact(count_params(c), c->cap, d_keys, d_slot, d_n, false, cs));
    HIP_TRY(launch_rank_scatter((int64_t)c->size, d_slot, d_rank, cs));
    HIP_TRY(launch_pair_dense(count_params(c), c->pcap, d_rank, reinterpret_cast<unsigned long long*>(d_counts), cs));
    unsigned long long got = 0;
    HIP_TRY(hipMemcpyAsync(&got, d_n, sizeof got, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    if (got != c->size) return fail(LDGPU_EDEVICE, "export_device: %llu grams, %llu expected", got,
                                    (unsigned long long)c->size);
    return ok();
}

extern "C" int ldgpu_counts_add_device(ldgpu_counts* c, int64_t n, const uint64_t* d_keys, const int64_t* d_counts,
                                       void* stream) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    if (c->comm) return fail(LDGPU_EINVAL, "the count table is merged (ldgpu_counts_merge): it takes no more counts");
    if (n < 0) return fail(LDGPU_EINVAL, "n < 0");
    if (n == 0) return ok();
    if (!d_keys || !d_counts) return fail(LDGPU_EINVAL, "device pointer is NULL");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    c->tbl_valid = false;
    c->sp_valid = false;
    hipStream_t st = (hipStream_t)stream;
    hipStream_t cs = c->ctx->stream;
    HIP_TRY(hipStreamSynchronize(st));
    // room for the block's nonzero counts (pairs) and keys
    unsigned long long nnz = 0;
    {
        DevBufs db;
        db.ctx = c->ctx;
        unsigned long long* d_nz;
        HIP_TRY(db.alloc(&d_nz, 1));
        HIP_TRY(hipMemsetAsync(d_nz, 0, sizeof(unsigned long long), cs));
        HIP_TRY(launch_nnz(reinterpret_cast<const unsigned long long*>(d_counts), n * (int64_t)c->L, d_nz, cs));
        HIP_TRY(hipMemcpyAsync(&nnz, d_nz, sizeof nnz, hipMemcpyDeviceToHost, cs));
        HIP_TRY(hipStreamSynchronize(cs));
    }
    if (int rc = reserve(c, (uint64_t)n, nnz)) return rc;
    if (int rc = ensure_ovf(c, (int64_t)std::max<unsigned long long>(nnz, 1))) return rc;
    HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), cs));
    HIP_TRY(launch_counts_add(count_params(c), d_keys, reinterpret_cast<const unsigned long long*>(d_counts), nullptr,
                              nullptr, n, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    if (int rc = after_batch(c)) return rc;
    return ok();
}

namespace {

// filterTopGrams (LanguageDetector.scala:100-132) over a presence table --
// keys sorted by (length, bytes), masks[n][S] -- into the cached table:
// per language the present grams by class k ascending, then (when fewer than
// K are present) zero-valued grams; ties by the (length, bytes) order.
int table_from_presence(ldgpu_counts* c, const std::vector<uint64_t>& keys, const std::vector<uint64_t>& masks,
                        int32_t K, int64_t* n_rows, int64_t* key_bytes) {
    const int L = c->L, S = (L + 63) / 64;
    const size_t n = keys.size();
    auto has = [&](size_t i, int l) { return (masks[i * S + l / 64] >> (l % 64)) & 1ull; };
    std::vector<int> kg(n, 0);
    for (size_t i = 0; i < n; ++i)
        for (int s = 0; s < S; ++s) kg[i] += __builtin_popcountll(masks[i * S + s]);
    std::vector<double> w(L + 1, 0.0);
    for (int k = 1; k <= L; ++k) w[k] = std::log(1.0 + 1.0 / (double)k);
    std::vector<uint8_t> chosen(n, 0);
    if (K > 0) {
        std::vector<int64_t> per((size_t)L * (L + 1), 0);
        for (size_t i = 0; i < n; ++i)
            for (int l = 0; l < L; ++l)
                if (has(i, l)) per[(size_t)l * (L + 1) + kg[i]]++;
        std::vector<int> kstar(L, L + 1);
        std::vector<int64_t> need(L, 0), absent_need(L, 0);
        for (int l = 0; l < L; ++l) {
            int64_t acc = 0;
            for (int k = 1; k <= L; ++k) {
                const int64_t c_k = per[(size_t)l * (L + 1) + k];
                if (acc + c_k >= K) {
                    kstar[l] = k;
                    need[l] = K - acc;
                    break;
                }
                acc += c_k;
            }
            if (kstar[l] == L + 1) absent_need[l] = K - acc;  // every present gram + zeros
        }
        std::vector<int64_t> taken(L, 0), absent_taken(L, 0);
        for (size_t i = 0; i < n; ++i) {
            for (int l = 0; l < L; ++l) {
                if (has(i, l)) {
                    if (kg[i] < kstar[l]) {
                        chosen[i] = 1;
                    } else if (kg[i] == kstar[l] && taken[l] < need[l]) {
                        taken[l]++;
                        chosen[i] = 1;
                    }
                } else if (absent_taken[l] < absent_need[l]) {
                    absent_taken[l]++;
                    chosen[i] = 1;
                }
            }
        }
    }
    std::vector<uint64_t> out_keys;
    c->tbl_masks.clear();
    c->tbl_vals.clear();
    for (size_t i = 0; i < n; ++i) {
        if (!chosen[i]) continue;
        out_keys.push_back(keys[i]);
        c->tbl_masks.insert(c->tbl_masks.end(), masks.begin() + i * S, masks.begin() + (i + 1) * S);
        c->tbl_vals.push_back(w[kg[i]]);
    }
    int64_t nb = 0;
    for (uint64_t k : out_keys) nb += gram_bytes(c, k, nullptr);
    c->tbl_bytes.assign((size_t)std::max<int64_t>(nb, 1), 0);
    c->tbl_off.assign(out_keys.size() + 1, 0);
    write_keys(c, out_keys, c->tbl_bytes.data(), c->tbl_off.data());
    c->tbl_valid = true;
    if (n_rows) *n_rows = (int64_t)out_keys.size();
    if (key_bytes) *key_bytes = nb;
    return LDGPU_OK;
}

// Host build from the full count table (used when some language has fewer
// than K present grams: the zero-valued fill needs every gram).
int fit_table_host(ldgpu_counts* c, int32_t K, int64_t* n_rows, int64_t* key_bytes) {
    Pulled t;
    if (int rc = counts_pull(c, t)) return rc;
    const int L = c->L, S = (L + 63) / 64;
    std::vector<uint64_t> masks(t.keys.size() * S, 0);
    for (size_t i = 0; i < t.keys.size(); ++i)
        for (int64_t j = t.poff[i]; j < t.poff[i + 1]; ++j)
            if (t.cnt[j]) masks[i * S + t.lang[j] / 64] |= 1ull << (t.lang[j] % 64);
    return table_from_presence(c, t.keys, masks, K, n_rows, key_bytes);
}
}  // namespace

// ------------------------------------------------------------ communicators
struct ldgpu_comm {
    ldgpu_ctx* ctx = nullptr;
    int rank = 0, world = 1;
    ncclComm_t nccl = nullptr;   // RCCL transport, else the host callbacks
    ldgpu_host_coll host{};
};

#define NCCL_TRY(expr)                                                                             \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess) return fail(LDGPU_EDEVICE, "%s: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

namespace {
// all-gather of `bytes` host bytes per rank into out[world * bytes]
int comm_allgather_host(ldgpu_comm* m, const void* send, int64_t bytes, void* out) {
    if (m->world == 1) {
        if (bytes) memcpy(out, send, (size_t)bytes);
        return LDGPU_OK;
    }
    if (!m->nccl) {
        if (m->host.allgather(m->host.user, send, bytes, out)) return fail(LDGPU_EDEVICE, "host all-gather failed");
        return LDGPU_OK;
    }
    hipStream_t st = m->ctx->stream;
    DevBufs db;
    uint8_t *d_s, *d_r;
    HIP_TRY(db.alloc(&d_s, (size_t)bytes));
    HIP_TRY(db.alloc(&d_r, (size_t)bytes * m->world));
    HIP_TRY(hipMemcpyAsync(d_s, send, (size_t)bytes, hipMemcpyHostToDevice, st));
    NCCL_TRY(ncclAllGather(d_s, d_r, (size_t)bytes, ncclUint8, m->nccl, st));
    HIP_TRY(hipMemcpyAsync(out, d_r, (size_t)bytes * m->world, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return LDGPU_OK;
}

// variable-size all-gather of host blobs (sizes first, then padded blobs)
int comm_allgatherv_host(ldgpu_comm* m, const std::vector<uint8_t>& mine, std::vector<std::vector<uint8_t>>& all) {
    const int W = m->world;
    int64_t n = (int64_t)mine.size();
    std::vector<int64_t> ns(W);
    if (int rc = comm_allgather_host(m, &n, sizeof n, ns.data())) return rc;
    const int64_t mx = std::max<int64_t>(1, *std::max_element(ns.begin(), ns.end()));
    std::vector<uint8_t> pad((size_t)mx, 0), buf((size_t)mx * W);
    if (n) memcpy(pad.data(), mine.data(), (size_t)n);
    if (int rc = comm_allgather_host(m, pad.data(), mx, buf.data())) return rc;
    all.assign(W, {});
    for (int r = 0; r < W; ++r) all[r].assign(buf.begin() + (size_t)r * mx, buf.begin() + (size_t)r * mx + ns[r]);
    return LDGPU_OK;
}

// all-to-all of device buffers: block r of d_send (sb[r] bytes) goes to rank
// r, block r of d_recv (rb[r] bytes) comes from rank r
int comm_alltoallv_dev(ldgpu_comm* m, const uint8_t* d_send, const std::vector<int64_t>& sb, uint8_t* d_recv,
                       const std::vector<int64_t>& rb) {
    const int W = m->world;
    hipStream_t st = m->ctx->stream;
    std::vector<int64_t> os(W + 1, 0), orr(W + 1, 0);
    for (int r = 0; r < W; ++r) {
        os[r + 1] = os[r] + sb[r];
        orr[r + 1] = orr[r] + rb[r];
    }
    if (m->nccl) {
        NCCL_TRY(ncclGroupStart());
        for (int r = 0; r < W; ++r) {
            if (sb[r]) NCCL_TRY(ncclSend(d_send + os[r], (size_t)sb[r], ncclUint8, r, m->nccl, st));
            if (rb[r]) NCCL_TRY(ncclRecv(d_recv + orr[r], (size_t)rb[r], ncclUint8, r, m->nccl, st));
        }
        NCCL_TRY(ncclGroupEnd());
        HIP_TRY(hipStreamSynchronize(st));
        return LDGPU_OK;
    }
    std::vector<uint8_t> hs((size_t)std::max<int64_t>(os[W], 1)), hr((size_t)std::max<int64_t>(orr[W], 1));
    if (os[W]) HIP_TRY(hipMemcpyAsync(hs.data(), d_send, (size_t)os[W], hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (W == 1) {
        hr = hs;
    } else if (m->host.alltoallv(m->host.user, hs.data(), sb.data(), hr.data(), rb.data())) {
        return fail(LDGPU_EDEVICE, "host all-to-all failed");
    }
    if (orr[W]) HIP_TRY(hipMemcpyAsync(d_recv, hr.data(), (size_t)orr[W], hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return LDGPU_OK;
}

template <typename T>
void put(std::vector<uint8_t>& b, const T* p, size_t n) {
    const uint8_t* q = reinterpret_cast<const uint8_t*>(p);
    b.insert(b.end(), q, q + n * sizeof(T));
}
}  // namespace

extern "C" int ldgpu_comm_unique_id(uint8_t* out_id) {
    if (!out_id) return fail(LDGPU_EINVAL, "out_id is NULL");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    memcpy(out_id, &id, LDGPU_COMM_ID_BYTES);
    return ok();
}

extern "C" int ldgpu_comm_create_rccl(ldgpu_ctx* ctx, const uint8_t* id, int32_t rank, int32_t world,
                                      ldgpu_comm** out) {
    if (!ctx || !id || !out) return fail(LDGPU_EINVAL, "NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fail(LDGPU_EINVAL, "rank %d outside world %d", rank, world);
    HIP_TRY(hipSetDevice(ctx->device));
    ncclUniqueId uid;
    memcpy(&uid, id, LDGPU_COMM_ID_BYTES);
    ncclComm_t comm = nullptr;
    NCCL_TRY(ncclCommInitRank(&comm, world, uid, rank));
    auto* m = new ldgpu_comm();
    m->ctx = ctx;
    m->rank = rank;
    m->world = world;
    m->nccl = comm;
    *out = m;
    return ok();
}

extern "C" int ldgpu_comm_create_host(ldgpu_ctx* ctx, int32_t rank, int32_t world, const ldgpu_host_coll* coll,
                                      ldgpu_comm** out) {
    if (!ctx || !coll || !out) return fail(LDGPU_EINVAL, "NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fail(LDGPU_EINVAL, "rank %d outside world %d", rank, world);
    if (world > 1 && (!coll->allgather || !coll->alltoallv)) return fail(LDGPU_EINVAL, "host collectives are NULL");
    auto* m = new ldgpu_comm();
    m->ctx = ctx;
    m->rank = rank;
    m->world = world;
    m->host = *coll;
    *out = m;
    return ok();
}

extern "C" int ldgpu_comm_destroy(ldgpu_comm* m) {
    if (!m) return ok();
    if (m->nccl) (void)ncclCommDestroy(m->nccl);
    delete m;
    return ok();
}

namespace {
uint32_t wide_owner(uint64_t lo, uint64_t hi, uint32_t world) {
    return (uint32_t)(((mix64(lo ^ mix64(hi)) & 0xffffffffull) * world) >> 32);
}

// The merge's wide grams (8..15 bytes, their own table): every rank's entries
// reach every rank over the host all-gather -- they are few next to the
// one-word grams -- and each rank keeps, summed, those it owns.  Sets
// c->merged_wide on every rank alike when any rank held one.
int merge_wide(ldgpu_counts* c, ldgpu_comm* m) {
    const int L = c->L;
    std::vector<uint64_t> wlo, whi;
    std::vector<unsigned long long> wc;
    if (int rc = wide_export(c, wlo, whi, wc)) return rc;
    std::vector<uint8_t> blob;
    put(blob, wlo.data(), wlo.size());
    put(blob, whi.data(), whi.size());
    put(blob, wc.data(), wc.size());
    std::vector<std::vector<uint8_t>> all;
    if (int rc = comm_allgatherv_host(m, blob, all)) return rc;
    std::vector<uint64_t> olo, ohi;
    std::vector<unsigned long long> orows;
    bool any = false;
    for (int r = 0; r < m->world; ++r) {
        const size_t nr = all[r].size() / (16 + 8 * (size_t)L);
        any |= nr > 0;
        const uint64_t* lo = reinterpret_cast<const uint64_t*>(all[r].data());
        const uint64_t* hi = lo + nr;
        const unsigned long long* rows = reinterpret_cast<const unsigned long long*>(hi + nr);
        for (size_t i = 0; i < nr; ++i) {
            if (wide_owner(lo[i], hi[i], (uint32_t)m->world) != (uint32_t)m->rank) continue;
            olo.push_back(lo[i]);
            ohi.push_back(hi[i]);
            orows.insert(orows.end(), rows + i * L, rows + (i + 1) * L);
        }
    }
    c->merged_wide = any;
    // this rank's wide table, rebuilt from the owned entries
    for (void* q : {(void*)c->d_wlo, (void*)c->d_whi, (void*)c->d_wcounts})
        if (q) (void)hipFree(q);
    c->d_wlo = c->d_whi = nullptr;
    c->d_wcounts = nullptr;
    c->wcap = 0;
    c->wsize = 0;
    if (c->d_wsize) HIP_TRY(hipMemsetAsync(c->d_wsize, 0, sizeof(unsigned long long), c->ctx->stream));
    const int64_t n = (int64_t)olo.size();
    if (!n) return LDGPU_OK;
    if (int rc = wide_ensure(c, (uint64_t)n)) return rc;
    DevBufs wb;
    uint64_t *d_lo, *d_hi;
    unsigned long long* d_r;
    HIP_TRY(wb.alloc(&d_lo, n));
    HIP_TRY(wb.alloc(&d_hi, n));
    HIP_TRY(wb.alloc(&d_r, (size_t)n * L));
    hipStream_t st = c->ctx->stream;
    HIP_TRY(hipMemcpyAsync(d_lo, olo.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_hi, ohi.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_r, orows.data(), (size_t)n * L * sizeof(unsigned long long), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_wide_add(wide_params(c), d_lo, d_hi, d_r, n, st));
    return wide_after(c);
}
}  // namespace

namespace {
// The merge's long grams (16 bytes or more, their own table): as the wide
// ones, every rank's (key, language, count) triples reach every rank over the
// host all-gather and each keeps those it owns (gen_hash of the bytes), summed
// into a fresh long table.  Raises c->merged_wide on every rank alike when any
// rank held one (the top-K then runs on the host over every rank's rows).
int merge_long(ldgpu_counts* c, ldgpu_comm* m) {
    Ext x;
    if (int rc = long_export(c, x, true)) return rc;
    std::vector<uint8_t> blob;
    const uint64_t nx = x.keys.size();
    put(blob, &nx, 1);
    for (uint64_t i = 0; i < nx; ++i) {
        const uint64_t len = x.keys[i].size(), np = (uint64_t)(x.poff[i + 1] - x.poff[i]);
        put(blob, &len, 1);
        put(blob, (const uint8_t*)x.keys[i].data(), len);
        put(blob, &np, 1);
        put(blob, x.lang.data() + x.poff[i], np);
        put(blob, x.cnt.data() + x.poff[i], np);
    }
    std::vector<std::vector<uint8_t>> all;
    if (int rc = comm_allgatherv_host(m, blob, all)) return rc;
    std::vector<uint8_t> kb;
    std::vector<int64_t> ko(1, 0);
    std::vector<int32_t> tl;
    std::vector<unsigned long long> tc;
    bool any = false;
    for (int r = 0; r < m->world; ++r) {
        const uint8_t* q = all[r].data();
        uint64_t cnt;
        memcpy(&cnt, q, 8);
        q += 8;
        any |= cnt > 0;
        for (uint64_t i = 0; i < cnt; ++i) {
            uint64_t len, np;
            memcpy(&len, q, 8);
            const uint8_t* key = q + 8;
            q += 8 + len;
            memcpy(&np, q, 8);
            q += 8;
            const int32_t* ls = reinterpret_cast<const int32_t*>(q);
            std::vector<int64_t> cs(np);
            memcpy(cs.data(), q + 4 * np, 8 * np);
            q += 12 * np;
            const uint64_t h = gen_hash(key, (int64_t)len);
            if ((uint32_t)(((h & 0xffffffffull) * (uint64_t)m->world) >> 32) != (uint32_t)m->rank) continue;
            for (uint64_t j = 0; j < np; ++j) {
                kb.insert(kb.end(), key, key + len);
                ko.push_back((int64_t)kb.size());
                int32_t l;
                memcpy(&l, ls + j, 4);
                tl.push_back(l);
                tc.push_back((unsigned long long)cs[j]);
            }
        }
    }
    c->merged_wide = c->merged_wide || any;
    // this rank's long table, rebuilt from the owned triples
    for (void* q : {(void*)c->d_lslots, (void*)c->d_larena, (void*)c->d_lpkeys,
                    (void*)c->d_lpcounts})
        if (q) (void)hipFree(q);
    c->d_lslots = nullptr;
    c->d_larena = nullptr;
    c->d_lpkeys = nullptr;
    c->d_lpcounts = nullptr;
    c->lcap = c->lpcap = c->larena_cap = 0;
    c->lsize = c->lpsize = c->larena_n = 0;
    if (c->d_lctr) HIP_TRY(hipMemsetAsync(c->d_lctr, 0, 4 * sizeof(unsigned long long), c->ctx->stream));
    return long_add_triples(c, kb, ko, tl, tc);
}

// Every rank's status before a collective phase: a failure that one rank
// alone meets (an allocation, a count check) ends the merge on EVERY rank
// instead of leaving the others waiting in the next exchange.  Returns the
// local code (with its message) or LDGPU_EDEVICE naming the failed rank.
int comm_agree(ldgpu_comm* m, int rc, const char* what = "merge") {
    if (m->world == 1) return rc;
    const std::string mine = g_err;
    int32_t v = rc;
    std::vector<int32_t> all(m->world);
    if (int r = comm_allgather_host(m, &v, sizeof v, all.data())) return r;
    if (rc) {
        g_err = mine;
        return rc;
    }
    for (int r = 0; r < m->world; ++r)
        if (all[r]) return fail(LDGPU_EDEVICE, "%s: rank %d failed (status %d)", what, r, all[r]);
    return LDGPU_OK;
}
}  // namespace

// Owner exchange: every rank partitions its table by owner, one
// all-to-all moves each rank's nonzero (gram, language) counts -- 16-B pairs
// (key, lang << 52 | count), not dense rows of L counters -- to their owners,
// and each rank rebuilds its table from what it received: the global counts
// of the grams it owns (integer sums: bit-exact in any order).  Every rank's
// status is agreed before each exchange (comm_agree).
extern "C" int ldgpu_counts_merge(ldgpu_counts* c, ldgpu_comm* m) {
    if (!c || !m) return fail(LDGPU_EINVAL, "NULL argument");
    if (c->comm) return fail(LDGPU_EINVAL, "the count table is already merged");
    if (m->ctx != c->ctx) return fail(LDGPU_EINVAL, "communicator and count table belong to different contexts");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    const int W = m->world;
    hipStream_t st = c->ctx->stream;
    DevBufs db;
    unsigned long long *d_nof = nullptr, *d_cur = nullptr;
    uint64_t *d_pairs = nullptr, *d_rpairs = nullptr;
    std::vector<unsigned long long> nof(W), cur(W);
    std::vector<int64_t> send_n(W);
    // phase 1: this rank's pairs, partitioned by owner
    auto partition = [&]() -> int {
        HIP_TRY(db.alloc(&d_nof, W));
        HIP_TRY(db.alloc(&d_cur, W));
        HIP_TRY(hipMemsetAsync(d_nof, 0, sizeof(unsigned long long) * W, st));
        HIP_TRY(launch_owner_pair_count(count_params(c), c->pcap, (uint32_t)W, d_nof, st));
        HIP_TRY(hipMemcpyAsync(nof.data(), d_nof, sizeof(unsigned long long) * W, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        unsigned long long acc = 0;
        for (int r = 0; r < W; ++r) {
            cur[r] = acc;
            acc += nof[r];
            send_n[r] = (int64_t)nof[r];
        }
        HIP_TRY(db.alloc(&d_pairs, 2 * (size_t)acc));
        HIP_TRY(hipMemcpyAsync(d_cur, cur.data(), sizeof(unsigned long long) * W, hipMemcpyHostToDevice, st));
        HIP_TRY(launch_owner_pair_scatter(count_params(c), c->pcap, (uint32_t)W, d_cur, d_pairs, st));
        HIP_TRY(hipStreamSynchronize(st));
        return LDGPU_OK;
    };
    if (int rc = comm_agree(m, partition())) return rc;
    std::vector<int64_t> all((size_t)W * W);
    if (int rc = comm_allgather_host(m, send_n.data(), sizeof(int64_t) * W, all.data())) return rc;
    std::vector<int64_t> recv_n(W);
    int64_t R = 0;
    for (int r = 0; r < W; ++r) R += recv_n[r] = all[(size_t)r * W + m->rank];
    // phase 2: receive buffers and the fresh owned-shard table, then the exchange
    auto prepare = [&]() -> int {
        HIP_TRY(db.alloc(&d_rpairs, 2 * (size_t)R));
        return LDGPU_OK;
    };
    if (int rc = comm_agree(m, prepare())) return rc;
    std::vector<int64_t> sb(W), rb(W);
    for (int r = 0; r < W; ++r) {
        sb[r] = send_n[r] * 16;
        rb[r] = recv_n[r] * 16;
    }
    if (int rc = comm_alltoallv_dev(m, (const uint8_t*)d_pairs, sb, (uint8_t*)d_rpairs, rb)) return rc;
    // the owned shard, rebuilt: one key may arrive from several ranks
    auto rebuild = [&]() -> int {
        HIP_TRY(hipStreamSynchronize(st));
        cache_free(c->ctx, c->d_keys, c->cap * sizeof(uint64_t));
        cache_free(c->ctx, c->d_kcnt, c->cap * sizeof(uint32_t));
        free_pairs(c->ctx, c->d_pkeys, c->pcap);
        c->d_keys = c->d_pkeys = nullptr;
        c->d_kcnt = nullptr;
        c->d_pcounts = nullptr;
        c->cap = c->pcap = next_pow2((uint64_t)std::max<int64_t>(1 << 12, 2 * R + 16));
        if (int rc = alloc_table(c, c->cap, &c->d_keys, reinterpret_cast<void**>(&c->d_kcnt)))
            return rc;
        if (int rc = alloc_pairs(c, c->pcap, &c->d_pkeys, &c->d_pcounts)) return rc;
        if (int rc = ensure_ovf(c, R)) return rc;
        HIP_TRY(hipMemsetAsync(c->d_size, 0, sizeof(unsigned long long), st));
        HIP_TRY(hipMemsetAsync(c->d_psize, 0, sizeof(unsigned long long), st));
        HIP_TRY(hipMemsetAsync(c->d_ovf_n, 0, sizeof(unsigned int), st));
        c->size = 0;
        c->psize = 0;
        HIP_TRY(launch_pairs_add(count_params(c), d_rpairs, R, st));
        HIP_TRY(hipStreamSynchronize(st));
        return after_batch(c);
    };
    if (int rc = comm_agree(m, rebuild())) return rc;
    if (int rc = comm_agree(m, merge_wide(c, m))) return rc;
    if (int rc = comm_agree(m, merge_long(c, m))) return rc;
    c->comm = m;
    c->tbl_valid = false;
    c->sp_valid = false;
    return ok();
}

namespace {
// Device build (SURVEY §8f "next" #3): from the sparse table's pairs the
// (language, k) histogram (k = the gram's language count, kept by the count
// kernels); the host picks each language's threshold class; the device flags
// the grams below it, resolves the threshold class's (length, bytes) ties and
// builds the chosen rows' presence masks from the pairs.  Only the chosen
// grams (<= L*K) cross PCIe.
// On a merged table (c->comm) the histogram is summed over the ranks, the
// ties are resolved against the ranks' candidate prefixes, and the chosen
// rows of every rank are gathered: every rank builds the same global table.
int fit_table_device(ldgpu_counts* c, int32_t K, int64_t* n_rows, int64_t* key_bytes, bool* fallback) {
    *fallback = false;
    ldgpu_comm* cm = c->comm;
    const int L = c->L, S = (L + 63) / 64;
    const int64_t n = (int64_t)c->size;
    hipStream_t st = c->ctx->stream;
    DevBufs db;
    db.ctx = c->ctx;
    const CountParams cp = count_params(c);
    // A merged table's build is collective: every rank agrees its status
    // before each collective (comm_agree), so a failure on one rank (an
    // allocation, a count check) ends the build on every rank instead of
    // leaving the others waiting in the next all-gather.
    auto agree = [&](int rc) { return cm ? comm_agree(cm, rc, "fit table") : rc; };
    uint64_t* d_keys = nullptr;
    uint64_t* d_rk = nullptr;  // per gram slot: row | k << 32
    int32_t* d_k = nullptr;
    unsigned long long* d_n = nullptr;
    unsigned int* d_hist = nullptr;
    std::vector<unsigned int> hist((size_t)L * (L + 1));
    PhaseMarks mark(st);
    auto hist_phase = [&]() -> int {
        if (int rc = injected("table_hist")) return rc;
        if (n > (int64_t)0xffffffffll) return fail(LDGPU_EUNSUPPORTED, "fit table: %lld grams", (long long)n);
        HIP_TRY(db.alloc(&d_keys, n));
        HIP_TRY(db.alloc(&d_k, n));
        HIP_TRY(db.alloc(&d_rk, c->cap));
        HIP_TRY(db.alloc(&d_n, 2));
        HIP_TRY(db.alloc(&d_hist, (size_t)L * (L + 1)));
        mark("table: scratch");
        HIP_TRY(hipMemsetAsync(d_n, 0, 2 * sizeof(unsigned long long), st));
        HIP_TRY(hipMemsetAsync(d_hist, 0, sizeof(unsigned int) * L * (L + 1), st));
        HIP_TRY(launch_gram_rows(cp, c->cap, d_keys, d_k, d_rk, d_n, st));
        mark("table: gram rows");
        HIP_TRY(launch_pair_hist(cp, c->pcap, L, d_rk, d_hist, c->ctx->cus, st));
        mark("table: pair histogram");
        unsigned long long got = 0;
        HIP_TRY(hipMemcpyAsync(hist.data(), d_hist, sizeof(unsigned int) * hist.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&got, d_n, sizeof got, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if ((int64_t)got != n) return fail(LDGPU_EDEVICE, "presence: %llu grams, %lld expected", got, (long long)n);
        return LDGPU_OK;
    };
    if (int rc = agree(hist_phase())) return rc;
    std::vector<int64_t> ghist(hist.begin(), hist.end());  // global (summed over ranks)
    if (cm && cm->world > 1) {
        std::vector<int64_t> mine(ghist), allh(ghist.size() * cm->world);
        if (int rc = comm_allgather_host(cm, mine.data(), (int64_t)(sizeof(int64_t) * mine.size()), allh.data()))
            return rc;
        for (size_t i = 0; i < ghist.size(); ++i) {
            ghist[i] = 0;
            for (int r = 0; r < cm->world; ++r) ghist[i] += allh[(size_t)r * ghist.size() + i];
        }
    }

    std::vector<int32_t> kstar(L, L + 1), need(L, 0);
    uint64_t cand_cap = 0;  // this rank's candidates
    for (int l = 0; l < L; ++l) {
        int64_t acc = 0;
        for (int k = 1; k <= L; ++k) {
            const int64_t ck = ghist[(size_t)l * (L + 1) + k];
            if (acc + ck >= K) {
                kstar[l] = k;
                need[l] = (int32_t)(K - acc);
                if (need[l] > 0) cand_cap += (uint64_t)hist[(size_t)l * (L + 1) + k];
                break;
            }
            acc += ck;
        }
        if (kstar[l] == L + 1 && acc < K) *fallback = true;  // zero-valued fill: every gram takes part
    }
    // a merged table with wide grams (c->merged_wide, alike on every rank)
    // selects on the host over every rank's presence rows, wide ones included
    if (cm && c->merged_wide) *fallback = true;
    if (*fallback) {
        if (!cm) return LDGPU_OK;  // the host build from the count table
        // merged table: gather every rank's presence rows, select on the host
        std::vector<uint64_t> hk(n), hm((size_t)n * S);
        auto rows_phase = [&]() -> int {
            if (int rc = injected("table_fallback")) return rc;
            if (!n) return LDGPU_OK;
            uint64_t* d_masks;
            HIP_TRY(db.alloc(&d_masks, (size_t)n * S));
            HIP_TRY(hipMemsetAsync(d_masks, 0, sizeof(uint64_t) * n * S, st));
            HIP_TRY(launch_pair_masks(cp, c->pcap, d_rk, nullptr, S, d_masks, st));
            HIP_TRY(hipMemcpyAsync(hk.data(), d_keys, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(hm.data(), d_masks, sizeof(uint64_t) * n * S, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            return LDGPU_OK;
        };
        if (int rc = agree(rows_phase())) return rc;
        std::vector<uint8_t> blob;
        put(blob, hk.data(), hk.size());
        put(blob, hm.data(), hm.size());
        std::vector<std::vector<uint8_t>> all;
        if (int rc = comm_allgatherv_host(cm, blob, all)) return rc;
        std::vector<std::pair<uint64_t, std::pair<int, size_t>>> order;
        std::vector<const uint64_t*> rk(cm->world), rm(cm->world);
        for (int r = 0; r < cm->world; ++r) {
            const size_t nr = all[r].size() / (8 * (1 + S));
            rk[r] = reinterpret_cast<const uint64_t*>(all[r].data());
            rm[r] = rk[r] + nr;
            for (size_t i = 0; i < nr; ++i) order.push_back({sort_key(rk[r][i]), {r, i}});
        }
        std::sort(order.begin(), order.end());
        std::vector<uint64_t> keys(order.size()), masks(order.size() * S);
        for (size_t j = 0; j < order.size(); ++j) {
            keys[j] = rk[order[j].second.first][order[j].second.second];
            memcpy(&masks[j * S], rm[order[j].second.first] + order[j].second.second * S, 8 * S);
        }
        if (c->merged_wide) {  // every rank's grams of 8 or more bytes after them, in (length, bytes) order
            Ext x;
            auto ext_phase = [&]() -> int {
                if (int rc = injected("table_wide")) return rc;
                return ext_export(c, x, true);
            };
            if (int rc = agree(ext_phase())) return rc;
            // blob: count, then per gram its length, bytes and S mask words
            std::vector<uint8_t> wblob;
            const uint64_t nx = x.keys.size();
            put(wblob, &nx, 1);
            for (uint64_t i = 0; i < nx; ++i) {
                const uint64_t len = x.keys[i].size();
                std::vector<uint64_t> m(S, 0);
                for (int64_t j = x.poff[i]; j < x.poff[i + 1]; ++j)
                    if (x.cnt[j]) m[x.lang[j] / 64] |= 1ull << (x.lang[j] % 64);
                put(wblob, &len, 1);
                put(wblob, (const uint8_t*)x.keys[i].data(), len);
                put(wblob, m.data(), m.size());
            }
            std::vector<std::vector<uint8_t>> wall;
            if (int rc = comm_allgatherv_host(cm, wblob, wall)) return rc;
            std::vector<std::pair<std::string, std::vector<uint64_t>>> g;
            for (int r = 0; r < cm->world; ++r) {
                const uint8_t* q = wall[r].data();
                uint64_t cnt;
                memcpy(&cnt, q, 8);
                q += 8;
                for (uint64_t i = 0; i < cnt; ++i) {
                    uint64_t len;
                    memcpy(&len, q, 8);
                    q += 8;
                    std::string k((const char*)q, (size_t)len);
                    q += len;
                    std::vector<uint64_t> m(S);
                    memcpy(m.data(), q, 8 * (size_t)S);
                    q += 8 * (size_t)S;
                    g.emplace_back(std::move(k), std::move(m));
                }
            }
            std::sort(g.begin(), g.end(), [](const auto& u, const auto& v) {
                return u.first.size() != v.first.size() ? u.first.size() < v.first.size() : u.first < v.first;
            });
            c->ext_sorted.resize(g.size());
            for (size_t r = 0; r < g.size(); ++r) {
                c->ext_sorted[r] = g[r].first;
                keys.push_back((kWideTag << 56) | r);
                masks.insert(masks.end(), g[r].second.begin(), g[r].second.end());
            }
        }
        *fallback = false;
        return table_from_presence(c, keys, masks, K, n_rows, key_bytes);
    }
    const bool multi = cm && cm->world > 1;
    int32_t *d_kstar = nullptr, *d_need = nullptr, *d_cl = nullptr;
    uint8_t* d_chosen = nullptr;
    uint64_t* d_ck = nullptr;
    uint32_t* d_ci = nullptr;
    unsigned int* d_cn = nullptr;
    uint64_t* d_thr = nullptr;
    unsigned int cn = 0;
    std::vector<int64_t> seg(L + 1, 0);
    // multi-rank: this rank's need[l] smallest threshold-class candidates of
    // each language (their sort keys), gathered from every rank
    std::vector<int64_t> take(L, 0);
    std::vector<uint64_t> pre;
    int64_t tot = 0;
    auto select_phase = [&]() -> int {
        if (int rc = injected("table_select")) return rc;
        HIP_TRY(db.alloc(&d_kstar, L));
        HIP_TRY(db.alloc(&d_need, L));
        HIP_TRY(db.alloc(&d_chosen, n));
        HIP_TRY(db.alloc(&d_cl, cand_cap));
        HIP_TRY(db.alloc(&d_ck, cand_cap));
        HIP_TRY(db.alloc(&d_ci, cand_cap));
        HIP_TRY(db.alloc(&d_cn, 2));
        // one rank: the threshold class's candidates per (language, length)
        // too (<= 512 languages: the counters in LDS)
        const bool split = !multi && L <= 512 && cand_cap > 0;
        unsigned int* d_lh = nullptr;
        if (split) {
            HIP_TRY(db.alloc(&d_lh, (size_t)16 * L));
            HIP_TRY(hipMemsetAsync(d_lh, 0, sizeof(unsigned int) * 16 * L, st));
        }
        HIP_TRY(hipMemcpyAsync(d_kstar, kstar.data(), sizeof(int32_t) * L, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(d_need, need.data(), sizeof(int32_t) * L, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemsetAsync(d_cn, 0, 2 * sizeof(unsigned int), st));
        HIP_TRY(hipMemsetAsync(d_chosen, 0, (size_t)n, st));
        HIP_TRY(launch_pair_select(cp, c->pcap, d_rk, d_keys, d_kstar, d_need, d_chosen, d_cl, d_ck, d_ci, d_cn, L,
                                   d_lh, st));
        std::vector<unsigned int> lh(split ? (size_t)16 * L : 0);
        HIP_TRY(hipMemcpyAsync(&cn, d_cn, sizeof cn, hipMemcpyDeviceToHost, st));
        if (split) HIP_TRY(hipMemcpyAsync(lh.data(), d_lh, sizeof(unsigned int) * lh.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (cn != cand_cap)
            return fail(LDGPU_EDEVICE, "select: %u candidates, %llu expected", cn, (unsigned long long)cand_cap);
        mark("table: select");
        // per language: the need[l] smallest (length, bytes) keys of its
        // threshold class (candidates of language l form segment l once sorted)
        for (int l = 0; l < L; ++l)
            seg[l + 1] = seg[l] + (need[l] > 0 && kstar[l] <= L ? (int64_t)hist[(size_t)l * (L + 1) + kstar[l]] : 0);
        if (seg[L] != (int64_t)cn)
            return fail(LDGPU_EDEVICE, "select: %u candidates, %lld by class", cn, (long long)seg[L]);
        if (split) {
            // The tie order is (length, bytes): per language, every candidate
            // shorter than the length at which the cumulative count reaches
            // need[l] is chosen outright, and only candidates of exactly that
            // length are ranked (config 5's fit: ~1G class pairs -> the few
            // thousand of one length per language, instead of sorting them all)
            std::vector<int32_t> thr(L, 0);
            std::vector<int64_t> seg2(L + 1, 0);
            for (int l = 0; l < L; ++l) {
                int64_t cnt_l = seg[l + 1] - seg[l], acc = 0;
                if (need[l] > 0 && cnt_l > 0) {
                    for (int len = 0; len < 16; ++len) {
                        const int64_t c_len = lh[(size_t)16 * l + len];
                        if (acc + c_len >= need[l]) {
                            thr[l] = len;
                            need[l] -= (int32_t)acc;
                            cnt_l = c_len;
                            break;
                        }
                        acc += c_len;
                    }
                }
                seg2[l + 1] = seg2[l] + cnt_l;
            }
            int32_t *d_thr_len, *d_cl2;
            uint64_t* d_ck2;
            uint32_t* d_ci2;
            const size_t n2 = (size_t)std::max<int64_t>(seg2[L], 1);
            HIP_TRY(db.alloc(&d_thr_len, L));
            HIP_TRY(db.alloc(&d_cl2, n2));
            HIP_TRY(db.alloc(&d_ck2, n2));
            HIP_TRY(db.alloc(&d_ci2, n2));
            HIP_TRY(hipMemcpyAsync(d_thr_len, thr.data(), sizeof(int32_t) * L, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(d_need, need.data(), sizeof(int32_t) * L, hipMemcpyHostToDevice, st));
            HIP_TRY(launch_cand_filter((int64_t)cn, d_cl, d_ck, d_ci, d_thr_len, d_chosen, d_cl2, d_ck2, d_ci2, d_cn + 1,
                                       st));
            unsigned int cn2 = 0;
            HIP_TRY(hipMemcpyAsync(&cn2, d_cn + 1, sizeof cn2, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if ((int64_t)cn2 != seg2[L])
                return fail(LDGPU_EDEVICE, "select: %u candidates of the split lengths, %lld expected", cn2,
                            (long long)seg2[L]);
            d_cl = d_cl2;
            d_ck = d_ck2;
            d_ci = d_ci2;
            cn = cn2;
            seg = seg2;
            mark("table: length split");
        }
        int64_t* d_seg;
        HIP_TRY(db.alloc(&d_seg, L + 1));
        HIP_TRY(hipMemcpyAsync(d_seg, seg.data(), sizeof(int64_t) * (L + 1), hipMemcpyHostToDevice, st));
        if (!multi) {
            HIP_TRY(launch_topk_candidates((int64_t)cn, L, d_cl, d_ck, d_ci, d_seg, d_need, d_chosen, nullptr, st));
            return LDGPU_OK;
        }
        // each rank's need[l] smallest candidates can hold the global ones:
        // gather those prefixes, the need[l]-th smallest key of language l is
        // its threshold, and every rank takes its candidates at or below it
        uint64_t* d_sk;
        HIP_TRY(db.alloc(&d_sk, cn));
        HIP_TRY(db.alloc(&d_thr, L));
        HIP_TRY(launch_topk_candidates((int64_t)cn, L, d_cl, d_ck, d_ci, d_seg, d_need, d_chosen, d_sk, st));
        for (int l = 0; l < L; ++l) tot += take[l] = std::min<int64_t>(need[l], seg[l + 1] - seg[l]);
        pre.assign((size_t)std::max<int64_t>(tot, 1), 0);
        int64_t at = 0;
        for (int l = 0; l < L; ++l) {
            if (take[l])
                HIP_TRY(hipMemcpyAsync(pre.data() + at, d_sk + seg[l], sizeof(uint64_t) * take[l],
                                       hipMemcpyDeviceToHost, st));
            at += take[l];
        }
        HIP_TRY(hipStreamSynchronize(st));
        return LDGPU_OK;
    };
    if (int rc = agree(select_phase())) return rc;
    std::vector<uint64_t> thr(L, 0);
    if (multi) {
        std::vector<uint8_t> blob;
        put(blob, take.data(), take.size());
        put(blob, pre.data(), (size_t)tot);
        std::vector<std::vector<uint8_t>> all;
        if (int rc = comm_allgatherv_host(cm, blob, all)) return rc;
        std::vector<std::vector<uint64_t>> per(L);
        for (int r = 0; r < cm->world; ++r) {
            const int64_t* tk = reinterpret_cast<const int64_t*>(all[r].data());
            const uint64_t* ks = reinterpret_cast<const uint64_t*>(tk + L);
            for (int l = 0; l < L; ++l) {
                per[l].insert(per[l].end(), ks, ks + tk[l]);
                ks += tk[l];
            }
        }
        // (from gathered data: every rank takes the same branch here)
        for (int l = 0; l < L; ++l) {
            if (need[l] <= 0) continue;
            if ((int64_t)per[l].size() < need[l])
                return fail(LDGPU_EDEVICE, "top-K: %zu candidates of language %d, %d needed", per[l].size(), l,
                            need[l]);
            std::nth_element(per[l].begin(), per[l].begin() + (need[l] - 1), per[l].end());
            thr[l] = per[l][need[l] - 1];
        }
    }
    mark("table: threshold ties");
    const int64_t cap_out = std::min<int64_t>(n, (int64_t)L * std::max<int32_t>(K, 0));
    uint64_t *d_ok = nullptr, *d_om = nullptr;
    int32_t* d_okk = nullptr;
    uint32_t* d_outrow = nullptr;
    unsigned long long m = 0;
    std::vector<uint64_t> ok, om;  // multi-rank: this rank's chosen rows, gathered below
    std::vector<int32_t> okk;
    auto rows_phase = [&]() -> int {
        if (int rc = injected("table_rows")) return rc;
        if (multi) {
            HIP_TRY(hipMemcpyAsync(d_thr, thr.data(), sizeof(uint64_t) * L, hipMemcpyHostToDevice, st));
            HIP_TRY(launch_mark_threshold((int64_t)cn, d_cl, d_ck, d_ci, d_thr, d_chosen, st));
        }
        HIP_TRY(db.alloc(&d_ok, cap_out));
        HIP_TRY(db.alloc(&d_okk, cap_out));
        HIP_TRY(db.alloc(&d_outrow, n));
        HIP_TRY(hipMemsetAsync(d_n + 1, 0, sizeof(unsigned long long), st));
        HIP_TRY(launch_gather_rows(n, d_chosen, d_keys, d_k, d_ok, d_okk, d_outrow, d_n + 1, cap_out, st));
        HIP_TRY(hipMemcpyAsync(&m, d_n + 1, sizeof m, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if ((int64_t)m > cap_out)
            return fail(LDGPU_EDEVICE, "top-K: %llu grams chosen, at most %lld expected", m, (long long)cap_out);
        mark("table: gather rows");
        HIP_TRY(db.alloc(&d_om, (size_t)std::max<unsigned long long>(m, 1) * S));
        HIP_TRY(hipMemsetAsync(d_om, 0, sizeof(uint64_t) * std::max<unsigned long long>(m, 1) * S, st));
        HIP_TRY(launch_rows_final(cp, c->cap, d_outrow, d_rk, st));  // (rk's rows are not read after this)
        HIP_TRY(launch_pair_masks(cp, c->pcap, d_rk, nullptr, S, d_om, st));
        mark("table: masks");
        if (multi && m) {
            ok.resize(m);
            om.resize((size_t)m * S);
            okk.resize(m);
            HIP_TRY(hipMemcpyAsync(ok.data(), d_ok, sizeof(uint64_t) * m, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(om.data(), d_om, sizeof(uint64_t) * m * S, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(okk.data(), d_okk, sizeof(int32_t) * m, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        return LDGPU_OK;
    };
    if (int rc = agree(rows_phase())) return rc;
    std::vector<double> w(L + 1, 0.0);
    for (int k = 1; k <= L; ++k) w[k] = std::log(1.0 + 1.0 / (double)k);
    if (!multi) {
        // one rank: the rows sorted by (length, bytes) on the device (radix
        // sort of the sort keys, then a gather), copied back in table order
        uint64_t *d_sk, *d_ok2, *d_om2;
        unsigned long long* d_idx;
        int32_t* d_okk2;
        const size_t mm = std::max<unsigned long long>(m, 1);
        HIP_TRY(db.alloc(&d_sk, mm));
        HIP_TRY(db.alloc(&d_idx, mm));
        HIP_TRY(db.alloc(&d_ok2, mm));
        HIP_TRY(db.alloc(&d_okk2, mm));
        HIP_TRY(db.alloc(&d_om2, mm * S));
        HIP_TRY(launch_sort_keys_of((int64_t)m, d_ok, d_sk, d_idx, st));
        HIP_TRY(sort_pairs_u64((int64_t)m, d_sk, d_idx, 64, st));
        HIP_TRY(launch_rows_permute((int64_t)m, S, d_idx, d_ok, d_okk, d_om, d_ok2, d_okk2, d_om2, st));
        mark("table: row sort");
        // the rows come back in one DMA into pinned memory (a copy into
        // pageable vectors ran at a fraction of PCIe), then host threads
        // fill the table cache from it
        // The rows stay in the context's pinned buffer, landed by one DMA
        // (pageable vectors took a copy at a fraction of PCIe plus page
        // faults): the exports copy from it straight into the caller's
        // buffers.  Another table's build first moves its owner's rows out.
        ldgpu_ctx* x = c->ctx;
        if (ldgpu_counts* o = x->h_tbl_owner; o && o != c) {
            if (o->tbl_valid) {
                tbl_materialize(o);
            } else {  // (a stale table: nothing to keep)
                o->tbl_pin = false;
                x->h_tbl_owner = nullptr;
            }
        }
        c->tbl_pin = false;
        const size_t hb = (size_t)m * (8 + 8 * (size_t)S + 4);
        HIP_TRY(x->h_tbl.ensure(hb + 16));
        uint64_t* h_keys = (uint64_t*)x->h_tbl.p;
        uint64_t* h_masks = h_keys + m;
        int32_t* h_k = (int32_t*)(h_masks + (size_t)m * S);
        if (m) {
            HIP_TRY(hipMemcpyAsync(h_keys, d_ok2, sizeof(uint64_t) * m, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(h_masks, d_om2, sizeof(uint64_t) * m * S, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(h_k, d_okk2, sizeof(int32_t) * m, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        mark("table: copy back");
        std::atomic<int64_t> nb_acc{0};
        par_for((int64_t)m, [&](int64_t a, int64_t b) {
            int64_t t = 0;
            for (int64_t r = a; r < b; ++r) t += key_len(h_keys[r]);
            nb_acc += t;
        });
        const int64_t nb = nb_acc.load();
        c->tbl_masks.clear();
        c->tbl_vals.clear();
        c->tbl_bytes.clear();
        c->tbl_off.assign(1, 0);
        c->tbl_rows = (int64_t)m;
        c->tbl_kb = nb;
        c->tbl_pin = true;
        x->h_tbl_owner = c;
        c->tbl_valid = true;
        if (n_rows) *n_rows = (int64_t)m;
        if (key_bytes) *key_bytes = nb;
        mark("table: host rows");
        return LDGPU_OK;
    }
    {  // every rank's chosen rows
        std::vector<uint8_t> blob;
        put(blob, ok.data(), ok.size());
        put(blob, om.data(), om.size());
        put(blob, okk.data(), okk.size());
        std::vector<std::vector<uint8_t>> all;
        if (int rc = comm_allgatherv_host(cm, blob, all)) return rc;
        ok.clear();
        om.clear();
        okk.clear();
        for (int r = 0; r < cm->world; ++r) {
            const size_t nr = all[r].size() / (8 + 8 * S + 4);
            const uint64_t* k = reinterpret_cast<const uint64_t*>(all[r].data());
            const uint64_t* mk = k + nr;
            const int32_t* kk = reinterpret_cast<const int32_t*>(mk + nr * S);
            ok.insert(ok.end(), k, k + nr);
            om.insert(om.end(), mk, mk + nr * S);
            okk.insert(okk.end(), kk, kk + nr);
        }
        m = ok.size();
    }
    std::vector<std::pair<uint64_t, uint64_t>> order(m);
    for (uint64_t i = 0; i < m; ++i) order[i] = {sort_key(ok[i]), i};
    std::sort(order.begin(), order.end());
    std::vector<uint64_t> out_keys(m);
    c->tbl_masks.assign((size_t)m * S, 0);
    c->tbl_vals.assign((size_t)m, 0.0);
    for (uint64_t r = 0; r < m; ++r) {
        const uint64_t i = order[r].second;
        out_keys[r] = ok[i];
        memcpy(&c->tbl_masks[r * S], &om[i * S], sizeof(uint64_t) * S);
        c->tbl_vals[r] = w[okk[i]];
    }
    int64_t nb = 0;
    for (uint64_t k : out_keys) nb += key_len(k);
    c->tbl_bytes.assign((size_t)std::max<int64_t>(nb, 1), 0);
    c->tbl_off.assign(out_keys.size() + 1, 0);
    write_keys(c, out_keys, c->tbl_bytes.data(), c->tbl_off.data());
    c->tbl_valid = true;
    if (n_rows) *n_rows = (int64_t)m;
    if (key_bytes) *key_bytes = nb;
    return LDGPU_OK;
}
}  // namespace

// computeProbabilities + filterTopGrams (LanguageDetector.scala:75-132).
// On a merged table: collective (every rank of the communicator calls it).
extern "C" int ldgpu_fit_table_size(ldgpu_counts* c, int32_t K, int64_t* n_rows, int64_t* key_bytes) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    HIP_TRY(hipSetDevice(c->ctx->device));
    // the previous table (pinned or in the vectors) is replaced whatever path builds this one
    c->tbl_valid = false;
    c->tbl_pin = false;
    if (c->ctx->h_tbl_owner == c) c->ctx->h_tbl_owner = nullptr;
    // a merged table takes the device path on every rank (its collectives
    // must match), even for K <= 0 or an empty shard
    // (tables holding grams of 8..15 bytes take the host top-K over the
    // pulled table, whose keys stay in (length, bytes) order)
    if (!c->comm && (K <= 0 || c->size == 0 || c->wsize > 0 || c->lsize > 0)) {
        if (int rc = fit_table_host(c, K, n_rows, key_bytes)) return rc;
        return ok();
    }
    if (K <= 0) {
        c->tbl_masks.clear();
        c->tbl_vals.clear();
        c->tbl_bytes.assign(1, 0);
        c->tbl_off.assign(1, 0);
        c->tbl_valid = true;
        if (n_rows) *n_rows = 0;
        if (key_bytes) *key_bytes = 0;
        return ok();
    }
    bool fallback = false;
    if (int rc = fit_table_device(c, K, n_rows, key_bytes, &fallback)) return rc;
    if (fallback) {
        if (int rc = fit_table_host(c, K, n_rows, key_bytes)) return rc;
    }
    return ok();
}

extern "C" int ldgpu_fit_table_info(ldgpu_counts* c, int64_t* n_rows, int64_t* key_bytes) {
    if (!c) return fail(LDGPU_EINVAL, "counts is NULL");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    if (!c->tbl_valid) return fail(LDGPU_EINVAL, "call ldgpu_fit_table_size first");
    if (n_rows) *n_rows = tbl_rows(c);
    if (key_bytes) *key_bytes = tbl_key_bytes(c);
    return ok();
}

extern "C" int ldgpu_fit_table_export(ldgpu_counts* c, uint8_t* key_bytes, int64_t* key_offsets, double* rows) {
    if (!c || !key_offsets || !rows) return fail(LDGPU_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    if (!c->tbl_valid) return fail(LDGPU_EINVAL, "call ldgpu_fit_table_size first");
    tbl_materialize(c);  // (dense rows: from the vectors)
    const size_t n = c->tbl_off.size() - 1;
    if (c->tbl_off[n] && !key_bytes) return fail(LDGPU_EINVAL, "key_bytes is NULL");
    if (c->tbl_off[n]) memcpy(key_bytes, c->tbl_bytes.data(), (size_t)c->tbl_off[n]);
    memcpy(key_offsets, c->tbl_off.data(), sizeof(int64_t) * (n + 1));
    const int L = c->L, S = (L + 63) / 64;
    for (size_t r = 0; r < n; ++r)
        for (int l = 0; l < L; ++l)
            rows[r * L + l] = ((c->tbl_masks[r * S + l / 64] >> (l % 64)) & 1ull) ? c->tbl_vals[r] : 0.0;
    return ok();
}

extern "C" int ldgpu_fit_table_export_masks(ldgpu_counts* c, uint8_t* key_bytes, int64_t* key_offsets,
                                            uint64_t* masks, double* vals) {
    if (!c || !key_offsets || !masks || !vals) return fail(LDGPU_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lock(c->ctx->mu);
    if (!c->tbl_valid) return fail(LDGPU_EINVAL, "call ldgpu_fit_table_size first");
    if (c->tbl_pin) {  // straight from the pinned rows into the caller's buffers
        const PinnedTable t = pinned_table(c);
        const int64_t m = c->tbl_rows;
        const int S = (c->L + 63) / 64;
        if (c->tbl_kb && !key_bytes) return fail(LDGPU_EINVAL, "key_bytes is NULL");
        key_offsets[0] = 0;
        for (int64_t i = 0; i < m; ++i) key_offsets[i + 1] = key_offsets[i] + key_len(t.keys[i]);
        par_for(m, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) {
                const uint64_t k = t.keys[i];
                for (int64_t j = 0; j < key_offsets[i + 1] - key_offsets[i]; ++j)
                    key_bytes[key_offsets[i] + j] = (uint8_t)(k >> (8 * j));
                vals[i] = row_value(t.k[i]);
            }
            memcpy(masks + (size_t)a * S, t.masks + (size_t)a * S, sizeof(uint64_t) * (size_t)(b - a) * S);
        });
        return ok();
    }
    const size_t n = c->tbl_off.size() - 1;
    if (c->tbl_off[n] && !key_bytes) return fail(LDGPU_EINVAL, "key_bytes is NULL");
    if (c->tbl_off[n]) par_memcpy(key_bytes, c->tbl_bytes.data(), (size_t)c->tbl_off[n]);
    par_memcpy(key_offsets, c->tbl_off.data(), sizeof(int64_t) * (n + 1));
    if (n) {
        par_memcpy(masks, c->tbl_masks.data(), sizeof(uint64_t) * c->tbl_masks.size());
        par_memcpy(vals, c->tbl_vals.data(), sizeof(double) * n);
    }
    return ok();
}
