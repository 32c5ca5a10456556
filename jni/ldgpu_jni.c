/* ldgpu_jni.c -- JNI shim between the Scala drop-in
 * (scala/.../LdgpuNative.scala, object LdgpuNative: its @native methods are
 * instance methods of the module class LdgpuNative$, hence the _00024 in the
 * symbol names) and the C ABI of libldgpu.so (include/ldgpu.h).
 *
 * Every buffer is a direct java.nio.ByteBuffer in native byte order; the shim
 * passes its address straight through (no copies) after checking that the
 * buffer's capacity covers every byte the call reads or writes (the C ABI
 * trusts its pointers: a short buffer would be read or written past its end).
 * A short or missing buffer fails the call with LDGPU_EINVAL and a message of
 * the shim's own (lastError).  Handles are the C pointers as jlong.  Status
 * codes are returned unchanged; the Scala side turns them into the
 * reference's exceptions (LdgpuNative.check).
 *
 * Build (on a box with a JDK; not in this image):
 *   make -C jni JAVA_HOME=/usr/lib/jvm/java-8-openjdk-amd64
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../include/ldgpu.h"

#define FN(name) Java_org_apache_spark_ml_feature_languagedetection_LdgpuNative_00024_##name

/* the shim's own failure message (a buffer check), else the library's */
static __thread char jerr[256];

static void jclear(void) { jerr[0] = 0; }

static void* addr(JNIEnv* env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }

/* LDGPU_OK when `buf` is a direct buffer of at least `bytes` bytes (or the
 * call touches none of it), else LDGPU_EINVAL with a message.  A negative
 * byte count (a size that went negative or overflowed on the way) fails. */
static int need(JNIEnv* env, jobject buf, int64_t bytes, const char* what) {
    if (bytes < 0) {
        snprintf(jerr, sizeof jerr, "%s: negative or overflowing size", what);
        return LDGPU_EINVAL;
    }
    if (bytes == 0) return LDGPU_OK;
    if (!buf) {
        snprintf(jerr, sizeof jerr, "%s is null but %lld bytes are needed", what, (long long)bytes);
        return LDGPU_EINVAL;
    }
    const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    if (cap < 0 || !addr(env, buf)) {
        snprintf(jerr, sizeof jerr, "%s is not a direct buffer", what);
        return LDGPU_EINVAL;
    }
    if ((int64_t)cap < bytes) {
        snprintf(jerr, sizeof jerr, "%s holds %lld bytes, the call needs %lld", what, (long long)cap,
                 (long long)bytes);
        return LDGPU_EINVAL;
    }
    return LDGPU_OK;
}

/* elem * a * b bytes, or -1 when a factor is negative or the product
 * overflows int64 (need() then fails the call) */
static int64_t bytes_of(int64_t elem, int64_t a, int64_t b) {
    if (a < 0 || b < 0) return -1;
    int64_t r;
    if (__builtin_mul_overflow(elem, a, &r) || __builtin_mul_overflow(r, b, &r)) return -1;
    return r;
}

/* an int64 offsets buffer of n + 1 entries (n >= 0) whose first entry is >= 0
 * and whose last is >= the first; *last = offsets[n] (the bytes a call reads
 * from the matching byte buffer).  (The library checks the entries between.) */
static int need_offsets(JNIEnv* env, jobject offsets, int64_t n, const char* what, int64_t* last) {
    const int rc = need(env, offsets, bytes_of(8, n < 0 || n == INT64_MAX ? -1 : n + 1, 1), what);
    if (rc != LDGPU_OK) return rc;
    const int64_t* o = (const int64_t*)addr(env, offsets);
    if (!o) {
        snprintf(jerr, sizeof jerr, "%s is not a direct buffer", what);
        return LDGPU_EINVAL;
    }
    if (o[0] < 0 || o[n] < o[0]) {
        snprintf(jerr, sizeof jerr, "%s: first entry %lld, last %lld", what, (long long)o[0], (long long)o[n]);
        return LDGPU_EINVAL;
    }
    *last = o[n];
    return LDGPU_OK;
}

/* LDGPU_OK when the caller's size equals the handle's own (the library sizes
 * every buffer from the handle: a caller that assumed another language count
 * or row count would read or write its rows with the wrong stride) */
static int same(int64_t caller, int64_t own, const char* what) {
    if (caller == own) return LDGPU_OK;
    snprintf(jerr, sizeof jerr, "%s %lld does not match the handle's %lld", what, (long long)caller, (long long)own);
    return LDGPU_EINVAL;
}

#define CHECK(expr)                      \
    do {                                 \
        const int rc_ = (expr);          \
        if (rc_ != LDGPU_OK) return rc_; \
    } while (0)

static int put_handle(JNIEnv* env, jlongArray out, void* h, int rc) {
    if (rc == LDGPU_OK) {
        jlong v = (jlong)(intptr_t)h;
        (*env)->SetLongArrayRegion(env, out, 0, 1, &v);
    }
    return rc;
}

/* a copy of a Java int[] (gram lengths) */
static int32_t* ints(JNIEnv* env, jintArray a, jsize* n) {
    *n = a ? (*env)->GetArrayLength(env, a) : 0;
    return a ? (int32_t*)(*env)->GetIntArrayElements(env, a, NULL) : NULL;
}

static void ints_release(JNIEnv* env, jintArray a, int32_t* p) {
    if (a && p) (*env)->ReleaseIntArrayElements(env, a, (jint*)p, JNI_ABORT);
}

JNIEXPORT jstring JNICALL FN(lastError)(JNIEnv* env, jobject self) {
    (void)self;
    return (*env)->NewStringUTF(env, jerr[0] ? jerr : ldgpu_last_error());
}

JNIEXPORT jint JNICALL FN(ctxCreate)(JNIEnv* env, jobject self, jint device, jlongArray out) {
    (void)self;
    jclear();
    ldgpu_ctx* c = NULL;
    const int rc = ldgpu_ctx_create(device, &c);
    return put_handle(env, out, c, rc);
}

/* pinned host memory wrapped as a direct ByteBuffer (NULL on failure) */
JNIEXPORT jobject JNICALL FN(hostAlloc)(JNIEnv* env, jobject self, jlong ctx, jlong bytes) {
    (void)self;
    jclear();
    void* p = NULL;
    if (bytes < 0 || ldgpu_host_alloc((ldgpu_ctx*)(intptr_t)ctx, bytes, &p) != LDGPU_OK || !p) return NULL;
    return (*env)->NewDirectByteBuffer(env, p, bytes > 0 ? bytes : 1);
}

JNIEXPORT jint JNICALL FN(hostFree)(JNIEnv* env, jobject self, jlong ctx, jobject buf) {
    (void)self;
    jclear();
    return ldgpu_host_free((ldgpu_ctx*)(intptr_t)ctx, addr(env, buf));
}

JNIEXPORT jint JNICALL FN(modelCreate)(JNIEnv* env, jobject self, jlong ctx, jlong n_rows, jobject key_bytes,
                                       jobject key_offsets, jobject rows, jobject row_ok, jint n_langs,
                                       jintArray gram_lengths, jlongArray out) {
    (void)self;
    jclear();
    if (n_rows < 0 || n_langs < 1) return ldgpu_model_create((ldgpu_ctx*)(intptr_t)ctx, n_rows, NULL, NULL, NULL,
                                                             NULL, n_langs, NULL, 0, NULL);  /* its own EINVAL */
    int64_t nb = 0;
    CHECK(need_offsets(env, key_offsets, n_rows, "keyOffsets", &nb));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    CHECK(need(env, rows, bytes_of(8, n_rows, n_langs), "rows"));
    if (row_ok) CHECK(need(env, row_ok, n_rows, "rowOk"));
    jsize ng = 0;
    int32_t* g = ints(env, gram_lengths, &ng);
    ldgpu_model* m = NULL;
    const int rc = ldgpu_model_create((ldgpu_ctx*)(intptr_t)ctx, n_rows, (const uint8_t*)addr(env, key_bytes),
                                      (const int64_t*)addr(env, key_offsets), (const double*)addr(env, rows),
                                      (const uint8_t*)addr(env, row_ok), n_langs, g, ng, &m);
    ints_release(env, gram_lengths, g);
    return put_handle(env, out, m, rc);
}

JNIEXPORT jint JNICALL FN(modelCreateMasks)(JNIEnv* env, jobject self, jlong ctx, jlong n_rows, jobject key_bytes,
                                            jobject key_offsets, jobject masks, jobject vals, jint n_langs,
                                            jintArray gram_lengths, jlongArray out) {
    (void)self;
    jclear();
    if (n_rows < 0 || n_langs < 1)
        return ldgpu_model_create_masks((ldgpu_ctx*)(intptr_t)ctx, n_rows, NULL, NULL, NULL, NULL, n_langs, NULL, 0,
                                        NULL);  /* its own EINVAL */
    int64_t nb = 0;
    CHECK(need_offsets(env, key_offsets, n_rows, "keyOffsets", &nb));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    CHECK(need(env, masks, bytes_of(8, n_rows, ((int64_t)n_langs + 63) / 64), "masks"));
    CHECK(need(env, vals, bytes_of(8, n_rows, 1), "vals"));
    jsize ng = 0;
    int32_t* g = ints(env, gram_lengths, &ng);
    ldgpu_model* m = NULL;
    const int rc = ldgpu_model_create_masks((ldgpu_ctx*)(intptr_t)ctx, n_rows, (const uint8_t*)addr(env, key_bytes),
                                            (const int64_t*)addr(env, key_offsets),
                                            (const uint64_t*)addr(env, masks), (const double*)addr(env, vals),
                                            n_langs, g, ng, &m);
    ints_release(env, gram_lengths, g);
    return put_handle(env, out, m, rc);
}

JNIEXPORT jint JNICALL FN(modelDestroy)(JNIEnv* env, jobject self, jlong model) {
    (void)env;
    (void)self;
    jclear();
    return ldgpu_model_destroy((ldgpu_model*)(intptr_t)model);
}

/* ldgpu_score: thread-safe; concurrent task threads run on their own streams.
 * The scores buffer is sized by the model's own language count, which the
 * caller's n_langs must equal. */
JNIEXPORT jint JNICALL FN(score)(JNIEnv* env, jobject self, jlong model, jobject bytes, jobject offsets,
                                 jlong n_docs, jobject labels, jobject scores, jint n_langs) {
    (void)self;
    jclear();
    if (n_docs < 0) return ldgpu_score((ldgpu_model*)(intptr_t)model, NULL, NULL, n_docs, NULL, NULL);
    int64_t nb = 0;
    CHECK(need_offsets(env, offsets, n_docs, "offsets", &nb));
    CHECK(need(env, bytes, nb, "bytes"));
    CHECK(need(env, labels, bytes_of(4, n_docs, 1), "labels"));
    if (scores) {
        int32_t L = 0;
        CHECK(ldgpu_model_langs((const ldgpu_model*)(intptr_t)model, &L));
        CHECK(same(n_langs, L, "nLangs"));
        CHECK(need(env, scores, bytes_of(8, n_docs, L), "scores"));
    }
    return ldgpu_score((ldgpu_model*)(intptr_t)model, (const uint8_t*)addr(env, bytes),
                       (const int64_t*)addr(env, offsets), n_docs, (int32_t*)addr(env, labels),
                       (double*)addr(env, scores));
}

JNIEXPORT jint JNICALL FN(countsCreate)(JNIEnv* env, jobject self, jlong ctx, jint n_langs, jintArray gram_lengths,
                                        jlong capacity_hint, jlongArray out) {
    (void)self;
    jclear();
    jsize ng = 0;
    int32_t* g = ints(env, gram_lengths, &ng);
    ldgpu_counts* c = NULL;
    const int rc = ldgpu_counts_create((ldgpu_ctx*)(intptr_t)ctx, n_langs, g, ng, capacity_hint, &c);
    ints_release(env, gram_lengths, g);
    return put_handle(env, out, c, rc);
}

JNIEXPORT jint JNICALL FN(countsDestroy)(JNIEnv* env, jobject self, jlong counts) {
    (void)env;
    (void)self;
    jclear();
    return ldgpu_counts_destroy((ldgpu_counts*)(intptr_t)counts);
}

JNIEXPORT jint JNICALL FN(count)(JNIEnv* env, jobject self, jlong counts, jobject bytes, jobject offsets,
                                 jobject doc_lang, jlong n_docs) {
    (void)self;
    jclear();
    if (n_docs < 0) return ldgpu_count((ldgpu_counts*)(intptr_t)counts, NULL, NULL, NULL, n_docs);
    int64_t nb = 0;
    CHECK(need_offsets(env, offsets, n_docs, "offsets", &nb));
    CHECK(need(env, bytes, nb, "bytes"));
    CHECK(need(env, doc_lang, bytes_of(4, n_docs, 1), "docLang"));
    return ldgpu_count((ldgpu_counts*)(intptr_t)counts, (const uint8_t*)addr(env, bytes),
                       (const int64_t*)addr(env, offsets), (const int32_t*)addr(env, doc_lang), n_docs);
}

JNIEXPORT jint JNICALL FN(countsSize)(JNIEnv* env, jobject self, jlong counts, jlongArray out) {
    (void)self;
    jclear();
    int64_t v[2] = {0, 0};
    const int rc = ldgpu_counts_size((ldgpu_counts*)(intptr_t)counts, &v[0], &v[1]);
    if (rc == LDGPU_OK) {
        jlong j[2] = {(jlong)v[0], (jlong)v[1]};
        (*env)->SetLongArrayRegion(env, out, 0, 2, j);
    }
    return rc;
}

/* sizes from the table itself (the caller's n_langs must equal its language count) */
JNIEXPORT jint JNICALL FN(countsExport)(JNIEnv* env, jobject self, jlong counts, jobject key_bytes,
                                        jobject key_offsets, jobject counts_out, jint n_langs) {
    (void)self;
    jclear();
    int64_t n = 0, nb = 0;
    int32_t L = 0;
    CHECK(ldgpu_counts_langs((const ldgpu_counts*)(intptr_t)counts, &L));
    CHECK(same(n_langs, L, "nLangs"));
    CHECK(ldgpu_counts_size((ldgpu_counts*)(intptr_t)counts, &n, &nb));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    CHECK(need(env, key_offsets, bytes_of(8, n + 1, 1), "keyOffsets"));
    CHECK(need(env, counts_out, bytes_of(8, n, L), "counts"));
    return ldgpu_counts_export((ldgpu_counts*)(intptr_t)counts, (uint8_t*)addr(env, key_bytes),
                               (int64_t*)addr(env, key_offsets), (int64_t*)addr(env, counts_out));
}

/* out(0) = key bytes, out(1) = (language, count) pairs of grams [first, first + n) */
JNIEXPORT jint JNICALL FN(countsSparseSize)(JNIEnv* env, jobject self, jlong counts, jlong first, jlong n,
                                            jlongArray out) {
    (void)self;
    jclear();
    int64_t v[2] = {0, 0};
    const int rc = ldgpu_counts_sparse_size((ldgpu_counts*)(intptr_t)counts, first, n, &v[0], &v[1]);
    if (rc == LDGPU_OK) {
        jlong j[2] = {(jlong)v[0], (jlong)v[1]};
        (*env)->SetLongArrayRegion(env, out, 0, 2, j);
    }
    return rc;
}

JNIEXPORT jint JNICALL FN(countsExportSparse)(JNIEnv* env, jobject self, jlong counts, jlong first, jlong n,
                                              jobject key_bytes, jobject key_offsets, jobject pair_offsets,
                                              jobject pair_langs, jobject pair_counts) {
    (void)self;
    jclear();
    int64_t nb = 0, np = 0;
    CHECK(ldgpu_counts_sparse_size((ldgpu_counts*)(intptr_t)counts, first, n, &nb, &np));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    CHECK(need(env, key_offsets, bytes_of(8, n + 1, 1), "keyOffsets"));
    CHECK(need(env, pair_offsets, bytes_of(8, n + 1, 1), "pairOffsets"));
    CHECK(need(env, pair_langs, bytes_of(4, np, 1), "pairLangs"));
    CHECK(need(env, pair_counts, bytes_of(8, np, 1), "pairCounts"));
    return ldgpu_counts_export_sparse((ldgpu_counts*)(intptr_t)counts, first, n, (uint8_t*)addr(env, key_bytes),
                                      (int64_t*)addr(env, key_offsets), (int64_t*)addr(env, pair_offsets),
                                      (int32_t*)addr(env, pair_langs), (int64_t*)addr(env, pair_counts));
}

JNIEXPORT jint JNICALL FN(countsAddSparse)(JNIEnv* env, jobject self, jlong counts, jlong n, jobject key_bytes,
                                           jobject key_offsets, jobject pair_offsets, jobject pair_langs,
                                           jobject pair_counts) {
    (void)self;
    jclear();
    if (n <= 0)
        return ldgpu_counts_add_sparse((ldgpu_counts*)(intptr_t)counts, n, NULL, NULL, NULL, NULL, NULL);
    int64_t nb = 0, pl = 0;
    CHECK(need_offsets(env, key_offsets, n, "keyOffsets", &nb));
    CHECK(need_offsets(env, pair_offsets, n, "pairOffsets", &pl));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    const int64_t* po = (const int64_t*)addr(env, pair_offsets);
    const int64_t np = pl - po[0];  /* the pairs are read from index 0 */
    CHECK(need(env, pair_langs, bytes_of(4, np, 1), "pairLangs"));
    CHECK(need(env, pair_counts, bytes_of(8, np, 1), "pairCounts"));
    return ldgpu_counts_add_sparse((ldgpu_counts*)(intptr_t)counts, n, (const uint8_t*)addr(env, key_bytes),
                                   (const int64_t*)addr(env, key_offsets), po, (const int32_t*)addr(env, pair_langs),
                                   (const int64_t*)addr(env, pair_counts));
}

/* rows are n x the table's own language count (the caller's n_langs must equal it) */
JNIEXPORT jint JNICALL FN(countsAdd)(JNIEnv* env, jobject self, jlong counts, jlong n, jobject key_bytes,
                                     jobject key_offsets, jobject rows, jint n_langs) {
    (void)self;
    jclear();
    if (n <= 0) return ldgpu_counts_add((ldgpu_counts*)(intptr_t)counts, n, NULL, NULL, NULL);
    int64_t nb = 0;
    int32_t L = 0;
    CHECK(ldgpu_counts_langs((const ldgpu_counts*)(intptr_t)counts, &L));
    CHECK(same(n_langs, L, "nLangs"));
    CHECK(need_offsets(env, key_offsets, n, "keyOffsets", &nb));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    CHECK(need(env, rows, bytes_of(8, n, L), "rows"));
    return ldgpu_counts_add((ldgpu_counts*)(intptr_t)counts, n, (const uint8_t*)addr(env, key_bytes),
                            (const int64_t*)addr(env, key_offsets), (const int64_t*)addr(env, rows));
}

JNIEXPORT jint JNICALL FN(fitTableSize)(JNIEnv* env, jobject self, jlong counts, jint profile_size, jlongArray out) {
    (void)self;
    jclear();
    int64_t v[2] = {0, 0};
    const int rc = ldgpu_fit_table_size((ldgpu_counts*)(intptr_t)counts, profile_size, &v[0], &v[1]);
    if (rc == LDGPU_OK) {
        jlong j[2] = {(jlong)v[0], (jlong)v[1]};
        (*env)->SetLongArrayRegion(env, out, 0, 2, j);
    }
    return rc;
}

/* The cached table's sizes come from the library (ldgpu_fit_table_info) and
 * the table's own language count; the caller's n_rows / key_bytes_n /
 * n_langs must equal them. */
static int table_sizes(jlong counts, int64_t* n_rows, int64_t* key_bytes, int32_t* L, int64_t c_rows, int64_t c_bytes,
                       int64_t c_langs) {
    CHECK(ldgpu_counts_langs((const ldgpu_counts*)(intptr_t)counts, L));
    CHECK(ldgpu_fit_table_info((ldgpu_counts*)(intptr_t)counts, n_rows, key_bytes));
    CHECK(same(c_langs, *L, "nLangs"));
    CHECK(same(c_rows, *n_rows, "nRows"));
    return same(c_bytes, *key_bytes, "keyBytesN");
}

JNIEXPORT jint JNICALL FN(fitTableExport)(JNIEnv* env, jobject self, jlong counts, jobject key_bytes,
                                          jobject key_offsets, jobject rows, jlong n_rows, jlong key_bytes_n,
                                          jint n_langs) {
    (void)self;
    jclear();
    int64_t nr = 0, nb = 0;
    int32_t L = 0;
    CHECK(table_sizes(counts, &nr, &nb, &L, n_rows, key_bytes_n, n_langs));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    CHECK(need(env, key_offsets, bytes_of(8, nr + 1, 1), "keyOffsets"));
    CHECK(need(env, rows, bytes_of(8, nr, L), "rows"));
    return ldgpu_fit_table_export((ldgpu_counts*)(intptr_t)counts, (uint8_t*)addr(env, key_bytes),
                                  (int64_t*)addr(env, key_offsets), (double*)addr(env, rows));
}

/* the same table in mask form: masks [n_rows][ceil(n_langs / 64)], vals [n_rows] */
JNIEXPORT jint JNICALL FN(fitTableExportMasks)(JNIEnv* env, jobject self, jlong counts, jobject key_bytes,
                                               jobject key_offsets, jobject masks, jobject vals, jlong n_rows,
                                               jlong key_bytes_n, jint n_langs) {
    (void)self;
    jclear();
    int64_t nr = 0, nb = 0;
    int32_t L = 0;
    CHECK(table_sizes(counts, &nr, &nb, &L, n_rows, key_bytes_n, n_langs));
    CHECK(need(env, key_bytes, nb, "keyBytes"));
    CHECK(need(env, key_offsets, bytes_of(8, nr + 1, 1), "keyOffsets"));
    CHECK(need(env, masks, bytes_of(8, nr, ((int64_t)L + 63) / 64), "masks"));
    CHECK(need(env, vals, bytes_of(8, nr, 1), "vals"));
    return ldgpu_fit_table_export_masks((ldgpu_counts*)(intptr_t)counts, (uint8_t*)addr(env, key_bytes),
                                        (int64_t*)addr(env, key_offsets), (uint64_t*)addr(env, masks),
                                        (double*)addr(env, vals));
}

/* ---- multi-GPU merge: one task per GPU (Spark barrier execution) */
JNIEXPORT jbyteArray JNICALL FN(commUniqueId)(JNIEnv* env, jobject self) {
    (void)self;
    jclear();
    uint8_t id[LDGPU_COMM_ID_BYTES];
    if (ldgpu_comm_unique_id(id) != LDGPU_OK) return NULL;
    jbyteArray a = (*env)->NewByteArray(env, LDGPU_COMM_ID_BYTES);
    if (a) (*env)->SetByteArrayRegion(env, a, 0, LDGPU_COMM_ID_BYTES, (const jbyte*)id);
    return a;
}

JNIEXPORT jint JNICALL FN(commCreateRccl)(JNIEnv* env, jobject self, jlong ctx, jbyteArray id, jint rank,
                                          jint world, jlongArray out) {
    (void)self;
    jclear();
    uint8_t buf[LDGPU_COMM_ID_BYTES];
    if (!id || (*env)->GetArrayLength(env, id) != LDGPU_COMM_ID_BYTES) {
        snprintf(jerr, sizeof jerr, "communicator id must hold %d bytes", LDGPU_COMM_ID_BYTES);
        return LDGPU_EINVAL;
    }
    (*env)->GetByteArrayRegion(env, id, 0, LDGPU_COMM_ID_BYTES, (jbyte*)buf);
    ldgpu_comm* m = NULL;
    const int rc = ldgpu_comm_create_rccl((ldgpu_ctx*)(intptr_t)ctx, buf, rank, world, &m);
    return put_handle(env, out, m, rc);
}

JNIEXPORT jint JNICALL FN(commDestroy)(JNIEnv* env, jobject self, jlong comm) {
    (void)env;
    (void)self;
    jclear();
    return ldgpu_comm_destroy((ldgpu_comm*)(intptr_t)comm);
}

JNIEXPORT jint JNICALL FN(countsMerge)(JNIEnv* env, jobject self, jlong counts, jlong comm) {
    (void)env;
    (void)self;
    jclear();
    return ldgpu_counts_merge((ldgpu_counts*)(intptr_t)counts, (ldgpu_comm*)(intptr_t)comm);
}

/* The device preprocessors (ldgpu_casemap_create / ldgpu_preprocess).  The
 * case map is the JVM's own: lower = Character.toLowerCase of every unit
 * (65536 u16), special = the units whose String.toLowerCase is not 1:1
 * (8192 bytes, one bit each) -- built once by the caller, so the device
 * lower-cases exactly as the executor's JVM does. */
JNIEXPORT jint JNICALL FN(casemapCreate)(JNIEnv* env, jobject self, jlong ctx, jobject lower, jobject special,
                                         jlongArray out) {
    (void)self;
    jclear();
    CHECK(need(env, lower, 2 * 65536, "lower"));
    CHECK(need(env, special, 65536 / 8, "special"));
    ldgpu_casemap* m = NULL;
    const int rc = ldgpu_casemap_create((ldgpu_ctx*)(intptr_t)ctx, (const uint16_t*)addr(env, lower),
                                        (const uint8_t*)addr(env, special), &m);
    return put_handle(env, out, m, rc);
}

JNIEXPORT jint JNICALL FN(casemapDestroy)(JNIEnv* env, jobject self, jlong map) {
    (void)env;
    (void)self;
    jclear();
    return ldgpu_casemap_destroy((ldgpu_casemap*)(intptr_t)map);
}

/* units: UTF-16 code units up to offsets[nDocs]; out: the worst case (every
 * unit kept) of offsets[nDocs] - offsets[0] units, or bytes with
 * LDGPU_PRE_LOW_BYTES; outOffsets nDocs + 1 longs; host and locale (nullable)
 * nDocs bytes. */
JNIEXPORT jint JNICALL FN(preprocess)(JNIEnv* env, jobject self, jlong map, jobject units, jobject offsets,
                                      jlong n_docs, jobject locale, jint flags, jobject out, jobject out_offsets,
                                      jobject host) {
    (void)self;
    jclear();
    int64_t nu = 0;
    CHECK(need_offsets(env, offsets, n_docs, "offsets", &nu));
    CHECK(need(env, units, bytes_of(2, nu, 1), "units"));
    const int64_t first = ((const int64_t*)addr(env, offsets))[0];
    CHECK(need(env, out, bytes_of((flags & LDGPU_PRE_LOW_BYTES) ? 1 : 2, nu - first, 1), "out"));
    CHECK(need(env, out_offsets, bytes_of(8, n_docs + 1, 1), "outOffsets"));
    CHECK(need(env, host, n_docs, "host"));
    if (locale) CHECK(need(env, locale, n_docs, "locale"));
    return ldgpu_preprocess((ldgpu_casemap*)(intptr_t)map, (const uint16_t*)addr(env, units),
                            (const int64_t*)addr(env, offsets), n_docs, (const uint8_t*)addr(env, locale), flags,
                            addr(env, out), (int64_t*)addr(env, out_offsets), (uint8_t*)addr(env, host));
}
