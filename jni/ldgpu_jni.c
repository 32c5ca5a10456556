/* ldgpu_jni.c -- JNI shim between the Scala drop-in
 * (scala/.../LdgpuNative.scala, object LdgpuNative: its @native methods are
 * instance methods of the module class LdgpuNative$, hence the _00024 in the
 * symbol names) and the C ABI of libldgpu.so (include/ldgpu.h).
 *
 * Every buffer is a direct java.nio.ByteBuffer in native byte order; the shim
 * passes its address straight through (no copies).  Handles are the C
 * pointers as jlong.  Status codes are returned unchanged; the Scala side
 * turns them into the reference's exceptions (LdgpuNative.check).
 *
 * Build (on a box with a JDK; not in this image):
 *   make -C jni JAVA_HOME=/usr/lib/jvm/java-8-openjdk-amd64
 */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "../include/ldgpu.h"

#define FN(name) Java_org_apache_spark_ml_feature_languagedetection_LdgpuNative_00024_##name

static void* addr(JNIEnv* env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }

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
    return (*env)->NewStringUTF(env, ldgpu_last_error());
}

JNIEXPORT jint JNICALL FN(ctxCreate)(JNIEnv* env, jobject self, jint device, jlongArray out) {
    (void)self;
    ldgpu_ctx* c = NULL;
    const int rc = ldgpu_ctx_create(device, &c);
    return put_handle(env, out, c, rc);
}

/* pinned host memory wrapped as a direct ByteBuffer (NULL on failure) */
JNIEXPORT jobject JNICALL FN(hostAlloc)(JNIEnv* env, jobject self, jlong ctx, jlong bytes) {
    (void)self;
    void* p = NULL;
    if (ldgpu_host_alloc((ldgpu_ctx*)(intptr_t)ctx, bytes, &p) != LDGPU_OK || !p) return NULL;
    return (*env)->NewDirectByteBuffer(env, p, bytes > 0 ? bytes : 1);
}

JNIEXPORT jint JNICALL FN(hostFree)(JNIEnv* env, jobject self, jlong ctx, jobject buf) {
    (void)self;
    return ldgpu_host_free((ldgpu_ctx*)(intptr_t)ctx, addr(env, buf));
}

JNIEXPORT jint JNICALL FN(modelCreate)(JNIEnv* env, jobject self, jlong ctx, jlong n_rows, jobject key_bytes,
                                       jobject key_offsets, jobject rows, jobject row_ok, jint n_langs,
                                       jintArray gram_lengths, jlongArray out) {
    (void)self;
    jsize ng = 0;
    int32_t* g = ints(env, gram_lengths, &ng);
    ldgpu_model* m = NULL;
    const int rc = ldgpu_model_create((ldgpu_ctx*)(intptr_t)ctx, n_rows, (const uint8_t*)addr(env, key_bytes),
                                      (const int64_t*)addr(env, key_offsets), (const double*)addr(env, rows),
                                      (const uint8_t*)addr(env, row_ok), n_langs, g, ng, &m);
    ints_release(env, gram_lengths, g);
    return put_handle(env, out, m, rc);
}

JNIEXPORT jint JNICALL FN(modelDestroy)(JNIEnv* env, jobject self, jlong model) {
    (void)env;
    (void)self;
    return ldgpu_model_destroy((ldgpu_model*)(intptr_t)model);
}

/* ldgpu_score: thread-safe; concurrent task threads run on their own streams */
JNIEXPORT jint JNICALL FN(score)(JNIEnv* env, jobject self, jlong model, jobject bytes, jobject offsets,
                                 jlong n_docs, jobject labels, jobject scores) {
    (void)self;
    return ldgpu_score((ldgpu_model*)(intptr_t)model, (const uint8_t*)addr(env, bytes),
                       (const int64_t*)addr(env, offsets), n_docs, (int32_t*)addr(env, labels),
                       (double*)addr(env, scores));
}

JNIEXPORT jint JNICALL FN(countsCreate)(JNIEnv* env, jobject self, jlong ctx, jint n_langs, jintArray gram_lengths,
                                        jlong capacity_hint, jlongArray out) {
    (void)self;
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
    return ldgpu_counts_destroy((ldgpu_counts*)(intptr_t)counts);
}

JNIEXPORT jint JNICALL FN(count)(JNIEnv* env, jobject self, jlong counts, jobject bytes, jobject offsets,
                                 jobject doc_lang, jlong n_docs) {
    (void)self;
    return ldgpu_count((ldgpu_counts*)(intptr_t)counts, (const uint8_t*)addr(env, bytes),
                       (const int64_t*)addr(env, offsets), (const int32_t*)addr(env, doc_lang), n_docs);
}

JNIEXPORT jint JNICALL FN(countsSize)(JNIEnv* env, jobject self, jlong counts, jlongArray out) {
    (void)self;
    int64_t v[2] = {0, 0};
    const int rc = ldgpu_counts_size((ldgpu_counts*)(intptr_t)counts, &v[0], &v[1]);
    if (rc == LDGPU_OK) {
        jlong j[2] = {(jlong)v[0], (jlong)v[1]};
        (*env)->SetLongArrayRegion(env, out, 0, 2, j);
    }
    return rc;
}

JNIEXPORT jint JNICALL FN(countsExport)(JNIEnv* env, jobject self, jlong counts, jobject key_bytes,
                                        jobject key_offsets, jobject counts_out) {
    (void)self;
    return ldgpu_counts_export((ldgpu_counts*)(intptr_t)counts, (uint8_t*)addr(env, key_bytes),
                               (int64_t*)addr(env, key_offsets), (int64_t*)addr(env, counts_out));
}

JNIEXPORT jint JNICALL FN(countsAdd)(JNIEnv* env, jobject self, jlong counts, jlong n, jobject key_bytes,
                                     jobject key_offsets, jobject rows) {
    (void)self;
    return ldgpu_counts_add((ldgpu_counts*)(intptr_t)counts, n, (const uint8_t*)addr(env, key_bytes),
                            (const int64_t*)addr(env, key_offsets), (const int64_t*)addr(env, rows));
}

JNIEXPORT jint JNICALL FN(fitTableSize)(JNIEnv* env, jobject self, jlong counts, jint profile_size, jlongArray out) {
    (void)self;
    int64_t v[2] = {0, 0};
    const int rc = ldgpu_fit_table_size((ldgpu_counts*)(intptr_t)counts, profile_size, &v[0], &v[1]);
    if (rc == LDGPU_OK) {
        jlong j[2] = {(jlong)v[0], (jlong)v[1]};
        (*env)->SetLongArrayRegion(env, out, 0, 2, j);
    }
    return rc;
}

JNIEXPORT jint JNICALL FN(fitTableExport)(JNIEnv* env, jobject self, jlong counts, jobject key_bytes,
                                          jobject key_offsets, jobject rows) {
    (void)self;
    return ldgpu_fit_table_export((ldgpu_counts*)(intptr_t)counts, (uint8_t*)addr(env, key_bytes),
                                  (int64_t*)addr(env, key_offsets), (double*)addr(env, rows));
}

/* ---- multi-GPU merge: one task per GPU (Spark barrier execution) */
JNIEXPORT jbyteArray JNICALL FN(commUniqueId)(JNIEnv* env, jobject self) {
    (void)self;
    uint8_t id[LDGPU_COMM_ID_BYTES];
    if (ldgpu_comm_unique_id(id) != LDGPU_OK) return NULL;
    jbyteArray a = (*env)->NewByteArray(env, LDGPU_COMM_ID_BYTES);
    if (a) (*env)->SetByteArrayRegion(env, a, 0, LDGPU_COMM_ID_BYTES, (const jbyte*)id);
    return a;
}

JNIEXPORT jint JNICALL FN(commCreateRccl)(JNIEnv* env, jobject self, jlong ctx, jbyteArray id, jint rank,
                                          jint world, jlongArray out) {
    (void)self;
    uint8_t buf[LDGPU_COMM_ID_BYTES];
    if (!id || (*env)->GetArrayLength(env, id) != LDGPU_COMM_ID_BYTES) return LDGPU_EINVAL;
    (*env)->GetByteArrayRegion(env, id, 0, LDGPU_COMM_ID_BYTES, (jbyte*)buf);
    ldgpu_comm* m = NULL;
    const int rc = ldgpu_comm_create_rccl((ldgpu_ctx*)(intptr_t)ctx, buf, rank, world, &m);
    return put_handle(env, out, m, rc);
}

JNIEXPORT jint JNICALL FN(commDestroy)(JNIEnv* env, jobject self, jlong comm) {
    (void)env;
    (void)self;
    return ldgpu_comm_destroy((ldgpu_comm*)(intptr_t)comm);
}

JNIEXPORT jint JNICALL FN(countsMerge)(JNIEnv* env, jobject self, jlong counts, jlong comm) {
    (void)env;
    (void)self;
    return ldgpu_counts_merge((ldgpu_counts*)(intptr_t)counts, (ldgpu_comm*)(intptr_t)comm);
}
