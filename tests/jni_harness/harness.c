/* harness.c -- TEST-ONLY: fake direct buffers and Java arrays behind the
 * stand-in jni.h, so tests/test_jni_shim.py can call the JNI shim's entry
 * points (jni/ldgpu_jni.c, compiled into the same .so) through ctypes:
 *   env = jh_env(); buf = jh_buf(ptr, capacity); arr = jh_longs(ptr, n) ...
 * A buffer's capacity can be given smaller than its memory, which is what the
 * shim's checks must catch before the C ABI reads or writes past it. */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

typedef struct { void* p; jlong cap; } fake_buf;        /* direct ByteBuffer */
typedef struct { void* p; jsize n; } fake_arr;          /* long[] / int[] / byte[] */

static void* get_addr(JNIEnv* e, jobject b) { (void)e; return b ? ((fake_buf*)b)->p : NULL; }
static jlong get_cap(JNIEnv* e, jobject b) { (void)e; return b ? ((fake_buf*)b)->cap : -1; }
static jstring new_str(JNIEnv* e, const char* s) { (void)e; return (jstring)s; }
static void set_longs(JNIEnv* e, jlongArray a, jsize at, jsize n, const jlong* v) {
    (void)e;
    memcpy((jlong*)((fake_arr*)a)->p + at, v, sizeof(jlong) * (size_t)n);
}
static jsize arr_len(JNIEnv* e, jarray a) { (void)e; return ((fake_arr*)a)->n; }
static jint* int_elems(JNIEnv* e, jintArray a, jboolean* c) { (void)e; if (c) *c = 0; return (jint*)((fake_arr*)a)->p; }
static void int_release(JNIEnv* e, jintArray a, jint* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jobject new_dbuf(JNIEnv* e, void* p, jlong cap) {
    (void)e;
    fake_buf* b = (fake_buf*)malloc(sizeof *b);
    b->p = p;
    b->cap = cap;
    return b;
}
static jbyteArray new_bytes(JNIEnv* e, jsize n) {
    (void)e;
    fake_arr* a = (fake_arr*)malloc(sizeof *a);
    a->p = calloc((size_t)n + 1, 1);
    a->n = n;
    return a;
}
static void set_bytes(JNIEnv* e, jbyteArray a, jsize at, jsize n, const jbyte* v) {
    (void)e;
    memcpy((jbyte*)((fake_arr*)a)->p + at, v, (size_t)n);
}
static void get_bytes(JNIEnv* e, jbyteArray a, jsize at, jsize n, jbyte* v) {
    (void)e;
    memcpy(v, (jbyte*)((fake_arr*)a)->p + at, (size_t)n);
}

static const struct JNINativeInterface_ table = {get_addr, get_cap,   new_str,  set_longs, arr_len,  int_elems,
                                                 int_release, new_dbuf, new_bytes, set_bytes, get_bytes};
static JNIEnv env = &table;

JNIEXPORT JNIEnv* jh_env(void) { return &env; }
JNIEXPORT jobject jh_buf(void* p, jlong cap) { return new_dbuf(&env, p, cap); }
JNIEXPORT jobject jh_arr(void* p, jsize n) {
    fake_arr* a = (fake_arr*)malloc(sizeof *a);
    a->p = p;
    a->n = n;
    return a;
}
JNIEXPORT void jh_free(void* o) { free(o); }
