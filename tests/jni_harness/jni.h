/* jni.h -- TEST-ONLY stand-in for the JDK's jni.h (there is no JDK in this
 * image): just the types and the JNIEnv functions jni/ldgpu_jni.c calls, so
 * tests/test_jni_shim.py can drive the shim's buffer checks through ctypes
 * with fake direct buffers (harness.c).  Never used to build the shim that
 * ships (jni/Makefile takes the JDK's header). */
#ifndef LDGPU_TEST_FAKE_JNI_H
#define LDGPU_TEST_FAKE_JNI_H
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef int32_t jsize;
typedef void* jobject;
typedef jobject jstring;
typedef jobject jarray;
typedef jobject jlongArray;
typedef jobject jintArray;
typedef jobject jbyteArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
    jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
    jstring (*NewStringUTF)(JNIEnv*, const char*);
    void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
    jsize (*GetArrayLength)(JNIEnv*, jarray);
    jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
    void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
    jobject (*NewDirectByteBuffer)(JNIEnv*, void*, jlong);
    jbyteArray (*NewByteArray)(JNIEnv*, jsize);
    void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
    void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
};

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
#endif
