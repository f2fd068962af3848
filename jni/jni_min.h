/* jni_min.h -- the part of the JNI interface curvezmq_jni.c uses, restated so the shim compiles
 * and is tested in an image without a JDK (build the production shim against the JDK's <jni.h>).
 *
 * Types follow the JNI specification ("JNI Types and Data Structures").  The JNIEnv is a pointer
 * to a pointer to the function table JNINativeInterface_, whose layout is fixed by the
 * specification's "Interface Function Table": four reserved slots, then the functions in a
 * documented order.  Only the slots the shim calls are named; every gap is padding, and the
 * static asserts pin each named slot to its index in that table, so a call through this header
 * reaches the same entry a real JVM's table holds.
 */
#ifndef CZ_JNI_MIN_H
#define CZ_JNI_MIN_H

#include <stddef.h>
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jobjectArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

#define CZ_JNI_PAD(a, b) void *pad_##a##_##b[(b) - (a)]

struct JNINativeInterface_ {
    CZ_JNI_PAD(0, 6);                                                                         /* reserved0-3, GetVersion, DefineClass */
    jclass (*FindClass)(JNIEnv *env, const char *name);                                       /* 6 */
    CZ_JNI_PAD(7, 14);
    jint (*ThrowNew)(JNIEnv *env, jclass cls, const char *msg);                               /* 14 */
    CZ_JNI_PAD(15, 23);
    void (*DeleteLocalRef)(JNIEnv *env, jobject obj);                                         /* 23 */
    CZ_JNI_PAD(24, 171);
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);                                       /* 171 */
    jobjectArray (*NewObjectArray)(JNIEnv *env, jsize len, jclass cls, jobject init);        /* 172 */
    void *GetObjectArrayElement;                                                              /* 173 */
    void (*SetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index, jobject val); /* 174 */
    CZ_JNI_PAD(175, 200);
    void (*GetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, jbyte *buf);   /* 200 */
    CZ_JNI_PAD(201, 208);
    void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf); /* 208 */
    CZ_JNI_PAD(209, 211);
    void (*SetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, const jint *buf); /* 211 */
    CZ_JNI_PAD(212, 222);
    void *(*GetPrimitiveArrayCritical)(JNIEnv *env, jarray array, jboolean *isCopy);          /* 222 */
    void (*ReleasePrimitiveArrayCritical)(JNIEnv *env, jarray array, void *carray, jint mode); /* 223 */
    CZ_JNI_PAD(224, 228);
    jboolean (*ExceptionCheck)(JNIEnv *env);                                                  /* 228 */
    jobject (*NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);              /* 229 */
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);                                /* 230 */
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);                               /* 231 */
    void *GetObjectRefType;                                                                   /* 232 */
};

#define CZ_JNI_SLOT(f, i) _Static_assert(offsetof(struct JNINativeInterface_, f) == (i) * sizeof(void *), #f)
CZ_JNI_SLOT(FindClass, 6);
CZ_JNI_SLOT(ThrowNew, 14);
CZ_JNI_SLOT(DeleteLocalRef, 23);
CZ_JNI_SLOT(GetArrayLength, 171);
CZ_JNI_SLOT(NewObjectArray, 172);
CZ_JNI_SLOT(SetObjectArrayElement, 174);
CZ_JNI_SLOT(GetByteArrayRegion, 200);
CZ_JNI_SLOT(SetByteArrayRegion, 208);
CZ_JNI_SLOT(SetIntArrayRegion, 211);
CZ_JNI_SLOT(GetPrimitiveArrayCritical, 222);
CZ_JNI_SLOT(ReleasePrimitiveArrayCritical, 223);
CZ_JNI_SLOT(ExceptionCheck, 228);
CZ_JNI_SLOT(NewDirectByteBuffer, 229);
CZ_JNI_SLOT(GetDirectBufferAddress, 230);
CZ_JNI_SLOT(GetDirectBufferCapacity, 231);

#endif
