/* fake_jni_env.c -- test double of a JVM's JNIEnv for tests/test_jni_shim.py (test infrastructure,
 * never shipped).  Builds the JNINativeInterface_ table of jni_min.h with the slots the shim calls
 * and fake Java objects behind jobject: byte[] / int[] arrays over host buffers the test owns,
 * direct ByteBuffers, ByteBuffer[] and a class handle.  Records every pin and release (and its
 * mode) so the test can check the shim's JNI discipline, and can emulate a VM that hands out COPIES
 * from GetPrimitiveArrayCritical (released with mode 0 = copy back, JNI_ABORT = discard), so a
 * wrong release mode shows up as wrong bytes in the Java array. */
#include <stdlib.h>
#include <string.h>

#include "curvezmq_mi355x.h"
#include "jni_min.h"

enum { K_BYTES = 1, K_INTS, K_DIRECT, K_CLASS, K_OBJARRAY };

struct _jobject {
    int kind;
    jsize len;      /* array elements */
    void *data;     /* array storage (owned by the test) or direct buffer address (NULL: not direct) */
    jlong cap;      /* direct buffer capacity */
    int pins, releases, last_mode;
    int gets, sets; /* Get/SetByteArrayRegion calls */
    void *copy;     /* the live copy handed out in copy mode */
    jobject *elems; /* K_OBJARRAY */
};

static int g_copy_mode, g_fail_pin_at = -1, g_pin_count, g_outstanding, g_calls_in_critical;
/* local references the shim created (NewDirectByteBuffer, NewObjectArray, FindClass results handed
 * out) and not deleted, their high-water mark, and an injected allocation failure: the n-th
 * NewDirectByteBuffer returns NULL with an OutOfMemoryError pending, as a JVM does */
static int g_live_refs, g_max_live_refs, g_fail_new_at = -1, g_new_count, g_exception;
static int g_modes[64], g_nmodes;
/* library calls the shim made (through the --wrap'ed cz_* entry points below) and how many of them
 * ran while a Java array was pinned: the GC would have been locked out across a GPU launch */
static int g_lib_calls, g_lib_calls_pinned;

static size_t elem_size(jobject o) { return o->kind == K_INTS ? 4 : 1; }

static jclass f_FindClass(JNIEnv *env, const char *name)
{
    (void)env;
    static struct _jobject cls = {.kind = K_CLASS};
    if (g_outstanding)
        g_calls_in_critical++;
    if (strcmp(name, "java/nio/ByteBuffer") != 0) {
        g_exception = 1; /* NoClassDefFoundError */
        return NULL;
    }
    if (++g_live_refs > g_max_live_refs)
        g_max_live_refs = g_live_refs;
    return &cls;
}

static void f_DeleteLocalRef(JNIEnv *env, jobject o)
{
    (void)env;
    if (o)
        g_live_refs--;
}

static jboolean f_ExceptionCheck(JNIEnv *env)
{
    (void)env;
    if (g_outstanding)
        g_calls_in_critical++;
    return (jboolean)(g_exception != 0);
}

static jsize f_GetArrayLength(JNIEnv *env, jarray a)
{
    (void)env;
    if (g_outstanding)
        g_calls_in_critical++;
    return a->len;
}

static jobjectArray f_NewObjectArray(JNIEnv *env, jsize len, jclass cls, jobject init)
{
    (void)env, (void)cls, (void)init;
    jobject o = (jobject)calloc(1, sizeof *o);
    if (++g_live_refs > g_max_live_refs)
        g_max_live_refs = g_live_refs;
    o->kind = K_OBJARRAY;
    o->len = len;
    o->elems = (jobject *)calloc(len ? (size_t)len : 1, sizeof(jobject));
    return o;
}

static void f_SetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i, jobject v)
{
    (void)env;
    if (i >= 0 && i < a->len)
        a->elems[i] = v;
}

static void f_SetIntArrayRegion(JNIEnv *env, jintArray a, jsize start, jsize len, const jint *buf)
{
    (void)env;
    if (start >= 0 && start + len <= a->len)
        memcpy((jint *)a->data + start, buf, (size_t)len * 4);
}

static void f_GetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize start, jsize len, jbyte *buf)
{
    (void)env;
    if (g_outstanding)
        g_calls_in_critical++;
    a->gets++;
    if (start < 0 || len < 0 || start + len > a->len) {
        g_exception = 1; /* ArrayIndexOutOfBoundsException */
        return;
    }
    memcpy(buf, (jbyte *)a->data + start, (size_t)len);
}

static void f_SetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize start, jsize len, const jbyte *buf)
{
    (void)env;
    if (g_outstanding)
        g_calls_in_critical++;
    a->sets++;
    if (start < 0 || len < 0 || start + len > a->len) {
        g_exception = 1;
        return;
    }
    memcpy((jbyte *)a->data + start, buf, (size_t)len);
}

static void *f_GetPrimitiveArrayCritical(JNIEnv *env, jarray a, jboolean *isCopy)
{
    (void)env;
    if (g_pin_count++ == g_fail_pin_at)
        return NULL;
    a->pins++;
    g_outstanding++;
    if (isCopy)
        *isCopy = (jboolean)g_copy_mode;
    if (!g_copy_mode)
        return a->data;
    const size_t n = (size_t)a->len * elem_size(a);
    a->copy = malloc(n ? n : 1);
    memcpy(a->copy, a->data, n);
    return a->copy;
}

static void f_ReleasePrimitiveArrayCritical(JNIEnv *env, jarray a, void *p, jint mode)
{
    (void)env;
    a->releases++;
    a->last_mode = mode;
    g_outstanding--;
    if (g_nmodes < 64)
        g_modes[g_nmodes++] = mode;
    if (g_copy_mode && p == a->copy) {
        if (mode != JNI_ABORT)
            memcpy(a->data, p, (size_t)a->len * elem_size(a));
        if (mode != JNI_COMMIT) {
            free(a->copy);
            a->copy = NULL;
        }
    }
}

static jobject f_NewDirectByteBuffer(JNIEnv *env, void *p, jlong cap)
{
    (void)env;
    if (g_new_count++ == g_fail_new_at) {
        g_exception = 1;
        return NULL;
    }
    if (++g_live_refs > g_max_live_refs)
        g_max_live_refs = g_live_refs;
    jobject o = (jobject)calloc(1, sizeof *o);
    o->kind = K_DIRECT;
    o->data = p;
    o->cap = cap;
    return o;
}

static void *f_GetDirectBufferAddress(JNIEnv *env, jobject b)
{
    (void)env;
    return b && b->kind == K_DIRECT ? b->data : NULL;
}

static jlong f_GetDirectBufferCapacity(JNIEnv *env, jobject b)
{
    (void)env;
    return b && b->kind == K_DIRECT && b->data ? b->cap : -1;
}

static struct JNINativeInterface_ g_table;
static const struct JNINativeInterface_ *g_env = &g_table;

JNIEnv *fake_env(void)
{
    g_table.FindClass = f_FindClass;
    g_table.DeleteLocalRef = f_DeleteLocalRef;
    g_table.ExceptionCheck = f_ExceptionCheck;
    g_table.GetArrayLength = f_GetArrayLength;
    g_table.NewObjectArray = f_NewObjectArray;
    g_table.SetObjectArrayElement = f_SetObjectArrayElement;
    g_table.SetIntArrayRegion = f_SetIntArrayRegion;
    g_table.GetByteArrayRegion = f_GetByteArrayRegion;
    g_table.SetByteArrayRegion = f_SetByteArrayRegion;
    g_table.GetPrimitiveArrayCritical = f_GetPrimitiveArrayCritical;
    g_table.ReleasePrimitiveArrayCritical = f_ReleasePrimitiveArrayCritical;
    g_table.NewDirectByteBuffer = f_NewDirectByteBuffer;
    g_table.GetDirectBufferAddress = f_GetDirectBufferAddress;
    g_table.GetDirectBufferCapacity = f_GetDirectBufferCapacity;
    return (JNIEnv *)&g_env;
}

static jobject new_obj(int kind, void *data, jsize len, jlong cap)
{
    jobject o = (jobject)calloc(1, sizeof *o);
    o->kind = kind;
    o->data = data;
    o->len = len;
    o->cap = cap;
    return o;
}

jobject fake_byte_array(void *data, jsize len) { return new_obj(K_BYTES, data, len, 0); }
jobject fake_int_array(void *data, jsize len) { return new_obj(K_INTS, data, len, 0); }
jobject fake_direct(void *p, jlong cap) { return new_obj(K_DIRECT, p, 0, cap); }
jobject fake_heap_buffer(void) { return new_obj(K_DIRECT, NULL, 0, 0); } /* a non-direct ByteBuffer */

void fake_set_copy_mode(int on) { g_copy_mode = on; }
void fake_fail_pin_at(int n) { g_fail_pin_at = n, g_pin_count = 0; }
void fake_reset_log(void) { g_nmodes = 0, g_calls_in_critical = 0, g_pin_count = 0, g_fail_pin_at = -1; }
void fake_reset_refs(void) { g_live_refs = g_max_live_refs = 0, g_new_count = 0, g_fail_new_at = -1, g_exception = 0; }
void fake_fail_new_at(int n) { g_fail_new_at = n, g_new_count = 0; }
int fake_live_refs(void) { return g_live_refs; }
int fake_max_live_refs(void) { return g_max_live_refs; }
int fake_exception(void) { return g_exception; }
int fake_outstanding(void) { return g_outstanding; }
int fake_calls_in_critical(void) { return g_calls_in_critical; }
int fake_nmodes(void) { return g_nmodes; }
int fake_mode(int i) { return i >= 0 && i < g_nmodes ? g_modes[i] : -1; }
int fake_pins(jobject o) { return o->pins; }
int fake_gets(jobject o) { return o->gets; }
int fake_sets(jobject o) { return o->sets; }
int fake_lib_calls(void) { return g_lib_calls; }
int fake_lib_calls_pinned(void) { return g_lib_calls_pinned; }
void fake_reset_lib_calls(void) { g_lib_calls = g_lib_calls_pinned = 0; }
void fake_raise(void) { g_exception = 1; }
/* hold an array pinned from the test (as another native of the thread might), and let it go */
void fake_pin(jobject o) { o->pins++, g_outstanding++; }
void fake_unpin(jobject o) { o->releases++, g_outstanding--; }
int fake_releases(jobject o) { return o->releases; }
int fake_last_mode(jobject o) { return o->last_mode; }
int fake_kind(jobject o) { return o ? o->kind : 0; }
jsize fake_len(jobject o) { return o->len; }
jobject fake_elem(jobject o, jsize i) { return o->elems[i]; }
void *fake_addr(jobject o) { return o->data; }
jlong fake_cap(jobject o) { return o->cap; }

/* The library entry points the byte[] natives call, interposed with -Wl,--wrap=<name> in the test
 * build: each call is counted, and counted again if any Java array is pinned at that moment. */
#define CZ_WRAP_NOTE() (g_lib_calls++, g_lib_calls_pinned += g_outstanding != 0)
int __real_cz_box_afternm(uint8_t *, const uint8_t *, uint64_t, const uint8_t *, const uint8_t *);
int __real_cz_box_open_afternm(uint8_t *, const uint8_t *, uint64_t, const uint8_t *, const uint8_t *);
int __real_cz_secretbox(uint8_t *, const uint8_t *, uint64_t, const uint8_t *, const uint8_t *);
int __real_cz_secretbox_open(uint8_t *, const uint8_t *, uint64_t, const uint8_t *, const uint8_t *);
int __real_cz_box_beforenm(uint8_t *, const uint8_t *, const uint8_t *);
int __real_cz_box(uint8_t *, const uint8_t *, uint64_t, const uint8_t *, const uint8_t *, const uint8_t *);
int __real_cz_box_open(uint8_t *, const uint8_t *, uint64_t, const uint8_t *, const uint8_t *, const uint8_t *);
int __real_cz_box_keypair(uint8_t *, uint8_t *);
int __real_cz_engine_add_conn(cz_engine *, int, const uint8_t *, uint64_t, uint64_t);
int __wrap_cz_box_afternm(uint8_t *c, const uint8_t *m, uint64_t l, const uint8_t *n, const uint8_t *k)
{
    CZ_WRAP_NOTE();
    return __real_cz_box_afternm(c, m, l, n, k);
}
int __wrap_cz_box_open_afternm(uint8_t *m, const uint8_t *c, uint64_t l, const uint8_t *n, const uint8_t *k)
{
    CZ_WRAP_NOTE();
    return __real_cz_box_open_afternm(m, c, l, n, k);
}
int __wrap_cz_secretbox(uint8_t *c, const uint8_t *m, uint64_t l, const uint8_t *n, const uint8_t *k)
{
    CZ_WRAP_NOTE();
    return __real_cz_secretbox(c, m, l, n, k);
}
int __wrap_cz_secretbox_open(uint8_t *m, const uint8_t *c, uint64_t l, const uint8_t *n, const uint8_t *k)
{
    CZ_WRAP_NOTE();
    return __real_cz_secretbox_open(m, c, l, n, k);
}
int __wrap_cz_box_beforenm(uint8_t *k, const uint8_t *pk, const uint8_t *sk)
{
    CZ_WRAP_NOTE();
    return __real_cz_box_beforenm(k, pk, sk);
}
int __wrap_cz_box(uint8_t *c, const uint8_t *m, uint64_t l, const uint8_t *n, const uint8_t *pk, const uint8_t *sk)
{
    CZ_WRAP_NOTE();
    return __real_cz_box(c, m, l, n, pk, sk);
}
int __wrap_cz_box_open(uint8_t *m, const uint8_t *c, uint64_t l, const uint8_t *n, const uint8_t *pk, const uint8_t *sk)
{
    CZ_WRAP_NOTE();
    return __real_cz_box_open(m, c, l, n, pk, sk);
}
int __wrap_cz_box_keypair(uint8_t *pk, uint8_t *sk)
{
    CZ_WRAP_NOTE();
    return __real_cz_box_keypair(pk, sk);
}
int __wrap_cz_engine_add_conn(cz_engine *e, int server, const uint8_t *precom, uint64_t a, uint64_t b)
{
    CZ_WRAP_NOTE();
    return __real_cz_engine_add_conn(e, server, precom, a, b);
}
