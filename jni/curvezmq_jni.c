/* curvezmq_jni.c -- JNI binding of the MI355X CURVE path for JeroMQ (INTEGRATION.md sections 2-3).
 *
 * Three Java classes bind here:
 *  - com.neilalexander.jnacl.crypto.curve25519xsalsa20poly1305 and ...xsalsa20poly1305: drop-in
 *    replacements of the jnacl classes zmq/io/mechanism/curve/Curve.java:5-6 imports.  Curve.java
 *    (:84-193) calls them unchanged: crypto_box_afternm / crypto_box_open_afternm on every
 *    MESSAGE (Curve.java:134-147), the rest during the handshake.  One message per call.
 *  - zmq.io.mechanism.curve.GpuCurveBatch: the batched, host-staged seal / open of many frames
 *    (cz_ctx_*), the throughput path a batching Mechanism drives (Mechanism.java:202-210).
 *  - zmq.io.GpuCurveEngine: the multi-connection batching engine (cz_engine_*), replacing
 *    StreamEngine's encode + V2Encoder / V2Decoder + decode loops (StreamEngine.java:379-535).
 *
 * Contracts:
 *  - jnacl calls return jnacl's 0 / -1.  Every array is checked against the lengths the call
 *    reads or writes before anything else happens (a short array is -1, never an overrun).  No
 *    Java array is pinned while the library runs: inputs are copied into native staging
 *    (GetByteArrayRegion), outputs copied back on success (SetByteArrayRegion), the staging wiped.
 *  - Batch and engine calls take direct ByteBuffers (pinned memory from hostAlloc / msgAlloc for
 *    full PCIe rate) and return the library's CZ_* codes; a buffer smaller than the call needs, or
 *    a non-direct buffer, is CZ_EINVAL before the library is entered.
 *
 * Build (production, with a JDK):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       jni/curvezmq_jni.c -Ljeromq_amd -lcurvezmq_mi355x -o libcurvezmq_jni.so
 * Without a JDK (this image; the CPU tests): add -DCZ_JNI_MIN to compile against jni/jni_min.h.
 */
#define _DEFAULT_SOURCE /* explicit_bzero */
#ifdef CZ_JNI_MIN
#include "jni_min.h"
#else
#include <jni.h>
#endif
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "curvezmq_mi355x.h"

/* ---- Java byte[] arguments: staged, never pinned across a library call ------------------------
 * A library call is a GPU launch and a stream sync (~20 us).  Holding a Java array with
 * GetPrimitiveArrayCritical across it would lock the GC out of every thread for that long, per
 * CURVE message.  So the byte[] natives copy their inputs into this thread's native staging with
 * GetByteArrayRegion, run the library on the staging, and on success copy the outputs back with
 * SetByteArrayRegion (a failed call -- a bad tag -- leaves the output array untouched).  The copies
 * are the ones the library makes into its pinned staging anyway, one level up.  The staging holds
 * plaintext and keys, so it is wiped after every call. */

typedef struct {
    jbyteArray a;
    jlong need; /* bytes the call touches */
    int out;    /* written by the call: copied back on success; inputs are only read */
    uint8_t *p; /* the argument's place in the staging */
} jarr_arg;

static _Thread_local uint8_t *t_stage;
static _Thread_local size_t t_stage_cap;
/* staging kept between calls up to this size; a larger one (a big box) is freed after its call */
#define STAGE_KEEP ((size_t)1 << 20)

static size_t stage_round(jlong need) { return ((size_t)need + 15u) & ~(size_t)15u; }

/* Check every array's length first (-1 with nothing read on a null or short array), then give every
 * argument its staging and copy the inputs in.  -1 if the staging cannot grow or the VM raised. */
static int stage_in(JNIEnv *env, jarr_arg *v, int n, size_t *used)
{
    size_t total = 0;
    *used = 0;
    for (int i = 0; i < n; i++) {
        v[i].p = NULL;
        if (!v[i].a || v[i].need < 0 || (jlong)(*env)->GetArrayLength(env, v[i].a) < v[i].need)
            return -1;
        total += stage_round(v[i].need);
    }
    if (total > t_stage_cap) {
        uint8_t *p = (uint8_t *)malloc(total);
        if (!p)
            return -1;
        if (t_stage) {
            explicit_bzero(t_stage, t_stage_cap);
            free(t_stage);
        }
        t_stage = p;
        t_stage_cap = total;
    }
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        v[i].p = t_stage + off;
        if (!v[i].out && v[i].need)
            (*env)->GetByteArrayRegion(env, v[i].a, 0, (jsize)v[i].need, (jbyte *)v[i].p);
        off += stage_round(v[i].need);
    }
    *used = off;
    if ((*env)->ExceptionCheck(env)) {
        explicit_bzero(t_stage, off);
        return -1;
    }
    return 0;
}

/* rc == 0: copy the outputs back; always: wipe the staging.  Returns rc. */
static int stage_out(JNIEnv *env, jarr_arg *v, int n, size_t used, int rc)
{
    if (rc == 0)
        for (int i = 0; i < n; i++)
            if (v[i].out && v[i].need)
                (*env)->SetByteArrayRegion(env, v[i].a, 0, (jsize)v[i].need, (const jbyte *)v[i].p);
    if (used)
        explicit_bzero(t_stage, used);
    if (t_stage_cap > STAGE_KEEP) {
        free(t_stage);
        t_stage = NULL;
        t_stage_cap = 0;
    }
    return rc;
}

#define U8(i) (v[i].p)

/* ---- com.neilalexander.jnacl.crypto.curve25519xsalsa20poly1305 ------------------------------- */

/* Curve.java:129-137 -> crypto_box_afternm(c, m, mlen, n, k): c = NaCl's box of m (any m[0:32]) */
JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_crypto_1box_1afternm(
    JNIEnv *env, jclass cls, jbyteArray c, jbyteArray m, jint mlen, jbyteArray n, jbyteArray k)
{
    (void)cls;
    if (mlen < 32)
        return -1;
    jarr_arg v[4] = {{c, mlen, 1, NULL}, {m, mlen, 0, NULL}, {n, 24, 0, NULL}, {k, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 4, &used))
        return -1;
    return stage_out(env, v, 4, used, cz_box_afternm(U8(0), U8(1), (uint64_t)mlen, U8(2), U8(3)));
}

/* Curve.java:139-147 -> crypto_box_open_afternm(m, c, clen, n, k): -1 on a bad tag */
JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_crypto_1box_1open_1afternm(
    JNIEnv *env, jclass cls, jbyteArray m, jbyteArray c, jint clen, jbyteArray n, jbyteArray k)
{
    (void)cls;
    if (clen < 32)
        return -1;
    jarr_arg v[4] = {{m, clen, 1, NULL}, {c, clen, 0, NULL}, {n, 24, 0, NULL}, {k, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 4, &used))
        return -1;
    return stage_out(env, v, 4, used, cz_box_open_afternm(U8(0), U8(1), (uint64_t)clen, U8(2), U8(3)));
}

/* Curve.java:124-127 */
JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_crypto_1box_1beforenm(
    JNIEnv *env, jclass cls, jbyteArray k, jbyteArray pk, jbyteArray sk)
{
    (void)cls;
    jarr_arg v[3] = {{k, 32, 1, NULL}, {pk, 32, 0, NULL}, {sk, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 3, &used))
        return -1;
    return stage_out(env, v, 3, used, cz_box_beforenm(U8(0), U8(1), U8(2)));
}

/* Curve.java:183-193 */
JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_crypto_1box(
    JNIEnv *env, jclass cls, jbyteArray c, jbyteArray m, jint mlen, jbyteArray n, jbyteArray pk, jbyteArray sk)
{
    (void)cls;
    if (mlen < 32)
        return -1;
    jarr_arg v[5] = {{c, mlen, 1, NULL}, {m, mlen, 0, NULL}, {n, 24, 0, NULL}, {pk, 32, 0, NULL}, {sk, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 5, &used))
        return -1;
    return stage_out(env, v, 5, used, cz_box(U8(0), U8(1), (uint64_t)mlen, U8(2), U8(3), U8(4)));
}

/* Curve.java:149-157 */
JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_crypto_1box_1open(
    JNIEnv *env, jclass cls, jbyteArray m, jbyteArray c, jint clen, jbyteArray n, jbyteArray pk, jbyteArray sk)
{
    (void)cls;
    if (clen < 32)
        return -1;
    jarr_arg v[5] = {{m, clen, 1, NULL}, {c, clen, 0, NULL}, {n, 24, 0, NULL}, {pk, 32, 0, NULL}, {sk, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 5, &used))
        return -1;
    return stage_out(env, v, 5, used, cz_box_open(U8(0), U8(1), (uint64_t)clen, U8(2), U8(3), U8(4)));
}

/* Curve.java:84-115 */
JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_crypto_1box_1keypair(
    JNIEnv *env, jclass cls, jbyteArray pk, jbyteArray sk)
{
    (void)cls;
    jarr_arg v[2] = {{pk, 32, 1, NULL}, {sk, 32, 1, NULL}};
    size_t used;
    if (stage_in(env, v, 2, &used))
        return -1;
    return stage_out(env, v, 2, used, cz_box_keypair(U8(0), U8(1)));
}

/* ---- com.neilalexander.jnacl.crypto.xsalsa20poly1305 (Curve.java:159-181: cookie boxes) ------ */

JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_xsalsa20poly1305_crypto_1secretbox(
    JNIEnv *env, jclass cls, jbyteArray c, jbyteArray m, jint mlen, jbyteArray n, jbyteArray k)
{
    (void)cls;
    if (mlen < 32)
        return -1;
    jarr_arg v[4] = {{c, mlen, 1, NULL}, {m, mlen, 0, NULL}, {n, 24, 0, NULL}, {k, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 4, &used))
        return -1;
    return stage_out(env, v, 4, used, cz_secretbox(U8(0), U8(1), (uint64_t)mlen, U8(2), U8(3)));
}

JNIEXPORT jint JNICALL Java_com_neilalexander_jnacl_crypto_xsalsa20poly1305_crypto_1secretbox_1open(
    JNIEnv *env, jclass cls, jbyteArray m, jbyteArray c, jint clen, jbyteArray n, jbyteArray k)
{
    (void)cls;
    if (clen < 32)
        return -1;
    jarr_arg v[4] = {{m, clen, 1, NULL}, {c, clen, 0, NULL}, {n, 24, 0, NULL}, {k, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 4, &used))
        return -1;
    return stage_out(env, v, 4, used, cz_secretbox_open(U8(0), U8(1), (uint64_t)clen, U8(2), U8(3)));
}

/* ---- direct ByteBuffers ----------------------------------------------------------------------- */

/* bytes a uniform batch touches: (count - 1) * stride + last; -1 (never a valid need) on overflow */
static jlong uniform_need(jint count, jlong stride, jlong last)
{
    jlong v;
    if (count <= 0)
        return 0;
    if (__builtin_mul_overflow((jlong)(count - 1), stride, &v) || __builtin_add_overflow(v, last, &v))
        return -1;
    return v;
}

/* address of a direct buffer holding at least `need` bytes; NULL if null, not direct, or short */
static void *direct(JNIEnv *env, jobject buf, jlong need)
{
    if (!buf || need < 0)
        return NULL;
    void *p = (*env)->GetDirectBufferAddress(env, buf);
    if (!p || (*env)->GetDirectBufferCapacity(env, buf) < need)
        return NULL;
    return p;
}

static jobject wrap(JNIEnv *env, const void *p, uint64_t len)
{
    /* a zero-length view still needs a non-null address for NewDirectByteBuffer */
    static uint8_t empty;
    return (*env)->NewDirectByteBuffer(env, p ? (void *)p : (void *)&empty, (jlong)len);
}

#define CTX(h) ((cz_ctx *)(intptr_t)(h))
#define ENG(h) ((cz_engine *)(intptr_t)(h))

/* ---- zmq.io.mechanism.curve.GpuCurveBatch (cz_ctx_*) ---------------- */

JNIEXPORT jlong JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_create(JNIEnv *env, jclass cls, jint device)
{
    (void)env, (void)cls;
    cz_ctx *c = NULL;
    return cz_ctx_create(&c, device) == CZ_OK ? (jlong)(intptr_t)c : 0;
}

JNIEXPORT void JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_destroy(JNIEnv *env, jclass cls, jlong ctx)
{
    (void)env, (void)cls;
    if (ctx)
        cz_ctx_destroy(CTX(ctx));
}

JNIEXPORT jint JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_setKeys(JNIEnv *env, jclass cls, jlong ctx,
                                                                          jobject precoms, jint nkeys, jint direction)
{
    (void)cls;
    const void *k = direct(env, precoms, 32 * (jlong)nkeys);
    if (!ctx || nkeys < 1 || !k)
        return CZ_EINVAL;
    return cz_ctx_set_keys(CTX(ctx), (const uint8_t *)k, (uint32_t)nkeys, direction);
}

/* descs: count x 40-byte cz_frame_desc (little-endian); the library bounds every descriptor by the
 * in / out capacities */
JNIEXPORT jint JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_seal(JNIEnv *env, jclass cls, jlong ctx, jobject descs,
                                                                       jint count, jobject in, jobject out)
{
    (void)cls;
    const void *d = direct(env, descs, (jlong)sizeof(cz_frame_desc) * count);
    void *pi = direct(env, in, 0), *po = direct(env, out, 0);
    if (!ctx || count < 0 || !d || !pi || !po)
        return CZ_EINVAL;
    return cz_ctx_seal(CTX(ctx), (const cz_frame_desc *)d, (uint32_t)count, pi,
                       (uint64_t)(*env)->GetDirectBufferCapacity(env, in), po,
                       (uint64_t)(*env)->GetDirectBufferCapacity(env, out));
}

JNIEXPORT jint JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_open(JNIEnv *env, jclass cls, jlong ctx, jobject descs,
                                                                       jint count, jobject in, jobject out,
                                                                       jobject status)
{
    (void)cls;
    const void *d = direct(env, descs, (jlong)sizeof(cz_frame_desc) * count);
    void *pi = direct(env, in, 0), *po = direct(env, out, 0), *ps = direct(env, status, 2 * (jlong)count);
    if (!ctx || count < 0 || !d || !pi || !po || !ps)
        return CZ_EINVAL;
    return cz_ctx_open(CTX(ctx), (const cz_frame_desc *)d, (uint32_t)count, pi,
                       (uint64_t)(*env)->GetDirectBufferCapacity(env, in), po,
                       (uint64_t)(*env)->GetDirectBufferCapacity(env, out), (uint16_t *)ps);
}

/* uniform batch: frame i at in + i*inStride, body i at out + i*outStride (whole slots) */
JNIEXPORT jint JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_sealUniform(
    JNIEnv *env, jclass cls, jlong ctx, jint count, jint len, jobject in, jlong inStride, jobject out, jlong outStride,
    jlong counter0, jobject flags, jint chunk)
{
    (void)cls;
    if (!ctx || count < 0 || len < 0 || inStride < 0 || outStride < 0 || chunk < 0)
        return CZ_EINVAL;
    if (count == 0)
        return CZ_OK;
    const jlong olen = (jlong)len + CZ_MESSAGE_OVERHEAD;
    /* whole output slots: count * outStride (one frame: the body) */
    const jlong in_need = count > 1 ? uniform_need(count, inStride, len) : len;
    const jlong out_need = count > 1 ? uniform_need(count, outStride, outStride) : olen;
    if (in_need < 0 || out_need < 0)
        return CZ_EINVAL;
    void *pi = direct(env, in, in_need), *po = direct(env, out, out_need);
    const void *pf = flags ? direct(env, flags, count) : NULL;
    if (!pi || !po || (flags && !pf))
        return CZ_EINVAL;
    return cz_ctx_seal_uniform(CTX(ctx), (uint32_t)count, (uint32_t)len, pi, (uint64_t)inStride, po,
                               (uint64_t)outStride, (uint64_t)counter0, (const uint8_t *)pf, (uint32_t)chunk);
}

JNIEXPORT jint JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_openUniform(
    JNIEnv *env, jclass cls, jlong ctx, jint count, jint size, jobject in, jlong inStride, jobject out, jlong outStride,
    jlong floor0, jboolean check, jobject status, jint chunk)
{
    (void)cls;
    if (!ctx || count < 0 || size < CZ_MESSAGE_OVERHEAD || inStride < 0 || outStride < 0 || chunk < 0)
        return CZ_EINVAL;
    if (count == 0)
        return CZ_OK;
    const jlong olen = (jlong)size - CZ_MESSAGE_OVERHEAD;
    const jlong in_need = count > 1 ? uniform_need(count, inStride, size) : size;
    const jlong out_need = count > 1 ? uniform_need(count, outStride, outStride) : olen;
    if (in_need < 0 || out_need < 0)
        return CZ_EINVAL;
    void *pi = direct(env, in, in_need), *po = direct(env, out, out_need), *ps = direct(env, status, 2 * (jlong)count);
    if (!pi || !po || !ps)
        return CZ_EINVAL;
    return cz_ctx_open_uniform(CTX(ctx), (uint32_t)count, (uint32_t)size, pi, (uint64_t)inStride, po,
                               (uint64_t)outStride, (uint64_t)floor0, check ? 1 : 0, (uint16_t *)ps, (uint32_t)chunk);
}

/* pinned host memory as a direct ByteBuffer (the pinned MsgAllocator, zmq/msg/MsgAllocator.java:5-8);
 * hostFree releases it: the library frees only base addresses hostAlloc returned (a slice, a
 * msgAlloc view, ByteBuffer.allocateDirect memory or a second free is refused), and the buffer
 * must not be used afterwards */
JNIEXPORT jobject JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_hostAlloc(JNIEnv *env, jclass cls, jlong bytes)
{
    (void)cls;
    if (bytes <= 0)
        return NULL;
    void *p = cz_host_alloc((uint64_t)bytes);
    return p ? (*env)->NewDirectByteBuffer(env, p, bytes) : NULL;
}

JNIEXPORT void JNICALL Java_zmq_io_mechanism_curve_GpuCurveBatch_hostFree(JNIEnv *env, jclass cls, jobject buf)
{
    (void)cls;
    void *p = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    if (p)
        cz_host_free(p);
}

/* ---- zmq.io.GpuCurveEngine (cz_engine_*, INTEGRATION.md "Batching engine") --------------------- */

JNIEXPORT jlong JNICALL Java_zmq_io_GpuCurveEngine_create(JNIEnv *env, jclass cls, jlong arenaBytes, jint device)
{
    (void)env, (void)cls;
    cz_engine *e = NULL;
    if (arenaBytes < 0)
        return 0;
    return cz_engine_create(&e, (uint64_t)arenaBytes, device) == CZ_OK ? (jlong)(intptr_t)e : 0;
}

JNIEXPORT void JNICALL Java_zmq_io_GpuCurveEngine_destroy(JNIEnv *env, jclass cls, jlong e)
{
    (void)env, (void)cls;
    if (e)
        cz_engine_destroy(ENG(e));
}

JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_addConn(JNIEnv *env, jclass cls, jlong e, jboolean server,
                                                           jbyteArray precom, jlong cnNonce, jlong cnPeerNonce)
{
    (void)cls;
    if (!e)
        return CZ_EINVAL;
    jarr_arg v[1] = {{precom, 32, 0, NULL}};
    size_t used;
    if (stage_in(env, v, 1, &used))
        return CZ_EINVAL;
    const int rc = cz_engine_add_conn(ENG(e), server ? 1 : 0, U8(0), (uint64_t)cnNonce, (uint64_t)cnPeerNonce);
    stage_out(env, v, 1, used, 0);  /* wipes the staged key (nothing to copy back) */
    return rc;
}

JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_removeConn(JNIEnv *env, jclass cls, jlong e, jint conn)
{
    (void)env, (void)cls;
    return e ? cz_engine_remove_conn(ENG(e), conn) : CZ_EINVAL;
}

JNIEXPORT jobject JNICALL Java_zmq_io_GpuCurveEngine_msgAlloc(JNIEnv *env, jclass cls, jlong e, jint len)
{
    (void)cls;
    if (!e || len < 0)
        return NULL;
    void *p = cz_engine_msg_alloc(ENG(e), (uint32_t)len);
    return p ? wrap(env, p, (uint64_t)len) : NULL;
}

JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_send(JNIEnv *env, jclass cls, jlong e, jint conn, jobject payload,
                                                        jint len, jint flags)
{
    (void)cls;
    const void *p = direct(env, payload, len);
    if (!e || len < 0 || !p)
        return CZ_EINVAL;
    return cz_engine_send(ENG(e), conn, p, (uint32_t)len, flags);
}

JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_flushOut(JNIEnv *env, jclass cls, jlong e)
{
    (void)env, (void)cls;
    return e ? cz_engine_flush_out(ENG(e)) : CZ_EINVAL;
}

/* one connection's wire bytes (for SocketChannel.write); valid until the next flushOut */
JNIEXPORT jobject JNICALL Java_zmq_io_GpuCurveEngine_wireOut(JNIEnv *env, jclass cls, jlong e, jint conn)
{
    (void)cls;
    const uint8_t *w = NULL;
    uint64_t len = 0;
    if (!e || cz_engine_wire_out(ENG(e), conn, &w, &len) != CZ_OK)
        return NULL;
    return wrap(env, w, len);
}

/* the same stream as gather-write pieces (SocketChannel.write(ByteBuffer[]), StreamEngine.java:509-535).
 * NULL with the JVM's exception pending when an allocation fails; each piece's local reference is
 * deleted once it is stored, so a stream of many pieces stays within the local-reference capacity. */
JNIEXPORT jobjectArray JNICALL Java_zmq_io_GpuCurveEngine_wireIov(JNIEnv *env, jclass cls, jlong e, jint conn)
{
    (void)cls;
    uint32_t n = 0;
    if (!e || cz_engine_wire_iov(ENG(e), conn, NULL, 0, &n) != CZ_OK)
        return NULL;
    cz_iovec *iov = (cz_iovec *)malloc(sizeof(cz_iovec) * (n ? n : 1));
    if (!iov)
        return NULL;
    jobjectArray out = NULL;
    if (cz_engine_wire_iov(ENG(e), conn, iov, n, &n) == CZ_OK) {
        jclass bb = (*env)->FindClass(env, "java/nio/ByteBuffer");
        if (bb && !(*env)->ExceptionCheck(env)) {
            out = (*env)->NewObjectArray(env, (jsize)n, bb, NULL);
            (*env)->DeleteLocalRef(env, bb);
            for (uint32_t i = 0; out && i < n; i++) {
                jobject piece = wrap(env, iov[i].base, iov[i].len);
                if (!piece || (*env)->ExceptionCheck(env)) {
                    (*env)->DeleteLocalRef(env, out);
                    out = NULL;
                    break;
                }
                (*env)->SetObjectArrayElement(env, out, (jsize)i, piece);
                (*env)->DeleteLocalRef(env, piece);
                if ((*env)->ExceptionCheck(env)) {
                    (*env)->DeleteLocalRef(env, out);
                    out = NULL;
                }
            }
        }
    }
    free(iov);
    return out;
}

JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_recv(JNIEnv *env, jclass cls, jlong e, jint conn, jobject wire,
                                                        jint len)
{
    (void)cls;
    const void *p = direct(env, wire, len);
    if (!e || len < 0 || !p)
        return CZ_EINVAL;
    return cz_engine_recv(ENG(e), conn, p, (uint64_t)len);
}

JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_flushIn(JNIEnv *env, jclass cls, jlong e)
{
    (void)env, (void)cls;
    return e ? cz_engine_flush_in(ENG(e)) : CZ_EINVAL;
}

JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_msgsIn(JNIEnv *env, jclass cls, jlong e, jint conn)
{
    (void)env, (void)cls;
    uint32_t n = 0;
    if (!e)
        return CZ_EINVAL;
    const int rc = cz_engine_msgs_in(ENG(e), conn, &n);
    return rc == CZ_OK ? (jint)n : rc;
}

/* decoded message i of the last flushIn (pinned, valid until the next one) -> session.pushMsg;
 * flags[0] = its MORE / COMMAND bits */
JNIEXPORT jobject JNICALL Java_zmq_io_GpuCurveEngine_msgIn(JNIEnv *env, jclass cls, jlong e, jint conn, jint i,
                                                            jintArray flags)
{
    (void)cls;
    const uint8_t *p = NULL;
    uint32_t len = 0;
    int fl = 0;
    if (!e || i < 0 || !flags || (*env)->GetArrayLength(env, flags) < 1 ||
        cz_engine_msg_in(ENG(e), conn, (uint32_t)i, &p, &len, &fl) != CZ_OK)
        return NULL;
    const jint f = fl;
    (*env)->SetIntArrayRegion(env, flags, 0, 1, &f);
    return wrap(env, p, len);
}

/* 0 while healthy; else CZ_EPROTO / CZ_EMSGSIZE and event[0] = the ZMTP protocol-error event
 * (StreamEngine -> socket.eventHandshakeFailedProtocol) */
JNIEXPORT jint JNICALL Java_zmq_io_GpuCurveEngine_connError(JNIEnv *env, jclass cls, jlong e, jint conn,
                                                             jintArray event)
{
    (void)cls;
    int ev = 0;
    if (!e || !event || (*env)->GetArrayLength(env, event) < 1)
        return CZ_EINVAL;
    const int rc = cz_engine_conn_error(ENG(e), conn, &ev);
    const jint v = ev;
    (*env)->SetIntArrayRegion(env, event, 0, 1, &v);
    return rc;
}
