/* jni_bench.c -- the host-resident CURVE path timed THROUGH the JNI shim (bench.py --config jni;
 * VERDICT r05 item 4).  The north star asks for the end-to-end rate including the JNI pinned-buffer
 * copies: this driver calls the natives of jni/curvezmq_jni.c exactly as the Java classes do
 * (GpuCurveBatch.sealUniform / openUniform over hostAlloc direct buffers, the jnacl
 * crypto_box_afternm / open_afternm per message over byte[] arrays, the GpuCurveEngine send /
 * flushOut / wireIov / recv / flushIn / msgIn loop of GpuCurveIoHook over 1024 connections), with
 * jni/fake_jni_env.c standing in for the JVM's JNIEnv (there is no JDK in this image).  Each leg is
 * also timed through the plain C-ABI in the same process, on the same buffers, so the shim's own
 * cost is the difference.  What the fake env cannot show is the JVM's side: the native-call
 * transition (tens of ns) and a real NewDirectByteBuffer (~0.1-0.5 us); the JSON reports how many
 * such calls each leg makes.  Prints one JSON line.
 *
 * Built by __graft_entry__.build() / jeromq_amd/build.py (build_jni_bench):
 *   gcc -O2 -DCZ_JNI_MIN -Ijni -Iinclude jni/jni_bench.c jni/curvezmq_jni.c jni/fake_jni_env.c
 *       -Ljeromq_amd -lcurvezmq_mi355x -Wl,--wrap=... -o tools/bin/jni_bench */
#define _POSIX_C_SOURCE 199309L /* clock_gettime */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "curvezmq_mi355x.h"
#include "jni_min.h"

/* ---- the natives (jni/curvezmq_jni.c) and the fake JNIEnv (jni/fake_jni_env.c) ------------------ */
#define BATCH(f) Java_zmq_io_mechanism_curve_GpuCurveBatch_##f
#define ENGINE(f) Java_zmq_io_GpuCurveEngine_##f
#define JNACL(f) Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_##f
jlong BATCH(create)(JNIEnv *, jclass, jint);
void BATCH(destroy)(JNIEnv *, jclass, jlong);
jint BATCH(setKeys)(JNIEnv *, jclass, jlong, jobject, jint, jint);
jint BATCH(sealUniform)(JNIEnv *, jclass, jlong, jint, jint, jobject, jlong, jobject, jlong, jlong, jobject, jint);
jint BATCH(openUniform)(JNIEnv *, jclass, jlong, jint, jint, jobject, jlong, jobject, jlong, jlong, jboolean, jobject,
                        jint);
jobject BATCH(hostAlloc)(JNIEnv *, jclass, jlong);
void BATCH(hostFree)(JNIEnv *, jclass, jobject);
jint JNACL(crypto_1box_1afternm)(JNIEnv *, jclass, jbyteArray, jbyteArray, jint, jbyteArray, jbyteArray);
jint JNACL(crypto_1box_1open_1afternm)(JNIEnv *, jclass, jbyteArray, jbyteArray, jint, jbyteArray, jbyteArray);
jlong ENGINE(create)(JNIEnv *, jclass, jlong, jint);
void ENGINE(destroy)(JNIEnv *, jclass, jlong);
jint ENGINE(addConn)(JNIEnv *, jclass, jlong, jboolean, jbyteArray, jlong, jlong);
jobject ENGINE(msgAlloc)(JNIEnv *, jclass, jlong, jint);
jint ENGINE(send)(JNIEnv *, jclass, jlong, jint, jobject, jint, jint);
jint ENGINE(flushOut)(JNIEnv *, jclass, jlong);
jobjectArray ENGINE(wireIov)(JNIEnv *, jclass, jlong, jint);
jint ENGINE(recv)(JNIEnv *, jclass, jlong, jint, jobject, jint);
jint ENGINE(flushIn)(JNIEnv *, jclass, jlong);
jint ENGINE(msgsIn)(JNIEnv *, jclass, jlong, jint);
jobject ENGINE(msgIn)(JNIEnv *, jclass, jlong, jint, jint, jintArray);
jint ENGINE(connError)(JNIEnv *, jclass, jlong, jint, jintArray);

JNIEnv *fake_env(void);
jobject fake_byte_array(void *data, jsize len);
jobject fake_int_array(void *data, jsize len);
jobject fake_direct(void *p, jlong cap);
void *fake_addr(jobject o);
jlong fake_cap(jobject o);
jsize fake_len(jobject o);
jobject fake_elem(jobject o, jsize i);

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static double median(double *v, int n)
{
    qsort(v, (size_t)n, sizeof(double), cmp_d);
    return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

#define FAIL(...) (fprintf(stderr, __VA_ARGS__), fputc('\n', stderr), exit(1))

static const uint8_t PRECOM[32] = {0x0e, 0x87, 0x90, 0xcb, 0x0d, 0xc8, 0x70, 0x3a, 0xf2, 0x53, 0x3c,
                                   0xc8, 0x59, 0x4e, 0xec, 0xfb, 0xf6, 0x2c, 0xa5, 0x60, 0xa6, 0x6e,
                                   0xbe, 0xe1, 0x25, 0x9c, 0xc0, 0xa3, 0x04, 0x35, 0xc6, 0xf3};

static void fill(uint8_t *p, uint64_t n, uint64_t seed)
{
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
    for (uint64_t i = 0; i < n; i += 8) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        const uint64_t k = n - i < 8 ? n - i : 8;
        memcpy(p + i, &x, k);
    }
}

/* ---- leg A: uniform batches through GpuCurveBatch (the pipelined host-staged path) --------------- */
static void uniform_leg(JNIEnv *env, int first, uint32_t n, uint32_t frames, int reps)
{
    const uint64_t ist = (n + 15u) & ~15u, ost = n >= 1024 ? (n + 33u + 127u) & ~127u : (n + 33u + 15u) & ~15u;
    const jint chunk = n >= 1024 ? 16384 : 0;
    const jlong ctx = BATCH(create)(env, NULL, 0);
    if (!ctx)
        FAIL("GpuCurveBatch.create: %s", cz_last_error());
    jobject keys = BATCH(hostAlloc)(env, NULL, 32);
    jobject in = BATCH(hostAlloc)(env, NULL, (jlong)(frames * ist));
    jobject out = BATCH(hostAlloc)(env, NULL, (jlong)(frames * ost));
    jobject back = BATCH(hostAlloc)(env, NULL, (jlong)(frames * ist));
    jobject st = BATCH(hostAlloc)(env, NULL, 2 * (jlong)frames);
    if (!keys || !in || !out || !back || !st)
        FAIL("hostAlloc: %s", cz_last_error());
    memcpy(fake_addr(keys), PRECOM, 32);
    if (BATCH(setKeys)(env, NULL, ctx, keys, 1, CZ_DIR_C2S) != CZ_OK)
        FAIL("setKeys: %s", cz_last_error());
    uint8_t *hin = (uint8_t *)fake_addr(in), *hback = (uint8_t *)fake_addr(back);
    fill(hin, frames * ist, n + frames);
    double ts[4][64];
    int nrep = reps < 64 ? reps : 64;
    /* 0: seal through the shim, 1: open through the shim, 2 / 3: the same through the C-ABI */
    for (int r = -1; r < nrep; r++) {
        double t0 = now();
        if (BATCH(sealUniform)(env, NULL, ctx, (jint)frames, (jint)n, in, (jlong)ist, out, (jlong)ost, 3, NULL, chunk))
            FAIL("sealUniform: %s", cz_last_error());
        double t1 = now();
        if (BATCH(openUniform)(env, NULL, ctx, (jint)frames, (jint)(n + 33), out, (jlong)ost, back, (jlong)ist, 2, 1, st,
                               chunk))
            FAIL("openUniform: %s", cz_last_error());
        double t2 = now();
        cz_ctx *c = (cz_ctx *)(intptr_t)ctx;
        if (cz_ctx_seal_uniform(c, frames, n, hin, ist, fake_addr(out), ost, 3, NULL, (uint32_t)chunk))
            FAIL("cz_ctx_seal_uniform: %s", cz_last_error());
        double t3 = now();
        if (cz_ctx_open_uniform(c, frames, n + 33, fake_addr(out), ost, hback, ist, 2, 1, (uint16_t *)fake_addr(st),
                                (uint32_t)chunk))
            FAIL("cz_ctx_open_uniform: %s", cz_last_error());
        double t4 = now();
        if (r >= 0)
            ts[0][r] = t1 - t0, ts[1][r] = t2 - t1, ts[2][r] = t3 - t2, ts[3][r] = t4 - t3;
    }
    int ok = 1;
    const uint16_t *s16 = (const uint16_t *)fake_addr(st);
    for (uint32_t i = 0; i < frames && ok; i++)
        ok = (s16[i] & 0xff) == 0 && memcmp(hin + i * ist, hback + i * ist, n) == 0;
    const double pay = (double)frames * n / (double)(1ull << 30);
    double m[4];
    for (int k = 0; k < 4; k++)
        m[k] = median(ts[k], nrep);
    printf("%s{\"payload_bytes\": %u, \"frames\": %u, \"seal_GiBps\": %.3f, \"open_GiBps\": %.3f, "
           "\"c_abi_seal_GiBps\": %.3f, \"c_abi_open_GiBps\": %.3f, \"seal_shim_over_c_abi\": %.4f, "
           "\"open_shim_over_c_abi\": %.4f, \"jni_calls_per_batch\": 1, \"verified\": %s}",
           first ? "" : ", ", n, frames, pay / m[0], pay / m[1], pay / m[2], pay / m[3], m[0] / m[2], m[1] / m[3],
           ok ? "true" : "false");
    BATCH(hostFree)(env, NULL, keys);
    BATCH(hostFree)(env, NULL, in);
    BATCH(hostFree)(env, NULL, out);
    BATCH(hostFree)(env, NULL, back);
    BATCH(hostFree)(env, NULL, st);
    BATCH(destroy)(env, NULL, ctx);
}

/* ---- leg B: one message per call through the jnacl natives (Curve.afternm / openAfternm) ---------- */
static void nacl_leg(JNIEnv *env, int first, uint32_t n)
{
    const uint32_t mlen = n + 32;
    uint8_t *m = calloc(mlen, 1), *c = calloc(mlen, 1), *b = calloc(mlen, 1), nonce[24], key[32];
    memcpy(nonce, "CurveZMQMESSAGEC\0\0\0\0\0\0\0\3", 24);
    memcpy(key, PRECOM, 32);
    fill(m + 32, n, n);
    jobject jm = fake_byte_array(m, (jsize)mlen), jc = fake_byte_array(c, (jsize)mlen), jb = fake_byte_array(b, (jsize)mlen);
    jobject jn = fake_byte_array(nonce, 24), jk = fake_byte_array(key, 32);
    enum { R = 200 };
    double ts[4][R];
    for (int r = -3; r < R; r++) {
        double t0 = now();
        if (JNACL(crypto_1box_1afternm)(env, NULL, jc, jm, (jint)mlen, jn, jk))
            FAIL("crypto_box_afternm");
        double t1 = now();
        if (JNACL(crypto_1box_1open_1afternm)(env, NULL, jb, jc, (jint)mlen, jn, jk))
            FAIL("crypto_box_open_afternm");
        double t2 = now();
        if (cz_box_afternm(c, m, mlen, nonce, key))
            FAIL("cz_box_afternm");
        double t3 = now();
        if (cz_box_open_afternm(b, c, mlen, nonce, key))
            FAIL("cz_box_open_afternm");
        double t4 = now();
        if (r >= 0)
            ts[0][r] = t1 - t0, ts[1][r] = t2 - t1, ts[2][r] = t3 - t2, ts[3][r] = t4 - t3;
    }
    const int ok = memcmp(b + 32, m + 32, n) == 0;
    double md[4];
    for (int k = 0; k < 4; k++)
        md[k] = median(ts[k], R);
    printf("%s{\"payload_bytes\": %u, \"seal_us\": %.2f, \"open_us\": %.2f, \"c_abi_seal_us\": %.2f, "
           "\"c_abi_open_us\": %.2f, \"verified\": %s}",
           first ? "" : ", ", n, md[0] * 1e6, md[1] * 1e6, md[2] * 1e6, md[3] * 1e6, ok ? "true" : "false");
    free(m), free(c), free(b);
}

/* ---- leg C: the batching engine through GpuCurveEngine, as GpuCurveIoHook drives it --------------- */
static void engine_leg(JNIEnv *env, int nconn, int per, uint32_t n)
{
    const uint64_t total = (uint64_t)nconn * per * n;
    const jlong cli = ENGINE(create)(env, NULL, (jlong)(total + (1u << 20)), 0);
    const jlong srv = ENGINE(create)(env, NULL, 1 << 20, 0);
    if (!cli || !srv)
        FAIL("GpuCurveEngine.create: %s", cz_last_error());
    int *cc = malloc(sizeof(int) * nconn), *sc = malloc(sizeof(int) * nconn);
    uint8_t key[32];
    jobject jkey = fake_byte_array(key, 32);
    for (int c = 0; c < nconn; c++) {
        for (int j = 0; j < 32; j++)
            key[j] = (uint8_t)(PRECOM[j] + c);
        cc[c] = ENGINE(addConn)(env, NULL, cli, 0, jkey, 3, 2);
        sc[c] = ENGINE(addConn)(env, NULL, srv, 1, jkey, 2, 2);
        if (cc[c] < 0 || sc[c] < 0)
            FAIL("addConn: %s", cz_last_error());
    }
    uint8_t *payload = malloc((size_t)per * n);
    fill(payload, (uint64_t)per * n, 77);
    int32_t flag = 0;
    jobject jflag = fake_int_array(&flag, 1);
    double t_send = 0, t_out = 0, t_iov = 0, t_recv = 0, t_in = 0, t_deliver = 0;
    uint64_t wire = 0, calls_out = 0, calls_in = 0;
    int ok = 1;
    for (int rep = 0; rep < 3; rep++) {   /* the first round warms allocations and clocks */
        double t0 = now();
        for (int c = 0; c < nconn; c++)
            for (int k = 0; k < per; k++) {   /* GpuCurveIoHook.queue: msgAlloc (pinnedMsg) + send */
                jobject b = ENGINE(msgAlloc)(env, NULL, cli, (jint)n);
                if (!b)
                    FAIL("msgAlloc: arena full");
                memcpy(fake_addr(b), payload + (size_t)k * n, n);
                if (ENGINE(send)(env, NULL, cli, cc[c], b, (jint)n, (k % 8 == 0) ? CZ_MSG_MORE : 0))
                    FAIL("send: %s", cz_last_error());
            }
        double t1 = now();
        if (ENGINE(flushOut)(env, NULL, cli))
            FAIL("flushOut: %s", cz_last_error());
        double t2 = now();
        /* endOfLoop's gathering write: the wireIov pieces of each connection (to the server here) */
        jobjectArray *iov = malloc(sizeof(jobjectArray) * nconn);
        wire = 0;
        for (int c = 0; c < nconn; c++) {
            iov[c] = ENGINE(wireIov)(env, NULL, cli, cc[c]);
            if (!iov[c])
                FAIL("wireIov: %s", cz_last_error());
        }
        double t3 = now();
        for (int c = 0; c < nconn; c++)   /* GpuCurveIoHook.inEvent: bytes read -> recv */
            for (jsize i = 0; i < fake_len(iov[c]); i++) {
                jobject p = fake_elem(iov[c], i);
                wire += (uint64_t)fake_cap(p);
                if (ENGINE(recv)(env, NULL, srv, sc[c], p, (jint)fake_cap(p)))
                    FAIL("recv: %s", cz_last_error());
            }
        double t4 = now();
        if (ENGINE(flushIn)(env, NULL, srv))
            FAIL("flushIn: %s", cz_last_error());
        double t5 = now();
        /* GpuCurveIoHook.deliver: msgsIn, msgIn per message, connError */
        for (int c = 0; c < nconn; c++) {
            const jint cnt = ENGINE(msgsIn)(env, NULL, srv, sc[c]);
            ok = ok && cnt == per;
            for (jint i = 0; i < cnt; i++) {
                jobject p = ENGINE(msgIn)(env, NULL, srv, sc[c], i, jflag);
                ok = ok && p && fake_cap(p) == (jlong)n;
                if (c == nconn - 1 && p)
                    ok = ok && memcmp(fake_addr(p), payload + (size_t)i * n, n) == 0 && flag == ((i % 8 == 0) ? 1 : 0);
            }
            ok = ok && ENGINE(connError)(env, NULL, srv, sc[c], jflag) == CZ_OK;
        }
        double t6 = now();
        free(iov);
        t_send = t1 - t0, t_out = t2 - t1, t_iov = t3 - t2, t_recv = t4 - t3, t_in = t5 - t4, t_deliver = t6 - t5;
        calls_out = (uint64_t)nconn * per * 2 + 1 + (uint64_t)nconn;
        calls_in = (uint64_t)nconn * per + (uint64_t)nconn * 2 + 1;
    }
    const double gib = (double)total / (double)(1ull << 30);
    printf("\"engine\": {\"connections\": %d, \"messages\": %d, \"payload_bytes\": %u, "
           "\"flush_out_GiBps\": %.3f, \"flush_in_GiBps\": %.3f, "
           "\"out_path_GiBps\": %.3f, \"in_path_GiBps\": %.3f, "
           "\"timings_s\": {\"msgAlloc_send_loop\": %.4f, \"flushOut\": %.4f, \"wireIov\": %.4f, \"recv_loop\": %.4f, "
           "\"flushIn\": %.4f, \"msgsIn_msgIn_loop\": %.4f}, \"jni_calls_out\": %llu, \"jni_calls_in\": %llu, "
           "\"wire_bytes\": %llu, \"verified\": %s}",
           nconn, nconn * per, n, gib / t_out, gib / t_in, gib / (t_send + t_out + t_iov),
           gib / (t_recv + t_in + t_deliver), t_send, t_out, t_iov, t_recv, t_in, t_deliver,
           (unsigned long long)calls_out, (unsigned long long)calls_in, (unsigned long long)wire, ok ? "true" : "false");
    ENGINE(destroy)(env, NULL, cli);
    ENGINE(destroy)(env, NULL, srv);
    free(cc), free(sc), free(payload);
}

int main(int argc, char **argv)
{
    /* argv[1]: largest 4 KiB uniform batch (default 2^20 frames); argv[2]: uniform reps */
    const uint32_t max4k = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    JNIEnv *env = fake_env();
    printf("{\"metric\": \"CURVE host path through the JNI shim (jni/curvezmq_jni.c over a fake JNIEnv), "
           "payload GiB/s\", \"uniform\": [");
    int first = 1;
    for (uint32_t f = 1u << 16; f <= max4k; f <<= 2, first = 0)
        uniform_leg(env, first, 4096, f, reps);
    uniform_leg(env, 0, 100, 1u << 16, reps);
    uniform_leg(env, 0, 100, 1u << 20, reps);
    printf("], \"jnacl\": [");
    nacl_leg(env, 1, 100);
    nacl_leg(env, 0, 4096);
    nacl_leg(env, 0, 65536);
    printf("], ");
    engine_leg(env, 1024, 256, 4096);
    printf("}\n");
    return 0;
}
