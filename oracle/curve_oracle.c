/*
 * curve_oracle.c -- CPU restatement of JeroMQ's CURVE per-message crypto path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the reported CPU baseline.  The product path
 * (jeromq_amd/, libcurvezmq_mi355x.so) never links or calls it.
 *
 * What it restates
 * ----------------
 * JeroMQ seals every ZMTP MESSAGE on a CURVE socket with
 *   Curve.afternm(box, plaintext, mlen, nonce, cnPrecom)
 *     jeromq-core/src/main/java/zmq/io/mechanism/curve/Curve.java:129-137
 * which forwards to the third-party jnacl artefact
 *   eu.neilalexander:jnacl:1.0.0  (jeromq-core/pom.xml:18-22)
 *   com.neilalexander.jnacl.crypto.curve25519xsalsa20poly1305.crypto_box_afternm
 * jnacl is NOT vendored in /root/reference, so the arithmetic below restates
 * the published NaCl construction it implements (crypto_box_afternm ==
 * crypto_secretbox_xsalsa20poly1305, NaCl 2011 / libsodium API):
 *   - Salsa20/20 core with feed-forward, HSalsa20 core (no feed-forward);
 *   - XSalsa20 stream: subkey = HSalsa20(k, n[0:16]); Salsa20(subkey, n[16:24]);
 *   - Poly1305 one-time MAC, key = keystream[0:32];
 *   - secretbox: c = m ^ keystream, c[16:32] = Poly1305(c[32:mlen]), c[0:16] = 0
 *     (32-byte ZEROBYTES in, 16-byte BOXZEROBYTES out).
 * The CurveZMQ MESSAGE framing follows
 *   CurveClientMechanism.encode/decode  CurveClientMechanism.java:126-224
 *   CurveServerMechanism.encode/decode  CurveServerMechanism.java:127-224
 *   nonce = "CurveZMQMESSAGE{C|S}" || BE64(cnNonce)   (Wire.putUInt64, Wire.java:124-136)
 *   body  = "\x07MESSAGE" || nonce[16:24] || box[16:mlen],  mlen = 32 + 1 + n
 *
 * Pinning: tests/test_oracle.py checks every function here against
 * the JSON fixtures in tests/golden/, which tests/golden/make_golden.py produced with
 * libsodium 1.0.18 (an independent implementation of the same NaCl
 * construction) and the CurveZMQ test keys published in the reference
 * (org/zeromq/ZMQ.java:4603-4624).
 *
 * The Poly1305 here deliberately uses 26-bit limbs (the device kernel uses a
 * 32-bit radix) so the oracle and the product share no arithmetic code.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#define ROTL32(v, c) (((v) << (c)) | ((v) >> (32 - (c))))

static uint32_t ld32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static void st32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

/* "expand 32-byte k" */
static const uint32_t SIGMA[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};

static void salsa_rounds(uint32_t x[16])
{
    for (int i = 0; i < 20; i += 2) {
        /* column round */
        x[4] ^= ROTL32(x[0] + x[12], 7);
        x[8] ^= ROTL32(x[4] + x[0], 9);
        x[12] ^= ROTL32(x[8] + x[4], 13);
        x[0] ^= ROTL32(x[12] + x[8], 18);
        x[9] ^= ROTL32(x[5] + x[1], 7);
        x[13] ^= ROTL32(x[9] + x[5], 9);
        x[1] ^= ROTL32(x[13] + x[9], 13);
        x[5] ^= ROTL32(x[1] + x[13], 18);
        x[14] ^= ROTL32(x[10] + x[6], 7);
        x[2] ^= ROTL32(x[14] + x[10], 9);
        x[6] ^= ROTL32(x[2] + x[14], 13);
        x[10] ^= ROTL32(x[6] + x[2], 18);
        x[3] ^= ROTL32(x[15] + x[11], 7);
        x[7] ^= ROTL32(x[3] + x[15], 9);
        x[11] ^= ROTL32(x[7] + x[3], 13);
        x[15] ^= ROTL32(x[11] + x[7], 18);
        /* row round */
        x[1] ^= ROTL32(x[0] + x[3], 7);
        x[2] ^= ROTL32(x[1] + x[0], 9);
        x[3] ^= ROTL32(x[2] + x[1], 13);
        x[0] ^= ROTL32(x[3] + x[2], 18);
        x[6] ^= ROTL32(x[5] + x[4], 7);
        x[7] ^= ROTL32(x[6] + x[5], 9);
        x[4] ^= ROTL32(x[7] + x[6], 13);
        x[5] ^= ROTL32(x[4] + x[7], 18);
        x[11] ^= ROTL32(x[10] + x[9], 7);
        x[8] ^= ROTL32(x[11] + x[10], 9);
        x[9] ^= ROTL32(x[8] + x[11], 13);
        x[10] ^= ROTL32(x[9] + x[8], 18);
        x[12] ^= ROTL32(x[15] + x[14], 7);
        x[13] ^= ROTL32(x[12] + x[15], 9);
        x[14] ^= ROTL32(x[13] + x[12], 13);
        x[15] ^= ROTL32(x[14] + x[13], 18);
    }
}

static void salsa_setup(uint32_t x[16], const uint8_t key[32], const uint8_t in16[16])
{
    x[0] = SIGMA[0];
    x[5] = SIGMA[1];
    x[10] = SIGMA[2];
    x[15] = SIGMA[3];
    for (int i = 0; i < 4; i++) {
        x[1 + i] = ld32(key + 4 * i);
        x[11 + i] = ld32(key + 16 + 4 * i);
        x[6 + i] = ld32(in16 + 4 * i);
    }
}

/* Salsa20/20 block: in16 = nonce8 || LE64(block counter). */
void or_salsa20_core(uint8_t out[64], const uint8_t in16[16], const uint8_t key[32])
{
    uint32_t x[16], j[16];
    salsa_setup(x, key, in16);
    memcpy(j, x, sizeof j);
    salsa_rounds(x);
    for (int i = 0; i < 16; i++)
        st32(out + 4 * i, x[i] + j[i]);
}

/* HSalsa20: 20 rounds, no feed-forward, output words 0,5,10,15,6,7,8,9. */
void or_hsalsa20(uint8_t out[32], const uint8_t in16[16], const uint8_t key[32])
{
    static const int pick[8] = {0, 5, 10, 15, 6, 7, 8, 9};
    uint32_t x[16];
    salsa_setup(x, key, in16);
    salsa_rounds(x);
    for (int i = 0; i < 8; i++)
        st32(out + 4 * i, x[pick[i]]);
}

/* XOR the Salsa20 stream (key, nonce8, starting block ic) over m into c. */
void or_salsa20_xor_ic(uint8_t *c, const uint8_t *m, uint64_t len, const uint8_t nonce8[8], uint64_t ic,
                       const uint8_t key[32])
{
    uint8_t in16[16], ks[64];
    memcpy(in16, nonce8, 8);
    uint64_t blk = ic;
    for (uint64_t off = 0; off < len; off += 64, blk++) {
        for (int i = 0; i < 8; i++)
            in16[8 + i] = (uint8_t)(blk >> (8 * i));
        or_salsa20_core(ks, in16, key);
        uint64_t take = len - off < 64 ? len - off : 64;
        for (uint64_t i = 0; i < take; i++)
            c[off + i] = (uint8_t)((m ? m[off + i] : 0) ^ ks[i]);
    }
}

void or_xsalsa20_xor(uint8_t *c, const uint8_t *m, uint64_t len, const uint8_t n24[24], const uint8_t key[32])
{
    uint8_t sub[32];
    or_hsalsa20(sub, n24, key);
    or_salsa20_xor_ic(c, m, len, n24 + 16, 0, sub);
}

/* ---- Poly1305, 5 x 26-bit limbs ---------------------------------------- */
typedef struct {
    uint32_t r[5], h[5], pad[4];
} poly26;

static void poly26_init(poly26 *st, const uint8_t key[32])
{
    st->r[0] = (ld32(key + 0)) & 0x3ffffff;
    st->r[1] = (ld32(key + 3) >> 2) & 0x3ffff03;
    st->r[2] = (ld32(key + 6) >> 4) & 0x3ffc0ff;
    st->r[3] = (ld32(key + 9) >> 6) & 0x3f03fff;
    st->r[4] = (ld32(key + 12) >> 8) & 0x00fffff;
    for (int i = 0; i < 5; i++)
        st->h[i] = 0;
    for (int i = 0; i < 4; i++)
        st->pad[i] = ld32(key + 16 + 4 * i);
}

/* one 16-byte block (blk already padded); hibit = 1<<24 for full blocks */
static void poly26_block(poly26 *st, const uint8_t blk[16], uint32_t hibit)
{
    const uint32_t r0 = st->r[0], r1 = st->r[1], r2 = st->r[2], r3 = st->r[3], r4 = st->r[4];
    const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
    uint32_t h0 = st->h[0], h1 = st->h[1], h2 = st->h[2], h3 = st->h[3], h4 = st->h[4];

    h0 += (ld32(blk + 0)) & 0x3ffffff;
    h1 += (ld32(blk + 3) >> 2) & 0x3ffffff;
    h2 += (ld32(blk + 6) >> 4) & 0x3ffffff;
    h3 += (ld32(blk + 9) >> 6) & 0x3ffffff;
    h4 += (ld32(blk + 12) >> 8) | hibit;

    uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
    uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
    uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
    uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
    uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;

    uint32_t c;
    c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & 0x3ffffff;
    d1 += c; c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & 0x3ffffff;
    d2 += c; c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & 0x3ffffff;
    d3 += c; c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & 0x3ffffff;
    d4 += c; c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & 0x3ffffff;
    h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
    h1 += c;

    st->h[0] = h0; st->h[1] = h1; st->h[2] = h2; st->h[3] = h3; st->h[4] = h4;
}

static void poly26_update(poly26 *st, const uint8_t *m, uint64_t len)
{
    while (len >= 16) {
        poly26_block(st, m, 1u << 24);
        m += 16;
        len -= 16;
    }
    if (len) {
        uint8_t blk[16] = {0};
        memcpy(blk, m, len);
        blk[len] = 1;
        poly26_block(st, blk, 0);
    }
}

static void poly26_finish(poly26 *st, uint8_t tag[16])
{
    uint32_t h0 = st->h[0], h1 = st->h[1], h2 = st->h[2], h3 = st->h[3], h4 = st->h[4], c;
    /* full carry */
    c = h1 >> 26; h1 &= 0x3ffffff;
    h2 += c; c = h2 >> 26; h2 &= 0x3ffffff;
    h3 += c; c = h3 >> 26; h3 &= 0x3ffffff;
    h4 += c; c = h4 >> 26; h4 &= 0x3ffffff;
    h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
    h1 += c;
    /* g = h + 5 - 2^130; pick g if it did not borrow */
    uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
    uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
    uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
    uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
    uint32_t g4 = h4 + c - (1u << 26);
    uint32_t mask = (g4 >> 31) - 1; /* all ones if no borrow */
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    h3 = (h3 & ~mask) | (g3 & mask);
    h4 = (h4 & ~mask) | (g4 & mask);
    /* to 4 x 32 bits, add pad mod 2^128 */
    uint32_t w0 = h0 | (h1 << 26);
    uint32_t w1 = (h1 >> 6) | (h2 << 20);
    uint32_t w2 = (h2 >> 12) | (h3 << 14);
    uint32_t w3 = (h3 >> 18) | (h4 << 8);
    uint64_t f;
    f = (uint64_t)w0 + st->pad[0]; st32(tag + 0, (uint32_t)f);
    f = (uint64_t)w1 + st->pad[1] + (f >> 32); st32(tag + 4, (uint32_t)f);
    f = (uint64_t)w2 + st->pad[2] + (f >> 32); st32(tag + 8, (uint32_t)f);
    f = (uint64_t)w3 + st->pad[3] + (f >> 32); st32(tag + 12, (uint32_t)f);
}

void or_poly1305(uint8_t tag[16], const uint8_t *m, uint64_t len, const uint8_t key[32])
{
    poly26 st;
    poly26_init(&st, key);
    poly26_update(&st, m, len);
    poly26_finish(&st, tag);
}

/* ---- NaCl secretbox / crypto_box_afternm --------------------------------- */
/* c and m are mlen bytes; m[0:32] must be zero (ZEROBYTES).  Returns 0 / -1. */
int or_secretbox(uint8_t *c, const uint8_t *m, uint64_t mlen, const uint8_t n24[24], const uint8_t key[32])
{
    if (mlen < 32)
        return -1;
    or_xsalsa20_xor(c, m, mlen, n24, key);
    or_poly1305(c + 16, c + 32, mlen - 32, c);
    memset(c, 0, 16);
    return 0;
}

int or_secretbox_open(uint8_t *m, const uint8_t *c, uint64_t clen, const uint8_t n24[24], const uint8_t key[32])
{
    uint8_t subkey_ks[32], tag[16];
    if (clen < 32)
        return -1;
    uint8_t sub[32];
    or_hsalsa20(sub, n24, key);
    or_salsa20_xor_ic(subkey_ks, NULL, 32, n24 + 16, 0, sub);
    or_poly1305(tag, c + 32, clen - 32, subkey_ks);
    uint8_t diff = 0;
    for (int i = 0; i < 16; i++)
        diff |= (uint8_t)(tag[i] ^ c[16 + i]);
    if (diff)
        return -1;
    or_salsa20_xor_ic(m, c, clen, n24 + 16, 0, sub);
    memset(m, 0, 32);
    return 0;
}

/* ---- CurveZMQ MESSAGE framing (CurveClientMechanism / CurveServerMechanism) ---- */
static void curve_nonce(uint8_t n24[24], int from_server, uint64_t counter)
{
    memcpy(n24, from_server ? "CurveZMQMESSAGES" : "CurveZMQMESSAGEC", 16);
    for (int i = 0; i < 8; i++)
        n24[16 + i] = (uint8_t)(counter >> (56 - 8 * i)); /* Wire.putUInt64: big-endian */
}

/*
 * Mechanism.encode for one MESSAGE: payload (n bytes) + flags -> body (33+n bytes).
 * from_server = 0: CurveClientMechanism.encode (nonce prefix ...MESSAGEC)
 * from_server = 1: CurveServerMechanism.encode (nonce prefix ...MESSAGES)
 * k = cnPrecom (crypto_box_beforenm output).  Returns the body length.
 */
uint64_t or_curve_encode(uint8_t *body, const uint8_t *payload, uint64_t n, uint8_t flags, uint64_t counter,
                         int from_server, const uint8_t k[32])
{
    uint64_t mlen = 33 + n;
    uint8_t *m = (uint8_t *)calloc(mlen, 1), *c = (uint8_t *)malloc(mlen);
    uint8_t n24[24];
    curve_nonce(n24, from_server, counter);
    m[32] = flags;
    if (n)
        memcpy(m + 33, payload, n);
    or_secretbox(c, m, mlen, n24, k);
    memcpy(body, "\x07MESSAGE", 8);
    memcpy(body + 8, n24 + 16, 8);
    memcpy(body + 16, c + 16, mlen - 16);
    free(m);
    free(c);
    return mlen;
}

/*
 * Mechanism.decode for one MESSAGE body (size bytes).  from_server names the
 * SENDER of the body (1: it was sealed by the server, i.e. we are the client).
 * Returns 0 and fills payload (size-33 bytes), *flags, *nonce; otherwise
 *   3 = not a MESSAGE command  (CurveClientMechanism.java:168-172)
 *   2 = shorter than 33 bytes  (CurveClientMechanism.java:174-178)
 *   1 = failed tag             (CurveClientMechanism.java:219-223)
 * The command test is Msgs.startsWith(msg, "MESSAGE", true) (zmq/io/Msgs.java:20-39):
 * size >= 8, byte 0 == 7, and bytes 1..6 == "MESSAG" -- its loop stops one
 * character short, so byte 7 is never compared.  Restated as is.
 * The replay check (nonce <= cnPeerNonce) is the caller's: CurveClientMechanism.java:186-193.
 */
int or_curve_decode(uint8_t *payload, uint8_t *flags, uint64_t *nonce, const uint8_t *body, uint64_t size,
                    int from_server, const uint8_t k[32])
{
    if (size < 8 || body[0] != 7 || memcmp(body + 1, "MESSAG", 6) != 0)
        return 3;
    if (size < 33)
        return 2;
    uint64_t clen = 16 + size - 16;
    uint8_t *c = (uint8_t *)calloc(clen, 1), *m = (uint8_t *)malloc(clen);
    uint8_t n24[24];
    memcpy(n24, from_server ? "CurveZMQMESSAGES" : "CurveZMQMESSAGEC", 16);
    memcpy(n24 + 16, body + 8, 8);
    uint64_t nn = 0;
    for (int i = 0; i < 8; i++)
        nn = (nn << 8) | body[8 + i];
    *nonce = nn;
    memcpy(c + 16, body + 16, size - 16);
    int rc = or_secretbox_open(m, c, clen, n24, k);
    if (rc == 0) {
        *flags = m[32];
        if (size > 33)
            memcpy(payload, m + 33, size - 33);
    }
    free(c);
    free(m);
    return rc == 0 ? 0 : 1;
}

/* ---- synthetic input generator shared with the device (counter-based SplitMix64) ---- */
uint64_t or_splitmix64(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* fill buf[0:len) with the byte stream of words or_splitmix64(seed, 0), (seed, 1), ... (LE) */
void or_fill(uint8_t *buf, uint64_t len, uint64_t seed)
{
    for (uint64_t w = 0; w * 8 < len; w++) {
        uint64_t v = or_splitmix64(seed, w);
        for (int i = 0; i < 8 && w * 8 + i < len; i++)
            buf[w * 8 + i] = (uint8_t)(v >> (8 * i));
    }
}

/* ---- batched seal over a descriptor list, used as the CPU baseline ---------------- */
/* Same descriptor layout as include/curvezmq_mi355x.h cz_frame_desc. */
typedef struct {
    uint64_t in_off, out_off;
    uint32_t len, key_idx;
    uint64_t counter;
    uint32_t flags;
    int32_t prev;
} or_frame_desc;

typedef struct {
    const or_frame_desc *d;
    uint64_t begin, end;
    const uint8_t *in;
    uint8_t *out;
    const uint8_t *precom; /* 32 B per key_idx: cnPrecom */
    int from_server;
} or_job;

static void *or_seal_worker(void *arg)
{
    or_job *j = (or_job *)arg;
    for (uint64_t i = j->begin; i < j->end; i++) {
        const or_frame_desc *d = &j->d[i];
        or_curve_encode(j->out + d->out_off, j->in + d->in_off, d->len, (uint8_t)d->flags, d->counter,
                        j->from_server, j->precom + 32ull * d->key_idx);
    }
    return NULL;
}

/* Seal count frames with nthreads POSIX threads (the reference's IO-thread parallelism analogue). */
void or_seal_batch(const or_frame_desc *d, uint64_t count, const uint8_t *in, uint8_t *out, const uint8_t *precom,
                   int from_server, int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    pthread_t th[256];
    or_job jobs[256];
    if (nthreads > 256)
        nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        jobs[t].d = d;
        jobs[t].begin = count * t / nthreads;
        jobs[t].end = count * (t + 1) / nthreads;
        jobs[t].in = in;
        jobs[t].out = out;
        jobs[t].precom = precom;
        jobs[t].from_server = from_server;
        pthread_create(&th[t], NULL, or_seal_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------------------
 * X25519 and crypto_box (the CURVE handshake's key agreement).
 *   Curve.beforenm  -> jnacl crypto_box_beforenm   Curve.java:124-127
 *   Curve.keypair   -> jnacl crypto_box_keypair    Curve.java:100-115
 *   Curve.box/open  -> jnacl crypto_box[_open]     Curve.java:149-193
 * Restated from RFC 7748 section 5 (Montgomery ladder, a24 = 121665, clamped scalar,
 * u masked to 255 bits) in radix 2^51 with 128-bit products -- the device uses radix
 * 2^25.5 with 32x32->64 multiply-adds, so again no arithmetic is shared.
 * beforenm(k, pk, sk) = HSalsa20(X25519(sk, pk), 0^16): NaCl crypto_box_beforenm.
 * ---------------------------------------------------------------------------------- */
typedef uint64_t or_fe[5];
typedef unsigned __int128 or_u128;
static const uint64_t OR_M51 = (1ull << 51) - 1;

static void or_fe_frombytes(or_fe h, const uint8_t s[32])
{
    uint64_t w[4];
    for (int i = 0; i < 4; i++) {
        w[i] = 0;
        for (int b = 7; b >= 0; b--)
            w[i] = (w[i] << 8) | s[8 * i + b];
    }
    h[0] = w[0] & OR_M51;
    h[1] = ((w[0] >> 51) | (w[1] << 13)) & OR_M51;
    h[2] = ((w[1] >> 38) | (w[2] << 26)) & OR_M51;
    h[3] = ((w[2] >> 25) | (w[3] << 39)) & OR_M51;
    h[4] = (w[3] >> 12) & OR_M51; /* bit 255 masked (RFC 7748 section 5) */
}

static void or_fe_carry(or_fe h)
{
    for (int r = 0; r < 2; r++) {
        uint64_t c;
        for (int i = 0; i < 4; i++) {
            c = h[i] >> 51;
            h[i] &= OR_M51;
            h[i + 1] += c;
        }
        c = h[4] >> 51;
        h[4] &= OR_M51;
        h[0] += 19 * c;
    }
}

static void or_fe_tobytes(uint8_t s[32], const or_fe f)
{
    or_fe h;
    memcpy(h, f, sizeof(or_fe));
    or_fe_carry(h);
    /* h < 2^255 + small: subtract p if h >= p */
    uint64_t q = (h[0] + 19) >> 51;
    q = (h[1] + q) >> 51;
    q = (h[2] + q) >> 51;
    q = (h[3] + q) >> 51;
    q = (h[4] + q) >> 51;
    h[0] += 19 * q;
    for (int i = 0; i < 4; i++) {
        h[i + 1] += h[i] >> 51;
        h[i] &= OR_M51;
    }
    h[4] &= OR_M51;
    uint64_t w[4] = {h[0] | (h[1] << 51), (h[1] >> 13) | (h[2] << 38), (h[2] >> 26) | (h[3] << 25),
                     (h[3] >> 39) | (h[4] << 12)};
    for (int i = 0; i < 4; i++)
        for (int b = 0; b < 8; b++)
            s[8 * i + b] = (uint8_t)(w[i] >> (8 * b));
}

static void or_fe_add(or_fe h, const or_fe f, const or_fe g)
{
    for (int i = 0; i < 5; i++)
        h[i] = f[i] + g[i];
}

/* h = f - g + 4p (limbs stay positive for carried inputs) */
static void or_fe_sub(or_fe h, const or_fe f, const or_fe g)
{
    static const uint64_t P4[5] = {4 * (OR_M51 - 18), 4 * OR_M51, 4 * OR_M51, 4 * OR_M51, 4 * OR_M51};
    for (int i = 0; i < 5; i++)
        h[i] = f[i] + P4[i] - g[i];
    or_fe_carry(h);
}

static void or_fe_mul(or_fe h, const or_fe f, const or_fe g)
{
    or_u128 t[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 5; j++) {
            or_u128 p = (or_u128)f[i] * g[j];
            if (i + j < 5)
                t[i + j] += p;
            else
                t[i + j - 5] += p * 19;
        }
    or_u128 c = 0;
    for (int i = 0; i < 5; i++) {
        t[i] += c;
        h[i] = (uint64_t)t[i] & OR_M51;
        c = t[i] >> 51;
    }
    h[0] += (uint64_t)c * 19;
    or_fe_carry(h);
}

static void or_fe_mul_small(or_fe h, const or_fe f, uint64_t k)
{
    or_u128 c = 0;
    for (int i = 0; i < 5; i++) {
        or_u128 t = (or_u128)f[i] * k + c;
        h[i] = (uint64_t)t & OR_M51;
        c = t >> 51;
    }
    h[0] += (uint64_t)c * 19;
    or_fe_carry(h);
}

static void or_fe_pow(or_fe h, const or_fe f, const uint8_t e[32]) /* square-and-multiply, e little-endian */
{
    or_fe r = {1, 0, 0, 0, 0};
    for (int bit = 255; bit >= 0; bit--) {
        or_fe_mul(r, r, r);
        if ((e[bit >> 3] >> (bit & 7)) & 1)
            or_fe_mul(r, r, f);
    }
    memcpy(h, r, sizeof(or_fe));
}

static void or_fe_cswap(or_fe a, or_fe b, uint64_t swap)
{
    const uint64_t m = 0 - swap;
    for (int i = 0; i < 5; i++) {
        uint64_t t = m & (a[i] ^ b[i]);
        a[i] ^= t;
        b[i] ^= t;
    }
}

/* X25519(k, u) per RFC 7748 section 5 */
void or_x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t u[32])
{
    uint8_t k[32];
    memcpy(k, scalar, 32);
    k[0] &= 248;
    k[31] &= 127;
    k[31] |= 64;
    or_fe x1, x2 = {1, 0, 0, 0, 0}, z2 = {0, 0, 0, 0, 0}, x3, z3 = {1, 0, 0, 0, 0};
    or_fe_frombytes(x1, u);
    memcpy(x3, x1, sizeof(or_fe));
    uint64_t swap = 0;
    for (int t = 254; t >= 0; t--) {
        const uint64_t kt = (k[t >> 3] >> (t & 7)) & 1;
        swap ^= kt;
        or_fe_cswap(x2, x3, swap);
        or_fe_cswap(z2, z3, swap);
        swap = kt;
        or_fe A, AA, B, BB, E, C, D, DA, CB, t0, t1;
        or_fe_add(A, x2, z2);
        or_fe_mul(AA, A, A);
        or_fe_sub(B, x2, z2);
        or_fe_mul(BB, B, B);
        or_fe_sub(E, AA, BB);
        or_fe_add(C, x3, z3);
        or_fe_sub(D, x3, z3);
        or_fe_mul(DA, D, A);
        or_fe_mul(CB, C, B);
        or_fe_add(t0, DA, CB);
        or_fe_mul(x3, t0, t0);
        or_fe_sub(t1, DA, CB);
        or_fe_mul(t1, t1, t1);
        or_fe_mul(z3, x1, t1);
        or_fe_mul(x2, AA, BB);
        or_fe_mul_small(t0, E, 121665);
        or_fe_add(t0, AA, t0);
        or_fe_mul(z2, E, t0);
    }
    or_fe_cswap(x2, x3, swap);
    or_fe_cswap(z2, z3, swap);
    /* z2^(p-2), p - 2 = 2^255 - 21 */
    static const uint8_t PM2[32] = {0xeb, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f};
    or_fe zi, r;
    or_fe_pow(zi, z2, PM2);
    or_fe_mul(r, x2, zi);
    or_fe_tobytes(out, r);
}

void or_scalarmult_base(uint8_t pk[32], const uint8_t sk[32])
{
    uint8_t nine[32] = {9};
    or_x25519(pk, sk, nine);
}

/* NaCl crypto_box_beforenm: k = HSalsa20(X25519(sk, pk), 0^16) */
void or_box_beforenm(uint8_t k[32], const uint8_t pk[32], const uint8_t sk[32])
{
    uint8_t s[32];
    static const uint8_t zero[16] = {0};
    or_x25519(s, sk, pk);
    or_hsalsa20(k, zero, s);
}
