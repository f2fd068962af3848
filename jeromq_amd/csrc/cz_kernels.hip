// cz_kernels.hip -- batched CurveZMQ MESSAGE seal/open kernels for MI355X (gfx950).
//
// Reference path:
//   CurveClientMechanism.encode / CurveServerMechanism.encode
//     (CurveClientMechanism.java:126-163, CurveServerMechanism.java:127-163)
//     -> Curve.afternm (Curve.java:129-137) -> jnacl crypto_box_afternm
//   CurveClientMechanism.decode / CurveServerMechanism.decode
//     (CurveClientMechanism.java:165-224, CurveServerMechanism.java:165-224)
//     -> Curve.openAfternm (Curve.java:139-147) -> jnacl crypto_box_open_afternm
//
// Work mapping: ONE FRAME PER LANE.  A lane walks its frame's Salsa20 blocks in
// order, keeps the 64-byte block state in VGPRs and accumulates Poly1305 with
// a serial Horner chain -- so there are no cross-lane reductions and no r^k
// power tables (Poly1305's key is different for every frame, so a power table
// would never amortise).  Frames of a wave are independent, so a uniform batch
// runs divergence-free.  Memory: each lane streams 64 B per step through four
// 16-byte loads/stores; the 33-byte MESSAGE header shift (flag byte + 32-byte
// NaCl zero prefix) is absorbed with v_alignbyte_b32 funnel shifts and a
// 1-dword (seal) / 4-dword (open) carry, so every global access is a 16-byte
// aligned dwordx4 when the frame offsets are 16-byte aligned (the fast path);
// other alignments take a byte-wise path with identical results.
//
// Layout (box coordinates, mlen = 33 + n for a MESSAGE):
//   box[0:32]   = NaCl ZEROBYTES (keystream bytes 0..31 are the Poly1305 key)
//   box[32]     = flags (MORE=1, COMMAND=2),  box[33:33+n] = payload
//   body[i]     = box[i] for i >= 16; body[0:8] = "\x07MESSAGE", body[8:16] = BE64(counter)
//   tag         = Poly1305(box[32:mlen]) stored at body[16:32]
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cz_device.h"
#include "../../include/curvezmq_mi355x.h"

using namespace cz;

namespace {

enum Mode { MODE_ZMQ = 0, MODE_NACL = 1 };

// "\x07MESSAGE" as two little-endian words
constexpr u32 HDR0 = 0x53454d07u, HDR1 = 0x45474153u;

struct V4 {
    u32 x, y, z, w;
};

__device__ __forceinline__ V4 zero4() { return V4{0u, 0u, 0u, 0u}; }

// Load 16 bytes from p.  avail = bytes of the object remaining at p.
// AL: p is 16-byte aligned, so reading the whole aligned chunk once any byte of
// it is valid cannot cross a page; bytes past the object are ignored by callers.
template <bool AL>
__device__ __forceinline__ V4 ld16(const uint8_t *__restrict__ p, u64 avail)
{
    if (avail == 0)
        return zero4();
    if constexpr (AL) {
        uint4 v = *reinterpret_cast<const uint4 *>(p);
        return V4{v.x, v.y, v.z, v.w};
    } else {
        u32 w[4] = {0u, 0u, 0u, 0u};
        u32 lim = avail < 16 ? (u32)avail : 16u;
        for (u32 i = 0; i < lim; i++)
            w[i >> 2] |= (u32)p[i] << (8 * (i & 3));
        return V4{w[0], w[1], w[2], w[3]};
    }
}

// Unguarded full-chunk load (caller proved all 16 bytes valid).
template <bool AL>
__device__ __forceinline__ V4 ld16f(const uint8_t *__restrict__ p)
{
    if constexpr (AL) {
        uint4 v = *reinterpret_cast<const uint4 *>(p);
        return V4{v.x, v.y, v.z, v.w};
    } else {
        return ld16<false>(p, 16);
    }
}

template <bool AL>
__device__ __forceinline__ void st16(uint8_t *__restrict__ p, u32 a, u32 b, u32 c, u32 d)
{
    if constexpr (AL) {
        *reinterpret_cast<uint4 *>(p) = make_uint4(a, b, c, d);
    } else {
        u32 w[4] = {a, b, c, d};
#pragma unroll
        for (int i = 0; i < 16; i++)
            p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// Store the first nb (0..16) bytes of a 16-byte chunk.
__device__ __forceinline__ void st_bytes(uint8_t *__restrict__ p, u32 a, u32 b, u32 c, u32 d, u32 nb)
{
    u32 w[4] = {a, b, c, d};
    for (u32 i = 0; i < nb; i++)
        p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ u32 funnel(u32 hi, u32 lo, u32 sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }

// MAC + store the 16-byte sub-blocks j in [j0, 4) of box block blk whose box
// bytes are < valid (relative to the block start).  Used for every block that
// is not a full 64-byte block, and for block 0's ciphertext half.
template <bool AL>
__device__ __forceinline__ void emit_guarded(Poly &P, const u32 C[16], int j0, u32 valid, uint8_t *__restrict__ dst,
                                             bool store)
{
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (j < j0)
            continue;
        u32 s = 16u * j;
        if (s >= valid)
            continue;
        u32 nb = valid - s;
        if (nb >= 16) {
            poly_block(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], 1u);
            if (store)
                st16<AL>(dst + s, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3]);
        } else {
            poly_block_partial(P, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], nb);
            if (store)
                st_bytes(dst + s, C[4 * j], C[4 * j + 1], C[4 * j + 2], C[4 * j + 3], nb);
        }
    }
}

// --------------------------------------------------------------------------
// SEAL one frame.
//   MODE_ZMQ : in = payload (n bytes), out = MESSAGE body (33 + n bytes)
//   MODE_NACL: in = m (mlen bytes, m[0:32] ignored/zero), out = c (mlen bytes)
// key = Salsa20 subkey (HSalsa20 already applied), nonce words from `counter`
// (ZMQ: BE64 counter; NaCl: the caller passes n[16:24] read big-endian).
// --------------------------------------------------------------------------
template <int MODE, bool AL>
__device__ void seal_frame(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, u32 n, u32 flags, u64 counter,
                           const u32 key[8])
{
    // Input shift: box byte i comes from in[i - SH] (ZMQ: SH = 33, NaCl: 0).
    // ZMQ funnel: box dword k of block b = alignbyte(P[16b+k-8], P[16b+k-9], 3)
    // where P[i] is payload dword i; the window of block b is P[16b-8 .. 16b+7]
    // (payload bytes [64b-32, 64b+32)), and P[16b-9] is carried from block b-1.
    const u32 mlen = (MODE == MODE_ZMQ) ? n + 33u : n;
    const u32 nfull = mlen >> 6;
    const u32 tailv = mlen & 63u;
    const u64 inlen = n;  // bytes readable at `in`
    u32 n0, n1;
    counter_nonce(counter, n0, n1);

    u32 x[16], C[16];
    salsa20_block(x, key, n0, n1, 0u, 0u);
    Poly P;
    poly_init(P, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);

    u32 carry;
    {
        // block 0: box bytes 32..63
        u32 W[16];
        if constexpr (MODE == MODE_ZMQ) {
            V4 a = ld16<AL>(in, inlen);
            V4 b = ld16<AL>(in + 16, inlen > 16 ? inlen - 16 : 0);
            W[7] = flags << 24;  // payload byte -1 is the flag byte (box[32])
            W[8] = a.x; W[9] = a.y; W[10] = a.z; W[11] = a.w;
            W[12] = b.x; W[13] = b.y; W[14] = b.z; W[15] = b.w;
#pragma unroll
            for (int k = 8; k < 16; k++)
                C[k] = funnel(W[k], W[k - 1], 3) ^ x[k];
            carry = W[15];
        } else {
            V4 a = ld16<AL>(in + 32, inlen > 32 ? inlen - 32 : 0);
            V4 b = ld16<AL>(in + 48, inlen > 48 ? inlen - 48 : 0);
            C[8] = a.x ^ x[8]; C[9] = a.y ^ x[9]; C[10] = a.z ^ x[10]; C[11] = a.w ^ x[11];
            C[12] = b.x ^ x[12]; C[13] = b.y ^ x[13]; C[14] = b.z ^ x[14]; C[15] = b.w ^ x[15];
            carry = 0;
        }
        if constexpr (MODE == MODE_ZMQ)
            st16<AL>(out, HDR0, HDR1, n0, n1);
        else
            st16<AL>(out, 0u, 0u, 0u, 0u);
        if (nfull >= 1) {
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
            st16<AL>(out + 32, C[8], C[9], C[10], C[11]);
            st16<AL>(out + 48, C[12], C[13], C[14], C[15]);
        } else {
            emit_guarded<AL>(P, C, 2, mlen, out, true);
        }
    }

    // steady state: full 64-byte blocks 1 .. nfull-1, all inputs in range
    for (u32 blk = 1; blk < nfull; blk++) {
        V4 q0, q1, q2, q3;
        if constexpr (MODE == MODE_ZMQ) {
            const uint8_t *src = in + 64u * blk - 32u;
            q0 = ld16f<AL>(src);
            q1 = ld16f<AL>(src + 16);
            q2 = ld16f<AL>(src + 32);
            q3 = ld16<AL>(src + 48, inlen - (64u * blk + 16u));  // may end inside this chunk
        } else {
            const uint8_t *src = in + 64u * blk;
            q0 = ld16f<AL>(src);
            q1 = ld16f<AL>(src + 16);
            q2 = ld16f<AL>(src + 32);
            q3 = ld16f<AL>(src + 48);
        }
        salsa20_block(x, key, n0, n1, blk, 0u);
        u32 W[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                     q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
        if constexpr (MODE == MODE_ZMQ) {
            C[0] = funnel(W[0], carry, 3) ^ x[0];
#pragma unroll
            for (int k = 1; k < 16; k++)
                C[k] = funnel(W[k], W[k - 1], 3) ^ x[k];
            carry = W[15];
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++)
                C[k] = W[k] ^ x[k];
        }
        uint8_t *dst = out + 64u * blk;
        st16<AL>(dst, C[0], C[1], C[2], C[3]);
        st16<AL>(dst + 16, C[4], C[5], C[6], C[7]);
        st16<AL>(dst + 32, C[8], C[9], C[10], C[11]);
        st16<AL>(dst + 48, C[12], C[13], C[14], C[15]);
        poly_block(P, C[0], C[1], C[2], C[3], 1u);
        poly_block(P, C[4], C[5], C[6], C[7], 1u);
        poly_block(P, C[8], C[9], C[10], C[11], 1u);
        poly_block(P, C[12], C[13], C[14], C[15], 1u);
    }

    // final partial block
    if (tailv != 0 && nfull >= 1) {
        const u32 blk = nfull;
        V4 q[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            long o = (MODE == MODE_ZMQ) ? (long)(64u * blk) - 32 + 16 * c : (long)(64u * blk) + 16 * c;
            u64 avail = (o >= 0 && (u64)o < inlen) ? inlen - (u64)o : 0;
            q[c] = ld16<AL>(in + o, avail);
        }
        salsa20_block(x, key, n0, n1, blk, 0u);
        u32 W[16] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w,
                     q[2].x, q[2].y, q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w};
        if constexpr (MODE == MODE_ZMQ) {
            C[0] = funnel(W[0], carry, 3) ^ x[0];
#pragma unroll
            for (int k = 1; k < 16; k++)
                C[k] = funnel(W[k], W[k - 1], 3) ^ x[k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++)
                C[k] = W[k] ^ x[k];
        }
        emit_guarded<AL>(P, C, 0, tailv, out + 64u * blk, true);
    }

    u32 tag[4];
    poly_finish(P, tag);
    st16<AL>(out + 16, tag[0], tag[1], tag[2], tag[3]);
}

// --------------------------------------------------------------------------
// OPEN one frame.  Returns a CZ_STATUS_* code.
//   MODE_ZMQ : in = MESSAGE body (size bytes), out = payload (size - 33 bytes);
//              *flags_out = box[32]; *nonce_out = BE64(body[8:16]).
//   MODE_NACL: in = c (size bytes), out = m (size bytes, m[0:32] = 0).
// The replay check of decode (CurveClientMechanism.java:186-193) compares the
// frame nonce against `floor` as signed 64-bit values, like Java's long.
// On a bad tag the plaintext already written is overwritten with zeros.
// --------------------------------------------------------------------------
template <int MODE, bool AL>
__device__ u32 open_frame(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, u32 size, const u32 key_in[8],
                          bool check_floor, long long floor, u32 *flags_out, u64 *nonce_out, u64 nacl_counter)
{
    u32 n0, n1;
    if constexpr (MODE == MODE_ZMQ) {
        // Msgs.startsWith(msg, "MESSAGE", true) (zmq/io/Msgs.java:20-39): size >= 8,
        // byte 0 == 7, bytes 1..6 == "MESSAG" (its loop never reaches byte 7).
        if (size < 8u)
            return CZ_STATUS_COMMAND;
        V4 h = ld16<AL>(in, size);
        if (h.x != HDR0 || (h.y & 0x00ffffffu) != (HDR1 & 0x00ffffffu))
            return CZ_STATUS_COMMAND;
        if (size < 33u)
            return CZ_STATUS_MALFORMED;
        n0 = h.z;
        n1 = h.w;
        u64 nonce = ((u64)bswap32(n0) << 32) | (u64)bswap32(n1);
        *nonce_out = nonce;
        if (check_floor && (long long)nonce <= floor)
            return CZ_STATUS_SEQUENCE;
    } else {
        if (size < 32u)
            return CZ_STATUS_MALFORMED;
        counter_nonce(nacl_counter, n0, n1);
    }
    u32 key[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        key[i] = key_in[i];

    const u32 mlen = size;
    const u32 nfull = mlen >> 6;
    const u32 tailv = mlen & 63u;
    const u32 nout = (MODE == MODE_ZMQ) ? size - 33u : size;  // bytes writable at out

    u32 x[16], C[16], X[16];
    salsa20_block(x, key, n0, n1, 0u, 0u);
    Poly P;
    poly_init(P, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
    V4 tin = ld16<AL>(in + 16, size - 16u);

    // ZMQ output schedule: payload dword j = alignbyte(D[j+9], D[j+8], 1) with D the
    // plaintext box dwords.  After block b the lane emits payload bytes
    // [64b-48, 64b+16) from D[16b-4 .. 16b+12]; D[16b-4 .. 16b-1] is the carry.
    u32 cy0 = 0, cy1 = 0, cy2 = 0, cy3 = 0;

    auto emit_zmq = [&](u32 blk, const u32 D[16], bool guarded) {
        // E[i] = D[16b-4+i], i = 0..16  (E[0..3] = carry, E[4..19] = D)
        u32 E[20] = {cy0, cy1, cy2, cy3, D[0], D[1], D[2], D[3], D[4], D[5], D[6], D[7],
                     D[8], D[9], D[10], D[11], D[12], D[13], D[14], D[15]};
        long base = (long)(64u * blk) - 48;  // payload byte offset of the first emitted chunk
#pragma unroll
        for (int c = 0; c < 4; c++) {
            // payload dword j = 16b-12 + 4c + t  ->  D[j+8] = E[4c+t], D[j+9] = E[4c+t+1]
            u32 o0 = funnel(E[4 * c + 1], E[4 * c + 0], 1);
            u32 o1 = funnel(E[4 * c + 2], E[4 * c + 1], 1);
            u32 o2 = funnel(E[4 * c + 3], E[4 * c + 2], 1);
            u32 o3 = funnel(E[4 * c + 4], E[4 * c + 3], 1);
            long o = base + 16 * c;
            if (!guarded) {
                st16<AL>(out + o, o0, o1, o2, o3);
            } else if (o >= 0 && (u64)o < nout) {
                u64 rem = nout - (u64)o;
                if (rem >= 16)
                    st16<AL>(out + o, o0, o1, o2, o3);
                else
                    st_bytes(out + o, o0, o1, o2, o3, (u32)rem);
            }
        }
        cy0 = D[12]; cy1 = D[13]; cy2 = D[14]; cy3 = D[15];
    };

    // block 0
    {
        V4 a = ld16<AL>(in + 32, size > 32 ? size - 32u : 0);
        V4 b = ld16<AL>(in + 48, size > 48 ? size - 48u : 0);
        C[8] = a.x; C[9] = a.y; C[10] = a.z; C[11] = a.w;
        C[12] = b.x; C[13] = b.y; C[14] = b.z; C[15] = b.w;
#pragma unroll
        for (int k = 0; k < 8; k++)
            C[k] = 0;
        if (nfull >= 1) {
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
        } else {
            emit_guarded<AL>(P, C, 2, mlen, nullptr, false);
        }
#pragma unroll
        for (int k = 0; k < 16; k++)
            X[k] = k < 8 ? 0u : (C[k] ^ x[k]);
        if constexpr (MODE == MODE_ZMQ) {
            *flags_out = X[8] & 0xffu;
            emit_zmq(0, X, true);
        } else {
            if (nfull >= 1) {
                st16<AL>(out, 0u, 0u, 0u, 0u);
                st16<AL>(out + 16, 0u, 0u, 0u, 0u);
                st16<AL>(out + 32, X[8], X[9], X[10], X[11]);
                st16<AL>(out + 48, X[12], X[13], X[14], X[15]);
            } else {
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    u32 s = 16u * c;
                    if (s < mlen) {
                        u32 nb = mlen - s;
                        if (nb >= 16)
                            st16<AL>(out + s, X[4 * c], X[4 * c + 1], X[4 * c + 2], X[4 * c + 3]);
                        else
                            st_bytes(out + s, X[4 * c], X[4 * c + 1], X[4 * c + 2], X[4 * c + 3], nb);
                    }
                }
            }
        }
    }

    for (u32 blk = 1; blk < nfull; blk++) {
        const uint8_t *src = in + 64u * blk;
        V4 q0 = ld16f<AL>(src), q1 = ld16f<AL>(src + 16), q2 = ld16f<AL>(src + 32), q3 = ld16f<AL>(src + 48);
        salsa20_block(x, key, n0, n1, blk, 0u);
        C[0] = q0.x; C[1] = q0.y; C[2] = q0.z; C[3] = q0.w;
        C[4] = q1.x; C[5] = q1.y; C[6] = q1.z; C[7] = q1.w;
        C[8] = q2.x; C[9] = q2.y; C[10] = q2.z; C[11] = q2.w;
        C[12] = q3.x; C[13] = q3.y; C[14] = q3.z; C[15] = q3.w;
        poly_block(P, C[0], C[1], C[2], C[3], 1u);
        poly_block(P, C[4], C[5], C[6], C[7], 1u);
        poly_block(P, C[8], C[9], C[10], C[11], 1u);
        poly_block(P, C[12], C[13], C[14], C[15], 1u);
#pragma unroll
        for (int k = 0; k < 16; k++)
            X[k] = C[k] ^ x[k];
        if constexpr (MODE == MODE_ZMQ) {
            emit_zmq(blk, X, false);
        } else {
            uint8_t *dst = out + 64u * blk;
            st16<AL>(dst, X[0], X[1], X[2], X[3]);
            st16<AL>(dst + 16, X[4], X[5], X[6], X[7]);
            st16<AL>(dst + 32, X[8], X[9], X[10], X[11]);
            st16<AL>(dst + 48, X[12], X[13], X[14], X[15]);
        }
    }

    u32 total_blocks = nfull;
    if (tailv != 0 && nfull >= 1) {
        const u32 blk = nfull;
        const uint8_t *src = in + 64u * blk;
        V4 q[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            u32 o = 64u * blk + 16u * c;
            q[c] = ld16<AL>(src + 16 * c, o < size ? size - o : 0);
        }
        salsa20_block(x, key, n0, n1, blk, 0u);
        u32 Q[16] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w,
                     q[2].x, q[2].y, q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w};
        emit_guarded<AL>(P, Q, 0, tailv, nullptr, false);
#pragma unroll
        for (int k = 0; k < 16; k++)
            X[k] = Q[k] ^ x[k];
        if constexpr (MODE == MODE_ZMQ) {
            emit_zmq(blk, X, true);
        } else {
            uint8_t *dst = out + 64u * blk;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                u32 s = 16u * c;
                if (s < tailv) {
                    u32 nb = tailv - s;
                    if (nb >= 16)
                        st16<AL>(dst + s, X[4 * c], X[4 * c + 1], X[4 * c + 2], X[4 * c + 3]);
                    else
                        st_bytes(dst + s, X[4 * c], X[4 * c + 1], X[4 * c + 2], X[4 * c + 3], nb);
                }
            }
        }
        total_blocks = nfull + 1;
    } else if (nfull == 0) {
        total_blocks = 1;
    }
    if constexpr (MODE == MODE_ZMQ) {
        // flush: payload bytes [64B-48, 64B+16) from the carry (D beyond the box are zero)
        u32 Z[16] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        emit_zmq(total_blocks, Z, true);
    }

    u32 tag[4];
    poly_finish(P, tag);
    u32 diff = (tag[0] ^ tin.x) | (tag[1] ^ tin.y) | (tag[2] ^ tin.z) | (tag[3] ^ tin.w);
    if (diff != 0) {
        // never release unauthenticated plaintext
        for (u32 o = 0; o < nout; o += 16) {
            u32 nb = nout - o < 16 ? nout - o : 16;
            if (nb == 16)
                st16<AL>(out + o, 0u, 0u, 0u, 0u);
            else
                st_bytes(out + o, 0u, 0u, 0u, 0u, nb);
        }
        return CZ_STATUS_CRYPTO;
    }
    return CZ_STATUS_OK;
}

__device__ __forceinline__ void load_key(const uint8_t *__restrict__ p, u32 k[8])
{
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 a = q[0], b = q[1];
    k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
    k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
}

__device__ __forceinline__ bool aligned16(const void *a, const void *b)
{
    return (((uintptr_t)a | (uintptr_t)b) & 15u) == 0;
}

// ---- kernels -------------------------------------------------------------

constexpr int BLOCK = 256;

// Uniform batch: frame i = in[i*in_stride .. +len) -> out[i*out_stride .. +len+33),
// nonce counter = counter0 + i, flags = flags8 ? flags8[i] : 0, one subkey.
__global__ __launch_bounds__(BLOCK) void k_seal_uniform(const uint8_t *__restrict__ in, uint64_t in_stride,
                                                         uint8_t *__restrict__ out, uint64_t out_stride,
                                                         uint32_t count, uint32_t len,
                                                         const uint8_t *__restrict__ subkey, uint64_t counter0,
                                                         const uint8_t *__restrict__ flags8)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= count)
        return;
    u32 key[8];
    load_key(subkey, key);
    const uint8_t *src = in + (uint64_t)i * in_stride;
    uint8_t *dst = out + (uint64_t)i * out_stride;
    const u32 fl = flags8 ? flags8[i] : 0u;
    if (aligned16(src, dst))
        seal_frame<MODE_ZMQ, true>(src, dst, len, fl, counter0 + i, key);
    else
        seal_frame<MODE_ZMQ, false>(src, dst, len, fl, counter0 + i, key);
}

__global__ __launch_bounds__(BLOCK) void k_seal_desc(const cz_frame_desc *__restrict__ desc,
                                                      const uint32_t *__restrict__ order, uint32_t count,
                                                      const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                      const uint8_t *__restrict__ subkeys)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= count)
        return;
    const uint32_t i = order ? order[t] : t;
    const cz_frame_desc d = desc[i];
    u32 key[8];
    load_key(subkeys + 32ull * d.key_idx, key);
    const uint8_t *src = in + d.in_off;
    uint8_t *dst = out + d.out_off;
    if (aligned16(src, dst))
        seal_frame<MODE_ZMQ, true>(src, dst, d.len, d.flags & 0xffu, d.counter, key);
    else
        seal_frame<MODE_ZMQ, false>(src, dst, d.len, d.flags & 0xffu, d.counter, key);
}

// status[i] = CZ_STATUS_* | (flags byte << 8)
__global__ __launch_bounds__(BLOCK) void k_open_desc(const cz_frame_desc *__restrict__ desc,
                                                      const uint32_t *__restrict__ order, uint32_t count,
                                                      const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                      const uint8_t *__restrict__ subkeys,
                                                      uint16_t *__restrict__ status, uint64_t *__restrict__ nonces)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= count)
        return;
    const uint32_t i = order ? order[t] : t;
    const cz_frame_desc d = desc[i];
    u32 key[8];
    load_key(subkeys + 32ull * d.key_idx, key);
    long long floor = (long long)d.counter;
    if (d.prev >= 0) {
        // replay floor = nonce of the previous frame of this connection in the batch
        const cz_frame_desc p = desc[d.prev];
        const uint8_t *pb = in + p.in_off + 8;
        u64 v = 0;
        for (int b = 0; b < 8; b++)
            v = (v << 8) | pb[b];
        floor = (long long)v;
    }
    const bool check = (d.flags & CZ_DESC_CHECK_NONCE) != 0;
    const uint8_t *src = in + d.in_off;
    uint8_t *dst = out + d.out_off;
    u32 fl = 0;
    u64 nonce = 0;
    u32 st;
    if (aligned16(src, dst))
        st = open_frame<MODE_ZMQ, true>(src, dst, d.len, key, check, floor, &fl, &nonce, 0);
    else
        st = open_frame<MODE_ZMQ, false>(src, dst, d.len, key, check, floor, &fl, &nonce, 0);
    status[i] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
    if (nonces)
        nonces[i] = nonce;
}

__global__ __launch_bounds__(BLOCK) void k_open_uniform(const uint8_t *__restrict__ in, uint64_t in_stride,
                                                         uint8_t *__restrict__ out, uint64_t out_stride,
                                                         uint32_t count, uint32_t size,
                                                         const uint8_t *__restrict__ subkey, uint64_t floor0,
                                                         int check, uint16_t *__restrict__ status)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= count)
        return;
    u32 key[8];
    load_key(subkey, key);
    const uint8_t *src = in + (uint64_t)i * in_stride;
    uint8_t *dst = out + (uint64_t)i * out_stride;
    // frames of one connection in order: frame i must beat frame i-1's nonce
    long long floor = (long long)floor0;
    if (i > 0) {
        const uint8_t *pb = src - in_stride + 8;
        u64 v = 0;
        for (int b = 0; b < 8; b++)
            v = (v << 8) | pb[b];
        floor = (long long)v;
    }
    u32 fl = 0;
    u64 nonce = 0;
    u32 st;
    if (aligned16(src, dst))
        st = open_frame<MODE_ZMQ, true>(src, dst, size, key, check != 0, floor, &fl, &nonce, 0);
    else
        st = open_frame<MODE_ZMQ, false>(src, dst, size, key, check != 0, floor, &fl, &nonce, 0);
    status[i] = (uint16_t)(st | (st == CZ_STATUS_OK ? (fl << 8) : 0u));
}

// NaCl-layout single frame (jnacl crypto_box_afternm / crypto_box_open_afternm drop-in).
// params: subkey (32 B device), counter = BE64(n[16:24]).
__global__ __launch_bounds__(64) void k_box_nacl(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                  uint32_t len, const uint8_t *__restrict__ subkey,
                                                  uint64_t counter, int open, int *__restrict__ rc)
{
    if (threadIdx.x != 0 || blockIdx.x != 0)
        return;
    u32 key[8];
    load_key(subkey, key);
    if (!open) {
        if (len < 32u) {
            *rc = -1;
            return;
        }
        if (aligned16(in, out))
            seal_frame<MODE_NACL, true>(in, out, len, 0u, counter, key);
        else
            seal_frame<MODE_NACL, false>(in, out, len, 0u, counter, key);
        *rc = 0;
    } else {
        u32 fl;
        u64 nonce;
        u32 st;
        if (aligned16(in, out))
            st = open_frame<MODE_NACL, true>(in, out, len, key, false, 0, &fl, &nonce, counter);
        else
            st = open_frame<MODE_NACL, false>(in, out, len, key, false, 0, &fl, &nonce, counter);
        *rc = st == CZ_STATUS_OK ? 0 : -1;
    }
}

// subkeys[i] = HSalsa20(precom[i], prefix16)
__global__ __launch_bounds__(BLOCK) void k_subkeys(const uint8_t *__restrict__ precom, uint8_t *__restrict__ out,
                                                    uint32_t nkeys, uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3)
{
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= nkeys)
        return;
    u32 k[8], o[8];
    const uint8_t *kp = precom + 32ull * i;
    for (int w = 0; w < 8; w++)
        k[w] = (u32)kp[4 * w] | ((u32)kp[4 * w + 1] << 8) | ((u32)kp[4 * w + 2] << 16) | ((u32)kp[4 * w + 3] << 24);
    const u32 in4[4] = {p0, p1, p2, p3};
    hsalsa20(o, k, in4);
    uint8_t *op = out + 32ull * i;
    for (int w = 0; w < 8; w++)
        for (int b = 0; b < 4; b++)
            op[4 * w + b] = (uint8_t)(o[w] >> (8 * b));
}

// Synthetic payload generator: counter-based SplitMix64 words (tests/cz_testlib.py splitmix_words).
__device__ __forceinline__ u64 splitmix(u64 seed, u64 idx)
{
    u64 z = seed + (idx + 1ull) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(BLOCK) void k_fill(uint8_t *__restrict__ buf, uint64_t nbytes, uint64_t seed)
{
    const uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;  // 16-byte chunk index
    const uint64_t off = w * 16;
    if (off >= nbytes)
        return;
    u64 a = splitmix(seed, 2 * w), b = splitmix(seed, 2 * w + 1);
    if (off + 16 <= nbytes) {
        *reinterpret_cast<uint4 *>(buf + off) = make_uint4((u32)a, (u32)(a >> 32), (u32)b, (u32)(b >> 32));
    } else {
        for (uint64_t i = 0; off + i < nbytes; i++)
            buf[off + i] = (uint8_t)((i < 8 ? a >> (8 * i) : b >> (8 * (i - 8))));
    }
}

// Lay out uniform-length frames into a packed strided layout (tests / host staging).
}  // namespace

// ---------------------------------------------------------------------------
// Launchers (called from cz_host.cpp).  No allocation, no synchronisation:
// safe to capture in a hipGraph.
// ---------------------------------------------------------------------------
extern "C" {

hipError_t czk_seal_uniform(const void *in, uint64_t in_stride, void *out, uint64_t out_stride, uint32_t count,
                            uint32_t len, const void *subkey, uint64_t counter0, const uint8_t *flags8,
                            hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_seal_uniform, grid, dim3(BLOCK), 0, s, (const uint8_t *)in, in_stride, (uint8_t *)out,
                       out_stride, count, len, (const uint8_t *)subkey, counter0, flags8);
    return hipGetLastError();
}

hipError_t czk_seal_desc(const cz_frame_desc *desc, const uint32_t *order, uint32_t count, const void *in, void *out,
                         const void *subkeys, hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_seal_desc, grid, dim3(BLOCK), 0, s, desc, order, count, (const uint8_t *)in,
                       (uint8_t *)out, (const uint8_t *)subkeys);
    return hipGetLastError();
}

hipError_t czk_open_desc(const cz_frame_desc *desc, const uint32_t *order, uint32_t count, const void *in, void *out,
                         const void *subkeys, uint16_t *status, uint64_t *nonces, hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_open_desc, grid, dim3(BLOCK), 0, s, desc, order, count, (const uint8_t *)in,
                       (uint8_t *)out, (const uint8_t *)subkeys, status, nonces);
    return hipGetLastError();
}

hipError_t czk_open_uniform(const void *in, uint64_t in_stride, void *out, uint64_t out_stride, uint32_t count,
                            uint32_t size, const void *subkey, uint64_t floor0, int check, uint16_t *status,
                            hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    dim3 grid((count + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_open_uniform, grid, dim3(BLOCK), 0, s, (const uint8_t *)in, in_stride, (uint8_t *)out,
                       out_stride, count, size, (const uint8_t *)subkey, floor0, check, status);
    return hipGetLastError();
}

hipError_t czk_box_nacl(const void *in, void *out, uint32_t len, const void *subkey, uint64_t counter, int open,
                        int *rc, hipStream_t s)
{
    hipLaunchKernelGGL(k_box_nacl, dim3(1), dim3(64), 0, s, (const uint8_t *)in, (uint8_t *)out, len,
                       (const uint8_t *)subkey, counter, open, rc);
    return hipGetLastError();
}

hipError_t czk_subkeys(const void *precom, void *out, uint32_t nkeys, const uint8_t prefix[16], hipStream_t s)
{
    if (nkeys == 0)
        return hipSuccess;
    u32 p[4];
    for (int w = 0; w < 4; w++)
        p[w] = (u32)prefix[4 * w] | ((u32)prefix[4 * w + 1] << 8) | ((u32)prefix[4 * w + 2] << 16) |
               ((u32)prefix[4 * w + 3] << 24);
    dim3 grid((nkeys + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_subkeys, grid, dim3(BLOCK), 0, s, (const uint8_t *)precom, (uint8_t *)out, nkeys, p[0], p[1],
                       p[2], p[3]);
    return hipGetLastError();
}

hipError_t czk_fill(void *buf, uint64_t nbytes, uint64_t seed, hipStream_t s)
{
    if (nbytes == 0)
        return hipSuccess;
    uint64_t chunks = (nbytes + 15) / 16;
    dim3 grid((unsigned)((chunks + BLOCK - 1) / BLOCK));
    hipLaunchKernelGGL(k_fill, grid, dim3(BLOCK), 0, s, (uint8_t *)buf, nbytes, seed);
    return hipGetLastError();
}

}  // extern "C"
