// cz_device.h -- CDNA4 (gfx950) device primitives for the CurveZMQ MESSAGE path.
//
// The arithmetic is the NaCl crypto_box_afternm construction that JeroMQ calls
// through jnacl (Curve.java:129-147 -> curve25519xsalsa20poly1305.crypto_box_afternm):
// Salsa20/20 keystream (HSalsa20-derived subkey) XOR + Poly1305 over c[32:mlen].
// Everything here is plain 32-bit integer VALU work: v_add_u32 / v_alignbit_b32
// (rotates) / v_xor_b32 for Salsa20, v_mad_u64_u32 chains for Poly1305 in a
// 2^32 radix.  No MFMA: the path is a stream cipher + a 130-bit MAC.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cz_salsa_lazy.h"
#include "cz_salsa_tail.h"

namespace cz {

typedef uint32_t u32;
typedef uint64_t u64;

// "expand 32-byte k"
constexpr u32 SIGMA0 = 0x61707865u, SIGMA1 = 0x3320646eu, SIGMA2 = 0x79622d32u, SIGMA3 = 0x6b206574u;

__device__ __forceinline__ u32 rotl(u32 v, int c) { return __builtin_amdgcn_alignbit(v, v, 32 - c); }

__device__ __forceinline__ void qr(u32 &a, u32 &b, u32 &c, u32 &d)
{
    b ^= rotl(a + d, 7);
    c ^= rotl(b + a, 9);
    d ^= rotl(c + b, 13);
    a ^= rotl(d + c, 18);
}

__device__ __forceinline__ void col_round(u32 x[16])
{
    qr(x[0], x[4], x[8], x[12]);
    qr(x[5], x[9], x[13], x[1]);
    qr(x[10], x[14], x[2], x[6]);
    qr(x[15], x[3], x[7], x[11]);
}

__device__ __forceinline__ void row_round(u32 x[16])
{
    qr(x[0], x[1], x[2], x[3]);
    qr(x[5], x[6], x[7], x[4]);
    qr(x[10], x[11], x[8], x[9]);
    qr(x[15], x[12], x[13], x[14]);
}

// rotl of a WAVE-UNIFORM value on the scalar unit.  Left to itself the compiler rotates
// uniform values with v_alignbit_b32 (there is no scalar rotate), which moves everything
// downstream to the VALU; 3 SALU instructions cost the VALU nothing.  Only call with
// values that are the same in every lane: an "s" operand of a divergent value would be
// silently narrowed to lane 0.
template <int C>
__device__ __forceinline__ u32 srotl(u32 v)
{
    u32 r, t;
    asm("s_lshl_b32 %0, %2, %3\n\ts_lshr_b32 %1, %2, %4\n\ts_or_b32 %0, %0, %1"
        : "=&s"(r), "=&s"(t)
        : "s"(v), "i"(C), "i"(32 - C)
        : "scc");
    return r;
}

// Rounds 1-2 when the key, the block counter and nonce word 6 are wave-uniform and only
// word 7 (the low counter word of a MESSAGE nonce) differs per lane (the UN0 kernels).
// Round 1's quarter-rounds B, C, D do not depend on the block counter: salsa_frame()
// runs them once per frame.  Per block, what depends on the block counter and is
// wave-uniform -- round 1's A, round 2's A and the first step of round 2's B -- rotates on
// the scalar unit (srotl); the per-lane rest is ~24 VALU.
struct SalsaFrame {
    u32 w[16];  // state after round 1's quarter-rounds B, C, D (words 0, 4, 8, 12 unused)
};

__device__ __forceinline__ SalsaFrame salsa_frame(const u32 k[8], u32 n0, u32 n1)
{
    u32 x[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1, 0u, 0u, SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
    x[9] ^= srotl<7>(x[5] + x[1]);   x[13] ^= srotl<9>(x[9] + x[5]);
    x[1] ^= srotl<13>(x[13] + x[9]); x[5] ^= srotl<18>(x[1] + x[13]);
    x[14] ^= srotl<7>(x[10] + x[6]); x[2] ^= srotl<9>(x[14] + x[10]);
    x[6] ^= srotl<13>(x[2] + x[14]); x[10] ^= srotl<18>(x[6] + x[2]);
    x[3] ^= srotl<7>(x[15] + x[11]); x[7] ^= srotl<9>(x[3] + x[15]);   // x7 per-lane from here
    x[11] ^= rotl(x[7] + x[3], 13);  x[15] ^= rotl(x[11] + x[7], 18);
    SalsaFrame f;
#pragma unroll
    for (int i = 0; i < 16; i++)
        f.w[i] = x[i];
    return f;
}

// rounds 1-2 of block c0 (block counter high word 0) from the frame's precomputed words
__device__ __forceinline__ void rounds12_frame(u32 x[16], const SalsaFrame &f, u32 c0, const u32 k[8])
{
#pragma unroll
    for (int i = 0; i < 16; i++)
        x[i] = f.w[i];
    x[0] = SIGMA0; x[4] = k[3]; x[8] = c0; x[12] = k[5];
    x[4] ^= srotl<7>(x[0] + x[12]);  x[8] ^= srotl<9>(x[4] + x[0]);
    x[12] ^= srotl<13>(x[8] + x[4]); x[0] ^= srotl<18>(x[12] + x[8]);
    // round 2 (rows)
    x[1] ^= srotl<7>(x[0] + x[3]);   x[2] ^= srotl<9>(x[1] + x[0]);
    x[3] ^= srotl<13>(x[2] + x[1]);  x[0] ^= srotl<18>(x[3] + x[2]);
    x[6] ^= srotl<7>(x[5] + x[4]);   x[7] ^= srotl<9>(x[6] + x[5]);
    x[4] ^= rotl(x[7] + x[6], 13);   x[5] ^= rotl(x[4] + x[7], 18);
    x[11] ^= rotl(x[10] + x[9], 7);  x[8] ^= rotl(x[11] + x[10], 9);
    x[9] ^= rotl(x[8] + x[11], 13);  x[10] ^= rotl(x[9] + x[8], 18);
    x[12] ^= rotl(x[15] + x[14], 7); x[13] ^= rotl(x[12] + x[15], 9);
    x[14] ^= rotl(x[13] + x[12], 13); x[15] ^= rotl(x[14] + x[13], 18);
}

// The 20 Salsa20 rounds with LAZY XORS (cz_salsa_lazy.h, generated and self-checked by
// tools/gen_salsa_lazy.py).  Every int32 VALU instruction costs its SIMD 4 cycles on gfx950
// whatever the opcode (tools/diag/salsa_ub.hip), so a block costs its instruction count.
// Rounds 1-2 stay in C: with the key, constants, block counter and high nonce word
// wave-uniform, the compiler moves 3 of round 1's quarter-rounds (and part of round 2) to
// the scalar unit and reads uniform words as SGPR operands.  Rounds 3..20 keep most
// `w ^= R` updates pending and let v_xad_u32 ((a ^ b) + c) and v_bitop3_b32 (a ^ b ^ c)
// absorb them: 736 VALU instead of 864.  On return word w is x[w] ^ d[w] for the bits of
// CZ_LAZY_PENDING, x[w] otherwise.
// R12: rounds 1-2 already done by the caller (rounds12_frame).
static_assert(CZ_LAZY_FIRST_ROUND == 3, "rounds_lazy runs rounds 1-2 in C");
template <bool R12 = false>
__device__ __forceinline__ void rounds_lazy(u32 x[16], u32 d[16])
{
    if constexpr (!R12) {
        col_round(x);
        row_round(x);
    }
    u32 t0, t1, t2, t3;
    asm(CZ_SALSA_LAZY_ASM
        : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
          "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]),
          "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]),
          "=&v"(d[8]), "=&v"(d[9]), "=&v"(d[10]), "=&v"(d[11]), "=&v"(d[12]), "=&v"(d[13]), "=&v"(d[14]),
          "=&v"(d[15]), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3));
}

__device__ __forceinline__ constexpr bool lazy_pending(int k) { return (CZ_LAZY_PENDING >> k) & 1u; }

// The 20 rounds with plain xors (compiler-scheduled).
__device__ __forceinline__ void rounds_eager(u32 x[16])
{
#pragma unroll
    for (int i = 0; i < 10; i++) {
        col_round(x);
        row_round(x);
    }
}

// One Salsa20/20 block: key k[8] (LE words), nonce words n0,n1 (LE loads of
// nonce bytes 16..23 of the XSalsa20 nonce), 64-bit block counter c0|c1.
// LAZY: rounds_lazy, whose pending deltas the feed-forward add absorbs (v_xad_u32).
// The lane-per-frame descriptor kernels take the plain rounds: on their ragged,
// tail-latency-bound batches the lazy core measured 9% slower.
template <bool LAZY = true>
__device__ __forceinline__ void salsa20_block(u32 x[16], const u32 k[8], u32 n0, u32 n1, u32 c0, u32 c1)
{
    const u32 in[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1, c0, c1, SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
#pragma unroll
    for (int i = 0; i < 16; i++)
        x[i] = in[i];
    if constexpr (LAZY) {
        u32 d[16];
        rounds_lazy(x, d);
#pragma unroll
        for (int i = 0; i < 16; i++)
            x[i] = lazy_pending(i) ? ((x[i] ^ d[i]) + in[i]) : (x[i] + in[i]);
    } else {
        rounds_eager(x);
#pragma unroll
        for (int i = 0; i < 16; i++)
            x[i] += in[i];
    }
}

// The same block in a UN0 kernel (key, n0 and the block counter wave-uniform; c1 = 0),
// rounds 1-2 from the frame's precomputed words (salsa_frame).
__device__ __forceinline__ void salsa20_block_frame(u32 x[16], const SalsaFrame &f, const u32 k[8], u32 n0, u32 n1,
                                                    u32 c0)
{
    const u32 in[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1, c0, 0u, SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
    u32 d[16];
    rounds12_frame(x, f, c0, k);
    rounds_lazy<true>(x, d);
#pragma unroll
    for (int i = 0; i < 16; i++)
        x[i] = lazy_pending(i) ? ((x[i] ^ d[i]) + in[i]) : (x[i] + in[i]);
}

// The last block of a box that uses at most 16 of its bytes (a 100-byte MESSAGE: 133-byte box, 5
// bytes of block 2): keystream words 0..3 only.  Rounds 3..20 run the tail schedule
// (cz_salsa_tail.h: the instructions words 0..3 depend on, 692 instead of 736) and the
// feed-forward covers 4 words; x[4..15] are left unspecified.
__device__ __forceinline__ void tail_lazy(u32 x[16], u32 d[16])
{
    u32 t0, t1, t2, t3;
    asm(CZ_SALSA_TAIL_ASM
        : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
          "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]),
          "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]),
          "=&v"(d[8]), "=&v"(d[9]), "=&v"(d[10]), "=&v"(d[11]), "=&v"(d[12]), "=&v"(d[13]), "=&v"(d[14]),
          "=&v"(d[15]), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3));
}
static_assert(CZ_SALSA_TAIL_WORDS == 4, "tail blocks use keystream words 0..3");

template <bool LAZY = true>
__device__ __forceinline__ void salsa20_block_w03(u32 x[16], const u32 k[8], u32 n0, u32 n1, u32 c0, u32 c1)
{
    const u32 in[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1, c0, c1, SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
#pragma unroll
    for (int i = 0; i < 16; i++)
        x[i] = in[i];
    if constexpr (LAZY) {
        u32 d[16];
        col_round(x);
        row_round(x);
        tail_lazy(x, d);
#pragma unroll
        for (int i = 0; i < 4; i++)
            x[i] = lazy_pending(i) ? ((x[i] ^ d[i]) + in[i]) : (x[i] + in[i]);
    } else {
        rounds_eager(x);
#pragma unroll
        for (int i = 0; i < 4; i++)
            x[i] += in[i];
    }
}

__device__ __forceinline__ void salsa20_block_frame_w03(u32 x[16], const SalsaFrame &f, const u32 k[8], u32 n0, u32 n1,
                                                        u32 c0)
{
    const u32 in[4] = {SIGMA0, k[0], k[1], k[2]};
    u32 d[16];
    rounds12_frame(x, f, c0, k);
    tail_lazy(x, d);
#pragma unroll
    for (int i = 0; i < 4; i++)
        x[i] = lazy_pending(i) ? ((x[i] ^ d[i]) + in[i]) : (x[i] + in[i]);
    (void)n0, (void)n1;
}

// HSalsa20(k, in16) -> out[8]: no feed-forward, words 0,5,10,15,6,7,8,9.
__device__ __forceinline__ void hsalsa20(u32 out[8], const u32 k[8], const u32 in[4])
{
    u32 x[16], d[16];
    x[0] = SIGMA0; x[1] = k[0]; x[2] = k[1]; x[3] = k[2];
    x[4] = k[3]; x[5] = SIGMA1; x[6] = in[0]; x[7] = in[1];
    x[8] = in[2]; x[9] = in[3]; x[10] = SIGMA2; x[11] = k[4];
    x[12] = k[5]; x[13] = k[6]; x[14] = k[7]; x[15] = SIGMA3;
    rounds_lazy(x, d);
    constexpr int w[8] = {0, 5, 10, 15, 6, 7, 8, 9};
#pragma unroll
    for (int i = 0; i < 8; i++)
        out[i] = lazy_pending(w[i]) ? (x[w[i]] ^ d[w[i]]) : x[w[i]];
}

// ---- Poly1305, radix 2^32 ------------------------------------------------
// h = h4:h3:h2:h1:h0 (h4 small), r clamped so that r1..r3 have their two low
// bits clear, hence 2^128 * r_i == (5/4) r_i (mod p) and s_i = r_i + r_i/4 is
// exact.  Per 16-byte block: 16 + 3 v_mad_u64_u32, one v_mul_lo_u32, and the
// carry chain.  Bounds: h0..h3 < 2^32, h4 <= 6, r_i < 2^28, s_i < 1.25*2^28,
// so each 4-term product column is < 2^62.4 and fits a u64.
struct Poly {
    u32 h0, h1, h2, h3, h4;
    u32 r0, r1, r2, r3;
    u32 s1, s2, s3;
    u32 p0, p1, p2, p3;
};

// key = keystream words 0..7 of block 0 (r = words 0..3 clamped, pad = 4..7)
__device__ __forceinline__ void poly_init(Poly &P, u32 k0, u32 k1, u32 k2, u32 k3, u32 k4, u32 k5, u32 k6, u32 k7)
{
    P.r0 = k0 & 0x0fffffffu;
    P.r1 = k1 & 0x0ffffffcu;
    P.r2 = k2 & 0x0ffffffcu;
    P.r3 = k3 & 0x0ffffffcu;
    P.s1 = P.r1 + (P.r1 >> 2);
    P.s2 = P.r2 + (P.r2 >> 2);
    P.s3 = P.r3 + (P.r3 >> 2);
    P.p0 = k4; P.p1 = k5; P.p2 = k6; P.p3 = k7;
    P.h0 = P.h1 = P.h2 = P.h3 = P.h4 = 0;
}

__device__ __forceinline__ u32 addc(u32 a, u32 b, u32 cin, u32 &cout)
{
    return __builtin_addc(a, b, cin, &cout);
}

__device__ __forceinline__ u64 mad64(u32 a, u32 b, u64 c) { return (u64)a * b + c; }

// h = (h + m + hibit*2^128) * r  (partially reduced).  Written as explicit 32-bit
// carry chains (v_add_co_u32 / v_addc_co_u32) around 19 v_mad_u64_u32: the plain
// u64 formulation compiled to zero-extension moves and 64-bit adds.
__device__ __forceinline__ void poly_block(Poly &P, u32 m0, u32 m1, u32 m2, u32 m3, u32 hibit)
{
    u32 c;
    const u32 h0 = addc(P.h0, m0, 0u, c);
    const u32 h1 = addc(P.h1, m1, c, c);
    const u32 h2 = addc(P.h2, m2, c, c);
    const u32 h3 = addc(P.h3, m3, c, c);
    const u32 h4 = P.h4 + c + hibit;

    const u64 d0 = mad64(h3, P.s1, mad64(h2, P.s2, mad64(h1, P.s3, mad64(h0, P.r0, 0))));
    const u64 d1 = mad64(h4, P.s1, mad64(h3, P.s2, mad64(h2, P.s3, mad64(h1, P.r0, mad64(h0, P.r1, 0)))));
    const u64 d2 = mad64(h4, P.s2, mad64(h3, P.s3, mad64(h2, P.r0, mad64(h1, P.r1, mad64(h0, P.r2, 0)))));
    const u64 d3 = mad64(h4, P.s3, mad64(h3, P.r0, mad64(h2, P.r1, mad64(h1, P.r2, mad64(h0, P.r3, 0)))));
    const u32 h4r = h4 * P.r0;  // the compiler fuses it with the add below (v_mad_u64_u32)

    // h = d0 + d1*2^32 + d2*2^64 + d3*2^96 + h4r*2^128, partially reduced with 2^130 == 5 in
    // ONE carry chain: the top word x = hi(d3) + h4r (< 2^30.4 + 2^30.6, no overflow) is split
    // as 4q + (x & 3) before the column carries run, and 5q enters limb 0 with them:
    //   h = (lo(d0) + 5q) + (lo(d1) + hi(d0))*2^32 + (lo(d2) + hi(d1))*2^64
    //       + (lo(d3) + hi(d2))*2^96 + (x & 3)*2^128          (mod 2^130 - 5)
    // Each step is a + b + carry < 2^33, one v_addc_co_u32 with carry 0 or 1; the chain's last
    // carry lands in h4 <= 4, the same bound as folding after a separate column chain.  Bounds
    // and exactness: tests/test_poly_radix32.py.  Against the two-chain form: 17 VALU fewer per
    // 128-byte block pair in the 4k seal loop (1961 -> 1944).
    const u32 x = (u32)(d3 >> 32) + h4r;
    const u32 q = x >> 2;
    // k = 5q as one v_lshl_add_u32: left to itself the compiler emits (x & ~3) + q, two VALU
    u32 k;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(k) : "v"(q));
    P.h0 = addc((u32)d0, k, 0u, c);
    P.h1 = addc((u32)d1, (u32)(d0 >> 32), c, c);
    P.h2 = addc((u32)d2, (u32)(d1 >> 32), c, c);
    P.h3 = addc((u32)d3, (u32)(d2 >> 32), c, c);
    P.h4 = (x & 3u) + c;
}

// Final block of len bytes (1..15): bytes >= len cleared, byte len = 0x01, no 2^128 bit.
__device__ __forceinline__ void poly_block_partial(Poly &P, u32 m0, u32 m1, u32 m2, u32 m3, u32 len)
{
    u32 m[4] = {m0, m1, m2, m3};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int rel = (int)len - 4 * i;  // bytes of this dword that are message
        u32 keep = rel >= 4 ? 0xffffffffu : (rel <= 0 ? 0u : ((1u << (8 * rel)) - 1u));
        u32 one = (rel >= 0 && rel < 4) ? (1u << (8 * rel)) : 0u;
        m[i] = (m[i] & keep) | one;
    }
    poly_block(P, m[0], m[1], m[2], m[3], 0u);
}

// tag = (h mod p + pad) mod 2^128
__device__ __forceinline__ void poly_finish(const Poly &P, u32 tag[4])
{
    u32 h0 = P.h0, h1 = P.h1, h2 = P.h2, h3 = P.h3, h4 = P.h4;
    u64 t;
    u32 c = (h4 >> 2) * 5u;
    h4 &= 3u;
    t = (u64)h0 + c; h0 = (u32)t;
    t = (u64)h1 + (t >> 32); h1 = (u32)t;
    t = (u64)h2 + (t >> 32); h2 = (u32)t;
    t = (u64)h3 + (t >> 32); h3 = (u32)t;
    h4 += (u32)(t >> 32);
    // g = h + 5; if g >= 2^130 then h = g - 2^130
    t = (u64)h0 + 5u; u32 g0 = (u32)t;
    t = (u64)h1 + (t >> 32); u32 g1 = (u32)t;
    t = (u64)h2 + (t >> 32); u32 g2 = (u32)t;
    t = (u64)h3 + (t >> 32); u32 g3 = (u32)t;
    u32 g4 = h4 + (u32)(t >> 32);
    bool ge = (g4 >> 2) != 0;
    h0 = ge ? g0 : h0; h1 = ge ? g1 : h1; h2 = ge ? g2 : h2; h3 = ge ? g3 : h3;
    t = (u64)h0 + P.p0; tag[0] = (u32)t;
    t = (u64)h1 + P.p1 + (t >> 32); tag[1] = (u32)t;
    t = (u64)h2 + P.p2 + (t >> 32); tag[2] = (u32)t;
    t = (u64)h3 + P.p3 + (t >> 32); tag[3] = (u32)t;
}

// ---- general arithmetic mod p = 2^130 - 5, radix 2^26 -----------------------
// Used to combine the Poly1305 partials of a frame split into segments: the
// frame's accumulator is H = sum_s h_s * r^(m_{s+1} + ... + m_{S-1}), evaluated
// as a Horner chain over segments with multipliers r^m.  r^m is not clamped, so
// the 2^32-radix 5/4 trick does not apply; 26-bit limbs with 5*b_j < 2^29 do.
struct F26 {
    u32 l[5];
};

// from 32-bit limbs h0..h3 + small h4 (h < 2^131)
__device__ __forceinline__ F26 f26_from32(u32 h0, u32 h1, u32 h2, u32 h3, u32 h4)
{
    F26 a;
    a.l[0] = h0 & 0x3ffffffu;
    a.l[1] = ((h0 >> 26) | (h1 << 6)) & 0x3ffffffu;
    a.l[2] = ((h1 >> 20) | (h2 << 12)) & 0x3ffffffu;
    a.l[3] = ((h2 >> 14) | (h3 << 18)) & 0x3ffffffu;
    a.l[4] = (h3 >> 8) | (h4 << 24);
    return a;
}

// a * b mod p (partially reduced: limbs < 2^26 except l[1] < 2^26 + 2^6); inputs' limbs < 2^27
__device__ __forceinline__ F26 f26_mul(const F26 &a, const F26 &b)
{
    const u32 s1 = b.l[1] * 5u, s2 = b.l[2] * 5u, s3 = b.l[3] * 5u, s4 = b.l[4] * 5u;
    u64 d0 = (u64)a.l[0] * b.l[0] + (u64)a.l[1] * s4 + (u64)a.l[2] * s3 + (u64)a.l[3] * s2 + (u64)a.l[4] * s1;
    u64 d1 = (u64)a.l[0] * b.l[1] + (u64)a.l[1] * b.l[0] + (u64)a.l[2] * s4 + (u64)a.l[3] * s3 + (u64)a.l[4] * s2;
    u64 d2 = (u64)a.l[0] * b.l[2] + (u64)a.l[1] * b.l[1] + (u64)a.l[2] * b.l[0] + (u64)a.l[3] * s4 + (u64)a.l[4] * s3;
    u64 d3 = (u64)a.l[0] * b.l[3] + (u64)a.l[1] * b.l[2] + (u64)a.l[2] * b.l[1] + (u64)a.l[3] * b.l[0] + (u64)a.l[4] * s4;
    u64 d4 = (u64)a.l[0] * b.l[4] + (u64)a.l[1] * b.l[3] + (u64)a.l[2] * b.l[2] + (u64)a.l[3] * b.l[1] + (u64)a.l[4] * b.l[0];
    F26 r;
    d1 += d0 >> 26; r.l[0] = (u32)d0 & 0x3ffffffu;
    d2 += d1 >> 26; r.l[1] = (u32)d1 & 0x3ffffffu;
    d3 += d2 >> 26; r.l[2] = (u32)d2 & 0x3ffffffu;
    d4 += d3 >> 26; r.l[3] = (u32)d3 & 0x3ffffffu;
    u64 c = d4 >> 26; r.l[4] = (u32)d4 & 0x3ffffffu;
    u64 t = (u64)r.l[0] + c * 5u;
    r.l[0] = (u32)t & 0x3ffffffu;
    r.l[1] += (u32)(t >> 26);
    return r;
}

__device__ __forceinline__ F26 f26_add(const F26 &a, const F26 &b)
{
    F26 r;
    u32 c = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) {
        u32 v = a.l[i] + b.l[i] + c;
        r.l[i] = v & 0x3ffffffu;
        c = v >> 26;
    }
    u32 t = r.l[0] + c * 5u;
    r.l[0] = t & 0x3ffffffu;
    r.l[1] += t >> 26;
    return r;
}

// r^e (square and multiply; r^0 = 1)
__device__ __forceinline__ F26 f26_pow(const F26 &r, u32 e)
{
    if (e == 0u)
        return F26{{1u, 0u, 0u, 0u, 0u}};
    F26 acc = r, base = r;
    bool have = false;
    for (u32 bit = 0; e >> bit; bit++) {
        if (bit)
            base = f26_mul(base, base);
        if ((e >> bit) & 1u) {
            acc = have ? f26_mul(acc, base) : base;
            have = true;
        }
    }
    return acc;
}

// back to 32-bit limbs h0..h3 + small h4 (input for poly_finish)
__device__ __forceinline__ void f26_to32(const F26 &a, u32 &h0, u32 &h1, u32 &h2, u32 &h3, u32 &h4)
{
    u32 l0 = a.l[0], l1 = a.l[1], l2 = a.l[2], l3 = a.l[3], l4 = a.l[4], c;
    c = l1 >> 26; l1 &= 0x3ffffffu;
    l2 += c; c = l2 >> 26; l2 &= 0x3ffffffu;
    l3 += c; c = l3 >> 26; l3 &= 0x3ffffffu;
    l4 += c; c = l4 >> 26; l4 &= 0x3ffffffu;
    l0 += c * 5u; c = l0 >> 26; l0 &= 0x3ffffffu;
    l1 += c;
    h0 = l0 | (l1 << 26);
    h1 = (l1 >> 6) | (l2 << 20);
    h2 = (l2 >> 12) | (l3 << 14);
    h3 = (l3 >> 18) | (l4 << 8);
    h4 = l4 >> 24;
}

__device__ __forceinline__ u32 bswap32(u32 v) { return __builtin_bswap32(v); }

// Salsa20 nonce words for a CurveZMQ MESSAGE counter: the nonce tail is
// BE64(counter) (Wire.putUInt64, Wire.java:124-136) loaded as two LE words.
__device__ __forceinline__ void counter_nonce(u64 counter, u32 &n0, u32 &n1)
{
    n0 = bswap32((u32)(counter >> 32));
    n1 = bswap32((u32)counter);
}

}  // namespace cz
