// cz_x25519.hip -- X25519 and NaCl crypto_box_beforenm on gfx950 (the CURVE handshake's key agreement).
//
// Reference: Curve.beforenm / keypair / box / open (jeromq-core/.../curve/Curve.java:100-193) call
// jnacl's curve25519xsalsa20poly1305.crypto_box_{beforenm,keypair,,_open}; a CURVE handshake runs
// two beforenm per side (HELLO/WELCOME boxes use C'/S', INITIATE's vouch uses C/S':
// CurveClientMechanism.java:246-419, CurveServerMechanism.java:254-507), and the MESSAGE key
// cnPrecom = beforenm(peer', our') (CurveClientMechanism.java:310).
//
// Algorithm: RFC 7748 section 5 -- clamped scalar, u masked to 255 bits, Montgomery ladder with
// a24 = 121665 and constant-time (masked) swaps, then x2 * z2^(p-2).  One lane per scalar
// multiplication: each lane's ladder is 255 serial steps of ~10 field multiplications, so a
// batch of independent key agreements (connection churn) fills the chip with no cross-lane work.
//
// Field arithmetic mod p = 2^255 - 19 in radix 2^25.5: 10 u32 limbs of 26/25 bits (limb i at bit
// ceil(25.5 i)).  A product is 100 v_mad_u64_u32 into u64 column sums; an odd*odd limb pair gains
// a factor 2 and a column >= 10 wraps with factor 19 (2^255 = 19 mod p).  Inputs to mul are kept
// below 2^27 per limb, so 19*g < 2^32 and each column stays below 2^63.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cz_device.h"

namespace {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr u32 M26 = (1u << 26) - 1;
constexpr u32 M25 = (1u << 25) - 1;

struct Fe {
    u32 v[10];
};

__device__ __forceinline__ u32 lw(int i) { return (i & 1) ? 25u : 26u; }

// u64 column sums -> carried limbs (limb 1 may exceed 25 bits by a few units; harmless for mul)
__device__ __forceinline__ void fe_carry(Fe &o, u64 h[10])
{
    u64 c;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        c = h[i] >> lw(i);
        h[i] &= (i & 1) ? M25 : M26;
        h[i + 1] += c;
    }
    c = h[9] >> 25;
    h[9] &= M25;
    h[0] += c * 19u;
    c = h[0] >> 26;
    h[0] &= M26;
    h[1] += c;
#pragma unroll
    for (int i = 0; i < 10; i++)
        o.v[i] = (u32)h[i];
}

// 32-bit carry pass for limbs below 2^31 (after add/sub)
__device__ __forceinline__ void fe_carry32(Fe &f)
{
    u32 c;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        c = f.v[i] >> lw(i);
        f.v[i] &= (i & 1) ? M25 : M26;
        f.v[i + 1] += c;
    }
    c = f.v[9] >> 25;
    f.v[9] &= M25;
    f.v[0] += c * 19u;
    c = f.v[0] >> 26;
    f.v[0] &= M26;
    f.v[1] += c;
}

__device__ __forceinline__ void fe_add(Fe &h, const Fe &f, const Fe &g)
{
#pragma unroll
    for (int i = 0; i < 10; i++)
        h.v[i] = f.v[i] + g.v[i];
}

// h = f - g + 2p, carried (f, g carried: limbs <= 2^26 + small)
__device__ __forceinline__ void fe_sub(Fe &h, const Fe &f, const Fe &g)
{
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const u32 p2 = i == 0 ? 2u * (M26 - 18u) : ((i & 1) ? 2u * M25 : 2u * M26);
        h.v[i] = f.v[i] + p2 - g.v[i];
    }
    fe_carry32(h);
}

__device__ __forceinline__ void fe_mul(Fe &o, const Fe &f, const Fe &g)
{
    u32 g19[10], f2[10];
#pragma unroll
    for (int j = 0; j < 10; j++)
        g19[j] = 19u * g.v[j];
#pragma unroll
    for (int i = 0; i < 10; i++)
        f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
    u64 h[10];
#pragma unroll
    for (int k = 0; k < 10; k++)
        h[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const int k = i + j;
            const u32 a = (i & 1) && (j & 1) ? f2[i] : f.v[i];
            const u32 b = k >= 10 ? g19[j] : g.v[j];
            h[k >= 10 ? k - 10 : k] += (u64)a * b;
        }
    }
    fe_carry(o, h);
}

// squaring: the symmetric products once, doubled (55 multiply-adds instead of 100)
__device__ __forceinline__ void fe_sq(Fe &o, const Fe &f)
{
    u32 f19[10], d[10];
#pragma unroll
    for (int j = 0; j < 10; j++) {
        f19[j] = 19u * f.v[j];
        d[j] = 2u * f.v[j];
    }
    u64 h[10];
#pragma unroll
    for (int k = 0; k < 10; k++)
        h[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = i; j < 10; j++) {
            const int k = i + j;
            // term f_i f_j (x2 if i != j), x2 if both odd, x19 if k >= 10
            u32 a = (i != j) ? d[i] : f.v[i];
            const bool oo = (i & 1) && (j & 1);
            const u32 b = k >= 10 ? f19[j] : f.v[j];
            u64 p = (u64)a * b;
            if (oo)
                p <<= 1;
            h[k >= 10 ? k - 10 : k] += p;
        }
    }
    fe_carry(o, h);
}

__device__ __forceinline__ void fe_mul_small(Fe &o, const Fe &f, u32 k)
{
    u64 h[10];
#pragma unroll
    for (int i = 0; i < 10; i++)
        h[i] = (u64)f.v[i] * k;
    fe_carry(o, h);
}

__device__ __forceinline__ void fe_sqn(Fe &o, const Fe &f, int n)
{
    fe_sq(o, f);
    for (int i = 1; i < n; i++)
        fe_sq(o, o);
}

// z^(p-2) = z^(2^255 - 21): the ref10 addition chain (254 squarings, 11 multiplications)
__device__ void fe_invert(Fe &out, const Fe &z)
{
    Fe t0, t1, t2, t3;
    fe_sq(t0, z);               // 2
    fe_sqn(t1, t0, 2);          // 8
    fe_mul(t1, z, t1);          // 9
    fe_mul(t0, t0, t1);         // 11
    fe_sq(t2, t0);              // 22
    fe_mul(t1, t1, t2);         // 2^5 - 1
    fe_sqn(t2, t1, 5);
    fe_mul(t1, t2, t1);         // 2^10 - 1
    fe_sqn(t2, t1, 10);
    fe_mul(t2, t2, t1);         // 2^20 - 1
    fe_sqn(t3, t2, 20);
    fe_mul(t2, t3, t2);         // 2^40 - 1
    fe_sqn(t2, t2, 10);
    fe_mul(t1, t2, t1);         // 2^50 - 1
    fe_sqn(t2, t1, 50);
    fe_mul(t2, t2, t1);         // 2^100 - 1
    fe_sqn(t3, t2, 100);
    fe_mul(t2, t3, t2);         // 2^200 - 1
    fe_sqn(t2, t2, 50);
    fe_mul(t1, t2, t1);         // 2^250 - 1
    fe_sqn(t1, t1, 5);          // 2^255 - 2^5
    fe_mul(out, t1, t0);        // 2^255 - 21
}

__device__ __forceinline__ void fe_cswap(Fe &a, Fe &b, u32 swap)
{
    const u32 m = 0u - swap;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const u32 t = m & (a.v[i] ^ b.v[i]);
        a.v[i] ^= t;
        b.v[i] ^= t;
    }
}

// 8 little-endian words -> limbs (bit 255 masked)
__device__ __forceinline__ void fe_from_words(Fe &h, const u32 w[8])
{
    // limb i covers bits [s_i, s_i + width): s = 0,26,51,77,102,128,153,179,204,230
    const int s[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const int b = s[i], wi = b >> 5, sh = b & 31;
        u64 x = (u64)w[wi] >> sh;
        if (wi + 1 < 8)
            x |= (u64)w[wi + 1] << (32 - sh);
        h.v[i] = (u32)x & ((i & 1) ? M25 : M26);
    }
}

// canonical little-endian encoding (full reduction mod p)
__device__ __forceinline__ void fe_to_words(u32 w[8], const Fe &f)
{
    Fe h = f;
    fe_carry32(h);
    fe_carry32(h);
    // q = 1 iff h >= p: propagate (h + 19) >> 255
    u32 q = (h.v[0] + 19u) >> 26;
#pragma unroll
    for (int i = 1; i < 10; i++)
        q = (h.v[i] + q) >> lw(i);
    h.v[0] += 19u * q;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        h.v[i + 1] += h.v[i] >> lw(i);
        h.v[i] &= (i & 1) ? M25 : M26;
    }
    h.v[9] &= M25;
    const int s[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
#pragma unroll
    for (int k = 0; k < 8; k++)
        w[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const int b = s[i], wi = b >> 5, sh = b & 31;
        w[wi] |= h.v[i] << sh;
        if (sh && wi + 1 < 8)
            w[wi + 1] |= (u32)((u64)h.v[i] >> (32 - sh));
    }
}

__device__ __forceinline__ void load_words(u32 w[8], const uint8_t *__restrict__ p)
{
#pragma unroll
    for (int i = 0; i < 8; i++)
        w[i] = (u32)p[4 * i] | ((u32)p[4 * i + 1] << 8) | ((u32)p[4 * i + 2] << 16) | ((u32)p[4 * i + 3] << 24);
}

__device__ __forceinline__ void store_words(uint8_t *__restrict__ p, const u32 w[8])
{
#pragma unroll
    for (int i = 0; i < 8; i++) {
        p[4 * i] = (uint8_t)w[i];
        p[4 * i + 1] = (uint8_t)(w[i] >> 8);
        p[4 * i + 2] = (uint8_t)(w[i] >> 16);
        p[4 * i + 3] = (uint8_t)(w[i] >> 24);
    }
}

// X25519(k, u), RFC 7748 section 5; k, u, out as little-endian words
__device__ void x25519(u32 out[8], const u32 kin[8], const u32 u[8])
{
    u32 k[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        k[i] = kin[i];
    k[0] &= ~7u;
    k[7] = (k[7] & 0x7fffffffu) | 0x40000000u;
    Fe x1, x2, z2, x3, z3;
    fe_from_words(x1, u);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        x2.v[i] = i == 0;
        z2.v[i] = 0;
        x3.v[i] = x1.v[i];
        z3.v[i] = i == 0;
    }
    u32 swap = 0;
    for (int t = 254; t >= 0; t--) {
        const u32 kt = (k[t >> 5] >> (t & 31)) & 1u;
        swap ^= kt;
        fe_cswap(x2, x3, swap);
        fe_cswap(z2, z3, swap);
        swap = kt;
        Fe A, B, C, D, AA, BB, E, DA, CB;
        fe_add(A, x2, z2);
        fe_sub(B, x2, z2);
        fe_add(C, x3, z3);
        fe_sub(D, x3, z3);
        fe_sq(AA, A);
        fe_sq(BB, B);
        fe_mul(DA, D, A);
        fe_mul(CB, C, B);
        fe_sub(E, AA, BB);
        fe_add(A, DA, CB);      // DA + CB
        fe_sub(B, DA, CB);      // DA - CB
        fe_sq(x3, A);
        fe_sq(B, B);
        fe_mul(z3, x1, B);
        fe_mul(x2, AA, BB);
        fe_mul_small(C, E, 121665u);
        fe_add(C, AA, C);
        fe_mul(z2, E, C);
    }
    fe_cswap(x2, x3, swap);
    fe_cswap(z2, z3, swap);
    Fe zi, r;
    fe_invert(zi, z2);
    fe_mul(r, x2, zi);
    fe_to_words(out, r);
}

// one lane per key agreement: out = X25519(scalar, point), point = 9 when points == nullptr
__global__ __launch_bounds__(64) void k_x25519(const uint8_t *__restrict__ scalars, const uint8_t *__restrict__ points,
                                                uint8_t *__restrict__ out, uint32_t count, int beforenm)
{
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= count)
        return;
    u32 k[8], u[8], r[8];
    load_words(k, scalars + 32ull * i);
    if (points) {
        load_words(u, points + 32ull * i);
    } else {
#pragma unroll
        for (int w = 0; w < 8; w++)
            u[w] = w == 0 ? 9u : 0u;
    }
    x25519(r, k, u);
    if (beforenm) {
        // NaCl crypto_box_beforenm: HSalsa20(shared, 0^16) with the "expand 32-byte k" constants
        u32 o[8];
        const u32 zero[4] = {0u, 0u, 0u, 0u};
        cz::hsalsa20(o, r, zero);
        store_words(out + 32ull * i, o);
    } else {
        store_words(out + 32ull * i, r);
    }
}

}  // namespace

extern "C" hipError_t czk_x25519(const void *scalars, const void *points, void *out, uint32_t count, int beforenm,
                                 hipStream_t s)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(k_x25519, dim3((count + 63) / 64), dim3(64), 0, s, (const uint8_t *)scalars,
                       (const uint8_t *)points, (uint8_t *)out, count, beforenm);
    return hipGetLastError();
}
