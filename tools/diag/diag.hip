// diag.hip -- diagnostic micro-benchmarks for the CURVE seal kernel (not product code).
//
// 1. instruction throughput on gfx950 for the ops the kernel leans on
// 2. ablations of the lane-per-frame 4 KiB seal loop: memory only, compute only,
//    Salsa only, Poly only, full -- to see which roof binds
// 3. coalesced copy of the same bytes (memory-side reference)
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/diag/diag tools/diag/diag.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../jeromq_amd/csrc/cz_device.h"

using namespace cz;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));  \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

// ---------------- instruction throughput ----------------
constexpr int ITERS = 256;

__global__ void ub_mad64(u64 *out, u32 a0, u32 b0)
{
    u32 a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
    u64 acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = j;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = (u64)(a + j) * b + acc[j];
        asm volatile("" : "+v"(a));
    }
    u64 s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void ub_add32(u64 *out, u32 a0, u32 b0)
{
    u32 a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
    u32 acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = j;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = (acc[j] ^ b) + a;  // v_xad_u32? keep as 2 ops
        asm volatile("" : "+v"(a));
    }
    u32 s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void ub_alignbit(u64 *out, u32 a0, u32 b0)
{
    u32 b = b0 ^ threadIdx.x;
    u32 acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = j + a0;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = __builtin_amdgcn_alignbit(acc[j], b, 7);
        asm volatile("" : "+v"(b));
    }
    u32 s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void ub_mullo(u64 *out, u32 a0, u32 b0)
{
    u32 b = b0 ^ threadIdx.x;
    u32 acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = j + a0;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = acc[j] * b;
        asm volatile("" : "+v"(b));
    }
    u32 s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void ub_mulhi(u64 *out, u32 a0, u32 b0)
{
    u32 b = b0 ^ threadIdx.x;
    u32 acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = j + a0;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = __umulhi(acc[j], b) + j;
        asm volatile("" : "+v"(b));
    }
    u32 s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void ub_add64(u64 *out, u32 a0, u32 b0)
{
    u64 b = ((u64)b0 << 32) ^ threadIdx.x;
    u64 acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = j + a0;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = acc[j] + (b >> 32);
        asm volatile("" : "+v"(b));
    }
    u64 s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void ub_fma64(u64 *out, u32 a0, u32 b0)
{
    double b = 1.0000001 + threadIdx.x * 1e-9;
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = j + a0;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = fma(acc[j], b, 0.5);
        asm volatile("" : "+v"(b));
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s += acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (u64)s;
}


// exact-instruction throughput: 8 independent chains of one opcode via inline asm
#define ASM_UB(NAME, INSTR)                                                                   \
__global__ void NAME(u64 *out, u32 a0, u32 b0)                                                \
{                                                                                             \
    u32 v0 = a0 + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 ^ 11,\
        v6 = v0 + 13, v7 = v0 + 17, b = b0 ^ threadIdx.x;                                     \
    for (int i = 0; i < ITERS; i++) {                                                         \
        asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)   \
                     : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) \
                     : "v"(b));                                                               \
    }                                                                                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;       \
}
#define I_ALIGNBIT(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 7\n"
#define I_XOR(k) "v_xor_b32 %" #k ", %" #k ", %8\n"
#define I_ADD(k) "v_add_u32 %" #k ", %" #k ", %8\n"
#define I_ALIGNBYTE(k) "v_alignbyte_b32 %" #k ", %" #k ", %8, 3\n"
#define I_XAD(k) "v_xad_u32 %" #k ", %" #k ", %8, %" #k "\n"
#define I_MULLO(k) "v_mul_lo_u32 %" #k ", %" #k ", %8\n"
#define I_MULHI(k) "v_mul_hi_u32 %" #k ", %" #k ", %8\n"
#define I_MUL24(k) "v_mul_u32_u24 %" #k ", %" #k ", %8\n"
#define I_BFI(k) "v_bfi_b32 %" #k ", %" #k ", %8, %" #k "\n"
ASM_UB(ua_alignbit, I_ALIGNBIT)
ASM_UB(ua_xor, I_XOR)
ASM_UB(ua_add, I_ADD)
ASM_UB(ua_alignbyte, I_ALIGNBYTE)
ASM_UB(ua_xad, I_XAD)
ASM_UB(ua_mullo, I_MULLO)
ASM_UB(ua_mulhi, I_MULHI)
ASM_UB(ua_mul24, I_MUL24)
ASM_UB(ua_bfi, I_BFI)

// v_mad_u64_u32 chains: 4 independent 64-bit accumulators
__global__ void ua_mad64(u64 *out, u32 a0, u32 b0)
{
    u64 acc0 = a0, acc1 = a0 * 3ull, acc2 = a0 * 5ull, acc3 = a0 * 7ull;
    u32 x = a0 + threadIdx.x, y = b0 ^ threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n"
                     "v_mad_u64_u32 %1, s[40:41], %4, %5, %1\n"
                     "v_mad_u64_u32 %2, s[40:41], %4, %5, %2\n"
                     "v_mad_u64_u32 %3, s[40:41], %4, %5, %3\n"
                     "v_mad_u64_u32 %0, s[40:41], %5, %4, %0\n"
                     "v_mad_u64_u32 %1, s[40:41], %5, %4, %1\n"
                     "v_mad_u64_u32 %2, s[40:41], %5, %4, %2\n"
                     "v_mad_u64_u32 %3, s[40:41], %5, %4, %3\n"
                     : "+v"(acc0), "+v"(acc1), "+v"(acc2), "+v"(acc3) : "v"(x), "v"(y) : "s40", "s41");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc0 ^ acc1 ^ acc2 ^ acc3;
}

// clock probe: one lane per wave stamps s_memtime / s_memrealtime around a busy VALU loop
__global__ void ua_clock(u64 *out, u32 a0, u32 b0)
{
    u32 v0 = a0 + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 ^ 11, v6 = v0 + 13,
        v7 = v0 + 17, b = b0 ^ threadIdx.x;
    u64 t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < 8 * ITERS; i++) {
        asm volatile(I_XOR(0) I_XOR(1) I_XOR(2) I_XOR(3) I_XOR(4) I_XOR(5) I_XOR(6) I_XOR(7)
                     : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
                     : "v"(b));
    }
    u64 t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = t1 - t0;
        out[2 * blockIdx.x + 1] = r1 - r0;
    }
    if ((v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7) == 0x12345) out[0] = 1;
}

// memory patterns: each wave copies its 64 frames (4096 B in, 4144 B out stride); lanes grouped
// G per frame; a group instruction moves 16*G contiguous bytes of one frame
template <int G>
__global__ __launch_bounds__(256) void k_copy_seg(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                   uint32_t count)
{
    const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const uint32_t f0 = wave * 64;
    if (f0 >= count) return;
    const uint32_t sub = lane % G, fl = lane / G;  // 64/G frames per instruction
    for (uint32_t off = 0; off < 4096; off += 16 * G) {
#pragma unroll
        for (uint32_t j = 0; j < G; j++) {  // G instructions cover the 64 frames
            uint32_t f = f0 + fl + j * (64 / G);
            uint4 v = *(const uint4 *)(in + (u64)f * 4096 + off + 16 * sub);
            *(uint4 *)(out + (u64)f * 4144 + off + 16 * sub) = v;
        }
    }
}

// ---------------- seal-loop ablations (lane-per-frame, 4 KiB frames, steady blocks only) --------
enum { F_LOAD = 1, F_STORE = 2, F_SALSA = 4, F_POLY = 8 };

template <int F>
__global__ __launch_bounds__(256) void k_ablate(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                 uint32_t count, const uint8_t *__restrict__ subkey, u64 *sink)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    u32 key[8];
    for (int w = 0; w < 8; w++) key[w] = ((const u32 *)subkey)[w];
    const uint8_t *src = in + (u64)i * 4096;
    uint8_t *dst = out + (u64)i * 4144;
    u32 n0 = i, n1 = 0x12345678u;
    Poly P;
    poly_init(P, key[0] ^ i, key[1], key[2], key[3], key[4], key[5], key[6], key[7]);
    u32 carry = 0, acc = 0;
    for (u32 blk = 1; blk < 64; blk++) {
        u32 W[16];
        if (F & F_LOAD) {
            const uint4 *s4 = (const uint4 *)(src + 64u * blk - 32u);
#pragma unroll
            for (int c = 0; c < 4; c++) {
                uint4 v = s4[c];
                W[4 * c] = v.x; W[4 * c + 1] = v.y; W[4 * c + 2] = v.z; W[4 * c + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) W[k] = blk * 0x9E3779B9u + k + i;
        }
        u32 x[16];
        if (F & F_SALSA) {
            salsa20_block(x, key, n0, n1, blk, 0u);
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) x[k] = key[k & 7] + blk;
        }
        u32 C[16];
        C[0] = __builtin_amdgcn_alignbyte(W[0], carry, 3) ^ x[0];
#pragma unroll
        for (int k = 1; k < 16; k++) C[k] = __builtin_amdgcn_alignbyte(W[k], W[k - 1], 3) ^ x[k];
        carry = W[15];
        if (F & F_STORE) {
            uint4 *d4 = (uint4 *)(dst + 64u * blk);
#pragma unroll
            for (int c = 0; c < 4; c++) d4[c] = make_uint4(C[4 * c], C[4 * c + 1], C[4 * c + 2], C[4 * c + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) acc ^= C[k];
        }
        if (F & F_POLY) {
            poly_block(P, C[0], C[1], C[2], C[3], 1u);
            poly_block(P, C[4], C[5], C[6], C[7], 1u);
            poly_block(P, C[8], C[9], C[10], C[11], 1u);
            poly_block(P, C[12], C[13], C[14], C[15], 1u);
        }
    }
    u32 tag[4];
    poly_finish(P, tag);
    if (acc == 0x7fffffffu || tag[0] == 0x13572468u) sink[i] = acc ^ tag[1];
}

__global__ __launch_bounds__(256) void k_copy_coalesced(const uint4 *__restrict__ in, uint4 *__restrict__ out,
                                                         u64 n16)
{
    for (u64 t = (u64)blockIdx.x * 256 + threadIdx.x; t < n16; t += (u64)gridDim.x * 256) out[t] = in[t];
}

// lane-per-frame pure copy with the real strides
__global__ __launch_bounds__(256) void k_copy_lanewise(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                        uint32_t count)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const uint4 *s = (const uint4 *)(in + (u64)i * 4096);
    uint4 *d = (uint4 *)(out + (u64)i * 4144);
    for (int c = 0; c < 256; c += 4) {
        uint4 a = s[c], b = s[c + 1], e = s[c + 2], f = s[c + 3];
        d[c] = a; d[c + 1] = b; d[c + 2] = e; d[c + 3] = f;
    }
}


// lane-per-frame copy with configurable strides and a per-lane step skew (tests channel camping)
template <int SKEW>
__global__ __launch_bounds__(256) void k_copy_skew(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                    uint32_t count, uint32_t is, uint32_t os)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const uint8_t *s = in + (u64)i * is;
    uint8_t *d = out + (u64)i * os;
    uint32_t start = SKEW ? ((i * SKEW) & 63u) : 0u;
    for (uint32_t t = 0; t < 64; t++) {
        uint32_t b = (t + start) & 63u;
        const uint4 *s4 = (const uint4 *)(s + 64u * b);
        uint4 a0 = s4[0], a1 = s4[1], a2 = s4[2], a3 = s4[3];
        uint4 *d4 = (uint4 *)(d + 64u * b);
        d4[0] = a0; d4[1] = a1; d4[2] = a2; d4[3] = a3;
    }
}

// better coalesced copy: 4 x 16 B per thread per iteration
__global__ __launch_bounds__(256) void k_copy_coal4(const uint4 *__restrict__ in, uint4 *__restrict__ out, u64 n16)
{
    u64 stride = (u64)gridDim.x * 256;
    for (u64 t = (u64)blockIdx.x * 256 + threadIdx.x; t + 3 * stride < n16; t += 4 * stride) {
        uint4 a = in[t], b = in[t + stride], c = in[t + 2 * stride], e = in[t + 3 * stride];
        out[t] = a; out[t + stride] = b; out[t + 2 * stride] = c; out[t + 3 * stride] = e;
    }
}

// read-only and write-only lanewise variants
__global__ __launch_bounds__(256) void k_read_lanewise(const uint8_t *__restrict__ in, uint32_t count, uint32_t is,
                                                        u64 *sink)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const uint4 *s = (const uint4 *)(in + (u64)i * is);
    u32 acc = 0;
    for (int c = 0; c < 256; c += 4) {
        uint4 a = s[c], b = s[c + 1], e = s[c + 2], f = s[c + 3];
        acc ^= a.x ^ b.y ^ e.z ^ f.w;
    }
    if (acc == 0x1234567u) sink[i] = acc;
}
__global__ __launch_bounds__(256) void k_write_lanewise(uint8_t *__restrict__ out, uint32_t count, uint32_t os)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    uint4 *d = (uint4 *)(out + (u64)i * os);
    for (int c = 0; c < 256; c += 4) {
        uint4 v = make_uint4(i, c, i ^ c, 7);
        d[c] = v; d[c + 1] = v; d[c + 2] = v; d[c + 3] = v;
    }
}


// write-only patterns: G lanes per frame, 16*G contiguous bytes per frame per instruction; NT = nontemporal
template <int G, bool NT>
__global__ __launch_bounds__(256) void k_write_seg(uint8_t *__restrict__ out, uint32_t count, uint32_t os)
{
    const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const uint32_t f0 = wave * 64;
    if (f0 >= count) return;
    const uint32_t sub = lane % G, fl = lane / G;
    for (uint32_t off = 0; off < 4096; off += 16 * G) {
#pragma unroll
        for (uint32_t j = 0; j < G; j++) {
            uint32_t f = f0 + fl + j * (64 / G);
            uint4 v = make_uint4(f, off, sub, j);
            uint4 *d = (uint4 *)(out + (u64)f * os + off + 16 * sub);
            if (NT) {
                __builtin_nontemporal_store(v.x, &((u32 *)d)[0]);
                __builtin_nontemporal_store(v.y, &((u32 *)d)[1]);
                __builtin_nontemporal_store(v.z, &((u32 *)d)[2]);
                __builtin_nontemporal_store(v.w, &((u32 *)d)[3]);
            } else {
                *d = v;
            }
        }
    }
}
// lane-wise write with a nontemporal 16 B store (vector type)
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_write_lanewise_nt(uint8_t *__restrict__ out, uint32_t count, uint32_t os)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    u32x4 *d = (u32x4 *)(out + (u64)i * os);
    for (int c = 0; c < 256; c++) {
        u32x4 v = {i, (u32)c, i ^ c, 7u};
        __builtin_nontemporal_store(v, d + c);
    }
}
template <int G>
__global__ __launch_bounds__(256) void k_write_seg_ntv(uint8_t *__restrict__ out, uint32_t count, uint32_t os)
{
    const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const uint32_t f0 = wave * 64;
    if (f0 >= count) return;
    const uint32_t sub = lane % G, fl = lane / G;
    for (uint32_t off = 0; off < 4096; off += 16 * G) {
#pragma unroll
        for (uint32_t j = 0; j < G; j++) {
            uint32_t f = f0 + fl + j * (64 / G);
            u32x4 v = {f, off, sub, j};
            __builtin_nontemporal_store(v, (u32x4 *)(out + (u64)f * os + off + 16 * sub));
        }
    }
}
__global__ __launch_bounds__(256) void k_write_coal(uint4 *__restrict__ out, u64 n16)
{
    for (u64 t = (u64)blockIdx.x * 256 + threadIdx.x; t < n16; t += (u64)gridDim.x * 256) out[t] = make_uint4(t, 1, 2, 3);
}

template <typename K, typename... A>
static float timeit(K kern, dim3 g, dim3 b, int reps, A... args)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, g, b, 0, 0, args...);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, g, b, 0, 0, args...);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main()
{
    u64 *sink;
    const int blocks = 256 * 16, threads = 256;
    CK(hipMalloc(&sink, sizeof(u64) * blocks * threads));
    const double winstr = (double)blocks * threads / 64 * ITERS * 8;  // wave-instructions of the op
    struct {
        const char *name;
        float ms;
    } r[] = {
        {"mad_u64_u32", timeit(ub_mad64, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
        {"xor+add u32 (2 ops)", timeit(ub_add32, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
        {"alignbit", timeit(ub_alignbit, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
        {"mul_lo_u32", timeit(ub_mullo, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
        {"mul_hi_u32 + add", timeit(ub_mulhi, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
        {"add u64", timeit(ub_add64, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
        {"fma_f64", timeit(ub_fma64, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
    };
    const double peak = 1024.0 * 2.4e9 / 2.0;  // wave64 instr/s at 1 per 2 cycles per SIMD
    for (auto &x : r)
        printf("ubench %-22s %8.3f ms  %7.1f G wave-instr/s  = %.3f of 1/2clk/SIMD @2.4GHz\n", x.name, x.ms,
               winstr / (x.ms * 1e-3) / 1e9, winstr / (x.ms * 1e-3) / peak);


    {
        struct { const char *name; float ms; } ra[] = {
            {"asm alignbit", timeit(ua_alignbit, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm xor", timeit(ua_xor, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm add_u32", timeit(ua_add, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm alignbyte", timeit(ua_alignbyte, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm xad_u32", timeit(ua_xad, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm mul_lo_u32", timeit(ua_mullo, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm mul_hi_u32", timeit(ua_mulhi, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm mul_u32_u24", timeit(ua_mul24, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm bfi", timeit(ua_bfi, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
            {"asm mad_u64_u32", timeit(ua_mad64, dim3(blocks), dim3(threads), 5, sink, 3u, 5u)},
        };
        for (auto &x : ra)
            printf("ubench %-22s %8.4f ms  %7.1f G wave-instr/s  = %.3f of 1/2clk/SIMD @2.4GHz\n", x.name, x.ms,
                   winstr / (x.ms * 1e-3) / 1e9, winstr / (x.ms * 1e-3) / peak);
        float cms = timeit(ua_clock, dim3(blocks), dim3(threads), 1, sink, 3u, 5u);
        std::vector<u64> h(2 * blocks);
        CK(hipMemcpy(h.data(), sink, 16 * blocks, hipMemcpyDeviceToHost));
        double ratio = 0;
        for (int q = 0; q < blocks; q++) ratio += (double)h[2 * q] / (double)h[2 * q + 1];
        printf("clock: busy-VALU loop %.3f ms, s_memtime/s_memrealtime*100MHz = %.3f GHz (mean over WGs)\n", cms,
               ratio / blocks * 0.1);
    }

    // ablations
    const uint32_t count = 1u << 20;
    uint8_t *in, *out, *key;
    CK(hipMalloc(&in, (size_t)count * 4096 + 4096));
    CK(hipMalloc(&out, (size_t)count * 4144 + 4096));
    CK(hipMalloc(&key, 64));
    CK(hipMemset(in, 0x5a, (size_t)count * 4096));
    CK(hipMemset(key, 0x11, 64));
    u64 *sink2;
    CK(hipMalloc(&sink2, sizeof(u64) * count));
    dim3 g((count + 255) / 256), b(256);
    const size_t in_bytes = (size_t)count * 4096 + 4096, out_bytes = (size_t)count * 4144 + 4096;
    auto nfit = [&](size_t is, size_t os) -> uint32_t {
        size_t a = in_bytes / is, c = out_bytes / os;
        size_t m = a < c ? a : c;
        return (uint32_t)(m < count ? m : count);
    };
    const double bytes = (double)count * 63 * 64 * 2;  // steady blocks only, read + write
    struct {
        const char *name;
        float ms;
    } a[] = {
        {"W lanewise 16B os=4144", timeit(k_write_lanewise, g, b, 5, out, count, 4144u)},
        {"W lanewise 16B os=4096", timeit(k_write_lanewise, g, b, 5, out, count, 4096u)},
        {"W lanewise 16B NT os=4144", timeit(k_write_lanewise_nt, g, b, 5, out, count, 4144u)},
        {"W seg G=4 (64B) os=4144", timeit(k_write_seg<4, false>, g, b, 5, out, count, 4144u)},
        {"W seg G=8 (128B) os=4144", timeit(k_write_seg<8, false>, g, b, 5, out, count, 4144u)},
        {"W seg G=8 (128B) os=4096", timeit(k_write_seg<8, false>, g, b, 5, out, count, 4096u)},
        {"W seg G=16 (256B) os=4096", timeit(k_write_seg<16, false>, g, b, 5, out, count, 4096u)},
        {"W seg G=64 (1KB) os=4096", timeit(k_write_seg<64, false>, g, b, 5, out, count, 4096u)},
        {"W seg G=4 NTv os=4144", timeit(k_write_seg_ntv<4>, g, b, 5, out, count, 4144u)},
        {"W seg G=8 NTv os=4096", timeit(k_write_seg_ntv<8>, g, b, 5, out, count, 4096u)},
        {"W seg G=16 NTv os=4096", timeit(k_write_seg_ntv<16>, g, b, 5, out, count, 4096u)},
        {"W coalesced", timeit(k_write_coal, dim3(8192), b, 5, (uint4 *)out, (u64)count * 4096 / 16)},
        {"R lanewise 4096", timeit(k_read_lanewise, g, b, 5, (const uint8_t *)in, count, 4096u, sink2)},
        {"copy coalesced x4", timeit(k_copy_coal4, dim3(4096), b, 5, (const uint4 *)in, (uint4 *)out, (u64)count * 4096 / 16)},
    };
    for (auto &x : a)
        printf("pattern %-30s %8.3f ms  %7.1f GB/s per 4 GiB moved\n", x.name, x.ms, (double)count * 4096 / (x.ms * 1e-3) / 1e9);
    return 0;
}
