// salsa_ub.hip -- register-only issue rate of the seal kernel's arithmetic on gfx950
// (diagnostics, not product code).  Asm double rounds: tools/diag/gen_salsa_ub.py.
//
// Each lane runs NB 64-byte Salsa20 blocks.  Occupancy is set with dynamic LDS:
// 160 KiB / k per 256-thread workgroup -> k workgroups per CU -> k waves per SIMD,
// grid = 8 rounds of 256 CUs x k workgroups.  Reported: SIMD cycles per wave-block =
// kernel time * clock * 1024 SIMDs / wave-blocks, clock = s_memtime / s_memrealtime
// (100 MHz) stamped by every wave of the same launch (median).
// build: python tools/diag/gen_salsa_ub.py &&
//        hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/diag/salsa_ub tools/diag/salsa_ub.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../jeromq_amd/csrc/cz_device.h"
#include "salsa_ub_asm.inc"
using namespace cz;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

enum { C_SALSA, C_SALSA_POLY, A_GROUPED, A_SERIAL, A_STAGGER, P_LATIN, P_IDENT };

#define X16                                                                                       \
    "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
        "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]),    \
        "+v"(x[15])
#define T4 "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
#define R10(X) X X X X X X X X X X

template <int V>
__global__ __launch_bounds__(256) void k_ub(u32 *out, u64 *clk, const u32 *__restrict__ keyg, int nb)
{
    u32 key[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        key[i] = keyg[i];
    const u32 gid = blockIdx.x * 256 + threadIdx.x;
    const u32 n1 = gid * 0x9e3779b9u;
    u32 acc[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        acc[k] = 0;
    Poly P;
    poly_init(P, n1, n1 * 3, n1 * 5, n1 * 7, 1, 2, 3, 4);
    if constexpr (V >= P_LATIN)
        asm volatile(P_INIT ::"v"(n1) : P_CLOBBERS);
    const u64 t0_ = __builtin_amdgcn_s_memtime();
    const u64 r0_ = __builtin_amdgcn_s_memrealtime();
    for (int b = 0; b < nb; b++) {
        if constexpr (V == P_LATIN) {
            asm volatile(R10(DR_P_LATIN)::: P_CLOBBERS);
        } else if constexpr (V == P_IDENT) {
            asm volatile(R10(DR_P_IDENT)::: P_CLOBBERS);
        } else {
            u32 x[16];
            if constexpr (V <= C_SALSA_POLY) {
                salsa20_block(x, key, 0x01020304u, n1, (u32)b, 0u);
            } else {
                const u32 in[16] = {SIGMA0, key[0], key[1], key[2], key[3], SIGMA1, 0x01020304u, n1,
                                    (u32)b, 0u, SIGMA2, key[4], key[5], key[6], key[7], SIGMA3};
#pragma unroll
                for (int k = 0; k < 16; k++)
                    x[k] = in[k];
#pragma unroll
                for (int r = 0; r < 10; r++) {
                    u32 t0, t1, t2, t3;
                    if constexpr (V == A_GROUPED)
                        asm volatile(DR_A_GROUPED : X16, T4);
                    else if constexpr (V == A_SERIAL)
                        asm volatile(DR_A_SERIAL : X16, T4);
                    else
                        asm volatile(DR_A_STAGGER : X16, T4);
                }
#pragma unroll
                for (int k = 0; k < 16; k++)
                    x[k] += in[k];
            }
            if constexpr (V == C_SALSA_POLY) {
                poly_block(P, x[0], x[1], x[2], x[3], 1u);
                poly_block(P, x[4], x[5], x[6], x[7], 1u);
                poly_block(P, x[8], x[9], x[10], x[11], 1u);
                poly_block(P, x[12], x[13], x[14], x[15], 1u);
            }
#pragma unroll
            for (int k = 0; k < 16; k++)
                acc[k] ^= x[k];
        }
    }
    const u64 t1_ = __builtin_amdgcn_s_memtime();
    const u64 r1_ = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const u32 w = gid >> 6;
        clk[2 * w] = t1_ - t0_;
        clk[2 * w + 1] = r1_ - r0_;
    }
    u32 s = P.h0 ^ P.h1 ^ P.h2 ^ P.h3 ^ P.h4;
#pragma unroll
    for (int k = 0; k < 16; k++)
        s ^= acc[k];
    if constexpr (V >= P_LATIN) {
        u32 pv;
        asm volatile("v_mov_b32 %0, v40" : "=v"(pv));
        s ^= pv;
    }
    out[gid] = s;
}

static u32 *d_out;
static u64 *d_clk;
static u32 *d_key;
constexpr int ROUNDS = 8;
constexpr int MAXK = 8;

template <int V>
void run(const char *name, int k, int nb)
{
    // k <= 2: one round of 256 x k workgroups and no LDS (64 KiB is the dynamic-LDS cap);
    // the dispatcher spreads them one per CU per k
    const int lds = k <= 2 ? 0 : (160 * 1024 / k) & ~255;
    const int blocks = k <= 2 ? 256 * k : 256 * k * ROUNDS;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0;
    for (int it = 0; it < 400; it++) {  // ramp the clock: >= 300 ms of back-to-back launches
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_ub<V>, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, d_key, nb);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 3 && (it + 1) * ms > 300.0f)
            break;
    }
    std::vector<float> t;
    for (int it = 0; it < 7; it++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_ub<V>, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, d_key, nb);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    ms = t[t.size() / 2];
    const int nw = blocks * 4;
    std::vector<u64> h(2 * (size_t)nw);
    CK(hipMemcpy(h.data(), d_clk, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    for (int w = 0; w < nw; w++)
        if (h[2 * w + 1])
            ghz.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);
    std::sort(ghz.begin(), ghz.end());
    const double clock = ghz.empty() ? 0.0 : ghz[ghz.size() / 2];
    const double wave_blocks_per_simd = (double)nw * nb / 1024.0;  // k <= 2: ~k waves on every SIMD
    const double cyc = ms * 1e-3 * clock * 1e9 / wave_blocks_per_simd;
    printf("%-13s k=%d  %8.3f ms  clock %.2f GHz  %6.0f SIMD-cycles/wave-block  %.3f per double-round VALU\n", name,
           k, ms, clock, cyc, cyc / 960.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main(int argc, char **argv)
{
    const int nb = argc > 1 ? atoi(argv[1]) : 32;
    CK(hipMalloc(&d_out, 256 * 256 * MAXK * ROUNDS * sizeof(u32)));
    CK(hipMalloc(&d_clk, 2 * 256 * MAXK * ROUNDS * 4 * sizeof(u64)));
    CK(hipMalloc(&d_key, 32));
    const u32 hk[8] = {0x1c0cdcc8u, 0x5efe8027u, 0x003e7ec2u, 0xb2b2ff1au,
                       0x15f329a9u, 0x96b142a6u, 0xc4db132cu, 0x6fd51f90u};
    CK(hipMemcpy(d_key, hk, 32, hipMemcpyHostToDevice));
    const char *ks = getenv("UB_WAVES");
    std::vector<int> kv;
    if (ks) {
        for (const char *c = ks; *c; c++)
            if (*c >= '1' && *c <= '8')
                kv.push_back(*c - '0');
    } else {
        kv = {4, 3, 5, 6, 8};
    }
    for (int k : kv) {
        run<C_SALSA>("c_salsa", k, nb);
        run<C_SALSA_POLY>("c_salsa_poly", k, nb);
        run<A_GROUPED>("a_grouped", k, nb);
        run<A_SERIAL>("a_serial", k, nb);
        run<A_STAGGER>("a_stagger", k, nb);
        if (k <= 6) {
            run<P_LATIN>("p_latin", k, nb);
            run<P_IDENT>("p_ident", k, nb);
        }
    }
    return 0;
}
