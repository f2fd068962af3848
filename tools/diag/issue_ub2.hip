// issue_ub2.hip -- second round of gfx950 VALU issue-cost probes (diagnostics, not product code).
//
// tools/diag/issue_ub.hip found two classes of 32-bit VALU instruction on MI355X: v_add_u32,
// v_xor_b32, v_mov_b32, v_bitop3_b32 and the f32 add/fma issue a wave64 instruction every
// 2 SIMD cycles; v_alignbit_b32, v_xad_u32, v_add3_u32, v_lshl_add_u32, v_perm_b32, the
// multiplies, the carry ops and every packed / 64-bit op take 4.  This probe classifies more
// opcodes, measures what an alternating fast/slow stream costs, and times one Salsa20 double
// round in its alignbit form against an all-fast shift form (tools/diag/gen_issue_ub2.py).
// Method as issue_ub.hip: k waves per SIMD by dynamic LDS, 8 rounds of 256 CUs x k workgroups,
// clock from s_memtime / s_memrealtime in every wave.
// build: python tools/diag/gen_issue_ub2.py &&
//        hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/diag/issue_ub2 tools/diag/issue_ub2.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../jeromq_amd/csrc/cz_device.h"
using namespace cz;

#define UB_CLOB                                                                                                    \
    "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", \
        "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "vcc", "s0", "s1", "s2"
#include "issue_ub2.inc"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

enum { K_SALSA_ALIGN = 1000, K_SALSA_SHIFT = 1001, K_SALSA_LAZY = 1002, K_SALSA_EAGER_C = 1003 };

__device__ __forceinline__ void ub_init()
{
    asm volatile("v_mov_b32 v4, 0x3f800001\n v_mov_b32 v5, 0x3f7ffffe\n v_mov_b32 v6, 0x3f800003\n"
                 "v_mov_b32 v7, 0x3f000001\n s_mov_b32 s2, 0x9e3779b9\n s_mov_b64 vcc, 0\n s_mov_b64 s[0:1], 0\n"
                 "v_mov_b32 v8, v4\n v_mov_b32 v9, v5\n v_mov_b32 v10, v6\n v_mov_b32 v11, v7\n"
                 "v_mov_b32 v12, v4\n v_mov_b32 v13, v5\n v_mov_b32 v14, v6\n v_mov_b32 v15, v7\n"
                 "v_mov_b32 v16, v4\n v_mov_b32 v17, v5\n v_mov_b32 v18, v6\n v_mov_b32 v19, v7\n"
                 "v_mov_b32 v20, v4\n v_mov_b32 v21, v5\n v_mov_b32 v22, v6\n v_mov_b32 v23, v7\n" ::
                     : "v4", "v5", "v6", "v7", UB_CLOB);
}

template <int I>
__global__ __launch_bounds__(256) void k_ub(u32 *out, u64 *clk, int nit)
{
    const u32 gid = blockIdx.x * 256 + threadIdx.x;
    u32 s = 0;
    const u64 t0_ = __builtin_amdgcn_s_memtime();
    const u64 r0_ = __builtin_amdgcn_s_memrealtime();
    if constexpr (I < 1000) {
        ub_init();
        for (int i = 0; i < nit; i++) {
            ub_body<I>(); ub_body<I>(); ub_body<I>(); ub_body<I>();
        }
        asm volatile("v_xor_b32 %0, v8, v23" : "=v"(s)::"v8", "v23");
    } else if constexpr (I == K_SALSA_ALIGN || I == K_SALSA_SHIFT) {
        ub_init();
        for (int i = 0; i < nit; i++) {
            if constexpr (I == K_SALSA_ALIGN)
                asm volatile(SALSA_DR_ALIGN SALSA_DR_ALIGN ::: UB_CLOB);
            else
                asm volatile(SALSA_DR_SHIFT SALSA_DR_SHIFT ::: UB_CLOB);
        }
        asm volatile("v_xor_b32 %0, v8, v23" : "=v"(s)::"v8", "v23");
    } else {
        // the product's rounds: 2 C rounds + 18 lazy asm rounds (LAZY), or 20 compiler-scheduled
        // eager rounds (EAGER_C); one "iteration" = 2 double rounds' worth (x 5 per block)
        u32 x[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
            x[k] = gid * (0x9e3779b9u + k);
        for (int i = 0; i < nit; i += 5) {
            if constexpr (I == K_SALSA_LAZY) {
                u32 d[16];
                rounds_lazy(x, d);
#pragma unroll
                for (int k = 0; k < 16; k++)
                    x[k] = lazy_pending(k) ? (x[k] ^ d[k]) : x[k];
            } else {
                rounds_eager(x);
            }
        }
#pragma unroll
        for (int k = 0; k < 16; k++)
            s ^= x[k];
    }
    const u64 t1_ = __builtin_amdgcn_s_memtime();
    const u64 r1_ = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const u32 w = gid >> 6;
        clk[2 * w] = t1_ - t0_;
        clk[2 * w + 1] = r1_ - r0_;
    }
    out[gid] = s;
}

static u32 *d_out;
static u64 *d_clk;
constexpr int ROUNDS = 8;
constexpr int MAXK = 8;

// per: wave-instructions (or double rounds, for the Salsa kernels) per iteration
template <int I>
void run(const char *name, int k, int nit, double per, const char *unit)
{
    const int lds = (160 * 1024 / k) & ~255;
    const int blocks = 256 * k * ROUNDS;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0;
    for (int it = 0; it < 400; it++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_ub<I>, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, nit);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 3 && (it + 1) * ms > 150.0f)
            break;
    }
    std::vector<float> t;
    for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_ub<I>, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, nit);
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
    const double units_per_simd = (double)nw * nit * per / 1024.0;
    const double cyc = ms * 1e-3 * clock * 1e9 / units_per_simd;
    printf("%-20s k=%d  %8.3f ms  clock %.2f GHz  %7.2f SIMD-cycles per %s\n", name, k, ms, clock, cyc, unit);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int I>
void run_singles(int nit)
{
    for (int k : {4, 8})
        run<I>(UB_NAMES[I], k, nit, 4.0 * UB_PER[I], "wave-instruction");
    if constexpr (I + 1 < UB_NSINGLE)
        run_singles<I + 1>(nit);
}

int main(int argc, char **argv)
{
    const int nit = argc > 1 ? atoi(argv[1]) : 256;
    CK(hipMalloc(&d_out, 256 * 256 * MAXK * ROUNDS * sizeof(u32)));
    CK(hipMalloc(&d_clk, 2 * 256 * MAXK * ROUNDS * 4 * sizeof(u64)));
    run_singles<0>(nit);
    const int dr = nit / 4;  // double rounds: 2 per iteration
    for (int k : {3, 4, 6, 8}) {
        run<K_SALSA_ALIGN>("salsa DR align", k, dr, 2.0, "double round (96 VALU: 32 alignbit)");
        run<K_SALSA_SHIFT>("salsa DR shift", k, dr, 2.0, "double round (128 VALU, all 2-cycle)");
        run<K_SALSA_EAGER_C>("salsa DR eager C", k, dr, 2.0, "double round (compiled, 10 per 5 it)");
        run<K_SALSA_LAZY>("salsa DR lazy (prod)", k, dr, 2.0, "double round (product lazy rounds)");
    }
    return 0;
}
