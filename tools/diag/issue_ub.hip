// issue_ub.hip -- per-opcode VALU issue cost on gfx950 (diagnostics, not product code).
//
// Each wave runs NIT iterations of 16 independent single-opcode instructions (16 chains, so no
// dependency stalls at >= 2 waves per SIMD).  Occupancy k waves per SIMD via dynamic LDS
// (160 KiB / k per 256-thread workgroup), grid = 8 rounds of 256 CUs x k workgroups.
// Reported: SIMD cycles per wave-instruction = kernel time * clock * 1024 SIMDs / wave-instructions,
// clock = s_memtime / s_memrealtime (100 MHz) stamped by every wave (median).
// Question it answers: is every int32 VALU opcode 4 cycles per wave64 instruction (DESIGN.md
// section 5), and which opcodes (if any) issue faster -- the guide quotes v_fma_f32 at 2.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/diag/issue_ub tools/diag/issue_ub.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned u32;
typedef unsigned long long u64;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

// 16 accumulators a0..a15 in v[8..23] (pairs for 64-bit ops use v[8..39]), operands v4..v7
#define REGS16(OP) OP(8) OP(9) OP(10) OP(11) OP(12) OP(13) OP(14) OP(15) OP(16) OP(17) OP(18) OP(19) OP(20) OP(21) OP(22) OP(23)
#define PAIRS8(OP) OP(8, 9) OP(10, 11) OP(12, 13) OP(14, 15) OP(16, 17) OP(18, 19) OP(20, 21) OP(22, 23)
#define S(x) #x
#define V(n) "v" S(n)

#define I_ADD(n) "v_add_u32_e32 " V(n) ", v4, " V(n) "\n"
#define I_XOR(n) "v_xor_b32_e32 " V(n) ", v4, " V(n) "\n"
#define I_ALIGNBIT(n) "v_alignbit_b32 " V(n) ", " V(n) ", " V(n) ", 7\n"
#define I_XAD(n) "v_xad_u32 " V(n) ", " V(n) ", v4, v5\n"
#define I_BITOP3(n) "v_bitop3_b32 " V(n) ", " V(n) ", v4, v5 bitop3:0x96\n"
#define I_ADD3(n) "v_add3_u32 " V(n) ", " V(n) ", v4, v5\n"
#define I_LSHLADD(n) "v_lshl_add_u32 " V(n) ", " V(n) ", 3, v5\n"
#define I_PERM(n) "v_perm_b32 " V(n) ", " V(n) ", v4, v5\n"
#define I_MAD24(n) "v_mad_u32_u24 " V(n) ", " V(n) ", v4, v5\n"
#define I_MULLO(n) "v_mul_lo_u32 " V(n) ", " V(n) ", v4\n"
#define I_ADDF(n) "v_add_f32_e32 " V(n) ", v4, " V(n) "\n"
#define I_FMAF(n) "v_fma_f32 " V(n) ", " V(n) ", v4, v5\n"
#define I_FMACF(n) "v_fmac_f32_e32 " V(n) ", v4, v5\n"
#define I_PKFMA(a, b) "v_pk_fma_f32 v[" S(a) ":" S(b) "], v[" S(a) ":" S(b) "], v[4:5], v[6:7]\n"
#define I_PKADDF(a, b) "v_pk_add_f32 v[" S(a) ":" S(b) "], v[" S(a) ":" S(b) "], v[4:5]\n"
#define I_PKADD16(n) "v_pk_add_u16 " V(n) ", " V(n) ", v4\n"
#define I_MAD64(a, b) "v_mad_u64_u32 v[" S(a) ":" S(b) "], s[0:1], v4, v5, v[" S(a) ":" S(b) "]\n"
#define I_LSHLADD64(a, b) "v_lshl_add_u64 v[" S(a) ":" S(b) "], v[" S(a) ":" S(b) "], 0, v[4:5]\n"
#define I_ADDCO(n) "v_add_co_u32_e32 " V(n) ", vcc, v4, " V(n) "\n"
#define I_MOV(n) "v_mov_b32_e32 " V(n) ", v4\n"
#define I_DOT2(n) "v_dot2_u32_u16 " V(n) ", v4, v5, " V(n) "\n"
// mixed streams: an int op and an f32 op alternating (co-issue from one wave?)
#define I_MIX_ADD_FMA(a, b) I_ADD(a) I_FMAF(b)
#define I_MIX_XOR_ALIGN(a, b) I_XOR(a) I_ALIGNBIT(b)

#define CLOB "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "vcc", "s0", "s1"

enum Op {
    O_ADD, O_XOR, O_ALIGNBIT, O_XAD, O_BITOP3, O_ADD3, O_LSHLADD, O_PERM, O_MAD24, O_MULLO, O_ADDF, O_FMAF, O_FMACF,
    O_PKFMA, O_PKADDF, O_PKADD16, O_MAD64, O_LSHLADD64, O_ADDCO, O_MOV, O_DOT2, O_MIX_ADD_FMA, O_MIX_XOR_ALIGN, O_N
};
static const char *NAMES[O_N] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_xad_u32", "v_bitop3_b32", "v_add3_u32",
                                 "v_lshl_add_u32", "v_perm_b32", "v_mad_u32_u24", "v_mul_lo_u32", "v_add_f32",
                                 "v_fma_f32", "v_fmac_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_pk_add_u16",
                                 "v_mad_u64_u32", "v_lshl_add_u64", "v_add_co_u32", "v_mov_b32", "v_dot2_u32_u16",
                                 "mix add+fma", "mix xor+alignbit"};
// wave-instructions per asm block
static const int PER[O_N] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 8, 8, 16, 8, 8, 16, 16, 16, 16, 16};

template <int O>
__device__ __forceinline__ void body()
{
    if constexpr (O == O_ADD) asm volatile(REGS16(I_ADD) ::: CLOB);
    if constexpr (O == O_XOR) asm volatile(REGS16(I_XOR) ::: CLOB);
    if constexpr (O == O_ALIGNBIT) asm volatile(REGS16(I_ALIGNBIT) ::: CLOB);
    if constexpr (O == O_XAD) asm volatile(REGS16(I_XAD) ::: CLOB);
    if constexpr (O == O_BITOP3) asm volatile(REGS16(I_BITOP3) ::: CLOB);
    if constexpr (O == O_ADD3) asm volatile(REGS16(I_ADD3) ::: CLOB);
    if constexpr (O == O_LSHLADD) asm volatile(REGS16(I_LSHLADD) ::: CLOB);
    if constexpr (O == O_PERM) asm volatile(REGS16(I_PERM) ::: CLOB);
    if constexpr (O == O_MAD24) asm volatile(REGS16(I_MAD24) ::: CLOB);
    if constexpr (O == O_MULLO) asm volatile(REGS16(I_MULLO) ::: CLOB);
    if constexpr (O == O_ADDF) asm volatile(REGS16(I_ADDF) ::: CLOB);
    if constexpr (O == O_FMAF) asm volatile(REGS16(I_FMAF) ::: CLOB);
    if constexpr (O == O_FMACF) asm volatile(REGS16(I_FMACF) ::: CLOB);
    if constexpr (O == O_PKFMA) asm volatile(PAIRS8(I_PKFMA) ::: CLOB);
    if constexpr (O == O_PKADDF) asm volatile(PAIRS8(I_PKADDF) ::: CLOB);
    if constexpr (O == O_PKADD16) asm volatile(REGS16(I_PKADD16) ::: CLOB);
    if constexpr (O == O_MAD64) asm volatile(PAIRS8(I_MAD64) ::: CLOB);
    if constexpr (O == O_LSHLADD64) asm volatile(PAIRS8(I_LSHLADD64) ::: CLOB);
    if constexpr (O == O_ADDCO) asm volatile(REGS16(I_ADDCO) ::: CLOB);
    if constexpr (O == O_MOV) asm volatile(REGS16(I_MOV) ::: CLOB);
    if constexpr (O == O_DOT2) asm volatile(REGS16(I_DOT2) ::: CLOB);
    if constexpr (O == O_MIX_ADD_FMA) asm volatile(PAIRS8(I_MIX_ADD_FMA) ::: CLOB);
    if constexpr (O == O_MIX_XOR_ALIGN) asm volatile(PAIRS8(I_MIX_XOR_ALIGN) ::: CLOB);
}

template <int O>
__global__ __launch_bounds__(256) void k_issue(u32 *out, u64 *clk, int nit)
{
    const u32 gid = blockIdx.x * 256 + threadIdx.x;
    // operands (v4..v7) and accumulators: small finite floats / arbitrary ints
    asm volatile("v_mov_b32 v4, 0x3f800001\n v_mov_b32 v5, 0x3f7ffffe\n v_mov_b32 v6, 0x3f800003\n v_mov_b32 v7, 0x3f000001\n"
                 "s_mov_b32 s0, 0\n s_mov_b32 s1, 0\n"
                 ::: "v4", "v5", "v6", "v7", "s0", "s1");
    asm volatile(REGS16(I_MOV) ::: CLOB);
    const u64 t0_ = __builtin_amdgcn_s_memtime();
    const u64 r0_ = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < nit; i++) {
        body<O>(); body<O>(); body<O>(); body<O>();
    }
    const u64 t1_ = __builtin_amdgcn_s_memtime();
    const u64 r1_ = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const u32 w = gid >> 6;
        clk[2 * w] = t1_ - t0_;
        clk[2 * w + 1] = r1_ - r0_;
    }
    u32 s;
    asm volatile("v_xor_b32 %0, v8, v23" : "=v"(s)::"v8", "v23");
    out[gid] = s;
}

static u32 *d_out;
static u64 *d_clk;
constexpr int ROUNDS = 8;
constexpr int MAXK = 8;

template <int O>
void run(int k, int nit)
{
    const int lds = (160 * 1024 / k) & ~255;
    const int blocks = 256 * k * ROUNDS;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0;
    for (int it = 0; it < 400; it++) {  // ramp the clock: >= 200 ms of back-to-back launches
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_issue<O>, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, nit);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 3 && (it + 1) * ms > 200.0f)
            break;
    }
    std::vector<float> t;
    for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_issue<O>, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, nit);
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
    const double winst_per_simd = (double)nw * nit * 4 * PER[O] / 1024.0;
    const double cyc = ms * 1e-3 * clock * 1e9 / winst_per_simd;
    printf("%-18s k=%d  %8.3f ms  clock %.2f GHz  %5.2f SIMD-cycles per wave-instruction\n", NAMES[O], k, ms, clock, cyc);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int O>
void run_all(const std::vector<int> &kv, int nit)
{
    for (int k : kv)
        run<O>(k, nit);
    if constexpr (O + 1 < O_N)
        run_all<O + 1>(kv, nit);
}

int main(int argc, char **argv)
{
    const int nit = argc > 1 ? atoi(argv[1]) : 256;
    CK(hipMalloc(&d_out, 256 * 256 * MAXK * ROUNDS * sizeof(u32)));
    CK(hipMalloc(&d_clk, 2 * 256 * MAXK * ROUNDS * 4 * sizeof(u64)));
    std::vector<int> kv = {3, 4, 8};
    run_all<0>(kv, nit);
    return 0;
}
