// cpi.hip -- cycles per VALU instruction on gfx950, measured in-kernel with s_memtime.
// Each wave runs a long unrolled loop of one instruction pattern over 8 independent
// chains; waves per SIMD controlled by the grid (256 CUs x 4 SIMDs).  Prints cycles per
// wave-instruction per SIMD = (wave cycles) / (instructions) / (waves per SIMD)^-1 ...
// i.e. SIMD-cycles per instruction = wave_cycles * 1 / (instr_per_wave * waves_per_simd).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/diag/cpi tools/diag/cpi.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
typedef unsigned int u32;
typedef unsigned long long u64;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

constexpr int ITERS = 2048;
#define R8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define OUTS "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
#define KERN(NAME, BODY, NPER)                                                              \
__global__ __launch_bounds__(256) void NAME(u64 *out, u32 a0, u32 b0) {                       \
    u32 v0 = a0 + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ 9, v5 = v0 ^ 11, \
        v6 = v0 + 13, v7 = v0 + 17, b = b0 ^ threadIdx.x;                                    \
    u64 t0 = __builtin_amdgcn_s_memtime();                                                   \
    for (int i = 0; i < ITERS; i++) { asm volatile(BODY : OUTS : "v"(b)); }                  \
    u64 t1 = __builtin_amdgcn_s_memtime();                                                   \
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * 256 + threadIdx.x) >> 6] = t1 - t0;       \
    if ((v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7) == 0x12345) out[0] = 0;                        \
}                                                                                             \
constexpr int NAME##_n = NPER;
#define I_XOR(k) "v_xor_b32 %" #k ", %" #k ", %8\n"
#define I_ADDE64(k) "v_add_u32_e64 %" #k ", %" #k ", %8\n"
#define I_ALIGNBIT(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 7\n"
#define I_MULLO(k) "v_mul_lo_u32 %" #k ", %" #k ", %8\n"
#define I_MULHI(k) "v_mul_hi_u32 %" #k ", %" #k ", %8\n"
#define I_MAD24(k) "v_mad_u32_u24 %" #k ", %" #k ", %8, %" #k "\n"
#define I_QR(k) "v_add_u32 %" #k ", %" #k ", %8\n" "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 25\n" "v_xor_b32 %" #k ", %" #k ", %8\n"
#define I_XOR3(k) "v_bitop3_b32 %" #k ", %" #k ", %8, %" #k " bitop3:0x96\n"
KERN(k_xor, R8(I_XOR) R8(I_XOR), 16)
KERN(k_adde64, R8(I_ADDE64) R8(I_ADDE64), 16)
KERN(k_alignbit, R8(I_ALIGNBIT) R8(I_ALIGNBIT), 16)
KERN(k_qr, R8(I_QR), 24)
KERN(k_xor3, R8(I_XOR3) R8(I_XOR3), 16)
KERN(k_mullo, R8(I_MULLO) R8(I_MULLO), 16)
KERN(k_mulhi, R8(I_MULHI) R8(I_MULHI), 16)
KERN(k_mad24, R8(I_MAD24) R8(I_MAD24), 16)

// 64-bit accumulators: 8 independent v_mad_u64_u32 chains (the Poly1305 / X25519 column sums)
#define OUTS64 "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3), "+v"(w4), "+v"(w5), "+v"(w6), "+v"(w7)
#define I_MAD64(k) "v_mad_u64_u32 %" #k ", vcc, %8, %9, %" #k "\n"
__global__ __launch_bounds__(256) void k_mad64(u64 *out, u32 a0, u32 b0)
{
    u64 w0 = a0 + threadIdx.x, w1 = w0 * 3, w2 = w0 * 5, w3 = w0 * 7, w4 = w0 ^ 9, w5 = w0 ^ 11, w6 = w0 + 13,
        w7 = w0 + 17;
    u32 b = b0 ^ threadIdx.x, c = b * 7;
    u64 t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; i++) {
        asm volatile(R8(I_MAD64) R8(I_MAD64) : OUTS64 : "v"(b), "v"(c) : "vcc");
    }
    u64 t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * 256 + threadIdx.x) >> 6] = t1 - t0;
    if ((w0 ^ w1 ^ w2 ^ w3 ^ w4 ^ w5 ^ w6 ^ w7) == 0x12345) out[0] = 0;
}
constexpr int k_mad64_n = 16;

template <typename K>
void run(const char *name, K k, int nper, int wps, u64 *d, std::vector<u64> &h)
{
    int blocks = 256 * wps;  // 4 waves per block, 4 SIMDs per CU -> wps waves per SIMD
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u, 5u);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u, 5u);
    hipEventRecord(e1); CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    int nw = blocks * 4;
    CK(hipMemcpy(h.data(), d, nw * sizeof(u64), hipMemcpyDeviceToHost));
    std::vector<u64> v(h.begin(), h.begin() + nw);
    std::sort(v.begin(), v.end());
    double med = (double)v[nw / 2];
    double instr = (double)ITERS * nper;
    // wps waves share one SIMD: SIMD cycles per instruction = wave_cycles / (instr * wps)
    double cpi = med / (instr * wps);
    double clock = med / (ms * 1e-3) / 1e9;  // rough: wave lifetime ~ kernel time
    printf("%-10s wps=%d  wave cycles %.0f  instr/wave %.0f  SIMD-cycles/instr %.2f  (kernel %.3f ms, ~%.2f GHz)\n",
           name, wps, med, instr, cpi, ms, clock);
}

int main()
{
    u64 *d; CK(hipMalloc(&d, 256 * 8 * 4 * sizeof(u64)));
    std::vector<u64> h(256 * 8 * 4);
    for (int wps : {1, 2, 4, 8}) {
        run("xor", k_xor, k_xor_n, wps, d, h);
        run("add_e64", k_adde64, k_adde64_n, wps, d, h);
        run("alignbit", k_alignbit, k_alignbit_n, wps, d, h);
        run("xor3", k_xor3, k_xor3_n, wps, d, h);
        run("qr-step", k_qr, k_qr_n, wps, d, h);
        run("mul_lo", k_mullo, k_mullo_n, wps, d, h);
        run("mul_hi", k_mulhi, k_mulhi_n, wps, d, h);
        run("mad_u24", k_mad24, k_mad24_n, wps, d, h);
        run("mad_u64", k_mad64, k_mad64_n, wps, d, h);
    }
    return 0;
}
