// latency_ub.hip -- host-visible latency floors for a one-message call on MI355X (diagnostics).
//
// What one jnacl-style call (host buffer in, host buffer out, one message) can cost at best:
//   launch+sync        an empty kernel, hipStreamSynchronize
//   mapped rw N        one workgroup reads N bytes from pinned host memory and writes N bytes back
//                      (zero-copy: the kernel touches host memory over PCIe directly)
//   copy+kernel+copy N hipMemcpyAsync H2D, an empty kernel, D2H, sync (pinned buffers)
// Wall clock of the host thread, median of many calls, after warm-up.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/diag/latency_ub tools/diag/latency_ub.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__global__ void k_empty(int *flag)
{
    if (threadIdx.x == 0 && flag)
        *flag = 1;
}

__global__ __launch_bounds__(256) void k_mapped(const uint4 *in, uint4 *out, unsigned n16)
{
    for (unsigned i = threadIdx.x; i < n16; i += blockDim.x) {
        uint4 v = in[i];
        v.x ^= 0x5a5a5a5au;
        out[i] = v;
    }
}

template <class F>
double median_us(F f, int reps = 2000)
{
    for (int i = 0; i < 50; i++)
        f();
    std::vector<double> t;
    t.reserve(reps);
    for (int i = 0; i < reps; i++) {
        auto a = std::chrono::steady_clock::now();
        f();
        auto b = std::chrono::steady_clock::now();
        t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv)
{
    if (argc > 1 && argv[1][0] == 's')  // "spin": host threads spin instead of yielding in syncs
        CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    if (argc > 1 && argv[1][0] == 'b')  // "block"
        CK(hipSetDeviceFlags(hipDeviceScheduleBlockingSync));
    printf("-- schedule mode: %s\n", argc > 1 ? argv[1] : "default");
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t cap = 1 << 17;
    uint8_t *hin, *hout, *din, *dout;
    CK(hipHostMalloc((void **)&hin, cap, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&hout, cap, hipHostMallocDefault));
    CK(hipMalloc((void **)&din, cap));
    CK(hipMalloc((void **)&dout, cap));
    memset(hin, 1, cap);
    int *dflag;
    CK(hipMalloc((void **)&dflag, 64));

    printf("launch+sync (empty kernel)        %7.2f us\n", median_us([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, dflag);
               CK(hipStreamSynchronize(s));
           }));
    printf("launch+sync (empty, null stream)  %7.2f us\n", median_us([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, dflag);
               CK(hipStreamSynchronize(0));
           }));
    for (unsigned n : {128u, 4096u, 65536u}) {
        char name[64];
        snprintf(name, sizeof name, "mapped rw %u B", n);
        printf("%-33s %7.2f us\n", name, median_us([&] {
                   hipLaunchKernelGGL(k_mapped, dim3(1), dim3(256), 0, s, (const uint4 *)hin, (uint4 *)hout, n / 16);
                   CK(hipStreamSynchronize(s));
               }));
        snprintf(name, sizeof name, "copy+kernel+copy %u B", n);
        printf("%-33s %7.2f us\n", name, median_us([&] {
                   CK(hipMemcpyAsync(din, hin, n, hipMemcpyHostToDevice, s));
                   hipLaunchKernelGGL(k_mapped, dim3(1), dim3(256), 0, s, (const uint4 *)din, (uint4 *)dout, n / 16);
                   CK(hipMemcpyAsync(hout, dout, n, hipMemcpyDeviceToHost, s));
                   CK(hipStreamSynchronize(s));
               }));
    }
    printf("launch + hipStreamQuery spin      %7.2f us\n", median_us([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, dflag);
               while (hipStreamQuery(s) == hipErrorNotReady) {
               }
           }));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    printf("launch + event query spin         %7.2f us\n", median_us([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, dflag);
               CK(hipEventRecord(ev, s));
               while (hipEventQuery(ev) == hipErrorNotReady) {
               }
           }));
    printf("launch API call only (no wait)    %7.2f us\n", median_us([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, dflag);
           }, 500));
    CK(hipStreamSynchronize(s));
    // the same, spinning on a host flag the kernel writes instead of hipStreamSynchronize
    volatile int *hflag;
    CK(hipHostMalloc((void **)&hflag, 64, hipHostMallocCoherent));
    printf("launch + spin on host flag        %7.2f us\n", median_us([&] {
               *hflag = 0;
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, (int *)hflag);
               while (*hflag == 0) {
               }
               CK(hipStreamSynchronize(s));
           }));
    return 0;
}
