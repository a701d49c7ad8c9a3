// Latency probe (one wave, s_memrealtime at 100 MHz): kernel-argument scalar load, global load
// (cold HBM / warm L2), and a kernel-entry-to-first-instruction spread.  Informs how many serial
// memory round trips a decode kernel can afford.
//   hipcc --offload-arch=gfx950 -O3 scripts/latency_probe.hip -o build/latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Args {
    const float * cold;
    const float * warm;
    unsigned long long * out;
    int pad[60];
};

__global__ void k_probe(Args a) {
    if (threadIdx.x != 0) return;
    const volatile int * ka = (const volatile int *)__builtin_amdgcn_kernarg_segment_ptr();
    unsigned long long t[8];
    t[0] = __builtin_amdgcn_s_memrealtime();
    int s = ka[40];  // a kernarg dword not needed so far
    t[1] = __builtin_amdgcn_s_memrealtime();
    s += ka[50];
    t[2] = __builtin_amdgcn_s_memrealtime();
    float v = *(const volatile float *)(a.cold + (size_t)blockIdx.x * 4096);
    t[3] = __builtin_amdgcn_s_memrealtime();
    v += *(const volatile float *)(a.warm);
    t[4] = __builtin_amdgcn_s_memrealtime();
    v += *(const volatile float *)(a.warm + 1);
    t[5] = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < 6; ++i) a.out[blockIdx.x * 8 + i] = t[i];
    a.out[blockIdx.x * 8 + 6] = (unsigned long long)(s + (int)v);
}

int main() {
    float *cold, *warm;
    unsigned long long * out;
    CK(hipMalloc(&cold, 512ull << 20));
    CK(hipMemset(cold, 0, 512ull << 20));
    CK(hipMalloc(&warm, 4096));
    CK(hipMemset(warm, 0, 4096));
    CK(hipMalloc(&out, 256 * 8 * 8));
    Args a{};
    a.warm = warm;
    a.out = out;
    unsigned long long h[256 * 8];
    for (int rep = 0; rep < 3; ++rep) {
        a.cold = cold + (size_t)rep * (64u << 20) / 4;  // fresh lines every repetition
        hipLaunchKernelGGL(k_probe, dim3(64), dim3(64), 0, 0, a);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, out, sizeof(h[0]) * 64 * 8, hipMemcpyDeviceToHost));
        double ka1 = 0, ka2 = 0, cold_us = 0, l2a = 0, l2b = 0;
        for (int b = 0; b < 64; ++b) {
            ka1 += (h[b * 8 + 1] - h[b * 8 + 0]) / 100.0;
            ka2 += (h[b * 8 + 2] - h[b * 8 + 1]) / 100.0;
            cold_us += (h[b * 8 + 3] - h[b * 8 + 2]) / 100.0;
            l2a += (h[b * 8 + 4] - h[b * 8 + 3]) / 100.0;
            l2b += (h[b * 8 + 5] - h[b * 8 + 4]) / 100.0;
        }
        printf("{\"rep\":%d,\"kernarg_load_us\":%.3f,\"kernarg_load2_us\":%.3f,\"global_cold_us\":%.3f,\"global_warm1_us\":%.3f,\"global_warm2_us\":%.3f}\n",
               rep, ka1 / 64, ka2 / 64, cold_us / 64, l2a / 64, l2b / 64);
    }
    return 0;
}
