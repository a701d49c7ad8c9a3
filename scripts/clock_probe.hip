// Shader clock seen by a kernel: s_memtime (shader cycles) against s_memrealtime (100 MHz) over a
// dependent ALU loop, cold (first launch after idle) and inside a back-to-back stream of launches.
//   hipcc --offload-arch=gfx950 -O3 scripts/clock_probe.hip -o build/clock_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_clock(unsigned long long * out, int iters, float seed) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    float v = seed + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 64; ++k) v = __fmaf_rn(v, 1.0000001f, 0.5f);
    }
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = r1 - r0;
        out[1] = c1 - c0;
        out[2] = (unsigned long long)v;
    }
}

__global__ void k_busy(float * p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5f + 1.f;
}

int main() {
    unsigned long long * out;
    float * buf;
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&buf, 64 << 20));
    unsigned long long h[3];
    auto probe = [&](const char * tag) {
        hipLaunchKernelGGL(k_clock, dim3(256), dim3(64), 0, 0, out, 20000, 1.f);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, out, 24, hipMemcpyDeviceToHost));
        printf("{\"when\":\"%s\",\"real_us\":%.2f,\"cycles\":%llu,\"mhz\":%.0f,\"ns_per_dep_fma\":%.3f}\n", tag, h[0] / 100.0, h[1], h[1] / (h[0] / 100.0), h[0] * 10.0 / (20000.0 * 64));
    };
    probe("cold");
    probe("second");
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_busy, dim3(256), dim3(256), 0, 0, buf, 1 << 16);
    hipLaunchKernelGGL(k_clock, dim3(256), dim3(64), 0, 0, out, 20000, 1.f);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, out, 24, hipMemcpyDeviceToHost));
    printf("{\"when\":\"after_2000_short_kernels\",\"real_us\":%.2f,\"cycles\":%llu,\"mhz\":%.0f}\n", h[0] / 100.0, h[1], h[1] / (h[0] / 100.0));
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_busy, dim3(65536), dim3(256), 0, 0, buf, 1 << 24);
    hipLaunchKernelGGL(k_clock, dim3(256), dim3(64), 0, 0, out, 20000, 1.f);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, out, 24, hipMemcpyDeviceToHost));
    printf("{\"when\":\"after_200_streaming_kernels\",\"real_us\":%.2f,\"cycles\":%llu,\"mhz\":%.0f}\n", h[0] / 100.0, h[1], h[1] / (h[0] / 100.0));
    return 0;
}
