// Probe: HIP virtual memory management on gfx950 -- one physical allocation mapped at two virtual
// addresses (its own range and a "window" that places several allocations at a fixed stride), as the
// step coalescer (graph_exec.hip) relies on.  Checks kernel / memcpy / memset coherence between the
// two mappings, graph replay through the window, and the streaming rate through either mapping.
// hipcc --offload-arch=gfx950 -O2 scripts/vmm_probe.hip -o /tmp/vmm_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void k_fill(float * p, size_t n, float base) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = base + (float)(i % 1000);
}
__global__ void k_sum(const float * p, size_t n, double * out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    atomicAdd(out, s);
}
__global__ void k_copy(const float4 * a, float4 * b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

int main() {
    CK(hipSetDevice(0));
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gmin = 0, grec = 0;
    CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
    CK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
    printf("granularity min %zu recommended %zu\n", gmin, grec);
    const size_t S = (size_t)256 << 20;  // per-allocation size
    const int N = 4;
    std::vector<hipMemGenericAllocationHandle_t> h(N);
    std::vector<void *> own(N);
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    for (int k = 0; k < N; ++k) {
        CK(hipMemCreate(&h[k], S, &prop, 0));
        CK(hipMemAddressReserve(&own[k], S, 0, nullptr, 0));
        CK(hipMemMap(own[k], S, 0, h[k], 0));
        CK(hipMemSetAccess(own[k], S, &acc, 1));
    }
    void * win = nullptr;
    CK(hipMemAddressReserve(&win, S * N, 0, nullptr, 0));
    for (int k = 0; k < N; ++k) CK(hipMemMap((char *)win + k * S, S, 0, h[k], 0));
    CK(hipMemSetAccess(win, S * N, &acc, 1));
    printf("own[0] %p win %p\n", own[0], win);
    hipPointerAttribute_t at{};
    const hipError_t pa = hipPointerGetAttributes(&at, own[0]);
    printf("pointer attrs own: %s type %d device %d\n", hipGetErrorString(pa), (int)at.type, at.device);
    const hipError_t pw = hipPointerGetAttributes(&at, win);
    printf("pointer attrs win: %s type %d device %d\n", hipGetErrorString(pw), (int)at.type, at.device);
    (void)hipGetLastError();

    hipStream_t st;
    CK(hipStreamCreate(&st));
    const size_t n = S / 4;
    bool ok = true;
    // 1. kernel writes through own[k], kernel reads through the window
    double * dsum;
    CK(hipMalloc(&dsum, sizeof(double) * N));
    CK(hipMemset(dsum, 0, sizeof(double) * N));
    for (int k = 0; k < N; ++k) hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, st, (float *)own[k], n, (float)(k * 10000));
    for (int k = 0; k < N; ++k) hipLaunchKernelGGL(k_sum, dim3(1024), dim3(256), 0, st, (const float *)((char *)win + k * S), n, dsum + k);
    std::vector<double> hs(N);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(hs.data(), dsum, sizeof(double) * N, hipMemcpyDeviceToHost));
    for (int k = 0; k < N; ++k) {
        double e = 0;
        for (size_t i = 0; i < n; ++i) e += (double)(float)((float)(k * 10000) + (float)(i % 1000));
        printf("member %d: window sum %.1f expected %.1f\n", k, hs[k], e);
        ok &= hs[k] == e;
    }
    // 2. H2D memcpy through own, D2H through window; memset through window, D2H through own
    std::vector<float> hv(1 << 20), hr(1 << 20);
    for (size_t i = 0; i < hv.size(); ++i) hv[i] = (float)i * 0.5f;
    CK(hipMemcpy((char *)own[2] + 4096, hv.data(), hv.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(hr.data(), (char *)win + 2 * S + 4096, hr.size() * 4, hipMemcpyDeviceToHost));
    bool m2 = hr == hv;
    CK(hipMemsetAsync((char *)win + 3 * S, 0x3F, 1 << 22, st));
    CK(hipMemcpyAsync(hr.data(), own[3], 1 << 22, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    const unsigned bits = 0x3F3F3F3Fu;
    bool m3 = true;
    for (size_t i = 0; i < hr.size(); ++i) m3 &= *(unsigned *)&hr[i] == bits;
    printf("memcpy own->win %s, memset win->own %s\n", m2 ? "ok" : "MISMATCH", m3 ? "ok" : "MISMATCH");
    ok &= m2 && m3;
    // 3. graph capture through the window, replayed after own[] contents change
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipMemset(dsum, 0, sizeof(double) * N));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < N; ++k) hipLaunchKernelGGL(k_sum, dim3(1024), dim3(256), 0, st, (const float *)((char *)win + k * S), n, dsum + k);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int k = 0; k < N; ++k) hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, st, (float *)own[k], n, 1.0f);
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(hs.data(), dsum, sizeof(double) * N, hipMemcpyDeviceToHost));
    double e1 = 0;
    for (size_t i = 0; i < n; ++i) e1 += (double)(1.0f + (float)(i % 1000));
    bool m4 = true;
    for (int k = 0; k < N; ++k) m4 &= hs[k] == e1;
    printf("graph replay through window %s\n", m4 ? "ok" : "MISMATCH");
    ok &= m4;
    // 4. streaming copy rate through own vs window (TLB / mapping cost)
    auto rate = [&](const char * a, char * b) {
        const size_t n4 = S / 16;
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, st, (const float4 *)a, (float4 *)b, n4);
        CK(hipStreamSynchronize(st));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, st));
        for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, st, (const float4 *)a, (float4 *)b, n4);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return 10.0 * 2.0 * S / (ms * 1e-3) / 1e9;
    };
    printf("copy GB/s own->own %.0f, win->win %.0f\n", rate((char *)own[0], (char *)own[1]), rate((char *)win, (char *)win + S));
    for (int k = 0; k < N; ++k) CK(hipMemUnmap((char *)win + k * S, S));
    CK(hipMemAddressFree(win, S * N));
    for (int k = 0; k < N; ++k) {
        CK(hipMemUnmap(own[k], S));
        CK(hipMemAddressFree(own[k], S));
        CK(hipMemRelease(h[k]));
    }
    printf(ok ? "VMM PROBE OK\n" : "VMM PROBE FAILED\n");
    return ok ? 0 : 2;
}
