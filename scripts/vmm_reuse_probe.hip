// Probe: a VMM allocation freed (unmap, free range, release) and a new one of the same size made: is the
// range reused, and do kernels see the new allocation's bytes?  (Stale GPU translations of a reused
// virtual range would show the old physical pages.)  hipcc --offload-arch=gfx950 -O2 scripts/vmm_reuse_probe.hip
#include <hip/hip_runtime.h>

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

struct V {
    void * va;
    size_t n;
    hipMemGenericAllocationHandle_t h;
};
static V vmm(size_t n) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t g = 0;
    CK(hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended));
    V v;
    v.n = (n + g - 1) / g * g;
    CK(hipMemCreate(&v.h, v.n, &prop, 0));
    CK(hipMemAddressReserve(&v.va, v.n, 0, nullptr, 0));
    CK(hipMemMap(v.va, v.n, 0, v.h, 0));
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(v.va, v.n, &acc, 1));
    return v;
}
static void vfree(V & v, bool keep_va) {
    CK(hipMemUnmap(v.va, v.n));
    if (!keep_va) CK(hipMemAddressFree(v.va, v.n));
    CK(hipMemRelease(v.h));
}
__global__ void k_sum(const float * p, size_t n, double * out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    atomicAdd(out, s);
}
__global__ void k_fill(float * p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

int main() {
    CK(hipSetDevice(0));
    double * d;
    CK(hipMalloc(&d, 8));
    int bad = 0;
    for (int keep = 0; keep < 2; ++keep) {
        const size_t n = 1089536 / 4;
        void * prev = nullptr;
        for (int it = 0; it < 6; ++it) {
            V v = vmm(n * 4);
            std::vector<float> h(n, (float)(it + 1));
            CK(hipMemcpy(v.va, h.data(), n * 4, hipMemcpyHostToDevice));
            CK(hipMemset(d, 0, 8));
            hipLaunchKernelGGL(k_sum, dim3(256), dim3(256), 0, 0, (const float *)v.va, n, d);
            double s = 0;
            CK(hipMemcpy(&s, d, 8, hipMemcpyDeviceToHost));
            // the kernel writes, the host reads
            hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, (float *)v.va, n, 5.0f);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), v.va, n * 4, hipMemcpyDeviceToHost));
            const bool ok1 = s == (double)(it + 1) * n, ok2 = h[0] == 5.0f && h[n - 1] == 5.0f;
            printf("keep_va %d iter %d va %p (%s) kernel sum %s, kernel write %s\n", keep, it, v.va, v.va == prev ? "REUSED" : "new",
                   ok1 ? "ok" : "WRONG", ok2 ? "ok" : "WRONG");
            bad += !ok1 + !ok2;
            prev = v.va;
            vfree(v, keep);
        }
    }
    printf(bad ? "VMM REUSE PROBE: %d failures\n" : "VMM REUSE PROBE OK\n", bad);
    return bad ? 2 : 0;
}
