// Probe: churn of VMM allocations the way the op tests use buffers (several buffers made, filled from
// pageable host memory with hipMemcpyAsync + stream sync, read by one kernel, results read back, all
// freed), many times; variant 0 as tts_hip_buffer_alloc did it, variant 1 with a device-wide
// synchronize after mapping, variant 2 with a stream-ordered memset of the new range, variant 3 with
// the kernel's result written to a VMM buffer and read back from it (as the op tests read outputs),
// variant 4 = 3 with hipMalloc / hipFree churn of other sizes in between.
// hipcc --offload-arch=gfx950 -O2 scripts/vmm_stress_probe.hip -o /tmp/vsp
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
    char * va;
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
    void * va;
    CK(hipMemAddressReserve(&va, v.n, 0, nullptr, 0));
    v.va = (char *)va;
    CK(hipMemMap(v.va, v.n, 0, v.h, 0));
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(v.va, v.n, &acc, 1));
    return v;
}
static void vfree(V & v) {
    CK(hipMemUnmap(v.va, v.n));
    CK(hipMemAddressFree(v.va, v.n));
    CK(hipMemRelease(v.h));
}
__global__ void k_sum3(const float * a, const float * b, const float * c, size_t n, double * out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i] + b[i] + c[i % 1000];
    atomicAdd(out, s);
}

int main() {
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    double * d;
    CK(hipMalloc(&d, 8));
    for (int variant = 0; variant < 5; ++variant) {
        int bad = 0;
        for (int it = 0; it < 300; ++it) {
            const size_t n = (size_t)(200000 + 37 * it % 100000);
            void * junk = nullptr;
            if (variant == 4) CK(hipMalloc(&junk, (size_t)(1 + it % 7) << 20));
            V a = vmm(n * 4), b = vmm(n * 4), c = vmm(1000 * 4 > 65536 ? 4000 : 65536);
            V o = vmm(65536);
            double * dd = variant >= 3 ? (double *)o.va : d;
            if (variant == 1) CK(hipDeviceSynchronize());
            if (variant == 2) {
                CK(hipMemsetAsync(a.va, 0, n * 4, st));
                CK(hipMemsetAsync(b.va, 0, n * 4, st));
                CK(hipMemsetAsync(c.va, 0, 4000, st));
            }
            std::vector<float> ha(n, 1.0f), hb(n, 2.0f), hc(1000, 0.5f);
            CK(hipMemcpyAsync(a.va, ha.data(), n * 4, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            CK(hipMemcpyAsync(b.va, hb.data(), n * 4, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            CK(hipMemcpyAsync(c.va, hc.data(), 4000, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            CK(hipMemsetAsync(dd, 0, 8, st));
            hipLaunchKernelGGL(k_sum3, dim3(256), dim3(256), 0, st, (const float *)a.va, (const float *)b.va, (const float *)c.va, n, dd);
            double s = 0;
            CK(hipMemcpyAsync(&s, dd, 8, hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            const double e = 3.5 * (double)n;
            if (s != e) {
                if (bad < 5) printf("variant %d iter %d: sum %.1f expected %.1f\n", variant, it, s, e);
                ++bad;
            }
            vfree(o);
            vfree(c);
            vfree(b);
            vfree(a);
            if (junk) CK(hipFree(junk));
        }
        printf("variant %d: %d / 300 wrong\n", variant, bad);
    }
    return 0;
}
