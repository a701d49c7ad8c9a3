// Probe: host <-> VMM-mapped device copies of several sizes and APIs (pageable / pinned host memory,
// hipMemcpy / hipMemcpyAsync on a non-blocking stream), each checked by reading the bytes back through
// a plain hipMalloc buffer.  hipcc --offload-arch=gfx950 -O2 scripts/vmm_copy_probe.hip -o /tmp/vcp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

static void * vmm(size_t n, size_t * msz) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t g = 0;
    CK(hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended));
    *msz = (n + g - 1) / g * g;
    hipMemGenericAllocationHandle_t h;
    CK(hipMemCreate(&h, *msz, &prop, 0));
    void * va;
    CK(hipMemAddressReserve(&va, *msz, 0, nullptr, 0));
    CK(hipMemMap(va, *msz, 0, h, 0));
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(va, *msz, &acc, 1));
    return va;
}

int main() {
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const size_t sizes[] = {4096, 700 << 10, 1 << 20, (1 << 20) + 4096, 1089536, 4 << 20, 33 << 20};
    int bad = 0;
    for (size_t n : sizes) {
        size_t ms;
        char * d = (char *)vmm(n, &ms);
        char * plain;
        CK(hipMalloc(&plain, n));
        std::vector<char> src(n), back(n);
        char * pin;
        CK(hipHostMalloc(&pin, n, hipHostMallocDefault));
        for (int mode = 0; mode < 4; ++mode) {
            for (size_t i = 0; i < n; ++i) src[i] = (char)(i * 7 + mode * 13 + 1);
            CK(hipMemset(d, 0, n));
            CK(hipDeviceSynchronize());
            const char * from = src.data();
            if (mode == 2 || mode == 3) {
                memcpy(pin, src.data(), n);
                from = pin;
            }
            if (mode == 0 || mode == 2) CK(hipMemcpy(d, from, n, hipMemcpyHostToDevice));
            else {
                CK(hipMemcpyAsync(d, from, n, hipMemcpyHostToDevice, st));
                CK(hipStreamSynchronize(st));
            }
            // read back H2D result via device-to-device into plain memory, then D2H from plain
            CK(hipMemcpy(plain, d, n, hipMemcpyDeviceToDevice));
            CK(hipMemcpy(back.data(), plain, n, hipMemcpyDeviceToHost));
            const bool h2d = back == src;
            // D2H straight from the VMM buffer, async on the stream to pageable memory
            std::fill(back.begin(), back.end(), 0);
            CK(hipMemcpyAsync(back.data(), d, n, hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            const bool d2h = back == src;
            printf("size %zu mode %d (%s %s): H2D %s, async D2H %s\n", n, mode, mode >= 2 ? "pinned" : "pageable",
                   (mode & 1) ? "async" : "sync", h2d ? "ok" : "WRONG", d2h ? "ok" : "WRONG");
            bad += !h2d + !d2h;
        }
        CK(hipHostFree(pin));
        CK(hipFree(plain));
    }
    printf(bad ? "VMM COPY PROBE: %d failures\n" : "VMM COPY PROBE OK\n", bad);
    return bad ? 2 : 0;
}
