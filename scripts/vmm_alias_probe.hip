// Probe: do VMM allocations alias each other (or hipMalloc memory) under churn?  Per iteration, four
// buffers are made (three ~1 MB, one 64 KiB), each filled with its own byte by hipMemsetAsync, then
// every buffer's first and last 4 KiB are read back and checked; the reserved ranges are checked for
// overlap with the live ones.  Mode 0: a reservation per buffer (hipMemAddressReserve / Free), as
// tts_hip_buffer_alloc did; mode 1: one big reservation made once, every iteration's buffers carved
// from its start (the same addresses each time: new physical memory mapped where the previous
// iteration's was); mode 2: the big reservation carved without reuse (addresses never seen before).
// hipcc --offload-arch=gfx950 -O2 scripts/vmm_alias_probe.hip -o /tmp/vap
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            printf("FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

static size_t g_gran = 0;
static hipMemAllocationProp g_prop{};
static char * g_big = nullptr;
static size_t g_big_n = 0, g_big_off = 0;

struct V {
    char * va;
    size_t n;
    hipMemGenericAllocationHandle_t h;
};

static V vmm(size_t bytes, int mode) {
    V v;
    v.n = (bytes + g_gran - 1) / g_gran * g_gran;
    CK(hipMemCreate(&v.h, v.n, &g_prop, 0));
    if (mode >= 1) {
        if (g_big_off + v.n > g_big_n) g_big_off = 0;
        v.va = g_big + g_big_off;
        g_big_off += v.n;
    } else {
        void * va;
        CK(hipMemAddressReserve(&va, v.n, 0, nullptr, 0));
        v.va = (char *)va;
    }
    CK(hipMemMap(v.va, v.n, 0, v.h, 0));
    hipMemAccessDesc acc{};
    acc.location = g_prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(v.va, v.n, &acc, 1));
    return v;
}
static void vfree(V & v, int mode) {
    CK(hipMemUnmap(v.va, v.n));
    if (mode == 0) CK(hipMemAddressFree(v.va, v.n));
    CK(hipMemRelease(v.h));
}

int main() {
    CK(hipSetDevice(0));
    g_prop.type = hipMemAllocationTypePinned;
    g_prop.location.type = hipMemLocationTypeDevice;
    g_prop.location.id = 0;
    CK(hipMemGetAllocationGranularity(&g_gran, &g_prop, hipMemAllocationGranularityRecommended));
    size_t gmin = 0;
    CK(hipMemGetAllocationGranularity(&gmin, &g_prop, hipMemAllocationGranularityMinimum));
    printf("granularity recommended %zu minimum %zu\n", g_gran, gmin);
    g_big_n = (size_t)16 << 30;
    void * big;
    CK(hipMemAddressReserve(&big, g_big_n, 0, nullptr, 0));
    g_big = (char *)big;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    char * d;
    CK(hipMalloc(&d, 1 << 20));
    std::vector<unsigned char> host(4096);
    for (int mode = 0; mode < 3; ++mode) {
        int bad = 0, overlap = 0;
        if (mode == 2) g_big_off = (size_t)8 << 30;  // addresses mode 1 never touched
        for (int it = 0; it < 300; ++it) {
            const size_t sizes[4] = {(size_t)(800000 + 4096 * (it % 50)), (size_t)(800000 + 4096 * (it % 50)), 65536, 65536};
            V v[4];
            for (int k = 0; k < 4; ++k) {
                v[k] = vmm(sizes[k], mode);
                for (int u = 0; u < k; ++u)
                    if (v[k].va < v[u].va + v[u].n && v[u].va < v[k].va + v[k].n) {
                        if (overlap < 5) printf("mode %d iter %d: range %d overlaps range %d\n", mode, it, k, u);
                        ++overlap;
                    }
                if (v[k].va < d + (1 << 20) && d < v[k].va + v[k].n) {
                    if (overlap < 5) printf("mode %d iter %d: range %d overlaps the hipMalloc buffer\n", mode, it, k);
                    ++overlap;
                }
            }
            CK(hipMemsetAsync(d, 0xEE, 1 << 20, st));
            for (int k = 0; k < 4; ++k) CK(hipMemsetAsync(v[k].va, 0x11 * (k + 1), sizes[k], st));
            CK(hipStreamSynchronize(st));
            bool ok = true;
            for (int k = 0; k < 4 && ok; ++k) {
                for (int e = 0; e < 2 && ok; ++e) {
                    const size_t off = e ? sizes[k] - 4096 : 0;
                    CK(hipMemcpyAsync(host.data(), v[k].va + off, 4096, hipMemcpyDeviceToHost, st));
                    CK(hipStreamSynchronize(st));
                    for (int i = 0; i < 4096; ++i)
                        if (host[i] != (unsigned char)(0x11 * (k + 1))) {
                            if (bad < 8) printf("mode %d iter %d: buffer %d (%s) byte %d = %02x, expected %02x\n", mode, it, k, e ? "tail" : "head", i, host[i], 0x11 * (k + 1));
                            ok = false;
                            break;
                        }
                }
            }
            CK(hipMemcpyAsync(host.data(), d, 4096, hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            if (host[0] != 0xEE || host[4095] != 0xEE) {
                if (bad < 8) printf("mode %d iter %d: hipMalloc buffer overwritten (%02x)\n", mode, it, host[0]);
                ok = false;
            }
            bad += !ok;
            for (int k = 3; k >= 0; --k) vfree(v[k], mode);
            if (mode == 1) g_big_off = 0;
        }
        printf("mode %d: %d / 300 iterations wrong, %d overlaps\n", mode, bad, overlap);
    }
    return 0;
}
