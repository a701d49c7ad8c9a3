// Probe: which access paths to VMM memory (hipMemCreate + hipMemMap) see the right bytes on this
// stack, under allocation churn.  Per iteration two buffers (~800 KB and 64 KiB) are made, written one
// way and read another, checked, freed:
//   path 0: kernel write -> kernel copy to a hipMalloc buffer -> D2H from it   (compute only)
//   path 1: kernel write -> D2H straight from the VMM buffer
//   path 2: H2D straight into the VMM buffer -> kernel copy to hipMalloc -> D2H
//   path 3: hipMemsetAsync on the VMM buffer -> kernel copy to hipMalloc -> D2H
// Address modes: A = a reservation per buffer, freed with it (hipMemAddressFree); B = a reservation per
// buffer never freed (the runtime cannot hand the same addresses out again).  Also reports how often a
// new reservation starts at an address freed before.
// hipcc --offload-arch=gfx950 -O2 scripts/vmm_path_probe.hip -o /tmp/vpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            printf("FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

static hipMemAllocationProp g_prop{};
static size_t g_gran = 4096;
static std::set<char *> g_freed;
static int g_reused = 0;

struct V {
    char * va;
    size_t n;
    hipMemGenericAllocationHandle_t h;
};
static V vmm(size_t bytes) {
    V v;
    v.n = (bytes + g_gran - 1) / g_gran * g_gran;
    CK(hipMemCreate(&v.h, v.n, &g_prop, 0));
    void * va;
    CK(hipMemAddressReserve(&va, v.n, 0, nullptr, 0));
    v.va = (char *)va;
    if (g_freed.count(v.va)) ++g_reused;
    CK(hipMemMap(v.va, v.n, 0, v.h, 0));
    hipMemAccessDesc acc{};
    acc.location = g_prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(v.va, v.n, &acc, 1));
    return v;
}
static void vfree(V & v, bool free_va) {
    CK(hipMemUnmap(v.va, v.n));
    if (free_va) {
        CK(hipMemAddressFree(v.va, v.n));
        g_freed.insert(v.va);
    }
    CK(hipMemRelease(v.h));
}

__global__ void k_fill(uint32_t * p, size_t n, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v ^ (uint32_t)i;
}
__global__ void k_copy(uint32_t * d, const uint32_t * s, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

int main() {
    CK(hipSetDevice(0));
    g_prop.type = hipMemAllocationTypePinned;
    g_prop.location.type = hipMemLocationTypeDevice;
    g_prop.location.id = 0;
    CK(hipMemGetAllocationGranularity(&g_gran, &g_prop, hipMemAllocationGranularityRecommended));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint32_t * stage;
    CK(hipMalloc(&stage, 1 << 20));
    std::vector<uint32_t> host(1 << 18), src(1 << 18);
    for (int amode = 0; amode < 2; ++amode) {
        for (int path = 0; path < 4; ++path) {
            int bad = 0;
            g_reused = 0;
            for (int it = 0; it < 200; ++it) {
                const size_t sizes[2] = {(size_t)(800000 + 4096 * (it % 50)) & ~(size_t)3, 65536};
                V v[2] = {vmm(sizes[0]), vmm(sizes[1])};
                bool ok = true;
                for (int k = 0; k < 2 && ok; ++k) {
                    const size_t n = sizes[k] / 4;
                    const uint32_t tag = 0x9E3779B9u * (uint32_t)(it * 2 + k + 1) + (uint32_t)(amode * 4 + path);
                    const uint32_t fillbyte = 0x10u + (uint32_t)((it * 2 + k) % 200);
                    if (path == 0 || path == 1) {
                        hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, st, (uint32_t *)v[k].va, n, tag);
                    } else if (path == 2) {
                        for (size_t i = 0; i < n; ++i) src[i] = tag ^ (uint32_t)i;
                        CK(hipMemcpyAsync(v[k].va, src.data(), n * 4, hipMemcpyHostToDevice, st));
                    } else {
                        CK(hipMemsetAsync(v[k].va, (int)fillbyte, n * 4, st));
                    }
                    if (path == 1) {
                        CK(hipMemcpyAsync(host.data(), v[k].va, n * 4, hipMemcpyDeviceToHost, st));
                    } else {
                        hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, st, stage, (const uint32_t *)v[k].va, n);
                        CK(hipMemcpyAsync(host.data(), stage, n * 4, hipMemcpyDeviceToHost, st));
                    }
                    CK(hipStreamSynchronize(st));
                    for (size_t i = 0; i < n; ++i) {
                        const uint32_t want = path == 3 ? fillbyte * 0x01010101u : tag ^ (uint32_t)i;
                        if (host[i] != want) {
                            if (bad < 3) printf("  addr %s path %d iter %d buf %d word %zu of %zu: %08x want %08x\n", amode ? "B" : "A", path, it, k, i, n,
                                                host[i], want);
                            ok = false;
                            break;
                        }
                    }
                }
                bad += !ok;
                vfree(v[1], amode == 0);
                vfree(v[0], amode == 0);
            }
            printf("address mode %s path %d: %d / 200 wrong (reservations at a freed address: %d)\n", amode ? "B(no free)" : "A(free)", path, bad,
                   g_reused);
            fflush(stdout);
        }
    }
    return 0;
}
