// Which CUs / XCDs run a stream's kernels under hipExtStreamCreateWithCUMask (CU-partitioned
// replicas study): per workgroup, record HW_REG_XCC_ID and HW_REG_HW_ID, then histogram.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void probe(unsigned * out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // XCC_ID[3:0]
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
        long long t = clock64();
        while (clock64() - t < 20000) {}
    }
}

static void run(const char * name, std::vector<uint32_t> mask) {
    hipStream_t s;
    if (mask.empty()) hipStreamCreate(&s);
    else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) { printf("%s: mask refused\n", name); return; }
    const int nb = 2048;
    unsigned * d;
    hipMalloc(&d, 8 * nb);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    std::vector<unsigned> h(2 * nb);
    hipMemcpy(h.data(), d, 8 * nb, hipMemcpyDeviceToHost);
    std::set<unsigned> xccs, cus;
    int per_xcc[16] = {0};
    for (int i = 0; i < nb; ++i) {
        xccs.insert(h[2 * i]);
        per_xcc[h[2 * i] & 15]++;
        const unsigned hw = h[2 * i + 1];
        cus.insert((h[2 * i] << 16) | ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4) | (((hw >> 12) & 1) << 7));
    }
    printf("%-28s xccs=%zu distinct (xcc,se,sh,cu)=%zu per-xcc:", name, xccs.size(), cus.size());
    for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
    printf("\n");
    hipFree(d);
    hipStreamDestroy(s);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("CUs %d\n", p.multiProcessorCount);
    run("default", {});
    run("bits 0-31", {0xFFFFFFFFu, 0, 0, 0, 0, 0, 0, 0});
    run("bits 0-63", {0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0, 0, 0, 0, 0});
    run("bits 0-127", {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0, 0, 0});
    run("bits 128-255", {0, 0, 0, 0, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu});
    run("every 2nd bit", {0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u});
    run("every 8th bit", {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u});
    run("every 4th bit", {0x11111111u, 0x11111111u, 0x11111111u, 0x11111111u, 0x11111111u, 0x11111111u, 0x11111111u, 0x11111111u});
    return 0;
}
