// Micro-benchmark: cost of a device-wide barrier inside one persistent kernel vs. the cost of a
// dependent kernel boundary (eager launches and HIP-graph replay).  Decides whether the decode step
// should run as a persistent "phase interpreter" or as a graph of fused kernels.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench_sync.hip -o build/microbench_sync
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Bar { unsigned count; unsigned gen; unsigned fail; unsigned pad; };

__device__ __forceinline__ bool grid_barrier(Bar * b, unsigned nblocks) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        __threadfence();
        unsigned g = __hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        unsigned arrived = __hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nblocks - 1) {
            __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&b->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            long spins = 0;
            while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spins > (1L << 24)) { atomicOr(&b->fail, 1u); ok = false; break; }   // never hang
            }
        }
    }
    __syncthreads();
    return ok;
}

__global__ void k_persistent(Bar * b, float * buf, int iters) {
    const unsigned nb = gridDim.x;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        // a little dependent work per phase: read a neighbour's value written last phase
        if (threadIdx.x == 0) {
            acc += buf[(blockIdx.x + it) % nb];
            buf[blockIdx.x] = acc;
        }
        if (!grid_barrier(b, nb)) return;
    }
}

__global__ void k_tiny(float * buf, int it) {
    if (threadIdx.x == 0) buf[blockIdx.x] += buf[(blockIdx.x + it) % gridDim.x];
}

int main(int argc, char ** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 2000;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int ncu = prop.multiProcessorCount;
    printf("device %s CUs %d\n", prop.name, ncu);
    Bar * b; float * buf;
    CK(hipMalloc(&b, sizeof(Bar)));
    CK(hipMalloc(&buf, 4096 * sizeof(float)));
    hipStream_t s; CK(hipStreamCreate(&s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));

    for (int nblk : {ncu / 8, ncu / 2, ncu, 2 * ncu}) {
        for (int threads : {64, 256}) {
            int maxb = 0;
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&maxb, k_persistent, threads, 0));
            if (nblk > maxb * ncu) continue;
            CK(hipMemset(b, 0, sizeof(Bar)));
            void * args[] = {&b, &buf, &iters};
            // warm
            CK(hipLaunchCooperativeKernel((void *) k_persistent, dim3(nblk), dim3(threads), args, 0, s));
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            CK(hipLaunchCooperativeKernel((void *) k_persistent, dim3(nblk), dim3(threads), args, 0, s));
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            Bar hb; CK(hipMemcpy(&hb, b, sizeof(Bar), hipMemcpyDeviceToHost));
            printf("{\"test\":\"grid_barrier\",\"blocks\":%d,\"threads\":%d,\"iters\":%d,\"us_per_barrier\":%.3f,\"fail\":%u}\n",
                   nblk, threads, iters, 1000.f * ms / iters, hb.fail);
        }
    }

    for (int nblk : {1, ncu}) {
        // eager dependent launches
        for (int i = 0; i < 50; ++i) k_tiny<<<nblk, 64, 0, s>>>(buf, i);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; ++i) k_tiny<<<nblk, 64, 0, s>>>(buf, i);
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"test\":\"eager_chain\",\"blocks\":%d,\"iters\":%d,\"us_per_kernel\":%.3f}\n", nblk, iters, 1000.f * ms / iters);

        // graph replay of the same chain
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < iters; ++i) k_tiny<<<nblk, 64, 0, s>>>(buf, i);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"test\":\"graph_chain\",\"blocks\":%d,\"iters\":%d,\"us_per_kernel\":%.3f}\n", nblk, iters, 1000.f * ms / iters);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    CK(hipFree(b)); CK(hipFree(buf));
    return 0;
}
