// Streaming-copy variants on MI355X (read + write bytes / s), to pick the form of k_copy_stream
// (tts_hip_copy_stream, the bench's measured HBM ceiling).  hipcc --offload-arch=gfx950 -O3 copy_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

// grid-stride, U loads in flight per lane, NT or plain
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stride(u4v * __restrict__ d, const u4v * __restrict__ s, int64_t n) {
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * gs < n; i += U * gs) {
        u4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * gs) : s[i + u * gs];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], d + i + u * gs);
            else d[i + u * gs] = v[u];
        }
    }
    for (; i < n; i += gs) d[i] = s[i];
}

// each workgroup copies one contiguous chunk, U consecutive 4 KB pieces per iteration
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_chunk(u4v * __restrict__ d, const u4v * __restrict__ s, int64_t n) {
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    int64_t i = b0 + threadIdx.x;
    for (; i + (U - 1) * 256 < b1; i += U * 256) {
        u4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * 256) : s[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], d + i + u * 256);
            else d[i + u * 256] = v[u];
        }
    }
    for (; i < b1; i += 256) d[i] = s[i];
}

template <typename K>
static void run(const char * name, K k, int grid, u4v * d, const u4v * s, int64_t n) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, s, n);
    hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, s, n);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s grid %6d: %7.1f GB/s\n", name, grid, 2.0 * n * 16 * reps / (ms * 1e-3) / 1e9);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (size_t bytes : {(size_t)1 << 30, (size_t)4 << 30}) {
        const int64_t n = (int64_t)(bytes / 16);
        u4v *s, *d;
        if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
        hipMemset(s, 1, bytes);
        printf("copy of %zu MiB (CUs %d)\n", bytes >> 20, cus);
        for (int g : {cus * 4, cus * 8, cus * 16}) {
            run("stride U4 nt", k_stride<4, true>, g, d, s, n);
            run("stride U4 plain", k_stride<4, false>, g, d, s, n);
            run("stride U8 nt", k_stride<8, true>, g, d, s, n);
            run("stride U8 plain", k_stride<8, false>, g, d, s, n);
            run("chunk U4 nt", k_chunk<4, true>, g, d, s, n);
            run("chunk U4 plain", k_chunk<4, false>, g, d, s, n);
            run("chunk U8 nt", k_chunk<8, true>, g, d, s, n);
            run("chunk U8 plain", k_chunk<8, false>, g, d, s, n);
        }
        hipFree(s);
        hipFree(d);
    }
    return 0;
}
