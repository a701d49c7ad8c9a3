// Peak rate of v_mfma_f64_16x16x4f64 on this GPU: every wave issues independent MFMAs into NACC
// accumulators; reports TFLOP/s over the whole chip for 1, 2 and 4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4_t __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_peak(double * out, int iters, double a0) {
    f64x4_t acc[NACC] = {};
    double a = a0 + threadIdx.x, b = a0 * 0.5 + blockIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
    }
    double s = 0;
    for (int t = 0; t < NACC; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
    if (s == 12345.0) out[0] = s;  // keep the loop
}

template <int NACC>
static void run(double * d) {
    const int iters = 16384 / NACC;
    for (int wpc : {4, 8, 16}) {  // waves per CU
        const int blocks = 256 * wpc / 4;
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        hipLaunchKernelGGL(k_peak<NACC>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_peak<NACC>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double flops = (double)blocks * 4 /*waves*/ * iters * NACC * 16 * 16 * 4 * 2;
        printf("{\"acc\": %d, \"waves_per_cu\": %d, \"ms\": %.3f, \"tflops_f64_mfma\": %.2f}\n", NACC, wpc, ms, flops / ms / 1e9);
    }
}

int main() {
    double * d;
    (void)hipMalloc(&d, 8);
    run<2>(d);
    run<4>(d);
    run<8>(d);
    return 0;
}
