// Standalone LayerNorm / RMSNorm (+ affine) replacing NORM -> MUL -> ADD
// (parler_build_layer_norm, model.cpp:412-418; dia_layer_norm / orpheus RMSNorm) wherever the
// output is not consumed by a Q4_K GEMV (those fold the norm into their prologue, k_gemv.hip).
// ggml_compute_forward_norm_f32 / rms_norm_f32 arithmetic exactly: f64 sums, mean and variance
// rounded to f32, scale = 1/sqrtf(var + eps), then MUL(w) and ADD(b) each rounded.
#include "hip_internal.h"

namespace tts {

// One workgroup (256 threads) per row; reductions by DPP within waves, then 4 wave partials.
template <bool RMS>
__global__ __launch_bounds__(256) void k_layernorm(TD dst, TD x, const float * __restrict__ w, const float * __restrict__ bias,
                                                   float eps) {
    __shared__ double shd[2][4];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % x.ne[1], i2 = (r / x.ne[1]) % x.ne[2], i3 = r / (x.ne[1] * x.ne[2]);
    const float * xr = (const float *)(x.data + i1 * x.nb[1] + i2 * x.nb[2] + i3 * x.nb[3]);
    float * yr = (float *)(dst.data + i1 * dst.nb[1] + i2 * dst.nb[2] + i3 * dst.nb[3]);
    const int n = (int)x.ne[0];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    auto bsum = [&](double v, int slot) {
        v = wave_sum_f64(v);
        if (lane == 0) shd[slot][wave] = v;
        __syncthreads();
        return ((shd[slot][0] + shd[slot][1]) + shd[slot][2]) + shd[slot][3];
    };
    float mean = 0.f;
    if (!RMS) {
        double s = 0.0;
        for (int i = tid; i < n; i += 256) s += (double)xr[i];
        mean = (float)(bsum(s, 0) / (double)n);
    }
    double s2 = 0.0;
    for (int i = tid; i < n; i += 256) {
        const float v = RMS ? xr[i] : __fsub_rn(xr[i], mean);
        s2 += (double)__fmul_rn(v, v);
    }
    const float var = (float)(bsum(s2, 1) / (double)n);
    const float scale = cr_divf(1.0f, cr_sqrtf(__fadd_rn(var, eps)));
    for (int i = tid; i < n; i += 256) {
        float v = RMS ? __fmul_rn(xr[i], scale) : __fmul_rn(__fsub_rn(xr[i], mean), scale);
        v = __fmul_rn(v, w[i]);
        if (!RMS) v = __fadd_rn(v, bias[i]);
        yr[i] = v;
    }
}

void launch_layernorm(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * x, const float * w, const float * b,
                      float eps, bool rms) {
    const int64_t nr = x->ne[1] * x->ne[2] * x->ne[3];
    if (rms)
        hipLaunchKernelGGL(k_layernorm<true>, dim3((unsigned)nr), dim3(256), 0, be->stream, make_td(dst), make_td(x), w, b, eps);
    else
        hipLaunchKernelGGL(k_layernorm<false>, dim3((unsigned)nr), dim3(256), 0, be->stream, make_td(dst), make_td(x), w, b, eps);
    TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
