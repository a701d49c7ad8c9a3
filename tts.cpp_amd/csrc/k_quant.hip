// Weight quantizers on the device: ggml's quantize_row_q4_K_ref and quantize_row_q8_0_ref
// (ggml-quants.c; restated in oracle/ggml_ref.c), so f32 weights can be turned into GGUF-compatible
// Q4_K / Q8_0 bytes where they live (the reference's examples/quantize path, quantize_impl.cpp:82-292,
// does this on the CPU).  Every float operation is the reference's, in source order, rounded to f32
// (-ffp-contract=off; sqrt and division correctly rounded), so the bytes equal the CPU's.
//
// Q4_K: one octet of lanes per 256-value block.  Lane s owns sub-block s (32 values): the weighted
// min / scale search (make_qkx2_quants, 21 candidate scales) runs per lane; the block's max scale /
// min come from an octet max; the 6-bit scale / min codes are gathered with shuffles into the
// packed 12-byte layout by lane 0; each lane then writes its 4-bit codes, pairing with its
// neighbour for the nibble interleave (sub-blocks 2j and 2j+1 share bytes).
#include "hip_internal.h"

namespace tts {

namespace {

__device__ __forceinline__ int q_nearest_int(float fval) {
    const float val = __fadd_rn(fval, 12582912.f);
    return (__float_as_int(val) & 0x007fffff) - 0x00400000;
}

// ggml_compute_fp32_to_fp16 (the FP16 library's scalar algorithm, RNE)
__device__ __forceinline__ uint16_t q_fp32_to_fp16(float f) {
    const float scale_to_inf = 0x1.0p+112f;
    const float scale_to_zero = 0x1.0p-110f;
    float base = __fmul_rn(__fmul_rn(fabsf(f), scale_to_inf), scale_to_zero);
    const uint32_t w = __float_as_uint(f);
    const uint32_t shl1_w = w + w;
    const uint32_t sign = w & 0x80000000u;
    uint32_t bias = shl1_w & 0xFF000000u;
    if (bias < 0x71000000u) bias = 0x71000000u;
    base = __fadd_rn(__uint_as_float((bias >> 1) + 0x07800000u), base);
    const uint32_t bits = __float_as_uint(base);
    const uint32_t exp_bits = (bits >> 13) & 0x00007C00u;
    const uint32_t mantissa_bits = bits & 0x00000FFFu;
    const uint32_t nonsign = exp_bits + mantissa_bits;
    return (uint16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

__device__ __forceinline__ float q_fp16_to_fp32(uint16_t h) { return __half2float(__ushort_as_half(h)); }

// make_qkx2_quants(32, 15, x, w, L, &min, Laux, -1, 0.1, 20, false) for one lane's sub-block
__device__ void q4k_search(const float * x, const float * w, uint8_t * L, float & the_min, float & the_scale) {
    float mn = x[0], mx = x[0];
    float sum_w = w[0];
    float sum_x = __fmul_rn(sum_w, x[0]);
    for (int i = 1; i < 32; ++i) {
        if (x[i] < mn) mn = x[i];
        if (x[i] > mx) mx = x[i];
        sum_w = __fadd_rn(sum_w, w[i]);
        sum_x = __fadd_rn(sum_x, __fmul_rn(w[i], x[i]));
    }
    if (mn > 0) mn = 0;
    if (mx == mn) {
        for (int i = 0; i < 32; ++i) L[i] = 0;
        the_min = -mn;
        the_scale = 0.f;
        return;
    }
    float iscale = cr_divf(15.f, __fsub_rn(mx, mn));
    float scale = cr_divf(1.f, iscale);
    float best_mad = 0;
    for (int i = 0; i < 32; ++i) {
        const int l = q_nearest_int(__fmul_rn(iscale, __fsub_rn(x[i], mn)));
        L[i] = (uint8_t)max(0, min(15, l));
        float diff = __fsub_rn(__fadd_rn(__fmul_rn(scale, (float)L[i]), mn), x[i]);
        diff = __fmul_rn(diff, diff);
        best_mad = __fadd_rn(best_mad, __fmul_rn(w[i], diff));
    }
    uint8_t Laux[32];
    for (int is = 0; is <= 20; ++is) {
        // (max - min) with the current min: an accepted candidate moves min for the later ones
        iscale = cr_divf(__fadd_rn(__fadd_rn(-1.f, __fmul_rn(0.1f, (float)is)), 15.f), __fsub_rn(mx, mn));
        float sum_l = 0, sum_l2 = 0, sum_xl = 0;
        for (int i = 0; i < 32; ++i) {
            int l = q_nearest_int(__fmul_rn(iscale, __fsub_rn(x[i], mn)));
            l = max(0, min(15, l));
            Laux[i] = (uint8_t)l;
            const float wl = __fmul_rn(w[i], (float)l);
            sum_l = __fadd_rn(sum_l, wl);
            sum_l2 = __fadd_rn(sum_l2, __fmul_rn(wl, (float)l));
            sum_xl = __fadd_rn(sum_xl, __fmul_rn(wl, x[i]));
        }
        const float D = __fsub_rn(__fmul_rn(sum_w, sum_l2), __fmul_rn(sum_l, sum_l));
        if (D > 0) {
            float this_scale = cr_divf(__fsub_rn(__fmul_rn(sum_w, sum_xl), __fmul_rn(sum_x, sum_l)), D);
            float this_min = cr_divf(__fsub_rn(__fmul_rn(sum_l2, sum_x), __fmul_rn(sum_l, sum_xl)), D);
            if (this_min > 0) {
                this_min = 0;
                this_scale = cr_divf(sum_xl, sum_l2);
            }
            float mad = 0;
            for (int i = 0; i < 32; ++i) {
                float diff = __fsub_rn(__fadd_rn(__fmul_rn(this_scale, (float)Laux[i]), this_min), x[i]);
                diff = __fmul_rn(diff, diff);
                mad = __fadd_rn(mad, __fmul_rn(w[i], diff));
            }
            if (mad < best_mad) {
                for (int i = 0; i < 32; ++i) L[i] = Laux[i];
                best_mad = mad;
                scale = this_scale;
                mn = this_min;
            }
        }
    }
    the_min = -mn;
    the_scale = scale;
}

__global__ __launch_bounds__(256) void k_quantize_q4_K(const float * __restrict__ x, uint8_t * __restrict__ dst, int64_t rows,
                                                      int64_t K) {
    const int lane = threadIdx.x & 63, s = lane & 7;
    const int64_t nbr = K / 256, nblk = rows * nbr;
    const int64_t blk = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3;
    const bool live = blk < nblk;
    const int64_t b = live ? blk : nblk - 1;  // dead octets shadow the last block (all lanes stay in the shuffles)
    const float * xs = x + (b / nbr) * K + (b % nbr) * 256 + 32 * s;
    float v[32], w[32];
    float sum_x2 = 0;
#pragma unroll
    for (int l = 0; l < 32; ++l) {
        v[l] = xs[l];
        sum_x2 = __fadd_rn(sum_x2, __fmul_rn(v[l], v[l]));
    }
    const float av_x = cr_sqrtf(__fmul_rn(sum_x2, 1.f / 32.f));  // sum_x2 / 32: exact power-of-two scaling
#pragma unroll
    for (int l = 0; l < 32; ++l) w[l] = __fadd_rn(av_x, fabsf(v[l]));
    uint8_t L[32];
    float mins, scales;
    q4k_search(v, w, L, mins, scales);
    // block max of the sub-block scales / mins (order-free)
    float max_scale = scales > 0 ? scales : 0.f, max_min = mins > 0 ? mins : 0.f;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        max_scale = fmaxf(max_scale, __shfl_xor(max_scale, o));
        max_min = fmaxf(max_min, __shfl_xor(max_min, o));
    }
    const float inv_scale = max_scale > 0 ? cr_divf(63.f, max_scale) : 0.f;
    const float inv_min = max_min > 0 ? cr_divf(63.f, max_min) : 0.f;
    const int ls = min(63, (int)(uint8_t)q_nearest_int(__fmul_rn(inv_scale, scales)));
    const int lm = min(63, (int)(uint8_t)q_nearest_int(__fmul_rn(inv_min, mins)));
    const uint16_t dh = q_fp32_to_fp16(cr_divf(max_scale, 63.f)), mh = q_fp32_to_fp16(cr_divf(max_min, 63.f));
    // get_scale_min_k4 of the packed codes is (ls, lm) itself for every sub-block
    const float d = __fmul_rn(q_fp16_to_fp32(dh), (float)ls);
    if (d != 0.f) {
        const float dm = __fmul_rn(q_fp16_to_fp32(mh), (float)lm);
#pragma unroll
        for (int ii = 0; ii < 32; ++ii) {
            const int l = q_nearest_int(cr_divf(__fadd_rn(v[ii], dm), d));
            L[ii] = (uint8_t)max(0, min(15, l));
        }
    }
    uint8_t * y = dst + b * 144;
    // 12-byte scale / min layout, assembled by lane 0 of the octet from all eight (ls, lm)
    int lsv[8], lmv[8];
    const int base = lane & ~7;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        lsv[j] = __shfl(ls, base + j);
        lmv[j] = __shfl(lm, base + j);
    }
    // nibble interleave: byte l of 64-value group g = L(sub 2g)[l] | L(sub 2g+1)[l] << 4
    uint32_t mine[8], other[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) mine[q] = (uint32_t)L[4 * q] | ((uint32_t)L[4 * q + 1] << 8) | ((uint32_t)L[4 * q + 2] << 16) | ((uint32_t)L[4 * q + 3] << 24);
#pragma unroll
    for (int q = 0; q < 8; ++q) other[q] = (uint32_t)__shfl_xor((int)mine[q], 1);
    if (!live) return;
    if (s == 0) {
        uint8_t sc[12] = {};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < 4) {
                sc[j] = (uint8_t)lsv[j];
                sc[j + 4] = (uint8_t)lmv[j];
            } else {
                sc[j + 4] = (uint8_t)((lsv[j] & 0xF) | ((lmv[j] & 0xF) << 4));
                sc[j - 4] |= (uint8_t)((lsv[j] >> 4) << 6);
                sc[j] |= (uint8_t)((lmv[j] >> 4) << 6);
            }
        }
        y[0] = (uint8_t)(dh & 0xFF), y[1] = (uint8_t)(dh >> 8);
        y[2] = (uint8_t)(mh & 0xFF), y[3] = (uint8_t)(mh >> 8);
#pragma unroll
        for (int j = 0; j < 12; ++j) y[4 + j] = sc[j];
    }
    if ((s & 1) == 0) {  // even lane: low nibbles mine, high nibbles from lane s + 1
        uint32_t * q = (uint32_t *)(y + 16 + 32 * (s >> 1));
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = (mine[k] & 0x0F0F0F0Fu) | ((other[k] & 0x0F0F0F0Fu) << 4);
    }
}

// quantize_row_q8_0_ref: one thread per 32-value block
__global__ __launch_bounds__(256) void k_quantize_q8_0(const float * __restrict__ x, uint8_t * __restrict__ dst, int64_t rows, int64_t K) {
    const int64_t nbr = K / 32, nblk = rows * nbr;
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblk) return;
    const float * xs = x + (b / nbr) * K + (b % nbr) * 32;
    float amax = 0.0f;
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(xs[j]));
    const float d = cr_divf(amax, 127.f);
    const float id = d != 0.f ? cr_divf(1.0f, d) : 0.0f;
    uint8_t * y = dst + b * 34;
    const uint16_t dh = q_fp32_to_fp16(d);
    y[0] = (uint8_t)(dh & 0xFF), y[1] = (uint8_t)(dh >> 8);
    for (int j = 0; j < 32; ++j) y[2 + j] = (uint8_t)(int8_t)roundf(__fmul_rn(xs[j], id));
}

}  // namespace

}  // namespace tts

extern "C" int tts_hip_quantize(tts_hip_backend_t be, int type, const float * x, void * dst, int64_t rows, int64_t K) {
    if (!be || !x || !dst || rows <= 0 || K <= 0) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    if (type == TTS_TYPE_Q4_K) {
        if (K % 256) return TTS_STATUS_BAD_ARG;
        const int64_t threads = rows * (K / 256) * 8;
        hipLaunchKernelGGL(tts::k_quantize_q4_K, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, be->stream, x, (uint8_t *)dst, rows, K);
    } else if (type == TTS_TYPE_Q8_0) {
        if (K % 32) return TTS_STATUS_BAD_ARG;
        const int64_t nblk = rows * (K / 32);
        hipLaunchKernelGGL(tts::k_quantize_q8_0, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, be->stream, x, (uint8_t *)dst, rows, K);
    } else {
        return TTS_STATUS_UNSUPPORTED;
    }
    TTS_HIP_CHECK(hipGetLastError());
    return 0;
}
