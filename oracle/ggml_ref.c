/*
 * oracle/ggml_ref.c — TEST INFRASTRUCTURE ONLY (see ggml_ref.h header for pinning status).
 *
 * Restatement of ggml-cpu scalar semantics for the ops emitted by TTS.cpp graph builders:
 *   Parler step   /root/reference/src/models/parler/model.cpp:387-614
 *   DAC / codec   /root/reference/src/decoder/dac_model.cpp:100-170,
 *                 /root/reference/src/decoder/general_neural_audio_codec.cpp:133-172
 *   helpers       /root/reference/src/util.cpp:86-217
 * The op arithmetic itself is in the unvendored ggml fork (upstream ggml-cpu, early-2025 base);
 * each function below names the upstream routine it restates.
 */
#define _GNU_SOURCE
#include "ggml_ref.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define MIN(a, b) ((a) < (b) ? (a) : (b))
#define MAX(a, b) ((a) > (b) ? (a) : (b))

typedef double ggml_float;

/* Transcendental policy: ggml-cpu calls libm expf/sinf/cosf/tanhf (or SIMD approximations in its
 * vectorised paths), whose last-ulp results are platform-specific.  The oracle pins them to the
 * correctly rounded f32 value, evaluated in f64; the HIP backend does the same (cr_expf ...). */
static inline float ref_expf(float x) { return (float)exp((double)x); }
static inline float ref_sinf(float x) { return (float)sin((double)x); }
static inline float ref_cosf(float x) { return (float)cos((double)x); }
static inline float ref_tanhf(float x) { return (float)tanh((double)x); }

/* ------------------------------------------------------------------------------------------ */
/* fp16 <-> fp32: ggml_compute_fp16_to_fp32 / ggml_compute_fp32_to_fp16 (ggml-impl.h, the     */
/* FP16 library's bit-exact scalar algorithm; identical to F16C _cvtss_sh RNE results).       */

static inline float bits_to_f32(uint32_t w) {
    float f;
    memcpy(&f, &w, 4);
    return f;
}
static inline uint32_t f32_to_bits(float f) {
    uint32_t w;
    memcpy(&w, &f, 4);
    return w;
}

float ref_fp16_to_fp32(ref_fp16_t h) {
    const uint32_t w = (uint32_t)h << 16;
    const uint32_t sign = w & 0x80000000u;
    const uint32_t two_w = w + w;
    const uint32_t exp_offset = 0xE0u << 23;
    const float exp_scale = 0x1.0p-112f;
    const float normalized = bits_to_f32((two_w >> 4) + exp_offset) * exp_scale;
    const uint32_t magic_mask = 126u << 23;
    const float magic_bias = 0.5f;
    const float denormalized = bits_to_f32((two_w >> 17) | magic_mask) - magic_bias;
    const uint32_t denorm_cutoff = 1u << 27;
    const uint32_t result = sign | (two_w < denorm_cutoff ? f32_to_bits(denormalized) : f32_to_bits(normalized));
    return bits_to_f32(result);
}

ref_fp16_t ref_fp32_to_fp16(float f) {
    const float scale_to_inf = 0x1.0p+112f;
    const float scale_to_zero = 0x1.0p-110f;
    float base = (fabsf(f) * scale_to_inf) * scale_to_zero;
    const uint32_t w = f32_to_bits(f);
    const uint32_t shl1_w = w + w;
    const uint32_t sign = w & 0x80000000u;
    uint32_t bias = shl1_w & 0xFF000000u;
    if (bias < 0x71000000u) bias = 0x71000000u;
    base = bits_to_f32((bias >> 1) + 0x07800000u) + base;
    const uint32_t bits = f32_to_bits(base);
    const uint32_t exp_bits = (bits >> 13) & 0x00007C00u;
    const uint32_t mantissa_bits = bits & 0x00000FFFu;
    const uint32_t nonsign = exp_bits + mantissa_bits;
    return (ref_fp16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

/* nearest_int (ggml-quants.c): round-to-nearest-even via the 1.5*2^23 magic constant. */
int ref_nearest_int(float fval) {
    float val = fval + 12582912.f;
    int i;
    memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

/* ------------------------------------------------------------------------------------------ */
/* K-quants: get_scale_min_k4, dequantize_row_q4_K, quantize_row_q8_K_ref,                     */
/* ggml_vec_dot_q4_K_q8_K (generic).                                                           */

void ref_get_scale_min_k4(int j, const uint8_t * q, uint8_t * d, uint8_t * m) {
    if (j < 4) {
        *d = q[j] & 63;
        *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

void ref_dequantize_row_q4_K(const ref_block_q4_K * x, float * y, int64_t k) {
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t * q = x[i].qs;
        const float d = ref_fp16_to_fp32(x[i].d);
        const float mn = ref_fp16_to_fp32(x[i].dmin);
        int is = 0;
        uint8_t sc, m;
        for (int j = 0; j < QK_K; j += 64) {
            ref_get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
            const float d1 = d * sc;
            const float m1 = mn * m;
            ref_get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
            const float d2 = d * sc;
            const float m2 = mn * m;
            for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
            for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
            q += 32;
            is += 2;
        }
    }
}

void ref_dequantize_row_q8_0(const ref_block_q8_0 * x, float * y, int64_t k) {
    const int64_t nb = k / QK8_0;
    for (int64_t i = 0; i < nb; i++) {
        const float d = ref_fp16_to_fp32(x[i].d);
        for (int j = 0; j < QK8_0; ++j) y[i * QK8_0 + j] = x[i].qs[j] * d;
    }
}

void ref_quantize_row_q8_K(const float * x, ref_block_q8_K * y, int64_t k) {
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        float max = 0;
        float amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            float ax = fabsf(x[j]);
            if (ax > amax) {
                amax = ax;
                max = x[j];
            }
        }
        if (!amax) {
            y[i].d = 0;
            memset(y[i].qs, 0, QK_K);
            memset(y[i].bsums, 0, sizeof(y[i].bsums));
            x += QK_K;
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < QK_K; ++j) {
            int v = ref_nearest_int(iscale * x[j]);
            y[i].qs[j] = (int8_t)MIN(127, v);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t)sum;
        }
        y[i].d = 1 / iscale;
        x += QK_K;
    }
}

/* quantize_row_q8_0_ref */
void ref_quantize_row_q8_0(const float * x, ref_block_q8_0 * y, int64_t k) {
    const int64_t nb = k / QK8_0;
    for (int64_t i = 0; i < nb; i++) {
        float amax = 0.0f;
        for (int j = 0; j < QK8_0; j++) amax = MAX(amax, fabsf(x[i * QK8_0 + j]));
        const float d = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        y[i].d = ref_fp32_to_fp16(d);
        for (int j = 0; j < QK8_0; ++j) {
            const float x0 = x[i * QK8_0 + j] * id;
            y[i].qs[j] = (int8_t)roundf(x0);
        }
    }
}

/* make_qkx2_quants (ggml-quants.c): weighted min/scale search for one sub-block, nmax = 15,
 * rmin = -1, rdelta = 0.1, nstep = 20, squared error (use_mad false), every operation rounded to f32
 * in source order (no contraction). */
static float ref_make_qkx2_quants(int n, int nmax, const float * x, const float * weights, uint8_t * L, float * the_min,
                                  uint8_t * Laux, float rmin, float rdelta, int nstep) {
    float min = x[0];
    float max = x[0];
    float sum_w = weights[0];
    float sum_x = sum_w * x[0];
    for (int i = 1; i < n; ++i) {
        if (x[i] < min) min = x[i];
        if (x[i] > max) max = x[i];
        const float w = weights[i];
        sum_w += w;
        sum_x += w * x[i];
    }
    if (min > 0) min = 0;
    if (max == min) {
        for (int i = 0; i < n; ++i) L[i] = 0;
        *the_min = -min;
        return 0.f;
    }
    float iscale = nmax / (max - min);
    float scale = 1 / iscale;
    float best_mad = 0;
    for (int i = 0; i < n; ++i) {
        const int l = ref_nearest_int(iscale * (x[i] - min));
        L[i] = (uint8_t)MAX(0, MIN(nmax, l));
        float diff = scale * L[i] + min - x[i];
        diff = diff * diff;
        const float w = weights[i];
        best_mad += w * diff;
    }
    for (int is = 0; is <= nstep; ++is) {
        iscale = (rmin + rdelta * is + nmax) / (max - min);
        float sum_l = 0, sum_l2 = 0, sum_xl = 0;
        for (int i = 0; i < n; ++i) {
            int l = ref_nearest_int(iscale * (x[i] - min));
            l = MAX(0, MIN(nmax, l));
            Laux[i] = (uint8_t)l;
            const float w = weights[i];
            sum_l += w * l;
            sum_l2 += w * l * l;
            sum_xl += w * l * x[i];
        }
        const float D = sum_w * sum_l2 - sum_l * sum_l;
        if (D > 0) {
            float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
            float this_min = (sum_l2 * sum_x - sum_l * sum_xl) / D;
            if (this_min > 0) {
                this_min = 0;
                this_scale = sum_xl / sum_l2;
            }
            float mad = 0;
            for (int i = 0; i < n; ++i) {
                float diff = this_scale * Laux[i] + this_min - x[i];
                diff = diff * diff;
                const float w = weights[i];
                mad += w * diff;
            }
            if (mad < best_mad) {
                for (int i = 0; i < n; ++i) L[i] = Laux[i];
                best_mad = mad;
                scale = this_scale;
                min = this_min;
            }
        }
    }
    *the_min = -min;
    return scale;
}

/* quantize_row_q4_K_ref (ggml-quants.c): per 256-block, make_qkx2_quants per 32 with weights
 * av_x + |x|, 6-bit scales / mins against the block's max, fp16 d / dmin, then the 4-bit codes
 * against the rounded scales (a sub-block whose rounded scale is 0 keeps the search's codes). */
void ref_quantize_row_q4_K(const float * x, ref_block_q4_K * y, int64_t k) {
    const int64_t nb = k / QK_K;
    uint8_t L[QK_K];
    uint8_t Laux[32];
    float weights[32];
    float mins[QK_K / 32];
    float scales[QK_K / 32];
    for (int64_t i = 0; i < nb; i++) {
        float max_scale = 0;
        float max_min = 0;
        for (int j = 0; j < QK_K / 32; ++j) {
            float sum_x2 = 0;
            for (int l = 0; l < 32; ++l) sum_x2 += x[32 * j + l] * x[32 * j + l];
            const float av_x = sqrtf(sum_x2 / 32);
            for (int l = 0; l < 32; ++l) weights[l] = av_x + fabsf(x[32 * j + l]);
            scales[j] = ref_make_qkx2_quants(32, 15, x + 32 * j, weights, L + 32 * j, &mins[j], Laux, -1.f, 0.1f, 20);
            const float scale = scales[j];
            if (scale > max_scale) max_scale = scale;
            const float min = mins[j];
            if (min > max_min) max_min = min;
        }
        const float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
        const float inv_min = max_min > 0 ? 63.f / max_min : 0.f;
        memset(y[i].scales, 0, sizeof(y[i].scales));
        for (int j = 0; j < QK_K / 32; ++j) {
            uint8_t ls = (uint8_t)ref_nearest_int(inv_scale * scales[j]);
            uint8_t lm = (uint8_t)ref_nearest_int(inv_min * mins[j]);
            ls = MIN(63, ls);
            lm = MIN(63, lm);
            if (j < 4) {
                y[i].scales[j] = ls;
                y[i].scales[j + 4] = lm;
            } else {
                y[i].scales[j + 4] = (uint8_t)((ls & 0xF) | ((lm & 0xF) << 4));
                y[i].scales[j - 4] |= (uint8_t)((ls >> 4) << 6);
                y[i].scales[j - 0] |= (uint8_t)((lm >> 4) << 6);
            }
        }
        y[i].d = ref_fp32_to_fp16(max_scale / 63.f);
        y[i].dmin = ref_fp32_to_fp16(max_min / 63.f);
        uint8_t sc, m;
        for (int j = 0; j < QK_K / 32; ++j) {
            ref_get_scale_min_k4(j, y[i].scales, &sc, &m);
            const float d = ref_fp16_to_fp32(y[i].d) * sc;
            if (!d) continue;
            const float dm = ref_fp16_to_fp32(y[i].dmin) * m;
            for (int ii = 0; ii < 32; ++ii) {
                int l = ref_nearest_int((x[32 * j + ii] + dm) / d);
                l = MAX(0, MIN(15, l));
                L[32 * j + ii] = (uint8_t)l;
            }
        }
        uint8_t * q = y[i].qs;
        for (int j = 0; j < QK_K; j += 64) {
            for (int l = 0; l < 32; ++l) q[l] = (uint8_t)(L[j + l] | (L[j + l + 32] << 4));
            q += 32;
        }
        x += QK_K;
    }
}

/* ---- SIMD accumulation order (oracle_set_simd_mode(1)) -------------------------------------------
 * A stock x86-64 ggml-cpu build (AVX2 + FMA + F16C, GGML_SIMD) does not run the generic loops above:
 *  - ggml_vec_dot_f16 / _f32: GGML_F16_STEP = GGML_F32_STEP = 32 elements per iteration in
 *    GGML_F32_ARR = 4 accumulators of 8 f32 lanes, sum[j] = fma(x, y, sum[j]) (_mm256_fmadd_ps),
 *    then GGML_F32x8_REDUCE: sum0 += sum2, sum1 += sum3, sum0 += sum1, the two 128-bit halves added,
 *    two horizontal adds; the tail (n % 32) is added after, in ggml_float for f16 and in f32 (fused
 *    multiply-add, -ffp-contract=fast) for f32.
 *  - ggml_vec_dot_q4_K_q8_K (__AVX2__): per super-block the integer sums land in 8 int32 lanes, lane k
 *    holding bytes 4k..4k+3 of every 32-byte chunk (maddubs + madd with the 6-bit scales); then
 *    acc[k] = fma(d, (float)sumi[k], acc[k]) with d = y.d * x.d, the mins term in 4 lanes
 *    acc_m = fma(-y.d * x.dmin, (float)prod, acc_m), and *s = hsum_float_8(acc) + hsum(acc_m).
 *  - ggml_vec_dot_q8_0_q8_0 (__AVX2__): per block the 32 products in 8 int32 lanes (4 bytes each),
 *    acc = fma(x.d * y.d, (float)lane, acc), *s = hsum_float_8(acc).
 *  - conv_transpose_1d (upstream's loop, which the fork extends with padding / dilation / groups): for
 *    each output channel, input position i and tap k, v = vec_dot over the input channels, then
 *    dst[i*s0 + k*d0 - p0] += v in f32.
 * Restated from the published upstream ggml-cpu sources (ggml-cpu.c / vec.cpp / ggml-quants.c /
 * simd-mappings.h of early 2025, the fork's base); the fork itself is absent, so this mode
 * bounds the scalar-vs-SIMD gap rather than reproducing a pinned binary. */
static int g_simd_mode = 0;
void oracle_set_simd_mode(int mode) { g_simd_mode = mode; }
int oracle_simd_mode(void) { return g_simd_mode; }

/* GGML_F32x8_REDUCE over four 8-lane accumulators */
static float simd_reduce4x8(float acc[4][8]) {
    for (int e = 0; e < 8; ++e) acc[0][e] = acc[0][e] + acc[2][e];
    for (int e = 0; e < 8; ++e) acc[1][e] = acc[1][e] + acc[3][e];
    for (int e = 0; e < 8; ++e) acc[0][e] = acc[0][e] + acc[1][e];
    float t0[4];
    for (int e = 0; e < 4; ++e) t0[e] = acc[0][e] + acc[0][4 + e];  /* low half + high half */
    const float h0 = t0[0] + t0[1], h1 = t0[2] + t0[3];              /* _mm_hadd_ps(t0, t0) */
    return h0 + h1;                                                   /* _mm_hadd_ps(t1, t1)[0] */
}

/* hsum_float_8 */
static float simd_hsum8(const float x[8]) {
    float r[4];
    for (int e = 0; e < 4; ++e) r[e] = x[4 + e] + x[e];
    const float a = r[0] + r[2], b = r[1] + r[3];
    return a + b;
}

static void simd_vec_dot_f16(int n, float * s, const ref_fp16_t * x, const ref_fp16_t * y) {
    const int np = n & ~31;
    float acc[4][8];
    memset(acc, 0, sizeof(acc));
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; ++j)
            for (int e = 0; e < 8; ++e)
                acc[j][e] = fmaf(ref_fp16_to_fp32(x[i + 8 * j + e]), ref_fp16_to_fp32(y[i + 8 * j + e]), acc[j][e]);
    ggml_float sumf = (ggml_float)simd_reduce4x8(acc);
    for (int i = np; i < n; ++i) sumf += (ggml_float)(ref_fp16_to_fp32(x[i]) * ref_fp16_to_fp32(y[i]));
    *s = (float)sumf;
}

static void simd_vec_dot_f32(int n, float * s, const float * x, const float * y) {
    const int np = n & ~31;
    float acc[4][8];
    memset(acc, 0, sizeof(acc));
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; ++j)
            for (int e = 0; e < 8; ++e) acc[j][e] = fmaf(x[i + 8 * j + e], y[i + 8 * j + e], acc[j][e]);
    float sumf = simd_reduce4x8(acc);
    for (int i = np; i < n; ++i) sumf = fmaf(x[i], y[i], sumf);
    *s = sumf;
}

static void simd_vec_dot_q4_K_q8_K(int n, float * s, const void * vx, const void * vy) {
    const ref_block_q4_K * x = (const ref_block_q4_K *)vx;
    const ref_block_q8_K * y = (const ref_block_q8_K *)vy;
    const int nb = n / QK_K;
    static const uint32_t kmask1 = 0x3f3f3f3f, kmask2 = 0x0f0f0f0f, kmask3 = 0x03030303;
    uint32_t utmp[4];
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, acc_m[4] = {0, 0, 0, 0};
    for (int i = 0; i < nb; ++i) {
        const float d = y[i].d * ref_fp16_to_fp32(x[i].d);
        const float dmin = -y[i].d * ref_fp16_to_fp32(x[i].dmin);
        memcpy(utmp, x[i].scales, 12);
        utmp[3] = ((utmp[2] >> 4) & kmask2) | (((utmp[1] >> 6) & kmask3) << 4);
        const uint32_t uaux = utmp[1] & kmask1;
        utmp[1] = (utmp[2] & kmask2) | (((utmp[0] >> 6) & kmask3) << 4);
        utmp[2] = uaux;
        utmp[0] &= kmask1;
        const uint8_t * sc = (const uint8_t *)&utmp[0];  /* scales[0..7] */
        const uint8_t * mn = (const uint8_t *)&utmp[2];  /* mins[0..7] */
        /* mins: q8s[p] = bsums[2p] + bsums[2p+1] (hadd), prod lane q = mn[2q]*q8s[2q] + mn[2q+1]*q8s[2q+1] */
        for (int q = 0; q < 4; ++q) {
            const int32_t s0 = y[i].bsums[4 * q] + y[i].bsums[4 * q + 1], s1 = y[i].bsums[4 * q + 2] + y[i].bsums[4 * q + 3];
            const int32_t prod = (int32_t)mn[2 * q] * s0 + (int32_t)mn[2 * q + 1] * s1;
            acc_m[q] = fmaf(dmin, (float)prod, acc_m[q]);
        }
        int32_t sumi[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint8_t * q4 = x[i].qs;
        const int8_t * q8 = y[i].qs;
        for (int j = 0; j < QK_K / 64; ++j) {
            for (int k = 0; k < 8; ++k) {
                int32_t lo = 0, hi = 0;
                for (int b = 4 * k; b < 4 * k + 4; ++b) {
                    lo += (int32_t)(q4[b] & 0xF) * q8[b];
                    hi += (int32_t)(q4[b] >> 4) * q8[32 + b];
                }
                sumi[k] += (int32_t)sc[2 * j] * lo + (int32_t)sc[2 * j + 1] * hi;
            }
            q4 += 32;
            q8 += 64;
        }
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(d, (float)sumi[k], acc[k]);
    }
    const float m0 = acc_m[0] + acc_m[2], m1 = acc_m[1] + acc_m[3];
    *s = simd_hsum8(acc) + (m0 + m1);
}

static void simd_vec_dot_q8_0_q8_0(int n, float * s, const void * vx, const void * vy) {
    const ref_block_q8_0 * x = (const ref_block_q8_0 *)vx;
    const ref_block_q8_0 * y = (const ref_block_q8_0 *)vy;
    const int nb = n / QK8_0;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int ib = 0; ib < nb; ++ib) {
        const float d = ref_fp16_to_fp32(x[ib].d) * ref_fp16_to_fp32(y[ib].d);
        for (int k = 0; k < 8; ++k) {
            int32_t l = 0;
            for (int b = 4 * k; b < 4 * k + 4; ++b) l += (int32_t)x[ib].qs[b] * y[ib].qs[b];
            acc[k] = fmaf(d, (float)l, acc[k]);
        }
    }
    *s = simd_hsum8(acc);
}

void ref_vec_dot_q4_K_q8_K(int n, float * s, const void * vx, const void * vy) {
    if (g_simd_mode) {
        simd_vec_dot_q4_K_q8_K(n, s, vx, vy);
        return;
    }
    const ref_block_q4_K * x = (const ref_block_q4_K *)vx;
    const ref_block_q8_K * y = (const ref_block_q8_K *)vy;
    const int nb = n / QK_K;
    static const uint32_t kmask1 = 0x3f3f3f3f;
    static const uint32_t kmask2 = 0x0f0f0f0f;
    static const uint32_t kmask3 = 0x03030303;
    uint32_t utmp[4];
    const uint8_t * scales = (const uint8_t *)&utmp[0];
    const uint8_t * mins = (const uint8_t *)&utmp[2];
    int8_t aux8[QK_K];
    int16_t aux16[8];
    float sums[8];
    int32_t aux32[8];
    memset(sums, 0, 8 * sizeof(float));
    float sumf = 0;
    for (int i = 0; i < nb; ++i) {
        const uint8_t * q4 = x[i].qs;
        const int8_t * q8 = y[i].qs;
        memset(aux32, 0, 8 * sizeof(int32_t));
        int8_t * a = aux8;
        for (int j = 0; j < QK_K / 64; ++j) {
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] & 0xF);
            a += 32;
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] >> 4);
            a += 32;
            q4 += 32;
        }
        memcpy(utmp, x[i].scales, 12);
        utmp[3] = ((utmp[2] >> 4) & kmask2) | (((utmp[1] >> 6) & kmask3) << 4);
        const uint32_t uaux = utmp[1] & kmask1;
        utmp[1] = (utmp[2] & kmask2) | (((utmp[0] >> 6) & kmask3) << 4);
        utmp[2] = uaux;
        utmp[0] &= kmask1;
        int sumi = 0;
        for (int j = 0; j < QK_K / 16; ++j) sumi += y[i].bsums[j] * mins[j / 2];
        a = aux8;
        int is = 0;
        for (int j = 0; j < QK_K / 32; ++j) {
            int32_t scale = scales[is++];
            for (int r = 0; r < 4; ++r) {
                for (int l = 0; l < 8; ++l) aux16[l] = q8[l] * a[l];
                for (int l = 0; l < 8; ++l) aux32[l] += scale * aux16[l];
                q8 += 8;
                a += 8;
            }
        }
        const float d = ref_fp16_to_fp32(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
        const float dmin = ref_fp16_to_fp32(x[i].dmin) * y[i].d;
        sumf -= dmin * sumi;
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    *s = sumf;
}

void ref_vec_dot_q8_0_q8_0(int n, float * s, const void * vx, const void * vy) {
    if (g_simd_mode) {
        simd_vec_dot_q8_0_q8_0(n, s, vx, vy);
        return;
    }
    const ref_block_q8_0 * x = (const ref_block_q8_0 *)vx;
    const ref_block_q8_0 * y = (const ref_block_q8_0 *)vy;
    const int nb = n / QK8_0;
    float sumf = 0;
    for (int ib = 0; ib < nb; ++ib) {
        int sumi = 0;
        for (int j = 0; j < QK8_0; j++) sumi += x[ib].qs[j] * y[ib].qs[j];
        sumf += sumi * (ref_fp16_to_fp32(x[ib].d) * ref_fp16_to_fp32(y[ib].d));
    }
    *s = sumf;
}

void ref_vec_dot_f16(int n, float * s, const ref_fp16_t * x, const ref_fp16_t * y) {
    if (g_simd_mode) {
        simd_vec_dot_f16(n, s, x, y);
        return;
    }
    ggml_float sumf = 0.0;
    for (int i = 0; i < n; ++i) sumf += (ggml_float)(ref_fp16_to_fp32(x[i]) * ref_fp16_to_fp32(y[i]));
    *s = (float)sumf;
}

void ref_vec_dot_f32(int n, float * s, const float * x, const float * y) {
    if (g_simd_mode) {
        simd_vec_dot_f32(n, s, x, y);
        return;
    }
    ggml_float sumf = 0.0;
    for (int i = 0; i < n; ++i) sumf += (ggml_float)(x[i] * y[i]);
    *s = (float)sumf;
}

/* ggml_gelu_f32 + GGML_GELU_FP16 table lookup (ggml_vec_gelu_f32). */
#define GELU_COEF_A 0.044715f
#define SQRT_2_OVER_PI 0.79788456080286535587989211986876f

float ref_gelu_f32(float x) {
    return 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
}

static ref_fp16_t g_gelu_table[1 << 16];
static pthread_once_t g_gelu_once = PTHREAD_ONCE_INIT;
static void gelu_table_init(void) {
    for (int i = 0; i < (1 << 16); ++i) {
        float f = ref_fp16_to_fp32((ref_fp16_t)i);
        g_gelu_table[i] = ref_fp32_to_fp16(ref_gelu_f32(f));
    }
}

float ref_gelu_table(float x) {
    pthread_once(&g_gelu_once, gelu_table_init);
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    ref_fp16_t t = ref_fp32_to_fp16(x);
    return ref_fp16_to_fp32(g_gelu_table[t]);
}

/* ------------------------------------------------------------------------------------------ */
/* type traits                                                                                */

static size_t ref_type_size(int type) {
    switch (type) {
        case TTS_TYPE_F32: return 4;
        case TTS_TYPE_F16: return 2;
        case TTS_TYPE_Q4_K: return sizeof(ref_block_q4_K);
        case TTS_TYPE_Q8_0: return sizeof(ref_block_q8_0);
        case TTS_TYPE_Q8_K: return sizeof(ref_block_q8_K);
        case TTS_TYPE_I32: return 4;
        case TTS_TYPE_I16: return 2;
        case TTS_TYPE_I8: return 1;
        default: return 0;
    }
}
static int64_t ref_blck_size(int type) {
    switch (type) {
        case TTS_TYPE_Q4_K: case TTS_TYPE_Q8_K: return QK_K;
        case TTS_TYPE_Q8_0: return QK8_0;
        default: return 1;
    }
}
static size_t ref_row_size(int type, int64_t ne) { return ref_type_size(type) * (ne / ref_blck_size(type)); }

/* ------------------------------------------------------------------------------------------ */
/* ref_gemv: ggml_compute_forward_mul_mat for a 2-D weight and M activation columns           */

typedef struct {
    int type;
    const void * w;
    const float * x;
    float * y;
    int64_t K, N, M;
    const void * xq; /* quantized activations, one row per column */
    size_t xq_row;
    int ith, nth;
} gemv_job;

static void gemv_rows(const gemv_job * j) {
    const size_t wrow = ref_row_size(j->type, j->K);
    const int64_t dr = (j->N + j->nth - 1) / j->nth;
    const int64_t r0 = dr * j->ith, r1 = MIN(r0 + dr, j->N);
    for (int64_t m = 0; m < j->M; ++m) {
        for (int64_t n = r0; n < r1; ++n) {
            const char * wr = (const char *)j->w + n * wrow;
            float s = 0;
            switch (j->type) {
                case TTS_TYPE_Q4_K:
                    ref_vec_dot_q4_K_q8_K((int)j->K, &s, wr, (const char *)j->xq + m * j->xq_row);
                    break;
                case TTS_TYPE_Q8_0:
                    ref_vec_dot_q8_0_q8_0((int)j->K, &s, wr, (const char *)j->xq + m * j->xq_row);
                    break;
                case TTS_TYPE_F16:
                    ref_vec_dot_f16((int)j->K, &s, (const ref_fp16_t *)wr,
                                    (const ref_fp16_t *)((const char *)j->xq + m * j->xq_row));
                    break;
                default:
                    ref_vec_dot_f32((int)j->K, &s, (const float *)wr, j->x + m * j->K);
                    break;
            }
            j->y[m * j->N + n] = s;
        }
    }
}

static void * gemv_thread(void * p) {
    gemv_rows((const gemv_job *)p);
    return NULL;
}

/* convert activation rows to the weight type's vec_dot_type (from_float) */
static void * quantize_activations(int type, const float * x, int64_t K, int64_t M, size_t * row) {
    int vtype = type == TTS_TYPE_Q4_K ? TTS_TYPE_Q8_K : type == TTS_TYPE_Q8_0 ? TTS_TYPE_Q8_0
              : type == TTS_TYPE_F16 ? TTS_TYPE_F16 : TTS_TYPE_F32;
    *row = ref_row_size(vtype, K);
    if (vtype == TTS_TYPE_F32) return NULL;
    char * q = (char *)malloc(*row * M);
    for (int64_t m = 0; m < M; ++m) {
        const float * xr = x + m * K;
        char * qr = q + m * *row;
        if (vtype == TTS_TYPE_Q8_K) ref_quantize_row_q8_K(xr, (ref_block_q8_K *)qr, K);
        else if (vtype == TTS_TYPE_Q8_0) ref_quantize_row_q8_0(xr, (ref_block_q8_0 *)qr, K);
        else for (int64_t k = 0; k < K; ++k) ((ref_fp16_t *)qr)[k] = ref_fp32_to_fp16(xr[k]);
    }
    return q;
}

void ref_gemv(int type, const void * w, const float * x, float * y, int64_t K, int64_t N, int64_t M, int n_threads) {
    size_t row = 0;
    void * xq = quantize_activations(type, x, K, M, &row);
    if (n_threads < 1) n_threads = 1;
    gemv_job jobs[256];
    pthread_t th[256];
    if (n_threads > 256) n_threads = 256;
    for (int t = 0; t < n_threads; ++t) {
        jobs[t] = (gemv_job){type, w, x, y, K, N, M, xq, row, t, n_threads};
    }
    for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, gemv_thread, &jobs[t]);
    gemv_rows(&jobs[0]);
    for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
    free(xq);
}

/* ------------------------------------------------------------------------------------------ */
/* Graph interpreter: ggml_compute_forward_* restatements over tts_tensor.                    */

#define PF(t, i0, i1, i2, i3) ((float *)((char *)(t)->data + (i0) * (t)->nb[0] + (i1) * (t)->nb[1] + (i2) * (t)->nb[2] + (i3) * (t)->nb[3]))

static inline float get_op_f(const tts_tensor * t, int i) {
    float f;
    memcpy(&f, &t->op_params[i], 4);
    return f;
}

static int64_t nelements(const tts_tensor * t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }
static int64_t nrows(const tts_tensor * t) { return t->ne[1] * t->ne[2] * t->ne[3]; }

static inline float load_elem(const tts_tensor * t, int64_t i0, int64_t i1, int64_t i2, int64_t i3) {
    const char * p = (const char *)t->data + i0 * t->nb[0] + i1 * t->nb[1] + i2 * t->nb[2] + i3 * t->nb[3];
    switch (t->type) {
        case TTS_TYPE_F16: return ref_fp16_to_fp32(*(const ref_fp16_t *)p);
        case TTS_TYPE_I32: return (float)*(const int32_t *)p;
        default: return *(const float *)p;
    }
}
static inline void store_elem(const tts_tensor * t, int64_t i0, int64_t i1, int64_t i2, int64_t i3, float v) {
    char * p = (char *)t->data + i0 * t->nb[0] + i1 * t->nb[1] + i2 * t->nb[2] + i3 * t->nb[3];
    switch (t->type) {
        case TTS_TYPE_F16: *(ref_fp16_t *)p = ref_fp32_to_fp16(v); break;
        case TTS_TYPE_I32: *(int32_t *)p = (int32_t)v; break;
        default: *(float *)p = v; break;
    }
}

static void unravel(int64_t k, const int64_t * ne, int64_t * i) {
    i[0] = k % ne[0]; k /= ne[0];
    i[1] = k % ne[1]; k /= ne[1];
    i[2] = k % ne[2]; k /= ne[2];
    i[3] = k;
}

/* ggml_compute_forward_dup: element k of src (flattened, i0 fastest) -> element k of dst. */
static void op_dup(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * src = dst->src[0];
    const int64_t n = nelements(dst);
    const int64_t dr = (n + nth - 1) / nth;
    const int64_t k0 = dr * ith, k1 = MIN(k0 + dr, n);
    int64_t is[4], id[4];
    if (src->type == dst->type && src->type == TTS_TYPE_I32) {
        for (int64_t k = k0; k < k1; ++k) {
            unravel(k, src->ne, is);
            unravel(k, dst->ne, id);
            *(int32_t *)((char *)dst->data + id[0] * dst->nb[0] + id[1] * dst->nb[1] + id[2] * dst->nb[2] + id[3] * dst->nb[3]) =
                *(const int32_t *)((const char *)src->data + is[0] * src->nb[0] + is[1] * src->nb[1] + is[2] * src->nb[2] + is[3] * src->nb[3]);
        }
        return;
    }
    for (int64_t k = k0; k < k1; ++k) {
        unravel(k, src->ne, is);
        unravel(k, dst->ne, id);
        store_elem(dst, id[0], id[1], id[2], id[3], load_elem(src, is[0], is[1], is[2], is[3]));
    }
}

/* ggml_compute_forward_cpy: cpy(a, b) writes a into b; dst is a view of b. */
static void op_cpy(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * src = dst->src[0];
    const int64_t n = nelements(src);
    const int64_t dr = (n + nth - 1) / nth;
    const int64_t k0 = dr * ith, k1 = MIN(k0 + dr, n);
    int64_t is[4], id[4];
    for (int64_t k = k0; k < k1; ++k) {
        unravel(k, src->ne, is);
        unravel(k, dst->ne, id);
        store_elem(dst, id[0], id[1], id[2], id[3], load_elem(src, is[0], is[1], is[2], is[3]));
    }
}

/* ggml_compute_forward_{add,sub,mul,div}_f32 with ggml_can_repeat broadcasting of src1. */
static void op_binary(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * b = dst->src[1];
    const int64_t nr = nrows(dst);
    const int64_t dr = (nr + nth - 1) / nth;
    const int64_t r0 = dr * ith, r1 = MIN(r0 + dr, nr);
    for (int64_t r = r0; r < r1; ++r) {
        const int64_t i3 = r / (dst->ne[2] * dst->ne[1]);
        const int64_t i2 = (r - i3 * dst->ne[2] * dst->ne[1]) / dst->ne[1];
        const int64_t i1 = r - i3 * dst->ne[2] * dst->ne[1] - i2 * dst->ne[1];
        const int64_t j3 = i3 % b->ne[3], j2 = i2 % b->ne[2], j1 = i1 % b->ne[1];
        for (int64_t i0 = 0; i0 < dst->ne[0]; ++i0) {
            const float x = load_elem(a, i0, i1, i2, i3);
            const float y = load_elem(b, i0 % b->ne[0], j1, j2, j3);
            float v;
            switch (dst->op) {
                case TTS_OP_ADD: v = x + y; break;
                case TTS_OP_SUB: v = x - y; break;
                case TTS_OP_MUL: v = x * y; break;
                default: v = x / y; break;
            }
            store_elem(dst, i0, i1, i2, i3, v);
        }
    }
}

/* ggml_vec_*_f32 unary maps (ggml-cpu vec.h); LEAKY_RELU / CLAMP / SCALE / fork ROUND, MOD. */
static float unary_apply(const tts_tensor * dst, float x) {
    switch (dst->op) {
        case TTS_OP_SQR: return x * x;
        case TTS_OP_SQRT: return sqrtf(x);
        case TTS_OP_SIN: return ref_sinf(x);
        case TTS_OP_COS: return ref_cosf(x);
        case TTS_OP_SCALE: return x * get_op_f(dst, 0);
        case TTS_OP_CLAMP: return MAX(MIN(x, get_op_f(dst, 1)), get_op_f(dst, 0));
        case TTS_OP_LEAKY_RELU: {
            const float ns = get_op_f(dst, 0);
            return ((x > 0.f) ? x : 0.f) + ns * ((x < 0.0f) ? x : 0.f);
        }
        case TTS_OP_ROUND: return roundf(x);
        case TTS_OP_MOD: return fmodf(x, get_op_f(dst, 0));
        case TTS_OP_UNARY:
            switch (dst->op_params[0]) {
                case TTS_UNARY_ABS: return fabsf(x);
                case TTS_UNARY_NEG: return -x;
                case TTS_UNARY_TANH: return ref_tanhf(x);
                case TTS_UNARY_RELU: return (x > 0.f) ? x : 0.f;
                case TTS_UNARY_SIGMOID: return 1.f / (1.f + ref_expf(-x));
                case TTS_UNARY_GELU: return ref_gelu_table(x);
                case TTS_UNARY_SILU: return x / (1.0f + ref_expf(-x));
                case TTS_UNARY_EXP: return ref_expf(x);
            }
    }
    return x;
}

static void op_unary(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const int64_t nr = nrows(dst);
    const int64_t dr = (nr + nth - 1) / nth;
    const int64_t r0 = dr * ith, r1 = MIN(r0 + dr, nr);
    for (int64_t r = r0; r < r1; ++r) {
        const int64_t i3 = r / (dst->ne[2] * dst->ne[1]);
        const int64_t i2 = (r - i3 * dst->ne[2] * dst->ne[1]) / dst->ne[1];
        const int64_t i1 = r - i3 * dst->ne[2] * dst->ne[1] - i2 * dst->ne[1];
        for (int64_t i0 = 0; i0 < dst->ne[0]; ++i0) {
            store_elem(dst, i0, i1, i2, i3, unary_apply(dst, load_elem(a, i0, i1, i2, i3)));
        }
    }
}

/* ggml_compute_forward_norm_f32 / rms_norm_f32: double accumulation, then float scale. */
static void op_norm(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const float eps = get_op_f(dst, 0);
    const int64_t ne00 = a->ne[0];
    for (int64_t i3 = 0; i3 < a->ne[3]; i3++) {
        for (int64_t i2 = 0; i2 < a->ne[2]; i2++) {
            for (int64_t i1 = ith; i1 < a->ne[1]; i1 += nth) {
                const float * x = PF(a, 0, i1, i2, i3);
                float * y = PF(dst, 0, i1, i2, i3);
                if (dst->op == TTS_OP_NORM) {
                    ggml_float sum = 0.0;
                    for (int64_t i = 0; i < ne00; i++) sum += (ggml_float)x[i];
                    const float mean = (float)(sum / ne00);
                    ggml_float sum2 = 0.0;
                    for (int64_t i = 0; i < ne00; i++) {
                        const float v = x[i] - mean;
                        y[i] = v;
                        sum2 += (ggml_float)(v * v);
                    }
                    const float variance = (float)(sum2 / ne00);
                    const float scale = 1.0f / sqrtf(variance + eps);
                    for (int64_t i = 0; i < ne00; i++) y[i] *= scale;
                } else {
                    ggml_float sum = 0.0;
                    for (int64_t i = 0; i < ne00; i++) sum += (ggml_float)(x[i] * x[i]);
                    const float mean = (float)(sum / ne00);
                    memmove(y, x, ne00 * sizeof(float));
                    const float scale = 1.0f / sqrtf(mean + eps);
                    for (int64_t i = 0; i < ne00; i++) y[i] *= scale;
                }
            }
        }
    }
}

/* ggml_compute_forward_soft_max_f32: wp = x*scale + slope*mask (mask row = i1 % ne01, row
 * stride ne00; per-dim broadcast for 3-D / 4-D masks), max, expf, double sum, scale by 1/sum. */
static void op_soft_max(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * mask = dst->src[1];
    const float scale = get_op_f(dst, 0);
    const int64_t nc = a->ne[0];
    const int64_t ne01 = a->ne[1];
    const int64_t nr = nrows(a);
    const int64_t dr = (nr + nth - 1) / nth;
    const int64_t r0 = dr * ith, r1 = MIN(r0 + dr, nr);
    float * wp = (float *)malloc(nc * sizeof(float));
    for (int64_t i1 = r0; i1 < r1; i1++) {
        const float * sp = (const float *)((const char *)a->data + i1 * a->nb[1]);
        float * dp = (float *)((char *)dst->data + i1 * dst->nb[1]);
        for (int64_t i = 0; i < nc; ++i) wp[i] = sp[i] * scale;
        if (mask) {
            /* a 2-D mask: row i1 % ne01 (the fork's rule); a mask with ne2 / ne3 > 1 (the per-sequence masks
             * of a ragged lock-step batch): row (i01 % ne11) of slice (i02 % ne12, i03 % ne13), as upstream
             * ggml_compute_forward_soft_max_f32 broadcasts it */
            int64_t mr = i1 % ne01;
            if (mask->ne[2] * mask->ne[3] > 1) {
                const int64_t i01 = i1 % a->ne[1], i02 = (i1 / a->ne[1]) % a->ne[2], i03 = i1 / (a->ne[1] * a->ne[2]);
                mr = (i01 % mask->ne[1]) + mask->ne[1] * ((i02 % mask->ne[2]) + mask->ne[2] * (i03 % mask->ne[3]));
            }
            for (int64_t i = 0; i < nc; ++i) {
                float mv = mask->type == TTS_TYPE_F16 ? ref_fp16_to_fp32(((const ref_fp16_t *)mask->data)[mr * nc + i])
                                                      : ((const float *)mask->data)[mr * nc + i];
                wp[i] += 1.0f * mv;
            }
        }
        float max = -INFINITY;
        for (int64_t i = 0; i < nc; ++i) max = MAX(max, wp[i]);
        ggml_float sum = 0.0;
        for (int64_t i = 0; i < nc; ++i) {
            const float val = ref_expf(wp[i] - max);
            sum += (ggml_float)val;
            dp[i] = val;
        }
        sum = 1.0 / sum;
        const float s = (float)sum;
        for (int64_t i = 0; i < nc; ++i) dp[i] *= s;
    }
    free(wp);
}

/* ggml_compute_forward_mul_mat: src0 [K,N,ne02,ne03] x src1 [K,M,ne12,ne13] -> [N,M,ne12,ne13];
 * src1 rows converted to vec_dot_type first; broadcast r2 = ne12/ne02, r3 = ne13/ne03. */
static void op_mul_mat(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * s0 = dst->src[0];
    const tts_tensor * s1 = dst->src[1];
    const int64_t K = s0->ne[0];
    const int64_t r2 = s1->ne[2] / s0->ne[2], r3 = s1->ne[3] / s0->ne[3];
    int vtype = s0->type == TTS_TYPE_Q4_K ? TTS_TYPE_Q8_K : s0->type == TTS_TYPE_Q8_0 ? TTS_TYPE_Q8_0
              : s0->type == TTS_TYPE_F16 ? TTS_TYPE_F16 : TTS_TYPE_F32;
    const size_t qrow = ref_row_size(vtype, K);
    float * xr = (float *)malloc(K * sizeof(float));
    char * xq = (char *)malloc(qrow);
    const int64_t nout = dst->ne[1] * dst->ne[2] * dst->ne[3];
    const int64_t dr = (nout + nth - 1) / nth;
    const int64_t c0 = dr * ith, c1 = MIN(c0 + dr, nout);
    for (int64_t c = c0; c < c1; ++c) {
        const int64_t i13 = c / (dst->ne[1] * dst->ne[2]);
        const int64_t i12 = (c - i13 * dst->ne[1] * dst->ne[2]) / dst->ne[1];
        const int64_t i11 = c - i13 * dst->ne[1] * dst->ne[2] - i12 * dst->ne[1];
        for (int64_t k = 0; k < K; ++k) xr[k] = load_elem(s1, k, i11, i12, i13);
        if (vtype == TTS_TYPE_Q8_K) ref_quantize_row_q8_K(xr, (ref_block_q8_K *)xq, K);
        else if (vtype == TTS_TYPE_Q8_0) ref_quantize_row_q8_0(xr, (ref_block_q8_0 *)xq, K);
        else if (vtype == TTS_TYPE_F16) for (int64_t k = 0; k < K; ++k) ((ref_fp16_t *)xq)[k] = ref_fp32_to_fp16(xr[k]);
        const int64_t i02 = i12 / r2, i03 = i13 / r3;
        for (int64_t i01 = 0; i01 < s0->ne[1]; ++i01) {
            const char * wr = (const char *)s0->data + i01 * s0->nb[1] + i02 * s0->nb[2] + i03 * s0->nb[3];
            float s = 0;
            switch (s0->type) {
                case TTS_TYPE_Q4_K: ref_vec_dot_q4_K_q8_K((int)K, &s, wr, xq); break;
                case TTS_TYPE_Q8_0: ref_vec_dot_q8_0_q8_0((int)K, &s, wr, xq); break;
                case TTS_TYPE_F16: ref_vec_dot_f16((int)K, &s, (const ref_fp16_t *)wr, (const ref_fp16_t *)xq); break;
                default: {
                    if (g_simd_mode) {
                        ref_vec_dot_f32((int)K, &s, (const float *)wr, xr);
                        break;
                    }
                    /* src0 rows may be strided in ne0 only if nb[0]==4 (ggml requires it) */
                    ggml_float sum = 0.0;
                    const float * w = (const float *)wr;
                    for (int64_t k = 0; k < K; ++k) sum += (ggml_float)(w[k] * xr[k]);
                    s = (float)sum;
                } break;
            }
            *PF(dst, i01, i11, i12, i13) = s;
        }
    }
    free(xr);
    free(xq);
}

/* ggml_compute_forward_im2col, 1-D (is_2D = 0): dst (ic*K + k, ol, n) = src1[ol*s0 + k*d0 - p0, ic, n]
 * or 0 outside the input, stored as dst->type (F16 rounds to nearest even, ggml_conv_1d's choice).
 * op_params {s0, s1, p0, p1, d0, d1, is_2D}. */
static void op_im2col(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * b = dst->src[1];
    const int s0 = dst->op_params[0], p0 = dst->op_params[2], d0 = dst->op_params[4];
    const int64_t K = a->ne[0], IC = b->ne[1], L = b->ne[0], OL = dst->ne[1], N = dst->ne[2];
    const int64_t nr = OL * N;
    const int64_t dr = (nr + nth - 1) / nth;
    const int64_t r0 = dr * ith, r1 = MIN(r0 + dr, nr);
    for (int64_t r = r0; r < r1; ++r) {
        const int64_t ol = r % OL, n = r / OL;
        for (int64_t ic = 0; ic < IC; ++ic) {
            for (int64_t k = 0; k < K; ++k) {
                const int64_t il = ol * s0 + k * d0 - p0;
                const float v = (il >= 0 && il < L) ? load_elem(b, il, ic, n, 0) : 0.0f;
                store_elem(dst, ic * K + k, ol, n, 0, v);
            }
        }
    }
}

/* Fork op conv_transpose_1d(a = kernel [K, OC/g, IC], b = input [L, IC]) with PyTorch
 * ConvTranspose1d semantics (the fork's source is absent, its converters
 * keep torch's (IC, OC/g, K) weight order): y[oc, o] = sum over ic in oc's group, k with
 * o = i*s0 - p0 + k*d0 of x[i, ic] * w[k, oc mod OC/g, ic].  f64 accumulation, one rounding.
 * An F16 kernel takes the input rounded to f16 first, as upstream ggml's conv_transpose_1d_f16_f32
 * converts src1 (products f16 x f16, exact in f64).
 * op_params {s0, p0, d0, output_padding, groups}. */
static void op_conv_transpose_1d(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * b = dst->src[1];
    const int s0 = dst->op_params[0], p0 = dst->op_params[1], d0 = dst->op_params[2], g = dst->op_params[4];
    const int64_t K = a->ne[0], OCg = a->ne[1], IC = b->ne[1], L = b->ne[0];
    const int64_t OL = dst->ne[0], OC = dst->ne[1], ICg = IC / g;
    const int64_t dr = (OC + nth - 1) / nth;
    const int64_t c0 = dr * ith, c1 = MIN(c0 + dr, OC);
    if (g_simd_mode) { /* upstream's loop: per (input position, tap) a vec_dot over the channels, f32 += */
        const int w16 = a->type == TTS_TYPE_F16;
        float * xs = (float *)malloc(ICg * sizeof(float));
        float * ws = (float *)malloc(ICg * sizeof(float));
        ref_fp16_t * xh = (ref_fp16_t *)malloc(ICg * sizeof(ref_fp16_t));
        ref_fp16_t * wh = (ref_fp16_t *)malloc(ICg * sizeof(ref_fp16_t));
        for (int64_t oc = c0; oc < c1; ++oc) {
            const int64_t grp = oc / OCg, ocl = oc % OCg;
            for (int64_t o = 0; o < OL; ++o) *PF(dst, o, oc, 0, 0) = 0.f;
            for (int64_t i = 0; i < L; ++i) {
                for (int64_t icl = 0; icl < ICg; ++icl) xs[icl] = load_elem(b, i, grp * ICg + icl, 0, 0);
                if (w16) for (int64_t icl = 0; icl < ICg; ++icl) xh[icl] = ref_fp32_to_fp16(xs[icl]);
                for (int64_t k = 0; k < K; ++k) {
                    const int64_t o = i * s0 + k * d0 - p0;
                    if (o < 0 || o >= OL) continue;
                    float v = 0.f;
                    if (w16) {
                        for (int64_t icl = 0; icl < ICg; ++icl) wh[icl] = ref_fp32_to_fp16(load_elem(a, k, ocl, grp * ICg + icl, 0));
                        ref_vec_dot_f16((int)ICg, &v, xh, wh);
                    } else {
                        for (int64_t icl = 0; icl < ICg; ++icl) ws[icl] = load_elem(a, k, ocl, grp * ICg + icl, 0);
                        ref_vec_dot_f32((int)ICg, &v, xs, ws);
                    }
                    *PF(dst, o, oc, 0, 0) += v;
                }
            }
        }
        free(xs);
        free(ws);
        free(xh);
        free(wh);
        return;
    }
    for (int64_t oc = c0; oc < c1; ++oc) {
        const int64_t grp = oc / OCg, ocl = oc % OCg;
        for (int64_t o = 0; o < OL; ++o) {
            ggml_float acc = 0.0;
            for (int64_t k = 0; k < K; ++k) {
                const int64_t num = o + p0 - k * d0;
                if (num < 0 || num % s0) continue;
                const int64_t i = num / s0;
                if (i >= L) continue;
                for (int64_t icl = 0; icl < ICg; ++icl) {
                    const int64_t ic = grp * ICg + icl;
                    float xv = load_elem(b, i, ic, 0, 0);
                    if (a->type == TTS_TYPE_F16) xv = ref_fp16_to_fp32(ref_fp32_to_fp16(xv));
                    acc += (ggml_float)xv * (ggml_float)load_elem(a, k, ocl, ic, 0);
                }
            }
            *PF(dst, o, oc, 0, 0) = (float)acc;
        }
    }
}

/* ggml_compute_forward_get_rows (f32 / f16 / q4_K / q8_0 source; I32 index). */
static void op_get_rows(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * s0 = dst->src[0];
    const tts_tensor * s1 = dst->src[1];
    const int64_t nc = s0->ne[0];
    const int64_t nr = s1->ne[0] * s1->ne[1] * s1->ne[2];
    const int64_t dr = (nr + nth - 1) / nth;
    const int64_t r0 = dr * ith, r1 = MIN(r0 + dr, nr);
    for (int64_t i = r0; i < r1; ++i) {
        const int64_t i12 = i / (s1->ne[1] * s1->ne[0]);
        const int64_t i11 = (i - i12 * s1->ne[1] * s1->ne[0]) / s1->ne[0];
        const int64_t i10 = i - i12 * s1->ne[1] * s1->ne[0] - i11 * s1->ne[0];
        const int64_t i01 = *(const int32_t *)((const char *)s1->data + i10 * s1->nb[0] + i11 * s1->nb[1] + i12 * s1->nb[2]);
        const char * src = (const char *)s0->data + i01 * s0->nb[1] + i11 * s0->nb[2] + i12 * s0->nb[3];
        float * out = (float *)((char *)dst->data + i10 * dst->nb[1] + i11 * dst->nb[2] + i12 * dst->nb[3]);
        switch (s0->type) {
            case TTS_TYPE_Q4_K: ref_dequantize_row_q4_K((const ref_block_q4_K *)src, out, nc); break;
            case TTS_TYPE_Q8_0: ref_dequantize_row_q8_0((const ref_block_q8_0 *)src, out, nc); break;
            case TTS_TYPE_F16: for (int64_t k = 0; k < nc; ++k) out[k] = ref_fp16_to_fp32(((const ref_fp16_t *)src)[k]); break;
            default: memcpy(out, src, nc * sizeof(float)); break;
        }
    }
}

/* ggml_compute_forward_concat (any dim). */
static void op_concat(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * b = dst->src[1];
    const int dim = dst->op_params[0];
    int64_t o[4] = {0, 0, 0, 0};
    o[dim] = a->ne[dim];
    const int64_t nr = nrows(dst);
    const int64_t dr = (nr + nth - 1) / nth;
    const int64_t r0 = dr * ith, r1 = MIN(r0 + dr, nr);
    for (int64_t r = r0; r < r1; ++r) {
        const int64_t i3 = r / (dst->ne[2] * dst->ne[1]);
        const int64_t i2 = (r - i3 * dst->ne[2] * dst->ne[1]) / dst->ne[1];
        const int64_t i1 = r - i3 * dst->ne[2] * dst->ne[1] - i2 * dst->ne[1];
        for (int64_t i0 = 0; i0 < dst->ne[0]; ++i0) {
            float v;
            if (i0 < a->ne[0] && i1 < a->ne[1] && i2 < a->ne[2] && i3 < a->ne[3]) v = load_elem(a, i0, i1, i2, i3);
            else v = load_elem(b, i0 - o[0], i1 - o[1], i2 - o[2], i3 - o[3]);
            store_elem(dst, i0, i1, i2, i3, v);
        }
    }
}

/* ggml_compute_forward_sum_rows_f32 (ggml_vec_sum_f32: double accumulation). */
static void op_sum_rows(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const int64_t nr = nrows(a);
    for (int64_t r = ith; r < nr; r += nth) {
        const int64_t i3 = r / (a->ne[2] * a->ne[1]);
        const int64_t i2 = (r - i3 * a->ne[2] * a->ne[1]) / a->ne[1];
        const int64_t i1 = r - i3 * a->ne[2] * a->ne[1] - i2 * a->ne[1];
        ggml_float s = 0.0;
        for (int64_t i0 = 0; i0 < a->ne[0]; ++i0) s += (ggml_float)load_elem(a, i0, i1, i2, i3);
        *PF(dst, 0, i1, i2, i3) = (float)s;
    }
}

/* ggml_compute_forward_repeat_f32: dst[i] = src[i mod ne_src]. */
static void op_repeat(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const int64_t nr = nrows(dst);
    for (int64_t r = ith; r < nr; r += nth) {
        const int64_t i3 = r / (dst->ne[2] * dst->ne[1]);
        const int64_t i2 = (r - i3 * dst->ne[2] * dst->ne[1]) / dst->ne[1];
        const int64_t i1 = r - i3 * dst->ne[2] * dst->ne[1] - i2 * dst->ne[1];
        for (int64_t i0 = 0; i0 < dst->ne[0]; ++i0)
            store_elem(dst, i0, i1, i2, i3, load_elem(a, i0 % a->ne[0], i1 % a->ne[1], i2 % a->ne[2], i3 % a->ne[3]));
    }
}

/* ggml_compute_forward_rope_f32, NEOX and NORM modes, optional freq_factors (src[2]), no YaRN.
 * op_params: [1]=n_dims [2]=mode [4]=n_ctx_orig [5]=freq_base [6]=freq_scale [7]=ext_factor
 *            [8]=attn_factor */
static void op_rope(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * pos = dst->src[1];
    const tts_tensor * ff = dst->src[2];
    const int n_dims = dst->op_params[1];
    const int mode = dst->op_params[2];
    const float freq_base = get_op_f(dst, 5);
    const float freq_scale = get_op_f(dst, 6);
    const float attn_factor = get_op_f(dst, 8);
    const int is_neox = mode & 2;
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    float * cache = (float *)malloc(a->ne[0] * sizeof(float));
    for (int64_t i3 = 0; i3 < a->ne[3]; i3++) {
        for (int64_t i2 = 0; i2 < a->ne[2]; i2++) {
            const int64_t p = ((const int32_t *)pos->data)[i2];
            float theta = (float)p;
            for (int64_t i0 = 0; i0 < a->ne[0]; i0 += 2) {
                const float f = ff ? ((const float *)ff->data)[i0 / 2] : 1.0f;
                const float th = freq_scale * (theta / f);
                cache[i0 + 0] = ref_cosf(th) * attn_factor;
                cache[i0 + 1] = ref_sinf(th) * attn_factor;
                theta *= theta_scale;
            }
            for (int64_t i1 = ith; i1 < a->ne[1]; i1 += nth) {
                for (int64_t i0 = 0; i0 < n_dims; i0 += 2) {
                    const float c = cache[i0], s = cache[i0 + 1];
                    if (is_neox) {
                        const int64_t ic = i0 / 2;
                        const float x0 = *PF(a, ic, i1, i2, i3);
                        const float x1 = *PF(a, ic + n_dims / 2, i1, i2, i3);
                        *PF(dst, ic, i1, i2, i3) = x0 * c - x1 * s;
                        *PF(dst, ic + n_dims / 2, i1, i2, i3) = x0 * s + x1 * c;
                    } else {
                        const float x0 = *PF(a, i0, i1, i2, i3);
                        const float x1 = *PF(a, i0 + 1, i1, i2, i3);
                        *PF(dst, i0, i1, i2, i3) = x0 * c - x1 * s;
                        *PF(dst, i0 + 1, i1, i2, i3) = x0 * s + x1 * c;
                    }
                }
                for (int64_t i0 = n_dims; i0 < a->ne[0]; i0++) *PF(dst, i0, i1, i2, i3) = *PF(a, i0, i1, i2, i3);
            }
        }
    }
    free(cache);
}

/* ---- fork audio ops (Kokoro sine source / iSTFTNet head) ----------------
 * The fork's ggml_cumsum / ggml_upscale_linear / ggml_stft / ggml_istft sources are absent
 * (SURVEY.md §8c); they restate PyTorch (Kokoro's torch model: cumsum, F.interpolate linear,
 * torch.stft(center, reflect) -> abs/angle, torch.istft), which is what tests/golden pins them to.
 * Call sites: build_sin_gen src/models/kokoro/model.cpp:173-193, build_generator :195-244,
 * stft/istft wrappers src/util.cpp:111-130. */

/* ggml_cumsum (dim 0): torch.cumsum on CPU accumulates float in double, one rounding per output. */
static void op_cumsum(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const int64_t nr = nrows(dst);
    for (int64_t r = ith; r < nr; r += nth) {
        const int64_t i3 = r / (dst->ne[2] * dst->ne[1]);
        const int64_t i2 = (r - i3 * dst->ne[2] * dst->ne[1]) / dst->ne[1];
        const int64_t i1 = r - i3 * dst->ne[2] * dst->ne[1] - i2 * dst->ne[1];
        ggml_float s = 0.0;
        for (int64_t i0 = 0; i0 < dst->ne[0]; ++i0) {
            s += (ggml_float)load_elem(a, i0, i1, i2, i3);
            store_elem(dst, i0, i1, i2, i3, (float)s);
        }
    }
}

/* UPSCALE, op_params[0] = mode.
 * 0 (ggml_upscale_ext, upstream nearest): dst[i] = src[(int64)(i / sf)], sf = (float)ne_dst/ne_src per dim.
 * 1 (fork ggml_upscale_linear, dim 0 only): torch F.interpolate(mode="linear", align_corners=False)
 *   as ATen's CPU kernel computes it: src index = fma(1/s, i + 0.5, -0.5) clamped at 0, lambda in
 *   float, out = fma(x0, l0, x1 * l1) (the contractions ATen's vectorised build performs). */
static void op_upscale(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const int mode = dst->op_params[0];
    const int64_t nr = nrows(dst);
    const float sc = (float)((double)a->ne[0] / (double)dst->ne[0]);
    float sf[4];
    for (int d = 0; d < 4; ++d) sf[d] = (float)dst->ne[d] / (float)a->ne[d];
    for (int64_t r = ith; r < nr; r += nth) {
        const int64_t i3 = r / (dst->ne[2] * dst->ne[1]);
        const int64_t i2 = (r - i3 * dst->ne[2] * dst->ne[1]) / dst->ne[1];
        const int64_t i1 = r - i3 * dst->ne[2] * dst->ne[1] - i2 * dst->ne[1];
        for (int64_t i0 = 0; i0 < dst->ne[0]; ++i0) {
            float v;
            if (mode == 0) {
                v = load_elem(a, (int64_t)((float)i0 / sf[0]), (int64_t)((float)i1 / sf[1]), (int64_t)((float)i2 / sf[2]),
                              (int64_t)((float)i3 / sf[3]));
            } else {
                float x = fmaf(sc, (float)i0 + 0.5f, -0.5f);
                if (x < 0.f) x = 0.f;
                const int64_t j0 = (int64_t)x;
                const int64_t j1 = j0 + (j0 < a->ne[0] - 1 ? 1 : 0);
                const float l1 = MIN(MAX(x - (float)j0, 0.f), 1.f);
                const float l0 = 1.f - l1;
                v = fmaf(load_elem(a, j0, i1, i2, i3), l0, load_elem(a, j1, i1, i2, i3) * l1);
            }
            store_elem(dst, i0, i1, i2, i3, v);
        }
    }
}

/* Twiddle cos/sin(2*pi*m/n): exact octant reduction, then fixed Taylor polynomials in f64 with
 * every operation written out (no libm), so the HIP kernels reproduce each bit
 * (tts.cpp_amd/csrc/k_audio.hip tw_sincos). */
static void tw_sincos(int64_t m, int64_t n, double * c, double * s) {
    m %= n;
    if (m < 0) m += n;
    const int64_t q = (4 * m) / n, r = 4 * m - q * n; /* angle = pi/2 * (q + r/n) */
    const int comp = 2 * r > n;
    const int64_t rr = comp ? n - r : r;               /* reduced angle pi/2 * rr/n in [0, pi/4] */
    const double x = (double)rr * (1.5707963267948966 / (double)n);
    const double x2 = x * x;
    const double sp = x * (1.0 + x2 * (-1.0 / 6 + x2 * (1.0 / 120 + x2 * (-1.0 / 5040 + x2 * (1.0 / 362880 + x2 * (-1.0 / 39916800 +
                      x2 * (1.0 / 6227020800.0 + x2 * (-1.0 / 1307674368000.0 + x2 * (1.0 / 355687428096000.0)))))))));
    const double cp = 1.0 + x2 * (-0.5 + x2 * (1.0 / 24 + x2 * (-1.0 / 720 + x2 * (1.0 / 40320 + x2 * (-1.0 / 3628800 +
                      x2 * (1.0 / 479001600.0 + x2 * (-1.0 / 87178291200.0 + x2 * (1.0 / 20922789888000.0))))))));
    const double c0 = comp ? sp : cp, s0 = comp ? cp : sp;
    switch (q) {
        case 0: *c = c0; *s = s0; break;
        case 1: *c = -s0; *s = c0; break;
        case 2: *c = -c0; *s = -s0; break;
        default: *c = s0; *s = -c0; break;
    }
}

/* ggml_stft(a = signal [L, B], window [N]) -> [N, F, B, 2], F = L/hop + 1: torch.stft(center=True,
 * pad_mode="reflect", onesided=False) per frame, direct DFT in f64 (x*w exact, n ascending), one
 * rounding to f32; DC and Nyquist imag = +0 (rfft convention).  abs_and_angle: [..,0] = |z|
 * (f64 sqrt of the f32 parts = hypotf), [..,1] = atan2f(im, re); else [..,0] = re, [..,1] = im.
 * op_params {n_fft, hop, abs_and_angle}. */
static void op_stft(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * win = dst->src[1];
    const int64_t N = dst->op_params[0], H = dst->op_params[1];
    const int abs_angle = dst->op_params[2];
    const int64_t L = a->ne[0], F = dst->ne[1], B = dst->ne[2];
    double * tc = (double *)malloc(2 * N * sizeof(double));
    for (int64_t m = 0; m < N; ++m) tw_sincos(m, N, &tc[2 * m], &tc[2 * m + 1]);
    for (int64_t r = ith; r < F * B; r += nth) {
        const int64_t t = r % F, b = r / F;
        for (int64_t k = 0; k < N; ++k) {
            double re = 0.0, im = 0.0;
            for (int64_t n = 0; n < N; ++n) {
                int64_t j = t * H + n - N / 2;
                if (j < 0) j = -j;
                if (j >= L) j = 2 * (L - 1) - j;
                const double xw = (double)load_elem(a, j, b, 0, 0) * (double)load_elem(win, n, 0, 0, 0);
                const int64_t m = (k * n) % N;
                re += xw * tc[2 * m];
                im -= xw * tc[2 * m + 1];
            }
            float fr = (float)re, fi = (float)im;
            if (k == 0 || 2 * k == N) fi = 0.0f;
            float o0 = fr, o1 = fi;
            if (abs_angle) {
                o0 = (float)sqrt((double)fr * (double)fr + (double)fi * (double)fi);
                o1 = (float)atan2((double)fi, (double)fr);
            }
            store_elem(dst, k, t, b, 0, o0);
            store_elem(dst, k, t, b, 1, o1);
        }
    }
    free(tc);
}

/* ggml_istft(a = one-sided spectrum [N/2+1, F, B, 2], window [N]) -> [(F-1)*hop, B]: torch.istft
 * (center=True, onesided) without the window-envelope division, which TTS.cpp applies as a separate
 * DIV by window_sq_sum (src/util.cpp:122-130).  abs_and_angle: z = a0 * e^{i*a1}, else z = a0 + i*a1.
 * Per output sample p (padded index j + N/2): for each covering frame t ascending,
 * v = (sum_k w_k * (Re_k cos(2pi kn/N) - Im_k sin(2pi kn/N))) / N, w_k = 1 for DC / Nyquist (their
 * imag ignored, c2r), else 2; y += v * window[n]; all in f64, one rounding. */
static double istft_frame_val(const tts_tensor * a, int64_t t, int64_t b, int64_t n, int64_t N, int abs_angle, const double * tc) {
    const int64_t K = a->ne[0];
    double acc = 0.0;
    for (int64_t k = 0; k < K; ++k) {
        const double a0 = (double)load_elem(a, k, t, b, 0), a1 = (double)load_elem(a, k, t, b, 1);
        double re = a0, im = a1;
        if (abs_angle) {
            re = a0 * cos(a1);
            im = a0 * sin(a1);
        }
        const int64_t m = (k * n) % N;
        double term;
        if (k == 0 || 2 * k == N) term = re * tc[2 * m];
        else term = 2.0 * (re * tc[2 * m] - im * tc[2 * m + 1]);
        acc += term;
    }
    return acc / (double)N;
}

static void op_istft(tts_tensor * dst, int ith, int nth) {
    const tts_tensor * a = dst->src[0];
    const tts_tensor * win = dst->src[1];
    const int64_t N = dst->op_params[0], H = dst->op_params[1];
    const int abs_angle = dst->op_params[2];
    const int64_t F = a->ne[1], B = dst->ne[1], Lout = dst->ne[0];
    double * tc = (double *)malloc(2 * N * sizeof(double));
    for (int64_t m = 0; m < N; ++m) tw_sincos(m, N, &tc[2 * m], &tc[2 * m + 1]);
    for (int64_t r = ith; r < Lout * B; r += nth) {
        const int64_t j = r % Lout, b = r / Lout;
        const int64_t p = j + N / 2;
        int64_t t0 = p - N + 1 > 0 ? (p - N + 1 + H - 1) / H : 0;
        int64_t t1 = p / H;
        if (t1 > F - 1) t1 = F - 1;
        double y = 0.0;
        for (int64_t t = t0; t <= t1; ++t) {
            const int64_t n = p - t * H;
            y += istft_frame_val(a, t, b, n, N, abs_angle, tc) * (double)load_elem(win, n, 0, 0, 0);
        }
        store_elem(dst, j, b, 0, 0, (float)y);
    }
    free(tc);
}

/* MAP_CUSTOM3 / uv_noise_compute (src/util.cpp:140-170): per upsampled sample r (threads split
 * r as the reference's ith/nth do), voiced = f0_up[r] > threshold; over harmonics h,
 * uv[h][r] = voiced ? sin_amp : 0, noise[h][r] = (voiced ? noise_std : sin_amp/3) * rand[h][r]. */
/* The uniform draw of element i when the graph asks for device-side draws (op_params[1] = 1):
 * splitmix64 of (seed, i), top 24 bits -> [0, 1).  The HIP kernel computes the same values. */
static float uv_draw(uint64_t seed, uint64_t i) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + i + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(z >> 40) * (1.0f / 16777216.0f);
}

static int op_map_custom3(tts_tensor * dst, int ith, int nth) {
    if (dst->op_params[0] != TTS_CUSTOM_UV_NOISE) return TTS_STATUS_UNSUPPORTED;
    const int hashed = dst->op_params[1] == 1;
    const uint64_t seed = (uint64_t)(uint32_t)dst->op_params[2] | ((uint64_t)(uint32_t)dst->op_params[3] << 32);
    const tts_tensor * a = dst->src[0];
    const tts_tensor * b = dst->src[1];
    const float * cd = (const float *)dst->src[2]->data;
    const float thr = cd[0], noise_std = cd[1], sin_amp = cd[2], amp_div = cd[3];
    const float * rnd = cd + 4;
    const float * tgt = (const float *)b->data;
    float * uv = (float *)dst->data;
    float * noise = (float *)((char *)dst->data + dst->nb[2]);
    const int64_t L = dst->ne[0];
    const int64_t rpt = (b->ne[0] + nth - 1) / nth;
    const int64_t r0 = ith * rpt, r1 = (ith + 1) * rpt < b->ne[0] ? (ith + 1) * rpt : b->ne[0];
    for (int64_t r = r0; r < r1; ++r) {
        const int voiced = tgt[r] > thr;
        for (int64_t h = 0; h < a->ne[1]; ++h) {
            const int64_t i = h * L + r;
            uv[i] = voiced ? sin_amp : 0.0f;
            noise[i] = (voiced ? noise_std : amp_div) * (hashed ? uv_draw(seed, (uint64_t)i) : rnd[i]);
        }
    }
    return 0;
}

/* MAP_CUSTOM2 / cfg_scale (src/util.cpp:175-200): per element out = c + scale * (c - u), each
 * operation rounded to f32; threads split the rows' element range as the reference's ith/nth do. */
static int op_map_custom2(tts_tensor * dst, int ith, int nth) {
    if (dst->op_params[0] != TTS_CUSTOM_CFG_SCALE) return TTS_STATUS_UNSUPPORTED;
    const tts_tensor * a = dst->src[0];
    const tts_tensor * b = dst->src[1];
    float scale;
    memcpy(&scale, &dst->op_params[1], sizeof(float));
    const int64_t ne0 = b->ne[0];
    const int64_t rpt = (ne0 + nth - 1) / nth;
    const int64_t r0 = ith * rpt, r1 = (ith + 1) * rpt < ne0 ? (ith + 1) * rpt : ne0;
    for (int64_t bt = 0; bt < b->ne[2]; ++bt)
        for (int64_t h = 0; h < b->ne[1]; ++h)
            for (int64_t r = r0; r < r1; ++r) {
                const float cr = load_elem(a, r, h, bt, 0), ur = load_elem(b, r, h, bt, 0);
                const float d = cr - ur;
                const float sd = scale * d;
                store_elem(dst, r, h, bt, 0, cr + sd);
            }
    return 0;
}

static int is_view_op(int op) {
    return op == TTS_OP_NONE || op == TTS_OP_VIEW || op == TTS_OP_RESHAPE || op == TTS_OP_PERMUTE || op == TTS_OP_TRANSPOSE;
}

static int compute_node_mt(tts_tensor * node, int ith, int nth) {
    switch (node->op) {
        case TTS_OP_NONE: case TTS_OP_VIEW: case TTS_OP_RESHAPE: case TTS_OP_PERMUTE: case TTS_OP_TRANSPOSE:
            return 0;
        case TTS_OP_DUP: case TTS_OP_CONT: op_dup(node, ith, nth); return 0;
        case TTS_OP_CPY: op_cpy(node, ith, nth); return 0;
        case TTS_OP_ADD: case TTS_OP_SUB: case TTS_OP_MUL: case TTS_OP_DIV: op_binary(node, ith, nth); return 0;
        case TTS_OP_SQR: case TTS_OP_SQRT: case TTS_OP_SIN: case TTS_OP_COS: case TTS_OP_SCALE: case TTS_OP_CLAMP:
        case TTS_OP_LEAKY_RELU: case TTS_OP_ROUND: case TTS_OP_MOD: case TTS_OP_UNARY:
            op_unary(node, ith, nth); return 0;
        case TTS_OP_NORM: case TTS_OP_RMS_NORM: op_norm(node, ith, nth); return 0;
        case TTS_OP_SOFT_MAX: op_soft_max(node, ith, nth); return 0;
        case TTS_OP_MUL_MAT: op_mul_mat(node, ith, nth); return 0;
        case TTS_OP_GET_ROWS: op_get_rows(node, ith, nth); return 0;
        case TTS_OP_CONCAT: op_concat(node, ith, nth); return 0;
        case TTS_OP_SUM_ROWS: op_sum_rows(node, ith, nth); return 0;
        case TTS_OP_REPEAT: op_repeat(node, ith, nth); return 0;
        case TTS_OP_ROPE: op_rope(node, ith, nth); return 0;
        case TTS_OP_IM2COL: op_im2col(node, ith, nth); return 0;
        case TTS_OP_CONV_TRANSPOSE_1D: op_conv_transpose_1d(node, ith, nth); return 0;
        case TTS_OP_CUMSUM: op_cumsum(node, ith, nth); return 0;
        case TTS_OP_UPSCALE: op_upscale(node, ith, nth); return 0;
        case TTS_OP_STFT: op_stft(node, ith, nth); return 0;
        case TTS_OP_ISTFT: op_istft(node, ith, nth); return 0;
        case TTS_OP_MAP_CUSTOM3: return op_map_custom3(node, ith, nth);
        case TTS_OP_MAP_CUSTOM2: return op_map_custom2(node, ith, nth);
        default: return TTS_STATUS_UNSUPPORTED;
    }
}

int oracle_compute_node(tts_tensor * node) { return compute_node_mt(node, 0, 1); }

/* ---- threaded graph execution: one barrier per node, as ggml_graph_compute does ---- */
typedef struct {
    tts_tensor * const * nodes;
    int n_nodes;
    int nth;
    pthread_barrier_t barrier;
    int status;
} graph_state;

typedef struct {
    graph_state * g;
    int ith;
} graph_worker;

static void * graph_thread(void * p) {
    graph_worker * w = (graph_worker *)p;
    graph_state * g = w->g;
    for (int i = 0; i < g->n_nodes; ++i) {
        tts_tensor * node = g->nodes[i];
        if (is_view_op(node->op)) continue;
        int st = compute_node_mt(node, w->ith, g->nth);
        if (st != 0 && w->ith == 0) g->status = st;
        pthread_barrier_wait(&g->barrier);
    }
    return NULL;
}

int oracle_graph_compute(tts_tensor * const * nodes, int n_nodes, int n_threads) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    graph_state g;
    g.nodes = nodes;
    g.n_nodes = n_nodes;
    g.nth = n_threads;
    g.status = 0;
    pthread_barrier_init(&g.barrier, NULL, (unsigned)n_threads);
    graph_worker w[256];
    pthread_t th[256];
    for (int t = 0; t < n_threads; ++t) w[t] = (graph_worker){&g, t};
    for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, graph_thread, &w[t]);
    graph_thread(&w[0]);
    for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&g.barrier);
    return g.status;
}

/* ---- backend vtable over host memory ---- */
static int g_oracle_threads = 1;
static void * ob_alloc(void * ctx, size_t size) {
    (void)ctx;
    void * p = NULL;
    if (posix_memalign(&p, 256, size ? size : 256) != 0) return NULL;
    memset(p, 0, size);
    return p;
}
static void ob_free(void * ctx, void * p) { (void)ctx; free(p); }
static int ob_set(void * ctx, void * dst, const void * src, size_t n) { (void)ctx; memcpy(dst, src, n); return 0; }
static int ob_get(void * ctx, void * dst, const void * src, size_t n) { (void)ctx; memcpy(dst, src, n); return 0; }
static size_t ob_tensor_bytes(const tts_tensor * t) {
    size_t n = ref_row_size(t->type, t->ne[0]);
    for (int i = 1; i < 4; ++i) n *= (size_t)t->ne[i];
    return n;
}
static int ob_set_tensor(void * ctx, tts_tensor * t, const void * src) { (void)ctx; memcpy(t->data, src, ob_tensor_bytes(t)); return 0; }
static int ob_memset(void * ctx, void * dst, int v, size_t n) { (void)ctx; memset(dst, v, n); return 0; }
static int ob_compute(void * ctx, tts_tensor * const * nodes, int n) { (void)ctx; return oracle_graph_compute(nodes, n, g_oracle_threads); }
static int ob_sync(void * ctx) { (void)ctx; return 0; }

int oracle_backend_iface(tts_backend_iface * out, int n_threads) {
    g_oracle_threads = n_threads < 1 ? 1 : n_threads;
    out->ctx = NULL;
    out->name = "oracle-cpu";
    out->alloc = ob_alloc;
    out->free = ob_free;
    out->set = ob_set;
    out->set_tensor = ob_set_tensor;
    out->get = ob_get;
    out->memset = ob_memset;
    out->compute = ob_compute;
    out->synchronize = ob_sync;
    out->prepare = NULL; /* the oracle computes synchronously: callers fall back to compute */
    out->launch = NULL;
    out->set_async = NULL;
    out->copy = NULL;
    out->greedy_step = NULL;
    out->sample_step = NULL;
    return 0;
}
