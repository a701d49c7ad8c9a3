// Fused kernels that replace ggml node groups inside graph_compute.
// Each reproduces the unfused ops' arithmetic exactly (same f32 operations, f64 where ggml-cpu
// accumulates in ggml_float), so fusion never changes a result bit:
//
//  k_attn_decode : cont(K view) -> mul_mat(K, q) -> soft_max_ext(mask, scale) -> mul_mat(kq, V)
//                  -> permute(2,0,1,3) -> cont        (Parler model.cpp:549-571, 583-594)
//                  K and V are read in place through their cache views: the reference's per-step
//                  `cont` copy of K (O(P*d) per layer per step) disappears.
//  k_layernorm   : norm(eps) -> mul(w) -> add(b)      (parler_build_layer_norm, model.cpp:412-418)
//                  with an optional Q8_K copy of the output for the GEMVs that consume it.
#include "hip_internal.h"

namespace tts {

// ------------------------------------------------------------------------------------------
// Decode attention, one workgroup per (head h, query t, sequence b).
struct AttnArgs {
    TD q;      // [hd, n, H, B]   (the permute view feeding ggml's cont(q))
    TD k;      // [hd, P, Hk, Bk] (K view of the cache, or cross_k)
    TD v;      // [P, hd, Hv, Bv] (V view of the cache, or cross_v)
    const float * mask;  // [rows >= n][P] f32, row stride P (ggml soft_max broadcast), or null
    float scale;
    float * out;         // [hd, H, n, B] contiguous
    int hd, P, H, n, B;
};

constexpr int ATTN_THREADS = 512;
constexpr int ATTN_MAXP = 8192;
constexpr int ATTN_UK = 8;  // K rows in flight per lane group (phase A)

__device__ __forceinline__ double wave_sum_d(double v) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__global__ __launch_bounds__(ATTN_THREADS) void k_attn_decode(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float s_p[ATTN_MAXP + 4];
    __shared__ double s_red[ATTN_THREADS / 64];
    __shared__ float s_redf[ATTN_THREADS / 64];
    const int h = blockIdx.x, t = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = a.P, hd = a.hd;
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const char * qbase = a.q.data + t * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3];

    // ---- phase A: kq[i] = sum_d (f32)(K[d,i] * q[d]), f64 accumulation (ggml_vec_dot_f32) ----
    // G lanes per position, each owning hd/G contiguous dims (4 when hd = 4G).
    const int G = hd / 4 <= 64 ? hd / 4 : 64;  // hd = 64 -> 16 lanes, 128 -> 32 lanes
    const int per_lane = hd / G;
    const int slot = tid % G, grp = tid / G, ngrp = ATTN_THREADS / G;
    float qv[8];
    for (int e = 0; e < per_lane && e < 8; ++e) qv[e] = *(const float *)(qbase + (int64_t)(slot * per_lane + e) * a.q.nb[0]);
    const bool vec4 = a.k.nb[0] == 4 && per_lane == 4 && (a.k.nb[1] % 16) == 0 && (((uintptr_t)kbase) % 16) == 0;
    for (int i0 = 0; i0 < P; i0 += ngrp * ATTN_UK) {
        float4 kvv[ATTN_UK];
        // issue every row load of the batch before the first use (memory-level parallelism)
#pragma unroll
        for (int u = 0; u < ATTN_UK; ++u) {
            const int i = i0 + u * ngrp + grp;
            kvv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < P) {
                const char * kr = kbase + (int64_t)i * a.k.nb[1] + (int64_t)(slot * per_lane) * a.k.nb[0];
                if (vec4) kvv[u] = *(const float4 *)kr;
                else {
                    kvv[u].x = *(const float *)kr;
                    kvv[u].y = *(const float *)(kr + a.k.nb[0]);
                    kvv[u].z = *(const float *)(kr + 2 * a.k.nb[0]);
                    kvv[u].w = *(const float *)(kr + 3 * a.k.nb[0]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < ATTN_UK; ++u) {
            double s = (double)__fmul_rn(kvv[u].x, qv[0]);
            s += (double)__fmul_rn(kvv[u].y, qv[1]);
            s += (double)__fmul_rn(kvv[u].z, qv[2]);
            s += (double)__fmul_rn(kvv[u].w, qv[3]);
            for (int off = G / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off);
            const int i = i0 + u * ngrp + grp;
            if (slot == 0 && i < P) s_p[i] = (float)s;
        }
    }
    __syncthreads();

    // ---- phase B: soft_max_ext: w = kq*scale + mask; max; e = expf(w - max); f64 sum ----
    const float * mrow = a.mask ? a.mask + (int64_t)t * P : nullptr;
    float mx = -INFINITY;
    for (int i = tid; i < P; i += ATTN_THREADS) {
        float w = __fmul_rn(s_p[i], a.scale);
        if (mrow) w = __fadd_rn(w, __fmul_rn(1.0f, mrow[i]));
        s_p[i] = w;
        mx = fmaxf(mx, w);
    }
    for (int off = 32; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    if (lane == 0) s_redf[wave] = mx;
    __syncthreads();
    mx = s_redf[0];
    for (int w = 1; w < ATTN_THREADS / 64; ++w) mx = fmaxf(mx, s_redf[w]);
    double sum = 0.0;
    for (int i = tid; i < P; i += ATTN_THREADS) {
        const float e = cr_expf(__fsub_rn(s_p[i], mx));
        s_p[i] = e;
        sum += (double)e;
    }
    sum = wave_sum_d(sum);
    if (lane == 0) s_red[wave] = sum;
    __syncthreads();
    sum = 0.0;
    for (int w = 0; w < ATTN_THREADS / 64; ++w) sum += s_red[w];
    const float inv = (float)(1.0 / sum);
    for (int i = tid; i < P; i += ATTN_THREADS) s_p[i] = __fmul_rn(s_p[i], inv);
    __syncthreads();

    // ---- phase C: out[d] = sum_i (f32)(p[i] * V[i,d]), f64 accumulation ----
    // V rows (one per d) are contiguous in i: a lane owns 4 consecutive i (16-B loads) and the
    // wave's DPW dims, so DPW x chunks loads are in flight per lane before the first FMA.
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3];
    float * orow = a.out + (((int64_t)b * a.n + t) * a.H + h) * hd;
    const int waves = ATTN_THREADS / 64;
    const bool vvec = a.v.nb[0] == 4 && (a.v.nb[1] % 16) == 0 && (((uintptr_t)vbase) % 16) == 0 &&
                      a.v.nb[1] >= (int64_t)16 * ((P + 3) / 4);
    if (vvec) {
        constexpr int DPW = 4;  // dims per pass per wave
        for (int d0 = wave * DPW; d0 < hd; d0 += waves * DPW) {
            double acc[DPW] = {0.0, 0.0, 0.0, 0.0};
            for (int i4 = lane * 4; i4 < P; i4 += 256 * 2) {
                float4 vv[2][DPW];
                float4 pp[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int ii = i4 + c * 256;
                    pp[c] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int u = 0; u < DPW; ++u) vv[c][u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (ii < P) {
                        pp[c] = *(const float4 *)(s_p + ii);
#pragma unroll
                        for (int u = 0; u < DPW; ++u)
                            if (d0 + u < hd) vv[c][u] = *(const float4 *)(vbase + (int64_t)(d0 + u) * a.v.nb[1] + (int64_t)ii * 4);
                    }
                }
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int ii = i4 + c * 256;
#pragma unroll
                    for (int u = 0; u < DPW; ++u) {
                        // positions >= P (vector tail) contribute nothing, as in the scalar sum
                        if (ii + 0 < P) acc[u] += (double)__fmul_rn(pp[c].x, vv[c][u].x);
                        if (ii + 1 < P) acc[u] += (double)__fmul_rn(pp[c].y, vv[c][u].y);
                        if (ii + 2 < P) acc[u] += (double)__fmul_rn(pp[c].z, vv[c][u].z);
                        if (ii + 3 < P) acc[u] += (double)__fmul_rn(pp[c].w, vv[c][u].w);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < DPW; ++u) {
                const double s = wave_sum_d(acc[u]);
                if (lane == 0 && d0 + u < hd) orow[d0 + u] = (float)s;
            }
        }
    } else {
        for (int d0 = wave * 4; d0 < hd; d0 += waves * 4) {
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
            for (int i = lane; i < P; i += 64) {
                const float p = s_p[i];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int d = d0 + u;
                    if (d < hd) {
                        const float vv = *(const float *)(vbase + (int64_t)d * a.v.nb[1] + (int64_t)i * a.v.nb[0]);
                        acc[u] += (double)__fmul_rn(p, vv);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double s = wave_sum_d(acc[u]);
                if (lane == 0 && d0 + u < hd) orow[d0 + u] = (float)s;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Decode attention for hd = 64 * DPR (Parler 64, Dia / Orpheus 128), same numerics as above, laid
// out for latency: every reduction is a 16-lane DPP row reduction (no LDS crossbar), every load
// batch is issued before its first use, and the only barriers are the two softmax reductions.
//   A: a 16-lane row per key position (lane t: dims 4(t + 16c) .. +3, c < DPR), 32 positions per
//      512-thread step, UK steps of loads in flight;
//   B: soft_max_ext over the P scores in LDS;
//   C: a 16-lane row per output dim (lane t: positions 4t + 64k as 16-B loads of the V row when
//      VVEC, else scalar positions t + 16k), 32 dims per step.
template <int DPR, bool VVEC>
__global__ __launch_bounds__(ATTN_THREADS) void k_attn_decode_rows(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float s_p[ATTN_MAXP + 64];
    __shared__ float s_wf[ATTN_THREADS / 64];
    __shared__ double s_wd[ATTN_THREADS / 64];
    const int h = blockIdx.x, tq = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane >> 4, t = lane & 15;
    const int P = a.P;
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const char * qbase = a.q.data + tq * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3];
    constexpr int NW = ATTN_THREADS / 64;

    // ---- A: kq[i] = sum_d (f32)(K[d,i] * q[d]) in f64 ----
    float qv[DPR][4];
#pragma unroll
    for (int c = 0; c < DPR; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) qv[c][e] = ((const float *)qbase)[4 * (t + 16 * c) + e];
    constexpr int UK = 16 / DPR;
    const int slot = wave * 4 + r;
    for (int i0 = 0; i0 < P; i0 += 4 * NW * UK) {
        float4 kv[UK][DPR];
#pragma unroll
        for (int u = 0; u < UK; ++u) {
            const int i = min(i0 + u * 4 * NW + slot, P - 1);
#pragma unroll
            for (int c = 0; c < DPR; ++c) kv[u][c] = *(const float4 *)(kbase + (int64_t)i * a.k.nb[1] + 16 * (t + 16 * c));
        }
        TTS_PIN_LOADS();
#pragma unroll
        for (int u = 0; u < UK; ++u) {
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < DPR; ++c) {
                s += (double)__fmul_rn(kv[u][c].x, qv[c][0]);
                s += (double)__fmul_rn(kv[u][c].y, qv[c][1]);
                s += (double)__fmul_rn(kv[u][c].z, qv[c][2]);
                s += (double)__fmul_rn(kv[u][c].w, qv[c][3]);
            }
            s += dpp_f64<DPP_XOR1>(s);
            s += dpp_f64<DPP_XOR2>(s);
            s += dpp_f64<DPP_HALF_MIRROR>(s);
            s += dpp_f64<DPP_MIRROR>(s);
            const int i = i0 + u * 4 * NW + slot;
            if (t == 0 && i < P) s_p[i] = (float)s;
        }
    }
    __syncthreads();

    // ---- B: soft_max_ext: w = kq*scale + mask; max; e = expf(w - max); f64 sum; p = e * (1/sum) ----
    const float * mrow = a.mask ? a.mask + (int64_t)tq * P : nullptr;
    float mx = -INFINITY;
    for (int i = tid; i < P; i += ATTN_THREADS) {
        float w = __fmul_rn(s_p[i], a.scale);
        if (mrow) w = __fadd_rn(w, __fmul_rn(1.0f, mrow[i]));
        s_p[i] = w;
        mx = fmaxf(mx, w);
    }
    mx = fmaxf(mx, dpp_f32<DPP_XOR1>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_XOR2>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_HALF_MIRROR>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_MIRROR>(mx));
    mx = fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 0)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 32)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 48))));
    if (lane == 0) s_wf[wave] = mx;
    __syncthreads();
    mx = s_wf[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) mx = fmaxf(mx, s_wf[w]);
    double sum = 0.0;
    for (int i = tid; i < P; i += ATTN_THREADS) {
        const float e = cr_expf(__fsub_rn(s_p[i], mx));
        s_p[i] = e;
        sum += (double)e;
    }
    sum = wave_sum_f64(sum);
    if (lane == 0) s_wd[wave] = sum;
    __syncthreads();
    sum = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += s_wd[w];
    const float inv = (float)(1.0 / sum);
    const int P4 = (P + 63) & ~63;
    for (int i = tid; i < P4; i += ATTN_THREADS) s_p[i] = i < P ? __fmul_rn(s_p[i], inv) : 0.f;
    __syncthreads();

    // ---- C: out[d] = sum_i (f32)(p[i] * V[d,i]) in f64 ----
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3];
    float * orow = a.out + (((int64_t)b * a.n + tq) * a.H + h) * a.hd;
    constexpr int UV = 8;
    for (int d0 = wave * 4; d0 < a.hd; d0 += 4 * NW) {
        const int d = d0 + r;
        const char * vrow = vbase + (int64_t)d * a.v.nb[1];
        double acc = 0.0;
        if (VVEC) {
            const int ilast = ((P - 1) >> 2) << 2;  // last 16-B chunk holding a position < P
            for (int k0 = 0; k0 < P; k0 += 64 * UV) {
                float4 vv[UV];
#pragma unroll
                for (int u = 0; u < UV; ++u) vv[u] = *(const float4 *)(vrow + 4 * (int64_t)min(k0 + 64 * u + 4 * t, ilast));
                TTS_PIN_LOADS();
#pragma unroll
                for (int u = 0; u < UV; ++u) {
                    const int i = k0 + 64 * u + 4 * t;
                    const float4 pp = *(const float4 *)(s_p + min(i, P4 - 4));
                    // positions >= P (tail and clamped chunks) contribute nothing, as in the scalar sum
                    acc += i + 0 < P ? (double)__fmul_rn(pp.x, vv[u].x) : 0.0;
                    acc += i + 1 < P ? (double)__fmul_rn(pp.y, vv[u].y) : 0.0;
                    acc += i + 2 < P ? (double)__fmul_rn(pp.z, vv[u].z) : 0.0;
                    acc += i + 3 < P ? (double)__fmul_rn(pp.w, vv[u].w) : 0.0;
                }
            }
        } else {
            for (int k0 = 0; k0 < P; k0 += 16 * UV) {
                float vv[UV];
#pragma unroll
                for (int u = 0; u < UV; ++u) vv[u] = *(const float *)(vrow + (int64_t)min(k0 + 16 * u + t, P - 1) * a.v.nb[0]);
                TTS_PIN_LOADS();
#pragma unroll
                for (int u = 0; u < UV; ++u) {
                    const int i = k0 + 16 * u + t;
                    acc += i < P ? (double)__fmul_rn(s_p[min(i, P - 1)], vv[u]) : 0.0;
                }
            }
        }
        acc += dpp_f64<DPP_XOR1>(acc);
        acc += dpp_f64<DPP_XOR2>(acc);
        acc += dpp_f64<DPP_HALF_MIRROR>(acc);
        acc += dpp_f64<DPP_MIRROR>(acc);
        if (t == 0) orow[d] = (float)acc;
    }
}

template <int DPR>
static void launch_attn_rows(tts_hip_backend * be, const AttnArgs & a, bool vvec) {
    const dim3 grid((unsigned)a.H, (unsigned)a.n, (unsigned)a.B);
    if (vvec) hipLaunchKernelGGL((k_attn_decode_rows<DPR, true>), grid, dim3(ATTN_THREADS), 0, be->stream, a);
    else hipLaunchKernelGGL((k_attn_decode_rows<DPR, false>), grid, dim3(ATTN_THREADS), 0, be->stream, a);
}

void launch_attn_decode(tts_hip_backend * be, const TD & q, const TD & k, const TD & v, const float * mask, float scale,
                        float * out, int hd, int P, int H, int n, int B) {
    AttnArgs a;
    a.q = q;
    a.k = k;
    a.v = v;
    a.mask = mask;
    a.scale = scale;
    a.out = out;
    a.hd = hd;
    a.P = P;
    a.H = H;
    a.n = n;
    a.B = B;
    // row kernel: hd = 64/128/256, K rows 16-B vectors (aligned base and row stride)
    const bool krows = (hd == 64 || hd == 128 || hd == 256) && k.nb[0] == 4 && (k.nb[1] % 16) == 0 &&
                       (((uintptr_t)k.data) % 16) == 0 && (k.nb[2] % 16) == 0 &&
                       (k.nb[3] % 16) == 0 && q.nb[0] == 4 && P > 0;
    if (krows) {
        const bool vvec = v.nb[0] == 4 && (v.nb[1] % 16) == 0 && (v.nb[2] % 16) == 0 && (v.nb[3] % 16) == 0 &&
                          (((uintptr_t)v.data) % 16) == 0 && v.nb[1] >= (size_t)16 * ((P + 3) / 4);
        if (hd == 64) launch_attn_rows<1>(be, a, vvec);
        else if (hd == 128) launch_attn_rows<2>(be, a, vvec);
        else launch_attn_rows<4>(be, a, vvec);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    hipLaunchKernelGGL(k_attn_decode, dim3((unsigned)H, (unsigned)n, (unsigned)B), dim3(ATTN_THREADS), 0, be->stream, a);
    TTS_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// LayerNorm row kernel: y = ((x - mean) * scale) * w + b with ggml's f64 sums; optional RMS
// variant (no mean, no bias) and optional Q8_K output in the GEMV activation layout.
template <bool RMS>
__global__ __launch_bounds__(256) void k_layernorm(TD dst, TD x, const float * __restrict__ w, const float * __restrict__ bias,
                                                   float eps, int8_t * __restrict__ qs, float * __restrict__ qd,
                                                   int32_t * __restrict__ qs32) {
    __shared__ double shd[4];
    __shared__ float s_y[8192];
    __shared__ float s_ax[4];
    __shared__ int s_idx[4];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % x.ne[1], i2 = (r / x.ne[1]) % x.ne[2], i3 = r / (x.ne[1] * x.ne[2]);
    const float * xr = (const float *)(x.data + i1 * x.nb[1] + i2 * x.nb[2] + i3 * x.nb[3]);
    float * yr = (float *)(dst.data + i1 * dst.nb[1] + i2 * dst.nb[2] + i3 * dst.nb[3]);
    const int n = (int)x.ne[0];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    auto bsum = [&](double v) {
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        __syncthreads();
        if (lane == 0) shd[wave] = v;
        __syncthreads();
        return shd[0] + shd[1] + shd[2] + shd[3];
    };
    float mean = 0.f;
    if (!RMS) {
        double s = 0.0;
        for (int i = tid; i < n; i += 256) s += (double)xr[i];
        mean = (float)(bsum(s) / (double)n);
    }
    double s2 = 0.0;
    for (int i = tid; i < n; i += 256) {
        const float v = RMS ? xr[i] : __fsub_rn(xr[i], mean);
        s2 += (double)__fmul_rn(v, v);
    }
    const float var = (float)(bsum(s2) / (double)n);
    const float scale = cr_divf(1.0f, cr_sqrtf(__fadd_rn(var, eps)));
    for (int i = tid; i < n; i += 256) {
        float v = RMS ? __fmul_rn(xr[i], scale) : __fmul_rn(__fsub_rn(xr[i], mean), scale);
        v = __fmul_rn(v, w[i]);
        if (!RMS) v = __fadd_rn(v, bias[i]);
        yr[i] = v;
        if (qs) s_y[i] = v;
    }
    if (!qs) return;
    // Q8_K of this row (quantize_row_q8_K_ref), one 256-block per pass
    const int nb = n / QK_K;
    __syncthreads();
    for (int blk = 0; blk < nb; ++blk) {
        const float v = s_y[blk * QK_K + tid];
        float ax = fabsf(v);
        int idx = tid;
        for (int off = 32; off >= 1; off >>= 1) {
            const float oax = __shfl_xor(ax, off);
            const int oidx = __shfl_xor(idx, off);
            if (oax > ax || (oax == ax && oidx < idx)) {
                ax = oax;
                idx = oidx;
            }
        }
        if (lane == 0) {
            s_ax[wave] = ax;
            s_idx[wave] = idx;
        }
        __syncthreads();
        float amax = s_ax[0];
        int imax = s_idx[0];
        for (int ww = 1; ww < 4; ++ww) {
            if (s_ax[ww] > amax || (s_ax[ww] == amax && s_idx[ww] < imax)) {
                amax = s_ax[ww];
                imax = s_idx[ww];
            }
        }
        const int j = tid >> 5, rr = tid & 31;
        const int off = (rr & 7) * 32 + (j & 1) * 16 + (j >> 1) * 4 + (rr >> 3);
        int qi = 0;
        if (amax != 0.f) {
            const float iscale = cr_divf(-127.f, s_y[blk * QK_K + imax]);
            const float val = __fadd_rn(__fmul_rn(iscale, v), 12582912.f);
            qi = (__float_as_int(val) & 0x007fffff) - 0x00400000;
            qi = qi < 127 ? qi : 127;
            if (tid == 0) qd[r * nb + blk] = cr_divf(1.f, iscale);
        } else if (tid == 0) {
            qd[r * nb + blk] = 0.f;
        }
        qs[(r * nb + blk) * QK_K + off] = (int8_t)qi;
        int s = qi;
        for (int o = 16; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if (rr == 0) qs32[(r * nb + blk) * 8 + j] = s;
        __syncthreads();
    }
}

void launch_layernorm(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * x, const float * w, const float * b,
                      float eps, bool rms, ActQuant * aq) {
    const int64_t nr = x->ne[1] * x->ne[2] * x->ne[3];
    int8_t * qs = nullptr;
    float * qd = nullptr;
    int32_t * q32 = nullptr;
    if (aq) {
        qs = aq->qs;
        qd = aq->d;
        q32 = aq->bsums;
    }
    if (rms)
        hipLaunchKernelGGL(k_layernorm<true>, dim3((unsigned)nr), dim3(256), 0, be->stream, make_td(dst), make_td(x), w, b, eps, qs, qd, q32);
    else
        hipLaunchKernelGGL(k_layernorm<false>, dim3((unsigned)nr), dim3(256), 0, be->stream, make_td(dst), make_td(x), w, b, eps, qs, qd, q32);
    TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
