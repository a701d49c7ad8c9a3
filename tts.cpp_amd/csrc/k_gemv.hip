// Quantized decode GEMV for gfx950: y = W x with W in Q4_K / Q8_0 / F16 / F32, M <= 8 columns.
//
// Replaces GGML_OP_MUL_MAT at every decode site (Parler model.cpp:544-546,571,583,594,601,603;
// Dia model.cpp:535-537,...; Orpheus model.cpp:254-256,...).
//
// Numerics follow ggml-cpu: the activation column is first quantized to the weight type's
// vec_dot_type (Q8_K for Q4_K, Q8_0 for Q8_0, F16 for F16) with the exact quantize_row_*_ref
// arithmetic, the per-block integer dot products are exact (v_dot4_i32_i8), and each block is
// combined in f32 as d*isum - dmin*imin.  F32/F16 dots take f32 products and accumulate them in
// f64, as ggml_vec_dot_f32/f16 do.  Only the order of the f32 adds across blocks differs from
// the CPU, so outputs agree to ~1e-6 relative (tests/test_gemv_parity.py).
//
// Memory shape (HBM-bound): one 8-lane octet owns one 144-B Q4_K block per step: lane t loads
// the 16-B block header and 16 B of nibbles (dwordx4), so a wave streams 8 blocks = 1152 B per
// load pair; rows are owned by octet groups, the activation (int8, L1/L2-resident) is re-read
// per column.  No LDS round trip: the weight stream is read once (guide §5 'GEMV / M <= 16').
#include "hip_internal.h"

namespace tts {

__device__ __forceinline__ float dev_fp16_to_fp32(uint16_t h) {
    return __half2float(__ushort_as_half(h));
}

__device__ __forceinline__ int dev_nearest_int(float f) {
    const float val = __fadd_rn(f, 12582912.f);
    const int i = __float_as_int(val);
    return (i & 0x007fffff) - 0x00400000;
}

// ------------------------------------------------------------------------------------------
// quantize_row_q8_K_ref: per 256-block, max |x| (first index on ties), iscale = -127/max,
// q = min(127, nearest_int(iscale*x)), d = 1/iscale.  grid (K/256, M), 256 threads.
// Output layout (device scratch, "lane-major", matches the repacked Q4_K weight):
//   qs  [M][nb][l=0..7][hi=0..1][c=0..3][k=0..3]  element p = 32*(2c+hi) + 8k + l
//   d   [M][nb]          f32 (y[i].d)
//   s32 [M][nb][8]       per-32 sums (bsums[2j] + bsums[2j+1]; ggml sums bsums*mins in int32)
__global__ __launch_bounds__(256) void k_quantize_q8_K(const float * __restrict__ x, int64_t xcs, int64_t K,
                                                       int8_t * __restrict__ qs, float * __restrict__ dout,
                                                       int32_t * __restrict__ s32) {
    const int blk = blockIdx.x;
    const int m = blockIdx.y;
    const int t = threadIdx.x;
    const int64_t nb = K / QK_K;
    const float v = x[m * xcs + (int64_t)blk * QK_K + t];
    float ax = fabsf(v);
    int idx = t;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float oax = __shfl_xor(ax, off);
        const int oidx = __shfl_xor(idx, off);
        if (oax > ax || (oax == ax && oidx < idx)) {
            ax = oax;
            idx = oidx;
        }
    }
    __shared__ float s_ax[4];
    __shared__ int s_idx[4];
    __shared__ float s_v[QK_K];
    s_v[t] = v;
    if ((t & 63) == 0) {
        s_ax[t >> 6] = ax;
        s_idx[t >> 6] = idx;
    }
    __syncthreads();
    float amax = s_ax[0];
    int imax = s_idx[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
        if (s_ax[w] > amax || (s_ax[w] == amax && s_idx[w] < imax)) {
            amax = s_ax[w];
            imax = s_idx[w];
        }
    }
    const int j = t >> 5, r = t & 31;
    const int off = (r & 7) * 32 + (j & 1) * 16 + (j >> 1) * 4 + (r >> 3);
    int8_t * q = qs + ((int64_t)m * nb + blk) * QK_K;
    int qi = 0;
    if (amax != 0.f) {
        const float mx = s_v[imax];
        const float iscale = __fdiv_rn(-127.f, mx);
        qi = dev_nearest_int(__fmul_rn(iscale, v));
        qi = qi < 127 ? qi : 127;
        if (t == 0) dout[m * nb + blk] = __fdiv_rn(1.f, iscale);
    } else if (t == 0) {
        dout[m * nb + blk] = 0.f;
    }
    q[off] = (int8_t)qi;
    int s = qi;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (r == 0) s32[((int64_t)m * nb + blk) * 8 + j] = s;
}

// Q4_K repack (the backend's own buffer layout for Q4_K matrices, like ggml-cpu's repack
// buffer type): within each 144-B block the header is unchanged and the 128 nibble bytes are
// permuted so that lane l of an octet reads, as one 16-B load, the dwords c = 0..3 whose bytes
// k = 0..3 hold weights 64c + 8k + l (low nibble) and 64c + 32 + 8k + l (high nibble):
//   repacked[l*16 + c*4 + k] = native[32c + 8k + l].
// Then sdot4 yields ggml's per-residue partial aux32[l] directly (vec_dot_q4_K_q8_K generic).
__global__ void k_repack_q4_K(const uint8_t * __restrict__ src, uint8_t * __restrict__ dst, int64_t nblocks, int inverse) {
    const int64_t b = (int64_t)blockIdx.x * 2 + (threadIdx.x >> 7);
    const int i = threadIdx.x & 127;
    if (b >= nblocks) return;
    const uint8_t * s = src + b * 144;
    uint8_t * d = dst + b * 144;
    if (i < 16) d[i] = s[i];
    const int l = i >> 4, c = (i >> 2) & 3, k = i & 3;
    const int nat = 32 * c + 8 * k + l;
    if (!inverse) d[16 + i] = s[16 + nat];
    else d[16 + nat] = s[16 + i];
}

// quantize_row_q8_0_ref: per 32-block d = amax/127, id = d ? 1/d : 0, q = roundf(x*id); the
// dot later uses fp16(d).  grid (K/256 rounded up, M), 256 threads = 8 blocks of 32.
__global__ __launch_bounds__(256) void k_quantize_q8_0(const float * __restrict__ x, int64_t xcs, int64_t K,
                                                       int8_t * __restrict__ qs, float * __restrict__ dout) {
    const int m = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= K) return;  // K % 32 == 0, so whole 32-blocks drop out together
    const float v = x[m * xcs + i];
    float a = fabsf(v);
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) a = fmaxf(a, __shfl_xor(a, off));
    const float d = __fdiv_rn(a, 127.f);
    const float id = d != 0.f ? __fdiv_rn(1.f, d) : 0.f;
    qs[m * K + i] = (int8_t)roundf(__fmul_rn(v, id));
    if ((threadIdx.x & 31) == 0) dout[m * (K / QK8_0) + i / QK8_0] = __half2float(__float2half_rn(d));
}

// F16 activations: GGML_FP32_TO_FP16 (round to nearest even).
__global__ void k_quantize_f16(const float * __restrict__ x, int64_t xcs, int64_t K, __half * __restrict__ out) {
    const int m = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < K) out[m * K + i] = __float2half_rn(x[m * xcs + i]);
}

// ------------------------------------------------------------------------------------------
// Q4_K x Q8_K GEMV on repacked weights, reproducing ggml_vec_dot_q4_K_q8_K's generic f32 order
// exactly: per row, blocks in ascending order, sums[l] += d*aux32[l] (l = 0..7), sumf -= dmin*sumi,
// then sumf += sums[0..7].  Integer work is spread over octets (one block per octet per
// iteration); the f32 accumulation is done by the row's leader octet, which pulls each block's
// aux32[l], d, dmin, sumi from the owning octet with shuffles, in block order.
// 256 threads = 4 waves; a wave covers RPI = 8/OPR rows, OPR octets per row.
__device__ __forceinline__ void q4k_scale_min(const uint8_t * q, int j, int & sc, int & mn) {
    if (j < 4) {
        sc = q[j] & 63;
        mn = q[j + 4] & 63;
    } else {
        sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        mn = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

template <int MC>
__global__ __launch_bounds__(256) void k_gemv_q4_K(const uint8_t * __restrict__ W, int64_t w_row_bytes,
                                                   const int8_t * __restrict__ xq, const float * __restrict__ xd,
                                                   const int32_t * __restrict__ xs32, float * __restrict__ y,
                                                   int64_t ycs, int64_t K, int64_t N, int M, int OPR) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 3;
    const int t = lane & 7;  // = residue l
    const int nb = (int)(K / QK_K);
    const int RPI = 8 / OPR;
    const int rg = g / OPR;                 // row group within the wave
    const int og = g % OPR;                 // octet within the row group
    const int base = rg * OPR * 8;          // first lane of the row group
    const int64_t row = ((int64_t)blockIdx.x * 4 + wave) * RPI + rg;
    const bool row_ok = row < N;
    float sums[MC], sumf[MC];
#pragma unroll
    for (int m = 0; m < MC; ++m) {
        sums[m] = 0.f;
        sumf[m] = 0.f;
    }
    const uint8_t * wrow = W + (row_ok ? row : 0) * w_row_bytes;
    const int iters = (nb + OPR - 1) / OPR;
    for (int it = 0; it < iters; ++it) {
        const int blk = og + it * OPR;
        const bool ok = row_ok && blk < nb;
        u32x4 hdr = {0u, 0u, 0u, 0u};
        u32x4 q = {0u, 0u, 0u, 0u};
        if (ok) {
            const uint8_t * bp = wrow + (int64_t)blk * 144;
            hdr = __builtin_nontemporal_load((const u32x4 *)bp);
            q = __builtin_nontemporal_load((const u32x4 *)(bp + 16 + t * 16));
        }
        const uint32_t sw[3] = {hdr.y, hdr.z, hdr.w};
        const uint8_t * scb = (const uint8_t *)sw;
        int sc[8], mymin, tmp;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) q4k_scale_min(scb, jj, sc[jj], tmp);
        q4k_scale_min(scb, t, tmp, mymin);
        const int lo0 = (int)(q.x & 0x0F0F0F0Fu), lo1 = (int)(q.y & 0x0F0F0F0Fu);
        const int lo2 = (int)(q.z & 0x0F0F0F0Fu), lo3 = (int)(q.w & 0x0F0F0F0Fu);
        const int hi0 = (int)((q.x >> 4) & 0x0F0F0F0Fu), hi1 = (int)((q.y >> 4) & 0x0F0F0F0Fu);
        const int hi2 = (int)((q.z >> 4) & 0x0F0F0F0Fu), hi3 = (int)((q.w >> 4) & 0x0F0F0F0Fu);
        const float dw = dev_fp16_to_fp32((uint16_t)(hdr.x & 0xFFFF));
        const float dmw = dev_fp16_to_fp32((uint16_t)(hdr.x >> 16));
#pragma unroll
        for (int m = 0; m < MC; ++m) {
            if (m >= M) break;
            int aux = 0, smin = 0;
            float dd = 0.f, dm = 0.f;
            if (ok) {
                const int64_t xb = ((int64_t)m * nb + blk);
                const int4 xl = *(const int4 *)(xq + xb * QK_K + t * 32);
                const int4 xh = *(const int4 *)(xq + xb * QK_K + t * 32 + 16);
                aux = sc[0] * __builtin_amdgcn_sdot4(lo0, xl.x, 0, false);
                aux += sc[2] * __builtin_amdgcn_sdot4(lo1, xl.y, 0, false);
                aux += sc[4] * __builtin_amdgcn_sdot4(lo2, xl.z, 0, false);
                aux += sc[6] * __builtin_amdgcn_sdot4(lo3, xl.w, 0, false);
                aux += sc[1] * __builtin_amdgcn_sdot4(hi0, xh.x, 0, false);
                aux += sc[3] * __builtin_amdgcn_sdot4(hi1, xh.y, 0, false);
                aux += sc[5] * __builtin_amdgcn_sdot4(hi2, xh.z, 0, false);
                aux += sc[7] * __builtin_amdgcn_sdot4(hi3, xh.w, 0, false);
                smin = mymin * xs32[xb * 8 + t];
                const float yd = xd[xb];
                dd = __fmul_rn(dw, yd);
                dm = __fmul_rn(dmw, yd);
            }
            smin += __shfl_xor(smin, 1);
            smin += __shfl_xor(smin, 2);
            smin += __shfl_xor(smin, 4);
            // ordered f32 accumulation of this iteration's blocks by the leader octet
            for (int bb = 0; bb < OPR; ++bb) {
                if (it * OPR + bb >= nb) break;  // uniform across the wave
                const int src = base + bb * 8 + t;
                const int a_b = __shfl(aux, src);
                const float dd_b = __shfl(dd, src);
                const float dm_b = __shfl(dm, src);
                const int s_b = __shfl(smin, src);
                sums[m] = __fadd_rn(sums[m], __fmul_rn(dd_b, (float)a_b));
                sumf[m] = __fsub_rn(sumf[m], __fmul_rn(dm_b, (float)s_b));
            }
        }
    }
#pragma unroll
    for (int m = 0; m < MC; ++m) {
        float f = sumf[m];
        for (int l = 0; l < 8; ++l) f = __fadd_rn(f, __shfl(sums[m], base + l));
        sumf[m] = f;
    }
    if (row_ok && og == 0 && t == 0) {
#pragma unroll
        for (int m = 0; m < MC; ++m) {
            if (m < M) y[m * ycs + row] = sumf[m];
        }
    }
}

// Q8_0 x Q8_0 GEMV reproducing ggml_vec_dot_q8_0_q8_0's generic order: per row, blocks in
// ascending order, sumf += (float)sumi * (d_w * d_x).  A wave owns a row: lane = block within a
// 64-block chunk computes sumi (exact int), then lane 0 folds the chunk in order via shuffles.
template <int MC>
__global__ __launch_bounds__(256) void k_gemv_q8_0(const uint8_t * __restrict__ W, int64_t w_row_bytes,
                                                   const int8_t * __restrict__ xq, const float * __restrict__ xd,
                                                   float * __restrict__ y, int64_t ycs, int64_t K, int64_t N, int M) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= N) return;  // wave-uniform
    const int nb = (int)(K / QK8_0);
    const uint8_t * wrow = W + row * w_row_bytes;
    float acc[MC];
#pragma unroll
    for (int m = 0; m < MC; ++m) acc[m] = 0.f;
    for (int b0 = 0; b0 < nb; b0 += 64) {
        const int b = b0 + lane;
        const bool ok = b < nb;
        float dw = 0.f;
        int wv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (ok) {
            const uint16_t * bp = (const uint16_t *)(wrow + (int64_t)b * 34);
            dw = dev_fp16_to_fp32(bp[0]);
#pragma unroll
            for (int k = 0; k < 8; ++k) wv[k] = (int)bp[1 + 2 * k] | ((int)bp[2 + 2 * k] << 16);
        }
        const int cnt = nb - b0 < 64 ? nb - b0 : 64;
#pragma unroll
        for (int m = 0; m < MC; ++m) {
            if (m >= M) break;
            int s = 0;
            float dxy = 0.f;
            if (ok) {
                const int4 * xb = (const int4 *)(xq + (int64_t)m * K + (int64_t)b * QK8_0);
                const int4 x0 = xb[0], x1 = xb[1];
                s = __builtin_amdgcn_sdot4(wv[0], x0.x, 0, false);
                s = __builtin_amdgcn_sdot4(wv[1], x0.y, s, false);
                s = __builtin_amdgcn_sdot4(wv[2], x0.z, s, false);
                s = __builtin_amdgcn_sdot4(wv[3], x0.w, s, false);
                s = __builtin_amdgcn_sdot4(wv[4], x1.x, s, false);
                s = __builtin_amdgcn_sdot4(wv[5], x1.y, s, false);
                s = __builtin_amdgcn_sdot4(wv[6], x1.z, s, false);
                s = __builtin_amdgcn_sdot4(wv[7], x1.w, s, false);
                dxy = __fmul_rn(dw, xd[(int64_t)m * nb + b]);
            }
            float a = acc[m];
            for (int i = 0; i < cnt; ++i) {
                const int si = __shfl(s, i);
                const float fi = __shfl(dxy, i);
                a = __fadd_rn(a, __fmul_rn((float)si, fi));
            }
            acc[m] = a;
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int m = 0; m < MC; ++m)
            if (m < M) y[m * ycs + row] = acc[m];
    }
}

// F32 / F16 GEMV: f32 products, f64 accumulation (ggml_vec_dot_f32 / _f16 generic), a wave per
// row, 16-B loads.  For F16 the activation was rounded to fp16 first (vec_dot_type F16).
template <int MC, bool F16>
__global__ __launch_bounds__(256) void k_gemv_float(const uint8_t * __restrict__ W, int64_t w_row_bytes,
                                                    const void * __restrict__ xv, int64_t xcs,
                                                    float * __restrict__ y, int64_t ycs, int64_t K, int64_t N, int M) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= N) return;
    double acc[MC];
#pragma unroll
    for (int m = 0; m < MC; ++m) acc[m] = 0.0;
    if (!F16) {
        const float * w = (const float *)(W + row * w_row_bytes);
        const float * x = (const float *)xv;
        const bool vec = (K % 4) == 0;
        if (vec) {
            for (int64_t k = lane * 4; k < K; k += 256) {
                const f32x4 wv = __builtin_nontemporal_load((const f32x4 *)(w + k));
#pragma unroll
                for (int m = 0; m < MC; ++m) {
                    if (m >= M) break;
                    const float4 xv4 = *(const float4 *)(x + m * xcs + k);
                    acc[m] += (double)__fmul_rn(wv.x, xv4.x);
                    acc[m] += (double)__fmul_rn(wv.y, xv4.y);
                    acc[m] += (double)__fmul_rn(wv.z, xv4.z);
                    acc[m] += (double)__fmul_rn(wv.w, xv4.w);
                }
            }
        } else {
            for (int64_t k = lane; k < K; k += 64) {
                const float wv = w[k];
#pragma unroll
                for (int m = 0; m < MC; ++m) {
                    if (m >= M) break;
                    acc[m] += (double)__fmul_rn(wv, x[m * xcs + k]);
                }
            }
        }
    } else {
        const __half * w = (const __half *)(W + row * w_row_bytes);
        const __half * x = (const __half *)xv;  // [M][K] fp16, dense
        for (int64_t k = lane; k < K; k += 64) {
            const float wv = __half2float(w[k]);
#pragma unroll
            for (int m = 0; m < MC; ++m) {
                if (m >= M) break;
                acc[m] += (double)__fmul_rn(wv, __half2float(x[m * K + k]));
            }
        }
    }
#pragma unroll
    for (int m = 0; m < MC; ++m) {
        double a = acc[m];
        for (int off = 32; off >= 1; off >>= 1) a += __shfl_xor(a, off);
        acc[m] = a;
    }
    if (lane == 0) {
#pragma unroll
        for (int m = 0; m < MC; ++m)
            if (m < M) y[m * ycs + row] = (float)acc[m];
    }
}

// ------------------------------------------------------------------------------------------

size_t act_quant_bytes(int wtype, int64_t K, int64_t M) {
    auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
    switch (wtype) {
        case TTS_TYPE_Q4_K: return al(K * M) + al(sizeof(float) * M * (K / QK_K)) + al(sizeof(int32_t) * M * (K / 32));
        case TTS_TYPE_Q8_0: return al(K * M) + al(sizeof(float) * M * (K / QK8_0));
        case TTS_TYPE_F16: return al(2 * K * M);
        default: return 0;
    }
}

void launch_quantize_act(tts_hip_backend * be, int wtype, const float * x, int64_t xcs, int64_t K, int64_t M, ActQuant & aq) {
    auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
    char * base = be->scratch;
    aq.K = K;
    aq.M = M;
    if (wtype == TTS_TYPE_Q4_K) {
        aq.vtype = TTS_TYPE_Q8_K;
        aq.qs = (int8_t *)base;
        aq.d = (float *)(base + al(K * M));
        aq.bsums = (int32_t *)(base + al(K * M) + al(sizeof(float) * M * (K / QK_K)));
        dim3 grid((unsigned)(K / QK_K), (unsigned)M);
        hipLaunchKernelGGL(k_quantize_q8_K, grid, dim3(256), 0, be->stream, x, xcs, K, aq.qs, aq.d, aq.bsums);
    } else if (wtype == TTS_TYPE_Q8_0) {
        aq.vtype = TTS_TYPE_Q8_0;
        aq.qs = (int8_t *)base;
        aq.d = (float *)(base + al(K * M));
        aq.bsums = nullptr;
        dim3 grid((unsigned)((K + 255) / 256), (unsigned)M);
        hipLaunchKernelGGL(k_quantize_q8_0, grid, dim3(256), 0, be->stream, x, xcs, K, aq.qs, aq.d);
    } else if (wtype == TTS_TYPE_F16) {
        aq.vtype = TTS_TYPE_F16;
        aq.qs = (int8_t *)base;
        aq.d = nullptr;
        aq.bsums = nullptr;
        dim3 grid((unsigned)((K + 255) / 256), (unsigned)M);
        hipLaunchKernelGGL(k_quantize_f16, grid, dim3(256), 0, be->stream, x, xcs, K, (__half *)aq.qs);
    } else {
        aq.vtype = TTS_TYPE_F32;
    }
    TTS_HIP_CHECK(hipGetLastError());
}

void launch_repack_q4_K(tts_hip_backend * be, const void * src, void * dst, int64_t nblocks, int inverse) {
    const unsigned grid = (unsigned)((nblocks + 1) / 2);
    hipLaunchKernelGGL(k_repack_q4_K, dim3(grid), dim3(256), 0, be->stream, (const uint8_t *)src, (uint8_t *)dst, nblocks, inverse);
    TTS_HIP_CHECK(hipGetLastError());
}

template <int MC>
static void launch_gemv_mc(tts_hip_backend * be, int wtype, const void * w, int64_t wrb, const float * x, int64_t xcs,
                           const ActQuant * aq, float * y, int64_t ycs, int64_t K, int64_t N, int64_t M) {
    const uint8_t * W = (const uint8_t *)w;
    switch (wtype) {
        case TTS_TYPE_Q4_K: {
            const int nb = (int)(K / QK_K);
            const int OPR = nb >= 8 ? 8 : nb >= 4 ? 4 : nb >= 2 ? 2 : 1;
            const int rows_per_wg = 4 * (8 / OPR);
            const unsigned grid = (unsigned)((N + rows_per_wg - 1) / rows_per_wg);
            hipLaunchKernelGGL(k_gemv_q4_K<MC>, dim3(grid), dim3(256), 0, be->stream, W, wrb, aq->qs, aq->d, aq->bsums, y,
                               ycs, K, N, (int)M, OPR);
        } break;
        case TTS_TYPE_Q8_0: {
            const unsigned grid = (unsigned)((N + 3) / 4);
            hipLaunchKernelGGL(k_gemv_q8_0<MC>, dim3(grid), dim3(256), 0, be->stream, W, wrb, aq->qs, aq->d, y, ycs, K, N,
                               (int)M);
        } break;
        case TTS_TYPE_F16: {
            const unsigned grid = (unsigned)((N + 3) / 4);
            hipLaunchKernelGGL((k_gemv_float<MC, true>), dim3(grid), dim3(256), 0, be->stream, W, wrb, (const void *)aq->qs,
                               K, y, ycs, K, N, (int)M);
        } break;
        default: {
            const unsigned grid = (unsigned)((N + 3) / 4);
            hipLaunchKernelGGL((k_gemv_float<MC, false>), dim3(grid), dim3(256), 0, be->stream, W, wrb, (const void *)x, xcs,
                               y, ycs, K, N, (int)M);
        } break;
    }
}

void launch_gemv(tts_hip_backend * be, int wtype, const void * w, int64_t wrb, const float * x, int64_t xcs,
                 const ActQuant * aq, float * y, int64_t ycs, int64_t K, int64_t N, int64_t M) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (be->profile_gemv) {
        if (be->ev_free.size() < 2) {
            hipEvent_t a, b;
            TTS_HIP_CHECK(hipEventCreate(&a));
            TTS_HIP_CHECK(hipEventCreate(&b));
            be->ev_free.push_back(a);
            be->ev_free.push_back(b);
        }
        e0 = be->ev_free.back();
        be->ev_free.pop_back();
        e1 = be->ev_free.back();
        be->ev_free.pop_back();
        TTS_HIP_CHECK(hipEventRecord(e0, be->stream));
    }
    for (int64_t m0 = 0; m0 < M; m0 += 8) {
        const int64_t mc = M - m0 < 8 ? M - m0 : 8;
        ActQuant sub = *aq;
        if (aq->vtype == TTS_TYPE_Q8_K) {
            sub.qs = aq->qs + m0 * K;
            sub.d = aq->d + m0 * (K / QK_K);
            sub.bsums = aq->bsums + m0 * (K / 32);
        } else if (aq->vtype == TTS_TYPE_Q8_0) {
            sub.qs = aq->qs + m0 * K;
            sub.d = aq->d + m0 * (K / QK8_0);
        } else if (aq->vtype == TTS_TYPE_F16) {
            sub.qs = aq->qs + m0 * K * 2;
        }
        const float * xs = x ? x + m0 * xcs : nullptr;
        float * ys = y + m0 * ycs;
        switch (mc) {
            case 1: launch_gemv_mc<1>(be, wtype, w, wrb, xs, xcs, &sub, ys, ycs, K, N, mc); break;
            case 2: launch_gemv_mc<2>(be, wtype, w, wrb, xs, xcs, &sub, ys, ycs, K, N, mc); break;
            case 3: case 4: launch_gemv_mc<4>(be, wtype, w, wrb, xs, xcs, &sub, ys, ycs, K, N, mc); break;
            default: launch_gemv_mc<8>(be, wtype, w, wrb, xs, xcs, &sub, ys, ycs, K, N, mc); break;
        }
    }
    TTS_HIP_CHECK(hipGetLastError());
    if (be->profile_gemv) {
        TTS_HIP_CHECK(hipEventRecord(e1, be->stream));
        be->ev_pending.push_back({e0, e1});
        // algorithmic bytes: weights once + activations + outputs
        be->ev_bytes.push_back((double)tts_row_size(wtype, K) * (double)N + 4.0 * (double)K * (double)M + 4.0 * (double)N * (double)M);
        be->ev_type.push_back(wtype);
    }
}

}  // namespace tts
