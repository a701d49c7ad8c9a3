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
        const float iscale = cr_divf(-127.f, mx);
        qi = dev_nearest_int(__fmul_rn(iscale, v));
        qi = qi < 127 ? qi : 127;
        if (t == 0) dout[m * nb + blk] = cr_divf(1.f, iscale);
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
    const float d = cr_divf(a, 127.f);
    const float id = d != 0.f ? cr_divf(1.f, d) : 0.f;
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
// exactly: per (row, column), blocks in ascending order, sums[l] += d*aux32[l] (l = 0..7),
// sumf -= dmin*sumi, then sumf += sums[0..7].
//
// One workgroup (256 threads) owns RW consecutive rows of one matrix (gridDim.y = matrices that
// share the activation, e.g. q/k/v).  Three phases:
//   0. issue the first weight loads (registers), stage the Q8_K activation of all M columns
//      in LDS (one HBM/L2 read per workgroup instead of one per octet);
//   1. integer phase: an octet (8 lanes) per (row, block) pair: lane l's 16-B load holds the
//      nibbles of residue l (lane layout), 8 x v_dot4_i32_i8 give aux32[l] per column; results,
//      d*yd and dmin*yd go to LDS;
//   2. ordered f32 phase: lane = (column m, residue l) walks the row's blocks in order; lane l=0
//      also carries sumf; one 8-lane fold in order l = 0..7 ends the row.
// The weight stream is read once with 16-B non-temporal loads; everything else is on-chip.
__device__ __forceinline__ void q4k_scale_min(const uint8_t * q, int j, int & sc, int & mn) {
    if (j < 4) {
        sc = q[j] & 63;
        mn = q[j + 4] & 63;
    } else {
        sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        mn = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

__device__ __forceinline__ size_t al16(size_t n) { return (n + 15) & ~(size_t)15; }

template <int MC>
__device__ __forceinline__ void gemv_store(const GemvJob & j, int mat, int64_t row, int m, float v) {
    if (j.epi == EPI_GELU) {
        if (v <= -10.0f) v = 0.0f;
        else if (v < 10.0f) v = __half2float(__ushort_as_half(j.gelu[__half_as_ushort(__float2half_rn(v))]));
    } else if (j.epi == EPI_ADD) {
        v = __fadd_rn(v, j.res[m * j.rcs + row]);
    }
    j.Y[mat][m * j.ycs[mat] + row * j.yrs[mat]] = v;
}

constexpr int Q4K_PMAX = 4;  // (row, block) pairs an octet keeps in flight

template <int MC>
__global__ __launch_bounds__(256) void k_gemv_q4_K(GemvJob j, int RW) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nb = (int)(j.K / QK_K);
    const int mat = blockIdx.y;
    const uint8_t * __restrict__ W = j.W[mat];
    float * Y = j.Y[mat];
    const int64_t row0 = (int64_t)blockIdx.x * RW;
    const int rows = (int)((j.N - row0) < RW ? (j.N - row0) : RW);
    const int M = j.M;
    int8_t * xq_s = (int8_t *)smem;
    float * xd_s = (float *)(smem + al16((size_t)MC * j.K));
    int * xs_s = (int *)((char *)xd_s + al16(sizeof(float) * MC * nb));
    int * aux_s = (int *)((char *)xs_s + al16(sizeof(int) * MC * nb * 8));
    float * dd_s = (float *)((char *)aux_s + al16(sizeof(int) * (size_t)RW * nb * MC * 8));
    float * dm_s = dd_s + (size_t)RW * nb * MC;
    int * sm_s = (int *)(dm_s + (size_t)RW * nb * MC);

    const int octet = threadIdx.x >> 3, l = threadIdx.x & 7;
    const int npairs = rows * nb;
    // phase 0a: first batch of weight loads
    u32x4 hdr[Q4K_PMAX], q[Q4K_PMAX];
#pragma unroll
    for (int i = 0; i < Q4K_PMAX; ++i) {
        const int p = octet + 32 * i;
        if (p < npairs) {
            const uint8_t * bp = W + (row0 + p / nb) * j.w_row_bytes + (int64_t)(p % nb) * 144;
            hdr[i] = __builtin_nontemporal_load((const u32x4 *)bp);
            q[i] = __builtin_nontemporal_load((const u32x4 *)(bp + 16 + l * 16));
        }
    }
    // phase 0b: activation -> LDS
    {
        const int4 * src = (const int4 *)j.aq.qs;
        int4 * dst = (int4 *)xq_s;
        const int n16 = (int)((int64_t)M * j.K / 16);
        for (int i = threadIdx.x; i < n16; i += 256) dst[i] = src[i];
        for (int i = threadIdx.x; i < M * nb; i += 256) xd_s[i] = j.aq.d[i];
        for (int i = threadIdx.x; i < M * nb * 8; i += 256) xs_s[i] = j.aq.bsums[i];
    }
    __syncthreads();
    // phase 1: integer work per (row, block) pair
    for (int base = 0; base < npairs; base += 32 * Q4K_PMAX) {
        if (base > 0) {
#pragma unroll
            for (int i = 0; i < Q4K_PMAX; ++i) {
                const int p = base + octet + 32 * i;
                if (p < npairs) {
                    const uint8_t * bp = W + (row0 + p / nb) * j.w_row_bytes + (int64_t)(p % nb) * 144;
                    hdr[i] = __builtin_nontemporal_load((const u32x4 *)bp);
                    q[i] = __builtin_nontemporal_load((const u32x4 *)(bp + 16 + l * 16));
                }
            }
        }
#pragma unroll
        for (int i = 0; i < Q4K_PMAX; ++i) {
            const int p = base + octet + 32 * i;
            if (p >= npairs) break;  // octet-uniform
            const int r = p / nb, b = p % nb;
            const uint32_t sw[3] = {hdr[i].y, hdr[i].z, hdr[i].w};
            const uint8_t * scb = (const uint8_t *)sw;
            int sc[8], mymin, tmp;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) q4k_scale_min(scb, jj, sc[jj], tmp);
            q4k_scale_min(scb, l, tmp, mymin);
            const int lo0 = (int)(q[i].x & 0x0F0F0F0Fu), lo1 = (int)(q[i].y & 0x0F0F0F0Fu);
            const int lo2 = (int)(q[i].z & 0x0F0F0F0Fu), lo3 = (int)(q[i].w & 0x0F0F0F0Fu);
            const int hi0 = (int)((q[i].x >> 4) & 0x0F0F0F0Fu), hi1 = (int)((q[i].y >> 4) & 0x0F0F0F0Fu);
            const int hi2 = (int)((q[i].z >> 4) & 0x0F0F0F0Fu), hi3 = (int)((q[i].w >> 4) & 0x0F0F0F0Fu);
            const float dw = dev_fp16_to_fp32((uint16_t)(hdr[i].x & 0xFFFF));
            const float dmw = dev_fp16_to_fp32((uint16_t)(hdr[i].x >> 16));
#pragma unroll
            for (int m = 0; m < MC; ++m) {
                if (m >= M) break;
                const int xb = m * nb + b;
                const int4 xl = *(const int4 *)(xq_s + xb * QK_K + l * 32);
                const int4 xh = *(const int4 *)(xq_s + xb * QK_K + l * 32 + 16);
                int aux = sc[0] * __builtin_amdgcn_sdot4(lo0, xl.x, 0, false);
                aux += sc[2] * __builtin_amdgcn_sdot4(lo1, xl.y, 0, false);
                aux += sc[4] * __builtin_amdgcn_sdot4(lo2, xl.z, 0, false);
                aux += sc[6] * __builtin_amdgcn_sdot4(lo3, xl.w, 0, false);
                aux += sc[1] * __builtin_amdgcn_sdot4(hi0, xh.x, 0, false);
                aux += sc[3] * __builtin_amdgcn_sdot4(hi1, xh.y, 0, false);
                aux += sc[5] * __builtin_amdgcn_sdot4(hi2, xh.z, 0, false);
                aux += sc[7] * __builtin_amdgcn_sdot4(hi3, xh.w, 0, false);
                int smin = mymin * xs_s[xb * 8 + l];
                smin += __shfl_xor(smin, 1);
                smin += __shfl_xor(smin, 2);
                smin += __shfl_xor(smin, 4);
                const int o = (r * nb + b) * MC + m;
                aux_s[o * 8 + l] = aux;
                if (l == 0) {
                    const float yd = xd_s[xb];
                    dd_s[o] = __fmul_rn(dw, yd);
                    dm_s[o] = __fmul_rn(dmw, yd);
                    sm_s[o] = smin;
                }
            }
        }
    }
    __syncthreads();
    // phase 2: ordered f32 accumulation, lane = (m, l)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int m = lane >> 3, l2 = lane & 7;
    for (int r = wave; r < rows; r += 4) {
        float sums = 0.f, sumf = 0.f;
        if (m < M) {
            for (int b = 0; b < nb; ++b) {
                const int o = (r * nb + b) * MC + m;
                sums = __fadd_rn(sums, __fmul_rn(dd_s[o], (float)aux_s[o * 8 + l2]));
                if (l2 == 0) sumf = __fsub_rn(sumf, __fmul_rn(dm_s[o], (float)sm_s[o]));
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float v = __shfl(sums, (lane & ~7) + k);
            if (l2 == 0) sumf = __fadd_rn(sumf, v);
        }
        if (l2 == 0 && m < M) gemv_store<MC>(j, mat, row0 + r, m, sumf);
    }
}

// Q8_0 x Q8_0 GEMV reproducing ggml_vec_dot_q8_0_q8_0's generic order: per (row, column),
// blocks in ascending order, sumf += (float)sumi * (d_w * d_x).  Phase 1: a thread per
// (row, block) computes the exact int dots for every column -> LDS; phase 2: a lane per
// (row, column) folds its blocks in order.
template <int MC>
__global__ __launch_bounds__(256) void k_gemv_q8_0(GemvJob j, int RW) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nb = (int)(j.K / QK8_0);
    const int mat = blockIdx.y;
    const uint8_t * __restrict__ W = j.W[mat];
    float * Y = j.Y[mat];
    const int64_t row0 = (int64_t)blockIdx.x * RW;
    const int rows = (int)((j.N - row0) < RW ? (j.N - row0) : RW);
    const int M = j.M;
    int8_t * xq_s = (int8_t *)smem;
    float * xd_s = (float *)(smem + al16((size_t)MC * j.K));
    int * s_s = (int *)((char *)xd_s + al16(sizeof(float) * MC * nb));
    float * f_s = (float *)((char *)s_s + al16(sizeof(int) * (size_t)RW * nb * MC));
    {
        const int4 * src = (const int4 *)j.aq.qs;
        int4 * dst = (int4 *)xq_s;
        const int n16 = (int)((int64_t)M * j.K / 16);
        for (int i = threadIdx.x; i < n16; i += 256) dst[i] = src[i];
        for (int i = threadIdx.x; i < M * nb; i += 256) xd_s[i] = j.aq.d[i];
    }
    __syncthreads();
    const int npairs = rows * nb;
    for (int p = threadIdx.x; p < npairs; p += 256) {
        const int r = p / nb, b = p % nb;
        const uint16_t * bp = (const uint16_t *)(W + (row0 + r) * j.w_row_bytes + (int64_t)b * 34);
        const float dw = dev_fp16_to_fp32(bp[0]);
        int wv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) wv[k] = (int)bp[1 + 2 * k] | ((int)bp[2 + 2 * k] << 16);
#pragma unroll
        for (int m = 0; m < MC; ++m) {
            if (m >= M) break;
            const int4 * xb = (const int4 *)(xq_s + (m * nb + b) * QK8_0);
            const int4 x0 = xb[0], x1 = xb[1];
            int s = __builtin_amdgcn_sdot4(wv[0], x0.x, 0, false);
            s = __builtin_amdgcn_sdot4(wv[1], x0.y, s, false);
            s = __builtin_amdgcn_sdot4(wv[2], x0.z, s, false);
            s = __builtin_amdgcn_sdot4(wv[3], x0.w, s, false);
            s = __builtin_amdgcn_sdot4(wv[4], x1.x, s, false);
            s = __builtin_amdgcn_sdot4(wv[5], x1.y, s, false);
            s = __builtin_amdgcn_sdot4(wv[6], x1.z, s, false);
            s = __builtin_amdgcn_sdot4(wv[7], x1.w, s, false);
            const int o = (r * MC + m) * nb + b;
            s_s[o] = s;
            f_s[o] = __fmul_rn(dw, xd_s[m * nb + b]);
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < rows * MC; t += 256) {
        const int r = t / MC, m = t % MC;
        if (m >= M) continue;
        float a = 0.f;
        const int o = (r * MC + m) * nb;
        for (int b = 0; b < nb; ++b) a = __fadd_rn(a, __fmul_rn((float)s_s[o + b], f_s[o + b]));
        gemv_store<MC>(j, mat, row0 + r, m, a);
    }
}

// F32 / F16 GEMV: f32 products, f64 accumulation (ggml_vec_dot_f32 / _f16 generic), a wave per
// row, 16-B loads.  For F16 the activation was rounded to fp16 first (vec_dot_type F16).
template <int MC, bool F16>
__global__ __launch_bounds__(256) void k_gemv_float(GemvJob j) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= j.N) return;
    const int mat = blockIdx.y;
    const int M = j.M;
    const int64_t K = j.K;
    double acc[MC];
#pragma unroll
    for (int m = 0; m < MC; ++m) acc[m] = 0.0;
    if (!F16) {
        const float * w = (const float *)(j.W[mat] + row * j.w_row_bytes);
        const float * x = j.x;
        for (int64_t k = lane * 4; k < K; k += 256) {
            const f32x4 wv = __builtin_nontemporal_load((const f32x4 *)(w + k));
#pragma unroll
            for (int m = 0; m < MC; ++m) {
                if (m >= M) break;
                const float4 xv4 = *(const float4 *)(x + m * j.xcs + k);
                acc[m] += (double)__fmul_rn(wv.x, xv4.x);
                acc[m] += (double)__fmul_rn(wv.y, xv4.y);
                acc[m] += (double)__fmul_rn(wv.z, xv4.z);
                acc[m] += (double)__fmul_rn(wv.w, xv4.w);
            }
        }
    } else {
        const __half * w = (const __half *)(j.W[mat] + row * j.w_row_bytes);
        const __half * x = (const __half *)j.aq.qs;  // [M][K] fp16, dense
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
            if (m < M) gemv_store<MC>(j, mat, row, m, (float)acc[m]);
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

void act_quant_layout(int wtype, char * base, int64_t K, int64_t M, ActQuant & aq) {
    auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
    aq.K = K;
    aq.M = M;
    aq.qs = (int8_t *)base;
    aq.d = nullptr;
    aq.bsums = nullptr;
    if (wtype == TTS_TYPE_Q4_K) {
        aq.vtype = TTS_TYPE_Q8_K;
        aq.d = (float *)(base + al(K * M));
        aq.bsums = (int32_t *)(base + al(K * M) + al(sizeof(float) * M * (K / QK_K)));
    } else if (wtype == TTS_TYPE_Q8_0) {
        aq.vtype = TTS_TYPE_Q8_0;
        aq.d = (float *)(base + al(K * M));
    } else if (wtype == TTS_TYPE_F16) {
        aq.vtype = TTS_TYPE_F16;
    } else {
        aq.vtype = TTS_TYPE_F32;
    }
}

void launch_quantize_act(tts_hip_backend * be, int wtype, const float * x, int64_t xcs, int64_t K, int64_t M, ActQuant & aq) {
    act_quant_layout(wtype, be->scratch, K, M, aq);
    if (wtype == TTS_TYPE_Q4_K) {
        dim3 grid((unsigned)(K / QK_K), (unsigned)M);
        hipLaunchKernelGGL(k_quantize_q8_K, grid, dim3(256), 0, be->stream, x, xcs, K, aq.qs, aq.d, aq.bsums);
    } else if (wtype == TTS_TYPE_Q8_0) {
        dim3 grid((unsigned)((K + 255) / 256), (unsigned)M);
        hipLaunchKernelGGL(k_quantize_q8_0, grid, dim3(256), 0, be->stream, x, xcs, K, aq.qs, aq.d);
    } else if (wtype == TTS_TYPE_F16) {
        dim3 grid((unsigned)((K + 255) / 256), (unsigned)M);
        hipLaunchKernelGGL(k_quantize_f16, grid, dim3(256), 0, be->stream, x, xcs, K, (__half *)aq.qs);
    }
    TTS_HIP_CHECK(hipGetLastError());
}

void launch_repack_q4_K(tts_hip_backend * be, const void * src, void * dst, int64_t nblocks, int inverse) {
    const unsigned grid = (unsigned)((nblocks + 1) / 2);
    hipLaunchKernelGGL(k_repack_q4_K, dim3(grid), dim3(256), 0, be->stream, (const uint8_t *)src, (uint8_t *)dst, nblocks, inverse);
    TTS_HIP_CHECK(hipGetLastError());
}

static size_t q4k_lds(int MC, int64_t K, int RW) {
    const int64_t nb = K / QK_K;
    auto a = [](size_t n) { return (n + 15) & ~(size_t)15; };
    return a((size_t)MC * K) + a(4 * MC * nb) + a(4 * MC * nb * 8) + a(4 * (size_t)RW * nb * MC * 8) + 3 * 4 * (size_t)RW * nb * MC;
}
static size_t q80_lds(int MC, int64_t K, int RW) {
    const int64_t nb = K / QK8_0;
    auto a = [](size_t n) { return (n + 15) & ~(size_t)15; };
    return a((size_t)MC * K) + a(4 * MC * nb) + a(4 * (size_t)RW * nb * MC) + 4 * (size_t)RW * nb * MC;
}

template <int MC>
static void launch_gemv_mc(tts_hip_backend * be, const GemvJob & j) {
    const unsigned nmat = (unsigned)j.nmat;
    switch (j.wtype) {
        case TTS_TYPE_Q4_K: {
            int RW = 8;
            while (RW > 1 && q4k_lds(MC, j.K, RW) > 64 * 1024) RW /= 2;
            const size_t lds = q4k_lds(MC, j.K, RW);
            const unsigned grid = (unsigned)((j.N + RW - 1) / RW);
            hipLaunchKernelGGL(k_gemv_q4_K<MC>, dim3(grid, nmat), dim3(256), lds, be->stream, j, RW);
        } break;
        case TTS_TYPE_Q8_0: {
            int RW = 8;
            while (RW > 1 && q80_lds(MC, j.K, RW) > 64 * 1024) RW /= 2;
            const size_t lds = q80_lds(MC, j.K, RW);
            const unsigned grid = (unsigned)((j.N + RW - 1) / RW);
            hipLaunchKernelGGL(k_gemv_q8_0<MC>, dim3(grid, nmat), dim3(256), lds, be->stream, j, RW);
        } break;
        case TTS_TYPE_F16: {
            const unsigned grid = (unsigned)((j.N + 3) / 4);
            hipLaunchKernelGGL((k_gemv_float<MC, true>), dim3(grid, nmat), dim3(256), 0, be->stream, j);
        } break;
        default: {
            const unsigned grid = (unsigned)((j.N + 3) / 4);
            hipLaunchKernelGGL((k_gemv_float<MC, false>), dim3(grid, nmat), dim3(256), 0, be->stream, j);
        } break;
    }
}

static void profile_begin(tts_hip_backend * be, hipEvent_t & e0, hipEvent_t & e1) {
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

void launch_gemv_job(tts_hip_backend * be, const GemvJob & job) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (be->profile_gemv) profile_begin(be, e0, e1);
    const int64_t K = job.K;
    for (int64_t m0 = 0; m0 < job.M; m0 += 8) {
        const int64_t mc = job.M - m0 < 8 ? job.M - m0 : 8;
        GemvJob j = job;
        j.M = mc;
        if (job.aq.vtype == TTS_TYPE_Q8_K) {
            j.aq.qs = job.aq.qs + m0 * K;
            j.aq.d = job.aq.d + m0 * (K / QK_K);
            j.aq.bsums = job.aq.bsums + m0 * (K / 32);
        } else if (job.aq.vtype == TTS_TYPE_Q8_0) {
            j.aq.qs = job.aq.qs + m0 * K;
            j.aq.d = job.aq.d + m0 * (K / QK8_0);
        } else if (job.aq.vtype == TTS_TYPE_F16) {
            j.aq.qs = job.aq.qs + m0 * K * 2;
        }
        if (job.x) j.x = job.x + m0 * job.xcs;
        for (int i = 0; i < job.nmat; ++i) j.Y[i] = job.Y[i] + m0 * job.ycs[i];
        if (job.res) j.res = job.res + m0 * job.rcs;
        switch (mc) {
            case 1: launch_gemv_mc<1>(be, j); break;
            case 2: launch_gemv_mc<2>(be, j); break;
            case 3: case 4: launch_gemv_mc<4>(be, j); break;
            default: launch_gemv_mc<8>(be, j); break;
        }
    }
    TTS_HIP_CHECK(hipGetLastError());
    if (be->profile_gemv) {
        TTS_HIP_CHECK(hipEventRecord(e1, be->stream));
        be->ev_pending.push_back({e0, e1});
        // algorithmic bytes: every weight byte once + activation + outputs
        be->ev_bytes.push_back((double)job.nmat * ((double)tts_row_size(job.wtype, K) * (double)job.N + 4.0 * (double)job.N * (double)job.M) +
                               4.0 * (double)K * (double)job.M);
        be->ev_type.push_back(job.wtype);
    }
}

}  // namespace tts
