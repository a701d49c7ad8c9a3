// Generic strided op kernels for the ggml ops TTS.cpp graphs emit.  Every kernel
// takes ggml-style (ne, nb) views so that VIEW / PERMUTE / TRANSPOSE nodes stay metadata-only,
// exactly as in ggml.  Reductions that ggml-cpu performs in double (NORM, RMS_NORM, SUM_ROWS,
// SOFT_MAX's denominator, f32 dot products) are done in f64 here as well, which keeps results
// within an ulp of the CPU oracle.  Fused fast paths live in k_fused.hip.
#include "hip_internal.h"

namespace tts {

// ---- copies: element k of src (flattened, i0 fastest) -> element k of dst (ggml dup/cpy) ----
__global__ void k_cpy(TD dst, TD src, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t a0, a1, a2, a3, b0, b1, b2, b3;
        unravel(k, src.ne, a0, a1, a2, a3);
        unravel(k, dst.ne, b0, b1, b2, b3);
        if (src.type == TTS_TYPE_I32 && dst.type == TTS_TYPE_I32) {
            *(int32_t *)(dst.data + b0 * dst.nb[0] + b1 * dst.nb[1] + b2 * dst.nb[2] + b3 * dst.nb[3]) =
                *(const int32_t *)(src.data + a0 * src.nb[0] + a1 * src.nb[1] + a2 * src.nb[2] + a3 * src.nb[3]);
        } else {
            td_store(dst, b0, b1, b2, b3, td_load(src, a0, a1, a2, a3));
        }
    }
}

// Contiguous device-to-device byte copy.  Every copy inside a step's launch sequence goes through
// this kernel rather than hipMemcpyAsync, so a recorded step is a graph of kernel nodes only
// (memcpy nodes were the one node kind the profiler's graph replay could not walk).
__global__ void k_copy_bytes(char * __restrict__ dst, const char * __restrict__ src, int64_t n) {
    const int64_t n16 = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0 ? n >> 4 : 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t k = t; k < n16; k += stride) ((uint4 *)dst)[k] = ((const uint4 *)src)[k];
    for (int64_t k = (n16 << 4) + t; k < n; k += stride) dst[k] = src[k];
}

void launch_copy_bytes(tts_hip_backend * be, void * dst, const void * src, size_t bytes) {
    if (bytes == 0 || dst == src) return;
    const int64_t units = (int64_t)(bytes >> 4) + 1;
    int64_t g = (units + 255) / 256;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_copy_bytes, dim3((unsigned)g), dim3(256), 0, be->stream, (char *)dst, (const char *)src, (int64_t)bytes);
    TTS_HIP_CHECK(hipGetLastError());
}

// One source copied into up to 4 destination views of the same shape (the planner's MCPY item:
// Orpheus' repeat-interleaved KV store); each element is read once.
struct CpyMulti {
    TD dst[4];
    int nd;
};
__global__ void k_cpy_multi(CpyMulti m, TD src, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t a0, a1, a2, a3, b0, b1, b2, b3;
        unravel(k, src.ne, a0, a1, a2, a3);
        const float v = td_load(src, a0, a1, a2, a3);
        unravel(k, m.dst[0].ne, b0, b1, b2, b3);
        for (int i = 0; i < m.nd; ++i) td_store(m.dst[i], b0, b1, b2, b3, v);
    }
}

void launch_cpy_multi(tts_hip_backend * be, const tts_tensor * src, const tts_tensor * const * dsts, int nd) {
    CpyMulti m{};
    m.nd = nd;
    for (int i = 0; i < nd; ++i) m.dst[i] = make_td(dsts[i]);
    const int64_t n = src->ne[0] * src->ne[1] * src->ne[2] * src->ne[3];
    if (n == 0) return;
    const int64_t g = (n + 255) / 256;
    hipLaunchKernelGGL(k_cpy_multi, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, be->stream, m, make_td(src), n);
    TTS_HIP_CHECK(hipGetLastError());
}

// dst(i0, i1, i2, i3) = a(i0, i1 / r, i2, i3): the planner's RINT item (Dia's repeat_interleave_dim1
// chain of view / cont / repeat / concat nodes, model.cpp:421-434) in one pass; pure copies.
__global__ void k_repeat_interleave1(TD dst, TD a, int r, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unravel(k, dst.ne, i0, i1, i2, i3);
        td_store(dst, i0, i1, i2, i3, td_load(a, i0, i1 / r, i2, i3));
    }
}

void launch_repeat_interleave1(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * a, int r) {
    const int64_t n = dst->ne[0] * dst->ne[1] * dst->ne[2] * dst->ne[3];
    if (n == 0) return;
    const int64_t g = (n + 255) / 256;
    hipLaunchKernelGGL(k_repeat_interleave1, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, be->stream, make_td(dst), make_td(a), r, n);
    TTS_HIP_CHECK(hipGetLastError());
}

// ---- binary with broadcast of src1 (ggml_can_repeat) ----
template <int OP>
__global__ void k_binary(TD dst, TD a, TD b, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unravel(k, dst.ne, i0, i1, i2, i3);
        const float x = td_load(a, i0, i1, i2, i3);
        const float y = td_load(b, i0 % b.ne[0], i1 % b.ne[1], i2 % b.ne[2], i3 % b.ne[3]);
        float v;
        if (OP == TTS_OP_ADD) v = __fadd_rn(x, y);
        else if (OP == TTS_OP_SUB) v = __fsub_rn(x, y);
        else if (OP == TTS_OP_MUL) v = __fmul_rn(x, y);
        else v = cr_divf(x, y);
        td_store(dst, i0, i1, i2, i3, v);
    }
}

// Contiguous fast path: dst, a contiguous f32; b contiguous f32 broadcast over rows.
template <int OP>
__global__ void k_binary_cont(float * __restrict__ dst, const float * __restrict__ a, const float * __restrict__ b,
                              int64_t n, int64_t nb_el) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const float x = a[k];
        const float y = b[k % nb_el];
        float v;
        if (OP == TTS_OP_ADD) v = __fadd_rn(x, y);
        else if (OP == TTS_OP_SUB) v = __fsub_rn(x, y);
        else if (OP == TTS_OP_MUL) v = __fmul_rn(x, y);
        else v = cr_divf(x, y);
        dst[k] = v;
    }
}

// Row broadcast (src1 [1, C]: a per-row scalar, e.g. a conv bias or snake's alpha), both sides
// contiguous, 4 elements per lane when rows are a multiple of 4.
template <int OP, int V>
__global__ void k_binary_rowbc(float * __restrict__ dst, const float * __restrict__ a, const float * __restrict__ b, int64_t n,
                               int64_t ne0, int64_t nb1) {
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * V; k < n; k += (int64_t)gridDim.x * blockDim.x * V) {
        const float y = b[(k / ne0) % nb1];
        float x[V], v[V];
        if (V == 4) {
            const float4 t = *(const float4 *)(a + k);
            x[0] = t.x, x[1] = t.y, x[2] = t.z, x[3] = t.w;
        } else {
            x[0] = a[k];
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            if (OP == TTS_OP_ADD) v[e] = __fadd_rn(x[e], y);
            else if (OP == TTS_OP_SUB) v[e] = __fsub_rn(x[e], y);
            else if (OP == TTS_OP_MUL) v[e] = __fmul_rn(x[e], y);
            else v[e] = cr_divf(x[e], y);
        }
        if (V == 4) *(float4 *)(dst + k) = make_float4(v[0], v[1], v[2], v[3]);
        else dst[k] = v[0];
    }
}

// ---- unary maps ----
struct UnaryParams {
    int op;
    int uop;
    float p0, p1;
    const uint16_t * gelu_table;
};

__device__ __forceinline__ float unary_apply(const UnaryParams & P, float x) {
    switch (P.op) {
        case TTS_OP_SQR: return __fmul_rn(x, x);
        case TTS_OP_SQRT: return cr_sqrtf(x);
        case TTS_OP_SIN: return cr_sinf(x);
        case TTS_OP_COS: return cr_cosf(x);
        case TTS_OP_SCALE: return __fmul_rn(x, P.p0);
        case TTS_OP_CLAMP: return fmaxf(fminf(x, P.p1), P.p0);
        case TTS_OP_LEAKY_RELU: return __fadd_rn((x > 0.f) ? x : 0.f, __fmul_rn(P.p0, (x < 0.f) ? x : 0.f));
        case TTS_OP_ROUND: return roundf(x);
        case TTS_OP_MOD: return fmodf(x, P.p0);
        default: break;
    }
    switch (P.uop) {
        case TTS_UNARY_ABS: return fabsf(x);
        case TTS_UNARY_NEG: return -x;
        case TTS_UNARY_TANH: return cr_tanhf(x);
        case TTS_UNARY_RELU: return x > 0.f ? x : 0.f;
        case TTS_UNARY_SIGMOID: return cr_divf(1.f, __fadd_rn(1.f, cr_expf(-x)));
        case TTS_UNARY_GELU: {
            if (x <= -10.0f) return 0.0f;
            if (x >= 10.0f) return x;
            const uint16_t h = __half_as_ushort(__float2half_rn(x));
            return __half2float(__ushort_as_half(P.gelu_table[h]));
        }
        case TTS_UNARY_SILU: return dev_silu(x);
        case TTS_UNARY_EXP: return cr_expf(x);
    }
    return x;
}

__global__ void k_unary(TD dst, TD a, int64_t n, UnaryParams P) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unravel(k, dst.ne, i0, i1, i2, i3);
        td_store(dst, i0, i1, i2, i3, unary_apply(P, td_load(a, i0, i1, i2, i3)));
    }
}

__global__ void k_unary_cont(float * __restrict__ dst, const float * __restrict__ a, int64_t n, UnaryParams P) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        dst[k] = unary_apply(P, a[k]);
}

// ---- block reductions in double ----
template <typename T>
__device__ __forceinline__ T block_sum(T v, T * sh) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    T r = 0;
    for (int i = 0; i < nw; ++i) r += sh[i];
    return r;
}
__device__ __forceinline__ float block_max(float v, float * sh) {
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    float r = sh[0];
    for (int i = 1; i < nw; ++i) r = fmaxf(r, sh[i]);
    return r;
}

// ---- NORM / RMS_NORM (ggml_compute_forward_norm_f32 / rms_norm_f32), one block per row ----
template <bool RMS>
__global__ __launch_bounds__(256) void k_norm(TD dst, TD a, float eps) {
    __shared__ double shd[8];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % a.ne[1], i2 = (r / a.ne[1]) % a.ne[2], i3 = r / (a.ne[1] * a.ne[2]);
    const float * x = (const float *)(a.data + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3]);
    float * y = (float *)(dst.data + i1 * dst.nb[1] + i2 * dst.nb[2] + i3 * dst.nb[3]);
    const int64_t n = a.ne[0];
    if (!RMS) {
        double s = 0.0;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += (double)x[i];
        s = block_sum<double>(s, shd);
        const float mean = (float)(s / (double)n);
        double s2 = 0.0;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const float v = __fsub_rn(x[i], mean);
            s2 += (double)__fmul_rn(v, v);
        }
        s2 = block_sum<double>(s2, shd);
        const float variance = (float)(s2 / (double)n);
        const float scale = cr_divf(1.0f, cr_sqrtf(__fadd_rn(variance, eps)));
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) y[i] = __fmul_rn(__fsub_rn(x[i], mean), scale);
    } else {
        double s = 0.0;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += (double)__fmul_rn(x[i], x[i]);
        s = block_sum<double>(s, shd);
        const float mean = (float)(s / (double)n);
        const float scale = cr_divf(1.0f, cr_sqrtf(__fadd_rn(mean, eps)));
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) y[i] = __fmul_rn(x[i], scale);
    }
}

// ---- SOFT_MAX ext (scale, optional mask: a 2-D mask's row i01 for every head and sequence, row stride
// ne00; a mask with ne2 / ne3 > 1 broadcast per dim as upstream ggml does, i02 % ne12, i03 % ne13 --
// the per-sequence masks of a ragged lock-step batch) ----
__global__ __launch_bounds__(256) void k_soft_max(TD dst, TD a, TD m, int mask_f16, float scale) {
    __shared__ double shd[8];
    __shared__ float shf[8];
    const int64_t r = blockIdx.x;
    const int64_t nc = a.ne[0];
    const float * sp = (const float *)(a.data + r * a.nb[1]);
    float * dp = (float *)(dst.data + r * dst.nb[1]);
    const int64_t i01 = r % a.ne[1], i02 = (r / a.ne[1]) % a.ne[2], i03 = r / (a.ne[1] * a.ne[2]);
    const char * mask = m.data ? m.data + (i01 % m.ne[1]) * m.nb[1] + (i02 % m.ne[2]) * m.nb[2] + (i03 % m.ne[3]) * m.nb[3] : nullptr;
    float mx = -INFINITY;
    for (int64_t i = threadIdx.x; i < nc; i += blockDim.x) {
        float w = __fmul_rn(sp[i], scale);
        if (mask) {
            const float mv = mask_f16 ? __half2float(((const __half *)mask)[i]) : ((const float *)mask)[i];
            w = __fadd_rn(w, __fmul_rn(1.0f, mv));
        }
        dp[i] = w;
        mx = fmaxf(mx, w);
    }
    mx = block_max(mx, shf);
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < nc; i += blockDim.x) {
        const float v = cr_expf(__fsub_rn(dp[i], mx));
        dp[i] = v;
        s += (double)v;
    }
    s = block_sum<double>(s, shd);
    const float inv = (float)(1.0 / s);
    for (int64_t i = threadIdx.x; i < nc; i += blockDim.x) dp[i] = __fmul_rn(dp[i], inv);
}

// ---- GET_ROWS (f32 / f16 / q4_K / q8_0 source, i32 index) ----
// element k of a table row (dequantize_row_q4_K / q8_0 arithmetic for quantized tables)
__device__ __forceinline__ float table_elem(const TD & s0, const char * src, int64_t k) {
    if (s0.type == TTS_TYPE_F32) return ((const float *)src)[k];
    if (s0.type == TTS_TYPE_F16) return __half2float(((const __half *)src)[k]);
    if (s0.type == TTS_TYPE_Q8_0) {
        const block_q8_0 * b = (const block_q8_0 *)src + k / QK8_0;
        return __fmul_rn((float)b->qs[k % QK8_0], __half2float(__ushort_as_half(b->d)));
    }
    // Q4_K: dequantize_row_q4_K
    const block_q4_K * b = (const block_q4_K *)src + k / QK_K;
    const int e = (int)(k % QK_K);
    const int j64 = e / 64, w = e % 64, hi = w >= 32, l = w % 32;
    // repacked lane layout: byte l*16 + c*4 + k holds weights 64c + 8k + l (+32)
    const int qbyte = (s0.pad & TTS_FLAG_REPACKED) ? ((l & 7) * 16 + j64 * 4 + (l >> 3)) : (32 * j64 + l);
    const int sb = 2 * j64 + hi;
    const uint8_t * q = b->scales;
    int sc, mn;
    if (sb < 4) {
        sc = q[sb] & 63;
        mn = q[sb + 4] & 63;
    } else {
        sc = (q[sb + 4] & 0xF) | ((q[sb - 4] >> 6) << 4);
        mn = (q[sb + 4] >> 4) | ((q[sb] >> 6) << 4);
    }
    const float d = __half2float(__ushort_as_half(b->d));
    const float dm = __half2float(__ushort_as_half(b->dmin));
    const uint8_t qb = b->qs[qbyte];
    const int qv = hi ? (qb >> 4) : (qb & 0xF);
    return __fsub_rn(__fmul_rn(__fmul_rn(d, (float)sc), (float)qv), __fmul_rn(dm, (float)mn));
}

// element k of row `row` of a Q4_K table in the 4-row tile layout (tts_repack_q4_K_tiled)
__device__ __forceinline__ float table_elem_q4K_tiled(const char * base, int64_t row, int64_t nb, int64_t k) {
    const uint8_t * g = (const uint8_t *)base + ((row >> 2) * nb + k / QK_K) * 576;
    const int i = (int)(row & 3);
    const uint8_t * hdr = g + i * 16;
    const int e = (int)(k % QK_K);
    const int c = e / 64, w = e % 64, hi = w >= 32, l = w % 32 % 8, kk = w % 32 / 8;
    const int sb = 2 * c + hi;
    const uint8_t * q = hdr + 4;
    int sc, mn;
    if (sb < 4) {
        sc = q[sb] & 63;
        mn = q[sb + 4] & 63;
    } else {
        sc = (q[sb + 4] & 0xF) | ((q[sb - 4] >> 6) << 4);
        mn = (q[sb + 4] >> 4) | ((q[sb] >> 6) << 4);
    }
    const float d = __half2float(__ushort_as_half(*(const uint16_t *)hdr));
    const float dm = __half2float(__ushort_as_half(*(const uint16_t *)(hdr + 2)));
    const uint8_t qb = g[64 + ((c * 2 + (l >> 2)) * 4 + i) * 16 + (l & 3) * 4 + kk];
    const int qv = hi ? (qb >> 4) : (qb & 0xF);
    return __fsub_rn(__fmul_rn(__fmul_rn(d, (float)sc), (float)qv), __fmul_rn(dm, (float)mn));
}

__global__ void k_get_rows(TD dst, TD s0, TD s1) {
    const int64_t i = blockIdx.x;  // index into flattened s1
    const int64_t i10 = i % s1.ne[0], i11 = (i / s1.ne[0]) % s1.ne[1], i12 = i / (s1.ne[0] * s1.ne[1]);
    const int64_t i01 = *(const int32_t *)(s1.data + i10 * s1.nb[0] + i11 * s1.nb[1] + i12 * s1.nb[2]);
    const char * src = s0.data + i01 * s0.nb[1] + i11 * s0.nb[2] + i12 * s0.nb[3];
    float * out = (float *)(dst.data + i10 * dst.nb[1] + i11 * dst.nb[2] + i12 * dst.nb[3]);
    const int64_t nc = s0.ne[0];
    if (s0.type == TTS_TYPE_Q4_K && (s0.pad & TTS_FLAG_TILED)) {  // 2-D tables only (weight_set)
        for (int64_t k = threadIdx.x; k < nc; k += blockDim.x) out[k] = table_elem_q4K_tiled(s0.data, i01, nc / QK_K, k);
        return;
    }
    for (int64_t k = threadIdx.x; k < nc; k += blockDim.x) out[k] = table_elem(s0, src, k);
}

// A chain of ADDs over GET_ROWS terms (parler_build_inp_embd, model.cpp:387-410: the 9 codebook
// embeddings summed, then the positional row) in one launch.  Terms are added in the chain's
// evaluation order, each add rounded to f32 as the unfused ADD nodes do; a term with one index
// row broadcasts over the output columns (ggml's ADD broadcast of src1).
struct EmbedTerm {
    TD table;
    const int32_t * idx;
    int64_t idx_stride;  // elements
    int64_t rows;        // 1 = broadcast
    const int64_t * moff;  // column m's index at idx[moff[m]] (a coalesced step's member-owned inputs), or null
};
struct EmbedArgs {
    EmbedTerm t[EMBED_MAX_TERMS];
    int n;
    float * out;
    int64_t H, M;
    int64_t ocs;  // floats between output columns
};

__global__ void k_embed_sum(EmbedArgs a) {
    const int64_t m = blockIdx.y;
    const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= a.H) return;
    float acc = 0.f;
    for (int t = 0; t < a.n; ++t) {
        const EmbedTerm & T = a.t[t];
        const int64_t r = T.moff ? T.idx[T.moff[m]] : T.idx[(T.rows == 1 ? 0 : m) * T.idx_stride];
        const float v = (T.table.type == TTS_TYPE_Q4_K && (T.table.pad & TTS_FLAG_TILED))
                            ? table_elem_q4K_tiled(T.table.data, r, T.table.ne[0] / QK_K, h)
                            : table_elem(T.table, T.table.data + r * T.table.nb[1], h);
        acc = t == 0 ? v : __fadd_rn(acc, v);
    }
    a.out[m * a.ocs + h] = acc;
}

void launch_embed_sum(tts_hip_backend * be, const tts_tensor * out, const tts_tensor * const * gr, int n, const BatchCtx * bat,
                      const ItemTab * tab) {
    EmbedArgs a{};
    a.n = n;
    a.out = (float *)out->data;
    a.H = out->ne[0];
    a.M = out->ne[1] * out->ne[2] * out->ne[3];
    a.ocs = a.H;
    for (int i = 0; i < n; ++i) {
        a.t[i].table = make_td(gr[i]->src[0]);
        a.t[i].idx = (const int32_t *)gr[i]->src[1]->data;
        a.t[i].idx_stride = (int64_t)(gr[i]->src[1]->nb[0] / 4);
        a.t[i].rows = gr[i]->ne[1] * gr[i]->ne[2] * gr[i]->ne[3];
    }
    if (bat) {  // one row per member (a coalesced step's one-token graphs): column m = member m
        a.M = bat->N;
        a.ocs = bat->stride(a.out) / 4;
        a.out = bat->win(a.out);
        for (int i = 0; i < n; ++i) {
            if (tab && tab->ioff[i]) {  // each member's own index tensor (an input)
                a.t[i].moff = tab->ioff[i];
                a.t[i].rows = bat->N;
                continue;
            }
            const int64_t s = bat->stride(a.t[i].idx);
            a.t[i].idx_stride = s / 4;
            a.t[i].rows = s ? bat->N : 1;
            a.t[i].idx = bat->win(a.t[i].idx);
        }
    }
    hipLaunchKernelGGL(k_embed_sum, dim3((unsigned)((a.H + 255) / 256), (unsigned)a.M), dim3(256), 0, be->stream, a);
    TTS_HIP_CHECK(hipGetLastError());
}

// ---- CONCAT / REPEAT / SUM_ROWS ----
__global__ void k_concat(TD dst, TD a, TD b, int dim, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t i[4];
        unravel(k, dst.ne, i[0], i[1], i[2], i[3]);
        float v;
        if (i[0] < a.ne[0] && i[1] < a.ne[1] && i[2] < a.ne[2] && i[3] < a.ne[3]) v = td_load(a, i[0], i[1], i[2], i[3]);
        else {
            i[dim] -= a.ne[dim];
            v = td_load(b, i[0], i[1], i[2], i[3]);
            i[dim] += a.ne[dim];
        }
        td_store(dst, i[0], i[1], i[2], i[3], v);
    }
}

__global__ void k_repeat(TD dst, TD a, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unravel(k, dst.ne, i0, i1, i2, i3);
        td_store(dst, i0, i1, i2, i3, td_load(a, i0 % a.ne[0], i1 % a.ne[1], i2 % a.ne[2], i3 % a.ne[3]));
    }
}

__global__ __launch_bounds__(256) void k_sum_rows(TD dst, TD a) {
    __shared__ double shd[8];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % a.ne[1], i2 = (r / a.ne[1]) % a.ne[2], i3 = r / (a.ne[1] * a.ne[2]);
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < a.ne[0]; i += blockDim.x) s += (double)td_load(a, i, i1, i2, i3);
    s = block_sum<double>(s, shd);
    if (threadIdx.x == 0) td_store(dst, 0, i1, i2, i3, (float)s);
}

// ---- ROPE (NORM / NEOX, optional freq factors; theta by repeated multiply as ggml_rope_cache_init) ----
// dst: one or more destinations of the source's shape (the planner's rope + repeat-copy item writes
// every repeat copy of the rotated K directly)
__global__ void k_rope(CpyMulti m, TD a, const int32_t * pos, const float * ff, int n_dims, int neox, float theta_scale,
                       float freq_scale, float attn_factor) {
    auto td_store_all = [&](int64_t j0, int64_t i1, int64_t i2, int64_t i3, float v) {
        for (int d = 0; d < m.nd; ++d) td_store(m.dst[d], j0, i1, i2, i3, v);
    };
    const int64_t i1 = blockIdx.x, i2 = blockIdx.y, i3 = blockIdx.z;
    const int64_t p = pos[i2];
    for (int64_t i0 = 2 * threadIdx.x; i0 < a.ne[0]; i0 += 2 * blockDim.x) {
        if (i0 < n_dims) {
            float theta = (float)p;
            for (int64_t k = 0; k < i0 / 2; ++k) theta = __fmul_rn(theta, theta_scale);
            const float f = ff ? ff[i0 / 2] : 1.0f;
            const float th = __fmul_rn(freq_scale, cr_divf(theta, f));
            const float c = __fmul_rn(cr_cosf(th), attn_factor), s = __fmul_rn(cr_sinf(th), attn_factor);
            int64_t j0, j1;
            if (neox) {
                j0 = i0 / 2;
                j1 = i0 / 2 + n_dims / 2;
            } else {
                j0 = i0;
                j1 = i0 + 1;
            }
            const float x0 = td_load(a, j0, i1, i2, i3), x1 = td_load(a, j1, i1, i2, i3);
            td_store_all(j0, i1, i2, i3, __fsub_rn(__fmul_rn(x0, c), __fmul_rn(x1, s)));
            td_store_all(j1, i1, i2, i3, __fadd_rn(__fmul_rn(x0, s), __fmul_rn(x1, c)));
        } else {
            const float x0 = td_load(a, i0, i1, i2, i3);
            const float x1 = i0 + 1 < a.ne[0] ? td_load(a, i0 + 1, i1, i2, i3) : 0.f;
            td_store_all(i0, i1, i2, i3, x0);
            if (i0 + 1 < a.ne[0]) td_store_all(i0 + 1, i1, i2, i3, x1);
        }
    }
}

// ---- generic MUL_MAT (attention products, small conv GEMMs): one wave per output, f64
// accumulation.  With an F16 src0, ggml converts src1 to F16 (vec_dot_type) before the dot
// (ggml_vec_dot_f16), so each src1 element is rounded to f16 here too; f16 x f16 products are
// exact in f32. ----
__global__ __launch_bounds__(256) void k_mul_mat_f32(TD dst, TD s0, TD s1, int64_t nout) {
    const int lane = threadIdx.x & 63;
    const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= nout) return;
    const int64_t i01 = o % dst.ne[0];
    int64_t rest = o / dst.ne[0];
    const int64_t i11 = rest % dst.ne[1];
    rest /= dst.ne[1];
    const int64_t i12 = rest % dst.ne[2];
    const int64_t i13 = rest / dst.ne[2];
    const int64_t i02 = i12 / (s1.ne[2] / s0.ne[2]), i03 = i13 / (s1.ne[3] / s0.ne[3]);
    const char * a = s0.data + i01 * s0.nb[1] + i02 * s0.nb[2] + i03 * s0.nb[3];
    const char * b = s1.data + i11 * s1.nb[1] + i12 * s1.nb[2] + i13 * s1.nb[3];
    double acc = 0.0;
    const int64_t K = s0.ne[0];
    for (int64_t k = lane; k < K; k += 64) {
        const float x = s0.type == TTS_TYPE_F16 ? __half2float(*(const __half *)(a + k * s0.nb[0])) : *(const float *)(a + k * s0.nb[0]);
        float y = s1.type == TTS_TYPE_F16 ? __half2float(*(const __half *)(b + k * s1.nb[0])) : *(const float *)(b + k * s1.nb[0]);
        if (s0.type == TTS_TYPE_F16) y = __half2float(__float2half_rn(y));
        acc += (double)__fmul_rn(x, y);
    }
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) *(float *)(dst.data + i01 * dst.nb[0] + i11 * dst.nb[1] + i12 * dst.nb[2] + i13 * dst.nb[3]) = (float)acc;
}

// Short rows (K <= 32: Kokoro's harmonic merge Linear(9, 1), the 1-tap noise conv over 22 STFT
// channels): one thread per output, the dot summed sequentially in f64 as the oracle does.
__global__ __launch_bounds__(256) void k_mul_mat_smallk(TD dst, TD s0, TD s1, int64_t nout) {
    const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= nout) return;
    const int64_t i01 = o % dst.ne[0];
    int64_t rest = o / dst.ne[0];
    const int64_t i11 = rest % dst.ne[1];
    rest /= dst.ne[1];
    const int64_t i12 = rest % dst.ne[2];
    const int64_t i13 = rest / dst.ne[2];
    const int64_t i02 = i12 / (s1.ne[2] / s0.ne[2]), i03 = i13 / (s1.ne[3] / s0.ne[3]);
    const char * a = s0.data + i01 * s0.nb[1] + i02 * s0.nb[2] + i03 * s0.nb[3];
    const char * b = s1.data + i11 * s1.nb[1] + i12 * s1.nb[2] + i13 * s1.nb[3];
    double acc = 0.0;
    const int64_t K = s0.ne[0];
    for (int64_t k = 0; k < K; ++k) {
        const float x = s0.type == TTS_TYPE_F16 ? __half2float(*(const __half *)(a + k * s0.nb[0])) : *(const float *)(a + k * s0.nb[0]);
        float y = s1.type == TTS_TYPE_F16 ? __half2float(*(const __half *)(b + k * s1.nb[0])) : *(const float *)(b + k * s1.nb[0]);
        if (s0.type == TTS_TYPE_F16) y = __half2float(__float2half_rn(y));
        acc += (double)__fmul_rn(x, y);
    }
    *(float *)(dst.data + i01 * dst.nb[0] + i11 * dst.nb[1] + i12 * dst.nb[2] + i13 * dst.nb[3]) = (float)acc;
}

// ------------------------------------------------------------------------------------------

static inline float op_f(const tts_tensor * t, int i) {
    float f;
    memcpy(&f, &t->op_params[i], 4);
    return f;
}
static inline int64_t nel(const tts_tensor * t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }
static inline bool is_cont(const tts_tensor * t) {
    size_t es = tts_type_size(t->type);
    return t->nb[0] == es && t->nb[1] == t->nb[0] * t->ne[0] && t->nb[2] == t->nb[1] * t->ne[1] && t->nb[3] == t->nb[2] * t->ne[2];
}
static inline unsigned grid_for(int64_t n, int bs = 256) {
    int64_t g = (n + bs - 1) / bs;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (unsigned)g;
}

// ROPE node `rope` over `src` (its source, or the tensor a skipped copy would have produced it from),
// written to every tensor in dsts (each of the source's shape)
void launch_rope_multi(tts_hip_backend * be, const tts_tensor * rope, const tts_tensor * src, const tts_tensor * const * dsts, int nd) {
    CpyMulti m{};
    m.nd = nd;
    for (int i = 0; i < nd; ++i) m.dst[i] = make_td(dsts[i]);
    const int n_dims = rope->op_params[1];
    const int mode = rope->op_params[2];
    const float freq_base = op_f(rope, 5), freq_scale = op_f(rope, 6), attn_factor = op_f(rope, 8);
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    const tts_tensor * ff = rope->src[2];
    dim3 grid((unsigned)src->ne[1], (unsigned)src->ne[2], (unsigned)src->ne[3]);
    hipLaunchKernelGGL(k_rope, grid, dim3(64), 0, be->stream, m, make_td(src), (const int32_t *)rope->src[1]->data,
                       ff ? (const float *)ff->data : nullptr, n_dims, (mode & 2) ? 1 : 0, theta_scale, freq_scale, attn_factor);
    TTS_HIP_CHECK(hipGetLastError());
}

int launch_op(tts_hip_backend * be, const tts_tensor * node) {
    hipStream_t st = be->stream;
    const tts_tensor * s0 = node->src[0];
    const tts_tensor * s1 = node->src[1];
    TD d = make_td(node);
    switch (node->op) {
        case TTS_OP_DUP:
        case TTS_OP_CONT:
        case TTS_OP_CPY: {
            const int64_t n = nel(s0);
            if (n == 0) return 0;
            if (is_cont(s0) && is_cont(node) && s0->type == node->type) {
                launch_copy_bytes(be, node->data, s0->data, n * tts_type_size(s0->type));
                return 0;
            }
            hipLaunchKernelGGL(k_cpy, dim3(grid_for(n)), dim3(256), 0, st, d, make_td(s0), n);
        } break;
        case TTS_OP_ADD:
        case TTS_OP_SUB:
        case TTS_OP_MUL:
        case TTS_OP_DIV: {
            const int64_t n = nel(node);
            if (n == 0) return 0;
            const bool fast = is_cont(node) && is_cont(s0) && is_cont(s1) && node->type == TTS_TYPE_F32 &&
                              s0->type == TTS_TYPE_F32 && s1->type == TTS_TYPE_F32 && s1->ne[0] == s0->ne[0] &&
                              (n % nel(s1)) == 0 &&
                              (s1->ne[1] == s0->ne[1] || s1->ne[1] == 1) && s1->ne[2] == 1 && s1->ne[3] == 1;
            const dim3 g(grid_for(n)), b(256);
            const bool rowbc = !fast && is_cont(node) && is_cont(s0) && is_cont(s1) && node->type == TTS_TYPE_F32 && s0->type == TTS_TYPE_F32 &&
                               s1->type == TTS_TYPE_F32 && s1->ne[0] == 1 && s0->ne[0] > 1 && (s1->ne[1] == s0->ne[1] || s1->ne[1] == 1) &&
                               s1->ne[2] == 1 && s1->ne[3] == 1 && nel(node) == nel(s0);
            if (rowbc) {
                const int64_t ne0 = s0->ne[0], nb1 = s1->ne[1];
                const bool v4 = ne0 % 4 == 0 && ((uintptr_t)node->data % 16) == 0 && ((uintptr_t)s0->data % 16) == 0;
                const dim3 g4(grid_for(v4 ? n / 4 : n));
                float * D = (float *)node->data;
                const float *A = (const float *)s0->data, *B = (const float *)s1->data;
#define TTS_ROWBC(OPV)                                                                                   \
    if (v4) hipLaunchKernelGGL((k_binary_rowbc<OPV, 4>), g4, b, 0, st, D, A, B, n, ne0, nb1);             \
    else hipLaunchKernelGGL((k_binary_rowbc<OPV, 1>), g4, b, 0, st, D, A, B, n, ne0, nb1);
                switch (node->op) {
                    case TTS_OP_ADD: TTS_ROWBC(TTS_OP_ADD) break;
                    case TTS_OP_SUB: TTS_ROWBC(TTS_OP_SUB) break;
                    case TTS_OP_MUL: TTS_ROWBC(TTS_OP_MUL) break;
                    default: TTS_ROWBC(TTS_OP_DIV) break;
                }
#undef TTS_ROWBC
            } else if (fast) {
                const int64_t nb_el = nel(s1);
                switch (node->op) {
                    case TTS_OP_ADD: hipLaunchKernelGGL(k_binary_cont<TTS_OP_ADD>, g, b, 0, st, (float *)node->data, (const float *)s0->data, (const float *)s1->data, n, nb_el); break;
                    case TTS_OP_SUB: hipLaunchKernelGGL(k_binary_cont<TTS_OP_SUB>, g, b, 0, st, (float *)node->data, (const float *)s0->data, (const float *)s1->data, n, nb_el); break;
                    case TTS_OP_MUL: hipLaunchKernelGGL(k_binary_cont<TTS_OP_MUL>, g, b, 0, st, (float *)node->data, (const float *)s0->data, (const float *)s1->data, n, nb_el); break;
                    default: hipLaunchKernelGGL(k_binary_cont<TTS_OP_DIV>, g, b, 0, st, (float *)node->data, (const float *)s0->data, (const float *)s1->data, n, nb_el); break;
                }
            } else {
                TD a = make_td(s0), bb = make_td(s1);
                switch (node->op) {
                    case TTS_OP_ADD: hipLaunchKernelGGL(k_binary<TTS_OP_ADD>, g, b, 0, st, d, a, bb, n); break;
                    case TTS_OP_SUB: hipLaunchKernelGGL(k_binary<TTS_OP_SUB>, g, b, 0, st, d, a, bb, n); break;
                    case TTS_OP_MUL: hipLaunchKernelGGL(k_binary<TTS_OP_MUL>, g, b, 0, st, d, a, bb, n); break;
                    default: hipLaunchKernelGGL(k_binary<TTS_OP_DIV>, g, b, 0, st, d, a, bb, n); break;
                }
            }
        } break;
        case TTS_OP_SQR: case TTS_OP_SQRT: case TTS_OP_SIN: case TTS_OP_COS: case TTS_OP_SCALE: case TTS_OP_CLAMP:
        case TTS_OP_LEAKY_RELU: case TTS_OP_ROUND: case TTS_OP_MOD: case TTS_OP_UNARY: {
            const int64_t n = nel(node);
            if (n == 0) return 0;
            UnaryParams P;
            P.op = node->op;
            P.uop = node->op == TTS_OP_UNARY ? node->op_params[0] : -1;
            P.p0 = op_f(node, 0);
            P.p1 = op_f(node, 1);
            P.gelu_table = be->gelu_table;
            if (is_cont(node) && is_cont(s0) && node->type == TTS_TYPE_F32 && s0->type == TTS_TYPE_F32)
                hipLaunchKernelGGL(k_unary_cont, dim3(grid_for(n)), dim3(256), 0, st, (float *)node->data, (const float *)s0->data, n, P);
            else
                hipLaunchKernelGGL(k_unary, dim3(grid_for(n)), dim3(256), 0, st, d, make_td(s0), n, P);
        } break;
        case TTS_OP_NORM:
        case TTS_OP_RMS_NORM: {
            const int64_t nr = s0->ne[1] * s0->ne[2] * s0->ne[3];
            if (node->op == TTS_OP_NORM) hipLaunchKernelGGL(k_norm<false>, dim3((unsigned)nr), dim3(256), 0, st, d, make_td(s0), op_f(node, 0));
            else hipLaunchKernelGGL(k_norm<true>, dim3((unsigned)nr), dim3(256), 0, st, d, make_td(s0), op_f(node, 0));
        } break;
        case TTS_OP_SOFT_MAX: {
            const int64_t nr = s0->ne[1] * s0->ne[2] * s0->ne[3];
            const tts_tensor * m = node->src[1];
            TD md{};
            if (m) {
                md = make_td(m);
                // rows of ne00 elements (ggml reads mask rows with stride ne00)
                md.nb[1] = (size_t)tts_type_size(m->type) * (size_t)s0->ne[0];
                if (m->ne[2] * m->ne[3] == 1) md.nb[2] = md.nb[3] = 0, md.ne[2] = md.ne[3] = 1;
            } else {
                md.ne[1] = md.ne[2] = md.ne[3] = 1;
            }
            hipLaunchKernelGGL(k_soft_max, dim3((unsigned)nr), dim3(256), 0, st, d, make_td(s0), md, m ? (m->type == TTS_TYPE_F16) : 0,
                               op_f(node, 0));
        } break;
        case TTS_OP_GET_ROWS: {
            const int64_t nr = s1->ne[0] * s1->ne[1] * s1->ne[2];
            hipLaunchKernelGGL(k_get_rows, dim3((unsigned)nr), dim3(256), 0, st, d, make_td(s0), make_td(s1));
        } break;
        case TTS_OP_CONCAT: {
            const int64_t n = nel(node);
            hipLaunchKernelGGL(k_concat, dim3(grid_for(n)), dim3(256), 0, st, d, make_td(s0), make_td(s1), node->op_params[0], n);
        } break;
        case TTS_OP_REPEAT: {
            const int64_t n = nel(node);
            hipLaunchKernelGGL(k_repeat, dim3(grid_for(n)), dim3(256), 0, st, d, make_td(s0), n);
        } break;
        case TTS_OP_SUM_ROWS: {
            const int64_t nr = s0->ne[1] * s0->ne[2] * s0->ne[3];
            hipLaunchKernelGGL(k_sum_rows, dim3((unsigned)nr), dim3(256), 0, st, d, make_td(s0));
        } break;
        case TTS_OP_ROPE: launch_rope_multi(be, node, s0, &node, 1); break;
        case TTS_OP_MUL_MAT: {
            // F16 src0 with many columns (conv_1d's GEMM) on the matrix cores; otherwise the generic
            // float path (quantized weights go through the GEMV kernels)
            if (launch_gemm_f16(be, node)) return 0;
            const int64_t nout = nel(node);
            // plain float GEMM (2-D weights, columns collapsible, dense output) on the tiled kernel
            if (s0->type == TTS_TYPE_F32 && s1->type == TTS_TYPE_F32 && node->type == TTS_TYPE_F32 && s0->ne[0] > 32 && s0->ne[1] >= 16 &&
                s0->ne[2] * s0->ne[3] == 1 && s0->nb[0] == 4 && s1->nb[0] == 4 && is_cont(node) && (s0->nb[1] % 4) == 0 &&
                (s1->nb[1] % 4) == 0 &&
                (s1->ne[2] * s1->ne[3] == 1 || (s1->nb[2] == s1->nb[1] * (size_t)s1->ne[1] && s1->nb[3] == s1->nb[2] * (size_t)s1->ne[2]))) {
                GemvJob j;
                j.wtype = TTS_TYPE_F32;
                j.K = s0->ne[0];
                j.N = s0->ne[1];
                j.M = s1->ne[1] * s1->ne[2] * s1->ne[3];
                j.w_row_bytes = (int64_t)s0->nb[1];
                j.W[0] = (const uint8_t *)s0->data;
                j.x = (const float *)s1->data;
                j.xcs = (int64_t)(s1->nb[1] / 4);
                j.Y[0] = (float *)node->data;
                j.ycs[0] = (int64_t)(node->nb[1] / 4);
                j.yrs[0] = 1;
                if (j.M > 8 && gemm_f32_ok(j)) {
                    launch_gemm_f32(be, j);
                    return 0;
                }
            }
            if (launch_bgemm_f32(be, node)) return 0;  // batched float products over many queries
            if (s0->ne[0] <= 32) {
                hipLaunchKernelGGL(k_mul_mat_smallk, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, st, d, make_td(s0), make_td(s1), nout);
                break;
            }
            hipLaunchKernelGGL(k_mul_mat_f32, dim3((unsigned)((nout + 3) / 4)), dim3(256), 0, st, d, make_td(s0), make_td(s1), nout);
        } break;
        case TTS_OP_IM2COL: launch_im2col(be, node); return 0;
        case TTS_OP_CONV_TRANSPOSE_1D: launch_conv_transpose_1d(be, node); return 0;
        case TTS_OP_CUMSUM: case TTS_OP_UPSCALE: case TTS_OP_STFT: case TTS_OP_ISTFT: case TTS_OP_MAP_CUSTOM3: case TTS_OP_MAP_CUSTOM2: return launch_audio_op(be, node);
        default:
            return TTS_STATUS_UNSUPPORTED;
    }
    TTS_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace tts

namespace tts {

// ---- streaming copy (tts_hip_copy_stream): the HBM ceiling the bench reports beside the 8 TB/s spec ----
// Each workgroup copies one contiguous chunk, four consecutive 4 KB pieces in flight per iteration
// (16-B non-temporal loads / stores per lane).  Measured on MI355X (scripts/copy_peak.hip,
// profiles/r06/copy_peak_variants.txt): 5.5-5.7 TB/s read + write at 16 workgroups per CU, against
// 4.4-5.1 for the grid-stride form of the same loads.
__global__ __launch_bounds__(256) void k_copy_stream(uint4 * __restrict__ dst, const uint4 * __restrict__ src, int64_t n16) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    u4v * d = (u4v *)dst;
    const u4v * s = (const u4v *)src;
    const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = b0 + per < n16 ? b0 + per : n16;
    int64_t i = b0 + threadIdx.x;
    for (; i + 3 * 256 < b1; i += 4 * 256) {
        u4v v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(s + i + u * 256);
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], d + i + u * 256);
    }
    for (; i < b1; i += 256) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

void launch_copy_stream(tts_hip_backend * be, void * dst, const void * src, int64_t n16) {
    hipLaunchKernelGGL(k_copy_stream, dim3((unsigned)(16 * be->cu_total)), dim3(256), 0, be->stream, (uint4 *)dst, (const uint4 *)src, n16);
}

}  // namespace tts
