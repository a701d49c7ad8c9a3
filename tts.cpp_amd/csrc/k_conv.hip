// Codec convolutions (DAC / SNAC / Kokoro vocoders):
//
//  k_im2col          : GGML_OP_IM2COL, 1-D form used by ggml_conv_1d (general_neural_audio_codec.cpp
//                      :133-149, dac_model.cpp:158,164): dst (ic*K + k, ol) = x[ol*s + k*d - p, ic],
//                      F16 (round to nearest even) or F32.
//  k_gemm_f16_mfma   : the MUL_MAT that follows it (src0 = im2col F16 [K', OL], src1 = kernel [K', OC]
//                      F32/F16, converted to F16 = ggml's vec_dot_type for an F16 src0) on the matrix
//                      cores: v_mfma_f32_16x16x32_f16, f32 accumulation.  fp16 x fp16 products are
//                      exact in f32; only the accumulation order/precision differs from ggml-cpu's
//                      f64 generic dot, so results agree to ~1e-6 relative (tests: conv vs oracle).
//  k_conv_transpose_1d: the fork's GGML_OP_CONV_TRANSPOSE_1D (general_neural_audio_codec.cpp:153,
//                      kokoro model.cpp:104,211) with PyTorch ConvTranspose1d semantics, one output
//                      per lane, only the taps that land on it (k = r + j*s for dilation 1), f64
//                      accumulation in the oracle's order.
#include "hip_internal.h"

namespace tts {

// ------------------------------------------------------------------------------------------
template <bool F16OUT>
__global__ void k_im2col(TD dst, TD x, int K, int s0, int p0, int d0, int64_t n) {
    const int64_t KW = dst.ne[0];  // IC*K
    const int64_t OL = dst.ne[1];
    const int64_t L = x.ne[0];
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t kk = e % KW;
        const int64_t ol = (e / KW) % OL;
        const int64_t nn = e / (KW * OL);
        const int64_t ic = kk / K, k = kk % K;
        const int64_t il = ol * s0 + k * d0 - p0;
        float v = 0.f;
        if (il >= 0 && il < L) v = *(const float *)(x.data + il * x.nb[0] + ic * x.nb[1] + nn * x.nb[2]);
        char * o = dst.data + kk * dst.nb[0] + ol * dst.nb[1] + nn * dst.nb[2];
        if (F16OUT) *(__half *)o = __float2half_rn(v);
        else *(float *)o = v;
    }
}

void launch_im2col(tts_hip_backend * be, const tts_tensor * node) {
    const tts_tensor * a = node->src[0];
    const tts_tensor * b = node->src[1];
    const int64_t n = node->ne[0] * node->ne[1] * node->ne[2];
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 65535 * 8);
    const int K = (int)a->ne[0], s0 = node->op_params[0], p0 = node->op_params[2], d0 = node->op_params[4];
    if (node->type == TTS_TYPE_F16)
        hipLaunchKernelGGL(k_im2col<true>, dim3(grid), dim3(256), 0, be->stream, make_td(node), make_td(b), K, s0, p0, d0, n);
    else
        hipLaunchKernelGGL(k_im2col<false>, dim3(grid), dim3(256), 0, be->stream, make_td(node), make_td(b), K, s0, p0, d0, n);
    TTS_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// dst[j][i] = sum_k A[i][k] * B[j][k] (ggml mul_mat: i = src0 row, j = src1 column).
// A F16 rows (stride lda elements), B F32 or F16 columns (stride ldb elements), K % 8 == 0, rows
// 16-B aligned.  Wave tile 32 (i) x 32 (j) = 2 x 2 MFMA 16x16x32 tiles; workgroup 2 x 2 waves =
// 64 x 64.  Lane l holds A[row l&15][k = 8(l>>4) .. +7] and B[k = 8(l>>4) .. +7][col l&15]; the
// accumulator's column is l&15 (j) and its row (l>>4)*4 + reg (i), so each lane stores 4
// consecutive i of one j.  Fragments for step k+32 are loaded before the MFMAs of step k.
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <bool BF16>
__device__ __forceinline__ half8_t load_b_frag(const void * B, int64_t ldb, int64_t col, int64_t k) {
    half8_t r;
    if (BF16) {
        const uint4 u = *(const uint4 *)((const __half *)B + col * ldb + k);
        r = __builtin_bit_cast(half8_t, u);
    } else {
        const float4 lo = *(const float4 *)((const float *)B + col * ldb + k);
        const float4 hi = *(const float4 *)((const float *)B + col * ldb + k + 4);
        r[0] = (_Float16)__float2half_rn(lo.x), r[1] = (_Float16)__float2half_rn(lo.y);
        r[2] = (_Float16)__float2half_rn(lo.z), r[3] = (_Float16)__float2half_rn(lo.w);
        r[4] = (_Float16)__float2half_rn(hi.x), r[5] = (_Float16)__float2half_rn(hi.y);
        r[6] = (_Float16)__float2half_rn(hi.z), r[7] = (_Float16)__float2half_rn(hi.w);
    }
    return r;
}

template <bool BF16>
__global__ __launch_bounds__(256) void k_gemm_f16_mfma(const __half * __restrict__ A, int64_t lda, const void * __restrict__ B, int64_t ldb,
                                                       float * __restrict__ D, int64_t ldd, int64_t M, int64_t N, int64_t K) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t i0 = (int64_t)blockIdx.x * 64 + (wave & 1) * 32;
    const int64_t j0 = (int64_t)blockIdx.y * 64 + (wave >> 1) * 32;
    const int r16 = lane & 15, kq = lane >> 4;
    int64_t ia[2], jb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        ia[t] = min(i0 + 16 * t + r16, M - 1);
        jb[t] = min(j0 + 16 * t + r16, N - 1);
    }
    f32x4_t acc[2][2] = {};
    half8_t a[2], b[2], an[2], bn[2];
    auto load = [&](int64_t k0, half8_t (&fa)[2], half8_t (&fb)[2]) {
        const int64_t k = k0 + 8 * kq;
        const bool kin = k < K;  // K % 8 == 0: a lane's 8 elements are all in or all out
        const int64_t kc = kin ? k : 0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            half8_t va = __builtin_bit_cast(half8_t, *(const uint4 *)(A + ia[t] * lda + kc));
            half8_t vb = load_b_frag<BF16>(B, ldb, jb[t], kc);
            const half8_t z = {};
            fa[t] = kin ? va : z;
            fb[t] = kin ? vb : z;
        }
    };
    load(0, a, b);
    for (int64_t k0 = 0; k0 < K; k0 += 32) {
        if (k0 + 32 < K) load(k0 + 32, an, bn);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ti], b[tj], acc[ti][tj], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 2; ++t) a[t] = an[t], b[t] = bn[t];
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
            const int64_t j = j0 + 16 * tj + r16;
            const int64_t i = i0 + 16 * ti + 4 * kq;
            if (j >= N) continue;
            float * dp = D + j * ldd + i;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (i + e < M) dp[e] = acc[ti][tj][e];
        }
    }
}

// The same product accumulated in f64 on the f64 matrix cores (v_mfma_f64_16x16x4_f64): fp16 x fp16
// products are exact in f64 and ggml-cpu's generic F16 dot sums them in f64 (ggml_vec_dot_f16), so
// the f32 result equals the oracle's except for f64 near-ties -- which keeps a deep codec (the fp16
// re-rounding of every conv input amplifies 1e-7 differences into 5e-4 PCM errors) inside the
// PCM bar.  Lane l covers k = k0 + 8(l>>4) + t at MFMA step t = 0..7 of a 32-wide K step: every k
// of the step is used once, so the lane loads its 8 contiguous k as one 16-B fragment.
// MFMA f64 16x16x4 maps: A[i = l&15][k], B[k][j = l&15]; D col = l&15 (j), row = (l>>4) + 4*reg (i).
typedef double f64x4_t __attribute__((ext_vector_type(4)));

template <bool BF16>
__global__ __launch_bounds__(256) void k_gemm_f16_f64acc(const __half * __restrict__ A, int64_t lda, const void * __restrict__ B, int64_t ldb,
                                                         float * __restrict__ D, int64_t ldd, int64_t M, int64_t N, int64_t K,
                                                         double * __restrict__ part = nullptr, int64_t kps = 0) {
    // split launch (part != null): workgroup z reduces k in [z*kps, (z+1)*kps) into part[z][j][i]
    const int64_t kb = part ? (int64_t)blockIdx.z * kps : 0;
    const int64_t ke = part ? min(K, kb + kps) : K;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t i0 = (int64_t)blockIdx.x * 64 + (wave & 1) * 32;
    const int64_t j0 = (int64_t)blockIdx.y * 64 + (wave >> 1) * 32;
    const int r16 = lane & 15, kq = lane >> 4;
    int64_t ia[2], jb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        ia[t] = min(i0 + 16 * t + r16, M - 1);
        jb[t] = min(j0 + 16 * t + r16, N - 1);
    }
    f64x4_t acc[2][2] = {};
    half8_t a[2], b[2], an[2], bn[2];
    auto load = [&](int64_t k0, half8_t (&fa)[2], half8_t (&fb)[2]) {
        const int64_t k = k0 + 8 * kq;
        const bool kin = k < ke;
        const int64_t kc = kin ? k : 0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            half8_t va = __builtin_bit_cast(half8_t, *(const uint4 *)(A + ia[t] * lda + kc));
            half8_t vb = load_b_frag<BF16>(B, ldb, jb[t], kc);
            const half8_t z = {};
            fa[t] = kin ? va : z;
            fb[t] = kin ? vb : z;
        }
    };
    load(kb, a, b);
    for (int64_t k0 = kb; k0 < ke; k0 += 32) {
        if (k0 + 32 < ke) load(k0 + 32, an, bn);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            double ad[2], bd[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) ad[u] = (double)(float)a[u][t], bd[u] = (double)(float)b[u][t];
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(ad[ti], bd[tj], acc[ti][tj], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) a[t] = an[t], b[t] = bn[t];
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
            const int64_t j = j0 + 16 * tj + r16;
            if (j >= N) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t i = i0 + 16 * ti + kq + 4 * e;
                if (i >= M) continue;
                if (part) part[((int64_t)blockIdx.z * N + j) * M + i] = acc[ti][tj][e];
                else D[j * ldd + i] = (float)acc[ti][tj][e];
            }
        }
    }
}

// Second pass of a split reduction: y[i + j*ldy] = f32(sum over z, in order, of part[z][j][i]),
// then + bias[j * bcs] and + res[i + j * rcs] (each rounded, as the ADD nodes they replace).
__global__ __launch_bounds__(256) void k_split_reduce(const double * __restrict__ part, int nz, int64_t M, int64_t N, float * __restrict__ y,
                                                      int64_t ldy, const float * __restrict__ bias, int64_t bcs, const float * __restrict__ res,
                                                      int64_t rcs) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= M * N) return;
    const int64_t j = e / M, i = e - j * M;
    double s = 0.0;
    for (int z = 0; z < nz; ++z) s += part[((int64_t)z * N + j) * M + i];
    float v = (float)s;
    if (bias) v = v + bias[j * bcs];
    if (res) v = res[i + j * rcs] + v;
    y[i + j * ldy] = v;
}

// Splits for a reduction of length K over an output grid of `tiles` workgroups: enough extra
// workgroups to fill the chip (~2 per CU) while each split keeps >= `minlen` of the reduction and
// the partials fit the scratch.  Returns 1 (no split) for grids that already fill the chip.
static int split_count(const tts_hip_backend * be, int64_t tiles, int64_t K, int64_t minlen, int64_t outs) {
    // aim for `target` workgroups (2 per CU by default; TTS_HIP_OPT_CONV_SPLIT > 1 sets it)
    const int64_t target = be->conv_split > 1 ? be->conv_split : 512;
    if (!be->conv_split || 2 * tiles >= target) return 1;
    int64_t z = (target + tiles - 1) / tiles;
    const int64_t zk = K / minlen;
    if (z > zk) z = zk;
    const int64_t zm = outs > 0 ? (int64_t)(be->conv_part_doubles / (size_t)outs) : 1;
    if (z > zm) z = zm;
    return z < 2 ? 1 : (int)z;
}

static void launch_split_reduce(tts_hip_backend * be, int nz, int64_t M, int64_t N, float * y, int64_t ldy, const float * bias, int64_t bcs,
                                const float * res, int64_t rcs) {
    const int64_t n = M * N;
    hipLaunchKernelGGL(k_split_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, be->stream, (const double *)be->conv_part, nz, M, N, y, ldy,
                       bias, bcs, res, rcs);
}

// MUL_MAT with an F16 src0 and many src1 columns (the conv_1d GEMM).  Returns false when the
// shapes do not fit the MFMA kernels (the caller then uses the generic path).  Default: the f64
// accumulating kernel (PCM parity); TTS_HIP_OPT_CONV_F32ACC selects the f16 MFMA / f32 accumulator.
bool launch_gemm_f16(tts_hip_backend * be, const tts_tensor * node) {
    const tts_tensor * a = node->src[0];
    const tts_tensor * b = node->src[1];
    if (a->type != TTS_TYPE_F16 || (b->type != TTS_TYPE_F32 && b->type != TTS_TYPE_F16)) return false;
    if (a->ne[2] * a->ne[3] != 1 || b->ne[2] * b->ne[3] != 1 || node->type != TTS_TYPE_F32) return false;
    const int64_t K = a->ne[0], M = a->ne[1], N = b->ne[1];
    const size_t bes = tts_type_size(b->type);
    if (K % 8 || a->nb[0] != 2 || b->nb[0] != bes || node->nb[0] != 4) return false;
    if (a->nb[1] % 16 || b->nb[1] % 16 || ((uintptr_t)a->data % 16) || ((uintptr_t)b->data % 16)) return false;
    dim3 grid((unsigned)((M + 63) / 64), (unsigned)((N + 63) / 64));
    if (!be->conv_f32acc) {
        // short sequences: split K over extra workgroups (f64 partials, summed in split order)
        const int nz = split_count(be, (int64_t)grid.x * grid.y, K, 256, M * N);
        const int64_t kps = nz > 1 ? (((K + nz - 1) / nz + 31) & ~(int64_t)31) : K;
        const int nzr = nz > 1 ? (int)((K + kps - 1) / kps) : 1;
        double * part = nzr > 1 ? be->conv_part : nullptr;
        grid.z = (unsigned)nzr;
        if (b->type == TTS_TYPE_F16)
            hipLaunchKernelGGL(k_gemm_f16_f64acc<true>, grid, dim3(256), 0, be->stream, (const __half *)a->data, (int64_t)(a->nb[1] / 2), b->data,
                               (int64_t)(b->nb[1] / 2), (float *)node->data, (int64_t)(node->nb[1] / 4), M, N, K, part, kps);
        else
            hipLaunchKernelGGL(k_gemm_f16_f64acc<false>, grid, dim3(256), 0, be->stream, (const __half *)a->data, (int64_t)(a->nb[1] / 2), b->data,
                               (int64_t)(b->nb[1] / 4), (float *)node->data, (int64_t)(node->nb[1] / 4), M, N, K, part, kps);
        TTS_HIP_CHECK(hipGetLastError());
        if (part) launch_split_reduce(be, nzr, M, N, (float *)node->data, (int64_t)(node->nb[1] / 4), nullptr, 0, nullptr, 0);
        return true;
    }
    if (b->type == TTS_TYPE_F16)
        hipLaunchKernelGGL(k_gemm_f16_mfma<true>, grid, dim3(256), 0, be->stream, (const __half *)a->data, (int64_t)(a->nb[1] / 2), b->data,
                           (int64_t)(b->nb[1] / 2), (float *)node->data, (int64_t)(node->nb[1] / 4), M, N, K);
    else
        hipLaunchKernelGGL(k_gemm_f16_mfma<false>, grid, dim3(256), 0, be->stream, (const __half *)a->data, (int64_t)(a->nb[1] / 2), b->data,
                           (int64_t)(b->nb[1] / 4), (float *)node->data, (int64_t)(node->nb[1] / 4), M, N, K);
    TTS_HIP_CHECK(hipGetLastError());
    return true;
}

// ------------------------------------------------------------------------------------------
// conv_1d as an implicit GEMM (ggml_conv_1d = IM2COL(F16) -> MUL_MAT, general_neural_audio_codec
// / Kokoro convs) with the conv's bias and residual ADDs as the epilogue; the im2col matrix is
// never written.  Values are the ones the node chain sees: x and the kernel are rounded to f16
// (im2col's dst type, MUL_MAT's vec_dot_type), products f16 x f16 are exact in f64 and summed
// in f64 on the matrix cores (as k_gemm_f16_f64acc), the sum rounds to f32, then + bias (f32),
// then + residual (f32) -- the same roundings as the three nodes.
// Workgroup tile: 64 output channels (MFMA rows) x 64 output positions (MFMA columns, so 16
// lanes store 16 consecutive positions); 4 waves of 32 x 32.  The reduction r = ic*K + k walks
// input channels in chunks of `icc`: per chunk the x window (positions ol0*s - p ..
// + 63*s + (K-1)*d, icc channels) and the kernel slice (64 channels x icc*K taps) are staged in
// LDS as f16-rounded floats; a per-r offset table maps r to its x-window slot (r >= R points at
// a zero slot) so the MFMA loop does no division.
// H32: the f16 matrix cores instead (v_mfma_f32_16x16x32_f16, 32x the f64 MFMA's K per cycle): each
// 32-wide reduction batch is one MFMA into a zeroed f32 accumulator -- its products are exact and
// only the 32-term sum rounds -- and the batch result is added to the f64 accumulator, so the
// rounding stays per 32 terms instead of compounding over the whole K (TTS_HIP_OPT_CONV_F32ACC 2).
typedef _Float16 h16x8_t __attribute__((ext_vector_type(8)));
template <bool W16, bool BIAS, bool RES, bool H32 = false>
__global__ __launch_bounds__(256) void k_conv1d_f64(Conv1dArgs a) {
    extern __shared__ float sm[];
    __shared__ int xoff[CONV1D_MAX_R];  // r -> x-window slot (ic*xw + k*d), zero slot past R
    __shared__ int wofs[CONV1D_MAX_R];  // r -> kernel element offset (k*wk + ic*wic), -1 past R
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c16 = lane & 15, kq = lane >> 4;
    const int64_t ol0 = (int64_t)blockIdx.x * 64;
    const int oc0 = blockIdx.y * 64;
    const int K = a.K, s = a.s, icc = a.icc, xw = a.xw, rs = a.rs;
    const int R = icc * K, Rp = (R + 31) & ~31;  // reduction padded to whole MFMA batches
    float * xs = sm;                 // [icc][xw] + 1 zero slot
    float * ws = sm + icc * xw + 1;  // [64 oc][rs]
    const int zslot = icc * xw;
    for (int r = threadIdx.x; r < Rp; r += 256) {
        const int ic = r / K, k = r - ic * K;
        xoff[r] = r < R ? ic * xw + k * a.d : zslot;
        wofs[r] = r < R ? (int)(k * a.wk + ic * a.wic) : -1;
    }
    if (threadIdx.x == 0) xs[zslot] = 0.f;
    __syncthreads();
    const int wr0 = (wave >> 1) * 32, wc0 = (wave & 1) * 32;  // wave's oc / ol offsets in the tile
    const bool wave_live = oc0 + wr0 < a.OC && ol0 + wc0 < a.OL;  // wave-uniform
    f64x4_t acc[2][2] = {};
    const int64_t base = ol0 * s - a.p;
    // Staging: thread t owns x-window elements e = t + 256u (u < CONV1D_XN) and kernel-slice
    // elements t + 256u (u < CONV1D_WN); their byte offsets relative to the chunk's first channel
    // are fixed for the whole kernel and computed once.  Loads go through buffer descriptors (an
    // out-of-range offset -- padding, the channel tail -- reads 0) into registers one chunk
    // ahead, so the next chunk's loads are in flight while the current one computes.
    const int EX = icc * xw, EW = 64 * Rp;
    constexpr int esz = W16 ? 2 : 4;
    const uint32_t OOB = 0x80000000u;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(a.x.data, 0, a.x_bytes, 0x00020000);
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.w), 0, a.w_bytes, 0x00020000);
    uint32_t xrel[CONV1D_XN], wrel[CONV1D_WN];
    int xic[CONV1D_XN], wic[CONV1D_WN];  // channel within the chunk (for the tail chunk), -1 = unused
#pragma unroll
    for (int u = 0; u < CONV1D_XN; ++u) {
        const int e = (int)threadIdx.x + 256 * u;
        const int ic = e / xw, q = e - ic * xw;
        const int64_t pos = base + q;
        const bool ok = e < EX && pos >= 0 && pos < a.L;
        xrel[u] = ok ? (uint32_t)(pos * a.x.nb[0] + (int64_t)ic * a.x.nb[1]) : OOB;
        xic[u] = e < EX ? ic : -1;
    }
#pragma unroll
    for (int u = 0; u < CONV1D_WN; ++u) {
        const int e = (int)threadIdx.x + 256 * u;
        const int oc = e / Rp, r = e - oc * Rp;
        const int wo = e < EW ? wofs[r] : -1;
        const bool ok = wo >= 0 && oc0 + oc < a.OC;
        wrel[u] = ok ? (uint32_t)(((int64_t)(oc0 + oc) * a.woc + wo) * esz) : OOB;
        wic[u] = e < EW ? (r < R ? r / K : icc) : -1;
    }
    float xv[CONV1D_XN], wv[CONV1D_WN];
    auto fetch = [&](int ic0) {
        const int nic = min(icc, (int)(a.IC - ic0));
        const uint32_t xc = (uint32_t)((int64_t)ic0 * a.x.nb[1]);
        const uint32_t wc = (uint32_t)((int64_t)ic0 * a.wic * esz);
#pragma unroll
        for (int u = 0; u < CONV1D_XN; ++u) {
            const uint32_t off = (xrel[u] == OOB || xic[u] >= nic) ? OOB : xrel[u] + xc;
            xv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
        }
#pragma unroll
        for (int u = 0; u < CONV1D_WN; ++u) {
            const uint32_t off = (wrel[u] == OOB || wic[u] >= nic) ? OOB : wrel[u] + wc;
            if (W16) wv[u] = __half2float(__builtin_bit_cast(__half, __builtin_amdgcn_raw_buffer_load_b16(wr, off, 0, 0)));
            else wv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, off, 0, 0));
        }
    };
    // split launch: this workgroup's input channels [ic_lo, ic_hi), whole chunks
    const int ic_lo = a.part ? (int)blockIdx.z * a.ic_per_split : 0;
    const int ic_hi = a.part ? (int)min((int64_t)(ic_lo + a.ic_per_split), a.IC) : (int)a.IC;
    fetch(ic_lo);
    for (int ic0 = ic_lo; ic0 < ic_hi; ic0 += icc) {
        // f16 rounding (im2col's dst type / MUL_MAT's vec_dot_type) on the way into LDS
#pragma unroll
        for (int u = 0; u < CONV1D_XN; ++u)
            if (xic[u] >= 0) xs[(int)threadIdx.x + 256 * u] = __half2float(__float2half_rn(xv[u]));
#pragma unroll
        for (int u = 0; u < CONV1D_WN; ++u)
            if (wic[u] >= 0) {
                const int e = (int)threadIdx.x + 256 * u;
                const int oc = e / Rp;
                ws[oc * rs + (e - oc * Rp)] = W16 ? wv[u] : __half2float(__float2half_rn(wv[u]));
            }
        __syncthreads();
        if (ic0 + icc < ic_hi) fetch(ic0 + icc);
        // a wave whose 32 x 32 sub-tile lies wholly past the last output channel or position (OC = 96
        // or OC = 1 tiles, short sequences) only stages operands: its MFMAs would feed no store
        if (!wave_live) {
            __syncthreads();
            continue;
        }
        // batches of 8 reduction quads: every operand of the batch is read from LDS first (the
        // offset-table reads, then the dependent operand reads, all independent of each other),
        // then 32 MFMAs issue back to back
        if (H32) {
            for (int r0 = 0; r0 < Rp; r0 += 32) {
                // lane (c16, kq) holds A[row c16][r0 + 8kq + j] and B[r0 + 8kq + j][col c16], j = 0..7
                int xo[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) xo[u] = xoff[r0 + 8 * kq + u];
                h16x8_t A[2], B[2];
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const bool z = xo[u] == zslot;
                        A[t][u] = (_Float16)ws[(wr0 + 16 * t + c16) * rs + r0 + 8 * kq + u];  // f16-rounded: exact
                        B[t][u] = (_Float16)xs[z ? zslot : xo[u] + (wc0 + 16 * t + c16) * s];
                    }
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int tj = 0; tj < 2; ++tj) {
                        const f32x4 pr = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[ti], B[tj], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
                        for (int e = 0; e < 4; ++e) acc[ti][tj][e] += (double)pr[e];
                    }
            }
        } else
        for (int r0 = 0; r0 < Rp; r0 += 32) {
            int xo[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) xo[u] = xoff[r0 + 4 * u + kq];
            float af[8][2], bf[8][2];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int r = r0 + 4 * u + kq;
                const bool z = xo[u] == zslot;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    af[u][t] = ws[(wr0 + 16 * t + c16) * rs + r];
                    bf[u][t] = xs[z ? zslot : xo[u] + (wc0 + 16 * t + c16) * s];
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int tj = 0; tj < 2; ++tj)
                        acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)af[u][ti], (double)bf[u][tj], acc[ti][tj], 0, 0, 0);
        }
        __syncthreads();
    }
    if (a.part) {  // partial sums of this split, no epilogue (k_split_reduce adds bias and residual)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
            const int64_t ol = ol0 + wc0 + 16 * tj + c16;
            if (ol >= a.OL) continue;
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int oc = oc0 + wr0 + 16 * ti + (H32 ? 4 * kq + e : kq + 4 * e);
                    if (oc < a.OC) a.part[((int64_t)blockIdx.z * a.OC + oc) * a.OL + ol] = acc[ti][tj][e];
                }
        }
        return;
    }
    // epilogue: bias and residual operands fetched for all 32 outputs first (clamped, branchless)
    float bv[2][4], rv[2][2][4];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            // accumulator row of register e: f64 MFMA (lane >> 4) + 4e, f32 MFMA 4 (lane >> 4) + e
            const int oc = min(oc0 + wr0 + 16 * ti + (H32 ? 4 * kq + e : kq + 4 * e), (int)a.OC - 1);
            bv[ti][e] = BIAS ? a.bias[(int64_t)oc * a.bcs] : 0.f;
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) {
                const int64_t ol = min(ol0 + wc0 + 16 * tj + c16, a.OL - 1);
                rv[tj][ti][e] = RES ? a.res[ol + (int64_t)oc * a.rcs] : 0.f;
            }
        }
#pragma unroll
    for (int tj = 0; tj < 2; ++tj) {
        const int64_t ol = ol0 + wc0 + 16 * tj + c16;
        if (ol >= a.OL) continue;
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int oc = oc0 + wr0 + 16 * ti + (H32 ? 4 * kq + e : kq + 4 * e);
                if (oc >= a.OC) continue;
                float v = (float)acc[ti][tj][e];
                if (BIAS) v = v + bv[ti][e];
                if (RES) v = rv[tj][ti][e] + v;
                a.y[ol + (int64_t)oc * a.ycs] = v;
            }
    }
}

bool conv1d_fused_ok(int64_t IC, int K, int s, int d, size_t * lds) {
    if (K < 1 || K > 64 || s < 1 || d < 1 || IC < 1) return false;
    const int xw = 63 * s + (K - 1) * d + 1;
    const int icc = conv1d_icc(IC, K, xw);
    if (icc < 1) return false;
    const int rs = ((icc * K + 31) & ~31) + 1;
    const size_t bytes = ((size_t)icc * xw + 1 + 64 * (size_t)rs) * 4;
    if (lds) *lds = bytes;
    return bytes <= 64 * 1024;
}

void launch_conv1d_fused(tts_hip_backend * be, Conv1dArgs a) {
    a.xw = 63 * a.s + (a.K - 1) * a.d + 1;
    a.icc = conv1d_icc(a.IC, a.K, a.xw);
    a.rs = ((a.icc * a.K + 31) & ~31) + 1;
    size_t lds = 0;
    if (!conv1d_fused_ok(a.IC, a.K, a.s, a.d, &lds)) {
        fprintf(stderr, "tts_hip: conv1d_fused shape unsupported\n");
        abort();
    }
    dim3 grid((unsigned)((a.OL + 63) / 64), (unsigned)((a.OC + 63) / 64));
    // short sequences: split the input channels over extra workgroups (whole chunks per split)
    Conv1dArgs e = a;  // the epilogue's operands, applied by the split reduction
    const int64_t nchunk = (a.IC + a.icc - 1) / a.icc;
    const int nz = be->conv_acc_mode == 2 ? 1 : split_count(be, (int64_t)grid.x * grid.y, nchunk, 2, a.OL * a.OC);
    if (nz > 1) {
        a.ic_per_split = (int)(((nchunk + nz - 1) / nz) * a.icc);
        grid.z = (unsigned)((a.IC + a.ic_per_split - 1) / a.ic_per_split);
        a.part = be->conv_part;
        a.bias = nullptr;
        a.res = nullptr;
    }
    const int sel = (a.w16 ? 4 : 0) | (a.bias ? 2 : 0) | (a.res ? 1 : 0);
    if (be->conv_acc_mode == 2) switch (sel) {
        case 0: hipLaunchKernelGGL((k_conv1d_f64<false, false, false, true>), grid, dim3(256), lds, be->stream, a); break;
        case 1: hipLaunchKernelGGL((k_conv1d_f64<false, false, true, true>), grid, dim3(256), lds, be->stream, a); break;
        case 2: hipLaunchKernelGGL((k_conv1d_f64<false, true, false, true>), grid, dim3(256), lds, be->stream, a); break;
        case 3: hipLaunchKernelGGL((k_conv1d_f64<false, true, true, true>), grid, dim3(256), lds, be->stream, a); break;
        case 4: hipLaunchKernelGGL((k_conv1d_f64<true, false, false, true>), grid, dim3(256), lds, be->stream, a); break;
        case 5: hipLaunchKernelGGL((k_conv1d_f64<true, false, true, true>), grid, dim3(256), lds, be->stream, a); break;
        case 6: hipLaunchKernelGGL((k_conv1d_f64<true, true, false, true>), grid, dim3(256), lds, be->stream, a); break;
        default: hipLaunchKernelGGL((k_conv1d_f64<true, true, true, true>), grid, dim3(256), lds, be->stream, a); break;
    }
    else switch (sel) {
        case 0: hipLaunchKernelGGL((k_conv1d_f64<false, false, false>), grid, dim3(256), lds, be->stream, a); break;
        case 1: hipLaunchKernelGGL((k_conv1d_f64<false, false, true>), grid, dim3(256), lds, be->stream, a); break;
        case 2: hipLaunchKernelGGL((k_conv1d_f64<false, true, false>), grid, dim3(256), lds, be->stream, a); break;
        case 3: hipLaunchKernelGGL((k_conv1d_f64<false, true, true>), grid, dim3(256), lds, be->stream, a); break;
        case 4: hipLaunchKernelGGL((k_conv1d_f64<true, false, false>), grid, dim3(256), lds, be->stream, a); break;
        case 5: hipLaunchKernelGGL((k_conv1d_f64<true, false, true>), grid, dim3(256), lds, be->stream, a); break;
        case 6: hipLaunchKernelGGL((k_conv1d_f64<true, true, false>), grid, dim3(256), lds, be->stream, a); break;
        default: hipLaunchKernelGGL((k_conv1d_f64<true, true, true>), grid, dim3(256), lds, be->stream, a); break;
    }
    TTS_HIP_CHECK(hipGetLastError());
    if (a.part) launch_split_reduce(be, (int)grid.z, a.OL, a.OC, e.y, e.ycs, e.bias, e.bcs, e.res, e.rcs);
    if (a.copy_dst)  // the output aliased the input: the kernel wrote a staging buffer
        launch_copy_bytes(be, a.copy_dst, a.y, (size_t)a.OL * (size_t)a.OC * 4);
}

// ------------------------------------------------------------------------------------------
// y[oc][o] = sum over (k, i) with o = i*s - p + k*d, ic in oc's group: x[i][ic] * w[k][oc%OCg][ic]
// One output position per lane; for d = 1 only taps k = r + j*s (r = (o+p) mod s) land on o.
__global__ __launch_bounds__(256) void k_conv_transpose_1d(TD y, TD x, TD w, int s, int p, int d, int g) {
    const int64_t OL = y.ne[0];
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int oc = blockIdx.y;
    if (o >= OL) return;
    const int K = (int)w.ne[0], OCg = (int)w.ne[1];
    const int64_t L = x.ne[0];
    const int IC = (int)x.ne[1], ICg = IC / g;
    const int grp = oc / OCg, ocl = oc % OCg;
    double acc = 0.0;  // f32 x f32 products are exact in f64; same (k, ic) order as the oracle
    const int64_t num0 = o + p;
    for (int k = (d == 1 ? (int)(num0 % s) : 0); k < K; k += (d == 1 ? s : 1)) {
        const int64_t num = num0 - (int64_t)k * d;
        if (num < 0) break;  // d == 1: num only decreases as k grows
        if (num % s) continue;
        const int64_t i = num / s;
        if (i >= L) continue;
        const char * xp = x.data + i * x.nb[0] + (int64_t)grp * ICg * x.nb[1];
        const char * wp = w.data + (int64_t)k * w.nb[0] + (int64_t)ocl * w.nb[1] + (int64_t)grp * ICg * w.nb[2];
        if (w.type == TTS_TYPE_F16) {  // input rounded to f16 (upstream conv_transpose_1d_f16_f32)
            for (int icl = 0; icl < ICg; ++icl)
                acc = __fma_rn((double)__half2float(__float2half_rn(*(const float *)(xp + icl * x.nb[1]))),
                               (double)__half2float(*(const __half *)(wp + icl * w.nb[2])), acc);
        } else {
            for (int icl = 0; icl < ICg; ++icl)
                acc = __fma_rn((double)*(const float *)(xp + icl * x.nb[1]), (double)*(const float *)(wp + icl * w.nb[2]), acc);
        }
    }
    *(float *)(y.data + o * y.nb[0] + (int64_t)oc * y.nb[1]) = (float)acc;
}

// Polyphase form on the f64 matrix cores (dilation 1, groups 1): outputs o = q*s + rr - p of one
// residue rr receive taps k = rr + s*j only, so per residue
//   y[oc][q*s + rr - p] = sum_{j, ic} w[k = rr + s*j][oc][ic] * x[q - j][ic]
// is a GEMM (rows oc, columns q, K = J*IC).  One wave per 16 (oc) x 16 (q) tile of one residue,
// v_mfma_f64_16x16x4_f64 (A[oc = l&15][kk], B[kk][q = l&15], kk = 4 consecutive ic per step):
// f32 x f32 products are exact in f64, so only the order of the f64 sum differs from the oracle.
__global__ __launch_bounds__(64) void k_conv_transpose_1d_mfma(TD y, TD x, TD w, int s, int p) {
    const int lane = threadIdx.x, r16 = lane & 15, kq = lane >> 4;
    const int rr = blockIdx.z;
    const int64_t q0 = (int64_t)blockIdx.x * 16;
    const int oc0 = blockIdx.y * 16;
    const int K = (int)w.ne[0], OC = (int)w.ne[1], IC = (int)w.ne[2];
    const int64_t L = x.ne[0], OL = y.ne[0];
    const int J = (K - rr + s - 1) / s;
    const int oca = min(oc0 + r16, OC - 1);
    const int64_t qb = q0 + r16;
    f64x4_t acc = {};
    for (int j = 0; j < J; ++j) {
        const int k = rr + s * j;
        const int64_t i = qb - j;
        const bool iin = i >= 0 && i < L;
        const char * wp = w.data + (int64_t)k * w.nb[0] + (int64_t)oca * w.nb[1];
        const char * xp = x.data + (iin ? i : 0) * x.nb[0];
        for (int ic0 = 0; ic0 < IC; ic0 += 16) {
            double av[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int ic = ic0 + 4 * u + kq;
                const int icc = min(ic, IC - 1);
                const bool w16 = w.type == TTS_TYPE_F16;
                const float wa = w16 ? __half2float(*(const __half *)(wp + (int64_t)icc * w.nb[2])) : *(const float *)(wp + (int64_t)icc * w.nb[2]);
                float xb = *(const float *)(xp + (int64_t)icc * x.nb[1]);
                if (w16) xb = __half2float(__float2half_rn(xb));
                av[u] = ic < IC ? (double)wa : 0.0;
                bv[u] = (ic < IC && iin) ? (double)xb : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
        }
    }
    const int64_t o = qb * s + rr - p;
    if (o < 0 || o >= OL) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int oc = oc0 + kq + 4 * e;
        if (oc < OC) *(float *)(y.data + o * y.nb[0] + (int64_t)oc * y.nb[1]) = (float)acc[e];
    }
}

// Polyphase conv_transpose_1d on the f64 matrix cores with LDS-staged operands.  A workgroup owns
// 32 output channels x 64 polyphase positions q (all S residues: outputs o = q*S + rr - p), and
// walks the input channels in chunks of 16: the x slice (positions q0 - J + 1 .. q0 + 63) and the
// weight slice (every tap k, 32 channels; contiguous K*32 floats per input channel in ggml's
// [K][OC][IC] layout) are staged in LDS with coalesced loads, then each wave (16 positions) runs
// v_mfma_f64_16x16x4_f64 over (ic quad, tap j, residue, channel half): one x operand feeds 2*S
// products.  f32 x f32 products are exact in f64; only the f64 summation order differs from the
// oracle (tests: rel 1e-5 per layer, PCM 1e-4 end to end).
template <int S, bool W16>
__global__ __launch_bounds__(256) void k_convt_f64_lds(TD y, TD x, TD w, int p, double * __restrict__ part = nullptr, int icps = 0) {
    constexpr int JM = 2, K = 2 * S;  // DAC / SNAC / Kokoro upsamplers: kernel = 2 * stride
    constexpr int QT = 64, OCT = 32, ICC = 16, XW = QT + JM - 1;
    constexpr int NX = ICC * XW, NW4 = ICC * K * OCT / 4;
    constexpr int XR = (NX + 255) / 256, WR = (NW4 + 255) / 256;
    // Padded LDS strides (ds_read_b32 / ds_write_b32 bank = dword index mod 32, per 32-lane half):
    //  - reads of one MFMA step: lanes (kq, c16) of a half take two consecutive input channels, so the
    //    x row stride XWP and the weight channel stride WIC are = 16 mod 32 (the two 16-lane groups on
    //    opposite bank halves);
    //  - the weight stage: a half's 32 lanes hold 4 taps of (channel oc, tap group kg); with a tap
    //    stride WK, 4 * WK = 32 / (K / 4) mod 32 spreads the tap groups over disjoint bank ranges
    //    (S = 8: 34, S = 4: 36; S = 2 has one group).  Unpadded, these were 2- to 4-way conflicts
    //    (5.3 per LDS instruction measured on S = 8).  Same values, same MFMA order: bit-identical.
    constexpr int XWP = 80;
    constexpr int WK = S == 8 ? 34 : S == 4 ? 36 : OCT + 1;
    constexpr int WIC0 = K * WK, WIC = WIC0 + ((16 - WIC0 % 32) + 32) % 32;
    __shared__ float xs[ICC][XWP];
    __shared__ float ws[ICC * WIC];  // [ic][k][oc] at ic * WIC + k * WK + oc
    const int lane = threadIdx.x & 63, qw = threadIdx.x >> 6;
    const int c16 = lane & 15, kq = lane >> 4;
    const int OC = (int)w.ne[1], IC = (int)w.ne[2];
    const int64_t L = x.ne[0], OL = y.ne[0];
    const int64_t q0 = (int64_t)blockIdx.x * QT;
    const int oc0 = blockIdx.y * OCT;
    f64x4_t acc[S][2];
#pragma unroll
    for (int r = 0; r < S; ++r) acc[r][0] = acc[r][1] = (f64x4_t){0.0, 0.0, 0.0, 0.0};
    // next chunk's operands are fetched into registers while the current one computes
    float xr[XR];
    float4 wr[WR];
    auto fetch = [&](int ic0) {
#pragma unroll
        for (int u = 0; u < XR; ++u) {
            const int t = threadIdx.x + 256 * u;
            const int ic = t / XW, qq = t - ic * XW;
            const int64_t pos = q0 - (JM - 1) + qq;
            const bool ok = t < NX && pos >= 0 && pos < L && ic0 + ic < IC;
            xr[u] = ok ? *(const float *)(x.data + pos * x.nb[0] + (int64_t)(ic0 + ic) * x.nb[1]) : 0.f;
            if (W16) xr[u] = __half2float(__float2half_rn(xr[u]));  // F16 kernel: the input rounded to f16
        }
#pragma unroll
        for (int u = 0; u < WR; ++u) {
            const int t = threadIdx.x + 256 * u;       // float4 index within [ic][oc][k] (global order)
            const int ic = t / (K * OCT / 4), rem = (t - ic * (K * OCT / 4)) * 4;
            const int oc = rem / K;
            const bool ok = t < NW4 && oc0 + oc < OC && ic0 + ic < IC;
            const char * src = w.data + (int64_t)(oc0 + oc) * w.nb[1] + (int64_t)(ic0 + ic) * w.nb[2] + (rem - oc * K) * (W16 ? 2 : 4);
            if (W16) {  // 4 taps = 8 B (K % 4 == 0 and 8-B aligned rows, host-checked)
                const uint2 h = ok ? *(const uint2 *)src : make_uint2(0u, 0u);
                wr[u] = make_float4(__half2float(__ushort_as_half((unsigned short)(h.x & 0xFFFF))), __half2float(__ushort_as_half((unsigned short)(h.x >> 16))),
                                    __half2float(__ushort_as_half((unsigned short)(h.y & 0xFFFF))), __half2float(__ushort_as_half((unsigned short)(h.y >> 16))));
            } else {
                wr[u] = ok ? *(const float4 *)src : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    auto stage = [&]() {
#pragma unroll
        for (int u = 0; u < XR; ++u) {
            const int t = threadIdx.x + 256 * u;
            if (t < NX) xs[t / XW][t % XW] = xr[u];
        }
#pragma unroll
        for (int u = 0; u < WR; ++u) {
            const int t = threadIdx.x + 256 * u;
            if (t >= NW4) continue;
            const int ic = t / (K * OCT / 4), rem = (t - ic * (K * OCT / 4)) * 4;
            const int oc = rem / K, k = rem - oc * K;  // 4 consecutive taps k..k+3 of channel oc
            float * o = ws + ic * WIC + k * WK + oc;
            o[0] = wr[u].x, o[WK] = wr[u].y, o[2 * WK] = wr[u].z, o[3 * WK] = wr[u].w;
        }
    };
    // split launch: input channels [ic_lo, ic_hi) (whole chunks), f64 partials to part[z][oc][o]
    const int ic_lo = part ? (int)blockIdx.z * icps : 0;
    const int ic_hi = part ? min(IC, ic_lo + icps) : IC;
    fetch(ic_lo);
    for (int ic0 = ic_lo; ic0 < ic_hi; ic0 += ICC) {
        stage();
        __syncthreads();
        if (ic0 + ICC < ic_hi) fetch(ic0 + ICC);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int icl = 4 * kk + kq;
            // every operand of this ic quad read from LDS first, then the MFMAs back to back
            float bx[JM], aw[JM][S][2];
#pragma unroll
            for (int j = 0; j < JM; ++j) {
                bx[j] = xs[icl][qw * 16 + c16 + (JM - 1) - j];
#pragma unroll
                for (int r = 0; r < S; ++r)
#pragma unroll
                    for (int h = 0; h < 2; ++h) aw[j][r][h] = ws[icl * WIC + (r + S * j) * WK + h * 16 + c16];
            }
#pragma unroll
            for (int j = 0; j < JM; ++j) {
                const double bv = (double)bx[j];
#pragma unroll
                for (int r = 0; r < S; ++r)
#pragma unroll
                    for (int h = 0; h < 2; ++h) acc[r][h] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)aw[j][r][h], bv, acc[r][h], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    const int64_t q = q0 + qw * 16 + c16;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const int64_t o = q * S + r - p;
        if (o < 0 || o >= OL) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int oc = oc0 + h * 16 + kq + 4 * e;
                if (oc >= OC) continue;
                if (part) part[((int64_t)blockIdx.z * OC + oc) * OL + o] = acc[r][h][e];
                else *(float *)(y.data + o * y.nb[0] + (int64_t)oc * y.nb[1]) = (float)acc[r][h][e];
            }
    }
}

void launch_conv_transpose_1d(tts_hip_backend * be, const tts_tensor * node) {
    const tts_tensor * w = node->src[0];
    const tts_tensor * x = node->src[1];
    const int s = node->op_params[0], p = node->op_params[1], d = node->op_params[2], g = node->op_params[4];
    // the LDS kernel reads whole 4-tap rows of the weight: contiguous taps, 16-B (F16: 8-B) aligned rows
    const bool w16 = w->type == TTS_TYPE_F16;
    const size_t wal = w16 ? 8 : 16;
    const bool wvec = w->nb[0] == (w16 ? 2u : 4u) && w->nb[1] % wal == 0 && w->nb[2] % wal == 0 && ((uintptr_t)w->data % 16) == 0;
    if (d == 1 && g == 1 && w->ne[1] >= 16 && x->ne[1] >= 16 && (s == 2 || s == 4 || s == 6 || s == 8 || s == 10) && w->ne[0] == 2 * s && wvec &&
        be->convt_lds && node->nb[0] == 4) {
        const int64_t nq = (node->ne[0] + p) / s + 1;
        dim3 grid((unsigned)((nq + 63) / 64), (unsigned)((w->ne[1] + 31) / 32));
        const TD Y = make_td(node), X = make_td(x), W = make_td(w);
        // short sequences: split the input channels (chunks of 16) over extra workgroups
        const int64_t IC = x->ne[1], OL = node->ne[0], OC = node->ne[1];
        const int64_t nchunk = (IC + 15) / 16;
        const int nz = split_count(be, (int64_t)grid.x * grid.y, nchunk, 2, OL * OC);
        const int icps = nz > 1 ? (int)(((nchunk + nz - 1) / nz) * 16) : 0;
        double * part = nz > 1 ? be->conv_part : nullptr;
        grid.z = nz > 1 ? (unsigned)((IC + icps - 1) / icps) : 1u;
#define TTS_CONVT_LDS(SS)                                                                                       \
    do {                                                                                                        \
        if (w16) hipLaunchKernelGGL((k_convt_f64_lds<SS, true>), grid, dim3(256), 0, be->stream, Y, X, W, p, part, icps);  \
        else hipLaunchKernelGGL((k_convt_f64_lds<SS, false>), grid, dim3(256), 0, be->stream, Y, X, W, p, part, icps);     \
    } while (0)
        if (s == 2) TTS_CONVT_LDS(2);
        else if (s == 4) TTS_CONVT_LDS(4);
        else if (s == 6) TTS_CONVT_LDS(6);
        else if (s == 8) TTS_CONVT_LDS(8);
        else TTS_CONVT_LDS(10);
#undef TTS_CONVT_LDS
        TTS_HIP_CHECK(hipGetLastError());
        if (part) launch_split_reduce(be, (int)grid.z, OL, OC, (float *)node->data, (int64_t)(node->nb[1] / 4), nullptr, 0, nullptr, 0);
        return;
    }
    if (d == 1 && g == 1 && w->ne[1] >= 16 && x->ne[1] >= 16) {
        const int64_t nq = (node->ne[0] + p) / s + 1;  // q with q*s + rr - p < OL for some rr
        const dim3 grid((unsigned)((nq + 15) / 16), (unsigned)((w->ne[1] + 15) / 16), (unsigned)s);
        hipLaunchKernelGGL(k_conv_transpose_1d_mfma, grid, dim3(64), 0, be->stream, make_td(node), make_td(x), make_td(w), s, p);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    const dim3 grid((unsigned)((node->ne[0] + 255) / 256), (unsigned)node->ne[1]);
    hipLaunchKernelGGL(k_conv_transpose_1d, grid, dim3(256), 0, be->stream, make_td(node), make_td(x), make_td(w), node->op_params[0],
                       node->op_params[1], node->op_params[2], node->op_params[4]);
    TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
