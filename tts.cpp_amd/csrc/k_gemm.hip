// F32 x F32 GEMM with ggml's float dot semantics: y(row, col) = sum_k (double)(w[row][k] * x[col][k])
// -- every product rounded to f32, the sum carried in f64 and taken in ascending k, rounded to f32
// once (ggml_vec_dot_f32's generic path, oracle/ggml_ref.c).  Used where a float MUL_MAT has more
// columns than the GEMV kernels batch (ALBERT's projections over a prompt, Kokoro's LSTM input
// projections and 1x1 shortcut convs over a duration-expanded sequence, the mask expansions).
//
// Tiles of 64 weight rows x 64 columns per 256-thread workgroup; K in slabs of 16 staged through
// LDS k-major, so a wave's 16 row-lanes read consecutive words.  Each thread owns a 4 x 4 block of
// outputs (rows tm + 16 i, columns tn + 16 j) and walks its K range in ascending order.  Skinny
// products (a 768 x 768 projection over 64 tokens is 12 tiles) split K over extra workgroups to fill
// the chip; their f64 partials are summed in split order by a second pass, so every output is a
// short chain of in-order f64 sums, equal to the oracle's sequential sum up to f64 rounding: the f32
// results agree unless an f64 sum lies within f64 rounding of an f32 rounding boundary.  The loop is VALU-bound (f32 multiply, f32->f64 convert, f64 add per MAC);
// the matrix cores cannot reproduce the per-product f32 rounding.
#include "hip_internal.h"

namespace tts {

namespace {

constexpr int GT = 64;   // tile rows / columns
constexpr int GK = 16;   // K slab
constexpr int GLD = GT + 4;

__device__ __forceinline__ void gemm_store(const GemvJob & j, int mat, int64_t row, int64_t col, double acc) {
    float v = (float)acc;
    if (j.epi == EPI_GELU) {
        if (v <= -10.0f) v = 0.0f;
        else if (v < 10.0f) v = __half2float(__ushort_as_half(j.gelu[__half_as_ushort(__float2half_rn(v))]));
    } else if (j.epi == EPI_ADD) {
        v = __fadd_rn(v, j.res[col * j.rcs + row]);
    }
    j.Y[mat][col * j.ycs[mat] + row * j.yrs[mat]] = v;
}

// ks > 1: blockIdx.z = mat * ks + split, K range [split * kc, (split + 1) * kc), f64 partials to
// part[((mat * ks + split) * M + col) * N + row]
template <bool VEC>
__global__ __launch_bounds__(256) void k_gemm_f32_f64(GemvJob j, int ks, int64_t kc, double * __restrict__ part) {
    __shared__ float As[GK][GLD];
    __shared__ float Bs[GK][GLD];
    const int tid = threadIdx.x;
    const int mat = blockIdx.z / ks, split = blockIdx.z % ks;
    const int64_t row0 = (int64_t)blockIdx.x * GT, col0 = (int64_t)blockIdx.y * GT;
    const int64_t N = j.N, M = j.M;
    const int64_t kbeg = (int64_t)split * kc, K = kbeg + kc < j.K ? kbeg + kc : j.K;
    const float * W = (const float *)j.W[mat];
    const int64_t wrs = j.w_row_bytes / 4;
    const int tm = tid & 15, tn = tid >> 4;
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
    // loader: thread -> (tile row / column lr, k quad kq)
    const int lr = tid >> 2, kq = (tid & 3) * 4;
    const int64_t wr = row0 + lr, xc = col0 + lr;
    const float * wp = W + (wr < N ? wr : N - 1) * wrs;
    const float * xp = j.x + (xc < M ? xc : M - 1) * j.xcs;
    for (int64_t k0 = kbeg; k0 < K; k0 += GK) {
        float wv[4], xv[4];
        const int64_t k = k0 + kq;
        if (VEC && k + 3 < K) {
            const float4 w4 = *(const float4 *)(wp + k), x4 = *(const float4 *)(xp + k);
            wv[0] = w4.x, wv[1] = w4.y, wv[2] = w4.z, wv[3] = w4.w;
            xv[0] = x4.x, xv[1] = x4.y, xv[2] = x4.z, xv[3] = x4.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                wv[e] = k + e < K ? wp[k + e] : 0.0f;
                xv[e] = k + e < K ? xp[k + e] : 0.0f;
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            As[kq + e][lr] = wv[e];
            Bs[kq + e][lr] = xv[e];
        }
        __syncthreads();
        const int kn = K - k0 < GK ? (int)(K - k0) : GK;
        if (kn == GK) {
#pragma unroll 4
            for (int kk = 0; kk < GK; ++kk) {
                float a[4], b[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = As[kk][tm + 16 * i];
#pragma unroll
                for (int i = 0; i < 4; ++i) b[i] = Bs[kk][tn + 16 * i];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[i][c] += (double)__fmul_rn(a[i], b[c]);
            }
        } else {
            for (int kk = 0; kk < kn; ++kk) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[i][c] += (double)__fmul_rn(As[kk][tm + 16 * i], Bs[kk][tn + 16 * c]);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int64_t col = col0 + tn + 16 * c;
        if (col >= M) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t row = row0 + tm + 16 * i;
            if (row >= N) continue;
            if (ks == 1) gemm_store(j, mat, row, col, acc[i][c]);
            else part[((int64_t)blockIdx.z * M + col) * N + row] = acc[i][c];
        }
    }
}

// Many rows x a few dozen columns (the 9 output heads at 32 lock-step prompts: 9 792 rows x 1 024 x 32):
// the 64 x 64 tiles above pad the columns and split K into partial sums; here every (row, column)
// output is ONE sequential f64 chain in ascending k -- exactly ggml_vec_dot_f32's generic order -- and
// every weight byte is read once.  A workgroup owns R = P * RW consecutive flat (matrix, row) rows; lane
// (slot s, column c) of wave w accumulates rows s + RPS * w + RW * p (p < P) in registers.  K runs in
// chunks of KC staged through LDS: the columns k-major, padded (lanes of one k read consecutive words), the
// rows padded by one word (the RPS row slots of a wave read different banks; a row's lanes share one
// broadcast word).  The next chunk is fetched into registers while the current one is summed.
constexpr int WKC = 64;
template <int MC, int P>
__global__ __launch_bounds__(256) void k_gemv_f32_wide(GemvJob j, int64_t rows_total) {
    constexpr int RPS = 64 / MC, RW = 4 * RPS, R = RW * P;
    constexpr int XN = WKC * MC, WN = R * WKC;                  // floats staged per chunk
    constexpr int XL = (XN + 255) / 256, WL = (WN + 255) / 256;  // per thread
    __shared__ float xs[WKC * (MC + 1)];
    __shared__ float ws[R * (WKC + 1)];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c = lane % MC, s = lane / MC;
    const int64_t r0 = (int64_t)blockIdx.x * R;
    const int64_t K = j.K, M = j.M, N = j.N, wrs = j.w_row_bytes / 4;
    double acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = 0.0;
    float xr[XL], wr[WL];
    auto fetch = [&](int64_t k0) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < XL; ++i) {  // x: element e = col * WKC + kk (coalesced along k)
            const int e = i * 256 + tid, col = e / WKC, kk = e % WKC;
            const int64_t k = k0 + kk;
            xr[i] = (e < XN && col < M && k < K) ? j.x[(int64_t)col * j.xcs + k] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < WL; ++i) {  // w: element e = row * WKC + kk (a row's chunk is contiguous)
            const int e = i * 256 + tid, rr = e / WKC, kk = e % WKC;
            const int64_t fr = r0 + rr, k = k0 + kk;
            float v = 0.0f;
            if (e < WN && fr < rows_total && k < K) {
                const int mat = (int)(fr / N);
                v = ((const float *)j.W[mat])[(fr - (int64_t)mat * N) * wrs + k];
            }
            wr[i] = v;
        }
    };
    fetch(0);
    for (int64_t k0 = 0; k0 < K; k0 += WKC) {
        __syncthreads();  // every lane is done with the previous chunk
#pragma unroll
        for (int i = 0; i < XL; ++i) {
            const int e = i * 256 + tid;
            if (e < XN) xs[(e % WKC) * (MC + 1) + e / WKC] = xr[i];
        }
#pragma unroll
        for (int i = 0; i < WL; ++i) {
            const int e = i * 256 + tid;
            if (e < WN) ws[(e / WKC) * (WKC + 1) + e % WKC] = wr[i];
        }
        __syncthreads();
        if (k0 + WKC < K) fetch(k0 + WKC);
        const int kn = K - k0 < WKC ? (int)(K - k0) : WKC;  // zero-filled tail: the padded terms are never added
        if (kn == WKC) {
#pragma unroll 8
            for (int kk = 0; kk < WKC; ++kk) {
                const float xv = xs[kk * (MC + 1) + c];
#pragma unroll
                for (int p = 0; p < P; ++p) acc[p] += (double)__fmul_rn(ws[(s + RPS * wave + RW * p) * (WKC + 1) + kk], xv);
            }
        } else {
            for (int kk = 0; kk < kn; ++kk) {
                const float xv = xs[kk * (MC + 1) + c];
#pragma unroll
                for (int p = 0; p < P; ++p) acc[p] += (double)__fmul_rn(ws[(s + RPS * wave + RW * p) * (WKC + 1) + kk], xv);
            }
        }
    }
    if (c >= M) return;
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int64_t fr = r0 + s + RPS * wave + RW * p;
        if (fr >= rows_total) continue;
        const int mat = (int)(fr / N);
        gemm_store(j, mat, fr - (int64_t)mat * N, c, acc[p]);
    }
}

// the splits' partials of each output summed in split order, then the f32 rounding and epilogue
__global__ __launch_bounds__(256) void k_gemm_reduce(GemvJob j, int ks, const double * __restrict__ part) {
    const int64_t per = j.M * j.N, n = per * j.nmat;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        const int mat = (int)(e / per);
        const int64_t r = e % per, col = r / j.N, row = r % j.N;
        double a = 0.0;
        for (int s = 0; s < ks; ++s) a += part[((int64_t)(mat * ks + s) * j.M + col) * j.N + row];
        gemm_store(j, mat, row, col, a);
    }
}

// Batched form for ggml's 3-D / 4-D float MUL_MAT (attention over many queries: Dia's 1024-position
// encoder, prompt prefills): dst[i0, i1, i2, i3] = dot(src0[:, i0, i2 / r2, i3 / r3], src1[:, i1, i2, i3]),
// the same f32 products, ascending-k f64 sums and single rounding per output as the 2-D kernel
// (no K split: equal to the oracle's sequential sum up to f64 rounding).  blockIdx.z = i2 + ne2 * i3.
struct BGemm {
    const char *a, *b;
    char * y;
    int64_t K, N, M, ne2, ne3, r2, r3;
    int64_t a1, a2, a3, b1, b2, b3, y0, y1, y2, y3;  // byte strides
};

__global__ __launch_bounds__(256) void k_bgemm_f32(BGemm g) {
    __shared__ float As[GK][GLD];
    __shared__ float Bs[GK][GLD];
    const int tid = threadIdx.x;
    const int64_t i2 = blockIdx.z % g.ne2, i3 = blockIdx.z / g.ne2;
    const int64_t row0 = (int64_t)blockIdx.x * GT, col0 = (int64_t)blockIdx.y * GT;
    const int64_t N = g.N, M = g.M, K = g.K;
    const char * A = g.a + (i2 / g.r2) * g.a2 + (i3 / g.r3) * g.a3;
    const char * B = g.b + i2 * g.b2 + i3 * g.b3;
    const int tm = tid & 15, tn = tid >> 4;
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
    const int lr = tid >> 2, kq = (tid & 3) * 4;
    const int64_t wr = row0 + lr, xc = col0 + lr;
    const float * wp = (const float *)(A + (wr < N ? wr : N - 1) * g.a1);
    const float * xp = (const float *)(B + (xc < M ? xc : M - 1) * g.b1);
    for (int64_t k0 = 0; k0 < K; k0 += GK) {
        const int64_t k = k0 + kq;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            As[kq + e][lr] = k + e < K ? wp[k + e] : 0.0f;
            Bs[kq + e][lr] = k + e < K ? xp[k + e] : 0.0f;
        }
        __syncthreads();
        const int kn = K - k0 < GK ? (int)(K - k0) : GK;
        if (kn == GK) {
#pragma unroll 4
            for (int kk = 0; kk < GK; ++kk) {
                float a[4], b[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = As[kk][tm + 16 * i];
#pragma unroll
                for (int i = 0; i < 4; ++i) b[i] = Bs[kk][tn + 16 * i];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[i][c] += (double)__fmul_rn(a[i], b[c]);
            }
        } else {
            for (int kk = 0; kk < kn; ++kk) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[i][c] += (double)__fmul_rn(As[kk][tm + 16 * i], Bs[kk][tn + 16 * c]);
            }
        }
        __syncthreads();
    }
    char * Y = g.y + i2 * g.y2 + i3 * g.y3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int64_t col = col0 + tn + 16 * c;
        if (col >= M) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t row = row0 + tm + 16 * i;
            if (row < N) *(float *)(Y + row * g.y0 + col * g.y1) = (float)acc[i][c];
        }
    }
}

}  // namespace

// Batched float MUL_MAT on the tiled kernel; false when the node does not fit it (the caller then
// uses the one-wave-per-output kernel).
bool launch_bgemm_f32(tts_hip_backend * be, const tts_tensor * node) {
    const tts_tensor * a = node->src[0];
    const tts_tensor * b = node->src[1];
    if (!be->bgemm_f32 || a->type != TTS_TYPE_F32 || b->type != TTS_TYPE_F32 || node->type != TTS_TYPE_F32) return false;
    if (a->nb[0] != 4 || b->nb[0] != 4 || a->ne[0] < 32 || a->ne[1] < 16 || b->ne[1] < 16) return false;
    if (b->ne[2] % a->ne[2] || b->ne[3] % a->ne[3]) return false;
    if ((a->nb[1] | b->nb[1] | node->nb[1] | node->nb[0]) % 4) return false;
    const int64_t batches = node->ne[2] * node->ne[3];
    if (batches > 65535 || (node->ne[1] + GT - 1) / GT > 65535) return false;
    BGemm g;
    g.a = (const char *)a->data, g.b = (const char *)b->data, g.y = (char *)node->data;
    g.K = a->ne[0], g.N = a->ne[1], g.M = b->ne[1], g.ne2 = node->ne[2], g.ne3 = node->ne[3];
    g.r2 = b->ne[2] / a->ne[2], g.r3 = b->ne[3] / a->ne[3];
    g.a1 = (int64_t)a->nb[1], g.a2 = (int64_t)a->nb[2], g.a3 = (int64_t)a->nb[3];
    g.b1 = (int64_t)b->nb[1], g.b2 = (int64_t)b->nb[2], g.b3 = (int64_t)b->nb[3];
    g.y0 = (int64_t)node->nb[0], g.y1 = (int64_t)node->nb[1], g.y2 = (int64_t)node->nb[2], g.y3 = (int64_t)node->nb[3];
    const dim3 grid((unsigned)((g.N + GT - 1) / GT), (unsigned)((g.M + GT - 1) / GT), (unsigned)batches);
    hipLaunchKernelGGL(k_bgemm_f32, grid, dim3(256), 0, be->stream, g);
    TTS_HIP_CHECK(hipGetLastError());
    return true;
}

bool gemm_f32_ok(const GemvJob & j) {
    // the tiled GEMM stores plain (column, row) targets: no GQA repeat copies, no mixed row counts
    return j.rep_mat < 0 && !j.hetero && j.wtype == TTS_TYPE_F32 && j.x && j.K > 0 && j.N > 0 && j.M > 0 && j.nmat >= 1 && (j.N + GT - 1) / GT <= INT32_MAX &&
           (j.M + GT - 1) / GT <= 65535 && (j.w_row_bytes % 4) == 0 && (j.xcs >= j.K);
}

template <int MC>
static void launch_wide(tts_hip_backend * be, const GemvJob & j, int64_t rows) {
    constexpr int RW = 4 * (64 / MC);
    // rows per lane: as few as keep >= 4 workgroups (16 waves) per CU -- each lane's f64 chains are
    // serial, so the SIMDs need several waves to overlap their latencies
    int64_t p = (rows + 4 * be->cus * RW - 1) / (4 * be->cus * RW);
    const int P = p <= 1 ? 1 : p <= 2 ? 2 : p <= 4 ? 4 : 8;
    const unsigned g = (unsigned)((rows + (int64_t)P * RW - 1) / ((int64_t)P * RW));
    switch (P) {
        case 1: hipLaunchKernelGGL((k_gemv_f32_wide<MC, 1>), dim3(g), dim3(256), 0, be->stream, j, rows); break;
        case 2: hipLaunchKernelGGL((k_gemv_f32_wide<MC, 2>), dim3(g), dim3(256), 0, be->stream, j, rows); break;
        case 4: hipLaunchKernelGGL((k_gemv_f32_wide<MC, 4>), dim3(g), dim3(256), 0, be->stream, j, rows); break;
        default: hipLaunchKernelGGL((k_gemv_f32_wide<MC, 8>), dim3(g), dim3(256), 0, be->stream, j, rows); break;
    }
}

// many rows (>= 2048 flat) x 9..64 columns: the wide GEMV (one sequential f64 chain per output)
static bool wide_ok(const tts_hip_backend * be, const GemvJob & j) {
    const int64_t rows = j.N * j.nmat;
    return be->gemv_f32_wide && j.M > 8 && j.M <= 64 && rows >= 2048 &&
           (j.epi == EPI_NONE || j.epi == EPI_GELU || j.epi == EPI_ADD);
}

void launch_gemm_f32(tts_hip_backend * be, const GemvJob & j) {
    if (wide_ok(be, j)) {
        const int64_t rows = j.N * j.nmat;
        if (j.M <= 16) launch_wide<16>(be, j, rows);
        else if (j.M <= 32) launch_wide<32>(be, j, rows);
        else launch_wide<64>(be, j, rows);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    bool vec = (j.K % 4) == 0 && (j.w_row_bytes % 16) == 0 && (j.xcs % 4) == 0 && ((uintptr_t)j.x % 16) == 0;
    for (int i = 0; i < j.nmat; ++i) vec = vec && ((uintptr_t)j.W[i] % 16) == 0;
    const int64_t tiles = ((j.N + GT - 1) / GT) * ((j.M + GT - 1) / GT) * j.nmat;
    // split K until ~2 workgroups per CU, each split keeping >= 64 of K (whole slabs)
    int ks = 1;
    const int64_t want = 2 * 256;
    while (ks < 64 && tiles * ks * 2 <= want && j.K / (ks * 2) >= 64) ks *= 2;
    const int64_t kc = ks == 1 ? j.K : ((j.K + ks - 1) / ks + GK - 1) / GK * GK;
    if (ks > 1 && (size_t)ks * j.M * j.N * j.nmat > be->conv_part_doubles) ks = 1;
    const dim3 grid((unsigned)((j.N + GT - 1) / GT), (unsigned)((j.M + GT - 1) / GT), (unsigned)(j.nmat * ks));
    const int64_t kcc = ks == 1 ? j.K : kc;
    if (vec) hipLaunchKernelGGL(k_gemm_f32_f64<true>, grid, dim3(256), 0, be->stream, j, ks, kcc, be->conv_part);
    else hipLaunchKernelGGL(k_gemm_f32_f64<false>, grid, dim3(256), 0, be->stream, j, ks, kcc, be->conv_part);
    if (ks > 1) {
        const int64_t n = j.M * j.N * j.nmat;
        int64_t g = (n + 255) / 256;
        if (g > 4096) g = 4096;
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)g), dim3(256), 0, be->stream, j, ks, (const double *)be->conv_part);
    }
    TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
