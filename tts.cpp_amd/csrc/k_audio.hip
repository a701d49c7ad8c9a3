// Fork audio ops of Kokoro's sine source and iSTFTNet head:
//   CUMSUM  (build_sin_gen, src/models/kokoro/model.cpp:175)
//   UPSCALE nearest (ggml_upscale_ext, :177) and linear (fork ggml_upscale_linear, :176)
//   STFT / ISTFT (src/util.cpp:111-130, used by build_generator model.cpp:199 and :241)
// The fork's sources are absent; the semantics are PyTorch's (Kokoro's reference model), restated
// in oracle/ggml_ref.c (op_cumsum, op_upscale, op_stft, op_istft) and pinned there to float32 torch
// fixtures.  These kernels reproduce the oracle's operation order: sequential f64 cumsum, ATen's
// fma-contracted linear interpolation, direct f64 DFTs over a deterministic twiddle table.
//
// All four are tiny next to the generator's convolutions (a few MB, thousands of frames): they are
// latency-bound, so each is one launch with its reuse staged in LDS (cumsum rows, twiddles, the
// per-tile complex spectrum of iSTFT), not a GEMM.
#include "hip_internal.h"

namespace tts {

// ---- CUMSUM along ne0 -------------------------------------------------------------------------
// One workgroup per row.  The row streams through LDS in chunks (coalesced loads / stores by all
// lanes); lane 0 walks each chunk with the running f64 sum -- torch's CPU accumulator and the
// oracle's order -- so the only serial work is one dependent f64 add per element.
constexpr int CUMSUM_CHUNK = 4096;

__global__ __launch_bounds__(256) void k_cumsum(TD dst, TD a) {
    __shared__ float buf[CUMSUM_CHUNK];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % dst.ne[1], i2 = (r / dst.ne[1]) % dst.ne[2], i3 = r / (dst.ne[1] * dst.ne[2]);
    const int64_t n = dst.ne[0];
    double s = 0.0;
    for (int64_t c0 = 0; c0 < n; c0 += CUMSUM_CHUNK) {
        const int cn = (int)(n - c0 < CUMSUM_CHUNK ? n - c0 : CUMSUM_CHUNK);
        for (int i = threadIdx.x; i < cn; i += blockDim.x) buf[i] = td_load(a, c0 + i, i1, i2, i3);
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 0; i < cn; ++i) {
                s += (double)buf[i];
                buf[i] = (float)s;
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < cn; i += blockDim.x) td_store(dst, c0 + i, i1, i2, i3, buf[i]);
        __syncthreads();
    }
}

// ---- UPSCALE ----------------------------------------------------------------------------------
// mode 0: upstream nearest, src index (int64)(i / sf) with sf = (float)ne_dst / ne_src per dim.
// mode 1: linear along ne0 as ATen's upsample_linear1d (align_corners = False) computes it.
__global__ void k_upscale(TD dst, TD a, int mode, float sc, float sf0, float sf1, float sf2, float sf3, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unravel(k, dst.ne, i0, i1, i2, i3);
        float v;
        if (mode == 0) {
            v = td_load(a, (int64_t)((float)i0 / sf0), (int64_t)((float)i1 / sf1), (int64_t)((float)i2 / sf2), (int64_t)((float)i3 / sf3));
        } else {
            float x = fmaf(sc, (float)i0 + 0.5f, -0.5f);
            if (x < 0.f) x = 0.f;
            const int64_t j0 = (int64_t)x;
            const int64_t j1 = j0 + (j0 < a.ne[0] - 1 ? 1 : 0);
            const float l1 = fminf(fmaxf(x - (float)j0, 0.f), 1.f);
            const float l0 = 1.f - l1;
            v = fmaf(td_load(a, j0, i1, i2, i3), l0, __fmul_rn(td_load(a, j1, i1, i2, i3), l1));
        }
        td_store(dst, i0, i1, i2, i3, v);
    }
}

// ---- twiddles ---------------------------------------------------------------------------------
// cos/sin(2*pi*m/n) by exact octant reduction and fixed f64 Taylor polynomials, operation for
// operation the oracle's tw_sincos (the build compiles with -ffp-contract=off, so no fusion).
__device__ __forceinline__ double2 tw_sincos(int m, int n) {
    m %= n;
    if (m < 0) m += n;
    const int q = (4 * m) / n, r = 4 * m - q * n;
    const bool comp = 2 * r > n;
    const int rr = comp ? n - r : r;
    const double x = __dmul_rn((double)rr, __ddiv_rn(1.5707963267948966, (double)n));
    const double x2 = x * x;
    const double sp = x * (1.0 + x2 * (-1.0 / 6 + x2 * (1.0 / 120 + x2 * (-1.0 / 5040 + x2 * (1.0 / 362880 + x2 * (-1.0 / 39916800 +
                      x2 * (1.0 / 6227020800.0 + x2 * (-1.0 / 1307674368000.0 + x2 * (1.0 / 355687428096000.0)))))))));
    const double cp = 1.0 + x2 * (-0.5 + x2 * (1.0 / 24 + x2 * (-1.0 / 720 + x2 * (1.0 / 40320 + x2 * (-1.0 / 3628800 +
                      x2 * (1.0 / 479001600.0 + x2 * (-1.0 / 87178291200.0 + x2 * (1.0 / 20922789888000.0))))))));
    const double c0 = comp ? sp : cp, s0 = comp ? cp : sp;
    double2 o;
    o.x = q == 0 ? c0 : q == 1 ? -s0 : q == 2 ? -c0 : s0;
    o.y = q == 0 ? s0 : q == 1 ? c0 : q == 2 ? -s0 : -c0;
    return o;
}

// ---- STFT -------------------------------------------------------------------------------------
// One thread per (bin k, frame t, batch b), k fastest so the [N, F, B, 2] planes are written
// coalesced.  Frame samples come from the reflect-padded signal (centre = True); the N twiddles
// live in LDS.  Per output: N-term f64 DFT in n order, one rounding, rfft's +0 imag at DC/Nyquist.
__global__ __launch_bounds__(256) void k_stft(TD dst, TD a, TD win, int N, int H, int abs_angle) {
    extern __shared__ double tw[];  // [N][2]
    for (int m = threadIdx.x; m < N; m += blockDim.x) {
        const double2 cs = tw_sincos(m, N);
        tw[2 * m] = cs.x;
        tw[2 * m + 1] = cs.y;
    }
    __syncthreads();
    const int64_t F = dst.ne[1], B = dst.ne[2], L = a.ne[0];
    const int64_t total = (int64_t)N * F * B;
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= total) return;
    const int k = (int)(o % N);
    const int64_t t = (o / N) % F, b = o / ((int64_t)N * F);
    double re = 0.0, im = 0.0;
    int m = 0;  // (k * n) mod N, stepped
    for (int n = 0; n < N; ++n) {
        int64_t j = t * H + n - N / 2;
        if (j < 0) j = -j;
        if (j >= L) j = 2 * (L - 1) - j;
        const double xw = (double)td_load(a, j, b, 0, 0) * (double)td_load(win, n, 0, 0, 0);
        re += xw * tw[2 * m];
        im -= xw * tw[2 * m + 1];
        m += k;
        if (m >= N) m -= N;
    }
    const float fr = (float)re;
    const float fi = (k == 0 || 2 * k == N) ? 0.0f : (float)im;
    float o0 = fr, o1 = fi;
    if (abs_angle) {
        o0 = (float)__dsqrt_rn((double)fr * (double)fr + (double)fi * (double)fi);
        o1 = (float)atan2((double)fi, (double)fr);
    }
    td_store(dst, k, t, b, 0, o0);
    td_store(dst, k, t, b, 1, o1);
}

// ---- ISTFT ------------------------------------------------------------------------------------
// One workgroup per tile of ISTFT_TILE output samples.  The tile's covering frames (plus the
// N/H - 1 frame halo) are converted once to f64 (Re, Im) in LDS -- the mag * e^{i phase} sincos
// is the expensive part and each frame feeds N output samples -- together with the twiddles.
// Each thread then overlap-adds its sample over the covering frames in ascending order.
constexpr int ISTFT_TILE = 256;

static int64_t istft_tile_frames(int N, int H) { return (ISTFT_TILE - 1 + N) / H + 2; }

__global__ __launch_bounds__(ISTFT_TILE) void k_istft(TD dst, TD a, TD win, int N, int H, int abs_angle) {
    extern __shared__ double lds[];
    const int K = (int)a.ne[0];
    const int64_t F = a.ne[1], Lout = dst.ne[0];
    const int64_t b = blockIdx.y;
    const int64_t j0 = (int64_t)blockIdx.x * ISTFT_TILE;
    const int64_t jl = (j0 + ISTFT_TILE < Lout ? j0 + ISTFT_TILE : Lout) - 1;
    const int64_t p0 = j0 + N / 2, p1 = jl + N / 2;
    const int64_t t_lo = p0 - N + 1 > 0 ? (p0 - N + 1 + H - 1) / H : 0;
    const int64_t t_hi = p1 / H < F - 1 ? p1 / H : F - 1;
    const int nt = (int)(t_hi - t_lo + 1);
    double * tw = lds;                 // [N][2]
    double * z = lds + 2 * N;          // [nt][K][2]
    for (int m = threadIdx.x; m < N; m += blockDim.x) {
        const double2 cs = tw_sincos(m, N);
        tw[2 * m] = cs.x;
        tw[2 * m + 1] = cs.y;
    }
    for (int i = threadIdx.x; i < nt * K; i += blockDim.x) {
        const int tt = i / K, k = i - tt * K;
        const double a0 = (double)td_load(a, k, t_lo + tt, b, 0), a1 = (double)td_load(a, k, t_lo + tt, b, 1);
        double re = a0, im = a1;
        if (abs_angle) {
            re = a0 * cos(a1);
            im = a0 * sin(a1);
        }
        z[2 * i] = re;
        z[2 * i + 1] = im;
    }
    __syncthreads();
    const int64_t j = j0 + threadIdx.x;
    if (j >= Lout) return;
    const int64_t p = j + N / 2;
    const int64_t t0 = p - N + 1 > 0 ? (p - N + 1 + H - 1) / H : 0;
    const int64_t t1 = p / H < F - 1 ? p / H : F - 1;
    double y = 0.0;
    for (int64_t t = t0; t <= t1; ++t) {
        const int n = (int)(p - t * H);
        const double * zt = z + 2 * (t - t_lo) * K;
        double acc = 0.0;
        int m = 0;  // (k * n) mod N
        for (int k = 0; k < K; ++k) {
            double term;
            if (k == 0 || 2 * k == N) term = zt[2 * k] * tw[2 * m];
            else term = 2.0 * (zt[2 * k] * tw[2 * m] - zt[2 * k + 1] * tw[2 * m + 1]);
            acc += term;
            m += n;
            if (m >= N) m -= N;
        }
        y += __ddiv_rn(acc, (double)N) * (double)td_load(win, n, 0, 0, 0);
    }
    td_store(dst, j, b, 0, 0, (float)y);
}

// ------------------------------------------------------------------------------------------

// ---- MAP_CUSTOM3 / uv_noise_compute (src/util.cpp:140-170) -------------------------------------
// One thread per (sample r, harmonic h): the reference's CPU callback as a device elementwise pass
// over the upsampled F0 it reads, so the sine source needs no mid-graph round trip to the host.
// hashed = 1: the draws come from splitmix64(seed, i) (oracle/ggml_ref.c uv_draw) instead of cdata.
__device__ __forceinline__ float uv_draw(uint64_t seed, uint64_t i) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + i + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(z >> 40) * (1.0f / 16777216.0f);
}

__global__ __launch_bounds__(256) void k_uv_noise(float * __restrict__ uv, float * __restrict__ noise, const float * __restrict__ f0up,
                                                  const float * __restrict__ cdata, int64_t L, int64_t n, int hashed, uint64_t seed) {
    const float thr = cdata[0], noise_std = cdata[1], sin_amp = cdata[2], amp_div = cdata[3];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const bool voiced = f0up[i % L] > thr;
        uv[i] = voiced ? sin_amp : 0.0f;
        const float r = hashed ? uv_draw(seed, (uint64_t)i) : cdata[4 + i];
        noise[i] = (voiced ? noise_std : amp_div) * r;
    }
}

// ---- MAP_CUSTOM2 / cfg_scale (src/util.cpp:175-200) -------------------------------------------
__global__ __launch_bounds__(256) void k_cfg_scale(TD dst, TD a, TD b, float scale, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
        int64_t i0, i1, i2, i3;
        unravel(k, dst.ne, i0, i1, i2, i3);
        const float cr = td_load(a, i0, i1, i2, i3), ur = td_load(b, i0, i1, i2, i3);
        td_store(dst, i0, i1, i2, i3, __fadd_rn(cr, __fmul_rn(scale, __fsub_rn(cr, ur))));
    }
}

static size_t istft_lds(int N, int H, int K) { return (size_t)16 * N + (size_t)16 * istft_tile_frames(N, H) * K; }

bool audio_op_supported(const tts_tensor * n) {
    const tts_tensor * a = n->src[0];
    if (!a || a->type != TTS_TYPE_F32 || n->type != TTS_TYPE_F32) return false;
    switch (n->op) {
        case TTS_OP_CUMSUM: return true;
        case TTS_OP_UPSCALE:
            if (n->op_params[0] == 0) return true;
            return n->op_params[0] == 1 && n->ne[1] == a->ne[1] && n->ne[2] == a->ne[2] && n->ne[3] == a->ne[3];
        case TTS_OP_STFT: {
            const int N = n->op_params[0], H = n->op_params[1];
            return N >= 1 && H >= 1 && 16 * (size_t)N <= 64 * 1024 && a->ne[0] > N / 2 && n->src[1] && n->src[1]->type == TTS_TYPE_F32;
        }
        case TTS_OP_MAP_CUSTOM2: {
            const tts_tensor * b = n->src[1];
            return n->op_params[0] == TTS_CUSTOM_CFG_SCALE && b && b->type == TTS_TYPE_F32 && b->ne[0] == a->ne[0] &&
                   b->ne[1] == a->ne[1] && b->ne[2] == a->ne[2] && b->ne[3] == a->ne[3];
        }
        case TTS_OP_MAP_CUSTOM3: {
            // contiguous [L, H, 2] destination, F0 of length L, data = 4 + L*H floats
            const tts_tensor *b = n->src[1], *c = n->src[2];
            return n->op_params[0] == TTS_CUSTOM_UV_NOISE && b && c && b->type == TTS_TYPE_F32 && c->type == TTS_TYPE_F32 &&
                   n->ne[2] == 2 && n->ne[3] == 1 && b->ne[0] == n->ne[0] && b->nb[0] == 4 && n->nb[0] == 4 &&
                   n->nb[1] == 4 * (size_t)n->ne[0] && n->nb[2] == n->nb[1] * (size_t)n->ne[1] &&
                   c->ne[0] * c->ne[1] * c->ne[2] * c->ne[3] >= 4 + (n->op_params[1] == 1 ? 0 : n->ne[0] * n->ne[1]);
        }
        case TTS_OP_ISTFT: {
            const int N = n->op_params[0], H = n->op_params[1];
            return N >= 1 && H >= 1 && a->ne[0] == N / 2 + 1 && istft_lds(N, H, (int)a->ne[0]) <= 160 * 1024 && n->src[1] &&
                   n->src[1]->type == TTS_TYPE_F32;
        }
    }
    return false;
}

static void set_lds(const void * fn, size_t lds) {
    if (lds > 64 * 1024) TTS_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}

int launch_audio_op(tts_hip_backend * be, const tts_tensor * n) {
    if (!audio_op_supported(n)) return TTS_STATUS_UNSUPPORTED;
    const TD d = make_td(n), a = make_td(n->src[0]);
    const int64_t ne = n->ne[0] * n->ne[1] * n->ne[2] * n->ne[3];
    switch (n->op) {
        case TTS_OP_CUMSUM:
            hipLaunchKernelGGL(k_cumsum, dim3((unsigned)(n->ne[1] * n->ne[2] * n->ne[3])), dim3(256), 0, be->stream, d, a);
            break;
        case TTS_OP_UPSCALE: {
            const tts_tensor * s = n->src[0];
            const float sc = (float)((double)s->ne[0] / (double)n->ne[0]);
            float sf[4];
            for (int i = 0; i < 4; ++i) sf[i] = (float)n->ne[i] / (float)s->ne[i];
            int64_t g = (ne + 255) / 256;
            if (g > 65536) g = 65536;
            hipLaunchKernelGGL(k_upscale, dim3((unsigned)g), dim3(256), 0, be->stream, d, a, n->op_params[0], sc, sf[0], sf[1], sf[2], sf[3], ne);
        } break;
        case TTS_OP_STFT: {
            const int N = n->op_params[0], H = n->op_params[1];
            const int64_t total = (int64_t)N * n->ne[1] * n->ne[2];
            hipLaunchKernelGGL(k_stft, dim3((unsigned)((total + 255) / 256)), dim3(256), (size_t)16 * N, be->stream, d, a,
                               make_td(n->src[1]), N, H, n->op_params[2]);
        } break;
        case TTS_OP_ISTFT: {
            const int N = n->op_params[0], H = n->op_params[1];
            const size_t lds = istft_lds(N, H, (int)n->src[0]->ne[0]);
            set_lds((const void *)k_istft, lds);
            const unsigned tiles = (unsigned)((n->ne[0] + ISTFT_TILE - 1) / ISTFT_TILE);
            hipLaunchKernelGGL(k_istft, dim3(tiles, (unsigned)n->ne[1]), dim3(ISTFT_TILE), lds, be->stream, d, a,
                               make_td(n->src[1]), N, H, n->op_params[2]);
        } break;
        case TTS_OP_MAP_CUSTOM2: {
            float scale;
            memcpy(&scale, &n->op_params[1], sizeof(float));
            int64_t g = (ne + 255) / 256;
            if (g > 8192) g = 8192;
            hipLaunchKernelGGL(k_cfg_scale, dim3((unsigned)(g < 1 ? 1 : g)), dim3(256), 0, be->stream, d, a, make_td(n->src[1]), scale, ne);
        } break;
        case TTS_OP_MAP_CUSTOM3: {
            const int64_t L = n->ne[0], cnt = L * n->ne[1];
            int64_t g = (cnt + 255) / 256;
            if (g > 8192) g = 8192;
            float * uv = (float *)n->data;
            hipLaunchKernelGGL(k_uv_noise, dim3((unsigned)(g < 1 ? 1 : g)), dim3(256), 0, be->stream, uv, (float *)((char *)n->data + n->nb[2]),
                               (const float *)n->src[1]->data, (const float *)n->src[2]->data, L, cnt, n->op_params[1] == 1 ? 1 : 0,
                               (uint64_t)(uint32_t)n->op_params[2] | ((uint64_t)(uint32_t)n->op_params[3] << 32));
        } break;
        default: return TTS_STATUS_UNSUPPORTED;
    }
    TTS_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace tts
