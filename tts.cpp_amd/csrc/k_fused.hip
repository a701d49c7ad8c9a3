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

// ---- fused LSTM step (Kokoro build_lstm_run, src/models/kokoro/model.cpp:56-86) ------------------
// The reference unrolls each time step into ~26 ggml nodes: four h-GEMVs (W_hh . h), bias adds,
// adds of the precomputed input projection column, sigmoid/tanh, the cell update and a concat
// that re-copies the whole output so far.  Here one launch runs a step: wave w of workgroup b owns
// hidden unit u = 4b + w and computes its four gate rows together (each lane keeps 4 partial f64
// sums over its k-slice, as ggml_vec_dot_f32 / _f16 accumulate in double), reduces them, and
// applies the node chain in the reference's order with every intermediate rounded to f32:
//   g = act(pre[u] + (float(W_g[u] . h) + b_g[u]))      act = sigmoid for I, F, O; tanh for G
//   c = F*c_prev + I*G,  h = tanh(c) * O
// Lanes 0-3 evaluate the four gate activations side by side (each an f64 transcendental), so the
// serial tail is one activation plus tanh(c).  blockIdx.y selects one of two independent chains
// (a bidirectional cell's forward and reverse runs advance in the same launch).
// F16 weights take the activation rounded to fp16 first (ggml's vec_dot_type for F16).
__global__ __launch_bounds__(256) void k_lstm_step(LstmStepArgs a0, LstmStepArgs a1) {
    const LstmStepArgs & a = blockIdx.y ? a1 : a0;
    const int lane = threadIdx.x & 63;
    const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u >= a.Hd) return;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = lane * 4; k < a.K; k += 256) {
        float4 h = *(const float4 *)(a.hprev + k);
        if (a.wtype == TTS_TYPE_F16) {
            h.x = __half2float(__float2half_rn(h.x));
            h.y = __half2float(__float2half_rn(h.y));
            h.z = __half2float(__float2half_rn(h.z));
            h.w = __half2float(__float2half_rn(h.w));
        }
        float4 w[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const char * row = (const char *)a.w[g] + (int64_t)u * a.w_rs[g];
            if (a.wtype == TTS_TYPE_F16) {
                const __half2 * hp = (const __half2 *)(row + 2 * (int64_t)k);
                const float2 lo = __half22float2(hp[0]), hi = __half22float2(hp[1]);
                w[g] = make_float4(lo.x, lo.y, hi.x, hi.y);
            } else {
                w[g] = *(const float4 *)(row + 4 * (int64_t)k);
            }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            acc[g] += (double)__fmul_rn(w[g].x, h.x);
            acc[g] += (double)__fmul_rn(w[g].y, h.y);
            acc[g] += (double)__fmul_rn(w[g].z, h.z);
            acc[g] += (double)__fmul_rn(w[g].w, h.w);
        }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = wave_sum_f64(acc[g]);  // wave-uniform
    // lane g (< 4) evaluates gate g
    const int g = lane & 3;
    const double dg = g == 0 ? acc[0] : g == 1 ? acc[1] : g == 2 ? acc[2] : acc[3];
    const float t1 = __fadd_rn((float)dg, a.bias[g][u]);
    const float x = __fadd_rn(a.pre[g][u], t1);
    const float gate = g == 2 ? cr_tanhf(x) : cr_divf(1.f, __fadd_rn(1.f, cr_expf(-x)));
    const float gi = __shfl(gate, 0), gf = __shfl(gate, 1), gg = __shfl(gate, 2), go = __shfl(gate, 3);
    if (lane != 0) return;
    const float c = __fadd_rn(__fmul_rn(gf, a.cprev[u]), __fmul_rn(gi, gg));
    a.c[u] = c;
    a.h[u] = __fmul_rn(cr_tanhf(c), go);
}

void launch_lstm_step(tts_hip_backend * be, const LstmStepArgs & a, const LstmStepArgs * b) {
    hipLaunchKernelGGL(k_lstm_step, dim3((unsigned)((a.Hd + 3) / 4), b ? 2u : 1u), dim3(256), 0, be->stream, a, b ? *b : a);
    TTS_HIP_CHECK(hipGetLastError());
}

// The chain's output (the last concat node, [Hd, T]) from the private hidden-state history.
__global__ void k_lstm_finish(TD out, const float * __restrict__ hist, int64_t Hd, int64_t n) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = e % Hd, t = e / Hd;
        *(float *)(out.data + k * out.nb[0] + t * out.nb[1]) = hist[e];
    }
}

void launch_lstm_finish(tts_hip_backend * be, const tts_tensor * out, const float * hist, int64_t Hd, int64_t T) {
    const int64_t n = Hd * T;
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_lstm_finish, dim3((unsigned)g), dim3(256), 0, be->stream, make_td(out), hist, Hd, n);
    TTS_HIP_CHECK(hipGetLastError());
}

// ---- snake_1d (src/util.cpp:98-101) ------------------------------------------------------------
// ADD(x, MUL(SQR(SIN(MUL(x, alpha))), recip)) in one pass instead of five, keeping each node's f32
// rounding: m = x*a, s = sin(m) (correctly rounded), q = s*s, r = q*recip, y = x + r.  alpha and
// recip are per-channel ([1, C]: one value per row of the [T, C] activation).
// recip == nullptr: r = one / alpha[c], the DIV node of reciprocal() (util.cpp:86-94) evaluated here.
// mask != nullptr: x = x * mask[t] first (t = the position along ne0; a MUL node's f32 product).
template <int V>
__global__ void k_snake(float * __restrict__ dst, const float * __restrict__ x, const float * __restrict__ alpha,
                        const float * __restrict__ recip, const float * __restrict__ one, const float * __restrict__ mask, int64_t n,
                        int64_t ne0, int64_t nc) {
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * V; k < n; k += (int64_t)gridDim.x * blockDim.x * V) {
        const int64_t c = (k / ne0) % nc;
        const float a = alpha[c], r = recip ? recip[c] : cr_divf(*one, a);
        float xv[V], y[V];
        if (V == 4) {
            const float4 t = *(const float4 *)(x + k);
            xv[0] = t.x, xv[1] = t.y, xv[2] = t.z, xv[3] = t.w;
        } else {
            xv[0] = x[k];
        }
        if (mask) {
            const int64_t t0 = k % ne0;  // V == 4: ne0 % 4 == 0, the 4 elements share a row
#pragma unroll
            for (int e = 0; e < V; ++e) xv[e] = __fmul_rn(xv[e], mask[t0 + e]);
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const float sn = cr_sinf(__fmul_rn(xv[e], a));
            y[e] = __fadd_rn(xv[e], __fmul_rn(__fmul_rn(sn, sn), r));
        }
        if (V == 4) *(float4 *)(dst + k) = make_float4(y[0], y[1], y[2], y[3]);
        else dst[k] = y[0];
    }
}

void launch_snake(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * x, const tts_tensor * alpha, const tts_tensor * recip,
                  const tts_tensor * one, const tts_tensor * mask) {
    const float * rp = recip ? (const float *)recip->data : nullptr;
    const float * op = one ? (const float *)one->data : nullptr;
    const float * mp = mask ? (const float *)mask->data : nullptr;
    const int64_t n = dst->ne[0] * dst->ne[1] * dst->ne[2] * dst->ne[3];
    const int64_t ne0 = x->ne[0], nc = alpha->ne[1];
    const bool v4 = ne0 % 4 == 0 && ((uintptr_t)dst->data % 16) == 0 && ((uintptr_t)x->data % 16) == 0;
    int64_t g = ((v4 ? n / 4 : n) + 255) / 256;
    if (g > 65536) g = 65536;
    if (v4)
        hipLaunchKernelGGL(k_snake<4>, dim3((unsigned)g), dim3(256), 0, be->stream, (float *)dst->data, (const float *)x->data,
                           (const float *)alpha->data, rp, op, mp, n, ne0, nc);
    else
        hipLaunchKernelGGL(k_snake<1>, dim3((unsigned)g), dim3(256), 0, be->stream, (float *)dst->data, (const float *)x->data,
                           (const float *)alpha->data, rp, op, mp, n, ne0, nc);
    TTS_HIP_CHECK(hipGetLastError());
}

// ---- AdaIN (+ snake) over one channel row (build_kokoro_generator_res_block, kokoro/model.cpp:
// 136-165): NORM over time -> CONT(TRANSPOSE) -> x + x*gamma[c] -> + beta[c] -> CONT(TRANSPOSE)
// [-> snake_1d with alpha[c], recip[c]] in one pass.  One 1024-thread workgroup per channel keeps
// the row in registers (NPT elements per thread): one HBM read and one write instead of the
// nine launches and the two transposes of the node chain.  Every f32 operation is the node's, in
// the node's order; the two f64 sums are block reductions, as k_norm's. ----
__device__ __forceinline__ double block_sum1024(double v, double * sh) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += sh[i];
    return t;
}

template <int NPT, bool SNAKE>
__global__ __launch_bounds__(1024) void k_adain_snake(AdainArgs a) {
    __shared__ double sh[16];
    const int64_t c = blockIdx.x;
    const int64_t T = a.T;
    const float * x = a.x + c * a.xcs;
    float * y = a.y + c * a.ycs;
    float v[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
        const int64_t t = threadIdx.x + 1024 * u;
        v[u] = t < T ? x[t] : 0.f;
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < NPT; ++u) s += (double)v[u];  // padding adds 0
    s = block_sum1024(s, sh);
    const float mean = (float)(s / (double)T);
    double s2 = 0.0;
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
        const int64_t t = threadIdx.x + 1024 * u;
        const float d = __fsub_rn(v[u], mean);
        if (t < T) s2 += (double)__fmul_rn(d, d);
    }
    s2 = block_sum1024(s2, sh);
    const float variance = (float)(s2 / (double)T);
    const float scale = cr_divf(1.0f, cr_sqrtf(__fadd_rn(variance, a.eps)));
    float g, b;
    if (a.gw) {
        // waves 0 / 1: the gamma / beta GEMV rows, lane l summing k = 4l + 256j in k_gemv_float's
        // order (f32 products, f64 sum, xor butterfly), then the bias ADD
        __shared__ float gbv[2];
        const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
        if (w < 2) {
            const float * wr = (w == 0 ? a.gw : a.bw) + c * a.S;
            double acc = 0.0;
            for (int64_t k = l * 4; k < a.S; k += 256) {
                const float4 wv = *(const float4 *)(wr + k);
                const float4 xv = *(const float4 *)(a.style + k);
                acc += (double)__fmul_rn(wv.x, xv.x);
                acc += (double)__fmul_rn(wv.y, xv.y);
                acc += (double)__fmul_rn(wv.z, xv.z);
                acc += (double)__fmul_rn(wv.w, xv.w);
            }
            for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
            if (l == 0) gbv[w] = __fadd_rn((float)acc, (w == 0 ? a.gb : a.bb)[c]);
        }
        __syncthreads();
        g = gbv[0], b = gbv[1];
    } else {
        g = a.gamma[c * a.gcs], b = a.beta[c * a.bcs];
    }
    const float al = SNAKE ? a.alpha[c * a.acs] : 0.f;
    const float rc = SNAKE ? (a.recip ? a.recip[c * a.rcs] : cr_divf(a.one[0], al)) : 0.f;
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
        const int64_t t = threadIdx.x + 1024 * u;
        if (t >= T) continue;
        const float n = __fmul_rn(__fsub_rn(v[u], mean), scale);
        float o = __fadd_rn(__fadd_rn(n, __fmul_rn(n, g)), b);
        if (SNAKE) {
            const float sn = cr_sinf(__fmul_rn(o, al));
            o = __fadd_rn(o, __fmul_rn(__fmul_rn(sn, sn), rc));
        }
        y[t] = o;
    }
}

bool adain_supported(int64_t T) { return T >= 1 && T <= 1024 * 64; }

__global__ void k_stage_vecs(float * __restrict__ dst, AdainArgs a) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.C) return;
    if (!a.gw) {
        dst[c] = a.gamma[c * a.gcs];
        dst[a.C + c] = a.beta[c * a.bcs];
    }
    if (a.alpha) dst[2 * a.C + c] = a.alpha[c * a.acs];
    if (a.alpha && a.recip) dst[3 * a.C + c] = a.recip[c * a.rcs];
    if (c == 0 && a.one) dst[4 * a.C] = a.one[0];
}

void launch_adain_snake(tts_hip_backend * be, const AdainArgs & args) {
    AdainArgs a = args;
    if (a.stage) {
        float * v = be->vec_scratch;
        hipLaunchKernelGGL(k_stage_vecs, dim3((unsigned)((a.C + 255) / 256)), dim3(256), 0, be->stream, v, args);
        if (!a.gw) a.gamma = v, a.gcs = 1, a.beta = v + a.C, a.bcs = 1;
        if (a.alpha) a.alpha = v + 2 * a.C, a.acs = 1;
        if (a.alpha && a.recip) a.recip = v + 3 * a.C, a.rcs = 1;
        if (a.one) a.one = v + 4 * a.C;
    }
    const bool sn = a.alpha != nullptr;
    const int npt = a.T <= 8192 ? 8 : a.T <= 16384 ? 16 : a.T <= 32768 ? 32 : 64;
    const dim3 grid((unsigned)a.C), block(1024);
#define TTS_ADAIN(N)                                                                                       \
    if (npt == N) {                                                                                        \
        if (sn) hipLaunchKernelGGL((k_adain_snake<N, true>), grid, block, 0, be->stream, a);               \
        else hipLaunchKernelGGL((k_adain_snake<N, false>), grid, block, 0, be->stream, a);                 \
    }
    TTS_ADAIN(8) TTS_ADAIN(16) TTS_ADAIN(32) TTS_ADAIN(64)
#undef TTS_ADAIN
    TTS_HIP_CHECK(hipGetLastError());
}

// ---- greedy sampling step (sampler::max, src/sampler.cpp:185-204) --------------------------------
// One wave per (prompt b, head h) row of the step's logits [B][NH][V]: each lane scans its strided
// slice keeping the first strict maximum (indices ascend within a lane), then the lanes combine by
// (larger value, then smaller index) -- the sequential scan's answer, NaN skipped, 0 when no value
// exceeds -inf.  Lane 0 applies Parler's next-token rule (next_decoder_token_ids, model.cpp:778-785).
__global__ __launch_bounds__(256) void k_greedy_step(const float * __restrict__ logits, int B, int NH, int V, int step, int bos, int eos,
                                                     int32_t * eos_seen, int32_t * hist, int32_t * next) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= B * NH) return;
    const float * l = logits + (int64_t)row * V;
    float best = -INFINITY;
    int bi = 0x7FFFFFFF;
    for (int i = lane; i < V; i += 64) {
        const float v = l[i];
        if (v > best) {
            best = v;
            bi = i;
        }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        if (ov > best || (ov == best && oi < bi)) {
            best = ov;
            bi = oi;
        }
    }
    if (lane != 0) return;
    const int tok = bi == 0x7FFFFFFF ? 0 : bi;
    const int b = row / NH, h = row % NH;
    hist[row] = tok;
    const int seen = eos_seen[row] | (tok == eos);
    eos_seen[row] = seen;
    next[h * B + b] = step + 1 > h ? (seen ? eos : tok) : bos;
}

// Large vocabularies (Orpheus: 156 940 logits per prompt): the row is split over `gridDim.x`
// workgroups; each folds its segment to (value, first index) and merges it into the row's 64-bit
// key with one atomicMax (orderable float bits high, ~index low: the larger value wins, then the
// smaller index -- sampler::max's first maximum).  The last workgroup of the row to arrive
// (device-scope counter) applies the same sample / EOS / next-token rule as k_greedy_step and
// clears the key and counter for the next launch.
__device__ __forceinline__ unsigned long long argmax_key(float v, int i) {
    unsigned u = __float_as_uint(v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // total order of non-NaN floats
    return ((unsigned long long)u << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
}

__global__ __launch_bounds__(256) void k_greedy_step_wide(const float * __restrict__ logits, int B, int NH, int V, int step, int bos,
                                                          int eos, int32_t * eos_seen, int32_t * hist, int32_t * next,
                                                          unsigned long long * keys, unsigned * counts) {
    __shared__ unsigned long long s_k[4];
    const int row = blockIdx.y, nseg = gridDim.x;
    const int64_t seg = ((int64_t)V + nseg - 1) / nseg;
    const int64_t i0 = (int64_t)blockIdx.x * seg, i1 = min((int64_t)V, i0 + seg);
    const float * l = logits + (int64_t)row * V;
    unsigned long long best = 0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
        const unsigned long long k = argmax_key(l[i], (int)i);
        best = k > best ? k : best;
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) s_k[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < 4; ++w) best = s_k[w] > best ? s_k[w] : best;
    atomicMax(keys + row, best);
    __threadfence();
    if (atomicAdd(counts + row, 1u) != (unsigned)nseg - 1) return;
    const unsigned long long k = atomicExch(keys + row, 0ull);
    atomicExch(counts + row, 0u);
    const int tok = k ? (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull)) : 0;
    const int b = row / NH, h = row % NH;
    hist[row] = tok;
    const int seen = eos_seen[row] | (tok == eos);
    eos_seen[row] = seen;
    next[h * B + b] = step + 1 > h ? (seen ? eos : tok) : bos;
}

void launch_greedy_step(tts_hip_backend * be, const float * logits, int B, int NH, int V, int step, int bos, int eos, int32_t * eos_seen,
                        int32_t * hist, int32_t * next) {
    if (V >= 16384 && B * NH <= kArgmaxRows) {
        const unsigned nseg = (unsigned)((V + 4095) / 4096 < 64 ? (V + 4095) / 4096 : 64);
        hipLaunchKernelGGL(k_greedy_step_wide, dim3(nseg, (unsigned)(B * NH)), dim3(256), 0, be->stream, logits, B, NH, V, step, bos, eos,
                           eos_seen, hist, next, be->argmax_keys, be->argmax_counts);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    hipLaunchKernelGGL(k_greedy_step, dim3((unsigned)((B * NH + 3) / 4)), dim3(256), 0, be->stream, logits, B, NH, V, step, bos, eos, eos_seen,
                       hist, next);
    TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
