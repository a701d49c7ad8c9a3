// Fused decode attention: one kernel replaces
//   cont(K view) -> mul_mat(K, q) -> soft_max_ext(mask, scale) -> mul_mat(kq, V) -> permute(2,0,1,3) -> cont
// (Parler model.cpp:549-571 self, 583-594 cross; Dia model.cpp:540-615; Orpheus model.cpp:259-285).
// K and V are read in place through their cache views: the reference's per-step `cont` copy of K
// (O(P*d) per layer per step) disappears.  Numerics are the unfused ops' exactly: f32 products
// accumulated in f64 (ggml_vec_dot_f32), ggml's soft_max (scale, mask, max, expf, f64 sum, 1/sum),
// with expf correctly rounded (transcendental policy, hip_internal.h).
#include "hip_internal.h"
#include <hip/hip_ext.h>

namespace tts {

// ------------------------------------------------------------------------------------------
// Decode attention, one workgroup per (head h, query t, sequence b).
struct AttnArgs {
    TD q;      // [hd, n, H, B]   (the permute view feeding ggml's cont(q))
    TD k;      // [hd, P, Hk, Bk] (K view of the cache, or cross_k)
    TD v;      // [P, hd, Hv, Bv] (V view of the cache, or cross_v)
    const float * mask;  // [rows >= n][P] f32, row stride P (ggml soft_max broadcast), or null
    float scale;
    float * out;         // [hd, H, n] per sequence, sequence b at out + b * obs
    int hd, P, H, n, B;
    float * out2 = nullptr;  // optional second copy of out (the next GEMV's private input), [hd, H, n, B] contiguous
    int64_t obs = 0;     // floats between sequences of out (n * H * hd when contiguous; a coalesced step's member stride)
    int64_t mbs = 0;     // floats between sequences' masks (0: one mask for all)
    unsigned long long * ts = nullptr;  // phase timestamps (scripts/attn_phase.hip builds only)
    // Ragged sequences (a coalesced step of runners at different KV lengths, coalesce.hip): per
    // sequence b, the byte offsets of its K and V views from k.data / v.data (the views' own nb[3] is
    // then 0), its mask row offset in floats (instead of b * mbs) and its key count (<= P, the grid's).
    // The mask's row stride is the sequence's key count, as each member's own [P_b, n] mask has.
    const int64_t * koff = nullptr;
    const int64_t * voff = nullptr;
    const int64_t * moff = nullptr;
    const int * pseq = nullptr;
};

// per-sequence views of a ragged launch (AttnArgs::koff / voff / moff / pseq)
__device__ __forceinline__ int seq_p(const AttnArgs & a, int b) { return a.pseq ? a.pseq[b] : a.P; }
__device__ __forceinline__ int64_t seq_koff(const AttnArgs & a, int b) { return a.koff ? a.koff[b] : 0; }
__device__ __forceinline__ int64_t seq_voff(const AttnArgs & a, int b) { return a.voff ? a.voff[b] : 0; }
__device__ __forceinline__ const float * seq_mrow(const AttnArgs & a, int b, int tq, int P) {
    return a.mask ? a.mask + (a.moff ? a.moff[b] : (int64_t)b * a.mbs) + (int64_t)tq * P : nullptr;
}

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
    const int P = seq_p(a, b), hd = a.hd;
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const char * qbase = a.q.data + t * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3] + seq_koff(a, b);

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
    const float * mrow = seq_mrow(a, b, t, P);
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
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + seq_voff(a, b);
    float * orow = a.out + (int64_t)b * a.obs + ((int64_t)t * a.H + h) * hd;
    // the shadow copy is per sequence at its contiguous place (a coalesced step's out stride is not)
    float * orow2 = a.out2 ? a.out2 + (((int64_t)b * a.n + t) * a.H + h) * hd : nullptr;
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
                if (lane == 0 && d0 + u < hd) {
                    orow[d0 + u] = (float)s;
                    if (orow2) orow2[d0 + u] = (float)s;
                }
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
                if (lane == 0 && d0 + u < hd) {
                    orow[d0 + u] = (float)s;
                    if (orow2) orow2[d0 + u] = (float)s;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Decode attention for hd = 64 * DPR (Parler 64, Dia / Orpheus 128), same numerics as above, laid
// out for memory latency (a round trip is ~0.8 us cold; the kernel is a handful of them):
//   - K, V (when PF: P <= 512 for hd 64) and q are all requested at kernel entry, so the whole
//     kernel waits on ONE memory round trip; V sits in registers until the softmax is done;
//   - A: a quad (4 lanes) per key position, lane q owning 16*DPR dims; 128 positions per 512-thread
//     step; the f64 dot is finished with two DPP quad steps;
//   - B: soft_max_ext over the P scores in LDS (two barrier-separated reductions);
//   - C: a 16-lane row per output dim (lane t: positions 4t + 64u as 16-B loads of the V row when
//     VVEC, else scalar positions t + 16u), 32 dims per pass, DPP row reduction in f64.
// No reduction goes through the LDS crossbar and every load batch is issued before its first use.
// ATTN_UV: V chunks (per lane, per dim pass) in flight.
template <int DPR, bool VVEC, bool PF, int ATTN_UV>
__global__ __launch_bounds__(ATTN_THREADS) void k_attn_decode_rows(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) float s_p[];  // (P rounded to 64) + 64 floats (launcher)
    __shared__ float s_wf[ATTN_THREADS / 64];
    __shared__ double s_wd[ATTN_THREADS / 64];
    constexpr int NW = ATTN_THREADS / 64;
    constexpr int F = 4 * DPR;                      // float4 per lane per key position (hd / 4 dims)
    constexpr int KS = PF ? 512 / ATTN_THREADS * 4 : 2;  // key steps of 128 positions in flight
    constexpr int NPASS = 2 * DPR;                  // dim passes in C (32 dims each)
    const int h = blockIdx.x, tq = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane >> 4, t = lane & 15, qd = lane & 3;
    const int P = seq_p(a, b);
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * qbase = a.q.data + tq * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3] + seq_koff(a, b);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + seq_voff(a, b);
    const int64_t knb1 = a.k.nb[1], vnb0 = a.v.nb[0], vnb1 = a.v.nb[1];
    TTS_TS(a, 0);

    // ---- loads: q (this lane's dims), K for the first KS steps, V for every pass (PF) ----
    float qv[F][4];
#pragma unroll
    for (int c = 0; c < F; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) qv[c][e] = ((const float *)qbase)[16 * DPR * qd + 4 * c + e];
    const int pos0 = wave * 16 + (lane >> 2);  // this quad's position within a 128-step
    float4 kv[KS][F];
    auto load_k = [&](int i0) {
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            const int i = min(i0 + 128 * u + pos0, P - 1);
#pragma unroll
            for (int c = 0; c < F; ++c) kv[u][c] = TTS_KVLOAD((const float4 *)(kbase + (int64_t)i * knb1 + 16 * (F * qd + c)));
        }
    };
    load_k(0);
    constexpr int VL = PF ? NPASS * ATTN_UV : 1;
    float4 vv4[VVEC ? VL : 1];
    float vv1[VVEC ? 1 : VL];
    const int ilast = ((P - 1) >> 2) << 2;  // last 16-B chunk holding a position < P
    if (PF) {
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
            const char * vrow = vbase + (int64_t)(ps * 32 + wave * 4 + r) * vnb1;
#pragma unroll
            for (int u = 0; u < ATTN_UV; ++u) {
                if (VVEC) vv4[VVEC ? ps * ATTN_UV + u : 0] = TTS_KVLOAD((const float4 *)(vrow + 4 * (int64_t)min(64 * u + 4 * t, ilast)));
                else vv1[VVEC ? 0 : ps * ATTN_UV + u] = *(const float *)(vrow + (int64_t)min(16 * u + t, P - 1) * vnb0);
            }
        }
    }
    TTS_PIN_LOADS();

    // ---- A: kq[i] = sum_d (f32)(K[d,i] * q[d]) in f64 ----
    for (int i0 = 0; i0 < P; i0 += 128 * KS) {
        if (i0 > 0) {
            load_k(i0);
            TTS_PIN_LOADS();
        }
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < F; ++c) {
                s += (double)__fmul_rn(kv[u][c].x, qv[c][0]);
                s += (double)__fmul_rn(kv[u][c].y, qv[c][1]);
                s += (double)__fmul_rn(kv[u][c].z, qv[c][2]);
                s += (double)__fmul_rn(kv[u][c].w, qv[c][3]);
            }
            s += dpp_f64<DPP_XOR1>(s);
            s += dpp_f64<DPP_XOR2>(s);
            const int i = i0 + 128 * u + pos0;
            if (qd == 0 && i < P) s_p[i] = (float)s;
        }
    }
    __syncthreads();
    TTS_TS(a, 1);

    // ---- B: soft_max_ext: w = kq*scale + mask; max; e = expf(w - max); f64 sum; p = e * (1/sum) ----
    const float * mrow = seq_mrow(a, b, tq, P);
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
    const int P64 = (P + 63) & ~63;
    for (int i = tid; i < P64; i += ATTN_THREADS) s_p[i] = i < P ? __fmul_rn(s_p[i], inv) : 0.f;
    __syncthreads();
    TTS_TS(a, 3);

    // ---- C: out[d] = sum_i (f32)(p[i] * V[d,i]) in f64 ----
    float * orow = a.out + (int64_t)b * a.obs + ((int64_t)tq * a.H + h) * a.hd;
    float * orow2 = a.out2 ? a.out2 + (((int64_t)b * a.n + tq) * a.H + h) * a.hd : nullptr;
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
        const int d = ps * 32 + wave * 4 + r;
        const char * vrow = vbase + (int64_t)d * vnb1;
        double acc = 0.0;
        const int kstep = VVEC ? 64 * ATTN_UV : 16 * ATTN_UV;
        for (int k0 = 0; k0 < P; k0 += kstep) {
            float4 w4[VVEC ? ATTN_UV : 1];
            float w1[VVEC ? 1 : ATTN_UV];
            if (PF) {
#pragma unroll
                for (int u = 0; u < ATTN_UV; ++u) {
                    if (VVEC) w4[VVEC ? u : 0] = vv4[VVEC ? ps * ATTN_UV + u : 0];
                    else w1[VVEC ? 0 : u] = vv1[VVEC ? 0 : ps * ATTN_UV + u];
                }
            } else {
#pragma unroll
                for (int u = 0; u < ATTN_UV; ++u) {
                    if (VVEC) w4[VVEC ? u : 0] = TTS_KVLOAD((const float4 *)(vrow + 4 * (int64_t)min(k0 + 64 * u + 4 * t, ilast)));
                    else w1[VVEC ? 0 : u] = *(const float *)(vrow + (int64_t)min(k0 + 16 * u + t, P - 1) * vnb0);
                }
                TTS_PIN_LOADS();
            }
#pragma unroll
            for (int u = 0; u < ATTN_UV; ++u) {
                if (VVEC) {
                    const int i = k0 + 64 * u + 4 * t;
                    const float4 pp = *(const float4 *)(s_p + min(i, P64 - 4));
                    const float4 vq = w4[VVEC ? u : 0];
                    // positions >= P (tail and clamped chunks) contribute nothing, as in the scalar sum
                    acc += i + 0 < P ? (double)__fmul_rn(pp.x, vq.x) : 0.0;
                    acc += i + 1 < P ? (double)__fmul_rn(pp.y, vq.y) : 0.0;
                    acc += i + 2 < P ? (double)__fmul_rn(pp.z, vq.z) : 0.0;
                    acc += i + 3 < P ? (double)__fmul_rn(pp.w, vq.w) : 0.0;
                } else {
                    const int i = k0 + 16 * u + t;
                    acc += i < P ? (double)__fmul_rn(s_p[min(i, P - 1)], w1[VVEC ? 0 : u]) : 0.0;
                }
            }
        }
        acc += dpp_f64<DPP_XOR1>(acc);
        acc += dpp_f64<DPP_XOR2>(acc);
        acc += dpp_f64<DPP_HALF_MIRROR>(acc);
        acc += dpp_f64<DPP_MIRROR>(acc);
        if (t == 0 && d < a.hd) {
            orow[d] = (float)acc;
            if (orow2) orow2[d] = (float)acc;
        }
    }
    TTS_TS(a, 4);
}

template <int DPR, bool PF, int UV = 8>
static void launch_attn_rows(tts_hip_backend * be, const AttnArgs & a, bool vvec) {
    const dim3 grid((unsigned)a.H, (unsigned)a.n, (unsigned)a.B);
    const size_t pl = (size_t)(((a.P + 63) & ~63) + 64) * sizeof(float);  // s_p: the context, not ATTN_MAXP
    if (vvec) hipLaunchKernelGGL((k_attn_decode_rows<DPR, true, PF, UV>), grid, dim3(ATTN_THREADS), pl, be->stream, a);
    else hipLaunchKernelGGL((k_attn_decode_rows<DPR, false, PF, UV>), grid, dim3(ATTN_THREADS), pl, be->stream, a);
}

// ------------------------------------------------------------------------------------------
// Split decode attention for long contexts (P >= be->attn_split_minp).  One workgroup per head
// leaves most of the chip idle at decode batch sizes (Parler B = 8: 128 workgroups on 256 CUs) and
// keeps too few bytes in flight per CU; the split runs the same arithmetic as k_attn_decode_rows
// over many more workgroups, in two launches whose boundary is the softmax's global max:
//   k_attn_scores: grid (P chunks, H, n*B): the masked, scaled scores w_i = f32(f32(q.K_i)*scale)
//                  (+ mask) of 128*KS positions -> attn_buf, and the chunk's max;
//   k_attn_pv:     grid (hd/16, H, n*B): every workgroup takes the global max from the chunk maxima,
//                  recomputes e_i = expf(w_i - max) and the f64 sum over all P (cheap, L2-resident),
//                  p_i = e_i * (1/sum), then 16 output dims of sum_i f32(p_i * V[d,i]) in f64.
// Each output dim is still one workgroup's sum in one fixed order, and the V stream for that
// workgroup is requested at kernel entry, before the softmax, so its latency hides under it.
template <int DPR, int KS>
__global__ __launch_bounds__(ATTN_THREADS) void k_attn_scores(AttnArgs a, float * __restrict__ sbuf, int pstride,
                                                             float * __restrict__ mxbuf, int nch) {
    __shared__ float s_wf[ATTN_THREADS / 64];
    constexpr int F = 4 * DPR;
    const int c = blockIdx.x, h = blockIdx.y, z = blockIdx.z;
    const int b = z / a.n, tq = z - b * a.n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, qd = lane & 3;
    const int P = seq_p(a, b);
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const char * qbase = a.q.data + tq * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3] + seq_koff(a, b);
    const int64_t knb1 = a.k.nb[1];
    const int i0 = c * 128 * KS + wave * 16 + (lane >> 2);
    float4 kv[KS][F];
#pragma unroll
    for (int u = 0; u < KS; ++u) {
        const int i = min(i0 + 128 * u, P - 1);
#pragma unroll
        for (int f = 0; f < F; ++f) kv[u][f] = TTS_KVLOAD((const float4 *)(kbase + (int64_t)i * knb1 + 16 * (F * qd + f)));
    }
    float qv[F][4];
#pragma unroll
    for (int f = 0; f < F; ++f)
#pragma unroll
        for (int e = 0; e < 4; ++e) qv[f][e] = ((const float *)qbase)[16 * DPR * qd + 4 * f + e];
    TTS_PIN_LOADS();
    const float * mrow = seq_mrow(a, b, tq, P);
    float * srow = sbuf + ((int64_t)z * a.H + h) * pstride;
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < KS; ++u) {
        double s = 0.0;
#pragma unroll
        for (int f = 0; f < F; ++f) {
            s += (double)__fmul_rn(kv[u][f].x, qv[f][0]);
            s += (double)__fmul_rn(kv[u][f].y, qv[f][1]);
            s += (double)__fmul_rn(kv[u][f].z, qv[f][2]);
            s += (double)__fmul_rn(kv[u][f].w, qv[f][3]);
        }
        s += dpp_f64<DPP_XOR1>(s);
        s += dpp_f64<DPP_XOR2>(s);
        const int i = i0 + 128 * u;
        if (i < P) {
            float w = __fmul_rn((float)s, a.scale);
            if (mrow) w = __fadd_rn(w, __fmul_rn(1.0f, mrow[i]));
            if (qd == 0) srow[i] = w;
            mx = fmaxf(mx, w);
        }
    }
    mx = fmaxf(mx, dpp_f32<DPP_XOR1>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_XOR2>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_HALF_MIRROR>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_MIRROR>(mx));
    mx = fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 0)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 32)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 48))));
    if (lane == 0) s_wf[wave] = mx;
    __syncthreads();
    if (tid == 0) {
        float m = s_wf[0];
#pragma unroll
        for (int w = 1; w < ATTN_THREADS / 64; ++w) m = fmaxf(m, s_wf[w]);
        mxbuf[((int64_t)z * a.H + h) * nch + c] = m;
    }
}

constexpr int PV_THREADS = 256;

template <bool VVEC, int UV, int NW = PV_THREADS / 64>
__global__ __launch_bounds__(64 * NW) void k_attn_pv(AttnArgs a, const float * __restrict__ sbuf, int pstride,
                                                    const float * __restrict__ mxbuf, int nch) {
    // NW waves x 4 output dims each (4 NW dims per workgroup)
    constexpr int NTH = 64 * NW;
    // the probabilities in dynamic LDS sized to the context (launcher: (P rounded to 64) + 64 floats): a
    // fixed ATTN_MAXP array (33 KB) held the P.V grid to 4 workgroups per CU
    extern __shared__ __attribute__((aligned(16))) float s_p[];
    __shared__ double s_wd[NW];
    const int h = blockIdx.y, z = blockIdx.z;
    const int b = z / a.n, tq = z - b * a.n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane >> 4, t = lane & 15;
    const int P = seq_p(a, b);
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + seq_voff(a, b);
    const int64_t vnb0 = a.v.nb[0], vnb1 = a.v.nb[1];
    const int d = blockIdx.x * 4 * NW + wave * 4 + r;
    const char * vrow = vbase + (int64_t)min(d, a.hd - 1) * vnb1;
    const int ilast = ((P - 1) >> 2) << 2;
    float4 w4[VVEC ? UV : 1];
    float w1[VVEC ? 1 : UV];
    auto load_v = [&](int k0) {
#pragma unroll
        for (int u = 0; u < UV; ++u) {
            if (VVEC) w4[VVEC ? u : 0] = TTS_KVLOAD((const float4 *)(vrow + 4 * (int64_t)min(k0 + 64 * u + 4 * t, ilast)));
            else w1[VVEC ? 0 : u] = *(const float *)(vrow + (int64_t)min(k0 + 16 * u + t, P - 1) * vnb0);
        }
    };
    load_v(0);  // in flight during the softmax
    const float * srow = sbuf + ((int64_t)z * a.H + h) * pstride;
    const float * mrow = mxbuf + ((int64_t)z * a.H + h) * nch;
    float mx = -INFINITY;
    for (int k = 0; k < nch; ++k) mx = fmaxf(mx, mrow[k]);
    double sum = 0.0;
    for (int i = tid; i < P; i += NTH) {
        const float e = cr_expf(__fsub_rn(srow[i], mx));
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
    const int P64 = (P + 63) & ~63;
    for (int i = tid; i < P64; i += NTH) s_p[i] = i < P ? __fmul_rn(s_p[i], inv) : 0.f;
    __syncthreads();

    double acc = 0.0;
    const int kstep = VVEC ? 64 * UV : 16 * UV;
    for (int k0 = 0; k0 < P; k0 += kstep) {
        if (k0 > 0) {
            load_v(k0);
            TTS_PIN_LOADS();
        }
#pragma unroll
        for (int u = 0; u < UV; ++u) {
            if (VVEC) {
                const int i = k0 + 64 * u + 4 * t;
                const float4 pp = *(const float4 *)(s_p + min(i, P64 - 4));
                const float4 vq = w4[VVEC ? u : 0];
                acc += i + 0 < P ? (double)__fmul_rn(pp.x, vq.x) : 0.0;
                acc += i + 1 < P ? (double)__fmul_rn(pp.y, vq.y) : 0.0;
                acc += i + 2 < P ? (double)__fmul_rn(pp.z, vq.z) : 0.0;
                acc += i + 3 < P ? (double)__fmul_rn(pp.w, vq.w) : 0.0;
            } else {
                const int i = k0 + 16 * u + t;
                acc += i < P ? (double)__fmul_rn(s_p[min(i, P - 1)], w1[VVEC ? 0 : u]) : 0.0;
            }
        }
    }
    acc += dpp_f64<DPP_XOR1>(acc);
    acc += dpp_f64<DPP_XOR2>(acc);
    acc += dpp_f64<DPP_HALF_MIRROR>(acc);
    acc += dpp_f64<DPP_MIRROR>(acc);
    if (t == 0 && d < a.hd) {
        const int64_t o = ((int64_t)tq * a.H + h) * a.hd + d;
        a.out[(int64_t)b * a.obs + o] = (float)acc;
        if (a.out2) a.out2[(int64_t)b * a.n * a.H * a.hd + o] = (float)acc;
    }
}

// The same P.V with NPASS passes of 4 * NW output dims per workgroup (all hd dims of a (head, query,
// sequence) at NPASS = hd / 16): the softmax (P correctly rounded expf and an f64 sum) runs once per
// workgroup instead of once per 16 dims -- at 64 lock-step prompts the P.V grid otherwise evaluates
// every exponential hd / 16 = 4 times.  The work is a sequence of items (pass, 64 * UV positions): a
// lane's V slice of one item is one batch of UV 16-B loads, and the next item's batch is requested
// before the current one is summed (two register buffers), so any context length streams.  Each output
// dim is the same f64 sum in the same lane order as k_attn_pv (positions 4t + 64u, ascending u across
// items, then the DPP row reduction): bit-identical.
template <int UV, int NW, int NPASS>
__global__ __launch_bounds__(64 * NW) void k_attn_pv_mp(AttnArgs a, const float * __restrict__ sbuf, int pstride,
                                                       const float * __restrict__ mxbuf, int nch) {
    constexpr int NTH = 64 * NW;
    constexpr int KSTEP = 64 * UV;
    extern __shared__ __attribute__((aligned(16))) float s_p[];
    __shared__ double s_wd[NW];
    const int h = blockIdx.y, z = blockIdx.z;
    const int b = z / a.n, tq = z - b * a.n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane >> 4, t = lane & 15;
    const int P = seq_p(a, b);
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + seq_voff(a, b);
    const int64_t vnb1 = a.v.nb[1];
    const int ilast = ((P - 1) >> 2) << 2;
    const int d0 = blockIdx.x * 4 * NW * NPASS + wave * 4 + r;
    const int nck = (P + KSTEP - 1) / KSTEP;  // items per pass
    const int nit = NPASS * nck;
    float4 w4[2][UV];
    auto load_v = [&](auto BUF, int j) __attribute__((always_inline)) {
        constexpr int bf = decltype(BUF)::value;
        const int pass = j / nck, k0 = (j - pass * nck) * KSTEP;
        const char * vrow = vbase + (int64_t)min(d0 + pass * 4 * NW, a.hd - 1) * vnb1;
#pragma unroll
        for (int u = 0; u < UV; ++u) w4[bf][u] = TTS_KVLOAD((const float4 *)(vrow + 4 * (int64_t)min(k0 + 64 * u + 4 * t, ilast)));
    };
    load_v(std::integral_constant<int, 0>{}, 0);  // in flight during the softmax
    const float * srow = sbuf + ((int64_t)z * a.H + h) * pstride;
    const float * mrow = mxbuf + ((int64_t)z * a.H + h) * nch;
    float mx = -INFINITY;
    for (int k = 0; k < nch; ++k) mx = fmaxf(mx, mrow[k]);
    double sum = 0.0;
    for (int i = tid; i < P; i += NTH) {
        const float e = cr_expf(__fsub_rn(srow[i], mx));
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
    const int P64 = (P + 63) & ~63;
    for (int i = tid; i < P64; i += NTH) s_p[i] = i < P ? __fmul_rn(s_p[i], inv) : 0.f;
    __syncthreads();
    double acc = 0.0;
    auto item_sum = [&](auto BUF, int j) __attribute__((always_inline)) {
        constexpr int bf = decltype(BUF)::value;
        const int pass = j / nck, k0 = (j - pass * nck) * KSTEP;
#pragma unroll
        for (int u = 0; u < UV; ++u) {
            const int i = k0 + 64 * u + 4 * t;
            const float4 pp = *(const float4 *)(s_p + min(i, P64 - 4));
            const float4 vq = w4[bf][u];
            acc += i + 0 < P ? (double)__fmul_rn(pp.x, vq.x) : 0.0;
            acc += i + 1 < P ? (double)__fmul_rn(pp.y, vq.y) : 0.0;
            acc += i + 2 < P ? (double)__fmul_rn(pp.z, vq.z) : 0.0;
            acc += i + 3 < P ? (double)__fmul_rn(pp.w, vq.w) : 0.0;
        }
        if (k0 + KSTEP < P) return;  // the pass continues in the next item (uniform)
        acc += dpp_f64<DPP_XOR1>(acc);
        acc += dpp_f64<DPP_XOR2>(acc);
        acc += dpp_f64<DPP_HALF_MIRROR>(acc);
        acc += dpp_f64<DPP_MIRROR>(acc);
        const int d = d0 + pass * 4 * NW;
        if (t == 0 && d < a.hd) {
            const int64_t o = ((int64_t)tq * a.H + h) * a.hd + d;
            a.out[(int64_t)b * a.obs + o] = (float)acc;
            if (a.out2) a.out2[(int64_t)b * a.n * a.H * a.hd + o] = (float)acc;
        }
        acc = 0.0;
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    for (int j = 0; j < nit; j += 2) {
        if (j + 1 < nit) load_v(B1{}, j + 1);
        item_sum(B0{}, j);
        if (j + 1 >= nit) break;
        if (j + 2 < nit) load_v(B0{}, j + 2);
        item_sum(B1{}, j + 1);
    }
}

// ------------------------------------------------------------------------------------------
// Fused decode attention for long contexts: ONE launch per attention, one 1024-thread workgroup per
// (head, query, sequence).  The split pair above pays two launch ramps and an L2 round trip of the
// scores; here every byte of K and V is requested as early as registers allow:
//   A: 256 quads x KS positions per group, two groups in flight (the second requested before the
//      first is summed); kq[i] = f64 sum of f32 products over the quad's dims, finished by DPP;
//   V: the first UVC 16-B chunks of every lane's V row slice are requested as soon as A has finished
//      with its registers -- the softmax runs while they are in flight;
//   B: soft_max_ext over the P scores in LDS (the k_attn_decode_rows arithmetic);
//   C: 16 lanes per output dim, 64 dims per pass (DPR passes), lane t holds positions 4t + 64u in
//      ascending u, f64 accumulation and the DPP row reduction of k_attn_decode_rows: the same sums
//      in the same order, so the output is bit-identical to that kernel.
constexpr int FUSED_THREADS = 1024;
template <int DPR, int UVC>
__global__ __launch_bounds__(FUSED_THREADS) void k_attn_fused(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) float s_p[];  // (P rounded to 64) + 64 floats (launcher)
    __shared__ float s_wf[FUSED_THREADS / 64];
    __shared__ double s_wd[FUSED_THREADS / 64];
    constexpr int NW = FUSED_THREADS / 64;
    constexpr int F = 4 * DPR;   // float4 per lane per key position
    constexpr int KS = 3 - DPR;  // positions per quad per group (2 for hd 64, 1 for hd 128)
    constexpr int GP = 256 * KS; // positions per group
    const int h = blockIdx.x, tq = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane >> 4, t = lane & 15, qd = lane & 3;
    const int P = seq_p(a, b);
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * qbase = a.q.data + tq * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3] + seq_koff(a, b);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + seq_voff(a, b);
    const int64_t knb1 = a.k.nb[1], vnb1 = a.v.nb[1];
    const int pos0 = wave * 16 + (lane >> 2);

    float4 kv[2][KS][F];
    auto load_k = [&](auto BS, int i0) {
        constexpr int bs = decltype(BS)::value;
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            const int i = min(i0 + 256 * u + pos0, P - 1);
#pragma unroll
            for (int c = 0; c < F; ++c) kv[bs][u][c] = TTS_KVLOAD((const float4 *)(kbase + (int64_t)i * knb1 + 16 * (F * qd + c)));
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    load_k(I0{}, 0);
    float qv[F][4];
#pragma unroll
    for (int c = 0; c < F; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) qv[c][e] = ((const float *)qbase)[16 * DPR * qd + 4 * c + e];
    load_k(I1{}, min(GP, ((P - 1) / GP) * GP));
    TTS_PIN_LOADS();

    auto score = [&](auto BS, int i0) {
        constexpr int bs = decltype(BS)::value;
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < F; ++c) {
                s += (double)__fmul_rn(kv[bs][u][c].x, qv[c][0]);
                s += (double)__fmul_rn(kv[bs][u][c].y, qv[c][1]);
                s += (double)__fmul_rn(kv[bs][u][c].z, qv[c][2]);
                s += (double)__fmul_rn(kv[bs][u][c].w, qv[c][3]);
            }
            s += dpp_f64<DPP_XOR1>(s);
            s += dpp_f64<DPP_XOR2>(s);
            const int i = i0 + 256 * u + pos0;
            if (qd == 0 && i < P) s_p[i] = (float)s;
        }
    };
    // ---- A: groups g = 0, 1, 2, ...: group g + 1 is in flight while group g is summed ----
    for (int i0 = 0; i0 < P; i0 += 2 * GP) {
        score(I0{}, i0);
        if (i0 + 2 * GP < P) {
            load_k(I0{}, i0 + 2 * GP);
            TTS_PIN_LOADS();
        }
        if (i0 + GP >= P) break;
        score(I1{}, i0 + GP);
        if (i0 + 3 * GP < P) {
            load_k(I1{}, i0 + 3 * GP);
            TTS_PIN_LOADS();
        }
    }

    // ---- V: the first UVC chunks of pass 0 are requested before the softmax ----
    const int ilast = ((P - 1) >> 2) << 2;
    float4 w4[UVC];
    auto load_v = [&](int ps, int k0) {
        const char * vrow = vbase + (int64_t)min(ps * 64 + wave * 4 + r, a.hd - 1) * vnb1;
#pragma unroll
        for (int u = 0; u < UVC; ++u) w4[u] = TTS_KVLOAD((const float4 *)(vrow + 4 * (int64_t)min(k0 + 64 * u + 4 * t, ilast)));
    };
    load_v(0, 0);
    TTS_PIN_LOADS();
    __syncthreads();

    // ---- B: soft_max_ext ----
    const float * mrow = seq_mrow(a, b, tq, P);
    float mx = -INFINITY;
    for (int i = tid; i < P; i += FUSED_THREADS) {
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
    for (int i = tid; i < P; i += FUSED_THREADS) {
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
    const int P64 = (P + 63) & ~63;
    for (int i = tid; i < P64; i += FUSED_THREADS) s_p[i] = i < P ? __fmul_rn(s_p[i], inv) : 0.f;
    __syncthreads();

    // ---- C: out[d] = sum_i (f32)(p[i] * V[d,i]) in f64 ----
    float * orow = a.out + (int64_t)b * a.obs + ((int64_t)tq * a.H + h) * a.hd;
    float * orow2 = a.out2 ? a.out2 + (((int64_t)b * a.n + tq) * a.H + h) * a.hd : nullptr;
    constexpr int kstep = 64 * UVC;
#pragma unroll
    for (int ps = 0; ps < DPR; ++ps) {
        const int d = ps * 64 + wave * 4 + r;
        double acc = 0.0;
        for (int k0 = 0; k0 < P; k0 += kstep) {
            if (ps > 0 || k0 > 0) {
                load_v(ps, k0);
                TTS_PIN_LOADS();
            }
#pragma unroll
            for (int u = 0; u < UVC; ++u) {
                const int i = k0 + 64 * u + 4 * t;
                const float4 pp = *(const float4 *)(s_p + min(i, P64 - 4));
                const float4 vq = w4[u];
                acc += i + 0 < P ? (double)__fmul_rn(pp.x, vq.x) : 0.0;
                acc += i + 1 < P ? (double)__fmul_rn(pp.y, vq.y) : 0.0;
                acc += i + 2 < P ? (double)__fmul_rn(pp.z, vq.z) : 0.0;
                acc += i + 3 < P ? (double)__fmul_rn(pp.w, vq.w) : 0.0;
            }
        }
        acc += dpp_f64<DPP_XOR1>(acc);
        acc += dpp_f64<DPP_XOR2>(acc);
        acc += dpp_f64<DPP_HALF_MIRROR>(acc);
        acc += dpp_f64<DPP_MIRROR>(acc);
        if (t == 0 && d < a.hd) {
            orow[d] = (float)acc;
            if (orow2) orow2[d] = (float)acc;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Short contexts (P <= 64: Parler's cross-attention over the T5 prompt encoding, n_enc = 3; the
// first decode steps): one wave per (head, query, sequence), lane = key position, every sum in the
// oracle's sequential order -- the q.K dot over d, the soft_max denominator over positions (lane 0
// walks the lanes' exponentials), and each output dim over positions.  All of K, q and V are
// requested at entry; there is no LDS and no barrier.
template <int HD>
__global__ __launch_bounds__(64) void k_attn_small(AttnArgs a) {
    constexpr int F = HD / 4;
    const int h = blockIdx.x, tq = blockIdx.y, b = blockIdx.z;
    const int lane = threadIdx.x;
    const int P = seq_p(a, b);
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * qbase = a.q.data + tq * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3] + seq_koff(a, b);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + seq_voff(a, b);
    const int p = min(lane, P - 1);
    float4 kr[F];
#pragma unroll
    for (int c = 0; c < F; ++c) kr[c] = TTS_KVLOAD((const float4 *)(kbase + (int64_t)p * a.k.nb[1] + 16 * c));
    float qv[HD];
#pragma unroll
    for (int d = 0; d < HD; ++d) qv[d] = *(const float *)(qbase + (int64_t)d * a.q.nb[0]);
    // V positions per batch, per output dim; two batches in flight (the next one is requested before
    // the current one is summed; loads are clamped, never guarded, so the wait counts stay exact)
    constexpr int VB = 16;
    float vv[2][HD / 64][VB];
    auto load_v = [&](auto BS, int i0) {
        constexpr int bs = decltype(BS)::value;
#pragma unroll
        for (int j = 0; j < HD / 64; ++j)
#pragma unroll
            for (int u = 0; u < VB; ++u)
                vv[bs][j][u] = *(const float *)(vbase + (int64_t)(lane + 64 * j) * a.v.nb[1] + (int64_t)min(i0 + u, P - 1) * a.v.nb[0]);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    load_v(I0{}, 0);
    TTS_PIN_LOADS();
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < F; ++c) {
        acc += (double)__fmul_rn(kr[c].x, qv[4 * c + 0]);
        acc += (double)__fmul_rn(kr[c].y, qv[4 * c + 1]);
        acc += (double)__fmul_rn(kr[c].z, qv[4 * c + 2]);
        acc += (double)__fmul_rn(kr[c].w, qv[4 * c + 3]);
    }
    float w = __fmul_rn((float)acc, a.scale);
    if (a.mask) w = __fadd_rn(w, __fmul_rn(1.0f, seq_mrow(a, b, tq, P)[p]));
    if (lane >= P) w = -INFINITY;
    float mx = w;
    mx = fmaxf(mx, dpp_f32<DPP_XOR1>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_XOR2>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_HALF_MIRROR>(mx));
    mx = fmaxf(mx, dpp_f32<DPP_MIRROR>(mx));
    mx = fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 0)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 32)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 48))));
    const float e = lane < P ? cr_expf(__fsub_rn(w, mx)) : 0.f;
    double sum = 0.0;
    for (int i = 0; i < P; ++i) sum += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), i));
    const float pr = __fmul_rn(e, (float)(1.0 / sum));
    double o[HD / 64];
#pragma unroll
    for (int j = 0; j < HD / 64; ++j) o[j] = 0.0;
    auto consume = [&](auto BS, int i0) {
        constexpr int bs = decltype(BS)::value;
#pragma unroll
        for (int u = 0; u < VB; ++u) {
            if (i0 + u >= P) break;
            const float pi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), i0 + u));
#pragma unroll
            for (int j = 0; j < HD / 64; ++j) o[j] += (double)__fmul_rn(pi, vv[bs][j][u]);
        }
    };
    for (int i0 = 0; i0 < P; i0 += 2 * VB) {
        load_v(I1{}, i0 + VB);
        TTS_PIN_LOADS();
        consume(I0{}, i0);
        if (i0 + VB >= P) break;
        load_v(I0{}, i0 + 2 * VB);
        TTS_PIN_LOADS();
        consume(I1{}, i0 + VB);
    }
    const int64_t orow = ((int64_t)tq * a.H + h) * a.hd;
#pragma unroll
    for (int j = 0; j < HD / 64; ++j) {
        a.out[(int64_t)b * a.obs + orow + lane + 64 * j] = (float)o[j];
        if (a.out2) a.out2[(int64_t)b * a.n * a.H * a.hd + orow + lane + 64 * j] = (float)o[j];
    }
}

// ------------------------------------------------------------------------------------------
// Short contexts with many queries (a prompt pass: Parler's self-attention over the prompt and its
// cross-attention over the T5 encoding, n = 8-18 queries per sequence): k_attn_small's arithmetic
// per (head, query, sequence), but one workgroup per (head, sequence) stages K and V into LDS once
// (rows padded off the bank period) and its 16 waves take the queries in turn.  k_attn_small
// gives every query its own wave, which re-reads the (head, sequence)'s V with one scalar load per
// (dim, position) across 64 rows.  The sums are k_attn_small's, in its order: bit-identical.
constexpr int ATTN_SQ_WAVES = 16;  // waves per (head, sequence) workgroup of k_attn_small_q: one or two queries each
template <int HD>
__global__ __launch_bounds__(64 * ATTN_SQ_WAVES) void k_attn_small_q(AttnArgs a) {
    constexpr int NW = ATTN_SQ_WAVES;
    constexpr int KP = HD + 1;  // floats per K row in LDS
    constexpr int VP = 65;      // floats per V row (dim) in LDS: positions 0..63
    __shared__ float sk[64 * KP];
    __shared__ float sv[HD * VP];
    const int h = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = seq_p(a, b);
    const int hk = h / (a.H / (int)a.k.ne[2]);
    const int bk = b / (a.B / (int)a.k.ne[3]);
    const int hv = h / (a.H / (int)a.v.ne[2]);
    const int bv = b / (a.B / (int)a.v.ne[3]);
    const char * kbase = a.k.data + (int64_t)hk * a.k.nb[2] + (int64_t)bk * a.k.nb[3] + seq_koff(a, b);
    const char * vbase = a.v.data + (int64_t)hv * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + seq_voff(a, b);
    const int64_t knb1 = a.k.nb[1], vnb0 = a.v.nb[0], vnb1 = a.v.nb[1];
    for (int i = tid; i < P * HD; i += 64 * NW) {  // K [p][d] (d contiguous in memory)
        const int p = i / HD, d = i - p * HD;
        sk[p * KP + d] = *(const float *)(kbase + (int64_t)p * knb1 + 4 * d);
    }
    for (int i = tid; i < P * HD; i += 64 * NW) {  // V [d][p]
        const int d = i / P, p = i - d * P;
        sv[d * VP + p] = *(const float *)(vbase + (int64_t)d * vnb1 + (int64_t)p * vnb0);
    }
    __syncthreads();
    const int p = min(lane, P - 1);
    for (int tq = wave; tq < a.n; tq += NW) {
        const char * qbase = a.q.data + tq * a.q.nb[1] + (int64_t)h * a.q.nb[2] + (int64_t)b * a.q.nb[3];
        double acc = 0.0;
#pragma unroll 16
        for (int d = 0; d < HD; ++d) acc += (double)__fmul_rn(sk[p * KP + d], *(const float *)(qbase + (int64_t)d * a.q.nb[0]));
        float w = __fmul_rn((float)acc, a.scale);
        if (a.mask) w = __fadd_rn(w, __fmul_rn(1.0f, seq_mrow(a, b, tq, P)[p]));
        if (lane >= P) w = -INFINITY;
        float mx = w;
        mx = fmaxf(mx, dpp_f32<DPP_XOR1>(mx));
        mx = fmaxf(mx, dpp_f32<DPP_XOR2>(mx));
        mx = fmaxf(mx, dpp_f32<DPP_HALF_MIRROR>(mx));
        mx = fmaxf(mx, dpp_f32<DPP_MIRROR>(mx));
        mx = fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 0)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 16))),
                   fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 32)), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 48))));
        const float e = lane < P ? cr_expf(__fsub_rn(w, mx)) : 0.f;
        double sum = 0.0;
        for (int i = 0; i < P; ++i) sum += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), i));
        const float pr = __fmul_rn(e, (float)(1.0 / sum));
        double o[HD / 64];
#pragma unroll
        for (int j = 0; j < HD / 64; ++j) o[j] = 0.0;
        for (int i = 0; i < P; ++i) {
            const float pi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), i));
#pragma unroll
            for (int j = 0; j < HD / 64; ++j) o[j] += (double)__fmul_rn(pi, sv[(lane + 64 * j) * VP + i]);
        }
        const int64_t orow = ((int64_t)tq * a.H + h) * a.hd;
#pragma unroll
        for (int j = 0; j < HD / 64; ++j) {
            a.out[(int64_t)b * a.obs + orow + lane + 64 * j] = (float)o[j];
            if (a.out2) a.out2[(int64_t)b * a.n * a.H * a.hd + orow + lane + 64 * j] = (float)o[j];
        }
    }
}

// ------------------------------------------------------------------------------------------
// KV prefetch into the memory-side Infinity Cache (MALL).  Decode attention streams the whole KV
// cache of a layer once per step (Parler B = 8, P = 900: 59 MB); cold from HBM the row kernel
// reaches about half the bandwidth it gets from MALL-resident data, while the GEMVs between two
// attentions are latency-bound and leave HBM idle.  This kernel reads the K or V view of the NEXT
// attention on a side stream during those GEMVs; the attention then hits the 256 MB MALL.  The
// position written in this step (index P-1 along `pdim`) is never touched, so no cache level can
// hold a stale copy of it; the rest of the cache was written by earlier steps.
__global__ __launch_bounds__(256) void k_kv_prefetch(const char * __restrict__ base, int64_t n1, int64_t nb1, int64_t n2, int64_t nb2,
                                                    int64_t n3, int64_t nb3, int cpr, unsigned * sink) {
    const int64_t total = n1 * n2 * n3 * cpr;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (int64_t c0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c0 < total; c0 += 4 * gs) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t c = min(c0 + u * gs, total - 1);
            const int64_t r = c / cpr, k = c - r * cpr;
            const int64_t i1 = r % n1, t = r / n1;
            const int64_t i2 = t % n2, i3 = t / n2;
            v[u] = *(const uint4 *)(base + i1 * nb1 + i2 * nb2 + i3 * nb3 + 16 * k);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x9E3779B9u && sink) *sink = acc;  // keeps the loads; practically never stores
}

// K view [hd, P, Hk, Bk] (pdim 1) or V view [P, hd, Hv, Bv] (pdim 0), f32, nb[0] == 4.
void launch_kv_prefetch(tts_hip_backend * be, hipStream_t st, const TD & t, int pdim, int blocks) {
    if (t.nb[0] != 4 || ((uintptr_t)t.data) % 16) return;
    const int64_t P = t.ne[pdim];
    if (P < 2) return;
    int64_t n1 = t.ne[1], row_bytes = t.ne[0] * 4;
    if (pdim == 1) n1 = P - 1;
    else row_bytes = (P - 1) * 4;
    const int cpr = (int)(row_bytes / 16);  // whole 16-B chunks only (never the chunk holding P-1)
    if (cpr <= 0 || (t.nb[1] % 16) || (t.nb[2] % 16) || (t.nb[3] % 16)) return;
    hipLaunchKernelGGL(k_kv_prefetch, dim3((unsigned)blocks), dim3(256), 0, st, (const char *)t.data, n1, (int64_t)t.nb[1],
                       t.ne[2], (int64_t)t.nb[2], t.ne[3], (int64_t)t.nb[3], cpr, (unsigned *)nullptr);
}

void launch_attn_decode(tts_hip_backend * be, const TD & q, const TD & k, const TD & v, const float * mask, float scale,
                        float * out, int hd, int P, int H, int n, int B, float * out2, int64_t obs, int64_t mbs, const int64_t * koff,
                        const int64_t * voff, const int64_t * moff, const int * pseq) {
    AttnArgs a;
    a.koff = koff;
    a.voff = voff;
    a.moff = moff;
    a.pseq = pseq;
    a.out2 = out2;
    a.obs = obs >= 0 ? obs : (int64_t)n * H * hd;
    a.mbs = mbs;
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
    // row kernel: hd = 64/128, K rows 16-B vectors (aligned base and row stride)
    const bool krows = (hd == 64 || hd == 128) && k.nb[0] == 4 && (k.nb[1] % 16) == 0 &&
                       (((uintptr_t)k.data) % 16) == 0 && (k.nb[2] % 16) == 0 &&
                       (k.nb[3] % 16) == 0 && q.nb[0] == 4 && P > 0;
    if (krows && P <= 64 && n >= 4) {  // a prompt pass: K / V staged once per (head, sequence)
        const dim3 grid((unsigned)H, (unsigned)B);
        if (hd == 64) hipLaunchKernelGGL(k_attn_small_q<64>, grid, dim3(64 * ATTN_SQ_WAVES), 0, be->stream, a);
        else hipLaunchKernelGGL(k_attn_small_q<128>, grid, dim3(64 * ATTN_SQ_WAVES), 0, be->stream, a);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    if (krows && P <= 64) {
        const dim3 grid((unsigned)H, (unsigned)n, (unsigned)B);
        if (hd == 64) hipLaunchKernelGGL(k_attn_small<64>, grid, dim3(64), 0, be->stream, a);
        else hipLaunchKernelGGL(k_attn_small<128>, grid, dim3(64), 0, be->stream, a);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    const bool vvec_all = v.nb[0] == 4 && (v.nb[1] % 16) == 0 && (v.nb[2] % 16) == 0 && (v.nb[3] % 16) == 0 &&
                          (((uintptr_t)v.data) % 16) == 0 && v.nb[1] >= (size_t)16 * ((P + 3) / 4);
    if (krows && vvec_all && be->attn_fused_minp > 0 && P >= be->attn_fused_minp && P <= ATTN_MAXP) {
        const dim3 grid((unsigned)H, (unsigned)n, (unsigned)B);
        const size_t pl = (size_t)(((P + 63) & ~63) + 64) * sizeof(float);
        if (hd == 64) hipLaunchKernelGGL((k_attn_fused<1, 8>), grid, dim3(FUSED_THREADS), pl, be->stream, a);
        else hipLaunchKernelGGL((k_attn_fused<2, 8>), grid, dim3(FUSED_THREADS), pl, be->stream, a);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    if (krows && be->attn_split_minp > 0 && P >= be->attn_split_minp && P <= ATTN_MAXP && hd % 16 == 0) {
        const int KS = be->attn_ks == 1 ? 1 : be->attn_ks == 4 ? 4 : 2;  // 128 * KS positions per scores workgroup
        const int nch = (P + 128 * KS - 1) / (128 * KS);
        const int pstride = (P + 63) & ~63;
        const size_t rows = (size_t)H * n * B;
        if (rows * ((size_t)pstride + nch) <= be->attn_floats) {
            float * sbuf = be->attn_buf;
            float * mxbuf = be->attn_buf + rows * pstride;
            const dim3 g1((unsigned)nch, (unsigned)H, (unsigned)(n * B));
            // profiled (TTS_HIP_OPT_PROFILE_GEMV): the pair's start / stop events ride in the two dispatch
            // packets, bytes = every K and V row read + q + the output
            hipEvent_t e0 = nullptr, e1 = nullptr;
            if (be->profile_gemv) profile_pair(be, e0, e1);
            auto scores = [&](auto DPR, auto KSc) {
                hipExtLaunchKernelGGL((k_attn_scores<decltype(DPR)::value, decltype(KSc)::value>), g1, dim3(ATTN_THREADS), 0, be->stream, e0,
                                      nullptr, 0u, a, sbuf, pstride, mxbuf, nch);
            };
            using C1 = std::integral_constant<int, 1>;
            using C2 = std::integral_constant<int, 2>;
            using C4 = std::integral_constant<int, 4>;
            if (hd == 64) KS == 1 ? scores(C1{}, C1{}) : KS == 4 ? scores(C1{}, C4{}) : scores(C1{}, C2{});
            else KS == 1 ? scores(C2{}, C1{}) : KS == 4 ? scores(C2{}, C4{}) : scores(C2{}, C2{});
            TTS_HIP_CHECK(hipGetLastError());
            const bool vvec = v.nb[0] == 4 && (v.nb[1] % 16) == 0 && (v.nb[2] % 16) == 0 && (v.nb[3] % 16) == 0 &&
                              (((uintptr_t)v.data) % 16) == 0 && v.nb[1] >= (size_t)16 * ((P + 3) / 4);
            const dim3 g2((unsigned)(hd / 16), (unsigned)H, (unsigned)(n * B));
            const dim3 g2h((unsigned)(hd / 8), (unsigned)H, (unsigned)(n * B));  // 8 dims per workgroup
            // P <= 1024: every lane's whole V slice (16 x 16 B) is requested before the softmax
            const uint32_t pl = (uint32_t)((((P + 63) & ~63) + 64) * sizeof(float));  // s_p
            // all dims of a (head, query, seq) per workgroup: one workgroup per row, so past 512 keys only
            // when the rows alone fill the chip (Dia's 1024-position cross-attention has 32 rows: 8 dims
            // per workgroup keeps 256 workgroups streaming V)
            if (vvec && be->attn_pv_mp && (hd == 64 || hd == 128) && (P <= 512 || rows >= (size_t)be->cus)) {
                const dim3 g3(1u, (unsigned)H, (unsigned)(n * B));
                // TTS_HIP_OPT_ATTN_PV_MP = 2: eight waves per workgroup (half the passes; same sums)
                if (be->attn_pv_mp == 2) {
                    if (hd == 64) hipExtLaunchKernelGGL((k_attn_pv_mp<8, 8, 2>), g3, dim3(512), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
                    else hipExtLaunchKernelGGL((k_attn_pv_mp<8, 8, 4>), g3, dim3(512), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
                } else if (hd == 64) {
                    hipExtLaunchKernelGGL((k_attn_pv_mp<8, 4, 4>), g3, dim3(256), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
                } else {
                    hipExtLaunchKernelGGL((k_attn_pv_mp<8, 4, 8>), g3, dim3(256), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
                }
            } else if (vvec && P <= 1024 && be->attn_pv_uv16)
                hipExtLaunchKernelGGL((k_attn_pv<true, 16>), g2, dim3(PV_THREADS), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
            else if (vvec && be->attn_pv8)
                hipExtLaunchKernelGGL((k_attn_pv<true, 8, 2>), g2h, dim3(128), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
            else if (vvec) hipExtLaunchKernelGGL((k_attn_pv<true, 8>), g2, dim3(PV_THREADS), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
            else hipExtLaunchKernelGGL((k_attn_pv<false, 8>), g2, dim3(PV_THREADS), pl, be->stream, nullptr, e1, 0u, a, sbuf, pstride, mxbuf, nch);
            TTS_HIP_CHECK(hipGetLastError());
            if (be->profile_gemv)
                profile_push(be, e0, e1, (double)rows * (2.0 * P * hd + 2.0 * hd) * 4.0, TTS_PROF_ATTN);
            return;
        }
    }
    if (krows) {
        const bool vvec = v.nb[0] == 4 && (v.nb[1] % 16) == 0 && (v.nb[2] % 16) == 0 && (v.nb[3] % 16) == 0 &&
                          (((uintptr_t)v.data) % 16) == 0 && v.nb[1] >= (size_t)16 * ((P + 3) / 4);
        // PF: the whole V slice fits the registers of one pass (16 x 16-B or 16 scalar loads per lane)
        const bool pf = hd == 64 && P <= (vvec ? 64 * 8 : 16 * 8);
        // (a 16-chunk prefetch covering P <= 1024 measured slower than streaming V: 20.3 vs 16.7 us)
        if (hd == 64 && pf) launch_attn_rows<1, true>(be, a, vvec);
        else if (hd == 64) launch_attn_rows<1, false>(be, a, vvec);
        else launch_attn_rows<2, false>(be, a, vvec);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    hipLaunchKernelGGL(k_attn_decode, dim3((unsigned)H, (unsigned)n, (unsigned)B), dim3(ATTN_THREADS), 0, be->stream, a);
    TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
