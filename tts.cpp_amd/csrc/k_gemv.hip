// Quantized decode GEMV for gfx950: y = W x with W in Q4_K / Q8_0 / F16 / F32, M <= 8 columns.
//
// Replaces GGML_OP_MUL_MAT at every decode site (Parler model.cpp:544-546,571,583,594,601,603;
// Dia model.cpp:535-537,...; Orpheus model.cpp:254-256,...).
//
// Numerics are ggml-cpu's generic scalar paths, bit for bit: the activation column is quantized to
// the weight type's vec_dot_type (Q8_K for Q4_K, Q8_0 for Q8_0, F16 for F16) with the exact
// quantize_row_*_ref arithmetic, the per-block integer dot products are exact (v_dot4_i32_i8), and
// the f32 combination follows vec_dot_*'s order exactly.  F32/F16 dots take f32 products and
// accumulate them in f64, as ggml_vec_dot_f32/f16 do (tests/test_gemv_gpu.py: bit-exact).
//
// Memory shape (HBM-bound): weights stream once with 16-B non-temporal loads; the activation of a
// launch is staged in LDS per workgroup (Q4_K: quantized in-kernel, optionally after LayerNorm).
#include "hip_internal.h"
#include <hip/hip_ext.h>

#include <atomic>
#include <type_traits>

#ifndef TTS_GEMV_EARLY16
#define TTS_GEMV_EARLY16 1  // long rows (K > 1024) also issue their first weight loads before a quantize-only prologue
                            // (the LN prologue holds a whole column in registers: those would spill)
#endif

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

// get_scale_min_k4: 6-bit scale and min of sub-block j from the 12 packed bytes
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

// XCD-contiguous workgroup order: the dispatcher hands workgroup b to XCD b % 8, so consecutive
// workgroups -- and the rows they own -- land on different XCDs and every XCD's L2 fetches the 128-B
// lines two neighbouring 576-B Q4_K rows share.  Renumbering b so that XCD x's workgroups take one
// contiguous span (prefix(x) + b / 8, a bijection on [0, n)) leaves one shared line per XCD boundary.
// The arithmetic per (row, column) is untouched.
__device__ __forceinline__ int xcd_contiguous(int b, int n) {
    const int x = b & 7, q = n >> 3, r = n & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// A kernel argument indexed by a matrix index the compiler cannot prove wave-uniform compiles to a
// VECTOR load of the kernarg segment, and the s_waitcnt vmcnt(0) that guards its use also waits for
// every weight and activation load already in flight (it serialised a GEMV's first weight loads
// behind its prologue's activation loads).  Callers pass indices that are uniform by construction
// through readfirstlane, and single-matrix jobs index 0.

template <int MC>
__device__ __forceinline__ void gemv_store(const GemvJob & j, int mat, int64_t row, int m, float v) {
    if (j.epi == EPI_GELU) {
        if (v <= -10.0f) v = 0.0f;
        else if (v < 10.0f) v = __half2float(__ushort_as_half(j.gelu[__half_as_ushort(__float2half_rn(v))]));
    } else if (j.epi == EPI_ADD) {
        v = __fadd_rn(v, j.res[m * j.rcs + row]);
    } else if (j.epi == EPI_SILU_MUL) {
        v = __fmul_rn(dev_silu(j.res[m * j.rcs + row]), v);
    }
    float * const Y = j.Y[mat] + ((j.yoff_mats >> mat) & 1 ? j.yoff[mat * j.yoff_ld + m] : 0);
    const int64_t ycs = j.ycs[mat], yrs = j.yrs[mat];
    if (mat == j.rep_mat) {
        const int64_t g = row / j.yrg;
        float * y = Y + m * ycs + g * j.yrgs + (row - g * j.yrg) * yrs;
        for (int k = 0; k < j.nrep; ++k) y[k * j.yrep] = v;
        return;
    }
    Y[m * ycs + row * yrs] = v;
}

// quantize_row_q8_K_ref for four 256-element blocks per wave: the 16-lane row r = lane >> 4 owns
// one block, lane t = lane & 15 its elements 16t..16t+15.  max |x| at its first index (strict '>'
// from 0, as ggml), iscale = -127/x[imax], q = min(127, nearest_int(iscale*x)), d = 1/iscale.
// Writes the lane-major LDS layout (element p = 64c + 32hi + 8k + l at byte l*32 + hi*16 + c*4 + k;
// elements 16t+e and 16t+e+8 are adjacent bytes), d and the eight per-32 sums as int16.  All
// reductions stay inside the row (DPP); the code is branch-free so the compiler can interleave it
// with neighbouring work.
__device__ __forceinline__ void q8k_quant16(const float (&v)[16], int lane, int (&q)[16], float & d, int & s) {
    float lax = 0.f, lval = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const float a = fabsf(v[e]);
        const bool gt = a > lax;
        lax = gt ? a : lax;
        lval = gt ? v[e] : lval;
    }
    unsigned mx = __float_as_uint(lax);  // non-negative floats order as their bit patterns
    mx = max(mx, (unsigned)dpp_i32<DPP_XOR1>((int)mx));
    mx = max(mx, (unsigned)dpp_i32<DPP_XOR2>((int)mx));
    mx = max(mx, (unsigned)dpp_i32<DPP_HALF_MIRROR>((int)mx));
    mx = max(mx, (unsigned)dpp_i32<DPP_MIRROR>((int)mx));
    const float ax = __uint_as_float(mx);
    const unsigned long long hit = __ballot(lax == ax);
    const unsigned rowbits = (unsigned)(hit >> (lane & 48)) & 0xFFFFu;
    const float val = __shfl(lval, (lane & 48) + (rowbits ? __ffs(rowbits) - 1 : 0));
    const bool nz = ax != 0.f;
    const float iscale = nz ? cr_divf(-127.f, val) : 0.f;  // iscale 0 quantizes everything to 0
    d = nz ? cr_divf(1.f, iscale) : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) q[e] = min(dev_nearest_int(__fmul_rn(iscale, v[e])), 127);
    s = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) s += q[e];
    s += dpp_i32<DPP_XOR1>(s);  // elements 32j..32j+31 = lanes 2j, 2j+1
}

__device__ __forceinline__ void q8k_row_block(const float (&v)[16], int lane, int8_t * xq, float * xd, int16_t * xs) {
    const int t = lane & 15;
    int q[16], s;
    float d;
    q8k_quant16(v, lane, q, d, s);
    const int base = ((t >> 1) & 1) * 16 + (t >> 2) * 4 + ((2 * t) & 3);
#pragma unroll
    for (int e = 0; e < 8; ++e)
        *(int16_t *)(xq + e * 32 + base) = (int16_t)((q[e] & 0xFF) | ((q[e + 8] & 0xFF) << 8));
    if ((t & 1) == 0) xs[t >> 1] = (int16_t)s;
    if (t == 0) *xd = d;
}

// The same Q8_K block written as the MFMA kernel's B operands (k_gemv_q4K_mf): f16 values (exact:
// |q| <= 127) at b16[(l*4 + c)*8 + 4h + kk] for element 64c + 32h + 8kk + l, and the per-32 sums
// split as bsum = 64*hi + lo (lo in [0, 63], both exact in f16) at sb[e] = lo_e, sb[8 + e] = hi_e.
__device__ __forceinline__ void q8k_row_block_mf(const float (&v)[16], int lane, _Float16 * b16, _Float16 * sb, float * xd) {
    const int t = lane & 15;
    int q[16], s;
    float d;
    q8k_quant16(v, lane, q, d, s);
    // lane t holds elements 16t + e: c = t >> 2, h = (t >> 1) & 1, kk = 2(t & 1) + (e >> 3), l = e & 7
    const int base = (t >> 2) * 8 + ((t >> 1) & 1) * 4 + 2 * (t & 1);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        h2 pr;
        pr.x = (_Float16)q[l];
        pr.y = (_Float16)q[l + 8];
        *(h2 *)(b16 + l * 32 + base) = pr;
    }
    if ((t & 1) == 0) {
        const int hi = s >> 6, lo = s - 64 * hi;  // arithmetic shift: floor(s / 64)
        sb[t >> 1] = (_Float16)lo;
        sb[8 + (t >> 1)] = (_Float16)hi;
    }
    if (t == 0) *xd = d;
}

// quantize_row_q8_0 (k_quantize_q8_0's arithmetic) of the 16 elements a lane holds: lanes 2k and 2k+1
// hold one 32-element block (amax by DPP over the pair); int8 values to xq (elements 16t .. 16t+15 of
// the 256-element chunk), the fp16-rounded d of block t/2 to xd[t/2].
__device__ __forceinline__ void q80_row_block(const float (&v)[16], int lane, int8_t * xq, float * xd) {
    const int t = lane & 15;
    float a = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) a = fmaxf(a, fabsf(v[e]));
    a = fmaxf(a, dpp_f32<DPP_XOR1>(a));
    const float d = cr_divf(a, 127.f);
    const float id = d != 0.f ? cr_divf(1.f, d) : 0.f;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t u = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) u |= ((uint32_t)(int)roundf(__fmul_rn(v[4 * k + e], id)) & 0xFFu) << (8 * e);
        w[k] = u;
    }
    *(uint4 *)(xq + 16 * t) = make_uint4(w[0], w[1], w[2], w[3]);
    if ((t & 1) == 0) xd[t >> 1] = __half2float(__float2half_rn(d));
}

// Loads are unconditional (addresses clamped into range) so that a wave issues all of them before
// the first use: a load under a guard is sunk next to its use, and every block then pays a full
// L2 round trip (measured: 0.4 us per block).  The launcher guarantees 16-B aligned x / lnw / lnb
// and 16-B aligned column strides.
__device__ __forceinline__ void ld4(const float * p, float (&v)[4]) {
    const f32x4 t = *gptr((const f32x4 *)p);
    v[0] = t.x, v[1] = t.y, v[2] = t.z, v[3] = t.w;
}

// Prologue: the Q8_K activation of all M columns into LDS, optionally after LayerNorm / RMSNorm
// with affine (ggml_compute_forward_norm_f32 / rms_norm_f32: f64 sums, mean and variance rounded
// to f32, scale = 1/sqrtf(var + eps), then MUL(w) and ADD(b) each rounded).
// MF: write the MFMA kernel's f16 operand layout (q8k_row_block_mf into mf_b16 / mf_sb) instead.
// `mid` runs once per wave right after that wave's first activation loads are issued and before any
// of them is used: callers issue their weight loads there.  Vector loads complete in issue order,
// so activation loads queued behind a row of HBM weight loads would make the prologue wait for the
// weights; issued first, they return from L2 / MALL while the weights are still in flight.
struct NoMid {
    __device__ void operator()() const {}
};
// Per-call overrides of the prologue (defaults: the whole workgroup, j.x's M columns, LDS slots from 0)
struct ProOv {
    int nwaves = 0;               // waves taking part (0 = the whole workgroup)
    const float * xcol = nullptr; // quantize this single column instead of j.x's M columns ...
    float * lncol = nullptr;      // ... and write its LN output here (or nowhere)
    int slot0 = 0;                // first output slot
    int trash = -1;               // slot absorbing padding writes (-1: M * nb)
    int col0 = 0;                 // a column tile: j.x's columns col0 .. col0 + mcols - 1 (LN output likewise)
    int mcols = 0;                // (0: j.M columns from col0)
};
template <int PRO, int NCH, bool MF = false, typename Mid = NoMid, bool Q80 = false>
__device__ __forceinline__ void q4k_prologue(const GemvJob & j, int nb, int8_t * xq_s, float * xd_s, int16_t * xs_s,
                                             _Float16 * mf_b16 = nullptr, _Float16 * mf_sb = nullptr, Mid mid = Mid{},
                                             ProOv ov = ProOv{}) {
    // ov.xcol: quantize one column instead of j.x's M columns.  Overriding fields here instead of
    // copying the job keeps every pointer a kernel argument, so the compiler keeps them in the global
    // address space (a copied job's pointers turned into flat loads, which complete out of order and
    // make every later wait a vmcnt(0))
    const int nwaves = ov.nwaves;
    const float * const xcol = ov.xcol;
    float * const lncol = ov.lncol;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = nwaves ? nwaves : blockDim.x >> 6;
    const int r = lane >> 4, t = lane & 15;
    const int M = xcol ? 1 : ov.mcols > 0 ? ov.mcols : (int)j.M;
    const float * const X = xcol ? xcol : j.x + (int64_t)ov.col0 * j.xcs;
    const int64_t xcs = xcol ? 0 : j.xcs;  // (one column: xcol)
    const int trash = M * nb;  // LDS slot that absorbs the writes of padding rows
    auto put = [&](const float (&v)[16], int lane, int slot) {
        slot = slot == trash ? (ov.trash >= 0 ? ov.trash : slot) : ov.slot0 + slot;
        if constexpr (Q80) q80_row_block(v, lane, xq_s + (int64_t)slot * QK_K, xd_s + (int64_t)slot * (QK_K / QK8_0));
        else if constexpr (MF) q8k_row_block_mf(v, lane, mf_b16 + (int64_t)slot * QK_K, mf_sb + slot * 16, xd_s + slot);
        else q8k_row_block(v, lane, xq_s + (int64_t)slot * QK_K, xd_s + slot, xs_s + slot * 8);
    };
    if (PRO == PRO_QUANT) {
        // pass p quantizes blocks 4p..4p+3 (block qb = column qb / nb, chunk qb % nb at x + column * xcs +
        // chunk * 256; columns contiguous or strided, e.g. a coalesced step's members)
        constexpr int QP = NCH <= 4 ? 2 : 4;  // passes whose loads a wave keeps in flight
        const int nq = M * nb, npass = (nq + 3) / 4;
        auto batch = [&](int p0, bool first) {
            float v[QP][16];
#pragma unroll
            for (int u = 0; u < QP; ++u) {
                const int qb = min(4 * min(p0 + u * nw, npass - 1) + r, nq - 1);
                const int mc = qb / nb;
                const float * src = X + (int64_t)mc * xcs + (int64_t)(qb - mc * nb) * QK_K + 16 * t;
#pragma unroll
                for (int k = 0; k < 4; ++k) ld4(src + 4 * k, *(float (*)[4]) & v[u][4 * k]);
            }
            TTS_PIN_LOADS();
            if (first) mid();
            TTS_PIN_LOADS();
#pragma unroll
            for (int u = 0; u < QP; ++u) {
                const int p = p0 + u * nw, qb = 4 * p + r;
                const int slot = (p < npass && qb < nq) ? qb : trash;
                put(v[u], lane, slot);
            }
        };
        // the first batch is peeled out of the loop: a loop header makes the compiler wait for every
        // outstanding load, including the weight loads issued before the prologue
        batch(wave, true);
        for (int p0 = wave + nw * QP; p0 < npass; p0 += nw * QP) batch(p0, false);
    } else {
        // one column per wave; pass p holds chunks 4p + r (K <= 4096: NP <= 4, host-checked).  For
        // K <= 1024 the affine parameters are loaded with x, so the prologue pays one L2 round trip.
        constexpr int NP = (NCH + 3) / 4;
        constexpr bool PRE = NCH <= 4;
        const double Kd = (double)j.K;
        float * const lno = xcol ? lncol : j.lnout ? j.lnout + (int64_t)ov.col0 * j.locs : nullptr;
        const bool write = lno && (xcol || blockIdx.x == 0);
        const float * lnb = j.lnb ? j.lnb : j.lnw;
        float wp[PRE ? NP : 1][16], bp[PRE ? NP : 1][16];
        if (PRE) {
#pragma unroll
            for (int p = 0; p < (PRE ? NP : 1); ++p) {
                const int off = min(4 * p + r, nb - 1) * QK_K + 16 * t;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    ld4(j.lnw + off + 4 * k, *(float (*)[4]) & wp[p][4 * k]);
                    ld4(lnb + off + 4 * k, *(float (*)[4]) & bp[p][4 * k]);
                }
            }
        }
        auto column = [&](int m, bool first, bool live = true) {
            const float * xr = X + m * j.xcs;
            float v[NP][16];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const int off = min(4 * p + r, nb - 1) * QK_K + 16 * t;
#pragma unroll
                for (int k = 0; k < 4; ++k) ld4(xr + off + 4 * k, *(float (*)[4]) & v[p][4 * k]);
            }
            TTS_PIN_LOADS();
            if (first) mid();
            TTS_PIN_LOADS();
            float mean = 0.f;
            if (!j.rms) {
                double s = 0.0;
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    double sp = 0.0;
#pragma unroll
                    for (int e = 0; e < 16; ++e) sp += (double)v[p][e];
                    s += 4 * p + r < nb ? sp : 0.0;
                }
                mean = (float)(wave_sum_f64(s) / Kd);
            }
            double s2 = 0.0;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                double sp = 0.0;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const float d = j.rms ? v[p][e] : __fsub_rn(v[p][e], mean);
                    sp += (double)__fmul_rn(d, d);
                }
                s2 += 4 * p + r < nb ? sp : 0.0;
            }
            const float var = (float)(wave_sum_f64(s2) / Kd);
            const float scale = cr_divf(1.0f, cr_sqrtf(__fadd_rn(var, j.eps)));
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                float w16[16], b16[16];
                const int off = min(4 * p + r, nb - 1) * QK_K + 16 * t;
                if (PRE) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) w16[e] = wp[PRE ? p : 0][e], b16[e] = bp[PRE ? p : 0][e];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        ld4(j.lnw + off + 4 * k, *(float (*)[4]) & w16[4 * k]);
                        ld4(lnb + off + 4 * k, *(float (*)[4]) & b16[4 * k]);
                    }
                }
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    float y = j.rms ? __fmul_rn(v[p][e], scale) : __fmul_rn(__fsub_rn(v[p][e], mean), scale);
                    y = __fmul_rn(y, w16[e]);
                    if (j.lnb) y = __fadd_rn(y, b16[e]);
                    v[p][e] = y;
                }
                const bool valid = live && 4 * p + r < nb;
                if (write && valid) {
                    float * o = lno + m * j.locs + off;
#pragma unroll
                    for (int k = 0; k < 4; ++k) *(float4 *)(o + 4 * k) = make_float4(v[p][4 * k], v[p][4 * k + 1], v[p][4 * k + 2], v[p][4 * k + 3]);
                }
                const int slot = valid ? m * nb + 4 * p + r : trash;
                put(v[p], lane, slot);
            }
        };
        if (wave < M) column(wave, true);  // peeled, as above
        else mid();
        for (int m = wave + nw; m < M; m += nw) column(m, false);
    }
}

// One Q4_K block of one (row, column) for lane l of an octet: aux32[l] from eight sdot4 with the
// 6-bit scales, sumi from the mins and the per-32 Q8_K sums, then ggml's f32 combine
// sums[l] += d*yd*aux32[l], sumf -= dmin*yd*sumi (vec_dot_q4_K_q8_K generic order).  `xb` is the
// Q8_K block index in LDS; an invalid (padding) block leaves the accumulators unchanged.
// The block's two terms of that chain, p = (d*yd)*aux32[l] and q = (dmin*yd)*sumi, each rounded as
// ggml rounds them; q4k_block folds them in (sums += p, sumf -= q), the K-split kernel hands them to
// the wave that owns the chain.
__device__ __forceinline__ void q4k_block_pq(const u32x4 & h, const u32x4 & qw, const int8_t * xq_s, const int16_t * xs_s,
                                             const float * xd_s, int xb, int l, float & p, float & q);
__device__ __forceinline__ void q4k_block(const u32x4 & h, const u32x4 & qw, const int8_t * xq_s, const int16_t * xs_s,
                                          const float * xd_s, int xb, int l, bool valid, float & sums, float & sumf) {
    float p, q;
    q4k_block_pq(h, qw, xq_s, xs_s, xd_s, xb, l, p, q);
    const float ns = __fadd_rn(sums, p);
    const float nf = __fsub_rn(sumf, q);
    sums = valid ? ns : sums;
    sumf = valid ? nf : sumf;
}
__device__ __forceinline__ void q4k_block_pq(const u32x4 & h, const u32x4 & qw, const int8_t * xq_s, const int16_t * xs_s,
                                             const float * xd_s, int xb, int l, float & p, float & q) {
    const uint32_t A = h.y, B = h.z, C = h.w;
    // 6-bit scales / mins of the eight 32-element sub-blocks, four per word (get_scale_min_k4)
    const uint32_t sc_lo = A & 0x3F3F3F3Fu, mn_lo = B & 0x3F3F3F3Fu;
    const uint32_t sc_hi = (C & 0x0F0F0F0Fu) | ((A >> 2) & 0x30303030u);
    const uint32_t mn_hi = ((C >> 4) & 0x0F0F0F0Fu) | ((B >> 2) & 0x30303030u);
    const int4 xl = *(const int4 *)(xq_s + xb * QK_K + l * 32);
    const int4 xh = *(const int4 *)(xq_s + xb * QK_K + l * 32 + 16);
    const uint32_t w0 = qw.x, w1 = qw.y, w2 = qw.z, w3 = qw.w;
    // aux32[l] = sum_j scale_j * dot4_j; |dot4| <= 7620 and scale <= 63 fit the 24-bit multiplier
    int aux = __mul24((int)(sc_lo & 0xFF), __builtin_amdgcn_sdot4((int)(w0 & 0x0F0F0F0Fu), xl.x, 0, false));
    aux += __mul24((int)((sc_lo >> 8) & 0xFF), __builtin_amdgcn_sdot4((int)((w0 >> 4) & 0x0F0F0F0Fu), xh.x, 0, false));
    aux += __mul24((int)((sc_lo >> 16) & 0xFF), __builtin_amdgcn_sdot4((int)(w1 & 0x0F0F0F0Fu), xl.y, 0, false));
    aux += __mul24((int)(sc_lo >> 24), __builtin_amdgcn_sdot4((int)((w1 >> 4) & 0x0F0F0F0Fu), xh.y, 0, false));
    aux += __mul24((int)(sc_hi & 0xFF), __builtin_amdgcn_sdot4((int)(w2 & 0x0F0F0F0Fu), xl.z, 0, false));
    aux += __mul24((int)((sc_hi >> 8) & 0xFF), __builtin_amdgcn_sdot4((int)((w2 >> 4) & 0x0F0F0F0Fu), xh.z, 0, false));
    aux += __mul24((int)((sc_hi >> 16) & 0xFF), __builtin_amdgcn_sdot4((int)(w3 & 0x0F0F0F0Fu), xl.w, 0, false));
    aux += __mul24((int)(sc_hi >> 24), __builtin_amdgcn_sdot4((int)((w3 >> 4) & 0x0F0F0F0Fu), xh.w, 0, false));
    // sumi = sum_j mins[j] * bsum32[j] (int16 pairs, v_dot2)
    const int4 bs = *(const int4 *)(xs_s + xb * 8);
    const int mn01 = (int)((mn_lo & 0xFF) | ((mn_lo & 0xFF00) << 8));
    const int mn23 = (int)(((mn_lo >> 16) & 0xFF) | ((mn_lo >> 8) & 0xFF0000));
    const int mn45 = (int)((mn_hi & 0xFF) | ((mn_hi & 0xFF00) << 8));
    const int mn67 = (int)(((mn_hi >> 16) & 0xFF) | ((mn_hi >> 8) & 0xFF0000));
    int sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, mn01), __builtin_bit_cast(short2_t, bs.x), 0, false);
    sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, mn23), __builtin_bit_cast(short2_t, bs.y), sumi, false);
    sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, mn45), __builtin_bit_cast(short2_t, bs.z), sumi, false);
    sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, mn67), __builtin_bit_cast(short2_t, bs.w), sumi, false);
    const float yd = xd_s[xb];
    const float dw = dev_fp16_to_fp32((uint16_t)(h.x & 0xFFFF));
    const float dmw = dev_fp16_to_fp32((uint16_t)(h.x >> 16));
    p = __fmul_rn(__fmul_rn(dw, yd), (float)aux);
    q = __fmul_rn(__fmul_rn(dmw, yd), (float)sumi);
}

// sumf += sums[0..7] in order; lane l = 0 of the octet reads lane l = k by row_shl:k
__device__ __forceinline__ float q4k_octet_total(float sumf, float sums) {
    float tot = __fadd_rn(sumf, sums);
    tot = __fadd_rn(tot, dpp_f32<DPP_ROW_SHL0 + 1>(sums));
    tot = __fadd_rn(tot, dpp_f32<DPP_ROW_SHL0 + 2>(sums));
    tot = __fadd_rn(tot, dpp_f32<DPP_ROW_SHL0 + 3>(sums));
    tot = __fadd_rn(tot, dpp_f32<DPP_ROW_SHL0 + 4>(sums));
    tot = __fadd_rn(tot, dpp_f32<DPP_ROW_SHL0 + 5>(sums));
    tot = __fadd_rn(tot, dpp_f32<DPP_ROW_SHL0 + 6>(sums));
    tot = __fadd_rn(tot, dpp_f32<DPP_ROW_SHL0 + 7>(sums));
    return tot;
}

// ------------------------------------------------------------------------------------------
// Q4_K x Q8_K GEMV on repacked weights, reproducing ggml_vec_dot_q4_K_q8_K's generic f32 order
// exactly: per (row, column), blocks in ascending order, sums[l] += d*aux32[l] (l = 0..7),
// sumf -= dmin*sumi, then sumf += sums[0..7].
//
// Lane mapping (wave64): lane = (row slot s, column m, residue l) with 8/MC row slots, so a wave
// covers 8/MC rows x MC columns and every lane does one (row, column, residue) triple: lane l
// of the octet loads the block header and, as one 16-B load, exactly the nibbles ggml folds
// into aux32[l] (lane layout, tts_repack_q4_K); the eight sdot4 results times the 6-bit scales
// are aux32[l]; the lane keeps sums[l] in a register across blocks in ascending order and
// every lane of the octet carries sumf, so the exact order costs no LDS round trip.
// Prologue (same workgroup): the activation is quantized to Q8_K straight into LDS, after an
// optional LayerNorm; the first row's weight loads are issued before it so the HBM latency
// overlaps the prologue.
template <int MC, int PRO, int NBMAX>
__global__ __launch_bounds__(NBMAX <= 4 ? 1024 : 512) void k_gemv_q4_K(GemvJob j) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nb = (int)(j.K / QK_K);
    int8_t * xq_s = (int8_t *)smem;
    const int nslot = MC * nb + 1;  // + the prologue's trash slot
    float * xd_s = (float *)(smem + al16((size_t)nslot * QK_K));
    int16_t * xs_s = (int16_t *)((char *)xd_s + al16(sizeof(float) * nslot));

    // rows of all j.nmat matrices form one flat range (the launcher guarantees N % S == 0 when
    // nmat > 1, so a wave's S rows never straddle two matrices)
    constexpr int S = 8 / MC;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int l = lane & 7, m = (lane >> 3) % MC, s = lane / (8 * MC);
    const int64_t G = ((int64_t)j.nmat * j.N + S - 1) / S;
    const int64_t gstride = (int64_t)gridDim.x * nw;
    int64_t g = (int64_t)xcd_contiguous(blockIdx.x, gridDim.x) * nw + wave;
    auto mat_of = [&](int64_t flat) {  // wave-uniform; nmat <= 16, so no 64-bit division
        int mt = 0;
        while (mt + 1 < j.nmat && flat >= (int64_t)(mt + 1) * j.N) ++mt;
        return mt;
    };

    u32x4 hdr[NBMAX], q[NBMAX];
    auto load_row = [&](int64_t gg, int b0) {
        const int64_t flat0 = gg * S;
        const int mat = __builtin_amdgcn_readfirstlane(mat_of(flat0));  // gg is the wave's: uniform
        int64_t row = flat0 - (int64_t)mat * j.N + s;
        row = row < j.N ? row : j.N - 1;
        const uint8_t * wr = j.W[mat] + row * j.w_row_bytes;
#pragma unroll
        for (int u = 0; u < NBMAX; ++u) {  // unconditional (clamped) so all loads issue before use
            const int64_t bo = (int64_t)min(b0 + u, nb - 1) * 144;
            hdr[u] = TTS_WLOAD((const u32x4 *)(wr + bo));
            q[u] = TTS_WLOAD((const u32x4 *)(wr + bo + 16 + l * 16));
        }
        TTS_PIN_LOADS();
    };
    // the first row's weights are in flight during the prologue (long rows with an LN prologue would
    // need more registers than it leaves, so they start after it)
    TTS_TS(j, 0);
    auto mid = [&]() {
        // unconditional (an idle wave loads the last row group): a load under a branch leaves the
        // paths after it with different numbers of loads in flight, and the compiler then guards the
        // prologue's first use of the activation with vmcnt(0) -- a wait for these weight loads too
        if (NBMAX <= 4 || (TTS_GEMV_EARLY16 && PRO == PRO_QUANT)) load_row(g < G ? g : G - 1, 0);
        TTS_TS(j, 1);
    };
    q4k_prologue<PRO, NBMAX>(j, nb, xq_s, xd_s, xs_s, nullptr, nullptr, mid);
    TTS_TS(j, 2);
    __syncthreads();
    TTS_TS(j, 3);
    if (NBMAX > 4 && !(TTS_GEMV_EARLY16 && PRO == PRO_QUANT) && g < G) load_row(g, 0);
#ifdef TTS_PHASE_TS
    __builtin_amdgcn_s_waitcnt(0);  // phase study only: when the first row's weights have landed
    TTS_TS(j, 6);
#endif

    for (; g < G; g += gstride) {
        float sums = 0.f, sumf = 0.f;
        for (int b0 = 0; b0 < nb; b0 += NBMAX) {
            if (b0 > 0) load_row(g, b0);
#pragma unroll
            for (int u = 0; u < NBMAX; ++u) {  // branch-free: padding blocks compute and are discarded
                const bool valid = b0 + u < nb;
                const int b = min(b0 + u, nb - 1);
                q4k_block(hdr[u], q[u], xq_s, xs_s, xd_s, m * nb + b, l, valid, sums, sumf);
            }
        }
        const float tot = q4k_octet_total(sumf, sums);
        const int64_t flat0 = g * S;
        const int mat = __builtin_amdgcn_readfirstlane(mat_of(flat0));
        const int64_t row = flat0 - (int64_t)mat * j.N + s;
        TTS_TS(j, 4);
        if (l == 0 && m < j.M && row < j.N && mat < j.nmat) gemv_store<MC>(j, mat, row, m, tot);
        if (g + gstride < G) load_row(g + gstride, 0);
    }
    TTS_TS(j, 5);
}

// ------------------------------------------------------------------------------------------
// The same GEMV with one weight read per lane ("unique-load" kernel, the decode default for the
// lane layout).  In k_gemv_q4_K every column's lane octet loads the row's bytes again (8x at
// M = 8), so at Parler shapes the CU's load pipe, not HBM, sets the pace.  Here octet o of the
// workgroup owns one (row, block) pair -- lane l loads the 16 nibble bytes of residue l and the
// block header -- decodes scales and nibbles once and loops over the M columns: aux32[l] from
// eight sdot4 against the Q8_K block in LDS, sumi from the per-32 sums, and ggml's two per-block
// terms p = (d*yd)*aux32[l] and q = (dmin*yd)*sumi, rounded exactly as the sequential code rounds
// them.  The terms go to LDS; lane (row, column, l) then runs ggml's chain over the blocks in
// ascending order (sums[l] += p, sumf -= q, then sumf += sums[0..7]) -- the same additions in the
// same order, so the result is bit-identical.  512 threads = 64 octets; R rows x nb blocks <= 64.
struct Q4KLaneBlock {
    uint32_t nib[8];  // sdot4 operands: nibbles of dword c, low (even) / high (odd) half
    int sc[8];        // the matching 6-bit scales
    int mn01, mn23, mn45, mn67;  // mins as int16 pairs (v_dot2 against the per-32 sums)
    float dw, dmw;
};

__device__ __forceinline__ void q4k_lane_decode(const u32x4 & h, const u32x4 & qw, Q4KLaneBlock & o) {
    const uint32_t A = h.y, B = h.z, C = h.w;
    const uint32_t sc_lo = A & 0x3F3F3F3Fu, mn_lo = B & 0x3F3F3F3Fu;
    const uint32_t sc_hi = (C & 0x0F0F0F0Fu) | ((A >> 2) & 0x30303030u);
    const uint32_t mn_hi = ((C >> 4) & 0x0F0F0F0Fu) | ((B >> 2) & 0x30303030u);
    const uint32_t w[4] = {qw.x, qw.y, qw.z, qw.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        o.nib[2 * c] = w[c] & 0x0F0F0F0Fu;
        o.nib[2 * c + 1] = (w[c] >> 4) & 0x0F0F0F0Fu;
        const uint32_t sw = c < 2 ? sc_lo : sc_hi;
        o.sc[2 * c] = (int)((sw >> (16 * (c & 1))) & 0xFF);
        o.sc[2 * c + 1] = (int)((sw >> (16 * (c & 1) + 8)) & 0xFF);
    }
    o.mn01 = (int)((mn_lo & 0xFF) | ((mn_lo & 0xFF00) << 8));
    o.mn23 = (int)(((mn_lo >> 16) & 0xFF) | ((mn_lo >> 8) & 0xFF0000));
    o.mn45 = (int)((mn_hi & 0xFF) | ((mn_hi & 0xFF00) << 8));
    o.mn67 = (int)(((mn_hi >> 16) & 0xFF) | ((mn_hi >> 8) & 0xFF0000));
    o.dw = dev_fp16_to_fp32((uint16_t)(h.x & 0xFFFF));
    o.dmw = dev_fp16_to_fp32((uint16_t)(h.x >> 16));
}

// p and q of a decoded block against Q8_K slot xb (same arithmetic as q4k_block_pq)
__device__ __forceinline__ void q4k_lane_pq(const Q4KLaneBlock & o, const int8_t * xq_s, const int16_t * xs_s, const float * xd_s,
                                            int xb, int l, float & p, float & q) {
    const int4 xl = *(const int4 *)(xq_s + xb * QK_K + l * 32);
    const int4 xh = *(const int4 *)(xq_s + xb * QK_K + l * 32 + 16);
    const int4 bs = *(const int4 *)(xs_s + xb * 8);
    const int xv[8] = {xl.x, xh.x, xl.y, xh.y, xl.z, xh.z, xl.w, xh.w};
    int aux = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) aux += __mul24(o.sc[i], __builtin_amdgcn_sdot4((int)o.nib[i], xv[i], 0, false));
    int sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn01), __builtin_bit_cast(short2_t, bs.x), 0, false);
    sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn23), __builtin_bit_cast(short2_t, bs.y), sumi, false);
    sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn45), __builtin_bit_cast(short2_t, bs.z), sumi, false);
    sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn67), __builtin_bit_cast(short2_t, bs.w), sumi, false);
    const float yd = xd_s[xb];
    p = __fmul_rn(__fmul_rn(o.dw, yd), (float)aux);
    q = __fmul_rn(__fmul_rn(o.dmw, yd), (float)sumi);
}

template <int MC, int PRO, int NCH>
__global__ __launch_bounds__(512) void k_gemv_q4_K_u(GemvJob j, int R, int NCG) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nb = (int)(j.K / QK_K);
    const int M = (int)j.M;
    int8_t * xq_s = (int8_t *)smem;
    const int nslot = MC * nb + 1;  // + the prologue's trash slot
    float * xd_s = (float *)(smem + al16((size_t)nslot * QK_K));
    int16_t * xs_s = (int16_t *)((char *)xd_s + al16(sizeof(float) * nslot));
    float * cp = (float *)((char *)xs_s + al16((size_t)16 * nslot));  // [R][MC][nb][8] p terms
    float * cq = cp + (size_t)R * MC * nb * 8;                          // [R][MC][nb]    q terms

    // octet = (row r, block b, column group cg): NCG groups of CPL columns share a (row, block) when
    // the workgroup has more octets than (row, block) pairs
    const int l = threadIdx.x & 7, oct = threadIdx.x >> 3;
    const int units = R * nb;
    const int cg = oct / units, u = oct - cg * units;
    const int r = u / nb, b = u - r * nb;
    const int CPL = (M + NCG - 1) / NCG;
    const int m0 = cg * CPL;
    const int64_t NR = (int64_t)j.nmat * j.N;
    const int64_t row0 = (int64_t)xcd_contiguous(blockIdx.x, gridDim.x) * R;
    const bool own = cg < NCG && m0 < M && row0 + r < NR;  // this octet has (row, block, columns) work
    u32x4 hdr, qw;
    TTS_TS(j, 0);
    auto mid = [&]() {
        int64_t flat = row0 + r;
        flat = flat < NR ? flat : NR - 1;  // clamped: every lane loads, unused results are dropped
        const uint8_t * bp = j.W[0] + flat * j.w_row_bytes + (int64_t)b * 144;  // single-matrix jobs (launcher)
        // unconditional (spare octets load a valid block and drop it): see k_gemv_q4_K's first loads
        hdr = TTS_WLOAD((const u32x4 *)bp);
        qw = TTS_WLOAD((const u32x4 *)(bp + 16 + l * 16));
        TTS_PIN_LOADS();
        TTS_TS(j, 1);
    };
    q4k_prologue<PRO, NCH>(j, nb, xq_s, xd_s, xs_s, nullptr, nullptr, mid);
    TTS_TS(j, 2);
    __syncthreads();
    TTS_TS(j, 3);
    if (own) {
        Q4KLaneBlock o;
        q4k_lane_decode(hdr, qw, o);
        constexpr int CM = MC;  // columns per lane, compile-time bound (CPL <= MC)
        int4 xl[CM], xh[CM], bs[CM];
        float yd[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) {  // every operand read from LDS first
            const int xb = min(m0 + c, M - 1) * nb + b;
            xl[c] = *(const int4 *)(xq_s + xb * QK_K + l * 32);
            xh[c] = *(const int4 *)(xq_s + xb * QK_K + l * 32 + 16);
            bs[c] = *(const int4 *)(xs_s + xb * 8);
            yd[c] = xd_s[xb];
        }
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            if (c >= CPL || m0 + c >= M) break;
            const int xv[8] = {xl[c].x, xh[c].x, xl[c].y, xh[c].y, xl[c].z, xh[c].z, xl[c].w, xh[c].w};
            int aux = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) aux += __mul24(o.sc[i], __builtin_amdgcn_sdot4((int)o.nib[i], xv[i], 0, false));
            int sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn01), __builtin_bit_cast(short2_t, bs[c].x), 0, false);
            sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn23), __builtin_bit_cast(short2_t, bs[c].y), sumi, false);
            sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn45), __builtin_bit_cast(short2_t, bs[c].z), sumi, false);
            sumi = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, o.mn67), __builtin_bit_cast(short2_t, bs[c].w), sumi, false);
            const float p = __fmul_rn(__fmul_rn(o.dw, yd[c]), (float)aux);
            const float q = __fmul_rn(__fmul_rn(o.dmw, yd[c]), (float)sumi);
            const int64_t e = ((int64_t)r * MC + m0 + c) * nb + b;
            cp[e * 8 + l] = p;
            if (l == 0) cq[e] = q;
        }
    }
    __syncthreads();
    TTS_TS(j, 4);
    // chain lanes: t = ((r * M + m) * 8 + l); whole octets per (row, column)
    const int nchain = R * M * 8;
    for (int t = threadIdx.x; t - l < nchain; t += 512) {
        const int rm = t >> 3;
        const int rr = rm / M, m = rm - rr * M;
        const bool ok = t < nchain && row0 + rr < NR;
        float sums = 0.f, sumf = 0.f;
        if (ok) {
            const float * pp = cp + ((int64_t)rr * MC + m) * nb * 8 + l;
            const float * qq = cq + ((int64_t)rr * MC + m) * nb;
            constexpr int CB = 16;  // terms fetched per batch (independent LDS reads), then chained in order
            for (int b0 = 0; b0 < nb; b0 += CB) {
                float pv[CB], qv[CB];
#pragma unroll
                for (int i = 0; i < CB; ++i) {
                    const int bb = min(b0 + i, nb - 1);
                    pv[i] = pp[bb * 8];
                    qv[i] = qq[bb];
                }
#pragma unroll
                for (int i = 0; i < CB; ++i) {
                    if (b0 + i >= nb) break;
                    sums = __fadd_rn(sums, pv[i]);
                    sumf = __fsub_rn(sumf, qv[i]);
                }
            }
        }
        const float tot = q4k_octet_total(sumf, sums);
        if (ok && l == 0) {
            gemv_store<8>(j, 0, row0 + rr, m, tot);
        }
    }
    TTS_TS(j, 5);
}

// ------------------------------------------------------------------------------------------
// Q4_K x Q8_K GEMV on the matrix cores, for large matrices at 2..16 columns (Orpheus / Dia-sized
// decode GEMVs at batch > 1).  The VALU kernel above spends ~45 instructions per (row, column,
// block) on integer dots; here the integer part of ggml's vec_dot_q4_K_q8_K runs as f16 MFMAs
// whose results are EXACT integers, so the f32 combine is unchanged and the output bit-identical:
//   aux32[l] (row, col) = sum_{j,kk} (sc_j * q4[32j + 8kk + l]) * q8[32j + 8kk + l]
// is one v_mfma_f32_16x16x32_f16 per residue l over K = 32 = (j, kk): A = sc_j * q4 <= 945 and
// B = q8 (|q8| <= 127) are exact in f16, the products (<= 120015) exact in f32, and every partial
// sum of a residue stays below 2^24 (<= 8 * 63 * 4 * 15 * 127 = 3.84e6), so the f32 accumulation
// is exact in any order.  sumi = sum_j mins_j * bsum_j is a 9th MFMA with bsum = 64*hi + lo split
// (A = [mins, 64*mins, 0, 0], B = [lo, hi, -, -]).
// Tile: 16 weight rows x 16 columns per wave, K index k = 8*kg + 4h + kk for lane group kg = c:
// lane (row r, kg) holds for each residue l the dword of bytes qs[32c + 8kk + l] (kk = 0..3; low
// nibble sub-block 2c, high 2c+1), read from the tile layout (tts_repack_q4_K_tiled) as two 16-B
// pieces; B comes from LDS in the matching order
// (q8k_row_block_mf).  C: column = lane & 15, rows 4*kg + reg.  Per (row, col) the lane then does
// ggml's f32 combine in block order: sums[l] += (d*yd)*aux32[l], sumf -= (dmin*yd)*sumi.
// Loads: 4-block batches, double-buffered across batches and tiles, the first issued before the
// prologue.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// bytes 0,1 (SEL 0x0C010C00) or 2,3 (0x0C030C02) of w (each <= 63) as u16 lanes of 1024 + n
__device__ __forceinline__ f16x2 byte2_f16_biased(uint32_t w, uint32_t sel) {
    return __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(0u, w, sel) | 0x64006400u);
}

// RS > 1 (residue split; the launcher guarantees one tile per wave slot and no SwiGLU epilogue): the
// RS waves w = part * (nw / RS) + slot of a workgroup share tile `slot`, wave `part` running the
// MFMAs and f32 chains of residues l = part * 8 / RS .. + 8 / RS - 1 (the last part also the mins
// chain).  ggml's chains are per residue (sums[l]) plus sumf, joined only at the end
// (sumf + sums[0] + ... + sums[7]), so after one barrier the last part adds the others' sums from LDS
// in residue order: the same additions as the one-wave kernel.  Few-tile matrices (Orpheus down:
// 192 tiles of 32 blocks) then keep all four SIMDs of a CU busy instead of one.
// Compile-time sequence C = B..E-1 of calls f(integral_constant<C>) (an unrolled chunk loop whose
// register buffers are indexed by constants)
template <int B, int E>
struct ChunkSeq {
    template <class F>
    __device__ __forceinline__ static void run(F && f) {
        f(std::integral_constant<int, B>{});
        ChunkSeq<B + 1, E>::run(f);
    }
};
template <int E>
struct ChunkSeq<E, E> {
    template <class F>
    __device__ __forceinline__ static void run(F &&) {}
};

// NCK > 0: every row tile is NCK chunks of 4 blocks (K = 1024 NCK) and the chunk loop is unrolled:
// straight-line code in which the compiler's wait counting stays exact (in the runtime loop it put
// address temporaries into the registers of the next chunk's in-flight loads and then had to wait
// for every load, the prefetch included, before each chunk)
template <int PRO, int NCH, int RS = 1, int NCK = 0>
__global__ __launch_bounds__(512) void k_gemv_q4K_mf(GemvJob j) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nb = (int)(j.K / QK_K);
    const int M = (int)j.M;
    const int nslot = M * nb + 1;  // + the prologue's trash slot
    _Float16 * b16 = (_Float16 *)smem;                     // [nslot][256] B operands per residue
    _Float16 * sbs = b16 + (size_t)nslot * QK_K;           // [nslot][16]  bsum lo / hi
    float * xd_s = (float *)(sbs + (size_t)nslot * 16);    // [nslot]      Q8_K d

    TTS_TS(j, 0);
    // wave-uniform by construction (readfirstlane): branches on the wave's part / slot are then scalar,
    // and the compiler's wait counting stays exact across them (exec-masked branches made it wait for
    // every load in flight, the next chunk's prefetch included, inside the row loop)
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
    const int r = lane & 15, kg = lane >> 4;
    const int cc = r < M ? r : M - 1;  // B / C column (padding columns compute and are dropped)
    constexpr int CH = 4;
    const int nch = NCK > 0 ? NCK : (nb + CH - 1) / CH;
    // EPI_SWIGLU: a wave runs tile t of gate, then tile t of up (units = tile pairs), and keeps the
    // gate results in registers until the up tile is done
    // When every pair fits one wave slot of the first half of the workgroups' waves (xpair), wave w
    // of the first half runs gate tile t and wave w + nw/2 up tile t instead, and the gate results
    // cross over through LDS after one barrier.
    const bool swiglu = j.epi == EPI_SWIGLU;
    const int64_t NR = swiglu ? j.N : job_rows(j);
    const int64_t T = (NR + 15) / 16;
    const int half = nw >> 1;
    const bool xpair = RS == 1 && swiglu && T <= (int64_t)gridDim.x * half;
    const int per = swiglu && !xpair ? 2 : 1;
    const int xmat = xpair && wave >= half ? 1 : 0;  // xpair: this wave's matrix (0 gate, 1 up)
    constexpr int LPW = 8 / RS;                      // residues per wave
    const int nws = nw / RS;                         // tile slots per workgroup
    const int part = RS > 1 ? wave / nws : 0;
    const int slot = RS > 1 ? wave - part * nws : wave;
    // tile t0 + k * tstride; consecutive tiles go to different workgroups, so a small matrix still
    // spreads over every CU
    const int64_t t0 = (int64_t)(slot - xmat * half) * gridDim.x + blockIdx.x;
    const int64_t tstride = (xpair || RS > 1) ? T : (int64_t)gridDim.x * nw;
    const int64_t nmine = (t0 < T && !(j.dbg & 1)) ? ((T - 1 - t0) / tstride + 1) * nch * per : 0;
    float * xg = (float *)(smem + al16((size_t)nslot * (2 * QK_K + 32 + 4)));  // xpair: [half][64 lanes][4]
    auto mat_of = [&](int64_t flat) {
        int mt = 0;
        while (mt + 1 < j.nmat && flat >= job_roff(j, mt + 1)) ++mt;
        return mt;
    };

    // tile layout (tts_repack_q4_K_tiled): lane (r, kg) reads its row's header and the two 16-B
    // pieces of chunk c = kg (residues 0..3, 4..7); a quarter wave covers four 64-B runs
    u32x4 hd[2][CH], qa[2][CH], qb[2][RS == 1 ? CH : 1];  // RS > 1: qa holds this wave's 16-B piece
    auto load = [&](auto BS, int64_t i) __attribute__((always_inline)) {
        constexpr int bs = decltype(BS)::value;
        const int64_t ti = i / nch;
        const int64_t t = t0 + (ti / per) * tstride;
        const int c = (int)(i % nch);
        int64_t flat = t * 16 + r;
        flat = flat < NR ? flat : NR - 1;
        // a 16-row tile never straddles two matrices (row counts are multiples of 16): the tile's
        // matrix is wave-uniform, and readfirstlane keeps W[mat] / roff[mat] scalar loads
        const int mat = __builtin_amdgcn_readfirstlane(xpair ? xmat : swiglu ? (int)(ti & 1) : mat_of(flat));
        const int64_t row = swiglu ? flat : flat - job_roff(j, mat);
        const uint8_t * wt = j.W[mat] + (row >> 2) * nb * 576;
        const int ri = (int)(row & 3);
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const uint8_t * bp = wt + (int64_t)min(c * CH + u, nb - 1) * 576;
            if (RS > 1) {  // the piece holding residues part * LPW ..: 0..3 (half 0) or 4..7 (half 1)
                hd[bs][u] = TTS_WLOAD((const u32x4 *)(bp + ri * 16));
                qa[bs][u] = TTS_WLOAD((const u32x4 *)(bp + 64 + ((kg * 2 + (part * LPW >= 4 ? 1 : 0)) * 4 + ri) * 16));
            } else if (j.dbg & 4) {  // phase study: plain (cached) loads
                hd[bs][u] = *(const u32x4 *)(bp + ri * 16);
                qa[bs][u] = *(const u32x4 *)(bp + 64 + ((kg * 2) * 4 + ri) * 16);
                qb[bs][RS == 1 ? u : 0] = *(const u32x4 *)(bp + 64 + ((kg * 2 + 1) * 4 + ri) * 16);
            } else {
                hd[bs][u] = TTS_WLOAD((const u32x4 *)(bp + ri * 16));
                qa[bs][u] = TTS_WLOAD((const u32x4 *)(bp + 64 + ((kg * 2) * 4 + ri) * 16));
                qb[bs][RS == 1 ? u : 0] = TTS_WLOAD((const u32x4 *)(bp + 64 + ((kg * 2 + 1) * 4 + ri) * 16));
            }
        }
        TTS_PIN_LOADS();
    };

    // ggml's f32 chain per (row q, column): sums[l] += (d*yd)*aux32[l], sumf -= (dmin*yd)*sumi, kept
    // as pairs of rows (q = 0,1 / 2,3) so the products and sums issue as packed f32 ops (each element
    // still one rounded multiply and one rounded add)
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v sums[LPW][2], sumf[2];
    float gate[4];
    auto compute = [&](auto BS, int64_t i) __attribute__((always_inline)) {
        constexpr int bs = decltype(BS)::value;
        const int64_t ti = i / nch;
        const int64_t t = t0 + (ti / per) * tstride;
        const int c = (int)(i % nch);
        if (c == 0) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                sumf[h] = f2v{0.f, 0.f};
#pragma unroll
                for (int l = 0; l < LPW; ++l) sums[l][h] = f2v{0.f, 0.f};
            }
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int b = c * CH + u;
            if (b >= nb) break;  // wave-uniform
            const u32x4 h = hd[bs][u];
            const uint32_t sc_lo = h.y & 0x3F3F3F3Fu, mn_lo = h.z & 0x3F3F3F3Fu;
            const uint32_t sc_hi = (h.w & 0x0F0F0F0Fu) | ((h.y >> 2) & 0x30303030u);
            const uint32_t mn_hi = ((h.w >> 4) & 0x0F0F0F0Fu) | ((h.z >> 2) & 0x30303030u);
            // A side: scales of sub-blocks 2kg (low nibbles) and 2kg + 1 (high nibbles)
            const uint32_t sw = (kg < 2 ? sc_lo : sc_hi) >> ((kg & 1) * 16);
            const _Float16 s0 = (_Float16)(float)(sw & 0xFF), s1 = (_Float16)(float)((sw >> 8) & 0xFF);
            const f16x2 S0 = {s0, s0}, S1 = {s1, s1};
            const _Float16 o0 = (_Float16)(-1024.f * (float)(sw & 0xFF)), o1 = (_Float16)(-1024.f * (float)((sw >> 8) & 0xFF));
            const f16x2 O0 = {o0, o0}, O1 = {o1, o1};
            const _Float16 * bsl = b16 + (size_t)(cc * nb + b) * QK_K + kg * 8;
            f32x4 acc[LPW];
#pragma unroll
            for (int ll = 0; ll < LPW; ++ll) {
                const int l = part * LPW + ll;
                uint32_t D;
                if (RS == 1) D = ll < 4 ? qa[bs][u][ll & 3] : qb[bs][RS == 1 ? u : 0][ll & 3];
                else if (RS == 2) D = qa[bs][u][ll];
                else D = (part & 1) ? qa[bs][u][2 + ll] : qa[bs][u][ll];
                const uint32_t lo = D & 0x0F0F0F0Fu, hi = (D >> 4) & 0x0F0F0F0Fu;
                // fma(1024 + n, s, -1024 s) = s * n exactly (single rounding of an exact value)
                const f16x2 a0 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C010C00u), S0, O0);
                const f16x2 a1 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C030C02u), S0, O0);
                const f16x2 a2 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C010C00u), S1, O1);
                const f16x2 a3 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C030C02u), S1, O1);
                const f16x8 A = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, a3.x, a3.y};
                const f16x8 B = *(const f16x8 *)(bsl + l * 32);
                acc[ll] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
            const bool mins = RS == 1 || part == RS - 1;  // wave-uniform
            // sumi: lane group 0 holds the 8 mins, group 1 the mins times 64, groups 2, 3 zero
            const _Float16 mm = (_Float16)(kg == 0 ? 1.f : kg == 1 ? 64.f : 0.f);
            const f16x2 MM = {mm, mm}, OFF = {(_Float16)-1024.f, (_Float16)-1024.f};
            const f16x2 m0 = (byte2_f16_biased(mn_lo, 0x0C010C00u) + OFF) * MM;
            const f16x2 m1 = (byte2_f16_biased(mn_lo, 0x0C030C02u) + OFF) * MM;
            const f16x2 m2 = (byte2_f16_biased(mn_hi, 0x0C010C00u) + OFF) * MM;
            const f16x2 m3 = (byte2_f16_biased(mn_hi, 0x0C030C02u) + OFF) * MM;
            const f16x8 As = {m0.x, m0.y, m1.x, m1.y, m2.x, m2.y, m3.x, m3.y};
            const f16x8 Bs = *(const f16x8 *)(sbs + (size_t)(cc * nb + b) * 16 + (kg & 1) * 8);
            f32x4 si = {0.f, 0.f, 0.f, 0.f};
            if (mins) si = __builtin_amdgcn_mfma_f32_16x16x32_f16(As, Bs, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            const float yd = xd_s[cc * nb + b];
            float dyq[4], dmyq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t hx = (uint32_t)__shfl((int)h.x, 4 * kg + q);  // d | dmin of row 4kg + q
                dyq[q] = __fmul_rn(dev_fp16_to_fp32((uint16_t)(hx & 0xFFFF)), yd);
                dmyq[q] = __fmul_rn(dev_fp16_to_fp32((uint16_t)(hx >> 16)), yd);
            }
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const f2v dy = {dyq[2 * hq], dyq[2 * hq + 1]}, dmy = {dmyq[2 * hq], dmyq[2 * hq + 1]};
#pragma unroll
                for (int l = 0; l < LPW; ++l) sums[l][hq] = sums[l][hq] + dy * f2v{acc[l][2 * hq], acc[l][2 * hq + 1]};
                if (mins) sumf[hq] = sumf[hq] - dmy * f2v{si[2 * hq], si[2 * hq + 1]};
            }
        }
        if (RS == 1 && c == nch - 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float tot = sumf[q >> 1][q & 1];
#pragma unroll
                for (int l = 0; l < LPW; ++l) tot = __fadd_rn(tot, sums[l][q >> 1][q & 1]);
                const int64_t flat = t * 16 + 4 * kg + q;
                if (xpair) {
                    gate[q] = tot;  // gate or up row: crossed over after the loop
                } else if (swiglu) {
                    if ((ti & 1) == 0) gate[q] = tot;  // gate row; the up row follows in this wave
                    else if (r < M && flat < NR) j.Y[0][r * j.ycs[0] + flat * j.yrs[0]] = __fmul_rn(dev_silu(gate[q]), tot);
                } else if (r < M && flat < NR) {
                    const int mat = __builtin_amdgcn_readfirstlane(mat_of(t * 16));  // the tile's matrix
                    gemv_store<8>(j, mat, flat - job_roff(j, mat), r, tot);
                }
            }
        }
    };

    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    auto mid = [&]() {
        if (nmine > 0) load(I0{}, 0);
        TTS_TS(j, 1);
    };
    if constexpr (PRO == PRO_COPY) {
        // the operands k_quant_mf wrote, in this kernel's LDS layout: 1 KiB per wave instruction by
        // LDS-DMA (no registers), the weight loads behind them
        const int nck = (int)(j.bq_bytes >> 10);
        for (int i = wave; i < nck; i += nw)
            __builtin_amdgcn_global_load_lds(gptr(j.bq + (size_t)i * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void *)(smem + (size_t)i * 1024), 16, 0, 0);
        TTS_PIN_LOADS();
        load(I0{}, 0);  // unconditional (clamped): the wait below counts exactly these loads
        TTS_PIN_LOADS();
        // this wave's DMA has landed once at most the weight loads issued after it are outstanding
        constexpr int NWL = (RS == 1 ? 3 : 2) * CH;
        __builtin_amdgcn_s_waitcnt((NWL & 15) | (7 << 4) | (15 << 8) | (((NWL >> 4) & 3) << 14));
    } else if (!(j.dbg & 2)) {
        q4k_prologue<PRO, NCH, true>(j, nb, nullptr, xd_s, nullptr, b16, sbs, mid);
    } else {
        mid();
    }
    TTS_TS(j, 2);
    __syncthreads();
    TTS_TS(j, 3);
    if constexpr (NCK > 0) {
        const int64_t units = nmine / NCK;  // tiles (SwiGLU: gate / up tiles) of this wave
        for (int64_t u = 0; u < units; ++u) {
            if (u > 0) load(I0{}, u * NCK);
            ChunkSeq<0, NCK>::run([&](auto CI) __attribute__((always_inline)) {
                constexpr int C = decltype(CI)::value;
                if constexpr (C + 1 < NCK) load(std::integral_constant<int, (C + 1) & 1>{}, u * NCK + C + 1);
                compute(std::integral_constant<int, C & 1>{}, u * NCK + C);
            });
        }
    } else {
        for (int64_t i = 0; i < nmine; i += 2) {
            load(I1{}, min(i + 1, nmine - 1));
            compute(I0{}, i);
            if (i + 1 >= nmine) break;
            load(I0{}, min(i + 2, nmine - 1));
            compute(I1{}, i + 1);
        }
    }
    if (RS > 1) {  // one tile per wave at most: join the parts' chains in residue order
        float * xs = xg;  // [RS - 1 parts][nws slots][64 lanes][LPW * 4]
        if (nmine > 0 && part < RS - 1) {
            float * o = xs + (((size_t)part * nws + slot) * 64 + lane) * LPW * 4;
#pragma unroll
            for (int l = 0; l < LPW; ++l)
                *(float4 *)(o + 4 * l) = make_float4(sums[l][0][0], sums[l][0][1], sums[l][1][0], sums[l][1][1]);
        }
        __syncthreads();
        if (nmine > 0 && part == RS - 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float tot = sumf[q >> 1][q & 1];
                for (int p = 0; p < RS - 1; ++p) {
                    const float * o = xs + (((size_t)p * nws + slot) * 64 + lane) * LPW * 4;
#pragma unroll
                    for (int l = 0; l < LPW; ++l) tot = __fadd_rn(tot, o[4 * l + q]);
                }
#pragma unroll
                for (int l = 0; l < LPW; ++l) tot = __fadd_rn(tot, sums[l][q >> 1][q & 1]);
                const int64_t flat = t0 * 16 + 4 * kg + q;
                if (r < M && flat < NR) {
                    const int mat = __builtin_amdgcn_readfirstlane(mat_of(t0 * 16));  // the tile's matrix
                    gemv_store<8>(j, mat, flat - job_roff(j, mat), r, tot);
                }
            }
        }
    }
    if (xpair) {  // one tile per wave at most: out = silu(gate) * up
        if (nmine > 0 && xmat == 0)
            *(float4 *)(xg + ((size_t)wave * 64 + lane) * 4) = make_float4(gate[0], gate[1], gate[2], gate[3]);
        __syncthreads();
        if (nmine > 0 && xmat == 1) {
            const float4 g4 = *(const float4 *)(xg + ((size_t)(wave - half) * 64 + lane) * 4);
            const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t flat = t0 * 16 + 4 * kg + q;
                if (r < M && flat < NR) j.Y[0][r * j.ycs[0] + flat * j.yrs[0]] = __fmul_rn(dev_silu(gv[q]), gate[q]);
            }
        }
    }
    TTS_TS(j, 5);
}

// ------------------------------------------------------------------------------------------
// Matrix-core Q4_K GEMV, "K relay" (k_gemv_q4K_kr): one workgroup per 16-row tile (SwiGLU: per gate /
// up tile pair), its waves splitting the tile's blocks: wave w owns the BPW consecutive blocks
// w*BPW .. (w+1)*BPW-1.  Every weight byte is loaded once (header + both 16-B residue pieces per
// lane, all of the wave's blocks requested at entry behind the operand DMA), the integer dots are
// the MFMAs of k_gemv_q4K_mf (8 residue MFMAs + the mins MFMA per block, exact), and each lane
// turns them into ggml's per-block terms p_l = (d*yd)*aux32[l], q = (dmin*yd)*sumi for its 4 rows x
// 1 column, kept in registers.  ggml's chain (sums[l] += p_l, sumf -= q over the blocks in
// ascending order) then runs as a relay: wave 0 folds its blocks, hands the 36 running sums per lane
// to wave 1 through LDS, and so on; the last wave adds sumf + sums[0..7] and stores.  Same additions
// in the same order as vec_dot_q4_K_q8_K: bit-identical.  A tile's weights stream through all its
// waves at once instead of one chunk at a time through one wave (k_gemv_q4K_mf's row phase).
// Operands: PRO_COPY (k_quant_mf's layout, DMA'd into LDS).
// LANE: weights in the lane layout (tts_repack_q4_K: residue l's 16 bytes of a block at 16 + 16 l,
// chunk c's dword at + 4 c -- the tile layout's piece dword for (c, l)), read as 8 dwords per block;
// otherwise the 4-row tile layout.  blockIdx.y = column tile (j.bq_tile > 0: 16 columns per tile,
// the many-column prefill GEMM).
// LOOP: a workgroup per CU walks tiles t = blockIdx.x + k * gridDim.x (the operands are copied once,
// the next tile's weights are requested before the current tile's relay); otherwise one tile per
// workgroup.  Terms and running sums are kept as row pairs (packed f32 ops, each element still one
// rounded multiply / add).
// PRO (PRO_QUANT / PRO_LN, K <= 4096): no operand pass -- the workgroup norms / quantizes the
// activation itself (q4k_prologue, the MFMA operand layout k_quant_mf writes), its first weight loads
// issued between the prologue's activation loads and their use.
// CTW = 2 (PRO_COPY, column tiles): a workgroup takes two column tiles of its row tile in turn -- the
// tile's weights are loaded into registers once and multiplied against both tiles' operands (both in
// LDS), instead of two workgroups streaming the same weights.
// CP (PRO_COPY, column tiles): the workgroup's two wave halves take column tiles 2y and 2y + 1 of the
// same row tile at once -- both halves request the same weight bytes, the second half's requests are
// served by the CU's caches, so each weight tile is streamed from HBM once for 32 columns while every
// tile keeps its own NWT-wave relay (same additions, same order as CTW = 1: bit-identical).
template <int BPW, bool SW, int NWT, bool LANE = false, bool LOOP = false, int PRO = PRO_COPY, int CTW = 1, bool CP = false>
__global__ __launch_bounds__(64 * NWT * ((SW || CP) ? 2 : 1)) void k_gemv_q4K_kr(GemvJob j) {
    constexpr int nwt = NWT;  // waves per tile: blocks w*BPW .. of a K = 256 * NWT * BPW row
    typedef float f2v __attribute__((ext_vector_type(2)));
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nb = (int)(j.K / QK_K);
    int tx = blockIdx.x, ty = blockIdx.y;
    if constexpr (!LOOP && CTW == 1) {
        // j.xcd_cols: the column tiles of one row tile on one XCD, dispatched back to back (the dispatcher
        // puts workgroup b on XCD b % 8): the second streams the tile's weights out of that XCD's L2
        // instead of HBM.  The work per (row tile, column tile) is unchanged.
        if (j.xcd_cols && gridDim.y > 1) {
            const int n = gridDim.x * gridDim.y;
            const int w = xcd_contiguous(blockIdx.x + gridDim.x * blockIdx.y, n);
            tx = w / gridDim.y;
            ty = w - tx * gridDim.y;
        }
    }
    constexpr int CT = CP ? 2 : CTW;            // column tiles per workgroup
    const int ct0 = ty * CT;                   // (first) column tile
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
    const int sub = (SW || CP) ? wave / nwt : 0;  // SwiGLU: 0 = gate tile, 1 = up tile; CP: the column tile ct0 + sub
    int c0 = j.bq_tile ? 16 * (ct0 + (CP ? sub : 0)) : 0;  // the first column
    int M = j.bq_tile ? min(16, (int)j.M - c0) : (int)j.M;  // (CP: <= 0 for the idle half of an odd last pair)
    const int ntile = CT == 1 ? 1 : min(CT, (int)((j.M + 15) / 16) - ct0);  // column tiles of this workgroup
    const char * const bqt = j.bq + (size_t)ct0 * j.bq_tile;
    const int64_t bqb = j.bq_tile ? j.bq_tile : j.bq_bytes;
    const int Ma = M > 0 ? M : 1;              // slot addressing of an idle half (it stores nothing)
    int nslot = Ma * nb + 1;
    _Float16 * b16 = (_Float16 *)(smem + (CP ? (size_t)sub * bqb : 0));
    _Float16 * sbs = b16 + (size_t)nslot * QK_K;
    float * xd_s = (float *)(sbs + (size_t)nslot * 16);
    float * relay = (float *)(smem + ((CT * bqb + 15) & ~(int64_t)15));  // [1 or 2 sub-tiles][64 lanes][36]

    const int r = lane & 15, kg = lane >> 4;
    int cc = r < Ma ? r : Ma - 1;
    const int w = wave - sub * nwt;         // position in the relay
    const int64_t NR = SW ? j.N : job_rows(j);
    const int64_t T = NR / 16;              // launcher: whole tiles
    auto mat_of = [&](int64_t flat) {
        int mt = 0;
        while (mt + 1 < j.nmat && flat >= job_roff(j, mt + 1)) ++mt;
        return mt;
    };
    auto tile_mat = [&](int64_t t) { return __builtin_amdgcn_readfirstlane(SW ? sub : mat_of(t * 16)); };
    auto tile_row0 = [&](int64_t t, int mat) { return SW ? t * 16 : t * 16 - job_roff(j, mat); };

    TTS_TS(j, 0);
    u32x4 hd[LOOP ? 2 : 1][BPW], qa[LOOP ? 2 : 1][BPW], qb[LOOP ? 2 : 1][BPW];
    // j.xcd_cols: the weights are loaded with the default (L2-allocating) policy, so the row tile's
    // other column tile, dispatched on the same XCD right after, reads them from that XCD's L2; a
    // non-temporal load would not leave them there
    auto load_w_pol = [&](auto BUF, auto PLAIN, int64_t t) __attribute__((always_inline)) {
        constexpr int bf = decltype(BUF)::value;
        constexpr bool plain = decltype(PLAIN)::value;
        auto ld = [](const auto * p) __attribute__((always_inline)) {
            if constexpr (plain) return *gptr(p);
            else return TTS_WLOAD(p);
        };
        t = t < T ? t : T - 1;
        const int mat = tile_mat(t);
        int64_t row = tile_row0(t, mat) + r;
        const int64_t rows_m = SW ? j.N : job_roff(j, mat + 1) - job_roff(j, mat);
        row = row < rows_m ? row : rows_m - 1;
        if constexpr (LANE) {
            const uint8_t * wr = j.W[mat] + row * j.w_row_bytes;
#pragma unroll
            for (int u = 0; u < BPW; ++u) {
                const uint8_t * bp = wr + (int64_t)min(w * BPW + u, nb - 1) * 144;
                hd[bf][u] = ld((const u32x4 *)bp);
#pragma unroll
                for (int l = 0; l < 4; ++l) {
                    qa[bf][u][l] = ld((const uint32_t *)(bp + 16 + l * 16 + kg * 4));
                    qb[bf][u][l] = ld((const uint32_t *)(bp + 16 + (l + 4) * 16 + kg * 4));
                }
            }
        } else {
            const uint8_t * wt = j.W[mat] + (row >> 2) * nb * 576;
            const int ri = (int)(row & 3);
#pragma unroll
            for (int u = 0; u < BPW; ++u) {
                const uint8_t * bp = wt + (int64_t)min(w * BPW + u, nb - 1) * 576;
                hd[bf][u] = ld((const u32x4 *)(bp + ri * 16));
                qa[bf][u] = ld((const u32x4 *)(bp + 64 + ((kg * 2) * 4 + ri) * 16));
                qb[bf][u] = ld((const u32x4 *)(bp + 64 + ((kg * 2 + 1) * 4 + ri) * 16));
            }
        }
        TTS_PIN_LOADS();
    };
    auto load_w = [&](auto BUF, int64_t t) __attribute__((always_inline)) {
        if (!LOOP && CTW == 1 && j.xcd_cols && gridDim.y > 1) load_w_pol(BUF, std::true_type{}, t);
        else load_w_pol(BUF, std::false_type{}, t);
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, LOOP ? 1 : 0>;
    int64_t t = tx;
    if constexpr (PRO == PRO_COPY) {
        // operands by LDS-DMA, then this wave's weights (unconditional, clamped)
        const int nck = (int)((ntile * bqb) >> 10);
        for (int i = wave; i < nck; i += nw)
            __builtin_amdgcn_global_load_lds(gptr(bqt + (size_t)i * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void *)(smem + (size_t)i * 1024), 16, 0, 0);
        TTS_PIN_LOADS();
        load_w(B0{}, t);
    } else {
        auto first = [&]() __attribute__((always_inline)) { load_w(B0{}, t); };
        ProOv ov;  // a column tile (j.bq_tile: the many-column GEMM at decode sizes) quantizes its own columns
        ov.col0 = c0;
        ov.mcols = M;
        q4k_prologue<PRO, 16, true, decltype(first)>(j, nb, nullptr, xd_s, nullptr, b16, sbs, first, ov);
    }
    TTS_TS(j, 1);
    __syncthreads();  // the operand DMA has landed (the compiler waits for all of it here)
    TTS_TS(j, 2);

    // the terms of this wave's blocks for rows 4kg + q (pairs h: q = 2h, 2h + 1), column r
    f2v tp[BPW][8][2], tq[BPW][2];
    auto terms = [&](auto BUF) __attribute__((always_inline)) {
        constexpr int bf = decltype(BUF)::value;
#pragma unroll
        for (int u = 0; u < BPW; ++u) {
            const int b = min(w * BPW + u, nb - 1);
            const u32x4 h = hd[bf][u];
            const uint32_t sc_lo = h.y & 0x3F3F3F3Fu, mn_lo = h.z & 0x3F3F3F3Fu;
            const uint32_t sc_hi = (h.w & 0x0F0F0F0Fu) | ((h.y >> 2) & 0x30303030u);
            const uint32_t mn_hi = ((h.w >> 4) & 0x0F0F0F0Fu) | ((h.z >> 2) & 0x30303030u);
            const uint32_t sw = (kg < 2 ? sc_lo : sc_hi) >> ((kg & 1) * 16);
            const _Float16 s0 = (_Float16)(float)(sw & 0xFF), s1 = (_Float16)(float)((sw >> 8) & 0xFF);
            const f16x2 S0 = {s0, s0}, S1 = {s1, s1};
            const _Float16 o0 = (_Float16)(-1024.f * (float)(sw & 0xFF)), o1 = (_Float16)(-1024.f * (float)((sw >> 8) & 0xFF));
            const f16x2 O0 = {o0, o0}, O1 = {o1, o1};
            const _Float16 * bsl = b16 + (size_t)(cc * nb + b) * QK_K + kg * 8;
            f32x4 acc[8];
#pragma unroll
            for (int l = 0; l < 8; ++l) {
                const uint32_t D = l < 4 ? qa[bf][u][l & 3] : qb[bf][u][l & 3];
                const uint32_t lo = D & 0x0F0F0F0Fu, hi = (D >> 4) & 0x0F0F0F0Fu;
                const f16x2 a0 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C010C00u), S0, O0);
                const f16x2 a1 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C030C02u), S0, O0);
                const f16x2 a2 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C010C00u), S1, O1);
                const f16x2 a3 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C030C02u), S1, O1);
                const f16x8 A = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, a3.x, a3.y};
                const f16x8 B = *(const f16x8 *)(bsl + l * 32);
                acc[l] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
            const _Float16 mm = (_Float16)(kg == 0 ? 1.f : kg == 1 ? 64.f : 0.f);
            const f16x2 MM = {mm, mm}, OFF = {(_Float16)-1024.f, (_Float16)-1024.f};
            const f16x2 m0 = (byte2_f16_biased(mn_lo, 0x0C010C00u) + OFF) * MM;
            const f16x2 m1 = (byte2_f16_biased(mn_lo, 0x0C030C02u) + OFF) * MM;
            const f16x2 m2 = (byte2_f16_biased(mn_hi, 0x0C010C00u) + OFF) * MM;
            const f16x2 m3 = (byte2_f16_biased(mn_hi, 0x0C030C02u) + OFF) * MM;
            const f16x8 As = {m0.x, m0.y, m1.x, m1.y, m2.x, m2.y, m3.x, m3.y};
            const f16x8 Bs = *(const f16x8 *)(sbs + (size_t)(cc * nb + b) * 16 + (kg & 1) * 8);
            const f32x4 si = __builtin_amdgcn_mfma_f32_16x16x32_f16(As, Bs, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            const float yd = xd_s[cc * nb + b];
            float dy[4], dmy[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t hx = (uint32_t)__shfl((int)h.x, 4 * kg + q);  // d | dmin of row 4kg + q
                dy[q] = __fmul_rn(dev_fp16_to_fp32((uint16_t)(hx & 0xFFFF)), yd);
                dmy[q] = __fmul_rn(dev_fp16_to_fp32((uint16_t)(hx >> 16)), yd);
            }
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const f2v d2 = {dy[2 * hq], dy[2 * hq + 1]}, dm2 = {dmy[2 * hq], dmy[2 * hq + 1]};
#pragma unroll
                for (int l = 0; l < 8; ++l) tp[u][l][hq] = d2 * f2v{acc[l][2 * hq], acc[l][2 * hq + 1]};
                tq[u][hq] = dm2 * f2v{si[2 * hq], si[2 * hq + 1]};
            }
        }
    };

    // the relay: wave w' folds its blocks into the running sums in block order, hands them on; the
    // last wave of the relay adds sumf + sums[0..7] and stores
    float * rl = relay + ((size_t)sub * 64 + lane) * 36;
    const int nblk = nb - w * BPW < BPW ? nb - w * BPW : BPW;  // the last wave may own fewer blocks
    auto relay_store = [&](int64_t tt) __attribute__((always_inline)) {
        f2v sums[8][2], sumf[2];
#pragma unroll
        for (int hq = 0; hq < 2; ++hq) {
            sumf[hq] = f2v{0.f, 0.f};
#pragma unroll
            for (int l = 0; l < 8; ++l) sums[l][hq] = f2v{0.f, 0.f};
        }
        for (int step = 0; step < nwt; ++step) {
            if (step == w) {
                if (w > 0) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {  // sums[2k], sums[2k + 1]: 4 floats
                        const float4 a = *(const float4 *)(rl + 4 * k);
                        const float4 c = *(const float4 *)(rl + 16 + 4 * k);
                        sums[2 * k][0] = f2v{a.x, a.y}, sums[2 * k][1] = f2v{a.z, a.w};
                        sums[2 * k + 1][0] = f2v{c.x, c.y}, sums[2 * k + 1][1] = f2v{c.z, c.w};
                    }
                    const float4 f = *(const float4 *)(rl + 32);
                    sumf[0] = f2v{f.x, f.y}, sumf[1] = f2v{f.z, f.w};
                }
#pragma unroll
                for (int u = 0; u < BPW; ++u) {
                    if (u >= nblk) break;  // wave-uniform
#pragma unroll
                    for (int hq = 0; hq < 2; ++hq) {
#pragma unroll
                        for (int l = 0; l < 8; ++l) sums[l][hq] = sums[l][hq] + tp[u][l][hq];
                        sumf[hq] = sumf[hq] - tq[u][hq];
                    }
                }
                if (w < nwt - 1) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        *(float4 *)(rl + 4 * k) = make_float4(sums[2 * k][0].x, sums[2 * k][0].y, sums[2 * k][1].x, sums[2 * k][1].y);
                        *(float4 *)(rl + 16 + 4 * k) =
                            make_float4(sums[2 * k + 1][0].x, sums[2 * k + 1][0].y, sums[2 * k + 1][1].x, sums[2 * k + 1][1].y);
                    }
                    *(float4 *)(rl + 32) = make_float4(sumf[0].x, sumf[0].y, sumf[1].x, sumf[1].y);
                }
            }
            if (step < nwt - 1) __syncthreads();
        }
        float tot[4];
        if (w == nwt - 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                tot[q] = sumf[q >> 1][q & 1];
#pragma unroll
                for (int l = 0; l < 8; ++l) tot[q] = __fadd_rn(tot[q], sums[l][q >> 1][q & 1]);
            }
        }
        if constexpr (SW) {  // out = silu(gate) * up, by the up tile's last wave
            float * xg = relay + 2 * 64 * 36;  // [64 lanes][4] after both relays
            if (w == nwt - 1 && sub == 0) *(float4 *)(xg + lane * 4) = make_float4(tot[0], tot[1], tot[2], tot[3]);
            __syncthreads();
            if (w == nwt - 1 && sub == 1) {
                const float4 g4 = *(const float4 *)(xg + lane * 4);
                const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int64_t flat = tt * 16 + 4 * kg + q;
                    if (r < M && flat < NR) j.Y[0][(c0 + r) * j.ycs[0] + flat * j.yrs[0]] = __fmul_rn(dev_silu(gv[q]), tot[q]);
                }
            }
        } else if (w == nwt - 1) {
            const int mat = tile_mat(tt);
            const int64_t row0 = tile_row0(tt, mat);
            const int64_t rows_m = job_roff(j, mat + 1) - job_roff(j, mat);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t rr = row0 + 4 * kg + q;
                if (r < M && rr < rows_m) gemv_store<8>(j, mat, rr, c0 + r, tot[q]);
            }
        }
    };

    if constexpr (LOOP) {
        const int64_t G = gridDim.x;
        for (; t < T; t += 2 * G) {
            terms(B0{});
            load_w(B1{}, t + G);  // clamped: the loads are unconditional
            TTS_TS(j, 3);
            relay_store(t);
            TTS_TS(j, 4);
            __syncthreads();  // the relay buffer is reused by the next tile
            if (t + G >= T) break;
            terms(B1{});
            load_w(B0{}, t + 2 * G);
            relay_store(t + G);
            __syncthreads();
        }
    } else {
        terms(B0{});
        TTS_TS(j, 3);
        relay_store(t);
        TTS_TS(j, 4);
        if constexpr (CTW > 1) {
            for (int k = 1; k < ntile; ++k) {  // the next column tile: same weight registers, its operands
                __syncthreads();  // the relay buffer is reused
                c0 = 16 * (ct0 + k);
                M = min(16, (int)j.M - c0);
                nslot = M * nb + 1;
                b16 = (_Float16 *)(smem + (size_t)k * bqb);
                sbs = b16 + (size_t)nslot * QK_K;
                xd_s = (float *)(sbs + (size_t)nslot * 16);
                cc = r < M ? r : M - 1;
                terms(B0{});
                relay_store(t);
            }
        }
    }
    TTS_TS(j, 5);
}

// ------------------------------------------------------------------------------------------
// Many-column Q4_K GEMM for prompt passes (k_gemm_q4K_pf): the K-relay kernel's per-block arithmetic
// (the same exact-integer f16 MFMA dots, the same rounded f32 terms) with the work cut the other way.
// At prefill sizes a K-relay workgroup computes one 16 x 16 (row tile, column tile) pair and copies
// its column tile's whole operand (16 columns x K) into LDS for it: a 1024 x 1024 matrix at 576
// columns moves 64 x 36 such copies of 35 KB through L2.  Here the operand tile is copied into LDS
// once for 4 x 2 row tiles (8 x 2 with TTS_HIP_OPT_GEMM_PF_NW = 8): each wave owns two row tiles of the column tile for the WHOLE row, every
// block in ascending order, so ggml's chain (sums[l] += p_l, sumf -= q, then sumf + sums[0..7]) runs
// in the wave's registers with no relay and no barrier; a block's operand fragments (from LDS) serve
// both row tiles.  The next block's weights are requested before the current block's MFMAs.  Same additions in the same order as vec_dot_q4_K_q8_K:
// bit-identical.  Operands: k_quant_mf's layout, one bq_tile per 16-column tile (j.bq, j.bq_tile).
constexpr int PF_RS = 2;                 // row tiles per wave
constexpr int PF_SLOT = QK_K + 8;        // halves per operand slot: columns 528 B apart, 16 B off the LDS bank period
template <int NB, bool LANE, int NW = 4>
__global__ __launch_bounds__(64 * NW) void k_gemm_q4K_pf(GemvJob j) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    constexpr int RS = PF_RS;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 15, kg = lane >> 4;
    const int ct = blockIdx.y;
    const int c0 = 16 * ct;
    const int M = min(16, (int)j.M - c0);
    const int cc = r < M ? r : M - 1;
    const int nslot = M * NB + 1;
    TTS_TS(j, 0);
    // the column tile's operands into LDS (the same bytes the K-relay kernel DMAs)
    {
        const char * src = j.bq + (size_t)ct * j.bq_tile;
        const int nck = (int)(((size_t)nslot * (2 * PF_SLOT + 32 + 4) + 1023) >> 10);
        for (int i = wave; i < nck; i += NW)
            __builtin_amdgcn_global_load_lds(gptr(src + (size_t)i * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void *)(smem + (size_t)i * 1024), 16, 0, 0);
    }
    const _Float16 * const b16 = (const _Float16 *)smem;
    const _Float16 * const sbs = b16 + (size_t)nslot * PF_SLOT;
    const float * const xd = (const float *)(sbs + (size_t)nslot * 16);
    const int64_t T = job_rows(j) / 16;  // launcher: whole row tiles
    const int64_t tw = ((int64_t)blockIdx.x * NW + wave) * RS;  // this wave's first row tile
    auto mat_of = [&](int64_t flat) {
        int mt = 0;
        while (mt + 1 < j.nmat && flat >= job_roff(j, mt + 1)) ++mt;
        return mt;
    };
    const uint8_t * wp[RS];  // LANE: this lane's row; tiled: its 4-row group (row & 3 in ri[])
    int ri[RS];
#pragma unroll
    for (int rs = 0; rs < RS; ++rs) {
        const int64_t t = tw + rs < T ? tw + rs : T - 1;
        const int mat = __builtin_amdgcn_readfirstlane(mat_of(t * 16));
        const int64_t row = t * 16 - job_roff(j, mat) + r;
        if constexpr (LANE) wp[rs] = j.W[mat] + row * j.w_row_bytes;
        else wp[rs] = j.W[mat] + (row >> 2) * NB * 576;
        ri[rs] = (int)(row & 3);
    }
    u32x4 hd[2][RS], qa[2][RS], qb[2][RS];
    auto load_w = [&](auto BUF, int b) __attribute__((always_inline)) {
        constexpr int bf = decltype(BUF)::value;
#pragma unroll
        for (int rs = 0; rs < RS; ++rs) {
            if constexpr (LANE) {
                const uint8_t * bp = wp[rs] + (int64_t)b * 144;
                hd[bf][rs] = TTS_WLOAD((const u32x4 *)bp);
#pragma unroll
                for (int l = 0; l < 4; ++l) {
                    qa[bf][rs][l] = TTS_WLOAD((const uint32_t *)(bp + 16 + l * 16 + kg * 4));
                    qb[bf][rs][l] = TTS_WLOAD((const uint32_t *)(bp + 16 + (l + 4) * 16 + kg * 4));
                }
            } else {
                const uint8_t * bp = wp[rs] + (int64_t)b * 576;
                hd[bf][rs] = TTS_WLOAD((const u32x4 *)(bp + ri[rs] * 16));
                qa[bf][rs] = TTS_WLOAD((const u32x4 *)(bp + 64 + ((kg * 2) * 4 + ri[rs]) * 16));
                qb[bf][rs] = TTS_WLOAD((const u32x4 *)(bp + 64 + ((kg * 2 + 1) * 4 + ri[rs]) * 16));
            }
        }
        TTS_PIN_LOADS();
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    load_w(B0{}, 0);
    TTS_TS(j, 1);
    __syncthreads();  // the operand DMA has landed (the compiler waits for all of it here)
    TTS_TS(j, 2);
    f2v sums[RS][8][2], sumf[RS][2];
#pragma unroll
    for (int rs = 0; rs < RS; ++rs)
#pragma unroll
        for (int hq = 0; hq < 2; ++hq) {
            sumf[rs][hq] = f2v{0.f, 0.f};
#pragma unroll
            for (int l = 0; l < 8; ++l) sums[rs][l][hq] = f2v{0.f, 0.f};
        }
    // one block: the integer dots of k_gemv_q4K_kr's terms, folded into the chain at once
    auto block = [&](auto BUF, int b) __attribute__((always_inline)) {
        constexpr int bf = decltype(BUF)::value;
        const size_t slot = (size_t)cc * NB + b;
        const _Float16 * bsl = b16 + slot * PF_SLOT + kg * 8;
        f16x8 B[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) B[l] = *(const f16x8 *)(bsl + l * 32);
        const f16x8 Bs = *(const f16x8 *)(sbs + slot * 16 + (kg & 1) * 8);
        const float yd = xd[slot];
#pragma unroll
        for (int rs = 0; rs < RS; ++rs) {
            const u32x4 h = hd[bf][rs];
            const uint32_t sc_lo = h.y & 0x3F3F3F3Fu, mn_lo = h.z & 0x3F3F3F3Fu;
            const uint32_t sc_hi = (h.w & 0x0F0F0F0Fu) | ((h.y >> 2) & 0x30303030u);
            const uint32_t mn_hi = ((h.w >> 4) & 0x0F0F0F0Fu) | ((h.z >> 2) & 0x30303030u);
            const uint32_t sw = (kg < 2 ? sc_lo : sc_hi) >> ((kg & 1) * 16);
            const _Float16 s0 = (_Float16)(float)(sw & 0xFF), s1 = (_Float16)(float)((sw >> 8) & 0xFF);
            const f16x2 S0 = {s0, s0}, S1 = {s1, s1};
            const _Float16 o0 = (_Float16)(-1024.f * (float)(sw & 0xFF)), o1 = (_Float16)(-1024.f * (float)((sw >> 8) & 0xFF));
            const f16x2 O0 = {o0, o0}, O1 = {o1, o1};
            f32x4 acc[8];
#pragma unroll
            for (int l = 0; l < 8; ++l) {
                const uint32_t D = l < 4 ? qa[bf][rs][l & 3] : qb[bf][rs][l & 3];
                const uint32_t lo = D & 0x0F0F0F0Fu, hi = (D >> 4) & 0x0F0F0F0Fu;
                const f16x2 a0 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C010C00u), S0, O0);
                const f16x2 a1 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C030C02u), S0, O0);
                const f16x2 a2 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C010C00u), S1, O1);
                const f16x2 a3 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C030C02u), S1, O1);
                const f16x8 A = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, a3.x, a3.y};
                acc[l] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B[l], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
            const _Float16 mm = (_Float16)(kg == 0 ? 1.f : kg == 1 ? 64.f : 0.f);
            const f16x2 MM = {mm, mm}, OFF = {(_Float16)-1024.f, (_Float16)-1024.f};
            const f16x2 m0 = (byte2_f16_biased(mn_lo, 0x0C010C00u) + OFF) * MM;
            const f16x2 m1 = (byte2_f16_biased(mn_lo, 0x0C030C02u) + OFF) * MM;
            const f16x2 m2 = (byte2_f16_biased(mn_hi, 0x0C010C00u) + OFF) * MM;
            const f16x2 m3 = (byte2_f16_biased(mn_hi, 0x0C030C02u) + OFF) * MM;
            const f16x8 As = {m0.x, m0.y, m1.x, m1.y, m2.x, m2.y, m3.x, m3.y};
            const f32x4 si = __builtin_amdgcn_mfma_f32_16x16x32_f16(As, Bs, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            float dy[4], dmy[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t hx = (uint32_t)__shfl((int)h.x, 4 * kg + q);  // d | dmin of row 4kg + q
                dy[q] = __fmul_rn(dev_fp16_to_fp32((uint16_t)(hx & 0xFFFF)), yd);
                dmy[q] = __fmul_rn(dev_fp16_to_fp32((uint16_t)(hx >> 16)), yd);
            }
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const f2v d2 = {dy[2 * hq], dy[2 * hq + 1]}, dm2 = {dmy[2 * hq], dmy[2 * hq + 1]};
#pragma unroll
                for (int l = 0; l < 8; ++l) sums[rs][l][hq] = sums[rs][l][hq] + d2 * f2v{acc[l][2 * hq], acc[l][2 * hq + 1]};
                sumf[rs][hq] = sumf[rs][hq] - dm2 * f2v{si[2 * hq], si[2 * hq + 1]};
            }
        }
    };
    // pairs of blocks, not unrolled (an unrolled chain lets the compiler hoist every block's operand
    // reads and spill); NB is even: each pair's second block's weights are requested before its
    // first block's MFMAs, the next pair's first block's before its second's
#pragma unroll 1
    for (int b = 0; b < NB; b += 2) {
        load_w(B1{}, b + 1);
        block(B0{}, b);
        if (b + 2 < NB) load_w(B0{}, b + 2);
        block(B1{}, b + 1);
        if (b == 0) TTS_TS(j, 3);
    }
    TTS_TS(j, 4);
#pragma unroll
    for (int rs = 0; rs < RS; ++rs) {
        if (tw + rs >= T) break;  // (wave-uniform)
        const int64_t t = tw + rs;
        const int mat = __builtin_amdgcn_readfirstlane(mat_of(t * 16));
        const int64_t row0 = t * 16 - job_roff(j, mat);
        const int64_t rows_m = job_roff(j, mat + 1) - job_roff(j, mat);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float tot = sumf[rs][q >> 1][q & 1];
#pragma unroll
            for (int l = 0; l < 8; ++l) tot = __fadd_rn(tot, sums[rs][l][q >> 1][q & 1]);
            const int64_t rr = row0 + 4 * kg + q;
            if (r < M && rr < rows_m) gemv_store<8>(j, mat, rr, c0 + r, tot);
        }
    }
    TTS_TS(j, 5);
}
// ------------------------------------------------------------------------------------------
// Matrix-core Q4_K GEMV for latency-bound decode matrices (k_gemv_q4K_ks).  Parler's matrices are
// 0.6-2.4 MB: the row phase of the VALU kernels is ~1.2-2.5 us of dependent integer dots at one wave
// per SIMD, and k_gemv_q4K_mf streams a tile's blocks through ONE wave.  Here a workgroup owns one
// 16-row tile and splits its work units (block b, residue half rh) over its waves, so every weight
// load of the tile is issued at kernel entry (before the prologue) and the integer dots are a few
// MFMAs per wave:
//   unit (b, rh): 4 v_mfma_f32_16x16x32_f16 for residues l = 4rh..4rh+3 (+ the mins MFMA when
//   rh = 0), exactly the integers of k_gemv_q4K_mf; the lane turns them into ggml's two per-block
//   terms p_l = (d*yd)*aux32[l] and q = (dmin*yd)*sumi, each rounded as the sequential code rounds
//   them, and writes them to LDS;
//   chain: lane (row, column, l) runs ggml's chain over the blocks in ascending order
//   (sums[l] += p_l, sumf -= q, then sumf += sums[0..7] across the octet) -- the same additions in
//   the same order as vec_dot_q4_K_q8_K, so the output is bit-identical.
// LDS: the Q8_K B operands of all M <= 8 columns (q4k_prologue, MF layout), then the terms
// p[nb][16 rows][8 columns][8] and q[nb][16 rows][8 columns].  Large grids loop over tiles.
template <int PRO, int NCH, int UPW, int NWMAX>
__global__ __launch_bounds__(64 * NWMAX) void k_gemv_q4K_ks(GemvJob j) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nb = (int)(j.K / QK_K);
    const int M = (int)j.M;
    const int nslot = M * nb + 1;  // + the prologue's trash slot
    _Float16 * b16 = (_Float16 *)smem;                   // [nslot][256]
    _Float16 * sbs = b16 + (size_t)nslot * QK_K;         // [nslot][16]
    float * xd_s = (float *)(sbs + (size_t)nslot * 16);  // [nslot]
    float * tp = (float *)(smem + al16((size_t)nslot * (2 * QK_K + 32 + 4)));  // [nb][16][8][8]
    float * tq = tp + (size_t)nb * 1024;                                       // [nb][16][8]

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
    const int r = lane & 15, kg = lane >> 4;
    const int cc = r < M ? r : M - 1;  // B / C column (padding columns compute and are dropped)
    const int nu = 2 * nb;
    const int64_t T = job_rows(j) / 16;  // launcher: every matrix a multiple of 16 rows, so a tile is in one matrix
    auto mat_of = [&](int64_t flat) {
        int mt = 0;
        while (mt + 1 < j.nmat && flat >= job_roff(j, mt + 1)) ++mt;
        return mt;
    };

    u32x4 hd[UPW], qv[UPW];
    auto load = [&](int64_t t) {
        const int mat = mat_of(t * 16);
        const int64_t row = t * 16 - job_roff(j, mat) + r;
        const uint8_t * wt = j.W[mat] + (row >> 2) * nb * 576;
        const int ri = (int)(row & 3);
#pragma unroll
        for (int k = 0; k < UPW; ++k) {  // unconditional (clamped): every load issues before any use
            const int u = min(wave + k * nw, nu - 1);
            const uint8_t * bp = wt + (int64_t)(u >> 1) * 576;
            hd[k] = TTS_WLOAD((const u32x4 *)(bp + ri * 16));
            qv[k] = TTS_WLOAD((const u32x4 *)(bp + 64 + ((kg * 2 + (u & 1)) * 4 + ri) * 16));
        }
        TTS_PIN_LOADS();
    };

    // the integer dots of this wave's units -> the terms in LDS
    auto units = [&]() {
#pragma unroll
        for (int k = 0; k < UPW; ++k) {
            const int u = wave + k * nw;
            if (u >= nu) break;  // wave-uniform
            const int b = u >> 1, rh = u & 1;
            const u32x4 h = hd[k];
            const uint32_t sc_lo = h.y & 0x3F3F3F3Fu, mn_lo = h.z & 0x3F3F3F3Fu;
            const uint32_t sc_hi = (h.w & 0x0F0F0F0Fu) | ((h.y >> 2) & 0x30303030u);
            const uint32_t mn_hi = ((h.w >> 4) & 0x0F0F0F0Fu) | ((h.z >> 2) & 0x30303030u);
            const uint32_t sw = (kg < 2 ? sc_lo : sc_hi) >> ((kg & 1) * 16);
            const _Float16 s0 = (_Float16)(float)(sw & 0xFF), s1 = (_Float16)(float)((sw >> 8) & 0xFF);
            const f16x2 S0 = {s0, s0}, S1 = {s1, s1};
            const _Float16 o0 = (_Float16)(-1024.f * (float)(sw & 0xFF)), o1 = (_Float16)(-1024.f * (float)((sw >> 8) & 0xFF));
            const f16x2 O0 = {o0, o0}, O1 = {o1, o1};
            const _Float16 * bsl = b16 + (size_t)(cc * nb + b) * QK_K + kg * 8 + rh * 128;
            f32x4 acc[4];
#pragma unroll
            for (int li = 0; li < 4; ++li) {
                const uint32_t D = qv[k][li];
                const uint32_t lo = D & 0x0F0F0F0Fu, hi = (D >> 4) & 0x0F0F0F0Fu;
                const f16x2 a0 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C010C00u), S0, O0);
                const f16x2 a1 = __builtin_elementwise_fma(byte2_f16_biased(lo, 0x0C030C02u), S0, O0);
                const f16x2 a2 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C010C00u), S1, O1);
                const f16x2 a3 = __builtin_elementwise_fma(byte2_f16_biased(hi, 0x0C030C02u), S1, O1);
                const f16x8 A = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, a3.x, a3.y};
                const f16x8 B = *(const f16x8 *)(bsl + li * 32);
                acc[li] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
            f32x4 si = {0.f, 0.f, 0.f, 0.f};
            if (rh == 0) {
                const _Float16 mm = (_Float16)(kg == 0 ? 1.f : kg == 1 ? 64.f : 0.f);
                const f16x2 MM = {mm, mm}, OFF = {(_Float16)-1024.f, (_Float16)-1024.f};
                const f16x2 m0 = (byte2_f16_biased(mn_lo, 0x0C010C00u) + OFF) * MM;
                const f16x2 m1 = (byte2_f16_biased(mn_lo, 0x0C030C02u) + OFF) * MM;
                const f16x2 m2 = (byte2_f16_biased(mn_hi, 0x0C010C00u) + OFF) * MM;
                const f16x2 m3 = (byte2_f16_biased(mn_hi, 0x0C030C02u) + OFF) * MM;
                const f16x8 As = {m0.x, m0.y, m1.x, m1.y, m2.x, m2.y, m3.x, m3.y};
                const f16x8 Bs = *(const f16x8 *)(sbs + (size_t)(cc * nb + b) * 16 + (kg & 1) * 8);
                si = __builtin_amdgcn_mfma_f32_16x16x32_f16(As, Bs, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
            const float yd = xd_s[cc * nb + b];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t hx = (uint32_t)__shfl((int)h.x, 4 * kg + q);  // d | dmin of row 4kg + q
                const float dy = __fmul_rn(dev_fp16_to_fp32((uint16_t)(hx & 0xFFFF)), yd);
                const int pr = (b * 16 + 4 * kg + q) * 8 + r;  // (block, row, column)
                if (r < M) {
                    *(float4 *)(tp + (size_t)pr * 8 + rh * 4) =
                        make_float4(__fmul_rn(dy, acc[0][q]), __fmul_rn(dy, acc[1][q]), __fmul_rn(dy, acc[2][q]), __fmul_rn(dy, acc[3][q]));
                    if (rh == 0) tq[pr] = __fmul_rn(__fmul_rn(dev_fp16_to_fp32((uint16_t)(hx >> 16)), yd), si[q]);
                }
            }
        }
    };

    int64_t t = blockIdx.x;
    TTS_TS(j, 0);
    auto mid = [&]() {
        if (t < T) load(t);
        TTS_TS(j, 1);
    };
    if constexpr (PRO == PRO_COPY) {  // operands from k_quant_mf (see k_gemv_q4K_mf)
        const int nck = (int)(j.bq_bytes >> 10);
        for (int i = wave; i < nck; i += nw)
            __builtin_amdgcn_global_load_lds(gptr(j.bq + (size_t)i * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void *)(smem + (size_t)i * 1024), 16, 0, 0);
        TTS_PIN_LOADS();
        load(t < T ? t : T - 1);
    } else {
        q4k_prologue<PRO, NCH, true>(j, nb, nullptr, xd_s, nullptr, b16, sbs, mid);
    }
    TTS_TS(j, 2);
    __syncthreads();
    TTS_TS(j, 3);
    for (; t < T; t += gridDim.x) {
        units();
        if (t + gridDim.x < T) load(t + gridDim.x);  // the next tile's weights fly during the chain
        __syncthreads();
        const int mat = mat_of(t * 16);
        TTS_TS(j, 4);
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) {  // i = (row * 8 + column) * 8 + l
            // every term is read before the chain starts (one LDS round trip, not one per block)
            float p[NCH], q[NCH];
#pragma unroll
            for (int b = 0; b < NCH; ++b) {
                const int bb = min(b, nb - 1);
                p[b] = tp[(size_t)bb * 1024 + i];
                q[b] = tq[bb * 128 + (i >> 3)];
            }
            float sums = 0.f, sumf = 0.f;
#pragma unroll
            for (int b = 0; b < NCH; ++b) {
                if (b < nb) {
                    sums = __fadd_rn(sums, p[b]);
                    sumf = __fsub_rn(sumf, q[b]);
                }
            }
            const float tot = q4k_octet_total(sumf, sums);
            const int col = (i >> 3) & 7, row = i >> 6;
            if ((i & 7) == 0 && col < M) gemv_store<8>(j, mat, t * 16 - job_roff(j, mat) + row, col, tot);
        }
        __syncthreads();
    }
    TTS_TS(j, 5);
}

// Cross-attention query GEMV + attention in one launch (Parler model.cpp:583-594: q = W_q
// LN(x), then cont(K) -> mul_mat -> soft_max_ext -> mul_mat(V) -> permute -> cont over the n_enc
// encoder positions).  Workgroup (h, b) owns head h of prompt b: 8 waves x 8 rows = the head's 64
// query rows for column b alone (MC = 1 lane mapping: row slot s = lane >> 3, residue l = lane & 7),
// with the LN / Q8_K prologue of that one column.  The 64 query values go to LDS and the last wave
// runs the short-context attention of k_attn_small<64> on them (lane = key position, every sum in
// the oracle's sequential order).  Each value is computed exactly as by the two separate launches
// (same per-(row, column) Q4_K order, same attention arithmetic), so the result is bit-identical;
// the launch and the attention kernel's whole latency chain disappear.  The attention's K, V and
// mask are requested at kernel entry, next to the weight rows.
template <int PRO>
__global__ __launch_bounds__(576) void k_gemv_q4K_xattn(GemvJob j, XAttnArgs a) {
    // waves 0..7: the query GEMV (8 rows each); wave 8: the attention, whose K / V loads are issued at
    // entry and never share a code path with the prologue's activation loads (a join of paths with
    // unequal loads in flight makes the compiler wait for all of them before the activation's use)
    constexpr int HD = 64, NW = 8, F = HD / 4, VB = 8;
    __shared__ __attribute__((aligned(16))) int8_t xq_s[5 * QK_K];  // nb <= 4 blocks + trash slot
    __shared__ float xd_s[8];
    __shared__ __attribute__((aligned(16))) int16_t xs_s[5 * 8];
    __shared__ float s_q[HD];
    const int h = blockIdx.x, b = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int l = lane & 7, s = lane >> 3;
    const int nb = (int)(j.K / QK_K);
    // attention operands for the attention wave (position p = lane)
    const int P = a.pseq ? a.pseq[b] : a.P;
    const int p = min(lane, P - 1);
    float4 kr[F];
    float vv[VB];
    float mk = 0.f;
    const int bk = b / (a.B / (int)a.k.ne[3]), bv = b / (a.B / (int)a.v.ne[3]);  // K/V shared across prompts or not
    const char * kbase = a.k.data + (int64_t)h * a.k.nb[2] + (int64_t)bk * a.k.nb[3] + (a.koff ? a.koff[b] : 0);
    const char * vbase = a.v.data + (int64_t)h * a.v.nb[2] + (int64_t)bv * a.v.nb[3] + (a.voff ? a.voff[b] : 0);
    u32x4 hdr[4], q[4];
    if (wave < NW) {
        const int64_t row = (int64_t)h * HD + wave * 8 + s;
        const uint8_t * wr = j.W[0] + row * j.w_row_bytes;
        // weight rows are requested behind the prologue's activation loads
        auto mid = [&]() {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t bo = (int64_t)min(u, nb - 1) * 144;
                hdr[u] = TTS_WLOAD((const u32x4 *)(wr + bo));
                q[u] = TTS_WLOAD((const u32x4 *)(wr + bo + 16 + l * 16));
            }
        };
        // this workgroup's column b (head 0's workgroup writes its LN output)
        ProOv ov;
        ov.nwaves = NW;
        ov.xcol = j.x + (int64_t)b * j.xcs;
        ov.lncol = j.lnout && h == 0 ? j.lnout + (int64_t)b * j.locs : nullptr;
        q4k_prologue<PRO, 4>(j, nb, xq_s, xd_s, xs_s, nullptr, nullptr, mid, ov);
    } else {
#pragma unroll
        for (int c = 0; c < F; ++c) kr[c] = *(const float4 *)(kbase + (int64_t)p * a.k.nb[1] + 16 * c);
#pragma unroll
        for (int u = 0; u < VB; ++u) vv[u] = *(const float *)(vbase + (int64_t)lane * a.v.nb[1] + (int64_t)min(u, P - 1) * a.v.nb[0]);
        mk = *(a.mask ? a.mask + (a.moff ? a.moff[b] : (int64_t)b * a.mbs) + p : (const float *)kbase);  // unconditional: no branch join before the barrier
    }
    __syncthreads();
    if (wave < NW) {
        float sums = 0.f, sumf = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) q4k_block(hdr[u], q[u], xq_s, xs_s, xd_s, min(u, nb - 1), l, u < nb, sums, sumf);
        const float tot = q4k_octet_total(sumf, sums);
        if (l == 0) s_q[wave * 8 + s] = tot;
    }
    __syncthreads();
    if (wave != NW) return;
    // ---- k_attn_small<64> on (h, b) with q from LDS ----
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < F; ++c) {
        acc += (double)__fmul_rn(kr[c].x, s_q[4 * c + 0]);
        acc += (double)__fmul_rn(kr[c].y, s_q[4 * c + 1]);
        acc += (double)__fmul_rn(kr[c].z, s_q[4 * c + 2]);
        acc += (double)__fmul_rn(kr[c].w, s_q[4 * c + 3]);
    }
    float w = __fmul_rn((float)acc, a.scale);
    if (a.mask) w = __fadd_rn(w, __fmul_rn(1.0f, mk));
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
    double o = 0.0;
    for (int i0 = 0; i0 < P; i0 += VB) {
        if (i0 > 0) {
#pragma unroll
            for (int u = 0; u < VB; ++u) vv[u] = *(const float *)(vbase + (int64_t)lane * a.v.nb[1] + (int64_t)min(i0 + u, P - 1) * a.v.nb[0]);
            TTS_PIN_LOADS();
        }
#pragma unroll
        for (int u = 0; u < VB; ++u) {
            if (i0 + u >= P) break;
            const float pi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pr), i0 + u));
            o += (double)__fmul_rn(pi, vv[u]);
        }
    }
    const int64_t orow = (int64_t)h * HD + lane;
    a.out[(int64_t)b * (a.obs ? a.obs : (int64_t)a.H * HD) + orow] = (float)o;
    if (a.out2) a.out2[(int64_t)b * a.H * HD + orow] = (float)o;
}

// Host checks (caller): Q4_K repacked weights, one matrix of N = H * 64 rows, K <= 1024, M = B
// columns with 16-B aligned, 16-B strided x; K rows 16-B vectors; P <= 64.
void launch_gemv_q4K_xattn(tts_hip_backend * be, const GemvJob & j, const XAttnArgs & a) {
    const dim3 grid((unsigned)a.H, (unsigned)a.B);
    if (j.pro == PRO_LN) hipLaunchKernelGGL(k_gemv_q4K_xattn<PRO_LN>, grid, dim3(576), 0, be->stream, j, a);
    else hipLaunchKernelGGL(k_gemv_q4K_xattn<PRO_QUANT>, grid, dim3(576), 0, be->stream, j, a);
    TTS_HIP_CHECK(hipGetLastError());
}

// Q8_0 x Q8_0 GEMV reproducing ggml_vec_dot_q8_0_q8_0's generic order: per (row, column),
// blocks in ascending order, sumf += (float)sumi * (d_w * d_x).  Phase 1: a thread per
// (row, block) computes the exact int dots for every column -> LDS; phase 2: a lane per
// (row, column) folds its blocks in order.
// PRO (PRO_QUANT / PRO_LN): the workgroup quantizes (after RMS / LayerNorm) the f32 activation itself
// (q4k_prologue with Q8_0 output: quantize_row_q8_0 per 32 elements, K % 256 == 0), with this thread's
// first (row, block) weights requested before it; PRO = 0: the activation was quantized by
// k_quantize_q8_0 (j.aq).  One launch instead of norm + quantize + GEMV.
template <int MC, int PRO = 0>
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
    float * xd_s = (float *)(smem + al16((size_t)MC * j.K + (PRO ? QK_K : 0)));  // + the prologue's trash slot
    int * s_s = (int *)((char *)xd_s + al16(sizeof(float) * (MC * nb + (PRO ? QK_K / QK8_0 : 0))));
    float * f_s = (float *)((char *)s_s + al16(sizeof(int) * (size_t)RW * nb * MC));
    const int npairs = rows * nb;
    // this thread's first (row, block): weights in registers before the prologue (clamped, unconditional)
    int wv0[8];
    uint16_t dw0;
    {
        const int p = min((int)threadIdx.x, npairs - 1);
        const int r = p / nb, b = p % nb;
        const uint16_t * bp = (const uint16_t *)(W + (row0 + r) * j.w_row_bytes + (int64_t)b * 34);
        dw0 = *gptr(bp);
#pragma unroll
        for (int k = 0; k < 8; ++k) wv0[k] = (int)*gptr(bp + 1 + 2 * k) | ((int)*gptr(bp + 2 + 2 * k) << 16);
    }
    TTS_PIN_LOADS();
    if constexpr (PRO != 0) {
        q4k_prologue<PRO, 16, false, NoMid, true>(j, (int)(j.K / QK_K), xq_s, xd_s, nullptr);
    } else {
        const int4 * src = (const int4 *)j.aq.qs;
        int4 * dst = (int4 *)xq_s;
        const int n16 = (int)((int64_t)M * j.K / 16);
        for (int i = threadIdx.x; i < n16; i += 256) dst[i] = src[i];
        for (int i = threadIdx.x; i < M * nb; i += 256) xd_s[i] = j.aq.d[i];
    }
    __syncthreads();
    for (int p = threadIdx.x; p < npairs; p += 256) {
        const int r = p / nb, b = p % nb;
        float dw;
        int wv[8];
        if (p == (int)threadIdx.x) {
            dw = dev_fp16_to_fp32(dw0);
#pragma unroll
            for (int k = 0; k < 8; ++k) wv[k] = wv0[k];
        } else {
            const uint16_t * bp = (const uint16_t *)(W + (row0 + r) * j.w_row_bytes + (int64_t)b * 34);
            dw = dev_fp16_to_fp32(bp[0]);
#pragma unroll
            for (int k = 0; k < 8; ++k) wv[k] = (int)bp[1 + 2 * k] | ((int)bp[2 + 2 * k] << 16);
        }
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

// Q8_0 GEMV, slab form (K % 256 == 0, 16-B aligned weights; decode, <= 8 columns).  A workgroup owns RW
// consecutive rows, i.e. one contiguous RW * row_bytes slab of the matrix: the whole slab is requested
// up front by LDS-DMA (16 B per lane, fully coalesced, no registers held), so each CU has tens of KB in
// flight and the launch costs about one memory latency plus slab / per-CU bandwidth, instead of one
// dependent 34-B block fetch per (row, block) round.  Then, from LDS:
//   terms: a thread per (row, block pair) -- the pair (2k, 2k+1) spans 68 B at a 4-B aligned offset
//          (17 dwords; block 2k's quants are the funnel-shifted dwords) -- eight sdot4 per block and
//          column, term = (float)sumi * (d_w * d_x) as ggml_vec_dot_q8_0_q8_0 rounds it;
//   chain: a thread per (row, column) adds the nb terms in block order (sumf += term, from 0).
// So the result is bit-identical to ggml's generic order.  The activation's Q8_0 blocks come from the
// quantize launch (PRO = 0, DMA'd with the slab) or from the prologue (PRO_QUANT / PRO_LN, whose
// activation loads are issued before the slab DMA so they do not queue behind it).
// LDS: slab al1K(RW*row_bytes) | xq al1K(MC*K + 256) | xd al1K(4*(MC*nb + 8)) | terms 4*RW*MC*nb.
__host__ __device__ constexpr int64_t al1k(int64_t v) { return (v + 1023) & ~(int64_t)1023; }
// LDS-DMA of `bytes` (a multiple of 16) from 16-B aligned global `src` to LDS `dst`; lanes past the end
// re-read the last 16 B and land in the 1 KB slack after dst + bytes
__device__ __forceinline__ void dma_span(char * dst, const char * src, int64_t bytes, int wave, int nw, int lane) {
    const int nck = (int)((bytes + 1023) >> 10);
    for (int i = wave; i < nck; i += nw) {
        int64_t off = (int64_t)i * 1024 + lane * 16;
        off = off < bytes - 16 ? off : bytes - 16;
        __builtin_amdgcn_global_load_lds(gptr(src + off), (__attribute__((address_space(3))) void *)(dst + (size_t)i * 1024), 16, 0, 0);
    }
}
static size_t q80s_lds(int MC, int64_t K, int RW) {
    const int64_t nb = K / QK8_0, rb = nb * 34;
    return (size_t)(al1k(RW * rb) + al1k(MC * K + QK_K) + al1k(4 * (MC * nb + 8)) + 4 * (int64_t)RW * MC * nb);
}
template <int MC, int PRO = 0>
__global__ __launch_bounds__(256) void k_gemv_q8_0s(GemvJob j, int RW) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = (int)(j.K / QK8_0), nbp = nb >> 1;
    const int64_t rb = j.w_row_bytes;
    const int mat = blockIdx.y;
    const int64_t row0 = (int64_t)blockIdx.x * RW;
    const int rows = (int)((j.N - row0) < RW ? (j.N - row0) : RW);
    const int M = j.M;
    char * ws = smem;
    int8_t * xq_s = (int8_t *)(smem + al1k(RW * rb));
    float * xd_s = (float *)((char *)xq_s + al1k(MC * j.K + QK_K));
    float * T = (float *)((char *)xd_s + al1k(4 * (MC * nb + 8)));
    const char * slab = (const char *)j.W[mat] + row0 * rb;
    auto dma_slab = [&]() { dma_span(ws, slab, rows * rb, wave, 4, lane); };
    if constexpr (PRO != 0) {
        struct Mid {
            decltype(dma_slab) & f;
            __device__ void operator()() const { f(); }
        };
        q4k_prologue<PRO, 16, false, Mid, true>(j, (int)(j.K / QK_K), xq_s, xd_s, nullptr, nullptr, nullptr, Mid{dma_slab});
    } else {
        dma_slab();
        dma_span((char *)xq_s, (const char *)j.aq.qs, (int64_t)M * j.K, wave, 4, lane);
        dma_span((char *)xd_s, (const char *)j.aq.d, (int64_t)4 * M * nb, wave, 4, lane);
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed (vmcnt, lgkmcnt 0)
    __syncthreads();
    for (int u = threadIdx.x; u < rows * nbp; u += 256) {
        const int r = u / nbp, k = u - r * nbp;
        const uint32_t * wl = (const uint32_t *)(ws + r * rb + 68 * k);
        uint32_t w[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) w[i] = wl[i];
        const float d0 = dev_fp16_to_fp32((uint16_t)(w[0] & 0xFFFFu));
        const float d1 = dev_fp16_to_fp32((uint16_t)(w[8] >> 16));
        int q0[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) q0[i] = (int)__builtin_amdgcn_alignbit(w[i + 1], w[i], 16);
#pragma unroll
        for (int m = 0; m < MC; ++m) {
            if (m >= M) break;
            const int4 * xb = (const int4 *)(xq_s + (m * nb + 2 * k) * QK8_0);
            const int4 x0 = xb[0], x1 = xb[1], x2 = xb[2], x3 = xb[3];
            int s0 = __builtin_amdgcn_sdot4(q0[0], x0.x, 0, false);
            s0 = __builtin_amdgcn_sdot4(q0[1], x0.y, s0, false);
            s0 = __builtin_amdgcn_sdot4(q0[2], x0.z, s0, false);
            s0 = __builtin_amdgcn_sdot4(q0[3], x0.w, s0, false);
            s0 = __builtin_amdgcn_sdot4(q0[4], x1.x, s0, false);
            s0 = __builtin_amdgcn_sdot4(q0[5], x1.y, s0, false);
            s0 = __builtin_amdgcn_sdot4(q0[6], x1.z, s0, false);
            s0 = __builtin_amdgcn_sdot4(q0[7], x1.w, s0, false);
            int s1 = __builtin_amdgcn_sdot4((int)w[9], x2.x, 0, false);
            s1 = __builtin_amdgcn_sdot4((int)w[10], x2.y, s1, false);
            s1 = __builtin_amdgcn_sdot4((int)w[11], x2.z, s1, false);
            s1 = __builtin_amdgcn_sdot4((int)w[12], x2.w, s1, false);
            s1 = __builtin_amdgcn_sdot4((int)w[13], x3.x, s1, false);
            s1 = __builtin_amdgcn_sdot4((int)w[14], x3.y, s1, false);
            s1 = __builtin_amdgcn_sdot4((int)w[15], x3.z, s1, false);
            s1 = __builtin_amdgcn_sdot4((int)w[16], x3.w, s1, false);
            const float2 xd = *(const float2 *)(xd_s + m * nb + 2 * k);
            float2 t;
            t.x = __fmul_rn((float)s0, __fmul_rn(d0, xd.x));
            t.y = __fmul_rn((float)s1, __fmul_rn(d1, xd.y));
            *(float2 *)(T + (r * MC + m) * nb + 2 * k) = t;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < rows * MC; t += 256) {
        const int r = t / MC, m = t % MC;
        if (m >= M) continue;
        const float4 * tr = (const float4 *)(T + (r * MC + m) * nb);
        float a = 0.f;
        for (int b = 0; b < (nb >> 2); ++b) {
            const float4 v = tr[b];
            a = __fadd_rn(a, v.x);
            a = __fadd_rn(a, v.y);
            a = __fadd_rn(a, v.z);
            a = __fadd_rn(a, v.w);
        }
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
            const f32x4 wv = TTS_WLOAD((const f32x4 *)(w + k));
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

__global__ void k_copy_cols(float * __restrict__ dst, const float * __restrict__ src, int64_t K, int64_t scs) {
    const int64_t m = blockIdx.y;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < K; i += (int64_t)gridDim.x * blockDim.x)
        dst[m * K + i] = src[m * scs + i];
}

void launch_copy_cols(tts_hip_backend * be, float * dst, const float * src, int64_t K, int64_t scs, int64_t M) {
    const unsigned gx = (unsigned)((K + 255) / 256 < 64 ? (K + 255) / 256 : 64);
    hipLaunchKernelGGL(k_copy_cols, dim3(gx, (unsigned)M), dim3(256), 0, be->stream, dst, src, K, scs);
    TTS_HIP_CHECK(hipGetLastError());
}

void launch_repack_q4_K(tts_hip_backend * be, const void * src, void * dst, int64_t nblocks, int inverse) {
    const unsigned grid = (unsigned)((nblocks + 1) / 2);
    hipLaunchKernelGGL(k_repack_q4_K, dim3(grid), dim3(256), 0, be->stream, (const uint8_t *)src, (uint8_t *)dst, nblocks, inverse);
    TTS_HIP_CHECK(hipGetLastError());
}

static size_t q4k_lds(int MC, int64_t K) {
    const int64_t nb = K / QK_K;
    auto a = [](size_t n) { return (n + 15) & ~(size_t)15; };
    const size_t nslot = (size_t)MC * nb + 1;  // kernel: + one trash slot for padding rows
    return a(nslot * QK_K) + a(4 * nslot) + 16 * nslot;
}

// columns per Q4_K launch: the whole Q8_K activation of a launch lives in LDS
static int64_t q4k_max_cols(int64_t K) {
    const int64_t c = (int64_t)(144 * 1024) / (K + 80);
    return c >= 8 ? 8 : c >= 4 ? 4 : c >= 2 ? 2 : 1;
}

void profile_pair(tts_hip_backend * be, hipEvent_t & e0, hipEvent_t & e1) {
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
}

void profile_push(tts_hip_backend * be, hipEvent_t e0, hipEvent_t e1, double bytes, int type) {
    be->ev_pending.push_back({e0, e1});
    be->ev_bytes.push_back(bytes);
    be->ev_type.push_back(type);
}

// algorithmic bytes of one launch: every weight byte once + the activation read + the outputs written
static double gemv_bytes(const GemvJob & j) {
    const double rows = (double)job_rows(j);
    return rows * ((double)tts_row_size(j.wtype, j.K) + 4.0 * (double)j.M) + 4.0 * (double)j.K * (double)j.M;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): replica backends call
// the launchers from several host threads, so the per-device flags are atomic
static void set_lds_attr_once(std::atomic<uint32_t> & done, int device, const void * fn) {
    const uint32_t bit = 1u << (device & 31);
    if (done.load(std::memory_order_acquire) & bit) return;
    TTS_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    done.fetch_or(bit, std::memory_order_acq_rel);
}

template <int MC, int PRO, int NBMAX>
static void launch_q4k(tts_hip_backend * be, const GemvJob & j, unsigned gx, int nw, size_t lds) {
    static std::atomic<uint32_t> attr_done{0};
    if (lds > 64 * 1024) set_lds_attr_once(attr_done, be->device, (const void *)k_gemv_q4_K<MC, PRO, NBMAX>);
    if (be->profile_gemv) {
        // Profiled: the start/stop events ride in the dispatch packet itself (hipExtLaunchKernel), so
        // they carry the kernel's own begin/end timestamps -- the ones the rocprofv3 kernel trace
        // reports -- rather than the dispatch latency an event recorded between launches adds.
        hipEvent_t e0, e1;
        profile_pair(be, e0, e1);
        hipExtLaunchKernelGGL((k_gemv_q4_K<MC, PRO, NBMAX>), dim3(gx), dim3(64 * nw), (uint32_t)lds, be->stream, e0, e1, 0u, j);
        profile_push(be, e0, e1, gemv_bytes(j), TTS_TYPE_Q4_K);
        return;
    }
    hipLaunchKernelGGL((k_gemv_q4_K<MC, PRO, NBMAX>), dim3(gx), dim3(64 * nw), lds, be->stream, j);
}

// Unique-load geometry (k_gemv_q4_K_u): R rows per 512-thread workgroup with R * nb <= 64 octets,
// as few rows per workgroup as spreads the matrix over every CU.  False when the shape does not fit.
static bool q4k_u_geometry(const GemvJob & j, int MC, int & R, int & NCG, int64_t & gx, size_t & lds, int64_t cus) {
    const int64_t nb = j.K / QK_K;
    if (nb < 1 || nb > 64) return false;
    const int64_t NR = (int64_t)j.nmat * j.N;
    const int64_t rmax = 64 / nb;
    int64_t r = (NR + cus - 1) / cus;
    r = r > rmax ? rmax : r < 1 ? 1 : r;
    R = (int)r;
    gx = (NR + r - 1) / r;
    // spare octets split the columns: NCG groups of ceil(M / NCG) columns per (row, block)
    int64_t ncg = 64 / (r * nb);
    NCG = (int)(ncg < 1 ? 1 : ncg > j.M ? j.M : ncg);
    lds = q4k_lds(MC, j.K) + (size_t)R * MC * nb * 9 * 4;
    return lds <= 160 * 1024;
}

template <int MC, int PRO, int NCH>
static void launch_q4k_u(tts_hip_backend * be, const GemvJob & j, unsigned gx, int R, int NCG, size_t lds) {
    static std::atomic<uint32_t> attr_done{0};
    if (lds > 64 * 1024) set_lds_attr_once(attr_done, be->device, (const void *)k_gemv_q4_K_u<MC, PRO, NCH>);
    if (be->profile_gemv) {
        hipEvent_t e0, e1;
        profile_pair(be, e0, e1);
        hipExtLaunchKernelGGL((k_gemv_q4_K_u<MC, PRO, NCH>), dim3(gx), dim3(512), (uint32_t)lds, be->stream, e0, e1, 0u, j, R, NCG);
        profile_push(be, e0, e1, gemv_bytes(j), TTS_TYPE_Q4_K);
        return;
    }
    hipLaunchKernelGGL((k_gemv_q4_K_u<MC, PRO, NCH>), dim3(gx), dim3(512), lds, be->stream, j, R, NCG);
}

template <int MC>
static void launch_gemv_q4k_mc(tts_hip_backend * be, const GemvJob & j) {
    constexpr int S = 8 / MC;
    // unique loads pay off once a row holds >= 8 blocks (Parler fc2: 14.0 -> 11.1 us in the decode
    // graph at M = 8); at K = 1024 the octet-per-column kernel is faster (6.1 vs 7.7 us)
    if (be->gemv_unique && j.K >= 8 * QK_K && j.nmat > 1) {  // the unique-load kernel takes one matrix per launch
        for (int i = 0; i < j.nmat; ++i) {
            GemvJob one = j;
            one.nmat = 1;
            one.hetero = 0;
            one.W[0] = j.W[i], one.Y[0] = j.Y[i], one.ycs[0] = j.ycs[i], one.yrs[0] = j.yrs[i];
            one.rep_mat = i == j.rep_mat ? 0 : -1;
            one.N = j.hetero ? j.roff[i + 1] - j.roff[i] : j.N;
            one.roff[0] = 0, one.roff[1] = one.N;
            launch_gemv_q4k_mc<MC>(be, one);
        }
        return;
    }
    if (be->gemv_unique && j.K >= 8 * QK_K) {
        int R, NCG;
        int64_t gx;
        size_t lds;
        if (q4k_u_geometry(j, MC, R, NCG, gx, lds, be->cus)) {
            const bool wide = j.K > 4 * QK_K;  // LN prologue: NP = NCH / 4 chunk passes per lane
            if (j.pro == PRO_LN) {
                if (wide) launch_q4k_u<MC, PRO_LN, 16>(be, j, (unsigned)gx, R, NCG, lds);
                else launch_q4k_u<MC, PRO_LN, 4>(be, j, (unsigned)gx, R, NCG, lds);
            } else {
                if (wide) launch_q4k_u<MC, PRO_QUANT, 16>(be, j, (unsigned)gx, R, NCG, lds);
                else launch_q4k_u<MC, PRO_QUANT, 4>(be, j, (unsigned)gx, R, NCG, lds);
            }
            return;
        }
    }
    if (j.nmat > 1 && j.N % S) {  // a wave's S rows must not straddle two matrices: one launch each
        for (int i = 0; i < j.nmat; ++i) {
            GemvJob one = j;
            one.nmat = 1;
            one.W[0] = j.W[i], one.Y[0] = j.Y[i], one.ycs[0] = j.ycs[i], one.yrs[0] = j.yrs[i];
            one.rep_mat = i == j.rep_mat ? 0 : -1;  // the repeat-copy target follows its matrix
            one.roff[0] = 0, one.roff[1] = j.roff[i + 1] - j.roff[i];
            launch_gemv_q4k_mc<MC>(be, one);
        }
        return;
    }
    // One workgroup per CU with enough waves that every wave owns ~1 row group of the flat
    // (matrix, row) range: the prologue (norm + quantize of the whole activation) is paid once per
    // CU and the rows run in parallel waves rather than one after another in a wave.  An LN
    // prologue wants a wave per column.  Big matrices loop (2 workgroups per CU).
    const bool small = j.K <= 4 * QK_K;
    const int nw_max = small ? 16 : 8;
    const int64_t G = ((int64_t)j.nmat * j.N + S - 1) / S;
    int64_t nw = (G + be->cus - 1) / be->cus;
    if (nw < be->gemv_nw_min) nw = be->gemv_nw_min;  // fewer, fuller workgroups (TTS_HIP_OPT_GEMV_NW_MIN)
    if (j.pro == PRO_LN && nw < j.M) nw = j.M;
    nw = nw < 1 ? 1 : nw > nw_max ? nw_max : nw;
    int64_t gx = (G + nw - 1) / nw;
    if (gx > 512) gx = 512;
    const size_t lds = q4k_lds(MC, j.K);
    if (j.pro == PRO_LN) {
        if (small) launch_q4k<MC, PRO_LN, 4>(be, j, (unsigned)gx, (int)nw, lds);
        else launch_q4k<MC, PRO_LN, 16>(be, j, (unsigned)gx, (int)nw, lds);
    } else {
        if (small) launch_q4k<MC, PRO_QUANT, 4>(be, j, (unsigned)gx, (int)nw, lds);
        else launch_q4k<MC, PRO_QUANT, 16>(be, j, (unsigned)gx, (int)nw, lds);
    }
}
static size_t q80_lds(int MC, int64_t K, int RW) {
    const int64_t nb = K / QK8_0;
    auto a = [](size_t n) { return (n + 15) & ~(size_t)15; };
    return a((size_t)MC * K) + a(4 * MC * nb) + a(4 * (size_t)RW * nb * MC) + 4 * (size_t)RW * nb * MC;
}

// ---- MFMA path (k_gemv_q4K_mf) ----
// + the cross-over buffer: SwiGLU gate results (4 waves x 64 lanes x 4 floats) or the residue-split
// partial chains ((RS - 1) / RS x 8 waves x 64 lanes x 8 / RS x 4 floats <= 16 KiB)
static size_t q4k_mf_lds(int64_t M, int64_t K) { return ((size_t)(M * (K / QK_K) + 1) * (2 * QK_K + 32 + 4) + 15) / 16 * 16 + 16384; }
static int64_t q4k_mf_max_cols(int64_t K) {
    const int64_t c = ((int64_t)(160 * 1024 - 16384 - 16) / (2 * QK_K + 32 + 4) - 1) / (K / QK_K);
    return c >= 16 ? 16 : c >= 8 ? 8 : c;
}
// The matrix-core GEMV's prologue as a pass of its own (TTS_HIP_OPT_GEMV_PREQUANT): one workgroup per
// column norms (PRO_LN) and quantizes it, writing the operands in the GEMV's LDS layout to j.bq; the
// GEMV's workgroups then copy them instead of each loading and quantizing the whole activation
// (Orpheus down: 256 KB of f32 and 64 k quantizations per workgroup).  Same arithmetic, same layout:
// bit-identical.
// Grid (ceil(nb / 4), M) single-wave workgroups: the 16-lane row r of wave (c, m) quantizes block
// 4c + r of column m (q8k_row_block_mf).  PRO_LN: every wave first reduces the whole column (f64 sums,
// then mean, variance and scale exactly as the in-kernel prologue: ggml's NORM / RMS_NORM), then
// applies the affine to its blocks and writes them to the LN output as well (K <= 4096).
template <int PRO>
__global__ __launch_bounds__(64) void k_quant_mf(GemvJob j) {
    const int m = blockIdx.y, lane = threadIdx.x, r = lane >> 4, t = lane & 15;
    const int nb = (int)(j.K / QK_K);
    // column tiles of 16 (bq_tile > 0) each hold their own slot layout; otherwise one tile of M columns
    const int ct = j.bq_tile ? m >> 4 : 0, lm = j.bq_tile ? m & 15 : m;
    const int Mt = j.bq_tile ? min(16, (int)j.M - 16 * ct) : (int)j.M;
    const int nslot = Mt * nb + 1;
    const int sh = j.bq_slot ? j.bq_slot : QK_K;  // halves per slot
    _Float16 * b16 = (_Float16 *)(j.bq + (size_t)ct * j.bq_tile);
    _Float16 * sb = b16 + (size_t)nslot * sh;
    float * xd = (float *)(sb + (size_t)nslot * 16);
    const float * x = j.x + (int64_t)m * j.xcs;
    const int b = blockIdx.x * 4 + r;
    const int bc = b < nb ? b : nb - 1;
    const int off = bc * QK_K + 16 * t;
    float v[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) ld4(x + off + 4 * k, *(float (*)[4]) & v[4 * k]);
    if (PRO == PRO_LN) {
        // the whole column, 16 floats per lane per pass (passes of 1024 elements)
        const int K = (int)j.K;
        const double Kd = (double)K;
        float w[16], bb[16];
        const float * lnb = j.lnb ? j.lnb : j.lnw;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ld4(j.lnw + off + 4 * k, *(float (*)[4]) & w[4 * k]);
            ld4(lnb + off + 4 * k, *(float (*)[4]) & bb[4 * k]);
        }
        constexpr int PMAX = 4;  // K <= 4096 (the planner's LN fusion)
        float c[PMAX][16];
#pragma unroll
        for (int p = 0; p < PMAX; ++p) {  // unconditional (clamped) loads
            const int e0 = p * 1024 + 16 * lane;
#pragma unroll
            for (int k = 0; k < 4; ++k) ld4(x + min(e0 + 4 * k, K - 4), *(float (*)[4]) & c[p][4 * k]);
        }
        float mean = 0.f;
        if (!j.rms) {
            double s = 0.0;
#pragma unroll
            for (int p = 0; p < PMAX; ++p) {
                if (p * 1024 >= K) break;
                double sp = 0.0;
#pragma unroll
                for (int e = 0; e < 16; ++e) sp += (double)c[p][e];
                s += p * 1024 + 16 * lane < K ? sp : 0.0;
            }
            mean = (float)(wave_sum_f64(s) / Kd);
        }
        double s2 = 0.0;
#pragma unroll
        for (int p = 0; p < PMAX; ++p) {
            if (p * 1024 >= K) break;
            double sp = 0.0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const float d = j.rms ? c[p][e] : __fsub_rn(c[p][e], mean);
                sp += (double)__fmul_rn(d, d);
            }
            s2 += p * 1024 + 16 * lane < K ? sp : 0.0;
        }
        const float var = (float)(wave_sum_f64(s2) / Kd);
        const float scale = cr_divf(1.0f, cr_sqrtf(__fadd_rn(var, j.eps)));
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            float y = j.rms ? __fmul_rn(v[e], scale) : __fmul_rn(__fsub_rn(v[e], mean), scale);
            y = __fmul_rn(y, w[e]);
            if (j.lnb) y = __fadd_rn(y, bb[e]);
            v[e] = y;
        }
        if (j.lnout && b < nb) {
            float * o = j.lnout + (int64_t)m * j.locs + off;
#pragma unroll
            for (int k = 0; k < 4; ++k) *(float4 *)(o + 4 * k) = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        }
    }
    const int slot = b < nb ? lm * nb + b : nslot - 1;
    q8k_row_block_mf(v, lane, b16 + (size_t)slot * sh, sb + (size_t)slot * 16, xd + slot);
}

static bool q4k_mf_eligible(const tts_hip_backend * be, const GemvJob & j) {
    (void)be;
    // at least one column's Q8_K operands must fit LDS (K <= ~76k); wider rows would make
    // launch_q4k_mf's column loop step by 0
    return j.wtype == TTS_TYPE_Q4_K && j.tiled && q4k_mf_max_cols(j.K) >= 1;
}
template <int PRO, int NCH, int RS, int NCK = 0>
static void launch_q4k_mf_rs(tts_hip_backend * be, const GemvJob & j, unsigned gx) {
    if constexpr (PRO == PRO_COPY && NCK == 0) {  // unrolled chunk loop for the common row lengths
        switch ((j.K / QK_K + 3) / 4 * (j.K % (4 * QK_K) == 0 ? 1 : 0)) {
            case 1: launch_q4k_mf_rs<PRO, NCH, RS, 1>(be, j, gx); return;
            case 2: launch_q4k_mf_rs<PRO, NCH, RS, 2>(be, j, gx); return;
            case 3: launch_q4k_mf_rs<PRO, NCH, RS, 3>(be, j, gx); return;
            case 4: launch_q4k_mf_rs<PRO, NCH, RS, 4>(be, j, gx); return;
            case 8: launch_q4k_mf_rs<PRO, NCH, RS, 8>(be, j, gx); return;
            default: break;
        }
    }
    static std::atomic<uint32_t> attr_done{0};
    set_lds_attr_once(attr_done, be->device, (const void *)k_gemv_q4K_mf<PRO, NCH, RS, NCK>);
    const size_t lds = q4k_mf_lds(j.M, j.K);
    if (be->profile_gemv) {
        hipEvent_t e0, e1;
        profile_pair(be, e0, e1);
        hipExtLaunchKernelGGL((k_gemv_q4K_mf<PRO, NCH, RS, NCK>), dim3(gx), dim3(512), (uint32_t)lds, be->stream, e0, e1, 0u, j);
        profile_push(be, e0, e1, gemv_bytes(j), TTS_TYPE_Q4_K);
        return;
    }
    hipLaunchKernelGGL((k_gemv_q4K_mf<PRO, NCH, RS, NCK>), dim3(gx), dim3(512), lds, be->stream, j);
}
template <int PRO, int NCH>
static void launch_q4k_mf_pro(tts_hip_backend * be, const GemvJob & j) {
    const int64_t T = (job_rows(j) + 15) / 16;
    const unsigned gx = (unsigned)(T < be->cus ? T : be->cus);
    // residue split when every tile fits one slot of RS waves (8 waves per workgroup)
    const int rs = j.epi == EPI_SWIGLU || !be->gemv_mf_rsplit ? 1 : T <= (int64_t)gx * 2 ? 4 : T <= (int64_t)gx * 4 ? 2 : 1;
    if (rs == 4) launch_q4k_mf_rs<PRO, NCH, 4>(be, j, gx);
    else if (rs == 2) launch_q4k_mf_rs<PRO, NCH, 2>(be, j, gx);
    else launch_q4k_mf_rs<PRO, NCH, 1>(be, j, gx);
}
static bool launch_q4k_kr(tts_hip_backend * be, const GemvJob & j);
static void launch_q4k_mf(tts_hip_backend * be, const GemvJob & job) {
    const int64_t cmax = q4k_mf_max_cols(job.K);
    for (int64_t m0 = 0; m0 < job.M; m0 += cmax) {
        GemvJob j = job;
        j.dbg = be->gemv_dbg;
        j.M = job.M - m0 < cmax ? job.M - m0 : cmax;
        if (job.lnout) j.lnout = job.lnout + m0 * job.locs;
        j.x = job.x + m0 * job.xcs;
        for (int i = 0; i < job.nmat; ++i) j.Y[i] = job.Y[i] + m0 * job.ycs[i];
        if (job.yoff) j.yoff = job.yoff + m0;
        if (job.res) j.res = job.res + m0 * job.rcs;
        // the LN prologue holds one column's K / 256 chunks in registers (K <= 4096, as the planner's
        // LN fusion requires)
        if (j.pro == PRO_LN && j.K > 4 * 1024) {
            fprintf(stderr, "tts_hip: LN-fused Q4_K GEMV with K = %lld > 4096\n", (long long)j.K);
            abort();
        }
        const int64_t nb = j.K / QK_K;
        const int64_t bq = (((j.M * nb + 1) * (2 * QK_K + 32 + 4)) + 1023) & ~(int64_t)1023;
        if (j.K <= be->gemv_kr_ink && !j.dbg) {  // K relay with the prologue in every workgroup
            GemvJob ji = j;
            ji.bq = nullptr;
            ji.bq_bytes = bq;
            if (launch_q4k_kr(be, ji)) continue;
        }
        if (be->gemv_mf_prequant && !j.dbg && (size_t)(bq + 4 * j.K * j.M) <= be->scratch_size) {
            // operands to the top of scratch (its bottom may hold this GEMV's staged input columns)
            j.bq = be->scratch + be->scratch_size - bq;
            j.bq_bytes = bq;
            const dim3 qg((unsigned)((nb + 3) / 4), (unsigned)j.M);
            if (j.pro == PRO_LN) hipLaunchKernelGGL(k_quant_mf<PRO_LN>, qg, dim3(64), 0, be->stream, j);
            else hipLaunchKernelGGL(k_quant_mf<PRO_QUANT>, qg, dim3(64), 0, be->stream, j);
            TTS_HIP_CHECK(hipGetLastError());
            j.pro = PRO_COPY;
            j.lnout = nullptr;  // written by the pass
            if (!launch_q4k_kr(be, j)) launch_q4k_mf_pro<PRO_COPY, 16>(be, j);
            continue;
        }
        if (j.pro == PRO_LN) launch_q4k_mf_pro<PRO_LN, 16>(be, j);
        else launch_q4k_mf_pro<PRO_QUANT, 16>(be, j);
    }
}

// ---- K-relay matrix-core path (k_gemv_q4K_kr) ----
static size_t q4k_kr_lds(int64_t bq_bytes, bool sw) { return (size_t)((bq_bytes + 15) & ~15) + (sw ? 2 * 64 * 36 * 4 + 64 * 16 : 64 * 36 * 4); }
template <int BPW, bool SW, int NWT, bool LANE = false, bool LOOP = false, int PRO = PRO_COPY, int CTW = 1, bool CP = false>
static void launch_q4k_kr_t(tts_hip_backend * be, const GemvJob & j, unsigned gx, unsigned gy = 1) {
    if constexpr (PRO == PRO_COPY && CTW == 1 && !CP) {  // in-kernel prologue (launch_q4k_kr / launch_gemm_q4k_kr decide)
        if (j.pro == PRO_LN) return launch_q4k_kr_t<BPW, SW, NWT, LANE, LOOP, PRO_LN>(be, j, gx, gy);
        if (j.pro == PRO_QUANT) return launch_q4k_kr_t<BPW, SW, NWT, LANE, LOOP, PRO_QUANT>(be, j, gx, gy);
    }
    if constexpr (SW && !LOOP && BPW <= 3 && CTW == 1) {  // (BPW 4: the prefetch registers would spill)
        // SwiGLU pairs (8 waves, ~170 VGPRs: one workgroup per CU): more pairs than CUs run as one
        // workgroup per CU walking its pairs, operands copied once, the next pair's weights prefetched
        if (be->gemv_kr_loop && gx > (unsigned)be->cus && gy == 1) {
            launch_q4k_kr_t<BPW, SW, NWT, LANE, true, PRO>(be, j, (unsigned)be->cus, gy);
            return;
        }
    }
    static std::atomic<uint32_t> attr_done{0};
    set_lds_attr_once(attr_done, be->device, (const void *)k_gemv_q4K_kr<BPW, SW, NWT, LANE, LOOP, PRO, CTW, CP>);
    const size_t lds = q4k_kr_lds((CP ? 2 : CTW) * (j.bq_tile ? j.bq_tile : j.bq_bytes), SW || CP);
    const dim3 blk(64 * NWT * ((SW || CP) ? 2 : 1));
    if (be->profile_gemv) {
        hipEvent_t e0, e1;
        profile_pair(be, e0, e1);
        hipExtLaunchKernelGGL((k_gemv_q4K_kr<BPW, SW, NWT, LANE, LOOP, PRO, CTW, CP>), dim3(gx, gy), blk, (uint32_t)lds, be->stream, e0, e1, 0u, j);
        profile_push(be, e0, e1, gemv_bytes(j), TTS_TYPE_Q4_K);
        return;
    }
    hipLaunchKernelGGL((k_gemv_q4K_kr<BPW, SW, NWT, LANE, LOOP, PRO, CTW, CP>), dim3(gx, gy), blk, lds, be->stream, j);
}

// LDS of one column tile's operands (k_quant_mf's slot layout, whole 1 KB DMA chunks)
static size_t q4k_pf_lds(int64_t nb) { return (size_t)((((16 * nb + 1) * (2 * PF_SLOT + 32 + 4)) + 1023) & ~(int64_t)1023); }
template <int NB, bool LANE, int NW>
static void launch_q4k_pf_nw(tts_hip_backend * be, const GemvJob & j, unsigned gy) {
    static std::atomic<uint32_t> attr_done{0};
    set_lds_attr_once(attr_done, be->device, (const void *)k_gemm_q4K_pf<NB, LANE, NW>);
    const unsigned gx = (unsigned)((job_rows(j) / 16 + NW * PF_RS - 1) / (NW * PF_RS));
    hipLaunchKernelGGL((k_gemm_q4K_pf<NB, LANE, NW>), dim3(gx, gy), dim3(64 * NW), (uint32_t)q4k_pf_lds(NB), be->stream, j);
}
// TTS_HIP_OPT_GEMM_PF_NW: waves per workgroup (4: 8 row tiles per operand copy; 8: 16)
template <int NB, bool LANE>
static void launch_q4k_pf_t(tts_hip_backend * be, const GemvJob & j, unsigned gy) {
    if (be->gemm_pf_nw == 8) launch_q4k_pf_nw<NB, LANE, 8>(be, j, gy);
    else launch_q4k_pf_nw<NB, LANE, 4>(be, j, gy);
}

// Many-column Q4_K MUL_MAT (prompt prefill) on the matrix cores: the operand pass over all M columns
// (16-column tiles), then the K-relay kernel over (row tile, column tile) -- the same per-(row,
// column) arithmetic as the GEMV, so bit-identical to ggml's order, in two launches instead of one
// 8-column GEMV launch per 8 columns.  Lane-layout or tile-layout weights, K = 1024 x {1, 2, 3, 4}.
static bool launch_gemm_q4k_kr(tts_hip_backend * be, const GemvJob & job, size_t lo_res = SIZE_MAX) {
    if (!be->gemv_kr || !be->gemv_mf_prequant || job.wtype != TTS_TYPE_Q4_K || job.M <= 8 || job.epi == EPI_SWIGLU || job.dbg) return false;
    if (job.pro != PRO_QUANT && job.pro != PRO_LN) return false;
    if (job.pro == PRO_LN && job.K > 4 * 1024) return false;
    const int64_t nb = job.K / QK_K;
    if (nb != 4 && nb != 8 && nb != 12 && nb != 16) return false;
    for (int m = 0; m <= job.nmat; ++m)
        if (job_roff(job, m) % 16) return false;
    // TTS_HIP_OPT_GEMM_KR_INKERNEL = max M: decode-sized products skip the operand pass, every (row tile,
    // column tile) workgroup norms / quantizes its 16 columns itself (q4k_prologue, its first weight
    // loads issued between the activation loads and their use); the same operand values, bit-identical
    // (bit 16 of the option: only the quantize-only jobs, whose prologue runs on every wave at once)
    const int64_t ink_m = be->gemm_kr_ink & 0xFFFF;
    const bool ink = ink_m > 0 && job.M <= ink_m && job.K <= 4 * 1024 && !job.dbg &&
                     (job.pro == PRO_LN || job.xcs == job.K) && (!(be->gemm_kr_ink & 0x10000) || job.pro == PRO_QUANT);
    // TTS_HIP_OPT_GEMM_PF = min columns: prompt-pass products on the prefill GEMM (k_gemm_q4K_pf), whose
    // operand slots are padded (PF_SLOT halves)
    const bool pf = be->gemm_pf > 0 && job.M >= be->gemm_pf && !ink;
    const int64_t tile = pf ? (int64_t)q4k_pf_lds(nb) : (((16 * nb + 1) * (2 * QK_K + 32 + 4)) + 1023) & ~(int64_t)1023;
    const int64_t nct = (job.M + 15) / 16;
    if (q4k_kr_lds(tile, false) > 160 * 1024) return false;
    // the operands go to the top of scratch; its bottom may hold this job's staged input columns
    const char * xs0 = (const char *)job.x;
    const char * xs1 = xs0 + 4 * (size_t)((job.M - 1) * job.xcs + job.K);
    // (a chunk pass keeps the whole job's reservation: later chunks' columns lie above its own)
    const size_t lo = lo_res != SIZE_MAX ? lo_res
                      : (xs0 >= be->scratch && xs0 < be->scratch + be->scratch_size) ? (size_t)(xs1 - be->scratch) : 0;
    const int64_t avail = lo < be->scratch_size ? (int64_t)(be->scratch_size - lo) : 0;
    if (tile * nct > avail || (lo == 0 && (size_t)(tile * nct + 4 * job.K * job.M) > be->scratch_size) || nct > 65535) {
        // more columns than the operand area holds (a many-prompt prefill): passes over column chunks
        // of whole 16-column tiles, each the same per-(row, column) arithmetic
        const int64_t per = (lo ? avail / tile : (int64_t)be->scratch_size / (tile + 16 * 4 * job.K)) * 16;
        if (per < 16 || job.rep_mat >= 0) return false;  // (epilogues are per output element: column offsets carry them)
        for (int64_t m0 = 0; m0 < job.M; m0 += per) {
            GemvJob j = job;
            j.M = job.M - m0 < per ? job.M - m0 : per;
            if (job.lnout) j.lnout = job.lnout + m0 * job.locs;
            j.x = job.x + m0 * job.xcs;
            for (int i = 0; i < job.nmat; ++i) j.Y[i] = job.Y[i] + m0 * job.ycs[i];
        if (job.yoff) j.yoff = job.yoff + m0;
            if (job.res) j.res = job.res + m0 * job.rcs;
            if (!launch_gemm_q4k_kr(be, j, lo)) return false;  // (the first chunk is checked before any launch below)
        }
        return true;
    }
    GemvJob j = job;
    j.bq_tile = tile;
    j.bq_bytes = tile * nct;
    j.bq_slot = pf ? PF_SLOT : 0;
    if (ink) {
        j.bq = nullptr;
    } else {
        j.bq = be->scratch + be->scratch_size - j.bq_bytes;
        const dim3 qg((unsigned)((nb + 3) / 4), (unsigned)j.M);
        if (j.pro == PRO_LN) hipLaunchKernelGGL(k_quant_mf<PRO_LN>, qg, dim3(64), 0, be->stream, j);
        else hipLaunchKernelGGL(k_quant_mf<PRO_QUANT>, qg, dim3(64), 0, be->stream, j);
        TTS_HIP_CHECK(hipGetLastError());
        j.pro = PRO_COPY;
        j.lnout = nullptr;
    }
    const unsigned gx = (unsigned)(job_rows(j) / 16), gy = (unsigned)nct;
    j.xcd_cols = be->gemm_kr_xcd && nct > 1 ? 1 : 0;
    // TTS_HIP_OPT_GEMM_KR_CT2: two column tiles per workgroup (weights streamed once for 32 columns) where
    // both tiles' operands fit the LDS (K = 1024 x {1, 2})
    const bool ct2 = be->gemm_kr_ct2 && !ink && nct >= 2 && (nb == 4 || nb == 8) && q4k_kr_lds(2 * tile, false) <= 160 * 1024;
    // TTS_HIP_OPT_GEMM_KR_CP: two column tiles per workgroup on parallel wave halves (weights from HBM once)
    const bool cp = be->gemm_kr_cp && !ink && nct >= 2 && (nb == 4 || nb == 8) && q4k_kr_lds(2 * tile, true) <= 160 * 1024;
    auto go = [&](auto LANE) {
        constexpr bool L = decltype(LANE)::value;
        // the prefill GEMM: a wave per two 16-row tiles of one 16-column tile over the whole row, no relay
        if (pf) {
            switch (nb) {
                case 4: launch_q4k_pf_t<4, L>(be, j, gy); break;
                case 8: launch_q4k_pf_t<8, L>(be, j, gy); break;
                case 12: launch_q4k_pf_t<12, L>(be, j, gy); break;
                default: launch_q4k_pf_t<16, L>(be, j, gy); break;
            }
            return;
        }
        if (cp) {
            const unsigned gy2 = (unsigned)((nct + 1) / 2);
            if (nb == 4) launch_q4k_kr_t<1, false, 4, L, false, PRO_COPY, 1, true>(be, j, gx, gy2);
            else launch_q4k_kr_t<2, false, 4, L, false, PRO_COPY, 1, true>(be, j, gx, gy2);
            return;
        }
        if (ct2) {
            const unsigned gy2 = (unsigned)((nct + 1) / 2);
            if (nb == 4) launch_q4k_kr_t<1, false, 4, L, false, PRO_COPY, 2>(be, j, gx, gy2);
            else launch_q4k_kr_t<2, false, 4, L, false, PRO_COPY, 2>(be, j, gx, gy2);
            return;
        }
        // TTS_HIP_OPT_GEMM_KR_WALK = G: G workgroups per column tile, each copying its column tile's operands
        // into LDS once and walking row tiles tx, tx + G, ... (the next tile's weights requested before the
        // current tile's relay): the operand tile crosses L2 -> LDS G times instead of once per row tile.
        // Same (row, column) arithmetic: bit-identical.
        const int walk = be->gemm_kr_walk;
        if (walk > 0 && nct > 4 && gx > (unsigned)walk && !ink) {
            switch (nb) {
                case 4: launch_q4k_kr_t<1, false, 4, L, true>(be, j, (unsigned)walk, gy); break;
                case 8: launch_q4k_kr_t<2, false, 4, L, true>(be, j, (unsigned)walk, gy); break;
                case 12: launch_q4k_kr_t<3, false, 4, L, true>(be, j, (unsigned)walk, gy); break;
                default: launch_q4k_kr_t<4, false, 4, L, true>(be, j, (unsigned)walk, gy); break;
            }
            return;
        }
        // TTS_HIP_OPT_GEMM_KR_NW = 8: a tile's blocks over eight waves (K >= 2048; a longer relay, half the
        // blocks per wave)
        const bool nw8 = be->gemm_kr_nw == 8;
        switch (nb) {
            case 4: launch_q4k_kr_t<1, false, 4, L>(be, j, gx, gy); break;
            case 8: nw8 ? launch_q4k_kr_t<1, false, 8, L>(be, j, gx, gy) : launch_q4k_kr_t<2, false, 4, L>(be, j, gx, gy); break;
            case 12: launch_q4k_kr_t<3, false, 4, L>(be, j, gx, gy); break;
            default: nw8 ? launch_q4k_kr_t<2, false, 8, L>(be, j, gx, gy) : launch_q4k_kr_t<4, false, 4, L>(be, j, gx, gy); break;
        }
    };
    if (j.tiled) go(std::false_type{});
    else go(std::true_type{});
    TTS_HIP_CHECK(hipGetLastError());
    return true;
}
// PRO_COPY jobs (operands in j.bq) whose row length has an instantiation; false otherwise.
// PRO_QUANT / PRO_LN jobs (K <= 4096, j.bq_bytes = the operands' LDS size): the in-kernel prologue.
static bool launch_q4k_kr(tts_hip_backend * be, const GemvJob & j) {
    if (!be->gemv_kr || j.M > 8) return false;
    if (j.pro != PRO_COPY && !((j.pro == PRO_QUANT || j.pro == PRO_LN) && j.K <= 4 * 1024 && !j.bq_tile)) return false;
    const bool sw = j.epi == EPI_SWIGLU;
    if (!sw) {
        for (int m = 0; m <= j.nmat; ++m)
            if (job_roff(j, m) % 16) return false;
    } else if (j.N % 16) {
        return false;
    }
    if (q4k_kr_lds(j.bq_bytes, sw) > 160 * 1024) return false;
    const int64_t T = sw ? j.N / 16 : job_rows(j) / 16;
    if (T < 1 || T > 0x7fffffff) return false;
    const unsigned gx = (unsigned)T;
    switch (j.K / QK_K) {
        case 4: sw ? launch_q4k_kr_t<1, true, 4>(be, j, gx) : launch_q4k_kr_t<1, false, 4>(be, j, gx); return true;
        case 8: sw ? launch_q4k_kr_t<2, true, 4>(be, j, gx) : launch_q4k_kr_t<2, false, 4>(be, j, gx); return true;
        case 12: sw ? launch_q4k_kr_t<3, true, 4>(be, j, gx) : launch_q4k_kr_t<3, false, 4>(be, j, gx); return true;
        case 16: sw ? launch_q4k_kr_t<4, true, 4>(be, j, gx) : launch_q4k_kr_t<4, false, 4>(be, j, gx); return true;
        case 32: if (sw) return false; launch_q4k_kr_t<4, false, 8>(be, j, gx); return true;
        default: return false;
    }
}

// ---- K-split matrix-core path (k_gemv_q4K_ks) ----
static size_t q4k_ks_lds(int64_t M, int64_t nb) {
    return (((size_t)(M * nb + 1) * (2 * QK_K + 32 + 4) + 15) & ~(size_t)15) + (size_t)nb * (1024 + 128) * 4;
}
static bool q4k_ks_eligible(const tts_hip_backend * be, const GemvJob & j) {
    if (be->gemv_ks_tiles <= 0 || j.wtype != TTS_TYPE_Q4_K || !j.tiled || j.M < 1 || j.M > 8 || j.epi == EPI_SWIGLU) return false;
    const int64_t nb = j.K / QK_K;
    if (nb < 1 || nb > 16) return false;
    for (int m = 0; m <= j.nmat; ++m)
        if (job_roff(j, m) % 16) return false;
    if (j.pro == PRO_LN && j.K > 4 * 1024) return false;  // the LN prologue holds <= 16 chunks per lane
    if (job_rows(j) / 16 > be->gemv_ks_tiles) return false;
    return q4k_ks_lds(j.M, nb) <= 160 * 1024;
}
template <int PRO, int NCH, int UPW, int NWMAX>
static void launch_q4k_ks_t(tts_hip_backend * be, const GemvJob & j, unsigned gx, int nw, size_t lds) {
    static std::atomic<uint32_t> attr_done{0};
    if (lds > 64 * 1024) set_lds_attr_once(attr_done, be->device, (const void *)k_gemv_q4K_ks<PRO, NCH, UPW, NWMAX>);
    if (be->profile_gemv) {
        hipEvent_t e0, e1;
        profile_pair(be, e0, e1);
        hipExtLaunchKernelGGL((k_gemv_q4K_ks<PRO, NCH, UPW, NWMAX>), dim3(gx), dim3(64 * nw), (uint32_t)lds, be->stream, e0, e1, 0u, j);
        profile_push(be, e0, e1, gemv_bytes(j), TTS_TYPE_Q4_K);
        return;
    }
    hipLaunchKernelGGL((k_gemv_q4K_ks<PRO, NCH, UPW, NWMAX>), dim3(gx), dim3(64 * nw), lds, be->stream, j);
}
static void launch_q4k_ks(tts_hip_backend * be, const GemvJob & j) {
    const int64_t nb = j.K / QK_K, T = job_rows(j) / 16;
    // units (block, residue half) per wave: one for nb <= 4 (<= 8 waves); above, two (<= 16 waves)
    // after a quantize-only prologue, four (<= 8 waves) after an LN prologue, whose K / 256 chunks
    // per lane need the registers of a 512-thread workgroup
    const unsigned gx = (unsigned)(T < 2048 ? T : 2048);
    const size_t lds = q4k_ks_lds(j.M, nb);
    const int64_t bq = (((j.M * nb + 1) * (2 * QK_K + 32 + 4)) + 1023) & ~(int64_t)1023;
    if (j.K <= be->gemv_kr_ink && !j.dbg) {  // K relay with the prologue in every workgroup
        GemvJob ji = j;
        ji.bq = nullptr;
        ji.bq_bytes = bq;
        if (launch_q4k_kr(be, ji)) return;
    }
    if (be->gemv_mf_prequant && !j.dbg && (size_t)(bq + 4 * j.K * j.M) <= be->scratch_size &&
        (size_t)bq <= lds) {
        // the prologue as a pass of its own (k_quant_mf), the GEMV copying its operands (k_gemv_q4K_mf);
        // the DMA's rounding up to 1 KiB lands in the term area, written only after the barrier
        GemvJob jc = j;
        jc.bq = be->scratch + be->scratch_size - bq;
        jc.bq_bytes = bq;
        const dim3 qg((unsigned)((nb + 3) / 4), (unsigned)j.M);
        if (j.pro == PRO_LN) hipLaunchKernelGGL(k_quant_mf<PRO_LN>, qg, dim3(64), 0, be->stream, jc);
        else hipLaunchKernelGGL(k_quant_mf<PRO_QUANT>, qg, dim3(64), 0, be->stream, jc);
        TTS_HIP_CHECK(hipGetLastError());
        jc.pro = PRO_COPY;
        jc.lnout = nullptr;
        if (launch_q4k_kr(be, jc)) return;
        const int upw = nb <= 4 ? 1 : 2;
        const int nw = (int)((2 * nb + upw - 1) / upw);
        if (nb <= 4) launch_q4k_ks_t<PRO_COPY, 4, 1, 8>(be, jc, gx, nw, lds);
        else launch_q4k_ks_t<PRO_COPY, 16, 2, 16>(be, jc, gx, nw, lds);
        return;
    }
    const int upw = nb <= 4 ? 1 : j.pro == PRO_LN ? 4 : 2;
    const int nw = (int)((2 * nb + upw - 1) / upw);
    if (nb <= 4) {
        if (j.pro == PRO_LN) launch_q4k_ks_t<PRO_LN, 4, 1, 8>(be, j, gx, nw, lds);
        else launch_q4k_ks_t<PRO_QUANT, 4, 1, 8>(be, j, gx, nw, lds);
    } else {
        if (j.pro == PRO_LN) launch_q4k_ks_t<PRO_LN, 16, 4, 8>(be, j, gx, nw, lds);
        else launch_q4k_ks_t<PRO_QUANT, 16, 2, 16>(be, j, gx, nw, lds);
    }
}

// ------------------------------------------------------------------------------------------
// Q8_0 x Q8_0 GEMM for many columns (Dia's 1024-position encoder, prompt prefills) on the int8
// matrix cores.  ggml_vec_dot_q8_0_q8_0 per (row, column): sumf += sumi_b * (d_w,b * d_x,b) over the
// 32-element blocks b in ascending order, sumi_b the exact int32 dot of the block.  One
// v_mfma_i32_16x16x32_i8 computes sumi_b for a 16 x 16 tile exactly (K = 32 = one block; A[i = l&15]
// [k = 8(l>>4)..+7], B[k][j = l&15], D col l&15, rows 4(l>>4)+e), and each lane then folds its
// outputs' terms into f32 sums in block order with ggml's roundings: bit-identical to the GEMV.
// Workgroup: 4 waves over a 64-row x 64-column tile (2 x 2 MFMA tiles per wave); the next block's
// operands are loaded before the current block's MFMAs.  Native Q8_0 rows (34-B blocks, 2-B
// aligned): a lane's 8 weight bytes come as four 16-bit loads; activations are the Q8_0 copy
// (int8 [M][K], fp16-rounded d [M][K/32]) prepare_act made.
typedef int i32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_gemm_q8_0(GemvJob j) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int mat = blockIdx.z;
    const int nb = (int)(j.K / QK8_0);
    const int64_t r0 = (int64_t)blockIdx.x * 64 + (wave & 1) * 32;
    const int64_t c0 = (int64_t)blockIdx.y * 64 + (wave >> 1) * 32;
    const int r16 = lane & 15, kq = lane >> 4;
    const uint8_t * W = j.W[mat];
    const uint8_t * wrow[2];
    const int8_t * xcol[2];
    const float * xd[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int64_t r = min(r0 + 16 * t + r16, j.N - 1);
        const int64_t c = min(c0 + 16 * t + r16, j.M - 1);
        wrow[t] = W + r * j.w_row_bytes;
        xcol[t] = j.aq.qs + c * j.K;
        xd[t] = j.aq.d + c * nb;
    }
    // rows of this lane's accumulator elements (t, e): r0 + 16 t + 4 kq + e
    const uint8_t * drow[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) drow[t][e] = W + min(r0 + 16 * t + 4 * kq + e, j.N - 1) * j.w_row_bytes;
    float acc[2][2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[a][b][e] = 0.0f;
    long av[2], bv[2], an[2], bn[2];
    float dwv[2][4], dxv[2], dwn[2][4], dxn[2];
    auto load = [&](int b, long (&fa)[2], long (&fb)[2], float (&fw)[2][4], float (&fx)[2]) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint16_t * q = (const uint16_t *)(wrow[t] + (int64_t)b * 34 + 2 + 8 * kq);
            const uint64_t w = (uint64_t)q[0] | ((uint64_t)q[1] << 16) | ((uint64_t)q[2] << 32) | ((uint64_t)q[3] << 48);
            fa[t] = (long)w;
            fb[t] = *(const long *)(xcol[t] + (int64_t)b * QK8_0 + 8 * kq);
            fx[t] = xd[t][b];
#pragma unroll
            for (int e = 0; e < 4; ++e) fw[t][e] = dev_fp16_to_fp32(*(const uint16_t *)(drow[t][e] + (int64_t)b * 34));
        }
    };
    load(0, av, bv, dwv, dxv);
    for (int b = 0; b < nb; ++b) {
        if (b + 1 < nb) load(b + 1, an, bn, dwn, dxn);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) {
                const i32x4_t z = {0, 0, 0, 0};
                const i32x4_t s = __builtin_amdgcn_mfma_i32_16x16x32_i8(av[ti], bv[tj], z, 0, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[ti][tj][e] = __fadd_rn(acc[ti][tj][e], __fmul_rn((float)s[e], __fmul_rn(dwv[ti][e], dxv[tj])));
            }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            av[t] = an[t], bv[t] = bn[t], dxv[t] = dxn[t];
#pragma unroll
            for (int e = 0; e < 4; ++e) dwv[t][e] = dwn[t][e];
        }
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
            const int64_t col = c0 + 16 * tj + r16;
            if (col >= j.M) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t row = r0 + 16 * ti + 4 * kq + e;
                if (row < j.N) gemv_store<1>(j, mat, row, (int)col, acc[ti][tj][e]);
            }
        }
}

// The staged form (K % 256 == 0, 16-B aligned weight rows and activation copy): a workgroup owns a
// 64-row x TC-column output tile; the K dimension runs in stages of 8 blocks (256 elements), each
// stage's operands fetched into registers while the previous stage computes, then stored to the other
// of two LDS buffers:
//   A: the 64 rows' native 272-B stage spans, row-major (17 x 16 B per row; row stride 68 dwords puts
//      the 16 rows an MFMA reads on distinct banks), read as 3 dwords + funnel shift (quants start
//      2 B into a block) and the block's fp16 d as one u16;
//   B: the TC columns' 256 int8, 16-B chunks XOR-swizzled by column (chunk q of column c at slot
//      q ^ (c & 15)) so the 16 columns of an MFMA read different banks;
//   dx: the TC columns' 8 block scales.
// Per block and 16 x 16 tile one v_mfma_i32_16x16x32_i8 gives the exact block dots; each lane folds
// its four outputs' terms into f32 in block order with ggml's roundings, as k_gemm_q8_0: bit-identical.
template <int TC>
struct Q8s {
    static constexpr int A_BYTES = 20 * 1024;  // 64 rows x 272 B (1088 chunks) as 20 x 64 uniform 16-B chunks
    static constexpr int B_BYTES = TC * 256;
    static constexpr int D_BYTES = TC * 32;
    static constexpr int STAGE = A_BYTES + B_BYTES + D_BYTES;
};
template <int TC>
__global__ __launch_bounds__(256) void k_gemm_q8_0s(GemvJob j) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int NT = TC / 32;  // 16-column tiles per wave
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l16 = lane & 15, kq = lane >> 4;
    const int mat = blockIdx.z;
    const int64_t row0 = (int64_t)blockIdx.x * 64, col0 = (int64_t)blockIdx.y * TC;
    const int64_t rb = j.w_row_bytes, K = j.K;
    const int nb = (int)(K / QK8_0), nst = nb / 8;
    const char * W = (const char *)j.W[mat];
    const char * xq = (const char *)j.aq.qs;
    const char * xdg = (const char *)j.aq.d;
    // a wave's share of one stage: 5 A chunks, TC / 16 B chunks, <= 1 dx chunk (16 B each), fetched into
    // registers while the previous stage computes, then stored to LDS (a lane's chunk of instruction
    // `ins` at slot ins * 64 + lane).  Register staging, not LDS-DMA: the compiler cannot tell a DMA's
    // LDS target from the buffer being read and would wait for the DMA before every LDS read.
    constexpr int NB_ = TC / 16;
    u32x4 ra[5], rbv[NB_], rd;
    auto stage_load = [&](int st) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            // A: linear chunk n = r * 17 + q (n < 1088; the rest re-read the last chunk into the slack)
            int n = (wave * 5 + i) * 64 + lane;
            n = n < 1088 ? n : 1087;
            const int r = n / 17, q = n - 17 * (n / 17);
            const int64_t row = row0 + r < j.N ? row0 + r : j.N - 1;
            ra[i] = *gptr((const u32x4 *)(W + row * rb + (int64_t)st * 272 + 16 * q));
        }
#pragma unroll
        for (int i = 0; i < NB_; ++i) {
            // B: slot idx = c * 16 + q' holds chunk q = q' ^ (c & 15) of column c
            const int idx = (wave * NB_ + i) * 64 + lane, c = idx >> 4, q = (idx & 15) ^ (c & 15);
            const int64_t col = col0 + c < j.M ? col0 + c : j.M - 1;
            rbv[i] = *gptr((const u32x4 *)(xq + col * K + (int64_t)st * 256 + 16 * q));
        }
        {
            // dx: column c's 8 scales as chunks 2c, 2c + 1 (waves 0 .. TC/32 - 1)
            const int idx = (wave < TC / 32 ? wave : 0) * 64 + lane, c = idx >> 1, h = idx & 1;
            const int64_t col = col0 + c < j.M ? col0 + c : j.M - 1;
            rd = *gptr((const u32x4 *)(xdg + col * (int64_t)nb * 4 + (int64_t)st * 32 + 16 * h));
        }
    };
    auto stage_store = [&](int buf) __attribute__((always_inline)) {
        char * base = smem + buf * Q8s<TC>::STAGE;
#pragma unroll
        for (int i = 0; i < 5; ++i) *(u32x4 *)(base + (wave * 5 + i) * 1024 + 16 * lane) = ra[i];
        char * bb = base + Q8s<TC>::A_BYTES;
#pragma unroll
        for (int i = 0; i < NB_; ++i) *(u32x4 *)(bb + (wave * NB_ + i) * 1024 + 16 * lane) = rbv[i];
        if (wave < TC / 32) *(u32x4 *)(bb + Q8s<TC>::B_BYTES + wave * 1024 + 16 * lane) = rd;
    };
    const int wr = (wave & 1) * 32, wc = (wave >> 1) * (TC / 2);
    float acc[2][NT][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[a][b][e] = 0.0f;
    stage_load(0);
    stage_store(0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        stage_load(st + 1 < nst ? st + 1 : st);  // unconditional (clamped): lands during this stage's MFMAs
        const char * base = smem + (st & 1) * Q8s<TC>::STAGE;
        const char * bb = base + Q8s<TC>::A_BYTES;
        const float * db = (const float *)(bb + Q8s<TC>::B_BYTES);
        // all of a block's MFMAs are issued before any result is folded, so they pipeline instead of
        // each waiting out the previous one's latency
#pragma unroll 2
        for (int b = 0; b < 8; ++b) {
            long av[2], bv[NT];
            float dw[2][4], dx[NT];
#pragma unroll
            for (int ti = 0; ti < 2; ++ti) {
                const int off = (wr + 16 * ti + l16) * 272 + b * 34 + 2 + 8 * kq;
                const uint32_t * p = (const uint32_t *)(base + (off & ~3));
                const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
                const uint32_t sh = (off & 3) * 8;
                const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, sh), hi = __builtin_amdgcn_alignbit(d2, d1, sh);
                av[ti] = (long)(((uint64_t)hi << 32) | lo);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    dw[ti][e] = dev_fp16_to_fp32(*(const uint16_t *)(base + (wr + 16 * ti + 4 * kq + e) * 272 + b * 34));
            }
#pragma unroll
            for (int tj = 0; tj < NT; ++tj) {
                const int c = wc + 16 * tj + l16;
                const int q = 2 * b + (kq >> 1);
                bv[tj] = *(const long *)(bb + (c * 16 + (q ^ (c & 15))) * 16 + 8 * (kq & 1));
                dx[tj] = db[c * 8 + b];
            }
            i32x4_t sv[2][NT];
#pragma unroll
            for (int tj = 0; tj < NT; ++tj)
#pragma unroll
                for (int ti = 0; ti < 2; ++ti) {
                    const i32x4_t z = {0, 0, 0, 0};
                    sv[ti][tj] = __builtin_amdgcn_mfma_i32_16x16x32_i8(av[ti], bv[tj], z, 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);  // keep the scheduler from re-serializing them into one accumulator
#pragma unroll
            for (int tj = 0; tj < NT; ++tj)
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        acc[ti][tj][e] = __fadd_rn(acc[ti][tj][e], __fmul_rn((float)sv[ti][tj][e], __fmul_rn(dw[ti][e], dx[tj])));
        }
        // every wave is done with the other buffer (stage st - 1) since the last barrier
        if (st + 1 < nst) stage_store((st + 1) & 1);
        __syncthreads();
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < NT; ++tj) {
            const int64_t col = col0 + wc + 16 * tj + l16;
            if (col >= j.M) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t row = row0 + wr + 16 * ti + 4 * kq + e;
                if (row < j.N) gemv_store<1>(j, mat, row, (int)col, acc[ti][tj][e]);
            }
        }
}

static bool gemm_q8s_ok(const tts_hip_backend * be, const GemvJob & j) {
    if (be->gemm_q8_staged <= 0 || j.K % QK_K || j.w_row_bytes % 16 || ((uintptr_t)j.aq.qs & 15) || ((uintptr_t)j.aq.d & 15)) return false;
    for (int m = 0; m < j.nmat; ++m)
        if ((uintptr_t)j.W[m] & 15) return false;
    return true;
}

static void launch_gemm_q8_0(tts_hip_backend * be, const GemvJob & j) {
    if (gemm_q8s_ok(be, j)) {
        static std::atomic<uint32_t> attr_done[2];
        if (be->gemm_q8_staged == 1) {
            set_lds_attr_once(attr_done[0], be->device, (const void *)k_gemm_q8_0s<64>);
            const dim3 grid((unsigned)((j.N + 63) / 64), (unsigned)((j.M + 63) / 64), (unsigned)j.nmat);
            hipLaunchKernelGGL(k_gemm_q8_0s<64>, grid, dim3(256), 2 * Q8s<64>::STAGE, be->stream, j);
        } else {
            set_lds_attr_once(attr_done[1], be->device, (const void *)k_gemm_q8_0s<128>);
            const dim3 grid((unsigned)((j.N + 63) / 64), (unsigned)((j.M + 127) / 128), (unsigned)j.nmat);
            hipLaunchKernelGGL(k_gemm_q8_0s<128>, grid, dim3(256), 2 * Q8s<128>::STAGE, be->stream, j);
        }
        return;
    }
    const dim3 grid((unsigned)((j.N + 63) / 64), (unsigned)((j.M + 63) / 64), (unsigned)j.nmat);
    hipLaunchKernelGGL(k_gemm_q8_0, grid, dim3(256), 0, be->stream, j);
}

// slab-form Q8_0 GEMV: whole 16-B aligned rows (K % 256 == 0), activation quantized by the prologue or
// by the quantize launch (Q8_0 blocks at j.aq)
static bool q80s_ok(const tts_hip_backend * be, const GemvJob & j) {
    if (!be->gemv_q80_slab || j.K % QK_K || j.hetero || j.dbg) return false;
    if (!j.pro && (j.aq.vtype != TTS_TYPE_Q8_0 || ((uintptr_t)j.aq.qs & 15) || ((uintptr_t)j.aq.d & 15))) return false;
    for (int m = 0; m < j.nmat; ++m)
        if ((uintptr_t)j.W[m] & 15) return false;
    return q80s_lds(8, j.K, 1) <= 160 * 1024;
}
template <int MC>
static void launch_q80s(tts_hip_backend * be, const GemvJob & j) {
    // rows per workgroup: the largest of 32 / 16 / 8 / 4 / 2 / 1 that still gives every CU a workgroup
    // and fits LDS (option TTS_HIP_OPT_GEMV_Q80_RW overrides)
    int RW = be->gemv_q80_rw > 0 ? be->gemv_q80_rw : 32;
    if (be->gemv_q80_rw <= 0)
        while (RW > 1 && (j.N + RW - 1) / RW * j.nmat < be->cus) RW /= 2;
    while (RW > 1 && q80s_lds(MC, j.K, RW) > (be->gemv_q80_rw > 0 ? 160 : 80) * 1024) RW /= 2;  // auto: 2+ workgroups per CU
    const size_t lds = q80s_lds(MC, j.K, RW);
    const dim3 grid((unsigned)((j.N + RW - 1) / RW), (unsigned)j.nmat);
    static std::atomic<uint32_t> attr_done[3];
    // profiled: in-packet events (the Dia leg's roofline; launch_gemv_job leaves Q8_0 slab jobs to this)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (be->profile_gemv) profile_pair(be, e0, e1);
    if (j.pro == PRO_LN) {
        set_lds_attr_once(attr_done[2], be->device, (const void *)k_gemv_q8_0s<MC, PRO_LN>);
        hipExtLaunchKernelGGL((k_gemv_q8_0s<MC, PRO_LN>), grid, dim3(256), (uint32_t)lds, be->stream, e0, e1, 0u, j, RW);
    } else if (j.pro == PRO_QUANT) {
        set_lds_attr_once(attr_done[1], be->device, (const void *)k_gemv_q8_0s<MC, PRO_QUANT>);
        hipExtLaunchKernelGGL((k_gemv_q8_0s<MC, PRO_QUANT>), grid, dim3(256), (uint32_t)lds, be->stream, e0, e1, 0u, j, RW);
    } else {
        set_lds_attr_once(attr_done[0], be->device, (const void *)k_gemv_q8_0s<MC>);
        hipExtLaunchKernelGGL(k_gemv_q8_0s<MC>, grid, dim3(256), (uint32_t)lds, be->stream, e0, e1, 0u, j, RW);
    }
    if (be->profile_gemv) profile_push(be, e0, e1, gemv_bytes(j), TTS_TYPE_Q8_0);
}

template <int MC>
static void launch_gemv_mc(tts_hip_backend * be, const GemvJob & j) {
    const unsigned nmat = (unsigned)j.nmat;
    switch (j.wtype) {
        case TTS_TYPE_Q4_K: launch_gemv_q4k_mc<MC>(be, j); break;
        case TTS_TYPE_Q8_0: {
            if (q80s_ok(be, j)) {
                launch_q80s<MC>(be, j);
                break;
            }
            int RW = 8;
            while (RW > 1 && q80_lds(MC, j.K, RW) > 64 * 1024) RW /= 2;
            const size_t lds = q80_lds(MC, j.K, RW) + (j.pro ? QK_K + 64 : 0);
            const unsigned grid = (unsigned)((j.N + RW - 1) / RW);
            if (j.pro == PRO_LN) hipLaunchKernelGGL((k_gemv_q8_0<MC, PRO_LN>), dim3(grid, nmat), dim3(256), lds, be->stream, j, RW);
            else if (j.pro == PRO_QUANT) hipLaunchKernelGGL((k_gemv_q8_0<MC, PRO_QUANT>), dim3(grid, nmat), dim3(256), lds, be->stream, j, RW);
            else hipLaunchKernelGGL(k_gemv_q8_0<MC>, dim3(grid, nmat), dim3(256), lds, be->stream, j, RW);
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

// Profiled passes are launched eagerly; a graph's worth of launches takes the host longer than the
// device needs to run them, so per-kernel events would also time the host's launch gaps.  A short
// device spin at the start of a profiled graph lets the host queue everything first: the events
// then bracket back-to-back kernels, as the kernel trace sees them.
__global__ void k_spin(long long ticks) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

void launch_profile_spin(tts_hip_backend * be, double us) {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, be->stream, (long long)(us * 100.0));  // 100 MHz counter
    TTS_HIP_CHECK(hipGetLastError());
}

void launch_gemv_job(tts_hip_backend * be, const GemvJob & job) {
    // Q4_K launches and Q8_0 slab GEMVs profile themselves (in-packet events); other jobs are timed whole
    const bool prof = be->profile_gemv && job.wtype != TTS_TYPE_Q4_K && !(job.wtype == TTS_TYPE_Q8_0 && job.M <= 8 && q80s_ok(be, job));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof) {
        profile_pair(be, e0, e1);
        TTS_HIP_CHECK(hipEventRecord(e0, be->stream));
    }
    const int64_t K = job.K;
    if (job.wtype == TTS_TYPE_F32 && job.M > 8 && gemm_f32_ok(job)) {
        launch_gemm_f32(be, job);  // one tiled pass instead of a GEMV launch per 8 columns
        if (prof) {
            TTS_HIP_CHECK(hipEventRecord(e1, be->stream));
            profile_push(be, e0, e1, gemv_bytes(job), job.wtype);
        }
        return;
    }
    if (job.wtype == TTS_TYPE_Q8_0 && job.M > 8 && job.aq.vtype == TTS_TYPE_Q8_0 && !job.hetero && be->gemm_q8) {
        launch_gemm_q8_0(be, job);  // one matrix-core pass instead of a GEMV launch per 8 columns
        TTS_HIP_CHECK(hipGetLastError());
        if (prof) {
            TTS_HIP_CHECK(hipEventRecord(e1, be->stream));
            profile_push(be, e0, e1, gemv_bytes(job), job.wtype);
        }
        return;
    }
    if (job.M > 8 && launch_gemm_q4k_kr(be, job)) return;  // prefill: matrix-core GEMM over column tiles
    if (q4k_ks_eligible(be, job)) {
        launch_q4k_ks(be, job);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    if (q4k_mf_eligible(be, job)) {
        launch_q4k_mf(be, job);
        TTS_HIP_CHECK(hipGetLastError());
        return;
    }
    if (job.epi == EPI_SWIGLU) {  // the planner forms these for tile-layout Q4_K pairs only
        fprintf(stderr, "tts_hip: SwiGLU GEMV epilogue needs the matrix-core Q4_K kernel\n");
        abort();
    }
    const int64_t cmax = job.wtype == TTS_TYPE_Q4_K ? q4k_max_cols(K) : 8;
    for (int64_t m0 = 0; m0 < job.M; m0 += cmax) {
        const int64_t mc = job.M - m0 < cmax ? job.M - m0 : cmax;
        GemvJob j = job;
        j.M = mc;
        if (job.lnout) j.lnout = job.lnout + m0 * job.locs;
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
        if (job.yoff) j.yoff = job.yoff + m0;
        if (job.res) j.res = job.res + m0 * job.rcs;
        switch (mc) {
            case 1: launch_gemv_mc<1>(be, j); break;
            case 2: launch_gemv_mc<2>(be, j); break;
            case 3: case 4: launch_gemv_mc<4>(be, j); break;
            default: launch_gemv_mc<8>(be, j); break;
        }
    }
    TTS_HIP_CHECK(hipGetLastError());
    if (prof) {
        TTS_HIP_CHECK(hipEventRecord(e1, be->stream));
        profile_push(be, e0, e1, gemv_bytes(job), job.wtype);
    }
}

}  // namespace tts
