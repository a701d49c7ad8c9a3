// Internal HIP backend state and kernel launchers (not part of the C-ABI).
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <tuple>
#include <vector>

#include "common.h"

#define TTS_HIP_CHECK(expr)                                                                          \
    do {                                                                                             \
        hipError_t err_ = (expr);                                                                    \
        if (err_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d: HIP error %s: %s\n", __FILE__, __LINE__, #expr, hipGetErrorString(err_)); \
            abort();                                                                                 \
        }                                                                                            \
    } while (0)

namespace tts {

constexpr int kArgmaxRows = 4096;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short short2_t __attribute__((ext_vector_type(2)));

// Tensor view handed to kernels by value: data pointer, shape and byte strides (ggml ne/nb).
struct TD {
    char * data;
    int64_t ne[4];
    int64_t nb[4];
    int32_t type;
    int32_t pad;  // tts_tensor.flags (TTS_FLAG_REPACKED matters to kernels)
};

// Transcendentals pinned to the correctly rounded f32 value (evaluated in f64), the same policy
// as the oracle (oracle/ggml_ref.c ref_expf ...), so GPU and CPU agree bit-for-bit except when
// the exact value lies within ~2^-52 of an f32 rounding midpoint.
#ifdef __HIPCC__
__device__ __forceinline__ float cr_expf(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float cr_sinf(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float cr_cosf(float x) { return (float)cos((double)x); }
__device__ __forceinline__ float cr_tanhf(float x) { return (float)tanh((double)x); }
// IEEE-exact f32 sqrt / division (gfx950's f32 sqrt lowering is not correctly rounded); the f64
// result rounded to f32 is the correctly rounded f32 value (53 >= 2*24 + 2).
__device__ __forceinline__ float cr_sqrtf(float x) { return (float)__dsqrt_rn((double)x); }
__device__ __forceinline__ float cr_divf(float a, float b) { return (float)__ddiv_rn((double)a, (double)b); }
// ggml's silu (ggml_vec_silu_f32 / ggml_silu_f32: x / (1 + exp(-x))), correctly rounded pieces
__device__ __forceinline__ float dev_silu(float x) { return cr_divf(x, __fadd_rn(1.0f, cr_expf(-x))); }

// Compiler memory barrier placed after a batch of independent loads: keeps the compiler from
// sinking a load into the (guarded) block that uses it, which would serialize the batch into one
// full memory round trip per load.  Emits no instruction.
#define TTS_PIN_LOADS() asm volatile("" ::: "memory")

// Cache policy of the two big decode streams (build-time, for the MALL-residency study):
// TTS_WLOAD = quantized weight rows (default non-temporal), TTS_KVLOAD = K/V cache rows of decode
// attention (default plain).
// Loads through an explicitly global (address space 1) pointer: a pointer the compiler cannot trace
// to a kernel argument would otherwise be a FLAT load, and flat loads complete out of order, so every
// later wait on any vector load becomes vmcnt(0) -- a wait for the weight stream in the prologue.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T * gptr(const T * p) {
    return (const __attribute__((address_space(1))) T *)p;
}
#ifdef TTS_W_PLAIN
#define TTS_WLOAD(p) (*gptr(p))
#else
#define TTS_WLOAD(p) __builtin_nontemporal_load(gptr(p))
#endif
__device__ __forceinline__ float4 kv_ld4(const float4 * p) {
#ifdef TTS_KV_NT
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = __builtin_nontemporal_load((const f4v *)p);
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
#define TTS_KVLOAD(p) kv_ld4(p)

// ---- wave64 cross-lane helpers on DPP + readlane (no LDS crossbar, no lgkmcnt waits) ----
// DPP controls (gfx9): quad_perm [1,0,3,2] = lane^1, [2,3,0,1] = lane^2, row_half_mirror (i <-> 7-i
// in each 8), row_mirror (i <-> 15-i in each 16), row_shl:n (lane i reads lane i+n in its row).
enum { DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140, DPP_ROW_SHL0 = 0x100 };
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(dpp_i32<CTRL>(__float_as_int(v)));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i32<CTRL>((int)(b & 0xFFFFFFFF)), hi = dpp_i32<CTRL>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFF), lane), hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// wave-uniform sum; every lane of a 16-lane row holds the same partial (a+b == b+a), the four row
// partials are added in row order
__device__ __forceinline__ double wave_sum_f64(double v) {
    v += dpp_f64<DPP_XOR1>(v);
    v += dpp_f64<DPP_XOR2>(v);
    v += dpp_f64<DPP_HALF_MIRROR>(v);
    v += dpp_f64<DPP_MIRROR>(v);
    return ((readlane_f64(v, 0) + readlane_f64(v, 16)) + readlane_f64(v, 32)) + readlane_f64(v, 48);
}
// wave-uniform max of non-negative floats (compared as their bit patterns)
__device__ __forceinline__ float wave_max_nonneg(float x) {
    unsigned v = __float_as_uint(x);
    v = max(v, (unsigned)dpp_i32<DPP_XOR1>((int)v));
    v = max(v, (unsigned)dpp_i32<DPP_XOR2>((int)v));
    v = max(v, (unsigned)dpp_i32<DPP_HALF_MIRROR>((int)v));
    v = max(v, (unsigned)dpp_i32<DPP_MIRROR>((int)v));
    const unsigned a = max((unsigned)__builtin_amdgcn_readlane((int)v, 0), (unsigned)__builtin_amdgcn_readlane((int)v, 16));
    const unsigned b = max((unsigned)__builtin_amdgcn_readlane((int)v, 32), (unsigned)__builtin_amdgcn_readlane((int)v, 48));
    return __uint_as_float(max(a, b));
}
// sum over the 8 lanes of an octet, result in all 8 lanes
__device__ __forceinline__ int octet_sum_i32(int v) {
    v += dpp_i32<DPP_XOR1>(v);
    v += dpp_i32<DPP_XOR2>(v);
    v += dpp_i32<DPP_HALF_MIRROR>(v);
    return v;
}
#endif

inline TD make_td(const tts_tensor * t) {
    TD d;
    d.data = (char *)t->data;
    for (int i = 0; i < 4; ++i) {
        d.ne[i] = t->ne[i];
        d.nb[i] = (int64_t)t->nb[i];
    }
    d.type = t->type;
    d.pad = t->flags;
    return d;
}
#ifdef __HIPCC__
// element access through a ggml view (F32 / F16 / I32), as the oracle's load_elem / store_elem
static __device__ __forceinline__ void unravel(int64_t k, const int64_t * ne, int64_t & i0, int64_t & i1, int64_t & i2, int64_t & i3) {
    i0 = k % ne[0];
    k /= ne[0];
    i1 = k % ne[1];
    k /= ne[1];
    i2 = k % ne[2];
    i3 = k / ne[2];
}

static __device__ __forceinline__ float td_load(const TD & t, int64_t i0, int64_t i1, int64_t i2, int64_t i3) {
    const char * p = t.data + i0 * t.nb[0] + i1 * t.nb[1] + i2 * t.nb[2] + i3 * t.nb[3];
    if (t.type == TTS_TYPE_F16) return __half2float(*(const __half *)p);
    if (t.type == TTS_TYPE_I32) return (float)*(const int32_t *)p;
    return *(const float *)p;
}
static __device__ __forceinline__ void td_store(const TD & t, int64_t i0, int64_t i1, int64_t i2, int64_t i3, float v) {
    char * p = t.data + i0 * t.nb[0] + i1 * t.nb[1] + i2 * t.nb[2] + i3 * t.nb[3];
    if (t.type == TTS_TYPE_F16) *(__half *)p = __float2half_rn(v);
    else if (t.type == TTS_TYPE_I32) *(int32_t *)p = (int32_t)v;
    else *(float *)p = v;
}
#endif

// Device scratch for quantized activations (Q8_K / Q8_0 / F16 copies of a mul_mat src1).
struct ActQuant {
    const void * src = nullptr;  // src1 data pointer the cache entry was built from
    int64_t K = 0, M = 0;
    int vtype = -1;
    int64_t graph_epoch = -1;
    int8_t * qs = nullptr;      // [M][K] int8 (Q8_K / Q8_0) or fp16 [M][K] (F16)
    float * d = nullptr;        // [M][K/256] (Q8_K) or [M][K/32] (Q8_0: fp16-rounded d as float)
    int32_t * bsums = nullptr;  // [M][K/256][8] per-32 sums (Q8_K)
};

// One GEMV launch: up to GEMV_MAX_MATS weight matrices of identical type/shape sharing one
// activation (q/k/v; the 9 codebook heads), y(row n, column m) = Y[i][m*ycs + n*yrs], with an
// optional fused epilogue (GELU table, or + residual(row n, column m) = res[m*rcs + n]).
// EPI_SWIGLU (matrix-core Q4_K kernel only, nmat == 2: gate, up): Y[0] = silu(gate) * up, the
// UNARY SILU and MUL of the SwiGLU MLP (Orpheus model.cpp:296-300); gate / up are never stored.
// EPI_SILU_MUL (Q8_0 kernels): y = silu(res) * product -- the up product's epilogue reading the gate
// product stored by the previous launch (Dia's MLP: MUL(SILU(gate x), up x)), as UNARY SILU then MUL round.
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_ADD = 2, EPI_SWIGLU = 3, EPI_SILU_MUL = 4 };
constexpr int GEMV_MAX_MATS = 16;
struct GemvJob {
    int wtype = 0;
    int nmat = 1;
    const uint8_t * W[GEMV_MAX_MATS] = {};
    float * Y[GEMV_MAX_MATS] = {};
    int64_t w_row_bytes = 0, K = 0, N = 0, M = 0;
    int64_t ycs[GEMV_MAX_MATS] = {}, yrs[GEMV_MAX_MATS] = {};  // per-matrix output strides
    const float * res = nullptr;
    int64_t rcs = 0;
    int epi = EPI_NONE;
    const uint16_t * gelu = nullptr;
    const float * x = nullptr;  // f32 activation (F32 weights; Q4_K quantizes it in-kernel)
    int64_t xcs = 0;
    ActQuant aq;
    // Q4_K prologue: PRO_QUANT = quantize x to Q8_K in LDS; PRO_LN = first x <- norm(x)*w (+b)
    // (NORM/RMS_NORM -> MUL -> ADD, parler_build_layer_norm), written to lnout by workgroup 0.
    int pro = 0;
    int tiled = 0;  // W in the 4-row tile layout (TTS_FLAG_TILED): k_gemv_q4K_mf
    // matrices of different row counts (tile-layout kernels only): matrix m holds flat rows
    // roff[m] .. roff[m + 1] - 1 (each a multiple of 16); otherwise N rows each
    int hetero = 0;
    int64_t roff[GEMV_MAX_MATS + 1] = {};
    // matrix rep_mat (at most one per launch; -1 = none) is written straight into the GQA copies of a
    // KV cache: row n -> (n / yrg) * yrgs + (n % yrg) * yrs, stored at +k * yrep for k < nrep.  Kept to
    // a few scalars: the job is a kernel argument re-set in every recorded step graph.
    int32_t rep_mat = -1, yrg = 0, nrep = 0;
    int64_t yrgs = 0, yrep = 0;
    int dbg = 0;    // phase study (TTS_HIP_OPT_GEMV_DEBUG): 1 = skip the row phase, 2 = skip the prologue
    const float * lnw = nullptr;
    const float * lnb = nullptr;
    float eps = 0.f;
    int rms = 0;
    float * lnout = nullptr;
    int64_t locs = 0;
    // PRO_COPY (matrix-core kernels): the Q8_K activation already in the kernel's LDS operand layout
    // ([M*nb + 1][256] f16, [M*nb + 1][16] f16 bsum halves, [M*nb + 1] f32 d; bq_bytes, a multiple of
    // 1 KiB), written by k_quant_mf
    const char * bq = nullptr;
    int64_t bq_bytes = 0;
    int64_t bq_tile = 0;  // > 0: columns in tiles of 16, tile c's operands at bq + c * bq_tile (its own slot layout)
    int32_t bq_slot = 0;  // halves per operand slot (0 = QK_K; the prefill GEMM pads slots to QK_K + 8 so a block's
                          // 16 columns sit on different LDS banks)
    unsigned long long * ts = nullptr;  // phase timestamps (scripts/gemv_phase.hip builds only)
    // ragged columns (a coalesced step's KV-cache stores, coalesce.hip): for the matrices in yoff_mats,
    // column m of matrix mat is stored at Y[mat] + m * ycs + yoff[mat * yoff_ld + m] (floats) -- each
    // member's cache row at its own position
    const int64_t * yoff = nullptr;
    int32_t yoff_mats = 0, yoff_ld = 0;
    int32_t xcd_cols = 0;  // many-column K-relay GEMM: a row tile's column tiles on one XCD (TTS_HIP_OPT_GEMM_KR_XCD)
};
__host__ __device__ inline int64_t job_roff(const GemvJob & j, int m) { return j.hetero ? j.roff[m] : (int64_t)m * j.N; }
__host__ __device__ inline int64_t job_rows(const GemvJob & j) { return job_roff(j, j.nmat); }
// In-kernel phase timestamps (s_memrealtime, 100 MHz) per wave, compiled in only by the
// micro-benchmark build (-DTTS_PHASE_TS): ts[(wg * waves + wave) * 8 + k].
#ifdef TTS_PHASE_TS
#define TTS_TS(job, k)                                                                                            \
    do {                                                                                                          \
        if ((job).ts && (threadIdx.x & 63) == 0)                                                                  \
            (job).ts[((((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + \
                      (threadIdx.x >> 6)) * 8 +                                                                   \
                     (k)] = __builtin_amdgcn_s_memrealtime();                                                     \
    } while (0)
#else
#define TTS_TS(job, k) \
    do {               \
    } while (0)
#endif
enum { PRO_QUANT = 1, PRO_LN = 2, PRO_COPY = 3 };  // PRO_COPY: operands pre-quantized at GemvJob::bq
// Cross-attention over a short context folded into the Q4_K GEMV that produces its query
// (k_gemv_q4K_xattn): K view [hd, P, H, B], V view [P, hd, H, B] (f32), out [hd, H, 1, B].
struct XAttnArgs {
    TD k, v;
    const float * mask = nullptr;  // [P] row 0 (n = 1), or null
    float scale = 1.f;
    float * out = nullptr;
    float * out2 = nullptr;        // optional private copy (the next GEMV's input, be->shadow), [hd, H, B] contiguous
    int P = 0, H = 0, B = 0;
    int64_t obs = 0;               // floats between sequences of out (0: H * hd, contiguous)
    int64_t mbs = 0;               // floats between sequences' masks (0: one mask for all)
    // ragged sequences (coalesce.hip): per-sequence K / V byte offsets, mask offsets (floats), key counts
    const int64_t * koff = nullptr;
    const int64_t * voff = nullptr;
    const int64_t * moff = nullptr;
    const int * pseq = nullptr;
};

// A coalesced decode step (coalesce.hip): N one-prompt decode graphs of different backends (TTS.cpp's
// server runs one runner per worker, examples/server/server.cpp:316-321) that differ at most in their KV
// lengths run as ONE plan of member 0's graph with M = N columns / B = N sequences.
//  - Intermediates (every tensor the graph allocator placed, i.e. not a leaf or a view of one) are
//    computed in executor-owned memory laid out as member 0's compute buffer, member k at win + k *
//    stride: one uniform column / sequence stride, which the GEMV, attention, norm and embedding
//    kernels take.  The graph's output node is copied to each member's own tensor afterwards.
//  - Member-owned operands (KV-cache views read by attention and written by the K / V store
//    epilogues, masks and token / position inputs) are each member's own tensors, found by node
//    position in its graph, and reach the kernels as per-member offset tables (ItemTab), together
//    with each member's own key count.
//  - Read-only model data (weights, norms, tables) is read through member 0's copy, checked equal to
//    each member's own copy on the device first.
constexpr int EMBED_MAX_TERMS = 16;
struct BatchCls {
    const char * b0 = nullptr;  // member 0's buffer
    size_t size = 0;
    char * win = nullptr;       // executor memory: member k's copy of the range at win + k * stride
    int64_t stride = 0;
};
// per-item tables of member-owned operands (device pointers, valid for the current coalesced plan)
struct ItemTab {
    const int64_t * yoff = nullptr;  // GEMV: [nmat][N] store offsets (floats) of the matrices in yoff_mats
    int32_t yoff_mats = 0;
    const int64_t *koff = nullptr, *voff = nullptr;  // ATTN: K / V view offsets per member (bytes)
    const int64_t * moff = nullptr;                  // ATTN: mask offsets per member (floats)
    const int * pseq = nullptr;                      // ATTN: key count per member
    int pmax = 0;
    const int64_t * ioff[EMBED_MAX_TERMS] = {};      // EMBED: index offsets per member (elements)
};
struct BatchCtx {
    int N = 0;
    uint64_t key = 0;  // the group: graph signature and member backends (coalesce.hip caches per key)
    std::vector<BatchCls> cls;  // sorted by b0
    std::vector<tts_tensor * const *> mnodes;  // every member's node list (member 0's first; equal lengths)
    std::vector<tts_hip_backend *> mbe;         // every member's backend (the read-back of its outputs)
    int n_nodes = 0;
    bool checked = false;       // this group's shapes and read-only operands were verified by an earlier step
    int canon = 0;              // the member whose read-only data every other member's is compared with (stable per set)
    bool ragged = false;        // (co_prepare) the members' KV lengths differ
    bool differs = false;       // refused because a member's read-only data differs (not for lack of a batched form)
    std::vector<ItemTab> tabs;  // per plan item (graph_exec.hip)
    void * comap = nullptr;     // graph_exec.hip: member 0's tensors -> graph positions (member k's counterparts)
    const BatchCls * find(const void * p) const {
        const char * c = (const char *)p;
        size_t lo = 0, hi = cls.size();
        while (lo < hi) {
            const size_t m = (lo + hi) / 2;
            if (cls[m].b0 <= c) lo = m + 1;
            else hi = m;
        }
        if (lo == 0) return nullptr;
        const BatchCls & b = cls[lo - 1];
        return c < b.b0 + b.size ? &b : nullptr;
    }
    // the executor address of member 0's intermediate p (p itself when it is not one)
    template <typename T>
    T * win(T * p) const {
        const BatchCls * b = p ? find(p) : nullptr;
        return b ? (T *)(b->win + ((const char *)p - b->b0)) : p;
    }
    int64_t stride(const void * p) const {  // bytes between members' copies (0: not an intermediate)
        const BatchCls * b = p ? find(p) : nullptr;
        return b ? b->stride : 0;
    }
    template <typename T>
    T * reloc(T * p, int k) const {  // member k's executor copy of member 0's intermediate p
        const BatchCls * b = p ? find(p) : nullptr;
        return b ? (T *)(b->win + k * b->stride + ((const char *)p - b->b0)) : p;
    }
};

}  // namespace tts

struct tts_hip_backend {
    int device = 0;
    hipStream_t stream = nullptr;
    char name[64] = {0};
    // scratch arena for activation quantization
    char * scratch = nullptr;
    size_t scratch_size = 0;
    // private second copy of an attention output, read by the GEMV that consumes it when the graph
    // allocator has placed that GEMV's output on the attention output's memory
    float * shadow = nullptr;
    size_t shadow_size = 0;
    // outputs of grouped products hoisted over nodes that still use their memory (graph_exec try_gemv)
    void * hoist = nullptr;
    size_t hoist_size = 0;
    // split decode attention: masked, scaled scores [B][n][H][P] and per-chunk maxima between the
    // scores kernel and the softmax + P.V kernel (consumed by the very next launch on the stream)
    float * attn_buf = nullptr;
    size_t attn_floats = 0;
    int attn_split_minp = 128;
    int attn_ks = 2;   // split scores: 128 * attn_ks positions per workgroup (TTS_HIP_OPT_ATTN_KS)
    int attn_pv_mp = 1;  // split P.V: every dim of a (head, query, sequence) in one workgroup (TTS_HIP_OPT_ATTN_PV_MP)
    int attn_pv8 = 0;  // split P.V: 8 output dims per workgroup instead of 16 (TTS_HIP_OPT_ATTN_PV8)
    int attn_pv_uv16 = 0;  // split P.V: one 16-chunk V batch per lane for P <= 1024 (TTS_HIP_OPT_ATTN_PV16; measured equal, off)
    int attn_fused_minp = 0;  // the one-launch 1024-thread decode attention from this many keys (0 = off: measured no faster in the Parler step)
    unsigned long long * argmax_keys = nullptr;  // k_greedy_step_wide: per-row keys / arrival counts (self-clearing)
    unsigned * argmax_counts = nullptr;
    // weight_set: Q4_K matrices >= this size use the tile layout + matrix-core GEMV (0 = never)
    int64_t q4k_tile_bytes = 4 << 20;
    // TTS_HIP_OPT_GEMV_DEBUG phase-study bitmask of the matrix-core GEMV: 1 = skip the row phase,
    // 2 = skip the prologue, 4 = plain (cached) weight loads (results invalid; micro-benchmarks only)
    int gemv_dbg = 0;
    // Q4_K GEMVs in the lane layout run the unique-load kernel (k_gemv_q4_K_u) where the shape fits
    int gemv_unique = 1;
    int gemm_q8 = 1;    // TTS_HIP_OPT_GEMM_Q8
    int64_t cus = 256;  // compute units this backend's stream may use (TTS_HIP_OPT_CU_PARTITION); grids are sized to it
    int cu_total = 256;
    int bgemm_f32 = 1;  // TTS_HIP_OPT_BGEMM_F32
    int gemv_f32_wide = 1;  // TTS_HIP_OPT_GEMV_F32_WIDE
    int gemm_kr_nw = 4;     // TTS_HIP_OPT_GEMM_KR_NW: waves per tile of the many-column K-relay GEMM (4 or 8)
    // tile-layout Q4_K GEMVs of at most this many 16-row tiles (M <= 8, K <= 4096) run the K-split
    // matrix-core kernel k_gemv_q4K_ks (0 = never)
    int64_t gemv_ks_tiles = 256;
    int gemv_mf_prequant = 1;  // TTS_HIP_OPT_GEMV_PREQUANT
    int gemv_kr = 1;           // TTS_HIP_OPT_GEMV_KRELAY
    int gemv_kr_loop = 1;      // TTS_HIP_OPT_GEMV_KRELAY_LOOP
    int gemv_q80_pro = 1;      // TTS_HIP_OPT_GEMV_Q80_PRO
    int gemv_q80_slab = 1;     // TTS_HIP_OPT_GEMV_Q80_SLAB
    int gemv_q80_rw = 0;       // TTS_HIP_OPT_GEMV_Q80_RW
    int gemm_q8_staged = 2;    // TTS_HIP_OPT_GEMM_Q8_STAGED
    int64_t gemv_kr_ink = 0;   // TTS_HIP_OPT_GEMV_KR_INKERNEL (max K)
    int gemm_kr_walk = 0;      // TTS_HIP_OPT_GEMM_KR_WALK: row-tile walkers per column tile of a many-column GEMM
    int gemm_pf = 64;          // TTS_HIP_OPT_GEMM_PF: many-column Q4_K products of >= value columns on k_gemm_q4K_pf (0 = off)
    int gemm_pf_nw = 4;        // TTS_HIP_OPT_GEMM_PF_NW: waves per prefill-GEMM workgroup (4 or 8)
    int gemm_kr_cp = 0;        // TTS_HIP_OPT_GEMM_KR_CP: two column tiles per workgroup on parallel wave halves
    int gemm_kr_xcd = 0;       // TTS_HIP_OPT_GEMM_KR_XCD: a row tile's column tiles on one XCD (measured no gain: off)
    int gemm_kr_ct2 = 0;       // TTS_HIP_OPT_GEMM_KR_CT2: two 16-column tiles per K-relay GEMM workgroup (K <= 2048)
    int64_t gemm_kr_ink = 0;   // TTS_HIP_OPT_GEMM_KR_INKERNEL (max M of the many-column K-relay GEMM without the operand pass)
    int gemv_nw_min = 0;       // TTS_HIP_OPT_GEMV_NW_MIN: minimum waves per lane-layout Q4_K GEMV workgroup
    int gemv_mf_rsplit = 1;  // matrix-core GEMV: split a tile's residues over 2 / 4 waves when tiles are few (TTS_HIP_OPT_GEMV_RSPLIT)
    // weight_set: lane-layout Q4_K matrices of >= this size (and below q4k_tile_bytes) also keep a
    // tile-layout copy (TTS_FLAG_TILED_COPY); GEMVs of >= 8 columns read it (0 = never)
    int64_t q4k_dual_bytes = 1 << 20;
    // (the tile-layout copies and the live buffer ranges are process-wide, tiled_copy_find: a weight
    // buffer is allocated and written through one backend and read by the graphs of others -- the
    // ggml adapter's buffer type allocates through a utility backend, each ggml_backend computes on
    // its own stream)
    void * sample_cand = nullptr;  // wide-vocabulary sampling candidates (k_sample.hip)
    size_t sample_cand_size = 0;
    // KV prefetch of the next attention into MALL on a side stream (0 = off; else min KV length)
    int kv_prefetch_minp = 0;  // measured slower (Parler B = 8: 2.04 -> 2.53..3.16 ms/step), off by default
    int kv_prefetch_blocks = 128;
    hipStream_t pf_stream = nullptr;
    hipEvent_t pf_fork = nullptr, pf_join = nullptr;
    // tts_hip_tensor_set_async staging: a pinned ring; a region is reused once the event recorded
    // after its copy has completed (ggml_backend_i::set_tensor_async semantics: the caller may
    // reuse its buffer at once, the copy is ordered on the compute stream)
    uint8_t * pin = nullptr;
    size_t pin_size = 0, pin_head = 0;
    struct PinRec {
        size_t off, size;
        hipEvent_t ev;
    };
    std::deque<PinRec> pin_pending;
    std::vector<hipEvent_t> pin_events;
    std::mutex pin_mu;  // the ring is shared by every thread that uploads through this backend
    // completion of each plan slot's last launch: a slot is re-recorded only after it ran
    hipEvent_t plan_ev[2] = {nullptr, nullptr};
    bool plan_ev_pending[2] = {false, false};
    float * lstm_buf = nullptr;  // fused LSTM chains: per chain [Hd] cell state + [Hd, T] hidden history
    float * conv_stage = nullptr;  // fused conv output staging when it would alias its input and the im2col buffer is too small
    size_t conv_stage_floats = 0;
    float * vec_scratch = nullptr;  // 256K floats: per-channel vectors a fused item copies away from its output
    size_t lstm_floats = 0;
    tts::ActQuant aq;
    int64_t graph_epoch = 0;
    uint16_t * gelu_table = nullptr;  // 65536 fp16 entries (GGML_GELU_FP16 table)
    bool convt_lds = true;  // conv_transpose_1d on the LDS-staged f64 MFMA kernel (A/B knob)
    // f64 partial sums of input-channel-split codec convolutions (short sequences: the output
    // tiles alone would leave most CUs idle), summed in split order by a second pass
    double * conv_part = nullptr;
    size_t conv_part_doubles = 0;
    int conv_split = 1;  // TTS_HIP_OPT_CONV_SPLIT: 1 = split short convolutions to ~512 workgroups, N > 1 = to ~N, 0 = never
    int fusion = 0x3FFF;  // bitmask of TTS_FUSE_* patterns (all on)
    bool profile_gemv = false;
    double gemv_ms[TTS_TYPE_COUNT] = {0};
    int64_t gemv_launches[TTS_TYPE_COUNT] = {0};
    double gemv_bytes[TTS_TYPE_COUNT] = {0};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    std::vector<double> ev_bytes;
    std::vector<int> ev_type;
    std::vector<hipEvent_t> ev_free;
    char * repack_tmp = nullptr;  // device temp for Q4_K matrices not stored repacked
    size_t repack_tmp_size = 0;
    std::vector<char *> repack_retired;  // outgrown repack temps (freed with the backend)
    // HIP graph replay of graph_compute (capture -> exec update -> one launch)
    bool use_graphs = false;
    // repeat detection for tts_hip_graph_compute: signatures of the last few graphs (node count, op
    // sequence, first / last shapes), each with its own executable graph so interleaved runners
    // (a decode step between vocoder calls) keep replaying
    static constexpr int N_GSIG = 4;
    uint64_t gsig[N_GSIG] = {};
    hipGraphExec_t gsig_exec[N_GSIG] = {};
    int gsig_next = 0;
    bool conv_f32acc = false;  // conv GEMM on f16 MFMA with f32 accumulation (faster, misses the PCM bar)
    int conv_acc_mode = 0;     // fused conv_1d: 0 = f64 MFMA, 2 = f16 MFMA per 32-term batch + f64 accumulation
    hipStream_t cap_stream = nullptr;  // records graphs (never runs work)
    int64_t graph_updates = 0, graph_instantiations = 0;
    int64_t lstm_chains = 0, lstm_steps = 0;
    int64_t plan_wait_ns = 0;
    int64_t cap_plan_ns = 0, cap_launch_ns = 0, cap_update_ns = 0;  // capture_into phases (host)  // host time spent in graph_prepare waiting for the slot's previous launch  // fused LSTM recurrences launched (tts_hip_counters)
    // two prepared plans (tts_hip_graph_prepare / _launch): step n+1 is recorded while step n runs
    hipGraphExec_t pexec[2] = {nullptr, nullptr};
    tts_tensor * const * plan_nodes[2] = {nullptr, nullptr};
    int plan_n[2] = {0, 0};
    bool plan_eager[2] = {true, true};
    bool plan_prepared[2] = {false, false};  // recorded by graph_prepare, not launched yet
    // step coalescer (coalesce.hip): set while this (hidden, per-device) backend runs a coalesced
    // plan; co_ev orders a member's stream with the coalesced launch
    tts::BatchCtx * bat = nullptr;
    hipEvent_t co_ev = nullptr;
    int64_t * co_tab = nullptr;  // device copy of a coalesced plan's per-item tables (ItemTab)
    size_t co_tab_bytes = 0;
    int64_t co_prep_ns = 0;      // host time of co_prepare + the tables' upload (coalesced steps)
    bool co_member = true;  // TTS_HIP_OPT_COALESCE: this backend's graph_compute calls may join a coalesced step
    // read-back of a coalesced step's outputs: the executor copies this member's output tensors into
    // rb_host (pinned) in the step's own stream order, so tts_hip_tensor_get of such a range is served
    // from host memory after a stream synchronize instead of one device-to-host copy per member.
    // Entries are valid until this backend's next write or compute call (rb_clear).
    struct RbEnt {
        const char * dev;
        size_t bytes, off;
    };
    char * rb_host = nullptr;
    size_t rb_cap = 0;
    std::vector<RbEnt> rb;
    std::mutex rb_mu;                  // rb: the executor's thread writes it, this backend's callers read / drop it
    std::atomic<bool> rb_any{false};   // rb non-empty (checked before taking rb_mu)
    void rb_clear() {
        if (!rb_any.load(std::memory_order_acquire)) return;
        std::lock_guard<std::mutex> l(rb_mu);
        rb.clear();
        rb_any.store(false, std::memory_order_release);
    }
};

namespace tts {

// ---- process-wide weight registry (backend.hip) ----
// The tile-layout copy of a lane-layout Q4_K weight (TTS_FLAG_TILED_COPY), or null.
const uint8_t * tiled_copy_find(const void * weight);

// ---- profiled launches (k_gemv.hip): a start / stop event pair carried in the dispatch packets
// (hipExtLaunchKernelGGL), folded into tts_hip_gemv_stats under `type` with `bytes` algorithmic bytes
void profile_pair(tts_hip_backend * be, hipEvent_t & e0, hipEvent_t & e1);
void profile_push(tts_hip_backend * be, hipEvent_t e0, hipEvent_t e1, double bytes, int type);

// ---- launchers (k_gemv.hip) ----
// Quantize M columns (column stride xcs floats) of x to the vec_dot type of `wtype`.
void launch_quantize_act(tts_hip_backend * be, int wtype, const float * x, int64_t xcs, int64_t K, int64_t M, ActQuant & aq);
void launch_gemv_job(tts_hip_backend * be, const GemvJob & job);
// F32 weights x many columns (k_gemm.hip): bit-identical to the sequential-f64 float dot
bool launch_bgemm_f32(tts_hip_backend * be, const tts_tensor * node);
bool gemm_f32_ok(const GemvJob & j);
void launch_gemm_f32(tts_hip_backend * be, const GemvJob & j);
void launch_copy_cols(tts_hip_backend * be, float * dst, const float * src, int64_t K, int64_t scs, int64_t M);
void launch_profile_spin(tts_hip_backend * be, double us);
void launch_im2col(tts_hip_backend * be, const tts_tensor * node);
// One fused LSTM recurrence step (Kokoro build_lstm_run, src/models/kokoro/model.cpp:56-86): the
// four h-GEMVs, bias and input-projection adds, gate activations and the cell update, gate order
// I, F, G, O (weights[1], [3], [5], [7] of the reference's cell).
struct LstmStepArgs {
    const float * pre[4];   // column t of each gate's input projection (W_ih x + b_ih), Hd floats
    const void * w[4];      // W_hh [Hd rows of K], F32 or F16
    int64_t w_rs[4];        // row stride, bytes
    const float * bias[4];  // b_hh [Hd]
    const float * hprev;    // [K]
    const float * cprev;    // [Hd]
    float * h;              // [Hd] out
    float * c;              // [Hd] out (may alias cprev: per-unit read-then-write)
    int Hd, K, wtype;
};
// b: a second, independent chain advanced by the same launch (bidirectional pairs), or null
void launch_lstm_step(tts_hip_backend * be, const LstmStepArgs & a, const LstmStepArgs * b = nullptr);
void launch_repeat_interleave1(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * a, int r);
void launch_copy_bytes(tts_hip_backend * be, void * dst, const void * src, size_t bytes);
void launch_cpy_multi(tts_hip_backend * be, const tts_tensor * src, const tts_tensor * const * dsts, int nd);
void launch_rope_multi(tts_hip_backend * be, const tts_tensor * rope, const tts_tensor * src, const tts_tensor * const * dsts, int nd);
void launch_greedy_step(tts_hip_backend * be, const float * logits, int B, int NH, int V, int step, int bos, int eos, int32_t * eos_seen,
                        int32_t * hist, int32_t * next);
int launch_sample_step(tts_hip_backend * be, const float * logits, int B, int NH, int V, const tts_sampling * c, int64_t call,
                       int32_t * rep_state, int step, int bos, int eos, int32_t * eos_seen, int32_t * hist, int32_t * next);
struct BatchCtx;
void launch_embed_sum(tts_hip_backend * be, const tts_tensor * out, const tts_tensor * const * gr, int n, const BatchCtx * bat = nullptr,
                      const ItemTab * tab = nullptr);
// recip == nullptr: the kernel evaluates reciprocal() = one[0] / alpha[c] itself (`one` a broadcast scalar)
void launch_snake(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * x, const tts_tensor * alpha, const tts_tensor * recip,
                  const tts_tensor * one = nullptr, const tts_tensor * mask = nullptr);
void launch_lstm_finish(tts_hip_backend * be, const tts_tensor * final_out, const float * hist, int64_t Hd, int64_t T);
bool audio_op_supported(const tts_tensor * n);
int launch_audio_op(tts_hip_backend * be, const tts_tensor * n);
void launch_conv_transpose_1d(tts_hip_backend * be, const tts_tensor * node);
// conv_1d chain (IM2COL -> MUL_MAT [-> ADD bias] [-> ADD residual]) as one implicit-GEMM kernel
constexpr int CONV1D_MAX_R = 128;
struct Conv1dArgs {
    TD x;                           // input [L, IC] f32 (any strides)
    const void * w = nullptr;       // kernel [K, IC, OC], element strides wk / wic / woc
    int w16 = 0;                    // kernel stored as F16 (else F32)
    int64_t wk = 0, wic = 0, woc = 0;
    float * y = nullptr;            // output [OL, OC]: y[ol + oc * ycs]
    int64_t ycs = 0;
    const float * bias = nullptr;   // bias[oc * bcs] or null
    int64_t bcs = 0;
    const float * res = nullptr;    // residual [OL, OC] (res[ol + oc * rcs]) or null
    int64_t rcs = 0;
    int64_t L = 0, IC = 0, OL = 0, OC = 0;
    int K = 1, s = 1, p = 0, d = 1;
    int icc = 0, xw = 0, rs = 0;    // set by the launcher
    float * copy_dst = nullptr;     // non-null: y is a staging buffer, copied here (contiguous) after the kernel
    uint32_t x_bytes = 0, w_bytes = 0;  // buffer-descriptor ranges (reads past them return 0)
    double * part = nullptr;        // split launch: f64 partial sums [gridDim.z][OC][OL], no epilogue
    int ic_per_split = 0;           // input channels per split (a multiple of icc)
};
constexpr int CONV1D_XN = 16, CONV1D_WN = 16;  // staged elements per thread (x window, kernel slice)
inline int conv1d_icc(int64_t IC, int K, int xw) {  // input channels per LDS chunk
    // the reduction (icc * K) is padded to whole batches of 32 and held to 64 (so the kernel
    // slice is 64 x 64 floats, CONV1D_WN per thread); the x window (icc * xw floats) to
    // CONV1D_XN per thread.  Pick the icc that wastes the least, preferring larger chunks.
    int best = 0;
    double best_eff = -1.0;
    const int top = (int)(IC < 64 ? IC : 64);
    for (int c = 1; c <= top; ++c) {
        const int r = c * K, rp = (r + 31) & ~31;
        if (rp > 64 || c * xw > 256 * CONV1D_XN) break;
        const double eff = (double)r / rp + 1e-4 * c;
        if (eff > best_eff) best_eff = eff, best = c;
    }
    return best;  // 0: the shape does not fit (K > 64 or a window too wide)
}
bool conv1d_fused_ok(int64_t IC, int K, int s, int d, size_t * lds);
// AdaIN (+ snake) per channel row: y[c][t] = snake((norm(x[c])[t] * (1 + g[c])...) -- see k_fused.hip
struct AdainArgs {
    const float * x = nullptr;   // NORM input rows: x[c * xcs + t], t < T
    int64_t xcs = 0;
    float * y = nullptr;         // output rows (the [T, C] tensor after the second transpose)
    int64_t ycs = 0;
    const float *gamma = nullptr, *beta = nullptr, *alpha = nullptr, *recip = nullptr;  // alpha null: no snake
    const float * one = nullptr;  // recip null: recip[c] = one[0] / alpha[c] (reciprocal()'s DIV)
    int stage = 0;  // 1: the output overlaps a vector's memory -> copy the vectors to be->vec_scratch first
    // gamma / beta evaluated in the kernel (their MUL_MAT + bias ADD absorbed): gamma[c] =
    // dot(gw[c * S ...], style) + gb[c], in k_gemv_float's exact order; gw null: read gamma / beta
    const float *gw = nullptr, *gb = nullptr, *bw = nullptr, *bb = nullptr, *style = nullptr;
    int64_t S = 0;
    int64_t gcs = 1, bcs = 1, acs = 1, rcs = 1;
    int64_t T = 0, C = 0;
    float eps = 0.f;
};
bool adain_supported(int64_t T);
void launch_adain_snake(tts_hip_backend * be, const AdainArgs & a);
void launch_conv1d_fused(tts_hip_backend * be, Conv1dArgs a);
bool launch_gemm_f16(tts_hip_backend * be, const tts_tensor * node);
size_t act_quant_bytes(int wtype, int64_t K, int64_t M);
// carve an ActQuant layout for weight type `wtype` out of `base` (no launch)
void act_quant_layout(int wtype, char * base, int64_t K, int64_t M, ActQuant & aq);

void launch_repack_q4_K(tts_hip_backend * be, const void * src, void * dst, int64_t nblocks, int inverse);

// ---- launchers (k_ops.hip) ----
int launch_op(tts_hip_backend * be, const tts_tensor * node);
void launch_copy_stream(tts_hip_backend * be, void * dst, const void * src, int64_t n16);  // tts_hip_copy_stream

// ---- graph execution (graph_exec.hip) and the step coalescer (coalesce.hip) ----
// Plan and launch a node list on be->stream (be->bat set: as a coalesced step of be->bat->N members;
// TTS_STATUS_UNSUPPORTED, before any launch, when the plan has an item without a coalesced form).
int graph_compute_launches(tts_hip_backend * be, tts_tensor * const * nodes, int n_nodes);
// graph_compute of a one-prompt decode graph while other backends on the device submit the same graph:
// one coalesced launch for all of them.  Returns kCoalesceNotTaken when the caller runs the graph itself.
constexpr int kCoalesceNotTaken = 1 << 20;
int coalesce_submit(tts_hip_backend * be, tts_tensor * const * nodes, int n_nodes);
// buffer registry (backend.hip): the live tts_hip_buffer_alloc range holding p
bool buffer_lookup(const void * p, const char ** base, size_t * size);
// a coalesced step's read-only operands read through member 0's copy: (member 0's, member k's, bytes)
// pairs, true when every pair holds equal bytes (checked on the device, cached until a host write)
bool coalesce_check_shared(tts_hip_backend * ex, const std::vector<std::tuple<const void *, const void *, size_t>> & pairs);
void coalesce_backend_gone(const tts_hip_backend * be); // a backend is freed: no longer awaited
void coalesce_written(const void * p, size_t size);     // host writes: content checks over the range are dropped
bool coalesce_enabled();
bool co_debug();  // TTS_HIP_COALESCE_DEBUG=1 (graph_exec.hip)

}  // namespace tts
