// Seeded sampling on the device (sampler::sample, /root/reference/src/sampler.cpp:3-204), bit-identical
// to the host restatement tts_sampler_sample (sampler.cpp): the same penalised / tempered values,
// the same top-k order (key descending, index ascending), the same sequential f32 sums in pick
// order, the same minstd_rand draws (jumped ahead to head h's draw), the same cumulative rule.
// One workgroup per (prompt b, head h) row.  The order is a bitonic sort in LDS of 64-bit keys
// (~orderable(key) << 32 | index), so ascending keys = values descending, then lower index first.
//
//  k_sample_rows  : V <= 4096 (Parler 1088, Dia 1028): every sampler configuration.
//  k_topk_segments + k_sample_wide: wider vocabularies (Orpheus, 156 940): each 4096-logit segment
//                   keeps its 64 best keys, one workgroup per row sorts the candidates and samples
//                   (0 < top_k <= 64, top_p >= 1: the generation_configuration default top_k = 50).
#include "hip_internal.h"

namespace tts {

namespace {

constexpr int SMAX = 4096;  // keys per LDS sort
constexpr int KC = 64;      // candidates kept per segment (wide vocabularies)

struct SampleArgs {
    const float * logits;
    int B, NH, V;
    float temperature, top_p, rep;
    int top_k, do_sample;
    uint64_t seed;
    int64_t call;
    int32_t * rep_state;  // [B*NH][2]: last token, count
    int step, bos, eos;
    int32_t *eos_seen, *hist, *next;
    unsigned long long * cand;  // wide: [B*NH][nseg][KC]
    int nseg;
};

__device__ __forceinline__ uint32_t ord_f32(float f) {
    const uint32_t u = __float_as_uint(__fadd_rn(f, 0.0f));  // -0 -> +0: equal floats, equal keys
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ unsigned long long sort_key(float v, int i) {
    return ((unsigned long long)(~ord_f32(v)) << 32) | (unsigned)i;
}

// ascending bitonic sort of n (power of two) keys in LDS, 256 threads
__device__ void bitonic(unsigned long long * k, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int t = threadIdx.x; t < n / 2; t += blockDim.x) {
                const int lo = 2 * t - (t & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = k[lo], b = k[hi];
                if ((a > b) == up) {
                    k[lo] = b;
                    k[hi] = a;
                }
            }
        }
    }
    __syncthreads();
}

// std::minstd_rand seeded with s, advanced n times (n >= 1): x <- 48271 x mod (2^31 - 1)
__device__ __forceinline__ uint32_t minstd_at(uint32_t s, int n) {
    uint64_t x = s;
    for (int i = 0; i < n; ++i) x = (x * 48271ull) % 2147483647ull;
    return (uint32_t)x;
}
// std::uniform_real_distribution<float>(0, 1) over minstd_rand (libstdc++ generate_canonical<float, 24>:
// one draw, float(g - 1) / 2^31, clamped below 1)
__device__ __forceinline__ float canonical_f32(uint32_t g) {
    const float r = __fmul_rn((float)(g - 1u), 4.656612873077392578125e-10f);
    return r >= 1.0f ? __uint_as_float(0x3F7FFFFFu) : r;
}

__device__ __forceinline__ uint32_t call_seed_dev(uint64_t seed, int stream, int64_t call) {
    uint64_t z = seed ^ ((uint64_t)(uint32_t)stream << 40) ^ ((uint64_t)call * 0x9E3779B97F4A7C15ull);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(1 + z % 2147483646ull);
}

struct RowState {
    int last, count;
    double pw;  // pow(penalty, count)
    bool rep, temp;
};

__device__ __forceinline__ float penal(const RowState & r, int i, float v) {
    return (r.rep && r.last == i) ? (float)((double)v / r.pw) : v;
}
__device__ __forceinline__ float temper(const SampleArgs & a, const RowState & r, float v) {
    return r.temp ? __fdiv_rn(v, a.temperature) : v;
}

// the draw of row (b, h), its cumulative choice over n picks with probabilities p[j], the
// repetition-penalty update and greedy_step's EOS / next-token rule (thread 0 only)
__device__ void finish_row(const SampleArgs & a, RowState & r, int row, int tok) {
    const int b = row / a.NH, h = row % a.NH;
    if (r.rep && a.do_sample) {  // sampler::max (do_sample = 0) leaves the penalty state alone
        if (r.last != tok) r.count = 0;
        r.last = tok;
        r.count += 1;
        a.rep_state[2 * row] = r.last;
        a.rep_state[2 * row + 1] = r.count;
    }
    a.hist[row] = tok;
    const int seen = a.eos_seen[row] | (tok == a.eos);
    a.eos_seen[row] = seen;
    a.next[h * a.B + b] = a.step + 1 > h ? (seen ? a.eos : tok) : a.bos;
}

__device__ int draw_pick(const SampleArgs & a, int row, const float * p, const int * pick, int n, float mhp, bool topp) {
    const int b = row / a.NH, h = row % a.NH;
    float u = canonical_f32(minstd_at(call_seed_dev(a.seed, b, a.call), h + 1));
    if (topp) u = __fmul_rn(u, mhp);
    float cum = 0.0f;
    for (int j = 0; j < n; ++j) {
        cum = __fadd_rn(cum, p[j]);
        if (u <= cum || j >= n - 1) return pick ? pick[j] : j;
    }
    return 0;
}

__device__ void load_state(const SampleArgs & a, int row, RowState & r) {
    r.rep = a.rep != 1.0f;
    r.temp = a.temperature != 1.0f;
    r.last = r.rep ? a.rep_state[2 * row] : -1;
    r.count = r.rep ? a.rep_state[2 * row + 1] : 0;
    r.pw = r.rep ? pow((double)a.rep, (double)(uint32_t)r.count) : 1.0;
}

}  // namespace

__global__ __launch_bounds__(256) void k_sample_rows(SampleArgs a) {
    __shared__ unsigned long long keys[SMAX];
    __shared__ float pv[SMAX];
    __shared__ int pk[SMAX];
    __shared__ int s_n;
    __shared__ float s_max, s_cum, s_mhp;
    const int row = blockIdx.x;
    const int V = a.V;
    const float * l = a.logits + (int64_t)row * V;
    RowState r;
    load_state(a, row, r);
    int n2 = 1;
    while (n2 < V) n2 <<= 1;
    // sampler::max: first maximum of the penalised logits = the smallest key
    for (int i = threadIdx.x; i < n2; i += 256) keys[i] = i < V ? sort_key(penal(r, i, l[i]), i) : ~0ull;
    __syncthreads();
    unsigned long long best = ~0ull;
    for (int i = threadIdx.x; i < V; i += 256) best = keys[i] < best ? keys[i] : best;
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o < best ? o : best;
    }
    __shared__ unsigned long long s_best[4];
    if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = best;
    __syncthreads();
    for (int w = 0; w < 4; ++w) best = s_best[w] < best ? s_best[w] : best;
    const int maxi = (int)(best & 0xFFFFFFFFu);
    if (!a.do_sample) {
        if (threadIdx.x == 0) finish_row(a, r, row, maxi);
        return;
    }
    const bool topp = a.top_p < 1.0f;
    const bool usek = a.top_k > 0 && a.top_k < V;
    const float max_val = temper(a, r, penal(r, maxi, l[maxi]));
    if (topp) {
        // softmax over the whole vocabulary (index order): e_j in parallel, the sum sequentially
        for (int i = threadIdx.x; i < V; i += 256) pv[i] = cr_expf(__fsub_rn(temper(a, r, penal(r, i, l[i])), max_val));
        __syncthreads();
        if (threadIdx.x == 0) {
            float c = 0.0f;
            for (int i = 0; i < V; ++i) c = __fadd_rn(c, pv[i]);
            s_cum = c;
        }
        __syncthreads();
        const float cum = s_cum;
        for (int i = threadIdx.x; i < V; i += 256) pv[i] = __fdiv_rn(pv[i], cum);
        __syncthreads();
        // topk (by probability) or topp's full sort
        for (int i = threadIdx.x; i < n2; i += 256) keys[i] = i < V ? sort_key(pv[i], i) : ~0ull;
        bitonic(keys, n2);
        const int n = usek ? a.top_k : V;
        for (int j = threadIdx.x; j < n; j += 256) pk[j] = (int)(keys[j] & 0xFFFFFFFFu);
        __syncthreads();
        if (threadIdx.x == 0) {
            float ps = 0.0f;
            int trim = -1;
            for (int j = 0; j < n; ++j) {
                ps = __fadd_rn(ps, pv[pk[j]]);
                if (ps >= a.top_p) {
                    trim = j + 1;
                    break;
                }
            }
            s_mhp = ps < a.top_p ? ps : a.top_p;
            s_n = trim > 0 ? trim : n;
        }
        __syncthreads();
        // probabilities in pick order for the draw (keys[] reused as f32 storage)
        float * pp = (float *)keys;
        const int n_ = s_n;
        for (int j = threadIdx.x; j < n_; j += 256) pp[j] = pv[pk[j]];
        __syncthreads();
        if (threadIdx.x == 0) finish_row(a, r, row, draw_pick(a, row, pp, pk, n_, s_mhp, true));
        return;
    }
    if (usek) {
        bitonic(keys, n2);  // penalised logits: the max scan's keys
        const int k = a.top_k;
        for (int j = threadIdx.x; j < k; j += 256) {
            const int i = (int)(keys[j] & 0xFFFFFFFFu);
            pk[j] = i;
            pv[j] = cr_expf(__fsub_rn(temper(a, r, penal(r, i, l[i])), max_val));
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            float c = 0.0f;
            for (int j = 0; j < k; ++j) c = __fadd_rn(c, pv[j]);
            s_cum = c;
        }
        __syncthreads();
        for (int j = threadIdx.x; j < k; j += 256) pv[j] = __fdiv_rn(pv[j], s_cum);
        __syncthreads();
        if (threadIdx.x == 0) finish_row(a, r, row, draw_pick(a, row, pv, pk, k, 1.0f, false));
        return;
    }
    // no top-k, no top-p: softmax and the draw over the vocabulary in index order
    for (int i = threadIdx.x; i < V; i += 256) pv[i] = cr_expf(__fsub_rn(temper(a, r, penal(r, i, l[i])), max_val));
    __syncthreads();
    if (threadIdx.x == 0) {
        float c = 0.0f;
        for (int i = 0; i < V; ++i) c = __fadd_rn(c, pv[i]);
        s_cum = c;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += 256) pv[i] = __fdiv_rn(pv[i], s_cum);
    __syncthreads();
    if (threadIdx.x == 0) finish_row(a, r, row, draw_pick(a, row, pv, nullptr, V, 1.0f, false));
}

// wide vocabularies, stage 1: segment blockIdx.x of row blockIdx.y keeps its KC best keys
__global__ __launch_bounds__(256) void k_topk_segments(SampleArgs a) {
    __shared__ unsigned long long keys[SMAX];
    const int row = blockIdx.y, seg = blockIdx.x;
    const float * l = a.logits + (int64_t)row * a.V;
    RowState r;
    load_state(a, row, r);
    const int i0 = seg * SMAX;
    for (int t = threadIdx.x; t < SMAX; t += 256) {
        const int i = i0 + t;
        keys[t] = i < a.V ? sort_key(penal(r, i, l[i]), i) : ~0ull;
    }
    bitonic(keys, SMAX);
    for (int t = threadIdx.x; t < KC; t += 256) a.cand[((int64_t)row * a.nseg + seg) * KC + t] = keys[t];
}

// stage 2: the row's candidates sorted, top_k picks, softmax in pick order, the draw
__global__ __launch_bounds__(256) void k_sample_wide(SampleArgs a) {
    __shared__ unsigned long long keys[SMAX];
    __shared__ float pv[KC];
    __shared__ int pk[KC];
    __shared__ float s_cum;
    const int row = blockIdx.x;
    const float * l = a.logits + (int64_t)row * a.V;
    RowState r;
    load_state(a, row, r);
    const int nc = a.nseg * KC;
    int n2 = 1;
    while (n2 < nc) n2 <<= 1;
    for (int t = threadIdx.x; t < n2; t += 256) keys[t] = t < nc ? a.cand[(int64_t)row * nc + t] : ~0ull;
    bitonic(keys, n2);
    const int maxi = (int)(keys[0] & 0xFFFFFFFFu);
    if (!a.do_sample) {
        if (threadIdx.x == 0) finish_row(a, r, row, maxi);
        return;
    }
    const float max_val = temper(a, r, penal(r, maxi, l[maxi]));
    const int k = a.top_k;
    for (int j = threadIdx.x; j < k; j += 256) {
        const int i = (int)(keys[j] & 0xFFFFFFFFu);
        pk[j] = i;
        pv[j] = cr_expf(__fsub_rn(temper(a, r, penal(r, i, l[i])), max_val));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float c = 0.0f;
        for (int j = 0; j < k; ++j) c = __fadd_rn(c, pv[j]);
        s_cum = c;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < k; j += 256) pv[j] = __fdiv_rn(pv[j], s_cum);
    __syncthreads();
    if (threadIdx.x == 0) finish_row(a, r, row, draw_pick(a, row, pv, pk, k, 1.0f, false));
}

int launch_sample_step(tts_hip_backend * be, const float * logits, int B, int NH, int V, const tts_sampling * c, int64_t call,
                       int32_t * rep_state, int step, int bos, int eos, int32_t * eos_seen, int32_t * hist, int32_t * next) {
    SampleArgs a;
    a.logits = logits;
    a.B = B, a.NH = NH, a.V = V;
    a.temperature = c->temperature, a.top_p = c->top_p, a.rep = c->repetition_penalty;
    a.top_k = c->top_k, a.do_sample = c->do_sample;
    a.seed = c->seed, a.call = call;
    a.rep_state = rep_state;
    a.step = step, a.bos = bos, a.eos = eos;
    a.eos_seen = eos_seen, a.hist = hist, a.next = next;
    a.cand = nullptr, a.nseg = 0;
    if (a.rep != 1.0f && !rep_state) return TTS_STATUS_BAD_ARG;
    const int rows = B * NH;
    if (V <= SMAX) {
        hipLaunchKernelGGL(k_sample_rows, dim3((unsigned)rows), dim3(256), 0, be->stream, a);
        TTS_HIP_CHECK(hipGetLastError());
        return 0;
    }
    const int nseg = (V + SMAX - 1) / SMAX;
    const bool ok = nseg * KC <= SMAX && (!c->do_sample || (c->top_k > 0 && c->top_k <= KC && c->top_p >= 1.0f));
    if (!ok) return TTS_STATUS_UNSUPPORTED;
    const size_t need = (size_t)rows * nseg * KC * sizeof(unsigned long long);
    if (need > be->sample_cand_size) {
        if (be->sample_cand) {
            TTS_HIP_CHECK(hipStreamSynchronize(be->stream));
            TTS_HIP_CHECK(hipFree(be->sample_cand));
        }
        TTS_HIP_CHECK(hipMalloc(&be->sample_cand, need));
        be->sample_cand_size = need;
    }
    a.cand = (unsigned long long *)be->sample_cand;
    a.nseg = nseg;
    hipLaunchKernelGGL(k_topk_segments, dim3((unsigned)nseg, (unsigned)rows), dim3(256), 0, be->stream, a);
    hipLaunchKernelGGL(k_sample_wide, dim3((unsigned)rows), dim3(256), 0, be->stream, a);
    TTS_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace tts
