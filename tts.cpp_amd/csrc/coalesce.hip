// Step coalescer: TTS.cpp's one-prompt-per-runner serving shape run as batched decode steps.
//
// TTS.cpp's server scales by independent workers, each with its own runner, backend and model copy
// (/root/reference/examples/server/server.cpp:316-321,885-895), and each runner decodes one sequence
// per step graph (parler_tts_runner::decode, /root/reference/src/models/parler/model.cpp:648-693,
// model.h:158-172).  Unchanged, that is N streams of M = 1 GEMVs that each re-read every weight.
//
// Here every backend's graph_compute of a one-prompt decode step enters a per-device rendezvous.
// When the other recently active backends arrive with the same kind of step graph -- same ops, types,
// parameters, wiring and weight shapes; their KV lengths (so their attention shapes, cache positions
// and compute-buffer layouts) may differ -- the step runs ONCE as member 0's plan with M = N columns
// (graph_exec.hip, be->bat):
//   - intermediates are computed in executor memory laid out as member 0's compute buffer, member k's
//     copy at win + k * stride: one uniform column / sequence stride, which the GEMV, attention, norm
//     and embedding kernels take; the graph's output is copied to each member's own tensor afterwards;
//   - member-owned operands (each member's KV-cache rows written by the K / V store epilogues, its cache
//     and cross-attention views with its own key count, its masks and token / position inputs) are found
//     by graph position in the member's own graph and reach the kernels as per-member offset tables;
//   - read-only model data (weights, norm parameters, embedding tables) is read through member 0's copy
//     after a device-side check that every member holds equal bytes (each worker loads its own copy of
//     the model), cached until a host write touches the range;
//   - the coalesced launches run on a hidden per-device backend's stream, after every member's stream
//     (their input uploads), and every member's stream waits for them, so each caller's
//     get_tensor_async sees its own logits (ggml_backend_sched_graph_compute_async is followed by an
//     immediate read, src/tts_model.cpp:25-36).
// Each member's results are the same sums in the same order as its own step: the kernels compute a
// column / sequence independently of the others (tests/test_coalesce_gpu.py checks the tokens bit-exact
// against each runner alone and against the CPU oracle, also for runners at different KV lengths).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "hip_internal.h"

namespace tts {
namespace {

using Clock = std::chrono::steady_clock;

struct Req {
    tts_hip_backend * be = nullptr;
    tts_tensor * const * nodes = nullptr;
    int n = 0;
    uint64_t sig = 0;
    int64_t count = 0;  // the backend's coalescable submissions so far (its decode step number)
    bool taken = false, done = false;
    int status = kCoalesceNotTaken;
};
struct Act {
    Clock::time_point t;
    int64_t count = 0;
    std::thread::id tid;  // the thread of its last submission
};

constexpr int kMaxDev = 16;

struct Dev {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Req *> pending;
    std::unordered_map<const tts_hip_backend *, Act> seen;  // active backends: last coalescable submit
    std::mutex exec_mu;                   // one coalesced step at a time (guards everything below)
    tts_hip_backend * exec = nullptr;     // hidden backend: stream + scratch of the coalesced launches
    char * mem = nullptr;                 // executor memory for the members' intermediates
    size_t mem_bytes = 0;
    // Backends whose graphs of one kind (signature) were verified against each other (same shapes, equal
    // read-only data), as classes of a union-find per kind: a set whose members all lie in one class skips
    // the checks.  Dropped whenever a host write invalidates content records (g_eq_epoch).
    std::unordered_map<uint64_t, std::unordered_map<uintptr_t, uintptr_t>> equal;
    uint64_t equal_epoch = 0;
    std::unordered_set<uint64_t> no_form;   // kinds of graph whose plan has no coalesced form (never waited for again)
    int * d_flags = nullptr;              // content-check mismatch flags
    int d_flags_n = 0;
    // counters (tts_hip_coalesce_stats)
    std::atomic<int64_t> launches{0}, member_steps{0}, alone{0}, refused{0}, max_group{0}, wait_us{0}, ragged{0};
    std::atomic<int64_t> exec_ns{0}, layout_ns{0};  // host time of run_group, of exec_layout
};
Dev g_dev[kMaxDev];
std::atomic<int> g_wait_us{5000};

// Ranges known to hold equal bytes in member 0 and member k (content-checked), dropped when a host
// write touches either side.
struct EqRec {
    const char *a, *b;
    size_t n;
    bool eq;  // false: known to differ (not re-checked until a write)
};
struct EqKey {
    const char *a, *b;
    size_t n;
    bool operator==(const EqKey & o) const { return a == o.a && b == o.b && n == o.n; }
};
struct EqKeyHash {
    size_t operator()(const EqKey & k) const {
        return std::hash<const void *>()(k.a) ^ (std::hash<const void *>()(k.b) * 0x9E3779B97F4A7C15ull) ^ (k.n * 0xC2B2AE3D27D4EB4Full);
    }
};
std::mutex g_eq_mu;
std::unordered_map<EqKey, EqRec, EqKeyHash> g_eq;
uint64_t g_eq_epoch = 1;                            // bumped whenever a write drops records
std::map<const char *, const char *> g_eq_cover;  // disjoint union of every checked range: start -> end

void cover_add(const char * a, size_t n) {
    const char * e = a + n;
    auto it = g_eq_cover.upper_bound(a);
    if (it != g_eq_cover.begin()) {
        auto pr = std::prev(it);
        if (pr->second >= a) {
            a = pr->first;
            e = std::max(e, pr->second);
            it = g_eq_cover.erase(pr);
        }
    }
    while (it != g_eq_cover.end() && it->first <= e) {
        e = std::max(e, it->second);
        it = g_eq_cover.erase(it);
    }
    g_eq_cover[a] = e;
}
bool cover_hits(const char * p, size_t n) {
    auto it = g_eq_cover.upper_bound(p + n - 1);
    if (it == g_eq_cover.begin()) return false;
    --it;
    return it->second > p;
}
const EqRec * eq_known(const char * a, const char * b, size_t n) {
    auto it = g_eq.find(EqKey{a, b, n});
    return it == g_eq.end() ? nullptr : &it->second;
}

// ---- rendezvous ----
// A one-prompt decode step: every product over a 2-D weight matrix (a leaf) has one column.
bool decode_like(tts_tensor * const * nodes, int n) {
    if (n < 8) return false;
    bool any = false;
    for (int i = 0; i < n; ++i) {
        const tts_tensor * t = nodes[i];
        if (t->op != TTS_OP_MUL_MAT) continue;
        const tts_tensor *a = t->src[0], *b = t->src[1];
        if (!a || !b || a->op != TTS_OP_NONE || a->view_src || a->ne[2] != 1 || a->ne[3] != 1) continue;
        if (b->ne[1] * b->ne[2] * b->ne[3] != 1) return false;
        any = true;
    }
    return any;
}

// The kind of step a graph is: ops, types, parameters, layout flags and wiring (a source is the node
// it is, or a leaf described by its type and role), plus every weight's shape -- everything but the
// shapes and places that follow the KV length (attention over the cache, the store positions, the
// compute-buffer layout).  Graphs with equal signatures are coalesced; co_prepare (graph_exec.hip)
// then checks them against each other item by item.  Two independent 64-bit hashes, folded.
uint64_t signature(tts_tensor * const * nodes, int n) {
    // node -> index: an open-addressing table per thread (every decode step of every runner hashes its graph)
    thread_local std::vector<std::pair<const tts_tensor *, int>> tab;
    size_t cap = 64;
    while (cap < 2 * (size_t)n) cap <<= 1;
    tab.assign(cap, {nullptr, -1});
    const size_t mask = cap - 1;
    auto slot = [&](const tts_tensor * t) {
        size_t i = (size_t)(((uint64_t)(uintptr_t)t * 0x9E3779B97F4A7C15ull) >> 32) & mask;
        while (tab[i].first && tab[i].first != t) i = (i + 1) & mask;
        return i;
    };
    for (int i = 0; i < n; ++i) tab[slot(nodes[i])] = {nodes[i], i};
    uint64_t h = 0xCBF29CE484222325ull ^ (uint64_t)n, h2 = 0x84222325CBF29CE4ull + (uint64_t)n;
    auto mix = [&](uint64_t v) {
        h = (h ^ v) * 0x100000001B3ull;
        h2 = (h2 + v + 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
        h2 ^= h2 >> 31;
    };
    constexpr int kLayout = TTS_FLAG_INPUT | TTS_FLAG_OUTPUT | TTS_FLAG_REPACKED | TTS_FLAG_TILED | TTS_FLAG_TILED_COPY | TTS_FLAG_PERSIST;
    auto kind = [&](const tts_tensor * t) {
        mix((uint64_t)t->op << 32 | (uint32_t)t->type);
        for (int k = 0; k < TTS_MAX_OP_PARAMS; ++k) mix((uint32_t)t->op_params[k]);
        mix((uint64_t)(t->flags & kLayout));
    };
    auto ref = [&](const tts_tensor * x) {  // a source / view source
        if (!x) {
            mix(0x51);
            return;
        }
        const auto & e = tab[slot(x)];
        if (e.first) {
            mix(0x1000000ull + e.second);
            return;
        }
        mix(0x4C00000000ull | (uint64_t)(uint32_t)x->type << 8 | (uint64_t)(x->flags & kLayout));  // a leaf: no parameters
    };
    for (int i = 0; i < n; ++i) {
        const tts_tensor * t = nodes[i];
        kind(t);
        ref(t->view_src);
        for (int s = 0; s < TTS_MAX_SRC; ++s) ref(t->src[s]);
        if (t->op == TTS_OP_MUL_MAT && t->src[0] && t->src[0]->op == TTS_OP_NONE)  // a weight's shape
            for (int d = 0; d < 4; ++d) mix((uint64_t)t->src[0]->ne[d]);
    }
    return (h ^ (h2 * 0x94D049BB133111EBull)) | 1;
}

void copy_options(tts_hip_backend * d, const tts_hip_backend * s) {
    d->fusion = s->fusion;
    d->attn_split_minp = s->attn_split_minp;
    d->attn_ks = s->attn_ks;
    d->attn_pv_mp = s->attn_pv_mp;
    d->attn_pv8 = s->attn_pv8;
    d->attn_pv_uv16 = s->attn_pv_uv16;
    d->attn_fused_minp = s->attn_fused_minp;
    d->gemv_unique = s->gemv_unique;
    d->gemm_q8 = s->gemm_q8;
    d->bgemm_f32 = s->bgemm_f32;
    d->gemv_f32_wide = s->gemv_f32_wide;
    d->gemm_kr_nw = s->gemm_kr_nw;
    d->gemv_ks_tiles = s->gemv_ks_tiles;
    d->gemv_mf_prequant = s->gemv_mf_prequant;
    d->gemv_kr = s->gemv_kr;
    d->gemv_kr_loop = s->gemv_kr_loop;
    d->gemv_q80_pro = s->gemv_q80_pro;
    d->gemv_q80_slab = s->gemv_q80_slab;
    d->gemv_q80_rw = s->gemv_q80_rw;
    d->gemm_q8_staged = s->gemm_q8_staged;
    d->gemv_kr_ink = s->gemv_kr_ink;
    d->gemm_kr_ct2 = s->gemm_kr_ct2;
    d->gemm_kr_xcd = s->gemm_kr_xcd;
    d->gemm_kr_cp = s->gemm_kr_cp;
    d->gemm_kr_ink = s->gemm_kr_ink;
    d->gemv_nw_min = s->gemv_nw_min;
    d->gemv_mf_rsplit = s->gemv_mf_rsplit;
    d->profile_gemv = s->profile_gemv;
}

__global__ void k_ne_bytes(const uint4 * __restrict__ a, const uint4 * __restrict__ b, size_t n16, const uint8_t * __restrict__ ta,
                           const uint8_t * __restrict__ tb, size_t tail, int * flag) {
    bool ne = false;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 x = a[i], y = b[i];
        ne |= x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w;
    }
    if (blockIdx.x == 0)
        for (size_t i = threadIdx.x; i < tail; i += blockDim.x) ne |= ta[i] != tb[i];
    if (ne) *flag = 1;  // any mismatch: the range is not shared
}

// Read-only operands every member reads through member 0's copy: (member 0's, member k's, bytes)
// pairs whose bytes must be equal.
bool check_shared(Dev & d, tts_hip_backend * ex, const BatchCtx & bc, const std::vector<std::tuple<const void *, const void *, size_t>> & pairs) {
    std::vector<EqRec> todo;
    {
        std::lock_guard<std::mutex> lk(g_eq_mu);
        for (const auto & pr : pairs) {
            const char * a = (const char *)std::get<0>(pr);
            const char * b = (const char *)std::get<1>(pr);
            const size_t n = std::get<2>(pr);
            const EqRec * e = eq_known(a, b, n);
            if (e && !e->eq) return false;
            if (!e) todo.push_back(EqRec{a, b, n, true});
        }
    }
    if (todo.empty()) return true;
    if (co_debug()) fprintf(stderr, "coalesce: content check of %zu ranges\n", todo.size());
    if (d.d_flags_n < (int)todo.size()) {
        if (d.d_flags) hipFree(d.d_flags);
        d.d_flags_n = std::max((int)todo.size(), 1024);
        TTS_HIP_CHECK(hipMalloc((void **)&d.d_flags, sizeof(int) * d.d_flags_n));
    }
    TTS_HIP_CHECK(hipMemsetAsync(d.d_flags, 0, sizeof(int) * todo.size(), ex->stream));
    for (size_t i = 0; i < todo.size(); ++i) {
        const EqRec & r = todo[i];
        const bool al = ((uintptr_t)r.a % 16) == 0 && ((uintptr_t)r.b % 16) == 0;
        const size_t n16 = al ? r.n / 16 : 0, tail = r.n - n16 * 16;
        size_t g = (n16 + 255) / 256;
        g = g < 1 ? 1 : g > 1024 ? 1024 : g;
        hipLaunchKernelGGL(k_ne_bytes, dim3((unsigned)g), dim3(256), 0, ex->stream, (const uint4 *)r.a, (const uint4 *)r.b, n16,
                           (const uint8_t *)r.a + n16 * 16, (const uint8_t *)r.b + n16 * 16, tail, d.d_flags + i);
    }
    std::vector<int> flags(todo.size());
    TTS_HIP_CHECK(hipMemcpyAsync(flags.data(), d.d_flags, sizeof(int) * todo.size(), hipMemcpyDeviceToHost, ex->stream));
    TTS_HIP_CHECK(hipStreamSynchronize(ex->stream));
    bool all = true;
    std::lock_guard<std::mutex> lk(g_eq_mu);
    for (size_t i = 0; i < todo.size(); ++i) {
        todo[i].eq = flags[i] == 0;
        all &= todo[i].eq;
        g_eq[EqKey{todo[i].a, todo[i].b, todo[i].n}] = todo[i];
        cover_add(todo[i].a, todo[i].n);
        cover_add(todo[i].b, todo[i].n);
    }
    (void)bc;
    return all;
}

// Executor memory for the intermediates of member 0's graph: every compute buffer its non-leaf,
// non-view tensors lie in, up to the last byte the graph uses there, N copies side by side.
bool exec_layout(Dev & d, BatchCtx & bc, tts_tensor * const * nodes, int n) {
    struct Rng {
        const char * base;
        size_t size, used;
    };
    std::vector<Rng> rs;
    const Rng * last = nullptr;
    for (int i = 0; i < n; ++i) {
        const tts_tensor * t = nodes[i];
        if (!t->data || t->view_src || t->op == TTS_OP_NONE || (t->flags & TTS_FLAG_PERSIST)) continue;
        const char * p = (const char *)t->data;
        size_t nb = tts_row_size(t->type, t->ne[0]) * (size_t)(t->ne[1] * t->ne[2] * t->ne[3]);
        Rng * r = nullptr;
        if (last && p >= last->base && p < last->base + last->size) r = const_cast<Rng *>(last);
        for (size_t k = 0; !r && k < rs.size(); ++k)
            if (p >= rs[k].base && p < rs[k].base + rs[k].size) r = &rs[k];
        if (!r) {
            const char * b = nullptr;
            size_t sz = 0;
            if (!buffer_lookup(p, &b, &sz)) return false;  // not a backend buffer
            rs.push_back(Rng{b, sz, 0});
            r = &rs.back();
        }
        r->used = std::max(r->used, (size_t)(p - r->base) + nb);
        last = r;
    }
    size_t total = 0;
    for (const Rng & r : rs) total += bc.N * ((r.used + 255) & ~(size_t)255);
    if (total > d.mem_bytes) {
        if (d.mem) {
            TTS_HIP_CHECK(hipStreamSynchronize(d.exec->stream));  // an earlier coalesced step may still use it
            TTS_HIP_CHECK(hipFree(d.mem));
        }
        d.mem_bytes = total + total / 4;
        if (hipMalloc((void **)&d.mem, d.mem_bytes) != hipSuccess) {
            (void)hipGetLastError();
            d.mem = nullptr;
            d.mem_bytes = 0;
            return false;
        }
    }
    size_t off = 0;
    bc.cls.clear();
    for (const Rng & r : rs) {
        BatchCls c;
        c.b0 = r.base;
        c.size = r.used;
        c.win = d.mem + off;
        c.stride = (int64_t)((r.used + 255) & ~(size_t)255);
        off += bc.N * (size_t)c.stride;
        bc.cls.push_back(c);
    }
    std::sort(bc.cls.begin(), bc.cls.end(), [](const BatchCls & a, const BatchCls & b) { return a.b0 < b.b0; });
    return true;
}

// Run one group (the caller holds no lock).  Statuses are written into the requests.
void run_group(Dev & d, std::vector<Req *> & g) {
    std::lock_guard<std::mutex> xl(d.exec_mu);
    const auto tg0 = Clock::now();
    struct Acc {  // run_group's host time, whatever the exit
        Dev & d;
        Clock::time_point t0;
        ~Acc() { d.exec_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count(); }
    } acc{d, tg0};
    Req * r0 = g[0];
    std::vector<Req *> mem;
    for (Req * q : g)
        if (q->n == r0->n) mem.push_back(q);
    if (mem.size() < 2) {
        if (co_debug()) fprintf(stderr, "coalesce: group refused: node counts differ\n");
        d.refused++;
        return;  // statuses stay kCoalesceNotTaken: every member runs its own graph
    }
    BatchCtx bc;
    bc.N = (int)mem.size();
    bc.n_nodes = r0->n;
    // the group key: the graph kind and the member backends as a set (whichever member arrived last and
    // plans its graph as member 0, the verified structure and shared-data checks hold for the set)
    std::vector<uintptr_t> bes;
    for (Req * m : mem) {
        bc.mnodes.push_back(m->nodes);
        bc.mbe.push_back(m->be);
        bes.push_back((uintptr_t)m->be);
    }
    for (size_t k = 1; k < bes.size(); ++k)
        if (bes[k] < bes[bc.canon]) bc.canon = (int)k;
    std::sort(bes.begin(), bes.end());
    bc.key = r0->sig;
    for (uintptr_t b : bes) bc.key = (bc.key ^ (uint64_t)b) * 0x100000001B3ull;
    if (!d.exec) {
        d.exec = tts_hip_backend_init(r0->be->device);
        if (!d.exec) {
            d.refused++;
            return;
        }
    }
    const auto tl0 = Clock::now();
    const bool lay = exec_layout(d, bc, r0->nodes, r0->n);
    d.layout_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - tl0).count();
    if (!lay) {
        if (co_debug()) fprintf(stderr, "coalesce: group refused: executor layout\n");
        d.refused++;
        return;
    }
    uint64_t epoch;
    {
        std::lock_guard<std::mutex> lk(g_eq_mu);
        epoch = g_eq_epoch;
    }
    if (d.equal_epoch != epoch) {
        d.equal.clear();
        d.equal_epoch = epoch;
    }
    auto & uf = d.equal[r0->sig];
    auto root = [&](uintptr_t x) {
        auto it = uf.find(x);
        if (it == uf.end()) return x;
        while (it->second != x) {
            x = it->second;
            it = uf.find(x);
        }
        return x;
    };
    {
        const uintptr_t r = uf.count((uintptr_t)mem[0]->be) ? root((uintptr_t)mem[0]->be) : 0;
        bc.checked = r != 0;
        for (size_t k = 1; k < mem.size() && bc.checked; ++k) bc.checked = uf.count((uintptr_t)mem[k]->be) && root((uintptr_t)mem[k]->be) == r;
    }
    tts_hip_backend * ex = d.exec;
    copy_options(ex, r0->be);
    // the members' queued work (their input uploads) first.  A member whose stream has drained (its
    // synchronous tensor_set uploads have, the usual case) has nothing to order behind: no fence.
    static const bool fence_all = getenv("TTS_CO_FENCE_ALL") != nullptr;
    for (Req * m : mem) {
        if (!fence_all) {
            const hipError_t q = hipStreamQuery(m->be->stream);
            if (q == hipSuccess) continue;
            if (q != hipErrorNotReady) TTS_HIP_CHECK(q);
        }
        TTS_HIP_CHECK(hipEventRecord(m->be->co_ev, m->be->stream));
        TTS_HIP_CHECK(hipStreamWaitEvent(ex->stream, m->be->co_ev, 0));
    }
    ex->bat = &bc;
    const int st = graph_compute_launches(ex, r0->nodes, r0->n);
    ex->bat = nullptr;
    if (st == TTS_STATUS_UNSUPPORTED) {  // refused before any launch: each member runs its own graph
        if (co_debug()) fprintf(stderr, "coalesce: group of %d refused by the plan\n", bc.N);
        d.refused++;
        // a graph kind whose members cannot share a step (an item with no batched form, weights that differ):
        // later steps of that kind run at once instead of waiting for peers again
        if (!bc.differs) {
            std::lock_guard<std::mutex> lk(d.mu);
            d.no_form.insert(r0->sig);
        }
        return;
    }
    if (!bc.checked && st == 0) {  // every member verified against the canonical one: one class
        const uintptr_t c = (uintptr_t)mem[bc.canon]->be;
        if (!uf.count(c)) uf[c] = c;
        const uintptr_t rc = root(c);
        for (Req * m : mem) {
            const uintptr_t b = (uintptr_t)m->be;
            if (!uf.count(b)) uf[b] = b;
            const uintptr_t rb = root(b);
            if (rb != rc) uf[rb] = rc;
        }
    }
    TTS_HIP_CHECK(hipEventRecord(ex->co_ev, ex->stream));
    for (Req * m : mem) {
        TTS_HIP_CHECK(hipStreamWaitEvent(m->be->stream, ex->co_ev, 0));
        m->status = st;
    }
    d.launches++;
    d.member_steps += (int64_t)mem.size();
    if (bc.ragged) d.ragged++;
    if ((int64_t)mem.size() > d.max_group.load()) d.max_group.store((int64_t)mem.size());
}

}  // namespace

bool coalesce_check_shared(tts_hip_backend * ex, const std::vector<std::tuple<const void *, const void *, size_t>> & pairs) {
    return check_shared(g_dev[ex->device % kMaxDev], ex, *ex->bat, pairs);
}

// Rendezvous.  A request waits until every active backend (one that submitted a decode step within
// the last 50 ms and has not submitted anything else since) has a request pending, then every pending
// request runs, grouped by kind of graph: runners that started at different times, at different
// prompt lengths, share launches at their own KV lengths.  A backend that submits a prompt pass or a
// codec decode leaves the active set at once (nobody waits for it), an idle or finished one after
// 50 ms.  A request that has waited g_wait_us runs with whatever peers it has.  A group of one, or a
// group refused by run_group, returns kCoalesceNotTaken: each member then runs its own graph.
int coalesce_submit(tts_hip_backend * be, tts_tensor * const * nodes, int n) {
    if (!coalesce_enabled() || !be->co_member || be->device < 0 || be->device >= kMaxDev) return kCoalesceNotTaken;
    Dev & d = g_dev[be->device];
    if (!decode_like(nodes, n)) {
        // a prompt pass, a codec decode: this backend is not stepping now -- nobody waits for it
        std::lock_guard<std::mutex> lk(d.mu);
        if (d.seen.erase(be)) d.cv.notify_all();
        return kCoalesceNotTaken;
    }
    const auto t0 = Clock::now();
    const auto window = std::chrono::milliseconds(50);
    Req r;
    r.be = be;
    r.nodes = nodes;
    r.n = n;
    r.sig = signature(nodes, n);  // outside the lock, in the caller's thread: ~1200 nodes
    std::unique_lock<std::mutex> lk(d.mu);
    if (d.no_form.count(r.sig)) {  // known to have no coalesced form: no rendezvous, and not waited for
        if (d.seen.erase(be)) d.cv.notify_all();
        return kCoalesceNotTaken;
    }
    Act & me = d.seen[be];
    me.t = t0;
    me.tid = std::this_thread::get_id();
    r.count = ++me.count;
    d.pending.push_back(&r);
    d.cv.notify_all();
    const auto deadline = t0 + std::chrono::microseconds(g_wait_us.load());
    // A request leaves d.pending in the same critical section that marks it done: its owner (which
    // returns, destroying the stack Req, once it sees done) can only observe done after re-locking, by
    // which time no list holds it.  Callers re-read d.pending after every run, never an older snapshot.
    auto run = [&](std::vector<Req *> & g) {
        for (Req * q : g) q->taken = true;
        // the caller's own request first: its graph is the one planned (member 0)
        std::stable_partition(g.begin(), g.end(), [&](Req * q) { return q == &r; });
        if (g.size() >= 2) {
            lk.unlock();
            run_group(d, g);
            lk.lock();
        }
        for (Req * q : g) q->done = true;
        d.pending.erase(std::remove_if(d.pending.begin(), d.pending.end(), [](Req * q) { return q->done; }), d.pending.end());
        d.cv.notify_all();
    };
    while (!r.done) {
        if (r.taken) {
            d.cv.wait(lk);
            continue;
        }
        const auto now = Clock::now();
        int active = 0;
        const std::thread::id tid = std::this_thread::get_id();
        for (auto it = d.seen.begin(); it != d.seen.end();) {
            if (now - it->second.t > window && it->first != be) {
                it = d.seen.erase(it);
                continue;
            }
            // a backend last driven from this very thread cannot submit while this thread waits here (one
            // thread stepping several runners in turn): not waited for
            bool here = it->first == be;
            if (!here && it->second.tid == tid) {
                for (Req * q : d.pending) here |= q->be == it->first && !q->taken;
                if (!here) {
                    ++it;
                    continue;
                }
            }
            ++active, ++it;
        }
        std::vector<Req *> open;
        for (Req * q : d.pending)
            if (!q->taken) open.push_back(q);
        bool ran = false;
        if ((int)open.size() >= active) {
            // everyone is here: every pending step runs now, one launch per kind of graph (members at
            // different KV lengths share it)
            std::vector<uint64_t> sigs;
            for (Req * q : open)
                if (std::find(sigs.begin(), sigs.end(), q->sig) == sigs.end()) sigs.push_back(q->sig);
            for (uint64_t sg : sigs) {
                std::vector<Req *> g;  // from d.pending as it is now (an earlier group's members are gone)
                for (Req * q : d.pending)
                    if (!q->taken && q->sig == sg) g.push_back(q);
                if (!g.empty()) run(g);
            }
            ran = true;
        } else if (now >= deadline) {  // waited long enough: run with the peers that share this graph
            std::vector<Req *> g;
            for (Req * q : open)
                if (q->sig == r.sig) g.push_back(q);
            run(g);
            ran = true;
        }
        if (ran) continue;
        d.cv.wait_until(lk, deadline);
    }
    d.wait_us += std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0).count();
    if (r.status == kCoalesceNotTaken) d.alone++;
    return r.status;
}

void coalesce_backend_gone(const tts_hip_backend * be) {
    if (be->device < 0 || be->device >= kMaxDev) return;
    Dev & d = g_dev[be->device];
    {
        // a later backend may reuse this address with other weights: no verified class survives it
        std::lock_guard<std::mutex> xl(d.exec_mu);
        d.equal.clear();
    }
    std::lock_guard<std::mutex> lk(d.mu);
    d.seen.erase(be);
    d.cv.notify_all();
}

void coalesce_written(const void * p, size_t size) {
    if (!size) return;
    std::lock_guard<std::mutex> lk(g_eq_mu);
    if (g_eq.empty() || !cover_hits((const char *)p, size)) return;
    const char * a = (const char *)p;
    auto hits = [&](const char * x, size_t n) { return x < a + size && a < x + n; };
    for (auto it = g_eq.begin(); it != g_eq.end();) {
        if (hits(it->second.a, it->second.n) || hits(it->second.b, it->second.n)) it = g_eq.erase(it);
        else ++it;
    }
    g_eq_epoch++;
    g_eq_cover.clear();
    for (const auto & kv : g_eq) cover_add(kv.second.a, kv.second.n), cover_add(kv.second.b, kv.second.n);
}

}  // namespace tts

extern "C" int tts_hip_coalesce_stats(int device, int64_t * out, int n) {
    if (device < 0 || device >= tts::kMaxDev || !out) return TTS_STATUS_BAD_ARG;
    tts::Dev & d = tts::g_dev[device];
    std::lock_guard<std::mutex> lk(d.mu);
    const tts_hip_backend * ex = d.exec;
    const int64_t v[11] = {d.launches, d.member_steps, d.alone, d.refused, d.max_group, d.wait_us, d.ragged, d.exec_ns / 1000,
                           d.layout_ns / 1000, ex ? ex->cap_plan_ns / 1000 : 0, ex ? ex->co_prep_ns / 1000 : 0};
    int k = 0;
    for (; k < n && k < 11; ++k) out[k] = v[k];
    return k;
}

extern "C" void tts_hip_coalesce_set_wait(int us) { tts::g_wait_us.store(us < 0 ? 0 : us); }
