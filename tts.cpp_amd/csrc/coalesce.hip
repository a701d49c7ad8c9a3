// Step coalescer: TTS.cpp's one-prompt-per-runner serving shape run as batched decode steps.
//
// TTS.cpp's server scales by independent workers, each with its own runner, backend and model copy
// (/root/reference/examples/server/server.cpp:316-321,885-895), and each runner decodes one sequence
// per step graph (parler_tts_runner::decode, /root/reference/src/models/parler/model.cpp:648-693,
// model.h:158-172).  Unchanged, that is N streams of M = 1 GEMVs that each re-read every weight.
//
// Here every backend's graph_compute of a one-prompt decode step enters a per-device rendezvous.
// When the other recently active backends arrive with the same step graph (same ops, shapes and
// topology: the runners are at the same KV length), the step runs ONCE as member 0's plan with M = N
// columns (graph_exec.hip, be->bat):
//   - every buffer member 0's graph uses has a counterpart in each member at the same offset (the
//     runners build and allocate identical graphs); the members' physical buffers are mapped side by
//     side into one virtual window (HIP virtual memory: tts_hip_buffer_alloc maps every buffer), so
//     member k's tensor is window + k * stride + offset -- one uniform column / sequence stride, which
//     the GEMV, attention, norm and embedding kernels already take;
//   - operands read once for all members (weights, norm parameters, embedding tables) must hold equal
//     bytes in every member (each worker loads its own copy of the model): checked on the device once
//     and cached until a host write touches the range;
//   - the coalesced launches run on a hidden per-device backend's stream, after every member's stream
//     (their input uploads), and every member's stream waits for them, so each caller's
//     get_tensor_async sees its own logits (ggml_backend_sched_graph_compute_async is followed by an
//     immediate read, src/tts_model.cpp:25-36).
// Each member's results are the same sums in the same order as its own step: the kernels compute a
// column independently of the others (tests/test_coalesce_gpu.py checks the tokens bit-exact against
// each runner alone and against the CPU oracle).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "hip_internal.h"

namespace tts {
namespace {

using Clock = std::chrono::steady_clock;

// A buffer a graph touches, in order of first appearance (signature): graphs with equal signatures
// touch their buffers at equal offsets, buffer j of one graph standing for buffer j of the other.
struct BufSlot {
    const char * base = nullptr;
    size_t size = 0, map_size = 0;
    bool vmm = false;
};
struct Req {
    tts_hip_backend * be = nullptr;
    tts_tensor * const * nodes = nullptr;
    int n = 0;
    uint64_t sig = 0;
    std::vector<BufSlot> bufs;
    int64_t count = 0;  // the backend's coalescable submissions so far (its decode step number)
    bool taken = false, done = false;
    int status = kCoalesceNotTaken;
};
struct Act {
    Clock::time_point t;
    int64_t count = 0;
    std::thread::id tid;  // the thread of its last submission
};

struct Window {
    std::vector<const char *> bases;  // member buffers, member order
    size_t stride = 0;
    char * va = nullptr;
    int dev = 0;
};

constexpr int kMaxDev = 16;

struct Dev {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Req *> pending;
    std::unordered_map<const tts_hip_backend *, Act> seen;  // active backends: last coalescable submit
    std::mutex exec_mu;                   // one coalesced step at a time (guards everything below)
    tts_hip_backend * exec = nullptr;     // hidden backend: stream + scratch of the coalesced launches
    std::vector<Window> windows;
    int * d_flags = nullptr;              // content-check mismatch flags
    int d_flags_n = 0;
    // counters (tts_hip_coalesce_stats)
    std::atomic<int64_t> launches{0}, member_steps{0}, alone{0}, refused{0}, max_group{0}, wait_us{0};
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
std::unordered_map<uint64_t, uint64_t> g_eq_group;  // group key -> epoch its shared operands were all found equal
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

// Structure AND placement of a graph: ops, types, shapes, strides, parameters, layout flags, the node
// each source is (leaves and views by description), and where every tensor lies -- (buffer j, offset)
// with buffer j the j-th distinct buffer met, described by its size / mapping size / kind.  Two graphs
// with equal signatures are the same step over buffers that correspond slot by slot (bufs): what
// pairing member k's tensors with member 0's needs, computed by each runner's own thread.  Two
// independent 64-bit hashes, folded.
uint64_t signature(tts_tensor * const * nodes, int n, std::vector<BufSlot> & bufs) {
    std::unordered_map<const tts_tensor *, int> idx;
    idx.reserve((size_t)n * 2);
    for (int i = 0; i < n; ++i) idx[nodes[i]] = i;
    bufs.clear();
    uint64_t h = 0xCBF29CE484222325ull ^ (uint64_t)n, h2 = 0x84222325CBF29CE4ull + (uint64_t)n;
    auto mix = [&](uint64_t v) {
        h = (h ^ v) * 0x100000001B3ull;
        h2 = (h2 + v + 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
        h2 ^= h2 >> 31;
    };
    auto loc = [&](const void * p) {
        if (!p) {
            mix(0xD0);
            return;
        }
        const char * c = (const char *)p;
        for (size_t j = 0; j < bufs.size(); ++j)
            if (c >= bufs[j].base && c < bufs[j].base + bufs[j].size) {
                mix(0xB0 + j), mix((uint64_t)(c - bufs[j].base));
                return;
            }
        BufSlot sl;
        void * hd = nullptr;
        if (!buffer_lookup(p, &sl.base, &sl.size, &hd, &sl.map_size)) {
            mix(0xE1), mix((uint64_t)(uintptr_t)p);  // not a backend buffer: the very same address in every member
            return;
        }
        sl.vmm = hd != nullptr;
        bufs.push_back(sl);
        mix(0xB0 + bufs.size() - 1), mix(sl.size), mix(sl.map_size), mix(sl.vmm), mix((uint64_t)(c - sl.base));
    };
    constexpr int kLayout = TTS_FLAG_INPUT | TTS_FLAG_OUTPUT | TTS_FLAG_REPACKED | TTS_FLAG_TILED | TTS_FLAG_TILED_COPY;
    auto tensor = [&](const tts_tensor * t) {
        mix((uint64_t)t->op << 32 | (uint32_t)t->type);
        for (int d = 0; d < 4; ++d) mix((uint64_t)t->ne[d]), mix((uint64_t)t->nb[d]);
        for (int k = 0; k < TTS_MAX_OP_PARAMS; ++k) mix((uint32_t)t->op_params[k]);
        mix((uint64_t)(t->flags & kLayout));
        loc(t->data);
    };
    auto ref = [&](const tts_tensor * x, int depth, auto & self) -> void {  // a source / view source
        if (!x) {
            mix(0x51);
            return;
        }
        auto it = idx.find(x);
        if (it != idx.end()) {
            mix(0x1000000ull + it->second);
            return;
        }
        tensor(x);
        if (depth < 4) self(x->view_src, depth + 1, self);
    };
    for (int i = 0; i < n; ++i) {
        tensor(nodes[i]);
        ref(nodes[i]->view_src, 0, ref);
        for (int s = 0; s < TTS_MAX_SRC; ++s) ref(nodes[i]->src[s], 0, ref);
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
    d->gemm_kr_ink = s->gemm_kr_ink;
    d->gemv_nw_min = s->gemv_nw_min;
    d->gemv_mf_rsplit = s->gemv_mf_rsplit;
    d->profile_gemv = s->profile_gemv;
}

char * window_for(Dev & d, const std::vector<const char *> & bases, size_t stride) {
    for (const Window & w : d.windows)
        if (w.bases == bases && w.stride == stride) return w.va;
    int dev = 0;
    hipGetDevice(&dev);
    const size_t total = stride * bases.size();
    char * va = va_alloc(dev, total);
    if (!va) return nullptr;
    size_t mapped = 0;
    bool ok = true;
    for (; mapped < bases.size(); ++mapped) {
        void * h = nullptr;
        size_t ms = 0;
        ok = buffer_lookup(bases[mapped], nullptr, nullptr, &h, &ms) && h && ms == stride &&
             hipMemMap(va + mapped * stride, stride, 0, (hipMemGenericAllocationHandle_t)h, 0) == hipSuccess;
        if (!ok) break;
    }
    hipMemAccessDesc acc{};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = dev;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (ok) ok = hipMemSetAccess(va, total, &acc, 1) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        for (size_t u = 0; u < mapped; ++u) hipMemUnmap(va + u * stride, stride);
        va_free(dev, va, total);
        return nullptr;
    }
    d.windows.push_back(Window{bases, stride, va, dev});
    return va;
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

// Operands every member reads through member 0's copy: their bytes must be equal in each member.
bool check_shared(Dev & d, tts_hip_backend * ex, const BatchCtx & bc, const std::vector<std::pair<const void *, size_t>> & shared) {
    std::vector<EqRec> todo;
    {
        std::lock_guard<std::mutex> lk(g_eq_mu);
        // the same group as a step before, with no write into a checked range since: every pair still holds
        auto gk = g_eq_group.find(bc.key);
        if (gk != g_eq_group.end() && gk->second == g_eq_epoch) return true;
        for (const auto & s : shared) {
            if (!bc.stride(s.first)) continue;  // the same memory for every member
            for (int k = 1; k < bc.N; ++k) {
                const char * a = (const char *)s.first;
                const char * b = bc.reloc(a, k);
                const EqRec * e = eq_known(a, b, s.second);
                if (e && !e->eq) return false;
                if (!e) todo.push_back(EqRec{a, b, s.second, true});
            }
        }
    }
    if (todo.empty()) {
        std::lock_guard<std::mutex> lk(g_eq_mu);
        g_eq_group[bc.key] = g_eq_epoch;
        return true;
    }
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
    if (all) g_eq_group[bc.key] = g_eq_epoch;
    return all;
}

// Run one group (the caller holds no lock).  Statuses are written into the requests.
void run_group(Dev & d, std::vector<Req *> & g) {
    std::lock_guard<std::mutex> xl(d.exec_mu);
    Req * r0 = g[0];
    // equal signatures: member k's buffer slot j stands for member 0's slot j (same sizes, same offsets)
    std::vector<Req *> mem{r0};
    for (size_t k = 1; k < g.size(); ++k)
        if (g[k]->n == r0->n && g[k]->bufs.size() == r0->bufs.size()) mem.push_back(g[k]);
    if (mem.size() < 2) {
        d.refused++;
        return;  // statuses stay kCoalesceNotTaken: every member runs its own graph
    }
    BatchCtx bc;
    bc.N = (int)mem.size();
    bc.key = r0->sig;
    for (Req * m : mem)
        for (const BufSlot & sl : m->bufs) bc.key = (bc.key ^ (uint64_t)(uintptr_t)sl.base) * 0x100000001B3ull;
    for (size_t j = 0; j < r0->bufs.size(); ++j) {
        const BufSlot & s0 = r0->bufs[j];
        std::vector<const char *> mb(mem.size());
        bool same = true, vmm = s0.vmm;
        for (size_t k = 0; k < mem.size(); ++k) {
            const BufSlot & sk = mem[k]->bufs[j];
            mb[k] = sk.base;
            same &= sk.base == s0.base;
            vmm &= sk.vmm && sk.map_size == s0.map_size && sk.size == s0.size;
        }
        if (same) continue;  // one buffer read by every member (stride 0)
        if (!vmm) {
            d.refused++;
            return;
        }
        char * w = window_for(d, mb, s0.map_size);
        if (!w) {
            d.refused++;
            return;
        }
        BatchCls c;
        c.b0 = s0.base;
        c.size = s0.size;
        c.win = w;
        c.stride = (int64_t)s0.map_size;
        c.mb = std::move(mb);
        bc.cls.push_back(std::move(c));
    }
    std::sort(bc.cls.begin(), bc.cls.end(), [](const BatchCls & a, const BatchCls & b) { return a.b0 < b.b0; });
    if (!d.exec) {
        d.exec = tts_hip_backend_init(r0->be->device);
        if (!d.exec) {
            d.refused++;
            return;
        }
    }
    tts_hip_backend * ex = d.exec;
    copy_options(ex, r0->be);
    // the members' queued work (their input uploads) first
    for (Req * m : mem) {
        TTS_HIP_CHECK(hipEventRecord(m->be->co_ev, m->be->stream));
        TTS_HIP_CHECK(hipStreamWaitEvent(ex->stream, m->be->co_ev, 0));
    }
    ex->bat = &bc;
    const int st = graph_compute_launches(ex, r0->nodes, r0->n);
    ex->bat = nullptr;
    if (st == TTS_STATUS_UNSUPPORTED) {  // refused before any launch: each member runs its own graph
        d.refused++;
        return;
    }
    TTS_HIP_CHECK(hipEventRecord(ex->co_ev, ex->stream));
    for (Req * m : mem) {
        TTS_HIP_CHECK(hipStreamWaitEvent(m->be->stream, ex->co_ev, 0));
        m->status = st;
    }
    d.launches++;
    d.member_steps += (int64_t)mem.size();
    if ((int64_t)mem.size() > d.max_group.load()) d.max_group.store((int64_t)mem.size());
}

}  // namespace

bool coalesce_check_shared(tts_hip_backend * ex, const std::vector<std::pair<const void *, size_t>> & shared) {
    return check_shared(g_dev[ex->device % kMaxDev], ex, *ex->bat, shared);
}

// Rendezvous.  A request waits until every active backend (one that submitted a decode step within
// the last 50 ms) has a request pending, then the requests of the backends furthest behind (lowest
// step count) run, grouped by graph: runners started at different times fall into step (a backend
// one step ahead waits for the others' next step), and an idle or finished runner drops out of the
// active set.  A request that has waited g_wait_us runs with whatever peers it has.  A group of one,
// or a group refused by run_group, returns kCoalesceNotTaken: each member then runs its own graph.
int coalesce_submit(tts_hip_backend * be, tts_tensor * const * nodes, int n) {
    if (!coalesce_enabled() || !be->co_member || be->device >= kMaxDev || !decode_like(nodes, n)) return kCoalesceNotTaken;
    Dev & d = g_dev[be->device];
    const auto t0 = Clock::now();
    const auto window = std::chrono::milliseconds(50);
    Req r;
    r.be = be;
    r.nodes = nodes;
    r.n = n;
    r.sig = signature(nodes, n, r.bufs);  // outside the lock, in the caller's thread: ~700 nodes
    std::unique_lock<std::mutex> lk(d.mu);
    Act & me = d.seen[be];
    me.t = t0;
    me.tid = std::this_thread::get_id();
    r.count = ++me.count;
    d.pending.push_back(&r);
    d.cv.notify_all();
    const auto deadline = t0 + std::chrono::microseconds(g_wait_us.load());
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
            // everyone is here: the backends furthest behind run now, one launch per distinct graph
            int64_t cmin = INT64_MAX;
            for (Req * q : open) cmin = std::min(cmin, q->count);
            std::vector<uint64_t> sigs;
            for (Req * q : open)
                if (q->count == cmin && std::find(sigs.begin(), sigs.end(), q->sig) == sigs.end()) sigs.push_back(q->sig);
            for (uint64_t sg : sigs) {
                std::vector<Req *> g;
                for (Req * q : open)
                    if (q->count == cmin && q->sig == sg && !q->taken) g.push_back(q);
                run(g);
            }
            ran = true;
        } else if (now >= deadline) {  // waited long enough: run with the peers that share this graph
            std::vector<Req *> g;
            for (Req * q : open)
                if (q->sig == r.sig) g.push_back(q);
            run(g);
            ran = true;
        }
        if (ran) {
            d.pending.erase(std::remove_if(d.pending.begin(), d.pending.end(), [](Req * q) { return q->done; }), d.pending.end());
            d.cv.notify_all();
            continue;
        }
        d.cv.wait_until(lk, deadline);
    }
    d.wait_us += std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0).count();
    if (r.status == kCoalesceNotTaken) d.alone++;
    return r.status;
}

void coalesce_backend_gone(const tts_hip_backend * be) {
    if (be->device < 0 || be->device >= kMaxDev) return;
    Dev & d = g_dev[be->device];
    std::lock_guard<std::mutex> lk(d.mu);
    d.seen.erase(be);
    d.cv.notify_all();
}

void coalesce_forget(const void * base, size_t size) {
    const char * a = (const char *)base;
    for (Dev & d : g_dev) {
        std::lock_guard<std::mutex> xl(d.exec_mu);
        for (size_t i = 0; i < d.windows.size();) {
            Window & w = d.windows[i];
            bool hit = false;
            for (const char * b : w.bases) hit |= b == a;
            if (!hit) {
                ++i;
                continue;
            }
            hipDeviceSynchronize();  // a coalesced step may still read the window
            for (size_t k = 0; k < w.bases.size(); ++k) hipMemUnmap(w.va + k * w.stride, w.stride);
            va_free(w.dev, w.va, w.stride * w.bases.size());
            d.windows.erase(d.windows.begin() + i);
        }
    }
    coalesce_written(base, size);
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
    const int64_t v[6] = {d.launches, d.member_steps, d.alone, d.refused, d.max_group, d.wait_us};
    int k = 0;
    for (; k < n && k < 6; ++k) out[k] = v[k];
    return k;
}

extern "C" void tts_hip_coalesce_set_wait(int us) { tts::g_wait_us.store(us < 0 ? 0 : us); }
