// graph_compute: plans and executes a ggml-style node list on one HIP stream
// (ggml_backend_i::graph_compute underneath ggml_backend_sched_graph_compute_async,
// /root/reference/src/models/parler/model.cpp:645).
//
// Planning pass (per call): consumer counts per tensor, then pattern fusion, each fused kernel
// reproducing the unfused ops bit-for-bit (see k_fused.hip / k_gemv.hip):
//   LN   : NORM -> MUL(w) -> ADD(b); folded into the prologue of the Q4_K GEMV that reads it
//   GEMV : adjacent MUL_MATs sharing src1 (q/k/v) in one launch; K / V outputs written straight
//          into the KV-cache views their CPY nodes target (parler_build_kv_store); adjacent
//          ADD(residual) or GELU consumer folded into the epilogue
//   HEADS: MUL_MAT_i chained by CONCAT(dim 1) (parler_build_head_outputs) -> one launch writing
//          each head's rows at its concat offset
//   ATTN : cont(K)/cont(q) -> MUL_MAT -> SOFT_MAX -> MUL_MAT(V) -> PERMUTE -> CONT
// A pattern fuses only when every intermediate tensor has a single consumer inside the group
// and the fused output does not overlap an input it reads (the graph arrives already
// allocated, so aliasing is checked on the real addresses).
#include <algorithm>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <vector>

#include <array>

#include "hip_internal.h"
#include <chrono>

using namespace tts;

namespace tts {
void launch_kv_prefetch(tts_hip_backend * be, hipStream_t st, const TD & t, int pdim, int blocks);
void launch_gemv_q4K_xattn(tts_hip_backend * be, const GemvJob & j, const XAttnArgs & a);
void launch_attn_decode(tts_hip_backend * be, const TD & q, const TD & k, const TD & v, const float * mask, float scale,
                        float * out, int hd, int P, int H, int n, int B, float * out2, int64_t obs = -1, int64_t mbs = 0,
                        const int64_t * koff = nullptr, const int64_t * voff = nullptr, const int64_t * moff = nullptr,
                        const int * pseq = nullptr);
void launch_layernorm(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * x, const float * w, const float * b,
                      float eps, bool rms);
}  // namespace tts

namespace {

size_t tbytes(const tts_tensor * t) {
    size_t n = tts_type_size(t->type);
    const int64_t bs = tts_blck_size(t->type);
    if (bs == 1) {
        for (int i = 0; i < 4; ++i) n += (size_t)(t->ne[i] - 1) * t->nb[i];
    } else {
        n = (size_t)(t->ne[0] / bs) * t->nb[0];
        for (int i = 1; i < 4; ++i) n += (size_t)(t->ne[i] - 1) * t->nb[i];
    }
    return n;
}

bool overlap(const tts_tensor * a, const tts_tensor * b) {
    if (!a || !b || !a->data || !b->data) return false;
    const char * a0 = (const char *)a->data;
    const char * b0 = (const char *)b->data;
    return a0 < b0 + tbytes(b) && b0 < a0 + tbytes(a);
}

bool is_view(int op) {
    return op == TTS_OP_NONE || op == TTS_OP_VIEW || op == TTS_OP_RESHAPE || op == TTS_OP_PERMUTE || op == TTS_OP_TRANSPOSE;
}

bool contiguous(const tts_tensor * t) {
    const size_t es = tts_type_size(t->type);
    return t->nb[0] == es && t->nb[1] == t->nb[0] * (size_t)(t->ne[0] / tts_blck_size(t->type)) &&
           t->nb[2] == t->nb[1] * (size_t)t->ne[1] && t->nb[3] == t->nb[2] * (size_t)t->ne[2];
}

// memory that outlives the graph: a leaf (model / input tensor) or a PERSIST tensor, through views
bool persistent_mem(const tts_tensor * t) {
    for (int hop = 0; t && hop < 8; ++hop) {
        if (t->op == TTS_OP_NONE || (t->flags & TTS_FLAG_PERSIST)) return true;
        if (!is_view(t->op)) return false;
        t = t->view_src ? t->view_src : t->src[0];
    }
    return false;
}

bool is_1d_f32(const tts_tensor * t, int64_t n) {
    return t->type == TTS_TYPE_F32 && t->ne[0] == n && t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1 && t->nb[0] == 4;
}

float opf(const tts_tensor * t, int i) {
    float f;
    memcpy(&f, &t->op_params[i], 4);
    return f;
}

// MUL_MAT with a 2-D weight matrix and evenly strided f32 columns: the decode GEMV.
static int64_t nel(const tts_tensor * t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }

bool is_gemv(const tts_tensor * n) {
    const tts_tensor * a = n->src[0];
    const tts_tensor * b = n->src[1];
    if (a->ne[2] != 1 || a->ne[3] != 1) return false;
    if (b->type != TTS_TYPE_F32 || b->nb[0] != 4) return false;
    if (b->ne[2] * b->ne[3] != 1 && !(b->nb[2] == b->nb[1] * (size_t)b->ne[1] && b->nb[3] == b->nb[2] * (size_t)b->ne[2]))
        return false;
    if (n->nb[0] != 4 || (n->ne[2] * n->ne[3] != 1 && !(n->nb[2] == n->nb[1] * (size_t)n->ne[1] && n->nb[3] == n->nb[2] * (size_t)n->ne[2])))
        return false;
    if (a->nb[0] != tts_type_size(a->type)) return false;
    // float weights against many columns (conv_1d's im2col GEMM) belong to the matrix cores
    if ((a->type == TTS_TYPE_F16 || a->type == TTS_TYPE_F32) && b->ne[1] * b->ne[2] * b->ne[3] > 64) return false;
    // F16 weights against more than 8 columns (Kokoro's F16 ALBERT / duration projections): the f64
    // matrix-core GEMM (launch_gemm_f16) instead of one GEMV launch per 8 columns
    if (a->type == TTS_TYPE_F16 && b->ne[1] * b->ne[2] * b->ne[3] > 8 && a->ne[0] % 8 == 0 && (b->nb[1] % 16) == 0 &&
        ((uintptr_t)b->data % 16) == 0 && (a->nb[1] % 16) == 0)
        return false;
    switch (a->type) {
        case TTS_TYPE_Q4_K: return a->ne[0] % 256 == 0;
        case TTS_TYPE_Q8_0: return a->ne[0] % 32 == 0;
        case TTS_TYPE_F32:
        case TTS_TYPE_F16: return a->ne[0] % 4 == 0 && (b->nb[1] % 16) == 0 && ((uintptr_t)b->data % 16) == 0;
        default: return false;
    }
}

struct GemvTarget {
    float * y;
    int64_t ycs, yrs;
    int32_t rg = 0, nrep = 1;  // row groups of rg rows, rgs apart; nrep copies, rep apart (floats)
    int64_t rgs = 0, rep = 0;
    const tts_tensor * yt = nullptr;  // the graph tensor y lies in (null: backend scratch); coalesced steps
};

struct Item {
    enum Kind { GEMV, ATTN, LN, LSTM, SNAKE, EMBED, CONV, ADAIN, MCPY, RINT, NODE, COPY } kind;
    // COPY: a grouped product hoisted into an earlier launch wrote its output to backend scratch;
    // at the product's own position it is copied to its tensor (cp_src -> cp_dst, cp_bytes)
    const void * cp_src = nullptr;
    void * cp_dst = nullptr;
    size_t cp_bytes = 0;
    // NODE: a node run with a rewritten source (TTS_FUSE_CONTREAD)
    tts_tensor node{};
    // MCPY: the ROPE node producing the copies' source, applied on the way (x = the rope's source)
    const tts_tensor * rope = nullptr;
    // GEMV
    std::vector<const tts_tensor *> mms;
    std::vector<GemvTarget> tgt;
    int epi = EPI_NONE;
    const tts_tensor * res = nullptr;
    // GEMV with a LayerNorm prologue (Q4_K): src1 = lndst = norm(lnx) * lnw (+ lnb)
    bool ln = false;
    const tts_tensor *lnx = nullptr, *lnw = nullptr, *lnb = nullptr, *lndst = nullptr;
    float lneps = 0.f;
    bool lnrms = false;
    bool x_shadow = false;  // src1 = the preceding attention output: read its private copy
    const tts_tensor * snake_one = nullptr;  // SNAKE: b == nullptr, recip = snake_one[0] / alpha in the kernel
    const tts_tensor * snake_mask = nullptr;  // SNAKE: x = x * mask[t] first (the MUL node of a batched DAC decode's gap mask)
    // EMBED, gather form (a codec quantizer's input, general_neural_audio_codec.cpp:166-172):
    // dst [T, C] = CONT(TRANSPOSE(GET_ROWS(w [C, rows], CONT(view of I32 codes)))) in one pass
    bool gather_t = false;
    const tts_tensor * gt_codes = nullptr;  // the codes view (t-th id at data + t * nb[1])
    const tts_tensor * xsrc = nullptr;  // src1 is a skipped CONT of this contiguous tensor (same bytes): read its data
    bool shadow = false;    // ATTN: also write the private copy (be->shadow)
    int xattn = -1;         // GEMV: index of the short-context ATTN item whose query it produces (one launch)
    bool fused = false;     // ATTN: launched by the GEMV item that produces its query
    // ATTN
    const tts_tensor *q = nullptr, *k = nullptr, *v = nullptr, *mask = nullptr, *out = nullptr;
    float scale = 1.f;
    // LN
    const tts_tensor *x = nullptr, *w = nullptr, *b = nullptr, *dst = nullptr;
    float eps = 0.f;
    bool rms = false;
    // EMBED: GET_ROWS terms summed in order into dst
    std::vector<const tts_tensor *> terms;
    // LSTM: bit 1 = run recurrence step `ls` (and `ls2` when lpair: two independent chains in one
    // launch), bit 2 = write the chain output(s) `lfinal` (`lfinal2`) from `lhist` (`lhist2`), bit 4 =
    // stash a paired chain's four input projections (lstash_src[g] -> lstash_dst[g], lstash_bytes)
    int lkind = 0;
    LstmStepArgs ls{}, ls2{};
    bool lpair = false;
    const tts_tensor *lfinal = nullptr, *lfinal2 = nullptr;
    const float *lhist = nullptr, *lhist2 = nullptr;
    int64_t lHd = 0, lT = 0;
    const void * lstash_src[4] = {};
    void * lstash_dst[4] = {};
    size_t lstash_bytes = 0;
    // CONV: implicit-GEMM conv_1d with its bias / residual ADDs
    Conv1dArgs conv{};
    // ADAIN: per-channel norm + affine (+ snake)
    AdainArgs adain{};
    // MCPY: src (x) copied into every view in `terms`
    // RINT: dst = repeat_interleave of x along dim 1 by `rint` (rint_cpy: into the stand-in `node`)
    bool rint_cpy = false;
    int rint = 1;
};

// Open-addressing map keyed by tensor address, for the planner's per-tensor tables (a 20k-node
// Kokoro graph spends more time in std::unordered_map's node allocations than in the planning).
// The unordered_map subset the planner uses: operator[] (inserting a default), find() returning an
// entry pointer with .first / .second or end() == nullptr, count().
// A tensor's consumer list: almost always one or two nodes, kept inline.
struct SmallIdx {
    int inl[3];
    std::vector<int> more;
    int n = 0;
    void push_back(int v) {
        if (n < 3) inl[n] = v;
        else more.push_back(v);
        ++n;
    }
    size_t size() const { return (size_t)n; }
    int operator[](size_t i) const { return i < 3 ? inl[i] : more[i - 3]; }
    struct iter {
        const SmallIdx * s;
        size_t i;
        int operator*() const { return (*s)[i]; }
        iter & operator++() {
            ++i;
            return *this;
        }
        bool operator!=(const iter & o) const { return i != o.i; }
        bool operator==(const iter & o) const { return i == o.i; }
        using iterator_category = std::input_iterator_tag;
        using value_type = int;
        using difference_type = std::ptrdiff_t;
        using pointer = const int *;
        using reference = int;
    };
    iter begin() const { return {this, 0}; }
    iter end() const { return {this, (size_t)n}; }
};

template <typename V>
struct PtrMap {
    struct Entry {
        const tts_tensor * first;
        V second;
    };
    std::vector<Entry> entries;
    std::vector<int32_t> slots;  // -1 empty, else index into entries
    size_t mask_ = 0;
    void reserve(size_t n) {
        size_t cap = 64;
        while (cap < 2 * n) cap <<= 1;
        slots.assign(cap, -1);
        mask_ = cap - 1;
        entries.clear();
        entries.reserve(n);
    }
    size_t slot(const tts_tensor * k) const {
        uint64_t h = (uint64_t)(uintptr_t)k * 0x9E3779B97F4A7C15ull;
        size_t i = (size_t)(h >> 32) & mask_;
        while (slots[i] >= 0 && entries[slots[i]].first != k) i = (i + 1) & mask_;
        return i;
    }
    V & operator[](const tts_tensor * k) {
        if (slots.empty()) reserve(64);
        size_t i = slot(k);
        if (slots[i] < 0) {
            if (2 * (entries.size() + 1) > slots.size()) {  // grow: rehash every entry
                std::vector<Entry> old;
                old.swap(entries);
                reserve(old.size() * 2 + 1);
                for (auto & e : old) {
                    const size_t j = slot(e.first);
                    slots[j] = (int32_t)entries.size();
                    entries.push_back(std::move(e));
                }
                i = slot(k);
            }
            slots[i] = (int32_t)entries.size();
            entries.push_back(Entry{k, V{}});
        }
        return entries[slots[i]].second;
    }
    Entry * find(const tts_tensor * k) {
        if (slots.empty()) return nullptr;
        const size_t i = slot(k);
        return slots[i] < 0 ? nullptr : &entries[slots[i]];
    }
    Entry * end() { return nullptr; }
    size_t count(const tts_tensor * k) { return find(k) ? 1 : 0; }
};

struct Planner {
    tts_tensor * const * nodes;
    int n;
    PtrMap<int> index;
    PtrMap<SmallIdx> consumers;
    // distinct consuming nodes of a tensor (a node listing it twice counts once): the size of its
    // consumer list, so one map serves both
    struct Uses {
        PtrMap<SmallIdx> * c;
        int operator[](const tts_tensor * t) const {
            auto * e = c->find(t);
            return e ? (int)e->second.size() : 0;
        }
    } uses{&consumers};
    std::vector<int> act;  // -1 skip, 0 run node, k>0 run items[k-1]
    std::vector<Item> items;
    std::deque<tts_tensor> derived;  // strided stand-ins for folded CONT nodes (stable addresses)
    int mask = 0xFF;
    bool q80pro = true;  // Q8_0 GEMVs of <= 8 columns take LN prologues too (TTS_HIP_OPT_GEMV_Q80_PRO)
    float * lstm_buf = nullptr;  // backend scratch for fused LSTM chains (hidden history + cell)
    size_t vec_cap = 0;          // floats of the backend's vector scratch (fused AdaIN staging)
    float * conv_stage = nullptr;  // backend scratch for fused conv outputs that cannot stage in their im2col buffer
    size_t conv_stage_cap = 0;
    char * hoist_buf = nullptr;  // backend scratch for hoisted products whose own memory is still in use (try_gemv)
    size_t hoist_cap = 0, hoist_used = 0;
    int hoist_live = -1;  // the last node position whose COPY item still reads the hoist buffer
    size_t lstm_cap = 0, lstm_used = 0;

    const tts_tensor * sole_consumer(const tts_tensor * t) {
        auto it = consumers.find(t);
        if (it == consumers.end() || it->second.size() != 1 || uses[t] != 1) return nullptr;
        return nodes[it->second[0]];
    }
    // next non-view node index after i (views allocate nothing)
    int next_real(int i) {
        for (int j = i + 1; j < n; ++j)
            if (!is_view(nodes[j]->op)) return j;
        return -1;
    }

    void build(tts_tensor * const * nodes_, int n_) {
        const auto t_build0 = std::chrono::steady_clock::now();
        nodes = nodes_;
        n = n_;
        act.assign(n, 0);
        index.reserve((size_t)n);
        consumers.reserve((size_t)n * 2);
        for (int i = 0; i < n; ++i) {
            index[nodes[i]] = i;
            for (int s = 0; s < TTS_MAX_SRC; ++s) {
                const tts_tensor * x = nodes[i]->src[s];
                if (!x) continue;
                // a node listing the same source twice counts once
                bool dup = false;
                for (int s2 = 0; s2 < s; ++s2) dup |= nodes[i]->src[s2] == x;
                if (dup) continue;
                consumers[x].push_back(i);
            }
        }
        // TTS_PLAN_TIMING=1: milliseconds per planner pass on stderr (host-cost study)
        static const bool timing = getenv("TTS_PLAN_TIMING") != nullptr;
        auto t_last = t_build0;
        char tbuf[512];
        int tlen = 0;
        auto tmark = [&](const char * what) {
            if (!timing) return;
            const auto now = std::chrono::steady_clock::now();
            tlen += snprintf(tbuf + tlen, sizeof(tbuf) - (size_t)tlen, " %s %.3f", what, std::chrono::duration<double, std::milli>(now - t_last).count());
            t_last = now;
        };
        tmark("index");
        if (mask & TTS_FUSE_LSTM) try_lstm();
        tmark("lstm");
        if (mask & TTS_FUSE_MCPY)  // roots first: a concat chain is claimed whole by its last CONCAT
            for (int i = n - 1; i >= 0; --i)
                if (act[i] == 0 && nodes[i]->op == TTS_OP_CONCAT) try_rint(i);
        tmark("rint");
        if (mask & TTS_FUSE_EMBED)  // roots first: a chain is claimed whole by its last ADD
            for (int i = n - 1; i >= 0; --i)
                if (act[i] == 0 && nodes[i]->op == TTS_OP_ADD) try_embed(i);
        tmark("embed");
        for (int i = 0; i < n; ++i) {
            if (act[i] != 0) continue;
            const tts_tensor * t = nodes[i];
            switch (t->op) {
                case TTS_OP_NORM:
                    if ((mask & TTS_FUSE_ADAIN) && try_adain(i)) break;
                    if (mask & TTS_FUSE_LN) try_ln(i);
                    break;
                case TTS_OP_RMS_NORM: if (mask & TTS_FUSE_LN) try_ln(i); break;
                case TTS_OP_SOFT_MAX: if (mask & TTS_FUSE_ATTN) try_attn(i); break;
                case TTS_OP_ADD: if (mask & TTS_FUSE_SNAKE) try_snake(i); break;
                case TTS_OP_IM2COL: if (mask & TTS_FUSE_CONV) try_conv(i); break;
                case TTS_OP_CPY: if (mask & TTS_FUSE_MCPY) try_mcpy(i); break;
                case TTS_OP_CONT: if (mask & TTS_FUSE_EMBED) try_gather_t(i); break;
                case TTS_OP_MUL_MAT:
                    if (!((mask & TTS_FUSE_HEADS) && try_heads(i)) && (mask & (TTS_FUSE_GROUP | TTS_FUSE_KV | TTS_FUSE_EPI))) try_gemv(i);
                    break;
                default: break;
            }
        }
        tmark("patterns");
        if (mask & TTS_FUSE_CONTREAD) skip_cont_reads();
        if (mask & TTS_FUSE_LN) fuse_ln_into_gemv();
        link_attn_shadow();
        if (mask & TTS_FUSE_XATTN) fuse_xattn();
        tmark("post");
        if (timing) fprintf(stderr, "plan %d nodes ms:%s\n", n, tbuf);
    }

    // attention output -> [views] -> Q4_K GEMV: the attention kernel also writes a private copy
    // that the GEMV reads, so the GEMV's outputs may land on the attention output's memory
    // (arena reuse) without a staging copy.
    void link_attn_shadow() {
        for (int i = 0; i < n; ++i) {
            const int a = act[i];
            if (a <= 0 || items[a - 1].kind != Item::ATTN) continue;
            const int nx = next_real(i);
            if (nx < 0 || act[nx] <= 0) continue;
            Item & A = items[a - 1];
            Item & G = items[act[nx] - 1];
            if (G.kind != Item::GEMV || G.ln || G.mms[0]->src[0]->type != TTS_TYPE_Q4_K) continue;
            const tts_tensor * x = G.mms[0]->src[1];
            if (x->data != A.out->data || !contiguous(x) || tbytes(x) != tbytes(A.out)) continue;
            A.shadow = G.x_shadow = true;
        }
    }

    // Short-context attention (P <= 64, hd 64, one query: Parler's cross-attention over the T5
    // encoding) whose query is the output of a single-matrix Q4_K GEMV item, through reshape /
    // permute views only: both run as one k_gemv_q4K_xattn launch at the GEMV's position.  Nothing
    // may run between the two (the attention output is written early).
    void fuse_xattn() {
        for (size_t ai = 0; ai < items.size(); ++ai) {
            Item & A = items[ai];
            if (A.kind != Item::ATTN || A.k->ne[1] > 64 || A.q->ne[0] != 64 || A.q->ne[1] != 1) continue;
            const tts_tensor * Q = A.q;
            const tts_tensor * t = Q;
            int hops = 0;
            while (t && is_view(t->op) && t->src[0] && hops < 4) {
                if (uses[t->src[0]] != 1) break;
                t = t->src[0];
                ++hops;
            }
            if (!t || t->op != TTS_OP_MUL_MAT || uses[t] != 1) continue;
            const int gi = act[index[t]];
            if (gi <= 0) continue;
            Item & G = items[gi - 1];
            if (G.kind != Item::GEMV || G.mms.size() != 1 || G.mms[0] != t || G.epi != EPI_NONE || G.res || G.xattn >= 0) continue;
            const tts_tensor * W = t->src[0];
            const int64_t H = Q->ne[2], B = Q->ne[3];
            if (W->type != TTS_TYPE_Q4_K || (W->flags & TTS_FLAG_TILED) || W->ne[0] > 1024 || W->ne[1] != 64 * H ||
                t->ne[1] * t->ne[2] * t->ne[3] != B) continue;
            if (G.tgt[0].y != (float *)t->data || G.tgt[0].ycs != W->ne[1] || G.tgt[0].yrs != 1) continue;
            if (Q->data != t->data || Q->nb[0] != 4 || Q->nb[2] != 256 || (int64_t)Q->nb[3] != 4 * W->ne[1]) continue;
            if (A.k->ne[2] != H || A.v->ne[2] != H || B % A.k->ne[3] || B % A.v->ne[3]) continue;  // K/V may be shared by all prompts
            if (A.mask && A.mask->ne[0] != A.k->ne[1]) continue;
            const int g_node = index[t], o_node = index[A.out];
            bool clear = g_node < o_node;
            for (int i = g_node + 1; clear && i < o_node; ++i)
                if (act[i] > 0 || (act[i] == 0 && !is_view(nodes[i]->op))) clear = false;
            if (!clear) continue;
            G.xattn = (int)ai;
            A.fused = true;
        }
    }

    // CONT C of a contiguous tensor of the same type (through views) whose only reader is the next
    // node R (an elementwise op or rope, still launched on its own): R reads C's source instead, and
    // the copy is skipped.  R's output must not overlap that source (the copy would have separated
    // them) unless it coincides with it exactly.
    void skip_cont_reads() {
        for (int i = 0; i < n; ++i) {
            const tts_tensor * C = nodes[i];
            if (act[i] != 0 || C->op != TTS_OP_CONT || !C->src[0]) continue;
            const tts_tensor * s = C->src[0];
            if (s->type != C->type || !contiguous(s) || !contiguous(C) || uses[C] != 1) continue;
            // the reader indexes its source by its own shape: a reshaping cont_Nd is not skippable
            if (s->ne[0] != C->ne[0] || s->ne[1] != C->ne[1] || s->ne[2] != C->ne[2] || s->ne[3] != C->ne[3]) continue;
            if (C->flags & (TTS_FLAG_OUTPUT | TTS_FLAG_PERSIST)) continue;  // read after the graph: must be written
            const int r = next_real(i);
            if (r < 0 || act[r] != 0) continue;
            const tts_tensor * R = nodes[r];
            if (R->src[0] != C || (R->op != TTS_OP_ROPE && R->op != TTS_OP_UNARY)) continue;
            bool other = false;
            for (int si = 1; si < TTS_MAX_SRC; ++si) other |= R->src[si] == C;
            // in place is fine when R's output coincides exactly with the source (rope and unary ops read
            // every element they write before writing it, in the same thread)
            bool same = R->data == s->data && R->type == s->type;
            for (int d = 0; d < 4 && same; ++d) same = R->ne[d] == s->ne[d] && R->nb[d] == s->nb[d];
            if (other || (overlap(R, s) && !same)) continue;
            Item it;
            it.kind = Item::NODE;
            it.node = *R;
            it.node.src[0] = const_cast<tts_tensor *>(s);
            act[i] = -1;
            act[r] = add_item(std::move(it));
        }
    }

    // An LN item directly followed by the Q4_K GEMV item (or Q8_0 GEMV item of <= 8 columns) that
    // reads its output becomes that GEMV's prologue (every workgroup normalizes + quantizes the
    // activation itself; workgroup 0 still writes the LN output tensor).
    void fuse_ln_into_gemv() {
        for (int i = 0; i < n; ++i) {
            const int a = act[i];
            if (a <= 0 || items[a - 1].kind != Item::LN) continue;
            const int nx = next_real(i);
            if (nx < 0 || act[nx] <= 0) continue;
            Item & L = items[a - 1];
            Item & G = items[act[nx] - 1];
            if (G.kind != Item::GEMV || G.ln || G.mms[0]->src[1] != L.dst) continue;
            const int wt = G.mms[0]->src[0]->type;
            const tts_tensor * B = G.mms[0]->src[1];
            if (wt != TTS_TYPE_Q4_K && !(wt == TTS_TYPE_Q8_0 && q80pro && B->ne[1] * B->ne[2] * B->ne[3] <= 8)) continue;
            const int64_t K = L.dst->ne[0];
            if (K % 256 || K > 4096) continue;
            if (((uintptr_t)L.w->data & 15) || (L.b && ((uintptr_t)L.b->data & 15)) || (L.dst->nb[1] & 15)) continue;
            G.ln = true;
            G.lnx = L.x;
            G.lnw = L.w;
            G.lnb = L.b;
            G.lndst = L.dst;
            G.lneps = L.eps;
            G.lnrms = L.rms;
            act[i] = -1;
        }
    }

    int add_item(Item && it) {
        items.push_back(std::move(it));
        return (int)items.size();
    }

    void try_ln(int i) {
        const tts_tensor * N = nodes[i];
        const tts_tensor * x = N->src[0];
        if (x->type != TTS_TYPE_F32 || x->nb[0] != 4 || x->ne[0] > 8192) return;
        const int64_t ne0 = x->ne[0];
        const tts_tensor * M = sole_consumer(N);
        if (!M || M->op != TTS_OP_MUL || M->src[0] != N || !is_1d_f32(M->src[1], ne0)) return;
        if (next_real(i) != index[M]) return;
        const tts_tensor * A = nullptr;
        if (N->op == TTS_OP_NORM) {
            A = sole_consumer(M);
            if (!A || A->op != TTS_OP_ADD || A->src[0] != M || !is_1d_f32(A->src[1], ne0)) return;
            if (next_real(index[M]) != index[A]) return;
        } else {
            A = M;
        }
        if (!contiguous(A) || A->type != TTS_TYPE_F32 || !contiguous(x)) return;
        if (overlap(A, x) && A->data != x->data) return;  // exact in-place is safe (per-row read-then-write)
        Item it;
        it.kind = Item::LN;
        it.x = x;
        it.w = M->src[1];
        it.b = N->op == TTS_OP_NORM ? A->src[1] : nullptr;
        it.dst = A;
        it.eps = opf(N, 0);
        it.rms = N->op == TTS_OP_RMS_NORM;
        act[i] = -1;
        if (A != M) act[index[M]] = -1;
        act[index[A]] = add_item(std::move(it));
    }

    // KV-store fusion: the GEMV output goes straight into the CPY destination (decode, 1 token).
    // mm -> RESHAPE c [hd, nkv, n, B] -> CPY into each of 2-4 repeat-interleaved views of the cache
    // (Orpheus' V store, orpheus/model.cpp:194-228): row kvh * hd + d goes to every copy
    // (c = the product itself or a RESHAPE of it; the copies may view another shape of the same
    // elements -- the reference copies Orpheus' [H, n] V product into [hd, nkv, n] cache views)
    bool repeat_target(const tts_tensor * mm, const tts_tensor * c, int64_t N, GemvTarget & t, std::vector<int> & skips) {
        auto ci = consumers.find(c);
        if (ci == consumers.end() || ci->second.size() < 2 || ci->second.size() > 4 || uses[c] != (int)ci->second.size()) return false;
        std::vector<int> idx(ci->second.begin(), ci->second.end());
        std::sort(idx.begin(), idx.end());
        const tts_tensor * D0 = nodes[idx[0]];
        if (D0->ne[0] * D0->ne[1] * D0->ne[2] * D0->ne[3] != mm->ne[0] * mm->ne[1] * mm->ne[2] * mm->ne[3]) return false;
        int64_t rep = 0;
        for (size_t a = 0; a < idx.size(); ++a) {
            const tts_tensor * D = nodes[idx[a]];
            if (D->op != TTS_OP_CPY || D->src[0] != c || act[idx[a]] != 0 || D->type != TTS_TYPE_F32 || D->nb[0] != 4) return false;
            for (int k = 0; k < 4; ++k)
                if (D->ne[k] != D0->ne[k] || D->nb[k] != D0->nb[k]) return false;
            const int64_t d = ((const char *)D->data - (const char *)D0->data);
            if (d % 4) return false;
            if (a == 1) rep = d / 4;
            if (a > 0 && d / 4 != rep * (int64_t)a) return false;
        }
        // rows: ne0 x ne1 = N; columns: the n x B of the product, one of them 1
        // the copies' runs of one row group are disjoint and fit inside the group stride
        if (D0->ne[0] * D0->ne[1] != N || rep < D0->ne[0] || rep * (int64_t)(idx.size() - 1) + D0->ne[0] > (int64_t)(D0->nb[1] / 4))
            return false;
        if (D0->ne[2] != 1 && D0->ne[3] != 1) return false;
        t.y = (float *)D0->data;
        t.yt = D0;
        t.yrs = 1;
        t.rg = (int32_t)D0->ne[0];
        t.rgs = (int64_t)(D0->nb[1] / 4);
        t.ycs = (int64_t)((D0->ne[2] == 1 ? D0->nb[3] : D0->nb[2]) / 4);
        t.nrep = (int32_t)idx.size();
        t.rep = rep;
        for (int k : idx) skips.push_back(k);
        return true;
    }

    bool kv_target(const tts_tensor * mm, int64_t M, GemvTarget & t, std::vector<int> & skips) {
        const int64_t N = mm->ne[0];
        if (mm->ne[1] != 1 && M != 1) return false;  // one token per column (decode)
        // the product copied straight into 2-4 repeat-interleaved cache views
        if (mm->type == TTS_TYPE_F32 && contiguous(mm) && repeat_target(mm, mm, N, t, skips)) return true;
        const tts_tensor * c = sole_consumer(mm);
        if (!c) return false;
        if (c->op == TTS_OP_CPY && c->src[0] == mm) {
            const tts_tensor * D = c;  // view of the K cache: [N] or [N, B] with row stride per sequence
            if (D->type != TTS_TYPE_F32 || D->nb[0] != 4 || D->ne[0] != N || D->ne[1] != M || D->ne[2] * D->ne[3] != 1) return false;
            t.y = (float *)D->data;
            t.yt = D;
            t.yrs = 1;
            t.ycs = (int64_t)(D->nb[1] / 4);
            skips.push_back(index[c]);
            return true;
        }
        // mm -> RESHAPE -> repeat copies (repeat_target; any mismatch falls through to the transpose chain below: Parler's V store starts with a
        // RESHAPE too)
        if (c->op == TTS_OP_RESHAPE && c->src[0] == mm && c->type == TTS_TYPE_F32 && repeat_target(mm, c, N, t, skips)) return true;
        // mm -> [RESHAPE] -> TRANSPOSE -> CONT -> CPY
        const tts_tensor * v = c;
        std::vector<int> vs;
        while (v && (v->op == TTS_OP_RESHAPE || v->op == TTS_OP_TRANSPOSE) && v->src[0]) {
            vs.push_back(index[v]);
            const tts_tensor * nx = sole_consumer(v);
            if (!nx) return false;
            if (nx->op == TTS_OP_CONT) {
                const tts_tensor * C = nx;
                const tts_tensor * cp = sole_consumer(C);
                if (!cp || cp->op != TTS_OP_CPY || cp->src[0] != C) return false;
                const tts_tensor * D = cp;
                if (D->type != TTS_TYPE_F32 || D->ne[0] != 1 || D->ne[1] != N || D->ne[2] * D->ne[3] != M) return false;
                t.y = (float *)D->data;
                t.yt = D;
                t.yrs = (int64_t)(D->nb[1] / 4);
                t.ycs = (int64_t)(D->nb[2] / 4);
                skips.push_back(index[C]);
                skips.push_back(index[cp]);
                return true;
            }
            v = nx;
        }
        return false;
    }

    // SwiGLU MLP (Orpheus model.cpp:296-300): MUL(UNARY SILU(MUL_MAT(gate, x)), MUL_MAT(up, x)) with
    // tile-layout Q4_K gate / up: one matrix-core GEMV launch over both matrices whose epilogue
    // writes silu(gate) * up to the MUL's output; gate, silu(gate) and up are never stored.  Every
    // node between the gate product and the MUL must belong to the pattern (or be a view), so the
    // MUL's output can be written at the gate product's position.
    bool try_swiglu(int i) {
        const tts_tensor * G = nodes[i];
        const tts_tensor * a0 = G->src[0];
        const tts_tensor * x = G->src[1];
        if (a0->type != TTS_TYPE_Q4_K || !(a0->flags & TTS_FLAG_TILED) || a0->ne[1] % 16) return false;
        const tts_tensor * S = sole_consumer(G);
        if (!S || S->op != TTS_OP_UNARY || S->op_params[0] != TTS_UNARY_SILU || S->src[0] != G) return false;
        const tts_tensor * E = sole_consumer(S);
        if (!E || E->op != TTS_OP_MUL || E->src[0] != S) return false;
        const tts_tensor * U = E->src[1];
        if (!U || U->op != TTS_OP_MUL_MAT || U->src[1] != x || uses[U] != 1 || !is_gemv(U)) return false;
        const tts_tensor * a = U->src[0];
        if (a->type != a0->type || a->ne[0] != a0->ne[0] || a->ne[1] != a0->ne[1] || a->nb[1] != a0->nb[1] ||
            ((a->flags ^ a0->flags) & (TTS_FLAG_REPACKED | TTS_FLAG_TILED)))
            return false;
        if (E->type != TTS_TYPE_F32 || !contiguous(E) || !contiguous(G) || !contiguous(S) || !contiguous(U)) return false;
        for (int d = 0; d < 4; ++d)
            if (E->ne[d] != G->ne[d] || U->ne[d] != G->ne[d] || S->ne[d] != G->ne[d]) return false;
        const int iS = index[S], iU = index[U], iE = index[E];
        if (iS <= i || iU <= i || iE <= iS || iE <= iU || act[iS] || act[iU] || act[iE]) return false;
        for (int k = i + 1; k < iE; ++k)
            if (k != iS && k != iU && !(is_view(nodes[k]->op) && act[k] == 0)) return false;
        Item it;
        it.kind = Item::GEMV;
        it.epi = EPI_SWIGLU;
        it.mms = {G, U};
        GemvTarget t{(float *)E->data, (int64_t)(E->nb[1] / 4), 1};
        t.yt = E;
        it.tgt = {t, t};
        act[iS] = act[iU] = act[iE] = -1;
        act[i] = add_item(std::move(it));
        return true;
    }

    // SwiGLU MLP on Q8_0 weights (Dia model.cpp:358): MUL(UNARY SILU(MUL_MAT(gate, x)), MUL_MAT(up, y)).
    // The gate product runs alone and is stored; the up product's epilogue reads it back and writes
    // silu(gate) * up to the MUL's output (EPI_SILU_MUL), so the SILU and MUL launches and their
    // tensors disappear.  Needs the gate product first in node order, every node between the up
    // product and the MUL a view (the MUL's output is written at the up product's position), and the
    // MUL's output disjoint from (or exactly) the gate product and disjoint from the up product's src1.
    bool try_silu_mul(int i) {
        const tts_tensor * G = nodes[i];
        if (G->src[0]->type != TTS_TYPE_Q8_0) return false;
        const tts_tensor * S = sole_consumer(G);
        if (!S || S->op != TTS_OP_UNARY || S->op_params[0] != TTS_UNARY_SILU || S->src[0] != G) return false;
        const tts_tensor * E = sole_consumer(S);
        if (!E || E->op != TTS_OP_MUL || E->src[0] != S) return false;
        const tts_tensor * U = E->src[1];
        if (!U || U->op != TTS_OP_MUL_MAT || uses[U] != 1 || !is_gemv(U) || U->src[0]->type != TTS_TYPE_Q8_0) return false;
        if (E->type != TTS_TYPE_F32 || !contiguous(E) || !contiguous(G) || !contiguous(S) || !contiguous(U)) return false;
        for (int d = 0; d < 4; ++d)
            if (E->ne[d] != G->ne[d] || U->ne[d] != G->ne[d] || S->ne[d] != G->ne[d]) return false;
        if ((overlap(E, G) && E->data != G->data) || overlap(E, U->src[1])) return false;
        const int iS = index[S], iU = index[U], iE = index[E];
        if (iS <= i || iU <= i || iE <= iS || iE <= iU || act[iS] || act[iU] || act[iE]) return false;
        for (int k = iU + 1; k < iE; ++k)
            if (k != iS && !(is_view(nodes[k]->op) && act[k] == 0)) return false;
        // G is read back by U's epilogue: nothing between G and U (the SILU aside) may write over it
        // (the allocator frees G's memory after the SILU, so a later node could be placed there)
        for (int k = i + 1; k < iU; ++k)
            if (k != iS && !is_view(nodes[k]->op) && overlap(nodes[k], G)) return false;
        Item g;
        g.kind = Item::GEMV;
        g.mms = {G};
        g.tgt = {GemvTarget{(float *)G->data, (int64_t)(G->nb[1] / 4), 1}};
        g.tgt[0].yt = G;
        Item u;
        u.kind = Item::GEMV;
        u.mms = {U};
        u.tgt = {GemvTarget{(float *)E->data, (int64_t)(E->nb[1] / 4), 1}};
        u.tgt[0].yt = E;
        u.epi = EPI_SILU_MUL;
        u.res = G;
        act[iS] = act[iE] = -1;
        act[i] = add_item(std::move(g));
        act[iU] = add_item(std::move(u));
        return true;
    }

    void try_gemv(int i) {
        const tts_tensor * mm0 = nodes[i];
        if (!is_gemv(mm0)) return;
        // every earlier hoisted product has been copied to its tensor before position i runs: the hoist
        // buffer is free again (a step hoists K and V over Q once per layer)
        if (i > hoist_live) hoist_used = 0;
        const tts_tensor * a0 = mm0->src[0];
        const tts_tensor * x = mm0->src[1];
        const int64_t M = x->ne[1] * x->ne[2] * x->ne[3];
        if ((mask & TTS_FUSE_EPI) && try_swiglu(i)) return;
        if ((mask & TTS_FUSE_EPI) && try_silu_mul(i)) return;
        Item it;
        it.kind = Item::GEMV;
        // src1 = a CONT made right before this product from a contiguous tensor of the same columns
        // (Dia's cont_3d of the attention output): read that tensor and skip the copy
        if ((mask & TTS_FUSE_CONTREAD) && x->op == TTS_OP_CONT && index.count(x) && act[index[x]] == 0 && uses[x] == 1 &&
            next_real(index[x]) == i && x->src[0] && !(x->flags & (TTS_FLAG_OUTPUT | TTS_FLAG_PERSIST))) {
            const tts_tensor * s0 = x->src[0];
            if (s0->type == TTS_TYPE_F32 && contiguous(s0) && contiguous(x) && nel(s0) == nel(x)) {  // the same bytes
                it.xsrc = s0;
                act[index[x]] = -1;
            }
        }
        std::vector<int> skips;
        // Group MUL_MATs sharing src1 and weight type / shape into one launch at the first one's
        // position.  The reference's node order separates them (parler_build_kv_store and
        // orpheus_build_kv_store pull K and V -- and K's rope and cache copies -- in before Q), so the
        // scan passes over views, the KV-store nodes of members already taken, and other nodes; a later
        // product is hoisted over those only if its output (or cache target) overlaps nothing they read
        // or write, and none of them writes src1.
        auto compatible = [&](const tts_tensor * mm) {
            const tts_tensor * a = mm->src[0];
            // another row count: only Q4_K matrices the tile-layout kernels can read (stored tiled, or
            // with a tile-layout copy), each a multiple of 16 rows; run_gemv_item splits the launch
            // when it ends up on a lane-layout kernel
            const bool tl = a->type == TTS_TYPE_Q4_K && (a->flags & (TTS_FLAG_TILED | TTS_FLAG_TILED_COPY)) &&
                            (a0->flags & (TTS_FLAG_TILED | TTS_FLAG_TILED_COPY)) && a->ne[1] % 16 == 0 && a0->ne[1] % 16 == 0;
            if (a->type != a0->type || a->ne[0] != a0->ne[0] || a->nb[1] != a0->nb[1] || (a->ne[1] != a0->ne[1] && !tl)) return false;
            if (a->type == TTS_TYPE_Q4_K && ((a->flags ^ a0->flags) & (TTS_FLAG_REPACKED | TTS_FLAG_TILED)) && !tl) return false;
            return true;
        };
        auto target_span = [&](const tts_tensor * mm, const GemvTarget & t, const char *& y0, const char *& y1) {
            const int64_t Mm = mm->ne[1] * mm->ne[2] * mm->ne[3], rows = mm->ne[0];
            int64_t last;
            if (t.rg > 0) {
                const int64_t g = (rows - 1) / t.rg;
                last = (Mm - 1) * t.ycs + g * t.rgs + (rows - 1 - g * t.rg) * t.yrs + (int64_t)(t.nrep - 1) * t.rep;
            } else {
                last = (Mm - 1) * t.ycs + (rows - 1) * t.yrs;
            }
            y0 = (const char *)t.y;
            y1 = y0 + 4 * (size_t)(last + 1);
        };
        auto hits = [&](const char * y0, const char * y1, const tts_tensor * u) {
            if (!u || !u->data) return false;
            const char * u0 = (const char *)u->data;
            return y0 < u0 + tbytes(u) && u0 < y1;
        };
        std::vector<const tts_tensor *> passed;  // nodes the later members are hoisted over
        const int max_mats = (mask & TTS_FUSE_GROUP) ? GEMV_MAX_MATS : 1;
        const int jend = std::min(n, i + 160);
        int j = i;
        while (j < jend && (int)it.mms.size() < max_mats) {
            const tts_tensor * mm = nodes[j];
            const bool member = j == i || (act[j] == 0 && mm->op == TTS_OP_MUL_MAT && mm->src[1] == x && is_gemv(mm) && compatible(mm));
            if (member) {
                GemvTarget t{(float *)mm->data, (int64_t)(mm->nb[1] / 4), 1};
                t.yt = mm;
                GemvTarget kt{nullptr, 0, 0};
                std::vector<int> ks;
                if ((mask & TTS_FUSE_KV) && mm->ne[1] * mm->ne[2] * mm->ne[3] == M && kv_target(mm, M, kt, ks)) t = kt;
                else ks.clear();
                bool ok = true;
                auto clear_of = [&](const GemvTarget & tt) {
                    const char *y0, *y1;
                    target_span(mm, tt, y0, y1);
                    bool c = true;
                    for (const tts_tensor * u : passed) c = c && !hits(y0, y1, u);
                    for (size_t k = 0; k < it.mms.size() && c; ++k) {
                        const char *z0, *z1;
                        target_span(it.mms[k], it.tgt[k], z0, z1);
                        c = !(y0 < z1 && z0 < y1);
                    }
                    return c;
                };
                if (j > i) ok = clear_of(t);
                // The product's own memory is still in use by what it is hoisted over (the graph
                // allocator reuses the memory of tensors dead at its original position -- Orpheus' Q on
                // K's): it writes backend scratch instead, copied to its tensor at its own position.
                int copy_back = -1;
                const size_t obytes = 4 * (size_t)(mm->ne[0] * mm->ne[1] * mm->ne[2] * mm->ne[3]);
                if (!ok && t.y == (float *)mm->data && t.rg == 0 && contiguous(mm) && hoist_buf &&
                    hoist_used + ((obytes + 255) & ~(size_t)255) <= hoist_cap) {
                    GemvTarget ht{(float *)(hoist_buf + hoist_used), (int64_t)(mm->nb[1] / 4), 1};
                    if (clear_of(ht)) {
                        t = ht;
                        copy_back = j;
                        hoist_used += (obytes + 255) & ~(size_t)255;
                        hoist_live = std::max(hoist_live, j);
                        ok = true;
                    }
                }
                if (ok) {
                    for (int s2 : ks) skips.push_back(s2);
                    it.mms.push_back(mm);
                    it.tgt.push_back(t);
                    if (j > i) act[j] = -1;
                    if (copy_back >= 0) {
                        Item cp;
                        cp.kind = Item::COPY;
                        cp.cp_src = t.y;
                        cp.cp_dst = mm->data;
                        cp.cp_bytes = obytes;
                        act[j] = add_item(std::move(cp));
                    }
                    ++j;
                    continue;
                }
                // not hoistable: it stays where it is, as a node passed over
            }
            if (!(mask & TTS_FUSE_GROUP)) break;
            if (std::find(skips.begin(), skips.end(), j) != skips.end()) {  // a member's KV store: absorbed
                ++j;
                continue;
            }
            if (act[j] == 0 && is_view(mm->op)) {
                ++j;
                continue;
            }
            // a node already claimed by another item is passed over like any other: every item writes
            // only tensors of its nodes (or backend scratch) and reads their sources, all listed here
            if (overlap(mm, x) || (int)passed.size() > 256) break;
            passed.push_back(mm);
            for (int s2 = 0; s2 < TTS_MAX_SRC; ++s2)
                if (mm->src[s2]) passed.push_back(mm->src[s2]);
            ++j;
        }
        if (it.mms.size() == 1 && (mask & TTS_FUSE_EPI)) {
            // epilogue: adjacent GELU or ADD(residual) consuming the single product -- directly, or
            // through a CONT of the contiguous product into another shape of the same columns (Dia's
            // cont_2d before the residual ADD, model.cpp:336-337 here), which is then never made
            const tts_tensor * E = sole_consumer(mm0);
            const tts_tensor * P = mm0;  // the node E reads
            int iP = i;
            if (E && E->op == TTS_OP_CONT && E->src[0] == mm0 && next_real(i) == index[E] && contiguous(E) && contiguous(mm0) &&
                E->type == TTS_TYPE_F32 && E->ne[0] == mm0->ne[0] && nel(E) == nel(mm0) && act[index[E]] == 0) {
                P = E;
                iP = index[E];
                E = sole_consumer(P);
            }
            if (E && next_real(iP) == index[E] && E->src[0] == P && E->type == TTS_TYPE_F32 && contiguous(E) && contiguous(mm0) &&
                E->ne[0] == mm0->ne[0] && nel(E) == nel(mm0) && act[index[E]] == 0) {
                if (E->op == TTS_OP_UNARY && E->op_params[0] == TTS_UNARY_GELU) {
                    it.epi = EPI_GELU;
                } else if (E->op == TTS_OP_ADD && E->src[1]->type == TTS_TYPE_F32 && contiguous(E->src[1]) &&
                           E->src[1]->ne[0] == E->ne[0] && E->src[1]->ne[1] == E->ne[1] && E->src[1]->ne[2] == E->ne[2] &&
                           E->src[1]->ne[3] == E->ne[3] && (!overlap(E, E->src[1]) || E->data == E->src[1]->data)) {
                    it.epi = EPI_ADD;
                    it.res = E->src[1];
                }
                if (it.epi != EPI_NONE && (a0->type != TTS_TYPE_F32 || !overlap(E, x))) {
                    it.tgt[0] = GemvTarget{(float *)E->data, (int64_t)(E->ne[0]), 1};  // contiguous: column stride ne0
                    it.tgt[0].yt = E;
                    act[index[E]] = -1;
                    if (P != mm0) act[iP] = -1;
                } else {
                    it.epi = EPI_NONE;
                    it.res = nullptr;
                }
            }
        }
        for (int s : skips) act[s] = -1;
        act[i] = add_item(std::move(it));
    }

    bool try_heads(int i) {
        const tts_tensor * mm0 = nodes[i];
        if (!is_gemv(mm0)) return false;
        const tts_tensor * x = mm0->src[1];
        const tts_tensor * a0 = mm0->src[0];
        const tts_tensor * C = sole_consumer(mm0);
        if (!C || C->op != TTS_OP_CONCAT || C->op_params[0] != 1 || C->src[0] != mm0) return false;
        Item it;
        it.kind = Item::GEMV;
        it.mms.push_back(mm0);
        std::vector<int> members{i};
        const tts_tensor * last = nullptr;
        while (C && C->op == TTS_OP_CONCAT && C->op_params[0] == 1 && (int)it.mms.size() < GEMV_MAX_MATS) {
            const tts_tensor * mm = C->src[1];
            if (!mm || mm->op != TTS_OP_MUL_MAT || mm->src[1] != x || !is_gemv(mm) || uses[mm] != 1) return false;
            const tts_tensor * a = mm->src[0];
            if (a->type != a0->type || a->ne[0] != a0->ne[0] || a->ne[1] != a0->ne[1] || a->nb[1] != a0->nb[1]) return false;
            if (mm->ne[1] != mm0->ne[1] || mm->ne[2] != mm0->ne[2]) return false;
            it.mms.push_back(mm);
            members.push_back(index[mm]);
            members.push_back(index[C]);
            last = C;
            const tts_tensor * nx = sole_consumer(C);
            if (nx && nx->op == TTS_OP_CONCAT && nx->src[0] == C) C = nx;
            else C = nullptr;
        }
        if (!last || !contiguous(last) || overlap(last, x)) return false;
        const int64_t n1 = mm0->ne[1], n2 = mm0->ne[2];
        int64_t ycs;
        if (n1 == 1) ycs = (int64_t)(last->nb[2] / 4);
        else if (n2 == 1) ycs = (int64_t)(last->nb[1] / 4);
        else return false;
        for (size_t k = 0; k < it.mms.size(); ++k)
            it.tgt.push_back(GemvTarget{(float *)((char *)last->data + k * n1 * last->nb[1]), ycs, 1});
        for (GemvTarget & t : it.tgt) t.yt = last;
        for (int m : members) act[m] = -1;
        act[index[last]] = add_item(std::move(it));
        return true;
    }

    // ---- LSTM recurrences (Kokoro build_lstm / build_lstm_run, src/models/kokoro/model.cpp:35-86) ----
    // Per time step the reference emits, for gates I, F, G, O (weights[1], [3], [5], [7]):
    //   act(ADD(VIEW(pre, column t), ADD(MUL_MAT(W_hh, h_prev), b_hh)))
    // then c = ADD(MUL(F, c_prev), MUL(I, G)), h = MUL(TANH(c), O), and
    // outputs = CONCAT(outputs, h, 1) (reversed: CONCAT(h, outputs, 1)).  A chain of such steps
    // linked through h / c becomes one k_lstm_step launch per step, writing h into a private
    // history; the intermediate concats (O(T^2) bytes of copies) disappear and one launch writes
    // the final concat's [Hd, T] output.  Fused only when nothing outside the chain reads any
    // intermediate (gates, c, h, partial concats), so skipping them is invisible.
    struct LGate {
        const tts_tensor *act, *addp, *view, *addb, *mm;
    };
    struct LStep {
        const tts_tensor *h = nullptr, *th = nullptr, *c = nullptr, *mf = nullptr, *mig = nullptr, *hprev = nullptr, *cprev = nullptr;
        LGate g[4];
        int64_t col = 0;
        int prev = -1, next = -1;
    };

    static bool f32_vec(const tts_tensor * t, int64_t ne0) {
        return t && t->type == TTS_TYPE_F32 && t->ne[0] == ne0 && t->ne[1] * t->ne[2] * t->ne[3] == 1 && t->nb[0] == 4;
    }

    bool lstm_gate(const tts_tensor * a, int uop, int64_t Hd, LGate & g) {
        if (!a || a->op != TTS_OP_UNARY || a->op_params[0] != uop || !f32_vec(a, Hd)) return false;
        const tts_tensor * ap = a->src[0];
        if (!ap || ap->op != TTS_OP_ADD || !f32_vec(ap, Hd)) return false;
        const tts_tensor *v = ap->src[0], *ab = ap->src[1];
        if (!v || v->op != TTS_OP_VIEW || !ab || ab->op != TTS_OP_ADD || !f32_vec(ab, Hd) || !f32_vec(v, Hd)) return false;
        const tts_tensor * mm = ab->src[0];
        if (!mm || mm->op != TTS_OP_MUL_MAT || !f32_vec(mm, Hd) || !f32_vec(ab->src[1], Hd)) return false;
        const tts_tensor * w = mm->src[0];
        if (!w || (w->type != TTS_TYPE_F32 && w->type != TTS_TYPE_F16) || w->ne[1] != Hd || w->ne[2] * w->ne[3] != 1 ||
            w->nb[0] != tts_type_size(w->type) || (w->nb[1] & 15) || ((uintptr_t)w->data & 15))
            return false;
        const tts_tensor * pre = v->src[0];
        if (!pre || pre->type != TTS_TYPE_F32 || pre->nb[0] != 4 || pre->ne[0] != Hd || pre->ne[2] * pre->ne[3] != 1) return false;
        g = LGate{a, ap, v, ab, mm};
        return true;
    }

    bool lstm_step(const tts_tensor * h, LStep & s) {
        if (h->op != TTS_OP_MUL) return false;
        const int64_t Hd = h->ne[0];
        if (!f32_vec(h, Hd) || Hd % 4) return false;
        const tts_tensor *th = h->src[0], *O = h->src[1];
        if (!th || th->op != TTS_OP_UNARY || th->op_params[0] != TTS_UNARY_TANH || !f32_vec(th, Hd)) return false;
        const tts_tensor * c = th->src[0];
        if (!c || c->op != TTS_OP_ADD || !f32_vec(c, Hd)) return false;
        const tts_tensor *mf = c->src[0], *mig = c->src[1];
        if (!mf || mf->op != TTS_OP_MUL || !mig || mig->op != TTS_OP_MUL || !f32_vec(mf, Hd) || !f32_vec(mig, Hd)) return false;
        if (!lstm_gate(mig->src[0], TTS_UNARY_SIGMOID, Hd, s.g[0]) || !lstm_gate(mf->src[0], TTS_UNARY_SIGMOID, Hd, s.g[1]) ||
            !lstm_gate(mig->src[1], TTS_UNARY_TANH, Hd, s.g[2]) || !lstm_gate(O, TTS_UNARY_SIGMOID, Hd, s.g[3]))
            return false;
        s.hprev = s.g[0].mm->src[1];
        const tts_tensor * w0 = s.g[0].mm->src[0];
        const int64_t K = w0->ne[0];
        if (K % 4 || !f32_vec(s.hprev, K) || ((uintptr_t)s.hprev->data & 15)) return false;
        s.cprev = mf->src[1];
        if (!f32_vec(s.cprev, Hd)) return false;
        for (int g = 0; g < 4; ++g) {
            const tts_tensor * w = s.g[g].mm->src[0];
            if (s.g[g].mm->src[1] != s.hprev || w->type != w0->type || w->ne[0] != K) return false;
            const tts_tensor * pre = s.g[g].view->src[0];
            const ptrdiff_t off = (const char *)s.g[g].view->data - (const char *)pre->data;
            if (off < 0 || off % (ptrdiff_t)pre->nb[1]) return false;
            const int64_t col = off / (ptrdiff_t)pre->nb[1];
            if (col >= pre->ne[1] || (g > 0 && col != s.col)) return false;
            s.col = col;
        }
        s.h = h;
        s.th = th;
        s.c = c;
        s.mf = mf;
        s.mig = mig;
        return true;
    }

    void try_lstm() {
        std::vector<LStep> st;
        PtrMap<int> by_h;
        for (int i = 0; i < n; ++i) {
            LStep s;
            if (nodes[i]->op == TTS_OP_MUL && lstm_step(nodes[i], s)) {
                by_h[s.h] = (int)st.size();
                st.push_back(s);
            }
        }
        for (size_t k = 0; k < st.size(); ++k) {
            auto it = by_h.find(st[k].hprev);
            if (it == by_h.end()) continue;
            LStep & p = st[it->second];
            if (p.c != st[k].cprev || p.next != -1 || p.h->ne[0] != st[k].hprev->ne[0]) return;  // ambiguous: fuse nothing
            st[k].prev = it->second;
            p.next = (int)k;
        }
        std::vector<ChainPlan> plans;
        for (size_t k0 = 0; k0 < st.size(); ++k0) {
            if (st[k0].prev != -1) continue;
            std::vector<int> seq;
            for (int k = (int)k0; k != -1; k = st[k].next) seq.push_back(k);
            ChainPlan cp;
            if (lstm_chain(st, seq, cp)) plans.push_back(std::move(cp));
        }
        std::sort(plans.begin(), plans.end(), [](const ChainPlan & x, const ChainPlan & y) { return x.steps[0] < y.steps[0]; });
        // build_lstm's bidirectional cell runs its forward chain, then its reverse chain: the two are
        // independent, so one launch can advance both.  The earlier chain (A) is delayed to the
        // later one's (B) step positions; its input projections are stashed first (their arena
        // memory may be handed to B's projections once A's own steps have passed) and its output
        // is written at B's end, which is safe when nothing reads it before then.
        std::vector<int> partner(plans.size(), -1);
        for (size_t a = 0; a + 1 < plans.size(); ++a) {
            if (partner[a] != -1) continue;
            ChainPlan & A = plans[a];
            ChainPlan & B = plans[a + 1];
            if (partner[a + 1] != -1 || A.Hd != B.Hd || A.T != B.T || A.K != B.K || A.wtype != B.wtype || A.fin_idx >= B.steps[0]) continue;
            bool ok = A.stash_ok && lstm_used + 4 * (size_t)A.Hd * (size_t)A.T <= lstm_cap;
            auto cs = consumers.find(A.fin);
            if (cs != consumers.end())
                for (int j : cs->second) ok = ok && j > B.fin_idx;
            if (!ok) continue;
            partner[a] = (int)a + 1;
            partner[a + 1] = (int)a;
        }
        for (size_t k = 0; k < plans.size(); ++k) {
            ChainPlan & P = plans[k];
            for (int m : P.members) act[m] = -1;
            if (partner[k] == -1) {
                emit_chain(P, nullptr);
            } else if (partner[k] > (int)k) {
                ChainPlan & B = plans[partner[k]];
                for (int m : B.members) act[m] = -1;
                if (lstm_used + 4 * (size_t)P.Hd * (size_t)P.T + 64 <= lstm_cap) {
                    emit_chain(B, &P);
                } else {  // no room left for the stash: two plain chains
                    emit_chain(P, nullptr);
                    emit_chain(B, nullptr);
                }
                ++k;
            }
        }
    }

    struct ChainPlan {
        std::vector<int> steps;  // node index of each step's h, in chain order
        std::vector<LstmStepArgs> args;
        std::vector<int> members;
        std::vector<int64_t> cols;
        const tts_tensor * fin = nullptr;
        int fin_idx = -1;
        const tts_tensor * pre[4] = {};
        bool stash_ok = false;
        float *hist = nullptr, *cbuf = nullptr;
        int64_t Hd = 0, T = 0, K = 0;
        int wtype = 0;
    };

    // One chain's items; with `other`, its steps also advance `other` (stashed projections) and its
    // output write also writes other's.
    void emit_chain(ChainPlan & P, ChainPlan * other) {
        float * stash = nullptr;
        if (other) {
            stash = lstm_buf + lstm_used;
            lstm_used += (4 * (size_t)other->Hd * (size_t)other->T + 63) & ~(size_t)63;
            Item it;
            it.kind = Item::LSTM;
            it.lkind = 4;
            for (int g = 0; g < 4; ++g) {
                it.lstash_src[g] = other->pre[g]->data;
                it.lstash_dst[g] = stash + (size_t)g * other->Hd * other->T;
            }
            it.lstash_bytes = sizeof(float) * (size_t)other->Hd * (size_t)other->T;
            act[other->steps[0]] = add_item(std::move(it));
            for (size_t s = 0; s < other->args.size(); ++s)
                for (int g = 0; g < 4; ++g) other->args[s].pre[g] = stash + (size_t)g * other->Hd * other->T + other->cols[s] * other->Hd;
        }
        for (int64_t s = 0; s < P.T; ++s) {
            Item it;
            it.kind = Item::LSTM;
            it.lkind = 1;
            it.ls = P.args[s];
            if (other) {
                it.ls2 = other->args[s];
                it.lpair = true;
            }
            if (s == P.T - 1 && P.T == 1) {
                it.lkind = 3;
                it.lfinal = P.fin, it.lhist = P.hist, it.lHd = P.Hd, it.lT = P.T;
                if (other) it.lfinal2 = other->fin, it.lhist2 = other->hist;
            }
            act[P.steps[s]] = add_item(std::move(it));
        }
        if (P.T > 1) {
            Item it;
            it.kind = Item::LSTM;
            it.lkind = 2;
            it.lfinal = P.fin, it.lhist = P.hist, it.lHd = P.Hd, it.lT = P.T;
            if (other) it.lfinal2 = other->fin, it.lhist2 = other->hist;
            act[P.fin_idx] = add_item(std::move(it));
        }
    }

    bool lstm_chain(const std::vector<LStep> & st, const std::vector<int> & seq, ChainPlan & P) {
        const int64_t T = (int64_t)seq.size();
        const LStep & s0 = st[seq[0]];
        const int64_t Hd = s0.h->ne[0];
        int dir = 1;
        if (T > 1) dir = (int)(st[seq[1]].col - s0.col);
        if (dir != 1 && dir != -1) return false;
        if (s0.col != (dir == 1 ? 0 : T - 1)) return false;
        for (int64_t s = 1; s < T; ++s)
            if (st[seq[s]].col != s0.col + dir * s) return false;
        // the concat chain that accumulates the outputs
        PtrMap<int> mem;  // chain members
        mem.reserve((size_t)T * 32);
        auto add = [&](const tts_tensor * t) { mem[t] = 1; };
        const tts_tensor * out = s0.h;
        for (int64_t s = 0; s < T; ++s) {
            const LStep & S = st[seq[s]];
            add(S.h), add(S.th), add(S.c), add(S.mf), add(S.mig);
            for (int g = 0; g < 4; ++g) add(S.g[g].act), add(S.g[g].addp), add(S.g[g].view), add(S.g[g].addb), add(S.g[g].mm);
            if (s == 0) continue;
            const tts_tensor * C = nullptr;
            auto cs = consumers.find(S.h);
            if (cs == consumers.end()) return false;
            for (int j : cs->second) {
                const tts_tensor * x = nodes[j];
                if (x->op != TTS_OP_CONCAT || x->op_params[0] != 1) continue;
                if ((dir == 1 && x->src[0] == out && x->src[1] == S.h) || (dir == -1 && x->src[0] == S.h && x->src[1] == out)) C = x;
            }
            if (!C) return false;
            add(C);
            out = C;
        }
        const tts_tensor * fin = out;
        if (fin->type != TTS_TYPE_F32 || fin->ne[0] != Hd || fin->ne[1] != T || fin->ne[2] * fin->ne[3] != 1 || fin->nb[0] != 4) return false;
        // nothing outside the chain may read an intermediate (the final output excepted)
        for (const auto & kv : mem.entries) {
            if (kv.first == fin) continue;
            auto cs = consumers.find(kv.first);
            if (cs == consumers.end()) continue;
            for (int j : cs->second)
                if (!mem.count(nodes[j])) return false;
        }
        for (const auto & kv : mem.entries)
            if (act[index[kv.first]] != 0) return false;
        const size_t need = (size_t)Hd * (size_t)(T + 1);
        if (!lstm_buf || lstm_used + need > lstm_cap) return false;
        float * cbuf = lstm_buf + lstm_used;
        float * hist = cbuf + Hd;
        lstm_used += (need + 63) & ~(size_t)63;
        P.members.reserve(mem.entries.size());
        for (const auto & kv : mem.entries) P.members.push_back(index[kv.first]);
        P.fin = fin;
        P.fin_idx = index[fin];
        P.hist = hist, P.cbuf = cbuf;
        P.Hd = Hd, P.T = T;
        P.K = s0.g[0].mm->src[0]->ne[0];
        P.wtype = s0.g[0].mm->src[0]->type;
        // the stash copies each gate's whole [Hd, T] projection: dense f32, four distinct tensors
        P.stash_ok = true;
        for (int g = 0; g < 4; ++g) {
            const tts_tensor * pre = s0.g[g].view->src[0];
            P.pre[g] = pre;
            P.stash_ok = P.stash_ok && pre->type == TTS_TYPE_F32 && pre->ne[0] == Hd && pre->ne[1] == T && pre->nb[1] == (size_t)Hd * 4 &&
                         contiguous(pre);
            for (int g2 = 0; g2 < g; ++g2) P.stash_ok = P.stash_ok && P.pre[g2] != pre;
            // a paired chain runs late: what it reads besides the stashed projections (initial h / c,
            // the biases) must be model / persistent memory, never arena memory a later node may reuse
            const tts_tensor * bt = s0.g[g].addb->src[1];
            P.stash_ok = P.stash_ok && persistent_mem(bt);
        }
        P.stash_ok = P.stash_ok && persistent_mem(s0.hprev) && persistent_mem(s0.cprev);
        for (int64_t s = 0; s < T; ++s) {
            const LStep & S = st[seq[s]];
            LstmStepArgs a;
            for (int g = 0; g < 4; ++g) {
                a.pre[g] = (const float *)S.g[g].view->data;
                a.w[g] = S.g[g].mm->src[0]->data;
                a.w_rs[g] = (int64_t)S.g[g].mm->src[0]->nb[1];
                a.bias[g] = (const float *)S.g[g].addb->src[1]->data;
            }
            a.hprev = s == 0 ? (const float *)S.hprev->data : hist + st[seq[s - 1]].col * Hd;
            a.cprev = s == 0 ? (const float *)S.cprev->data : cbuf;
            a.h = hist + S.col * Hd;
            a.c = cbuf;
            a.Hd = (int)Hd;
            a.K = (int)S.g[0].mm->src[0]->ne[0];
            a.wtype = S.g[0].mm->src[0]->type;
            P.args.push_back(a);
            P.steps.push_back(index[S.h]);
            P.cols.push_back(S.col);
        }
        return true;
    }

    // snake_1d (src/util.cpp:98-101): ADD(x, MUL(SQR(SIN(MUL(x, alpha))), recip)) -> one pass.
    // recip (reciprocal(alpha), a DIV node) is computed where it stands; alpha / recip are [1, C].
    static bool chan_vec(const tts_tensor * t, int64_t C) {
        return t && t->type == TTS_TYPE_F32 && contiguous(t) && t->ne[0] == 1 && (t->ne[1] == C || t->ne[1] == 1) && t->ne[2] * t->ne[3] == 1;
    }
    void try_snake(int i) {
        const tts_tensor * A = nodes[i];
        const tts_tensor *x = A->src[0], *M2 = A->src[1];
        if (!x || !M2 || M2->op != TTS_OP_MUL || sole_consumer(M2) != A) return;
        const tts_tensor *Q = M2->src[0], *R = M2->src[1];
        if (!Q || Q->op != TTS_OP_SQR || sole_consumer(Q) != M2) return;
        const tts_tensor * S = Q->src[0];
        if (!S || S->op != TTS_OP_SIN || sole_consumer(S) != Q) return;
        const tts_tensor * M1 = S->src[0];
        if (!M1 || M1->op != TTS_OP_MUL || sole_consumer(M1) != S || M1->src[0] != x) return;
        const tts_tensor * alpha = M1->src[1];
        const tts_tensor * same[5] = {x, M1, S, Q, M2};
        for (const tts_tensor * t : same)
            if (t->type != TTS_TYPE_F32 || !contiguous(t) || t->ne[0] != A->ne[0] || t->ne[1] != A->ne[1] || t->ne[2] != A->ne[2] ||
                t->ne[3] != A->ne[3])
                return;
        if (A->type != TTS_TYPE_F32 || !contiguous(A) || x->ne[0] < 2) return;
        if (!chan_vec(alpha, x->ne[1]) || !chan_vec(R, x->ne[1]) || alpha->ne[1] != R->ne[1]) return;
        if (overlap(A, x) && A->data != x->data) return;
        if (overlap(A, alpha) || overlap(A, R)) return;
        Item it;
        it.kind = Item::SNAKE;
        it.x = x, it.w = alpha, it.b = R, it.dst = A;
        // reciprocal() = DIV(broadcast view of a scalar, alpha) feeding only this snake (DAC, SNAC):
        // the kernel divides itself (the same correctly rounded division) and the node is skipped
        const tts_tensor * O = R->src[0];
        const bool rfuse = R->op == TTS_OP_DIV && O && R->src[1] == alpha && sole_consumer(R) == M2 && index.count(R) && act[index[R]] == 0 &&
                           O->type == TTS_TYPE_F32 && O->ne[0] == 1 && O->nb[1] == 0 && O->ne[2] * O->ne[3] == 1 && !overlap(A, O);
        // a time mask in front, read by this snake only (tts_dac_decode_batch zeroes the gaps between
        // prompts): x = MUL(x0, m [ne0, 1]) -> the kernel multiplies (the same f32 product) and the node is skipped.
        // x0 and m are then read at the snake's position instead of the MUL's: no node still executed in
        // between may write over them (the allocator may hand x0's memory on once the MUL has read it)
        auto untouched_since = [&](const tts_tensor * t, int from) {
            for (int k = from + 1; k < i; ++k) {
                const tts_tensor * nk = nodes[k];
                // (a node folded into another item, act -1, is still written when that item runs: checked too)
                if (is_view(nk->op) || nk == M1 || nk == S || nk == Q || nk == M2 || (rfuse && nk == R)) continue;
                if (overlap(nk, t)) return false;
            }
            return true;
        };
        if (x->op == TTS_OP_MUL && index.count(x) && act[index[x]] == 0 && uses[x] == 2 && untouched_since(x->src[0], index[x]) &&
            (!x->src[1] || untouched_since(x->src[1], index[x]))) {
            const tts_tensor *x0 = x->src[0], *m = x->src[1];
            const auto ci = consumers.find(x);
            bool only = ci != consumers.end() && ci->second.size() == 2;
            if (only)
                for (int c : ci->second) only &= nodes[c] == M1 || nodes[c] == A;
            if (only && x0 && m && x0->type == TTS_TYPE_F32 && contiguous(x0) && x0->ne[0] == x->ne[0] && x0->ne[1] == x->ne[1] &&
                x0->ne[2] == x->ne[2] && x0->ne[3] == x->ne[3] && m->type == TTS_TYPE_F32 && contiguous(m) && m->ne[0] == x->ne[0] &&
                m->ne[1] * m->ne[2] * m->ne[3] == 1 && !overlap(A, m) && !(overlap(A, x0) && A->data != x0->data)) {
                it.x = x0;
                it.snake_mask = m;
                act[index[x]] = -1;
            }
        }
        act[index[M1]] = act[index[S]] = act[index[Q]] = act[index[M2]] = -1;
        if (rfuse) {
            it.b = nullptr;
            it.snake_one = O;
            act[index[R]] = -1;
        }
        act[i] = add_item(std::move(it));
    }

    // AdaIN1d as build_kokoro_generator_res_block emits it (kokoro/model.cpp:136-165):
    //   n = NORM(x [T, C]); c1 = CONT(TRANSPOSE(n)); y = ADD(ADD(c1, MUL(c1, gamma)), beta);
    //   c2 = CONT(TRANSPOSE(y)) [T, C]; optionally snake_1d(alpha, c2) (util.cpp:98-101)
    // -> one pass per channel row (k_adain_snake).  The item runs where the last absorbed node
    // ran, so the nodes executed in between (the recip DIV, ...) must not write over its inputs.
    static bool vec_c(const tts_tensor * t, int64_t C) {  // [C] or [C, 1] f32, or [1, C] (stride 4)
        if (!t || t->type != TTS_TYPE_F32 || t->ne[2] * t->ne[3] != 1 || t->nb[0] != 4) return false;
        return (t->ne[0] == C && t->ne[1] == 1) || (t->ne[0] == 1 && t->ne[1] == C && t->nb[1] == 4);
    }
    static bool same_shape(const tts_tensor * a, int64_t n0, int64_t n1) {
        return a->type == TTS_TYPE_F32 && a->ne[0] == n0 && a->ne[1] == n1 && a->ne[2] * a->ne[3] == 1;
    }
    // TTS_PLAN_DEBUG=1: report why a fusion pattern was not taken
    static bool plan_debug() {
        static const bool dbg = getenv("TTS_PLAN_DEBUG") != nullptr;
        return dbg;
    }
    static void plan_reject(const char * what, int code) {
        if (plan_debug()) fprintf(stderr, "plan: %s not fused (check %d)\n", what, code);
    }
    static bool adain_fail(int code) {
        plan_reject("adain", code);
        return false;
    }
    bool try_adain(int i) {
        const tts_tensor * N = nodes[i];
        const tts_tensor * X = N->src[0];
        if (!X || X->type != TTS_TYPE_F32 || N->type != TTS_TYPE_F32 || X->nb[0] != 4 || N->ne[2] * N->ne[3] != 1) return adain_fail(1);
        const int64_t T = N->ne[0], C = N->ne[1];
        if (!adain_supported(T)) return adain_fail(2);
        const tts_tensor * T1 = sole_consumer(N);
        if (!T1 || T1->op != TTS_OP_TRANSPOSE) return adain_fail(3);
        const tts_tensor * C1 = sole_consumer(T1);
        if (!C1 || C1->op != TTS_OP_CONT || !same_shape(C1, C, T) || uses[C1] != 2) return adain_fail(4);
        const auto & cc = consumers[C1];
        if (cc.size() != 2) return adain_fail(5);
        const tts_tensor *M = nodes[cc[0]], *A1 = nodes[cc[1]];
        if (M->op != TTS_OP_MUL || M->src[0] != C1 || !vec_c(M->src[1], C) || sole_consumer(M) != A1) return adain_fail(6);
        if (A1->op != TTS_OP_ADD || A1->src[0] != C1 || A1->src[1] != M || !same_shape(A1, C, T)) return adain_fail(7);
        const tts_tensor * A2 = sole_consumer(A1);
        if (!A2 || A2->op != TTS_OP_ADD || A2->src[0] != A1 || !vec_c(A2->src[1], C) || !same_shape(A2, C, T)) return adain_fail(8);
        const tts_tensor * T2 = sole_consumer(A2);
        if (!T2 || T2->op != TTS_OP_TRANSPOSE) return adain_fail(9);
        const tts_tensor * C2 = sole_consumer(T2);
        if (!C2 || C2->op != TTS_OP_CONT || !same_shape(C2, T, C) || !contiguous(C2)) return adain_fail(10);
        const tts_tensor *gamma = M->src[1], *beta = A2->src[1];
        std::vector<int> absorbed = {i, index[C1], index[M], index[A1], index[A2], index[C2]};
        // gamma / beta = ADD(MUL_MAT(W [S, C] f32, style [S]), bias [C]) used only here: evaluated
        // in the kernel, so neither their nodes nor their (aliasable) outputs are needed
        auto affine_src = [&](const tts_tensor * v, const tts_tensor * user, const tts_tensor *& W, const tts_tensor *& B,
                              const tts_tensor *& st) {
            if (!v || v->op != TTS_OP_ADD || sole_consumer(v) != user) return false;
            const tts_tensor * mm = v->src[0];
            if (!mm || mm->op != TTS_OP_MUL_MAT || sole_consumer(mm) != v || !vec_c(v->src[1], C) || v->src[1]->ne[0] != C) return false;
            W = mm->src[0], st = mm->src[1], B = v->src[1];
            const int64_t S = W->ne[0];
            return W->type == TTS_TYPE_F32 && contiguous(W) && W->ne[1] == C && W->ne[2] * W->ne[3] == 1 && S % 4 == 0 &&
                   ((uintptr_t)W->data % 16) == 0 && st->type == TTS_TYPE_F32 && contiguous(st) && st->ne[0] == S &&
                   st->ne[1] * st->ne[2] * st->ne[3] == 1 && ((uintptr_t)st->data % 16) == 0;
        };
        const tts_tensor *gW = nullptr, *gB = nullptr, *gS = nullptr, *bW = nullptr, *bB = nullptr, *bS = nullptr;
        const bool inline_gb = affine_src(gamma, M, gW, gB, gS) && affine_src(beta, A2, bW, bB, bS) && gS == bS;
        if (inline_gb) {
            for (const tts_tensor * t : {gamma, (const tts_tensor *)gamma->src[0], beta, (const tts_tensor *)beta->src[0]}) absorbed.push_back(index[t]);
            gamma = beta = nullptr;  // no longer read
        }
        const tts_tensor * out = C2;
        const tts_tensor *alpha = nullptr, *recip = nullptr, *one = nullptr;
        // snake_1d on C2: M1 = MUL(C2, alpha), S = SIN(M1), Q = SQR(S), M2 = MUL(Q, R), A = ADD(C2, M2)
        if ((mask & TTS_FUSE_SNAKE) && uses[C2] == 2) {
            const auto & sc = consumers[C2];
            const tts_tensor *M1 = nodes[sc[0]], *SA = nodes[sc[1]];
            const tts_tensor *S = sole_consumer(M1), *Q = S ? sole_consumer(S) : nullptr, *M2 = Q ? sole_consumer(Q) : nullptr;
            // reciprocal() (util.cpp:86-94) = DIV(broadcast view of a scalar, alpha): when it feeds
            // only this snake, the kernel evaluates it itself (same division) and the node is skipped
            const tts_tensor * R = M2 ? M2->src[1] : nullptr;
            const tts_tensor * O = R ? R->src[0] : nullptr;
            const bool r_inline = R && R->op == TTS_OP_DIV && O && R->src[1] == M1->src[1] && sole_consumer(R) == M2 &&
                                  O->type == TTS_TYPE_F32 && O->nb[1] == 0 && O->ne[0] == 1 && O->ne[2] * O->ne[3] == 1 &&
                                  same_shape(R, 1, C);
            if (M1->op == TTS_OP_MUL && M1->src[0] == C2 && S && S->op == TTS_OP_SIN && Q && Q->op == TTS_OP_SQR && M2 &&
                M2->op == TTS_OP_MUL && M2->src[0] == Q && sole_consumer(M2) == SA && SA->op == TTS_OP_ADD && SA->src[0] == C2 &&
                SA->src[1] == M2 && vec_c(M1->src[1], C) && vec_c(M2->src[1], C) && same_shape(SA, T, C) && contiguous(SA) &&
                same_shape(M1, T, C) && same_shape(S, T, C) && same_shape(Q, T, C) && same_shape(M2, T, C)) {
                alpha = M1->src[1];
                recip = M2->src[1];
                out = SA;
                for (const tts_tensor * t : {M1, S, Q, M2, SA}) absorbed.push_back(index[t]);
                if (r_inline) {
                    absorbed.push_back(index[R]);
                    recip = nullptr;
                    one = O;
                }
            }
        }
        // rows are read whole before they are written, so out may be X itself (same rows), but
        // no other aliasing with the inputs
        const bool in_place = out->data == X->data && out->nb[1] == X->nb[1];
        if (overlap(out, X) && !in_place) return adain_fail(11);
        // ggml-alloc may place the output over gamma / beta (freed after their absorbed consumers):
        // then the launch first copies the vectors to the backend's scratch
        bool stage = false;
        for (const tts_tensor * t : {gamma, beta, alpha, recip, one})
            if (t && overlap(out, t)) stage = true;
        if (inline_gb)
            for (const tts_tensor * t : {gW, gB, bW, bB, gS})
                if (overlap(out, t)) return adain_fail(14);
        if (stage && 4 * C + 1 > (int64_t)vec_cap) return adain_fail(12);
        const int last = *std::max_element(absorbed.begin(), absorbed.end());
        std::vector<bool> is_abs(n, false);
        for (int k : absorbed) is_abs[k] = true;
        for (int k = i + 1; k < last; ++k) {  // nodes that still run between the NORM and the item
            // (a node folded into another item, act -1, is still written when that item runs: checked too)
            if (is_abs[k] || is_view(nodes[k]->op)) continue;
            const tts_tensor * w = nodes[k];
            for (const tts_tensor * t : {X, gamma, beta, alpha, recip, one, gW, gB, bW, bB, gS})
                if (t && t != w && overlap(w, t)) {
                    if (plan_debug()) fprintf(stderr, "plan: adain node %d (%s) between %d..%d overlaps an input\n", k, tts_op_name(w->op), i, last);
                    return adain_fail(13);
                }
        }
        AdainArgs a;
        a.x = (const float *)X->data;
        a.xcs = (int64_t)(X->nb[1] / 4);
        a.y = (float *)out->data;
        a.ycs = (int64_t)(out->nb[1] / 4);
        auto vstride = [](const tts_tensor * t) { return t->ne[0] == 1 ? (int64_t)(t->nb[1] / 4) : (int64_t)1; };
        if (inline_gb) {
            a.gw = (const float *)gW->data, a.gb = (const float *)gB->data;
            a.bw = (const float *)bW->data, a.bb = (const float *)bB->data;
            a.style = (const float *)gS->data, a.S = gW->ne[0];
        } else {
            a.gamma = (const float *)gamma->data, a.gcs = vstride(gamma);
            a.beta = (const float *)beta->data, a.bcs = vstride(beta);
        }
        if (alpha) {
            a.alpha = (const float *)alpha->data, a.acs = vstride(alpha);
            if (recip) a.recip = (const float *)recip->data, a.rcs = vstride(recip);
            else a.one = (const float *)one->data;
        }
        a.T = T, a.C = C;
        a.stage = stage;
        memcpy(&a.eps, &N->op_params[0], 4);
        Item it;
        it.kind = Item::ADAIN;
        it.adain = a;
        it.dst = out;
        for (int k : absorbed)
            if (k != last) act[k] = -1;
        act[last] = add_item(std::move(it));
        return true;
    }

    // ggml_conv_1d's IM2COL(F16) -> RESHAPE -> MUL_MAT -> RESHAPE, then optionally ADD of a
    // per-channel bias and ADD of a same-shape residual (build_residual_unit,
    // general_neural_audio_codec.cpp:133-149; build_kokoro_generator_res_block,
    // kokoro/model.cpp:136-165) -> one implicit-GEMM kernel that never writes the im2col matrix.
    static const tts_tensor * through_view(const tts_tensor * t) { return t && t->op == TTS_OP_RESHAPE ? t->src[0] : t; }
    void try_conv(int i) {
        const tts_tensor * col = nodes[i];
        const tts_tensor *kern = col->src[0], *x = col->src[1];
        if (col->type != TTS_TYPE_F16 || col->op_params[6] != 0 || col->ne[2] * col->ne[3] != 1) return plan_reject("conv", 1);  // 1-D, one batch
        if (!x || x->type != TTS_TYPE_F32 || x->ne[2] * x->ne[3] != 1) return plan_reject("conv", 2);
        if (!kern || (kern->type != TTS_TYPE_F32 && kern->type != TTS_TYPE_F16) || kern->ne[3] != 1) return plan_reject("conv", 3);
        const tts_tensor * cv = sole_consumer(col);
        if (!cv || cv->op != TTS_OP_RESHAPE || !contiguous(col)) return plan_reject("conv", 4);
        const tts_tensor * mm = sole_consumer(cv);
        if (!mm || mm->op != TTS_OP_MUL_MAT || mm->src[0] != cv || mm->type != TTS_TYPE_F32) return plan_reject("conv", 5);
        const tts_tensor * wv = mm->src[1];
        if (!wv || through_view(wv) != kern) return plan_reject("conv", 6);
        const int K = (int)kern->ne[0];
        const int64_t IC = kern->ne[1], OC = kern->ne[2], L = x->ne[0], OL = col->ne[1];
        if (x->ne[1] != IC || mm->ne[0] != OL || mm->ne[1] != OC || !contiguous(mm)) return plan_reject("conv", 7);
        const int s = col->op_params[0], p = col->op_params[2], d = col->op_params[4];
        if (!conv1d_fused_ok(IC, K, s, d, nullptr)) return plan_reject("conv", 8);
        if (kern->nb[0] != tts_type_size(kern->type)) return plan_reject("conv", 9);
        // the conv output may continue into a RESHAPE (ggml_conv_1d's reshape_3d), bias ADD, residual ADD
        const tts_tensor * out = mm;
        std::vector<int> absorbed = {i, (int)index[mm]};
        const tts_tensor * r3 = sole_consumer(mm);
        const tts_tensor * cur = mm;
        if (r3 && r3->op == TTS_OP_RESHAPE && r3->ne[0] == OL && r3->ne[1] == OC) cur = r3;
        Conv1dArgs a;
        const tts_tensor * bias = nullptr;
        const tts_tensor * res = nullptr;
        const tts_tensor * nb = sole_consumer(cur);
        if (nb && nb->op == TTS_OP_ADD && nb->src[0] == cur && nb->type == TTS_TYPE_F32 && contiguous(nb) && nb->ne[0] == OL &&
            nb->ne[1] == OC && nb->ne[2] * nb->ne[3] == 1 && chan_vec(nb->src[1], OC) && nb->src[1]->ne[1] == OC) {
            bias = nb->src[1];
            out = nb;
            absorbed.push_back(index[nb]);
            const tts_tensor * nr = sole_consumer(nb);
            if (nr && nr->op == TTS_OP_ADD && nr->type == TTS_TYPE_F32 && contiguous(nr) && nr->ne[0] == OL && nr->ne[1] == OC &&
                nr->ne[2] * nr->ne[3] == 1) {
                const tts_tensor * other = nr->src[0] == nb ? nr->src[1] : nr->src[0];
                if (other && other != nb && other->type == TTS_TYPE_F32 && contiguous(other) && other->ne[0] == OL && other->ne[1] == OC &&
                    other->ne[2] * other->ne[3] == 1 && (!overlap(nr, other) || nr->data == other->data)) {
                    res = other;
                    out = nr;
                    absorbed.push_back(index[nr]);
                }
            }
        }
        // The kernel reads x windows across tiles while writing its output, so the output must
        // not alias x.  ggml-alloc often hands a conv's output the memory of its input (freed
        // after IM2COL); then the kernel writes the im2col buffer instead -- dead in the fused
        // form, allocated while x was alive -- and a D2D copy moves the result into place.
        // The fused item runs at the last absorbed node but reads x (and writes the staging
        // buffer) then: a node scheduled in between (e.g. a shortcut branch ahead of the residual
        // ADD, kokoro/model.cpp:122-133) may own that memory by then.  Without the residual the
        // span usually closes; otherwise the chain is left unfused.
        float * stage = nullptr;
        for (;;) {
            if (overlap(out, kern) || (bias && overlap(out, bias))) return plan_reject("conv", 10);
            stage = nullptr;
            bool ok = true;
            bool in_col = false;
            if (overlap(out, x)) {
                const size_t need = (size_t)OL * (size_t)OC * 4;
                if (tbytes(col) >= need && !overlap(col, x) && !overlap(col, out) && !(res && overlap(col, res)) && !overlap(col, kern) &&
                    !(bias && overlap(col, bias))) {
                    stage = (float *)col->data;
                    in_col = true;
                } else if (conv_stage && need <= 4 * conv_stage_cap) {
                    stage = conv_stage;  // the backend's own staging buffer (never arena memory)
                } else {
                    ok = false;
                }
            }
            for (int j = i + 1; ok && j < absorbed.back(); ++j) {
                if (std::find(absorbed.begin(), absorbed.end(), j) != absorbed.end() || is_view(nodes[j]->op)) continue;
                if (overlap(nodes[j], x) || (in_col && overlap(nodes[j], col))) ok = false;
            }
            if (ok) break;
            if (!res) return plan_reject("conv", 11);
            res = nullptr;  // retry with the chain ending at the bias ADD
            absorbed.pop_back();
            out = bias ? nb : mm;
        }
        a.x = make_td(x);
        a.w = kern->data;
        a.w16 = kern->type == TTS_TYPE_F16;
        const size_t es = tts_type_size(kern->type);
        a.wk = (int64_t)(kern->nb[0] / es), a.wic = (int64_t)(kern->nb[1] / es), a.woc = (int64_t)(kern->nb[2] / es);
        a.y = (float *)out->data;
        a.ycs = (int64_t)(out->nb[1] / 4);
        if (stage) {
            a.copy_dst = a.y;
            a.y = stage;
            a.ycs = OL;
        }
        if (bias) a.bias = (const float *)bias->data, a.bcs = bias->ne[1] == 1 ? 0 : (int64_t)(bias->nb[1] / 4);
        if (res) a.res = (const float *)res->data, a.rcs = (int64_t)(res->nb[1] / 4);
        a.L = L, a.IC = IC, a.OL = OL, a.OC = OC;
        a.K = K, a.s = s, a.p = p, a.d = d;
        const size_t xb = (size_t)((x->ne[0] - 1) * x->nb[0] + (x->ne[1] - 1) * x->nb[1]) + 4;
        const size_t wb = tbytes(kern);
        if (xb >= 0x80000000u || wb >= 0x80000000u) return plan_reject("conv", 12);  // 32-bit buffer offsets
        a.x_bytes = (uint32_t)xb, a.w_bytes = (uint32_t)wb;
        Item it;
        it.kind = Item::CONV;
        it.conv = a;
        it.dst = out;
        for (size_t k = 0; k + 1 < absorbed.size(); ++k) act[absorbed[k]] = -1;
        act[absorbed.back()] = add_item(std::move(it));
    }

    // ADD chain over GET_ROWS terms (parler_build_inp_embd, model.cpp:387-410) -> one launch.
    // Linear chains only (each ADD has at most one ADD operand), evaluated innermost pair first.
    bool embed_terms(const tts_tensor * a, const tts_tensor * root, std::vector<const tts_tensor *> & terms, std::vector<int> & members) {
        if (a->op != TTS_OP_ADD || a->type != TTS_TYPE_F32) return false;
        for (int d = 0; d < 4; ++d)
            if (a->ne[d] != root->ne[d]) return false;
        const tts_tensor *l = a->src[0], *r = a->src[1];
        if (!l || !r) return false;
        const bool la = l->op == TTS_OP_ADD, ra = r->op == TTS_OP_ADD;
        if (la && ra) return false;
        auto leaf_ok = [&](const tts_tensor * g) {
            if (g->op != TTS_OP_GET_ROWS || sole_consumer(g) != a || g->type != TTS_TYPE_F32) return false;
            const tts_tensor *tab = g->src[0], *idx = g->src[1];
            if (tab->type != TTS_TYPE_F32 && tab->type != TTS_TYPE_F16 && tab->type != TTS_TYPE_Q8_0 && tab->type != TTS_TYPE_Q4_K) return false;
            if (idx->type != TTS_TYPE_I32 || idx->ne[1] * idx->ne[2] * idx->ne[3] != 1 || (idx->nb[0] % 4)) return false;
            if (tab->ne[0] != root->ne[0] || g->ne[0] != root->ne[0] || tab->ne[2] * tab->ne[3] != 1) return false;
            const int64_t rows = g->ne[1] * g->ne[2] * g->ne[3], M = root->ne[1] * root->ne[2] * root->ne[3];
            return idx->ne[0] == rows && (rows == 1 || rows == M);
        };
        if (la || ra) {
            const tts_tensor * inner = la ? l : r;
            const tts_tensor * leaf = la ? r : l;
            if (sole_consumer(inner) != a || !leaf_ok(leaf)) return false;
            if (!embed_terms(inner, root, terms, members)) return false;
            terms.push_back(leaf);
            members.push_back(index[leaf]);
            members.push_back(index[inner]);
            return true;
        }
        if (!leaf_ok(l) || !leaf_ok(r)) return false;
        terms.push_back(l);
        terms.push_back(r);
        members.push_back(index[l]);
        members.push_back(index[r]);
        return true;
    }
    // repeat_interleave_dim1 (Dia model.cpp:421-434): CONCAT(dim 1) over REPEAT(CONT(VIEW(a, slice i
    // of dim 1))) for i = 0..n-1 -> one pass, dst(i0, i1, i2, i3) = a(i0, i1 / r, i2, i3)
    void try_rint(int i) {
        const tts_tensor * R = nodes[i];
        if (R->type != TTS_TYPE_F32 || R->op_params[0] != 1 || !contiguous(R)) return;
        std::vector<const tts_tensor *> leaves;
        std::vector<int> members{i};
        const tts_tensor * t = R;
        while (t->op == TTS_OP_CONCAT && t->op_params[0] == 1) {
            leaves.push_back(t->src[1]);
            t = t->src[0];
            if (t->op == TTS_OP_CONCAT) {
                if (uses[t] != 1 || !index.count(t)) return;
                members.push_back(index[t]);
            }
        }
        leaves.push_back(t);
        std::reverse(leaves.begin(), leaves.end());
        const tts_tensor * a = nullptr;
        int64_t r = 0;
        for (size_t k = 0; k < leaves.size(); ++k) {
            const tts_tensor * rp = leaves[k];
            if (rp->op != TTS_OP_REPEAT || uses[rp] != 1 || !index.count(rp)) return;
            const tts_tensor * c = rp->src[0];
            if (!c || c->op != TTS_OP_CONT || uses[c] != 1 || !index.count(c)) return;
            const tts_tensor * v = c->src[0];
            if (!v || v->op != TTS_OP_VIEW || !v->view_src || v->ne[1] != 1) return;
            const tts_tensor * base = v->view_src;
            if (k == 0) {
                a = base;
                r = rp->ne[1];
                if (a->type != TTS_TYPE_F32 || (int64_t)leaves.size() != a->ne[1]) return;
            }
            if (base != a || rp->ne[1] != r || (const char *)v->data != (const char *)a->data + k * a->nb[1]) return;
            for (int d = 0; d < 4; ++d)
                if (d != 1 && (v->ne[d] != a->ne[d] || v->nb[d] != a->nb[d] || rp->ne[d] != a->ne[d])) return;
            members.push_back(index[rp]);
            members.push_back(index[c]);
        }
        if (!a || R->ne[1] != a->ne[1] * r || overlap(R, a)) return;
        for (int m : members)
            if (act[m] != 0) return;
        // a is read at R's position: nothing that still runs after a's first (skipped) reader may
        // have been given a's arena memory
        const int first = *std::min_element(members.begin(), members.end());
        for (int j = first + 1; j < i; ++j) {
            if (is_view(nodes[j]->op) || std::find(members.begin(), members.end(), j) != members.end()) continue;
            if (overlap(nodes[j], a)) return;
        }
        Item it;
        it.kind = Item::RINT;
        it.x = a;
        it.dst = R;
        it.rint = (int)r;
        for (int m : members) act[m] = -1;
        // input: a = CONT of a same-shape tensor (Dia's cont(reshape_4d(k / v))) whose every reader is
        // one of the leaves' views: read that tensor in place (TD strides) and skip the copy
        if (a->op == TTS_OP_CONT && a->src[0] && index.count(a) && act[index[a]] == 0) {
            const tts_tensor * s0 = a->src[0];
            bool ok = s0->type == TTS_TYPE_F32 && !overlap(R, s0);
            for (int d = 0; d < 4; ++d) ok &= s0->ne[d] == a->ne[d];
            auto ca = consumers.find(a);
            ok &= ca != consumers.end();
            if (ok)
                for (int k : ca->second) {
                    const tts_tensor * v = nodes[k];
                    const tts_tensor * u = sole_consumer(v);
                    ok &= v->op == TTS_OP_VIEW && u && std::find(members.begin(), members.end(), index[u]) != members.end();
                }
            const int ia = ok ? index[a] : 0;
            for (int j = ia + 1; ok && j < i; ++j) {
                if (is_view(nodes[j]->op) || std::find(members.begin(), members.end(), j) != members.end()) continue;
                if (overlap(nodes[j], s0)) ok = false;
            }
            if (ok) {
                it.x = s0;
                act[ia] = -1;
            }
        }
        // output: R only feeds a CPY into a cache view, directly or through a CONT of a reshape (Dia's
        // self K / V store, model.cpp:317-322 here): write the cache view in R's shape and skip both
        rint_to_cpy(i, R, it);
        act[i] = add_item(std::move(it));
    }

    // R [n0, n1, n2, n3] contiguous -> [RESHAPE ->] [CONT ->] CPY into D with D->ne[0] == n0 n1 n2 and
    // D->ne[1] == n3 (flat order: D(j0, j1) = R(i0, i1, i2, i3), j0 = i0 + n0 i1 + n0 n1 i2, j1 = i3):
    // the RINT writes D through a stand-in tensor with R's shape and D's strides (it.node)
    void rint_to_cpy(int i, const tts_tensor * R, Item & it) {
        const tts_tensor * X = sole_consumer(R);
        std::vector<int> skip;
        while (X && X->op == TTS_OP_RESHAPE && X->src[0] && contiguous(X)) X = sole_consumer(X);
        if (X && X->op == TTS_OP_CONT && contiguous(X) && index.count(X) && act[index[X]] == 0) {
            skip.push_back(index[X]);
            X = sole_consumer(X);
        }
        if (!X || X->op != TTS_OP_CPY || !index.count(X) || act[index[X]] != 0) return;
        const int iP = index[X];
        skip.push_back(iP);
        const tts_tensor * D = X;  // the CPY's result is its destination view
        if (D->type != TTS_TYPE_F32 || D->nb[0] != 4 || D->ne[0] != R->ne[0] * R->ne[1] * R->ne[2] || D->ne[1] != R->ne[3] ||
            D->ne[2] != 1 || D->ne[3] != 1 || overlap(D, it.x))
            return;
        for (int j = i + 1; j < iP; ++j)
            if (!is_view(nodes[j]->op) && std::find(skip.begin(), skip.end(), j) == skip.end()) return;
        tts_tensor t = *R;
        t.data = D->data;
        t.nb[0] = 4;
        t.nb[1] = 4 * R->ne[0];
        t.nb[2] = t.nb[1] * R->ne[1];
        t.nb[3] = D->nb[1];
        it.node = t;
        it.rint_cpy = true;
        for (int k : skip) act[k] = -1;
    }

    // CONT(TRANSPOSE(GET_ROWS(W, RESHAPE(CONT(V))))) with V a strided I32 view (DAC / SNAC quantizer
    // inputs, general_neural_audio_codec.cpp:166-172 after dac_build_audio_inputs' per-codebook view):
    // three launches of a few hundred bytes each -> one gather writing the transposed rows.  Copies only.
    void try_gather_t(int i) {
        const tts_tensor * C2 = nodes[i];
        const tts_tensor * Tv = C2->src[0];
        if (!Tv || Tv->op != TTS_OP_TRANSPOSE || C2->type != TTS_TYPE_F32 || !contiguous(C2) || uses[Tv] != 1) return;
        const tts_tensor * G = Tv->view_src ? Tv->view_src : Tv->src[0];
        if (!G || G->op != TTS_OP_GET_ROWS || !index.count(G) || act[index[G]] != 0 || uses[G] != 1 || G->type != TTS_TYPE_F32 ||
            !contiguous(G) || G->ne[2] * G->ne[3] != 1)
            return;
        const tts_tensor *W = G->src[0], *ix = G->src[1];
        if (!W || W->type != TTS_TYPE_F32 || W->nb[0] != 4 || W->ne[2] * W->ne[3] != 1 || !ix || ix->type != TTS_TYPE_I32) return;
        // ix: a RESHAPE view of C1 = CONT(V), or C1 itself
        const tts_tensor * C1 = ix->op == TTS_OP_RESHAPE ? (ix->view_src ? ix->view_src : ix->src[0]) : ix;
        if (ix != C1 && uses[ix] != 1) return;
        if (!C1 || C1->op != TTS_OP_CONT || !index.count(C1) || act[index[C1]] != 0 || uses[C1] != 1) return;
        const tts_tensor * V = C1->src[0];
        const int64_t T = G->ne[1];
        if (!V || V->type != TTS_TYPE_I32 || V->ne[0] != 1 || V->ne[1] * V->ne[2] * V->ne[3] != T || V->ne[2] * V->ne[3] != 1) return;
        if (C2->ne[0] != T || C2->ne[1] != G->ne[0] || overlap(C2, V) || overlap(C2, W)) return;
        Item it;
        it.kind = Item::EMBED;
        it.gather_t = true;
        it.dst = C2;
        it.w = W;
        it.gt_codes = V;
        act[index[C1]] = act[index[G]] = -1;
        act[i] = add_item(std::move(it));
    }

    void try_embed(int i) {
        const tts_tensor * R = nodes[i];
        if (!contiguous(R)) return;
        std::vector<const tts_tensor *> terms;
        std::vector<int> members;
        if (!embed_terms(R, R, terms, members) || terms.size() < 2 || terms.size() > (size_t)EMBED_MAX_TERMS) return;
        for (const tts_tensor * g : terms)
            if (overlap(R, g->src[0]) || overlap(R, g->src[1])) return;
        for (int m : members)
            if (act[m] != 0) return;
        Item it;
        it.kind = Item::EMBED;
        it.dst = R;
        it.terms = terms;
        for (int m : members) act[m] = -1;
        act[i] = add_item(std::move(it));
    }

    // orpheus_build_kv_store (Orpheus model.cpp:194-228): `repeat` CPYs of one source into strided
    // cache views, K's and V's interleaved.  All CPY consumers of the source run as one pass when
    // nothing but CPYs and views sits between the first and the last (the destinations are disjoint
    // cache views nobody reads in between).
    void try_mcpy(int i) {
        const tts_tensor * C = nodes[i];
        const tts_tensor * src = C->src[0];
        if (!src || src->type != TTS_TYPE_F32 || C->type != TTS_TYPE_F32) return;
        auto it = consumers.find(src);
        if (it == consumers.end() || it->second.size() < 2 || it->second.size() > 4) return;
        std::vector<int> idx(it->second.begin(), it->second.end());
        std::sort(idx.begin(), idx.end());
        if (idx[0] != i) return;
        for (int j : idx) {
            const tts_tensor * D = nodes[j];
            if (D->op != TTS_OP_CPY || D->src[0] != src || act[j] != 0 || D->type != TTS_TYPE_F32) return;
            for (int k = 0; k < 4; ++k)
                if (D->ne[k] != C->ne[k]) return;
        }
        // destinations: same shape and strides, bases interleaved inside one dim-1 period (the
        // repeat copies), so their element sets are disjoint although their byte spans overlap
        auto interleaved = [](const tts_tensor * a, const tts_tensor * b) {
            for (int k = 0; k < 4; ++k)
                if (a->nb[k] != b->nb[k]) return false;
            const int64_t d = std::llabs((const char *)a->data - (const char *)b->data);
            const int64_t run = a->ne[0] * (int64_t)a->nb[0], p1 = (int64_t)a->nb[1];
            if (a->nb[0] != 4 || d < run || d + run > p1) return false;
            for (int k = 2; k < 4; ++k)
                if (a->ne[k] > 1 && a->nb[k] % p1) return false;
            return true;
        };
        for (size_t a = 0; a < idx.size(); ++a) {
            if (overlap(nodes[idx[a]], src)) return;
            for (size_t b = a + 1; b < idx.size(); ++b)
                if (overlap(nodes[idx[a]], nodes[idx[b]]) && !interleaved(nodes[idx[a]], nodes[idx[b]])) return;
        }
        // between the copies: views, copies, or nodes a GEMV item planned before this one absorbed
        // (it ran earlier: act -1 with the product's launch at a lower position)
        for (int j = idx.front() + 1; j < idx.back(); ++j)
            if (!is_view(nodes[j]->op) && nodes[j]->op != TTS_OP_CPY && act[j] != -1) return;
        Item m;
        m.kind = Item::MCPY;
        m.x = src;
        // the source is a ROPE read only by these copies, with nothing but views since it ran (Orpheus'
        // rope(K) -> repeat copies into the cache, model.cpp:194-228): rotate straight into every copy,
        // and read a contiguous CONT's source the same way (the copy before the rope is never made)
        const auto only_views = [&](int a, int b) {
            for (int k = a + 1; k < b; ++k)
                if (!is_view(nodes[k]->op) || act[k] != 0) return false;
            return true;
        };
        if (src->op == TTS_OP_ROPE && act[index[src]] == 0 && uses[src] == (int)idx.size() && only_views(index[src], i)) {
            const tts_tensor * rs = src->src[0];
            bool ok = true;
            for (int d = 0; d < 4; ++d) ok &= rs->ne[d] == src->ne[d] && C->ne[d] == src->ne[d];
            for (int j : idx) ok &= !overlap(nodes[j], rs);
            if (ok) {
                m.rope = src;
                act[index[src]] = -1;
                if (rs->op == TTS_OP_CONT && act[index[rs]] == 0 && uses[rs] == 1 && rs->src[0] && rs->src[0]->type == rs->type &&
                    contiguous(rs) && contiguous(rs->src[0]) && only_views(index[rs], index[src])) {
                    bool ok2 = true;
                    for (int d = 0; d < 4; ++d) ok2 &= rs->src[0]->ne[d] == rs->ne[d];  // k_rope indexes by rs's shape
                    for (int j : idx) ok2 &= !overlap(nodes[j], rs->src[0]);
                    if (ok2) {
                        act[index[rs]] = -1;
                        rs = rs->src[0];
                    }
                }
                m.x = rs;
            }
        }
        for (int j : idx) {
            m.terms.push_back(nodes[j]);
            act[j] = -1;
        }
        act[i] = add_item(std::move(m));
    }

    void try_attn(int i) {
        const tts_tensor * S = nodes[i];
        const tts_tensor * KQ = S->src[0];
        const tts_tensor * mask = S->src[1];
        if (!KQ || KQ->op != TTS_OP_MUL_MAT || uses[KQ] != 1) return;
        if (opf(S, 1) != 0.0f) return;  // ALiBi not used by TTS graphs
        const tts_tensor * KQV = sole_consumer(S);
        if (!KQV || KQV->op != TTS_OP_MUL_MAT || KQV->src[0] != S) return;
        const tts_tensor * PERM = sole_consumer(KQV);
        if (!PERM || PERM->op != TTS_OP_PERMUTE || PERM->op_params[0] != 2 || PERM->op_params[1] != 0 || PERM->op_params[2] != 1 ||
            PERM->op_params[3] != 3)
            return;
        const tts_tensor * O = sole_consumer(PERM);
        if (!O || O->op != TTS_OP_CONT || !contiguous(O) || O->type != TTS_TYPE_F32) return;
        const tts_tensor * Ka = KQ->src[0];
        const tts_tensor * Qa = KQ->src[1];
        const tts_tensor * V = KQV->src[1];
        const tts_tensor * K = Ka;
        int skip_k = -1, skip_q = -1, skip_v = -1;
        // V = cont_{3,4}d(transpose(view of a [dims, positions] cache)) (Orpheus model.cpp:265-272): read the
        // transposed cache in place, V'(p, d, h, b) = T(p, d + hd*h, b); the per-step transpose copy disappears
        // folds only read tensors whose storage outlives the graph (caches, weights, inputs): an arena
        // tensor's memory may be handed to another node once its CONT consumer is skipped
        auto leaf_backed = [](const tts_tensor * t) {
            while (t->view_src) t = t->view_src;
            return t->op == TTS_OP_NONE;
        };
        if (V->op == TTS_OP_CONT && uses[V] == 1 && V->src[0] && V->src[0]->data && leaf_backed(V->src[0])) {
            const tts_tensor * T = V->src[0];
            if (T->ne[3] == 1 && V->ne[0] == T->ne[0] && V->ne[1] * V->ne[2] == T->ne[1] && V->ne[3] == T->ne[2] &&
                T->type == TTS_TYPE_F32 && V->type == TTS_TYPE_F32) {
                tts_tensor & d = derived.emplace_back(*V);
                d.op = TTS_OP_VIEW;
                d.data = T->data;
                d.nb[0] = T->nb[0];
                d.nb[1] = T->nb[1];
                d.nb[2] = T->nb[1] * V->ne[1];
                d.nb[3] = T->nb[2];
                d.view_src = T->view_src ? T->view_src : const_cast<tts_tensor *>(T);
                for (int k = 0; k < TTS_MAX_SRC; ++k) d.src[k] = nullptr;
                skip_v = index[V];
                V = &d;
            }
        }
        if (Ka->op == TTS_OP_CONT && uses[Ka] == 1) {
            K = Ka->src[0];
            skip_k = index[Ka];
        }
        // a same-shape CONT of a (permuted) cache view (Dia model.cpp:548,592: cont(cont(permute(view))))
        // is read in place too, so the attention never reads an arena copy its output may overlap
        int skip_k2 = -1, skip_v2 = -1;
        auto same_shape = [](const tts_tensor * a, const tts_tensor * b) {
            for (int d = 0; d < 4; ++d)
                if (a->ne[d] != b->ne[d]) return false;
            return true;
        };
        if (K->op == TTS_OP_CONT && uses[K] == 1 && K->src[0] && K->src[0]->data && same_shape(K, K->src[0]) && leaf_backed(K->src[0]) &&
            index.count(K)) {
            skip_k2 = index[K];
            K = K->src[0];
        }
        if (V->op == TTS_OP_CONT && uses[V] == 1 && V->src[0] && V->src[0]->data && same_shape(V, V->src[0]) && leaf_backed(V->src[0])) {
            skip_v2 = index[V];
            V = V->src[0];
        }
        const tts_tensor * Q = Qa;
        if (Qa->op == TTS_OP_CONT && uses[Qa] == 1) {
            Q = Qa->src[0];
            skip_q = index[Qa];
        }
        if (K->type != TTS_TYPE_F32 || Q->type != TTS_TYPE_F32 || V->type != TTS_TYPE_F32) return;
        const int64_t hd = Q->ne[0], P = K->ne[1];
        if (K->ne[0] != hd || hd % 4 || hd > 256 || P > 8192 || S->ne[0] != P || V->ne[0] != P || V->ne[1] != hd) return;
        if (Q->nb[0] != 4 || K->nb[0] != 4 || V->nb[0] % 4 || (skip_v < 0 && V->nb[0] != 4)) return;
        const int64_t H = Q->ne[2], nq = Q->ne[1], B = Q->ne[3];
        if (H % K->ne[2] || B % K->ne[3] || H % V->ne[2] || B % V->ne[3]) return;
        if (V->ne[2] != H || V->ne[3] != B) return;  // kqv = mul_mat(kq, V): V carries the batch dims
        if (mask && (mask->type != TTS_TYPE_F32 || !contiguous(mask) || mask->ne[0] < P)) return;
        if (mask && mask->ne[0] != P) return;  // ggml reads mask rows with stride ne00 == P
        // a 2-D mask serves every head and sequence; [P, rows, 1, B]: one per sequence (a ragged lock-step batch)
        if (mask && (mask->ne[1] < nq || mask->ne[2] != 1 || (mask->ne[3] != 1 && mask->ne[3] != B))) return;
        if (nq * H * B * hd != O->ne[0] * O->ne[1] * O->ne[2] * O->ne[3]) return;
        // aliasing: O may coincide exactly with Q's storage (read-before-write per workgroup), nothing else
        const tts_tensor * Qbase = Q->view_src ? Q->view_src : Q;
        if (overlap(O, K) || overlap(O, V) || (mask && overlap(O, mask))) return;
        if (overlap(O, Qbase) && O->data != Qbase->data) return;
        // a folded operand is read where its skipped CONT would have copied it from: no node that
        // still runs between that CONT and the attention (it launches at O) may write over it
        // (the arena can hand the source's memory on once its CONT consumer has "run")
        {
            const int io = index[O];
            const int mine[] = {i, index[KQ], index[KQV], index[PERM], skip_k, skip_q, skip_v, skip_k2, skip_v2};
            // span starts at the earliest skipped CONT that read the operand (the inner one of a chain)
            const std::pair<const tts_tensor *, int> folded[] = {
                {K, skip_k2 >= 0 ? skip_k2 : skip_k}, {Q, skip_q}, {V, skip_v >= 0 ? skip_v : skip_v2}};
            for (const auto & f : folded) {
                if (f.second < 0) continue;
                for (int j = f.second + 1; j < io; ++j) {
                    if (is_view(nodes[j]->op)) continue;  // (nodes folded into other items are written when those run)
                    bool own = false;
                    for (int m : mine) own |= m == j;
                    if (!own && overlap(nodes[j], f.first)) return;
                }
            }
        }
        Item it;
        it.kind = Item::ATTN;
        it.q = Q;
        it.k = K;
        it.v = V;
        it.mask = mask;
        it.out = O;
        it.scale = opf(S, 0);
        act[i] = -1;
        act[index[KQ]] = -1;
        act[index[KQV]] = -1;
        if (skip_k >= 0) act[skip_k] = -1;
        if (skip_q >= 0) act[skip_q] = -1;
        if (skip_v >= 0) act[skip_v] = -1;
        if (skip_k2 >= 0) act[skip_k2] = -1;
        if (skip_v2 >= 0) act[skip_v2] = -1;
        act[index[O]] = add_item(std::move(it));
    }
};

}  // namespace

// Backend scratch of at least `bytes` (eager launches only).  Prompt passes over many prompts stage
// column copies larger than the default 64 MiB (Parler, 64 prompts x 448 tokens x 4096: 470 MB): the
// buffer is re-allocated after the stream drains.  Recorded graphs hold the old address, so every
// cached step graph is dropped (re-recorded on its next call); with a prepared plan outstanding, or
// while recording, the buffer cannot move and the caller's fallback applies.
static bool ensure_scratch(tts_hip_backend * be, size_t bytes) {
    if (bytes <= be->scratch_size) return true;
    // a plan recorded but not launched yet holds the old address: the buffer cannot move
    if (be->stream == be->cap_stream || be->plan_prepared[0] || be->plan_prepared[1]) return false;
    TTS_HIP_CHECK(hipStreamSynchronize(be->stream));  // (every launched plan has run)
    for (int k = 0; k < tts_hip_backend::N_GSIG; ++k) {
        if (be->gsig_exec[k]) TTS_HIP_CHECK(hipGraphExecDestroy(be->gsig_exec[k]));
        be->gsig_exec[k] = nullptr;
        be->gsig[k] = 0;
    }
    for (int k = 0; k < 2; ++k) {  // launched plans recorded the old address: re-recorded by their next prepare
        if (be->pexec[k]) TTS_HIP_CHECK(hipGraphExecDestroy(be->pexec[k]));
        be->pexec[k] = nullptr;
        be->plan_ev_pending[k] = false;
    }
    const size_t n = (bytes + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
    char * p = nullptr;
    if (hipMalloc((void **)&p, n) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    TTS_HIP_CHECK(hipFree(be->scratch));
    be->scratch = p;
    be->scratch_size = n;
    be->aq.src = nullptr;
    return true;
}

// ---- activation preparation (cached per graph by src pointer) ----
static int prepare_act(tts_hip_backend * be, int wtype, const float * x, int64_t xcs, int64_t K, int64_t M, ActQuant & out) {
    ActQuant & aq = be->aq;
    if (wtype == TTS_TYPE_F32) {
        out = ActQuant();
        out.vtype = TTS_TYPE_F32;
        return 0;
    }
    const int vt = wtype == TTS_TYPE_Q4_K ? TTS_TYPE_Q8_K : wtype;
    const bool hit = aq.src == x && aq.K == K && aq.M == M && aq.vtype == vt && aq.graph_epoch == be->graph_epoch;
    if (!hit) {
        if (!ensure_scratch(be, act_quant_bytes(wtype, K, M))) return TTS_STATUS_ALLOC_FAILED;
        launch_quantize_act(be, wtype, x, xcs, K, M, aq);
        aq.src = x;
        aq.graph_epoch = be->graph_epoch;
    }
    out = aq;
    return 0;
}

static const void * weight_ptr(tts_hip_backend * be, const tts_tensor * a, bool tiled_copy = false) {
    if (tiled_copy) {
        const uint8_t * c = tiled_copy_find(a->data);
        if (!c) {
            fprintf(stderr, "tts_hip: missing tile-layout copy of %s\n", a->name);
            abort();
        }
        return c;
    }
    if (a->type != TTS_TYPE_Q4_K || (a->flags & TTS_FLAG_REPACKED)) return a->data;
    // Q4_K matrix written with plain tensor_set (native ggml layout): repack into a temp
    const size_t bytes = (size_t)a->nb[1] * (size_t)a->ne[1];
    if (be->repack_tmp_size < bytes) {
        // a bigger temp; the old one is retired, not freed: a recorded step graph (gsig_exec / pexec)
        // may still repack into it on replay, and this may run under stream capture, where neither a
        // stream synchronize nor hipFree (device-synchronizing) is allowed
        if (be->repack_tmp) be->repack_retired.push_back(be->repack_tmp);
        TTS_HIP_CHECK(hipMalloc((void **)&be->repack_tmp, bytes));
        be->repack_tmp_size = bytes;
    }
    launch_repack_q4_K(be, a->data, be->repack_tmp, (int64_t)(bytes / 144), 0);
    return be->repack_tmp;
}

// ---- coalesced steps (be->bat, coalesce.hip) ----
// Member 0's tensor -> its position in the graph: node i itself, its view source, or its source s.
// Member k's counterpart is the tensor at the same position of member k's graph (the graphs match
// node by node: same signature, checked item by item in co_prepare).
struct CoMap {
    PtrMap<int64_t> pos;  // (i << 5) | slot: 31 = node i, 30 = its view source, s = its src[s]
    void build(tts_tensor * const * nodes, int n) {
        pos.reserve((size_t)n * 3);
        for (int i = 0; i < n; ++i) pos[nodes[i]] = ((int64_t)i << 5) | 31;
        for (int i = 0; i < n; ++i) {
            const tts_tensor * t = nodes[i];
            if (t->view_src && !pos.find(t->view_src)) pos[t->view_src] = ((int64_t)i << 5) | 30;
            for (int s = 0; s < TTS_MAX_SRC; ++s)
                if (t->src[s] && !pos.find(t->src[s])) pos[t->src[s]] = ((int64_t)i << 5) | s;
        }
    }
    const tts_tensor * member(const BatchCtx & bc, const tts_tensor * t, int k) {
        if (k == 0 || !t) return t;
        auto * e = pos.find(t);
        if (!e) return nullptr;
        const int64_t c = e->second;
        const tts_tensor * nd = bc.mnodes[k][c >> 5];
        const int slot = (int)(c & 31);
        const tts_tensor * r = slot == 31 ? nd : slot == 30 ? nd->view_src : nd->src[slot];
        return r && r->op == t->op && r->type == t->type ? r : nullptr;
    }
};
static const tts_tensor * co_member(const BatchCtx & bc, const tts_tensor * t, int k) {
    return ((CoMap *)bc.comap)->member(bc, t, k);
}
// The tensor whose memory t is (a view's -- CPY included -- is its view source's, ggml's view_src).
static const tts_tensor * mem_root(const tts_tensor * t) { return t && t->view_src ? t->view_src : t; }
// memory that is each member's own and outlives the step: a leaf's (weights, caches, inputs) or a
// PERSIST tensor's, through any view (a KV-store CPY writes its cache's memory)
static bool owned_mem(const tts_tensor * t) {
    const tts_tensor * r = mem_root(t);
    return r && (r->op == TTS_OP_NONE || (r->flags & TTS_FLAG_PERSIST) || persistent_mem(r));
}
// memory of an input (a leaf marked input, through views): each member's own, never shared
static bool input_mem(const tts_tensor * t) {
    const tts_tensor * r = mem_root(t);
    return r && r->op == TTS_OP_NONE && (r->flags & TTS_FLAG_INPUT) != 0;
}

// An intermediate of member 0's graph as the N members' copies along dim 3 (member k's at executor
// memory win + k * stride); anything else is left as it is (stride 0: read by every member).
static void batch_td(const BatchCtx & bc, TD & t) {
    const int64_t s = bc.stride(t.data);
    t.data = bc.win(t.data);
    if (s) {
        t.ne[3] = bc.N;
        t.nb[3] = s;
    }
}
static int batch_n(const tts_hip_backend * be) { return be->bat ? be->bat->N : 1; }

static int run_attn_item(tts_hip_backend * be, const Item & it, const ItemTab * tab = nullptr) {
    TD q = make_td(it.q), k = make_td(it.k), v = make_td(it.v);
    float * out = (float *)it.out->data;
    const float * mask = it.mask ? (const float *)it.mask->data : nullptr;
    int B = (int)it.q->ne[3], P = (int)it.k->ne[1];
    int64_t obs = -1, mbs = it.mask && it.mask->ne[3] > 1 ? (int64_t)(it.mask->nb[3] / 4) : 0;  // per-sequence masks
    if (const BatchCtx * bc = be->bat) {  // (co_prepare-checked: one sequence per member)
        batch_td(*bc, q);
        if (tab && tab->koff) k.ne[3] = bc->N, k.nb[3] = 0;  // each member's own cache view: koff
        else batch_td(*bc, k);
        if (tab && tab->voff) v.ne[3] = bc->N, v.nb[3] = 0;
        else batch_td(*bc, v);
        obs = bc->stride(out) / 4;
        out = bc->win(out);
        if (mask && !(tab && tab->moff)) {
            mbs = bc->stride(mask) / 4;
            mask = bc->win(mask);
        }
        B = bc->N;
        if (tab && tab->pseq) P = tab->pmax;
    }
    float * out2 = it.shadow && tbytes(it.out) * (size_t)batch_n(be) <= be->shadow_size ? be->shadow : nullptr;
    launch_attn_decode(be, q, k, v, mask, it.scale, out, (int)it.q->ne[0], P, (int)it.q->ne[2], (int)it.q->ne[1], B, out2, obs, mbs,
                       tab ? tab->koff : nullptr, tab ? tab->voff : nullptr, tab ? tab->moff : nullptr, tab ? tab->pseq : nullptr);
    return 0;
}

static int run_gemv_item(tts_hip_backend * be, const Item & it, const Item * xattn = nullptr, const ItemTab * tab = nullptr,
                         const ItemTab * xtab = nullptr) {
    const tts_tensor * mm0 = it.mms[0];
    const tts_tensor * a0 = mm0->src[0];
    // a skipped CONT (it.xsrc): its contiguous source holds the same bytes; read them in src1's shape
    tts_tensor bx;
    if (it.xsrc) {
        bx = *mm0->src[1];
        bx.data = it.xsrc->data;
    }
    const tts_tensor * b = it.xsrc ? &bx : mm0->src[1];
    GemvJob j;
    j.wtype = a0->type;
    j.K = a0->ne[0];
    j.N = a0->ne[1];
    j.M = nel(b) / b->ne[0];
    j.w_row_bytes = (int64_t)a0->nb[1];
    j.x = (const float *)b->data;
    j.xcs = (int64_t)(b->nb[1] / 4);
    const BatchCtx * bc = be->bat;  // a coalesced step: M = 1 per member (planner-checked) -> N columns
    const int64_t NB = bc ? bc->N : 1;
    j.epi = it.epi;
    j.gelu = be->gelu_table;
    if (it.res) {
        j.res = (const float *)it.res->data;
        j.rcs = (int64_t)(it.res->nb[1] / 4);
    }
    // Q8_0 with <= 8 columns (K % 256 == 0): the same prologue, writing Q8_0 blocks (k_gemv_q8_0<MC, PRO>)
    const bool q80pro = j.wtype == TTS_TYPE_Q8_0 && j.K % QK_K == 0 && j.M <= 8 && (it.ln || be->gemv_q80_pro);
    if (j.wtype == TTS_TYPE_Q4_K || q80pro) {
        // the kernel quantizes (and normalizes) src1 itself in every workgroup
        j.pro = it.ln ? PRO_LN : PRO_QUANT;
        j.tiled = (a0->flags & TTS_FLAG_TILED) ? 1 : 0;
        if (it.ln) {
            j.x = (const float *)it.lnx->data;
            j.xcs = (int64_t)(it.lnx->nb[1] / 4);
            j.lnw = (const float *)it.lnw->data;
            j.lnb = it.lnb ? (const float *)it.lnb->data : nullptr;
            j.eps = it.lneps;
            j.rms = it.lnrms ? 1 : 0;
            j.lnout = (float *)it.lndst->data;
            j.locs = (int64_t)(it.lndst->nb[1] / 4);
        }
        // Outputs written while other workgroups still read src1 must not alias it (arena reuse can
        // place an epilogue / LN output on memory whose last reader is this item).
        auto span_y = [&](size_t k, const char *& y0, const char *& y1) {
            const tts_tensor * mm = it.mms[k];
            const int64_t Mm = mm->ne[1] * mm->ne[2] * mm->ne[3];
            y0 = (const char *)it.tgt[k].y;
            y1 = y0 + 4 * (size_t)((Mm - 1) * it.tgt[k].ycs + (mm->ne[0] - 1) * it.tgt[k].yrs + 1);
        };
        const bool xs = it.x_shadow && (size_t)(4 * j.K * j.M * NB) <= be->shadow_size;
        if (xs) {
            j.x = be->shadow;  // written by the preceding attention item (link_attn_shadow)
            j.xcs = j.K;
        }
        // aliasing on member 0's addresses (every member's buffers share one layout; members never alias)
        const char * x0 = (const char *)j.x;
        const char * x1 = x0 + 4 * (size_t)((j.M - 1) * j.xcs + j.K);
        const char * l0 = (const char *)j.lnout;
        const char * l1 = l0 ? l0 + 4 * (size_t)((j.M - 1) * j.locs + j.K) : nullptr;
        bool x_hit = l0 && l0 < x1 && x0 < l1;
        for (size_t k = 0; k < it.tgt.size(); ++k) {
            const char *y0, *y1;
            span_y(k, y0, y1);
            x_hit |= y0 < x1 && x0 < y1;
            if (l0 && y0 < l1 && l0 < y1) j.lnout = nullptr;  // LN output already dead: its memory is an output
        }
        if (bc) {  // member k = column k: window addresses, member stride as the column stride
            if (!xs) {
                j.xcs = bc->stride(j.x) / 4;
                j.x = bc->win(j.x);
            }
            if (j.lnout) {
                j.locs = bc->stride(j.lnout) / 4;
                j.lnout = bc->win(j.lnout);
            }
            j.M = NB;
        }
        // the prologue reads 16-B vectors: x 16-B aligned, columns 16-B strided
        x_hit |= ((uintptr_t)j.x & 15) != 0 || (j.xcs & 3) != 0;
        if (x_hit) {
            if (!ensure_scratch(be, (size_t)(4 * j.K * j.M))) return TTS_STATUS_ALLOC_FAILED;
            launch_copy_cols(be, (float *)be->scratch, j.x, j.K, j.xcs, j.M);
            be->aq.src = nullptr;
            j.x = (const float *)be->scratch;
            j.xcs = j.K;
        }
    } else {
        if (it.ln) return TTS_STATUS_UNSUPPORTED;  // planner invariant: a fused LN always runs as a prologue
        if (bc) {
            j.xcs = bc->stride(j.x) / 4;
            j.x = bc->win(j.x);
            j.M = NB;
        }
        int st = prepare_act(be, j.wtype, j.x, j.xcs, j.K, j.M, j.aq);
        if (st) return st;
    }
    if (bc && j.res) {
        j.rcs = bc->stride(j.res) / 4;
        j.res = bc->win(j.res);
    }
    // a Q4_K matrix in native layout goes through the one-matrix repack temp: launch it alone
    const bool tmp = a0->type == TTS_TYPE_Q4_K && !(a0->flags & TTS_FLAG_REPACKED);
    if (xattn) {
        const Item & A = *xattn;
        TD k = make_td(A.k), v = make_td(A.v);
        // aliasing on member 0's addresses (the x / LN-output spans of one member)
        const char * o0 = (const char *)A.out->data;
        const char * o1 = o0 + tbytes(A.out);
        const float * xm = bc ? (const float *)(it.ln ? it.lnx->data : b->data) : j.x;
        const int64_t xmcs = bc ? 0 : j.xcs, mm = bc ? 1 : j.M;
        const char * x0 = (const char *)xm;
        const char * x1 = x0 + 4 * (size_t)((mm - 1) * xmcs + j.K);
        const bool ok = !tmp && !j.tiled && j.wtype == TTS_TYPE_Q4_K && j.K <= 1024 && j.N == 64 * A.q->ne[2] && k.nb[0] == 4 &&
                        (k.nb[1] % 16) == 0 && (k.nb[2] % 16) == 0 && (k.nb[3] % 16) == 0 && ((uintptr_t)k.data % 16) == 0 &&
                        A.k->ne[1] >= 1 && A.k->ne[1] <= 64 && !(o0 < x1 && x0 < o1) && contiguous(A.out);
        if (ok) {
            GemvJob jj = j;
            jj.nmat = 1;
            jj.W[0] = (const uint8_t *)weight_ptr(be, a0);
            jj.Y[0] = nullptr;
            if (jj.lnout) {  // the LN output may already be dead and its memory the attention output
                const char * l0 = it.ln ? (const char *)it.lndst->data : (const char *)jj.lnout;
                const char * l1 = l0 + 4 * (size_t)((mm - 1) * (bc ? 0 : j.locs) + j.K);
                if (l0 < o1 && o0 < l1) jj.lnout = nullptr;
            }
            XAttnArgs xa;
            xa.k = k;
            xa.v = v;
            xa.mask = A.mask ? (const float *)A.mask->data : nullptr;
            xa.scale = A.scale;
            xa.out = (float *)A.out->data;
            xa.out2 = A.shadow && tbytes(A.out) * (size_t)NB <= be->shadow_size ? be->shadow : nullptr;
            xa.P = (int)A.k->ne[1];
            xa.H = (int)A.q->ne[2];
            xa.B = (int)A.q->ne[3];
            if (bc) {
                if (xtab && xtab->koff) xa.k.ne[3] = NB, xa.k.nb[3] = 0;  // each member's own cross K / V: offset tables
                else batch_td(*bc, xa.k);
                if (xtab && xtab->voff) xa.v.ne[3] = NB, xa.v.nb[3] = 0;
                else batch_td(*bc, xa.v);
                if (xtab && xtab->moff) {
                    xa.moff = xtab->moff;
                } else {
                    xa.mbs = bc->stride(xa.mask) / 4;
                    xa.mask = bc->win(xa.mask);
                }
                xa.koff = xtab ? xtab->koff : nullptr;
                xa.voff = xtab ? xtab->voff : nullptr;
                if (xtab && xtab->pseq) xa.pseq = xtab->pseq, xa.P = xtab->pmax;
                xa.obs = bc->stride(xa.out) / 4;
                xa.out = bc->win(xa.out);
                xa.B = (int)NB;
            }
            launch_gemv_q4K_xattn(be, jj, xa);
            return 0;
        }
    }
    // lane-layout matrices with tile-layout copies: GEMVs of >= 8 columns over >= 2048 rows of
    // K >= 2048 read the copies on the matrix-core kernels (enough 16-row tiles to fill the chip)
    // (a group holding a matrix stored tiled runs there whatever M is: that matrix has no other layout)
    bool all_tl = j.wtype == TTS_TYPE_Q4_K && !tmp, any_tiled = false;
    int64_t rows = 0;
    for (const tts_tensor * mm : it.mms) {
        const int f = mm->src[0]->flags;
        all_tl &= (f & (TTS_FLAG_TILED | TTS_FLAG_TILED_COPY)) != 0;
        any_tiled |= (f & TTS_FLAG_TILED) != 0;
        rows += mm->src[0]->ne[1];
    }
    // (K >= 2048: for K = 1024 rows the lane-layout kernels' short prologue wins)
    const bool use_copy = all_tl && (any_tiled || (j.M >= 8 && rows >= 2048 && j.K >= 2048));
    if (use_copy) j.tiled = 1;
    size_t k = 0;
    while (k < it.mms.size()) {
        GemvJob jj = j;
        jj.nmat = 0;
        jj.hetero = 0;
        jj.roff[0] = 0;
        if (bc && tab && tab->yoff) {  // members' own KV-cache rows: per-column store offsets ([target][N])
            jj.yoff = tab->yoff + k * NB;
            jj.yoff_ld = (int32_t)NB;
            jj.yoff_mats = (int32_t)((uint32_t)tab->yoff_mats >> k);
        }
        while (k < it.mms.size() && jj.nmat < GEMV_MAX_MATS) {
            const tts_tensor * a = it.mms[k]->src[0];
            // matrices of another row count share a launch only on the tile-layout kernels
            if (jj.nmat > 0 && a->ne[1] != jj.N && !jj.tiled) break;
            if (it.tgt[k].rg > 0 && jj.rep_mat >= 0) break;  // one repeat-copy target per launch
            if (jj.nmat > 0 && a->ne[1] != jj.N) jj.hetero = 1;
            jj.W[jj.nmat] = (const uint8_t *)weight_ptr(be, a, use_copy && !(a->flags & TTS_FLAG_TILED));
            jj.Y[jj.nmat] = bc ? bc->win(it.tgt[k].y) : it.tgt[k].y;
            jj.ycs[jj.nmat] = bc ? bc->stride(it.tgt[k].y) / 4 : it.tgt[k].ycs;
            jj.yrs[jj.nmat] = it.tgt[k].yrs;
            if (it.tgt[k].rg > 0) {
                jj.rep_mat = jj.nmat;
                jj.yrg = it.tgt[k].rg;
                jj.yrgs = it.tgt[k].rgs;
                jj.nrep = it.tgt[k].nrep;
                jj.yrep = it.tgt[k].rep;
            }
            if (jj.nmat == 0) jj.N = a->ne[1];
            jj.roff[jj.nmat + 1] = jj.roff[jj.nmat] + a->ne[1];
            jj.nmat++;
            k++;
            if (tmp) break;
        }
        if (jj.hetero) jj.N = 0;  // every row count comes from roff
        launch_gemv_job(be, jj);
    }
    if (xattn) return run_attn_item(be, *xattn, xtab);  // unfused fallback: the attention right after its query
    return 0;
}

// dst[c * T + t] = W[ids[t] row, c]: GET_ROWS of an I32 view, then the transpose's CONT (try_gather_t)
__global__ void k_gather_t(float * __restrict__ dst, const char * __restrict__ w, int64_t wnb1, const char * __restrict__ ids,
                           int64_t inb1, int64_t T, int64_t C) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * C; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = e / T, t = e - c * T;
        const int32_t id = *(const int32_t *)(ids + t * inb1);
        dst[e] = *(const float *)(w + (int64_t)id * wnb1 + 4 * c);
    }
}

static void launch_gather_t(tts_hip_backend * be, const tts_tensor * dst, const tts_tensor * w, const tts_tensor * ids) {
    const int64_t T = dst->ne[0], C = dst->ne[1];
    int64_t g = (T * C + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_gather_t, dim3((unsigned)g), dim3(256), 0, be->stream, (float *)dst->data, (const char *)w->data,
                       (int64_t)w->nb[1], (const char *)ids->data, (int64_t)ids->nb[1], T, C);
    TTS_HIP_CHECK(hipGetLastError());
}

static int run_node(tts_hip_backend * be, const tts_tensor * n);

// An intermediate of member 0's graph as the N members' copies along dim 3 (member k's at executor memory
// win + k * stride); read-only model data (stride 0) is left as it is and broadcast.
static bool batch_tensor(const BatchCtx & bc, const tts_tensor * t, tts_tensor & o) {
    o = *t;
    const int64_t s = bc.stride(t->data);
    o.data = bc.win(t->data);
    if (!s) return true;
    if (t->ne[3] != 1) return false;
    o.ne[3] = bc.N;
    o.nb[3] = (size_t)s;
    return true;
}

// An unfused node of a coalesced step (n: member 0's node).  Ops that act on every dim-3 slice on its
// own (elementwise with broadcasting, norms, copies, concat below dim 3) run once over the members'
// intermediates when no input or member-owned tensor is involved; any other node runs once per member,
// on that member's own tensors (inputs, caches) and its executor copies of the intermediates.
static int run_node_coalesced(tts_hip_backend * be, const tts_tensor * n) {
    const BatchCtx & bc = *be->bat;
    bool per_slice = false;
    switch (n->op) {
        case TTS_OP_ADD: case TTS_OP_SUB: case TTS_OP_MUL: case TTS_OP_DIV: case TTS_OP_SQR: case TTS_OP_SQRT: case TTS_OP_SIN:
        case TTS_OP_COS: case TTS_OP_SCALE: case TTS_OP_CLAMP: case TTS_OP_LEAKY_RELU: case TTS_OP_UNARY: case TTS_OP_ROUND:
        case TTS_OP_MOD: case TTS_OP_NORM: case TTS_OP_RMS_NORM: case TTS_OP_CONT: case TTS_OP_CPY: case TTS_OP_DUP:
            per_slice = true;
            break;
        case TTS_OP_CONCAT: per_slice = n->op_params[0] < 3; break;
        default: break;
    }
    tts_tensor t, srcs[TTS_MAX_SRC];
    if (per_slice && !owned_mem(n) && bc.stride(n->data) && batch_tensor(bc, n, t)) {
        for (int i = 0; i < TTS_MAX_SRC && per_slice; ++i) {
            const tts_tensor * x = n->src[i];
            if (!x) continue;
            // an input is each member's own; read-only model data (checked equal, co_prepare) broadcasts
            if (input_mem(x) || (!owned_mem(x) && !bc.stride(x->data))) {
                per_slice = false;
                break;
            }
            per_slice = batch_tensor(bc, x, srcs[i]);
            // a copy reads as many elements as it writes: its source must be per member too
            if ((n->op == TTS_OP_CONT || n->op == TTS_OP_CPY || n->op == TTS_OP_DUP) && !bc.stride(x->data)) per_slice = false;
            t.src[i] = &srcs[i];
        }
        if (per_slice) return launch_op(be, &t);
    }
    BatchCtx * keep = be->bat;
    be->bat = nullptr;  // member k's own node, run as in an uncoalesced step
    int st = 0;
    auto addr = [&](const tts_tensor * x, int k) -> void * {  // member k's bytes of member 0's tensor x
        if (!owned_mem(x)) return bc.reloc(x->data, k);
        const tts_tensor * m = co_member(bc, x, k);
        return m ? m->data : nullptr;
    };
    for (int k = 0; k < bc.N && st == 0; ++k) {
        t = *n;
        t.data = addr(n, k);
        for (int i = 0; i < TTS_MAX_SRC; ++i) {
            if (!n->src[i]) continue;
            srcs[i] = *n->src[i];
            srcs[i].data = addr(n->src[i], k);
            if (!srcs[i].data) st = TTS_STATUS_FAILED;
            t.src[i] = &srcs[i];
        }
        if (!t.data) st = TTS_STATUS_FAILED;
        if (st == 0) st = run_node(be, &t);
    }
    be->bat = keep;
    return st;
}

static int run_node(tts_hip_backend * be, const tts_tensor * n) {
    if (be->bat) return run_node_coalesced(be, n);
    if (n->op == TTS_OP_MUL_MAT) {
        const tts_tensor * a = n->src[0], * b = n->src[1];
        if (a->ne[0] != b->ne[0] || b->ne[2] % a->ne[2] || b->ne[3] % a->ne[3]) return TTS_STATUS_UNSUPPORTED;  // ggml_can_mul_mat
        if (is_gemv(n)) {
            Item it;
            it.kind = Item::GEMV;
            it.mms.push_back(n);
            it.tgt.push_back(GemvTarget{(float *)n->data, (int64_t)(n->nb[1] / 4), 1});
            it.tgt.back().yt = n;
            return run_gemv_item(be, it);
        }
        const int t = n->src[0]->type;
        if (t == TTS_TYPE_F32 || t == TTS_TYPE_F16) return launch_op(be, n);
        return TTS_STATUS_UNSUPPORTED;
    }
    return launch_op(be, n);
}

static int run_item(tts_hip_backend * be, const Item & it, const std::vector<Item> & items) {
    // a coalesced plan's tables of member-owned operands (co_prepare), by item index
    const ItemTab * tab = be->bat ? &be->bat->tabs[&it - items.data()] : nullptr;
    switch (it.kind) {
        case Item::GEMV:
            return run_gemv_item(be, it, it.xattn >= 0 ? &items[it.xattn] : nullptr, tab,
                                 be->bat && it.xattn >= 0 ? &be->bat->tabs[it.xattn] : nullptr);
        case Item::ATTN:
            if (it.fused) return 0;  // launched with its query GEMV
            return run_attn_item(be, it, tab);
        case Item::LN:
            if (be->bat) {  // rows of every member (planner-checked: one-row tensors of member buffers)
                tts_tensor d, x;
                if (!batch_tensor(*be->bat, it.dst, d) || !batch_tensor(*be->bat, it.x, x)) return TTS_STATUS_UNSUPPORTED;
                launch_layernorm(be, &d, &x, (const float *)it.w->data, it.b ? (const float *)it.b->data : nullptr, it.eps, it.rms);
                return 0;
            }
            launch_layernorm(be, it.dst, it.x, (const float *)it.w->data, it.b ? (const float *)it.b->data : nullptr, it.eps, it.rms);
            return 0;
        case Item::EMBED:
            if (it.gather_t) launch_gather_t(be, it.dst, it.w, it.gt_codes);
            else launch_embed_sum(be, it.dst, it.terms.data(), (int)it.terms.size(), be->bat, tab);
            return 0;
        case Item::SNAKE:
            launch_snake(be, it.dst, it.x, it.w, it.b, it.snake_one, it.snake_mask);
            return 0;
        case Item::CONV:
            launch_conv1d_fused(be, it.conv);
            return 0;
        case Item::ADAIN:
            launch_adain_snake(be, it.adain);
            return 0;
        case Item::MCPY:
            if (it.rope) launch_rope_multi(be, it.rope, it.x, it.terms.data(), (int)it.terms.size());
            else launch_cpy_multi(be, it.x, it.terms.data(), (int)it.terms.size());
            return 0;
        case Item::RINT:
            launch_repeat_interleave1(be, it.rint_cpy ? &it.node : it.dst, it.x, it.rint);
            return 0;
        case Item::NODE:
            return run_node(be, &it.node);
        case Item::COPY:
            launch_copy_bytes(be, it.cp_dst, it.cp_src, it.cp_bytes);
            return 0;
        case Item::LSTM:
            if (it.lkind & 4)
                for (int g = 0; g < 4; ++g)
                    launch_copy_bytes(be, it.lstash_dst[g], it.lstash_src[g], it.lstash_bytes);
            if (it.lkind & 1) {
                launch_lstm_step(be, it.ls, it.lpair ? &it.ls2 : nullptr);
                be->lstm_steps += it.lpair ? 2 : 1;
            }
            if (it.lkind & 2) {
                launch_lstm_finish(be, it.lfinal, it.lhist, it.lHd, it.lT);
                be->lstm_chains++;
                if (it.lfinal2) {
                    launch_lstm_finish(be, it.lfinal2, it.lhist2, it.lHd, it.lT);
                    be->lstm_chains++;
                }
            }
            return 0;
    }
    return TTS_STATUS_FAILED;
}

// TTS_HIP_COALESCE_DEBUG=1: why a coalesced step was refused (stderr), for diagnosing a group that never forms
bool tts::co_debug() {
    static const bool on = [] {
        const char * e = getenv("TTS_HIP_COALESCE_DEBUG");
        return e && e[0] == '1';
    }();
    return on;
}
#define CO_NO()                                                                                   \
    do {                                                                                          \
        if (tts::co_debug()) fprintf(stderr, "coalesce: step refused at graph_exec.hip:%d\n", __LINE__); \
        return false;                                                                             \
    } while (0)

// A node of a coalesced step launched once over every member's intermediates (run_node_coalesced's
// rule): a per-slice op whose output and sources are intermediates or read-only model data.
static bool co_per_slice(const BatchCtx & bc, const tts_tensor * n) {
    switch (n->op) {
        case TTS_OP_ADD: case TTS_OP_SUB: case TTS_OP_MUL: case TTS_OP_DIV: case TTS_OP_SQR: case TTS_OP_SQRT: case TTS_OP_SIN:
        case TTS_OP_COS: case TTS_OP_SCALE: case TTS_OP_CLAMP: case TTS_OP_LEAKY_RELU: case TTS_OP_UNARY: case TTS_OP_ROUND:
        case TTS_OP_MOD: case TTS_OP_NORM: case TTS_OP_RMS_NORM: case TTS_OP_CONT: case TTS_OP_CPY: case TTS_OP_DUP: break;
        case TTS_OP_CONCAT:
            if (n->op_params[0] < 3) break;
            return false;
        default: return false;
    }
    if (owned_mem(n) || !bc.stride(n->data) || n->ne[3] != 1) return false;
    for (int i = 0; i < TTS_MAX_SRC; ++i) {
        const tts_tensor * x = n->src[i];
        if (!x) continue;
        if (input_mem(x) || (!owned_mem(x) && !bc.stride(x->data))) return false;
        if (bc.stride(x->data) && x->ne[3] != 1) return false;
        if ((n->op == TTS_OP_CONT || n->op == TTS_OP_CPY || n->op == TTS_OP_DUP) && !bc.stride(x->data)) return false;
    }
    return true;
}

// Everything a coalesced step needs before its first launch, or false (nothing launched; each member
// then runs its own graph):
//  - every item has a batched form, with one column / sequence per member;
//  - member k's graph matches member 0's item by item: the same shapes everywhere except each
//    attention's key count (the members' KV lengths);
//  - the tables of member-owned operands (ItemTab, as offsets into `tab` until uploaded): each
//    member's KV-cache store rows, cache / cross views, masks and input indices;
//  - the read-only operands read through member 0's copy: (member 0's, member k's, bytes) pairs whose
//    bytes must be equal;
//  - the output copies: the graph's output intermediates, from the executor memory to each member's
//    own tensor (src, dst, bytes triples in `tab` at *scatter, *n_scatter of them).
static bool co_prepare(tts_hip_backend * be, Planner & pl, tts_tensor * const * nodes, int n_nodes,
                       std::vector<std::tuple<const void *, const void *, size_t>> & shared, std::vector<int64_t> & tab,
                       std::vector<std::array<int64_t, 5>> & offs, int64_t * scatter, int * n_scatter) {
    BatchCtx & bc = *be->bat;
    CoMap & cm = *(CoMap *)bc.comap;
    const int N = bc.N;
    auto same_ne = [](const tts_tensor * a, const tts_tensor * b) {
        return a && b && a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
    };
    auto inter = [&](const tts_tensor * t) { return t && !owned_mem(t) && bc.stride(t->data) != 0; };
    auto equal_all = [&](const tts_tensor * t) {  // every member's counterpart has t's shape
        if (bc.checked) return true;
        for (int k = 1; k < N; ++k)
            if (!same_ne(t, cm.member(bc, t, k))) return false;
        return true;
    };
    // read-only data read through member 0's copy: every member's copy equal to the set's canonical
    // member's (equality is transitive; the pairs stay the same whichever member plans, so they cache)
    auto share = [&](const tts_tensor * t) {
        if (!t || bc.checked) return true;
        const tts_tensor * tc = cm.member(bc, t, bc.canon);
        if (!same_ne(t, tc) || !tc->data) return false;
        for (int k = 0; k < N; ++k) {
            if (k == bc.canon) continue;
            const tts_tensor * m = cm.member(bc, t, k);
            if (!same_ne(t, m) || !m->data) return false;
            if (m->data != tc->data) shared.emplace_back(tc->data, m->data, tbytes(t));
        }
        return true;
    };
    auto alloc = [&](size_t n64) {
        const int64_t o = (int64_t)tab.size();
        tab.resize(tab.size() + n64, 0);
        return o;
    };
    // per-member byte offsets of member k's counterpart of t from t (null: not resolvable)
    auto offsets = [&](const tts_tensor * t, int64_t o, int64_t unit) {
        for (int k = 0; k < N; ++k) {
            const tts_tensor * m = cm.member(bc, t, k);
            if (!m || !m->data) return false;
            const int64_t d = (int64_t)((const char *)m->data - (const char *)t->data);
            if (d % unit) return false;
            tab[o + k] = d / unit;
        }
        return true;
    };
    bc.tabs.assign(pl.items.size(), ItemTab{});
    offs.assign(pl.items.size(), std::array<int64_t, 5>{-1, -1, -1, -1, -1});
    std::vector<std::array<int64_t, EMBED_MAX_TERMS>> ioffs(pl.items.size());
    for (auto & r : ioffs) r.fill(-1);
    for (int i = 0; i < n_nodes; ++i) {
        const int a = pl.act[i];
        const tts_tensor * nd = nodes[i];
        if (a < 0) continue;
        if (a == 0) {
            if (is_view(nd->op)) continue;
            if (!equal_all(nd)) CO_NO();
            for (int s2 = 0; s2 < TTS_MAX_SRC; ++s2)
                if (nd->src[s2] && !equal_all(nd->src[s2])) CO_NO();
            if (co_per_slice(bc, nd))
                for (int s2 = 0; s2 < TTS_MAX_SRC; ++s2)
                    if (nd->src[s2] && owned_mem(nd->src[s2]) && !share(nd->src[s2])) CO_NO();
            continue;
        }
        Item & it = pl.items[a - 1];
        ItemTab & tb = bc.tabs[a - 1];
        auto & of = offs[a - 1];
        switch (it.kind) {
            case Item::GEMV: {
                if (it.epi == EPI_SWIGLU || it.epi == EPI_SILU_MUL) CO_NO();
                const tts_tensor * x = it.mms[0]->src[1];
                if (nel(x) != x->ne[0]) CO_NO();  // one column per member
                const tts_tensor * xt = it.ln ? it.lnx : it.xsrc ? it.xsrc : x;
                if (!it.x_shadow && !inter(xt)) CO_NO();
                if (it.res && !inter(it.res)) CO_NO();
                if (it.ln && it.lndst && !inter(it.lndst)) CO_NO();
                if (it.ln && (!share(it.lnw) || !share(it.lnb))) CO_NO();
                bool owned = false;
                for (size_t k = 0; k < it.mms.size(); ++k) {
                    if (!equal_all(it.mms[k]) || !share(it.mms[k]->src[0])) CO_NO();
                    const GemvTarget & t = it.tgt[k];
                    if (!t.yt) CO_NO();  // backend scratch (a hoisted product): no per-member form
                    if (!owned_mem(t.yt)) {
                        if (!bc.stride(t.y)) CO_NO();
                        continue;
                    }
                    if (bc.stride(t.y)) CO_NO();  // member-owned memory inside a compute buffer: no uniform form
                    owned = true;
                }
                if (owned) {  // members' own cache rows (KV stores): [target][N] float offsets
                    of[0] = alloc(it.mms.size() * (size_t)N);
                    for (size_t k = 0; k < it.mms.size(); ++k) {
                        const GemvTarget & t = it.tgt[k];
                        if (!owned_mem(t.yt)) continue;
                        if (k >= 32 || !equal_all(t.yt) || !offsets(t.yt, of[0] + (int64_t)k * N, 4)) CO_NO();
                        tb.yoff_mats |= 1 << k;
                    }
                }
                break;
            }
            case Item::ATTN: {
                if (it.q->ne[3] != 1 || !inter(it.q) || !inter(it.out) || !equal_all(it.q) || !equal_all(it.out)) CO_NO();
                if (it.mask && it.mask->ne[2] * it.mask->ne[3] != 1) CO_NO();
                // each member's own key count; K [hd, P, Hk], V [P, hd, Hv] with the cache's strides
                of[3] = alloc(((size_t)N + 1) / 2);
                int * pseq = (int *)&tab[of[3]];
                int pmax = 0;
                bool ragged = false;
                for (int k = 0; k < N; ++k) {
                    const tts_tensor * mk = cm.member(bc, it.k, k);
                    const tts_tensor * mv = cm.member(bc, it.v, k);
                    if (!mk || !mv || mk->ne[0] != it.k->ne[0] || mk->ne[2] != it.k->ne[2] || mk->ne[3] != 1 || mv->ne[1] != it.v->ne[1] ||
                        mv->ne[2] != it.v->ne[2] || mv->ne[3] != 1 || mv->ne[0] != mk->ne[1] || mk->nb[1] != it.k->nb[1] ||
                        mk->nb[2] != it.k->nb[2] || mv->nb[1] != it.v->nb[1] || mv->nb[2] != it.v->nb[2] || mk->nb[0] != it.k->nb[0] ||
                        mv->nb[0] != it.v->nb[0])
                        CO_NO();
                    pseq = (int *)&tab[of[3]];  // (tab may have moved)
                    pseq[k] = (int)mk->ne[1];
                    pmax = std::max(pmax, (int)mk->ne[1]);
                    ragged |= mk->ne[1] != it.k->ne[1];
                    if (it.mask) {
                        const tts_tensor * mm = cm.member(bc, it.mask, k);
                        if (!mm || mm->ne[0] != mk->ne[1] || mm->ne[1] < it.q->ne[1]) CO_NO();
                    }
                }
                tb.pmax = pmax;
                bc.ragged |= ragged;
                for (int w = 0; w < 2; ++w) {  // K, V: an intermediate (equal lengths only) or each member's own view
                    const tts_tensor * kv = w ? it.v : it.k;
                    if (inter(kv)) {
                        if (ragged) CO_NO();
                        continue;
                    }
                    if (bc.stride(kv->data)) CO_NO();
                    of[1 + w] = alloc(N);
                    if (!offsets(kv, of[1 + w], 16)) CO_NO();  // 16-B aligned: the kernels' vector loads
                    for (int k = 0; k < N; ++k) tab[of[1 + w] + k] *= 16;
                }
                if (it.mask) {
                    if (inter(it.mask)) {
                        if (ragged) CO_NO();
                    } else {
                        of[4] = alloc(N);
                        if (!offsets(it.mask, of[4], 4)) CO_NO();
                    }
                }
                break;
            }
            case Item::LN:
                if (it.dst->ne[3] != 1 || it.x->ne[3] != 1 || !inter(it.dst) || !inter(it.x) || !equal_all(it.dst) || !equal_all(it.x)) CO_NO();
                if (!share(it.w) || !share(it.b)) CO_NO();
                break;
            case Item::EMBED:
                if (it.gather_t || it.dst->ne[1] * it.dst->ne[2] * it.dst->ne[3] != 1 || !inter(it.dst) || !equal_all(it.dst)) CO_NO();
                if (it.terms.size() > (size_t)EMBED_MAX_TERMS) CO_NO();
                for (size_t t = 0; t < it.terms.size(); ++t) {
                    const tts_tensor * g = it.terms[t];
                    if (g->ne[1] * g->ne[2] * g->ne[3] != 1 || !equal_all(g) || !share(g->src[0])) CO_NO();
                    const tts_tensor * idx = g->src[1];
                    if (inter(idx)) continue;
                    if (!input_mem(idx) || !equal_all(idx)) CO_NO();
                    ioffs[a - 1][t] = alloc(N);
                    if (!offsets(idx, ioffs[a - 1][t], 4)) CO_NO();
                }
                break;
            case Item::NODE: {
                // its node copy stands at the original's graph position (run_node_coalesced finds members' tensors by it)
                auto * e = cm.pos.find(nd);
                if (!e) CO_NO();
                cm.pos[&it.node] = e->second;
                if (!equal_all(nd)) CO_NO();
                for (int s2 = 0; s2 < TTS_MAX_SRC; ++s2) {
                    const tts_tensor * x = it.node.src[s2];
                    if (!x) continue;
                    if (!cm.pos.find(x) && owned_mem(x)) CO_NO();  // a stand-in over member-owned memory
                    if (cm.pos.find(x) && !equal_all(x)) CO_NO();
                }
                if (co_per_slice(bc, &it.node))
                    for (int s2 = 0; s2 < TTS_MAX_SRC; ++s2)
                        if (it.node.src[s2] && owned_mem(it.node.src[s2]) && !share(it.node.src[s2])) CO_NO();
                break;
            }
            default: CO_NO();  // LSTM / SNAKE / CONV / ADAIN / MCPY / RINT / COPY: vocoder and prefill items
        }
    }
    // the output intermediates back to every member: the last node and nodes marked output
    *n_scatter = 0;
    std::vector<const tts_tensor *> outs;
    for (int i = 0; i < n_nodes; ++i)
        if ((nodes[i]->flags & TTS_FLAG_OUTPUT) || i == n_nodes - 1) outs.push_back(nodes[i]);
    std::vector<std::array<int64_t, 3>> sc;
    for (const tts_tensor * o : outs) {
        if (owned_mem(o) || is_view(o->op)) continue;  // written in place per member (or a view of what is)
        if (!inter(o) || !contiguous(o) || (tbytes(o) & 3) || !equal_all(o)) CO_NO();
        for (int k = 0; k < N; ++k) {
            const tts_tensor * m = cm.member(bc, o, k);
            if (!m || !m->data || !contiguous(m)) CO_NO();
            sc.push_back({(int64_t)(uintptr_t)bc.reloc(o->data, k), (int64_t)(uintptr_t)m->data, (int64_t)tbytes(o)});
        }
    }
    if (!sc.empty()) {
        *scatter = alloc(3 * sc.size());
        for (size_t e = 0; e < sc.size(); ++e)
            for (int c = 0; c < 3; ++c) tab[*scatter + 3 * (int64_t)e + c] = sc[e][c];
        *n_scatter = (int)sc.size();
    }
    for (size_t a = 0; a < pl.items.size(); ++a)
        for (int t = 0; t < EMBED_MAX_TERMS; ++t)
            if (ioffs[a][t] >= 0) bc.tabs[a].ioff[t] = (const int64_t *)(intptr_t)(ioffs[a][t] + 1);  // offset + 1 until uploaded
    return true;
}

// A coalesced step's outputs also go to each member's pinned read-back buffer, in this stream's order
// after the step (member k's entries are k, k + N, ... of the output copies): the member's
// tts_hip_tensor_get of its logits is then a stream synchronize and a host memcpy, instead of N
// device-to-host copies issued by N threads one after another.
static void co_readback(tts_hip_backend * be, const std::vector<int64_t> & sc, int n_sc) {
    BatchCtx & bc = *be->bat;
    const int N = bc.N;
    if ((int)bc.mbe.size() != N) return;
    std::vector<size_t> need(N, 0), off(N, 0);
    for (int e = 0; e < n_sc; ++e) need[e % N] += ((size_t)sc[3 * e + 2] + 255) & ~(size_t)255;
    for (int k = 0; k < N; ++k) {
        tts_hip_backend * m = bc.mbe[k];
        m->rb_clear();
        if (need[k] <= m->rb_cap) continue;
        if (m->rb_host) {  // an earlier step's copy into it is ordered before this point of this stream
            TTS_HIP_CHECK(hipStreamSynchronize(be->stream));
            TTS_HIP_CHECK(hipHostFree(m->rb_host));
            m->rb_host = nullptr;
            m->rb_cap = 0;
        }
        if (hipHostMalloc((void **)&m->rb_host, need[k], hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            m->rb_host = nullptr;
            continue;
        }
        m->rb_cap = need[k];
    }
    for (int e = 0; e < n_sc; ++e) {
        const int k = e % N;
        tts_hip_backend * m = bc.mbe[k];
        if (!m->rb_host) continue;
        const size_t bytes = (size_t)sc[3 * e + 2];
        TTS_HIP_CHECK(hipMemcpyAsync(m->rb_host + off[k], (const void *)(uintptr_t)sc[3 * e], bytes, hipMemcpyDeviceToHost, be->stream));
        std::lock_guard<std::mutex> l(m->rb_mu);
        m->rb.push_back({(const char *)(uintptr_t)sc[3 * e + 1], bytes, off[k]});
        m->rb_any.store(true, std::memory_order_release);
        off[k] += (bytes + 255) & ~(size_t)255;
    }
}

// A coalesced step's output copies: entry e = (src, dst, bytes), one workgroup row per entry.
__global__ void k_co_scatter(const int64_t * __restrict__ tab, int n) {
    const int e = blockIdx.y;
    if (e >= n) return;
    const uint32_t * src = (const uint32_t *)(uintptr_t)tab[3 * e];
    uint32_t * dst = (uint32_t *)(uintptr_t)tab[3 * e + 1];
    const int64_t w = tab[3 * e + 2] / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < w; i += (int64_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

// Replay through a HIP graph only for step-sized graphs: prompt-sized ones (many activation
// columns) run once and are launched directly.
static bool capture_worthy(tts_hip_backend * be, tts_tensor * const * nodes, int n_nodes) {
    if (!be->use_graphs || be->profile_gemv) return false;
    for (int i = 0; i < n_nodes; ++i) {
        const tts_tensor * t = nodes[i];
        // prefill-sized products (more than 64 columns per matrix) run once: not worth recording.
        // Decode attention's batched q.K / p.V products have one column per (head, prompt).
        if (t->op == TTS_OP_MUL_MAT && t->src[1] && t->src[1]->ne[1] > 64) return false;
    }
    return true;
}

// Record the graph's launches into `ex` without running them.  Topology is stable from step to
// step (only shapes/offsets move with the KV length), so the executable graph is updated in place
// (hipGraphExecUpdate) and re-instantiated only when that fails.
static int capture_into(tts_hip_backend * be, tts_tensor * const * nodes, int n_nodes, hipGraphExec_t & ex) {
    // record on a stream of its own: beginning a capture on the compute stream would first wait
    // for the step still running there, and the whole point of a prepared plan is to overlap it
    hipStream_t run = be->stream;
    be->stream = be->cap_stream;
    const auto t0 = std::chrono::steady_clock::now();
    TTS_HIP_CHECK(hipStreamBeginCapture(be->stream, hipStreamCaptureModeThreadLocal));
    const int st = graph_compute_launches(be, nodes, n_nodes);
    hipGraph_t graph = nullptr;
    TTS_HIP_CHECK(hipStreamEndCapture(be->stream, &graph));
    be->stream = run;
    const auto t1 = std::chrono::steady_clock::now();
    be->cap_launch_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    if (st != 0) {
        if (graph) hipGraphDestroy(graph);
        return st;
    }
    bool ok = false;
    if (ex) {
        hipGraphNode_t err_node = nullptr;
        hipGraphExecUpdateResult res;
        ok = hipGraphExecUpdate(ex, graph, &err_node, &res) == hipSuccess && res == hipGraphExecUpdateSuccess;
        if (ok) be->graph_updates++;
        else {
            (void)hipGetLastError();
            TTS_HIP_CHECK(hipGraphExecDestroy(ex));
            ex = nullptr;
        }
    }
    if (!ok) {
        TTS_HIP_CHECK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
        be->graph_instantiations++;
    }
    TTS_HIP_CHECK(hipGraphDestroy(graph));
    be->cap_update_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t1).count();
    return 0;
}

extern "C" int tts_hip_graph_compute(tts_hip_backend_t be, tts_tensor * const * nodes, int n_nodes) {
    if (!be) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();  // this step may write what the last coalesced step's read-back holds
    // a one-prompt decode step other backends on this device are also submitting: one coalesced launch
    const int cs = coalesce_submit(be, nodes, n_nodes);
    if (cs != kCoalesceNotTaken) return cs;
    // Recording pays off when the same graph comes back (a decode step): the first call of a
    // shape launches eagerly, so one-shot graphs (a Kokoro prompt's duration / synthesis graphs,
    // whose sizes follow the prompt) never pay for a capture and an instantiation.
    // signature: node count + every node's op + the first and last nodes' shapes (a decode step's
    // graph repeats with the same topology; its data pointers may move, exec update handles that)
    uint64_t sig = 0x9E3779B97F4A7C15ull ^ (uint64_t)n_nodes;
    for (int i = 0; i < n_nodes; ++i) sig = (sig ^ (uint64_t)nodes[i]->op) * 0x100000001B3ull;
    if (n_nodes > 0)
        for (int d = 0; d < 4; ++d)
            sig = (sig ^ (uint64_t)nodes[0]->ne[d] ^ ((uint64_t)nodes[n_nodes - 1]->ne[d] << 32)) * 0x100000001B3ull;
    sig |= 1;  // 0 = empty slot
    int slot = -1;
    for (int k = 0; k < tts_hip_backend::N_GSIG; ++k)
        if (be->gsig[k] == sig) slot = k;
    if (slot < 0) {  // first sighting: launch eagerly, remember the shape
        slot = be->gsig_next;
        be->gsig_next = (be->gsig_next + 1) % tts_hip_backend::N_GSIG;
        be->gsig[slot] = sig;
        if (be->gsig_exec[slot]) {
            TTS_HIP_CHECK(hipGraphExecDestroy(be->gsig_exec[slot]));
            be->gsig_exec[slot] = nullptr;
        }
        return graph_compute_launches(be, nodes, n_nodes);
    }
    if (!capture_worthy(be, nodes, n_nodes)) return graph_compute_launches(be, nodes, n_nodes);
    // the step's launches replay back to back on the device instead of at the host's launch rate
    const int st = capture_into(be, nodes, n_nodes, be->gsig_exec[slot]);
    if (st != 0) return st;
    TTS_HIP_CHECK(hipGraphLaunch(be->gsig_exec[slot], be->stream));
    return 0;
}

// graph_plan_create / graph_plan_compute: record now, launch later.  A plan slot holds either a
// recorded HIP graph or (graphs off / prompt-sized graphs) the node list, launched eagerly by
// tts_hip_graph_launch -- so the node array must stay alive until then.
extern "C" int tts_hip_graph_prepare(tts_hip_backend_t be, tts_tensor * const * nodes, int n_nodes, int slot) {
    if (!be || slot < 0 || slot > 1) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();
    if (be->plan_ev_pending[slot]) {  // the slot's previous launch must have run before it is re-recorded
        const auto t0 = std::chrono::steady_clock::now();
        TTS_HIP_CHECK(hipEventSynchronize(be->plan_ev[slot]));
        be->plan_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        be->plan_ev_pending[slot] = false;
    }
    be->plan_nodes[slot] = nodes;
    be->plan_n[slot] = n_nodes;
    be->plan_eager[slot] = !capture_worthy(be, nodes, n_nodes);
    if (be->plan_eager[slot]) return 0;
    const int st = capture_into(be, nodes, n_nodes, be->pexec[slot]);
    be->plan_prepared[slot] = st == 0;
    return st;
}

extern "C" int tts_hip_graph_launch(tts_hip_backend_t be, int slot) {
    if (!be || slot < 0 || slot > 1) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();
    if (be->plan_eager[slot]) {
        const int st = graph_compute_launches(be, be->plan_nodes[slot], be->plan_n[slot]);
        if (st != 0) return st;
    } else {
        if (!be->pexec[slot]) return TTS_STATUS_BAD_ARG;
        TTS_HIP_CHECK(hipGraphLaunch(be->pexec[slot], be->stream));
        be->plan_prepared[slot] = false;
    }
    TTS_HIP_CHECK(hipEventRecord(be->plan_ev[slot], be->stream));
    be->plan_ev_pending[slot] = true;
    return 0;
}

// Fusion coverage of a graph without a device (tests, tooling): counts[k] = items of kind k
// (Item::Kind order), counts[12] = MUL_MATs inside GEMV items, counts[13] = the most in one item,
// counts[14] = attention items folded into their query GEMV (TTS_FUSE_XATTN), counts[15] = nodes still
// launched one by one.  Returns the item count.
extern "C" int tts_hip_plan_stats(tts_tensor * const * nodes, int n_nodes, int mask, int32_t * counts) {
    Planner pl;
    pl.mask = mask;
    pl.vec_cap = 1u << 18;
    // the LSTM scratch is only addressed, never touched, while planning: a stand-in base with the
    // backend's capacity lets the stats see the fusions a device run makes
    static float lstm_stand_in alignas(256);
    pl.lstm_buf = &lstm_stand_in;
    pl.lstm_cap = (size_t)4 << 20;
    static float conv_stand_in alignas(256);
    pl.conv_stage = &conv_stand_in;
    pl.conv_stage_cap = (size_t)8 << 20;
    static char hoist_stand_in alignas(256);
    pl.hoist_buf = &hoist_stand_in;
    pl.hoist_cap = (size_t)8 << 20;
    if (mask) pl.build(nodes, n_nodes);
    else pl.act.assign(n_nodes, 0);
    for (int k = 0; k < 16; ++k) counts[k] = 0;  // (NODE items count under counts[10])
    for (const Item & it : pl.items) {
        counts[(int)it.kind]++;
        if (it.xattn >= 0) counts[14]++;
        if (it.kind == Item::GEMV) {
            counts[12] += (int32_t)it.mms.size();  // products in GEMV launches
            if ((int32_t)it.mms.size() > counts[13]) counts[13] = (int32_t)it.mms.size();
        }
    }
    static const bool dump = getenv("TTS_PLAN_DUMP") != nullptr;  // list the nodes launched one by one
    if (dump)
        for (int i = 0; i < n_nodes; ++i)
            if (pl.act[i] > 0) {
                const Item & it = pl.items[pl.act[i] - 1];
                fprintf(stderr, "item %d kind %d", i, (int)it.kind);
                if (it.kind == Item::GEMV)
                    fprintf(stderr, " mms %d K %lld N %lld M %lld epi %d ln %d", (int)it.mms.size(), (long long)it.mms[0]->src[0]->ne[0],
                            (long long)it.mms[0]->src[0]->ne[1], (long long)(nel(it.mms[0]->src[1]) / it.mms[0]->src[1]->ne[0]), it.epi, (int)it.ln);
                if (it.kind == Item::COPY) fprintf(stderr, " bytes %zu", it.cp_bytes);
                fprintf(stderr, "\n");
            }
    for (int i = 0; i < n_nodes; ++i)
        if (pl.act[i] == 0 && !is_view(nodes[i]->op)) {
            counts[15]++;
            if (dump)
                fprintf(stderr, "unfused %d op %d [%lld %lld %lld %lld] %s <- %s\n", i, (int)nodes[i]->op, (long long)nodes[i]->ne[0],
                        (long long)nodes[i]->ne[1], (long long)nodes[i]->ne[2], (long long)nodes[i]->ne[3], nodes[i]->name,
                        nodes[i]->src[0] ? nodes[i]->src[0]->name : "");
        }
    return (int)pl.items.size();
}

namespace tts {
// The planner's view of a backend: fusion mask and the backend scratch its items may target.
static void plan_setup(Planner & pl, const tts_hip_backend * be) {
    pl.mask = be->fusion;
    pl.q80pro = be->gemv_q80_pro != 0;
    pl.lstm_buf = be->lstm_buf;
    pl.lstm_cap = be->lstm_floats;
    pl.vec_cap = be->vec_scratch ? (1u << 18) : 0;
    pl.conv_stage = be->conv_stage;
    pl.conv_stage_cap = be->conv_stage_floats;
    pl.hoist_buf = (char *)be->hoist;
    pl.hoist_cap = be->hoist_size;
}

int graph_compute_launches(tts_hip_backend_t be, tts_tensor * const * nodes, int n_nodes) {
    be->graph_epoch++;
    be->aq.src = nullptr;
    if (be->profile_gemv) launch_profile_spin(be, 4000.0);  // see launch_profile_spin (k_gemv.hip)
    const auto tp0 = std::chrono::steady_clock::now();
    Planner pl;
    plan_setup(pl, be);
    if (be->fusion) pl.build(nodes, n_nodes);
    else pl.act.assign(n_nodes, 0);
    be->cap_plan_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tp0).count();
    // a coalesced step: checks, the member-owned operand tables (uploaded before any launch) and the
    // output copies (co_prepare)
    CoMap cm;
    int64_t sc_off = -1;
    int n_sc = 0;
    std::vector<int64_t> sc_host;  // the output copies (src, dst, bytes), member k's at entries k, k + N, ...
    if (be->bat) {
        const auto tq0 = std::chrono::steady_clock::now();
        struct Acc {
            tts_hip_backend * be;
            std::chrono::steady_clock::time_point t0;
            ~Acc() { be->co_prep_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(); }
        } acc{be, tq0};
        BatchCtx & bc = *be->bat;
        cm.build(nodes, n_nodes);
        bc.comap = &cm;
        std::vector<std::tuple<const void *, const void *, size_t>> shared;
        std::vector<int64_t> tab;
        std::vector<std::array<int64_t, 5>> offs;
        if (!co_prepare(be, pl, nodes, n_nodes, shared, tab, offs, &sc_off, &n_sc)) {
            bc.comap = nullptr;
            return TTS_STATUS_UNSUPPORTED;
        }
        if (!coalesce_check_shared(be, shared)) {
            bc.differs = true;
            bc.comap = nullptr;
            return TTS_STATUS_UNSUPPORTED;
        }
        if (n_sc > 0) sc_host.assign(tab.begin() + sc_off, tab.begin() + sc_off + 3 * (int64_t)n_sc);
        if (!tab.empty()) {
            const size_t bytes = tab.size() * sizeof(int64_t);
            if (bytes > be->co_tab_bytes) {
                TTS_HIP_CHECK(hipStreamSynchronize(be->stream));  // the previous tables may still be read
                if (be->co_tab) TTS_HIP_CHECK(hipFree(be->co_tab));
                be->co_tab_bytes = std::max(bytes * 2, (size_t)64 << 10);
                TTS_HIP_CHECK(hipMalloc((void **)&be->co_tab, be->co_tab_bytes));
            }
            if (tts_hip_tensor_set_async(be, be->co_tab, tab.data(), bytes) != 0) {
                bc.comap = nullptr;
                return TTS_STATUS_UNSUPPORTED;
            }
        }
        for (size_t a = 0; a < pl.items.size(); ++a) {
            ItemTab & tb = bc.tabs[a];
            const auto & of = offs[a];
            tb.yoff = of[0] >= 0 ? be->co_tab + of[0] : nullptr;
            tb.koff = of[1] >= 0 ? be->co_tab + of[1] : nullptr;
            tb.voff = of[2] >= 0 ? be->co_tab + of[2] : nullptr;
            tb.pseq = of[3] >= 0 ? (const int *)(be->co_tab + of[3]) : nullptr;
            tb.moff = of[4] >= 0 ? be->co_tab + of[4] : nullptr;
            for (auto & io : tb.ioff)
                if (io) io = be->co_tab + ((intptr_t)io - 1);
        }
    }
    // long-context attention items in launch order: each one's K/V is prefetched into MALL on the
    // side stream right after the previous one ran (fork), and joined just before it runs
    std::vector<int> pf_items;
    if (be->fusion && be->kv_prefetch_minp > 0) {
        for (int i = 0; i < n_nodes; ++i) {
            const int a = pl.act[i];
            if (a > 0 && pl.items[a - 1].kind == Item::ATTN && pl.items[a - 1].k->ne[1] >= be->kv_prefetch_minp) pf_items.push_back(a - 1);
        }
    }
    size_t pf_next = 0;
    int pf_pending = -1;  // item whose prefetch was forked and not yet joined
    auto pf_fork = [&]() {
        if (pf_next >= pf_items.size()) return;
        const Item & t = pl.items[pf_items[pf_next]];
        TTS_HIP_CHECK(hipEventRecord(be->pf_fork, be->stream));
        TTS_HIP_CHECK(hipStreamWaitEvent(be->pf_stream, be->pf_fork, 0));
        launch_kv_prefetch(be, be->pf_stream, make_td(t.k), 1, be->kv_prefetch_blocks);
        launch_kv_prefetch(be, be->pf_stream, make_td(t.v), 0, be->kv_prefetch_blocks);
        TTS_HIP_CHECK(hipEventRecord(be->pf_join, be->pf_stream));
        pf_pending = pf_items[pf_next];
    };
    pf_fork();
    for (int i = 0; i < n_nodes; ++i) {
        tts_tensor * n = nodes[i];
        const int a = be->fusion ? pl.act[i] : 0;
        if (a < 0) continue;
        if (a == 0 && is_view(n->op)) continue;
        const bool is_pf = a > 0 && pf_pending == a - 1;
        if (is_pf) {
            TTS_HIP_CHECK(hipStreamWaitEvent(be->stream, be->pf_join, 0));
            pf_pending = -1;
        }
        const int st = a > 0 ? run_item(be, pl.items[a - 1], pl.items) : run_node(be, n);
        if (is_pf) {
            ++pf_next;
            pf_fork();
        }
        if (st != 0) {
            fprintf(stderr, "tts_hip_graph_compute: node %d (%s, %s) failed: %d\n", i, n->name, tts_op_name(n->op), st);
            if (pf_pending >= 0) (void)hipStreamWaitEvent(be->stream, be->pf_join, 0);
            return st;
        }
        // The Q8_K activation cache is keyed by address and the graph reuses freed memory, so it
        // survives only launches that cannot have written over the cached source: an LN that
        // just produced it, or GEMVs whose outputs do not overlap it.
        // (a coalesced step keys the cache by window addresses, the items below by member 0's: no reuse)
        if (be->bat) be->aq.src = nullptr;
        if (be->aq.src) {
            const char * s0 = (const char *)be->aq.src;
            const char * s1 = s0 + (size_t)be->aq.K * (size_t)be->aq.M * 4;
            bool keep = false;
            if (a > 0) {
                const Item & it = pl.items[a - 1];
                if (it.kind == Item::GEMV) {
                    keep = true;
                    for (size_t k = 0; k < it.tgt.size(); ++k) {
                        const char * y0 = (const char *)it.tgt[k].y;
                        const tts_tensor * mm = it.mms[k];
                        const int64_t Mm = mm->ne[1] * mm->ne[2] * mm->ne[3];
                        const char * y1 = y0 + 4 * (size_t)((Mm - 1) * it.tgt[k].ycs + (mm->ne[0] - 1) * it.tgt[k].yrs + 1);
                        if (y0 < s1 && s0 < y1) keep = false;
                    }
                }
            } else if (n->op == TTS_OP_MUL_MAT) {
                const char * y0 = (const char *)n->data;
                keep = !(y0 < s1 && s0 < y0 + tbytes(n));
            }
            if (!keep) be->aq.src = nullptr;
        }
    }
    if (pf_pending >= 0) TTS_HIP_CHECK(hipStreamWaitEvent(be->stream, be->pf_join, 0));  // every fork rejoins
    if (be->bat) {
        if (n_sc > 0) {  // the output intermediates to every member's own tensors
            hipLaunchKernelGGL(k_co_scatter, dim3(4, (unsigned)n_sc), dim3(256), 0, be->stream, (const int64_t *)be->co_tab + sc_off, n_sc);
            TTS_HIP_CHECK(hipGetLastError());
            co_readback(be, sc_host, n_sc);
        }
        be->bat->comap = nullptr;
    }
    return 0;
}
}  // namespace tts

extern "C" int tts_hip_gemv(tts_hip_backend_t be, int type, const void * w, const float * x, float * y, int64_t K, int64_t N,
                            int64_t M) {
    return tts_hip_gemv_ex(be, type, w, x, y, K, N, M, 0);
}

extern "C" int tts_hip_gemv_ex(tts_hip_backend_t be, int type, const void * w, const float * x, float * y, int64_t K, int64_t N,
                               int64_t M, int32_t wflags) {
    if (!be) return TTS_STATUS_BAD_ARG;
    if ((wflags & TTS_FLAG_TILED) && (type != TTS_TYPE_Q4_K || N % 4)) return TTS_STATUS_BAD_ARG;
    if (type == TTS_TYPE_Q4_K && K % 256) return TTS_STATUS_BAD_ARG;
    if (type == TTS_TYPE_Q8_0 && K % 32) return TTS_STATUS_BAD_ARG;
    if (type != TTS_TYPE_Q4_K && type != TTS_TYPE_Q8_0 && type != TTS_TYPE_F16 && type != TTS_TYPE_F32) return TTS_STATUS_UNSUPPORTED;
    if ((type == TTS_TYPE_F32 || type == TTS_TYPE_F16) && K % 4) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    GemvJob j;
    j.wtype = type;
    j.K = K;
    j.N = N;
    j.M = M;
    j.w_row_bytes = (int64_t)tts_row_size(type, K);
    j.W[0] = (const uint8_t *)w;
    j.Y[0] = y;
    j.ycs[0] = N;
    j.yrs[0] = 1;
    j.x = x;
    j.xcs = K;
    const bool q80pro = type == TTS_TYPE_Q8_0 && K % QK_K == 0 && M <= 8 && be->gemv_q80_pro;
    if (type == TTS_TYPE_Q4_K || q80pro) {
        j.pro = PRO_QUANT;
        j.tiled = (wflags & TTS_FLAG_TILED) ? 1 : 0;
        if ((uintptr_t)x & 15) {  // the prologue reads 16-B vectors
            if ((size_t)(4 * K * M) > be->scratch_size) return TTS_STATUS_ALLOC_FAILED;
            launch_copy_cols(be, (float *)be->scratch, x, K, K, M);
            be->aq.src = nullptr;
            j.x = (const float *)be->scratch;
        }
    } else if (type != TTS_TYPE_F32) {
        if (act_quant_bytes(type, K, M) > be->scratch_size) return TTS_STATUS_ALLOC_FAILED;
        launch_quantize_act(be, type, x, K, K, M, j.aq);
    } else {
        j.aq.vtype = TTS_TYPE_F32;
    }
    be->aq.src = nullptr;  // scratch overwritten
    launch_gemv_job(be, j);
    return 0;
}
