// Orpheus-3B decoder runner: builds the same per-step graph as orpheus_runner::build_orpheus_graph
// (/root/reference/src/models/orpheus/model.cpp:230-311), stores K/V with the reference's
// repeat-interleave copies (orpheus_build_kv_store, :194-228), builds the causal mask like
// build_attn_mask / set_inputs (:127-131, 344-352) and samples greedily (sampler::max,
// /root/reference/src/sampler.cpp:185-204) in the generate_from_batch loop (:381-396).
//
// Extension (batch > 1): B independent prompts stepped in lockstep share every weight GEMV
// (M = B columns); each keeps its own KV cache (a 4th "sequence" view dimension).  With batch == 1
// the node list is the reference's.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tts_runners.h"
#include "graph.h"
#include "synth.h"

using namespace tts;

struct orpheus_layer {
    tts_tensor *input_norm, *q, *k, *v, *o, *post_attention_norm, *gate, *up, *down;
};

struct tts_orpheus {
    tts_orpheus_config cfg;
    tts_backend_iface be;
    tg::context wctx;
    void * wbuf = nullptr;
    size_t wbytes = 0;
    void * kvbuf = nullptr;
    std::vector<orpheus_layer> layers;
    tts_tensor *embd = nullptr, *head = nullptr, *output_norm = nullptr, *rope_frequencies = nullptr;
    std::vector<tts_tensor *> k_l, v_l;
    char * arena = nullptr;
    size_t arena_size = 0;
    tg::context gctx;
    tts_tensor * res = nullptr;
    tts_tensor *in_tokens = nullptr, *in_positions = nullptr, *in_mask = nullptr;
    int32_t position = 0;
    int32_t last_nodes = 0;
    bool prepared = false;
    int prep_slot = 0, prep_n = 0;
    void * launched_out = nullptr;
    int64_t host_steps = 0;
    std::vector<std::vector<int32_t>> output_tokens;
    uint64_t tensor_index = 0;
    // seeded sampling (tts_orpheus_set_sampling); greedy when off
    bool sampling = false;
    tts_sampling samp{};
    int64_t sample_calls = 0;
    std::vector<int32_t> rep_last, rep_count;  // [batch]
    std::vector<tts_tensor *> wlist;  // every weight, declaration order (tts_orpheus_weight)
};

extern "C" void tts_orpheus_set_sampling(tts_orpheus * p, const tts_sampling * cfg) {
    p->sampling = cfg != nullptr;
    if (cfg) p->samp = *cfg;
}

extern "C" void tts_orpheus_default_config(tts_orpheus_config * c) {
    // orpheus_model defaults (src/models/orpheus/model.h:31-46); Llama-3.2-3B rope scaling
    c->n_layers = 28;
    c->hidden_size = 3072;
    c->n_attn_heads = 24;
    c->n_kv_attn_heads = 8;
    c->head_size = 128;
    c->ffn_size = 8192;
    c->vocab_size = 156940;
    c->max_ctx = 1024 + 2100;  // max_context_length + max_generation_size
    c->weight_type = TTS_TYPE_Q4_K;
    c->batch = 1;
    c->seed = 0x5EED;
    c->arena_bytes = 0;
    c->rope_theta = 500000.0f;
    c->rope_factor = 32.0f;
    c->rope_low_freq_factor = 1.0f;
    c->rope_high_freq_factor = 4.0f;
    c->rope_original_ctx = 8192;
    c->pad_ = 0;
}

static tts_tensor * wnew(tts_orpheus * p, std::vector<std::pair<tts_tensor *, int>> & specs, int type, int64_t ne0, int64_t ne1,
                         int kind, const std::string & name) {
    tts_tensor * t = ne1 > 1 ? tg::new_tensor_2d(p->wctx, type, ne0, ne1) : tg::new_tensor_1d(p->wctx, type, ne0);
    tg::set_name(t, name);
    t->flags |= tg::TG_FLAG_PERSIST;
    specs.push_back({t, kind});
    return t;
}

// orpheus_gguf_encoder.prepare_rope_frequencies (py-gguf/tts_encoders/orpheus_gguf_encoder.py:144-173)
static void rope_factors(const tts_orpheus_config & cf, float * out) {
    const int dim = cf.head_size;
    const double low_wl = cf.rope_original_ctx / cf.rope_low_freq_factor;
    const double high_wl = cf.rope_original_ctx / cf.rope_high_freq_factor;
    for (int i = 0; i < dim / 2; ++i) {
        const float freq = (float)(1.0 / std::pow((double)cf.rope_theta, (double)(2 * i) / dim));
        const double wavelen = 2 * M_PI / freq;
        double f;
        if (wavelen < high_wl) f = 1.0;
        else if (wavelen > low_wl) f = cf.rope_factor;
        else {
            const double smooth = (cf.rope_original_ctx / wavelen - cf.rope_low_freq_factor) / (cf.rope_high_freq_factor - cf.rope_low_freq_factor);
            f = 1.0 / ((1.0 - smooth) / cf.rope_factor + smooth);
        }
        out[i] = (float)f;
    }
}

static bool upload_weights(tts_orpheus * p, std::vector<std::pair<tts_tensor *, int>> & specs) {
    size_t total = 0;
    for (auto & s : specs) total += (tg::nbytes(s.first) + 255) & ~(size_t)255;
    p->wbuf = p->be.alloc(p->be.ctx, total);
    if (!p->wbuf) return false;
    p->wbytes = total;
    size_t off = 0;
    std::vector<char> host;
    uint64_t idx = 0;
    for (auto & s : specs) {
        tts_tensor * t = s.first;
        const uint64_t seed = p->cfg.seed ^ (idx++);
        const size_t nb = tg::nbytes(t);
        t->data = (char *)p->wbuf + off;
        off += (nb + 255) & ~(size_t)255;
        host.resize(nb);
        const int64_t K = t->ne[0], rows = tg::nelements(t) / t->ne[0];
        if (s.second == 1) synth_f32((float *)host.data(), (size_t)(K * rows), seed, 0.1f, 1.0f);       // norm weights ~1
        else if (s.second == 4) rope_factors(p->cfg, (float *)host.data());                             // rope factors
        else synth_fill(t->type, host.data(), rows, K, seed, s.second == 3 ? 0.25f : 0.02f);          // matrices / embd
        if (p->be.set_tensor(p->be.ctx, t, host.data()) != 0) return false;
    }
    return true;
}

extern "C" tts_orpheus * tts_orpheus_create(const tts_backend_iface * be, const tts_orpheus_config * cfg) {
    auto * p = new tts_orpheus();
    p->cfg = *cfg;
    p->be = *be;
    auto & cf = p->cfg;
    if (cf.batch < 1) cf.batch = 1;
    const int64_t H = cf.hidden_size, KVH = (int64_t)cf.n_kv_attn_heads * cf.head_size;
    if ((int64_t)cf.n_attn_heads * cf.head_size != H || cf.n_attn_heads % cf.n_kv_attn_heads) {
        delete p;
        return nullptr;
    }
    std::vector<std::pair<tts_tensor *, int>> specs;
    p->embd = wnew(p, specs, cf.weight_type, H, cf.vocab_size, 3, "token_embd");
    p->head = wnew(p, specs, cf.weight_type, H, cf.vocab_size, 0, "output");
    p->output_norm = wnew(p, specs, TTS_TYPE_F32, H, 1, 1, "output_norm");
    p->rope_frequencies = wnew(p, specs, TTS_TYPE_F32, cf.head_size / 2, 1, 4, "rope_frequencies");
    p->layers.resize(cf.n_layers);
    for (int l = 0; l < cf.n_layers; ++l) {
        orpheus_layer & L = p->layers[l];
        const std::string pre = "layers." + std::to_string(l);
        L.input_norm = wnew(p, specs, TTS_TYPE_F32, H, 1, 1, pre + ".input_norm");
        L.q = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".q");
        L.k = wnew(p, specs, cf.weight_type, H, KVH, 0, pre + ".k");
        L.v = wnew(p, specs, cf.weight_type, H, KVH, 0, pre + ".v");
        L.o = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".o");
        L.post_attention_norm = wnew(p, specs, TTS_TYPE_F32, H, 1, 1, pre + ".post_attention_norm");
        L.gate = wnew(p, specs, cf.weight_type, H, cf.ffn_size, 0, pre + ".gate");
        L.up = wnew(p, specs, cf.weight_type, H, cf.ffn_size, 0, pre + ".up");
        L.down = wnew(p, specs, cf.weight_type, cf.ffn_size, H, 0, pre + ".down");
    }
    for (auto & s : specs) p->wlist.push_back(s.first);
    if (!upload_weights(p, specs)) {
        fprintf(stderr, "orpheus: weight allocation/upload failed\n");
        tts_orpheus_free(p);
        return nullptr;
    }
    // orpheus_kv_cache_init: F32 1-D [hidden * (max_ctx + max_gen)] per layer (x B sequences), cleared
    const size_t kvl = (size_t)H * cf.max_ctx * 4 * (size_t)cf.batch;
    p->kvbuf = p->be.alloc(p->be.ctx, 2 * kvl * cf.n_layers);
    if (!p->kvbuf) {
        tts_orpheus_free(p);
        return nullptr;
    }
    p->be.memset(p->be.ctx, p->kvbuf, 0, 2 * kvl * cf.n_layers);
    char * kp = (char *)p->kvbuf;
    for (int l = 0; l < cf.n_layers; ++l) {
        tts_tensor * k = tg::new_tensor_1d(p->wctx, TTS_TYPE_F32, H * cf.max_ctx * cf.batch);
        k->data = kp;
        kp += kvl;
        tts_tensor * v = tg::new_tensor_1d(p->wctx, TTS_TYPE_F32, H * cf.max_ctx * cf.batch);
        v->data = kp;
        kp += kvl;
        tg::set_name(k, "cache_k_l" + std::to_string(l));
        tg::set_name(v, "cache_v_l" + std::to_string(l));
        p->k_l.push_back(k);
        p->v_l.push_back(v);
    }
    p->arena_size = cf.arena_bytes ? cf.arena_bytes : (512ull << 20);
    p->arena = (char *)p->be.alloc(p->be.ctx, p->arena_size);
    if (!p->arena) {
        tts_orpheus_free(p);
        return nullptr;
    }
    tts_orpheus_reset(p);
    return p;
}

extern "C" void tts_orpheus_free(tts_orpheus * p) {
    if (!p) return;
    if (p->arena) p->be.free(p->be.ctx, p->arena);
    if (p->kvbuf) p->be.free(p->be.ctx, p->kvbuf);
    if (p->wbuf) p->be.free(p->be.ctx, p->wbuf);
    delete p;
}

extern "C" void tts_orpheus_reset(tts_orpheus * p) {
    p->position = 0;
    p->prepared = false;
    p->output_tokens.assign(p->cfg.batch, {});
    p->sample_calls = 0;  // sampler::reset (orpheus/model.cpp:426)
    p->rep_last.assign(p->cfg.batch, -1);
    p->rep_count.assign(p->cfg.batch, 0);
}

static tts_tensor * rms_norm_mul(tg::context & c, tts_tensor * x, tts_tensor * w) {
    // orpheus_build_layer_norm (model.cpp:122-125): rms_norm eps 1e-5, then mul
    return tg::mul(c, tg::rms_norm(c, x, 0.00001f), w);
}

static tts_tensor * rope(tts_orpheus * p, tg::context & c, tts_tensor * x) {
    // ggml_rope_ext(..., rope_frequencies, head_size, 2 (neox), 0, 500000, 1, 0, 1, 0, 0)
    return tg::rope_ext(c, x, p->in_positions, p->rope_frequencies, p->cfg.head_size, 2, 0, p->cfg.rope_theta, 1.0f, 0.0f, 1.0f,
                        0.0f, 0.0f);
}

// build_orpheus_graph for n tokens per sequence (n = 1 while generating).
static tts_tensor * build_graph(tts_orpheus * p, int n) {
    const auto & cf = p->cfg;
    const int B = cf.batch;
    const int64_t H = cf.hidden_size, hd = cf.head_size, nh = cf.n_attn_heads, nkv = cf.n_kv_attn_heads;
    const int repeat = (int)(nh / nkv);
    const int64_t full = p->position + n;
    const size_t S = (size_t)H * cf.max_ctx * 4;  // per-sequence cache stride
    const size_t es = 4;
    tg::context & c = p->gctx;
    c.reset();

    p->in_positions = tg::new_tensor_1d(c, TTS_TYPE_I32, n);
    tg::set_input(p->in_positions);
    p->in_tokens = tg::new_tensor_1d(c, TTS_TYPE_I32, (int64_t)n * B);
    tg::set_input(p->in_tokens);
    tts_tensor * inpL = tg::get_rows(c, p->embd, p->in_tokens);  // [H, n*B]
    if (B > 1) inpL = tg::reshape_3d(c, inpL, H, n, B);
    // build_attn_mask (model.cpp:127-131): [full, full], rows < n written by set_inputs
    p->in_mask = tg::new_tensor_2d(c, TTS_TYPE_F32, full, full);
    tg::set_input(p->in_mask);

    tts_tensor * cur = nullptr;
    for (int l = 0; l < cf.n_layers; ++l) {
        orpheus_layer & L = p->layers[l];
        tts_tensor * residual = inpL;
        cur = rms_norm_mul(c, inpL, L.input_norm);
        tts_tensor * attn_out;
        {
            tts_tensor * Qcur = tg::mul_mat(c, L.q, cur);
            tts_tensor * Kcur = tg::mul_mat(c, L.k, cur);
            tts_tensor * Vcur = tg::mul_mat(c, L.v, cur);
            // orpheus_build_kv_store (model.cpp:194-228): rope K, then `repeat` strided copies each of K and
            // V (V copied as the [H, n] product itself); the node order is the reference's (K's chain,
            // then V, Q only at the attention), which the planner groups across (try_gemv)
            tts_tensor * kr = B == 1 ? tg::reshape_3d(c, Kcur, hd, nkv, n) : tg::reshape_4d(c, Kcur, hd, nkv, n, B);
            kr = rope(p, c, tg::cont(c, kr));
            tts_tensor * vr = Vcur;
            for (int i = 0; i < repeat; ++i) {
                const size_t off = es * (size_t)H * p->position + (size_t)i * es * hd;
                tts_tensor *kv, *vv;
                if (B == 1) {
                    kv = tg::view_3d(c, p->k_l[l], hd, nkv, n, es * hd * repeat, es * H, off);
                    vv = tg::view_3d(c, p->v_l[l], hd, nkv, n, es * hd * repeat, es * H, off);
                } else {
                    kv = tg::view_4d(c, p->k_l[l], hd, nkv, n, B, es * hd * repeat, es * H, S, off);
                    vv = tg::view_4d(c, p->v_l[l], hd, nkv, n, B, es * hd * repeat, es * H, S, off);
                }
                tg::build_forward_expand(c, tg::cpy(c, kr, kv));
                tg::build_forward_expand(c, tg::cpy(c, vr, vv));
            }
            tts_tensor *k, *v;
            if (B == 1) {
                k = tg::cont(c, tg::view_3d(c, p->k_l[l], hd, full, nh, es * H, es * hd, 0));
                v = tg::view_2d(c, p->v_l[l], H, full, es * H, 0);
                v = tg::cont_3d(c, tg::transpose(c, v), full, hd, nh);
                Qcur = tg::reshape_3d(c, Qcur, hd, nh, n);
            } else {
                k = tg::cont(c, tg::view_4d(c, p->k_l[l], hd, full, nh, B, es * H, es * hd, S, 0));
                v = tg::view_3d(c, p->v_l[l], H, full, B, es * H, S, 0);
                v = tg::cont_4d(c, tg::transpose(c, v), full, hd, nh, B);
                Qcur = tg::reshape_4d(c, Qcur, hd, nh, n, B);
            }
            Qcur = rope(p, c, tg::cont(c, Qcur));
            tts_tensor * q = tg::cont(c, tg::permute(c, Qcur, 0, 2, 1, 3));
            tts_tensor * kq = tg::mul_mat(c, k, q);
            kq = tg::soft_max_ext(c, kq, p->in_mask, 1.0f / sqrtf((float)hd), 0.0f);
            tts_tensor * kqv = tg::mul_mat(c, kq, v);
            tts_tensor * merged = tg::permute(c, kqv, 2, 0, 1, 3);
            attn_out = B == 1 ? tg::cont_2d(c, merged, H, n) : tg::cont_3d(c, merged, H, n, B);
            attn_out = tg::mul_mat(c, L.o, attn_out);
        }
        cur = tg::add(c, attn_out, residual);
        tts_tensor * residualffn = cur;
        cur = rms_norm_mul(c, cur, L.post_attention_norm);
        cur = tg::mul(c, tg::silu(c, tg::mul_mat(c, L.gate, cur)), tg::mul_mat(c, L.up, cur));
        cur = tg::mul_mat(c, L.down, cur);
        cur = tg::add(c, cur, residualffn);
        inpL = cur;
    }
    cur = rms_norm_mul(c, cur, p->output_norm);
    cur = tg::mul_mat(c, p->head, cur);  // [vocab, n(, B)]
    if (n > 1) {  // only the last token's logits (model.cpp:301-303)
        if (B == 1) cur = tg::cont(c, tg::view_1d(c, cur, cf.vocab_size, es * (size_t)(cur->ne[1] - 1) * cf.vocab_size));
        else cur = tg::cont(c, tg::view_2d(c, cur, cf.vocab_size, B, cur->nb[2], es * (size_t)(n - 1) * cf.vocab_size));
    }
    tg::set_name(cur, "logits");
    tg::set_output(cur);
    tg::build_forward_expand(c, cur);
    return cur;
}

static int set_inputs(tts_orpheus * p, const int32_t * tokens, int n, bool async) {
    auto & be = p->be;
    auto set = [&](void * d, const void * s, size_t bytes) {
        return (async && be.set_async) ? be.set_async(be.ctx, d, s, bytes) : be.set(be.ctx, d, s, bytes);
    };
    int st = 0;
    if (tokens) st |= set(p->in_tokens->data, tokens, sizeof(int32_t) * (size_t)n * p->cfg.batch);
    std::vector<int32_t> pos(n);
    for (int i = 0; i < n; ++i) pos[i] = p->position + i;
    st |= set(p->in_positions->data, pos.data(), sizeof(int32_t) * n);
    // set_inputs (model.cpp:344-352): mask rows i < n, causal
    const int64_t full = p->position + n;
    std::vector<float> mask((size_t)n * full);
    for (int i = 0; i < n; ++i)
        for (int64_t j = 0; j < full; ++j) mask[(size_t)i * full + j] = j > pos[i] ? -INFINITY : 0.0f;
    st |= set(p->in_mask->data, mask.data(), mask.size() * sizeof(float));
    return st;
}

static int prepare_step(tts_orpheus * p, int n) {
    if (p->position + n > p->cfg.max_ctx) return TTS_STATUS_BAD_ARG;
    p->res = build_graph(p, n);
    if (!tg::alloc_graph(p->gctx, p->arena, p->arena_size, true)) {
        fprintf(stderr, "orpheus: compute arena too small (%zu needed)\n", p->gctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    p->last_nodes = (int32_t)p->gctx.nodes.size();
    p->prep_slot = (int)(p->host_steps & 1);
    p->prep_n = n;
    if (p->be.prepare) {
        const int st = p->be.prepare(p->be.ctx, p->gctx.nodes.data(), (int)p->gctx.nodes.size(), p->prep_slot);
        if (st != 0) return st;
    }
    p->prepared = true;
    return 0;
}

static int launch_step(tts_orpheus * p, const int32_t * tokens, bool async) {
    if (!p->prepared) return TTS_STATUS_FAILED;
    if (set_inputs(p, tokens, p->prep_n, async) != 0) return TTS_STATUS_FAILED;
    const int st = p->be.launch ? p->be.launch(p->be.ctx, p->prep_slot)
                                : p->be.compute(p->be.ctx, p->gctx.nodes.data(), (int)p->gctx.nodes.size());
    if (st != 0) return st;
    p->prepared = false;
    p->launched_out = p->res->data;
    p->position += p->prep_n;
    p->host_steps += 1;
    return 0;
}

static int decode(tts_orpheus * p, const int32_t * tokens, int n, float * logits) {
    int st = p->prepared ? 0 : prepare_step(p, n);
    if (st == 0 && p->prep_n != n) return TTS_STATUS_FAILED;
    if (st == 0) st = launch_step(p, tokens, false);
    if (st == 0 && logits) st = p->be.get(p->be.ctx, logits, p->launched_out, sizeof(float) * (size_t)p->cfg.batch * p->cfg.vocab_size);
    if (st == 0) st = p->be.synchronize(p->be.ctx);
    return st;
}

extern "C" int tts_orpheus_prefill(tts_orpheus * p, const int32_t * tokens, int32_t n, float * logits) {
    return decode(p, tokens, n, logits);
}

extern "C" int tts_orpheus_decode(tts_orpheus * p, const int32_t * tokens, float * logits) { return decode(p, tokens, 1, logits); }

// sampler::max (sampler.cpp:185-204): first maximum
static int32_t argmax(const float * l, int64_t V) {
    float mx = -INFINITY;
    int32_t id = 0;
    for (int64_t i = 0; i < V; ++i)
        if (l[i] > mx) {
            mx = l[i];
            id = (int32_t)i;
        }
    return id;
}

// generate_from_batch (model.cpp:381-396) with greedy sampling for n_steps tokens after the last
// decoded position; first_tokens [B] are the tokens fed at the first step (the previous step's
// samples).  On a backend with greedy_step the samples never leave the device until the end.
extern "C" int tts_orpheus_generate(tts_orpheus * p, const int32_t * first_tokens, int32_t n_steps, int32_t * tokens_out) {
    const auto & cf = p->cfg;
    const int B = cf.batch;
    const int64_t V = cf.vocab_size;
    auto & be = p->be;
    if (n_steps <= 0) return 0;
    if (p->prepared && p->prep_n != 1) return TTS_STATUS_FAILED;
    const bool dev_sample = !p->sampling || (be.sample_step && tts_sampling_device_ok(&p->samp, (int32_t)V));
    if (be.greedy_step && be.set_async && be.copy && be.prepare && dev_sample) {
        const size_t rowi = (size_t)B * sizeof(int32_t);
        int32_t * d_seen = (int32_t *)be.alloc(be.ctx, rowi);
        int32_t * d_next = (int32_t *)be.alloc(be.ctx, rowi);
        int32_t * d_hist = (int32_t *)be.alloc(be.ctx, rowi * (size_t)n_steps);
        int32_t * d_rep = p->sampling ? (int32_t *)be.alloc(be.ctx, 2 * rowi) : nullptr;
        int st = (d_seen && d_next && d_hist && (!p->sampling || d_rep)) ? 0 : TTS_STATUS_ALLOC_FAILED;
        if (st == 0) st = be.memset(be.ctx, d_seen, 0, rowi);
        std::vector<int32_t> rep(2 * (size_t)B);
        if (st == 0 && d_rep) {
            for (int b = 0; b < B; ++b) rep[2 * b] = p->rep_last[b], rep[2 * b + 1] = p->rep_count[b];
            st = be.set(be.ctx, d_rep, rep.data(), 2 * rowi);
        }
        if (st == 0 && !p->prepared) st = prepare_step(p, 1);
        if (st == 0) st = launch_step(p, first_tokens, true);
        for (int s = 0; st == 0 && s < n_steps; ++s) {
            const float * logits = (const float *)p->launched_out;
            if (s + 1 < n_steps) st = prepare_step(p, 1);  // recorded while the device runs step s
            // one head, no BOS / EOS rule (eos -1): next = the sample itself
            if (st == 0 && p->sampling)
                st = be.sample_step(be.ctx, logits, B, 1, (int32_t)V, &p->samp, p->sample_calls + s, d_rep, 0, 0, -1, d_seen, d_hist + (size_t)s * B,
                                    d_next);
            else if (st == 0)
                st = be.greedy_step(be.ctx, logits, B, 1, (int32_t)V, 0, 0, -1, d_seen, d_hist + (size_t)s * B, d_next);
            if (st == 0 && s + 1 < n_steps) {
                st = be.copy(be.ctx, p->in_tokens->data, d_next, rowi);
                if (st == 0) st = launch_step(p, nullptr, true);
            }
        }
        std::vector<int32_t> hist((size_t)n_steps * B);
        if (st == 0) st = be.get(be.ctx, hist.data(), d_hist, hist.size() * sizeof(int32_t));
        if (st == 0 && d_rep) {
            st = be.get(be.ctx, rep.data(), d_rep, 2 * rowi);
            for (int b = 0; b < B; ++b) p->rep_last[b] = rep[2 * b], p->rep_count[b] = rep[2 * b + 1];
        }
        if (st == 0 && p->sampling) p->sample_calls += n_steps;
        if (d_rep) be.free(be.ctx, d_rep);
        if (d_seen) be.free(be.ctx, d_seen);
        if (d_next) be.free(be.ctx, d_next);
        if (d_hist) be.free(be.ctx, d_hist);
        if (st != 0) return st;
        for (int s = 0; s < n_steps; ++s)
            for (int b = 0; b < B; ++b) {
                p->output_tokens[b].push_back(hist[(size_t)s * B + b]);
                if (tokens_out) tokens_out[(size_t)b * n_steps + s] = hist[(size_t)s * B + b];
            }
        return 0;
    }
    std::vector<float> logits((size_t)B * V);
    std::vector<int32_t> next(first_tokens, first_tokens + B);
    for (int s = 0; s < n_steps; ++s) {
        int st = decode(p, next.data(), 1, logits.data());
        if (st != 0) return st;
        for (int b = 0; b < B; ++b) {
            if (p->sampling) {  // sampler::sample (orpheus/model.cpp:392), prompt b's own generator
                st = tts_sampler_sample(&p->samp, logits.data() + (size_t)b * V, 1, (int32_t)V, tts_sampler_call_seed(p->samp.seed, b, p->sample_calls),
                                        &p->rep_last[b], &p->rep_count[b], &next[b]);
                if (st != 0) return st;
            } else {
                next[b] = argmax(logits.data() + (size_t)b * V, V);
            }
            p->output_tokens[b].push_back(next[b]);
            if (tokens_out) tokens_out[(size_t)b * n_steps + s] = next[b];
        }
        if (p->sampling) p->sample_calls += 1;
    }
    return 0;
}

extern "C" int32_t tts_orpheus_position(const tts_orpheus * p) { return p->position; }
extern "C" int32_t tts_orpheus_last_graph_nodes(const tts_orpheus * p) { return p->last_nodes; }
extern "C" uint64_t tts_orpheus_weight_bytes(const tts_orpheus * p) { return p->wbytes; }
extern "C" int32_t tts_orpheus_n_weights(const tts_orpheus * p) { return p ? (int32_t)p->wlist.size() : 0; }
extern "C" uint64_t tts_orpheus_weight(tts_orpheus * p, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst,
                                       uint64_t cap) {
    if (!p || i < 0 || i >= (int32_t)p->wlist.size()) return 0;
    return tg::weight_out(p->be, p->wlist[i], name, name_cap, ne, type, dst, cap);
}
extern "C" tts_tensor * const * tts_orpheus_graph(const tts_orpheus * p, int32_t * n_nodes) {
    if (n_nodes) *n_nodes = p ? (int32_t)p->gctx.nodes.size() : 0;
    return p ? p->gctx.nodes.data() : nullptr;
}
