// Parler-TTS decoder runner: builds the same per-step graph as
// parler_tts_runner::build_parler_graph (/root/reference/src/models/parler/model.cpp:520-614),
// stores K/V like parler_build_kv_store (:420-439), precomputes cross K/V like
// prep_cross_key_values (:110-173) and samples greedily like sampler::max
// (/root/reference/src/sampler.cpp:185-204) inside the generate_from_batch loop (:762-792).
//
// Extension (batch > 1): B independent prompts stepped in lockstep share every weight GEMV
// (M = B columns) while each keeps its own KV cache (attention gets a 4th "sequence" dim).
// Prompts of different lengths (tts_parler_prefill_ragged) share one prompt pass: sequence b's
// prompt holds KV slots [0, len_b), slots [len_b, n_max) are padding its own mask hides, and from
// slot n_max on every sequence's decode tokens share slots; position ids and masks are per
// sequence.  Each sequence then sees exactly its own prompt's keys, in order.
// With batch == 1 the node list is exactly the reference's.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tts_gguf.h"
#include "../../include/tts_runners.h"
#include "graph.h"
#include "synth.h"

using namespace tts;

struct parler_layer {
    tts_tensor *q, *k, *v, *o, *sa_norm, *sa_norm_b;
    tts_tensor *aq, *ak, *av, *ao, *a_norm, *a_norm_b;
    tts_tensor *cross_k, *cross_v;
    tts_tensor *fc1, *fc2, *f_norm, *f_norm_b;
};

struct tts_parler {
    tts_parler_config cfg;
    tts_backend_iface be;
    tg::context wctx;
    void * wbuf = nullptr;
    size_t wbytes = 0;
    void * kvbuf = nullptr;
    size_t kvbytes = 0;
    std::vector<tts_tensor *> embds, heads;
    std::vector<parler_layer> layers;
    tts_tensor *pos_embd = nullptr, *prompt_embd = nullptr, *text_encoding = nullptr, *norm = nullptr, *norm_b = nullptr;
    std::vector<tts_tensor *> k_l, v_l;
    char * arena = nullptr;
    size_t arena_size = 0;
    tg::context gctx;
    tts_tensor * res = nullptr;
    tts_tensor *in_tokens = nullptr, *in_positions = nullptr, *in_mask = nullptr, *in_mask_cross = nullptr;
    int32_t position = 0;  // KV slots in use (every sequence)
    int32_t current_step = 0;
    // ragged lock-step batch (tts_parler_prefill_ragged): sequence b's prompt is seq_len[b] tokens,
    // slots [seq_len[b], hole_end) are never attended, slot s >= hole_end has position id
    // seq_len[b] + s - hole_end
    bool ragged = false;
    std::vector<int32_t> seq_len;
    int32_t hole_end = 0;
    int32_t last_nodes = 0;
    double host_us[5] = {0, 0, 0, 0, 0};  // build, alloc, set_inputs, compute (record + launch), get (wait)
    bool prepared = false;  // a step is built and recorded, waiting for launch_step
    bool device_sampling = true;  // greedy sampling on the device when the backend offers it
    int prep_slot = 0, prep_n = 0;
    bool prep_audio = true;
    void * launched_out = nullptr;  // logits of the last launched step (device)
    int launched_n = 0;
    int64_t host_steps = 0;
    std::vector<std::vector<int32_t>> output_tokens;  // per sequence, flat [steps][heads]
    std::vector<std::vector<char>> eos_seen;
    uint64_t tensor_index = 0;
    // seeded sampling (tts_parler_set_sampling); greedy (sampler::max) when off
    bool sampling = false;
    tts_sampling samp{};
    int64_t sample_calls = 0;                 // sampler::sample calls so far (one per step)
    std::vector<int32_t> rep_last, rep_count;  // [batch][heads] repetition-penalty state
    const tts_gguf * gguf = nullptr;  // weight source while creating from a file (else synthetic)
    std::vector<tts_tensor *> wlist;  // every weight, declaration order (tts_parler_weight)
};

extern "C" void tts_parler_default_config(tts_parler_config * c) {
    c->n_layers = 24;
    c->hidden_size = 1024;
    c->n_attn_heads = 16;
    c->ffn_size = 4096;
    c->n_output_heads = 9;
    c->output_vocab = 1088;
    c->audio_vocab = 1024;
    c->max_ctx = 4096;
    c->n_encode = 3;
    c->prompt_vocab = 32128;
    c->max_positions = 4102;
    c->weight_type = TTS_TYPE_Q4_K;
    c->head_type = TTS_TYPE_F32;
    c->use_cross_attn = 1;
    c->batch = 1;
    c->eos_token = 1024;
    c->bos_token = 1025;
    c->seed = 0x5EED;
    c->arena_bytes = 0;
    c->debug_no_reuse = 0;
    c->pad_ = 0;
}

// ---- weights ----
struct wspec {
    tts_tensor * t;
    int kind;  // 0 = matrix (synth_fill), 1 = norm weight (~1), 2 = bias (~0), 3 = embedding f32
    uint64_t seed;
};

// Tensor names are the GGUF names without the "decoder." prefix (parler/model.cpp:4-27, :501-505).
static std::string gguf_name(const tts_tensor * t) { return std::string("decoder.") + t->name; }

static tts_tensor * wnew(tts_parler * p, std::vector<wspec> & specs, int type, int64_t ne0, int64_t ne1, int kind,
                         const std::string & name) {
    if (p->gguf) {  // the file decides the storage type (quantize_impl.cpp's per-tensor rules)
        const int64_t i = tts_gguf_find_tensor(p->gguf, ("decoder." + name).c_str());
        if (i >= 0) type = tts_gguf_tensor_type(p->gguf, i);
    }
    tts_tensor * t = ne1 > 1 ? tg::new_tensor_2d(p->wctx, type, ne0, ne1) : tg::new_tensor_1d(p->wctx, type, ne0);
    tg::set_name(t, name);
    t->flags |= tg::TG_FLAG_PERSIST;
    specs.push_back({t, kind, p->cfg.seed ^ (p->tensor_index++)});
    return t;
}

// The synthetic bytes tts_parler_create uploads for a spec (host).
static void synth_host(const wspec & s, std::vector<char> & host) {
    const tts_tensor * t = s.t;
    host.resize(tg::nbytes(t));
    const int64_t K = t->ne[0], rows = tg::nelements(t) / t->ne[0];
    const int kind = (t->type == TTS_TYPE_F32) ? s.kind : 0;
    const float std = s.kind == 3 ? 0.25f : 0.02f;
    switch (kind) {
        case 1: synth_f32((float *)host.data(), (size_t)(K * rows), s.seed, 0.1f, 1.0f); break;
        case 2: synth_f32((float *)host.data(), (size_t)(K * rows), s.seed, 0.02f, 0.0f); break;
        case 3: synth_f32((float *)host.data(), (size_t)(K * rows), s.seed, 0.5f, 0.0f); break;
        default: synth_fill(t->type, host.data(), rows, K, s.seed, std); break;
    }
}

// Same elements in the same order: equal after dropping the 1-sized dimensions (a GGUF bias [C]
// against a [1, C] tensor, assign_to_layer's transposed dup).
static bool same_squeezed_shape(const int64_t * a, const int64_t * b) {
    int64_t x[4], y[4];
    int nx = 0, ny = 0;
    for (int d = 0; d < 4; ++d) {
        if (a[d] != 1) x[nx++] = a[d];
        if (b[d] != 1) y[ny++] = b[d];
    }
    if (nx != ny) return false;
    for (int d = 0; d < nx; ++d)
        if (x[d] != y[d]) return false;
    return true;
}

// File tensor for t: present, same type and element layout; NULL (reason on stderr) otherwise.
static const void * gguf_source(const tts_gguf * g, const std::string & fname, const tts_tensor * t) {
    const int64_t i = tts_gguf_find_tensor(g, fname.c_str());
    if (i < 0) {
        fprintf(stderr, "gguf: tensor '%s' is missing\n", fname.c_str());
        return nullptr;
    }
    int64_t ne[4];
    tts_gguf_tensor_ndims(g, i, ne);
    if (tts_gguf_tensor_type(g, i) != t->type || !same_squeezed_shape(ne, t->ne) || tts_gguf_tensor_size(g, i) != tg::nbytes(t)) {
        fprintf(stderr, "gguf: tensor '%s' has type %d [%lld %lld %lld %lld], the runner needs type %d [%lld %lld %lld %lld]\n", fname.c_str(),
                tts_gguf_tensor_type(g, i), (long long)ne[0], (long long)ne[1], (long long)ne[2], (long long)ne[3], t->type, (long long)t->ne[0],
                (long long)t->ne[1], (long long)t->ne[2], (long long)t->ne[3]);
        return nullptr;
    }
    return tts_gguf_tensor_data(g, i);
}

static bool upload_weights(tts_parler * p, std::vector<wspec> & specs) {
    size_t total = 0;
    for (auto & s : specs) total += (tg::nbytes(s.t) + 255) & ~(size_t)255;
    p->wbuf = p->be.alloc(p->be.ctx, total);
    if (!p->wbuf) return false;
    p->wbytes = total;
    size_t off = 0;
    std::vector<char> host;
    for (auto & s : specs) {
        tts_tensor * t = s.t;
        const size_t nb = tg::nbytes(t);
        t->data = (char *)p->wbuf + off;
        off += (nb + 255) & ~(size_t)255;
        const void * src;
        if (p->gguf) {  // assign_weight: the mapped file bytes, uploaded whole
            src = gguf_source(p->gguf, gguf_name(t), t);
            if (!src) return false;
        } else {
            synth_host(s, host);
            src = host.data();
        }
        // whole-tensor upload: the backend may keep its own layout (HIP: Q4_K lane layout)
        if (p->be.set_tensor(p->be.ctx, t, src) != 0) return false;
    }
    return true;
}

static tts_tensor * layer_norm(tg::context & c, tts_tensor * x, tts_tensor * w, tts_tensor * b) {
    // parler_build_layer_norm (model.cpp:412-418): eps 1e-5, norm -> mul -> add
    x = tg::norm(c, x, 0.00001f);
    x = tg::mul(c, x, w);
    return tg::add(c, x, b);
}

static bool run_graph(tts_parler * p, tg::context & c) {
    if (!tg::alloc_graph(c, p->arena, p->arena_size, !p->cfg.debug_no_reuse)) {
        fprintf(stderr, "parler: compute arena too small (%zu needed)\n", c.arena_used);
        return false;
    }
    return true;
}

// prep_cross_key_values: per layer cross_k = cont(permute(reshape(K . text_encoding))) [hd, n_enc, H],
// cross_v = cont_3d(transpose(V . text_encoding), n_enc, hd, H) (model.cpp:146-156).
static bool prep_cross_key_values(tts_parler * p) {
    const auto & cf = p->cfg;
    const int hd = cf.hidden_size / cf.n_attn_heads;
    tg::context & c = p->gctx;
    c.reset();
    for (int l = 0; l < cf.n_layers; ++l) {
        parler_layer & L = p->layers[l];
        tts_tensor * Kc = tg::mul_mat(c, L.ak, p->text_encoding);
        tts_tensor * Vc = tg::mul_mat(c, L.av, p->text_encoding);
        Kc = tg::reshape_3d(c, Kc, hd, cf.n_attn_heads, cf.n_encode);
        Vc = tg::transpose(c, Vc);
        tts_tensor * k = tg::cont(c, tg::permute(c, Kc, 0, 2, 1, 3));
        tts_tensor * v = tg::cont_3d(c, Vc, cf.n_encode, hd, cf.n_attn_heads);
        if (cf.batch > 1) {
            tts_tensor * shape = tg::new_tensor_4d(c, TTS_TYPE_F32, cf.n_encode, hd, cf.n_attn_heads, cf.batch);
            shape->data = L.cross_v->data;  // metadata only (repeat reads shape->ne)
            v = tg::repeat(c, v, shape);
        }
        tg::build_forward_expand(c, tg::cpy(c, k, L.cross_k));
        tg::build_forward_expand(c, tg::cpy(c, v, L.cross_v));
    }
    if (!run_graph(p, c)) return false;
    if (p->be.compute(p->be.ctx, c.nodes.data(), (int)c.nodes.size()) != 0) return false;
    return p->be.synchronize(p->be.ctx) == 0;
}

extern "C" void tts_parler_free(tts_parler * p);

// Declares every weight tensor in the reference's order (synthetic seeds follow this order).
static void declare_weights(tts_parler * p, std::vector<wspec> & specs) {
    const auto & cf = p->cfg;
    const int64_t H = cf.hidden_size;
    // decoder.embed_tokens.{i} (Q4_K when quantized), decoder.lm_heads.{i}.weight.head (F32)
    for (int i = 0; i < cf.n_output_heads; ++i)
        p->embds.push_back(wnew(p, specs, cf.weight_type, H, cf.output_vocab, 3, "embed_tokens." + std::to_string(i) + ".weight"));
    for (int i = 0; i < cf.n_output_heads; ++i)
        p->heads.push_back(wnew(p, specs, cf.head_type, H, cf.output_vocab, 0, "lm_heads." + std::to_string(i) + ".weight.head"));
    p->pos_embd = wnew(p, specs, TTS_TYPE_F32, H, cf.max_positions, 3, "positional_embed");
    p->prompt_embd = wnew(p, specs, TTS_TYPE_F32, H, cf.prompt_vocab, 3, "embed_prompts");
    p->text_encoding = wnew(p, specs, TTS_TYPE_F32, H, cf.n_encode, 3, "text_encoding");
    p->norm = wnew(p, specs, TTS_TYPE_F32, H, 1, 1, "layer_norm.weight");
    p->norm_b = wnew(p, specs, TTS_TYPE_F32, H, 1, 2, "layer_norm.bias");
    p->layers.resize(cf.n_layers);
    for (int l = 0; l < cf.n_layers; ++l) {
        parler_layer & L = p->layers[l];
        const std::string pre = "layers." + std::to_string(l);
        L.q = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".self_attn.q_proj.weight");
        L.k = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".self_attn.k_proj.weight");
        L.v = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".self_attn.v_proj.weight");
        L.o = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".self_attn.out_proj.weight");
        L.sa_norm = wnew(p, specs, TTS_TYPE_F32, H, 1, 1, pre + ".self_attn_layer_norm.weight");
        L.sa_norm_b = wnew(p, specs, TTS_TYPE_F32, H, 1, 2, pre + ".self_attn_layer_norm.bias");
        L.aq = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".encoder_attn.q_proj.weight");
        // encoder_attn k/v stay F32 (quantize_impl.cpp: quantize_cross_attn_kv off by default)
        L.ak = wnew(p, specs, TTS_TYPE_F32, H, H, 0, pre + ".encoder_attn.k_proj.weight");
        L.av = wnew(p, specs, TTS_TYPE_F32, H, H, 0, pre + ".encoder_attn.v_proj.weight");
        L.ao = wnew(p, specs, cf.weight_type, H, H, 0, pre + ".encoder_attn.out_proj.weight");
        L.a_norm = wnew(p, specs, TTS_TYPE_F32, H, 1, 1, pre + ".encoder_attn_layer_norm.weight");
        L.a_norm_b = wnew(p, specs, TTS_TYPE_F32, H, 1, 2, pre + ".encoder_attn_layer_norm.bias");
        L.fc1 = wnew(p, specs, cf.weight_type, H, cf.ffn_size, 0, pre + ".fc1.weight");
        L.fc2 = wnew(p, specs, cf.weight_type, cf.ffn_size, H, 0, pre + ".fc2.weight");
        L.f_norm = wnew(p, specs, TTS_TYPE_F32, H, 1, 1, pre + ".final_layer_norm.weight");
        L.f_norm_b = wnew(p, specs, TTS_TYPE_F32, H, 1, 2, pre + ".final_layer_norm.bias");
    }
}

static tts_parler * parler_create(const tts_backend_iface * be, const tts_parler_config * cfg, const tts_gguf * g) {
    auto * p = new tts_parler();
    p->cfg = *cfg;
    p->be = *be;
    p->gguf = g;
    const auto & cf = p->cfg;
    const int64_t H = cf.hidden_size;
    const int hd = cf.hidden_size / cf.n_attn_heads;
    const int B = cf.batch < 1 ? 1 : cf.batch;
    p->cfg.batch = B;
    std::vector<wspec> specs;
    declare_weights(p, specs);
    for (auto & s : specs) p->wlist.push_back(s.t);
    if (!upload_weights(p, specs)) {
        fprintf(stderr, "parler: weight allocation/upload failed\n");
        tts_parler_free(p);
        return nullptr;
    }
    // cross K/V + KV caches in one persistent buffer
    const size_t ck = (size_t)hd * cf.n_encode * cf.n_attn_heads * 4;
    const size_t cv = ck * (size_t)B;
    const size_t kvl = (size_t)H * cf.max_ctx * 4 * (size_t)B;
    p->kvbytes = (size_t)cf.n_layers * (((ck + 255) & ~(size_t)255) + ((cv + 255) & ~(size_t)255) + 2 * kvl);
    p->kvbuf = p->be.alloc(p->be.ctx, p->kvbytes);
    if (!p->kvbuf) {
        tts_parler_free(p);
        return nullptr;
    }
    p->be.memset(p->be.ctx, p->kvbuf, 0, p->kvbytes);  // ggml_backend_buffer_clear(buf, 0)
    char * kp = (char *)p->kvbuf;
    for (int l = 0; l < cf.n_layers; ++l) {
        parler_layer & L = p->layers[l];
        L.cross_k = tg::new_tensor_3d(p->wctx, TTS_TYPE_F32, hd, cf.n_encode, cf.n_attn_heads);
        L.cross_k->data = kp;
        kp += (ck + 255) & ~(size_t)255;
        if (B > 1) L.cross_v = tg::new_tensor_4d(p->wctx, TTS_TYPE_F32, cf.n_encode, hd, cf.n_attn_heads, B);
        else L.cross_v = tg::new_tensor_3d(p->wctx, TTS_TYPE_F32, cf.n_encode, hd, cf.n_attn_heads);
        L.cross_v->data = kp;
        kp += (cv + 255) & ~(size_t)255;
        // parler_kv_cache_init: 1-D F32 [hidden*max_ctx] per layer (x B sequences)
        tts_tensor * k = tg::new_tensor_1d(p->wctx, TTS_TYPE_F32, H * cf.max_ctx * B);
        k->data = kp;
        kp += kvl;
        tts_tensor * v = tg::new_tensor_1d(p->wctx, TTS_TYPE_F32, H * cf.max_ctx * B);
        v->data = kp;
        kp += kvl;
        tg::set_name(k, "cache_k_l" + std::to_string(l));
        tg::set_name(v, "cache_v_l" + std::to_string(l));
        p->k_l.push_back(k);
        p->v_l.push_back(v);
    }
    p->arena_size = cf.arena_bytes ? cf.arena_bytes : (256ull << 20);
    p->arena = (char *)p->be.alloc(p->be.ctx, p->arena_size);
    if (!p->arena) {
        tts_parler_free(p);
        return nullptr;
    }
    if (cf.use_cross_attn && !prep_cross_key_values(p)) {
        fprintf(stderr, "parler: cross K/V precompute failed\n");
        tts_parler_free(p);
        return nullptr;
    }
    p->gguf = nullptr;
    tts_parler_reset(p);
    return p;
}

extern "C" tts_parler * tts_parler_create(const tts_backend_iface * be, const tts_parler_config * cfg) { return parler_create(be, cfg, nullptr); }

extern "C" void tts_parler_free(tts_parler * p) {
    if (!p) return;
    if (p->arena) p->be.free(p->be.ctx, p->arena);
    if (p->kvbuf) p->be.free(p->be.ctx, p->kvbuf);
    if (p->wbuf) p->be.free(p->be.ctx, p->wbuf);
    delete p;
}

extern "C" void tts_parler_reset(tts_parler * p) {
    p->position = 0;
    p->ragged = false;
    p->seq_len.clear();
    p->hole_end = 0;
    p->current_step = 0;
    p->prepared = false;
    p->output_tokens.assign(p->cfg.batch, {});
    p->eos_seen.assign(p->cfg.batch, std::vector<char>(p->cfg.n_output_heads, 0));
    p->sample_calls = 0;
    p->rep_last.assign((size_t)p->cfg.batch * p->cfg.n_output_heads, -1);  // sampler::reset
    p->rep_count.assign((size_t)p->cfg.batch * p->cfg.n_output_heads, 0);
}

extern "C" void tts_parler_set_sampling(tts_parler * p, const tts_sampling * cfg) {
    p->sampling = cfg != nullptr;
    if (cfg) p->samp = *cfg;
}

// build_parler_graph for n tokens per sequence (n = 1 in audio generation).
static tts_tensor * build_graph(tts_parler * p, bool audio, int n) {
    const auto & cf = p->cfg;
    const int B = cf.batch;
    const int64_t H = cf.hidden_size;
    const int hd = cf.hidden_size / cf.n_attn_heads;
    const int nh = cf.n_attn_heads;
    const int64_t full = p->position + n;
    const size_t S = (size_t)H * cf.max_ctx * 4;  // per-sequence cache stride
    tg::context & c = p->gctx;
    c.reset();

    // parler_build_inp_embd (model.cpp:387-410); a ragged batch: positions per sequence ([B][n])
    const bool rg = p->ragged && B > 1;
    p->in_positions = tg::new_tensor_1d(c, TTS_TYPE_I32, rg ? (int64_t)n * B : n);
    tg::set_input(p->in_positions);
    tts_tensor * inp = nullptr;
    if (audio) {
        if (B == 1) {
            tts_tensor * tok = tg::reshape_2d(c, tg::new_tensor_1d(c, TTS_TYPE_I32, (int64_t)n * cf.n_output_heads), n, cf.n_output_heads);
            p->in_tokens = tok->view_src;
            tg::set_input(p->in_tokens);
            for (int i = 0; i < cf.n_output_heads; ++i) {
                tts_tensor * e = tg::get_rows(c, p->embds[i], tg::view_2d(c, tok, 1, n, tok->nb[1], i * sizeof(int32_t)));
                inp = i == 0 ? e : tg::add(c, e, inp);
            }
        } else {
            // head-major [heads][B] so that each head's ids are one contiguous 1-D index
            p->in_tokens = tg::new_tensor_1d(c, TTS_TYPE_I32, (int64_t)B * cf.n_output_heads);
            tg::set_input(p->in_tokens);
            for (int i = 0; i < cf.n_output_heads; ++i) {
                tts_tensor * idx = tg::view_1d(c, p->in_tokens, B, (size_t)i * B * sizeof(int32_t));
                tts_tensor * e = tg::get_rows(c, p->embds[i], idx);  // [H, B]
                inp = i == 0 ? e : tg::add(c, e, inp);
            }
        }
    } else {
        if (B == 1) {
            p->in_tokens = tg::new_tensor_1d(c, TTS_TYPE_I32, n);
            tg::set_input(p->in_tokens);
            inp = tg::get_rows(c, p->prompt_embd, p->in_tokens);
        } else {
            p->in_tokens = tg::new_tensor_1d(c, TTS_TYPE_I32, (int64_t)n * B);
            tg::set_input(p->in_tokens);
            inp = tg::reshape_3d(c, tg::get_rows(c, p->prompt_embd, p->in_tokens), H, n, B);  // [H, n, B]
        }
    }
    tts_tensor * pe = tg::get_rows(c, p->pos_embd, p->in_positions);
    if (rg && !audio) pe = tg::reshape_3d(c, pe, H, n, B);
    tts_tensor * inpL = tg::add(c, inp, pe);
    if (B > 1 && audio) inpL = tg::reshape_3d(c, inpL, H, 1, B);

    // build_attn_mask / build_attn_mask_cross (model.cpp:459-471); a ragged batch: one per sequence
    p->in_mask = rg ? tg::new_tensor_4d(c, TTS_TYPE_F32, full, n, 1, B) : tg::new_tensor_2d(c, TTS_TYPE_F32, full, full);
    tg::set_input(p->in_mask);
    p->in_mask_cross = tg::new_tensor_2d(c, TTS_TYPE_F32, cf.n_encode, n);
    tg::set_input(p->in_mask_cross);

    const float kq_scale = 1.0f / sqrtf((float)hd);
    tts_tensor * cur = nullptr;
    for (int l = 0; l < cf.n_layers; ++l) {
        parler_layer & L = p->layers[l];
        tts_tensor * residual = inpL;
        cur = layer_norm(c, inpL, L.sa_norm, L.sa_norm_b);
        tts_tensor * attn_out;
        {
            tts_tensor * Qcur = tg::mul_mat(c, L.q, cur);
            tts_tensor * Kcur = tg::mul_mat(c, L.k, cur);
            tts_tensor * Vcur = tg::mul_mat(c, L.v, cur);
            // parler_build_kv_store (model.cpp:420-439): its expands pull K and V into the node list
            // first, Q follows at the attention -- the reference's order, which the planner groups
            // across (graph_exec.hip try_gemv)
            if (B == 1) {
                tts_tensor * kv = tg::view_1d(c, p->k_l[l], (int64_t)n * H, tts_row_size(TTS_TYPE_F32, H) * p->position);
                tg::build_forward_expand(c, tg::cpy(c, Kcur, kv));
                tts_tensor * vv = tg::view_2d(c, p->v_l[l], n, H, (size_t)cf.max_ctx * 4, (size_t)p->position * 4);
                tts_tensor * vt = tg::cont(c, tg::transpose(c, Vcur));
                tg::build_forward_expand(c, tg::cpy(c, vt, vv));
            } else {
                tts_tensor * kv = tg::view_2d(c, p->k_l[l], (int64_t)n * H, B, S, tts_row_size(TTS_TYPE_F32, H) * p->position);
                tg::build_forward_expand(c, tg::cpy(c, Kcur, kv));
                tts_tensor * vv = tg::view_3d(c, p->v_l[l], n, H, B, (size_t)cf.max_ctx * 4, S, (size_t)p->position * 4);
                tts_tensor * V3 = tg::reshape_3d(c, Vcur, H, n, B);
                tts_tensor * vt = tg::cont(c, tg::transpose(c, V3));
                tg::build_forward_expand(c, tg::cpy(c, vt, vv));
            }
            tts_tensor *k, *v, *q;
            if (B == 1) {
                k = tg::view_3d(c, p->k_l[l], hd, full, nh, tts_row_size(TTS_TYPE_F32, H), tts_row_size(TTS_TYPE_F32, hd), 0);
                v = tg::view_3d(c, p->v_l[l], full, hd, nh, 4 * (size_t)cf.max_ctx, 4 * (size_t)cf.max_ctx * hd, 0);
                Qcur = tg::reshape_3d(c, Qcur, hd, nh, n);
            } else {
                k = tg::view_4d(c, p->k_l[l], hd, full, nh, B, tts_row_size(TTS_TYPE_F32, H), tts_row_size(TTS_TYPE_F32, hd), S, 0);
                v = tg::view_4d(c, p->v_l[l], full, hd, nh, B, 4 * (size_t)cf.max_ctx, 4 * (size_t)cf.max_ctx * hd, S, 0);
                Qcur = tg::reshape_4d(c, Qcur, hd, nh, n, B);
            }
            q = tg::cont(c, tg::permute(c, Qcur, 0, 2, 1, 3));
            tts_tensor * kq = tg::mul_mat(c, tg::cont(c, k), q);
            kq = tg::soft_max_ext(c, kq, p->in_mask, kq_scale, 0.0f);
            tts_tensor * kqv = tg::mul_mat(c, kq, v);
            tts_tensor * merged = tg::permute(c, kqv, 2, 0, 1, 3);
            attn_out = B == 1 ? tg::cont_2d(c, merged, H, n) : tg::cont_3d(c, merged, H, n, B);
            attn_out = tg::mul_mat(c, L.o, attn_out);
        }
        cur = tg::add(c, attn_out, residual);
        if (cf.use_cross_attn) {
            tts_tensor * residuala = cur;
            cur = layer_norm(c, cur, L.a_norm, L.a_norm_b);
            tts_tensor * Qcur = tg::mul_mat(c, L.aq, cur);
            Qcur = B == 1 ? tg::reshape_3d(c, Qcur, hd, nh, n) : tg::reshape_4d(c, Qcur, hd, nh, n, B);
            tts_tensor * q = tg::cont(c, tg::permute(c, Qcur, 0, 2, 1, 3));
            tts_tensor * kq = tg::mul_mat(c, L.cross_k, q);
            kq = tg::soft_max_ext(c, kq, p->in_mask_cross, kq_scale, 0.0f);
            tts_tensor * kqv = tg::mul_mat(c, kq, L.cross_v);
            tts_tensor * merged = tg::permute(c, kqv, 2, 0, 1, 3);
            cur = B == 1 ? tg::cont_2d(c, merged, H, n) : tg::cont_3d(c, merged, H, n, B);
            cur = tg::mul_mat(c, L.ao, cur);
            cur = tg::add(c, cur, residuala);
        }
        tts_tensor * residualffn = cur;
        cur = layer_norm(c, cur, L.f_norm, L.f_norm_b);
        cur = tg::mul_mat(c, L.fc1, cur);
        cur = tg::gelu(c, cur);
        cur = tg::mul_mat(c, L.fc2, cur);
        cur = tg::add(c, cur, residualffn);
        inpL = cur;
    }
    if (!audio && B > 1) {
        // a batched prompt pass (our extension; B = 1 keeps the reference's node list): its logits are
        // never read (tts_parler_prefill / _ragged pass no output), so the final norm and the nine heads
        // over every prompt token (9 x 1088 rows x n * B columns of F32 products) are not built
        tg::set_output(cur);
        tg::build_forward_expand(c, cur);
        return cur;
    }
    cur = layer_norm(c, cur, p->norm, p->norm_b);
    // parler_build_head_outputs (model.cpp:441-457)
    tts_tensor * out = nullptr;
    for (int i = 0; i < cf.n_output_heads; ++i) {
        tts_tensor * h = tg::mul_mat(c, p->heads[i], cur);
        out = i == 0 ? h : tg::concat(c, out, h, 1);
    }
    tg::set_name(out, "final_out");
    if (B == 1) {
        const int64_t sql = tg::nelements(out) / ((int64_t)cf.output_vocab * cf.n_output_heads);
        out = tg::cont_3d(c, out, cf.output_vocab, sql, cf.n_output_heads);
    }
    tg::set_output(out);
    tg::build_forward_expand(c, out);
    return out;
}

// set_inputs (model.cpp:616-643): only rows < n of the causal mask are written/read.
static int set_inputs(tts_parler * p, const int32_t * tokens, bool audio, int n, bool async = false) {
    const auto & cf = p->cfg;
    const int B = cf.batch;
    auto & be0 = p->be;
    struct {
        tts_backend_iface & b;
        bool a;
        void * ctx;
        int set(void *, void * d, const void * s, size_t n) { return a ? b.set_async(b.ctx, d, s, n) : b.set(b.ctx, d, s, n); }
    } be{be0, async && be0.set_async, be0.ctx};
    int st = 0;
    if (audio && !tokens) {
        // tokens already on the device (device sampling path)
    } else if (audio) {
        if (B == 1) {
            // audio tokens arrive as [heads] for n == 1; layout [heads][n] otherwise
            st |= be.set(be.ctx, p->in_tokens->data, tokens, sizeof(int32_t) * n * cf.n_output_heads);
        } else {
            std::vector<int32_t> hm((size_t)B * cf.n_output_heads);  // [B][heads] -> [heads][B]
            for (int b = 0; b < B; ++b)
                for (int h = 0; h < cf.n_output_heads; ++h) hm[(size_t)h * B + b] = tokens[(size_t)b * cf.n_output_heads + h];
            st |= be.set(be.ctx, p->in_tokens->data, hm.data(), sizeof(int32_t) * hm.size());
        }
    } else {
        st |= be.set(be.ctx, p->in_tokens->data, tokens, sizeof(int32_t) * n * B);
    }
    const int64_t full = p->position + n;
    if (p->ragged && B > 1) {
        // per sequence: slot s's position id, and a mask hiding later slots and the padding slots
        std::vector<int32_t> pos((size_t)n * B);
        std::vector<float> mask((size_t)B * n * full);
        for (int b = 0; b < B; ++b) {
            const int32_t L = p->seq_len[b];
            for (int i = 0; i < n; ++i) {
                const int32_t s = p->position + i;
                pos[(size_t)b * n + i] = s < p->hole_end ? s : L + (s - p->hole_end);
                for (int64_t j = 0; j < full; ++j)
                    mask[((size_t)b * n + i) * full + j] = j > s || (j >= L && j < p->hole_end) ? -INFINITY : 0.0f;
            }
        }
        st |= be.set(be.ctx, p->in_positions->data, pos.data(), sizeof(int32_t) * pos.size());
        st |= be.set(be.ctx, p->in_mask->data, mask.data(), mask.size() * sizeof(float));
    } else {
        std::vector<int32_t> pos(n);
        for (int i = 0; i < n; ++i) pos[i] = p->position + i;
        st |= be.set(be.ctx, p->in_positions->data, pos.data(), sizeof(int32_t) * n);
        std::vector<float> mask((size_t)n * full);
        for (int i = 0; i < n; ++i)
            for (int64_t j = 0; j < full; ++j) mask[(size_t)i * full + j] = j > pos[i] ? -INFINITY : 0.0f;
        st |= be.set(be.ctx, p->in_mask->data, mask.data(), mask.size() * sizeof(float));
    }
    std::vector<float> mc((size_t)cf.n_encode * n, 0.0f);
    st |= be.set(be.ctx, p->in_mask_cross->data, mc.data(), mc.size() * sizeof(float));
    return st;
}

// A step is prepared (graph built, allocated and recorded into backend plan slot `slot`), then
// launched with its inputs, then finished (logits read).  generate() prepares step s+1 while the
// device runs step s, so the host's graph work overlaps the device (ggml's graph_plan_create /
// graph_plan_compute split).
static int prepare_step(tts_parler * p, bool audio, int n) {
    const auto & cf = p->cfg;
    if (p->position + n > cf.max_ctx) return TTS_STATUS_BAD_ARG;
    auto t0 = std::chrono::steady_clock::now();
    p->res = build_graph(p, audio, n);
    auto t1 = std::chrono::steady_clock::now();
    if (!run_graph(p, p->gctx)) return TTS_STATUS_ALLOC_FAILED;
    auto t2 = std::chrono::steady_clock::now();
    p->last_nodes = (int32_t)p->gctx.nodes.size();
    p->prep_slot = (int)(p->host_steps & 1);
    p->prep_audio = audio;
    p->prep_n = n;
    if (p->be.prepare) {
        const int st = p->be.prepare(p->be.ctx, p->gctx.nodes.data(), (int)p->gctx.nodes.size(), p->prep_slot);
        if (st != 0) return st;
    }
    auto t3 = std::chrono::steady_clock::now();
    p->prepared = true;
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    p->host_us[0] += us(t0, t1);
    p->host_us[1] += us(t1, t2);
    p->host_us[3] += us(t2, t3);
    return 0;
}

static int launch_step(tts_parler * p, const int32_t * tokens, bool async = false) {
    if (!p->prepared) return TTS_STATUS_FAILED;
    auto t0 = std::chrono::steady_clock::now();
    if (set_inputs(p, tokens, p->prep_audio, p->prep_n, async) != 0) return TTS_STATUS_FAILED;
    auto t1 = std::chrono::steady_clock::now();
    const int st = p->be.launch ? p->be.launch(p->be.ctx, p->prep_slot)
                                : p->be.compute(p->be.ctx, p->gctx.nodes.data(), (int)p->gctx.nodes.size());
    if (st != 0) return st;
    auto t2 = std::chrono::steady_clock::now();
    p->prepared = false;
    p->launched_out = p->res->data;
    p->launched_n = p->prep_n;
    p->position += p->prep_n;
    p->host_steps += 1;
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    p->host_us[2] += us(t0, t1);
    p->host_us[3] += us(t1, t2);
    return 0;
}

static int finish_step(tts_parler * p, float * logits) {
    const auto & cf = p->cfg;
    auto t0 = std::chrono::steady_clock::now();
    int st = 0;
    if (logits) {
        const size_t bytes = (size_t)cf.batch * p->launched_n * cf.n_output_heads * cf.output_vocab * sizeof(float);
        st = p->be.get(p->be.ctx, logits, p->launched_out, bytes);
    }
    auto t1 = std::chrono::steady_clock::now();
    p->host_us[4] += std::chrono::duration<double, std::micro>(t1 - t0).count();
    return st;
}

static int decode(tts_parler * p, const int32_t * tokens, bool audio, int n, float * logits) {
    int st = prepare_step(p, audio, n);
    if (st == 0) st = launch_step(p, tokens);
    if (st == 0) st = finish_step(p, logits);
    return st;
}

extern "C" int tts_parler_prefill(tts_parler * p, const int32_t * tokens, int32_t n) {
    int st = decode(p, tokens, false, n, nullptr);
    if (st == 0) p->be.synchronize(p->be.ctx);
    return st;
}

// One prompt pass over B prompts of different lengths (lens[b] <= n_max tokens each, row b of
// `tokens` holding n_max ids, the tail past lens[b] ignored) from an empty cache: a ragged lock-step
// batch (see the top of the file).  Every sequence's later tokens equal its own prompt's alone.
extern "C" int tts_parler_prefill_ragged(tts_parler * p, const int32_t * tokens, const int32_t * lens, int32_t n_max) {
    if (!p || !tokens || !lens || n_max < 1 || p->position != 0 || p->current_step != 0) return TTS_STATUS_BAD_ARG;
    const int B = p->cfg.batch;
    for (int b = 0; b < B; ++b)
        if (lens[b] < 1 || lens[b] > n_max) return TTS_STATUS_BAD_ARG;
    p->seq_len.assign(lens, lens + B);
    p->hole_end = n_max;
    p->ragged = B > 1;
    std::vector<int32_t> tok((size_t)B * n_max);
    for (int b = 0; b < B; ++b)
        for (int i = 0; i < n_max; ++i) tok[(size_t)b * n_max + i] = i < lens[b] ? tokens[(size_t)b * n_max + i] : 0;  // padding: never attended
    int st = decode(p, tok.data(), false, n_max, nullptr);
    if (st == 0) p->be.synchronize(p->be.ctx);
    return st;
}

extern "C" int tts_parler_decode(tts_parler * p, const int32_t * audio_tokens, float * logits) {
    return decode(p, audio_tokens, true, 1, logits);
}

// sampler::max (sampler.cpp:185-204) without repetition penalty
static int32_t argmax_head(const float * l, int vocab) {
    float mx = -INFINITY;
    int32_t id = 0;
    for (int i = 0; i < vocab; ++i) {
        if (l[i] > mx) {
            mx = l[i];
            id = i;
        }
    }
    return id;
}

// Device-resident greedy loop (backends with set_async / copy / greedy_step): the step's logits
// never leave the device.  After step s is launched the host records step s+1, then queues the
// greedy step (tokens of step s -> history, EOS state, step s+1's input tokens) and step s+1's
// positions / masks behind it, and launches step s+1 -- the host never waits for the device, so
// its graph work hides completely behind the device's step.  Tokens are identical to the host
// path (same first-maximum rule, same next-token rule); tests/test_parler_gpu.py checks them
// against the oracle.
static int generate_device(tts_parler * p, int32_t n_steps, int32_t * tokens_out) {
    const auto & cf = p->cfg;
    const int B = cf.batch, NH = cf.n_output_heads, V = cf.output_vocab;
    auto & be = p->be;
    const size_t rowi = (size_t)B * NH * sizeof(int32_t);
    int32_t * d_seen = (int32_t *)be.alloc(be.ctx, rowi);
    int32_t * d_next = (int32_t *)be.alloc(be.ctx, rowi);
    int32_t * d_hist = (int32_t *)be.alloc(be.ctx, rowi * (size_t)n_steps);
    int32_t * d_rep = p->sampling ? (int32_t *)be.alloc(be.ctx, 2 * rowi) : nullptr;
    // every exit frees whatever was allocated
    auto release = [&] {
        for (int32_t * q : {d_rep, d_seen, d_next, d_hist})
            if (q) be.free(be.ctx, q);
    };
    if (!d_seen || !d_next || !d_hist || (p->sampling && !d_rep)) {
        release();
        return TTS_STATUS_ALLOC_FAILED;
    }
    std::vector<int32_t> rep(2 * (size_t)B * NH);
    if (p->sampling) {
        for (size_t r = 0; r < (size_t)B * NH; ++r) rep[2 * r] = p->rep_last[r], rep[2 * r + 1] = p->rep_count[r];
        if (be.set(be.ctx, d_rep, rep.data(), 2 * rowi) != 0) {
            release();
            return TTS_STATUS_FAILED;
        }
    }
    std::vector<int32_t> seen((size_t)B * NH), next((size_t)B * NH);
    for (int b = 0; b < B; ++b)
        for (int h = 0; h < NH; ++h) {
            seen[(size_t)b * NH + h] = p->eos_seen[b][h] ? 1 : 0;
            const auto & ot = p->output_tokens[b];
            next[(size_t)b * NH + h] = p->current_step > h ? (p->eos_seen[b][h] ? cf.eos_token : ot[ot.size() - NH + h]) : cf.bos_token;
        }
    int st = be.set(be.ctx, d_seen, seen.data(), rowi);
    if (st == 0 && !p->prepared) st = prepare_step(p, true, 1);
    if (st == 0) st = launch_step(p, next.data(), true);
    for (int s = 0; st == 0 && s < n_steps; ++s) {
        const float * logits = (const float *)p->launched_out;
        if (s + 1 < n_steps) st = prepare_step(p, true, 1);  // records step s+1 while the device runs step s
        if (st == 0 && p->sampling)
            st = be.sample_step(be.ctx, logits, B, NH, V, &p->samp, p->sample_calls + s, d_rep, p->current_step + s, cf.bos_token, cf.eos_token,
                                d_seen, d_hist + (size_t)s * B * NH, d_next);
        else if (st == 0)
            st = be.greedy_step(be.ctx, logits, B, NH, V, p->current_step + s, cf.bos_token, cf.eos_token, d_seen,
                                d_hist + (size_t)s * B * NH, d_next);
        if (st == 0 && s + 1 < n_steps) {
            st = be.copy(be.ctx, p->in_tokens->data, d_next, rowi);
            if (st == 0) st = launch_step(p, nullptr, true);
        }
    }
    std::vector<int32_t> hist((size_t)n_steps * B * NH);
    if (st == 0) st = be.get(be.ctx, hist.data(), d_hist, hist.size() * sizeof(int32_t));
    if (st == 0) st = be.get(be.ctx, seen.data(), d_seen, rowi);
    if (st == 0 && d_rep) {
        st = be.get(be.ctx, rep.data(), d_rep, 2 * rowi);
        for (size_t r = 0; r < (size_t)B * NH; ++r) p->rep_last[r] = rep[2 * r], p->rep_count[r] = rep[2 * r + 1];
    }
    release();
    if (st != 0) return st;
    for (int s = 0; s < n_steps; ++s)
        for (int b = 0; b < B; ++b)
            for (int h = 0; h < NH; ++h) {
                const int32_t t = hist[((size_t)s * B + b) * NH + h];
                p->output_tokens[b].push_back(t);
                if (tokens_out) tokens_out[((size_t)b * n_steps + s) * NH + h] = t;
            }
    for (int b = 0; b < B; ++b)
        for (int h = 0; h < NH; ++h) p->eos_seen[b][h] = seen[(size_t)b * NH + h] != 0;
    p->current_step += n_steps;
    p->sample_calls += n_steps;
    return 0;
}

extern "C" int tts_parler_generate(tts_parler * p, int32_t n_steps, int32_t * tokens_out) {
    const auto & cf = p->cfg;
    if (n_steps <= 0) return 0;
    const bool dev_sample = !p->sampling || (p->be.sample_step && tts_sampling_device_ok(&p->samp, cf.output_vocab));
    if (p->be.greedy_step && p->be.set_async && p->be.copy && p->be.prepare && p->device_sampling && dev_sample)
        return generate_device(p, n_steps, tokens_out);
    const int B = cf.batch, NH = cf.n_output_heads;
    std::vector<float> logits((size_t)B * NH * cf.output_vocab);
    std::vector<int32_t> next((size_t)B * NH);
    for (int s = 0; s < n_steps; ++s) {
        // next_decoder_token_ids (model.cpp:778-785): BOS until step > head, then last token / EOS
        for (int b = 0; b < B; ++b) {
            const auto & ot = p->output_tokens[b];
            for (int h = 0; h < NH; ++h) {
                int32_t t;
                if (p->current_step > h) {
                    t = p->eos_seen[b][h] ? cf.eos_token : ot[ot.size() - NH + h];
                } else {
                    t = cf.bos_token;
                }
                next[(size_t)b * NH + h] = t;
            }
        }
        int st = p->prepared ? 0 : prepare_step(p, true, 1);
        if (st == 0) st = launch_step(p, next.data());
        if (st == 0 && s + 1 < n_steps) st = prepare_step(p, true, 1);  // overlaps the device's step s
        if (st == 0) st = finish_step(p, logits.data());
        if (st != 0) return st;
        std::vector<int32_t> drawn((size_t)B * NH);
        if (p->sampling) {  // sampler::sample per prompt, its own seeded generator
            for (int b = 0; b < B; ++b) {
                const int st2 = tts_sampler_sample(&p->samp, logits.data() + (size_t)b * NH * cf.output_vocab, NH, cf.output_vocab,
                                                   tts_sampler_call_seed(p->samp.seed, b, p->sample_calls), &p->rep_last[(size_t)b * NH],
                                                   &p->rep_count[(size_t)b * NH], &drawn[(size_t)b * NH]);
                if (st2 != 0) return st2;
            }
            p->sample_calls += 1;
        }
        for (int b = 0; b < B; ++b) {
            for (int h = 0; h < NH; ++h) {
                const int32_t t = p->sampling ? drawn[(size_t)b * NH + h]
                                              : argmax_head(logits.data() + ((size_t)b * NH + h) * cf.output_vocab, cf.output_vocab);
                p->output_tokens[b].push_back(t);
                if (tokens_out) tokens_out[((size_t)b * n_steps + s) * NH + h] = t;
                p->eos_seen[b][h] = p->eos_seen[b][h] || t == cf.eos_token;
            }
        }
        p->current_step += 1;
    }
    return 0;
}

extern "C" int32_t tts_parler_position(const tts_parler * p) { return p->position; }

// Timing harness (bench.py's cpu_baseline): continue as if the KV cache held `position` tokens, the
// rows in between keeping whatever they hold, so a slow backend can time decode steps at the GPU
// bench's KV length without running its prompt prefill.  Not for generating audio.
extern "C" int tts_parler_set_position(tts_parler * p, int32_t position) {
    if (position < p->position || position >= p->cfg.max_ctx) return TTS_STATUS_BAD_ARG;
    p->position = position;
    p->prepared = false;
    return 0;
}
extern "C" void tts_parler_set_device_sampling(tts_parler * p, int32_t on) { p->device_sampling = on != 0; }

extern "C" int64_t tts_parler_host_stats(tts_parler * p, double * us5, int reset) {
    for (int i = 0; i < 5; ++i) us5[i] = p->host_us[i];
    const int64_t n = p->host_steps;
    if (reset) {
        for (int i = 0; i < 5; ++i) p->host_us[i] = 0;
        p->host_steps = 0;
    }
    return n;
}
extern "C" int32_t tts_parler_last_graph_nodes(const tts_parler * p) { return p->last_nodes; }
extern "C" int32_t tts_parler_n_weights(const tts_parler * p) { return p ? (int32_t)p->wlist.size() : 0; }
extern "C" uint64_t tts_parler_weight(tts_parler * p, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst,
                                      uint64_t cap) {
    if (!p || i < 0 || i >= (int32_t)p->wlist.size()) return 0;
    return tg::weight_out(p->be, p->wlist[i], name, name_cap, ne, type, dst, cap);
}
extern "C" uint64_t tts_parler_weight_bytes(const tts_parler * p) { return p->wbytes; }

// The last step graph's node list (valid until the next step is prepared), e.g. for tts_hip_plan_stats.
extern "C" tts_tensor * const * tts_parler_graph(const tts_parler * p, int32_t * n_nodes) {
    if (n_nodes) *n_nodes = p ? (int32_t)p->gctx.nodes.size() : 0;
    return p ? p->gctx.nodes.data() : nullptr;
}

// Debug: node i of the last step graph -> op, type, ne[4]; copies its bytes if contiguous and cap fits.
extern "C" uint64_t tts_parler_node(tts_parler * p, int32_t i, int32_t * op, int32_t * type, int64_t * ne, void * dst, uint64_t cap) {
    if (i < 0 || i >= (int32_t)p->gctx.nodes.size()) return 0;
    const tts_tensor * t = p->gctx.nodes[i];
    *op = t->op;
    *type = t->type;
    for (int k = 0; k < 4; ++k) ne[k] = t->ne[k];
    if (!tg::is_contiguous(t) || !dst) return 0;
    const size_t nb = tg::nbytes(t);
    if (nb > cap) return 0;
    if (p->be.get(p->be.ctx, dst, t->data, nb) != 0) return 0;
    return nb;
}

extern "C" uint64_t tts_parler_get_node(tts_parler * p, const char * name, void * dst, uint64_t cap) {
    for (auto * t : p->gctx.nodes) {
        if (strcmp(t->name, name) == 0) {
            if (!tg::is_contiguous(t)) return 0;
            size_t nb = tg::nbytes(t);
            if (nb > cap) return 0;
            if (p->be.get(p->be.ctx, dst, t->data, nb) != 0) return 0;
            return nb;
        }
    }
    return 0;
}

// ---- GGUF loader path (runner_from_file + parler_tts_model::prep_constants / assign_weight) ----
namespace tts {
void dac_write_synthetic(const tts_dac_config * cfg, tts_gguf_writer * w);
}

static bool gguf_u32(const tts_gguf * g, std::initializer_list<const char *> keys, int32_t * out) {
    for (const char * k : keys) {  // search_for_gguf_keys: first key present wins
        const int64_t i = tts_gguf_find_key(g, k);
        uint32_t v;
        if (i >= 0 && tts_gguf_get_u32(g, i, &v)) {
            *out = (int32_t)v;
            return true;
        }
    }
    return false;
}

static int64_t gguf_dim(const tts_gguf * g, const char * name, int d) {
    const int64_t i = tts_gguf_find_tensor(g, name);
    if (i < 0) return -1;
    int64_t ne[4];
    tts_gguf_tensor_ndims(g, i, ne);
    return ne[d];
}

extern "C" int tts_parler_config_from_gguf(const tts_gguf * g, tts_parler_config * c) {
    if (!g || !c) return TTS_STATUS_BAD_ARG;
    const int64_t ak = tts_gguf_find_key(g, "general.architecture");
    if (ak >= 0 && (!tts_gguf_get_str(g, ak) || strcmp(tts_gguf_get_str(g, ak), "parler-tts") != 0)) {
        fprintf(stderr, "gguf: not a parler-tts file\n");
        return TTS_STATUS_BAD_ARG;
    }
    // prep_constants (model.cpp:51-108); encode_length is the one required key
    if (!gguf_u32(g, {"parler-tts.decoder.encode_length", "encode_length"}, &c->n_encode)) {
        fprintf(stderr, "gguf: key 'parler-tts.decoder.encode_length' must be specified\n");
        return TTS_STATUS_BAD_ARG;
    }
    gguf_u32(g, {"parler-tts.decoder.hidden_size", "hidden_size"}, &c->hidden_size);
    gguf_u32(g, {"parler-tts.decoder.output_heads", "output_heads"}, &c->n_output_heads);
    gguf_u32(g, {"parler-tts.decoder.attention.head_count", "attn_heads"}, &c->n_attn_heads);
    gguf_u32(g, {"parler-tts.decoder.out_vocab_size", "out_vocab_size"}, &c->output_vocab);
    gguf_u32(g, {"parler-tts.decoder.audio_vocab_size", "audio_vocab_size"}, &c->audio_vocab);
    gguf_u32(g, {"parler-tts.decoder.num_hidden_layers", "num_hidden_layers"}, &c->n_layers);
    gguf_u32(g, {"audio.bos_token_id", "bos_token_id"}, &c->bos_token);
    gguf_u32(g, {"audio.eos_token_id", "eos_token_id"}, &c->eos_token);
    // sizes the reference takes from the tensors themselves
    const int64_t ffn = gguf_dim(g, "decoder.layers.0.fc1.weight", 1);
    const int64_t pv = gguf_dim(g, "decoder.embed_prompts", 1);
    const int64_t mp = gguf_dim(g, "decoder.positional_embed", 1);
    const int64_t wt = tts_gguf_find_tensor(g, "decoder.layers.0.self_attn.q_proj.weight");
    const int64_t ht = tts_gguf_find_tensor(g, "decoder.lm_heads.0.weight.head");
    if (ffn < 0 || pv < 0 || mp < 0 || wt < 0 || ht < 0) {
        fprintf(stderr, "gguf: decoder tensors missing\n");
        return TTS_STATUS_BAD_ARG;
    }
    c->ffn_size = (int32_t)ffn;
    c->prompt_vocab = (int32_t)pv;
    c->max_positions = (int32_t)mp;
    c->weight_type = tts_gguf_tensor_type(g, wt);
    c->head_type = tts_gguf_tensor_type(g, ht);
    c->use_cross_attn = tts_gguf_find_tensor(g, "decoder.layers.0.encoder_attn.q_proj.weight") >= 0 ? 1 : 0;
    if (!c->use_cross_attn) {
        fprintf(stderr, "gguf: parler files without cross attention are not supported\n");
        return TTS_STATUS_UNSUPPORTED;
    }
    return TTS_STATUS_SUCCESS;
}

extern "C" tts_parler * tts_parler_create_from_gguf(const tts_backend_iface * be, const tts_parler_config * cfg, const tts_gguf * g) {
    if (!be || !cfg || !g) return nullptr;
    return parler_create(be, cfg, g);
}

extern "C" int tts_parler_write_synthetic_gguf(const tts_parler_config * cfg, const tts_dac_config * dac_cfg, const char * path) {
    if (!cfg || !path) return TTS_STATUS_BAD_ARG;
    tts_parler p;  // declarations only: no backend, no buffers
    p.cfg = *cfg;
    std::vector<wspec> specs;
    declare_weights(&p, specs);
    tts_gguf_writer * w = tts_gguf_writer_new();
    const auto & c = *cfg;
    // the keys prep_constants reads (parler_tts_gguf_encoder.py writes them)
    tts_gguf_set_str(w, "general.architecture", "parler-tts");
    tts_gguf_set_u32(w, "parler-tts.decoder.encode_length", (uint32_t)c.n_encode);
    tts_gguf_set_u32(w, "parler-tts.decoder.hidden_size", (uint32_t)c.hidden_size);
    tts_gguf_set_u32(w, "parler-tts.decoder.output_heads", (uint32_t)c.n_output_heads);
    tts_gguf_set_u32(w, "parler-tts.decoder.context_length", (uint32_t)c.max_ctx);
    tts_gguf_set_u32(w, "parler-tts.decoder.attention.head_count", (uint32_t)c.n_attn_heads);
    tts_gguf_set_u32(w, "parler-tts.decoder.out_vocab_size", (uint32_t)c.output_vocab);
    tts_gguf_set_u32(w, "parler-tts.decoder.audio_vocab_size", (uint32_t)c.audio_vocab);
    tts_gguf_set_u32(w, "parler-tts.decoder.max_generation", (uint32_t)c.max_ctx);
    tts_gguf_set_u32(w, "parler-tts.decoder.num_hidden_layers", (uint32_t)c.n_layers);
    tts_gguf_set_u32(w, "audio.bos_token_id", (uint32_t)c.bos_token);
    tts_gguf_set_u32(w, "audio.eos_token_id", (uint32_t)c.eos_token);
    int st = TTS_STATUS_SUCCESS;
    std::vector<char> host;
    for (auto & s : specs) {
        synth_host(s, host);
        const int nd = s.t->ne[1] > 1 ? 2 : 1;
        st = tts_gguf_add_tensor(w, gguf_name(s.t).c_str(), s.t->type, nd, s.t->ne, host.data(), host.size());
        if (st != TTS_STATUS_SUCCESS) break;
    }
    if (st == TTS_STATUS_SUCCESS && dac_cfg) dac_write_synthetic(dac_cfg, w);
    if (st == TTS_STATUS_SUCCESS) st = tts_gguf_writer_write(w, path);
    tts_gguf_writer_free(w);
    return st;
}
