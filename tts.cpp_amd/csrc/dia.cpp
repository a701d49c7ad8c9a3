// Dia-1.6B runner: builds the same graphs as dia_runner::build_dia_graph
// (/root/reference/src/models/dia/model.cpp:705-720): the encoder over the padded 1024-token text
// context (build_dia_encoder, :364-419) fused into the first decoder step together with the cross
// K/V store (build_dia_cross_kv_store, :476-514), and the decoder step (build_dia_decoder, :516-637)
// with the GQA repeat-interleave KV store (build_dia_self_kv_store, :443-474).  Classifier-free
// guidance runs the conditioned and unconditioned sequences as the graph's batch of 2; the heads'
// cfg_scale (util.cpp:175-200, a CPU map_custom2 in the reference) is the same MAP_CUSTOM2 node here,
// run by the backend on the device: cond + 3 * (cond - uncond), each op rounded to f32.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tts_runners.h"
#include "graph.h"
#include "synth.h"

using namespace tts;

struct dia_enc_layer {
    tts_tensor *self_attn_norm, *q, *k, *v, *o, *mlp_norm, *gate, *up, *out;
};
struct dia_dec_layer {
    tts_tensor *self_attn_norm, *q, *k, *v, *o;
    tts_tensor *cross_attn_norm, *cq, *ck, *cv, *co;
    tts_tensor *mlp_norm, *gate, *up, *out;
};

struct tts_dia {
    tts_dia_config cfg;
    tts_backend_iface be;
    tg::context wctx;
    void * wbuf = nullptr;
    size_t wbytes = 0;
    void * kvbuf = nullptr;
    tts_tensor *enc_embd = nullptr, *enc_norm = nullptr, *dec_norm = nullptr;
    std::vector<dia_enc_layer> enc;
    std::vector<dia_dec_layer> dec;
    std::vector<tts_tensor *> embds, heads;
    std::vector<tts_tensor *> wlist;  // every weight, declaration order (tts_dia_weight)
    std::vector<tts_tensor *> k_l, v_l, cross_k_l, cross_v_l;
    char * arena = nullptr;
    size_t arena_size = 0;
    tg::context gctx;
    tts_tensor * res = nullptr;
    tts_tensor *in_text = nullptr, *in_enc_pos = nullptr, *in_enc_mask = nullptr, *in_audio = nullptr, *in_pos = nullptr;
    int32_t position = 0;
    int32_t prompt_size = 0;
    int32_t last_nodes = 0;
    // seeded sampling of the CFG heads (tts_dia_set_sampling); greedy when off
    bool sampling = false;
    tts_sampling samp{};
    int64_t sample_calls = 0;
    std::vector<int32_t> rep_last, rep_count;  // [heads]
};

extern "C" void tts_dia_set_sampling(tts_dia * p, const tts_sampling * cfg) {
    p->sampling = cfg != nullptr;
    if (cfg) p->samp = *cfg;
}

extern "C" void tts_dia_default_config(tts_dia_config * c) {
    // dia_model defaults (src/models/dia/model.h:62-85); FFN widths of Dia-1.6B
    c->n_output_heads = 9;
    c->n_encoder_layers = 12;
    c->n_decoder_layers = 18;
    c->encoder_hidden_size = 1024;
    c->decoder_hidden_size = 2048;
    c->encoder_attn_heads = 16;
    c->decoder_attn_heads = 16;
    c->decoder_query_heads = 4;
    c->head_size = 128;
    c->encoder_ffn_size = 4096;
    c->decoder_ffn_size = 8192;
    c->output_vocab_size = 1028;
    c->encoder_vocab_size = 256;
    c->max_generation_size = 3072;
    c->max_encoder_context_length = 1024;
    c->weight_type = TTS_TYPE_Q8_0;
    c->head_type = TTS_TYPE_F32;
    c->cfg_scale = 3.0f;
    c->seed = 0x5EED;
    c->arena_bytes = 0;
}

static tts_tensor * wnew(tts_dia * p, std::vector<std::pair<tts_tensor *, int>> & specs, int type, int64_t ne0, int64_t ne1, int kind,
                         const std::string & name) {
    tts_tensor * t = ne1 > 1 ? tg::new_tensor_2d(p->wctx, type, ne0, ne1) : tg::new_tensor_1d(p->wctx, type, ne0);
    tg::set_name(t, name);
    t->flags |= tg::TG_FLAG_PERSIST;
    specs.push_back({t, kind});
    return t;
}

static bool upload_weights(tts_dia * p, std::vector<std::pair<tts_tensor *, int>> & specs) {
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
        if (s.second == 1) synth_f32((float *)host.data(), (size_t)(K * rows), seed, 0.1f, 1.0f);  // norm weights ~1
        else synth_fill(t->type, host.data(), rows, K, seed, s.second == 3 ? 0.25f : 0.02f);
        if (p->be.set_tensor(p->be.ctx, t, host.data()) != 0) return false;
    }
    return true;
}

extern "C" tts_dia * tts_dia_create(const tts_backend_iface * be, const tts_dia_config * cfg) {
    auto * p = new tts_dia();
    p->cfg = *cfg;
    p->be = *be;
    const auto & cf = p->cfg;
    const int64_t E = cf.encoder_hidden_size, D = cf.decoder_hidden_size, hd = cf.head_size;
    const int64_t EA = (int64_t)cf.encoder_attn_heads * hd, DA = (int64_t)cf.decoder_attn_heads * hd;
    const int64_t DKV = DA / cf.decoder_query_heads;
    std::vector<std::pair<tts_tensor *, int>> specs;
    p->enc_embd = wnew(p, specs, cf.weight_type, E, cf.encoder_vocab_size, 3, "encoder.embedding");
    p->enc.resize(cf.n_encoder_layers);
    for (int l = 0; l < cf.n_encoder_layers; ++l) {
        auto & L = p->enc[l];
        const std::string pre = "encoder.layers." + std::to_string(l);
        L.self_attn_norm = wnew(p, specs, TTS_TYPE_F32, E, 1, 1, pre + ".self_attn_norm");
        L.q = wnew(p, specs, cf.weight_type, E, EA, 0, pre + ".q");
        L.k = wnew(p, specs, cf.weight_type, E, EA, 0, pre + ".k");
        L.v = wnew(p, specs, cf.weight_type, E, EA, 0, pre + ".v");
        L.o = wnew(p, specs, cf.weight_type, EA, E, 0, pre + ".o");
        L.mlp_norm = wnew(p, specs, TTS_TYPE_F32, E, 1, 1, pre + ".mlp_norm");
        L.gate = wnew(p, specs, cf.weight_type, E, cf.encoder_ffn_size, 0, pre + ".gate");
        L.up = wnew(p, specs, cf.weight_type, E, cf.encoder_ffn_size, 0, pre + ".up");
        L.out = wnew(p, specs, cf.weight_type, cf.encoder_ffn_size, E, 0, pre + ".out");
    }
    p->enc_norm = wnew(p, specs, TTS_TYPE_F32, E, 1, 1, "encoder.norm");
    for (int i = 0; i < cf.n_output_heads; ++i)
        p->embds.push_back(wnew(p, specs, cf.weight_type, D, cf.output_vocab_size, 3, "decoder.embds." + std::to_string(i)));
    p->dec.resize(cf.n_decoder_layers);
    for (int l = 0; l < cf.n_decoder_layers; ++l) {
        auto & L = p->dec[l];
        const std::string pre = "decoder.layers." + std::to_string(l);
        L.self_attn_norm = wnew(p, specs, TTS_TYPE_F32, D, 1, 1, pre + ".self_attn_norm");
        L.q = wnew(p, specs, cf.weight_type, D, DA, 0, pre + ".self_attn_q");
        L.k = wnew(p, specs, cf.weight_type, D, DKV, 0, pre + ".self_attn_k");
        L.v = wnew(p, specs, cf.weight_type, D, DKV, 0, pre + ".self_attn_v");
        L.o = wnew(p, specs, cf.weight_type, DA, D, 0, pre + ".self_attn_o");
        L.cross_attn_norm = wnew(p, specs, TTS_TYPE_F32, D, 1, 1, pre + ".cross_attn_norm");
        L.cq = wnew(p, specs, cf.weight_type, D, DA, 0, pre + ".cross_attn_q");
        L.ck = wnew(p, specs, cf.weight_type, E, DA, 0, pre + ".cross_attn_k");
        L.cv = wnew(p, specs, cf.weight_type, E, DA, 0, pre + ".cross_attn_v");
        L.co = wnew(p, specs, cf.weight_type, DA, D, 0, pre + ".cross_attn_o");
        L.mlp_norm = wnew(p, specs, TTS_TYPE_F32, D, 1, 1, pre + ".mlp_norm");
        L.gate = wnew(p, specs, cf.weight_type, D, cf.decoder_ffn_size, 0, pre + ".gate");
        L.up = wnew(p, specs, cf.weight_type, D, cf.decoder_ffn_size, 0, pre + ".up");
        L.out = wnew(p, specs, cf.weight_type, cf.decoder_ffn_size, D, 0, pre + ".out");
    }
    p->dec_norm = wnew(p, specs, TTS_TYPE_F32, D, 1, 1, "decoder.norm");
    for (int i = 0; i < cf.n_output_heads; ++i)
        p->heads.push_back(wnew(p, specs, cf.head_type, D, cf.output_vocab_size, 0, "decoder.heads." + std::to_string(i)));
    for (auto & s : specs) p->wlist.push_back(s.first);
    if (!upload_weights(p, specs)) {
        fprintf(stderr, "dia: weight allocation/upload failed\n");
        tts_dia_free(p);
        return nullptr;
    }
    // dia_kv_cache_init: self K/V [DA * max_gen * 2], cross K [hd, H, 2, enc_ctx], cross V [enc_ctx, hd, H, 2]
    const size_t selfb = (size_t)DA * cf.max_generation_size * 2 * 4;
    const size_t crossb = (size_t)DA * cf.max_encoder_context_length * 2 * 4;
    const size_t total = (size_t)cf.n_decoder_layers * 2 * (selfb + crossb);
    p->kvbuf = p->be.alloc(p->be.ctx, total);
    if (!p->kvbuf) {
        tts_dia_free(p);
        return nullptr;
    }
    p->be.memset(p->be.ctx, p->kvbuf, 0, total);
    char * kp = (char *)p->kvbuf;
    for (int l = 0; l < cf.n_decoder_layers; ++l) {
        tts_tensor * t;
        t = tg::new_tensor_1d(p->wctx, TTS_TYPE_F32, DA * cf.max_generation_size * 2);
        t->data = kp, kp += selfb, p->k_l.push_back(t);
        t = tg::new_tensor_1d(p->wctx, TTS_TYPE_F32, DA * cf.max_generation_size * 2);
        t->data = kp, kp += selfb, p->v_l.push_back(t);
        t = tg::new_tensor_4d(p->wctx, TTS_TYPE_F32, hd, cf.decoder_attn_heads, 2, cf.max_encoder_context_length);
        t->data = kp, kp += crossb, p->cross_k_l.push_back(t);
        t = tg::new_tensor_4d(p->wctx, TTS_TYPE_F32, cf.max_encoder_context_length, hd, cf.decoder_attn_heads, 2);
        t->data = kp, kp += crossb, p->cross_v_l.push_back(t);
    }
    p->arena_size = cf.arena_bytes ? cf.arena_bytes : (2ull << 30);
    p->arena = (char *)p->be.alloc(p->be.ctx, p->arena_size);
    if (!p->arena) {
        tts_dia_free(p);
        return nullptr;
    }
    return p;
}

extern "C" void tts_dia_free(tts_dia * p) {
    if (!p) return;
    if (p->arena) p->be.free(p->be.ctx, p->arena);
    if (p->kvbuf) p->be.free(p->be.ctx, p->kvbuf);
    if (p->wbuf) p->be.free(p->be.ctx, p->wbuf);
    delete p;
}

static tts_tensor * rms(tg::context & c, tts_tensor * x, tts_tensor * w) {
    return tg::mul(c, tg::rms_norm(c, x, 0.00001f), w);  // dia_layer_norm (model.cpp:344-349)
}

static tts_tensor * rope_neox(tg::context & c, tts_tensor * x, tts_tensor * pos, int hd) {
    // ggml_rope(ctx, x, pos, hd, 2): freq_base 10000, no scaling
    return tg::rope_ext(c, x, pos, nullptr, hd, 2, 0, 10000.0f, 1.0f, 0.0f, 1.0f, 0.0f, 0.0f);
}

// repeat_interleave_dim1 (model.cpp:421-434): [ne0, n, ne2, ne3] -> each slice along dim 1 repeated
static tts_tensor * repeat_interleave_dim1(tg::context & c, tts_tensor * a, int repeat) {
    tts_tensor * running = nullptr;
    for (int64_t i = 0; i < a->ne[1]; ++i) {
        tts_tensor * t = tg::cont(c, tg::view_4d(c, a, a->ne[0], 1, a->ne[2], a->ne[3], a->nb[1], a->nb[2], a->nb[3], (size_t)i * a->nb[1]));
        tts_tensor * shape = tg::new_tensor_4d(c, TTS_TYPE_F32, a->ne[0], repeat, a->ne[2], a->ne[3]);
        t = tg::repeat(c, t, shape);
        running = i == 0 ? t : tg::concat(c, running, t, 1);
    }
    return running;
}

static tts_tensor * build_encoder(tts_dia * p, tg::context & c) {
    const auto & cf = p->cfg;
    const int64_t E = cf.encoder_hidden_size, T = cf.max_encoder_context_length, hd = cf.head_size, H = cf.encoder_attn_heads;
    p->in_text = tg::new_tensor_1d(c, TTS_TYPE_I32, T * 2);
    tg::set_input(p->in_text);
    p->in_enc_pos = tg::new_tensor_1d(c, TTS_TYPE_I32, T);
    tg::set_input(p->in_enc_pos);
    p->in_enc_mask = tg::new_tensor_2d(c, TTS_TYPE_F32, T, T);
    tg::set_input(p->in_enc_mask);
    tts_tensor * cur = tg::reshape_3d(c, tg::get_rows(c, p->enc_embd, p->in_text), E, T, 2);
    for (auto & L : p->enc) {
        tts_tensor * residual = cur;
        cur = rms(c, cur, L.self_attn_norm);
        tts_tensor * Q = tg::mul_mat(c, L.q, cur);
        tts_tensor * K = tg::mul_mat(c, L.k, cur);
        tts_tensor * V = tg::mul_mat(c, L.v, cur);
        Q = rope_neox(c, tg::cont(c, tg::reshape_4d(c, Q, hd, H, T, 2)), p->in_enc_pos, (int)hd);
        K = rope_neox(c, tg::cont(c, tg::reshape_4d(c, K, hd, H, T, 2)), p->in_enc_pos, (int)hd);
        tts_tensor * q = tg::cont(c, tg::permute(c, Q, 0, 2, 1, 3));
        tts_tensor * k = tg::cont(c, tg::permute(c, K, 0, 2, 1, 3));
        tts_tensor * kq = tg::soft_max_ext(c, tg::mul_mat(c, k, q), p->in_enc_mask, 1.0f, 0.0f);
        tts_tensor * v = tg::cont_4d(c, tg::transpose(c, V), T, hd, H, 2);
        tts_tensor * kqv = tg::mul_mat(c, kq, v);
        cur = tg::cont_3d(c, tg::permute(c, kqv, 2, 0, 1, 3), H * hd, T, 2);
        cur = tg::add(c, tg::mul_mat(c, L.o, cur), residual);
        tts_tensor * residual_mlp = cur;
        cur = rms(c, cur, L.mlp_norm);
        cur = tg::mul(c, tg::silu(c, tg::mul_mat(c, L.gate, cur)), tg::mul_mat(c, L.up, cur));
        cur = tg::add(c, tg::mul_mat(c, L.out, cur), residual_mlp);
    }
    return rms(c, cur, p->enc_norm);
}

static void build_cross_kv_store(tts_dia * p, tg::context & c, tts_tensor * enc, int l) {
    const auto & cf = p->cfg;
    const int64_t E = cf.encoder_hidden_size, T = cf.max_encoder_context_length, hd = cf.head_size, H = cf.decoder_attn_heads;
    auto & L = p->dec[l];
    tts_tensor * keys = tg::cont(c, tg::view_3d(c, enc, E, p->prompt_size, 2, 4 * E, 4 * E * T, 0));
    tts_tensor * k = tg::mul_mat(c, L.ck, keys);
    tts_tensor * posv = tg::view_1d(c, p->in_enc_pos, p->prompt_size, 0);
    k = rope_neox(c, tg::cont(c, tg::reshape_4d(c, k, hd, H, p->prompt_size, 2)), posv, (int)hd);
    k = tg::cont(c, tg::permute(c, k, 0, 1, 3, 2));
    tts_tensor * kv = tg::view_4d(c, p->cross_k_l[l], hd, H, 2, p->prompt_size, 4 * hd, 4 * hd * H, 4 * hd * H * 2, 0);
    tg::build_forward_expand(c, tg::cpy(c, k, kv));
    tts_tensor * v = tg::cont(c, tg::transpose(c, tg::mul_mat(c, L.cv, enc)));
    v = tg::cont_4d(c, v, T, hd, H, 2);
    tts_tensor * vv = tg::view_4d(c, p->cross_v_l[l], T, hd, H, 2, 4 * T, 4 * T * hd, 4 * T * hd * H, 0);
    tg::build_forward_expand(c, tg::cpy(c, v, vv));
}

// build_dia_graph: the encoder + cross K/V store on the encoder step, then one decoder step
static tts_tensor * build_graph(tts_dia * p, bool encoder_step) {
    const auto & cf = p->cfg;
    const int64_t D = cf.decoder_hidden_size, hd = cf.head_size, H = cf.decoder_attn_heads, T = cf.max_encoder_context_length;
    const int64_t DA = H * hd, nkv = H / cf.decoder_query_heads, G = cf.max_generation_size;
    const int64_t full = p->position + 1;
    tg::context & c = p->gctx;
    c.reset();
    tts_tensor * enc = encoder_step ? build_encoder(p, c) : nullptr;
    if (enc) tg::build_forward_expand(c, enc);

    p->in_pos = tg::new_tensor_1d(c, TTS_TYPE_I32, 1);
    tg::set_input(p->in_pos);
    // build_dia_decoder_inp_embd (model.cpp:327-342): head i's (cond, uncond) ids at stride n_heads
    p->in_audio = tg::new_tensor_1d(c, TTS_TYPE_I32, (int64_t)cf.n_output_heads * 2);
    tg::set_input(p->in_audio);
    tts_tensor * cur = nullptr;
    for (int i = 0; i < cf.n_output_heads; ++i) {
        tts_tensor * view = tg::view_1d(c, p->in_audio, 2, (size_t)i * 4);
        view->nb[0] = (size_t)cf.n_output_heads * 4;
        tts_tensor * e = tg::get_rows(c, p->embds[i], view);
        cur = i == 0 ? e : tg::add(c, e, cur);
    }
    for (int l = 0; l < cf.n_decoder_layers; ++l) {
        auto & L = p->dec[l];
        tts_tensor * residual = cur;
        cur = rms(c, cur, L.self_attn_norm);
        {
            tts_tensor * Q = tg::mul_mat(c, L.q, cur);
            tts_tensor * K = tg::mul_mat(c, L.k, cur);
            tts_tensor * V = tg::mul_mat(c, L.v, cur);
            // build_dia_self_kv_store (model.cpp:443-474)
            tts_tensor * kc = tg::view_2d(c, p->k_l[l], DA, 2, 4 * DA * G, 4 * DA * (size_t)p->position);
            tts_tensor * k = rope_neox(c, tg::cont(c, tg::reshape_4d(c, K, hd, nkv, 1, 2)), p->in_pos, (int)hd);
            k = repeat_interleave_dim1(c, tg::cont(c, tg::reshape_4d(c, k, hd, nkv, 1, 2)), cf.decoder_query_heads);
            k = tg::cont(c, tg::reshape_2d(c, k, DA, 2));
            tg::build_forward_expand(c, tg::cpy(c, k, kc));
            tts_tensor * vc = tg::view_2d(c, p->v_l[l], DA, 2, 4 * DA * G, 4 * DA * (size_t)p->position);
            tts_tensor * v = repeat_interleave_dim1(c, tg::cont(c, tg::reshape_4d(c, V, hd, nkv, 1, 2)), cf.decoder_query_heads);
            tg::build_forward_expand(c, tg::cpy(c, v, vc));

            tts_tensor * kk = tg::view_4d(c, p->k_l[l], hd, H, full, 2, 4 * hd, 4 * DA, 4 * DA * G, 0);
            kk = tg::cont(c, tg::permute(c, kk, 0, 2, 1, 3));
            tts_tensor * vv = tg::view_3d(c, p->v_l[l], DA, full, 2, 4 * DA, 4 * DA * G, 0);
            vv = tg::cont_4d(c, tg::transpose(c, vv), full, hd, H, 2);
            Q = rope_neox(c, tg::cont(c, tg::reshape_4d(c, Q, hd, H, 1, 2)), p->in_pos, (int)hd);
            tts_tensor * q = tg::cont(c, tg::permute(c, Q, 0, 2, 1, 3));
            tts_tensor * kq = tg::soft_max_ext(c, tg::mul_mat(c, tg::cont(c, kk), q), nullptr, 1.0f, 0.0f);
            tts_tensor * kqv = tg::mul_mat(c, kq, vv);
            tts_tensor * merged = tg::cont(c, tg::permute(c, kqv, 2, 0, 1, 3));
            cur = tg::cont_3d(c, merged, D, 1, 2);
            cur = tg::mul_mat(c, L.o, cur);
        }
        cur = tg::cont_2d(c, cur, cur->ne[0], 2);
        cur = tg::add(c, cur, residual);
        tts_tensor * residual_cross = cur;
        cur = rms(c, cur, L.cross_attn_norm);
        {
            tts_tensor * cQ = tg::mul_mat(c, L.cq, cur);
            if (encoder_step) build_cross_kv_store(p, c, enc, l);
            tts_tensor * ck = tg::view_4d(c, p->cross_k_l[l], hd, H, 2, T, 4 * hd, 4 * hd * H, 4 * hd * H * 2, 0);
            ck = tg::cont(c, tg::permute(c, tg::permute(c, ck, 0, 1, 3, 2), 0, 2, 1, 3));
            tts_tensor * cv = tg::cont(c, tg::view_4d(c, p->cross_v_l[l], T, hd, H, 2, 4 * T, 4 * T * hd, 4 * T * hd * H, 0));
            cQ = rope_neox(c, tg::cont(c, tg::reshape_4d(c, cQ, hd, H, 1, 2)), p->in_pos, (int)hd);
            tts_tensor * cq = tg::cont(c, tg::permute(c, cQ, 0, 2, 1, 3));
            tts_tensor * ckq = tg::soft_max_ext(c, tg::mul_mat(c, ck, cq), nullptr, 1.0f, 0.0f);
            tts_tensor * ckqv = tg::mul_mat(c, ckq, cv);
            tts_tensor * merged = tg::cont(c, tg::permute(c, ckqv, 2, 0, 1, 3));
            cur = tg::cont_3d(c, merged, D, 1, 2);
            cur = tg::mul_mat(c, L.co, cur);
        }
        cur = tg::cont_2d(c, cur, cur->ne[0], 2);
        cur = tg::add(c, cur, residual_cross);
        tts_tensor * residual_mlp = cur;
        cur = rms(c, cur, L.mlp_norm);
        cur = tg::mul(c, tg::silu(c, tg::mul_mat(c, L.gate, cur)), tg::mul_mat(c, L.up, cur));
        cur = tg::mul_mat(c, L.out, cur);
        cur = tg::add(c, cur, residual_mlp);
    }
    cur = rms(c, cur, p->dec_norm);
    // build_dia_head_outputs (model.cpp:358-371): heads concatenated on dim 2, then cfg_scale
    tts_tensor * out = nullptr;
    for (int i = 0; i < cf.n_output_heads; ++i) {
        tts_tensor * h = tg::mul_mat(c, p->heads[i], cur);
        out = i == 0 ? h : tg::concat(c, out, h, 2);
    }
    tts_tensor * cond = tg::cont(c, tg::view_2d(c, out, out->ne[0], out->ne[2], out->nb[2], 0));
    tts_tensor * uncond = tg::cont(c, tg::view_2d(c, out, out->ne[0], out->ne[2], out->nb[2], out->nb[1]));
    // ggml_map_custom2(cond, uncond, cfg_scale) as the reference builds it, run on the device
    tts_tensor * logits = tg::map_custom2(c, cond, uncond, TTS_CUSTOM_CFG_SCALE);
    memcpy(&logits->op_params[1], &cf.cfg_scale, sizeof(float));
    tg::set_name(logits, "decoder_output");
    tg::set_output(logits);
    tg::build_forward_expand(c, logits);
    return logits;
}

static int prepare(tts_dia * p, bool encoder_step) {
    const auto & cf = p->cfg;
    if (p->position + 1 > cf.max_generation_size) return TTS_STATUS_BAD_ARG;
    p->res = build_graph(p, encoder_step);
    if (!tg::alloc_graph(p->gctx, p->arena, p->arena_size, true)) {
        fprintf(stderr, "dia: compute arena too small (%zu needed)\n", p->gctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    p->last_nodes = (int32_t)p->gctx.nodes.size();
    return 0;
}

static int run_step(tts_dia * p, bool encoder_step, const int32_t * text, int32_t n_text, const int32_t * audio, float * logits) {
    const auto & cf = p->cfg;
    int st = prepare(p, encoder_step);
    if (st != 0) return st;
    auto & be = p->be;
    if (encoder_step) {
        // set_inputs (model.cpp:722-737): text ids for (cond, uncond), positions, padded-block mask
        const int64_t T = cf.max_encoder_context_length;
        std::vector<int32_t> pos(T);
        std::vector<float> mask((size_t)T * T);
        for (int64_t i = 0; i < T; ++i) {
            pos[i] = (int32_t)i;
            for (int64_t j = 0; j < T; ++j)
                mask[(size_t)i * T + j] = (i < n_text) ? (j < n_text ? 0.0f : -INFINITY) : (j >= n_text ? 0.0f : -INFINITY);
        }
        st |= be.set(be.ctx, p->in_text->data, text, sizeof(int32_t) * T * 2);
        st |= be.set(be.ctx, p->in_enc_pos->data, pos.data(), sizeof(int32_t) * T);
        st |= be.set(be.ctx, p->in_enc_mask->data, mask.data(), mask.size() * sizeof(float));
    }
    std::vector<int32_t> a2((size_t)cf.n_output_heads * 2);
    for (int i = 0; i < cf.n_output_heads; ++i) a2[i] = a2[cf.n_output_heads + i] = audio[i];
    st |= be.set(be.ctx, p->in_audio->data, a2.data(), a2.size() * sizeof(int32_t));
    const int32_t pp = p->position;
    st |= be.set(be.ctx, p->in_pos->data, &pp, sizeof(int32_t));
    if (st != 0) return TTS_STATUS_FAILED;
    st = be.compute(be.ctx, p->gctx.nodes.data(), (int)p->gctx.nodes.size());
    if (st == 0 && logits) st = be.get(be.ctx, logits, p->res->data, sizeof(float) * cf.n_output_heads * cf.output_vocab_size);
    if (st == 0) st = be.synchronize(be.ctx);
    if (st == 0) p->position += 1;
    return st;
}

// The encoder step: text [2][max_encoder_context_length] byte tokens (cond row, then the uncond
// row, both padded), n_text real tokens, the first audio tokens [n_output_heads]; logits [heads][vocab].
extern "C" int tts_dia_prefill(tts_dia * p, const int32_t * text, int32_t n_text, const int32_t * audio, float * logits) {
    if (n_text < 1 || n_text > p->cfg.max_encoder_context_length) return TTS_STATUS_BAD_ARG;
    p->position = 0;
    p->prompt_size = n_text;
    p->sample_calls = 0;  // a new prompt: sampler::reset (dia/model.cpp:883)
    p->rep_last.assign(p->cfg.n_output_heads, -1);
    p->rep_count.assign(p->cfg.n_output_heads, 0);
    return run_step(p, true, text, n_text, audio, logits);
}

extern "C" int tts_dia_decode(tts_dia * p, const int32_t * audio, float * logits) {
    if (p->prompt_size == 0) return TTS_STATUS_FAILED;
    return run_step(p, false, nullptr, 0, audio, logits);
}

// generate loop with greedy heads (sampler::max per head, fed back as the next step's tokens for
// both CFG rows): on a backend with graph plans and greedy_step, step s+1 is recorded while the
// device runs step s and the samples never leave the device until the end.  tokens_out [steps][heads].
extern "C" int tts_dia_generate(tts_dia * p, const int32_t * first_audio, int32_t n_steps, int32_t * tokens_out) {
    const auto & cf = p->cfg;
    auto & be = p->be;
    const int NH = cf.n_output_heads;
    if (p->prompt_size == 0 || n_steps <= 0) return n_steps <= 0 ? 0 : TTS_STATUS_FAILED;
    const bool dev_sample = !p->sampling || (be.sample_step && tts_sampling_device_ok(&p->samp, cf.output_vocab_size));
    if (!(be.greedy_step && be.set_async && be.copy && be.prepare && be.launch && dev_sample)) {
        std::vector<float> lg((size_t)NH * cf.output_vocab_size);
        std::vector<int32_t> a(first_audio, first_audio + NH);
        for (int s = 0; s < n_steps; ++s) {
            int st = run_step(p, false, nullptr, 0, a.data(), lg.data());
            if (st != 0) return st;
            if (p->sampling) {  // sampler::sample over the CFG-combined heads (dia/model.cpp:855)
                st = tts_sampler_sample(&p->samp, lg.data(), NH, cf.output_vocab_size, tts_sampler_call_seed(p->samp.seed, 0, p->sample_calls++),
                                        p->rep_last.data(), p->rep_count.data(), a.data());
                if (st != 0) return st;
                for (int h = 0; h < NH; ++h) tokens_out[(size_t)s * NH + h] = a[h];
                continue;
            }
            for (int h = 0; h < NH; ++h) {
                const float * l = lg.data() + (size_t)h * cf.output_vocab_size;
                int best = 0;
                for (int i = 1; i < cf.output_vocab_size; ++i)
                    if (l[i] > l[best]) best = i;
                a[h] = tokens_out[(size_t)s * NH + h] = best;
            }
        }
        return 0;
    }
    const size_t rowi = (size_t)NH * sizeof(int32_t);
    int32_t * d_seen = (int32_t *)be.alloc(be.ctx, rowi);
    int32_t * d_next = (int32_t *)be.alloc(be.ctx, rowi);
    int32_t * d_hist = (int32_t *)be.alloc(be.ctx, rowi * (size_t)n_steps);
    int32_t * d_rep = p->sampling ? (int32_t *)be.alloc(be.ctx, 2 * rowi) : nullptr;
    int st = (d_seen && d_next && d_hist && (!p->sampling || d_rep)) ? 0 : TTS_STATUS_ALLOC_FAILED;
    if (st == 0) st = be.memset(be.ctx, d_seen, 0, rowi);
    std::vector<int32_t> rep(2 * (size_t)NH);
    if (st == 0 && d_rep) {
        for (int h = 0; h < NH; ++h) rep[2 * h] = p->rep_last[h], rep[2 * h + 1] = p->rep_count[h];
        st = be.set(be.ctx, d_rep, rep.data(), 2 * rowi);
    }
    std::vector<int32_t> a2((size_t)NH * 2);
    for (int h = 0; h < NH; ++h) a2[h] = a2[NH + h] = first_audio[h];
    auto launch = [&](int slot, bool host_tokens) {
        int r = host_tokens ? be.set_async(be.ctx, p->in_audio->data, a2.data(), a2.size() * sizeof(int32_t)) : 0;
        const int32_t pp = p->position;
        if (r == 0) r = be.set_async(be.ctx, p->in_pos->data, &pp, sizeof(int32_t));
        if (r == 0) r = be.launch(be.ctx, slot);
        if (r == 0) p->position += 1;
        return r;
    };
    void * out = nullptr;
    if (st == 0) st = prepare(p, false);
    if (st == 0) st = be.prepare(be.ctx, p->gctx.nodes.data(), (int)p->gctx.nodes.size(), 0);
    if (st == 0) {
        out = p->res->data;
        st = launch(0, true);
    }
    for (int s = 0; st == 0 && s < n_steps; ++s) {
        const int slot = (s + 1) & 1;
        void * next_out = nullptr;
        if (s + 1 < n_steps) {  // record step s+1 while the device runs step s
            st = prepare(p, false);
            if (st == 0) st = be.prepare(be.ctx, p->gctx.nodes.data(), (int)p->gctx.nodes.size(), slot);
            next_out = p->res->data;
        }
        // step = NH: past every head's delay, so next = the sample itself (eos -1 never matches)
        if (st == 0 && p->sampling)
            st = be.sample_step(be.ctx, (const float *)out, 1, NH, cf.output_vocab_size, &p->samp, p->sample_calls + s, d_rep, NH, 0, -1, d_seen,
                                d_hist + (size_t)s * NH, d_next);
        else if (st == 0)
            st = be.greedy_step(be.ctx, (const float *)out, 1, NH, cf.output_vocab_size, NH, 0, -1, d_seen, d_hist + (size_t)s * NH, d_next);
        if (st == 0 && s + 1 < n_steps) {
            st = be.copy(be.ctx, p->in_audio->data, d_next, rowi);
            if (st == 0) st = be.copy(be.ctx, (int32_t *)p->in_audio->data + NH, d_next, rowi);
            if (st == 0) st = launch(slot, false);
            out = next_out;
        }
    }
    if (st == 0) st = be.get(be.ctx, tokens_out, d_hist, rowi * (size_t)n_steps);
    if (st == 0 && d_rep) {
        st = be.get(be.ctx, rep.data(), d_rep, 2 * rowi);
        for (int h = 0; h < NH; ++h) p->rep_last[h] = rep[2 * h], p->rep_count[h] = rep[2 * h + 1];
    }
    if (st == 0 && p->sampling) p->sample_calls += n_steps;
    if (d_rep) be.free(be.ctx, d_rep);
    if (d_seen) be.free(be.ctx, d_seen);
    if (d_next) be.free(be.ctx, d_next);
    if (d_hist) be.free(be.ctx, d_hist);
    return st;
}

extern "C" int32_t tts_dia_position(const tts_dia * p) { return p->position; }
extern "C" int32_t tts_dia_last_graph_nodes(const tts_dia * p) { return p->last_nodes; }
extern "C" uint64_t tts_dia_weight_bytes(const tts_dia * p) { return p->wbytes; }
extern "C" int32_t tts_dia_n_weights(const tts_dia * p) { return p ? (int32_t)p->wlist.size() : 0; }
extern "C" uint64_t tts_dia_weight(tts_dia * p, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst,
                                   uint64_t cap) {
    if (!p || i < 0 || i >= (int32_t)p->wlist.size()) return 0;
    return tg::weight_out(p->be, p->wlist[i], name, name_cap, ne, type, dst, cap);
}
extern "C" tts_tensor * const * tts_dia_graph(const tts_dia * p, int32_t * n_nodes) {
    if (n_nodes) *n_nodes = p ? (int32_t)p->gctx.nodes.size() : 0;
    return p ? p->gctx.nodes.data() : nullptr;
}
