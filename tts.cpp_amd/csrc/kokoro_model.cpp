// Kokoro-82M end to end: phoneme tokens -> durations -> decoder features -> iSTFTNet PCM.
//
// Two graphs, as the reference runs them (src/models/kokoro/model.cpp):
//  * the duration graph, kokoro_duration_runner::build_kokoro_duration_graph (:938-1047): ALBERT
//    inputs (build_albert_inputs :10-22, build_albert_norm :24-30), n_recurrence passes over the
//    shared layer group (self-attention with a zero mask, FFN with GELU, post-norms), the
//    bert_encoder projection, the DurationEncoder (bidirectional LSTM -> AdaLayerNorm -> style
//    concat, x3), the duration LSTM + projection -> sigmoid -> sum_rows -> round -> clamp(1, 50);
//  * the main graph, kokoro_runner::build_kokoro_graph (:1141-1242): the duration-mask expansion
//    (a mul_mat of the transposed [total, n] mask with the hidden states), the shared LSTM, the F0
//    and N AdaIN residual stacks (build_ada_residual_conv :88-134, with the depthwise
//    conv_transpose_1d "pool" and nearest x2 shortcut), the text encoder (embedding, conv k5 /
//    LayerNorm / leaky_relu x3, LSTM), the decoder (F0 / N stride-2 convs, encoder block, asr_res
//    1x1, four decode blocks), then build_generator -- the same builder the standalone generator
//    runner uses (kokoro.cpp), including the uv_noise MAP_CUSTOM3 node.
// Between the graphs the host does what kokoro_runner::run / set_inputs do (:1253-1325): read the
// lengths and hidden states back, sum the lengths, build the 0/1 duration mask, upload.
// LSTMs are build_lstm / build_lstm_run (:32-86) node for node; the HIP planner fuses each
// recurrence into one kernel per step (graph_exec.hip try_lstm).
// Weights are deterministic synthetic tensors in Kokoro-82M shapes (no checkpoints offline),
// named as the GGUF converter names them (py-gguf/tts_encoders/kokoro_gguf_encoder.py).
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "graph.h"
#include "kokoro_gen.h"
#include "synth.h"
#include "tts_hip.h"
#include "tts_runners.h"

using namespace tts;

namespace {

struct wspec {
    tts_tensor * t;
    float scale, offset;
    uint64_t seed;
};

struct kk_lstm {  // lstm / lstm_cell (model.h): one cell, optionally bidirectional
    tts_tensor *w[8], *b[8], *rw[8], *rb[8];
    tts_tensor *h0, *c0;
    bool bidir = true;
};

struct kk_ada {  // ada_residual_conv_block (model.h)
    tts_tensor *n1gw, *n1gb, *n1bw, *n1bb, *n2gw, *n2gb, *n2bw, *n2bb;
    tts_tensor *c1w, *c1b, *c2w, *c2b;
    tts_tensor *pool = nullptr, *pool_b = nullptr, *up = nullptr;
};

struct kk_albert_layer {
    tts_tensor *q, *qb, *k, *kb, *v, *vb, *o, *ob, *anw, *anb, *ffn, *ffnb, *ffo, *ffob, *onw, *onb;
};

struct kk_dur_layer {
    kk_lstm rnn;
    tts_tensor *gw, *gb, *bw, *bb;
};

struct kk_te_layer {
    tts_tensor *w, *b, *gamma, *beta;
};

}  // namespace

struct tts_kokoro {
    tts_kokoro_config cfg;
    tts_backend_iface be;
    tts_kokoro_gen * gen = nullptr;
    tg::context wctx;
    void * wbuf = nullptr;
    std::vector<wspec> specs;
    uint64_t tensor_index = 0;
    // ALBERT
    tts_tensor *tok_embd, *pos_embd, *tt_values, *in_nw, *in_nb, *embd_hidden, *embd_hidden_b;
    std::vector<kk_albert_layer> layers;
    // prosody predictor
    tts_tensor *encode, *encode_b, *dur_proj, *dur_proj_b, *f0_proj, *f0_proj_b, *n_proj, *n_proj_b;
    std::vector<kk_dur_layer> dur_layers;
    kk_lstm dur_lstm, shared_lstm;
    std::vector<kk_ada> f0_blocks, n_blocks;
    // text encoder
    tts_tensor * te_embd;
    std::vector<kk_te_layer> te;
    kk_lstm te_lstm;
    // decoder
    tts_tensor *f0_conv, *f0_conv_b, *n_conv, *n_conv_b, *asr_conv, *asr_conv_b;
    kk_ada enc;
    std::vector<kk_ada> dec;
    tts_tensor *voice, *sqrt2;
    // graphs
    char * arena = nullptr;
    size_t arena_size = 0;
    tg::context dctx, gctx;
    tts_tensor *d_tokens = nullptr, *d_pos = nullptr, *d_mask = nullptr, *d_hidden = nullptr, *d_len = nullptr;
    tts_tensor *m_tokens = nullptr, *m_dmask = nullptr, *m_dpred = nullptr, *m_out = nullptr;
    std::vector<float> h_dmask, h_zero, h_hidden, h_len;
    std::vector<int32_t> h_pos;
};

extern "C" void tts_kokoro_default_config(tts_kokoro_config * c) {
    memset(c, 0, sizeof(*c));
    tts_kokoro_gen_default_config(&c->gen);
    c->n_vocab = 178;
    c->embd = 128;
    c->hidden = 768;
    c->n_heads = 12;
    c->ffn = 2048;
    c->n_layers = 1;
    c->n_recurrence = 12;
    c->max_context = 512;
    c->d_model = 512;
    c->n_dur_layers = 3;
    c->max_dur = 50;
    c->te_kernel = 5;
    c->te_depth = 3;
    c->dec_dim = 1024;
    c->asr_res_dim = 64;
    c->n_decode = 4;
    c->n_voice_rows = 510;
    c->max_tokens = 128;
    c->max_total = 1024;
    c->dur_bias = -2.6f;
    c->f0_mean = 140.0f;
    c->seed = 0x6B0C0F0ull;
}

// gguf = false: a constant built at load time (post_load_assign), never in the file (F32)
static tts_tensor * wnew(tts_kokoro * k, float scale, float offset, int64_t ne0, int64_t ne1, int64_t ne2, const std::string & name,
                         bool gguf = true) {
    const int ty = gguf && k->cfg.weight_type == TTS_TYPE_F16 && kokoro_f16_tensor(name, ne1) ? TTS_TYPE_F16 : TTS_TYPE_F32;
    tts_tensor * t = ne1 == 0 ? tg::new_tensor_1d(k->wctx, ty, ne0)
                   : ne2 == 0 ? tg::new_tensor_2d(k->wctx, ty, ne0, ne1)
                              : tg::new_tensor_3d(k->wctx, ty, ne0, ne1, ne2);
    tg::set_name(t, name);
    t->flags |= tg::TG_FLAG_PERSIST;
    k->specs.push_back({t, scale, offset, k->cfg.seed ^ (k->tensor_index++ * 0x9E3779B97F4A7C15ull)});
    return t;
}

// Linear(in -> out) as ggml holds it: [in, out], uniform +-gain*sqrt(3/in)
static tts_tensor * lin(tts_kokoro * k, int64_t in, int64_t out, const std::string & name, float gain = 1.0f) {
    return wnew(k, gain * std::sqrt(3.0f / (float)in), 0.f, in, out, 0, name);
}

static tts_tensor * conv_w(tts_kokoro * k, int K, int IC, int OC, const std::string & name, float gain = 1.0f) {
    return wnew(k, gain * std::sqrt(3.0f / (float)(K * IC)), 0.f, K, IC, OC, name);
}

// prepare_lstm_tensor's split: weights[2g] = W_i{g} [in, H], weights[2g+1] = W_h{g} [H, H]
static kk_lstm make_lstm(tts_kokoro * k, int in, int hd, const std::string & pre) {
    kk_lstm r;
    const float s = 1.0f / std::sqrt((float)hd);  // torch.nn.LSTM's uniform(+-1/sqrt(H))
    for (int dir = 0; dir < 2; ++dir) {
        const std::string part = dir ? ".0.reverse_" : ".0.";
        for (int i = 0; i < 8; ++i) {
            tts_tensor * w = wnew(k, s, 0.f, i % 2 ? hd : in, hd, 0, pre + part + "weights." + std::to_string(i));
            tts_tensor * b = wnew(k, s, 0.f, hd, 0, 0, pre + part + "biases." + std::to_string(i));
            (dir ? r.rw : r.w)[i] = w;
            (dir ? r.rb : r.b)[i] = b;
        }
    }
    r.h0 = wnew(k, 0.f, 0.f, hd, 0, 0, pre + ".0.hidden");
    r.c0 = wnew(k, 0.f, 0.f, hd, 0, 0, pre + ".0.state");
    return r;
}

// AdainResBlk1d(dim_in, dim_out, style, upsample): AdaIN fc halves as gamma / beta [S, C]
static kk_ada make_ada(tts_kokoro * k, int cin, int cout, bool upsample, const std::string & pre) {
    const int S = k->cfg.gen.style_dim;
    const float sw = 0.1f * std::sqrt(3.0f / (float)S);
    kk_ada a;
    a.n1gw = wnew(k, sw, 0.f, S, cin, 0, pre + ".norm1_gamma_weight");
    a.n1gb = wnew(k, 0.05f, 0.f, cin, 0, 0, pre + ".norm1_gamma_bias");
    a.n1bw = wnew(k, sw, 0.f, S, cin, 0, pre + ".norm1_beta_weight");
    a.n1bb = wnew(k, 0.05f, 0.f, cin, 0, 0, pre + ".norm1_beta_bias");
    a.n2gw = wnew(k, sw, 0.f, S, cout, 0, pre + ".norm2_gamma_weight");
    a.n2gb = wnew(k, 0.05f, 0.f, cout, 0, 0, pre + ".norm2_gamma_bias");
    a.n2bw = wnew(k, sw, 0.f, S, cout, 0, pre + ".norm2_beta_weight");
    a.n2bb = wnew(k, 0.05f, 0.f, cout, 0, 0, pre + ".norm2_beta_bias");
    a.c1w = conv_w(k, 3, cin, cout, pre + ".conv1_weight");
    a.c1b = wnew(k, 0.01f, 0.f, 1, cout, 0, pre + ".conv1_bias");
    a.c2w = conv_w(k, 3, cout, cout, pre + ".conv2_weight");
    a.c2b = wnew(k, 0.01f, 0.f, 1, cout, 0, pre + ".conv2_bias");
    if (upsample) {  // ConvTranspose1d(cin, cin, 3, stride 2, groups cin, padding 1, output_padding 1)
        a.pool = wnew(k, std::sqrt(3.0f / 3.0f), 0.f, 3, 1, cin, pre + ".pool_weight");
        a.pool_b = wnew(k, 0.01f, 0.f, 1, cin, 0, pre + ".pool_bias");
    }
    if (cin != cout) a.up = lin(k, cin, cout, pre + ".conv1x1_weight");  // squeeze_3d_2d_e0'd [1, cin, cout]
    return a;
}

static bool upload(tts_kokoro * k) {
    size_t total = 0;
    for (auto & s : k->specs) total += (tg::nbytes(s.t) + 255) & ~(size_t)255;
    k->wbuf = k->be.alloc(k->be.ctx, total);
    if (!k->wbuf) return false;
    size_t off = 0;
    std::vector<float> host;
    for (auto & s : k->specs) {
        const size_t n = (size_t)tg::nelements(s.t);
        s.t->data = (char *)k->wbuf + off;
        off += (tg::nbytes(s.t) + 255) & ~(size_t)255;
        host.resize(n);
        synth_f32(host.data(), n, s.seed, s.scale, s.offset);
        if (!kokoro_upload_weight(k->be, s.t, host.data(), n)) return false;
    }
    return true;
}

extern "C" tts_kokoro * tts_kokoro_create(const tts_backend_iface * be, const tts_kokoro_config * cfg) {
    if (!be || !cfg) return nullptr;
    const auto & c = *cfg;
    if (c.hidden % c.n_heads || c.d_model % 2 || c.max_tokens < 3 || c.max_tokens > c.max_context || c.max_total < 1 || c.n_decode < 1 ||
        c.te_kernel % 2 == 0 || c.n_dur_layers < 1 || c.te_depth < 0 || c.n_voice_rows < c.max_tokens - 2 || c.max_dur < 1)
        return nullptr;
    auto * k = new tts_kokoro();
    k->cfg = c;
    k->be = *be;
    // the generator runs inside the main graph: its own arena is unused
    tts_kokoro_gen_config gc = c.gen;
    gc.weight_type = c.weight_type;
    gc.max_frames = 2 * c.max_total;
    gc.arena_bytes = 256;
    k->gen = tts_kokoro_gen_create(be, &gc);
    if (!k->gen) {
        delete k;
        return nullptr;
    }
    const int S = c.gen.style_dim, D = c.d_model, H2 = c.d_model / 2;
    // ALBERT (assign_albert_weight)
    k->tok_embd = wnew(k, 1.0f, 0.f, c.embd, c.n_vocab, 0, "albert.token_embd");
    k->pos_embd = wnew(k, 0.5f, 0.f, c.embd, c.max_context, 0, "albert.position_embd");
    k->tt_values = wnew(k, 0.1f, 0.f, c.embd, 0, 0, "albert.token_type_embd");
    k->in_nw = wnew(k, 0.1f, 1.0f, c.embd, 0, 0, "albert.norm");
    k->in_nb = wnew(k, 0.05f, 0.f, c.embd, 0, 0, "albert.norm_bias");
    k->embd_hidden = lin(k, c.embd, c.hidden, "albert.embd");
    k->embd_hidden_b = wnew(k, 0.02f, 0.f, c.hidden, 0, 0, "albert.embd_bias");
    for (int l = 0; l < c.n_layers; ++l) {
        const std::string p = "albert.layer." + std::to_string(l);
        kk_albert_layer L;
        L.q = lin(k, c.hidden, c.hidden, p + ".q"), L.qb = wnew(k, 0.02f, 0.f, c.hidden, 0, 0, p + ".q_bias");
        L.k = lin(k, c.hidden, c.hidden, p + ".k"), L.kb = wnew(k, 0.02f, 0.f, c.hidden, 0, 0, p + ".k_bias");
        L.v = lin(k, c.hidden, c.hidden, p + ".v"), L.vb = wnew(k, 0.02f, 0.f, c.hidden, 0, 0, p + ".v_bias");
        L.o = lin(k, c.hidden, c.hidden, p + ".o"), L.ob = wnew(k, 0.02f, 0.f, c.hidden, 0, 0, p + ".o_bias");
        L.anw = wnew(k, 0.1f, 1.0f, c.hidden, 0, 0, p + ".attn_norm"), L.anb = wnew(k, 0.05f, 0.f, c.hidden, 0, 0, p + ".attn_norm_bias");
        L.ffn = lin(k, c.hidden, c.ffn, p + ".ffn"), L.ffnb = wnew(k, 0.02f, 0.f, c.ffn, 0, 0, p + ".ffn_bias");
        L.ffo = lin(k, c.ffn, c.hidden, p + ".ffn_out"), L.ffob = wnew(k, 0.02f, 0.f, c.hidden, 0, 0, p + ".ffn_out_bias");
        L.onw = wnew(k, 0.1f, 1.0f, c.hidden, 0, 0, p + ".layer_out_norm");
        L.onb = wnew(k, 0.05f, 0.f, c.hidden, 0, 0, p + ".layer_out_norm_bias");
        k->layers.push_back(L);
    }
    // prosody predictor (assign_duration_weight)
    const std::string dp = "duration_predictor";
    k->encode = lin(k, c.hidden, D, dp + ".encode");
    k->encode_b = wnew(k, 0.02f, 0.f, D, 0, 0, dp + ".encode_bias");
    for (int l = 0; l < c.n_dur_layers; ++l) {
        kk_dur_layer L;
        const std::string p = dp + ".layers." + std::to_string(2 * l);
        const std::string pn = dp + ".layers." + std::to_string(2 * l + 1);
        L.rnn = make_lstm(k, D + S, H2, p + ".lstm");
        const float sw = 0.1f * std::sqrt(3.0f / (float)S);
        L.gw = wnew(k, sw, 0.f, S, D, 0, pn + ".gamma_weight");
        L.gb = wnew(k, 0.05f, 0.f, D, 0, 0, pn + ".gamma_bias");
        L.bw = wnew(k, sw, 0.f, S, D, 0, pn + ".beta_weight");
        L.bb = wnew(k, 0.05f, 0.f, D, 0, 0, pn + ".beta_bias");
        k->dur_layers.push_back(L);
    }
    k->dur_lstm = make_lstm(k, D + S, H2, dp + ".duration_lstm");
    // small weights around a negative bias: sigmoid sums of ~4 frames per token, as real speech
    k->dur_proj = lin(k, D, c.max_dur, dp + ".duration_proj", 4.0f);
    k->dur_proj_b = wnew(k, 0.3f, c.dur_bias, c.max_dur, 0, 0, dp + ".duration_proj_bias");
    k->shared_lstm = make_lstm(k, D + S, H2, dp + ".shared_lstm");
    for (int i = 0; i < 3; ++i) {
        const int cin = i == 0 ? D : H2 * (i == 1 ? 2 : 1), cout = i == 0 ? D : H2;
        k->f0_blocks.push_back(make_ada(k, cin, cout, i == 1, dp + ".f0_blocks." + std::to_string(i)));
    }
    for (int i = 0; i < 3; ++i) {
        const int cin = i == 0 ? D : H2 * (i == 1 ? 2 : 1), cout = i == 0 ? D : H2;
        k->n_blocks.push_back(make_ada(k, cin, cout, i == 1, dp + ".n_blocks." + std::to_string(i)));
    }
    // F0 in Hz around f0_mean (a few frames fall below the voicing threshold), N near zero
    k->f0_proj = wnew(k, 70.0f * std::sqrt(3.0f / (float)H2), 0.f, H2, 1, 0, dp + ".f0_proj_kernel");
    k->f0_proj_b = wnew(k, 0.f, c.f0_mean, 1, 1, 0, dp + ".f0_proj_bias");
    k->n_proj = lin(k, H2, 1, dp + ".n_proj_kernel");
    k->n_proj_b = wnew(k, 0.01f, 0.f, 1, 1, 0, dp + ".n_proj_bias");
    // text encoder (assign_text_encoder_weight)
    k->te_embd = wnew(k, 1.0f, 0.f, D, c.n_vocab, 0, "text_encoder.embedding_weight");
    for (int l = 0; l < c.te_depth; ++l) {
        const std::string p = "text_encoder.layers." + std::to_string(l);
        kk_te_layer L;
        L.w = conv_w(k, c.te_kernel, D, D, p + ".weight");
        L.b = wnew(k, 0.01f, 0.f, 1, D, 0, p + ".bias");
        L.gamma = wnew(k, 0.1f, 1.0f, D, 0, 0, p + ".gamma");
        L.beta = wnew(k, 0.05f, 0.f, D, 0, 0, p + ".beta");
        k->te.push_back(L);
    }
    k->te_lstm = make_lstm(k, D, H2, "text_encoder.lstm");
    // decoder (assign_decoder_weight); F0 / N convs see Hz-scale inputs: small kernels
    k->f0_conv = wnew(k, 0.01f, 0.f, 3, 1, 1, "decoder.f0_conv_weight");
    k->f0_conv_b = wnew(k, 0.01f, 0.f, 1, 1, 0, "decoder.f0_conv_bias");
    k->n_conv = wnew(k, std::sqrt(3.0f / 3.0f), 0.f, 3, 1, 1, "decoder.n_conv_weight");
    k->n_conv_b = wnew(k, 0.01f, 0.f, 1, 1, 0, "decoder.n_conv_bias");
    k->asr_conv = lin(k, D, c.asr_res_dim, "decoder.asr_conv_weight");
    k->asr_conv_b = wnew(k, 0.01f, 0.f, 1, c.asr_res_dim, 0, "decoder.asr_conv_bias");
    k->enc = make_ada(k, D + 2, c.dec_dim, false, "decoder.encoder_block");
    for (int i = 0; i < c.n_decode; ++i) {
        const bool last = i == c.n_decode - 1;
        k->dec.push_back(make_ada(k, c.dec_dim + 2 + c.asr_res_dim, last ? c.gen.in_channels : c.dec_dim, last,
                                  "decoder.decoder_blocks." + std::to_string(i)));
    }
    k->voice = wnew(k, 0.5f, 0.f, 2 * S, c.n_voice_rows, 0, "voice_tensors.synthetic");
    k->sqrt2 = wnew(k, 0.f, (float)std::sqrt(2.0), 1, 0, 0, "sqrt_tensor", false);
    if (!upload(k)) {
        tts_kokoro_free(k);
        return nullptr;
    }
    // arena: the main graph's widest live set is the decoder's [total, ~1090] activations plus
    // their conv im2cols, and the generator's per-frame tensors (as the generator sizes them)
    const size_t Tm = (size_t)c.max_total, n = (size_t)c.max_tokens;
    const size_t dec = Tm * (size_t)(c.dec_dim + 2 + c.asr_res_dim) * 4 * 12 + Tm * 3 * (size_t)(c.dec_dim + 2 + c.asr_res_dim) * 2 * 2;
    const size_t lstm = (Tm + n) * (size_t)(D + S) * 4 * 8 + (Tm + n) * (size_t)H2 * 4 * 40;
    const size_t albert = n * (size_t)c.ffn * 4 * 4 + n * n * (size_t)c.n_heads * 4 * 3 + n * (size_t)c.hidden * 4 * 16;
    const int64_t U = 300;
    const size_t L = 2 * Tm * U;
    const size_t genb = 2 * Tm * (size_t)(U / c.gen.hop) * (size_t)(c.gen.in_channels / 4) * 4 * 14 +
                        2 * Tm * (size_t)(U / c.gen.hop) * 11 * (size_t)(c.gen.in_channels / 4) * 2 * 2 + L * (size_t)(c.gen.harmonic_num + 1) * 4 * 16 +
                        2 * Tm * (size_t)c.gen.in_channels * 4 * 16;
    k->arena_size = c.arena_bytes ? c.arena_bytes : dec + lstm + albert + genb + ((size_t)64 << 20);
    k->arena = (char *)k->be.alloc(k->be.ctx, k->arena_size);
    if (!k->arena) {
        tts_kokoro_free(k);
        return nullptr;
    }
    return k;
}

extern "C" void tts_kokoro_free(tts_kokoro * k) {
    if (!k) return;
    if (k->arena) k->be.free(k->be.ctx, k->arena);
    if (k->wbuf) k->be.free(k->be.ctx, k->wbuf);
    tts_kokoro_gen_free(k->gen);
    delete k;
}

// TTS_KOKORO_TIMING=1: host phase times per call on stderr (build / alloc / inputs / compute / read)
namespace {
struct phase_clock {
    bool on = getenv("TTS_KOKORO_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    char buf[256];
    int len = 0;
    void mark(const char * what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        len += snprintf(buf + len, sizeof(buf) - len, " %s %.3f", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
    void done(const char * which) {
        if (on) fprintf(stderr, "kokoro %s ms:%s\n", which, buf);
    }
};
}  // namespace

// build_albert_norm (model.cpp:24-30): eps 1e-12
static tts_tensor * albert_norm(tg::context & c, tts_tensor * cur, tts_tensor * w, tts_tensor * b) {
    cur = tg::norm(c, cur, 0.000000000001f);
    return tg::cont(c, tg::add(c, tg::mul(c, cur, w), b));
}

// build_lstm_run (model.cpp:56-86)
static tts_tensor * lstm_run(tg::context & c, tts_tensor * input, tts_tensor * h0, tts_tensor * c0, tts_tensor * const * w, tts_tensor * const * b,
                             int64_t T, bool reversed) {
    tts_tensor * I = tg::add(c, tg::mul_mat(c, w[0], input), b[0]);
    tts_tensor * F = tg::add(c, tg::mul_mat(c, w[2], input), b[2]);
    tts_tensor * G = tg::add(c, tg::mul_mat(c, w[4], input), b[4]);
    tts_tensor * O = tg::add(c, tg::mul_mat(c, w[6], input), b[6]);
    tts_tensor * outputs = nullptr;
    for (int64_t index = 0; index < T; ++index) {
        const int64_t i = reversed ? T - 1 - index : index;
        auto gate = [&](tts_tensor * P, int wi, bool tanh_) {
            tts_tensor * cur = tg::view_3d(c, P, P->ne[0], 1, P->ne[2], P->nb[0], P->nb[1], P->nb[1] * i);
            cur = tg::add(c, cur, tg::add(c, tg::mul_mat(c, w[wi], h0), b[wi]));
            return tanh_ ? tg::tanh(c, cur) : tg::sigmoid(c, cur);
        };
        tts_tensor * Ic = gate(I, 1, false);
        tts_tensor * Fc = gate(F, 3, false);
        tts_tensor * Gc = gate(G, 5, true);
        tts_tensor * Oc = gate(O, 7, false);
        c0 = tg::add(c, tg::mul(c, Fc, c0), tg::mul(c, Ic, Gc));
        h0 = tg::mul(c, tg::tanh(c, c0), Oc);
        if (index == 0) outputs = h0;
        else outputs = reversed ? tg::concat(c, h0, outputs, 1) : tg::concat(c, outputs, h0, 1);
        tg::build_forward_expand(c, outputs);
    }
    return outputs;
}

// build_lstm (model.cpp:35-54), one cell
static tts_tensor * lstm(tg::context & c, tts_tensor * input, const kk_lstm & r, int64_t T) {
    tg::build_forward_expand(c, input);
    tts_tensor * resp = lstm_run(c, input, r.h0, r.c0, r.w, r.b, T, false);
    if (!r.bidir) return resp;
    tts_tensor * rev = lstm_run(c, input, r.h0, r.c0, r.rw, r.rb, T, true);
    return tg::concat(c, resp, rev, 0);
}

// build_ada_residual_conv (model.cpp:88-134); x is [T, C] (time fastest)
static tts_tensor * ada_block(tts_kokoro * k, tg::context & c, tts_tensor * x, const kk_ada & b, tts_tensor * style) {
    tts_tensor * gamma = tg::add(c, tg::mul_mat(c, b.n1gw, style), b.n1gb);
    tts_tensor * beta = tg::add(c, tg::mul_mat(c, b.n1bw, style), b.n1bb);
    tts_tensor * cur = tg::norm(c, x, 0.00001f);
    cur = tg::add(c, cur, tg::mul(c, cur, tg::transpose(c, gamma)));
    cur = tg::add(c, cur, tg::transpose(c, beta));
    cur = tg::leaky_relu(c, cur, 0.2f);
    if (b.pool) {
        cur = tg::conv_transpose_1d(c, b.pool, cur, 2, 1, 1, 1, (int)cur->ne[1]);
        cur = tg::add(c, cur, b.pool_b);
    }
    cur = tg::conv_1d(c, b.c1w, cur, 1, 1, 1);
    cur = tg::add(c, cur, b.c1b);
    gamma = tg::add(c, tg::mul_mat(c, b.n2gw, style), b.n2gb);
    beta = tg::add(c, tg::mul_mat(c, b.n2bw, style), b.n2bb);
    cur = tg::norm(c, cur, 0.00001f);
    cur = tg::add(c, cur, tg::mul(c, cur, tg::transpose(c, gamma)));
    cur = tg::add(c, cur, tg::transpose(c, beta));
    cur = tg::leaky_relu(c, cur, 0.2f);
    cur = tg::add(c, tg::conv_1d(c, b.c2w, cur, 1, 1, 1), b.c2b);
    tts_tensor * res = cur;
    cur = x;
    if (b.up) {
        cur = tg::cont(c, tg::transpose(c, cur));
        if (b.pool) cur = tg::upscale_ext(c, cur, cur->ne[0], cur->ne[1] * 2, cur->ne[2], cur->ne[3]);
        cur = tg::mul_mat(c, b.up, cur);
        cur = tg::cont(c, tg::transpose(c, cur));
    }
    return tg::div(c, tg::add(c, res, cur), k->sqrt2);
}

// style_half (prosody) = second half of voice row n-3, style_half2 (decoder) = the first half
static tts_tensor * style_view(tts_kokoro * k, tg::context & c, int64_t n, bool second) {
    tts_tensor * v = k->voice;
    const size_t off = (second ? (size_t)(v->ne[0] / 2) * v->nb[0] : 0) + (size_t)(n - 3) * v->nb[1];
    return tg::view_1d(c, v, v->ne[0] / 2, off);
}

// kokoro_duration_runner::build_kokoro_duration_graph (model.cpp:938-1047)
static tts_tensor * build_duration_graph(tts_kokoro * k, int64_t n) {
    const auto & cf = k->cfg;
    tg::context & c = k->dctx;
    c.reset();
    k->d_tokens = tg::new_tensor_1d(c, TTS_TYPE_I32, n);
    k->d_pos = tg::new_tensor_1d(c, TTS_TYPE_I32, n);
    tg::set_input(k->d_tokens);
    tg::set_input(k->d_pos);
    // build_albert_inputs (model.cpp:10-22), static token types
    tts_tensor * tinp = tg::cont(c, tg::get_rows(c, k->tok_embd, k->d_tokens));
    tts_tensor * pinp = tg::get_rows(c, k->pos_embd, k->d_pos);
    tts_tensor * inp = tg::cont(c, tg::add(c, tinp, pinp));
    inp = tg::add(c, inp, k->tt_values);
    inp = tg::cont(c, albert_norm(c, inp, k->in_nw, k->in_nb));
    tts_tensor * cur = tg::add(c, tg::mul_mat(c, k->embd_hidden, inp), k->embd_hidden_b);
    tg::set_name(cur, "albert_embeddings");
    k->d_mask = tg::new_tensor_2d(c, TTS_TYPE_F32, n, n);
    tg::set_input(k->d_mask);
    const int64_t hs = cf.hidden / cf.n_heads;
    const float scale = 1.0f / std::sqrt((float)hs);
    for (int r = 0; r < cf.n_recurrence; ++r) {
        for (int l = 0; l < cf.n_layers; ++l) {
            const kk_albert_layer & L = k->layers[l];
            tts_tensor * residual = cur;
            tts_tensor * Q = tg::add(c, tg::mul_mat(c, L.q, cur), L.qb);
            tts_tensor * K = tg::add(c, tg::mul_mat(c, L.k, cur), L.kb);
            tts_tensor * V = tg::add(c, tg::mul_mat(c, L.v, cur), L.vb);
            Q = tg::reshape_3d(c, Q, hs, cf.n_heads, n);
            K = tg::reshape_3d(c, K, hs, cf.n_heads, n);
            tts_tensor * q = tg::permute(c, Q, 0, 2, 1, 3);
            tts_tensor * kk = tg::cont(c, tg::permute(c, K, 0, 2, 1, 3));
            tts_tensor * kq = tg::mul_mat(c, kk, q);
            kq = tg::soft_max_ext(c, kq, k->d_mask, scale, 0.0f);
            tts_tensor * v = tg::cont_3d(c, tg::transpose(c, V), n, hs, cf.n_heads);
            tts_tensor * kqv = tg::mul_mat(c, kq, v);
            tts_tensor * merged = tg::permute(c, kqv, 2, 0, 1, 3);
            tts_tensor * attn = tg::cont_2d(c, merged, cf.hidden, n);
            attn = tg::add(c, tg::mul_mat(c, L.o, attn), L.ob);
            cur = tg::add(c, attn, residual);
            cur = albert_norm(c, cur, L.anw, L.anb);
            tts_tensor * rffn = cur;
            cur = tg::gelu(c, tg::add(c, tg::mul_mat(c, L.ffn, cur), L.ffnb));
            cur = tg::add(c, tg::mul_mat(c, L.ffo, cur), L.ffob);
            cur = tg::add(c, cur, rffn);
            cur = albert_norm(c, cur, L.onw, L.onb);
        }
        tg::build_forward_expand(c, cur);
    }
    tg::set_name(cur, "albert_out");
    cur = tg::add(c, tg::mul_mat(c, k->encode, cur), k->encode_b);
    tts_tensor * sh = k->voice;
    tts_tensor * style_half = tg::cont(c, tg::view_1d(c, sh, sh->ne[0] / 2, (size_t)(sh->ne[0] / 2) * sh->nb[0] + (size_t)(n - 3) * sh->nb[1]));
    cur = tg::concat(c, cur, tg::repeat(c, style_half, tg::new_tensor_2d(c, TTS_TYPE_F32, style_half->ne[0], cur->ne[1])), 0);
    for (const auto & L : k->dur_layers) {
        cur = lstm(c, cur, L.rnn, n);
        tts_tensor * gamma = tg::add(c, tg::mul_mat(c, L.gw, style_half), L.gb);
        tts_tensor * beta = tg::add(c, tg::mul_mat(c, L.bw, style_half), L.bb);
        cur = tg::norm(c, cur, 0.00001f);
        cur = tg::add(c, tg::add(c, cur, tg::mul(c, cur, gamma)), beta);
        cur = tg::concat(c, cur, tg::repeat(c, style_half, tg::new_tensor_2d(c, TTS_TYPE_F32, style_half->ne[0], cur->ne[1])), 0);
    }
    tts_tensor * d = tg::cont(c, cur);
    tg::set_name(d, "duration_hidden_states");
    tg::set_output(d);
    tg::build_forward_expand(c, d);
    k->d_hidden = d;
    cur = lstm(c, cur, k->dur_lstm, n);
    cur = tg::sigmoid(c, tg::add(c, tg::mul_mat(c, k->dur_proj, cur), k->dur_proj_b));
    tg::set_name(cur, "duration_probs");
    tts_tensor * len = tg::clamp(c, tg::round(c, tg::sum_rows(c, cur)), 1.0f, (float)cf.max_dur);
    tg::set_name(len, "lengths");
    tg::set_output(len);
    tg::build_forward_expand(c, len);
    k->d_len = len;
    return len;
}

// kokoro_runner::build_kokoro_graph (model.cpp:1141-1242); total = sum of the lengths
static tts_tensor * build_main_graph(tts_kokoro * k, int64_t n, int64_t total, bool device_draws) {
    const auto & cf = k->cfg;
    tg::context & c = k->gctx;
    c.reset();
    tts_tensor * style_half = style_view(k, c, n, true);
    k->m_tokens = tg::new_tensor_1d(c, TTS_TYPE_I32, n);
    tg::set_input(k->m_tokens);
    k->m_dmask = tg::new_tensor_2d(c, TTS_TYPE_F32, total, n);
    tg::set_input(k->m_dmask);
    k->m_dpred = tg::new_tensor_2d(c, TTS_TYPE_F32, cf.d_model + cf.gen.style_dim, n);
    tg::set_input(k->m_dpred);

    tts_tensor * cur = tg::mul_mat(c, tg::cont(c, tg::transpose(c, k->m_dmask)), tg::cont(c, tg::transpose(c, k->m_dpred)));
    cur = tg::cont(c, tg::transpose(c, cur));
    cur = lstm(c, cur, k->shared_lstm, cur->ne[1]);
    tg::set_name(cur, "shared_lstm");

    tts_tensor * f0 = tg::cont(c, tg::transpose(c, cur));
    for (const auto & b : k->f0_blocks) f0 = ada_block(k, c, f0, b, style_half);
    f0 = tg::cont(c, tg::transpose(c, f0));
    f0 = tg::mul_mat(c, k->f0_proj, f0);
    f0 = tg::reshape_2d(c, f0, f0->ne[1], f0->ne[2]);  // squeeze_3d_2d_e0
    f0 = tg::add(c, f0, k->f0_proj_b);
    tg::set_name(f0, "f0_out");
    tts_tensor * f0_curve = f0;

    tts_tensor * nn = tg::cont(c, tg::transpose(c, cur));
    for (const auto & b : k->n_blocks) nn = ada_block(k, c, nn, b, style_half);
    nn = tg::cont(c, tg::transpose(c, nn));
    nn = tg::mul_mat(c, k->n_proj, nn);
    nn = tg::reshape_2d(c, nn, nn->ne[1], nn->ne[2]);
    nn = tg::add(c, nn, k->n_proj_b);
    tg::set_name(nn, "n_out");
    tg::build_forward_expand(c, nn);

    // text encoder
    cur = tg::get_rows(c, k->te_embd, k->m_tokens);
    for (const auto & L : k->te) {
        cur = tg::cont(c, tg::transpose(c, tg::add(c, tg::conv_1d(c, L.w, tg::cont(c, tg::transpose(c, cur)), 1, cf.te_kernel / 2, 1), L.b)));
        cur = tg::norm(c, cur, 0.00001f);
        cur = tg::add(c, tg::mul(c, cur, L.gamma), L.beta);
        cur = tg::leaky_relu(c, cur, 0.2f);
    }
    cur = lstm(c, cur, k->te_lstm, n);
    tg::set_name(cur, "text_encoder");
    tts_tensor * asr = tg::mul_mat(c, tg::cont(c, tg::transpose(c, cur)), tg::cont(c, tg::transpose(c, k->m_dmask)));
    tg::set_name(asr, "asr");

    // decoder
    tts_tensor * style_half2 = style_view(k, c, n, false);
    tts_tensor * f0d = tg::add(c, tg::conv_1d(c, k->f0_conv, f0_curve, 2, 1, 1), k->f0_conv_b);
    tts_tensor * nd = tg::add(c, tg::conv_1d(c, k->n_conv, nn, 2, 1, 1), k->n_conv_b);
    cur = tg::concat(c, tg::concat(c, tg::cont(c, tg::transpose(c, asr)), f0d, 1), nd, 1);
    cur = ada_block(k, c, cur, k->enc, style_half2);
    tg::set_name(cur, "encoder_block");
    tg::build_forward_expand(c, cur);
    tts_tensor * asr_res = tg::mul_mat(c, k->asr_conv, asr);
    asr_res = tg::add(c, asr_res, tg::transpose(c, k->asr_conv_b));
    asr_res = tg::cont(c, tg::transpose(c, asr_res));
    for (size_t i = 0; i < k->dec.size(); ++i) {
        cur = tg::concat(c, tg::concat(c, tg::concat(c, cur, asr_res, 1), f0d, 1), nd, 1);
        cur = ada_block(k, c, cur, k->dec[i], style_half2);
        tg::set_name(cur, "decoder_block." + std::to_string(i));
        tg::build_forward_expand(c, cur);
    }
    cur = tg::cont(c, tg::transpose(c, cur));
    tg::set_name(cur, "decoder_out");

    cur = kokoro_gen_build(k->gen, c, cur, f0_curve, style_half2, f0_curve->ne[0], device_draws);
    tg::set_output(cur);
    tg::build_forward_expand(c, cur);
    k->m_out = cur;
    return cur;
}

extern "C" int tts_kokoro_durations(tts_kokoro * k, const int32_t * tokens, int32_t n, float * hidden, float * lengths) {
    if (!k || !tokens || n < 3 || n > k->cfg.max_tokens) return TTS_STATUS_BAD_ARG;
    for (int32_t i = 0; i < n; ++i)
        if (tokens[i] < 0 || tokens[i] >= k->cfg.n_vocab) return TTS_STATUS_BAD_ARG;
    phase_clock pc;
    build_duration_graph(k, n);
    pc.mark("build");
    if (!tg::alloc_graph(k->dctx, k->arena, k->arena_size, !k->cfg.debug_no_reuse)) {
        fprintf(stderr, "kokoro: compute arena too small (%zu needed)\n", k->dctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    // kokoro_duration_runner::set_inputs (model.cpp:1054-1067): positions 0..n-1, zero mask
    k->h_pos.resize(n);
    for (int32_t i = 0; i < n; ++i) k->h_pos[i] = i;
    k->h_zero.assign((size_t)n * n, 0.0f);
    int st = k->be.set(k->be.ctx, k->d_tokens->data, tokens, sizeof(int32_t) * (size_t)n);
    if (st == 0) st = k->be.set(k->be.ctx, k->d_pos->data, k->h_pos.data(), sizeof(int32_t) * (size_t)n);
    if (st == 0) st = k->be.set(k->be.ctx, k->d_mask->data, k->h_zero.data(), sizeof(float) * k->h_zero.size());
    pc.mark("alloc+inputs");
    if (st == 0) st = k->be.compute(k->be.ctx, k->dctx.nodes.data(), (int)k->dctx.nodes.size());
    pc.mark("compute");
    if (st == 0 && lengths) st = k->be.get(k->be.ctx, lengths, k->d_len->data, sizeof(float) * (size_t)n);
    if (st == 0 && hidden) st = k->be.get(k->be.ctx, hidden, k->d_hidden->data, tg::nbytes(k->d_hidden));
    pc.mark("read");
    pc.done("durations");
    return st;
}

extern "C" int tts_kokoro_decode(tts_kokoro * k, const int32_t * tokens, int32_t n, const float * hidden, const float * lengths,
                                 const float * rand, float * pcm, uint64_t pcm_cap) {
    if (!k || !tokens || !hidden || !lengths || n < 3 || n > k->cfg.max_tokens) return TTS_STATUS_BAD_ARG;
    // kokoro_runner::run (model.cpp:1281-1287): total = sum of (uint32_t) lengths
    int64_t total = 0;
    for (int32_t i = 0; i < n; ++i) {
        if (!(lengths[i] >= 0.0f) || lengths[i] > (float)k->cfg.max_dur) return TTS_STATUS_BAD_ARG;
        total += (int64_t)(uint32_t)lengths[i];
    }
    if (total < 1 || total > k->cfg.max_total) return TTS_STATUS_BAD_ARG;
    if (pcm && pcm_cap < (uint64_t)(600 * total) * sizeof(float)) return TTS_STATUS_BAD_ARG;
    phase_clock pc;
    build_main_graph(k, n, total, rand == nullptr);
    pc.mark("build");
    if (!tg::alloc_graph(k->gctx, k->arena, k->arena_size, !k->cfg.debug_no_reuse)) {
        fprintf(stderr, "kokoro: compute arena too small (%zu needed)\n", k->gctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    pc.mark("alloc");
    // kokoro_runner::set_inputs (model.cpp:1253-1275): duration mask row i covers frames
    // [running, running + lengths[i]) in f32, as the reference compares them
    k->h_dmask.assign((size_t)(total * n), 0.0f);
    float running = 0.0f;
    for (int32_t i = 0; i < n; ++i) {
        const float next = running + lengths[i];
        for (int64_t j = 0; j < total; ++j) k->h_dmask[(size_t)i * total + j] = (float)j >= running && (float)j < next ? 1.0f : 0.0f;
        running = next;
    }
    int st = kokoro_gen_set_inputs(k->gen, 2 * total, rand);
    if (st == 0) st = k->be.set(k->be.ctx, k->m_tokens->data, tokens, sizeof(int32_t) * (size_t)n);
    if (st == 0) st = k->be.set(k->be.ctx, k->m_dpred->data, hidden, tg::nbytes(k->m_dpred));
    if (st == 0) st = k->be.set(k->be.ctx, k->m_dmask->data, k->h_dmask.data(), sizeof(float) * k->h_dmask.size());
    pc.mark("inputs");
    if (st == 0) st = k->be.compute(k->be.ctx, k->gctx.nodes.data(), (int)k->gctx.nodes.size());
    pc.mark("compute");
    if (st == 0 && pcm) st = k->be.get(k->be.ctx, pcm, k->m_out->data, tg::nbytes(k->m_out));
    pc.mark("read");
    pc.done("decode");
    return st;
}

extern "C" int tts_kokoro_run(tts_kokoro * k, const int32_t * tokens, int32_t n, const float * rand, float * pcm, uint64_t pcm_cap,
                              int64_t * n_samples) {
    if (!k || !tokens || n < 3 || n > k->cfg.max_tokens) return TTS_STATUS_BAD_ARG;
    k->h_hidden.resize((size_t)n * (size_t)(k->cfg.d_model + k->cfg.gen.style_dim));
    k->h_len.resize((size_t)n);
    int st = tts_kokoro_durations(k, tokens, n, k->h_hidden.data(), k->h_len.data());
    if (st != 0) return st;
    int64_t total = 0;
    for (float l : k->h_len) total += (int64_t)(uint32_t)l;
    if (n_samples) *n_samples = 600 * total;
    return tts_kokoro_decode(k, tokens, n, k->h_hidden.data(), k->h_len.data(), rand, pcm, pcm_cap);
}

extern "C" int32_t tts_kokoro_last_graph_nodes(const tts_kokoro * k, int32_t which) {
    if (!k) return 0;
    return (int32_t)(which ? k->gctx.nodes.size() : k->dctx.nodes.size());
}

extern "C" int32_t tts_kokoro_n_weights(const tts_kokoro * k) {
    return k ? (int32_t)k->specs.size() + tts_kokoro_gen_n_weights(k->gen) : 0;
}

extern "C" uint64_t tts_kokoro_weight(tts_kokoro * k, int32_t i, char * name, uint64_t name_cap, int64_t * ne, float * dst, uint64_t cap) {
    if (!k || i < 0) return 0;
    if (i >= (int32_t)k->specs.size()) return tts_kokoro_gen_weight(k->gen, i - (int32_t)k->specs.size(), name, name_cap, ne, dst, cap);
    const tts_tensor * t = k->specs[i].t;
    if (name && name_cap) {
        strncpy(name, t->name, name_cap - 1);
        name[name_cap - 1] = 0;
    }
    if (ne)
        for (int d = 0; d < 4; ++d) ne[d] = t->ne[d];
    return kokoro_read_weight(k->be, t, dst, cap);
}

extern "C" uint64_t tts_kokoro_get_node(tts_kokoro * k, int32_t which, const char * name, void * dst, uint64_t cap) {
    if (!k || !name) return 0;
    for (tts_tensor * t : (which ? k->gctx : k->dctx).nodes) {
        if (strcmp(t->name, name) != 0 || !tg::is_contiguous(t)) continue;
        const uint64_t nb = tg::nbytes(t);
        if (dst && cap >= nb && k->be.get(k->be.ctx, dst, t->data, nb) != 0) return 0;
        return nb;
    }
    return 0;
}

extern "C" tts_tensor * const * tts_kokoro_graph(const tts_kokoro * k, int32_t which, int32_t * n_nodes) {
    const tg::context * c = k ? (which ? &k->gctx : &k->dctx) : nullptr;
    if (n_nodes) *n_nodes = c ? (int32_t)c->nodes.size() : 0;
    return c ? c->nodes.data() : nullptr;
}
