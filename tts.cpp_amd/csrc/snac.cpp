// SNAC (Scale Neural Audio Codec, 24 kHz) decoder runner -- Orpheus' vocoder: three codebook
// streams at 1/4, 1/2 and 1x the latent frame rate -> PCM.  The node list of
// snac_runner::build_snac_graph (/root/reference/src/decoder/snac_model.cpp:130-159) with
// snac_build_audio_inputs (:86-109: per-head codebook lookup + 1x1 projection, repeat_interleave
// of the coarse heads through ggml_repeat), the depthwise input conv (ggml_conv_1d_dw, :141) and
// general_neural_audio_codec::build_layer / build_residual_unit / build_quantize_layer
// (general_neural_audio_codec.cpp:133-172) with the noise branch (conv_1d k = 1, MUL by the noise
// row, ADD) and grouped (depthwise) residual units.  The reference draws the noise on the host
// (random_normal_gen in snac_runner::set_inputs, :178); here the caller passes it in.
// Weights are deterministic synthetic tensors in SNAC-24kHz shapes (hubertsiuzdak/snac_24khz as
// Orpheus uses it: codebook 4096 x 8, latent 768, decoder 1024, rates 8,8,4,2, vq strides 4,2,1).
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "graph.h"
#include "synth.h"
#include "tts_hip.h"
#include "tts_runners.h"

using namespace tts;

namespace {

struct snac_ru {  // residual unit (general_neural_audio_codec.h:29-41), grouped: depthwise conv
    tts_tensor *in_alpha, *in_kernel, *in_bias, *out_alpha, *out_kernel, *out_bias;
    int padding, dilation;
};

struct snac_layer {  // decoder block (general_neural_audio_codec.h:43-58) with its noise kernel
    tts_tensor *in_alpha, *kernel, *bias, *noise_kernel;
    int stride, padding;
    snac_ru ru[3];
};

struct snac_quant {  // residual_vector_quantize_layer
    tts_tensor *codebook, *out_kernel, *out_bias;
};

struct wspec {
    tts_tensor * t;
    float scale, offset;
    uint64_t seed;
};

}  // namespace

struct tts_snac {
    tts_snac_config cfg;
    tts_backend_iface be;
    tg::context wctx;
    void * wbuf = nullptr;
    std::vector<snac_quant> quant;
    tts_tensor *in_kernel = nullptr, *in_bias = nullptr, *up_kernel = nullptr, *up_bias = nullptr;
    tts_tensor *out_alpha = nullptr, *out_kernel = nullptr, *out_bias = nullptr;
    tts_tensor * one = nullptr;  // the scalar 1.0 of reciprocal() (a device tensor, not a host static)
    std::vector<snac_layer> layers;
    char * arena = nullptr;
    size_t arena_size = 0;
    tg::context gctx;
    tts_tensor *in_codes = nullptr, *in_noise = nullptr;
    uint64_t tensor_index = 0;
    std::vector<wspec> specs;
};

extern "C" void tts_snac_default_config(tts_snac_config * c) {
    memset(c, 0, sizeof(*c));
    c->n_heads = 3;
    c->codebook_size = 4096;
    c->codebook_dim = 8;
    c->latent_dim = 768;
    c->decoder_dim = 1024;
    c->n_layers = 4;
    const int rates[4] = {8, 8, 4, 2};
    for (int i = 0; i < 4; ++i) c->rates[i] = rates[i];
    const int reps[3] = {4, 2, 1};
    for (int i = 0; i < 3; ++i) c->repeats[i] = reps[i];
    c->max_frames = 2048;
    c->seed = 0x5AAC5EEDull;
    c->arena_bytes = 0;
}

static tts_tensor * wnew(tts_snac * d, float scale, float offset, int64_t ne0, int64_t ne1, int64_t ne2, const std::string & name) {
    tts_tensor * t = tg::new_tensor_3d(d->wctx, TTS_TYPE_F32, ne0, ne1, ne2);
    tg::set_name(t, name);
    t->flags |= tg::TG_FLAG_PERSIST;
    d->specs.push_back({t, scale, offset, d->cfg.seed ^ (d->tensor_index++)});
    return t;
}

// conv kernel [K, IC, OC], uniform +-gain*sqrt(3/fan_in)
static tts_tensor * conv_w(tts_snac * d, int K, int IC, int OC, const std::string & name, float gain = 1.0f) {
    return wnew(d, gain * std::sqrt(3.0f / (float)(K * IC)), 0.f, K, IC, OC, name);
}

static bool upload(tts_snac * d) {
    size_t total = 0;
    for (auto & s : d->specs) total += (tg::nbytes(s.t) + 255) & ~(size_t)255;
    d->wbuf = d->be.alloc(d->be.ctx, total);
    if (!d->wbuf) return false;
    size_t off = 0;
    std::vector<float> host;
    for (auto & s : d->specs) {
        const size_t n = (size_t)tg::nelements(s.t);
        s.t->data = (char *)d->wbuf + off;
        off += (tg::nbytes(s.t) + 255) & ~(size_t)255;
        host.resize(n);
        synth_f32(host.data(), n, s.seed, s.scale, s.offset);
        if (d->be.set_tensor(d->be.ctx, s.t, host.data()) != 0) return false;
    }
    return true;
}

static int64_t snac_hop(const tts_snac_config & c) {
    int64_t hop = 1;
    for (int l = 0; l < c.n_layers; ++l) hop *= c.rates[l];
    return hop;
}

extern "C" tts_snac * tts_snac_create(const tts_backend_iface * be, const tts_snac_config * cfg) {
    if (!be || !cfg || cfg->n_heads < 1 || cfg->n_heads > 4 || cfg->n_layers < 1 || cfg->n_layers > 8) return nullptr;
    auto * d = new tts_snac();
    d->cfg = *cfg;
    d->be = *be;
    const auto & c = d->cfg;
    for (int i = 0; i < c.n_heads; ++i) {
        snac_quant q;
        const std::string pre = "quantizers." + std::to_string(i);
        q.codebook = wnew(d, 1.0f, 0.f, c.codebook_dim, c.codebook_size, 1, pre + ".codebook.weight");
        q.out_kernel = conv_w(d, 1, c.codebook_dim, c.latent_dim, pre + ".out_proj.weight");
        q.out_bias = wnew(d, 0.01f, 0.f, 1, c.latent_dim, 1, pre + ".out_proj.bias");
        d->quant.push_back(q);
    }
    // depthwise input conv (kernel [7, 1, latent]) and the 1x1 up projection (snac_model.cpp:141-144)
    d->in_kernel = wnew(d, std::sqrt(3.0f / 7.0f), 0.f, 7, 1, c.latent_dim, "in.weight");
    d->in_bias = wnew(d, 0.01f, 0.f, 1, c.latent_dim, 1, "in.bias");
    d->up_kernel = conv_w(d, 1, c.latent_dim, c.decoder_dim, "up.weight");
    d->up_bias = wnew(d, 0.01f, 0.f, 1, c.decoder_dim, 1, "up.bias");
    int ch = c.decoder_dim;
    for (int l = 0; l < c.n_layers; ++l) {
        const int s = c.rates[l], oc = ch / 2;
        snac_layer L;
        const std::string pre = "layers." + std::to_string(l);
        L.stride = s;
        L.padding = (s + 1) / 2;  // SNAC DecoderBlock: ceil(stride / 2), output_padding stride % 2 = 0
        L.in_alpha = wnew(d, 0.5f, 1.0f, 1, ch, 1, pre + ".alpha");
        L.kernel = wnew(d, std::sqrt(3.0f / (float)(2 * ch)), 0.f, 2 * s, oc, ch, pre + ".weight");
        L.bias = wnew(d, 0.01f, 0.f, 1, oc, 1, pre + ".bias");
        L.noise_kernel = conv_w(d, 1, oc, oc, pre + ".noise_weight", 0.3f);
        for (int r = 0; r < 3; ++r) {
            snac_ru & u = L.ru[r];
            const std::string rp = pre + ".residual_unit." + std::to_string(r);
            u.dilation = (int)std::pow(3, r);
            u.padding = 3 * u.dilation;  // pow(3, r + 1) (general_neural_audio_codec.h:46)
            u.in_alpha = wnew(d, 0.5f, 1.0f, 1, oc, 1, rp + ".in_alpha");
            u.in_kernel = wnew(d, 0.5f * std::sqrt(3.0f / 7.0f), 0.f, 7, 1, oc, rp + ".in_weight");  // groups = channels
            u.in_bias = wnew(d, 0.01f, 0.f, 1, oc, 1, rp + ".in_bias");
            u.out_alpha = wnew(d, 0.5f, 1.0f, 1, oc, 1, rp + ".out_alpha");
            u.out_kernel = conv_w(d, 1, oc, oc, rp + ".out_weight", 0.5f);
            u.out_bias = wnew(d, 0.01f, 0.f, 1, oc, 1, rp + ".out_bias");
        }
        d->layers.push_back(L);
        ch = oc;
    }
    d->out_alpha = wnew(d, 0.5f, 1.0f, 1, ch, 1, "alpha_out");
    d->out_kernel = conv_w(d, 7, ch, 1, "final.weight", 0.1f);
    d->out_bias = wnew(d, 0.01f, 0.f, 1, 1, 1, "final.bias");
    d->one = wnew(d, 0.f, 1.0f, 1, 1, 1, "one");
    if (!upload(d)) {
        tts_snac_free(d);
        return nullptr;
    }
    // arena: the widest activations are the last blocks' [T*hop, C] tensors plus their F16 im2cols
    const int64_t hop = snac_hop(c);
    const size_t last = (size_t)c.max_frames * (size_t)hop * (size_t)(c.decoder_dim >> c.n_layers) * 4;
    d->arena_size = c.arena_bytes ? c.arena_bytes : last * 24 + ((size_t)64 << 20);
    d->arena = (char *)d->be.alloc(d->be.ctx, d->arena_size);
    if (!d->arena) {
        tts_snac_free(d);
        return nullptr;
    }
    return d;
}

extern "C" void tts_snac_free(tts_snac * d) {
    if (!d) return;
    if (d->arena) d->be.free(d->be.ctx, d->arena);
    if (d->wbuf) d->be.free(d->be.ctx, d->wbuf);
    delete d;
}

extern "C" int64_t tts_snac_hop(const tts_snac * d) { return snac_hop(d->cfg); }

extern "C" int64_t tts_snac_noise_per_frame(const tts_snac * d) {
    // noise_steps (snac_model.h:19): the cumulative upsampling after each block, 8 + 64 + 256 + 512
    int64_t n = 0, up = 1;
    for (int l = 0; l < d->cfg.n_layers; ++l) n += (up *= d->cfg.rates[l]);
    return n;
}

// snake_1d (util.cpp:98-101): x + sin(alpha*x)^2 * (1/alpha), reciprocal() as DIV of a broadcast 1.0
static tts_tensor * snake(tts_snac * d, tg::context & c, tts_tensor * alpha, tts_tensor * x) {
    tts_tensor * one = tg::view_2d(c, d->one, 1, alpha->ne[1], 0, 0);
    tts_tensor * recip = tg::div(c, one, alpha);
    return tg::add(c, x, tg::mul(c, tg::sqr(c, tg::sin(c, tg::mul(c, x, alpha))), recip));
}

static tts_tensor * build_graph(tts_snac * d, int64_t T) {
    const auto & cf = d->cfg;
    tg::context & c = d->gctx;
    c.reset();
    // snac_build_audio_inputs (snac_model.cpp:86-109): head i holds T / repeats[i] codes, stored
    // back to back in one I32 input
    int64_t ncodes = 0;
    for (int i = 0; i < cf.n_heads; ++i) ncodes += T / cf.repeats[i];
    d->in_codes = tg::new_tensor_1d(c, TTS_TYPE_I32, ncodes);
    tg::set_input(d->in_codes);
    tts_tensor * embd = nullptr;
    size_t stride = 0;
    for (int i = 0; i < cf.n_heads; ++i) {
        const int64_t Ti = T / cf.repeats[i];
        tts_tensor * head = tg::cont(c, tg::view_1d(c, d->in_codes, Ti, stride));
        stride += (size_t)Ti * 4;
        // build_quantize_layer (general_neural_audio_codec.cpp:166-172)
        tts_tensor * code = tg::get_rows(c, d->quant[i].codebook, head);
        code = tg::cont(c, tg::transpose(c, code));
        code = tg::conv_1d(c, d->quant[i].out_kernel, code, 1, 0, 1);
        code = tg::add(c, code, d->quant[i].out_bias);
        if (cf.repeats[i] > 1) {
            // repeat_interleave along time through ggml_repeat (snac_model.cpp:97-101)
            tts_tensor * shape = tg::new_tensor_3d(c, TTS_TYPE_F32, cf.repeats[i], code->ne[0], cf.latent_dim);
            code = tg::repeat(c, tg::cont_3d(c, code, 1, code->ne[0], code->ne[1]), shape);
            code = tg::cont_2d(c, code, T, code->ne[2]);
        }
        embd = i == 0 ? code : tg::add(c, embd, code);
    }
    d->in_noise = tg::new_tensor_1d(c, TTS_TYPE_F32, tts_snac_noise_per_frame(d) * T);
    tg::set_input(d->in_noise);
    tg::set_name(embd, "embd");
    tts_tensor * cur = tg::conv_1d_dw(c, d->in_kernel, embd, 1, 3, 1);
    cur = tg::add(c, cur, d->in_bias);
    tg::set_name(cur, "in_conv");
    cur = tg::conv_1d(c, d->up_kernel, cur, 1, 0, 1);
    cur = tg::add(c, cur, d->up_bias);
    tg::set_name(cur, "up");
    int li = 0;
    size_t noise_off = 0;
    int64_t up = 1;
    for (auto & L : d->layers) {
        up *= L.stride;
        tts_tensor * noise = tg::cont(c, tg::view_1d(c, d->in_noise, up * T, noise_off));
        noise_off += (size_t)(up * T) * 4;
        // general_neural_audio_codec::build_layer (general_neural_audio_codec.cpp:151-164)
        cur = snake(d, c, L.in_alpha, cur);
        cur = tg::conv_transpose_1d(c, L.kernel, cur, L.stride, L.padding, 1, 0, 1);
        cur = tg::add(c, cur, L.bias);
        tg::set_name(cur, "convt." + std::to_string(li));
        tts_tensor * x = tg::conv_1d(c, L.noise_kernel, cur, 1, 0, 1);
        x = tg::mul(c, x, noise);
        cur = tg::add(c, cur, x);
        tg::set_name(cur, "noise." + std::to_string(li));
        int ri = 0;
        for (auto & u : L.ru) {
            // build_residual_unit (general_neural_audio_codec.cpp:133-149), groups > 1
            tts_tensor * residual = cur;
            cur = snake(d, c, u.in_alpha, cur);
            cur = tg::conv_1d_dw(c, u.in_kernel, cur, 1, u.padding, u.dilation);
            cur = tg::add(c, cur, u.in_bias);
            cur = snake(d, c, u.out_alpha, cur);
            cur = tg::conv_1d(c, u.out_kernel, cur, 1, 0, 1);
            cur = tg::add(c, cur, u.out_bias);
            cur = tg::add(c, cur, residual);
            tg::set_name(cur, "ru." + std::to_string(li) + "." + std::to_string(ri++));
        }
        ++li;
    }
    cur = snake(d, c, d->out_alpha, cur);
    cur = tg::conv_1d(c, d->out_kernel, cur, 1, 3, 1);
    cur = tg::add(c, cur, d->out_bias);
    cur = tg::tanh(c, cur);
    tg::set_name(cur, "pcm");
    tg::set_output(cur);
    tg::build_forward_expand(c, cur);
    return cur;
}

extern "C" int tts_snac_decode(tts_snac * d, const int32_t * codes, int32_t T, const float * noise, float * pcm) {
    if (!d || !codes || !noise || T <= 0 || T > d->cfg.max_frames) return TTS_STATUS_BAD_ARG;
    for (int i = 0; i < d->cfg.n_heads; ++i)
        if (T % d->cfg.repeats[i]) return TTS_STATUS_BAD_ARG;  // every head covers whole frames
    tts_tensor * out = build_graph(d, T);
    if (!tg::alloc_graph(d->gctx, d->arena, d->arena_size, !d->cfg.debug_no_reuse)) {
        fprintf(stderr, "snac: compute arena too small (%zu needed)\n", d->gctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    int st = d->be.set(d->be.ctx, d->in_codes->data, codes, tg::nbytes(d->in_codes));
    if (st == 0) st = d->be.set(d->be.ctx, d->in_noise->data, noise, tg::nbytes(d->in_noise));
    if (st == 0) st = d->be.compute(d->be.ctx, d->gctx.nodes.data(), (int)d->gctx.nodes.size());
    if (st == 0 && pcm) st = d->be.get(d->be.ctx, pcm, out->data, sizeof(float) * (size_t)tg::nelements(out));
    return st;
}

extern "C" int32_t tts_snac_last_graph_nodes(const tts_snac * d) { return (int32_t)d->gctx.nodes.size(); }

extern "C" int32_t tts_snac_n_weights(const tts_snac * d) { return d ? (int32_t)d->specs.size() : 0; }

extern "C" uint64_t tts_snac_weight(tts_snac * d, int32_t i, char * name, uint64_t name_cap, int64_t * ne, float * dst, uint64_t cap) {
    if (!d || i < 0 || i >= (int32_t)d->specs.size()) return 0;
    const tts_tensor * t = d->specs[i].t;
    if (name && name_cap) {
        strncpy(name, t->name, name_cap - 1);
        name[name_cap - 1] = 0;
    }
    if (ne)
        for (int k = 0; k < 4; ++k) ne[k] = t->ne[k];
    const uint64_t n = tg::nbytes(t);
    if (dst && cap >= n && d->be.get(d->be.ctx, dst, t->data, n) != 0) return 0;
    return n;
}

// Debug: copy the named node of the last graph to host (contiguous nodes only); returns bytes.
extern "C" uint64_t tts_snac_get_node(tts_snac * d, const char * name, void * dst, uint64_t cap) {
    if (!d || !name) return 0;
    for (tts_tensor * t : d->gctx.nodes) {
        if (strcmp(t->name, name) != 0 || !tg::is_contiguous(t)) continue;
        const uint64_t n = tg::nbytes(t);
        if (dst && cap >= n && d->be.get(d->be.ctx, dst, t->data, n) != 0) return 0;
        return n;
    }
    return 0;
}
