// DAC (Descript Audio Codec, 44.1 kHz) decoder runner: codec tokens -> PCM, the node list of
// dac_runner::build_dac_graph (/root/reference/src/decoder/dac_model.cpp:139-170) with
// general_neural_audio_codec::build_layer / build_residual_unit / build_quantize_layer
// (general_neural_audio_codec.cpp:133-172) and snake_1d / reciprocal (util.cpp:86-101).
// Runs on any tts_backend_iface (HIP backend, or the oracle in tests).  Weights are deterministic
// synthetic tensors in DAC-44k shapes (no checkpoints offline).
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

struct dac_ru {  // residual unit (general_neural_audio_codec.h:30-40)
    tts_tensor *in_alpha, *in_kernel, *in_bias, *out_alpha, *out_kernel, *out_bias;
    int padding, dilation;
};

struct dac_layer {  // decoder block (general_neural_audio_codec.h:44-56)
    tts_tensor *in_alpha, *kernel, *bias;
    int stride, padding;
    dac_ru ru[3];
};

struct dac_quant {  // residual_vector_quantize_layer
    tts_tensor *codebook, *out_kernel, *out_bias;
};

struct wspec {
    tts_tensor * t;
    float scale, offset;
    uint64_t seed;
};

}  // namespace

struct tts_dac {
    tts_dac_config cfg;
    tts_backend_iface be;
    tg::context wctx;
    void * wbuf = nullptr;
    std::vector<dac_quant> quant;
    tts_tensor *in_kernel = nullptr, *in_bias = nullptr, *out_alpha = nullptr, *out_kernel = nullptr, *out_bias = nullptr;
    tts_tensor * one = nullptr;  // the scalar 1.0 of reciprocal() (a device tensor, not a host static)
    std::vector<dac_layer> layers;
    char * arena = nullptr;
    size_t arena_size = 0;
    tg::context gctx;
    tts_tensor * in_codes = nullptr;
    uint64_t tensor_index = 0;
    std::vector<wspec> specs;
};

extern "C" void tts_dac_default_config(tts_dac_config * c) {
    memset(c, 0, sizeof(*c));
    c->n_codebooks = 9;
    c->codebook_size = 1024;
    c->codebook_dim = 8;
    c->latent_dim = 1024;
    c->decoder_dim = 1536;
    c->n_layers = 4;
    const int rates[4] = {8, 8, 4, 2};
    for (int i = 0; i < 4; ++i) c->rates[i] = rates[i];
    c->max_frames = 1024;
    c->seed = 0xDAC5EED;
    c->arena_bytes = 0;
}

static tts_tensor * wnew(tts_dac * d, float scale, float offset, int64_t ne0, int64_t ne1, int64_t ne2, const std::string & name) {
    tts_tensor * t = tg::new_tensor_3d(d->wctx, TTS_TYPE_F32, ne0, ne1, ne2);
    tg::set_name(t, name);
    t->flags |= tg::TG_FLAG_PERSIST;
    d->specs.push_back({t, scale, offset, d->cfg.seed ^ (d->tensor_index++)});
    return t;
}

// conv kernel [K, IC, OC], uniform +-gain*sqrt(3/fan_in): gain 1 preserves the variance; the
// residual branches use less so the synthetic decoder keeps activations O(1) and the final tanh
// out of saturation (a trained DAC does the same through its weights)
static tts_tensor * conv_w(tts_dac * d, int K, int IC, int OC, const std::string & name, float gain = 1.0f) {
    return wnew(d, gain * std::sqrt(3.0f / (float)(K * IC)), 0.f, K, IC, OC, name);
}

static bool upload(tts_dac * d) {
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

extern "C" tts_dac * tts_dac_create(const tts_backend_iface * be, const tts_dac_config * cfg) {
    auto * d = new tts_dac();
    d->cfg = *cfg;
    d->be = *be;
    const auto & c = d->cfg;
    for (int i = 0; i < c.n_codebooks; ++i) {
        dac_quant q;
        q.codebook = wnew(d, 1.0f, 0.f, c.codebook_dim, c.codebook_size, 1, "quantizer." + std::to_string(i) + ".codebook");
        q.out_kernel = conv_w(d, 1, c.codebook_dim, c.latent_dim, "quantizer." + std::to_string(i) + ".out_proj.weight");
        q.out_bias = wnew(d, 0.01f, 0.f, 1, c.latent_dim, 1, "quantizer." + std::to_string(i) + ".out_proj.bias");
        d->quant.push_back(q);
    }
    d->in_kernel = conv_w(d, 7, c.latent_dim, c.decoder_dim, "decoder.in.weight");
    d->in_bias = wnew(d, 0.01f, 0.f, 1, c.decoder_dim, 1, "decoder.in.bias");
    int ch = c.decoder_dim;
    for (int l = 0; l < c.n_layers; ++l) {
        const int s = c.rates[l], oc = ch / 2;
        dac_layer L;
        const std::string pre = "decoder.layer." + std::to_string(l);
        L.stride = s;
        L.padding = (s + 1) / 2;  // DAC: ceil(stride / 2)
        L.in_alpha = wnew(d, 0.5f, 1.0f, 1, ch, 1, pre + ".alpha");
        L.kernel = wnew(d, std::sqrt(3.0f / (float)(2 * ch)), 0.f, 2 * s, oc, ch, pre + ".convT.weight");
        L.bias = wnew(d, 0.01f, 0.f, 1, oc, 1, pre + ".convT.bias");
        for (int r = 0; r < 3; ++r) {
            dac_ru & u = L.ru[r];
            const std::string rp = pre + ".res." + std::to_string(r);
            u.dilation = (int)std::pow(3, r);
            u.padding = 3 * u.dilation;
            u.in_alpha = wnew(d, 0.5f, 1.0f, 1, oc, 1, rp + ".alpha1");
            u.in_kernel = conv_w(d, 7, oc, oc, rp + ".conv1.weight", 0.5f);
            u.in_bias = wnew(d, 0.01f, 0.f, 1, oc, 1, rp + ".conv1.bias");
            u.out_alpha = wnew(d, 0.5f, 1.0f, 1, oc, 1, rp + ".alpha2");
            u.out_kernel = conv_w(d, 1, oc, oc, rp + ".conv2.weight", 0.5f);
            u.out_bias = wnew(d, 0.01f, 0.f, 1, oc, 1, rp + ".conv2.bias");
        }
        d->layers.push_back(L);
        ch = oc;
    }
    d->out_alpha = wnew(d, 0.5f, 1.0f, 1, ch, 1, "decoder.out.alpha");
    d->out_kernel = conv_w(d, 7, ch, 1, "decoder.out.weight", 0.3f);
    d->out_bias = wnew(d, 0.01f, 0.f, 1, 1, 1, "decoder.out.bias");
    d->one = wnew(d, 0.f, 1.0f, 1, 1, 1, "one");
    if (!upload(d)) {
        tts_dac_free(d);
        return nullptr;
    }
    // arena: the largest activations are the last stage's [T*hop, C/16] tensors (a few alive at
    // once) plus its im2col [7*C/16, T*hop] in F16
    int64_t hop = 1;
    for (int l = 0; l < c.n_layers; ++l) hop *= c.rates[l];
    const int64_t chl = c.decoder_dim >> c.n_layers;
    d->arena_size = c.arena_bytes ? c.arena_bytes : (size_t)c.max_frames * (size_t)hop * (size_t)chl * 4 * 12 + ((size_t)64 << 20);
    d->arena = (char *)d->be.alloc(d->be.ctx, d->arena_size);
    if (!d->arena) {
        tts_dac_free(d);
        return nullptr;
    }
    return d;
}

extern "C" void tts_dac_free(tts_dac * d) {
    if (!d) return;
    if (d->arena) d->be.free(d->be.ctx, d->arena);
    if (d->wbuf) d->be.free(d->be.ctx, d->wbuf);
    delete d;
}

extern "C" int64_t tts_dac_hop(const tts_dac * d) {
    int64_t hop = 1;
    for (int l = 0; l < d->cfg.n_layers; ++l) hop *= d->cfg.rates[l];
    return hop;
}

// snake_1d (util.cpp:98-101): x + sin(alpha*x)^2 * (1/alpha), reciprocal() as DIV of a broadcast 1.0
static tts_tensor * snake(tts_dac * d, tg::context & c, tts_tensor * alpha, tts_tensor * x) {
    tts_tensor * one = tg::view_2d(c, d->one, 1, alpha->ne[1], 0, 0);
    tts_tensor * recip = tg::div(c, one, alpha);
    return tg::add(c, x, tg::mul(c, tg::sqr(c, tg::sin(c, tg::mul(c, x, alpha))), recip));
}

static tts_tensor * build_graph(tts_dac * d, int64_t T) {
    const auto & cf = d->cfg;
    tg::context & c = d->gctx;
    c.reset();
    // dac_build_audio_inputs (dac_model.cpp:100-123): codes [T * n_codebooks], time-major
    d->in_codes = tg::new_tensor_1d(c, TTS_TYPE_I32, T * cf.n_codebooks);
    tg::set_input(d->in_codes);
    tts_tensor * embd = nullptr;
    for (int i = 0; i < cf.n_codebooks; ++i) {
        tts_tensor * code = tg::cont(c, tg::view_2d(c, d->in_codes, 1, T, (size_t)cf.n_codebooks * 4, (size_t)i * 4));
        code = tg::reshape_1d(c, code, T);
        // build_quantize_layer (general_neural_audio_codec.cpp:166-172)
        tts_tensor * cur = tg::get_rows(c, d->quant[i].codebook, code);
        cur = tg::cont(c, tg::transpose(c, cur));
        cur = tg::conv_1d(c, d->quant[i].out_kernel, cur, 1, 0, 1);
        cur = tg::add(c, cur, d->quant[i].out_bias);
        embd = i == 0 ? cur : tg::add(c, embd, cur);
    }
    tts_tensor * cur = tg::conv_1d(c, d->in_kernel, embd, 1, 3, 1);
    cur = tg::add(c, cur, d->in_bias);
    for (auto & L : d->layers) {
        // build_layer (general_neural_audio_codec.cpp:151-163)
        cur = snake(d, c, L.in_alpha, cur);
        cur = tg::conv_transpose_1d(c, L.kernel, cur, L.stride, L.padding, 1, 0, 1);
        cur = tg::add(c, cur, L.bias);
        for (auto & u : L.ru) {
            // build_residual_unit (general_neural_audio_codec.cpp:133-149), groups = 1
            tts_tensor * residual = cur;
            cur = snake(d, c, u.in_alpha, cur);
            cur = tg::conv_1d(c, u.in_kernel, cur, 1, u.padding, u.dilation);
            cur = tg::add(c, cur, u.in_bias);
            cur = snake(d, c, u.out_alpha, cur);
            cur = tg::conv_1d(c, u.out_kernel, cur, 1, 0, 1);
            cur = tg::add(c, cur, u.out_bias);
            cur = tg::add(c, cur, residual);
        }
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

extern "C" int tts_dac_decode(tts_dac * d, const int32_t * codes, int32_t T, float * pcm) {
    if (!d || T <= 0 || T > d->cfg.max_frames) return TTS_STATUS_BAD_ARG;
    tts_tensor * out = build_graph(d, T);
    if (!tg::alloc_graph(d->gctx, d->arena, d->arena_size, true)) {
        fprintf(stderr, "dac: compute arena too small (%zu needed)\n", d->gctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    int st = d->be.set(d->be.ctx, d->in_codes->data, codes, sizeof(int32_t) * (size_t)T * d->cfg.n_codebooks);
    if (st == 0) st = d->be.compute(d->be.ctx, d->gctx.nodes.data(), (int)d->gctx.nodes.size());
    if (st == 0 && pcm) st = d->be.get(d->be.ctx, pcm, out->data, sizeof(float) * (size_t)tg::nelements(out));
    return st;
}

extern "C" int32_t tts_dac_last_graph_nodes(const tts_dac * d) { return (int32_t)d->gctx.nodes.size(); }
