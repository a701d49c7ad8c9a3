// DAC (Descript Audio Codec, 44.1 kHz) decoder runner: codec tokens -> PCM, the node list of
// dac_runner::build_dac_graph (/root/reference/src/decoder/dac_model.cpp:139-170) with
// general_neural_audio_codec::build_layer / build_residual_unit / build_quantize_layer
// (general_neural_audio_codec.cpp:133-172) and snake_1d / reciprocal (util.cpp:86-101).
// Runs on any tts_backend_iface (HIP backend, or the oracle in tests).  Weights are deterministic
// synthetic tensors in DAC-44k shapes (no checkpoints offline).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tts_gguf.h"
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
    const tts_gguf * gguf = nullptr;  // weight source while creating from a file (else synthetic)
    // batched decode (tts_dac_decode_batch): the prompt masks of the last (nb, T, gap), one per rate
    void * mask_buf = nullptr;
    size_t mask_bytes = 0;
    int32_t mask_key[3] = {0, 0, 0};
    std::vector<size_t> mask_off;  // float offset of rate level l's mask
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

// GGUF name of a weight: the reference's (dac_gguf_encoder.py's mapping, read back by
// dac_model.cpp:58-98 / general_neural_audio_codec.cpp:36-127); the runner's own constant has none.
static std::string gguf_name(const tts_tensor * t) { return std::string("audio_encoder.") + t->name; }

static bool same_squeezed_shape(const int64_t * a, const int64_t * b) {
    int64_t x[4], y[4];
    int nx = 0, ny = 0;
    for (int k = 0; k < 4; ++k) {
        if (a[k] != 1) x[nx++] = a[k];
        if (b[k] != 1) y[ny++] = b[k];
    }
    if (nx != ny) return false;
    for (int k = 0; k < nx; ++k)
        if (x[k] != y[k]) return false;
    return true;
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
        const void * src = nullptr;
        if (d->gguf && s.t != d->one) {  // assign_weight: the mapped file bytes
            const std::string fname = gguf_name(s.t);
            const int64_t i = tts_gguf_find_tensor(d->gguf, fname.c_str());
            int64_t ne[4] = {1, 1, 1, 1};
            if (i >= 0) tts_gguf_tensor_ndims(d->gguf, i, ne);
            if (i < 0 || tts_gguf_tensor_type(d->gguf, i) != TTS_TYPE_F32 || !same_squeezed_shape(ne, s.t->ne)) {
                fprintf(stderr, "gguf: DAC tensor '%s' %s (the decoder takes F32 [%lld %lld %lld])\n", fname.c_str(),
                        i < 0 ? "is missing" : "has another type or shape", (long long)s.t->ne[0], (long long)s.t->ne[1], (long long)s.t->ne[2]);
                return false;
            }
            src = tts_gguf_tensor_data(d->gguf, i);
        } else {
            host.resize(n);
            synth_f32(host.data(), n, s.seed, s.scale, s.offset);
            src = host.data();
        }
        if (d->be.set_tensor(d->be.ctx, s.t, src) != 0) return false;
    }
    return true;
}

// Declares every weight in the reference's order (synthetic seeds follow this order).
static void declare_weights(tts_dac * d) {
    const auto & c = d->cfg;
    for (int i = 0; i < c.n_codebooks; ++i) {
        dac_quant q;
        q.codebook = wnew(d, 1.0f, 0.f, c.codebook_dim, c.codebook_size, 1, "quantizers." + std::to_string(i) + ".codebook.weight");
        q.out_kernel = conv_w(d, 1, c.codebook_dim, c.latent_dim, "quantizers." + std::to_string(i) + ".out_proj.weight");
        q.out_bias = wnew(d, 0.01f, 0.f, 1, c.latent_dim, 1, "quantizers." + std::to_string(i) + ".out_proj.bias");
        d->quant.push_back(q);
    }
    d->in_kernel = conv_w(d, 7, c.latent_dim, c.decoder_dim, "initial.weight");
    d->in_bias = wnew(d, 0.01f, 0.f, 1, c.decoder_dim, 1, "initial.bias");
    int ch = c.decoder_dim;
    for (int l = 0; l < c.n_layers; ++l) {
        const int s = c.rates[l], oc = ch / 2;
        dac_layer L;
        const std::string pre = "decoder_block." + std::to_string(l + 1);
        L.stride = s;
        L.padding = (s + 1) / 2;  // DAC: ceil(stride / 2)
        L.in_alpha = wnew(d, 0.5f, 1.0f, 1, ch, 1, pre + ".final.alpha");
        L.kernel = wnew(d, std::sqrt(3.0f / (float)(2 * ch)), 0.f, 2 * s, oc, ch, pre + ".final.weight");
        L.bias = wnew(d, 0.01f, 0.f, 1, oc, 1, pre + ".final.bias");
        for (int r = 0; r < 3; ++r) {
            dac_ru & u = L.ru[r];
            const std::string rp = pre + ".residual_unit." + std::to_string(r);
            u.dilation = (int)std::pow(3, r);
            u.padding = 3 * u.dilation;
            u.in_alpha = wnew(d, 0.5f, 1.0f, 1, oc, 1, rp + ".res.initial.alpha");
            u.in_kernel = conv_w(d, 7, oc, oc, rp + ".res.initial.weight", 0.5f);
            u.in_bias = wnew(d, 0.01f, 0.f, 1, oc, 1, rp + ".res.initial.bias");
            u.out_alpha = wnew(d, 0.5f, 1.0f, 1, oc, 1, rp + ".res.final.alpha");
            u.out_kernel = conv_w(d, 1, oc, oc, rp + ".res.final.weight", 0.5f);
            u.out_bias = wnew(d, 0.01f, 0.f, 1, oc, 1, rp + ".res.final.bias");
        }
        d->layers.push_back(L);
        ch = oc;
    }
    d->out_alpha = wnew(d, 0.5f, 1.0f, 1, ch, 1, "final.alpha");
    d->out_kernel = conv_w(d, 7, ch, 1, "final.weight", 0.3f);
    d->out_bias = wnew(d, 0.01f, 0.f, 1, 1, 1, "final.bias");
    d->one = wnew(d, 0.f, 1.0f, 1, 1, 1, "one");
}

static tts_dac * dac_create(const tts_backend_iface * be, const tts_dac_config * cfg, const tts_gguf * g) {
    auto * d = new tts_dac();
    d->cfg = *cfg;
    d->be = *be;
    d->gguf = g;
    const auto & c = d->cfg;
    declare_weights(d);
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
    d->gguf = nullptr;
    return d;
}

extern "C" tts_dac * tts_dac_create(const tts_backend_iface * be, const tts_dac_config * cfg) { return dac_create(be, cfg, nullptr); }

extern "C" void tts_dac_free(tts_dac * d) {
    if (!d) return;
    if (d->arena) d->be.free(d->be.ctx, d->arena);
    if (d->mask_buf) d->be.free(d->be.ctx, d->mask_buf);
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

// masks (batched decode): masks[l] = [T_l, 1] f32 of rate level l (0 = latent frames, l = after block
// l), 1 inside a prompt's span and 0 in the gaps between prompts; `cur` is multiplied by the level's
// mask wherever a conv with reach > 0 (or a transposed conv) reads it next, so every prompt's outputs
// see zeros beyond its ends, exactly as the zero padding of a decode of its own
static tts_tensor * build_graph(tts_dac * d, int64_t T, const std::vector<tts_tensor *> * masks = nullptr) {
    const auto & cf = d->cfg;
    tg::context & c = d->gctx;
    c.reset();
    std::vector<tts_tensor *> mk;
    if (masks)
        for (size_t l = 0; l < masks->size(); ++l) {
            tts_tensor * m = tg::new_tensor_2d(c, TTS_TYPE_F32, (*masks)[l]->ne[0], 1);
            m->data = (*masks)[l]->data;  // the runner's mask buffer (not arena memory)
            mk.push_back(m);
        }
    auto gate = [&](tts_tensor * x, size_t l) { return l < mk.size() ? tg::mul(c, x, mk[l]) : x; };
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
    tts_tensor * cur = tg::conv_1d(c, d->in_kernel, gate(embd, 0), 1, 3, 1);
    cur = tg::add(c, cur, d->in_bias);
    size_t lvl = 0;
    for (auto & L : d->layers) {
        // build_layer (general_neural_audio_codec.cpp:151-163)
        cur = snake(d, c, L.in_alpha, gate(cur, lvl++));
        cur = tg::conv_transpose_1d(c, L.kernel, cur, L.stride, L.padding, 1, 0, 1);
        cur = tg::add(c, cur, L.bias);
        for (auto & u : L.ru) {
            // build_residual_unit (general_neural_audio_codec.cpp:133-149), groups = 1
            tts_tensor * residual = cur;  // (its gap values never reach a prompt: the next conv input is gated)
            cur = snake(d, c, u.in_alpha, gate(cur, lvl));
            cur = tg::conv_1d(c, u.in_kernel, cur, 1, u.padding, u.dilation);
            cur = tg::add(c, cur, u.in_bias);
            cur = snake(d, c, u.out_alpha, cur);
            cur = tg::conv_1d(c, u.out_kernel, cur, 1, 0, 1);
            cur = tg::add(c, cur, u.out_bias);
            cur = tg::add(c, cur, residual);
        }
    }
    cur = snake(d, c, d->out_alpha, gate(cur, lvl));
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

// Batched decode: nb prompts of T frames each as ONE graph over nb * T + (nb - 1) * gap frames, the
// prompts laid out along time with `gap` frames between them and the rate-level masks zeroing the
// gaps before every conv that reaches across (build_graph).  A prompt's PCM is the samples of its
// span: each of its outputs is the same sum of the same products as in a decode of its own (the
// terms a lone decode takes from zero padding come from the zeroed gap), so it is bit-identical to
// tts_dac_decode of that prompt.  Every node keeps the reference op's semantics (a serving-side
// layout, not a new op), so the oracle runs the same batched graph.  gap = 0: the smallest gap the
// convs' reach allows.
static int64_t dac_min_gap(const tts_dac * d) {
    int64_t g = 3, rate = 1;  // the initial conv (k 7, pad 3) at the latent rate
    for (const auto & L : d->layers) {
        rate *= L.stride;
        for (const auto & u : L.ru) g = std::max(g, (u.padding + rate - 1) / rate);
        g = std::max<int64_t>(g, 1);  // a transposed conv's first output of the next prompt: (T + gap) * s - p >= T * s
    }
    return std::max<int64_t>(g, (3 + rate - 1) / rate);  // the final conv (k 7, pad 3)
}

extern "C" int tts_dac_decode_batch(tts_dac * d, const int32_t * codes, int32_t nb, int32_t T, int32_t gap, float * pcm) {
    if (!d || nb <= 0 || T <= 0 || gap < 0) return TTS_STATUS_BAD_ARG;
    if (nb == 1) return tts_dac_decode(d, codes, T, pcm);
    // the layout assumes every transposed conv outputs exactly T * stride samples per prompt:
    // (T - 1) s - 2 ceil(s / 2) + 2 s = T s needs an even stride (an odd one gives T s - 1)
    for (const auto & L : d->layers)
        if (2 * L.padding != L.stride) return TTS_STATUS_BAD_ARG;
    const int64_t G = gap ? gap : dac_min_gap(d);
    if (G < dac_min_gap(d)) return TTS_STATUS_BAD_ARG;
    const int64_t span = T + G, Tt = (int64_t)nb * span - G;
    if (Tt > d->cfg.max_frames) return TTS_STATUS_BAD_ARG;
    const int ncb = d->cfg.n_codebooks;
    // the masks of (nb, T, G), kept while the shape repeats
    const int nl = (int)d->layers.size() + 1;
    if (d->mask_key[0] != nb || d->mask_key[1] != T || d->mask_key[2] != (int32_t)G || !d->mask_buf) {
        std::vector<float> host;
        d->mask_off.assign(nl, 0);
        int64_t rate = 1;
        for (int l = 0; l < nl; ++l) {
            if (l > 0) rate *= d->layers[l - 1].stride;
            d->mask_off[l] = host.size();
            const int64_t n = Tt * rate;
            for (int64_t i = 0; i < n; ++i) host.push_back((i / rate) % span < T ? 1.0f : 0.0f);
        }
        const size_t bytes = host.size() * sizeof(float);
        if (bytes > d->mask_bytes) {
            if (d->mask_buf) d->be.free(d->be.ctx, d->mask_buf);
            d->mask_buf = d->be.alloc(d->be.ctx, bytes);
            d->mask_bytes = d->mask_buf ? bytes : 0;
            if (!d->mask_buf) return TTS_STATUS_ALLOC_FAILED;
        }
        const int st = d->be.set(d->be.ctx, d->mask_buf, host.data(), bytes);
        if (st != 0) return st;
        d->mask_key[0] = nb, d->mask_key[1] = T, d->mask_key[2] = (int32_t)G;
    }
    tg::context mctx;  // the masks' descriptors (data in mask_buf)
    std::vector<tts_tensor *> masks;
    int64_t rate = 1;
    for (int l = 0; l < nl; ++l) {
        if (l > 0) rate *= d->layers[l - 1].stride;
        tts_tensor * m = tg::new_tensor_2d(mctx, TTS_TYPE_F32, Tt * rate, 1);
        m->data = (char *)d->mask_buf + d->mask_off[l] * sizeof(float);
        masks.push_back(m);
    }
    tts_tensor * out = build_graph(d, Tt, &masks);
    if (!tg::alloc_graph(d->gctx, d->arena, d->arena_size, true)) {
        fprintf(stderr, "dac: compute arena too small (%zu needed)\n", d->gctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    // codes of the gaps: code 0 (their embeddings are masked before the first conv)
    std::vector<int32_t> all((size_t)Tt * ncb, 0);
    for (int z = 0; z < nb; ++z)
        memcpy(all.data() + (size_t)z * span * ncb, codes + (size_t)z * T * ncb, sizeof(int32_t) * (size_t)T * ncb);
    int st = d->be.set(d->be.ctx, d->in_codes->data, all.data(), sizeof(int32_t) * all.size());
    if (st == 0) st = d->be.compute(d->be.ctx, d->gctx.nodes.data(), (int)d->gctx.nodes.size());
    const int64_t hop = tts_dac_hop(d);
    for (int z = 0; st == 0 && pcm && z < nb; ++z)
        st = d->be.get(d->be.ctx, pcm + (size_t)z * T * hop, (const char *)out->data + sizeof(float) * (size_t)z * span * hop,
                       sizeof(float) * (size_t)T * hop);
    return st;
}

extern "C" int64_t tts_dac_min_gap(const tts_dac * d) { return d ? dac_min_gap(d) : 0; }

extern "C" int32_t tts_dac_last_graph_nodes(const tts_dac * d) { return (int32_t)d->gctx.nodes.size(); }
extern "C" int32_t tts_dac_n_weights(const tts_dac * d) { return d ? (int32_t)d->specs.size() : 0; }
extern "C" uint64_t tts_dac_weight(tts_dac * d, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst,
                                   uint64_t cap) {
    if (!d || i < 0 || i >= (int32_t)d->specs.size()) return 0;
    return tg::weight_out(d->be, d->specs[i].t, name, name_cap, ne, type, dst, cap);
}

extern "C" tts_tensor * const * tts_dac_graph(const tts_dac * d, int32_t * n_nodes) {
    if (n_nodes) *n_nodes = d ? (int32_t)d->gctx.nodes.size() : 0;
    return d ? d->gctx.nodes.data() : nullptr;
}

// ---- GGUF loader path (dac_model::prep_constants / prep_layers / assign_weight) ----
static bool key_u32(const tts_gguf * g, std::initializer_list<const char *> keys, uint32_t * out) {
    for (const char * k : keys) {
        const int64_t i = tts_gguf_find_key(g, k);
        if (i >= 0 && tts_gguf_get_u32(g, i, out)) return true;
    }
    return false;
}

static int64_t tdim(const tts_gguf * g, const std::string & name, int k) {
    const int64_t i = tts_gguf_find_tensor(g, name.c_str());
    if (i < 0) return -1;
    int64_t ne[4];
    tts_gguf_tensor_ndims(g, i, ne);
    return ne[k];
}

extern "C" int tts_dac_config_from_gguf(const tts_gguf * g, tts_dac_config * c) {
    if (!g || !c) return TTS_STATUS_BAD_ARG;
    uint32_t v = 0;
    if (key_u32(g, {"parler-tts.decoder.output_heads", "output_heads", "dia.decoder.output_heads"}, &v)) c->n_codebooks = (int32_t)v;
    int n_layers = 0;
    for (int l = 0; l < 8; ++l) {  // prep_layers: dac_layer_stride_{l} / dac_layer_padding_{l} per block
        const std::string sk = "dac_layer_stride_" + std::to_string(l), pk = "dac_layer_padding_" + std::to_string(l);
        uint32_t s = 0, pd = 0;
        if (!key_u32(g, {("dac." + sk).c_str(), sk.c_str()}, &s)) break;
        if (!key_u32(g, {("dac." + pk).c_str(), pk.c_str()}, &pd)) {
            fprintf(stderr, "gguf: key %s must be specified for the DAC decoder\n", pk.c_str());
            return TTS_STATUS_BAD_ARG;
        }
        if (pd != (s + 1) / 2) {
            fprintf(stderr, "gguf: DAC block %d padding %u, the decoder assumes ceil(stride / 2) = %u\n", l, pd, (s + 1) / 2);
            return TTS_STATUS_UNSUPPORTED;
        }
        c->rates[l] = (int32_t)s;
        n_layers = l + 1;
    }
    if (n_layers == 0) {
        fprintf(stderr, "gguf: key dac_layer_stride_0 must be specified for the DAC decoder\n");
        return TTS_STATUS_BAD_ARG;
    }
    c->n_layers = n_layers;
    const int64_t cd = tdim(g, "audio_encoder.quantizers.0.codebook.weight", 0), cs = tdim(g, "audio_encoder.quantizers.0.codebook.weight", 1);
    const int64_t lat = tdim(g, "audio_encoder.initial.weight", 1), dd = tdim(g, "audio_encoder.initial.weight", 2);
    if (cd < 0 || cs < 0 || lat < 0 || dd < 0) {
        fprintf(stderr, "gguf: DAC tensors missing\n");
        return TTS_STATUS_BAD_ARG;
    }
    c->codebook_dim = (int32_t)cd;
    c->codebook_size = (int32_t)cs;
    c->latent_dim = (int32_t)lat;
    c->decoder_dim = (int32_t)dd;
    return TTS_STATUS_SUCCESS;
}

extern "C" tts_dac * tts_dac_create_from_gguf(const tts_backend_iface * be, const tts_dac_config * cfg, const tts_gguf * g) {
    if (!be || !cfg || !g) return nullptr;
    return dac_create(be, cfg, g);
}

namespace tts {
// The synthetic DAC-44k decoder as "audio_encoder.*" tensors + dac.* keys (dac_gguf_encoder.py:99-110).
void dac_write_synthetic(const tts_dac_config * cfg, tts_gguf_writer * w) {
    tts_dac d;  // declarations only
    d.cfg = *cfg;
    declare_weights(&d);
    int64_t hop = 1;
    for (int l = 0; l < cfg->n_layers; ++l) {
        hop *= cfg->rates[l];
        tts_gguf_set_u32(w, ("dac.dac_layer_stride_" + std::to_string(l)).c_str(), (uint32_t)cfg->rates[l]);
        tts_gguf_set_u32(w, ("dac.dac_layer_padding_" + std::to_string(l)).c_str(), (uint32_t)((cfg->rates[l] + 1) / 2));
    }
    tts_gguf_set_u32(w, "dac.up_scaling_factor", (uint32_t)hop);
    std::vector<float> host;
    for (auto & s : d.specs) {
        if (s.t == d.one) continue;
        const size_t n = (size_t)tg::nelements(s.t);
        host.resize(n);
        synth_f32(host.data(), n, s.seed, s.scale, s.offset);
        int nd = 3;
        while (nd > 1 && s.t->ne[nd - 1] == 1) --nd;
        tts_gguf_add_tensor(w, gguf_name(s.t).c_str(), TTS_TYPE_F32, nd, s.t->ne, host.data(), n * 4);
    }
}
}  // namespace tts
