// Kokoro-82M iSTFTNet generator runner: decoder features + F0 curve + style -> 24 kHz PCM.  The
// node list of build_generator (/root/reference/src/models/kokoro/model.cpp:195-244) with
// build_sin_gen (:172-193), build_noise_block (:167-171), build_kokoro_generator_res_block
// (:136-165), snake_1d / reciprocal (util.cpp:86-101) and the util.cpp stft / istft wrappers
// (:111-130).  The reference's uv / noise custom map (uv_noise_compute, util.cpp:140-170, a CPU
// ggml_map_custom3) is the same MAP_CUSTOM3 node here, run by the backend on the device over the
// upscaled F0 it reads; its uniform draws and the window-envelope normaliser
// (compute_window_squared_sum, util.cpp:203-217) are host inputs, as in kokoro_runner::set_inputs.
// Weights are deterministic synthetic tensors in Kokoro-82M shapes (no checkpoints offline).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "graph.h"
#include "common.h"
#include "kokoro_gen.h"
#include "synth.h"
#include "tts_hip.h"
#include "tts_runners.h"

using namespace tts;

namespace {

// kokoro_generator_residual_block (model.h): three AdaIN -> snake -> dilated conv -> AdaIN ->
// snake -> conv units, each added back onto the block input
struct kk_res {
    tts_tensor *g1w[3], *g1b[3], *b1w[3], *b1b[3], *g2w[3], *g2b[3], *b2w[3], *b2b[3];
    tts_tensor *a1[3], *a2[3], *c1w[3], *c1b[3], *c2w[3], *c2b[3];
    int pad[3], dil[3];
};

struct kk_up {  // kokoro_generator_upsample_block + its kokoro_noise_residual_block
    tts_tensor *w, *b;
    int stride, padding;
    tts_tensor *nw, *nb;
    int nstride, npadding;
    kk_res nres;
};

struct wspec {
    tts_tensor * t;
    float scale, offset;
    uint64_t seed;
};

constexpr int kUpsample = 300;  // build_sin_gen's fixed interpolation factor (model.cpp:175, :196)

}  // namespace

struct tts_kokoro_gen {
    tts_kokoro_gen_config cfg;
    tts_backend_iface be;
    tg::context wctx;
    void * wbuf = nullptr;
    std::vector<wspec> specs;
    uint64_t tensor_index = 0;
    std::vector<kk_up> ups;
    std::vector<kk_res> res;  // n_ups * n_kernels
    tts_tensor *m_w = nullptr, *m_b = nullptr, *out_w = nullptr, *out_b = nullptr;
    // constants the reference builds in post_load_assign (model.cpp:305-392)
    tts_tensor *window = nullptr, *harm_norm = nullptr, *samp_scalar = nullptr, *nker = nullptr, *one = nullptr;
    char * arena = nullptr;
    size_t arena_size = 0;
    tg::context gctx;
    tts_tensor *in_x = nullptr, *in_f0 = nullptr, *in_style = nullptr, *in_uvdata = nullptr, *in_wss = nullptr;
    bool device_draws = false;
    std::vector<float> h_uvdata, h_wss, h_window;
    int64_t h_wss_len = -1;  // h_wss holds the window sum of squares for this output length (reused while it repeats)
};

extern "C" void tts_kokoro_gen_default_config(tts_kokoro_gen_config * c) {
    memset(c, 0, sizeof(*c));
    c->in_channels = 512;
    c->style_dim = 128;
    c->n_ups = 2;
    c->up_rates[0] = 10, c->up_rates[1] = 6;
    c->up_kernels[0] = 20, c->up_kernels[1] = 12;
    c->n_kernels = 3;
    c->res_kernels[0] = 3, c->res_kernels[1] = 7, c->res_kernels[2] = 11;
    c->res_dilations[0] = 1, c->res_dilations[1] = 3, c->res_dilations[2] = 5;
    c->noise_res_kernels[0] = 7, c->noise_res_kernels[1] = 11;
    c->n_fft = 20;
    c->hop = 5;
    c->harmonic_num = 8;
    c->sample_rate = 24000.0f;
    c->sin_amp = 0.1f;
    c->noise_std = 0.003f;
    c->voice_threshold = 10.0f;
    c->max_frames = 1024;
    c->seed = 0x6B0C0E0;
    c->arena_bytes = 0;
}

// gguf = false: a constant kokoro's post_load_assign builds (model.cpp:305-392), never in the file (F32)
static tts_tensor * wnew(tts_kokoro_gen * k, float scale, float offset, int64_t ne0, int64_t ne1, int64_t ne2, const std::string & name,
                         bool gguf = true) {
    const int ty = gguf && k->cfg.weight_type == TTS_TYPE_F16 && kokoro_f16_tensor(name, ne1) ? TTS_TYPE_F16 : TTS_TYPE_F32;
    tts_tensor * t = ne1 == 0 ? tg::new_tensor_1d(k->wctx, ty, ne0) : tg::new_tensor_3d(k->wctx, ty, ne0, ne1, ne2);
    tg::set_name(t, name);
    t->flags |= tg::TG_FLAG_PERSIST;
    k->specs.push_back({t, scale, offset, k->cfg.seed ^ (k->tensor_index++)});
    return t;
}

// conv kernel [K, IC, OC], uniform +-gain*sqrt(3/fan_in)
static tts_tensor * conv_w(tts_kokoro_gen * k, int K, int IC, int OC, const std::string & name, float gain = 1.0f) {
    return wnew(k, gain * std::sqrt(3.0f / (float)(K * IC)), 0.f, K, IC, OC, name);
}

static void make_res(tts_kokoro_gen * k, kk_res & r, int C, int kernel, const std::string & pre) {
    const int S = k->cfg.style_dim;
    const float sw = 0.1f * std::sqrt(3.0f / (float)S);  // AdaIN gamma / beta stay ~0.1
    for (int i = 0; i < 3; ++i) {
        const std::string p = pre + "." + std::to_string(i);
        r.dil[i] = k->cfg.res_dilations[i];
        r.pad[i] = r.dil[i] * (kernel - 1) / 2;
        r.g1w[i] = wnew(k, sw, 0.f, S, C, 1, p + ".gamma1_weight");
        r.g1b[i] = wnew(k, 0.05f, 0.f, C, 0, 0, p + ".gamma1_bias");
        r.b1w[i] = wnew(k, sw, 0.f, S, C, 1, p + ".beta1_weight");
        r.b1b[i] = wnew(k, 0.05f, 0.f, C, 0, 0, p + ".beta1_bias");
        r.g2w[i] = wnew(k, sw, 0.f, S, C, 1, p + ".gamma2_weight");
        r.g2b[i] = wnew(k, 0.05f, 0.f, C, 0, 0, p + ".gamma2_bias");
        r.b2w[i] = wnew(k, sw, 0.f, S, C, 1, p + ".beta2_weight");
        r.b2b[i] = wnew(k, 0.05f, 0.f, C, 0, 0, p + ".beta2_bias");
        r.a1[i] = wnew(k, 0.5f, 1.0f, 1, C, 1, p + ".alpha1");
        r.a2[i] = wnew(k, 0.5f, 1.0f, 1, C, 1, p + ".alpha2");
        r.c1w[i] = conv_w(k, kernel, C, C, p + ".convs1_weight", 0.5f);
        r.c1b[i] = wnew(k, 0.01f, 0.f, 1, C, 1, p + ".convs1_bias");
        r.c2w[i] = conv_w(k, kernel, C, C, p + ".convs2_weight", 0.5f);
        r.c2b[i] = wnew(k, 0.01f, 0.f, 1, C, 1, p + ".convs2_bias");
    }
}

static int64_t upsample_total(const tts_kokoro_gen_config & c) {
    int64_t u = c.hop;
    for (int i = 0; i < c.n_ups; ++i) u *= c.up_rates[i];
    return u;
}

static bool upload(tts_kokoro_gen * k) {
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

namespace tts {
bool kokoro_upload_weight(const tts_backend_iface & be, tts_tensor * t, const float * host, size_t n) {
    if (t->type != TTS_TYPE_F16) return be.set_tensor(be.ctx, t, host) == 0;
    std::vector<uint16_t> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = fp32_to_fp16_host(host[i]);
    return be.set_tensor(be.ctx, t, h.data()) == 0;
}

// f32 values of a weight (F16 weights widened), for the tests' float references
uint64_t kokoro_read_weight(const tts_backend_iface & be, const tts_tensor * t, float * dst, uint64_t cap) {
    const uint64_t n = (uint64_t)tg::nelements(t) * 4;
    if (!dst || cap < n) return n;
    if (t->type == TTS_TYPE_F16) {
        std::vector<uint16_t> h((size_t)tg::nelements(t));
        if (be.get(be.ctx, h.data(), t->data, h.size() * 2) != 0) return 0;
        for (size_t i = 0; i < h.size(); ++i) dst[i] = fp16_to_fp32_host(h[i]);
        return n;
    }
    return be.get(be.ctx, dst, t->data, n) != 0 ? 0 : n;
}
}  // namespace tts

extern "C" tts_kokoro_gen * tts_kokoro_gen_create(const tts_backend_iface * be, const tts_kokoro_gen_config * cfg) {
    const auto & c = *cfg;
    if (c.n_ups < 1 || c.n_ups > 4 || c.n_kernels < 1 || c.n_kernels > 4 || c.n_fft < 2 || c.hop < 1 || c.harmonic_num < 0)
        return nullptr;
    // the sine source always interpolates by 300 (model.cpp:175), so the upsamplers and the iSTFT
    // hop must multiply to 300 for the harmonic branch and the main branch to line up
    if (upsample_total(c) != kUpsample) return nullptr;
    for (int i = 0; i < c.n_ups; ++i)
        if (c.up_kernels[i] < c.up_rates[i] || (c.up_kernels[i] - c.up_rates[i]) % 2) return nullptr;
    auto * k = new tts_kokoro_gen();
    k->cfg = c;
    k->be = *be;
    const int nbins = c.n_fft / 2 + 1;
    int ch = c.in_channels;
    for (int i = 0; i < c.n_ups; ++i) {
        kk_up u;
        const int oc = ch / 2;
        const std::string pre = "gen.ups." + std::to_string(i);
        u.stride = c.up_rates[i];
        u.padding = (c.up_kernels[i] - c.up_rates[i]) / 2;  // Kokoro: (k - u) // 2
        u.w = wnew(k, std::sqrt(3.0f / (float)ch * (float)u.stride / (float)c.up_kernels[i]), 0.f, c.up_kernels[i], oc, ch, pre + ".weight");
        u.b = wnew(k, 0.01f, 0.f, 1, oc, 1, pre + ".bias");
        // noise_convs[i]: stride_f0 = prod(rates[i+1:]), kernel 2*stride_f0 (1 at the last level)
        int sf0 = 1;
        for (int j = i + 1; j < c.n_ups; ++j) sf0 *= c.up_rates[j];
        const int nk = sf0 > 1 ? 2 * sf0 : 1;
        u.nstride = sf0;
        u.npadding = sf0 > 1 ? (sf0 + 1) / 2 : 0;
        const std::string np = "gen.noise_blocks." + std::to_string(i);
        u.nw = conv_w(k, nk, 2 * nbins, oc, np + ".input_conv.weight");
        u.nb = wnew(k, 0.01f, 0.f, 1, oc, 1, np + ".input_conv.bias");
        make_res(k, u.nres, oc, c.noise_res_kernels[i], np + ".res_block");
        k->ups.push_back(u);
        for (int j = 0; j < c.n_kernels; ++j) {
            kk_res r;
            make_res(k, r, oc, c.res_kernels[j], "gen.res_blocks." + std::to_string(i * c.n_kernels + j));
            k->res.push_back(r);
        }
        ch = oc;
    }
    k->m_w = wnew(k, std::sqrt(3.0f / (float)(c.harmonic_num + 1)), 0.f, c.harmonic_num + 1, 1, 1, "gen.m_source_weight");
    k->m_b = wnew(k, 0.01f, 0.f, 1, 0, 0, "gen.m_source_bias");
    k->out_w = conv_w(k, 7, ch, 2 * (c.n_fft / 2 + 1), "gen.conv_post.weight", 0.3f);
    k->out_b = wnew(k, 0.01f, 0.f, 1, 2 * nbins, 1, "gen.conv_post.bias");
    // post_load_assign constants (model.cpp:305-392): the values are set after the synthetic fill
    k->window = wnew(k, 0.f, 0.f, c.n_fft, 0, 0, "stft_window", false);
    k->harm_norm = wnew(k, 0.f, 0.f, 1, c.harmonic_num + 1, 1, "harmonic_sampling_norm", false);
    k->samp_scalar = wnew(k, 0.f, 0.f, 1, 0, 0, "sampling_factor_scalar", false);
    k->nker = wnew(k, 0.f, 0.f, 1, 0, 0, "n_kernels_tensor", false);
    k->one = wnew(k, 0.f, 1.0f, 1, 1, 1, "one", false);
    if (!upload(k)) {
        tts_kokoro_gen_free(k);
        return nullptr;
    }
    // hann_window (util.cpp:132-137): sin(pi * i / n)^2 in double, stored as f32
    k->h_window.resize(c.n_fft);
    for (int i = 0; i < c.n_fft; ++i) k->h_window[i] = (float)std::pow(std::sin(M_PI * (double)i / (double)c.n_fft), 2.0);
    std::vector<float> hn(c.harmonic_num + 1);
    for (int i = 0; i <= c.harmonic_num; ++i) hn[i] = ((float)i + 1.0f) / c.sample_rate;
    const float ss = (float)((float)kUpsample * 2.0f * M_PI);  // upsample_scale * 2.0f * M_PI
    const float nk = (float)c.n_kernels;
    if (k->be.set_tensor(k->be.ctx, k->window, k->h_window.data()) || k->be.set_tensor(k->be.ctx, k->harm_norm, hn.data()) ||
        k->be.set_tensor(k->be.ctx, k->samp_scalar, &ss) || k->be.set_tensor(k->be.ctx, k->nker, &nk)) {
        tts_kokoro_gen_free(k);
        return nullptr;
    }
    // arena: per input frame the last level holds ~a dozen [60, C/4] f32 activations alive plus
    // the 11-tap im2col in f16; the sine source adds a few [300, 9] tensors
    const int64_t U = kUpsample;
    const size_t per_frame = (size_t)(U / c.hop) * (size_t)ch * 4 * 14 + (size_t)(U / c.hop) * 11 * (size_t)ch * 2 * 2 +
                             (size_t)U * (size_t)(c.harmonic_num + 1) * 4 * 16 + (size_t)(U / c.hop / c.up_rates[c.n_ups - 1]) * (size_t)c.in_channels * 4 * 16;
    k->arena_size = c.arena_bytes ? c.arena_bytes : (size_t)c.max_frames * per_frame + ((size_t)64 << 20);
    k->arena = (char *)k->be.alloc(k->be.ctx, k->arena_size);
    if (!k->arena) {
        tts_kokoro_gen_free(k);
        return nullptr;
    }
    return k;
}

extern "C" void tts_kokoro_gen_free(tts_kokoro_gen * k) {
    if (!k) return;
    if (k->arena) k->be.free(k->be.ctx, k->arena);
    if (k->wbuf) k->be.free(k->be.ctx, k->wbuf);
    delete k;
}

extern "C" int64_t tts_kokoro_gen_samples_per_frame(const tts_kokoro_gen * k) { return k ? upsample_total(k->cfg) : 0; }

// snake_1d (util.cpp:98-101): x + sin(alpha*x)^2 * (1/alpha), reciprocal() as DIV of a broadcast 1.0
static tts_tensor * snake(tts_kokoro_gen * k, tg::context & c, tts_tensor * alpha, tts_tensor * x) {
    tts_tensor * one = tg::view_2d(c, k->one, 1, alpha->ne[1], 0, 0);
    tts_tensor * recip = tg::div(c, one, alpha);
    return tg::add(c, x, tg::mul(c, tg::sqr(c, tg::sin(c, tg::mul(c, x, alpha))), recip));
}

// build_kokoro_generator_res_block (model.cpp:136-165); x is [T, C] (time fastest)
static tts_tensor * res_block(tts_kokoro_gen * k, tg::context & c, const kk_res & r, tts_tensor * x, tts_tensor * style) {
    tts_tensor * inpl = x;
    for (int i = 0; i < 3; ++i) {
        tts_tensor * gamma = tg::add(c, tg::mul_mat(c, r.g1w[i], style), r.g1b[i]);
        tts_tensor * beta = tg::add(c, tg::mul_mat(c, r.b1w[i], style), r.b1b[i]);
        tts_tensor * cur = tg::cont(c, tg::transpose(c, tg::norm(c, inpl, 0.00001f)));
        cur = tg::add(c, tg::add(c, cur, tg::mul(c, cur, gamma)), beta);
        cur = snake(k, c, r.a1[i], tg::cont(c, tg::transpose(c, cur)));
        cur = tg::add(c, tg::conv_1d(c, r.c1w[i], cur, 1, r.pad[i], r.dil[i]), r.c1b[i]);
        gamma = tg::add(c, tg::mul_mat(c, r.g2w[i], style), r.g2b[i]);
        beta = tg::add(c, tg::mul_mat(c, r.b2w[i], style), r.b2b[i]);
        cur = tg::cont(c, tg::transpose(c, tg::norm(c, cur, 0.00001f)));
        cur = tg::cont(c, tg::transpose(c, tg::add(c, tg::add(c, cur, tg::mul(c, cur, gamma)), beta)));
        cur = snake(k, c, r.a2[i], cur);
        cur = tg::add(c, tg::conv_1d(c, r.c2w[i], cur, 1, r.pad[0], 1), r.c2b[i]);
        inpl = tg::add(c, inpl, cur);
    }
    return inpl;
}

// build_sin_gen + build_generator (model.cpp:172-244) into `c`: x [C, T] features (channel
// fastest), f0 [T] (or [T, 1]) Hz, style [style_dim].  Registers the uv_noise data and envelope
// inputs on k (filled by kokoro_gen_set_inputs) and returns the PCM node [300 T].
// device_draws: the custom map draws its uniforms from a counter hash on the device (seeded from
// cfg.seed) instead of reading [H][L] host draws -- no host RNG loop and no upload per call.
tts_tensor * tts::kokoro_gen_build(tts_kokoro_gen * k, tg::context & c, tts_tensor * x, tts_tensor * f0, tts_tensor * style, int64_t T,
                                   bool device_draws) {
    const auto & cf = k->cfg;
    const int64_t H = cf.harmonic_num + 1, L = T * kUpsample;
    k->device_draws = device_draws;
    k->in_uvdata = tg::new_tensor_1d(c, TTS_TYPE_F32, device_draws ? 4 : 4 + L * H);
    k->in_wss = tg::new_tensor_1d(c, TTS_TYPE_F32, L);
    tg::set_input(k->in_uvdata);
    tg::set_input(k->in_wss);

    // build_sin_gen (model.cpp:172-193): harmonic phases, x300 linear interpolation, sin, and the
    // uv / noise planes from the custom map over the nearest-x300 F0
    tts_tensor * cur = tg::mul(c, tg::repeat(c, f0, tg::new_tensor_2d(c, TTS_TYPE_F32, T, H)), k->harm_norm);
    cur = tg::mul(c, tg::cumsum(c, tg::mod(c, cur, 1.0f)), k->samp_scalar);
    cur = tg::upscale_linear(c, cur, kUpsample);
    tts_tensor * upscaled = tg::upscale_ext(c, f0, f0->ne[0] * kUpsample, f0->ne[1], f0->ne[2], f0->ne[3]);
    tts_tensor * fake = tg::new_tensor_3d(c, TTS_TYPE_F32, L, H, 2);
    tts_tensor * uv_noise = tg::map_custom3(c, fake, upscaled, k->in_uvdata, TTS_CUSTOM_UV_NOISE);
    if (device_draws) {
        const uint64_t seed = cf.seed ^ 0x5A5Aull;
        uv_noise->op_params[1] = 1;
        uv_noise->op_params[2] = (int32_t)(uint32_t)seed;
        uv_noise->op_params[3] = (int32_t)(uint32_t)(seed >> 32);
    }
    tg::set_name(uv_noise, "uv_noise");
    tts_tensor * noise = tg::cont(c, tg::view_2d(c, uv_noise, uv_noise->ne[0], uv_noise->ne[1], uv_noise->nb[1], uv_noise->nb[2]));
    tts_tensor * uv = tg::cont(c, tg::view_2d(c, uv_noise, uv_noise->ne[0], uv_noise->ne[1], uv_noise->nb[1], 0));
    tts_tensor * sing = tg::cont(c, tg::transpose(c, tg::add(c, tg::mul(c, tg::sin(c, cur), uv), noise)));

    // build_generator (model.cpp:195-244)
    tts_tensor * har = tg::tanh(c, tg::add(c, tg::mul_mat(c, k->m_w, sing), k->m_b));
    // stft(..., one_sided) (util.cpp:111-121): keep the n_fft/2+1 non-negative bins
    har = tg::stft(c, tg::cont(c, tg::transpose(c, har)), k->window, cf.n_fft, cf.hop, true);
    har = tg::cont(c, tg::view_4d(c, har, cf.n_fft / 2 + 1, har->ne[1], har->ne[2], har->ne[3], har->nb[1], har->nb[2], har->nb[3], 0));
    tts_tensor * mhar = tg::cont(c, tg::view_3d(c, har, har->ne[0], har->ne[1], har->ne[2], har->nb[1], har->nb[2], 0));
    tts_tensor * phhar = tg::cont(c, tg::view_3d(c, har, har->ne[0], har->ne[1], har->ne[2], har->nb[1], har->nb[2], har->nb[3]));
    tts_tensor * combined = tg::cont(c, tg::transpose(c, tg::concat(c, mhar, phhar, 0)));
    tg::set_name(sing, "sine_source");
    tg::set_name(combined, "har_spec");

    cur = x;
    for (int i = 0; i < cf.n_ups; ++i) {
        const kk_up & u = k->ups[i];
        cur = tg::leaky_relu(c, cur, 0.1f);
        cur = tg::add(c, tg::conv_transpose_1d(c, u.w, tg::cont(c, tg::transpose(c, cur)), u.stride, u.padding, 1, 0, 1), u.b);
        if (i == cf.n_ups - 1) {
            // front reflection pad by one sample (model.cpp:212-217)
            tts_tensor * tmp = tg::cont(c, tg::view_3d(c, cur, 1, cur->ne[1], cur->ne[2], cur->nb[1], cur->nb[2], cur->nb[0]));
            cur = tg::concat(c, tmp, cur, 0);
        }
        // build_noise_block (model.cpp:167-171)
        tts_tensor * src = tg::add(c, tg::conv_1d(c, u.nw, tg::cont(c, combined), u.nstride, u.npadding, 1), u.nb);
        tg::set_name(cur, "up." + std::to_string(i));
        tg::set_name(src, "noise_conv." + std::to_string(i));
        src = res_block(k, c, u.nres, src, style);
        tg::set_name(src, "noise_res." + std::to_string(i));
        cur = tg::add(c, cur, src);
        tts_tensor * x = cur;
        for (int j = 0; j < cf.n_kernels; ++j) {
            tts_tensor * rb = res_block(k, c, k->res[i * cf.n_kernels + j], x, style);
            cur = j == 0 ? rb : tg::add(c, cur, rb);
        }
        cur = tg::cont(c, tg::transpose(c, tg::div(c, cur, k->nker)));
        tg::set_name(cur, "level." + std::to_string(i));
        tg::build_forward_expand(c, cur);
    }
    cur = tg::leaky_relu(c, cur, 0.01f);
    cur = tg::add(c, tg::conv_1d(c, k->out_w, tg::cont(c, tg::transpose(c, cur)), 1, 3, 1), k->out_b);
    tg::set_name(cur, "conv_post");
    const int nb = cf.n_fft / 2 + 1;
    tts_tensor * spec = tg::view_3d(c, cur, cur->ne[0], nb, cur->ne[2], cur->nb[1], cur->nb[2], 0);
    tts_tensor * phase = tg::view_3d(c, cur, cur->ne[0], cur->ne[1] - nb, cur->ne[2], cur->nb[1], cur->nb[2], cur->nb[1] * nb);
    phase = tg::sin(c, phase);
    spec = tg::exp(c, spec);
    cur = tg::concat(c, spec, phase, 3);
    // istft (util.cpp:123-130): ggml_istft then divide by the squared-window envelope
    cur = tg::istft(c, tg::cont(c, tg::transpose(c, cur)), k->window, cf.n_fft, cf.hop, true);
    cur = tg::div(c, cur, k->in_wss);
    tg::set_name(cur, "after_res_gen");
    return cur;
}

static tts_tensor * build_graph(tts_kokoro_gen * k, int64_t T, bool device_draws) {
    const auto & cf = k->cfg;
    tg::context & c = k->gctx;
    c.reset();
    k->in_x = tg::new_tensor_2d(c, TTS_TYPE_F32, cf.in_channels, T);
    k->in_f0 = tg::new_tensor_1d(c, TTS_TYPE_F32, T);
    k->in_style = tg::new_tensor_1d(c, TTS_TYPE_F32, cf.style_dim);
    for (tts_tensor * t : {k->in_x, k->in_f0, k->in_style}) tg::set_input(t);
    tts_tensor * cur = kokoro_gen_build(k, c, k->in_x, k->in_f0, k->in_style, T, device_draws);
    tg::set_output(cur);
    tg::build_forward_expand(c, cur);
    return cur;
}

// kokoro_runner::set_inputs (model.cpp:1253-1256): the uv_noise custom map's data block -- its
// four constants, then random_uniform_gen's [H][300 T] draws (given by the caller, or drawn on the
// device when the graph was built with device_draws) -- and compute_window_squared_sum
// (util.cpp:203-217); uploads both to the inputs kokoro_gen_build registered.
int tts::kokoro_gen_set_inputs(tts_kokoro_gen * k, int64_t T, const float * rand) {
    const auto & cf = k->cfg;
    const int64_t H = cf.harmonic_num + 1, L = T * kUpsample;
    if (k->device_draws == (rand != nullptr)) return TTS_STATUS_BAD_ARG;  // built for the other mode
    k->h_uvdata.resize((size_t)(rand ? 4 + L * H : 4));
    float * d = k->h_uvdata.data();
    d[0] = cf.voice_threshold, d[1] = cf.noise_std, d[2] = cf.sin_amp, d[3] = cf.sin_amp / 3.0f;
    if (rand) memcpy(d + 4, rand, sizeof(float) * (size_t)(L * H));
    if (k->h_wss_len != L) {  // a function of the length alone: built once per length
        const int64_t n_frames = L / cf.hop, cutoff = n_frames * cf.hop, half = cf.n_fft / 2;
        std::vector<float> w2((size_t)cf.n_fft);
        for (int64_t j = 0; j < cf.n_fft; ++j) w2[(size_t)j] = powf(k->h_window[(size_t)j], 2);  // the same squares, once
        k->h_wss.assign((size_t)L, 0.0f);
        for (int64_t i = 0; i < n_frames + half / cf.hop; ++i) {
            // the same additions in the same order (frame i, then window index j), only the bounds hoisted
            const int64_t j0 = std::max<int64_t>(0, half - i * cf.hop), j1 = std::min<int64_t>(cf.n_fft, cutoff + half - i * cf.hop);
            const int64_t base = i * cf.hop - half;
            for (int64_t j = j0; j < j1; ++j) k->h_wss[(size_t)(base + j)] += w2[(size_t)j];
        }
        k->h_wss_len = L;
    }
    int st = k->be.set(k->be.ctx, k->in_uvdata->data, k->h_uvdata.data(), sizeof(float) * k->h_uvdata.size());
    if (st == 0) st = k->be.set(k->be.ctx, k->in_wss->data, k->h_wss.data(), sizeof(float) * k->h_wss.size());
    return st;
}

extern "C" int tts_kokoro_gen_run(tts_kokoro_gen * k, const float * x, const float * f0, const float * style, const float * rand,
                                  int32_t T, float * pcm) {
    if (!k || !x || !f0 || !style || T <= 0 || T > k->cfg.max_frames) return TTS_STATUS_BAD_ARG;
    tts_tensor * out = build_graph(k, T, rand == nullptr);
    if (!tg::alloc_graph(k->gctx, k->arena, k->arena_size, !k->cfg.debug_no_reuse)) {
        fprintf(stderr, "kokoro: compute arena too small (%zu needed)\n", k->gctx.arena_used);
        return TTS_STATUS_ALLOC_FAILED;
    }
    const auto & cf = k->cfg;
    int st = kokoro_gen_set_inputs(k, T, rand);
    if (st == 0) st = k->be.set(k->be.ctx, k->in_x->data, x, sizeof(float) * (size_t)T * cf.in_channels);
    if (st == 0) st = k->be.set(k->be.ctx, k->in_f0->data, f0, sizeof(float) * (size_t)T);
    if (st == 0) st = k->be.set(k->be.ctx, k->in_style->data, style, sizeof(float) * (size_t)cf.style_dim);
    if (st == 0) st = k->be.compute(k->be.ctx, k->gctx.nodes.data(), (int)k->gctx.nodes.size());
    if (st == 0 && pcm) st = k->be.get(k->be.ctx, pcm, out->data, sizeof(float) * (size_t)tg::nelements(out));
    return st;
}

extern "C" int32_t tts_kokoro_gen_last_graph_nodes(const tts_kokoro_gen * k) { return (int32_t)k->gctx.nodes.size(); }

extern "C" int32_t tts_kokoro_gen_n_weights(const tts_kokoro_gen * k) { return (int32_t)k->specs.size(); }

// Weight i: name, ne[4] and (when dst is non-null and cap suffices) its f32 values; returns bytes.
extern "C" uint64_t tts_kokoro_gen_weight(tts_kokoro_gen * k, int32_t i, char * name, uint64_t name_cap, int64_t * ne, float * dst,
                                          uint64_t cap) {
    if (!k || i < 0 || i >= (int32_t)k->specs.size()) return 0;
    const tts_tensor * t = k->specs[i].t;
    if (name && name_cap) {
        strncpy(name, t->name, name_cap - 1);
        name[name_cap - 1] = 0;
    }
    if (ne)
        for (int d = 0; d < 4; ++d) ne[d] = t->ne[d];
    return kokoro_read_weight(k->be, t, dst, cap);
}

// Debug: copy the named node of the last graph to host (contiguous nodes only); returns bytes.
extern "C" uint64_t tts_kokoro_gen_get_node(tts_kokoro_gen * k, const char * name, void * dst, uint64_t cap) {
    if (!k || !name) return 0;
    for (tts_tensor * t : k->gctx.nodes) {
        if (strcmp(t->name, name) != 0 || !tg::is_contiguous(t)) continue;
        const uint64_t n = tg::nbytes(t);
        if (dst && cap >= n && k->be.get(k->be.ctx, dst, t->data, n) != 0) return 0;
        return n;
    }
    return 0;
}

// Debug: node i of the last graph: op / type / ne; copies its bytes when contiguous (returns size).
extern "C" uint64_t tts_kokoro_gen_node(tts_kokoro_gen * k, int32_t i, int32_t * op, int32_t * type, int64_t * ne, void * dst, uint64_t cap) {
    if (!k || i < 0 || i >= (int32_t)k->gctx.nodes.size()) return 0;
    const tts_tensor * t = k->gctx.nodes[i];
    *op = t->op;
    *type = t->type;
    for (int d = 0; d < 4; ++d) ne[d] = t->ne[d];
    if (!tg::is_contiguous(t) || !dst) return 0;
    const uint64_t n = tg::nbytes(t);
    if (n > cap || k->be.get(k->be.ctx, dst, t->data, n) != 0) return 0;
    return n;
}

// The last graph's node list (valid until the next run), e.g. for tts_hip_plan_stats.
extern "C" tts_tensor * const * tts_kokoro_gen_graph(const tts_kokoro_gen * k, int32_t * n_nodes) {
    if (n_nodes) *n_nodes = k ? (int32_t)k->gctx.nodes.size() : 0;
    return k ? k->gctx.nodes.data() : nullptr;
}
