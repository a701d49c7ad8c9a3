#include "graph.h"

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <unordered_map>
#include <unordered_set>

namespace tg {

static void fail(const char * msg) {
    fprintf(stderr, "tg: %s\n", msg);
    abort();
}

static tts_tensor * alloc_meta(context & c) {
    c.tensors.emplace_back();
    tts_tensor * t = &c.tensors.back();
    memset(t, 0, sizeof(*t));
    return t;
}

static void set_strides(tts_tensor * t) {
    t->nb[0] = tts_type_size(t->type);
    t->nb[1] = t->nb[0] * (size_t)(t->ne[0] / tts_blck_size(t->type));
    for (int i = 2; i < 4; ++i) t->nb[i] = t->nb[i - 1] * (size_t)t->ne[i - 1];
}

tts_tensor * new_tensor(context & c, int type, int n_dims, const int64_t * ne) {
    tts_tensor * t = alloc_meta(c);
    t->type = type;
    t->op = TTS_OP_NONE;
    for (int i = 0; i < 4; ++i) t->ne[i] = i < n_dims ? ne[i] : 1;
    set_strides(t);
    return t;
}
tts_tensor * new_tensor_1d(context & c, int type, int64_t ne0) {
    int64_t ne[1] = {ne0};
    return new_tensor(c, type, 1, ne);
}
tts_tensor * new_tensor_2d(context & c, int type, int64_t ne0, int64_t ne1) {
    int64_t ne[2] = {ne0, ne1};
    return new_tensor(c, type, 2, ne);
}
tts_tensor * new_tensor_3d(context & c, int type, int64_t ne0, int64_t ne1, int64_t ne2) {
    int64_t ne[3] = {ne0, ne1, ne2};
    return new_tensor(c, type, 3, ne);
}
tts_tensor * new_tensor_4d(context & c, int type, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    int64_t ne[4] = {ne0, ne1, ne2, ne3};
    return new_tensor(c, type, 4, ne);
}

void set_name(tts_tensor * t, const std::string & name) {
    snprintf(t->name, sizeof(t->name), "%s", name.c_str());
}
void set_input(tts_tensor * t) { t->flags |= TG_FLAG_INPUT; }
void set_output(tts_tensor * t) { t->flags |= TG_FLAG_OUTPUT; }

int64_t nelements(const tts_tensor * t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }

size_t nbytes(const tts_tensor * t) {
    // ggml_nbytes: last byte reachable + 1
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

bool is_contiguous(const tts_tensor * t) {
    return t->nb[0] == tts_type_size(t->type) && t->nb[1] == t->nb[0] * (size_t)(t->ne[0] / tts_blck_size(t->type)) &&
           t->nb[2] == t->nb[1] * (size_t)t->ne[1] && t->nb[3] == t->nb[2] * (size_t)t->ne[2];
}

static tts_tensor * base_of(tts_tensor * a) { return a->view_src ? a->view_src : a; }

static tts_tensor * make_view(context & c, tts_tensor * a, int op, size_t offset) {
    tts_tensor * t = alloc_meta(c);
    t->type = a->type;
    t->op = op;
    t->view_src = base_of(a);
    t->view_offs = (a->view_src ? a->view_offs : 0) + offset;
    t->src[0] = a;
    if (t->view_src->data) t->data = (char *)t->view_src->data + t->view_offs;
    return t;
}

tts_tensor * view_1d(context & c, tts_tensor * a, int64_t ne0, size_t offset) {
    tts_tensor * t = make_view(c, a, TTS_OP_VIEW, offset);
    t->ne[0] = ne0;
    t->ne[1] = t->ne[2] = t->ne[3] = 1;
    set_strides(t);
    return t;
}
tts_tensor * view_2d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, size_t nb1, size_t offset) {
    tts_tensor * t = make_view(c, a, TTS_OP_VIEW, offset);
    t->ne[0] = ne0;
    t->ne[1] = ne1;
    t->ne[2] = t->ne[3] = 1;
    t->nb[0] = tts_type_size(a->type);
    t->nb[1] = nb1;
    t->nb[2] = t->nb[1] * ne1;
    t->nb[3] = t->nb[2];
    return t;
}
tts_tensor * view_3d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, size_t nb1, size_t nb2, size_t offset) {
    tts_tensor * t = make_view(c, a, TTS_OP_VIEW, offset);
    t->ne[0] = ne0;
    t->ne[1] = ne1;
    t->ne[2] = ne2;
    t->ne[3] = 1;
    t->nb[0] = tts_type_size(a->type);
    t->nb[1] = nb1;
    t->nb[2] = nb2;
    t->nb[3] = nb2 * ne2;
    return t;
}
tts_tensor * view_4d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3, size_t nb1, size_t nb2,
                     size_t nb3, size_t offset) {
    tts_tensor * t = make_view(c, a, TTS_OP_VIEW, offset);
    t->ne[0] = ne0;
    t->ne[1] = ne1;
    t->ne[2] = ne2;
    t->ne[3] = ne3;
    t->nb[0] = tts_type_size(a->type);
    t->nb[1] = nb1;
    t->nb[2] = nb2;
    t->nb[3] = nb3;
    return t;
}

static tts_tensor * reshape_n(context & c, tts_tensor * a, int n, const int64_t * ne) {
    if (!is_contiguous(a)) fail("reshape of non-contiguous tensor");
    int64_t tot = 1;
    for (int i = 0; i < n; ++i) tot *= ne[i];
    if (tot != nelements(a)) fail("reshape: element count mismatch");
    tts_tensor * t = make_view(c, a, TTS_OP_RESHAPE, 0);
    for (int i = 0; i < 4; ++i) t->ne[i] = i < n ? ne[i] : 1;
    set_strides(t);
    return t;
}
tts_tensor * reshape_1d(context & c, tts_tensor * a, int64_t ne0) {
    int64_t ne[1] = {ne0};
    return reshape_n(c, a, 1, ne);
}
tts_tensor * reshape_2d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1) {
    int64_t ne[2] = {ne0, ne1};
    return reshape_n(c, a, 2, ne);
}
tts_tensor * reshape_3d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2) {
    int64_t ne[3] = {ne0, ne1, ne2};
    return reshape_n(c, a, 3, ne);
}
tts_tensor * reshape_4d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    int64_t ne[4] = {ne0, ne1, ne2, ne3};
    return reshape_n(c, a, 4, ne);
}

tts_tensor * permute(context & c, tts_tensor * a, int ax0, int ax1, int ax2, int ax3) {
    tts_tensor * t = make_view(c, a, TTS_OP_PERMUTE, 0);
    const int ax[4] = {ax0, ax1, ax2, ax3};
    for (int i = 0; i < 4; ++i) {
        t->ne[ax[i]] = a->ne[i];
        t->nb[ax[i]] = a->nb[i];
    }
    t->op_params[0] = ax0;
    t->op_params[1] = ax1;
    t->op_params[2] = ax2;
    t->op_params[3] = ax3;
    return t;
}

tts_tensor * transpose(context & c, tts_tensor * a) {
    tts_tensor * t = make_view(c, a, TTS_OP_TRANSPOSE, 0);
    t->ne[0] = a->ne[1];
    t->ne[1] = a->ne[0];
    t->nb[0] = a->nb[1];
    t->nb[1] = a->nb[0];
    t->ne[2] = a->ne[2];
    t->ne[3] = a->ne[3];
    t->nb[2] = a->nb[2];
    t->nb[3] = a->nb[3];
    return t;
}

static tts_tensor * new_op(context & c, int op, int type, const int64_t * ne, tts_tensor * a, tts_tensor * b = nullptr) {
    tts_tensor * t = new_tensor(c, type, 4, ne);
    t->op = op;
    t->src[0] = a;
    t->src[1] = b;
    return t;
}

tts_tensor * cont(context & c, tts_tensor * a) { return new_op(c, TTS_OP_CONT, a->type, a->ne, a); }

tts_tensor * cont_2d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1) {
    if (ne0 * ne1 != nelements(a)) fail("cont_2d: element count mismatch");
    int64_t ne[4] = {ne0, ne1, 1, 1};
    return new_op(c, TTS_OP_CONT, a->type, ne, a);
}

tts_tensor * cont_3d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2) {
    if (ne0 * ne1 * ne2 != nelements(a)) fail("cont_3d: element count mismatch");
    int64_t ne[4] = {ne0, ne1, ne2, 1};
    return new_op(c, TTS_OP_CONT, a->type, ne, a);
}

tts_tensor * cont_4d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    if (ne0 * ne1 * ne2 * ne3 != nelements(a)) fail("cont_4d: element count mismatch");
    int64_t ne[4] = {ne0, ne1, ne2, ne3};
    return new_op(c, TTS_OP_CONT, a->type, ne, a);
}

tts_tensor * cpy(context & c, tts_tensor * a, tts_tensor * b) {
    if (nelements(a) != nelements(b)) fail("cpy: element count mismatch");
    tts_tensor * t = make_view(c, b, TTS_OP_CPY, 0);
    for (int i = 0; i < 4; ++i) {
        t->ne[i] = b->ne[i];
        t->nb[i] = b->nb[i];
    }
    t->src[0] = a;
    t->src[1] = b;
    return t;
}

static bool can_repeat(const tts_tensor * small, const tts_tensor * big) {
    for (int i = 0; i < 4; ++i)
        if (small->ne[i] == 0 || big->ne[i] % small->ne[i] != 0) return false;
    return true;
}

static tts_tensor * binary(context & c, int op, tts_tensor * a, tts_tensor * b) {
    if (!can_repeat(b, a)) fail("binary op: src1 cannot be broadcast to src0");
    return new_op(c, op, TTS_TYPE_F32, a->ne, a, b);
}
tts_tensor * add(context & c, tts_tensor * a, tts_tensor * b) { return binary(c, TTS_OP_ADD, a, b); }
tts_tensor * sub(context & c, tts_tensor * a, tts_tensor * b) { return binary(c, TTS_OP_SUB, a, b); }
tts_tensor * mul(context & c, tts_tensor * a, tts_tensor * b) { return binary(c, TTS_OP_MUL, a, b); }
tts_tensor * div(context & c, tts_tensor * a, tts_tensor * b) { return binary(c, TTS_OP_DIV, a, b); }

static void set_f(tts_tensor * t, int i, float v) { memcpy(&t->op_params[i], &v, 4); }

static tts_tensor * map1(context & c, int op, tts_tensor * a) { return new_op(c, op, TTS_TYPE_F32, a->ne, a); }
tts_tensor * scale(context & c, tts_tensor * a, float s) {
    tts_tensor * t = map1(c, TTS_OP_SCALE, a);
    set_f(t, 0, s);
    return t;
}
tts_tensor * sqr(context & c, tts_tensor * a) { return map1(c, TTS_OP_SQR, a); }
tts_tensor * sqrt(context & c, tts_tensor * a) { return map1(c, TTS_OP_SQRT, a); }
tts_tensor * sin(context & c, tts_tensor * a) { return map1(c, TTS_OP_SIN, a); }
tts_tensor * cos(context & c, tts_tensor * a) { return map1(c, TTS_OP_COS, a); }
tts_tensor * unary(context & c, tts_tensor * a, int uop) {
    tts_tensor * t = map1(c, TTS_OP_UNARY, a);
    t->op_params[0] = uop;
    return t;
}
tts_tensor * gelu(context & c, tts_tensor * a) { return unary(c, a, TTS_UNARY_GELU); }
tts_tensor * silu(context & c, tts_tensor * a) { return unary(c, a, TTS_UNARY_SILU); }
tts_tensor * tanh(context & c, tts_tensor * a) { return unary(c, a, TTS_UNARY_TANH); }
tts_tensor * sigmoid(context & c, tts_tensor * a) { return unary(c, a, TTS_UNARY_SIGMOID); }
tts_tensor * exp(context & c, tts_tensor * a) { return unary(c, a, TTS_UNARY_EXP); }
tts_tensor * leaky_relu(context & c, tts_tensor * a, float slope) {
    tts_tensor * t = map1(c, TTS_OP_LEAKY_RELU, a);
    set_f(t, 0, slope);
    return t;
}
tts_tensor * clamp(context & c, tts_tensor * a, float mn, float mx) {
    tts_tensor * t = map1(c, TTS_OP_CLAMP, a);
    set_f(t, 0, mn);
    set_f(t, 1, mx);
    return t;
}
tts_tensor * round(context & c, tts_tensor * a) { return map1(c, TTS_OP_ROUND, a); }
tts_tensor * mod(context & c, tts_tensor * a, float m) {
    tts_tensor * t = map1(c, TTS_OP_MOD, a);
    set_f(t, 0, m);
    return t;
}
tts_tensor * norm(context & c, tts_tensor * a, float eps) {
    tts_tensor * t = map1(c, TTS_OP_NORM, a);
    set_f(t, 0, eps);
    return t;
}
tts_tensor * rms_norm(context & c, tts_tensor * a, float eps) {
    tts_tensor * t = map1(c, TTS_OP_RMS_NORM, a);
    set_f(t, 0, eps);
    return t;
}

tts_tensor * mul_mat(context & c, tts_tensor * a, tts_tensor * b) {
    if (a->ne[0] != b->ne[0]) fail("mul_mat: K mismatch");
    if (b->ne[2] % a->ne[2] != 0 || b->ne[3] % a->ne[3] != 0) fail("mul_mat: batch broadcast mismatch");
    int64_t ne[4] = {a->ne[1], b->ne[1], b->ne[2], b->ne[3]};
    return new_op(c, TTS_OP_MUL_MAT, TTS_TYPE_F32, ne, a, b);
}

// ggml_im2col, 1-D form (is_2D = false): a = kernel [K, IC, OC], b = input [L, IC, N] ->
// [IC*K, OL, N] with element (ic*K + k, ol, n) = b[ol*s0 + k*d0 - p0, ic, n] (0 outside),
// op_params {s0, s1, p0, p1, d0, d1, is_2D} as ggml.
tts_tensor * im2col(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0, int dst_type) {
    const int64_t K = a->ne[0], IC = b->ne[1];
    if (a->ne[1] != IC) fail("im2col: channel mismatch");
    const int64_t OL = (b->ne[0] + 2 * p0 - d0 * (K - 1) - 1) / s0 + 1;
    if (OL <= 0) fail("im2col: empty output");
    int64_t ne[4] = {IC * K, OL, b->ne[2], 1};
    tts_tensor * t = new_op(c, TTS_OP_IM2COL, dst_type, ne, a, b);
    const int32_t prm[7] = {s0, 1, p0, 0, d0, 1, 0};
    for (int i = 0; i < 7; ++i) t->op_params[i] = prm[i];
    return t;
}

// ggml_conv_1d = im2col (F16) -> mul_mat -> reshape: [OL, OC, N]
tts_tensor * conv_1d(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0) {
    tts_tensor * col = im2col(c, a, b, s0, p0, d0, TTS_TYPE_F16);
    tts_tensor * r = mul_mat(c, reshape_2d(c, col, col->ne[0], col->ne[2] * col->ne[1]), reshape_2d(c, a, a->ne[0] * a->ne[1], a->ne[2]));
    return reshape_3d(c, r, col->ne[1], a->ne[2], col->ne[2]);
}

// ggml_conv_1d_dw (depthwise, SNAC's input conv and grouped residual units,
// /root/reference/src/decoder/snac_model.cpp:141, general_neural_audio_codec.cpp:140): kernel
// a [K, 1, C] and input b [L, C] viewed as [K, 1, C, 1] / [L, 1, C, 1], im2col (F16) treats the
// channels as the batch -> [K, OL, C], one mul_mat per channel against its own K taps ->
// [OL, 1, C], reshaped to [L, C] (upstream reshapes with b's length: same-padding convs only).
tts_tensor * conv_1d_dw(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0) {
    tts_tensor * na = reshape_4d(c, a, a->ne[0], 1, a->ne[1], a->ne[2]);
    tts_tensor * nb = reshape_4d(c, b, b->ne[0], 1, b->ne[1], b->ne[2]);
    tts_tensor * col = im2col(c, na, nb, s0, p0, d0, TTS_TYPE_F16);
    tts_tensor * r = mul_mat(c, col, a);
    return reshape_3d(c, r, b->ne[0], b->ne[1], 1);
}

// Fork op ggml_conv_transpose_1d(a, b, s0, p0, d0, output_padding, groups) with PyTorch
// ConvTranspose1d semantics: a = kernel [K, OC/g, IC], b = input [L, IC] ->
// [(L-1)*s0 - 2*p0 + d0*(K-1) + op + 1, OC]; op_params {s0, p0, d0, op, g}.
tts_tensor * conv_transpose_1d(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0, int op, int g) {
    const int64_t K = a->ne[0], IC = b->ne[1];
    if (a->ne[2] != IC || IC % g != 0) fail("conv_transpose_1d: channel mismatch");
    const int64_t OC = a->ne[1] * g;
    const int64_t OL = (b->ne[0] - 1) * s0 - 2 * p0 + d0 * (K - 1) + op + 1;
    if (OL <= 0) fail("conv_transpose_1d: empty output");
    int64_t ne[4] = {OL, OC, 1, 1};
    tts_tensor * t = new_op(c, TTS_OP_CONV_TRANSPOSE_1D, TTS_TYPE_F32, ne, a, b);
    const int32_t prm[5] = {s0, p0, d0, op, g};
    for (int i = 0; i < 5; ++i) t->op_params[i] = prm[i];
    return t;
}

tts_tensor * soft_max_ext(context & c, tts_tensor * a, tts_tensor * mask, float scale_, float max_bias) {
    tts_tensor * t = new_op(c, TTS_OP_SOFT_MAX, TTS_TYPE_F32, a->ne, a, mask);
    set_f(t, 0, scale_);
    set_f(t, 1, max_bias);
    return t;
}

tts_tensor * get_rows(context & c, tts_tensor * a, tts_tensor * idx) {
    // ggml_get_rows: GGML_ASSERT(a->ne[2] == b->ne[1]) -- idx batch dims index a's dims 2/3
    if (a->ne[2] != idx->ne[1] || idx->type != TTS_TYPE_I32) fail("get_rows: a->ne[2] must equal idx->ne[1]");
    int64_t ne[4] = {a->ne[0], idx->ne[0], idx->ne[1], idx->ne[2]};
    return new_op(c, TTS_OP_GET_ROWS, TTS_TYPE_F32, ne, a, idx);
}

tts_tensor * concat(context & c, tts_tensor * a, tts_tensor * b, int dim) {
    int64_t ne[4];
    for (int i = 0; i < 4; ++i) {
        if (i != dim && a->ne[i] != b->ne[i]) fail("concat: shape mismatch");
        ne[i] = a->ne[i] + (i == dim ? b->ne[i] : 0);
    }
    tts_tensor * t = new_op(c, TTS_OP_CONCAT, a->type, ne, a, b);
    t->op_params[0] = dim;
    return t;
}

// ---- fork audio ops (Kokoro sine source / iSTFTNet head), PyTorch semantics (oracle/ggml_ref.c) ----
tts_tensor * cumsum(context & c, tts_tensor * a) { return new_op(c, TTS_OP_CUMSUM, TTS_TYPE_F32, a->ne, a); }

// ggml_upscale_ext (nearest, upstream) to the given shape
tts_tensor * upscale_ext(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    int64_t ne[4] = {ne0, ne1, ne2, ne3};
    tts_tensor * t = new_op(c, TTS_OP_UPSCALE, TTS_TYPE_F32, ne, a);
    t->op_params[0] = 0;
    return t;
}

// fork ggml_upscale_linear(a, factor): linear interpolation (align_corners = false) along ne0
tts_tensor * upscale_linear(context & c, tts_tensor * a, int factor) {
    int64_t ne[4] = {a->ne[0] * factor, a->ne[1], a->ne[2], a->ne[3]};
    tts_tensor * t = new_op(c, TTS_OP_UPSCALE, TTS_TYPE_F32, ne, a);
    t->op_params[0] = 1;
    return t;
}

// fork ggml_stft(a = [L, B], window [n_fft]) -> [n_fft, L/hop + 1, B, 2] (centre, reflect)
tts_tensor * stft(context & c, tts_tensor * a, tts_tensor * window, int n_fft, int hop, bool abs_and_angle) {
    int64_t ne[4] = {n_fft, (a->ne[0] + 2 * (n_fft / 2) - n_fft) / hop + 1, a->ne[1], 2};
    tts_tensor * t = new_op(c, TTS_OP_STFT, TTS_TYPE_F32, ne, a, window);
    t->op_params[0] = n_fft, t->op_params[1] = hop, t->op_params[2] = abs_and_angle ? 1 : 0;
    return t;
}

// fork ggml_istft(a = [n_fft/2+1, F, B, 2], window) -> [(F-1)*hop, B] (no envelope division)
tts_tensor * istft(context & c, tts_tensor * a, tts_tensor * window, int n_fft, int hop, bool abs_and_angle) {
    int64_t ne[4] = {(a->ne[1] - 1) * hop, a->ne[2], 1, 1};
    tts_tensor * t = new_op(c, TTS_OP_ISTFT, TTS_TYPE_F32, ne, a, window);
    t->op_params[0] = n_fft, t->op_params[1] = hop, t->op_params[2] = abs_and_angle ? 1 : 0;
    return t;
}

// ggml_map_custom3(a, b, c, fn): dst has a's shape; fn is one of tts_custom_op (the reference's
// CPU callback, restated on the device by the backend)
tts_tensor * map_custom3(context & c, tts_tensor * a, tts_tensor * b, tts_tensor * cc, int fn) {
    tts_tensor * t = new_op(c, TTS_OP_MAP_CUSTOM3, TTS_TYPE_F32, a->ne, a, b);
    t->src[2] = cc;
    t->op_params[0] = fn;
    return t;
}

// ggml_map_custom2(a, b, fn): dst has a's shape (tts_custom_op fn, restated on the device)
tts_tensor * map_custom2(context & c, tts_tensor * a, tts_tensor * b, int fn) {
    tts_tensor * t = new_op(c, TTS_OP_MAP_CUSTOM2, TTS_TYPE_F32, a->ne, a, b);
    t->op_params[0] = fn;
    return t;
}

tts_tensor * sum_rows(context & c, tts_tensor * a) {
    int64_t ne[4] = {1, a->ne[1], a->ne[2], a->ne[3]};
    return new_op(c, TTS_OP_SUM_ROWS, TTS_TYPE_F32, ne, a);
}

tts_tensor * repeat(context & c, tts_tensor * a, tts_tensor * shape) {
    if (!can_repeat(a, shape)) fail("repeat: shape mismatch");
    return new_op(c, TTS_OP_REPEAT, a->type, shape->ne, a);
}

tts_tensor * rope_ext(context & c, tts_tensor * a, tts_tensor * pos, tts_tensor * ff, int n_dims, int mode, int n_ctx_orig,
                      float freq_base, float freq_scale, float ext_factor, float attn_factor, float beta_fast,
                      float beta_slow) {
    tts_tensor * t = new_op(c, TTS_OP_ROPE, TTS_TYPE_F32, a->ne, a, pos);
    t->src[2] = ff;
    t->op_params[1] = n_dims;
    t->op_params[2] = mode;
    t->op_params[4] = n_ctx_orig;
    set_f(t, 5, freq_base);
    set_f(t, 6, freq_scale);
    set_f(t, 7, ext_factor);
    set_f(t, 8, attn_factor);
    set_f(t, 9, beta_fast);
    set_f(t, 10, beta_slow);
    return t;
}

// ---- ggml_build_forward_expand ----
// Visited marks live in the tensors' pad_ field (cleared by the builder that owns them), so an
// expand is O(new nodes) like ggml's hash set, not O(graph).
static constexpr int32_t kVisited = 0x5A5A;

static void visit(context & c, tts_tensor * t) {
    if (!t || t->pad_ == kVisited) return;
    t->pad_ = kVisited;
    c.visited.push_back(t);
    for (int i = 0; i < TTS_MAX_SRC; ++i) visit(c, t->src[i]);
    if (t->op == TTS_OP_NONE) c.leafs.push_back(t);
    else c.nodes.push_back(t);
}

void build_forward_expand(context & c, tts_tensor * t) { visit(c, t); }

// ---- allocator: first-fit free list with coalescing, freed after last use ----
namespace {
struct FreeList {
    std::map<size_t, size_t> blocks;  // offset -> size
    size_t top = 0, peak = 0, cap = 0;
    static size_t al(size_t n) { return (n + 255) & ~(size_t)255; }
    bool alloc(size_t n, size_t & off) {
        n = al(n);
        for (auto it = blocks.begin(); it != blocks.end(); ++it) {
            if (it->second >= n) {
                off = it->first;
                size_t rem = it->second - n;
                size_t noff = it->first + n;
                blocks.erase(it);
                if (rem) blocks[noff] = rem;
                return true;
            }
        }
        off = top;
        top += n;
        peak = std::max(peak, top);
        return top <= cap;
    }
    void release(size_t off, size_t n) {
        n = al(n);
        auto it = blocks.emplace(off, n).first;
        auto nx = std::next(it);
        if (nx != blocks.end() && it->first + it->second == nx->first) {
            it->second += nx->second;
            blocks.erase(nx);
        }
        if (it != blocks.begin()) {
            auto pv = std::prev(it);
            if (pv->first + pv->second == it->first) {
                pv->second += it->second;
                blocks.erase(it);
                it = pv;
            }
        }
        if (it->first + it->second == top) {
            top = it->first;
            blocks.erase(it);
        }
    }
};
}  // namespace

// Per-tensor slots for the allocator: open addressing on the tensor address (a 20k-node graph
// would otherwise spend most of its allocation time in std::unordered_map node allocations).
namespace {
struct TensorSlots {
    std::vector<tts_tensor *> keys;
    std::vector<int> last_use;
    std::vector<int64_t> off;  // -1: not (or no longer) allocated by this pass
    size_t mask = 0;
    explicit TensorSlots(size_t n) {
        size_t cap = 64;
        while (cap < 2 * n) cap <<= 1;
        keys.assign(cap, nullptr);
        last_use.assign(cap, -1);
        off.assign(cap, -1);
        mask = cap - 1;
    }
    size_t at(tts_tensor * t) {  // insert if absent
        size_t i = (size_t)(((uint64_t)(uintptr_t)t * 0x9E3779B97F4A7C15ull) >> 32) & mask;
        while (keys[i] && keys[i] != t) i = (i + 1) & mask;
        keys[i] = t;
        return i;
    }
};
}  // namespace

bool alloc_graph(context & c, char * arena_base, size_t arena_size, bool reuse) {
    FreeList fl;
    fl.cap = arena_size;
    const int n = (int)c.nodes.size();
    TensorSlots ts((size_t)n + c.leafs.size() + 16);
    auto needs_alloc = [](tts_tensor * t) { return t && !t->data && !t->view_src; };
    for (int i = 0; i < n; ++i) {
        tts_tensor * t = c.nodes[i];
        for (int s = 0; s < TTS_MAX_SRC; ++s) {
            tts_tensor * x = t->src[s];
            if (!x) continue;
            tts_tensor * b = x->view_src ? x->view_src : x;
            ts.last_use[ts.at(b)] = i;
        }
        if (t->view_src) {
            int & lu = ts.last_use[ts.at(t->view_src)];
            lu = std::max(lu, i);
        }
    }
    bool ok = true;
    // inputs (leafs without data) live for the whole graph
    for (auto * l : c.leafs) {
        if (needs_alloc(l)) {
            size_t off;
            ok &= fl.alloc(nbytes(l), off);
            ts.off[ts.at(l)] = (int64_t)off;
            l->data = arena_base + off;
        }
    }
    for (int i = 0; i < n; ++i) {
        tts_tensor * t = c.nodes[i];
        if (needs_alloc(t)) {
            size_t off;
            ok &= fl.alloc(nbytes(t), off);
            ts.off[ts.at(t)] = (int64_t)off;
            t->data = arena_base + off;
        } else if (t->view_src && !t->data) {
            if (!t->view_src->data) {
                // view of a node allocated earlier in this pass
                fail("view of unallocated tensor");
            }
            t->data = (char *)t->view_src->data + t->view_offs;
        }
        // release tensors whose last use is this node (never outputs or inputs)
        for (int s = 0; s < TTS_MAX_SRC; ++s) {
            tts_tensor * x = t->src[s];
            if (!x) continue;
            tts_tensor * b = x->view_src ? x->view_src : x;
            const size_t k = ts.at(b);
            if (ts.off[k] < 0) continue;
            if (reuse && ts.last_use[k] == i && !(b->flags & (TG_FLAG_OUTPUT | TG_FLAG_INPUT)) && b->op != TTS_OP_NONE) {
                fl.release((size_t)ts.off[k], nbytes(b));
                ts.off[k] = -1;
            }
        }
    }
    c.arena_used = fl.peak;
    return ok;
}

uint64_t weight_out(const tts_backend_iface & be, const tts_tensor * t, char * name, uint64_t name_cap, int64_t * ne, int32_t * type,
                    void * dst, uint64_t cap) {
    if (name && name_cap) {
        strncpy(name, t->name, name_cap - 1);
        name[name_cap - 1] = 0;
    }
    if (ne)
        for (int k = 0; k < 4; ++k) ne[k] = t->ne[k];
    if (type) *type = t->type;
    const uint64_t n = nbytes(t);
    if (dst && cap >= n && be.get(be.ctx, dst, t->data, n) != 0) return 0;
    return n;
}

}  // namespace tg
