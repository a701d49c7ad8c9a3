// Minimal ggml-compatible graph builder used by the runners in this package.  It emits exactly
// the node lists TTS.cpp's builders emit (same op, shape, view and permute semantics as ggml:
// ggml_view_*, ggml_permute, ggml_cont_*, ggml_cpy, ggml_build_forward_expand), so the backend
// sees the reference's graphs; with the fork present the same nodes arrive through the ggml
// adapter instead.
#pragma once

#include <deque>
#include <string>
#include <vector>

#include "common.h"

namespace tg {

enum { TG_FLAG_INPUT = 1, TG_FLAG_HOSTDATA = 2, TG_FLAG_OUTPUT = 4, TG_FLAG_PERSIST = 8 };

struct context {
    std::deque<tts_tensor> tensors;  // stable addresses
    std::vector<tts_tensor *> nodes;  // execution order (ggml_cgraph nodes)
    std::vector<tts_tensor *> leafs;
    size_t arena_used = 0;            // bytes of the arena the last alloc used (peak)
    std::vector<tts_tensor *> visited;  // tensors already in nodes/leafs (flag bit on the tensor)

    void reset() {
        for (auto * t : visited) t->pad_ = 0;  // un-mark shared leaves (weights, caches) first
        visited.clear();
        tensors.clear();
        nodes.clear();
        leafs.clear();
        arena_used = 0;
    }
    ~context() { reset(); }
};

tts_tensor * new_tensor(context & c, int type, int n_dims, const int64_t * ne);
tts_tensor * new_tensor_1d(context & c, int type, int64_t ne0);
tts_tensor * new_tensor_2d(context & c, int type, int64_t ne0, int64_t ne1);
tts_tensor * new_tensor_3d(context & c, int type, int64_t ne0, int64_t ne1, int64_t ne2);
tts_tensor * new_tensor_4d(context & c, int type, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
void set_name(tts_tensor * t, const std::string & name);
void set_input(tts_tensor * t);
void set_output(tts_tensor * t);

size_t nbytes(const tts_tensor * t);
int64_t nelements(const tts_tensor * t);
bool is_contiguous(const tts_tensor * t);

tts_tensor * view_1d(context & c, tts_tensor * a, int64_t ne0, size_t offset);
tts_tensor * view_2d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, size_t nb1, size_t offset);
tts_tensor * view_3d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, size_t nb1, size_t nb2, size_t offset);
tts_tensor * view_4d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3, size_t nb1, size_t nb2,
                     size_t nb3, size_t offset);
tts_tensor * reshape_1d(context & c, tts_tensor * a, int64_t ne0);
tts_tensor * reshape_2d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1);
tts_tensor * reshape_3d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2);
tts_tensor * reshape_4d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
tts_tensor * permute(context & c, tts_tensor * a, int ax0, int ax1, int ax2, int ax3);
tts_tensor * transpose(context & c, tts_tensor * a);
tts_tensor * cont(context & c, tts_tensor * a);
tts_tensor * cont_2d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1);
tts_tensor * cont_3d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2);
tts_tensor * cont_4d(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
tts_tensor * cpy(context & c, tts_tensor * a, tts_tensor * b);

tts_tensor * add(context & c, tts_tensor * a, tts_tensor * b);
tts_tensor * sub(context & c, tts_tensor * a, tts_tensor * b);
tts_tensor * mul(context & c, tts_tensor * a, tts_tensor * b);
tts_tensor * div(context & c, tts_tensor * a, tts_tensor * b);
tts_tensor * scale(context & c, tts_tensor * a, float s);
tts_tensor * sqr(context & c, tts_tensor * a);
tts_tensor * sqrt(context & c, tts_tensor * a);
tts_tensor * sin(context & c, tts_tensor * a);
tts_tensor * cos(context & c, tts_tensor * a);
tts_tensor * unary(context & c, tts_tensor * a, int uop);
tts_tensor * gelu(context & c, tts_tensor * a);
tts_tensor * silu(context & c, tts_tensor * a);
tts_tensor * tanh(context & c, tts_tensor * a);
tts_tensor * sigmoid(context & c, tts_tensor * a);
tts_tensor * exp(context & c, tts_tensor * a);
tts_tensor * leaky_relu(context & c, tts_tensor * a, float slope);
tts_tensor * clamp(context & c, tts_tensor * a, float mn, float mx);
tts_tensor * round(context & c, tts_tensor * a);
tts_tensor * mod(context & c, tts_tensor * a, float m);
tts_tensor * norm(context & c, tts_tensor * a, float eps);
tts_tensor * rms_norm(context & c, tts_tensor * a, float eps);
tts_tensor * mul_mat(context & c, tts_tensor * a, tts_tensor * b);
tts_tensor * soft_max_ext(context & c, tts_tensor * a, tts_tensor * mask, float scale, float max_bias);
tts_tensor * im2col(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0, int dst_type);
tts_tensor * conv_1d(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0);
tts_tensor * conv_1d_dw(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0);
tts_tensor * conv_transpose_1d(context & c, tts_tensor * a, tts_tensor * b, int s0, int p0, int d0, int op, int g);
tts_tensor * get_rows(context & c, tts_tensor * a, tts_tensor * idx);
tts_tensor * concat(context & c, tts_tensor * a, tts_tensor * b, int dim);
tts_tensor * sum_rows(context & c, tts_tensor * a);
tts_tensor * cumsum(context & c, tts_tensor * a);
tts_tensor * upscale_ext(context & c, tts_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
tts_tensor * upscale_linear(context & c, tts_tensor * a, int factor);
tts_tensor * stft(context & c, tts_tensor * a, tts_tensor * window, int n_fft, int hop, bool abs_and_angle);
tts_tensor * istft(context & c, tts_tensor * a, tts_tensor * window, int n_fft, int hop, bool abs_and_angle);
tts_tensor * repeat(context & c, tts_tensor * a, tts_tensor * shape);
tts_tensor * map_custom3(context & c, tts_tensor * a, tts_tensor * b, tts_tensor * cc, int fn);
tts_tensor * map_custom2(context & c, tts_tensor * a, tts_tensor * b, int fn);
tts_tensor * rope_ext(context & c, tts_tensor * a, tts_tensor * pos, tts_tensor * freq_factors, int n_dims, int mode,
                      int n_ctx_orig, float freq_base, float freq_scale, float ext_factor, float attn_factor,
                      float beta_fast, float beta_slow);

// ggml_build_forward_expand: DFS post-order over src, appending unvisited op nodes.
void build_forward_expand(context & c, tts_tensor * t);

// ggml-gallocr equivalent: assigns data to every non-view tensor without data from an arena of
// `arena_size` bytes at `arena_base` (device or host pointer; never dereferenced), reusing
// memory after a tensor's last use.  Returns false if the arena is too small.
bool alloc_graph(context & c, char * arena_base, size_t arena_size, bool reuse = true);

// A runner's weight i for tests and tools (tts_*_weight): name, ne, ggml type and its bytes as the
// backend stores them (F32 / F16 as ggml's; quantized types in the backend's layout).  Returns the size.
uint64_t weight_out(const tts_backend_iface & be, const tts_tensor * t, char * name, uint64_t name_cap, int64_t * ne, int32_t * type,
                    void * dst, uint64_t cap);
}  // namespace tg
