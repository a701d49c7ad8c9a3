// Test harness: a tts_backend_iface (include/tts_hip.h) whose every call goes through the ggml
// adapter's vtables (src/ggml_backend/ggml-tts-hip.cpp), the way TTS.cpp reaches a ggml backend:
//   reg -> device -> init_backend / buffer type (src/tts_model.cpp:25-67,134-164)
//   alloc      -> buffer_type.alloc_buffer            (ggml_backend_buft_alloc_buffer, tts_model.cpp:150)
//   set_tensor -> buffer.set_tensor of a whole weight  (ggml_backend_tensor_set, tts_model.cpp:157-164)
//   set        -> buffer.set_tensor of an input        (set_inputs, parler/model.cpp:624-641)
//   compute    -> backend.graph_compute of ggml_tensor nodes (ggml_backend_sched, parler/model.cpp:645)
//   get        -> backend.get_tensor_async, read at once with no synchronize (parler/model.cpp:680-683)
// The runners (tts.cpp_amd/csrc, standing in for TTS.cpp's graph builders) then run unchanged on top
// of the adapter, so tests/test_adapter_gpu.py compares them with the same runners on the direct
// C-ABI.  Each call builds ggml_tensor mirrors of the runner's tts_tensor nodes: ops and unary ops by
// upstream name, custom maps as function pointers registered through get_proc_address.
// Test infrastructure: built by `make adapter-harness`, loaded only by tests/.
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "ggml-backend-impl.h"
#include "ggml-backend.h"
#include "ggml-impl.h"
#include "ggml-tts-hip.h"
#include "ggml.h"
#include "tts_hip.h"

namespace {

// stand-ins for util.cpp's CPU callbacks: only their addresses matter (the adapter maps them to the
// device restatements); never called
void harness_uv_noise(ggml_tensor *, const ggml_tensor *, const ggml_tensor *, const ggml_tensor *, int, int, void *) { GGML_ABORT("called"); }
void harness_cfg_scale(ggml_tensor *, const ggml_tensor *, const ggml_tensor *, int, int, void *) { GGML_ABORT("called"); }

struct Harness {
    ggml_backend_reg_t reg = nullptr;
    ggml_backend_dev_t dev = nullptr;
    ggml_backend_t backend = nullptr;
    ggml_backend_buffer_type_t buft = nullptr;
    std::map<uintptr_t, ggml_backend_buffer_t> bufs;  // base -> buffer
    std::vector<ggml_tensor> store;
    std::unordered_map<const tts_tensor *, ggml_tensor *> done;
    std::vector<ggml_tensor *> nodes;
    std::deque<float> scales;  // cfg_scale userdata (lives as long as the harness)
    bool check_support = true;
    // stats: graph_compute calls, nodes handed over, nodes supports_op refused, whole-tensor weight
    // sets, buffers allocated, input sets, reads, compute failures
    int64_t st[8] = {0};
    std::string last_refused;

    ggml_backend_buffer_t find(const void * p) {
        const uintptr_t a = (uintptr_t)p;
        auto it = bufs.upper_bound(a);
        if (it == bufs.begin()) return nullptr;
        --it;
        ggml_backend_buffer_t b = it->second;
        return a < it->first + b->size ? b : nullptr;
    }
};

int op_to_ggml(int tts_op) {
    const char * n = tts_op_name(tts_op);
    for (int o = 0; o < GGML_OP_COUNT; ++o)
        if (std::strcmp(ggml_op_name((enum ggml_op)o), n) == 0) return o;
    return -1;
}

int unary_to_ggml(int tts_unary) {
    static const char * names[TTS_UNARY_COUNT] = {"ABS", "NEG", "TANH", "RELU", "SIGMOID", "GELU", "SILU", "EXP"};
    if (tts_unary < 0 || tts_unary >= TTS_UNARY_COUNT) return -1;
    for (int u = 0; u < GGML_UNARY_OP_COUNT; ++u)
        if (std::strcmp(ggml_unary_op_name((enum ggml_unary_op)u), names[tts_unary]) == 0) return u;
    return -1;
}

ggml_tensor * to_ggml(Harness & h, const tts_tensor * t) {
    if (!t) return nullptr;
    auto it = h.done.find(t);
    if (it != h.done.end()) return it->second;
    if (h.store.size() == h.store.capacity()) return nullptr;  // sized by the caller: pointers stay valid
    h.store.emplace_back();
    ggml_tensor * g = &h.store.back();
    std::memset(g, 0, sizeof(*g));
    h.done[t] = g;
    g->type = (enum ggml_type)t->type;
    for (int i = 0; i < 4; ++i) g->ne[i] = t->ne[i], g->nb[i] = t->nb[i];
    const int op = op_to_ggml(t->op);
    if (op < 0) return nullptr;
    g->op = (enum ggml_op)op;
    static_assert(sizeof(t->op_params) <= sizeof(g->op_params), "op_params");
    std::memcpy(g->op_params, t->op_params, sizeof(t->op_params));
    if (t->op == TTS_OP_UNARY) g->op_params[0] = unary_to_ggml(t->op_params[0]);
    if (t->op == TTS_OP_MAP_CUSTOM3) {
        ggml_map_custom3_op_params p = {harness_uv_noise, 1, nullptr};
        std::memset(g->op_params, 0, sizeof(g->op_params));
        std::memcpy(g->op_params, &p, sizeof(p));
    }
    if (t->op == TTS_OP_MAP_CUSTOM2) {
        float s;
        std::memcpy(&s, &t->op_params[1], sizeof(float));
        h.scales.push_back(s);
        ggml_map_custom2_op_params p = {harness_cfg_scale, 1, &h.scales.back()};
        std::memset(g->op_params, 0, sizeof(g->op_params));
        std::memcpy(g->op_params, &p, sizeof(p));
    }
    for (int i = 0; i < TTS_MAX_SRC; ++i) {
        if (!t->src[i]) continue;
        g->src[i] = to_ggml(h, t->src[i]);
        if (!g->src[i]) return nullptr;
    }
    if (t->view_src && !(g->view_src = to_ggml(h, t->view_src))) return nullptr;
    g->view_offs = t->view_offs;
    g->data = t->data;
    g->buffer = h.find(t->data);
    if (t->flags & TTS_FLAG_INPUT) g->flags |= GGML_TENSOR_FLAG_INPUT;
    if (t->flags & TTS_FLAG_OUTPUT) g->flags |= GGML_TENSOR_FLAG_OUTPUT;
    std::strncpy(g->name, t->name, GGML_MAX_NAME - 1);
    return g;
}

// a scratch tensor spanning [p, p + n) bytes of a buffer, as ggml_backend_tensor_set(t, data, offset, size) addresses it
ggml_tensor span(ggml_backend_buffer_t b, void * p, size_t n) {
    ggml_tensor t;
    std::memset(&t, 0, sizeof(t));
    t.type = GGML_TYPE_I8;
    t.ne[0] = (int64_t)n, t.ne[1] = t.ne[2] = t.ne[3] = 1;
    t.nb[0] = 1, t.nb[1] = t.nb[2] = t.nb[3] = n;
    t.data = p;
    t.buffer = b;
    return t;
}

// ---- tts_backend_iface over the adapter ----
void * h_alloc(void * ctx, size_t size) {
    auto * h = (Harness *)ctx;
    ggml_backend_buffer_t b = h->buft->iface.alloc_buffer(h->buft, size);
    if (!b) return nullptr;
    void * base = b->iface.get_base(b);
    h->bufs[(uintptr_t)base] = b;
    h->st[4]++;
    return base;
}

void h_free(void * ctx, void * p) {
    auto * h = (Harness *)ctx;
    auto it = h->bufs.find((uintptr_t)p);
    if (it == h->bufs.end()) return;
    ggml_backend_buffer_free(it->second);
    h->bufs.erase(it);
}

int h_set(void * ctx, void * dst, const void * src, size_t size) {
    auto * h = (Harness *)ctx;
    ggml_backend_buffer_t b = h->find(dst);
    if (!b) return TTS_STATUS_BAD_ARG;
    ggml_tensor t = span(b, dst, size);
    b->iface.set_tensor(b, &t, src, 0, size);
    h->st[5]++;
    return 0;
}

int h_set_tensor(void * ctx, tts_tensor * w, const void * src) {
    auto * h = (Harness *)ctx;
    ggml_backend_buffer_t b = h->find(w->data);
    if (!b) return TTS_STATUS_BAD_ARG;
    ggml_tensor g;
    std::memset(&g, 0, sizeof(g));
    g.type = (enum ggml_type)w->type;
    for (int i = 0; i < 4; ++i) g.ne[i] = w->ne[i], g.nb[i] = w->nb[i];
    g.data = w->data;
    g.buffer = b;
    std::strncpy(g.name, w->name, GGML_MAX_NAME - 1);
    b->iface.set_tensor(b, &g, src, 0, ggml_nbytes(&g));  // ggml_backend_tensor_set of the whole tensor
    h->st[3]++;
    return 0;
}

int h_get(void * ctx, void * dst, const void * src, size_t size) {
    auto * h = (Harness *)ctx;
    ggml_backend_buffer_t b = h->find(src);
    if (!b) return TTS_STATUS_BAD_ARG;
    ggml_tensor t = span(b, (void *)src, size);
    h->backend->iface.get_tensor_async(h->backend, &t, dst, 0, size);  // read right away, no synchronize
    h->st[6]++;
    return 0;
}

int h_memset(void * ctx, void * dst, int value, size_t size) {
    auto * h = (Harness *)ctx;
    ggml_backend_buffer_t b = h->find(dst);
    if (!b) return TTS_STATUS_BAD_ARG;
    ggml_tensor t = span(b, dst, size);
    b->iface.memset_tensor(b, &t, (uint8_t)value, 0, size);
    return 0;
}

int h_compute(void * ctx, tts_tensor * const * nodes, int n) {
    auto * h = (Harness *)ctx;
    h->store.clear();
    h->store.reserve((size_t)n * (TTS_MAX_SRC + 2) + 64);
    h->done.clear();
    h->nodes.clear();
    for (int i = 0; i < n; ++i) {
        ggml_tensor * g = to_ggml(*h, nodes[i]);
        if (!g) return TTS_STATUS_FAILED;
        h->nodes.push_back(g);
    }
    // ggml-alloc places the graph's own tensors in a compute buffer: a buffer holding a node that is
    // neither a leaf nor a view is one
    for (ggml_tensor * g : h->nodes)
        if (g->op != GGML_OP_NONE && !g->view_src && g->buffer) g->buffer->usage = GGML_BACKEND_BUFFER_USAGE_COMPUTE;
    if (h->check_support) {
        for (ggml_tensor * g : h->nodes) {
            if (!h->dev->iface.supports_op(h->dev, g)) {
                h->st[2]++;
                h->last_refused = std::string(g->name) + " (" + ggml_op_name(g->op) + ")";
            }
        }
    }
    ggml_cgraph cg{(int)h->nodes.size(), h->nodes.data()};
    const enum ggml_status s = h->backend->iface.graph_compute(h->backend, &cg);
    h->st[0]++;
    h->st[1] += n;
    if (s != GGML_STATUS_SUCCESS) {
        h->st[7]++;
        return TTS_STATUS_FAILED;
    }
    return 0;
}

int h_sync(void * ctx) {
    auto * h = (Harness *)ctx;
    h->backend->iface.synchronize(h->backend);
    return 0;
}

}  // namespace

extern "C" {

void * tts_ggml_harness_create(int device, int check_support) {
    auto * h = new Harness();
    h->check_support = check_support != 0;
    h->reg = ggml_backend_tts_hip_reg();
    if (!h->reg || (size_t)device >= h->reg->iface.get_device_count(h->reg)) {
        delete h;
        return nullptr;
    }
    h->dev = h->reg->iface.get_device(h->reg, (size_t)device);
    ggml_backend_dev_props props;
    h->dev->iface.get_props(h->dev, &props);
    if (props.type != GGML_BACKEND_DEVICE_TYPE_GPU) {
        delete h;
        return nullptr;
    }
    h->backend = h->dev->iface.init_backend(h->dev, nullptr);
    h->buft = h->dev->iface.get_buffer_type(h->dev);
    if (!h->backend || !h->buft || !h->dev->iface.supports_buft(h->dev, h->buft)) {
        delete h;
        return nullptr;
    }
    // the custom-map callbacks, registered through the registry's proc address as a caller would
    auto reg_custom = (void (*)(const void *, int))h->reg->iface.get_proc_address(h->reg, "ggml_backend_tts_hip_register_custom");
    if (!reg_custom) {
        delete h;
        return nullptr;
    }
    reg_custom((const void *)&harness_uv_noise, TTS_CUSTOM_UV_NOISE);
    reg_custom((const void *)&harness_cfg_scale, TTS_CUSTOM_CFG_SCALE);
    return h;
}

void tts_ggml_harness_free(void * p) {
    auto * h = (Harness *)p;
    if (!h) return;
    for (auto & kv : h->bufs) ggml_backend_buffer_free(kv.second);
    if (h->backend) h->backend->iface.free(h->backend);
    delete h;
}

int tts_ggml_harness_iface(void * p, tts_backend_iface * out) {
    std::memset(out, 0, sizeof(*out));
    out->ctx = p;
    out->name = "ggml-adapter(TTS-HIP)";
    out->alloc = h_alloc;
    out->free = h_free;
    out->set = h_set;
    out->set_tensor = h_set_tensor;
    out->get = h_get;
    out->memset = h_memset;
    out->compute = h_compute;
    out->synchronize = h_sync;
    // prepare / launch / set_async / copy / greedy_step / sample_step stay NULL: the runners take
    // TTS.cpp's own loop (graph_compute, logits to the host, host sampler)
    return 0;
}

int tts_ggml_harness_stats(void * p, int64_t * out, int n) {
    auto * h = (Harness *)p;
    for (int i = 0; i < n && i < 8; ++i) out[i] = h->st[i];
    return 0;
}

const char * tts_ggml_harness_last_refused(void * p) { return ((Harness *)p)->last_refused.c_str(); }

const char * tts_ggml_harness_device_name(void * p) {
    auto * h = (Harness *)p;
    return h->dev->iface.get_name(h->dev);
}

// supports_op on a DIV whose divisor is a buffer-less host leaf (util.cpp:86-94's reciprocal():
// ggml_new_tensor_1d + data = a static float, no buffer); the other source is a device tensor
int tts_ggml_harness_hostleaf_supported(void * p) {
    auto * h = (Harness *)p;
    static float one = 1.0f;
    void * dev_mem = h_alloc(h, 256);
    if (!dev_mem) return -1;
    ggml_tensor a, leaf, div;
    for (ggml_tensor * t : {&a, &leaf, &div}) {
        std::memset(t, 0, sizeof(*t));
        t->type = GGML_TYPE_F32;
        t->ne[0] = 1, t->ne[1] = t->ne[2] = t->ne[3] = 1;
        t->nb[0] = 4, t->nb[1] = t->nb[2] = t->nb[3] = 4;
    }
    a.data = dev_mem, a.buffer = h->find(dev_mem);
    leaf.data = &one;  // no buffer
    div.op = GGML_OP_DIV, div.src[0] = &a, div.src[1] = &leaf, div.data = (char *)dev_mem + 64, div.buffer = a.buffer;
    const int with_host_leaf = h->dev->iface.supports_op(h->dev, &div) ? 1 : 0;
    leaf.data = (char *)dev_mem + 128, leaf.buffer = a.buffer;  // the same leaf in device memory
    const int with_dev_leaf = h->dev->iface.supports_op(h->dev, &div) ? 1 : 0;
    h_free(h, dev_mem);
    return with_host_leaf | (with_dev_leaf << 1);
}

}  // extern "C"
