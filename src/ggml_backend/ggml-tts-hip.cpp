// ggml backend adapter: the ggml_backend_reg / device / buffer-type / buffer / backend vtables of
// the ggml fork TTS.cpp builds against (/root/reference/.gitmodules:1-4, an absent submodule), each
// slot forwarded to the C-ABI of libtts_hip.so (include/tts_hip.h).  SURVEY §8(b) lists the
// interface; INTEGRATION.md says where TTS.cpp calls it.
//
// Compiled only inside the fork: `make ggml-adapter TTS_GGML_DIR=<fork checkout>` (this repo has no
// ggml sources; tests/test_adapter_cpu.py compiles this file against a declaration-only stand-in of
// the few upstream ggml declarations it uses, as a syntax / ABI-usage check, never as ggml).
//
// What it does beyond forwarding:
//  * weights: a whole-tensor set_tensor of a Q4_K tensor goes to tts_hip_weight_set (the backend's
//    lane / tile layouts) whatever the buffer's usage -- TTS.cpp never calls
//    ggml_backend_buffer_set_usage (tts_model::set_tensor, src/tts_model.cpp:157-164); the layout
//    flags it returns are kept per buffer and put on every mirror of that tensor.  get_tensor of
//    such a tensor returns ggml's native bytes (tts_hip_weight_get);
//  * graph_compute mirrors the split's nodes into tts_tensor (same ne / nb / op_params / data /
//    view_src; ops and unary ops matched by name) in ggml's node order, so the backend's planner
//    sees exactly what ggml_backend_sched hands over;
//  * hazards of the unchanged callers: (1) get_tensor_async synchronises (no caller
//    ever calls ggml_backend_synchronize); (3) a buffer-less host-data leaf (util.cpp:86-94) makes
//    supports_op false; (4) set_tensor accepts another backend's device pointer as its source
//    (Parler's cross K/V copied out of a device-resident prep graph);
//    (5) map_custom2/3 are supported only for the two callbacks with device restatements.
//    (2), the host read of Kokoro's window->data, cannot be fixed behind the API (the pointer is a
//    device address): INTEGRATION.md §3 gives the caller-side edit.
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "ggml-backend-impl.h"
#include "ggml-backend.h"
#include "ggml-impl.h"
#include "ggml-tts-hip.h"
#include "ggml.h"
#include "tts_hip.h"

// the CPU callbacks of src/util.cpp, resolved if the final link has them (weak: absent = null)
extern void uv_noise_compute(struct ggml_tensor *, const struct ggml_tensor *, const struct ggml_tensor *, const struct ggml_tensor *, int, int,
                             void *) __attribute__((weak));
extern void cfg_scale(struct ggml_tensor *, const struct ggml_tensor *, const struct ggml_tensor *, int, int, void *) __attribute__((weak));

namespace {

// ---------------------------------------------------------------------------------------------
// op / unary mapping by name (tts_op / tts_unary_op do not share ggml's numbering)
int map_op(enum ggml_op op) {
    static std::vector<int> table = [] {
        std::vector<int> t(GGML_OP_COUNT, -1);
        for (int o = 0; o < GGML_OP_COUNT; ++o) {
            const char * gn = ggml_op_name((enum ggml_op)o);
            for (int k = 0; k < TTS_OP_COUNT; ++k)
                if (gn && std::strcmp(gn, tts_op_name(k)) == 0) t[o] = k;
        }
        return t;
    }();
    return (int)op >= 0 && (int)op < GGML_OP_COUNT ? table[op] : -1;
}

int map_unary(int ggml_unary) {
    static const char * names[TTS_UNARY_COUNT] = {"ABS", "NEG", "TANH", "RELU", "SIGMOID", "GELU", "SILU", "EXP"};
    const char * gn = ggml_unary_op_name((enum ggml_unary_op)ggml_unary);
    for (int k = 0; k < TTS_UNARY_COUNT; ++k)
        if (gn && std::strcmp(gn, names[k]) == 0) return k;
    return -1;
}

std::mutex g_custom_mu;
std::unordered_map<const void *, int> g_custom;  // registered callbacks -> tts_custom_op

int custom_kind(const void * fn) {
    if (!fn) return TTS_CUSTOM_NONE;
    if ((const void *)&uv_noise_compute != nullptr && fn == (const void *)&uv_noise_compute) return TTS_CUSTOM_UV_NOISE;
    if ((const void *)&cfg_scale != nullptr && fn == (const void *)&cfg_scale) return TTS_CUSTOM_CFG_SCALE;
    std::lock_guard<std::mutex> lk(g_custom_mu);
    auto it = g_custom.find(fn);
    return it == g_custom.end() ? TTS_CUSTOM_NONE : it->second;
}

// ---------------------------------------------------------------------------------------------
// devices
struct DevCtx {
    int device;
    std::string name, desc;
    tts_hip_backend_t util = nullptr;  // allocations made through the buffer type (no backend yet)
    ggml_backend_buffer_type buft;
    std::mutex mu;
    tts_hip_backend_t utility() {
        std::lock_guard<std::mutex> lk(mu);
        if (!util) util = tts_hip_backend_init(device);
        return util;
    }
};

struct RegCtx {
    std::vector<ggml_backend_device> devs;
    std::vector<DevCtx *> ctx;
};

const char * kBuftName = "TTS-HIP";

// ---------------------------------------------------------------------------------------------
// buffers: device memory from tts_hip_buffer_alloc; the layout flags tts_hip_weight_set chose for
// each weight, keyed by its data address
struct BufCtx {
    tts_hip_backend_t be;
    void * base;
    size_t size;
    std::mutex mu;
    std::unordered_map<const void *, int32_t> layout;  // data -> TTS_FLAG_REPACKED / TILED / TILED_COPY
    int32_t flags_of(const void * p) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = layout.find(p);
        return it == layout.end() ? 0 : it->second;
    }
};

tts_tensor weight_view(const ggml_tensor * t) {
    tts_tensor w;
    std::memset(&w, 0, sizeof(w));
    w.type = (int32_t)t->type;
    for (int i = 0; i < 4; ++i) w.ne[i] = t->ne[i], w.nb[i] = t->nb[i];
    w.data = t->data;
    return w;
}

void buf_free(ggml_backend_buffer_t b) {
    auto * c = (BufCtx *)b->context;
    tts_hip_buffer_free(c->be, c->base);
    delete c;
}
void * buf_base(ggml_backend_buffer_t b) { return ((BufCtx *)b->context)->base; }

void buf_memset(ggml_backend_buffer_t b, ggml_tensor * t, uint8_t value, size_t offset, size_t size) {
    auto * c = (BufCtx *)b->context;
    tts_hip_memset(c->be, (char *)t->data + offset, value, size);
    tts_hip_synchronize(c->be);
}

void buf_set(ggml_backend_buffer_t b, ggml_tensor * t, const void * data, size_t offset, size_t size) {
    auto * c = (BufCtx *)b->context;
    if (tts_hip_is_device_pointer(data)) {  // another backend's device tensor as the source (hazard 4)
        tts_hip_tensor_copy(c->be, (char *)t->data + offset, data, size);
        tts_hip_synchronize(c->be);
        return;
    }
    // a whole Q4_K tensor is a weight (nothing else in TTS.cpp is Q4_K): the backend's own layouts
    if (t->type == GGML_TYPE_Q4_K && offset == 0 && size == ggml_nbytes(t) && !t->view_src) {
        tts_tensor w = weight_view(t);
        const int st = tts_hip_weight_set(c->be, &w, data);
        std::lock_guard<std::mutex> lk(c->mu);
        if (st == 0) {
            c->layout[t->data] = w.flags & (TTS_FLAG_REPACKED | TTS_FLAG_TILED | TTS_FLAG_TILED_COPY);
            return;
        }
        // no backend layout (e.g. the tiled copy could not be allocated): the native bytes, no flags,
        // so the weight is never left as uninitialised device memory (set_tensor cannot report failure)
        c->layout.erase(t->data);
        if (tts_hip_tensor_set(c->be, t->data, data, size) != 0) GGML_ABORT("tts-hip: set_tensor of the weight %s failed", t->name);
        return;
    }
    if (c->flags_of(t->data) && !(offset == 0 && size == ggml_nbytes(t))) {
        // a partial write into a weight stored in a backend layout would mix layouts: refuse loudly
        GGML_ABORT("tts-hip: partial set_tensor on the repacked weight %s", t->name);
    }
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->layout.erase(t->data);
    }
    tts_hip_tensor_set(c->be, (char *)t->data + offset, data, size);
}

void buf_get(ggml_backend_buffer_t b, const ggml_tensor * t, void * data, size_t offset, size_t size) {
    auto * c = (BufCtx *)b->context;
    const int32_t f = c->flags_of(t->data);
    if (f && offset == 0 && size == ggml_nbytes(t)) {
        tts_tensor w = weight_view(t);
        w.flags = f;
        tts_hip_weight_get(c->be, &w, data);  // ggml's native bytes
        return;
    }
    if (f) GGML_ABORT("tts-hip: partial get_tensor on the repacked weight %s", t->name);
    tts_hip_tensor_get(c->be, data, (const char *)t->data + offset, size);
}

bool buf_cpy(ggml_backend_buffer_t b, const ggml_tensor * src, ggml_tensor * dst) {
    if (!src->buffer || src->buffer->buft->iface.get_name != b->buft->iface.get_name) return false;
    auto * c = (BufCtx *)b->context;  // the destination's buffer
    // each tensor's layout flags live in its own buffer's map (the source may be another TTS-HIP
    // buffer); a weight in a backend layout goes through the host (ggml's get + set fallback)
    const int32_t fs = ((BufCtx *)src->buffer->context)->flags_of(src->data);
    if (fs || c->flags_of(dst->data)) return false;
    tts_hip_tensor_copy(c->be, dst->data, src->data, ggml_nbytes(src));
    tts_hip_synchronize(c->be);
    return true;
}

void buf_clear(ggml_backend_buffer_t b, uint8_t value) {
    auto * c = (BufCtx *)b->context;
    tts_hip_memset(c->be, c->base, value, c->size);
    tts_hip_synchronize(c->be);
}

const char * buft_name(ggml_backend_buffer_type_t) { return kBuftName; }

ggml_backend_buffer_t buft_alloc(ggml_backend_buffer_type_t buft, size_t size) {
    auto * d = (DevCtx *)buft->context;
    tts_hip_backend_t be = d->utility();
    if (!be) return nullptr;
    void * p = tts_hip_buffer_alloc(be, size);
    if (!p) return nullptr;
    auto * c = new BufCtx();
    c->be = be;
    c->base = p;
    c->size = size;
    ggml_backend_buffer_i iface;
    std::memset(&iface, 0, sizeof(iface));
    iface.free_buffer = buf_free;
    iface.get_base = buf_base;
    iface.memset_tensor = buf_memset;
    iface.set_tensor = buf_set;
    iface.get_tensor = buf_get;
    iface.cpy_tensor = buf_cpy;
    iface.clear = buf_clear;
    return ggml_backend_buffer_init(buft, iface, c, size);
}

size_t buft_align(ggml_backend_buffer_type_t) { return tts_hip_buffer_alignment(); }
size_t buft_max(ggml_backend_buffer_type_t) { return SIZE_MAX; }
// both Q4_K layouts hold exactly ggml_nbytes bytes: no padding
size_t buft_alloc_size(ggml_backend_buffer_type_t, const ggml_tensor * t) { return ggml_nbytes(t); }
bool buft_is_host(ggml_backend_buffer_type_t) { return false; }

bool is_ours(ggml_backend_buffer_type_t buft) { return buft && buft->iface.get_name == buft_name; }

// ---------------------------------------------------------------------------------------------
// node mirrors
struct Mirror {
    std::vector<tts_tensor> store;  // reserved up front: pointers stay valid
    std::vector<tts_tensor *> nodes;
    std::unordered_map<const ggml_tensor *, tts_tensor *> done;
    void reset(size_t n) {
        store.clear();
        store.reserve(n);
        nodes.clear();
        done.clear();
    }
};

bool mirror_ok(const Mirror & m) { return m.store.size() < m.store.capacity(); }

// depth < 0: the whole ancestry (graph_compute); otherwise sources this many levels down (supports_op)
tts_tensor * mirror(Mirror & m, const ggml_tensor * g, int depth = -1) {
    if (!g) return nullptr;
    auto it = m.done.find(g);
    if (it != m.done.end()) return it->second;
    if (!mirror_ok(m)) return nullptr;  // caller sized the store; never reallocate
    m.store.emplace_back();
    tts_tensor * t = &m.store.back();
    std::memset(t, 0, sizeof(*t));
    m.done[g] = t;
    t->type = (int32_t)g->type;
    t->op = map_op(g->op);
    for (int i = 0; i < 4; ++i) t->ne[i] = g->ne[i], t->nb[i] = g->nb[i];
    static_assert(sizeof(t->op_params) <= sizeof(g->op_params), "op_params");
    std::memcpy(t->op_params, g->op_params, sizeof(t->op_params));
    if (g->op == GGML_OP_UNARY) {
        t->op_params[0] = map_unary(ggml_get_op_params_i32(g, 0));
        if (t->op_params[0] < 0) t->op = -1;
    }
    if (g->op == GGML_OP_MAP_CUSTOM3 || g->op == GGML_OP_MAP_CUSTOM2) {
        int kind;
        float scale = 0.0f;
        if (g->op == GGML_OP_MAP_CUSTOM3) {
            const auto * p = (const struct ggml_map_custom3_op_params *)g->op_params;
            kind = custom_kind((const void *)p->fun);
            if (kind != TTS_CUSTOM_UV_NOISE) kind = TTS_CUSTOM_NONE;
        } else {
            const auto * p = (const struct ggml_map_custom2_op_params *)g->op_params;
            kind = custom_kind((const void *)p->fun);
            if (kind != TTS_CUSTOM_CFG_SCALE) kind = TTS_CUSTOM_NONE;
            else if (p->userdata) std::memcpy(&scale, p->userdata, sizeof(float));  // cfg_scale's userdata[0]
        }
        std::memset(t->op_params, 0, sizeof(t->op_params));
        t->op_params[0] = kind;
        std::memcpy(&t->op_params[1], &scale, sizeof(float));
        if (kind == TTS_CUSTOM_NONE) t->op = -1;
    }
    if (depth != 0) {
        for (int i = 0; i < TTS_MAX_SRC && i < GGML_MAX_SRC; ++i) t->src[i] = mirror(m, g->src[i], depth - 1);
        t->view_src = mirror(m, g->view_src, depth - 1);
    }
    t->view_offs = g->view_offs;
    t->data = g->data;
    int32_t f = 0;
    if (g->flags & GGML_TENSOR_FLAG_INPUT) f |= TTS_FLAG_INPUT;
    if (g->flags & GGML_TENSOR_FLAG_OUTPUT) f |= TTS_FLAG_OUTPUT;
    const ggml_tensor * base = g->view_src ? g->view_src : g;
    if (!base->buffer && base->data) f |= TTS_FLAG_HOSTDATA;  // util.cpp:86-94's static leaf
    if (base->buffer && ggml_backend_buffer_get_usage(base->buffer) != GGML_BACKEND_BUFFER_USAGE_COMPUTE) f |= TTS_FLAG_PERSIST;
    if (g->buffer && is_ours(g->buffer->buft) && !g->view_src) f |= ((BufCtx *)g->buffer->context)->flags_of(g->data);
    t->flags = f;
    std::strncpy(t->name, g->name, TTS_MAX_NAME - 1);
    return t;
}

// every source of an op this backend is asked to run must live in device memory of this device
bool srcs_on_device(const ggml_tensor * op, ggml_backend_dev_t dev) {
    for (int i = 0; i < GGML_MAX_SRC; ++i) {
        const ggml_tensor * s = op->src[i];
        if (!s) continue;
        const ggml_tensor * b = s->view_src ? s->view_src : s;
        if (!b->buffer && b->data) return false;  // hazard 3: host data without a buffer
        if (b->buffer && !ggml_backend_buffer_is_host(b->buffer) && !is_ours(b->buffer->buft)) return false;
        if (b->buffer && is_ours(b->buffer->buft) && b->buffer->buft->device != dev) return false;
    }
    return true;
}

// ---------------------------------------------------------------------------------------------
// backend
struct BackendCtx {
    int device;
    tts_hip_backend_t be;
    Mirror m;
};

const char * be_name(ggml_backend_t b) { return tts_hip_backend_name(((BackendCtx *)b->context)->be); }
void be_free(ggml_backend_t b) {
    auto * c = (BackendCtx *)b->context;
    tts_hip_backend_free(c->be);
    delete c;
    delete b;
}
void be_set_async(ggml_backend_t b, ggml_tensor * t, const void * data, size_t offset, size_t size) {
    auto * c = (BackendCtx *)b->context;
    if (t->buffer && is_ours(t->buffer->buft) && ((BufCtx *)t->buffer->context)->flags_of(t->data))
        GGML_ABORT("tts-hip: async write into the repacked weight %s", t->name);
    tts_hip_tensor_set_async(c->be, (char *)t->data + offset, data, size);
}
// hazard 1: callers read the host copy right after get_tensor_async, with no synchronize
void be_get_async(ggml_backend_t b, const ggml_tensor * t, void * data, size_t offset, size_t size) {
    auto * c = (BackendCtx *)b->context;
    if (t->buffer && is_ours(t->buffer->buft) && ((BufCtx *)t->buffer->context)->flags_of(t->data)) {
        buf_get(t->buffer, t, data, offset, size);
        return;
    }
    tts_hip_tensor_get(c->be, data, (const char *)t->data + offset, size);
}
void be_sync(ggml_backend_t b) { tts_hip_synchronize(((BackendCtx *)b->context)->be); }

enum ggml_status be_graph_compute(ggml_backend_t b, struct ggml_cgraph * cg) {
    auto * c = (BackendCtx *)b->context;
    const int n = ggml_graph_n_nodes(cg);
    c->m.reset((size_t)n * (GGML_MAX_SRC + 2) + 64);
    for (int i = 0; i < n; ++i) {
        tts_tensor * t = mirror(c->m, ggml_graph_node(cg, i));
        if (!t) return GGML_STATUS_FAILED;
        c->m.nodes.push_back(t);
    }
    const int st = tts_hip_graph_compute(c->be, c->m.nodes.data(), (int)c->m.nodes.size());
    return st == TTS_STATUS_SUCCESS ? GGML_STATUS_SUCCESS : st == TTS_STATUS_ALLOC_FAILED ? GGML_STATUS_ALLOC_FAILED : GGML_STATUS_FAILED;
}

void be_event_record(ggml_backend_t b, ggml_backend_event_t ev) { tts_hip_event_record(((BackendCtx *)b->context)->be, ev->context); }
void be_event_wait(ggml_backend_t b, ggml_backend_event_t ev) { tts_hip_event_wait(((BackendCtx *)b->context)->be, ev->context); }

ggml_guid_t be_guid() {
    static ggml_guid guid = {0x74, 0x74, 0x73, 0x2d, 0x68, 0x69, 0x70, 0x2d, 0x67, 0x66, 0x78, 0x39, 0x35, 0x30, 0x00, 0x01};
    return &guid;
}

// ---------------------------------------------------------------------------------------------
// device vtable
const char * dev_name(ggml_backend_dev_t d) { return ((DevCtx *)d->context)->name.c_str(); }
const char * dev_desc(ggml_backend_dev_t d) { return ((DevCtx *)d->context)->desc.c_str(); }
void dev_memory(ggml_backend_dev_t d, size_t * free_b, size_t * total) {
    if (tts_hip_device_memory(((DevCtx *)d->context)->device, free_b, total) != 0) *free_b = *total = 0;
}
enum ggml_backend_dev_type dev_type(ggml_backend_dev_t) { return GGML_BACKEND_DEVICE_TYPE_GPU; }
void dev_props(ggml_backend_dev_t d, struct ggml_backend_dev_props * p) {
    p->name = dev_name(d);
    p->description = dev_desc(d);
    p->type = GGML_BACKEND_DEVICE_TYPE_GPU;
    dev_memory(d, &p->memory_free, &p->memory_total);
    p->caps.async = true;
    p->caps.host_buffer = false;
    p->caps.buffer_from_host_ptr = false;
    p->caps.events = true;
}

ggml_backend_t dev_init(ggml_backend_dev_t d, const char *) {
    auto * dc = (DevCtx *)d->context;
    tts_hip_backend_t be = tts_hip_backend_init(dc->device);
    if (!be) return nullptr;
    auto * c = new BackendCtx();
    c->device = dc->device;
    c->be = be;
    ggml_backend_i iface;
    std::memset(&iface, 0, sizeof(iface));
    iface.get_name = be_name;
    iface.free = be_free;
    iface.set_tensor_async = be_set_async;
    iface.get_tensor_async = be_get_async;
    iface.synchronize = be_sync;
    iface.graph_compute = be_graph_compute;
    iface.event_record = be_event_record;
    iface.event_wait = be_event_wait;
    return new ggml_backend{be_guid(), iface, d, c};
}

ggml_backend_buffer_type_t dev_buft(ggml_backend_dev_t d) { return &((DevCtx *)d->context)->buft; }

bool dev_supports_op(ggml_backend_dev_t d, const ggml_tensor * op) {
    if (!srcs_on_device(op, d)) return false;
    Mirror m;
    m.reset(256);
    const tts_tensor * t = mirror(m, op, 2);
    if (!t || t->op < 0) return false;
    for (const tts_tensor * s : t->src)
        if (s && (s->flags & TTS_FLAG_HOSTDATA)) return false;
    return tts_hip_supports_op(t) != 0;
}

bool dev_supports_buft(ggml_backend_dev_t d, ggml_backend_buffer_type_t buft) {
    return is_ours(buft) && buft->device == d;
}

// weights in a host buffer: worth the upload only for batched products (prefill, encoders)
bool dev_offload_op(ggml_backend_dev_t, const ggml_tensor * op) { return op->op == GGML_OP_MUL_MAT && op->ne[1] >= 32; }

ggml_backend_event_t dev_event_new(ggml_backend_dev_t d) {
    void * ev = tts_hip_event_new(((DevCtx *)d->context)->device);
    return ev ? new ggml_backend_event{d, ev} : nullptr;
}
void dev_event_free(ggml_backend_dev_t, ggml_backend_event_t ev) {
    tts_hip_event_free(ev->context);
    delete ev;
}
void dev_event_sync(ggml_backend_dev_t, ggml_backend_event_t ev) { tts_hip_event_synchronize(ev->context); }

// ---------------------------------------------------------------------------------------------
// registry
const char * reg_name(ggml_backend_reg_t) { return "TTS-HIP"; }
size_t reg_count(ggml_backend_reg_t r) { return ((RegCtx *)r->context)->devs.size(); }
ggml_backend_dev_t reg_device(ggml_backend_reg_t r, size_t i) {
    auto * c = (RegCtx *)r->context;
    return i < c->devs.size() ? &c->devs[i] : nullptr;
}
void * reg_proc(ggml_backend_reg_t, const char * name) {
    if (std::strcmp(name, "ggml_backend_tts_hip_register_custom") == 0) return (void *)ggml_backend_tts_hip_register_custom;
    return nullptr;
}

ggml_backend_reg * make_reg() {
    static ggml_backend_reg reg;
    static RegCtx ctx;
    ggml_backend_reg_i ri;
    std::memset(&ri, 0, sizeof(ri));
    ri.get_name = reg_name;
    ri.get_device_count = reg_count;
    ri.get_device = reg_device;
    ri.get_proc_address = reg_proc;
    reg.api_version = GGML_BACKEND_API_VERSION;
    reg.iface = ri;
    reg.context = &ctx;
    const int n = tts_hip_device_count();
    ctx.devs.resize(n > 0 ? n : 0);  // no reallocation afterwards: devices keep their addresses
    for (int i = 0; i < n; ++i) {
        auto * dc = new DevCtx();
        dc->device = i;
        dc->name = "TTS-HIP" + std::to_string(i);
        dc->desc = "AMD Instinct MI355X (gfx950), libtts_hip";
        ggml_backend_device_i di;
        std::memset(&di, 0, sizeof(di));
        di.get_name = dev_name;
        di.get_description = dev_desc;
        di.get_memory = dev_memory;
        di.get_type = dev_type;
        di.get_props = dev_props;
        di.init_backend = dev_init;
        di.get_buffer_type = dev_buft;
        di.supports_op = dev_supports_op;
        di.supports_buft = dev_supports_buft;
        di.offload_op = dev_offload_op;
        di.event_new = dev_event_new;
        di.event_free = dev_event_free;
        di.event_synchronize = dev_event_sync;
        ggml_backend_buffer_type_i bi;
        std::memset(&bi, 0, sizeof(bi));
        bi.get_name = buft_name;
        bi.alloc_buffer = buft_alloc;
        bi.get_alignment = buft_align;
        bi.get_max_size = buft_max;
        bi.get_alloc_size = buft_alloc_size;
        bi.is_host = buft_is_host;
        ctx.devs[i].iface = di;
        ctx.devs[i].reg = &reg;
        ctx.devs[i].context = dc;
        dc->buft.iface = bi;
        dc->buft.device = &ctx.devs[i];
        dc->buft.context = dc;
        ctx.ctx.push_back(dc);
    }
    return &reg;
}

}  // namespace

extern "C" ggml_backend_reg_t ggml_backend_tts_hip_reg(void) {
    static ggml_backend_reg * reg = make_reg();
    return reg;
}

extern "C" int ggml_backend_tts_hip_default_device(void) {
    const char * e = std::getenv("TTS_HIP_DEVICE");
    return e ? std::atoi(e) : 0;
}

extern "C" ggml_backend_t ggml_backend_tts_hip_init(int device) {
    ggml_backend_reg_t r = ggml_backend_tts_hip_reg();
    ggml_backend_dev_t d = reg_device(r, (size_t)device);
    return d ? dev_init(d, nullptr) : nullptr;
}

extern "C" ggml_backend_buffer_type_t ggml_backend_tts_hip_buffer_type(int device) {
    ggml_backend_dev_t d = reg_device(ggml_backend_tts_hip_reg(), (size_t)device);
    return d ? dev_buft(d) : nullptr;
}

extern "C" bool ggml_backend_is_tts_hip(ggml_backend_t backend) {
    return backend && backend->iface.get_name == be_name;
}

extern "C" void ggml_backend_tts_hip_register_custom(const void * fn, int kind) {
    std::lock_guard<std::mutex> lk(g_custom_mu);
    g_custom[fn] = kind;
}

#ifdef GGML_BACKEND_DL
GGML_BACKEND_DL_IMPL(ggml_backend_tts_hip_reg)
#endif
