// GGUF reader / writer and the quantize tool (include/tts_gguf.h).
//
// File layout (GGUF v2/v3, little endian): "GGUF", u32 version, u64 n_tensors, u64 n_kv, the KV pairs
// (string key, u32 type, value; arrays carry u32 element type + u64 count), the tensor infos (string
// name, u32 n_dims, i64 ne[n_dims], u32 ggml_type, u64 offset into the data section), padding to
// general.alignment (default 32), then the data section with every tensor at an aligned offset.
// The reader maps the file read-only and validates every length against the mapping, the writer
// lays a file out the way gguf_write_to_file does (tensors in insertion order, padded).
// The quantize tool follows examples/quantize/quantize_impl.cpp:181-292 (its per-architecture rules
// at :14-80); the row quantizer is a callback so the device kernels (tts_hip_quantize) do the work.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "tts_gguf.h"

namespace {

struct kv_entry {
    std::string key;
    int32_t type = 0;
    std::vector<uint8_t> scalar;  // numeric / bool value bytes
    std::string str;
    int32_t arr_type = -1;
    std::vector<uint8_t> arr;     // packed numeric array
    std::vector<std::string> arr_str;
};

struct tensor_info {
    std::string name;
    int32_t n_dims = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    int32_t type = 0;
    uint64_t offset = 0;
    uint64_t size = 0;
};

size_t scalar_size(int32_t t) {
    switch (t) {
        case TTS_GGUF_UINT8: case TTS_GGUF_INT8: case TTS_GGUF_BOOL: return 1;
        case TTS_GGUF_UINT16: case TTS_GGUF_INT16: return 2;
        case TTS_GGUF_UINT32: case TTS_GGUF_INT32: case TTS_GGUF_FLOAT32: return 4;
        case TTS_GGUF_UINT64: case TTS_GGUF_INT64: case TTS_GGUF_FLOAT64: return 8;
        default: return 0;
    }
}

bool scalar_to_f64(int32_t t, const uint8_t * p, double * out) {
    switch (t) {
        case TTS_GGUF_UINT8: *out = *p; return true;
        case TTS_GGUF_INT8: *out = (int8_t)*p; return true;
        case TTS_GGUF_BOOL: *out = *p != 0; return true;
        case TTS_GGUF_UINT16: { uint16_t v; memcpy(&v, p, 2); *out = v; return true; }
        case TTS_GGUF_INT16: { int16_t v; memcpy(&v, p, 2); *out = v; return true; }
        case TTS_GGUF_UINT32: { uint32_t v; memcpy(&v, p, 4); *out = v; return true; }
        case TTS_GGUF_INT32: { int32_t v; memcpy(&v, p, 4); *out = v; return true; }
        case TTS_GGUF_FLOAT32: { float v; memcpy(&v, p, 4); *out = v; return true; }
        case TTS_GGUF_UINT64: { uint64_t v; memcpy(&v, p, 8); *out = (double)v; return true; }
        case TTS_GGUF_INT64: { int64_t v; memcpy(&v, p, 8); *out = (double)v; return true; }
        case TTS_GGUF_FLOAT64: memcpy(out, p, 8); return true;
        default: return false;
    }
}

bool scalar_to_i64(int32_t t, const uint8_t * p, int64_t * out) {
    switch (t) {
        case TTS_GGUF_UINT64: { uint64_t v; memcpy(&v, p, 8); *out = (int64_t)v; return true; }
        case TTS_GGUF_INT64: memcpy(out, p, 8); return true;
        case TTS_GGUF_FLOAT32: case TTS_GGUF_FLOAT64: return false;
        default: {
            double d;
            if (!scalar_to_f64(t, p, &d)) return false;
            *out = (int64_t)d;
            return true;
        }
    }
}

// Bounds-checked cursor over the mapping.
struct cursor {
    const uint8_t * p;
    const uint8_t * end;
    bool ok = true;
    bool take(void * dst, size_t n) {
        if (!ok || (size_t)(end - p) < n) return ok = false;
        memcpy(dst, p, n);
        p += n;
        return true;
    }
    template <typename T> bool get(T & v) { return take(&v, sizeof(T)); }
    bool str(std::string & s) {
        uint64_t n = 0;
        if (!get(n) || (uint64_t)(end - p) < n) return ok = false;
        s.assign((const char *)p, (size_t)n);
        p += n;
        return true;
    }
};

}  // namespace

struct tts_gguf {
    void * map = nullptr;
    size_t map_size = 0;
    uint32_t version = 0;
    uint64_t alignment = 32;
    uint64_t data_offset = 0;
    std::vector<kv_entry> kv;
    std::vector<tensor_info> tensors;
    std::unordered_map<std::string, int64_t> kv_index, tensor_index;
};

struct tts_gguf_writer {
    std::vector<kv_entry> kv;
    std::vector<tensor_info> tensors;
    std::vector<std::vector<uint8_t>> data;
    kv_entry & slot(const char * key) {
        for (auto & e : kv)
            if (e.key == key) {
                e = kv_entry();
                e.key = key;
                return e;
            }
        kv.emplace_back();
        kv.back().key = key;
        return kv.back();
    }
};

extern "C" {

size_t tts_gguf_type_size(int32_t type) {
    switch (type) {
        case 0: return 4;    // F32
        case 1: return 2;    // F16
        case 2: return 18;   // Q4_0
        case 3: return 20;   // Q4_1
        case 6: return 22;   // Q5_0
        case 7: return 24;   // Q5_1
        case 8: return 34;   // Q8_0
        case 9: return 36;   // Q8_1
        case 10: return 84;  // Q2_K
        case 11: return 110; // Q3_K
        case 12: return 144; // Q4_K
        case 13: return 176; // Q5_K
        case 14: return 210; // Q6_K
        case 15: return 292; // Q8_K
        case 24: return 1;   // I8
        case 25: return 2;   // I16
        case 26: return 4;   // I32
        case 27: return 8;   // I64
        case 28: return 8;   // F64
        case 30: return 2;   // BF16
        default: return 0;
    }
}

int64_t tts_gguf_blck_size(int32_t type) {
    switch (type) {
        case 2: case 3: case 6: case 7: case 8: case 9: return 32;
        case 10: case 11: case 12: case 13: case 14: case 15: return 256;
        default: return tts_gguf_type_size(type) ? 1 : 0;
    }
}

// Element count of ne[0..3] (each >= 0), or -1 when the product would not fit int64 (ggml's gguf
// reader rejects such files the same way: INT64_MAX / ne[1] / ne[2] / ne[3] bounds).
static int64_t checked_nelements(const int64_t * ne) {
    int64_t n = 1;
    for (int d = 0; d < 4; ++d) {
        if (ne[d] < 0) return -1;
        if (ne[d] == 0) return 0;
        if (n > INT64_MAX / ne[d]) return -1;
        n *= ne[d];
    }
    return n;
}

// bytes of a tensor, or 0 for an unknown type / ragged blocks / a size that overflows 64 bits
static uint64_t tensor_bytes(int32_t type, const int64_t * ne) {
    const size_t ts = tts_gguf_type_size(type);
    const int64_t bs = tts_gguf_blck_size(type);
    if (!ts || !bs || ne[0] % bs || checked_nelements(ne) < 0) return 0;
    uint64_t b = (uint64_t)(ne[0] / bs);
    const uint64_t f[4] = {(uint64_t)ts, (uint64_t)ne[1], (uint64_t)ne[2], (uint64_t)ne[3]};
    for (uint64_t v : f) {
        if (v && b > UINT64_MAX / v) return 0;
        b *= v;
    }
    return b;
}

tts_gguf * tts_gguf_open(const char * path) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) {
        fprintf(stderr, "gguf: cannot open %s\n", path);
        return nullptr;
    }
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size < 24) {
        fprintf(stderr, "gguf: %s is too short\n", path);
        ::close(fd);
        return nullptr;
    }
    void * map = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (map == MAP_FAILED) {
        fprintf(stderr, "gguf: mmap of %s failed\n", path);
        return nullptr;
    }
    auto * g = new tts_gguf();
    g->map = map;
    g->map_size = (size_t)st.st_size;
    auto fail = [&](const char * why) -> tts_gguf * {
        fprintf(stderr, "gguf: %s: %s\n", path, why);
        tts_gguf_close(g);
        return nullptr;
    };
    cursor c{(const uint8_t *)map, (const uint8_t *)map + g->map_size};
    char magic[4];
    c.take(magic, 4);
    if (memcmp(magic, "GGUF", 4) != 0) return fail("bad magic");
    uint64_t n_tensors = 0, n_kv = 0;
    c.get(g->version);
    if (g->version < 2 || g->version > 3) return fail("unsupported version (2 or 3)");
    c.get(n_tensors);
    c.get(n_kv);
    if (!c.ok || n_kv > (1u << 24) || n_tensors > (1u << 24)) return fail("bad header");
    for (uint64_t i = 0; i < n_kv; ++i) {
        kv_entry e;
        c.str(e.key);
        c.get(e.type);
        if (!c.ok) return fail("truncated KV section");
        if (e.type == TTS_GGUF_STRING) {
            c.str(e.str);
        } else if (e.type == TTS_GGUF_ARRAY) {
            uint64_t n = 0;
            c.get(e.arr_type);
            c.get(n);
            if (!c.ok) return fail("truncated array");
            if (e.arr_type == TTS_GGUF_STRING) {
                if (n > (uint64_t)(c.end - c.p) / 8) return fail("bad string array length");
                e.arr_str.resize((size_t)n);
                for (uint64_t j = 0; j < n && c.ok; ++j) c.str(e.arr_str[(size_t)j]);
            } else {
                const size_t es = scalar_size(e.arr_type);
                if (!es || n > (uint64_t)(c.end - c.p) / es) return fail("bad array");
                e.arr.resize((size_t)n * es);
                c.take(e.arr.data(), e.arr.size());
            }
        } else {
            const size_t es = scalar_size(e.type);
            if (!es) return fail("unknown KV type");
            e.scalar.resize(es);
            c.take(e.scalar.data(), es);
        }
        if (!c.ok) return fail("truncated KV value");
        g->kv_index[e.key] = (int64_t)g->kv.size();
        g->kv.push_back(std::move(e));
    }
    const auto al = g->kv_index.find("general.alignment");
    if (al != g->kv_index.end()) {
        uint32_t a = 0;
        if (!tts_gguf_get_u32(g, al->second, &a) || a == 0 || (a & (a - 1))) return fail("bad general.alignment");
        g->alignment = a;
    }
    for (uint64_t i = 0; i < n_tensors; ++i) {
        tensor_info t;
        c.str(t.name);
        uint32_t nd = 0;
        c.get(nd);
        if (!c.ok || nd < 1 || nd > 4) return fail("bad tensor dims");
        t.n_dims = (int32_t)nd;
        for (uint32_t d = 0; d < nd; ++d) c.get(t.ne[d]);
        c.get(t.type);
        c.get(t.offset);
        if (!c.ok) return fail("truncated tensor info");
        for (int d = 0; d < 4; ++d)
            if (t.ne[d] < 0) return fail("negative dimension");
        const int64_t nel = checked_nelements(t.ne);
        if (nel < 0) return fail("element count overflows int64");
        t.size = tensor_bytes(t.type, t.ne);
        if (t.size == 0 && nel != 0) return fail("unknown tensor type, ragged blocks or size overflow");
        if (t.offset % g->alignment) return fail("unaligned tensor offset");
        if (g->tensor_index.count(t.name)) return fail("duplicate tensor name");
        g->tensor_index[t.name] = (int64_t)g->tensors.size();
        g->tensors.push_back(std::move(t));
    }
    const uint64_t hdr = (uint64_t)(c.p - (const uint8_t *)map);
    g->data_offset = (hdr + g->alignment - 1) / g->alignment * g->alignment;
    // overflow-safe: each term is compared with what is left of the mapping, never summed first
    if (!g->tensors.empty() && g->data_offset > g->map_size) return fail("tensor data past the end of the file");
    const uint64_t avail = g->data_offset > g->map_size ? 0 : g->map_size - g->data_offset;
    for (auto & t : g->tensors)
        if (t.offset > avail || t.size > avail - t.offset) return fail("tensor data past the end of the file");
    return g;
}

void tts_gguf_close(tts_gguf * g) {
    if (!g) return;
    if (g->map) munmap(g->map, g->map_size);
    delete g;
}

uint32_t tts_gguf_version(const tts_gguf * g) { return g->version; }
uint64_t tts_gguf_alignment(const tts_gguf * g) { return g->alignment; }
uint64_t tts_gguf_data_offset(const tts_gguf * g) { return g->data_offset; }
int64_t tts_gguf_n_kv(const tts_gguf * g) { return (int64_t)g->kv.size(); }

int64_t tts_gguf_find_key(const tts_gguf * g, const char * key) {
    const auto it = g->kv_index.find(key);
    return it == g->kv_index.end() ? -1 : it->second;
}

static const kv_entry * kv_at(const tts_gguf * g, int64_t i) { return (i >= 0 && i < (int64_t)g->kv.size()) ? &g->kv[(size_t)i] : nullptr; }

const char * tts_gguf_key(const tts_gguf * g, int64_t i) {
    const kv_entry * e = kv_at(g, i);
    return e ? e->key.c_str() : nullptr;
}

int32_t tts_gguf_kv_type(const tts_gguf * g, int64_t i) {
    const kv_entry * e = kv_at(g, i);
    return e ? e->type : -1;
}

int tts_gguf_get_u32(const tts_gguf * g, int64_t i, uint32_t * out) {
    int64_t v;
    if (!tts_gguf_get_i64(g, i, &v) || v < 0 || v > 0xFFFFFFFFll) return 0;
    *out = (uint32_t)v;
    return 1;
}

int tts_gguf_get_i64(const tts_gguf * g, int64_t i, int64_t * out) {
    const kv_entry * e = kv_at(g, i);
    return e && !e->scalar.empty() && scalar_to_i64(e->type, e->scalar.data(), out) ? 1 : 0;
}

int tts_gguf_get_f64(const tts_gguf * g, int64_t i, double * out) {
    const kv_entry * e = kv_at(g, i);
    return e && !e->scalar.empty() && scalar_to_f64(e->type, e->scalar.data(), out) ? 1 : 0;
}

const char * tts_gguf_get_str(const tts_gguf * g, int64_t i) {
    const kv_entry * e = kv_at(g, i);
    return e && e->type == TTS_GGUF_STRING ? e->str.c_str() : nullptr;
}

int32_t tts_gguf_arr_type(const tts_gguf * g, int64_t i) {
    const kv_entry * e = kv_at(g, i);
    return e && e->type == TTS_GGUF_ARRAY ? e->arr_type : -1;
}

int64_t tts_gguf_arr_n(const tts_gguf * g, int64_t i) {
    const kv_entry * e = kv_at(g, i);
    if (!e || e->type != TTS_GGUF_ARRAY) return 0;
    return e->arr_type == TTS_GGUF_STRING ? (int64_t)e->arr_str.size() : (int64_t)(e->arr.size() / scalar_size(e->arr_type));
}

const void * tts_gguf_arr_data(const tts_gguf * g, int64_t i) {
    const kv_entry * e = kv_at(g, i);
    return e && e->type == TTS_GGUF_ARRAY && e->arr_type != TTS_GGUF_STRING ? e->arr.data() : nullptr;
}

const char * tts_gguf_arr_str(const tts_gguf * g, int64_t i, int64_t j) {
    const kv_entry * e = kv_at(g, i);
    if (!e || e->type != TTS_GGUF_ARRAY || e->arr_type != TTS_GGUF_STRING || j < 0 || j >= (int64_t)e->arr_str.size()) return nullptr;
    return e->arr_str[(size_t)j].c_str();
}

int64_t tts_gguf_n_tensors(const tts_gguf * g) { return (int64_t)g->tensors.size(); }

int64_t tts_gguf_find_tensor(const tts_gguf * g, const char * name) {
    const auto it = g->tensor_index.find(name);
    return it == g->tensor_index.end() ? -1 : it->second;
}

static const tensor_info * ti_at(const tts_gguf * g, int64_t i) { return (i >= 0 && i < (int64_t)g->tensors.size()) ? &g->tensors[(size_t)i] : nullptr; }

const char * tts_gguf_tensor_name(const tts_gguf * g, int64_t i) {
    const tensor_info * t = ti_at(g, i);
    return t ? t->name.c_str() : nullptr;
}

int32_t tts_gguf_tensor_type(const tts_gguf * g, int64_t i) {
    const tensor_info * t = ti_at(g, i);
    return t ? t->type : -1;
}

int32_t tts_gguf_tensor_ndims(const tts_gguf * g, int64_t i, int64_t * ne4) {
    const tensor_info * t = ti_at(g, i);
    if (!t) return 0;
    if (ne4)
        for (int d = 0; d < 4; ++d) ne4[d] = t->ne[d];
    return t->n_dims;
}

uint64_t tts_gguf_tensor_offset(const tts_gguf * g, int64_t i) {
    const tensor_info * t = ti_at(g, i);
    return t ? t->offset : 0;
}

uint64_t tts_gguf_tensor_size(const tts_gguf * g, int64_t i) {
    const tensor_info * t = ti_at(g, i);
    return t ? t->size : 0;
}

const void * tts_gguf_tensor_data(const tts_gguf * g, int64_t i) {
    const tensor_info * t = ti_at(g, i);
    return t ? (const char *)g->map + g->data_offset + t->offset : nullptr;
}

// ---- writer ----
tts_gguf_writer * tts_gguf_writer_new(void) { return new tts_gguf_writer(); }
void tts_gguf_writer_free(tts_gguf_writer * w) { delete w; }

static void set_scalar(tts_gguf_writer * w, const char * key, int32_t type, const void * v) {
    kv_entry & e = w->slot(key);
    e.type = type;
    e.scalar.resize(scalar_size(type));
    memcpy(e.scalar.data(), v, e.scalar.size());
}

void tts_gguf_set_u32(tts_gguf_writer * w, const char * key, uint32_t v) { set_scalar(w, key, TTS_GGUF_UINT32, &v); }
void tts_gguf_set_i32(tts_gguf_writer * w, const char * key, int32_t v) { set_scalar(w, key, TTS_GGUF_INT32, &v); }
void tts_gguf_set_f32(tts_gguf_writer * w, const char * key, float v) { set_scalar(w, key, TTS_GGUF_FLOAT32, &v); }
void tts_gguf_set_u64(tts_gguf_writer * w, const char * key, uint64_t v) { set_scalar(w, key, TTS_GGUF_UINT64, &v); }
void tts_gguf_set_bool(tts_gguf_writer * w, const char * key, int v) {
    const uint8_t b = v ? 1 : 0;
    set_scalar(w, key, TTS_GGUF_BOOL, &b);
}

void tts_gguf_set_str(tts_gguf_writer * w, const char * key, const char * v) {
    kv_entry & e = w->slot(key);
    e.type = TTS_GGUF_STRING;
    e.str = v;
}

void tts_gguf_set_arr(tts_gguf_writer * w, const char * key, int32_t elem_type, const void * data, int64_t n) {
    kv_entry & e = w->slot(key);
    e.type = TTS_GGUF_ARRAY;
    e.arr_type = elem_type;
    e.arr.resize((size_t)n * scalar_size(elem_type));
    if (!e.arr.empty()) memcpy(e.arr.data(), data, e.arr.size());
}

void tts_gguf_set_arr_str(tts_gguf_writer * w, const char * key, const char * const * v, int64_t n) {
    kv_entry & e = w->slot(key);
    e.type = TTS_GGUF_ARRAY;
    e.arr_type = TTS_GGUF_STRING;
    e.arr_str.assign(v, v + n);
}

void tts_gguf_copy_kv(tts_gguf_writer * w, const tts_gguf * src) {
    for (const auto & e : src->kv) w->slot(e.key.c_str()) = e;
}

int tts_gguf_add_tensor(tts_gguf_writer * w, const char * name, int32_t type, int32_t n_dims, const int64_t * ne, const void * data,
                        uint64_t nbytes) {
    if (n_dims < 1 || n_dims > 4) return TTS_STATUS_BAD_ARG;
    tensor_info t;
    t.name = name;
    t.type = type;
    t.n_dims = n_dims;
    for (int d = 0; d < n_dims; ++d) t.ne[d] = ne[d];
    t.size = tensor_bytes(type, t.ne);
    if (t.size != nbytes) return TTS_STATUS_BAD_ARG;
    for (const auto & o : w->tensors)
        if (o.name == t.name) return TTS_STATUS_BAD_ARG;
    w->tensors.push_back(t);
    w->data.emplace_back((const uint8_t *)data, (const uint8_t *)data + nbytes);
    return TTS_STATUS_SUCCESS;
}

int tts_gguf_writer_write(const tts_gguf_writer * w, const char * path) {
    uint64_t align = 32;
    for (const auto & e : w->kv)
        if (e.key == "general.alignment" && !e.scalar.empty()) {
            int64_t a = 0;
            if (scalar_to_i64(e.type, e.scalar.data(), &a) && a > 0 && !(a & (a - 1))) align = (uint64_t)a;
        }
    std::vector<uint8_t> out;
    auto put = [&](const void * p, size_t n) { out.insert(out.end(), (const uint8_t *)p, (const uint8_t *)p + n); };
    auto put_str = [&](const std::string & s) {
        const uint64_t n = s.size();
        put(&n, 8);
        put(s.data(), s.size());
    };
    put("GGUF", 4);
    const uint32_t version = 3;
    const uint64_t n_tensors = w->tensors.size(), n_kv = w->kv.size();
    put(&version, 4);
    put(&n_tensors, 8);
    put(&n_kv, 8);
    for (const auto & e : w->kv) {
        put_str(e.key);
        put(&e.type, 4);
        if (e.type == TTS_GGUF_STRING) {
            put_str(e.str);
        } else if (e.type == TTS_GGUF_ARRAY) {
            put(&e.arr_type, 4);
            const uint64_t n = e.arr_type == TTS_GGUF_STRING ? e.arr_str.size() : e.arr.size() / scalar_size(e.arr_type);
            put(&n, 8);
            if (e.arr_type == TTS_GGUF_STRING)
                for (const auto & s : e.arr_str) put_str(s);
            else
                put(e.arr.data(), e.arr.size());
        } else {
            put(e.scalar.data(), e.scalar.size());
        }
    }
    uint64_t off = 0;
    for (const auto & t : w->tensors) {
        put_str(t.name);
        const uint32_t nd = (uint32_t)t.n_dims;
        put(&nd, 4);
        put(t.ne, 8 * (size_t)nd);
        put(&t.type, 4);
        put(&off, 8);
        off += (t.size + align - 1) / align * align;
    }
    out.resize((out.size() + align - 1) / align * align, 0);
    FILE * f = fopen(path, "wb");
    if (!f) {
        fprintf(stderr, "gguf: cannot write %s\n", path);
        return TTS_STATUS_BAD_ARG;
    }
    bool ok = fwrite(out.data(), 1, out.size(), f) == out.size();
    static const uint8_t zeros[256] = {};
    for (size_t i = 0; ok && i < w->tensors.size(); ++i) {
        const auto & d = w->data[i];
        ok = fwrite(d.data(), 1, d.size(), f) == d.size();
        size_t pad = (size_t)((d.size() + align - 1) / align * align - d.size());
        while (ok && pad) {
            const size_t n = pad < sizeof(zeros) ? pad : sizeof(zeros);
            ok = fwrite(zeros, 1, n, f) == n;
            pad -= n;
        }
    }
    ok = (fclose(f) == 0) && ok;
    if (!ok) fprintf(stderr, "gguf: short write to %s\n", path);
    return ok ? TTS_STATUS_SUCCESS : TTS_STATUS_BAD_ARG;
}

// ---- quantize tool ----
static bool ends_with(const std::string & s, const char * suf) {
    const size_t n = strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}
static bool starts_with(const std::string & s, const char * pre) { return s.rfind(pre, 0) == 0; }
static bool contains(const std::string & s, const char * sub) { return s.find(sub) != std::string::npos; }

// kokoro_is_f16_compatible (quantize_impl.cpp:14-18)
static bool kokoro_f16_compatible(const std::string & n) {
    return !contains(n, "voice_tensors") && !contains(n, "bias") && !contains(n, "gamma") && !contains(n, "beta") && !contains(n, "alpha") &&
           !ends_with(n, "embd") && !ends_with(n, "norm");
}

int tts_gguf_tensor_rule(const char * arch_c, const char * name_c, const tts_quantize_params * p) {
    const std::string arch = arch_c ? arch_c : "parler-tts", n = name_c;
    bool q = false;
    if (arch == "parler-tts") {  // parler_is_quanitizable (:51-67)
        q = !starts_with(n, "audio_encoder") && !ends_with(n, "norm.weight") && !ends_with(n, "text_encoding") && !ends_with(n, "positional_embed") &&
            !ends_with(n, "norm.bias");
        if (!p->quantize_output_heads) q = q && !ends_with(n, "weight.head");
        if (!p->quantize_text_embeddings) q = q && !ends_with(n, "embed_prompts");
        if (!p->quantize_cross_attn_kv) q = q && !ends_with(n, "encoder_attn.k_proj.weight") && !ends_with(n, "encoder_attn.v_proj.weight");
    } else if (arch == "dia") {  // dia_is_quantizable (:42-49)
        q = !starts_with(n, "audio_encoder") && !ends_with(n, "norm");
        if (!p->quantize_output_heads) q = q && !starts_with(n, "dia.decoder.heads");
    } else if (arch == "kokoro") {  // kokoro_is_quantizable (:20-40)
        if (kokoro_f16_compatible(n)) {
            if (starts_with(n, "kokoro.albert") || starts_with(n, "kokoro.text_encoder.lstm")) q = true;
            else if (starts_with(n, "kokoro.duration_predictor.")) {
                const size_t a = n.find('.', 0), b = a == std::string::npos ? a : n.find('.', a + 1);
                const size_t c = b == std::string::npos ? b : n.find('.', b + 1);
                const std::string part = b == std::string::npos ? "" : n.substr(b + 1, c == std::string::npos ? std::string::npos : c - b - 1);
                q = part == "duration_proj" || part == "encode" || part == "shared_lstm" || part == "duration_lstm" || part == "layers";
            }
        }
    } else if (arch == "orpheus") {  // not in the reference (it aborts): every matrix except norms
        q = ends_with(n, ".weight") && !contains(n, "norm");
        if (!p->quantize_output_heads) q = q && !contains(n, "lm_head");
    } else {
        return -1;
    }
    if (q) return 1;
    // quantize_impl.cpp:264-265: non-quantizable Kokoro tensors / DAC tensors to F16 when asked
    if ((p->convert_non_quantizable_to_f16 && kokoro_f16_compatible(n)) ||
        (p->convert_dac_to_f16 && starts_with(n, "audio_encoder") && !ends_with(n, "alpha")))
        return 2;
    return 0;
}

// ggml_fp32_to_fp16: round to nearest even, subnormals, overflow to inf, NaN kept quiet
static uint16_t f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7FFFFFFFu;
    if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u | ((ax >> 13) & 0x3FFu));  // NaN
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);                          // rounds to inf
    if (ax < 0x38800000u) {                                                            // f16 subnormal / zero
        if (ax < 0x33000000u) return (uint16_t)sign;                                   // < half the smallest subnormal
        const uint32_t m = (ax & 0x7FFFFFu) | 0x800000u;
        const int shift = 126 - (int)(ax >> 23);  // 14 + (113 - e)
        uint32_t r = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (r & 1))) ++r;
        return (uint16_t)(sign | r);
    }
    uint32_t r = ((ax >> 13) - (112u << 10));
    const uint32_t rem = ax & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (r & 1))) ++r;
    return (uint16_t)(sign | r);
}

int tts_gguf_quantize(const char * in_path, const char * out_path, const tts_quantize_params * p, tts_quantize_rows_fn fn, void * fn_ctx) {
    if (!p || (p->quantize_type != TTS_TYPE_Q4_K && p->quantize_type != TTS_TYPE_Q8_0 && p->quantize_type != TTS_TYPE_F16)) {
        fprintf(stderr, "gguf quantize: type must be Q4_K, Q8_0 or F16\n");
        return TTS_STATUS_BAD_ARG;
    }
    tts_gguf * g = tts_gguf_open(in_path);
    if (!g) return TTS_STATUS_BAD_ARG;
    std::string arch = "parler-tts";  // only parler-tts files lack general.architecture (:188)
    const int64_t ak = tts_gguf_find_key(g, "general.architecture");
    if (ak >= 0 && tts_gguf_get_str(g, ak)) arch = tts_gguf_get_str(g, ak);
    int st = TTS_STATUS_SUCCESS;
    tts_gguf_writer * w = tts_gguf_writer_new();
    tts_gguf_copy_kv(w, g);
    tts_gguf_set_u32(w, "general.quantization_version", 2);  // GGML_QNT_VERSION
    tts_gguf_set_u32(w, "general.quantization_type", (uint32_t)p->quantize_type);
    std::vector<uint8_t> buf;
    std::vector<uint16_t> h16;
    for (int64_t i = 0; i < tts_gguf_n_tensors(g) && st == TTS_STATUS_SUCCESS; ++i) {
        const std::string name = tts_gguf_tensor_name(g, i);
        if (name.empty()) continue;
        int64_t ne[4];
        const int nd = tts_gguf_tensor_ndims(g, i, ne);
        const int32_t type = tts_gguf_tensor_type(g, i);
        const void * src = tts_gguf_tensor_data(g, i);
        const int rule = tts_gguf_tensor_rule(arch.c_str(), name.c_str(), p);
        if (rule < 0) {
            fprintf(stderr, "gguf quantize: architecture '%s' is not supported\n", arch.c_str());
            st = TTS_STATUS_BAD_ARG;
            break;
        }
        const int64_t n = ne[0] * ne[1] * ne[2] * ne[3];
        int32_t new_type = type;
        const void * data = src;
        uint64_t size = tts_gguf_tensor_size(g, i);
        if (rule > 0 && type != TTS_TYPE_F32) {  // :248-253 / :266-271
            fprintf(stderr, "gguf quantize: tensor '%s' must be F32 to be converted (type %d)\n", name.c_str(), type);
            st = TTS_STATUS_BAD_ARG;
            break;
        }
        if (rule > 0 && n == 0) {  // the reader bounds n (int64, inside the mapping); an empty row cannot be converted
            fprintf(stderr, "gguf quantize: tensor '%s' to be converted is empty\n", name.c_str());
            st = TTS_STATUS_BAD_ARG;
            break;
        }
        if (rule == 1 && p->quantize_type != TTS_TYPE_F16) {
            new_type = p->quantize_type;
            const int64_t bs = tts_gguf_blck_size(new_type);
            if (ne[0] % bs) {
                fprintf(stderr, "gguf quantize: tensor '%s' row length %lld is not a multiple of %lld\n", name.c_str(), (long long)ne[0],
                        (long long)bs);
                st = TTS_STATUS_BAD_ARG;
                break;
            }
            size = tensor_bytes(new_type, ne);
            buf.resize((size_t)size);
            if (fn(fn_ctx, new_type, (const float *)src, buf.data(), n / ne[0], ne[0]) != 0) {
                st = TTS_STATUS_BAD_ARG;
                break;
            }
            data = buf.data();
        } else if (rule >= 1) {  // F16 (rule 2, or quantize_type F16)
            new_type = TTS_TYPE_F16;
            h16.resize((size_t)n);
            const float * x = (const float *)src;
            for (int64_t e = 0; e < n; ++e) h16[(size_t)e] = f32_to_f16(x[e]);
            data = h16.data();
            size = (uint64_t)n * 2;
        }
        st = tts_gguf_add_tensor(w, name.c_str(), new_type, nd, ne, data, size);
    }
    if (st == TTS_STATUS_SUCCESS) st = tts_gguf_writer_write(w, out_path);
    tts_gguf_writer_free(w);
    tts_gguf_close(g);
    return st;
}

// device rows: host -> device, tts_hip_quantize, device -> host (one tensor at a time)
static int hip_rows(void * ctx, int32_t type, const float * x, void * dst, int64_t rows, int64_t K) {
    auto * be = (tts_hip_backend_t)ctx;
    const size_t xb = (size_t)rows * (size_t)K * 4;
    const size_t qb = (size_t)rows * (size_t)(K / tts_gguf_blck_size(type)) * tts_gguf_type_size(type);
    void * dx = tts_hip_buffer_alloc(be, xb);
    void * dq = tts_hip_buffer_alloc(be, qb);
    int st = (dx && dq) ? TTS_STATUS_SUCCESS : TTS_STATUS_ALLOC_FAILED;
    if (st == TTS_STATUS_SUCCESS) st = tts_hip_tensor_set(be, dx, x, xb);
    if (st == TTS_STATUS_SUCCESS) st = tts_hip_quantize(be, type, (const float *)dx, dq, rows, K);
    if (st == TTS_STATUS_SUCCESS) st = tts_hip_tensor_get(be, dst, dq, qb);
    if (st == TTS_STATUS_SUCCESS) st = tts_hip_synchronize(be);
    if (dx) tts_hip_buffer_free(be, dx);
    if (dq) tts_hip_buffer_free(be, dq);
    return st;
}

int tts_hip_gguf_quantize(tts_hip_backend_t be, const char * in_path, const char * out_path, const tts_quantize_params * params) {
    if (!be) {
        fprintf(stderr, "gguf quantize: no HIP backend\n");
        return TTS_STATUS_BAD_ARG;
    }
    return tts_gguf_quantize(in_path, out_path, params, hip_rows, be);
}

}  // extern "C"
