// HIP backend: the C-ABI of include/tts_hip.h.  One backend = one device + one HIP stream
// (one per runner, as TTS.cpp's server runs one runner per worker thread:
// /root/reference/examples/server/server.cpp:316-321).
#include <cmath>
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "hip_internal.h"
#include <hip/hip_ext.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

using namespace tts;


// GGML_GELU_FP16 table: fp16(ggml_gelu_f32(fp16_to_fp32(i))) for every fp16 bit pattern,
// computed on the host with the same f32 expression ggml uses (no contraction; see Makefile).
static void build_gelu_table(uint16_t * t) {
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    for (int i = 0; i < 65536; ++i) {
        const float x = fp16_to_fp32_host((uint16_t)i);
        const float g = 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
        t[i] = fp32_to_fp16_host(g);
    }
}

static const size_t kScratchBytes = 64u << 20;
static const size_t kShadowBytes = 4u << 20;  // private copy of an attention output (decode: 32 KB per 8 prompts)
static const size_t kLstmFloats = 4u << 20;
static const size_t kAttnFloats = 4u << 20;  // split attention scores: e.g. B 8 x H 16 x P 4096 = 512K floats
static const size_t kVecScratchFloats = 1u << 18;  // per-channel vectors staged by fused items (AdaIN)
static const size_t kPinBytes = 16u << 20;   // pinned staging ring for set_tensor_async   // 16 MB: e.g. 2 chains of Hd 256 x T 8191

// Process-wide registries: the live tts_hip_buffer_alloc ranges and the tile-layout copies of
// medium lane-layout Q4_K weights, keyed by device address.  A weight buffer may be allocated and
// written through one backend and read by the graphs of another (the ggml adapter allocates through
// a utility backend, every ggml_backend computes on its own stream), so neither is per backend.
namespace {
std::mutex g_reg_mu;
struct BufRec {
    size_t size = 0;
};
std::map<const char *, BufRec> g_buffers;                // base -> record (ordered: range lookups)
std::unordered_map<const void *, uint8_t *> g_tiled;     // weight -> its tile-layout copy
std::atomic<size_t> g_tiled_n{0};
}  // namespace

namespace tts {
const uint8_t * tiled_copy_find(const void * w) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_tiled.find(w);
    return it == g_tiled.end() ? nullptr : it->second;
}
// process-wide coalescer switch (tts_hip_coalesce_enable; TTS_HIP_COALESCE=0 at load turns it off)
static std::atomic<int> g_coalesce_on{[] {
    const char * e = getenv("TTS_HIP_COALESCE");
    return e && e[0] == '0' ? 0 : 1;
}()};
bool coalesce_enabled() { return g_coalesce_on.load(std::memory_order_relaxed) != 0; }
bool buffer_lookup(const void * p, const char ** base, size_t * size) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_buffers.upper_bound((const char *)p);
    if (it == g_buffers.begin()) return false;
    --it;
    if ((const char *)p >= it->first + it->second.size) return false;
    if (base) *base = it->first;
    if (size) *size = it->second.size;
    return true;
}
}  // namespace tts

extern "C" {

int tts_hip_coalesce_enable(int on) { return tts::g_coalesce_on.exchange(on ? 1 : 0); }

int tts_hip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

tts_hip_backend_t tts_hip_backend_init(int device) {
    int n = tts_hip_device_count();
    if (device < 0 || device >= n) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    auto * be = new tts_hip_backend();
    be->device = device;
    TTS_HIP_CHECK(hipStreamCreateWithFlags(&be->stream, hipStreamNonBlocking));
    TTS_HIP_CHECK(hipStreamCreateWithFlags(&be->cap_stream, hipStreamNonBlocking));
    TTS_HIP_CHECK(hipStreamCreateWithFlags(&be->pf_stream, hipStreamNonBlocking));
    TTS_HIP_CHECK(hipEventCreateWithFlags(&be->co_ev, hipEventDisableTiming));
    TTS_HIP_CHECK(hipEventCreateWithFlags(&be->pf_fork, hipEventDisableTiming));
    TTS_HIP_CHECK(hipEventCreateWithFlags(&be->pf_join, hipEventDisableTiming));
    hipDeviceProp_t prop;
    TTS_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    snprintf(be->name, sizeof(be->name), "HIP%d(%s)", device, prop.gcnArchName);
    be->cu_total = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    be->cus = be->cu_total;
    TTS_HIP_CHECK(hipMalloc((void **)&be->scratch, kScratchBytes));
    be->scratch_size = kScratchBytes;
    TTS_HIP_CHECK(hipMalloc((void **)&be->shadow, kShadowBytes));
    be->shadow_size = kShadowBytes;
    be->hoist_size = (size_t)8 << 20;
    TTS_HIP_CHECK(hipMalloc(&be->hoist, be->hoist_size));
    TTS_HIP_CHECK(hipMalloc((void **)&be->lstm_buf, kLstmFloats * sizeof(float)));
    TTS_HIP_CHECK(hipMalloc((void **)&be->attn_buf, kAttnFloats * sizeof(float)));
    be->attn_floats = kAttnFloats;
    TTS_HIP_CHECK(hipMalloc((void **)&be->vec_scratch, kVecScratchFloats * sizeof(float)));
    be->conv_stage_floats = (size_t)8 << 20;  // 32 MiB: a [T, C] conv output of the largest vocoder level
    TTS_HIP_CHECK(hipMalloc((void **)&be->conv_stage, be->conv_stage_floats * sizeof(float)));
    be->conv_part_doubles = (size_t)8 << 20;  // 64 MiB of f64 partial sums
    TTS_HIP_CHECK(hipMalloc((void **)&be->conv_part, be->conv_part_doubles * sizeof(double)));
    be->lstm_floats = kLstmFloats;
    TTS_HIP_CHECK(hipMalloc((void **)&be->argmax_keys, kArgmaxRows * sizeof(unsigned long long)));
    TTS_HIP_CHECK(hipMalloc((void **)&be->argmax_counts, kArgmaxRows * sizeof(unsigned)));
    TTS_HIP_CHECK(hipMemset(be->argmax_keys, 0, kArgmaxRows * sizeof(unsigned long long)));
    TTS_HIP_CHECK(hipMemset(be->argmax_counts, 0, kArgmaxRows * sizeof(unsigned)));
    TTS_HIP_CHECK(hipHostMalloc((void **)&be->pin, kPinBytes, hipHostMallocDefault));
    be->pin_size = kPinBytes;
    for (auto & e : be->plan_ev) TTS_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    std::vector<uint16_t> tab(65536);
    build_gelu_table(tab.data());
    TTS_HIP_CHECK(hipMalloc((void **)&be->gelu_table, 65536 * sizeof(uint16_t)));
    TTS_HIP_CHECK(hipMemcpy(be->gelu_table, tab.data(), 65536 * sizeof(uint16_t), hipMemcpyHostToDevice));
    return be;
}

void tts_hip_backend_free(tts_hip_backend_t be) {
    if (!be) return;
    tts::coalesce_backend_gone(be);
    hipSetDevice(be->device);
    hipStreamSynchronize(be->stream);
    for (auto & p : be->ev_pending) {
        hipEventDestroy(p.first);
        hipEventDestroy(p.second);
    }
    for (auto e : be->ev_free) hipEventDestroy(e);
    for (auto & r : be->pin_pending) hipEventDestroy(r.ev);
    for (auto e : be->pin_events) hipEventDestroy(e);
    for (auto e : be->plan_ev) hipEventDestroy(e);
    hipHostFree(be->pin);
    if (be->rb_host) hipHostFree(be->rb_host);
    hipFree(be->scratch);
    hipFree(be->shadow);
    hipFree(be->argmax_keys);
    hipFree(be->argmax_counts);
    hipFree(be->lstm_buf);
    hipFree(be->hoist);
    hipFree(be->attn_buf);
    hipFree(be->vec_scratch);
    hipFree(be->conv_stage);
    hipFree(be->conv_part);
    hipFree(be->gelu_table);
    if (be->sample_cand) hipFree(be->sample_cand);
    if (be->repack_tmp) hipFree(be->repack_tmp);
    for (char * r : be->repack_retired) hipFree(r);
    for (auto & ex : be->gsig_exec)
        if (ex) hipGraphExecDestroy(ex);
    for (auto & ex : be->pexec)
        if (ex) hipGraphExecDestroy(ex);
    hipStreamDestroy(be->stream);
    hipStreamDestroy(be->cap_stream);
    hipStreamDestroy(be->pf_stream);
    hipEventDestroy(be->pf_fork);
    hipEventDestroy(be->pf_join);
    hipEventDestroy(be->co_ev);
    delete be;
}

const char * tts_hip_backend_name(tts_hip_backend_t be) { return be ? be->name : "HIP(null)"; }

int tts_hip_device_memory(int device, size_t * free_bytes, size_t * total_bytes) {
    if (device < 0 || device >= tts_hip_device_count()) return TTS_STATUS_NO_DEVICE;
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(device);
    size_t f = 0, t = 0;
    const hipError_t e = hipMemGetInfo(&f, &t);
    hipSetDevice(prev);
    if (e != hipSuccess) return TTS_STATUS_FAILED;
    if (free_bytes) *free_bytes = f;
    if (total_bytes) *total_bytes = t;
    return 0;
}

void * tts_hip_event_new(int device) {
    if (device < 0 || device >= tts_hip_device_count()) return nullptr;
    hipSetDevice(device);
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
    return (void *)ev;
}
void tts_hip_event_free(void * event) {
    if (event) hipEventDestroy((hipEvent_t)event);
}
int tts_hip_event_record(tts_hip_backend_t be, void * event) {
    if (!be || !event) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    return hipEventRecord((hipEvent_t)event, be->stream) == hipSuccess ? 0 : TTS_STATUS_FAILED;
}
int tts_hip_event_wait(tts_hip_backend_t be, void * event) {
    if (!be || !event) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    return hipStreamWaitEvent(be->stream, (hipEvent_t)event, 0) == hipSuccess ? 0 : TTS_STATUS_FAILED;
}
int tts_hip_event_synchronize(void * event) {
    if (!event) return TTS_STATUS_BAD_ARG;
    return hipEventSynchronize((hipEvent_t)event) == hipSuccess ? 0 : TTS_STATUS_FAILED;
}
int tts_hip_is_device_pointer(const void * p) {
    if (!p) return 0;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return a.type == hipMemoryTypeDevice ? 1 : 0;
}

size_t tts_hip_buffer_alignment(void) { return 256; }

void * tts_hip_buffer_alloc(tts_hip_backend_t be, size_t size) {
    if (!be) return nullptr;
    hipSetDevice(be->device);
    void * p = nullptr;
    BufRec r;
    r.size = size ? size : 256;
    if (hipMalloc(&p, r.size) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_buffers[(const char *)p] = r;
    return p;
}

// Tile-layout copies of weights inside [p, p + n): freed when their weight buffer goes away or its
// bytes are overwritten by a plain tensor_set (a stale copy must never be read: run_gemv_item aborts
// on a TILED_COPY weight whose copy is gone instead).  The device is synchronised first: a graph on
// any stream may still read a copy.
static void drop_tiled_copies(const void * p, size_t n) {
    if (g_tiled_n.load(std::memory_order_acquire) == 0) return;
    const char * a = (const char *)p;
    std::vector<uint8_t *> dead;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        for (auto it = g_tiled.begin(); it != g_tiled.end();) {
            const char * k = (const char *)it->first;
            if (k >= a && k < a + n) {
                dead.push_back(it->second);
                it = g_tiled.erase(it);
            } else {
                ++it;
            }
        }
        g_tiled_n.store(g_tiled.size(), std::memory_order_release);
    }
    if (dead.empty()) return;
    hipDeviceSynchronize();
    for (uint8_t * c : dead) hipFree(c);
}

void tts_hip_buffer_free(tts_hip_backend_t be, void * ptr) {
    if (!be || !ptr) return;
    hipSetDevice(be->device);
    hipStreamSynchronize(be->stream);
    BufRec r;
    bool known = false;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto b = g_buffers.find((const char *)ptr);
        if (b != g_buffers.end()) {
            r = b->second;
            known = true;
            g_buffers.erase(b);
        }
    }
    if (known) {
        drop_tiled_copies(ptr, r.size);
        tts::coalesce_written(ptr, r.size);  // the coalescer's equal-content records over the range go
    }
    hipFree(ptr);
}

int tts_hip_tensor_set(tts_hip_backend_t be, void * dst, const void * src, size_t size) {
    if (!be) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();
    drop_tiled_copies(dst, size);
    tts::coalesce_written(dst, size);
    // synchronous (the copy has landed on return, as ggml_backend_tensor_set promises).  Small inputs (a
    // step's tokens, positions, masks) are staged through this backend's own pinned ring: a pageable
    // copy goes through the runtime's staging buffer, which many runners' threads (the step
    // coalescer's one-prompt runners) take in turn
    if (size > 0 && size <= be->pin_size / 4) {
        const int st = tts_hip_tensor_set_async(be, dst, src, size);
        if (st != 0) return st;
    } else if (hipMemcpyAsync(dst, src, size, hipMemcpyHostToDevice, be->stream) != hipSuccess) {
        return TTS_STATUS_FAILED;
    }
    if (hipStreamSynchronize(be->stream) != hipSuccess) return TTS_STATUS_FAILED;
    return 0;
}

// ggml_backend_i::set_tensor_async: the bytes are staged in pinned memory now (the caller may reuse
// `src` at once) and copied in stream order, so the host does not wait for work already queued.
int tts_hip_tensor_set_async(tts_hip_backend_t be, void * dst, const void * src, size_t size) {
    if (!be) return TTS_STATUS_BAD_ARG;
    if (size == 0) return 0;
    hipSetDevice(be->device);
    be->rb_clear();
    if (size > be->pin_size / 2) return tts_hip_tensor_set(be, dst, src, size);
    tts::coalesce_written(dst, size);
    std::lock_guard<std::mutex> pl(be->pin_mu);
    // recycle finished regions
    while (!be->pin_pending.empty() && hipEventQuery(be->pin_pending.front().ev) == hipSuccess) {
        be->pin_events.push_back(be->pin_pending.front().ev);
        be->pin_pending.pop_front();
    }
    size_t off = (be->pin_head + 255) & ~(size_t)255;
    if (off + size > be->pin_size) off = 0;
    // wait for the newest pending copy whose staging overlaps; older ones finished before it
    int last = -1;
    for (int i = 0; i < (int)be->pin_pending.size(); ++i) {
        const auto & r = be->pin_pending[i];
        if (r.off < off + size && off < r.off + r.size) last = i;
    }
    if (last >= 0) {
        if (hipEventSynchronize(be->pin_pending[last].ev) != hipSuccess) return TTS_STATUS_FAILED;
        for (int i = 0; i <= last; ++i) {
            be->pin_events.push_back(be->pin_pending.front().ev);
            be->pin_pending.pop_front();
        }
    }
    memcpy(be->pin + off, src, size);
    if (hipMemcpyAsync(dst, be->pin + off, size, hipMemcpyHostToDevice, be->stream) != hipSuccess) return TTS_STATUS_FAILED;
    hipEvent_t ev;
    if (be->pin_events.empty()) {
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return TTS_STATUS_FAILED;
    } else {
        ev = be->pin_events.back();
        be->pin_events.pop_back();
    }
    if (hipEventRecord(ev, be->stream) != hipSuccess) return TTS_STATUS_FAILED;
    be->pin_pending.push_back({off, size, ev});
    be->pin_head = off + size;
    return 0;
}

int tts_hip_greedy_step(tts_hip_backend_t be, const float * logits, int32_t B, int32_t NH, int32_t V, int32_t step, int32_t bos,
                        int32_t eos, int32_t * eos_seen, int32_t * hist, int32_t * next) {
    if (!be || !logits || B <= 0 || NH <= 0 || V <= 0) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();
    launch_greedy_step(be, logits, B, NH, V, step, bos, eos, eos_seen, hist, next);
    return 0;
}

int tts_hip_sample_step(tts_hip_backend_t be, const float * logits, int32_t B, int32_t NH, int32_t V, const tts_sampling * cfg, int64_t call,
                        int32_t * rep_state, int32_t step, int32_t bos, int32_t eos, int32_t * eos_seen, int32_t * hist, int32_t * next) {
    if (!be || !logits || !cfg || B <= 0 || NH <= 0 || V <= 0) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();
    return launch_sample_step(be, logits, B, NH, V, cfg, call, rep_state, step, bos, eos, eos_seen, hist, next);
}

int tts_hip_tensor_get(tts_hip_backend_t be, void * dst, const void * src, size_t size) {
    if (!be) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    // an output of this backend's last coalesced step: the executor already copied it to host memory
    // in stream order (co_readback)
    if (be->rb_any.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> l(be->rb_mu);
        for (const auto & r : be->rb) {
            const char * s = (const char *)src;
            if (s >= r.dev && s + size <= r.dev + r.bytes) {
                if (hipStreamSynchronize(be->stream) != hipSuccess) return TTS_STATUS_FAILED;
                memcpy(dst, be->rb_host + r.off + (s - r.dev), size);
                return 0;
            }
        }
    }
    // The reference reads the host copy right after get_tensor_async with no synchronize
    // (src/tts_model.cpp:25-36), so this call completes the stream first.
    if (hipMemcpyAsync(dst, src, size, hipMemcpyDeviceToHost, be->stream) != hipSuccess) return TTS_STATUS_FAILED;
    if (hipStreamSynchronize(be->stream) != hipSuccess) return TTS_STATUS_FAILED;
    return 0;
}

int tts_hip_copy_stream(tts_hip_backend_t be, void * dst, const void * src, size_t size) {
    if (!be || !dst || !src || size % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16) return TTS_STATUS_BAD_ARG;
    if (size == 0) return 0;
    hipSetDevice(be->device);
    be->rb_clear();
    tts::launch_copy_stream(be, dst, src, (int64_t)(size / 16));
    return hipGetLastError() == hipSuccess ? 0 : TTS_STATUS_FAILED;
}

int tts_hip_tensor_copy(tts_hip_backend_t be, void * dst, const void * src, size_t size) {
    if (!be) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();
    tts::coalesce_written(dst, size);
    tts::launch_copy_bytes(be, dst, src, size);  // a kernel, not a blit: ~2 us less host time per step
    return hipGetLastError() == hipSuccess ? 0 : TTS_STATUS_FAILED;
}

int tts_hip_memset(tts_hip_backend_t be, void * dst, int value, size_t size) {
    if (!be) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    be->rb_clear();
    tts::coalesce_written(dst, size);
    return hipMemsetAsync(dst, value, size, be->stream) == hipSuccess ? 0 : TTS_STATUS_FAILED;
}

int tts_hip_synchronize(tts_hip_backend_t be) {
    if (!be) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    return hipStreamSynchronize(be->stream) == hipSuccess ? 0 : TTS_STATUS_FAILED;
}

void tts_repack_q4_K(const void * src, void * dst, int64_t nblocks, int inverse) {
    const uint8_t * s = (const uint8_t *)src;
    uint8_t * d = (uint8_t *)dst;
    for (int64_t b = 0; b < nblocks; ++b) {
        const uint8_t * sb = s + b * 144;
        uint8_t * db = d + b * 144;
        memcpy(db, sb, 16);
        for (int i = 0; i < 128; ++i) {
            const int l = i >> 4, c = (i >> 2) & 3, k = i & 3;
            const int nat = 32 * c + 8 * k + l;
            if (!inverse) db[16 + i] = sb[16 + nat];
            else db[16 + nat] = sb[16 + i];
        }
    }
}

static void repack_tiled_rows(const uint8_t * s, uint8_t * d, int64_t r0, int64_t r1, int64_t nb, int inverse) {
    const int64_t rb = nb * 144;
    for (int64_t row = r0; row < r1; ++row) {
        const int64_t t = row >> 2, i = row & 3;
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t nat = row * rb + b * 144;           // native block
            const int64_t til = (t * nb + b) * 576;           // tile-layout block group
            const uint8_t * a = inverse ? s + til : s + nat;  // source side
            uint8_t * o = inverse ? d + nat : d + til;
            if (!inverse) memcpy(o + i * 16, a, 16);
            else memcpy(o, a + i * 16, 16);
            for (int c = 0; c < 4; ++c)
                for (int h = 0; h < 2; ++h)
                    for (int lp = 0; lp < 4; ++lp)
                        for (int kk = 0; kk < 4; ++kk) {
                            const int64_t tpos = 64 + ((c * 2 + h) * 4 + i) * 16 + lp * 4 + kk;
                            const int64_t npos = 16 + 32 * c + 8 * kk + 4 * h + lp;
                            if (!inverse) o[tpos] = a[npos];
                            else o[npos] = a[tpos];
                        }
        }
    }
}

void tts_repack_q4_K_tiled(const void * src, void * dst, int64_t nrows, int64_t nb, int inverse) {
    const uint8_t * s = (const uint8_t *)src;
    uint8_t * d = (uint8_t *)dst;
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt < 1 ? 1 : nt > 16 ? 16 : nt;
    if (nrows * nb < 4096 || nt == 1) {
        repack_tiled_rows(s, d, 0, nrows, nb, inverse);
        return;
    }
    std::vector<std::thread> th;
    const int64_t chunk = ((nrows + nt - 1) / nt + 3) & ~(int64_t)3;  // whole 4-row tiles per thread
    for (int64_t r0 = 0; r0 < nrows; r0 += chunk)
        th.emplace_back(repack_tiled_rows, s, d, r0, r0 + chunk < nrows ? r0 + chunk : nrows, nb, inverse);
    for (auto & t : th) t.join();
}

static size_t tensor_bytes(const tts_tensor * t) {
    size_t n = tts_row_size(t->type, t->ne[0]);
    for (int i = 1; i < 4; ++i) n *= (size_t)t->ne[i];
    return n;
}

static int weight_set_impl(tts_hip_backend_t be, tts_tensor * t, const void * src);
static std::atomic<bool> g_fault_weight_set{false};

// Crash diagnostics (tts_hip_install_crash_handler): on SIGSEGV / SIGBUS the faulting address, every
// frame as library + offset (+ symbol when exported), and the /proc/self/maps lines around the fault
// address go to stderr; then the previous handler (a profiler's, or the default) runs.  For hosts where
// a fault inside the HIP runtime must be attributed from the log alone (tracer fault).
static struct sigaction g_prev_segv, g_prev_bus;
static void crash_write(const char * s, int n) {
    while (n > 0) {
        const ssize_t w = write(2, s, (size_t)n);
        if (w <= 0) return;
        s += w, n -= (int)w;
    }
}
// Everything below runs in the signal handler, so only async-signal-safe calls: write / read / open /
// close, hand-rolled hex formatting, and backtrace() (libgcc is loaded at install by a first call, so
// the handler's call does not allocate).  Frames are attributed to a mapping by reading /proc/self/maps
// into a static buffer: "#i addr path+0xfileoffset".
static char g_crash_maps[1 << 20];
static int crash_hex(char * o, unsigned long v) {
    char t[16];
    int n = 0;
    do t[n++] = "0123456789abcdef"[v & 15], v >>= 4; while (v);
    o[0] = '0', o[1] = 'x';
    for (int i = 0; i < n; ++i) o[2 + i] = t[n - 1 - i];
    return n + 2;
}
static int crash_dec(char * o, int v) {
    char t[12];
    int n = 0;
    do t[n++] = (char)('0' + v % 10), v /= 10; while (v);
    for (int i = 0; i < n; ++i) o[i] = t[n - 1 - i];
    return n;
}
static const char * crash_parse_hex(const char * p, unsigned long * v) {
    unsigned long x = 0;
    for (;; ++p) {
        const char c = *p;
        const int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1;
        if (d < 0) break;
        x = x * 16 + (unsigned long)d;
    }
    *v = x;
    return p;
}
// one maps line: start-end perms offset dev inode path
static bool crash_map_line(const char * l, const char * e, unsigned long * a, unsigned long * b, unsigned long * off, const char ** path, int * plen) {
    const char * p = crash_parse_hex(l, a);
    if (*p != '-') return false;
    p = crash_parse_hex(p + 1, b);
    while (p < e && *p == ' ') ++p;
    while (p < e && *p != ' ') ++p;  // perms
    while (p < e && *p == ' ') ++p;
    p = crash_parse_hex(p, off);
    for (int f = 0; f < 2; ++f) {  // dev, inode
        while (p < e && *p == ' ') ++p;
        while (p < e && *p != ' ') ++p;
    }
    while (p < e && *p == ' ') ++p;
    *path = p, *plen = (int)(e - p);
    return true;
}
static void crash_handler(int sig, siginfo_t * si, void * uc) {
    char buf[640];
    int n = 0;
    const char h1[] = "tts_hip: signal ";
    for (const char * c = h1; *c; ++c) buf[n++] = *c;
    n += crash_dec(buf + n, sig);
    const char h2[] = ", fault address ";
    for (const char * c = h2; *c; ++c) buf[n++] = *c;
    const uintptr_t fa = si ? (uintptr_t)si->si_addr : 0;
    n += crash_hex(buf + n, fa);
    buf[n++] = '\n';
    crash_write(buf, n);
    int mlen = 0;
    {
        const int fd = open("/proc/self/maps", O_RDONLY);
        if (fd >= 0) {
            ssize_t r;
            while (mlen < (int)sizeof g_crash_maps - 1 && (r = read(fd, g_crash_maps + mlen, sizeof g_crash_maps - 1 - mlen)) > 0) mlen += (int)r;
            close(fd);
        }
    }
    void * fr[64];
    const int nf = backtrace(fr, 64);
    for (int i = 0; i < nf; ++i) {
        n = 0;
        buf[n++] = ' ', buf[n++] = ' ', buf[n++] = '#';
        n += crash_dec(buf + n, i);
        buf[n++] = ' ';
        n += crash_hex(buf + n, (unsigned long)(uintptr_t)fr[i]);
        buf[n++] = ' ';
        bool found = false;
        for (int l0 = 0; l0 < mlen && !found;) {
            int l1 = l0;
            while (l1 < mlen && g_crash_maps[l1] != '\n') ++l1;
            unsigned long a = 0, b = 0, off = 0;
            const char * path = nullptr;
            int plen = 0;
            if (crash_map_line(g_crash_maps + l0, g_crash_maps + l1, &a, &b, &off, &path, &plen) && (uintptr_t)fr[i] >= a &&
                (uintptr_t)fr[i] < b && plen > 0) {
                for (int k = 0; k < plen && n < (int)sizeof buf - 24; ++k) buf[n++] = path[k];
                buf[n++] = '+';
                n += crash_hex(buf + n, (unsigned long)(uintptr_t)fr[i] - a + off);
                found = true;
            }
            l0 = l1 + 1;
        }
        if (!found) buf[n++] = '?';
        buf[n++] = '\n';
        crash_write(buf, n);
    }
    // the mappings within 64 MiB of the fault address
    crash_write("tts_hip: maps near the fault address:\n", 38);
    for (int l0 = 0; l0 < mlen;) {
        int l1 = l0;
        while (l1 < mlen && g_crash_maps[l1] != '\n') ++l1;
        unsigned long a = 0, b = 0, off = 0;
        const char * path = nullptr;
        int plen = 0;
        if (crash_map_line(g_crash_maps + l0, g_crash_maps + l1, &a, &b, &off, &path, &plen) && fa + (64ul << 20) >= a && fa <= b + (64ul << 20))
            crash_write(g_crash_maps + l0, l1 - l0 + (l1 < mlen ? 1 : 0));
        l0 = l1 + 1;
    }
    const struct sigaction & prev = sig == SIGBUS ? g_prev_bus : g_prev_segv;
    if (prev.sa_flags & SA_SIGINFO) {
        if (prev.sa_sigaction) prev.sa_sigaction(sig, si, uc);
    } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN && prev.sa_handler) {
        prev.sa_handler(sig);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

int tts_hip_install_crash_handler(void) {
    void * warm[2];
    (void)backtrace(warm, 2);  // loads libgcc's unwinder now, outside any signal context
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = crash_handler;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGSEGV, &sa, &g_prev_segv) != 0 || sigaction(SIGBUS, &sa, &g_prev_bus) != 0) return TTS_STATUS_FAILED;
    return 0;
}

int tts_hip_test_hook(int hook, int value) {
    if (hook == TTS_HIP_HOOK_FAULT_WEIGHT_SET) {
        g_fault_weight_set.store(value != 0);
        return 0;
    }
    return TTS_STATUS_BAD_ARG;
}

int tts_hip_weight_set(tts_hip_backend_t be, tts_tensor * t, const void * src) {
    if (!be || !t) return TTS_STATUS_BAD_ARG;
    // fault injection for the callers' failure paths (tests/test_adapter_gpu.py, tts_hip_test_hook):
    // no layout is written
    if (t->type == TTS_TYPE_Q4_K && g_fault_weight_set.load(std::memory_order_relaxed)) return TTS_STATUS_ALLOC_FAILED;
    return weight_set_impl(be, t, src);
}

static int weight_set_impl(tts_hip_backend_t be, tts_tensor * t, const void * src) {
    const size_t n = tensor_bytes(t);
    if (t->type == TTS_TYPE_Q4_K && t->ne[0] % 256 == 0 && t->ne[1] % 4 == 0 && t->ne[2] == 1 && t->ne[3] == 1 &&
        be->q4k_tile_bytes > 0 && (int64_t)n >= be->q4k_tile_bytes) {
        // large matrix: the matrix-core GEMV's tile layout
        std::vector<uint8_t> tmp(n);
        tts_repack_q4_K_tiled(src, tmp.data(), t->ne[1], t->ne[0] / 256, 0);
        int st = tts_hip_tensor_set(be, t->data, tmp.data(), n);
        if (st == 0) t->flags |= TTS_FLAG_REPACKED | TTS_FLAG_TILED;
        return st;
    }
    if (t->type == TTS_TYPE_Q4_K && t->ne[0] % 256 == 0) {
        std::vector<uint8_t> tmp(n);
        tts_repack_q4_K(src, tmp.data(), (int64_t)(n / 144), 0);
        t->flags &= ~TTS_FLAG_TILED_COPY;  // a re-upload replaces the copy (tensor_set drops the old one)
        int st = tts_hip_tensor_set(be, t->data, tmp.data(), n);
        if (st == 0) t->flags |= TTS_FLAG_REPACKED;
        // (K >= 2048 only: run_gemv_item reads the copies of such matrices alone)
        if (st == 0 && be->q4k_dual_bytes > 0 && (int64_t)n >= be->q4k_dual_bytes && t->ne[0] >= 2048 && t->ne[1] % 16 == 0 &&
            t->ne[2] == 1 && t->ne[3] == 1) {
            // medium matrix: also a tile-layout copy for the matrix-core kernels at >= 8 columns
            tts_repack_q4_K_tiled(src, tmp.data(), t->ne[1], t->ne[0] / 256, 0);
            uint8_t * cp = nullptr;
            if (hipMalloc((void **)&cp, n) != hipSuccess) return TTS_STATUS_ALLOC_FAILED;
            if (hipMemcpy(cp, tmp.data(), n, hipMemcpyHostToDevice) != hipSuccess) {
                hipFree(cp);
                return TTS_STATUS_FAILED;
            }
            {
                std::lock_guard<std::mutex> lk(g_reg_mu);
                g_tiled[t->data] = cp;
                g_tiled_n.store(g_tiled.size(), std::memory_order_release);
            }
            t->flags |= TTS_FLAG_TILED_COPY;
        }
        return st;
    }
    return tts_hip_tensor_set(be, t->data, src, n);
}

int tts_hip_weight_get(tts_hip_backend_t be, const tts_tensor * t, void * dst) {
    if (!be || !t) return TTS_STATUS_BAD_ARG;
    const size_t n = tensor_bytes(t);
    if (t->type == TTS_TYPE_Q4_K && (t->flags & TTS_FLAG_TILED)) {
        std::vector<uint8_t> tmp(n);
        int st = tts_hip_tensor_get(be, tmp.data(), t->data, n);
        if (st == 0) tts_repack_q4_K_tiled(tmp.data(), dst, t->ne[1], t->ne[0] / 256, 1);
        return st;
    }
    if (t->type == TTS_TYPE_Q4_K && (t->flags & TTS_FLAG_REPACKED)) {
        std::vector<uint8_t> tmp(n);
        int st = tts_hip_tensor_get(be, tmp.data(), t->data, n);
        if (st == 0) tts_repack_q4_K(tmp.data(), dst, (int64_t)(n / 144), 1);
        return st;
    }
    return tts_hip_tensor_get(be, dst, t->data, n);
}

static bool is_f32(const tts_tensor * t) { return t && t->type == TTS_TYPE_F32; }

int tts_hip_supports_op(const tts_tensor * n) {
    if (!n) return 0;
    // a buffer-less host leaf (util.cpp:86-94 reciprocal trick) cannot be read by the device;
    // the adapter flags such sources with flags bit 1 (host data).
    for (int i = 0; i < TTS_MAX_SRC; ++i)
        if (n->src[i] && (n->src[i]->flags & 2)) return 0;
    switch (n->op) {
        case TTS_OP_NONE: case TTS_OP_VIEW: case TTS_OP_RESHAPE: case TTS_OP_PERMUTE: case TTS_OP_TRANSPOSE:
            return 1;
        case TTS_OP_DUP: case TTS_OP_CONT: case TTS_OP_CPY:
            return (n->type == TTS_TYPE_F32 || n->type == TTS_TYPE_F16 || n->type == TTS_TYPE_I32) &&
                   (n->src[0]->type == TTS_TYPE_F32 || n->src[0]->type == TTS_TYPE_F16 || n->src[0]->type == TTS_TYPE_I32);
        case TTS_OP_ADD: case TTS_OP_SUB: case TTS_OP_MUL: case TTS_OP_DIV:
        case TTS_OP_SQR: case TTS_OP_SQRT: case TTS_OP_SIN: case TTS_OP_COS: case TTS_OP_SCALE: case TTS_OP_CLAMP:
        case TTS_OP_LEAKY_RELU: case TTS_OP_ROUND: case TTS_OP_MOD: case TTS_OP_UNARY: case TTS_OP_CONCAT:
        case TTS_OP_REPEAT: case TTS_OP_SUM_ROWS:
            return 1;
        case TTS_OP_NORM: case TTS_OP_RMS_NORM:
            return is_f32(n->src[0]) && n->src[0]->nb[0] == 4;
        case TTS_OP_SOFT_MAX:
            return is_f32(n->src[0]);
        case TTS_OP_ROPE:
            return is_f32(n->src[0]);
        case TTS_OP_IM2COL:
            return is_f32(n->src[1]) && n->op_params[6] == 0 && (n->type == TTS_TYPE_F16 || n->type == TTS_TYPE_F32);
        case TTS_OP_CONV_TRANSPOSE_1D:
            return is_f32(n->src[0]) && is_f32(n->src[1]) && n->op_params[4] >= 1;
        case TTS_OP_CUMSUM: case TTS_OP_UPSCALE: case TTS_OP_STFT: case TTS_OP_ISTFT: case TTS_OP_MAP_CUSTOM3: case TTS_OP_MAP_CUSTOM2:
            return tts::audio_op_supported(n);
        case TTS_OP_GET_ROWS:
            return n->src[1]->type == TTS_TYPE_I32 &&
                   (n->src[0]->type == TTS_TYPE_F32 || n->src[0]->type == TTS_TYPE_F16 || n->src[0]->type == TTS_TYPE_Q4_K ||
                    n->src[0]->type == TTS_TYPE_Q8_0);
        case TTS_OP_MUL_MAT: {
            const tts_tensor * a = n->src[0];
            const tts_tensor * b = n->src[1];
            if (!is_f32(b)) return 0;
            // ggml_can_mul_mat: src1 broadcasts over src0 in dims 2 and 3
            if (a->ne[0] != b->ne[0] || b->ne[2] % a->ne[2] || b->ne[3] % a->ne[3]) return 0;
            if (a->type == TTS_TYPE_F32 || a->type == TTS_TYPE_F16) return 1;
            if (a->type == TTS_TYPE_Q4_K) return a->ne[0] % 256 == 0;
            if (a->type == TTS_TYPE_Q8_0) return a->ne[0] % 32 == 0;
            return 0;
        }
        default:
            return 0;
    }
}

}  // extern "C"

extern "C" int tts_hip_set_option(tts_hip_backend_t be, int option, int value) {
    if (!be) return TTS_STATUS_BAD_ARG;
    switch (option) {
        case TTS_HIP_OPT_FUSION: be->fusion = value; return 0;
        case TTS_HIP_OPT_CONVT_LDS: be->convt_lds = value != 0; return 0;
        case TTS_HIP_OPT_CONV_SPLIT: be->conv_split = value < 0 ? 1 : value; return 0;
        case TTS_HIP_OPT_PROFILE_GEMV: be->profile_gemv = value != 0; return 0;
        case TTS_HIP_OPT_GRAPHS: be->use_graphs = value != 0; return 0;
        case TTS_HIP_OPT_CONV_F32ACC:
            be->conv_f32acc = value == 1;
            be->conv_acc_mode = value == 2 ? 2 : 0;
            return 0;
        case TTS_HIP_OPT_ATTN_SPLIT: be->attn_split_minp = value; return 0;
        case TTS_HIP_OPT_ATTN_FUSED: be->attn_fused_minp = value; return 0;
        case TTS_HIP_OPT_ATTN_PV16: be->attn_pv_uv16 = value != 0; return 0;
        case TTS_HIP_OPT_KV_PREFETCH: be->kv_prefetch_minp = value; return 0;
        case TTS_HIP_OPT_Q4K_TILE_BYTES: be->q4k_tile_bytes = value; return 0;
        case TTS_HIP_OPT_Q4K_DUAL_BYTES: be->q4k_dual_bytes = value; return 0;
        case TTS_HIP_OPT_GEMV_RSPLIT: be->gemv_mf_rsplit = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_PREQUANT: be->gemv_mf_prequant = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_KRELAY: be->gemv_kr = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_KRELAY_LOOP: be->gemv_kr_loop = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_Q80_PRO: be->gemv_q80_pro = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_Q80_SLAB: be->gemv_q80_slab = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_KR_INKERNEL:
            if (value < 0) return TTS_STATUS_BAD_ARG;
            be->gemv_kr_ink = value;
            return 0;
        case TTS_HIP_OPT_GEMM_Q8_STAGED:
            if (value < 0 || value > 2) return TTS_STATUS_BAD_ARG;
            be->gemm_q8_staged = value;
            return 0;
        case TTS_HIP_OPT_GEMV_Q80_RW:
            if (value < 0 || value > 32 || (value & (value - 1))) return TTS_STATUS_BAD_ARG;
            be->gemv_q80_rw = value;
            return 0;
        case TTS_HIP_OPT_ATTN_KS: be->attn_ks = value; return 0;
        case TTS_HIP_OPT_GEMV_NW_MIN: be->gemv_nw_min = value; return 0;
        case TTS_HIP_OPT_ATTN_PV8: be->attn_pv8 = value != 0; return 0;
        case TTS_HIP_OPT_GEMM_KR_CT2: be->gemm_kr_ct2 = value != 0; return 0;
        case TTS_HIP_OPT_GEMM_KR_INKERNEL: be->gemm_kr_ink = value < 0 ? 0 : value; return 0;
        case TTS_HIP_OPT_ATTN_PV_MP: be->attn_pv_mp = value == 2 ? 2 : value != 0; return 0;
        case TTS_HIP_OPT_GEMM_KR_NW: be->gemm_kr_nw = value == 8 ? 8 : 4; return 0;
        case TTS_HIP_OPT_GEMM_Q8: be->gemm_q8 = value != 0; return 0;
        case TTS_HIP_OPT_CU_PARTITION: {
            const int count = value & 0xFF, index = (value >> 8) & 0xFF;
            const bool inter = (value >> 16) & 1;
            hipSetDevice(be->device);
            TTS_HIP_CHECK(hipStreamSynchronize(be->stream));
            hipStream_t ns = nullptr;
            if (count <= 1) {
                TTS_HIP_CHECK(hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
                be->cus = be->cu_total;
            } else {
                if (index >= count) return TTS_STATUS_BAD_ARG;
                std::vector<uint32_t> mask((be->cu_total + 31) / 32, 0u);
                const int per = be->cu_total / count;
                int n = 0;
                for (int c = 0; c < be->cu_total; ++c) {
                    const bool on = inter ? (c % count == index) : (c / per == index && c < per * count);
                    if (on) mask[c / 32] |= 1u << (c % 32), ++n;
                }
                if (hipExtStreamCreateWithCUMask(&ns, (uint32_t)mask.size(), mask.data()) != hipSuccess) return TTS_STATUS_FAILED;
                be->cus = n;
            }
            TTS_HIP_CHECK(hipStreamDestroy(be->stream));
            be->stream = ns;
            // executable graphs were recorded for the old stream's launches: drop them
            for (auto & ex : be->gsig_exec)
                if (ex) hipGraphExecDestroy(ex), ex = nullptr;
            for (auto & g : be->gsig) g = 0;
            return 0;
        }
        case TTS_HIP_OPT_BGEMM_F32: be->bgemm_f32 = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_F32_WIDE: be->gemv_f32_wide = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_DEBUG: be->gemv_dbg = value; return 0;
        case TTS_HIP_OPT_GEMV_UNIQUE: be->gemv_unique = value != 0; return 0;
        case TTS_HIP_OPT_GEMV_KS: be->gemv_ks_tiles = value > 0 ? value : 0; return 0;
        case TTS_HIP_OPT_COALESCE: be->co_member = value != 0; return 0;
        case TTS_HIP_OPT_GEMM_KR_XCD: be->gemm_kr_xcd = value != 0; return 0;
        case TTS_HIP_OPT_GEMM_KR_CP: be->gemm_kr_cp = value != 0; return 0;
        case TTS_HIP_OPT_GEMM_KR_WALK: be->gemm_kr_walk = value < 0 ? 0 : value; return 0;
        case TTS_HIP_OPT_GEMM_PF: be->gemm_pf = value < 0 ? 0 : value; return 0;
        case TTS_HIP_OPT_GEMM_PF_NW: be->gemm_pf_nw = value == 8 ? 8 : 4; return 0;
        case TTS_HIP_OPT_KV_PREFETCH_BLOCKS: be->kv_prefetch_blocks = value > 0 ? value : 1; return 0;
        default: return TTS_STATUS_BAD_ARG;
    }
}

extern "C" int tts_hip_counters(tts_hip_backend_t be, int64_t * out, int n) {
    if (!be || !out) return TTS_STATUS_BAD_ARG;
    const int64_t v[8] = {be->graph_updates, be->graph_instantiations, be->lstm_chains, be->lstm_steps, be->plan_wait_ns,
                          be->cap_plan_ns, be->cap_launch_ns, be->cap_update_ns};
    int k = 0;
    for (; k < n && k < 8; ++k) out[k] = v[k];
    return k;
}

extern "C" int tts_hip_gemv_stats(tts_hip_backend_t be, int type, double * ms, int64_t * launches, double * bytes, int reset) {
    if (!be) return TTS_STATUS_BAD_ARG;
    hipSetDevice(be->device);
    TTS_HIP_CHECK(hipStreamSynchronize(be->stream));
    for (size_t i = 0; i < be->ev_pending.size(); ++i) {
        float t = 0;
        TTS_HIP_CHECK(hipEventElapsedTime(&t, be->ev_pending[i].first, be->ev_pending[i].second));
        const int ty = be->ev_type[i];
        be->gemv_ms[ty] += t;
        be->gemv_launches[ty] += 1;
        be->gemv_bytes[ty] += be->ev_bytes[i];
        be->ev_free.push_back(be->ev_pending[i].first);
        be->ev_free.push_back(be->ev_pending[i].second);
    }
    be->ev_pending.clear();
    be->ev_bytes.clear();
    be->ev_type.clear();
    double a = 0, c = 0;
    int64_t b = 0;
    for (int ty = 0; ty < TTS_TYPE_COUNT; ++ty) {
        if (type >= 0 && ty != type) continue;
        a += be->gemv_ms[ty];
        b += be->gemv_launches[ty];
        c += be->gemv_bytes[ty];
    }
    if (ms) *ms = a;
    if (launches) *launches = b;
    if (bytes) *bytes = c;
    if (reset) {
        for (int ty = 0; ty < TTS_TYPE_COUNT; ++ty) {
            be->gemv_ms[ty] = 0;
            be->gemv_launches[ty] = 0;
            be->gemv_bytes[ty] = 0;
        }
    }
    return 0;
}

// ---- generic vtable over this backend ----
static void * hb_alloc(void * c, size_t n) { return tts_hip_buffer_alloc((tts_hip_backend_t)c, n); }
static void hb_free(void * c, void * p) { tts_hip_buffer_free((tts_hip_backend_t)c, p); }
static int hb_set(void * c, void * d, const void * s, size_t n) { return tts_hip_tensor_set((tts_hip_backend_t)c, d, s, n); }
static int hb_set_tensor(void * c, tts_tensor * t, const void * s) { return tts_hip_weight_set((tts_hip_backend_t)c, t, s); }
static int hb_get(void * c, void * d, const void * s, size_t n) { return tts_hip_tensor_get((tts_hip_backend_t)c, d, s, n); }
static int hb_memset(void * c, void * d, int v, size_t n) { return tts_hip_memset((tts_hip_backend_t)c, d, v, n); }
static int hb_compute(void * c, tts_tensor * const * nodes, int n) { return tts_hip_graph_compute((tts_hip_backend_t)c, nodes, n); }
static int hb_sync(void * c) { return tts_hip_synchronize((tts_hip_backend_t)c); }
static int hb_prepare(void * c, tts_tensor * const * nodes, int n, int slot) {
    return tts_hip_graph_prepare((tts_hip_backend_t)c, nodes, n, slot);
}
static int hb_launch(void * c, int slot) { return tts_hip_graph_launch((tts_hip_backend_t)c, slot); }
static int hb_set_async(void * c, void * d, const void * s, size_t n) { return tts_hip_tensor_set_async((tts_hip_backend_t)c, d, s, n); }
static int hb_copy(void * c, void * d, const void * s, size_t n) { return tts_hip_tensor_copy((tts_hip_backend_t)c, d, s, n); }
static int hb_greedy(void * c, const float * l, int B, int NH, int V, int step, int bos, int eos, int32_t * seen, int32_t * hist, int32_t * next) {
    return tts_hip_greedy_step((tts_hip_backend_t)c, l, B, NH, V, step, bos, eos, seen, hist, next);
}
static int hb_sample(void * c, const float * l, int B, int NH, int V, const tts_sampling * cfg, int64_t call, int32_t * rep, int step, int bos,
                     int eos, int32_t * seen, int32_t * hist, int32_t * next) {
    return tts_hip_sample_step((tts_hip_backend_t)c, l, B, NH, V, cfg, call, rep, step, bos, eos, seen, hist, next);
}

extern "C" int tts_hip_backend_iface(tts_hip_backend_t be, tts_backend_iface * out) {
    if (!be || !out) return TTS_STATUS_BAD_ARG;
    out->ctx = be;
    out->name = be->name;
    out->alloc = hb_alloc;
    out->free = hb_free;
    out->set = hb_set;
    out->set_tensor = hb_set_tensor;
    out->get = hb_get;
    out->memset = hb_memset;
    out->compute = hb_compute;
    out->synchronize = hb_sync;
    out->prepare = hb_prepare;
    out->launch = hb_launch;
    out->set_async = hb_set_async;
    out->copy = hb_copy;
    out->greedy_step = hb_greedy;
    out->sample_step = hb_sample;
    return 0;
}
