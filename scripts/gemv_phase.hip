// Phase timeline of the Q4_K GEMV (s_memrealtime per wave at kernel entry, after the first weight
// loads are issued, after the prologue, after the barrier, after each row, at exit).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Itts.cpp_amd/csrc \
//         scripts/gemv_phase.hip -o build/gemv_phase
// Prints one JSON line per shape: event-timed duration, body span and per-phase medians (us).
#define TTS_PHASE_TS
#include "../tts.cpp_amd/csrc/k_gemv.hip"
#include "../tts.cpp_amd/csrc/k_gemm.hip"
#include "../tts.cpp_amd/csrc/types.cpp"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

using namespace tts;

struct Shape {
    const char * name;
    int64_t K, N, M;
    int pro, nmat;
};

static double med(std::vector<double> v) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const Shape parler[] = {
        {"oproj_quant_m8", 1024, 1024, 8, PRO_QUANT, 1}, {"qkv_ln_m8", 1024, 1024, 8, PRO_LN, 3},
        {"fc1_ln_m8", 1024, 4096, 8, PRO_LN, 1},         {"fc2_quant_m8", 4096, 1024, 8, PRO_QUANT, 1},
        {"oproj_quant_m1", 1024, 1024, 1, PRO_QUANT, 1}, {"fc2_quant_m1", 4096, 1024, 1, PRO_QUANT, 1},
    };
    // GEMV_PHASE_ORPHEUS: Orpheus-3B decode matrices (hidden 3072, ffn 8192) at M = 8
    const Shape orpheus[] = {
        {"orph_q_ln_m8", 3072, 3072, 8, PRO_LN, 1},        {"orph_o_quant_m8", 3072, 3072, 8, PRO_QUANT, 1},
        {"orph_gateup_ln_m8", 3072, 8192, 8, PRO_LN, 2},   {"orph_down_quant_m8", 8192, 3072, 8, PRO_QUANT, 1},
        {"orph_qkv_ln_m8", 3072, 5120, 8, PRO_LN, 1},
    };
    // GEMV_PHASE_PREFILL: the batched prompt pass's products (576 columns: 32 prompts x 18 tokens) on the
    // prefill GEMM (k_gemm_q4K_pf; ts 0 entry, 1 loads issued, 2 operands landed, 3 first block pair, 4 last, 5 exit)
    const Shape prefill[] = {
        {"pf_oproj_576", 1024, 1024, 576, PRO_QUANT, 1}, {"pf_fc1_576", 1024, 4096, 576, PRO_QUANT, 1},
        {"pf_fc2_576", 4096, 1024, 576, PRO_QUANT, 1},
    };
    const bool orph = getenv("GEMV_PHASE_ORPHEUS") != nullptr;
    const bool pfs = getenv("GEMV_PHASE_PREFILL") != nullptr;
    const std::vector<Shape> shapes = pfs ? std::vector<Shape>(std::begin(prefill), std::end(prefill))
                                      : orph ? std::vector<Shape>(std::begin(orpheus), std::end(orpheus))
                                             : std::vector<Shape>(std::begin(parler), std::end(parler));
    tts_hip_backend be;
    be.gemv_unique = getenv("GEMV_UNIQUE") ? atoi(getenv("GEMV_UNIQUE")) : 1;
    if (getenv("GEMV_KS")) be.gemv_ks_tiles = atoi(getenv("GEMV_KS"));
    TTS_HIP_CHECK(hipStreamCreate(&be.stream));
    be.scratch_size = (size_t)64 << 20;  // the operand pass (GEMV_PREQUANT) writes the top of scratch
    TTS_HIP_CHECK(hipMalloc((void **)&be.scratch, be.scratch_size));
    if (getenv("GEMV_PREQUANT")) be.gemv_mf_prequant = atoi(getenv("GEMV_PREQUANT"));
    if (getenv("GEMV_KRELAY")) be.gemv_kr = atoi(getenv("GEMV_KRELAY"));
    std::mt19937 rng(1);
    const size_t wbytes = 3ull * 4096 * 4096 / 256 * 144;
    std::vector<uint8_t> hw(wbytes);
    for (size_t i = 0; i < wbytes; ++i) hw[i] = (uint8_t)rng();
    for (size_t b = 0; b < wbytes / 144; ++b) {  // finite fp16 d / dmin
        hw[b * 144 + 0] = 0x00, hw[b * 144 + 1] = 0x20;
        hw[b * 144 + 2] = 0x00, hw[b * 144 + 3] = 0x1C;
    }
    uint8_t * W;
    float *x, *y, *lnw, *lnb, *lno;
    unsigned long long * ts;
    const size_t nts = 1 << 20;
    TTS_HIP_CHECK(hipMalloc(&W, wbytes));
    TTS_HIP_CHECK(hipMemcpy(W, hw.data(), wbytes, hipMemcpyHostToDevice));
    std::vector<float> hx(576 * 4096);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (auto & v : hx) v = nd(rng);
    TTS_HIP_CHECK(hipMalloc(&x, hx.size() * 4));
    TTS_HIP_CHECK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    TTS_HIP_CHECK(hipMalloc(&y, (size_t)4 * 576 * 8192 * 4));
    TTS_HIP_CHECK(hipMalloc(&lnw, 4096 * 4));
    TTS_HIP_CHECK(hipMalloc(&lnb, 4096 * 4));
    TTS_HIP_CHECK(hipMalloc(&lno, 8 * 4096 * 4));
    TTS_HIP_CHECK(hipMemcpy(lnw, hx.data(), 4096 * 4, hipMemcpyHostToDevice));
    TTS_HIP_CHECK(hipMemcpy(lnb, hx.data() + 4096, 4096 * 4, hipMemcpyHostToDevice));
    TTS_HIP_CHECK(hipMalloc(&ts, nts * 8));
    // cold-cache reps: a 512 MiB write between launches evicts the weights from L2 and the
    // Infinity Cache, as a decode step's other traffic does in the real graph
    const bool cold = getenv("GEMV_PHASE_COLD") != nullptr;
    void * flush = nullptr;
    const size_t flush_bytes = (size_t)512 << 20;
    if (cold) TTS_HIP_CHECK(hipMalloc(&flush, flush_bytes));
    hipEvent_t e0, e1;
    TTS_HIP_CHECK(hipEventCreate(&e0));
    TTS_HIP_CHECK(hipEventCreate(&e1));

    for (const Shape & s : shapes) {
        GemvJob j;
        j.wtype = TTS_TYPE_Q4_K;
        j.nmat = s.nmat;
        j.K = s.K;
        j.N = s.N;
        j.M = s.M;
        j.w_row_bytes = s.K / 256 * 144;
        for (int i = 0; i < s.nmat; ++i) {
            j.W[i] = W + (size_t)i * s.N * j.w_row_bytes;
            j.Y[i] = y + (size_t)i * s.M * s.N;  // y holds 4 x 576 x 8192
            j.ycs[i] = s.N;
            j.yrs[i] = 1;
        }
        j.x = x;
        j.xcs = s.K;
        j.pro = s.pro;
        j.tiled = getenv("GEMV_PHASE_TILED") ? 1 : 0;  // tile layout (random bytes: layout-agnostic timing)
        if (s.pro == PRO_LN) {
            j.lnw = lnw, j.lnb = lnb, j.eps = 1e-5f, j.lnout = lno, j.locs = s.K;
        }
        for (int w = 0; w < 5; ++w) launch_gemv_job(&be, j);
        TTS_HIP_CHECK(hipStreamSynchronize(be.stream));
        std::vector<double> ev, span, p01, p12, p23, p3e, t0spread, endspread, p36, p64, p45, p34, p45b;
        for (int r = 0; r < 20; ++r) {
            TTS_HIP_CHECK(hipMemsetAsync(ts, 0, nts * 8, be.stream));
            if (cold) TTS_HIP_CHECK(hipMemsetAsync(flush, r, flush_bytes, be.stream));
            GemvJob jt = j;
            jt.ts = ts;
            TTS_HIP_CHECK(hipEventRecord(e0, be.stream));
            launch_gemv_job(&be, jt);
            TTS_HIP_CHECK(hipEventRecord(e1, be.stream));
            TTS_HIP_CHECK(hipStreamSynchronize(be.stream));
            float ms;
            TTS_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            ev.push_back(1000.0 * ms);
            std::vector<unsigned long long> h(nts);
            TTS_HIP_CHECK(hipMemcpy(h.data(), ts, nts * 8, hipMemcpyDeviceToHost));
            unsigned long long tmin = ~0ull, tmax = 0, t0max = 0, t5min = ~0ull;
            std::vector<double> a, b, c, d, e6, e4, e5, f34, f45;
            for (size_t w = 0; w + 8 <= nts; w += 8) {
                if (!h[w]) continue;
                tmin = std::min(tmin, h[w]);
                t0max = std::max(t0max, h[w]);
                tmax = std::max(tmax, h[w + 5]);
                t5min = std::min(t5min, h[w + 5]);
                a.push_back((h[w + 1] - h[w]) / 100.0);
                b.push_back((h[w + 2] - h[w + 1]) / 100.0);
                c.push_back((h[w + 3] - h[w + 2]) / 100.0);
                d.push_back((h[w + 5] - h[w + 3]) / 100.0);
                if (h[w + 4]) {
                    f34.push_back(((long long)h[w + 4] - (long long)h[w + 3]) / 100.0);
                    f45.push_back(((long long)h[w + 5] - (long long)h[w + 4]) / 100.0);
                }
                if (h[w + 6] && h[w + 4]) {
                    e6.push_back((h[w + 6] - h[w + 3]) / 100.0);
                    e4.push_back(((long long)h[w + 4] - (long long)h[w + 6]) / 100.0);
                    e5.push_back((h[w + 5] - h[w + 4]) / 100.0);
                }
            }
            span.push_back((tmax - tmin) / 100.0);
            t0spread.push_back((t0max - tmin) / 100.0);
            endspread.push_back((tmax - t5min) / 100.0);
            p01.push_back(med(a)), p12.push_back(med(b)), p23.push_back(med(c)), p3e.push_back(med(d));
            p36.push_back(med(e6)), p64.push_back(med(e4)), p45.push_back(med(e5));
            p34.push_back(med(f34)), p45b.push_back(med(f45));
        }
        // in-chain cost: 50 back-to-back launches captured as one HIP graph, replayed (warm caches)
        double chain_us = 0;
        {
            hipGraph_t g;
            hipGraphExec_t ge;
            TTS_HIP_CHECK(hipStreamBeginCapture(be.stream, hipStreamCaptureModeRelaxed));
            for (int i = 0; i < 50; ++i) launch_gemv_job(&be, j);
            TTS_HIP_CHECK(hipStreamEndCapture(be.stream, &g));
            TTS_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int w = 0; w < 3; ++w) TTS_HIP_CHECK(hipGraphLaunch(ge, be.stream));
            TTS_HIP_CHECK(hipStreamSynchronize(be.stream));
            TTS_HIP_CHECK(hipEventRecord(e0, be.stream));
            for (int r = 0; r < 10; ++r) TTS_HIP_CHECK(hipGraphLaunch(ge, be.stream));
            TTS_HIP_CHECK(hipEventRecord(e1, be.stream));
            TTS_HIP_CHECK(hipStreamSynchronize(be.stream));
            float ms;
            TTS_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            chain_us = 1000.0 * ms / 500.0;
            TTS_HIP_CHECK(hipGraphExecDestroy(ge));
            TTS_HIP_CHECK(hipGraphDestroy(g));
        }
        printf("{\"chain_us\":%.2f,\"cold\":%d,\"shape\":\"%s\",\"K\":%lld,\"N\":%lld,\"M\":%lld,\"nmat\":%d,\"event_us\":%.2f,\"span_us\":%.2f,"
               "\"start_spread_us\":%.2f,\"end_spread_us\":%.2f,\"issue_us\":%.2f,\"prologue_us\":%.2f,\"barrier_us\":%.2f,\"rows_us\":%.2f,\"wait_w_us\":%.2f,\"compute_us\":%.2f,\"store_exit_us\":%.2f,\"t34_us\":%.2f,\"t45_us\":%.2f}\n",
               chain_us, (int)cold, s.name, (long long)s.K, (long long)s.N, (long long)s.M, s.nmat, med(ev), med(span), med(t0spread), med(endspread), med(p01),
               med(p12), med(p23), med(p3e), med(p36), med(p64), med(p45), med(p34), med(p45b));
    }
    return 0;
}
