// Phase timeline of the decode attention kernel (s_memrealtime per wave: entry, after the scores,
// after the softmax, exit) for Parler's self-attention (P = 450 in a 4096-position cache) and
// cross-attention (P = 3, contiguous K / V).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Itts.cpp_amd/csrc \
//         scripts/attn_phase.hip -o build/attn_phase
#define TTS_PHASE_TS
#include "../tts.cpp_amd/csrc/k_attn.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace tts;

static double med(std::vector<double> v) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static TD td(void * data, std::initializer_list<int64_t> ne, std::initializer_list<int64_t> nb) {
    TD t{};
    t.data = (char *)data;
    int i = 0;
    for (auto v : ne) t.ne[i++] = v;
    i = 0;
    for (auto v : nb) t.nb[i++] = v;
    t.type = TTS_TYPE_F32;
    return t;
}

int main() {
    tts_hip_backend be;
    TTS_HIP_CHECK(hipStreamCreate(&be.stream));
    const int hd = 64, H = 16, B = 8, nctx = 4096, hidden = hd * H;
    float *kc, *vc, *q, *out, *mask, *ck, *cv;
    const size_t cache = (size_t)nctx * hidden * B;
    TTS_HIP_CHECK(hipMalloc(&kc, cache * 4));
    TTS_HIP_CHECK(hipMalloc(&vc, cache * 4));
    TTS_HIP_CHECK(hipMemset(kc, 0, cache * 4));
    TTS_HIP_CHECK(hipMemset(vc, 0, cache * 4));
    TTS_HIP_CHECK(hipMalloc(&q, hidden * B * 4));
    TTS_HIP_CHECK(hipMemset(q, 0, hidden * B * 4));
    TTS_HIP_CHECK(hipMalloc(&out, hidden * B * 4));
    TTS_HIP_CHECK(hipMalloc(&mask, nctx * 4));
    TTS_HIP_CHECK(hipMemset(mask, 0, nctx * 4));
    TTS_HIP_CHECK(hipMalloc(&ck, hd * 3 * H * 4));
    TTS_HIP_CHECK(hipMalloc(&cv, 3 * hd * H * B * 4));
    TTS_HIP_CHECK(hipMemset(ck, 0, hd * 3 * H * 4));
    TTS_HIP_CHECK(hipMemset(cv, 0, 3 * hd * H * B * 4));
    unsigned long long * ts;
    const size_t nts = 1 << 16;
    TTS_HIP_CHECK(hipMalloc(&ts, nts * 8));
    hipEvent_t e0, e1;
    TTS_HIP_CHECK(hipEventCreate(&e0));
    TTS_HIP_CHECK(hipEventCreate(&e1));

    struct Case {
        const char * name;
        AttnArgs a;
    };
    std::vector<Case> cases;
    for (int P : {450, 1500}) {
        AttnArgs a;
        a.q = td(q, {hd, 1, H, B}, {4, hidden * 4, hd * 4, hidden * 4});
        a.k = td(kc, {hd, P, H, B}, {4, hidden * 4, hd * 4, (int64_t)nctx * hidden * 4});
        a.v = td(vc, {P, hd, H, B}, {4, nctx * 4, (int64_t)nctx * hd * 4, (int64_t)nctx * hidden * 4});
        a.mask = mask;
        a.scale = 0.125f;
        a.out = out;
        a.hd = hd, a.P = P, a.H = H, a.n = 1, a.B = B;
        cases.push_back({P == 450 ? "self_p450" : "self_p1500", a});
    }
    {
        AttnArgs a;
        a.q = td(q, {hd, 1, H, B}, {4, hidden * 4, hd * 4, hidden * 4});
        a.k = td(ck, {hd, 3, H, 1}, {4, hd * 4, hd * 3 * 4, hd * 3 * H * 4});
        a.v = td(cv, {3, hd, H, B}, {4, 3 * 4, 3 * hd * 4, 3 * hd * H * 4});
        a.mask = nullptr;
        a.scale = 0.125f;
        a.out = out;
        a.hd = hd, a.P = 3, a.H = H, a.n = 1, a.B = B;
        cases.push_back({"cross_p3", a});
    }
    for (auto & c : cases) {
        const bool vvec = c.a.v.nb[1] % 16 == 0 && c.a.v.nb[1] >= 16 * ((c.a.P + 3) / 4);
        auto launch = [&](AttnArgs a) {
            const dim3 grid(H, 1, B);
            const bool pf = a.P <= (vvec ? 64 * ATTN_UV : 16 * ATTN_UV);
            if (vvec && pf) hipLaunchKernelGGL((k_attn_decode_rows<1, true, true>), grid, dim3(ATTN_THREADS), 0, be.stream, a);
            else if (vvec) hipLaunchKernelGGL((k_attn_decode_rows<1, true, false>), grid, dim3(ATTN_THREADS), 0, be.stream, a);
            else hipLaunchKernelGGL((k_attn_decode_rows<1, false, true>), grid, dim3(ATTN_THREADS), 0, be.stream, a);
        };
        for (int w = 0; w < 5; ++w) launch(c.a);
        TTS_HIP_CHECK(hipStreamSynchronize(be.stream));
        std::vector<double> ev, span, pa, pb, pc;
        for (int r = 0; r < 20; ++r) {
            TTS_HIP_CHECK(hipMemsetAsync(ts, 0, nts * 8, be.stream));
            AttnArgs a = c.a;
            a.ts = ts;
            TTS_HIP_CHECK(hipEventRecord(e0, be.stream));
            launch(a);
            TTS_HIP_CHECK(hipEventRecord(e1, be.stream));
            TTS_HIP_CHECK(hipStreamSynchronize(be.stream));
            float ms;
            TTS_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            ev.push_back(1000.0 * ms);
            std::vector<unsigned long long> h(nts);
            TTS_HIP_CHECK(hipMemcpy(h.data(), ts, nts * 8, hipMemcpyDeviceToHost));
            unsigned long long tmin = ~0ull, tmax = 0;
            std::vector<double> A, Bv, C;
            for (size_t w = 0; w + 8 <= nts; w += 8) {
                if (!h[w]) continue;
                tmin = std::min(tmin, h[w]);
                tmax = std::max(tmax, h[w + 4]);
                A.push_back((h[w + 1] - h[w]) / 100.0);
                Bv.push_back((h[w + 3] - h[w + 1]) / 100.0);
                C.push_back((h[w + 4] - h[w + 3]) / 100.0);
            }
            span.push_back((tmax - tmin) / 100.0);
            pa.push_back(med(A)), pb.push_back(med(Bv)), pc.push_back(med(C));
        }
        printf("{\"case\":\"%s\",\"P\":%d,\"vvec\":%d,\"event_us\":%.2f,\"span_us\":%.2f,\"scores_us\":%.2f,\"softmax_us\":%.2f,\"pv_us\":%.2f}\n",
               c.name, c.a.P, (int)vvec, med(ev), med(span), med(pa), med(pb), med(pc));
    }
    return 0;
}
