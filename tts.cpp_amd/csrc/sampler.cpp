// Seeded restatement of TTS.cpp's host sampler (sampler::sample / softmax / topk / topp / max,
// /root/reference/src/sampler.cpp:3-204) -- the runners' host sampling path and the reference the
// device sampler (k_sample.hip) is checked against.  The reference's arithmetic is kept step for
// step; what differs is documented in tts_hip.h: the per-call generator is seeded from
// (seed, prompt, call) instead of std::random_device, expf is the correctly rounded value, and
// top-k ties go to the lower index.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "tts_hip.h"

extern "C" void tts_sampling_default(tts_sampling * c) {
    memset(c, 0, sizeof(*c));
    c->temperature = 1.0f;
    c->top_p = 1.0f;
    c->repetition_penalty = 1.0f;
    c->top_k = 50;
    c->do_sample = 1;
    c->seed = 0x5EED;
}

extern "C" int tts_sampling_device_ok(const tts_sampling * cfg, int32_t V) {
    return V <= 4096 || !cfg->do_sample || (cfg->top_k > 0 && cfg->top_k <= 64 && cfg->top_p >= 1.0f);
}

extern "C" uint32_t tts_sampler_call_seed(uint64_t seed, int32_t stream, int64_t call) {
    uint64_t z = seed ^ ((uint64_t)(uint32_t)stream << 40) ^ ((uint64_t)call * 0x9E3779B97F4A7C15ull);
    z += 0x9E3779B97F4A7C15ull;  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(1 + z % 2147483646ull);
}

namespace {

inline float cr_expf_host(float x) { return (float)std::exp((double)x); }

}  // namespace

extern "C" int tts_sampler_sample(const tts_sampling * cfg, const float * logits, int32_t NH, int32_t V, uint32_t call_seed, int32_t * last,
                                  int32_t * count, int32_t * out) {
    if (!cfg || !logits || !out || NH <= 0 || V <= 0) return TTS_STATUS_BAD_ARG;
    const bool rep = cfg->repetition_penalty != 1.0f;
    if (rep && (!last || !count)) return TTS_STATUS_BAD_ARG;
    const bool temp = cfg->temperature != 1.0f;
    // v / pow(penalty, count): float / double in double, rounded to float (sampler.cpp:97-99)
    auto penal = [&](int h, int i, float v) -> float {
        if (rep && last[h] == i) return (float)((double)v / std::pow((double)cfg->repetition_penalty, (double)(uint32_t)count[h]));
        return v;
    };
    // sampler::max (:185-204): first maximum of the penalised logits
    std::vector<int32_t> maxi(NH);
    for (int h = 0; h < NH; ++h) {
        float mx = -INFINITY;
        int32_t id = 0;
        for (int i = 0; i < V; ++i) {
            const float v = penal(h, i, logits[(size_t)h * V + i]);
            if (v > mx) mx = v, id = i;
        }
        maxi[h] = id;
    }
    if (!cfg->do_sample) {
        for (int h = 0; h < NH; ++h) out[h] = maxi[h];
        return 0;
    }
    // working copy: the reference's softmax writes probabilities into `logits`
    std::vector<float> lw(logits, logits + (size_t)NH * V);
    std::vector<std::vector<int32_t>> picks;
    std::vector<float> max_head_probs;
    bool nucleus = false;
    // softmax (:71-104) over picks (or the whole vocabulary when there are none)
    auto softmax = [&]() {
        const bool use = !picks.empty();
        for (int h = 0; h < NH; ++h) {
            float * row = lw.data() + (size_t)h * V;
            float cumsum = 0.0f;
            float max_val = row[maxi[h]];
            if (rep && last[h] == maxi[h]) max_val = (float)((double)max_val / std::pow((double)cfg->repetition_penalty, (double)(uint32_t)count[h]));
            if (temp) max_val /= cfg->temperature;
            const int n = use ? (int)picks[h].size() : V;
            for (int j = 0; j < n; ++j) {
                const int ii = use ? picks[h][j] : j;
                float v = penal(h, ii, row[ii]);
                if (temp) v /= cfg->temperature;
                v = cr_expf_host(v - max_val);
                cumsum += v;
                row[ii] = v;
            }
            for (int j = 0; j < n; ++j) {
                const int ii = use ? picks[h][j] : j;
                row[ii] = row[ii] / cumsum;
            }
        }
    };
    // a head's order: key descending, then index ascending
    auto sorted = [&](int h, bool penalised) {
        std::vector<int32_t> idx(V);
        std::iota(idx.begin(), idx.end(), 0);
        const float * row = lw.data() + (size_t)h * V;
        std::vector<float> key(V);
        for (int i = 0; i < V; ++i) key[i] = penalised ? penal(h, i, row[i]) : row[i];
        std::sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return key[a] > key[b] || (key[a] == key[b] && a < b); });
        return idx;
    };
    bool performed_softmax = false;
    if (cfg->top_p < 1.0f) {
        softmax();
        performed_softmax = true;
    }
    if (cfg->top_k > 0 && cfg->top_k < V) {  // topk (:139-183)
        picks.clear();
        for (int h = 0; h < NH; ++h) {
            std::vector<int32_t> idx = sorted(h, !performed_softmax);
            idx.resize(cfg->top_k);
            picks.push_back(std::move(idx));
        }
        nucleus = true;
    }
    if (cfg->top_p >= 1.0f) {
        softmax();
        performed_softmax = true;
    }
    if (cfg->top_p < 1.0f) {  // topp (:106-137)
        if (picks.empty())
            for (int h = 0; h < NH; ++h) picks.push_back(sorted(h, false));
        for (int h = 0; h < NH; ++h) {
            float prob_sum = 0.0f;
            int trim_to = -1;
            for (size_t ii = 0; ii < picks[h].size(); ++ii) {
                prob_sum += lw[(size_t)h * V + picks[h][ii]];
                if (prob_sum >= cfg->top_p) {
                    trim_to = (int)ii + 1;
                    break;
                }
            }
            max_head_probs.push_back(std::min(prob_sum, cfg->top_p));
            if (trim_to > 0) picks[h].resize(trim_to);
        }
        nucleus = true;
    }
    // draws (:45-61): one per head, in head order
    std::minstd_rand gen(call_seed);
    std::uniform_real_distribution<float> dist(0.0f, 1.0f);
    for (int h = 0; h < NH; ++h) {
        const float assignment = cfg->top_p < 1.0f ? dist(gen) * max_head_probs[h] : dist(gen);
        float cumulative = 0.0f;
        const int n = nucleus ? (int)picks[h].size() : V;
        for (int j = 0; j < n; ++j) {
            const int ii = nucleus ? picks[h][j] : j;
            cumulative += lw[(size_t)h * V + ii];
            if (assignment <= cumulative || j >= n - 1) {
                if (rep) {
                    if (last[h] != ii) count[h] = 0;
                    last[h] = ii;
                    count[h] += 1;
                }
                out[h] = ii;
                break;
            }
        }
    }
    return 0;
}
