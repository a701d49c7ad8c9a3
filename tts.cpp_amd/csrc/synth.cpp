#include "synth.h"

#include <cstring>
#include <thread>
#include <vector>

#include "common.h"

namespace tts {

uint64_t synth_hash(uint64_t seed, uint64_t i) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + i + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline float u01(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

template <typename F>
static void parallel_for(size_t n, F f) {
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0) nt = 1;
    if (nt > 16) nt = 16;
    if (n < 65536 || nt == 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    size_t chunk = (n + nt - 1) / nt;
    for (unsigned t = 0; t < nt; ++t) {
        size_t a = t * chunk, b = std::min(n, a + chunk);
        if (a >= b) break;
        th.emplace_back([=]() { f(a, b); });
    }
    for (auto & x : th) x.join();
}

void synth_f32(float * dst, size_t n, uint64_t seed, float scale, float offset) {
    parallel_for(n, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) dst[i] = offset + scale * (2.0f * u01(synth_hash(seed, i)) - 1.0f);
    });
}

void synth_f16(uint16_t * dst, size_t n, uint64_t seed, float scale) {
    parallel_for(n, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) dst[i] = fp32_to_fp16_host(scale * (2.0f * u01(synth_hash(seed, i)) - 1.0f));
    });
}

void synth_q4_K(void * dst, int64_t rows, int64_t K, uint64_t seed, float std) {
    const int64_t nblk = rows * (K / QK_K);
    block_q4_K * b = (block_q4_K *)dst;
    // weight = d*sc*q - dmin*m, q ~ U{0..15}, sc ~ U{32..63}, m ~ U{32..63}:
    // mean ~ d*47.5*7.5 - dmin*47.5 = 0 for dmin = 7.5 d; std ~ d*47.5*4.6
    const float d = std / (47.5f * 4.61f);
    parallel_for((size_t)nblk, [&](size_t a, size_t e) {
        for (size_t i = a; i < e; ++i) {
            block_q4_K & x = b[i];
            const uint64_t h0 = synth_hash(seed, i * 20 + 0);
            const float jitter = 0.75f + 0.5f * u01(h0);
            x.d = fp32_to_fp16_host(d * jitter);
            x.dmin = fp32_to_fp16_host(7.5f * d * jitter);
            uint8_t sc[8], mn[8];
            const uint64_t h1 = synth_hash(seed, i * 20 + 1);
            for (int j = 0; j < 8; ++j) {
                sc[j] = 32 + ((h1 >> (j * 5)) & 31);
                mn[j] = 32 + ((h1 >> (40 + j * 3)) & 7) * 4 + ((h0 >> (j * 2)) & 3);
            }
            // pack 6-bit scales/mins exactly as quantize_row_q4_K_ref does
            memset(x.scales, 0, 12);
            for (int j = 0; j < 8; ++j) {
                const uint8_t ls = sc[j] & 63, lm = mn[j] & 63;
                if (j < 4) {
                    x.scales[j] = ls;
                    x.scales[j + 4] = lm;
                } else {
                    x.scales[j + 4] = (ls & 0xF) | ((lm & 0xF) << 4);
                    x.scales[j - 4] |= ((ls >> 4) << 6);
                    x.scales[j - 0] |= ((lm >> 4) << 6);
                }
            }
            for (int k = 0; k < 16; ++k) {
                const uint64_t h = synth_hash(seed, i * 20 + 2 + k);
                memcpy(x.qs + 8 * k, &h, 8);
            }
        }
    });
}

void synth_q8_0(void * dst, int64_t rows, int64_t K, uint64_t seed, float std) {
    const int64_t nblk = rows * (K / QK8_0);
    block_q8_0 * b = (block_q8_0 *)dst;
    const float d = std / 73.6f;  // U{-127..127} has std ~73.6
    parallel_for((size_t)nblk, [&](size_t a, size_t e) {
        for (size_t i = a; i < e; ++i) {
            const uint64_t h0 = synth_hash(seed, i * 5);
            b[i].d = fp32_to_fp16_host(d * (0.75f + 0.5f * u01(h0)));
            for (int k = 0; k < 4; ++k) {
                uint64_t h = synth_hash(seed, i * 5 + 1 + k);
                for (int j = 0; j < 8; ++j) {
                    int v = (int)((h >> (8 * j)) & 0xFF) - 128;
                    if (v == -128) v = -127;
                    b[i].qs[k * 8 + j] = (int8_t)v;
                }
            }
        }
    });
}

void synth_fill(int type, void * dst, int64_t rows, int64_t K, uint64_t seed, float std) {
    switch (type) {
        case TTS_TYPE_Q4_K: synth_q4_K(dst, rows, K, seed, std); break;
        case TTS_TYPE_Q8_0: synth_q8_0(dst, rows, K, seed, std); break;
        case TTS_TYPE_F16: synth_f16((uint16_t *)dst, (size_t)(rows * K), seed, std * 1.7320508f); break;
        default: synth_f32((float *)dst, (size_t)(rows * K), seed, std * 1.7320508f, 0.0f); break;
    }
}

}  // namespace tts
