// Internal definitions shared by the HIP backend, the graph builder and the runners.
// Block formats follow ggml's (Q4_K: ggml-common.h block_q4_K, 144 B / 256 weights;
// Q8_0: block_q8_0, 34 B / 32 weights) so that weight bytes produced by TTS.cpp's loader
// (/root/reference/src/models/loaders.cpp:79-88) are consumed unchanged.
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/tts_hip.h"

#ifdef __HIPCC__
#define TTS_HD __host__ __device__ __forceinline__
#else
#define TTS_HD inline
#endif

namespace tts {

constexpr int QK_K = 256;
constexpr int QK8_0 = 32;

struct block_q4_K {
    uint16_t d;
    uint16_t dmin;
    uint8_t scales[12];
    uint8_t qs[QK_K / 2];
};
static_assert(sizeof(block_q4_K) == 144, "q4_K block");

struct block_q8_0 {
    uint16_t d;
    int8_t qs[QK8_0];
};
static_assert(sizeof(block_q8_0) == 34, "q8_0 block");

// Host fp16 conversion: same bit-exact algorithm as ggml_compute_fp{16,32}_to_fp{32,16}.
inline float fp16_to_fp32_host(uint16_t h) {
    const uint32_t w = (uint32_t)h << 16;
    const uint32_t sign = w & 0x80000000u;
    const uint32_t two_w = w + w;
    uint32_t nb = (two_w >> 4) + (0xE0u << 23);
    float normalized;
    memcpy(&normalized, &nb, 4);
    normalized *= 0x1.0p-112f;
    uint32_t db = (two_w >> 17) | (126u << 23);
    float denorm;
    memcpy(&denorm, &db, 4);
    denorm -= 0.5f;
    uint32_t rb;
    if (two_w < (1u << 27)) memcpy(&rb, &denorm, 4);
    else memcpy(&rb, &normalized, 4);
    rb |= sign;
    float r;
    memcpy(&r, &rb, 4);
    return r;
}

inline uint16_t fp32_to_fp16_host(float f) {
    float base = (__builtin_fabsf(f) * 0x1.0p+112f) * 0x1.0p-110f;
    uint32_t w;
    memcpy(&w, &f, 4);
    const uint32_t shl1_w = w + w;
    const uint32_t sign = w & 0x80000000u;
    uint32_t bias = shl1_w & 0xFF000000u;
    if (bias < 0x71000000u) bias = 0x71000000u;
    uint32_t bb = (bias >> 1) + 0x07800000u;
    float bf;
    memcpy(&bf, &bb, 4);
    base = bf + base;
    uint32_t bits;
    memcpy(&bits, &base, 4);
    const uint32_t exp_bits = (bits >> 13) & 0x00007C00u;
    const uint32_t mantissa_bits = bits & 0x00000FFFu;
    const uint32_t nonsign = exp_bits + mantissa_bits;
    return (uint16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

}  // namespace tts
