// Deterministic synthetic weights (no checkpoints offline: BASELINE.md §3).  Seed per tensor =
// 0x5EED ^ tensor_index; values are a counter-based hash, so any byte can be regenerated
// independently (and in parallel) on the host.
#pragma once

#include <cstddef>
#include <cstdint>

namespace tts {

uint64_t synth_hash(uint64_t seed, uint64_t i);
// uniform in [-scale, scale) + offset
void synth_f32(float * dst, size_t n, uint64_t seed, float scale, float offset);
void synth_f16(uint16_t * dst, size_t n, uint64_t seed, float scale);
// Valid Q4_K blocks with random nibbles / 6-bit scales / mins and d, dmin chosen so that the
// dequantized weights are roughly zero-mean with std ~ `std`.
void synth_q4_K(void * dst, int64_t rows, int64_t K, uint64_t seed, float std);
void synth_q8_0(void * dst, int64_t rows, int64_t K, uint64_t seed, float std);
void synth_fill(int type, void * dst, int64_t rows, int64_t K, uint64_t seed, float std);

}  // namespace tts
