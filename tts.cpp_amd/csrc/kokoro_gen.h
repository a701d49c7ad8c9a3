// Internal: the Kokoro generator builder shared by the standalone generator runner (kokoro.cpp)
// and the full Kokoro runner (kokoro_model.cpp), which builds it into its own graph the way
// kokoro_runner::build_kokoro_graph calls build_generator (src/models/kokoro/model.cpp:1237).
#pragma once

#include "graph.h"

struct tts_kokoro_gen;

namespace tts {

// build_sin_gen + build_generator into c: x [C, T] (channel fastest), f0 [T] or [T, 1], style
// [style_dim]; returns the PCM node [300 T] and registers the generator's host inputs on k.
// device_draws: the uv_noise map draws its uniforms on the device (counter hash) instead of
// reading host draws; kokoro_gen_set_inputs must then be given rand = NULL.
tts_tensor * kokoro_gen_build(tts_kokoro_gen * k, tg::context & c, tts_tensor * x, tts_tensor * f0, tts_tensor * style, int64_t T,
                              bool device_draws);
// After tg::alloc_graph: fill and upload those inputs (uv_noise data block, window envelope);
// rand = [harmonic_num + 1][300 T] uniform draws, or NULL for a graph built with device_draws.
int kokoro_gen_set_inputs(tts_kokoro_gen * k, int64_t T, const float * rand);

}  // namespace tts
