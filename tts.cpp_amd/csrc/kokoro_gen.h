// Internal: the Kokoro generator builder shared by the standalone generator runner (kokoro.cpp)
// and the full Kokoro runner (kokoro_model.cpp), which builds it into its own graph the way
// kokoro_runner::build_kokoro_graph calls build_generator (src/models/kokoro/model.cpp:1237).
#pragma once

#include <cstring>
#include <string>

#include "graph.h"
#include "tts_runners.h"

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

// Which GGUF tensors an F16 Kokoro file holds as F16: kokoro_is_f16_compatible
// (/root/reference/examples/quantize/quantize_impl.cpp:14-18; `quantize -qt F16 -nqf` converts every
// such tensor, the quantizable ALBERT / LSTM / duration ones included).  Only matrices and conv
// kernels (>= 2-D) are converted here: the 1-D f16-compatible tensors of the real file (LSTM initial
// states) are zeros either way, and constants built by post_load_assign are not in the file.
inline bool kokoro_f16_tensor(const std::string & name, int64_t ne1) {
    auto has = [&](const char * w) { return name.find(w) != std::string::npos; };
    auto ends = [&](const char * w) {
        const size_t n = strlen(w);
        return name.size() >= n && name.compare(name.size() - n, n, w) == 0;
    };
    return ne1 > 0 && !has("voice_tensors") && !has("bias") && !has("gamma") && !has("beta") && !has("alpha") && !ends("embd") &&
           !ends("norm");
}

// Host upload of one synthetic weight as its tensor type (F32, or F16 rounded to nearest even).
bool kokoro_upload_weight(const tts_backend_iface & be, tts_tensor * t, const float * host, size_t n);
// f32 values of a weight (F16 widened) into dst; returns nelements * 4 (0 on a failed read)
uint64_t kokoro_read_weight(const tts_backend_iface & be, const tts_tensor * t, float * dst, uint64_t cap);

}  // namespace tts
