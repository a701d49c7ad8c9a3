// Public entry points of the MI355X ggml backend adapter (ggml-tts-hip.cpp), the HIP counterpart
// of ggml-metal.h's ggml_backend_metal_init / ggml_backend_metal_buffer_type that TTS.cpp's 14
// `#ifdef GGML_USE_METAL` selection sites call.  Built only inside the ggml fork
// (make ggml-adapter TTS_GGML_DIR=<fork checkout>), linked against libtts_hip.so.
#pragma once

#include "ggml-backend.h"

#ifdef __cplusplus
extern "C" {
#endif

// registry: one device per visible HIP device (ggml_backend_reg_i)
ggml_backend_reg_t ggml_backend_tts_hip_reg(void);
// device index -> backend (one HIP stream) / its device-memory buffer type
ggml_backend_t ggml_backend_tts_hip_init(int device);
ggml_backend_buffer_type_t ggml_backend_tts_hip_buffer_type(int device);
bool ggml_backend_is_tts_hip(ggml_backend_t backend);
// device index from TTS_HIP_DEVICE (default 0): what the selection sites pass
int ggml_backend_tts_hip_default_device(void);

// The two CPU callbacks on TTS.cpp's hot path that have device restatements (util.cpp:140-200:
// uv_noise_compute, cfg_scale).  ggml_map_custom2/3 only carry a function pointer; the adapter
// recognises these through weak references to the callbacks, or through this registration when
// the callbacks are not link-visible to the adapter (kind: 1 = uv_noise_compute, 2 = cfg_scale).
void ggml_backend_tts_hip_register_custom(const void * fn, int kind);

#ifdef __cplusplus
}
#endif
