/*
 * tts_runners.h — C-ABI of the host-side runners that drive the backend with TTS.cpp's graphs.
 *
 * The runners mirror the reference's runner interface (parler_tts_runner::decode /
 * generate_from_batch, /root/reference/src/models/parler/model.cpp:648-693, 762-792) over a
 * tts_backend_iface, so the same graphs run on the HIP backend (product) or on the CPU oracle
 * (tests and bench cpu_baseline only).  Weights are deterministic synthetic tensors of the exact
 * shapes/types of the named config (no checkpoints offline: BASELINE.md §3).
 */
#ifndef TTS_RUNNERS_H
#define TTS_RUNNERS_H

#include "tts_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parler-TTS decoder config (defaults = Parler-TTS mini v1, src/models/parler/model.h:67-81). */
typedef struct tts_parler_config {
    int32_t n_layers;        /* 24 */
    int32_t hidden_size;     /* 1024 */
    int32_t n_attn_heads;    /* 16 */
    int32_t ffn_size;        /* 4096 */
    int32_t n_output_heads;  /* 9 codebooks */
    int32_t output_vocab;    /* 1088 */
    int32_t audio_vocab;     /* 1024 */
    int32_t max_ctx;         /* 4096 (KV capacity) */
    int32_t n_encode;        /* 3 ("female voice" T5 tokens) */
    int32_t prompt_vocab;    /* 32128 (T5) */
    int32_t max_positions;   /* 4102 */
    int32_t weight_type;     /* TTS_TYPE_Q4_K for config 3 */
    int32_t head_type;       /* TTS_TYPE_F32 (heads unquantized by default) */
    int32_t use_cross_attn;  /* 1 */
    int32_t batch;           /* independent prompts stepped in lockstep (1 = reference graph) */
    int32_t eos_token;       /* 1024 */
    int32_t bos_token;       /* 1025 */
    uint64_t seed;           /* synthetic weight seed base (0x5EED) */
    uint64_t arena_bytes;    /* compute arena (0 = default 256 MiB) */
    int32_t debug_no_reuse;  /* 1 = every node gets its own arena memory (node dumps) */
    int32_t pad_;
} tts_parler_config;

typedef struct tts_parler tts_parler;

void tts_parler_default_config(tts_parler_config * cfg);
tts_parler * tts_parler_create(const tts_backend_iface * be, const tts_parler_config * cfg);
void tts_parler_free(tts_parler * p);
/* Resets positions / EOS state (KV contents become unreachable). */
void tts_parler_reset(tts_parler * p);
/* Text-prompt pass: tokens [batch][n] (parler batch_from_sentence path). */
int tts_parler_prefill(tts_parler * p, const int32_t * tokens, int32_t n);
/* One prompt pass over `batch` prompts of different lengths from an empty cache (a ragged lock-step batch):
 * tokens [batch][n_max], prompt b = its first lens[b] ids.  Later steps decode every prompt in lockstep, each at
 * its own position with its own mask (TTS.cpp runs one prompt per runner: parler_tts_runner::prepare_post_load /
 * generate, src/models/parler/model.cpp:838-858; this batches them). */
int tts_parler_prefill_ragged(tts_parler * p, const int32_t * tokens, const int32_t * lens, int32_t n_max);
/* One AR decode step: audio tokens [batch][n_output_heads] -> logits [batch][n_output_heads][vocab]. */
int tts_parler_decode(tts_parler * p, const int32_t * audio_tokens, float * logits);
/* Greedy generation loop (generate_from_batch with sampler::max): runs n_steps AR steps after the
 * current position and writes sampled tokens [batch][n_steps][n_output_heads]. */
int tts_parler_generate(tts_parler * p, int32_t n_steps, int32_t * tokens_out);
/* 1 (default): greedy sampling stays on the device when the backend offers greedy_step (the host
 * never waits per step); 0: logits are read back and sampled on the host every step. */
void tts_parler_set_device_sampling(tts_parler * p, int32_t on);
/* Seeded sampling (sampler::sample, include/tts_hip.h tts_sampling) for tts_parler_generate; NULL =
 * greedy (the default).  Prompt b of the batch draws from its own generator (stream b). */
void tts_parler_set_sampling(tts_parler * p, const tts_sampling * cfg);
/* Timing harness only (bench.py's cpu_baseline): continue as if `position` tokens were decoded. */
int tts_parler_set_position(tts_parler * p, int32_t position);
int32_t tts_parler_position(const tts_parler * p);
/* Host time per phase summed over steps (us): build graph, allocate, set inputs, compute enqueue,
 * wait for logits.  Returns the step count; reset zeroes the sums. */
int64_t tts_parler_host_stats(tts_parler * p, double * us5, int reset);
/* Nodes in the last step graph and bytes of the compute arena it used. */
int32_t tts_parler_last_graph_nodes(const tts_parler * p);
/* The last step graph's node list (valid until the next step is prepared). */
tts_tensor * const * tts_parler_graph(const tts_parler * p, int32_t * n_nodes);
uint64_t tts_parler_weight_bytes(const tts_parler * p);
/* Weight introspection for tests (every weight in declaration order): name, ne[4], ggml type and the bytes
 * as the backend stores them (F32 / F16 as ggml's); returns the byte size (dst NULL or too small: size only). */
int32_t tts_parler_n_weights(const tts_parler * p);
uint64_t tts_parler_weight(tts_parler * p, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst, uint64_t cap);
/* Debug: copy a named node of the last graph to host (returns bytes, 0 if not found). */
uint64_t tts_parler_get_node(tts_parler * p, const char * name, void * dst, uint64_t cap);
/* Debug: node i of the last graph: op / type / ne; copies its bytes when contiguous (returns size). */
uint64_t tts_parler_node(tts_parler * p, int32_t i, int32_t * op, int32_t * type, int64_t * ne, void * dst, uint64_t cap);

/* Orpheus-3B decoder config (defaults = orpheus_model, src/models/orpheus/model.h:31-46; rope
 * factors from Llama-3.2 rope scaling as py-gguf/tts_encoders/orpheus_gguf_encoder.py:144-173). */
typedef struct tts_orpheus_config {
    int32_t n_layers;         /* 28 */
    int32_t hidden_size;      /* 3072 */
    int32_t n_attn_heads;     /* 24 */
    int32_t n_kv_attn_heads;  /* 8 (K/V stored repeat-interleaved x3, orpheus_build_kv_store) */
    int32_t head_size;        /* 128 */
    int32_t ffn_size;         /* 8192 */
    int32_t vocab_size;       /* 156940 */
    int32_t max_ctx;          /* 1024 + 2100 (KV capacity) */
    int32_t weight_type;      /* TTS_TYPE_Q4_K for config 5 (all matrices incl. embedding and head) */
    int32_t batch;            /* independent prompts stepped in lockstep (1 = reference graph) */
    uint64_t seed;            /* synthetic weight seed base (0x5EED) */
    uint64_t arena_bytes;     /* compute arena (0 = default 512 MiB) */
    float rope_theta;         /* 500000 */
    float rope_factor;        /* 32 */
    float rope_low_freq_factor;   /* 1 */
    float rope_high_freq_factor;  /* 4 */
    int32_t rope_original_ctx;    /* 8192 */
    int32_t pad_;
} tts_orpheus_config;

typedef struct tts_orpheus tts_orpheus;

void tts_orpheus_default_config(tts_orpheus_config * cfg);
tts_orpheus * tts_orpheus_create(const tts_backend_iface * be, const tts_orpheus_config * cfg);
void tts_orpheus_free(tts_orpheus * p);
void tts_orpheus_reset(tts_orpheus * p);
/* Prompt pass (orpheus_runner::decode over batch_from_sentence): tokens [batch][n]; logits of the last
 * token [batch][vocab] when `logits` is not NULL. */
int tts_orpheus_prefill(tts_orpheus * p, const int32_t * tokens, int32_t n, float * logits);
/* One AR step: tokens [batch] -> logits [batch][vocab]. */
int tts_orpheus_decode(tts_orpheus * p, const int32_t * tokens, float * logits);
/* Greedy loop (generate_from_batch, sampler::max): feeds first_tokens [batch], then each step's samples;
 * writes tokens [batch][n_steps].  Samples stay on the device when the backend offers greedy_step. */
int tts_orpheus_generate(tts_orpheus * p, const int32_t * first_tokens, int32_t n_steps, int32_t * tokens_out);
/* Seeded sampling for tts_orpheus_generate (NULL = greedy, the default); prompt b = stream b. */
void tts_orpheus_set_sampling(tts_orpheus * p, const tts_sampling * cfg);
int32_t tts_orpheus_position(const tts_orpheus * p);
int32_t tts_orpheus_last_graph_nodes(const tts_orpheus * p);
uint64_t tts_orpheus_weight_bytes(const tts_orpheus * p);
/* Weight introspection for tests, as tts_parler_weight. */
int32_t tts_orpheus_n_weights(const tts_orpheus * p);
uint64_t tts_orpheus_weight(tts_orpheus * p, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst, uint64_t cap);
tts_tensor * const * tts_orpheus_graph(const tts_orpheus * p, int32_t * n_nodes);

/* Dia-1.6B config (defaults = dia_model, src/models/dia/model.h:62-85; Q8_0 weights for config 4,
 * F32 heads).  Classifier-free guidance runs a (conditioned, unconditioned) pair as the graph batch. */
typedef struct tts_dia_config {
    int32_t n_output_heads;             /* 9 */
    int32_t n_encoder_layers;           /* 12 */
    int32_t n_decoder_layers;           /* 18 */
    int32_t encoder_hidden_size;        /* 1024 */
    int32_t decoder_hidden_size;        /* 2048 */
    int32_t encoder_attn_heads;         /* 16 */
    int32_t decoder_attn_heads;         /* 16 */
    int32_t decoder_query_heads;        /* 4 (GQA: 4 K/V heads, repeat-interleaved into the cache) */
    int32_t head_size;                  /* 128 */
    int32_t encoder_ffn_size;           /* 4096 */
    int32_t decoder_ffn_size;           /* 8192 */
    int32_t output_vocab_size;          /* 1028 */
    int32_t encoder_vocab_size;         /* 256 (byte tokens) */
    int32_t max_generation_size;        /* 3072 */
    int32_t max_encoder_context_length; /* 1024 */
    int32_t weight_type;                /* TTS_TYPE_Q8_0 */
    int32_t head_type;                  /* TTS_TYPE_F32 */
    float cfg_scale;                    /* 3.0 */
    uint64_t seed;                      /* synthetic weight seed base (0x5EED) */
    uint64_t arena_bytes;               /* compute arena (0 = default 2 GiB: the encoder step's 1024 x 1024 scores) */
} tts_dia_config;

typedef struct tts_dia tts_dia;

void tts_dia_default_config(tts_dia_config * cfg);
tts_dia * tts_dia_create(const tts_backend_iface * be, const tts_dia_config * cfg);
void tts_dia_free(tts_dia * p);
/* Encoder step + first decoder step (dia_runner::decode with encoder_step): text [2][max_encoder_context_length]
 * (conditioned row, unconditioned row), n_text real tokens, audio [n_output_heads]; logits [n_output_heads][vocab]
 * after cfg_scale. */
int tts_dia_prefill(tts_dia * p, const int32_t * text, int32_t n_text, const int32_t * audio, float * logits);
/* One decoder step: audio [n_output_heads] -> logits [n_output_heads][vocab]. */
int tts_dia_decode(tts_dia * p, const int32_t * audio, float * logits);
/* Greedy decode loop: feeds first_audio [n_output_heads], then each step's per-head argmax of the CFG
 * logits (both CFG rows); writes tokens [n_steps][n_output_heads].  Device-resident when the backend
 * offers plans + greedy_step. */
int tts_dia_generate(tts_dia * p, const int32_t * first_audio, int32_t n_steps, int32_t * tokens_out);
/* Seeded sampling of the CFG heads for tts_dia_generate (NULL = greedy, the default). */
void tts_dia_set_sampling(tts_dia * p, const tts_sampling * cfg);
int32_t tts_dia_position(const tts_dia * p);
int32_t tts_dia_last_graph_nodes(const tts_dia * p);
uint64_t tts_dia_weight_bytes(const tts_dia * p);
/* Weight introspection for tests, as tts_parler_weight. */
int32_t tts_dia_n_weights(const tts_dia * p);
uint64_t tts_dia_weight(tts_dia * p, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst, uint64_t cap);
tts_tensor * const * tts_dia_graph(const tts_dia * p, int32_t * n_nodes);

/* DAC decoder (codec tokens -> PCM): dac_runner::run / build_dac_graph,
 * /root/reference/src/decoder/dac_model.cpp:139-212.  Defaults = DAC 44.1 kHz as used by
 * Parler-TTS mini v1 (9 codebooks x 1024 x 8, latent 1024, decoder 1536, rates 8,8,4,2: 512
 * samples per latent frame). */
typedef struct tts_dac_config {
    int32_t n_codebooks;   /* 9 */
    int32_t codebook_size; /* 1024 */
    int32_t codebook_dim;  /* 8 */
    int32_t latent_dim;    /* 1024 */
    int32_t decoder_dim;   /* 1536; halves per layer */
    int32_t n_layers;      /* 4 */
    int32_t rates[8];      /* 8, 8, 4, 2 (upsampling stride per layer) */
    int32_t max_frames;    /* latent frames per decode call (arena sizing) */
    int32_t pad_;
    uint64_t seed;         /* synthetic weight seed base */
    uint64_t arena_bytes;  /* compute arena (0 = sized from max_frames) */
} tts_dac_config;

typedef struct tts_dac tts_dac;
void tts_dac_default_config(tts_dac_config * cfg);
tts_dac * tts_dac_create(const tts_backend_iface * be, const tts_dac_config * cfg);
void tts_dac_free(tts_dac * d);
/* codes: [T][n_codebooks] int32 (time-major, dac_build_audio_inputs' view); pcm: [T * hop] f32. */
int tts_dac_decode(tts_dac * d, const int32_t * codes, int32_t T, float * pcm);
int64_t tts_dac_hop(const tts_dac * d);
int32_t tts_dac_last_graph_nodes(const tts_dac * d);
/* Weight introspection for tests, as tts_parler_weight. */
int32_t tts_dac_n_weights(const tts_dac * d);
uint64_t tts_dac_weight(tts_dac * d, int32_t i, char * name, uint64_t name_cap, int64_t * ne, int32_t * type, void * dst, uint64_t cap);
/* Batched decode of nb prompts of T frames each (a serving-side layout; TTS.cpp decodes one prompt per
 * dac_runner::run): ONE graph over nb * T + (nb - 1) * gap frames, the gaps zeroed before every conv that
 * reaches across them, so each prompt's PCM is bit-identical to tts_dac_decode of that prompt.
 * codes: [nb][T][n_codebooks]; pcm: [nb][T * hop]; gap 0 = tts_dac_min_gap; nb * T + (nb - 1) * gap
 * <= max_frames. */
int tts_dac_decode_batch(tts_dac * d, const int32_t * codes, int32_t nb, int32_t T, int32_t gap, float * pcm);
int64_t tts_dac_min_gap(const tts_dac * d);
/* The last decode's node array (fusion statistics: tts_hip_plan_stats). */
tts_tensor * const * tts_dac_graph(const tts_dac * d, int32_t * n_nodes);

/* SNAC decoder (Orpheus' vocoder: three codebook streams -> 24 kHz PCM): snac_runner::run /
 * build_snac_graph, /root/reference/src/decoder/snac_model.cpp:86-208, with the shared codec layers
 * of general_neural_audio_codec.cpp:133-172 (noise branch, depthwise residual units).  Defaults =
 * SNAC 24 kHz as used by Orpheus-3B (3 heads x 4096 x 8, vq strides 4,2,1, latent 768, decoder
 * 1024, rates 8,8,4,2: 512 samples per finest-head frame). */
typedef struct tts_snac_config {
    int32_t n_heads;       /* 3 (snac.audio_token_channels) */
    int32_t codebook_size; /* 4096 */
    int32_t codebook_dim;  /* 8 */
    int32_t latent_dim;    /* 768 (snac_model::embd) */
    int32_t decoder_dim;   /* 1024; halves per layer */
    int32_t n_layers;      /* 4 */
    int32_t rates[8];      /* 8, 8, 4, 2 (snac_layer_stride_i) */
    int32_t repeats[4];    /* 4, 2, 1 (repeat_interleave of head i, snac_model.h:17) */
    int32_t max_frames;    /* finest-head frames per decode call (arena sizing) */
    int32_t debug_no_reuse; /* 1 = every graph tensor keeps its own arena memory (node taps in tests) */
    uint64_t seed;         /* synthetic weight seed base */
    uint64_t arena_bytes;  /* compute arena (0 = sized from max_frames) */
} tts_snac_config;

typedef struct tts_snac tts_snac;
void tts_snac_default_config(tts_snac_config * cfg);
tts_snac * tts_snac_create(const tts_backend_iface * be, const tts_snac_config * cfg);
void tts_snac_free(tts_snac * d);
/* codes: the heads back to back (head i: T / repeats[i] int32 ids, the inp_tokens layout of
 * snac_runner::set_inputs, snac_model.cpp:161-176); noise: [noise_per_frame * T] f32 (layer l's
 * T * prod(rates[0..l]) normal draws in order, random_normal_gen's role); pcm: [T * hop] f32. */
int tts_snac_decode(tts_snac * d, const int32_t * codes, int32_t T, const float * noise, float * pcm);
int64_t tts_snac_hop(const tts_snac * d);
int64_t tts_snac_noise_per_frame(const tts_snac * d);
int32_t tts_snac_last_graph_nodes(const tts_snac * d);
/* Weight introspection for tests: count, then name / ne[4] / f32 values of weight i (bytes). */
int32_t tts_snac_n_weights(const tts_snac * d);
uint64_t tts_snac_weight(tts_snac * d, int32_t i, char * name, uint64_t name_cap, int64_t * ne, float * dst, uint64_t cap);
/* Debug: bytes of the named node of the last graph ("embd", "in_conv", "up", "convt.<l>",
 * "noise.<l>", "ru.<l>.<r>", "pcm"), copied to dst when cap suffices; 0 if absent. */
uint64_t tts_snac_get_node(tts_snac * d, const char * name, void * dst, uint64_t cap);

/* Kokoro-82M iSTFTNet generator (decoder features + F0 + style -> 24 kHz PCM): build_generator,
 * build_sin_gen, build_noise_block and build_kokoro_generator_res_block,
 * /root/reference/src/models/kokoro/model.cpp:136-244, fed as kokoro_runner::set_inputs feeds it
 * (model.cpp:1256-1262): the uv/noise custom map (util.cpp:140-170) and the squared-window
 * envelope (util.cpp:203-217) are computed on the host, as the reference does on its CPU.
 * Defaults = Kokoro-82M (upsample_initial_channel 512, rates 10,6, kernels 20,12, resblock
 * kernels 3,7,11 x dilations 1,3,5, gen_istft_n_fft 20, hop 5: 300 samples per input frame). */
typedef struct tts_kokoro_gen_config {
    int32_t in_channels;          /* 512 (halves per upsampler) */
    int32_t style_dim;            /* 128 (style_half_size) */
    int32_t n_ups;                /* 2 */
    int32_t up_rates[4];          /* 10, 6 */
    int32_t up_kernels[4];        /* 20, 12 */
    int32_t n_kernels;            /* 3 residual blocks per level */
    int32_t res_kernels[4];       /* 3, 7, 11 */
    int32_t res_dilations[3];     /* 1, 3, 5 */
    int32_t noise_res_kernels[4]; /* 7, 11 */
    int32_t n_fft;                /* 20 (true_n_fft) */
    int32_t hop;                  /* 5 (stft_hop) */
    int32_t harmonic_num;         /* 8 */
    float sample_rate;            /* 24000 */
    float sin_amp;                /* 0.1 */
    float noise_std;              /* 0.003 */
    float voice_threshold;        /* 10 */
    int32_t max_frames;           /* generator input frames per call (arena sizing) */
    int32_t debug_no_reuse;       /* 1 = every node keeps its own arena memory (node dumps) */
    int32_t weight_type;          /* TTS_TYPE_F32 (0) or TTS_TYPE_F16 (1): the F16 GGUF's matrices / conv kernels
                                     (examples/quantize/quantize_impl.cpp:14-18 kokoro_is_f16_compatible) */
    uint64_t seed;                /* synthetic weight seed base */
    uint64_t arena_bytes;         /* compute arena (0 = sized from max_frames) */
} tts_kokoro_gen_config;

typedef struct tts_kokoro_gen tts_kokoro_gen;
void tts_kokoro_gen_default_config(tts_kokoro_gen_config * cfg);
/* NULL when prod(up_rates) * hop != 300 (build_sin_gen's fixed x300 interpolation). */
tts_kokoro_gen * tts_kokoro_gen_create(const tts_backend_iface * be, const tts_kokoro_gen_config * cfg);
void tts_kokoro_gen_free(tts_kokoro_gen * k);
/* x: [T][in_channels] decoder features (channel fastest); f0: [T] Hz; style: [style_dim];
 * rand: [harmonic_num+1][300*T] uniform [0,1) noise draws (random_uniform_gen) or NULL for the
 * runner's own seeded draws; pcm: [300*T] f32. */
int tts_kokoro_gen_run(tts_kokoro_gen * k, const float * x, const float * f0, const float * style, const float * rand, int32_t T,
                       float * pcm);
int64_t tts_kokoro_gen_samples_per_frame(const tts_kokoro_gen * k);
int32_t tts_kokoro_gen_last_graph_nodes(const tts_kokoro_gen * k);
/* Weight introspection for tests: count, then name / ne[4] / f32 values of weight i (bytes). */
int32_t tts_kokoro_gen_n_weights(const tts_kokoro_gen * k);
uint64_t tts_kokoro_gen_weight(tts_kokoro_gen * k, int32_t i, char * name, uint64_t name_cap, int64_t * ne, float * dst, uint64_t cap);
/* Debug: bytes of the named node of the last graph ("sine_source", "har_spec", "up.<i>",
 * "noise_conv.<i>", "noise_res.<i>", "level.<i>", "conv_post", "after_res_gen"), copied to dst
 * when cap suffices; 0 if absent. */
uint64_t tts_kokoro_gen_get_node(tts_kokoro_gen * k, const char * name, void * dst, uint64_t cap);
/* Debug: node i of the last graph: op / type / ne; copies its bytes when contiguous (returns size). */
uint64_t tts_kokoro_gen_node(tts_kokoro_gen * k, int32_t i, int32_t * op, int32_t * type, int64_t * ne, void * dst, uint64_t cap);
/* The last graph's node list (valid until the next run), e.g. for tts_hip_plan_stats. */
tts_tensor * const * tts_kokoro_gen_graph(const tts_kokoro_gen * k, int32_t * n_nodes);

/* Kokoro-82M end to end (phoneme tokens -> 24 kHz PCM): kokoro_duration_runner's graph
 * (ALBERT x n_recurrence, prosody DurationEncoder, duration LSTM + projection -> per-token
 * lengths; src/models/kokoro/model.cpp:938-1047) and kokoro_runner's graph (duration-mask
 * expansion, shared LSTM, F0 / N AdaIN residual stacks, text encoder, decoder blocks, then the
 * generator above; model.cpp:1141-1242), with the host steps between them as kokoro_runner::run /
 * set_inputs do them (model.cpp:1253-1325): read the lengths back, build the [total, n] duration
 * mask, upload.  Defaults = Kokoro-82M (ALBERT 178 x 128 -> 768, 12 heads, ffn 2048, one shared
 * layer x 12; d_model 512; decoder 1024; style 2 x 128).  Synthetic weights. */
typedef struct tts_kokoro_config {
    tts_kokoro_gen_config gen; /* generator (gen.in_channels = last decoder block width, gen.style_dim = style half) */
    int32_t n_vocab;           /* 178 phoneme ids */
    int32_t embd;              /* 128 ALBERT embedding width */
    int32_t hidden;            /* 768 ALBERT hidden */
    int32_t n_heads;           /* 12 */
    int32_t ffn;               /* 2048 */
    int32_t n_layers;          /* 1 (ALBERT's shared layer group) */
    int32_t n_recurrence;      /* 12 */
    int32_t max_context;       /* 512 positions */
    int32_t d_model;           /* 512: duration_hidden_size, text encoder channels */
    int32_t n_dur_layers;      /* 3 DurationEncoder LSTM + AdaLayerNorm layers */
    int32_t max_dur;           /* 50: duration_proj width (and the clamp bound) */
    int32_t te_kernel;         /* 5 */
    int32_t te_depth;          /* 3 */
    int32_t dec_dim;           /* 1024 */
    int32_t asr_res_dim;       /* 64 */
    int32_t n_decode;          /* 4 decoder blocks (the last upsamples x2) */
    int32_t n_voice_rows;      /* 510 rows per voice pack */
    int32_t max_tokens;        /* per call (arena sizing), <= max_context */
    int32_t max_total;         /* duration frames per call (arena sizing); PCM = 600 per frame */
    float dur_bias;            /* synthetic duration_proj bias (-2.6: ~4 frames per token) */
    float f0_mean;             /* synthetic F0 projection bias (Hz) */
    int32_t debug_no_reuse;
    int32_t weight_type;       /* TTS_TYPE_F32 (0) or TTS_TYPE_F16 (1), for the whole model (gen.weight_type follows it) */
    uint64_t seed;
    uint64_t arena_bytes;      /* 0 = sized from max_tokens / max_total */
} tts_kokoro_config;

typedef struct tts_kokoro tts_kokoro;
void tts_kokoro_default_config(tts_kokoro_config * cfg);
tts_kokoro * tts_kokoro_create(const tts_backend_iface * be, const tts_kokoro_config * cfg);
void tts_kokoro_free(tts_kokoro * k);
/* The duration graph alone (kokoro_duration_runner::run): tokens [n] (3 <= n <= max_tokens) ->
 * hidden [n][d_model + style half] and lengths [n] (rounded, clamped to [1, max_dur]). */
int tts_kokoro_durations(tts_kokoro * k, const int32_t * tokens, int32_t n, float * hidden, float * lengths);
/* The main graph from given durations (kokoro_runner's graph + set_inputs): hidden / lengths as
 * tts_kokoro_durations returns them; rand = [harmonic_num + 1][600 * total] draws or NULL;
 * pcm gets 600 * total samples (total = sum of lengths). */
int tts_kokoro_decode(tts_kokoro * k, const int32_t * tokens, int32_t n, const float * hidden, const float * lengths,
                      const float * rand, float * pcm, uint64_t pcm_cap);
/* Both (kokoro_runner::run); *n_samples = 600 * total. */
int tts_kokoro_run(tts_kokoro * k, const int32_t * tokens, int32_t n, const float * rand, float * pcm, uint64_t pcm_cap,
                   int64_t * n_samples);
int32_t tts_kokoro_last_graph_nodes(const tts_kokoro * k, int32_t which); /* 0 = duration, 1 = main */
int32_t tts_kokoro_n_weights(const tts_kokoro * k);
/* Weight i (front half first, then the generator's): name, ne[4], f32 values; returns bytes. */
uint64_t tts_kokoro_weight(tts_kokoro * k, int32_t i, char * name, uint64_t name_cap, int64_t * ne, float * dst, uint64_t cap);
/* Debug: bytes of the named node of the last duration (which = 0) or main (1) graph. */
uint64_t tts_kokoro_get_node(tts_kokoro * k, int32_t which, const char * name, void * dst, uint64_t cap);
tts_tensor * const * tts_kokoro_graph(const tts_kokoro * k, int32_t which, int32_t * n_nodes);

#ifdef __cplusplus
}
#endif

#endif
