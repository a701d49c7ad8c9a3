/* GGUF model files: reader (mmap), writer, the quantize tool and the runners' loader path.
 *
 * The reference loads every model through ggml's gguf API: runner_from_file mmaps the file and points
 * each tensor's data into the mapping (src/models/loaders.cpp:34-95), reads the architecture and the
 * model constants from the KV section (e.g. parler_tts_model::prep_constants,
 * src/models/parler/model.cpp:51-108) and hands every named tensor to the runner's assign_weight
 * (parler/model.cpp:263-307, dac_model.cpp:58-98, general_neural_audio_codec.cpp:36-127).  The
 * quantize example rewrites an F32 file per-architecture (examples/quantize/quantize_impl.cpp:14-292).
 * These entry points are that path for this backend: the runners take their weights from a GGUF file
 * instead of the synthetic generator, uploaded whole-tensor so the HIP backend keeps its own layouts.
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "tts_hip.h"
#include "tts_runners.h"

#ifdef __cplusplus
extern "C" {
#endif

/* gguf_type (value types of the KV section) */
enum tts_gguf_type {
    TTS_GGUF_UINT8 = 0,
    TTS_GGUF_INT8 = 1,
    TTS_GGUF_UINT16 = 2,
    TTS_GGUF_INT16 = 3,
    TTS_GGUF_UINT32 = 4,
    TTS_GGUF_INT32 = 5,
    TTS_GGUF_FLOAT32 = 6,
    TTS_GGUF_BOOL = 7,
    TTS_GGUF_STRING = 8,
    TTS_GGUF_ARRAY = 9,
    TTS_GGUF_UINT64 = 10,
    TTS_GGUF_INT64 = 11,
    TTS_GGUF_FLOAT64 = 12,
};

/* ---- reader (gguf_init_from_file with no_alloc + llama_mmap) ---- */
typedef struct tts_gguf tts_gguf;

/* NULL on a missing / malformed file (the reason goes to stderr). */
tts_gguf * tts_gguf_open(const char * path);
void tts_gguf_close(tts_gguf * g);
uint32_t tts_gguf_version(const tts_gguf * g);
uint64_t tts_gguf_alignment(const tts_gguf * g);
uint64_t tts_gguf_data_offset(const tts_gguf * g); /* gguf_get_data_offset */

int64_t tts_gguf_n_kv(const tts_gguf * g);
int64_t tts_gguf_find_key(const tts_gguf * g, const char * key); /* -1 if absent */
const char * tts_gguf_key(const tts_gguf * g, int64_t i);
int32_t tts_gguf_kv_type(const tts_gguf * g, int64_t i);
/* scalar value of any numeric / bool type converted to the requested C type; 0 on a type mismatch */
int tts_gguf_get_u32(const tts_gguf * g, int64_t i, uint32_t * out);
int tts_gguf_get_i64(const tts_gguf * g, int64_t i, int64_t * out);
int tts_gguf_get_f64(const tts_gguf * g, int64_t i, double * out);
const char * tts_gguf_get_str(const tts_gguf * g, int64_t i); /* NULL unless a string */
int32_t tts_gguf_arr_type(const tts_gguf * g, int64_t i);      /* -1 unless an array */
int64_t tts_gguf_arr_n(const tts_gguf * g, int64_t i);
const void * tts_gguf_arr_data(const tts_gguf * g, int64_t i); /* numeric arrays: packed elements */
const char * tts_gguf_arr_str(const tts_gguf * g, int64_t i, int64_t j);

int64_t tts_gguf_n_tensors(const tts_gguf * g);
int64_t tts_gguf_find_tensor(const tts_gguf * g, const char * name); /* -1 if absent */
const char * tts_gguf_tensor_name(const tts_gguf * g, int64_t i);
int32_t tts_gguf_tensor_type(const tts_gguf * g, int64_t i); /* ggml_type numbering (= TTS_TYPE_*) */
int32_t tts_gguf_tensor_ndims(const tts_gguf * g, int64_t i, int64_t * ne4);
uint64_t tts_gguf_tensor_offset(const tts_gguf * g, int64_t i); /* relative to the data section */
uint64_t tts_gguf_tensor_size(const tts_gguf * g, int64_t i);
const void * tts_gguf_tensor_data(const tts_gguf * g, int64_t i); /* into the mapping */
/* bytes of one block / elements per block of a ggml_type (0 if unknown) */
size_t tts_gguf_type_size(int32_t type);
int64_t tts_gguf_blck_size(int32_t type);

/* ---- writer (gguf_init_empty / gguf_set_* / gguf_add_tensor / gguf_write_to_file) ---- */
typedef struct tts_gguf_writer tts_gguf_writer;

tts_gguf_writer * tts_gguf_writer_new(void);
void tts_gguf_writer_free(tts_gguf_writer * w);
/* setting an existing key replaces its value (gguf_set_val_*) */
void tts_gguf_set_u32(tts_gguf_writer * w, const char * key, uint32_t v);
void tts_gguf_set_i32(tts_gguf_writer * w, const char * key, int32_t v);
void tts_gguf_set_f32(tts_gguf_writer * w, const char * key, float v);
void tts_gguf_set_u64(tts_gguf_writer * w, const char * key, uint64_t v);
void tts_gguf_set_bool(tts_gguf_writer * w, const char * key, int v);
void tts_gguf_set_str(tts_gguf_writer * w, const char * key, const char * v);
void tts_gguf_set_arr(tts_gguf_writer * w, const char * key, int32_t elem_type, const void * data, int64_t n);
void tts_gguf_set_arr_str(tts_gguf_writer * w, const char * key, const char * const * v, int64_t n);
/* gguf_set_kv: every KV pair of a file */
void tts_gguf_copy_kv(tts_gguf_writer * w, const tts_gguf * src);
/* The data is copied; nbytes must equal the type's row size x rows.  0 on success. */
int tts_gguf_add_tensor(tts_gguf_writer * w, const char * name, int32_t type, int32_t n_dims, const int64_t * ne,
                        const void * data, uint64_t nbytes);
int tts_gguf_writer_write(const tts_gguf_writer * w, const char * path); /* 0 on success */

/* ---- quantize tool (examples/quantize/quantize_impl.cpp) ---- */
typedef struct tts_quantize_params {
    int32_t quantize_type;                  /* TTS_TYPE_Q4_K, TTS_TYPE_Q8_0 or TTS_TYPE_F16 */
    int32_t quantize_output_heads;          /* quantization_params fields, same meaning */
    int32_t quantize_text_embeddings;
    int32_t quantize_cross_attn_kv;
    int32_t convert_dac_to_f16;
    int32_t convert_non_quantizable_to_f16;
} tts_quantize_params;

/* Rows of x [rows][K] f32 (host memory) -> type's blocks in dst (host memory); 0 on success. */
typedef int (*tts_quantize_rows_fn)(void * ctx, int32_t type, const float * x, void * dst, int64_t rows, int64_t K);

/* quantize_impl.cpp:14-80 (parler / dia / kokoro; orpheus: every ".weight" matrix except norms,
 * where the reference aborts): 1 = quantize, 2 = convert to F16, 0 = copy unchanged. */
int tts_gguf_tensor_rule(const char * arch, const char * name, const tts_quantize_params * params);
/* quantize_gguf: KV pairs copied + general.quantization_version / general.quantization_type, every
 * tensor in file order, quantized rows from `fn`, F16 by round-to-nearest-even.  0 on success. */
int tts_gguf_quantize(const char * in_path, const char * out_path, const tts_quantize_params * params,
                      tts_quantize_rows_fn fn, void * fn_ctx);
/* The same with the device quantizers (tts_hip_quantize, k_quant.hip). */
int tts_hip_gguf_quantize(tts_hip_backend_t be, const char * in_path, const char * out_path, const tts_quantize_params * params);

/* ---- loader path (runner_from_file -> assign_weight) ---- */
/* parler_tts_model::prep_constants + tensor types: fills the model fields of cfg from the file
 * (n_layers, hidden_size, heads, vocabularies, n_encode, weight / head types); batch, max_ctx, seed
 * and arena stay as given.  0 on success. */
int tts_parler_config_from_gguf(const tts_gguf * g, tts_parler_config * cfg);
/* A Parler runner whose weights are the file's "decoder.*" tensors (parler/model.cpp:501-505);
 * NULL (with the reason on stderr) on a missing tensor or a shape / type the runner cannot take. */
tts_parler * tts_parler_create_from_gguf(const tts_backend_iface * be, const tts_parler_config * cfg, const tts_gguf * g);
/* Writes the runner's synthetic weights (the ones tts_parler_create uploads for cfg) as a GGUF file
 * with the reference's tensor names and keys, plus a DAC-44k decoder ("audio_encoder.*", dac.* keys)
 * for dac_cfg when not NULL -- the F32 input of the quantize tool in the tests. */
int tts_parler_write_synthetic_gguf(const tts_parler_config * cfg, const tts_dac_config * dac_cfg, const char * path);

/* dac_model::prep_constants / prep_layers: codebooks, strides from the dac.* keys.  0 on success. */
int tts_dac_config_from_gguf(const tts_gguf * g, tts_dac_config * cfg);
/* A DAC decoder whose weights are the file's "audio_encoder.*" tensors (F32). */
tts_dac * tts_dac_create_from_gguf(const tts_backend_iface * be, const tts_dac_config * cfg, const tts_gguf * g);

#ifdef __cplusplus
}
#endif
