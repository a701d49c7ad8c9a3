/*
 * oracle/ggml_ref.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the ggml-cpu arithmetic that TTS.cpp's graphs rely on.  The arithmetic
 * lives in the unvendored fork `ggml/` (https://github.com/mmwillet/ggml.git, branch
 * support-for-tts, commit unrecorded: /root/reference/.gitmodules:1-4), so this file restates
 * the published ggml-cpu *scalar reference* paths (quantize_row_*_ref, dequantize_row_*,
 * generic ggml_vec_dot_*, ggml_compute_forward_*), compiled with -ffp-contract=off so that
 * every a*b+c is two roundings, as in the scalar C source.
 *
 * Parity pinning: the reference tree holds NO golden vectors for this path.
 * This oracle is pinned by (1) known-answer tests on hand-built quant blocks, (2) torch-CPU
 * generated fixtures for the float ops (tests/golden/, script committed), (3) analytic
 * identities.  Where none covers a result it is marked "parity unpinned" in DESIGN.md.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code.
 */
#ifndef ORACLE_GGML_REF_H
#define ORACLE_GGML_REF_H

#include <stddef.h>
#include <stdint.h>

#include "../include/tts_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define QK_K 256
#define K_SCALE_SIZE 12
#define QK8_0 32

typedef uint16_t ref_fp16_t;

typedef struct {
    ref_fp16_t d;
    ref_fp16_t dmin;
    uint8_t scales[K_SCALE_SIZE];
    uint8_t qs[QK_K / 2];
} ref_block_q4_K; /* 144 bytes */

typedef struct {
    ref_fp16_t d;
    int8_t qs[QK8_0];
} ref_block_q8_0; /* 34 bytes */

typedef struct {
    float d;
    int8_t qs[QK_K];
    int16_t bsums[QK_K / 16];
} ref_block_q8_K; /* 292 bytes */

float ref_fp16_to_fp32(ref_fp16_t h);
ref_fp16_t ref_fp32_to_fp16(float f);
int ref_nearest_int(float fval);

void ref_get_scale_min_k4(int j, const uint8_t * q, uint8_t * d, uint8_t * m);
void ref_dequantize_row_q4_K(const ref_block_q4_K * x, float * y, int64_t k);
void ref_dequantize_row_q8_0(const ref_block_q8_0 * x, float * y, int64_t k);
void ref_quantize_row_q8_K(const float * x, ref_block_q8_K * y, int64_t k);
void ref_quantize_row_q8_0(const float * x, ref_block_q8_0 * y, int64_t k);
void ref_quantize_row_q4_K(const float * x, ref_block_q4_K * y, int64_t k);
void ref_vec_dot_q4_K_q8_K(int n, float * s, const void * vx, const void * vy);
void ref_vec_dot_q8_0_q8_0(int n, float * s, const void * vx, const void * vy);
void ref_vec_dot_f16(int n, float * s, const ref_fp16_t * x, const ref_fp16_t * y);
void ref_vec_dot_f32(int n, float * s, const float * x, const float * y);

float ref_gelu_f32(float x);
/* ggml's GELU goes through a 65536-entry fp16 table (GGML_GELU_FP16). */
float ref_gelu_table(float x);

/* y[m][n] = sum_k W[n][k] x[m][k] with ggml-cpu mul_mat semantics for a weight of `type`. */
void ref_gemv(int type, const void * w, const float * x, float * y, int64_t K, int64_t N, int64_t M, int n_threads);

/* Graph interpreter: executes nodes (tts_tensor with host data pointers) in order. */
int oracle_graph_compute(tts_tensor * const * nodes, int n_nodes, int n_threads);
/* Single node, single thread. */
int oracle_compute_node(tts_tensor * node);
/* 0 (default): ggml-cpu's generic scalar loops; 1: the x86 AVX2/FMA/F16C accumulation order of
 * vec_dot_f16 / _f32 / q4_K_q8_K / q8_0_q8_0 and upstream's conv_transpose_1d loop (ggml_ref.c). */
void oracle_set_simd_mode(int mode);
int oracle_simd_mode(void);

/* Backend vtable (host memory) for the C++ runners. */
int oracle_backend_iface(tts_backend_iface * out, int n_threads);

#ifdef __cplusplus
}
#endif

#endif
