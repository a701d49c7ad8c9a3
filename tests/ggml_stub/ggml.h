// Minimal stand-in for the ggml declarations the adapter uses (test infrastructure; see README.md).
// Not ggml: enough of the upstream early-2025 API shape to compile src/ggml_backend/ggml-tts-hip.cpp
// and, with ggml_runtime.cpp, to run it in tests/test_adapter_gpu.py.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>
#define GGML_MAX_DIMS 4
#define GGML_MAX_SRC 10
#define GGML_MAX_NAME 64
#define GGML_MAX_OP_PARAMS 64
#ifdef __cplusplus
extern "C" {
#endif
enum ggml_type { GGML_TYPE_F32 = 0, GGML_TYPE_F16 = 1, GGML_TYPE_Q8_0 = 8, GGML_TYPE_Q4_K = 12, GGML_TYPE_I8 = 24, GGML_TYPE_I16 = 25,
                 GGML_TYPE_I32 = 26 };
// upstream's op order (ggml.h, early 2025), then the TTS fork's ops; the adapter matches by name
enum ggml_op {
    GGML_OP_NONE = 0, GGML_OP_DUP, GGML_OP_ADD, GGML_OP_ADD1, GGML_OP_ACC, GGML_OP_SUB, GGML_OP_MUL, GGML_OP_DIV, GGML_OP_SQR,
    GGML_OP_SQRT, GGML_OP_LOG, GGML_OP_SIN, GGML_OP_COS, GGML_OP_SUM, GGML_OP_SUM_ROWS, GGML_OP_MEAN, GGML_OP_ARGMAX,
    GGML_OP_COUNT_EQUAL, GGML_OP_REPEAT, GGML_OP_REPEAT_BACK, GGML_OP_CONCAT, GGML_OP_SILU_BACK, GGML_OP_NORM, GGML_OP_RMS_NORM,
    GGML_OP_RMS_NORM_BACK, GGML_OP_GROUP_NORM, GGML_OP_MUL_MAT, GGML_OP_MUL_MAT_ID, GGML_OP_OUT_PROD, GGML_OP_SCALE, GGML_OP_SET,
    GGML_OP_CPY, GGML_OP_CONT, GGML_OP_RESHAPE, GGML_OP_VIEW, GGML_OP_PERMUTE, GGML_OP_TRANSPOSE, GGML_OP_GET_ROWS,
    GGML_OP_GET_ROWS_BACK, GGML_OP_DIAG, GGML_OP_DIAG_MASK_INF, GGML_OP_DIAG_MASK_ZERO, GGML_OP_SOFT_MAX, GGML_OP_SOFT_MAX_BACK,
    GGML_OP_ROPE, GGML_OP_ROPE_BACK, GGML_OP_CLAMP, GGML_OP_CONV_TRANSPOSE_1D, GGML_OP_IM2COL, GGML_OP_IM2COL_BACK,
    GGML_OP_CONV_TRANSPOSE_2D, GGML_OP_POOL_1D, GGML_OP_POOL_2D, GGML_OP_POOL_2D_BACK, GGML_OP_UPSCALE, GGML_OP_PAD,
    GGML_OP_PAD_REFLECT_1D, GGML_OP_ARANGE, GGML_OP_TIMESTEP_EMBEDDING, GGML_OP_ARGSORT, GGML_OP_LEAKY_RELU, GGML_OP_FLASH_ATTN_EXT,
    GGML_OP_FLASH_ATTN_BACK, GGML_OP_SSM_CONV, GGML_OP_SSM_SCAN, GGML_OP_WIN_PART, GGML_OP_WIN_UNPART, GGML_OP_GET_REL_POS,
    GGML_OP_ADD_REL_POS, GGML_OP_RWKV_WKV6, GGML_OP_GATED_LINEAR_ATTN, GGML_OP_UNARY, GGML_OP_MAP_UNARY, GGML_OP_MAP_BINARY,
    GGML_OP_MAP_CUSTOM1_F32, GGML_OP_MAP_CUSTOM2_F32, GGML_OP_MAP_CUSTOM3_F32, GGML_OP_MAP_CUSTOM1, GGML_OP_MAP_CUSTOM2,
    GGML_OP_MAP_CUSTOM3, GGML_OP_CROSS_ENTROPY_LOSS, GGML_OP_CROSS_ENTROPY_LOSS_BACK, GGML_OP_OPT_STEP_ADAMW,
    GGML_OP_CUMSUM, GGML_OP_MOD, GGML_OP_ROUND, GGML_OP_STFT, GGML_OP_ISTFT,
    GGML_OP_COUNT
};
enum ggml_unary_op {
    GGML_UNARY_OP_ABS, GGML_UNARY_OP_SGN, GGML_UNARY_OP_NEG, GGML_UNARY_OP_STEP, GGML_UNARY_OP_TANH, GGML_UNARY_OP_ELU,
    GGML_UNARY_OP_RELU, GGML_UNARY_OP_SIGMOID, GGML_UNARY_OP_GELU, GGML_UNARY_OP_GELU_QUICK, GGML_UNARY_OP_SILU,
    GGML_UNARY_OP_HARDSWISH, GGML_UNARY_OP_HARDSIGMOID, GGML_UNARY_OP_EXP, GGML_UNARY_OP_COUNT
};
enum ggml_status { GGML_STATUS_ALLOC_FAILED = -2, GGML_STATUS_FAILED = -1, GGML_STATUS_SUCCESS = 0, GGML_STATUS_ABORTED = 1 };
enum ggml_tensor_flag { GGML_TENSOR_FLAG_INPUT = 1, GGML_TENSOR_FLAG_OUTPUT = 2, GGML_TENSOR_FLAG_PARAM = 4, GGML_TENSOR_FLAG_LOSS = 8 };
typedef struct ggml_backend_buffer * ggml_backend_buffer_t;
struct ggml_tensor {
    enum ggml_type type;
    ggml_backend_buffer_t buffer;
    int64_t ne[GGML_MAX_DIMS];
    size_t nb[GGML_MAX_DIMS];
    enum ggml_op op;
    int32_t op_params[GGML_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct ggml_tensor * src[GGML_MAX_SRC];
    struct ggml_tensor * view_src;
    size_t view_offs;
    void * data;
    char name[GGML_MAX_NAME];
    void * extra;
};
// the graph's node list (upstream's struct has more members; only the nodes are read through the API)
struct ggml_cgraph {
    int n_nodes;
    struct ggml_tensor ** nodes;
};
typedef void (*ggml_custom2_op_t)(struct ggml_tensor *, const struct ggml_tensor *, const struct ggml_tensor *, int, int, void *);
typedef void (*ggml_custom3_op_t)(struct ggml_tensor *, const struct ggml_tensor *, const struct ggml_tensor *, const struct ggml_tensor *, int, int, void *);
const char * ggml_op_name(enum ggml_op op);
const char * ggml_unary_op_name(enum ggml_unary_op op);
size_t ggml_nbytes(const struct ggml_tensor * tensor);
int ggml_graph_n_nodes(struct ggml_cgraph * cgraph);
struct ggml_tensor * ggml_graph_node(struct ggml_cgraph * cgraph, int i);
void ggml_abort(const char * file, int line, const char * fmt, ...);
#define GGML_ABORT(...) ggml_abort(__FILE__, __LINE__, __VA_ARGS__)
typedef uint8_t ggml_guid[16];
typedef ggml_guid * ggml_guid_t;
#ifdef __cplusplus
}
#endif
