// Definitions for the stand-in ggml declarations (tests/ggml_stub/*.h): just enough runtime for the
// adapter (src/ggml_backend/ggml-tts-hip.cpp) to execute in tests/test_adapter_gpu.py.  Test
// infrastructure, not ggml: op / unary names are upstream's strings (ggml.c GGML_OP_NAME,
// GGML_UNARY_OP_NAME), sizes follow upstream's ggml_nbytes, buffers are plain structs.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "ggml-backend-impl.h"
#include "ggml-backend.h"
#include "ggml.h"

static const char * kOpNames[GGML_OP_COUNT] = {
    "NONE", "DUP", "ADD", "ADD1", "ACC", "SUB", "MUL", "DIV", "SQR", "SQRT", "LOG", "SIN", "COS", "SUM", "SUM_ROWS", "MEAN",
    "ARGMAX", "COUNT_EQUAL", "REPEAT", "REPEAT_BACK", "CONCAT", "SILU_BACK", "NORM", "RMS_NORM", "RMS_NORM_BACK", "GROUP_NORM",
    "MUL_MAT", "MUL_MAT_ID", "OUT_PROD", "SCALE", "SET", "CPY", "CONT", "RESHAPE", "VIEW", "PERMUTE", "TRANSPOSE", "GET_ROWS",
    "GET_ROWS_BACK", "DIAG", "DIAG_MASK_INF", "DIAG_MASK_ZERO", "SOFT_MAX", "SOFT_MAX_BACK", "ROPE", "ROPE_BACK", "CLAMP",
    "CONV_TRANSPOSE_1D", "IM2COL", "IM2COL_BACK", "CONV_TRANSPOSE_2D", "POOL_1D", "POOL_2D", "POOL_2D_BACK", "UPSCALE", "PAD",
    "PAD_REFLECT_1D", "ARANGE", "TIMESTEP_EMBEDDING", "ARGSORT", "LEAKY_RELU", "FLASH_ATTN_EXT", "FLASH_ATTN_BACK", "SSM_CONV",
    "SSM_SCAN", "WIN_PART", "WIN_UNPART", "GET_REL_POS", "ADD_REL_POS", "RWKV_WKV6", "GATED_LINEAR_ATTN", "UNARY", "MAP_UNARY",
    "MAP_BINARY", "MAP_CUSTOM1_F32", "MAP_CUSTOM2_F32", "MAP_CUSTOM3_F32", "MAP_CUSTOM1", "MAP_CUSTOM2", "MAP_CUSTOM3",
    "CROSS_ENTROPY_LOSS", "CROSS_ENTROPY_LOSS_BACK", "OPT_STEP_ADAMW", "CUMSUM", "MOD", "ROUND", "STFT", "ISTFT"};

static const char * kUnaryNames[GGML_UNARY_OP_COUNT] = {"ABS", "SGN", "NEG", "STEP", "TANH", "ELU", "RELU", "SIGMOID", "GELU",
                                                         "GELU_QUICK", "SILU", "HARDSWISH", "HARDSIGMOID", "EXP"};

extern "C" {

const char * ggml_op_name(enum ggml_op op) { return (int)op >= 0 && op < GGML_OP_COUNT ? kOpNames[op] : nullptr; }
const char * ggml_unary_op_name(enum ggml_unary_op op) { return (int)op >= 0 && op < GGML_UNARY_OP_COUNT ? kUnaryNames[op] : nullptr; }

static size_t type_size(enum ggml_type t) {
    switch (t) {
        case GGML_TYPE_F32: case GGML_TYPE_I32: return 4;
        case GGML_TYPE_F16: case GGML_TYPE_I16: return 2;
        case GGML_TYPE_I8: return 1;
        case GGML_TYPE_Q8_0: return 34;
        case GGML_TYPE_Q4_K: return 144;
    }
    return 0;
}
static int64_t blck_size(enum ggml_type t) { return t == GGML_TYPE_Q8_0 ? 32 : t == GGML_TYPE_Q4_K ? 256 : 1; }

// upstream ggml_nbytes: the byte span of the (possibly strided) tensor
size_t ggml_nbytes(const struct ggml_tensor * t) {
    size_t n;
    const int64_t bs = blck_size(t->type);
    if (bs == 1) {
        n = type_size(t->type);
        for (int i = 0; i < GGML_MAX_DIMS; ++i) n += (size_t)(t->ne[i] - 1) * t->nb[i];
    } else {
        n = (size_t)t->ne[0] * t->nb[0] / (size_t)bs;
        for (int i = 1; i < GGML_MAX_DIMS; ++i) n += (size_t)(t->ne[i] - 1) * t->nb[i];
    }
    return n;
}

int ggml_graph_n_nodes(struct ggml_cgraph * g) { return g->n_nodes; }
struct ggml_tensor * ggml_graph_node(struct ggml_cgraph * g, int i) { return g->nodes[i < 0 ? g->n_nodes + i : i]; }

void ggml_abort(const char * file, int line, const char * fmt, ...) {
    fprintf(stderr, "%s:%d: GGML_ABORT: ", file, line);
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fputc('\n', stderr);
    abort();
}

ggml_backend_buffer_t ggml_backend_buffer_init(ggml_backend_buffer_type_t buft, struct ggml_backend_buffer_i iface, void * context, size_t size) {
    auto * b = new ggml_backend_buffer();
    b->iface = iface;
    b->buft = buft;
    b->context = context;
    b->size = size;
    b->usage = GGML_BACKEND_BUFFER_USAGE_ANY;
    return b;
}

void ggml_backend_buffer_free(ggml_backend_buffer_t b) {
    if (!b) return;
    if (b->iface.free_buffer) b->iface.free_buffer(b);
    delete b;
}

enum ggml_backend_buffer_usage ggml_backend_buffer_get_usage(ggml_backend_buffer_t b) { return b->usage; }
bool ggml_backend_buffer_is_host(ggml_backend_buffer_t b) { return b->buft->iface.is_host ? b->buft->iface.is_host(b->buft) : false; }

}  // extern "C"
