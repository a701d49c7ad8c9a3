// Declaration-only stand-in (compile check of the adapter; see README.md).  Not ggml.
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
enum ggml_type { GGML_TYPE_F32 = 0, GGML_TYPE_F16 = 1, GGML_TYPE_Q8_0 = 8, GGML_TYPE_Q4_K = 12, GGML_TYPE_I32 = 26 };
enum ggml_op { GGML_OP_NONE = 0, GGML_OP_MUL_MAT, GGML_OP_UNARY, GGML_OP_MAP_CUSTOM2, GGML_OP_MAP_CUSTOM3, GGML_OP_COUNT };
enum ggml_unary_op { GGML_UNARY_OP_ABS, GGML_UNARY_OP_TANH, GGML_UNARY_OP_COUNT };
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
struct ggml_cgraph;
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
