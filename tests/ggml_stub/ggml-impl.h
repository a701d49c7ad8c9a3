// Declaration-only stand-in (compile check of the adapter; see README.md).  Not ggml.
#pragma once
#include "ggml.h"
struct ggml_map_custom2_op_params { ggml_custom2_op_t fun; int n_tasks; void * userdata; };
struct ggml_map_custom3_op_params { ggml_custom3_op_t fun; int n_tasks; void * userdata; };
static inline int32_t ggml_get_op_params_i32(const struct ggml_tensor * tensor, uint32_t i) { return tensor->op_params[i]; }
