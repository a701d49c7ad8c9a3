/*
 * tts_hip.h — C-ABI of the MI355X (gfx950) compute backend for TTS.cpp's decode path.
 *
 * This is the drop-in boundary.  TTS.cpp builds ggml graphs (e.g. build_parler_graph,
 * /root/reference/src/models/parler/model.cpp:520-614) and hands them to a ggml backend through
 * ggml_backend_sched (/root/reference/src/tts_model.cpp:53-67).  A ggml backend is a vtable
 * (ggml_backend_i / ggml_backend_buffer_i / ggml_backend_device_i, fork `ggml/` submodule,
 * .gitmodules:1-4, absent here).  Every entry point below is what that vtable needs underneath:
 *
 *   tts_hip_backend_init        <- ggml_backend_dev_init / ggml_backend_metal_init()
 *                                  (selection sites: src/tts_model.cpp:40,56,134;
 *                                   src/models/parler/model.cpp:327,345; src/decoder/dac_model.cpp:128 ...)
 *   tts_hip_buffer_alloc/free   <- ggml_backend_buffer_type_i::alloc_buffer / buffer_i::free_buffer
 *                                  (callers: src/tts_model.cpp:150, src/models/parler/model.cpp:377)
 *   tts_hip_tensor_set          <- ggml_backend_tensor_set (src/tts_model.cpp:157-164)
 *   tts_hip_tensor_get          <- ggml_backend_tensor_get_async (src/tts_model.cpp:25-36); it
 *                                  synchronises the compute stream first, because no caller in
 *                                  the reference ever calls ggml_backend_synchronize.
 *   tts_hip_memset              <- ggml_backend_buffer_clear (src/models/parler/model.cpp:383)
 *   tts_hip_supports_op         <- ggml_backend_device_i::supports_op
 *   tts_hip_graph_compute       <- ggml_backend_i::graph_compute
 *                                  (reached from ggml_backend_sched_graph_compute_async,
 *                                   src/models/parler/model.cpp:645)
 *   tts_hip_synchronize         <- ggml_backend_i::synchronize
 *
 * Tensors cross the boundary as `tts_tensor`, a plain C mirror of the ggml_tensor fields a backend
 * reads (type, ne, nb, op, op_params, src, data).  Type ids use ggml's numbering so the ggml
 * adapter maps them 1:1.  No torch or HIP types appear in any signature.
 *
 * Errors: every int-returning entry point returns TTS_STATUS_* (0 = success), mirroring
 * ggml_status; allocation failure returns NULL (reference checks NULL, model.cpp:377-380).
 */
#ifndef TTS_HIP_H
#define TTS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TTS_MAX_DIMS 4
#define TTS_MAX_SRC 4
#define TTS_MAX_OP_PARAMS 16
#define TTS_MAX_NAME 64 /* GGML_MAX_NAME */

/* ggml_type numbering (ggml.h of the fork's early-2025 base). */
enum tts_type {
    TTS_TYPE_F32 = 0,
    TTS_TYPE_F16 = 1,
    TTS_TYPE_Q4_0 = 2,
    TTS_TYPE_Q4_1 = 3,
    TTS_TYPE_Q5_0 = 6,
    TTS_TYPE_Q5_1 = 7,
    TTS_TYPE_Q8_0 = 8,
    TTS_TYPE_Q8_1 = 9,
    TTS_TYPE_Q4_K = 12,
    TTS_TYPE_Q6_K = 14,
    TTS_TYPE_Q8_K = 15,
    TTS_TYPE_I8 = 24,
    TTS_TYPE_I16 = 25,
    TTS_TYPE_I32 = 26,
    TTS_TYPE_COUNT = 40
};

/* Ops the TTS.cpp graphs emit.  Names follow ggml_op; numbering is our own
 * (the adapter maps ggml_op -> tts_op by name). */
enum tts_op {
    TTS_OP_NONE = 0,
    TTS_OP_DUP,
    TTS_OP_ADD,
    TTS_OP_SUB,
    TTS_OP_MUL,
    TTS_OP_DIV,
    TTS_OP_SQR,
    TTS_OP_SQRT,
    TTS_OP_SIN,
    TTS_OP_COS,
    TTS_OP_SUM_ROWS,
    TTS_OP_REPEAT,
    TTS_OP_CONCAT,
    TTS_OP_NORM,
    TTS_OP_RMS_NORM,
    TTS_OP_MUL_MAT,
    TTS_OP_SCALE,
    TTS_OP_CPY,
    TTS_OP_CONT,
    TTS_OP_RESHAPE,
    TTS_OP_VIEW,
    TTS_OP_PERMUTE,
    TTS_OP_TRANSPOSE,
    TTS_OP_GET_ROWS,
    TTS_OP_SOFT_MAX,
    TTS_OP_ROPE,
    TTS_OP_CLAMP,
    TTS_OP_CONV_TRANSPOSE_1D,
    TTS_OP_IM2COL,
    TTS_OP_UPSCALE,
    TTS_OP_PAD,
    TTS_OP_LEAKY_RELU,
    TTS_OP_UNARY,
    TTS_OP_CUMSUM, /* fork op */
    TTS_OP_MOD,    /* fork op */
    TTS_OP_ROUND,  /* fork op */
    TTS_OP_STFT,   /* fork op */
    TTS_OP_ISTFT,  /* fork op */
    TTS_OP_MAP_CUSTOM3, /* ggml_map_custom3 with a CPU callback in the reference; op_params[0] names
                           which one (tts_custom_op) and the backend runs its device restatement */
    TTS_OP_MAP_CUSTOM2, /* ggml_map_custom2, likewise */
    TTS_OP_COUNT
};

/* The reference's ggml_map_custom* callbacks a graph may carry (op_params[0] of MAP_CUSTOM3). */
enum tts_custom_op {
    TTS_CUSTOM_NONE = 0,
    /* uv_noise_compute (src/util.cpp:140-170): a = shape [L, H, 2], b = upscaled F0 [L],
     * c = [threshold, noise_std, sin_amp, sin_amp/3, rand[H][L]] (f32) -> plane 0 uv, plane 1 noise */
    TTS_CUSTOM_UV_NOISE = 1,
    /* cfg_scale (src/util.cpp:175-200, MAP_CUSTOM2 in build_dia_head_outputs, src/models/dia/model.cpp:370):
     * a = cond, b = uncond (same shape) -> cond + scale * (cond - uncond); op_params[1] = scale (f32 bits).
     * The callback's "-INFINITY past max_output" store is overwritten by the next line, so it has no effect. */
    TTS_CUSTOM_CFG_SCALE = 2
};

enum tts_unary_op {
    TTS_UNARY_ABS = 0,
    TTS_UNARY_NEG,
    TTS_UNARY_TANH,
    TTS_UNARY_RELU,
    TTS_UNARY_SIGMOID,
    TTS_UNARY_GELU,
    TTS_UNARY_SILU,
    TTS_UNARY_EXP,
    TTS_UNARY_COUNT
};

enum tts_status {
    TTS_STATUS_SUCCESS = 0,
    TTS_STATUS_FAILED = -1,
    TTS_STATUS_ALLOC_FAILED = -2,
    TTS_STATUS_UNSUPPORTED = -3,
    TTS_STATUS_BAD_ARG = -4,
    TTS_STATUS_NO_DEVICE = -5
};

/* tts_tensor.flags bits */
/* tts_hip_gemv_stats type slot of the decode attention launches (the split scores + P.V pair, timed
 * from the first kernel's start to the second's end; bytes = the K and V rows read + q + output) */
#define TTS_PROF_ATTN 39

#define TTS_FLAG_INPUT 1
#define TTS_FLAG_HOSTDATA 2 /* data is host memory without a buffer (util.cpp:86-94 trick) */
#define TTS_FLAG_OUTPUT 4
#define TTS_FLAG_PERSIST 8
#define TTS_FLAG_REPACKED 16 /* set by the HIP backend: the tensor is stored in its Q4_K lane layout */
#define TTS_FLAG_TILED_COPY 64 /* set by the HIP backend: a lane-layout Q4_K matrix that also has a tile-layout copy
                                  (medium matrices, TTS_HIP_OPT_Q4K_DUAL_BYTES), read by GEMVs of >= 8 columns */
#define TTS_FLAG_TILED 32    /* set by the HIP backend: Q4_K stored in its 4-row tile layout (tts_repack_q4_K_tiled),
                                read by the matrix-core GEMV (large matrices, tts_hip_weight_set) */

/* Plain mirror of the ggml_tensor fields a backend reads.  `data` is a device pointer for
 * tensors handed to tts_hip_* (a host pointer for the CPU oracle in oracle/).  op_params hold
 * int32 and float (bit-cast) parameters exactly where ggml_set_op_params puts them. */
typedef struct tts_tensor {
    int32_t type;
    int32_t op;
    int64_t ne[TTS_MAX_DIMS];
    size_t nb[TTS_MAX_DIMS];
    int32_t op_params[TTS_MAX_OP_PARAMS];
    struct tts_tensor * src[TTS_MAX_SRC];
    struct tts_tensor * view_src;
    size_t view_offs;
    void * data;
    int32_t flags;
    int32_t pad_;
    char name[TTS_MAX_NAME];
} tts_tensor;

/* ---- type traits (host, no device needed) ---- */
size_t tts_type_size(int type);       /* bytes per block */
int64_t tts_blck_size(int type);      /* elements per block */
size_t tts_row_size(int type, int64_t ne0);
const char * tts_type_name(int type);
const char * tts_op_name(int op);

/* ---- device / backend (ggml_backend_i + ggml_backend_buffer_i underneath) ---- */
typedef struct tts_hip_backend * tts_hip_backend_t;

int tts_hip_device_count(void);
/* Free / total device memory of `device` (ggml_backend_device_i::get_memory). */
int tts_hip_device_memory(int device, size_t * free_bytes, size_t * total_bytes);
/* Stream events (ggml_backend_device_i::event_new / event_free / event_synchronize,
 * ggml_backend_i::event_record / event_wait): an opaque hipEvent_t. */
void * tts_hip_event_new(int device);
void tts_hip_event_free(void * event);
int tts_hip_event_record(tts_hip_backend_t backend, void * event);
int tts_hip_event_wait(tts_hip_backend_t backend, void * event); /* the backend's stream waits for it */
int tts_hip_event_synchronize(void * event);
/* Whether `p` is device memory (UVA query): the adapter's set_tensor copies device-to-device when a
 * caller hands it another backend's device buffer as the "host" source. */
int tts_hip_is_device_pointer(const void * p);
tts_hip_backend_t tts_hip_backend_init(int device); /* NULL if no device */
void tts_hip_backend_free(tts_hip_backend_t backend);
const char * tts_hip_backend_name(tts_hip_backend_t backend);

void * tts_hip_buffer_alloc(tts_hip_backend_t backend, size_t size); /* 256-B aligned device memory */
void tts_hip_buffer_free(tts_hip_backend_t backend, void * ptr);
size_t tts_hip_buffer_alignment(void);

int tts_hip_tensor_set(tts_hip_backend_t backend, void * dst_dev, const void * src_host, size_t size);
int tts_hip_tensor_get(tts_hip_backend_t backend, void * dst_host, const void * src_dev, size_t size);
int tts_hip_tensor_copy(tts_hip_backend_t backend, void * dst_dev, const void * src_dev, size_t size); /* stream-ordered */
/* Measurement helper (bench.py's measured HBM ceiling): the same copy as a streaming kernel -- 16-B loads and
 * stores per lane, non-temporal, 16 workgroups per CU each copying one contiguous chunk -- the guide's float4-copy
 * method.  size % 16 == 0
 * and both pointers 16-B aligned, else TTS_STATUS_BAD_ARG.  Stream-ordered. */
int tts_hip_copy_stream(tts_hip_backend_t backend, void * dst_dev, const void * src_dev, size_t size);
/* ggml_backend_i::set_tensor_async: `src_host` is staged at once (reusable on return), the copy runs
 * in stream order after the work already queued. */
/* Fusion coverage of a node list without a device: counts[0..14] = fused items per kind (GEMV, ATTN,
 * LN, LSTM, SNAKE, EMBED, CONV, ADAIN), counts[15] = nodes still launched one by one. */
int tts_hip_plan_stats(tts_tensor * const * nodes, int n_nodes, int mask, int32_t * counts);
int tts_hip_tensor_set_async(tts_hip_backend_t backend, void * dst_dev, const void * src_host, size_t size);
int tts_hip_memset(tts_hip_backend_t backend, void * dst_dev, int value, size_t size);
int tts_hip_synchronize(tts_hip_backend_t backend);

/* ggml_backend_buffer_i::set_tensor / get_tensor for a whole weight tensor.  The HIP buffer keeps
 * Q4_K matrices in its own lane layout (like ggml-cpu's repack buffer type): set repacks and sets
 * TTS_FLAG_REPACKED on `t`; get returns ggml's native bytes. */
int tts_hip_weight_set(tts_hip_backend_t backend, tts_tensor * t, const void * src_host);
int tts_hip_weight_get(tts_hip_backend_t backend, const tts_tensor * t, void * dst_host);
/* Weight quantization on the device, ggml's quantize_row_q4_K_ref / quantize_row_q8_0_ref
 * (ggml-quants.c; the reference's examples/quantize path, quantize_impl.cpp:82-292): x [rows][K] f32
 * -> dst [rows][K / blck] ggml blocks (native layout, both device pointers; K % 256 == 0 for Q4_K,
 * K % 32 == 0 for Q8_0).  Bytes equal the CPU reference's (f32 operations in source order). */
int tts_hip_quantize(tts_hip_backend_t backend, int type, const float * x_dev, void * dst_dev, int64_t rows, int64_t K);
/* Host helper: (inverse = 0) ggml Q4_K blocks -> backend lane layout, (1) the reverse. */
void tts_repack_q4_K(const void * src, void * dst, int64_t nblocks, int inverse);
/* The 4-row tile layout of a Q4_K matrix [nrows][nb blocks] (nrows % 4 == 0): per (tile t of rows
 * 4t..4t+3, block b) 576 bytes at (t*nb + b)*576: the four 16-B block headers (d, dmin, scales),
 * then for chunk c = 0..3, half h = 0..1, row i = 0..3 a 16-B piece whose dword l' holds the bytes
 * qs[32c + 8kk + 4h + l'] (kk = 0..3) -- one lane's MFMA operand for residues 4h..4h+3. */
void tts_repack_q4_K_tiled(const void * src, void * dst, int64_t nrows, int64_t nb, int inverse);

int tts_hip_supports_op(const tts_tensor * node);
int tts_hip_graph_compute(tts_hip_backend_t backend, tts_tensor * const * nodes, int n_nodes);
/* ggml_backend_i::graph_plan_create / graph_plan_compute: record a graph into plan slot 0 or 1
 * without running it, then launch it later.  A caller records step n+1 on the host while step n
 * runs on the device (the node array must stay alive until the slot is launched). */
int tts_hip_graph_prepare(tts_hip_backend_t backend, tts_tensor * const * nodes, int n_nodes, int slot);
int tts_hip_graph_launch(tts_hip_backend_t backend, int slot);

/* Backend options (env-free knobs used by the bench / tests). */
enum tts_hip_option {
    TTS_HIP_OPT_FUSION = 0,      /* TTS_FUSE_* bitmask of enabled patterns (default: all bits, 0 = off) */
    TTS_HIP_OPT_PROFILE_GEMV = 1, /* 1 = time quantized GEMV launches with HIP events */
    TTS_HIP_OPT_GRAPHS = 2,       /* 1 = replay each graph_compute as a HIP graph (capture + exec update) */
    TTS_HIP_OPT_CONV_F32ACC = 3,  /* 1 = conv GEMMs accumulate in f32 on f16 MFMA (default 0: f64, PCM parity);
                                     2 = fused conv_1d on f16 MFMA per 32-term batch, batches summed in f64 */
    TTS_HIP_OPT_CONVT_LDS = 4,    /* 1 (default) = conv_transpose_1d on the LDS-staged f64 MFMA kernel, 0 = per-wave kernel */
    TTS_HIP_OPT_ATTN_SPLIT = 5,   /* decode attention over P >= value keys runs as two position/dim-split kernels
                                     (scores, then softmax + P.V); 0 = always the one-workgroup-per-head kernel */
    TTS_HIP_OPT_KV_PREFETCH = 6,  /* prefetch the next decode attention's K/V (KV length >= value) into the
                                     Infinity Cache on a side stream during the GEMVs before it; 0 = off */
    TTS_HIP_OPT_KV_PREFETCH_BLOCKS = 7, /* workgroups of the prefetch kernel (default 128) */
    TTS_HIP_OPT_Q4K_TILE_BYTES = 8, /* tts_hip_weight_set stores Q4_K matrices of >= value bytes (ne1 % 4 == 0) in the
                                     4-row tile layout; their GEMVs run on the matrix-core kernel (exact integer f16
                                     MFMAs, bit-identical).  Default 4 MiB; 0 = never */
    TTS_HIP_OPT_GEMV_DEBUG = 10, /* matrix-core GEMV phase study: 1 = skip the row phase, 2 = skip the prologue
                                     (results invalid; micro-benchmarks only) */
    TTS_HIP_OPT_CONV_SPLIT = 12, /* 1 (default) = codec convolutions over short sequences split their input channels
                                     over extra workgroups (f64 partial sums, reduced in split order) until a launch
                                     has ~512 workgroups; N > 1 = until ~N workgroups; 0 = never */
    TTS_HIP_OPT_GEMV_UNIQUE = 11, /* 1 (default) = lane-layout Q4_K GEMVs run the unique-load kernel (an octet per
                                     (row, block), every weight byte loaded once, all columns per lane, ggml's chain
                                     finished from LDS: bit-identical); 0 = the octet-per-(row, column) kernel */
    TTS_HIP_OPT_GEMV_KS = 13,     /* tile-layout Q4_K GEMVs of at most `value` 16-row tiles (M <= 8 columns, K <= 4096)
                                     run the K-split matrix-core kernel (a workgroup per tile, its blocks over the
                                     waves, ggml's chain finished from LDS: bit-identical).  Default 256; 0 = never */
    TTS_HIP_OPT_ATTN_FUSED = 14,  /* decode attention over P >= value keys (hd 64 / 128, 16-B K and V rows) runs as
                                     ONE 1024-thread launch per attention (k_attn_fused; default 0 = off: the split pair,
                                     TTS_HIP_OPT_ATTN_SPLIT; tests and studies use 128) */
    TTS_HIP_OPT_GEMM_Q8 = 18,     /* 1 (default) = Q8_0 products of more than 8 columns run the int8 matrix-core GEMM
                                     (k_gemm_q8_0, bit-identical); 0 = one GEMV launch per 8 columns */
    TTS_HIP_OPT_BGEMM_F32 = 19,   /* 1 (default) = batched float products (attention over many queries: encoders,
                                     prefill) run the tiled f64-accumulating GEMM; 0 = the one-wave-per-output kernel */
    TTS_HIP_OPT_CU_PARTITION = 20, /* (index << 8) | count, count > 1: the backend's stream runs on partition `index` of
                                     `count` equal CU sets (hipExtStreamCreateWithCUMask; bit 16 set = interleaved CU
                                     numbers, else contiguous), and kernel grids are sized to that share -- concurrent
                                     replica backends then stop competing for CUs.  0 = all CUs */
    TTS_HIP_OPT_Q4K_DUAL_BYTES = 16, /* tts_hip_weight_set keeps a tile-layout copy of lane-layout Q4_K matrices of >= value
                                        bytes (default 1 MiB; 0 = never); a GEMV of >= 8 columns over >= 2048 rows (K >= 2048)
                                        of such matrices runs on the matrix-core kernels, and matrices of different row counts
                                        sharing the activation (Orpheus q / k / v) then run as one launch */
    TTS_HIP_OPT_GEMV_RSPLIT = 17, /* 1 (default): matrix-core Q4_K GEMVs with few 16-row tiles split each tile's residues over
                                     2 or 4 waves (chains joined in ggml's order: bit-identical); 0 = one wave per tile */
    TTS_HIP_OPT_ATTN_PV16 = 15,   /* 1: the split P.V kernel requests a lane's whole V slice (16 x 16 B) before the
                                     softmax when P <= 1024; 0 (default): two 8-chunk batches (measured equal) */
    TTS_HIP_OPT_GEMV_PREQUANT = 21, /* 1 (default): a matrix-core Q4_K GEMV's activation is normed / quantized once, by a
                                     pass writing its MFMA operands to backend scratch, which every workgroup copies into
                                     LDS by LDS-DMA; 0 = every workgroup quantizes the whole activation itself */
    TTS_HIP_OPT_GEMV_KRELAY = 22, /* 1 (default): pre-quantized matrix-core Q4_K GEMVs of K = 1024 / 2048 / 3072 / 4096 /
                                     8192 run the K-relay kernel (a 16-row tile's blocks split over 4-8 waves, ggml's
                                     chain handed from wave to wave in block order); 0 = k_gemv_q4K_mf */
    TTS_HIP_OPT_ATTN_KS = 23,     /* split decode attention: 128 * value key positions per scores workgroup (1, 2 default, 4) */
    TTS_HIP_OPT_ATTN_PV8 = 24,    /* 1: the split P.V kernel covers 8 output dims per workgroup (twice the workgroups); 0 = 16 */
    TTS_HIP_OPT_GEMV_KRELAY_LOOP = 26, /* 1 (default): K-relay SwiGLU launches with more tile pairs than CUs run one workgroup
                                     per CU over its pairs (operands copied once, next pair prefetched); 0 = one per pair */
    TTS_HIP_OPT_GEMV_Q80_PRO = 27, /* 1 (default): Q8_0 GEMVs of <= 8 columns with K % 256 == 0 quantize (and, fused with a
                                     preceding LayerNorm / RMSNorm of K <= 4096, normalize) the activation in every
                                     workgroup: one launch instead of norm + quantize + GEMV; 0 = separate launches */
    TTS_HIP_OPT_GEMV_Q80_SLAB = 28, /* 1 (default): Q8_0 GEMVs with K % 256 == 0 run the slab kernel (a workgroup's rows
                                     fetched whole by LDS-DMA, terms then ggml's block-order chain from LDS);
                                     0 = the (row, block)-per-thread kernel */
    TTS_HIP_OPT_GEMV_Q80_RW = 29,  /* slab Q8_0 GEMV rows per workgroup (0 = auto: the most that still fills every CU) */
    TTS_HIP_OPT_GEMM_Q8_STAGED = 30, /* many-column Q8_0 GEMM with K % 256 == 0: 2 (default) = staged LDS-DMA kernel over
                                     64 x 128 output tiles, 1 = over 64 x 64 tiles, 0 = the direct-load kernel */
    TTS_HIP_OPT_GEMV_KR_INKERNEL = 31, /* K-relay Q4_K GEMVs with K <= value (<= 4096) norm / quantize the activation in every
                                     workgroup instead of after the operand pass (0 = always the operand pass) */
    TTS_HIP_OPT_GEMV_F32_WIDE = 32, /* 1 (default): F32 MUL_MATs of >= 2048 rows x 9..64 columns (the output heads of a
                                       many-prompt step) run the wide GEMV (one sequential f64 chain per output, each
                                       weight read once) instead of the tiled GEMM; 0 = tiled GEMM */
    TTS_HIP_OPT_ATTN_PV_MP = 33, /* 1 (default): the split P.V runs every output dim of a (head, query, sequence) in one
                                    workgroup (hd / 16 passes of 512-position items, any P): the softmax once instead of hd / 16 times;
                                    2: the same with eight waves per workgroup (hd / 32 passes); 0: 16 dims per workgroup */
    TTS_HIP_OPT_GEMM_KR_INKERNEL = 35, /* many-column (> 8) K-relay Q4_K GEMMs with at most `value` columns skip the operand
                                          pass: each (row tile, column tile) workgroup norms / quantizes its 16 columns (0 = off;
                                          + 0x10000: only the jobs without a norm) */
    TTS_HIP_OPT_GEMM_KR_CT2 = 36, /* 1: the many-column K-relay Q4_K GEMM (K = 1024 / 2048) takes two 16-column tiles per
                                     workgroup, each weight tile loaded once for both (0 = one tile per workgroup) */
    TTS_HIP_OPT_GEMM_KR_NW = 34, /* waves per 16-row tile of the many-column (> 8) K-relay Q4_K GEMM: 4 (default) or 8 (K >= 2048) */
    TTS_HIP_OPT_GEMV_NW_MIN = 25, /* lane-layout Q4_K GEMVs: at least `value` waves per workgroup (fewer, fuller workgroups;
                                     0 = default geometry, about one row group per wave over every CU) */
    TTS_HIP_OPT_GEMM_KR_XCD = 38, /* 1: the many-column K-relay GEMM places a row tile's 16-column tiles on one XCD, dispatched
                                     back to back (for the second to stream the weights from that XCD's L2); 0 (default) = grid
                                     order (no gain in HBM bytes or step time) */
    TTS_HIP_OPT_GEMM_KR_CP = 39,  /* 1: the many-column K-relay GEMM (K = 1024 / 2048) gives a workgroup two 16-column tiles on two
                                     parallel wave halves (the weight tile streamed from HBM once for both; 0 = one tile each) */
    TTS_HIP_OPT_GEMM_KR_WALK = 40, /* many-column K-relay GEMMs of more than 4 16-column tiles (prompt passes):
                                      `value` workgroups per column tile, each copying its operand tile once and walking every
                                      `value`-th row tile (the next tile's weights requested before the current tile's relay);
                                      0 = one workgroup per (row tile, column tile) */
    TTS_HIP_OPT_GEMM_PF = 41,     /* many-column Q4_K products (prompt passes) of at least `value` columns (default 64) on the
                                     prefill GEMM: a wave per two 16-row tiles of one 16-column tile over the whole row, ggml's
                                     block chain in registers (no relay); 0 = the K-relay GEMM for every column count */
    TTS_HIP_OPT_GEMM_PF_NW = 42,  /* waves per prefill-GEMM workgroup: 4 (default; 8 row tiles share one operand copy) or 8 (16) */
    TTS_HIP_OPT_COALESCE = 37,    /* 1 (default): while the process-wide coalescer is on (tts_hip_coalesce_enable), this
                                     backend's graph_compute of a one-prompt decode step may join the same step of other
                                     backends on the device as one coalesced launch (tts_hip_coalesce_stats); 0 = never */
};
enum tts_fuse_bits {
    TTS_FUSE_LN = 1, TTS_FUSE_GROUP = 2, TTS_FUSE_KV = 4, TTS_FUSE_EPI = 8, TTS_FUSE_HEADS = 16, TTS_FUSE_ATTN = 32,
    TTS_FUSE_LSTM = 64, /* Kokoro build_lstm_run's unrolled recurrence -> one kernel per step, no O(T^2) concat */
    TTS_FUSE_SNAKE = 128, /* snake_1d's five elementwise nodes -> one pass */
    TTS_FUSE_EMBED = 256, /* an ADD chain over GET_ROWS terms (codebook + positional embeddings) -> one launch */
    TTS_FUSE_CONV = 512,  /* conv_1d's IM2COL -> MUL_MAT (+ bias ADD, + residual ADD) -> one implicit-GEMM kernel */
    TTS_FUSE_ADAIN = 1024, /* Kokoro AdaIN1d (norm, transposes, affine) + snake_1d -> one pass per channel row */
    TTS_FUSE_XATTN = 2048, /* short-context attention (P <= 64) folded into the Q4_K GEMV producing its query */
    TTS_FUSE_MCPY = 4096,  /* CPYs of one source into several views (Orpheus' repeat-interleaved KV store) -> one pass;
                              Dia's repeat_interleave_dim1 view/cont/repeat/concat chain -> one pass */
    TTS_FUSE_CONTREAD = 8192 /* CONT of a contiguous tensor whose only reader is the next node (Orpheus' cont before
                                rope): that node reads the source and the copy is never made */
};
int tts_hip_set_option(tts_hip_backend_t backend, int option, int value);
/* Step coalescer counters of `device` since process start: out[0] coalesced launches, [1] member steps they
 * carried, [2] steps a member ran alone after waiting, [3] groups refused (no coalesced form / mismatched
 * members), [4] the largest group, [5] host microseconds spent waiting for members, [6] coalesced launches whose
 * members were at different KV lengths, [7] host microseconds in the coalesced steps' execution (grouping,
 * layout, plan, tables, launches), [8] of it in the executor layout, [9] planning, [10] tables (co_prepare + upload).
 * Returns the number written. */
int tts_hip_coalesce_stats(int device, int64_t * out, int n);
/* Coalescer rendezvous window (microseconds a step waits for the other active members; default 5000). */
void tts_hip_coalesce_set_wait(int us);
/* The step coalescer, process-wide: one-prompt decode steps of several backends on one device rendezvous and run
 * as one batched plan, also at different KV lengths.  On by default; the environment variable
 * TTS_HIP_COALESCE=0 turns it off at load.  Returns the previous setting. */
int tts_hip_coalesce_enable(int on);
/* Test hooks (process-wide, off by default; never read from the environment):
 * TTS_HIP_HOOK_FAULT_WEIGHT_SET = 1: tts_hip_weight_set of a Q4_K tensor fails (the callers' fallback paths). */
#define TTS_HIP_HOOK_FAULT_WEIGHT_SET 1
int tts_hip_test_hook(int hook, int value);
/* Diagnostics: on SIGSEGV / SIGBUS print the fault address, every frame as library + offset (+ symbol) and
 * the /proc/self/maps lines near the fault, then chain to the previous handler. */
int tts_hip_install_crash_handler(void);
/* Sum of timed GEMV launch durations (ms), launches and algorithmic bytes since last reset, for
 * weight type `type` (-1 = all types). */
int tts_hip_gemv_stats(tts_hip_backend_t backend, int type, double * ms, int64_t * launches, double * bytes, int reset);
/* Greedy sampling on the device for an AR step (stream-ordered, no host round trip): for each
 * (prompt b, head h) row of logits [B][NH][V] the first strict maximum (sampler::max,
 * src/sampler.cpp:185-204) -> hist[b*NH + h]; eos_seen[b*NH + h] |= (token == eos); and the next
 * step's input token (next_decoder_token_ids, src/models/parler/model.cpp:778-785):
 * next[h*B + b] = step + 1 > h ? (eos_seen ? eos : token) : bos. */
int tts_hip_greedy_step(tts_hip_backend_t backend, const float * logits, int32_t B, int32_t NH, int32_t V, int32_t step,
                        int32_t bos, int32_t eos, int32_t * eos_seen, int32_t * hist, int32_t * next);
/* ---- seeded sampling (sampler::sample, /root/reference/src/sampler.cpp:3-62) ----
 * The reference draws from std::minstd_rand(std::random_device{}()) on every call (:47), so its
 * samples cannot be reproduced; here the generator of call c for prompt b is seeded with
 * tts_sampler_call_seed(seed, b, c) and everything else is the reference's arithmetic: repetition
 * penalty (v / pow(penalty, count) in double, for the last token only), temperature (f32 division),
 * max-subtracted expf softmax with a sequential f32 sum (expf = the correctly rounded value, as every
 * transcendental of this backend), top-k by the penalised logits (or by probability after a top-p
 * softmax), top-p trimming, one std::uniform_real_distribution<float> draw per head in head order,
 * then the first pick whose cumulative probability reaches the draw.  Ties in the top-k order go to
 * the lower index (std::sort leaves them unspecified).  do_sample = 0 is sampler::max. */
typedef struct tts_sampling {
    float temperature;        /* 1.0 (generation_configuration defaults, include/common.h:45-66) */
    float top_p;              /* 1.0 */
    float repetition_penalty; /* 1.0 */
    int32_t top_k;            /* 50 */
    int32_t do_sample;        /* 1; 0 = greedy */
    int32_t pad_;
    uint64_t seed;
} tts_sampling;
void tts_sampling_default(tts_sampling * cfg);
/* minstd_rand seed (1 .. 2^31 - 2) of sampler call `call` of prompt `stream`. */
uint32_t tts_sampler_call_seed(uint64_t seed, int32_t stream, int64_t call);
/* Host sampler: one sample() call over NH heads of V logits (logits are not modified); last /
 * count [NH] are the repetition-penalty state (last = -1, count = 0 initially; updated only when
 * the penalty is not 1), out [NH] the tokens. */
int tts_sampler_sample(const tts_sampling * cfg, const float * logits, int32_t NH, int32_t V, uint32_t call_seed, int32_t * last,
                       int32_t * count, int32_t * out);
/* The same on the device for an AR step, followed by greedy_step's EOS / next-token rule:
 * rows [B][NH] of logits [B][NH][V], prompt b's generator seeded with tts_sampler_call_seed(seed, b,
 * call); rep_state [B*NH][2] (last, count) in device memory.  V <= 4096 (Parler, Dia) handles every
 * configuration; wider vocabularies (Orpheus) need 0 < top_k <= 64 and top_p >= 1, else
 * TTS_STATUS_UNSUPPORTED (the runner then samples on the host). */
int tts_hip_sample_step(tts_hip_backend_t backend, const float * logits, int32_t B, int32_t NH, int32_t V, const tts_sampling * cfg,
                        int64_t call, int32_t * rep_state, int32_t step, int32_t bos, int32_t eos, int32_t * eos_seen, int32_t * hist,
                        int32_t * next);
/* Whether tts_hip_sample_step covers (cfg, V): runners sample on the host otherwise. */
int tts_sampling_device_ok(const tts_sampling * cfg, int32_t V);
/* Diagnostic counters since creation: out[0] HIP-graph exec updates, [1] instantiations,
 * [2] fused LSTM chains, [3] fused LSTM steps.  Returns the number written (<= n). */
int tts_hip_counters(tts_hip_backend_t backend, int64_t * out, int n);

/* Raw kernel entry points for micro-benchmarks (device pointers, current backend stream).
 * y[M][N] = W[N][K] . x[M][K]; W is `type` (Q4_K / Q8_0 / F16 / F32) row-major, N rows of K.
 * Q4_K weights must already be in the backend lane layout (tts_repack_q4_K). */
int tts_hip_gemv(tts_hip_backend_t backend, int type, const void * w, const float * x, float * y,
                 int64_t K, int64_t N, int64_t M);
/* As tts_hip_gemv for a weight stored with tts_tensor flags `wflags` (TTS_FLAG_TILED: the tile layout). */
int tts_hip_gemv_ex(tts_hip_backend_t backend, int type, const void * w, const float * x, float * y,
                    int64_t K, int64_t N, int64_t M, int32_t wflags);

/* ---- generic backend vtable: lets the same C++ runners target the HIP backend or the CPU oracle
 * (the latter lives in oracle/ and is only linked by tests and bench.py's cpu_baseline leg). ---- */
typedef struct tts_backend_iface {
    void * ctx;
    const char * name;
    void * (*alloc)(void * ctx, size_t size);
    void (*free)(void * ctx, void * ptr);
    int (*set)(void * ctx, void * dst, const void * src, size_t size);
    int (*set_tensor)(void * ctx, tts_tensor * t, const void * src); /* whole weight tensor */
    int (*get)(void * ctx, void * dst, const void * src, size_t size);
    int (*memset)(void * ctx, void * dst, int value, size_t size);
    int (*compute)(void * ctx, tts_tensor * const * nodes, int n_nodes);
    int (*synchronize)(void * ctx);
    /* optional (NULL = use compute): record into plan slot 0/1 now, launch later */
    int (*prepare)(void * ctx, tts_tensor * const * nodes, int n_nodes, int slot);
    int (*launch)(void * ctx, int slot);
    /* optional (NULL = host sampling path): stream-ordered set / device copy / greedy step */
    int (*set_async)(void * ctx, void * dst, const void * src, size_t size);
    int (*copy)(void * ctx, void * dst, const void * src, size_t size);
    int (*greedy_step)(void * ctx, const float * logits, int B, int NH, int V, int step, int bos, int eos, int32_t * eos_seen,
                       int32_t * hist, int32_t * next);
    /* optional (NULL or TTS_STATUS_UNSUPPORTED = sample on the host): tts_hip_sample_step */
    int (*sample_step)(void * ctx, const float * logits, int B, int NH, int V, const tts_sampling * cfg, int64_t call, int32_t * rep_state,
                       int step, int bos, int eos, int32_t * eos_seen, int32_t * hist, int32_t * next);
} tts_backend_iface;

/* Fills `out` with the HIP backend's vtable. */
int tts_hip_backend_iface(tts_hip_backend_t backend, tts_backend_iface * out);

#ifdef __cplusplus
}
#endif

#endif /* TTS_HIP_H */
