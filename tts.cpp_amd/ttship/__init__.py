"""ctypes binding of libtts_hip.so (include/tts_hip.h, include/tts_runners.h).

The product path is the HIP library; there is no Python or CPU fallback: if the shared object is
missing or no device is visible, the calls below raise.
"""
import ctypes
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
PKG_ROOT = _HERE.parent
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = PKG_ROOT / "lib" / "libtts_hip.so"

# ggml type ids (include/tts_hip.h)
F32, F16, Q4_0, Q8_0, Q4_K, Q8_K, I32 = 0, 1, 2, 8, 12, 15, 26
PROF_ATTN = 39  # tts_hip_gemv_stats slot of the decode attention pair (TTS_PROF_ATTN)

OPS = ["NONE", "DUP", "ADD", "SUB", "MUL", "DIV", "SQR", "SQRT", "SIN", "COS", "SUM_ROWS", "REPEAT",
       "CONCAT", "NORM", "RMS_NORM", "MUL_MAT", "SCALE", "CPY", "CONT", "RESHAPE", "VIEW", "PERMUTE",
       "TRANSPOSE", "GET_ROWS", "SOFT_MAX", "ROPE", "CLAMP", "CONV_TRANSPOSE_1D", "IM2COL", "UPSCALE",
       "PAD", "LEAKY_RELU", "UNARY", "CUMSUM", "MOD", "ROUND", "STFT", "ISTFT", "MAP_CUSTOM3", "MAP_CUSTOM2"]
OP = {n: i for i, n in enumerate(OPS)}
# TTS_FUSE_* bits (include/tts_hip.h); FUSE_ALL is the backend default
FUSE = {"LN": 1, "GROUP": 2, "KV": 4, "EPI": 8, "HEADS": 16, "ATTN": 32, "LSTM": 64, "SNAKE": 128, "EMBED": 256, "CONV": 512, "ADAIN": 1024, "XATTN": 2048, "MCPY": 4096, "CONTREAD": 8192}
FUSE_ALL = sum(FUSE.values())
UNARY = {"ABS": 0, "NEG": 1, "TANH": 2, "RELU": 3, "SIGMOID": 4, "GELU": 5, "SILU": 6, "EXP": 7}

# tts_hip_option ids (include/tts_hip.h)
OPT = {"FUSION": 0, "PROFILE_GEMV": 1, "GRAPHS": 2, "CONV_F32ACC": 3, "CONVT_LDS": 4, "ATTN_SPLIT": 5, "KV_PREFETCH": 6, "KV_PREFETCH_BLOCKS": 7, "Q4K_TILE_BYTES": 8, "GEMV_DEBUG": 10, "GEMV_UNIQUE": 11, "CONV_SPLIT": 12, "GEMV_KS": 13, "ATTN_FUSED": 14, "ATTN_PV16": 15, "Q4K_DUAL_BYTES": 16, "GEMV_RSPLIT": 17, "GEMM_Q8": 18, "BGEMM_F32": 19, "CU_PARTITION": 20, "GEMV_PREQUANT": 21, "GEMV_KRELAY": 22, "ATTN_KS": 23, "ATTN_PV8": 24, "GEMV_NW_MIN": 25, "GEMV_KRELAY_LOOP": 26, "GEMV_Q80_PRO": 27, "GEMV_Q80_SLAB": 28, "GEMV_Q80_RW": 29, "GEMM_Q8_STAGED": 30, "GEMV_KR_INKERNEL": 31, "GEMV_F32_WIDE": 32, "ATTN_PV_MP": 33, "GEMM_KR_NW": 34, "GEMM_KR_INKERNEL": 35, "GEMM_KR_CT2": 36, "COALESCE": 37, "GEMM_KR_XCD": 38, "GEMM_KR_CP": 39, "GEMM_KR_WALK": 40, "GEMM_PF": 41, "GEMM_PF_NW": 42}
ATTN_SPLIT_DEFAULT = 128  # backend default: P >= 128 keys -> split (scores + softmax/P.V) kernels
ATTN_FUSED_ON = 128  # P >= 128 keys -> one 1024-thread launch (k_attn_fused; backend default 0 = off)

TYPE_SIZE = {F32: 4, F16: 2, Q4_K: 144, Q8_0: 34, I32: 4}
BLCK_SIZE = {F32: 1, F16: 1, Q4_K: 256, Q8_0: 32, I32: 1}


class TtsTensor(ctypes.Structure):
    pass


TtsTensor._fields_ = [
    ("type", ctypes.c_int32),
    ("op", ctypes.c_int32),
    ("ne", ctypes.c_int64 * 4),
    ("nb", ctypes.c_uint64 * 4),
    ("op_params", ctypes.c_int32 * 16),
    ("src", ctypes.POINTER(TtsTensor) * 4),
    ("view_src", ctypes.POINTER(TtsTensor)),
    ("view_offs", ctypes.c_uint64),
    ("data", ctypes.c_void_p),
    ("flags", ctypes.c_int32),
    ("pad_", ctypes.c_int32),
    ("name", ctypes.c_char * 64),
]


class BackendIface(ctypes.Structure):
    _fields_ = [
        ("ctx", ctypes.c_void_p),
        ("name", ctypes.c_char_p),
        ("alloc", ctypes.c_void_p),
        ("free", ctypes.c_void_p),
        ("set", ctypes.c_void_p),
        ("set_tensor", ctypes.c_void_p),
        ("get", ctypes.c_void_p),
        ("memset", ctypes.c_void_p),
        ("compute", ctypes.c_void_p),
        ("synchronize", ctypes.c_void_p),
        ("prepare", ctypes.c_void_p),
        ("launch", ctypes.c_void_p),
        ("set_async", ctypes.c_void_p),
        ("copy", ctypes.c_void_p),
        ("greedy_step", ctypes.c_void_p),
        ("sample_step", ctypes.c_void_p),
    ]


class Sampling(ctypes.Structure):
    """tts_sampling (include/tts_hip.h): sampler::sample's configuration + the seed."""
    _fields_ = [
        ("temperature", ctypes.c_float),
        ("top_p", ctypes.c_float),
        ("repetition_penalty", ctypes.c_float),
        ("top_k", ctypes.c_int32),
        ("do_sample", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
    ]


def sampling(**kw):
    """tts_sampling with generation_configuration defaults (top_k 50, temperature 1, sample)."""
    c = Sampling()
    lib().tts_sampling_default(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def call_seed(seed, stream, call):
    return int(lib().tts_sampler_call_seed(seed, stream, call))


def host_sample(cfg, logits, call_seed_, last=None, count=None):
    """Host sampler (tts_sampler_sample) over logits [NH, V]; last / count: int32 arrays updated in
    place (repetition-penalty state).  Returns the NH tokens."""
    import numpy as np
    lg = np.ascontiguousarray(logits, dtype=np.float32)
    NH, V = lg.shape
    out = np.zeros(NH, dtype=np.int32)
    if last is None:
        last = np.full(NH, -1, dtype=np.int32)
    if count is None:
        count = np.zeros(NH, dtype=np.int32)
    st = lib().tts_sampler_sample(ctypes.byref(cfg), lg.ctypes.data, NH, V, call_seed_, last.ctypes.data, count.ctypes.data, out.ctypes.data)
    if st != 0:
        raise RuntimeError(f"tts_sampler_sample failed {st}")
    return out


class ParlerConfig(ctypes.Structure):
    _fields_ = [
        ("n_layers", ctypes.c_int32),
        ("hidden_size", ctypes.c_int32),
        ("n_attn_heads", ctypes.c_int32),
        ("ffn_size", ctypes.c_int32),
        ("n_output_heads", ctypes.c_int32),
        ("output_vocab", ctypes.c_int32),
        ("audio_vocab", ctypes.c_int32),
        ("max_ctx", ctypes.c_int32),
        ("n_encode", ctypes.c_int32),
        ("prompt_vocab", ctypes.c_int32),
        ("max_positions", ctypes.c_int32),
        ("weight_type", ctypes.c_int32),
        ("head_type", ctypes.c_int32),
        ("use_cross_attn", ctypes.c_int32),
        ("batch", ctypes.c_int32),
        ("eos_token", ctypes.c_int32),
        ("bos_token", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("arena_bytes", ctypes.c_uint64),
        ("debug_no_reuse", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
    ]


class OrpheusConfig(ctypes.Structure):
    _fields_ = [
        ("n_layers", ctypes.c_int32),
        ("hidden_size", ctypes.c_int32),
        ("n_attn_heads", ctypes.c_int32),
        ("n_kv_attn_heads", ctypes.c_int32),
        ("head_size", ctypes.c_int32),
        ("ffn_size", ctypes.c_int32),
        ("vocab_size", ctypes.c_int32),
        ("max_ctx", ctypes.c_int32),
        ("weight_type", ctypes.c_int32),
        ("batch", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("arena_bytes", ctypes.c_uint64),
        ("rope_theta", ctypes.c_float),
        ("rope_factor", ctypes.c_float),
        ("rope_low_freq_factor", ctypes.c_float),
        ("rope_high_freq_factor", ctypes.c_float),
        ("rope_original_ctx", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
    ]


class DiaConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_output_heads", "n_encoder_layers", "n_decoder_layers", "encoder_hidden_size", "decoder_hidden_size",
        "encoder_attn_heads", "decoder_attn_heads", "decoder_query_heads", "head_size", "encoder_ffn_size",
        "decoder_ffn_size", "output_vocab_size", "encoder_vocab_size", "max_generation_size",
        "max_encoder_context_length", "weight_type", "head_type")] + [
        ("cfg_scale", ctypes.c_float), ("seed", ctypes.c_uint64), ("arena_bytes", ctypes.c_uint64)]


class DacConfig(ctypes.Structure):
    _fields_ = [
        ("n_codebooks", ctypes.c_int32),
        ("codebook_size", ctypes.c_int32),
        ("codebook_dim", ctypes.c_int32),
        ("latent_dim", ctypes.c_int32),
        ("decoder_dim", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("rates", ctypes.c_int32 * 8),
        ("max_frames", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("arena_bytes", ctypes.c_uint64),
    ]


class SnacConfig(ctypes.Structure):
    _fields_ = [
        ("n_heads", ctypes.c_int32),
        ("codebook_size", ctypes.c_int32),
        ("codebook_dim", ctypes.c_int32),
        ("latent_dim", ctypes.c_int32),
        ("decoder_dim", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("rates", ctypes.c_int32 * 8),
        ("repeats", ctypes.c_int32 * 4),
        ("max_frames", ctypes.c_int32),
        ("debug_no_reuse", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("arena_bytes", ctypes.c_uint64),
    ]


class KokoroGenConfig(ctypes.Structure):
    _fields_ = [
        ("in_channels", ctypes.c_int32),
        ("style_dim", ctypes.c_int32),
        ("n_ups", ctypes.c_int32),
        ("up_rates", ctypes.c_int32 * 4),
        ("up_kernels", ctypes.c_int32 * 4),
        ("n_kernels", ctypes.c_int32),
        ("res_kernels", ctypes.c_int32 * 4),
        ("res_dilations", ctypes.c_int32 * 3),
        ("noise_res_kernels", ctypes.c_int32 * 4),
        ("n_fft", ctypes.c_int32),
        ("hop", ctypes.c_int32),
        ("harmonic_num", ctypes.c_int32),
        ("sample_rate", ctypes.c_float),
        ("sin_amp", ctypes.c_float),
        ("noise_std", ctypes.c_float),
        ("voice_threshold", ctypes.c_float),
        ("max_frames", ctypes.c_int32),
        ("debug_no_reuse", ctypes.c_int32),
        ("weight_type", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("arena_bytes", ctypes.c_uint64),
    ]


class KokoroConfig(ctypes.Structure):
    _fields_ = [
        ("gen", KokoroGenConfig),
        ("n_vocab", ctypes.c_int32),
        ("embd", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("n_heads", ctypes.c_int32),
        ("ffn", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("n_recurrence", ctypes.c_int32),
        ("max_context", ctypes.c_int32),
        ("d_model", ctypes.c_int32),
        ("n_dur_layers", ctypes.c_int32),
        ("max_dur", ctypes.c_int32),
        ("te_kernel", ctypes.c_int32),
        ("te_depth", ctypes.c_int32),
        ("dec_dim", ctypes.c_int32),
        ("asr_res_dim", ctypes.c_int32),
        ("n_decode", ctypes.c_int32),
        ("n_voice_rows", ctypes.c_int32),
        ("max_tokens", ctypes.c_int32),
        ("max_total", ctypes.c_int32),
        ("dur_bias", ctypes.c_float),
        ("f0_mean", ctypes.c_float),
        ("debug_no_reuse", ctypes.c_int32),
        ("weight_type", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("arena_bytes", ctypes.c_uint64),
    ]


_lib = None


class QuantizeParams(ctypes.Structure):
    """tts_quantize_params (quantize_impl.h quantization_params without n_threads)."""
    _fields_ = [("quantize_type", ctypes.c_int32), ("quantize_output_heads", ctypes.c_int32),
                ("quantize_text_embeddings", ctypes.c_int32), ("quantize_cross_attn_kv", ctypes.c_int32),
                ("convert_dac_to_f16", ctypes.c_int32), ("convert_non_quantizable_to_f16", ctypes.c_int32)]


# tts_quantize_rows_fn(ctx, type, x, dst, rows, K)
QUANTIZE_ROWS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int64, ctypes.c_int64)


def row_size(t, ne0):
    return TYPE_SIZE[t] * (ne0 // BLCK_SIZE[t])


def lib():
    """Load libtts_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = LIB_PATH
    variant = os.environ.get("TTS_HIP_LIB_VARIANT")  # build-variant studies (scripts/): lib/<variant>/libtts_hip.so
    if variant:
        path = PKG_ROOT / "lib" / variant / "libtts_hip.so"
    if not path.exists():
        raise RuntimeError(f"{path} missing: run `make -j8` (or __graft_entry__.build())")
    L = ctypes.CDLL(str(path))
    vp, i32, i64, u64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "tts_type_size": (sz, [ctypes.c_int]),
        "tts_blck_size": (i64, [ctypes.c_int]),
        "tts_row_size": (sz, [ctypes.c_int, i64]),
        "tts_type_name": (ctypes.c_char_p, [ctypes.c_int]),
        "tts_op_name": (ctypes.c_char_p, [ctypes.c_int]),
        "tts_hip_device_count": (ctypes.c_int, []),
        "tts_hip_backend_init": (vp, [ctypes.c_int]),
        "tts_hip_backend_free": (None, [vp]),
        "tts_hip_backend_name": (ctypes.c_char_p, [vp]),
        "tts_hip_buffer_alloc": (vp, [vp, sz]),
        "tts_hip_buffer_free": (None, [vp, vp]),
        "tts_hip_buffer_alignment": (sz, []),
        "tts_hip_tensor_set": (ctypes.c_int, [vp, vp, vp, sz]),
        "tts_hip_tensor_get": (ctypes.c_int, [vp, vp, vp, sz]),
        "tts_hip_tensor_copy": (ctypes.c_int, [vp, vp, vp, sz]),
        "tts_hip_copy_stream": (ctypes.c_int, [vp, vp, vp, sz]),
        "tts_hip_memset": (ctypes.c_int, [vp, vp, ctypes.c_int, sz]),
        "tts_hip_synchronize": (ctypes.c_int, [vp]),
        "tts_hip_supports_op": (ctypes.c_int, [ctypes.POINTER(TtsTensor)]),
        "tts_hip_graph_compute": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.POINTER(TtsTensor)), ctypes.c_int]),
        "tts_hip_set_option": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
        "tts_hip_gemv_stats": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64),
                                              ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
        "tts_hip_gemv": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, i64, i64, i64]),
        "tts_hip_gemv_ex": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, i64, i64, i64, i32]),
        "tts_hip_counters": (ctypes.c_int, [vp, ctypes.POINTER(i64), ctypes.c_int]),
        "tts_hip_coalesce_stats": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(i64), ctypes.c_int]),
        "tts_hip_coalesce_set_wait": (None, [ctypes.c_int]),
        "tts_hip_coalesce_enable": (ctypes.c_int, [ctypes.c_int]),
        "tts_hip_test_hook": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
        "tts_hip_install_crash_handler": (ctypes.c_int, []),
        "tts_parler_n_weights": (i32, [vp]),
        "tts_dia_n_weights": (i32, [vp]),
        "tts_dia_weight": (u64, [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(i64), ctypes.POINTER(i32), vp, u64]),
        "tts_parler_weight": (u64, [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(i64), ctypes.POINTER(i32), vp, u64]),
        "tts_orpheus_n_weights": (i32, [vp]),
        "tts_orpheus_weight": (u64, [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(i64), ctypes.POINTER(i32), vp, u64]),
        "tts_dac_n_weights": (i32, [vp]),
        "tts_dac_weight": (u64, [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(i64), ctypes.POINTER(i32), vp, u64]),
        "tts_sampling_default": (None, [ctypes.POINTER(Sampling)]),
        "tts_parler_set_sampling": (None, [vp, ctypes.POINTER(Sampling)]),
        "tts_parler_set_position": (ctypes.c_int, [vp, i32]),
        "tts_dia_set_sampling": (None, [vp, ctypes.POINTER(Sampling)]),
        "tts_orpheus_set_sampling": (None, [vp, ctypes.POINTER(Sampling)]),
        "tts_sampler_call_seed": (ctypes.c_uint32, [ctypes.c_uint64, i32, i64]),
        "tts_sampler_sample": (ctypes.c_int, [ctypes.POINTER(Sampling), vp, i32, i32, ctypes.c_uint32, vp, vp, vp]),
        "tts_hip_sample_step": (ctypes.c_int, [vp, vp, i32, i32, i32, ctypes.POINTER(Sampling), i64, vp, i32, i32, i32, vp, vp, vp]),
        "tts_hip_greedy_step": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
        "tts_hip_backend_iface": (ctypes.c_int, [vp, ctypes.POINTER(BackendIface)]),
        "tts_hip_weight_set": (ctypes.c_int, [vp, ctypes.POINTER(TtsTensor), vp]),
        "tts_hip_quantize": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, i64, i64]),
        "tts_hip_weight_get": (ctypes.c_int, [vp, ctypes.POINTER(TtsTensor), vp]),
        "tts_repack_q4_K": (None, [vp, vp, i64, ctypes.c_int]),
        "tts_repack_q4_K_tiled": (None, [vp, vp, i64, i64, ctypes.c_int]),
        "tts_dia_default_config": (None, [ctypes.POINTER(DiaConfig)]),
        "tts_dia_create": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(DiaConfig)]),
        "tts_dia_free": (None, [vp]),
        "tts_dia_prefill": (ctypes.c_int, [vp, vp, i32, vp, vp]),
        "tts_dia_decode": (ctypes.c_int, [vp, vp, vp]),
        "tts_dia_generate": (ctypes.c_int, [vp, vp, i32, vp]),
        "tts_dia_position": (i32, [vp]),
        "tts_dia_last_graph_nodes": (i32, [vp]),
        "tts_dia_weight_bytes": (u64, [vp]),
        "tts_dia_graph": (vp, [vp, ctypes.POINTER(i32)]),
        "tts_orpheus_default_config": (None, [ctypes.POINTER(OrpheusConfig)]),
        "tts_orpheus_create": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(OrpheusConfig)]),
        "tts_orpheus_free": (None, [vp]),
        "tts_orpheus_reset": (None, [vp]),
        "tts_orpheus_prefill": (ctypes.c_int, [vp, vp, i32, vp]),
        "tts_orpheus_decode": (ctypes.c_int, [vp, vp, vp]),
        "tts_orpheus_generate": (ctypes.c_int, [vp, vp, i32, vp]),
        "tts_orpheus_position": (i32, [vp]),
        "tts_orpheus_last_graph_nodes": (i32, [vp]),
        "tts_orpheus_weight_bytes": (u64, [vp]),
        "tts_orpheus_graph": (vp, [vp, ctypes.POINTER(i32)]),
        "tts_parler_default_config": (None, [ctypes.POINTER(ParlerConfig)]),
        "tts_parler_create": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(ParlerConfig)]),
        "tts_parler_free": (None, [vp]),
        "tts_parler_set_device_sampling": (None, [vp, ctypes.c_int32]),
        "tts_parler_reset": (None, [vp]),
        "tts_parler_prefill": (ctypes.c_int, [vp, vp, i32]),
        "tts_parler_prefill_ragged": (ctypes.c_int, [vp, vp, vp, i32]),
        "tts_parler_decode": (ctypes.c_int, [vp, vp, vp]),
        "tts_parler_generate": (ctypes.c_int, [vp, i32, vp]),
        "tts_parler_position": (i32, [vp]),
        "tts_parler_host_stats": (i64, [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
        "tts_parler_last_graph_nodes": (i32, [vp]),
        "tts_parler_graph": (vp, [vp, ctypes.POINTER(i32)]),
        "tts_parler_weight_bytes": (u64, [vp]),
        "tts_parler_get_node": (u64, [vp, ctypes.c_char_p, vp, u64]),
        "tts_parler_node": (u64, [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i64), vp, u64]),
        "tts_dac_default_config": (None, [ctypes.POINTER(DacConfig)]),
        "tts_dac_create": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(DacConfig)]),
        "tts_dac_free": (None, [vp]),
        "tts_dac_decode": (ctypes.c_int, [vp, vp, i32, vp]),
        "tts_dac_hop": (i64, [vp]),
        "tts_dac_last_graph_nodes": (i32, [vp]),
        "tts_dac_decode_batch": (ctypes.c_int, [vp, vp, i32, i32, i32, vp]),
        "tts_dac_min_gap": (i64, [vp]),
        "tts_dac_graph": (vp, [vp, ctypes.POINTER(i32)]),
        "tts_snac_default_config": (None, [ctypes.POINTER(SnacConfig)]),
        "tts_snac_create": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(SnacConfig)]),
        "tts_snac_free": (None, [vp]),
        "tts_snac_decode": (ctypes.c_int, [vp, vp, i32, vp, vp]),
        "tts_snac_hop": (i64, [vp]),
        "tts_snac_noise_per_frame": (i64, [vp]),
        "tts_snac_last_graph_nodes": (i32, [vp]),
        "tts_snac_n_weights": (i32, [vp]),
        "tts_snac_get_node": (u64, [vp, ctypes.c_char_p, vp, u64]),
        "tts_snac_weight": (u64, [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(ctypes.c_int64), vp, u64]),
        "tts_kokoro_default_config": (None, [ctypes.POINTER(KokoroConfig)]),
        "tts_kokoro_create": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(KokoroConfig)]),
        "tts_kokoro_free": (None, [vp]),
        "tts_kokoro_durations": (ctypes.c_int, [vp, vp, i32, vp, vp]),
        "tts_kokoro_decode": (ctypes.c_int, [vp, vp, i32, vp, vp, vp, vp, u64]),
        "tts_kokoro_run": (ctypes.c_int, [vp, vp, i32, vp, vp, u64, ctypes.POINTER(ctypes.c_int64)]),
        "tts_kokoro_last_graph_nodes": (i32, [vp, i32]),
        "tts_kokoro_n_weights": (i32, [vp]),
        "tts_kokoro_weight": (u64, [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(ctypes.c_int64), vp, u64]),
        "tts_kokoro_get_node": (u64, [vp, i32, ctypes.c_char_p, vp, u64]),
        "tts_kokoro_graph": (vp, [vp, i32, ctypes.POINTER(i32)]),
        "tts_kokoro_gen_default_config": (None, [ctypes.POINTER(KokoroGenConfig)]),
        "tts_kokoro_gen_create": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(KokoroGenConfig)]),
        "tts_kokoro_gen_free": (None, [vp]),
        "tts_kokoro_gen_run": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, vp]),
        "tts_kokoro_gen_samples_per_frame": (i64, [vp]),
        "tts_kokoro_gen_last_graph_nodes": (i32, [vp]),
        "tts_kokoro_gen_n_weights": (i32, [vp]),
        "tts_kokoro_gen_get_node": (u64, [vp, ctypes.c_char_p, vp, u64]),
        "tts_kokoro_gen_node": (u64, [vp, i32, vp, vp, vp, vp, u64]),
        "tts_kokoro_gen_graph": (vp, [vp, ctypes.POINTER(i32)]),
        "tts_hip_plan_stats": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(i32)]),
        "tts_kokoro_gen_weight": (u64, [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(ctypes.c_int64), vp, u64]),
        # GGUF files (include/tts_gguf.h)
        "tts_gguf_open": (vp, [ctypes.c_char_p]),
        "tts_gguf_close": (None, [vp]),
        "tts_gguf_version": (ctypes.c_uint32, [vp]),
        "tts_gguf_alignment": (u64, [vp]),
        "tts_gguf_data_offset": (u64, [vp]),
        "tts_gguf_n_kv": (i64, [vp]),
        "tts_gguf_find_key": (i64, [vp, ctypes.c_char_p]),
        "tts_gguf_key": (ctypes.c_char_p, [vp, i64]),
        "tts_gguf_kv_type": (i32, [vp, i64]),
        "tts_gguf_get_u32": (ctypes.c_int, [vp, i64, ctypes.POINTER(ctypes.c_uint32)]),
        "tts_gguf_get_i64": (ctypes.c_int, [vp, i64, ctypes.POINTER(i64)]),
        "tts_gguf_get_f64": (ctypes.c_int, [vp, i64, ctypes.POINTER(ctypes.c_double)]),
        "tts_gguf_get_str": (ctypes.c_char_p, [vp, i64]),
        "tts_gguf_arr_type": (i32, [vp, i64]),
        "tts_gguf_arr_n": (i64, [vp, i64]),
        "tts_gguf_arr_data": (vp, [vp, i64]),
        "tts_gguf_arr_str": (ctypes.c_char_p, [vp, i64, i64]),
        "tts_gguf_n_tensors": (i64, [vp]),
        "tts_gguf_find_tensor": (i64, [vp, ctypes.c_char_p]),
        "tts_gguf_tensor_name": (ctypes.c_char_p, [vp, i64]),
        "tts_gguf_tensor_type": (i32, [vp, i64]),
        "tts_gguf_tensor_ndims": (i32, [vp, i64, ctypes.POINTER(i64)]),
        "tts_gguf_tensor_offset": (u64, [vp, i64]),
        "tts_gguf_tensor_size": (u64, [vp, i64]),
        "tts_gguf_tensor_data": (vp, [vp, i64]),
        "tts_gguf_type_size": (sz, [i32]),
        "tts_gguf_blck_size": (i64, [i32]),
        "tts_gguf_writer_new": (vp, []),
        "tts_gguf_writer_free": (None, [vp]),
        "tts_gguf_set_u32": (None, [vp, ctypes.c_char_p, ctypes.c_uint32]),
        "tts_gguf_set_i32": (None, [vp, ctypes.c_char_p, i32]),
        "tts_gguf_set_f32": (None, [vp, ctypes.c_char_p, ctypes.c_float]),
        "tts_gguf_set_u64": (None, [vp, ctypes.c_char_p, u64]),
        "tts_gguf_set_bool": (None, [vp, ctypes.c_char_p, ctypes.c_int]),
        "tts_gguf_set_str": (None, [vp, ctypes.c_char_p, ctypes.c_char_p]),
        "tts_gguf_set_arr": (None, [vp, ctypes.c_char_p, i32, vp, i64]),
        "tts_gguf_set_arr_str": (None, [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), i64]),
        "tts_gguf_copy_kv": (None, [vp, vp]),
        "tts_gguf_add_tensor": (ctypes.c_int, [vp, ctypes.c_char_p, i32, i32, ctypes.POINTER(i64), vp, u64]),
        "tts_gguf_writer_write": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "tts_gguf_tensor_rule": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(QuantizeParams)]),
        "tts_gguf_quantize": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(QuantizeParams), vp, vp]),
        "tts_hip_gguf_quantize": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(QuantizeParams)]),
        "tts_parler_config_from_gguf": (ctypes.c_int, [vp, ctypes.POINTER(ParlerConfig)]),
        "tts_parler_create_from_gguf": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(ParlerConfig), vp]),
        "tts_parler_write_synthetic_gguf": (ctypes.c_int, [ctypes.POINTER(ParlerConfig), ctypes.POINTER(DacConfig), ctypes.c_char_p]),
        "tts_dac_config_from_gguf": (ctypes.c_int, [vp, ctypes.POINTER(DacConfig)]),
        "tts_dac_create_from_gguf": (vp, [ctypes.POINTER(BackendIface), ctypes.POINTER(DacConfig), vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    if os.environ.get("TTS_HIP_CRASH_HANDLER") == "1":  # tracing / repro runs: symbolized frames + maps on a fault
        L.tts_hip_install_crash_handler()
    return L


class HipBackend:
    """One device + one HIP stream (tts_hip_backend_t)."""

    def __init__(self, device=0):
        L = lib()
        n = L.tts_hip_device_count()
        if n <= device:
            raise RuntimeError(f"no HIP device {device} (device count {n})")
        self.ptr = L.tts_hip_backend_init(device)
        if not self.ptr:
            raise RuntimeError("tts_hip_backend_init failed")
        self.L = L

    def iface(self, reference_flow=False):
        """The backend vtable.  reference_flow=True keeps only what TTS.cpp's own step loop uses (graph_compute,
        logits read back, host sampler: parler_tts_runner::decode, src/models/parler/model.cpp:648-693): no
        prepared plans, no device sampling -- the path the step coalescer serves."""
        it = BackendIface()
        if self.L.tts_hip_backend_iface(self.ptr, ctypes.byref(it)) != 0:
            raise RuntimeError("tts_hip_backend_iface failed")
        if reference_flow:
            for f in ("prepare", "launch", "set_async", "copy", "greedy_step", "sample_step"):
                setattr(it, f, None)
        return it

    def alloc(self, nbytes):
        p = self.L.tts_hip_buffer_alloc(self.ptr, nbytes)
        if not p:
            raise MemoryError(f"tts_hip_buffer_alloc({nbytes}) failed")
        return p

    def free(self, p):
        self.L.tts_hip_buffer_free(self.ptr, p)

    def set(self, dev, host_arr):
        st = self.L.tts_hip_tensor_set(self.ptr, dev, host_arr.ctypes.data, host_arr.nbytes)
        if st != 0:
            raise RuntimeError(f"tensor_set failed {st}")

    def get(self, host_arr, dev):
        st = self.L.tts_hip_tensor_get(self.ptr, host_arr.ctypes.data, dev, host_arr.nbytes)
        if st != 0:
            raise RuntimeError(f"tensor_get failed {st}")

    def sample_step(self, logits, cfg, call, rep_state=None, step=100, bos=-2, eos=-3, eos_seen=None):
        """tts_hip_sample_step on logits [B, NH, V] (host arrays staged through device buffers).
        Returns (tokens [B, NH], next [NH, B], eos_seen, rep_state)."""
        import numpy as np
        lg = np.ascontiguousarray(logits, dtype=np.float32)
        B, NH, V = lg.shape
        rs = np.ascontiguousarray(rep_state if rep_state is not None else np.tile(np.array([-1, 0], np.int32), B * NH), dtype=np.int32)
        es = np.ascontiguousarray(eos_seen if eos_seen is not None else np.zeros(B * NH, np.int32), dtype=np.int32)
        bufs = [self.alloc(n) for n in (lg.nbytes, rs.nbytes, es.nbytes, B * NH * 4, B * NH * 4)]
        try:
            self.set(bufs[0], lg)
            self.set(bufs[1], rs)
            self.set(bufs[2], es)
            st = self.L.tts_hip_sample_step(self.ptr, bufs[0], B, NH, V, ctypes.byref(cfg), call, bufs[1], step, bos, eos, bufs[2], bufs[3], bufs[4])
            if st != 0:
                raise RuntimeError(f"tts_hip_sample_step failed {st}")
            hist = np.zeros((B, NH), np.int32)
            nxt = np.zeros((NH, B), np.int32)
            self.get(hist, bufs[3])
            self.get(nxt, bufs[4])
            self.get(rs, bufs[1])
            self.get(es, bufs[2])
            return hist, nxt, es, rs
        finally:
            for b in bufs:
                self.free(b)

    def quantize(self, wtype, x):
        """Device quantization of f32 rows x [N][K] to ggml Q4_K / Q8_0 bytes (host array out)."""
        import numpy as np
        x = np.ascontiguousarray(x, dtype=np.float32)
        N, K = x.shape
        rs = K // 256 * 144 if wtype == Q4_K else K // 32 * 34
        dx, dq = self.alloc(x.nbytes), self.alloc(N * rs)
        try:
            self.set(dx, x)
            st = self.L.tts_hip_quantize(self.ptr, wtype, dx, dq, N, K)
            if st != 0:
                raise RuntimeError(f"tts_hip_quantize failed {st}")
            out = np.empty(N * rs, dtype=np.uint8)
            self.get(out, dq)
            return out
        finally:
            self.free(dx)
            self.free(dq)

    def sync(self):
        if self.L.tts_hip_synchronize(self.ptr) != 0:
            raise RuntimeError("synchronize failed")

    def set_option(self, opt, value):
        self.L.tts_hip_set_option(self.ptr, opt, value)

    def gemv_stats(self, wtype=-1, reset=True):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        b = ctypes.c_double()
        self.L.tts_hip_gemv_stats(self.ptr, wtype, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b), 1 if reset else 0)
        return ms.value, n.value, b.value

    def counters(self):
        """{graph_updates, graph_instantiations, lstm_chains, lstm_steps, plan_wait_ns} since creation."""
        out = (ctypes.c_int64 * 8)()
        n = self.L.tts_hip_counters(self.ptr, out, 8)
        keys = ("graph_updates", "graph_instantiations", "lstm_chains", "lstm_steps", "plan_wait_ns",
                "cap_plan_ns", "cap_launch_ns", "cap_update_ns")
        return {keys[i]: int(out[i]) for i in range(n)}

    def close(self):
        if self.ptr:
            self.L.tts_hip_backend_free(self.ptr)
            self.ptr = None


def runner_weights(n_fn, w_fn, ptr):
    """{name: array shaped like torch (reversed ggml ne, leading 1s dropped)} of a runner's F32 / F16 weights
    (tts_parler_weight / tts_orpheus_weight / tts_dac_weight); quantized weights are skipped."""
    import numpy as np
    out = {}
    for i in range(n_fn(ptr)):
        name = ctypes.create_string_buffer(128)
        ne = (ctypes.c_int64 * 4)()
        ty = ctypes.c_int32()
        n = w_fn(ptr, i, name, 128, ne, ctypes.byref(ty), None, 0)
        if ty.value not in (F32, F16):
            continue
        a = np.empty(n, dtype=np.uint8)
        w_fn(ptr, i, name, 128, ne, ctypes.byref(ty), a.ctypes.data, n)
        a = a.view(np.float32 if ty.value == F32 else np.float16).astype(np.float32)
        shape = [int(v) for v in reversed(list(ne))]
        while len(shape) > 1 and shape[0] == 1:
            shape.pop(0)
        out[name.value.decode()] = a.reshape(shape)
    return out


def coalesce_stats(device=0):
    """Step-coalescer counters of `device` (tts_hip_coalesce_stats)."""
    out = (ctypes.c_int64 * 11)()
    n = lib().tts_hip_coalesce_stats(device, out, 11)
    keys = ("launches", "member_steps", "alone", "refused", "max_group", "wait_us", "ragged_launches", "exec_us", "layout_us",
            "plan_us", "tables_us")
    return {keys[i]: int(out[i]) for i in range(max(n, 0))}


def coalesce_set_wait(us):
    lib().tts_hip_coalesce_set_wait(int(us))


def coalesce_enable(on=True):
    """The step coalescer, process-wide (tts_hip_coalesce_enable; on by default, TTS_HIP_COALESCE=0 at
    load turns it off): one-prompt decode steps of backends on one device rendezvous and run as batched
    launches.  Returns the previous setting."""
    return bool(lib().tts_hip_coalesce_enable(1 if on else 0))


def dia_config(**kw):
    cfg = DiaConfig()
    lib().tts_dia_default_config(ctypes.byref(cfg))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


class Dia:
    """Dia-1.6B runner (encoder step + CFG decoder steps) over a backend vtable."""

    def __init__(self, iface, cfg):
        self.L = lib()
        self.cfg = cfg
        self._iface = iface
        self.ptr = self.L.tts_dia_create(ctypes.byref(iface), ctypes.byref(cfg))
        if not self.ptr:
            raise RuntimeError("tts_dia_create failed")

    def prefill(self, text_ids, audio):
        """text_ids: byte tokens of the conditioned prompt (the unconditioned row is all padding 0)."""
        import numpy as np
        c = self.cfg
        T = c.max_encoder_context_length
        t = np.zeros((2, T), dtype=np.int32)
        t[0, :len(text_ids)] = text_ids
        a = np.ascontiguousarray(audio, dtype=np.int32)
        out = np.empty((c.n_output_heads, c.output_vocab_size), dtype=np.float32)
        st = self.L.tts_dia_prefill(self.ptr, t.ctypes.data, len(text_ids), a.ctypes.data, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"prefill failed {st}")
        return out

    def decode(self, audio):
        import numpy as np
        c = self.cfg
        a = np.ascontiguousarray(audio, dtype=np.int32)
        out = np.empty((c.n_output_heads, c.output_vocab_size), dtype=np.float32)
        st = self.L.tts_dia_decode(self.ptr, a.ctypes.data, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"decode failed {st}")
        return out

    def generate(self, first_audio, n_steps):
        import numpy as np
        a = np.ascontiguousarray(first_audio, dtype=np.int32)
        out = np.empty((n_steps, self.cfg.n_output_heads), dtype=np.int32)
        st = self.L.tts_dia_generate(self.ptr, a.ctypes.data, n_steps, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"generate failed {st}")
        return out

    def set_sampling(self, cfg=None):
        """Seeded sampling (ttship.sampling(...)) for generate(); None = greedy."""
        self._samp = cfg
        self.L.tts_dia_set_sampling(self.ptr, ctypes.byref(cfg) if cfg is not None else None)

    def position(self):
        return self.L.tts_dia_position(self.ptr)

    def weight_bytes(self):
        return self.L.tts_dia_weight_bytes(self.ptr)

    def weights(self):
        return runner_weights(self.L.tts_dia_n_weights, self.L.tts_dia_weight, self.ptr)

    def plan_stats(self, mask=None):
        n = ctypes.c_int32()
        p = self.L.tts_dia_graph(self.ptr, ctypes.byref(n))
        return plan_stats(p, n.value, FUSE_ALL if mask is None else mask)

    def close(self):
        if self.ptr:
            self.L.tts_dia_free(self.ptr)
            self.ptr = None


def orpheus_config(**kw):
    cfg = OrpheusConfig()
    lib().tts_orpheus_default_config(ctypes.byref(cfg))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


class Orpheus:
    """Orpheus-3B decoder runner over a backend vtable (HIP, or the oracle in tests)."""

    def __init__(self, iface, cfg):
        self.L = lib()
        self.cfg = cfg
        self._iface = iface
        self.ptr = self.L.tts_orpheus_create(ctypes.byref(iface), ctypes.byref(cfg))
        if not self.ptr:
            raise RuntimeError("tts_orpheus_create failed")

    def prefill(self, tokens, want_logits=True):
        import numpy as np
        tok = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.empty((self.cfg.batch, self.cfg.vocab_size), dtype=np.float32) if want_logits else None
        st = self.L.tts_orpheus_prefill(self.ptr, tok.ctypes.data, tok.shape[-1], out.ctypes.data if out is not None else None)
        if st != 0:
            raise RuntimeError(f"prefill failed {st}")
        return out

    def decode(self, tokens):
        import numpy as np
        tok = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.empty((self.cfg.batch, self.cfg.vocab_size), dtype=np.float32)
        st = self.L.tts_orpheus_decode(self.ptr, tok.ctypes.data, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"decode failed {st}")
        return out

    def generate(self, first_tokens, n_steps):
        import numpy as np
        ft = np.ascontiguousarray(first_tokens, dtype=np.int32)
        out = np.empty((self.cfg.batch, n_steps), dtype=np.int32)
        st = self.L.tts_orpheus_generate(self.ptr, ft.ctypes.data, n_steps, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"generate failed {st}")
        return out

    def set_sampling(self, cfg=None):
        """Seeded sampling (ttship.sampling(...)) for generate(); None = greedy."""
        self._samp = cfg
        self.L.tts_orpheus_set_sampling(self.ptr, ctypes.byref(cfg) if cfg is not None else None)

    def position(self):
        return self.L.tts_orpheus_position(self.ptr)

    def last_graph_nodes(self):
        return self.L.tts_orpheus_last_graph_nodes(self.ptr)

    def weight_bytes(self):
        return self.L.tts_orpheus_weight_bytes(self.ptr)

    def weights(self):
        return runner_weights(self.L.tts_orpheus_n_weights, self.L.tts_orpheus_weight, self.ptr)

    def plan_stats(self, mask=None):
        """Fusion coverage of the last step graph (no device needed)."""
        n = ctypes.c_int32()
        p = self.L.tts_orpheus_graph(self.ptr, ctypes.byref(n))
        return plan_stats(p, n.value, FUSE_ALL if mask is None else mask)

    def close(self):
        if self.ptr:
            self.L.tts_orpheus_free(self.ptr)
            self.ptr = None


def parler_config(**kw):
    cfg = ParlerConfig()
    lib().tts_parler_default_config(ctypes.byref(cfg))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


class Parler:
    """Parler-TTS decoder runner over a backend vtable (HIP, or the oracle in tests)."""

    def __init__(self, iface, cfg, gguf=None):
        """gguf: a Gguf file whose "decoder.*" tensors are the weights (cfg from parler_config_from_gguf)."""
        import numpy as np  # noqa: F401
        self.L = lib()
        self.cfg = cfg
        self._iface = iface  # keep alive
        if gguf is None:
            self.ptr = self.L.tts_parler_create(ctypes.byref(iface), ctypes.byref(cfg))
        else:
            self.ptr = self.L.tts_parler_create_from_gguf(ctypes.byref(iface), ctypes.byref(cfg), gguf.ptr)
        if not self.ptr:
            raise RuntimeError("tts_parler_create failed")

    def prefill(self, tokens):
        import numpy as np
        tok = np.ascontiguousarray(tokens, dtype=np.int32)
        n = tok.shape[-1]
        st = self.L.tts_parler_prefill(self.ptr, tok.ctypes.data, n)
        if st != 0:
            raise RuntimeError(f"prefill failed {st}")

    def prefill_ragged(self, prompts):
        """One prompt pass over cfg.batch prompts of different lengths (tts_parler_prefill_ragged): a list of
        1-D id arrays, one per sequence."""
        import numpy as np
        lens = np.asarray([len(q) for q in prompts], dtype=np.int32)
        n_max = int(lens.max())
        tok = np.zeros((len(prompts), n_max), dtype=np.int32)
        for b, q in enumerate(prompts):
            tok[b, :len(q)] = q
        st = self.L.tts_parler_prefill_ragged(self.ptr, tok.ctypes.data, lens.ctypes.data, n_max)
        if st != 0:
            raise RuntimeError(f"prefill_ragged failed {st}")

    def decode(self, audio_tokens):
        import numpy as np
        c = self.cfg
        tok = np.ascontiguousarray(audio_tokens, dtype=np.int32)
        out = np.empty((c.batch, c.n_output_heads, c.output_vocab), dtype=np.float32)
        st = self.L.tts_parler_decode(self.ptr, tok.ctypes.data, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"decode failed {st}")
        return out

    def generate(self, n_steps):
        import numpy as np
        c = self.cfg
        out = np.empty((c.batch, n_steps, c.n_output_heads), dtype=np.int32)
        st = self.L.tts_parler_generate(self.ptr, n_steps, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"generate failed {st}")
        return out

    def reset(self):
        self.L.tts_parler_reset(self.ptr)

    def set_device_sampling(self, on):
        """Greedy sampling on the device (default when the backend supports it) or on the host."""
        self.L.tts_parler_set_device_sampling(self.ptr, 1 if on else 0)

    def set_position(self, position):
        """Timing harness only: continue as if `position` tokens had been decoded."""
        if self.L.tts_parler_set_position(self.ptr, position) != 0:
            raise RuntimeError("set_position failed")

    def set_sampling(self, cfg=None):
        """Seeded sampling (ttship.sampling(...)) for generate(); None = greedy."""
        self._samp = cfg
        self.L.tts_parler_set_sampling(self.ptr, ctypes.byref(cfg) if cfg is not None else None)

    @property
    def position(self):
        return self.L.tts_parler_position(self.ptr)

    def last_graph_nodes(self):
        return self.L.tts_parler_last_graph_nodes(self.ptr)

    def plan_stats(self, mask=None):
        """Fusion coverage of the last step graph (no device needed)."""
        n = ctypes.c_int32()
        p = self.L.tts_parler_graph(self.ptr, ctypes.byref(n))
        return plan_stats(p, n.value, FUSE_ALL if mask is None else mask)

    def host_stats(self, reset=True):
        """Mean host microseconds per step: build, alloc, set_inputs, compute enqueue, logits wait."""
        us = (ctypes.c_double * 5)()
        n = self.L.tts_parler_host_stats(self.ptr, us, 1 if reset else 0)
        names = ["build", "alloc", "set_inputs", "compute_enqueue", "logits_wait"]
        return {k: round(us[i] / max(n, 1), 1) for i, k in enumerate(names)}

    def node(self, i, cap=1 << 26):
        """(op, type, ne, float32 array or None) of node i of the last step graph (debugging)."""
        import numpy as np
        op, ty = ctypes.c_int32(), ctypes.c_int32()
        ne = (ctypes.c_int64 * 4)()
        buf = np.empty(cap // 4, dtype=np.float32)
        n = self.L.tts_parler_node(self.ptr, i, ctypes.byref(op), ctypes.byref(ty), ne, buf.ctypes.data, cap)
        data = buf[: n // 4].copy() if n else None
        return OPS[op.value], ty.value, tuple(ne), data

    def weight_bytes(self):
        return self.L.tts_parler_weight_bytes(self.ptr)

    def weights(self):
        return runner_weights(self.L.tts_parler_n_weights, self.L.tts_parler_weight, self.ptr)

    def close(self):
        if self.ptr:
            self.L.tts_parler_free(self.ptr)
            self.ptr = None


def dac_config(**kw):
    cfg = DacConfig()
    lib().tts_dac_default_config(ctypes.byref(cfg))
    for k, v in kw.items():
        if k == "rates":
            for i, r in enumerate(v):
                cfg.rates[i] = r
        else:
            setattr(cfg, k, v)
    return cfg


class Dac:
    """DAC decoder runner (codec tokens -> PCM) over a backend vtable (HIP, or the oracle in tests)."""

    def __init__(self, iface, cfg, gguf=None):
        """gguf: a Gguf file whose "audio_encoder.*" tensors are the weights (cfg from dac_config_from_gguf)."""
        self.L = lib()
        self.cfg = cfg
        self._iface = iface
        if gguf is None:
            self.ptr = self.L.tts_dac_create(ctypes.byref(iface), ctypes.byref(cfg))
        else:
            self.ptr = self.L.tts_dac_create_from_gguf(ctypes.byref(iface), ctypes.byref(cfg), gguf.ptr)
        if not self.ptr:
            raise RuntimeError("tts_dac_create failed")

    @property
    def hop(self):
        return self.L.tts_dac_hop(self.ptr)

    def weights(self):
        return runner_weights(self.L.tts_dac_n_weights, self.L.tts_dac_weight, self.ptr)

    def decode(self, codes):
        """codes: (T, n_codebooks) int -> (T * hop,) float32 PCM."""
        import numpy as np
        c = np.ascontiguousarray(codes, dtype=np.int32)
        T = c.shape[0]
        pcm = np.empty(T * self.hop, dtype=np.float32)
        st = self.L.tts_dac_decode(self.ptr, c.ctypes.data, T, pcm.ctypes.data)
        if st != 0:
            raise RuntimeError(f"tts_dac_decode failed {st}")
        return pcm

    def decode_batch(self, codes, gap=0):
        """codes: (nb, T, n_codebooks) int -> (nb, T * hop) float32 PCM, one graph for all nb prompts
        (tts_dac_decode_batch: bit-identical to nb decode() calls)."""
        import numpy as np
        c = np.ascontiguousarray(codes, dtype=np.int32)
        nb, T = c.shape[0], c.shape[1]
        pcm = np.empty((nb, T * self.hop), dtype=np.float32)
        st = self.L.tts_dac_decode_batch(self.ptr, c.ctypes.data, nb, T, gap, pcm.ctypes.data)
        if st != 0:
            raise RuntimeError(f"tts_dac_decode_batch failed {st}")
        return pcm

    @property
    def min_gap(self):
        return self.L.tts_dac_min_gap(self.ptr)

    def plan_stats(self, mask=None):
        """Fusion coverage of the last decode graph (no device needed)."""
        n = ctypes.c_int32()
        p = self.L.tts_dac_graph(self.ptr, ctypes.byref(n))
        return plan_stats(p, n.value, FUSE_ALL if mask is None else mask)

    def last_graph_nodes(self):
        return self.L.tts_dac_last_graph_nodes(self.ptr)

    def close(self):
        if self.ptr:
            self.L.tts_dac_free(self.ptr)
            self.ptr = None


def snac_config(**kw):
    cfg = SnacConfig()
    lib().tts_snac_default_config(ctypes.byref(cfg))
    for k, v in kw.items():
        if k in ("rates", "repeats"):
            for i, r in enumerate(v):
                getattr(cfg, k)[i] = r
        else:
            setattr(cfg, k, v)
    return cfg


class Snac:
    """SNAC decoder runner (Orpheus' three codebook streams -> 24 kHz PCM) over a backend vtable."""

    def __init__(self, iface, cfg):
        self.L = lib()
        self.cfg = cfg
        self._iface = iface
        self.ptr = self.L.tts_snac_create(ctypes.byref(iface), ctypes.byref(cfg))
        if not self.ptr:
            raise RuntimeError("tts_snac_create failed")

    @property
    def hop(self):
        return self.L.tts_snac_hop(self.ptr)

    @property
    def noise_per_frame(self):
        return self.L.tts_snac_noise_per_frame(self.ptr)

    def decode(self, heads, noise):
        """heads: list of n_heads int arrays (head i: T / repeats[i] codes); noise: (noise_per_frame * T,)
        float32 normal draws -> (T * hop,) float32 PCM."""
        import numpy as np
        T = len(heads[-1])
        c = np.ascontiguousarray(np.concatenate([np.asarray(h, dtype=np.int32) for h in heads]))
        z = np.ascontiguousarray(noise, dtype=np.float32)
        if z.size != self.noise_per_frame * T:
            raise ValueError(f"noise needs {self.noise_per_frame * T} values")
        pcm = np.empty(T * self.hop, dtype=np.float32)
        st = self.L.tts_snac_decode(self.ptr, c.ctypes.data, T, z.ctypes.data, pcm.ctypes.data)
        if st != 0:
            raise RuntimeError(f"tts_snac_decode failed {st}")
        return pcm

    def last_graph_nodes(self):
        return self.L.tts_snac_last_graph_nodes(self.ptr)

    def node(self, name, cap=1 << 26):
        """Named node of the last decode as a flat float32 array (ggml order), or None."""
        import numpy as np
        buf = np.empty(cap // 4, dtype=np.float32)
        n = self.L.tts_snac_get_node(self.ptr, name.encode(), buf.ctypes.data, cap)
        return buf[: n // 4].copy() if n else None

    def weights(self):
        """{name: float32 array shaped like torch (reversed ggml ne, leading 1s dropped)}."""
        import numpy as np
        out = {}
        for i in range(self.L.tts_snac_n_weights(self.ptr)):
            name = ctypes.create_string_buffer(128)
            ne = (ctypes.c_int64 * 4)()
            n = self.L.tts_snac_weight(self.ptr, i, name, 128, ne, None, 0)
            a = np.empty(n // 4, dtype=np.float32)
            self.L.tts_snac_weight(self.ptr, i, name, 128, ne, a.ctypes.data, n)
            shape = [int(v) for v in reversed(list(ne))]
            while len(shape) > 1 and shape[0] == 1:
                shape.pop(0)
            out[name.value.decode()] = a.reshape(shape)
        return out

    def close(self):
        if self.ptr:
            self.L.tts_snac_free(self.ptr)
            self.ptr = None


def kokoro_gen_config(**kw):
    cfg = KokoroGenConfig()
    lib().tts_kokoro_gen_default_config(ctypes.byref(cfg))
    for k, v in kw.items():
        if isinstance(v, (list, tuple)):
            arr = getattr(cfg, k)
            for i, r in enumerate(v):
                arr[i] = r
        else:
            setattr(cfg, k, v)
    return cfg


def kokoro_config(gen=None, **kw):
    """tts_kokoro_config with Kokoro-82M defaults; gen = dict of generator fields."""
    cfg = KokoroConfig()
    lib().tts_kokoro_default_config(ctypes.byref(cfg))
    for k, v in (gen or {}).items():
        if isinstance(v, (list, tuple)):
            arr = getattr(cfg.gen, k)
            for i, r in enumerate(v):
                arr[i] = r
        else:
            setattr(cfg.gen, k, v)
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


class Kokoro:
    """Kokoro-82M end to end (phoneme ids -> durations -> 24 kHz PCM) over a backend vtable."""

    def __init__(self, iface, cfg):
        self.L = lib()
        self.cfg = cfg
        self._iface = iface
        self.ptr = self.L.tts_kokoro_create(ctypes.byref(iface), ctypes.byref(cfg))
        if not self.ptr:
            raise RuntimeError("tts_kokoro_create failed")

    def durations(self, tokens):
        """tokens (n,) int -> (hidden (n, d_model + style), lengths (n,))."""
        import numpy as np
        t = np.ascontiguousarray(tokens, dtype=np.int32)
        n = t.shape[0]
        hidden = np.empty((n, self.cfg.d_model + self.cfg.gen.style_dim), dtype=np.float32)
        lens = np.empty(n, dtype=np.float32)
        st = self.L.tts_kokoro_durations(self.ptr, t.ctypes.data, n, hidden.ctypes.data, lens.ctypes.data)
        if st != 0:
            raise RuntimeError(f"tts_kokoro_durations failed {st}")
        return hidden, lens

    def decode(self, tokens, hidden, lengths, rand=None):
        """-> (600 * sum(lengths),) float32 PCM; rand (harmonic_num + 1, 600 * total) or None."""
        import numpy as np
        t = np.ascontiguousarray(tokens, dtype=np.int32)
        hidden = np.ascontiguousarray(hidden, dtype=np.float32)
        lengths = np.ascontiguousarray(lengths, dtype=np.float32)
        total = int(sum(int(v) for v in lengths))
        pcm = np.empty(600 * total, dtype=np.float32)
        rp = None
        if rand is not None:
            rand = np.ascontiguousarray(rand, dtype=np.float32)
            assert rand.shape == (self.cfg.gen.harmonic_num + 1, 600 * total)
            rp = rand.ctypes.data
        st = self.L.tts_kokoro_decode(self.ptr, t.ctypes.data, t.shape[0], hidden.ctypes.data, lengths.ctypes.data, rp,
                                      pcm.ctypes.data, pcm.nbytes)
        if st != 0:
            raise RuntimeError(f"tts_kokoro_decode failed {st}")
        return pcm

    def run(self, tokens, rand=None, max_samples=None):
        """Both graphs (kokoro_runner::run) -> PCM."""
        import numpy as np
        t = np.ascontiguousarray(tokens, dtype=np.int32)
        cap = max_samples or 600 * self.cfg.max_total
        pcm = np.empty(cap, dtype=np.float32)
        ns = ctypes.c_int64()
        rp = None
        if rand is not None:
            rand = np.ascontiguousarray(rand, dtype=np.float32)
            rp = rand.ctypes.data
        st = self.L.tts_kokoro_run(self.ptr, t.ctypes.data, t.shape[0], rp, pcm.ctypes.data, pcm.nbytes, ctypes.byref(ns))
        if st != 0:
            raise RuntimeError(f"tts_kokoro_run failed {st}")
        return pcm[: ns.value]

    def weights(self):
        """{name: float32 array shaped like torch (reversed ggml ne, leading 1s dropped)}."""
        import numpy as np
        out = {}
        for i in range(self.L.tts_kokoro_n_weights(self.ptr)):
            name = ctypes.create_string_buffer(128)
            ne = (ctypes.c_int64 * 4)()
            n = self.L.tts_kokoro_weight(self.ptr, i, name, 128, ne, None, 0)
            a = np.empty(n // 4, dtype=np.float32)
            self.L.tts_kokoro_weight(self.ptr, i, name, 128, ne, a.ctypes.data, n)
            shape = [int(v) for v in reversed(list(ne))]
            while len(shape) > 1 and shape[0] == 1:
                shape.pop(0)
            out[name.value.decode()] = a.reshape(shape)
        return out

    def node(self, name, which=1):
        """float32 values of a named node of the last duration (0) / main (1) graph, or None."""
        import numpy as np
        n = self.L.tts_kokoro_get_node(self.ptr, which, name.encode(), None, 0)
        if not n:
            return None
        a = np.empty(n // 4, dtype=np.float32)
        self.L.tts_kokoro_get_node(self.ptr, which, name.encode(), a.ctypes.data, n)
        return a

    def plan_stats(self, which=1, mask=None):
        n = ctypes.c_int32()
        p = self.L.tts_kokoro_graph(self.ptr, which, ctypes.byref(n))
        return plan_stats(p, n.value, FUSE_ALL if mask is None else mask)

    def last_graph_nodes(self, which=1):
        return self.L.tts_kokoro_last_graph_nodes(self.ptr, which)

    def close(self):
        if self.ptr:
            self.L.tts_kokoro_free(self.ptr)
            self.ptr = None


class KokoroGenerator:
    """Kokoro iSTFTNet generator runner (features + F0 + style -> PCM) over a backend vtable."""

    def __init__(self, iface, cfg):
        self.L = lib()
        self.cfg = cfg
        self._iface = iface
        self.ptr = self.L.tts_kokoro_gen_create(ctypes.byref(iface), ctypes.byref(cfg))
        if not self.ptr:
            raise RuntimeError("tts_kokoro_gen_create failed")

    @property
    def samples_per_frame(self):
        return self.L.tts_kokoro_gen_samples_per_frame(self.ptr)

    def run(self, x, f0, style, rand=None, out=None):
        """x: (T, in_channels), f0: (T,), style: (style_dim,), rand: (harmonic_num+1, 300*T) or
        None -> (300*T,) float32 PCM."""
        import numpy as np
        x = np.ascontiguousarray(x, dtype=np.float32)
        f0 = np.ascontiguousarray(f0, dtype=np.float32)
        style = np.ascontiguousarray(style, dtype=np.float32)
        T = x.shape[0]
        assert x.shape[1] == self.cfg.in_channels and f0.shape == (T,) and style.shape == (self.cfg.style_dim,)
        rp = None
        if rand is not None:
            rand = np.ascontiguousarray(rand, dtype=np.float32)
            assert rand.shape == (self.cfg.harmonic_num + 1, T * self.samples_per_frame)
            rp = rand.ctypes.data
        pcm = out if out is not None else np.empty(T * self.samples_per_frame, dtype=np.float32)
        st = self.L.tts_kokoro_gen_run(self.ptr, x.ctypes.data, f0.ctypes.data, style.ctypes.data, rp, T,
                                       pcm.ctypes.data if pcm is not None else None)
        if st != 0:
            raise RuntimeError(f"tts_kokoro_gen_run failed {st}")
        return pcm

    def weights(self):
        """{name: float32 array shaped like torch (reversed ggml ne, leading 1s dropped)}."""
        import numpy as np
        out = {}
        for i in range(self.L.tts_kokoro_gen_n_weights(self.ptr)):
            name = ctypes.create_string_buffer(128)
            ne = (ctypes.c_int64 * 4)()
            n = self.L.tts_kokoro_gen_weight(self.ptr, i, name, 128, ne, None, 0)
            a = np.empty(n // 4, dtype=np.float32)
            self.L.tts_kokoro_gen_weight(self.ptr, i, name, 128, ne, a.ctypes.data, n)
            shape = [int(v) for v in reversed(list(ne))]
            while len(shape) > 1 and shape[0] == 1:
                shape.pop(0)
            out[name.value.decode()] = a.reshape(shape)
        return out

    def node_at(self, i, cap=1 << 26):
        """(op, type, ne, float32 array or None) of node i of the last graph (debugging)."""
        import numpy as np
        op, ty = ctypes.c_int32(), ctypes.c_int32()
        ne = (ctypes.c_int64 * 4)()
        buf = np.empty(cap // 4, dtype=np.float32)
        n = self.L.tts_kokoro_gen_node(self.ptr, i, ctypes.byref(op), ctypes.byref(ty), ne, buf.ctypes.data, cap)
        return OPS[op.value], ty.value, tuple(ne), (buf[: n // 4].copy() if n else None)

    def plan_stats(self, mask=None):
        """Fusion coverage of the last graph (no device needed): {item kind: count, "unfused": n}."""
        return plan_stats(*self._graph(), FUSE_ALL if mask is None else mask)

    def _graph(self):
        n = ctypes.c_int32()
        p = self.L.tts_kokoro_gen_graph(self.ptr, ctypes.byref(n))
        return p, n.value

    def node(self, name):
        """float32 values of a named node of the last run (flat), or None."""
        import numpy as np
        n = self.L.tts_kokoro_gen_get_node(self.ptr, name.encode(), None, 0)
        if not n:
            return None
        a = np.empty(n // 4, dtype=np.float32)
        self.L.tts_kokoro_gen_get_node(self.ptr, name.encode(), a.ctypes.data, n)
        return a

    def last_graph_nodes(self):
        return self.L.tts_kokoro_gen_last_graph_nodes(self.ptr)

    def close(self):
        if self.ptr:
            self.L.tts_kokoro_gen_free(self.ptr)
            self.ptr = None


PLAN_KINDS = ["gemv", "attn", "ln", "lstm", "snake", "embed", "conv", "adain", "mcpy", "rint", "node", "copy"]


def plan_stats(nodes_ptr, n_nodes, mask):
    """tts_hip_plan_stats over a node array: {kind: items, "unfused": nodes launched one by one}."""
    counts = (ctypes.c_int32 * 16)()
    lib().tts_hip_plan_stats(nodes_ptr, n_nodes, mask, counts)
    out = {k: int(counts[i]) for i, k in enumerate(PLAN_KINDS)}
    out["gemv_products"] = int(counts[12])
    out["gemv_max_group"] = int(counts[13])
    out["xattn"] = int(counts[14])
    out["unfused"] = int(counts[15])
    return out


# ---- GGUF files (include/tts_gguf.h) ----
GGUF_TYPES = {"u8": 0, "i8": 1, "u16": 2, "i16": 3, "u32": 4, "i32": 5, "f32": 6, "bool": 7, "str": 8, "arr": 9, "u64": 10,
              "i64": 11, "f64": 12}
_GGUF_NP = {0: "u1", 1: "i1", 2: "<u2", 3: "<i2", 4: "<u4", 5: "<i4", 6: "<f4", 7: "u1", 10: "<u8", 11: "<i8", 12: "<f8"}


class Gguf:
    """A GGUF file mapped read-only (gguf_init_from_file + llama_mmap)."""

    def __init__(self, path):
        self.L = lib()
        self.ptr = self.L.tts_gguf_open(str(path).encode())
        if not self.ptr:
            raise RuntimeError(f"cannot read GGUF file {path}")

    @property
    def version(self):
        return self.L.tts_gguf_version(self.ptr)

    @property
    def alignment(self):
        return self.L.tts_gguf_alignment(self.ptr)

    @property
    def data_offset(self):
        return self.L.tts_gguf_data_offset(self.ptr)

    def keys(self):
        return [self.L.tts_gguf_key(self.ptr, i).decode() for i in range(self.L.tts_gguf_n_kv(self.ptr))]

    def get(self, key, default=None):
        """Value of a key: int / float / bool / str, or a list / numpy array for arrays."""
        import numpy as np
        L, g = self.L, self.ptr
        i = L.tts_gguf_find_key(g, key.encode())
        if i < 0:
            return default
        t = L.tts_gguf_kv_type(g, i)
        if t == 8:
            return L.tts_gguf_get_str(g, i).decode()
        if t == 9:
            at, n = L.tts_gguf_arr_type(g, i), L.tts_gguf_arr_n(g, i)
            if at == 8:
                return [L.tts_gguf_arr_str(g, i, j).decode() for j in range(n)]
            dt = np.dtype(_GGUF_NP[at])
            buf = (ctypes.c_char * (n * dt.itemsize)).from_address(L.tts_gguf_arr_data(g, i)) if n else b""
            return np.frombuffer(bytes(buf), dtype=dt).copy()
        if t in (6, 12):
            v = ctypes.c_double()
            L.tts_gguf_get_f64(g, i, ctypes.byref(v))
            return v.value
        v = ctypes.c_int64()
        L.tts_gguf_get_i64(g, i, ctypes.byref(v))
        return bool(v.value) if t == 7 else v.value

    def tensors(self):
        """[(name, type, ne (4), offset, nbytes)] in file order."""
        L, g = self.L, self.ptr
        out = []
        for i in range(L.tts_gguf_n_tensors(g)):
            ne = (ctypes.c_int64 * 4)()
            nd = L.tts_gguf_tensor_ndims(g, i, ne)
            out.append((L.tts_gguf_tensor_name(g, i).decode(), L.tts_gguf_tensor_type(g, i), tuple(ne[:nd]),
                        L.tts_gguf_tensor_offset(g, i), L.tts_gguf_tensor_size(g, i)))
        return out

    def tensor_bytes(self, name):
        """The tensor's bytes (a copy of the mapping) as uint8."""
        import numpy as np
        i = self.L.tts_gguf_find_tensor(self.ptr, name.encode())
        if i < 0:
            raise KeyError(name)
        n = self.L.tts_gguf_tensor_size(self.ptr, i)
        return np.frombuffer(bytes((ctypes.c_char * n).from_address(self.L.tts_gguf_tensor_data(self.ptr, i))), dtype=np.uint8)

    def tensor_type(self, name):
        i = self.L.tts_gguf_find_tensor(self.ptr, name.encode())
        return None if i < 0 else self.L.tts_gguf_tensor_type(self.ptr, i)

    def close(self):
        if self.ptr:
            self.L.tts_gguf_close(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class GgufWriter:
    """gguf_init_empty / gguf_set_* / gguf_add_tensor / gguf_write_to_file."""

    def __init__(self):
        self.L = lib()
        self.ptr = self.L.tts_gguf_writer_new()

    def set(self, key, value, kind=None):
        """kind: u32 (int default), i32, u64, f32 (float default), bool, str, or ("arr", elem kind) for lists."""
        import numpy as np
        k, L, w = key.encode(), self.L, self.ptr
        if isinstance(value, (list, tuple, np.ndarray)):
            ek = kind[1] if isinstance(kind, tuple) else ("str" if value and isinstance(value[0], str) else "i32")
            if ek == "str":
                arr = (ctypes.c_char_p * len(value))(*[v.encode() for v in value])
                L.tts_gguf_set_arr_str(w, k, arr, len(value))
            else:
                a = np.ascontiguousarray(value, dtype=np.dtype(_GGUF_NP[GGUF_TYPES[ek]]))
                L.tts_gguf_set_arr(w, k, GGUF_TYPES[ek], a.ctypes.data, a.size)
            return
        kind = kind or ("bool" if isinstance(value, bool) else "str" if isinstance(value, str) else
                        "f32" if isinstance(value, float) else "u32")
        fn = {"u32": L.tts_gguf_set_u32, "i32": L.tts_gguf_set_i32, "u64": L.tts_gguf_set_u64, "f32": L.tts_gguf_set_f32,
              "bool": L.tts_gguf_set_bool, "str": L.tts_gguf_set_str}[kind]
        fn(w, k, value.encode() if kind == "str" else value)

    def copy_kv(self, g):
        self.L.tts_gguf_copy_kv(self.ptr, g.ptr)

    def add_tensor(self, name, ttype, ne, data):
        import numpy as np
        d = np.ascontiguousarray(data)
        ne_a = (ctypes.c_int64 * len(ne))(*ne)
        st = self.L.tts_gguf_add_tensor(self.ptr, name.encode(), ttype, len(ne), ne_a, d.ctypes.data, d.nbytes)
        if st != 0:
            raise ValueError(f"add_tensor({name}) failed {st}")

    def write(self, path):
        if self.L.tts_gguf_writer_write(self.ptr, str(path).encode()) != 0:
            raise RuntimeError(f"writing {path} failed")

    def close(self):
        if self.ptr:
            self.L.tts_gguf_writer_free(self.ptr)
            self.ptr = None


def quantize_params(quantize_type=Q4_K, **kw):
    p = QuantizeParams()
    p.quantize_type = quantize_type
    for k, v in kw.items():
        setattr(p, k, int(v))
    return p


def gguf_tensor_rule(arch, name, params=None):
    """1 = quantize, 2 = convert to F16, 0 = copy (quantize_impl.cpp's is_quantizable / F16 rules)."""
    p = params or quantize_params()
    return lib().tts_gguf_tensor_rule(arch.encode() if arch else None, name.encode(), ctypes.byref(p))


def quantize_gguf(src, dst, params=None, backend=None, rows_fn=None):
    """examples/quantize's quantize_gguf.  The rows are quantized by the device (backend: HipBackend) or by
    rows_fn(type, x[rows][K] float32) -> bytes (tests: the CPU oracle)."""
    import numpy as np
    L = lib()
    p = params or quantize_params()
    if backend is not None:
        st = L.tts_hip_gguf_quantize(backend.ptr, str(src).encode(), str(dst).encode(), ctypes.byref(p))
    else:
        def cb(_ctx, ttype, x, dst_p, rows, K):
            try:
                xa = np.ctypeslib.as_array(ctypes.cast(x, ctypes.POINTER(ctypes.c_float)), shape=(rows, K))
                q = np.ascontiguousarray(rows_fn(ttype, xa.copy()), dtype=np.uint8)
                ctypes.memmove(dst_p, q.ctypes.data, q.nbytes)
                return 0
            except Exception:  # noqa: BLE001 -- reported as a failed conversion
                import traceback
                traceback.print_exc()
                return -1
        fn = QUANTIZE_ROWS_FN(cb)
        st = L.tts_gguf_quantize(str(src).encode(), str(dst).encode(), ctypes.byref(p), ctypes.cast(fn, ctypes.c_void_p), None)
    if st != 0:
        raise RuntimeError(f"quantize_gguf failed {st}")


def parler_config_from_gguf(g, **kw):
    cfg = parler_config(**kw)
    if lib().tts_parler_config_from_gguf(g.ptr, ctypes.byref(cfg)) != 0:
        raise RuntimeError("not a usable parler-tts GGUF file")
    for k, v in kw.items():  # caller overrides (batch, max_ctx, arena) win
        setattr(cfg, k, v)
    return cfg


def dac_config_from_gguf(g, **kw):
    cfg = dac_config(**kw)
    if lib().tts_dac_config_from_gguf(g.ptr, ctypes.byref(cfg)) != 0:
        raise RuntimeError("no usable DAC decoder in the GGUF file")
    return cfg


def write_parler_synthetic_gguf(path, cfg, dac_cfg=None):
    """The runner's synthetic weights for cfg (and a DAC decoder) as a GGUF file with the reference's names."""
    st = lib().tts_parler_write_synthetic_gguf(ctypes.byref(cfg), ctypes.byref(dac_cfg) if dac_cfg is not None else None,
                                               str(path).encode())
    if st != 0:
        raise RuntimeError(f"writing {path} failed {st}")
