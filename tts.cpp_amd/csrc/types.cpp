// Type traits and op names (ggml_type_size / ggml_blck_size / ggml_row_size / ggml_op_name).
#include "common.h"

extern "C" {

size_t tts_type_size(int type) {
    switch (type) {
        case TTS_TYPE_F32: return 4;
        case TTS_TYPE_F16: return 2;
        case TTS_TYPE_Q4_K: return sizeof(tts::block_q4_K);
        case TTS_TYPE_Q8_0: return sizeof(tts::block_q8_0);
        case TTS_TYPE_Q8_K: return 292;
        case TTS_TYPE_I32: return 4;
        case TTS_TYPE_I16: return 2;
        case TTS_TYPE_I8: return 1;
        default: return 0;
    }
}

int64_t tts_blck_size(int type) {
    switch (type) {
        case TTS_TYPE_Q4_K:
        case TTS_TYPE_Q8_K: return tts::QK_K;
        case TTS_TYPE_Q8_0: return tts::QK8_0;
        default: return 1;
    }
}

size_t tts_row_size(int type, int64_t ne0) { return tts_type_size(type) * (size_t)(ne0 / tts_blck_size(type)); }

const char * tts_type_name(int type) {
    switch (type) {
        case TTS_TYPE_F32: return "f32";
        case TTS_TYPE_F16: return "f16";
        case TTS_TYPE_Q4_K: return "q4_K";
        case TTS_TYPE_Q8_0: return "q8_0";
        case TTS_TYPE_Q8_K: return "q8_K";
        case TTS_TYPE_I32: return "i32";
        case TTS_TYPE_I16: return "i16";
        case TTS_TYPE_I8: return "i8";
        default: return "?";
    }
}

const char * tts_op_name(int op) {
    static const char * names[TTS_OP_COUNT] = {
        "NONE", "DUP", "ADD", "SUB", "MUL", "DIV", "SQR", "SQRT", "SIN", "COS", "SUM_ROWS", "REPEAT",
        "CONCAT", "NORM", "RMS_NORM", "MUL_MAT", "SCALE", "CPY", "CONT", "RESHAPE", "VIEW", "PERMUTE",
        "TRANSPOSE", "GET_ROWS", "SOFT_MAX", "ROPE", "CLAMP", "CONV_TRANSPOSE_1D", "IM2COL", "UPSCALE",
        "PAD", "LEAKY_RELU", "UNARY", "CUMSUM", "MOD", "ROUND", "STFT", "ISTFT", "MAP_CUSTOM3", "MAP_CUSTOM2"};
    if (op < 0 || op >= TTS_OP_COUNT) return "?";
    return names[op];
}

}  // extern "C"
