"""The ggml backend adapter (src/ggml_backend/ggml-tts-hip.cpp) executed end to end.

tests/ggml_stub/adapter_harness.cpp is a tts_backend_iface whose every call goes through the
adapter's ggml vtables, the way TTS.cpp reaches a backend: registry -> device -> init_backend /
buffer type (src/tts_model.cpp:25-67,134-164), whole-tensor set_tensor of the weights
(tts_model.cpp:157-164; Q4_K routed to the backend's layouts with no buffer usage set), set_tensor
of the inputs, graph_compute of ggml_tensor nodes whose ops / unary ops are matched by upstream name,
get_tensor_async read at once with no synchronize (parler/model.cpp:680-683), the host sampler.
The same runners then run on the adapter and on the direct C-ABI; outputs must be bit-identical.
The ggml side is a runtime stand-in (tests/ggml_stub/ggml_runtime.cpp: names, ggml_nbytes, buffer
structs), since the fork the adapter is built against in production is absent here."""
import ctypes
import os
import pathlib

import numpy as np
import pytest

import py_oracle
import ttship

ROOT = pathlib.Path(__file__).resolve().parents[1]
HARNESS = ROOT / "tests" / "ggml_stub" / "_build" / "libtts_ggml_harness.so"


class AdapterBackend:
    """tts_backend_iface over the ggml adapter's vtables (test harness)."""

    def __init__(self, device=0, check_support=True):
        ttship.lib()  # the harness links the same libtts_hip.so
        if not HARNESS.exists():
            raise RuntimeError(f"{HARNESS} missing: run `make adapter-harness`")
        L = ctypes.CDLL(str(HARNESS))
        vp = ctypes.c_void_p
        L.tts_ggml_harness_create.restype = vp
        L.tts_ggml_harness_create.argtypes = [ctypes.c_int, ctypes.c_int]
        L.tts_ggml_harness_free.argtypes = [vp]
        L.tts_ggml_harness_iface.argtypes = [vp, ctypes.POINTER(ttship.BackendIface)]
        L.tts_ggml_harness_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
        L.tts_ggml_harness_last_refused.restype = ctypes.c_char_p
        L.tts_ggml_harness_last_refused.argtypes = [vp]
        L.tts_ggml_harness_device_name.restype = ctypes.c_char_p
        L.tts_ggml_harness_device_name.argtypes = [vp]
        L.tts_ggml_harness_hostleaf_supported.argtypes = [vp]
        self.L = L
        self.ptr = L.tts_ggml_harness_create(device, 1 if check_support else 0)
        if not self.ptr:
            raise RuntimeError("adapter harness: no TTS-HIP device through ggml_backend_tts_hip_reg")

    def iface(self):
        it = ttship.BackendIface()
        self.L.tts_ggml_harness_iface(self.ptr, ctypes.byref(it))
        return it

    def stats(self):
        a = (ctypes.c_int64 * 8)()
        self.L.tts_ggml_harness_stats(self.ptr, a, 8)
        keys = ["graph_computes", "nodes", "refused", "weight_sets", "buffers", "input_sets", "reads", "compute_failures"]
        return dict(zip(keys, list(a)))

    def last_refused(self):
        return self.L.tts_ggml_harness_last_refused(self.ptr).decode()

    def close(self):
        if self.ptr:
            self.L.tts_ggml_harness_free(self.ptr)
            self.ptr = None


@pytest.fixture
def adapter():
    a = AdapterBackend(0)
    yield a
    a.close()


TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=128, prompt_vocab=512,
            max_positions=160)


def _check_stats(a, n_weights_min):
    s = a.stats()
    assert s["compute_failures"] == 0, s
    assert s["refused"] == 0, (s, a.last_refused())
    assert s["graph_computes"] > 0 and s["weight_sets"] >= n_weights_min and s["buffers"] >= 2, s
    return s


@pytest.mark.gpu
def test_registry_device_and_host_leaf(adapter):
    """The registry exposes the device; supports_op refuses a DIV whose divisor is a buffer-less host
    leaf (util.cpp:86-94's reciprocal() static) and accepts the same DIV with a device leaf."""
    assert adapter.L.tts_ggml_harness_device_name(adapter.ptr).decode().startswith("TTS-HIP")
    assert adapter.L.tts_ggml_harness_hostleaf_supported(adapter.ptr) == 0b10


@pytest.mark.gpu
def test_parler_mini_b1_through_adapter_is_bit_identical(hip, adapter):
    """Parler-mini Q4_K at batch 1 (the reference's node order, TTS.cpp's one-prompt runner): the
    runner on the adapter (host sampling, logits read back every step as TTS.cpp does) vs the same
    runner on the direct C-ABI: tokens and logits bit-identical, every node accepted by supports_op."""
    cfg = dict(batch=1)
    d = ttship.Parler(hip.iface(), ttship.parler_config(**cfg))
    g = ttship.Parler(adapter.iface(), ttship.parler_config(**cfg))
    try:
        prompt = np.array([[11, 29, 400, 7, 1, 3000, 16, 9]], dtype=np.int32)
        d.prefill(prompt)
        g.prefill(prompt)
        d.set_device_sampling(False)
        td, tg = d.generate(6), g.generate(6)
        assert np.array_equal(td, tg), f"token mismatch\n{td}\n{tg}"
        toks = np.full((1, 9), 5, dtype=np.int32)
        ld, lg = d.decode(toks), g.decode(toks)
        assert np.array_equal(ld, lg), float(np.max(np.abs(ld - lg)))
        s = _check_stats(adapter, 24 * 8)
        print("adapter stats", s)
    finally:
        d.close()
        g.close()


@pytest.mark.gpu
def test_parler_tiny_through_adapter_matches_oracle(adapter):
    """The adapter path against the CPU oracle (greedy tokens bit-exact, logits 1e-4)."""
    g = ttship.Parler(adapter.iface(), ttship.parler_config(batch=2, **TINY))
    c = ttship.Parler(py_oracle.iface(8), ttship.parler_config(batch=2, **TINY))
    try:
        prompt = (np.arange(14, dtype=np.int32).reshape(2, 7) * 37) % 512
        g.prefill(prompt)
        c.prefill(prompt)
        tg, tc = g.generate(10), c.generate(10)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
        toks = np.full((2, 9), 5, dtype=np.int32)
        lg, lc = g.decode(toks), c.decode(toks)
        assert np.abs(lg - lc).max() <= 1e-4 * np.abs(lc).max() + 1e-4
        _check_stats(adapter, 2 * 8)
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
def test_weight_set_failure_falls_back_to_native_bytes(hip):
    """When the backend cannot write a weight's layout (fault injected into tts_hip_weight_set), the
    adapter's set_tensor stores ggml's native Q4_K bytes with no layout flags and the graphs still
    compute the same tokens (the weight was left uninitialised before)."""
    ttship.lib().tts_hip_test_hook(1, 1)  # TTS_HIP_HOOK_FAULT_WEIGHT_SET
    a = AdapterBackend(0)
    try:
        g = ttship.Parler(a.iface(), ttship.parler_config(batch=1, **TINY))
    finally:
        ttship.lib().tts_hip_test_hook(1, 0)
    d = ttship.Parler(hip.iface(), ttship.parler_config(batch=1, **TINY))
    try:
        prompt = (np.arange(7, dtype=np.int32).reshape(1, 7) * 53) % 512
        g.prefill(prompt)
        d.prefill(prompt)
        d.set_device_sampling(False)
        assert np.array_equal(g.generate(8), d.generate(8))
    finally:
        g.close()
        d.close()
        a.close()


DIA_TINY = dict(n_encoder_layers=1, n_decoder_layers=2, encoder_hidden_size=64, decoder_hidden_size=128, encoder_attn_heads=4,
                decoder_attn_heads=4, decoder_query_heads=2, head_size=32, encoder_ffn_size=128, decoder_ffn_size=256,
                max_generation_size=64, max_encoder_context_length=32)


@pytest.mark.gpu
def test_dia_cfg_scale_custom_map_through_adapter(hip, adapter):
    """Dia's CFG heads carry cfg_scale as ggml_map_custom2 (util.cpp:175-200): the adapter recognises
    the registered callback and runs the device restatement; logits bit-identical to the direct path."""
    d = ttship.Dia(hip.iface(), ttship.dia_config(**DIA_TINY))
    g = ttship.Dia(adapter.iface(), ttship.dia_config(**DIA_TINY))
    try:
        text = np.frombuffer(b"\x01 The birch canoe slid on the smooth planks.", dtype=np.uint8).astype(np.int32)[:32]
        audio = np.full(9, 1026, dtype=np.int32)
        for s in range(4):
            ld = d.prefill(text, audio) if s == 0 else d.decode(audio)
            lg = g.prefill(text, audio) if s == 0 else g.decode(audio)
            assert np.array_equal(ld, lg), (s, float(np.max(np.abs(ld - lg))))
            audio = ld.argmax(axis=1).astype(np.int32)
        _check_stats(adapter, 8)
    finally:
        d.close()
        g.close()


@pytest.mark.gpu
def test_dac_through_adapter(hip, adapter):
    """The DAC-44k codec graph (conv_1d / conv_transpose_1d / snake with the reciprocal leaf in a
    buffer) on the adapter: PCM bit-identical to the direct path."""
    dcfg = ttship.dac_config(max_frames=6)
    d = ttship.Dac(hip.iface(), dcfg)
    g = ttship.Dac(adapter.iface(), dcfg)
    try:
        codes = (np.arange(6 * dcfg.n_codebooks, dtype=np.int32).reshape(6, dcfg.n_codebooks) * 97) % dcfg.codebook_size
        pd, pg = d.decode(codes), g.decode(codes)
        assert pd.shape == pg.shape and np.array_equal(pd, pg)
        _check_stats(adapter, 8)
    finally:
        d.close()
        g.close()


@pytest.mark.gpu
def test_kokoro_uv_noise_custom_map_through_adapter(hip, adapter):
    """Kokoro's sine source carries uv_noise_compute as ggml_map_custom3 (util.cpp:140-170): tiny
    Kokoro end to end on the adapter, PCM bit-identical to the direct path at the same draws."""
    from test_kokoro_model_cpu import TINY as KTINY, tokens
    cfg = ttship.kokoro_config(**dict(KTINY))
    toks = tokens(7, 0)
    d = ttship.Kokoro(hip.iface(), cfg)
    g = ttship.Kokoro(adapter.iface(), cfg)
    try:
        hd, ld = d.durations(toks)
        hg, lg = g.durations(toks)
        assert np.array_equal(ld, lg) and np.array_equal(hd, hg)
        rand = np.random.default_rng(7).random((cfg.gen.harmonic_num + 1, 600 * int(ld.sum())), dtype=np.float32)
        assert np.array_equal(d.decode(toks, hd, ld, rand), g.decode(toks, hg, lg, rand))
        _check_stats(adapter, 8)
    finally:
        d.close()
        g.close()
