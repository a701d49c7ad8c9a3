"""GGUF files on the host (no device): the reader / writer against an independent pure-Python parser of
the GGUF v3 layout, malformed files, the quantize tool's per-architecture rules
(examples/quantize/quantize_impl.cpp:14-80) and its output bytes (CPU oracle quantizer as the row
callback), and the loader path (runner_from_file -> assign_weight, src/models/loaders.cpp:34-95):
a Parler / DAC runner built from a file decodes exactly like the runner holding the same weights."""
import struct

import numpy as np
import pytest

import py_oracle
import ttship

TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=512, output_vocab=1088, max_ctx=64,
            prompt_vocab=512, max_positions=96, n_encode=3)
DAC_TINY = dict(latent_dim=64, decoder_dim=64, rates=[2, 2, 2, 2], n_layers=4, max_frames=16)


def parse_gguf(path):
    """Independent reader of the on-disk layout: header, KV pairs, tensor infos, aligned data."""
    b = open(path, "rb").read()
    pos = 0

    def take(fmt):
        nonlocal pos
        v = struct.unpack_from("<" + fmt, b, pos)
        pos += struct.calcsize("<" + fmt)
        return v[0] if len(v) == 1 else v

    def string():
        nonlocal pos
        n = take("Q")
        s = b[pos:pos + n].decode()
        pos += n
        return s

    scal = {0: "B", 1: "b", 2: "H", 3: "h", 4: "I", 5: "i", 6: "f", 7: "?", 10: "Q", 11: "q", 12: "d"}

    def value(t):
        if t == 8:
            return string()
        if t == 9:
            at, n = take("I"), take("Q")
            return [value(at) for _ in range(n)]
        return take(scal[t])

    assert b[:4] == b"GGUF"
    pos = 4
    version, n_t, n_kv = take("I"), take("Q"), take("Q")
    kv = {}
    for _ in range(n_kv):
        k = string()
        kv[k] = value(take("I"))
    infos = []
    for _ in range(n_t):
        name = string()
        nd = take("I")
        ne = [take("q") for _ in range(nd)]
        infos.append((name, ne, take("I"), take("Q")))
    align = kv.get("general.alignment", 32)
    data0 = (pos + align - 1) // align * align
    return version, kv, infos, data0, b


def test_writer_reader_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    w = ttship.GgufWriter()
    w.set("general.architecture", "parler-tts")
    w.set("general.alignment", 64)
    w.set("a.u32", 7)
    w.set("a.i32", -5, "i32")
    w.set("a.u64", 1 << 40, "u64")
    w.set("a.f32", 0.25)
    w.set("a.bool", True)
    w.set("a.arr_i32", [1, -2, 3], ("arr", "i32"))
    w.set("a.arr_f32", [0.5, 1.5], ("arr", "f32"))
    w.set("a.arr_str", ["x", "yz", ""], ("arr", "str"))
    w.set("a.u32", 9)  # replaces, keeps the first position
    f32 = rng.standard_normal((3, 64)).astype(np.float32)
    f16 = rng.standard_normal(40).astype(np.float16)
    q4k = rng.integers(0, 256, size=2 * 2 * 144, dtype=np.uint8)
    i32 = np.arange(5, dtype=np.int32)
    w.add_tensor("t.f32", ttship.F32, (64, 3), f32)
    w.add_tensor("t.f16", ttship.F16, (40,), f16)
    w.add_tensor("t.q4k", ttship.Q4_K, (512, 2), q4k)
    w.add_tensor("t.i32", ttship.I32, (5,), i32)
    with pytest.raises(ValueError):
        w.add_tensor("t.bad", ttship.Q4_K, (100, 1), np.zeros(144, np.uint8))  # ragged blocks
    with pytest.raises(ValueError):
        w.add_tensor("t.f32", ttship.F32, (1,), np.zeros(1, np.float32))      # duplicate name
    path = tmp_path / "rt.gguf"
    w.write(path)
    w.close()

    version, kv, infos, data0, raw = parse_gguf(path)
    assert version == 3 and data0 % 64 == 0
    assert list(kv)[:3] == ["general.architecture", "general.alignment", "a.u32"] and kv["a.u32"] == 9
    assert kv["a.arr_str"] == ["x", "yz", ""] and kv["a.arr_i32"] == [1, -2, 3]
    want = {"t.f32": f32.tobytes(), "t.f16": f16.tobytes(), "t.q4k": q4k.tobytes(), "t.i32": i32.tobytes()}
    for name, ne, ty, off in infos:
        assert off % 64 == 0
        assert raw[data0 + off: data0 + off + len(want[name])] == want[name]

    with ttship.Gguf(path) as g:
        assert g.version == 3 and g.alignment == 64 and g.data_offset == data0
        assert g.get("a.u32") == 9 and g.get("a.i32") == -5 and g.get("a.u64") == 1 << 40
        assert g.get("a.f32") == 0.25 and g.get("a.bool") is True and g.get("missing", 3) == 3
        assert list(g.get("a.arr_i32")) == [1, -2, 3] and list(g.get("a.arr_f32")) == [0.5, 1.5]
        assert g.get("a.arr_str") == ["x", "yz", ""]
        ts = {t[0]: t for t in g.tensors()}
        assert ts["t.q4k"][1:3] == (ttship.Q4_K, (512, 2)) and ts["t.q4k"][4] == 2 * 2 * 144
        for name, data in want.items():
            assert g.tensor_bytes(name).tobytes() == data


def test_malformed_files_are_rejected(tmp_path):
    w = ttship.GgufWriter()
    w.set("k", 1)
    w.add_tensor("t", ttship.F32, (256,), np.ones(256, np.float32))
    good = tmp_path / "good.gguf"
    w.write(good)
    w.close()
    raw = good.read_bytes()
    cases = {"magic": b"GGUX" + raw[4:], "version": raw[:4] + struct.pack("<I", 9) + raw[8:],
             "truncated_kv": raw[:30], "truncated_data": raw[:-8], "empty": b""}
    # tensor info of "t": name (u64 length + bytes), n_dims u32, ne[0] i64, type u32, offset u64
    ti = raw.index(struct.pack("<Q", 1) + b"t") + 9
    ne_at, off_at = ti + 4, ti + 4 + 8 + 4

    def patch(at, fmt, v):
        return raw[:at] + struct.pack(fmt, v) + raw[at + struct.calcsize(fmt):]
    # an aligned offset near 2^64: data_offset + offset + size wraps past the mapping check
    cases["huge_offset"] = patch(off_at, "<Q", (1 << 64) - 32)
    cases["offset_past_end"] = patch(off_at, "<Q", 1 << 20)
    # 2^62 F32 elements: the byte size overflows 64 bits
    cases["huge_ne"] = patch(ne_at, "<q", 1 << 62)
    cases["huge_ne_2"] = patch(ne_at, "<q", (1 << 63) - 1)
    for name, data in cases.items():
        p = tmp_path / f"{name}.gguf"
        p.write_bytes(data)
        with pytest.raises(RuntimeError):
            ttship.Gguf(p)
    with pytest.raises(RuntimeError):
        ttship.Gguf(tmp_path / "absent.gguf")
    ttship.Gguf(good).close()


def test_quantize_rules():
    r = ttship.gguf_tensor_rule
    # parler_is_quanitizable (:51-67)
    assert r("parler-tts", "decoder.layers.3.fc1.weight") == 1
    assert r("parler-tts", "decoder.embed_tokens.0.weight") == 1
    for name in ("decoder.layer_norm.weight", "decoder.layers.0.self_attn_layer_norm.bias", "decoder.text_encoding",
                 "decoder.positional_embed", "decoder.lm_heads.0.weight.head", "decoder.embed_prompts",
                 "decoder.layers.1.encoder_attn.k_proj.weight", "decoder.layers.1.encoder_attn.v_proj.weight",
                 "audio_encoder.initial.weight"):
        assert r("parler-tts", name) == 0, name
    full = ttship.quantize_params(quantize_output_heads=1, quantize_text_embeddings=1, quantize_cross_attn_kv=1)
    assert r("parler-tts", "decoder.lm_heads.0.weight.head", full) == 1
    assert r("parler-tts", "decoder.embed_prompts", full) == 1
    assert r("parler-tts", "decoder.layers.1.encoder_attn.k_proj.weight", full) == 1
    dac16 = ttship.quantize_params(convert_dac_to_f16=1)
    assert r("parler-tts", "audio_encoder.initial.weight", dac16) == 2
    assert r("parler-tts", "audio_encoder.final.alpha", dac16) == 0
    # dia_is_quantizable (:42-49)
    assert r("dia", "dia.decoder.layers.0.self_attn.q_proj") == 1
    assert r("dia", "dia.decoder.heads.0") == 0 and r("dia", "dia.encoder.norm") == 0
    assert r("dia", "dia.decoder.heads.0", full) == 1
    # kokoro_is_quantizable (:14-40)
    assert r("kokoro", "kokoro.albert.layers.0.attn.q") == 1
    assert r("kokoro", "kokoro.text_encoder.lstm.weight") == 1
    assert r("kokoro", "kokoro.duration_predictor.duration_proj.weight") == 1
    assert r("kokoro", "kokoro.duration_predictor.layers.0.weight") == 1
    assert r("kokoro", "kokoro.duration_predictor.f0_blocks.0.weight") == 0
    assert r("kokoro", "kokoro.albert.layers.0.bias") == 0 and r("kokoro", "kokoro.albert.norm") == 0
    assert r("kokoro", "kokoro.decoder.generator.conv.weight", ttship.quantize_params(convert_non_quantizable_to_f16=1)) == 2
    assert r("kokoro", "kokoro.voice_tensors.af", ttship.quantize_params(convert_non_quantizable_to_f16=1)) == 0
    # orpheus (aborts in the reference): every matrix but the norms
    assert r("orpheus", "orpheus.layers.0.mlp.down_proj.weight") == 1 and r("orpheus", "orpheus.layers.0.input_norm.weight") == 0
    assert r("unknown-arch", "x") == -1


def _oracle_rows(ttype, x):
    if ttype in (ttship.Q4_K, ttship.Q8_0):
        return py_oracle.quantize(ttype, x)
    raise AssertionError(f"unexpected row type {ttype}")


@pytest.fixture(scope="module")
def parler_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("gguf")
    cfg32 = ttship.parler_config(weight_type=ttship.F32, head_type=ttship.F32, **TINY)
    src = d / "parler-f32.gguf"
    ttship.write_parler_synthetic_gguf(src, cfg32, ttship.dac_config(**DAC_TINY))
    q4 = d / "parler-q4_k.gguf"
    ttship.quantize_gguf(src, q4, ttship.quantize_params(ttship.Q4_K), rows_fn=_oracle_rows)
    return cfg32, src, q4


def test_quantize_tool_output(parler_files):
    _, src, q4 = parler_files
    with ttship.Gguf(src) as a, ttship.Gguf(q4) as b:
        assert b.get("general.quantization_type") == ttship.Q4_K and b.get("general.quantization_version") == 2
        for k in a.keys():  # gguf_set_kv: every key copied
            assert b.get(k) == a.get(k), k
        ta, tb = a.tensors(), b.tensors()
        assert [t[0] for t in ta] == [t[0] for t in tb]  # file order kept
        n_q = 0
        for (name, ty, ne, _, _), (_, ty2, ne2, _, _) in zip(ta, tb):
            assert ty == ttship.F32 and ne == ne2
            if ttship.gguf_tensor_rule("parler-tts", name) == 1:
                n_q += 1
                assert ty2 == ttship.Q4_K, name
                x = a.tensor_bytes(name).view(np.float32).reshape(-1, ne[0])
                assert np.array_equal(b.tensor_bytes(name), py_oracle.quantize(ttship.Q4_K, x)), name
            else:
                assert ty2 == ttship.F32 and np.array_equal(b.tensor_bytes(name), a.tensor_bytes(name)), name
        assert n_q == 9 + 8 * TINY["n_layers"]  # embeddings; q, k, v, o, cross-q, cross-o, fc1, fc2 per layer


def test_quantize_tool_f16_conversion(tmp_path):
    x = np.array([0.0, -0.0, 1.0, 65504.0, 65520.0, 1e-8, 6.0e-8, 2.98e-8, -3.1e-5, np.inf, -np.inf, 1 / 3, 2049.0, 2051.0],
                 dtype=np.float32)
    x = np.concatenate([x, np.random.default_rng(2).standard_normal(242).astype(np.float32) * 1e3])
    w = ttship.GgufWriter()
    w.set("general.architecture", "kokoro")
    w.add_tensor("kokoro.decoder.generator.conv.weight", ttship.F32, (256,), x)
    w.add_tensor("kokoro.albert.norm", ttship.F32, (256,), x)
    src, dst = tmp_path / "k.gguf", tmp_path / "k16.gguf"
    w.write(src)
    w.close()
    ttship.quantize_gguf(src, dst, ttship.quantize_params(ttship.Q8_0, convert_non_quantizable_to_f16=1), rows_fn=_oracle_rows)
    with ttship.Gguf(dst) as g:
        assert g.tensor_type("kokoro.decoder.generator.conv.weight") == ttship.F16
        assert g.tensor_type("kokoro.albert.norm") == ttship.F32
        got = g.tensor_bytes("kokoro.decoder.generator.conv.weight").view(np.uint16)
    with np.errstate(over="ignore"):  # 65520 rounds to inf, as it should
        want = x.astype(np.float16).view(np.uint16)
    assert np.array_equal(got, want)  # round to nearest even


def test_quantize_tool_rejects_non_f32(tmp_path):
    w = ttship.GgufWriter()
    w.add_tensor("decoder.layers.0.fc1.weight", ttship.F16, (256, 2), np.zeros(512, np.float16))
    src = tmp_path / "p16.gguf"
    w.write(src)
    w.close()
    with pytest.raises(RuntimeError):
        ttship.quantize_gguf(src, tmp_path / "out.gguf", rows_fn=_oracle_rows)


def test_parler_config_from_gguf(parler_files):
    cfg32, src, q4 = parler_files
    with ttship.Gguf(q4) as g:
        c = ttship.parler_config_from_gguf(g, batch=2)
    for k in ("n_layers", "hidden_size", "n_attn_heads", "ffn_size", "output_vocab", "prompt_vocab", "max_positions",
              "n_encode", "n_output_heads", "eos_token", "bos_token", "audio_vocab"):
        assert getattr(c, k) == getattr(cfg32, k), k
    assert c.weight_type == ttship.Q4_K and c.head_type == ttship.F32 and c.batch == 2


def _decode_logits(runner, batch, steps=3):
    prompt = (np.arange(5 * batch, dtype=np.int32).reshape(batch, 5) * 37) % TINY["prompt_vocab"]
    runner.prefill(prompt)
    out = []
    for s in range(steps):
        out.append(runner.decode(np.full((batch, 9), 11 + s, dtype=np.int32)))
    return np.stack(out)


def test_parler_from_gguf_equals_synthetic_runner(parler_files):
    """F32 file -> runner: every tensor lands where the synthetic runner puts the same values."""
    cfg32, src, _ = parler_files
    it = py_oracle.iface(4)
    ref = ttship.Parler(it, cfg32)
    with ttship.Gguf(src) as g:
        run = ttship.Parler(it, ttship.parler_config_from_gguf(g, max_ctx=TINY["max_ctx"]), gguf=g)
    try:
        assert run.weight_bytes() == ref.weight_bytes()
        assert np.array_equal(_decode_logits(run, 1), _decode_logits(ref, 1))
    finally:
        run.close()
        ref.close()


def test_parler_from_quantized_gguf_decodes(parler_files):
    _, _, q4 = parler_files
    with ttship.Gguf(q4) as g:
        cfg = ttship.parler_config_from_gguf(g, max_ctx=TINY["max_ctx"], batch=2)
        r = ttship.Parler(py_oracle.iface(4), cfg, gguf=g)
    try:  # the mapping may close: the runner holds its own copy of the weights
        a = _decode_logits(r, 2)
        assert np.all(np.isfinite(a)) and a.std() > 0
        st = r.plan_stats()
        assert st["gemv"] >= 6 * TINY["n_layers"], st  # Q4_K matrices from the file reach the fused GEMV items
    finally:
        r.close()


def test_parler_from_gguf_missing_tensor(tmp_path, parler_files):
    _, src, _ = parler_files
    with ttship.Gguf(src) as g:
        w = ttship.GgufWriter()
        w.copy_kv(g)
        for name, ty, ne, _, _ in g.tensors():
            if name != "decoder.layers.1.fc2.weight":
                w.add_tensor(name, ty, ne, g.tensor_bytes(name))
        p = tmp_path / "missing.gguf"
        w.write(p)
        w.close()
        cfg = ttship.parler_config_from_gguf(g, max_ctx=TINY["max_ctx"])
    with ttship.Gguf(p) as g2:
        with pytest.raises(RuntimeError):
            ttship.Parler(py_oracle.iface(2), cfg, gguf=g2)


def test_dac_from_gguf_equals_synthetic(parler_files):
    _, src, q4 = parler_files
    codes = np.random.default_rng(5).integers(0, 1024, size=(4, 9))
    ref = ttship.Dac(py_oracle.iface(4), ttship.dac_config(**DAC_TINY))
    with ttship.Gguf(q4) as g:  # the DAC tensors pass through the quantize tool unchanged
        cfg = ttship.dac_config_from_gguf(g, max_frames=DAC_TINY["max_frames"])
        assert list(cfg.rates[:cfg.n_layers]) == DAC_TINY["rates"] and cfg.latent_dim == 64 and cfg.decoder_dim == 64
        d = ttship.Dac(py_oracle.iface(4), cfg, gguf=g)
    try:
        assert np.array_equal(d.decode(codes), ref.decode(codes))
    finally:
        d.close()
        ref.close()
