"""DAC decoder graph pinned to an independent implementation: transformers' DacModel.

TTS.cpp decodes Parler's codec tokens with DAC-44k: dac_runner::build_dac_graph
(/root/reference/src/decoder/dac_model.cpp:139-170) over the shared codec layers of
general_neural_audio_codec.cpp:133-172 (quantizer out-projections, the initial conv, per layer snake +
conv_transpose_1d + three dilated residual units, final snake + conv + tanh), with the weights
dac_gguf_encoder.py writes (weight norm folded, /root/reference/py-gguf/tts_encoders/dac_gguf_encoder.py:43-97).
Here transformers' DacModel (quantizer.from_codes + decoder) runs the runner's own F32 weights (tiny
widths, two upsampling layers) under the one precision rule TTS.cpp's graph adds: ggml_conv_1d builds
its im2col in F16, so every conv_1d multiplies f16-rounded inputs by f16-rounded kernels (mul_mat's
vec_dot_type), accumulating wider (f64 here, as the oracle); conv_transpose_1d (the fork's op) stays F32
(an f64 sum rounded once, as the oracle restates it).  Snake's 1e-9 in transformers is kept (TTS.cpp's
snake_1d has none; alpha ~ 1 makes it invisible).

Tolerance: the f16 rounding of every conv input makes the decoder sensitive to the last bit of a sum --
one f16 flip near the input spreads through the upsampling layers (the CPU backend's scalar and
SIMD builds differ by 1.5e-3 on DAC-44k for this reason).  A graph mistake moves PCM by O(0.1-1); the two
implementations here agree to <= 5e-4 with a median below 1e-4 (measured 2e-5 / 1e-6 at 6 frames,
3e-4 / 4e-5 at 17 frames, where an early flip spreads)."""
import numpy as np
import pytest

import py_oracle
import ttship

torch = pytest.importorskip("torch")
pytest.importorskip("transformers")

RATES = [4, 2]


def dac_from_runner(w, cfg):
    from transformers import DacConfig, DacModel
    # transformers derives the latent width (encoder_hidden_size * 2 ** len(ratios)) and the decoder's
    # upsampling ratios (the reversed downsampling ratios) from the encoder side
    dc = DacConfig(encoder_hidden_size=cfg.latent_dim // 2 ** len(RATES), downsampling_ratios=RATES[::-1],
                   decoder_hidden_size=cfg.decoder_dim, n_codebooks=cfg.n_codebooks, codebook_size=cfg.codebook_size,
                   codebook_dim=cfg.codebook_dim)
    m = DacModel(dc).eval()
    assert m.config.hidden_size == cfg.latent_dim and list(m.config.upsampling_ratios) == RATES
    f16 = lambda a: a.astype(np.float16).astype(np.float32)  # noqa: E731  conv_1d kernels through the F16 im2col product
    sd = {}
    for i in range(cfg.n_codebooks):
        sd[f"quantizer.quantizers.{i}.codebook.weight"] = w[f"quantizers.{i}.codebook.weight"]
        sd[f"quantizer.quantizers.{i}.out_proj.weight"] = f16(w[f"quantizers.{i}.out_proj.weight"])
        sd[f"quantizer.quantizers.{i}.out_proj.bias"] = w[f"quantizers.{i}.out_proj.bias"].reshape(-1)
    sd["decoder.conv1.weight"] = f16(w["initial.weight"])
    sd["decoder.conv1.bias"] = w["initial.bias"].reshape(-1)
    for l in range(cfg.n_layers):
        pre, hp = f"decoder_block.{l + 1}", f"decoder.block.{l}"
        sd[f"{hp}.snake1.alpha"] = w[f"{pre}.final.alpha"].reshape(1, -1, 1)
        sd[f"{hp}.conv_t1.weight"] = w[f"{pre}.final.weight"]
        sd[f"{hp}.conv_t1.bias"] = w[f"{pre}.final.bias"].reshape(-1)
        for r in range(3):
            rp, hr = f"{pre}.residual_unit.{r}", f"{hp}.res_unit{r + 1}"
            sd[f"{hr}.snake1.alpha"] = w[f"{rp}.res.initial.alpha"].reshape(1, -1, 1)
            sd[f"{hr}.conv1.weight"] = f16(w[f"{rp}.res.initial.weight"])
            sd[f"{hr}.conv1.bias"] = w[f"{rp}.res.initial.bias"].reshape(-1)
            sd[f"{hr}.snake2.alpha"] = w[f"{rp}.res.final.alpha"].reshape(1, -1, 1)
            sd[f"{hr}.conv2.weight"] = f16(w[f"{rp}.res.final.weight"])
            sd[f"{hr}.conv2.bias"] = w[f"{rp}.res.final.bias"].reshape(-1)
    sd["decoder.snake1.alpha"] = w["final.alpha"].reshape(1, -1, 1)
    sd["decoder.conv2.weight"] = f16(w["final.weight"].reshape(1, -1, 7))
    sd["decoder.conv2.bias"] = w["final.bias"].reshape(-1)
    t = {k: torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)) for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(t, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith("encoder.") or ".in_proj." in k for k in missing), missing
    # conv_1d inputs rounded to f16 (ggml_conv_1d's F16 im2col); products accumulated in f64 as ggml's f16 dot
    # does; conv_transpose_1d in f32 with one rounding of an f64 sum (the oracle's restatement of the fork op)
    for mod in list(m.decoder.modules()) + [q.out_proj for q in m.quantizer.quantizers]:
        if isinstance(mod, torch.nn.Conv1d):
            mod.register_forward_pre_hook(lambda _m, args: (args[0].to(torch.float16).to(torch.float64),))
        if isinstance(mod, (torch.nn.Conv1d, torch.nn.ConvTranspose1d)):
            if isinstance(mod, torch.nn.ConvTranspose1d):
                mod.register_forward_pre_hook(lambda _m, args: (args[0].to(torch.float64),))
            mod.register_forward_hook(lambda _m, _a, out: out.to(torch.float32))
            mod.double()
    return m


@pytest.mark.parametrize("T", [6, 17])
def test_dac_graph_matches_transformers_dac(T):
    cfg = ttship.dac_config(n_codebooks=3, codebook_size=64, codebook_dim=8, latent_dim=64, decoder_dim=64, n_layers=len(RATES),
                            rates=RATES + [1] * (8 - len(RATES)), max_frames=32)
    d = ttship.Dac(py_oracle.iface(4), cfg)
    try:
        w = d.weights()
        codes = np.random.default_rng(T).integers(0, cfg.codebook_size, (T, cfg.n_codebooks)).astype(np.int32)
        got = d.decode(codes)
    finally:
        d.close()
    m = dac_from_runner(w, cfg)
    with torch.no_grad():
        z = m.quantizer.from_codes(torch.from_numpy(codes.T.astype(np.int64))[None])[0]
        ref = m.decoder(z)[0, 0].numpy()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    e = np.abs(got - ref)
    assert e.max() <= 5e-4 and np.median(e) <= 1e-4, (float(e.max()), float(np.median(e)))
