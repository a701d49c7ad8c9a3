"""Dia graph pinned to an independent implementation: transformers' DiaForConditionalGeneration.

TTS.cpp's build_dia_graph (/root/reference/src/models/dia/model.cpp:376-420 encoder, :518-640 decoder,
:358-371 heads + cfg_scale) runs Dia-1.6B: a RMSNorm/SwiGLU encoder over byte tokens for a conditioned and
an unconditioned row, a GQA decoder over the sum of nine codebook embeddings with cross-attention into the
encoder, nine heads combined as cond + scale * (cond - uncond).  The oracle runs the runner's node list
(tts.cpp_amd/csrc/dia.cpp) on tiny F32 weights; transformers' Dia layers run the same weights over the
whole audio sequence at once (encoder layers, decoder layers, norms, multi-channel embedding and
logits_dense are transformers' modules; the weights are mapped as dia_gguf_encoder.py names them).

Three things TTS.cpp does that the transformers port does not, restated here so the comparison is of
the same model (each is what the runner must reproduce, so each is kept, not papered over):
  - the encoder mask is block-diagonal: prompt tokens attend prompt tokens and padding attends padding
    (dia_runner::set_inputs, model.cpp:726-736), where transformers masks padding keys for every query;
  - cross-attention is rotated: Q by the decoder position, K by the encoder position (model.cpp:489,606,
    as nari-labs' Dia does) -- transformers' DiaCrossAttention has no RoPE; here forward hooks on the
    cross q_proj / k_proj apply transformers' own rotate_half RoPE;
  - cross K is stored for the prompt positions only and the rest of the zero-initialised cache is read
    unmasked (build_dia_cross_kv_store, model.cpp:476-512; the cache is cleared at init, :318): the
    k_proj hook zeroes K past the prompt, and no cross mask is passed.
Logits of every step (after cfg_scale) must agree to 1e-4 of their scale, argmax exactly (measured 2e-6;
leaving out the cross-attention RoPE alone moves them by 2e-2)."""
import numpy as np
import pytest

import py_oracle
import ttship

torch = pytest.importorskip("torch")
pytest.importorskip("transformers")

TINY = dict(n_output_heads=3, n_encoder_layers=2, n_decoder_layers=2, encoder_hidden_size=64, decoder_hidden_size=128, encoder_attn_heads=4,
            decoder_attn_heads=4, decoder_query_heads=2, head_size=32, encoder_ffn_size=128, decoder_ffn_size=256, output_vocab_size=96,
            encoder_vocab_size=256, max_generation_size=32, max_encoder_context_length=24, weight_type=ttship.F32, head_type=ttship.F32)


def dia_from_runner(w, cfg):
    from transformers import DiaConfig, DiaForConditionalGeneration
    from transformers.models.dia.configuration_dia import DiaDecoderConfig, DiaEncoderConfig
    rope = {"rope_type": "default", "rope_theta": 10000.0}  # ggml_rope(..., mode 2): neox, base 10000
    H, hd = cfg.decoder_attn_heads, cfg.head_size
    enc = DiaEncoderConfig(max_position_embeddings=cfg.max_encoder_context_length, num_hidden_layers=cfg.n_encoder_layers,
                           hidden_size=cfg.encoder_hidden_size, num_attention_heads=cfg.encoder_attn_heads,
                           num_key_value_heads=cfg.encoder_attn_heads, head_dim=hd, intermediate_size=cfg.encoder_ffn_size, norm_eps=1e-5,
                           vocab_size=cfg.encoder_vocab_size, rope_parameters=dict(rope))
    dec = DiaDecoderConfig(max_position_embeddings=cfg.max_generation_size, num_hidden_layers=cfg.n_decoder_layers,
                           hidden_size=cfg.decoder_hidden_size, intermediate_size=cfg.decoder_ffn_size, num_attention_heads=H,
                           num_key_value_heads=H // cfg.decoder_query_heads, head_dim=hd, cross_num_attention_heads=H, cross_head_dim=hd,
                           cross_num_key_value_heads=H, cross_hidden_size=cfg.encoder_hidden_size, norm_eps=1e-5,
                           vocab_size=cfg.output_vocab_size, num_channels=cfg.n_output_heads, rope_parameters=dict(rope),
                           pad_token_id=None, eos_token_id=None, bos_token_id=None)
    dc = DiaConfig(encoder_config=enc, decoder_config=dec, delay_pattern=list(range(cfg.n_output_heads)))
    dc._attn_implementation = "eager"
    dc.encoder_config._attn_implementation = "eager"
    dc.decoder_config._attn_implementation = "eager"
    m = DiaForConditionalGeneration(dc).eval()
    sd = {"model.encoder.embedding.weight": w["encoder.embedding"], "model.encoder.norm.weight": w["encoder.norm"],
          "model.decoder.norm.weight": w["decoder.norm"]}
    for l in range(cfg.n_encoder_layers):
        src, dst = f"encoder.layers.{l}", f"model.encoder.layers.{l}"
        sd[f"{dst}.pre_sa_norm.weight"] = w[f"{src}.self_attn_norm"]
        sd[f"{dst}.post_sa_norm.weight"] = w[f"{src}.mlp_norm"]
        for p in "qkvo":
            sd[f"{dst}.self_attention.{p}_proj.weight"] = w[f"{src}.{p}"]
        sd[f"{dst}.mlp.gate_up_proj.weight"] = np.concatenate([w[f"{src}.gate"], w[f"{src}.up"]])  # chunk(2): gate first
        sd[f"{dst}.mlp.down_proj.weight"] = w[f"{src}.out"]
    for l in range(cfg.n_decoder_layers):
        src, dst = f"decoder.layers.{l}", f"model.decoder.layers.{l}"
        sd[f"{dst}.pre_sa_norm.weight"] = w[f"{src}.self_attn_norm"]
        sd[f"{dst}.pre_ca_norm.weight"] = w[f"{src}.cross_attn_norm"]
        sd[f"{dst}.pre_mlp_norm.weight"] = w[f"{src}.mlp_norm"]
        for p in "qkvo":
            sd[f"{dst}.self_attention.{p}_proj.weight"] = w[f"{src}.self_attn_{p}"]
            sd[f"{dst}.cross_attention.{p}_proj.weight"] = w[f"{src}.cross_attn_{p}"]
        sd[f"{dst}.mlp.gate_up_proj.weight"] = np.concatenate([w[f"{src}.gate"], w[f"{src}.up"]])
        sd[f"{dst}.mlp.down_proj.weight"] = w[f"{src}.out"]
    C = cfg.n_output_heads
    sd["model.decoder.embeddings.embed.weight"] = np.concatenate([w[f"decoder.embds.{i}"] for i in range(C)])
    sd["logits_dense.weight"] = np.concatenate([w[f"decoder.heads.{i}"] for i in range(C)])
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    return m


def rope_heads(x, cos, sin, hd):
    """transformers' rotate_half RoPE on a projection output [B, S, heads*hd] with cos/sin [1, S, hd]."""
    from transformers.models.dia.modeling_dia import rotate_half
    B, S, _ = x.shape
    h = x.view(B, S, -1, hd)
    c, s = cos[:, :, None, :], sin[:, :, None, :]
    return (h * c + rotate_half(h) * s).reshape(B, S, -1)


def run_transformers(m, cfg, text_rows, n_text, audio):
    """Logits [steps, heads, vocab] after cfg_scale of the audio sequence `audio` [steps, heads]."""
    T, hd = cfg.max_encoder_context_length, cfg.head_size
    enc_m, dec_m = m.model.encoder, m.model.decoder
    with torch.no_grad():
        ids = torch.from_numpy(text_rows.astype(np.int64))
        h = enc_m.embedding(ids)
        epos = torch.arange(T)[None]
        ecos, esin = enc_m.rotary_emb(h, position_ids=epos)
        real = torch.arange(T) < n_text
        same = real[:, None] == real[None, :]  # block-diagonal: prompt <-> prompt, padding <-> padding
        emask = torch.where(same, 0.0, float("-inf"))[None, None]
        for layer in enc_m.layers:
            h = layer(h, position_embeddings=(ecos, esin), attention_mask=emask)
        enc_out = enc_m.norm(h)

        S = len(audio)
        a = torch.from_numpy(np.asarray(audio, dtype=np.int64))[None].expand(2, S, -1)
        x = dec_m.embeddings(a)
        dcos, dsin = dec_m.rotary_emb(x, position_ids=torch.arange(S)[None])
        dmask = torch.triu(torch.full((S, S), float("-inf")), diagonal=1)[None, None]
        hooks = []
        for layer in dec_m.layers:
            ca = layer.cross_attention
            hooks.append(ca.q_proj.register_forward_hook(lambda _m, _a, out: rope_heads(out, dcos, dsin, hd)))

            def k_hook(_m, _a, out):
                out = rope_heads(out, ecos, esin, hd).clone()
                out[:, n_text:] = 0.0  # cross K stored for the prompt positions only; the rest stays cleared
                return out
            hooks.append(ca.k_proj.register_forward_hook(k_hook))
        try:
            for layer in dec_m.layers:
                x = layer(x, (dcos, dsin), dmask, enc_out, encoder_attention_mask=None, past_key_values=None)
        finally:
            for hk in hooks:
                hk.remove()
        x = dec_m.norm(x)
        lg = m.logits_dense(x).view(2, S, cfg.n_output_heads, cfg.output_vocab_size)
        cond, uncond = lg[0], lg[1]
        return (cond + cfg.cfg_scale * (cond - uncond)).numpy()


@pytest.mark.parametrize("text,steps", [(b"\x01 hi.", 4), (b"\x01 hello there, pin me.", 6)])
def test_dia_graph_matches_transformers_dia(text, steps):
    cfg = ttship.dia_config(**TINY)
    d = ttship.Dia(py_oracle.iface(4), cfg)
    try:
        w = d.weights()
        ids = np.frombuffer(text, dtype=np.uint8).astype(np.int32)
        rng = np.random.default_rng(len(text))
        audio = rng.integers(0, cfg.output_vocab_size, (steps, cfg.n_output_heads)).astype(np.int32)
        got = [d.prefill(ids, audio[0])]
        for s in range(1, steps):
            got.append(d.decode(audio[s]))
        got = np.stack(got)
    finally:
        d.close()
    rows = np.zeros((2, cfg.max_encoder_context_length), dtype=np.int32)
    rows[0, :len(ids)] = ids
    m = dia_from_runner(w, cfg)
    ref = run_transformers(m, cfg, rows, len(ids), audio.tolist())
    scale = np.abs(ref).max()
    err = np.abs(got - ref).max()
    assert err <= 1e-4 * scale, (err, scale)
    assert np.array_equal(got.argmax(-1), ref.argmax(-1))
