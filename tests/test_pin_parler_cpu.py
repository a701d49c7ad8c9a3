"""Parler decoder graph pinned to an independent implementation: transformers' Musicgen decoder.

The oracle and the HIP backend both run the node lists built by tts.cpp_amd/csrc/parler.cpp, so the
GPU suite proves kernels == oracle on that list, not that the list is the reference's model (VERDICT r4,
weak 1).  Parler-TTS's decoder is MusicGen's (ParlerTTSForCausalLM forks MusicgenForCausalLM): pre-norm
LayerNorm blocks of self-attention, cross-attention over the text encoding and a GELU MLP, a final
LayerNorm and one head per codebook -- what TTS.cpp's build_parler_graph restates
(/root/reference/src/models/parler/model.cpp:520-614, weights per
/root/reference/py-gguf/tts_encoders/parler_tts_gguf_encoder.py).  Here transformers'
MusicgenDecoderLayer stack, final LayerNorm and lm_heads run on the runner's own (F32, tiny) weights:
  - the inputs are composed as the runner composes them (prompt-token embeddings for the prompt pass,
    the sum of the nine codebook embeddings for an audio step, plus the stored positional table,
    parler_build_inp_embd model.cpp:387-410): MusicgenModel's own inputs_embeds path adds one position
    to every token, so the embeddings are added here and the decoder layers are called directly;
  - the MLP activation is ggml's GELU (TTS.cpp's ggml_gelu: tanh form looked up through an fp16 table),
    not MusicGen's erf GELU, which TTS.cpp does not compute;
  - the whole sequence (prompt + audio steps) runs at once under a causal mask, against the runner's
    prompt pass + step-by-step KV-cache decode.
Logits of every audio step must agree to 1e-4 of their scale.  Parity vs ggml-cpu itself stays
unpinned (no reference vectors); this pins the graph structure."""
import numpy as np
import pytest

import py_oracle
import ttship

torch = pytest.importorskip("torch")
transformers = pytest.importorskip("transformers")

CFG = dict(n_layers=2, hidden_size=128, n_attn_heads=4, ffn_size=256, max_ctx=64, prompt_vocab=300, max_positions=80,
           n_encode=3, weight_type=ttship.F32, head_type=ttship.F32, batch=1)


class GgmlGelu(torch.nn.Module):
    """ggml_gelu_f32 through the fp16 table (GGML_GELU_FP16): x rounded to fp16, the tanh form in f32, the
    result rounded to fp16."""

    def forward(self, x):
        h = x.to(torch.float16).to(torch.float32)
        c = float(np.float32(0.79788456080286535587989211986876))
        g = 0.5 * h * (1.0 + torch.tanh(c * h * (1.0 + 0.044715 * h * h)))
        return g.to(torch.float16).to(torch.float32)


def musicgen_from_runner(w, cfg):
    from transformers import MusicgenDecoderConfig, MusicgenForCausalLM
    mc = MusicgenDecoderConfig(vocab_size=cfg.output_vocab, max_position_embeddings=cfg.max_positions, num_hidden_layers=cfg.n_layers,
                               ffn_dim=cfg.ffn_size, num_attention_heads=cfg.n_attn_heads, hidden_size=cfg.hidden_size,
                               num_codebooks=cfg.n_output_heads, dropout=0.0, activation_function="gelu",
                               pad_token_id=None, bos_token_id=None)
    mc._attn_implementation = "eager"
    m = MusicgenForCausalLM(mc).eval()
    sd = {}
    for l in range(cfg.n_layers):
        pre = f"layers.{l}"
        for blk in ("self_attn", "encoder_attn"):
            for pr in ("q_proj", "k_proj", "v_proj", "out_proj"):
                sd[f"model.decoder.{pre}.{blk}.{pr}.weight"] = w[f"{pre}.{blk}.{pr}.weight"]
        for ln in ("self_attn_layer_norm", "encoder_attn_layer_norm", "final_layer_norm"):
            sd[f"model.decoder.{pre}.{ln}.weight"] = w[f"{pre}.{ln}.weight"]
            sd[f"model.decoder.{pre}.{ln}.bias"] = w[f"{pre}.{ln}.bias"]
        sd[f"model.decoder.{pre}.fc1.weight"] = w[f"{pre}.fc1.weight"]
        sd[f"model.decoder.{pre}.fc2.weight"] = w[f"{pre}.fc2.weight"]
    sd["model.decoder.layer_norm.weight"] = w["layer_norm.weight"]
    sd["model.decoder.layer_norm.bias"] = w["layer_norm.bias"]
    for i in range(cfg.n_output_heads):
        sd[f"lm_heads.{i}.weight"] = w[f"lm_heads.{i}.weight.head"]
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}, strict=False)
    assert not unexpected, unexpected
    # left out on purpose: the token embeddings (composed here) and the sinusoidal buffer (the runner's table is used)
    assert all(k.startswith("model.decoder.embed_tokens.") for k in missing), missing
    for layer in m.model.decoder.layers:
        layer.activation_fn = GgmlGelu()
    return m


def run_musicgen(m, w, cfg, prompt, audio):
    """Logits [steps, heads, vocab] of the audio positions of prompt + audio steps."""
    n, k = len(prompt), len(audio)
    pos = w["positional_embed"]
    emb = [w["embed_prompts"][t] + pos[j] for j, t in enumerate(prompt)]
    for s, toks in enumerate(audio):
        e = sum(w[f"embed_tokens.{i}.weight"][t] for i, t in enumerate(toks))
        emb.append(e + pos[n + s])
    h = torch.from_numpy(np.stack(emb).astype(np.float32))[None]
    T = n + k
    mask = torch.triu(torch.full((T, T), float("-inf")), diagonal=1)[None, None]
    enc = torch.from_numpy(w["text_encoding"].reshape(cfg.n_encode, cfg.hidden_size))[None]
    with torch.no_grad():
        for layer in m.model.decoder.layers:
            h = layer(h, attention_mask=mask, encoder_hidden_states=enc, encoder_attention_mask=None, past_key_values=None, use_cache=False)
            h = h[0] if isinstance(h, tuple) else h
        h = m.model.decoder.layer_norm(h)
        logits = torch.stack([head(h) for head in m.lm_heads], dim=2)  # [1, T, heads, vocab]
    return logits[0, n:].numpy()


@pytest.mark.parametrize("n_prompt,steps", [(5, 4), (11, 6)])
def test_parler_graph_matches_musicgen_decoder(n_prompt, steps):
    cfg = ttship.parler_config(**CFG)
    p = ttship.Parler(py_oracle.iface(4), cfg)
    try:
        w = p.weights()
        rng = np.random.default_rng(n_prompt)
        prompt = rng.integers(0, cfg.prompt_vocab, n_prompt).astype(np.int32)
        audio = rng.integers(0, cfg.audio_vocab, (steps, cfg.n_output_heads)).astype(np.int32)
        p.prefill(prompt.reshape(1, -1))
        got = np.stack([p.decode(audio[s].reshape(1, -1)).reshape(cfg.n_output_heads, cfg.output_vocab) for s in range(steps)])
    finally:
        p.close()
    m = musicgen_from_runner(w, cfg)
    ref = run_musicgen(m, w, cfg, prompt.tolist(), audio.tolist())
    scale = np.abs(ref).max()
    err = np.abs(got - ref).max()
    assert err <= 1e-4 * scale, (err, scale)
    assert np.array_equal(got.argmax(-1), ref.argmax(-1))


def test_parler_lockstep_batch_matches_musicgen_per_prompt():
    """The lock-step batch the headline bench decodes (batch > 1: every GEMV with B columns, each prompt its
    own KV-cache sequence): every prompt's logits are transformers' decoder run on that prompt alone."""
    B, n_prompt, steps = 3, 6, 4
    cfg = ttship.parler_config(**dict(CFG, batch=B))
    p = ttship.Parler(py_oracle.iface(4), cfg)
    try:
        w = p.weights()
        rng = np.random.default_rng(77)
        prompts = rng.integers(0, cfg.prompt_vocab, (B, n_prompt)).astype(np.int32)
        audio = rng.integers(0, cfg.audio_vocab, (steps, B, cfg.n_output_heads)).astype(np.int32)
        p.prefill(prompts)
        got = np.stack([p.decode(audio[s]).reshape(B, cfg.n_output_heads, cfg.output_vocab) for s in range(steps)], axis=1)
    finally:
        p.close()
    m = musicgen_from_runner(w, cfg)
    for b in range(B):
        ref = run_musicgen(m, w, cfg, prompts[b].tolist(), audio[:, b].tolist())
        scale = np.abs(ref).max()
        err = np.abs(got[b] - ref).max()
        assert err <= 1e-4 * scale, (b, err, scale)
        assert np.array_equal(got[b].argmax(-1), ref.argmax(-1)), b
