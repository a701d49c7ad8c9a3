"""Orpheus decoder graph pinned to an independent implementation: transformers' LlamaForCausalLM.

Orpheus-3B is a Llama-3.2-3B checkpoint (the reference's converter loads it as LlamaForCausalLM,
/root/reference/py-gguf/tts_encoders/orpheus_gguf_encoder.py:5-6, and writes the Llama-3 rope scaling as
per-dimension frequency factors, :144-173).  TTS.cpp's build_orpheus_graph
(/root/reference/src/models/orpheus/model.cpp:233-312) restates it on ggml: RMSNorm, GQA attention with
neox rope_ext + the factors, SwiGLU MLP, final RMSNorm, the output head.  The oracle runs the runner's
node list (tts.cpp_amd/csrc/orpheus.cpp) on tiny F32 weights; LlamaForCausalLM runs the same weights
(names mapped as the converter maps them) over the whole token sequence.  The prompt pass's last logits
and every decode step's logits must agree to 1e-4 of their scale."""
import numpy as np
import pytest

import py_oracle
import ttship

torch = pytest.importorskip("torch")
pytest.importorskip("transformers")

CFG = dict(n_layers=2, hidden_size=128, n_attn_heads=4, n_kv_attn_heads=2, head_size=32, ffn_size=256, vocab_size=320, max_ctx=64,
           weight_type=ttship.F32, batch=1)


def llama_from_runner(w, cfg):
    from transformers import LlamaConfig, LlamaForCausalLM
    lc = LlamaConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.ffn_size, num_hidden_layers=cfg.n_layers,
                     num_attention_heads=cfg.n_attn_heads, num_key_value_heads=cfg.n_kv_attn_heads, head_dim=cfg.head_size,
                     rms_norm_eps=1e-5, rope_theta=float(cfg.rope_theta), max_position_embeddings=131072, tie_word_embeddings=False,
                     rope_scaling={"rope_type": "llama3", "factor": float(cfg.rope_factor), "low_freq_factor": float(cfg.rope_low_freq_factor),
                                   "high_freq_factor": float(cfg.rope_high_freq_factor),
                                   "original_max_position_embeddings": int(cfg.rope_original_ctx)},
                     attention_bias=False, mlp_bias=False, pad_token_id=None, bos_token_id=None, eos_token_id=None)
    lc._attn_implementation = "eager"
    m = LlamaForCausalLM(lc).eval()
    sd = {"model.embed_tokens.weight": w["token_embd"], "lm_head.weight": w["output"], "model.norm.weight": w["output_norm"]}
    names = {"input_norm": "input_layernorm", "post_attention_norm": "post_attention_layernorm", "q": "self_attn.q_proj",
             "k": "self_attn.k_proj", "v": "self_attn.v_proj", "o": "self_attn.o_proj", "gate": "mlp.gate_proj", "up": "mlp.up_proj",
             "down": "mlp.down_proj"}
    for l in range(cfg.n_layers):
        for ours, hf in names.items():
            sd[f"model.layers.{l}.{hf}.weight"] = w[f"layers.{l}.{ours}"]
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}, strict=False)
    assert not unexpected and not [k for k in missing if "rotary" not in k], (missing, unexpected)
    return m


@pytest.mark.parametrize("n_prompt,steps", [(6, 5), (13, 3)])
def test_orpheus_graph_matches_llama(n_prompt, steps):
    cfg = ttship.orpheus_config(**CFG)
    o = ttship.Orpheus(py_oracle.iface(4), cfg)
    try:
        w = o.weights()
        rng = np.random.default_rng(n_prompt + 100)
        prompt = rng.integers(0, cfg.vocab_size, n_prompt).astype(np.int32)
        toks = rng.integers(0, cfg.vocab_size, steps).astype(np.int32)
        got = [o.prefill(prompt.reshape(1, -1)).reshape(-1)]
        for t in toks:
            got.append(o.decode(np.array([t], np.int32)).reshape(-1))
        got = np.stack(got)
    finally:
        o.close()
    m = llama_from_runner(w, cfg)
    ids = torch.from_numpy(np.concatenate([prompt, toks]).astype(np.int64))[None]
    with torch.no_grad():
        ref = m(input_ids=ids).logits[0, n_prompt - 1:].numpy()
    scale = np.abs(ref).max()
    err = np.abs(got - ref).max()
    assert err <= 1e-4 * scale, (err, scale)
    assert np.array_equal(got.argmax(-1), ref.argmax(-1))


def test_orpheus_lockstep_batch_matches_llama_per_prompt():
    """The lock-step batch (configs[4] decodes 8 prompts per GPU this way): each prompt's last prompt-pass
    logits and decode-step logits are LlamaForCausalLM's on that prompt alone."""
    B, n_prompt, steps = 3, 7, 3
    cfg = ttship.orpheus_config(**dict(CFG, batch=B))
    o = ttship.Orpheus(py_oracle.iface(4), cfg)
    try:
        w = o.weights()
        rng = np.random.default_rng(123)
        prompts = rng.integers(0, cfg.vocab_size, (B, n_prompt)).astype(np.int32)
        toks = rng.integers(0, cfg.vocab_size, (steps, B)).astype(np.int32)
        got = [o.prefill(prompts).reshape(B, -1)]
        for t in toks:
            got.append(o.decode(t).reshape(B, -1))
        got = np.stack(got, axis=1)  # [B, 1 + steps, vocab]
    finally:
        o.close()
    m = llama_from_runner(w, cfg)
    for b in range(B):
        ids = torch.from_numpy(np.concatenate([prompts[b], toks[:, b]]).astype(np.int64))[None]
        with torch.no_grad():
            ref = m(input_ids=ids).logits[0, n_prompt - 1:].numpy()
        scale = np.abs(ref).max()
        err = np.abs(got[b] - ref).max()
        assert err <= 1e-4 * scale, (b, err, scale)
        assert np.array_equal(got[b].argmax(-1), ref.argmax(-1)), b
