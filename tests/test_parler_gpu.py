"""End-to-end Parler decoder parity: the HIP backend vs the CPU oracle on the same graph.

Bars (BASELINE.json north_star): greedy (sampler::max) token ids bit-exact at fixed seed;
logits within 1e-4 * max|logit| + 1e-4 (f32 reduction order is the only difference).
"""
import numpy as np
import pytest

import py_oracle
import ttship

TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=128,
            prompt_vocab=512, max_positions=160)


def make_pair(hip, **kw):
    cfg = ttship.parler_config(**kw)
    g = ttship.Parler(hip.iface(), cfg)
    c = ttship.Parler(py_oracle.iface(8), ttship.parler_config(**kw))
    return g, c


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3])
def test_tiny_tokens_and_logits(hip, batch):
    g, c = make_pair(hip, batch=batch, **TINY)
    try:
        prompt = (np.arange(7 * batch, dtype=np.int32).reshape(batch, 7) * 37) % 512
        g.prefill(prompt)
        c.prefill(prompt)
        tg = g.generate(12)
        tc = c.generate(12)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
        toks = np.full((batch, 9), 5, dtype=np.int32)
        lg = g.decode(toks)
        lc = c.decode(toks)
        tol = 1e-4 * np.abs(lc).max() + 1e-4
        assert np.abs(lg - lc).max() <= tol, np.abs(lg - lc).max()
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
def test_full_parler_mini_q4k_tokens(hip):
    """Full Parler-mini shapes (24 layers, d=1024, Q4_K), batch 2, 6 greedy steps."""
    g, c = make_pair(hip, batch=2)
    try:
        prompt = np.array([[11, 29, 400, 7, 1, 3000, 16], [5, 6, 7, 8, 9, 10, 11]], dtype=np.int32)
        g.prefill(prompt)
        c.prefill(prompt)
        tg = g.generate(6)
        tc = c.generate(6)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ks", [0, 256])
def test_full_parler_mini_q4k_tokens_mfma(hip, ks):
    """Full Parler-mini at batch 3 with every Q4_K matrix in the tile layout: all GEMVs (LN /
    quantize prologues, grouped q/k/v with KV-store epilogues, GELU / residual epilogues) on a
    matrix-core kernel (k_gemv_q4K_mf with GEMV_KS = 0, the K-split k_gemv_q4K_ks otherwise),
    cross-attention unfused, embeddings gathered from tiled tables."""
    hip.set_option(ttship.OPT["Q4K_TILE_BYTES"], 1)  # every Q4_K matrix (and embedding table) tiled
    hip.set_option(ttship.OPT["GEMV_KS"], ks)
    try:
        g, c = make_pair(hip, batch=3)
    finally:
        hip.set_option(ttship.OPT["Q4K_TILE_BYTES"], 4 << 20)
    try:
        prompt = np.array([[11, 29, 400, 7, 1, 3000, 16], [5, 6, 7, 8, 9, 10, 11], [1, 1, 2, 3, 5, 8, 13]], dtype=np.int32)
        g.prefill(prompt)
        c.prefill(prompt)
        tg = g.generate(6)
        tc = c.generate(6)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
    finally:
        hip.set_option(ttship.OPT["GEMV_KS"], 256)
        g.close()
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("device_sampling", [True, False])
def test_generate_in_chunks_and_sampling_paths(hip, device_sampling):
    """generate(5) + generate(7) on the HIP runner (device-resident greedy loop or host sampling)
    == generate(12) on the oracle: the EOS / last-token state carries across calls."""
    g, c = make_pair(hip, batch=3, **TINY)
    try:
        g.set_device_sampling(device_sampling)
        prompt = (np.arange(21, dtype=np.int32).reshape(3, 7) * 53) % 512
        g.prefill(prompt)
        c.prefill(prompt)
        tg = np.concatenate([g.generate(5), g.generate(7)], axis=1)
        tc = c.generate(12)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
def test_device_sampling_eos_rule(hip):
    """Pick an EOS id the model actually emits (from an oracle run), so heads hit EOS mid-run and
    must keep feeding EOS afterwards (next_decoder_token_ids); device path == oracle."""
    prompt = (np.arange(14, dtype=np.int32).reshape(2, 7) * 41) % 512
    probe = ttship.Parler(py_oracle.iface(8), ttship.parler_config(batch=2, **TINY))
    try:
        probe.prefill(prompt)
        t = probe.generate(10)
    finally:
        probe.close()
    vals, counts = np.unique(t[:, 3:6, :], return_counts=True)
    eos = int(vals[np.argmax(counts)])
    kw = dict(TINY, batch=2)
    cfg_g, cfg_c = ttship.parler_config(**kw), ttship.parler_config(**kw)
    cfg_g.eos_token = cfg_c.eos_token = eos
    g = ttship.Parler(hip.iface(), cfg_g)
    c = ttship.Parler(py_oracle.iface(8), cfg_c)
    try:
        g.prefill(prompt)
        c.prefill(prompt)
        tg, tc = g.generate(12), c.generate(12)
        assert (tc == eos).any()
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 4])
def test_graph_replay_across_kernel_switches(hip, batch):
    """The step graph is recorded once and then updated in place (hipGraphExecUpdate) every step; here the
    KV length crosses the attention kernel boundaries (k_attn_small up to 64 keys, the row kernel, the
    split pair from 128 keys, its chunk count growing), so the update sees new grids and new kernels.
    Tokens bit-exact vs the oracle over 75 steps, and the replayed runner's logits bit-identical to a
    runner on a backend that launches every step eagerly (graphs off)."""
    kw = dict(TINY, max_ctx=192, max_positions=256)
    g, c = make_pair(hip, batch=batch, **kw)
    eager_be = ttship.HipBackend(0)
    eager_be.set_option(ttship.OPT["GRAPHS"], 0)
    e = ttship.Parler(eager_be.iface(), ttship.parler_config(batch=batch, **kw))
    try:
        prompt = (np.arange(60 * batch, dtype=np.int32).reshape(batch, 60) * 53 + 11) % 512
        for r in (g, c, e):
            r.prefill(prompt)
        tg, tc, te = g.generate(75), c.generate(75), e.generate(75)
        assert np.array_equal(tg, tc), f"token mismatch vs oracle\n{tg}\n{tc}"
        assert np.array_equal(tg, te)
        toks = np.full((batch, 9), 5, dtype=np.int32)
        lg, le = g.decode(toks), e.decode(toks)
        assert np.array_equal(lg, le)
    finally:
        e.close()
        eager_be.close()
        g.close()
        c.close()


@pytest.mark.gpu
def test_many_prompt_step_in_kernel_operands(hip):
    """Parler-mini Q4_K at 32 lock-step prompts (every decode product has M = 32 > 8 columns: the K-relay
    GEMM over two column tiles) with the LN / quantize prologues inside the GEMM workgroups
    (TTS_HIP_OPT_GEMM_KR_INKERNEL), with both column tiles in one workgroup in turn (TTS_HIP_OPT_GEMM_KR_CT2)
    and on parallel wave halves (TTS_HIP_OPT_GEMM_KR_CP), against the default: tokens and logits bit-identical, tokens equal to the oracle's."""
    B = 32
    prompt = (np.arange(7 * B, dtype=np.int32).reshape(B, 7) * 41 + 3) % 1000
    ink_be = ttship.HipBackend(0)
    ink_be.set_option(ttship.OPT["GEMM_KR_INKERNEL"], 64)
    ct2_be = ttship.HipBackend(0)
    ct2_be.set_option(ttship.OPT["GEMM_KR_CT2"], 1)
    k2 = ttship.Parler(ct2_be.iface(), ttship.parler_config(batch=B))
    cp_be = ttship.HipBackend(0)
    cp_be.set_option(ttship.OPT["GEMM_KR_CP"], 1)
    k3 = ttship.Parler(cp_be.iface(), ttship.parler_config(batch=B))
    g, c = make_pair(hip, batch=B)
    k = ttship.Parler(ink_be.iface(), ttship.parler_config(batch=B))
    try:
        for r in (g, c, k, k2, k3):
            r.prefill(prompt)
        tg, tc, tk, t2, t3 = g.generate(4), c.generate(4), k.generate(4), k2.generate(4), k3.generate(4)
        assert np.array_equal(tg, tc), f"token mismatch vs oracle\n{tg}\n{tc}"
        assert np.array_equal(tk, tg) and np.array_equal(t2, tg) and np.array_equal(t3, tg)
        toks = np.full((B, 9), 5, dtype=np.int32)
        lg = g.decode(toks)
        assert np.array_equal(lg, k.decode(toks)) and np.array_equal(lg, k2.decode(toks)) and np.array_equal(lg, k3.decode(toks))
    finally:
        k3.close()
        cp_be.close()
        k2.close()
        ct2_be.close()
        k.close()
        ink_be.close()
        g.close()
        c.close()


@pytest.mark.gpu
def test_scratch_grows_after_plans_ran():
    """A runner that has generated (plans recorded into the backend's two slots) then runs a prompt pass
    whose staged columns exceed the 64 MiB scratch: the scratch grows once the launched plans have run
    and their recordings are dropped (growth used to be refused for good once any plan had been
    recorded).  Tokens after the second prompt pass equal a fresh runner's."""
    be = ttship.HipBackend(0)
    be.set_option(ttship.OPT["GRAPHS"], 1)
    cfg = ttship.parler_config(batch=16, max_ctx=512, arena_bytes=8 << 30)
    small = (np.arange(16 * 8, dtype=np.int32).reshape(16, 8) * 37) % cfg.prompt_vocab
    big = (np.arange(16 * 448, dtype=np.int32).reshape(16, 448) * 53) % cfg.prompt_vocab
    p = ttship.Parler(be.iface(), cfg)
    try:
        p.prefill(small)
        p.generate(4)  # plans recorded and launched
        p.reset()
        p.prefill(big)  # 16 x 448 columns of K = 4096: > 64 MiB of staged columns
        got = p.generate(3)
    finally:
        p.close()
    q = ttship.Parler(be.iface(), cfg)
    try:
        q.prefill(big)
        ref = q.generate(3)
    finally:
        q.close()
        be.close()
    assert np.array_equal(got, ref)


def _ragged_prompts(lens, vocab):
    return [((np.arange(L, dtype=np.int32) * (31 + 2 * r) + 5 * r + 1) % vocab).astype(np.int32) for r, L in enumerate(lens)]


@pytest.mark.gpu
@pytest.mark.parametrize("device_sampling", [True, False])
def test_ragged_batch_tiny(hip, device_sampling):
    """Prompts of 5, 9, 7 and 12 tokens in ONE prompt pass (tts_parler_prefill_ragged), then decoded in
    lockstep, each at its own position with its own mask: tokens equal the oracle's ragged batch and each
    prompt's own B = 1 run on the GPU."""
    lens = [5, 9, 7, 12]
    prompts = _ragged_prompts(lens, 512)
    g, c = make_pair(hip, batch=4, **TINY)
    try:
        g.set_device_sampling(device_sampling)
        g.prefill_ragged(prompts)
        c.prefill_ragged(prompts)
        tg = g.generate(12)
        tc = c.generate(12)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
    finally:
        g.close()
        c.close()
    one = ttship.Parler(hip.iface(), ttship.parler_config(batch=1, **TINY))
    try:
        for r, p in enumerate(prompts):
            one.reset()
            one.prefill(p.reshape(1, -1))
            assert np.array_equal(one.generate(12)[0], tg[r]), f"prompt {r}"
    finally:
        one.close()


@pytest.mark.gpu
def test_ragged_prompt_pass_parler_mini(hip):
    """Parler-mini Q4_K (full shapes): the perf_battery sentences' word-piece lengths (bench.py
    sentence_tokens) as one ragged prompt pass of 8 prompts, 16 decode steps: every prompt's tokens equal
    its own prompt pass and decode alone (TTS.cpp's one-prompt generate, model.cpp:838-858)."""
    import sys
    import pathlib
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
    import bench
    cfg = ttship.parler_config(batch=8, max_ctx=256)
    prompts = [bench.sentence_tokens(bench.HARVARD[g], cfg.prompt_vocab) for g in range(8)]
    assert len({len(p) for p in prompts}) >= 3  # ragged
    g = ttship.Parler(hip.iface(), cfg)
    try:
        g.prefill_ragged(prompts)
        tg = g.generate(16)
    finally:
        g.close()
    one = ttship.Parler(hip.iface(), ttship.parler_config(batch=1, max_ctx=256))
    try:
        for r, p in enumerate(prompts):
            one.reset()
            one.prefill(p.reshape(1, -1))
            assert np.array_equal(one.generate(16)[0], tg[r]), f"prompt {r}"
    finally:
        one.close()
