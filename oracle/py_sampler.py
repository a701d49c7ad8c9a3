"""TEST INFRASTRUCTURE ONLY (parity oracle; never imported by the product path).

Pure-Python / numpy-float32 restatement of TTS.cpp's sampler (sampler::sample, softmax, topk, topp,
max; /root/reference/src/sampler.cpp:3-204) with the seeded generator the backend documents in
include/tts_hip.h (tts_sampler_call_seed): the per-call std::minstd_rand of sampler.cpp:47 seeded
from (seed, prompt, call), and std::uniform_real_distribution<float> as libstdc++ computes it
(generate_canonical<float, 24>: one draw, float(g - 1) / 2^31, clamped below 1).  Every f32
operation is done on np.float32 scalars so each rounds as the C++ float expression does; expf is
the correctly rounded value (float(exp(double))), the backend's policy for every transcendental.
Ties in the top-k order go to the lower index (std::sort leaves them unspecified).

Checks: tests/test_sampler_cpu.py (host C++ sampler == this), tests/test_sampler_gpu.py (device
sampler == host sampler), and the runner-level sampled-token tests against the oracle backend.
"""
import math

import numpy as np

F = np.float32
M31 = 2147483647


def call_seed(seed, stream, call):
    """tts_sampler_call_seed: splitmix64 of (seed, stream, call) -> 1 .. 2^31 - 2."""
    mask = (1 << 64) - 1
    z = (seed ^ ((stream & 0xFFFFFFFF) << 40) ^ ((call * 0x9E3779B97F4A7C15) & mask)) & mask
    z = (z + 0x9E3779B97F4A7C15) & mask
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & mask
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & mask
    z ^= z >> 31
    return 1 + z % 2147483646


class MinStd:
    """std::minstd_rand (x <- 48271 x mod 2^31 - 1) with uniform_real_distribution<float>(0, 1)."""

    def __init__(self, s):
        self.x = s % M31 or 1

    def uniform(self):
        self.x = (self.x * 48271) % M31
        r = F(F(self.x - 1) * F(2.0 ** -31))
        return F(np.nextafter(F(1), F(0))) if r >= F(1) else r


def expf(x):
    return F(math.exp(float(x)))


class Sampler:
    """One runner's sampler (sampler.h): configuration + repetition state per head."""

    def __init__(self, n_heads, vocab, temperature=1.0, top_k=50, top_p=1.0, repetition_penalty=1.0, do_sample=True, seed=0x5EED):
        self.NH, self.V = n_heads, vocab
        self.temperature, self.top_k, self.top_p = F(temperature), top_k, F(top_p)
        self.rep = F(repetition_penalty)
        self.do_sample, self.seed = do_sample, seed
        self.reset()

    def reset(self):
        self.last = [-1] * self.NH
        self.count = [0] * self.NH

    def _penal(self, h, i, v):
        if self.rep != F(1) and self.last[h] == i:
            return F(float(v) / math.pow(float(self.rep), float(self.count[h])))
        return F(v)

    def sample(self, logits, stream=0, call=0):
        """logits: [NH, V] float32 (not modified) -> list of NH token ids."""
        NH, V = self.NH, self.V
        L = [np.array(logits[h], dtype=np.float32).copy() for h in range(NH)]
        maxi = []
        for h in range(NH):  # sampler::max
            mx, idx = F(-np.inf), 0
            for i in range(V):
                v = self._penal(h, i, L[h][i])
                if v > mx:
                    mx, idx = v, i
            maxi.append(idx)
        if not self.do_sample:
            return maxi
        temp = self.temperature != F(1)
        picks = []

        def softmax():
            use = len(picks) > 0
            for h in range(NH):
                row = L[h]
                mv = self._penal(h, maxi[h], row[maxi[h]])
                if temp:
                    mv = F(mv / self.temperature)
                cum = F(0)
                order = picks[h] if use else range(V)
                for ii in order:
                    v = self._penal(h, ii, row[ii])
                    if temp:
                        v = F(v / self.temperature)
                    v = expf(F(v - mv))
                    cum = F(cum + v)
                    row[ii] = v
                for ii in order:
                    row[ii] = F(row[ii] / cum)

        def order_of(h, penalised):
            key = [self._penal(h, i, L[h][i]) if penalised else F(L[h][i]) for i in range(V)]
            return sorted(range(V), key=lambda i: (-float(key[i]), i))

        performed = False
        nucleus = False
        if self.top_p < F(1):
            softmax()
            performed = True
        if 0 < self.top_k < V:
            picks = [order_of(h, not performed)[: self.top_k] for h in range(NH)]
            nucleus = True
        if self.top_p >= F(1):
            softmax()
        mhp = []
        if self.top_p < F(1):
            if not picks:
                picks = [order_of(h, False) for h in range(NH)]
            for h in range(NH):
                ps, trim = F(0), -1
                for ii, idx in enumerate(picks[h]):
                    ps = F(ps + L[h][idx])
                    if ps >= self.top_p:
                        trim = ii + 1
                        break
                mhp.append(min(ps, self.top_p))
                if trim > 0:
                    picks[h] = picks[h][:trim]
            nucleus = True
        gen = MinStd(call_seed(self.seed, stream, call))
        out = []
        for h in range(NH):
            u = gen.uniform()
            a = F(u * mhp[h]) if self.top_p < F(1) else u
            cum = F(0)
            order = picks[h] if nucleus else list(range(V))
            for j, ii in enumerate(order):
                cum = F(cum + L[h][ii])
                if a <= cum or j >= len(order) - 1:
                    if self.rep != F(1):
                        if self.last[h] != ii:
                            self.count[h] = 0
                        self.last[h] = ii
                        self.count[h] += 1
                    out.append(ii)
                    break
        return out
