"""Deterministic ``next_token_probs`` providers for the generic-provider fixtures (test infrastructure).

``ContextDictLM`` returns a ``{id: p}`` ProbDist over 40 ids whose choice and weights depend on the context it
is given (its length and last three ids), so a coder that feeds the provider the wrong context -- or trims it
differently from ``max_context`` -- diverges at once.
"""

from __future__ import annotations

import numpy as np


class ContextDictLM:
    def __init__(self, vocab: int = 500, seed: int = 5, support: int = 40):
        self.vocab, self.seed, self.support = int(vocab), int(seed), int(support)
        self.calls = []

    def next_token_probs(self, context_ids):
        ctx = [int(t) for t in context_ids]
        self.calls.append(tuple(ctx))
        key = [self.seed, len(ctx)] + ctx[-3:]
        rng = np.random.default_rng(key)
        ids = rng.choice(self.vocab, size=self.support, replace=False)
        w = rng.random(self.support) ** 3 + 1e-3
        w = w / w.sum()
        return {int(i): float(p) for i, p in zip(ids, w)}


def near_tie_values(rng, n: int, alpha: float, scale: float) -> np.ndarray:
    """Zipf(alpha) weights over n ranks in clusters of four whose members differ by 1e-9 .. 1e-8 relative (far
    above float64 resolution, far below float32's), scaled by ``scale`` (rows need not sum to 1: the reference's
    apply_quality filters the raw values), in a random id order."""
    w = np.arange(1, n + 1, dtype=np.float64) ** -float(alpha)
    w /= w.sum()
    head = w[(np.arange(n) // 4) * 4]  # every member takes its cluster head's weight ...
    u = rng.uniform(1e-9, 1e-8, size=(n + 3) // 4)
    step = np.repeat(u, 4)[:n] * (3 - np.arange(n) % 4)  # ... times 1 + 3u, 1 + 2u, 1 + u, 1
    vals = head * (1.0 + step) * float(scale)
    return vals[rng.permutation(n)]


class NearTieLM:
    """float64 ndarray ProbDist over ``vocab`` ids (default GPT-2's 50,257) with near-tied neighbours in the
    ranking (near_tie_values): a coder that stages the row at float32 merges the neighbours and breaks the
    ties by id, so its tokens and the top_p / min_prob boundaries differ from the reference's.  Context
    dependent (length and last two ids)."""

    def __init__(self, vocab: int = 50257, seed: int = 8, alpha: float = 1.05, scale: float = 1.21):
        self.vocab, self.seed, self.alpha, self.scale = int(vocab), int(seed), float(alpha), float(scale)
        self.calls = []

    def next_token_probs(self, context_ids):
        ctx = [int(t) for t in context_ids]
        self.calls.append(tuple(ctx))
        rng = np.random.default_rng([self.seed, len(ctx)] + ctx[-2:])
        return near_tie_values(rng, self.vocab, self.alpha, self.scale)


class NearTieDictLM:
    """``{id: p}`` ProbDist over ``support`` ids drawn from a large id space (ids beyond 2^17), near-tied as
    NearTieLM, context dependent."""

    def __init__(self, vocab: int = 200000, support: int = 3000, seed: int = 9, alpha: float = 0.9,
                 scale: float = 1.0):
        self.vocab, self.support, self.seed = int(vocab), int(support), int(seed)
        self.alpha, self.scale = float(alpha), float(scale)
        self.calls = []

    def next_token_probs(self, context_ids):
        ctx = [int(t) for t in context_ids]
        self.calls.append(tuple(ctx))
        rng = np.random.default_rng([self.seed, len(ctx)] + ctx[-3:])
        ids = rng.choice(self.vocab, size=self.support, replace=False)
        vals = near_tie_values(rng, self.support, self.alpha, self.scale)
        return {int(i): float(p) for i, p in zip(ids, vals)}
