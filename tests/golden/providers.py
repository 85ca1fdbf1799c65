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
