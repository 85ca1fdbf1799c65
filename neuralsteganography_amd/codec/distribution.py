"""``next_token_probs`` providers (``src/neuralstego/codec/distribution.py``; a15 of SURVEY §8).

* :class:`HipTransformersLM` -- ``TransformersLM.next_token_probs`` (``:107-142``) on the GPU: GPT-2 logits of
  the context (KV cache kept and extended when the next query appends one token, instead of the
  reference's full re-forward per query), float64 softmax of ``logits / temperature`` and the
  ``top_k`` / ``top_p`` / ``min_prob`` support renormalised, computed by the HIP rank kernel
  (``ns_token_probs``).
* :class:`MockLM` -- the fixed Zipf distribution of ``:17-37`` (host).
* :class:`CachedLM` -- the LRU memo of ``:40-60`` (host).
* :class:`ProviderBatchedLM` -- the batched-LM protocol over ANY ``next_token_probs`` provider (the L2 protocol
  of ``codec/types.py:41-45``), so the rank kernel serves ``encode_with_lm`` / ``decode_with_lm`` for user
  providers too (``codec/arithmetic.py:122-231`` takes any provider).
"""

from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Optional, Sequence

import numpy as np

from .. import _lib
from ..exceptions import ConfigurationError


class MockLM:
    """Context-free Zipf prior: p(rank r) proportional to r^-alpha over ``vocab_size`` ids."""

    def __init__(self, vocab_size: int = 32, alpha: float = 1.2):
        if vocab_size <= 0:
            raise ValueError("vocab_size must be positive")
        if alpha <= 0:
            raise ValueError("alpha must be positive")
        w = np.arange(1, vocab_size + 1, dtype=np.float64) ** -float(alpha)
        self.vocab_size, self.alpha = int(vocab_size), float(alpha)
        self._p = w / w.sum()

    def next_token_probs(self, context_ids: Sequence[int]) -> np.ndarray:
        del context_ids
        return self._p.copy()


class CachedLM:
    """Memoise ``next_token_probs`` per context tuple (least recently used eviction beyond ``maxsize``)."""

    def __init__(self, lm, *, maxsize: int = 128):
        if maxsize <= 0:
            raise ValueError("maxsize must be positive")
        self._lm, self._maxsize = lm, int(maxsize)
        self._memo: "OrderedDict[tuple, object]" = OrderedDict()

    def next_token_probs(self, context_ids: Sequence[int]):
        key = tuple(int(t) for t in context_ids)
        if key in self._memo:
            self._memo.move_to_end(key)
        else:
            self._memo[key] = self._lm.next_token_probs(list(key))
            while len(self._memo) > self._maxsize:
                self._memo.popitem(last=False)
        val = self._memo[key]
        return dict(val) if isinstance(val, dict) else np.array(val, copy=True)


class HipTransformersLM:
    """GPU ``next_token_probs`` over a batched GPT-2 (or any ``prefill``/``step`` batched LM)."""

    def __init__(self, model=None, *, batched_lm=None, temperature: float = 1.0, top_k: Optional[int] = None,
                 top_p: Optional[float] = None, min_prob: Optional[float] = None, max_context: Optional[int] = None,
                 logits_dtype: str = "f32", tokenizer=None):
        import torch

        from ..coder import CoderContext, CoderParams, rank_quality

        if temperature <= 0.0:
            raise ValueError("temperature must be positive")
        if not torch.cuda.is_available():
            raise _lib.NativeLibraryError("HipTransformersLM needs a ROCm GPU")
        if batched_lm is None:
            from ..lm.gpt2 import BatchedGPT2

            ldt = torch.float16 if logits_dtype == "f16" else torch.float32
            batched_lm = BatchedGPT2(model, device=torch.device("cuda", torch.cuda.current_device()), logits_dtype=ldt)
        self.lm, self.tokenizer = batched_lm, tokenizer
        self.vocab = self.lm.shape.vocab
        self.temperature = float(temperature)
        self.max_context = max_context
        self._q = rank_quality({"top_k": top_k, "top_p": top_p, "min_prob": min_prob})
        self._filters = (top_k, top_p, min_prob)
        params = CoderParams(vocab=self.vocab, precision=16, temp=1.0, topk=self.vocab, dtype=logits_dtype, banned=[])
        self._ctx = CoderContext(params, max_batch=1)
        dev = torch.device("cuda", self._ctx.device)
        self._probs = torch.zeros((1, self.vocab), dtype=torch.float64, device=dev)
        self._state = torch.zeros((1, 4), dtype=torch.int64, device=dev)
        self._last: Optional[tuple] = None
        self._logits = None

    def _window(self) -> Optional[int]:
        if self.max_context is not None and self.max_context > 0:
            return int(self.max_context)
        return int(getattr(self.lm.shape, "n_positions", 0)) or None

    def next_token_probs(self, context_ids: Sequence[int]) -> np.ndarray:
        return self._probs_with(context_ids, self._q)

    def _probs_with(self, context_ids: Sequence[int], q) -> np.ndarray:
        """next_token_probs under the quality struct ``q`` (the crypto quality LM passes its own)."""
        import torch

        from ..coder import _ptr, _stream_handle

        ctx = tuple(int(t) for t in context_ids)
        if not ctx:
            raise ValueError("context_ids must contain at least one token")
        win = self._window()
        if win is not None and len(ctx) > win:
            ctx = ctx[-win:]
            self._last = None  # a sliding window changes every position: recompute
        if self._last is not None and len(ctx) == len(self._last) + 1 and ctx[:-1] == self._last:
            self._logits = self.lm.step(torch.tensor([ctx[-1]], device=self._probs.device, dtype=torch.long))
        else:
            self._logits = self.lm.prefill(list(ctx), 1, 64)
        self._last = ctx
        lg = self._logits
        rc = _lib.lib().ns_token_probs(self._ctx._h, _ptr(lg), lg.stride(0), 1, self.temperature,
                                       ctypes.byref(q), _ptr(self._probs), self._probs.stride(0),
                                       _ptr(self._state), _stream_handle())
        self._ctx.check(rc, "ns_token_probs")
        return self._probs[0].cpu().numpy().copy()


# probability 0 (or negative / non-finite) as a log-probability: far enough below every real entry that the
# kernel's canonical exp gives exactly 0 (exp_canon(d) = 0 for d < -700), so the id leaves the support as the
# reference's ``probs > 0`` mask drops it (codec/arithmetic.py:366-370); finite, so key ranges stay finite
ZERO_LOGIT_GAP = 800.0


def dist_to_row(dist, vocab: int) -> np.ndarray:
    """A ProbDist (float64 ndarray by id, or ``{id: p}`` dict, ``codec/arithmetic.py:388-398``) as a float64
    probability row of ``vocab`` entries (absent ids: 0)."""
    if isinstance(dist, np.ndarray):
        row = np.asarray(dist, dtype=np.float64).reshape(-1)
        if row.size > vocab:
            raise ConfigurationError(f"distribution over {row.size} ids for a {vocab}-id vocabulary")
        if row.size < vocab:
            row = np.concatenate([row, np.zeros(vocab - row.size)])
        return row
    if isinstance(dist, dict):
        row = np.zeros(vocab, dtype=np.float64)
        for tok, prob in dist.items():
            t = int(tok)
            if not 0 <= t < vocab:
                raise ConfigurationError(f"token id {t} outside the {vocab}-id vocabulary")
            row[t] = float(prob)
        return row
    raise TypeError(f"Unsupported probability distribution type: {type(dist)!r}")


def dist_vocab(dist) -> int:
    """Vocabulary size implied by one ProbDist (ndarray length, or the largest dict id + 1)."""
    if isinstance(dist, np.ndarray):
        return int(dist.size)
    if isinstance(dist, dict):
        return max((int(t) for t in dist), default=-1) + 1
    raise TypeError(f"Unsupported probability distribution type: {type(dist)!r}")


def probs_to_logits(rows: np.ndarray) -> np.ndarray:
    """float64 probability rows -> float32 log-probability rows whose softmax (temperature 1, the rank kernel's
    ``_ModelAdapter`` form) has the same support and the same order: log p, and ``max - ZERO_LOGIT_GAP`` for
    entries that are not positive and finite.  Rows without positive mass stay all-equal (no capacity)."""
    rows = np.asarray(rows, dtype=np.float64)
    pos = np.isfinite(rows) & (rows > 0)
    with np.errstate(divide="ignore", invalid="ignore"):
        lg = np.where(pos, np.log(np.where(pos, rows, 1.0)), -np.inf)
    top = np.max(lg, axis=1, keepdims=True)
    top = np.where(np.isfinite(top), top, 0.0)
    lg = np.where(pos, lg, top - ZERO_LOGIT_GAP)
    return lg.astype(np.float32)


def _declared_vocab(provider) -> int:
    for name in ("vocab_size", "n_vocab", "vocab"):
        v = getattr(provider, name, None)
        if isinstance(v, int) and not isinstance(v, bool) and v > 0:
            return v
    return 0


class ProviderBatchedLM:
    """``prefill(context, B, max_new)`` / ``step(tokens)`` over a ``next_token_probs`` provider: every stream's
    context grows by its emitted token, each step queries the provider once per stream (on the host -- that is
    the provider protocol) with the context trimmed to ``context_window`` (``_next_distribution``,
    ``codec/arithmetic.py:337-347``), and hands the kernel ``[B, ld]`` float32 log-probability rows
    (:func:`probs_to_logits`).  ``first`` is the distribution of ``context`` if the caller already has it (it
    also fixes the vocabulary size)."""

    takes_full_context = True  # HipRankLM: pass the context untrimmed (no 1022-token cut, no [0] for empty)

    def __init__(self, provider, context, *, context_window: Optional[int] = None, first=None, device=None):
        import torch
        from types import SimpleNamespace

        self.provider = provider
        self.window = int(context_window) if context_window else None
        self._first_ctx = tuple(int(t) for t in context)
        self._first = first if first is not None else provider.next_token_probs(self._trim(self._first_ctx))
        # a dict ProbDist names only its support: the id range is the provider's declared vocabulary
        # (MockLM.vocab_size, a model's vocab) when it has one, else what the first distribution implies
        V = max(dist_vocab(self._first), _declared_vocab(provider))
        if V < 2:
            raise ConfigurationError("the provider's distribution needs at least two token ids")
        self.shape = SimpleNamespace(vocab=V, n_positions=0)
        from ..coder import row_stride

        self.ld = row_stride(V, "f32")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ctxs = []

    def _trim(self, ctx):
        return tuple(ctx[-self.window:]) if self.window is not None and len(ctx) > self.window else tuple(ctx)

    def _rows(self):
        import torch

        V = self.shape.vocab
        out = np.full((len(self.ctxs), self.ld), -np.inf, dtype=np.float64)
        for b, ctx in enumerate(self.ctxs):
            if ctx == self._first_ctx and self._first is not None:
                dist = self._first
            else:
                dist = self.provider.next_token_probs(self._trim(ctx))
            try:
                out[b, :V] = dist_to_row(dist, V)
            except ConfigurationError as exc:
                raise ConfigurationError(f"{exc} (the provider declares no vocab_size; the first distribution "
                                         f"implied {V} ids)") from None
        lg = np.zeros((len(self.ctxs), self.ld), dtype=np.float32)
        lg[:, :V] = probs_to_logits(out[:, :V])
        return torch.from_numpy(lg).to(self.device)

    def prefill(self, context, B: int, max_new: int):
        del max_new
        self.ctxs = [tuple(int(t) for t in context)] * int(B)
        return self._rows()

    def step(self, tokens):
        toks = tokens.detach().cpu().tolist() if hasattr(tokens, "detach") else list(tokens)
        self._first = None  # only the prefill's query is shared
        self.ctxs = [ctx + (int(t),) for ctx, t in zip(self.ctxs, toks)]
        return self._rows()


__all__ = ["MockLM", "CachedLM", "HipTransformersLM", "ProviderBatchedLM", "dist_to_row", "probs_to_logits"]
