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


def dist_arrays(dist):
    """``_dist_to_arrays`` (codec/arithmetic.py:388-398, codec/quality.py:144-158): (float64 values, int32 token
    ids or None when the array position is the id, dict flag) -- an ndarray ProbDist by id, a dict's items sorted
    by id."""
    if isinstance(dist, np.ndarray):
        return np.ascontiguousarray(np.asarray(dist, dtype=np.float64).reshape(-1)), None, False
    if isinstance(dist, dict):
        items = sorted(dist.items())
        ids = np.array([int(t) for t, _ in items], dtype=np.int64)
        if ids.size and (ids.min() < -(1 << 31) or ids.max() >= (1 << 31)):
            raise ConfigurationError("token ids must fit int32")
        return (np.array([float(p) for _, p in items], dtype=np.float64), ids.astype(np.int32), True)
    raise TypeError(f"Unsupported probability distribution type: {type(dist)!r}")


# the rank kernel keys positions below 2^17 (ns_create: vocab < 131072 on the wide path); ids are any int32
MAX_ROW_ENTRIES = 0x1FFFF


class ProbRows:
    """A step's provider ProbDists staged for the rank kernel at float64 (``NS_DTYPE_F64``, ``ns_set_rank_rows``):
    ``values`` [B, ld] float64 (the provider's own values in ``_dist_to_arrays`` order), ``count`` [B] int32
    entries per row, ``idmap`` [B, ld] int32 token id per entry (None when every row is an ndarray: position = id),
    ``dict_rows``; ``flags`` per row (host): negative / NaN / +inf entries, for the reference's quality errors."""

    prob_rows = True

    def __init__(self, dists, device, min_cols: int = 2):
        import torch

        arrs = [dist_arrays(d) for d in dists]
        kinds = {a[2] for a in arrs}
        self.dict_rows = True in kinds
        self.mixed = len(kinds) > 1
        n = max([a[0].size for a in arrs] + [int(min_cols)])
        if n > MAX_ROW_ENTRIES:
            raise ConfigurationError(f"a ProbDist of {n} entries exceeds the rank kernel's {MAX_ROW_ENTRIES}")
        from ..coder import row_stride

        self.ncols = n
        ld = row_stride(n, "f64")
        B = len(arrs)
        vals = np.zeros((B, ld), dtype=np.float64)
        cnt = np.zeros(B, dtype=np.int32)
        ids = np.zeros((B, ld), dtype=np.int32) if self.dict_rows else None
        self.neg = np.zeros(B, bool)
        self.nan = np.zeros(B, bool)
        self.posinf = np.zeros(B, bool)
        for b, (v, idv, _) in enumerate(arrs):
            m = v.size
            vals[b, :m] = v
            cnt[b] = m
            if ids is not None:
                ids[b, :m] = idv if idv is not None else np.arange(m, dtype=np.int32)
            self.neg[b] = bool(np.any(v < 0))
            self.nan[b] = bool(np.any(np.isnan(v)))
            self.posinf[b] = bool(np.any(np.isposinf(v)))
        self.values = torch.from_numpy(vals).to(device)
        self.count = torch.from_numpy(cnt).to(device)
        self.idmap = torch.from_numpy(ids).to(device) if ids is not None else None

    def check_quality(self, q) -> None:
        """The errors the reference's quality code raises on such rows (host check before the launch):
        codec/quality.py:155-156 negative probabilities; a NaN kept by the filters or +inf make the
        normalisation total non-finite (:174-178); the crypto policy normalises every row first
        (crypto/quality.py:118-122)."""
        from .errors import QualityConfigError

        top_k, top_p, min_prob = q.top_k > 0, q.top_p > 0.0, q.min_prob >= 0.0
        cap, crypto = q.cap_bits > 0, q.prob_temp > 0.0
        if crypto:
            if np.any(self.neg | self.nan | self.posinf):
                raise QualityConfigError("Probability mass vanished during normalisation")
            return
        if not (top_k or top_p or min_prob or cap):
            return
        if np.any(self.neg):
            raise QualityConfigError("Probabilities must be non-negative")
        if np.any(self.posinf) or (np.any(self.nan) and not min_prob):
            raise QualityConfigError("Probability mass vanished after filtering")
        if cap and self.mixed:
            raise ConfigurationError("cap_per_token_bits over a mix of dict and ndarray ProbDists in one step")


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
    ``codec/arithmetic.py:337-347``), and hands the rank kernel the ProbDists themselves at float64
    (:class:`ProbRows`: ranked, filtered and renormalised on the device exactly as the reference's numpy does; the
    round-3 float32 log-probability staging merged near-tied probabilities).  Any ids per step: a dict's ids map
    through the row's id table and a longer row grows the coder context.  ``first`` is the distribution of
    ``context`` if the caller already has it."""

    takes_full_context = True  # HipRankLM: pass the context untrimmed (no 1022-token cut, no [0] for empty)
    prob_rows = True  # HipRankLM: the steps return ProbRows for a NS_DTYPE_F64 coder context

    def __init__(self, provider, context, *, context_window: Optional[int] = None, first=None, device=None):
        import torch
        from types import SimpleNamespace

        self.provider = provider
        self.window = int(context_window) if context_window else None
        self._first_ctx = tuple(int(t) for t in context)
        self._first = first if first is not None else provider.next_token_probs(self._trim(self._first_ctx))
        V = max(dist_arrays(self._first)[0].size, _declared_vocab(provider), 2)
        self.shape = SimpleNamespace(vocab=min(V, MAX_ROW_ENTRIES), n_positions=0)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ctxs = []

    def _trim(self, ctx):
        return tuple(ctx[-self.window:]) if self.window is not None and len(ctx) > self.window else tuple(ctx)

    def _rows(self) -> ProbRows:
        dists = []
        for ctx in self.ctxs:
            if ctx == self._first_ctx and self._first is not None:
                dists.append(self._first)
            else:
                dists.append(self.provider.next_token_probs(self._trim(ctx)))
        rows = ProbRows(dists, self.device, min_cols=self.shape.vocab)
        self.shape.vocab = max(self.shape.vocab, rows.ncols)  # rows never narrower than the coder context
        return rows

    def prefill(self, context, B: int, max_new: int):
        del max_new
        self.ctxs = [tuple(int(t) for t in context)] * int(B)
        return self._rows()

    def step(self, tokens):
        toks = tokens.detach().cpu().tolist() if hasattr(tokens, "detach") else list(tokens)
        self._first = None  # only the prefill's query is shared
        self.ctxs = [ctx + (int(t),) for ctx, t in zip(self.ctxs, toks)]
        return self._rows()


__all__ = ["MockLM", "CachedLM", "HipTransformersLM", "ProviderBatchedLM", "ProbRows", "dist_arrays"]
