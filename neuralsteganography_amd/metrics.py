"""Cover-text metrics of the quality guard (``src/neuralstego/metrics/``), SURVEY §8(f) 2.

* Text statistics (``metrics/text_stats.py:10-51``): ``ngram_repeat_ratio``, ``type_token_ratio``,
  ``avg_sentence_len`` -- string heuristics, evaluated on the host exactly as the reference does.
* :class:`LMScorer` (``metrics/lm_scorer.py:37-131``) and :func:`avg_entropy` (``metrics/entropy.py:30-46``):
  with ``prefer_transformers=False`` (the api's default guard, ``api.py:118-127``) the deterministic
  fallback -- an empirical unigram model of the text's own whitespace tokens; otherwise a GPU scorer.
* :class:`HipLMScorer`: the transformers branch for many texts at once -- one causal GPT-2 forward over the
  padded batch (PyTorch-ROCm GEMMs) and the HIP row kernel ``ns_score_rows`` (``include/nsg_score.h``), which
  streams each position's logits once for the label's NLL and the row entropy.  ``ppl = exp(mean NLL)``
  over positions ``t < T-1`` with labels ``ids[t+1]`` (the Hugging Face shifted loss) and ``avg_entropy`` =
  mean row entropy over the same positions.
"""

from __future__ import annotations

import math
import re
from collections import Counter
from typing import Dict, List, Optional, Sequence

_SENTENCE_SPLIT = re.compile(r"[.!؟?\n]+")  # text_stats.py:9 (Persian question mark included)


def _words(text: str) -> List[str]:
    """text_stats.py:13-15: regex whitespace split of the stripped text."""
    return [w for w in re.split(r"\s+", text.strip()) if w]


def _ws_tokens(text: str) -> List[str]:
    """lm_scorer.py:80-82 / entropy.py:12-14: str.split of the stripped text."""
    return [w for w in text.strip().split() if w]


def ngram_repeat_ratio(text: str, n: int = 3) -> float:
    """Share of n-gram occurrences whose n-gram occurs more than once (``text_stats.py:24-36``)."""
    words = _words(text)
    if n <= 0 or len(words) < n:
        return 0.0
    grams = Counter(tuple(words[i:i + n]) for i in range(len(words) - n + 1))
    total = len(words) - n + 1
    return sum(c for c in grams.values() if c > 1) / total if total else 0.0


def type_token_ratio(text: str) -> float:
    """Distinct lower-cased words over words (``text_stats.py:39-46``)."""
    words = _words(text)
    return len({w.lower() for w in words}) / len(words) if words else 0.0


def avg_sentence_len(text: str) -> float:
    """Mean words per sentence, sentences split on ``. ! ? ؟`` and newlines (``text_stats.py:49-58``)."""
    parts = [seg.strip() for seg in _SENTENCE_SPLIT.split(text) if seg.strip()]
    if not parts:
        parts = [text.strip()] if text.strip() else []
    if not parts:
        return 0.0
    counts = [len(_words(p)) for p in parts]
    return sum(counts) / len(counts)


def _fallback_score(tokens: Sequence[str]) -> Dict[str, float]:
    """Unigram self-model of the text (``lm_scorer.py:84-95``): NLL summed in token order."""
    tokens = list(tokens)
    if not tokens:
        return {"ppl": 0.0, "avg_nll": 0.0, "token_count": 0}
    counts, total = Counter(tokens), len(tokens)
    nll = 0.0
    for tok in tokens:
        nll -= math.log(counts[tok] / total)
    avg = nll / total
    return {"ppl": math.exp(avg), "avg_nll": avg, "token_count": total}


def _fallback_entropy(text: str) -> float:
    """Entropy of the text's unigram distribution (``entropy.py:17-27``), summed in first-seen order."""
    tokens = _ws_tokens(text)
    if not tokens:
        return 0.0
    counts, total = Counter(tokens), len(tokens)
    h = 0.0
    for c in counts.values():
        p = c / total
        h -= p * math.log(p)
    return h


class HipLMScorer:
    """GPU perplexity / average-entropy scorer over a batched GPT-2 (``forward_sequences``) and the HIP
    ``ns_score_rows`` kernel.  ``rows_per_batch`` bounds the padded ``B*T`` logits held at once."""

    def __init__(self, batched_lm, tokenizer, *, rows_per_batch: int = 32768):
        import torch

        if not torch.cuda.is_available():
            from ._lib import NativeLibraryError

            raise NativeLibraryError("HipLMScorer needs a ROCm GPU (ns_score_rows has no CPU path)")
        self.lm, self.tokenizer = batched_lm, tokenizer
        self.rows_per_batch = int(rows_per_batch)

    @classmethod
    def from_provider(cls, provider, **kw) -> "HipLMScorer":
        """Score with the provider's own model and tokenizer (a ``HipArithmeticLM`` / ``HipRankLM``)."""
        return cls(provider.lm, provider.tokenizer, **kw)

    def _ids(self, text: str) -> List[int]:
        tok = self.tokenizer
        try:
            ids = tok.encode(text, add_special_tokens=False)
        except TypeError:
            ids = tok.encode(text)
        return [int(i) for i in ids]

    def _row_scores(self, seqs: List[List[int]]):
        """Per sequence: (sum NLL over t < T-1, sum entropy over t < T-1, T)."""
        import numpy as np
        import torch

        from . import _lib
        from .coder import _stream_handle

        L = _lib.lib()
        V = self.lm.shape.vocab
        dt = _lib.NS_DTYPE_F16 if self.lm.logits_dtype == torch.float16 else _lib.NS_DTYPE_F32
        out = [None] * len(seqs)
        order = sorted(range(len(seqs)), key=lambda i: len(seqs[i]))
        i = 0
        while i < len(order):
            T = max(len(seqs[order[i]]), 1)
            j = i
            while j < len(order) and (j - i + 1) * max(len(seqs[order[j]]), 1) <= max(self.rows_per_batch, T):
                j += 1
            group = order[i:j]
            T = max(len(seqs[g]) for g in group)
            ids = np.zeros((len(group), T), dtype=np.int64)
            labels = np.full((len(group), T), -1, dtype=np.int32)
            for r, g in enumerate(group):
                s = seqs[g]
                ids[r, : len(s)] = s
                labels[r, : max(len(s) - 1, 0)] = s[1:]
            dev = self.lm.device
            logits = self.lm.forward_sequences(torch.from_numpy(ids).to(dev))
            lab = torch.from_numpy(labels).to(dev).reshape(-1)
            nll = torch.empty(lab.numel(), dtype=torch.float64, device=dev)
            ent = torch.empty_like(nll)
            rows = logits.reshape(-1, logits.shape[-1])
            rc = L.ns_score_rows(rows.data_ptr(), rows.stride(0), rows.shape[0], V, dt, lab.data_ptr(),
                                 nll.data_ptr(), ent.data_ptr(), _stream_handle())
            if rc != 0:
                raise RuntimeError(f"ns_score_rows failed ({rc})")
            # per text, its own len - 1 positions summed on the host (numpy's order depends on that count only):
            # the metrics of a text do not depend on the padded length of the batch it was scored in
            nh = nll.view(len(group), T).cpu().numpy()
            eh = ent.view(len(group), T).cpu().numpy()
            for r, g in enumerate(group):
                n = max(len(seqs[g]) - 1, 0)
                out[g] = (float(nh[r, :n].sum()), float(eh[r, :n].sum()), len(seqs[g]))
            del logits, rows
            i = j
        return out

    def metrics_batch(self, texts: Sequence[str]) -> List[Dict[str, float]]:
        """``{"ppl", "avg_nll", "token_count", "avg_entropy"}`` per text, one forward per batch."""
        seqs = [self._ids(t) for t in texts]
        todo = [i for i, t in enumerate(texts) if _ws_tokens(t) and seqs[i]]
        n = self.lm.shape.n_positions
        for i in todo:
            if len(seqs[i]) > n:
                raise ValueError(f"text of {len(seqs[i])} tokens exceeds the model's {n} positions")
        res = [{"ppl": 0.0, "avg_nll": 0.0, "token_count": 0, "avg_entropy": 0.0} for _ in texts]
        for i, (sn, se, T) in zip(todo, self._row_scores([seqs[i] for i in todo])):
            npos = T - 1
            avg = sn / npos if npos > 0 else float("nan")  # a 1-token text: the reference's mean of nothing
            res[i] = {"ppl": math.exp(avg) if npos > 0 else float("nan"), "avg_nll": avg, "token_count": T,
                      "avg_entropy": se / npos if npos > 0 else float("nan")}
        return res

    def score(self, text: str) -> Dict[str, float]:
        m = self.metrics_batch([text])[0]
        return {k: m[k] for k in ("ppl", "avg_nll", "token_count")}

    def avg_entropy(self, text: str) -> float:
        return self.metrics_batch([text])[0]["avg_entropy"]


class LMScorer:
    """``metrics/lm_scorer.py:37-131``.  ``prefer_transformers=False``: the fallback unigram scorer (the
    api's default guard).  ``True``: ``model_name`` is loaded offline-first (``lm.load_lm``) and scored on the
    GPU by :class:`HipLMScorer`; a ``scorer`` may be passed directly (e.g. ``HipLMScorer.from_provider``)."""

    def __init__(self, model_name: str = "HooshvareLab/gpt2-fa", prefer_transformers: bool = True,
                 scorer: Optional[HipLMScorer] = None):
        self.model_name = model_name
        self.prefer_transformers = prefer_transformers or scorer is not None
        self._scorer = scorer

    def _gpu(self) -> HipLMScorer:
        if self._scorer is None:
            from .lm import load_lm

            name = {"HooshvareLab/gpt2-fa": "gpt2-fa"}.get(self.model_name, self.model_name)
            self._scorer = HipLMScorer.from_provider(load_lm(name))
        return self._scorer

    def score(self, text: str) -> Dict[str, float]:
        tokens = _ws_tokens(text)
        if not tokens:
            return {"ppl": 0.0, "avg_nll": 0.0, "token_count": 0}
        if not self.prefer_transformers:
            return _fallback_score(tokens)
        return self._gpu().score(text)

    def metrics_batch(self, texts: Sequence[str]) -> List[Dict[str, float]]:
        """score() and avg_entropy() of every text (one GPU forward per batch on the transformers branch)."""
        if not self.prefer_transformers:
            out = []
            for t in texts:
                m = self.score(t)
                m["avg_entropy"] = avg_entropy(t, self)
                out.append(m)
            return out
        return self._gpu().metrics_batch(texts)


def avg_entropy(text: str, lm_scorer: Optional[LMScorer] = None) -> float:
    """``metrics/entropy.py:30-46``."""
    if not _ws_tokens(text):
        return 0.0
    scorer = lm_scorer or LMScorer()
    if not scorer.prefer_transformers:
        return _fallback_entropy(text)
    return scorer._gpu().avg_entropy(text)


__all__ = ["LMScorer", "HipLMScorer", "avg_entropy", "avg_sentence_len", "ngram_repeat_ratio", "type_token_ratio"]
